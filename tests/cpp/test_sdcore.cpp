// Tests of the C++ host mirror (include/sdcore.hpp) against the CPU oracle.
// TEST INFRASTRUCTURE: links oracle/build/liboracle.so as the checker.
//
//   test_sdcore            full run on a GPU (cas_ids, checksums, errors,
//                          identifier job at batch 100 and 1000, validator)
//   test_sdcore --no-gpu   checks that Engine::open fails loudly (LibraryError)
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <map>
#include <set>
#include <vector>

#include "../../oracle/oracle.h"
#include "sdcore.hpp"

using namespace sdcore;

static int failures = 0;
#define CHECK(cond, ...)                                       \
  do {                                                         \
    if (!(cond)) {                                             \
      ++failures;                                              \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                       \
      std::fprintf(stderr, "\n");                              \
    }                                                          \
  } while (0)

static void write_file(const std::string& path, const std::vector<uint8_t>& data) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(2);
  }
  if (!data.empty()) std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
}

static std::vector<uint8_t> content(uint64_t seed, size_t n) {
  std::mt19937_64 g(seed);
  std::vector<uint8_t> v(n);
  for (size_t i = 0; i < n; i += 8) {
    const uint64_t x = g();
    std::memcpy(&v[i], &x, std::min<size_t>(8, n - i));
  }
  return v;
}

static std::string oracle_cas(const std::string& p, uint64_t size, int* st) {
  char h[17];
  *st = oracle_generate_cas_id(p.c_str(), size, h);
  return *st ? std::string() : std::string(h, 16);
}

static std::string oracle_sum(const std::string& p) {
  char h[65];
  return oracle_file_checksum(p.c_str(), h) ? std::string() : std::string(h, 64);
}

static void test_hashes(Engine& eng, const std::string& dir) {
  const std::vector<size_t> sizes = {0, 1, 1023, 1024, 1025, 65536, 102400, 102401, 300000, (3u << 20) + 17};
  std::vector<std::pair<std::string, uint64_t>> files;
  std::vector<std::string> paths;
  for (size_t i = 0; i < sizes.size(); ++i) {
    const std::string p = dir + "/h" + std::to_string(i) + ".bin";
    write_file(p, content(100 + i, sizes[i]));
    files.emplace_back(p, sizes[i]);
    paths.push_back(p);
  }
  auto cas = eng.generate_cas_ids(files);
  auto sums = eng.file_checksums(paths);
  for (size_t i = 0; i < sizes.size(); ++i) {
    int st;
    const std::string want = oracle_cas(paths[i], sizes[i], &st);
    CHECK(cas[i].ok() && cas[i].value() == want, "cas_id size %zu", sizes[i]);
    CHECK(sums[i].ok() && sums[i].value() == oracle_sum(paths[i]), "checksum size %zu", sizes[i]);
  }
  // single-file forms (cas.rs:23, hash.rs:11)
  auto one = generate_cas_id(eng, paths[3], sizes[3]);
  CHECK(one.ok() && one.value() == cas[3].value(), "generate_cas_id single");
  auto s1 = file_checksum(eng, paths[9]);
  CHECK(s1.ok() && s1.value() == sums[9].value(), "file_checksum single");
  // errors: a missing file is ENOENT; a file shorter than the sampled
  // windows of its recorded size is UnexpectedEof (cas.rs:36,43,56)
  auto miss = generate_cas_id(eng, dir + "/missing.bin", 5000);
  CHECK(!miss.ok() && miss.error().code == ENOENT, "missing file -> ENOENT (%d)", miss.ok() ? 0 : miss.error().code);
  const std::string shrunk = dir + "/shrunk.bin";
  write_file(shrunk, content(7, 20000));
  auto eof = generate_cas_id(eng, shrunk, 500000);
  int st;
  oracle_cas(shrunk, 500000, &st);
  CHECK(!eof.ok() && eof.error().unexpected_eof() && st == ORACLE_STATUS_UNEXPECTED_EOF, "shrunk -> UnexpectedEof");
  auto sm = file_checksum(eng, dir + "/missing.bin");
  CHECK(!sm.ok() && sm.error().code == ENOENT, "checksum missing -> ENOENT");
  // file_metadata_batch: empty files have no cas_id (mod.rs:78-86)
  auto md = file_metadata_batch(eng, {{paths[0], 3}, {paths[4], 1}, {dir + "/missing.bin", 0}});
  CHECK(md[0].ok() && !md[0].value().cas_id && md[0].value().kind == 3, "empty file metadata");
  CHECK(md[1].ok() && md[1].value().cas_id == cas[4].value() && md[1].value().len == 1025, "metadata cas_id");
  CHECK(!md[2].ok() && md[2].error().code == ENOENT, "metadata of a missing file");
  // the kind from the path (mod.rs:72-76, Extension::resolve_conflicting)
  write_file(dir + "/clip.ts", {0x47, 0x40, 0x11, 0x10});
  write_file(dir + "/app.ts", {'l', 'e', 't'});
  auto mk = file_metadata_batch(eng, {{dir + "/clip.ts", kKindFromPath}, {dir + "/app.ts", kKindFromPath},
                                      {paths[4], kKindFromPath}});
  CHECK(mk[0].ok() && mk[0].value().kind == ObjectKindVideo && mk[1].ok() && mk[1].value().kind == ObjectKindCode &&
            mk[2].ok() && mk[2].value().kind == object_kind_of(paths[4]),
        "metadata kinds from paths");
  std::printf("hashes: %zu files ok\n", sizes.size());
}

// a location of `n` files: contents drawn from `distinct` seeds (duplicates in
// and across 100-row chunks), some empty, one row whose file is missing
struct Corpus {
  MemoryLibrary lib;
  Location loc;
  std::vector<uint64_t> keys;
  std::vector<uint8_t> has_key;
  std::vector<int32_t> status;
  std::vector<uint64_t> existing;  // pre-existing Object keys, DB order
};

static Corpus make_corpus(const std::string& dir, size_t n, size_t distinct) {
  Corpus c;
  c.loc = {1, dir};
  std::mt19937_64 g(42);
  mkdir((dir + "/sub").c_str(), 0755);
  // two pre-existing Objects, each with an identified file_path
  for (int e = 0; e < 2; ++e) {
    const std::string name = "old" + std::to_string(e);
    const auto data = content(1000 + e, 5000);  // the same contents as seeds 0 and 1 below
    write_file(dir + "/" + name + ".dat", data);
    int st;
    const std::string cas = oracle_cas(dir + "/" + name + ".dat", data.size(), &st);
    const int32_t oid = c.lib.create_object(0, 0);
    FilePathRow r;
    r.location_id = 1;
    r.name = name;
    r.extension = "dat";
    r.size_in_bytes = data.size();
    r.cas_id = cas;
    r.object_id = oid;
    c.lib.add_file_path(r);
    c.existing.push_back(hex_to_key(cas));
  }
  for (size_t i = 0; i < n; ++i) {
    FilePathRow r;
    r.location_id = 1;
    r.materialized_path = (i % 3 == 0) ? "/sub/" : "/";
    r.name = "f" + std::to_string(i);
    r.extension = (i % 5 == 0) ? "" : "bin";
    r.date_created = (int64_t)i;
    r.kind = (int32_t)(i % 7);
    const std::string p = full_path(c.loc, r);
    size_t which = g() % distinct;
    // empty files (cas_id None) here and there, and at some step ends, where
    // the next step reads them again (the cursor is the step's last row)
    if (i % 300 == 199) which = 5;
    size_t size = which % 13 == 5 ? 0 : 100 + (which * 7919) % 150000;
    std::vector<uint8_t> data = which < 2 ? content(1000 + which, 5000) : content(which, size);
    const bool missing = (i == n / 2 - 1);  // an I/O error at a step end
    if (!missing) write_file(p, data);
    r.size_in_bytes = data.empty() ? 1 : data.size();  // DB size: non-zero (orphan filter)
    c.lib.add_file_path(r);
    int st = 0;
    const std::string cas = missing || data.empty() ? std::string() : oracle_cas(p, data.size(), &st);
    c.keys.push_back(cas.empty() ? 0 : hex_to_key(cas));
    c.has_key.push_back(!cas.empty());
    c.status.push_back(missing ? ENOENT : st);
  }
  return c;
}

static void test_identifier_job(Engine& eng, const std::string& dir) {
  const size_t n = 1000;
  std::vector<std::vector<int32_t>> objects_by_batch;
  for (size_t batch : {100, 1000, 400}) {
    const std::string d = dir + "/loc" + std::to_string(batch);
    mkdir(d.c_str(), 0755);
    Corpus c = make_corpus(d, n, 300);
    // the same library in SQLite (objects first, so their ids match), run
    // through the same job below
    auto sql = SqliteLibrary::open(":memory:");
    for (const auto& o : c.lib.objects) sql->create_object(o.kind, o.date_created);
    std::vector<FilePathRow> rows = c.lib.file_paths;
    sql->add_file_paths(rows);
    // the oracle: reference chunks of 100 over the orphans in id order
    std::vector<int64_t> link(n);
    int64_t linked = 0;
    const int64_t created = oracle_identifier_dedup(n, c.keys.data(), c.has_key.data(), c.status.data(), 100,
                                                    c.existing.size(), c.existing.data(), link.data(), &linked);
    FileIdentifierJobInit init{c.loc, "", batch};
    auto meta = run_file_identifier_job(eng, c.lib, init);
    CHECK(meta.total_orphan_paths == n, "orphans %zu", meta.total_orphan_paths);
    CHECK((int64_t)meta.total_objects_created == created && (int64_t)meta.total_objects_linked == linked,
          "batch %zu: created/linked %zu/%zu, oracle %lld/%lld", batch, meta.total_objects_created,
          meta.total_objects_linked, (long long)created, (long long)linked);
    CHECK(meta.steps == (n + 99) / 100, "steps %zu", meta.steps);
    CHECK(meta.rereads > 0, "no step re-read its predecessor's last row");
    // every file's Object follows the oracle's link
    std::vector<int32_t> obj(n, 0);
    for (size_t i = 0; i < n; ++i) obj[i] = c.lib.file_path((int32_t)(i + 3))->object_id.value_or(-1);
    for (size_t i = 0; i < n; ++i) {
      const int64_t l = link[i];
      if (l == SDCAS_LINK_DEFERRED) CHECK(obj[i] == -1, "deferred file %zu has an Object", i);
      else if (l == INT64_MIN) CHECK(obj[i] == -1, "dropped file %zu has an Object", i);
      else if (l < 0) CHECK(obj[i] == (int32_t)(-(l + 1)) + 1, "file %zu -> existing %lld got %d", i, (long long)l, obj[i]);
      else if (l < (int64_t)i) CHECK(obj[i] == obj[(size_t)l], "file %zu shares file %lld's Object", i, (long long)l);
      else CHECK(obj[i] > 2, "file %zu owns a new Object", i);
    }
    // new Objects carry their file's kind and date_created (mod.rs:266-291)
    for (size_t i = 0; i < n; ++i)
      if (link[i] == (int64_t)i) {
        const auto& o = c.lib.objects[(size_t)obj[i] - 1];
        CHECK(o.kind == (int32_t)(i % 7) && o.date_created == (int64_t)i, "object of file %zu", i);
      }
    // cas_id written per processed file (mod.rs:157-178)
    for (size_t i = 0; i < n; ++i) {
      const auto* r = c.lib.file_path((int32_t)(i + 3));
      if (c.status[i] || link[i] == SDCAS_LINK_DEFERRED) CHECK(!r->cas_id, "failed / unread file %zu has a cas_id", i);
      else if (c.has_key[i]) CHECK(r->cas_id && hex_to_key(*r->cas_id) == c.keys[i], "cas_id of file %zu", i);
    }
    // a second run finds the failed row, the empty files (which keep cas_id
    // NULL and are orphans again, as in the reference) and the rows the
    // job's task_count did not reach (a re-read costs a row of the budget)
    size_t left = 0;
    for (size_t i = 0; i < n; ++i)
      left += c.status[i] || !c.has_key[i] || link[i] == SDCAS_LINK_DEFERRED;
    CHECK(c.lib.count_orphan_file_paths(1, "") == left, "orphans left %zu, want %zu",
          c.lib.count_orphan_file_paths(1, ""), left);
    // sub-path filter (materialized_path LIKE '/sub/%')
    size_t sub = 0;
    for (const auto& r : c.lib.file_paths) sub += r.materialized_path == "/sub/" && (!r.object_id || !r.cas_id);
    CHECK(c.lib.count_orphan_file_paths(1, "/sub/") == sub, "sub orphans");
    objects_by_batch.push_back(obj);
    auto msql = run_file_identifier_job(eng, *sql, init);
    CHECK(msql.total_objects_created == meta.total_objects_created &&
              msql.total_objects_linked == meta.total_objects_linked && msql.steps == meta.steps,
          "sqlite job batch %zu", batch);
    for (size_t i = 0; i < n; ++i) {
      auto r = sql->file_path((int32_t)(i + 3));
      CHECK(r && r->object_id.value_or(-1) == obj[i] && r->cas_id == c.lib.file_path((int32_t)(i + 3))->cas_id,
            "sqlite file %zu", i);
    }
    std::printf("identifier job batch %zu: created %zu linked %zu steps %zu\n", batch, meta.total_objects_created,
                meta.total_objects_linked, meta.steps);
  }
  CHECK(objects_by_batch[0] == objects_by_batch[1] && objects_by_batch[0] == objects_by_batch[2],
        "batch 100, 1000 and 400 give the same Objects");
}

static void test_validator(Engine& eng, const std::string& dir) {
  const std::string d = dir + "/val";
  mkdir(d.c_str(), 0755);
  MemoryLibrary lib;
  Location loc{2, d};
  std::vector<std::string> paths;
  for (int i = 0; i < 250; ++i) {
    FilePathRow r;
    r.location_id = 2;
    r.name = "v" + std::to_string(i);
    r.extension = "bin";
    r.size_in_bytes = 1;
    if (i == 7) r.integrity_checksum = std::string(64, '0');  // already validated: not selected
    const auto& row = lib.add_file_path(r);
    write_file(full_path(loc, row), content(5000 + i, i == 11 ? (2u << 20) + 5 : 37 * i));
    paths.push_back(full_path(loc, row));
  }
  ObjectValidatorJobInit init{loc, "", 64};
  auto rep = run_object_validator_job(eng, lib, init);
  CHECK(rep.task_count == 249 && rep.checksummed == 249 && !rep.error, "validator %zu/%zu", rep.checksummed,
        rep.task_count);
  for (int i = 0; i < 250; ++i) {
    const auto* r = lib.file_path(i + 1);
    if (i == 7) CHECK(*r->integrity_checksum == std::string(64, '0'), "pre-validated row changed");
    else CHECK(r->integrity_checksum && *r->integrity_checksum == oracle_sum(paths[i]), "checksum %d", i);
  }
  // a missing file stops the job at that row (validator_job.rs:154-156)
  MemoryLibrary lib2;
  for (int i = 0; i < 5; ++i) {
    FilePathRow r;
    r.location_id = 2;
    r.name = i == 3 ? "gone" : "v" + std::to_string(i);
    r.extension = "bin";
    lib2.add_file_path(r);
  }
  auto rep2 = run_object_validator_job(eng, lib2, init);
  CHECK(rep2.error && rep2.error->code == ENOENT && rep2.checksummed == 3, "validator error stop");
  std::printf("validator: %zu checksums ok\n", rep.checksummed);
}

// a location on disk end to end: walk -> SQLite -> identifier job -> validator
static void test_location_scan(Engine& eng, const std::string& dir) {
  const std::string root = dir + "/scan";
  mkdir(root.c_str(), 0755);
  std::mt19937_64 g(3);
  std::vector<std::string> subdirs = {"", "docs", "docs/old", "media", "media/raw", ".cache"};
  for (const auto& d : subdirs)
    if (!d.empty()) mkdir((root + "/" + d).c_str(), 0755);
  for (int i = 0; i < 640; ++i) {
    const auto& d = subdirs[g() % subdirs.size()];
    const uint64_t which = g() % 220;  // shared contents
    const size_t size = 1 + (which * 104729) % 300000;
    static const char* const exts[] = {"", ".dat", ".JPG", ".ts", ".md", ".mts", ".json"};
    const std::string name = "f" + std::to_string(i) + exts[i % 7];
    write_file(root + (d.empty() ? "" : "/" + d) + "/" + name, content(which + 9000, size));
  }
  std::vector<IoError> errs;
  auto rows = walk_location(Location{3, root}, &errs);
  CHECK(errs.empty(), "walk errors");
  auto sql = SqliteLibrary::open(":memory:");
  sql->add_file_paths(rows);
  FileIdentifierJobInit init{Location{3, root}, "", 1000};
  auto meta = run_file_identifier_job(eng, *sql, init);
  // the oracle over the same orphans (files in id order)
  std::vector<uint64_t> keys;
  std::vector<uint8_t> has;
  std::vector<int32_t> ids;
  for (const auto& r : rows) {
    if (r.is_dir) continue;
    int st;
    const std::string cas = oracle_cas(full_path(Location{3, root}, r), r.size_in_bytes, &st);
    keys.push_back(hex_to_key(cas));
    has.push_back(1);
    ids.push_back(r.id);
  }
  std::vector<int64_t> link(keys.size());
  int64_t linked = 0;
  const int64_t created =
      oracle_identifier_dedup(keys.size(), keys.data(), has.data(), nullptr, 100, 0, nullptr, link.data(), &linked);
  CHECK((int64_t)meta.total_objects_created == created && (int64_t)meta.total_objects_linked == linked,
        "scan: created/linked %zu/%zu, oracle %lld/%lld", meta.total_objects_created, meta.total_objects_linked,
        (long long)created, (long long)linked);
  for (size_t k = 0; k < ids.size(); ++k) {
    auto r = sql->file_path(ids[k]);
    CHECK(r && r->cas_id && hex_to_key(*r->cas_id) == keys[k], "scan cas_id of row %d", ids[k]);
    if (link[k] >= 0 && link[k] != (int64_t)k)
      CHECK(r->object_id == sql->file_path(ids[(size_t)link[k]])->object_id, "scan object of row %d", ids[k]);
  }
  // a created Object takes its file's kind (mod.rs:266-291), derived from the
  // path by FileMetadata::new (mod.rs:72-76)
  std::map<int32_t, ObjectKind> object_kind;
  for (const auto& o : sql->objects()) object_kind[o.id] = o.kind;
  std::set<ObjectKind> kinds_seen;
  for (size_t k = 0; k < ids.size(); ++k) {
    if (link[k] != (int64_t)k) continue;
    auto r = sql->file_path(ids[k]);
    const ObjectKind want = object_kind_of(full_path(Location{3, root}, *r));
    kinds_seen.insert(want);
    CHECK(r->object_id && object_kind[*r->object_id] == want, "scan kind of row %d", ids[k]);
  }
  CHECK(kinds_seen.size() >= 5, "scan saw %zu kinds", kinds_seen.size());
  auto rep = run_object_validator_job(eng, *sql, ObjectValidatorJobInit{Location{3, root}, "", 256});
  CHECK(rep.task_count == ids.size() && rep.checksummed == ids.size() && !rep.error, "scan validator");
  for (int32_t id : ids) {
    auto r = sql->file_path(id);
    CHECK(r->integrity_checksum == oracle_sum(full_path(Location{3, root}, *r)), "scan checksum of row %d", id);
  }
  std::printf("location scan: %zu entries, %zu files, created %zu linked %zu, checksums ok\n", rows.size(),
              ids.size(), meta.total_objects_created, meta.total_objects_linked);
}

// light_scan_location's shallow identifier (shallow.rs:24-142) on the GPU:
// only the orphans of one directory level, against the oracle's job over them
static void test_shallow_scan(Engine& eng, const std::string& dir) {
  const std::string root = dir + "/shallow";
  mkdir(root.c_str(), 0755);
  mkdir((root + "/docs").c_str(), 0755);
  mkdir((root + "/docs/old").c_str(), 0755);
  std::mt19937_64 g(5);
  for (int i = 0; i < 900; ++i) {
    const char* d = i % 3 == 0 ? "" : (i % 3 == 1 ? "/docs" : "/docs/old");
    const uint64_t which = g() % 150;
    const size_t size = which % 17 == 3 ? 0 : 1 + (which * 104729) % 200000;  // some empty files
    write_file(root + d + "/g" + std::to_string(i) + ".dat", content(which + 7000, size));
  }
  auto rows = walk_location(Location{4, root});
  for (auto& r : rows)
    if (!r.is_dir && r.size_in_bytes == 0) r.size_in_bytes = 1;  // indexed before the file was emptied
  auto sql = SqliteLibrary::open(":memory:");
  sql->add_file_paths(rows);
  auto rep = shallow_file_identifier(eng, *sql, Location{4, root}, "/docs/", 1000);
  std::vector<uint64_t> keys;
  std::vector<uint8_t> has;
  std::vector<int32_t> ids;
  for (const auto& r : rows) {
    if (r.is_dir || r.materialized_path != "/docs/") continue;
    const std::string p = full_path(Location{4, root}, r);
    struct stat sb;
    stat(p.c_str(), &sb);
    int st = 0;
    const std::string cas = sb.st_size ? oracle_cas(p, (uint64_t)sb.st_size, &st) : std::string();
    keys.push_back(cas.empty() ? 0 : hex_to_key(cas));
    has.push_back(!cas.empty());
    ids.push_back(r.id);
  }
  std::vector<int64_t> link(keys.size());
  int64_t linked = 0;
  const int64_t created =
      oracle_identifier_dedup(keys.size(), keys.data(), has.data(), nullptr, 100, 0, nullptr, link.data(), &linked);
  CHECK(rep.orphans == ids.size() && (int64_t)rep.created == created && (int64_t)rep.linked == linked,
        "shallow: %zu orphans created/linked %zu/%zu, oracle %zu %lld/%lld", rep.orphans, rep.created, rep.linked,
        ids.size(), (long long)created, (long long)linked);
  for (size_t k = 0; k < ids.size(); ++k) {
    auto r = sql->file_path(ids[k]);
    if (link[k] == SDCAS_LINK_DEFERRED) continue;
    CHECK(r && r->object_id, "shallow row %d has no Object", ids[k]);
    if (has[k]) CHECK(r->cas_id && hex_to_key(*r->cas_id) == keys[k], "shallow cas_id of row %d", ids[k]);
    if (link[k] >= 0 && link[k] != (int64_t)k)
      CHECK(r->object_id == sql->file_path(ids[(size_t)link[k]])->object_id, "shallow object of row %d", ids[k]);
  }
  for (const auto& r : rows)
    if (r.materialized_path != "/docs/") {
      auto s = sql->file_path(r.id);
      CHECK(s && !s->cas_id && !s->object_id, "shallow touched row %d outside its level", r.id);
    }
  std::printf("shallow identifier /docs/: %zu orphans, created %zu linked %zu in %zu steps (%zu re-reads)\n",
              rep.orphans, rep.created, rep.linked, rep.steps, rep.rereads);
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--no-gpu") == 0) {
    try {
      auto e = Engine::open();
      std::fprintf(stderr, "Engine::open succeeded without a GPU\n");
      return 1;
    } catch (const LibraryError& e) {
      std::printf("Engine::open -> LibraryError %d (%s)\n", e.code, e.what());
      return e.code == SDCAS_E_NO_DEVICE ? 0 : 1;
    }
  }
  char tmpl[] = "/tmp/sdcore_testXXXXXX";
  const std::string dir = mkdtemp(tmpl);
  auto eng = Engine::open();
  test_hashes(*eng, dir);
  test_identifier_job(*eng, dir);
  test_validator(*eng, dir);
  test_location_scan(*eng, dir);
  test_shallow_scan(*eng, dir);
  std::string cmd = "rm -rf " + dir;
  if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "cleanup failed\n");
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "ALL OK", failures);
  return failures ? 1 : 0;
}
