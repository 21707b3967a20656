// CPU tests of the DB side of the identifier join:
// SqliteLibrary against MemoryLibrary (the reference's query semantics in
// memory) and the oracle's chunked group-by, without a GPU.
// TEST INFRASTRUCTURE: links oracle/build/liboracle.so as the checker.
//
//   test_sdcore_db            query parity + a simulated identifier job on both
//   test_sdcore_db --bench N  DB-side rows/s of the identifier step over N
//                             file_paths in a SQLite file (one JSON line)
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <tuple>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../oracle/oracle.h"
#include "../../spacedrive_amd/host/sqlite3_min.h"
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

static uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// rows of two locations: files and dirs, empty DB sizes, a sub directory,
// already identified rows (cas_id + object) and validated ones
static std::vector<FilePathRow> make_rows(size_t n, uint64_t seed) {
  std::mt19937_64 g(seed);
  std::vector<FilePathRow> rows;
  for (size_t i = 0; i < n; ++i) {
    FilePathRow r;
    r.location_id = (g() % 10) ? 1 : 2;
    r.materialized_path = (g() % 3) ? "/" : ((g() % 2) ? "/sub/" : "/sub/deeper/");
    r.name = "f" + std::to_string(i);
    r.extension = (g() % 4) ? "bin" : "";
    r.is_dir = (g() % 25) == 0;
    r.size_in_bytes = (g() % 40) ? 1 + g() % 200000 : 0;
    r.date_created = (int64_t)(1700000000 + i);
    r.kind = (int32_t)(g() % 9);
    r.inode = g();
    r.hidden = g() % 7 == 0;
    if (g() % 11 == 0) r.integrity_checksum = std::string(64, 'a');
    rows.push_back(r);
  }
  return rows;
}

// FileMetadata per row: cas ids from a pool (duplicates in and across
// chunks), some empty files (None), some I/O errors
static uint64_t g_err_mod = 97, g_none_mod = 31;  // 1 in N rows fails / has no cas_id
static std::vector<Result<FileMetadata>> make_metadata(const std::vector<FilePathRow>& rows, size_t pool) {
  std::vector<Result<FileMetadata>> md;
  for (const auto& r : rows) {
    const uint64_t h = mix((uint64_t)r.id * 7919);
    if (h % g_err_mod == 0) {
      md.emplace_back(IoError{ENOENT, r.name});
      continue;
    }
    FileMetadata m;
    m.kind = r.kind;
    m.len = r.size_in_bytes;
    if ((h / g_err_mod) % g_none_mod != 0) m.cas_id = key_to_hex(mix(h % pool));
    md.emplace_back(m);
  }
  return md;
}

static GroupBy oracle_group_by(size_t chunk_size) {
  return [chunk_size](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
                      const std::vector<uint64_t>& e, sdcas_job_window& w) {
    Engine::Dedup d;
    d.link.assign(k.size(), 0);
    int64_t linked = 0;
    oracle_job_window ow{w.max_steps, (int32_t)w.more, 0, 0, 0, 0};
    d.created = oracle_identifier_job(k.size(), k.data(), h.data(), st.data(), chunk_size, e.size(),
                                      e.empty() ? nullptr : e.data(), &ow, d.link.data(), &linked);
    d.linked = linked;
    w.steps = ow.steps;
    w.rows = ow.rows;
    w.rereads = ow.rereads;
    return d;
  };
}

// the identifier job's loop (run_file_identifier_job_with: the reference's
// file_identifier_job.rs:125-236 in batches) with the metadata supplied
// instead of read from files, and the oracle as the group-by
static FileIdentifierJobRunMetadata run_job(Library& db, int32_t loc, size_t batch, uint64_t pool, bool bulk = false) {
  FileIdentifierJobInit init{Location{loc, "/nowhere"}, "", batch};
  init.bulk_identify = bulk;
  return run_file_identifier_job_with(
      db, init, [&](const std::vector<FilePathRow>& rows) { return make_metadata(rows, pool); }, oracle_group_by(100));
}

// The reference's job restated literally on a Library, as an independent
// ground truth for run_file_identifier_job_with (which plans steps, defers
// cas_id writes into the link, probes first_objects and batches): init
// (file_identifier_job.rs:125-176), then per step the next 100 orphans with
// id >= cursor (:296-319) through identifier_job_step exactly as mod.rs:98-350
// orders its calls — every processed row's cas_id written (:157-178), the
// existing-Object query (:181-188), each row with a cas_id linked to the
// first such Object (:202-238), a new Object for each row whose cas_id no
// existing Object carries or that has none (:246-342) — and the cursor moved
// to the step's last row (mod.rs:401-405). HashMap order is canonicalised to
// row id order.
static FileIdentifierJobRunMetadata literal_job(Library& db, int32_t loc, uint64_t pool) {
  FileIdentifierJobRunMetadata meta;
  meta.total_orphan_paths = db.count_orphan_file_paths(loc, "");
  if (!meta.total_orphan_paths) return meta;
  int32_t cursor = db.get_orphan_file_paths(loc, 0, "", 1)[0].id;
  const size_t task_count = (meta.total_orphan_paths + 99) / 100;
  for (size_t step = 0; step < task_count; ++step) {
    const auto rows = db.get_orphan_file_paths(loc, cursor, "", 100);
    if (rows.empty()) {
      meta.early_finish = true;
      break;
    }
    const auto md = make_metadata(rows, pool);
    std::vector<size_t> ok;  // mod.rs:105-147: rows whose FileMetadata failed drop out
    for (size_t i = 0; i < rows.size(); ++i)
      if (md[i].ok()) ok.push_back(i);
    std::vector<std::string> unique;
    for (size_t i : ok)
      if (md[i].value().cas_id && std::find(unique.begin(), unique.end(), *md[i].value().cas_id) == unique.end())
        unique.push_back(*md[i].value().cas_id);
    for (size_t i : ok) db.set_cas_id(rows[i].id, md[i].value().cas_id);
    const auto existing = db.existing_objects(unique);
    std::set<std::string> existing_cas;
    for (const auto& [oid, cs] : existing) existing_cas.insert(cs.begin(), cs.end());
    for (size_t i : ok) {
      const auto& c = md[i].value().cas_id;
      if (!c) continue;
      for (const auto& [oid, cs] : existing)
        if (std::find(cs.begin(), cs.end(), *c) != cs.end()) {
          db.connect(rows[i].id, oid);
          ++meta.total_objects_linked;
          break;
        }
    }
    for (size_t i : ok) {
      const auto& c = md[i].value().cas_id;
      if (c && existing_cas.count(*c)) continue;
      db.connect(rows[i].id, db.create_object(md[i].value().kind, rows[i].date_created));
      ++meta.total_objects_created;
    }
    ++meta.steps;
    cursor = rows.back().id;
  }
  meta.cursor = cursor;
  return meta;
}

static bool same_row(const FilePathRow& a, const FilePathRow& b) {
  return a.id == b.id && a.pub_id == b.pub_id && a.location_id == b.location_id &&
         a.materialized_path == b.materialized_path && a.name == b.name && a.extension == b.extension &&
         a.is_dir == b.is_dir && a.size_in_bytes == b.size_in_bytes && a.cas_id == b.cas_id &&
         a.object_id == b.object_id && a.integrity_checksum == b.integrity_checksum &&
         a.date_created == b.date_created && a.kind == b.kind && a.inode == b.inode && a.hidden == b.hidden;
}

static bool same_rows(const std::vector<FilePathRow>& a, const std::vector<FilePathRow>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!same_row(a[i], b[i])) return false;
  return true;
}

// the shallow identifier (shallow.rs:24-142) on memory and SQLite, batches of
// 100 and 10000: one directory level only, its own task_count, the same
// cursor steps; against the oracle's job over exactly that level's orphans
static void test_shallow() {
  MemoryLibrary base;
  auto rows = make_rows(4000, 17);
  for (auto& r : rows) r = base.add_file_path(r);
  g_err_mod = 7;
  g_none_mod = 5;
  for (const char* dir : {"/sub/", "", "/sub/deeper/", "/nope/"}) {
    // a fresh library per level, so the oracle sees no existing Objects
    MemoryLibrary mem = base, mem_b = base;
    auto sql = SqliteLibrary::open(":memory:");
    std::vector<FilePathRow> copy = base.file_paths;
    sql->add_file_paths(copy);
    const std::string d = *dir ? dir : "/";
    const auto orphans = mem.get_orphan_file_paths_in_dir(1, 0, d, 1u << 30);
    for (const auto& r : orphans) CHECK(r.materialized_path == d, "shallow orphan outside %s", d.c_str());
    CHECK(mem.count_orphan_file_paths_in_dir(1, d) == orphans.size() &&
              sql->count_orphan_file_paths_in_dir(1, d) == orphans.size(),
          "shallow count %s", d.c_str());
    // the oracle over the level's orphans in id order (nothing exists before)
    auto md = make_metadata(orphans, 300);
    std::vector<uint64_t> keys(orphans.size(), 0);
    std::vector<uint8_t> has(orphans.size(), 0);
    std::vector<int32_t> st(orphans.size(), 0);
    for (size_t i = 0; i < orphans.size(); ++i) {
      if (!md[i].ok()) st[i] = md[i].error().code;
      else if (md[i].value().cas_id) has[i] = 1, keys[i] = hex_to_key(*md[i].value().cas_id);
    }
    std::vector<int64_t> link(orphans.size());
    int64_t linked = 0;
    const int64_t created = oracle_identifier_dedup(orphans.size(), keys.data(), has.data(), st.data(), 100, 0,
                                                    nullptr, link.data(), &linked);
    auto meta = [&](const std::vector<FilePathRow>& r) { return make_metadata(r, 300); };
    const Location loc{1, "/nowhere"};
    auto a = shallow_file_identifier_with(mem, loc, dir, 100, meta, oracle_group_by(100));
    auto b = shallow_file_identifier_with(*sql, loc, dir, 100, meta, oracle_group_by(100));
    auto c = shallow_file_identifier_with(mem_b, loc, dir, 10000, meta, oracle_group_by(100));
    CHECK(a.orphans == orphans.size() && (int64_t)a.created == created && (int64_t)a.linked == linked,
          "shallow %s: created/linked %zu/%zu, oracle %lld/%lld", d.c_str(), a.created, a.linked, (long long)created,
          (long long)linked);
    for (const auto* o : {&b, &c})
      CHECK(o->created == a.created && o->linked == a.linked && o->steps == a.steps && o->cursor == a.cursor &&
                o->rereads == a.rereads,
            "shallow %s: %zu/%zu/%zu steps vs %zu/%zu/%zu", d.c_str(), a.created, a.linked, a.steps, o->created,
            o->linked, o->steps);
    std::printf("shallow %s: %zu orphans, created %zu linked %zu in %zu steps, %zu re-reads (memory == sqlite, "
                "batches 100 == 10000 == oracle)\n",
                d.c_str(), a.orphans, a.created, a.linked, a.steps, a.rereads);
    for (const auto& r : mem.file_paths) {
      auto s = sql->file_path(r.id);
      CHECK(s && same_row(r, *s), "shallow row %d memory vs sqlite", r.id);
      const FilePathRow* b = mem_b.file_path(r.id);
      CHECK(b && same_row(r, *b), "shallow row %d batch 100 vs 10000", r.id);
      // rows of other levels are untouched
      if (r.materialized_path != d) CHECK(same_row(r, *base.file_path(r.id)), "shallow touched row %d", r.id);
    }
  }
  g_err_mod = 97;
  g_none_mod = 31;
}

static void test_parity(bool cas_index) {
  MemoryLibrary mem;
  auto sql = SqliteLibrary::open(":memory:", cas_index);
  auto rows = make_rows(3000, 5);
  for (auto& r : rows) r = mem.add_file_path(r);
  sql->add_file_paths(rows);
  // an identified slice with Objects, in both
  for (int32_t id = 1; id <= 3000; id += 17) {
    const auto* r = mem.file_path(id);
    if (r->is_dir || r->size_in_bytes == 0) continue;
    const std::string cas = key_to_hex(mix((uint64_t)id % 50));
    mem.set_cas_id(id, cas);
    sql->set_cas_id(id, cas);
    const int32_t om = mem.create_object(3, id), os = sql->create_object(3, id);
    CHECK(om == os, "object ids %d %d", om, os);
    mem.connect(id, om);
    sql->connect(id, os);
    // every third of them changed on disk: the indexer nulls cas_id and keeps
    // the Object (location/indexer), so the identifier re-reads them and
    // their Object becomes an existing one for their new cas_id in their step
    if (id % 3 == 1) {
      mem.set_cas_id(id, std::nullopt);
      sql->set_cas_id(id, std::nullopt);
    }
  }
  for (int32_t loc : {1, 2})
    for (const char* sub : {"", "/sub/", "/sub/deeper/", "/nope/"}) {
      CHECK(mem.count_orphan_file_paths(loc, sub) == sql->count_orphan_file_paths(loc, sub), "count %d %s", loc, sub);
      for (int32_t cursor : {0, 1, 500, 2999, 5000})
        for (size_t take : {1, 100, 10000})
          CHECK(same_rows(mem.get_orphan_file_paths(loc, cursor, sub, take),
                          sql->get_orphan_file_paths(loc, cursor, sub, take)),
                "orphans loc %d sub %s cursor %d take %zu", loc, sub, cursor, take);
      CHECK(same_rows(mem.file_paths_without_checksum(loc, sub), sql->file_paths_without_checksum(loc, sub)),
            "without checksum %d %s", loc, sub);
    }
  std::vector<std::string> want;
  for (int k = 0; k < 60; k += 3) want.push_back(key_to_hex(mix((uint64_t)k)));
  CHECK(mem.existing_objects(want) == sql->existing_objects(want), "existing objects");
  CHECK(sql->existing_objects({}).empty(), "existing objects of nothing");
  {
    auto a = mem.first_objects(want), b = sql->first_objects(want);  // one pair per cas_id, any order
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    CHECK(a == b && !a.empty(), "first objects");
  }
  CHECK(sql->first_objects({}).empty(), "first objects of nothing");
  {
    // one cas_id on two Objects (the smaller id is the first in DB order),
    // an Object with two cas_ids, a row without an Object, a cas_id nowhere
    for (bool index : {true, false}) {
      auto s = SqliteLibrary::open(":memory:", index);
      MemoryLibrary m;
      std::vector<FilePathRow> rows(5);
      const char* cas[5] = {"00000000000000aa", "00000000000000aa", "00000000000000aa", "00000000000000bb",
                            "00000000000000cc"};
      for (int i = 0; i < 5; ++i) {
        rows[i].location_id = 1;
        rows[i].materialized_path = "/";
        rows[i].name = "f" + std::to_string(i);
        rows[i].size_in_bytes = 1;
        rows[i].cas_id = std::string(cas[i]);
      }
      s->add_file_paths(rows);
      for (auto& r : rows) m.add_file_path(r);
      for (int k = 0; k < 3; ++k) {
        s->create_object(1, 0);
        m.create_object(1, 0);
      }
      const int32_t link[5][2] = {{1, 2}, {2, 1}, {3, 0}, {4, 3}, {5, 3}};
      for (const auto& l : link)
        if (l[1]) {
          s->connect(l[0], l[1]);
          m.connect(l[0], l[1]);
        }
      const std::vector<std::string> q{"00000000000000aa", "00000000000000bb", "00000000000000cc", "00000000000000dd"};
      const std::vector<std::pair<std::string, int32_t>> expect{
          {"00000000000000aa", 1}, {"00000000000000bb", 3}, {"00000000000000cc", 3}};
      auto fs = s->first_objects(q), fm = m.first_objects(q);
      std::sort(fs.begin(), fs.end());
      std::sort(fm.begin(), fm.end());
      CHECK(fs == expect, "first objects (cas_id index %d)", (int)index);
      CHECK(fm == expect, "first objects in memory");
      // the combined write leaves the row as set_cas_id then connect would
      s->set_cas_id_and_connect(3, std::string("00000000000000dd"), 2);
      const auto r3 = s->file_path(3);
      CHECK(r3 && r3->cas_id == std::string("00000000000000dd") && r3->object_id == 2, "set_cas_id_and_connect");
      s->set_cas_id_and_connect(3, std::nullopt, 1);
      CHECK(!s->file_path(3)->cas_id && s->file_path(3)->object_id == 1, "set_cas_id_and_connect null cas");
    }
  }

  // the identifier job on both: 100-row fetches (the reference's steps) on
  // one copy of each library, 1000- and 10000-row batches on others; every
  // result must be the same (a step's last row that stays an orphan — an
  // I/O error, an empty file — is read again by the next step, inside a
  // batch as across fetches)
  MemoryLibrary mem_b = mem, mem_c = mem, mem_lit = mem;
  // a second SQLite copy runs the job in 10000-row batches with the lookup
  // index traded for the host map (bulk identify); the re-identified rows
  // make it restore the index mid-job
  auto sql_bulk = SqliteLibrary::open(":memory:", cas_index);
  {
    std::vector<FilePathRow> all = mem.file_paths;
    sql_bulk->add_file_paths(all);
    for (const auto& o : mem.objects) sql_bulk->create_object(o.kind, o.date_created);
  }
  // and a file database in 1000-row batches: its job reads each next batch
  // through a second connection while the current batch's writes are open
  char fpath[] = "/tmp/sdcore_dbfXXXXXX";
  {
    const int fd = mkstemp(fpath);
    if (fd >= 0) close(fd);
    std::remove(fpath);
  }
  auto sql_file = SqliteLibrary::open(fpath, cas_index);
  {
    std::vector<FilePathRow> all = mem.file_paths;
    sql_file->add_file_paths(all);
    for (const auto& o : mem.objects) sql_file->create_object(o.kind, o.date_created);
  }
  CHECK(sql_file->concurrent_orphan_reads(), "a file database offers the read-ahead connection");
  CHECK(!sql->concurrent_orphan_reads(), "an in-memory database does not");
  size_t rereads = 0;
  for (int32_t loc : {1, 2}) {
    const auto orphans = mem.get_orphan_file_paths(loc, 0, "", 1u << 30);
    auto jf = run_job(*sql_file, loc, 1000, 400);
    auto jm = run_job(mem, loc, 100, 400);
    auto js = run_job(*sql, loc, 100, 400);
    auto jb = run_job(mem_b, loc, 1000, 400);
    auto jc = run_job(mem_c, loc, 10000, 400);
    FileIdentifierJobInit binit{Location{loc, "/nowhere"}, "", 10000};
    binit.bulk_identify = true;
    auto jk = run_file_identifier_job_with(
        *sql_bulk, binit, [&](const std::vector<FilePathRow>& rows) { return make_metadata(rows, 400); },
        oracle_group_by(100));
    CHECK(!sql_bulk->bulk_identify_active(), "bulk identify left on after the job");
    // taken for the first location; the second's 253 orphans are fewer than
    // a quarter of the rows the first left with a cas_id (probing is cheaper)
    if (cas_index) CHECK(jk.bulk_identify == (loc == 1), "bulk identify %d at loc %d", (int)jk.bulk_identify, loc);
    // the literal restatement of the reference's steps: no early finish
    // here, so it runs the same steps over the same rows
    auto jl = literal_job(mem_lit, loc, 400);
    CHECK(jl.total_objects_created == jm.total_objects_created && jl.total_objects_linked == jm.total_objects_linked &&
              jl.steps == jm.steps && jl.cursor == jm.cursor,
          "job loc %d vs the literal steps: created %zu/%zu linked %zu/%zu steps %zu/%zu cursor %d/%d", loc,
          jm.total_objects_created, jl.total_objects_created, jm.total_objects_linked, jl.total_objects_linked,
          jm.steps, jl.steps, jm.cursor, jl.cursor);
    for (const auto* j : {&js, &jb, &jc, &jk, &jf})
      CHECK(jm.total_objects_created == j->total_objects_created && jm.total_objects_linked == j->total_objects_linked &&
                jm.steps == j->steps && jm.cursor == j->cursor && jm.rereads == j->rereads,
            "job loc %d: memory/100 %zu/%zu/%zu steps cursor %d rereads %zu, other %zu/%zu/%zu steps cursor %d "
            "rereads %zu",
            loc, jm.total_objects_created, jm.total_objects_linked, jm.steps, jm.cursor, jm.rereads,
            j->total_objects_created, j->total_objects_linked, j->steps, j->cursor, j->rereads);
    rereads += jm.rereads;
    std::printf("job loc %d: %zu orphans, created %zu linked %zu in %zu steps, %zu re-reads (memory == sqlite, "
                "batches 100 == 1000 == 10000)\n",
                loc, orphans.size(), js.total_objects_created, js.total_objects_linked, js.steps, jm.rereads);
  }
  CHECK(rereads > 0, "no step re-read its predecessor's last row");
  for (const auto& r : mem.file_paths) {
    const FilePathRow* b = mem_b.file_path(r.id);
    const FilePathRow* c = mem_c.file_path(r.id);
    const FilePathRow* l = mem_lit.file_path(r.id);
    CHECK(b && c && same_row(r, *b) && same_row(r, *c), "row %d: batch 100 / 1000 / 10000 differ", r.id);
    CHECK(l && same_row(r, *l), "row %d: the job and the literal steps differ", r.id);
  }
  CHECK(mem_b.objects.size() == mem.objects.size() && mem_c.objects.size() == mem.objects.size() &&
            mem_lit.objects.size() == mem.objects.size(),
        "objects: %zu %zu %zu %zu", mem.objects.size(), mem_b.objects.size(), mem_c.objects.size(),
        mem_lit.objects.size());
  for (size_t i = 0; i < mem.objects.size() && i < mem_lit.objects.size(); ++i)
    CHECK(mem_lit.objects[i].id == mem.objects[i].id && mem_lit.objects[i].kind == mem.objects[i].kind &&
              mem_lit.objects[i].date_created == mem.objects[i].date_created,
          "object %zu vs the literal steps", i);
  for (int32_t id = 1; id <= 3000; ++id) {
    auto s = sql->file_path(id);
    CHECK(s && same_row(*mem.file_path(id), *s), "row %d after the job", id);
    auto k = sql_bulk->file_path(id);
    CHECK(k && same_row(*mem.file_path(id), *k), "row %d after the bulk job", id);
    auto f = sql_file->file_path(id);
    CHECK(f && same_row(*mem.file_path(id), *f), "row %d after the file database's job", id);
  }
  for (auto* lib : {sql.get(), sql_bulk.get(), sql_file.get()}) {
    auto so = lib->objects();
    CHECK(so.size() == mem.objects.size(), "object count %zu %zu", so.size(), mem.objects.size());
    for (size_t i = 0; i < so.size() && i < mem.objects.size(); ++i)
      CHECK(so[i].id == mem.objects[i].id && so[i].kind == mem.objects[i].kind &&
                so[i].date_created == mem.objects[i].date_created,
            "object %zu", i);
  }
  // the bulk job's library answers lookups as before (its index is back)
  CHECK(sql_bulk->existing_objects(want) == mem.existing_objects(want), "existing objects after the bulk job");
  sql_file.reset();
  for (const char* suf : {"", "-wal", "-shm"}) std::remove((std::string(fpath) + suf).c_str());
  // validator writes
  for (const auto& r : sql->file_paths_without_checksum(1, "/sub/")) {
    sql->set_integrity_checksum(r.id, std::string(64, 'b'));
    mem.set_integrity_checksum(r.id, std::string(64, 'b'));
  }
  CHECK(same_rows(mem.file_paths_without_checksum(1, ""), sql->file_paths_without_checksum(1, "")), "validator");
}

// forwards everything but the batch hooks: every write its own transaction
struct Autocommit : Library {
  Library& d;
  explicit Autocommit(Library& x) : d(x) {}
  size_t count_orphan_file_paths(int32_t l, const std::string& s) override { return d.count_orphan_file_paths(l, s); }
  std::vector<FilePathRow> get_orphan_file_paths(int32_t l, int32_t c, const std::string& s, size_t t) override {
    return d.get_orphan_file_paths(l, c, s, t);
  }
  size_t count_orphan_file_paths_in_dir(int32_t l, const std::string& s) override {
    return d.count_orphan_file_paths_in_dir(l, s);
  }
  std::vector<FilePathRow> get_orphan_file_paths_in_dir(int32_t l, int32_t c, const std::string& s,
                                                        size_t t) override {
    return d.get_orphan_file_paths_in_dir(l, c, s, t);
  }
  void set_cas_id(int32_t i, const std::optional<std::string>& c) override { d.set_cas_id(i, c); }
  std::vector<std::pair<int32_t, std::vector<std::string>>> existing_objects(
      const std::vector<std::string>& c) override {
    return d.existing_objects(c);
  }
  std::vector<std::pair<std::string, int32_t>> first_objects(const std::vector<std::string>& c) override {
    return d.first_objects(c);
  }
  void set_cas_id_and_connect(int32_t i, const std::optional<std::string>& c, int32_t o) override {
    d.set_cas_id_and_connect(i, c, o);
  }
  int32_t create_object(ObjectKind k, int64_t t) override { return d.create_object(k, t); }
  void connect(int32_t f, int32_t o) override { d.connect(f, o); }
  std::vector<FilePathRow> file_paths_without_checksum(int32_t l, const std::string& s) override {
    return d.file_paths_without_checksum(l, s);
  }
  void set_integrity_checksum(int32_t i, const std::string& c) override { d.set_integrity_checksum(i, c); }
};

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// forwards everything, timing each kind of call (where a step's DB time goes)
struct Timed : Library {
  Library& d;
  double t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  // reference_calls: the reference's calls only (the existing-Object query;
  // set_cas_id and connect as two writes), not first_objects' probes or the
  // combined write
  bool reference_calls;
  explicit Timed(Library& x, bool ref = false) : d(x), reference_calls(ref) {}
  template <class F>
  auto tm(int k, F f) -> decltype(f()) {
    const double t0 = now();
    struct G {
      double* acc;
      double t0;
      ~G() { *acc += now() - t0; }
    } g{&t[k], t0};
    return f();
  }
  size_t count_orphan_file_paths(int32_t l, const std::string& s) override {
    return tm(0, [&] { return d.count_orphan_file_paths(l, s); });
  }
  std::vector<FilePathRow> get_orphan_file_paths(int32_t l, int32_t c, const std::string& s, size_t n) override {
    return tm(1, [&] { return d.get_orphan_file_paths(l, c, s, n); });
  }
  size_t count_orphan_file_paths_in_dir(int32_t l, const std::string& s) override {
    return d.count_orphan_file_paths_in_dir(l, s);
  }
  std::vector<FilePathRow> get_orphan_file_paths_in_dir(int32_t l, int32_t c, const std::string& s,
                                                        size_t n) override {
    return tm(1, [&] { return d.get_orphan_file_paths_in_dir(l, c, s, n); });
  }
  void set_cas_id(int32_t i, const std::optional<std::string>& c) override { tm(2, [&] { d.set_cas_id(i, c); }); }
  std::vector<std::pair<int32_t, std::vector<std::string>>> existing_objects(
      const std::vector<std::string>& c) override {
    return tm(3, [&] { return d.existing_objects(c); });
  }
  std::vector<std::pair<std::string, int32_t>> first_objects(const std::vector<std::string>& c) override {
    if (reference_calls) return Library::first_objects(c);  // times existing_objects
    return tm(3, [&] { return d.first_objects(c); });
  }
  void set_cas_id_and_connect(int32_t i, const std::optional<std::string>& c, int32_t o) override {
    if (reference_calls) return Library::set_cas_id_and_connect(i, c, o);  // times both writes
    tm(8, [&] { d.set_cas_id_and_connect(i, c, o); });
  }
  int32_t create_object(ObjectKind k, int64_t t_) override { return tm(4, [&] { return d.create_object(k, t_); }); }
  std::vector<int32_t> create_objects(const std::vector<std::pair<ObjectKind, int64_t>>& kd) override {
    if (reference_calls) return Library::create_objects(kd);  // one insert per Object
    return tm(4, [&] { return d.create_objects(kd); });
  }
  void connect(int32_t f, int32_t o) override { tm(5, [&] { d.connect(f, o); }); }
  std::vector<FilePathRow> file_paths_without_checksum(int32_t l, const std::string& s) override {
    return d.file_paths_without_checksum(l, s);
  }
  void set_integrity_checksum(int32_t i, const std::string& c) override { d.set_integrity_checksum(i, c); }
  void begin_batch() override { tm(6, [&] { d.begin_batch(); }); }
  void end_batch() override { tm(7, [&] { d.end_batch(); }); }
  bool begin_bulk_identify(size_t n) override { return tm(3, [&] { return d.begin_bulk_identify(n); }); }
  void end_bulk_identify() override { tm(7, [&] { d.end_bulk_identify(); }); }
  // the read-ahead runs beside the writes (not timed: it overlaps them)
  bool concurrent_orphan_reads() override { return !reference_calls && d.concurrent_orphan_reads(); }
  std::vector<FilePathRow> get_orphan_file_paths_concurrent(int32_t l, int32_t c, const std::string& s,
                                                            size_t n) override {
    return d.get_orphan_file_paths_concurrent(l, c, s, n);
  }
};

static int bench(size_t n) {
  std::string out = "{\"what\": \"DB side of the identifier step (SqliteLibrary, WAL, synchronous=NORMAL), "
                    "group-by by the CPU oracle, metadata synthetic\", \"file_paths\": " + std::to_string(n);
  struct Mode {
    const char* name;
    size_t batch;
    bool autocommit, cas_index, bulk = false;
  };
  // the reference's shape: 100-row steps, a commit per write, no cas_id index
  // (a bounded sample: it is slow); then this library's batching and index
  for (Mode m : {Mode{"reference_shape_batch100_autocommit_no_cas_index", 100, true, false},
                 Mode{"batch100_autocommit", 100, true, true}, Mode{"batch100_txn", 100, false, true},
                 Mode{"batch10000_txn", 10000, false, true}, Mode{"batch10000_txn_bulk_identify", 10000, false, true, true}}) {
    const size_t rows_n = m.autocommit ? std::min<size_t>(n, 20000) : n;
    char path[] = "/tmp/sdcore_dbXXXXXX";
    const int fd = mkstemp(path);
    if (fd >= 0) close(fd);
    std::remove(path);
    {
      auto sql = SqliteLibrary::open(path, m.cas_index);
      auto rows = make_rows(rows_n, 9);
      for (auto& r : rows) {
        r.location_id = 1;
        r.is_dir = false;
        r.size_in_bytes = 1 + r.size_in_bytes;
        r.integrity_checksum.reset();
      }
      sql->add_file_paths(rows);
      Autocommit ac(*sql);
      Timed timed(m.autocommit ? static_cast<Library&>(ac) : *sql, !m.cas_index);
      const double t0 = now();
      auto meta = run_job(timed, 1, m.batch, rows_n / 3, m.bulk);
      const double dt = now() - t0;
      char b[512];
      std::snprintf(b, sizeof b,
                    ", \"%s\": {\"rows\": %zu, \"seconds\": %.3f, \"rows_per_s\": %.0f, \"created\": %zu, "
                    "\"linked\": %zu, \"seconds_by_call\": {\"count_orphans\": %.3f, \"get_orphans\": %.3f, "
                    "\"set_cas_id\": %.3f, \"existing_objects\": %.3f, \"create_object\": %.3f, "
                    "\"connect\": %.3f, \"set_cas_id_and_connect\": %.3f, \"begin\": %.3f, \"commit\": %.3f}}",
                    m.name, rows_n, dt, rows_n / dt, meta.total_objects_created, meta.total_objects_linked,
                    timed.t[0], timed.t[1], timed.t[2], timed.t[3], timed.t[4], timed.t[5], timed.t[8], timed.t[6],
                    timed.t[7]);
      out += b;
    }
    for (const char* suf : {"", "-wal", "-shm"}) std::remove((std::string(path) + suf).c_str());
  }
  std::printf("%s}\n", out.c_str());
  return 0;
}

static void touch(const std::string& p, size_t n) {
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) return;
  for (size_t i = 0; i < n; ++i) std::fputc((int)(i * 7), f);
  std::fclose(f);
}

// walk_location: IsolatedFilePathData naming, Rust's file_stem / extension,
// breadth-first order, symlinks skipped
static void test_walk() {
  char tmpl[] = "/tmp/sdcore_walkXXXXXX";
  const std::string root = mkdtemp(tmpl);
  mkdir((root + "/sub").c_str(), 0755);
  mkdir((root + "/sub/deeper").c_str(), 0755);
  mkdir((root + "/x.y").c_str(), 0755);
  touch(root + "/a.tar.gz", 10);
  touch(root + "/.bashrc", 3);
  touch(root + "/foo.", 0);
  touch(root + "/..hidden", 5);
  touch(root + "/noext", 1);
  touch(root + "/sub/b.TXT", 2000);
  touch(root + "/sub/deeper/c.bin", 200000);
  if (symlink((root + "/noext").c_str(), (root + "/link.bin").c_str()) != 0) std::perror("symlink");
  std::vector<IoError> errs;
  auto rows = walk_location(Location{7, root + "/"}, &errs);
  // expected in breadth-first, name order
  std::vector<std::tuple<std::string, std::string, std::string, bool, bool, uint64_t>> exp = {
      {"/", ".", "hidden", false, true, 5},      // "..hidden": rsplit at the last dot -> (".", "hidden")
      {"/", ".bashrc", "", false, true, 3},      // a leading dot alone is not an extension
      {"/", "a.tar", "gz", false, false, 10},
      {"/", "foo", "", false, false, 0},         // "foo.": extension Some("")
      {"/", "noext", "", false, false, 1},
      {"/", "sub", "", true, false, 0},
      {"/", "x.y", "", true, false, 0},          // directories keep their whole name
      {"/sub/", "b", "TXT", false, false, 2000},
      {"/sub/", "deeper", "", true, false, 0},
      {"/sub/deeper/", "c", "bin", false, false, 200000},
  };
  CHECK(errs.empty(), "walk errors");
  CHECK(rows.size() == exp.size(), "walk found %zu entries, want %zu", rows.size(), exp.size());
  for (size_t i = 0; i < rows.size() && i < exp.size(); ++i) {
    const auto& [mp, name, ext, dir, hidden, size] = exp[i];
    const auto& r = rows[i];
    CHECK(r.materialized_path == mp && r.name == name && r.extension == ext && r.is_dir == dir &&
              r.hidden == hidden && (dir || r.size_in_bytes == size) && r.location_id == 7 && r.inode != 0,
          "walk entry %zu: got (%s, %s, %s, %d, %d, %llu)", i, r.materialized_path.c_str(), r.name.c_str(),
          r.extension.c_str(), (int)r.is_dir, (int)r.hidden, (unsigned long long)r.size_in_bytes);
  }
  // full_path inverts the naming for files with an extension or none
  CHECK(full_path(Location{7, root}, rows[2]) == root + "/a.tar.gz", "full_path a.tar.gz");
  CHECK(full_path(Location{7, root}, rows[7]) == root + "/sub/b.TXT", "full_path sub/b.TXT");
  std::string cmd = "rm -rf " + root;
  if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "cleanup failed\n");
  std::printf("walk: %zu entries ok\n", rows.size());
}

static void write_bytes(const std::string& p, const std::string& bytes) {
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) { std::perror(p.c_str()); return; }
  std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
}

// kind detection (crates/file-ext: extensions.rs, magic.rs:176-235) as
// FileMetadata::new uses it; cases derived by hand from the reference tables
// and its extension_from_str test (extensions.rs:370-389). Its magic_bytes
// test (extensions.rs:391-564) passes bare extensions as paths and needs the
// absent packages/test-files corpus, so the magic cases here are synthetic.
static void test_kind() {
  // Extension::from_str
  CHECK(extension_kinds("jpg") == std::vector<ObjectKind>{ObjectKindImage}, "jpg");
  CHECK((extension_kinds("ts") == std::vector<ObjectKind>{ObjectKindVideo, ObjectKindCode}), "ts conflicts");
  CHECK((extension_kinds("MTS") == std::vector<ObjectKind>{ObjectKindVideo, ObjectKindCode}), "MTS conflicts");
  CHECK(extension_kinds("jeff").empty(), "jeff");
  CHECK(extension_kinds("").empty() && extension_kinds("j pg").empty(), "empty / space");
  CHECK(extension_kinds("3GP") == std::vector<ObjectKind>{ObjectKindVideo}, "3gp (serde rename)");
  CHECK(extension_kinds("7z") == std::vector<ObjectKind>{ObjectKindArchive}, "7z (serde rename)");
  CHECK(extension_kinds("_3gp").empty() && extension_kinds("_7z").empty(), "variant identifiers are not names");
  CHECK(extension_kinds("\xE2\x84\xAA" "ey") == std::vector<ObjectKind>{ObjectKindDocument}, "Kelvin sign lowercases to k");
  CHECK(extension_kinds("caf\xC3\xA9").empty(), "non-ASCII");
  const std::pair<const char*, ObjectKind> one[] = {
      {"pdf", ObjectKindDocument}, {"key", ObjectKindDocument}, {"hwp", ObjectKindDocument},
      {"mkv", ObjectKindVideo},    {"f4v", ObjectKindVideo},    {"raw", ObjectKindImage},
      {"rw2", ObjectKindImage},    {"flac", ObjectKindAudio},   {"ast", ObjectKindAudio},
      {"bz2", ObjectKindArchive},  {"jar", ObjectKindExecutable}, {"bat", ObjectKindExecutable},
      {"markdown", ObjectKindText}, {"bytes", ObjectKindEncrypted}, {"block", ObjectKindEncrypted},
      {"pub", ObjectKindKey},      {"keychain", ObjectKindKey}, {"woff2", ObjectKindFont},
      {"obj", ObjectKindMesh},     {"php6", ObjectKindCode},    {"dockerfile", ObjectKindCode},
      {"r", ObjectKindCode},       {"mdx", ObjectKindCode},     {"db", ObjectKindDatabase},
      {"azw3", ObjectKindBook},    {"tsconfig", ObjectKindConfig}, {"CSV", ObjectKindConfig},
  };
  for (const auto& [e, k] : one)
    CHECK(extension_kinds(e) == std::vector<ObjectKind>{k}, "extension %s", e);
  // resolve_conflicting on real files
  char tmpl[] = "/tmp/sdcore_kindXXXXXX";
  const std::string d = mkdtemp(tmpl);
  const std::string mpeg_ts("\x47\x40\x11\x10", 4);
  struct Case { std::string name, bytes; ObjectKind want; const char* why; };
  const Case cases[] = {
      {"clip.ts", mpeg_ts, ObjectKindVideo, "ts with the MPEG-TS sync byte"},
      {"app.ts", "export const x = 1;\n", ObjectKindCode, "typescript"},
      {"empty.ts", "", ObjectKindCode, "empty ts: the magic read fails -> Code"},
      {"clip.mts", mpeg_ts, ObjectKindVideo, "mts, sync byte first"},
      {"m2ts.mts", std::string("\x00\x00\x00\x47\x40", 5), ObjectKindVideo, "mts, sync byte at offset 3"},
      {"short.mts", "abc", ObjectKindCode, "mts shorter than the 4-byte window"},
      {"mod.mts", "export {}\n", ObjectKindCode, "typescript module"},
      {"UPPER.TS", mpeg_ts, ObjectKindUnknown, "conflict matched on the extension as written"},
      {"Photo.JPG", "x", ObjectKindImage, "case-insensitive"},
      {"notes.md", "# hi", ObjectKindText, "text"},
      {"a.tar.gz", "", ObjectKindArchive, "last extension"},
      {"Makefile", "all:", ObjectKindUnknown, "no extension"},
      {".bashrc", "x", ObjectKindUnknown, "dotfile: no extension"},
      {"trail.", "x", ObjectKindUnknown, "empty extension"},
      {"data.bin", "x", ObjectKindUnknown, "unknown extension"},
      {"k.\xE2\x84\xAA" "ey", "x", ObjectKindDocument, "Kelvin sign"},
      {"bad.\xFF" "ts", "x", ObjectKindUnknown, "extension not UTF-8"},
  };
  for (const auto& c : cases) {
    write_bytes(d + "/" + c.name, c.bytes);
    const ObjectKind got = object_kind_of(d + "/" + c.name);
    CHECK(got == c.want, "kind of %s (%s): %d, want %d", c.name.c_str(), c.why, got, c.want);
  }
  CHECK(object_kind_of(d + "/missing.jpg") == ObjectKindUnknown, "a file that does not open -> Unknown");
  // "x/." names x (a trailing "." is not a component); a file does not open
  // as a directory, a directory opens but its magic read fails -> Code
  CHECK(object_kind_of(d + "/clip.ts/.") == ObjectKindUnknown, "regular file with a trailing /.");
  mkdir((d + "/dir.ts").c_str(), 0755);
  CHECK(object_kind_of(d + "/dir.ts/.") == ObjectKindCode && object_kind_of(d + "/dir.ts//") == ObjectKindCode,
        "directory named *.ts");
  CHECK(!resolve_conflicting_kind(d + "/..") && !resolve_conflicting_kind("/"), "no file name");
  std::string cmd = "rm -rf " + d;
  if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "cleanup failed\n");
  std::printf("kind: %zu files ok\n", sizeof cases / sizeof cases[0]);
}

// SqliteLibrary's Object ids, a failing index rebuild and the read-ahead
// guard (round 5's review findings)
static void raw_sql(const char* path, const char* sql, int64_t* out = nullptr) {
  sqlite3* raw = nullptr;
  sqlite3_open_v2(path, &raw, SQLITE_OPEN_READWRITE, nullptr);
  sqlite3_stmt* st = nullptr;
  CHECK(sqlite3_prepare_v2(raw, sql, -1, &st, nullptr) == SQLITE_OK, "raw sql: %s", sql);
  const int rc = sqlite3_step(st);
  if (out && rc == SQLITE_ROW) *out = sqlite3_column_int64(st, 0);
  sqlite3_finalize(st);
  sqlite3_close(raw);
}

static void test_library_edges() {
  char fpath[] = "/tmp/sdcore_idsXXXXXX";
  {
    const int fd = mkstemp(fpath);
    if (fd >= 0) close(fd);
    std::remove(fpath);
  }
  {
    auto db = SqliteLibrary::open(fpath, true);
    for (int i = 0; i < 5; ++i) db->create_object(ObjectKindImage, 0);  // ids 1..5
  }
  // the top Objects deleted: AUTOINCREMENT never hands out 4 or 5 again, and
  // neither may the multi-row INSERTs, which give their ids
  raw_sql(fpath, "DELETE FROM object WHERE id > 3");
  {
    auto db = SqliteLibrary::open(fpath, true);
    const auto ids = db->create_objects(std::vector<std::pair<ObjectKind, int64_t>>(70, {ObjectKindImage, 0}));
    bool seq = ids.size() == 70;
    for (size_t i = 0; seq && i < ids.size(); ++i) seq = ids[i] == (int32_t)(6 + i);
    CHECK(seq, "bulk Object ids after deleted top Objects start at %d", ids.empty() ? -1 : ids[0]);
    const int32_t one = db->create_object(ObjectKindImage, 0);
    CHECK(one == 76, "the next single Object %d", one);
  }
  // an index rebuild that fails inside a batch: the batch stays usable (its
  // commit succeeds), bulk identify stays on, and a later restore rebuilds
  {
    auto db = SqliteLibrary::open(fpath, true);
    CHECK(db->begin_bulk_identify(100), "bulk identify on an empty file_path table");
    db->begin_batch();
    setenv("SDCORE_FAULT", "index_restore", 1);
    bool threw = false;
    try {
      db->end_bulk_identify();
    } catch (const std::exception&) {
      threw = true;
    }
    unsetenv("SDCORE_FAULT");
    CHECK(threw && db->bulk_identify_active(), "a failing rebuild raises and keeps bulk identify on");
    const int32_t id = db->create_object(ObjectKindText, 0);
    bool committed = true;
    try {
      db->end_batch();
    } catch (const std::exception&) {
      committed = false;
    }
    CHECK(committed && id == 77, "the batch after a failing rebuild commits (object %d)", id);
    db->end_bulk_identify();
    CHECK(!db->bulk_identify_active(), "the second rebuild ends bulk identify");
  }
  int64_t idx = 0, objs = 0;
  raw_sql(fpath, "SELECT COUNT(*) FROM sqlite_master WHERE name = 'file_path_cas_id_idx'", &idx);
  raw_sql(fpath, "SELECT COUNT(*) FROM object", &objs);
  CHECK(idx == 1 && objs == 3 + 70 + 1 + 1, "index restored (%lld), objects %lld", (long long)idx, (long long)objs);
  // the read-ahead call without its connection refuses instead of reading
  // through the writer's (NOMUTEX) connection
  auto mem = SqliteLibrary::open(":memory:", true);
  bool refused = false;
  try {
    (void)mem->get_orphan_file_paths_concurrent(1, 0, "", 10);
  } catch (const std::logic_error&) {
    refused = !mem->concurrent_orphan_reads();
  }
  CHECK(refused, "concurrent read without the read-ahead connection");
  for (const char* suf : {"", "-wal", "-shm"}) std::remove((std::string(fpath) + suf).c_str());
}

// set_cas_ids_and_connect (64 rows per UPDATE ... FROM (VALUES ...)) against
// the same writes one by one: with and without bulk identify, a chunk holding
// rows that already have an Object (bulk: the statement skips them, they take
// the general path) and a remainder shorter than a chunk
static void test_cas_links() {
  for (bool bulk : {false, true}) {
    auto many = SqliteLibrary::open(":memory:", true);
    auto one = SqliteLibrary::open(":memory:", true);
    for (auto* db : {many.get(), one.get()}) {
      std::vector<FilePathRow> rows(150);
      for (size_t i = 0; i < rows.size(); ++i) {
        rows[i].location_id = 1;
        rows[i].materialized_path = "/";
        rows[i].name = "f" + std::to_string(i);
        rows[i].size_in_bytes = 1 + i;
      }
      db->add_file_paths(rows);
      for (int i = 0; i < 40; ++i) db->create_object(ObjectKindImage, i);
      // rows 10 and 70 have an Object (and 10 a cas_id) before the job
      db->set_cas_id_and_connect(10, std::string("00000000000000aa"), 3);
      db->connect(70, 4);
      if (bulk) CHECK(db->begin_bulk_identify(150), "bulk identify (%d)", (int)bulk);
    }
    std::vector<Library::CasLink> w;
    for (int32_t id = 1; id <= 150; ++id) {
      std::optional<std::string> cas;
      if (id % 11) {
        char b[17];
        std::snprintf(b, sizeof b, "%016x", (unsigned)(id % 37));
        cas = std::string(b);
      }
      w.push_back({id, cas, 1 + (id * 7) % 40});
    }
    many->set_cas_ids_and_connect(w);
    for (const auto& x : w) one->set_cas_id_and_connect(x.file_path_id, x.cas_id, x.object_id);
    std::vector<std::string> want;
    for (int k = 0; k < 37; ++k) {
      char b[17];
      std::snprintf(b, sizeof b, "%016x", (unsigned)k);
      want.push_back(b);
    }
    want.push_back("00000000000000aa");
    auto sorted = [](std::vector<std::pair<std::string, int32_t>> v) {
      std::sort(v.begin(), v.end());
      return v;
    };
    CHECK(sorted(many->first_objects(want)) == sorted(one->first_objects(want)), "first objects (bulk %d)", (int)bulk);
    if (bulk) {
      many->end_bulk_identify();
      one->end_bulk_identify();
      CHECK(sorted(many->first_objects(want)) == sorted(one->first_objects(want)), "first objects after the rebuild");
    }
    for (int32_t id = 1; id <= 150; ++id) {
      const auto a = many->file_path(id), b = one->file_path(id);
      CHECK(a && b && a->cas_id == b->cas_id && a->object_id == b->object_id, "row %d (bulk %d)", id, (int)bulk);
    }
  }
}

int main(int argc, char** argv) {
  if (argc > 2 && std::strcmp(argv[1], "--bench") == 0) return bench((size_t)std::atoll(argv[2]));
  test_parity(true);
  test_parity(false);
  test_shallow();
  // many rows that stay orphans: re-reads at most step ends
  g_err_mod = 7;
  g_none_mod = 5;
  test_parity(true);
  g_err_mod = 97;
  g_none_mod = 31;
  test_walk();
  test_kind();
  test_library_edges();
  test_cas_links();
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "ALL OK", failures);
  return failures ? 1 : 0;
}
