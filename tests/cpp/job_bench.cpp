// The whole identifier job on real files, GPU against the reference's shape.
// TEST INFRASTRUCTURE: links oracle/build/liboracle.so for the CPU leg.
//
//   job_bench N [sample]
//
// Writes N files (C2 sizes: uniform 1 B..100 KiB, 15 % copies of an earlier
// file's content, a few empty files) into a temporary location, indexes them
// (walk_location) into a SQLite file and runs the file identifier job
// (file_identifier_job.rs:33-319) over them three ways, each on a fresh copy
// of the database:
//
//   gpu_batch10000    run_file_identifier_job, 10000-row fetches (GPU cas_ids
//                     and group-by, SqliteLibrary's probes and combined writes)
//   gpu_batch100      the same, 100-row fetches (the reference's step size)
//   reference_shape   100-row steps with the reference's CPU shape: per step
//                     metadata + cas.rs reads on 16 I/O threads and upstream
//                     BLAKE3 on one thread (oracle_cpu_faithful), the oracle's
//                     group-by, the reference's DB calls (existing-Object query
//                     without a cas_id index; set_cas_id and connect as two
//                     writes), over the first `sample` rows' worth of steps
//
// metadata_s: the legs' FileMetadata time (stat, kind, cas_ids); the job's
// loop computes a batch's while the previous batch's Objects are written, so
// it overlaps the DB time (seconds is the wall time of the whole job).
//
// Every leg must leave the same rows: cas_id and object_id per file_path and
// the same Objects (kind, date_created); the program exits non-zero if not.
// Prints one JSON line. Files live in the page cache (just written).
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../oracle/oracle.h"
#include "sdcore.hpp"

using namespace sdcore;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Spec {
  std::string path;
  uint64_t size, content;
};

static std::vector<Spec> make_files(const std::string& root, size_t n) {
  std::vector<Spec> f(n);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t h = mix(i + 1);
    const size_t dir = i / 1000;
    char name[64];
    std::snprintf(name, sizeof name, "/d%03zu/f%07zu.bin", dir, i);
    f[i].path = root + name;
    if (h % 500 == 0) {
      f[i].size = 0;  // empty: not an orphan (size != 0 filter)
      f[i].content = 0;
    } else if (i > 0 && (h >> 20) % 100 < 15) {
      f[i] = {f[i].path, 0, 0};
      const Spec& src = f[(h >> 32) % i];  // a copy of an earlier file
      f[i].size = src.size;
      f[i].content = src.content;
    } else {
      f[i].size = 1 + (h >> 11) % (100 * 1024);
      f[i].content = h;
    }
  }
  for (size_t d = 0; d * 1000 < n; ++d) {
    char dir[32];
    std::snprintf(dir, sizeof dir, "/d%03zu", d);
    mkdir((root + dir).c_str(), 0755);
  }
  const unsigned T = 16;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::vector<uint64_t> buf;
      for (size_t i = t; i < n; i += T) {
        buf.resize((f[i].size + 7) / 8);
        for (size_t w = 0; w < buf.size(); ++w) buf[w] = mix(f[i].content ^ (w * 0x100000001B3ull));
        FILE* o = std::fopen(f[i].path.c_str(), "wb");
        if (!o) {
          std::perror(f[i].path.c_str());
          std::exit(2);
        }
        if (f[i].size) std::fwrite(buf.data(), 1, f[i].size, o);
        std::fclose(o);
      }
    });
  for (auto& x : th) x.join();
  return f;
}

// the reference's DB calls only: the existing-Object query for the lookup,
// set_cas_id and connect as two writes
struct ReferenceCalls : Library {
  Library& d;
  explicit ReferenceCalls(Library& x) : d(x) {}
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
  int32_t create_object(ObjectKind k, int64_t t) override { return d.create_object(k, t); }
  void connect(int32_t f, int32_t o) override { d.connect(f, o); }
  std::vector<FilePathRow> file_paths_without_checksum(int32_t l, const std::string& s) override {
    return d.file_paths_without_checksum(l, s);
  }
  void set_integrity_checksum(int32_t i, const std::string& c) override { d.set_integrity_checksum(i, c); }
  void begin_batch() override { d.begin_batch(); }
  void end_batch() override { d.end_batch(); }
};

static GroupBy oracle_group_by() {
  return [](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
            const std::vector<uint64_t>& e, sdcas_job_window& w) {
    Engine::Dedup d;
    d.link.assign(k.size(), 0);
    int64_t linked = 0;
    oracle_job_window ow{w.max_steps, (int32_t)w.more, 0, 0, 0, 0};
    d.created = oracle_identifier_job(k.size(), k.data(), h.data(), st.data(), SDCAS_IDENTIFIER_CHUNK_SIZE, e.size(),
                                      e.empty() ? nullptr : e.data(), &ow, d.link.data(), &linked);
    d.linked = linked;
    w.steps = ow.steps;
    w.rows = ow.rows;
    w.rereads = ow.rereads;
    return d;
  };
}

struct Leg {
  std::string name;
  double seconds = 0, metadata_s = 0, group_by_s = 0;
  size_t rows = 0;
  FileIdentifierJobRunMetadata meta;
  std::vector<std::tuple<int32_t, std::optional<std::string>, std::optional<int32_t>>> state;
  std::vector<std::pair<int32_t, int64_t>> objects;
};

static std::string fresh_db() {
  char path[] = "/tmp/sd_jobXXXXXX";
  const int fd = mkstemp(path);
  if (fd >= 0) close(fd);
  std::remove(path);
  return path;
}

static void drop_db(const std::string& p) {
  for (const char* suf : {"", "-wal", "-shm"}) std::remove((p + suf).c_str());
}

static void snapshot(SqliteLibrary& sql, const std::vector<FilePathRow>& rows, Leg& L) {
  for (const auto& r : rows) {
    auto x = sql.file_path(r.id);
    L.state.emplace_back(r.id, x->cas_id, x->object_id);
  }
  for (const auto& o : sql.objects()) L.objects.emplace_back(o.kind, o.date_created);
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)std::atoll(argv[1]) : 100000;
  const size_t sample = argc > 2 ? (size_t)std::atoll(argv[2]) : SIZE_MAX;  // file_path rows
  std::unique_ptr<Engine> engine;
  try {
    // JOB_IO_THREADS: the library's reader threads (A/B: the readers and
    // SQLite's one writer share the box's CPU quota)
    Engine::Options o;
    if (const char* v = std::getenv("JOB_IO_THREADS")) o.io_threads = (uint32_t)std::atoi(v);
    engine = Engine::open(o);
  } catch (const LibraryError& e) {
    std::fprintf(stderr, "job_bench: %s\n", e.what());
    return 2;
  }
  char tmpl[] = "/tmp/sd_job_filesXXXXXX";
  const std::string root = mkdtemp(tmpl);
  double t0 = now();
  const auto files = make_files(root, n);
  const double write_s = now() - t0;
  {
    // the engine's one-time set-up (staging memory, reader threads, kernel
    // loads: 0.13-0.19 s on the box) is no leg's: one call over a few files
    std::vector<std::pair<std::string, uint64_t>> warm;
    for (size_t i = 0; i < std::min<size_t>(files.size(), 64); ++i) warm.emplace_back(files[i].path, files[i].size);
    (void)engine->generate_cas_ids(warm);
  }
  uint64_t bytes = 0;
  for (const auto& f : files) bytes += f.size;
  const Location loc{1, root};
  auto rows = walk_location(loc);  // breadth-first, names sorted
  for (size_t i = 0; i < rows.size(); ++i) rows[i].id = (int32_t)(i + 1);

  std::vector<Leg> legs;
  auto run_leg = [&](const std::string& name, size_t batch, bool reference, bool bulk = false) {
    Leg L;
    L.name = name;
    const std::string db = fresh_db();
    {
      auto sql = SqliteLibrary::open(db, !reference);
      std::vector<FilePathRow> copy = rows;
      sql->add_file_paths(copy);
      ReferenceCalls rc(*sql);
      Library& lib = reference ? static_cast<Library&>(rc) : *sql;
      FileIdentifierJobInit init{loc, "", batch};
      init.bulk_identify = bulk;
      MetadataFn md;
      GroupBy gb;
      if (!reference) {
        md = [&](const std::vector<FilePathRow>& r) {
          const double a = now();
          std::vector<std::pair<std::string, ObjectKind>> f(r.size());
          std::vector<uint64_t> hints(r.size());
          for (size_t i = 0; i < r.size(); ++i) {
            f[i] = {full_path(loc, r[i]), r[i].kind};
            hints[i] = r[i].size_in_bytes;  // the indexer's sizes (walk_location)
          }
          auto out = file_metadata_batch(*engine, f, &hints);
          L.metadata_s += now() - a;
          L.rows += r.size();
          return out;
        };
        gb = [&](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
                 const std::vector<uint64_t>& e, sdcas_job_window& w) {
          const double a = now();
          auto d = engine->dedup(k, h, st, SDCAS_IDENTIFIER_CHUNK_SIZE, e, &w);
          L.group_by_s += now() - a;
          return d;
        };
      } else {
        md = [&](const std::vector<FilePathRow>& r) {
          const double a = now();
          const size_t m = r.size();
          std::vector<std::string> paths(m);
          std::vector<const char*> cp;
          std::vector<uint64_t> sizes;
          std::vector<size_t> idx;
          std::vector<Result<FileMetadata>> out;
          std::vector<FileMetadata> fm(m);
          std::vector<std::optional<IoError>> err(m);
          for (size_t i = 0; i < m; ++i) {
            paths[i] = full_path(loc, r[i]);
            struct stat sb;
            if (::stat(paths[i].c_str(), &sb) != 0) {
              err[i] = IoError{errno, paths[i]};
              continue;
            }
            fm[i].kind = r[i].kind >= 0 ? r[i].kind : object_kind_of(paths[i]);
            fm[i].len = (uint64_t)sb.st_size;
            if (fm[i].len) {
              cp.push_back(paths[i].c_str());
              sizes.push_back(fm[i].len);
              idx.push_back(i);
            }
          }
          std::vector<uint64_t> keys(cp.size());
          std::vector<int32_t> st(cp.size());
          double secs[2] = {0, 0};
          int kind = 0;
          char ver[64];
          if (!cp.empty())
            oracle_cpu_faithful(cp.data(), sizes.data(), cp.size(), SDCAS_IDENTIFIER_CHUNK_SIZE, 16, 1, keys.data(),
                                st.data(), secs, &kind, ver);
          for (size_t k = 0; k < idx.size(); ++k) {
            if (st[k]) err[idx[k]] = IoError{st[k], paths[idx[k]]};
            else fm[idx[k]].cas_id = key_to_hex(keys[k]);
          }
          for (size_t i = 0; i < m; ++i) {
            if (err[i]) out.emplace_back(*err[i]);
            else out.emplace_back(fm[i]);
          }
          L.metadata_s += now() - a;
          L.rows += m;
          return out;
        };
        auto og = oracle_group_by();
        gb = [&, og](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
                     const std::vector<uint64_t>& e, sdcas_job_window& w) {
          const double a = now();
          auto d = og(k, h, st, e, w);
          L.group_by_s += now() - a;
          return d;
        };
      }
      const double a = now();
      L.meta = run_file_identifier_job_with(lib, init, md, gb);
      L.seconds = now() - a;
      snapshot(*sql, rows, L);
    }
    drop_db(db);
    legs.push_back(std::move(L));
  };
  run_leg("gpu_batch10000", 10000, false);
  run_leg("gpu_batch100", 100, false);
  run_leg("gpu_batch10000_bulk_identify", 10000, false, true);
  // the reference shape over a bounded sample: the first `sample` files only
  // (a fresh location holding just them keeps every leg's job whole)
  const bool sampled = sample < rows.size();
  if (sampled) rows.resize(sample);
  run_leg("reference_shape", 100, true);
  if (sampled) {
    // the GPU at batch 10000 over the same sample, for the equality check
    run_leg("gpu_batch10000_sample", 10000, false);
  }
  int bad = 0;
  auto same = [&](const Leg& a, const Leg& b) {
    return a.state == b.state && a.objects == b.objects &&
           a.meta.total_objects_created == b.meta.total_objects_created &&
           a.meta.total_objects_linked == b.meta.total_objects_linked;
  };
  if (!same(legs[0], legs[1]) || !same(legs[0], legs[2])) ++bad;
  if (!same(legs[3], sampled ? legs[4] : legs[0])) ++bad;
  std::string out = "{\"what\": \"the file identifier job end to end on real files (page cache) into SQLite\", ";
  char b[1024];
  std::snprintf(b, sizeof b,
                "\"files\": %zu, \"bytes\": %llu, \"orphans\": %zu, \"files_written_s\": %.2f, \"sample\": %zu, "
                "\"equal_end_state\": %s",
                n, (unsigned long long)bytes, legs[0].meta.total_orphan_paths, write_s, sampled ? sample : n,
                bad ? "false" : "true");
  out += b;
  for (const auto& L : legs) {
    std::snprintf(b, sizeof b,
                  ", \"%s\": {\"orphans\": %zu, \"seconds\": %.3f, \"orphans_per_s\": %.0f, \"metadata_s\": %.3f, "
                  "\"group_by_s\": %.3f, \"rows_fetched\": %zu, \"steps\": %zu, \"batches\": %zu, "
                  "\"created\": %zu, \"linked\": %zu, \"bulk_identify\": %s}",
                  L.name.c_str(), L.meta.total_orphan_paths, L.seconds, L.meta.total_orphan_paths / L.seconds,
                  L.metadata_s, L.group_by_s, L.rows, L.meta.steps, L.meta.batches,
                  L.meta.total_objects_created, L.meta.total_objects_linked, L.meta.bulk_identify ? "true" : "false");
    out += b;
  }
  std::printf("%s}\n", out.c_str());
  std::fflush(stdout);
  for (const auto& f : files) std::remove(f.path.c_str());
  for (size_t d = 0; d * 1000 < n; ++d) {
    char dir[32];
    std::snprintf(dir, sizeof dir, "/d%03zu", d);
    rmdir((root + dir).c_str());
  }
  rmdir(root.c_str());
  return bad ? 1 : 0;
}
