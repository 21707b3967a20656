// sqlite_library.cpp — SqliteLibrary: the DB side of the identifier join
//  over SQLite, with the columns of the reference's
// file_path / object models (core/prisma/schema.prisma) and its queries
// (file_identifier_job.rs:251-319, mod.rs:157-342, validator_job.rs:107-172)
// as prepared statements. See include/sdcore.hpp.
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <unordered_map>

#include "sdcore.hpp"
#include "sqlite3_min.h"

namespace sdcore {

namespace {

struct Stmt {
  sqlite3_stmt* s = nullptr;
  ~Stmt() {
    if (s) sqlite3_finalize(s);
  }
};

void be64(uint64_t v, uint8_t out[8]) {
  for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(v >> (56 - 8 * i));
}

uint64_t from_be64(const void* p, int n) {
  uint64_t v = 0;
  const uint8_t* b = (const uint8_t*)p;
  for (int i = 0; i < n && i < 8; ++i) v = (v << 8) | b[i];
  return v;
}

// as MemoryLibrary's (sdcore.cpp pub_id_of): tag, then the id big-endian in
// the last 8 bytes, so the UNIQUE pub_id index appends in creation order
PubId pub_id(uint32_t tag, int64_t id) {
  PubId p{};
  std::memcpy(p.data(), &tag, 4);
  for (int i = 0; i < 8; ++i) p[8 + i] = (uint8_t)((uint64_t)id >> (56 - 8 * i));
  return p;
}

}  // namespace

struct SqliteLibrary::Impl {
  sqlite3* db = nullptr;
  Stmt count_orphans_dir, get_orphans_dir;
  Stmt count_orphans, get_orphans, set_cas, want_clear, want_add, existing, new_object, connect, no_checksum,
      set_checksum, add_path, get_path, all_objects, first_object, set_cas_connect;
  Stmt row_state, set_cas_connect_free, count_cas, load_first;
  static constexpr int kManyObjects = 64;
  Stmt new_objects;  // kManyObjects rows of (id, pub_id, kind, date_created)
  static constexpr int kManyLinks = 64;
  Stmt links, links_free;  // kManyLinks rows of (id, cas_id, object_id); _free: rows without an Object
  // the job's read-ahead connection (concurrent_orphan_reads): read-only, one
  // statement, used by one thread at a time
  std::string path;
  sqlite3* rdb = nullptr;
  Stmt r_get_orphans;
  bool reader_tried = false;
  std::mutex rmu;
  int64_t next_object = 1;
  bool cas_index = false;
  int batch_depth = 0;
  // bulk identify (begin_bulk_identify): the cas_id index is dropped and its
  // answer to first_objects kept here, cas_id -> MIN(object_id) over the
  // rows with both
  bool bulk = false;
  std::unordered_map<std::string, int32_t> first;
  // the WAL checkpoint a bulk job deferred, run after it on a connection of
  // its own (joined by the next bulk job and at close)
  std::thread checkpointer;
  void join_checkpoint() {
    if (checkpointer.joinable()) checkpointer.join();
  }
  ~Impl() { join_checkpoint(); }

  void first_min(const std::string& cas, int32_t oid) {
    auto it = first.find(cas);
    if (it == first.end()) first.emplace(cas, oid);
    else if (oid < it->second) it->second = oid;
  }
  // (cas_id, object_id) of a row before a write
  std::pair<std::optional<std::string>, std::optional<int32_t>> state(int32_t id) {
    sqlite3_bind_int64(row_state.s, 1, id);
    std::pair<std::optional<std::string>, std::optional<int32_t>> r;
    const int rc = sqlite3_step(row_state.s);
    if (rc == SQLITE_ROW) {
      r.first = col_text(row_state.s, 0);
      if (sqlite3_column_type(row_state.s, 1) != SQLITE_NULL) r.second = (int32_t)sqlite3_column_int64(row_state.s, 1);
    } else if (rc != SQLITE_DONE) {
      fail("row state");
    }
    sqlite3_reset(row_state.s);
    sqlite3_clear_bindings(row_state.s);
    return r;
  }
  void index_restore() {
    if (!bulk) return;
    if (batch_depth) exec("COMMIT");  // CREATE INDEX in its own transaction
    try {
      static const bool trace = [] {
        const char* v = getenv("SDCORE_TRACE_JOB");
        return v && *v && strcmp(v, "0") != 0;
      }();
      // (PRAGMA temp_store = MEMORY for the sort measured no faster, 31-34 ms
      // either way, and changing temp_store drops the connection's TEMP
      // tables — want_cas)
      const auto t0 = std::chrono::steady_clock::now();
      // the sorter may use helper threads for the one big sort (PRAGMA threads)
      exec("PRAGMA threads = 4");
      if (const char* f = getenv("SDCORE_FAULT"); f && !strcmp(f, "index_restore"))  // tests: a failing rebuild
        exec("CREATE INDEX file_path_cas_id_idx_fault ON no_such_table (x)");
      exec("CREATE INDEX IF NOT EXISTS file_path_cas_id_idx ON file_path (cas_id)");
      exec("PRAGMA threads = 0");
      const auto t1 = std::chrono::steady_clock::now();
      // the WAL checkpoints the job deferred, once (begin_bulk_identify):
      // copying the job's pages from the WAL into the database file is
      // housekeeping no reader waits for (WAL readers see the pages either
      // way), so a file database runs it on a connection of its own after
      // the job (SDCORE_CHECKPOINT=sync: here, A/B)
      static const bool sync_ckpt = [] {
        const char* v = getenv("SDCORE_CHECKPOINT");
        return v && strcmp(v, "sync") == 0;
      }();
      const bool file_db = !path.empty() && path != ":memory:" && path.rfind("file:", 0) != 0;
      if (sync_ckpt || !file_db) {
        exec("PRAGMA wal_checkpoint(PASSIVE)");
      } else {
        join_checkpoint();
        const std::string p = path;
        checkpointer = std::thread([p] {
          sqlite3* c = nullptr;
          if (sqlite3_open_v2(p.c_str(), &c, SQLITE_OPEN_READWRITE | SQLITE_OPEN_NOMUTEX, nullptr) == SQLITE_OK) {
            sqlite3_busy_timeout(c, 5000);
            sqlite3_exec(c, "PRAGMA wal_checkpoint(PASSIVE)", nullptr, nullptr, nullptr);
          }
          if (c) sqlite3_close(c);
        });
      }
      exec("PRAGMA wal_autocheckpoint = 1000");
      if (trace)
        fprintf(stderr, "sqlite index_restore ms: create index %.2f wal checkpoint %.2f\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    } catch (...) {
      // leave the caller's batch open as it was (its end_batch commits it)
      // and stay in bulk mode, so that a later restore (end_bulk_identify)
      // rebuilds the index
      sqlite3_exec(db, "PRAGMA threads = 0", nullptr, nullptr, nullptr);
      if (batch_depth) sqlite3_exec(db, "BEGIN IMMEDIATE", nullptr, nullptr, nullptr);
      throw;
    }
    if (batch_depth) exec("BEGIN IMMEDIATE");
    bulk = false;
    first.clear();
  }

  [[noreturn]] void fail(const std::string& what) {
    throw std::runtime_error("sqlite: " + what + ": " + (db ? sqlite3_errmsg(db) : "no database"));
  }
  void exec(const char* sql) {
    char* err = nullptr;
    if (sqlite3_exec(db, sql, nullptr, nullptr, &err) != SQLITE_OK) {
      std::string m = err ? err : "?";
      sqlite3_free(err);
      throw std::runtime_error(std::string("sqlite: ") + sql + ": " + m);
    }
  }
  void prepare(Stmt& st, const char* sql) {
    if (sqlite3_prepare_v2(db, sql, -1, &st.s, nullptr) != SQLITE_OK) fail(sql);
  }
  void done(Stmt& st) {
    if (sqlite3_step(st.s) != SQLITE_DONE) fail("step");
    sqlite3_reset(st.s);
    sqlite3_clear_bindings(st.s);
  }
  void text(Stmt& st, int i, const std::string& v) { sqlite3_bind_text(st.s, i, v.data(), (int)v.size(), SQLITE_TRANSIENT); }
  void opt_text(Stmt& st, int i, const std::optional<std::string>& v) {
    if (v) text(st, i, *v);
    else sqlite3_bind_null(st.s, i);
  }
  static std::optional<std::string> col_text(sqlite3_stmt* s, int i) {
    if (sqlite3_column_type(s, i) == SQLITE_NULL) return std::nullopt;
    return std::string((const char*)sqlite3_column_text(s, i), (size_t)sqlite3_column_bytes(s, i));
  }
  // bind (location, sub path) of the orphan / validator filters at 1, 2, 3
  void bind_scope(Stmt& st, int32_t location_id, const std::string& sub) {
    sqlite3_bind_int64(st.s, 1, location_id);
    text(st, 2, sub);
  }
  static FilePathRow row_of(sqlite3_stmt* s) {
    // id, pub_id, location_id, materialized_path, name, extension, is_dir,
    // size_in_bytes_bytes, cas_id, object_id, integrity_checksum,
    // date_created, kind_hint
    FilePathRow r;
    r.id = (int32_t)sqlite3_column_int64(s, 0);
    if (sqlite3_column_bytes(s, 1) == 16) std::memcpy(r.pub_id.data(), sqlite3_column_blob(s, 1), 16);
    r.location_id = (int32_t)sqlite3_column_int64(s, 2);
    r.materialized_path = col_text(s, 3).value_or("");
    r.name = col_text(s, 4).value_or("");
    r.extension = col_text(s, 5).value_or("");
    r.is_dir = sqlite3_column_int64(s, 6) != 0;
    r.size_in_bytes = from_be64(sqlite3_column_blob(s, 7), sqlite3_column_bytes(s, 7));
    r.cas_id = col_text(s, 8);
    if (sqlite3_column_type(s, 9) != SQLITE_NULL) r.object_id = (int32_t)sqlite3_column_int64(s, 9);
    r.integrity_checksum = col_text(s, 10);
    r.date_created = sqlite3_column_int64(s, 11);
    r.kind = (int32_t)sqlite3_column_int64(s, 12);
    r.inode = from_be64(sqlite3_column_blob(s, 13), sqlite3_column_bytes(s, 13));
    r.hidden = sqlite3_column_int64(s, 14) != 0;
    return r;
  }
  std::vector<FilePathRow> rows(Stmt& st) {
    std::vector<FilePathRow> out;
    int rc;
    while ((rc = sqlite3_step(st.s)) == SQLITE_ROW) out.push_back(row_of(st.s));
    if (rc != SQLITE_DONE) fail("query");
    sqlite3_reset(st.s);
    sqlite3_clear_bindings(st.s);
    return out;
  }
};

#define SD_COLS \
  "id, pub_id, location_id, materialized_path, name, extension, is_dir, size_in_bytes_bytes, cas_id, object_id, " \
  "integrity_checksum, date_created, kind_hint, inode, hidden"
// orphan_path_filters (file_identifier_job.rs:251-283)
#define SD_ORPHAN                                                                                       \
  "(object_id IS NULL OR cas_id IS NULL) AND is_dir = 0 AND location_id = ?1 AND "                      \
  "size_in_bytes_bytes != x'0000000000000000' AND substr(materialized_path, 1, length(?2)) = ?2"

#define SD_ORPHAN_DIR                                                                                   \
  "(object_id IS NULL OR cas_id IS NULL) AND is_dir = 0 AND location_id = ?1 AND "                      \
  "size_in_bytes_bytes != x'0000000000000000' AND materialized_path = ?2"

SqliteLibrary::SqliteLibrary(std::unique_ptr<Impl> d) : d_(std::move(d)) {}

SqliteLibrary::~SqliteLibrary() {
  if (!d_) return;
  sqlite3* db = d_->db;
  sqlite3* rdb = d_->rdb;
  Impl* p = d_.release();
  delete p;  // statements finalize before the databases close
  if (rdb) sqlite3_close(rdb);
  if (db) sqlite3_close(db);
}

std::unique_ptr<SqliteLibrary> SqliteLibrary::open(const std::string& path, bool cas_id_index, bool object_id_index) {
  auto d = std::make_unique<Impl>();
  if (sqlite3_open_v2(path.c_str(), &d->db, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE | SQLITE_OPEN_NOMUTEX,
                      nullptr) != SQLITE_OK) {
    std::string m = d->db ? sqlite3_errmsg(d->db) : "open failed";
    if (d->db) sqlite3_close(d->db);
    throw std::runtime_error("sqlite: " + path + ": " + m);
  }
  d->exec("PRAGMA journal_mode = WAL");
  d->exec("PRAGMA synchronous = NORMAL");
  // the step's random probes and index updates stay in memory: a 256 MiB
  // page cache (SQLite's default is 2 MiB) and reads through mmap
  d->exec("PRAGMA cache_size = -262144");
  d->exec("PRAGMA mmap_size = 4294967296");
  d->exec(
      "CREATE TABLE IF NOT EXISTS object ("
      " id INTEGER PRIMARY KEY AUTOINCREMENT, pub_id BLOB NOT NULL UNIQUE, kind INTEGER, key_id INTEGER,"
      " hidden BOOLEAN, favorite BOOLEAN, important BOOLEAN, note TEXT, date_created INTEGER, date_accessed INTEGER)");
  d->exec(
      "CREATE TABLE IF NOT EXISTS file_path ("
      " id INTEGER PRIMARY KEY AUTOINCREMENT, pub_id BLOB NOT NULL UNIQUE, is_dir BOOLEAN, cas_id TEXT,"
      " integrity_checksum TEXT, location_id INTEGER, materialized_path TEXT, name TEXT COLLATE NOCASE,"
      " extension TEXT COLLATE NOCASE, hidden BOOLEAN, size_in_bytes TEXT, size_in_bytes_bytes BLOB, inode BLOB,"
      " object_id INTEGER REFERENCES object (id) ON DELETE SET NULL, key_id INTEGER, date_created INTEGER,"
      " date_modified INTEGER, date_indexed INTEGER, kind_hint INTEGER)");
  d->exec("CREATE INDEX IF NOT EXISTS file_path_location_id_idx ON file_path (location_id)");
  d->exec("CREATE INDEX IF NOT EXISTS file_path_location_id_materialized_path_idx ON file_path (location_id, "
          "materialized_path)");
  // not in the reference's schema: the existing-Object lookup by cas_id
  if (cas_id_index) d->exec("CREATE INDEX IF NOT EXISTS file_path_cas_id_idx ON file_path (cas_id)");
  if (object_id_index) d->exec("CREATE INDEX IF NOT EXISTS file_path_object_id_idx ON file_path (object_id)");
  d->exec("CREATE TEMP TABLE IF NOT EXISTS want_cas (cas_id TEXT PRIMARY KEY)");
  Impl& x = *d;
  x.path = path;
  x.prepare(x.count_orphans, "SELECT COUNT(*) FROM file_path WHERE " SD_ORPHAN);
  // a rowid range scan from the cursor (the location index would make every
  // step rescan the whole location: quadratic over a job)
  x.prepare(x.get_orphans,
            "SELECT " SD_COLS " FROM file_path NOT INDEXED WHERE " SD_ORPHAN " AND id >= ?3 ORDER BY id LIMIT ?4");
  // shallow.rs:120-142: one directory level (materialized_path = ?2)
  x.prepare(x.count_orphans_dir, "SELECT COUNT(*) FROM file_path WHERE " SD_ORPHAN_DIR);
  x.prepare(x.get_orphans_dir,
            "SELECT " SD_COLS " FROM file_path WHERE " SD_ORPHAN_DIR " AND id >= ?3 ORDER BY id LIMIT ?4");
  x.prepare(x.set_cas, "UPDATE file_path SET cas_id = ?1 WHERE id = ?2");
  x.prepare(x.want_clear, "DELETE FROM want_cas");
  x.prepare(x.want_add, "INSERT OR IGNORE INTO want_cas (cas_id) VALUES (?1)");
  // mod.rs:181-188 (objects with a file_path whose cas_id is wanted) plus the
  // cas_ids of all their file_paths, objects in DB order
  // (join order and indexes pinned: the planner otherwise walks every
  // identified file_path per step — measured 29 ms per 100-row step at 50 K
  // rows, quadratic over a job)
  if (cas_id_index && object_id_index)
    x.prepare(x.existing,
              "WITH objs AS (SELECT DISTINCT f2.object_id AS oid FROM want_cas w CROSS JOIN file_path f2"
              " INDEXED BY file_path_cas_id_idx ON f2.cas_id = w.cas_id WHERE f2.object_id IS NOT NULL)"
              " SELECT fp.object_id, fp.cas_id FROM objs CROSS JOIN file_path fp INDEXED BY file_path_object_id_idx"
              " ON fp.object_id = objs.oid WHERE fp.cas_id IS NOT NULL ORDER BY fp.object_id, fp.id");
  else if (cas_id_index)  // the Objects by index probes, their file_paths by one scan
    x.prepare(x.existing,
              "SELECT fp.object_id, fp.cas_id FROM file_path fp WHERE fp.cas_id IS NOT NULL AND fp.object_id IN"
              " (SELECT f2.object_id FROM want_cas w CROSS JOIN file_path f2 INDEXED BY file_path_cas_id_idx"
              " ON f2.cas_id = w.cas_id WHERE f2.object_id IS NOT NULL) ORDER BY fp.object_id, fp.id");
  else  // the reference's schema: the same query over an unindexed cas_id
    x.prepare(x.existing,
              "SELECT fp.object_id, fp.cas_id FROM file_path fp WHERE fp.cas_id IS NOT NULL AND fp.object_id IN"
              " (SELECT f2.object_id FROM file_path f2 WHERE f2.object_id IS NOT NULL AND f2.cas_id IN"
              " (SELECT cas_id FROM want_cas)) ORDER BY fp.object_id, fp.id");
  x.prepare(x.new_object, "INSERT INTO object (pub_id, kind, date_created) VALUES (?1, ?2, ?3)");
  {
    std::string q = "INSERT INTO object (id, pub_id, kind, date_created) VALUES ";
    for (int k = 0; k < Impl::kManyObjects; ++k) q += k ? ", (?, ?, ?, ?)" : "(?, ?, ?, ?)";
    x.prepare(x.new_objects, q.c_str());
  }
  for (int free = 0; free < 2; ++free) {
    std::string q = "UPDATE file_path SET cas_id = v.column2, object_id = v.column3 FROM (VALUES ";
    for (int k = 0; k < Impl::kManyLinks; ++k) q += k ? ", (?, ?, ?)" : "(?, ?, ?)";
    q += ") AS v WHERE file_path.id = v.column1";
    if (free) q += " AND file_path.object_id IS NULL";
    x.prepare(free ? x.links_free : x.links, q.c_str());
  }
  x.prepare(x.connect, "UPDATE file_path SET object_id = ?1 WHERE id = ?2");
  x.prepare(x.set_cas_connect, "UPDATE file_path SET cas_id = ?1, object_id = ?2 WHERE id = ?3");
  // first_objects: the smallest object id among the file_paths with the
  // cas_id (objects come back in id order from existing_objects' query)
  x.cas_index = cas_id_index;
  if (cas_id_index)
    x.prepare(x.first_object,
              "SELECT MIN(object_id) FROM file_path INDEXED BY file_path_cas_id_idx"
              " WHERE cas_id = ?1 AND object_id IS NOT NULL");
  x.prepare(x.no_checksum,
            "SELECT " SD_COLS " FROM file_path WHERE location_id = ?1 AND is_dir = 0 AND integrity_checksum IS NULL"
            " AND substr(materialized_path, 1, length(?2)) = ?2 ORDER BY id");
  x.prepare(x.set_checksum, "UPDATE file_path SET integrity_checksum = ?1 WHERE id = ?2");
  x.prepare(x.add_path,
            "INSERT INTO file_path (id, pub_id, location_id, materialized_path, name, extension, is_dir,"
            " size_in_bytes_bytes, cas_id, object_id, integrity_checksum, date_created, kind_hint, inode, hidden)"
            " VALUES (?1, ?2, ?3, ?4, ?5, ?6, ?7, ?8, ?9, ?10, ?11, ?12, ?13, ?14, ?15)");
  x.prepare(x.get_path, "SELECT " SD_COLS " FROM file_path WHERE id = ?1");
  x.prepare(x.row_state, "SELECT cas_id, object_id FROM file_path WHERE id = ?1");
  // bulk identify: the combined write of a row without an Object, which
  // leaves any other row alone (sqlite3_changes() tells which happened)
  x.prepare(x.set_cas_connect_free, "UPDATE file_path SET cas_id = ?1, object_id = ?2 WHERE id = ?3 AND object_id IS NULL");
  x.prepare(x.count_cas, "SELECT COUNT(*) FROM file_path WHERE cas_id IS NOT NULL");
  x.prepare(x.load_first,
            "SELECT cas_id, MIN(object_id) FROM file_path WHERE cas_id IS NOT NULL AND object_id IS NOT NULL"
            " GROUP BY cas_id");
  x.prepare(x.all_objects, "SELECT id, pub_id, kind, date_created FROM object ORDER BY id");
  {
    // the id AUTOINCREMENT would assign next: past the largest id the table
    // ever held (sqlite_sequence keeps it after the top Objects are deleted),
    // not only past the largest it holds now (create_objects gives ids)
    Stmt mx;
    x.prepare(mx,
              "SELECT MAX(COALESCE((SELECT MAX(id) FROM object), 0),"
              " COALESCE((SELECT seq FROM sqlite_sequence WHERE name = 'object'), 0))");
    if (sqlite3_step(mx.s) == SQLITE_ROW) x.next_object = sqlite3_column_int64(mx.s, 0) + 1;
  }
  return std::unique_ptr<SqliteLibrary>(new SqliteLibrary(std::move(d)));
}

void SqliteLibrary::begin_batch() {
  if (d_->batch_depth++ == 0) d_->exec("BEGIN IMMEDIATE");
}

void SqliteLibrary::end_batch() {
  if (d_->batch_depth > 0 && --d_->batch_depth == 0) d_->exec("COMMIT");
}

void SqliteLibrary::add_file_paths(std::vector<FilePathRow>& rows) {
  Impl& x = *d_;
  x.index_restore();  // new rows may carry cas_ids and Objects
  int64_t next = 1;
  {
    Stmt mx;
    x.prepare(mx, "SELECT COALESCE(MAX(id), 0) FROM file_path");
    if (sqlite3_step(mx.s) == SQLITE_ROW) next = sqlite3_column_int64(mx.s, 0) + 1;
  }
  begin_batch();
  for (auto& r : rows) {
    if (r.id == 0) r.id = (int32_t)next;
    next = std::max<int64_t>(next, (int64_t)r.id + 1);
    if (r.pub_id == PubId{}) r.pub_id = pub_id(0x46504154u, r.id);
    Stmt& st = x.add_path;
    uint8_t sz[8];
    be64(r.size_in_bytes, sz);
    sqlite3_bind_int64(st.s, 1, r.id);
    sqlite3_bind_blob(st.s, 2, r.pub_id.data(), 16, SQLITE_TRANSIENT);
    sqlite3_bind_int64(st.s, 3, r.location_id);
    x.text(st, 4, r.materialized_path);
    x.text(st, 5, r.name);
    x.text(st, 6, r.extension);
    sqlite3_bind_int64(st.s, 7, r.is_dir ? 1 : 0);
    sqlite3_bind_blob(st.s, 8, sz, 8, SQLITE_TRANSIENT);
    x.opt_text(st, 9, r.cas_id);
    if (r.object_id) sqlite3_bind_int64(st.s, 10, *r.object_id);
    else sqlite3_bind_null(st.s, 10);
    x.opt_text(st, 11, r.integrity_checksum);
    sqlite3_bind_int64(st.s, 12, r.date_created);
    sqlite3_bind_int64(st.s, 13, r.kind);
    uint8_t ino[8];
    be64(r.inode, ino);
    sqlite3_bind_blob(st.s, 14, ino, 8, SQLITE_TRANSIENT);
    sqlite3_bind_int64(st.s, 15, r.hidden ? 1 : 0);
    x.done(st);
  }
  end_batch();
}

std::optional<FilePathRow> SqliteLibrary::file_path(int32_t id) {
  sqlite3_bind_int64(d_->get_path.s, 1, id);
  auto r = d_->rows(d_->get_path);
  if (r.empty()) return std::nullopt;
  return r[0];
}

std::vector<ObjectRow> SqliteLibrary::objects() {
  std::vector<ObjectRow> out;
  sqlite3_stmt* s = d_->all_objects.s;
  while (sqlite3_step(s) == SQLITE_ROW) {
    ObjectRow o;
    o.id = (int32_t)sqlite3_column_int64(s, 0);
    if (sqlite3_column_bytes(s, 1) == 16) std::memcpy(o.pub_id.data(), sqlite3_column_blob(s, 1), 16);
    o.kind = (int32_t)sqlite3_column_int64(s, 2);
    o.date_created = sqlite3_column_int64(s, 3);
    out.push_back(o);
  }
  sqlite3_reset(s);
  return out;
}

size_t SqliteLibrary::count_orphan_file_paths(int32_t location_id, const std::string& sub) {
  Impl& x = *d_;
  x.bind_scope(x.count_orphans, location_id, sub);
  if (sqlite3_step(x.count_orphans.s) != SQLITE_ROW) x.fail("count orphans");
  const size_t n = (size_t)sqlite3_column_int64(x.count_orphans.s, 0);
  sqlite3_reset(x.count_orphans.s);
  sqlite3_clear_bindings(x.count_orphans.s);
  return n;
}

size_t SqliteLibrary::count_orphan_file_paths_in_dir(int32_t location_id, const std::string& dir) {
  Impl& x = *d_;
  x.bind_scope(x.count_orphans_dir, location_id, dir);
  if (sqlite3_step(x.count_orphans_dir.s) != SQLITE_ROW) x.fail("count orphans in dir");
  const size_t n = (size_t)sqlite3_column_int64(x.count_orphans_dir.s, 0);
  sqlite3_reset(x.count_orphans_dir.s);
  sqlite3_clear_bindings(x.count_orphans_dir.s);
  return n;
}

std::vector<FilePathRow> SqliteLibrary::get_orphan_file_paths_in_dir(int32_t location_id, int32_t cursor,
                                                                     const std::string& dir, size_t take) {
  Impl& x = *d_;
  x.bind_scope(x.get_orphans_dir, location_id, dir);
  sqlite3_bind_int64(x.get_orphans_dir.s, 3, cursor);
  sqlite3_bind_int64(x.get_orphans_dir.s, 4, (int64_t)take);
  return x.rows(x.get_orphans_dir);
}

std::vector<FilePathRow> SqliteLibrary::get_orphan_file_paths(int32_t location_id, int32_t cursor,
                                                              const std::string& sub, size_t take) {
  Impl& x = *d_;
  x.bind_scope(x.get_orphans, location_id, sub);
  sqlite3_bind_int64(x.get_orphans.s, 3, cursor);
  sqlite3_bind_int64(x.get_orphans.s, 4, (int64_t)take);
  return x.rows(x.get_orphans);
}

void SqliteLibrary::set_cas_id(int32_t id, const std::optional<std::string>& cas_id) {
  Impl& x = *d_;
  std::optional<int32_t> oid;
  if (x.bulk) {
    auto [old_cas, old_oid] = x.state(id);
    // a row with an Object leaving a cas_id: its MIN may move, only the index knows
    if (old_oid && old_cas && old_cas != cas_id) x.index_restore();
    oid = old_oid;
  }
  x.opt_text(x.set_cas, 1, cas_id);
  sqlite3_bind_int64(x.set_cas.s, 2, id);
  x.done(x.set_cas);
  if (x.bulk && oid && cas_id) x.first_min(*cas_id, *oid);
}

std::vector<std::pair<int32_t, std::vector<std::string>>> SqliteLibrary::existing_objects(
    const std::vector<std::string>& cas_ids) {
  Impl& x = *d_;
  x.index_restore();  // the join reads the cas_id index
  begin_batch();
  x.done(x.want_clear);
  for (const auto& c : cas_ids) {
    x.text(x.want_add, 1, c);
    x.done(x.want_add);
  }
  std::vector<std::pair<int32_t, std::vector<std::string>>> out;
  int rc;
  while ((rc = sqlite3_step(x.existing.s)) == SQLITE_ROW) {
    const int32_t oid = (int32_t)sqlite3_column_int64(x.existing.s, 0);
    if (out.empty() || out.back().first != oid) out.push_back({oid, {}});
    out.back().second.push_back(*Impl::col_text(x.existing.s, 1));
  }
  if (rc != SQLITE_DONE) x.fail("existing objects");
  sqlite3_reset(x.existing.s);
  end_batch();
  return out;
}

int32_t SqliteLibrary::create_object(ObjectKind kind, int64_t date_created) {
  Impl& x = *d_;
  const PubId p = pub_id(0x4F424A54u, x.next_object);
  sqlite3_bind_blob(x.new_object.s, 1, p.data(), 16, SQLITE_TRANSIENT);
  sqlite3_bind_int64(x.new_object.s, 2, kind);
  sqlite3_bind_int64(x.new_object.s, 3, date_created);
  x.done(x.new_object);
  const int64_t id = sqlite3_last_insert_rowid(x.db);
  x.next_object = id + 1;
  return (int32_t)id;
}

std::vector<int32_t> SqliteLibrary::create_objects(const std::vector<std::pair<ObjectKind, int64_t>>& kinds_dates) {
  Impl& x = *d_;
  std::vector<int32_t> ids;
  ids.reserve(kinds_dates.size());
  size_t k = 0;
  // whole groups of kManyObjects in one statement each, ids given explicitly
  // (the ids the table would assign: one past its largest), the rest one by one
  begin_batch();
  for (; k + Impl::kManyObjects <= kinds_dates.size(); k += Impl::kManyObjects) {
    sqlite3_stmt* st = x.new_objects.s;
    for (int r = 0; r < Impl::kManyObjects; ++r) {
      const int64_t id = x.next_object + r;
      const PubId p = pub_id(0x4F424A54u, id);
      sqlite3_bind_int64(st, 4 * r + 1, id);
      sqlite3_bind_blob(st, 4 * r + 2, p.data(), 16, SQLITE_TRANSIENT);
      sqlite3_bind_int64(st, 4 * r + 3, kinds_dates[k + r].first);
      sqlite3_bind_int64(st, 4 * r + 4, kinds_dates[k + r].second);
      ids.push_back((int32_t)id);
    }
    x.done(x.new_objects);
    x.next_object += Impl::kManyObjects;
  }
  for (; k < kinds_dates.size(); ++k) ids.push_back(create_object(kinds_dates[k].first, kinds_dates[k].second));
  end_batch();
  return ids;
}

std::vector<std::pair<std::string, int32_t>> SqliteLibrary::first_objects(const std::vector<std::string>& cas_ids) {
  Impl& x = *d_;
  if (!x.cas_index) return Library::first_objects(cas_ids);
  std::vector<std::pair<std::string, int32_t>> out;
  if (x.bulk) {
    for (const auto& c : cas_ids) {
      auto it = x.first.find(c);
      if (it != x.first.end()) out.emplace_back(c, it->second);
    }
    return out;
  }
  begin_batch();
  for (const auto& c : cas_ids) {
    x.text(x.first_object, 1, c);
    if (sqlite3_step(x.first_object.s) != SQLITE_ROW) x.fail("first object");
    if (sqlite3_column_type(x.first_object.s, 0) != SQLITE_NULL)
      out.emplace_back(c, (int32_t)sqlite3_column_int64(x.first_object.s, 0));
    sqlite3_reset(x.first_object.s);
  }
  sqlite3_clear_bindings(x.first_object.s);
  end_batch();
  return out;
}

void SqliteLibrary::set_cas_id_and_connect(int32_t file_path_id, const std::optional<std::string>& cas_id,
                                           int32_t object_id) {
  Impl& x = *d_;
  if (x.bulk) {
    // the step's rows have no Object: one write, no read
    x.opt_text(x.set_cas_connect_free, 1, cas_id);
    sqlite3_bind_int64(x.set_cas_connect_free.s, 2, object_id);
    sqlite3_bind_int64(x.set_cas_connect_free.s, 3, file_path_id);
    x.done(x.set_cas_connect_free);
    if (sqlite3_changes(x.db) == 1) {
      if (cas_id) x.first_min(*cas_id, object_id);
      return;
    }
    set_cas_id(file_path_id, cas_id);  // a row with an Object (or none at all): the general path
    connect(file_path_id, object_id);
    return;
  }
  x.opt_text(x.set_cas_connect, 1, cas_id);
  sqlite3_bind_int64(x.set_cas_connect.s, 2, object_id);
  sqlite3_bind_int64(x.set_cas_connect.s, 3, file_path_id);
  x.done(x.set_cas_connect);
}

void SqliteLibrary::set_cas_ids_and_connect(const std::vector<CasLink>& rows) {
  Impl& x = *d_;
  size_t k = 0;
  begin_batch();
  for (; k + Impl::kManyLinks <= rows.size(); k += Impl::kManyLinks) {
    Stmt& st = x.bulk ? x.links_free : x.links;
    for (int r = 0; r < Impl::kManyLinks; ++r) {
      const CasLink& w = rows[k + r];
      sqlite3_bind_int64(st.s, 3 * r + 1, w.file_path_id);
      x.opt_text(st, 3 * r + 2, w.cas_id);
      sqlite3_bind_int64(st.s, 3 * r + 3, w.object_id);
    }
    x.done(st);
    if (!x.bulk) continue;
    const bool all = sqlite3_changes(x.db) == Impl::kManyLinks;
    for (int r = 0; r < Impl::kManyLinks; ++r) {
      const CasLink& w = rows[k + r];
      if (!all) {
        // a row that had an Object kept it (or is gone): the general path,
        // as set_cas_id_and_connect takes for it
        auto [cas, oid] = x.state(w.file_path_id);
        if (!(oid && *oid == w.object_id && cas == w.cas_id)) {
          set_cas_id(w.file_path_id, w.cas_id);
          connect(w.file_path_id, w.object_id);
          continue;
        }
      }
      if (w.cas_id) x.first_min(*w.cas_id, w.object_id);
    }
  }
  for (; k < rows.size(); ++k) set_cas_id_and_connect(rows[k].file_path_id, rows[k].cas_id, rows[k].object_id);
  end_batch();
}

void SqliteLibrary::connect(int32_t file_path_id, int32_t object_id) {
  Impl& x = *d_;
  std::optional<std::string> cas;
  if (x.bulk) {
    auto [old_cas, old_oid] = x.state(file_path_id);
    if (old_cas && old_oid && *old_oid != object_id) x.index_restore();  // its cas_id's MIN may move
    cas = old_cas;
  }
  sqlite3_bind_int64(x.connect.s, 1, object_id);
  sqlite3_bind_int64(x.connect.s, 2, file_path_id);
  x.done(x.connect);
  if (x.bulk && cas) x.first_min(*cas, object_id);
}

bool SqliteLibrary::begin_bulk_identify(size_t orphans) {
  Impl& x = *d_;
  if (!x.cas_index || x.bulk || x.batch_depth) return false;
  x.join_checkpoint();  // the previous bulk job's deferred checkpoint
  if (sqlite3_step(x.count_cas.s) != SQLITE_ROW) x.fail("count cas_ids");
  const uint64_t with_cas = (uint64_t)sqlite3_column_int64(x.count_cas.s, 0);
  sqlite3_reset(x.count_cas.s);
  if (with_cas > 4 * (uint64_t)orphans) return false;
  x.first.clear();
  x.first.reserve((size_t)with_cas + orphans);
  int rc;
  while ((rc = sqlite3_step(x.load_first.s)) == SQLITE_ROW)
    x.first.emplace(*Impl::col_text(x.load_first.s, 0), (int32_t)sqlite3_column_int64(x.load_first.s, 1));
  if (rc != SQLITE_DONE) x.fail("load cas_ids");
  sqlite3_reset(x.load_first.s);
  x.exec("DROP INDEX IF EXISTS file_path_cas_id_idx");
  // no WAL checkpoint after every ~1000 pages of the job's commits: one at
  // the end (index_restore) writes each page back once
  x.exec("PRAGMA wal_autocheckpoint = 0");
  x.bulk = true;
  return true;
}

void SqliteLibrary::end_bulk_identify() { d_->index_restore(); }

bool SqliteLibrary::bulk_identify_active() const { return d_->bulk; }

bool SqliteLibrary::concurrent_orphan_reads() {
  Impl& x = *d_;
  if (x.rdb) return true;
  if (x.reader_tried || x.path.empty() || x.path == ":memory:" || x.path.rfind("file:", 0) == 0) return false;
  x.reader_tried = true;
  if (sqlite3_open_v2(x.path.c_str(), &x.rdb, SQLITE_OPEN_READONLY | SQLITE_OPEN_NOMUTEX, nullptr) != SQLITE_OK) {
    if (x.rdb) sqlite3_close(x.rdb);
    x.rdb = nullptr;
    return false;
  }
  // a WAL recovery or checkpoint of the writer can hold the read a moment:
  // wait for it rather than fail the job
  sqlite3_busy_timeout(x.rdb, 5000);
  char* err = nullptr;
  if (sqlite3_exec(x.rdb, "PRAGMA mmap_size = 4294967296", nullptr, nullptr, &err) != SQLITE_OK ||
      sqlite3_prepare_v2(x.rdb,
                         "SELECT " SD_COLS " FROM file_path NOT INDEXED WHERE " SD_ORPHAN
                         " AND id >= ?3 ORDER BY id LIMIT ?4",
                         -1, &x.r_get_orphans.s, nullptr) != SQLITE_OK) {
    sqlite3_free(err);
    if (x.r_get_orphans.s) sqlite3_finalize(x.r_get_orphans.s);
    x.r_get_orphans.s = nullptr;
    sqlite3_close(x.rdb);
    x.rdb = nullptr;
    return false;
  }
  return true;
}

std::vector<FilePathRow> SqliteLibrary::get_orphan_file_paths_concurrent(int32_t location_id, int32_t cursor,
                                                                         const std::string& sub, size_t take) {
  Impl& x = *d_;
  // the writer's connection is opened NOMUTEX: reading through it from
  // another thread would race with the writes
  if (!x.rdb)
    throw std::logic_error("sqlite: get_orphan_file_paths_concurrent without the read-ahead connection "
                           "(concurrent_orphan_reads() returned false or was not called)");
  std::lock_guard<std::mutex> g(x.rmu);
  Stmt& st = x.r_get_orphans;
  sqlite3_bind_int64(st.s, 1, location_id);
  sqlite3_bind_text(st.s, 2, sub.data(), (int)sub.size(), SQLITE_TRANSIENT);
  sqlite3_bind_int64(st.s, 3, cursor);
  sqlite3_bind_int64(st.s, 4, (int64_t)take);
  std::vector<FilePathRow> out;
  int rc;
  while ((rc = sqlite3_step(st.s)) == SQLITE_ROW) out.push_back(Impl::row_of(st.s));
  sqlite3_reset(st.s);
  sqlite3_clear_bindings(st.s);
  if (rc != SQLITE_DONE)
    throw std::runtime_error(std::string("sqlite: read-ahead: ") + sqlite3_errmsg(x.rdb));
  return out;
}

std::vector<FilePathRow> SqliteLibrary::file_paths_without_checksum(int32_t location_id, const std::string& sub) {
  Impl& x = *d_;
  x.bind_scope(x.no_checksum, location_id, sub);
  return x.rows(x.no_checksum);
}

void SqliteLibrary::set_integrity_checksum(int32_t id, const std::string& checksum) {
  Impl& x = *d_;
  x.text(x.set_checksum, 1, checksum);
  sqlite3_bind_int64(x.set_checksum.s, 2, id);
  x.done(x.set_checksum);
}

}  // namespace sdcore
