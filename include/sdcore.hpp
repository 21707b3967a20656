// sdcore.hpp — C++ host mirror of sd-core's content-identification path,
// layered on the C ABI of libsdcas.so (include/sdcas.h).
//
// The reference host is Rust (sd-core); there is no Rust toolchain in this
// image, so the host side above the C ABI is written in C++ with the
// reference's names, argument meaning and error behaviour:
//
//   generate_cas_id / generate_cas_ids   core/src/object/cas.rs:23-62
//   file_checksum / file_checksums       core/src/object/validation/hash.rs:9-25
//   FileMetadata::new (batched)          core/src/object/file_identifier/mod.rs:48-96
//   identifier_job_step                  core/src/object/file_identifier/mod.rs:98-350
//   run_file_identifier_job              core/src/object/file_identifier/file_identifier_job.rs:33-319
//   run_object_validator_job             core/src/object/validation/validator_job.rs:38-200
//
// The database side (prisma in sd-core) is the abstract `Library`; a
// `MemoryLibrary` implements it over in-memory tables with the reference's
// query semantics (filters, DB order, cursor) for tests and examples.
//
// Hashing runs on the GPU through libsdcas. There is no CPU fallback in this
// layer: when the engine cannot open (no device) `Engine::open` throws
// `LibraryError`, which is the point where the Rust host keeps its own CPU
// path (include/sdcas.h, "Conventions").
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sdcas.h"

namespace sdcore {

// std::io::Error as the Rust host sees it (crates/utils/src/error.rs:5-22
// FileIOError = path + io::Error): an errno, or UnexpectedEof from read_exact
// (cas.rs:36,43,56), which has no errno.
struct IoError {
  int code = 0;
  std::string path;
  bool unexpected_eof() const { return code == SDCAS_STATUS_UNEXPECTED_EOF; }
  std::string message() const;
};

// io::Result<T>
template <class T>
class Result {
 public:
  Result(T v) : v_(std::move(v)) {}
  Result(IoError e) : e_(std::move(e)) {}
  bool ok() const { return v_.has_value(); }
  const T& value() const {
    if (!v_) throw std::logic_error("Result::value on an error: " + e_.message());
    return *v_;
  }
  const IoError& error() const { return e_; }

 private:
  std::optional<T> v_;
  IoError e_;
};

// A library failure (negative SDCAS_E_* return): the whole batch must take the
// host's CPU path.
class LibraryError : public std::runtime_error {
 public:
  LibraryError(int code, const std::string& what) : std::runtime_error(what), code(code) {}
  int code;
};

class Engine {
 public:
  struct Options {
    int device = -1;             // HIP device ordinal, -1: current
    uint32_t io_threads = 0;     // reader threads (0: library default)
    uint64_t staging_bytes = 0;  // pinned staging per slot (0: library default)
    uint32_t flags = 0;          // SDCAS_OPT_* (SDCAS_OPT_DIRECT_IO: big-file checksums bypass the page cache)
    // progress / cancellation of the batch calls (sdcas.h "Conventions"): the
    // job's progress hook (job/worker.rs:458-480) and its cancel command
    // (job/mod.rs:862-960)
    sdcas_progress_fn progress = nullptr;
    void* progress_user = nullptr;
    const volatile int32_t* cancel = nullptr;
  };
  static std::unique_ptr<Engine> open(const Options& opts);
  static std::unique_ptr<Engine> open() { return open(Options{}); }
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // cas.rs:23-62 over a batch: (path, size from fs::metadata) -> 16 lowercase hex
  std::vector<Result<std::string>> generate_cas_ids(const std::vector<std::pair<std::string, uint64_t>>& files);
  // hash.rs:11-25 over a batch: path -> 64 lowercase hex
  std::vector<Result<std::string>> file_checksums(const std::vector<std::string>& paths);
  // fs::metadata + generate_cas_id of FileMetadata::new (mod.rs:48-96) in one
  // call (sdcas_file_metadata: the length from fstat of the descriptor the
  // reads use)
  struct RawMetadata {
    std::vector<uint64_t> size, key;
    std::vector<int32_t> status;
    std::vector<uint8_t> flags;  // SDCAS_META_*
  };
  RawMetadata file_metadata(const std::vector<const char*>& paths, const uint64_t* size_hints = nullptr);

  // the canonical group-by of mod.rs:149-254 over the job's steps
  // (sdcas_dedup_window; sdcas_dedup encoding of out_link). window may be
  // null: the whole job over these rows.
  struct Dedup {
    std::vector<int64_t> link;
    int64_t created = 0, linked = 0;
  };
  Dedup dedup(const std::vector<uint64_t>& keys, const std::vector<uint8_t>& has_key,
              const std::vector<int32_t>& status, size_t chunk_size, const std::vector<uint64_t>& existing_keys,
              sdcas_job_window* window = nullptr);

  sdcas_ctx* raw() { return ctx_; }

 private:
  explicit Engine(sdcas_ctx* c, int device) : ctx_(c), device_(device) {}
  [[noreturn]] void fail(int rc, const char* what) const;
  [[noreturn]] void fail_on(sdcas_ctx* c, int rc, const char* what) const;
  sdcas_ctx* dedup_ctx();
  sdcas_ctx* ctx_;
  // the group-by's own context (created with the first dedup): a job's
  // read-ahead holds ctx_ through its path calls, which the group-by of the
  // batch being written would otherwise wait for (SDCORE_DEDUP_CTX=same: ctx_)
  int device_ = -1;
  sdcas_ctx* dedup_ctx_ = nullptr;
  std::mutex dedup_mu_;
};

// single-file forms with the reference signatures (cas.rs:23, hash.rs:11)
Result<std::string> generate_cas_id(Engine& engine, const std::string& path, uint64_t size);
Result<std::string> file_checksum(Engine& engine, const std::string& path);

// cas key <-> the 16-hex cas_id string (cas.rs:61: to_hex()[..16])
std::string key_to_hex(uint64_t key);
uint64_t hex_to_key(const std::string& cas_id);

// ---- rows (the prisma columns this path reads or writes) -------------------

using ObjectKind = int32_t;  // sd_file_ext::kind::ObjectKind discriminant; 0 = Unknown
// the discriminants of crates/file-ext/src/kind.rs:4-59
enum : ObjectKind {
  ObjectKindUnknown = 0, ObjectKindDocument = 1, ObjectKindFolder = 2, ObjectKindText = 3, ObjectKindPackage = 4,
  ObjectKindImage = 5, ObjectKindAudio = 6, ObjectKindVideo = 7, ObjectKindArchive = 8, ObjectKindExecutable = 9,
  ObjectKindAlias = 10, ObjectKindEncrypted = 11, ObjectKindKey = 12, ObjectKindLink = 13,
  ObjectKindWebPageArchive = 14, ObjectKindWidget = 15, ObjectKindAlbum = 16, ObjectKindCollection = 17,
  ObjectKindFont = 18, ObjectKindMesh = 19, ObjectKindCode = 20, ObjectKindDatabase = 21, ObjectKindBook = 22,
  ObjectKindConfig = 23, ObjectKindDotfile = 24, ObjectKindScreenshot = 25,
};
// FilePathRow::kind / file_metadata_batch: derive the kind from the path
constexpr ObjectKind kKindFromPath = -1;

// ---- kind detection (crates/file-ext, file_ext.cpp) ---------------------------

// Extension::from_str (magic.rs:63-79): the ObjectKinds of the categories
// accepting `ext` (case-insensitive), in the Extension enum's order; empty =
// None, one = Known, two = Conflicts ("ts", "mts": Video and Code)
std::vector<ObjectKind> extension_kinds(const std::string& ext);
// Extension::resolve_conflicting(path, false) (magic.rs:176-235) as an
// ObjectKind: nullopt when the path has no (UTF-8) extension, the extension
// is unknown, the file does not open, or a conflict is not "ts"/"mts" as
// written; "ts"/"mts" are Video when the file has the MPEG-TS magic bytes,
// else Code
std::optional<ObjectKind> resolve_conflicting_kind(const std::string& path);
// FileMetadata::new's kind (mod.rs:72-76): the above, or Unknown
ObjectKind object_kind_of(const std::string& path);
using PubId = std::array<uint8_t, 16>;

struct Location {  // location::Data (id, path)
  int32_t id = 0;
  std::string path;
};

// file_path, with the columns of file_path_for_file_identifier and
// file_path_for_object_validator (crates/file-path-helper/src/lib.rs:30-47)
struct FilePathRow {
  int32_t id = 0;
  PubId pub_id{};
  int32_t location_id = 0;
  std::string materialized_path = "/";  // "/" or "/a/b/" (isolated_file_path_data.rs)
  std::string name, extension;
  bool is_dir = false;
  uint64_t size_in_bytes = 0;
  std::optional<std::string> cas_id;
  std::optional<int32_t> object_id;
  std::optional<std::string> integrity_checksum;
  int64_t date_created = 0;
  uint64_t inode = 0;   // FilePathMetadata (crates/file-path-helper/src/lib.rs:125-131)
  bool hidden = false;
  // kKindFromPath: FileMetadata::new derives it (object_kind_of, mod.rs:72-76);
  // >= 0: a kind already known to the caller, used as is
  ObjectKind kind = kKindFromPath;
};

struct ObjectRow {  // object (id, pub_id, kind, date_created)
  int32_t id = 0;
  PubId pub_id{};
  ObjectKind kind = 0;
  int64_t date_created = 0;
};

// location path joined with the row's relative path (assemble_relative_path /
// join_location_relative_path, isolated_file_path_data.rs:533-560)
std::string full_path(const Location& location, const FilePathRow& row);

// The indexer's walk (core/src/location/indexer/walk.rs:432-560) without
// indexer rules: every directory and regular file under the location,
// breadth first, entries of a directory in name order; symlinks skipped
// (walk.rs: `metadata.is_symlink()`); IsolatedFilePathData::new naming
// (isolated_file_path_data.rs:49-87): materialized_path "/a/b/", a file's
// name is Rust's Path::file_stem and its extension Path::extension, a
// directory keeps its whole file name; hidden = name starts with '.'
// (lib.rs:133-147). Rows come back with id 0 (the library assigns ids);
// entries that cannot be read are skipped and reported in `errors`.
std::vector<FilePathRow> walk_location(const Location& location, std::vector<IoError>* errors = nullptr);

// Rust's Path::file_stem / Path::extension of a file name
std::pair<std::string, std::optional<std::string>> file_stem_and_extension(const std::string& file_name);

// ---- the database seam ------------------------------------------------------

class Library {
 public:
  virtual ~Library() = default;
  // orphan_path_filters (file_identifier_job.rs:251-283): (object_id IS NULL OR
  // cas_id IS NULL) AND is_dir = false AND location_id = ? AND size != 0
  // [AND materialized_path LIKE sub%] [AND id >= cursor], ORDER BY id
  virtual size_t count_orphan_file_paths(int32_t location_id, const std::string& sub_materialized_path) = 0;
  virtual std::vector<FilePathRow> get_orphan_file_paths(int32_t location_id, int32_t cursor,
                                                         const std::string& sub_materialized_path, size_t take) = 0;
  // the shallow identifier's orphan_path_filters (shallow.rs:120-142): the
  // same with materialized_path = dir (one directory level, "/" = the
  // location's root) instead of the sub-path prefix
  virtual size_t count_orphan_file_paths_in_dir(int32_t location_id, const std::string& dir) = 0;
  virtual std::vector<FilePathRow> get_orphan_file_paths_in_dir(int32_t location_id, int32_t cursor,
                                                                const std::string& dir, size_t take) = 0;
  // mod.rs:157-178: file_path.cas_id = ? per processed file
  virtual void set_cas_id(int32_t file_path_id, const std::optional<std::string>& cas_id) = 0;
  // mod.rs:181-188: Objects having a file_path whose cas_id is in `cas_ids`,
  // in DB order, each with the cas_ids of its file_paths
  virtual std::vector<std::pair<int32_t, std::vector<std::string>>> existing_objects(
      const std::vector<std::string>& cas_ids) = 0;
  // what the identifier step takes from that lookup (mod.rs:181-188 with the
  // find of :214-224): per cas_id, the first Object in DB order having a
  // file_path with it, in no particular order; cas_ids without one are left
  // out. The default derives it from existing_objects; a database can answer
  // it with one index probe per cas_id.
  virtual std::vector<std::pair<std::string, int32_t>> first_objects(const std::vector<std::string>& cas_ids);
  // set_cas_id then connect of one row as one write: the row's state after
  // mod.rs:157-178 and :352-377. The step uses it for rows without an Object,
  // whose cas_id no lookup of the step can see before the link.
  virtual void set_cas_id_and_connect(int32_t file_path_id, const std::optional<std::string>& cas_id,
                                      int32_t object_id) {
    set_cas_id(file_path_id, cas_id);
    connect(file_path_id, object_id);
  }
  // set_cas_id_and_connect of many rows, one write per row, each row at most
  // once (the default writes them one by one)
  struct CasLink {
    int32_t file_path_id;
    std::optional<std::string> cas_id;
    int32_t object_id;
  };
  virtual void set_cas_ids_and_connect(const std::vector<CasLink>& rows) {
    for (const auto& r : rows) set_cas_id_and_connect(r.file_path_id, r.cas_id, r.object_id);
  }
  // mod.rs:290-327: object::create_unchecked(kind, date_created) -> object id
  virtual int32_t create_object(ObjectKind kind, int64_t date_created) = 0;
  // object::create_many (mod.rs:314-327): Objects created in this order, ids
  // returned in the same order (the default creates them one by one)
  virtual std::vector<int32_t> create_objects(const std::vector<std::pair<ObjectKind, int64_t>>& kinds_dates) {
    std::vector<int32_t> ids;
    ids.reserve(kinds_dates.size());
    for (const auto& [k, d] : kinds_dates) ids.push_back(create_object(k, d));
    return ids;
  }
  // connect_file_path_to_object (mod.rs:352-377)
  virtual void connect(int32_t file_path_id, int32_t object_id) = 0;
  // validator_job.rs:107-123: location_id = ? AND is_dir = false AND
  // integrity_checksum IS NULL [AND materialized_path LIKE sub%]
  virtual std::vector<FilePathRow> file_paths_without_checksum(int32_t location_id,
                                                               const std::string& sub_materialized_path) = 0;
  virtual void set_integrity_checksum(int32_t file_path_id, const std::string& checksum) = 0;
  // the writes between these calls are one batch (sync.write_ops batches a
  // step's operations, core/crates/sync/src/manager.rs:70-93): one
  // transaction in a database; no-ops in memory
  virtual void begin_batch() {}
  virtual void end_batch() {}
  // A job about to identify `orphans` rows may let the database keep what
  // first_objects answers on the host for the job's duration instead of in
  // an index it would update row by row (SqliteLibrary: the cas_id index is
  // dropped, its content kept as a cas_id -> first Object map that every
  // write of the job updates, and the index rebuilt in one pass by
  // end_bulk_identify). Returns whether it did. Every query answers as
  // before; the job must be the library's only writer meanwhile.
  virtual bool begin_bulk_identify(size_t orphans) {
    (void)orphans;
    return false;
  }
  virtual void end_bulk_identify() {}
  // The job reads its next batch (orphans past the current batch's last row,
  // which the current batch never writes) while the current batch's writes
  // are still open. A database that can serve that read from another
  // connection without waiting for them (SQLite in WAL mode: a second,
  // read-only connection) says so here; the job then fetches on its
  // metadata thread, concurrently with the writes. The concurrent call
  // answers what get_orphan_file_paths would after the current batch commits.
  virtual bool concurrent_orphan_reads() { return false; }
  virtual std::vector<FilePathRow> get_orphan_file_paths_concurrent(int32_t location_id, int32_t cursor,
                                                                    const std::string& sub_materialized_path,
                                                                    size_t take) {
    return get_orphan_file_paths(location_id, cursor, sub_materialized_path, take);
  }
};

// In-memory tables with the reference's query semantics (ids ascending = DB order)
class MemoryLibrary : public Library {
 public:
  std::vector<FilePathRow> file_paths;  // kept sorted by id
  std::vector<ObjectRow> objects;       // ids ascending

  FilePathRow& add_file_path(FilePathRow row);  // assigns id and pub_id when 0
  const FilePathRow* file_path(int32_t id) const;

  size_t count_orphan_file_paths(int32_t location_id, const std::string& sub) override;
  std::vector<FilePathRow> get_orphan_file_paths(int32_t location_id, int32_t cursor, const std::string& sub,
                                                 size_t take) override;
  size_t count_orphan_file_paths_in_dir(int32_t location_id, const std::string& dir) override;
  std::vector<FilePathRow> get_orphan_file_paths_in_dir(int32_t location_id, int32_t cursor, const std::string& dir,
                                                        size_t take) override;
  void set_cas_id(int32_t file_path_id, const std::optional<std::string>& cas_id) override;
  std::vector<std::pair<int32_t, std::vector<std::string>>> existing_objects(
      const std::vector<std::string>& cas_ids) override;
  int32_t create_object(ObjectKind kind, int64_t date_created) override;
  void connect(int32_t file_path_id, int32_t object_id) override;
  std::vector<FilePathRow> file_paths_without_checksum(int32_t location_id, const std::string& sub) override;
  void set_integrity_checksum(int32_t file_path_id, const std::string& checksum) override;

 private:
  FilePathRow* find(int32_t id);
  bool orphan(const FilePathRow& r, int32_t location_id, const std::string& sub) const;
  int32_t next_file_path_id_ = 1, next_object_id_ = 1;
};

// SQLite tables with the columns of the reference's file_path / object
// models (core/prisma/schema.prisma) and the reference's queries as prepared
// statements (the DB side of the join). Differences, both
// deliberate: an index on file_path(cas_id), which the reference's schema
// lacks (the existing-Object lookup of mod.rs:181-188 then scans the table),
// and a `kind_hint` column carrying FilePathRow::kind (kKindFromPath unless a
// caller supplies a kind).
// Batches are transactions (begin_batch / end_batch).
class SqliteLibrary : public Library {
 public:
  // path of the database file, or ":memory:"; throws std::runtime_error.
  // cas_id_index = false keeps the reference's schema (no index on cas_id),
  // for comparison. object_id_index: an index on file_path(object_id), which
  // the reference's schema lacks too and the identifier step does not read
  // (only existing_objects' join does); off by default, since every link
  // would update it.
  static std::unique_ptr<SqliteLibrary> open(const std::string& path, bool cas_id_index = true,
                                             bool object_id_index = false);
  ~SqliteLibrary() override;

  // insert rows (ids and pub_ids assigned when 0), one transaction
  void add_file_paths(std::vector<FilePathRow>& rows);
  std::optional<FilePathRow> file_path(int32_t id);
  std::vector<ObjectRow> objects();

  size_t count_orphan_file_paths(int32_t location_id, const std::string& sub) override;
  std::vector<FilePathRow> get_orphan_file_paths(int32_t location_id, int32_t cursor, const std::string& sub,
                                                 size_t take) override;
  size_t count_orphan_file_paths_in_dir(int32_t location_id, const std::string& dir) override;
  std::vector<FilePathRow> get_orphan_file_paths_in_dir(int32_t location_id, int32_t cursor, const std::string& dir,
                                                        size_t take) override;
  void set_cas_id(int32_t file_path_id, const std::optional<std::string>& cas_id) override;
  std::vector<std::pair<int32_t, std::vector<std::string>>> existing_objects(
      const std::vector<std::string>& cas_ids) override;
  // one probe of the cas_id index per cas_id (the reference's schema, without
  // that index: the existing_objects query)
  std::vector<std::pair<std::string, int32_t>> first_objects(const std::vector<std::string>& cas_ids) override;
  void set_cas_id_and_connect(int32_t file_path_id, const std::optional<std::string>& cas_id,
                              int32_t object_id) override;
  // UPDATE ... FROM (VALUES ...) of up to 64 rows per statement (bulk
  // identify: of rows without an Object, a row found with one takes the
  // general path)
  void set_cas_ids_and_connect(const std::vector<CasLink>& rows) override;
  int32_t create_object(ObjectKind kind, int64_t date_created) override;
  // multi-row INSERTs of up to 64 Objects each
  std::vector<int32_t> create_objects(const std::vector<std::pair<ObjectKind, int64_t>>& kinds_dates) override;
  void connect(int32_t file_path_id, int32_t object_id) override;
  std::vector<FilePathRow> file_paths_without_checksum(int32_t location_id, const std::string& sub) override;
  void set_integrity_checksum(int32_t file_path_id, const std::string& checksum) override;
  void begin_batch() override;
  void end_batch() override;
  // with the cas_id index, when the library holds at most 4x `orphans` rows
  // with a cas_id (loading them costs less than indexing the job's rows one
  // by one): the index goes, a host map of its MIN(object_id) per cas_id
  // stays; a write that could make the map stale (a row with an Object and
  // a cas_id gets another of either) restores the index first — inside a
  // batch that commits the batch's writes so far and opens a new
  // transaction for the rest (CREATE INDEX runs in its own)
  bool begin_bulk_identify(size_t orphans) override;
  void end_bulk_identify() override;
  bool bulk_identify_active() const;
  // a file database (not ":memory:") opens a second, read-only connection
  // for the job's read-ahead (WAL readers do not wait for the writer)
  bool concurrent_orphan_reads() override;
  std::vector<FilePathRow> get_orphan_file_paths_concurrent(int32_t location_id, int32_t cursor,
                                                            const std::string& sub, size_t take) override;

 private:
  struct Impl;
  explicit SqliteLibrary(std::unique_ptr<Impl> d);
  std::unique_ptr<Impl> d_;
};

// ---- file_identifier ----------------------------------------------------------

// FileMetadata (mod.rs:48-53)
struct FileMetadata {
  std::optional<std::string> cas_id;  // None for an empty file (mod.rs:78-86)
  ObjectKind kind = 0;
  uint64_t len = 0;  // fs_metadata.len()
};

// FileMetadata::new for a batch of (full path, kind): fs::metadata, the
// is_dir assertion (mod.rs:67-70, std::logic_error here), the kind from the
// path (object_kind_of) unless the pair carries one (>= 0), cas_id only for
// len != 0, one generate_cas_ids call for the batch (the join_all of
// mod.rs:105-147). Errors carry the path (FileIOError). size_hints (may be
// null; one per file): the indexer's sizes (file_path size_in_bytes), which
// only plan the reads' staging (sdcas_file_metadata: the metadata is fstat of
// each read's descriptor).
std::vector<Result<FileMetadata>> file_metadata_batch(Engine& engine,
                                                      const std::vector<std::pair<std::string, ObjectKind>>& files,
                                                      const std::vector<uint64_t>* size_hints = nullptr);

// The DB half of the job's steps over a batch of its orphans (mod.rs:157-342
// per step): write the cas_id of every row the steps read, look up the
// existing Objects of their cas_ids, group (the GPU's sdcas_dedup_window in
// identifier_job_step; any function with its encoding here), create Objects
// and link. md[i] is file_paths[i]'s FileMetadata. window (in: max_steps,
// more; out: steps, rows, rereads) may be null: the whole job over these rows.
// The steps' bookkeeping comes from sdcas_job_plan before any write. A batch
// must not hold a row to re-identify — an Object but no cas_id (the indexer
// nulls cas_id of a changed file) — past its first step: its cas_id, written
// in its own step, makes its Object an existing one for the steps after
// (mod.rs:157-188); the job cuts its batches there (run_file_identifier_job),
// and this function throws std::invalid_argument if one is left.
using GroupBy = std::function<Engine::Dedup(const std::vector<uint64_t>& keys, const std::vector<uint8_t>& has_key,
                                            const std::vector<int32_t>& status,
                                            const std::vector<uint64_t>& existing_keys, sdcas_job_window& window)>;
std::pair<size_t, size_t> identifier_step_db(Library& db, const std::vector<FilePathRow>& file_paths,
                                             const std::vector<Result<FileMetadata>>& md, const GroupBy& group_by,
                                             sdcas_job_window* window = nullptr,
                                             size_t chunk_size = SDCAS_IDENTIFIER_CHUNK_SIZE);

// sdcas_job_plan over the rows' FileMetadata: per row the step that first
// reads it (UINT64_MAX: none) and how many steps read it
struct StepPlan {
  std::vector<uint64_t> step;
  std::vector<uint32_t> reads;
};
StepPlan plan_steps(const std::vector<Result<FileMetadata>>& md, size_t chunk_size, sdcas_job_window& window);

// identifier_job_step (mod.rs:98-350) over `file_paths` in id order: one
// step of the reference per chunk_size rows (CHUNK_SIZE = 100), the cursor
// rule included (a step's last row that stays an orphan is read again by the
// next step). window as in identifier_step_db. Returns (total_created,
// total_linked) as mod.rs:349 does, summed over the steps.
std::pair<size_t, size_t> identifier_job_step(Engine& engine, Library& db, const Location& location,
                                              const std::vector<FilePathRow>& file_paths,
                                              size_t chunk_size = SDCAS_IDENTIFIER_CHUNK_SIZE,
                                              sdcas_job_window* window = nullptr);

// FileIdentifierJobRunMetadata (file_identifier_job.rs:54-71)
struct FileIdentifierJobRunMetadata {
  int32_t cursor = 0;
  size_t total_orphan_paths = 0;
  size_t total_objects_created = 0;
  size_t total_objects_linked = 0;
  size_t total_objects_ignored = 0;
  size_t steps = 0;           // the reference's steps
  size_t batches = 0;         // fetches of `batch` rows
  size_t rereads = 0;         // rows two consecutive steps read
  bool early_finish = false;  // JobError::EarlyFinish (file_identifier_job.rs:184-191)
  bool bulk_identify = false; // the library kept its lookups on the host (FileIdentifierJobInit::bulk_identify)
};

// FileIdentifierJobInit (file_identifier_job.rs:33-37); batch = orphans
// fetched per GPU call (the reference fetches CHUNK_SIZE = 100 per step; a
// larger batch runs several of its steps in one call with identical results)
struct FileIdentifierJobInit {
  Location location;
  std::string sub_materialized_path;  // "" or "/sub/dir/"
  size_t batch = SDCAS_IDENTIFIER_CHUNK_SIZE;
  // let the library trade its lookup index for a host map during the job
  // (Library::begin_bulk_identify); the rows and Objects the job leaves are
  // the same either way
  bool bulk_identify = false;
};

// init (count orphans, cursor = first orphan id, task_count = ceil(count /
// CHUNK_SIZE) steps, file_identifier_job.rs:125-176), then batches: fetch
// `batch` orphans with id >= cursor, run as many of the job's steps over them
// as fit (identifier_job_step with a window), advance the cursor to the last
// row the steps read (mod.rs:401-405). meta.steps counts the reference's
// steps, meta.batches the fetches.
FileIdentifierJobRunMetadata run_file_identifier_job(Engine& engine, Library& db, const FileIdentifierJobInit& init);

// the same loop with any group-by (tests: the CPU oracle), metadata from
// `metadata` (tests: synthetic) instead of the files
using MetadataFn = std::function<std::vector<Result<FileMetadata>>(const std::vector<FilePathRow>& rows)>;
FileIdentifierJobRunMetadata run_file_identifier_job_with(Library& db, const FileIdentifierJobInit& init,
                                                          const MetadataFn& metadata, const GroupBy& group_by);

// the shallow identifier (file_identifier/shallow.rs:24-118, run by
// light_scan_location): the same steps over the orphans of ONE directory
// level (materialized_path = dir; "" or "/" = the location's root), task_count
// = ceil(orphans / CHUNK_SIZE) with no early finish — a step that finds no
// rows leaves the cursor where it is (mod.rs:401-405). Its first cursor comes
// from an unordered find_first (shallow.rs:74-84, `.order_by` commented out):
// the canonical pick here is the lowest orphan id, which is what SQLite returns
// for that query when it scans in rowid order. `batch` as in
// FileIdentifierJobInit.
struct ShallowIdentifierReport {
  size_t orphans = 0, steps = 0, batches = 0, rereads = 0;
  size_t created = 0, linked = 0;
  int32_t cursor = 0;
};
ShallowIdentifierReport shallow_file_identifier(Engine& engine, Library& db, const Location& location,
                                                const std::string& dir, size_t batch = SDCAS_IDENTIFIER_CHUNK_SIZE);
ShallowIdentifierReport shallow_file_identifier_with(Library& db, const Location& location, const std::string& dir,
                                                     size_t batch, const MetadataFn& metadata,
                                                     const GroupBy& group_by);

// ---- object validator -----------------------------------------------------------

struct ObjectValidatorJobInit {  // validator_job.rs:38-42
  Location location;
  std::string sub_materialized_path;
  size_t batch = SDCAS_IDENTIFIER_CHUNK_SIZE;  // the reference runs one file per step
};

struct ObjectValidatorReport {
  size_t task_count = 0;   // rows selected at init
  size_t checksummed = 0;  // integrity_checksum written
  // the first file whose checksum failed: the reference's execute_step returns
  // ValidatorError::FileIO (validator_job.rs:154-156) and the job stops there
  std::optional<IoError> error;
};

ObjectValidatorReport run_object_validator_job(Engine& engine, Library& db, const ObjectValidatorJobInit& init);

}  // namespace sdcore
