// sdcore.cpp — C++ host mirror of sd-core's content-identification path over
// libsdcas (see include/sdcore.hpp for the reference file:line of each entry).
#include "sdcore.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <exception>
#include <future>
#include <mutex>
#include <set>
#include <thread>
#include <unordered_map>
#include <unordered_set>

namespace sdcore {

std::string IoError::message() const {
  std::string m = unexpected_eof() ? "failed to fill whole buffer" : std::strerror(code);
  return path.empty() ? m : m + " <path='" + path + "'>";
}

// ---- Engine -------------------------------------------------------------------

void Engine::fail(int rc, const char* what) const { fail_on(ctx_, rc, what); }

void Engine::fail_on(sdcas_ctx* c, int rc, const char* what) const {
  throw LibraryError(rc, std::string(what) + ": " + sdcas_last_error(c));
}

sdcas_ctx* Engine::dedup_ctx() {
  static const bool same = [] {
    const char* v = getenv("SDCORE_DEDUP_CTX");
    return v && strcmp(v, "same") == 0;
  }();
  if (same) return ctx_;
  std::lock_guard<std::mutex> g(dedup_mu_);
  if (!dedup_ctx_) {
    sdcas_options opts = SDCAS_OPTIONS_INIT;
    opts.device = device_;
    sdcas_ctx* c = nullptr;
    if (sdcas_init(&opts, &c) != SDCAS_OK) {  // no second context: share the first
      if (c) sdcas_destroy(c);
      return ctx_;
    }
    dedup_ctx_ = c;
  }
  return dedup_ctx_;
}

std::unique_ptr<Engine> Engine::open(const Options& o) {
  sdcas_options opts = SDCAS_OPTIONS_INIT;
  opts.device = o.device;
  opts.io_threads = o.io_threads;
  opts.flags = o.flags;
  opts.staging_bytes = o.staging_bytes;
  opts.progress = o.progress;
  opts.progress_user = o.progress_user;
  opts.cancel = o.cancel;
  sdcas_ctx* c = nullptr;
  const int rc = sdcas_init(&opts, &c);
  if (rc != SDCAS_OK) {
    std::string msg = c ? sdcas_last_error(c) : "sdcas_init failed";
    if (c) sdcas_destroy(c);
    throw LibraryError(rc, msg);
  }
  return std::unique_ptr<Engine>(new Engine(c, o.device));
}

Engine::~Engine() {
  if (dedup_ctx_) sdcas_destroy(dedup_ctx_);
  sdcas_destroy(ctx_);
}

std::string key_to_hex(uint64_t key) {
  char b[17];
  sdcas_key_to_hex(key, b);
  return std::string(b, 16);
}

uint64_t hex_to_key(const std::string& cas_id) {
  if (cas_id.size() != 16) throw std::invalid_argument("cas_id must be 16 hex chars: " + cas_id);
  return std::stoull(cas_id, nullptr, 16);
}

Engine::RawMetadata Engine::file_metadata(const std::vector<const char*>& paths, const uint64_t* size_hints) {
  const size_t n = paths.size();
  RawMetadata m;
  m.size.resize(n);
  m.key.resize(n);
  m.status.resize(n);
  m.flags.resize(n);
  if (n) {
    const int rc = sdcas_file_metadata(ctx_, paths.data(), size_hints, n, m.size.data(), m.key.data(),
                                       m.status.data(), m.flags.data());
    if (rc != SDCAS_OK) fail(rc, "sdcas_file_metadata");
  }
  return m;
}

std::vector<Result<std::string>> Engine::generate_cas_ids(
    const std::vector<std::pair<std::string, uint64_t>>& files) {
  const size_t n = files.size();
  std::vector<const char*> paths(n);
  std::vector<uint64_t> sizes(n), keys(n);
  std::vector<int32_t> st(n);
  for (size_t i = 0; i < n; ++i) {
    paths[i] = files[i].first.c_str();
    sizes[i] = files[i].second;
  }
  if (n) {
    const int rc = sdcas_cas_ids(ctx_, paths.data(), sizes.data(), n, keys.data(), st.data());
    if (rc != SDCAS_OK) fail(rc, "sdcas_cas_ids");
  }
  std::vector<Result<std::string>> out;
  out.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (st[i]) out.emplace_back(IoError{st[i], files[i].first});
    else out.emplace_back(key_to_hex(keys[i]));
  }
  return out;
}

std::vector<Result<std::string>> Engine::file_checksums(const std::vector<std::string>& files) {
  const size_t n = files.size();
  std::vector<const char*> paths(n);
  std::vector<uint8_t> d(32 * n);
  std::vector<int32_t> st(n);
  for (size_t i = 0; i < n; ++i) paths[i] = files[i].c_str();
  if (n) {
    const int rc = sdcas_checksums(ctx_, paths.data(), n, d.data(), st.data());
    if (rc != SDCAS_OK) fail(rc, "sdcas_checksums");
  }
  std::vector<Result<std::string>> out;
  out.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (st[i]) {
      out.emplace_back(IoError{st[i], files[i]});
    } else {
      char h[65];
      sdcas_digest_to_hex(&d[32 * i], h);
      out.emplace_back(std::string(h, 64));
    }
  }
  return out;
}

Engine::Dedup Engine::dedup(const std::vector<uint64_t>& keys, const std::vector<uint8_t>& has_key,
                            const std::vector<int32_t>& status, size_t chunk_size,
                            const std::vector<uint64_t>& existing_keys, sdcas_job_window* window) {
  const size_t n = keys.size();
  if (has_key.size() != n || (!status.empty() && status.size() != n))
    throw std::invalid_argument("dedup: keys / has_key / status lengths differ");
  Dedup r;
  r.link.assign(n, 0);
  if (!n) {
    if (window) window->steps = window->rows = window->rereads = 0;
    return r;
  }
  sdcas_ctx* dc = dedup_ctx();
  const int rc = sdcas_dedup_window(dc, keys.data(), has_key.data(), status.empty() ? nullptr : status.data(), n,
                                    chunk_size, existing_keys.empty() ? nullptr : existing_keys.data(),
                                    existing_keys.size(), window, r.link.data(), &r.created, &r.linked);
  if (rc != SDCAS_OK) fail_on(dc, rc, "sdcas_dedup_window");
  return r;
}

Result<std::string> generate_cas_id(Engine& engine, const std::string& path, uint64_t size) {
  return std::move(engine.generate_cas_ids({{path, size}})[0]);
}

Result<std::string> file_checksum(Engine& engine, const std::string& path) {
  return std::move(engine.file_checksums({path})[0]);
}

// ---- paths --------------------------------------------------------------------

std::string full_path(const Location& location, const FilePathRow& row) {
  // assemble_relative_path: materialized_path without its leading '/', then
  // name, then ".extension" for a file with a non-empty extension
  std::string rel = row.materialized_path.size() > 1 ? row.materialized_path.substr(1) : std::string();
  rel += row.name;
  if (!row.is_dir && !row.extension.empty()) rel += "." + row.extension;
  std::string base = location.path;
  if (!base.empty() && base.back() != '/') base += '/';
  return base + rel;
}

// ---- indexer walk ------------------------------------------------------------------

std::pair<std::string, std::optional<std::string>> file_stem_and_extension(const std::string& name) {
  // std::path's rsplit_file_at_dot: "..": no extension; the text before the
  // last dot empty (".bashrc"): no extension; else (before, after)
  if (name == "..") return {name, std::nullopt};
  const size_t dot = name.rfind('.');
  if (dot == std::string::npos) return {name, std::nullopt};
  if (dot == 0) return {name, std::nullopt};
  return {name.substr(0, dot), name.substr(dot + 1)};
}

std::vector<FilePathRow> walk_location(const Location& location, std::vector<IoError>* errors) {
  std::vector<FilePathRow> out;
  std::string root = location.path;
  while (root.size() > 1 && root.back() == '/') root.pop_back();
  std::vector<std::string> queue{""};  // relative directory paths, "" = the location itself
  for (size_t qi = 0; qi < queue.size(); ++qi) {
    const std::string rel = queue[qi];
    const std::string dir = rel.empty() ? root : root + "/" + rel;
    DIR* d = opendir(dir.c_str());
    if (!d) {
      if (errors) errors->push_back(IoError{errno, dir});
      continue;
    }
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
      if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
      names.emplace_back(e->d_name);
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    for (const auto& name : names) {
      const std::string full = dir + "/" + name;
      struct stat sb;
      if (lstat(full.c_str(), &sb) != 0) {
        if (errors) errors->push_back(IoError{errno, full});
        continue;
      }
      if (S_ISLNK(sb.st_mode)) continue;
      const bool is_dir = S_ISDIR(sb.st_mode);
      if (!is_dir && !S_ISREG(sb.st_mode)) continue;  // sockets, fifos, devices
      FilePathRow r;
      r.location_id = location.id;
      r.is_dir = is_dir;
      r.materialized_path = rel.empty() ? "/" : "/" + rel + "/";
      if (is_dir) {
        r.name = name;
      } else {
        auto [stem, ext] = file_stem_and_extension(name);
        r.name = stem;
        r.extension = ext.value_or("");
      }
      r.size_in_bytes = (uint64_t)sb.st_size;
      r.inode = (uint64_t)sb.st_ino;
      r.hidden = !name.empty() && name[0] == '.';
      r.date_created = (int64_t)sb.st_mtime;  // created_or_now(): birth time is not in struct stat
      out.push_back(std::move(r));
      if (is_dir) queue.push_back(rel.empty() ? name : rel + "/" + name);
    }
  }
  return out;
}

// ---- MemoryLibrary ------------------------------------------------------------------

// pub_ids in creation order: a tag, then the id big-endian in the last 8
// bytes, so that consecutive rows sort together (memcmp order) — the
// reference draws them at random (Uuid::new_v4, mod.rs:273), which is why it
// cannot be matched byte for byte, and an ordered id keeps the UNIQUE index
// on pub_id appending instead of inserting at random (as UUIDv7 does)
static PubId pub_id_of(uint32_t tag, int64_t id) {
  PubId p{};
  std::memcpy(p.data(), &tag, 4);
  for (int i = 0; i < 8; ++i) p[8 + i] = (uint8_t)((uint64_t)id >> (56 - 8 * i));
  return p;
}

FilePathRow& MemoryLibrary::add_file_path(FilePathRow row) {
  if (row.id == 0) row.id = next_file_path_id_;
  next_file_path_id_ = std::max(next_file_path_id_, row.id + 1);
  if (row.pub_id == PubId{}) row.pub_id = pub_id_of(0x46504154u, row.id);
  auto it = std::lower_bound(file_paths.begin(), file_paths.end(), row.id,
                             [](const FilePathRow& a, int32_t id) { return a.id < id; });
  if (it != file_paths.end() && it->id == row.id) throw std::invalid_argument("duplicate file_path id");
  return *file_paths.insert(it, std::move(row));
}

FilePathRow* MemoryLibrary::find(int32_t id) {
  auto it = std::lower_bound(file_paths.begin(), file_paths.end(), id,
                             [](const FilePathRow& a, int32_t v) { return a.id < v; });
  return it != file_paths.end() && it->id == id ? &*it : nullptr;
}

const FilePathRow* MemoryLibrary::file_path(int32_t id) const {
  return const_cast<MemoryLibrary*>(this)->find(id);
}

static bool under(const FilePathRow& r, const std::string& sub) {
  return sub.empty() || r.materialized_path.compare(0, sub.size(), sub) == 0;
}

bool MemoryLibrary::orphan(const FilePathRow& r, int32_t location_id, const std::string& sub) const {
  return (!r.object_id || !r.cas_id) && !r.is_dir && r.location_id == location_id && r.size_in_bytes != 0 &&
         under(r, sub);
}

size_t MemoryLibrary::count_orphan_file_paths(int32_t location_id, const std::string& sub) {
  return (size_t)std::count_if(file_paths.begin(), file_paths.end(),
                               [&](const FilePathRow& r) { return orphan(r, location_id, sub); });
}

std::vector<FilePathRow> MemoryLibrary::get_orphan_file_paths(int32_t location_id, int32_t cursor,
                                                              const std::string& sub, size_t take) {
  std::vector<FilePathRow> out;
  for (const auto& r : file_paths) {
    if (out.size() >= take) break;
    if (r.id >= cursor && orphan(r, location_id, sub)) out.push_back(r);
  }
  return out;
}

static bool orphan_in_dir(const FilePathRow& r, int32_t location_id, const std::string& dir) {
  return (!r.object_id || !r.cas_id) && !r.is_dir && r.location_id == location_id && r.size_in_bytes != 0 &&
         r.materialized_path == dir;
}

size_t MemoryLibrary::count_orphan_file_paths_in_dir(int32_t location_id, const std::string& dir) {
  return (size_t)std::count_if(file_paths.begin(), file_paths.end(),
                               [&](const FilePathRow& r) { return orphan_in_dir(r, location_id, dir); });
}

std::vector<FilePathRow> MemoryLibrary::get_orphan_file_paths_in_dir(int32_t location_id, int32_t cursor,
                                                                     const std::string& dir, size_t take) {
  std::vector<FilePathRow> out;
  for (const auto& r : file_paths) {
    if (out.size() >= take) break;
    if (r.id >= cursor && orphan_in_dir(r, location_id, dir)) out.push_back(r);
  }
  return out;
}

void MemoryLibrary::set_cas_id(int32_t id, const std::optional<std::string>& cas_id) {
  if (auto* r = find(id)) r->cas_id = cas_id;
}

std::vector<std::pair<int32_t, std::vector<std::string>>> MemoryLibrary::existing_objects(
    const std::vector<std::string>& cas_ids) {
  const std::set<std::string> want(cas_ids.begin(), cas_ids.end());
  std::map<int32_t, std::vector<std::string>> by_object;  // object id order = DB order
  std::set<int32_t> hit;
  for (const auto& r : file_paths) {
    if (!r.object_id) continue;
    if (r.cas_id && want.count(*r.cas_id)) hit.insert(*r.object_id);
  }
  for (const auto& r : file_paths)
    if (r.object_id && hit.count(*r.object_id) && r.cas_id) by_object[*r.object_id].push_back(*r.cas_id);
  return {by_object.begin(), by_object.end()};
}

std::vector<std::pair<std::string, int32_t>> Library::first_objects(const std::vector<std::string>& cas_ids) {
  const std::set<std::string> want(cas_ids.begin(), cas_ids.end());
  std::set<std::string> got;
  std::vector<std::pair<std::string, int32_t>> out;
  for (const auto& [oid, cs] : existing_objects(cas_ids))  // objects in DB order
    for (const auto& c : cs)
      if (want.count(c) && got.insert(c).second) out.emplace_back(c, oid);
  return out;
}

int32_t MemoryLibrary::create_object(ObjectKind kind, int64_t date_created) {
  ObjectRow o;
  o.id = next_object_id_++;
  o.pub_id = pub_id_of(0x4F424A54u, o.id);
  o.kind = kind;
  o.date_created = date_created;
  objects.push_back(o);
  return o.id;
}

void MemoryLibrary::connect(int32_t file_path_id, int32_t object_id) {
  if (auto* r = find(file_path_id)) r->object_id = object_id;
}

std::vector<FilePathRow> MemoryLibrary::file_paths_without_checksum(int32_t location_id, const std::string& sub) {
  std::vector<FilePathRow> out;
  for (const auto& r : file_paths)
    if (r.location_id == location_id && !r.is_dir && !r.integrity_checksum && under(r, sub)) out.push_back(r);
  return out;
}

void MemoryLibrary::set_integrity_checksum(int32_t id, const std::string& checksum) {
  if (auto* r = find(id)) r->integrity_checksum = checksum;
}

// ---- file_identifier ----------------------------------------------------------------

// SDCORE_DIRFD=0: the stat pass by full path (A/B)
static bool stat_dirfd() {
  static const bool on = [] {
    const char* v = getenv("SDCORE_DIRFD");
    return !(v && strcmp(v, "0") == 0);
  }();
  return on;
}

// SDCORE_FOLD_STAT=0: fs::metadata as its own fstatat pass before the cas_id
// reads (round 5) instead of inside them (sdcas_file_metadata) (A/B)
static bool fold_stat() {
  static const bool on = [] {
    const char* v = getenv("SDCORE_FOLD_STAT");
    return !(v && strcmp(v, "0") == 0);
  }();
  return on;
}

std::vector<Result<FileMetadata>> file_metadata_batch(Engine& engine,
                                                      const std::vector<std::pair<std::string, ObjectKind>>& files,
                                                      const std::vector<uint64_t>* size_hints) {
  const size_t n = files.size();
  if (size_hints && size_hints->size() != n) throw std::invalid_argument("file_metadata_batch: one size hint per file");
  if (fold_stat()) {
    // fs::metadata, the kind and generate_cas_id (mod.rs:63-86) in one library
    // call: the metadata is the fstat of the descriptor the reads use
    std::vector<const char*> paths(n);
    for (size_t i = 0; i < n; ++i) paths[i] = files[i].first.c_str();
    const auto t0 = std::chrono::steady_clock::now();
    const Engine::RawMetadata raw = engine.file_metadata(paths, size_hints ? size_hints->data() : nullptr);
    static const bool trace = [] {
      const char* v = getenv("SDCORE_TRACE_JOB");
      return v && *v && strcmp(v, "0") != 0;
    }();
    const auto t1 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n; ++i)
      if (raw.flags[i] & SDCAS_META_DIR)
        throw std::logic_error("We can't generate cas_id for directories");  // mod.rs:67-70
    // the results (the kind from the extension, the hex cas_id) on a few
    // threads for a big batch: this thread's part of the job's read-ahead
    std::vector<Result<FileMetadata>> out(n, Result<FileMetadata>(IoError{}));
    auto fill = [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        if (raw.status[i]) {
          out[i] = IoError{raw.status[i], files[i].first};
          continue;
        }
        FileMetadata m;
        m.kind = files[i].second >= 0 ? files[i].second : object_kind_of(files[i].first);  // mod.rs:72-76
        m.len = raw.size[i];
        if (raw.flags[i] & SDCAS_META_HAS_CAS_ID) m.cas_id = key_to_hex(raw.key[i]);
        out[i] = std::move(m);
      }
    };
    const size_t parts = std::min<size_t>(4, n / 2048 + 1);
    if (parts < 2) {
      fill(0, n);
    } else {
      std::vector<std::thread> th;
      for (size_t t = 1; t < parts; ++t) th.emplace_back(fill, n * t / parts, n * (t + 1) / parts);
      fill(0, n / parts);
      for (auto& x : th) x.join();
    }
    if (trace)
      fprintf(stderr, "sdcore file_metadata_batch: %zu files, sdcas_file_metadata %.2f ms, results %.2f ms\n", n,
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    return out;
  }
  std::vector<std::optional<IoError>> err(n);
  std::vector<FileMetadata> md(n);
  std::vector<uint8_t> is_dir(n, 0);
  // fs::metadata and the kind per file (mod.rs:63-76), on up to 16 threads for
  // a big batch (the reference's join_all runs them concurrently too)
  // each file is stat'ed relative to its directory, whose descriptor a
  // thread keeps while consecutive files share it (one path component walked
  // instead of all; the library's readers open the same way, cas_io.cpp)
  auto stat_range = [&](size_t lo, size_t hi) {
    std::string dir;
    int dfd = -1;
    for (size_t i = lo; i < hi; ++i) {
      struct stat sb;
      const std::string& p = files[i].first;
      const size_t slash = p.rfind('/');
      int at = AT_FDCWD;
      const char* name = p.c_str();
      if (stat_dirfd() && slash != std::string::npos && slash > 0 && slash + 1 < p.size()) {
        if (dfd < 0 || dir.size() != slash || p.compare(0, slash, dir) != 0) {
          if (dfd >= 0) ::close(dfd);
          dir.assign(p, 0, slash);
          dfd = ::open(dir.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
        }
        if (dfd >= 0) {
          at = dfd;
          name = p.c_str() + slash + 1;
        }
      }
      if (::fstatat(at, name, &sb, 0) != 0) {  // fs::metadata (mod.rs:63-65)
        err[i] = IoError{errno, files[i].first};
        continue;
      }
      if (S_ISDIR(sb.st_mode)) {
        is_dir[i] = 1;
        continue;
      }
      md[i].kind = files[i].second >= 0 ? files[i].second : object_kind_of(files[i].first);  // mod.rs:72-76
      md[i].len = (uint64_t)sb.st_size;
    }
    if (dfd >= 0) ::close(dfd);
  };
  static const bool trace = [] {
    const char* v = getenv("SDCORE_TRACE_JOB");
    return v && *v && strcmp(v, "0") != 0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  const size_t threads = std::min<size_t>(16, n / 512);
  if (threads < 2) {
    stat_range(0, n);
  } else {
    std::vector<std::thread> pool;
    for (size_t t = 0; t < threads; ++t) pool.emplace_back(stat_range, n * t / threads, n * (t + 1) / threads);
    for (auto& th : pool) th.join();
  }
  std::vector<std::pair<std::string, uint64_t>> to_hash;
  std::vector<size_t> hashed_index;
  for (size_t i = 0; i < n; ++i) {
    if (is_dir[i]) throw std::logic_error("We can't generate cas_id for directories");  // mod.rs:67-70
    if (err[i]) continue;
    if (md[i].len != 0) {  // mod.rs:78-86: empty files get no cas_id
      to_hash.emplace_back(files[i].first, md[i].len);
      hashed_index.push_back(i);
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  auto cas = engine.generate_cas_ids(to_hash);
  if (trace)
    fprintf(stderr, "sdcore file_metadata_batch: %zu files, stat+kind %.2f ms, cas_ids %.2f ms\n", n,
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  for (size_t k = 0; k < cas.size(); ++k) {
    const size_t i = hashed_index[k];
    if (cas[k].ok()) md[i].cas_id = cas[k].value();
    else err[i] = cas[k].error();
  }
  std::vector<Result<FileMetadata>> out;
  out.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (err[i]) out.emplace_back(*err[i]);
    else out.emplace_back(std::move(md[i]));
  }
  return out;
}

static void flags_of(const std::vector<Result<FileMetadata>>& md, std::vector<uint8_t>& has_key,
                     std::vector<int32_t>& status) {
  const size_t n = md.size();
  has_key.assign(n, 0);
  status.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    if (!md[i].ok()) status[i] = md[i].error().code;
    else has_key[i] = md[i].value().cas_id ? 1 : 0;
  }
}

StepPlan plan_steps(const std::vector<Result<FileMetadata>>& md, size_t chunk_size, sdcas_job_window& window) {
  std::vector<uint8_t> has_key;
  std::vector<int32_t> status;
  flags_of(md, has_key, status);
  StepPlan p;
  p.step.resize(md.size());
  p.reads.resize(md.size());
  const int rc =
      sdcas_job_plan(has_key.data(), status.data(), md.size(), chunk_size, &window, p.step.data(), p.reads.data());
  if (rc != SDCAS_OK) throw LibraryError(rc, "sdcas_job_plan");
  return p;
}

// a row to re-identify: an Object but no cas_id (the indexer nulled it when
// the file changed); writing its new cas_id makes its Object "existing" for
// that cas_id from its own step on (mod.rs:157-188)
static bool reidentified(const FilePathRow& r, const Result<FileMetadata>& md) {
  return r.object_id && !r.cas_id && md.ok() && md.value().cas_id;
}

// SDCORE_TRACE_JOB=1: where the identifier job's wall time goes, per phase
// of its main thread, summed over the job and printed to stderr at its end
// (a diagnostic; the phases of the read-ahead thread overlap them)
namespace {
struct JobTrace {
  enum { kMetadata, kWaitAhead, kFetch, kPlan, kCasWrites, kLookup, kGroupBy, kObjects, kIndex, kInit, kN };
  bool on = [] {
    const char* v = getenv("SDCORE_TRACE_JOB");
    return v && *v && strcmp(v, "0") != 0;
  }();
  double t[kN] = {};
  const std::chrono::steady_clock::time_point start = std::chrono::steady_clock::now();
  std::chrono::steady_clock::time_point m = start;
  void mark() { m = std::chrono::steady_clock::now(); }
  void lap(int k) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    t[k] += std::chrono::duration<double>(now - m).count();
    m = now;
  }
  void print() const {
    if (!on) return;
    double sum = 0;
    for (double x : t) sum += x;
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    fprintf(stderr,
            "sdcore job trace s: metadata %.3f wait_ahead %.3f fetch %.3f plan %.3f cas_writes %.3f lookup %.3f "
            "group_by %.3f objects_links %.3f index %.3f init %.3f other %.3f wall %.3f\n",
            t[kMetadata], t[kWaitAhead], t[kFetch], t[kPlan], t[kCasWrites], t[kLookup], t[kGroupBy], t[kObjects],
            t[kIndex], t[kInit], wall - sum, wall);
  }
};
thread_local JobTrace* g_trace = nullptr;
void trace_lap(int k) {
  if (g_trace) g_trace->lap(k);
}
void trace_mark() {
  if (g_trace) g_trace->mark();
}
}  // namespace

// once the batch's steps are planned, before any of its writes: the job's
// loop starts reading its next batch there (run_steps)
using OnGrouped = std::function<void(const sdcas_job_window& done)>;

static std::pair<size_t, size_t> step_db(Library& db, const std::vector<FilePathRow>& file_paths,
                                         const std::vector<Result<FileMetadata>>& md, const GroupBy& group_by,
                                         sdcas_job_window* window, size_t chunk_size, const OnGrouped* on_grouped,
                                         const OnGrouped* after_group_by = nullptr,
                                         const OnGrouped* after_lookup = nullptr);

std::pair<size_t, size_t> identifier_step_db(Library& db, const std::vector<FilePathRow>& file_paths,
                                             const std::vector<Result<FileMetadata>>& md, const GroupBy& group_by,
                                             sdcas_job_window* window, size_t chunk_size) {
  return step_db(db, file_paths, md, group_by, window, chunk_size, nullptr);
}

static std::pair<size_t, size_t> step_db(Library& db, const std::vector<FilePathRow>& file_paths,
                                         const std::vector<Result<FileMetadata>>& md, const GroupBy& group_by,
                                         sdcas_job_window* window, size_t chunk_size, const OnGrouped* on_grouped,
                                         const OnGrouped* after_group_by, const OnGrouped* after_lookup) {
  const size_t n = file_paths.size();
  if (md.size() != n) throw std::invalid_argument("identifier_step_db: one metadata per file_path");
  sdcas_job_window win{};
  if (window) {
    win.max_steps = window->max_steps;
    win.more = window->more;
  }
  // which rows the steps read: only theirs are written (mod.rs:157-178)
  trace_mark();
  const StepPlan plan = plan_steps(md, chunk_size, win);
  const auto& step = plan.step;
  // the plan fixes which rows the steps read, so the job's read-ahead of its
  // next batch (rows past the last of them) starts now, beside this batch's
  // writes, lookup and group-by
  if (on_grouped) (*on_grouped)(win);
  trace_lap(JobTrace::kFetch);
  for (size_t i = 0; i < n; ++i)
    if (step[i] != UINT64_MAX && step[i] > 0 && reidentified(file_paths[i], md[i]))
      throw std::invalid_argument("identifier_step_db: a row to re-identify past the batch's first step");
  std::vector<uint64_t> keys(n, 0);
  std::vector<uint8_t> has_key(n, 0);
  std::vector<int32_t> status(n, 0);
  std::vector<std::string> unique;
  std::unordered_set<uint64_t> seen;  // by cas key: cas_ids are canonical 16-hex (cas.rs:61)
  seen.reserve(n);
  // cas_id writes (mod.rs:157-178): a row with an Object now, since the
  // lookup below can find its Object by it; a row without one together with
  // its link (set_cas_id_and_connect), the same end state in one write
  std::vector<uint8_t> cas_pending(n, 0);
  db.begin_batch();
  for (size_t i = 0; i < n; ++i) {
    if (!md[i].ok()) {
      status[i] = md[i].error().code;
      continue;
    }
    const auto& cas = md[i].value().cas_id;
    if (cas) {
      keys[i] = hex_to_key(*cas);
      has_key[i] = 1;
    }
    if (step[i] == UINT64_MAX) continue;  // no step reads it: it stays as it is
    if (cas && seen.insert(keys[i]).second) unique.push_back(*cas);
    if (file_paths[i].object_id) db.set_cas_id(file_paths[i].id, cas);
    else cas_pending[i] = 1;
  }
  db.end_batch();
  trace_lap(JobTrace::kCasWrites);
  // the first existing Object carrying each cas_id, DB order (mod.rs:181-188
  // and the find of :214-224): one existing-key entry per cas_id
  std::vector<uint64_t> ekeys;
  std::vector<int32_t> eobj;
  for (const auto& [c, oid] : db.first_objects(unique)) {
    ekeys.push_back(hex_to_key(c));
    eobj.push_back(oid);
  }
  trace_lap(JobTrace::kLookup);
  // (or here: the chunked loop's read-ahead beside the group-by and the
  // writes, not beside the lookup's index probes)
  if (after_lookup) (*after_lookup)(win);
  sdcas_job_window gw{};
  gw.max_steps = win.max_steps;
  gw.more = win.more;
  auto d = group_by(keys, has_key, status, ekeys, gw);
  trace_lap(JobTrace::kGroupBy);
  // (the chunked loop's read-ahead starts here: its FileMetadata call would
  // otherwise hold the engine while this batch's group-by waits for it)
  if (after_group_by) (*after_group_by)(win);
  if (d.link.size() != n) throw std::logic_error("identifier_step_db: group-by returned a wrong link count");
  if (gw.steps != win.steps || gw.rows != win.rows)
    throw std::logic_error("identifier_step_db: the group-by ran other steps than the plan");
  // new Objects (mod.rs:246-342) in the order the steps create them: step by
  // step, rows in id order within a step; a row without cas_id that several
  // steps read gets an Object from each, the last one its link. They take
  // the kind and date_created of their file (mod.rs:266-291).
  std::vector<std::pair<uint64_t, size_t>> creates;
  for (size_t i = 0; i < n; ++i)
    if (d.link[i] == (int64_t)i)
      for (uint32_t r = 0; r < plan.reads[i]; ++r) creates.emplace_back(plan.step[i] + r, i);
  std::stable_sort(creates.begin(), creates.end(),
                   [](const std::pair<uint64_t, size_t>& a, const std::pair<uint64_t, size_t>& b) {
                     return a.first < b.first;
                   });
  // each row's last link: a row several steps read links to the Object of
  // the last (creates are in step order); 0 = not linked
  std::vector<int32_t> created_object(n, 0), link_to(n, 0);
  db.begin_batch();
  {
    // object::create_many (mod.rs:314-327), then the links of :331-342
    std::vector<std::pair<ObjectKind, int64_t>> kd;
    kd.reserve(creates.size());
    for (const auto& [s, i] : creates) kd.emplace_back(md[i].value().kind, file_paths[i].date_created);
    const std::vector<int32_t> oids = db.create_objects(kd);
    if (oids.size() != creates.size()) throw std::logic_error("identifier_step_db: create_objects returned a wrong count");
    for (size_t k = 0; k < creates.size(); ++k) {
      const size_t i = creates[k].second;
      created_object[i] = link_to[i] = oids[k];
    }
  }
  // links to the first Object carrying the cas_id (mod.rs:202-238)
  for (size_t i = 0; i < n; ++i) {
    const int64_t l = d.link[i];
    if (l == SDCAS_LINK_DROPPED || l == SDCAS_LINK_DEFERRED || l == (int64_t)i) continue;
    link_to[i] = l >= 0 ? created_object[(size_t)l] : eobj[(size_t)(-(l + 1))];
  }
  // one write per row, in row order: a row without an Object takes its
  // cas_id and its link together (set_cas_ids_and_connect), a row with one
  // its link (connect); a row read but not linked its cas_id (none such today)
  std::vector<Library::CasLink> writes;
  writes.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (link_to[i] && cas_pending[i]) writes.push_back({file_paths[i].id, md[i].value().cas_id, link_to[i]});
    else if (link_to[i]) db.connect(file_paths[i].id, link_to[i]);
    else if (cas_pending[i]) db.set_cas_id(file_paths[i].id, md[i].value().cas_id);
  }
  // SDCORE_LINKS=each: the rows one statement each (A/B)
  static const bool each = [] {
    const char* v = getenv("SDCORE_LINKS");
    return v && !strcmp(v, "each");
  }();
  if (each) db.Library::set_cas_ids_and_connect(writes);
  else db.set_cas_ids_and_connect(writes);
  db.end_batch();
  trace_lap(JobTrace::kObjects);
  if (window) *window = win;
  return {(size_t)d.created, (size_t)d.linked};
}
std::pair<size_t, size_t> identifier_job_step(Engine& engine, Library& db, const Location& location,
                                              const std::vector<FilePathRow>& file_paths, size_t chunk_size,
                                              sdcas_job_window* window) {
  const size_t n = file_paths.size();
  std::vector<std::pair<std::string, ObjectKind>> files(n);
  std::vector<uint64_t> hints(n);
  for (size_t i = 0; i < n; ++i) {
    files[i] = {full_path(location, file_paths[i]), file_paths[i].kind};
    hints[i] = file_paths[i].size_in_bytes;
  }
  // FileMetadata::new for every row (mod.rs:105-147): failing files are
  // logged and left out of the rest of the step (mod.rs:125-141)
  auto md = file_metadata_batch(engine, files, &hints);
  return identifier_step_db(
      db, file_paths, md,
      [&](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
          const std::vector<uint64_t>& e, sdcas_job_window& w) { return engine.dedup(k, h, st, chunk_size, e, &w); },
      window, chunk_size);
}

namespace {
// The steps of the identifier over its orphans, `batch` rows per fetch
// (file_identifier_job.rs:180-236 and shallow.rs:92-112 share it): each batch
// runs as many of the job's 100-row steps as it holds (identifier_step_db),
// and the cursor moves to the last row they read (mod.rs:401-405).
struct StepLoop {
  size_t created = 0, linked = 0, steps = 0, batches = 0, rereads = 0;
  int32_t cursor = 0;
  bool ran_dry = false;  // a fetch found no rows
};
using Fetch = std::function<std::vector<FilePathRow>(int32_t cursor, size_t take)>;

// Round 6: the orphans read ahead in chunks on the read-ahead connection by a
// thread of their own, `batch` rows past the last row read so far, up to two
// chunks ahead. Rows past the job's cursor are never written by the batch
// that fetched them (its steps write only the rows they read, all at or
// before the cursor), so a chunk fetched before a batch's writes is what a
// fetch after them would return.
class ChunkFetcher {
 public:
  struct Chunk {
    std::vector<FilePathRow> rows;
    bool full = false;  // `take` rows: more may follow
    std::exception_ptr err;
  };
  ChunkFetcher(const Fetch& fetch, int32_t after, size_t take) : fetch_(fetch), after_(after), take_(take) {
    th_ = std::thread([this] { loop(); });
  }
  ~ChunkFetcher() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  // the next chunk (empty rows: none left), in id order
  Chunk next() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return !q_.empty(); });
    Chunk c = std::move(q_.front());
    q_.pop_front();
    cv_.notify_all();
    return c;
  }

 private:
  static constexpr size_t kDepth = 2;
  void loop() {
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return stop_ || q_.size() < kDepth; });
        if (stop_) return;
      }
      Chunk c;
      try {
        c.rows = fetch_(after_ + 1, take_);  // id >= after + 1 ORDER BY id
        c.full = c.rows.size() == take_;
        if (!c.rows.empty()) after_ = c.rows.back().id;
      } catch (...) {
        c.err = std::current_exception();
      }
      const bool last = c.err || !c.full;
      {
        std::lock_guard<std::mutex> g(m_);
        q_.push_back(std::move(c));
      }
      cv_.notify_all();
      if (last) return;
    }
  }
  const Fetch& fetch_;
  int32_t after_;
  const size_t take_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<Chunk> q_;
  bool stop_ = false;
  std::thread th_;
};

// SDCORE_PIPELINE=0: round 5's loop (the next batch fetched after the plan,
// on the same thread as its FileMetadata) (A/B)
static bool pipeline_enabled() {
  static const bool on = [] {
    const char* v = getenv("SDCORE_PIPELINE");
    return !(v && strcmp(v, "0") == 0);
  }();
  return on;
}

// Where the chunked loop's read-ahead FileMetadata starts in a batch
// (SDCORE_AHEAD_AT): "lookup" (the default) after the existing-Object
// lookup — beside the group-by (its own context, Engine::dedup_ctx, so the
// read-ahead's path call does not hold it up) and the writes, but not beside
// the lookup's index probes, which it slowed (10 000-row batches without bulk
// identify 316 -> 240-280 K orphans/s at "plan"); "plan" at the plan; "groupby"
// after the group-by (A/B)
enum AheadAt { kAheadPlan, kAheadLookup, kAheadGroupBy };
static AheadAt ahead_at() {
  static const AheadAt at = [] {
    const char* v = getenv("SDCORE_AHEAD_AT");
    if (v && strcmp(v, "plan") == 0) return kAheadPlan;
    if (v && strcmp(v, "groupby") == 0) return kAheadGroupBy;
    return kAheadLookup;
  }();
  return at;
}

// The step loop with the chunk fetcher: each batch is the cursor row when it
// stays an orphan (fetched again after the writes: its Object may be new),
// then the rows the batch fetched but its steps did not read, then the next
// chunk, whose FileMetadata runs beside this batch's writes (as round 5's
// read-ahead) but no longer waits for its own fetch.
StepLoop run_steps_chunked(Library& db, uint64_t task_count, int32_t cursor, size_t batch_rows, const Fetch& fetch,
                           const MetadataFn& metadata, const GroupBy& group_by, const Fetch& fetch_ahead) {
  StepLoop L;
  L.cursor = cursor;
  const size_t cs = SDCAS_IDENTIFIER_CHUNK_SIZE;
  const size_t batch = std::max(cs, batch_rows);
  uint64_t steps_left = task_count;
  trace_mark();
  // a short first batch: the pipeline's fill is its FileMetadata alone (the
  // next chunk's runs while it is written)
  const size_t first_take = batch >= 8 * cs ? std::max(cs, batch / 8) : batch;
  std::vector<FilePathRow> rows = fetch(L.cursor, first_take);  // id >= cursor ORDER BY id (file_identifier_job.rs:296-319)
  trace_lap(JobTrace::kFetch);
  bool more = rows.size() == first_take;
  std::unique_ptr<ChunkFetcher> fetcher;
  if (more) fetcher = std::make_unique<ChunkFetcher>(fetch_ahead, rows.back().id, batch);
  trace_mark();
  std::vector<Result<FileMetadata>> md = metadata(rows);
  trace_lap(JobTrace::kMetadata);
  struct Ahead {
    ChunkFetcher::Chunk chunk;
    std::vector<Result<FileMetadata>> md;
  };
  while (steps_left) {
    if (rows.empty()) {
      L.ran_dry = true;
      break;
    }
    if (L.batches && rows[0].id == L.cursor) ++L.rereads;  // the cursor row is still an orphan
    sdcas_job_window w{};
    w.max_steps = steps_left;
    w.more = more;
    // a row to re-identify must sit in the batch's first step (identifier_step_db)
    {
      sdcas_job_window probe = w;
      const StepPlan plan = plan_steps(md, cs, probe);
      uint64_t cut = UINT64_MAX;
      for (size_t i = 0; i < rows.size(); ++i)
        if (plan.step[i] != UINT64_MAX && plan.step[i] > 0 && reidentified(rows[i], md[i]))
          cut = std::min(cut, plan.step[i]);
      if (cut != UINT64_MAX) w.max_steps = cut;
    }
    std::future<Ahead> next_md;
    const OnGrouped start_next = [&](const sdcas_job_window& done) {
      if (done.steps == 0 || done.steps >= steps_left || !fetcher) return;
      ChunkFetcher* f = fetcher.get();
      next_md = std::async(std::launch::async, [f, &metadata] {
        Ahead a;
        a.chunk = f->next();
        if (!a.chunk.err && !a.chunk.rows.empty()) a.md = metadata(a.chunk.rows);
        return a;
      });
    };
    const AheadAt at = ahead_at();
    auto [created, linked] = step_db(db, rows, md, group_by, &w, cs, at == kAheadPlan ? &start_next : nullptr,
                                     at == kAheadGroupBy ? &start_next : nullptr,
                                     at == kAheadLookup ? &start_next : nullptr);
    if (w.steps == 0) break;  // cannot happen: a batch of >= cs rows holds a whole step
    L.created += created;
    L.linked += linked;
    L.steps += w.steps;
    L.rereads += w.rereads;
    ++L.batches;
    steps_left -= std::min<uint64_t>(steps_left, w.steps);
    const size_t last = w.rows - 1;
    L.cursor = rows[last].id;
    if (!steps_left) break;
    // the next batch: the cursor row again if it stays an orphan, the rows
    // past it, the next chunk
    std::vector<FilePathRow> nrows;
    std::vector<Result<FileMetadata>> nmd;
    trace_mark();
    if (!md[last].ok() || !md[last].value().cas_id) {
      std::vector<FilePathRow> cur = fetch(L.cursor, 1);
      if (cur.size() == 1 && cur[0].id == L.cursor) {
        nrows.push_back(std::move(cur[0]));
        nmd.push_back(md[last]);  // the same file: its FileMetadata as this batch read it
      }
    }
    trace_lap(JobTrace::kFetch);
    for (size_t i = w.rows; i < rows.size(); ++i) {
      nrows.push_back(std::move(rows[i]));
      nmd.push_back(std::move(md[i]));
    }
    if (next_md.valid()) {
      trace_mark();
      Ahead a = next_md.get();
      trace_lap(JobTrace::kWaitAhead);
      if (a.chunk.err) std::rethrow_exception(a.chunk.err);
      more = a.chunk.full;
      if (!more) fetcher.reset();  // the fetcher has ended
      for (size_t i = 0; i < a.chunk.rows.size(); ++i) {
        nrows.push_back(std::move(a.chunk.rows[i]));
        nmd.push_back(std::move(a.md[i]));
      }
    } else if (!fetcher) {
      more = false;
    }
    rows = std::move(nrows);
    md = std::move(nmd);
  }
  return L;
}

StepLoop run_steps(Library& db, uint64_t task_count, int32_t cursor, size_t batch_rows, const Fetch& fetch,
                   const MetadataFn& metadata, const GroupBy& group_by, const Fetch* fetch_ahead = nullptr) {
  if (fetch_ahead && pipeline_enabled())
    return run_steps_chunked(db, task_count, cursor, batch_rows, fetch, metadata, group_by, *fetch_ahead);
  StepLoop L;
  L.cursor = cursor;
  const size_t cs = SDCAS_IDENTIFIER_CHUNK_SIZE;
  const size_t batch = std::max(cs, batch_rows);  // a batch holds at least one whole step
  uint64_t steps_left = task_count;
  std::vector<FilePathRow> rows = fetch(L.cursor, batch);  // id >= cursor ORDER BY id (file_identifier_job.rs:296-319)
  std::vector<Result<FileMetadata>> md;
  bool have_md = false;
  while (steps_left) {
    if (rows.empty()) {
      L.ran_dry = true;
      break;
    }
    trace_mark();
    if (!have_md) md = metadata(rows);
    trace_lap(JobTrace::kMetadata);
    if (L.batches && rows[0].id == L.cursor) ++L.rereads;  // the cursor row is still an orphan
    sdcas_job_window w{};
    w.max_steps = steps_left;
    w.more = rows.size() == batch;
    // a row to re-identify must sit in the batch's first step (identifier_step_db)
    {
      sdcas_job_window probe = w;
      const StepPlan plan = plan_steps(md, cs, probe);
      uint64_t cut = UINT64_MAX;
      for (size_t i = 0; i < rows.size(); ++i)
        if (plan.step[i] != UINT64_MAX && plan.step[i] > 0 && reidentified(rows[i], md[i]))
          cut = std::min(cut, plan.step[i]);
      if (cut != UINT64_MAX) w.max_steps = cut;
    }
    // The next batch is read while this one's Objects are written: the next
    // fetch (id >= the cursor) is the cursor row if it stays an orphan (an
    // error or no cas_id: nothing makes it whole) and then orphans past the
    // cursor, which this batch does not write. Those are fetched and their
    // FileMetadata computed on another thread after the group-by; the cursor
    // row is fetched again once the writes are done.
    std::vector<FilePathRow> next;
    using Ahead = std::pair<std::vector<FilePathRow>, std::vector<Result<FileMetadata>>>;
    std::future<Ahead> next_md;
    bool stays = false;
    int32_t next_cursor = 0;
    const OnGrouped prefetch = [&](const sdcas_job_window& done) {
      if (done.steps == 0 || done.steps >= steps_left) return;
      const size_t last = done.rows - 1;
      next_cursor = rows[last].id;
      stays = !md[last].ok() || !md[last].value().cas_id;
      std::vector<FilePathRow> head;
      if (stays) head.push_back(rows[last]);  // the same file; its row is re-read below
      const size_t take = batch - (stays ? 1 : 0);
      if (fetch_ahead) {
        // the fetch too runs beside this batch's writes (a second connection)
        next_md = std::async(std::launch::async, [&metadata, fetch_ahead, head = std::move(head), next_cursor, take] {
          Ahead a;
          a.first = (*fetch_ahead)(next_cursor + 1, take);
          std::vector<FilePathRow> ahead = head;
          ahead.insert(ahead.end(), a.first.begin(), a.first.end());
          if (!ahead.empty()) a.second = metadata(ahead);
          return a;
        });
        return;
      }
      next = fetch(next_cursor + 1, take);
      std::vector<FilePathRow> ahead = std::move(head);
      ahead.insert(ahead.end(), next.begin(), next.end());
      if (ahead.empty()) return;
      next_md = std::async(std::launch::async, [&metadata, ahead = std::move(ahead)] {
        return Ahead{{}, metadata(ahead)};
      });
    };
    auto [created, linked] = step_db(db, rows, md, group_by, &w, cs, &prefetch);
    if (w.steps == 0) break;  // cannot happen: a batch of `batch` >= cs rows holds a whole step
    L.created += created;
    L.linked += linked;
    L.steps += w.steps;
    L.rereads += w.rereads;
    ++L.batches;
    steps_left -= std::min<uint64_t>(steps_left, w.steps);
    L.cursor = rows[w.rows - 1].id;
    have_md = false;
    if (next_md.valid()) {
      trace_mark();
      Ahead got = next_md.get();
      trace_lap(JobTrace::kWaitAhead);
      if (fetch_ahead) next = std::move(got.first);
      auto ahead_md = std::move(got.second);
      if (ahead_md.empty()) {  // nothing past the cursor, nor a cursor row to read again
        if (steps_left) rows = fetch(L.cursor, batch);
        continue;
      }
      std::vector<FilePathRow> cur;
      if (stays) cur = fetch(L.cursor, 1);
      if (!stays || (cur.size() == 1 && cur[0].id == L.cursor)) {
        rows = std::move(cur);
        rows.insert(rows.end(), next.begin(), next.end());
        md = std::move(ahead_md);
        have_md = true;
        continue;
      }
    }
    trace_mark();
    if (steps_left) rows = fetch(L.cursor, batch);
    trace_lap(JobTrace::kFetch);
  }
  return L;
}
}  // namespace

FileIdentifierJobRunMetadata run_file_identifier_job_with(Library& db, const FileIdentifierJobInit& init,
                                                          const MetadataFn& metadata, const GroupBy& group_by) {
  FileIdentifierJobRunMetadata meta;
  const int32_t loc = init.location.id;
  const std::string& sub = init.sub_materialized_path;
  JobTrace trace;
  // init (file_identifier_job.rs:125-176)
  meta.total_orphan_paths = db.count_orphan_file_paths(loc, sub);
  if (meta.total_orphan_paths == 0) return meta;
  auto first = db.get_orphan_file_paths(loc, 0, sub, 1);
  meta.cursor = first.empty() ? 0 : first[0].id;
  const uint64_t task_count = (meta.total_orphan_paths + SDCAS_IDENTIFIER_CHUNK_SIZE - 1) / SDCAS_IDENTIFIER_CHUNK_SIZE;
  struct TraceScope {
    JobTrace* t;
    explicit TraceScope(JobTrace* x) : t(x) { g_trace = x->on ? x : nullptr; }
    ~TraceScope() {
      t->print();
      g_trace = nullptr;
    }
  } trace_scope(&trace);
  // the lookup index traded for a host map for the job's duration, restored
  // on every way out (Library::begin_bulk_identify)
  struct Bulk {
    Library& db;
    bool on;
    ~Bulk() {
      if (!on) return;
      trace_mark();
      try {
        db.end_bulk_identify();
        trace_lap(JobTrace::kIndex);
      } catch (...) {  // unwinding already; the index is rebuilt by the next bulk job or existing_objects
      }
    }
  } bulk{db, init.bulk_identify && db.begin_bulk_identify(meta.total_orphan_paths)};
  meta.bulk_identify = bulk.on;
  const Fetch ahead = [&](int32_t cursor, size_t take) {
    return db.get_orphan_file_paths_concurrent(loc, cursor, sub, take);
  };
  const bool concurrent = db.concurrent_orphan_reads();
  trace.lap(JobTrace::kInit);
  const StepLoop L = run_steps(
      db, task_count, meta.cursor, init.batch,
      [&](int32_t cursor, size_t take) { return db.get_orphan_file_paths(loc, cursor, sub, take); }, metadata,
      group_by, concurrent ? &ahead : nullptr);
  meta.total_objects_created = L.created;
  meta.total_objects_linked = L.linked;
  meta.steps = L.steps;
  meta.batches = L.batches;
  meta.rereads = L.rereads;
  meta.cursor = L.cursor;
  meta.early_finish = L.ran_dry;  // EarlyFinish (:203-209)
  return meta;
}

ShallowIdentifierReport shallow_file_identifier_with(Library& db, const Location& location, const std::string& dir,
                                                     size_t batch, const MetadataFn& metadata,
                                                     const GroupBy& group_by) {
  ShallowIdentifierReport rep;
  const std::string d = dir.empty() ? "/" : dir;  // materialized_path_for_children of the root
  rep.orphans = db.count_orphan_file_paths_in_dir(location.id, d);  // shallow.rs:62-66
  if (rep.orphans == 0) return rep;
  // find_first without ordering (shallow.rs:74-84): the lowest orphan id
  auto first = db.get_orphan_file_paths_in_dir(location.id, 0, d, 1);
  if (first.empty()) return rep;  // "another Job finishing first" (shallow.rs:81-83)
  const uint64_t task_count = (rep.orphans + SDCAS_IDENTIFIER_CHUNK_SIZE - 1) / SDCAS_IDENTIFIER_CHUNK_SIZE;
  // every step runs (shallow.rs:92-112): one that finds no rows changes
  // nothing, so the loop may stop at the first empty fetch
  const StepLoop L = run_steps(
      db, task_count, first[0].id, batch,
      [&](int32_t cursor, size_t take) { return db.get_orphan_file_paths_in_dir(location.id, cursor, d, take); },
      metadata, group_by);
  rep.steps = L.steps;
  rep.batches = L.batches;
  rep.rereads = L.rereads;
  rep.created = L.created;
  rep.linked = L.linked;
  rep.cursor = L.cursor;
  return rep;
}

static std::vector<Result<FileMetadata>> metadata_of(Engine& engine, const Location& location,
                                                     const std::vector<FilePathRow>& rows) {
  std::vector<std::pair<std::string, ObjectKind>> files(rows.size());
  std::vector<uint64_t> hints(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    files[i] = {full_path(location, rows[i]), rows[i].kind};
    hints[i] = rows[i].size_in_bytes;
  }
  return file_metadata_batch(engine, files, &hints);
}

static GroupBy gpu_group_by(Engine& engine) {
  return [&engine](const std::vector<uint64_t>& k, const std::vector<uint8_t>& h, const std::vector<int32_t>& st,
                   const std::vector<uint64_t>& e, sdcas_job_window& w) {
    return engine.dedup(k, h, st, SDCAS_IDENTIFIER_CHUNK_SIZE, e, &w);
  };
}

ShallowIdentifierReport shallow_file_identifier(Engine& engine, Library& db, const Location& location,
                                                const std::string& dir, size_t batch) {
  return shallow_file_identifier_with(
      db, location, dir, batch, [&](const std::vector<FilePathRow>& rows) { return metadata_of(engine, location, rows); },
      gpu_group_by(engine));
}

FileIdentifierJobRunMetadata run_file_identifier_job(Engine& engine, Library& db, const FileIdentifierJobInit& init) {
  return run_file_identifier_job_with(
      db, init, [&](const std::vector<FilePathRow>& rows) { return metadata_of(engine, init.location, rows); },
      gpu_group_by(engine));
}

// ---- object validator -----------------------------------------------------------------

ObjectValidatorReport run_object_validator_job(Engine& engine, Library& db, const ObjectValidatorJobInit& init) {
  ObjectValidatorReport rep;
  auto rows = db.file_paths_without_checksum(init.location.id, init.sub_materialized_path);
  rep.task_count = rows.size();
  const size_t batch = std::max<size_t>(1, init.batch);
  for (size_t lo = 0; lo < rows.size(); lo += batch) {
    const size_t hi = std::min(rows.size(), lo + batch);
    std::vector<std::string> paths;
    for (size_t i = lo; i < hi; ++i) paths.push_back(full_path(init.location, rows[i]));
    auto sums = engine.file_checksums(paths);
    db.begin_batch();
    for (size_t i = lo; i < hi; ++i) {
      const auto& r = sums[i - lo];
      if (!r.ok()) {  // validator_job.rs:154-156: the step fails with FileIO
        rep.error = r.error();
        db.end_batch();
        return rep;
      }
      db.set_integrity_checksum(rows[i].id, r.value());  // validator_job.rs:158-172
      ++rep.checksummed;
    }
    db.end_batch();
  }
  return rep;
}

}  // namespace sdcore
