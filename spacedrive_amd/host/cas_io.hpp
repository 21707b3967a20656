// cas_io.hpp — the host file I/O of libsdcas's path calls, GPU-free so that it
// is tested under ASan/UBSan and TSan on the CPU (tests/cpp/test_cas_io.cpp).
//
// The reads follow the reference exactly: generate_cas_id's
// (core/src/object/cas.rs:23-62 — fs::read of a file up to 100 KiB; else an
// 8 KiB header, four 10 KiB samples at 8192 + k * ((size - 16384) / 4) and
// an 8 KiB footer at EOF - 8192, each with read_exact's UnexpectedEof), and
// file_checksum's whole-content read (core/src/object/validation/hash.rs:15-21).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sdcas_io {

// per-item status of read_exact running out of file (tokio's UnexpectedEof;
// include/sdcas.h SDCAS_STATUS_UNEXPECTED_EOF)
constexpr int32_t kUnexpectedEof = 100001;

// staged messages start on 128-byte (L2/HBM line) boundaries
inline uint64_t align_line(uint64_t x) { return (x + 127) & ~127ull; }

// read_exact at `off` (tokio AsyncReadExt::read_exact): fill n bytes or fail
// with UnexpectedEof; returns 0 or a status
int pread_exact(int fd, uint8_t* dst, uint64_t n, uint64_t off);

// The O_DIRECT form of pread_exact for the big-file checksum path: `off`
// and `dst` 4 KiB aligned, the length read is n rounded up to 4 KiB (dst must
// have room), a read shorter than that ends at EOF; fails with UnexpectedEof
// when fewer than n bytes were there.
constexpr uint64_t kDirectAlign = 4096;
int pread_direct(int fd, uint8_t* dst, uint64_t n, uint64_t off);

// open(path) for reading, with O_DIRECT when `direct` and the filesystem
// accepts it (tmpfs and some overlays refuse it: then the page cache is
// used); *is_direct says which. Returns the fd or -errno.
int open_for_read(const char* path, bool direct, bool* is_direct);
// a path call begins: the reader threads' cached directory descriptors
// (open_for_read) are not reused past it
void new_path_epoch();
// close the calling thread's cached directory descriptor (if any)
void drop_dir_cache();

// Whole file into dst (capacity cap > expect, the size the indexer or a stat
// just saw); returns status, *len = bytes read; sets *overflow when the file
// holds at least cap bytes (it grew). A read that stops short exactly at
// `expect` is taken as EOF — one pread per unchanged file instead of a second
// one returning 0; shorter reads keep reading to EOF as fs::read does.
int read_whole(int fd, uint8_t* dst, uint64_t cap, uint64_t expect, uint64_t* len, bool* overflow);

// Bytes [off, off + n) of an O_DIRECT descriptor (any off and n): the 4 KiB
// blocks holding them are read into a per-thread aligned bounce buffer and
// the span copied to dst; *got = the bytes there were (fewer at EOF).
int read_span_direct(int fd, uint8_t* dst, uint64_t n, uint64_t off, uint64_t* got);

// read_whole with aligned (O_DIRECT) reads when `aligned`
int read_whole_any(int fd, bool aligned, uint8_t* dst, uint64_t cap, uint64_t expect, uint64_t* len,
                   bool* overflow);

// cas.rs:23-62 message of one file into dst (capacity cap >= the message
// length `size` predicts + 1). Returns status; *len = message length.
// *retry_len != 0 asks the caller to retry with a slot of that capacity (the
// file grew past `size` since it was indexed). `direct`: open with O_DIRECT
// (cold storage) where the filesystem takes it, every read then aligned
// through read_span_direct; the bytes and statuses are the same.
int read_cas_message(const char* path, uint64_t size, uint8_t* dst, uint64_t cap, uint64_t* len,
                     uint64_t* retry_len, bool direct = false);
// the same read pattern on an open descriptor (`aligned`: O_DIRECT reads)
int read_cas_message_fd(int fd, bool aligned, uint64_t size, uint8_t* dst, uint64_t cap, uint64_t* len,
                        uint64_t* retry_len);
// FileMetadata::new (file_identifier/mod.rs:48-96) of one file: open, the
// metadata as fstat of that descriptor (*size, *is_dir), then — unless a
// directory or empty (no cas_id: *len = 0) — its cas.rs message of that
// length into dst (capacity cap). *retry_len != 0: the message needs a slot
// of that capacity (the file is not the size the slot was planned for). An
// open refused where the metadata succeeds (no read permission) reports the
// metadata and, for a non-empty file, the open's errno; the reference never
// opens an empty file.
int read_file_metadata(const char* path, bool direct, uint8_t* dst, uint64_t cap, uint64_t* len,
                       uint64_t* retry_len, uint64_t* size, bool* is_dir);

// The next staging batch: items order[p], order[p+1], ... of `need` bytes
// each (line-aligned here) go to offsets in one slot of `cap` bytes and at
// most cap_n items; the first item always fits (a message larger than the
// slot gets a slot of its own). Returns q (items [p, q) taken) and fills
// offs[0 .. q-p) and *used.
size_t plan_batch(const uint64_t* need, const size_t* order, size_t p, size_t end, uint64_t cap, size_t cap_n,
                  std::vector<uint64_t>& offs, uint64_t* used);

// f(i) for i in [0, n) on up to `threads` threads (items claimed from a
// shared counter)
template <class F>
void parallel_for(uint32_t threads, size_t n, F f) {
  if (n == 0) return;
  threads = (uint32_t)std::max<size_t>(1, std::min<size_t>(threads, n));
  if (threads == 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& th : pool) th.join();
}

// The same on a pool of threads kept for the life of a context: `threads`
// workers in all, the calling thread being one of them (no thread is created
// per batch). run() is not reentrant; a context serialises its calls.
class WorkerPool {
 public:
  explicit WorkerPool(uint32_t threads);
  ~WorkerPool();
  WorkerPool(const WorkerPool&) = delete;
  WorkerPool& operator=(const WorkerPool&) = delete;
  uint32_t threads() const { return (uint32_t)workers_.size() + 1; }
  template <class F>
  void run(size_t n, F f) {
    if (n == 0) return;
    if (workers_.empty() || n == 1) {
      for (size_t i = 0; i < n; ++i) f(i);
      return;
    }
    std::function<void(size_t)> fn(f);
    dispatch(n, &fn);
  }

 private:
  void dispatch(size_t n, const std::function<void(size_t)>* fn);
  void drain();
  void loop();
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable go_, done_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  size_t active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace sdcas_io
