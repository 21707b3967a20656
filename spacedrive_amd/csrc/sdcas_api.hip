// sdcas_api.hip — the C ABI of include/sdcas.h: context, staging, file I/O
// and the batch calls that sd-core's Rust host binds.
//
// Host work here is exactly what the reference does around the hash
// (core/src/object/cas.rs:23-62, core/src/object/validation/hash.rs:11-25):
// the same reads at the same offsets, with the same error kinds — but into a
// pinned staging buffer laid out as device messages, after which one H2D
// copy and one kernel sequence hash the whole batch. There is no CPU hashing
// path: every digest this library returns comes from the HIP kernels.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <chrono>
#include <memory>
#include <vector>

#include "../../include/sdcas.h"
#include "../../include/sdcas_bench.h"
#include "../host/cas_io.hpp"
#include "b3_batch.h"
#include "dist_dedup.h"
#include "synth.h"

using namespace sdcas;

namespace {

// file I/O with the reference's read pattern (GPU-free, in
// spacedrive_amd/host/cas_io.cpp: tested under ASan / UBSan / TSan by
// tests/cpp/test_cas_io.cpp)
using sdcas_io::open_for_read;
using sdcas_io::plan_batch;
using sdcas_io::pread_direct;
using sdcas_io::pread_exact;
using sdcas_io::read_cas_message;
using sdcas_io::read_whole;
using sdcas_io::read_whole_any;

constexpr uint64_t kMin = SDCAS_MINIMUM_FILE_SIZE;  // cas.rs:15 (the reads themselves: host/cas_io.cpp)
constexpr uint64_t kSlack = 64;  // readable bytes kept after every message

// staged messages start on 128-byte (L2/HBM line) boundaries
inline uint64_t align16(uint64_t x) { return sdcas_io::align_line(x); }
inline uint64_t chunks_of(uint64_t len) { return len == 0 ? 1 : (len + 1023) / 1024; }

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 16);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// One pinned staging slot: message bytes, per-message metadata and results,
// their device twins, and the event that fences the slot's GPU work.
struct Slot {
  uint8_t* h = nullptr;   // pinned message bytes
  size_t h_cap = 0;
  bool h_mapped = false;  // h is an mmap'd, hipHostRegister'ed range (SDCAS_STAGING_THP)
  uint64_t* hm = nullptr;  // pinned: offs[cap_n] | lens[cap_n] | results (32 B per message)
  size_t cap_n = 0;
  DevBuf<uint8_t> d_blob;
  DevBuf<uint64_t> d_meta;  // offs | lens (or piece descriptors)
  DevBuf<uint8_t> d_res;
  hipEvent_t ev = nullptr;
  hipEvent_t h2d = nullptr;  // the slot's uploads done (on the copy stream)
  bool busy = false, res32 = false;
  size_t n = 0;
  uint64_t used = 0, chunks = 0;
  uint64_t content = 0;  // input bytes whose results this slot's batch makes final (progress)
  std::vector<size_t> idx;  // caller index of message k
  const uint8_t* src = nullptr;  // message bytes DMA'd from here instead of h (a pinned caller buffer)
  bool blob_uploaded = false;    // the bytes went up in parts while the slot was being read (slot_submit skips them)
  uint64_t* offs() { return hm; }
  uint64_t* lens() { return hm + cap_n; }
  uint8_t* res() { return reinterpret_cast<uint8_t*>(hm + 2 * cap_n); }
};

// Small host arrays (the device stream's message and segment descriptors)
// sent to the device in stream order without a host wait: each put copies
// into the next of kN page-locked buffers and enqueues the upload from it; a
// buffer is reused only after the event recorded behind its last upload.
struct HostStage {
  static constexpr int kN = 4;
  uint8_t* h[kN] = {};
  size_t cap[kN] = {};
  hipEvent_t ev[kN] = {};
  bool recorded[kN] = {};
  int next = 0;
  hipError_t put(const void* src, size_t bytes, void* d_dst, hipStream_t st) {
    if (!bytes) return hipSuccess;
    const int i = next;
    next = (next + 1) % kN;
    hipError_t e;
    if (recorded[i] && (e = hipEventSynchronize(ev[i]))) return e;
    recorded[i] = false;
    if (bytes > cap[i]) {
      if (h[i]) (void)hipHostFree(h[i]);
      h[i] = nullptr;
      cap[i] = 0;
      const size_t want = std::max<size_t>(bytes + bytes / 4, 64 << 10);
      if ((e = hipHostMalloc(&h[i], want, hipHostMallocDefault))) return e;
      cap[i] = want;
    }
    if (!ev[i] && (e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming))) return e;
    memcpy(h[i], src, bytes);
    if ((e = hipMemcpyAsync(d_dst, h[i], bytes, hipMemcpyHostToDevice, st))) return e;
    if ((e = hipEventRecord(ev[i], st))) return e;
    recorded[i] = true;
    return hipSuccess;
  }
  void release() {
    for (int i = 0; i < kN; ++i) {
      if (recorded[i]) (void)hipEventSynchronize(ev[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      if (h[i]) (void)hipHostFree(h[i]);
      h[i] = nullptr, ev[i] = nullptr, cap[i] = 0, recorded[i] = false;
    }
  }
};

}  // namespace

struct sdcas_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // staging slots' host-to-device copies
  std::string err;
  std::mutex mu;
  // reader threads: 16 unless the machine has fewer CPUs (C-ABI probe, C2
  // files from the page cache, profiles/r02_latency_threads.json: 16 against
  // 8 cut 100 / 1000 / 10000-file calls by 8 / 17 / 18 %; 32 no better)
  uint32_t io_threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  static constexpr uint32_t kMaxIoThreads = 256;
  std::unique_ptr<sdcas_io::WorkerPool> pool;  // io_threads readers (the calling thread is one)
  uint64_t staging_bytes = 256ull << 20;
  bool direct_io = false;  // SDCAS_OPT_DIRECT_IO: big-file checksum reads bypass the page cache

  BatchWorkspace ws;
  DevBuf<uint64_t> ws_S, ws_total, ws_soffs, ws_slens;
  DevBuf<uint32_t> ws_tile_first, ws_nodes, ws_perm, ws_sort_keys;
  DevBuf<uint8_t> ws_scan;

  // host-API device buffers
  DevBuf<uint8_t> d_out32;
  DevBuf<FileDesc> d_files;
  DevBuf<uint32_t> d_file_nodes;
  Slot slots[2];  // double-buffered pinned staging (host fills one, GPU hashes the other)

  // sdcas_dedup's device copies of the caller's host arrays
  DevBuf<uint64_t> dd_keys, dd_ekeys, dd_ids;
  DevBuf<uint8_t> dd_has;
  DevBuf<int32_t> dd_status;
  DevBuf<int64_t> dd_link;
  DevBuf<unsigned long long> dd_counts;

  // multi-GPU dedup stages
  DistWs dist;

  // device-resident big-message stream (sdcas_dev_stream_*)
  std::vector<FileDesc> sm_files;
  DevBuf<FileDesc> sm_d_files;
  DevBuf<uint32_t> sm_nodes;
  DevBuf<PieceDesc> sm_pieces;
  DevBuf<SegDesc> sm_segs;
  HostStage sm_stage;             // descriptor uploads without a host wait
  bool sm_active = false;
  bool sm_begin_pending = false;  // stream_begin's descriptor upload and node-list clear, enqueued by the next call
  uint64_t sm_node_bytes = 0;
  DevBuf<uint32_t> piece_ctr;  // the persistent piece kernels' work counter
  DevBuf<uint32_t> piece_l4;   // piece variant 19's level-4 nodes (kPieceL4Words per piece)
  int piece_variant = -1;

  // Every call that enqueues work on the context's device scratch (the
  // workspaces above) may name its own stream. The scratch is shared, so a
  // call first makes its stream wait for the previous call's work (the event
  // recorded at the end of that call), then records the event anew: calls on
  // one context are ordered on the device as they are on the host, whatever
  // streams they name.
  hipEvent_t scratch_ev = nullptr;
  hipStream_t scratch_st = nullptr;
  bool scratch_pending = false;
  // sdcas_dev_bind_stream: streams whose identity the caller named
  std::vector<std::pair<hipStream_t, uint64_t>> bound;
  uint64_t scratch_token = 0;  // the token of the stream the last call used (0: none)
  bool scratch_recorded = true;  // scratch_ev marks the last call's end (else: record it first)
  uint64_t token_of(hipStream_t st) const {
    for (const auto& b : bound)
      if (b.first == st) return b.second;
    return 0;
  }
  uint32_t upload_parts = 4;  // sdcas_cas_ids: a lone slot's reads and upload overlapped in this many parts (0/1: off)
  bool plan_small = true;      // small batches planned on the host (SDCAS_PLAN_SMALL=0: on the device)
  bool small_direct = true;    // such a batch: metadata behind its bytes, results written to pinned memory (slot_submit)

  // progress / cancellation of the path APIs (sdcas_options, sdcas_set_progress)
  sdcas_progress_fn progress = nullptr;
  void* progress_user = nullptr;
  const volatile int32_t* cancel = nullptr;

  // profiling
  bool profile = false;
  std::vector<hipEvent_t> ev_free;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_leaf, ev_all;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    return fail(e == hipErrorOutOfMemory ? SDCAS_E_OOM : SDCAS_E_HIP, "%s: %s", what, hipGetErrorString(e));
  }
  // before enqueuing on st: wait for the previous call's use of the scratch
  // — unless it ran on this same stream, which only a bound token can tell
  // (a handle value may have been reused by a new stream after the caller
  // destroyed the old one)
  hipError_t fence_in(hipStream_t st) {
    if (!scratch_pending) return hipSuccess;
    if (st == scratch_st && scratch_token && token_of(st) == scratch_token) return hipSuccess;
    hipError_t e = scratch_event();
    return e ? e : hipStreamWaitEvent(st, scratch_ev, 0);
  }
  // after enqueuing on st. On a bound stream the event is recorded only when
  // something needs it — a call on another stream, a host wait for the
  // scratch — and then on that stream, behind everything enqueued on it so
  // far: a recorded event is a barrier packet that idled the GPU ~6-8 us
  // between two calls on the step's stream (the C5 step's kernel trace)
  hipError_t fence_out(hipStream_t st) {
    scratch_st = st;
    scratch_token = token_of(st);
    scratch_pending = true;
    scratch_recorded = false;
    return scratch_token ? hipSuccess : scratch_event();
  }
  // the scratch event, recorded on the last call's stream if it was not yet
  hipError_t scratch_event() {
    if (scratch_recorded) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!scratch_ev && (e = hipEventCreateWithFlags(&scratch_ev, hipEventDisableTiming))) return e;
    if ((e = hipEventRecord(scratch_ev, scratch_st))) return e;
    scratch_recorded = true;
    return hipSuccess;
  }
  // the host waits until no enqueued call still uses the scratch
  hipError_t scratch_sync() {
    if (!scratch_pending) return hipSuccess;
    hipError_t e = scratch_event();
    return e ? e : hipEventSynchronize(scratch_ev);
  }
  bool cancelled() const { return cancel && __atomic_load_n(cancel, __ATOMIC_ACQUIRE) != 0; }
  void report(uint64_t done, uint64_t total) {
    if (progress) progress(progress_user, done, total);
  }
  hipEvent_t event() {
    if (!ev_free.empty()) {
      hipEvent_t e = ev_free.back();
      ev_free.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
};

namespace {

int reserve_ws(sdcas_ctx* c, size_t max_msgs, uint64_t max_chunks) {
  hipError_t e;
  // the chunk scan takes an int count (hipcub)
  if (max_msgs > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "batch of %zu messages exceeds 2^31 - 1", max_msgs);
  if ((e = c->ws_S.ensure(max_msgs + 1))) return c->hip_fail(e, "workspace S");
  // room for the quad layout's padding too: < 4 dead slots per message (of
  // as many messages as the workspace takes)
  // (rounded up, +3: cap_chunks below comes out >= max_chunks, so that
  // slots_prepare's check holds on the next call instead of re-reserving)
  const uint64_t tiles = (max_chunks + 3 * (uint64_t)(c->ws_S.cap - 1) + 8 + kTile - 1) / kTile + 3;
  // tile_first also serves the small-batch kernel's tiles (kSmallTile slots)
  const uint64_t small_tiles = (std::min<uint64_t>(max_chunks, kSmallSlots) + kSmallTile - 1) / kSmallTile + 3;
  if ((e = c->ws_total.ensure(4))) return c->hip_fail(e, "workspace total");
  if ((e = c->ws_tile_first.ensure(std::max<uint64_t>(tiles, small_tiles))))
    return c->hip_fail(e, "workspace tile_first");
  if ((e = c->ws_nodes.ensure(8 * (tiles * kTile)))) return c->hip_fail(e, "workspace nodes");
  size_t tb = batch_scan_temp_bytes((uint32_t)std::max<size_t>(max_msgs, 1));
  if ((e = c->ws_scan.ensure(tb))) return c->hip_fail(e, "workspace scan");
  if ((e = c->ws_perm.ensure(max_msgs + 1)) || (e = c->ws_soffs.ensure(max_msgs + 1)) ||
      (e = c->ws_slens.ensure(max_msgs + 1)) || (e = c->ws_sort_keys.ensure(sort_key_words(max_msgs + 1))))
    return c->hip_fail(e, "workspace sort");
  c->ws.S = c->ws_S.p;
  c->ws.total = c->ws_total.p;
  c->ws.tile_first = c->ws_tile_first.p;
  c->ws.nodes = c->ws_nodes.p;
  c->ws.scan_tmp = c->ws_scan.p;
  c->ws.scan_tmp_bytes = c->ws_scan.cap;
  c->ws.perm = c->ws_perm.p;
  c->ws.soffs = c->ws_soffs.p;
  c->ws.slens = c->ws_slens.p;
  c->ws.cap_msgs =
      (uint32_t)std::min<size_t>({c->ws_S.cap - 1, c->ws_perm.cap - 1, c->ws_soffs.cap - 1, c->ws_slens.cap - 1});
  c->ws.sort_keys = c->ws_sort_keys.p;
  // every tile the leaf kernel may touch needs a tile_first entry and its node slots
  c->ws.cap_slots = std::min<uint64_t>((c->ws_tile_first.cap - 1) * kTile, c->ws_nodes.cap / 8 - 2 * kTile);
  c->ws.cap_small_tiles = c->ws_tile_first.cap;
  const uint64_t pad = 3 * (uint64_t)(c->ws_S.cap - 1) + 8;
  c->ws.cap_chunks = c->ws.cap_slots > pad ? c->ws.cap_slots - pad : 0;
  return SDCAS_OK;
}

// Enqueue the hash of n device messages (the one launch sequence every API
// ends in), with optional HIP-event profiling of the leaf kernel.
int launch_batch(sdcas_ctx* c, const uint8_t* blob, const uint64_t* offs, const uint64_t* lens, uint32_t n,
                 uint8_t* out32, uint64_t* keys, hipStream_t st, uint64_t max_chunks = 0,
                 const BatchPlan* plan = nullptr) {
  hipError_t e;
  if (c->profile) {
    hipEvent_t a = c->event(), b = c->event(), la = c->event(), lb = c->event();
    (void)hipEventRecord(a, st);
    e = batch_hash(c->ws, blob, offs, lens, n, out32, keys, st, max_chunks, la, lb, plan);
    (void)hipEventRecord(b, st);
    c->ev_all.push_back({a, b});
    c->ev_leaf.push_back({la, lb});
  } else {
    e = batch_hash(c->ws, blob, offs, lens, n, out32, keys, st, max_chunks, nullptr, nullptr, plan);
  }
  if (e) return c->hip_fail(e, "batch_hash");
  return SDCAS_OK;
}

// ---- double-buffered pinned staging ------------------------------------------
//
// Host work (file reads, or copies out of the caller's buffer) fills one
// pinned slot while the GPU copies and hashes the other: each slot's H2D,
// kernels and D2H are enqueued on the context stream and fenced by the slot's
// event, which is waited for only when the slot is about to be refilled.

// The message slots are anonymous mappings advised to transparent huge
// pages and then pinned (hipHostRegister): the readers' page-cache copies
// into a slot walk 2 MiB pages instead of hipHostMalloc's 4 KiB ones
// (profiles/r05_staging_thp_ab.json). A mapping or registration that fails
// falls back to hipHostMalloc; SDCAS_STAGING_THP=0 always takes it (A/B).
static bool staging_thp() {
  static const bool on = [] {
    const char* v = getenv("SDCAS_STAGING_THP");
    return !(v && strcmp(v, "0") == 0);
  }();
  return on;
}

static void free_staging(Slot& s) {
  if (!s.h) return;
  if (s.h_mapped) {
    (void)hipHostUnregister(s.h);
    munmap(s.h, s.h_cap);
  } else {
    (void)hipHostFree(s.h);
  }
  s.h = nullptr;
  s.h_cap = 0;
  s.h_mapped = false;
}

int slot_prepare(sdcas_ctx* c, Slot& s, uint64_t bytes, size_t n) {
  hipError_t e;
  if (bytes + kSlack > s.h_cap) {
    free_staging(s);
    const size_t want = bytes + kSlack;
    if (staging_thp()) {
      const size_t huge = 2u << 20, len = (want + huge - 1) / huge * huge;
      void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p != MAP_FAILED) {
        (void)madvise(p, len, MADV_HUGEPAGE);
        if (hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess) {
          s.h = static_cast<uint8_t*>(p);
          s.h_cap = len;
          s.h_mapped = true;
        } else {
          (void)hipGetLastError();  // the fallback below; not this call's error
          munmap(p, len);
        }
      }
    }
    if (!s.h) {
      if ((e = hipHostMalloc(&s.h, want, hipHostMallocDefault))) return c->hip_fail(e, "pinned staging");
      s.h_cap = want;
    }
  }
  if (n > s.cap_n) {
    if (s.hm) (void)hipHostFree(s.hm);
    s.hm = nullptr;
    s.cap_n = 0;
    const size_t want = std::max<size_t>(n, 1024);
    // offs[cap_n] | lens[cap_n] | results (32 B per message)
    if ((e = hipHostMalloc(&s.hm, 48 * want, hipHostMallocDefault))) return c->hip_fail(e, "pinned metadata");
    s.cap_n = want;
  }
  if ((e = s.d_blob.ensure(s.h_cap)) || (e = s.d_meta.ensure(2 * s.cap_n)) || (e = s.d_res.ensure(32 * s.cap_n)))
    return c->hip_fail(e, "device staging");
  if (!s.ev && (e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming))) return c->hip_fail(e, "event");
  if (!s.h2d && (e = hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming))) return c->hip_fail(e, "event");
  return SDCAS_OK;
}

void slot_release(Slot& s) {
  free_staging(s);
  if (s.hm) (void)hipHostFree(s.hm);
  s.hm = nullptr;
  s.cap_n = 0;
  s.d_blob.release();
  s.d_meta.release();
  s.d_res.release();
  if (s.ev) (void)hipEventDestroy(s.ev);
  if (s.h2d) (void)hipEventDestroy(s.h2d);
  s.ev = s.h2d = nullptr;
}

// Both slots sized for `cap` staging bytes, and the kernel workspace for the
// largest batch such a slot can hold, so that no buffer is reallocated while
// the other slot's work is in flight.
int slots_prepare(sdcas_ctx* c, uint64_t cap, size_t cap_n) {
  int rc;
  for (Slot& s : c->slots)
    if ((rc = slot_prepare(c, s, cap, cap_n))) return rc;
  if (cap_n > c->ws.cap_msgs || cap / 1024 + cap_n > c->ws.cap_chunks) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e) return c->hip_fail(e, "sync");
    return reserve_ws(c, std::max<size_t>(cap_n, c->ws.cap_msgs),
                      std::max<uint64_t>(cap / 1024 + cap_n, c->ws.cap_chunks));
  }
  return SDCAS_OK;
}

// While the other slot's batch is in flight, a slot's host-to-device copies
// run on the context's copy stream, so that they overlap that batch's kernels
// on the compute stream (PCIe and the CUs work at once: the path calls are
// bound by the copy); the compute stream waits for them before this slot's
// kernels. With nothing to overlap (a call's first or only slot) they go on
// the compute stream itself: the event and the cross-stream wait would only
// add latency. Refilling a slot waits for its previous batch on the host
// first (slot_complete), so a copy never lands under kernels still reading
// the slot.
template <class Copies>
hipError_t slot_upload(sdcas_ctx* c, Slot& s, Copies copies) {
  const Slot& other = &s == &c->slots[0] ? c->slots[1] : c->slots[0];
  if (!other.busy) return copies(c->stream);
  hipError_t e;
  if ((e = copies(c->copy_stream)) || (e = hipEventRecord(s.h2d, c->copy_stream))) return e;
  return hipStreamWaitEvent(c->stream, s.h2d, 0);
}

// Enqueue the slot's batch: s.n messages at s.offs()/s.lens() in s.h (s.used
// bytes, s.chunks chunks); results land in s.res() (digests if res32, else
// cas keys) once s.ev has fired.
int slot_submit(sdcas_ctx* c, Slot& s, bool res32) {
  s.res32 = res32;
  const bool uploaded = s.blob_uploaded;  // this batch's bytes only: the flag never outlives its submit
  s.blob_uploaded = false;
  if (!s.n) return SDCAS_OK;
  int rc;
  hipStream_t st = c->stream;
  hipError_t e;
  if (s.n > c->ws.cap_msgs || s.chunks > c->ws.cap_chunks) {
    // growing the kernel workspace frees buffers the other slot's kernels may
    // still be using: drain the stream first (rare: slots are pre-reserved)
    if ((e = hipStreamSynchronize(st))) return c->hip_fail(e, "sync");
    if ((rc = reserve_ws(c, std::max<size_t>(s.n, c->ws.cap_msgs), std::max<uint64_t>(s.chunks, c->ws.cap_chunks))))
      return rc;
  }
  // offsets and lengths in one copy: the lengths are moved up behind the
  // offsets when they fit there (each small copy is a blit kernel of its own)
  const bool packed = 2 * s.n <= s.cap_n;
  if (packed) memcpy(s.hm + s.n, s.lens(), 8 * s.n);
  // A batch for the small kernel in caller order is planned here and its
  // plan goes up behind the lengths in the same copy: the scan, k_tile_first
  // and (when no message crosses a tile) k_finish_t are not launched.
  uint64_t meta_words = packed ? 2 * s.n : s.n;
  const uint64_t plan_tiles = s.chunks / kSmallTile + 2;
  const uint64_t plan_words = s.n + (plan_tiles + 1) / 2 + 4;
  const bool use_plan = c->plan_small && packed && s.n < kSortMinMsgs && s.chunks <= c->ws.small_slots &&
                        2 * s.n + plan_words <= s.cap_n;
  if (use_plan) meta_words = 2 * s.n + plan_words;
  // Round 6, a small planned batch read into the slot (the latency-bound
  // calls: a lone file of the watcher or of browse): its metadata words go up
  // behind its bytes in the SAME copy (at a 256-byte offset past them, inside
  // the slot's capacity), and the kernels write the results straight into the
  // slot's pinned result words (device-visible host memory) instead of a
  // device buffer and a download. Two copies (and their API calls) fewer;
  // the event the host waits on follows the kernels, so their writes to
  // host memory are visible when it fires. SDCAS_SMALL_DIRECT=0: off (A/B).
  const uint64_t moff = (s.used + 255) & ~uint64_t(255);
  const bool direct = c->small_direct && use_plan && !uploaded && !s.src &&
                      moff + 8 * meta_words + kSlack <= std::min<uint64_t>(s.h_cap, s.d_blob.cap);
  uint64_t* dm = direct ? reinterpret_cast<uint64_t*>(s.d_blob.p + moff) : s.d_meta.p;
  const uint64_t* d_lens = dm + (packed ? s.n : s.cap_n);
  BatchPlan plan;
  if (use_plan) {
    uint64_t* hS = s.hm + 2 * s.n;
    uint32_t* htf = reinterpret_cast<uint32_t*>(hS + s.n);
    uint64_t* htot = hS + s.n + (plan_tiles + 1) / 2;
    batch_plan_host(s.lens(), (uint32_t)s.n, kSmallTile, c->ws.cap_slots, hS, htf, htot, &plan.crossing);
    plan.S = dm + 2 * s.n;
    plan.tile_first = reinterpret_cast<const uint32_t*>(plan.S + s.n);
    plan.total = dm + 2 * s.n + s.n + (plan_tiles + 1) / 2;
    plan.tile = kSmallTile;
  }
  if (direct) memcpy(s.h + moff, s.hm, 8 * meta_words);
  if ((e = slot_upload(c, s, [&](hipStream_t cs) {
         hipError_t r;
         if (direct) return hipMemcpyAsync(s.d_blob.p, s.h, moff + 8 * meta_words, hipMemcpyHostToDevice, cs);
         if ((!uploaded && (r = hipMemcpyAsync(s.d_blob.p, s.src ? s.src : s.h, s.used, hipMemcpyHostToDevice, cs))) ||
             (r = hipMemcpyAsync(s.d_meta.p, s.hm, 8 * meta_words, hipMemcpyHostToDevice, cs)))
           return r;
         return packed ? hipSuccess
                       : hipMemcpyAsync(s.d_meta.p + s.cap_n, s.hm + s.cap_n, 8 * s.n, hipMemcpyHostToDevice, cs);
       })))
    return c->hip_fail(e, "H2D");
  uint8_t* res = direct ? s.res() : s.d_res.p;
  if ((rc = launch_batch(c, s.d_blob.p, dm, d_lens, (uint32_t)s.n, res32 ? res : nullptr,
                         res32 ? nullptr : reinterpret_cast<uint64_t*>(res), st, s.chunks,
                         use_plan ? &plan : nullptr)))
    return rc;
  if ((!direct && (e = hipMemcpyAsync(s.res(), s.d_res.p, (res32 ? 32 : 8) * s.n, hipMemcpyDeviceToHost, st))) ||
      (e = hipEventRecord(s.ev, st)))
    return c->hip_fail(e, "D2H");
  s.busy = true;
  return SDCAS_OK;
}

// Progress of one path call: bytes of input whose results are final.
struct Progress {
  sdcas_ctx* c;
  uint64_t total = 0, done = 0;
  void add(uint64_t bytes) {
    done += bytes;
    c->report(done, total);
  }
};

// Wait for the slot's batch, hand message k's result to sink(k, ptr) and
// report the slot's input bytes as done.
template <class Sink>
int slot_complete(sdcas_ctx* c, Slot& s, Sink sink, Progress* pr = nullptr) {
  if (!s.busy) return SDCAS_OK;
  s.busy = false;
  hipError_t e = hipEventSynchronize(s.ev);
  if (e) return c->hip_fail(e, "batch");
  for (size_t k = 0; k < s.n; ++k) sink(k, s.res() + (s.res32 ? 32 : 8) * k);
  if (pr) pr->add(s.content);
  return SDCAS_OK;
}

// Big messages (> 1 MiB) from host memory: 1 MiB pieces streamed through the
// two staging slots (one window filled while the GPU hashes the other). A
// window's pieces are filled by the I/O threads in parallel (several reads in
// flight: what cold storage needs, and page-cache copies scale with threads
// too); `fill(k, dst, off, len)` provides bytes [off, off+len) of item k and
// returns a status (0 ok). Pieces sit at 4 KiB-aligned window offsets (the
// O_DIRECT rule; the device needs 16 B). Digests go to
// out32_host[32 * out_index]. Cancellation is checked once per window: items
// whose every piece was submitted by then are finished, the rest get
// SDCAS_STATUS_CANCELLED and *cancelled is set.
struct BigItem {
  uint64_t len;
  uint64_t out_index;
};

inline uint64_t align_page(uint64_t x) { return (x + sdcas_io::kDirectAlign - 1) & ~(sdcas_io::kDirectAlign - 1); }

template <class Fill>
int run_big(sdcas_ctx* c, const std::vector<BigItem>& items, uint8_t* out32_host, Fill fill, int32_t* status,
            Progress& pr, bool* cancelled) {
  *cancelled = false;
  if (items.empty()) return SDCAS_OK;
  hipError_t e;
  int rc;
  const uint64_t piece_bytes = 1024ull * kTile;
  const uint64_t window = std::max<uint64_t>(piece_bytes, (c->staging_bytes / piece_bytes) * piece_bytes);
  const size_t max_pieces = (size_t)(window / piece_bytes);
  for (Slot& s : c->slots)
    if ((rc = slot_prepare(c, s, window, 2 * max_pieces))) return rc;
  std::vector<FileDesc> files(items.size());
  uint64_t nodes = 0;
  for (size_t i = 0; i < items.size(); ++i) {
    files[i].C = chunks_of(items[i].len);
    files[i].node_base = nodes;
    files[i].out_index = i;
    nodes += bigfile_node_count(files[i].C);
  }
  if ((e = c->d_file_nodes.ensure(8 * nodes + 8))) return c->hip_fail(e, "file nodes");
  if ((e = c->d_files.ensure(items.size()))) return c->hip_fail(e, "file descs");
  if ((e = c->d_out32.ensure(32 * items.size()))) return c->hip_fail(e, "device digests");
  if ((e = c->piece_ctr.ensure(1))) return c->hip_fail(e, "piece counter");
  if ((e = c->piece_l4.ensure(kPieceL4Words * 2 * max_pieces))) return c->hip_fail(e, "piece level-4 nodes");
  hipStream_t st = c->stream;
  int cur = 0;
  struct Job {
    size_t item;
    uint64_t off, dst;
    uint32_t len;
  };
  std::vector<Job> jobs;
  std::vector<int32_t> jst;
  uint64_t used = 0, content = 0;
  std::vector<int32_t> item_st(items.size(), 0);
  auto wait_slot = [&](Slot& s) -> int {
    if (!s.busy) return SDCAS_OK;
    s.busy = false;
    hipError_t ee = hipEventSynchronize(s.ev);
    if (ee) return c->hip_fail(ee, "piece window");
    pr.add(s.content);
    return SDCAS_OK;
  };
  // fill the window's pieces (in parallel), then copy and hash them
  auto flush = [&]() -> int {
    if (jobs.empty()) return SDCAS_OK;
    Slot& s = c->slots[cur];
    jst.assign(jobs.size(), 0);
    c->pool->run(jobs.size(), [&](size_t k) {
      const Job& jb = jobs[k];
      jst[k] = fill(jb.item, s.h + jb.dst, jb.off, jb.len);
    });
    PieceDesc* hp = reinterpret_cast<PieceDesc*>(s.hm);
    for (size_t k = 0; k < jobs.size(); ++k) {
      if (jst[k] && !item_st[jobs[k].item]) item_st[jobs[k].item] = jst[k];
      PieceDesc pd{};
      pd.off = jobs[k].dst;
      pd.j0 = jobs[k].off / 1024;
      pd.node_base = files[jobs[k].item].node_base;
      pd.len = jobs[k].len;
      hp[k] = pd;  // a failed item's pieces are hashed too: its digest is never returned
    }
    PieceDesc* dp = reinterpret_cast<PieceDesc*>(s.d_meta.p);
    if (kPieceL4Words * jobs.size() > c->piece_l4.cap)  // a window holds at most 2 pieces per MiB
      return c->fail(SDCAS_E_CAPACITY, "piece window: %zu pieces", jobs.size());
    hipError_t ee;
    if ((ee = slot_upload(c, s, [&](hipStream_t cs) {
           hipError_t r = hipMemcpyAsync(s.d_blob.p, s.h, used, hipMemcpyHostToDevice, cs);
           return r ? r : hipMemcpyAsync(dp, hp, sizeof(PieceDesc) * jobs.size(), hipMemcpyHostToDevice, cs);
         })))
      return c->hip_fail(ee, "H2D pieces");
    if ((ee = piece_hash(s.d_blob.p, dp, (uint32_t)jobs.size(), c->d_file_nodes.p, c->piece_ctr.p, c->piece_l4.p,
                         c->piece_variant,
                         st)))
      return c->hip_fail(ee, "piece_hash");
    if ((ee = hipEventRecord(s.ev, st))) return c->hip_fail(ee, "event");
    s.busy = true;
    s.content = content;
    cur ^= 1;
    jobs.clear();
    used = 0;
    content = 0;
    return wait_slot(c->slots[cur]);  // the next window's buffers are free again
  };
  if ((rc = wait_slot(c->slots[cur]))) return rc;
  size_t complete = items.size();  // items [0, complete) have every piece submitted
  for (size_t i = 0; i < items.size() && !*cancelled; ++i) {
    const uint64_t len = items[i].len;
    for (uint64_t off = 0; off < len && !item_st[i]; off += piece_bytes) {
      const uint32_t pl = (uint32_t)std::min<uint64_t>(piece_bytes, len - off);
      if (used + align_page(pl) > window) {
        if ((rc = flush())) return rc;
        if (c->cancelled()) {
          *cancelled = true;
          complete = i;  // item i has pieces left (or none submitted yet): not complete
          break;
        }
      }
      jobs.push_back({i, off, used, pl});
      used += align_page(pl);
      content += pl;
    }
  }
  if (*cancelled) {
    jobs.clear();  // pieces of an incomplete item are never hashed
    used = content = 0;
  }
  if ((rc = flush())) return rc;
  for (Slot& s : c->slots)
    if ((rc = wait_slot(s))) return rc;
  for (size_t i = 0; i < items.size(); ++i)
    if (status && item_st[i] && !status[items[i].out_index]) status[items[i].out_index] = item_st[i];
  const size_t nf = complete;
  if (nf) {
    if ((e = hipMemcpyAsync(c->d_files.p, files.data(), sizeof(FileDesc) * nf, hipMemcpyHostToDevice, st)))
      return c->hip_fail(e, "H2D files");
    if ((e = bigfile_finish(c->d_files.p, (uint32_t)nf, c->d_file_nodes.p, c->d_out32.p, st)))
      return c->hip_fail(e, "bigfile_finish");
    std::vector<uint8_t> tmp(32 * nf);
    if ((e = hipMemcpyAsync(tmp.data(), c->d_out32.p, tmp.size(), hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return c->hip_fail(e, "D2H big digests");
    for (size_t i = 0; i < nf; ++i) memcpy(out32_host + 32 * items[i].out_index, &tmp[32 * i], 32);
  }
  for (size_t i = nf; i < items.size(); ++i)
    if (status && !status[items[i].out_index]) status[items[i].out_index] = SDCAS_STATUS_CANCELLED;
  return SDCAS_OK;
}



}  // namespace

// ===========================================================================

extern "C" {

const char* sdcas_version(void) { return "sdcas-mi355x 0.3.0 (gfx950)"; }

int sdcas_abi_version(void) { return SDCAS_ABI_VERSION; }

int sdcas_init(const sdcas_options* opts, sdcas_ctx** out) {
  if (!out) return SDCAS_E_INVALID;
  *out = nullptr;
  if (opts && opts->struct_size != sizeof(sdcas_options)) return SDCAS_E_INVALID;  // another revision of the struct
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SDCAS_E_NO_DEVICE;
  auto* c = new sdcas_ctx();
  int dev = -1;
  if (opts) {
    dev = opts->device;
    if (opts->io_threads) c->io_threads = std::min<uint32_t>(opts->io_threads, sdcas_ctx::kMaxIoThreads);
    if (opts->staging_bytes) c->staging_bytes = std::max<uint64_t>(opts->staging_bytes, 1ull << 20);
    c->direct_io = (opts->flags & SDCAS_OPT_DIRECT_IO) != 0;
    c->progress = opts->progress;
    c->progress_user = opts->progress_user;
    c->cancel = opts->cancel;
  }
  if (dev < 0) (void)hipGetDevice(&dev);
  if (dev >= count) {
    delete c;
    return SDCAS_E_NO_DEVICE;
  }
  // the largest batch (chunk slots) the default leaf kernel hands to the
  // small-batch kernel (b3_batch.h kSmallSlots; 0: never), for A/B runs
  if (const char* e = getenv("SDCAS_SMALL_SLOTS")) c->ws.small_slots = strtoull(e, nullptr, 0);
  if (const char* e = getenv("SDCAS_SMALL_VARIANT")) c->ws.small_variant = atoi(e);
  if (const char* e = getenv("SDCAS_UPLOAD_PARTS")) c->upload_parts = (uint32_t)std::min(atoi(e) > 0 ? atoi(e) : 0, 16);
  if (const char* e = getenv("SDCAS_PLAN_SMALL")) c->plan_small = atoi(e) != 0;
  if (const char* e = getenv("SDCAS_SMALL_DIRECT")) c->small_direct = atoi(e) != 0;
  // pinned staging per slot in MiB, over the caller's choice (A/B runs)
  if (const char* e = getenv("SDCAS_STAGING_MB"); e && atoi(e) > 0) c->staging_bytes = (uint64_t)atoi(e) << 20;
  c->device = dev;
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return SDCAS_E_NO_DEVICE;
  }
  *out = c;
  return SDCAS_OK;
}

void sdcas_destroy(sdcas_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  // a bound stream's last call may not have recorded its event, and the
  // caller's stream may be gone by now: wait for the whole device instead
  if (!c->scratch_recorded) (void)hipDeviceSynchronize();
  else (void)c->scratch_sync();
  for (auto* b : {&c->ws_S, &c->ws_total, &c->ws_soffs, &c->ws_slens, &c->dd_keys, &c->dd_ekeys, &c->dd_ids})
    b->release();
  for (auto* b : {&c->ws_tile_first, &c->ws_nodes, &c->ws_perm, &c->ws_sort_keys, &c->d_file_nodes, &c->piece_ctr, &c->piece_l4})
    b->release();
  for (auto* b : {&c->ws_scan, &c->d_out32, &c->dd_has}) b->release();
  c->d_files.release();
  c->dd_status.release();
  c->dd_link.release();
  c->dd_counts.release();
  c->dist.release();
  c->sm_d_files.release();
  c->sm_nodes.release();
  c->sm_pieces.release();
  c->sm_segs.release();
  c->sm_stage.release();
  for (Slot& s : c->slots) slot_release(s);
  for (auto e : c->ev_free) (void)hipEventDestroy(e);
  for (auto& p : c->ev_leaf) (void)hipEventDestroy(p.first), (void)hipEventDestroy(p.second);
  for (auto& p : c->ev_all) (void)hipEventDestroy(p.first), (void)hipEventDestroy(p.second);
  if (c->scratch_ev) (void)hipEventDestroy(c->scratch_ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  delete c;
}

const char* sdcas_last_error(const sdcas_ctx* c) { return c ? c->err.c_str() : "no context"; }

int sdcas_set_progress(sdcas_ctx* c, sdcas_progress_fn progress, void* user, const volatile int32_t* cancel) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  c->progress = progress;
  c->progress_user = user;
  c->cancel = cancel;
  return SDCAS_OK;
}

uint64_t sdcas_cas_message_len(uint64_t size) { return size <= kMin ? size + 8 : SDCAS_SAMPLED_MESSAGE_LEN; }

// The host's copy of k_plan_walk (dist_dedup.hip; the rule is described
// there): the job needs to know which rows its steps read before it writes
// their cas_ids (mod.rs:157-178 precede the lookup of :181-188), and that
// depends only on the rows' status and has_key.
int sdcas_job_plan(const uint8_t* has_key, const int32_t* status, size_t n, size_t chunk_size,
                   sdcas_job_window* win, uint64_t* out_step, uint32_t* out_reads) {
  if (!win || (n && !has_key)) return SDCAS_E_INVALID;
  const uint64_t cs = chunk_size ? chunk_size : SDCAS_IDENTIFIER_CHUNK_SIZE;
  auto stays = [&](size_t i) { return (status && status[i] != 0) || !has_key[i]; };
  std::vector<uint64_t> rr;  // re-read rows
  size_t first = SIZE_MAX;
  for (size_t p = 0; p < n; ++p) {
    if (!stays(p)) continue;
    if (first == SIZE_MAX) first = p;
    if (cs > 1 && p + 1 < n && (p + rr.size()) % cs == cs - 1) rr.push_back(p);
  }
  const uint64_t T = win->max_steps ? win->max_steps : (n + cs - 1) / cs;
  uint64_t loop = UINT64_MAX, reads = 0, steps, limit, rows = 0;
  if (cs == 1 && first != SIZE_MAX && first < T) {
    loop = first;
    reads = T - first;
    steps = T;
    limit = first;
    rows = first + 1;
  } else {
    const uint64_t E = n + rr.size();
    const uint64_t avail = win->more ? E / cs : (E + cs - 1) / cs;
    steps = std::min(avail, T);
    limit = steps * cs;
    if (steps) {
      const uint64_t P = std::min(limit, E) - 1;
      uint64_t k = 0;
      while (k < rr.size() && rr[k] + k + 1 <= P) ++k;
      rows = P - k + 1;
    }
    if (!win->more && T > avail && n && stays(n - 1)) {
      loop = n - 1;
      reads = 1 + (T - avail);
      steps = T;
    }
  }
  uint64_t run = 0;
  while (run < rr.size() && rr[run] + run + 1 < limit) ++run;
  win->steps = steps;
  win->rows = rows;
  win->rereads = run + (loop != UINT64_MAX ? reads - 1 : 0);
  if (out_step || out_reads) {
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
      while (k < rr.size() && rr[k] < i) ++k;
      const uint64_t pos = i + k;
      uint64_t s = UINT64_MAX;
      uint32_t r = 0;
      if (loop != UINT64_MAX && i >= loop) {
        if (i == loop) s = pos / cs, r = (uint32_t)std::min<uint64_t>(reads, UINT32_MAX);
      } else if (pos < limit) {
        s = pos / cs;
        r = 1 + (k < rr.size() && rr[k] == i && pos + 1 < limit ? 1 : 0);
      }
      if (out_step) out_step[i] = s;
      if (out_reads) out_reads[i] = r;
    }
  }
  return SDCAS_OK;
}

void sdcas_key_to_hex(uint64_t key, char out[17]) {
  static const char* H = "0123456789abcdef";
  for (int i = 0; i < 16; ++i) out[i] = H[(key >> (60 - 4 * i)) & 15];
  out[16] = 0;
}

void sdcas_digest_to_hex(const uint8_t d[32], char out[65]) {
  static const char* H = "0123456789abcdef";
  for (int i = 0; i < 32; ++i) {
    out[2 * i] = H[d[i] >> 4];
    out[2 * i + 1] = H[d[i] & 15];
  }
  out[64] = 0;
}

// A device-stream call: holds the context's mutex, orders its stream after
// the previous call's use of the device scratch (sdcas_ctx::fence_in) and
// marks its own use when it returns.
struct DevCall {
  sdcas_ctx* c;
  std::lock_guard<std::mutex> g;
  hipStream_t st;
  int rc = SDCAS_OK;
  DevCall(sdcas_ctx* cc, void* stream) : c(cc), g(cc->mu), st(stream ? (hipStream_t)stream : cc->stream) {
    (void)hipSetDevice(c->device);
    hipError_t e = c->fence_in(st);
    if (e) rc = c->hip_fail(e, "stream wait");
  }
  ~DevCall() { (void)c->fence_out(st); }
};

int sdcas_dev_reserve(sdcas_ctx* c, size_t max_msgs, uint64_t max_chunks) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  // the workspace is reallocated: no earlier call may still be using it
  if (hipError_t e = c->scratch_sync()) return c->hip_fail(e, "sync");
  return reserve_ws(c, max_msgs, max_chunks);
}

int sdcas_dev_hash_messages(sdcas_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets, const uint64_t* d_lens,
                            size_t n, uint8_t* d_out32, uint64_t* d_out_keys, void* stream) {
  if (!c || (n && (!d_blob || !d_offsets || !d_lens))) return SDCAS_E_INVALID;
  if (n == 0) return SDCAS_OK;
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (n > c->ws.cap_msgs || !c->ws.S)
    return c->fail(SDCAS_E_CAPACITY, "dev_hash_messages: %zu messages > reserved %u", n, c->ws.cap_msgs);
  return launch_batch(c, d_blob, d_offsets, d_lens, (uint32_t)n, d_out32, d_out_keys, call.st);
}

int sdcas_dev_bind_stream(sdcas_ctx* c, void* stream, uint64_t token) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  const hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  // the last call's event, owed by this stream, is recorded while the
  // stream surely lives (a caller unbinds before destroying it)
  if (c->scratch_pending && st == c->scratch_st)
    if (hipError_t e = c->scratch_event()) return c->hip_fail(e, "dev_bind_stream");
  for (size_t i = 0; i < c->bound.size(); ++i) {
    if (c->bound[i].first != st) continue;
    if (token) c->bound[i].second = token;
    else c->bound.erase(c->bound.begin() + (long)i);
    return SDCAS_OK;
  }
  if (!token) return SDCAS_OK;
  if (c->bound.size() >= 64) return c->fail(SDCAS_E_CAPACITY, "dev_bind_stream: 64 streams bound");
  c->bound.push_back({st, token});
  return SDCAS_OK;
}

int sdcas_dev_sync(sdcas_ctx* c, void* stream) {
  if (!c) return SDCAS_E_INVALID;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  hipError_t e = hipStreamSynchronize(st);
  if (e) return c->hip_fail(e, "sync");
  uint64_t total = 0;
  if (c->ws.total && (e = hipMemcpy(&total, c->ws.total, 8, hipMemcpyDeviceToHost))) return c->hip_fail(e, "total");
  if (total > c->ws.cap_slots)
    return c->fail(SDCAS_E_CAPACITY, "batch of %llu chunk slots exceeds reserved %llu", (unsigned long long)total,
                   (unsigned long long)c->ws.cap_slots);
  return SDCAS_OK;
}

int sdcas_dev_profile(sdcas_ctx* c, int enable) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  c->profile = enable != 0;
  for (auto* v : {&c->ev_all, &c->ev_leaf}) {
    for (auto& p : *v) c->ev_free.push_back(p.first), c->ev_free.push_back(p.second);
    v->clear();
  }
  return SDCAS_OK;
}

static float mean_ms(std::vector<std::pair<hipEvent_t, hipEvent_t>>& v) {
  float sum = 0;
  int cnt = 0;
  for (auto& p : v) {
    if (hipEventSynchronize(p.second) != hipSuccess) continue;
    float ms = 0;
    if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
      sum += ms;
      ++cnt;
    }
  }
  return cnt ? sum / cnt : 0.f;
}

int sdcas_dev_last_kernel_ms(sdcas_ctx* c, float* leaf_ms, float* total_ms) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  if (leaf_ms) *leaf_ms = mean_ms(c->ev_leaf);
  if (total_ms) *total_ms = mean_ms(c->ev_all);
  return SDCAS_OK;
}

int sdcas_hash_messages(sdcas_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* lens, size_t n,
                        uint8_t* out32);
// page-locked host memory (hipHostMalloc / hipHostRegister)? Pageable
// pointers make the query fail; its error is cleared.
static bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof a);
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost && a.hostPointer != nullptr;
}

// The path calls hold the context's mutex and run on its stream; they order
// themselves after any device call that used the scratch on another stream,
// and mark their own use when they return.
struct PathCall {
  sdcas_ctx* c;
  std::lock_guard<std::mutex> g;
  int rc = SDCAS_OK;
  explicit PathCall(sdcas_ctx* cc) : c(cc), g(cc->mu) {
    (void)hipSetDevice(c->device);
    // the readers start with the context's first path call (a context used
    // only for device-resident batches never creates them)
    if (!c->pool) c->pool.reset(new sdcas_io::WorkerPool(c->io_threads));
    sdcas_io::new_path_epoch();
    hipError_t e = c->fence_in(c->stream);
    if (e) rc = c->hip_fail(e, "stream wait");
  }
  ~PathCall() {
    (void)c->fence_out(c->stream);
    sdcas_io::drop_dir_cache();  // the caller's thread (big-file opens) keeps no directory open
  }
};

// Staging bytes per slot for one path call. The two slots alternate: the I/O
// threads fill one while the GPU copies and hashes the other, so a call whose
// files fit one slot runs read -> copy -> hash -> copy back in series. A call
// of up to a few slots' worth is therefore cut into kSplit slots, but none
// below kMinSlot, where a slot's fixed cost (its copies and launches) would
// outweigh what the overlap hides. Same-process A/B with the call order
// rotated (profiles/r02_batch_split_ab.json, C2 files from the page cache):
// 3000 files per call 9.4 -> 7.8 ms, 10000 per call 22.6 -> 20.7 ms; calls
// of up to 16 MiB (the reference's 100-file step) unchanged.
constexpr uint64_t kSplit = 8, kMinSlot = 16ull << 20;
// a lone slot's reads and upload overlapped in parts (sdcas_cas_ids;
// sdcas_ctx::upload_parts, SDCAS_UPLOAD_PARTS) from this many slot bytes
constexpr uint64_t kUploadSplitMin = 1ull << 20;
static uint64_t split_cap(const uint64_t* need, const size_t* order, size_t n, uint64_t cap) {
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += sdcas_io::align_line(need[order ? order[i] : i]);
  return std::min<uint64_t>(cap, std::max<uint64_t>(total / kSplit + 1, kMinSlot));
}

static int hash_host_messages(sdcas_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* lens,
                              size_t n, uint8_t* out32, uint64_t* keys) {
  if (!c || (n && (!blob || !offsets || !lens))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "batch of %zu messages exceeds 2^31 - 1", n);
  PathCall call(c);
  if (call.rc) return call.rc;
  const uint64_t big_cut = 1024ull * kTile;  // > 1 MiB: piece path
  const uint64_t cap = c->staging_bytes;
  const size_t cap_n = (size_t)(cap / 128) + 1;
  int rc;
  if ((rc = slots_prepare(c, cap, cap_n))) return rc;
  Progress pr{c};
  uint64_t small_bytes = 0;
  for (size_t i = 0; i < n; ++i) {
    pr.total += lens[i];
    if (lens[i] <= big_cut) small_bytes += sdcas_io::align_line(lens[i]);
  }
  const uint64_t scap = split_cap(&small_bytes, nullptr, 1, cap);
  std::vector<BigItem> big;
  int cur = 0;
  // Direct DMA: a caller buffer in pinned (page-locked) host memory whose
  // messages lie in ascending, non-overlapping, 16-byte aligned ranges is
  // copied range by range straight into the device slot (no host memcpy; the
  // path then runs at the PCIe H2D rate).
  bool direct = n > 0 && host_pinned(blob);
  for (size_t i = 0; direct && i < n; ++i)
    if ((offsets[i] & 15) || (i && offsets[i] < offsets[i - 1] + lens[i - 1])) direct = false;
  uint64_t base = 0;  // caller offset of the current direct slot's first byte
  auto begin = [&](Slot& s) -> int {
    const int r = slot_complete(
        c, s,
        [&](size_t k, const uint8_t* res) {
          const size_t i = s.idx[k];
          if (out32) memcpy(out32 + 32 * i, res, 32);
          if (keys) {
            uint64_t kk = 0;
            if (s.res32)
              for (int t = 0; t < 8; ++t) kk = (kk << 8) | res[t];
            else
              memcpy(&kk, res, 8);
            keys[i] = kk;
          }
        },
        &pr);
    s.n = 0, s.used = 0, s.chunks = 0, s.content = 0;
    s.idx.clear();
    s.src = nullptr;
    return r;
  };
  // the copy into pinned staging is the host-side cost of this path: it runs
  // on the I/O threads, one slot at a time, while the GPU hashes the other
  auto fill_submit = [&](Slot& s) -> int {
    if (direct) {
      s.src = blob + base;
    } else {
      c->pool->run(s.n, [&](size_t k) {
        memcpy(s.h + s.offs()[k], blob + offsets[s.idx[k]], s.lens()[k]);
      });
    }
    return slot_submit(c, s, out32 != nullptr);
  };
  bool cancelled = false;
  if ((rc = begin(c->slots[cur]))) return rc;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t L = lens[i];
    if (L > big_cut) {
      big.push_back({L, i});
      continue;
    }
    Slot* s = &c->slots[cur];
    const uint64_t end = direct ? offsets[i] + L - (s->n ? base : offsets[i]) : s->used + align16(L);
    if (s->n && (end > scap || s->n == cap_n)) {
      if ((rc = fill_submit(*s))) return rc;
      cur ^= 1;
      s = &c->slots[cur];
      if ((rc = begin(*s))) return rc;
      if ((cancelled = c->cancelled())) break;
    }
    if (direct && s->n == 0) base = offsets[i];
    s->offs()[s->n] = direct ? offsets[i] - base : s->used;
    s->lens()[s->n] = L;
    s->idx.push_back(i);
    s->n++;
    s->used = direct ? offsets[i] + L - base : s->used + align16(L);
    s->chunks += chunks_of(L);
    s->content += L;
  }
  if (!cancelled && (rc = fill_submit(c->slots[cur]))) return rc;
  for (Slot& s : c->slots)
    if ((rc = begin(s))) return rc;
  if (!cancelled && !big.empty()) {
    std::vector<uint8_t> d32(32 * n);
    rc = run_big(c, big, d32.data(),
                 [&](size_t k, uint8_t* dst, uint64_t off, uint32_t len) {
                   memcpy(dst, blob + offsets[big[k].out_index] + off, len);
                   return 0;
                 },
                 nullptr, pr, &cancelled);
    if (rc) return rc;
    for (auto& b : big) {
      if (out32) memcpy(out32 + 32 * b.out_index, &d32[32 * b.out_index], 32);
      if (keys) {
        uint64_t k = 0;
        for (int t = 0; t < 8; ++t) k = (k << 8) | d32[32 * b.out_index + t];
        keys[b.out_index] = k;
      }
    }
  }
  return cancelled ? c->fail(SDCAS_E_CANCELLED, "cancelled") : SDCAS_OK;
}

int sdcas_hash_messages(sdcas_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* lens, size_t n,
                        uint8_t* out32) {
  if (!out32 && n) return SDCAS_E_INVALID;
  return hash_host_messages(c, blob, offsets, lens, n, out32, nullptr);
}

int sdcas_cas_ids_from_messages(sdcas_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* lens,
                                size_t n, uint64_t* out_keys) {
  if (!out_keys && n) return SDCAS_E_INVALID;
  return hash_host_messages(c, blob, offsets, lens, n, nullptr, out_keys);
}

// SDCAS_TRACE_IO=1: per-call wall time of sdcas_cas_ids' phases on stderr
// (measurement aid for the page-cache path; no effect otherwise)
static bool last_parts() {
  static const bool on = [] {
    const char* v = getenv("SDCAS_LAST_PARTS");
    return v && strcmp(v, "1") == 0;
  }();
  return on;
}

struct IoTrace {
  bool on = getenv("SDCAS_TRACE_IO") != nullptr;
  double t[5] = {0, 0, 0, 0, 0};  // drain, plan, read, bookkeeping, submit
  std::chrono::steady_clock::time_point m = std::chrono::steady_clock::now();
  void lap(int k) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    t[k] += std::chrono::duration<double, std::milli>(now - m).count();
    m = now;
  }
  ~IoTrace() {
    if (on)
      fprintf(stderr, "sdcas_cas_ids trace ms: drain %.3f plan %.3f read %.3f book %.3f submit %.3f\n", t[0], t[1],
              t[2], t[3], t[4]);
  }
};

// The cas_ids of n files whose sizes are known, under a PathCall. fds (may be
// null): a file already open (fds[i] >= 0, `aligned[i]` = opened with
// O_DIRECT; sdcas_file_metadata) is read through its descriptor; any other
// is opened by path.
// meta (sdcas_file_metadata): `sizes` only plan the staging; each read takes
// the file's metadata from fstat of its descriptor (meta->sizes, meta->flags)
struct Meta {
  uint64_t* sizes;
  uint8_t* flags;
};

static int cas_ids_core(sdcas_ctx* c, const char* const* paths, const int* fds, const uint8_t* aligned,
                        const uint64_t* sizes, size_t n, uint64_t* out_keys, int32_t* out_status,
                        const Meta* meta = nullptr) {
  const uint64_t cap = c->staging_bytes;
  const size_t cap_n = (size_t)(cap / 128) + 1;
  int rc;
  if ((rc = slots_prepare(c, cap, cap_n))) return rc;
  // slot sizes: the message the indexer's size predicts (cas.rs:27); a file
  // that grew is retried in a later batch with its actual size
  std::vector<uint64_t> want(n);
  Progress pr{c};
  // (+1: room for the byte that tells a grown file from an unchanged one)
  for (size_t i = 0; i < n; ++i) {
    want[i] = sdcas_cas_message_len(sizes[i]) + (sizes[i] <= kMin ? 1 : 0);
    pr.total += sdcas_cas_message_len(sizes[i]) - 8;  // file bytes cas.rs reads
  }
  std::vector<size_t> todo(n);
  for (size_t i = 0; i < n; ++i) todo[i] = i;
  const uint64_t scap = split_cap(want.data(), nullptr, n, cap);
  int cur = 0;
  auto drain = [&](Slot& s) -> int {
    return slot_complete(c, s, [&](size_t k, const uint8_t* r) { memcpy(&out_keys[s.idx[k]], r, 8); }, &pr);
  };
  bool cancelled = false;
  IoTrace tr;
  for (int round = 0; round < 4 && !todo.empty() && !cancelled; ++round) {
    std::vector<size_t> retry;
    size_t p = 0;
    while (p < todo.size()) {
      // batch [p, q) fitting one staging slot (a message larger than the slot
      // — a whole-file cas message of a file grown past it — gets its own)
      Slot& s = c->slots[cur];
      tr.lap(4);
      if ((rc = drain(s))) return rc;
      tr.lap(0);
      if ((cancelled = c->cancelled())) {
        for (size_t k = p; k < todo.size(); ++k) out_status[todo[k]] = SDCAS_STATUS_CANCELLED;
        for (size_t i : retry) out_status[i] = SDCAS_STATUS_CANCELLED;
        retry.clear();
        break;
      }
      std::vector<uint64_t> slot_off;
      uint64_t used = 0;
      const size_t q = plan_batch(want.data(), todo.data(), p, todo.size(), scap, cap_n, slot_off, &used);
      if ((rc = slot_prepare(c, s, std::max<uint64_t>(used, cap), cap_n))) return rc;
      const size_t m = q - p;
      std::vector<uint64_t> mlen(m), retry_len(m);
      std::vector<int32_t> st(m);
      tr.lap(1);
      auto read_files = [&](size_t k0, size_t k1) {
        c->pool->run(k1 - k0, [&](size_t kk) {
          const size_t k = k0 + kk, i = todo[p + k];
          if (meta) {
            bool dir = false;
            st[k] = sdcas_io::read_file_metadata(paths[i], c->direct_io, s.h + slot_off[k], align16(want[i]),
                                                  &mlen[k], &retry_len[k], &meta->sizes[i], &dir);
            meta->flags[i] = dir ? SDCAS_META_DIR : 0;
            return;
          }
          st[k] = fds && fds[i] >= 0 ? sdcas_io::read_cas_message_fd(fds[i], aligned[i] != 0, sizes[i],
                                                                     s.h + slot_off[k], align16(want[i]), &mlen[k],
                                                                     &retry_len[k])
                                     : read_cas_message(paths[i], sizes[i], s.h + slot_off[k], align16(want[i]),
                                                        &mlen[k], &retry_len[k], c->direct_io);
        });
      };
      // A call that fits one slot is latency-bound: read -> upload -> hash in
      // series. Its files are then read in upload_parts parts of about equal
      // bytes, each part's bytes going up while the next part is read, so that
      // only the last part's upload stands between the reads and the kernels.
      const Slot& other = &s == &c->slots[0] ? c->slots[1] : c->slots[0];
      // (only for a call that fits this one slot: in a call of several slots
      // the next slot's reads already overlap this one's upload and kernels,
      // and the parts measured slower there, profiles/r03_small_calls.json)
      const uint32_t parts = c->upload_parts;
      // the flag is set only once every part is enqueued: a failed part
      // returns with it clear, so no later submit of this slot skips an upload
      s.blob_uploaded = false;
      // (and, SDCAS_LAST_PARTS=1, the last slot of a longer call: its upload
      // is the call's tail, the reads being over when it starts)
      const bool in_parts = parts > 1 && (!other.busy || last_parts()) && (p == 0 || last_parts()) &&
                            q == todo.size() && round == 0 && used >= kUploadSplitMin && m >= parts;
      if (in_parts) {
        size_t k0 = 0;
        for (uint32_t part = 1; part <= parts && k0 < m; ++part) {
          size_t k1 = k0 + 1;
          const uint64_t edge = used / parts * part;
          while (k1 < m && (part == parts || slot_off[k1] < edge)) ++k1;
          read_files(k0, k1);
          const uint64_t b0 = slot_off[k0], b1 = k1 < m ? slot_off[k1] : used;
          hipError_t e = hipMemcpyAsync(s.d_blob.p + b0, s.h + b0, b1 - b0, hipMemcpyHostToDevice, c->stream);
          if (e) return c->hip_fail(e, "H2D part");
          k0 = k1;
        }
        s.blob_uploaded = true;
      } else {
        read_files(0, m);
      }
      tr.lap(2);
      s.n = 0, s.chunks = 0, s.used = used, s.content = 0;
      s.idx.clear();
      for (size_t k = 0; k < m; ++k) {
        const size_t i = todo[p + k];
        if (retry_len[k] && !st[k]) {
          want[i] = retry_len[k];
          retry.push_back(i);
          continue;
        }
        out_status[i] = st[k];
        s.content += sdcas_cas_message_len(sizes[i]) - 8;
        if (st[k]) continue;
        if (meta && mlen[k] == 0) continue;  // a directory or an empty file: no cas_id
        if (meta) meta->flags[i] = SDCAS_META_HAS_CAS_ID;
        s.offs()[s.n] = slot_off[k];
        s.lens()[s.n] = mlen[k];
        s.idx.push_back(i);
        s.n++;
        s.chunks += chunks_of(mlen[k]);
      }
      tr.lap(3);
      if ((rc = slot_submit(c, s, false))) return rc;
      if (!s.n) pr.add(s.content);  // nothing to hash: the slot's files are final now
      cur ^= 1;
      p = q;
    }
    for (Slot& s : c->slots)
      if ((rc = drain(s))) return rc;
    todo.swap(retry);
  }
  for (size_t i : todo) out_status[i] = cancelled ? SDCAS_STATUS_CANCELLED : EAGAIN;  // EAGAIN: kept growing
  return cancelled ? c->fail(SDCAS_E_CANCELLED, "cancelled") : SDCAS_OK;
}

int sdcas_cas_ids(sdcas_ctx* c, const char* const* paths, const uint64_t* sizes, size_t n, uint64_t* out_keys,
                  int32_t* out_status) {
  if (!c || (n && (!paths || !sizes || !out_keys || !out_status))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "batch of %zu files exceeds 2^31 - 1", n);
  PathCall call(c);
  if (call.rc) return call.rc;
  return cas_ids_core(c, paths, nullptr, nullptr, sizes, n, out_keys, out_status);
}

int sdcas_file_metadata(sdcas_ctx* c, const char* const* paths, const uint64_t* size_hints, size_t n,
                        uint64_t* out_sizes, uint64_t* out_keys, int32_t* out_status, uint8_t* out_flags) {
  if (!c || (n && (!paths || !out_sizes || !out_keys || !out_status || !out_flags))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "batch of %zu files exceeds 2^31 - 1", n);
  PathCall call(c);
  if (call.rc) return call.rc;
  std::fill(out_sizes, out_sizes + n, 0);
  std::fill(out_keys, out_keys + n, 0);
  std::fill(out_flags, out_flags + n, 0);
  // the staging plan: the caller's sizes (the indexer's), else one fstatat
  // pass; either way each read takes the metadata from fstat of its own
  // descriptor and a file of another size is read again with room for it
  std::vector<uint64_t> plan(n);
  if (size_hints) {
    std::copy(size_hints, size_hints + n, plan.begin());
  } else {
    c->pool->run(n, [&](size_t i) {
      struct stat sb;
      plan[i] = stat(paths[i], &sb) == 0 && S_ISREG(sb.st_mode) ? (uint64_t)sb.st_size : 0;
    });
  }
  Meta meta{out_sizes, out_flags};
  return cas_ids_core(c, paths, nullptr, nullptr, plan.data(), n, out_keys, out_status, &meta);
}

int sdcas_checksums(sdcas_ctx* c, const char* const* paths, size_t n, uint8_t* out32, int32_t* out_status) {
  if (!c || (n && (!paths || !out32 || !out_status))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "batch of %zu files exceeds 2^31 - 1", n);
  PathCall call(c);
  if (call.rc) return call.rc;
  const uint64_t cap = c->staging_bytes, big_cut = 1024ull * kTile;
  const size_t cap_n = (size_t)(cap / 128) + 1;
  int rc;
  if ((rc = slots_prepare(c, cap, cap_n))) return rc;
  // file lengths first (hash.rs reads to EOF; a regular file's EOF is its length)
  std::vector<uint64_t> flen(n);
  std::vector<int32_t> fst(n);
  c->pool->run(n, [&](size_t i) {
    struct stat sb;
    if (stat(paths[i], &sb) != 0) fst[i] = errno;
    else if (S_ISDIR(sb.st_mode)) fst[i] = EISDIR;
    else flen[i] = (uint64_t)sb.st_size, fst[i] = 0;
  });
  std::vector<size_t> small;
  std::vector<BigItem> big;
  std::vector<uint64_t> fneed(n);  // staging bytes: the stat length + the byte that tells a grown file
  Progress pr{c};
  for (size_t i = 0; i < n; ++i) {
    out_status[i] = fst[i];
    fneed[i] = flen[i] + 1;
    if (fst[i]) continue;
    pr.total += flen[i];
    if (flen[i] > big_cut) big.push_back({flen[i], i});
    else small.push_back(i);
  }
  const uint64_t scap = split_cap(fneed.data(), small.data(), small.size(), cap);
  int cur = 0;
  auto drain = [&](Slot& s) -> int {
    return slot_complete(c, s, [&](size_t k, const uint8_t* r) { memcpy(out32 + 32 * s.idx[k], r, 32); }, &pr);
  };
  bool cancelled = false;
  size_t p = 0;
  while (p < small.size()) {
    Slot& s = c->slots[cur];
    if ((rc = drain(s))) return rc;
    if ((cancelled = c->cancelled())) break;
    std::vector<uint64_t> slot;
    uint64_t used = 0;
    const size_t q = plan_batch(fneed.data(), small.data(), p, small.size(), scap, cap_n, slot, &used);
    const size_t m = q - p;
    std::vector<uint64_t> got(m);
    std::vector<int32_t> st(m);
    c->pool->run(m, [&](size_t k) {
      const size_t i = small[p + k];
      bool isd = false;
      const int fd = open_for_read(paths[i], c->direct_io, &isd);
      if (fd < 0) {
        st[k] = -fd;
        return;
      }
      bool over = false;
      // hash.rs stops at its first short read; a file that grew since the
      // stat above is hashed over its stat length (sdcas.h)
      st[k] = read_whole_any(fd, isd, s.h + slot[k], flen[i] + 1, flen[i], &got[k], &over);
      if (over) got[k] = flen[i];
      close(fd);
    });
    s.n = 0, s.chunks = 0, s.used = used, s.content = 0;
    s.idx.clear();
    for (size_t k = 0; k < m; ++k) {
      const size_t i = small[p + k];
      out_status[i] = st[k];
      s.content += flen[i];
      if (st[k]) continue;
      s.offs()[s.n] = slot[k];
      s.lens()[s.n] = got[k];
      s.idx.push_back(i);
      s.n++;
      s.chunks += chunks_of(got[k]);
    }
    if ((rc = slot_submit(c, s, true))) return rc;
    if (!s.n) pr.add(s.content);
    cur ^= 1;
    p = q;
  }
  for (Slot& s : c->slots)
    if ((rc = drain(s))) return rc;
  if (cancelled) {
    for (size_t k = p; k < small.size(); ++k) out_status[small[k]] = SDCAS_STATUS_CANCELLED;
    for (auto& b : big) out_status[b.out_index] = SDCAS_STATUS_CANCELLED;
    return c->fail(SDCAS_E_CANCELLED, "cancelled");
  }
  if (!big.empty()) {
    // hash.rs reads the file to EOF in 1 MiB blocks; here a window's 1 MiB
    // pieces are read in parallel, with O_DIRECT when asked for and accepted
    std::vector<int> fds(big.size(), -1), oerr(big.size(), 0);
    std::vector<uint8_t> direct(big.size(), 0);
    for (size_t k = 0; k < big.size(); ++k) {
      bool d = false;
      fds[k] = open_for_read(paths[big[k].out_index], c->direct_io, &d);
      if (fds[k] < 0) oerr[k] = -fds[k];
      direct[k] = d;
    }
    std::vector<uint8_t> d32(32 * n);
    rc = run_big(c, big, d32.data(),
                 [&](size_t k, uint8_t* dst, uint64_t off, uint32_t len) -> int {
                   if (fds[k] < 0) return oerr[k];
                   return direct[k] ? pread_direct(fds[k], dst, len, off) : pread_exact(fds[k], dst, len, off);
                 },
                 out_status, pr, &cancelled);
    for (int fd : fds)
      if (fd >= 0) close(fd);
    if (rc) return rc;
    for (auto& b : big)
      if (!out_status[b.out_index]) memcpy(out32 + 32 * b.out_index, &d32[32 * b.out_index], 32);
  }
  return cancelled ? c->fail(SDCAS_E_CANCELLED, "cancelled") : SDCAS_OK;
}


// ---- dedup -----------------------------------------------------------------
//
// One implementation: the hash-table group-by of dist_dedup.hip. A single
// rank (this call) runs it fused (dd_local: files and existing Objects go
// straight into the resolve table; one insert pass per side, one apply
// pass); a node of ranks runs the same stages split at the exchange
// (sdcas_dev_dedup_combine / resolve / apply).

__global__ void k_iota64(uint64_t* __restrict__ p, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

static hipError_t iota(DevBuf<uint64_t>& b, size_t n, hipStream_t st) {
  hipError_t e = b.ensure(std::max<size_t>(n, 1));
  if (e || !n) return e;
  hipLaunchKernelGGL(k_iota64, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, b.p, (uint32_t)n);
  return hipGetLastError();
}

// the resolve table holds 2 * (files + existing) entries, at most 2^31
static bool dedup_fits(size_t n, size_t ne) { return (uint64_t)n + ne <= (1ull << 30); }

int sdcas_dedup_window(sdcas_ctx* c, const uint64_t* keys, const uint8_t* has_key, const int32_t* status, size_t n,
                       size_t chunk_size, const uint64_t* existing_keys, size_t n_existing, sdcas_job_window* win,
                       int64_t* out_link, int64_t* out_created, int64_t* out_linked) {
  if (!c || (n && (!keys || !has_key || !out_link)) || (n_existing && !existing_keys)) return SDCAS_E_INVALID;
  if (!dedup_fits(n, n_existing))
    return c->fail(SDCAS_E_CAPACITY, "dedup of %zu files + %zu Objects exceeds 2^30", n, n_existing);
  PathCall call(c);
  if (call.rc) return call.rc;
  if (chunk_size == 0) chunk_size = SDCAS_IDENTIFIER_CHUNK_SIZE;
  hipError_t e;
  hipStream_t st = c->stream;
  if ((e = c->dd_keys.ensure(n)) || (e = c->dd_has.ensure(n)) || (e = c->dd_link.ensure(n)) ||
      (status && (e = c->dd_status.ensure(n))) || (e = c->dd_ekeys.ensure(n_existing + 1)) ||
      (e = c->dd_counts.ensure(2)))
    return c->hip_fail(e, "dedup buffers");
  if ((e = hipMemcpyAsync(c->dd_keys.p, keys, 8 * n, hipMemcpyHostToDevice, st)) ||
      (e = hipMemcpyAsync(c->dd_has.p, has_key, n, hipMemcpyHostToDevice, st)) ||
      (status && (e = hipMemcpyAsync(c->dd_status.p, status, 4 * n, hipMemcpyHostToDevice, st))) ||
      (n_existing && (e = hipMemcpyAsync(c->dd_ekeys.p, existing_keys, 8 * n_existing, hipMemcpyHostToDevice, st))) ||
      (e = hipMemsetAsync(c->dd_counts.p, 0, 2 * sizeof(unsigned long long), st)))
    return c->hip_fail(e, "dedup H2D");
  // files are ordinals 0..n-1 in orphan order, existing Objects 0..ne-1 in DB
  // order: one iota serves both (ids of the first min(n, ne) coincide)
  if ((e = iota(c->dd_ids, std::max(n, n_existing), st))) return c->hip_fail(e, "dedup ids");
  StepWindow sw;
  sw.n_total = n;
  sw.max_steps = win ? win->max_steps : 0;
  sw.more = win ? win->more : 0;
  if ((e = dd_local(c->dist, c->dd_keys.p, c->dd_has.p, status ? c->dd_status.p : nullptr, c->dd_ids.p, (uint32_t)n,
                    c->dd_ekeys.p, c->dd_ids.p, (uint32_t)n_existing, chunk_size, sw, c->dd_link.p, c->dd_counts.p,
                    st)))
    return c->hip_fail(e, "dedup");
  unsigned long long cnt[2] = {0, 0};
  uint64_t hdr[kPlanHeader] = {};
  if ((n && (e = hipMemcpyAsync(out_link, c->dd_link.p, 8 * n, hipMemcpyDeviceToHost, st))) ||
      (e = hipMemcpyAsync(cnt, c->dd_counts.p, sizeof cnt, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(hdr, c->dist.plan.p, sizeof hdr, hipMemcpyDeviceToHost, st)))
    return c->hip_fail(e, "dedup D2H");
  if ((e = hipStreamSynchronize(st))) return c->hip_fail(e, "dedup sync");
  if (out_created) *out_created = (int64_t)cnt[0];
  if (out_linked) *out_linked = (int64_t)cnt[1];
  if (win) {
    win->steps = hdr[kPlanSteps];
    win->rows = hdr[kPlanRows];
    win->rereads = hdr[kPlanRereadsRun];
  }
  return SDCAS_OK;
}

int sdcas_dedup(sdcas_ctx* c, const uint64_t* keys, const uint8_t* has_key, const int32_t* status, size_t n,
                size_t chunk_size, const uint64_t* existing_keys, size_t n_existing, int64_t* out_link,
                int64_t* out_created, int64_t* out_linked) {
  return sdcas_dedup_window(c, keys, has_key, status, n, chunk_size, existing_keys, n_existing, nullptr, out_link,
                            out_created, out_linked);
}

int sdcas_dev_dedup(sdcas_ctx* c, const uint64_t* d_keys, const uint8_t* d_has_key, const int32_t* d_status,
                    size_t n, size_t chunk_size, int64_t* d_out_link, uint64_t* d_counts, void* stream) {
  if (!c || (n && (!d_keys || !d_has_key || !d_out_link))) return SDCAS_E_INVALID;
  if (!dedup_fits(n, 0)) return c->fail(SDCAS_E_CAPACITY, "dev_dedup of %zu files exceeds 2^30", n);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (chunk_size == 0) chunk_size = SDCAS_IDENTIFIER_CHUNK_SIZE;
  hipError_t e;
  if (d_counts && (e = hipMemsetAsync(d_counts, 0, 2 * sizeof(uint64_t), call.st))) return c->hip_fail(e, "counts");
  if ((e = iota(c->dd_ids, n, call.st))) return c->hip_fail(e, "dev_dedup ids");
  e = dd_local(c->dist, d_keys, d_has_key, d_status, c->dd_ids.p, (uint32_t)n, nullptr, nullptr, 0, chunk_size,
               StepWindow{}, d_out_link, (unsigned long long*)d_counts, call.st);
  return e ? c->hip_fail(e, "dev_dedup") : SDCAS_OK;
}

int sdcas_dev_set_sort(sdcas_ctx* c, int enable) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  c->ws.sort = enable ? 1 : 0;
  return SDCAS_OK;
}

int sdcas_dev_set_leaf_variant(sdcas_ctx* c, int variant) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  if (variant != -1 && !leaf_variant_available(variant))
    return c->fail(SDCAS_E_INVALID, "leaf variant %d is not in this build", variant);
  c->ws.variant = variant;
  return SDCAS_OK;
}

int sdcas_dev_set_piece_variant(sdcas_ctx* c, int variant) {
  if (!c) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  if (variant != -1 && !piece_variant_available(variant))
    return c->fail(SDCAS_E_INVALID, "piece variant %d is not in this build", variant);
  c->piece_variant = variant;
  return SDCAS_OK;
}

// ---- synthetic corpora -------------------------------------------------------

int sdcas_dev_synth_cas_messages(sdcas_ctx* c, const uint64_t* d_keys, const uint64_t* d_sizes,
                                 const uint64_t* d_offs, size_t n, uint8_t* d_blob, void* stream) {
  if (!c) return SDCAS_E_INVALID;
  (void)hipSetDevice(c->device);
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  hipError_t e = synth_cas_messages(d_keys, d_sizes, d_offs, (uint32_t)n, d_blob, st);
  return e ? c->hip_fail(e, "synth") : SDCAS_OK;
}

int sdcas_dev_synth_content(sdcas_ctx* c, const uint64_t* d_keys, const uint64_t* d_starts, const uint64_t* d_lens,
                            const uint64_t* d_offs, size_t n, uint8_t* d_blob, void* stream) {
  if (!c) return SDCAS_E_INVALID;
  (void)hipSetDevice(c->device);
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  hipError_t e = synth_content(d_keys, d_starts, d_lens, d_offs, (uint32_t)n, d_blob, st);
  return e ? c->hip_fail(e, "synth") : SDCAS_OK;
}

// ---- multi-GPU dedup stages -----------------------------------

int sdcas_dev_dedup_combine(sdcas_ctx* c, const uint64_t* d_keys, const uint8_t* d_has_key, const int32_t* d_status,
                            const uint64_t* d_ids, size_t n, uint32_t world, uint64_t* d_rec, uint32_t* d_slot,
                            uint64_t* out_starts, void* stream) {
  if (!c || world == 0 || !out_starts || (n && (!d_keys || !d_ids || !d_rec))) return SDCAS_E_INVALID;
  // record indices and slot codes are 32-bit
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "dedup_combine: %zu records exceed 2^31 - 1", n);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  uint64_t u = 0;
  hipError_t e = dd_combine(c->dist, d_keys, d_has_key, d_status, d_ids, (uint32_t)n, world, d_rec, d_slot,
                            out_starts, &u, call.st);
  return e ? c->hip_fail(e, "dedup_combine") : SDCAS_OK;
}

int sdcas_dev_dedup_combine_async(sdcas_ctx* c, const uint64_t* d_keys, const uint8_t* d_has_key,
                                  const int32_t* d_status, const uint64_t* d_ids, size_t n, uint32_t world,
                                  uint64_t* d_rec, uint32_t* d_slot, uint32_t* d_starts, void* stream) {
  if (!c || world == 0 || !d_starts || (n && (!d_keys || !d_ids || !d_rec))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "dedup_combine: %zu records exceed 2^31 - 1", n);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_combine_dev(c->dist, d_keys, d_has_key, d_status, d_ids, (uint32_t)n, world, d_rec, d_slot,
                                d_starts, call.st);
  return e ? c->hip_fail(e, "dedup_combine_async") : SDCAS_OK;
}

int sdcas_dev_dedup_combine_buckets(sdcas_ctx* c, const uint64_t* d_keys, const uint8_t* d_has_key,
                                    const int32_t* d_status, const uint64_t* d_ids, size_t n, uint32_t world,
                                    size_t cap, uint64_t* d_send, uint32_t* d_slot, int64_t* d_counts,
                                    uint32_t* d_overflow, void* stream) {
  if (!c || world == 0 || !d_counts || !d_overflow || (n && (!d_keys || !d_ids || !d_send))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH || (uint64_t)world * cap > SDCAS_MAX_BATCH)
    return c->fail(SDCAS_E_CAPACITY, "dedup_combine_buckets: %zu records / %u x %zu buckets exceed 2^31 - 1", n,
                   world, cap);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_combine_buckets(c->dist, d_keys, d_has_key, d_status, d_ids, (uint32_t)n, world, (uint32_t)cap,
                                    d_send, d_slot, d_counts, d_overflow, call.st);
  return e ? c->hip_fail(e, "dedup_combine_buckets") : SDCAS_OK;
}

int sdcas_dev_dedup_resolve(sdcas_ctx* c, const uint64_t* d_frec, size_t nf, const uint64_t* d_erec, size_t ne,
                            int64_t* d_result, void* stream) {
  if (!c || (nf && (!d_frec || !d_result)) || (ne && !d_erec)) return SDCAS_E_INVALID;
  if (!dedup_fits(nf, ne)) return c->fail(SDCAS_E_CAPACITY, "dedup_resolve: %zu + %zu records exceed 2^30", nf, ne);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_resolve(c->dist, d_frec, (uint32_t)nf, d_erec, (uint32_t)ne, d_result, call.st);
  return e ? c->hip_fail(e, "dedup_resolve") : SDCAS_OK;
}

int sdcas_dev_dedup_resolve_buckets(sdcas_ctx* c, const uint64_t* d_frec, size_t fcap, const int64_t* d_fcounts,
                                    const uint64_t* d_erec, size_t ecap, const int64_t* d_ecounts, uint32_t world,
                                    int64_t* d_result, void* stream) {
  if (!c || world == 0 || (fcap && (!d_frec || !d_fcounts || !d_result)) || (ecap && (!d_erec || !d_ecounts)))
    return SDCAS_E_INVALID;
  if (!dedup_fits((uint64_t)world * fcap, (uint64_t)world * ecap))
    return c->fail(SDCAS_E_CAPACITY, "dedup_resolve_buckets: %u x (%zu + %zu) records exceed 2^30", world, fcap, ecap);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_resolve_buckets(c->dist, d_frec, (uint32_t)fcap, d_fcounts, d_erec, (uint32_t)ecap, d_ecounts,
                                    world, d_result, call.st);
  return e ? c->hip_fail(e, "dedup_resolve_buckets") : SDCAS_OK;
}

int sdcas_dev_dedup_local(sdcas_ctx* c, const uint64_t* d_keys, const uint8_t* d_has_key, const int32_t* d_status,
                          const uint64_t* d_ids, size_t n, const uint64_t* d_ekeys, const uint64_t* d_eids, size_t ne,
                          size_t chunk_size, uint64_t n_total, uint64_t max_steps, uint32_t more, int64_t* d_link,
                          uint64_t* d_counts, uint64_t* d_plan_header, void* stream) {
  if (!c || (n && (!d_keys || !d_ids || !d_link)) || (ne && (!d_ekeys || !d_eids))) return SDCAS_E_INVALID;
  if (!dedup_fits(n, ne)) return c->fail(SDCAS_E_CAPACITY, "dedup_local: %zu + %zu records exceed 2^30", n, ne);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  StepWindow sw;
  sw.n_total = n_total;
  sw.max_steps = max_steps;
  sw.more = more;
  hipError_t e = dd_local(c->dist, d_keys, d_has_key, d_status, d_ids, (uint32_t)n, d_ekeys, d_eids, (uint32_t)ne,
                          chunk_size ? chunk_size : SDCAS_IDENTIFIER_CHUNK_SIZE, sw, d_link,
                          (unsigned long long*)d_counts, call.st);
  if (!e && d_plan_header)
    e = hipMemcpyAsync(d_plan_header, c->dist.plan.p, 8 * kPlanHeader, hipMemcpyDeviceToDevice, call.st);
  return e ? c->hip_fail(e, "dedup_local") : SDCAS_OK;
}

int sdcas_dev_dedup_stays(sdcas_ctx* c, const uint8_t* d_has_key, const int32_t* d_status, const uint64_t* d_ids,
                          size_t n, size_t cap, uint64_t* d_stays, int64_t* d_count, void* stream) {
  if (!c || (n && (d_has_key || d_status) && !d_ids) || (cap && !d_stays)) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH || cap > SDCAS_MAX_BATCH)
    return c->fail(SDCAS_E_CAPACITY, "dedup_stays: %zu files / %zu entries exceed 2^31 - 1", n, cap);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_stays(c->dist, d_has_key, d_status, d_ids, (uint32_t)n, (uint32_t)cap, d_stays, d_count, call.st);
  return e ? c->hip_fail(e, "dedup_stays") : SDCAS_OK;
}

int sdcas_dev_dedup_plan(sdcas_ctx* c, const uint64_t* d_stays, size_t n_stays, uint64_t n_total, size_t chunk_size,
                         uint64_t max_steps, uint32_t more, uint64_t* d_plan, void* stream) {
  if (!c || !d_plan || (n_stays && !d_stays)) return SDCAS_E_INVALID;
  if (n_stays > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "dedup_plan: %zu entries exceed 2^31 - 1", n_stays);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  StepWindow sw;
  sw.n_total = n_total;
  sw.max_steps = max_steps;
  sw.more = more;
  hipError_t e = dd_plan(c->dist, d_stays, (uint32_t)n_stays, chunk_size ? chunk_size : SDCAS_IDENTIFIER_CHUNK_SIZE,
                         sw, d_plan, call.st);
  return e ? c->hip_fail(e, "dedup_plan") : SDCAS_OK;
}

int sdcas_dev_dedup_apply(sdcas_ctx* c, const uint64_t* d_ids, const uint32_t* d_slot, size_t n,
                          const int64_t* d_result, size_t chunk_size, const uint64_t* d_plan, int64_t* d_link,
                          uint64_t* d_counts, void* stream) {
  if (!c || (n && (!d_ids || !d_slot || !d_link))) return SDCAS_E_INVALID;
  if (n > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "dedup_apply: %zu files exceed 2^31 - 1", n);
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  hipError_t e = dd_apply(c->dist, d_ids, d_slot, (uint32_t)n, d_result, chunk_size ? chunk_size : SDCAS_IDENTIFIER_CHUNK_SIZE,
                          d_plan, d_link, (unsigned long long*)d_counts, call.st);
  return e ? c->hip_fail(e, "dedup_apply") : SDCAS_OK;
}

// ---- device-resident big-message stream (C4, file_checksum of huge files) --------

// A device buffer about to grow is freed and reallocated: the context's
// enqueued work (any stream) must be done with it first. Growth happens on a
// session larger than every earlier one, so the steady state never waits.
}  // extern "C"
template <typename T>
static hipError_t grow(sdcas_ctx* c, DevBuf<T>& b, size_t n, hipStream_t st = nullptr) {
  if (n <= b.cap) return hipSuccess;
  hipError_t e;
  if (st && (e = hipStreamSynchronize(st))) return e;
  if ((e = c->scratch_sync())) return e;
  return b.ensure(n);
}
extern "C" {

// The session's message descriptors go up and its node list is cleared on
// the stream of the session's first device call (stream_begin names none):
// no host wait, ordered after the previous session's kernels by the fence.
static hipError_t stream_flush_begin(sdcas_ctx* c, hipStream_t st) {
  if (!c->sm_begin_pending) return hipSuccess;
  c->sm_begin_pending = false;
  hipError_t e;
  if (!c->sm_files.empty() &&
      (e = c->sm_stage.put(c->sm_files.data(), sizeof(FileDesc) * c->sm_files.size(), c->sm_d_files.p, st)))
    return e;
  // node entries no segment of this session writes stay zero, so that the
  // node lists of ranks that hashed disjoint pieces of the same messages add
  // up to the complete list (sdcas_dev_stream_import)
  if (c->sm_node_bytes && (e = hipMemsetAsync(c->sm_nodes.p, 0, c->sm_node_bytes, st))) return e;
  return hipSuccess;
}

int sdcas_dev_stream_begin(sdcas_ctx* c, const uint64_t* lens, size_t nfiles) {
  if (!c || (nfiles && !lens)) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  std::vector<FileDesc> files(nfiles, FileDesc{});
  uint64_t nodes = 0;
  for (size_t i = 0; i < nfiles; ++i) {
    const uint64_t C = chunks_of(lens[i]);
    if (C <= kTile) return c->fail(SDCAS_E_INVALID, "stream message %zu: %llu bytes (must exceed 1 MiB)", i,
                                   (unsigned long long)lens[i]);
    files[i].C = C;
    files[i].node_base = nodes;
    files[i].out_index = i;
    nodes += bigfile_node_count(C);
  }
  // the descriptors and node list are rewritten in stream order by the
  // session's first device call (stream_flush_begin); only a buffer that must
  // grow waits for the previous session here
  hipError_t e;
  if ((e = grow(c, c->sm_nodes, 8 * nodes + 8)) || (e = grow(c, c->sm_d_files, nfiles + 1)) ||
      (e = grow(c, c->piece_ctr, 1)))
    return c->hip_fail(e, "stream workspace");
  c->sm_files.swap(files);
  c->sm_node_bytes = 32 * nodes;
  c->sm_active = true;
  c->sm_begin_pending = true;
  return SDCAS_OK;
}

size_t sdcas_dev_stream_node_bytes(sdcas_ctx* c) { return c && c->sm_active ? (size_t)c->sm_node_bytes : 0; }

int sdcas_dev_stream_export(sdcas_ctx* c, uint8_t* d_dst, size_t bytes, void* stream) {
  if (!c || (bytes && !d_dst)) return SDCAS_E_INVALID;
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (!c->sm_active || bytes != c->sm_node_bytes)
    return c->fail(SDCAS_E_INVALID, "stream_export: %zu bytes, the session's node list holds %llu", bytes,
                   (unsigned long long)c->sm_node_bytes);
  hipError_t e = stream_flush_begin(c, call.st);
  if (!e && bytes) e = hipMemcpyAsync(d_dst, c->sm_nodes.p, bytes, hipMemcpyDeviceToDevice, call.st);
  return e ? c->hip_fail(e, "stream_export") : SDCAS_OK;
}

int sdcas_dev_stream_import(sdcas_ctx* c, const uint8_t* d_src, size_t bytes, void* stream) {
  if (!c || (bytes && !d_src)) return SDCAS_E_INVALID;
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (!c->sm_active || bytes != c->sm_node_bytes)
    return c->fail(SDCAS_E_INVALID, "stream_import: %zu bytes, the session's node list holds %llu", bytes,
                   (unsigned long long)c->sm_node_bytes);
  hipError_t e = stream_flush_begin(c, call.st);
  if (!e && bytes) e = hipMemcpyAsync(c->sm_nodes.p, d_src, bytes, hipMemcpyDeviceToDevice, call.st);
  return e ? c->hip_fail(e, "stream_import") : SDCAS_OK;
}

int sdcas_dev_stream_update(sdcas_ctx* c, size_t nseg, const uint64_t* h_file, const uint64_t* h_msg_off,
                            const uint64_t* h_len, const uint64_t* h_dev_addr, void* stream) {
  if (!c || (nseg && (!h_file || !h_msg_off || !h_len || !h_dev_addr))) return SDCAS_E_INVALID;
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (!c->sm_active) return c->fail(SDCAS_E_INVALID, "stream_update without stream_begin");
  const uint64_t piece_bytes = 1024ull * kTile;
  uint64_t base = ~0ull;
  for (size_t k = 0; k < nseg; ++k) base = std::min(base, h_dev_addr[k]);
  // one descriptor per segment (the caller's few hundred); the device expands
  // them into the per-piece list (expand_pieces)
  std::vector<SegDesc> segs(nseg);
  uint64_t npieces = 0;
  for (size_t k = 0; k < nseg; ++k) {
    if (h_file[k] >= c->sm_files.size()) return c->fail(SDCAS_E_INVALID, "segment %zu: no such message", k);
    const FileDesc& fd = c->sm_files[h_file[k]];
    const uint64_t mlen = fd.C * 1024;  // upper bound; the last chunk may be short
    const uint64_t off = h_msg_off[k], len = h_len[k];
    if ((off % piece_bytes) || (h_dev_addr[k] & 15) || !len || off + len > mlen ||
        ((len % piece_bytes) && chunks_of(off + len) != fd.C))
      return c->fail(SDCAS_E_INVALID, "segment %zu: offset/length not on 1 MiB pieces", k);
    segs[k] = SegDesc{h_dev_addr[k] - base, off / 1024, fd.node_base, len, npieces};
    npieces += (len + piece_bytes - 1) / piece_bytes;
  }
  hipStream_t st = call.st;
  hipError_t e = stream_flush_begin(c, st);
  if (e) return c->hip_fail(e, "stream descs");
  if (!npieces) return SDCAS_OK;
  if (npieces > SDCAS_MAX_BATCH) return c->fail(SDCAS_E_CAPACITY, "stream_update: %llu pieces",
                                                (unsigned long long)npieces);
  // stream-ordered: a previous update's kernels on any stream are behind the
  // fence, so the descriptor buffers are free once this call's work starts
  if ((e = grow(c, c->sm_pieces, npieces, st)) || (e = grow(c, c->sm_segs, nseg, st)) ||
      (e = grow(c, c->piece_l4, kPieceL4Words * npieces, st)))
    return c->hip_fail(e, "piece descs");
  if ((e = c->sm_stage.put(segs.data(), sizeof(SegDesc) * nseg, c->sm_segs.p, st)) ||
      (e = expand_pieces(c->sm_segs.p, (uint32_t)nseg, c->sm_pieces.p, (uint32_t)npieces, st)))
    return c->hip_fail(e, "piece descs");
  hipEvent_t a = nullptr, b = nullptr;
  if (c->profile) {
    a = c->event();
    b = c->event();
    (void)hipEventRecord(a, st);
  }
  e = piece_hash(reinterpret_cast<const uint8_t*>(base), c->sm_pieces.p, (uint32_t)npieces, c->sm_nodes.p,
                 c->piece_ctr.p, c->piece_l4.p, c->piece_variant, st);
  if (c->profile) {
    (void)hipEventRecord(b, st);
    c->ev_leaf.push_back({a, b});
    c->ev_all.push_back({c->event(), c->event()});
    (void)hipEventRecord(c->ev_all.back().first, st);
    (void)hipEventRecord(c->ev_all.back().second, st);
  }
  return e ? c->hip_fail(e, "piece_hash") : SDCAS_OK;
}

int sdcas_dev_stream_finish(sdcas_ctx* c, uint8_t* d_out32, void* stream) {
  if (!c || !d_out32) return SDCAS_E_INVALID;
  DevCall call(c, stream);
  if (call.rc) return call.rc;
  if (!c->sm_active) return c->fail(SDCAS_E_INVALID, "stream_finish without stream_begin");
  hipStream_t st = call.st;
  hipError_t e = stream_flush_begin(c, st);
  if (e) return c->hip_fail(e, "stream descs");
  c->sm_active = false;
  e = bigfile_finish(c->sm_d_files.p, (uint32_t)c->sm_files.size(), c->sm_nodes.p, d_out32, st);
  return e ? c->hip_fail(e, "bigfile_finish") : SDCAS_OK;
}

}  // extern "C"
