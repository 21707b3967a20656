// sdcas_node.hip — one host process driving several GPUs (a node).
//
// sd-core is one process: Node::new (apps/server/src/main.rs:40) owns every
// library, and the job manager runs jobs in-process (core/src/job/manager.rs:32).
// A node here is that process's view of its GPUs: one libsdcas context per
// device entry, the batch calls sharded over them, and the identifier
// group-by's one exchange step run between the contexts in
// this process:
//   - RCCL (ncclCommInitAll over the node's devices, ncclSend / ncclRecv in one
//     group) when every device is distinct;
//   - device-to-device copies (hipMemcpyPeerAsync) otherwise — a device may
//     appear twice (two contexts on one GPU), which is how a one-GPU machine
//     exercises the whole exchange.
// The node is an orchestrator over the public per-context calls
// (sdcas_cas_ids, sdcas_checksums, sdcas_dev_dedup_*); RCCL is bound at run
// time (dlopen), so libsdcas.so has no link-time dependency on it and a
// process that already loaded torch's RCCL shares it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/stat.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdcas.h"

namespace {

// ---- RCCL, bound at run time -------------------------------------------------
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool load() {
    for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
    if (!h) return false;
    comm_init_all = (decltype(comm_init_all))dlsym(h, "ncclCommInitAll");
    comm_destroy = (decltype(comm_destroy))dlsym(h, "ncclCommDestroy");
    send = (decltype(send))dlsym(h, "ncclSend");
    recv = (decltype(recv))dlsym(h, "ncclRecv");
    group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
    group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
    error_string = (decltype(error_string))dlsym(h, "ncclGetErrorString");
    return comm_init_all && comm_destroy && send && recv && group_start && group_end && error_string;
  }
};

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n, 16);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (!e) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

__global__ void k_iota_from(uint64_t* __restrict__ p, uint64_t first, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = first + i;
}

struct Rank {
  int dev = 0;
  sdcas_ctx* ctx = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  hipEvent_t ev_starts = nullptr;  // the owner ranges are on the host
  uint32_t* hstarts = nullptr;     // pinned: owner ranges of the files' and the existing Objects' records
  size_t hstarts_cap = 0;
  // dedup shard: files [lo, hi) and existing Objects [elo, ehi) of the batch
  size_t lo = 0, hi = 0, elo = 0, ehi = 0;
  DBuf<uint64_t> keys, ids, ekeys, eids, rec, erec, frecv, erecv, stays, gstays, plan, counts;
  DBuf<uint8_t> has;
  DBuf<int32_t> status;
  DBuf<uint32_t> slot, dstarts;
  DBuf<int64_t> answer, back, link, scount;
  std::vector<uint64_t> starts, estarts;
  uint64_t done = 0, total = 0;  // progress of this rank's share of a path call
  void release() {
    for (auto* b : {&keys, &ids, &ekeys, &eids, &rec, &erec, &frecv, &erecv, &stays, &gstays, &plan, &counts}) b->release();
    has.release();
    status.release();
    slot.release();
    dstarts.release();
    for (auto* b : {&answer, &back, &link, &scount}) b->release();
    if (hstarts) (void)hipHostFree(hstarts);
    hstarts = nullptr;
    hstarts_cap = 0;
  }
};

}  // namespace

struct sdcas_node;
namespace {
struct RankProgress {  // the progress function's user pointer of one rank's context
  sdcas_node* node;
  size_t r;
};
}  // namespace

struct sdcas_node {
  std::vector<Rank> ranks;
  std::vector<RankProgress> slots;  // sized once at init: the contexts hold pointers into it
  bool rccl = false;
  Rccl nccl;
  std::vector<ncclComm_t> comms;
  std::string err;
  std::mutex mu;        // one node call at a time
  std::mutex prog_mu;   // the ranks' progress reports, merged
  sdcas_progress_fn progress = nullptr;
  void* progress_user = nullptr;
  std::chrono::steady_clock::time_point t_call;  // the running node call's start (SDCAS_NODE_TRACE)
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
  int ctx_fail(size_t r, int rc, const char* what) {
    return fail(rc, "%s on rank %zu (device %d): %s", what, r, ranks[r].dev, sdcas_last_error(ranks[r].ctx));
  }
};

namespace {

// every rank reports its own share; the caller sees the node's sums
void node_progress(void* user, uint64_t done, uint64_t total) {
  auto* rp = static_cast<RankProgress*>(user);
  sdcas_node* n = rp->node;
  std::lock_guard<std::mutex> g(n->prog_mu);
  n->ranks[rp->r].done = done;
  n->ranks[rp->r].total = total;
  if (!n->progress) return;
  uint64_t d = 0, t = 0;
  for (const Rank& k : n->ranks) d += k.done, t += k.total;
  n->progress(n->progress_user, d, t);
}

// one copy of the exchange: bytes from rank `src` to rank `dst`
struct Copy {
  size_t src, dst;
  const void* from;
  void* to;
  size_t bytes;
};

// Run a set of copies between the ranks' device buffers, ordered after each
// rank's work so far on its stream and before its next.
int exchange(sdcas_node* n, const std::vector<Copy>& copies, const char* what) {
  const size_t R = n->ranks.size();
  hipError_t e;
  if (n->rccl) {
    // local copies first (a rank's own segment needs no network)
    for (const Copy& c : copies)
      if (c.src == c.dst && c.bytes) {
        (void)hipSetDevice(n->ranks[c.dst].dev);
        if ((e = hipMemcpyAsync(c.to, c.from, c.bytes, hipMemcpyDeviceToDevice, n->ranks[c.dst].st)))
          return n->hip_fail(e, what);
      }
    ncclResult_t r = n->nccl.group_start();
    for (const Copy& c : copies) {
      if (c.src == c.dst || !c.bytes || r != ncclSuccess) continue;
      r = n->nccl.send(c.from, c.bytes, ncclUint8, (int)c.dst, n->comms[c.src], n->ranks[c.src].st);
      if (r == ncclSuccess)
        r = n->nccl.recv(c.to, c.bytes, ncclUint8, (int)c.src, n->comms[c.dst], n->ranks[c.dst].st);
    }
    const ncclResult_t r2 = n->nccl.group_end();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return n->fail(SDCAS_E_HIP, "%s: RCCL %s", what, n->nccl.error_string(r != ncclSuccess ? r : r2));
    return SDCAS_OK;
  }
  // device-to-device copies on the receiving rank's stream, after the sender's work
  for (size_t r = 0; r < R; ++r) {
    (void)hipSetDevice(n->ranks[r].dev);
    if ((e = hipEventRecord(n->ranks[r].ev, n->ranks[r].st))) return n->hip_fail(e, what);
  }
  for (const Copy& c : copies) {
    if (!c.bytes) continue;
    Rank& d = n->ranks[c.dst];
    (void)hipSetDevice(d.dev);
    if (c.src != c.dst && (e = hipStreamWaitEvent(d.st, n->ranks[c.src].ev, 0))) return n->hip_fail(e, what);
    if ((e = hipMemcpyPeerAsync(c.to, d.dev, c.from, n->ranks[c.src].dev, c.bytes, d.st))) return n->hip_fail(e, what);
  }
  // the senders' buffers are free again once the receivers are past the copies
  for (size_t r = 0; r < R; ++r) {
    (void)hipSetDevice(n->ranks[r].dev);
    if ((e = hipEventRecord(n->ranks[r].ev, n->ranks[r].st))) return n->hip_fail(e, what);
  }
  for (size_t r = 0; r < R; ++r)
    for (size_t d = 0; d < R; ++d)
      if (d != r) {
        (void)hipSetDevice(n->ranks[r].dev);
        if ((e = hipStreamWaitEvent(n->ranks[r].st, n->ranks[d].ev, 0))) return n->hip_fail(e, what);
      }
  return SDCAS_OK;
}

// SDCAS_NODE_TRACE=1: one stderr line per host wait of a node call (the
// dedup waits once for the owner ranges and once for the results, whatever
// the number of ranks)
bool node_trace() {
  const char* v = getenv("SDCAS_NODE_TRACE");
  return v && *v && strcmp(v, "0") != 0;
}

void trace_wait(const sdcas_node* n, const char* phase) {
  if (node_trace()) fprintf(stderr, "sdcas_node: host wait [%s] over %zu ranks\n", phase, n->ranks.size());
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// after a traced wait: how long the host waited, and the call's time so far
void trace_waited(const sdcas_node* n, const char* phase, std::chrono::steady_clock::time_point t_wait) {
  if (node_trace())
    fprintf(stderr, "sdcas_node: waited [%s] %.3f ms, call at %.3f ms\n", phase, ms_since(t_wait), ms_since(n->t_call));
}

int sync_all(sdcas_node* n, const char* what) {
  trace_wait(n, what);
  const auto t0 = std::chrono::steady_clock::now();
  for (Rank& k : n->ranks) {
    (void)hipSetDevice(k.dev);
    hipError_t e = hipStreamSynchronize(k.st);
    if (e) return n->hip_fail(e, what);
  }
  trace_waited(n, what, t0);
  return SDCAS_OK;
}

// contiguous ranges of [0, n) with about equal weight each
std::vector<size_t> cut_ranges(size_t n, size_t R, const std::vector<uint64_t>& w) {
  std::vector<size_t> cut(R + 1, n);
  cut[0] = 0;
  uint64_t total = 0;
  for (uint64_t x : w) total += x;
  uint64_t acc = 0;
  size_t r = 1;
  for (size_t i = 0; i < n && r < R; ++i) {
    acc += w[i];
    while (r < R && acc * R >= total * r) cut[r++] = i + 1;
  }
  for (; r < R; ++r) cut[r] = n;
  return cut;
}

}  // namespace

extern "C" {

int sdcas_node_init(const int32_t* devices, size_t n_devices, const sdcas_options* opts, sdcas_node** out) {
  if (!out || !devices || n_devices == 0 || n_devices > 64) return SDCAS_E_INVALID;
  *out = nullptr;
  if (opts && opts->struct_size != sizeof(sdcas_options)) return SDCAS_E_INVALID;
  auto* n = new sdcas_node();
  n->ranks.resize(n_devices);
  if (opts) {
    n->progress = opts->progress;
    n->progress_user = opts->progress_user;
  }
  n->slots.resize(n_devices);
  int rc = SDCAS_OK;
  for (size_t r = 0; r < n_devices && rc == SDCAS_OK; ++r) {
    n->slots[r] = RankProgress{n, r};
    sdcas_options o = SDCAS_OPTIONS_INIT;
    if (opts) o = *opts;
    o.device = devices[r];
    o.progress = node_progress;
    o.progress_user = &n->slots[r];
    Rank& k = n->ranks[r];
    k.dev = devices[r];
    rc = sdcas_init(&o, &k.ctx);
    if (rc) break;
    (void)hipSetDevice(k.dev);
    if (hipStreamCreateWithFlags(&k.st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&k.ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&k.ev_starts, hipEventDisableTiming) != hipSuccess)
      rc = SDCAS_E_NO_DEVICE;
  }
  // The exchange is device-to-device copies (hipMemcpyPeerAsync: over xGMI
  // between distinct GPUs, a local copy when a device repeats). RCCL between
  // distinct devices is opt-in (SDCAS_NODE_EXCHANGE=rccl; it refuses two ranks
  // on one device) until it has been run against the oracle on a multi-GPU box.
  std::vector<int> devs(devices, devices + n_devices);
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  const char* mode = getenv("SDCAS_NODE_EXCHANGE");
  if (rc == SDCAS_OK && distinct && n_devices > 1 && mode && !strcmp(mode, "rccl") && n->nccl.load()) {
    n->comms.resize(n_devices);
    if (n->nccl.comm_init_all(n->comms.data(), (int)n_devices, devs.data()) == ncclSuccess) n->rccl = true;
    else n->comms.clear();
  }
  if (rc) {
    sdcas_node_destroy(n);
    return rc;
  }
  *out = n;
  return SDCAS_OK;
}

void sdcas_node_destroy(sdcas_node* n) {
  if (!n) return;
  for (Rank& k : n->ranks) {
    if (k.st) {
      (void)hipSetDevice(k.dev);
      (void)hipStreamSynchronize(k.st);
    }
  }
  for (ncclComm_t c : n->comms) (void)n->nccl.comm_destroy(c);
  for (Rank& k : n->ranks) {
    (void)hipSetDevice(k.dev);
    k.release();
    if (k.ev) (void)hipEventDestroy(k.ev);
    if (k.ev_starts) (void)hipEventDestroy(k.ev_starts);
    if (k.st) (void)hipStreamDestroy(k.st);
    if (k.ctx) sdcas_destroy(k.ctx);
  }
  delete n;
}

const char* sdcas_node_last_error(const sdcas_node* n) { return n ? n->err.c_str() : ""; }

size_t sdcas_node_size(const sdcas_node* n) { return n ? n->ranks.size() : 0; }

int sdcas_node_uses_rccl(const sdcas_node* n) { return n && n->rccl ? 1 : 0; }

// ---- the batch path calls, sharded ------------------------------------------------

int sdcas_node_cas_ids(sdcas_node* n, const char* const* paths, const uint64_t* sizes, size_t nf, uint64_t* out_keys,
                       int32_t* out_status) {
  if (!n || (nf && (!paths || !sizes || !out_keys || !out_status))) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(n->mu);
  const size_t R = n->ranks.size();
  // contiguous ranges of about equal cas-message bytes (what each GPU reads and hashes)
  std::vector<uint64_t> w(nf);
  for (size_t i = 0; i < nf; ++i) w[i] = sdcas_cas_message_len(sizes[i]);
  const auto cut = cut_ranges(nf, R, w);
  for (Rank& k : n->ranks) k.done = k.total = 0;
  std::vector<int> rc(R, SDCAS_OK);
  std::vector<std::thread> th;
  for (size_t r = 0; r < R; ++r)
    th.emplace_back([&, r] {
      const size_t lo = cut[r], hi = cut[r + 1];
      if (hi > lo) rc[r] = sdcas_cas_ids(n->ranks[r].ctx, paths + lo, sizes + lo, hi - lo, out_keys + lo, out_status + lo);
    });
  for (auto& t : th) t.join();
  bool cancelled = false;
  for (size_t r = 0; r < R; ++r) {
    if (rc[r] == SDCAS_E_CANCELLED) cancelled = true;
    else if (rc[r]) return n->ctx_fail(r, rc[r], "sdcas_cas_ids");
  }
  return cancelled ? n->fail(SDCAS_E_CANCELLED, "cancelled") : SDCAS_OK;
}

int sdcas_node_checksums(sdcas_node* n, const char* const* paths, size_t nf, uint8_t* out32, int32_t* out_status) {
  if (!n || (nf && (!paths || !out32 || !out_status))) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(n->mu);
  const size_t R = n->ranks.size();
  // largest file first to the least loaded GPU (at most one
  // file of imbalance); a file that does not stat weighs nothing (its rank
  // reports its error)
  std::vector<uint64_t> size(nf, 0);
  for (size_t i = 0; i < nf; ++i) {
    struct stat sb;
    if (stat(paths[i], &sb) == 0) size[i] = (uint64_t)sb.st_size;
  }
  std::vector<size_t> order(nf);
  for (size_t i = 0; i < nf; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return size[a] > size[b]; });
  std::vector<uint64_t> load(R, 0);
  std::vector<std::vector<size_t>> mine(R);
  for (size_t i : order) {
    const size_t r = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
    mine[r].push_back(i);
    load[r] += size[i] + 4096;
  }
  for (auto& m : mine) std::sort(m.begin(), m.end());
  for (Rank& k : n->ranks) k.done = k.total = 0;
  std::vector<int> rc(R, SDCAS_OK);
  std::vector<std::thread> th;
  for (size_t r = 0; r < R; ++r)
    th.emplace_back([&, r] {
      const auto& m = mine[r];
      if (m.empty()) return;
      std::vector<const char*> p(m.size());
      for (size_t k = 0; k < m.size(); ++k) p[k] = paths[m[k]];
      std::vector<uint8_t> d(32 * m.size());
      std::vector<int32_t> s(m.size());
      rc[r] = sdcas_checksums(n->ranks[r].ctx, p.data(), m.size(), d.data(), s.data());
      if (rc[r] != SDCAS_OK && rc[r] != SDCAS_E_CANCELLED) return;
      for (size_t k = 0; k < m.size(); ++k) {
        memcpy(out32 + 32 * m[k], &d[32 * k], 32);
        out_status[m[k]] = s[k];
      }
    });
  for (auto& t : th) t.join();
  bool cancelled = false;
  for (size_t r = 0; r < R; ++r) {
    if (rc[r] == SDCAS_E_CANCELLED) cancelled = true;
    else if (rc[r]) return n->ctx_fail(r, rc[r], "sdcas_checksums");
  }
  return cancelled ? n->fail(SDCAS_E_CANCELLED, "cancelled") : SDCAS_OK;
}

// ---- the identifier group-by over the node ------------------------------------------
//
// The batch's orphans are cut into one contiguous range of ordinals per rank
// and the existing Objects into contiguous ranges of DB indices; then, per
// rank on its own stream: stays -> (all-gather) -> plan; combine files and
// existing Objects into owner-grouped records (their owner ranges go to the
// host: in one process that costs a stream sync, not a network round);
// exchange -> resolve on the owner -> exchange back -> apply. The result has
// sdcas_dedup_window's encoding over the batch's ordinals.
int sdcas_node_dedup_window(sdcas_node* n, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                            size_t nf, size_t chunk_size, const uint64_t* existing_keys, size_t n_existing,
                            sdcas_job_window* win, int64_t* out_link, int64_t* out_created, int64_t* out_linked) {
  if (!n || (nf && (!keys || !has_key || !out_link)) || (n_existing && !existing_keys)) return SDCAS_E_INVALID;
  if ((uint64_t)nf + n_existing > (1ull << 30))
    return n->fail(SDCAS_E_CAPACITY, "node dedup of %zu files + %zu Objects exceeds 2^30", nf, n_existing);
  std::lock_guard<std::mutex> g(n->mu);
  n->t_call = std::chrono::steady_clock::now();
  const size_t R = n->ranks.size();
  const uint32_t world = (uint32_t)R;
  if (chunk_size == 0) chunk_size = SDCAS_IDENTIFIER_CHUNK_SIZE;
  hipError_t e;
  int rc;
  // shards
  {
    std::vector<uint64_t> one(nf, 1), eone(n_existing, 1);
    const auto cut = cut_ranges(nf, R, one), ecut = cut_ranges(n_existing, R, eone);
    for (size_t r = 0; r < R; ++r) {
      Rank& k = n->ranks[r];
      k.lo = cut[r], k.hi = cut[r + 1], k.elo = ecut[r], k.ehi = ecut[r + 1];
    }
  }
  // this rank's stays rows: the host holds the flags, so the counts are exact
  std::vector<size_t> nstay(R, 0);
  for (size_t r = 0; r < R; ++r)
    for (size_t i = n->ranks[r].lo; i < n->ranks[r].hi; ++i) nstay[r] += (status && status[i]) || !has_key[i];
  size_t stays_total = 0;
  for (size_t c : nstay) stays_total += c;
  // upload + stays, per rank
  for (size_t r = 0; r < R; ++r) {
    Rank& k = n->ranks[r];
    const size_t m = k.hi - k.lo, me = k.ehi - k.elo;
    (void)hipSetDevice(k.dev);
    if ((e = k.keys.ensure(m)) || (e = k.ids.ensure(m)) || (e = k.has.ensure(m)) || (e = k.status.ensure(m)) ||
        (e = k.slot.ensure(m)) || (e = k.link.ensure(m)) || (e = k.rec.ensure(2 * m)) || (e = k.ekeys.ensure(me)) ||
        (e = k.eids.ensure(me)) || (e = k.erec.ensure(2 * me)) || (e = k.stays.ensure(nstay[r])) ||
        (e = k.gstays.ensure(stays_total)) || (e = k.plan.ensure(SDCAS_PLAN_WORDS(stays_total))) ||
        (e = k.counts.ensure(2)) || (e = k.scount.ensure(1)))
      return n->hip_fail(e, "node dedup buffers");
    if ((m && ((e = hipMemcpyAsync(k.keys.p, keys + k.lo, 8 * m, hipMemcpyHostToDevice, k.st)) ||
               (e = hipMemcpyAsync(k.has.p, has_key + k.lo, m, hipMemcpyHostToDevice, k.st)) ||
               (status && (e = hipMemcpyAsync(k.status.p, status + k.lo, 4 * m, hipMemcpyHostToDevice, k.st))))) ||
        (me && (e = hipMemcpyAsync(k.ekeys.p, existing_keys + k.elo, 8 * me, hipMemcpyHostToDevice, k.st))) ||
        (e = hipMemsetAsync(k.counts.p, 0, 16, k.st)))
      return n->hip_fail(e, "node dedup H2D");
    if (m) hipLaunchKernelGGL(k_iota_from, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, k.st, k.ids.p, (uint64_t)k.lo, (uint32_t)m);
    if (me) hipLaunchKernelGGL(k_iota_from, dim3((unsigned)((me + 255) / 256)), dim3(256), 0, k.st, k.eids.p, (uint64_t)k.elo, (uint32_t)me);
    if ((rc = sdcas_dev_dedup_stays(k.ctx, k.has.p, status ? k.status.p : nullptr, k.ids.p, m, nstay[r], k.stays.p,
                                    k.scount.p, k.st)))
      return n->ctx_fail(r, rc, "dedup_stays");
  }
  // all-gather the stays ordinals; every rank builds the same plan
  {
    std::vector<Copy> cp;
    for (size_t d = 0; d < R; ++d) {
      size_t off = 0;
      for (size_t r = 0; r < R; ++r) {
        cp.push_back(Copy{r, d, n->ranks[r].stays.p, n->ranks[d].gstays.p + off, 8 * nstay[r]});
        off += nstay[r];
      }
    }
    if ((rc = exchange(n, cp, "stays all-gather"))) return rc;
    for (size_t d = 0; d < R; ++d) {
      Rank& k = n->ranks[d];
      if ((rc = sdcas_dev_dedup_plan(k.ctx, k.gstays.p, stays_total, nf, chunk_size, win ? win->max_steps : 0,
                                     win ? win->more : 0, k.plan.p, k.st)))
        return n->ctx_fail(d, rc, "dedup_plan");
    }
  }
  // combine: every rank's files and existing Objects are enqueued before any
  // owner range is read, so the GPUs sort concurrently and the host waits
  // once for the phase (the ranges size the exchange exactly)
  std::vector<std::vector<uint64_t>> fcnt(R, std::vector<uint64_t>(R, 0)), ecnt(R, std::vector<uint64_t>(R, 0));
  for (size_t r = 0; r < R; ++r) {
    Rank& k = n->ranks[r];
    const size_t m = k.hi - k.lo, me = k.ehi - k.elo;
    (void)hipSetDevice(k.dev);
    if ((e = k.dstarts.ensure(2 * (R + 1)))) return n->hip_fail(e, "node dedup buffers");
    if (k.hstarts_cap < 2 * (R + 1)) {
      if (k.hstarts) (void)hipHostFree(k.hstarts);
      k.hstarts = nullptr;
      k.hstarts_cap = 0;
      if ((e = hipHostMalloc(&k.hstarts, sizeof(uint32_t) * 2 * (R + 1), hipHostMallocDefault)))
        return n->hip_fail(e, "node dedup pinned ranges");
      k.hstarts_cap = 2 * (R + 1);
    }
    if ((rc = sdcas_dev_dedup_combine_async(k.ctx, k.keys.p, k.has.p, status ? k.status.p : nullptr, k.ids.p, m,
                                            world, k.rec.p, k.slot.p, k.dstarts.p, k.st)))
      return n->ctx_fail(r, rc, "dedup_combine");
    if ((rc = sdcas_dev_dedup_combine_async(k.ctx, k.ekeys.p, nullptr, nullptr, k.eids.p, me, world, k.erec.p, nullptr,
                                            k.dstarts.p + (R + 1), k.st)))
      return n->ctx_fail(r, rc, "dedup_combine (existing)");
    (void)hipSetDevice(k.dev);
    if ((e = hipMemcpyAsync(k.hstarts, k.dstarts.p, sizeof(uint32_t) * 2 * (R + 1), hipMemcpyDeviceToHost, k.st)) ||
        (e = hipEventRecord(k.ev_starts, k.st)))
      return n->hip_fail(e, "node dedup owner ranges");
  }
  trace_wait(n, "owner ranges");
  const auto t_ranges = std::chrono::steady_clock::now();
  for (size_t r = 0; r < R; ++r) {
    Rank& k = n->ranks[r];
    (void)hipSetDevice(k.dev);
    if ((e = hipEventSynchronize(k.ev_starts))) return n->hip_fail(e, "node dedup owner ranges");
    k.starts.assign(k.hstarts, k.hstarts + (R + 1));
    k.estarts.assign(k.hstarts + (R + 1), k.hstarts + 2 * (R + 1));
    for (size_t d = 0; d < R; ++d) {
      fcnt[r][d] = k.starts[d + 1] - k.starts[d];
      ecnt[r][d] = k.estarts[d + 1] - k.estarts[d];
    }
  }
  trace_waited(n, "owner ranges", t_ranges);
  // records to their owners
  std::vector<size_t> nf_recv(R, 0), ne_recv(R, 0);
  for (size_t d = 0; d < R; ++d)
    for (size_t r = 0; r < R; ++r) nf_recv[d] += fcnt[r][d], ne_recv[d] += ecnt[r][d];
  {
    std::vector<Copy> cp;
    for (size_t d = 0; d < R; ++d) {
      Rank& kd = n->ranks[d];
      (void)hipSetDevice(kd.dev);
      if ((e = kd.frecv.ensure(2 * nf_recv[d])) || (e = kd.erecv.ensure(2 * ne_recv[d])) ||
          (e = kd.answer.ensure(nf_recv[d])))
        return n->hip_fail(e, "node dedup receive buffers");
      size_t fo = 0, eo = 0;
      for (size_t r = 0; r < R; ++r) {
        Rank& kr = n->ranks[r];
        cp.push_back(Copy{r, d, kr.rec.p + 2 * kr.starts[d], kd.frecv.p + 2 * fo, 16 * fcnt[r][d]});
        cp.push_back(Copy{r, d, kr.erec.p + 2 * kr.estarts[d], kd.erecv.p + 2 * eo, 16 * ecnt[r][d]});
        fo += fcnt[r][d];
        eo += ecnt[r][d];
      }
    }
    if ((rc = exchange(n, cp, "record exchange"))) return rc;
  }
  for (size_t d = 0; d < R; ++d) {
    Rank& k = n->ranks[d];
    if (nf_recv[d] && (rc = sdcas_dev_dedup_resolve(k.ctx, k.frecv.p, nf_recv[d], k.erecv.p, ne_recv[d],
                                                    k.answer.p, k.st)))
      return n->ctx_fail(d, rc, "dedup_resolve");
  }
  // answers back, in each rank's send order
  {
    std::vector<Copy> cp;
    for (size_t r = 0; r < R; ++r) {
      Rank& kr = n->ranks[r];
      (void)hipSetDevice(kr.dev);
      if ((e = kr.back.ensure(kr.starts[R] + 1))) return n->hip_fail(e, "node dedup answer buffers");
    }
    for (size_t d = 0; d < R; ++d) {
      size_t fo = 0;
      for (size_t r = 0; r < R; ++r) {
        Rank& kr = n->ranks[r];
        cp.push_back(Copy{d, r, n->ranks[d].answer.p + fo, kr.back.p + kr.starts[d], 8 * fcnt[r][d]});
        fo += fcnt[r][d];
      }
    }
    if ((rc = exchange(n, cp, "answer exchange"))) return rc;
  }
  // apply, results home
  std::vector<std::array<uint64_t, 2>> cnt(R);
  uint64_t hdr[SDCAS_PLAN_HEADER_WORDS] = {};
  for (size_t r = 0; r < R; ++r) {
    Rank& k = n->ranks[r];
    const size_t m = k.hi - k.lo;
    if (m && (rc = sdcas_dev_dedup_apply(k.ctx, k.ids.p, k.slot.p, m, k.back.p, chunk_size,
                                         k.plan.p, k.link.p, k.counts.p, k.st)))
      return n->ctx_fail(r, rc, "dedup_apply");
    (void)hipSetDevice(k.dev);
    if ((m && (e = hipMemcpyAsync(out_link + k.lo, k.link.p, 8 * m, hipMemcpyDeviceToHost, k.st))) ||
        (e = hipMemcpyAsync(cnt[r].data(), k.counts.p, 16, hipMemcpyDeviceToHost, k.st)) ||
        (r == 0 && (e = hipMemcpyAsync(hdr, k.plan.p, sizeof hdr, hipMemcpyDeviceToHost, k.st))))
      return n->hip_fail(e, "node dedup D2H");
  }
  if ((rc = sync_all(n, "results"))) return rc;
  int64_t created = 0, linked = 0;
  for (auto& c : cnt) created += (int64_t)c[0], linked += (int64_t)c[1];
  if (out_created) *out_created = created;
  if (out_linked) *out_linked = linked;
  if (win) {
    win->steps = hdr[2];
    win->rows = hdr[3];
    win->rereads = hdr[8];
  }
  return SDCAS_OK;
}

int sdcas_node_set_progress(sdcas_node* n, sdcas_progress_fn progress, void* user, const volatile int32_t* cancel) {
  if (!n) return SDCAS_E_INVALID;
  std::lock_guard<std::mutex> g(n->mu);
  {
    std::lock_guard<std::mutex> p(n->prog_mu);
    n->progress = progress;
    n->progress_user = user;
  }
  for (size_t r = 0; r < n->ranks.size(); ++r) {
    const int rc = sdcas_set_progress(n->ranks[r].ctx, node_progress, &n->slots[r], cancel);
    if (rc) return n->ctx_fail(r, rc, "sdcas_set_progress");
  }
  return SDCAS_OK;
}

}  // extern "C"
