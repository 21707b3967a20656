// dist_dedup.h — device stages of the multi-GPU cas_id -> Object group-by
// (SURVEY.md §8e): combine (per rank) -> all-to-all -> resolve (per owner)
// -> all-to-all back -> apply (per rank). The collectives are the caller's
// (RCCL through torch.distributed in spacedrive_amd/dist_dedup.py); these
// stages only touch this GPU's HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdcas {

// slot codes of files that own no combined record
constexpr uint32_t kSlotNoKey = 0xFFFFFFFFu;    // cas_id None: the file creates its own Object
constexpr uint32_t kSlotDropped = 0xFFFFFFFEu;  // I/O error: the file is dropped

// owner rank of a cas key: the top 12 bits (the 3-hex thumbnail shard prefix,
// object/media/thumbnail/shard.rs:10-13) split into `world` equal, contiguous
// bucket ranges, so owner() is monotone in the key and a key-sorted record
// array is already grouped by owner
__host__ __device__ inline uint32_t dd_owner(uint64_t key, uint32_t world) {
  return (uint32_t)(((key >> 52) * (uint64_t)world) >> 12);
}

struct DistWs {
  template <class T>
  struct Buf {
    T* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
      if (n <= cap) return hipSuccess;
      if (p) (void)hipFree(p);
      p = nullptr;
      cap = 0;
      size_t want = n < 16 ? 16 : n;
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
  Buf<uint32_t> idx_a, idx_b, starts;  // the combine's table, the files' slots, owner starts (and resolve's cfg)
  Buf<uint32_t> ocnt;                  // the combine's per-owner record counts / fills
  Buf<uint64_t> tkey, tmin;  // resolve's hash table: keys, (files' min, existing min) per entry
  Buf<uint32_t> tpos;        // table entry of each received file record
  Buf<uint32_t> stay_idx, nstay;  // the batch's stay-orphan rows (dd_local's plan)
  Buf<uint32_t> stay_cnt;         // per-tile stays counts (select_stays, the fused insert, the bitmap)
  Buf<uint32_t> flag;              // the fused insert's non-contiguous-ordinals flag
  Buf<unsigned long long> shard;  // the applies' (created, linked) counts, kCountShards pairs (kept zeroed)
  bool shard_dirty = false;       // a failed call may have left partial sums in `shard`: zero before use
  Buf<uint64_t> plan, stay_sorted;
  Buf<uint32_t> bitmap;           // dd_plan: the stays ordinals of a long gathered list
  Buf<uint64_t> ridx;             // the coarse index of a plan's re-read list (k_rr_index), stamped
  void release();
};

// ---- the job's steps over the batch (file_identifier_job.rs:180-236) ----------
//
// The reference reads its orphans CHUNK_SIZE at a time with id >= cursor, the
// cursor being the previous step's LAST row (file_identifier_job.rs:296-319,
// mod.rs:401-405). A row that stays an orphan after its step (an I/O error,
// mod.rs:125-141, or a cas_id of None, mod.rs:78-86 — "stays" rows) is read
// again by the next step when it was the last row, so every later step starts
// one row earlier. In the sequence of rows the steps read — a re-read row
// twice — step k covers positions [k*cs, (k+1)*cs): file ordinal o sits at
// position o + (re-reads of ordinals below o). The plan holds what that
// needs: the re-read ordinals, found by one wave walking the sorted stays
// ordinals, and the position limit of the steps the job may run.
constexpr uint32_t kPlanHeader = 12;  // u64 words before the re-read ordinals (SDCAS_PLAN_HEADER_WORDS)
enum : uint32_t {
  kPlanLimit = 0,    // first position not run (steps * cs)
  kPlanRereads = 1,  // re-read ordinals that follow the header (ascending)
  kPlanSteps = 2,    // steps run
  kPlanRows = 3,     // last ordinal the steps read + 1 (0: none)
  kPlanNTotal = 4,
  kPlanChunk = 5,
  kPlanLoop = 6,       // a row every remaining step reads again (all-ones: none); rows after it are not reached
  kPlanLoopReads = 7,  // how many steps read it
  kPlanRereadsRun = 8, // rows two steps the job runs read (sdcas_job_window.rereads)
  kPlanIndex = 9,      // the stamp of the re-read list's coarse index built for this plan (0: none)
};
struct StepWindow {
  uint64_t n_total = 0;    // the job's orphans are ordinals [0, n_total)
  uint64_t max_steps = 0;  // steps the job may run (0: ceil(n_total / cs), file_identifier_job.rs:146)
  uint32_t more = 0;       // more orphans follow ordinal n_total - 1: a step reaching past it is not run
};

// ordinals of this rank's stays rows -> out[0..cap) ascending, padded with
// all-ones; count (device int64) = every stays row, even past cap (the
// caller then gathers exactly)
hipError_t dd_stays(DistWs& w, const uint8_t* has_key, const int32_t* status, const uint64_t* ids, uint32_t n,
                    uint32_t cap, uint64_t* out, int64_t* count, hipStream_t st);
// the plan from every rank's stays ordinals (n_stays entries in any order,
// all-ones entries ignored) -> plan[kPlanHeader + n_stays] (device)
hipError_t dd_plan(DistWs& w, const uint64_t* stays, uint32_t n_stays, uint64_t cs, const StepWindow& win,
                   uint64_t* plan, hipStream_t st);

// Stage 1. keys/has_key/status/ids: [n] (has_key, status may be null = all
// present / all ok); ids ascending (the rank's files in orphan order, or the
// rank's existing Objects in DB order). Writes one (key, min id) record per
// distinct key to rec[2*u..2*u+1], grouped by owner (in no particular order
// within an owner's range), the
// record index of every file to slot[i] (or kSlotNoKey/kSlotDropped; slot may
// be null), and starts[0..world] (record index where each owner's range
// begins) to h_starts after a stream sync. Returns the record count in *h_u.
hipError_t dd_combine(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                      const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                      uint64_t* h_starts, uint64_t* h_u, hipStream_t st);

// Stage 1 with the owner ranges left on the device: starts[0..world] (u32,
// device) instead of the host copy, no host synchronisation, so that a
// process driving several GPUs enqueues every GPU's combine before it waits
// for any (sdcas_node_dedup_window).
hipError_t dd_combine_dev(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                          const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                          uint32_t* d_starts, hipStream_t st);

// Stage 1 into fixed-capacity owner buckets, without a host synchronisation:
// send[(r * cap + p) * 2 ..] = record p of owner r (p < counts[r] <= cap),
// counts[world] (device int64), slot[i] = bucket position r * cap + p of file
// i's record (or kSlotNoKey / kSlotDropped). *overflow (device) is set to 1
// when an owner has more than cap records: the buckets are then incomplete
// and the caller must use the exact path (dd_combine).
hipError_t dd_combine_buckets(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                              const uint64_t* ids, uint32_t n, uint32_t world, uint32_t cap, uint64_t* send,
                              uint32_t* slot, int64_t* counts, uint32_t* overflow, hipStream_t st);

// Stage 2 over received buckets: frec / erec hold world buckets of fcap / ecap
// records, bucket r's first fcounts[r] / ecounts[r] valid (device int64).
// result[r * fcap + p] answers file record p of bucket r (padding untouched).
hipError_t dd_resolve_buckets(DistWs& w, const uint64_t* frec, uint32_t fcap, const int64_t* fcounts,
                              const uint64_t* erec, uint32_t ecap, const int64_t* ecounts, uint32_t world,
                              int64_t* result, hipStream_t st);

// Stage 2 (owner). frec: nf received (key, min file id) records, erec: ne
// received (key, min DB index) records of existing Objects. result[p] for
// file record p = -(db+1) if an existing Object carries the key (the first in
// DB order), else the global minimum file id carrying the key.
hipError_t dd_resolve(DistWs& w, const uint64_t* frec, uint32_t nf, const uint64_t* erec, uint32_t ne,
                      int64_t* result, hipStream_t st);

// Stage 3. result: [U] per this rank's record (returned in send order).
// link[i] (global ids): INT64_MIN dropped; ids[i] creates; -(db+1) existing;
// rep id otherwise — a file in the chunk of the key's first file creates its
// own Object (mod.rs:246-254), later chunks link to that file's Object.
// counts[0..1] += (created, linked) (device, zeroed by the caller).
// With a plan (may be null: no stays rows and the steps read every row),
// chunks are the steps' positions, a file past the plan's limit is
// SDCAS_LINK_DEFERRED, and a re-read file without cas_id creates a second
// Object when its second read is inside the limit.
hipError_t dd_apply(DistWs& w, const uint64_t* ids, const uint32_t* slot, uint32_t n, const int64_t* result,
                    uint64_t chunk_size, const uint64_t* plan, int64_t* link, unsigned long long* counts,
                    hipStream_t st);

// Stages 1-3 fused for a world of one (no exchange, so no combine): files
// and existing Objects (ekeys/eids[ne], eids = DB order) go straight into the
// resolve table. Same link / counts as combine -> resolve -> apply. The plan
// is built from this batch's own stays rows (a world of one holds them all)
// into w.plan, whose header the caller may read after the call.
hipError_t dd_local(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                    const uint64_t* ids, uint32_t n, const uint64_t* ekeys, const uint64_t* eids, uint32_t ne,
                    uint64_t chunk_size, const StepWindow& win, int64_t* link, unsigned long long* counts,
                    hipStream_t st);

}  // namespace sdcas
