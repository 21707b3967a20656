// b3_batch.h — host-side interface of the batched multi-message BLAKE3 engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdcas {

constexpr uint32_t kTile = 1024;  // chunk slots per workgroup tile (1 MiB of message bytes)
constexpr uint32_t kWG = 512;     // threads per workgroup: 2 slots per lane
// Batches of at most kSmallSlots chunk slots (the staging slots of a path call
// that small, e.g. the reference's 100-file step) run the small-batch kernel:
// tiles of kSmallTile slots, so that they spread over many CUs instead of
// running a few 1 MiB tiles one CU each (leaf variant kSmallVariant: since
// round 4 variant 73, a quad of lanes per slot — sdcas_cas_ids of 1 / 10 /
// 100 / 300 files 68.3 / 124.8 / 291.9 / 545.7 us -> 53.1 / 112.0 / 280.1 /
// 521.6 us against 71, profiles/r04_small_quad.json; since round 6 variant
// 84, 73 with four blocks of each chunk in flight and each quad's block
// staged in LDS, profiles/r06_latency_small.json).
constexpr uint32_t kSmallTile = 128;
constexpr uint64_t kSmallSlots = 1ull << 14;
constexpr int kSmallVariant = 84;
// The shape sort's workspace: the 256 bin totals, then each scatter
// workgroup's (kSortPerWG messages) count per bin, bin-major.
constexpr uint32_t kSortTotalsWords = 256;
constexpr uint32_t kSortPerWG = 4096;
inline size_t sort_key_words(size_t max_msgs) { return kSortTotalsWords + 256 * (max_msgs / kSortPerWG + 1); }

// Device workspace owned by the library context (caller never sees it).
struct BatchWorkspace {
  uint64_t* S = nullptr;           // [cap_msgs] first slot of each message
  uint32_t* tile_first = nullptr;  // [cap_tiles] message owning each tile's first slot
  uint64_t* total = nullptr;       // [4] total slots, error word, leaf tile counter
  uint32_t* nodes = nullptr;       // [cap_chunks * 8] maximal in-tile node CVs, by first slot
  void* scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  uint32_t cap_msgs = 0;
  uint64_t cap_chunks = 0;  // chunks a batch of up to cap_msgs messages may hold
  uint64_t cap_slots = 0;   // slots the workspace holds (chunks + the quad layout's padding)
  int variant = -1;  // leaf kernel variant (-1: default / SDCAS_LEAF_VARIANT; unavailable ones: default)
  uint64_t small_slots = kSmallSlots;  // default variant: batches up to this many slots take the small kernel (0: never)
  int small_variant = kSmallVariant;   // which small-tile variant (A/B runs)
  uint64_t cap_small_tiles = 0;        // tile_first entries (the small kernel's tiles need kTile / kSmallTile times more)
  // length-sorted slot order (messages of equal length share waves, so the
  // lanes of a wave run the same number of blocks): perm[slot-order index] =
  // caller index; soffs/slens = offsets/lengths in slot order
  int sort = 1;
  uint32_t* perm = nullptr;        // [cap_msgs]
  uint64_t* soffs = nullptr;       // [cap_msgs]
  uint64_t* slens = nullptr;       // [cap_msgs]
  uint32_t* sort_keys = nullptr;   // [sort_key_words(cap_msgs)] shape-bin totals and per-workgroup counts
};

size_t batch_scan_temp_bytes(uint32_t max_msgs);
int leaf_variant();
int leaf_variant_count();
bool leaf_variant_available(int v);  // compiled into this build (the diagnostic ones never are in libsdcas.so)
bool leaf_variant_forced();          // SDCAS_LEAF_VARIANT names an available variant
bool piece_variant_available(int v);

// A small batch's slot plan, computed by a caller that has the lengths on the
// host (the staging path) and uploaded with them: what the scan and
// k_tile_first would write for tiles of `tile` slots, so that batch_hash
// launches neither; `crossing` = some message spans a tile boundary (else
// k_finish_t has nothing to do and is not launched either). Used only for a
// batch the kernel takes in caller order (fewer than kSortMinMsgs messages)
// with that tile size; any other batch plans on the device.
constexpr uint32_t kSortMinMsgs = 128;  // smaller batches keep the caller's order
struct BatchPlan {
  const uint64_t* S = nullptr;           // device: first slot of each message
  const uint32_t* tile_first = nullptr;  // device: message owning each tile's first slot
  uint64_t* total = nullptr;             // device: [4] total slots, 0, 0 (leaf tile counter), 0
  uint32_t tile = 0;
  bool crossing = true;
};
// Host side of BatchPlan: S[n], tile_first[tiles] and total[4] for tiles of
// `tile` slots (tile_first entries below cap_slots only, as k_tile_first);
// returns the tile count and sets *crossing.
uint64_t batch_plan_host(const uint64_t* lens, uint32_t n, uint32_t tile, uint64_t cap_slots, uint64_t* S,
                         uint32_t* tile_first, uint64_t* total, bool* crossing);

// Hash n messages (blob + offs[i], lens[i] bytes; offsets 16-byte aligned),
// all pointers device pointers. Writes 32-byte digests to out32 and/or cas
// keys (digest bytes 0..7 big-endian) to out_keys (either may be null).
// Total chunks must not exceed ws.cap_chunks (checked by the caller).
// max_chunks: the batch's chunk count if the caller knows it (the staging
// slots do), which sizes the leaf and finish grids to the batch; 0 sizes them
// to the workspace (device-resident batches, whose lengths the host never
// sees).
hipError_t batch_hash(const BatchWorkspace& ws, const uint8_t* blob, const uint64_t* offs, const uint64_t* lens,
                      uint32_t n, uint8_t* out32, uint64_t* out_keys, hipStream_t st, uint64_t max_chunks = 0,
                      hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, const BatchPlan* plan = nullptr);

// ---- big files (C > kTile chunks), hashed as 1 MiB pieces -------------------
struct PieceDesc {
  uint64_t off;        // byte offset of the piece in the blob (16-byte aligned)
  uint64_t j0;         // first chunk index (multiple of kTile)
  uint64_t node_base;  // file's first entry in the file-node list
  uint32_t len;        // bytes (<= 1 MiB; < 1 MiB only for a file's last piece)
  uint32_t pad;
};
// A segment of a device-resident stream update (sdcas_dev_stream_update): a
// run of whole 1 MiB pieces of one message, expanded into PieceDescs on the
// device (expand_pieces) so that the host never builds or uploads the
// per-piece list.
struct SegDesc {
  uint64_t off;          // byte offset of the segment in the blob
  uint64_t j0;           // first chunk index (multiple of kTile)
  uint64_t node_base;    // message's first entry in the node list
  uint64_t len;          // bytes (a multiple of 1 MiB unless the segment ends the message)
  uint64_t piece_first;  // index of the segment's first piece in the update (exclusive scan)
};
struct FileDesc {
  uint64_t C;          // file chunk count (> kTile)
  uint64_t node_base;  // first entry in the file-node list (Q + popcount(C mod kTile) entries)
  uint64_t out_index;  // digest slot in out32
};
inline uint64_t bigfile_node_count(uint64_t C) {
  return C / kTile + (uint64_t)__builtin_popcountll(C % kTile);
}
// Piece variant 19 stops a full piece's tree at this level and finishes the
// levels above it over many pieces at once (k_piece_top).
constexpr uint32_t kPieceDeferLevel = 4;
// device scratch of piece_hash's l4 argument: u32 words per piece
constexpr uint64_t kPieceL4Words = 8ull * (kTile >> kPieceDeferLevel);
// ctr: one u32 of device scratch (the persistent variants' piece counter);
// l4: kPieceL4Words * npieces u32 of device scratch (variant 19);
// variant: piece kernel variant (-1: default / SDCAS_PIECE_VARIANT)
hipError_t piece_hash(const uint8_t* blob, const PieceDesc* pieces, uint32_t npieces, uint32_t* file_nodes,
                      uint32_t* ctr, uint32_t* l4, int variant, hipStream_t st);
// pieces[piece_first(k) ..] of every segment k; one thread per piece
hipError_t expand_pieces(const SegDesc* segs, uint32_t nseg, PieceDesc* pieces, uint32_t npieces, hipStream_t st);
hipError_t bigfile_finish(const FileDesc* files, uint32_t nfiles, const uint32_t* file_nodes, uint8_t* out32,
                          hipStream_t st);

}  // namespace sdcas
