// Device-side planning of one shard of a direct (pinned-arena) host call.
//
// msha_digest_batch on a pinned arena (what the Go adapter does,
// go/pkg/processor/gpuhash.go) used to plan every shard's lanes on the host:
// alias detection over the whole batch, a counting sort of the lanes by (upload
// piece, descending block count), lane-indexed metadata. On one GPU that was
// ~25-30 ms of host work per 2^23-action storm before the first kernel could
// start, and it did not shrink with more GPUs (the host threads are shared).
// Here the host only marks which byte ranges of the arena a shard touches and
// stages the shard's raw (off, len) pairs; these kernels do the rest on the GPU
// in four passes over the shard's messages:
//
//   k_plan_remap    device offset of every message (caller offset through the
//                   granule map of the compacted upload) and, when the shard's
//                   payloads overlap, its slot in an open-addressing table keyed
//                   by (off, len): the slot keeps the smallest index with that
//                   key (atomicCAS claims, atomicMin keeps the first)
//   k_plan_keys     rep[i] = that first index (an alias folds into it, as the
//                   reference's N^2 EpochChange re-hashes do, epoch_target.go:
//                   486-505); lanes (rep[i] == i) get the bucket key (upload
//                   piece holding the payload's end) * B + (bmax - blocks),
//                   counted into a histogram; per piece, the lowest lane index
//   k_plan_scan     exclusive scan of the histogram; cut[c] = first lane of
//                   piece c; info = lane count
//   k_plan_scatter  each lane takes a position in its bucket (tile-aggregated
//                   atomics) and writes its lane-indexed off / len / digest slot
//
// Lanes end up grouped by the 64 MiB upload piece whose arrival completes their
// payloads (so each group hashes as soon as it lands) and, inside a group, by
// descending block count (a wave's lanes run equal block counts). The order
// inside a bucket is not stable; digests do not depend on it. The host reads
// back only the cuts, the per-piece minima and the lane count (and rep, for
// the alias fill).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.hpp"

namespace msha {

// Planner stamps: diagnostic build only (-DMSHA_PLAN_STAMPS, tools/plan_stamps.py).
// Thread 0 of every workgroup of the folded planner's kernels records the 100 MHz
// wall clock (s_memrealtime) at phase boundaries into a fixed slot (kind, block):
// 16 words a record, word 15 = HW_ID | XCC_ID << 32. The product build compiles
// every PLAN_STAMP to nothing.
enum PlanStampKind : uint32_t { kPsInsert = 0, kPsScatter = 1, kPsScan = 2, kPsFill = 3, kPsGate = 4, kPsLongs = 5 };
#ifdef MSHA_PLAN_STAMPS
__device__ uint64_t* g_plan_stamps;
__device__ uint32_t g_plan_stamp_per;  // records per kind
__device__ __forceinline__ void plan_stamp(uint32_t kind, uint32_t ph) {
  if (threadIdx.x != 0 || !g_plan_stamps || blockIdx.x >= g_plan_stamp_per) return;
  uint64_t* r = g_plan_stamps + ((uint64_t)kind * g_plan_stamp_per + blockIdx.x) * 16;
  r[ph] = __builtin_amdgcn_s_memrealtime();
  if (ph == 0)
    r[15] = (uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
            ((uint64_t)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32);
}
__device__ __forceinline__ void plan_stamp_val(uint32_t kind, uint32_t w, uint64_t v) {
  if (threadIdx.x != 0 || !g_plan_stamps || blockIdx.x >= g_plan_stamp_per) return;
  g_plan_stamps[((uint64_t)kind * g_plan_stamp_per + blockIdx.x) * 16 + w] = v;
}
#define PLAN_STAMP(kind, ph) plan_stamp(kind, ph)
#define PLAN_STAMP_VAL(kind, w, v) plan_stamp_val(kind, w, v)
#else
#define PLAN_STAMP(kind, ph)
#define PLAN_STAMP_VAL(kind, w, v)
#endif

// A wave-uniform lane's value (every use here names a lane found by a ballot):
// v_readlane, where __shfl is a ds_bpermute through the LDS crossbar -- the
// planner's LDS is busy enough with its atomics.
__device__ __forceinline__ uint32_t lane_value(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

__device__ __forceinline__ uint64_t dev_blocks_for(uint64_t len) { return (len >> 6) + ((len & 63) < 56 ? 1 : 2); }

__device__ __forceinline__ uint64_t plan_hash(uint64_t off, uint64_t len) {
  uint64_t h = off ^ (len * 0x9E3779B97F4A7C15ull);  // splitmix64 finaliser over both fields
  h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
  h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
  return h ^ (h >> 31);
}

__global__ __launch_bounds__(256) void k_plan_remap(PlanArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m) return;
  const uint64_t o = a.off[i], l = a.len[i];
  // A zero-length message needs no payload bytes (the kernel masks the whole
  // block it reads): it points at device offset 0, inside the arena.
  uint64_t d = 0;
  if (l) {
    const uint64_t r = o - a.glo;
    d = a.gmap[(r >> a.gshift) - a.gbase] + (r & ((1ull << a.gshift) - 1));
  }
  a.dev_off[i] = d;
  if (!a.table) return;
  uint64_t h = plan_hash(o, l) & a.tmask;
  const uint32_t me = (uint32_t)i + 1;  // 0 = empty slot
  for (;;) {
    // a plain read first: a claimed slot never empties, so a hot key (one
    // EpochChange payload named by thousands of messages) costs a cached read
    // per message, not a serialised atomic
    uint32_t v = __hip_atomic_load(&a.table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0) v = atomicCAS(&a.table[h], 0u, me);
    if (v == 0) break;
    const uint64_t j = v - 1;
    if (a.off[j] == o && a.len[j] == l) {  // same key: the slot keeps the smallest index
      if (me < v) atomicMin(&a.table[h], me);
      break;
    }
    h = (h + 1) & a.tmask;
  }
  a.slot[i] = (uint32_t)h;
}

// k_plan_keys and k_plan_scatter work on tiles of kPlanTile messages per
// workgroup and aggregate by key in an LDS table first: a tile holds few
// distinct keys (one per (piece, block count) it touches; a request batch: one),
// so each costs one global atomic per tile instead of one per message or per
// wave (wave-aggregated global atomics made these two kernels 3.5 ms of c5's
// 4 ms plan: ~2K waves of a piece queued on one hot counter).
constexpr uint32_t kPlanItems = 16;                  // messages per thread
constexpr uint32_t kPlanTile = 256 * kPlanItems;     // messages per workgroup
constexpr uint32_t kPlanSlots = 1024;                // LDS key table (power of two)
constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;

struct TileTable {
  uint32_t key[kPlanSlots];
  uint32_t cnt[kPlanSlots];
  uint32_t aux[kPlanSlots];  // keys: lowest lane index; scatter: the bucket base
};

__device__ __forceinline__ void tile_clear(TileTable& t, uint32_t aux0) {
  for (uint32_t j = threadIdx.x; j < kPlanSlots; j += blockDim.x) {
    t.key[j] = kEmptyKey;
    t.cnt[j] = 0;
    t.aux[j] = aux0;
  }
}

// The LDS slot of key k (claimed on first sight), or kPlanSlots when the table is full.
__device__ __forceinline__ uint32_t tile_slot(TileTable& t, uint32_t k) {
  uint32_t h = (k * 0x9E3779B1u) >> (32 - 10);  // 10 = log2(kPlanSlots)
  for (uint32_t probe = 0; probe < kPlanSlots; ++probe, h = (h + 1) & (kPlanSlots - 1)) {
    const uint32_t cur = t.key[h];
    if (cur == k) return h;
    if (cur == kEmptyKey) {
      const uint32_t prev = atomicCAS(&t.key[h], kEmptyKey, k);
      if (prev == kEmptyKey || prev == k) return h;
    }
  }
  return kPlanSlots;
}

// Wave-aggregated tile count: the lanes of a wave holding valid keys take one
// LDS atomic per distinct key among them (a request batch's wave: one), not
// one per lane -- 64 lanes adding to one LDS word serialise. Calls
// done(lane's slot, lane's rank) on every valid lane: slot < kPlanSlots is the
// tile table's entry (rank inside the tile), kPlanSlots the global counter
// (rank = global position); lanes are ranked in lane order, and the wave's
// lowest lane of each key is its leader (min_idx: atomicMin of its index into
// aux, the host planner's lowest lane per piece).
template <bool kMinAux, class Done>
__device__ __forceinline__ void wave_count(TileTable& t, uint32_t* gcnt, uint32_t* gmin, uint32_t B,
                                           bool valid, uint32_t k, uint32_t idx, Done&& done) {
  uint64_t pend = __ballot(valid);
  const unsigned lane = __lane_id();
  while (pend) {
    const int leader = __ffsll((long long)pend) - 1;
    const uint32_t k0 = lane_value(k, leader);
    const uint64_t same = __ballot(valid && k == k0) & pend;
    uint32_t j = 0, base = 0;
    if ((int)lane == leader) {
      const uint32_t c = (uint32_t)__popcll(same);
      j = tile_slot(t, k0);
      if (j < kPlanSlots) {
        base = atomicAdd(&t.cnt[j], c);
        if (kMinAux) atomicMin(&t.aux[j], idx);
      } else {
        base = atomicAdd(&gcnt[k0], c);
        if (kMinAux) atomicMin(&gmin[k0 / B], idx);
      }
    }
    j = lane_value(j, leader);
    base = lane_value(base, leader);
    if ((same >> lane) & 1) done(j, base + (uint32_t)__popcll(same & ((1ull << lane) - 1)));
    pend &= ~same;
  }
}

// Bucket key of message i when it is a lane (rep[i] == i): group * B + (bmax -
// blocks), group = region * pieces + (piece holding the payload's end); region
// 0 holds the long chains (the host uploads their payloads first and runs them
// on a head kernel of their own), region 1 the rest.
__device__ __forceinline__ uint32_t lane_key(const PlanArgs& a, uint64_t i, uint32_t* chunk_out) {
  const uint64_t l = a.len[i];
  const uint64_t end = a.dev_off[i] + (l ? l : 1) - 1;
  const uint64_t blocks = dev_blocks_for(l);
  const uint64_t region = a.long_blocks && blocks < a.long_blocks ? 1 : 0;
  const uint32_t chunk = (uint32_t)(region * (a.chunks - a.pieces) + min((uint64_t)(end >> a.piece_shift),
                                                                        a.pieces - 1));
  if (chunk_out) *chunk_out = chunk;
  return chunk * (uint32_t)a.B + (a.B > 1 ? (uint32_t)(a.bmax - blocks) : 0u);
}

__global__ __launch_bounds__(256) void k_plan_keys(PlanArgs a) {
  __shared__ TileTable t;
  tile_clear(t, 0xFFFFFFFFu);
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile;
#pragma unroll 4
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const uint64_t i = base + r * 256 + threadIdx.x;
    bool lane_ok = i < a.m;
    uint32_t k = 0;
    if (lane_ok) {
      const uint32_t rp = a.table ? a.table[a.slot[i]] - 1 : (uint32_t)i;
      a.rep[i] = rp;
      lane_ok = rp == (uint32_t)i;
      if (lane_ok) k = lane_key(a, i, nullptr);
    }
    // table full: straight to the global counters (lowest lane per piece)
    wave_count<true>(t, a.cnt, a.gmin, (uint32_t)a.B, lane_ok, k, (uint32_t)i, [](uint32_t, uint32_t) {});
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < kPlanSlots; j += blockDim.x) {
    if (t.key[j] == kEmptyKey || t.cnt[j] == 0) continue;
    atomicAdd(&a.cnt[t.key[j]], t.cnt[j]);
    atomicMin(&a.gmin[t.key[j] / (uint32_t)a.B], t.aux[j]);
  }
}

// One workgroup: exclusive scan of cnt[0, nb) in place (cnt becomes the
// buckets' first positions); cut[c] = first position of piece c's buckets,
// cut[chunks] = info[0] = lanes.
__global__ __launch_bounds__(1024) void k_plan_scan(PlanArgs a) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (a.nb + 1023) / 1024;
  const uint64_t b0 = min((uint64_t)t * per, a.nb), b1 = min(b0 + per, a.nb);
  uint32_t s = 0;
  for (uint64_t b = b0; b < b1; ++b) s += a.cnt[b];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;  // exclusive prefix of this thread's range
  for (uint64_t b = b0; b < b1; ++b) {
    const uint32_t c = a.cnt[b];
    a.cnt[b] = run;
    if (b % a.B == 0) a.cut[b / a.B] = run;
    run += c;
  }
  if (t == 1023) {
    a.cut[a.chunks] = part[1023];
    a.info[0] = part[1023];
  }
}

// Each lane takes the next position of its bucket: a rank inside its tile's key
// (LDS atomic), plus the tile's base in the bucket (one global atomic per key
// per tile), then writes its lane-indexed off / len / digest slot.
__global__ __launch_bounds__(256) void k_plan_scatter(PlanArgs a) {
  __shared__ TileTable t;
  tile_clear(t, 0);
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile;
  uint32_t slot[kPlanItems], rank[kPlanItems];
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const uint64_t i = base + r * 256 + threadIdx.x;
    slot[r] = kEmptyKey;
    const bool lane_ok = i < a.m && a.rep[i] == (uint32_t)i;
    const uint32_t k = lane_ok ? lane_key(a, i, nullptr) : 0u;
    // table full (slot kPlanSlots): a position straight from the global counter
    wave_count<false>(t, a.cnt, nullptr, 1, lane_ok, k, 0, [&](uint32_t j, uint32_t rk) {
      slot[r] = j;
      rank[r] = rk;
    });
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < kPlanSlots; j += blockDim.x)
    if (t.key[j] != kEmptyKey && t.cnt[j]) t.aux[j] = atomicAdd(&a.cnt[t.key[j]], t.cnt[j]);
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    if (slot[r] == kEmptyKey) continue;
    const uint64_t i = base + r * 256 + threadIdx.x;
    const uint32_t pos = slot[r] < kPlanSlots ? t.aux[slot[r]] + rank[r] : rank[r];
    a.lane_off[pos] = a.dev_off[i];
    a.lane_len[pos] = a.len[i];
    a.lane_slot[pos] = (uint32_t)i;
  }
}

hipError_t launch_plan(const PlanArgs& a, hipStream_t st) {
  if (a.m == 0) return hipSuccess;
  const unsigned grid = (unsigned)((a.m + 255) / 256);
  const unsigned tiles = (unsigned)((a.m + kPlanTile - 1) / kPlanTile);
  hipLaunchKernelGGL(k_plan_remap, dim3(grid), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_plan_keys, dim3(tiles), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(k_plan_scatter, dim3(tiles), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Device-resident batches (msha_digest_batch_device_planned): the same tile-
// aggregated bucket sort, over the caller's device arrays, with no host round
// trip. The lane count and the head of long chains stay on the GPU (info[]):
// the hash launches read them (kernels.hpp LaneGate), so the whole call is
// enqueued at once.
//
//   k_fold_tilemax, k_fold_tilescan, k_fold_insert   (folding only) messages
//                   that may repeat an earlier payload claim (off, len) in an
//                   open-addressing table; the claimer is the key's lane (any one
//                   will do: the digest is the same), rep[i] = that lane; and the
//                   lanes counted per descending block-count bucket
//   k_fold_keys     (no folding) the same count, every message a lane
//   k_fold_scan     one workgroup: bucket starts, lanes, the batch's lane blocks,
//                   its longest chain, and the head: lanes whose chain on the
//                   lane kernel would outlast the launch's floor (FoldArgs)
//   k_fold_scatter  order[position] = message; kNoLane past the last lane
// ---------------------------------------------------------------------------
// Ascending class of a message (kernels.hpp kFoldExactLen): exact length below
// 1 KiB, so a wave of lanes sorted together holds one length -- round 4 keyed by
// block count alone, and a 9-block bucket mixing 512-byte requests with 544-byte
// Batches left most of folded c5's request waves with two lengths, off the
// scalar-unit padding path (c2's 1,356 VALU instructions a block against ~1,400).
__device__ __forceinline__ uint32_t fold_class(uint64_t len) {
  if (len < kFoldExactLen) return (uint32_t)len;
  const uint64_t blocks = dev_blocks_for(len);
  if (blocks < 4096) return kFoldExactLen + (uint32_t)(blocks - kFoldLowBlocks);
  return kFoldExactLen + (4096 - kFoldLowBlocks) + (uint32_t)(63 - __clzll((long long)blocks)) - 12u;
}
__device__ __forceinline__ uint64_t fold_class_blocks(uint32_t c) {  // exact, or the lower bound (big classes)
  if (c < kFoldExactLen) return dev_blocks_for(c);
  if (c < kFoldExactLen + (4096 - kFoldLowBlocks)) return c - kFoldExactLen + kFoldLowBlocks;
  return 1ull << (c - (kFoldExactLen + (4096 - kFoldLowBlocks)) + 12);
}
__device__ __forceinline__ uint32_t fold_key(uint64_t len) {  // descending class
  return kFoldBuckets - 1 - fold_class(len);
}

// Candidates first (the host path's rule, msha_alias_first): a message whose
// offset is above every earlier message's cannot repeat an earlier payload, so
// it is its own lane without touching the table; only the others (a storm's
// EpochChange re-hashes: 5 %) probe and claim. A key first named by a
// non-candidate and then by candidates is hashed twice -- once for the
// non-candidate, once for the candidates' claimant -- with the same digest.
// Tiles of kPlanTile messages, 16 consecutive per thread; tmax[t] = the
// largest offset of tiles before t (k_fold_tilemax, then k_fold_tilescan).
//
// A thread's run of 16 consecutive messages is 128 bytes of off and 128 of len:
// with a.vec (both arrays 16-byte aligned) it loads as eight 16-byte vectors
// each -- every load instruction then moves whole 16-byte lane slices of a line
// the lane reads entirely, instead of 16 scalar 8-byte loads per array that
// each touch 64 lines for 8 bytes apiece (round 4: k_fold_insert moved 1.10 GB
// per c5 step for 134 MB of off/len).
__device__ __forceinline__ void load_run(const uint64_t* __restrict__ p, uint64_t base, uint64_t n, bool vec,
                                         uint64_t (&v)[kPlanItems]) {
  if (vec && base + kPlanItems <= n) {
    const uint4* q = reinterpret_cast<const uint4*>(p + base);
#pragma unroll
    for (uint32_t k = 0; k < kPlanItems / 2; ++k) {
      const uint4 x = q[k];
      v[2 * k] = (uint64_t)x.x | ((uint64_t)x.y << 32);
      v[2 * k + 1] = (uint64_t)x.z | ((uint64_t)x.w << 32);
    }
  } else {
#pragma unroll
    for (uint32_t r = 0; r < kPlanItems; ++r) v[r] = base + r < n ? p[base + r] : 0;
  }
}

// With the early head (a.long_blocks) the same pass also reads the tile's
// lengths and sizes it for k_fold_tilescan's decision: the tile's short
// messages' blocks (the lane kernel's share, without the distinct long
// payloads) and its longest chain, into tsum.
__global__ __launch_bounds__(256) void k_fold_tilemax(FoldArgs a) {
  __shared__ uint64_t part[256];
  __shared__ unsigned long long s_sum[4], s_max[4];
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile + (uint64_t)threadIdx.x * kPlanItems;
  uint64_t o[kPlanItems];
  load_run(a.off, base, a.n, a.vec, o);
  uint64_t m = 0;
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) m = max(m, o[r]);
  part[threadIdx.x] = m;
  const bool sizes = a.long_blocks && !a.early_fork;  // else k_fold_longs_gate decides
  if (sizes) {
    uint64_t l[kPlanItems];
    load_run(a.len, base, a.n, a.vec, l);
    uint64_t sum = 0, mx = 0;
#pragma unroll
    for (uint32_t r = 0; r < kPlanItems; ++r) {
      const uint64_t blocks = base + r < a.n ? dev_blocks_for(l[r]) : 0;
      mx = max(mx, blocks);
      if (blocks < a.long_blocks) sum += blocks;
    }
    for (uint32_t d = 32; d > 0; d >>= 1) {  // wave sums, then one LDS word per wave
      sum += __shfl_xor(sum, d);
      mx = max(mx, (uint64_t)__shfl_xor(mx, d));
    }
    if (__lane_id() == 0) s_sum[threadIdx.x >> 6] = sum, s_max[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  for (uint32_t d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < d) part[threadIdx.x] = max(part[threadIdx.x], part[threadIdx.x + d]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.tmax[blockIdx.x] = part[0];
    if (sizes) {
      a.tsum[2 * blockIdx.x] = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
      a.tsum[2 * blockIdx.x + 1] = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    }
  }
}

// One workgroup: the exclusive prefix max of the tile maxima and, with the early
// head, a first decision: when the short messages' blocks alone -- x
// wave_block_cycles over the SIMDs -- keep the lane kernel busy past the
// longest chain on the head (c5 on one GPU: ~60 M blocks against one 1,427-block
// chain), the early head cannot pay and stands down before listing anything
// (info[6] = 0; k_fold_longs then returns at once). Otherwise info[6] = 1 and
// k_fold_longs lists and claims the long payloads and decides on the exact rule.
__global__ __launch_bounds__(1024) void k_fold_tilescan(FoldArgs a, uint64_t tiles) {
  __shared__ uint64_t part[1024];
  __shared__ unsigned long long s_sum[16], s_max[16];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (tiles + 1023) / 1024;
  const uint64_t b0 = min((uint64_t)t * per, tiles), b1 = min(b0 + per, tiles);
  const bool sizes = a.long_blocks && !a.early_fork;  // else k_fold_longs_gate decides
  uint64_t m = 0, sum = 0, mx = 0;
  for (uint64_t b = b0; b < b1; ++b) {
    m = max(m, a.tmax[b]);
    if (sizes) {
      sum += a.tsum[2 * b];
      mx = max(mx, a.tsum[2 * b + 1]);
    }
  }
  part[t] = m;
  if (sizes) {
    for (uint32_t d = 32; d > 0; d >>= 1) {
      sum += __shfl_xor(sum, d);
      mx = max(mx, (uint64_t)__shfl_xor(mx, d));
    }
    if (__lane_id() == 0) s_sum[t >> 6] = sum, s_max[t >> 6] = mx;
  }
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive prefix max
    const uint64_t v = t >= d ? part[t - d] : 0ull;
    __syncthreads();
    part[t] = max(part[t], v);
    __syncthreads();
  }
  uint64_t run = t ? part[t - 1] : 0ull;  // exclusive
  for (uint64_t b = b0; b < b1; ++b) {
    const uint64_t v = a.tmax[b];
    a.tmax[b] = run;
    run = max(run, v);
  }
  if (sizes && t == 0) {
    unsigned long long ss = 0, sm = 0;
    for (int w = 0; w < 16; ++w) ss += s_sum[w], sm = max(sm, s_max[w]);
    const uint64_t t_body = ss * a.wave_block_cycles / (64ull * a.simds);
    const uint64_t t_head = sm * a.early_cycles;
    a.info[6] = sm >= a.long_blocks && t_body < t_head ? 1u : 0u;
  }
}

// The alias table's slots are 64-bit (epoch << 32 | message + 1): a slot whose
// epoch is not this call's is empty, so the table is never cleared between
// calls (the host clears it only when it is (re)allocated or the epoch wraps).
__device__ __forceinline__ uint32_t fold_claim(const FoldArgs& a, uint64_t i, uint64_t o, uint64_t l) {
  uint64_t h = plan_hash(o, l) & a.tmask;
  const uint64_t ep = (uint64_t)a.epoch << 32;
  const uint64_t me = ep | ((uint64_t)i + 1);
  for (;;) {
    // a plain read first: a claimed slot never empties within a call, and a hot
    // key (one payload named by thousands of messages) then costs a cached read
    uint64_t v = __hip_atomic_load(&a.table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((v & ~0xFFFFFFFFull) != ep) {  // empty: claim it
      const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&a.table[h]), v, me);
      if (prev == v) return (uint32_t)i;
      v = prev;
      if ((v & ~0xFFFFFFFFull) != ep) continue;  // not claimed by this call: look again
    }
    const uint64_t j = (v & 0xFFFFFFFFull) - 1;
    if (a.off[j] == o && a.len[j] == l) return (uint32_t)j;
    h = (h + 1) & a.tmask;
  }
}

// Lanes counted per descending block-count key in a tile's LDS histogram (and,
// for the power-of-two classes, their largest block count and block sum), then
// flushed to the global counters: one global atomic per key present in the tile.
struct FoldHist {
  uint32_t n[kFoldBuckets];
  unsigned long long bmax[kFoldBigBuckets], bsum[kFoldBigBuckets];
};
__device__ __forceinline__ void fold_hist_clear(FoldHist& h) {
  for (uint32_t j = threadIdx.x; j < kFoldBuckets; j += blockDim.x) h.n[j] = 0;
  if (threadIdx.x < kFoldBigBuckets) h.bmax[threadIdx.x] = h.bsum[threadIdx.x] = 0;
}
__device__ __forceinline__ void fold_hist_big(FoldHist& h, uint32_t k, uint64_t blocks) {
  if (k < kFoldBigBuckets) {  // >= 4,096 blocks (1/4 MiB): rare
    atomicMax(&h.bmax[k], (unsigned long long)blocks);
    atomicAdd(&h.bsum[k], (unsigned long long)blocks);
  }
}
__device__ __forceinline__ void fold_hist_add(FoldHist& h, uint64_t len) {
  const uint64_t blocks = dev_blocks_for(len);
  const uint32_t k = fold_key(len);
  atomicAdd(&h.n[k], 1u);
  fold_hist_big(h, k, blocks);
}
// Over a wave's valid lanes by key, for message i: the lanes sharing the first
// valid lane's key add once, together (a storm's wave: ~70 % one key, which one
// LDS atomic per lane serialises ~45 deep), the rest one each -- a loop of one
// atomic per distinct key measured far slower (exact-length classes: many keys a
// wave; profiles/r06_plan9/). The length is read again only for the rare
// power-of-two classes, whose block counts the head's cost model needs exactly.
__device__ __forceinline__ void fold_hist_add_wave_key(const FoldArgs& a, FoldHist& h, bool valid, uint32_t k,
                                                       uint64_t i) {
  const uint64_t any = __ballot(valid);
  if (!any) return;
  const uint32_t k0 = lane_value(k, __ffsll((long long)any) - 1);
  const uint64_t same = __ballot(valid && k == k0);
  const unsigned lane = __lane_id();
  if ((same >> lane) & 1) {
    if ((same & ((1ull << lane) - 1)) == 0) atomicAdd(&h.n[k0], (uint32_t)__popcll(same));
  } else if (valid) {
    atomicAdd(&h.n[k], 1u);
  }
  if (valid && k < kFoldBigBuckets) fold_hist_big(h, k, dev_blocks_for(a.len[i]));
}
// Each key present in the tile: one global atomic, whose return is the tile's
// offset in the key's bucket, kept in the tile's key list (FoldArgs::tkeys) for
// the scatter. nk: an LDS counter the caller zeroed before a barrier; every
// thread of the workgroup calls this.
__device__ __forceinline__ void fold_hist_flush(const FoldArgs& a, FoldHist& h, uint32_t& nk) {
  uint64_t* tl = a.tkeys + (uint64_t)blockIdx.x * kPlanTile;
  for (uint32_t j = threadIdx.x; j < kFoldBuckets; j += blockDim.x)
    if (h.n[j]) {
      const uint32_t off = atomicAdd(&a.cnt[j], h.n[j]);
      tl[atomicAdd(&nk, 1u)] = ((uint64_t)j << 32) | off;
    }
  if (threadIdx.x < kFoldBigBuckets && h.bsum[threadIdx.x]) {
    atomicMax(reinterpret_cast<unsigned long long*>(&a.big[threadIdx.x]), h.bmax[threadIdx.x]);
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.big[kFoldBigBuckets + threadIdx.x]), h.bsum[threadIdx.x]);
  }
  __syncthreads();
  if (threadIdx.x == 0) a.tkcount[blockIdx.x] = nk;
}

// Also counts the tile's lanes into the bucket histogram (what k_fold_keys
// does without folding): a fresh message is its own lane, a candidate is one
// when its claim returns itself -- so the lanes' metadata is read once.
// Round 5: each thread's 16 consecutive (off, len) load as 16-byte vectors
// (load_run), the tile's keys gather in LDS and go out as words of consecutive
// messages per wave instruction (whole lines, not 2 bytes per lane at a 32-byte
// stride), and the candidates' list is appended and the histogram counted
// wave-aggregated.

// Round 6: the tile prefix inside the insert (FoldArgs::tstat), a decoupled
// look-back: each tile posts its own largest offset (kTileAgg) as soon as it has
// it, then wave 0 combines the posts of the tiles before it, 64 a step, back to
// the nearest tile that has posted its inclusive prefix (kTileIncl), and posts
// its own. A post is 62 bits of offset (an arena offset past 2^62 bytes is
// clamped: the threshold then only folds less) and 2 bits of state; 0 = not yet.
//
// Waiting is on earlier tiles only, and a tile posts its own offset before it
// waits: the lowest unposted tile waits on nobody, and each XCD dispatches its
// tiles in order, so that tile is resident or next in line and the look-backs end.
// Still, one that has waited kLookbackSpins polls gives up and returns the largest
// threshold, under which no message is fresh and every one claims in the table --
// the same digests, less folding -- and counts itself in tstat[tiles] (tests expect
// 0; a -DMSHA_LOOKBACK_GIVEUP_TEST build forces it, tools/r06_race.sh).
constexpr uint64_t kTileAgg = 1ull << 62, kTileIncl = 2ull << 62, kTileVal = kTileAgg - 1;
constexpr uint32_t kLookbackSpins = 1u << 16;
__device__ __forceinline__ uint64_t tile_lookback_give_up(const FoldArgs& a) {
  if (__lane_id() == 0) {
    const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.tstat[tiles]), 1ull);
  }
  return kTileVal;
}
__device__ __forceinline__ uint64_t tile_lookback(const FoldArgs& a, uint64_t tile) {
#ifdef MSHA_LOOKBACK_GIVEUP_TEST  // test build only (tests/test_gpu_planned.py, tools/r06_race.sh)
  if (tile % 3 == 1) return tile_lookback_give_up(a);
#endif
  const unsigned lane = __lane_id();
  uint64_t acc = 0;
  uint32_t spins = 0;
  for (int64_t hi = (int64_t)tile - 1; hi >= 0; hi -= 64) {
    const int64_t j = hi - (int64_t)lane;  // lane 0 the nearest tile
    uint64_t v = j >= 0 ? __hip_atomic_load(&a.tstat[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kTileIncl;
    uint64_t incl;
    for (;;) {  // until every tile up to the nearest inclusive post has posted
      const uint64_t ready = __ballot(v != 0);
      incl = __ballot((v & ~kTileVal) == kTileIncl);
      const uint64_t need = incl ? ((incl & (0ull - incl)) << 1) - 1 : ~0ull;
      if ((ready & need) == need) break;
      if (++spins > kLookbackSpins) return tile_lookback_give_up(a);
      __builtin_amdgcn_s_sleep(2);
      if (v == 0) v = __hip_atomic_load(&a.tstat[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int stop = incl ? __ffsll((long long)incl) - 1 : 63;  // lanes 0..stop count
    uint64_t x = (int)lane <= stop ? (v & kTileVal) : 0ull;
    for (uint32_t d = 32; d > 0; d >>= 1) x = max(x, (uint64_t)__shfl_xor(x, d));
    acc = max(acc, x);
    if (incl) break;
  }
  return acc;
}

// trep's index of tile position p: a pad word after every 16, so the per-thread
// runs (thread t writes positions 16 t + r) hit 32 different banks, not 2
__device__ __forceinline__ uint32_t trep_at(uint32_t p) { return p + (p >> 4); }

__global__ __launch_bounds__(256, 4) void k_fold_insert(FoldArgs a) {
  __shared__ uint64_t wmax[4];
  __shared__ FoldHist hist;
  // the tile's key16 by position (trep_at): a lane's key, 0xFFFF for a folded
  // message (whose (rep, i) pair the claim writes). Round 6: 16 bits, not a 32-bit
  // representative a message -- 4 workgroups a CU in LDS instead of 3.
  __shared__ uint16_t trep[kPlanTile + kPlanTile / 16];
  __shared__ uint16_t cand[kPlanTile];   // candidates' positions in the tile
  __shared__ uint32_t ncand, nalias, nkeys;
  __shared__ uint64_t s_before;  // the largest offset of the tiles before this one
  PLAN_STAMP(kPsInsert, 0);
  fold_hist_clear(hist);
  if (threadIdx.x == 0) ncand = nalias = nkeys = 0;
  const uint64_t tile0 = (uint64_t)blockIdx.x * kPlanTile;
  const uint32_t lb = threadIdx.x * kPlanItems;
  const uint64_t base = tile0 + lb;
  const unsigned lane = __lane_id(), wave = threadIdx.x >> 6;
  uint64_t o[kPlanItems], l[kPlanItems];
  load_run(a.off, base, a.n, a.vec, o);
  load_run(a.len, base, a.n, a.vec, l);
  uint64_t m = 0;
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) m = max(m, o[r]);
  PLAN_STAMP(kPsInsert, 1);
  // in-tile prefix max: inclusive over the wave by shuffles, then the waves before
  uint64_t incl = m;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t v = (uint64_t)__shfl_up((unsigned long long)incl, d);
    if (lane >= d) incl = max(incl, v);
  }
  if (lane == 63) wmax[wave] = incl;
  __syncthreads();
  uint64_t run = (uint64_t)__shfl_up((unsigned long long)incl, 1);
  if (lane == 0) run = 0;
  for (uint32_t w = 0; w < wave; ++w) run = max(run, wmax[w]);  // max offset before this thread's run
  // Round 6: the tile's own largest offset is posted before anything else, and the
  // look-back (wave 0, after its share of the first pass) then overlaps the other
  // waves' first pass; the tiles before this one are applied in a second pass.
  if (a.tstat && threadIdx.x == 0) {
    const uint64_t own = min(max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3])), kTileVal);
    __hip_atomic_store(&a.tstat[blockIdx.x], (blockIdx.x ? kTileAgg : kTileIncl) | own, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  PLAN_STAMP(kPsInsert, 2);
  const bool first_ever = blockIdx.x == 0 && threadIdx.x == 0;
  // Candidates are few (c5: 5 %) but spread over every wave: claiming them in
  // place would run each wave's claim loop (a load -> CAS -> compare chain of
  // memory round trips) once per item row. They go to an LDS list instead and
  // the workgroup's threads claim them side by side.
  // First pass, against the tile's own earlier messages only: a message above them
  // all is fresh so far (bit r of `local`), the rest are candidates.
  uint32_t local = 0;
  uint32_t kk[kPlanItems / 2] = {};
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const uint64_t i = base + r;
    const bool valid = i < a.n;
    // above every earlier offset (a long message never: with the early head it
    // claims, so its representative is the one k_fold_longs lists)
    const bool lng = valid && a.long_blocks && dev_blocks_for(l[r]) >= a.long_blocks;
    const bool fresh = valid && !lng && (o[r] > run || (first_ever && r == 0));
    const bool is_cand = valid && !fresh;
    const uint32_t k = fold_key(l[r]);
    // the keys, two a register: the lengths are dead after this pass (the insert
    // then fits 128 VGPRs, 4 waves a SIMD, without spilling)
    kk[r / 2] |= (r & 1) ? k << 16 : k;
    if (fresh) {
      trep[trep_at(lb + r)] = (uint16_t)k;
      local |= 1u << r;
    }
    const uint64_t cm = __ballot(is_cand);
    if (cm) {
      uint32_t at = 0;
      const int leader = __ffsll((long long)cm) - 1;
      if ((int)lane == leader) at = atomicAdd(&ncand, (uint32_t)__popcll(cm));
      at = lane_value(at, leader);
      if (is_cand) cand[at + (uint32_t)__popcll(cm & ((1ull << lane) - 1))] = (uint16_t)(lb + r);
    }
    run = max(run, o[r]);
  }
  if (wave == 0) {
    uint64_t b = 0;
    if (!a.tstat) {
      b = a.tmax[blockIdx.x];
    } else if (blockIdx.x) {
      b = tile_lookback(a, blockIdx.x);
      if (threadIdx.x == 0) {
        const uint64_t own = min(max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3])), kTileVal);
        __hip_atomic_store(&a.tstat[blockIdx.x], kTileIncl | max(b, own), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (threadIdx.x == 0) s_before = b;
  }
  __syncthreads();
  PLAN_STAMP(kPsInsert, 3);
  // Second pass: a message fresh so far stays fresh when it is also above every
  // offset of the tiles before (tile 0: none); otherwise it joins the candidates
  // (c5: none -- the packed payloads' offsets rise). The lanes are counted here.
  const uint64_t before = s_before;
  const bool check = blockIdx.x != 0;
#pragma unroll
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const bool was = (local >> r) & 1;
    const bool fresh = was && (!check || o[r] > before);
    fold_hist_add_wave_key(a, hist, fresh, (kk[r / 2] >> ((r & 1) * 16)) & 0xFFFFu, base + r);
    const bool demoted = was && !fresh;
    const uint64_t cm = __ballot(demoted);
    if (cm) {
      uint32_t at = 0;
      const int leader = __ffsll((long long)cm) - 1;
      if ((int)lane == leader) at = atomicAdd(&ncand, (uint32_t)__popcll(cm));
      at = lane_value(at, leader);
      if (demoted) cand[at + (uint32_t)__popcll(cm & ((1ull << lane) - 1))] = (uint16_t)(lb + r);
    }
  }
  __syncthreads();
  PLAN_STAMP(kPsInsert, 4);
  PLAN_STAMP_VAL(kPsInsert, 8, ncand);
  // the claims, side by side; a folded message's (rep, i) pair goes straight into
  // the tile's segment of apairs, so the fill reads only them (c5: 5 % of the
  // messages) instead of a representative per message
  const uint32_t nc = ncand;
  for (uint32_t c0 = 0; c0 < nc; c0 += blockDim.x) {
    const uint32_t c = c0 + threadIdx.x;
    uint32_t li = 0, rp = 0;
    uint64_t i = 0;
    if (c < nc) {
      li = cand[c];
      i = tile0 + li;
      const uint64_t ln = a.len[i];
      rp = fold_claim(a, i, a.off[i], ln);
      if (rp == (uint32_t)i) fold_hist_add(hist, ln);
      trep[trep_at(li)] = rp == (uint32_t)i ? (uint16_t)fold_key(ln) : (uint16_t)0xFFFFu;
      // (insert_list) a long payload's claimant is the early head's: listed here, as
      // k_fold_longs would (every long message is a candidate, so every long lane)
      if (a.insert_list && rp == (uint32_t)i && dev_blocks_for(ln) >= a.long_blocks) {
        const uint32_t k = atomicAdd(&a.info[2], 1u);
        if (k < a.long_cap) a.longs[k] = (uint32_t)i;
      }
    }
    const bool folded = c < nc && rp != (uint32_t)i;
    const uint64_t fm = __ballot(folded);
    if (fm) {
      uint32_t at = 0;
      const int leader = __ffsll((long long)fm) - 1;
      if ((int)lane == leader) at = atomicAdd(&nalias, (uint32_t)__popcll(fm));
      at = lane_value(at, leader);
      if (folded) a.apairs[tile0 + at + (uint32_t)__popcll(fm & ((1ull << lane) - 1))] = ((uint64_t)rp << 32) | (uint32_t)i;
    }
  }
  __syncthreads();
  PLAN_STAMP(kPsInsert, 5);
  // key16 out, consecutive messages per wave instruction
#pragma unroll 4
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const uint32_t li = r * 256 + threadIdx.x;
    const uint64_t i = tile0 + li;
    if (i < a.n) a.key16[i] = trep[trep_at(li)];
  }
  PLAN_STAMP(kPsInsert, 6);
  fold_hist_flush(a, hist, nkeys);  // (its barrier also completes nalias)
  if (threadIdx.x == 0) a.acount[blockIdx.x] = nalias;
  PLAN_STAMP(kPsInsert, 7);
  PLAN_STAMP_VAL(kPsInsert, 9, nkeys);
}

// The fold planner's keys are few (kFoldBuckets), so a tile counts them in a
// directly indexed LDS histogram: one LDS atomic per message, no probing and
// no per-key wave loop (a storm's wave holds ~15 distinct block counts: the
// hash-table tile with a wave-aggregated loop per key cost c5's 8.4 M messages
// 210-270 us per pass, latency-bound).
constexpr uint32_t kFoldItems = kPlanItems;          // messages per thread
constexpr uint32_t kFoldTile = 256 * kFoldItems;     // messages per workgroup
static_assert(kFoldTile == kPlanTile, "the insert, the counts and the scatter share one tiling (tkeys, apairs)");
static_assert(kFoldBuckets < 0xFFFFu, "keys fit key16 below its no-lane mark");

// Without folding every message is a lane (with folding k_fold_insert counts).
__global__ __launch_bounds__(256) void k_fold_keys(FoldArgs a) {
  __shared__ FoldHist hist;
  __shared__ uint32_t nkeys;
  fold_hist_clear(hist);
  if (threadIdx.x == 0) nkeys = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kFoldTile;
#pragma unroll 4
  for (uint32_t r = 0; r < kFoldItems; ++r) {
    const uint64_t i = base + r * 256 + threadIdx.x;
    // one LDS atomic a message: the wave-aggregated count (k_fold_insert's)
    // measured slower here, 70.6 -> 84.5 us on c5 (round 6, profiles/r06_plan2/)
    if (i < a.n) {
      const uint64_t l = a.len[i];
      fold_hist_add(hist, l);
      a.key16[i] = (uint16_t)fold_key(l);
    }
  }
  __syncthreads();
  fold_hist_flush(a, hist, nkeys);
}

// Key k's longest chain and its c lanes' blocks: exact below 4,096 blocks (one
// class per count), measured by k_fold_keys for the power-of-two classes above.
__device__ __forceinline__ uint64_t key_max_blocks(const FoldArgs& a, uint32_t k) {
  return k < kFoldBigBuckets ? a.big[k] : fold_class_blocks(kFoldBuckets - 1 - k);
}
__device__ __forceinline__ uint64_t key_sum_blocks(const FoldArgs& a, uint32_t k, uint32_t c) {
  return k < kFoldBigBuckets ? a.big[kFoldBigBuckets + k] : (uint64_t)c * fold_class_blocks(kFoldBuckets - 1 - k);
}

// The head. Per candidate cut k (lanes with keys below k -- the longest -- go
// to the cooperative kernel, h(k) of them on ceil(h / 128) CUs of their own),
// the launch's estimated end in SIMD cycles:
//   T(k) = max( h > 0 ? longest chain x coop_cycles : 0,
//               remaining lane blocks / 64 / remaining SIMDs x wave_block_cycles,
//               longest remaining chain x lane_cycles )
// The cut with the smallest T wins. Cuts whose T is the head's own term tie on
// it, and among them the one whose lane-kernel part -- max(body, longest
// remaining chain) -- leaves the most room wins: the cost is T + that part / 8
// (ties after that: the smaller head; MSHA_PLAN_TIEBREAK=0: T alone, round 3's
// rule -- equal on c5's slices, profiles/r04_tiebreak/). What moved c5 at 8
// GPUs was the two-lane head's calibration (3,800 -> 3,500 cycles a block):
// at 3,800 the model saw room under the head for the 652-block EpochChange
// payloads on the lane kernel, whose chain then ended ~0.12 ms after the
// head's (rocprofv3 timeline, profiles/r04_tiebreak/); folded slice 2.25-2.30
// -> 2.15-2.16 ms. head_pct scales the head's term (A/B: 1 = a nearly free
// head, large = none).
__device__ __forceinline__ uint64_t head_cost(const FoldArgs& a, uint64_t h, uint64_t bh, uint64_t btot,
                                              uint64_t max_blocks, uint64_t next_blocks) {
  // (k_fold_scan evaluates this for every non-empty bucket on one CU: the 64-bit
  // divisions it used to make were most of the scan's time. h <= head_cap fits 32
  // bits; the body's quotient is exact in double below 2^53, far above any batch.)
  if (h > a.head_cap) return ~0ull;
  const uint64_t cus = a.simds / 4, hcus = ((uint32_t)h + a.head_per_wg - 1u) / a.head_per_wg;
  if (hcus >= cus) return ~0ull;
  const uint64_t t_head = h ? max_blocks * a.coop_cycles / 100 * a.head_pct : 0;
  const uint64_t t_body =
      (uint64_t)((double)((btot - bh) * a.wave_block_cycles) / (double)(64ull * 4 * (cus - hcus)));
  const uint64_t t_lanes = max(t_body, next_blocks * a.lane_cycles);
  // work-stealing lane kernel: a cut that leaves a long chain on it loses to any
  // that does not (FoldArgs::ws_long)
  const uint64_t ws_penalty = a.ws_long && next_blocks >= a.ws_long ? (1ull << 36) : 0;
  return max(t_head, t_lanes) + (a.tiebreak ? t_lanes / 8 : 0) + ws_penalty;
}

constexpr uint64_t kCostMax = (uint64_t(1) << 40) - 1;

// Round 6: each thread's six buckets are read ONCE into registers, and the scans
// and reductions run over the wave by shuffles, then over the 16 waves' totals in
// LDS -- 3 barriers instead of ~40, and no loop of dependent bucket loads (the
// longest-chain search read up to six counters one after another): 14 -> ~3 us.
__global__ __launch_bounds__(1024) void k_fold_scan(FoldArgs a) {
  __shared__ uint32_t w_cnt[16], w_min[16], w_h[16];
  __shared__ uint64_t w_blk[16], w_key[16];
  __shared__ uint32_t s_long;  // lanes of >= long_blocks blocks
  __shared__ unsigned long long s_long_blocks;  // and their blocks
  PLAN_STAMP(kPsScan, 0);
  const uint32_t t = threadIdx.x, lane = __lane_id(), wave = t >> 6;
  if (t == 0) s_long = 0, s_long_blocks = 0;
  constexpr uint32_t per = (kFoldBuckets + 1023) / 1024;
  const uint32_t b0 = min(t * per, kFoldBuckets);
  uint32_t c[per];
  uint64_t sb[per];
  uint32_t s = 0, first = kFoldBuckets;
  uint64_t bl = 0;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k) c[k] = b0 + k < kFoldBuckets ? a.cnt[b0 + k] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k) {
    sb[k] = c[k] ? key_sum_blocks(a, b0 + k, c[k]) : 0ull;
    s += c[k];
    bl += sb[k];
    if (c[k] && first == kFoldBuckets) first = b0 + k;
  }
  // inclusive scans of counts and blocks over the wave; the longest chain is the
  // first non-empty key (lowest key, most blocks)
  uint32_t si = s;
  uint64_t bi = bl;
  uint32_t fm = first;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(si, d);
    const uint64_t w = (uint64_t)__shfl_up((unsigned long long)bi, d);
    if (lane >= d) si += v, bi += w;
    fm = min(fm, (uint32_t)__shfl_xor((int)fm, d));
  }
  if (lane == 63) w_cnt[wave] = si, w_blk[wave] = bi;
  if (lane == 0) w_min[wave] = fm;
  __syncthreads();
  uint32_t lanes = 0, run = si - s, kmax = kFoldBuckets;
  uint64_t btot = 0, brun = bi - bl;
  for (uint32_t w = 0; w < 16; ++w) {
    if (w < wave) run += w_cnt[w], brun += w_blk[w];
    lanes += w_cnt[w];
    btot += w_blk[w];
    kmax = min(kmax, w_min[w]);
  }
  const uint64_t max_blocks = kmax < kFoldBuckets ? key_max_blocks(a, kmax) : 0;
  // each thread: the best cut at its buckets' boundaries, packed (cost, key)
  uint64_t mine = ~0ull;
  uint32_t mine_h = 0;
  // the early head's lanes must be exactly the lanes of >= long_blocks blocks:
  // keys up to that of a long_blocks-block message (fold_key: descending classes)
  const uint32_t klong = a.long_blocks ? fold_key((uint64_t)(a.long_blocks - 1) * 64) + 1 : 0u;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k) {  // cut before bucket b: h = run, its longest = bucket b
    const uint32_t b = b0 + k;
    if (b >= kFoldBuckets) break;
    if (b == klong) s_long = run, s_long_blocks = brun;
    if (c[k] && a.head_cap) {
      const uint64_t cost = head_cost(a, run, brun, btot, max_blocks, key_max_blocks(a, b));
      const uint64_t key = (min(cost, kCostMax) << 20) | b;
      if (key < mine) {
        mine = key;
        mine_h = run;
      }
    }
    a.cnt[b] = run;
    run += c[k];
    brun += sb[k];
  }
  if (t == 1023 && a.head_cap) {  // the cut after the last bucket: every lane on the head
    const uint64_t cost = head_cost(a, run, brun, btot, max_blocks, 0);
    const uint64_t key = (min(cost, kCostMax) << 20) | kFoldBuckets;
    if (key < mine) {
      mine = key;
      mine_h = run;
    }
  }
  uint64_t wk = mine;
  for (uint32_t d = 32; d > 0; d >>= 1) wk = min(wk, (uint64_t)__shfl_xor((unsigned long long)wk, d));
  if (lane == 0) w_key[wave] = wk;
  if (mine == wk && wk != ~0ull) w_h[wave] = mine_h;  // keys are distinct (the bucket is in them)
  __syncthreads();
  uint64_t best_key = ~0ull;
  uint32_t best_h = 0;
  if (t == 0)
    for (uint32_t w = 0; w < 16; ++w)
      if (w_key[w] < best_key) best_key = w_key[w], best_h = w_h[w];
  if (t == 0) {
    // The head's last workgroup has room to spare (a workgroup runs as long as
    // its longest chain): fill it with the next-longest lanes, which would
    // otherwise run as lone chains on the lane kernel (folded c5: 37 -> 128).
    const uint32_t h = best_key == ~0ull ? 0u : best_h;
    const uint32_t hfill = (h + a.head_per_wg - 1) / a.head_per_wg * a.head_per_wg;
    const uint32_t late = min(min(hfill, lanes), a.head_cap);
    // an early head (k_fold_longs) is exactly the lanes of >= long_blocks blocks:
    // the first info[4] positions of the descending order. A defensive invariant,
    // not a race the kernels can produce: whichever of k_fold_longs and the alias
    // insert claims a long payload first, k_fold_longs claims every long message
    // and so reads back -- and lists -- each claimant. Should the two
    // counts ever differ (forced only by the MSHA_FOLD_RACE_TEST build), nothing is
    // skipped: the scan's cut (late head) and the lane kernel hash every lane,
    // the listed ones a second time with the same digests.
    // (resolved against info[4] by k_fold_scatter: the scan no longer waits for
    // k_fold_longs, whose head stream the scatter waits for instead)
    a.info[0] = lanes;
    a.info[16] = s_long;
    a.info[17] = late;
    if (a.insert_list) {
      // The early head listed by the insert: always (every distinct long payload the
      // list holds), on the eight-lane kernel when its chain is the call's long pole
      // -- the lanes' other blocks over the SIMDs take less -- else the two-lane one
      const uint32_t c = a.info[2];
      const uint64_t t_body = (btot - s_long_blocks) * a.wave_block_cycles / (64ull * a.simds);
      const bool pole = t_body < max_blocks * a.early_cycles;
      const uint32_t e = c <= a.long_cap ? c : 0u;
      a.info[4] = e;
      a.info[20] = pole ? e : 0u;
      a.info[21] = pole ? 0u : e;
    }
    PLAN_STAMP(kPsScan, 1);
  }
}

// Each lane's position: its key's bucket start, plus its tile's offset in the
// bucket (taken by the insert or the counts, FoldArgs::tkeys), plus its rank
// inside the tile (LDS atomic); order[position] = i. No global atomics: round 4
// took each tile's offsets here, 2,048 tiles' returning atomics on the few hot
// keys of a storm.
__global__ __launch_bounds__(256) void k_fold_scatter(FoldArgs a) {
  __shared__ uint32_t pos[kFoldBuckets];  // next position of each key the tile holds
  PLAN_STAMP(kPsScatter, 0);
  const uint64_t base = (uint64_t)blockIdx.x * kFoldTile;
  // Round 6: the thread's 16 keys load first, unconditionally (a clamped index),
  // beside the bucket starts below: a guarded load per row compiled to a branch
  // and a wait on each, 16 memory round trips one after another (the order loop's
  // ~11 us a workgroup, profiles/r06_plan7/ stamps)
  uint32_t kr[kFoldItems];
#pragma unroll
  for (uint32_t r = 0; r < kFoldItems; ++r) kr[r] = a.key16[min(base + r * 256 + threadIdx.x, a.n - 1)];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // The heads, now that k_fold_longs is done (the stream waited for it after the
    // scan): the early head's lanes or else the scan's cut (info[17]).
#ifndef MSHA_SCAN_NO_EARLY_CHECK
    const uint32_t early = a.long_blocks && a.info[4] == a.info[16] ? a.info[4] : 0u;
#else  // round 5's committed rule, for the check's regression test (tools/r05_race.sh)
    const uint32_t early = a.long_blocks ? a.info[4] : 0u;
#endif
    const uint32_t late = a.early_only ? 0u : a.info[17];  // (early_only: no late head)
    a.info[1] = early ? early : late;
    a.info[5] = early ? 0u : late;
  }
  const uint32_t nk = a.tkcount[blockIdx.x];
  const uint64_t* tl = a.tkeys + (uint64_t)blockIdx.x * kPlanTile;
  for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) {
    const uint64_t v = tl[k];
    pos[v >> 32] = a.cnt[v >> 32] + (uint32_t)v;  // bucket start (k_fold_scan) + the tile's offset
  }
  __syncthreads();
  PLAN_STAMP(kPsScatter, 1);
#pragma unroll
  for (uint32_t r = 0; r < kFoldItems; ++r) {
    const uint64_t i = base + r * 256 + threadIdx.x;
    const uint32_t k = i < a.n ? kr[r] : 0xFFFFu;
    const bool valid = k != 0xFFFFu;
    // Round 6: the lanes sharing the first valid lane's key (a storm's wave: ~70 %
    // one key) take their positions with ONE LDS atomic, ranked by lane; 64 atomics
    // on one LDS word serialise. The rest one each, as before (one atomic per
    // distinct key measured far slower: profiles/r06_plan9/).
    const uint64_t any = __ballot(valid);
    if (!any) continue;
    const unsigned lane = __lane_id();
    const uint32_t k0 = lane_value(k, __ffsll((long long)any) - 1);
    const uint64_t same = __ballot(valid && k == k0);
    const uint32_t before = (uint32_t)__popcll(same & ((1ull << lane) - 1));
    uint32_t b0 = 0;
    if (((same >> lane) & 1) && before == 0) b0 = atomicAdd(&pos[k0], (uint32_t)__popcll(same));
    b0 = lane_value(b0, __ffsll((long long)same) - 1);
    if ((same >> lane) & 1)
      a.order[b0 + before] = (uint32_t)i;
    else if (valid)
      a.order[atomicAdd(&pos[k], 1u)] = (uint32_t)i;
  }
  PLAN_STAMP(kPsScatter, 2);
  // positions past the last lane (the folded aliases' share) hold kNoLane
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = a.info[0] + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += stride)
    a.order[q] = kNoLane;
  PLAN_STAMP(kPsScatter, 3);
}

// A grid's (sum, max) and "am I the last workgroup" without one hot word (round 6:
// each of k_fold_longs' and k_fold_longs_gate's 256-1,024 workgroups ended in three
// atomics on the same words, serialised at ~20 ns each -- ~23 us of an N = 8 rank's
// 65 us before its chain starts, profiles/r06_n8_trace/). Workgroup w adds to group
// w mod G's slots and counts itself there; a group's last workgroup adds the group's
// totals to the top slots and counts the group; the last group's last workgroup
// returns true with the grid's totals. Thread 0 only. ws: kGridWords zeroed words,
// one 64-byte slot a group ([0] count, [2..3] sum, [4..5] max), then the top slot.
__device__ __forceinline__ bool grid_reduce_last(uint32_t* ws, uint64_t sum, uint64_t mx, uint64_t& tot,
                                                 uint64_t& top_max) {
  const uint32_t groups = min(gridDim.x, kGridGroups);
  const uint32_t g = blockIdx.x % groups;
  uint32_t* gs = ws + g * 16;
  unsigned long long* gsum = reinterpret_cast<unsigned long long*>(gs + 2);
  unsigned long long* gmax = reinterpret_cast<unsigned long long*>(gs + 4);
  atomicAdd(gsum, (unsigned long long)sum);
  atomicMax(gmax, (unsigned long long)mx);
  __threadfence();  // this workgroup's results (and sums) before its count
  if (atomicAdd(&gs[0], 1u) != (gridDim.x - g + groups - 1) / groups - 1) return false;
  __threadfence();
  const uint64_t s = __hip_atomic_load(gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t m = __hip_atomic_load(gmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t* top = ws + kGridGroups * 16;
  unsigned long long* tsum = reinterpret_cast<unsigned long long*>(top + 2);
  unsigned long long* tmx = reinterpret_cast<unsigned long long*>(top + 4);
  atomicAdd(tsum, (unsigned long long)s);
  atomicMax(tmx, (unsigned long long)m);
  __threadfence();
  if (atomicAdd(&top[0], 1u) != groups - 1) return false;
  __threadfence();
  tot = __hip_atomic_load(tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  top_max = __hip_atomic_load(tmx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// The early head's list: every message of >= long_blocks blocks claims its
// (off, len) in the alias table (a hot payload costs a cached read after the
// first claim); each claimant -- one per distinct long payload -- is listed. It
// runs beside k_fold_insert, after the tile prefix: whichever claims a key
// first, both read the same claimant back, and the claimant, a long message
// itself, lists itself here. The last workgroup to finish publishes the list's
// length as the early head, or 0 when it is longer than long_cap or the lane
// kernel's share -- every short message's blocks plus the distinct long ones --
// outlasts the head's chain anyway (then the scan's cut decides, as without it).
// k_fold_tilescan already stood it down (info[6] == 0) when the short blocks
// alone do: then every workgroup returns at once (c5 on one GPU: round 4 ran
// the whole list, 110-234 us of claims beside the insert, to stand down).
// Round 5: a workgroup takes tiles of kPlanTile consecutive messages, loads each
// thread's 16 lengths as 16-byte vectors, lists the tile's long messages in
// LDS, and its threads then claim them side by side (round 4 claimed in the
// stride loop: every wave's load -> compare chain once per iteration).
__global__ __launch_bounds__(256) void k_fold_longs(FoldArgs a) {
  if (a.info[6] == 0) return;  // uniform: the first decision (k_fold_tilescan or k_fold_longs_gate)
  __shared__ uint32_t list[kPlanTile];
  __shared__ uint32_t nlist;
  __shared__ unsigned long long s_sum, s_max;
  if (threadIdx.x == 0) s_sum = s_max = 0;
  uint64_t sum = 0, mx = 0;
  const unsigned lane = __lane_id();
  const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    if (threadIdx.x == 0) nlist = 0;
    __syncthreads();
    const uint64_t base = tile * kPlanTile + (uint64_t)threadIdx.x * kPlanItems;
    uint64_t l[kPlanItems];
    load_run(a.len, base, a.n, a.vec, l);
#pragma unroll
    for (uint32_t r = 0; r < kPlanItems; ++r) {
      const bool valid = base + r < a.n;
      const uint64_t blocks = valid ? dev_blocks_for(l[r]) : 0;
      mx = max(mx, blocks);
      const bool lng = valid && blocks >= a.long_blocks;
      if (valid && !lng) sum += blocks;
      const uint64_t lm = __ballot(lng);
      if (lm) {
        uint32_t at = 0;
        const int leader = __ffsll((long long)lm) - 1;
        if ((int)lane == leader) at = atomicAdd(&nlist, (uint32_t)__popcll(lm));
        at = lane_value(at, leader);
        if (lng) list[at + (uint32_t)__popcll(lm & ((1ull << lane) - 1))] = (uint32_t)(base + r);
      }
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < nlist; c += blockDim.x) {
      const uint64_t i = list[c];
      const uint64_t ln = a.len[i];
#ifdef MSHA_FOLD_RACE_TEST  // test build only (tests/test_gpu_planned.py, tools/r06_race.sh)
      if (a.race_test && (plan_hash(a.off[i], ln) & 1)) continue;  // left to the insert
#endif
      if (fold_claim(a, i, a.off[i], ln) == (uint32_t)i) {
        sum += dev_blocks_for(ln);
        const uint32_t k = atomicAdd(&a.info[2], 1u);
        if (k < a.long_cap) a.longs[k] = (uint32_t)i;
      }
    }
    __syncthreads();  // the list is rewritten by the next tile
  }
  atomicAdd(&s_sum, (unsigned long long)sum);
  atomicMax(&s_max, (unsigned long long)mx);
  __syncthreads();
  uint64_t tot = 0, lng = 0;
  if (threadIdx.x == 0 && grid_reduce_last(a.grid_ws, s_sum, s_max, tot, lng)) {  // (its fences cover the list)
    const uint32_t c = __hip_atomic_load(&a.info[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t_body = tot * a.wave_block_cycles / (64ull * a.simds);
    const uint64_t t_head = lng * a.early_cycles;
    const bool pole = t_body < t_head;  // the head's chain outlasts the lane kernel's share
    if (a.early_only) {
      const uint32_t e = c <= a.long_cap ? c : 0u;
      a.info[4] = e;
      a.info[20] = pole ? e : 0u;
      a.info[21] = pole ? 0u : e;
    } else {
      a.info[4] = c <= a.long_cap && pole ? c : 0u;
    }
  }
}

// The early head's first decision without the tile prefix (FoldArgs::early_fork):
// one pass over len alone -- the short messages' blocks (the lane kernel's share
// without the long payloads) and the longest chain -- and the last workgroup to
// finish decides as k_fold_tilescan would (info[6]). It runs first on the head's
// stream, forked right after the planner's memsets, beside k_fold_tilemax.
__global__ __launch_bounds__(256) void k_fold_longs_gate(FoldArgs a) {
  __shared__ unsigned long long s_sum, s_max;
  PLAN_STAMP(kPsGate, 0);
  if (threadIdx.x == 0) s_sum = s_max = 0;
  __syncthreads();
  uint64_t sum = 0, mx = 0;
  const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const uint64_t base = tile * kPlanTile + (uint64_t)threadIdx.x * kPlanItems;
    uint64_t l[kPlanItems];
    load_run(a.len, base, a.n, a.vec, l);
#pragma unroll
    for (uint32_t r = 0; r < kPlanItems; ++r) {
      const uint64_t blocks = base + r < a.n ? dev_blocks_for(l[r]) : 0;
      mx = max(mx, blocks);
      if (blocks < a.long_blocks) sum += blocks;
    }
  }
  for (uint32_t d = 32; d > 0; d >>= 1) {  // wave sums, then one LDS atomic per wave
    sum += __shfl_xor(sum, d);
    mx = max(mx, (uint64_t)__shfl_xor(mx, d));
  }
  if (__lane_id() == 0) {
    atomicAdd(&s_sum, (unsigned long long)sum);
    atomicMax(&s_max, (unsigned long long)mx);
  }
  __syncthreads();
  uint64_t ss = 0, sm = 0;
  if (threadIdx.x == 0 && grid_reduce_last(a.grid_ws + kGridWords, s_sum, s_max, ss, sm)) {
    const uint64_t t_body = ss * a.wave_block_cycles / (64ull * a.simds);
    const uint64_t t_head = sm * a.early_cycles;
    a.info[6] = sm >= a.long_blocks && (a.early_only || t_body < t_head) ? 1u : 0u;
  }
  PLAN_STAMP(kPsGate, 1);
}

hipError_t launch_fold_longs(const FoldArgs& a, int cus, hipStream_t st) {
  if (a.n == 0 || !a.long_blocks) return hipSuccess;
  // a.longs_wgs (A/B): fewer workgroups, fewer of the same-address atomics that end
  // each one (each costs ~20 ns serialised: profiles/r06_call4/)
  const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
  const uint64_t cap = a.longs_wgs ? a.longs_wgs : (uint64_t)cus * 4;
  const unsigned grid = (unsigned)std::min<uint64_t>(tiles, cap);
  // the gate on 64 workgroups unless MSHA_GATE_WGS says otherwise: each ends in
  // same-address atomics (1,024 of them: ~60 us serialised beside the prefix,
  // profiles/r06_call4/); partials summed by k_fold_longs instead cost the insert
  // more bandwidth than they saved (round 6, profiles/r06_plan5/)
  // (a batch of at most a tile a CU: one workgroup a tile -- an N = 8 rank's gate ran
  // its 4 tiles a workgroup one after another, 27 us before the list could start)
  const unsigned ggrid = (unsigned)std::min<uint64_t>(
      tiles, a.gate_wgs ? a.gate_wgs : (tiles <= (uint64_t)cus ? (uint64_t)cus : 64u));
  if (a.early_fork) hipLaunchKernelGGL(k_fold_longs_gate, dim3(ggrid), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_fold_longs, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

// One workgroup per insert tile: its folded messages copy their representative's
// digest (32 bytes each).
__global__ __launch_bounds__(256) void k_fold_fill(FoldArgs a, uint8_t* __restrict__ out) {
  PLAN_STAMP(kPsFill, 0);
  const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const uint64_t* p = a.apairs + tile * kPlanTile;
    // the first pair loads beside the count (a tile's segment holds kPlanTile
    // entries, inside the batch): two dependent memory trips a pair, not three
    const uint64_t v0 = a.apairs[min(tile * kPlanTile + threadIdx.x, a.n - 1)];  // unconditional: no branch
    const uint32_t cnt = a.acount[tile];
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) {
      const uint64_t v = k == threadIdx.x ? v0 : p[k];
      const uint4* src = reinterpret_cast<const uint4*>(out + 32 * (v >> 32));
      uint4* dst = reinterpret_cast<uint4*>(out + 32 * (v & 0xFFFFFFFFull));
      const uint4 x0 = src[0], x1 = src[1];  // both loads before either store (out may alias)
      dst[0] = x0;
      dst[1] = x1;
    }
  }
  PLAN_STAMP(kPsFill, 1);
}

hipError_t launch_fold_prefix(const FoldArgs& a, hipStream_t st) {
  if (a.n == 0 || !a.table || a.tstat) return hipSuccess;  // (tstat: the insert looks back itself)
  const unsigned ptiles = (unsigned)((a.n + kPlanTile - 1) / kPlanTile);
  hipLaunchKernelGGL(k_fold_tilemax, dim3(ptiles), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_fold_tilescan, dim3(1), dim3(1024), 0, st, a, (uint64_t)ptiles);
  return hipGetLastError();
}

hipError_t launch_fold_plan(const FoldArgs& a, hipStream_t st, hipStream_t sst, hipEvent_t fork,
                            hipEvent_t scatter_after, hipEvent_t after_scan) {
  if (a.n == 0) return hipSuccess;
  const unsigned ptiles = (unsigned)((a.n + kPlanTile - 1) / kPlanTile);
  if (a.table) hipLaunchKernelGGL(k_fold_insert, dim3(ptiles), dim3(256), 0, st, a);
  const unsigned ftiles = (unsigned)((a.n + kFoldTile - 1) / kFoldTile);
  if (!a.table) hipLaunchKernelGGL(k_fold_keys, dim3(ftiles), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_fold_scan, dim3(1), dim3(1024), 0, st, a);
  if (after_scan) {
    const hipError_t e = hipEventRecord(after_scan, st);
    if (e != hipSuccess) return e;
  }
  if (sst != st) {
    hipError_t e = hipEventRecord(fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(sst, fork, 0);
    if (e != hipSuccess) return e;
  }
  if (scatter_after) {
    const hipError_t e = hipStreamWaitEvent(sst, scatter_after, 0);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_fold_scatter, dim3(ftiles), dim3(256), 0, sst, a);
  return hipGetLastError();
}

hipError_t launch_fold_fill(const FoldArgs& a, uint8_t* out, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  // one workgroup a tile (256 workgroups looping over tiles measured the same:
  // profiles/r06_ws/prefetch/)
  const uint64_t tiles = (a.n + kPlanTile - 1) / kPlanTile;
  hipLaunchKernelGGL(k_fold_fill, dim3((unsigned)tiles), dim3(256), 0, st, a, out);
  return hipGetLastError();
}

}  // namespace msha

#ifdef MSHA_PLAN_STAMPS
// Diagnostic build only: points the planner stamps at `buf` (device memory, 6 x per
// records of 16 words; the caller zeroes it before the call it wants). NULL: off.
extern "C" int msha_diag_plan_stamps(void* buf, uint32_t per) {
  uint64_t* b = static_cast<uint64_t*>(buf);
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::g_plan_stamps), &b, sizeof b) != hipSuccess) return 3;
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::g_plan_stamp_per), &per, sizeof per) != hipSuccess) return 3;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
#endif
