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

#include "kernels.hpp"

namespace msha {

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
    const uint32_t v = atomicCAS(&a.table[h], 0u, me);
    if (v == 0) break;
    const uint64_t j = v - 1;
    if (a.off[j] == o && a.len[j] == l) {  // same key: the slot keeps the smallest index
      atomicMin(&a.table[h], me);
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

// Bucket key of message i when it is a lane (rep[i] == i): (piece holding the
// payload's end) * B + (bmax - blocks).
__device__ __forceinline__ uint32_t lane_key(const PlanArgs& a, uint64_t i, uint32_t* chunk_out) {
  const uint64_t l = a.len[i];
  const uint64_t end = a.dev_off[i] + (l ? l : 1) - 1;
  const uint32_t chunk = (uint32_t)min((uint64_t)(end >> kDirectChunkShift), a.chunks - 1);
  if (chunk_out) *chunk_out = chunk;
  return chunk * (uint32_t)a.B + (a.B > 1 ? (uint32_t)(a.bmax - dev_blocks_for(l)) : 0u);
}

__global__ __launch_bounds__(256) void k_plan_keys(PlanArgs a) {
  __shared__ TileTable t;
  tile_clear(t, 0xFFFFFFFFu);
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile;
#pragma unroll 4
  for (uint32_t r = 0; r < kPlanItems; ++r) {
    const uint64_t i = base + r * 256 + threadIdx.x;
    if (i >= a.m) break;
    const uint32_t rp = a.table ? a.table[a.slot[i]] - 1 : (uint32_t)i;
    a.rep[i] = rp;
    if (rp != (uint32_t)i) continue;
    uint32_t chunk;
    const uint32_t k = lane_key(a, i, &chunk);
    const uint32_t j = tile_slot(t, k);
    if (j < kPlanSlots) {
      atomicAdd(&t.cnt[j], 1u);
      atomicMin(&t.aux[j], (uint32_t)i);
    } else {  // table full: straight to the global counters
      atomicAdd(&a.cnt[k], 1u);
      atomicMin(&a.gmin[chunk], (uint32_t)i);
    }
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
    if (i >= a.m || a.rep[i] != (uint32_t)i) continue;
    const uint32_t k = lane_key(a, i, nullptr);
    const uint32_t j = tile_slot(t, k);
    if (j < kPlanSlots) {
      slot[r] = j;
      rank[r] = atomicAdd(&t.cnt[j], 1u);
    } else {  // table full: a position straight from the global counter
      slot[r] = kPlanSlots;
      rank[r] = atomicAdd(&a.cnt[k], 1u);
    }
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

}  // namespace msha
