// Host-side launchers for the gfx950 SHA-256 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msha {

// Bytes that must be readable after the last message of a device arena: the
// kernels read a message's final block as one whole 64-byte block.
constexpr uint64_t kArenaSlack = 64;

// Lane i hashes message m = order ? order[i] : i (arena + off[m], len[m]) into
// digest slot o = out_idx ? out_idx[i] : m (out + 32 o). The device API passes
// order (message-indexed metadata); the host pipeline passes lane-indexed
// metadata and out_idx. policy: MSHA_KERNEL_AUTO / _LANE / _COOP (mirsha.h).
//
// split (may be null): run the launch as split chaining (kernels.hip), planned
// by plan_split(); the caller fills flags/epoch (see SplitPlan).
struct SplitPlan {
  uint64_t n_main = 0;      // messages [0, n_main) run one lane each, to completion
  uint32_t chains = 0;      // surplus waves: messages [n_main, n) in chains of 64
  uint32_t segments = 0;    // segments per chain
  uint32_t groups = 0;      // segment workgroups per segment (4 chains each, padded)
  uint32_t stall_chain = 0xFFFFFFFFu;  // failure-path test only (MSHA_SPLIT_STALL=1):
                                       // this chain's first segment never hands over
  uint64_t epoch = 0;       // unique (mod 2^24) among the launches that share flags
  uint64_t* flags = nullptr;  // device, >= chains entries, one word per chain:
                              // epoch | segments done | progress beat (kernels.hip)
};
// Segment caps of split chaining: arena messages / digest-of-digests (kernels.hip).
constexpr int kMaxSegmentsArena = 12;
constexpr int kMaxSegmentsDod = 12;
bool plan_split(uint64_t n, int cus, int policy, SplitPlan* sp, int cap);

// Which kernel a launcher ran (msha_stats launch counters; tests assert them).
enum LaunchKind { kLaunchNone = 0, kLaunchLane, kLaunchPipe, kLaunchCoop, kLaunchSplit, kLaunchDod };

hipError_t launch_digest_batch(const uint8_t* arena, const uint64_t* off, const uint64_t* len,
                               const uint32_t* order, const uint32_t* out_idx, uint64_t n,
                               uint8_t* out, uint32_t* err, int cus, int policy, hipStream_t st,
                               const SplitPlan* split = nullptr, LaunchKind* kind = nullptr);
// Does launch_digest_batch use cooperative chaining for an n-message launch?
bool uses_coop(uint64_t n, int cus, int policy);
hipError_t launch_digest_uniform(const uint8_t* arena, uint64_t stride, uint64_t msg_len,
                                 uint64_t n, uint8_t* out, uint32_t* err, int cus,
                                 hipStream_t st, LaunchKind* kind = nullptr);
// err: device error word (bit 2: a split-chaining handoff timed out).
hipError_t launch_digest_of_digests(const uint8_t* table, const uint32_t* idx,
                                    const uint64_t* begin, uint64_t n, uint8_t* out,
                                    uint32_t* err, hipStream_t st,
                                    const SplitPlan* split = nullptr, LaunchKind* kind = nullptr);

// Direct (pinned-arena) host calls upload a shard's byte ranges in device-space
// pieces of 2^kDirectChunkShift bytes (64 MiB), one event each.
constexpr unsigned kDirectChunkShift = 26;

// Device-side planning of one shard of a direct host call (plan.hip). Every
// array is device memory of the shard's GPU; m messages, shard-local indices.
struct PlanArgs {
  const uint64_t* off;    // caller offsets (raw, as passed to msha_digest_batch)
  const uint64_t* len;
  const uint64_t* gmap;   // uploaded granule g (caller offset glo + g << gshift) -> device
                          // offset, indexed g - gbase
  uint64_t glo = 0, gbase = 0;
  uint32_t gshift = 16;
  uint64_t m = 0;
  uint64_t* dev_off;      // out: device offset of each message
  uint32_t* table;        // alias table, tmask + 1 zeroed entries; null: no aliases
  uint64_t tmask = 0;
  uint32_t* slot;         // m: each message's table slot (with table)
  uint32_t* rep;          // out, m: the first message with the same (off, len)
  uint64_t chunks = 1;    // upload pieces of the shard
  uint64_t B = 1;         // block-count classes per piece (1: pieces only)
  uint64_t bmax = 0;      // largest block count (key = piece * B + bmax - blocks)
  uint64_t nb = 1;        // chunks * B buckets
  uint32_t* cnt;          // nb zeroed counters -> bucket starts
  uint32_t* gmin;         // chunks entries, 0xFFFFFFFF-filled: lowest lane index per piece
  uint32_t* cut;          // out, chunks + 1: first lane of each piece's group
  uint32_t* info;         // out: [0] = lanes
  uint64_t* lane_off;     // out, per lane: device offset, length, digest slot
  uint64_t* lane_len;
  uint32_t* lane_slot;
};
hipError_t launch_plan(const PlanArgs& a, hipStream_t st);

}  // namespace msha
