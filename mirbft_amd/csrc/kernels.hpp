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
bool plan_split(uint64_t n, int cus, int policy, SplitPlan* sp);

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

}  // namespace msha
