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
// kLaunchChain2 / kLaunchChain8 count as cooperative launches too (launches_coop).
// kLaunchLaneWs (the work-stealing lane kernel) counts as a lane launch too.
enum LaunchKind { kLaunchNone = 0, kLaunchLane, kLaunchPipe, kLaunchCoop, kLaunchSplit, kLaunchDod,
                  kLaunchChain2, kLaunchChain8, kLaunchLaneWs };

// GPU-planned device launches (plan.hip: msha_digest_batch_device_planned). The
// planner's lane order holds kNoLane at positions it leaves unused (folded
// aliases, at the end), and *head (device memory, known only on the GPU) lanes
// at the front are long chains routed to the cooperative kernel. A gated launch
// over the whole order either is that head (head_part: cooperative, lanes at or
// past *head idle) or the rest (lanes below *head idle); neither splits.
constexpr uint32_t kNoLane = 0xFFFFFFFFu;
constexpr uint32_t kWsSlots = 64, kWsStride = 16;  // work-stealing tile counters, 64 B apart
// The planner's two-level grid reductions (plan.hip grid_reduce_last): 16 group
// slots and a top slot, 64 B each, zeroed words
constexpr uint32_t kGridGroups = 16, kGridWords = (kGridGroups + 1) * 16;
struct LaneGate {
  const uint32_t* head = nullptr;
  bool head_part = false;
  bool two_lane = false;  // head_part: k_digest_chain2 instead of the cooperative kernel
  bool eight_lane = false;  // head_part: k_digest_chain8 (eight lanes a message, 24 a CU)
  // the body (not head_part): kWsSlots x kWsStride zeroed device words -> the
  // work-stealing lane kernel (k_digest_batch_ws), with `lanes` (device, may be
  // null) the positions worth visiting
  uint32_t* ws_ctr = nullptr;
  const uint32_t* lanes = nullptr;
};

hipError_t launch_digest_batch(const uint8_t* arena, const uint64_t* off, const uint64_t* len,
                               const uint32_t* order, const uint32_t* out_idx, uint64_t n,
                               uint8_t* out, uint32_t* err, int cus, int policy, hipStream_t st,
                               const SplitPlan* split = nullptr, LaunchKind* kind = nullptr,
                               const LaneGate* gate = nullptr);
// Does launch_digest_batch use cooperative chaining for an n-message launch?
bool uses_coop(uint64_t n, int cus, int policy);
// Messages per workgroup of the cooperative kernel (one workgroup per CU) and
// of the two-lane head chain (k_digest_chain2).
constexpr unsigned kCoopMsgsPerWg = 128;
constexpr unsigned kChain2MsgsPerWg = 64;
constexpr unsigned kChain8MsgsPerWg = 16;
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
  uint64_t pieces = 1;    // upload pieces of the shard
  uint32_t piece_shift = kDirectChunkShift;  // a piece is 2^piece_shift device bytes
  // Lane groups: one per (region, piece), region 0 = long chains (blocks >=
  // long_blocks; long_blocks 0: no such region), region 1 = the rest; group
  // g = region * pieces + piece, chunks = the number of groups.
  uint64_t long_blocks = 0;
  uint64_t chunks = 1;
  uint64_t B = 1;         // block-count classes per group (1: groups only)
  uint64_t bmax = 0;      // largest block count (key = group * B + bmax - blocks)
  uint64_t nb = 1;        // chunks * B buckets
  uint32_t* cnt;          // nb zeroed counters -> bucket starts
  uint32_t* gmin;         // chunks entries, 0xFFFFFFFF-filled: lowest lane index per group
  uint32_t* cut;          // out, chunks + 1: first lane of each group
  uint32_t* info;         // out: [0] = lanes
  uint64_t* lane_off;     // out, per lane: device offset, length, digest slot
  uint64_t* lane_len;
  uint32_t* lane_slot;
};
hipError_t launch_plan(const PlanArgs& a, hipStream_t st);

// Device-side planning of a device-resident batch (plan.hip,
// msha_digest_batch_device_planned): every array is device memory of one GPU.
// Lanes = messages, or with a table only the first of each (off, len) key
// (aliases fold into it); the order lists lanes by descending block count,
// kNoLane past the last; info[1] = the head of lanes whose chains would outlast
// the lane kernel's throughput time, for the cooperative kernel (at most
// head_cap). Block-count buckets: exact below 4,096 blocks, powers of two above.
// Classes, ascending: a message shorter than kFoldExactLen bytes by its exact
// length (a wave of one length hashes its padding block's schedule on the
// scalar unit, kernels.hip compress_uniform_pad), then exact block counts in
// [kFoldLowBlocks, 4096), then powers of two. Keys are descending classes.
constexpr uint32_t kFoldExactLen = 1024;
constexpr uint32_t kFoldLowBlocks = 16;   // (blocks of kFoldExactLen bytes: 17; 16 keeps the count even)
constexpr uint32_t kFoldBigBuckets = 52;  // the power-of-two classes (>= 4,096 blocks): keys [0, 52)
constexpr uint32_t kFoldBuckets = kFoldExactLen + (4096 - kFoldLowBlocks) + kFoldBigBuckets;
static_assert(kFoldBuckets % 2 == 0, "FoldArgs::big follows the counters 8-byte aligned");
struct FoldArgs {
  const uint64_t* off;
  const uint64_t* len;
  uint64_t n = 0;
  uint64_t* table = nullptr;  // tmask + 1 slots (epoch << 32 | message + 1); null: no folding
  uint64_t tmask = 0;
  uint32_t epoch = 1;         // this call's tag: a slot of another epoch is empty (never 0)
  // (with table) the folded messages, per tile of 4,096: apairs[tile * 4096 + k] =
  // rep << 32 | i for k < acount[tile] -- message i's digest is message rep's
  uint64_t* apairs = nullptr;
  uint32_t* acount = nullptr;
  uint64_t* tmax = nullptr;   // (with table) ceil(n / 4096): largest offset before each tile
  uint64_t* tsum = nullptr;   // (early head) 2 per tile: the tile's short messages' blocks, its longest chain
  // Round 6: (with table, non-null) the insert finds its tile's prefix itself, by a
  // decoupled look-back over ceil(n / 4096) zeroed status words (plan.hip
  // tile_lookback) -- no k_fold_tilemax / k_fold_tilescan; then one more zeroed
  // word: look-backs that gave up waiting (0 expected; see tile_lookback)
  uint64_t* tstat = nullptr;
  // 2 x kGridWords zeroed words: k_fold_longs' then k_fold_longs_gate's grid reduction
  uint32_t* grid_ws = nullptr;
  uint32_t* cnt;              // kFoldBuckets zeroed counters (by key) -> bucket starts
  uint64_t* big = nullptr;    // 2 x kFoldBigBuckets zeroed: per power-of-two key, the largest
                              // block count and the block sum (the head's cost model needs the
                              // real longest chain, not the class's lower bound)
  uint32_t* order;            // n, kNoLane-filled -> position -> message index
  uint16_t* key16 = nullptr;  // n: message i's key when it is a lane, else 0xFFFF (written by the
                              // insert or the counts, read by the scatter instead of len and rep)
  // Per tile of 4,096 messages, the keys its lanes hold and the tile's offset in
  // each key's bucket, taken when the insert (or the counts) added its lanes to
  // the bucket counters: tkeys[tile * 4096 + k] = key << 32 | offset for k <
  // tkcount[tile]. The scatter places lanes at bucket start + offset + rank with
  // no global atomics of its own.
  uint64_t* tkeys = nullptr;
  uint32_t* tkcount = nullptr;
  uint32_t* info;             // [0] lanes, [1] positions the lane kernel skips (the head's),
                              // [2] distinct long payloads, [3] unused,
                              // [4] the early head's lanes (0: none), [5] the late head's,
                              // [6] the first decision (0: no early head), by k_fold_tilescan,
                              // or with early_fork by k_fold_longs_gate, [7..15] unused (the
                              // list's and the gate's sums: grid_ws),
                              // [16] lanes of >= long_blocks blocks, [17] the scan's cut (the
                              // scatter resolves [1] and [5] from them and [4]), [20] / [21]
                              // (early_only) the eight- / two-lane early head's lanes
                              // (all 32 words zeroed by the caller)
  // The early head (folding only; long_blocks 0: off): k_fold_tilescan sizes the
  // batch (info[6]: 0 when the short messages alone outlast the longest chain);
  // unless it stood down there, k_fold_longs claims every message of >=
  // long_blocks blocks in the alias table beside the insert, listing each
  // distinct one in longs; when there are at most long_cap, and their chain
  // outlasts the lane kernel's share, they are the head (info[4]), launched right
  // then on the two-lane kernel over longs instead of after the scan and
  // scatter, and k_fold_insert never takes a long message as fresh (so its
  // representative is the listed one).
  uint32_t* longs = nullptr;
  // off and len both 16-byte aligned: the per-thread runs of 16 messages load as
  // 16-byte vectors (plan.hip load_run)
  uint32_t vec = 0;
  uint32_t long_blocks = 0;
  // Round 6: the early head's first decision and list run on the
  // head's stream forked BEFORE the tile prefix (k_fold_longs_gate, a pass over len
  // alone, then k_fold_longs), so the head's chain does not wait for the prefix;
  // k_fold_tilemax / k_fold_tilescan then size only the offsets.
  uint32_t early_fork = 0;
  // Round 6: with the work-stealing lane kernel (k_digest_batch_ws) the head's cut
  // keeps every lane of at least ws_long blocks off the lane kernel when it can
  // (a long chain there shares a SIMD with same-age waves: kernels.hip); 0: off.
  uint32_t ws_long = 0;
  uint32_t longs_wgs = 0;  // k_fold_longs / k_fold_longs_gate workgroups (0: 4 a CU; A/B MSHA_LONGS_WGS)
  uint32_t gate_wgs = 0;   // k_fold_longs_gate's workgroups (0: 64; MSHA_GATE_WGS)
  // (early_fork, A/B MSHA_EARLY_ONLY) the early head takes every distinct long payload
  // the list holds: info[20] arms the eight-lane launch (its chain the long pole),
  // info[21] the two-lane one; no late head (the scatter leaves info[1] = the early
  // head's lanes or 0)
  uint32_t early_only = 0;
  // Round 6: the insert's claims list the early head (every claimant of >= long_blocks
  // blocks) and the scan decides it (info[4], [20], [21]): no k_fold_longs_gate /
  // k_fold_longs pass beside the insert; implies early_only
  uint32_t insert_list = 0;
  uint32_t long_cap = 0;
  uint32_t head_cap = 0;      // 0: no head
  uint32_t simds = 1024;
  // The head: the cut of the longest lanes that minimises the launch's
  // estimated end (plan.hip head_cost), in SIMD cycles per block, measured (c5
  // slices, rocprofv3 timelines, profiles/r03_planned/): the lane kernel's
  // throughput on a storm's mixed lanes ~6,500 per wave-block (uniform batches:
  // 5,700); a long chain on the lane kernel among loaded SIMDs ~8,000 (7,000 as
  // the oldest wave of a lightly loaded one); on the cooperative consumer, alone
  // on its CU at top priority, ~4,200 (the two-lane head ~3,500 since round 4). A sweep of the
  // first two (MSHA_PLAN_LANE_CYCLES / MSHA_PLAN_WAVE_CYCLES,
  // profiles/r03_planned/calibration/): 8,000 / 6,500 ran c5 over 8 GPUs 3.00 ->
  // 2.85 ms, equal at 2 and 4. head_pct scales the head's term (A/B).
  uint32_t wave_block_cycles = 6500;
  uint32_t lane_cycles = 8000;
  uint32_t coop_cycles = 4200;
  uint32_t early_cycles = 3500;  // the same for the early head's kernel (its stand-down rule)
  uint32_t head_pct = 100;
  uint32_t head_per_wg = 128;    // messages per head workgroup (one CU each)
  uint32_t tiebreak = 1;         // head-bound ties go to the cut with the most lane-kernel room (A/B: 0)
  // test build only (-DMSHA_FOLD_RACE_TEST, MSHA_FOLD_LONGS_SKIP_ODD=1): k_fold_longs
  // leaves every long payload whose table hash is odd unlisted, a state the product
  // kernels cannot reach, to exercise the scan/scatter defensive check
  uint32_t race_test = 0;
};
// Folding only: the tile maxima and their prefix (k_fold_tilemax, k_fold_tilescan),
// with the early head's list and decision when long_blocks is set; then
// launch_fold_plan: the insert (or, unfolded, the counts), scan and scatter.
hipError_t launch_fold_prefix(const FoldArgs& a, hipStream_t st);
// The insert and the scan on st; the scatter on sst (the side stream of the late
// head: when it is not st, st records `fork` after the scan and sst waits for it),
// after scatter_after (may be null: the early head's list, against which the scatter
// resolves the heads).
// after_scan (may be null): recorded on st right after the scan (the early head's
// stream waits for it when the insert lists the early head: FoldArgs::insert_list).
hipError_t launch_fold_plan(const FoldArgs& a, hipStream_t st, hipStream_t sst, hipEvent_t fork,
                            hipEvent_t scatter_after, hipEvent_t after_scan = nullptr);
// The early head's list (FoldArgs::longs): on a stream of its own, after the
// prefix, beside the alias insert (both claim through the same table).
hipError_t launch_fold_longs(const FoldArgs& a, int cus, hipStream_t st);
// out[i] = out[rep] for every folded message (FoldArgs::apairs), after the hashing.
hipError_t launch_fold_fill(const FoldArgs& a, uint8_t* out, hipStream_t st);

// Clock probe (msha_clock_probe): `workgroups` x 256 lanes compress `blocks`
// register-resident blocks each; stamps gets (memtime, memrealtime) at start and
// end per workgroup, 4 words each.
hipError_t launch_clock_probe(uint32_t blocks, uint32_t workgroups, uint64_t* stamps, uint32_t* sink,
                              hipStream_t st);

}  // namespace msha
