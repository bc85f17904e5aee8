/*
 * mirsha.h -- C ABI of the MI355X batched SHA-256 digest engine for MirBFT's
 * hash path (libmirsha.so, built from mirbft_amd/csrc/).
 *
 * This is the drop-in boundary. In the reference, hashing is
 *
 *   processor.Hasher                 /root/reference/pkg/processor/serial.go:21-23
 *       New() hash.Hash              (crypto.SHA256: mirbft_test.go:392, testengine/recorder.go:781)
 *   processor.ProcessHashActions     /root/reference/pkg/processor/serial.go:180-198
 *       (hasher, *ActionList) -> (*EventList, error)
 *
 * called once per accumulated ActionList from Node.doHashWork
 * (/root/reference/mirbft.go:282-302) and from the testengine
 * (/root/reference/pkg/testengine/recorder.go:604-610). A cgo adapter packs the
 * ActionList's [][]byte parts into one arena (cgo forbids passing Go memory that
 * holds Go pointers, so [][]byte cannot cross as-is) and makes ONE call below per
 * list; see INTEGRATION.md for the binding.
 *
 * Conventions
 *  - Every function returns MSHA_OK (0) or a positive MSHA_ERR_* code; nothing
 *    throws or aborts across the ABI. msha_last_error() describes the last
 *    failure on a context (or, for ctx == NULL, the last failed context
 *    creation in the process; msha_ctx_create_err returns it with the call).
 *  - Host pointers are owned by the caller and only used during the call; the
 *    library copies into its own pinned staging and device memory and never
 *    retains them. Digests are written to caller memory (32 bytes each, in input
 *    order), so the caller can hand out fresh copies (the state machine keeps
 *    digests as map keys: batch_tracker.go:85-91, epoch_change.go:42-50).
 *  - A context may be shared between threads: calls on one context are
 *    serialised inside the library (a second caller waits for the first; the
 *    reference hashes on one goroutine anyway, mirbft.go:470), and distinct
 *    contexts run concurrently. msha_last_error(ctx) is the context's last
 *    failure, whichever thread made it. Each call selects its device(s)
 *    explicitly, so OS-thread migration between calls (goroutines) is harmless.
 *  - There is no CPU fallback: with no usable GPU, msha_ctx_create fails with
 *    MSHA_ERR_NO_DEVICE.
 */
#ifndef MIRSHA_H_
#define MIRSHA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSHA_ABI_VERSION 10u

enum {
  MSHA_OK = 0,
  MSHA_ERR_INVALID_ARG = 1, /* null pointer, range outside arena, bad bounds */
  MSHA_ERR_NO_DEVICE = 2,   /* no GPU, or device_mask names a missing device */
  MSHA_ERR_HIP = 3,         /* a HIP runtime call failed (message has details) */
  MSHA_ERR_OUT_OF_MEMORY = 4,
  MSHA_ERR_ALIGNMENT = 5    /* device-resident message not 16-byte aligned */
};

/* Bytes that must stay readable after the last message of a DEVICE arena
 * passed to the *_device entry points (the kernels read a message's final
 * block as one whole 64-byte block; bytes past each message are masked). */
#define MSHA_DEVICE_ARENA_SLACK 64u
/* Device-resident message starts must be multiples of this. */
#define MSHA_DEVICE_ALIGN 16u

typedef struct msha_ctx msha_ctx;

typedef struct {
  uint64_t calls;          /* batch calls completed */
  uint64_t messages;       /* digests produced */
  uint64_t message_bytes;  /* sum of unpadded message lengths */
  uint64_t blocks;         /* 64-byte compressions performed */
  /* Last host-memory call, milliseconds of wall time: */
  double plan_ms;          /* host planning: validation .. every shard's work queued (pinned
                              arenas: .. the last shard's kernels queued, lanes planned on the GPU) */
  double pack_ms;          /* gathering payload bytes into pinned staging (summed over shards) */
  double device_ms;        /* first upload .. last kernel on the device (HIP events, max over GPUs;
                              msha_shard_stats splits it into upload_ms and kernel_ms) */
  double total_ms;         /* whole call */
  uint64_t direct_calls;   /* host calls whose arena was uploaded as is (pinned, 16-B aligned) */
  /* Kernel launches by kind, cumulative over every entry point: */
  uint64_t launches_lane;   /* one lane per message (k_digest_batch / k_digest_uniform) */
  uint64_t launches_pipe;   /* software-pipelined lane kernel (k_digest_*_pipe), <= 1 wave/SIMD */
  uint64_t launches_coop;   /* cooperative chaining (k_digest_coop) */
  uint64_t launches_split;  /* split chaining (k_digest_split, arena or digest-of-digests) */
  uint64_t launches_dod;    /* digest-of-digests, unsplit (k_digest_of_digests) */
  uint64_t split_retries;   /* host-call shards whose split launch timed out and were re-run unsplit */
  /* Last host-memory call, summed over GPUs (see msha_get_shard_stats): */
  uint64_t h2d_bytes;       /* payload + metadata uploaded */
  uint64_t d2h_bytes;       /* digests + status words downloaded */
  uint64_t small_calls;     /* host calls served by the small-call (latency) path: one H2D, one launch, one D2H */
  uint64_t staged_calls;    /* host calls whose pageable arena had the direct path's shape (16-B aligned,
                               dense): its touched runs went up through pinned staging, lanes planned
                               on the GPU (ABI 6) */
  uint64_t planned_device_calls; /* msha_digest_batch_device_planned calls (ABI 7) */
  /* Of launches_coop, the ones that ran a chain kernel (ABI 10): */
  uint64_t launches_chain2; /* two lanes a message (k_digest_chain2): late/host heads, small AUTO launches */
  uint64_t launches_chain8; /* eight lanes a message (k_digest_chain8): the folded early head, small launches */
  uint64_t small_zc_calls;  /* of small_calls, those served zero-copy: the kernel read the packed list and wrote
                               the digests in coherent pinned memory, no H2D or D2H (ABI 10) */
  uint64_t launches_lane_ws; /* of launches_lane, the work-stealing lane kernel (k_digest_batch_ws: folded
                                planned calls; ABI 10) */
} msha_stats;

/* Per-GPU figures of the last host-memory call (one entry per shard; a shard is
 * one GPU, or one virtual shard under MSHA_VIRTUAL_SHARDS). Times are
 * milliseconds since the call began. */
typedef struct {
  int32_t device;              /* HIP device id */
  uint32_t head_lanes;         /* pinned arenas: long chains run as heads (two-lane chain kernel, CUs of
                                  their own, payloads uploaded first; ABI 8) */
  uint64_t messages;           /* messages of this shard */
  uint64_t lanes;              /* distinct payloads hashed (aliases fold) */
  uint64_t h2d_payload_bytes;  /* message bytes uploaded (compacted byte ranges or staged chunks) */
  uint64_t h2d_bytes;          /* payload + metadata */
  uint64_t d2h_bytes;
  uint64_t launches;           /* kernel launches */
  double gather_begin_ms;      /* pageable arenas: first / last gather into pinned staging */
  double gather_end_ms;
  double gather_ms;            /* time spent gathering (sum over chunks) */
  double device_ms;            /* first H2D (metadata or payload) starts .. last kernel ends (HIP
                                  events on the shard's copy and compute streams) */
  double upload_ms;            /* first H2D starts .. last payload H2D ends: h2d_bytes / upload_ms
                                  is the shard's achieved PCIe rate */
  double kernel_ms;            /* first hash kernel starts .. last kernel ends */
  double first_launch_ms;      /* host: call start .. the shard's first hash kernel enqueued */
  double plan_kernel_ms;       /* pinned arenas: the GPU lane planner's kernels (plan.hip) */
} msha_shard_stats;

uint32_t msha_abi_version(void);

/* The build this library is: "src=<16 hex>;flags=<compile flags>", where src is
 * a hash of the sources it was compiled from (mirbft_amd/csrc/Makefile). A test
 * log names the build it ran with it; tests/conftest.py refuses a GPU session
 * whose library is not the tree's own (an experiment's build left in place).
 * Diagnostic, no reference counterpart (ABI 9). */
const char* msha_build_id(void);

/* Number of visible HIP devices (0 when none). */
int msha_device_count(int* n);

/* Create a context on the devices in device_mask (bit i = HIP device i);
 * device_mask == 0 means "device 0". Independent actions are sharded across
 * the masked devices (one stream per device, partitioned by cumulative block
 * count); no inter-GPU collective is used.
 * On failure the reason is written, NUL-terminated, into errbuf (when errbuf
 * is not NULL and errbuf_len > 0): the error travels with the call, so a
 * caller whose thread may change between two calls (a goroutine) still gets it. */
int msha_ctx_create_err(uint32_t device_mask, msha_ctx** out, char* errbuf, uint64_t errbuf_len);
/* The same; the reason of the most recent failed creation in the PROCESS is
 * then readable through msha_last_error(NULL) (prefer msha_ctx_create_err when
 * several threads create contexts). */
int msha_ctx_create(uint32_t device_mask, msha_ctx** out);
void msha_ctx_destroy(msha_ctx* ctx);
/* The context's last failure (ctx == NULL: the last failed creation). The
 * pointer stays valid for the context's life, but another thread's failing call
 * on the same context may rewrite the text while it is read: read it only while
 * no other call runs on the context, or use msha_last_error_copy. */
const char* msha_last_error(const msha_ctx* ctx);
/* Copy of the same text into buf (NUL-terminated, truncated to buf_len - 1),
 * taken under the context's lock: safe while other threads use the context.
 * Returns the text's full length. */
uint64_t msha_last_error_copy(const msha_ctx* ctx, char* buf, uint64_t buf_len);
int msha_get_stats(const msha_ctx* ctx, msha_stats* out);
/* Shards of the context (GPUs in device_mask, or virtual shards). */
int msha_shard_count(const msha_ctx* ctx, uint32_t* n);
int msha_get_shard_stats(const msha_ctx* ctx, uint32_t shard, msha_shard_stats* out);

/*
 * ProcessHashActions over a packed arena (serial.go:180-198).
 *   part j           = arena[part_off[j] : part_off[j] + part_len[j]]
 *   action i's parts = parts [action_part_begin[i], action_part_begin[i+1])
 *   out[32*i ...]    = SHA-256(concatenation of action i's parts)
 * Zero-part actions hash the empty string; empty parts contribute nothing;
 * parts may overlap or repeat. action_part_begin has n_actions+1 entries,
 * non-decreasing, action_part_begin[0] == 0, last == n_parts.
 */
int msha_hash_actions(msha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* part_off, const uint64_t* part_len, uint64_t n_parts,
                      const uint64_t* action_part_begin, uint64_t n_actions, uint8_t* out);

/*
 * One-part messages (request digests, clients.go:189-192; or any action whose
 * parts the caller already concatenated): out[32*i] = SHA-256(arena[off[i] :
 * off[i]+len[i]]). Several messages may alias one payload (EpochChange
 * re-hashing, epoch_target.go:486-505): it is copied to the device once.
 */
int msha_digest_batch(msha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* off, const uint64_t* len, uint64_t n, uint8_t* out);

/*
 * Batch / VerifyBatch digest over request-ack digests (sequence.go:155-158,
 * batch_tracker.go:175-178) when every part is a 32-byte digest:
 *   out[32*i] = SHA-256(table[idx[k]] for k in [begin[i], begin[i+1]))
 * table is n_table x 32 bytes; begin has n+1 entries.
 */
int msha_digest_of_digests(msha_ctx* ctx, const uint8_t* table, uint64_t n_table,
                           const uint32_t* idx, uint64_t n_idx, const uint64_t* begin,
                           uint64_t n, uint8_t* out);

/*
 * Device-resident (kernel-resident) forms, for callers that keep inputs in
 * HBM: every pointer is device memory on the context's FIRST device and the
 * work is enqueued on `stream` (a hipStream_t, NULL = the context's own
 * stream); the call returns after enqueueing. Arena rules: message starts
 * MSHA_DEVICE_ALIGN-aligned, MSHA_DEVICE_ARENA_SLACK readable bytes after the
 * last message. A misaligned start is reported by msha_device_status() and its
 * digest is zeroed (never a wrong digest). d_order (may be NULL) is a
 * permutation of [0, n): lane i hashes message d_order[i] (digest still lands
 * at d_out + 32*d_order[i]); pass msha_order_by_blocks()'s output for batches
 * of mixed sizes so every wavefront's lanes run the same number of blocks.
 */
int msha_digest_batch_device(msha_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                             const uint64_t* d_len, const uint32_t* d_order, uint64_t n,
                             uint8_t* d_out, void* stream);
/*
 * The same messages, planned on the GPU inside the call's own launches (no host
 * round trip, nothing precomputed by the caller): lanes are ordered by
 * descending block count; with MSHA_PLAN_FOLD_ALIASES, messages with equal
 * (d_off, d_len) -- EpochChange payloads re-hashed N^2 times,
 * epoch_target.go:486-505 -- are hashed once and the digest copied to every
 * such slot; and the longest chains, when one alone would outlast the rest of
 * the launch (a mixed storm sharded over several GPUs), run on the cooperative
 * kernel beside the lane kernel (a side stream forked from and joined back to
 * `stream`). Same arena rules and error reporting as msha_digest_batch_device;
 * n < 2^31. Returns after enqueueing. Not capturable into a HIP graph: the
 * call orders itself after the previous planned call through a library event
 * and forks to a library-owned stream, so on a capturing stream it fails with
 * MSHA_ERR_INVALID_ARG (msha_digest_batch_device captures).
 */
enum { MSHA_PLAN_FOLD_ALIASES = 1u };
int msha_digest_batch_device_planned(msha_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                                     const uint64_t* d_len, uint64_t n, uint32_t flags, uint8_t* d_out,
                                     void* stream);
/* Uniform layout: message i = d_arena[i*stride : i*stride + msg_len] (stride a
 * multiple of 16; messages may overlap, stride 0 hashes one message n times). */
int msha_digest_uniform_device(msha_ctx* ctx, const uint8_t* d_arena, uint64_t stride,
                               uint64_t msg_len, uint64_t n, uint8_t* d_out, void* stream);
int msha_digest_of_digests_device(msha_ctx* ctx, const uint8_t* d_table, const uint32_t* d_idx,
                                  const uint64_t* d_begin, uint64_t n, uint8_t* d_out,
                                  void* stream);
/* Synchronizes the context's first device and reports (then clears) any
 * device-side error flag raised by *_device calls: MSHA_OK, MSHA_ERR_ALIGNMENT, or
 * MSHA_ERR_HIP if a split-chaining handoff (kernels.hip) waited over 100 ms. */
int msha_device_status(msha_ctx* ctx);

/*
 * Kernel policy for one-part messages (msha_digest_batch, msha_hash_actions,
 * msha_digest_batch_device). Results are identical under every policy.
 *  MSHA_KERNEL_AUTO  (default) one lane per message when a launch has enough
 *                    messages to give every SIMD a wavefront; otherwise
 *                    cooperative chaining
 *  MSHA_KERNEL_LANE  always one wavefront lane per message
 *  MSHA_KERNEL_COOP  always cooperative chaining: per 64 messages a producer
 *                    wavefront expands the message schedules into LDS while a
 *                    consumer wavefront runs only the rounds (lower latency per
 *                    message; for few, large messages)
 */
enum { MSHA_KERNEL_AUTO = 0, MSHA_KERNEL_LANE = 1, MSHA_KERNEL_COOP = 2 };
int msha_set_kernel_policy(msha_ctx* ctx, int policy);

/*
 * Diagnostics (ABI 8): the clock the context's first GPU holds under the hash
 * kernels' instruction mix. A probe kernel compresses register-resident blocks
 * at the lane kernel's occupancy (8 waves per SIMD) and stamps s_memtime (shader
 * clock) and s_memrealtime (100 MHz) at each workgroup's start and end; the
 * clock is their ratio. Synchronous; run it right after the work whose clock
 * matters (the hash kernels carry no stamps). blocks_per_lane in [1, 100000]
 * (48: about 1 ms).
 */
typedef struct {
  double ghz_median;     /* over workgroups */
  double ghz_min;
  double ghz_max;
  double kernel_ms;      /* the probe launch, HIP events */
  double gblocks_per_s;  /* register-resident compression rate of the probe */
  uint32_t workgroups;
  uint32_t blocks_per_lane;
} msha_clock_info;
int msha_clock_probe(msha_ctx* ctx, uint32_t blocks_per_lane, msha_clock_info* out);

/* Pinned host memory for callers that want zero-copy staging: when the arena
 * passed to msha_digest_batch lies in such memory, every message start is
 * 16-byte aligned and the messages are packed without large gaps, each GPU's
 * byte span of it is DMA'd as is (no gather copy into the library's staging).
 * On a context whose GPUs sit on several NUMA nodes the allocation is cut into
 * one region per shard, in shard order, each placed on its GPU's node and
 * page-locked with hipHostRegister (MSHA_PINNED_STRIPE=1 forces, =0 disables):
 * a batch packed in message order then feeds each GPU from its own socket. */
int msha_pinned_alloc(msha_ctx* ctx, uint64_t bytes, void** p);
int msha_pinned_free(msha_ctx* ctx, void* p);

/*
 * Host-only helpers (no GPU needed).
 * msha_blocks_for_len: number of 64-byte compressions for an L-byte message,
 *   floor(L/64) + (L%64 < 56 ? 1 : 2)  (FIPS 180-4 5.1.1 padding).
 * msha_partition_by_blocks: split messages [0, n) into n_shards contiguous
 *   ranges of near-equal cumulative block count; bounds[0..n_shards]
 *   (bounds[0] = 0, bounds[n_shards] = n). Used for multi-GPU sharding.
 */
uint64_t msha_blocks_for_len(uint64_t len);
/* Permutation of [0, n) ordering messages by descending block count (stable). */
int msha_order_by_blocks(const uint64_t* len, uint64_t n, uint32_t* order);
int msha_partition_by_blocks(const uint64_t* len, uint64_t n, uint32_t n_shards,
                             uint64_t* bounds);
/* Alias detection the host entry points run before hashing (EpochChange
 * payloads re-hashed N^2 times, epoch_target.go:486-505): first[i] = the
 * smallest j <= i with (off[j], len[j]) == (off[i], len[i]); such messages are
 * hashed once and share the digest. */
int msha_alias_first(const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* first);

#ifdef __cplusplus
}
#endif

#endif /* MIRSHA_H_ */
