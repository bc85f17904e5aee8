// HIP kernels for the batched SHA-256 digest engine (gfx950 only).
//
// Replaces, per message, Go crypto/sha256 as driven by
// processor.ProcessHashActions (/root/reference/pkg/processor/serial.go:180-198):
// every lane of a wavefront owns one hash action's message and runs
// New/Write/Sum for it entirely in VGPRs. The kernels apply FIPS 180-4 padding
// themselves from the length, so the host never writes padding bytes.
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   arena  : message bytes, each message 16-byte aligned (the host packer
//            guarantees this; a misaligned device-API message is flagged and
//            its digest zeroed, never computed wrongly), 64 B slack at the end
//   off/len: uint64 per message (several messages may alias one payload)
//   order  : optional uint32 permutation (size-class binning: lanes of a wave
//            get messages of equal block count so no lane idles)
//   out    : 32 bytes per message, digest i at out + 32*i
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "sha256_device.hpp"
#include "kernels.hpp"

namespace msha {

// ---------------------------------------------------------------------------
// Wave stamps: diagnostic build only (-DMSHA_LANE_STAMPS, tools/lane_stamps.sh;
// VERDICT r5 item 1). Every wave of the hash kernels records, from lane 0, the
// shader clock (s_memtime) and the 100 MHz wall clock (s_memrealtime) when it
// starts and when its last lane is done, the SIMD / CU / SE / XCD it ran on
// (HW_ID, XCC_ID) and which kernel it was, into a buffer of its own
// (msha_diag_stamps): the in-kernel clock, when each workgroup started, and how
// many SIMDs each kernel held over time, for one step of a real launch. The
// product build compiles every hook below to nothing (tools/kernel_isa.py shows
// the kernels' code unchanged).
// ---------------------------------------------------------------------------
enum StampKind : uint32_t { kStampLane = 1, kStampPipe = 2, kStampChain2 = 3, kStampChain8 = 4, kStampCoop = 5 };
#ifdef MSHA_LANE_STAMPS
struct WaveStampRec {
  uint64_t t0, r0, t1, r1;  // s_memtime / s_memrealtime at the wave's start and end
  uint32_t hw_id, xcc_id, kind, block;
  uint32_t wave, work;      // work: the lane kernel's largest block count in the wave | active lanes << 16
  uint64_t pad1;
};
__device__ WaveStampRec* g_wave_stamps;
__device__ uint32_t* g_wave_stamp_count;  // [1]: records per kind (the buffer holds 5 x that)
struct WaveStamp {
  uint64_t t0, r0;
  __device__ __forceinline__ WaveStamp() : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ __forceinline__ void close(uint32_t kind, uint32_t nb = 0, uint64_t at = ~0ull) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t mx = nb;
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
    const uint32_t lanes = (uint32_t)__popcll(__ballot(nb != 0));
    if ((threadIdx.x & 63) != 0 || !g_wave_stamps) return;
    // a fixed slot per (kind, wave): a shared counter's returning atomic at every
    // wave's end queued the waves behind it (c2's stamped step ran 2.3x longer)
    const uint32_t per = g_wave_stamp_count[1];
    const uint64_t w = at != ~0ull ? at : (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= per) return;
    const uint64_t k = (uint64_t)(kind - 1) * per + w;
    WaveStampRec r;
    r.t0 = t0;
    r.r0 = r0;
    r.t1 = t1;
    r.r1 = r1;
    r.hw_id = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID, 32 bits
    r.xcc_id = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID, 4 bits
    r.kind = kind;
    r.block = blockIdx.x;
    r.wave = threadIdx.x >> 6;
    r.work = min(mx, 0xFFFFu) | (lanes << 16);
    r.pad1 = 0;
    g_wave_stamps[k] = r;
  }
};
#define MSHA_WAVE_STAMP_OPEN() WaveStamp wave_stamp_;
#define MSHA_WAVE_STAMP_CLOSE(kind) wave_stamp_.close(kind);
#define MSHA_WAVE_STAMP_CLOSE_NB(kind, nb) wave_stamp_.close(kind, nb);
#define MSHA_WAVE_STAMP_CLOSE_AT(kind, nb, at) wave_stamp_.close(kind, nb, at);
}  // namespace msha
// Diagnostic build only: points the stamps at `buf` (device memory, 5 x per
// records of 64 B: one region per StampKind, a wave's record at its wave index)
// and `counter` (device uint32[2]: [1] = per). The caller zeroes the buffer
// before the launch it wants; a record with t0 == 0 was not written. NULL buf:
// stamps off.
extern "C" int msha_diag_wave_stamps(void* buf, void* counter) {
  msha::WaveStampRec* b = static_cast<msha::WaveStampRec*>(buf);
  uint32_t* c = static_cast<uint32_t*>(counter);
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::g_wave_stamps), &b, sizeof b) != hipSuccess) return 3;
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::g_wave_stamp_count), &c, sizeof c) != hipSuccess) return 3;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
namespace msha {
#else
#define MSHA_WAVE_STAMP_OPEN()
#define MSHA_WAVE_STAMP_CLOSE(kind)
#define MSHA_WAVE_STAMP_CLOSE_NB(kind, nb)
#define MSHA_WAVE_STAMP_CLOSE_AT(kind, nb, at)
#endif

template <int MODE = 0>
__device__ __forceinline__ void load_block16(const uint8_t* p, uint32_t (&raw)[16]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 v = q[i];
    raw[4 * i + 0] = v.x; raw[4 * i + 1] = v.y; raw[4 * i + 2] = v.z; raw[4 * i + 3] = v.w;
  }
}

__device__ __forceinline__ void to_words(const uint32_t (&raw)[16], uint32_t (&w)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = bswap(raw[j]);
}

// How a lane brings its message blocks in from HBM (all modes are bit-identical):
//  kSingle   load block b at the top of iteration b; latency hidden by the
//            other waves of the SIMD (high occupancy)
//  kPrefetch load block b+1 while block b is compressed (16 more live VGPRs):
//            for few, long messages, where there are too few waves to hide it
//  kPair     at even b load blocks b and b+1 together: both halves of a
//            128-byte line are requested back to back, so the line is read
//            from HBM once instead of being evicted and re-fetched between
//            the two half-line requests (lane stride >= 128 B is the norm)
// (Rejected after A/B, profiles/r01_ab_modes, r01_ab_nt: an LDS-DMA prefetch
// mode, 6 % slower on c2, and nontemporal payload loads, 5-10 % slower.)
enum LoadMode { kSingle = 0, kPrefetch = 1, kPair = 2, kPipe = 3 };

// Hash one message of `len` bytes starting at p (device memory, 16-byte
// aligned, with kArenaSlack (kernels.hpp) readable bytes after the arena's last
// message) into out. One compress() call site: full blocks, the tail block
// and the optional extra length block all go through the same loop body.
// The tail block is read as a whole 64-byte block (it may run into the next
// message or the slack); build_tail() masks every byte at or past `len`.
template <int MODE>
__device__ __forceinline__ void hash_message(const uint8_t* p, uint64_t len, uint8_t* out) {
  State s;
  state_init(s);
  const uint32_t nfull = (uint32_t)(len >> 6);  // < 2^32 blocks: messages < 256 GiB
  const uint32_t r = (uint32_t)(len & 63);
  const uint32_t nblocks = nfull + (r < 56 ? 1 : 2);
  // Wave-uniform length (the common batch shape: request digests, Batch
  // digests, large payloads) whose last block carries no message byte: that
  // block goes to compress_uniform_pad() (schedule on the SALU) after the loop.
  const uint32_t len_lo0 = __builtin_amdgcn_readfirstlane((uint32_t)len);
  const uint32_t len_hi0 = __builtin_amdgcn_readfirstlane((uint32_t)(len >> 32));
  const uint64_t len0 = ((uint64_t)len_hi0 << 32) | len_lo0;
  const bool uniform = __ballot(len != len0) == 0;
  const uint32_t r0 = len_lo0 & 63;
  const bool upad = uniform && (r0 == 0 || r0 >= 56);
  const uint32_t nvalu = nblocks - (upad ? 1 : 0);
  uint32_t raw[16];
  uint32_t w[16];
  constexpr int LM = MODE;  // load mode
  if (LM == kPrefetch) load_block16<MODE>(p, raw);
  for (uint32_t b = 0; b < nvalu; ++b) {
    const uint8_t* pb = p + 64 * (uint64_t)b;
    if (LM == kSingle && b <= nfull) load_block16<MODE>(pb, raw);
    if (LM == kPair && b == nfull && !(b & 1)) load_block16<MODE>(pb, raw);
    if (b < nfull) {
      if (LM == kPair) {
        if (!(b & 1)) {
          uint32_t t[16];
          load_block16<MODE>(pb, t);
          load_block16<MODE>(pb + 64, raw);  // block b+1, or the tail block's bytes (slack-safe)
          to_words(t, w);
        } else {
          to_words(raw, w);
        }
      } else {
        to_words(raw, w);
        if (LM == kPrefetch) load_block16<MODE>(pb + 64, raw);
      }
    } else if (b == nfull) {
      // Launder r so the 16 per-dword tail masks are built here, once, and
      // not hoisted out of the loop into 32 loop-long VGPRs.
      uint32_t rr = r;
      asm volatile("" : "+v"(rr));
      build_tail(raw, rr, len, w);
    } else {
      length_block(len, w);
    }
    compress(s, w);
  }
  if (upad) {
    const uint64_t bits = len0 * 8;
    compress_uniform_pad(s, r0 == 0 ? 0x80000000u : 0u, (uint32_t)(bits >> 32), (uint32_t)bits);
  }
  store_digest(s, out);
}

// ---------------------------------------------------------------------------
// Software-pipelined lane kernel (kPipe) for launches of about one wave per
// SIMD (few, long messages: c4's 65,536 x 64 KiB is exactly 1,024 waves on
// 1,024 SIMDs). A lone wave issues a VALU instruction only every ~4.6 cycles
// (vs ~3.9 with 2+ waves): nothing else on the SIMD fills the gaps
// of the round chain, and in compress() rounds 0-15 have no schedule work at
// all. Here block b's 64 rounds consume a fully expanded schedule W[64], and
// the same straight-line code expands block b+1's schedule (independent of
// the rounds) into a second array, one word per round; the raw bytes of block
// b+2 are loaded at the top of the step. Two schedule arrays and two raw
// buffers ping-pong, so nothing is copied. ~190 VGPRs: one wave per SIMD.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void expand_block(const uint32_t (&raw)[16], uint32_t (&N)[64]) {
#pragma unroll
  for (int i = 0; i < 64; ++i)
    N[i] = i < 16 ? bswap(raw[i]) : sig1(N[i - 2]) + N[i - 7] + sig0(N[i - 15]) + N[i - 16];
}

constexpr int pipe_slot(int j) { return j < 16 ? j / 4 : 4 + (j - 16) * 5 / 4; }

// 64 rounds over the expanded W, interleaved word by word with the expansion
// of `raw` (the next block) into N.
__device__ __forceinline__ void rounds_expand(State& s, const uint32_t (&W)[64], uint32_t (&N)[64],
                                              const uint32_t (&raw)[16]) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = h + K[i] + W[i] + Sig1(e) + ch(e, f, g);
    const uint32_t t2 = Sig0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
    // Words due at round i (pipe_slot): byte swaps in rounds 0-3, then the 48
    // expanded words spread evenly over rounds 4-62.
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = (i < 4 ? 4 * i : 16 + (i - 4) * 4 / 5) + k;
      if (j < 64 && pipe_slot(j) == i) {
        N[j] = j < 16 ? bswap(raw[j]) : sig1(N[j - 2]) + N[j - 7] + sig0(N[j - 15]) + N[j - 16];
        asm volatile("" : "+v"(N[j]));
      }
    }
    // Keep round i and its words together: left alone, instruction selection
    // lumps the expansion into a few rounds and leaves the rest bare. Passing
    // the values through an empty volatile asm orders them (emits nothing).
    asm volatile("" : "+v"(a), "+v"(e));
  }
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

__device__ __forceinline__ void hash_message_pipe(const uint8_t* p, uint64_t len, uint8_t* out) {
  State s;
  state_init(s);
  const uint32_t nfull = (uint32_t)(len >> 6);
  const uint32_t r = (uint32_t)(len & 63);
  const uint32_t nblocks = nfull + (r < 56 ? 1 : 2);
  const uint32_t len_lo0 = __builtin_amdgcn_readfirstlane((uint32_t)len);
  const uint32_t len_hi0 = __builtin_amdgcn_readfirstlane((uint32_t)(len >> 32));
  const uint64_t len0 = ((uint64_t)len_hi0 << 32) | len_lo0;
  const bool uniform = __ballot(len != len0) == 0;
  const uint32_t r0 = len_lo0 & 63;
  const bool upad = uniform && (r0 == 0 || r0 >= 56);
  const uint32_t nvalu = nblocks - (upad ? 1 : 0);
  // Block j's bytes, clamped to the tail block (always readable: arena slack).
  auto blk = [&](uint32_t j) { return p + 64 * (uint64_t)(j < nfull ? j : nfull); };
  uint32_t tail[16];
  if (nfull == 0) {
    load_block16(p, tail);
  } else {
    // Raw block buffers X, Y, Z, V rotate over four steps; each pair of blocks
    // (b+2, b+3 with b even) is requested together, both halves of a 128-byte
    // line back to back, so the line is read from HBM once (one block per
    // request read c4's lines twice: 1.14x the algorithmic bytes).
    uint32_t A[64], B[64], X[16], Y[16], Z[16], V[16];
    load_block16(p, X);
    expand_block(X, A);
    load_block16(blk(1), X);
    uint32_t b = 0;
    // The tail block's bytes are loaded again after the loop (one 64-byte load a
    // message) rather than taken from whichever raw buffer held them: with exit
    // copies out of the rotating buffers the register allocator copied raw
    // buffers inside the loop (8 v_mov a block).
    for (;;) {
      // A = schedule of block b (b % 4 == 0), X = bytes of block b+1 (clamped)
      load_block16(blk(b + 2), Y);
      load_block16(blk(b + 3), Z);
      rounds_expand(s, A, B, X);
      if (++b >= nfull) break;
      rounds_expand(s, B, A, Y);  // B = block b, Y = block b+1
      if (++b >= nfull) break;
      load_block16(blk(b + 2), V);
      load_block16(blk(b + 3), X);
      rounds_expand(s, A, B, Z);  // A = block b, Z = block b+1
      if (++b >= nfull) break;
      rounds_expand(s, B, A, V);  // B = block b, V = block b+1
      if (++b >= nfull) break;
    }
    load_block16(blk(nfull), tail);
  }
  uint32_t w[16];
  for (uint32_t b = nfull; b < nvalu; ++b) {
    if (b == nfull) {
      uint32_t rr = r;
      asm volatile("" : "+v"(rr));
      build_tail(tail, rr, len, w);
    } else {
      length_block(len, w);
    }
    compress(s, w);
  }
  if (upad) {
    const uint64_t bits = len0 * 8;
    compress_uniform_pad(s, r0 == 0 ? 0x80000000u : 0u, (uint32_t)(bits >> 32), (uint32_t)bits);
  }
  store_digest(s, out);
}

// Misaligned message start: not produced by the library's packers; flagged
// (device word *err |= 1) and the digest zeroed rather than computed wrongly.
__device__ __forceinline__ bool check_aligned(const uint8_t* p, uint8_t* out, uint32_t* err) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) return true;
  atomicOr(err, 1u);
  reinterpret_cast<uint4*>(out)[0] = make_uint4(0, 0, 0, 0);
  reinterpret_cast<uint4*>(out)[1] = make_uint4(0, 0, 0, 0);
  return false;
}

// Returns the message's length (diagnostic stamps only; 0 for an idle lane).
template <int MODE>
__device__ __forceinline__ uint64_t digest_batch_lane(const uint8_t* __restrict__ arena,
                                                      const uint64_t* __restrict__ off,
                                                      const uint64_t* __restrict__ len,
                                                      const uint32_t* __restrict__ order,
                                                      const uint32_t* __restrict__ out_idx, uint64_t n,
                                                      uint8_t* __restrict__ out, uint32_t* __restrict__ err,
                                                      const uint32_t* __restrict__ skip_below) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return 0;
  if (skip_below && i < *skip_below) return 0;  // a long chain: the cooperative launch has it
  uint64_t m = i;                             // metadata index
  if (order) {
    const uint32_t v = order[i];
    if (v == kNoLane) return 0;               // planned launch: a folded alias's position
    m = v;
  }
  const uint64_t o = out_idx ? (uint64_t)out_idx[i] : m;  // digest slot
  const uint8_t* p = arena + off[m];
  const uint64_t l = len[m];
  if (check_aligned(p, out + 32 * o, err))
    hash_message<MODE>(p, l, out + 32 * o);
  return l + 1;
}

template <int MODE>
__global__ __launch_bounds__(256, 8) void k_digest_batch(const uint8_t* __restrict__ arena,
                                                      const uint64_t* __restrict__ off,
                                                      const uint64_t* __restrict__ len,
                                                      const uint32_t* __restrict__ order,
                                                      const uint32_t* __restrict__ out_idx,
                                                      uint64_t n, uint8_t* __restrict__ out,
                                                      uint32_t* __restrict__ err,
                                                      const uint32_t* __restrict__ skip_below) {
  MSHA_WAVE_STAMP_OPEN()
  const uint64_t l1 = digest_batch_lane<MODE>(arena, off, len, order, out_idx, n, out, err, skip_below);
  MSHA_WAVE_STAMP_CLOSE_NB(kStampLane, l1 ? (uint32_t)((l1 - 1) >> 6) + ((((l1 - 1) & 63) < 56) ? 1u : 2u) : 0u)
  (void)l1;
}

// ---------------------------------------------------------------------------
// The lane kernel with work stealing (round 6, VERDICT r5 item 1: folded c5's lane
// kernel ran at 0.465 of the peak against c2's 0.502 with equal instructions and
// cycles per instruction). Wave stamps of a folded step (tools/lane_stamps.py,
// profiles/r06_xcd/) showed why: a launch's workgroups go to the XCDs by blockIdx
// mod 8, and an XCD that also holds a long-lived wave -- the late head's chain
// (2 ms), or a 652-block chain left on the lane kernel -- dispatches its lane
// workgroups at ~3 resident waves per SIMD instead of 8, so its fixed eighth of
// the lanes ends ~250 us after the other XCDs' while they idle (SIMDs busy 91 %
// of the span, against 98 % on c2; cycles per wave-block while busy equal).
// Here a grid of resident workgroups (8 a CU) takes 64-lane tiles from kWsSlots
// counters: slot s owns the tiles t = s + kWsSlots k, so every slot holds the same
// mix of classes (descending, as the lanes are ordered), and workgroup b starts on
// slot b mod kWsSlots (the same XCD as b). A wave whose slot is used up looks at
// every other slot at once (one counter a lane, agent-scope loads) and takes a
// tile from the first with some left. Nothing is dispatched after the start, so a
// throttled dispatcher costs nothing but its few late workgroups, and an XCD that
// runs slow takes fewer tiles. 64 counters, 64 bytes apart: eight (one an XCD)
// serialised ~2.3 M claims/s each and ran folded c5 at 7 ms (profiles/r06_ws/).
// Termination: a claim past a slot's count proves the slot used up (counters only
// grow), and the scan's loads are coherent, so each wave fails on a slot at most
// once and leaves when no slot has tiles left.
// ctr: kWsSlots x kWsStride zeroed words (the planner's memset); lanes_dev (may be
// null): a device count of the positions worth visiting (the planner's lanes: the
// kNoLane tail past it is never claimed).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256, 8) void k_digest_batch_ws(const uint8_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ off,
                                                         const uint64_t* __restrict__ len,
                                                         const uint32_t* __restrict__ order,
                                                         const uint32_t* __restrict__ out_idx, uint64_t n,
                                                         uint8_t* __restrict__ out, uint32_t* __restrict__ err,
                                                         const uint32_t* __restrict__ skip_below,
                                                         uint32_t* __restrict__ ctr,
                                                         const uint32_t* __restrict__ lanes_dev) {
  static_assert(kWsSlots == 64, "the steal scan gives each lane one slot");
  const uint64_t n_eff = lanes_dev ? min(n, (uint64_t)*lanes_dev) : n;
  const uint32_t tiles = (uint32_t)((n_eff + 63) / 64);
  const unsigned lane = threadIdx.x & 63;
  uint32_t slot = blockIdx.x % kWsSlots;
  // A claim taken one tile ahead (its atomic issued as a tile starts, read as it
  // ends) measured 30 us slower on folded c5 (2.656 vs 2.625 ms, 3 reps,
  // profiles/r06_ws/prefetch/): the atomic sits ahead of the tile's block loads in
  // the in-order vmcnt, so the first load's wait paid its latency anyway.
  for (;;) {
    const uint32_t cnt = slot < tiles ? (tiles - 1 - slot) / kWsSlots + 1 : 0;
    uint32_t* c = ctr + slot * kWsStride;
    uint32_t k = cnt;
    if (lane == 0 && __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cnt) k = atomicAdd(c, 1u);
    k = __builtin_amdgcn_readfirstlane(k);
    if (k >= cnt) {  // used up: the slots with tiles left, one per lane
      const uint32_t s2 = (slot + 1 + lane) % kWsSlots;
      const uint32_t c2 = s2 < tiles ? (tiles - 1 - s2) / kWsSlots + 1 : 0;
      const bool left = __hip_atomic_load(ctr + s2 * kWsStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c2;
      const uint64_t any = __ballot(left);
      if (!any) break;
      slot = __builtin_amdgcn_readfirstlane(__shfl(s2, __ffsll((long long)any) - 1));
      continue;
    }
    const uint32_t t = k * kWsSlots + slot;
    MSHA_WAVE_STAMP_OPEN()
    const uint64_t i = (uint64_t)t * 64 + lane;
    uint64_t l1 = 0;
    uint64_t m = i;
    bool live = i < n_eff && !(skip_below && i < *skip_below);
    if (live && order) {
      const uint32_t v = order[i];
      live = v != kNoLane;
      m = v;
    }
    const uint64_t l = live ? len[m] : 0;
    const uint64_t mo = live ? off[m] : 0;  // issued beside len's load, before the priority's reduction
    // Issue priority by the tile's longest chain. A statically mapped launch
    // dispatches its longest lanes first, and the SIMD's oldest-first issue then
    // runs those chains nearly alone; resident waves are all the same age, so
    // without this a long chain shared its SIMD evenly with short tiles and ended
    // last (unfolded c5 13.3 -> 20.8 ms, profiles/r06_ws/).
    uint32_t nb = live ? (uint32_t)(l >> 6) + ((l & 63) < 56 ? 1u : 2u) : 0u;
    for (int d = 32; d > 0; d >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, d));
    nb = __builtin_amdgcn_readfirstlane(nb);
    if (nb >= 256)
      __builtin_amdgcn_s_setprio(3);
    else if (nb >= 48)
      __builtin_amdgcn_s_setprio(2);
    else if (nb >= 16)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
    if (live) {
      const uint64_t o = out_idx ? (uint64_t)out_idx[i] : m;
      const uint8_t* p = arena + mo;
      if (check_aligned(p, out + 32 * o, err)) hash_message<MODE>(p, l, out + 32 * o);
      l1 = l + 1;
    }
    MSHA_WAVE_STAMP_CLOSE_AT(kStampLane, l1 ? (uint32_t)((l1 - 1) >> 6) + ((((l1 - 1) & 63) < 56) ? 1u : 2u) : 0u, t)
    (void)l1;
  }
}

// k_digest_batch with the pipelined message loop; no occupancy hint (one wave
// per SIMD is the design point, the VGPRs are the schedule arrays).
__global__ __launch_bounds__(256) void k_digest_batch_pipe(const uint8_t* __restrict__ arena,
                                                           const uint64_t* __restrict__ off,
                                                           const uint64_t* __restrict__ len,
                                                           const uint32_t* __restrict__ order,
                                                           const uint32_t* __restrict__ out_idx,
                                                           uint64_t n, uint8_t* __restrict__ out,
                                                           uint32_t* __restrict__ err,
                                                           const uint32_t* __restrict__ skip_below) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip_below && i < *skip_below) return;
  uint64_t m = i;
  if (order) {
    const uint32_t v = order[i];
    if (v == kNoLane) return;
    m = v;
  }
  const uint64_t o = out_idx ? (uint64_t)out_idx[i] : m;
  const uint8_t* p = arena + off[m];
  if (check_aligned(p, out + 32 * o, err))
    hash_message_pipe(p, len[m], out + 32 * o);
}

// ---------------------------------------------------------------------------
// Split chaining (tail balance). One lane per message leaves a launch of
// q*S + r wavefronts (S = SIMDs, 0 < r < S) with r SIMDs running q+1 waves
// while the rest run q: c3's 200 K Batch digests are 3,125 waves on 1,024
// SIMDs, so 53 SIMDs set the time at 4 waves' worth of work (VALU busy 66 %).
// A message's chain is serial, but it can be paused: its 32-byte state saved
// and resumed by another wavefront. The launch runs the first q*S waves as
// usual ("main" workgroups) and hands the remaining r waves' messages to r
// chains of S_seg segments each; segment s of a chain does blocks
// [nb*s/S_seg, nb*(s+1)/S_seg) of its 64 messages on a wave of its own, at high
// issue priority, then publishes the state (in the message's own digest slot)
// and a flag; segment s+1 (another workgroup, so usually another SIMD) waits for
// that flag. Each SIMD then carries at most ~1/S_seg of a surplus wave instead
// of a whole one. Segment workgroups come first in the grid and a segment
// only ever waits on a lower workgroup id of its own XCD (dispatched before
// it), so every wait is on a resident or finished wave.
//
// A chain's flag word: epoch (bits 63..40) | segments done (39..32) | beat.
// The running segment stores a new beat every kBeatBlocks (8) blocks, so a
// waiter can tell a long chain (huge messages) from a stuck one: only 100 ms
// without any change of the word (never expected) raises error bit 2 and
// unblocks the chain, so every wave exits. The host entry points then re-run
// the launch unsplit (msha_stats.split_retries); the device entry points
// report MSHA_ERR_HIP through msha_device_status. The clock only runs while
// the waiter itself runs: a gap of over 1 ms between two of its own polls
// means the queue was descheduled (time slicing, another process), and the
// running segment was frozen with it, so the wait restarts.
// ---------------------------------------------------------------------------
constexpr uint64_t kSplitWaitTicks = 10000000;  // 100 ms of s_memrealtime (100 MHz)
constexpr uint64_t kSplitDeschedTicks = 100000;  // 1 ms between two polls: descheduled

__device__ __forceinline__ uint64_t split_word(uint64_t epoch, uint32_t done, uint32_t beat) {
  return ((epoch & 0xFFFFFFu) << 40) | ((uint64_t)(done & 0xFFu) << 32) | beat;
}

// Progress beat of the running segment, every 8 blocks (one store per ~20 us;
// a beat per block cost c3 1.5 %). ArenaSrc beats between 8-block runs of its
// block loop: a conditional store inside that loop made the compiler spill.
constexpr uint32_t kBeatBlocks = 8;
struct Beat {
  uint64_t* flag;
  uint64_t base;
  __device__ __forceinline__ void operator()(uint32_t b) const {
    __hip_atomic_store(flag, base | b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// Blocks [b0, b1) of the message at p (len bytes), state in/out in s.
__device__ __forceinline__ void hash_blocks(State& s, const uint8_t* p, uint64_t len, uint32_t b0,
                                            uint32_t b1) {
  const uint32_t nfull = (uint32_t)(len >> 6);
  const uint32_t r = (uint32_t)(len & 63);
  uint32_t w[16];  // loaded, then byte-swapped / masked in place (no second array)
  for (uint32_t b = b0; b < b1; ++b) {
    if (b <= nfull) load_block16(p + 64 * (uint64_t)b, w);
    if (b < nfull) {
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
    } else if (b == nfull) {
      uint32_t rr = r;
      asm volatile("" : "+v"(rr));
      build_tail(w, rr, len, w);
    } else {
      length_block(len, w);
    }
    compress(s, w);
  }
}

// Message sources of the split kernel. full<MODE>(i) hashes message i start to
// end (main workgroups); open(i, seg) locates message i for a segment wave (the
// first segment also runs the source's checks) and blocks() runs its blocks
// [b0, b1).
struct ArenaSrc {  // messages arena[off[m] : off[m]+len[m]] (k_digest_batch's form)
  static constexpr int kMinWaves = 8;  // occupancy hint (__launch_bounds__): <= 64 VGPRs
  // segment waves fetch their first block before the handoff wait (fits in the
  // 64 VGPRs: SGPR spills to VGPR lanes only)
  static constexpr bool kPreload = true;
  const uint8_t* arena;
  const uint64_t* off;
  const uint64_t* len;
  const uint32_t* order;    // lane i -> message m (may be null)
  const uint32_t* out_idx;  // lane i -> digest slot (may be null: slot m)
  uint32_t* err;
  struct Msg {
    const uint8_t* p;
    uint64_t len;
    uint8_t* slot;
    uint32_t nb;
    bool ok;
  };
  template <int MODE>
  __device__ __forceinline__ void full(uint64_t i, uint8_t* out) const {
    const uint64_t m = order ? (uint64_t)order[i] : i;
    const uint64_t o = out_idx ? (uint64_t)out_idx[i] : m;
    const uint8_t* p = arena + off[m];
    if (check_aligned(p, out + 32 * o, err)) hash_message<MODE>(p, len[m], out + 32 * o);
  }
  __device__ __forceinline__ Msg open(uint64_t i, uint32_t seg, uint8_t* out) const {
    Msg g;
    const uint64_t m = order ? (uint64_t)order[i] : i;
    const uint64_t o = out_idx ? (uint64_t)out_idx[i] : m;
    g.p = arena + off[m];
    g.len = len[m];
    g.slot = out + 32 * o;
    g.nb = (uint32_t)((g.len >> 6) + ((g.len & 63) < 56 ? 1 : 2));
    g.ok = seg == 0 ? check_aligned(g.p, g.slot, err) : (reinterpret_cast<uintptr_t>(g.p) & 15) == 0;
    return g;
  }
  // The finished words of block b (byte-swapped, or the padded tail / length block).
  __device__ __forceinline__ void preload(const Msg& g, uint32_t b, uint32_t (&w)[16]) const {
    const uint32_t nfull = (uint32_t)(g.len >> 6);
    if (b <= nfull) load_block16(g.p + 64 * (uint64_t)b, w);
    if (b < nfull) {
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
    } else if (b == nfull) {
      uint32_t rr = (uint32_t)(g.len & 63);
      asm volatile("" : "+v"(rr));
      build_tail(w, rr, g.len, w);
    } else {
      length_block(g.len, w);
    }
  }
  // Blocks [b0, b1); block b0's words w0 were preloaded (before the handoff wait).
  __device__ __forceinline__ void blocks(const Msg& g, State& st, uint32_t b0, uint32_t b1,
                                         const Beat& beat, uint32_t (&w0)[16]) const {
    compress(st, w0);
    for (uint32_t c = b0 + 1; c < b1; c += kBeatBlocks) {
      hash_blocks(st, g.p, g.len, c, std::min(c + kBeatBlocks, b1));
      beat(c);
    }
  }
};

// Batch / VerifyBatch digests over a table of 32-byte digests
// (k_digest_of_digests' form): block b < cnt/2 holds digests 2b and 2b+1.
__device__ __forceinline__ void dod_pair_words(const uint4* tab, uint32_t i0, uint32_t i1, uint32_t (&w)[16]) {
  const uint4* d0 = tab + 2 * (uint64_t)i0;
  const uint4* d1 = tab + 2 * (uint64_t)i1;
  uint4 v0 = d0[0], v1 = d0[1], v2 = d1[0], v3 = d1[1];
  w[0] = bswap(v0.x); w[1] = bswap(v0.y); w[2] = bswap(v0.z); w[3] = bswap(v0.w);
  w[4] = bswap(v1.x); w[5] = bswap(v1.y); w[6] = bswap(v1.z); w[7] = bswap(v1.w);
  w[8] = bswap(v2.x); w[9] = bswap(v2.y); w[10] = bswap(v2.z); w[11] = bswap(v2.w);
  w[12] = bswap(v3.x); w[13] = bswap(v3.y); w[14] = bswap(v3.z); w[15] = bswap(v3.w);
}
__device__ __forceinline__ void dod_pair_block(const uint4* tab, const uint32_t* idx, uint64_t k,
                                               uint32_t (&w)[16]) {
  dod_pair_words(tab, idx[k], idx[k + 1], w);
}
// The final block: the odd digest left (has_one: row i0), 0x80, zeros, the bit length.
__device__ __forceinline__ void dod_final_words(const uint4* tab, uint32_t i0, bool has_one, uint64_t cnt,
                                                uint32_t (&w)[16]) {
  if (has_one) {  // one digest left: 32 bytes + 0x80 + zeros + length fit one block
    const uint4* d0 = tab + 2 * (uint64_t)i0;
    uint4 v0 = d0[0], v1 = d0[1];
    w[0] = bswap(v0.x); w[1] = bswap(v0.y); w[2] = bswap(v0.z); w[3] = bswap(v0.w);
    w[4] = bswap(v1.x); w[5] = bswap(v1.y); w[6] = bswap(v1.z); w[7] = bswap(v1.w);
    w[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 14; ++j) w[j] = 0;
  } else {
    w[0] = 0x80000000u;
#pragma unroll
    for (int j = 1; j < 14; ++j) w[j] = 0;
  }
  const uint64_t bits = 256 * cnt;
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
}
__device__ __forceinline__ void dod_final_block(const uint4* tab, const uint32_t* idx, uint64_t k,
                                                uint64_t cnt, uint32_t (&w)[16]) {
  dod_final_words(tab, k < cnt ? idx[k] : 0u, k < cnt, cnt, w);
}

struct DigestSrc {
  // Occupancy hint: the paired digest loads hold a second block (16 VGPRs) while
  // the first is compressed, and full() has an LDS-staged and a direct index
  // path: ~95 VGPRs in the split kernel, so 5 waves per SIMD (the LDS staging
  // allows 6). That still hides the loads: the compression loop's issue rate is
  // flat from 2 to 8 waves, and Batch launches run ~3 per SIMD.
  static constexpr int kMinWaves = 5;
  // no early fetch: the held block costs this kernel 2 VGPR spills (c3dd 92.1 ->
  // 92.9-93.2 us, profiles/r03_ab_c3_preload/)
  static constexpr bool kPreload = false;
  const uint8_t* table;
  const uint32_t* idx;
  const uint64_t* begin;
  struct Msg {
    uint64_t k0, cnt;
    uint8_t* slot;
    uint32_t nb;
    bool ok;
  };
  // One Batch digest from its part indices, ix(k) = the k-th part's table row.
  template <class Ix>
  __device__ __forceinline__ void digest(const uint4* tab, Ix ix, uint64_t cnt, State& s) const {
    uint32_t w[16], nx[16];
    uint64_t k = 0;
    // Two blocks (four digests) per step, all requested before the first is
    // compressed: with a contiguous idx (the Batch shape) that is both halves
    // of a 128-byte line back to back, so the line is fetched from HBM once
    // instead of being evicted between two half-line requests a block apart
    // (1.57x the algorithmic bytes before, profiles/r01_pmc.json).
    for (; k + 4 <= cnt; k += 4) {
      dod_pair_words(tab, ix(k), ix(k + 1), w);
      dod_pair_words(tab, ix(k + 2), ix(k + 3), nx);
#pragma unroll
      for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(nx[j]));  // keep the second load here
      compress(s, w);
      compress(s, nx);
    }
    if (k + 2 <= cnt) {
      dod_pair_words(tab, ix(k), ix(k + 1), w);
      compress(s, w);
      k += 2;
    }
    // A wave-uniform even count (the Batch shape: BatchSize acks per batch) leaves a
    // final block of padding and length only, the same for every lane: its schedule
    // runs on the SALU (compress_uniform_pad), the VALU does only the rounds.
    const uint32_t c_lo = __builtin_amdgcn_readfirstlane((uint32_t)cnt);
    const uint32_t c_hi = __builtin_amdgcn_readfirstlane((uint32_t)(cnt >> 32));
    const uint64_t cnt0 = ((uint64_t)c_hi << 32) | c_lo;
    if (__ballot(cnt != cnt0) == 0 && !(c_lo & 1)) {
      const uint64_t bits = 256 * cnt0;
      compress_uniform_pad(s, 0x80000000u, (uint32_t)(bits >> 32), (uint32_t)bits);
    } else {
      dod_final_words(tab, k < cnt ? ix(k) : 0u, k < cnt, cnt, w);
      compress(s, w);
    }
  }
  // Part indices staged per wave in LDS: a wave's lanes are consecutive Batches,
  // so their index lists form one contiguous span of idx, copied once with
  // coalesced loads; each lane then reads its indices from LDS. Read straight
  // from idx, a wave's 64 index lists (80 B each for BatchSize 20) were fetched
  // from L2/MALL again at every step (c3dd 1.12x its algorithmic bytes). Spans
  // over kIdxStage / 64 indices per active lane read idx directly.
  static constexpr uint32_t kIdxStage = 1536;  // 6 KiB per wave, 24 KiB per workgroup
  template <int MODE>
  __device__ __forceinline__ void full(uint64_t i, uint8_t* out) const {
    __shared__ uint32_t sidx[4][kIdxStage];
    const uint64_t k0 = begin[i], k1 = begin[i + 1], cnt = k1 - k0;
    const uint4* tab = reinterpret_cast<const uint4*>(table);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the active lanes are a prefix of the wave (messages past n returned)
    const uint32_t act = (uint32_t)__popcll(__ballot(1));
    const uint64_t s0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(k0 >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)k0);
    const uint64_t s1 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(k1 >> 32), act - 1) << 32) |
                        __builtin_amdgcn_readlane((uint32_t)k1, act - 1);
    State s;
    state_init(s);
    constexpr int kPer = kIdxStage / 64;  // staged indices per lane
    if (s1 - s0 <= (uint64_t)kPer * act) {
      uint32_t* st = sidx[wv];
      const uint32_t span = (uint32_t)(s1 - s0);
      // all of a lane's share in flight at once (kPer loads; a dependent
      // load -> store per element would serialize ~20 HBM latencies before the
      // first block)
      uint32_t v[kPer];
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const uint32_t j = r * act + lane;
        v[r] = j < span ? idx[s0 + j] : 0u;
      }
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const uint32_t j = r * act + lane;
        if (j < span) st[j] = v[r];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t base = (uint32_t)(k0 - s0);
      digest(tab, [&](uint64_t k) { return st[base + (uint32_t)k]; }, cnt, s);
    } else {
      const uint32_t* ix = idx + k0;
      digest(tab, [&](uint64_t k) { return ix[k]; }, cnt, s);
    }
    store_digest(s, out + 32 * i);
  }
  __device__ __forceinline__ Msg open(uint64_t i, uint32_t, uint8_t* out) const {
    Msg g;
    g.k0 = begin[i];
    g.cnt = begin[i + 1] - g.k0;
    g.slot = out + 32 * i;
    g.nb = (uint32_t)(g.cnt / 2 + 1);
    g.ok = true;
    return g;
  }
  __device__ __forceinline__ void preload(const Msg& g, uint32_t b, uint32_t (&w)[16]) const {
    const uint4* tab = reinterpret_cast<const uint4*>(table);
    if (b < g.cnt / 2) dod_pair_block(tab, idx + g.k0, 2 * (uint64_t)b, w);
    else dod_final_block(tab, idx + g.k0, 2 * (uint64_t)b, g.cnt, w);
  }
  __device__ __forceinline__ void blocks(const Msg& g, State& st, uint32_t b0, uint32_t b1,
                                         const Beat& beat) const {
    uint32_t w[16];
    for (uint32_t b = b0; b < b1; ++b) {
      preload(g, b, w);
      compress(st, w);
      if (b % kBeatBlocks == 0) beat(b);  // spill-free here (53 VGPRs)
    }
  }
};

template <int MODE, class Src>
__global__ __launch_bounds__(256, Src::kMinWaves) void k_digest_split(Src src, uint64_t n, uint8_t* __restrict__ out,
                                                      uint32_t* __restrict__ err, SplitPlan sp) {
  const uint32_t seg_wgs = sp.segments * sp.groups;
  if (blockIdx.x >= seg_wgs) {  // main workgroups: one lane per message, [0, n_main)
    const uint64_t i = (uint64_t)(blockIdx.x - seg_wgs) * blockDim.x + threadIdx.x;
    if (i < sp.n_main) src.template full<MODE>(i, out);
    return;
  }
  const uint32_t seg = blockIdx.x / sp.groups;
  const uint32_t chain = (blockIdx.x % sp.groups) * 4 + threadIdx.x / 64;
  if (chain >= sp.chains) return;  // whole wave
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = threadIdx.x & 63;
  uint64_t* flag = sp.flags + chain;
  const uint64_t ep = split_word(sp.epoch, 0, 0);
  // Everything that does not depend on the previous segment is fetched before
  // waiting for it: the message's metadata and this segment's first block (into
  // registers: the acquire below invalidates the caches), so the handoff costs
  // the flag and the 32-byte state, not a payload round trip as well.
  const uint64_t i = sp.n_main + (uint64_t)chain * 64 + lane;
  typename Src::Msg g{};
  uint32_t b0 = 0, b1 = 0;
  uint32_t w0[Src::kPreload ? 16 : 1];
  const bool mine = i < n;
  if (mine) {
    g = src.open(i, seg, out);
    if (g.ok) {
      b0 = (uint32_t)((uint64_t)g.nb * seg / sp.segments);
      b1 = (uint32_t)((uint64_t)g.nb * (seg + 1) / sp.segments);
      if constexpr (Src::kPreload) {
        if (b0 < b1) src.preload(g, b0, w0);
      }
    }
  }
  if (seg > 0) {  // wait until seg segments of this chain are done (same launch: same epoch)
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t prev = t0;
    uint64_t seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((seen >> 40) != (ep >> 40) || ((seen >> 32) & 0xFF) < seg) {
      __builtin_amdgcn_s_sleep(8);
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      const uint64_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v != seen || now - prev > kSplitDeschedTicks) {
        // the chain moved (a beat or a handoff), or this wave was descheduled
        // (and the running segment with it): restart the clock
        seen = v;
        t0 = now;
      } else if (now - t0 > kSplitWaitTicks) {
        if (lane == 0) {
          atomicOr(err, 2u);
          __hip_atomic_store(flag, split_word(sp.epoch, seg + 1, 0), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
      }
      prev = now;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  const Beat beat{flag, split_word(sp.epoch, seg, 0)};
  if (mine && g.ok) {
    State st;
    if (seg == 0) {
      state_init(st);
    } else {  // the previous segment's state, parked in this message's digest slot
      const uint4 lo = reinterpret_cast<const uint4*>(g.slot)[0];
      const uint4 hi = reinterpret_cast<const uint4*>(g.slot)[1];
      st.h[0] = lo.x; st.h[1] = lo.y; st.h[2] = lo.z; st.h[3] = lo.w;
      st.h[4] = hi.x; st.h[5] = hi.y; st.h[6] = hi.z; st.h[7] = hi.w;
    }
    if (b0 < b1) {  // (a segment may have no block)
      if constexpr (Src::kPreload) src.blocks(g, st, b0, b1, beat, w0);
      else src.blocks(g, st, b0, b1, beat);
    }
    if (seg + 1 == sp.segments) {
      store_digest(st, g.slot);
    } else {  // raw state words, resumed by the next segment: written through (sc1)
      uint64_t* q = reinterpret_cast<uint64_t*>(g.slot);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __hip_atomic_store(q + j, ((uint64_t)st.h[2 * j + 1] << 32) | st.h[2 * j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // Hand-off (cdna_hip_programming.md Guideline 16, R1): the state went out
  // write-through (sc1), so no release fence (buffer_wbl2 sc1 would write back
  // the XCD L2's every dirty line -- the main waves' digests among them -- at
  // 1.7-6.5 us per hand-off); this wave drains its stores, then one lane stores
  // the flag. The next segment polls it relaxed and takes ONE agent acquire.
  if (seg + 1 < sp.segments && !(seg == 0 && chain == sp.stall_chain)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(flag, split_word(sp.epoch, seg + 1, 0), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// Cooperative chaining (few, large messages). A message's 64 rounds per block
// are a serial chain, but its message schedule is not part of that chain: it
// depends only on the block's bytes. A workgroup of two waves serves 64
// messages: wave 1 (producer) lane l loads block b+1 of message l, expands its
// schedule and writes K[t]+W[t] for t = 0..63 into an LDS slot, while wave 0
// (consumer) lane l runs the 64 rounds of block b from the other slot. The
// chain then costs 14 VALU instructions per round plus 16 ds_read_b128 per
// block instead of 1,400 instructions per block: ~1.5x lower latency per
// message, for batches too small to fill the chip with one lane per message.
// ---------------------------------------------------------------------------
// kw slot layout: [quad t/4][lane] x 16 B (K[t..t+3] + W[t..t+3]); every
// ds_write_b128 / ds_read_b128 of a wave covers 1 KiB contiguously.
constexpr int kCoopSlotQuads = 16;

#define MSHA_CROUND(a, b, c, d, e, f, g, h, kw)          \
  {                                                       \
    uint32_t t1 = h + (kw) + Sig1(e) + ch(e, f, g);       \
    d += t1;                                              \
    h = t1 + Sig0(a) + maj(a, b, c);                      \
  }
#define MSHA_C8(q)                                                     \
  {                                                                    \
    const uint4 v0 = kv[q], v1 = kv[(q) + 1];                          \
    nxt[q] = nslot[(q) * 64];                                          \
    nxt[(q) + 1] = nslot[((q) + 1) * 64];                              \
    MSHA_CROUND(a, b, c, d, e, f, g, h, v0.x)                          \
    MSHA_CROUND(h, a, b, c, d, e, f, g, v0.y)                          \
    MSHA_CROUND(g, h, a, b, c, d, e, f, v0.z)                          \
    MSHA_CROUND(f, g, h, a, b, c, d, e, v0.w)                          \
    MSHA_CROUND(e, f, g, h, a, b, c, d, v1.x)                          \
    MSHA_CROUND(d, e, f, g, h, a, b, c, v1.y)                          \
    MSHA_CROUND(c, d, e, f, g, h, a, b, v1.z)                          \
    MSHA_CROUND(b, c, d, e, f, g, h, a, v1.w)                          \
  }

// Consumer: the 64 rounds of one block from its K+W quads kv (read from LDS
// during the previous block), reading the next block's quads from nslot (the
// lane's column of the other slot) into nxt meanwhile, so no block waits for
// an LDS round trip (k_digest_coop alternates the two register sets).
__device__ __forceinline__ void compress_kw(State& s, const uint4 (&kv)[16], uint4 (&nxt)[16],
                                            const uint4* __restrict__ nslot) {
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
  MSHA_C8(0) MSHA_C8(2) MSHA_C8(4) MSHA_C8(6) MSHA_C8(8) MSHA_C8(10) MSHA_C8(12) MSHA_C8(14)
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}
#undef MSHA_C8
#undef MSHA_CROUND

// Producer: expand block words w into K[t]+W[t], t = 0..63, written to the slot.
__device__ __forceinline__ void schedule_kw(uint32_t (&w)[16], uint4* __restrict__ slot) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 4 * q + j;
      if (t >= 16) MSHA_SCHED(w, t);
      x[j] = w[t & 15] + K[t];
    }
    slot[q * 64] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}

// k_digest_chain2's packing (its consumers alternate E- and A-rounds): quad 2g
// holds the K+W words of rounds 8g, 8g+2, 8g+4, 8g+6 (the e-lanes'), quad 2g+1
// those of rounds 8g+1, ..., 8g+7 (the a-lanes').
__device__ __forceinline__ void schedule_kw_eo(uint32_t (&w)[16], uint4* __restrict__ slot) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = 8 * g + j;
      if (t >= 16) MSHA_SCHED(w, t);
      x[j] = w[t & 15] + K[t];
    }
    slot[(2 * g) * 64] = make_uint4(x[0], x[2], x[4], x[6]);
    slot[(2 * g + 1) * 64] = make_uint4(x[1], x[3], x[5], x[7]);
  }
}

// Workgroup = 4 waves serving 128 messages: waves 0/1 consume (rounds) for
// message groups 0/1, waves 2/3 produce (schedules) for the same groups. A
// workgroup's waves take SIMDs in the cyclic order 0->2->1->3, so each wave
// gets a SIMD of its own; the launch reserves enough LDS (kCoopLdsBytes) that
// a CU holds ONE such workgroup, so a consumer never shares its SIMD with
// another consumer (that would forfeit the latency gain).
constexpr size_t kCoopDynLds = 40 * 1024;  // + 64 KiB static = 104 KiB > 160/2 KiB

// EXCL (a planned launch's head): the waves claim every register of their SIMD
// (an empty asm clobbering v255 and a255: 512 per lane), so a CU running a
// head workgroup holds nothing else -- lane-kernel waves beside it would
// either stall the chain (their older waves win issue) or, with the head at
// top priority, be starved themselves for the whole chain (c5 over 4 GPUs:
// 5.0 -> 6.4 ms). The head's CUs run the head; the lane kernel has the rest.
template <int MODE, bool EXCL = false>
__global__ __launch_bounds__(256) void k_digest_coop(const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ off,
                                                     const uint64_t* __restrict__ len,
                                                     const uint32_t* __restrict__ order,
                                                     const uint32_t* __restrict__ out_idx,
                                                     uint64_t n, uint8_t* __restrict__ out,
                                                     uint32_t* __restrict__ err,
                                                     const uint32_t* __restrict__ limit) {
  __shared__ uint4 kw[2][2][kCoopSlotQuads * 64];  // [slot][group][quad][lane]: 64 KiB
  __shared__ uint32_t s_nb;
  const unsigned lane = threadIdx.x & 63;
  const unsigned wave = threadIdx.x >> 6;
  const bool producer = wave >= 2;
  const unsigned group = wave & 1;
  const uint64_t i = (uint64_t)blockIdx.x * kCoopMsgsPerWg + group * 64 + lane;
  // limit: a planned launch's head of long chains ends at *limit (device-side).
  // That launch runs beside the lane kernel, whose older waves would win issue
  // arbitration on the SIMDs it shares with them (a chain then crawls at a
  // fraction of its rate): the head's waves take the highest issue priority.
  if (EXCL) asm volatile("" ::: "v255", "a255");
  if (limit) __builtin_amdgcn_s_setprio(3);
  bool active = i < n && (!limit || i < *limit);
  uint64_t m = i;  // metadata index
  if (active && order) {
    const uint32_t v = order[i];
    active = v != kNoLane;
    m = active ? v : 0;
  }
  if (!active) m = 0;
  const uint64_t o = active ? (out_idx ? (uint64_t)out_idx[i] : m) : 0;  // digest slot
  const uint8_t* p = arena;
  uint64_t L = 0;
  if (active) {
    p = arena + off[m];
    L = len[m];
    if (reinterpret_cast<uintptr_t>(p) & 15) {  // flagged and zeroed by the consumer only
      active = false;
      L = 0;
      if (!producer) check_aligned(p, out + 32 * o, err);
    }
  }
  const uint32_t nfull = (uint32_t)(L >> 6), r = (uint32_t)(L & 63);
  const uint32_t nb = nfull + (r < 56 ? 1 : 2);
  if (threadIdx.x == 0) s_nb = 0;
  __syncthreads();
  if (!producer && active) atomicMax(&s_nb, nb);
  __syncthreads();
  const uint32_t NB = s_nb;  // blocks of the workgroup's longest message
  // One barrier per block in every wave: after barrier k the producers have
  // filled slot k&1 and the consumers are done with slot (k-1)&1.
  if (producer) {
    uint32_t raw[16], w[16];
    if (active) load_block16<MODE>(p, raw);
    for (uint32_t b = 0; b < NB; ++b) {
      if (b < nfull) {
        to_words(raw, w);
      } else if (b == nfull) {
        uint32_t rr = r;
        asm volatile("" : "+v"(rr));
        build_tail(raw, rr, L, w);
      } else {
        length_block(L, w);
      }
      if (active && b + 1 <= nfull) load_block16<MODE>(p + 64 * (uint64_t)(b + 1), raw);  // prefetch
      schedule_kw(w, &kw[b & 1][group][lane]);
      __syncthreads();  // barrier b: slot b & 1 holds block b
    }
    __syncthreads();  // barrier NB: the consumers' last (they wait one block ahead)
  } else {
    // As in k_digest_chain2: block b's K+W is read during block b-1 (barrier
    // b+1 opens block b once slot (b+1) & 1 is written; the producer refills
    // the slot block b-1 read, complete at barrier b+1), two register sets
    // alternating by unrolling the block loop twice.
    State s;
    state_init(s);
    uint4 ka[16], kb[16];
    __syncthreads();  // barrier 0
#pragma unroll
    for (int q = 0; q < 16; ++q) ka[q] = kw[0][group][q * 64 + lane];
    for (uint32_t b = 0; b < NB; ++b) {
      __syncthreads();  // barrier b+1
      compress_kw(s, ka, kb, &kw[(b + 1) & 1][group][lane]);  // a read past the last block is unused
      if (active && b + 1 == nb) store_digest(s, out + 32 * o);
      if (++b == NB) break;
      __syncthreads();  // barrier b+1
      compress_kw(s, kb, ka, &kw[(b + 1) & 1][group][lane]);
      if (active && b + 1 == nb) store_digest(s, out + 32 * o);
    }
  }
}

// ---------------------------------------------------------------------------
// The planned launch's head of long chains (msha_digest_batch_device_planned):
// what bounds it is one chain's latency, and the cooperative consumer is
// issue-bound at 14 VALU instructions a round. Here TWO lanes carry a message:
// lane p < 8 of each 16-lane row the e-side (e f g h), lane 15 - p the a-side
// (a b c d). One v_alignbit x3 + xor3 then computes Sigma1 in the e-lane and
// Sigma0 in the a-lane (per-lane rotate amounts), Ch and Maj are one bitop3
// each, and the two new words come from two row_mirror DPP adds that write only
// their side's lanes (bank_mask) -- 11 instructions a round (below):
//   e' = mirror(d) + T1,   a' = mirror(T1) + T2
// Register-resident, one wave alone on its SIMD: 21.1 against 23.7 ns a round
// (tools/chain_dpp_microbench.hip, profiles/r03_chain_dpp/). Workgroup = one
// producer wave (64 messages: loads, padding, K+W schedules into LDS, as in
// k_digest_coop) and two consumer waves of 32 messages; EXCL as above (the
// head's CUs hold nothing else); each lane stores its side's four digest words.
// The rounds are inline asm (MSHA_DQ below): a DPP read of a VGPR needs 2 wait
// states after the VALU write of it, and the compiler's hazard recognizer does
// not look inside asm text, so the asm orders its own instructions to satisfy
// that, and tools/check_dpp_hazards.py checks every DPP of the built library.
// ---------------------------------------------------------------------------
// The rounds in asm (X Y Z W: this lane's side, newest to oldest; the new word
// replaces W). Both lanes of a message run the same instruction stream; what a
// lane computes that its side does not need is simply not used.
//  E-round (11 instructions; K is read in the e-lanes only):
//    s = Sigma (3 v_alignbit + xor3; Sigma1 in the e-lanes, Sigma0 in the
//    a-lanes), c = Ch, m = Maj (one bitop3 each), u = s + W + c, T1 = u + K
//    (the e-lanes' W is h), t = s + m (T2 in the a-lanes), then two row_mirror
//    DPP adds that write only their side's lanes (bank_mask):
//    e' = mirror(d) + T1, a' = mirror(T1) + t.
//  A-round (11 instructions; K is read in the a-lanes only): y = W + K (d + K
//    in the a-lanes), s, c, m, u = s + W + c (Sigma1 + h + Ch in the e-lanes),
//    t = s + K + m (Sigma0 + K + Maj in the a-lanes), then e' = mirror(y) + u
//    and a' = mirror(u) + t -- the same two sums, K carried on the other side.
// Rounds alternate E, A, E, A, ..., so each lane needs the K+W words of every
// OTHER round: the producer packs rounds 8g, 8g+2, 8g+4, 8g+6 into the e-lanes'
// quad and 8g+1, ..., 8g+7 into the a-lanes', and a consumer lane reads ONE
// ds_read_b128 per 8 rounds (MSHA_CHAIN2_FORM 4). Round 3's consumer ran
// E-rounds only, the a-lanes reading 16 zero quads a block to get K = 0: 16
// reads a block instead of 8 (MSHA_CHAIN2_FORM 3, kept for the A/B). On a lone
// wave a ds_read_b128 costs ~14 shader cycles of issue (one VALU slot plus its
// 1 KiB return), 3.6 cycles a round at one per 4 rounds
// (tools/round_issue_microbench.hip, profiles/r04_chain2_forms/). Named
// operands: sh1-3 the lane's rotate amounts, K the round's K+W word, the rest
// scratch.
#ifndef MSHA_CHAIN2_FORM
#define MSHA_CHAIN2_FORM 4
#endif
#ifndef MSHA_CHAIN2_PAIR
#define MSHA_CHAIN2_PAIR 1
#endif
constexpr uint32_t kC2Per = MSHA_CHAIN2_PAIR ? 2 : 1;  // LDS slots' blocks (the most per barrier)
// A workgroup pairs blocks per barrier only when its longest message has at
// least this many: pairing delays the consumers' first block by two producer
// blocks, which a short chain pays in full (1,024 x 640 B: 22.3 -> 25.5 us)
// while a long one gains (256 x 64 KiB: 1.420 -> 1.405 ms; tools/ab_lib.sh).
constexpr uint32_t kC2PairMinBlocks = 64;
#define MSHA_ASM_SIGMA(X)                                                                        \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                                       \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"                                       \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"                                       \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"
#define MSHA_ASM_CHMAJ(X, Y, Z)                                                                  \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                           \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"
// E-round. The second DPP reads T1 (sk) two instructions after writing it (t and
// the first DPP between): the 2 wait states a DPP source needs after a VALU
// write; the first reads W, written four rounds earlier.
#define MSHA_ASM_EROUND(X, Y, Z, W, K)                                                           \
  MSHA_ASM_SIGMA(X) MSHA_ASM_CHMAJ(X, Y, Z)                                                      \
  "v_add3_u32 %[u], %[s], %[" #W "], %[c]\n\t"                                                    \
  "v_add_u32 %[sk], %[u], %[" #K "]\n\t"                                                          \
  "v_add_u32 %[t], %[s], %[m]\n\t"                                                                \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[sk] row_mirror row_mask:0xf bank_mask:0x3\n\t"          \
  "v_add_u32_dpp %[" #W "], %[sk], %[t] row_mirror row_mask:0xf bank_mask:0xc\n\t"
// A-round: y is written first, nine instructions before the DPP that reads it;
// the second DPP reads u two instructions after writing it.
#define MSHA_ASM_AROUND(X, Y, Z, W, K)                                                           \
  "v_add_u32 %[y], %[" #W "], %[" #K "]\n\t"                                                      \
  MSHA_ASM_SIGMA(X) MSHA_ASM_CHMAJ(X, Y, Z)                                                      \
  "v_add3_u32 %[u], %[s], %[" #W "], %[c]\n\t"                                                    \
  "v_add3_u32 %[t], %[s], %[" #K "], %[m]\n\t"                                                    \
  "v_add_u32_dpp %[" #W "], %[y], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t"                \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_mirror row_mask:0xf bank_mask:0xc\n\t"
// Round 3's round (form 3): sk = Sigma + K (K 0 in the a-lanes), u = sk + W + Ch,
// t = sk + Maj; the second DPP reads u three instructions after writing it.
#define MSHA_ASM_ROUND3(X, Y, Z, W, K)                                                           \
  MSHA_ASM_SIGMA(X)                                                                              \
  "v_add_u32 %[sk], %[s], %[" #K "]\n\t"                                                          \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                           \
  "v_add3_u32 %[u], %[sk], %[" #W "], %[c]\n\t"                                                   \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"                           \
  "v_add_u32 %[t], %[sk], %[m]\n\t"                                                               \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t"           \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_mirror row_mask:0xf bank_mask:0xc\n\t"
#define MSHA_ASM_OPERANDS                                                                        \
  : [X] "+v"(X), [Y] "+v"(Y), [Z] "+v"(Z), [W] "+v"(W), [s1] "=&v"(s1_), [s2] "=&v"(s2_),      \
    [s3] "=&v"(s3_), [s] "=&v"(s_), [sk] "=&v"(sk_), [c] "=&v"(c_), [u] "=&v"(u_), [m] "=&v"(m_), \
    [t] "=&v"(t_), [y] "=&v"(y_)                                                                 \
  : [sh1] "v"(sh1), [sh2] "v"(sh2), [sh3] "v"(sh3), [k0] "v"(v_.x), [k1] "v"(v_.y),              \
    [k2] "v"(v_.z), [k3] "v"(v_.w)
// One K+W quad of cur: 8 rounds (form 4) or 4 (form 3) in ONE asm statement --
// a lone wave issues one instruction per ~4.1-4.6 cycles whatever it is, and
// the compiler puts an s_nop after every asm statement whose output the next
// VALU instruction reads (it cannot see whether the asm ended in a
// dst-forwarding instruction): a statement per round cost 2 s_nops a round
// (+16 % a block; tools/chain2_anatomy.hip). The same quad of the NEXT block is
// read from LDS slot nxt meanwhile, so its latency hides under the rounds.
// tools/check_dpp_hazards.py checks every DPP of the built library.
#if MSHA_CHAIN2_FORM == 4
constexpr int kC2Quads = 8;  // K+W quads a consumer lane reads per block
#define MSHA_DQ(cur, nxt, q)                                                                     \
  {                                                                                              \
    const uint4 v_ = cur[q];                                                                     \
    nxt[q] = nk[col + (q) * qstride];                                                            \
    uint32_t s1_, s2_, s3_, s_, sk_, c_, u_, m_, t_, y_;                                         \
    asm volatile(MSHA_ASM_EROUND(X, Y, Z, W, k0) MSHA_ASM_AROUND(W, X, Y, Z, k0)                 \
                 MSHA_ASM_EROUND(Z, W, X, Y, k1) MSHA_ASM_AROUND(Y, Z, W, X, k1)                 \
                 MSHA_ASM_EROUND(X, Y, Z, W, k2) MSHA_ASM_AROUND(W, X, Y, Z, k2)                 \
                 MSHA_ASM_EROUND(Z, W, X, Y, k3) MSHA_ASM_AROUND(Y, Z, W, X, k3)                 \
                 MSHA_ASM_OPERANDS);                                                             \
  }
#else
constexpr int kC2Quads = 16;
#define MSHA_DQ(cur, nxt, q)                                                                     \
  {                                                                                              \
    const uint4 v_ = cur[q];                                                                     \
    nxt[q] = nk[col + (q) * qstride];                                                            \
    uint32_t s1_, s2_, s3_, s_, sk_, c_, u_, m_, t_, y_;                                         \
    asm volatile(MSHA_ASM_ROUND3(X, Y, Z, W, k0) MSHA_ASM_ROUND3(W, X, Y, Z, k1)                 \
                 MSHA_ASM_ROUND3(Z, W, X, Y, k2) MSHA_ASM_ROUND3(Y, Z, W, X, k3)                 \
                 MSHA_ASM_OPERANDS);                                                             \
    (void)y_;                                                                                    \
  }
#endif
// One block b from cur (read during the previous block), reading block b+1's
// K+W (its LDS slot nk) into nxt; the digest is stored after the message's last block.
#define MSHA_DBLOCK(cur, nxt)                                                                    \
  {                                                                                              \
    uint32_t X = H0, Y = H1, Z = H2, W = H3;                                                     \
    _Pragma("unroll") for (int q_ = 0; q_ < kC2Quads; ++q_) MSHA_DQ(cur, nxt, q_)                \
    H0 += X; H1 += Y; H2 += Z; H3 += W;                                                          \
    if (active && b + 1 == nb)                                                                   \
      *reinterpret_cast<uint4*>(out + 32 * o + (eside ? 16 : 0)) =                               \
          make_uint4(bswap(H0), bswap(H1), bswap(H2), bswap(H3));                                \
  }

// Diagnostic build only (tools/chain2_anatomy.hip defines MSHA_CHAIN2_STAMPS):
// lane 0 of each wave of workgroup 0 stamps s_memtime before and after every
// barrier, stamps[wave * 4096 + 2 j (+1)] for barrier j. The product build has
// no stamps.
#ifdef MSHA_CHAIN2_STAMPS
__device__ uint64_t* g_chain2_stamps;
#define MSHA_C2_BARRIER(j)                                                                      \
  {                                                                                             \
    const uint64_t j_ = (j);                                                                    \
    if (blockIdx.x == 0 && lane == 0 && j_ < 2047)                                              \
      g_chain2_stamps[wave * 4096 + 2 * j_] = __builtin_amdgcn_s_memtime();                     \
    __syncthreads();                                                                            \
    if (blockIdx.x == 0 && lane == 0 && j_ < 2047)                                              \
      g_chain2_stamps[wave * 4096 + 2 * j_ + 1] = __builtin_amdgcn_s_memtime();                 \
  }
#else
#define MSHA_C2_BARRIER(j) __syncthreads();
#endif

// Also AUTO's kernel for launches of at most 64 messages per CU (a call of a
// few actions at low load: one chain's latency is the call's), where every
// workgroup gets a CU of its own: EXCL false there. order, out_idx and limit
// may be null (identity, slot = message, no device-side limit).
template <int MODE, bool EXCL>
__device__ __forceinline__ void chain2_body(const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ out_idx,
                                                       uint64_t n, uint8_t* __restrict__ out,
                                                       uint32_t* __restrict__ err,
                                                       const uint32_t* __restrict__ limit) {
  // [slot][quad t/4][message] x 16 B, then (form 3 only) 16 zero quads, the
  // a-lanes' K+W. 2 x 2 x 16 KiB = 64 KiB with pairing: two workgroups a CU at
  // most (a head launch, EXCL, runs one a CU anyway).
  __shared__ uint4 kw[2][kC2Per][kCoopSlotQuads * 64 + (MSHA_CHAIN2_FORM == 3 ? kCoopSlotQuads : 0)];
  __shared__ uint32_t s_nb;
  if (EXCL) asm volatile("" ::: "v255", "a255");  // exclusive CU (see k_digest_coop EXCL)
  if (EXCL) __builtin_amdgcn_s_setprio(3);
  const unsigned lane = threadIdx.x & 63;
  const unsigned wave = threadIdx.x >> 6;
  const bool producer = wave == 0;
  const unsigned p = lane & 15;
  const bool eside = p < 8;
  // message of this lane inside the workgroup
  const unsigned msg = producer ? lane : (wave - 1) * 32 + (lane >> 4) * 8 + (eside ? p : 15 - p);
  const uint64_t i = (uint64_t)blockIdx.x * kChain2MsgsPerWg + msg;
  bool active = i < n && (!limit || i < *limit);
  uint64_t m = i;  // metadata index
  if (active && order) {
    const uint32_t v = order[i];
    active = v != kNoLane;
    m = v;
  }
  uint64_t o = m;  // digest slot
  if (active && out_idx) o = out_idx[i];
  if (!active) m = o = 0;
  const uint8_t* pa = arena;
  uint64_t L = 0;
  if (active) {
    pa = arena + off[m];
    L = len[m];
    if (reinterpret_cast<uintptr_t>(pa) & 15) {
      active = false;
      L = 0;
      if (!producer && eside) check_aligned(pa, out + 32 * o, err);
    }
  }
  const uint32_t nfull = (uint32_t)(L >> 6), r = (uint32_t)(L & 63);
  const uint32_t nb = nfull + (r < 56 ? 1 : 2);
  if (threadIdx.x == 0) s_nb = 0;
#if MSHA_CHAIN2_FORM == 3
  if (threadIdx.x < 2 * kC2Per * kCoopSlotQuads)  // form 3: the a-lanes' zero quads
    kw[threadIdx.x / (kC2Per * 16)][(threadIdx.x >> 4) % kC2Per][kCoopSlotQuads * 64 + (threadIdx.x & 15)] =
        make_uint4(0, 0, 0, 0);
#endif
  __syncthreads();
  if (producer && active) atomicMax(&s_nb, nb);
  __syncthreads();
  const uint32_t NB = s_nb;
  const uint32_t per = kC2Per == 2 && NB >= kC2PairMinBlocks ? 2u : 1u;  // blocks per barrier
  if (producer) {
    uint32_t raw[16], w[16];
    if (active) load_block16<MODE>(pa, raw);
    for (uint32_t b = 0; b < NB; ++b) {
      if (b < nfull) {
        to_words(raw, w);
      } else if (b == nfull) {
        uint32_t rr = r;
        asm volatile("" : "+v"(rr));
        build_tail(raw, rr, L, w);
      } else {
        length_block(L, w);
      }
      if (active && b + 1 <= nfull) load_block16<MODE>(pa + 64 * (uint64_t)(b + 1), raw);
      uint4* slot = &kw[(b / per) & 1][b % per][lane];
      if (MSHA_CHAIN2_FORM == 4)
        schedule_kw_eo(w, slot);
      else
        schedule_kw(w, slot);
      // barrier g: slot g & 1 holds group g (per blocks)
      if (b % per == per - 1 || b + 1 == NB) MSHA_C2_BARRIER(b / per)
    }
    MSHA_C2_BARRIER((NB + per - 1) / per)  // the consumers' last (they wait one group ahead)
  } else {
    // e-side: e f g h, rotates 6 11 25; a-side: a b c d, rotates 2 13 22
    uint32_t H0 = eside ? 0x510e527fu : 0x6a09e667u, H1 = eside ? 0x9b05688cu : 0xbb67ae85u;
    uint32_t H2 = eside ? 0x1f83d9abu : 0x3c6ef372u, H3 = eside ? 0x5be0cd19u : 0xa54ff53au;
    const uint32_t sh1 = eside ? 6 : 2, sh2 = eside ? 11 : 13, sh3 = eside ? 25 : 22;
#if MSHA_CHAIN2_FORM == 4
    // quad 2g: the e-lanes' K+W of rounds 8g, 8g+2, 8g+4, 8g+6; 2g+1: the a-lanes'
    const unsigned col = (eside ? 0 : 64) + msg, qstride = 128;
#else
    const unsigned col = eside ? msg : kCoopSlotQuads * 64;  // a-lanes read the zero quads
    const unsigned qstride = eside ? 64 : 1;
#endif
    // Block b's K+W is read from LDS during block b-1's rounds (MSHA_DQ), so a
    // block starts on registers: barrier b+1 (the producer has written slot
    // (b+1) & 1) opens block b, whose rounds read it. The producer fills slot
    // b+2 -- the one block b-1 read, complete at barrier b+1 (__syncthreads
    // waits for every outstanding LDS read) -- while block b computes. Two
    // register sets alternate by unrolling the block loop twice, so nothing is
    // copied between blocks.
    // MSHA_CHAIN2_PAIR: a barrier per PAIR of blocks -- the producer schedules
    // two blocks into a slot, the consumers hold four register sets (the pair
    // they compute, the pair they read) -- halving the barriers a chain pays.
#if MSHA_CHAIN2_PAIR
    if (per == 2) {
    uint4 ka[kC2Quads], kb[kC2Quads], kc[kC2Quads], kd[kC2Quads];
    MSHA_C2_BARRIER(0)  // barrier 0: slot 0 holds blocks 0 and 1
#pragma unroll
    for (int q = 0; q < kC2Quads; ++q) {
      ka[q] = kw[0][0][col + q * qstride];
      kb[q] = kw[0][1][col + q * qstride];
    }
    const uint32_t NP = (NB + 1) / 2;
    for (uint32_t g = 0; g < NP; ++g) {
      MSHA_C2_BARRIER(g + 1)  // reads past the last block are harmless (unused)
      {
        const uint32_t b = 2 * g;
        const uint4* nk = kw[(g + 1) & 1][0];
        MSHA_DBLOCK(ka, kc)
      }
      {
        const uint32_t b = 2 * g + 1;
        const uint4* nk = kw[(g + 1) & 1][1];
        MSHA_DBLOCK(kb, kd)
      }
      if (++g == NP) break;
      MSHA_C2_BARRIER(g + 1)
      {
        const uint32_t b = 2 * g;
        const uint4* nk = kw[(g + 1) & 1][0];
        MSHA_DBLOCK(kc, ka)
      }
      {
        const uint32_t b = 2 * g + 1;
        const uint4* nk = kw[(g + 1) & 1][1];
        MSHA_DBLOCK(kd, kb)
      }
    }
    return;
    }
#endif
    uint4 ka[kC2Quads], kb[kC2Quads];
    MSHA_C2_BARRIER(0)  // barrier 0: slot 0 holds block 0
#pragma unroll
    for (int q = 0; q < kC2Quads; ++q) ka[q] = kw[0][0][col + q * qstride];
    for (uint32_t b = 0; b < NB; ++b) {
      MSHA_C2_BARRIER(b + 1)
      const uint4* nk = kw[(b + 1) & 1][0];  // a read past the last block is harmless (unused)
      MSHA_DBLOCK(ka, kb)
      if (++b == NB) break;
      MSHA_C2_BARRIER(b + 1)
      nk = kw[(b + 1) & 1][0];
      MSHA_DBLOCK(kb, ka)
    }
  }
}

template <int MODE, bool EXCL>
__global__ __launch_bounds__(192) void k_digest_chain2(const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ out_idx,
                                                       uint64_t n, uint8_t* __restrict__ out,
                                                       uint32_t* __restrict__ err,
                                                       const uint32_t* __restrict__ limit) {
  MSHA_WAVE_STAMP_OPEN()
  chain2_body<MODE, EXCL>(arena, off, len, order, out_idx, n, out, err, limit);
  MSHA_WAVE_STAMP_CLOSE(kStampChain2)
}

// ---------------------------------------------------------------------------
// Eight lanes a message (round 5; VERDICT r4 #3: the chain that bounds c5 over 8
// GPUs). The two-lane round spends 3 of its 11 instructions on the three
// rotations of Sigma, one after another in each lane. Here a message is two
// quads -- the e-side (e f g h) in lanes 0-3 and the a-side (a b c d) in lanes
// 4-7 of its 8 -- and each lane makes ONE rotation of its side's word (e: 6,
// 11, 25, 6; a: 2, 13, 22, 2), the quad's three then XORed by two quad_perm
// DPP xors that leave Sigma in all four lanes; Ch and Maj one bitop3 each; the
// two new words by two DPP adds across the quads (row_ror:12 reads the a-quad
// four lanes up, row_ror:4 the e-quad four down; bank_mask writes one side).
// 10 instructions a round, 4 of them DPP: 41.4 shader cycles a round on a lone
// wave against 45.4 for the two-lane round (tools/round_issue_microbench.hip
// oct10, profiles/r05_chain/). Every lane of a quad holds its side's whole
// state, so nothing is broadcast.
//  E-round: s1 = rot, c = Ch, m = Maj, s2 = s1 ^ qp[1,0,3,1](s1), sk = W + K
//    (h + K+W in the e-quad), s = s2 ^ qp[2,2,1,2](s1), u = s + c + sk (T1),
//    t = s + m (T2 in the a-quad), e' = ror12(W) + u (d from the a-quad),
//    a' = ror4(u) + t (T1 from the e-quad).
//  A-round: y = W + K first (d + K+W in the a-quad), ..., u = s + c + W
//    (Sigma1 + Ch + h), t = s + m + K (T2 + K+W), e' = ror12(y) + u, a' = ror4(u) + t.
// K+W exactly as the two-lane kernel's form 4 (the e-quad reads the even
// rounds' quad, the a-quad the odd rounds'): the same producer, one
// ds_read_b128 per lane per 8 rounds. DPP sources read here are written >= 2
// instructions earlier (tools/check_dpp_hazards.py checks the built library).
// A consumer wave is 8 messages and each wave owns a SIMD: two producers (even
// and odd blocks) and two consumer waves a workgroup, 16 messages a CU (the
// two-lane kernel: 64) -- a latency kernel for the few long payloads of a
// folded head.
constexpr unsigned kC8Producers = 2;
// ---------------------------------------------------------------------------
#define MSHA_ASM_E8(X, Y, Z, W, K)                                                               \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh]\n\t"                                        \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                           \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"                           \
  "v_xor_b32_dpp %[s2], %[s1], %[s1] quad_perm:[1,0,3,1] row_mask:0xf bank_mask:0xf\n\t"         \
  "v_add_u32 %[sk], %[" #W "], %[" #K "]\n\t"                                                     \
  "v_xor_b32_dpp %[s], %[s1], %[s2] quad_perm:[2,2,1,2] row_mask:0xf bank_mask:0xf\n\t"          \
  "v_add3_u32 %[u], %[s], %[c], %[sk]\n\t"                                                        \
  "v_add_u32 %[t], %[s], %[m]\n\t"                                                                \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_ror:12 row_mask:0xf bank_mask:0x5\n\t"           \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
#define MSHA_ASM_A8(X, Y, Z, W, K)                                                               \
  "v_add_u32 %[y], %[" #W "], %[" #K "]\n\t"                                                      \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh]\n\t"                                        \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                           \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"                           \
  "v_xor_b32_dpp %[s2], %[s1], %[s1] quad_perm:[1,0,3,1] row_mask:0xf bank_mask:0xf\n\t"         \
  "v_xor_b32_dpp %[s], %[s1], %[s2] quad_perm:[2,2,1,2] row_mask:0xf bank_mask:0xf\n\t"          \
  "v_add3_u32 %[u], %[s], %[c], %[" #W "]\n\t"                                                    \
  "v_add3_u32 %[t], %[s], %[m], %[" #K "]\n\t"                                                    \
  "v_add_u32_dpp %[" #W "], %[y], %[u] row_ror:12 row_mask:0xf bank_mask:0x5\n\t"                \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
#define MSHA_ASM8_OPERANDS                                                                       \
  : [X] "+v"(X), [Y] "+v"(Y), [Z] "+v"(Z), [W] "+v"(W), [s1] "=&v"(s1_), [s2] "=&v"(s2_),      \
    [s] "=&v"(s_), [sk] "=&v"(sk_), [c] "=&v"(c_), [u] "=&v"(u_), [m] "=&v"(m_), [t] "=&v"(t_),  \
    [y] "=&v"(y_)                                                                                \
  : [sh] "v"(sh), [k0] "v"(v_.x), [k1] "v"(v_.y), [k2] "v"(v_.z), [k3] "v"(v_.w)
#define MSHA_DQ8(cur, nxt, q)                                                                    \
  {                                                                                              \
    const uint4 v_ = cur[q];                                                                     \
    nxt[q] = nk[col + (q) * 128];                                                                \
    uint32_t s1_, s2_, s_, sk_, c_, u_, m_, t_, y_;                                              \
    asm volatile(MSHA_ASM_E8(X, Y, Z, W, k0) MSHA_ASM_A8(W, X, Y, Z, k0)                         \
                 MSHA_ASM_E8(Z, W, X, Y, k1) MSHA_ASM_A8(Y, Z, W, X, k1)                         \
                 MSHA_ASM_E8(X, Y, Z, W, k2) MSHA_ASM_A8(W, X, Y, Z, k2)                         \
                 MSHA_ASM_E8(Z, W, X, Y, k3) MSHA_ASM_A8(Y, Z, W, X, k3)                         \
                 MSHA_ASM8_OPERANDS);                                                            \
  }
#define MSHA_DBLOCK8(cur, nxt)                                                                   \
  {                                                                                              \
    uint32_t X = H0, Y = H1, Z = H2, W = H3;                                                     \
    _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_) MSHA_DQ8(cur, nxt, q_)                      \
    H0 += X; H1 += Y; H2 += Z; H3 += W;                                                          \
    if (active && sub == 0 && b + 1 == nb)                                                       \
      *reinterpret_cast<uint4*>(out + 32 * o + (eside ? 16 : 0)) =                               \
          make_uint4(bswap(H0), bswap(H1), bswap(H2), bswap(H3));                                \
  }

template <int MODE, bool EXCL>
__device__ __forceinline__ void chain8_body(const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ out_idx,
                                                       uint64_t n, uint8_t* __restrict__ out,
                                                       uint32_t* __restrict__ err,
                                                       const uint32_t* __restrict__ limit) {
  static_assert(MSHA_CHAIN2_FORM == 4, "the eight-lane rounds read form 4's K+W layout");
  __shared__ uint4 kw[2][kC2Per][kCoopSlotQuads * 64];
  __shared__ uint32_t s_nb;
  if (EXCL) asm volatile("" ::: "v255", "a255");  // exclusive CU (see k_digest_coop EXCL)
  if (EXCL) __builtin_amdgcn_s_setprio(3);
  const unsigned lane = threadIdx.x & 63;
  const unsigned wave = threadIdx.x >> 6;
  const bool producer = wave < kC8Producers;
  const bool eside = (lane & 4) == 0;
  const unsigned sub = lane & 3;
  // message of this lane inside the workgroup: each producer's lanes 0-15, each
  // consumer wave's 8 (8 lanes each)
  const unsigned msg = producer ? lane : (wave - kC8Producers) * 8 + (lane >> 3);
  const uint64_t i = (uint64_t)blockIdx.x * kChain8MsgsPerWg + msg;
  bool active = msg < kChain8MsgsPerWg && i < n && (!limit || i < *limit);
  uint64_t m = i;  // metadata index
  if (active && order) {
    const uint32_t v = order[i];
    active = v != kNoLane;
    m = v;
  }
  uint64_t o = m;  // digest slot
  if (active && out_idx) o = out_idx[i];
  if (!active) m = o = 0;
  const uint8_t* pa = arena;
  uint64_t L = 0;
  if (active) {
    pa = arena + off[m];
    L = len[m];
    if (reinterpret_cast<uintptr_t>(pa) & 15) {
      active = false;
      L = 0;
      if (!producer && eside && sub == 0) check_aligned(pa, out + 32 * o, err);
    }
  }
  const uint32_t nfull = (uint32_t)(L >> 6), r = (uint32_t)(L & 63);
  const uint32_t nb = nfull + (r < 56 ? 1 : 2);
  if (threadIdx.x == 0) s_nb = 0;
  __syncthreads();
  if (producer && active) atomicMax(&s_nb, nb);
  __syncthreads();
  const uint32_t NB = s_nb;
  const uint32_t per = kC2Per == 2 && NB >= kC2PairMinBlocks ? 2u : 1u;  // blocks per barrier
  if (producer) {
    // producer w schedules blocks w, w + 2, w + 4, ...: one producer's schedule of
    // a block (~3,160 shader cycles) outlasted the consumers' rounds (~3,010), so
    // one producer bounded the chain (tools/chain2_anatomy 1427 8)
    const uint32_t pw = wave;
    uint32_t raw[16], w[16];
    if (active && pw <= nfull) load_block16<MODE>(pa + 64 * (uint64_t)pw, raw);
    for (uint32_t b = 0; b < NB; ++b) {
      if (b % kC8Producers == pw) {
        if (b < nfull) {
          to_words(raw, w);
        } else if (b == nfull) {
          uint32_t rr = r;
          asm volatile("" : "+v"(rr));
          build_tail(raw, rr, L, w);
        } else {
          length_block(L, w);
        }
        if (active && b + kC8Producers <= nfull) load_block16<MODE>(pa + 64 * (uint64_t)(b + kC8Producers), raw);
        schedule_kw_eo(w, &kw[(b / per) & 1][b % per][lane]);
      }
      if (b % per == per - 1 || b + 1 == NB) MSHA_C2_BARRIER(b / per)  // barrier g: slot g & 1 holds group g
    }
    MSHA_C2_BARRIER((NB + per - 1) / per)  // the consumers' last (they wait one group ahead)
  } else {
    uint32_t H0 = eside ? 0x510e527fu : 0x6a09e667u, H1 = eside ? 0x9b05688cu : 0xbb67ae85u;
    uint32_t H2 = eside ? 0x1f83d9abu : 0x3c6ef372u, H3 = eside ? 0x5be0cd19u : 0xa54ff53au;
    const uint32_t sh = eside ? (sub == 1 ? 11u : sub == 2 ? 25u : 6u) : (sub == 1 ? 13u : sub == 2 ? 22u : 2u);
    const unsigned col = (eside ? 0 : 64) + msg;  // form 4: even rounds' quads, then the odd rounds'
#if MSHA_CHAIN2_PAIR
    if (per == 2) {
      uint4 ka[8], kb[8], kc[8], kd[8];
      MSHA_C2_BARRIER(0)  // barrier 0: slot 0 holds blocks 0 and 1
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        ka[q] = kw[0][0][col + q * 128];
        kb[q] = kw[0][1][col + q * 128];
      }
      const uint32_t NP = (NB + 1) / 2;
      for (uint32_t g = 0; g < NP; ++g) {
        MSHA_C2_BARRIER(g + 1)  // reads past the last block are harmless (unused)
        {
          const uint32_t b = 2 * g;
          const uint4* nk = kw[(g + 1) & 1][0];
          MSHA_DBLOCK8(ka, kc)
        }
        {
          const uint32_t b = 2 * g + 1;
          const uint4* nk = kw[(g + 1) & 1][1];
          MSHA_DBLOCK8(kb, kd)
        }
        if (++g == NP) break;
        MSHA_C2_BARRIER(g + 1)
        {
          const uint32_t b = 2 * g;
          const uint4* nk = kw[(g + 1) & 1][0];
          MSHA_DBLOCK8(kc, ka)
        }
        {
          const uint32_t b = 2 * g + 1;
          const uint4* nk = kw[(g + 1) & 1][1];
          MSHA_DBLOCK8(kd, kb)
        }
      }
      return;
    }
#endif
    uint4 ka[8], kb[8];
    MSHA_C2_BARRIER(0)  // barrier 0: slot 0 holds block 0
#pragma unroll
    for (int q = 0; q < 8; ++q) ka[q] = kw[0][0][col + q * 128];
    for (uint32_t b = 0; b < NB; ++b) {
      MSHA_C2_BARRIER(b + 1)
      const uint4* nk = kw[(b + 1) & 1][0];  // a read past the last block is harmless (unused)
      MSHA_DBLOCK8(ka, kb)
      if (++b == NB) break;
      MSHA_C2_BARRIER(b + 1)
      nk = kw[(b + 1) & 1][0];
      MSHA_DBLOCK8(kb, ka)
    }
  }
}

template <int MODE, bool EXCL>
__global__ __launch_bounds__(256) void k_digest_chain8(const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ out_idx,
                                                       uint64_t n, uint8_t* __restrict__ out,
                                                       uint32_t* __restrict__ err,
                                                       const uint32_t* __restrict__ limit) {
  MSHA_WAVE_STAMP_OPEN()
  chain8_body<MODE, EXCL>(arena, off, len, order, out_idx, n, out, err, limit);
  MSHA_WAVE_STAMP_CLOSE(kStampChain8)
}

#undef MSHA_DBLOCK8
#undef MSHA_DQ8
#undef MSHA_ASM8_OPERANDS
#undef MSHA_ASM_A8
#undef MSHA_ASM_E8

#undef MSHA_DBLOCK
#undef MSHA_DQ
#undef MSHA_ASM_OPERANDS
#undef MSHA_ASM_ROUND3
#undef MSHA_ASM_AROUND
#undef MSHA_ASM_EROUND
#undef MSHA_ASM_CHMAJ
#undef MSHA_ASM_SIGMA
#undef MSHA_C2_BARRIER

// Uniform layout: message i is arena[i*stride : i*stride + msg_len].
template <int MODE>
__global__ __launch_bounds__(256, 8) void k_digest_uniform(const uint8_t* __restrict__ arena,
                                                        uint64_t stride, uint64_t msg_len,
                                                        uint64_t n, uint8_t* __restrict__ out,
                                                        uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = arena + i * stride;
  if (check_aligned(p, out + 32 * i, err))
    hash_message<MODE>(p, msg_len, out + 32 * i);
}

__global__ __launch_bounds__(256) void k_digest_uniform_pipe(const uint8_t* __restrict__ arena,
                                                             uint64_t stride, uint64_t msg_len,
                                                             uint64_t n, uint8_t* __restrict__ out,
                                                             uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = arena + i * stride;
  if (check_aligned(p, out + 32 * i, err))
    hash_message_pipe(p, msg_len, out + 32 * i);
}

// Digest-of-digests (Batch / VerifyBatch actions, /root/reference/pkg/statemachine/
// sequence.go:155-158, batch_tracker.go:175-178): out[i] = SHA256(concat over
// k in [begin[i], begin[i+1]) of table[idx[k]]), every part a 32-byte digest
// already resident in HBM (e.g. request digests produced by k_digest_batch).
// Two digests fill one 64-byte block; the tail block holds 0 or 1 digest.
__global__ __launch_bounds__(256, DigestSrc::kMinWaves) void k_digest_of_digests(const uint8_t* __restrict__ table,
                                                           const uint32_t* __restrict__ idx,
                                                           const uint64_t* __restrict__ begin,
                                                           uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DigestSrc{table, idx, begin}.full<0>(i, out);
}

// ---------------------------------------------------------------------------
// Clock probe (msha_clock_probe; bench.py's effective_clock_ghz). The compression
// on register-resident data at the lane kernel's occupancy (8 waves per SIMD,
// the same VALU mix), with one (s_memtime, s_memrealtime) pair stamped by the
// first lane of each workgroup at its start and end: the in-kernel clock is
// d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// A separate kernel: the hash kernels carry no stamps. Run right after a timed
// region, it reads the clock the chip holds under this instruction mix.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 8) void k_clock_probe(uint32_t blocks, uint64_t* __restrict__ stamps,
                                                        uint32_t* __restrict__ sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = (blockIdx.x * 256 + threadIdx.x) * 16 + k;
  for (uint32_t b = 0; b < blocks; ++b) {
    compress(s, w);
    w[0] ^= s.h[0];  // the next block depends on this one
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    uint64_t* st = stamps + 4 * (uint64_t)blockIdx.x;
    st[0] = t0;
    st[1] = r0;
    st[2] = t1;
    st[3] = r1;
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= s.h[k];
  if (x == 0x9E3779B9u) sink[0] = x;  // keeps the work; practically never stores
}

hipError_t launch_clock_probe(uint32_t blocks, uint32_t workgroups, uint64_t* stamps, uint32_t* sink,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_clock_probe, dim3(workgroups), dim3(256), 0, st, blocks, stamps, sink);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Launchers (host side). Grids are one lane per message, 256-thread blocks.
// ---------------------------------------------------------------------------
static inline unsigned grid_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

// Fewer than ~3 waves per SIMD cannot hide HBM latency by occupancy: use the
// register-prefetching variant then; otherwise pair loads. At one wave per
// SIMD or less the pipelined kernel (kPipe, k_digest_batch_pipe) gives the lone
// wave independent work: c4 2.78 -> 2.64 ms; at 1.5, 2 and 3 waves per SIMD it
// ties or loses (profiles/r01_ab_pipe/). For A/B measurements MSHA_LOAD_MODE
// (0/1/2/3) forces the load mode.
static inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static inline int pick_mode(uint64_t n, int cus) {
  static const int forced = env_int("MSHA_LOAD_MODE", -1);
  if (forced >= kSingle && forced <= kPipe) return forced;
  if (n <= (uint64_t)cus * 4 * 64) return kPipe;
  return n < (uint64_t)cus * 4 * 64 * 3 ? kPrefetch : kPair;
}

// Cooperative chaining (AUTO) when every workgroup of the launch gets a CU of
// its own (n <= 128 per CU): below that one lane per message leaves at least
// half the SIMDs idle, and each consumer's chain runs 905 instead of ~1,400
// instructions per block (profiles/r01_ab_coop: 1.2-1.5x). Above it a second
// round of workgroups would cost more than the lane kernel's single round.
bool uses_coop(uint64_t n, int cus, int policy) {
  if (policy == 2) return true;   // MSHA_KERNEL_COOP
  if (policy == 1) return false;  // MSHA_KERNEL_LANE
  return n <= (uint64_t)cus * kCoopMsgsPerWg;
}

// Calls f(std::integral_constant<int, MODE>) for a runtime load mode of the
// templated lane kernels (kSingle / kPrefetch / kPair). kPipe is not one of
// them: the pipelined loop has kernels of its own (k_digest_*_pipe), and the
// callers pick those before getting here.
template <class F>
static inline void with_mode(int mode, F&& f) {
  switch (mode) {
    case kSingle: f(std::integral_constant<int, kSingle>()); break;
    case kPrefetch: f(std::integral_constant<int, kPrefetch>()); break;
    default: f(std::integral_constant<int, kPair>()); break;
  }
}

// Load mode of a split launch's main workgroups (q = n_main / (64 SIMDs) full
// rounds of waves, q >= 1): prefetching below 3 waves per SIMD, paired loads
// from 3 (the same thresholds as pick_mode, without its kPipe range: the split
// kernel's segment waves share the SIMDs, so the main waves are never alone).
static inline int split_mode(const SplitPlan& sp, int cus) {
  static const int forced = env_int("MSHA_LOAD_MODE", -1);
  if (forced >= kSingle && forced <= kPair) return forced;
  return sp.n_main < (uint64_t)cus * 4 * 64 * 3 ? kPrefetch : kPair;
}

// Split chaining (AUTO and LANE) when the launch is q >= 1 full rounds of waves
// over the SIMDs plus a surplus of r <= SIMDs/2 waves: r chains of
// clamp(SIMDs / r, 2, cap) segments, so no SIMD carries more than one segment.
// The cap (kernels.hpp) is 12 for both sources since round 3 made a hand-off
// cheap -- the arena segment's first block fetched before its wait, the state
// handed over write-through with no release fence: c3 8 / 10 / 12 / 14 / 16
// segments 89.5-90.0 / 89.9 / 88.3-88.9 / 88.9-89.3 / 89.5-89.6 us
// (profiles/r03_ab_c3_preload/); c3dd 92.3 -> 90.3 us at 12, 91.2 at 16, 93.9
// at 24 (profiles/r03_ab_split_sc1/; 8 before, profiles/r01_ab_segs/).
// MSHA_SPLIT_SEGS overrides both (A/B).
bool plan_split(uint64_t n, int cus, int policy, SplitPlan* sp, int cap) {
  static const int forced = env_int("MSHA_SPLIT", -1);  // A/B: 0 = never
  static const int forced_segs = env_int("MSHA_SPLIT_SEGS", 0);
  const int max_segs = std::min(64, std::max(2, forced_segs > 0 ? forced_segs : cap));
  static const uint64_t min_q = (uint64_t)std::max(1, env_int("MSHA_SPLIT_MIN_Q", 1));  // A/B
  if (forced == 0 || policy == 2) return false;
  const uint64_t simds = (uint64_t)cus * 4;
  const uint64_t waves = (n + 63) / 64;
  const uint64_t q = waves / simds, r = waves % simds;
  if (q < min_q || r == 0 || r > simds / 2) return false;
  sp->n_main = q * simds * 64;
  sp->chains = (uint32_t)r;
  sp->segments = (uint32_t)std::min<uint64_t>(max_segs, std::max<uint64_t>(2, simds / r));
  // 4 chains per 256-thread workgroup; a multiple of 8 workgroups per segment
  // keeps a chain's segments on one XCD (workgroup id mod 8)
  sp->groups = (uint32_t)(((r + 3) / 4 + 7) / 8 * 8);
  // Failure-path test (tests/test_gpu_failure.py): MSHA_SPLIT_STALL=1 makes chain
  // 0's first segment skip its handoff, so the waiting segments time out. Read
  // per launch (not cached) so a test can toggle it in one process.
  const char* stall = getenv("MSHA_SPLIT_STALL");
  sp->stall_chain = stall && atoi(stall) == 1 ? 0u : 0xFFFFFFFFu;
  return true;
}

static inline void set_kind(LaunchKind* kind, LaunchKind k) {
  if (kind) *kind = k;
}

hipError_t launch_digest_batch(const uint8_t* arena, const uint64_t* off, const uint64_t* len,
                               const uint32_t* order, const uint32_t* out_idx, uint64_t n,
                               uint8_t* out, uint32_t* err, int cus, int policy, hipStream_t st,
                               const SplitPlan* split, LaunchKind* kind, const LaneGate* gate) {
  set_kind(kind, kLaunchNone);
  if (n == 0) return hipSuccess;
  const uint32_t* head = gate ? gate->head : nullptr;
  if (gate && gate->head_part) {  // the planned launch's long chains, up to *head
#ifdef MSHA_HEAD_NO_EXCL  // A/B build (tools/r06_xcd.sh): heads share their CUs, normal priority
    constexpr bool kX = false;
#else
    constexpr bool kX = true;
#endif
    if (gate->eight_lane) {
      const unsigned grid = (unsigned)((n + kChain8MsgsPerWg - 1) / kChain8MsgsPerWg);
      hipLaunchKernelGGL((k_digest_chain8<kPrefetch, kX>), dim3(grid), dim3(256), 0, st, arena, off, len,
                         order, out_idx, n, out, err, head);
      set_kind(kind, kLaunchChain8);
    } else if (gate->two_lane) {
      const unsigned grid = (unsigned)((n + kChain2MsgsPerWg - 1) / kChain2MsgsPerWg);
      hipLaunchKernelGGL((k_digest_chain2<kPrefetch, kX>), dim3(grid), dim3(192), 0, st, arena, off, len,
                         order, out_idx, n, out, err, head);
      set_kind(kind, kLaunchChain2);
    } else {
      const unsigned grid = (unsigned)((n + kCoopMsgsPerWg - 1) / kCoopMsgsPerWg);
      hipLaunchKernelGGL((k_digest_coop<kPrefetch, kX>), dim3(grid), dim3(256), kCoopDynLds, st, arena, off,
                         len, order, out_idx, n, out, err, head);
      set_kind(kind, kLaunchCoop);
    }
    return hipGetLastError();
  }
  if (split && !gate) {
    const unsigned grid = split->segments * split->groups + (unsigned)(split->n_main / 256);
    const ArenaSrc src{arena, off, len, order, out_idx, err};
    with_mode(split_mode(*split, cus), [&](auto m) {
      hipLaunchKernelGGL((k_digest_split<decltype(m)::value, ArenaSrc>), dim3(grid), dim3(256), 0,
                         st, src, n, out, err, *split);
    });
    set_kind(kind, kLaunchSplit);
    return hipGetLastError();
  }
  if (uses_coop(n, cus, policy) && !head) {
    static const int small8 = env_int("MSHA_SMALL_CHAIN8", 1);
    if (policy == 0 && n <= (uint64_t)cus * kChain8MsgsPerWg && small8) {
      // AUTO, at most 16 messages per CU (a call of a few actions: the latency
      // path): the eight-lane chain, one workgroup per CU (64 KiB of dynamic LDS
      // on top of its 64 KiB keeps a second one off the CU). MSHA_SMALL_CHAIN8=0:
      // the two-lane chain below (A/B).
      const unsigned grid = (unsigned)((n + kChain8MsgsPerWg - 1) / kChain8MsgsPerWg);
      hipLaunchKernelGGL((k_digest_chain8<kPrefetch, false>), dim3(grid), dim3(256), 64 * 1024, st, arena, off,
                         len, order, out_idx, n, out, err, nullptr);
      set_kind(kind, kLaunchChain8);
      return hipGetLastError();
    }
    if (policy == 0 && n <= (uint64_t)cus * kChain2MsgsPerWg && env_int("MSHA_SMALL_CHAIN2", 1)) {
      // AUTO, at most 64 messages per CU: the two-lane chain, one workgroup per CU
      // (64 KiB of dynamic LDS on top of its 33 KiB keeps a second one off the CU,
      // whose consumers would share SIMDs with the first's)
      const unsigned grid = (unsigned)((n + kChain2MsgsPerWg - 1) / kChain2MsgsPerWg);
      hipLaunchKernelGGL((k_digest_chain2<kPrefetch, false>), dim3(grid), dim3(192), 64 * 1024, st, arena, off,
                         len, order, out_idx, n, out, err, nullptr);
      set_kind(kind, kLaunchChain2);
      return hipGetLastError();
    }
    const unsigned grid = (unsigned)((n + kCoopMsgsPerWg - 1) / kCoopMsgsPerWg);
    hipLaunchKernelGGL(k_digest_coop<kPrefetch>, dim3(grid), dim3(256), kCoopDynLds, st, arena, off, len,
                       order, out_idx, n, out, err, nullptr);
    set_kind(kind, kLaunchCoop);
    return hipGetLastError();
  }
  const int mode = pick_mode(n, cus);
  if (mode == kPipe) {
    hipLaunchKernelGGL(k_digest_batch_pipe, dim3(grid_for(n)), dim3(256), 0, st, arena, off, len,
                       order, out_idx, n, out, err, head);
    set_kind(kind, kLaunchPipe);
    return hipGetLastError();
  }
  if (gate && gate->ws_ctr) {  // resident workgroups stealing 64-lane tiles (k_digest_batch_ws)
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cus * 8, (n + 255) / 256);
    with_mode(mode, [&](auto m) {
      hipLaunchKernelGGL(k_digest_batch_ws<decltype(m)::value>, dim3(grid), dim3(256), 0, st, arena, off, len,
                         order, out_idx, n, out, err, head, gate->ws_ctr, gate->lanes);
    });
    set_kind(kind, kLaunchLaneWs);
    return hipGetLastError();
  }
  with_mode(mode, [&](auto m) {
    hipLaunchKernelGGL(k_digest_batch<decltype(m)::value>, dim3(grid_for(n)), dim3(256), 0, st,
                       arena, off, len, order, out_idx, n, out, err, head);
  });
  set_kind(kind, kLaunchLane);
  return hipGetLastError();
}

hipError_t launch_digest_uniform(const uint8_t* arena, uint64_t stride, uint64_t msg_len,
                                 uint64_t n, uint8_t* out, uint32_t* err, int cus,
                                 hipStream_t st, LaunchKind* kind) {
  set_kind(kind, kLaunchNone);
  if (n == 0) return hipSuccess;
  const int mode = pick_mode(n, cus);
  if (mode == kPipe) {
    hipLaunchKernelGGL(k_digest_uniform_pipe, dim3(grid_for(n)), dim3(256), 0, st, arena, stride,
                       msg_len, n, out, err);
    set_kind(kind, kLaunchPipe);
    return hipGetLastError();
  }
  with_mode(mode, [&](auto m) {
    hipLaunchKernelGGL(k_digest_uniform<decltype(m)::value>, dim3(grid_for(n)), dim3(256), 0, st,
                       arena, stride, msg_len, n, out, err);
  });
  set_kind(kind, kLaunchLane);
  return hipGetLastError();
}

hipError_t launch_digest_of_digests(const uint8_t* table, const uint32_t* idx,
                                    const uint64_t* begin, uint64_t n, uint8_t* out,
                                    uint32_t* err, hipStream_t st, const SplitPlan* split,
                                    LaunchKind* kind) {
  set_kind(kind, kLaunchNone);
  if (n == 0) return hipSuccess;
  if (split) {
    const unsigned grid = split->segments * split->groups + (unsigned)(split->n_main / 256);
    hipLaunchKernelGGL((k_digest_split<0, DigestSrc>), dim3(grid), dim3(256), 0, st,
                       DigestSrc{table, idx, begin}, n, out, err, *split);
    set_kind(kind, kLaunchSplit);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_digest_of_digests, dim3(grid_for(n)), dim3(256), 0, st, table, idx, begin,
                     n, out);
  set_kind(kind, kLaunchDod);
  return hipGetLastError();
}

}  // namespace msha
