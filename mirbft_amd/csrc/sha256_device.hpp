// SHA-256 compression for gfx950 (CDNA4), one message per wavefront lane.
//
// This is the device half of the replacement for Go crypto/sha256's block
// function, which the reference reaches through processor.Hasher
// (/root/reference/pkg/processor/serial.go:21-23, :186-191). Algorithm:
// FIPS 180-4 section 6.2.2; the CPU restatement that checks it is
// oracle/sha256_oracle.c.
//
// Instruction selection is driven by measured gfx950 issue rates
// (tools/valu_microbench*.hip, profiles/r01_valu_microbench*.jsonl):
//   full rate (~2 SIMD cycles / wave64 instr): v_add_u32 (VGPR operands),
//       v_xor_b32, v_lshrrev_b32, v_bitop3_b32
//   half rate (~4 cycles): v_alignbit_b32, v_add3_u32, v_bfi_b32, v_perm_b32,
//       v_xad_u32, and any VOP2 with an SGPR operand
// gfx950 has no v_xor3_b32, but it has v_bitop3_b32 (arbitrary 3-input
// boolean function, full rate): it gives xor3 (Sigma/sigma), Ch and Maj in
// one full-rate instruction each. Rotates stay v_alignbit_b32 (one half-rate
// op beats the two full-rate shifts plus merge). Byte swaps are v_perm_b32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msha {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
// bitop3 truth table index = (src0 << 2) | (src1 << 1) | src2.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t Sig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t Sig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t sig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t sig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

#define MSHA_K_TABLE                                                                                 \
  0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,        \
      0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,    \
      0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,    \
      0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,    \
      0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,    \
      0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,    \
      0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,    \
      0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,    \
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,    \
      0xc67178f2u

struct State {
  uint32_t h[8];
};

__device__ __forceinline__ void state_init(State& s) {
  s.h[0] = 0x6a09e667u; s.h[1] = 0xbb67ae85u; s.h[2] = 0x3c6ef372u; s.h[3] = 0xa54ff53au;
  s.h[4] = 0x510e527fu; s.h[5] = 0x9b05688cu; s.h[6] = 0x1f83d9abu; s.h[7] = 0x5be0cd19u;
}

// One round; the eight working variables rotate by renaming (no moves).
#define MSHA_ROUND(a, b, c, d, e, f, g, h, Kt, Wt)      \
  {                                                     \
    uint32_t t1 = (h + (Kt) + (Wt)) + Sig1(e) + ch(e, f, g); \
    d += t1;                                            \
    h = t1 + Sig0(a) + maj(a, b, c);                    \
  }

// Schedule update for round i >= 16 over the rolling 16-word window.
#define MSHA_SCHED(w, i) \
  (w[(i) & 15] += sig1(w[((i) - 2) & 15]) + w[((i) - 7) & 15] + sig0(w[((i) - 15) & 15]))

#define MSHA_R8(i, W)                                                   \
  MSHA_ROUND(a, b, c, d, e, f, g, h, K[(i) + 0], W((i) + 0))            \
  MSHA_ROUND(h, a, b, c, d, e, f, g, K[(i) + 1], W((i) + 1))            \
  MSHA_ROUND(g, h, a, b, c, d, e, f, K[(i) + 2], W((i) + 2))            \
  MSHA_ROUND(f, g, h, a, b, c, d, e, K[(i) + 3], W((i) + 3))            \
  MSHA_ROUND(e, f, g, h, a, b, c, d, K[(i) + 4], W((i) + 4))            \
  MSHA_ROUND(d, e, f, g, h, a, b, c, K[(i) + 5], W((i) + 5))            \
  MSHA_ROUND(c, d, e, f, g, h, a, b, K[(i) + 6], W((i) + 6))            \
  MSHA_ROUND(b, c, d, e, f, g, h, a, K[(i) + 7], W((i) + 7))

// Compress one 64-byte block whose 16 big-endian words are already in w[]
// (w is clobbered: it ends holding schedule words 48..63).
__device__ __forceinline__ void compress(State& s, uint32_t (&w)[16]) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#define MSHA_W_DIRECT(i) w[(i) & 15]
#define MSHA_W_SCHED(i) MSHA_SCHED(w, i)
  MSHA_R8(0, MSHA_W_DIRECT)
  MSHA_R8(8, MSHA_W_DIRECT)
  MSHA_R8(16, MSHA_W_SCHED)
  MSHA_R8(24, MSHA_W_SCHED)
  MSHA_R8(32, MSHA_W_SCHED)
  MSHA_R8(40, MSHA_W_SCHED)
  MSHA_R8(48, MSHA_W_SCHED)
  MSHA_R8(56, MSHA_W_SCHED)
#undef MSHA_W_DIRECT
#undef MSHA_W_SCHED
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// ---- scalar-unit (SALU) helpers for wave-uniform values -------------------
// SALU has no rotate; LLVM would turn a shift/or rotate back into the VALU
// v_alignbit_b32, so the scalar rotate is spelled out in asm.
template <int N>
__device__ __forceinline__ uint32_t srotr(uint32_t x) {
  uint32_t r, t;
  asm("s_lshr_b32 %0, %2, %3\n\ts_lshl_b32 %1, %2, %4\n\ts_or_b32 %0, %0, %1"
      : "=&s"(r), "=&s"(t)
      : "s"(x), "i"(N), "i"(32 - N)
      : "scc");
  return r;
}
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return srotr<7>(x) ^ srotr<18>(x) ^ (x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return srotr<17>(x) ^ srotr<19>(x) ^ (x >> 10); }

// Compress a final block whose words are all wave-uniform: the padding-only
// block of a message with len % 64 == 0 (w0 = 0x80000000) or the length-only
// block after a tail of >= 56 bytes (w0 = 0). Its 48-word schedule depends
// only on the length, so it is expanded once per wave on the scalar unit and
// every round takes K[t]+W[t] from an SGPR: the VALU does only the 64 rounds.
__device__ __forceinline__ void compress_uniform_pad(State& s, uint32_t w0, uint32_t bits_hi,
                                                     uint32_t bits_lo) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t w[16];
  w[0] = w0;
#pragma unroll
  for (int j = 1; j < 14; ++j) w[j] = 0;
  w[14] = bits_hi;
  w[15] = bits_lo;
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#define MSHA_W_UDIRECT(i) w[(i) & 15]
#define MSHA_W_USCHED(i) \
  (w[(i) & 15] += ssig1(w[((i) - 2) & 15]) + w[((i) - 7) & 15] + ssig0(w[((i) - 15) & 15]))
#define MSHA_UROUND(a, b, c, d, e, f, g, h, i, W)           \
  {                                                         \
    const uint32_t kw = K[i] + W(i); /* SALU */             \
    uint32_t t1 = h + kw + Sig1(e) + ch(e, f, g);           \
    d += t1;                                                \
    h = t1 + Sig0(a) + maj(a, b, c);                        \
  }
#define MSHA_UR8(i, W)                              \
  MSHA_UROUND(a, b, c, d, e, f, g, h, (i) + 0, W)   \
  MSHA_UROUND(h, a, b, c, d, e, f, g, (i) + 1, W)   \
  MSHA_UROUND(g, h, a, b, c, d, e, f, (i) + 2, W)   \
  MSHA_UROUND(f, g, h, a, b, c, d, e, (i) + 3, W)   \
  MSHA_UROUND(e, f, g, h, a, b, c, d, (i) + 4, W)   \
  MSHA_UROUND(d, e, f, g, h, a, b, c, (i) + 5, W)   \
  MSHA_UROUND(c, d, e, f, g, h, a, b, (i) + 6, W)   \
  MSHA_UROUND(b, c, d, e, f, g, h, a, (i) + 7, W)
  MSHA_UR8(0, MSHA_W_UDIRECT)
  MSHA_UR8(8, MSHA_W_UDIRECT)
  MSHA_UR8(16, MSHA_W_USCHED)
  MSHA_UR8(24, MSHA_W_USCHED)
  MSHA_UR8(32, MSHA_W_USCHED)
  MSHA_UR8(40, MSHA_W_USCHED)
  MSHA_UR8(48, MSHA_W_USCHED)
  MSHA_UR8(56, MSHA_W_USCHED)
#undef MSHA_UR8
#undef MSHA_UROUND
#undef MSHA_W_USCHED
#undef MSHA_W_UDIRECT
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// Words of the final (padded) block(s), built from the r = len % 64 leftover
// bytes whose little-endian dwords are raw[0..15] (dwords at or past r are
// ignored). Returns 1 if a second, all-padding block is needed (r >= 56).
__device__ __forceinline__ int build_tail(const uint32_t (&raw)[16], uint32_t r, uint64_t len,
                                          uint32_t (&w)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    int k = (int)r - 4 * j;  // valid bytes in dword j
    uint32_t x = raw[j];
    uint32_t keep = k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : (0xffffffffu >> (32 - 8 * k)));
    uint32_t pad = (k >= 0 && k < 4) ? (0x80u << (8 * k)) : 0u;
    w[j] = bswap((x & keep) | pad);
  }
  const uint64_t bits = len * 8;
  if (r < 56) {
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    return 0;
  }
  return 1;
}

__device__ __forceinline__ void length_block(uint64_t len, uint32_t (&w)[16]) {
#pragma unroll
  for (int j = 0; j < 14; ++j) w[j] = 0;
  const uint64_t bits = len * 8;
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
}

// Store the digest (big-endian words) as 32 contiguous bytes.
__device__ __forceinline__ void store_digest(const State& s, uint8_t* out) {
  uint4 lo = make_uint4(bswap(s.h[0]), bswap(s.h[1]), bswap(s.h[2]), bswap(s.h[3]));
  uint4 hi = make_uint4(bswap(s.h[4]), bswap(s.h[5]), bswap(s.h[6]), bswap(s.h[7]));
  reinterpret_cast<uint4*>(out)[0] = lo;
  reinterpret_cast<uint4*>(out)[1] = hi;
}

}  // namespace msha
