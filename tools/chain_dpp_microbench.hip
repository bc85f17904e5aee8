// Latency of ONE SHA-256 round chain on a lone wave -- the regime of the
// cooperative head's consumer, whose ~1.75 us per block (14 VALU instructions a
// round, issue-bound: profiles/r03_ab_coop_round3/) is c5's floor over several
// GPUs. Variant A: one lane per chain (the shipped round). Variant B: two lanes
// per chain -- lane p < 8 of each 16-lane row holds the e-side (e f g h), lane
// 15 - p the a-side (a b c d) -- so ONE v_alignbit x3 + xor3 computes Sigma1 in
// the e-lane and Sigma0 in the a-lane (per-lane rotate amounts), Ch and Maj are
// one bitop3 each, and the two new words come from two row_mirror DPP adds that
// write only their side's lanes (bank_mask): 11 instructions a round.
//   e-lane: U = Sig1 + Ch + (h + KW) = T1;  e' = mirror(d) + T1
//   a-lane: T = Sig0 + Maj + 0       = T2;  a' = mirror(T1) + T2
// Both variants run the same R rounds from the same state with the same K+W
// stream; B's final state is checked against A's. One 64-thread workgroup per
// launch (one wave alone on its SIMD), kernel time from HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/chain_dpp_microbench tools/chain_dpp_microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int kChains = 32;
constexpr int kOuter = 4096;  // x 64 rounds

__device__ __forceinline__ uint32_t init_word(uint32_t c, uint32_t j) { return (c + 1) * 0x9E3779B9u ^ (j * 0x85EBCA6Bu); }
__device__ __forceinline__ uint32_t kw_word(uint32_t c, uint32_t t) { return (c + 7) * 0xC2B2AE35u + t * 0x27D4EB2Fu; }

#define RND_A(a, b, c, d, e, f, g, h, kw)               \
  {                                                    \
    uint32_t t1 = h + (kw) + Sig1(e) + ch(e, f, g);    \
    d += t1;                                           \
    h = t1 + Sig0(a) + maj(a, b, c);                   \
  }

__global__ __launch_bounds__(64) void k_chain_lane(uint32_t* out) {
  const uint32_t c = threadIdx.x % kChains;
  uint32_t a = init_word(c, 0), b = init_word(c, 1), cc = init_word(c, 2), d = init_word(c, 3);
  uint32_t e = init_word(c, 4), f = init_word(c, 5), g = init_word(c, 6), h = init_word(c, 7);
  uint32_t kw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kw[j] = kw_word(c, j);
  for (int o = 0; o < kOuter; ++o) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      RND_A(a, b, cc, d, e, f, g, h, kw[0]) RND_A(h, a, b, cc, d, e, f, g, kw[1])
      RND_A(g, h, a, b, cc, d, e, f, kw[2]) RND_A(f, g, h, a, b, cc, d, e, kw[3])
      RND_A(e, f, g, h, a, b, cc, d, kw[4]) RND_A(d, e, f, g, h, a, b, cc, kw[5])
      RND_A(cc, d, e, f, g, h, a, b, kw[6]) RND_A(b, cc, d, e, f, g, h, a, kw[7])
    }
  }
  if (threadIdx.x < kChains) {
    uint32_t* o = out + 8 * c;
    o[0] = a; o[1] = b; o[2] = cc; o[3] = d; o[4] = e; o[5] = f; o[6] = g; o[7] = h;
  }
}

// One round of variant B. X Y Z W: this lane's side (e f g h or a b c d).
#define RND_B(X, Y, Z, W, kw)                                                                  \
  {                                                                                            \
    const uint32_t s = xor3(__builtin_amdgcn_alignbit(X, X, sh1), __builtin_amdgcn_alignbit(X, X, sh2), \
                            __builtin_amdgcn_alignbit(X, X, sh3));                             \
    const uint32_t cch = ch(X, Y, Z), cmj = maj(X, Y, Z);                                      \
    const uint32_t u = s + cch + (W + (kw));                                                   \
    uint32_t t = s + cmj + (kw);                                                               \
    asm volatile("v_add_u32_dpp %0, %1, %2 row_mirror row_mask:0xf bank_mask:0x3"              \
                 : "+v"(t) : "v"(W), "v"(u));                                                  \
    asm volatile("v_add_u32_dpp %0, %1, %0 row_mirror row_mask:0xf bank_mask:0xc"  \
                 : "+v"(t) : "v"(u));                                                          \
    W = t;                                                                                     \
  }

__global__ __launch_bounds__(64) void k_chain_dpp(uint32_t* out) {
  const uint32_t lane = threadIdx.x, p = lane & 15, row = lane >> 4;
  const bool eside = p < 8;
  const uint32_t c = row * 8 + (eside ? p : 15 - p);  // chain 0..31
  // e-side: X..W = e f g h, rotates 6 11 25; a-side: a b c d, rotates 2 13 22
  uint32_t X = init_word(c, eside ? 4 : 0), Y = init_word(c, eside ? 5 : 1);
  uint32_t Z = init_word(c, eside ? 6 : 2), W = init_word(c, eside ? 7 : 3);
  const uint32_t sh1 = eside ? 6 : 2, sh2 = eside ? 11 : 13, sh3 = eside ? 25 : 22;
  uint32_t kw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kw[j] = eside ? kw_word(c, j) : 0u;
  for (int o = 0; o < kOuter; ++o) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      // the new word lands in the oldest register (W), the others shift by renaming
      RND_B(X, Y, Z, W, kw[0]) RND_B(W, X, Y, Z, kw[1]) RND_B(Z, W, X, Y, kw[2]) RND_B(Y, Z, W, X, kw[3])
      RND_B(X, Y, Z, W, kw[4]) RND_B(W, X, Y, Z, kw[5]) RND_B(Z, W, X, Y, kw[6]) RND_B(Y, Z, W, X, kw[7])
    }
  }
  // after a multiple of 4 rounds the names are back in place: X..W = newest..oldest
  uint32_t* o = out + 8 * c + (eside ? 4 : 0);
  o[0] = X; o[1] = Y; o[2] = Z; o[3] = W;
}

int main() {
  uint32_t *d_a, *d_b;
  CHECK(hipMalloc(&d_a, 8 * kChains * 4));
  CHECK(hipMalloc(&d_b, 8 * kChains * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // warm the clocks: a few hundred ms of both
  for (int i = 0; i < 40; ++i) {
    hipLaunchKernelGGL(k_chain_lane, dim3(1), dim3(64), 0, 0, d_a);
    hipLaunchKernelGGL(k_chain_dpp, dim3(1), dim3(64), 0, 0, d_b);
  }
  CHECK(hipDeviceSynchronize());
  const double rounds = 64.0 * kOuter;
  for (int rep = 0; rep < 3; ++rep) {
    float ms_a, ms_b;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_chain_lane, dim3(1), dim3(64), 0, 0, d_a);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms_a, e0, e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_chain_dpp, dim3(1), dim3(64), 0, 0, d_b);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms_b, e0, e1));
    printf("{\"rep\": %d, \"lane_ns_per_round\": %.3f, \"dpp_ns_per_round\": %.3f, \"lane_us_per_block\": %.3f, "
           "\"dpp_us_per_block\": %.3f}\n",
           rep, ms_a * 1e6 / rounds, ms_b * 1e6 / rounds, ms_a * 1e3 / rounds * 64, ms_b * 1e3 / rounds * 64);
  }
  uint32_t ha[8 * kChains], hb[8 * kChains];
  CHECK(hipMemcpy(ha, d_a, sizeof ha, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb, d_b, sizeof hb, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 8 * kChains; ++i) bad += ha[i] != hb[i];
  printf("{\"state_words_differing\": %d, \"of\": %d}\n", bad, 8 * kChains);
  return bad ? 1 : 0;
}
