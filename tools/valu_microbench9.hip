// Integer-VALU microbenchmark, part 9 (gfx950): an all-full-rate SHA-256?
// Part 8 showed that full-rate VALU ops only reach their 2-cycle rate when
// two waves issue full-rate ops back to back; interleaved with half-rate ops
// (v_alignbit_b32, v_add3_u32, ...) every instruction costs ~4 cycles. So the
// compression function is rebuilt from full-rate ops only and compared with the
// production form on register-resident data (part 4's harness):
//   ALIGN: rotr via v_alignbit_b32 (half rate)
//   SHIFT: rotr via v_lshrrev + v_lshlrev, the pieces folded into v_bitop3 XOR trees
//   ADD3 : sums via v_add3_u32 (half rate)          ADD2: v_add_u32_e32 only (full rate; K as literal)
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench9 tools/valu_microbench9.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int NBLK = 64;

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <uint32_t K>
__device__ __forceinline__ uint32_t addk(uint32_t a) {
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "i"(K), "v"(a));
  return r;
}
template <int N> __device__ __forceinline__ uint32_t shr(uint32_t x) {
  uint32_t r;
  asm("v_lshrrev_b32_e32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
  return r;
}
template <int N> __device__ __forceinline__ uint32_t shl(uint32_t x) {
  uint32_t r;
  asm("v_lshlrev_b32_e32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Sigma via 6 shifts + 2 bitop3 + 1 xor
template <int A, int B, int C> __device__ __forceinline__ uint32_t SigS(uint32_t x) {
  return x3(x3(shr<A>(x), shl<32 - A>(x), shr<B>(x)), shl<32 - B>(x), shr<C>(x)) ^ shl<32 - C>(x);
}
// sigma (two rotates + one shift): 5 shifts + 2 bitop3
template <int A, int B, int C> __device__ __forceinline__ uint32_t sigS(uint32_t x) {
  return x3(x3(shr<A>(x), shl<32 - A>(x), shr<B>(x)), shl<32 - B>(x), shr<C>(x));
}

template <bool SHIFT, bool ADD2>
struct V {
  static __device__ __forceinline__ uint32_t S1(uint32_t e) { return SHIFT ? SigS<6, 11, 25>(e) : Sig1(e); }
  static __device__ __forceinline__ uint32_t S0(uint32_t a) { return SHIFT ? SigS<2, 13, 22>(a) : Sig0(a); }
  static __device__ __forceinline__ uint32_t s0(uint32_t x) { return SHIFT ? sigS<7, 18, 3>(x) : sig0(x); }
  static __device__ __forceinline__ uint32_t s1(uint32_t x) { return SHIFT ? sigS<17, 19, 10>(x) : sig1(x); }
};

#define VROUND(a, b, c, d, e, f, g, h, Kt, Wt)                                         \
  {                                                                                   \
    uint32_t t1;                                                                      \
    if (ADD2) t1 = add2(add2(add2(addk<Kt>(h), Wt), P::S1(e)), ch(e, f, g));          \
    else t1 = (h + (Kt) + (Wt)) + P::S1(e) + ch(e, f, g);                             \
    if (ADD2) { d = add2(d, t1); h = add2(add2(t1, P::S0(a)), maj(a, b, c)); }        \
    else { d += t1; h = t1 + P::S0(a) + maj(a, b, c); }                               \
  }
#define VSCHED(w, i)                                                                                      \
  (ADD2 ? (w[(i) & 15] = add2(add2(add2(w[(i) & 15], P::s1(w[((i) - 2) & 15])), w[((i) - 7) & 15]),      \
                                 P::s0(w[((i) - 15) & 15])))                                             \
        : (w[(i) & 15] += P::s1(w[((i) - 2) & 15]) + w[((i) - 7) & 15] + P::s0(w[((i) - 15) & 15])))
#define VR8(i, W)                                                   \
  VROUND(a, b, c, d, e, f, g, h, K[(i) + 0], W((i) + 0))            \
  VROUND(h, a, b, c, d, e, f, g, K[(i) + 1], W((i) + 1))            \
  VROUND(g, h, a, b, c, d, e, f, K[(i) + 2], W((i) + 2))            \
  VROUND(f, g, h, a, b, c, d, e, K[(i) + 3], W((i) + 3))            \
  VROUND(e, f, g, h, a, b, c, d, K[(i) + 4], W((i) + 4))            \
  VROUND(d, e, f, g, h, a, b, c, K[(i) + 5], W((i) + 5))            \
  VROUND(c, d, e, f, g, h, a, b, K[(i) + 6], W((i) + 6))            \
  VROUND(b, c, d, e, f, g, h, a, K[(i) + 7], W((i) + 7))

template <bool SHIFT, bool ADD2>
__device__ __forceinline__ void compress_v(State& s, uint32_t (&w)[16]) {
  using P = V<SHIFT, ADD2>;
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#define WD(i) w[(i) & 15]
#define WS(i) VSCHED(w, i)
  VR8(0, WD) VR8(8, WD) VR8(16, WS) VR8(24, WS) VR8(32, WS) VR8(40, WS) VR8(48, WS) VR8(56, WS)
#undef WD
#undef WS
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

template <int WPS, bool SHIFT, bool ADD2>
__global__ __launch_bounds__(256, WPS) void k_v(unsigned* out, unsigned seed) {
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x;
  for (int blk = 0; blk < NBLK; ++blk) {
    compress_v<SHIFT, ADD2>(s, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] ^= s.h[j & 7] + j;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= s.h[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// correctness: every variant must produce the same digest words as compress()
template <bool SHIFT, bool ADD2>
__global__ void k_check(unsigned* bad) {
  State s0, s1;
  state_init(s0);
  state_init(s1);
  uint32_t w0[16], w1[16];
  for (int j = 0; j < 16; ++j) w0[j] = w1[j] = 0x9e3779b9u * (j + 1) ^ threadIdx.x;
  compress(s0, w0);
  compress_v<SHIFT, ADD2>(s1, w1);
  for (int j = 0; j < 8; ++j)
    if (s0.h[j] != s1.h[j]) atomicAdd(bad, 1u);
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048 * 2));
  unsigned* bad;
  CHECK(hipMalloc(&bad, 4));
  CHECK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL((k_check<true, true>), dim3(1), dim3(256), 0, 0, bad);
  hipLaunchKernelGGL((k_check<true, false>), dim3(1), dim3(256), 0, 0, bad);
  hipLaunchKernelGGL((k_check<false, true>), dim3(1), dim3(256), 0, 0, bad);
  unsigned hbad = 0;
  CHECK(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
  printf("{\"check_mismatches\": %u}\n", hbad);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 7; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best;
  };
  auto report = [&](const char* name, int wps, float ms) {
    double blocks = (double)cus * wps * 256 * NBLK;
    printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gblocks_per_s\": %.3f, "
           "\"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
           name, wps, ms, blocks / (ms * 1e-3) / 1e9, ms * 1e-3 * 2.4e9 / (wps * NBLK));
  };
#define RUN(WPS, SH, A2, NAME) report(NAME, WPS, timeit([&] { hipLaunchKernelGGL((k_v<WPS, SH, A2>), dim3(cus * WPS), dim3(256), 0, 0, out, 7u); }))
  for (int rep = 0; rep < 2; ++rep) {
    RUN(8, false, false, "ALIGN+ADD3 (production)");
    RUN(8, true, true, "SHIFT+ADD2 (all full rate)");
    RUN(8, true, false, "SHIFT+ADD3");
    RUN(8, false, true, "ALIGN+ADD2");
    RUN(4, false, false, "ALIGN+ADD3 (production)");
    RUN(4, true, true, "SHIFT+ADD2 (all full rate)");
    RUN(2, true, true, "SHIFT+ADD2 (all full rate)");
  }
  return 0;
}
