// Integer-VALU microbenchmark, part 19 (gfx950): an "H-heavy" SHA-256. Parts
// 13-18: gfx950 overlaps a full-rate op (v_add, v_xor, v_bitop3, v_lshrrev) of
// one wave with a half-rate op (v_alignbit, v_add3, v_bfi, v_lshlrev, ...) of
// another only when the full-rate op's wave is (nearly) all full-rate, or the
// half-rate op's wave is mostly half-rate (H3F1 + F: 2.2 cycles/instr), while
// two waves alternating the classes get ~4. The production round is 9 half- +
// 5 full-rate ops. Here the same instruction count with more of them half-rate
// (Ch as v_bfi, e' = v_add3(d, t1, 0); in the schedule, x >> n as
// v_alignbit(0, x, n) and both adds as v_add3) -- 11+3 per round, 8+2 per
// schedule word -- on register-resident data (part 4's harness), against the
// production compress(), at 2, 4 and 8 waves per SIMD; digests compared.
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench19 tools/valu_microbench19.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int NBLK = 64;

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t add3z(uint32_t a, uint32_t b) {  // a + b as a half-rate v_add3
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t add3v(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t add3k(uint32_t a, uint32_t k, uint32_t b) {  // k: wave-uniform (SGPR)
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(b));
  return r;
}
template <int N> __device__ __forceinline__ uint32_t shr_h(uint32_t x) {  // x >> N as v_alignbit(0, x, N)
  uint32_t r;
  asm("v_alignbit_b32 %0, 0, %1, %2" : "=v"(r) : "v"(x), "i"(N));
  return r;
}
__device__ __forceinline__ uint32_t hsig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), shr_h<3>(x)); }
__device__ __forceinline__ uint32_t hsig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), shr_h<10>(x)); }

// H-heavy round (11 half-rate + 3 full-rate): t1 = (h + K + W) + (Sig1 + Ch);
// e' = v_add3(d, t1, 0); a' = v_add3(t1, Sig0, Maj).
#define HH_ROUND(a, b, c, d, e, f, g, h, Kt, Wt)        \
  {                                                     \
    const uint32_t hkw = add3k(h, (Kt), (Wt));          \
    const uint32_t t1 = add3v(hkw, Sig1(e), bfi(e, f, g)); \
    d = add3z(d, t1);                                   \
    h = add3v(t1, Sig0(a), maj(a, b, c));               \
  }
#define HH_SCHED(w, i) \
  (w[(i) & 15] = add3z(add3v(hsig1(w[((i) - 2) & 15]), w[((i) - 7) & 15], hsig0(w[((i) - 15) & 15])), w[(i) & 15]))
#define HH_R8(i, W)                                                 \
  HH_ROUND(a, b, c, d, e, f, g, h, K[(i) + 0], W((i) + 0))          \
  HH_ROUND(h, a, b, c, d, e, f, g, K[(i) + 1], W((i) + 1))          \
  HH_ROUND(g, h, a, b, c, d, e, f, K[(i) + 2], W((i) + 2))          \
  HH_ROUND(f, g, h, a, b, c, d, e, K[(i) + 3], W((i) + 3))          \
  HH_ROUND(e, f, g, h, a, b, c, d, K[(i) + 4], W((i) + 4))          \
  HH_ROUND(d, e, f, g, h, a, b, c, K[(i) + 5], W((i) + 5))          \
  HH_ROUND(c, d, e, f, g, h, a, b, K[(i) + 6], W((i) + 6))          \
  HH_ROUND(b, c, d, e, f, g, h, a, K[(i) + 7], W((i) + 7))

template <bool HROUND, bool HSCHED>
__device__ __forceinline__ void compress_v(State& s, uint32_t (&w)[16]) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#define WD(i) w[(i) & 15]
#define WP(i) MSHA_SCHED(w, i)
#define WH(i) HH_SCHED(w, i)
  if (HROUND) {
    if (HSCHED) { HH_R8(0, WD) HH_R8(8, WD) HH_R8(16, WH) HH_R8(24, WH) HH_R8(32, WH) HH_R8(40, WH) HH_R8(48, WH) HH_R8(56, WH) }
    else { HH_R8(0, WD) HH_R8(8, WD) HH_R8(16, WP) HH_R8(24, WP) HH_R8(32, WP) HH_R8(40, WP) HH_R8(48, WP) HH_R8(56, WP) }
  } else {
    if (HSCHED) { MSHA_R8(0, WD) MSHA_R8(8, WD) MSHA_R8(16, WH) MSHA_R8(24, WH) MSHA_R8(32, WH) MSHA_R8(40, WH) MSHA_R8(48, WH) MSHA_R8(56, WH) }
    else { MSHA_R8(0, WD) MSHA_R8(8, WD) MSHA_R8(16, WP) MSHA_R8(24, WP) MSHA_R8(32, WP) MSHA_R8(40, WP) MSHA_R8(48, WP) MSHA_R8(56, WP) }
  }
#undef WD
#undef WP
#undef WH
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

template <int WPS, bool HROUND, bool HSCHED>
__global__ __launch_bounds__(256, WPS) void k_sha(unsigned* out, unsigned seed) {
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x + blockIdx.x * 977u;
  for (int blk = 0; blk < NBLK; ++blk) {
    compress_v<HROUND, HSCHED>(s, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] ^= s.h[j & 7] + j;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) out[(size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 8 + j] = s.h[j];
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const size_t nmax = (size_t)cus * 2048 * 8;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * nmax));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 400.f;) {
      for (int i = 0; i < 8; ++i) launch();
      CHECK(hipEventRecord(w1));
      CHECK(hipEventSynchronize(w1));
      CHECK(hipEventElapsedTime(&el, w0, w1));
    }
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best;
  };
  std::vector<unsigned> ref(nmax), got(nmax);
  auto run = [&](const char* name, int wps, auto kern) {
    const dim3 grid(cus * wps);
    float ms = timeit([&] { hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, out, 7u); });
    const size_t n = (size_t)cus * wps * 256 * 8;
    CHECK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
    return std::make_pair(ms, n);
  };
#define RUNV(WPS, HR, HS, NAME)                                                                               \
  {                                                                                                           \
    auto pr = run(NAME, WPS, k_sha<WPS, false, false>);                                                       \
    const size_t n = pr.second;                                                                               \
    std::copy(got.begin(), got.begin() + n, ref.begin());                                                     \
    auto pv = run(NAME, WPS, k_sha<WPS, HR, HS>);                                                             \
    size_t bad = 0;                                                                                           \
    for (size_t i = 0; i < n; ++i) bad += got[i] != ref[i];                                                   \
    const double wb = (double)wps_ * NBLK;                                                                    \
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"prod_ms\": %.4f, \"ms\": %.4f, "                   \
           "\"prod_cycles_per_wave_block\": %.1f, \"cycles_per_wave_block\": %.1f, \"speedup\": %.4f, "        \
           "\"mismatches\": %zu}\n",                                                                          \
           NAME, WPS, pr.first, pv.first, pr.first * 1e-3 * 2.4e9 / wb, pv.first * 1e-3 * 2.4e9 / wb,         \
           pr.first / pv.first, bad);                                                                         \
    fflush(stdout);                                                                                           \
  }
  for (int rep = 0; rep < 2; ++rep) {
    { const int wps_ = 8; RUNV(8, true, true, "H-heavy round + schedule") }
    { const int wps_ = 8; RUNV(8, true, false, "H-heavy round") }
    { const int wps_ = 8; RUNV(8, false, true, "H-heavy schedule") }
    { const int wps_ = 4; RUNV(4, true, true, "H-heavy round + schedule") }
    { const int wps_ = 2; RUNV(2, true, true, "H-heavy round + schedule") }
  }
  return 0;
}
