// Integer-VALU microbenchmark, part 4 (gfx950): does instruction-level
// parallelism inside a wave beat occupancy for the SHA-256 stream?
//
//  k_compress1: the production compress() (one message per lane)
//  k_compress2: two independent messages per lane, rounds interleaved
//               (A-round, B-round, ...) so every dependent pair of
//               instructions has an independent one between them
// Both on register-resident data, at several waves/SIMD. Reports SIMD cycles
// per block (at the measured wall time x 2.4 GHz).
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench4 tools/valu_microbench4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int NBLK = 64;

#define R2(a, b, c, d, e, f, g, h, A, B, C, D, E, F, G, H, i, WA, WB) \
  MSHA_ROUND(a, b, c, d, e, f, g, h, K[i], WA)                      \
  MSHA_ROUND(A, B, C, D, E, F, G, H, K[i], WB)

#define R2x8(i, WA, WB)                                                                  \
  R2(a, b, c, d, e, f, g, h, A, B, C, D, E, F, G, H, (i) + 0, WA(wa, (i) + 0), WB(wb, (i) + 0)) \
  R2(h, a, b, c, d, e, f, g, H, A, B, C, D, E, F, G, (i) + 1, WA(wa, (i) + 1), WB(wb, (i) + 1)) \
  R2(g, h, a, b, c, d, e, f, G, H, A, B, C, D, E, F, (i) + 2, WA(wa, (i) + 2), WB(wb, (i) + 2)) \
  R2(f, g, h, a, b, c, d, e, F, G, H, A, B, C, D, E, (i) + 3, WA(wa, (i) + 3), WB(wb, (i) + 3)) \
  R2(e, f, g, h, a, b, c, d, E, F, G, H, A, B, C, D, (i) + 4, WA(wa, (i) + 4), WB(wb, (i) + 4)) \
  R2(d, e, f, g, h, a, b, c, D, E, F, G, H, A, B, C, (i) + 5, WA(wa, (i) + 5), WB(wb, (i) + 5)) \
  R2(c, d, e, f, g, h, a, b, C, D, E, F, G, H, A, B, (i) + 6, WA(wa, (i) + 6), WB(wb, (i) + 6)) \
  R2(b, c, d, e, f, g, h, a, B, C, D, E, F, G, H, A, (i) + 7, WA(wa, (i) + 7), WB(wb, (i) + 7))

#define WD(w, i) w[(i) & 15]
#define WS(w, i) MSHA_SCHED(w, i)

__device__ __forceinline__ void compress2(State& sa, uint32_t (&wa)[16], State& sb, uint32_t (&wb)[16]) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = sa.h[0], b = sa.h[1], c = sa.h[2], d = sa.h[3], e = sa.h[4], f = sa.h[5], g = sa.h[6], h = sa.h[7];
  uint32_t A = sb.h[0], B = sb.h[1], C = sb.h[2], D = sb.h[3], E = sb.h[4], F = sb.h[5], G = sb.h[6], H = sb.h[7];
  R2x8(0, WD, WD) R2x8(8, WD, WD)
  R2x8(16, WS, WS) R2x8(24, WS, WS) R2x8(32, WS, WS) R2x8(40, WS, WS) R2x8(48, WS, WS) R2x8(56, WS, WS)
  sa.h[0] += a; sa.h[1] += b; sa.h[2] += c; sa.h[3] += d; sa.h[4] += e; sa.h[5] += f; sa.h[6] += g; sa.h[7] += h;
  sb.h[0] += A; sb.h[1] += B; sb.h[2] += C; sb.h[3] += D; sb.h[4] += E; sb.h[5] += F; sb.h[6] += G; sb.h[7] += H;
}

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k_compress1(unsigned* out, unsigned seed) {
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x;
  for (int blk = 0; blk < NBLK; ++blk) {
    compress(s, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] ^= s.h[j & 7] + j;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= s.h[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k_compress2(unsigned* out, unsigned seed) {
  State sa, sb;
  state_init(sa);
  state_init(sb);
  uint32_t wa[16], wb[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) { wa[j] = seed * (j + 1) + threadIdx.x; wb[j] = seed * (j + 3) ^ threadIdx.x; }
  for (int blk = 0; blk < NBLK / 2; ++blk) {   // same total blocks per lane as k_compress1
    compress2(sa, wa, sb, wb);
#pragma unroll
    for (int j = 0; j < 16; ++j) { wa[j] ^= sa.h[j & 7] + j; wb[j] ^= sb.h[j & 7] + j; }
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= sa.h[j] ^ sb.h[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048 * 2));
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
  auto report = [&](const char* name, int wps, float ms, double blocks_per_lane) {
    double blocks = (double)cus * wps * 256 * blocks_per_lane;
    printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"Gblocks_per_s\": %.3f, "
           "\"simd_cycles_per_lane_block_x64_at_2.4GHz\": %.1f}\n",
           name, wps, ms, blocks / (ms * 1e-3) / 1e9, ms * 1e-3 * 2.4e9 / (wps * blocks_per_lane));
  };
  // k_compress1: each lane NBLK blocks; k_compress2: each lane 2 x NBLK/2 blocks
  report("compress1", 8, timeit([&] { hipLaunchKernelGGL(k_compress1<8>, dim3(cus * 8), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress1", 4, timeit([&] { hipLaunchKernelGGL(k_compress1<4>, dim3(cus * 4), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress2", 4, timeit([&] { hipLaunchKernelGGL(k_compress2<4>, dim3(cus * 4), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress2", 6, timeit([&] { hipLaunchKernelGGL(k_compress2<6>, dim3(cus * 6), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress2", 8, timeit([&] { hipLaunchKernelGGL(k_compress2<8>, dim3(cus * 8), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress2", 2, timeit([&] { hipLaunchKernelGGL(k_compress2<2>, dim3(cus * 2), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress1", 2, timeit([&] { hipLaunchKernelGGL(k_compress1<2>, dim3(cus * 2), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress1", 1, timeit([&] { hipLaunchKernelGGL(k_compress1<1>, dim3(cus * 1), dim3(256), 0, 0, out, 7u); }), NBLK);
  report("compress2", 1, timeit([&] { hipLaunchKernelGGL(k_compress2<1>, dim3(cus * 1), dim3(256), 0, 0, out, 7u); }), NBLK);
  return 0;
}
