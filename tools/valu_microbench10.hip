// Integer-VALU microbenchmark, part 10 (gfx950): does phase-aligning the waves
// that share a SIMD help the SHA-256 mix? Part 8: full-rate ops reach 2 cycles
// only when two waves have one ready together; in the production kernel the 8
// waves of a SIMD (from 8 different workgroups) drift apart. Here the waves of
// one workgroup (512 or 1024 threads: 2 or 4 per SIMD) re-align with
// s_barrier every R rounds, on register-resident data (part 4's harness).
// Every variant is timed after >= 500 ms of warm load (settled clocks); the
// 256-thread, no-barrier row is the production form's ceiling (bench.py's
// ISA_MIX_CEILING_TOPS).
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench10 tools/valu_microbench10.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int NBLK = 64;

#define SYNC(R, i) if (R > 0 && ((i) % (R)) == 0) __builtin_amdgcn_s_barrier();
#define SROUND(a, b, c, d, e, f, g, h, i, W) \
  SYNC(R, i)                                 \
  MSHA_ROUND(a, b, c, d, e, f, g, h, K[i], W(i))
#define SR8(i, W)                                       \
  SROUND(a, b, c, d, e, f, g, h, (i) + 0, W)            \
  SROUND(h, a, b, c, d, e, f, g, (i) + 1, W)            \
  SROUND(g, h, a, b, c, d, e, f, (i) + 2, W)            \
  SROUND(f, g, h, a, b, c, d, e, (i) + 3, W)            \
  SROUND(e, f, g, h, a, b, c, d, (i) + 4, W)            \
  SROUND(d, e, f, g, h, a, b, c, (i) + 5, W)            \
  SROUND(c, d, e, f, g, h, a, b, (i) + 6, W)            \
  SROUND(b, c, d, e, f, g, h, a, (i) + 7, W)

template <int R>
__device__ __forceinline__ void compress_sync(State& s, uint32_t (&w)[16]) {
  constexpr uint32_t K[64] = {MSHA_K_TABLE};
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
  uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#define WD(i) w[(i) & 15]
#define WS(i) MSHA_SCHED(w, i)
  SR8(0, WD) SR8(8, WD) SR8(16, WS) SR8(24, WS) SR8(32, WS) SR8(40, WS) SR8(48, WS) SR8(56, WS)
#undef WD
#undef WS
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

template <int TPB, int R>
__global__ __launch_bounds__(TPB, 8) void k_sync(unsigned* out, unsigned seed) {
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x;
  for (int blk = 0; blk < NBLK; ++blk) {
    compress_sync<R>(s, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] ^= s.h[j & 7] + j;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= s.h[j];
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
    // clocks settle after ~100 ms of load: keep the GPU busy for >= 500 ms first
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 500.f;) {
      for (int i = 0; i < 20; ++i) launch();
      CHECK(hipEventRecord(w1));
      CHECK(hipEventSynchronize(w1));
      CHECK(hipEventElapsedTime(&el, w0, w1));
    }
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
  // 8 waves per SIMD in every variant: 2048 threads per CU
  auto report = [&](const char* name, int tpb, int rounds, float ms) {
    double blocks = (double)cus * 2048 * NBLK;
    printf("{\"kernel\": \"%s\", \"threads_per_wg\": %d, \"barrier_every_rounds\": %d, \"ms\": %.4f, "
           "\"Gblocks_per_s\": %.3f, \"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
           name, tpb, rounds, ms, blocks / (ms * 1e-3) / 1e9, ms * 1e-3 * 2.4e9 / (8 * NBLK));
  };
#define RUN(TPB, R) report("compress", TPB, R, timeit([&] { hipLaunchKernelGGL((k_sync<TPB, R>), dim3(cus * 2048 / TPB), dim3(TPB), 0, 0, out, 7u); }))
  for (int rep = 0; rep < 2; ++rep) {
    RUN(256, 0);
    RUN(512, 0);
    RUN(1024, 0);
    RUN(512, 8);
    RUN(512, 1);
    RUN(1024, 8);
    RUN(1024, 2);
    RUN(1024, 1);
    RUN(256, 8);
  }
  return 0;
}
