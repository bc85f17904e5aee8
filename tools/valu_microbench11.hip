// Integer-VALU microbenchmark, part 11 (gfx950): does a wave whose exec mask
// holds only half (or a quarter) of its 64 lanes issue its VALU instructions
// faster than a full wave? If the SIMD-32 skips an all-zero 32-lane pass, two
// half-waves per SIMD cost what one full wave costs while giving the SIMD two
// instruction streams to interleave -- the lone-wave regime (c4: one wave of
// messages per SIMD, 4.32 SIMD cycles per instruction vs 4.04 at 8 waves)
// could then run at the multi-wave rate. Register-resident SHA-256 blocks
// (part 4's harness), timed after >= 500 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench11 tools/valu_microbench11.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace msha;
constexpr int NBLK = 256;

// ACTIVE lanes of each wave hash; the other lanes leave at once. PATTERN 0:
// lanes [0, ACTIVE); 1: every (64/ACTIVE)-th lane (spread over both halves).
template <int ACTIVE, int PATTERN>
__global__ __launch_bounds__(256, 8) void k_masked(unsigned* out, unsigned seed) {
  const unsigned lane = threadIdx.x & 63;
  const bool on = PATTERN == 0 ? lane < ACTIVE : (lane % (64 / ACTIVE)) == 0;
  if (!on) return;
  State s;
  state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x + blockIdx.x;
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

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 500.f;) {
      for (int i = 0; i < 4; ++i) launch();
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
  auto report = [&](int waves_per_simd, int active, int pattern, float ms) {
    const double lane_blocks = (double)cus * 4 * waves_per_simd * active * NBLK;
    const double wave_blocks_per_simd = (double)waves_per_simd * NBLK;
    printf("{\"waves_per_simd\": %d, \"active_lanes\": %d, \"pattern\": \"%s\", \"ms\": %.4f, "
           "\"G_lane_blocks_per_s\": %.3f, \"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
           waves_per_simd, active, pattern ? "strided" : "low", ms, lane_blocks / (ms * 1e-3) / 1e9,
           ms * 1e-3 * 2.4e9 / wave_blocks_per_simd);
    fflush(stdout);
  };
#define RUN(WPS, A, P) \
  report(WPS, A, P, timeit([&] { hipLaunchKernelGGL((k_masked<A, P>), dim3(cus * WPS), dim3(256), 0, 0, out, 7u); }))
  for (int rep = 0; rep < 2; ++rep) {
    RUN(1, 64, 0);
    RUN(2, 64, 0);
    RUN(8, 64, 0);
    RUN(2, 32, 0);
    RUN(2, 32, 1);
    RUN(4, 16, 0);
    RUN(4, 16, 1);
    RUN(1, 32, 0);
    RUN(8, 32, 0);
  }
  return 0;
}
