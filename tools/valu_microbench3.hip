// Integer-VALU microbenchmark, part 3 (gfx950): VGPR bank conflicts and the
// compiled SHA-256 compression loop with no memory traffic.
//
//  * v_add3_u32 / v_bitop3_b32 with the three sources in one VGPR bank
//    (reg % 4 equal) vs in three different banks (physical registers pinned
//    in the asm text).
//  * compress(): the production compression function (sha256_device.hpp) run
//    back to back on register-resident blocks at 1..8 waves/SIMD; reports
//    blocks/s and SIMD-cycles per block, i.e. the ceiling of the kernel's
//    instruction stream before any load, tail or launch effect.
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/valu_microbench3 tools/valu_microbench3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 2048;

// 8 chains in v[32..63] with pinned registers. "diff": srcs in banks 0/1/2 offsets; "same": all one bank.
#define BODY_DIFF(OP)                                                        \
  asm volatile(OP " v32, v32, v33, v34\n" OP " v36, v36, v37, v38\n"         \
               OP " v40, v40, v41, v42\n" OP " v44, v44, v45, v46\n"         \
               OP " v48, v48, v49, v50\n" OP " v52, v52, v53, v54\n"         \
               OP " v56, v56, v57, v58\n" OP " v60, v60, v61, v62\n"         \
               ::: "v32","v33","v34","v36","v37","v38","v40","v41","v42","v44","v45","v46", \
                   "v48","v49","v50","v52","v53","v54","v56","v57","v58","v60","v61","v62");
#define BODY_SAME(OP)                                                        \
  asm volatile(OP " v32, v32, v36, v40\n" OP " v33, v33, v37, v41\n"         \
               OP " v34, v34, v38, v42\n" OP " v35, v35, v39, v43\n"         \
               OP " v48, v48, v52, v56\n" OP " v49, v49, v53, v57\n"         \
               OP " v50, v50, v54, v58\n" OP " v51, v51, v55, v59\n"         \
               ::: "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43", \
                   "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59");

#define KBANK(name, B)                                                \
  __global__ void name(unsigned* out) {                               \
    for (int i = 0; i < ITERS; ++i) { B B B B }                       \
    unsigned x;                                                       \
    asm volatile("v_mov_b32 %0, v32" : "=v"(x));                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                   \
  }

KBANK(k_add3_diff, BODY_DIFF("v_add3_u32"))
KBANK(k_add3_same, BODY_SAME("v_add3_u32"))
KBANK(k_bop3_diff, BODY_DIFF("v_bitop3_b32"))
KBANK(k_bop3_same, BODY_SAME("v_bitop3_b32"))

// The production compression on register-resident data.
constexpr int NBLK = 64;
__global__ __launch_bounds__(256, 8) void k_compress(unsigned* out, unsigned seed) {
  msha::State s;
  msha::state_init(s);
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = seed * (j + 1) + threadIdx.x;
  for (int b = 0; b < NBLK; ++b) {
    msha::compress(s, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] ^= s.h[j & 7] + j;   // next block depends on the state
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
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch();
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
  struct { const char* name; void (*f)(unsigned*); } ks[] = {
    {"add3 srcs 3 banks", k_add3_diff}, {"add3 srcs 1 bank", k_add3_same},
    {"bitop3 srcs 3 banks", k_bop3_diff}, {"bitop3 srcs 1 bank", k_bop3_same}};
  for (auto& k : ks) {
    for (int wps : {2, 8}) {
      float ms = timeit([&] { hipLaunchKernelGGL(k.f, dim3(cus * wps), dim3(256), 0, 0, out); });
      double instr = (double)ITERS * 4 * 8;
      double cyc = ms * 1e-3 * 2.4e9 / (instr * wps);   // per SIMD: wps waves x instr
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
             k.name, wps, ms, cyc);
    }
  }
  for (int wps : {1, 2, 4, 8}) {
    float ms = timeit([&] { hipLaunchKernelGGL(k_compress, dim3(cus * wps), dim3(256), 0, 0, out, 7u); });
    double blocks = (double)cus * wps * 256 * NBLK;
    double cyc_per_wave_block = ms * 1e-3 * 2.4e9 / (wps * NBLK);
    printf("{\"op\": \"compress() register-resident\", \"waves_per_simd\": %d, \"ms\": %.4f, "
           "\"Gblocks_per_s\": %.3f, \"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
           wps, ms, blocks / (ms * 1e-3) / 1e9, cyc_per_wave_block);
  }
  return 0;
}
