// Integer-VALU microbenchmark, part 12 (gfx950): dependent-issue latency of a
// LONE wave (one wave per SIMD, c4's regime). c4's pipelined kernel issues a
// VALU instruction every 4.32 SIMD cycles where a lone wave's independent
// stream costs 4 (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'). If an
// instruction that reads the result of the one just before it waits longer
// than that, the round's back-to-back dependent pairs (alignbit -> bitop3,
// bitop3 -> add3, add3 -> add3) are where the 8 % goes, and a hand-interleaved
// round order would win it back. Chains of 1, 2, 3 and 4 interleaved dependent
// streams per body, for a half-rate (v_alignbit) and a full-rate (v_add) op,
// plus the mixed alignbit -> bitop3 pair, each at 1 and 2 waves per SIMD,
// timed after >= 500 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench12 tools/valu_microbench12.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 8192;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","vcc"

// 8 instructions per body in every variant
#define AL(d) "v_alignbit_b32 " d ", " d ", " d ", 7\n"
#define AD(d) "v_add_u32_e32 " d ", " d ", v33\n"
#define B_AL_IND "v_alignbit_b32 v48, v32, v32, 7\n v_alignbit_b32 v49, v34, v34, 7\n v_alignbit_b32 v50, v36, v36, 7\n" \
                 "v_alignbit_b32 v51, v38, v38, 7\n v_alignbit_b32 v52, v40, v40, 7\n v_alignbit_b32 v53, v42, v42, 7\n" \
                 "v_alignbit_b32 v54, v44, v44, 7\n v_alignbit_b32 v55, v46, v46, 7\n"
#define B_AL_DEP1 AL("v48") AL("v48") AL("v48") AL("v48") AL("v48") AL("v48") AL("v48") AL("v48")
#define B_AL_DEP2 AL("v48") AL("v49") AL("v48") AL("v49") AL("v48") AL("v49") AL("v48") AL("v49")
#define B_AL_DEP3 AL("v48") AL("v49") AL("v50") AL("v48") AL("v49") AL("v50") AL("v48") AL("v49")
#define B_AL_DEP4 AL("v48") AL("v49") AL("v50") AL("v51") AL("v48") AL("v49") AL("v50") AL("v51")
#define B_AD_IND "v_add_u32_e32 v48, v32, v33\n v_add_u32_e32 v49, v34, v35\n v_add_u32_e32 v50, v36, v37\n" \
                 "v_add_u32_e32 v51, v38, v39\n v_add_u32_e32 v52, v40, v41\n v_add_u32_e32 v53, v42, v43\n" \
                 "v_add_u32_e32 v54, v44, v45\n v_add_u32_e32 v55, v46, v47\n"
#define B_AD_DEP1 AD("v48") AD("v48") AD("v48") AD("v48") AD("v48") AD("v48") AD("v48") AD("v48")
#define B_AD_DEP2 AD("v48") AD("v49") AD("v48") AD("v49") AD("v48") AD("v49") AD("v48") AD("v49")
#define B_AD_DEP4 AD("v48") AD("v49") AD("v50") AD("v51") AD("v48") AD("v49") AD("v50") AD("v51")
// alignbit -> bitop3 that reads it, back to back (the Sigma pattern) vs separated by one independent op
#define B_PAIR_ADJ "v_alignbit_b32 v48, v32, v32, 6\n v_bitop3_b32 v49, v48, v34, v35 bitop3:0x96\n" \
                   "v_alignbit_b32 v50, v36, v36, 6\n v_bitop3_b32 v51, v50, v38, v39 bitop3:0x96\n" \
                   "v_alignbit_b32 v52, v40, v40, 6\n v_bitop3_b32 v53, v52, v42, v43 bitop3:0x96\n" \
                   "v_alignbit_b32 v54, v44, v44, 6\n v_bitop3_b32 v55, v54, v46, v47 bitop3:0x96\n"
#define B_PAIR_SEP "v_alignbit_b32 v48, v32, v32, 6\n v_alignbit_b32 v50, v36, v36, 6\n" \
                   "v_bitop3_b32 v49, v48, v34, v35 bitop3:0x96\n v_alignbit_b32 v52, v40, v40, 6\n" \
                   "v_bitop3_b32 v51, v50, v38, v39 bitop3:0x96\n v_alignbit_b32 v54, v44, v44, 6\n" \
                   "v_bitop3_b32 v53, v52, v42, v43 bitop3:0x96\n v_bitop3_b32 v55, v54, v46, v47 bitop3:0x96\n"

#define KERN(name, BODY)                                                                            \
  __global__ __launch_bounds__(256) void name(unsigned* out, unsigned seed) {                       \
    unsigned x = seed ^ threadIdx.x;                                                                \
    asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n" \
                 "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n" \
                 "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n" \
                 "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 13\n" \
                 "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n" \
                 :: "v"(x) : CLOB);                                                                 \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY BODY BODY BODY ::: CLOB);                     \
    unsigned y;                                                                                     \
    asm volatile("v_xor_b32 %0, v48, v49" : "=v"(y));                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;                                                 \
  }

KERN(k_al_ind, B_AL_IND)
KERN(k_al_dep1, B_AL_DEP1)
KERN(k_al_dep2, B_AL_DEP2)
KERN(k_al_dep3, B_AL_DEP3)
KERN(k_al_dep4, B_AL_DEP4)
KERN(k_ad_ind, B_AD_IND)
KERN(k_ad_dep1, B_AD_DEP1)
KERN(k_ad_dep2, B_AD_DEP2)
KERN(k_ad_dep4, B_AD_DEP4)
KERN(k_pair_adj, B_PAIR_ADJ)
KERN(k_pair_sep, B_PAIR_SEP)

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(unsigned*, unsigned); } ks[] = {
    {"alignbit independent", k_al_ind}, {"alignbit 1 dependent chain", k_al_dep1},
    {"alignbit 2 interleaved chains", k_al_dep2}, {"alignbit 3 interleaved chains", k_al_dep3},
    {"alignbit 4 interleaved chains", k_al_dep4}, {"add independent", k_ad_ind},
    {"add 1 dependent chain", k_ad_dep1}, {"add 2 interleaved chains", k_ad_dep2},
    {"add 4 interleaved chains", k_ad_dep4}, {"alignbit->bitop3 adjacent pairs", k_pair_adj},
    {"alignbit->bitop3 pairs, one op apart", k_pair_sep}};
  // warm the clocks (>= 500 ms of load)
  {
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 500.f;) {
      for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_al_ind, dim3(cus * 8), dim3(256), 0, 0, out, 1u);
      CHECK(hipEventRecord(w1));
      CHECK(hipEventSynchronize(w1));
      CHECK(hipEventElapsedTime(&el, w0, w1));
    }
  }
  for (int rep = 0; rep < 2; ++rep)
    for (int wps : {1, 2})
      for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(cus * wps), dim3(256), 0, 0, out, 1u);
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
          CHECK(hipEventRecord(e0));
          hipLaunchKernelGGL(k.f, dim3(cus * wps), dim3(256), 0, 0, out, 3u + r);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        const double instr = (double)ITERS * 4 * 8 * wps;  // per SIMD
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_instr_at_2.4GHz\": %.3f}\n",
               k.name, wps, best, best * 1e-3 * 2.4e9 / instr);
        fflush(stdout);
      }
  return 0;
}
