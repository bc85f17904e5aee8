// Integer-VALU microbenchmark, part 7 (gfx950): is a SHA-256 round cheaper with
// its three v_add3_u32 (half rate, 2 additions each) split into six v_add_u32
// (full rate)? Same dependent-round harness as part 5.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench7 tools/valu_microbench7.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 1024;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47"

#define DEP_ROUND_ADD3(a,b,c,d,e,f,g,h) \
  "v_alignbit_b32 v40, " e ", " e ", 6\n v_alignbit_b32 v41, " e ", " e ", 11\n v_alignbit_b32 v42, " e ", " e ", 25\n" \
  "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v41, " e ", " f ", " g " bitop3:0xca\n" \
  "v_add3_u32 v43, " h ", v44, v41\n v_add3_u32 v43, v43, v40, v45\n" \
  "v_alignbit_b32 v40, " a ", " a ", 2\n v_alignbit_b32 v41, " a ", " a ", 13\n v_alignbit_b32 v42, " a ", " a ", 22\n" \
  "v_add_u32 " d ", v43, " d "\n v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n" \
  "v_bitop3_b32 v41, " a ", " b ", " c " bitop3:0xe8\n v_add3_u32 " h ", v40, v41, v43\n"
#define DEP_ROUND_ADD(a,b,c,d,e,f,g,h) \
  "v_alignbit_b32 v40, " e ", " e ", 6\n v_alignbit_b32 v41, " e ", " e ", 11\n v_alignbit_b32 v42, " e ", " e ", 25\n" \
  "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v41, " e ", " f ", " g " bitop3:0xca\n" \
  "v_add_u32 v43, " h ", v44\n v_add_u32 v43, v43, v41\n v_add_u32 v43, v43, v40\n v_add_u32 v43, v43, v45\n" \
  "v_alignbit_b32 v40, " a ", " a ", 2\n v_alignbit_b32 v41, " a ", " a ", 13\n v_alignbit_b32 v42, " a ", " a ", 22\n" \
  "v_add_u32 " d ", v43, " d "\n v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n" \
  "v_bitop3_b32 v41, " a ", " b ", " c " bitop3:0xe8\n v_add_u32 " h ", v40, v41\n v_add_u32 " h ", " h ", v43\n"
#define R8(R) \
  R("v32","v33","v34","v35","v36","v37","v38","v39") R("v39","v32","v33","v34","v35","v36","v37","v38") \
  R("v38","v39","v32","v33","v34","v35","v36","v37") R("v37","v38","v39","v32","v33","v34","v35","v36") \
  R("v36","v37","v38","v39","v32","v33","v34","v35") R("v35","v36","v37","v38","v39","v32","v33","v34") \
  R("v34","v35","v36","v37","v38","v39","v32","v33") R("v33","v34","v35","v36","v37","v38","v39","v32")

#define KERN(name, BODY)                                                    \
  __global__ void name(unsigned* out, unsigned seed) {                      \
    unsigned x = seed ^ threadIdx.x;                                        \
    asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n" \
                 "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n" \
                 "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n" :: "v"(x) : CLOB); \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY ::: CLOB);            \
    unsigned y;                                                             \
    asm volatile("v_xor_b32 %0, v32, v40" : "=v"(y));                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;                         \
  }
KERN(k_add3, R8(DEP_ROUND_ADD3))
KERN(k_add, R8(DEP_ROUND_ADD))

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(unsigned*, unsigned); int instrs; } ks[] = {
    {"round with 3 add3 + 1 add (14 instr)", k_add3, 14}, {"round with 8 add (18 instr)", k_add, 18}};
  for (int rep = 0; rep < 3; ++rep)
  for (auto& k : ks)
  for (int wps : {4, 8}) {
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
    double rounds = (double)ITERS * 8 * wps;
    printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_round_at_2.4GHz\": %.2f}\n",
           k.name, wps, best, best * 1e-3 * 2.4e9 / rounds);
  }
  return 0;
}
