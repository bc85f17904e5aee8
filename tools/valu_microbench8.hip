// Integer-VALU microbenchmark, part 8 (gfx950): which operand/encoding forms
// are full rate? Same harness as part 6 (8 independent ops per body, 8
// waves/SIMD, register-resident). Hypotheses tested: a VGPR (not inline)
// rotate amount for v_alignbit_b32; VOP3 (_e64) encodings of VOP2 ops; 3-source
// VOP3 integer ops (max3/med3/and_or/or3/xad); DPP-modified VOP2; v_bitop3 with a
// constant operand; carry-out adds.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench8 tools/valu_microbench8.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 2048;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","vcc"

#define R8(OP, TAIL) OP " v48, v32, v33" TAIL "\n" OP " v49, v34, v35" TAIL "\n" OP " v50, v36, v37" TAIL "\n" \
                     OP " v51, v38, v39" TAIL "\n" OP " v52, v40, v41" TAIL "\n" OP " v53, v42, v43" TAIL "\n" \
                     OP " v54, v44, v45" TAIL "\n" OP " v55, v46, v32" TAIL "\n"
#define B_ALIGN_VSHIFT R8("v_alignbit_b32", ", v47")
#define B_ALIGN_CONST  R8("v_alignbit_b32", ", 7")
#define B_ADD_E64      R8("v_add_u32_e64", "")
#define B_ADD_E32      R8("v_add_u32_e32", "")
#define B_XOR_E64      R8("v_xor_b32_e64", "")
#define B_LSHR_VV      R8("v_lshrrev_b32_e32", "")
#define B_ADD3         R8("v_add3_u32", ", v47")
#define B_MAX3         R8("v_max3_u32", ", v47")
#define B_ANDOR        R8("v_and_or_b32", ", v47")
#define B_OR3          R8("v_or3_b32", ", v47")
#define B_BITOP3_VVV   R8("v_bitop3_b32", ", v47 bitop3:0x96")
#define B_BITOP3_CONST R8("v_bitop3_b32", ", 7 bitop3:0x96")
#define B_ADDCO        R8("v_add_co_u32_e32", "")
#define B_ADD_DPP      R8("v_add_u32_dpp", " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
#define B_SUB          R8("v_sub_u32_e32", "")
#define B_ADD_SGPR     "v_add_u32_e32 v48, s4, v32\n v_add_u32_e32 v49, s4, v34\n v_add_u32_e32 v50, s4, v36\n" \
                       "v_add_u32_e32 v51, s4, v38\n v_add_u32_e32 v52, s4, v40\n v_add_u32_e32 v53, s4, v42\n" \
                       "v_add_u32_e32 v54, s4, v44\n v_add_u32_e32 v55, s4, v46\n"
#define B_ADD_LIT      "v_add_u32_e32 v48, 0x428a2f98, v32\n v_add_u32_e32 v49, 0x71374491, v34\n" \
                       "v_add_u32_e32 v50, 0xb5c0fbcf, v36\n v_add_u32_e32 v51, 0xe9b5dba5, v38\n" \
                       "v_add_u32_e32 v52, 0x3956c25b, v40\n v_add_u32_e32 v53, 0x59f111f1, v42\n" \
                       "v_add_u32_e32 v54, 0x923f82a4, v44\n v_add_u32_e32 v55, 0xab1c5ed5, v46\n"
// mixes (per body: 8 ops)
#define B_MIX_AB_ADD   "v_alignbit_b32 v48, v32, v32, 6\n v_add_u32_e32 v49, v34, v35\n v_alignbit_b32 v50, v36, v36, 11\n" \
                       "v_add_u32_e32 v51, v38, v39\n v_alignbit_b32 v52, v40, v40, 25\n v_add_u32_e32 v53, v42, v43\n" \
                       "v_alignbit_b32 v54, v44, v44, 2\n v_add_u32_e32 v55, v46, v47\n"
#define B_MIX_AB_BOP   "v_alignbit_b32 v48, v32, v32, 6\n v_bitop3_b32 v49, v34, v35, v36 bitop3:0x96\n v_alignbit_b32 v50, v36, v36, 11\n" \
                       "v_bitop3_b32 v51, v38, v39, v40 bitop3:0x96\n v_alignbit_b32 v52, v40, v40, 25\n v_bitop3_b32 v53, v42, v43, v44 bitop3:0x96\n" \
                       "v_alignbit_b32 v54, v44, v44, 2\n v_bitop3_b32 v55, v46, v47, v32 bitop3:0x96\n"
#define B_MIX_4AB_4ADD "v_alignbit_b32 v48, v32, v32, 6\n v_alignbit_b32 v50, v36, v36, 11\n v_alignbit_b32 v52, v40, v40, 25\n" \
                       "v_alignbit_b32 v54, v44, v44, 2\n v_add_u32_e32 v49, v34, v35\n v_add_u32_e32 v51, v38, v39\n" \
                       "v_add_u32_e32 v53, v42, v43\n v_add_u32_e32 v55, v46, v47\n"

#define KERN(name, BODY)                                                    \
  __global__ void name(unsigned* out, unsigned seed) {                      \
    unsigned x = seed ^ threadIdx.x;                                        \
    asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n" \
                 "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n" \
                 "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n" \
                 "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 13\n" \
                 "s_mov_b32 s4, 0x428a2f98\n" :: "v"(x) : CLOB, "s4");              \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY BODY BODY BODY ::: CLOB); \
    unsigned y;                                                             \
    asm volatile("v_xor_b32 %0, v48, v49" : "=v"(y));                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;                         \
  }

KERN(k_align_vshift, B_ALIGN_VSHIFT)
KERN(k_align_const, B_ALIGN_CONST)
KERN(k_add_e64, B_ADD_E64)
KERN(k_add_e32, B_ADD_E32)
KERN(k_xor_e64, B_XOR_E64)
KERN(k_lshr_vv, B_LSHR_VV)
KERN(k_add3, B_ADD3)
KERN(k_max3, B_MAX3)
KERN(k_andor, B_ANDOR)
KERN(k_or3, B_OR3)
KERN(k_bitop3_vvv, B_BITOP3_VVV)
KERN(k_bitop3_const, B_BITOP3_CONST)
KERN(k_addco, B_ADDCO)
KERN(k_add_dpp, B_ADD_DPP)
KERN(k_sub, B_SUB)
KERN(k_add_sgpr, B_ADD_SGPR)
KERN(k_add_lit, B_ADD_LIT)
KERN(k_mix_ab_add, B_MIX_AB_ADD)
KERN(k_mix_ab_bop, B_MIX_AB_BOP)
KERN(k_mix_4ab_4add, B_MIX_4AB_4ADD)

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(unsigned*, unsigned); } ks[] = {
    {"v_alignbit_b32 v,v,v,VGPR-shift", k_align_vshift}, {"v_alignbit_b32 v,v,v,const", k_align_const},
    {"v_add_u32_e64", k_add_e64}, {"v_add_u32_e32", k_add_e32}, {"v_xor_b32_e64", k_xor_e64},
    {"v_lshrrev_b32_e32 VGPR shift", k_lshr_vv}, {"v_add3_u32", k_add3}, {"v_max3_u32", k_max3},
    {"v_and_or_b32", k_andor}, {"v_or3_b32", k_or3}, {"v_bitop3_b32 vvv", k_bitop3_vvv},
    {"v_bitop3_b32 vv+inline-const", k_bitop3_const}, {"v_add_co_u32_e32", k_addco},
    {"v_add_u32_dpp quad_perm", k_add_dpp}, {"v_sub_u32_e32", k_sub}, {"v_add_u32_e32 SGPR", k_add_sgpr},
    {"v_add_u32_e32 literal", k_add_lit}, {"mix alignbit/add alternating", k_mix_ab_add},
    {"mix alignbit/bitop3 alternating", k_mix_ab_bop}, {"mix 4 alignbit then 4 add", k_mix_4ab_4add}};
  for (int rep = 0; rep < 2; ++rep)
  for (auto& k : ks) {
    const int wps = 8;
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
    double bodies = (double)ITERS * 4 * wps;  // per SIMD
    double cyc_body = best * 1e-3 * 2.4e9 / bodies;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_instr_at_2.4GHz\": %.3f}\n",
           k.name, wps, best, cyc_body / 8);
  }
  return 0;
}
