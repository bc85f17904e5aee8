// Integer-VALU microbenchmark, part 6 (gfx950): candidate rotate forms.
// SHA-256 spends ~55% of its VALU cycles in v_alignbit_b32 rotates, which are
// half-rate. Are any other ways to rotate full-rate? Measured per opcode at
// 8 waves/SIMD with 8 independent chains (same harness as part 1):
//   v_lshrrev_b64 / v_lshlrev_b64 (64-bit shift of a duplicated pair gives a
//   32-bit rotate in its low word), v_pk_mov_b32 (duplicate into a pair),
//   v_alignbyte_b32, v_bfe_u32, SDWA VOP2 (word selects), v_pk_lshrrev_b16,
//   v_lshl_add_u64, v_mov_b32, and the 64-bit-shift rotate as used in a
//   Sigma function (dup + 3 shifts + bitop3) vs the alignbit form.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench6 tools/valu_microbench6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 2048;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"

// 8 independent ops per body; sources v32..v47 (pairs at even regs), dests v48..v63
#define B_LSHR64 "v_lshrrev_b64 v[48:49], 6, v[32:33]\n v_lshrrev_b64 v[50:51], 11, v[34:35]\n" \
                 "v_lshrrev_b64 v[52:53], 25, v[36:37]\n v_lshrrev_b64 v[54:55], 2, v[38:39]\n" \
                 "v_lshrrev_b64 v[56:57], 13, v[40:41]\n v_lshrrev_b64 v[58:59], 22, v[42:43]\n" \
                 "v_lshrrev_b64 v[60:61], 7, v[44:45]\n v_lshrrev_b64 v[62:63], 18, v[46:47]\n"
#define B_LSHL64 "v_lshlrev_b64 v[48:49], 6, v[32:33]\n v_lshlrev_b64 v[50:51], 11, v[34:35]\n" \
                 "v_lshlrev_b64 v[52:53], 25, v[36:37]\n v_lshlrev_b64 v[54:55], 2, v[38:39]\n" \
                 "v_lshlrev_b64 v[56:57], 13, v[40:41]\n v_lshlrev_b64 v[58:59], 22, v[42:43]\n" \
                 "v_lshlrev_b64 v[60:61], 7, v[44:45]\n v_lshlrev_b64 v[62:63], 18, v[46:47]\n"
#define B_PKMOV  "v_pk_mov_b32 v[48:49], v[32:33], v[32:33] op_sel:[0,0]\n v_pk_mov_b32 v[50:51], v[34:35], v[34:35] op_sel:[0,0]\n" \
                 "v_pk_mov_b32 v[52:53], v[36:37], v[36:37] op_sel:[0,0]\n v_pk_mov_b32 v[54:55], v[38:39], v[38:39] op_sel:[0,0]\n" \
                 "v_pk_mov_b32 v[56:57], v[40:41], v[40:41] op_sel:[0,0]\n v_pk_mov_b32 v[58:59], v[42:43], v[42:43] op_sel:[0,0]\n" \
                 "v_pk_mov_b32 v[60:61], v[44:45], v[44:45] op_sel:[0,0]\n v_pk_mov_b32 v[62:63], v[46:47], v[46:47] op_sel:[0,0]\n"
#define B_MOV    "v_mov_b32 v48, v32\n v_mov_b32 v49, v33\n v_mov_b32 v50, v34\n v_mov_b32 v51, v35\n" \
                 "v_mov_b32 v52, v36\n v_mov_b32 v53, v37\n v_mov_b32 v54, v38\n v_mov_b32 v55, v39\n"
#define B_ALBYTE "v_alignbyte_b32 v48, v32, v33, 1\n v_alignbyte_b32 v49, v34, v35, 2\n" \
                 "v_alignbyte_b32 v50, v36, v37, 3\n v_alignbyte_b32 v51, v38, v39, 1\n" \
                 "v_alignbyte_b32 v52, v40, v41, 2\n v_alignbyte_b32 v53, v42, v43, 3\n" \
                 "v_alignbyte_b32 v54, v44, v45, 1\n v_alignbyte_b32 v55, v46, v47, 2\n"
#define B_BFE    "v_bfe_u32 v48, v32, 6, 26\n v_bfe_u32 v49, v33, 6, 26\n v_bfe_u32 v50, v34, 6, 26\n v_bfe_u32 v51, v35, 6, 26\n" \
                 "v_bfe_u32 v52, v36, 6, 26\n v_bfe_u32 v53, v37, 6, 26\n v_bfe_u32 v54, v38, 6, 26\n v_bfe_u32 v55, v39, 6, 26\n"
#define B_SDWA   "v_xor_b32_sdwa v48, v32, v33 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v49, v34, v35 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v50, v36, v37 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v51, v38, v39 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v52, v40, v41 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v53, v42, v43 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v54, v44, v45 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
                 "v_xor_b32_sdwa v55, v46, v47 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
#define B_PKSHR  "v_pk_lshrrev_b16 v48, 6, v32\n v_pk_lshrrev_b16 v49, 6, v33\n v_pk_lshrrev_b16 v50, 6, v34\n v_pk_lshrrev_b16 v51, 6, v35\n" \
                 "v_pk_lshrrev_b16 v52, 6, v36\n v_pk_lshrrev_b16 v53, 6, v37\n v_pk_lshrrev_b16 v54, 6, v38\n v_pk_lshrrev_b16 v55, 6, v39\n"
#define B_LSHLADD64 "v_lshl_add_u64 v[48:49], v[32:33], 0, v[34:35]\n v_lshl_add_u64 v[50:51], v[36:37], 0, v[38:39]\n" \
                 "v_lshl_add_u64 v[52:53], v[40:41], 0, v[42:43]\n v_lshl_add_u64 v[54:55], v[44:45], 0, v[46:47]\n" \
                 "v_lshl_add_u64 v[56:57], v[32:33], 0, v[36:37]\n v_lshl_add_u64 v[58:59], v[34:35], 0, v[38:39]\n" \
                 "v_lshl_add_u64 v[60:61], v[40:41], 0, v[44:45]\n v_lshl_add_u64 v[62:63], v[42:43], 0, v[46:47]\n"
#define B_ALIGNBIT "v_alignbit_b32 v48, v32, v32, 6\n v_alignbit_b32 v49, v33, v33, 11\n v_alignbit_b32 v50, v34, v34, 25\n" \
                 "v_alignbit_b32 v51, v35, v35, 2\n v_alignbit_b32 v52, v36, v36, 13\n v_alignbit_b32 v53, v37, v37, 22\n" \
                 "v_alignbit_b32 v54, v38, v38, 7\n v_alignbit_b32 v55, v39, v39, 18\n"
// Sigma forms (2 independent Sigmas per body): alignbit form = 3 alignbit + bitop3;
// 64-bit form = pk_mov dup + 3 lshrrev_b64 + bitop3 on the low words
#define SIG_AB(x, d) "v_alignbit_b32 v56, " x ", " x ", 6\n v_alignbit_b32 v57, " x ", " x ", 11\n" \
                     "v_alignbit_b32 v58, " x ", " x ", 25\n v_bitop3_b32 " d ", v56, v57, v58 bitop3:0x96\n"
#define SIG_64(x, d) "v_pk_mov_b32 v[40:41], " x ", " x " op_sel:[0,0]\n" \
                     "v_lshrrev_b64 v[42:43], 6, v[40:41]\n v_lshrrev_b64 v[44:45], 11, v[40:41]\n" \
                     "v_lshrrev_b64 v[46:47], 25, v[40:41]\n v_bitop3_b32 " d ", v42, v44, v46 bitop3:0x96\n"
#define B_SIGAB  SIG_AB("v32", "v48") SIG_AB("v33", "v49") SIG_AB("v34", "v50") SIG_AB("v35", "v51")
#define B_SIG64  SIG_64("v[32:33]", "v48") SIG_64("v[34:35]", "v49") SIG_64("v[36:37]", "v50") SIG_64("v[38:39]", "v51")

#define KERN(name, BODY)                                                    \
  __global__ void name(unsigned* out, unsigned seed) {                      \
    unsigned x = seed ^ threadIdx.x;                                        \
    asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n" \
                 "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n" \
                 "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n" \
                 "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0\n" :: "v"(x) : CLOB); \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY BODY BODY BODY ::: CLOB); \
    unsigned y;                                                             \
    asm volatile("v_xor_b32 %0, v48, v49" : "=v"(y));                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;                         \
  }

KERN(k_lshr64, B_LSHR64)
KERN(k_lshl64, B_LSHL64)
KERN(k_pkmov, B_PKMOV)
KERN(k_mov, B_MOV)
KERN(k_albyte, B_ALBYTE)
KERN(k_bfe, B_BFE)
KERN(k_sdwa, B_SDWA)
KERN(k_pkshr, B_PKSHR)
KERN(k_lshladd64, B_LSHLADD64)
KERN(k_alignbit, B_ALIGNBIT)
KERN(k_sigab, B_SIGAB)
KERN(k_sig64, B_SIG64)

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(unsigned*, unsigned); double instr_per_body; double sigmas_per_body; } ks[] = {
    {"v_lshrrev_b64", k_lshr64, 8, 0}, {"v_lshlrev_b64", k_lshl64, 8, 0}, {"v_pk_mov_b32", k_pkmov, 8, 0},
    {"v_mov_b32", k_mov, 8, 0}, {"v_alignbyte_b32", k_albyte, 8, 0}, {"v_bfe_u32", k_bfe, 8, 0},
    {"v_xor_b32_sdwa WORD_1", k_sdwa, 8, 0}, {"v_pk_lshrrev_b16", k_pkshr, 8, 0},
    {"v_lshl_add_u64", k_lshladd64, 8, 0}, {"v_alignbit_b32", k_alignbit, 8, 0},
    {"Sigma: 3 alignbit + bitop3", k_sigab, 16, 4}, {"Sigma: pk_mov + 3 lshrrev_b64 + bitop3", k_sig64, 20, 4}};
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
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_instr_at_2.4GHz\": %.3f, "
           "\"simd_cycles_per_sigma\": %.2f}\n", k.name, wps, best, cyc_body / k.instr_per_body,
           k.sigmas_per_body ? cyc_body / k.sigmas_per_body : 0.0);
  }
  return 0;
}
