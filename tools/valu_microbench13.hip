// Integer-VALU microbenchmark, part 13 (gfx950): can two waves on ONE SIMD
// overlap instructions of different rate classes? Parts 8/12: a full-rate op
// (v_add, v_bitop3) costs ~2.3 SIMD cycles when two waves issue only full-rate
// ops, a half-rate op (v_alignbit, v_add3) ~4.3, but in a stream that mixes
// them every op costs ~4. If a wave issuing only half-rate ops and a wave
// issuing only full-rate ops on the same SIMD ran side by side (time ~ the
// longer of the two alone), a SHA-256 split by rate class across two waves
// could beat the mixed stream; if their times add, it cannot.
// One 512-thread workgroup per CU (two waves per SIMD); each wave's body is
// chosen by its SIMD slot so every SIMD holds one wave of each kind (checked:
// the kernel records each wave's HW_ID SIMD field). Timed after >= 500 ms of
// warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench13 tools/valu_microbench13.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","vcc"
#define B_H "v_alignbit_b32 v48, v32, v32, 7\n v_alignbit_b32 v49, v34, v34, 7\n v_alignbit_b32 v50, v36, v36, 7\n" \
            "v_alignbit_b32 v51, v38, v38, 7\n v_alignbit_b32 v52, v40, v40, 7\n v_alignbit_b32 v53, v42, v42, 7\n" \
            "v_alignbit_b32 v54, v44, v44, 7\n v_alignbit_b32 v55, v46, v46, 7\n"
#define B_F "v_add_u32_e32 v48, v32, v33\n v_add_u32_e32 v49, v34, v35\n v_add_u32_e32 v50, v36, v37\n" \
            "v_add_u32_e32 v51, v38, v39\n v_add_u32_e32 v52, v40, v41\n v_add_u32_e32 v53, v42, v43\n" \
            "v_add_u32_e32 v54, v44, v45\n v_add_u32_e32 v55, v46, v47\n"
#define B_B "v_bitop3_b32 v48, v32, v33, v34 bitop3:0x96\n v_bitop3_b32 v49, v34, v35, v36 bitop3:0x96\n" \
            "v_bitop3_b32 v50, v36, v37, v38 bitop3:0x96\n v_bitop3_b32 v51, v38, v39, v40 bitop3:0x96\n" \
            "v_bitop3_b32 v52, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v53, v42, v43, v44 bitop3:0x96\n" \
            "v_bitop3_b32 v54, v44, v45, v46 bitop3:0x96\n v_bitop3_b32 v55, v46, v47, v32 bitop3:0x96\n"
#define B_M "v_alignbit_b32 v48, v32, v32, 6\n v_add_u32_e32 v49, v34, v35\n v_alignbit_b32 v50, v36, v36, 11\n" \
            "v_add_u32_e32 v51, v38, v39\n v_alignbit_b32 v52, v40, v40, 25\n v_add_u32_e32 v53, v42, v43\n" \
            "v_alignbit_b32 v54, v44, v44, 2\n v_add_u32_e32 v55, v46, v47\n"

template <int KIND>
__device__ __forceinline__ void body() {
  for (int i = 0; i < ITERS; ++i) {
    if (KIND == 0) asm volatile(B_H B_H B_H B_H ::: CLOB);
    if (KIND == 1) asm volatile(B_F B_F B_F B_F ::: CLOB);
    if (KIND == 2) asm volatile(B_B B_B B_B B_B ::: CLOB);
    if (KIND == 3) asm volatile(B_M B_M B_M B_M ::: CLOB);
  }
}

// Waves whose first SIMD occupant (slot 0: waves 0-3 of the workgroup) runs
// KA, the second (waves 4-7) KB; KA or KB = -1 leaves that wave idle (exits).
template <int KA, int KB>
__global__ __launch_bounds__(512) void k_pair(unsigned* out, unsigned* ids, unsigned seed) {
  const unsigned wave = threadIdx.x >> 6;
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) ids[wave] = hw;
  const int kind = wave < 4 ? KA : KB;
  if (kind < 0) return;
  unsigned x = seed ^ threadIdx.x;
  asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n"
               "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n"
               "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
               "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 13\n" :: "v"(x) : CLOB);
  if (kind == 0) body<0>();
  if (kind == 1) body<1>();
  if (kind == 2) body<2>();
  if (kind == 3) body<3>();
  unsigned y;
  asm volatile("v_xor_b32 %0, v48, v49" : "=v"(y));
  out[blockIdx.x * blockDim.x + threadIdx.x] = y;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned *out, *ids;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 512));
  CHECK(hipMalloc(&ids, sizeof(unsigned) * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* a; const char* b; void (*f)(unsigned*, unsigned*, unsigned); } ks[] = {
    {"alignbit", "-", k_pair<0, -1>}, {"add", "-", k_pair<1, -1>}, {"bitop3", "-", k_pair<2, -1>},
    {"alignbit", "alignbit", k_pair<0, 0>}, {"add", "add", k_pair<1, 1>}, {"bitop3", "bitop3", k_pair<2, 2>},
    {"alignbit", "add", k_pair<0, 1>}, {"alignbit", "bitop3", k_pair<0, 2>},
    {"mix(alignbit/add)", "mix(alignbit/add)", k_pair<3, 3>}, {"mix(alignbit/add)", "-", k_pair<3, -1>}};
  {
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 500.f;) {
      for (int i = 0; i < 8; ++i) hipLaunchKernelGGL((k_pair<0, 0>), dim3(cus * 4), dim3(512), 0, 0, out, ids, 1u);
      CHECK(hipEventRecord(w1));
      CHECK(hipEventSynchronize(w1));
      CHECK(hipEventElapsedTime(&el, w0, w1));
    }
  }
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, ids, 1u);
      CHECK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, ids, 3u + r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      unsigned h[8];
      CHECK(hipMemcpy(h, ids, sizeof(h), hipMemcpyDeviceToHost));
      char simds[64];
      int o = 0;
      for (int w = 0; w < 8; ++w) o += snprintf(simds + o, sizeof(simds) - o, "%u", (h[w] >> 4) & 3);
      const double per_wave = (double)ITERS * 4 * 8;  // instructions per wave
      printf("{\"slot0\": \"%s\", \"slot1\": \"%s\", \"ms\": %.4f, \"simd_cycles_per_slot0_instr_at_2.4GHz\": %.3f, "
             "\"simd_of_waves_0_7\": \"%s\"}\n",
             k.a, k.b, best, best * 1e-3 * 2.4e9 / per_wave, simds);
      fflush(stdout);
    }
  return 0;
}
