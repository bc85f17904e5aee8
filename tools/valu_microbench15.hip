// Integer-VALU microbenchmark, part 15 (gfx950): what keeps two waves on one
// SIMD overlapping? Part 14: a wave of half-rate ops (H: v_alignbit) and a wave
// of full-rate ops (F: v_add) run side by side, but as soon as one wave on the
// SIMD mixes both classes every instruction costs ~4 cycles again. Here:
//   - the real H-class ops a SHA-256 round could be written in (v_alignbit,
//     v_xad_u32, v_bfi_b32, v_add3_u32 with an SGPR operand, v_perm_b32) and the
//     real F-class ops its message schedule could be written in (v_lshrrev /
//     v_lshlrev by a constant, v_bitop3, v_add with a literal): do they overlap?
//   - one H op in 32 F ops (and one F in 32 H): is a single stray op enough to
//     lose the overlap?
//   - LDS traffic (ds_write_b32 / ds_read_b32 + s_waitcnt) inside pure streams;
//   - 2 and 4 waves of each kind per SIMD.
// Independent operands. One or two 1,024-thread workgroups per CU; wave w runs
// the stream of its slot (w / 4) % 4. Timed after >= 500 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench15 tools/valu_microbench15.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","v56","vcc","s4","s5"
#define H(d, s) "v_alignbit_b32 v" #d ", v" #s ", v" #s ", 7\n"
#define F(d, s) "v_add_u32_e32 v" #d ", v" #s ", v33\n"
#define H8 H(48, 32) H(49, 34) H(50, 36) H(51, 38) H(52, 40) H(53, 42) H(54, 44) H(55, 46)
#define F8 F(48, 32) F(49, 34) F(50, 36) F(51, 38) F(52, 40) F(53, 42) F(54, 44) F(55, 46)
// SHA-round-like H-class ops
#define HX8 "v_alignbit_b32 v48, v32, v32, 6\n v_xad_u32 v49, v34, v35, 0\n v_bfi_b32 v50, v36, v37, v38\n" \
            "v_add3_u32 v51, v38, v39, s4\n v_alignbit_b32 v52, v40, v40, 11\n v_xad_u32 v53, v42, v43, v44\n" \
            "v_perm_b32 v54, v44, v44, s5\n v_add3_u32 v55, v46, v47, v32\n"
// schedule-like F-class ops
#define FX8 "v_lshrrev_b32_e32 v48, 7, v32\n v_lshlrev_b32_e32 v49, 25, v34\n v_bitop3_b32 v50, v36, v37, v38 bitop3:0x96\n" \
            "v_add_u32_e32 v51, 0x428a2f98, v38\n v_lshrrev_b32_e32 v52, 18, v40\n v_lshlrev_b32_e32 v53, 14, v42\n" \
            "v_bitop3_b32 v54, v44, v45, v46 bitop3:0xca\n v_add_u32_e32 v55, v46, v47\n"
#define LDSW "ds_write_b32 v56, v48\n"
#define LDSR "ds_read_b32 v49, v56\n"

enum { kH, kF, kHX, kFX, kF31H1, kH31F1, kHlds, kFlds, kN };
static const char* kNames[] = {"H", "F", "Hx", "Fx", "F31H1", "H31F1", "H+lds", "F+lds"};

template <int K>
__device__ __forceinline__ void run() {
  for (int i = 0; i < ITERS; ++i) {
    if (K == kH) asm volatile(H8 H8 H8 H8 ::: CLOB);
    if (K == kF) asm volatile(F8 F8 F8 F8 ::: CLOB);
    if (K == kHX) asm volatile(HX8 HX8 HX8 HX8 ::: CLOB);
    if (K == kFX) asm volatile(FX8 FX8 FX8 FX8 ::: CLOB);
    if (K == kF31H1) asm volatile(F8 F8 F8 F(48, 32) F(49, 34) F(50, 36) F(51, 38) F(52, 40) F(53, 42) F(54, 44) H(55, 46) ::: CLOB);
    if (K == kH31F1) asm volatile(H8 H8 H8 H(48, 32) H(49, 34) H(50, 36) H(51, 38) H(52, 40) H(53, 42) H(54, 44) F(55, 46) ::: CLOB);
    if (K == kHlds) asm volatile(H8 LDSW H8 H8 LDSR H8 "s_waitcnt lgkmcnt(0)\n" ::: CLOB, "memory");
    if (K == kFlds) asm volatile(F8 LDSW F8 F8 LDSR F8 "s_waitcnt lgkmcnt(0)\n" ::: CLOB, "memory");
  }
}

template <int K0, int K1, int K2, int K3>
__global__ __launch_bounds__(1024) void k_mix(unsigned* out, unsigned seed) {
  __shared__ unsigned lds[1024];
  const unsigned slot = ((threadIdx.x >> 6) / 4) % 4;
  const int kind = slot == 0 ? K0 : slot == 1 ? K1 : slot == 2 ? K2 : K3;
  lds[threadIdx.x] = seed;
  __syncthreads();
  if (kind < 0) return;
  unsigned x = seed ^ threadIdx.x;
  const unsigned addr = threadIdx.x * 4;  // byte offset in LDS: lds[] is the only LDS allocation (offset 0)
  asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n"
               "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n"
               "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
               "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 13\n"
               "v_mov_b32 v56, %1\n s_mov_b32 s4, 0x71374491\n s_mov_b32 s5, 0x00010203\n" :: "v"(x), "v"(addr) : CLOB);
  switch (kind) {
    case kH: run<kH>(); break;
    case kF: run<kF>(); break;
    case kHX: run<kHX>(); break;
    case kFX: run<kFX>(); break;
    case kF31H1: run<kF31H1>(); break;
    case kH31F1: run<kH31F1>(); break;
    case kHlds: run<kHlds>(); break;
    case kFlds: run<kFlds>(); break;
  }
  unsigned y;
  asm volatile("v_xor_b32 %0, v48, v49" : "=v"(y));
  out[blockIdx.x * blockDim.x + threadIdx.x] = y;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  constexpr int I = -1;
  struct Case { int k[4]; int wgs_per_cu; void (*f)(unsigned*, unsigned); };
#define C(a, b, c, d, w) Case{{a, b, c, d}, w, k_mix<a, b, c, d>}
  const Case cs[] = {
    C(kH, kF, I, I, 1), C(kHX, I, I, I, 1), C(kFX, I, I, I, 1),
    C(kHX, kHX, I, I, 1), C(kFX, kFX, I, I, 1), C(kHX, kFX, I, I, 1),
    C(kF31H1, kF31H1, I, I, 1), C(kH31F1, kH31F1, I, I, 1), C(kH, kF31H1, I, I, 1), C(kH31F1, kF, I, I, 1),
    C(kHlds, kFlds, I, I, 1), C(kHlds, kF, I, I, 1), C(kH, kFlds, I, I, 1),
    C(kHX, kHX, kFX, kFX, 1), C(kHX, kFX, kHX, kFX, 1), C(kHX, kHX, kHX, kFX, 1),
    C(kHX, kHX, kFX, kFX, 2),   // 8 waves per SIMD: 4 Hx + 4 Fx
    C(kHX, kHX, kHX, kHX, 2), C(kFX, kFX, kFX, kFX, 2),
  };
  {
    hipEvent_t w0, w1;
    CHECK(hipEventCreate(&w0)); CHECK(hipEventCreate(&w1));
    CHECK(hipEventRecord(w0));
    for (float el = 0; el < 500.f;) {
      for (int i = 0; i < 8; ++i) hipLaunchKernelGGL((k_mix<kH, kH, kH, kH>), dim3(cus * 2), dim3(1024), 0, 0, out, 1u);
      CHECK(hipEventRecord(w1));
      CHECK(hipEventSynchronize(w1));
      CHECK(hipEventElapsedTime(&el, w0, w1));
    }
  }
  for (int rep = 0; rep < 2; ++rep)
    for (const Case& c : cs) {
      const dim3 grid(cus * c.wgs_per_cu);
      hipLaunchKernelGGL(c.f, grid, dim3(1024), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(c.f, grid, dim3(1024), 0, 0, out, 3u + r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      int waves = 0;
      char name[128];
      int o = 0;
      for (int s = 0; s < 4; ++s) {
        if (c.k[s] < 0) continue;
        waves += c.wgs_per_cu;
        o += snprintf(name + o, sizeof(name) - o, "%s%s", o ? "+" : "", kNames[c.k[s]]);
      }
      const double per_wave = (double)ITERS * 32;  // VALU instructions per wave
      printf("{\"waves\": \"%s%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_valu_instr_at_2.4GHz\": %.3f, "
             "\"cycles_per_wave_instr\": %.3f}\n",
             c.wgs_per_cu == 2 ? "2x " : "", name, waves, best, best * 1e-3 * 2.4e9 / (per_wave * waves),
             best * 1e-3 * 2.4e9 / per_wave);
      fflush(stdout);
    }
  return 0;
}
