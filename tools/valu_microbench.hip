// Integer-VALU throughput microbenchmark for gfx950 (MI355X).
//
// Purpose: pin the roofline denominator used by bench.py. SHA-256 on the GPU is
// integer-VALU bound; the instructions it compiles to are v_add3_u32,
// v_xor3_b32, v_alignbit_b32, v_bfi_b32, v_perm_b32, v_add_u32, v_lshrrev_b32.
// Each kernel runs 8 independent dependency chains of ONE instruction kind
// (inline asm, so the exact opcode is what runs) and reports lane-ops/s at
// several waves-per-SIMD occupancies, plus a half-EXEC variant (lanes 32..63
// masked) to see whether a half-populated wave64 issues in one pass.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench tools/valu_microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;
constexpr int CHAINS = 8;

#define OP3(name) \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a4) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a5) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a6) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2" : "+v"(a7) : "v"(b), "v"(c));

#define OP3B(name) \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a1) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a2) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a3) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a4) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a5) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a6) : "v"(b), "v"(c)); \
  asm volatile(name " %0, %0, %1, %2 bitop3:0x96" : "+v"(a7) : "v"(b), "v"(c));

#define OP2(name) \
  asm volatile(name " %0, %0, %1" : "+v"(a0) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a1) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a2) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a3) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a4) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a5) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a6) : "v"(b)); \
  asm volatile(name " %0, %0, %1" : "+v"(a7) : "v"(b));

#define KERNEL(kname, BODY) \
__global__ void kname(unsigned* out, unsigned seed, int half) { \
  unsigned lane = threadIdx.x & 63; \
  if (half && lane >= 32) return; \
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x; \
  unsigned a0 = b + 1, a1 = b + 2, a2 = b + 3, a3 = b + 4, a4 = b + 5, a5 = b + 6, a6 = b + 7, a7 = b + 8; \
  for (int i = 0; i < ITERS; ++i) { BODY BODY BODY BODY } \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}

KERNEL(k_add3, OP3("v_add3_u32"))
KERNEL(k_bitop3, OP3B("v_bitop3_b32"))
KERNEL(k_xad, OP3("v_xad_u32"))
KERNEL(k_alignbit, OP3("v_alignbit_b32"))
KERNEL(k_bfi, OP3("v_bfi_b32"))
KERNEL(k_perm, OP3("v_perm_b32"))
KERNEL(k_add, OP2("v_add_u32"))
KERNEL(k_xor, OP2("v_xor_b32"))

typedef void (*kfn)(unsigned*, unsigned, int);

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, cus, p.clockRate);
  struct { const char* name; kfn f; } ks[] = {
    {"v_add3_u32", k_add3}, {"v_bitop3_b32", k_bitop3}, {"v_xad_u32", k_xad}, {"v_alignbit_b32", k_alignbit},
    {"v_bfi_b32", k_bfi}, {"v_perm_b32", k_perm}, {"v_add_u32", k_add}, {"v_xor_b32", k_xor}};
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const long ops_per_lane = (long)ITERS * 4 * CHAINS;
  for (auto& k : ks) {
    for (int wps : {1, 2, 4, 8}) {       // waves per SIMD
      for (int half = 0; half < 2; ++half) {
        dim3 grid(cus * wps), block(256);  // 4 waves per WG -> one per SIMD
        hipLaunchKernelGGL(k.f, grid, block, 0, 0, out, 12345u, half);  // warm
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
          CHECK(hipEventRecord(e0));
          hipLaunchKernelGGL(k.f, grid, block, 0, 0, out, 777u + r, half);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
        }
        double waves = (double)cus * wps * 4;
        double lanes_active = waves * (half ? 32 : 64);
        double wave_instr = waves * ops_per_lane;
        double lane_ops = lanes_active * ops_per_lane;
        // cycles per wave-instruction per SIMD at 2.4 GHz
        double simd_cyc = (best * 1e-3 * 2.4e9) / (wave_instr / (cus * 4.0));
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"half_exec\": %d, \"ms\": %.4f, "
               "\"T_lane_ops_per_s\": %.3f, \"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
               k.name, wps, half, best, lane_ops / (best * 1e-3) / 1e12, simd_cyc);
      }
    }
  }
  CHECK(hipFree(out));
  return 0;
}
