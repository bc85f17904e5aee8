// Integer-VALU microbenchmark, part 2 (gfx950): operand forms and mixes.
//
// Part 1 (valu_microbench.hip) showed VOP2 ops (v_add_u32, v_xor_b32) and
// v_bitop3_b32 issue at ~2.4 SIMD-cycles per wave64 instruction (8 waves/SIMD),
// while v_alignbit/v_add3/v_bfi/v_perm/v_xad take ~4.2. This part checks:
//  * rotate form v_alignbit_b32 x, x, <inline const>   (what SHA-256 uses)
//  * shifts with inline constants, v_add_u32 with an SGPR operand, VOP3-encoded add
//  * MIXED streams: does a half-rate op overlap with full-rate ops of other waves?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench2 tools/valu_microbench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 2048;

// Each body below applies its instruction pattern to 8 independent chains a0..a7.
#define EACH(S) S(a0) S(a1) S(a2) S(a3) S(a4) S(a5) S(a6) S(a7)

#define ROT(a)    asm volatile("v_alignbit_b32 %0, %0, %0, 6" : "+v"(a));
#define SHR(a)    asm volatile("v_lshrrev_b32 %0, 6, %0" : "+v"(a));
#define ADDS(a)   asm volatile("v_add_u32 %0, %1, %0" : "+v"(a) : "s"(s));
#define ADD64(a)  asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a) : "v"(b));
#define LSHLOR(a) asm volatile("v_lshl_or_b32 %0, %0, 26, %1" : "+v"(a) : "v"(b));
#define OR3(a)    asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
#define BITOP3(a) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(a) : "v"(b), "v"(c));
#define XOR(a)    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
#define ADD3S(a)  asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "s"(s), "v"(b));
#define PERM(a)   asm volatile("v_perm_b32 %0, 0, %0, %1" : "+v"(a) : "s"(s));
// mixes (per chain): 1 half-rate + 1 full-rate, 1 half + 2 full, 1 half + 3 full
#define MIX11(a)  ROT(a) XOR(a)
#define MIX12(a)  ROT(a) XOR(a) BITOP3(a)
#define MIX13(a)  ROT(a) XOR(a) BITOP3(a) ADDS(a)
// SHA-256-round-like instruction mix: 6 alignbit, 4 bitop3, 6 add (as VOP2)
#define SHAMIX(a) ROT(a) ROT(a) ROT(a) BITOP3(a) BITOP3(a) ADDS(a) ADDS(a) ADDS(a) \
                  ROT(a) ROT(a) ROT(a) BITOP3(a) BITOP3(a) ADDS(a) ADDS(a) ADDS(a)

#define KERNEL(kname, S, NOPS) \
__global__ void kname(unsigned* out, unsigned seed) { \
  unsigned s = __builtin_amdgcn_readfirstlane(seed * 7u); \
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x; \
  unsigned a0 = b + 1, a1 = b + 2, a2 = b + 3, a3 = b + 4, a4 = b + 5, a5 = b + 6, a6 = b + 7, a7 = b + 8; \
  for (int i = 0; i < ITERS; ++i) { EACH(S) EACH(S) } \
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
}

KERNEL(k_rot, ROT, 1)
KERNEL(k_shr, SHR, 1)
KERNEL(k_adds, ADDS, 1)
KERNEL(k_add64, ADD64, 1)
KERNEL(k_lshlor, LSHLOR, 1)
KERNEL(k_or3, OR3, 1)
KERNEL(k_add3s, ADD3S, 1)
KERNEL(k_perm, PERM, 1)
KERNEL(k_mix11, MIX11, 2)
KERNEL(k_mix12, MIX12, 3)
KERNEL(k_mix13, MIX13, 4)
KERNEL(k_shamix, SHAMIX, 16)

typedef void (*kfn)(unsigned*, unsigned);

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  struct { const char* name; kfn f; int nops; } ks[] = {
    {"alignbit_rot_const", k_rot, 1}, {"lshrrev_const", k_shr, 1}, {"add_u32_sgpr", k_adds, 1},
    {"add_u32_e64", k_add64, 1}, {"lshl_or_b32", k_lshlor, 1}, {"or3_b32", k_or3, 1},
    {"add3_u32_sgpr", k_add3s, 1}, {"perm_b32_bswap", k_perm, 1},
    {"mix 1H+1F", k_mix11, 2}, {"mix 1H+2F", k_mix12, 3}, {"mix 1H+3F", k_mix13, 4},
    {"sha-round-mix 6H+10F", k_shamix, 16}};
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (auto& k : ks) {
    for (int wps : {2, 4, 8}) {
      dim3 grid(cus * wps), block(256);
      hipLaunchKernelGGL(k.f, grid, block, 0, 0, out, 12345u);
      CHECK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, grid, block, 0, 0, out, 777u + r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      double instr_per_wave = (double)ITERS * 2 * 8 * k.nops;
      double waves = (double)cus * wps * 4;
      double simd_cyc = (best * 1e-3 * 2.4e9) / (waves * instr_per_wave / (cus * 4.0));
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"T_lane_ops_per_s\": %.3f, "
             "\"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
             k.name, wps, best, waves * 64 * instr_per_wave / (best * 1e-3) / 1e12, simd_cyc);
    }
  }
  CHECK(hipFree(out));
  return 0;
}
