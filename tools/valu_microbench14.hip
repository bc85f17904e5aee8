// Integer-VALU microbenchmark, part 14 (gfx950): which instruction streams of
// two (or four) waves sharing a SIMD overlap? Part 13: a wave of half-rate ops
// (v_alignbit) and a wave of full-rate ops (v_add) run side by side (each at
// its lone-wave rate), yet two waves that each alternate alignbit/add cost ~4
// cycles per instruction. Here: runs of 1, 4 and 16 of each class, in phase and
// in opposite phase across the two waves, pure waves beside mixed ones, and two
// pure pairs per SIMD. Independent operands throughout (no dependency waits).
// One workgroup per CU, 4 x S waves (S = waves per SIMD); wave w's stream is
// chosen by its slot w / 4, so each SIMD holds one wave per slot (checked via
// HW_ID in part 13). Timed after >= 500 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench14 tools/valu_microbench14.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;
#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","vcc"
#define H(d, s) "v_alignbit_b32 v" #d ", v" #s ", v" #s ", 7\n"
#define F(d, s) "v_add_u32_e32 v" #d ", v" #s ", v33\n"
#define H4 H(48, 32) H(49, 34) H(50, 36) H(51, 38)
#define H4b H(52, 40) H(53, 42) H(54, 44) H(55, 46)
#define F4 F(48, 32) F(49, 34) F(50, 36) F(51, 38)
#define F4b F(52, 40) F(53, 42) F(54, 44) F(55, 46)
#define HF4 H(48, 32) F(49, 34) H(50, 36) F(51, 38)
#define HF4b H(52, 40) F(53, 42) H(54, 44) F(55, 46)
#define FH4 F(48, 32) H(49, 34) F(50, 36) H(51, 38)
#define FH4b F(52, 40) H(53, 42) F(54, 44) H(55, 46)
// 32-instruction bodies
#define S_H32 H4 H4b H4 H4b H4 H4b H4 H4b
#define S_F32 F4 F4b F4 F4b F4 F4b F4 F4b
#define S_HF HF4 HF4b HF4 HF4b HF4 HF4b HF4 HF4b
#define S_FH FH4 FH4b FH4 FH4b FH4 FH4b FH4 FH4b
#define S_H4F4 H4 F4b H4 F4b H4 F4b H4 F4b
#define S_F4H4 F4 H4b F4 H4b F4 H4b F4 H4b
#define S_H16F16 H4 H4b H4 H4b F4 F4b F4 F4b
#define S_F16H16 F4 F4b F4 F4b H4 H4b H4 H4b

enum { kH = 0, kF, kHF, kFH, kH4F4, kF4H4, kH16F16, kF16H16, kIdle = -1 };
static const char* kNames[] = {"H", "F", "HF", "FH", "H4F4", "F4H4", "H16F16", "F16H16"};

template <int K>
__device__ __forceinline__ void run() {
  for (int i = 0; i < ITERS; ++i) {
    if (K == kH) asm volatile(S_H32 ::: CLOB);
    if (K == kF) asm volatile(S_F32 ::: CLOB);
    if (K == kHF) asm volatile(S_HF ::: CLOB);
    if (K == kFH) asm volatile(S_FH ::: CLOB);
    if (K == kH4F4) asm volatile(S_H4F4 ::: CLOB);
    if (K == kF4H4) asm volatile(S_F4H4 ::: CLOB);
    if (K == kH16F16) asm volatile(S_H16F16 ::: CLOB);
    if (K == kF16H16) asm volatile(S_F16H16 ::: CLOB);
  }
}

template <int K0, int K1, int K2, int K3>
__global__ __launch_bounds__(1024) void k_mix(unsigned* out, unsigned seed) {
  const unsigned slot = (threadIdx.x >> 6) / 4;
  const int kind = slot == 0 ? K0 : slot == 1 ? K1 : slot == 2 ? K2 : K3;
  if (kind < 0) return;
  unsigned x = seed ^ threadIdx.x;
  asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n"
               "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n"
               "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
               "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 13\n" :: "v"(x) : CLOB);
  switch (kind) {
    case kH: run<kH>(); break;
    case kF: run<kF>(); break;
    case kHF: run<kHF>(); break;
    case kFH: run<kFH>(); break;
    case kH4F4: run<kH4F4>(); break;
    case kF4H4: run<kF4H4>(); break;
    case kH16F16: run<kH16F16>(); break;
    case kF16H16: run<kF16H16>(); break;
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
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 1024));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct Case { int k[4]; void (*f)(unsigned*, unsigned); };
#define C(a, b, c, d) Case{{a, b, c, d}, k_mix<a, b, c, d>}
  const Case cs[] = {
    C(kH, kIdle, kIdle, kIdle), C(kF, kIdle, kIdle, kIdle), C(kHF, kIdle, kIdle, kIdle),
    C(kH, kF, kIdle, kIdle), C(kH, kH, kIdle, kIdle), C(kF, kF, kIdle, kIdle),
    C(kHF, kHF, kIdle, kIdle), C(kHF, kFH, kIdle, kIdle),
    C(kH4F4, kH4F4, kIdle, kIdle), C(kH4F4, kF4H4, kIdle, kIdle),
    C(kH16F16, kH16F16, kIdle, kIdle), C(kH16F16, kF16H16, kIdle, kIdle),
    C(kH, kHF, kIdle, kIdle), C(kF, kHF, kIdle, kIdle),
    C(kH, kH, kF, kF), C(kH, kF, kH, kF), C(kHF, kHF, kHF, kHF), C(kH16F16, kF16H16, kH16F16, kF16H16),
    C(kH, kF, kF, kIdle), C(kH, kH, kF, kIdle),
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
      hipLaunchKernelGGL(c.f, dim3(cus), dim3(1024), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(c.f, dim3(cus), dim3(1024), 0, 0, out, 3u + r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      int waves = 0;
      char name[96];
      int o = 0;
      for (int s = 0; s < 4; ++s) {
        if (c.k[s] < 0) continue;
        ++waves;
        o += snprintf(name + o, sizeof(name) - o, "%s%s", o ? "+" : "", kNames[c.k[s]]);
      }
      const double per_wave = (double)ITERS * 32;
      printf("{\"waves\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_instr_at_2.4GHz\": %.3f, "
             "\"cycles_per_wave_instr\": %.3f}\n",
             name, waves, best, best * 1e-3 * 2.4e9 / (per_wave * waves), best * 1e-3 * 2.4e9 / per_wave);
      fflush(stdout);
    }
  return 0;
}
