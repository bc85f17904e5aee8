// Integer-VALU microbenchmark, part 5 (gfx950): does the ORDER of half-rate
// (H: v_alignbit/v_add3) and full-rate (F: v_bitop3/v_add) instructions in a
// wave's stream change throughput, with no data dependencies inside a round?
// Same multiset per "round" as SHA-256: 6 alignbit + 3 add3 + 4 bitop3 + 1 add.
// Orders: grouped (9 H then 5 F), alternating (H F H F ...), and the order
// hipcc emits for a real round (sha256_device.hpp). Each also with true
// round-to-round dependencies (the SHA pattern) vs none.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_microbench5 tools/valu_microbench5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 1024;

#define CLOB "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"

// independent: destinations v40..v53, sources v32..v39 (never written in the loop)
#define H1 "v_alignbit_b32 v40, v32, v32, 6\n"
#define H2 "v_alignbit_b32 v41, v33, v33, 11\n"
#define H3 "v_alignbit_b32 v42, v34, v34, 25\n"
#define H4 "v_alignbit_b32 v43, v35, v35, 2\n"
#define H5 "v_alignbit_b32 v44, v36, v36, 13\n"
#define H6 "v_alignbit_b32 v45, v37, v37, 22\n"
#define A1 "v_add3_u32 v46, v32, v33, v34\n"
#define A2 "v_add3_u32 v47, v35, v36, v37\n"
#define A3 "v_add3_u32 v48, v38, v39, v32\n"
#define F1 "v_bitop3_b32 v49, v32, v33, v34 bitop3:0x96\n"
#define F2 "v_bitop3_b32 v50, v35, v36, v37 bitop3:0xca\n"
#define F3 "v_bitop3_b32 v51, v38, v39, v32 bitop3:0x96\n"
#define F4 "v_bitop3_b32 v52, v33, v34, v35 bitop3:0xe8\n"
#define D1 "v_add_u32 v53, v36, v37\n"

#define ORDER_GROUPED H1 H2 H3 H4 H5 H6 A1 A2 A3 F1 F2 F3 F4 D1
#define ORDER_ALT H1 F1 H2 F2 H3 F3 H4 F4 H5 D1 H6 A1 A2 A3
#define ORDER_HIPCC H1 H2 H3 F1 F2 A1 A2 H4 H5 H6 D1 F3 F4 A3

// dependent SHA-like round on registers a..h = v32..v39, temps v40..v43, K/W in v44,v45
#define DEP_ROUND(a,b,c,d,e,f,g,h) \
  "v_alignbit_b32 v40, " e ", " e ", 6\n" \
  "v_alignbit_b32 v41, " e ", " e ", 11\n" \
  "v_alignbit_b32 v42, " e ", " e ", 25\n" \
  "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n" \
  "v_bitop3_b32 v41, " e ", " f ", " g " bitop3:0xca\n" \
  "v_add3_u32 v43, " h ", v44, v41\n" \
  "v_add3_u32 v43, v43, v40, v45\n" \
  "v_alignbit_b32 v40, " a ", " a ", 2\n" \
  "v_alignbit_b32 v41, " a ", " a ", 13\n" \
  "v_alignbit_b32 v42, " a ", " a ", 22\n" \
  "v_add_u32 " d ", v43, " d "\n" \
  "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n" \
  "v_bitop3_b32 v41, " a ", " b ", " c " bitop3:0xe8\n" \
  "v_add3_u32 " h ", v40, v41, v43\n"
#define DEP8 \
  DEP_ROUND("v32","v33","v34","v35","v36","v37","v38","v39") \
  DEP_ROUND("v39","v32","v33","v34","v35","v36","v37","v38") \
  DEP_ROUND("v38","v39","v32","v33","v34","v35","v36","v37") \
  DEP_ROUND("v37","v38","v39","v32","v33","v34","v35","v36") \
  DEP_ROUND("v36","v37","v38","v39","v32","v33","v34","v35") \
  DEP_ROUND("v35","v36","v37","v38","v39","v32","v33","v34") \
  DEP_ROUND("v34","v35","v36","v37","v38","v39","v32","v33") \
  DEP_ROUND("v33","v34","v35","v36","v37","v38","v39","v32")

// Diagnostic clock stamps: lane 0 of each wave records (s_memtime, s_memrealtime)
// at start and end into clk[]; in-kernel clock = d(memtime)/d(realtime) x 100 MHz.
__device__ unsigned long long g_clk[4096 * 4];
#define KERN(name, BODY, ROUNDS_PER_ITER)                                   \
  __global__ void name(unsigned* out, unsigned seed) {                      \
    unsigned x = seed ^ threadIdx.x;                                        \
    const unsigned wid = (blockIdx.x * blockDim.x + threadIdx.x) / 64;     \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                   \
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();               \
    asm volatile("v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n" \
                 "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n" \
                 "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n" :: "v"(x) : CLOB); \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY ::: CLOB);            \
    unsigned y;                                                             \
    asm volatile("v_xor_b32 %0, v32, v40" : "=v"(y));                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;                         \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                   \
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();               \
    if ((threadIdx.x & 63) == 0 && wid < 4096) {                            \
      g_clk[4 * wid] = t0; g_clk[4 * wid + 1] = r0;                         \
      g_clk[4 * wid + 2] = t1; g_clk[4 * wid + 3] = r1;                     \
    }                                                                       \
  }

#define X8(s) s s s s s s s s
KERN(k_grouped, X8(ORDER_GROUPED), 8)
KERN(k_alt, X8(ORDER_ALT), 8)
KERN(k_hipcc, X8(ORDER_HIPCC), 8)
KERN(k_dep, DEP8, 8)

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  unsigned* out;
  CHECK(hipMalloc(&out, sizeof(unsigned) * cus * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct { const char* name; void (*f)(unsigned*, unsigned); } ks[] = {
    {"independent grouped 9H+5F", k_grouped}, {"independent alternating", k_alt},
    {"independent hipcc order", k_hipcc}, {"dependent SHA round", k_dep}};
  for (int rep = 0; rep < 2; ++rep)
  for (auto& k : ks) {
    for (int wps : {1, 2, 4, 8}) {
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
      static unsigned long long clk[4096 * 4];
      CHECK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk)));
      int nw = cus * wps * 4 < 4096 ? cus * wps * 4 : 4096;
      double ghz_sum = 0; int cnt = 0;
      for (int i = 0; i < nw; ++i) {
        double dt = (double)(clk[4 * i + 2] - clk[4 * i]), dr = (double)(clk[4 * i + 3] - clk[4 * i + 1]);
        if (dr > 0) { ghz_sum += dt / dr * 0.1; ++cnt; }
      }
      double ghz = cnt ? ghz_sum / cnt : 0;
      double rounds = (double)ITERS * 8 * wps;   // per SIMD
      printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_round_at_2.4GHz\": %.2f, "
             "\"in_kernel_GHz\": %.3f, \"simd_cycles_per_round_in_kernel_clock\": %.2f, \"model_cycles_9H5F\": 46}\n",
             k.name, wps, best, best * 1e-3 * 2.4e9 / rounds, ghz, best * 1e-3 * ghz * 1e9 / rounds);
    }
  }
  return 0;
}
