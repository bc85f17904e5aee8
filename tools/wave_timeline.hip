// Diagnostic (not product code): per-wave start/end timestamps of the lane
// kernel's message loop, to see where a launch's time goes beyond the steady
// compression rate -- ramp (waves starting late), drain (waves ending early
// while others still run), per-SIMD occupancy over time.
//
// It includes kernels.hip itself, so the timed loop is the shipped
// hash_message<kPair> (the form k_digest_batch / k_digest_uniform run at >= 3
// waves per SIMD). Output: a raw record per wave (t_start, t_end in
// s_memrealtime ticks of 10 ns, HW_ID, XCC_ID) for each launch config, written to
// gpurun_out/timeline/<n>_<len>.bin; tools/wave_timeline.py summarises them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/wave_timeline.hip -o tools/wave_timeline
//   tools/wave_timeline 196608 640 1048576 512 ...
#include "../mirbft_amd/csrc/kernels.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ __launch_bounds__(256, 8) void k_timeline(const uint8_t* __restrict__ arena, uint64_t stride,
                                                     uint64_t msg_len, uint64_t n, uint8_t* __restrict__ out,
                                                     uint64_t* __restrict__ rec) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t hwid, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) msha::hash_message<msha::kPair>(arena + i * stride, msg_len, out + 32 * i);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if ((threadIdx.x & 63) == 0) {
    rec[4 * wave + 0] = t0;
    rec[4 * wave + 1] = t1;
    rec[4 * wave + 2] = hwid;
    rec[4 * wave + 3] = xcc;
  }
}

int main(int argc, char** argv) {
  if (argc < 3 || (argc - 1) % 2) {
    fprintf(stderr, "usage: %s N LEN [N LEN ...]\n", argv[0]);
    return 2;
  }
  std::string dir = "gpurun_out/timeline";
  (void)system(("mkdir -p " + dir).c_str());
  for (int a = 1; a + 1 < argc; a += 2) {
    const uint64_t n = strtoull(argv[a], nullptr, 0), len = strtoull(argv[a + 1], nullptr, 0);
    const uint64_t stride = (len + 15) / 16 * 16;
    const uint64_t waves = (n + 63) / 64;
    uint8_t *arena, *out;
    uint64_t* rec;
    CK(hipMalloc(&arena, n * stride + 64));
    CK(hipMemset(arena, 0x5a, n * stride + 64));
    CK(hipMalloc(&out, 32 * n));
    CK(hipMalloc(&rec, 32 * waves));
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // warm the clocks (>= 300 ms of load), then time 5 launches and keep the last record
    auto t_start = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() < 0.4) {
      for (int r = 0; r < 8; ++r)
        hipLaunchKernelGGL(k_timeline, dim3(grid), dim3(256), 0, 0, arena, stride, len, n, out, rec);
      CK(hipDeviceSynchronize());
    }
    float ms = 0;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r)
      hipLaunchKernelGGL(k_timeline, dim3(grid), dim3(256), 0, 0, arena, stride, len, n, out, rec);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint64_t> h(4 * waves);
    CK(hipMemcpy(h.data(), rec, 32 * waves, hipMemcpyDeviceToHost));
    const std::string f = dir + "/" + std::to_string(n) + "_" + std::to_string(len) + ".bin";
    FILE* fp = fopen(f.c_str(), "wb");
    fwrite(h.data(), 8, h.size(), fp);
    fclose(fp);
    printf("{\"n\": %llu, \"len\": %llu, \"waves\": %llu, \"ms_per_launch\": %.5f, \"file\": \"%s\"}\n",
           (unsigned long long)n, (unsigned long long)len, (unsigned long long)waves, ms / 5, f.c_str());
    CK(hipFree(arena));
    CK(hipFree(out));
    CK(hipFree(rec));
  }
  return 0;
}
