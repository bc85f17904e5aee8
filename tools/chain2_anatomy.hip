// Where a head chain's time goes (k_digest_chain2, the planned/host heads): the
// shipped kernel built with MSHA_CHAIN2_STAMPS, one message of NB blocks (argv[1],
// default 1,427: c5's longest EpochChange payload), one workgroup on its own CU
// (the EXCL head launch). Lane 0 of the producer and of each consumer wave stamps
// s_memtime before and after every barrier; per block: the consumers' compute
// (barrier j+1 .. barrier j+2 arrival) and wait, the producer's compute and wait,
// in shader-clock ticks; the clock from s_memrealtime around the whole launch.
// One JSON line. After ~0.5 s of warm launches (clock ramp). argv[2] == 8: the
// eight-lane head (k_digest_chain8, round 5) instead. argv[3]: messages (default 1;
// 16 fills an eight-lane workgroup: the same payload, every lane active).
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -I include -o tools/chain2_anatomy tools/chain2_anatomy.hip
#ifndef MSHA_ANATOMY_NO_STAMPS  // -DMSHA_ANATOMY_NO_STAMPS: the kernel's time alone (stamp fields 0)
#define MSHA_CHAIN2_STAMPS 1
#endif
#include "kernels.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}
static double mean(const std::vector<double>& v) {
  double s = 0;
  for (double x : v) s += x;
  return v.empty() ? 0 : s / v.size();
}

int main(int argc, char** argv) {
  const uint64_t NB = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1427;
  const uint64_t L = NB * 64 - 20;  // NB blocks (the last one holds the length)
  const uint64_t M = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
  uint8_t *arena, *out;
  uint64_t *off, *len, *stamps;
  uint32_t* err;
  CHECK(hipMalloc(&arena, L + 64));
  CHECK(hipMemset(arena, 0x5a, L + 64));
  CHECK(hipMalloc(&off, 8 * M));
  CHECK(hipMalloc(&len, 8 * M));
  CHECK(hipMemset(off, 0, 8 * M));
  std::vector<uint64_t> lens(M, L);
  CHECK(hipMemcpy(len, lens.data(), 8 * M, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, 32 * M + 32));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMemset(err, 0, 4));
  CHECK(hipMalloc(&stamps, 4 * 4096 * 8));
#ifndef MSHA_ANATOMY_NO_STAMPS
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(msha::g_chain2_stamps), &stamps, sizeof stamps));
#endif
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  msha::LaneGate g;
  g.head_part = true;
  g.two_lane = true;
  g.eight_lane = argc > 2 && atoi(argv[2]) == 8;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&] {
    msha::LaunchKind kind;
    CHECK(msha::launch_digest_batch(arena, off, len, nullptr, nullptr, M, out, err, prop.multiProcessorCount,
                                    2 /* MSHA_KERNEL_COOP */, 0, nullptr, &kind, &g));
  };
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.5) {
    launch();
    CHECK(hipDeviceSynchronize());
  }
  CHECK(hipMemset(stamps, 0, 4 * 4096 * 8));
  CHECK(hipEventRecord(e0));
  launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(4 * 4096);
  CHECK(hipMemcpy(h.data(), stamps, 8 * h.size(), hipMemcpyDeviceToHost));
  // consumer wave: 1 for the two-lane kernel, 2 for the eight-lane one (waves 0-1 produce)
  const int cw = g.eight_lane ? 2 : 1;
  auto st = [&](int wave, uint64_t j, int after) { return (double)h[wave * 4096 + 2 * j + after]; };
  const uint64_t nb = std::min<uint64_t>(NB, 2040);
  std::vector<double> c_comp, c_wait, p_comp, p_wait;
  for (uint64_t b = 1; b + 2 < nb; ++b) {  // steady state: skip the first and last blocks
    c_comp.push_back(st(cw, b + 2, 0) - st(cw, b + 1, 1));  // block b: after barrier b+1 .. barrier b+2
    c_wait.push_back(st(cw, b + 1, 1) - st(cw, b + 1, 0));
    p_comp.push_back(st(0, b, 0) - st(0, b - 1, 1));      // block b's slot: after barrier b-1 .. barrier b
    p_wait.push_back(st(0, b, 1) - st(0, b, 0));
  }
  const double total_ticks = st(cw, nb, 1) - st(cw, 0, 0);
  const double ghz = total_ticks / (ms * 1e-3) / 1e9;  // approx: ticks over the launch's event time
  printf("{\"kernel\": \"%s\", \"blocks\": %llu, \"kernel_ms\": %.4f, \"us_per_block\": %.4f, \"ticks_per_block\": %.1f, "
         "\"approx_clock_ghz\": %.3f, \"consumer_compute_ticks_median\": %.1f, \"consumer_compute_ticks_mean\": %.1f, "
         "\"consumer_wait_ticks_median\": %.1f, \"consumer_wait_ticks_mean\": %.1f, "
         "\"producer_compute_ticks_median\": %.1f, \"producer_wait_ticks_median\": %.1f}\n",
         g.eight_lane ? "chain8" : "chain2", (unsigned long long)NB, ms, ms * 1e3 / NB, total_ticks / nb, ghz, median(c_comp), mean(c_comp),
         median(c_wait), mean(c_wait), median(p_comp), median(p_wait));
  return 0;
}
