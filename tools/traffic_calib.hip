// FETCH_SIZE calibration for the engine's load pattern (gfx950).
//
// MI355X_MICROARCH.md: FETCH_SIZE reads exactly 1/2 of the bytes of a wide
// coalesced stream on gfx950 and is uncalibrated for other access widths. The
// SHA kernels read 16 B per lane per instruction with a 512-B lane stride (c2)
// -- not a coalesced stream -- so this kernel reads a known byte count with the
// SAME per-lane pattern (kPair: 8 x dwordx4 = one 128-B line per lane per step,
// lane stride = message stride) and no compute. rocprofv3 --pmc FETCH_SIZE on
// it gives the counter-to-bytes factor used to correct the c2 measurement.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/traffic_calib tools/traffic_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read_like_c2(const u32x4* __restrict__ arena, unsigned stride16,
                                                      unsigned lines_per_msg, unsigned n, unsigned* out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4* p = arena + (size_t)i * stride16;
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned l = 0; l < lines_per_msg; ++l) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= p[8 * l + k];
  }
  out[i] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main(int argc, char** argv) {
  const unsigned n = 1u << 20, msg = 512, stride = 512;
  const size_t bytes = (size_t)n * stride;
  u32x4* arena;
  unsigned* out;
  CHECK(hipMalloc(&arena, bytes + 64));
  CHECK(hipMalloc(&out, n * sizeof(unsigned)));
  CHECK(hipMemset(arena, 0x5a, bytes + 64));
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_read_like_c2, dim3(n / 256), dim3(256), 0, 0, arena, stride / 16, msg / 128, n, out);
    CHECK(hipDeviceSynchronize());
  }
  printf("{\"calib\": \"c2 read pattern\", \"bytes_read\": %zu, \"bytes_written\": %zu}\n", (size_t)n * msg,
         (size_t)n * 4);
  return 0;
}
