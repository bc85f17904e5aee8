// Latency floor of the HIP operations one small msha_digest_batch call issues
// (pinned host buffers, one stream, each sequence followed by a stream sync):
// what a call of a few messages costs before any hashing, and which of its
// operations are worth merging. Median microseconds over 2,000 repetitions.
//
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/op_latency tools/op_latency.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void k_touch(const unsigned* in, unsigned* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = in[0] + 1;
}

static double us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median_us(const std::function<void()>& f) {
  for (int i = 0; i < 200; ++i) f();
  std::vector<double> t(2000);
  for (double& x : t) {
    const double a = us();
    f();
    x = us() - a;
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc(&h_in, 1 << 20, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, 1 << 20, hipHostMallocDefault));
  CK(hipMalloc(&d_in, 1 << 20));
  CK(hipMalloc(&d_out, 1 << 20));
  auto sync = [&] { (void)hipStreamSynchronize(s); };
  struct Row {
    const char* name;
    std::function<void()> f;
  };
  const std::vector<Row> rows = {
      {"sync only", [&] { sync(); }},
      {"H2D 16 B", [&] { (void)hipMemcpyAsync(d_in, h_in, 16, hipMemcpyHostToDevice, s); sync(); }},
      {"H2D 64 KiB", [&] { (void)hipMemcpyAsync(d_in, h_in, 65536, hipMemcpyHostToDevice, s); sync(); }},
      {"D2H 36 B", [&] { (void)hipMemcpyAsync(h_out, d_out, 36, hipMemcpyDeviceToHost, s); sync(); }},
      {"memset 4 B", [&] { (void)hipMemsetAsync(d_out, 0, 4, s); sync(); }},
      {"kernel", [&] { k_touch<<<1, 64, 0, s>>>(d_in, d_out); sync(); }},
      {"H2D + kernel + D2H",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, 16, hipMemcpyHostToDevice, s);
         k_touch<<<1, 64, 0, s>>>(d_in, d_out);
         (void)hipMemcpyAsync(h_out, d_out, 36, hipMemcpyDeviceToHost, s);
         sync();
       }},
      {"2 H2D + memset + kernel + 2 D2H",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, 8, hipMemcpyHostToDevice, s);
         (void)hipMemcpyAsync(d_in + 2, h_in + 2, 8, hipMemcpyHostToDevice, s);
         (void)hipMemsetAsync(d_out + 8, 0, 4, s);
         k_touch<<<1, 64, 0, s>>>(d_in, d_out);
         (void)hipMemcpyAsync(h_out, d_out, 32, hipMemcpyDeviceToHost, s);
         (void)hipMemcpyAsync(h_out + 8, d_out + 8, 4, hipMemcpyDeviceToHost, s);
         sync();
       }},
      {"H2D on stream 2 + event wait + kernel + D2H",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, 16, hipMemcpyHostToDevice, s2);
         (void)hipEventRecord(ev, s2);
         (void)hipStreamWaitEvent(s, ev, 0);
         k_touch<<<1, 64, 0, s>>>(d_in, d_out);
         (void)hipMemcpyAsync(h_out, d_out, 36, hipMemcpyDeviceToHost, s);
         sync();
       }},
      {"kernel reading pinned host + writing pinned host (zero-copy)",
       [&] {
         k_touch<<<1, 64, 0, s>>>(h_in, h_out);
         sync();
       }},
  };
  for (const Row& r : rows) printf("{\"op\": \"%s\", \"median_us\": %.1f}\n", r.name, median_us(r.f));
  return 0;
}
