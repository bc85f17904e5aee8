// Per-call latency of the host entry points (C ABI, no Python in the loop), the
// way MirBFT's single hash worker calls them: one ActionList per call, its size
// set by how many hash actions accumulated (mirbft.go:282-302, work.go:159-160).
//
// Build (one line): g++ -O2 -std=c++17 -Iinclude -o tools/latency tools/latency.cpp
//   -Lmirbft_amd -lmirsha -Wl,-rpath,'$ORIGIN/../mirbft_amd' -Wl,-rpath,/opt/rocm/lib
// Run:   ./tools/latency > gpurun_out/latency.jsonl
//
// For each entry point and batch size: median / p90 / p99 microseconds per call
// over >= 200 calls (after 20 warmup calls), pinned and pageable arenas.
#include <mirsha.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(call)                                                                     \
  do {                                                                                  \
    int rc_ = (call);                                                                   \
    if (rc_ != MSHA_OK) {                                                               \
      fprintf(stderr, "%s failed: %d %s\n", #call, rc_, msha_last_error(ctx));          \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

struct Stat {
  double p50, p90, p99, mean;
};

template <class F>
static Stat timed(F&& call) {
  for (int i = 0; i < 20; ++i) call();
  std::vector<double> t;
  const double t_end = now_us() + 500e3;
  while (t.size() < 200 || (now_us() < t_end && t.size() < 5000)) {
    const double a = now_us();
    call();
    t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  double s = 0;
  for (double x : t) s += x;
  auto q = [&](double p) { return t[std::min(t.size() - 1, (size_t)(p * t.size()))]; };
  return {q(0.5), q(0.9), q(0.99), s / t.size()};
}

static void emit(const char* api, const char* arena, uint64_t n, uint64_t bytes, const Stat& s) {
  printf("{\"api\": \"%s\", \"arena\": \"%s\", \"n\": %llu, \"bytes\": %llu, \"p50_us\": %.1f, \"p90_us\": %.1f, "
         "\"p99_us\": %.1f, \"mean_us\": %.1f, \"digests_per_s_at_p50\": %.0f}\n",
         api, arena, (unsigned long long)n, (unsigned long long)bytes, s.p50, s.p90, s.p99, s.mean, n / (s.p50 * 1e-6));
  fflush(stdout);
}

int main() {
  msha_ctx* ctx = nullptr;
  char err[512];
  if (msha_ctx_create_err(1, &ctx, err, sizeof err) != MSHA_OK) {
    fprintf(stderr, "ctx: %s\n", err);
    return 1;
  }
  const uint64_t kMaxN = 262144, kMsg = 512, kArena = kMaxN * kMsg + 64;
  uint8_t* pinned = nullptr;
  uint8_t* pinned_out = nullptr;
  CHECK(msha_pinned_alloc(ctx, kArena, (void**)&pinned));
  CHECK(msha_pinned_alloc(ctx, 32 * kMaxN, (void**)&pinned_out));
  std::vector<uint8_t> pageable(kArena), out(32 * kMaxN);
  std::mt19937_64 rng(0x4D49524246540000ull);
  for (uint64_t i = 0; i < kArena; ++i) pageable[i] = pinned[i] = (uint8_t)rng();
  std::vector<uint64_t> off(kMaxN), len(kMaxN, kMsg);
  for (uint64_t i = 0; i < kMaxN; ++i) off[i] = kMsg * i;

  const uint64_t sizes[] = {1, 4, 16, 64, 256, 1024, 4096, 16384, 65536, 262144};
  // request digests (clients.go:189-192): n x 512 B
  for (uint64_t n : sizes) {
    emit("msha_digest_batch", "pinned", n, n * kMsg, timed([&] {
           CHECK(msha_digest_batch(ctx, pinned, kArena, off.data(), len.data(), n, pinned_out));
         }));
    emit("msha_digest_batch", "pageable", n, n * kMsg, timed([&] {
           CHECK(msha_digest_batch(ctx, pageable.data(), kArena, off.data(), len.data(), n, out.data()));
         }));
  }
  // Batch digests (sequence.go:155-158): n batches x 20 request-ack digests
  std::vector<uint32_t> idx(20 * kMaxN);
  std::vector<uint64_t> begin(kMaxN + 1);
  for (uint64_t i = 0; i < idx.size(); ++i) idx[i] = (uint32_t)(rng() % 4096);
  for (uint64_t i = 0; i <= kMaxN; ++i) begin[i] = 20 * i;
  for (uint64_t n : sizes) {
    emit("msha_digest_of_digests", "pageable", n, n * 640, timed([&] {
           CHECK(msha_digest_of_digests(ctx, pageable.data(), 4096, idx.data(), 20 * n, begin.data(), n,
                                        out.data()));
         }));
  }
  // generic ProcessHashActions (serial.go:180-198): n actions x 20 parts of 32 B
  std::vector<uint64_t> poff(20 * kMaxN), plen(20 * kMaxN, 32);
  for (uint64_t i = 0; i < poff.size(); ++i) poff[i] = 32 * (uint64_t)idx[i];
  for (uint64_t n : sizes) {
    emit("msha_hash_actions", "pageable", n, n * 640, timed([&] {
           CHECK(msha_hash_actions(ctx, pageable.data(), kArena, poff.data(), plen.data(), 20 * n, begin.data(), n,
                                   out.data()));
         }));
  }
  msha_pinned_free(ctx, pinned);
  msha_pinned_free(ctx, pinned_out);
  msha_ctx_destroy(ctx);
  return 0;
}
