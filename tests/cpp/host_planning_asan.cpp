// Host planning code of libmirsha under AddressSanitizer + UndefinedBehaviorSanitizer,
// on the CPU (no GPU, no kernels): the alias detection, the size-class order,
// the block partition and the direct-mode lane planner are the intricate,
// index-heavy parts of the host pipeline (mirbft_amd/csrc/mirsha.cpp). This
// file includes mirsha.cpp itself so its internal functions are reachable, stubs
// the kernel launchers (never called here), and checks every result against a
// plain reference computed in this file, over random and edge-case inputs.
// Built by tests/cpp/Makefile (target asan) with g++ -fsanitize=address,undefined;
// run by tests/test_host_sanitize.py.
#include "../../mirbft_amd/csrc/mirsha.cpp"

#include <cstdio>
#include <map>
#include <random>

namespace msha {
// Kernel launchers are GPU code (kernels.hip); the host planning never launches.
bool plan_split(uint64_t, int, int, SplitPlan*) { return false; }
hipError_t launch_digest_batch(const uint8_t*, const uint64_t*, const uint64_t*, const uint32_t*,
                               const uint32_t*, uint64_t, uint8_t*, uint32_t*, int, int, hipStream_t,
                               const SplitPlan*, LaunchKind*) {
  abort();
}
hipError_t launch_digest_uniform(const uint8_t*, uint64_t, uint64_t, uint64_t, uint8_t*, uint32_t*, int,
                                 hipStream_t, LaunchKind*) {
  abort();
}
hipError_t launch_digest_of_digests(const uint8_t*, const uint32_t*, const uint64_t*, uint64_t, uint8_t*,
                                    uint32_t*, hipStream_t, const SplitPlan*, LaunchKind*) {
  abort();
}
}  // namespace msha

static int failures = 0;
#define CHECK(c, ...)                                     \
  do {                                                    \
    if (!(c)) {                                           \
      ++failures;                                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
    }                                                     \
  } while (0)

static std::vector<uint64_t> first_ref(const std::vector<uint64_t>& off, const std::vector<uint64_t>& len) {
  std::map<std::pair<uint64_t, uint64_t>, uint64_t> seen;
  std::vector<uint64_t> out(off.size());
  for (size_t i = 0; i < off.size(); ++i) out[i] = seen.emplace(std::make_pair(off[i], len[i]), i).first->second;
  return out;
}

static void check_alias(const char* name, const std::vector<uint64_t>& off, const std::vector<uint64_t>& len) {
  std::vector<uint64_t> uid, table, bucket;
  std::vector<uint32_t> tag;
  alias_uids(off.data(), len.data(), off.size(), uid, table, bucket, tag);
  const std::vector<uint64_t> exp = first_ref(off, len);
  size_t bad = 0;
  for (size_t i = 0; i < off.size(); ++i) bad += uid[i] != exp[i];
  CHECK(bad == 0, "alias %s: %zu of %zu wrong", name, bad, off.size());
}

static void alias_cases(std::mt19937_64& rng) {
  // forward only; a shared pool pointed back into (c5 shape, both table paths);
  // everything aliased; zero lengths at shared offsets; dense random repeats
  for (uint64_t n : {1ull, 2ull, 1000ull, 70000ull, (1ull << 20) + 5}) {
    std::vector<uint64_t> off(n), len(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
      len[i] = rng() % 700;
      off[i] = pos;
      pos += (len[i] + 15) & ~15ull;
    }
    check_alias("forward", off, len);
    for (uint64_t i = 0; i < n; ++i)
      if (rng() % 20 == 0) {  // 5 %: back into a 100-entry pool at the start
        const uint64_t p = rng() % 100;
        off[i] = p * 4096;
        len[i] = 1 + p * 13;
      } else {
        off[i] += 1 << 20;
      }
    check_alias("pool", off, len);
    for (uint64_t i = 0; i < n; ++i) {
      off[i] = (rng() % 64) * 16;
      len[i] = rng() % 3 == 0 ? 0 : 16;
    }
    check_alias("dense", off, len);
  }
  std::vector<uint64_t> off(5000, 128), len(5000, 7);
  check_alias("all_same", off, len);
}

static void order_cases(std::mt19937_64& rng) {
  for (uint64_t n : {0ull, 1ull, 777ull, 300000ull}) {
    for (uint64_t maxlen : {100ull, 5000ull, 1ull << 27}) {
      std::vector<uint64_t> len(n);
      for (auto& l : len) l = rng() % maxlen;
      std::vector<uint32_t> order(n), tmp;
      const uint64_t m = order_by_blocks_desc(len.data(), n, order.data(), tmp);
      CHECK(m == n, "order: %llu of %llu", (unsigned long long)m, (unsigned long long)n);
      std::vector<uint32_t> exp(n);
      for (uint64_t i = 0; i < n; ++i) exp[i] = (uint32_t)i;
      std::stable_sort(exp.begin(), exp.end(),
                       [&](uint32_t a, uint32_t b) { return blocks_for(len[a]) > blocks_for(len[b]); });
      CHECK(order == exp, "order n=%llu maxlen=%llu", (unsigned long long)n, (unsigned long long)maxlen);
    }
  }
}

// Plain sequential statement of the partition rule: bounds[s] = the first i
// whose block-range midpoint acc_i + b_i / 2 reaches total * s / k.
static std::vector<uint64_t> partition_ref(const std::vector<uint64_t>& len, uint32_t k) {
  const uint64_t n = len.size();
  std::vector<uint64_t> b(k + 1, 0);
  unsigned __int128 total = 0;
  for (uint64_t l : len) total += blocks_for(l);
  uint64_t i = 0, acc = 0;
  for (uint32_t s = 1; s < k; ++s) {
    while (i < n && (unsigned __int128)2 * k * acc + (unsigned __int128)k * blocks_for(len[i]) < 2 * s * total)
      acc += blocks_for(len[i++]);
    b[s] = i;
  }
  b[k] = n;
  return b;
}

static void partition_cases(std::mt19937_64& rng) {
  // the threaded partition (chunk sums, one short scan per bound) against the
  // sequential rule, on batches large enough to run on several threads
  for (uint64_t n : {(1ull << 18) + 7, (1ull << 20) + 1})
    for (int shape = 0; shape < 3; ++shape)
      for (uint32_t k : {2u, 3u, 7u, 8u, 64u}) {
        std::vector<uint64_t> len(n);
        for (uint64_t i = 0; i < n; ++i)
          len[i] = shape == 0 ? 512 : shape == 1 ? rng() % 5000 : (i == n / 3 ? (1ull << 34) : rng() % 100);
        std::vector<uint64_t> b(k + 1);
        partition(len.data(), n, k, b.data());
        CHECK(b == partition_ref(len, k), "partition n=%llu shape=%d k=%u differs from the sequential rule",
              (unsigned long long)n, shape, k);
      }
  for (uint64_t n : {0ull, 1ull, 3ull, 100000ull})
    for (uint32_t k : {1u, 2u, 3u, 8u}) {
      std::vector<uint64_t> len(n), b(k + 1);
      uint64_t maxb = 0;
      for (auto& l : len) {
        l = rng() % 100000;
        maxb = std::max(maxb, blocks_for(l));
      }
      partition(len.data(), n, k, b.data());
      CHECK(b[0] == 0 && b[k] == n, "partition bounds");
      uint64_t lo = UINT64_MAX, hi = 0;
      for (uint32_t s = 0; s < k; ++s) {
        CHECK(b[s] <= b[s + 1], "partition monotone");
        uint64_t blk = 0;
        for (uint64_t i = b[s]; i < b[s + 1]; ++i) blk += blocks_for(len[i]);
        lo = std::min(lo, blk);
        hi = std::max(hi, blk);
      }
      CHECK(n < 1000 || hi - lo <= 2 * maxb, "partition balance %llu..%llu", (unsigned long long)lo,
            (unsigned long long)hi);
    }
}

// Direct-mode lane planner over a fake shard: granule map = identity over the
// span, lanes grouped by the 64 MiB upload chunk holding each payload's end,
// descending block count inside a group, stable, identity order detected.
static void direct_lane_cases(std::mt19937_64& rng) {
  for (int shape = 0; shape < 4; ++shape) {
    const uint64_t m = shape == 3 ? 5 : 200000;
    std::vector<uint64_t> off(m), len(m);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < m; ++i) {
      len[i] = shape == 0 ? 512 : (shape == 2 ? (rng() % 4) * 4096 + rng() % 64 : rng() % 2000);
      off[i] = pos;
      pos += (len[i] + 15) & ~15ull;
    }
    if (shape == 2) std::reverse(off.begin(), off.end());  // lanes descend through the span
    Device d;
    d.direct_glo = 0;
    d.direct_gshift = 16;
    const uint64_t nG = (pos >> 16) + 1;
    d.direct_map.resize(nG);
    for (uint64_t g = 0; g < nG; ++g) d.direct_map[g] = g << 16;
    d.arena_bytes = nG << 16;
    Plan P;
    P.m = m;
    P.lanes = m;
    P.perm.resize(m);
    std::vector<uint64_t> h_off(m), h_len(m), tdev;
    plan_direct_lanes(P, d, off.data(), len.data(), h_off.data(), h_len.data(), tdev);
    std::vector<uint8_t> seen(m, 0);
    bool perm_ok = true;
    for (uint64_t q = 0; q < m; ++q) {
      const uint32_t i = P.perm[q];
      perm_ok &= i < m && !seen[i];
      if (i < m) seen[i] = 1;
      perm_ok &= h_off[q] == off[i] && h_len[q] == len[i];
    }
    CHECK(perm_ok, "direct shape %d: not a permutation with matching metadata", shape);
    auto chunk = [&](uint64_t q) { return (h_off[q] + std::max<uint64_t>(h_len[q], 1) - 1) / kDirectChunk; };
    bool grouped = true;
    for (uint64_t q = 1; q < m; ++q) {
      const uint64_t c0 = chunk(q - 1), c1 = chunk(q);
      grouped &= c1 >= c0;
      if (c1 == c0) {
        const uint64_t b0 = blocks_for(h_len[q - 1]), b1 = blocks_for(h_len[q]);
        grouped &= b1 <= b0 && (b1 < b0 || P.perm[q] > P.perm[q - 1]);
      }
    }
    CHECK(grouped, "direct shape %d: not grouped by chunk / block order / stable", shape);
    CHECK(P.lane_cut.front() == 0 && P.lane_cut.back() == m && P.cut_chunk.size() + 1 == P.lane_cut.size(),
          "direct shape %d: lane groups", shape);
    for (size_t g = 0; g + 1 < P.lane_cut.size(); ++g)
      for (uint64_t q = P.lane_cut[g]; q < P.lane_cut[g + 1]; q += 997)
        CHECK(chunk(q) == P.cut_chunk[g], "direct shape %d: lane %llu outside its group's chunk", shape,
              (unsigned long long)q);
    CHECK(shape != 0 || !P.ordered, "a uniform ascending request batch keeps identity lanes");
    if (P.ordered) {  // streamed D2H: later_min[g] = lowest slot written by groups >= g
      plan_stream_back(P);
      const size_t G = P.lane_cut.size() - 1;
      bool ok = P.later_min.size() == G + 1 && P.later_min[G] == m;
      uint64_t mn = m;
      for (size_t g = G; g-- > 0 && ok;) {
        for (uint64_t q = P.lane_cut[g]; q < P.lane_cut[g + 1]; ++q) mn = std::min<uint64_t>(mn, P.perm[q]);
        ok &= P.later_min[g] == mn;
      }
      CHECK(ok, "direct shape %d: later_min is not the suffix minimum of the groups' slots", shape);
      CHECK(shape != 2 || P.later_min[1] == 0, "reversed lanes: nothing is final before the last group");
    }
  }
}

// A context over several physical GPUs runs its whole-batch phases on a pool of
// its full host-thread share (guarded() installs it for the call, then restores
// the caller's pool); alias detection on it matches the reference.
static void wide_pool_case(std::mt19937_64& rng) {
  setenv("MSHA_HOST_THREADS", "12", 1);
  {
    msha_ctx ctx;
    ctx.devs.resize(2);
    ctx.devs[0].id = 0;
    ctx.devs[1].id = 1;  // two physical GPUs: host_threads_total = 12 (the override)
    unsigned seen = 0;
    const int rc = guarded(&ctx, [&] { seen = plan_threads(1u << 20); });
    CHECK(rc == MSHA_OK && seen == 12, "wide pool: %u threads (rc %d)", seen, rc);
    CHECK(tl_pool == nullptr, "wide pool: caller's pool not restored");
    const uint64_t n = (1u << 20) + 3;
    std::vector<uint64_t> off(n), len(n);
    for (uint64_t i = 0; i < n; ++i) {
      len[i] = rng() % 300;
      off[i] = rng() % 16 == 0 ? (rng() % 64) * 512 : (1u << 20) + 512 * i;
    }
    guarded(&ctx, [&] { check_alias("wide pool", off, len); });
  }
  unsetenv("MSHA_HOST_THREADS");
}

int main() {
  std::mt19937_64 rng(0x4D49524246540000ull);
  alias_cases(rng);
  wide_pool_case(rng);
  order_cases(rng);
  partition_cases(rng);
  direct_lane_cases(rng);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("host planning: all checks passed\n");
  return 0;
}
