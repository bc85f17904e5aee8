// Host planning code of libmirsha under AddressSanitizer + UndefinedBehaviorSanitizer,
// on the CPU (no GPU, no kernels): the alias detection, the size-class order,
// the batch scan and block partition, and the direct path's granule marking and
// upload enumeration are the intricate, index-heavy parts of the host pipeline
// (mirbft_amd/csrc/mirsha.cpp; the direct path's lane planning runs on the GPU,
// plan.hip, and is covered by the -m gpu tests). This
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
bool plan_split(uint64_t, int, int, SplitPlan*, int) { return false; }
hipError_t launch_digest_batch(const uint8_t*, const uint64_t*, const uint64_t*, const uint32_t*,
                               const uint32_t*, uint64_t, uint8_t*, uint32_t*, int, int, hipStream_t,
                               const SplitPlan*, LaunchKind*, const LaneGate*) {
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
hipError_t launch_plan(const PlanArgs&, hipStream_t) { abort(); }
hipError_t launch_fold_prefix(const FoldArgs&, hipStream_t) { abort(); }
hipError_t launch_fold_plan(const FoldArgs&, hipStream_t, hipEvent_t) { abort(); }
hipError_t launch_fold_longs(const FoldArgs&, int, hipStream_t) { abort(); }
hipError_t launch_fold_fill(const FoldArgs&, uint8_t*, hipStream_t) { abort(); }
hipError_t launch_clock_probe(uint32_t, uint32_t, uint64_t*, uint32_t*, hipStream_t) { abort(); }
bool uses_coop(uint64_t, int, int) { abort(); }
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

// scan_batch: the first bad message is reported; totals, bmax and the piece
// sums match a plain pass; the partition from its piece sums is the sequential rule.
static void scan_cases(std::mt19937_64& rng) {
  for (uint64_t n : {1ull, 5000ull, (1ull << 18) + 77}) {
    std::vector<uint64_t> off(n), len(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
      len[i] = rng() % 3 == 0 ? 0 : rng() % 9000;
      off[i] = pos;
      pos += (len[i] + 15) & ~15ull;
    }
    const uint64_t arena_len = pos + 64;
    BatchScan sc;
    scan_batch(reinterpret_cast<const uint8_t*>(uintptr_t(4096)), arena_len, off.data(), len.data(), n, sc);
    uint64_t lo = UINT64_MAX, hi = 0, sum = 0, blocks = 0, bmax = 0;
    for (uint64_t i = 0; i < n; ++i) {
      lo = std::min(lo, off[i]);
      hi = std::max(hi, off[i] + len[i]);
      sum += len[i];
      blocks += blocks_for(len[i]);
      bmax = std::max(bmax, blocks_for(len[i]));
    }
    CHECK(sc.lo == lo && sc.hi == hi && sc.sum == sum && sc.blocks == blocks && sc.bmax == bmax,
          "scan totals n=%llu", (unsigned long long)n);
    std::vector<uint64_t> cs;
    piece_sums(len.data(), n, cs);
    CHECK(cs == sc.csum, "scan piece sums n=%llu", (unsigned long long)n);
    for (uint32_t k : {1u, 3u, 8u}) {
      std::vector<uint64_t> b(k + 1);
      partition_pieces(len.data(), n, k, sc.csum, b.data());
      CHECK(b == partition_ref(len, k), "partition from scan n=%llu k=%u", (unsigned long long)n, k);
    }
    // two bad messages: the lower index is the one reported
    const uint64_t b1 = n / 2, b2 = n - 1;
    std::vector<uint64_t> bad = len;
    bad[b2] = arena_len + 1;
    bad[b1] = arena_len - off[b1] + 1;
    std::string what;
    try {
      scan_batch(nullptr, arena_len, off.data(), bad.data(), n, sc);
    } catch (const MshaError& e) {
      what = e.what();
    }
    CHECK(what == "message " + std::to_string(b1) + " [off+len] outside arena", "scan error: '%s'", what.c_str());
  }
}

// Direct path's host share over random shards: staged metadata, granule marks,
// the compacted device map and the upload enumeration. Simulated DMA: every
// upload piece is copied into a fake device arena; then each message's bytes
// must sit at its remapped device offset, no upload may read outside the
// caller's arena (a zero-length message at its very end included) or cross a
// 64 MiB device piece, and lanes whose payload ends in piece c are complete once
// the uploads that end at or below (c+1) * 64 MiB are.
static void direct_upload_cases(std::mt19937_64& rng) {
  for (int shape = 0; shape < 12; ++shape) {
    // shapes 6..11: shapes 0..5 with long chains marked (their granules go up first)
    const uint64_t long_blocks = shape >= 6 ? 256 : 0;
    const int sh_kind = shape % 6;
    const uint64_t n = sh_kind == 4 ? 3 : 40000;
    std::vector<uint64_t> off(n), len(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
      len[i] = sh_kind == 0 ? 512 : rng() % 5000;
      if (sh_kind == 1 && rng() % 7 == 0) len[i] = 0;
      if (sh_kind == 5 && rng() % 100 == 0) len[i] = 16000 + rng() % 90000;  // long chains, scattered
      off[i] = pos;
      pos += (len[i] + 15) & ~15ull;
      if (sh_kind == 3 && rng() % 100 == 0) pos += rng() % (3u << 20);  // gaps: untouched granules
    }
    if (sh_kind == 2)  // an aliased pool at the start (c5 shape): 5% point back into it
      for (uint64_t i = 0; i < n; ++i)
        if (rng() % 20 == 0) {
          off[i] = (rng() % 50) * 4096;
          len[i] = 1 + rng() % 4000;
        }
    const uint64_t arena_len = pos;
    off[n - 1] = arena_len;  // a zero-length message exactly at the arena's end
    len[n - 1] = 0;
    std::vector<uint8_t> host(arena_len + 1);
    for (auto& b : host) b = (uint8_t)rng();
    BatchScan sc;
    scan_batch(host.data(), arena_len, off.data(), len.data(), n, sc);
    unsigned gs = sh_kind == 3 ? 12 : 16;  // small granules: many runs
    const uint64_t glo = sc.lo & ~((1ull << gs) - 1);
    const uint64_t nG = ((sc.hi - glo) >> gs) + 1;
    // the shard: the second half of the batch (a sub-range like a real shard)
    const uint64_t a = n / 2, m = n - a;
    std::vector<uint64_t> h_off(m), h_len(m);
    std::vector<uint8_t> mark(nG, 0);
    const ShardSpan sh =
        stage_and_mark(off.data() + a, len.data() + a, m, glo, gs, h_off.data(), h_len.data(), mark, long_blocks);
    bool staged = true;
    for (uint64_t i = 0; i < m; ++i) staged &= h_off[i] == off[a + i] && h_len[i] == len[a + i];
    CHECK(staged, "direct shape %d: staged metadata differs", shape);
    CHECK(sh.any(), "direct shape %d: no payload", shape);
    {  // backward: some message starts at or below an earlier one (may alias)
      bool back = false;
      uint64_t mx = 0;
      for (uint64_t i = 0; i < m; ++i) {
        back |= i > 0 && off[a + i] <= mx;
        mx = i ? std::max(mx, off[a + i]) : off[a + i];
      }
      CHECK(sh.backward == back, "direct shape %d: backward %d, want %d", shape, (int)sh.backward, (int)back);
      CHECK(sh_kind != 2 || back, "direct shape %d: the aliased pool is not seen", shape);
      CHECK(sh_kind != 0 || !back, "direct shape %d: a forward batch flagged", shape);
    }
    const uint64_t gbase = sh.g0, ng = sh.g1 - sh.g0 + 1;
    std::vector<uint64_t> gmap(ng);
    const uint64_t dev_bytes = build_gmap(mark, gbase, ng, gs, gmap.data());
    std::vector<uint8_t> dev(dev_bytes + 64, 0xEE);
    uint64_t last_end = 0;
    bool inside = true, ascending = true, in_piece = true;
    for_each_upload(gmap.data(), mark, ng, gbase, glo, gs, sh.lo, sh.hi, [&](uint64_t p, uint64_t d, uint64_t bytes) {
      inside &= bytes > 0 && p + bytes <= arena_len && d + bytes <= dev_bytes;
      ascending &= d >= last_end;
      in_piece &= d / kDirectChunk == (d + bytes - 1) / kDirectChunk;
      last_end = d + bytes;
      if (p + bytes <= arena_len && d + bytes <= dev_bytes) std::memcpy(dev.data() + d, host.data() + p, bytes);
    });
    CHECK(inside, "direct shape %d: an upload reads past the arena or writes past the device span", shape);
    CHECK(ascending && in_piece, "direct shape %d: uploads not ascending / crossing a 64 MiB piece", shape);
    const uint64_t G = 1ull << gs;
    uint64_t bad = 0;
    for (uint64_t i = 0; i < m; ++i) {
      const uint64_t o = h_off[i], l = h_len[i];
      if (!l) continue;
      const uint64_t r = o - glo;
      const uint64_t dv = gmap[(r >> gs) - gbase] + (r & (G - 1));
      bad += dv == UINT64_MAX || dv + l > dev_bytes || std::memcmp(dev.data() + dv, host.data() + o, l) != 0;
    }
    CHECK(bad == 0, "direct shape %d: %llu messages not intact at their device offset", shape,
          (unsigned long long)bad);
    if (long_blocks) {  // every long payload lies in the device prefix the long granules fill
      uint64_t long_bytes = 0, late = 0, longs = 0;
      for (uint64_t g = 0; g < ng; ++g) long_bytes += (mark[gbase + g] & kMarkLong) ? G : 0;
      for (uint64_t i = 0; i < m; ++i) {
        const uint64_t o = h_off[i], l = h_len[i];
        if (!l || blocks_for(l) < long_blocks) continue;
        ++longs;
        const uint64_t r = o - glo;
        late += gmap[(r >> gs) - gbase] + (r & (G - 1)) + l > long_bytes;
      }
      CHECK(late == 0 && (sh_kind != 5 || longs > 0), "direct shape %d: %llu of %llu long payloads not first",
            shape, (unsigned long long)late, (unsigned long long)longs);
    }
    if (sh_kind == 2) {  // the pool's granules are uploaded, the first half's own bytes are not
      uint64_t total = 0;
      for_each_upload(gmap.data(), mark, ng, gbase, glo, gs, sh.lo, sh.hi,
                      [&](uint64_t, uint64_t, uint64_t b) { total += b; });
      CHECK(total < arena_len * 3 / 4, "direct shape 2: %llu of %llu bytes uploaded for half the batch",
            (unsigned long long)total, (unsigned long long)arena_len);
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
    ctx.devs[1].id = 1;  // two physical GPUs: host_threads_total = 12 (the override), at most the machine's
    const unsigned want = std::min(12u, std::max(1u, std::thread::hardware_concurrency()));
    unsigned seen = 0;
    const int rc = guarded(&ctx, [&] { seen = plan_threads(1u << 20); });
    CHECK(rc == MSHA_OK && (seen == want || (want <= 16 && seen == WorkerPool::get().size())),
          "wide pool: %u threads, want %u (rc %d)", seen, want, rc);
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
  scan_cases(rng);
  direct_upload_cases(rng);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("host planning: all checks passed\n");
  return 0;
}
