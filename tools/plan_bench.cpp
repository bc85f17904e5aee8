// Host-only timing of the planning steps of msha_digest_batch on a c5-shaped
// batch (8M messages: 70% 512 B, 25% k x 32 B, 5% aliases of 100 ~49 KB
// payloads). No GPU: the helpers are compiled straight from mirsha.cpp. First
// the pageable path's host planning (alias table, size-class order, placement),
// then the pinned path's whole host share (the scan, and per shard the marking
// pass and granule map; its lanes are planned on the GPU, plan.hip) at 1 and 8
// shards, each shard on the pool the library would give it.
// Build: g++ -O3 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Wno-subobject-linkage \
//        -o tools/plan_bench tools/plan_bench.cpp -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -pthread
#include "../mirbft_amd/csrc/mirsha.cpp"

#include <cstdio>
#include <map>
#include <random>

// The launchers live in kernels.hip; this host-only harness never launches.
namespace msha {
bool plan_split(uint64_t, int, int, SplitPlan*, int) { return false; }
hipError_t launch_plan(const PlanArgs&, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_digest_batch(const uint8_t*, const uint64_t*, const uint64_t*, const uint32_t*,
                               const uint32_t*, uint64_t, uint8_t*, uint32_t*, int, int, hipStream_t,
                               const SplitPlan*, LaunchKind*, const LaneGate*) {
  return hipErrorNotSupported;
}
hipError_t launch_fold_plan(const FoldArgs&, hipStream_t, hipEvent_t) { return hipErrorNotSupported; }
hipError_t launch_fold_longs(const FoldArgs&, int, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_fold_fill(const uint32_t*, uint64_t, uint8_t*, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_clock_probe(uint32_t, uint32_t, uint64_t*, uint32_t*, hipStream_t) { return hipErrorNotSupported; }
bool uses_coop(uint64_t, int, int) { return false; }
hipError_t launch_digest_uniform(const uint8_t*, uint64_t, uint64_t, uint64_t, uint8_t*, uint32_t*, int,
                                 hipStream_t, LaunchKind*) {
  return hipErrorNotSupported;
}
hipError_t launch_digest_of_digests(const uint8_t*, const uint32_t*, const uint64_t*, uint64_t, uint8_t*,
                                    uint32_t*, hipStream_t, const SplitPlan*, LaunchKind*) {
  return hipErrorNotSupported;
}
}  // namespace msha

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 23);
  std::vector<uint64_t> off(n), len(n);
  std::mt19937_64 rng(1);
  uint64_t pool_off[100], pool_len[100], pos = 0;
  for (int j = 0; j < 100; ++j) { pool_len[j] = 30000 + rng() % 40000; pool_off[j] = pos; pos += round16(pool_len[j]); }
  for (uint64_t i = 0; i < n; ++i) {
    const double r = (rng() >> 11) * 0x1.0p-53;
    if (r < 0.95) { len[i] = r < 0.70 ? 512 : 32 * (1 + rng() % 20); off[i] = pos; pos += round16(len[i]); }
    else { const int j = rng() % 100; off[i] = pool_off[j]; len[i] = pool_len[j]; }
  }
  auto T = [](const char* what, double t0) { std::printf("%-28s %8.1f ms\n", what, now_ms() - t0); return now_ms(); };
  double t = now_ms();
  uint64_t lo = UINT64_MAX, hi = 0, sum = 0, blocks = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (len[i] > pos || off[i] > pos - len[i]) return 1;
    lo = std::min(lo, off[i]); hi = std::max(hi, off[i] + len[i]); sum += len[i]; blocks += blocks_for(len[i]);
  }
  t = T("validate+span+blocks", t);
  std::vector<uint64_t> uid;
  std::vector<uint64_t> table, bucket;
  std::vector<uint32_t> tags;
  for (int rep_i = 0; rep_i < 3; ++rep_i) {  // later rounds: buffers warm (as in a context)
    alias_uids(off.data(), len.data(), n, uid, table, bucket, tags);
    t = T("alias_uids", t);
  }
  {  // check against a plain map: uid[i] = first index with the same (off, len)
    std::map<std::pair<uint64_t, uint64_t>, uint64_t> first;
    for (uint64_t i = 0; i < n; ++i) {
      auto it = first.emplace(std::make_pair(off[i], len[i]), i).first;
      if (uid[i] != it->second) { std::printf("alias mismatch at %llu\n", (unsigned long long)i); return 2; }
    }
    t = T("(check vs std::map)", t);
  }
  std::vector<uint32_t> rep(n);
  uint64_t lanes = 0;
  for (uint64_t i = 0; i < n; ++i) { rep[i] = (uint32_t)uid[i]; lanes += uid[i] == i; }
  t = T("rep", t);
  std::vector<uint32_t> perm(lanes), tmp;
  order_by_blocks_desc(len.data(), n, perm.data(), tmp, rep.data());
  t = T("order_by_blocks_desc(subset)", t);
  std::vector<uint64_t> h_off(lanes), h_len(lanes), ppos(lanes);
  uint64_t acc = 0;
  for (uint64_t q = 0; q < lanes; ++q) { const uint32_t i = perm[q]; ppos[q] = acc; h_off[q] = acc; h_len[q] = len[i]; acc += round16(len[i]); }
  t = T("placement", t);
  std::printf("n=%llu lanes=%llu\n", (unsigned long long)n, (unsigned long long)lanes);
  // The pinned path's host share (run_direct): scan, then per shard mark + map.
  for (uint32_t k : {1u, 8u}) {
    for (int rep_i = 0; rep_i < 2; ++rep_i) {
      t = now_ms();
      BatchScan sc;
      scan_batch(reinterpret_cast<const uint8_t*>(uintptr_t(4096)), pos, off.data(), len.data(), n, sc);
      const double t_scan = now_ms() - t;
      std::vector<uint64_t> bounds(k + 1);
      partition_pieces(len.data(), n, k, sc.csum, bounds.data());
      unsigned gs = 16;
      while (((sc.hi - (sc.lo & ~((1ull << gs) - 1))) >> gs) >= (1ull << 20)) ++gs;
      const uint64_t glo = sc.lo & ~((1ull << gs) - 1), nG = ((sc.hi - glo) >> gs) + 1;
      // each shard on a pool of its share of the process pool's threads, side by side
      const unsigned per = std::max(1u, WorkerPool::get().size() / k);
      std::vector<std::unique_ptr<WorkerPool>> pools;
      for (uint32_t s = 0; s < k; ++s) pools.emplace_back(new WorkerPool(per - 1));
      std::vector<double> done(k);
      const double t1 = now_ms();
      std::vector<std::thread> th;
      for (uint32_t s = 0; s < k; ++s)
        th.emplace_back([&, s] {
          tl_pool = k > 1 ? pools[s].get() : nullptr;
          const uint64_t a = bounds[s], m = bounds[s + 1] - a;
          std::vector<uint8_t> mark(nG, 0);
          const ShardSpan sh = stage_and_mark(off.data() + a, len.data() + a, m, glo, gs, nullptr, nullptr, mark,
                                              long_chain_blocks(sc.bmax, MSHA_KERNEL_AUTO));
          std::vector<uint64_t> gmap(sh.g1 - sh.g0 + 1);
          build_gmap(mark, sh.g0, gmap.size(), gs, gmap.data());
          done[s] = now_ms() - t1;
          tl_pool = nullptr;
        });
      for (auto& x : th) x.join();
      std::printf("pinned path host share, %u shard(s): scan %.1f ms, then mark+map per shard done after %.1f ms "
                  "(slowest of %u, %u threads each); host share %.1f ms\n",
                  k, t_scan, *std::max_element(done.begin(), done.end()), k, k > 1 ? per : WorkerPool::get().size(),
                  t_scan + *std::max_element(done.begin(), done.end()));
    }
  }
  return 0;
}
