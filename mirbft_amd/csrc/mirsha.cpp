// libmirsha: host side of the MI355X batched SHA-256 engine (C ABI in include/mirsha.h).
//
// One call == one processor.ProcessHashActions over a whole ActionList
// (/root/reference/pkg/processor/serial.go:180-198): validate, pack into
// pinned staging, shard across the context's GPUs by cumulative block count,
// H2D per shard on that GPU's stream, one kernel launch per shard, D2H of the
// digests, join. There is no collective and no CPU hashing anywhere here.
#include <hip/hip_runtime.h>

#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <functional>
#include <condition_variable>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mirsha.h"
#include "kernels.hpp"

namespace {

struct MshaError : std::runtime_error {
  int code;
  MshaError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw MshaError(e_ == hipErrorOutOfMemory ? MSHA_ERR_OUT_OF_MEMORY : MSHA_ERR_HIP,     \
                      std::string(#expr) + ": " + hipGetErrorString(e_));                    \
  } while (0)

// Reason of the most recent failed context creation in the process
// (msha_last_error(NULL)). A fixed, always NUL-terminated buffer written under a
// mutex: a reader on another thread never sees freed memory. msha_ctx_create_err
// hands the reason back with the call instead (no cross-call state at all).
std::mutex g_create_mu;
char g_create_error[512] = "";

void set_create_error(const std::string& msg, char* errbuf, uint64_t errbuf_len) {
  {
    std::lock_guard<std::mutex> g(g_create_mu);
    std::snprintf(g_create_error, sizeof(g_create_error), "%s", msg.c_str());
  }
  if (errbuf && errbuf_len) std::snprintf(errbuf, (size_t)std::min<uint64_t>(errbuf_len, 1u << 20), "%s", msg.c_str());
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

inline uint64_t blocks_for(uint64_t len) { return (len >> 6) + ((len & 63) < 56 ? 1 : 2); }
inline uint64_t round16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// Growable device buffer (never shrinks; reallocation only between calls).
struct DevBuf {
  void* p = nullptr;
  uint64_t cap = 0;
  void ensure(uint64_t bytes) {
    if (bytes <= cap) return;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    cap = 0;
    uint64_t want = std::max<uint64_t>(bytes + bytes / 4, 4096);
    HIPCHK(hipMalloc(&p, want));
    cap = want;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// Growable pinned host buffer.
struct PinBuf {
  void* p = nullptr;
  uint64_t cap = 0;
  // hipHostMallocCoherent: the GPU reads and writes it over PCIe uncached (the
  // latency path's zero-copy buffers, which kernels access in place)
  unsigned flags = hipHostMallocPortable;
  void ensure(uint64_t bytes) {
    if (bytes <= cap) return;
    if (p) HIPCHK(hipHostFree(p));
    p = nullptr;
    cap = 0;
    uint64_t want = std::max<uint64_t>(bytes + bytes / 4, 4096);
    HIPCHK(hipHostMalloc(&p, want, flags));
    cap = want;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// Worker pool for those phases (thread creation would otherwise cost ~0.1 ms
// per thread per phase): one process-wide pool, plus one per GPU of a
// multi-GPU context for its gather thread (pageable arenas). run(T, job) calls
// job(t) for t in [0, T) on the workers and the calling thread, and returns
// when all are done. One run at a time: a caller that finds the pool busy
// (another context planning concurrently) runs its tasks on fresh threads.
class WorkerPool {
 public:
  static WorkerPool& get() {
    // 16 threads (one GPU's host share), or MSHA_HOST_THREADS; never above the machine's
    static WorkerPool pool([] {
      const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
      const char* env = getenv("MSHA_HOST_THREADS");
      const unsigned want = env ? (unsigned)std::max(1L, std::strtol(env, nullptr, 10)) : 16u;
      return std::min(want, hw) - 1;
    }());
    return pool;
  }
  explicit WorkerPool(unsigned helpers) {
    for (unsigned i = 0; i < helpers; ++i) workers_.emplace_back([this] { loop(); });
  }
  unsigned size() const { return (unsigned)workers_.size() + 1; }
  void run(unsigned T, const std::function<void(unsigned)>& job) {
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock() || workers_.empty()) {
      std::vector<std::thread> th;
      for (unsigned t = 1; t < T; ++t) th.emplace_back(job, t);
      job(0);
      for (auto& x : th) x.join();
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &job;
      ntasks_ = T;
      next_ = 0;
      pending_ = T;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
  }

 private:
  void work() {  // claim and run tasks of the current generation
    for (;;) {
      unsigned t;
      const std::function<void(unsigned)>* job;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!job_ || next_ >= ntasks_) return;
        t = next_++;
        job = job_;
      }
      (*job)(t);
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(unsigned)>* job_ = nullptr;
  unsigned ntasks_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Per-GPU state: stream, timing events, device buffers, pinned staging.
struct Device {
  int id = 0;
  uint32_t index = 0;  // shard number in the context
  int numa = -1;       // NUMA node of the GPU's PCI device (-1: unknown)
  int cus = 256;
  hipStream_t stream = nullptr;       // kernels (and everything on single-stream paths)
  hipStream_t copy_stream = nullptr;  // H2D of staged chunks, overlapping the kernels
  hipStream_t d2h_stream = nullptr;   // host calls: digests back, behind their kernels (ev_k);
                                      // only on a GPU no other shard shares (d2h_stream_after)
  hipEvent_t ev_k = nullptr;          // the latest hash launch of a host call
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // device_ms / upload_ms / kernel_ms of the last host call: first H2D (copy
  // stream) .. last H2D, first hash kernel .. last kernel (msha_shard_stats)
  hipEvent_t ev_up0 = nullptr, ev_up1 = nullptr, ev_k0 = nullptr;
  hipEvent_t ev_meta = nullptr, ev_plan = nullptr;  // direct path: metadata landed / GPU plan done
  hipEvent_t ev_p0 = nullptr, ev_p1 = nullptr;      // direct path: the planner kernels (plan_kernel_ms)
  hipEvent_t slot_free[2] = {nullptr, nullptr};  // staging slot s may be refilled
  hipEvent_t chunk_in = nullptr;                 // last chunk's bytes are on the device
  std::vector<hipEvent_t> span_ev;               // direct mode: upload piece c is on the device
  DevBuf arena, off, len, order, out, err, idx, begin, table;
  // pinned staging, allocated with this GPU current (the runtime's pool for its NUMA node)
  PinBuf h_arena, h_meta, h_out, slot[2];
  // small-call path (run_small): [meta | payload] in, [error word | digests] out
  DevBuf sm_in, sm_out;
  PinBuf sm_stage, sm_res;
  // zero-copy latency path: [meta | payload] and the digests in coherent pinned
  // memory the kernel reads and writes in place (no H2D, no D2H)
  PinBuf sm_zc_in{nullptr, 0, hipHostMallocPortable | hipHostMallocCoherent};
  PinBuf sm_zc_out{nullptr, 0, hipHostMallocPortable | hipHostMallocCoherent};
  // direct path, planned on the GPU (plan.hip): raw metadata, granule map,
  // device offsets, alias table and slots, representatives, bucket counters,
  // [gmin | cut | info] read back to h_small; rep read back to h_rep
  DevBuf p_meta, p_gmap, p_devoff, p_table, p_slot, p_rep, p_cnt, p_small;
  PinBuf h_gmap, h_small, h_rep;
  // planned device calls (msha_digest_batch_device_planned): alias table,
  // representatives, bucket counters, lane order, [lanes | head]; the head of
  // long chains runs on side_stream, forked from and joined to the caller's
  DevBuf f_table, f_rep, f_tmax, f_cnt, f_order, f_key, f_tkeys, f_longs;
  hipStream_t head_stream = nullptr;  // a folded call's early head (FoldArgs::longs)
  hipEvent_t ev_longs = nullptr, ev_join2 = nullptr, ev_hready = nullptr;
  uint32_t f_epoch = 0;  // the alias table's epoch tag of the last folded call (plan.hip fold_claim)
  DevBuf probe;  // msha_clock_probe: stamps + sink
  // direct path heads (launch_head): their digests, lane-indexed; read back with
  // their lanes' digest slots into h_head ([digests | slots])
  DevBuf p_head;
  PinBuf h_head;
  hipEvent_t ev_head = nullptr;  // the latest head launch (side stream)
  bool head_side = false;        // this call's heads went on side_stream
  hipStream_t side_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_fplan = nullptr, ev_join = nullptr, ev_fdone = nullptr;
  bool fdone_recorded = false;  // ev_fdone: the last planned call's work is queued behind it
  // per-call shard description
  uint64_t lo = 0, hi = 0;        // message/action range
  uint64_t arena_bytes = 0;       // staged arena size (without slack)
  std::vector<uint8_t> direct_mark;  // direct path: granules of the arena this shard touches
  msha_shard_stats st{};          // last host call (msha_get_shard_stats)
  // Multi-GPU host calls: this GPU's share of the host threads (its shard is
  // planned, and its pageable chunks gathered, on them) and planning scratch.
  std::unique_ptr<WorkerPool> gather_pool;
  std::vector<uint32_t> sort_tmp;
  std::vector<uint64_t> tmp_dev;
  // split chaining (kernels.hip): kSplitRing flag arrays of cus*2 entries,
  // allocated once and zeroed, never reallocated (launches may be in flight)
  uint64_t* split_flags = nullptr;
  uint64_t split_epoch = 0;
  void release() {
    gather_pool.reset();
    for (DevBuf* b : {&arena, &off, &len, &order, &out, &err, &idx, &begin, &table, &sm_in, &sm_out, &p_meta,
                      &p_gmap, &p_devoff, &p_table, &p_slot, &p_rep, &p_cnt, &p_small, &f_table, &f_rep,
                      &f_tmax, &f_cnt, &f_order, &f_key, &f_tkeys, &f_longs, &probe, &p_head})
      b->release();
    if (split_flags) (void)hipFree(split_flags);
    split_flags = nullptr;
    for (PinBuf* b : {&h_arena, &h_meta, &h_out, &slot[0], &slot[1], &sm_stage, &sm_res, &sm_zc_in, &sm_zc_out, &h_gmap, &h_small, &h_rep,
                      &h_head})
      b->release();
    for (hipEvent_t* e : {&ev0, &ev1, &ev_up0, &ev_up1, &ev_k0, &ev_meta, &ev_plan, &ev_p0, &ev_p1, &slot_free[0],
                          &slot_free[1], &chunk_in, &ev_fork, &ev_fplan, &ev_join, &ev_fdone, &ev_head,
                          &ev_longs, &ev_join2, &ev_hready}) {
      if (*e) (void)hipEventDestroy(*e);
      *e = nullptr;
    }
    for (hipEvent_t e : span_ev) (void)hipEventDestroy(e);
    span_ev.clear();
    if (stream) (void)hipStreamDestroy(stream);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    if (d2h_stream) (void)hipStreamDestroy(d2h_stream);
    if (side_stream) (void)hipStreamDestroy(side_stream);
    if (head_stream) (void)hipStreamDestroy(head_stream);
    if (ev_k) (void)hipEventDestroy(ev_k);
    ev_k = nullptr;
    stream = copy_stream = d2h_stream = side_stream = head_stream = nullptr;
  }
};

// Split-chaining plan for an n-message launch on d (nullptr: plain launch).
// Consecutive launches use different flag arrays of a ring and unique epochs,
// so a launch never reads another launch's flags.
constexpr uint64_t kSplitRing = 16;
const msha::SplitPlan* split_for(Device& d, uint64_t n, int policy, msha::SplitPlan& sp,
                                 int cap = msha::kMaxSegmentsArena) {
  if (!msha::plan_split(n, d.cus, policy, &sp, cap)) return nullptr;
  const uint64_t per = (uint64_t)d.cus * 2;  // plan_split: chains <= SIMDs / 2
  if (!d.split_flags) {
    HIPCHK(hipMalloc(&d.split_flags, kSplitRing * per * sizeof(uint64_t)));
    HIPCHK(hipMemset(d.split_flags, 0, kSplitRing * per * sizeof(uint64_t)));
  }
  sp.epoch = ++d.split_epoch;
  sp.flags = d.split_flags + (sp.epoch % kSplitRing) * per;
  return &sp;
}

// MSHA_TRACE=1: host-side phase timestamps (ms since the call began) on stderr.
inline bool trace_on() {
  static const bool on = getenv("MSHA_TRACE") != nullptr;
  return on;
}
inline void trace(const char* what, double t0) {
  if (trace_on()) fprintf(stderr, "[msha] %-24s %9.2f ms\n", what, now_ms() - t0);
}
// the same, for one shard's thread of a multi-shard call
inline void trace(const char* what, uint32_t shard, double t0) {
  if (trace_on()) fprintf(stderr, "[msha] shard %u %-16s %9.2f ms\n", shard, what, now_ms() - t0);
}

// Host planning of large batches runs on a few threads: [0, n) is split into
// T contiguous chunks and f(t, lo, hi) runs for each (T = 1 below 256 K items).
// The threads are those of the calling thread's pool: the process-wide one,
// or, while one GPU's shard of a multi-GPU call is planned on a thread of its
// own, that GPU's pool (tl_pool), so the shards are planned side by side.
thread_local WorkerPool* tl_pool = nullptr;
inline WorkerPool& cur_pool() { return tl_pool ? *tl_pool : WorkerPool::get(); }
inline unsigned plan_threads(uint64_t n) {
  if (n < (1u << 18)) return 1;
  return cur_pool().size();
}
template <class F>
void parallel_chunks(uint64_t n, unsigned T, F&& f) {
  if (T <= 1) {
    f(0u, (uint64_t)0, n);
    return;
  }
  const std::function<void(unsigned)> job = [&](unsigned t) { f(t, n * t / T, n * (t + 1) / T); };
  cur_pool().run(T, job);
}

// Descending-block-count permutation so every wavefront gets messages of equal
// length and no lane idles. Stable. Batches rarely hold more than a few dozen
// distinct block counts, so a one-pass counting sort over [0, max blocks]
// (scattered writes into that many sequential streams) is the common path;
// messages beyond 2^20 blocks (64 MiB) fall back to a two-pass LSD radix.
// rep (may be null): only messages with rep[i] == i are ordered (aliases of
// another message get no lane). Returns the number of entries written.
uint64_t order_by_blocks_desc(const uint64_t* len, uint64_t n, uint32_t* order,
                              std::vector<uint32_t>& tmp, const uint32_t* rep = nullptr) {
  auto keep = [&](uint64_t i) { return !rep || rep[i] == i; };
  const unsigned T0 = plan_threads(n);
  std::vector<uint64_t> tmax(T0, 0);
  parallel_chunks(n, T0, [&](unsigned t, uint64_t lo, uint64_t hi) {
    uint64_t b = 0;
    for (uint64_t i = lo; i < hi; ++i) b = std::max(b, blocks_for(len[i]));
    tmax[t] = b;
  });
  const uint64_t bmax = *std::max_element(tmax.begin(), tmax.end());
  if (bmax <= (1u << 20)) {
    // per-thread histograms only while all of them together stay small (at most
    // 2^20 counters: a wide pool of 128 threads must not zero and scan 128 x 64 K)
    const uint64_t B = bmax + 1;               // bucket j = block count bmax - j
    const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(T0, (1u << 20) / B));
    std::vector<uint64_t> cnt((uint64_t)T * B, 0);
    parallel_chunks(n, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
      uint64_t* c = cnt.data() + (uint64_t)t * B;
      for (uint64_t i = lo; i < hi; ++i)
        if (keep(i)) c[bmax - blocks_for(len[i])]++;
    });
    uint64_t run = 0;  // stable: bucket-major, then thread (= index) order
    for (uint64_t j = 0; j < B; ++j)
      for (unsigned t = 0; t < T; ++t) {
        const uint64_t c = cnt[(uint64_t)t * B + j];
        cnt[(uint64_t)t * B + j] = run;
        run += c;
      }
    parallel_chunks(n, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
      uint64_t* c = cnt.data() + (uint64_t)t * B;
      for (uint64_t i = lo; i < hi; ++i)
        if (keep(i)) order[c[bmax - blocks_for(len[i])]++] = (uint32_t)i;
    });
    return run;
  }
  uint64_t m = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (keep(i)) order[m++] = (uint32_t)i;
  std::vector<uint32_t> key(n);
  for (uint64_t i = 0; i < n; ++i)
    key[i] = 0xffffffffu - (uint32_t)std::min<uint64_t>(blocks_for(len[i]), 0xffffffffu);
  tmp.resize(m);
  uint32_t* src = order;
  uint32_t* dst = tmp.data();
  for (int shift = 0; shift < 32; shift += 16) {
    std::vector<uint64_t> cnt(65537, 0);
    for (uint64_t q = 0; q < m; ++q) cnt[((key[src[q]] >> shift) & 0xffff) + 1]++;
    for (int d = 0; d < 65536; ++d) cnt[d + 1] += cnt[d];
    for (uint64_t q = 0; q < m; ++q) dst[cnt[(key[src[q]] >> shift) & 0xffff]++] = src[q];
    std::swap(src, dst);
  }
  // two passes: result is back in `order`
  return m;
}

bool all_equal_blocks(const uint64_t* len, uint64_t n) {
  if (n == 0) return true;
  uint64_t b0 = blocks_for(len[0]);
  for (uint64_t i = 1; i < n; ++i)
    if (blocks_for(len[i]) != b0) return false;
  return true;
}

// Messages per counted piece of the partition: a bound's scan stays short.
constexpr uint64_t kPiece = 1u << 16;

// csum[p] = blocks of the messages before piece p (P + 1 entries), threaded.
void piece_sums(const uint64_t* len, uint64_t n, std::vector<uint64_t>& csum) {
  const uint64_t P = std::max<uint64_t>(1, (n + kPiece - 1) / kPiece);
  csum.assign(P + 1, 0);
  parallel_chunks(P, std::min<unsigned>(plan_threads(n), (unsigned)P), [&](unsigned, uint64_t p0, uint64_t p1) {
    for (uint64_t p = p0; p < p1; ++p) {
      uint64_t sum = 0;
      for (uint64_t i = p * kPiece, e = std::min(n, (p + 1) * kPiece); i < e; ++i) sum += blocks_for(len[i]);
      csum[p + 1] = sum;
    }
  });
  for (uint64_t p = 0; p < P; ++p) csum[p + 1] += csum[p];
}

// bounds[s] = the first message whose block-range midpoint reaches s/k of the
// total: acc_i + b_i / 2 >= total * s / k, in integers 2k acc_i + k b_i >=
// 2 s total (acc_i = blocks before i). Midpoints never decrease, so each bound
// lies in the one piece where the running count crosses the target: one short
// scan per bound over the piece sums (a serial pass over c5's 8 M messages cost
// 30-45 ms before any upload began).
void partition_pieces(const uint64_t* len, uint64_t n, uint32_t k, const std::vector<uint64_t>& csum,
                      uint64_t* bounds) {
  const uint64_t P = csum.size() - 1;
  using u128 = unsigned __int128;
  const u128 total = csum[P];
  auto bound = [&](uint32_t s) -> uint64_t {
    const u128 goal = 2 * (u128)s * total;
    // the last piece starting below the target (midpoints of earlier pieces are below it too)
    uint64_t p = 0;
    while (p + 1 < P && (u128)2 * k * csum[p + 1] < goal) ++p;
    const uint64_t a = p * kPiece, b = std::min(n, (p + 1) * kPiece);
    if ((u128)2 * k * csum[p] >= goal) return a;  // the piece's first message already reaches it
    uint64_t acc = csum[p];
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t bi = blocks_for(len[i]);
      if ((u128)2 * k * acc + (u128)k * bi >= goal) return i;
      acc += bi;
    }
    return b;
  };
  bounds[0] = 0;
  for (uint32_t s = 1; s < k; ++s) bounds[s] = bound(s);
  bounds[k] = n;
}

void partition(const uint64_t* len, uint64_t n, uint32_t k, uint64_t* bounds) {
  if (k == 1) {
    bounds[0] = 0;
    bounds[1] = n;
    return;
  }
  std::vector<uint64_t> csum;
  piece_sums(len, n, csum);
  partition_pieces(len, n, k, csum, bounds);
}

// Direct-mode uploads go out in device-space pieces of this size, each with its
// own event, so kernels over the lanes whose payloads have landed start while
// the rest is still crossing PCIe (and their digests come back meanwhile).
constexpr uint64_t kDirectChunk = 1ull << msha::kDirectChunkShift;

// Per-GPU plan of one host-memory call (kept in the context: its vectors are
// reused call after call, so planning does not page-fault fresh memory).
struct Plan {
  uint64_t m = 0;
  bool ordered = false;
  std::vector<uint32_t> perm;       // sorted lane -> shard-local message (pageable path)
  std::vector<uint64_t> lane_cut;   // group boundaries in sorted lanes
  size_t next = 0;                  // next group to issue
  uint64_t launched = 0;            // lanes [0, launched) have a kernel enqueued
  uint64_t lanes = 0;               // messages that get a lane (one per distinct payload)
  std::vector<uint32_t> rep;        // shard-local message -> its lane's message (empty: identity)
  const uint32_t* rep_dev = nullptr;  // direct path: the same, planned on the GPU (pinned copy)
  std::vector<uint64_t> cut_chunk;  // direct mode: upload piece lane group g waits for
  // direct mode: later_min[g] = the lowest message any lane of groups >= g
  // writes (later_min[groups] = m), so once groups < g are hashed the digest
  // slots below later_min[g] are final; d2h_done = slots already D2H'd
  std::vector<uint64_t> later_min;
  uint64_t d2h_done = 0;
  // direct mode: lanes [0, head) are long chains run as heads (launch_head),
  // their digests lane-indexed in Device::p_head, placed by finish_shard
  uint64_t head = 0;
  bool k0 = false;  // the shard's first kernel is queued (Device::ev_k0 recorded)
  bool identity() const { return !ordered && rep.empty(); }  // lane q hashes message q
  const uint32_t* rep_of() const { return rep_dev ? rep_dev : (rep.empty() ? nullptr : rep.data()); }
};

}  // namespace

struct msha_ctx {
  // Calls on one context are serialised here (a second caller waits), so a
  // context may be shared between threads; distinct contexts run concurrently.
  mutable std::mutex mu;
  std::vector<Device> devs;
  char err[512] = "";  // last failure on the context (fixed buffer: msha_last_error's pointer stays valid)
  msha_stats stats{};
  // allocations handed out by msha_pinned_alloc: (pointer, mapped bytes), 0 =
  // hipHostMalloc, else an mmap striped over NUMA nodes and hipHostRegister'ed
  std::vector<std::pair<void*, uint64_t>> pinned;
  std::vector<uint64_t> tmp_len;
  int kernel_policy = MSHA_KERNEL_AUTO;
  // host planning buffers reused across calls
  std::vector<Plan> plans;
  std::vector<uint64_t> uid;
  std::vector<uint64_t> alias_table, alias_bucket;
  std::vector<uint32_t> alias_tag;
  // Several physical GPUs: the whole-batch planning phases (validation, alias
  // detection, upload marking) run on a pool of the context's full host-thread
  // share (host_threads_total) instead of the process-wide 16; made on first use.
  std::unique_ptr<WorkerPool> wide;
};

namespace {

int fail(msha_ctx* ctx, int code, const std::string& msg) {
  if (ctx) std::snprintf(ctx->err, sizeof(ctx->err), "%s", msg.c_str());
  return code;
}

// Host threads for a call on ctx: 16 per physical GPU (virtual shards of one
// GPU share its 16), at most the machine's, MSHA_HOST_THREADS overriding. On an
// 8-GPU node each shard then plans its 1/8 of the batch on 16 threads, as one
// GPU plans a whole batch, so planning stays under each link's shorter upload.
unsigned host_threads_total(const msha_ctx* ctx) {
  std::vector<int> ids;
  for (const Device& d : ctx->devs)
    if (std::find(ids.begin(), ids.end(), d.id) == ids.end()) ids.push_back(d.id);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const char* env = getenv("MSHA_HOST_THREADS");
  const unsigned want = env ? (unsigned)std::max(1L, std::strtol(env, nullptr, 10))
                            : 16u * (unsigned)std::max<size_t>(ids.size(), 1);
  return std::min(want, hw);
}

template <class F>
int guarded(msha_ctx* ctx, F&& f) {
  struct PoolScope {  // the context's wide pool for this call's whole-batch phases
    WorkerPool* prev = tl_pool;
    explicit PoolScope(msha_ctx* c) {
      if (c && !c->devs.empty()) {
        const unsigned total = host_threads_total(c);
        if (!c->wide && total > WorkerPool::get().size()) c->wide.reset(new WorkerPool(total - 1));
        if (c->wide) tl_pool = c->wide.get();
      }
    }
    ~PoolScope() { tl_pool = prev; }
  };
  try {
    PoolScope scope(ctx);
    f();
    if (ctx) ctx->err[0] = '\0';
    return MSHA_OK;
  } catch (const MshaError& e) {
    return fail(ctx, e.code, e.what());
  } catch (const std::bad_alloc&) {
    return fail(ctx, MSHA_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(ctx, MSHA_ERR_HIP, e.what());
  } catch (...) {
    return fail(ctx, MSHA_ERR_HIP, "unknown error");
  }
}

// Split [0, n) into nearly equal contiguous pieces and run f(lo, hi) on the
// threads of `pool` (gathering into pinned staging is host-bandwidth bound).
template <class F>
void parallel_ranges(WorkerPool& pool, uint64_t n, uint64_t bytes, F&& f) {
  unsigned t = (unsigned)std::min<uint64_t>({(uint64_t)pool.size(), bytes / (4u << 20) + 1, n});
  if (t <= 1) {
    f(0, n);
    return;
  }
  const std::function<void(unsigned)> job = [&](unsigned k) { f(n * k / t, n * (k + 1) / t); };
  pool.run(t, job);
}

// Count a kernel launch in the context's counters (atomically: the pageable
// multi-GPU path launches from one thread per GPU) and in the shard's.
void count_launch(msha_ctx* ctx, Device* d, msha::LaunchKind kind) {
  uint64_t* f = nullptr;
  switch (kind) {
    case msha::kLaunchLane: f = &ctx->stats.launches_lane; break;
    case msha::kLaunchPipe: f = &ctx->stats.launches_pipe; break;
    case msha::kLaunchCoop: f = &ctx->stats.launches_coop; break;
    case msha::kLaunchSplit: f = &ctx->stats.launches_split; break;
    case msha::kLaunchDod: f = &ctx->stats.launches_dod; break;
    case msha::kLaunchChain2:
      f = &ctx->stats.launches_coop;
      __atomic_fetch_add(&ctx->stats.launches_chain2, 1, __ATOMIC_RELAXED);
      break;
    case msha::kLaunchChain8:
      f = &ctx->stats.launches_coop;
      __atomic_fetch_add(&ctx->stats.launches_chain8, 1, __ATOMIC_RELAXED);
      break;
    case msha::kLaunchLaneWs:
      f = &ctx->stats.launches_lane;
      __atomic_fetch_add(&ctx->stats.launches_lane_ws, 1, __ATOMIC_RELAXED);
      break;
    default: return;
  }
  __atomic_fetch_add(f, 1, __ATOMIC_RELAXED);
  if (d) d->st.launches++;
}

// Runs f(s) for every shard s of the context: inline for one shard; for
// several, one thread per shard, each with its GPU's share of the host threads
// as its planning pool (tl_pool), so per-GPU work (upload queueing, lane
// planning, pageable gathers) proceeds side by side. Rethrows the first error.
template <class F>
void for_each_shard(msha_ctx* ctx, F&& f) {
  const uint32_t k = (uint32_t)ctx->devs.size();
  if (k == 1) {
    f(0u);
    return;
  }
  const unsigned per = std::max(1u, host_threads_total(ctx) / k);
  for (Device& d : ctx->devs)
    if (!d.gather_pool || d.gather_pool->size() != per) d.gather_pool.reset(new WorkerPool(per - 1));
  std::vector<std::exception_ptr> errs(k);
  std::vector<std::thread> th;
  for (uint32_t s = 0; s < k; ++s)
    th.emplace_back([&, s] {
      tl_pool = ctx->devs[s].gather_pool.get();
      try {
        f(s);
      } catch (...) {
        errs[s] = std::current_exception();
      }
      tl_pool = nullptr;
    });
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// Device entry points: the context's first device, its error word zeroed once.
void device_prologue(msha_ctx* ctx, void* stream, hipStream_t* st) {
  if (ctx->devs.empty()) throw MshaError(MSHA_ERR_INVALID_ARG, "context has no device");
  Device& d = ctx->devs[0];
  HIPCHK(hipSetDevice(d.id));
  if (!d.err.p) {  // first device call: a zeroed error word (hipMalloc does not zero)
    d.err.ensure(4);
    HIPCHK(hipMemset(d.err.p, 0, 4));
  }
  *st = stream ? static_cast<hipStream_t>(stream) : d.stream;
}

// Is p inside page-locked host memory the GPU can DMA from (hipHostMalloc /
// hipHostRegister)? Pageable memory makes the query fail; clear that error.
bool is_pinned_host(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// NUMA node of GPU dev: its PCI device's numa_node in sysfs (-1: unknown).
int gpu_numa_node(int dev) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  char path[192];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

// Does msha_pinned_alloc stripe its allocations over NUMA nodes? When the
// context's GPUs sit on two or more nodes; MSHA_PINNED_STRIPE=1 forces it (a
// one-node box exercises the path), =0 turns it off.
bool stripe_pinned(const msha_ctx* ctx) {
  if (const char* e = getenv("MSHA_PINNED_STRIPE")) return atoi(e) != 0;
  for (const Device& d : ctx->devs)
    if (d.numa >= 0 && d.numa != ctx->devs[0].numa) return true;
  return false;
}

// A pinned allocation for a multi-socket context: cut into one region per shard,
// in shard order, each preferring its shard's GPU's NUMA node (mbind), touched,
// then page-locked for every GPU (hipHostRegister, portable). A caller that packs
// a batch in message order (the Go adapter) then has each GPU's span -- shards
// are contiguous message ranges -- mostly in its own socket's memory, instead of
// every link reading one socket's. nullptr when a step fails (the caller then
// takes hipHostMalloc); *mapped = the mapping's size.
void* striped_pinned_alloc(const msha_ctx* ctx, uint64_t bytes, uint64_t* mapped) {
  constexpr uint64_t kAlign = 2ull << 20;  // region edges on huge-page boundaries
  const uint64_t size = (std::max<uint64_t>(bytes, 1) + kAlign - 1) & ~(kAlign - 1);
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  const uint64_t k = ctx->devs.size();
  for (uint64_t s = 0; s < k; ++s) {
    const int node = ctx->devs[s].numa;
    const uint64_t a = (size / k * s) & ~(kAlign - 1);
    const uint64_t b = s + 1 == k ? size : (size / k * (s + 1)) & ~(kAlign - 1);
    if (node < 0 || node >= 1024 || b <= a) continue;
    unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    constexpr int kMpolPreferred = 1;  // <linux/mempolicy.h>; best effort: no error if refused
    (void)syscall(SYS_mbind, static_cast<char*>(p) + a, b - a, kMpolPreferred, mask, 1024ul + 1, 0u);
  }
  // first touch places every page by its region's policy (several threads)
  parallel_ranges(WorkerPool::get(), size / kAlign, size, [&](uint64_t a, uint64_t b) {
    std::memset(static_cast<char*>(p) + a * kAlign, 0, (b - a) * kAlign);
  });
  if (hipHostRegister(p, size, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, size);
    return nullptr;
  }
  *mapped = size;
  return p;
}

void pinned_release(const std::pair<void*, uint64_t>& a) {
  if (a.second) {
    (void)hipHostUnregister(a.first);
    munmap(a.first, a.second);
  } else {
    (void)hipHostFree(a.first);
  }
}

inline uint32_t alias_tag(uint64_t off, uint64_t len) {
  uint64_t h = off ^ (len * 0x9E3779B97F4A7C15ull);  // splitmix64 finalizer over both fields
  h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
  h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((h ^ (h >> 31)) >> 32);
}

// uid[i] = the first index j <= i with (off[j], len[j]) == (off[i], len[i]).
//
// Candidates first: a message whose offset is greater than every earlier
// message's ("forward") cannot repeat an earlier payload, so uid[i] = i. Only
// the others (offset at or below an earlier one) can be aliases. A batch of
// requests and batches packed in order plus a shared pool of EpochChange
// payloads (c5: ~5 % of the actions point back into the pool) has few of them,
// so the table is built over the candidates only and the forward messages just
// probe it (each key has at most one forward message: its offset is unique),
// instead of inserting all n keys (c5, 8 M actions: 22 ms -> a few ms).
// With more than n/4 candidates the table simply takes every message.
//
// The table: open addressing (linear probing) over R regions picked by the key
// hash's top bits. Pass 1 hashes every key and counts keys per (index chunk,
// region); pass 2 scatters (tag << 32 | index) into per-region buckets, in
// index order; pass 3 builds each region's table on its own worker from its
// bucket alone, prefetching the slot of the key kPrefetch ahead (the probes are
// the cost: random accesses into a table far larger than the caches). A table
// entry is (tag << 32) | (index + 1); off/len are dereferenced only on a tag
// match, and "first" is preserved because a region inserts its keys in index order.
void alias_uids(const uint64_t* off, const uint64_t* len, uint64_t n, std::vector<uint64_t>& uid,
                std::vector<uint64_t>& table, std::vector<uint64_t>& bucket, std::vector<uint32_t>& tagv) {
  uid.resize(n);
  tagv.resize(n);
  const unsigned T = plan_threads(n);
  // forward messages (uid = self) and the candidate list, in index order
  std::vector<uint64_t> cmax(T, 0);
  parallel_chunks(n, T, [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t mx = 0;
    for (uint64_t i = a; i < b; ++i) mx = std::max(mx, off[i] + 1);
    cmax[t] = mx;
  });
  // the forward pass also hashes every key (the probe below reads the tags)
  // and copies each candidate's key out while it streams off/len
  struct Cand {
    std::vector<uint32_t> idx;
    std::vector<uint64_t> off, len;
  };
  std::vector<Cand> tcand(T);
  parallel_chunks(n, T, [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t run = 0;  // max(off + 1) over every earlier message
    for (unsigned u = 0; u < t; ++u) run = std::max(run, cmax[u]);
    Cand& c = tcand[t];
    for (uint64_t i = a; i < b; ++i) {
      tagv[i] = alias_tag(off[i], len[i]);
      if (off[i] + 1 > run) {
        uid[i] = i;
        run = off[i] + 1;
      } else {
        uid[i] = UINT64_MAX;  // candidate: resolved below
        c.idx.push_back((uint32_t)i);
        c.off.push_back(off[i]);
        c.len.push_back(len[i]);
      }
    }
  });
  uint64_t m = 0;
  for (auto& c : tcand) m += c.idx.size();
  if (m == 0) return;
  const bool subset = m <= n / 4;
  // Items of the table: the candidates (subset mode; their keys in compact
  // arrays, so the table build does not miss the cache on every key) or every
  // message. Item k's key is (ko[k], kl[k]); its message is cand[k] (or k).
  std::vector<uint32_t> cand;
  std::vector<uint64_t> cko, ckl;
  if (subset) {
    cand.resize(m);
    cko.resize(m);
    ckl.resize(m);
    std::vector<uint64_t> at(T + 1, 0);
    for (unsigned t = 0; t < T; ++t) at[t + 1] = at[t] + tcand[t].idx.size();
    const std::function<void(unsigned)> copy = [&](unsigned t) {
      const Cand& c = tcand[t];
      std::memcpy(cand.data() + at[t], c.idx.data(), 4 * c.idx.size());
      std::memcpy(cko.data() + at[t], c.off.data(), 8 * c.off.size());
      std::memcpy(ckl.data() + at[t], c.len.data(), 8 * c.len.size());
    };
    if (T == 1) copy(0);
    else WorkerPool::get().run(T, copy);
  } else {
    m = n;
  }
  tcand.clear();
  const uint64_t* ko = subset ? cko.data() : off;
  const uint64_t* kl = subset ? ckl.data() : len;
  bucket.resize(m);
  const unsigned rbits = m >= (1u << 20) ? 4 : 0;
  const unsigned R = 1u << rbits;  // regions (one pass-3 task each)
  const unsigned Tm = plan_threads(m);
  std::vector<uint64_t> cnt((size_t)Tm * R, 0);
  // item k's tag, then (subset mode) the table slot of its key; every
  // message's tag stays in tagv for the forward probe
  std::vector<uint32_t> ctag;
  std::vector<uint32_t>& tag_k = subset ? ctag : tagv;
  if (subset) ctag.resize(m);
  // pass 1: region histogram (subset mode: the candidates' tags, from their keys)
  parallel_chunks(m, Tm, [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t* c = cnt.data() + (size_t)t * R;
    for (uint64_t k = a; k < b; ++k) {
      const uint32_t tag = subset ? alias_tag(ko[k], kl[k]) : tagv[k];
      tag_k[k] = tag;
      ++c[rbits ? tag >> (32 - rbits) : 0];
    }
  });
  // bucket layout: region-major, chunk order inside a region (= index order)
  std::vector<uint64_t> rstart(R + 1, 0), base((size_t)Tm * R);
  {
    uint64_t acc = 0;
    for (unsigned r = 0; r < R; ++r) {
      rstart[r] = acc;
      for (unsigned t = 0; t < Tm; ++t) {
        base[(size_t)t * R + r] = acc;
        acc += cnt[(size_t)t * R + r];
      }
    }
    rstart[R] = acc;
  }
  // pass 2: scatter
  parallel_chunks(m, Tm, [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t* w = base.data() + (size_t)t * R;
    for (uint64_t k = a; k < b; ++k) {
      const uint32_t tag = tag_k[k];
      bucket[w[rbits ? tag >> (32 - rbits) : 0]++] = (uint64_t)tag << 32 | k;
    }
  });
  // per-region table capacity: a power of two >= 2x its keys
  std::vector<uint64_t> cap(R), tstart(R + 1, 0);
  for (unsigned r = 0; r < R; ++r) {
    uint64_t c = 16;
    while (c < 2 * (rstart[r + 1] - rstart[r])) c <<= 1;
    cap[r] = c;
    tstart[r + 1] = tstart[r] + c;
  }
  if (table.size() < tstart[R]) table.resize(tstart[R]);
  // pass 3: one task per region. first_k[k] = the first item with k's key;
  // in subset mode tag_k[k] becomes the global slot of k's key (for the
  // forward probe below).
  std::vector<uint32_t> first_k(subset ? m : 0);
  constexpr uint64_t kPrefetch = 16;
  const std::function<void(unsigned)> build = [&](unsigned r) {
    uint64_t* reg = table.data() + tstart[r];
    const uint64_t mask = cap[r] - 1;
    std::memset(reg, 0, cap[r] * sizeof(uint64_t));  // 0 = empty
    const uint64_t* bk = bucket.data() + rstart[r];
    const uint64_t cnt_r = rstart[r + 1] - rstart[r];
    for (uint64_t q = 0; q < cnt_r; ++q) {
      const uint64_t ahead = q + kPrefetch < cnt_r ? bk[q + kPrefetch] : bk[q];
      __builtin_prefetch(reg + ((ahead >> 32) & mask), 1);
      const uint64_t e0 = bk[q];
      const uint64_t k = e0 & 0xffffffffull, tag = e0 & 0xffffffff00000000ull;
      for (uint64_t p = (e0 >> 32) & mask;; p = (p + 1) & mask) {
        const uint64_t e = reg[p];
        uint64_t j = k;
        if (e == 0) {
          reg[p] = tag | (k + 1);
        } else {
          j = (e & 0xffffffffull) - 1;
          if ((e & 0xffffffff00000000ull) != tag || ko[j] != ko[k] || kl[j] != kl[k]) continue;
        }
        if (subset) {
          first_k[k] = (uint32_t)j;
          tag_k[k] = (uint32_t)(tstart[r] + p);
        } else {
          uid[k] = j;
        }
        break;
      }
    }
  };
  if (R == 1) build(0);
  else WorkerPool::get().run(R, build);
  if (!subset) return;
  // Forward messages that carry a candidate's key are its first occurrence
  // (an offset above every earlier one precedes every repeat of it). A 2^20-bit
  // filter over the candidates' tags (128 KiB, cache-resident) turns away
  // almost every forward message before it touches the table.
  std::vector<uint64_t> filter(1u << 14, 0);
  for (uint64_t g = 0; g < tstart[R]; ++g)
    if (table[g]) {
      const uint32_t tag = (uint32_t)(table[g] >> 32);
      filter[(tag >> 6) & 0x3fff] |= 1ull << (tag & 63);
    }
  std::vector<uint64_t> fwd(tstart[R], UINT64_MAX);
  parallel_chunks(n, T, [&](unsigned, uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      if (uid[i] != i) continue;  // candidates: resolved below
      const uint32_t tag = tagv[i];
      if (!((filter[(tag >> 6) & 0x3fff] >> (tag & 63)) & 1)) continue;
      const unsigned r = rbits ? tag >> (32 - rbits) : 0;
      const uint64_t* reg = table.data() + tstart[r];
      const uint64_t mask = cap[r] - 1;
      for (uint64_t p = tag & mask;; p = (p + 1) & mask) {
        const uint64_t e = reg[p];
        if (e == 0) break;
        const uint64_t j = (e & 0xffffffffull) - 1;
        if ((e >> 32) == tag && ko[j] == off[i] && kl[j] == len[i]) {
          fwd[tstart[r] + p] = i;  // i is forward: the first occurrence of the key
          break;
        }
      }
    }
  });
  parallel_chunks(m, Tm, [&](unsigned, uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; ++k) {
      const uint64_t f = fwd[tag_k[k]];
      uid[cand[k]] = f != UINT64_MAX ? f : cand[first_k[k]];
    }
  });
}

// Host-memory execution of one batch (the body of every host entry point):
//   shard messages [0, n) over the context's GPUs by cumulative block count;
//   per GPU, give one lane to each distinct payload (aliases fold into their
//   first occurrence), order lanes by descending block count (a wave's lanes
//   then run equal block counts), place the payloads at 16-byte aligned
//   offsets of the device arena, upload lane-indexed off/len + the lane ->
//   message map, and stream the payload in chunks through two pinned staging
//   slots: host threads gather chunk c+1 while chunk c's H2D runs on the copy
//   stream. Kernels (compute stream, event-ordered after their chunks) run over
//   accumulated chunks once these fill the GPU, or at the last chunk. Digests
//   come back with one D2H per GPU; aliases copy their representative's.
//   gather(i, dst) copies message i's bytes to dst.
constexpr uint64_t kChunkBytes = 32ull << 20;

// uid (may be null): messages with equal uid[i] have identical bytes (aliases,
// e.g. one EpochChange re-hashed N^2 times, epoch_target.go:486-505); their
// payload is copied and hashed once per GPU.
// t0: when the entry point was called (plan_ms includes its validation).

// Re-run shard s of a host call in one unsplit launch over all its lanes, after
// a split-chain handoff timed out (error bit 2: some of its digests are
// undefined). Its payload and metadata are still on the device. Synchronous.
void rerun_unsplit(msha_ctx* ctx, Device& d, const Plan& P, uint8_t* d2h_dst) {
  HIPCHK(hipSetDevice(d.id));
  HIPCHK(hipMemsetAsync(d.err.p, 0, 4, d.stream));
  msha::LaunchKind kind;
  HIPCHK(msha::launch_digest_batch(d.arena.as<uint8_t>(), d.off.as<uint64_t>(), d.len.as<uint64_t>(),
                                   nullptr, P.ordered ? d.order.as<uint32_t>() : nullptr, P.lanes,
                                   d.out.as<uint8_t>(), d.err.as<uint32_t>(), d.cus, ctx->kernel_policy,
                                   d.stream, nullptr, &kind));
  count_launch(ctx, &d, kind);
  HIPCHK(hipMemcpyAsync(d2h_dst, d.out.p, 32 * P.m, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipMemcpyAsync(d.h_out.as<uint8_t>() + 32 * P.m, d.err.p, 4, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  __atomic_fetch_add(&ctx->stats.split_retries, 1, __ATOMIC_RELAXED);
}

// ---------------------------------------------------------------------------
// Small calls: the latency path. MirBFT's hash worker hands over one
// ActionList per call (mirbft.go:282-302), and at low load that is a handful of
// actions. run_pipeline's round trip costs ~60-80 us whatever the size (seven
// queue operations over two streams, events, planning passes), while the GPU
// floor of H2D + kernel + D2H is ~18 us (tools/op_latency.hip). A call of at
// most small_msgs() messages and small_bytes() of payload (limits below)
// therefore runs on the context's first GPU as: messages packed behind their
// metadata in one pinned staging buffer -> ONE H2D (a pinned, 16-byte aligned
// arena span over 512 KiB is uploaded as is instead: metadata H2D + span H2D),
// one launch, ONE D2H of [error word | digests]. No alias folding (an identical
// payload is simply hashed again) and no sharding: neither pays at this size.
// ---------------------------------------------------------------------------
uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* e = getenv(name);
  return e ? strtoull(e, nullptr, 10) : dflt;
}
// Limits, read per call (a getenv is ~0.1 us; tests switch paths within one
// process). Measured per call (tools/latency.cpp, profiles/r02_latency/): packing
// on the calling thread beats the pipeline up to a few MiB (512-B requests: 4,096
// 132 vs 193 us, 16,384 388 vs 448 us; 65,536 = 32 MiB 2.5 vs 1.3 ms); a pinned
// span needs no packing and wins up to one 64 MiB upload piece (65,536 x 512 B 861
// vs 898 us); digest-of-digests keeps its own path above 1 MiB (its table goes up
// once, nothing is gathered: 4,096 Batches 137 us vs 184 packed).
uint64_t small_bytes() { return env_u64("MSHA_SMALL_BYTES", 4ull << 20); }   // packed payload; 0 disables
uint64_t small_msgs() { return env_u64("MSHA_SMALL_MSGS", 65536); }
uint64_t small_span_bytes() { return std::min<uint64_t>(env_u64("MSHA_SMALL_SPAN_BYTES", kDirectChunk), kDirectChunk); }
constexpr uint64_t kSmallSpanMin = 512ull << 10;  // below: pack it anyway (one H2D beats two)
constexpr uint64_t kSmallDodBytes = 1ull << 20;
inline bool small_call(uint64_t n, uint64_t bytes) {
  return n <= small_msgs() && bytes <= small_bytes() && small_bytes() > 0;
}

// Stats of a latency-path call (run_small, run_small_zc).
void small_stats(msha_ctx* ctx, Device& d, double t0, double t_pack, double t_dev, uint64_t m, uint64_t pay,
                 uint64_t h2d, uint64_t d2h, bool packed, msha::LaunchKind kind) {
  for (Device& o : ctx->devs) {
    o.st = msha_shard_stats{};
    o.st.device = o.id;
  }
  d.st.messages = d.st.lanes = m;
  d.st.h2d_payload_bytes = pay;
  d.st.h2d_bytes = h2d;
  d.st.d2h_bytes = d2h;
  d.st.device_ms = t_dev - t_pack;
  count_launch(ctx, &d, kind);
  ctx->stats.calls++;
  ctx->stats.small_calls++;
  ctx->stats.plan_ms = t_pack - t0;
  ctx->stats.pack_ms = packed ? t_pack - t0 : 0;
  ctx->stats.device_ms = t_dev - t_pack;
  ctx->stats.h2d_bytes = h2d;
  ctx->stats.d2h_bytes = d2h;
  ctx->stats.total_ms = now_ms() - t0;
  trace("done", t0);
}

// The zero-copy latency path (see run_small): [off | len | payload] packed into
// coherent pinned memory, read in place by the kernel, digests written in place.
template <class Fill>
void run_small_zc(msha_ctx* ctx, Device& d, double t0, uint64_t m, uint64_t meta, uint64_t pay, const uint64_t* len,
                  uint8_t* out, Fill& fill, const uint64_t* first) {
  d.sm_zc_in.ensure(meta + pay + msha::kArenaSlack);
  d.sm_zc_out.ensure(32 * m);
  uint64_t* h_off = d.sm_zc_in.as<uint64_t>();
  uint64_t* h_len = h_off + m;
  uint8_t* h_pay = d.sm_zc_in.as<uint8_t>() + meta;
  uint64_t a = 0;
  for (uint64_t i = 0; i < m; ++i) {
    h_len[i] = len[i];
    if (first && first[i] != i) {
      h_off[i] = h_off[first[i]];
    } else {
      h_off[i] = a;
      if (len[i]) fill(i, h_pay + a);
      a += round16(len[i]);
    }
  }
  const double t_pack = now_ms();
  HIPCHK(hipSetDevice(d.id));
  const uint64_t out_cap = d.sm_out.cap;
  d.sm_out.ensure(32);  // the device error word (never set here: the packer's offsets are aligned)
  if (d.sm_out.cap != out_cap) HIPCHK(hipMemsetAsync(d.sm_out.p, 0, 32, d.stream));
  void *dev_in = nullptr, *dev_out = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dev_in, d.sm_zc_in.p, 0));
  HIPCHK(hipHostGetDevicePointer(&dev_out, d.sm_zc_out.p, 0));
  const uint64_t* d_off = static_cast<const uint64_t*>(dev_in);
  // Completion by polling the digests themselves (MSHA_SMALL_ZC_POLL=0: a stream
  // synchronize, A/B): every 8-byte word starts as a sentinel, and the kernel
  // overwrites each with its final value in one PCIe write (16-byte digest halves).
  // A word that still reads as the sentinel is waited for until hipStreamQuery
  // reports the launch done -- so a digest word that happens to equal the
  // sentinel (2^-64 a word) only costs the wait, never a wrong digest -- and a
  // failed launch is reported from there.
  const bool poll = env_u64("MSHA_SMALL_ZC_POLL", 1) != 0;
  constexpr uint64_t kSentinel = 0xC3A55A3C96E1F00Full;
  volatile uint64_t* words = static_cast<volatile uint64_t*>(d.sm_zc_out.p);
  if (poll)
    for (uint64_t k = 0; k < 4 * m; ++k) words[k] = kSentinel;
  msha::LaunchKind kind;
  HIPCHK(msha::launch_digest_batch(static_cast<const uint8_t*>(dev_in) + meta, d_off, d_off + m, nullptr, nullptr, m,
                                   static_cast<uint8_t*>(dev_out), d.sm_out.as<uint32_t>(), d.cus, MSHA_KERNEL_AUTO,
                                   d.stream, nullptr, &kind));
  if (poll) {
    uint64_t k = 0;
    for (uint64_t spin = 1; k < 4 * m; ++spin) {
      while (k < 4 * m && words[k] != kSentinel) ++k;
      if (k == 4 * m || spin % 64) {
        __builtin_ia32_pause();
        continue;
      }
      const hipError_t q = hipStreamQuery(d.stream);
      if (q == hipSuccess) break;  // done: every word is final, whatever it reads
      if (q != hipErrorNotReady) HIPCHK(q);
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else {
    HIPCHK(hipStreamSynchronize(d.stream));
  }
  const double t_dev = now_ms();
  std::memcpy(out, d.sm_zc_out.p, 32 * m);
  ctx->stats.small_zc_calls++;
  small_stats(ctx, d, t0, t_pack, t_dev, m, pay, 0, 0, true, kind);
}

// The caller's pinned arena, uploaded as is: messages i at base + off[i], all
// inside [lo, hi), 16-byte aligned.
struct SmallSpan {
  const uint8_t* base;
  const uint64_t* off;
  uint64_t lo, hi;
};

// first (may be null): first[i] = the earliest message with message i's (off,
// len) (alias_uids): an aliased payload is packed once and its aliases point at
// it (EpochChange re-hashes, epoch_target.go:486-505; the Go adapter shares a
// payload between actions, gpuhash.go epochChangeAliases).
//
// Zero-copy (round 6): a call of at most small_zc_msgs()
// messages and small_zc_bytes() packed (a few actions: MirBFT's hash worker at low
// load) skips both copies. The list is packed into coherent pinned memory that the
// kernel (the eight-lane chain: at most 16 messages a CU) reads in place over PCIe,
// and the digests are written straight into coherent pinned memory: one launch and
// one synchronize per call. The packer's own 16-byte aligned offsets cannot raise
// the device error word (check_aligned), so it stays on the device.
// Limits measured per call (tools/latency.cpp, profiles/r06_latency/): 512-B
// requests zero-copy / copying, 1: 29.6 / 38.1 us, 64: 31.7 / 42.0, 256: 33.9 /
// 46.8, 1,024: 47.9 / 70.5, 4,096: 108.1 / 111.2 (the kernel's PCIe reads then cost
// what the copy saved).
uint64_t small_zc_bytes() { return env_u64("MSHA_SMALL_ZC_BYTES", 1ull << 20); }  // 0 disables
uint64_t small_zc_msgs(const Device& d) { return std::min<uint64_t>(env_u64("MSHA_SMALL_ZC_MSGS", 2048),
                                                                    (uint64_t)d.cus * msha::kChain8MsgsPerWg); }

template <class Fill>
void run_small(msha_ctx* ctx, double t0, uint64_t m, const uint64_t* len, uint8_t* out, Fill&& fill,
               const SmallSpan* span = nullptr, const uint64_t* first = nullptr) {
  Device& d = ctx->devs[0];
  const uint64_t meta = (16 * m + 63) & ~uint64_t(63);  // off[m], len[m]; payload 64-B aligned after
  uint64_t pay = 0;
  if (span) {
    pay = span->hi - span->lo;
  } else {
    for (uint64_t i = 0; i < m; ++i)
      if (!first || first[i] == i) pay += round16(len[i]);
  }
  const bool zc = !span && ctx->kernel_policy == MSHA_KERNEL_AUTO && m <= small_zc_msgs(d) &&
                  meta + pay <= small_zc_bytes();
  if (zc) return run_small_zc(ctx, d, t0, m, meta, pay, len, out, fill, first);
  d.sm_stage.ensure(meta + (span ? 0 : pay));
  uint64_t* h_off = d.sm_stage.as<uint64_t>();
  uint64_t* h_len = h_off + m;
  uint8_t* h_pay = d.sm_stage.as<uint8_t>() + meta;
  uint64_t a = 0;
  for (uint64_t i = 0; i < m; ++i) {
    h_len[i] = len[i];
    if (span) {
      h_off[i] = span->off[i] - span->lo;
    } else if (first && first[i] != i) {
      h_off[i] = h_off[first[i]];
    } else {
      h_off[i] = a;
      if (len[i]) fill(i, h_pay + a);
      a += round16(len[i]);
    }
  }
  const double t_pack = now_ms();
  HIPCHK(hipSetDevice(d.id));
  d.sm_in.ensure(meta + pay + msha::kArenaSlack);
  const uint64_t out_cap = d.sm_out.cap;
  d.sm_out.ensure(32 + 32 * m);
  // the error word heads the output buffer; zeroed once per allocation and
  // again only after a call that found it set
  if (d.sm_out.cap != out_cap) HIPCHK(hipMemsetAsync(d.sm_out.p, 0, 32, d.stream));
  d.sm_res.ensure(32 + 32 * m);
  uint8_t* dev_in = d.sm_in.as<uint8_t>();
  if (span) {
    HIPCHK(hipMemcpyAsync(dev_in, h_off, 16 * m, hipMemcpyHostToDevice, d.stream));
    if (pay) HIPCHK(hipMemcpyAsync(dev_in + meta, span->base + span->lo, pay, hipMemcpyHostToDevice, d.stream));
  } else {
    HIPCHK(hipMemcpyAsync(dev_in, h_off, meta + pay, hipMemcpyHostToDevice, d.stream));
  }
  msha::LaunchKind kind;
  HIPCHK(msha::launch_digest_batch(dev_in + meta, reinterpret_cast<const uint64_t*>(dev_in),
                                   reinterpret_cast<const uint64_t*>(dev_in) + m, nullptr, nullptr, m,
                                   d.sm_out.as<uint8_t>() + 32, d.sm_out.as<uint32_t>(), d.cus,
                                   ctx->kernel_policy, d.stream, nullptr, &kind));
  HIPCHK(hipMemcpyAsync(d.sm_res.p, d.sm_out.p, 32 + 32 * m, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  const double t_dev = now_ms();
  uint32_t errflag;
  std::memcpy(&errflag, d.sm_res.p, 4);
  if (errflag) {  // cannot happen (aligned payloads, no split chains): leave the word clean, report
    HIPCHK(hipMemsetAsync(d.sm_out.p, 0, 32, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    throw MshaError(MSHA_ERR_HIP, "internal: device error flag " + std::to_string(errflag) + " on a small call");
  }
  std::memcpy(out, d.sm_res.as<uint8_t>() + 32, 32 * m);
  const uint64_t h2d = 16 * m + (span ? pay : meta - 16 * m + pay);
  small_stats(ctx, d, t0, t_pack, t_dev, m, pay, h2d, 32 + 32 * m, !span, kind);
}

// Launch shard d's lanes accumulated since its last launch, up to the end of
// lane group c, once they fill the GPU (2 waves per SIMD) or at the last group:
// hashing runs ~30x faster than PCIe delivers bytes, so a launch per group would
// only buy overlap worth a few % while a group of large messages (512 x 64 KiB)
// leaves most SIMDs idle for the whole of its long chains. Then bring back the
// digests that are final: identity lanes' own slots, or (ordered lanes with
// later_min) every slot below the lowest slot a later group writes -- into the
// caller's buffer itself when it is pinned -- while later groups upload.
// The stream a host call's digest D2H goes on: d2h_stream, ordered after
// everything queued so far on `after` (its kernels). On the kernel stream itself
// a D2H would hold up the next launch for as long as the copy takes, and on a
// box whose PCIe writes are slowed by other traffic that delayed c5's last
// kernels by up to 9 ms. MSHA_D2H_STREAM=0 keeps the D2H on the kernel stream
// (A/B, tools/ab_d2h.py). Shards sharing one GPU (MSHA_VIRTUAL_SHARDS) keep it
// on the kernel stream: HIP multiplexes streams over GPU_MAX_HW_QUEUES (4)
// hardware queues per device, and a third stream per shard put D2H waits in
// front of other shards' uploads (c5 at 2 virtual shards 71.5 -> 89 ms per call).
hipStream_t d2h_stream_after(Device& d, hipStream_t after) {
  if (!d.d2h_stream || env_u64("MSHA_D2H_STREAM", 1) == 0) return after;
  HIPCHK(hipEventRecord(d.ev_k, after));
  HIPCHK(hipStreamWaitEvent(d.d2h_stream, d.ev_k, 0));
  return d.d2h_stream;
}

void launch_lanes(msha_ctx* ctx, Device& d, Plan& P, size_t c, bool last, double t0, uint8_t* out,
                  bool out_pinned) {
  const uint64_t q1 = P.lane_cut[c + 1];
  const uint64_t fill = (uint64_t)d.cus * 4 * 64 * 2;
  if (!last && q1 - P.launched < fill) return;
  const uint64_t l0 = P.launched, lanes = q1 - l0;
  P.launched = q1;
  if (!P.k0) {
    HIPCHK(hipEventRecord(d.ev_k0, d.stream));
    d.st.first_launch_ms = now_ms() - t0;
    P.k0 = true;
    trace("first launch", d.index, t0);
  }
  // off/len are lane-indexed; out_idx maps lane -> shard-local message
  // (identity placement: lane q is message q)
  msha::SplitPlan sp;
  msha::LaunchKind kind;
  HIPCHK(msha::launch_digest_batch(
      d.arena.as<uint8_t>(), d.off.as<uint64_t>() + l0, d.len.as<uint64_t>() + l0, nullptr,
      P.ordered ? d.order.as<uint32_t>() + l0 : nullptr, lanes,
      d.out.as<uint8_t>() + (P.ordered ? 0 : 32 * l0), d.err.as<uint32_t>(), d.cus,
      ctx->kernel_policy, d.stream, split_for(d, lanes, ctx->kernel_policy, sp), &kind));
  count_launch(ctx, &d, kind);
  uint8_t* dst = out_pinned ? out + 32 * d.lo : d.h_out.as<uint8_t>();
  const bool d2h = P.identity() || (!P.later_min.empty() && P.later_min[c + 1] > P.d2h_done);
  hipStream_t ds = d2h ? d2h_stream_after(d, d.stream) : d.stream;
  if (P.identity()) {
    HIPCHK(hipMemcpyAsync(dst + 32 * l0, d.out.as<uint8_t>() + 32 * l0, 32 * lanes, hipMemcpyDeviceToHost, ds));
    d.st.d2h_bytes += 32 * lanes;
  } else if (!P.later_min.empty()) {
    // aliases among the streamed slots are filled on the host after the sync
    const uint64_t x = P.later_min[c + 1];
    if (x > P.d2h_done) {
      HIPCHK(hipMemcpyAsync(dst + 32 * P.d2h_done, d.out.as<uint8_t>() + 32 * P.d2h_done, 32 * (x - P.d2h_done),
                            hipMemcpyDeviceToHost, ds));
      d.st.d2h_bytes += 32 * (x - P.d2h_done);
      P.d2h_done = x;
    }
  }
}

// Long chains on the direct path: a payload of at least kLongBlocks blocks
// (16 KiB: ~0.8 ms as a chain on the lane kernel, more than an upload piece
// takes to land) when the batch has one; MSHA_HOST_HEAD=0 disables (A/B). A
// context held to the lane kernel (MSHA_KERNEL_LANE) runs no heads, as the
// device-planned path does not: its long payloads stay ordinary lanes.
constexpr uint64_t kLongBlocks = 256;
uint64_t long_chain_blocks(uint64_t bmax, uint32_t policy) {
  if (env_u64("MSHA_HOST_HEAD", 1) == 0 || policy == MSHA_KERNEL_LANE) return 0;
  return bmax >= kLongBlocks ? kLongBlocks : 0;
}
// At most this many long lanes run as heads (two-lane chains, 64 per CU): half
// the CUs. More long chains than that fill the GPU by themselves, and the lane
// kernel runs them.
uint64_t head_cap(const Device& d) { return (uint64_t)d.cus * msha::kChain2MsgsPerWg / 2; }

// Lanes [l0, l1) of shard d (long chains, lane-indexed metadata) as a head:
// k_digest_chain2 with CUs of its own, behind the upload piece `piece_in`,
// digests lane-indexed into p_head. On a GPU of its own the heads go on the
// side stream and run beside the lane kernel; on a shared GPU
// (MSHA_VIRTUAL_SHARDS) a third stream per shard would contend for the GPU's
// hardware queues (d2h_stream_after), so they go on the kernel stream.
void launch_head(msha_ctx* ctx, Device& d, Plan& P, uint64_t l0, uint64_t l1, hipEvent_t piece_in, double t0) {
  hipStream_t hs = d.stream;
  d.head_side = d.d2h_stream != nullptr;
  if (d.head_side) {
    if (!d.side_stream) HIPCHK(hipStreamCreateWithFlags(&d.side_stream, hipStreamNonBlocking));
    if (!d.ev_head) HIPCHK(hipEventCreateWithFlags(&d.ev_head, hipEventDisableTiming));
    hs = d.side_stream;
  }
  HIPCHK(hipStreamWaitEvent(hs, piece_in, 0));
  if (!P.k0) {
    HIPCHK(hipEventRecord(d.ev_k0, hs));
    d.st.first_launch_ms = now_ms() - t0;
    P.k0 = true;
    trace("first launch (head)", d.index, t0);
  }
  msha::LaneGate hg;
  hg.head_part = true;
  hg.two_lane = true;
  msha::LaunchKind kind;
  HIPCHK(msha::launch_digest_batch(d.arena.as<uint8_t>(), d.off.as<uint64_t>() + l0, d.len.as<uint64_t>() + l0,
                                   nullptr, nullptr, l1 - l0, d.p_head.as<uint8_t>() + 32 * l0, d.err.as<uint32_t>(),
                                   d.cus, MSHA_KERNEL_COOP, hs, nullptr, &kind, &hg));
  count_launch(ctx, &d, kind);
  if (d.head_side) HIPCHK(hipEventRecord(d.ev_head, hs));
}

// Queue the end of shard d's call on its stream: ev1 after its last kernel,
// the digest slots not streamed back yet, the error word.
void queue_tail(Device& d, Plan& P, uint8_t* out, bool out_pinned) {
  const uint64_t m = P.m;
  if (m == 0) return;
  HIPCHK(hipSetDevice(d.id));
  if (P.head) {  // the heads' digests and their lanes' slots, behind the heads
    if (d.head_side) HIPCHK(hipStreamWaitEvent(d.stream, d.ev_head, 0));
    HIPCHK(hipMemcpyAsync(d.h_head.p, d.p_head.p, 32 * P.head, hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipMemcpyAsync(d.h_head.as<uint8_t>() + 32 * P.head, d.order.p, 4 * P.head, hipMemcpyDeviceToHost,
                          d.stream));
    d.st.d2h_bytes += 36 * P.head;
  }
  HIPCHK(hipEventRecord(d.ev1, d.stream));
  const hipStream_t ds = d2h_stream_after(d, d.stream);
  const uint64_t done = P.d2h_done;  // slots streamed back after earlier launches
  if (!P.identity() && done < m) {
    // d.out is message-ordered (lane q wrote its message's slot); a pinned result
    // buffer takes it as is, the aliases' slots are filled on the host afterwards
    HIPCHK(hipMemcpyAsync((out_pinned ? out + 32 * d.lo : d.h_out.as<uint8_t>()) + 32 * done,
                          d.out.as<uint8_t>() + 32 * done, 32 * (m - done), hipMemcpyDeviceToHost, ds));
    d.st.d2h_bytes += 32 * (m - done);
  }
  HIPCHK(hipMemcpyAsync(d.h_out.as<uint8_t>() + 32 * m, d.err.p, 4, hipMemcpyDeviceToHost, ds));
  d.st.d2h_bytes += 4;
}

float elapsed_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  HIPCHK(hipEventSynchronize(b));
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

// Finish shard s of a host call, on the shard's own thread (shards finish side
// by side): wait for its stream, re-run it unsplit if a split chain's hand-off
// timed out, fill its aliases' digests (each copies its representative's) and
// complete its msha_shard_stats: device_ms = first upload .. last kernel,
// upload_ms = first .. last upload, kernel_ms = first kernel .. last (HIP events).
void finish_shard(msha_ctx* ctx, uint32_t s, uint8_t* out, bool out_pinned, double t0) {
  Device& d = ctx->devs[s];
  Plan& P = ctx->plans[s];
  const uint64_t m = P.m;
  if (m == 0) return;
  HIPCHK(hipSetDevice(d.id));
  HIPCHK(hipStreamSynchronize(d.stream));
  if (d.d2h_stream) HIPCHK(hipStreamSynchronize(d.d2h_stream));
  d.st.device_ms = elapsed_ms(d.ev_up0, d.ev1);
  d.st.upload_ms = elapsed_ms(d.ev_up0, d.ev_up1);
  d.st.kernel_ms = elapsed_ms(d.ev_k0, d.ev1);
  if (trace_on())
    fprintf(stderr, "[msha] shard %u %-16s %9.2f ms (device %.2f, upload %.2f, kernels %.2f ms)\n", s, "synced",
            now_ms() - t0, d.st.device_ms, d.st.upload_ms, d.st.kernel_ms);
  uint32_t errflag;
  std::memcpy(&errflag, d.h_out.as<uint8_t>() + 32 * m, 4);
  const bool straight = out_pinned;  // the digests were D2H'd straight into out
  if (errflag & 2) {
    // a split chain's handoff timed out: its digests are undefined; the
    // payload is still on the device, so re-hash the shard unsplit
    rerun_unsplit(ctx, d, P, straight ? out + 32 * d.lo : d.h_out.as<uint8_t>());
    d.st.d2h_bytes += 32 * m + 4;
    std::memcpy(&errflag, d.h_out.as<uint8_t>() + 32 * m, 4);
    if (errflag & 2) throw MshaError(MSHA_ERR_HIP, "split-chain handoff timed out (re-run failed)");
  }
  if (errflag) throw MshaError(MSHA_ERR_ALIGNMENT, "internal: misaligned staged message");
  d.st.h2d_bytes += d.st.h2d_payload_bytes;
  const uint32_t* rep = P.rep_of();
  const uint8_t* h = d.h_out.as<uint8_t>();
  if (P.head) {  // the heads' digests into their slots (before the aliases copy them)
    const uint8_t* hd = d.h_head.as<uint8_t>();
    const uint32_t* slot = reinterpret_cast<const uint32_t*>(hd + 32 * P.head);
    uint8_t* base = straight ? out + 32 * d.lo : d.h_out.as<uint8_t>();
    for (uint64_t i = 0; i < P.head; ++i) std::memcpy(base + 32 * (uint64_t)slot[i], hd + 32 * i, 32);
  }
  if (straight) {
    if (rep)  // aliases copy their representative's digest
      parallel_chunks(m, plan_threads(m), [&](unsigned, uint64_t a, uint64_t b) {
        uint8_t* o = out + 32 * d.lo;
        for (uint64_t i = a; i < b; ++i)
          if (rep[i] != i) std::memcpy(o + 32 * i, o + 32 * (uint64_t)rep[i], 32);
      });
    return;
  }
  parallel_chunks(m, plan_threads(m), [&](unsigned, uint64_t a, uint64_t b) {
    if (!rep)
      std::memcpy(out + 32 * (d.lo + a), h + 32 * a, 32 * (b - a));
    else
      for (uint64_t i = a; i < b; ++i) std::memcpy(out + 32 * (d.lo + i), h + 32 * (uint64_t)rep[i], 32);
  });
}

// The call's figures (msha_stats) from its finished shards'.
void call_stats(msha_ctx* ctx, double t0, double t_plan) {
  double device_ms = 0, gather_ms = 0;
  uint64_t h2d = 0, d2h = 0;
  for (uint32_t s = 0; s < (uint32_t)ctx->devs.size(); ++s) {
    if (ctx->plans[s].m == 0) continue;
    const msha_shard_stats& st = ctx->devs[s].st;
    device_ms = std::max(device_ms, st.device_ms);
    gather_ms += st.gather_ms;
    h2d += st.h2d_bytes;
    d2h += st.d2h_bytes;
  }
  ctx->stats.calls++;
  ctx->stats.plan_ms = t_plan - t0;
  ctx->stats.pack_ms = gather_ms;
  ctx->stats.device_ms = device_ms;
  ctx->stats.h2d_bytes = h2d;
  ctx->stats.d2h_bytes = d2h;
  ctx->stats.total_ms = now_ms() - t0;
}

template <class Gather>
void run_pipeline(msha_ctx* ctx, double t0, uint64_t n, const uint64_t* len, const uint64_t* uid,
                  uint8_t* out, Gather&& gather, const uint64_t* pre_bounds = nullptr) {
  const uint32_t k = (uint32_t)ctx->devs.size();
  const bool out_pinned = is_pinned_host(out) && is_pinned_host(out + 32 * n - 1);
  std::vector<uint64_t> bounds(k + 1);
  if (pre_bounds) std::copy(pre_bounds, pre_bounds + k + 1, bounds.begin());
  else partition(len, n, k, bounds.data());

  std::vector<Plan>& plans = ctx->plans;
  plans.resize(k);
  for (uint32_t s = 0; s < k; ++s) {
    Plan& P = plans[s];
    P.m = 0;
    P.next = 0;
    P.launched = 0;
    P.d2h_done = 0;
    P.later_min.clear();
    P.rep_dev = nullptr;
    P.head = 0;
    P.k0 = false;
    msha_shard_stats& st = ctx->devs[s].st;
    st = msha_shard_stats{};
    st.device = ctx->devs[s].id;
  }
  for (uint32_t s = 0; s < k; ++s) {
    ctx->devs[s].lo = bounds[s];
    ctx->devs[s].hi = bounds[s + 1];
  }
  // Plan every shard (several GPUs: side by side, for_each_shard).
  for_each_shard(ctx, [&](uint32_t s) {
    Device& d = ctx->devs[s];
    Plan& P = plans[s];
    P.m = d.hi - d.lo;
    d.st.messages = P.m;
    if (P.m == 0) return;
    // this GPU current before any staging allocation: without
    // hipHostMallocNumaUser the runtime takes pinned memory from the host pool
    // of the current device's nearest CPU agent (its NUMA node)
    HIPCHK(hipSetDevice(d.id));
    const uint64_t* L = len + d.lo;
    // Aliases (same uid) have identical bytes, hence identical digests: only
    // the first message of each uid gets a lane; the others copy its digest
    // after the D2H (EpochChange re-hashing, epoch_target.go:486-505).
    P.rep.clear();
    P.lanes = P.m;
    if (uid && k == 1) {  // one shard: uid[i] (the first index with i's payload) is the lane's message
      P.rep.resize(P.m);
      const unsigned T = plan_threads(P.m);
      std::vector<uint64_t> nl(T, 0);
      parallel_chunks(P.m, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
        uint64_t c = 0;
        for (uint64_t i = lo; i < hi; ++i) {
          P.rep[i] = (uint32_t)uid[i];
          c += uid[i] == i;
        }
        nl[t] = c;
      });
      P.lanes = 0;
      for (uint64_t c : nl) P.lanes += c;
      if (P.lanes == P.m) P.rep.clear();
    } else if (uid) {
      // rep[i] = the shard-local index of the shard's first message with i's
      // payload. uid[i] (the batch-wide first occurrence) at or past the shard's
      // start lies in this shard, so it is also the shard's first: threaded.
      // An earlier uid (a payload first seen by an earlier shard, e.g. the shared
      // EpochChange pool) is resolved in index order through `placed`, over
      // those messages only.
      P.rep.resize(P.m);
      const unsigned T = plan_threads(P.m);
      std::vector<uint64_t> nl(T, 0);
      std::vector<std::vector<uint32_t>> cross(T);
      parallel_chunks(P.m, T, [&](unsigned t, uint64_t a, uint64_t b) {
        uint64_t c = 0;
        for (uint64_t i = a; i < b; ++i) {
          const uint64_t u = uid[d.lo + i];
          if (u >= d.lo) {
            P.rep[i] = (uint32_t)(u - d.lo);
            c += u == d.lo + i;
          } else {
            cross[t].push_back((uint32_t)i);
          }
        }
        nl[t] = c;
      });
      P.lanes = 0;
      for (uint64_t c : nl) P.lanes += c;
      uint64_t ncross = 0;
      for (const std::vector<uint32_t>& v : cross) ncross += v.size();
      std::unordered_map<uint64_t, uint32_t> first;  // uid -> the shard's first message with it
      first.reserve(std::min<uint64_t>(ncross, 1u << 16));
      for (const std::vector<uint32_t>& v : cross)
        for (uint32_t i : v) {
          const auto it = first.try_emplace(uid[d.lo + i], i);
          P.rep[i] = it.first->second;
          P.lanes += it.second;
        }
      if (P.lanes == P.m) P.rep.clear();
    }
    d.st.lanes = P.lanes;
    trace("representatives", t0);
    P.perm.resize(P.lanes);
    d.h_meta.ensure(16 * P.m + 4 * P.m);
    uint64_t* h_off = d.h_meta.as<uint64_t>();
    uint64_t* h_len = h_off + P.m;
    if (!P.rep.empty()) {  // lanes = the representatives, by descending block count
      order_by_blocks_desc(L, P.m, P.perm.data(), d.sort_tmp, P.rep.data());
      P.ordered = true;
    } else {
      P.ordered = !all_equal_blocks(L, P.m);
      if (P.ordered) order_by_blocks_desc(L, P.m, P.perm.data(), d.sort_tmp);
      else for (uint64_t i = 0; i < P.m; ++i) P.perm[i] = (uint32_t)i;
    }
    trace("lane order", t0);
    // Place payloads in lane order (each lane's payload is distinct: aliases
    // were folded into their representative above), so every lane of chunk c
    // reads bytes uploaded by the end of chunk c.
    uint64_t acc = 0;
    {
      // lane-indexed metadata: an exclusive scan of the 16-byte-rounded lengths
      // (lane q's payload lands at h_off[q]; payloads are placed in lane order)
      const unsigned T = plan_threads(P.lanes);
      std::vector<uint64_t> part(T + 1, 0);
      parallel_chunks(P.lanes, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
        uint64_t a = 0;
        for (uint64_t q = lo; q < hi; ++q) {
          const uint64_t l = L[P.perm[q]];
          h_len[q] = l;
          a += round16(l);
        }
        part[t + 1] = a;
      });
      for (unsigned t = 0; t < T; ++t) part[t + 1] += part[t];
      parallel_chunks(P.lanes, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
        uint64_t a = part[t];
        for (uint64_t q = lo; q < hi; ++q) {
          h_off[q] = a;
          a += round16(h_len[q]);
        }
      });
      acc = part[T];
      // greedy chunks of >= kChunkBytes: cut after the first lane whose end
      // reaches the chunk's start + kChunkBytes (binary search on the scan)
      P.lane_cut.assign(1, 0);
      for (uint64_t q0 = 0;;) {
        const uint64_t target = h_off[q0] + kChunkBytes;
        const uint64_t r = (uint64_t)(std::lower_bound(h_off + q0 + 1, h_off + P.lanes, target) - h_off);
        if (r >= P.lanes) break;  // the rest (ending at acc) is the last chunk
        P.lane_cut.push_back(r);
        q0 = r;
      }
      P.lane_cut.push_back(P.lanes);
    }
    d.arena_bytes = acc;
    trace("placement", t0);
    if (P.ordered) std::memcpy(h_len + P.m, P.perm.data(), 4 * P.lanes);
    {
      uint64_t slot_bytes = 0;
      for (size_t c = 0; c + 1 < P.lane_cut.size(); ++c) {
        const uint64_t e = P.lane_cut[c + 1] < P.lanes ? h_off[P.lane_cut[c + 1]] : acc;
        slot_bytes = std::max(slot_bytes, e - h_off[P.lane_cut[c]]);
      }
      d.slot[0].ensure(std::max<uint64_t>(slot_bytes, 16));
      d.slot[1].ensure(std::max<uint64_t>(slot_bytes, 16));
    }
    HIPCHK(hipSetDevice(d.id));
    d.arena.ensure(acc + msha::kArenaSlack);
    d.h_out.ensure(32 * P.m + 4);
    d.off.ensure(8 * P.m);
    d.len.ensure(8 * P.m);
    d.out.ensure(32 * P.m);
    d.err.ensure(4);
    if (P.ordered) d.order.ensure(4 * P.lanes);
    HIPCHK(hipEventRecord(d.ev_up0, d.stream));
    HIPCHK(hipMemcpyAsync(d.off.p, h_off, 8 * P.lanes, hipMemcpyHostToDevice, d.stream));
    HIPCHK(hipMemcpyAsync(d.len.p, h_len, 8 * P.lanes, hipMemcpyHostToDevice, d.stream));
    d.st.h2d_bytes = 16 * P.lanes;
    if (P.ordered) {
      HIPCHK(hipMemcpyAsync(d.order.p, h_len + P.m, 4 * P.lanes, hipMemcpyHostToDevice, d.stream));
      d.st.h2d_bytes += 4 * P.lanes;
    }
    HIPCHK(hipMemsetAsync(d.err.p, 0, 4, d.stream));
    HIPCHK(hipEventRecord(d.ev0, d.stream));
    HIPCHK(hipStreamWaitEvent(d.copy_stream, d.ev0, 0));  // uploads start after ev0: device_ms spans them
    HIPCHK(hipEventRecord(d.slot_free[0], d.copy_stream));
    HIPCHK(hipEventRecord(d.slot_free[1], d.copy_stream));
  });
  const double t_plan = now_ms();
  trace("planned (metadata H2D queued)", t0);

  // Issue chunk P.next of shard s: gather it into a staging slot, upload it, and
  // launch the lanes accumulated so far when they fill the GPU (launch_lanes).
  // Returns whether shard s has chunks left.
  auto issue_chunk = [&](uint32_t s, WorkerPool& pool) -> bool {
    Device& d = ctx->devs[s];
    Plan& P = plans[s];
    if (P.m == 0 || P.next + 1 >= P.lane_cut.size()) return false;
    const size_t c = P.next++;
    const uint64_t u0 = P.lane_cut[c], u1 = P.lane_cut[c + 1];
    const uint64_t* h_off = d.h_meta.as<uint64_t>();  // lane -> arena offset
    HIPCHK(hipSetDevice(d.id));
    const uint64_t b0 = h_off[u0];
    const uint64_t b1 = u1 >= P.lanes ? d.arena_bytes : h_off[u1];
    PinBuf& slot = d.slot[c & 1];
    HIPCHK(hipEventSynchronize(d.slot_free[c & 1]));  // its previous H2D has drained
    const double g0 = now_ms();
    uint8_t* dst = slot.as<uint8_t>();
    parallel_ranges(pool, u1 - u0, b1 - b0, [&](uint64_t a, uint64_t b) {
      for (uint64_t u = u0 + a; u < u0 + b; ++u) gather(d.lo + P.perm[u], dst + (h_off[u] - b0));
    });
    const double g1 = now_ms();
    if (d.st.gather_begin_ms == 0) d.st.gather_begin_ms = std::max(g0 - t0, 1e-6);
    d.st.gather_end_ms = g1 - t0;
    d.st.gather_ms += g1 - g0;
    if (b1 > b0)
      HIPCHK(hipMemcpyAsync(d.arena.as<uint8_t>() + b0, slot.p, b1 - b0, hipMemcpyHostToDevice,
                            d.copy_stream));
    d.st.h2d_payload_bytes += b1 - b0;
    HIPCHK(hipEventRecord(d.slot_free[c & 1], d.copy_stream));
    HIPCHK(hipEventRecord(d.chunk_in, d.copy_stream));
    const bool last = P.next + 1 >= P.lane_cut.size();
    if (last) HIPCHK(hipEventRecord(d.ev_up1, d.copy_stream));
    HIPCHK(hipStreamWaitEvent(d.stream, d.chunk_in, 0));
    launch_lanes(ctx, d, P, c, last, t0, out, out_pinned);
    return !last;
  };
  if (k > 1) {
    // Pageable arenas over several GPUs: one issuing thread per GPU, each with
    // its own gather helpers, so the host copy for GPU s+1 never waits on GPU
    // s's staging slot (msha_shard_stats gather_begin/end show the overlap).
    for_each_shard(ctx, [&](uint32_t s) {
      while (issue_chunk(s, cur_pool())) {
      }
    });
  } else {
    // One GPU: the calling thread issues its chunks.
    for (bool more = true; more;) {
      more = false;
      for (uint32_t s = 0; s < k; ++s) more |= issue_chunk(s, WorkerPool::get());
    }
  }
  for_each_shard(ctx, [&](uint32_t s) {
    queue_tail(ctx->devs[s], plans[s], out, out_pinned);
    finish_shard(ctx, s, out, out_pinned, t0);
  });
  call_stats(ctx, t0, t_plan);
}

// Direct path, pass 1 over one shard's messages (threaded): stage their raw
// (off, len) for the planner kernels (h_off null: the caller's arrays are
// pinned and go up as they are), mark the granules (1 << gs bytes of the
// caller's arena, numbered from glo) their payload bytes touch, and return the
// shard's payload span. Zero-length messages need no bytes and mark nothing
// (so one at the arena's very end uploads nothing past it).
struct ShardSpan {
  uint64_t lo = UINT64_MAX, hi = 0, sum = 0, g0 = UINT64_MAX, g1 = 0;
  // some message starts at or below an earlier message's start (the candidates-
  // first test of alias_uids): only then can two messages share (off, len)
  bool backward = false;
  bool any() const { return hi > 0; }
};

// Granule marks: kMarkTouched (a payload byte is in it), kMarkLong (a payload
// of at least long_blocks blocks is: uploaded first, so the long chains start
// as the call begins, wherever their bytes sit in the caller's arena).
// kMarkCross on granule g: a payload runs on from g into g + 1 -- the two must
// then be uploaded in the same class, or the payload would not be contiguous on
// the device (stage_and_mark closes the long class over such boundaries).
constexpr uint8_t kMarkTouched = 1, kMarkLong = 2, kMarkCross = 4;

template <bool kStage>
ShardSpan stage_and_mark_t(const uint64_t* O, const uint64_t* L, uint64_t m, uint64_t glo, unsigned gs,
                           uint64_t* h_off, uint64_t* h_len, std::vector<uint8_t>& mark, uint64_t long_blocks) {
  const unsigned T = plan_threads(m);
  std::vector<ShardSpan> acc(T);
  std::vector<uint64_t> omin(T, UINT64_MAX), omax(T, 0);
  parallel_chunks(m, T, [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t lo = UINT64_MAX, hi = 0, sum = 0;
    uint64_t last = UINT64_MAX;  // the granule this thread marked last
    uint64_t first_off = UINT64_MAX, max_off = 0;
    bool backward = false;
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t o = O[i], l = L[i];
      if (kStage) {
        h_off[i] = o;
        h_len[i] = l;
      }
      backward |= i > a && o <= max_off;
      max_off = i > a ? std::max(max_off, o) : o;
      if (i == a) first_off = o;
      if (!l) continue;
      const uint64_t e = o + l;
      lo = std::min(lo, o);
      hi = std::max(hi, e);
      sum += l;
      // consecutive messages mostly share a granule (128 x 512 B per 64 KiB):
      // mark a granule once per run, not once per message
      const uint64_t g0 = (o - glo) >> gs, g1 = (e - 1 - glo) >> gs;
      // Marks only grow, so a granule that already holds the bits needs no
      // atomic: a read first (an EpochChange storm names its few long payloads
      // from every thread -- c5: 419K messages on ~75 granules -- and
      // unconditional read-modify-writes there serialised the marking pass on
      // those cache lines: c5's first kernel 5.0 -> 12.3 ms into the call).
      auto mark_or = [&](uint64_t g, uint8_t bits) {
        if ((__atomic_load_n(&mark[g], __ATOMIC_RELAXED) & bits) != bits)
          __atomic_fetch_or(&mark[g], bits, __ATOMIC_RELAXED);
      };
      if (long_blocks && blocks_for(l) >= long_blocks) {  // threads may race on a granule: atomic OR
        for (uint64_t g = g0; g <= g1; ++g) mark_or(g, kMarkTouched | kMarkLong | (g < g1 ? kMarkCross : 0));
        last = UINT64_MAX;
        continue;
      }
      if (g0 == last && g1 == last) continue;
      for (uint64_t g = g0; g <= g1; ++g) mark_or(g, long_blocks && g < g1 ? kMarkTouched | kMarkCross : kMarkTouched);
      last = g1;
    }
    ShardSpan& r = acc[t];
    r.lo = lo;
    r.hi = hi;
    r.sum = sum;
    r.backward = backward;
    omin[t] = first_off;  // the chunk's first start: compared with the earlier chunks' largest
    omax[t] = max_off;
  });
  ShardSpan sh;
  uint64_t run = 0;
  bool seen = false;
  for (unsigned t = 0; t < T; ++t) {
    const ShardSpan& r = acc[t];
    sh.lo = std::min(sh.lo, r.lo);
    sh.hi = std::max(sh.hi, r.hi);
    sh.sum += r.sum;
    if (omin[t] == UINT64_MAX && omax[t] == 0) continue;  // an empty chunk
    sh.backward |= r.backward || (seen && omin[t] <= run);
    run = seen ? std::max(run, omax[t]) : omax[t];
    seen = true;
  }
  if (sh.any()) {  // the granules of the span's ends are the extreme marked ones
    sh.g0 = (sh.lo - glo) >> gs;
    sh.g1 = (sh.hi - 1 - glo) >> gs;
  }
  if (long_blocks && sh.any()) {
    // A payload crossing from a long granule into a plain one (or back) takes
    // the plain one into the long class: a forward sweep carries the class
    // right across crossed boundaries, a backward sweep left. (A long payload
    // marked every granule it touches, and its boundaries crossed.)
    for (uint64_t g = sh.g0; g < sh.g1; ++g)
      if ((mark[g] & (kMarkLong | kMarkCross)) == (kMarkLong | kMarkCross)) mark[g + 1] |= kMarkLong;
    for (uint64_t g = sh.g1; g-- > sh.g0;)
      if ((mark[g] & kMarkCross) && (mark[g + 1] & kMarkLong)) mark[g] |= kMarkLong;
  }
  return sh;
}

ShardSpan stage_and_mark(const uint64_t* O, const uint64_t* L, uint64_t m, uint64_t glo, unsigned gs,
                         uint64_t* h_off, uint64_t* h_len, std::vector<uint8_t>& mark, uint64_t long_blocks) {
  return h_off ? stage_and_mark_t<true>(O, L, m, glo, gs, h_off, h_len, mark, long_blocks)
               : stage_and_mark_t<false>(O, L, m, glo, gs, h_off, h_len, mark, long_blocks);
}

// gmap[g] = device offset of granule gbase + g or UINT64_MAX (not uploaded), g
// < ng; gbase == UINT64_MAX: nothing is marked. Granules holding long payloads
// (kMarkLong) come first, then the other marked ones, each class back to back
// in granule order. Returns the device bytes.
uint64_t build_gmap(const std::vector<uint8_t>& mark, uint64_t gbase, uint64_t ng, unsigned gs, uint64_t* gmap) {
  uint64_t dev = 0;
  for (int cls = 0; cls < 2; ++cls)
    for (uint64_t g = 0; g < ng; ++g) {
      const uint8_t mk = gbase != UINT64_MAX ? mark[gbase + g] : 0;
      if (!mk) {
        if (cls == 0) gmap[g] = UINT64_MAX;
        continue;
      }
      if (((mk & kMarkLong) != 0) != (cls == 0)) continue;
      gmap[g] = dev;
      dev += 1ull << gs;
    }
  return dev;
}

// The shard's uploads: f(caller offset, device offset, bytes) for each run of
// mapped granules, clipped to the shard's payload span [lo, hi) (so never past
// the arena), in ascending device order (the long payloads' granules first,
// build_gmap), split where device offsets cross a kDirectChunk boundary.
template <class F>
void for_each_upload(const uint64_t* gmap, const std::vector<uint8_t>& mark, uint64_t ng, uint64_t gbase,
                     uint64_t glo, unsigned gs, uint64_t lo, uint64_t hi, F&& f, uint64_t piece_bytes = kDirectChunk) {
  const uint64_t G = 1ull << gs;
  for (int cls = 0; cls < 2; ++cls) {
    auto in_cls = [&](uint64_t g) {
      return gmap[g] != UINT64_MAX && ((mark[gbase + g] & kMarkLong) != 0) == (cls == 0);
    };
    for (uint64_t g = 0; g < ng;) {
      if (!in_cls(g)) {
        ++g;
        continue;
      }
      uint64_t g1 = g;
      while (g1 < ng && in_cls(g1)) ++g1;  // a run of one class: contiguous on the device
      const uint64_t h0 = std::max(lo, glo + (gbase + g) * G), h1 = std::min(hi, glo + (gbase + g1) * G);
      for (uint64_t pos = h0; pos < h1;) {
        const uint64_t r = pos - glo;
        const uint64_t dev = gmap[(r >> gs) - gbase] + (r & (G - 1));
        const uint64_t piece = std::min(h1 - pos, (dev / piece_bytes + 1) * piece_bytes - dev);
        f(pos, dev, piece);
        pos += piece;
      }
      g = g1;
    }
  }
}

// One pass over a host call's messages (threaded): validation (every message
// inside the arena), the covered span, totals, the OR of the offsets
// (alignment), the largest block count, and the partition's piece sums.
struct BatchScan {
  uint64_t lo = UINT64_MAX, hi = 0, sum = 0, blocks = 0, offbits = 0, bmax = 0;
  std::vector<uint64_t> csum;  // piece_sums() layout
};

void scan_batch(const uint8_t* arena, uint64_t arena_len, const uint64_t* off, const uint64_t* len, uint64_t n,
                BatchScan& r) {
  const uint64_t P = std::max<uint64_t>(1, (n + kPiece - 1) / kPiece);
  r.csum.assign(P + 1, 0);
  struct Acc {
    uint64_t lo = UINT64_MAX, hi = 0, sum = 0, offbits = 0, bmax = 0, bad = UINT64_MAX;
  };
  const unsigned T = std::min<unsigned>(plan_threads(n), (unsigned)P);
  std::vector<Acc> acc(T);
  parallel_chunks(P, T, [&](unsigned t, uint64_t p0, uint64_t p1) {
    Acc a;
    for (uint64_t p = p0; p < p1 && a.bad == UINT64_MAX; ++p) {
      // branch-free over the piece (the compiler vectorises it); a piece with a
      // bad message is re-scanned for the first one
      const uint64_t i0 = p * kPiece, i1 = std::min(n, (p + 1) * kPiece);
      uint64_t blocks = 0, lo = a.lo, hi = a.hi, sum = a.sum, bits = a.offbits, bmax = a.bmax, bad = 0;
      for (uint64_t i = i0; i < i1; ++i) {
        const uint64_t o = off[i], l = len[i];
        bad |= (uint64_t)(l > arena_len) | (uint64_t)(o > arena_len - l);
        bits |= o;
        lo = std::min(lo, o);
        hi = std::max(hi, o + l);
        sum += l;
        const uint64_t b = blocks_for(l);
        blocks += b;
        bmax = std::max(bmax, b);
      }
      if (bad) {
        for (uint64_t i = i0; i < i1; ++i)
          if (len[i] > arena_len || off[i] > arena_len - len[i]) {
            a.bad = i;
            break;
          }
        break;
      }
      a.lo = lo;
      a.hi = hi;
      a.sum = sum;
      a.offbits = bits;
      a.bmax = bmax;
      r.csum[p + 1] = blocks;
    }
    acc[t] = a;
  });
  r.offbits = reinterpret_cast<uintptr_t>(arena);
  for (const Acc& a : acc) {  // pieces in index order: the first bad message is reported
    if (a.bad != UINT64_MAX)
      throw MshaError(MSHA_ERR_INVALID_ARG, "message " + std::to_string(a.bad) + " [off+len] outside arena");
    r.lo = std::min(r.lo, a.lo);
    r.hi = std::max(r.hi, a.hi);
    r.sum += a.sum;
    r.offbits |= a.offbits;
    r.bmax = std::max(r.bmax, a.bmax);
  }
  for (uint64_t p = 0; p < P; ++p) r.csum[p + 1] += r.csum[p];
  r.blocks = r.csum[P];
}

// Direct (pinned-arena) host call, planned on the GPU. Each shard, on a host
// thread of its own (for_each_shard), and with no whole-batch phase after the
// scan:
//   1. one threaded pass over its messages stages their raw (off, len) in
//      pinned memory and marks the granules (>= 64 KiB) of the arena they touch;
//   2. the copy stream uploads the metadata and granule map, then the marked
//      byte ranges (runs of granules, compacted) in 64 MiB device pieces with
//      one event each -- no gather copy;
//   3. the planner kernels (plan.hip) fold aliases, order the lanes by (piece
//      completing the payload, descending block count) and write lane-indexed
//      off/len/slot; the host reads back the group cuts and per-group minima;
//   4. each lane group is launched behind its piece's event, and the digest
//      slots that are final stream back after each launch.
// The host's share of the call is the scan and pass 1, ~2 passes over 16 bytes
// per message; everything per-lane runs on the GPU.
// A one-use barrier for the shard threads of one call. A thread that leaves
// early (an empty shard, an exception) still counts itself in (Arrival's
// destructor) so the others never wait forever.
struct CallBarrier {
  std::mutex mu;
  std::condition_variable cv;
  uint32_t left;
  explicit CallBarrier(uint32_t n) : left(n) {}
  void arrive(bool wait) {
    std::unique_lock<std::mutex> g(mu);
    if (--left == 0) cv.notify_all();
    else if (wait) cv.wait(g, [&] { return left == 0; });
  }
};
struct Arrival {
  CallBarrier* b;
  bool done = false;
  void wait() {
    if (b && !done) b->arrive(true);
    done = true;
  }
  ~Arrival() {
    if (b && !done) b->arrive(false);
  }
};

// Has event e completed? (A not-ready query leaves no error behind for a later
// hipGetLastError to pick up.)
bool event_done(hipEvent_t e) {
  const hipError_t r = hipEventQuery(e);
  if (r == hipSuccess) return true;
  (void)hipGetLastError();
  if (r != hipErrorNotReady) HIPCHK(r);
  return false;
}

// memcpy of a large contiguous range on the calling thread's pool (>= 2 MiB a thread).
void copy_threads(uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  WorkerPool& pool = cur_pool();
  const unsigned T = (unsigned)std::min<uint64_t>(pool.size(), std::max<uint64_t>(1, bytes >> 21));
  if (T <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const std::function<void(unsigned)> job = [&](unsigned t) {
    const uint64_t a = (bytes * t / T) & ~uint64_t(63), b = t + 1 == T ? bytes : (bytes * (t + 1) / T) & ~uint64_t(63);
    std::memcpy(dst + a, src + a, b - a);
  };
  pool.run(T, job);
}

// Pinned off/len of a one-shard call: uploaded to the shard's p_meta as the
// call starts, before validation, which the link would otherwise sit idle for
// (c5 on one GPU: 1.3 ms of a 72 ms call). Only the direct path consumes the
// upload; on any other path (or an error) the destructor drains it, so off/len
// are no longer read once the call returns.
struct EarlyMeta {
  Device* d = nullptr;
  bool used = false;
  EarlyMeta(msha_ctx* ctx, const uint64_t* off, const uint64_t* len, uint64_t n) {
    if (ctx->devs.size() != 1 || n <= small_msgs()) return;
    if (!(is_pinned_host(off) && is_pinned_host(off + n - 1) && is_pinned_host(len) && is_pinned_host(len + n - 1)))
      return;
    Device& dv = ctx->devs[0];
    HIPCHK(hipSetDevice(dv.id));
    dv.p_meta.ensure(16 * n);
    HIPCHK(hipEventRecord(dv.ev_up0, dv.copy_stream));
    HIPCHK(hipMemcpyAsync(dv.p_meta.p, off, 8 * n, hipMemcpyHostToDevice, dv.copy_stream));
    HIPCHK(hipMemcpyAsync(dv.p_meta.as<uint64_t>() + n, len, 8 * n, hipMemcpyHostToDevice, dv.copy_stream));
    d = &dv;
  }
  bool queued() const { return d != nullptr; }
  ~EarlyMeta() {
    if (d && !used) (void)hipStreamSynchronize(d->copy_stream);
  }
};

void run_direct(msha_ctx* ctx, double t0, uint64_t n, const uint64_t* off, const uint64_t* len,
                const uint8_t* arena, uint8_t* out, const BatchScan& sc, EarlyMeta* early, bool staged) {
  const uint32_t k = (uint32_t)ctx->devs.size();
  const bool out_pinned = is_pinned_host(out) && is_pinned_host(out + 32 * n - 1);
  // Interleaving knobs (tests, read per call): upload pieces of 2^MSHA_DIRECT_PIECE_SHIFT
  // device bytes (16..26; 26 = 64 MiB, the default) and, on the staged path,
  // staging slots of MSHA_STAGED_SLOT_BYTES (64 KiB .. 32 MiB, the default) with
  // a pause of MSHA_STAGED_DELAY_US before each refill. Small pieces and slots
  // and a pause make the plan arrive, and heads and lane groups launch, between
  // slot refills while later pieces still upload (tests/test_gpu_parity.py
  // test_staged_direct_interleaved).
  const unsigned piece_shift =
      (unsigned)std::min<uint64_t>(msha::kDirectChunkShift, std::max<uint64_t>(16, env_u64("MSHA_DIRECT_PIECE_SHIFT", msha::kDirectChunkShift)));
  const uint64_t piece_bytes = 1ull << piece_shift;
  const uint64_t slot_bytes =
      std::min<uint64_t>(kChunkBytes, std::max<uint64_t>(64 << 10, env_u64("MSHA_STAGED_SLOT_BYTES", kChunkBytes))) & ~uint64_t(63);
  const uint64_t slot_delay_us = std::min<uint64_t>(env_u64("MSHA_STAGED_DELAY_US", 0), 100000);
  // off/len in pinned memory (msha_pinned_alloc, as the Go adapter packs them):
  // uploaded as they are, no staging copy (one shard: already on the way, EarlyMeta)
  const bool meta_early = early && early->queued();
  if (meta_early) early->used = true;
  const bool meta_pinned = meta_early || (is_pinned_host(off) && is_pinned_host(off + n - 1) &&
                                          is_pinned_host(len) && is_pinned_host(len + n - 1));
  std::vector<uint64_t> bounds(k + 1);
  if (k == 1) {
    bounds[0] = 0;
    bounds[1] = n;
  } else {
    partition_pieces(len, n, k, sc.csum, bounds.data());
  }
  // One granule grid over the batch's span: at most 2^20 granules of >= 64 KiB.
  unsigned gs = 16;
  while (((sc.hi - (sc.lo & ~((1ull << gs) - 1))) >> gs) >= (1ull << 20)) ++gs;
  const uint64_t G = 1ull << gs;
  const uint64_t glo = sc.lo & ~(G - 1);
  const uint64_t nG = ((sc.hi - glo) >> gs) + 1;
  // Shards sharing one GPU (MSHA_VIRTUAL_SHARDS) share its PCIe link and DMA
  // engines: every shard's metadata goes up before any shard's payload, or a
  // shard's planner waits behind the other shards' payload (up to the whole
  // batch). Separate GPUs have links of their own and never wait on each other.
  bool shared_gpu = false;
  for (uint32_t s = 1; s < k; ++s) shared_gpu |= ctx->devs[s].id == ctx->devs[0].id;
  CallBarrier meta_up(k), plan_up(k);
  std::vector<uint8_t> meta_queued(k, 0);
  std::vector<Plan>& plans = ctx->plans;
  plans.resize(k);
  for (uint32_t s = 0; s < k; ++s) {
    Plan& P = plans[s];
    P = Plan{};
    P.ordered = true;
    Device& d = ctx->devs[s];
    d.lo = bounds[s];
    d.hi = bounds[s + 1];
    d.st = msha_shard_stats{};
    d.st.device = d.id;
  }
  for_each_shard(ctx, [&](uint32_t s) {
    Device& d = ctx->devs[s];
    Plan& P = plans[s];
    Arrival arrival{shared_gpu ? &meta_up : nullptr}, arrival2{shared_gpu ? &plan_up : nullptr};
    const uint64_t m = d.hi - d.lo;
    P.m = m;
    d.st.messages = m;
    if (m == 0) return;
    const uint64_t* O = off + d.lo;
    const uint64_t* L = len + d.lo;
    HIPCHK(hipSetDevice(d.id));
    // 1. stage (off, len) (unless the caller's arrays are pinned), mark granules, the shard's span.
    // Pinned off/len go up right away, under the marking pass (c5 on one GPU:
    // 134 MB, ~2.5 ms of PCIe that no longer waits for the host).
    d.p_meta.ensure(16 * m);
    if (meta_pinned && !meta_early) {
      HIPCHK(hipEventRecord(d.ev_up0, d.copy_stream));
      HIPCHK(hipMemcpyAsync(d.p_meta.p, O, 8 * m, hipMemcpyHostToDevice, d.copy_stream));
      HIPCHK(hipMemcpyAsync(d.p_meta.as<uint64_t>() + m, L, 8 * m, hipMemcpyHostToDevice, d.copy_stream));
    }
    if (!meta_pinned) d.h_meta.ensure(16 * m);
    uint64_t* h_off = meta_pinned ? nullptr : d.h_meta.as<uint64_t>();
    uint64_t* h_len = meta_pinned ? nullptr : h_off + m;
    std::vector<uint8_t>& mark = d.direct_mark;
    mark.assign(nG, 0);
    // Long chains (>= kLongBlocks blocks) get their payloads uploaded first and,
    // when few enough, a head launch of their own (below).
    const uint64_t long_blocks = long_chain_blocks(sc.bmax, ctx->kernel_policy);
    const ShardSpan sh = stage_and_mark(O, L, m, glo, gs, h_off, h_len, mark, long_blocks);
    const bool any = sh.any();                       // some payload byte at all
    const uint64_t gbase = any ? sh.g0 : 0, ng = any ? sh.g1 - sh.g0 + 1 : 1;
    d.h_gmap.ensure(8 * ng);
    uint64_t* gmap = d.h_gmap.as<uint64_t>();
    const uint64_t dev_bytes = build_gmap(mark, any ? gbase : UINT64_MAX, ng, gs, gmap);
    d.arena_bytes = dev_bytes;
    trace("staged + marked", s, t0);
    // 2. uploads: metadata + granule map first (the planner needs them)
    const uint64_t pieces = std::max<uint64_t>(1, (dev_bytes + piece_bytes - 1) / piece_bytes);
    const uint64_t chunks = long_blocks ? 2 * pieces : pieces;  // lane groups: (region, piece)
    d.arena.ensure(dev_bytes + msha::kArenaSlack);
    d.p_gmap.ensure(8 * ng);
    while (d.span_ev.size() < pieces) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      d.span_ev.push_back(e);
    }
    if (!meta_pinned) {
      HIPCHK(hipEventRecord(d.ev_up0, d.copy_stream));
      HIPCHK(hipMemcpyAsync(d.p_meta.p, h_off, 16 * m, hipMemcpyHostToDevice, d.copy_stream));
    }
    HIPCHK(hipMemcpyAsync(d.p_gmap.p, gmap, 8 * ng, hipMemcpyHostToDevice, d.copy_stream));
    HIPCHK(hipEventRecord(d.ev_meta, d.copy_stream));
    meta_queued[s] = 1;
    arrival.wait();  // shared GPU: every shard's metadata is queued before any planner or payload
    // 3. planning on the GPU, behind the metadata. Queued before the payload:
    // with streams of several shards sharing a GPU's hardware queues (HIP
    // multiplexes streams over GPU_MAX_HW_QUEUES), a planner queued behind
    // another stream's payload or kernel waits would wait for them too.
    // a message at or below an earlier start may repeat a payload: fold aliases
    // (a span test -- bytes > span -- missed a shard whose own messages are sparse
    // in the arena while its EpochChange re-hashes point back into a shared pool)
    const bool aliases = m > 1 && any && sh.backward;
    const uint64_t B = chunks * (sc.bmax + 1) <= (1u << 20) ? sc.bmax + 1 : 1;
    const uint64_t nb = chunks * B;
    uint64_t cap = 1024;
    while (cap < 2 * m) cap <<= 1;
    d.p_devoff.ensure(8 * m);
    d.p_rep.ensure(4 * m);
    d.p_cnt.ensure(4 * nb);
    d.p_small.ensure(4 * (2 * chunks + 2));
    if (aliases) {
      d.p_table.ensure(4 * cap);
      d.p_slot.ensure(4 * m);
    }
    d.off.ensure(8 * m);
    d.len.ensure(8 * m);
    d.order.ensure(4 * m);
    d.out.ensure(32 * m);
    d.err.ensure(4);
    d.h_out.ensure(32 * m + 4);
    d.h_small.ensure(4 * (2 * chunks + 2));
    if (aliases) d.h_rep.ensure(4 * m);
    if (aliases) HIPCHK(hipMemsetAsync(d.p_table.p, 0, 4 * cap, d.stream));
    HIPCHK(hipMemsetAsync(d.p_cnt.p, 0, 4 * nb, d.stream));
    HIPCHK(hipMemsetAsync(d.p_small.p, 0xFF, 4 * chunks, d.stream));  // gmin
    HIPCHK(hipMemsetAsync(d.err.p, 0, 4, d.stream));
    HIPCHK(hipStreamWaitEvent(d.stream, d.ev_meta, 0));
    HIPCHK(hipEventRecord(d.ev_p0, d.stream));
    msha::PlanArgs pa;
    pa.off = d.p_meta.as<uint64_t>();
    pa.len = pa.off + m;
    pa.gmap = d.p_gmap.as<uint64_t>();
    pa.glo = glo;
    pa.gbase = gbase;
    pa.gshift = gs;
    pa.m = m;
    pa.dev_off = d.p_devoff.as<uint64_t>();
    pa.table = aliases ? d.p_table.as<uint32_t>() : nullptr;
    pa.tmask = cap - 1;
    pa.slot = aliases ? d.p_slot.as<uint32_t>() : nullptr;
    pa.rep = d.p_rep.as<uint32_t>();
    pa.pieces = pieces;
    pa.piece_shift = piece_shift;
    pa.long_blocks = long_blocks;
    pa.chunks = chunks;
    pa.B = B;
    pa.bmax = sc.bmax;
    pa.nb = nb;
    pa.cnt = d.p_cnt.as<uint32_t>();
    pa.gmin = d.p_small.as<uint32_t>();
    pa.cut = pa.gmin + chunks;
    pa.info = pa.cut + chunks + 1;
    pa.lane_off = d.off.as<uint64_t>();
    pa.lane_len = d.len.as<uint64_t>();
    pa.lane_slot = d.order.as<uint32_t>();
    HIPCHK(msha::launch_plan(pa, d.stream));
    HIPCHK(hipEventRecord(d.ev_p1, d.stream));
    HIPCHK(hipMemcpyAsync(d.h_small.p, d.p_small.p, 4 * (2 * chunks + 2), hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipEventRecord(d.ev_plan, d.stream));
    if (aliases) HIPCHK(hipMemcpyAsync(d.h_rep.p, d.p_rep.p, 4 * m, hipMemcpyDeviceToHost, d.stream));
    d.st.d2h_bytes = 4 * (2 * chunks + 2) + (aliases ? 4 * m : 0);
    // 4. the payload: behind every shard's metadata on a shared GPU
    arrival2.wait();  // shared GPU: every shard's planner is queued before any payload
    for (uint32_t o = 0; shared_gpu && o < k; ++o)
      if (o != s && meta_queued[o] && ctx->devs[o].id == d.id)
        HIPCHK(hipStreamWaitEvent(d.copy_stream, ctx->devs[o].ev_meta, 0));
    // 5. the plan's lane groups (read back once the planner is done), each
    // launched behind the upload piece that completes its payloads. The long
    // chains' groups (region 0: their payloads went up first), when they hold
    // at most head_cap lanes, run as heads: the two-lane chain kernel on CUs of
    // their own (k_digest_chain2 EXCL), on the side stream, so they start as
    // soon as their piece lands, beside the lane kernel, instead of crawling on
    // it (~2x the cycles per block) -- or ending the call when the caller packed
    // them last (weak #6 of round 3). Their digests go to p_head, lane-indexed,
    // and are placed after the sync (finish_shard).
    bool planned = false;
    size_t groups = 0, next_group = 0, next_head = 0;
    std::vector<std::pair<uint64_t, uint64_t>> head_groups;  // (lane cut, piece) of region-0 groups
    auto read_plan = [&] {
      d.st.plan_kernel_ms = elapsed_ms(d.ev_p0, d.ev_p1);
      const uint32_t* gmin = d.h_small.as<uint32_t>();
      const uint32_t* cut = gmin + chunks;
      P.lanes = cut[chunks];
      d.st.lanes = P.lanes;
      P.rep_dev = aliases ? d.h_rep.as<uint32_t>() : nullptr;
      const uint64_t head_lanes = long_blocks ? cut[pieces] : 0;  // region 0 = lanes [0, cut[pieces])
      const bool heads = head_lanes > 0 && head_lanes <= head_cap(d);
      P.head = heads ? head_lanes : 0;
      P.launched = P.head;
      d.st.head_lanes = (uint32_t)P.head;
      // lane groups: one per (region, piece) that completes at least one payload
      P.lane_cut.assign(1, P.head);
      P.cut_chunk.clear();
      head_groups.clear();
      std::vector<uint64_t> gm;
      for (uint64_t q = 0; q < chunks; ++q) {
        if (cut[q + 1] == cut[q]) continue;
        if (heads && q < pieces) {
          head_groups.push_back({cut[q + 1], q});
          continue;
        }
        P.lane_cut.push_back(cut[q + 1]);
        P.cut_chunk.push_back(q % pieces);
        gm.push_back(gmin[q]);
      }
      groups = gm.size();
      P.later_min.assign(groups + 1, m);
      for (size_t g = groups; g-- > 0;) P.later_min[g] = std::min<uint64_t>(gm[g], P.later_min[g + 1]);
      if (heads) {
        d.p_head.ensure(32 * P.head);
        d.h_head.ensure(36 * P.head);
      }
      planned = true;
      trace("planned on GPU", s, t0);
    };
    auto launch_upto = [&](uint64_t pieces_queued) {  // pieces [0, pieces_queued) have their events
      for (; next_head < head_groups.size() && head_groups[next_head].second < pieces_queued; ++next_head)
        launch_head(ctx, d, P, next_head ? head_groups[next_head - 1].first : 0, head_groups[next_head].first,
                    d.span_ev[head_groups[next_head].second], t0);
      for (; next_group < groups && P.cut_chunk[next_group] < pieces_queued; ++next_group) {
        HIPCHK(hipStreamWaitEvent(d.stream, d.span_ev[P.cut_chunk[next_group]], 0));
        launch_lanes(ctx, d, P, next_group, next_group + 1 == groups, t0, out, out_pinned);
      }
    };
    // event c once every byte below device offset (c+1)*piece_bytes is queued
    uint64_t c = 0, uploaded = 0;
    auto pieces_done = [&](uint64_t dev_end) {
      for (; c < pieces && (c + 1) * piece_bytes <= dev_end; ++c) HIPCHK(hipEventRecord(d.span_ev[c], d.copy_stream));
    };
    unsigned slot_i = 0;
    if (staged) {  // two pinned staging slots, refilled as their H2D drains
      d.slot[0].ensure(kChunkBytes);
      d.slot[1].ensure(kChunkBytes);
      HIPCHK(hipEventRecord(d.slot_free[0], d.copy_stream));
      HIPCHK(hipEventRecord(d.slot_free[1], d.copy_stream));
    }
    if (any)
      for_each_upload(gmap, mark, ng, gbase, glo, gs, sh.lo, sh.hi, [&](uint64_t pos, uint64_t dev, uint64_t bytes) {
        if (!staged) {  // the caller's pinned bytes, DMA'd as they are
          HIPCHK(hipMemcpyAsync(d.arena.as<uint8_t>() + dev, arena + pos, bytes, hipMemcpyHostToDevice,
                                d.copy_stream));
          uploaded += bytes;
          pieces_done(dev + bytes);
          return;
        }
        // pageable: copied into a staging slot by the shard's threads (large
        // contiguous runs, not message by message), then DMA'd; kernels start
        // as their pieces land and the planner's result is in
        for (uint64_t o = 0; o < bytes;) {
          const uint64_t take = std::min(bytes - o, slot_bytes);
          const unsigned si = slot_i++ & 1;
          HIPCHK(hipEventSynchronize(d.slot_free[si]));
          if (slot_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(slot_delay_us));
          const double g0 = now_ms();
          copy_threads(d.slot[si].as<uint8_t>(), arena + pos + o, take);
          const double g1 = now_ms();
          if (d.st.gather_begin_ms == 0) d.st.gather_begin_ms = std::max(g0 - t0, 1e-6);
          d.st.gather_end_ms = g1 - t0;
          d.st.gather_ms += g1 - g0;
          HIPCHK(hipMemcpyAsync(d.arena.as<uint8_t>() + dev + o, d.slot[si].p, take, hipMemcpyHostToDevice,
                                d.copy_stream));
          HIPCHK(hipEventRecord(d.slot_free[si], d.copy_stream));
          o += take;
          uploaded += take;
          pieces_done(dev + o);
          if (!planned && event_done(d.ev_plan)) read_plan();
          if (planned) launch_upto(c);
        }
      }, piece_bytes);
    for (; c < pieces; ++c) HIPCHK(hipEventRecord(d.span_ev[c], d.copy_stream));
    HIPCHK(hipEventRecord(d.ev_up1, d.copy_stream));
    d.st.h2d_payload_bytes = uploaded;
    d.st.h2d_bytes = 16 * m + 8 * ng;
    trace("payload queued", s, t0);
    if (!planned) {
      HIPCHK(hipEventSynchronize(d.ev_plan));
      read_plan();
    }
    launch_upto(pieces);
    queue_tail(d, P, out, out_pinned);
    finish_shard(ctx, s, out, out_pinned, t0);
  });
  double t_plan = t0;  // plan_ms: until the last shard's first kernel is queued
  for (const Device& d : ctx->devs) t_plan = std::max(t_plan, t0 + d.st.first_launch_ms);
  call_stats(ctx, t0, t_plan);
}

}  // namespace

extern "C" {

uint32_t msha_abi_version(void) { return MSHA_ABI_VERSION; }

int msha_device_count(int* n) {
  if (!n) return MSHA_ERR_INVALID_ARG;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) {
    (void)hipGetLastError();
    c = 0;
  }
  *n = c;
  return MSHA_OK;
}

int msha_ctx_create_err(uint32_t device_mask, msha_ctx** out, char* errbuf, uint64_t errbuf_len) {
  if (errbuf && errbuf_len) errbuf[0] = 0;
  if (!out) {
    set_create_error("null out pointer", errbuf, errbuf_len);
    return MSHA_ERR_INVALID_ARG;
  }
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    (void)hipGetLastError();
    set_create_error("no HIP device available (the engine has no CPU fallback)", errbuf, errbuf_len);
    return MSHA_ERR_NO_DEVICE;
  }
  if (device_mask == 0) device_mask = 1;
  msha_ctx* ctx = new (std::nothrow) msha_ctx();
  if (!ctx) {
    set_create_error("host allocation failed", errbuf, errbuf_len);
    return MSHA_ERR_OUT_OF_MEMORY;
  }
  int rc = guarded(ctx, [&] {
    // MSHA_VIRTUAL_SHARDS=k (testing only): a one-device mask is split into k
    // shards on that same GPU, each with its own streams and buffers, so the
    // multi-GPU sharding path can be exercised on a one-GPU box.
    int virt = 1;
    if (const char* e = getenv("MSHA_VIRTUAL_SHARDS")) virt = std::max(1, std::min(8, atoi(e)));
    if ((device_mask & (device_mask - 1)) != 0) virt = 1;
    for (int i = 0; i < 32; ++i) {
      if (!(device_mask & (1u << i))) continue;
      if (i >= count)
        throw MshaError(MSHA_ERR_NO_DEVICE, "device_mask names device " + std::to_string(i) + " but only " +
                                                std::to_string(count) + " visible");
      for (int v = 0; v < virt; ++v) {
        Device d;
        d.id = i;
        HIPCHK(hipSetDevice(i));
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, i));
        d.cus = prop.multiProcessorCount;
        d.numa = gpu_numa_node(i);
        HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&d.copy_stream, hipStreamNonBlocking));
        if (virt == 1) {
          HIPCHK(hipStreamCreateWithFlags(&d.d2h_stream, hipStreamNonBlocking));
          HIPCHK(hipEventCreateWithFlags(&d.ev_k, hipEventDisableTiming));
        }
        HIPCHK(hipEventCreate(&d.ev0));
        HIPCHK(hipEventCreate(&d.ev1));
        HIPCHK(hipEventCreate(&d.ev_up0));
        HIPCHK(hipEventCreate(&d.ev_up1));
        HIPCHK(hipEventCreate(&d.ev_k0));
        HIPCHK(hipEventCreate(&d.ev_p0));
        HIPCHK(hipEventCreate(&d.ev_p1));
        HIPCHK(hipEventCreateWithFlags(&d.ev_meta, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.ev_plan, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.slot_free[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.slot_free[1], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.chunk_in, hipEventDisableTiming));
        d.st.device = i;
        d.index = (uint32_t)ctx->devs.size();
        ctx->devs.push_back(std::move(d));
      }
    }
  });
  if (rc != MSHA_OK) {
    set_create_error(std::string(ctx->err), errbuf, errbuf_len);
    for (auto& d : ctx->devs) d.release();
    delete ctx;
    return rc;
  }
  *out = ctx;
  return MSHA_OK;
}

int msha_ctx_create(uint32_t device_mask, msha_ctx** out) {
  return msha_ctx_create_err(device_mask, out, nullptr, 0);
}

void msha_ctx_destroy(msha_ctx* ctx) {
  if (!ctx) return;
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d.id);
    for (hipStream_t st : {d.stream, d.copy_stream, d.d2h_stream})
      if (st) (void)hipStreamSynchronize(st);
    d.release();
  }
  for (const auto& a : ctx->pinned) pinned_release(a);
  delete ctx;
}

const char* msha_last_error(const msha_ctx* ctx) { return ctx ? ctx->err : g_create_error; }

uint64_t msha_last_error_copy(const msha_ctx* ctx, char* buf, uint64_t buf_len) {
  std::unique_lock<std::mutex> lock(ctx ? ctx->mu : g_create_mu);
  const char* e = ctx ? ctx->err : g_create_error;
  const uint64_t n = std::strlen(e);
  if (buf && buf_len) {
    const uint64_t c = std::min(n, buf_len - 1);
    std::memcpy(buf, e, c);
    buf[c] = 0;
  }
  return n;
}

int msha_get_stats(const msha_ctx* ctx, msha_stats* out) {
  if (!ctx || !out) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  *out = ctx->stats;
  return MSHA_OK;
}

int msha_shard_count(const msha_ctx* ctx, uint32_t* n) {
  if (!ctx || !n) return MSHA_ERR_INVALID_ARG;
  *n = (uint32_t)ctx->devs.size();
  return MSHA_OK;
}

int msha_get_shard_stats(const msha_ctx* ctx, uint32_t shard, msha_shard_stats* out) {
  if (!ctx || !out || shard >= ctx->devs.size()) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);
  *out = ctx->devs[shard].st;
  return MSHA_OK;
}

uint64_t msha_blocks_for_len(uint64_t len) { return blocks_for(len); }

int msha_order_by_blocks(const uint64_t* len, uint64_t n, uint32_t* order) {
  if (n && (!len || !order)) return MSHA_ERR_INVALID_ARG;
  if (n > 0xffffffffull) return MSHA_ERR_INVALID_ARG;
  try {
    std::vector<uint32_t> tmp;
    order_by_blocks_desc(len, n, order, tmp);
  } catch (...) {
    return MSHA_ERR_OUT_OF_MEMORY;
  }
  return MSHA_OK;
}

int msha_partition_by_blocks(const uint64_t* len, uint64_t n, uint32_t n_shards, uint64_t* bounds) {
  if (!bounds || n_shards == 0 || (n && !len)) return MSHA_ERR_INVALID_ARG;
  partition(len, n, n_shards, bounds);
  return MSHA_OK;
}

int msha_alias_first(const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* first) {
  if (n && (!off || !len || !first)) return MSHA_ERR_INVALID_ARG;
  if (n >= 0xffffffffull) return MSHA_ERR_INVALID_ARG;
  try {
    std::vector<uint64_t> uid, table, bucket;
    std::vector<uint32_t> tag;
    alias_uids(off, len, n, uid, table, bucket, tag);
    std::memcpy(first, uid.data(), 8 * n);
  } catch (...) {
    return MSHA_ERR_OUT_OF_MEMORY;
  }
  return MSHA_OK;
}

int msha_digest_batch(msha_ctx* ctx, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                      const uint64_t* len, uint64_t n, uint8_t* out) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!off || !len || !out || (arena_len && !arena))
    return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  if (n >= 0xffffffffull) return fail(ctx, MSHA_ERR_INVALID_ARG, "more than 2^32-2 messages in one call");
  const double t0 = now_ms();
  return guarded(ctx, [&] {
    EarlyMeta early(ctx, off, len, n);
    BatchScan sc;
    scan_batch(arena, arena_len, off, len, n, sc);
    const uint64_t lo = sc.lo, hi = sc.hi, sum = sc.sum;
    const bool aligned16 = (sc.offbits & 15) == 0;
    auto count = [&] {
      ctx->stats.messages += n;
      ctx->stats.message_bytes += sum;
      ctx->stats.blocks += sc.blocks;
    };
    if (n <= small_msgs()) {  // the latency path (run_small)
      // A pinned arena goes up as is only above 512 KiB: below that, packing it
      // behind the metadata (one H2D instead of two) is the faster of the two
      // (tools/latency.cpp: 32 KiB pinned 57 us as two copies, 44 us packed).
      const bool span = small_bytes() > 0 && aligned16 && hi - lo > kSmallSpanMin &&
                        hi - lo <= small_span_bytes() && is_pinned_host(arena + lo) &&
                        is_pinned_host(arena + hi - 1);
      // Packed, an aliased payload goes up once: offsets that strictly increase
      // cannot repeat a payload (the common case, one pass); otherwise the
      // host's alias detection names each message's first.
      uint64_t packed = 0;
      bool increasing = true;
      for (uint64_t i = 0; i < n && !span; ++i) {
        packed += round16(len[i]);
        increasing = increasing && (i == 0 || off[i] > off[i - 1]);
      }
      std::vector<uint64_t> first;
      if (!span && !increasing) {
        std::vector<uint64_t> table, bucket;
        std::vector<uint32_t> tag;
        alias_uids(off, len, n, first, table, bucket, tag);
        packed = 0;
        for (uint64_t i = 0; i < n; ++i)
          if (first[i] == i) packed += round16(len[i]);
      }
      if (span || small_call(n, packed)) {
        const SmallSpan sp{arena, off, lo, hi};
        run_small(ctx, t0, n, len, out, [&](uint64_t i, uint8_t* dst) { std::memcpy(dst, arena + off[i], len[i]); },
                  span ? &sp : nullptr, first.empty() ? nullptr : first.data());
        ctx->stats.direct_calls += span;
        count();
        return;
      }
    }
    trace("validated", t0);
    // Zero-copy upload when the caller packed into pinned memory (msha_pinned_alloc)
    // with 16-byte aligned message starts and little waste between messages:
    // the touched byte ranges go up as they are and the GPU plans the lanes.
    // A pageable arena of the same shape takes the same path, its touched runs
    // copied through pinned staging slots (staged_calls; MSHA_STAGED_DIRECT=0:
    // the gather pipeline below instead).
    const bool dense = aligned16 && hi > lo && hi - lo <= std::min(sum, hi - lo) + 16 * n + (1u << 20);
    const bool pinned = dense && is_pinned_host(arena + lo) && is_pinned_host(arena + hi - 1);
    if (pinned || (dense && env_u64("MSHA_STAGED_DIRECT", 1) != 0)) {
      run_direct(ctx, t0, n, off, len, arena, out, sc, &early, !pinned);
      (pinned ? ctx->stats.direct_calls : ctx->stats.staged_calls)++;
      count();
      return;
    }
    // Overlapping payloads (sum of lengths > the span they cover) means there
    // may be aliases: give every message the index of the first message with
    // the same (off, len).
    const bool aliases = n > 1 && sum > hi - lo;
    if (aliases) alias_uids(off, len, n, ctx->uid, ctx->alias_table, ctx->alias_bucket, ctx->alias_tag);
    trace("aliases", t0);
    std::vector<uint64_t> bounds(ctx->devs.size() + 1);
    partition_pieces(len, n, (uint32_t)ctx->devs.size(), sc.csum, bounds.data());
    run_pipeline(ctx, t0, n, len, aliases ? ctx->uid.data() : nullptr, out,
                 [&](uint64_t i, uint8_t* dst) { std::memcpy(dst, arena + off[i], len[i]); }, bounds.data());
    count();
  });
}

int msha_hash_actions(msha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* part_off, const uint64_t* part_len, uint64_t n_parts,
                      const uint64_t* action_part_begin, uint64_t n_actions, uint8_t* out) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n_actions == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!action_part_begin || !out || (n_parts && (!part_off || !part_len)) || (arena_len && !arena))
    return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  if (action_part_begin[0] != 0 || action_part_begin[n_actions] != n_parts)
    return fail(ctx, MSHA_ERR_INVALID_ARG, "action_part_begin must start at 0 and end at n_parts");
  const double t0 = now_ms();
  return guarded(ctx, [&] {
    // One threaded pass (2^18 parts and up) after the cheap monotonicity check:
    // each thread validates the parts of its actions and sums their lengths
    // (h.Write appends, so an action's message is its parts back to back). The
    // error names the first bad part, as a serial scan would.
    const unsigned T = plan_threads(std::max(n_actions, n_parts));
    std::vector<uint64_t> bad(T, UINT64_MAX);
    parallel_chunks(n_actions, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i)
        if (action_part_begin[i + 1] < action_part_begin[i]) {
          bad[t] = i;
          return;
        }
    });
    for (uint64_t b : bad)
      if (b != UINT64_MAX) throw MshaError(MSHA_ERR_INVALID_ARG, "action_part_begin must be non-decreasing");
    std::vector<uint64_t>& alen = ctx->tmp_len;
    alen.resize(n_actions);
    std::vector<uint64_t> packed_t(T, 0), bytes_t(T, 0), blocks_t(T, 0);
    parallel_chunks(n_actions, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
      uint64_t packed = 0, bytes = 0, blocks = 0;
      for (uint64_t i = lo; i < hi; ++i) {
        uint64_t l = 0;
        for (uint64_t j = action_part_begin[i]; j < action_part_begin[i + 1]; ++j) {
          if (part_len[j] > arena_len || part_off[j] > arena_len - part_len[j]) {
            bad[t] = j;
            return;
          }
          l += part_len[j];
        }
        alen[i] = l;
        packed += round16(l);
        bytes += l;
        blocks += blocks_for(l);
      }
      packed_t[t] = packed;
      bytes_t[t] = bytes;
      blocks_t[t] = blocks;
    });
    for (uint64_t b : bad)
      if (b != UINT64_MAX) throw MshaError(MSHA_ERR_INVALID_ARG, "part " + std::to_string(b) + " outside arena");
    uint64_t packed = 0, bytes = 0, blocks = 0;
    for (unsigned t = 0; t < T; ++t) {
      packed += packed_t[t];
      bytes += bytes_t[t];
      blocks += blocks_t[t];
    }
    auto gather = [&](uint64_t a, uint8_t* dst) {
      for (uint64_t j = action_part_begin[a]; j < action_part_begin[a + 1]; ++j) {
        std::memcpy(dst, arena + part_off[j], part_len[j]);
        dst += part_len[j];
      }
    };
    if (small_call(n_actions, packed))
      run_small(ctx, t0, n_actions, alen.data(), out, gather);
    else
      run_pipeline(ctx, t0, n_actions, alen.data(), nullptr, out, gather);
    ctx->stats.messages += n_actions;
    ctx->stats.message_bytes += bytes;
    ctx->stats.blocks += blocks;
  });
}

int msha_digest_of_digests(msha_ctx* ctx, const uint8_t* table, uint64_t n_table,
                           const uint32_t* idx, uint64_t n_idx, const uint64_t* begin, uint64_t n,
                           uint8_t* out) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!begin || !out || (n_idx && !idx) || (n_table && !table))
    return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  if (begin[0] != 0 || begin[n] != n_idx)
    return fail(ctx, MSHA_ERR_INVALID_ARG, "begin must start at 0 and end at n_idx");
  for (uint64_t i = 0; i < n; ++i)
    if (begin[i + 1] < begin[i]) return fail(ctx, MSHA_ERR_INVALID_ARG, "begin must be non-decreasing");
  return guarded(ctx, [&] {
    {  // threaded from 2^18 indices on
      const unsigned T = plan_threads(n_idx);
      std::vector<uint8_t> bad(T, 0);
      parallel_chunks(n_idx, T, [&](unsigned t, uint64_t lo, uint64_t hi) {
        uint32_t worst = 0;
        for (uint64_t k = lo; k < hi; ++k) worst = std::max(worst, idx[k]);
        bad[t] = hi > lo && worst >= n_table;
      });
      for (uint8_t b : bad)
        if (b) throw MshaError(MSHA_ERR_INVALID_ARG, "idx out of table range");
    }
    std::vector<uint64_t>& alen = ctx->tmp_len;
    alen.resize(n);
    uint64_t packed = 0;
    for (uint64_t i = 0; i < n; ++i) {
      alen[i] = 32 * (begin[i + 1] - begin[i]);
      packed += alen[i];  // multiples of 32: already 16-aligned
    }
    if (small_call(n, packed) && packed <= kSmallDodBytes) {  // latency path: a Batch's digests = one message
      run_small(ctx, now_ms(), n, alen.data(), out, [&](uint64_t i, uint8_t* dst) {
        for (uint64_t k = begin[i]; k < begin[i + 1]; ++k, dst += 32) std::memcpy(dst, table + 32 * (uint64_t)idx[k], 32);
      });
      uint64_t blocks = 0;
      for (uint64_t i = 0; i < n; ++i) blocks += blocks_for(alen[i]);
      ctx->stats.messages += n;
      ctx->stats.message_bytes += 32 * n_idx;
      ctx->stats.blocks += blocks;
      return;
    }
    const uint32_t k = (uint32_t)ctx->devs.size();
    std::vector<uint64_t> bounds(k + 1);
    partition(alen.data(), n, k, bounds.data());
    double t0 = now_ms();
    for (uint32_t s = 0; s < k; ++s) {
      Device& d = ctx->devs[s];
      const uint64_t lo = bounds[s], hi = bounds[s + 1], m = hi - lo;
      d.lo = lo;
      d.hi = hi;
      d.st = msha_shard_stats{};
      d.st.device = d.id;
      d.st.messages = d.st.lanes = m;
      if (m == 0) continue;
      const uint64_t i0 = begin[lo], i1 = begin[hi];
      HIPCHK(hipSetDevice(d.id));
      d.table.ensure(32 * std::max<uint64_t>(n_table, 1));
      d.idx.ensure(4 * std::max<uint64_t>(i1 - i0, 1));
      d.begin.ensure(8 * (m + 1));
      d.out.ensure(32 * m);
      d.h_meta.ensure(8 * (m + 1));
      uint64_t* hb = d.h_meta.as<uint64_t>();
      for (uint64_t i = 0; i <= m; ++i) hb[i] = begin[lo + i] - i0;
      if (n_table) HIPCHK(hipMemcpyAsync(d.table.p, table, 32 * n_table, hipMemcpyHostToDevice, d.stream));
      if (i1 > i0) HIPCHK(hipMemcpyAsync(d.idx.p, idx + i0, 4 * (i1 - i0), hipMemcpyHostToDevice, d.stream));
      HIPCHK(hipMemcpyAsync(d.begin.p, hb, 8 * (m + 1), hipMemcpyHostToDevice, d.stream));
      d.err.ensure(4);
      HIPCHK(hipMemsetAsync(d.err.p, 0, 4, d.stream));
      HIPCHK(hipEventRecord(d.ev0, d.stream));
      d.st.h2d_payload_bytes = 32 * n_table;
      d.st.h2d_bytes = 32 * n_table + 4 * (i1 - i0) + 8 * (m + 1);
      msha::SplitPlan sp;
      msha::LaunchKind kind;
      HIPCHK(msha::launch_digest_of_digests(d.table.as<uint8_t>(), d.idx.as<uint32_t>(),
                                            d.begin.as<uint64_t>(), m, d.out.as<uint8_t>(),
                                            d.err.as<uint32_t>(), d.stream,
                                            split_for(d, m, ctx->kernel_policy, sp, msha::kMaxSegmentsDod),
                                            &kind));
      count_launch(ctx, &d, kind);
      HIPCHK(hipEventRecord(d.ev1, d.stream));
      d.h_out.ensure(32 * m + 4);
      HIPCHK(hipMemcpyAsync(d.h_out.p, d.out.p, 32 * m, hipMemcpyDeviceToHost, d.stream));
      HIPCHK(hipMemcpyAsync(d.h_out.as<uint8_t>() + 32 * m, d.err.p, 4, hipMemcpyDeviceToHost, d.stream));
      d.st.d2h_bytes = 32 * m + 4;
    }
    double kernel_ms = 0;
    uint64_t h2d = 0, d2h = 0;
    for (uint32_t s = 0; s < k; ++s) {
      Device& d = ctx->devs[s];
      const uint64_t m = d.hi - d.lo;
      if (m == 0) continue;
      HIPCHK(hipSetDevice(d.id));
      HIPCHK(hipStreamSynchronize(d.stream));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, d.ev0, d.ev1));
      d.st.device_ms = ms;
      kernel_ms = std::max<double>(kernel_ms, ms);
      uint32_t errflag;
      std::memcpy(&errflag, d.h_out.as<uint8_t>() + 32 * m, 4);
      if (errflag & 2) {
        // a split chain's handoff timed out (its digests are undefined): the
        // inputs are still on the device, re-hash the shard unsplit
        HIPCHK(hipMemsetAsync(d.err.p, 0, 4, d.stream));
        msha::LaunchKind kind;
        HIPCHK(msha::launch_digest_of_digests(d.table.as<uint8_t>(), d.idx.as<uint32_t>(),
                                              d.begin.as<uint64_t>(), m, d.out.as<uint8_t>(),
                                              d.err.as<uint32_t>(), d.stream, nullptr, &kind));
        count_launch(ctx, &d, kind);
        HIPCHK(hipMemcpyAsync(d.h_out.p, d.out.p, 32 * m, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        d.st.d2h_bytes += 32 * m;
        ctx->stats.split_retries++;
      }
      std::memcpy(out + 32 * d.lo, d.h_out.p, 32 * m);
      h2d += d.st.h2d_bytes;
      d2h += d.st.d2h_bytes;
    }
    uint64_t blocks = 0;
    for (uint64_t i = 0; i < n; ++i) blocks += blocks_for(alen[i]);
    ctx->stats.calls++;
    ctx->stats.messages += n;
    ctx->stats.message_bytes += 32 * n_idx;
    ctx->stats.blocks += blocks;
    ctx->stats.plan_ms = 0;
    ctx->stats.pack_ms = 0;
    ctx->stats.device_ms = kernel_ms;
    ctx->stats.h2d_bytes = h2d;
    ctx->stats.d2h_bytes = d2h;
    ctx->stats.total_ms = now_ms() - t0;
  });
}

int msha_digest_batch_device(msha_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                             const uint64_t* d_len, const uint32_t* d_order, uint64_t n,
                             uint8_t* d_out, void* stream) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!d_arena || !d_off || !d_len || !d_out) return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  return guarded(ctx, [&] {
    hipStream_t st;
    device_prologue(ctx, stream, &st);
    Device& d = ctx->devs[0];
    msha::SplitPlan sp;
    msha::LaunchKind kind;
    HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, d_order, nullptr, n, d_out,
                                     d.err.as<uint32_t>(), d.cus, ctx->kernel_policy, st,
                                     split_for(d, n, ctx->kernel_policy, sp), &kind));
    count_launch(ctx, nullptr, kind);
  });
}

int msha_digest_batch_device_planned(msha_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                                     const uint64_t* d_len, uint64_t n, uint32_t flags, uint8_t* d_out,
                                     void* stream) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!d_arena || !d_off || !d_len || !d_out) return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  if (flags & ~(uint32_t)MSHA_PLAN_FOLD_ALIASES) return fail(ctx, MSHA_ERR_INVALID_ARG, "unknown plan flags");
  if (n >= (1ull << 31)) return fail(ctx, MSHA_ERR_INVALID_ARG, "planned device batches hold < 2^31 messages");
  return guarded(ctx, [&] {
    hipStream_t st;
    device_prologue(ctx, stream, &st);
    Device& d = ctx->devs[0];
    // Not capturable into a HIP graph (mirsha.h): the call waits on the previous
    // planned call's event, recorded outside any capture, and forks to and joins
    // from a library-owned side stream. Say so instead of failing inside HIP.
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cap_status));
    if (cap_status != hipStreamCaptureStatusNone)
      throw MshaError(MSHA_ERR_INVALID_ARG,
                     "msha_digest_batch_device_planned cannot be captured into a HIP graph; "
                     "use msha_digest_batch_device there");
    const bool fold = flags & MSHA_PLAN_FOLD_ALIASES;
    // Few messages: one cooperative launch over the planned order (every
    // workgroup gets a CU); otherwise the lane kernel, its longest chains
    // (if any outlast the launch) on the cooperative kernel beside it.
    const bool all_coop = msha::uses_coop(n, d.cus, ctx->kernel_policy);
    const bool head = !all_coop && ctx->kernel_policy != MSHA_KERNEL_LANE && env_u64("MSHA_PLAN_HEAD", 1) != 0;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    // one zeroed block: info (32 words, 128 bytes), the bucket counters,
    // then FoldArgs::big -- cleared by ONE memset per call
    // (+ the work-stealing lane kernel's tile counters)
    const uint64_t fold_zero_fixed = 128 + 4 * msha::kFoldBuckets + 16 * msha::kFoldBigBuckets +
                                     4 * msha::kWsSlots * msha::kWsStride + 4 * 2 * msha::kGridWords;
    // Round 6: a folded call's insert finds its tile prefix by look-back (plan.hip
    // tile_lookback) over status words zeroed with the rest -- no k_fold_tilemax /
    // k_fold_tilescan and their two dependent launches. MSHA_FOLD_LOOKBACK=0: the
    // two-kernel prefix (A/B).
    const bool lookback = fold && env_u64("MSHA_FOLD_LOOKBACK", 1) != 0;
    const uint64_t ptiles = (n + 4095) / 4096;
    static_assert((128 + 4 * msha::kFoldBuckets + 16 * msha::kFoldBigBuckets + 4 * msha::kWsSlots * msha::kWsStride +
                   4 * 2 * msha::kGridWords) % 8 == 0,
                  "the look-back's status words follow 8-byte aligned");
    // (a multiple of 64 bytes: an unaligned tail made hipMemsetAsync a second fill kernel)
    const uint64_t fold_zero = (fold_zero_fixed + (lookback ? 8 * (ptiles + 1) : 0) + 63) / 64 * 64;
    d.f_cnt.ensure(fold_zero);
    d.f_key.ensure(2 * n);
    d.f_tkeys.ensure(8 * n + 4 * ((n + 4095) / 4096) + 8 * 4096);  // per-tile key lists, then their counts
    d.f_order.ensure(4 * n);
    bool clear_table = false;
    if (fold) {
      // epoch-tagged slots (plan.hip fold_claim): cleared only when the table
      // is (re)allocated -- hipMalloc does not zero -- or the epoch wraps. A
      // reallocation is told by the capacity, not the pointer: hipFree then
      // hipMalloc can hand back the same address, and the grown tail would then
      // hold recycled words whose high half may equal the current epoch.
      const uint64_t cap_before = d.f_table.cap;
      d.f_table.ensure(8 * cap);
      const bool grown = d.f_table.cap != cap_before;
      // MSHA_POISON_FOLD_TABLE=1 (tests): a fresh allocation is filled with words
      // tagged with the coming epoch, as recycled memory may be -- a table that
      // was not cleared then claims garbage indices (tests/test_gpu_planned.py)
      if (grown && env_u64("MSHA_POISON_FOLD_TABLE", 0))
        HIPCHK(hipMemsetD32Async((hipDeviceptr_t)d.f_table.p, d.f_epoch + 1, d.f_table.cap / 4, st));
      if (grown || d.f_epoch == 0xFFFFFFFFu) {
        clear_table = true;
        d.f_epoch = 0;
      }
      ++d.f_epoch;
      d.f_rep.ensure(8 * n + 4 * ((n + 4095) / 4096));  // alias pairs, then their count per tile
      d.f_tmax.ensure(8 * 3 * ((n + 4095) / 4096));  // tile maxima, then 2 x tsum per tile
    }
    // The planner's scratch (table, order, counters) is the context's: a call
    // on another stream must not overwrite it while an earlier call still reads it.
    if (!d.ev_fdone) HIPCHK(hipEventCreateWithFlags(&d.ev_fdone, hipEventDisableTiming));
    if (d.fdone_recorded) HIPCHK(hipStreamWaitEvent(st, d.ev_fdone, 0));
    // With a head, the planner and then the head's cooperative launch run on
    // the side stream, and the lane kernel on `stream` waits for the planner's
    // event: the head's packet follows the planner in its own queue while the
    // lane kernel's needs a cross-queue signal, so the head's workgroups are
    // resident before the lane kernel fills every SIMD (queued the other way
    // round, the head could not get a CU's registers until the lane kernel
    // drained: c5 folded 6.2 ms, its 1,427-block chain starting at the end).
    // Round 6: the memsets, the insert and the scan run on the caller's stream, and
    // the side stream joins at the scatter (with the early head's list), so a step
    // starts without a cross-queue hand-off (~20 us of a folded c5 step's timeline,
    // profiles/r06_plan7/).
    hipStream_t ps = st;  // the scatter's and the late head's
    if (head) {
      if (!d.side_stream) HIPCHK(hipStreamCreateWithFlags(&d.side_stream, hipStreamNonBlocking));
      for (hipEvent_t* e : {&d.ev_fork, &d.ev_fplan, &d.ev_join})
        if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
      ps = d.side_stream;
    }
    if (clear_table) HIPCHK(hipMemsetAsync(d.f_table.p, 0, d.f_table.cap, st));
    HIPCHK(hipMemsetAsync(d.f_cnt.p, 0, fold_zero, st));
    // (the order's positions past the last lane are filled by k_fold_scatter)
    msha::FoldArgs fa;
    fa.off = d_off;
    fa.len = d_len;
    fa.n = n;
    fa.vec = ((reinterpret_cast<uintptr_t>(d_off) | reinterpret_cast<uintptr_t>(d_len)) & 15) == 0;
    fa.table = fold ? d.f_table.as<uint64_t>() : nullptr;
    fa.tmask = cap - 1;
    fa.epoch = d.f_epoch;
    fa.apairs = fold ? d.f_rep.as<uint64_t>() : nullptr;
    fa.acount = fold ? reinterpret_cast<uint32_t*>(fa.apairs + n) : nullptr;
    fa.tmax = fold ? d.f_tmax.as<uint64_t>() : nullptr;
    fa.tsum = fold ? fa.tmax + (n + 4095) / 4096 : nullptr;
    fa.info = d.f_cnt.as<uint32_t>();
    fa.cnt = fa.info + 32;
    fa.key16 = d.f_key.as<uint16_t>();
    fa.tkeys = d.f_tkeys.as<uint64_t>();
    fa.tkcount = reinterpret_cast<uint32_t*>(fa.tkeys + (n + 4095) / 4096 * 4096);
    fa.big = reinterpret_cast<uint64_t*>(fa.cnt + msha::kFoldBuckets);  // kFoldBuckets is even: 8-byte aligned
    fa.order = d.f_order.as<uint32_t>();
    fa.tstat = lookback ? reinterpret_cast<uint64_t*>(d.f_cnt.as<uint8_t>() + fold_zero_fixed) : nullptr;
    fa.grid_ws = reinterpret_cast<uint32_t*>(fa.big + 2 * msha::kFoldBigBuckets) + msha::kWsSlots * msha::kWsStride;
    fa.simds = (uint32_t)d.cus * 4;
    // The head's kernel. Folded, a head is the few distinct long payloads: the
    // two-lane chain (k_digest_chain2, 64 messages per CU, ~10 % fewer cycles a
    // block) shortens it. Unfolded, a storm's head can be thousands of chains
    // (19,456 over 8 GPUs): the cooperative kernel holds twice as many per CU,
    // and the two-lane one made that case 3.0 -> 4.2 ms (profiles/r03_chain_dpp/).
    // MSHA_HEAD_CHAIN2: 0 never, 2 always (A/B).
    const uint64_t chain2_env = env_u64("MSHA_HEAD_CHAIN2", 1);
    const bool two_lane = chain2_env == 2 || (chain2_env == 1 && fold);
    // Round 5: the EARLY head runs on the eight-lane kernel (k_digest_chain8:
    // ~9 % fewer cycles a round, 24 messages a CU instead of 64). It exists only
    // when its chain outlasts the lane kernel's share, so its latency is the
    // call's; the late head (after the scan's cut, when the early head stood
    // down: the lane kernel is the long pole) keeps the denser two-lane kernel --
    // on it the eight-lane one took 5 CUs' worth of the lane kernel's SIMDs for
    // c5's 100 payloads, one GPU 2.73 -> 2.84 ms (profiles/r05_chain8/).
    // MSHA_HEAD_CHAIN8=0: the early head on the two-lane kernel too (A/B).
    const bool eight_lane = two_lane && env_u64("MSHA_HEAD_CHAIN8", 1) != 0;
    fa.head_per_wg = two_lane ? msha::kChain2MsgsPerWg : msha::kCoopMsgsPerWg;
    fa.head_cap = head ? (uint32_t)std::min<uint64_t>(n, (uint64_t)d.cus * fa.head_per_wg) : 0;
    // cycles a chain block: two-lane head 1,427 blocks in 2.04 ms at ~2.4 GHz (r04);
    // eight-lane (the early head): tools/chain2_anatomy 1427 8, profiles/r05_chain8/
    fa.coop_cycles = two_lane ? 3500 : 4200;
    fa.early_cycles = eight_lane ? 3250 : 3500;  // eight-lane: 1,427 blocks in 1.93 ms at ~2.4 GHz (r05)
    fa.tiebreak = (uint32_t)env_u64("MSHA_PLAN_TIEBREAK", 1);
    fa.race_test = (uint32_t)env_u64("MSHA_FOLD_LONGS_SKIP_ODD", 0);
    // The lane kernel of a folded call steals work (k_digest_batch_ws: folded c5
    // 2.79 -> 2.69 ms, profiles/r06_ws/); an unfolded one keeps the statically
    // mapped kernel, whose oldest-first issue runs a storm's thousands of long
    // chains one after another (work stealing: 13.3 -> 17.6 ms). MSHA_LANE_WS:
    // 0 never, 2 always (A/B).
    const uint64_t lane_ws = env_u64("MSHA_LANE_WS", 1);
    const bool ws = !all_coop && (lane_ws == 2 || (lane_ws == 1 && fold));
    // MSHA_WS_LONG=k (A/B): the cut also keeps chains of >= k blocks off it. Every
    // k tried lost to the cost model alone, which takes fewer head CUs (folded c5,
    // 3 reps: 2.661-2.669 ms; k = 600 / 256 / 64: 2.715-2.719 / 2.709-2.744 /
    // 2.725-2.736; static lane kernel 2.78-2.89; profiles/r06_ws2/)
    const uint64_t ws_long_env = env_u64("MSHA_WS_LONG", 0);
    fa.ws_long = ws ? (ws_long_env ? (uint32_t)std::min<uint64_t>(ws_long_env, 0xFFFFFFFFull) : 0xFFFFFFFFu) : 0u;
    fa.head_pct = (uint32_t)env_u64("MSHA_PLAN_HEAD_PCT", 100);
    fa.lane_cycles = (uint32_t)env_u64("MSHA_PLAN_LANE_CYCLES", fa.lane_cycles);  // A/B of the cost model
    fa.wave_block_cycles = (uint32_t)env_u64("MSHA_PLAN_WAVE_CYCLES", fa.wave_block_cycles);
    // The early head (folded calls with a two-lane head): unless the tile prefix
    // already stood it down (the short messages alone outlast the longest chain),
    // the distinct payloads of >= kLongBlocks blocks are listed (k_fold_longs,
    // beside the alias insert) and, when at most an eighth of the CUs' worth,
    // start on the two-lane kernel on a stream of their own right then, while
    // the insert, the scan and the scatter still run -- a folded storm's head
    // does not wait for the whole plan. MSHA_EARLY_HEAD=0: the head after the
    // scan's cut (A/B).
    const bool early = fold && head && two_lane && env_u64("MSHA_EARLY_HEAD", 1) != 0;
    if (early) {
      fa.long_blocks = (uint32_t)kLongBlocks;
      fa.long_cap = (uint32_t)(d.cus * (eight_lane ? msha::kChain8MsgsPerWg : msha::kChain2MsgsPerWg) / 8);
      d.f_longs.ensure(4 * (uint64_t)fa.long_cap);
      fa.longs = d.f_longs.as<uint32_t>();
      if (!d.head_stream) HIPCHK(hipStreamCreateWithFlags(&d.head_stream, hipStreamNonBlocking));
      for (hipEvent_t* e : {&d.ev_longs, &d.ev_join2})
        if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    // Round 6 A/B (MSHA_EARLY_FORK=1): the head's stream forks before the tile
    // prefix, right after the memsets, and makes its first decision itself
    // (k_fold_longs_gate over len). The chain then starts ~13 us sooner over 8
    // GPUs with no measurable step change, and one GPU lost ~27 us (the gate's
    // pass beside the prefix): off by default (profiles/r06_call4/).
    // With the look-back there is no tile prefix to decide in: the gate always
    // decides (64 workgroups; MSHA_GATE_WGS).
    // Round 6 (MSHA_INSERT_LIST): with the look-back, the insert's own claims list
    // the early head and the scan decides it -- no gate or list pass beside the
    // insert -- and no late head runs (FoldArgs::insert_list).
    const bool insert_list = early && lookback && env_u64("MSHA_INSERT_LIST", 0) != 0;
    fa.insert_list = insert_list;
    fa.early_fork = early && !insert_list && (lookback || env_u64("MSHA_EARLY_FORK", 0) != 0);
    fa.longs_wgs = (uint32_t)env_u64("MSHA_LONGS_WGS", 0);
    fa.gate_wgs = (uint32_t)env_u64("MSHA_GATE_WGS", 0);
    // Round 6 A/B (MSHA_EARLY_ONLY=1): the early head takes every distinct long
    // payload whether or not its chain is the call's long pole -- on the eight-lane
    // kernel when it is, the two-lane one when the lane kernel is (both launched, the
    // list's last workgroup arms one) -- and no late head is launched: the scatter
    // and the lane kernel follow on the caller's stream, without the side stream's
    // two cross-queue hand-offs. Payloads the list cannot hold stay lanes.
    const bool early_only = insert_list || (fa.early_fork && env_u64("MSHA_EARLY_ONLY", 0) != 0);
    fa.early_only = early_only;
    const bool late_head = head && !early_only;
    if (fa.early_fork) {
      HIPCHK(hipEventRecord(d.ev_longs, st));
      HIPCHK(hipStreamWaitEvent(d.head_stream, d.ev_longs, 0));
    }
    HIPCHK(msha::launch_fold_prefix(fa, st));
    // the early head's launches on its stream: after the list (k_fold_longs) or,
    // listed by the insert, after the scan (its event recorded by launch_fold_plan,
    // so these are queued after that call)
    auto launch_early_head = [&]() {
      msha::LaneGate eg;
      eg.head = early_only && eight_lane ? fa.info + 20 : fa.info + 4;
      eg.head_part = true;
      eg.two_lane = true;
      eg.eight_lane = eight_lane;
      msha::LaunchKind ek;
      HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, fa.longs, nullptr, fa.long_cap, d_out,
                                       d.err.as<uint32_t>(), d.cus, MSHA_KERNEL_COOP, d.head_stream, nullptr,
                                       &ek, &eg));
      count_launch(ctx, nullptr, ek);
      if (early_only && eight_lane) {  // the same list on the two-lane kernel when not the long pole
        eg.head = fa.info + 21;
        eg.eight_lane = false;
        HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, fa.longs, nullptr, fa.long_cap, d_out,
                                         d.err.as<uint32_t>(), d.cus, MSHA_KERNEL_COOP, d.head_stream, nullptr,
                                         &ek, &eg));
        count_launch(ctx, nullptr, ek);
      }
      HIPCHK(hipEventRecord(d.ev_join2, d.head_stream));
    };
    if (early && !insert_list) {
      // the list runs beside the tile prefix (forked) or after it, and beside the
      // alias insert
      if (!fa.early_fork) {
        HIPCHK(hipEventRecord(d.ev_longs, st));
        HIPCHK(hipStreamWaitEvent(d.head_stream, d.ev_longs, 0));
      }
      HIPCHK(msha::launch_fold_longs(fa, d.cus, d.head_stream));
      HIPCHK(hipEventRecord(d.ev_longs, d.head_stream));
      launch_early_head();
    }
    HIPCHK(msha::launch_fold_plan(fa, st, late_head ? ps : st, d.ev_fork,
                                  early && !insert_list ? d.ev_longs : nullptr,
                                  insert_list ? d.ev_longs : nullptr));
    if (insert_list) {  // (ev_longs here: after the scan, on st)
      HIPCHK(hipStreamWaitEvent(d.head_stream, d.ev_longs, 0));
      // the lane kernel waits until the head's stream reaches its launches (an event
      // recorded just before them): dispatched together, the lane kernel ran ~25 %
      // more cycles a block (profiles/r06_il_stamps/); the wait overlaps the scatter
      if (env_u64("MSHA_INSERT_LIST_SYNC", 1)) {
        if (!d.ev_hready) HIPCHK(hipEventCreateWithFlags(&d.ev_hready, hipEventDisableTiming));
        HIPCHK(hipEventRecord(d.ev_hready, d.head_stream));
      }
      launch_early_head();
    }
    const uint32_t* order = d.f_order.as<uint32_t>();
    msha::LaunchKind kind;
    if (all_coop) {
      HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, order, nullptr, n, d_out, d.err.as<uint32_t>(),
                                       d.cus, MSHA_KERNEL_COOP, st, nullptr, &kind));
      count_launch(ctx, nullptr, kind);
    } else {
      msha::LaneGate body;
      body.head = fa.info + 1;
      // Round 6: the body on the work-stealing lane kernel (kernels.hip
      // k_digest_batch_ws), over the planned lanes only (fa.ws_long, set before
      // the plan: the cut then keeps long chains off it)
      if (fa.ws_long) {
        body.ws_ctr = reinterpret_cast<uint32_t*>(fa.big + 2 * msha::kFoldBigBuckets);
        body.lanes = fa.info;
      }
      if (late_head) {
        HIPCHK(hipEventRecord(d.ev_fplan, d.side_stream));
        msha::LaneGate hg;
        hg.head = fa.info + 5;  // the scan's cut (0 when the early head has the long lanes)
        hg.head_part = true;
        hg.two_lane = two_lane;
        HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, order, nullptr, fa.head_cap, d_out,
                                         d.err.as<uint32_t>(), d.cus, MSHA_KERNEL_COOP, d.side_stream, nullptr,
                                         &kind, &hg));
        count_launch(ctx, nullptr, kind);
        HIPCHK(hipEventRecord(d.ev_join, d.side_stream));
        HIPCHK(hipStreamWaitEvent(st, d.ev_fplan, 0));
      }
      if (insert_list && env_u64("MSHA_INSERT_LIST_SYNC", 1)) HIPCHK(hipStreamWaitEvent(st, d.ev_hready, 0));
      HIPCHK(msha::launch_digest_batch(d_arena, d_off, d_len, order, nullptr, n, d_out, d.err.as<uint32_t>(),
                                       d.cus, ctx->kernel_policy, st, nullptr, &kind, &body));
      count_launch(ctx, nullptr, kind);
      if (late_head) HIPCHK(hipStreamWaitEvent(st, d.ev_join, 0));
      if (early) HIPCHK(hipStreamWaitEvent(st, d.ev_join2, 0));
    }
    if (fold) HIPCHK(msha::launch_fold_fill(fa, d_out, st));
    if (lookback && env_u64("MSHA_CHECK_LOOKBACK", 0)) {  // tests: no look-back gave up (waits for the call)
      uint64_t gave_up = 0;
      HIPCHK(hipStreamSynchronize(st));
      HIPCHK(hipMemcpy(&gave_up, fa.tstat + ptiles, sizeof gave_up, hipMemcpyDeviceToHost));
      if (gave_up)
        throw MshaError(MSHA_ERR_HIP, "planner tile look-back gave up waiting " + std::to_string(gave_up) +
                                          " time(s) (digests exact, folding reduced)");
    }
    HIPCHK(hipEventRecord(d.ev_fdone, st));
    d.fdone_recorded = true;
    ctx->stats.planned_device_calls++;
    if (trace_on() || env_u64("MSHA_TRACE_PLAN", 0)) {  // MSHA_TRACE: the GPU's plan (waits for the call)
      uint32_t info[2] = {0, 0};
      HIPCHK(hipStreamSynchronize(st));
      HIPCHK(hipMemcpy(info, fa.info, sizeof info, hipMemcpyDeviceToHost));
      fprintf(stderr, "[msha] planned device call: %llu messages, %u lanes, head %u\n", (unsigned long long)n,
              info[0], info[1]);
    }
  });
}

int msha_digest_uniform_device(msha_ctx* ctx, const uint8_t* d_arena, uint64_t stride,
                               uint64_t msg_len, uint64_t n, uint8_t* d_out, void* stream) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!d_arena || !d_out) return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  if (stride % MSHA_DEVICE_ALIGN) return fail(ctx, MSHA_ERR_ALIGNMENT, "stride must be a multiple of 16");
  return guarded(ctx, [&] {
    hipStream_t st;
    device_prologue(ctx, stream, &st);
    Device& d = ctx->devs[0];
    msha::LaunchKind kind;
    HIPCHK(msha::launch_digest_uniform(d_arena, stride, msg_len, n, d_out, d.err.as<uint32_t>(), d.cus, st,
                                       &kind));
    count_launch(ctx, nullptr, kind);
  });
}

int msha_digest_of_digests_device(msha_ctx* ctx, const uint8_t* d_table, const uint32_t* d_idx,
                                  const uint64_t* d_begin, uint64_t n, uint8_t* d_out, void* stream) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  if (n == 0) return MSHA_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (!d_table || !d_idx || !d_begin || !d_out) return fail(ctx, MSHA_ERR_INVALID_ARG, "null pointer argument");
  return guarded(ctx, [&] {
    hipStream_t st;
    device_prologue(ctx, stream, &st);
    Device& d = ctx->devs[0];
    msha::SplitPlan sp;
    msha::LaunchKind kind;
    HIPCHK(msha::launch_digest_of_digests(d_table, d_idx, d_begin, n, d_out, d.err.as<uint32_t>(), st,
                                          split_for(d, n, ctx->kernel_policy, sp, msha::kMaxSegmentsDod),
                                          &kind));
    count_launch(ctx, nullptr, kind);
  });
}

int msha_set_kernel_policy(msha_ctx* ctx, int policy) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);

  if (policy != MSHA_KERNEL_AUTO && policy != MSHA_KERNEL_LANE && policy != MSHA_KERNEL_COOP)
    return fail(ctx, MSHA_ERR_INVALID_ARG, "unknown kernel policy " + std::to_string(policy));
  ctx->kernel_policy = policy;
  return MSHA_OK;
}

int msha_device_status(msha_ctx* ctx) {
  if (!ctx || ctx->devs.empty()) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);

  uint32_t flag = 0;
  int rc = guarded(ctx, [&] {
    Device& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    HIPCHK(hipDeviceSynchronize());
    if (!d.err.p) return;
    HIPCHK(hipMemcpy(&flag, d.err.p, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(d.err.p, 0, 4));
  });
  if (rc != MSHA_OK) return rc;
  if (flag & 2) return fail(ctx, MSHA_ERR_HIP, "split-chain handoff timed out (digests undefined)");
  if (flag) return fail(ctx, MSHA_ERR_ALIGNMENT, "device arena message start not 16-byte aligned");
  return MSHA_OK;
}

int msha_clock_probe(msha_ctx* ctx, uint32_t blocks_per_lane, msha_clock_info* out) {
  if (!ctx || ctx->devs.empty() || !out || blocks_per_lane == 0 || blocks_per_lane > 100000)
    return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);

  return guarded(ctx, [&] {
    Device& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    const uint32_t wgs = (uint32_t)d.cus * 8;  // 8 waves per SIMD, as the lane kernel runs
    d.probe.ensure(32ull * wgs + 64);
    uint64_t* stamps = d.probe.as<uint64_t>();
    uint32_t* sink = reinterpret_cast<uint32_t*>(stamps + 4ull * wgs);
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    struct Ev {
      hipEvent_t a, b;
      ~Ev() {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
      }
    } ev{e0, e1};
    HIPCHK(hipEventRecord(e0, d.stream));
    HIPCHK(msha::launch_clock_probe(blocks_per_lane, wgs, stamps, sink, d.stream));
    HIPCHK(hipEventRecord(e1, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint64_t> h(4ull * wgs);
    HIPCHK(hipMemcpy(h.data(), stamps, 8 * h.size(), hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    ghz.reserve(wgs);
    for (uint32_t g = 0; g < wgs; ++g) {
      const uint64_t dt = h[4 * g + 2] - h[4 * g], dr = h[4 * g + 3] - h[4 * g + 1];
      if (dr > 0) ghz.push_back((double)dt / (double)dr * 0.1);  // memrealtime: 100 MHz
    }
    if (ghz.empty()) throw MshaError(MSHA_ERR_HIP, "clock probe: no workgroup advanced memrealtime");
    std::sort(ghz.begin(), ghz.end());
    out->ghz_median = ghz[ghz.size() / 2];
    out->ghz_min = ghz.front();
    out->ghz_max = ghz.back();
    out->kernel_ms = ms;
    out->workgroups = wgs;
    out->blocks_per_lane = blocks_per_lane;
    out->gblocks_per_s = ms > 0 ? (double)wgs * 256 * blocks_per_lane / (ms * 1e-3) / 1e9 : 0;
  });
}

int msha_pinned_alloc(msha_ctx* ctx, uint64_t bytes, void** p) {
  if (!ctx || !p) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);

  return guarded(ctx, [&] {
    HIPCHK(hipSetDevice(ctx->devs[0].id));
    uint64_t mapped = 0;
    *p = stripe_pinned(ctx) ? striped_pinned_alloc(ctx, bytes, &mapped) : nullptr;
    if (!*p) HIPCHK(hipHostMalloc(p, std::max<uint64_t>(bytes, 1), hipHostMallocPortable));
    ctx->pinned.emplace_back(*p, mapped);
  });
}

int msha_pinned_free(msha_ctx* ctx, void* p) {
  if (!ctx) return MSHA_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lock(ctx->mu);

  auto it = std::find_if(ctx->pinned.begin(), ctx->pinned.end(), [&](const auto& a) { return a.first == p; });
  if (it == ctx->pinned.end()) return fail(ctx, MSHA_ERR_INVALID_ARG, "pointer not from msha_pinned_alloc");
  const std::pair<void*, uint64_t> a = *it;
  ctx->pinned.erase(it);
  return guarded(ctx, [&] {
    if (a.second) {
      HIPCHK(hipHostUnregister(a.first));
      munmap(a.first, a.second);
    } else {
      HIPCHK(hipHostFree(a.first));
    }
  });
}

}  // extern "C"
