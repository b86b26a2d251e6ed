// cpu_lane.cpp -- host build of the device arithmetic for the small-call path
// (see cpu_lane.hpp).  Compiled by g++ (NT_HD empty): the same verify_one<>,
// wcomb_acc<> and sha512_prefixed<> the gfx950 kernels run, with per-call
// tables on the stack and a 12-bit host comb of B.
#include "cpu_lane.hpp"

#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

// The device headers are compiled here into a namespace of their own (nt_lane),
// with the host-lane field multiply (NT_HOST_FAST_FE, fe25519.hpp): no inline
// definition of this TU can be merged with -- or interposed by -- the device
// arithmetic's host build in any other object or library.
#define NT_HOST_FAST_FE 1
#define nt nt_lane
#include "ed25519_ops.hpp"
#undef nt

namespace nt {
namespace cpu {
namespace {
using namespace nt_lane;

constexpr int kHostBBits = 12;
using HG = CombGeom<kHostBBits>;

std::vector<uint32_t>* g_comb = nullptr;
std::once_flag g_once;

// [pos][entry][kWStride words] as on the device (ed25519_ops.hpp wide combs)
struct HostComb {
  static constexpr int kBits = kHostBBits;
  const uint32_t* base;
  void load(uint32_t pos, uint32_t idx, ge_niels& q) const {
    const uint32_t* e = base + ((size_t)pos * HG::kEntries + idx) * kWStride;
    for (int i = 0; i < 10; ++i) {
      q.ypx.v[i] = e[i];
      q.ymx.v[i] = e[10 + i];
      q.xy2d.v[i] = e[20 + i];
    }
  }
};

// the lane's j*(+-A), j*(-R) tables (entries 0..8, 9..17)
struct HostATab {
  ge_cached e[18];
  void store(uint32_t j, const ge_cached& c) { e[j] = c; }
  void load(uint32_t j, ge_cached& c) const { c = e[j]; }
  void load_signed(uint32_t e0, int32_t d, ge_cached& c) const {
    c = e[e0 + (uint32_t)(d < 0 ? -d : d)];
    ge_cached_cneg(c, d < 0);
  }
};

void build(int threads) {
  auto* comb = new std::vector<uint32_t>(HG::kWordsPerPoint, 0u);
  uint32_t enc[8];
  for (int i = 0; i < 8; ++i) enc[i] = kBaseEnc[i];
  ge_p3 B;
  ge_frombytes_w(B, enc);
  std::vector<uint32_t> bases((size_t)HG::kPos * 40);
  wcomb_bases<kHostBBits>(bases.data(), B);
  parallel_for((uint64_t)HG::kPos * HG::kChunks, threads, [&](uint64_t t) {
    const uint32_t pos = (uint32_t)(t / HG::kChunks), c = (uint32_t)(t % HG::kChunks);
    uint32_t tmp[kWChunk * 10];
    uint32_t* dst = comb->data() + ((size_t)pos * HG::kEntries + 1 + (size_t)kWChunk * c) * kWStride;
    wcomb_fill<kHostBBits>(dst, tmp, bases.data() + (size_t)pos * 40, c);
  });
  g_comb = comb;
}

// Persistent workers for parallel_for_fn: a small call must not pay a thread
// creation per item (16 std::thread spawns cost ~400 us, more than a 67-vote
// certificate's verification on 16 threads).  A call enqueues a job; workers
// and the caller claim its items one at a time under the pool lock.
struct Job {
  const std::function<void(uint64_t)>* fn;
  uint64_t n;
  uint64_t next = 0;                // next unclaimed item (pool lock)
  std::atomic<uint64_t> done{0};    // finished items
};

class Pool {
 public:
  explicit Pool(int workers) {
    for (int t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(uint64_t n, const std::function<void(uint64_t)>& fn) {
    Job j;
    j.fn = &fn;
    j.n = n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(&j);
    }
    cv_.notify_all();
    for (;;) {  // the caller works on its own job
      uint64_t i;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (j.next >= n) break;
        i = j.next++;
        if (j.next == n) erase(&j);
      }
      fn(i);
      j.done.fetch_add(1);
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return j.done.load() == n; });
  }

 private:
  void erase(Job* j) {
    for (auto it = q_.begin(); it != q_.end(); ++it)
      if (*it == j) {
        q_.erase(it);
        return;
      }
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (stop_) return;
      Job* j = q_.front();
      const uint64_t i = j->next++, n = j->n;
      if (j->next == n) q_.pop_front();
      const std::function<void(uint64_t)>* fn = j->fn;
      lk.unlock();
      (*fn)(i);
      // the last access to *j: once done == n its caller may return
      const bool last = j->done.fetch_add(1) + 1 == n;
      lk.lock();
      if (last) done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Job*> q_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};

// One pool per process, sized once for the machine (at most 64 threads with
// the caller): a call's parallelism is its item count, capped by the pool.
int machine_threads() {
  const unsigned hw = std::thread::hardware_concurrency();
  return std::max(1, std::min(64, (int)(hw ? hw : 1)));
}
Pool& pool() {
  static Pool p(machine_threads() - 1);
  return p;
}

}  // namespace

void parallel_for_fn(uint64_t n, int threads, const std::function<void(uint64_t)>& fn) {
  // at most `threads` threads work on this call: it becomes T contiguous ranges
  const uint64_t T = std::min<uint64_t>(n, (uint64_t)std::max(1, std::min(threads, machine_threads())));
  if (T == n) {
    pool().run(n, fn);
    return;
  }
  const std::function<void(uint64_t)> range = [&](uint64_t t) {
    for (uint64_t i = n * t / T; i < n * (t + 1) / T; ++i) fn(i);
  };
  pool().run(T, range);
}

int pool_threads() { return machine_threads(); }

void init(int threads) {
  std::call_once(g_once, [threads] { build(threads); });
}

bool ready() { return g_comb != nullptr; }

void sha512_trunc32(const uint8_t* msg, uint64_t len, uint8_t out32[32]) {
  uint64_t st[8];
  sha512_prefixed<0>(st, nullptr, msg, len);
  uint32_t w[8];
  sha512_out_words(w, st, 8);
  std::memcpy(out32, w, 32);
}

bool key_decodes(const uint8_t pk32[32]) {
  uint32_t w[8];
  std::memcpy(w, pk32, 32);
  ge_p3 P;
  return ge_frombytes_w(P, w) != 0;
}

bool verify(int mode, const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t* msg, uint64_t len) {
  uint32_t A[8], R[8], S[8];
  std::memcpy(A, pk32, 32);
  std::memcpy(R, sig64, 32);
  std::memcpy(S, sig64 + 32, 32);
  HostATab at;
  const HostComb wb{g_comb->data()};
  const uint32_t ok = mode == nt_lane::kStrict ? verify_one<nt_lane::kStrict>(A, R, S, msg, len, at, wb)
                                               : verify_one<nt_lane::kCofactorless>(A, R, S, msg, len, at, wb);
  return ok != 0;
}

}  // namespace cpu
}  // namespace nt
