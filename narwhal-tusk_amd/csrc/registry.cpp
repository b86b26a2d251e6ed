// registry.cpp -- the key registry: the committee key cache behind the
// unchanged entry points (include/ntcrypto.h nt_set_key_cache).
//
// The reference's crate binds `Signature::verify` / `verify_batch`
// (crypto/src/lib.rs:200-219) with raw `PublicKey`s: no committee handle ever
// crosses it.  Every key that reaches those calls is a committee member --
// Header/Vote/Certificate::verify check the author's and each voter's stake
// first (primary/src/messages.rs:86-100, 155-163, 189-215) -- and the committee
// is static for the life of the process (config/src/lib.rs:140-143).  So the
// library keeps, per context, a registry of keys it has seen: a key that misses
// is verified by the uncached kernel and queued; a background thread builds its
// wide comb of -A on every device entry (the same tables as nt_keyset_create)
// and publishes a new snapshot; later calls find it (host-side index,
// key_table.hpp) and verify it through the key-cache kernel.  The registry
// holds at most `capacity` keys (no eviction: the committee is static), its
// comb width is chosen at the first admission for the whole capacity (the
// width policy of key sets, reserved against the context's HBM budget), and
// keys that do not decode are never admitted (they reject either way).
#include <hip/hip_runtime.h>

#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <thread>

#include "cpu_lane.hpp"
#include "runtime.hpp"

namespace ntrt {

using Key32 = std::array<uint8_t, 32>;

struct KeyReg {
  nt_ctx* ctx = nullptr;
  uint32_t cap = 0;          // most keys the registry admits
  uint32_t admit_after = 1;  // sightings of a missed key before it is queued
  std::mutex mu;             // everything below
  std::condition_variable cv;       // worker: work queued / stop
  std::condition_variable idle_cv;  // nt_key_cache_sync: queue drained
  std::shared_ptr<const RegSnap> snap;  // published (null until the first admission)
  std::shared_ptr<KsTables> t;          // device tables (capacity keys), worker-owned until published
  int bits = 0;
  std::vector<uint8_t> enc;             // admitted keys, in index order
  std::deque<Key32> queue;
  std::set<Key32> pending;              // queued or being built
  std::set<Key32> refused;              // do not decode: never admitted
  std::map<Key32, uint32_t> seen;       // sightings of missed keys (bounded)
  bool stop = false, building = false;
  int error = NT_OK;                    // first failure of an admission (the registry then stops admitting)
  std::vector<hipStream_t> streams;     // one low-priority stream per device entry (admission builds)
  std::atomic<uint64_t> hits{0}, misses{0}, admitted{0}, nrefused{0};
  uint64_t alloc_us = 0, build_us = 0;  // time the worker spent allocating tables / building combs
  std::thread worker;

  ~KeyReg() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    if (worker.joinable()) worker.join();
    for (size_t i = 0; i < streams.size(); ++i)
      if (streams[i]) {
        (void)hipSetDevice(ctx->devs[i]->ordinal);
        (void)hipStreamDestroy(streams[i]);
      }
  }

  // device tables for `cap` keys on every device entry, at the widest key-comb
  // width that fits (the key-set policy, keyset_comb_bits), or a narrower one
  // when hipMalloc refuses it (another process may take the memory between the
  // check and the allocation); worker thread
  int allocate() {
    for (auto& d : ctx->devs) {
      std::lock_guard<std::mutex> lk(d->mu);
      NT_CHK(comb_b_for(*d));  // the comb of B takes its share of the budget first
    }
    int rc = NT_ENOMEM;
    for (const int w : {nt::kKeyCombReduced, nt::kKeyCombWide, nt::kKeyCombMid, nt::kKeyCombNarrow}) {
      const int b = keyset_comb_bits(ctx, cap);
      if (b == 0) return NT_ENOMEM;
      if (w > b) continue;  // wider than what fits
      rc = allocate_at(w);
      if (rc != NT_ENOMEM) return rc;
    }
    return rc;
  }

  int allocate_at(int b) {
    auto T = std::make_shared<KsTables>();
    T->nkeys = cap;
    T->bits = b;
    T->dev.resize(ctx->devs.size());
    for (size_t di = 0; di < ctx->devs.size(); ++di) {
      Device& dv = *ctx->devs[di];
      auto& pd = T->dev[di];
      NT_TRY(hipSetDevice(dv.ordinal));
      pd.ordinal = dv.ordinal;
      const uint64_t comb = nt::wcomb_bytes_per_key(b) * cap;
      if (!dv.budget->reserve(comb)) return NT_ENOMEM;  // T's destructor releases what was reserved
      pd.budget = dv.budget;
      pd.reserved = comb;
      if (hipMalloc(&pd.d_enc, 32ull * cap) != hipSuccess || hipMalloc(&pd.d_meta, 4ull * cap) != hipSuccess ||
          table_malloc((void**)&pd.d_comb, comb) != hipSuccess) {
        (void)hipGetLastError();
        return NT_ENOMEM;
      }
      if (streams.size() < ctx->devs.size()) streams.resize(ctx->devs.size(), nullptr);
      if (!streams[di]) {
        int lo = 0, hi = 0;
        NT_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        NT_TRY(hipStreamCreateWithPriority(&streams[di], hipStreamNonBlocking, lo));
      }
    }
    t = T;
    bits = b;
    return NT_OK;
  }

  // combs of keys[0 .. k) at indices nk .. nk + k on every device entry; worker thread
  int build(const std::vector<Key32>& keys, uint32_t nk) {
    const uint32_t k = (uint32_t)keys.size();
    std::vector<uint8_t> buf(32ull * k);
    for (uint32_t i = 0; i < k; ++i) std::memcpy(buf.data() + 32ull * i, keys[i].data(), 32);
    const size_t words = nt::wcomb_bytes_per_key(bits) / 4;
    for (size_t di = 0; di < ctx->devs.size(); ++di) {
      Device& dv = *ctx->devs[di];
      auto& pd = t->dev[di];
      NT_TRY(hipSetDevice(dv.ordinal));
      NT_CHK(dv.build_wcombs(bits, (const uint32_t*)buf.data(), k, 1, pd.d_comb + words * nk, pd.d_meta + nk,
                             streams[di]));
      NT_TRY(hipMemcpyAsync(pd.d_enc + 8ull * nk, buf.data(), 32ull * k, hipMemcpyHostToDevice, streams[di]));
      NT_TRY(hipStreamSynchronize(streams[di]));
    }
    return NT_OK;
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !queue.empty(); });
      if (stop) return;
      std::vector<Key32> batch(queue.begin(), queue.end());
      queue.clear();
      building = true;
      const uint32_t nk = snap ? snap->table.nkeys : 0;
      lk.unlock();
      // keys that do not decode reject on every path: no comb for them
      std::vector<Key32> ok, bad;
      for (const Key32& key : batch) (nt::cpu::key_decodes(key.data()) ? ok : bad).push_back(key);
      int rc = NT_OK;
      const auto t0 = std::chrono::steady_clock::now();
      if (!ok.empty() && !t) rc = allocate();
      const auto t1 = std::chrono::steady_clock::now();
      if (rc == NT_OK && !ok.empty()) rc = build(ok, nk);
      const auto t2 = std::chrono::steady_clock::now();
      if (std::getenv("NT_REG_TRACE")) {  // diagnosis: where an admission's time goes
        std::fprintf(stderr, "[registry] %zu keys (%zu refused): allocate %.1f ms, build %.1f ms, rc %d\n", ok.size(),
                     bad.size(), std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(t2 - t1).count(), rc);
      }
      lk.lock();
      alloc_us += (uint64_t)std::chrono::duration<double, std::micro>(t1 - t0).count();
      build_us += (uint64_t)std::chrono::duration<double, std::micro>(t2 - t1).count();
      building = false;
      for (const Key32& key : batch) pending.erase(key);
      for (const Key32& key : bad) refused.insert(key);
      nrefused += bad.size();
      if (rc != NT_OK) {
        error = rc;  // stop admitting; calls keep verifying through the uncached kernel
        nrefused += ok.size();
      } else if (!ok.empty()) {
        for (const Key32& key : ok) enc.insert(enc.end(), key.begin(), key.end());
        auto s = std::make_shared<RegSnap>();
        s->table.build(enc.data(), (uint32_t)(enc.size() / 32), admitted.load() + 1);
        s->t = t;
        s->bits = bits;
        snap = s;
        admitted += ok.size();
      }
      idle_cv.notify_all();
    }
  }

  // queue `key` unless it is known, queued, refused or over capacity (caller holds mu)
  void offer(const Key32& key) {
    if (error != NT_OK || pending.count(key) || refused.count(key)) return;
    const uint32_t nk = snap ? snap->table.nkeys : 0;
    if (nk + pending.size() >= cap) return;
    if (snap && snap->table.find(key.data()) != nt::kKeyMiss) return;
    pending.insert(key);
    queue.push_back(key);
    if (!worker.joinable()) worker = std::thread([this] { run(); });
    cv.notify_one();
  }
};

std::shared_ptr<const RegSnap> reg_snapshot(nt_ctx* ctx) {
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (!r) return nullptr;
  std::lock_guard<std::mutex> lk(r->mu);
  return r->snap;
}

void reg_count(nt_ctx* ctx, uint64_t hits, uint64_t misses) {
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (!r) return;
  r->hits += hits;
  r->misses += misses;
}

void reg_note_misses(nt_ctx* ctx, const std::vector<const uint8_t*>& keys) {
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (!r || keys.empty()) return;
  std::set<Key32> distinct;
  for (const uint8_t* p : keys) {
    Key32 k;
    std::memcpy(k.data(), p, 32);
    distinct.insert(k);
    if (distinct.size() >= kRegNoteMax) break;
  }
  std::lock_guard<std::mutex> lk(r->mu);
  if (r->seen.size() > 65536) r->seen.clear();  // bounded: a flood of one-off keys forgets, it never grows
  for (const Key32& k : distinct)
    if (++r->seen[k] >= r->admit_after) {
      r->seen.erase(k);
      r->offer(k);
    }
}

}  // namespace ntrt

using namespace ntrt;

extern "C" {

int nt_set_key_cache(nt_ctx* ctx, uint32_t max_keys, uint32_t admit_after) {
  if (!ctx || max_keys > NT_KEY_CACHE_MAX) return NT_EINVAL;
  ctx->reg.reset();  // joins the previous registry's worker; its tables go with the last snapshot held
  if (max_keys == 0) return NT_OK;
  auto r = std::make_shared<KeyReg>();
  r->ctx = ctx;
  r->cap = max_keys;
  r->admit_after = std::max<uint32_t>(1, admit_after);
  ctx->reg = r;
  return NT_OK;
}

int nt_key_cache_add(nt_ctx* ctx, const uint8_t* pk32, uint32_t n) {
  if (!ctx || (n && !pk32)) return NT_EINVAL;
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (!r) return NT_EINVAL;
  {
    std::lock_guard<std::mutex> lk(r->mu);
    for (uint32_t i = 0; i < n; ++i) {
      std::array<uint8_t, 32> k;
      std::memcpy(k.data(), pk32 + 32ull * i, 32);
      r->offer(k);
    }
  }
  return nt_key_cache_sync(ctx);
}

int nt_key_cache_sync(nt_ctx* ctx) {
  if (!ctx) return NT_EINVAL;
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (!r) return NT_OK;
  std::unique_lock<std::mutex> lk(r->mu);
  r->idle_cv.wait(lk, [&] { return r->queue.empty() && !r->building; });
  return r->error;
}

int nt_key_cache_info(const nt_ctx* ctx, uint64_t* out12) {
  if (!ctx || !out12) return NT_EINVAL;
  uint64_t v[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  std::shared_ptr<KeyReg> r = ctx->reg;
  if (r) {
    std::lock_guard<std::mutex> lk(r->mu);
    v[0] = r->snap ? r->snap->table.nkeys : 0;
    v[1] = r->cap;
    v[2] = (uint64_t)r->bits;
    v[3] = r->bits ? (nt::wcomb_bytes_per_key(r->bits) + 36) * (uint64_t)r->cap : 0;
    v[4] = r->hits.load();
    v[5] = r->misses.load();
    v[6] = r->admitted.load();
    v[7] = r->nrefused.load();
    v[8] = r->pending.size();
    v[9] = (uint64_t)(-(int64_t)r->error);
    v[10] = r->alloc_us;
    v[11] = r->build_us;
  }
  std::memcpy(out12, v, sizeof v);
  return NT_OK;
}

}  // extern "C"
