// ntcrypto.cpp -- host side of the C ABI (include/ntcrypto.h).
//
// Owns one `Device` per GPU (per entry of nt_init_devices: a repeated ordinal
// gets its own): non-blocking HIP streams and grow-only device/pinned staging;
// on the first call that needs them, the wide comb of B (24-bit digits, 11.8 GB,
// shared per device ordinal; 20-bit, 872 MB, under an HBM budget or when the
// device cannot hold the wide one) and the per-lane [k]A table workspace.
// Host entry points shard items over devices by contiguous index ranges (one
// host thread per device), stage through pinned memory, launch, and gather the
// bitmaps / digests.  There is deliberately no CPU compute path: if HIP or the
// gfx950 code object is unavailable the call fails with a negative code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ntcrypto.h"
#include "cpu_lane.hpp"
#include "kernels.hpp"
#include "pipe_plan.hpp"
#include "runtime.hpp"

namespace ntrt {

// NT_TABLE_ALLOC=contig (A/B): comb tables from physically contiguous VRAM
// (hipExtMallocWithFlags + hipDeviceMallocContiguous; hipMalloc when that is
// refused), to see whether the key-cache kernel's random comb lines pay for
// address translation beyond what the driver's own placement gives
hipError_t table_malloc(void** p, size_t bytes) {
  static const bool contig = [] {
    const char* e = std::getenv("NT_TABLE_ALLOC");
    return e && std::strcmp(e, "contig") == 0;
  }();
  if (contig) {
    const hipError_t e = hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
    if (std::getenv("NT_REG_TRACE"))
      std::fprintf(stderr, "[alloc] contiguous %.2f GB: %s\n", bytes / 1e9, e == hipSuccess ? "ok" : "refused");
    if (e == hipSuccess) return e;
    (void)hipGetLastError();
  }
  return hipMalloc(p, bytes);
}

// nt_host_alloc registry (runtime.hpp)
std::mutex g_pin_mu;
std::map<uintptr_t, uint64_t> g_pinned;

bool is_pinned(const void* p, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound((uintptr_t)p);
  if (it == g_pinned.begin()) return false;
  --it;
  return (uintptr_t)p + bytes <= it->first + it->second;
}

// comb of B per (device ordinal, digit width), shared across device entries and contexts
std::mutex g_combb_mu;
std::map<std::pair<int, int>, std::weak_ptr<CombB>> g_combb;

std::shared_ptr<CombB> shared_comb_b(Device& dv, int bits, int& rc) {
  static const uint32_t kB[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                                 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};  // encoding of B
  std::lock_guard<std::mutex> lk(g_combb_mu);
  if (auto c = g_combb[{dv.ordinal, bits}].lock()) return c;
  auto c = std::make_shared<CombB>();
  c->ordinal = dv.ordinal;
  c->bits = bits;
  if (hipSetDevice(dv.ordinal) != hipSuccess) {
    rc = NT_EHIP;
    return nullptr;
  }
  if (table_malloc((void**)&c->p, nt::wcomb_bytes_per_key(bits)) != hipSuccess) {
    (void)hipGetLastError();  // an out-of-memory hipMalloc leaves no sticky error: clear it
    c->p = nullptr;
    rc = NT_ENOMEM;
    return nullptr;
  }
  rc = dv.build_wcombs(bits, kB, 1, 0, c->p, nullptr);
  if (rc != NT_OK) return nullptr;
  g_combb[{dv.ordinal, bits}] = c;
  return c;
}

// NT_BCOMB_BITS=24|20 forces the width of the comb of B (A/B runs, tests)
static int forced_bcomb_bits() {
  const char* e = std::getenv("NT_BCOMB_BITS");
  const int b = e ? std::atoi(e) : 0;
  return b == nt::kBCombBits || b == nt::kBCombFallback ? b : 0;
}

// HBM the device must keep free beside a 24-bit comb of B (two slots' verify
// workspaces + staging); below it the entry takes the 20-bit comb
constexpr uint64_t kCombHeadroom = 4ull << 30;

// The comb of B of execution slot dv: its entry's, created on first use.  The
// entry picks the widest width that (a) fits the context's HBM budget on the
// entry, (b) leaves kCombHeadroom of the device free and (c) hipMalloc grants:
// 24-bit digits (11 additions per [s]B, 11.8 GB), else 20-bit (13, 872 MB).
// The fast path reads only the slot's own comb_ready (the entry's
// fields are written under tables_mu by whichever slot builds the comb first).
int comb_b_for(Device& dv) {
  if (dv.comb_ready.load(std::memory_order_acquire)) return NT_OK;
  Device& e = *dv.entry;
  std::lock_guard<std::mutex> lk(e.tables_mu);
  if (!e.combB) {
    const int forced = forced_bcomb_bits();
    int rc = NT_ENOMEM;
    for (const int w : {nt::kBCombBits, nt::kBCombFallback}) {
      if (forced && w != forced) continue;
      const uint64_t bytes = nt::wcomb_bytes_per_key(w);
      if (!forced && w == nt::kBCombBits) {
        size_t fr = 0, tot = 0;
        if (hipSetDevice(e.ordinal) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) return NT_EHIP;
        // an existing comb of this width on the ordinal costs nothing more
        std::shared_ptr<CombB> have;
        {
          std::lock_guard<std::mutex> g(g_combb_mu);
          auto it = g_combb.find({e.ordinal, w});
          if (it != g_combb.end()) have = it->second.lock();
        }
        if (!have && fr < bytes + kCombHeadroom) continue;
      }
      if (!e.budget->reserve(bytes)) continue;
      auto c = shared_comb_b(e, w, rc);
      if (!c) {
        e.budget->release(bytes);
        if (rc != NT_ENOMEM) return rc;
        continue;
      }
      e.combB = c;
      e.d_combB = c->p;
      e.bbits = w;
      e.comb_reserved = bytes;
      rc = NT_OK;
      break;
    }
    if (rc != NT_OK) return rc;
  }
  dv.combB = e.combB;
  dv.d_combB = e.d_combB;
  dv.bbits = e.bbits;
  dv.comb_ready.store(1, std::memory_order_release);
  return NT_OK;
}

// everything the verify kernel of slot dv reads besides its inputs
int verify_tables(Device& dv) {
  NT_CHK(comb_b_for(dv));
  return dv.ensure_ws();
}

// Comb width of a new key set: the widest of 21 (reduced scalars) / 20 / 18 /
// 16-bit digits (12 / 13 / 15 / 16 additions per [k]A; 1.61 GB / 872 / 252 /
// 67 MB per key) that, on every device entry of the context, fits the
// context's HBM budget beside the comb of B and the tables the entry already
// holds, and leaves 1/8 of the device's HBM free.  With no width passing the
// free-memory test the 16-bit combs are tried anyway (hipMalloc decides); 0 =
// not even those fit the budget.  NT_KEYSET_COMB_BITS=16|18|20|21 forces one.
int keyset_comb_bits(nt_ctx* ctx, uint32_t nkeys) {
  if (const char* e = std::getenv("NT_KEYSET_COMB_BITS")) {
    const int b = std::atoi(e);
    if (b == nt::kKeyCombReduced || b == nt::kKeyCombWide || b == nt::kKeyCombMid || b == nt::kKeyCombNarrow)
      return b;
  }
  const uint64_t nk = std::max<uint32_t>(nkeys, 1);
  for (const int w : {nt::kKeyCombReduced, nt::kKeyCombWide, nt::kKeyCombMid, nt::kKeyCombNarrow}) {
    const uint64_t comb = nt::wcomb_bytes_per_key(w) * nk;
    const uint64_t need = comb + nt::wcomb_fill_tmp_bytes_per_key(w) * nt::wcomb_fill_batch(w);
    bool ok = true;
    for (auto& d : ctx->devs) {
      size_t fr = 0, tot = 0;
      if (!d->budget->fits(comb) || hipSetDevice(d->ordinal) != hipSuccess ||
          hipMemGetInfo(&fr, &tot) != hipSuccess || fr < need + tot / 8) {
        ok = false;
        break;
      }
    }
    if (ok) return w;
  }
  for (auto& d : ctx->devs)
    if (!d->budget->fits(nt::wcomb_bytes_per_key(nt::kKeyCombNarrow) * nk)) return 0;
  return nt::kKeyCombNarrow;
}


}  // namespace ntrt

using namespace ntrt;

static double env_or(const char* name, double dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atof(e) : dflt;
}
static NtSmallModel with_env(NtSmallModel m) {
  m.cpu_verify_us = env_or("NT_SMALL_CPU_VERIFY_US", m.cpu_verify_us);
  m.gpu_verify_us = env_or("NT_SMALL_GPU_VERIFY_US", m.gpu_verify_us);
  m.cpu_sha_mbs = env_or("NT_SMALL_CPU_SHA_MBS", m.cpu_sha_mbs);
  m.gpu_lane_mbs = env_or("NT_SMALL_GPU_LANE_MBS", m.gpu_lane_mbs);
  m.gpu_call_us = env_or("NT_SMALL_GPU_CALL_US", m.gpu_call_us);
  m.pcie_gbs = env_or("NT_SMALL_PCIE_GBS", m.pcie_gbs);
  m.spawn_us = env_or("NT_SMALL_SPAWN_US", m.spawn_us);
  m.gpu_keyset_us = env_or("NT_SMALL_GPU_KEYSET_US", m.gpu_keyset_us);
  return m;
}
static int calibrate_small(nt_ctx* ctx);

extern "C" {

const char* nt_strerror(int code) {
  switch (code) {
    case NT_OK: return "ok";
    case NT_EINVAL: return "invalid argument";
    case NT_EHIP: return "HIP runtime error";
    case NT_ENOMEM: return "out of device or pinned memory";
    case NT_ENODEV: return "no usable gfx950 device (this library has no CPU path)";
    default: return "unknown error";
  }
}

const char* nt_version(void) { return "ntcrypto 0.1 gfx950"; }

static long env_slots() {
  const char* e = std::getenv("NT_SLOTS");
  return e && *e ? std::atol(e) : 2;
}

// NT_HBM_BUDGET: bytes of tables per device entry, with an optional K / M / G suffix (0 / unset = no cap)
static uint64_t env_budget() {
  const char* e = std::getenv("NT_HBM_BUDGET");
  if (!e || !*e) return 0;
  char* end = nullptr;
  const double v = std::strtod(e, &end);
  double mul = 1;
  if (end && (*end == 'k' || *end == 'K')) mul = 1024.0;
  if (end && (*end == 'm' || *end == 'M')) mul = 1024.0 * 1024;
  if (end && (*end == 'g' || *end == 'G')) mul = 1024.0 * 1024 * 1024;
  return v > 0 ? (uint64_t)(v * mul) : 0;
}

static int init_common(nt_ctx** out, const std::vector<int>& ords) {
  if (!out) return NT_EINVAL;
  *out = nullptr;
  auto ctx = std::make_unique<nt_ctx>();
  ctx->small_model = with_env(NtSmallModel{});
  ctx->hbm_budget = env_budget();
  const int slots = std::max(1, std::min(8, (int)env_slots()));
  for (int o : ords) {
    auto d = std::make_unique<Device>();
    int rc = d->init(o, (int)ctx->devs.size());
    if (rc != NT_OK) return rc;
    d->budget->limit = ctx->hbm_budget;
    for (int k = 1; k < slots; ++k) {
      auto x = std::make_unique<Device>();
      rc = x->init(o, (int)ctx->devs.size(), d.get());
      if (rc != NT_OK) return rc;
      d->extra.push_back(std::move(x));
    }
    ctx->devs.push_back(std::move(d));
  }
  if (ctx->devs.empty()) return NT_ENODEV;
  // NT_KEY_CACHE=<max_keys>[:<admit_after>]: the key registry (nt_set_key_cache)
  if (const char* e = std::getenv("NT_KEY_CACHE")) {
    const long k = std::atol(e);
    const char* c = std::strchr(e, ':');
    const long a = c ? std::atol(c + 1) : 1;
    if (k > 0) {
      const int rc = nt_set_key_cache(ctx.get(), (uint32_t)std::min<long>(k, NT_KEY_CACHE_MAX), (uint32_t)std::max(1L, a));
      if (rc != NT_OK) return rc;
    }
  }
  *out = ctx.release();
  return NT_OK;
}

int nt_init(nt_ctx** out, int num_gpus) {
  if (num_gpus < 0) return NT_ENODEV;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NT_ENODEV;
  if (num_gpus == 0 || num_gpus > count) num_gpus = count;
  std::vector<int> ords;
  for (int i = 0; i < num_gpus; ++i) ords.push_back(i);
  return init_common(out, ords);
}

int nt_init_device(nt_ctx** out, int device_ordinal) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NT_ENODEV;
  if (device_ordinal < 0 || device_ordinal >= count) return NT_EINVAL;
  return init_common(out, {device_ordinal});
}

int nt_init_devices(nt_ctx** out, const int* ordinals, int n) {
  int count = 0;
  if (!ordinals || n <= 0) return NT_EINVAL;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NT_ENODEV;
  std::vector<int> ords(ordinals, ordinals + n);
  for (int o : ords)
    if (o < 0 || o >= count) return NT_EINVAL;
  return init_common(out, ords);
}

void nt_free(nt_ctx* ctx) { delete ctx; }

int nt_num_devices(const nt_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int nt_set_hbm_budget(nt_ctx* ctx, uint64_t bytes_per_device) {
  if (!ctx) return NT_EINVAL;
  ctx->hbm_budget = bytes_per_device;
  for (auto& d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->budget->mu);
    d->budget->limit = bytes_per_device;
  }
  return NT_OK;
}

int nt_memory_info(nt_ctx* ctx, int dev, uint64_t* out8) {
  if (!ctx || !out8 || dev < 0 || dev >= (int)ctx->devs.size()) return NT_EINVAL;
  Device& e = *ctx->devs[dev];
  uint64_t ws = 0, stash = 0, staging = 0;
  std::vector<Device*> slots{&e};
  for (auto& x : e.extra) slots.push_back(x.get());
  for (Device* sl : slots) {
    std::lock_guard<std::mutex> lk(sl->mu);
    ws += (sl->d_ws ? nt::ws_bytes_per_slot() * sl->ws_slots : 0) + sl->ws2.cap;
    stash += sl->d[B_STASH].cap + sl->d[B_SORT].cap + sl->stash2.cap + sl->sort2.cap;
    for (int b = 0; b < B_NBUF; ++b)
      if (b != B_STASH && b != B_SORT) staging += sl->d[b].cap;
  }
  uint64_t comb_bits = 0, comb_bytes = 0, reserved = 0;
  {
    std::lock_guard<std::mutex> lk(e.tables_mu);
    if (e.combB) {
      comb_bits = (uint64_t)e.bbits;
      comb_bytes = nt::wcomb_bytes_per_key(e.bbits);
    }
    reserved = e.comb_reserved;
  }
  uint64_t limit = 0, held = 0;
  {
    std::lock_guard<std::mutex> lk(e.budget->mu);
    limit = e.budget->limit;
    held = e.budget->held;
  }
  const uint64_t v[8] = {comb_bits, comb_bytes, held - std::min(held, reserved), ws, stash, staging, limit, held};
  std::memcpy(out8, v, sizeof v);
  return NT_OK;
}

int nt_dev_stream(nt_ctx* ctx, int dev, int which, void** out) {
  if (!ctx || !out || dev < 0 || dev >= (int)ctx->devs.size() || (which != 0 && which != 1)) return NT_EINVAL;
  Device& d = *ctx->devs[dev];
  *out = (void*)(which ? d.stream2 : d.stream);
  return NT_OK;
}

int nt_set_small_call_path(nt_ctx* ctx, int mode, int threads) {
  if (!ctx || mode < NT_SMALL_OFF || mode > NT_SMALL_ALWAYS) return NT_EINVAL;
  if (threads <= 0) threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  threads = std::min(threads, nt::cpu::pool_threads());  // the host lane's real parallelism
  ctx->small_mode = NT_SMALL_OFF;  // calibration runs the GPU paths
  ctx->small_threads = threads;
  if (mode != NT_SMALL_OFF) {
    nt::cpu::init(threads);
    if (!ctx->small_model.calibrated) {
      const int rc = calibrate_small(ctx);
      if (rc != NT_OK) return rc;
    }
  }
  ctx->small_mode = mode;
  return NT_OK;
}

int nt_small_call_model(const nt_ctx* ctx, double* out10) {
  if (!ctx || !out10) return NT_EINVAL;
  const NtSmallModel& m = ctx->small_model;
  const double v[10] = {m.cpu_verify_us, m.gpu_verify_us, m.cpu_sha_mbs, m.gpu_lane_mbs, m.gpu_call_us,
                        m.pcie_gbs,      m.spawn_us,      (double)ctx->small_threads.load(), (double)m.calibrated,
                        m.gpu_keyset_us};
  std::memcpy(out10, v, sizeof v);
  return NT_OK;
}

int nt_call_counts(const nt_ctx* ctx, uint64_t* host_calls, uint64_t* gpu_calls) {
  if (!ctx) return NT_EINVAL;
  if (host_calls) *host_calls = ctx->calls_host.load();
  if (gpu_calls) *gpu_calls = ctx->calls_gpu.load();
  return NT_OK;
}

void* nt_host_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<uint64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[(uintptr_t)p] = std::max<uint64_t>(bytes, 1);
  return p;
}

void nt_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pinned.erase((uintptr_t)p);
  }
  (void)hipHostFree(p);
}

}  // extern "C"

namespace {

// Stage the message span used by items [lo, hi) (rebased offsets, 16-B phase kept).
int stage_messages(Device& dv, const uint8_t* data, const uint64_t* off, const uint64_t* len,
                   uint64_t lo, uint64_t hi, uint64_t* base_out, uint64_t* span_out) {
  uint64_t mn = UINT64_MAX, mx = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    if (len[i] == 0) continue;
    mn = std::min(mn, off[i]);
    mx = std::max(mx, off[i] + len[i]);
  }
  if (mn == UINT64_MAX) mn = mx = 0;
  const uint64_t base = mn & ~(uint64_t)15;
  const uint64_t span = mx - base;
  const uint64_t m = hi - lo;
  NT_CHK(dv.d[B_DATA].ensure(span + 64));
  NT_CHK(dv.d[B_OFF].ensure(m * 8));
  NT_CHK(dv.d[B_LEN].ensure(m * 8));
  NT_CHK(dv.h[B_OFF].ensure(m * 8));
  NT_CHK(dv.h[B_LEN].ensure(m * 8));
  uint64_t* ho = dv.h[B_OFF].as<uint64_t>();
  uint64_t* hl = dv.h[B_LEN].as<uint64_t>();
  for (uint64_t i = lo; i < hi; ++i) {
    ho[i - lo] = len[i] ? off[i] - base : 0;
    hl[i - lo] = len[i];
  }
  if (span) NT_TRY(hipMemcpyAsync(dv.d[B_DATA].p, data + base, span, hipMemcpyHostToDevice, dv.stream));
  NT_TRY(hipMemcpyAsync(dv.d[B_OFF].p, ho, m * 8, hipMemcpyHostToDevice, dv.stream));
  NT_TRY(hipMemcpyAsync(dv.d[B_LEN].p, hl, m * 8, hipMemcpyHostToDevice, dv.stream));
  *base_out = base;
  *span_out = span;
  return NT_OK;
}

void words_to_bitmap(uint8_t* out, const uint64_t* words, uint64_t nbits) {
  const uint64_t nbytes = (nbits + 7) / 8;
  std::memcpy(out, words, nbytes);  // little-endian words == LSB-first bytes
  if (nbits & 7) out[nbytes - 1] &= (uint8_t)((1u << (nbits & 7)) - 1);
}

// ---- chunked staging of the host entry points ----------------------------
// A shard's items are split into up to kMaxChunks contiguous chunks (multiples
// of 64 items, so each chunk owns whole 64-bit verdict words).  Chunk c's inputs
// are copied on the copy stream, and its kernels wait only for those copies:
// the PCIe transfer of chunk c+1 runs under the kernels of chunk c instead of
// before all of them.  NT_PIPE_CHUNKS caps the count (1 = one copy, one launch;
// default kMaxChunks).
using nt::kMaxChunks;

int pipe_chunks_cap() {
  const char* e = std::getenv("NT_PIPE_CHUNKS");
  const int v = e ? std::atoi(e) : kMaxChunks;
  return std::max(1, std::min(kMaxChunks, v));
}

// NT_PIPE_ROUND overrides the round size (tests use it to split small inputs)
uint64_t pipe_round(uint64_t R) {
  const char* e = std::getenv("NT_PIPE_ROUND");
  if (!e) return R;
  const uint64_t v = (uint64_t)std::max(64ll, std::atoll(e));
  return (v + 63) / 64 * 64;
}

// [0, m) -> chunks with the chunk_targets sizes (R a multiple of 64, so every
// boundary is too: each chunk owns whole 64-bit verdict words)
std::vector<uint64_t> chunk_targets(uint64_t total, uint64_t R);
std::vector<std::pair<uint64_t, uint64_t>> plan_chunks(uint64_t m, uint64_t R) {
  std::vector<std::pair<uint64_t, uint64_t>> r;
  uint64_t a = 0;
  for (uint64_t t : chunk_targets(m, R)) {
    r.emplace_back(a, a + t);
    a += t;
  }
  return r;
}

// Message bytes of items [lo, hi): the device buffer mirrors the host span
// [base, base + span) (16-B phase kept); chunk c copies just the bytes its items
// use, unless the items are not laid out in order, in which case chunk 0 copies
// the whole span once.
struct MsgStage {
  uint64_t base = 0, span = 0;
  bool whole = false;
  std::vector<std::pair<uint64_t, uint64_t>> piece;  // per chunk [mn, mx), host-absolute
};

int msg_prepare(Device& dv, const uint64_t* off, const uint64_t* len, uint64_t lo,
                const std::vector<std::pair<uint64_t, uint64_t>>& ch, MsgStage& ms) {
  uint64_t gmn = UINT64_MAX, gmx = 0, sum = 0;
  ms.piece.clear();
  for (const auto& c : ch) {
    uint64_t mn = UINT64_MAX, mx = 0;
    for (uint64_t i = lo + c.first; i < lo + c.second; ++i) {
      if (len[i] == 0) continue;
      mn = std::min(mn, off[i]);
      mx = std::max(mx, off[i] + len[i]);
    }
    if (mn == UINT64_MAX) mn = mx = 0;
    ms.piece.emplace_back(mn, mx);
    sum += mx - mn;
    if (mx > mn) {
      gmn = std::min(gmn, mn);
      gmx = std::max(gmx, mx);
    }
  }
  if (gmn == UINT64_MAX) gmn = gmx = 0;
  ms.base = gmn & ~(uint64_t)15;
  ms.span = gmx - ms.base;
  ms.whole = sum > ms.span + ms.span / 4 + 4096;
  const uint64_t m = ch.back().second;
  NT_CHK(dv.d[B_DATA].ensure(ms.span + 64));
  NT_CHK(dv.d[B_OFF].ensure(std::max<uint64_t>(m, 1) * 16));
  NT_CHK(dv.h[B_OFF].ensure(std::max<uint64_t>(m, 1) * 16));
  return NT_OK;
}

// Device offsets / lengths of chunk [a, b) staged by msg_copy: words [2a, 2b) of
// B_OFF hold the chunk's b - a rebased offsets, then its b - a lengths (one copy)
inline const uint64_t* chunk_off(Device& dv, uint64_t a) { return dv.d[B_OFF].as<uint64_t>() + 2 * a; }
inline const uint64_t* chunk_len(Device& dv, uint64_t a, uint64_t b) {
  return dv.d[B_OFF].as<uint64_t>() + 2 * a + (b - a);
}

// copies (copy stream) of chunk c = items [lo + a, lo + b): rebased offsets,
// lengths, and the chunk's message bytes
int msg_copy(Device& dv, const uint8_t* data, const uint64_t* off, const uint64_t* len, uint64_t lo,
             const MsgStage& ms, size_t c, uint64_t a, uint64_t b) {
  uint64_t* ho = dv.h[B_OFF].as<uint64_t>() + 2 * a;
  uint64_t* hl = ho + (b - a);
  for (uint64_t i = a; i < b; ++i) {
    ho[i - a] = len[lo + i] ? off[lo + i] - ms.base : 0;
    hl[i - a] = len[lo + i];
  }
  const auto& pc = ms.piece[c];
  if (ms.whole) {
    if (c == 0 && ms.span)
      NT_TRY(hipMemcpyAsync(dv.d[B_DATA].p, data + ms.base, ms.span, hipMemcpyHostToDevice, dv.cstream));
  } else if (pc.second > pc.first) {
    NT_TRY(hipMemcpyAsync(dv.d[B_DATA].as<uint8_t>() + (pc.first - ms.base), data + pc.first, pc.second - pc.first,
                          hipMemcpyHostToDevice, dv.cstream));
  }
  if (b > a)
    NT_TRY(hipMemcpyAsync(dv.d[B_OFF].as<uint64_t>() + 2 * a, ho, (b - a) * 16, hipMemcpyHostToDevice, dv.cstream));
  return NT_OK;
}

// every message byte a staged call copies lies in nt_host_alloc memory
bool ms_pinned(const MsgStage& ms, const uint8_t* data) {
  if (ms.span == 0) return true;
  if (ms.whole) return is_pinned(data + ms.base, ms.span);
  for (const auto& pc : ms.piece)
    if (pc.second > pc.first && !is_pinned(data + pc.first, pc.second - pc.first)) return false;
  return true;
}

// The chunk pipeline of a host entry point: copies(c) on the copy stream, then
// kernels(c) on compute stream cstr(c), launched by the host once it has waited
// for chunk c's copies -- a compute stream never holds a wait for the copy
// stream (a cross-queue wait pending at the head of a hardware queue slows the
// dispatches of the other queues: profiles/r05/ab_join.txt).  With every source
// in pinned memory (`async`) hipMemcpyAsync returns at once, and the copies of
// chunk c + 1 are queued before the host waits for chunk c, so the link never
// idles.  From pageable memory HIP stages the copy and returns when it is done
// (NT_PIPE_TRACE, profiles/r05/host_pipe_*.txt): then chunk c's kernels are
// launched before the copies of chunk c + 1 are issued, so they run under them.
// Returns with every kernel launched; finish_chunks() then waits for both
// compute streams on the host.
// NT_PIPE_TRACE=1: host timestamps of every step of run_chunks on stderr (diagnosis)
static bool pipe_trace() {
  static const bool on = [] {
    const char* e = std::getenv("NT_PIPE_TRACE");
    return e && *e == '1';
  }();
  return on;
}
static double pipe_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class Copy, class Launch>
int run_chunks(Device& dv, size_t C, bool async, Copy&& copy, Launch&& launch) {
  if (C == 0) return NT_OK;
  if (C > (size_t)kMaxChunks) return NT_EINVAL;
  const bool tr = pipe_trace();
  const double t0 = tr ? pipe_now_us() : 0.0;
  auto issue = [&](size_t c) -> int {
    NT_CHK(copy(c));
    NT_TRY(hipEventRecord(dv.cev[c], dv.cstream));
    if (tr) std::fprintf(stderr, "[pipe] %9.1f copies %zu issued%s\n", pipe_now_us() - t0, c, async ? "" : " (staged)");
    return NT_OK;
  };
  if (async) NT_CHK(issue(0));
  for (size_t c = 0; c < C; ++c) {
    if (!async) NT_CHK(issue(c));
    else if (c + 1 < C) NT_CHK(issue(c + 1));
    NT_TRY(hipEventSynchronize(dv.cev[c]));
    if (tr) std::fprintf(stderr, "[pipe] %9.1f copies %zu done\n", pipe_now_us() - t0, c);
    NT_CHK(launch(c));
    if (tr) std::fprintf(stderr, "[pipe] %9.1f kernels %zu launched\n", pipe_now_us() - t0, c);
  }
  return NT_OK;
}

// run_chunks for sources that need host staging (a memcpy into the pinned
// buffers before the DMA): a helper thread stages and issues the copies of every
// chunk in order, running ahead of the launches, while this thread waits for each
// chunk's copies and launches its kernels -- the staging of chunk c+1 overlaps
// both chunk c's DMA and its kernels, and no launch waits behind a memcpy.  The
// copy callbacks run on the helper thread only (they must not share mutable
// state with the launch callbacks).
template <class Copy, class Launch>
int run_chunks_staged(Device& dv, size_t C, Copy&& copy, Launch&& launch) {
  if (C <= 1) return run_chunks(dv, C, false, copy, launch);
  if (C > (size_t)kMaxChunks) return NT_EINVAL;
  const bool tr = pipe_trace();
  const double t0 = tr ? pipe_now_us() : 0.0;
  int hip_dev = 0;
  NT_TRY(hipGetDevice(&hip_dev));
  std::mutex mu;
  std::condition_variable cv;
  size_t issued = 0;
  int err = NT_OK;
  std::thread helper([&] {
    int rc = hipSetDevice(hip_dev) == hipSuccess ? NT_OK : NT_EHIP;
    for (size_t c = 0; c < C && rc == NT_OK; ++c) {
      rc = copy(c);
      if (rc == NT_OK && hipEventRecord(dv.cev[c], dv.cstream) != hipSuccess) rc = NT_EHIP;
      if (tr && rc == NT_OK) std::fprintf(stderr, "[pipe] %9.1f copies %zu staged+issued\n", pipe_now_us() - t0, c);
      std::lock_guard<std::mutex> lk(mu);
      if (rc == NT_OK) ++issued;
      else err = rc;
      cv.notify_one();
    }
  });
  int rc = NT_OK;
  for (size_t c = 0; c < C && rc == NT_OK; ++c) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return issued > c || err != NT_OK; });
      if (issued <= c) break;  // the helper failed before issuing chunk c
    }
    if (hipEventSynchronize(dv.cev[c]) != hipSuccess) {
      rc = NT_EHIP;
      break;
    }
    if (tr) std::fprintf(stderr, "[pipe] %9.1f copies %zu done\n", pipe_now_us() - t0, c);
    rc = launch(c);
    if (tr) std::fprintf(stderr, "[pipe] %9.1f kernels %zu launched\n", pipe_now_us() - t0, c);
  }
  helper.join();
  return rc != NT_OK ? rc : err;
}

// both compute streams drained (host-side), so work issued next on dv.stream
// follows every chunk's kernels without a cross-queue wait
int finish_chunks(Device& dv) {
  if (dv.stream2 != dv.stream) NT_TRY(hipStreamSynchronize(dv.stream2));
  return NT_OK;
}

// NT_PIPE_PLAN=round restores round 4's chunk plan (A/B; pipe_plan.hpp)
static bool pipe_plan_round4() {
  static const bool r4 = [] {
    const char* e = std::getenv("NT_PIPE_PLAN");
    return e && std::strcmp(e, "round") == 0;
  }();
  return r4;
}
std::vector<uint64_t> chunk_targets(uint64_t total, uint64_t R) {
  return nt::chunk_targets(total, R, (uint64_t)pipe_chunks_cap(), pipe_plan_round4());
}
std::vector<uint64_t> verify_chunk_targets(uint64_t total, uint64_t R1) {
  return nt::verify_chunk_targets(total, R1, (uint64_t)pipe_chunks_cap());
}
using nt::plan_group_chunks;

Device* dev_of(nt_ctx* ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[dev].get();
}

// ---- small-call path (cpu_lane.hpp) -----------------------------
// Cost model of one host entry-point call (NtSmallModel, runtime.hpp).  A GPU
// call below one round of resident waves costs a fixed floor (launch + copies
// + the two signatures every lane of the verify kernel runs); the digest
// kernel's time is set by its LONGEST message (one lane's serial chain) plus
// the PCIe copy.  nt_set_small_call_path calibrates the fields on the
// context's host threads and device (calibrate_small below); NT_SMALL_*
// environment variables override single fields (A/B runs).
const NtSmallModel& small_model(const nt_ctx* ctx) { return ctx->small_model; }

int small_threads(const nt_ctx* ctx, uint64_t items) {
  const uint64_t t = (uint64_t)std::max(1, ctx->small_threads.load());
  return (int)std::max<uint64_t>(1, std::min(t, items));
}

// host lane iff the call's estimated host time on the context's threads is
// below the GPU floor of the kernel it would run (small_model.hpp)
bool small_verify(nt_ctx* ctx, uint64_t nsig, int kind = nt::kRouteUncached) {
  const int mode = ctx->small_mode.load();
  if (mode == NT_SMALL_ALWAYS) return true;
  if (mode != NT_SMALL_AUTO || !nt::cpu::ready()) return false;
  return nt::small_verify_on_host(small_model(ctx), nsig, small_threads(ctx, nsig), kind);
}

bool small_sha(nt_ctx* ctx, uint64_t n, const uint64_t* len) {
  const int mode = ctx->small_mode.load();
  if (mode == NT_SMALL_ALWAYS) return true;
  if (mode != NT_SMALL_AUTO) return false;
  uint64_t total = 0, mx = 0;
  for (uint64_t i = 0; i < n; ++i) {
    total += len[i];
    mx = std::max(mx, len[i]);
  }
  return nt::small_sha_on_host(small_model(ctx), n, total, mx, small_threads(ctx, n));
}

void bits_from_bytes(uint8_t* bitmap, const std::vector<uint8_t>& v) {
  std::memset(bitmap, 0, (v.size() + 7) / 8);
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i]) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
}

// certificate groups on host threads: per-signature rule, AND per group.
// key(e, A) writes signature e's key encoding to A and returns its mode
// (kStrict / kCofactorless) or -1 for "no such key" (reject).
template <class KeyOf>
int host_groups(nt_ctx* ctx, const uint8_t* sig64, const uint64_t* first, const uint32_t* cnt, const uint8_t* msg32,
                uint64_t G, uint8_t* out_group_bitmap, uint8_t* out_sig_bitmap, KeyOf&& key) {
  std::vector<uint64_t> gbase(G + 1, 0);
  uint64_t nsig_total = 0;
  for (uint64_t g = 0; g < G; ++g) {
    gbase[g + 1] = gbase[g] + cnt[g];
    nsig_total = std::max(nsig_total, first[g] + cnt[g]);
  }
  const uint64_t m = gbase[G];
  std::vector<uint8_t> ok(m, 0);
  nt::cpu::parallel_for(m, small_threads(ctx, m), [&](uint64_t e) {
    const uint64_t g = (uint64_t)(std::upper_bound(gbase.begin(), gbase.end(), e) - gbase.begin()) - 1;
    const uint64_t s = first[g] + (e - gbase[g]);
    uint8_t A[32];
    const int mode = key(s, A);
    ok[e] = mode >= 0 && nt::cpu::verify(mode, A, sig64 + 64 * s, msg32 + 32 * g, 32);
  });
  std::memset(out_group_bitmap, 0, (G + 7) / 8);
  if (out_sig_bitmap) std::memset(out_sig_bitmap, 0, (nsig_total + 7) / 8);
  for (uint64_t g = 0; g < G; ++g) {
    bool all = true;
    for (uint64_t e = gbase[g]; e < gbase[g + 1]; ++e) {
      all = all && ok[e];
      const uint64_t s = first[g] + (e - gbase[g]);
      if (out_sig_bitmap && ok[e]) out_sig_bitmap[s >> 3] |= (uint8_t)(1u << (s & 7));
    }
    if (all) out_group_bitmap[g >> 3] |= (uint8_t)(1u << (g & 7));
  }
  ctx->calls_host++;
  return NT_OK;
}

}  // namespace

extern "C" {

int nt_sha512_trunc32(nt_ctx* ctx, const uint8_t* data, const uint64_t* off, const uint64_t* len,
                      uint64_t n, uint8_t* out32) {
  if (!ctx || (n && (!off || !len || !out32))) return NT_EINVAL;
  if (n == 0) return NT_OK;
  if (small_sha(ctx, n, len)) {
    nt::cpu::parallel_for(n, small_threads(ctx, n), [&](uint64_t i) {
      nt::cpu::sha512_trunc32(data + off[i], len[i], out32 + 32 * i);
    });
    ctx->calls_host++;
    return NT_OK;
  }
  ctx->calls_gpu++;
  return run_sharded(ctx, n, 64, [&](Device& dv, uint64_t lo, uint64_t hi) -> int {
    const uint64_t m = hi - lo;
    // a launch's time is set by its longest message: chunks of >= 64k messages
    const auto ch = plan_chunks(m, pipe_round(1 << 16));
    MsgStage ms;
    NT_CHK(msg_prepare(dv, off, len, lo, ch, ms));
    NT_CHK(dv.d[B_OUT].ensure(m * 32));
    NT_CHK(run_chunks(dv, ch.size(), ms_pinned(ms, data), [&](size_t c) -> int {
      return msg_copy(dv, data, off, len, lo, ms, c, ch[c].first, ch[c].second);
    }, [&](size_t c) -> int {
      const uint64_t a = ch[c].first, b = ch[c].second;
      uint64_t ml = 0;  // the chunk's longest message selects the kernel
      for (uint64_t i = lo + a; i < lo + b; ++i) ml = std::max(ml, len[i]);
      NT_TRY(nt::launch_sha512_trunc32(dv.d[B_DATA].as<uint8_t>(), ms.span, chunk_off(dv, a),
                                       chunk_len(dv, a, b), b - a, dv.d[B_OUT].as<uint8_t>() + 32 * a,
                                       dv.cstr((int)c), ml));
      return NT_OK;
    }));
    NT_CHK(finish_chunks(dv));
    NT_TRY(hipMemcpyAsync(out32 + 32 * lo, dv.d[B_OUT].p, m * 32, hipMemcpyDeviceToHost, dv.stream));
    NT_TRY(hipStreamSynchronize(dv.stream));
    return NT_OK;
  }, sha_latency(n, len));
}

}  // extern "C"

namespace {

// nt_ed25519_verify_strict's GPU body: the uncached verify kernel over the
// shard's chunks (copies of chunk c + 1 under the kernels of chunk c)
int verify_strict_gpu(nt_ctx* ctx, const uint8_t* pk32, const uint8_t* sig64, const uint8_t* msg, const uint64_t* off,
                      const uint64_t* len, uint64_t n, uint8_t* out_bitmap) {
  return run_sharded(ctx, n, 64, [&](Device& dv, uint64_t lo, uint64_t hi) -> int {
    NT_CHK(verify_tables(dv));
    const uint64_t m = hi - lo, words = (m + 63) / 64;
    const uint64_t R1 = pipe_round(nt::verify_round_sigs(dv.cus, 1));
    std::vector<std::pair<uint64_t, uint64_t>> ch;
    {
      uint64_t a = 0;
      for (uint64_t t : verify_chunk_targets(m, R1)) {
        ch.emplace_back(a, a + t);
        a += t;
      }
    }
    MsgStage ms;
    NT_CHK(msg_prepare(dv, off, len, lo, ch, ms));
    NT_CHK(dv.d[B_PK].ensure(m * 32));
    NT_CHK(dv.d[B_SIG].ensure(m * 64));
    NT_CHK(dv.d[B_OUT].ensure(words * 8));
    NT_CHK(dv.h[B_OUT].ensure(words * 8));
    const bool pinned = ms_pinned(ms, msg) && is_pinned(pk32 + 32 * lo, 32 * m) && is_pinned(sig64 + 64 * lo, 64 * m);
    NT_CHK(run_chunks(dv, ch.size(), pinned, [&](size_t c) -> int {
      const uint64_t a = ch[c].first, b = ch[c].second;
      NT_CHK(msg_copy(dv, msg, off, len, lo, ms, c, a, b));
      NT_TRY(hipMemcpyAsync(dv.d[B_PK].as<uint8_t>() + 32 * a, pk32 + 32 * (lo + a), (b - a) * 32,
                            hipMemcpyHostToDevice, dv.cstream));
      NT_TRY(hipMemcpyAsync(dv.d[B_SIG].as<uint8_t>() + 64 * a, sig64 + 64 * (lo + a), (b - a) * 64,
                            hipMemcpyHostToDevice, dv.cstream));
      return NT_OK;
    }, [&](size_t c) -> int {
      const uint64_t a = ch[c].first, b = ch[c].second;
      // chunks of at most one round: one signature per lane (half the launch latency)
      return dv.verify_chunk((int)c, NT_MODE_STRICT, dv.d[B_PK].as<uint8_t>() + 32 * a,
                             dv.d[B_SIG].as<uint8_t>() + 64 * a, dv.d[B_DATA].as<uint8_t>(), ms.span,
                             chunk_off(dv, a), chunk_len(dv, a, b), b - a, dv.d[B_OUT].as<uint64_t>() + a / 64,
                             b - a <= R1 ? 1 : 0);
    }));
    NT_CHK(finish_chunks(dv));
    NT_TRY(hipMemcpyAsync(dv.h[B_OUT].p, dv.d[B_OUT].p, words * 8, hipMemcpyDeviceToHost, dv.stream));
    NT_TRY(hipStreamSynchronize(dv.stream));
    words_to_bitmap(out_bitmap + lo / 8, dv.h[B_OUT].as<uint64_t>(), m);
    return NT_OK;
  }, latency_sized(ctx, (n + ctx->devs.size() - 1) / ctx->devs.size(), nt::verify_round_sigs(ctx->devs[0]->cus)));
}

int verify_keyset_gpu(nt_ctx* ctx, const KeyDev& kd, int mode, const uint32_t* key_idx, const uint8_t* sig64,
                      const uint8_t* msg, const uint64_t* off, const uint64_t* len, uint64_t n, uint8_t* out_bitmap);

// Registry lookups (key_table.hpp) of n consecutive 32-byte keys into kid (nt::kKeyMiss where the index does not hold the key), on up to 16 of
// the host lane's pool threads above 16k keys; returns the misses
uint64_t reg_lookup(const nt::KeyTable& tab, const uint8_t* pk, uint64_t n, uint32_t* kid) {
  const uint64_t T = std::min<uint64_t>(16, 1 + n / 16384);
  std::vector<uint64_t> miss(T, 0);
  auto work = [&](uint64_t t) {
    uint64_t m = 0;
    for (uint64_t i = n * t / T; i < n * (t + 1) / T; ++i) {
      kid[i] = tab.find(pk + 32 * i);
      m += kid[i] == nt::kKeyMiss;
    }
    miss[t] = m;
  };
  if (T == 1) work(0);
  else nt::cpu::parallel_for_fn(T, (int)T, work);
  uint64_t m = 0;
  for (uint64_t x : miss) m += x;
  return m;
}

// up to kRegNoteMax keys of the items that missed (kid null: of every item), for the registry's sightings
std::vector<const uint8_t*> missed_keys(const uint8_t* pk, uint64_t n, const uint32_t* kid) {
  std::vector<const uint8_t*> v;
  for (uint64_t i = 0; i < n && v.size() < 4 * kRegNoteMax; ++i)
    if (!kid || kid[i] == nt::kKeyMiss) v.push_back(pk + 32 * i);
  return v;
}

void bits_set(uint8_t* bm, uint64_t i, bool v) {
  if (v) bm[i >> 3] |= (uint8_t)(1u << (i & 7));
  else bm[i >> 3] &= (uint8_t)~(1u << (i & 7));
}

// verify_strict with the registry's snapshot: every item through the key-cache
// kernel in strict mode (a missed key carries kKeyMiss: unknown, reject), then
// the misses through the uncached kernel, their verdicts merged
int verify_strict_reg(nt_ctx* ctx, const RegSnap& snap, const std::vector<uint32_t>& kid, uint64_t miss,
                      const uint8_t* pk32, const uint8_t* sig64, const uint8_t* msg, const uint64_t* off,
                      const uint64_t* len, uint64_t n, uint8_t* out_bitmap) {
  NT_CHK0(verify_keyset_gpu(ctx, snap.dev(), NT_MODE_STRICT, kid.data(), sig64, msg, off, len, n, out_bitmap));
  if (!miss) return NT_OK;
  std::vector<uint64_t> idx;
  idx.reserve(miss);
  uint64_t bytes = 0, mn = UINT64_MAX, mx = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (kid[i] == nt::kKeyMiss) {
      idx.push_back(i);
      bytes += len[i];
      if (len[i]) {
        mn = std::min(mn, off[i]);
        mx = std::max(mx, off[i] + len[i]);
      }
    }
  const uint64_t M = idx.size();
  std::vector<uint8_t> pk(32 * M), sg(64 * M), bm((M + 7) / 8 + 1);
  std::vector<uint64_t> o(M), l(M);
  // the misses' messages: gathered when they are a small part of the span they
  // lie in (a few scattered misses must not copy the whole buffer), else in place
  const bool gather = mn < mx && bytes < (mx - mn) / 4;
  std::vector<uint8_t> gm(gather ? bytes + 1 : 0);
  uint64_t at = 0;
  for (uint64_t j = 0; j < M; ++j) {
    const uint64_t i = idx[j];
    std::memcpy(pk.data() + 32 * j, pk32 + 32 * i, 32);
    std::memcpy(sg.data() + 64 * j, sig64 + 64 * i, 64);
    l[j] = len[i];
    if (gather) {
      if (len[i]) std::memcpy(gm.data() + at, msg + off[i], len[i]);
      o[j] = at;
      at += len[i];
    } else {
      o[j] = off[i];
    }
  }
  NT_CHK0(verify_strict_gpu(ctx, pk.data(), sg.data(), gather ? gm.data() : msg, o.data(), l.data(), M, bm.data()));
  for (uint64_t j = 0; j < M; ++j) bits_set(out_bitmap, idx[j], (bm[j >> 3] >> (j & 7)) & 1);
  return NT_OK;
}

}  // namespace

extern "C" {

int nt_ed25519_verify_strict(nt_ctx* ctx, const uint8_t* pk32, const uint8_t* sig64,
                             const uint8_t* msg, const uint64_t* off, const uint64_t* len,
                             uint64_t n, uint8_t* out_bitmap) {
  if (!ctx || (n && (!pk32 || !sig64 || !off || !len || !out_bitmap))) return NT_EINVAL;
  if (n == 0) return NT_OK;
  // the key registry (nt_set_key_cache): registered keys through the key cache
  std::shared_ptr<const RegSnap> snap = ctx->reg ? reg_snapshot(ctx) : nullptr;
  std::vector<uint32_t> kid;
  uint64_t miss = n;
  if (snap) {
    kid.resize(n);
    miss = reg_lookup(snap->table, pk32, n, kid.data());
    reg_count(ctx, n - miss, miss);
  }
  if (ctx->reg && miss) reg_note_misses(ctx, missed_keys(pk32, n, snap ? kid.data() : nullptr));
  const bool cached = snap && miss < n;
  if (small_verify(ctx, n, cached && !miss ? nt::kRouteKeyCache : nt::kRouteUncached)) {
    std::vector<uint8_t> ok(n);
    nt::cpu::parallel_for(n, small_threads(ctx, n), [&](uint64_t i) {
      ok[i] = nt::cpu::verify(nt::kStrict, pk32 + 32 * i, sig64 + 64 * i, msg + off[i], len[i]);
    });
    bits_from_bytes(out_bitmap, ok);
    ctx->calls_host++;
    return NT_OK;
  }
  ctx->calls_gpu++;
  if (cached) return verify_strict_reg(ctx, *snap, kid, miss, pk32, sig64, msg, off, len, n, out_bitmap);
  return verify_strict_gpu(ctx, pk32, sig64, msg, off, len, n, out_bitmap);
}

// Stage certificate groups [glo, ghi) contiguously into pinned host buffers:
// per signature its key (kw bytes: 32-byte encoding or 4-byte key index) and
// signature, message offset 32 * (group - glo) and length 32; per group its
// compacted first / cnt.  Copies are split over host threads by signature count
// (a config-3 batch stages ~0.6 GB; one thread would take ~50 ms of it).
// meta = false: hfirst / hcnt already hold the groups' chunk-local starts and counts.
static void stage_groups(uint64_t glo, uint64_t ghi, const uint64_t* first, const uint32_t* cnt, size_t kw,
                         const uint8_t* keys, const uint8_t* sig64, uint8_t* hkey, uint8_t* hsig, uint64_t* hfirst,
                         uint32_t* hcnt, bool copy_keys, bool copy_sigs, bool meta = true) {
  uint64_t e = 0;
  for (uint64_t g = glo; g < ghi; ++g) {
    if (meta) {
      hfirst[g - glo] = e;
      hcnt[g - glo] = cnt[g];
    }
    e += cnt[g];
  }
  const uint64_t m = e;
  if (!copy_keys && !copy_sigs) return;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned T = m < (1u << 16) ? 1u : hw;
  auto work = [&](unsigned t) {
    // groups whose first compacted signature falls in this thread's share
    const uint64_t slo = m * t / T, shi = m * (t + 1) / T;
    uint64_t g = glo + (std::lower_bound(hfirst, hfirst + (ghi - glo), slo) - hfirst);
    for (; g < ghi && hfirst[g - glo] < shi; ++g) {
      const uint64_t e0 = hfirst[g - glo], c = cnt[g];
      if (!c) continue;
      if (copy_keys) std::memcpy(hkey + kw * e0, keys + kw * first[g], kw * c);
      if (copy_sigs) std::memcpy(hsig + 64 * e0, sig64 + 64 * first[g], 64 * c);
    }
  };
  if (T == 1) {
    work(0);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

}  // extern "C"

namespace {

int dev_index(nt_ctx*, const Device& dv) { return dv.group; }

// A signature whose key the registry index does not hold (verify_groups):
// its bit in the shard's verdict words, its group and the group's chunk
struct GroupMiss {
  uint64_t bit;   // 64 W[c] + chunk-local signature index
  uint64_t g;     // caller group index
  uint32_t c;     // chunk
  uint32_t t;     // index within the group
};

// Certificate groups through one of three key forms:
//   kd == nullptr        32-byte encodings, the uncached verify kernel (cofactorless);
//   kd, tab == nullptr   4-byte committee indices into kd's tables (the key-cache kernel);
//   kd and tab           32-byte encodings looked up in the registry index `tab` on
//                        host threads as each chunk is staged, so the chunk carries 4-byte
//                        indices (68 B per vote over PCIe instead of 96); the signatures
//                        whose key misses verify afterwards through the uncached kernel
//                        and their groups' verdicts are recomputed (`missed`: their keys).
// Per shard, groups are staged chunk by chunk into pinned memory (host threads)
// and copied on the copy stream; chunk c's verify and group-AND launches wait
// only for chunk c's copies.
int verify_groups(nt_ctx* ctx, const KeyDev* kd, const nt::KeyTable* tab, const uint8_t* keys, const uint8_t* sig64,
                  const uint64_t* first, const uint32_t* cnt, const uint8_t* msg32, uint64_t G,
                  uint8_t* out_group_bitmap, uint8_t* out_sig_bitmap, std::vector<const uint8_t*>* missed = nullptr,
                  uint64_t* nmissed = nullptr) {
  const size_t kw = kd && !tab ? 4 : 32;  // key bytes per signature in the caller's array
  const size_t kdv = kd ? 4 : 32;         // ... and on the device
  uint64_t nsig_total = 0;
  for (uint64_t g = 0; g < G; ++g) nsig_total = std::max(nsig_total, first[g] + cnt[g]);
  if (nsig_total && (!keys || !sig64)) return NT_EINVAL;
  if (out_sig_bitmap) std::memset(out_sig_bitmap, 0, (nsig_total + 7) / 8);
  std::mutex sig_mu;
  std::atomic<uint64_t> nmiss{0};
  const int rc = run_sharded(ctx, G, 64, [&](Device& dv, uint64_t glo, uint64_t ghi) -> int {
    NT_CHK(kd ? comb_b_for(dv) : verify_tables(dv));
    const uint64_t gm = ghi - glo;
    uint64_t m = 0;
    for (uint64_t g = glo; g < ghi; ++g) m += cnt[g];
    const uint64_t R = pipe_round(kd ? nt::keyset_round_sigs(dv.cus) : nt::verify_round_sigs(dv.cus));
    const auto ch = plan_group_chunks(glo, ghi, cnt, chunk_targets(m, R));
    const size_t C = ch.size();
    // per chunk: first compacted signature, signature count, verdict-word base
    std::vector<uint64_t> E(C + 1, 0), W(C + 1, 0);
    for (size_t c = 0; c < C; ++c) {
      uint64_t mc = 0;
      for (uint64_t g = ch[c].first; g < ch[c].second; ++g) mc += cnt[g];
      E[c + 1] = E[c] + mc;
      W[c + 1] = W[c] + (mc + 63) / 64;
    }
    const uint64_t sw = W[C], gw = (gm + 63) / 64;
    const uint64_t mm = std::max<uint64_t>(m, 1);
    // densely packed keys and signatures are copied straight from the caller's
    // arrays: a DMA from nt_host_alloc memory, or HIP's own staged copy from
    // pageable memory (which returns when it is done: run_chunks' staged order);
    // scattered groups are gathered into the pinned staging on a helper thread.
    // Registry lookups always write their indices into the pinned staging, on the
    // helper thread ahead of the launches (run_chunks_staged).
    bool direct = m > 0;
    for (uint64_t g = glo; direct && g + 1 < ghi; ++g) direct = first[g + 1] == first[g] + cnt[g];
    const bool direct_pinned = direct && (tab || is_pinned(keys + kw * first[glo], kw * m)) &&
                               is_pinned(sig64 + 64 * first[glo], 64 * m);
    if (direct && !direct_pinned && std::getenv("NT_GROUPS_GATHER")) direct = false;  // A/B: round-5 staging
    NT_CHK(dv.h[B_PK].ensure(tab ? mm * 4 : (direct ? 1 : mm * kw)));
    NT_CHK(dv.h[B_SIG].ensure(direct ? 1 : mm * 64));
    NT_CHK(dv.h[B_FIRST].ensure(gm * 8));
    NT_CHK(dv.h[B_CNT].ensure(gm * 4));
    NT_CHK(dv.h[B_OUT].ensure(sw * 8 + 8));
    NT_CHK(dv.h[B_OUT2].ensure(gw * 8));
    NT_CHK(dv.d[B_PK].ensure(mm * kdv));
    NT_CHK(dv.d[B_SIG].ensure(mm * 64));
    NT_CHK(dv.d[B_OFF].ensure(mm * 8));
    NT_CHK(dv.d[B_LEN].ensure(mm * 8));
    NT_CHK(dv.d[B_DATA].ensure(gm * 32 + 64));
    NT_CHK(dv.d[B_FIRST].ensure(gm * 8));
    NT_CHK(dv.d[B_CNT].ensure(gm * 4));
    NT_CHK(dv.d[B_OUT].ensure(sw * 8 + 8));
    NT_CHK(dv.d[B_OUT2].ensure(gw * 8));
    const KsTables::PerDev* pd = nullptr;
    if (kd) {
      uint64_t mc = 0;
      for (size_t c = 0; c < C; ++c) mc = std::max(mc, E[c + 1] - E[c]);
      NT_CHK(dv.ensure_stash(0, mc));
      if (C > 1) NT_CHK(dv.ensure_stash(1, mc));
      pd = &kd->t->dev[dev_index(ctx, dv)];
    }
    uint8_t* hkey = dv.h[B_PK].as<uint8_t>();
    uint8_t* hsig = dv.h[B_SIG].as<uint8_t>();
    uint64_t* hfirst = dv.h[B_FIRST].as<uint64_t>();
    uint32_t* hcnt = dv.h[B_CNT].as<uint32_t>();
    // header digests from pageable memory go through the pinned staging too (32 B
    // per group): a copy from pageable memory returns only when it is done
    const bool msg_direct = is_pinned(msg32 + 32 * glo, 32 * gm);
    NT_CHK(dv.h[B_DATA].ensure(msg_direct ? 1 : gm * 32));
    uint8_t* hmsg = dv.h[B_DATA].as<uint8_t>();
    hipStream_t cs = dv.cstream;
    std::vector<std::vector<GroupMiss>> miss_c(C);  // written by the copy callbacks only
    NT_TRY(hipMemsetAsync(dv.d[B_OUT].p, 0, sw * 8 + 8, cs));  // before chunk 0's copy-done event
    // registry lookups of chunk c's keys into hkey (4-byte indices; kKeyMiss = unknown)
    auto lookup = [&](size_t c) {
      const uint64_t g0 = ch[c].first, g1 = ch[c].second, gl = g0 - glo, e0 = E[c], mc = E[c + 1] - E[c];
      const uint64_t* hf = hfirst + gl;  // chunk-local group starts
      uint32_t* kid = (uint32_t*)hkey + e0;
      const uint64_t T = std::min<uint64_t>(16, 1 + mc / 16384);
      std::vector<std::vector<GroupMiss>> part(T);
      auto work = [&](uint64_t t) {
        const uint64_t lo = mc * t / T, hi = mc * (t + 1) / T;
        uint64_t j = (uint64_t)(std::upper_bound(hf, hf + (g1 - g0), lo) - hf) - 1;
        for (uint64_t e = lo; e < hi; ++e) {
          while (e >= hf[j] + cnt[g0 + j]) ++j;
          const uint64_t g = g0 + j, q = e - hf[j];
          const uint32_t k = tab->find(keys + 32 * (first[g] + q));
          kid[e] = k;
          if (k == nt::kKeyMiss) part[t].push_back(GroupMiss{64 * W[c] + e, g, (uint32_t)c, (uint32_t)q});
        }
      };
      if (T == 1) work(0);
      else nt::cpu::parallel_for_fn(T, (int)T, work);
      for (auto& v : part) miss_c[c].insert(miss_c[c].end(), v.begin(), v.end());
    };
    // Registry lookups run on a thread of their own, chunk by chunk ahead of the
    // copies: a pageable signature copy (HIP stages it and returns when it is
    // done) of chunk c then overlaps the lookups of chunk c + 1.
    struct Ahead {
      std::thread th;
      std::mutex mu;
      std::condition_variable cv;
      size_t ready = 0;
      std::atomic<bool> stop{false};
      ~Ahead() {
        stop = true;
        if (th.joinable()) th.join();
      }
    } ahead;
    if (tab && m) {
      for (size_t c = 0; c < C; ++c) {  // chunk-local group starts (stage_groups leaves them)
        uint64_t e = 0;
        for (uint64_t g = ch[c].first; g < ch[c].second; ++g) {
          hfirst[g - glo] = e;
          hcnt[g - glo] = cnt[g];
          e += cnt[g];
        }
      }
      ahead.th = std::thread([&] {
        for (size_t c = 0; c < C && !ahead.stop; ++c) {
          if (E[c + 1] > E[c]) lookup(c);
          std::lock_guard<std::mutex> lk(ahead.mu);
          ahead.ready = c + 1;
          ahead.cv.notify_all();
        }
      });
    }
    // direct from pinned memory: every copy is a DMA, so chunk c+1's copies are
    // queued before the host waits on chunk c; direct from pageable memory: chunk
    // c's kernels are launched before chunk c+1's (synchronous) copies; gathered
    // or looked up: a helper thread stages (host memcpy of keys and signatures,
    // waits for the chunk's registry lookups) and issues the chunks ahead of the
    // launches (run_chunks_staged)
    auto copy = [&](size_t c) -> int {
      const uint64_t g0 = ch[c].first, g1 = ch[c].second, gl = g0 - glo, e0 = E[c], mc = E[c + 1] - E[c];
      // chunk-local: hfirst relative to e0; message offsets 32 * (g - g0) made on the device
      if (!tab || !direct)
        stage_groups(g0, g1, first, cnt, kw, keys, sig64, hkey + kw * e0, hsig + 64 * e0, hfirst + gl, hcnt + gl,
                     !direct && !tab, !direct, !tab);
      // the signatures first: they do not depend on the registry lookups, so their
      // copy (94 % of a registry chunk's bytes) runs while the chunk's lookups finish
      if (mc) {
        const uint8_t* ss = direct ? sig64 + 64 * (first[glo] + e0) : hsig + 64 * e0;
        NT_TRY(hipMemcpyAsync(dv.d[B_SIG].as<uint8_t>() + 64 * e0, ss, mc * 64, hipMemcpyHostToDevice, cs));
      }
      if (tab && mc) {
        std::unique_lock<std::mutex> lk(ahead.mu);
        ahead.cv.wait(lk, [&] { return ahead.ready > c; });
      }
      if (mc) {
        const uint8_t* sk = tab ? hkey + 4 * e0 : direct ? keys + kw * (first[glo] + e0) : hkey + kw * e0;
        NT_TRY(hipMemcpyAsync(dv.d[B_PK].as<uint8_t>() + kdv * e0, sk, mc * kdv, hipMemcpyHostToDevice, cs));
      }
      const uint8_t* sm = msg32 + 32 * g0;
      if (!msg_direct) {
        std::memcpy(hmsg + 32 * gl, sm, (g1 - g0) * 32);
        sm = hmsg + 32 * gl;
      }
      NT_TRY(hipMemcpyAsync(dv.d[B_DATA].as<uint8_t>() + 32 * gl, sm, (g1 - g0) * 32, hipMemcpyHostToDevice, cs));
      NT_TRY(hipMemcpyAsync(dv.d[B_FIRST].as<uint64_t>() + gl, hfirst + gl, (g1 - g0) * 8, hipMemcpyHostToDevice, cs));
      NT_TRY(hipMemcpyAsync(dv.d[B_CNT].as<uint32_t>() + gl, hcnt + gl, (g1 - g0) * 4, hipMemcpyHostToDevice, cs));
      return NT_OK;
    };
    auto launch = [&](size_t c) -> int {
      const uint64_t g0 = ch[c].first, g1 = ch[c].second, gl = g0 - glo, e0 = E[c], mc = E[c + 1] - E[c];
      hipStream_t s = dv.cstr((int)c);
      const uint8_t* dk = dv.d[B_PK].as<uint8_t>() + kdv * e0;
      const uint8_t* dsig = dv.d[B_SIG].as<uint8_t>() + 64 * e0;
      const uint8_t* dmsg = dv.d[B_DATA].as<uint8_t>() + 32 * gl;
      const uint64_t* doff = dv.d[B_OFF].as<uint64_t>() + e0;
      const uint64_t* dlen = dv.d[B_LEN].as<uint64_t>() + e0;
      uint64_t* dout = dv.d[B_OUT].as<uint64_t>() + W[c];
      if (mc) {
        NT_TRY(nt::launch_group_msgs(dv.d[B_FIRST].as<uint64_t>() + gl, dv.d[B_CNT].as<uint32_t>() + gl, g1 - g0,
                                     (uint64_t*)doff, (uint64_t*)dlen, s));
        if (kd) {
          // the key-cache launch ANDs the chunk's groups itself (its kernel's epilogue)
          void* st = (c & 1) ? dv.stash2.p : dv.d[B_STASH].p;
          void* so = (c & 1) ? dv.sort2.p : dv.d[B_SORT].p;
          NT_CHK(dv.keyset_launch(s, st, [&] {
            return nt::launch_verify_keyset(NT_MODE_COFACTORLESS, kd->bits, (const uint32_t*)dk, dsig, dmsg,
                                            32 * (g1 - g0), doff, dlen, mc, pd->d_meta, pd->d_enc, pd->d_comb,
                                            kd->nkeys, dv.d_combB, dv.bbits, st, so, dout, dv.cus, s,
                                            dv.d[B_FIRST].as<uint64_t>() + gl, dv.d[B_CNT].as<uint32_t>() + gl,
                                            g1 - g0, dv.d[B_OUT2].as<uint64_t>() + gl / 64);
          }));
          return NT_OK;
        }
        NT_CHK(dv.verify_chunk((int)c, NT_MODE_COFACTORLESS, dk, dsig, dmsg, 32 * (g1 - g0), doff, dlen, mc, dout));
      }
      NT_TRY(nt::launch_group_and(dv.d[B_FIRST].as<uint64_t>() + gl, dv.d[B_CNT].as<uint32_t>() + gl, g1 - g0, dout,
                                  dv.d[B_OUT2].as<uint64_t>() + gl / 64, s));
      return NT_OK;
    };
    NT_CHK(!tab && (direct || m == 0) ? run_chunks(dv, C, direct_pinned || m == 0, copy, launch)
                                      : run_chunks_staged(dv, C, copy, launch));
    hipStream_t s = dv.stream;
    NT_CHK(finish_chunks(dv));
    if (ahead.th.joinable()) ahead.th.join();  // every chunk's lookups are done: miss_c is final
    std::vector<GroupMiss> miss;
    for (auto& v : miss_c) miss.insert(miss.end(), v.begin(), v.end());
    NT_TRY(hipMemcpyAsync(dv.h[B_OUT2].p, dv.d[B_OUT2].p, gw * 8, hipMemcpyDeviceToHost, s));
    if ((out_sig_bitmap || !miss.empty()) && m)
      NT_TRY(hipMemcpyAsync(dv.h[B_OUT].p, dv.d[B_OUT].p, sw * 8, hipMemcpyDeviceToHost, s));
    NT_TRY(hipStreamSynchronize(s));
    uint64_t* sbits = dv.h[B_OUT].as<uint64_t>();
    uint64_t* gbits = dv.h[B_OUT2].as<uint64_t>();
    if (!miss.empty()) {
      // the keys the registry does not hold: the uncached kernel over just those
      // signatures (each over its group's digest, already on the device), then
      // their bits set and their groups' verdicts recomputed on the host
      const uint64_t M = miss.size();
      nmiss += M;
      NT_CHK(verify_tables(dv));
      NT_CHK(dv.h[B_PK].ensure(M * 32));
      NT_CHK(dv.h[B_SIG].ensure(M * 64));
      NT_CHK(dv.h[B_OFF].ensure(M * 16));
      NT_CHK(dv.d[B_PK].ensure(M * 32));
      NT_CHK(dv.d[B_SIG].ensure(M * 64));
      NT_CHK(dv.d[B_OFF].ensure(M * 16));
      NT_CHK(dv.d[B_OUT2].ensure(((M + 63) / 64) * 8));
      uint8_t* pk = dv.h[B_PK].as<uint8_t>();
      uint8_t* sg = dv.h[B_SIG].as<uint8_t>();
      uint64_t* ol = dv.h[B_OFF].as<uint64_t>();
      for (uint64_t j = 0; j < M; ++j) {
        const uint64_t o = first[miss[j].g] + miss[j].t;
        std::memcpy(pk + 32 * j, keys + 32 * o, 32);
        std::memcpy(sg + 64 * j, sig64 + 64 * o, 64);
        ol[j] = 32 * (miss[j].g - glo);
        ol[M + j] = 32;
      }
      NT_TRY(hipMemcpyAsync(dv.d[B_PK].p, pk, M * 32, hipMemcpyHostToDevice, s));
      NT_TRY(hipMemcpyAsync(dv.d[B_SIG].p, sg, M * 64, hipMemcpyHostToDevice, s));
      NT_TRY(hipMemcpyAsync(dv.d[B_OFF].p, ol, M * 16, hipMemcpyHostToDevice, s));
      const uint64_t R1 = nt::verify_round_sigs(dv.cus, 1);
      NT_CHK(dv.verify_chunk(0, NT_MODE_COFACTORLESS, dv.d[B_PK].as<uint8_t>(), dv.d[B_SIG].as<uint8_t>(),
                             dv.d[B_DATA].as<uint8_t>(), 32 * gm, dv.d[B_OFF].as<uint64_t>(),
                             dv.d[B_OFF].as<uint64_t>() + M, M, dv.d[B_OUT2].as<uint64_t>(), M <= R1 ? 1 : 0));
      std::vector<uint64_t> mw((M + 63) / 64);
      NT_TRY(hipMemcpyAsync(mw.data(), dv.d[B_OUT2].p, mw.size() * 8, hipMemcpyDeviceToHost, s));
      NT_TRY(hipStreamSynchronize(s));
      std::vector<std::pair<uint64_t, uint32_t>> groups;  // (group, chunk) of every miss
      for (uint64_t j = 0; j < M; ++j) {
        if ((mw[j >> 6] >> (j & 63)) & 1) sbits[miss[j].bit >> 6] |= 1ull << (miss[j].bit & 63);
        groups.emplace_back(miss[j].g, miss[j].c);
      }
      std::sort(groups.begin(), groups.end());
      groups.erase(std::unique(groups.begin(), groups.end()), groups.end());
      for (const auto& gc : groups) {
        const uint64_t g = gc.first, b0 = 64 * W[gc.second] + hfirst[g - glo];
        bool all = true;
        for (uint64_t q = 0; q < cnt[g] && all; ++q) all = (sbits[(b0 + q) >> 6] >> ((b0 + q) & 63)) & 1;
        const uint64_t gl = g - glo;
        if (all) gbits[gl >> 6] |= 1ull << (gl & 63);
        else gbits[gl >> 6] &= ~(1ull << (gl & 63));
      }
      if (missed) {
        std::lock_guard<std::mutex> lk(sig_mu);
        for (uint64_t j = 0; j < M && missed->size() < 4 * kRegNoteMax; ++j)
          missed->push_back(keys + 32 * (first[miss[j].g] + miss[j].t));
      }
    }
    words_to_bitmap(out_group_bitmap + glo / 8, gbits, gm);
    if (out_sig_bitmap && m) {
      std::lock_guard<std::mutex> lk(sig_mu);
      for (size_t c = 0; c < C; ++c) {
        uint64_t e2 = 64 * W[c];
        for (uint64_t g = ch[c].first; g < ch[c].second; ++g)
          for (uint32_t t = 0; t < cnt[g]; ++t, ++e2)
            if ((sbits[e2 >> 6] >> (e2 & 63)) & 1) {
              const uint64_t o = first[g] + t;
              out_sig_bitmap[o >> 3] |= (uint8_t)(1u << (o & 7));
            }
      }
    }
    return NT_OK;
  }, latency_sized(ctx, (nsig_total + ctx->devs.size() - 1) / ctx->devs.size(),
                   kd ? nt::keyset_round_sigs(ctx->devs[0]->cus) : nt::verify_round_sigs(ctx->devs[0]->cus)));
  if (nmissed) *nmissed = nmiss.load();
  return rc;
}

// any key of the groups' signatures the registry index does not hold
bool groups_miss(const nt::KeyTable& tab, const uint8_t* pk32, const uint64_t* first, const uint32_t* cnt,
                 uint64_t G) {
  for (uint64_t g = 0; g < G; ++g)
    for (uint32_t q = 0; q < cnt[g]; ++q)
      if (tab.find(pk32 + 32 * (first[g] + q)) == nt::kKeyMiss) return true;
  return false;
}

}  // namespace

extern "C" {

int nt_ed25519_verify_batch_groups(nt_ctx* ctx, const uint8_t* pk32, const uint8_t* sig64,
                                   const uint64_t* first, const uint32_t* cnt,
                                   const uint8_t* msg32, uint64_t G, uint8_t* out_group_bitmap,
                                   uint8_t* out_sig_bitmap) {
  if (!ctx || (G && (!first || !cnt || !msg32 || !out_group_bitmap))) return NT_EINVAL;
  if (G == 0) return NT_OK;
  uint64_t m = 0, nsig = 0;
  for (uint64_t g = 0; g < G; ++g) {
    m += cnt[g];
    nsig = std::max(nsig, first[g] + cnt[g]);
  }
  if (m && (!pk32 || !sig64)) return NT_EINVAL;
  // the key registry (nt_set_key_cache): route by the kernel the call would run --
  // the key cache when every key hits, the uncached kernel otherwise
  std::shared_ptr<const RegSnap> snap = ctx->reg ? reg_snapshot(ctx) : nullptr;
  bool host = small_verify(ctx, m, snap ? nt::kRouteKeyCache : nt::kRouteUncached);
  if (!host && snap && small_verify(ctx, m, nt::kRouteUncached)) host = groups_miss(snap->table, pk32, first, cnt, G);
  if (host) {
    if (ctx->reg) {  // sightings of the keys the registry does not hold yet
      std::vector<const uint8_t*> ks;
      for (uint64_t g = 0; g < G && ks.size() < 4 * kRegNoteMax; ++g)
        for (uint32_t q = 0; q < cnt[g]; ++q) {
          const uint8_t* p = pk32 + 32 * (first[g] + q);
          if (!snap || snap->table.find(p) == nt::kKeyMiss) ks.push_back(p);
        }
      reg_note_misses(ctx, ks);
    }
    return host_groups(ctx, sig64, first, cnt, msg32, G, out_group_bitmap, out_sig_bitmap,
                       [&](uint64_t s, uint8_t A[32]) {
                         std::memcpy(A, pk32 + 32 * s, 32);
                         return (int)nt::kCofactorless;
                       });
  }
  ctx->calls_gpu++;
  if (snap) {
    std::vector<const uint8_t*> missed;
    uint64_t nmiss = 0;
    const KeyDev kd = snap->dev();
    const int rc = verify_groups(ctx, &kd, &snap->table, pk32, sig64, first, cnt, msg32, G, out_group_bitmap,
                                 out_sig_bitmap, &missed, &nmiss);
    reg_count(ctx, m - std::min(m, nmiss), nmiss);
    if (!missed.empty()) reg_note_misses(ctx, missed);
    return rc;
  }
  if (ctx->reg) {  // an empty registry: the first keys of the call are its first sightings
    std::vector<const uint8_t*> ks;
    for (uint64_t g = 0; g < G && ks.size() < 4 * kRegNoteMax; ++g)
      for (uint32_t q = 0; q < cnt[g] && ks.size() < 4 * kRegNoteMax; ++q) ks.push_back(pk32 + 32 * (first[g] + q));
    reg_note_misses(ctx, ks);
  }
  return verify_groups(ctx, nullptr, nullptr, pk32, sig64, first, cnt, msg32, G, out_group_bitmap, out_sig_bitmap);
}

int nt_ed25519_sign_batch(nt_ctx* ctx, const uint8_t* seed32, const uint8_t* msg,
                          const uint64_t* off, const uint64_t* len, uint64_t n, uint8_t* pk32,
                          uint8_t* sig64) {
  if (!ctx || (n && (!seed32 || !pk32))) return NT_EINVAL;
  if (sig64 && n && (!off || !len)) return NT_EINVAL;
  if (n == 0) return NT_OK;
  return run_sharded(ctx, n, 64, [&](Device& dv, uint64_t lo, uint64_t hi) -> int {
    NT_CHK(comb_b_for(dv));
    const uint64_t m = hi - lo;
    const uint8_t* d_msg = nullptr;
    const uint64_t *d_off = nullptr, *d_len = nullptr;
    uint64_t span = 0;
    if (sig64) {
      uint64_t base;
      NT_CHK(stage_messages(dv, msg, off, len, lo, hi, &base, &span));
      d_msg = dv.d[B_DATA].as<uint8_t>();
      d_off = dv.d[B_OFF].as<uint64_t>();
      d_len = dv.d[B_LEN].as<uint64_t>();
    }
    NT_CHK(dv.d[B_PK].ensure(m * 32));
    NT_CHK(dv.d[B_SIG].ensure(m * 64));
    NT_CHK(dv.d[B_OUT].ensure(m * 32));
    NT_TRY(hipMemcpyAsync(dv.d[B_OUT].p, seed32 + 32 * lo, m * 32, hipMemcpyHostToDevice, dv.stream));
    NT_TRY(nt::launch_sign(dv.d[B_OUT].as<uint8_t>(), d_msg, span, d_off, d_len, m, dv.d_combB, dv.bbits,
                           dv.d[B_PK].as<uint8_t>(), sig64 ? dv.d[B_SIG].as<uint8_t>() : nullptr,
                           dv.sign_blocks, dv.stream));
    NT_TRY(hipMemcpyAsync(pk32 + 32 * lo, dv.d[B_PK].p, m * 32, hipMemcpyDeviceToHost, dv.stream));
    if (sig64)
      NT_TRY(hipMemcpyAsync(sig64 + 64 * lo, dv.d[B_SIG].p, m * 64, hipMemcpyDeviceToHost, dv.stream));
    NT_TRY(hipStreamSynchronize(dv.stream));
    return NT_OK;
  });
}

int nt_ed25519_keypair_batch(nt_ctx* ctx, const uint8_t* seed32, uint64_t n, uint8_t* pk32) {
  return nt_ed25519_sign_batch(ctx, seed32, nullptr, nullptr, nullptr, n, pk32, nullptr);
}

// ---- committee key cache --------------------------------------------------
// Small-call path: key encoding and check mode of one key-cache entry, as
// the key-cache kernel's loader decodes key_idx (k_keyset.inc KsLoader): in
// NT_MODE_MIXED bit 31 selects strict; an index >= nkeys is no key (-1, reject).
static int keyset_key(const nt_keyset* ks, int mode, uint32_t kraw, uint8_t A[32]) {
  int m = mode == NT_MODE_STRICT ? nt::kStrict : nt::kCofactorless;
  if (mode == NT_MODE_MIXED) {
    m = (kraw & NT_KEY_STRICT_BIT) ? nt::kStrict : nt::kCofactorless;
    kraw &= ~NT_KEY_STRICT_BIT;
  }
  if (kraw >= ks->nkeys) return -1;
  std::memcpy(A, ks->enc.data() + 32ull * kraw, 32);
  return m;
}

}  // extern "C"

// nt_keyset_create at a given key-comb width (0 = the widest that fits)
static int keyset_create(nt_ctx* ctx, const uint8_t* pk32, uint32_t nkeys, int bits, nt_keyset** out) {
  if (!ctx || !out || (nkeys && !pk32)) return NT_EINVAL;
  *out = nullptr;
  // verification against the set reads the comb of B: it takes its share of the
  // budget first, the key combs get what is left
  for (auto& d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    NT_CHK(comb_b_for(*d));
  }
  auto ks = std::make_unique<nt_keyset>();
  ks->ctx = ctx;
  ks->nkeys = nkeys;
  ks->bits = bits ? bits : keyset_comb_bits(ctx, nkeys);
  if (ks->bits == 0) return NT_ENOMEM;
  ks->flags.assign(nkeys, 0);
  if (nkeys) ks->enc.assign(pk32, pk32 + 32ull * nkeys);
  ks->t = std::make_shared<KsTables>();
  KsTables& T = *ks->t;
  T.nkeys = nkeys;
  T.bits = ks->bits;
  T.dev.resize(ctx->devs.size());
  for (size_t di = 0; di < ctx->devs.size(); ++di) {
    Device& dv = *ctx->devs[di];
    std::lock_guard<std::mutex> lk(dv.mu);
    NT_TRY(hipSetDevice(dv.ordinal));
    auto& pd = T.dev[di];
    pd.ordinal = dv.ordinal;
    const size_t nk = std::max<uint32_t>(nkeys, 1);
    const uint64_t comb = nt::wcomb_bytes_per_key(ks->bits) * nk;
    if (!dv.budget->reserve(comb)) return NT_ENOMEM;
    pd.budget = dv.budget;
    pd.reserved = comb;
    if (hipMalloc(&pd.d_enc, 32 * nk) != hipSuccess) return NT_ENOMEM;
    if (hipMalloc(&pd.d_meta, 4 * nk) != hipSuccess) return NT_ENOMEM;
    if (table_malloc((void**)&pd.d_comb, comb) != hipSuccess) {
      (void)hipGetLastError();
      pd.d_comb = nullptr;
      return NT_ENOMEM;
    }
    if (nkeys) {
      NT_TRY(hipMemcpyAsync(pd.d_enc, pk32, 32ull * nkeys, hipMemcpyHostToDevice, dv.stream));
      NT_TRY(hipStreamSynchronize(dv.stream));
      const int rc = dv.build_wcombs(ks->bits, (const uint32_t*)pk32, nkeys, 1, pd.d_comb, pd.d_meta);
      if (rc != NT_OK) return rc;
      if (di == 0)
        NT_TRY(hipMemcpyAsync(ks->flags.data(), pd.d_meta, 4ull * nkeys, hipMemcpyDeviceToHost, dv.stream));
    }
    NT_TRY(hipStreamSynchronize(dv.stream));
  }
  *out = ks.release();
  return NT_OK;
}

extern "C" {

int nt_keyset_create(nt_ctx* ctx, const uint8_t* pk32, uint32_t nkeys, nt_keyset** out) {
  // the widest width that fits, or -- when hipMalloc refuses it (another process on the
  // device may take the memory between the check and the allocation) -- the next narrower
  const int b = keyset_comb_bits(ctx, nkeys);
  if (b == 0 || std::getenv("NT_KEYSET_COMB_BITS")) return keyset_create(ctx, pk32, nkeys, b, out);
  int rc = NT_ENOMEM;
  for (const int w : {nt::kKeyCombReduced, nt::kKeyCombWide, nt::kKeyCombMid, nt::kKeyCombNarrow}) {
    if (w > b) continue;
    rc = keyset_create(ctx, pk32, nkeys, w, out);
    if (rc != NT_ENOMEM) return rc;
  }
  return rc;
}

void nt_keyset_free(nt_keyset* ks) { delete ks; }

int nt_keyset_flags(const nt_keyset* ks, uint32_t i, uint32_t* flags) {
  if (!ks || !flags || i >= ks->nkeys) return NT_EINVAL;
  *flags = ks->flags[i];
  return NT_OK;
}


int nt_keyset_info(const nt_keyset* ks, uint32_t* comb_bits, uint64_t* bytes_per_device) {
  if (!ks) return NT_EINVAL;
  const uint64_t nk = std::max<uint32_t>(ks->nkeys, 1);
  if (comb_bits) *comb_bits = (uint32_t)ks->bits;
  if (bytes_per_device) *bytes_per_device = (nt::wcomb_bytes_per_key(ks->bits) + 36) * nk;
  return NT_OK;
}

}  // extern "C"

namespace {
// key-cache verification of n (key index, signature, message) items against kd's tables
int verify_keyset_gpu(nt_ctx* ctx, const KeyDev& kd, int mode, const uint32_t* key_idx, const uint8_t* sig64,
                      const uint8_t* msg, const uint64_t* off, const uint64_t* len, uint64_t n, uint8_t* out_bitmap) {
  return run_sharded(ctx, n, 64, [&](Device& dv, uint64_t lo, uint64_t hi) -> int {
    NT_CHK(comb_b_for(dv));
    const auto& pd = kd.t->dev[dev_index(ctx, dv)];
    const uint64_t m = hi - lo, words = (m + 63) / 64;
    const auto ch = plan_chunks(m, pipe_round(nt::keyset_round_sigs(dv.cus)));
    MsgStage ms;
    NT_CHK(msg_prepare(dv, off, len, lo, ch, ms));
    NT_CHK(dv.d[B_PK].ensure(m * 4));
    NT_CHK(dv.d[B_SIG].ensure(m * 64));
    NT_CHK(dv.d[B_OUT].ensure(words * 8));
    NT_CHK(dv.h[B_OUT].ensure(words * 8));
    uint64_t mc = 0;
    for (const auto& c : ch) mc = std::max(mc, c.second - c.first);
    NT_CHK(dv.ensure_stash(0, mc));
    if (ch.size() > 1) NT_CHK(dv.ensure_stash(1, mc));
    const bool pinned = ms_pinned(ms, msg) && is_pinned(key_idx + lo, 4 * m) && is_pinned(sig64 + 64 * lo, 64 * m);
    NT_CHK(run_chunks(dv, ch.size(), pinned, [&](size_t c) -> int {
      const uint64_t a = ch[c].first, b = ch[c].second;
      NT_CHK(msg_copy(dv, msg, off, len, lo, ms, c, a, b));
      NT_TRY(hipMemcpyAsync(dv.d[B_PK].as<uint32_t>() + a, key_idx + lo + a, (b - a) * 4, hipMemcpyHostToDevice,
                            dv.cstream));
      NT_TRY(hipMemcpyAsync(dv.d[B_SIG].as<uint8_t>() + 64 * a, sig64 + 64 * (lo + a), (b - a) * 64,
                            hipMemcpyHostToDevice, dv.cstream));
      return NT_OK;
    }, [&](size_t c) -> int {
      const uint64_t a = ch[c].first, b = ch[c].second;
      void* st = (c & 1) ? dv.stash2.p : dv.d[B_STASH].p;
      void* so = (c & 1) ? dv.sort2.p : dv.d[B_SORT].p;
      hipStream_t s = dv.cstr((int)c);
      return dv.keyset_launch(s, st, [&] {
        return nt::launch_verify_keyset(mode, kd.bits, dv.d[B_PK].as<uint32_t>() + a,
                                        dv.d[B_SIG].as<uint8_t>() + 64 * a, dv.d[B_DATA].as<uint8_t>(), ms.span,
                                        chunk_off(dv, a), chunk_len(dv, a, b), b - a,
                                        pd.d_meta, pd.d_enc, pd.d_comb, kd.nkeys, dv.d_combB, dv.bbits, st, so,
                                        dv.d[B_OUT].as<uint64_t>() + a / 64, dv.cus, s);
      });
    }));
    NT_CHK(finish_chunks(dv));
    NT_TRY(hipMemcpyAsync(dv.h[B_OUT].p, dv.d[B_OUT].p, words * 8, hipMemcpyDeviceToHost, dv.stream));
    NT_TRY(hipStreamSynchronize(dv.stream));
    words_to_bitmap(out_bitmap + lo / 8, dv.h[B_OUT].as<uint64_t>(), m);
    return NT_OK;
  }, latency_sized(ctx, (n + ctx->devs.size() - 1) / ctx->devs.size(), nt::keyset_round_sigs(ctx->devs[0]->cus)));
}
}  // namespace

extern "C" {

int nt_ed25519_verify_keyset(nt_ctx* ctx, const nt_keyset* ks, int mode, const uint32_t* key_idx,
                             const uint8_t* sig64, const uint8_t* msg, const uint64_t* off,
                             const uint64_t* len, uint64_t n, uint8_t* out_bitmap) {
  if (!ctx || !ks || ks->ctx != ctx || (mode != NT_MODE_STRICT && mode != NT_MODE_COFACTORLESS && mode != NT_MODE_MIXED))
    return NT_EINVAL;
  if (n && (!key_idx || !sig64 || !off || !len || !out_bitmap)) return NT_EINVAL;
  if (n == 0) return NT_OK;
  if (small_verify(ctx, n, nt::kRouteKeyCache)) {
    std::vector<uint8_t> ok(n);
    nt::cpu::parallel_for(n, small_threads(ctx, n), [&](uint64_t i) {
      uint8_t A[32];
      const int m = keyset_key(ks, mode, key_idx[i], A);
      ok[i] = m >= 0 && nt::cpu::verify(m, A, sig64 + 64 * i, msg + off[i], len[i]);
    });
    bits_from_bytes(out_bitmap, ok);
    ctx->calls_host++;
    return NT_OK;
  }
  ctx->calls_gpu++;
  return verify_keyset_gpu(ctx, KeyDev{ks->t.get(), ks->bits, ks->nkeys}, mode, key_idx, sig64, msg, off, len, n,
                           out_bitmap);
}

int nt_ed25519_verify_batch_groups_keyset(nt_ctx* ctx, const nt_keyset* ks, const uint32_t* key_idx,
                                          const uint8_t* sig64, const uint64_t* first,
                                          const uint32_t* cnt, const uint8_t* msg32, uint64_t G,
                                          uint8_t* out_group_bitmap, uint8_t* out_sig_bitmap) {
  if (!ctx || !ks || ks->ctx != ctx) return NT_EINVAL;
  if (G && (!first || !cnt || !msg32 || !out_group_bitmap)) return NT_EINVAL;
  if (G == 0) return NT_OK;
  uint64_t m = 0;
  for (uint64_t g = 0; g < G; ++g) m += cnt[g];
  if (small_verify(ctx, m, nt::kRouteKeyCache)) {
    if (m && (!key_idx || !sig64)) return NT_EINVAL;
    return host_groups(ctx, sig64, first, cnt, msg32, G, out_group_bitmap, out_sig_bitmap,
                       [&](uint64_t s, uint8_t A[32]) { return keyset_key(ks, NT_MODE_COFACTORLESS, key_idx[s], A); });
  }
  ctx->calls_gpu++;
  const KeyDev kd{ks->t.get(), ks->bits, ks->nkeys};
  return verify_groups(ctx, &kd, nullptr, (const uint8_t*)key_idx, sig64, first, cnt, msg32, G, out_group_bitmap,
                       out_sig_bitmap);
}

// ---- device-resident entry points ---------------------------------------
// `stream` is the caller's; NULL is HIP's NULL stream (not the library's), so a
// caller whose inputs come from work on the NULL stream is ordered after it.
int nt_dev_sha512_trunc32(nt_ctx* ctx, int dev, void* stream, const uint8_t* d_data, uint64_t data_bytes,
                          const uint64_t* d_off, const uint64_t* d_len, uint64_t n, uint32_t* d_bad,
                          uint8_t* d_out32) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || (n && (!d_data || !d_off || !d_len || !d_out32))) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  NT_TRY(nt::launch_sha512_trunc32(d_data, data_bytes, d_off, d_len, n, d_out32, (hipStream_t)stream, ~0ull, d_bad));
  return NT_OK;
}

int nt_dev_sha512_trunc32_bounded(nt_ctx* ctx, int dev, void* stream, const uint8_t* d_data, uint64_t data_bytes,
                                  const uint64_t* d_off, const uint64_t* d_len, uint64_t n, uint64_t max_len,
                                  uint32_t* d_bad, uint8_t* d_out32) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || (n && (!d_data || !d_off || !d_len || !d_out32))) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  NT_TRY(nt::launch_sha512_trunc32(d_data, data_bytes, d_off, d_len, n, d_out32, (hipStream_t)stream, max_len, d_bad));
  return NT_OK;
}

int nt_dev_ed25519_verify(nt_ctx* ctx, int dev, void* stream, int mode, const uint8_t* d_pk32,
                          const uint8_t* d_sig64, const uint8_t* d_msg, uint64_t msg_bytes, const uint64_t* d_off,
                          const uint64_t* d_len, uint64_t n, uint64_t* d_out_words) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || (mode != NT_MODE_STRICT && mode != NT_MODE_COFACTORLESS)) return NT_EINVAL;
  if (n && (!d_pk32 || !d_sig64 || !d_msg || !d_off || !d_len || !d_out_words)) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  // the [k]A workspaces are per device: launches that use one are ordered by its event
  std::lock_guard<std::mutex> lk(dv->mu);
  NT_CHK(verify_tables(*dv));
  NT_TRY(dv->verify_dev(mode, d_pk32, d_sig64, d_msg, msg_bytes, d_off, d_len, n, d_out_words, (hipStream_t)stream));
  return NT_OK;
}

int nt_dev_group_and(nt_ctx* ctx, int dev, void* stream, const uint64_t* d_first,
                     const uint32_t* d_cnt, uint64_t G, const uint64_t* d_sig_words,
                     uint64_t* d_group_words) {
  Device* dv = dev_of(ctx, dev);
  if (!dv) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  NT_TRY(nt::launch_group_and(d_first, d_cnt, G, d_sig_words, d_group_words, (hipStream_t)stream));
  return NT_OK;
}

int nt_dev_ed25519_verify_keyset(nt_ctx* ctx, const nt_keyset* ks, int dev, void* stream, int mode,
                                 const uint32_t* d_key_idx, const uint8_t* d_sig64, const uint8_t* d_msg,
                                 uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                                 uint64_t* d_out_words) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || !ks || ks->ctx != ctx || (mode != NT_MODE_STRICT && mode != NT_MODE_COFACTORLESS && mode != NT_MODE_MIXED))
    return NT_EINVAL;
  if (n && (!d_key_idx || !d_sig64 || !d_msg || !d_off || !d_len || !d_out_words)) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  hipStream_t s = (hipStream_t)stream;
  const auto& pd = ks->t->dev[dev];
  // the device's two stashes, shared with the host entry points, each ordered
  // against every other user by its event whatever the streams; successive
  // device-API calls alternate between them (like nt_dev_ed25519_verify's
  // workspaces), so batches on two streams can overlap
  std::lock_guard<std::mutex> lk(dv->mu);
  NT_CHK(comb_b_for(*dv));
  const int k = (int)(dv->ks_calls++ & 1u);
  NT_CHK(dv->ensure_stash(k, n));
  void* stash = k ? dv->stash2.p : dv->d[B_STASH].p;
  void* so = k ? dv->sort2.p : dv->d[B_SORT].p;
  return dv->keyset_launch(s, stash, [&] {
    return nt::launch_verify_keyset(mode, ks->bits, d_key_idx, d_sig64, d_msg, msg_bytes, d_off, d_len, n, pd.d_meta,
                                    pd.d_enc, pd.d_comb, ks->nkeys, dv->d_combB, dv->bbits, stash, so, d_out_words,
                                    dv->cus, s);
  });
}

int nt_dev_clock_probe(nt_ctx* ctx, int dev, void* stream, uint32_t iters, uint64_t* d_out2, uint64_t* wall_khz) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || !d_out2 || iters == 0) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  if (wall_khz) {
    int khz = 0;
    NT_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dv->ordinal));
    *wall_khz = (uint64_t)khz;
  }
  NT_TRY(nt::launch_clock_probe(iters, dv->cus, d_out2, (hipStream_t)stream));
  return NT_OK;
}

int nt_dev_ed25519_verify_keyset_groups(nt_ctx* ctx, const nt_keyset* ks, int dev, void* stream, int mode,
                                        const uint32_t* d_key_idx, const uint8_t* d_sig64, const uint8_t* d_msg,
                                        uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                                        const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G,
                                        uint64_t* d_out_words, uint64_t* d_group_words) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || !ks || ks->ctx != ctx || (mode != NT_MODE_STRICT && mode != NT_MODE_COFACTORLESS && mode != NT_MODE_MIXED))
    return NT_EINVAL;
  if (n && (!d_key_idx || !d_sig64 || !d_msg || !d_off || !d_len || !d_out_words)) return NT_EINVAL;
  if (G && (!d_first || !d_cnt || !d_group_words)) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return G ? (nt::launch_group_and(d_first, d_cnt, G, d_out_words, d_group_words, s) == hipSuccess
                              ? NT_OK : NT_EHIP)
                       : NT_OK;
  const auto& pd = ks->t->dev[dev];
  std::lock_guard<std::mutex> lk(dv->mu);
  NT_CHK(comb_b_for(*dv));
  const int k = (int)(dv->ks_calls++ & 1u);
  NT_CHK(dv->ensure_stash(k, n));
  void* stash = k ? dv->stash2.p : dv->d[B_STASH].p;
  void* so = k ? dv->sort2.p : dv->d[B_SORT].p;
  return dv->keyset_launch(s, stash, [&] {
    return nt::launch_verify_keyset(mode, ks->bits, d_key_idx, d_sig64, d_msg, msg_bytes, d_off, d_len, n, pd.d_meta,
                                    pd.d_enc, pd.d_comb, ks->nkeys, dv->d_combB, dv->bbits, stash, so, d_out_words,
                                    dv->cus, s, d_first, d_cnt, G, d_group_words);
  });
}

int nt_dev_ed25519_sign(nt_ctx* ctx, int dev, void* stream, const uint8_t* d_seed32, const uint8_t* d_msg,
                        uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                        uint8_t* d_pk32, uint8_t* d_sig64) {
  Device* dv = dev_of(ctx, dev);
  if (!dv || (n && (!d_seed32 || !d_pk32))) return NT_EINVAL;
  if (n && d_sig64 && (!d_msg || !d_off || !d_len)) return NT_EINVAL;
  NT_TRY(hipSetDevice(dv->ordinal));
  std::lock_guard<std::mutex> lk(dv->mu);
  NT_CHK(comb_b_for(*dv));
  NT_TRY(nt::launch_sign(d_seed32, d_sig64 ? d_msg : nullptr, msg_bytes, d_off, d_len, n, dv->d_combB, dv->bbits,
                         d_pk32, d_sig64, dv->sign_blocks, (hipStream_t)stream));
  return NT_OK;
}

}  // extern "C"

// ---- calibration of the small-call cost model (nt_set_small_call_path) ------
// Host lane: verify_strict of the RFC 8032 section 7.1 TEST 1 vector (a valid
// signature over the empty message) and SHA-512 of 1 MiB, on the calling
// thread; the pool wake-up from a no-op call on `threads` threads.  GPU: one
// signature through nt_ed25519_verify_strict (below one round: the launch +
// copy floor), a 64-byte digest (the digest call floor) and a 1 MiB digest
// (one lane's serial chain), medians of a few calls after a warm-up.
// NT_SMALL_* variables override single fields afterwards.
static double median_of(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static int calibrate_small(nt_ctx* ctx) {
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); };
  static const uint8_t kPk[32] = {0xd7, 0x5a, 0x98, 0x01, 0x82, 0xb1, 0x0a, 0xb7, 0xd5, 0x4b, 0xfe,
                                  0xd3, 0xc9, 0x64, 0x07, 0x3a, 0x0e, 0xe1, 0x72, 0xf3, 0xda, 0xa6,
                                  0x23, 0x25, 0xaf, 0x02, 0x1a, 0x68, 0xf7, 0x07, 0x51, 0x1a};
  static const uint8_t kSig[64] = {0xe5, 0x56, 0x43, 0x00, 0xc3, 0x60, 0xac, 0x72, 0x90, 0x86, 0xe2, 0xcc, 0x80,
                                   0x6e, 0x82, 0x8a, 0x84, 0x87, 0x7f, 0x1e, 0xb8, 0xe5, 0xd9, 0x74, 0xd8, 0x73,
                                   0xe0, 0x65, 0x22, 0x49, 0x01, 0x55, 0x5f, 0xb8, 0x82, 0x15, 0x90, 0xa3, 0x3b,
                                   0xac, 0xc6, 0x1e, 0x39, 0x70, 0x1c, 0xf9, 0xb4, 0x6b, 0xd2, 0x5b, 0xf5, 0xf0,
                                   0x59, 0x5b, 0xbe, 0x24, 0x65, 0x51, 0x41, 0x43, 0x8e, 0x7a, 0x10, 0x0b};
  static const uint8_t kEmpty[1] = {0};
  NtSmallModel m;
  // host lane, one thread
  bool ok = nt::cpu::verify(nt::kStrict, kPk, kSig, kEmpty, 0);
  {
    std::vector<double> t;
    for (int r = 0; r < 5; ++r) {
      const auto a = clk::now();
      for (int k = 0; k < 8; ++k) ok &= nt::cpu::verify(nt::kStrict, kPk, kSig, kEmpty, 0);
      t.push_back(us(a) / 8);
    }
    if (!ok) return NT_EHIP;  // the host lane must accept a known-good signature
    m.cpu_verify_us = median_of(t);
  }
  std::vector<uint8_t> big(1u << 20, 0x5a);
  {
    uint8_t d[32];
    std::vector<double> t;
    for (int r = 0; r < 3; ++r) {
      const auto a = clk::now();
      nt::cpu::sha512_trunc32(big.data(), big.size(), d);
      t.push_back(us(a));
    }
    m.cpu_sha_mbs = (double)big.size() / median_of(t);  // bytes per us = MB/s
  }
  {
    const int T = std::max(1, ctx->small_threads.load());
    std::vector<double> t;
    for (int r = 0; r < 7; ++r) {
      const auto a = clk::now();
      nt::cpu::parallel_for((uint64_t)T, T, [](uint64_t) {});
      t.push_back(us(a));
    }
    m.spawn_us = T > 1 ? median_of(t) : 0.0;
  }
  // GPU floors (the caller set small_mode = OFF: these calls run the kernels)
  {
    const uint64_t off = 0, len = 0;
    uint8_t bm = 0;
    std::vector<double> t;
    for (int r = 0; r < 6; ++r) {
      const auto a = clk::now();
      NT_CHK0(nt_ed25519_verify_strict(ctx, kPk, kSig, kEmpty, &off, &len, 1, &bm));
      if (r) t.push_back(us(a));
    }
    if (!(bm & 1)) return NT_EHIP;
    m.gpu_verify_us = median_of(t);
  }
  {
    // the key-cache kernel's floor: one signature through a one-key set (16-bit
    // key combs, 67 MB, freed after; the floor is the launch and one lane's
    // serial chain -- 27 comb additions and an inversion -- whatever the width)
    nt_keyset* ks = nullptr;
    NT_CHK0(keyset_create(ctx, kPk, 1, nt::kKeyCombNarrow, &ks));
    const uint64_t off = 0, len = 0;
    const uint32_t k0 = 0;
    uint8_t bm = 0;
    std::vector<double> t;
    int rc = NT_OK;
    for (int r = 0; r < 6 && rc == NT_OK; ++r) {
      const auto a = clk::now();
      rc = nt_ed25519_verify_keyset(ctx, ks, NT_MODE_STRICT, &k0, kSig, kEmpty, &off, &len, 1, &bm);
      if (r) t.push_back(us(a));
    }
    nt_keyset_free(ks);
    if (rc != NT_OK) return rc;
    if (!(bm & 1)) return NT_EHIP;
    m.gpu_keyset_us = median_of(t);
  }
  {
    uint8_t d[32];
    const uint64_t off = 0, len64 = 64, len1m = big.size();
    std::vector<double> ts, tb;
    for (int r = 0; r < 6; ++r) {
      auto a = clk::now();
      NT_CHK0(nt_sha512_trunc32(ctx, big.data(), &off, &len64, 1, d));
      if (r) ts.push_back(us(a));
    }
    for (int r = 0; r < 3; ++r) {
      auto a = clk::now();
      NT_CHK0(nt_sha512_trunc32(ctx, big.data(), &off, &len1m, 1, d));
      if (r) tb.push_back(us(a));
    }
    m.gpu_call_us = median_of(ts);
    const double lane = median_of(tb) - m.gpu_call_us - (double)big.size() / (m.pcie_gbs * 1e3);
    m.gpu_lane_mbs = (double)big.size() / std::max(lane, 1.0);
  }
  m.calibrated = 1;
  ctx->small_model = with_env(m);
  return NT_OK;
}
