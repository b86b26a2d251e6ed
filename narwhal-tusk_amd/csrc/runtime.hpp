// runtime.hpp -- the host runtime's internal types, shared by the C-ABI
// translation units (ntcrypto.cpp: hashing / verification / key cache;
// ingest_gpu.cpp: wire ingestion on the device).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ntcrypto.h"
#include "kernels.hpp"
#include "key_table.hpp"
#include "small_model.hpp"

struct nt_ctx;
namespace ntrt {
struct KeyReg;


#define NT_TRY(expr)                       \
  do {                                     \
    hipError_t _e = (expr);                \
    if (_e != hipSuccess) return NT_EHIP;  \
  } while (0)

#define NT_CHK0(expr)             \
  do {                            \
    int _rc = (expr);             \
    if (_rc != NT_OK) return _rc; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return NT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    want = (want + 4095) & ~(size_t)4095;
    if (hipMalloc(&p, want) != hipSuccess) return NT_ENOMEM;
    cap = want;
    return NT_OK;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return NT_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    want = (want + 4095) & ~(size_t)4095;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return NT_ENOMEM;
    cap = want;
    return NT_OK;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

// nt_host_alloc registry: [base, base + bytes) of every live pinned buffer (ntcrypto.cpp)
extern std::mutex g_pin_mu;
extern std::map<uintptr_t, uint64_t> g_pinned;
bool is_pinned(const void* p, uint64_t bytes);

enum { B_DATA, B_OFF, B_LEN, B_PK, B_SIG, B_OUT, B_OUT2, B_FIRST, B_CNT, B_STASH, B_SORT, B_NBUF };

// The wide comb of B of one digit width on one device ordinal, shared by every
// device entry of every context of the process that runs on that ordinal at
// that width (11.8 GB at 24-bit digits, 872 MB at 20: round 2 paid it per entry
// -- repeated ordinals, a second Backend, the contention probe's contexts;
// ADVICE r02).  Built by the first verify / sign call that needs it (never at
// nt_init: a digest-only worker pays nothing), freed with the last user
// (ntcrypto.cpp: shared_comb_b, comb_b_for).
struct CombB {
  int ordinal = -1;
  int bits = 0;
  uint32_t* p = nullptr;
  ~CombB() {
    if (!p) return;
    (void)hipSetDevice(ordinal);
    (void)hipFree(p);
  }
};
struct Device;
std::shared_ptr<CombB> shared_comb_b(Device& dv, int bits, int& rc);
// the comb of B of a slot (created by its entry on first use; ntcrypto.cpp)
int comb_b_for(Device& dv);

// The context's HBM budget on one device entry (shared by its execution slots
// and by the key sets built on it): the TABLES whose width degrades to fit --
// the comb of B (24 -> 20 bits) and the committee key combs (20 -> 18 -> 16) --
// are reserved against `limit` (NT_HBM_BUDGET / nt_set_hbm_budget; 0 = no cap,
// only the device's free memory decides).  Workspaces, stashes and staging are
// per-call and not budgeted (nt_memory_info reports them).
struct Budget {
  std::mutex mu;
  uint64_t limit = 0;
  uint64_t held = 0;
  bool reserve(uint64_t b) {
    std::lock_guard<std::mutex> lk(mu);
    if (limit && held + b > limit) return false;
    held += b;
    return true;
  }
  void release(uint64_t b) {
    std::lock_guard<std::mutex> lk(mu);
    held -= std::min(held, b);
  }
  bool fits(uint64_t b) {
    std::lock_guard<std::mutex> lk(mu);
    return !limit || held + b <= limit;
  }
};

// The device entry's two compute streams.  Default: plain non-blocking
// streams (ordered against no other stream, the NULL stream included -- ADVICE
// r04: a CU-masked stream is a BLOCKING stream, so every launch on it waited
// for, and held up, work on the NULL stream of the whole process).  HIP
// multiplexes a process's streams over GPU_MAX_HW_QUEUES (4) queues per
// priority and hands a new stream the least-used one, so the two may share a
// hardware queue with other streams of the process; NT_STREAMS=mask gives each
// one a queue of its own (a CU mask enabling every CU: a masked stream never
// shares its queue) at the price of NULL-stream ordering, NT_STREAMS=prio puts
// the second at the highest priority.  Measured (profiles/r04/ab_streams.txt,
// profiles/r05/): the kinds give the same rates when the pipelined steps run on
// the library's streams.
inline hipError_t compute_stream(hipStream_t* s, uint32_t cus, int which) {
  static const int kind = [] {
    const char* e = std::getenv("NT_STREAMS");
    if (!e) return 1;
    return std::strcmp(e, "mask") == 0 ? 0 : std::strcmp(e, "prio") == 0 ? 2 : 1;
  }();
  if (kind == 1 || (kind == 2 && which == 0)) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  if (kind == 2) {
    int lo = 0, hi = 0;
    const hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    return e != hipSuccess ? e : hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
  }
  std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

struct Device {
  int ordinal = -1;
  int group = -1;               // index of this device entry in nt_ctx::devs (keyset tables)
  Device* entry = this;         // the device entry this execution slot belongs to
  std::shared_ptr<Budget> budget;  // the entry's (shared with its slots)
  std::mutex tables_mu;         // (entry) lazy creation of the comb of B
  std::shared_ptr<CombB> combB;  // holds d_combB (shared per ordinal and width, see CombB); null until first needed
  uint64_t comb_reserved = 0;   // (entry) bytes of the comb of B reserved in the budget
  hipStream_t stream = nullptr;
  uint32_t* d_combB = nullptr;  // wide comb of B (verify, key-cache verify, sign): comb_b_for() sets it
  int bbits = 0;                // its digit width (nt::kBCombBits or nt::kBCombFallback)
  std::atomic<int> comb_ready{0};  // this slot's d_combB / bbits are set (comb_b_for's lock-free fast path)
  void* d_ws = nullptr;         // verify workspace: ensure_ws() on the first verify
  uint32_t ws_slots = 0;
  uint32_t sign_blocks = 0;
  uint32_t cus = 0;
  hipEvent_t ws_done = nullptr;  // orders every kernel that uses d_ws, whatever its stream
  hipEvent_t stash_done = nullptr;  // same for the key-cache stash d[B_STASH] (host and device API)
  // host entry points: chunk c's H2D copies go on cstream, cev[c] marks them
  // done, and the host launches chunk c's kernels once it has waited for cev[c]
  // (ntcrypto.cpp run_chunks), so copies of chunk c+1 overlap kernels of chunk c
  hipStream_t cstream = nullptr;
  hipEvent_t cev[16] = {};
  // ... and chunks alternate between two compute streams, so the waves of chunk
  // c+1 fill the CUs that chunk c's last waves leave idle.  Stream 2 has its own
  // verify workspace and key-cache stash.
  hipStream_t stream2 = nullptr;
  hipEvent_t ws2_done = nullptr, stash2_done = nullptr;
  DevBuf ws2, stash2, sort2;
  std::mutex mu;
  uint64_t dev_calls = 0;  // device-API verify calls (workspace alternation), under mu
  uint64_t ks_calls = 0;   // device-API key-cache calls (stash alternation), under mu
  DevBuf d[B_NBUF];
  HostBuf h[B_NBUF];
  // Extra execution slots of the same device entry (NT_SLOTS, default 2 in
  // all): each has its own streams, workspace and staging and shares the comb
  // of B, so a long call (a batch of digests) on one slot does not block a
  // concurrent call (a certificate batch) on the device -- both run on the GPU
  // at once.  Host entry points take the first free slot (SURVEY §8(b):
  // "per-call stream acquisition from a pool").
  std::vector<std::unique_ptr<Device>> extra;
  // state of the wire-ingestion entry point on this slot (ingest_gpu.cpp), created on first use
  std::shared_ptr<void> ingest;

  ~Device() {
    if (comb_reserved && budget) budget->release(comb_reserved);
    if (ordinal < 0) return;
    (void)hipSetDevice(ordinal);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& b : d)
      if (b.p) (void)hipFree(b.p);
    for (auto& b : h)
      if (b.p) (void)hipHostFree(b.p);
    extra.clear();  // before this entry's comb, which the extra slots borrow
    (void)hipSetDevice(ordinal);
    if (d_ws) (void)hipFree(d_ws);
    if (ws_done) (void)hipEventDestroy(ws_done);
    if (stash_done) (void)hipEventDestroy(stash_done);
    for (auto& e : cev)
      if (e) (void)hipEventDestroy(e);
    if (stream2 && stream2 != stream) (void)hipStreamSynchronize(stream2);
    if (ws2.p) (void)hipFree(ws2.p);
    if (stash2.p) (void)hipFree(stash2.p);
    if (sort2.p) (void)hipFree(sort2.p);
    if (ws2_done) (void)hipEventDestroy(ws2_done);
    if (stash2_done) (void)hipEventDestroy(stash2_done);
    if (stream2 && stream2 != stream) (void)hipStreamDestroy(stream2);
    if (cstream && cstream != stream) (void)hipStreamDestroy(cstream);
    if (stream) (void)hipStreamDestroy(stream);
  }

  int init(int ord, int grp, Device* share = nullptr) {
    ordinal = ord;
    group = grp;
    entry = share ? share : this;
    budget = share ? share->budget : std::make_shared<Budget>();
    NT_TRY(hipSetDevice(ord));
    hipDeviceProp_t prop;
    NT_TRY(hipGetDeviceProperties(&prop, ord));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NT_ENODEV;
    if (share) {
      // an extra (latency) slot: ONE stream at the highest priority for its
      // copies and kernels, so it does not share a hardware queue with the
      // bulk streams of the entry's first slot (HIP multiplexes a process's
      // streams over GPU_MAX_HW_QUEUES = 4 queues; a kernel behind a 17 ms
      // digest flush in the same queue waits for it)
      int lo = 0, hi = 0;
      NT_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
      NT_TRY(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, hi));
      cstream = stream2 = stream;
    } else {
      // the two compute streams (compute_stream)
      NT_TRY(compute_stream(&stream, (uint32_t)prop.multiProcessorCount, 0));
      NT_TRY(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
      NT_TRY(compute_stream(&stream2, (uint32_t)prop.multiProcessorCount, 1));
    }
    NT_TRY(hipEventCreateWithFlags(&ws_done, hipEventDisableTiming));
    NT_TRY(hipEventCreateWithFlags(&stash_done, hipEventDisableTiming));
    for (auto& e : cev) NT_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    NT_TRY(hipEventCreateWithFlags(&ws2_done, hipEventDisableTiming));
    NT_TRY(hipEventCreateWithFlags(&stash2_done, hipEventDisableTiming));
    // Nothing large is allocated here: the comb of B and the verify workspace
    // come with the first call that needs them (comb_b_for, ensure_ws).
    // Workspace slots = grid cap of the verify kernel.  Four times the resident
    // workgroups (256-thread blocks, `occupancy` waves per SIMD, 4 SIMDs per CU):
    // up to 2M signatures per launch the grid is then one 512-signature block per
    // slot and the hardware dispatcher balances the tail (interleaved A/B on
    // MI355X, tools/ab_env.sh: ~1% over 1x and 2x resident).
    uint32_t slots = (uint32_t)prop.multiProcessorCount * (uint32_t)nt::verify_occupancy() * 4;
    if (const char* e = std::getenv("NT_WS_SLOTS")) slots = (uint32_t)std::max(1, std::atoi(e));
    ws_slots = slots;
    sign_blocks = (uint32_t)prop.multiProcessorCount * 8;
    cus = (uint32_t)prop.multiProcessorCount;
    NT_TRY(hipEventRecord(ws_done, stream));
    NT_TRY(hipEventRecord(stash_done, stream));
    NT_TRY(hipEventRecord(ws2_done, stream));
    NT_TRY(hipEventRecord(stash2_done, stream));
    NT_TRY(hipStreamSynchronize(stream));
    return NT_OK;
  }

  // Wide combs of nkeys encoded points (host words) into d_comb (device);
  // negate: comb of -P (committee keys) instead of P (the base point).
  // s: the stream the build runs on (null = the slot's `stream`; the key
  // registry's admissions pass a low-priority stream of their own)
  int build_wcombs(int bits, const uint32_t* enc_host, uint32_t nkeys, int negate, uint32_t* d_comb, uint32_t* d_meta,
                   hipStream_t s = nullptr) {
    if (nkeys == 0) return NT_OK;
    if (!s) s = stream;
    const uint32_t batch = std::min<uint32_t>(nkeys, nt::wcomb_fill_batch(bits));
    uint32_t *d_enc = nullptr, *d_bases = nullptr, *d_tmp = nullptr;
    int rc = NT_OK;
    if (hipMalloc(&d_enc, 32ull * nkeys) != hipSuccess ||
        hipMalloc(&d_bases, nt::wcomb_bases_bytes_per_key(bits) * nkeys) != hipSuccess ||
        hipMalloc(&d_tmp, nt::wcomb_fill_tmp_bytes_per_key(bits) * batch) != hipSuccess) {
      rc = NT_ENOMEM;
    } else if (hipMemcpyAsync(d_enc, enc_host, 32ull * nkeys, hipMemcpyHostToDevice, s) != hipSuccess ||
               nt::launch_wcomb_build(bits, d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s) !=
                   hipSuccess ||
               hipStreamSynchronize(s) != hipSuccess) {
      rc = NT_EHIP;
    }
    if (d_enc) (void)hipFree(d_enc);
    if (d_bases) (void)hipFree(d_bases);
    if (d_tmp) (void)hipFree(d_tmp);
    return rc;
  }

  // the [k]A workspace of the verify kernel (ws_slots x 737 KB, ~1.5 GB at
  // 2,048 slots), on the slot's first verify
  int ensure_ws() {
    if (d_ws) return NT_OK;
    if (hipMalloc(&d_ws, nt::ws_bytes_per_slot() * ws_slots) != hipSuccess) {
      (void)hipGetLastError();
      d_ws = nullptr;
      return NT_ENOMEM;
    }
    return NT_OK;
  }

  // compute stream of chunk c
  hipStream_t cstr(int c) const { return (c & 1) ? stream2 : stream; }

  // verify launch of chunk c: even chunks use the device workspace on `stream`,
  // odd chunks stream2's own workspace (grown to the chunk's grid); per_lane as
  // in nt::launch_verify
  int verify_chunk(int c, int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t msg_bytes,
                   const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* out, int per_lane = 0) {
    if (!(c & 1))
      return verify(mode, pk, sig, msg, msg_bytes, off, len, n, out, stream, per_lane) == hipSuccess ? NT_OK : NT_EHIP;
    const uint64_t blocks = nt::verify_grid(n, ws_slots, per_lane);
    const int rc = grow_ws2(blocks);
    if (rc != NT_OK) return rc;
    if (hipStreamWaitEvent(stream2, ws2_done, 0) != hipSuccess ||
        nt::launch_verify(mode, pk, sig, msg, msg_bytes, off, len, n, d_combB, bbits, ws2.p,
                          (uint32_t)std::max<uint64_t>(blocks, 1), out, stream2, per_lane) != hipSuccess ||
        hipEventRecord(ws2_done, stream2) != hipSuccess)
      return NT_EHIP;
    return NT_OK;
  }

  // Key-cache launch on stream s with stash st: every launch waits for the
  // previous user of its stash (d[B_STASH]: stash_done, stash2: stash2_done --
  // host chunks on `stream` / stream2 and device-API calls on any stream) and
  // marks it, like the [k]A workspaces.  The key-grouping scratch (d[B_SORT] /
  // sort2) goes with its stash.
  template <class F>
  int keyset_launch(hipStream_t s, void* st, F&& launch) {
    const hipEvent_t ev = st == d[B_STASH].p ? stash_done : (st == stash2.p ? stash2_done : nullptr);
    if (ev && hipStreamWaitEvent(s, ev, 0) != hipSuccess) return NT_EHIP;
    if (launch() != hipSuccess) return NT_EHIP;
    if (ev && hipEventRecord(ev, s) != hipSuccess) return NT_EHIP;
    return NT_OK;
  }

  // Grow a buffer that enqueue-only device-API calls may still be using: wait
  // for its last user (the launch that recorded ev) before freeing it.
  int grow_synced(DevBuf& b, size_t bytes, hipEvent_t ev) {
    if (bytes <= b.cap) return NT_OK;
    if (b.p && hipEventSynchronize(ev) != hipSuccess) return NT_EHIP;
    return b.ensure(bytes);
  }
  // the stash / key-grouping scratch pair of slot k (0: d[B_STASH] / d[B_SORT],
  // 1: stash2 / sort2) for launches of up to m signatures
  int ensure_stash(int k, uint64_t m) {
    DevBuf& st = k ? stash2 : d[B_STASH];
    DevBuf& so = k ? sort2 : d[B_SORT];
    const hipEvent_t ev = k ? stash2_done : stash_done;
    const int rc = grow_synced(st, nt::keyset_stash_bytes(m, cus), ev);
    return rc != NT_OK ? rc : grow_synced(so, nt::keyset_sort_bytes(m), ev);
  }

  // ws2 holds >= blocks workspace slots; a grown buffer is freed only after its
  // last user (the kernel that recorded ws2_done) has finished
  int grow_ws2(uint64_t blocks) {
    const size_t need = nt::ws_bytes_per_slot() * std::max<uint64_t>(blocks, 1);
    if (need <= ws2.cap) return NT_OK;
    if (ws2.p && hipEventSynchronize(ws2_done) != hipSuccess) return NT_EHIP;
    return ws2.ensure(need);
  }

  // Device-API verify (nt_dev_ed25519_verify): successive calls alternate between
  // the two workspaces, each ordered by its own event, so back-to-back batches
  // issued on two caller streams overlap -- the waves of the next batch fill the
  // SIMDs the previous batch's last round leaves idle.  Calls on one stream stay
  // in stream order.  (Caller holds mu.)
  hipError_t verify_dev(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t msg_bytes,
                        const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* out, hipStream_t s) {
    if ((dev_calls++ & 1u) == 0) return verify(mode, pk, sig, msg, msg_bytes, off, len, n, out, s);
    if (grow_ws2(ws_slots) != NT_OK) return hipErrorOutOfMemory;
    hipError_t e = hipStreamWaitEvent(s, ws2_done, 0);
    if (e != hipSuccess) return e;
    e = nt::launch_verify(mode, pk, sig, msg, msg_bytes, off, len, n, d_combB, bbits, ws2.p, ws_slots, out, s);
    if (e != hipSuccess) return e;
    return hipEventRecord(ws2_done, s);
  }

  // verify launch that shares the workspace: wait for the previous user, then mark
  hipError_t verify(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t msg_bytes,
                    const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* out, hipStream_t s,
                    int per_lane = 0) {
    hipError_t e = hipStreamWaitEvent(s, ws_done, 0);
    if (e != hipSuccess) return e;
    e = nt::launch_verify(mode, pk, sig, msg, msg_bytes, off, len, n, d_combB, bbits, d_ws, ws_slots, out, s,
                          per_lane);
    if (e != hipSuccess) return e;
    return hipEventRecord(ws_done, s);
  }
};


}  // namespace ntrt

struct nt_ctx {
  std::vector<std::unique_ptr<ntrt::Device>> devs;
  uint64_t hbm_budget = 0;   // per device entry (Budget::limit); NT_HBM_BUDGET at init
  NtSmallModel small_model;  // written by nt_set_small_call_path before small_mode
  // small-call path (cpu_lane.hpp): NT_SMALL_OFF / AUTO / ALWAYS, host threads
  std::atomic<int> small_mode{NT_SMALL_OFF};
  std::atomic<int> small_threads{1};
  std::atomic<uint64_t> calls_host{0}, calls_gpu{0};
  // the key registry (nt_set_key_cache; registry.cpp): declared after devs so
  // that it -- its admission thread and device tables -- goes first
  std::shared_ptr<ntrt::KeyReg> reg;
};

namespace ntrt {
// Device tables of a key set, shared by its nt_keyset handle and every
// nt_committee built on it: a committee keeps them alive, so freeing the key set
// before the committee is safe.  The key combs' bytes are reserved
// in each device entry's budget while the tables live.
struct KsTables {
  uint32_t nkeys = 0;
  int bits = 0;                 // comb digit width of every key (nt::kKeyComb{Wide,Mid,Narrow})
  struct PerDev {
    int ordinal = -1;
    uint32_t* d_enc = nullptr;
    uint32_t* d_meta = nullptr;
    uint32_t* d_comb = nullptr;
    std::shared_ptr<Budget> budget;
    uint64_t reserved = 0;
  };
  std::vector<PerDev> dev;
  ~KsTables() {
    for (auto& d : dev) {
      if (d.budget && d.reserved) d.budget->release(d.reserved);
      if (d.ordinal < 0) continue;
      (void)hipSetDevice(d.ordinal);
      if (d.d_enc) (void)hipFree(d.d_enc);
      if (d.d_meta) (void)hipFree(d.d_meta);
      if (d.d_comb) (void)hipFree(d.d_comb);
    }
  }
};

// The device tables one key-cache launch reads: a key set's, or a published
// snapshot of the key registry's (keys >= nkeys verify as unknown -> reject).
struct KeyDev {
  const KsTables* t = nullptr;
  int bits = 0;
  uint32_t nkeys = 0;
};

// A published state of the key registry (registry.cpp): the host index of
// keys 0 .. table.nkeys - 1 and the device tables that hold their combs
// (allocated for `capacity` keys at the first admission; entries below
// table.nkeys are never written again, so a call that holds this snapshot
// reads them while later admissions fill the entries above).
struct RegSnap {
  nt::KeyTable table;
  std::shared_ptr<KsTables> t;
  int bits = 0;
  KeyDev dev() const { return KeyDev{t.get(), bits, table.nkeys}; }
};
// the published snapshot of ctx's registry, or null (registry off / empty)
std::shared_ptr<const RegSnap> reg_snapshot(nt_ctx* ctx);
// keys a call could not find: up to kRegNoteMax distinct ones are counted as
// sightings (and queued for admission once seen `admit_after` times)
constexpr uint32_t kRegNoteMax = 256;
void reg_note_misses(nt_ctx* ctx, const std::vector<const uint8_t*>& keys);
void reg_count(nt_ctx* ctx, uint64_t hits, uint64_t misses);
// first-use tables and width choice shared with nt_keyset_create (ntcrypto.cpp)
int keyset_comb_bits(nt_ctx* ctx, uint32_t nkeys);
hipError_t table_malloc(void** p, size_t bytes);  // comb tables (NT_TABLE_ALLOC)
int comb_b_for(Device& dv);

}  // namespace ntrt

struct nt_keyset {
  nt_ctx* ctx = nullptr;
  uint32_t nkeys = 0;
  std::vector<uint8_t> enc;     // host copy of the key encodings (small-call path)
  int bits = 0;                 // = t->bits
  std::vector<uint32_t> flags;  // host copy of kKey* bits
  std::shared_ptr<ntrt::KsTables> t;
};

namespace ntrt {

// Split [0, n) into one contiguous range per device, boundaries multiple of `align`.
inline std::vector<std::pair<uint64_t, uint64_t>> shard(uint64_t n, size_t ndev, uint64_t align) {
  std::vector<std::pair<uint64_t, uint64_t>> r;
  uint64_t per = (n + ndev - 1) / ndev;
  per = (per + align - 1) / align * align;
  uint64_t lo = 0;
  for (size_t d = 0; d < ndev; ++d) {
    const uint64_t hi = std::min(n, lo + per);
    r.emplace_back(lo, hi);
    lo = hi;
  }
  return r;
}

// The execution slot of device entry d a call runs on, locked into lk.  Bulk
// calls take the entry's own slot (waiting for it), so the extra
// high-priority slots stay free for latency-sized calls; a latency-sized call
// takes the first free extra slot, else the entry's own slot if free, else
// waits for the first extra slot (two concurrent bulk calls must
// not occupy both slots and block a certificate-sized call behind a digest).
inline Device& acquire_slot(nt_ctx* ctx, size_t d, bool latency, std::unique_lock<std::mutex>& lk) {
  Device& p = *ctx->devs[d];
  if (!latency || p.extra.empty()) {
    lk = std::unique_lock<std::mutex>(p.mu);
    return p;
  }
  std::vector<Device*> order;
  for (auto& x : p.extra) order.push_back(x.get());
  order.push_back(&p);
  for (Device* s : order) {
    std::unique_lock<std::mutex> l(s->mu, std::try_to_lock);
    if (l.owns_lock()) {
      lk = std::move(l);
      return *s;
    }
  }
  lk = std::unique_lock<std::mutex>(order[0]->mu);
  return *order[0];
}

// digests whose longest message is short (header / vote / certificate
// preimages) finish fast; long ones (worker batches) are bulk
inline bool sha_latency(uint64_t n, const uint64_t* len) {
  for (uint64_t i = 0; i < n; ++i)
    if (len[i] > (64u << 10)) return false;
  return true;
}

// work below one round of resident waves: a latency-sized call
inline bool latency_sized(const nt_ctx* ctx, uint64_t items_per_device, uint64_t round) {
  (void)ctx;
  return items_per_device <= round;
}

template <class F>
int run_sharded(nt_ctx* ctx, uint64_t n, uint64_t align, F&& fn, bool latency = false) {
  const size_t nd = ctx->devs.size();
  auto parts = shard(n, nd, align);
  if (nd == 1) {
    std::unique_lock<std::mutex> lk;
    Device& dv = acquire_slot(ctx, 0, latency, lk);
    if (hipSetDevice(dv.ordinal) != hipSuccess) return NT_EHIP;
    return fn(dv, parts[0].first, parts[0].second);
  }
  std::vector<int> rcs(nd, NT_OK);
  std::vector<std::thread> th;
  for (size_t d = 0; d < nd; ++d) {
    if (parts[d].first >= parts[d].second) continue;
    th.emplace_back([&, d] {
      std::unique_lock<std::mutex> lk;
      Device& dv = acquire_slot(ctx, d, latency, lk);
      if (hipSetDevice(dv.ordinal) != hipSuccess) {
        rcs[d] = NT_EHIP;
        return;
      }
      rcs[d] = fn(dv, parts[d].first, parts[d].second);
    });
  }
  for (auto& t : th) t.join();
  for (int rc : rcs)
    if (rc != NT_OK) return rc;
  return NT_OK;
}

#define NT_CHK(expr)              \
  do {                            \
    int _rc = (expr);             \
    if (_rc != NT_OK) return _rc; \
  } while (0)


}  // namespace ntrt
