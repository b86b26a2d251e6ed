// small_model.hpp -- the small-call path's cost model and routing rules
// (host-only; shared by ntcrypto.cpp and the host test harness, so the routing
// decision is tested on the CPU: tests/test_small_route.py).
//
// The reference calls the hot path one message at a time (Core::run,
// primary/src/core.rs:349-411; Processor, worker/src/processor.rs:36-38).  A
// GPU call that small costs a fixed floor; below it the host lane
// (cpu_lane.cpp) is faster.  The floor depends on the kernel the call would
// run: the uncached verify kernel (decompression of A and R, ~130 doublings per
// lane) or the key-cache kernel (no doublings; one inversion per lane batch),
// so the model holds one GPU floor per kernel and a call is compared with the
// floor of the kernel it would actually run.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cmath>

// Calibrated by nt_set_small_call_path on the context's own host threads and
// device (ntcrypto.cpp calibrate_small); NT_SMALL_* environment variables
// override single fields.  The defaults are round-2 / round-6 measurements.
struct NtSmallModel {
  double cpu_verify_us = 36.0;    // one host-lane verify_strict on one thread
  double gpu_verify_us = 1300.0;  // a GPU verify call below one round of resident waves (uncached kernel)
  double cpu_sha_mbs = 850.0;     // host-lane SHA-512, one thread
  double gpu_lane_mbs = 30.0;     // one GPU lane's serial SHA-512 chain
  double gpu_call_us = 60.0;      // a GPU digest call's fixed cost (launch + copies)
  double pcie_gbs = 20.0;         // host -> device copy of digest inputs
  double spawn_us = 15.0;         // waking the host lane's worker pool
  int calibrated = 0;
  double gpu_keyset_us = 400.0;   // a GPU verify call below one round through the key cache
};

namespace nt {

// which GPU kernel a verify call would run
enum SmallKind { kRouteUncached = 0, kRouteKeyCache = 1 };

// host lane iff its estimated time on T = min(threads, nsig) threads is below
// the GPU floor of the kernel the call would run
inline bool small_verify_on_host(const NtSmallModel& m, uint64_t nsig, int threads, int kind) {
  const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, threads), nsig));
  const double cpu = std::ceil((double)nsig / (double)T) * m.cpu_verify_us + (T > 1 ? m.spawn_us : 0.0);
  return cpu < (kind == kRouteKeyCache ? m.gpu_keyset_us : m.gpu_verify_us);
}

// a digest call: the host's longest serial chain vs the GPU call floor + the
// longest lane + the PCIe copy (bytes, microseconds)
inline bool small_sha_on_host(const NtSmallModel& m, uint64_t n, uint64_t total, uint64_t longest, int threads) {
  const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, threads), n));
  const double cpu = std::max((double)longest, (double)total / (double)T) / m.cpu_sha_mbs + (T > 1 ? m.spawn_us : 0.0);
  const double gpu = m.gpu_call_us + (double)longest / m.gpu_lane_mbs + (double)total / (m.pcie_gbs * 1e3);
  return cpu < gpu;
}

}  // namespace nt
