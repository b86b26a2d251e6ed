// co_dispatch.hip -- does a short kernel on one stream run while a long
// VALU-bound kernel of another stream occupies every SIMD?  (DESIGN.md §10:
// in the config-3 pipeline a 15 us digest launch enqueued beside a key-cache
// launch finishes only at that launch's tail.)
//
// `busy`: 2 workgroups of 256 threads per CU (2 waves per SIMD, like the
// key-cache launch of an 8-GPU shard), a bounded VALU loop with NV live
// registers per lane.  `tiny`: 49 workgroups of 256 threads, a short VALU loop,
// optionally at wave priority PRIO (s_setprio).  Printed: tiny's duration
// alone and when enqueued 1 ms into busy (HIP events on tiny's own stream),
// for NV = 24 / 100 and PRIO = 0 / 2 / 3; then the same with a busy kernel that
// streams random 128-byte table lines (like the key-cache launch) and a tiny
// kernel that reads its 72-80-byte messages first.  Every loop is bounded.
// Build: hipcc -O3 --offload-arch=gfx950 co_dispatch.hip -o co_dispatch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int NV>
__global__ __launch_bounds__(256, 2) void busy(uint32_t* out, uint32_t iters) {
  uint32_t v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = threadIdx.x * 2654435761u + (uint32_t)i * 7u;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = v[i] * 0x9E3779B1u + v[(i + 1) % NV];
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NV; ++i) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// busy_mem: like the key-cache launch -- random 128-byte line reads from a
// large table (8 x 16 B per lane per step) between VALU work
__global__ __launch_bounds__(256, 2) void busy_mem(const uint4* __restrict__ tab, uint64_t lines, uint32_t* out,
                                                   uint32_t iters) {
  uint32_t x = blockIdx.x * 256 + threadIdx.x, acc = x;
  for (uint32_t it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    const uint4* e = tab + (uint64_t)(x % (uint32_t)lines) * 8;
    uint4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = e[i];
#pragma unroll
    for (int r = 0; r < 40; ++r) acc = acc * 0x9E3779B1u + (r & 1 ? v[r & 7].x : v[r & 7].w);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// tiny_mem: per lane a 72-byte message read (5 x 16 B) and a short VALU chain,
// like a certificate-digest launch
template <int PRIO>
__global__ __launch_bounds__(256) void tiny_mem(const uint4* __restrict__ msg, uint32_t* out, uint32_t iters) {
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t x = i;
#pragma unroll
  for (int k = 0; k < 5; ++k) x ^= msg[(uint64_t)i * 5 + k].x;
  for (uint32_t it = 0; it < iters; ++it) x = x * 0x9E3779B1u + it;
  out[i] = x;
}

// tiny_wide: the tiny loop holding NT live registers per lane (~2 NT VGPRs,
// like a digest launch's 84)
template <int PRIO, int NT>
__global__ __launch_bounds__(256) void tiny_wide(uint32_t* out, uint32_t iters) {
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  uint32_t v[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) v[i] = threadIdx.x + (uint32_t)i;
  for (uint32_t it = 0; it < iters / 16; ++it) {
#pragma unroll
    for (int i = 0; i < NT; ++i) v[i] = v[i] * 0x9E3779B1u + v[(i + 1) % NT];
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NT; ++i) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int PRIO>
__global__ __launch_bounds__(256) void tiny(uint32_t* out, uint32_t iters) {
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  uint32_t x = threadIdx.x;
  for (uint32_t it = 0; it < iters; ++it) x = x * 0x9E3779B1u + it;
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int NV, int PRIO>
static int run(hipStream_t sa, hipStream_t sb, uint32_t* d_busy, uint32_t* d_tiny, uint32_t busy_iters,
               uint32_t tiny_iters, int cus) {
  hipEvent_t e0, e1, b0, b1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  // alone
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL(tiny<PRIO>, dim3(49), dim3(256), 0, sb, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipStreamSynchronize(sb));
  float alone = 0;
  CK(hipEventElapsedTime(&alone, e0, e1));
  // beside busy
  CK(hipEventRecord(b0, sa));
  hipLaunchKernelGGL(busy<NV>, dim3(2 * cus), dim3(256), 0, sa, d_busy, busy_iters);
  CK(hipEventRecord(b1, sa));
  std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL(tiny<PRIO>, dim3(49), dim3(256), 0, sb, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipDeviceSynchronize());
  float beside = 0, busy_ms = 0, tiny_start = 0;
  CK(hipEventElapsedTime(&beside, e0, e1));
  CK(hipEventElapsedTime(&busy_ms, b0, b1));
  CK(hipEventElapsedTime(&tiny_start, b0, e0));
  std::printf("NV %3d prio %d: tiny alone %8.1f us | beside busy %8.1f us (enqueued %.2f ms into a %.2f ms busy launch)\n",
              NV, PRIO, alone * 1e3, beside * 1e3, tiny_start, busy_ms);
  return 0;
}

template <int PRIO>
static int run_mem(hipStream_t sa, hipStream_t sb, const uint4* tab, uint64_t lines, const uint4* msg,
                   uint32_t* d_busy, uint32_t* d_tiny, uint32_t busy_iters, uint32_t tiny_iters, int cus) {
  hipEvent_t e0, e1, b0, b1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL(tiny_mem<PRIO>, dim3(49), dim3(256), 0, sb, msg, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipStreamSynchronize(sb));
  float alone = 0;
  CK(hipEventElapsedTime(&alone, e0, e1));
  CK(hipEventRecord(b0, sa));
  hipLaunchKernelGGL(busy_mem, dim3(2 * cus), dim3(256), 0, sa, tab, lines, d_busy, busy_iters);
  CK(hipEventRecord(b1, sa));
  std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL(tiny_mem<PRIO>, dim3(49), dim3(256), 0, sb, msg, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipDeviceSynchronize());
  float beside = 0, busy_ms = 0, tiny_start = 0;
  CK(hipEventElapsedTime(&beside, e0, e1));
  CK(hipEventElapsedTime(&busy_ms, b0, b1));
  CK(hipEventElapsedTime(&tiny_start, b0, e0));
  std::printf("memory-bound busy, prio %d: tiny_mem alone %8.1f us | beside busy %8.1f us (enqueued %.2f ms into a "
              "%.2f ms busy launch)\n", PRIO, alone * 1e3, beside * 1e3, tiny_start, busy_ms);
  return 0;
}

// tiny_wide beside one or two co-resident busy<NV> launches (2 waves per SIMD each)
template <int NV, int PRIO, int NT>
static int run_wide(hipStream_t sa, hipStream_t sa2, hipStream_t sb, uint32_t* d_busy, uint32_t* d_busy2,
                    uint32_t* d_tiny, uint32_t busy_iters, uint32_t tiny_iters, int cus, int nbusy) {
  hipEvent_t e0, e1, b0, b1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL((tiny_wide<PRIO, NT>), dim3(49), dim3(256), 0, sb, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipStreamSynchronize(sb));
  float alone = 0;
  CK(hipEventElapsedTime(&alone, e0, e1));
  CK(hipEventRecord(b0, sa));
  hipLaunchKernelGGL(busy<NV>, dim3(2 * cus), dim3(256), 0, sa, d_busy, busy_iters);
  if (nbusy > 1) hipLaunchKernelGGL(busy<NV>, dim3(2 * cus), dim3(256), 0, sa2, d_busy2, busy_iters);
  CK(hipEventRecord(b1, sa));
  std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CK(hipEventRecord(e0, sb));
  hipLaunchKernelGGL((tiny_wide<PRIO, NT>), dim3(49), dim3(256), 0, sb, d_tiny, tiny_iters);
  CK(hipEventRecord(e1, sb));
  CK(hipDeviceSynchronize());
  float beside = 0, busy_ms = 0, tiny_start = 0;
  CK(hipEventElapsedTime(&beside, e0, e1));
  CK(hipEventElapsedTime(&busy_ms, b0, b1));
  CK(hipEventElapsedTime(&tiny_start, b0, e0));
  std::printf("%d x busy<%d>, tiny_wide<%d> prio %d: alone %8.1f us | beside %8.1f us (enqueued %.2f ms into a "
              "%.2f ms busy launch)\n", nbusy, NV, NT, PRIO, alone * 1e3, beside * 1e3, tiny_start, busy_ms);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  uint32_t *d_busy = nullptr, *d_tiny = nullptr;
  CK(hipMalloc(&d_busy, (size_t)2 * cus * 256 * 4));
  CK(hipMalloc(&d_tiny, (size_t)49 * 256 * 4));
  const uint32_t busy_iters = 20000, tiny_iters = 2000;
  // warm-up
  hipLaunchKernelGGL(busy<24>, dim3(2 * cus), dim3(256), 0, sa, d_busy, 100u);
  hipLaunchKernelGGL(tiny<0>, dim3(49), dim3(256), 0, sb, d_tiny, 10u);
  CK(hipDeviceSynchronize());
  if (run<24, 0>(sa, sb, d_busy, d_tiny, busy_iters, tiny_iters, cus)) return 1;
  if (run<24, 2>(sa, sb, d_busy, d_tiny, busy_iters, tiny_iters, cus)) return 1;
  if (run<100, 0>(sa, sb, d_busy, d_tiny, busy_iters / 4, tiny_iters, cus)) return 1;
  if (run<100, 2>(sa, sb, d_busy, d_tiny, busy_iters / 4, tiny_iters, cus)) return 1;
  if (run<100, 3>(sa, sb, d_busy, d_tiny, busy_iters / 4, tiny_iters, cus)) return 1;
  {
    hipStream_t sa2;
    uint32_t* d_busy2 = nullptr;
    CK(hipStreamCreateWithFlags(&sa2, hipStreamNonBlocking));
    CK(hipMalloc(&d_busy2, (size_t)2 * cus * 256 * 4));
    if (run_wide<53, 2, 40>(sa, sa2, sb, d_busy, d_busy2, d_tiny, busy_iters / 2, tiny_iters, cus, 1)) return 1;
    if (run_wide<53, 2, 40>(sa, sa2, sb, d_busy, d_busy2, d_tiny, busy_iters / 2, tiny_iters, cus, 2)) return 1;
    if (run_wide<53, 0, 40>(sa, sa2, sb, d_busy, d_busy2, d_tiny, busy_iters / 2, tiny_iters, cus, 1)) return 1;
    if (run_wide<53, 2, 2>(sa, sa2, sb, d_busy, d_busy2, d_tiny, busy_iters / 2, tiny_iters, cus, 2)) return 1;
    CK(hipFree(d_busy2));
  }
  // a 4 GB table of 128-byte lines, 49 x 256 messages of 80 bytes
  const uint64_t lines = (4ull << 30) / 128;
  uint4 *tab = nullptr, *msg = nullptr;
  CK(hipMalloc(&tab, lines * 128));
  CK(hipMemset(tab, 1, lines * 128));
  CK(hipMalloc(&msg, (size_t)49 * 256 * 80));
  CK(hipMemset(msg, 2, (size_t)49 * 256 * 80));
  CK(hipDeviceSynchronize());
  if (run_mem<0>(sa, sb, tab, lines, msg, d_busy, d_tiny, 4000, tiny_iters, cus)) return 1;
  if (run_mem<2>(sa, sb, tab, lines, msg, d_busy, d_tiny, 4000, tiny_iters, cus)) return 1;
  CK(hipFree(tab));
  CK(hipFree(msg));
  CK(hipFree(d_busy));
  CK(hipFree(d_tiny));
  return 0;
}
