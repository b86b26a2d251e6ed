// Does a wave64 VALU instruction run faster when only some lanes are active?
// One wave per SIMD (1,024 waves), C independent dependency chains of
// v_alignbit_b32 (the SHA-512 rotate), lanes >= ACTIVE masked off by a branch.
// If masked 16-lane quarters were skipped, ACTIVE = 16 would run ~4x faster
// per instruction than ACTIVE = 64 (the question behind config 4's layout).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 8192;

template <int C>
__global__ __launch_bounds__(64) void k_chain(uint32_t* out, uint32_t seed, int active) {
  uint32_t a[C], b[C];
  for (int i = 0; i < C; ++i) { a[i] = seed + threadIdx.x * C + i; b[i] = a[i] * 2654435761u; }
  if ((int)threadIdx.x < active) {
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < C; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 14" : "+v"(a[i]) : "v"(b[i]));
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int C>
int run(uint32_t* d, int waves, int active) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_chain<C>, dim3(waves), dim3(64), 0, 0, d, 1u, active);  // warm-up
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(k_chain<C>, dim3(waves), dim3(64), 0, 0, d, 1u, active);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double cyc = ms * 1e-3 * 2.4e9 / ((double)ITERS * C);
  printf("C=%d waves=%d active=%2d: %.3f ms, %.2f cycles per instruction per wave (2.4 GHz)\n", C, waves, active, ms,
         cyc);
  return 0;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int waves = cus * 4;  // one per SIMD
  uint32_t* d = nullptr;
  CHECK(hipMalloc(&d, (size_t)waves * 64 * 4 * 4));
  for (int active : {64, 32, 16, 8})
    if (run<1>(d, waves, active) || run<4>(d, waves, active) || run<8>(d, waves, active)) return 1;
  for (int active : {64, 16})
    if (run<8>(d, waves * 4, active)) return 1;
  CHECK(hipFree(d));
  return 0;
}
