// Single-wave issue/latency probe on gfx950: one 64-lane wave per SIMD, C
// independent dependency chains of one instruction.  cycles/instr vs C gives
// the dependent latency (C small) and the single-wave issue limit (C large).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 4096;

template <int C>
__global__ void k_mad(uint32_t* out, uint32_t seed) {
  uint64_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
  }
  uint64_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}
template <int C>
__global__ void k_madnc(uint32_t* out, uint32_t seed) {  // no carry-out (null SGPR dest)
  uint64_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) { uint64_t cy; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[i]), "=s"(cy) : "v"(b), "v"(c)); }
  }
  uint64_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}
template <int C>
__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int C>
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int C>
__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int C>
__global__ void k_addu64(uint32_t* out, uint32_t seed) {
  uint64_t a[C]; for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x * C + i;
  uint64_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(b));
  }
  uint64_t r = 0; for (int i = 0; i < C; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

typedef void (*kfn)(uint32_t*, uint32_t);
template <template <int> class K> struct Set {};

int run(const char* name, kfn f, int chains, int waves_per_simd, uint32_t* d, int cus) {
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int block = 256 * waves_per_simd;  // 4*w waves per block -> w waves per SIMD
  hipLaunchKernelGGL(f, dim3(cus), dim3(block), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(f, dim3(cus), dim3(block), 0, 0, d, (uint32_t)r);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double instr = (double)ITERS * chains * 3 * waves_per_simd;  // per SIMD
  printf("%-16s chains=%2d waves/SIMD=%d  %6.2f cyc per instr per SIMD\n", name, chains, waves_per_simd,
         ms * 1e-3 * 2.4e9 / instr);
  return 0;
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d; CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 1024));
#define ALL(K, NAME) \
  run(NAME, K<1>, 1, 1, d, cus); run(NAME, K<2>, 2, 1, d, cus); run(NAME, K<4>, 4, 1, d, cus); \
  run(NAME, K<8>, 8, 1, d, cus); run(NAME, K<16>, 16, 1, d, cus); run(NAME, K<8>, 8, 2, d, cus); \
  run(NAME, K<8>, 8, 4, d, cus);
  ALL(k_mad, "v_mad_u64_u32")
  ALL(k_madnc, "mad_u64 sgpr-cy")
  ALL(k_add, "v_add_u32")
  ALL(k_mullo, "v_mul_lo_u32")
  ALL(k_alignbit, "v_alignbit_b32")
  ALL(k_addu64, "v_lshl_add_u64")
  return 0;
}
