// Microbenchmark: is a field squaring with its carries folded into the column
// chains (start column k+1's accumulation at carry_k; two chains, columns 0-4
// and 5-9, joined at limbs 5 and 0: ~29 carry instructions instead of ~40)
// faster than the current fe_sq (10 independent columns + a 12-step carry
// chain) at the occupancies the verify kernel runs?  Dependent chains of
// squarings per lane (as in fe_pow22523) with CH independent chains per lane
// (CH = 1: a serial exponentiation; CH = 2: two independent operations, as in
// a point formula), W waves per SIMD.  Prints squarings/s and agreement of the
// two variants' canonical results.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../narwhal-tusk_amd/csrc/fe25519.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

namespace nt {
// acc + a * b as one v_mad_u64_u32 the compiler cannot reassociate (it otherwise
// sums a column from 0 and adds the carry at the end, undoing the fold)
__device__ __forceinline__ uint64_t madc(uint64_t acc, uint32_t a, uint32_t b) {
  uint64_t r;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(acc) : "vcc");
  return r;
}
// f^2 with folded carries (same input contract as fe_sq: reduced limbs)
__device__ __forceinline__ void fe_sq_fold(fe& out, const fe& f) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = 2u * f0, f1_2 = 2u * f1, f2_2 = 2u * f2, f3_2 = 2u * f3;
  const uint32_t f4_2 = 2u * f4, f5_2 = 2u * f5, f6_2 = 2u * f6, f7_2 = 2u * f7;
  const uint32_t f5_38 = 38u * f5, f6_19 = 19u * f6, f7_38 = 38u * f7, f8_19 = 19u * f8, f9_38 = 38u * f9;
  // chain A: columns 0..4, each starting from the previous column's carry
  uint64_t h = (uint64_t)f0 * f0;
  h = madc(h, f1_2, f9_38); h = madc(h, f2_2, f8_19); h = madc(h, f3_2, f7_38); h = madc(h, f4_2, f6_19);
  h = madc(h, f5, f5_38);
  uint32_t l0 = (uint32_t)h & NT_M26;
  h = madc(h >> 26, f0_2, f1); h = madc(h, f2, f9_38); h = madc(h, f3_2, f8_19); h = madc(h, f4, f7_38);
  h = madc(h, f5_2, f6_19);
  uint32_t l1 = (uint32_t)h & NT_M25;
  h = madc(h >> 25, f0_2, f2); h = madc(h, f1_2, f1); h = madc(h, f3_2, f9_38); h = madc(h, f4_2, f8_19);
  h = madc(h, f5_2, f7_38); h = madc(h, f6, f6_19);
  uint32_t l2 = (uint32_t)h & NT_M26;
  h = madc(h >> 26, f0_2, f3); h = madc(h, f1_2, f2); h = madc(h, f4, f9_38); h = madc(h, f5_2, f8_19);
  h = madc(h, f6, f7_38);
  uint32_t l3 = (uint32_t)h & NT_M25;
  h = madc(h >> 25, f0_2, f4); h = madc(h, f1_2, f3_2); h = madc(h, f2, f2); h = madc(h, f5_2, f9_38);
  h = madc(h, f6_2, f8_19); h = madc(h, f7, f7_38);
  uint32_t l4 = (uint32_t)h & NT_M26;
  const uint64_t c4 = h >> 26;
  // chain B: columns 5..9
  uint64_t g = (uint64_t)f0_2 * f5;
  g = madc(g, f1_2, f4); g = madc(g, f2_2, f3); g = madc(g, f6, f9_38); g = madc(g, f7_2, f8_19);
  const uint64_t t5 = (g & NT_M25) + c4;
  g = madc(g >> 25, f0_2, f6); g = madc(g, f1_2, f5_2); g = madc(g, f2_2, f4); g = madc(g, f3_2, f3);
  g = madc(g, f7_2, f9_38); g = madc(g, f8, f8_19);
  uint32_t l6 = (uint32_t)g & NT_M26;
  g = madc(g >> 26, f0_2, f7); g = madc(g, f1_2, f6); g = madc(g, f2_2, f5); g = madc(g, f3_2, f4);
  g = madc(g, f8, f9_38);
  uint32_t l7 = (uint32_t)g & NT_M25;
  g = madc(g >> 25, f0_2, f8); g = madc(g, f1_2, f7_2); g = madc(g, f2_2, f6); g = madc(g, f3_2, f5_2);
  g = madc(g, f4, f4); g = madc(g, f9, f9_38);
  uint32_t l8 = (uint32_t)g & NT_M26;
  g = madc(g >> 26, f0_2, f9); g = madc(g, f1_2, f8); g = madc(g, f2_2, f7); g = madc(g, f3_2, f6);
  g = madc(g, f4_2, f5);
  uint32_t l9 = (uint32_t)g & NT_M25;
  const uint64_t c9 = g >> 25;
  // joins: limb 5 takes chain A's carry, limb 0 chain B's (x 19)
  out.v[5] = (uint32_t)t5 & NT_M25;
  l6 += (uint32_t)(t5 >> 25);
  const uint64_t t0 = (uint64_t)l0 + 19u * c9;
  out.v[0] = (uint32_t)t0 & NT_M26;
  l1 += (uint32_t)(t0 >> 26);
  out.v[1] = l1; out.v[2] = l2; out.v[3] = l3; out.v[4] = l4;
  out.v[6] = l6; out.v[7] = l7; out.v[8] = l8; out.v[9] = l9;
#pragma unroll
  for (int i = 0; i < 10; ++i) NT_OPAQUE32(out.v[i]);
  NT_MUL_FENCE();
}
}  // namespace nt

using namespace nt;

template <int FOLD, int CH>
__global__ __launch_bounds__(256) void k_sq(uint32_t* io, int iters) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int i = 0; i < 10; ++i) x[c].v[i] = io[(t * CH + c) * 10 + i];
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (FOLD) fe_sq_fold(x[c], x[c]);
      else fe_sq(x[c], x[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    uint32_t w[8];
    fe_tobytes_w(w, x[c]);
#pragma unroll
    for (int i = 0; i < 8; ++i) io[(t * CH + c) * 10 + i] = w[i];
  }
}

template <int FOLD, int CH>
static int run(int cus, int waves_per_simd, int iters, uint32_t* d, uint32_t* h, size_t words, double* rate) {
  const int blocks = cus * waves_per_simd;  // 4 waves per block: one per SIMD
  const size_t n = (size_t)blocks * 256;
  CHECK(hipMemcpy(d, h, n * CH * 10 * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_sq<FOLD, CH>), dim3(blocks), dim3(256), 0, 0, d, 8);  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(d, h, n * CH * 10 * 4, hipMemcpyHostToDevice));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_sq<FOLD, CH>), dim3(blocks), dim3(256), 0, 0, d, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  *rate = (double)n * CH * iters / (ms * 1e-3);
  (void)words;
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int iters = 20000;
  const size_t maxn = (size_t)cus * 3 * 256 * 2 * 10;
  uint32_t* h = (uint32_t*)malloc(maxn * 4);
  uint32_t* h2 = (uint32_t*)malloc(maxn * 4);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < maxn; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)s & ((i % 10) & 1 ? NT_M25 : NT_M26);
  }
  uint32_t* d;
  CHECK(hipMalloc(&d, maxn * 4));
  printf("device CUs=%d, %d dependent squarings per chain\n", cus, iters);
  for (int w = 1; w <= 3; ++w) {
    double r00, r01, r10, r11;
    if (run<0, 1>(cus, w, iters, d, h, maxn, &r00)) return 1;
    CHECK(hipMemcpy(h2, d, (size_t)cus * w * 256 * 10 * 4, hipMemcpyDeviceToHost));
    if (run<1, 1>(cus, w, iters, d, h, maxn, &r10)) return 1;
    uint32_t* h3 = (uint32_t*)malloc((size_t)cus * w * 256 * 10 * 4);
    CHECK(hipMemcpy(h3, d, (size_t)cus * w * 256 * 10 * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < (size_t)cus * w * 256; ++i)
      for (int k = 0; k < 8; ++k) bad += h2[i * 10 + k] != h3[i * 10 + k];
    free(h3);
    if (run<0, 2>(cus, w, iters, d, h, maxn, &r01)) return 1;
    if (run<1, 2>(cus, w, iters, d, h, maxn, &r11)) return 1;
    printf("waves/SIMD=%d  1 chain: fe_sq %.3f G/s  folded %.3f G/s (%+.1f%%)  |  2 chains: fe_sq %.3f G/s  folded %.3f G/s (%+.1f%%)  results differ in %zu words\n",
           w, r00 / 1e9, r10 / 1e9, 100.0 * (r10 / r00 - 1), r01 / 1e9, r11 / 1e9, 100.0 * (r11 / r01 - 1), bad);
  }
  return 0;
}
