// gfx950 integer-ALU issue-rate microbenchmark.
// Measures lane-ops/s for the instructions the field / SHA-512 kernels are built from.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

// 8 independent chains per lane, each op a dependency on its own chain.
#define CHAIN8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u64_u32(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

__global__ void k_mul_lo_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_u32_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u32_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed + 7;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_addc_co_u32(uint32_t* out, uint32_t seed) {
  // 64-bit add as a v_add_co_u32 / v_addc_co_u32 pair: counts 2 ops per pair.
  uint32_t lo[8], hi[8]; for (int i = 0; i < 8; ++i) { lo[i] = seed + threadIdx.x * 8 + i; hi[i] = i; }
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS / 2; ++it) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo[i]), "+v"(hi[i]) : "v"(b) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= lo[i] ^ hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_add_u64(uint32_t* out, uint32_t seed) {
  // gfx950 v_lshl_add_u64 (64-bit shift+add in one VALU op)
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint64_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_xor3(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 5;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma_f64(uint32_t* out, uint32_t seed) {
  double a[8]; for (int i = 0; i < 8; ++i) a[i] = (double)(seed + threadIdx.x * 8 + i);
  double b = 0.999999, c = 1e-9;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  double r = 0; for (int i = 0; i < 8; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r;
}

__global__ void k_add3_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 5;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi_u32_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_lshr_b64(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(a[i]));
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}
__global__ void k_cndmask(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_and(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mad_partial(uint32_t* out, uint32_t seed) {
  // only 16 of 64 lanes active: does a wave64 instruction issue faster?
  if ((threadIdx.x & 63) >= 16) return;
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}
__global__ void k_mad_onewave(uint32_t* out, uint32_t seed) {
  // one wave per SIMD: single-wave issue rate with 8 independent chains
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
  for (int it = 0; it < ITERS; ++it) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  struct { const char* name; kfn f; double ops_per_iter; } ks[] = {
    {"v_add_u32", k_add_u32, 8}, {"v_add3_u32", k_add3_u32, 8}, {"v_bfi_b32", k_xor3, 8},
    {"v_alignbit_b32", k_alignbit, 8}, {"v_add_co+v_addc_co (ops)", k_addc_co_u32, 8},
    {"v_lshl_add_u64", k_add_u64, 8}, {"v_mul_u32_u24", k_mul_u32_u24, 8},
    {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 8}, {"v_mad_u32_u24", k_mad_u32_u24, 8},
    {"v_mul_lo_u32", k_mul_lo_u32, 8}, {"v_mul_hi_u32", k_mul_hi_u32, 8},
    {"v_mad_u64_u32", k_mad_u64_u32, 8}, {"v_fma_f64", k_fma_f64, 8},
    {"v_lshrrev_b64", k_lshr_b64, 8}, {"v_cmp+v_cndmask (ops)", k_cndmask, 16}, {"v_and_b32", k_and, 8},
  };
  int dev = 0; hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, dev));
  printf("device %s CUs=%d clock=%d kHz\n", prop.name, prop.multiProcessorCount, prop.clockRate);
  const int block = 256, grid = prop.multiProcessorCount * 8;  // 8 waves/SIMD
  uint32_t* d; CHECK(hipMalloc(&d, sizeof(uint32_t) * grid * block));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, 1u);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, (uint32_t)r);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    double lane_ops = (double)grid * block * ITERS * k.ops_per_iter * reps;
    double rate = lane_ops / (ms * 1e-3);
    // cycles per wave64 instruction per SIMD at 2.4 GHz
    double simds = prop.multiProcessorCount * 4.0;
    double cyc = simds * 2.4e9 * 64.0 / rate;
    printf("%-28s %8.2f T lane-ops/s   %5.2f cyc/wave-instr/SIMD (@2.4GHz)\n", k.name, rate / 1e12, cyc);
  }
  // issue-rate probes for latency-bound kernels (SHA-512 config 4)
  {
    const int g1 = prop.multiProcessorCount;  // 1 block of 256 = 1 wave per SIMD
    for (int pass = 0; pass < 2; ++pass) {
      kfn f = pass == 0 ? k_mad_onewave : k_mad_partial;
      hipLaunchKernelGGL(f, dim3(g1), dim3(256), 0, 0, d, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(g1), dim3(256), 0, 0, d, (uint32_t)r);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double instr_per_wave = (double)ITERS * 8 * 5;
      const double cyc = ms * 1e-3 * 2.4e9 / instr_per_wave;
      printf("%-28s %5.2f cyc/instr for ONE wave per SIMD (%s)\n", "v_mad_u64_u32 1 wave/SIMD", cyc,
             pass == 0 ? "64 lanes active" : "16 lanes active");
    }
  }
  return 0;
}
