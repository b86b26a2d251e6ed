// ISA probe (compiled only, never launched): one loop per field primitive of
// fe25519.hpp, so the loop bodies in the gfx950 assembly are exactly one
// fe_mul / fe_sq / fe_sq_wide each, with the verify kernel's compile flags.
// tools/isa/isa_classes.py classifies them (profiles/r04/verify_isa_classes.txt).
#include <hip/hip_runtime.h>

#include "../../narwhal-tusk_amd/csrc/ge25519.hpp"

namespace nt {
__global__ void isa_fe_mul(uint32_t* io, int n) {
  fe a, b;
  for (int i = 0; i < 10; ++i) { a.v[i] = io[threadIdx.x * 20 + i]; b.v[i] = io[threadIdx.x * 20 + 10 + i]; }
#pragma unroll 1
  for (int k = 0; k < n; ++k) fe_mul(a, a, b);
  for (int i = 0; i < 10; ++i) io[threadIdx.x * 20 + i] = a.v[i];
}
__global__ void isa_fe_sq(uint32_t* io, int n) {
  fe a;
  for (int i = 0; i < 10; ++i) a.v[i] = io[threadIdx.x * 10 + i];
#pragma unroll 1
  for (int k = 0; k < n; ++k) fe_sq(a, a);
  for (int i = 0; i < 10; ++i) io[threadIdx.x * 10 + i] = a.v[i];
}
// a projective doubling + conversion (the ladder's inner loop: ge_dbl_p2)
__global__ void isa_dbl_p2(uint32_t* io, int n) {
  ge_p2 p;
  for (int i = 0; i < 10; ++i) { p.X.v[i] = io[threadIdx.x * 30 + i]; p.Y.v[i] = io[threadIdx.x * 30 + 10 + i]; p.Z.v[i] = io[threadIdx.x * 30 + 20 + i]; }
#pragma unroll 1
  for (int k = 0; k < n; ++k) ge_dbl_p2(p, p);
  for (int i = 0; i < 10; ++i) { io[threadIdx.x * 30 + i] = p.X.v[i]; io[threadIdx.x * 30 + 10 + i] = p.Y.v[i]; io[threadIdx.x * 30 + 20 + i] = p.Z.v[i]; }
}
}  // namespace nt
