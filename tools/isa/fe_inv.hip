// ISA probe (compiled only, never launched): the key-cache batch inversion
// (fe_inv_vt.hpp) in a loop, so its inner-step and outer-iteration bodies can
// be counted in the gfx950 assembly (tools/isa/isa_classes.py loops).
#include <hip/hip_runtime.h>

#include "../../narwhal-tusk_amd/csrc/fe_inv_vt.hpp"

namespace nt {
__global__ void isa_fe_invert_vt(uint32_t* io, int n) {
  fe a;
  for (int i = 0; i < 10; ++i) a.v[i] = io[threadIdx.x * 10 + i];
#pragma unroll 1
  for (int k = 0; k < n; ++k) fe_invert_vt(a, a);
  for (int i = 0; i < 10; ++i) io[threadIdx.x * 10 + i] = a.v[i];
}
}  // namespace nt
