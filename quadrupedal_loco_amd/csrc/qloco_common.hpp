// qloco_common.hpp -- shared device helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qloco.h"

#define QLOCO_WAVE 64

// grouped force-QP dispatch (qloco_force.hip): 5 swing-leg patterns x 16
// iteration bins; the ordering workspace is 2 B + 2 kForceClasses int32
#define QLOCO_FORCE_CLASSES 80

namespace qloco {

// thread-local last HIP error (qloco_last_error)
void set_last_error(const char *where, hipError_t e);
// the same with a library message instead of a HIP error (RCCL, dlopen)
void set_last_error_msg(const char *where, const char *what);

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Make a value provably wave-uniform (SGPR) so branches on it stay scalar.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// OSQP limit_scaling (scaling.c): < MIN_SCALING -> 1, > MAX_SCALING -> MAX
__device__ __forceinline__ float limit_scaling(float d) {
  d = d < 1e-4f ? 1.0f : d;
  return d > 1e4f ? 1e4f : d;
}

}  // namespace qloco

#define QLOCO_HIP_CHECK(call, where)                   \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) {                            \
      qloco::set_last_error(where, _e);                \
      return QLOCO_ERR_DEVICE;                         \
    }                                                  \
  } while (0)
