// qloco_gi_wide.hpp -- host-side entry of the wide Goldfarb-Idnani kernel
// (qloco_gi_wide.hip), used by qloco_eiquadprog_solve's size dispatch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qloco {

// the reference's QPBaseClass capacity (QPBaseClass.h:49-51: MAX_VARS 60,
// MAX_N_INEQ 300), rounded up to the wavefront / a 64-multiple
constexpr int kGiWideN = 64;
constexpr int kGiWideP = 64;
constexpr int kGiWideM = 320;

int gi_wide_launch(int n, int p, int m, int64_t batch, const double *G, int64_t sG,
                   const double *g0, int64_t sg0, const double *CE, int64_t sCE,
                   const double *ce0, int64_t sce0, const double *CI, int64_t sCI,
                   const double *ci0, int64_t sci0, double *x, double *f, int32_t *status,
                   int32_t *iters, hipStream_t stream);

}  // namespace qloco
