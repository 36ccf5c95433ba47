// qloco_gi.hip -- batched Goldfarb-Idnani dual active-set QP for gfx950.
//
// Replaces QPsolver_EiQuadProg::solve -> Eigen::QP::solve_quadprog
// (rt_mpc_qp/src/QP/QPBaseClass.cpp:36-58, utils/EiQuadProg/EiQuadProg.cpp:
// 4-513) for the small QPs of the hot path: the Go1 force QP (n = 12,
// p = 12, m = 24; dynmics_compute.cpp:265-445) and the body-inclination QP
// (n = 8, p = 0, m = 48; PRMPCClass.cpp:799-849).
//
// Mapping (this generic kernel): one QP instance per 16-lane group, four per
// wavefront (one wavefront per workgroup); the force and body kernels use
// 8-lane groups (qloco_gi_core.hpp: the results do not depend on the width).
// J, R (packed) and the vectors live in LDS, s(x) and the active-set
// snapshots in registers; lane i of a group owns row/column/constraint
// i, i + GW, ... in the vector steps.  Control flow is
// the reference's goto machine (l1/l2/l2a), uniform inside a group; groups
// of one wave may diverge (exec masking).  Double precision, compiled with
// -ffp-contract=off, and every dot product is summed by ONE lane in the
// reference's index order, so the arithmetic is the restatement's
// (oracle/eiquadprog.c) operation for operation -- active-set decisions and
// results agree bit for bit in the common case (tests/test_qp_gpu.py).
//
// The index quirks of the reference are kept: me = p
// counts skipped zero CE columns, equality markers are stored at A(i), the
// l1 / t1 loops start at me, and delete_constraint searches from p.  Where
// the reference would read an uninitialised index the instance reports
// QLOCO_UB_PATH instead of guessing.
#include <string.h>

#include "qloco_gi_core.hpp"
#include "qloco_gi_wide.hpp"

namespace qloco {

__global__ __launch_bounds__(64) void gi_kernel(const GiArgs a) {
  __shared__ GiLds lds[GI_GROUPS];
  const int lane = threadIdx.x;
  const int grp = lane >> 4;
  const int li = lane & 15;
  const int64_t inst = (int64_t)blockIdx.x * GI_GROUPS + grp;
  if (inst >= a.batch) return;  // whole group leaves together
  double f;
  int st, it;
  gi_solve_group(lds[grp], li, a.n, a.p, a.m, a.G + inst * a.sG, a.n, a.g0 + inst * a.sg0,
                 a.CE ? a.CE + inst * a.sCE : nullptr, a.ce0 ? a.ce0 + inst * a.sce0 : nullptr,
                 a.CI ? a.CI + inst * a.sCI : nullptr, a.ci0 ? a.ci0 + inst * a.sci0 : nullptr,
                 a.x + inst * a.n, f, st, it);
  if (li == 0) {
    if (a.f) a.f[inst] = f;
    if (a.status) a.status[inst] = st;
    if (a.iters) a.iters[inst] = it;
  }
}

}  // namespace qloco

using namespace qloco;

// the fast path's variable limit (four QPs per wavefront, gi_kernel) -- what
// this query has always meant; the capacity limits are qloco_gi_limits
extern "C" int qloco_max_gi_vars(void) { return GI_N; }

extern "C" void qloco_gi_fast_limits(int32_t *n, int32_t *p, int32_t *m) {
  if (n) *n = GI_N;
  if (p) *p = GI_P;
  if (m) *m = GI_M;
}

extern "C" void qloco_gi_limits(int32_t *n, int32_t *p, int32_t *m) {
  if (n) *n = kGiWideN;
  if (p) *p = kGiWideP;
  if (m) *m = kGiWideM;
}

extern "C" int qloco_eiquadprog_solve(int32_t n, int32_t p, int32_t m, int64_t batch,
                                      const double *G, int64_t G_stride, const double *g0,
                                      int64_t g0_stride, const double *CE, int64_t CE_stride,
                                      const double *ce0, int64_t ce0_stride, const double *CI,
                                      int64_t CI_stride, const double *ci0, int64_t ci0_stride,
                                      double *x, double *f, int32_t *status, int32_t *iters,
                                      void *stream) {
  if (n < 1 || n > kGiWideN || p < 0 || p > kGiWideP || m < 0 || m > kGiWideM)
    return QLOCO_BAD_SIZE;
  if (batch < 0 || !G || !g0 || !x) return QLOCO_ERR_ARG;
  if ((p > 0 && (!CE || !ce0)) || (m > 0 && (!CI || !ci0))) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  // the small QPs of the hot path (force QP 12/12/24, body QP 8/0/48): four
  // per wavefront; anything larger up to QPBaseClass's capacity: one per
  // wavefront (qloco_gi_wide.hip)
  if (n > GI_N || p > GI_P || m > GI_M)
    return gi_wide_launch(n, p, m, batch, G, G_stride, g0, g0_stride, CE, CE_stride, ce0,
                          ce0_stride, CI, CI_stride, ci0, ci0_stride, x, f, status, iters,
                          (hipStream_t)stream);
  GiArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.p = p;
  a.m = m;
  a.batch = batch;
  a.G = G;
  a.g0 = g0;
  a.CE = CE;
  a.ce0 = ce0;
  a.CI = CI;
  a.ci0 = ci0;
  a.sG = G_stride;
  a.sg0 = g0_stride;
  a.sCE = CE_stride;
  a.sce0 = ce0_stride;
  a.sCI = CI_stride;
  a.sci0 = ci0_stride;
  a.x = x;
  a.f = f;
  a.status = status;
  a.iters = iters;
  const unsigned blocks = (unsigned)((batch + GI_GROUPS - 1) / GI_GROUPS);
  hipLaunchKernelGGL(gi_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "gi_kernel launch");
  return QLOCO_OK;
}
