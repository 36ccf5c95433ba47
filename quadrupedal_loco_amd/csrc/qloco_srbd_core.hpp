// qloco_srbd_core.hpp -- definitions shared by the SRBD kernel translation
// units (qloco_srbd.hip: the stance-only and two-wave / wide classes;
// qloco_srbd_lit.hip: the literal QP through the wrench space).
#pragma once
#include <stdint.h>

#include <type_traits>

#include "qloco_common.hpp"
#include "qloco_dpp.inc"

namespace qloco {

struct SrbdArgs {
  int N, feet_per_step, contacts_per_step, output_frame;
  float dt, mass;
  float inertia[9];
  float q2[13];  // 2 * q_weights (Q diagonal, ConvexMpc.cpp:18-24)
  float r2[12];  // 2 * r_weights (R diagonal, :38-45)
  float mu, fz_min, fz_max;
  float rho, sigma, alpha, eps_abs, eps_rel;
  int max_iter, check_termination, scaling, adaptive_rho, rho_interval;
  float rho_tol;
  int warm_start;
  // 1: the reference's full 12N-variable QP (every (step, leg) pair is a
  // variable; swing legs held by fz in [0, 0] rows), 0: stance-only reduction
  int literal;
  // instances with nlegs outside [leg_lo, leg_hi] belong to the other
  // launch of a split batch (qloco_srbd_solve_ex) and are skipped
  int leg_lo, leg_hi;
  int64_t batch;
  const float *x0, *xref, *feet;
  const uint8_t *contacts;
  float *u0, *u, *obj, *warm;
  int *status, *iters, *rho_updates;
  // optional instance list (positions 0..count-1 -> instance ids) and its
  // device-side length (qloco_srbd_solve_ex's class lists)
  const int *list;
  const int *count;
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// One register row of K / K^-1; every index is static after unrolling, so
// SROA keeps it in VGPRs.
template <int W>
struct Row {
  float k[64 * W];
};
#define KE(K, c) ((K).k[(c)])

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF,
                                                            0xF, false));
}
// Compile-time loop over columns C..E-1 (the DPP control of a column's
// broadcast must be a constant expression).
template <int C, int E>
struct ColLoop {
  template <class F>
  static __device__ __forceinline__ void run(F &&f) {
    f(std::integral_constant<int, C>{});
    ColLoop<C + 1, E>::run(f);
  }
};
template <int E>
struct ColLoop<E, E> {
  template <class F>
  static __device__ __forceinline__ void run(F &&) {}
};
// Column c of a 60-vector read as one 16-byte chunk per lane (lane l holds
// elements 4(l % 16) .. +3): DPP row_newbcast:(c / 4) of component c % 4.
template <int C>
__device__ __forceinline__ float dpp_col(const f4v &d) {
  constexpr int e = C & 3;
  const float v = e == 0 ? d.x : (e == 1 ? d.y : (e == 2 ? d.z : d.w));
  return dpp<0x150 + (C >> 2)>(v);
}

__device__ __forceinline__ float lane_prev(float v) { return dpp<0x138>(v); }  // wave_shr:1
__device__ __forceinline__ float lane_next(float v) { return dpp<0x130>(v); }  // wave_shl:1
__device__ __forceinline__ float rlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// Wave-uniform max / sum over 64 lanes: DPP within 16-lane rows, then the
// four row results combined in a fixed order (deterministic).
__device__ __forceinline__ float wmax(float v) {
  v = fmaxf(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp<0x124>(v));  // row_ror:4
  v = fmaxf(v, dpp<0x128>(v));  // row_ror:8
  return fmaxf(fmaxf(rlane(v, 0), rlane(v, 16)), fmaxf(rlane(v, 32), rlane(v, 48)));
}
__device__ __forceinline__ float wsum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x124>(v);
  v += dpp<0x128>(v);
  return (rlane(v, 0) + rlane(v, 16)) + (rlane(v, 32) + rlane(v, 48));
}

// Block-wide reductions (wave-uniform results).
// Wave max of a NON-NEGATIVE float: the bits order like unsigned integers,
// so v_max_u32_dpp does each step in one op (no NaN canonicalisation): the
// four in-row steps, then row_bcast:15 / row_bcast:31 fold the rows into lane
// 63 (gfx9 DPP), read once.
#define QL_DMAXU(U, CTRL)                                                       \
  asm("s_nop 1\n\tv_max_u32_dpp %0, %0, %0 " CTRL " bank_mask:0xf" : "+v"(U))
__device__ __forceinline__ float wmax_nonneg(float v) {
  unsigned u = __builtin_bit_cast(unsigned, v);
  QL_DMAXU(u, "quad_perm:[1,0,3,2] row_mask:0xf");
  QL_DMAXU(u, "quad_perm:[2,3,0,1] row_mask:0xf");
  QL_DMAXU(u, "row_ror:4 row_mask:0xf");
  QL_DMAXU(u, "row_ror:8 row_mask:0xf");
  QL_DMAXU(u, "row_bcast:15 row_mask:0xa");  // rows 1, 3 += rows 0, 2
  QL_DMAXU(u, "row_bcast:31 row_mask:0xc");  // rows 2, 3 += lane 31
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(u, 63));
}

// K0 / K2 horizon sums (exact small integers in fp32).
__device__ __forceinline__ void k0k2(float ja, float jb, float Nf, float &K0, float &K2) {
  const float M = fmaxf(ja, jb);
  const float T = Nf - M;
  const float al = M - ja, be = M - jb;
  const float S1 = 0.5f * T * (T - 1.0f);
  const float S2 = rintf(S1 * (2.0f * T - 1.0f) * (1.0f / 3.0f));
  K0 = T;
  K2 = S2 + (al + be) * S1 + al * be * T;
}

// Gauss-Jordan: pivots above this get their column written exactly (qloco_srbd.hip)
constexpr float kGjExactPivot = 16.0f;

// the literal QP for N <= kLitN through the wrench space (qloco_srbd_lit.hip)
constexpr int kLitN = 10;
int srbd_lit_launch(const SrbdArgs &a, bool warm, hipStream_t stream);

}  // namespace qloco
