// qloco_srbd_lit.hip -- the reference's LITERAL 12N-variable SRBD QP for
// N <= 20 (every (step, leg) pair an ADMM variable, swing legs held by their
// fz in [0, 0] rows: A1RobotControl.cpp:557-578, ConvexMpc.cpp:162-264),
// the OSQP linear solve through the per-step wrench space, one wavefront per
// instance for N <= 10 and two for 11 <= N <= 20 (dispatched by
// qloco_srbd_solve_ex, qloco_srbd.hip).
//
// Why the wrench space.  The forces enter the SRBD dynamics
// only through each step's wrench increment w_j = Bb u_j (Bb: the omega / v
// rows of B_d, 6 x 12), so the condensed Hessian is H = Vu' G Vu + R with
// Vu = I_N (x) Bb and G = K0 (x) Qb + K2 (x) Te (6N x 6N, the closed-form
// horizon sums of DESIGN.md §3).  OSQP's reduced KKT matrix factors as
//   K = P~ + sigma I + A~' rho A~ = D [c Vu' G Vu + W0] D,
//   W0 = c R + D^-1 (sigma I + A~' rho A~) D^-1   (3 x 3 per (step, leg)),
// and by the push-through identity
//   K^-1 b = D^-1 (a - W0^-1 Vu' T Vu a),  a = W0^-1 D^-1 b,
//   T = (I + cG U)^-1 cG = (cG) L S^-1 L^-1   (symmetric, 6N x 6N),
//   U = Vu W0^-1 Vu' = L L' (6 x 6 per step),  S = I + L' (cG) L  (SPD, >= I).
// The 12N-variable KKT inverse becomes a 6N x 6N inverse of the
// well-conditioned S (eigenvalues >= 1, so pivot-free Gauss-Jordan is
// stable) plus a 6N x 6N product, and each ADMM iteration a 6N x 6N matvec
// plus leg-local 3 x 3 blocks and per-step wrench sums.  Same arithmetic as
// OSQP up to rounding (tools/proto_lit.py: float64 iterates agree to 1e-10,
// a float32 solve to 4e-7 relative; iteration counts equal on every instance
// tried).
//
// Lane layout (template W = waves per instance).  Wave w holds the steps
// [w H, w H + N_w) (W = 1: H = N_0 = N; W = 2: H = ceil(N / 2), N_1 = N - H,
// at most 10 steps a wave), laid out exactly as the one-wave kernel lays out
// its N <= 10 steps: lane l holds two variables (slot h = 0, 1: local
// v = 60 h + l, l < 60; step w H + v / 12, leg (v % 12) / 3, component
// v % 3 -- leg triples never straddle), their <= 2 constraint rows each,
// and wrench row l (step w H + l / 6, component l % 6: 0..2 omega, 3..5 v).
// Everything leg- or step-local stays inside a wave; the couplings across
// steps (the K0 / K2 horizon sums, the rows of S and T, the matvec with T)
// run in a "column space" of W halves of 60 (half w' = wave w''s wrench rows),
// so a lane's row of S / T is 60 W registers and the Gauss-Jordan and the
// matvec are W of the one-wave kernel's 60-column DPP forms.
#include <math.h>
#include <stddef.h>

#include <type_traits>

#include "qloco_srbd_core.hpp"

namespace qloco {

constexpr int kLitWpe = 4;   // one wave:  waves per SIMD: 128 VGPRs, <= 10 KB of LDS (static_assert below)
constexpr int kLit2Wpe = 2;  // two waves: 256 VGPRs (a 120-register row of S / T per lane)

template <int W>
struct LitLds {
  // steps the per-step loops unroll over; the per-step tables (K0 / K2, Ruiz
  // column scales) are indexed by COLUMN-SPACE step 10 w' + kl
  // (wave w''s local step kl; two waves: the steps past a wave's N_w are
  // padding with zero K0 / K2 weights), so every table index in the unrolled
  // loops is a compile-time constant plus the wave's offset
  static constexpr int NS = W == 1 ? kLitN : kLitN2;
  static constexpr int NT = NS;
  f4v bc[W][W][16];         // broadcast rows: 60-vectors read as one 16-B chunk per lane, [parity][half]
                            // (one wave: its LDS ops run in order, so one buffer serves every reuse;
                            // two waves: double-buffered by iteration / pivot parity, one barrier each)
  float av[W][2][64];       // per wave, per slot exchange (a, D x, t)
  float wv[W][64];          // per wave, wrench rows (s, w)
  f2v k0k2[NT][NT];         // horizon sums K0 / K2 (row step, column step; column-space steps)
  float Bb[6][12];          // wrench map (constant feet), rows omega 0..2, v 3..5
  float Te[6][6];           // dt^2 blockdiag(Rz' Qtheta Rz, Qp)
  float q2[16], r2[12], x0[16];
  float ctf[4 * NT];        // contact flags as floats
  f4v arz[W][2][64];        // per slot: scaled A entries (ra0, ra1, rz0, rz1)
  float zh[W][2][64];       // per slot: row 0's scaled upper bound (x / y rows: inf); the lower
                            // bound is 0 (x / y) or zh fz_min / fz_max (z rows)
  float dr[W][2][64];       // per slot: the Ruiz column scale D (read where needed: not a
                            // register live across the ADMM loop)
  float qvl[W][2][64];      // per slot: the scaled gradient q~ (read where needed)
  // block-uniform solver state, one copy per wave (both waves take identical
  // decisions): read into SGPRs where a phase needs it, so no register carries
  // it across the ADMM iterations
  struct {
    float rho, cs, cinv, qn0, qn1, alpha, oma, sigma, dtm;
    float sxy[2][2];  // S of the omega x / y block: G^-1 = sum_a S[.][a] A_a^-1 S[.][a] (see the G^-1 tables)
    int iter, status, rho_updates, ctm, interval;
  } sc[W];
  union alignas(16) {       // phase-local storage (LDS bounds the one-wave occupancy: <= 10 KB;
                            // 16-byte aligned: dcol is read as f4v, a misaligned ds_read_b128
                            // cost the one-wave kernel 46 us per launch)
    struct {                // gradient + Ruiz
      f2v beps[12][12];     // (beta, eps)[w][w']: the P entries' per-column coefficients
      float dcol[12 * NT];  // Ruiz column scales D (read as same-address broadcasts)
      float err[12 * NT];   // gradient scans
      float Wc[12 * NT];
    };
    struct {                // factorisation
      float w0i[W][3][2][64];   // per variable its row of W0^-1 (x, y, z), read by the U rows
      f2v gtab[NT][NT][3];      // G^-1 blocks: per (row step, column step) in
                                // column-space order, (W0, W1), (W2, V0), (V1, V2)
    };
  };
  float piv[W == 1 ? 0 : 2];       // two waves: the Gauss-Jordan pivot, [parity]
  float red[W == 1 ? 0 : 2][16];   // two waves: per-wave partials of the block reductions
};
static_assert(sizeof(LitLds<1>) <= 10240, "literal kernel: four workgroups per SIMD need <= 160 KB / 16 of LDS");
static_assert(sizeof(LitLds<2>) <= 40960, "two-wave literal kernel: four workgroups per CU need <= 40 KB");
static_assert(offsetof(LitLds<1>, dcol) % 16 == 0 && offsetof(LitLds<2>, dcol) % 16 == 0,
              "dcol is read as f4v (ds_read_b128 needs 16-byte alignment)");

// Wave-level helpers for the one-wave literal kernel
__device__ __forceinline__ void lsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// the instance's workgroup: a wave barrier for one wave, s_barrier for two
template <int W>
__device__ __forceinline__ void bsync() {
  if constexpr (W == 1)
    lsync();
  else
    __syncthreads();
}

// Block-wide combination of W wave-uniform partials (fixed order: every wave
// computes the same value bit for bit, so the loop control stays uniform)
template <int W, int K>
__device__ __forceinline__ void bcombine_max(LitLds<W> &S, float (&v)[K], int wv) {
  if constexpr (W == 2) {
    static_assert(K <= 16, "red holds 16 partials per wave");
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) S.red[wv][k] = v[k];
    }
    bsync<W>();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = fmaxf(S.red[0][k], S.red[1][k]);
    bsync<W>();
  }
}
template <int W>
__device__ __forceinline__ float bsum(LitLds<W> &S, float v, int wv) {
  if constexpr (W == 2) {
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) S.red[wv][0] = v;
    bsync<W>();
    v = S.red[0][0] + S.red[1][0];
    bsync<W>();
  }
  return v;
}
template <int W>
__device__ __forceinline__ float bmax1(LitLds<W> &S, float v, int wv) {
  float t[1] = {v};
  bcombine_max<W, 1>(S, t, wv);
  return t[0];
}

// The three entries of this lane's leg triple (components 0, 1, 2) of a
// per-lane value: lanes 3m, 3m+1, 3m+2 hold one leg.
struct Triple {
  float v0, v1, v2;
};
__device__ __forceinline__ Triple triple(float v, int comp) {
  const float n1 = lane_next(v), n2 = lane_next(n1);
  const float p1 = lane_prev(v), p2 = lane_prev(p1);
  Triple t;
  t.v0 = comp == 0 ? v : (comp == 1 ? p1 : p2);
  t.v1 = comp == 0 ? n1 : (comp == 1 ? v : p1);
  t.v2 = comp == 0 ? n2 : (comp == 1 ? n1 : v);
  return t;
}

// A leg-triple dot product sum_j a_j v(leg, j) as lane shifts d = j - comp:
// v(l + d) with coefficient c_d (zero where l + d leaves the leg), five fused
// multiply-adds with DPP operands instead of the triple's 4 moves + 6 selects
// + 3 multiply-adds.
struct Shift5 {
  float cm2, cm1, c0, cp1, cp2;
};
__device__ __forceinline__ Shift5 shift5(float a0, float a1, float a2, int comp) {
  Shift5 c;
  c.c0 = comp == 0 ? a0 : (comp == 1 ? a1 : a2);
  c.cm1 = comp == 1 ? a0 : (comp == 2 ? a1 : 0.0f);
  c.cm2 = comp == 2 ? a0 : 0.0f;
  c.cp1 = comp == 0 ? a1 : (comp == 1 ? a2 : 0.0f);
  c.cp2 = comp == 0 ? a2 : 0.0f;
  return c;
}
__device__ __forceinline__ float tdot(float v, const Shift5 &c) {
  float a, t, u;
  asm("s_nop 1\n\t"
      "v_mov_b32_dpp %1, %3 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
      "v_mov_b32_dpp %2, %3 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
      "v_mul_f32 %0, %3, %4\n\t"
      "v_fmac_f32_dpp %0, %3, %5 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
      "v_fmac_f32_dpp %0, %3, %7 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
      "v_fmac_f32_dpp %0, %1, %6 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
      "v_fmac_f32_dpp %0, %2, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
      : "=&v"(a), "=&v"(t), "=&v"(u)
      : "v"(v), "v"(c.c0), "v"(c.cm1), "v"(c.cm2), "v"(c.cp1), "v"(c.cp2));
  return a;
}

// In-place Gauss-Jordan inverse of the 60 x 60 SPD S (one row per lane,
// pivots <= 1 after the 1/max-diagonal scaling): invert_w1's scheme (DESIGN.md
// §3) with one pivot of look-ahead -- pivot k first applies its update to
// column k + 1 alone (the same fused multiply-add the full update performs,
// so bit-identical) and publishes pivot k + 1's broadcast row, then runs the
// other 59 columns while that LDS write is in flight.
__device__ __forceinline__ void lit_invert(LitLds<1> &S, int lane, int ncol, Row<1> &K) {
  int nc = __builtin_amdgcn_readfirstlane(ncol);
  {
    const float v = K.k[0];
    const float p = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    reinterpret_cast<float *>(&S.bc[0][0][0])[lane] = lane == 0 ? p + 1.0f : v;
  }
  ColLoop<0, 60>::run([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    asm volatile("" : "+s"(nc));
    if (k >= nc) return;
    const int tt = fresh_lane();
    lsync();
    const f4v r0 = S.bc[0][0][lane & 15];
    const float v = K.k[k];
    const float p = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
    const float pinv = __builtin_amdgcn_rcpf(p);
    const float ng = -((tt == k) ? (1.0f - pinv) : v * pinv);
    if constexpr (k + 1 < 60) {  // unconditional (harmless past the last pivot): no branch to join
      const float la = fmaf(dpp_col<k + 1>(r0), ng, K.k[k + 1]);
      const float p1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, la), k + 1));
      reinterpret_cast<float *>(&S.bc[0][0][0])[tt] = (tt == k + 1) ? p1 + 1.0f : ((tt < k + 1) ? -la : la);
    }
    QL_DPP_GJ60(K.k, 0, r0, ng);
    if (p > kGjExactPivot) K.k[k] = (tt == k) ? pinv : ng;
  });
  lsync();
}

// The two-wave form: S is (60 + 60) x (60 + 60) in column space (wave w's
// rows are rows 60 w .. 60 w + 59, its first nc_w valid), one row of 120
// registers per lane.  Each pivot publishes its column (the pivot row up to
// the Gauss-Jordan signs) from both waves into the parity buffer, one
// workgroup barrier, then both halves take the one-wave DPP update.  The
// look-ahead publishes the next pivot's column before the 120-column update,
// so the barrier never waits on that write; the pivot value itself travels
// through LDS (the other wave cannot read the owner's register).
//
// Pivot order: LAST step first (half 1 from its last valid row down, then
// half 0).  S's early steps carry the largest horizon weights (K0 = N - j,
// K2 ~ (N - j)^3 / 3): eliminating them first, as the one-wave kernel's
// natural order does, grows the error of the pivot-free fp32 Gauss-Jordan
// past what ADMM tolerates at N = 16 / 20 and small rho (57 + 4 of 65,536
// N = 16 trot instances ended at max_iter / solved-inaccurate; the float32
// emulation, tools/proto_lit_fused.py, reproduces it and converges with the
// reversed order on every one of them).
template <int HF, int KL>
__device__ __forceinline__ void lit2_pivot(LitLds<2> &S, int wv, int nc, Row<2> &K) {
  const int tt = fresh_lane();
  if constexpr (KL >= 1) {
    if (KL == nc) {  // the half's first pivot (column KL - 1): a plain publish
      constexpr int k1 = 60 * HF + KL - 1;
      const float v = K.k[k1];
      const bool own1 = wv == HF && tt == KL - 1;
      const bool before = HF == 0 && wv == 1;  // half 1 is done when half 0 starts
      reinterpret_cast<float *>(&S.bc[k1 & 1][wv][0])[tt] = own1 ? v + 1.0f : (before ? -v : v);
      if (own1) S.piv[k1 & 1] = v;
    }
  }
  if constexpr (KL < 60) {
    constexpr int k = 60 * HF + KL;
    constexpr int pb = k & 1;
    if (KL >= nc) return;
    bsync<2>();
    const f4v r0 = S.bc[pb][0][tt & 15];
    const f4v r1 = S.bc[pb][1][tt & 15];
    const float p = S.piv[pb];
    const float v = K.k[k];
    const float pinv = __builtin_amdgcn_rcpf(p);
    const bool own = wv == HF && tt == KL;
    const float ng = -(own ? (1.0f - pinv) : v * pinv);
    if constexpr (KL >= 1) {  // look-ahead: the next pivot is column k - 1 of this half
      const float la = fmaf(dpp_col<KL - 1>(HF ? r1 : r0), ng, K.k[k - 1]);
      const bool own1 = wv == HF && tt == KL - 1;
      const bool before = HF ? (wv == 1 && tt >= KL) : (wv == 1 || tt >= KL);
      reinterpret_cast<float *>(&S.bc[pb ^ 1][wv][0])[tt] = own1 ? la + 1.0f : (before ? -la : la);
      if (own1) S.piv[pb ^ 1] = la;
    }
    QL_DPP_GJ60(K.k, 0, r0, ng);
    QL_DPP_GJ60(K.k, 60, r1, ng);
    if (p > kGjExactPivot) K.k[k] = own ? pinv : ng;
  }
}

__device__ __forceinline__ void lit_invert2(LitLds<2> &S, int wv, int nc0, int nc1, Row<2> &K) {
  nc0 = __builtin_amdgcn_readfirstlane(nc0);
  nc1 = __builtin_amdgcn_readfirstlane(nc1);
  ColLoop<0, 61>::run([&](auto kc) {  // half 1, KL = 60 .. 0
    asm volatile("" : "+s"(nc1));
    lit2_pivot<1, 60 - decltype(kc)::value>(S, wv, nc1, K);
  });
  ColLoop<0, 61>::run([&](auto kc) {  // half 0
    asm volatile("" : "+s"(nc0));
    lit2_pivot<0, 60 - decltype(kc)::value>(S, wv, nc0, K);
  });
  bsync<2>();
}

// Lane-derived indices re-derived from an opaque copy of the lane at the top
// of a phase: the address arithmetic on them is then recomputed there (a few
// VALU) instead of hoisted to the kernel entry and kept live -- at 128 VGPRs
// the hoisted offsets were the setup's scratch spills.  jr / stepl: the
// wave-local step (per-wave LDS rows); step: the global step (the
// gradient, the contact flags, the persistent record); jc: the column-space
// step (the horizon tables: 10 w + jr).  Padding lanes sit on steps whose
// K0 / K2 weights are zero.
#define QL_LIT_LANE_INDICES(LX)                                                                    \
  const int LX = fresh_lane();                                                                     \
  const int jr = LX < 60 ? LX / 6 : kLitN - 1, sr = LX < 60 ? LX - 6 * (LX / 6) : 0;               \
  const int jc = W == 1 ? jr : 10 * wv + jr;                                                       \
  const bool wvalid = LX < nw;                                                                     \
  const int step[2] = {LX < 60 && LX < nvl ? so + LX / 12 : so, LX < 60 && 60 + LX < nvl ? so + (60 + LX) / 12 : so}; \
  const int stepl[2] = {step[0] - so, step[1] - so};                                               \
  const int leg[2] = {LX < 60 && LX < nvl ? (LX % 12) / 3 : 0, LX < 60 && 60 + LX < nvl ? ((60 + LX) % 12) / 3 : 0}; \
  const int comp = LX % 3;                                                                         \
  const bool xy = comp < 2;                                                                        \
  const bool valid[2] = {LX < 60 && LX < nvl, LX < 60 && 60 + LX < nvl};                           \
  (void)jr; (void)sr; (void)jc; (void)wvalid; (void)stepl; (void)step; (void)leg; (void)comp; (void)xy; (void)valid

// WS: a warm-start mode (1 or 2) may be set (the persistent record of
// DESIGN.md §3c, literal semantics: the update path on every call).
template <int W, bool WS>
__device__ __forceinline__ void srbd_lit_one(const SrbdArgs &a, LitLds<W> &S, const int64_t b) {
  constexpr int NS = LitLds<W>::NS, NT = LitLds<W>::NT;
  const int lane = W == 1 ? (int)threadIdx.x : (int)(threadIdx.x & 63);
  const int tid = threadIdx.x;
  const int wv = W == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int N = a.N;
  const float Nf = (float)N;
  const float dt = a.dt;
  const float dtm = dt / a.mass, dt2m = dt * dt / a.mass;
  // this wave's steps: [so, so + Nw) (W = 1: all N)
  const int H = W == 1 ? N : (N + 1) / 2;
  const int so = W == 1 ? 0 : wv * H;
  const int Nw = W == 1 ? N : (wv ? N - H : H);
  const int nvar = 12 * N, nvl = 12 * Nw, nw = 6 * Nw;

  // ---------------- 1. inputs -> LDS
  if (tid < 13) S.x0[tid] = a.x0[b * 13 + tid];
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 13; ++k) S.q2[k] = a.q2[k];
#pragma unroll
    for (int k = 0; k < 12; ++k) S.r2[k] = a.r2[k];
  }
  {
    const int nct = a.contacts_per_step ? 4 * N : 4;
    if (tid < 4 * N) S.ctf[tid] = a.contacts[b * nct + (a.contacts_per_step ? tid : (tid & 3))] ? 1.0f : 0.0f;
  }
  for (int idx = tid; idx < NT * NT; idx += 64 * W) {
    const int sr = idx / NT, sc = idx - NT * sr;
    float K0 = 0.0f, K2 = 0.0f;
    if constexpr (W == 1) {
      if (sr < N && sc < N) k0k2((float)sr, (float)sc, Nf, K0, K2);
    } else {  // column-space steps -> global steps (-1: padding)
      const int gr = sr % 10 < (sr >= 10 ? N - H : H) ? (sr >= 10 ? H : 0) + sr % 10 : -1;
      const int gc = sc % 10 < (sc >= 10 ? N - H : H) ? (sc >= 10 ? H : 0) + sc % 10 : -1;
      if (gr >= 0 && gc >= 0) k0k2((float)gr, (float)gc, Nf, K0, K2);
    }
    S.k0k2[sr][sc] = (f2v){K0, K2};
  }
  if constexpr (W == 2) {  // Ruiz column scales of the padding steps stay 0
    for (int idx = tid; idx < 12 * NT; idx += 64 * W) S.dcol[idx] = 0.0f;
  }
  bsync<W>();

  // ---------------- 2. SRBD model (ConvexMpc.cpp:111-160, compute_grf :502-549)
  const float yaw = S.x0[2];
  const float cy = cosf(yaw), sy = sinf(yaw);
  const float R00 = cy, R01 = sy, R10 = -sy, R11 = cy;  // A1RobotControl.cpp:506-508
  float Ii[3][3];
  {
    const float *I = a.inertia;
    const float Rm[3][3] = {{R00, R01, 0.f}, {R10, R11, 0.f}, {0.f, 0.f, 1.f}};
    float RI[3][3], Iw[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        RI[r][c] = Rm[r][0] * I[c * 3 + 0] + Rm[r][1] * I[c * 3 + 1] + Rm[r][2] * I[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        Iw[r][c] = RI[r][0] * Rm[c][0] + RI[r][1] * Rm[c][1] + RI[r][2] * Rm[c][2];
    const float c00 = Iw[1][1] * Iw[2][2] - Iw[1][2] * Iw[2][1];
    const float c01 = Iw[1][2] * Iw[2][0] - Iw[1][0] * Iw[2][2];
    const float c02 = Iw[1][0] * Iw[2][1] - Iw[1][1] * Iw[2][0];
    const float id = 1.0f / (Iw[0][0] * c00 + Iw[0][1] * c01 + Iw[0][2] * c02);
    Ii[0][0] = c00 * id;
    Ii[1][0] = c01 * id;
    Ii[2][0] = c02 * id;
    Ii[0][1] = (Iw[0][2] * Iw[2][1] - Iw[0][1] * Iw[2][2]) * id;
    Ii[1][1] = (Iw[0][0] * Iw[2][2] - Iw[0][2] * Iw[2][0]) * id;
    Ii[2][1] = (Iw[0][1] * Iw[2][0] - Iw[0][0] * Iw[2][1]) * id;
    Ii[0][2] = (Iw[0][1] * Iw[1][2] - Iw[0][2] * Iw[1][1]) * id;
    Ii[1][2] = (Iw[0][2] * Iw[1][0] - Iw[0][0] * Iw[1][2]) * id;
    Ii[2][2] = (Iw[0][0] * Iw[1][1] - Iw[0][1] * Iw[1][0]) * id;
  }
  // per slot: the variable, its B_d column (omega rows: ba) and E column
  const int comp = lane % 3;
  const bool xy = comp < 2;
  bool valid[2];
  int step[2], leg[2], cst[2];  // global / column-space step
  f4v lo[2], hi[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int v = 60 * h + lane;
    valid[h] = lane < 60 && v < nvl;
    step[h] = valid[h] ? so + v / 12 : 0;
    cst[h] = W == 1 ? step[h] : (valid[h] ? 10 * wv + v / 12 : 0);
    leg[h] = valid[h] ? (v % 12) / 3 : 0;
    const float *rf = a.feet + b * 12 + 3 * leg[h];
    const float rx = rf[0], ry = rf[1], rz = rf[2];
    const float tv0 = comp == 0 ? 0.f : (comp == 1 ? -rz : ry);  // skew(r) e_comp (Utils.cpp:35-41)
    const float tv1 = comp == 0 ? rz : (comp == 1 ? 0.f : -rx);
    const float tv2 = comp == 0 ? -ry : (comp == 1 ? rx : 0.f);
    float ba[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) ba[r] = dt * (Ii[r][0] * tv0 + Ii[r][1] * tv1 + Ii[r][2] * tv2);
    lo[h] = (f4v){ba[0], ba[1], ba[2], dt * (R00 * ba[0] + R01 * ba[1])};
    hi[h] = (f4v){dt * (R10 * ba[0] + R11 * ba[1]), dt * ba[2], (float)step[h], (float)comp};
    if (!valid[h]) {
      lo[h] = (f4v)(0.0f);
      hi[h] = (f4v){0.0f, 0.0f, 0.0f, -1.0f};
    }
    // the wrench map (constant feet): column v % 12 of Bb from the step-0 lanes
    if (h == 0 && tid < 12) {
      S.Bb[0][lane] = ba[0];
      S.Bb[1][lane] = ba[1];
      S.Bb[2][lane] = ba[2];
      S.Bb[3][lane] = comp == 0 ? dtm : 0.0f;
      S.Bb[4][lane] = comp == 1 ? dtm : 0.0f;
      S.Bb[5][lane] = comp == 2 ? dtm : 0.0f;
    }
  }
  // Te = dt^2 blockdiag(Rz' diag(q2[0:3]) Rz, diag(q2[3:6]))
  if (tid < 36) {
    const int r = lane / 6, c = lane - 6 * (lane / 6);
    const float Rm[3][3] = {{R00, R01, 0.f}, {R10, R11, 0.f}, {0.f, 0.f, 1.f}};
    float v = 0.0f;
    if (r < 3 && c < 3)
      v = dt * dt * (Rm[0][r] * S.q2[0] * Rm[0][c] + Rm[1][r] * S.q2[1] * Rm[1][c] + Rm[2][r] * S.q2[2] * Rm[2][c]);
    else if (r >= 3 && c == r)
      v = dt * dt * S.q2[r];
    S.Te[r][c] = v;
  }
  float r2v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) r2v[h] = valid[h] ? S.r2[3 * leg[h] + comp] : 0.0f;

  // ---------------- 3. gradient g = Bqp' Q (Aqp x0 - x_ref) (ConvexMpc.cpp:219-221)
  for (int idx = tid; idx < 12 * N; idx += 64 * W) {
    const int i = idx / 12, s = idx - 12 * i;
    const float k = (float)(i + 1);
    const float *x0 = S.x0;
    float xf;
    if (s < 3) {
      const float rw = s == 0 ? (R00 * x0[6] + R01 * x0[7]) : (s == 1 ? (R10 * x0[6] + R11 * x0[7]) : x0[8]);
      xf = x0[s] + k * dt * rw;
    } else if (s < 6) {
      xf = x0[s] + k * dt * x0[s + 6];
      if (s == 5) xf += 0.5f * k * (k - 1.0f) * dt * dt * x0[12];
    } else if (s < 9) {
      xf = x0[s];
    } else {
      xf = x0[s] + (s == 11 ? k * dt * x0[12] : 0.0f);
    }
    S.err[idx] = S.q2[s] * (xf - a.xref[b * 13 * N + 13 * i + s]);
  }
  bsync<W>();
  if (tid < 12) {  // suffix scans per state row (row_scans of the two-wave kernel)
    const int r = lane;
    const bool brow = r >= 6;
    float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
    for (int j = NS - 1; j >= 0; --j) {
      if (j < N) {
        s1 += s0;
        s0 += S.err[12 * j + r];
        S.Wc[12 * j + r] = brow ? s0 : s1;
      }
    }
  }
  bsync<W>();
  float qv[2], qsv[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float g = 0.0f;
    if (valid[h]) {
      const float *w = S.Wc + 12 * step[h];
      g = lo[h].x * w[6] + lo[h].y * w[7] + lo[h].z * w[8];
      g += lo[h].w * w[0] + hi[h].x * w[1] + hi[h].y * w[2];
      g += dtm * w[9 + comp] + dt2m * w[3 + comp];
    }
    qv[h] = g;
    qsv[h] = g;
  }
  // from here on a variable's B_d column is all the iterations need of lo/hi:
  // its omega rows (the wrench map's torque part; the force part is dtm e_comp)
  // persistent solver (warm_start == 2): literal semantics -- after the
  // first call every call takes OSQP's update path
  const int NP = 100 * N;
  float *prec = (WS && a.warm_start == 2) ? a.warm + b * (int64_t)(NP + 4) : nullptr;
  bool p_init = false;
  if (prec) p_init = prec[NP + 1] > 0.5f;
  const bool p_same = p_init;
  if (p_same) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (valid[h]) qsv[h] = prec[84 * N + 12 * step[h] + 3 * leg[h] + comp];
  }
  if (prec) {  // the record's q for the next call, written now (each variable's own entry, just read)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (valid[h]) prec[84 * N + 12 * step[h] + 3 * leg[h] + comp] = qv[h];
  }

  // ---------------- 4. constraint rows owned by each slot (ConvexMpc.cpp:47-59, :227-249)
  float ra0[2], ra1[2], rz0[2], rz1[2], rl0[2], ru0[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    ra0[h] = valid[h] ? 1.0f : 0.0f;
    ra1[h] = (valid[h] && xy) ? 1.0f : 0.0f;
    rz0[h] = (valid[h] && xy) ? a.mu : 0.0f;
    rz1[h] = (valid[h] && xy) ? -a.mu : 0.0f;
    const float cflag = valid[h] ? S.ctf[4 * step[h] + leg[h]] : 0.0f;
    rl0[h] = !valid[h] ? 0.0f : (xy ? 0.0f : a.fz_min * cflag);
    ru0[h] = !valid[h] ? 0.0f : (xy ? INFINITY : a.fz_max * cflag);
  }

  // ---------------- 5. modified Ruiz equilibration (OSQP scaling.c), P rows
  // generated from the wrench structure: P[(j,w),(k,w')] = K0(j,k) beta[w][w']
  // + K2(j,k) eps[w][w'] + R delta, beta = <b_w, b_w'>_Qb, eps = <b_w, b_w'>_Te
  float rE0[2] = {1.0f, 1.0f}, rE1[2] = {1.0f, 1.0f}, Dr[2] = {1.0f, 1.0f}, cs = 1.0f;
  {
    // beta / eps tables (12 x 12, constant feet) in LDS: beta[w][w'] =
    // sum_s Qb_s Bb[s][w] Bb[s][w'], eps[w][w'] = Bb[:,w]' Te Bb[:,w']
    bsync<W>();
    for (int e = tid; e < 144; e += 64 * W) {
      const int w = e / 12, wp = e - 12 * (e / 12);
      float bb = 0.0f, ee = 0.0f;
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        bb = fmaf(S.q2[6 + s] * S.Bb[s][w], S.Bb[s][wp], bb);
        float tw = 0.0f;
#pragma unroll
        for (int t = 0; t < 6; ++t) tw = fmaf(S.Te[s][t], S.Bb[t][wp], tw);
        ee = fmaf(S.Bb[s][w], tw, ee);
      }
      S.beps[w][wp] = (f2v){bb, ee};
    }
    bsync<W>();
    // this lane's diagonal P entries (R included)
    float pdiag[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int wl = valid[h] ? (60 * h + lane) % 12 : 0;
      const f2v kk = S.k0k2[cst[h]][cst[h]];
      const f2v be = S.beps[wl][wl];
      pdiag[h] = valid[h] ? fmaf(kk.y, be.y, kk.x * be.x) + r2v[h] : 0.0f;
    }
    // this lane's (beta, eps) rows, per slot (registers for the whole of
    // Ruiz: every column step reuses them)
    float bet[2][12], eps[2][12];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int wl = h == 0 ? (valid[0] ? lane % 12 : 0) : (valid[1] ? (60 + lane) % 12 : 0);
#pragma unroll
      for (int w = 0; w < 12; ++w) {
        const f2v be = S.beps[wl][w];
        bet[h][w] = valid[h] ? be.x : 0.0f;
        eps[h][w] = valid[h] ? be.y : 0.0f;
      }
    }
    // row inf-norms |P_vc| D_c of both slots' rows in one sweep over the 12N
    // columns, step-major: per column step the K0 / K2 weights of the two
    // rows' steps and the step's 12 column scales (same-address LDS reads,
    // a broadcast), then 12 entries per row from the (beta, eps) rows
    auto row_norms = [&](bool scaled, float (&m)[2]) {
      // loop-invariant tables: opaque per call (no hoisting of all 240 entries)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int w = 0; w < 12; ++w) asm volatile("" : "+v"(bet[h][w]), "+v"(eps[h][w]));
      // both slots' rows as fp32 pairs (v_pk_fma / v_pk_mul), two max chains
      // each; the next column step's LDS reads are issued before this step's
      // arithmetic (one step of look-ahead, no more: all ten would be live)
      f2v ma = (f2v)(0.0f), mb = (f2v)(0.0f);
      const f4v one4 = (f4v)(1.0f);
      f2v k0 = S.k0k2[cst[0]][0], k1 = S.k0k2[cst[1]][0];
      f4v da = scaled ? reinterpret_cast<const f4v *>(&S.dcol[0])[0] : one4,
          db = scaled ? reinterpret_cast<const f4v *>(&S.dcol[0])[1] : one4,
          dd = scaled ? reinterpret_cast<const f4v *>(&S.dcol[0])[2] : one4;
#pragma unroll
      for (int kc = 0; kc < NS; ++kc) {
        const int kn = kc + 1 < NS ? kc + 1 : kc;
        asm volatile("" ::: "memory");  // table reads stay in the pass (no LICM)
        const f2v k0n = S.k0k2[cst[0]][kn], k1n = S.k0k2[cst[1]][kn];
        const f4v *dcn = reinterpret_cast<const f4v *>(&S.dcol[12 * kn]);
        const f4v dan = scaled ? dcn[0] : one4, dbn = scaled ? dcn[1] : one4, ddn = scaled ? dcn[2] : one4;
        __builtin_amdgcn_sched_barrier(0);
        const f2v kx = {k0.x, k1.x}, ky = {k0.y, k1.y};
        const float dv[12] = {da.x, da.y, da.z, da.w, db.x, db.y, db.z, db.w, dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int w = 0; w < 12; ++w) {
          const f2v be = {bet[0][w], bet[1][w]}, ep = {eps[0][w], eps[1][w]};
          const f2v p = __builtin_elementwise_fma(ky, ep, kx * be) * (f2v)(dv[w]);
          f2v &acc = (w & 1) ? mb : ma;
          acc.x = fmaxf(acc.x, fabsf(p.x));
          acc.y = fmaxf(acc.y, fabsf(p.y));
        }
        // pin the step's arithmetic here (no sinking into a late masked block
        // that would keep every step's loads live)
        asm volatile("" : "+v"(ma), "+v"(mb));
        __builtin_amdgcn_sched_barrier(0);
        k0 = k0n;
        k1 = k1n;
        da = dan;
        db = dbn;
        dd = ddn;
      }
      m[0] = valid[0] ? fmaxf(ma.x, mb.x) : 0.0f;
      m[1] = valid[1] ? fmaxf(ma.y, mb.y) : 0.0f;
    };
    float cnP[2];
    {
      float m[2];
      row_norms(false, m);
#pragma unroll
      for (int h = 0; h < 2; ++h) cnP[h] = valid[h] ? fmaxf(m[h], pdiag[h]) : 0.0f;
    }
    const float inv_n = 1.0f / (float)nvar;
    for (int it = 0; it < a.scaling; ++it) {
      float Dt[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float cnA = fmaxf(fabsf(ra0[h]), fabsf(ra1[h]));
        const float zmax = fmaxf(fabsf(rz0[h]), fabsf(rz1[h]));
        const float zm1 = lane_prev(zmax), zm2 = lane_prev(zm1);
        if (comp == 2) cnA = fmaxf(cnA, fmaxf(zm1, zm2));
        Dt[h] = valid[h] ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(cnP[h], cnA))) : 1.0f;
        const float Et0 = valid[h] ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(fabsf(ra0[h]), fabsf(rz0[h])))) : 1.0f;
        const float Et1 = (valid[h] && xy) ? __builtin_amdgcn_rsqf(limit_scaling(fmaxf(fabsf(ra1[h]), fabsf(rz1[h])))) : 1.0f;
        const float Dn1 = lane_next(Dt[h]), Dn2 = lane_next(Dn1);
        const float Dz = comp == 0 ? Dn2 : (comp == 1 ? Dn1 : Dt[h]);
        ra0[h] *= Et0 * Dt[h];
        ra1[h] *= Et1 * Dt[h];
        rz0[h] *= Et0 * Dz;
        rz1[h] *= Et1 * Dz;
        rE0[h] *= Et0;
        rE1[h] *= Et1;
        qv[h] *= Dt[h];
        qsv[h] *= Dt[h];
        Dr[h] *= Dt[h];
        if constexpr (W == 1) {
          if (lane < 60) S.dcol[60 * h + lane] = valid[h] ? Dr[h] : 0.0f;
        } else {
          if (valid[h]) S.dcol[120 * wv + 60 * h + lane] = Dr[h];  // column-space order
        }
      }
      bsync<W>();
      float cn2[2], mr[2];
      row_norms(true, mr);
#pragma unroll
      for (int h = 0; h < 2; ++h) cn2[h] = valid[h] ? Dr[h] * fmaxf(mr[h], pdiag[h] * Dr[h]) : 0.0f;
      // cost scaling: mean column norm of the scaled P vs ||q||_inf
      const float sumP = bsum<W>(S, wsum(cn2[0] + cn2[1]), wv);
      const float qm = bmax1<W>(S, wmax_nonneg(fmaxf(valid[0] ? fabsf(qsv[0]) : 0.0f, valid[1] ? fabsf(qsv[1]) : 0.0f)), wv);
      const float meanP = cs * sumP * inv_n;
      const float ctc = __builtin_amdgcn_rcpf(limit_scaling(fmaxf(meanP, limit_scaling(qm))));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        qv[h] *= ctc;
        qsv[h] *= ctc;
        cnP[h] = cn2[h] * cs * ctc;
      }
      cs *= ctc;
      bsync<W>();
    }
  }
  // block-uniform scalars live in SGPRs (a VGPR copy would be kept, and
  // spilled, across the whole ADMM loop)
  cs = sgpr_f(cs);
  const float cinv0 = sgpr_f(1.0f / cs);
  bool eq0[2];
  float qn[2] = {0.0f, 0.0f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float lh0 = rl0[h] * rE0[h], uh0 = ru0[h] * rE0[h];
    eq0[h] = valid[h] && !xy && (uh0 - lh0 < 1e-4f);  // OSQP set_rho_vec: RHO_TOL
    S.zh[wv][h][lane] = uh0;
    S.dr[wv][h][lane] = Dr[h];
    S.qvl[wv][h][lane] = qv[h];
    S.arz[wv][h][lane] = (f4v){ra0[h], ra1[h], rz0[h], rz1[h]};
    qn[0] = fmaxf(qn[0], valid[h] ? fabsf(qv[h] / Dr[h]) : 0.0f);
    qn[1] = fmaxf(qn[1], valid[h] ? fabsf(qv[h]) : 0.0f);
  }
  qn[0] = wmax_nonneg(qn[0]);
  qn[1] = wmax_nonneg(qn[1]);
  bcombine_max<W, 2>(S, qn, wv);
  S.sc[wv].cs = cs;  // every lane the same value
  S.sc[wv].cinv = cinv0;
  S.sc[wv].qn0 = qn[0];
  S.sc[wv].qn1 = qn[1];
  lsync();

  // row scaling E of a slot's two rows, from A~ = E A D (each row's entry in
  // its own variable's column is 1 before scaling)
  auto row_e = [&](int h) -> f2v {
    const int fl = fresh_lane();
    const f4v arz = S.arz[wv][h][fl];
    const float d = S.dr[wv][h][fl];
    return (f2v){valid[h] ? arz.x / d : 1.0f, (valid[h] && xy) ? arz.y / d : 1.0f};
  };

  // wrench row of this lane: step jr, component sr; its row of Bb (12)
  const bool wvalid = lane < nw;
  // lanes 6N..59 carry the (identity) factors of the padding steps, whose
  // K0 / K2 weights are zero; lanes 60..63 only pad
  const int jr = lane < 60 ? lane / 6 : kLitN - 1, sr = lane < 60 ? lane - 6 * (lane / 6) : 0;
  // this lane's row of Bb (12) is read from LDS where used (registers are
  // the factorisation's bound); padding wrench lanes get zeros
  // through their K0 / K2 weights and masks
  // this lane's variables' wrench columns (omega rows = lo.xyz, v row = dtm at comp)
  S.sc[wv].rho = sgpr_f(fminf(fmaxf(p_same ? prec[NP] : a.rho, 1e-6f), 1e6f));

  // ---------------- 6. ADMM (osqp_solve) with its (re)factorisations
  float x[2] = {0.0f, 0.0f};
  f2v z[2] = {(f2v)(0.0f), (f2v)(0.0f)}, y[2] = {(f2v)(0.0f), (f2v)(0.0f)};
  {
    S.sc[wv].alpha = a.alpha;
    S.sc[wv].oma = 1.0f - a.alpha;
    S.sc[wv].sigma = a.sigma;
    S.sc[wv].dtm = dtm;
    const int ctm = a.check_termination;
    S.sc[wv].ctm = ctm;
    S.sc[wv].interval = (a.adaptive_rho && a.rho_interval == 0) ? (ctm ? 4 * ctm : 100)
                                                                : (a.adaptive_rho ? a.rho_interval : 0);
    S.sc[wv].iter = 0;
    S.sc[wv].status = QLOCO_MAX_ITER;
    S.sc[wv].rho_updates = 0;
  }
  lsync();
  auto uf = [&](const float &v) { return sgpr_f(v); };  // an LDS scalar into an SGPR
  auto ui = [&](const int &v) { return __builtin_amdgcn_readfirstlane(v); };
  Row<W> T;        // T = (I + cG U)^-1 cG, this lane's wrench row (column space)
  Shift5 W1[2];  // per slot: this lane's row of W0^-1 as leg-triple shifts

  // P~ x (scaled) per slot: c D (Vu' G Vu + R) D x through the wrench rows
  auto p_times_x = [&](float (&out)[2]) {
    if constexpr (W == 2) bsync<W>();  // the other wave is done with the iteration's broadcast rows
    QL_LIT_LANE_INDICES(lxp);
    const float drp[2] = {S.dr[wv][0][lxp], S.dr[wv][1][lxp]};
    const float csl = uf(S.sc[wv].cs), dtm = uf(S.sc[wv].dtm);
#pragma unroll
    for (int h = 0; h < 2; ++h) S.av[wv][h][lxp] = valid[h] ? x[h] * drp[h] : 0.0f;
    lsync();
    // w = Vu (D x): wrench row (jr, sr) sums its step's 12 variables
    float wr = 0.0f;
    {
      const int hh = jr >= 5 ? 1 : 0, base = 12 * (jr - 5 * hh);
      const f4v *src = reinterpret_cast<const f4v *>(&S.av[wv][hh][base]);
      const f4v u0 = src[0], u1 = src[1], u2 = src[2];
      const float uv[12] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w, u2.x, u2.y, u2.z, u2.w};
      const f4v *br = reinterpret_cast<const f4v *>(S.Bb[sr]);
      const f4v b0 = br[0], b1 = br[1], b2 = br[2];
      const float bv[12] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w};
#pragma unroll
      for (int w = 0; w < 12; ++w) wr = fmaf(bv[w], uv[w], wr);
      wr = wvalid ? wr : 0.0f;
    }
    S.wv[wv][lxp] = wr;
    lsync();
    // Te w per row (needs the step's 6 wrench values)
    {
      float tw = 0.0f;
#pragma unroll
      for (int t = 0; t < 6; ++t) tw = fmaf(S.Te[sr][t], S.wv[wv][6 * jr + t], tw);
      reinterpret_cast<float *>(&S.bc[0][wv][0])[lxp] = wvalid ? tw : 0.0f;  // Te w (bc is free in a check)
    }
    bsync<W>();
    // (G w)[(jr, sr)] = Qb_s sum_k K0(jr,k) w(k,sr) + sum_k K2(jr,k) (Te w_k)_sr
    float gw = 0.0f;
    {
      const float qb = S.q2[6 + sr];
      float s0 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int wp = 0; wp < W; ++wp) {
#pragma unroll
        for (int k = 0; k < kLitN; ++k) {
          const f2v kk = S.k0k2[jc][10 * wp + k];
          s0 = fmaf(kk.x, S.wv[wp][6 * k + sr], s0);
          s2 = fmaf(kk.y, reinterpret_cast<const float *>(&S.bc[0][wp][0])[6 * k + sr], s2);
        }
      }
      gw = wvalid ? fmaf(qb, s0, s2) : 0.0f;
    }
    bsync<W>();
    S.wv[wv][lxp] = gw;
    lsync();
    // Vu' (G w) + R (D x), then c D (...)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float acc = 0.0f;
      if (valid[h]) {
        const float *gs = &S.wv[wv][6 * stepl[h]];
        const int wc = lxp % 12;  // the variable's column of Bb (both slots: 60 = 5 x 12)
        acc = S.Bb[0][wc] * gs[0] + S.Bb[1][wc] * gs[1] + S.Bb[2][wc] * gs[2] + dtm * gs[3 + comp];
        acc = fmaf(S.r2[3 * leg[h] + comp], x[h] * drp[h], acc);  // valid slot: r2 of its leg
      }
      out[h] = csl * drp[h] * acc;
    }
    lsync();
  };

  auto residuals = [&](float (&o)[6], float (&r)[6], bool want_r) {
    float px[2];
    p_times_x(px);
    QL_LIT_LANE_INDICES(lxr);
#pragma unroll
    for (int k = 0; k < 6; ++k) o[k] = r[k] = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float Drl = S.dr[wv][h][lxr];
      const float Dinvl = __builtin_amdgcn_rcpf(Drl);
      const f4v arz = S.arz[wv][h][lxr];
      // E^-1 of the slot's rows from A~ = E A D (unit own-column entries)
      const f2v Einv = {valid[h] ? Drl * __builtin_amdgcn_rcpf(arz.x) : 1.0f,
                        (valid[h] && xy) ? Drl * __builtin_amdgcn_rcpf(arz.y) : 1.0f};
      const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
      const float n1 = lane_next(x[h]), n2 = lane_next(n1);
      const float xz = comp == 0 ? n2 : (comp == 1 ? n1 : x[h]);
      const f2v ay = ra * y[h], az = rz * y[h];
      const float ay_z = az.x + az.y;
      const float p1 = lane_prev(ay_z), p2 = lane_prev(p1);
      const float aty = valid[h] ? ((ay.x + ay.y) + (comp == 2 ? (p1 + p2) : 0.0f)) : 0.0f;
      const float rd = valid[h] ? (S.qvl[wv][h][lxr] + px[h] + aty) : 0.0f;
      const f2v ax = ra * x[h] + rz * xz;
      const f2v rp = ax - z[h];
      const f2v erp = Einv * rp, ez = Einv * z[h], eax = Einv * ax;
      o[0] = fmaxf(o[0], fmaxf(fabsf(erp.x), fabsf(erp.y)));
      o[1] = fmaxf(o[1], fmaxf(fabsf(ez.x), fabsf(ez.y)));
      o[2] = fmaxf(o[2], fmaxf(fabsf(eax.x), fabsf(eax.y)));
      o[3] = fmaxf(o[3], fabsf(Dinvl * rd));
      o[4] = fmaxf(o[4], fabsf(Dinvl * aty));
      o[5] = fmaxf(o[5], fabsf(Dinvl * px[h]));
      if (want_r) {
        r[0] = fmaxf(r[0], fmaxf(fabsf(rp.x), fabsf(rp.y)));
        r[1] = fmaxf(r[1], fmaxf(fabsf(z[h].x), fabsf(z[h].y)));
        r[2] = fmaxf(r[2], fmaxf(fabsf(ax.x), fabsf(ax.y)));
        r[3] = fmaxf(r[3], fabsf(rd));
        r[4] = fmaxf(r[4], fabsf(aty));
        r[5] = fmaxf(r[5], fabsf(px[h]));
      }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) o[k] = wmax_nonneg(o[k]);
    if (want_r) {
#pragma unroll
      for (int k = 0; k < 6; ++k) r[k] = wmax_nonneg(r[k]);
    }
    if constexpr (W == 2) {  // block maxima (r only where the rho estimate needs them)
      float v[12];
#pragma unroll
      for (int k = 0; k < 6; ++k) v[k] = o[k], v[6 + k] = want_r ? r[k] : 0.0f;
      bcombine_max<W, 12>(S, v, wv);
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = v[k], r[k] = v[6 + k];
    }
  };

  // warm start (x, z, y) before the first factorisation
  if (WS) {
    QL_LIT_LANE_INDICES(lxs);  // record addresses derived here, not shared with the write-back
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int vidx = 12 * step[h] + 3 * leg[h] + comp, rbase = 20 * step[h] + 5 * leg[h] + 2 * comp;
      if (p_same) {
        x[h] = valid[h] ? prec[vidx] : 0.0f;
        z[h].x = valid[h] ? prec[12 * N + rbase] : 0.0f;
        z[h].y = (valid[h] && xy) ? prec[12 * N + rbase + 1] : 0.0f;
        y[h].x = valid[h] ? prec[32 * N + rbase] : 0.0f;
        y[h].y = (valid[h] && xy) ? prec[32 * N + rbase + 1] : 0.0f;
      } else if (a.warm_start == 1) {
        const float *wx = a.warm + b * (32 * N);
        const float *wy = wx + 12 * N;
        x[h] = valid[h] ? wx[vidx] / S.dr[wv][h][lxs] : 0.0f;
        const f2v e = row_e(h);
        const float csl = uf(S.sc[wv].cs);
        y[h].x = valid[h] ? wy[rbase] / e.x * csl : 0.0f;
        y[h].y = (valid[h] && xy) ? wy[rbase + 1] / e.y * csl : 0.0f;
        const float n1 = lane_next(x[h]), n2 = lane_next(n1);
        const float xz = comp == 0 ? n2 : (comp == 1 ? n1 : x[h]);
        const f4v arz = S.arz[wv][h][lxs];
        z[h] = (f2v){arz.x, arz.y} * x[h] + (f2v){arz.z, arz.w} * xz;
      }
    }
  }
  // G^-1 in six N x N blocks.  G = K0 (x) Qb + K2 (x) Te
  // (Qb = diag(q_omega, q_v), Te = dt^2 blockdiag(Rz' diag(q_theta) Rz,
  // diag(q_p))) splits by wrench component: each v axis and omega_z alone
  // (A_a = alpha_a K0 + beta_a K2), omega_x / omega_y together:
  // G_xy = K0 (x) Q + K2 (x) dt^2 T, Q = diag(q_omega_x, q_omega_y),
  // T = [Rz' diag(q_theta) Rz]_xy.  The 2 x 2 pair (T, Q) is diagonalised
  // together -- S' Q S = I, S' T S = diag(lambda) with S = Q^-1/2 V, V the
  // eigenvectors of Q^-1/2 T Q^-1/2 (one Jacobi rotation) -- so
  // G_xy^-1 = (I (x) S) diag_a (K0 + dt^2 lambda_a K2)^-1 (I (x) S'): two more
  // N x N inverses, recombined through S in the factorisation.  Any omega
  // weights work (q_omega_x != q_omega_y couples the axes: the reference's
  // isaac_a1_mpc.yaml); with q_omega_x = q_omega_y S is Rz' / sqrt(q_omega).
  // One N x N Gauss-Jordan per (axis, row) lane in float64, once per solve,
  // instead of a 6N x 6N one per factorisation.
  float gmx;  // max diag G^-1 (block-uniform; an SPD matrix's largest entry)
  {
    double row[NS];
    const int r = tid;
    const bool live = r < 6 * N;
    const int ax = live ? r / N : 0, ri = live ? r - N * (r / N) : 0;
    double sxy[2][2], sn2 = 1.0;  // S; sn2: this lane's axis' S column norm^2 (the gmx bound)
    {
      const double dt2 = (double)dt * (double)dt;
      double lam[2];
      {
        const double qx = (double)S.q2[6], qy = (double)S.q2[7];
        const double yw = (double)S.x0[2], cw = cos(yw), sw = sin(yw);
        const double Rm[2][2] = {{cw, sw}, {-sw, cw}};  // Rz (A1RobotControl.cpp:506-508)
        double T[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            T[i][j] = Rm[0][i] * (double)S.q2[0] * Rm[0][j] + Rm[1][i] * (double)S.q2[1] * Rm[1][j];
        const double ix = 1.0 / sqrt(qx), iy = 1.0 / sqrt(qy);
        const double c00 = T[0][0] * ix * ix, c01 = T[0][1] * ix * iy, c11 = T[1][1] * iy * iy;
        double t = 0.0;  // one Jacobi rotation: tan of the angle that diagonalises C
        if (c01 != 0.0) {
          const double tau = (c11 - c00) / (2.0 * c01);
          t = tau == 0.0 ? 1.0 : (tau > 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
        }
        const double cs = 1.0 / sqrt(1.0 + t * t), sn = t * cs;
        lam[0] = c00 - t * c01;
        lam[1] = c11 + t * c01;
        sxy[0][0] = ix * cs;  // S = Q^-1/2 V, V = [[cs, sn], [-sn, cs]]
        sxy[0][1] = ix * sn;
        sxy[1][0] = -iy * sn;
        sxy[1][1] = iy * cs;
        if (ax < 2) sn2 = sxy[0][ax] * sxy[0][ax] + sxy[1][ax] * sxy[1][ax];
      }
      const double al = ax < 2 ? 1.0 : (ax == 2 ? (double)S.q2[8] : (double)S.q2[9 + ax - 3]);
      const double be = ax < 2 ? dt2 * lam[ax] : dt2 * (double)S.q2[ax];  // q_theta_z / q_p: q2[2..5]
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int M = ri > k ? ri : k;
        const double T0 = (double)(N - M), ia = (double)(M - ri), ib = (double)(M - k);
        const double S1 = 0.5 * T0 * (T0 - 1.0), S2 = (T0 - 1.0) * T0 * (2.0 * T0 - 1.0) / 6.0;
        const double K2 = S2 + (ia + ib) * S1 + ia * ib * T0;
        row[k] = (live && k < N) ? fma(al, T0, be * K2) : (k == ri ? 1.0 : 0.0);
      }
    }
    // in-place Gauss-Jordan, the pivot row through LDS (double-buffered in the
    // table area, which is written only after the last pivot)
    double *xch = reinterpret_cast<double *>(&S.gtab[0][0][0]);
    static_assert(sizeof(S.gtab) >= 2 * 6 * NS * sizeof(double), "pivot-row exchange fits the table area");
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      if (k >= N) continue;  // uniform; not a break (the loop must unroll: row[] stays in registers)
      double *buf = xch + (k & 1) * (6 * NS);
      if (live && ri == k) {
#pragma unroll
        for (int c = 0; c < NS; ++c) buf[ax * NS + c] = row[c];
      }
      bsync<W>();
      const double *pr = buf + ax * NS;  // the pivot row, read as it is used (no second register row)
      const double pinv = 1.0 / pr[k];
      const double fk = row[k] * pinv;
#pragma unroll
      for (int c = 0; c < NS; ++c) {
        if (c == k) continue;
        const double pc = pr[c];
        row[c] = ri == k ? pc * pinv : fma(-fk, pc, row[c]);
      }
      row[k] = ri == k ? pinv : -fk;
    }
    bsync<W>();
    // the padding entries of the tables are zero
    for (int idx = tid; idx < NT * NT * 3; idx += 64 * W) (&S.gtab[0][0][0])[idx] = (f2v)(0.0f);
    bsync<W>();
    float dmax = 0.0f;
    if (live) {
      const int csi = W == 1 ? ri : (ri < H ? ri : 10 + ri - H);
      float *dst = reinterpret_cast<float *>(&S.gtab[csi][0][0]);
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        if (k < N) {
          const int csk = W == 1 ? k : (k < H ? k : 10 + k - H);
          dst[csk * 6 + ax] = (float)row[k];
        }
        // world-frame diagonal of the xy block <= 2 max_a |S[.][a]|^2 A_a^-1(j, j)
        dmax = k == ri ? (float)(sn2 * row[k]) : dmax;
      }
    }
    if (tid == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) S.sc[wv].sxy[i][j] = (float)sxy[i][j];
    }
    if constexpr (W == 2) {
      if (tid == 64) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) S.sc[1].sxy[i][j] = (float)sxy[i][j];
      }
    }
    gmx = sgpr_f(bmax1<W>(S, wmax_nonneg(dmax), wv));
    bsync<W>();
  }
  for (;;) {
    // ---------------- 6a. factorisation for the current rho
    {
      // opaque per factorisation: nothing derived from these is hoisted out of
      // the refactor loop (it would stay live through the ADMM iterations)
      int ln = fresh_lane();
      asm volatile("" : "+v"(ln));
      const float rho = uf(S.sc[wv].rho), cinv = uf(S.sc[wv].cinv), sigma = uf(S.sc[wv].sigma);
      QL_LIT_LANE_INDICES(lxf);
      // this lane's row of W0^-1 for slot h (W0 = D^-1 (sigma I + A~' rho A~) D^-1 +
      // c R, 3 x 3 per leg): written for the U rows, recomputed for the
      // iteration coefficients after the T phase (its LDS is the T passes')
      // (D^-1 and c re-laundered per call: the first call's copies do not stay
      // live across S^-1 for the second)
      auto w0_inv_row = [&](int h, float &i0, float &i1, float &i2) {
        float dinv_h = valid[h] ? 1.0f / S.dr[wv][h][lxf] : 0.0f, csw = uf(S.sc[wv].cs);
        asm volatile("" : "+v"(dinv_h), "+v"(csw));
        const f4v arz = S.arz[wv][h][lxf];
        const float rv0 = eq0[h] ? 1e3f * rho : rho, rv1 = rho;
        const float d_own = rv0 * arz.x * arz.x + rv1 * arz.y * arz.y;
        const float d_oz = rv0 * arz.x * arz.z + rv1 * arz.y * arz.w;
        const float d_zz = rv0 * arz.z * arz.z + rv1 * arz.w * arz.w;
        const float oz1 = lane_prev(d_oz), oz2 = lane_prev(oz1);
        const float zz1 = lane_prev(d_zz), zz2 = lane_prev(zz1);
        float m0, m1, m2;  // this lane's row of sigma I + A~' rho A~ (scaled space)
        if (comp == 0) {
          m0 = d_own + sigma; m1 = 0.0f; m2 = d_oz;
        } else if (comp == 1) {
          m0 = 0.0f; m1 = d_own + sigma; m2 = d_oz;
        } else {
          m0 = oz2; m1 = oz1; m2 = d_own + zz1 + zz2 + sigma;
        }
        const Triple dd = triple(dinv_h, comp);
        // W0 row = D^-1 M D^-1 + c R (diagonal)
        float w0 = dinv_h * m0 * dd.v0, w1 = dinv_h * m1 * dd.v1, w2 = dinv_h * m2 * dd.v2;
        const float cr = csw * (valid[h] ? S.r2[3 * leg[h] + comp] : 0.0f);
        w0 += comp == 0 ? cr : 0.0f;
        w1 += comp == 1 ? cr : 0.0f;
        w2 += comp == 2 ? cr : 0.0f;
        if (!valid[h]) { w0 = comp == 0 ? 1.0f : 0.0f; w1 = comp == 1 ? 1.0f : 0.0f; w2 = comp == 2 ? 1.0f : 0.0f; }
        // the full 3 x 3 leg block: rows from the triple's lanes
        const Triple c0 = triple(w0, comp), c1 = triple(w1, comp), c2 = triple(w2, comp);
        // rows: row0 = (c0.v0, c1.v0, c2.v0), row1 = (c0.v1, ...), row2 = (c0.v2, ...)
        const float a00 = c0.v0, a01 = c1.v0, a02 = c2.v0;
        const float a10 = c0.v1, a11 = c1.v1, a12 = c2.v1;
        const float a20 = c0.v2, a21 = c1.v2, a22 = c2.v2;
        const float k00 = a11 * a22 - a12 * a21, k01 = a02 * a21 - a01 * a22, k02 = a01 * a12 - a02 * a11;
        const float k10 = a12 * a20 - a10 * a22, k11 = a00 * a22 - a02 * a20, k12 = a02 * a10 - a00 * a12;
        const float k20 = a10 * a21 - a11 * a20, k21 = a01 * a20 - a00 * a21, k22 = a00 * a11 - a01 * a10;
        const float idet = 1.0f / (a00 * k00 + a01 * k10 + a02 * k20);
        i0 = (comp == 0 ? k00 : (comp == 1 ? k10 : k20)) * idet;  // row comp of W0^-1
        i1 = (comp == 0 ? k01 : (comp == 1 ? k11 : k21)) * idet;
        i2 = (comp == 0 ? k02 : (comp == 1 ? k12 : k22)) * idet;
      };
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float i0, i1, i2;
        w0_inv_row(h, i0, i1, i2);
        S.w0i[wv][0][h][lxf] = i0;
        S.w0i[wv][1][h][lxf] = i1;
        S.w0i[wv][2][h][lxf] = i2;
      }
      lsync();
      // U_j rows: wrench lane (jr, sr): U[sr][t] = sum_w Bb[sr][w] (W0^-1 Bb')[w][t]
      float Urow[6];  // this lane's row of U_jr, in registers (padding lanes: identity)
      {
        float yv[12];
        const int hh = jr >= 5 ? 1 : 0, base = 12 * (jr - 5 * hh);
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // leg g of the step: 3 x 3 block
          const int v0 = base + 3 * g;
          const f4v r0 = {S.w0i[wv][0][hh][v0], S.w0i[wv][1][hh][v0], S.w0i[wv][2][hh][v0], 0.0f},
                    r1 = {S.w0i[wv][0][hh][v0 + 1], S.w0i[wv][1][hh][v0 + 1], S.w0i[wv][2][hh][v0 + 1], 0.0f},
                    r2 = {S.w0i[wv][0][hh][v0 + 2], S.w0i[wv][1][hh][v0 + 2], S.w0i[wv][2][hh][v0 + 2], 0.0f};
          const float b0 = S.Bb[sr][3 * g], b1 = S.Bb[sr][3 * g + 1], b2 = S.Bb[sr][3 * g + 2];
          yv[3 * g + 0] = b0 * r0.x + b1 * r1.x + b2 * r2.x;
          yv[3 * g + 1] = b0 * r0.y + b1 * r1.y + b2 * r2.y;
          yv[3 * g + 2] = b0 * r0.z + b1 * r1.z + b2 * r2.z;
        }
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          float acc = 0.0f;
#pragma unroll
          for (int w = 0; w < 12; ++w) acc = fmaf(yv[w], S.Bb[t][w], acc);
          Urow[t] = wvalid ? acc : (t == sr ? 1.0f : 0.0f);
        }
      }
      // T = (I + cG U)^-1 cG = (U + (cG)^-1)^-1: this lane's
      // row of M = G^-1 / c + U (G^-1 from the per-solve tables through the
      // omega block's rotation; U block-diagonal: this lane's row of U_jr in
      // its own step's six columns), scaled by 1 / (max diag G^-1 / c + max
      // diag U) -- a bound within 2x of max diag M (SPD) -- and inverted in
      // place.  (Round 4's S = I + L'cGL form left a KKT backward error of
      // 1e-3 .. 1e-2 at rho <= 3e-4; M keeps it at 1e-5 .. 5e-4,
      // tools/lit_numerics.py.)
      float sM;
      {
        float uii = 0.0f;
#pragma unroll
        for (int t = 0; t < 6; ++t) uii = t == sr ? Urow[t] : uii;
        sM = sgpr_f(1.0f / fmaf(gmx, cinv, bmax1<W>(S, wmax_nonneg(wvalid ? uii : 0.0f), wv)));
        // omega x / y block coefficients S[sr][a] S[t][a], a, t in {0, 1}
        // (the G^-1 tables hold the eigen axes' A_a^-1)
        const float s00 = uf(S.sc[wv].sxy[0][0]), s01 = uf(S.sc[wv].sxy[0][1]), s10 = uf(S.sc[wv].sxy[1][0]),
                    s11 = uf(S.sc[wv].sxy[1][1]);
        const float r0 = sr == 0 ? s00 : (sr == 1 ? s10 : 0.0f), r1 = sr == 0 ? s01 : (sr == 1 ? s11 : 0.0f);
        const float c00 = r0 * s00, c01 = r0 * s10, c10 = r1 * s01, c11 = r1 * s11;
        const float m2 = sr == 2 ? 1.0f : 0.0f, m3 = sr == 3 ? 1.0f : 0.0f, m4 = sr == 4 ? 1.0f : 0.0f,
                    m5 = sr == 5 ? 1.0f : 0.0f;
        const float scale = sM * cinv;
#pragma unroll
        for (int wp = 0; wp < W; ++wp) {
#pragma unroll
          for (int k = 0; k < kLitN; ++k) {
            const f2v e0 = S.gtab[jc][10 * wp + k][0], e1 = S.gtab[jc][10 * wp + k][1],
                      e2 = S.gtab[jc][10 * wp + k][2];
            const float gv[6] = {fmaf(c00, e0.x, c10 * e0.y), fmaf(c01, e0.x, c11 * e0.y), m2 * e1.x,
                                 m3 * e1.y, m4 * e2.x, m5 * e2.y};
            const bool blk = wp == wv && k == jr;  // this row's own step block
#pragma unroll
            for (int t = 0; t < 6; ++t) {
              const int c = 60 * wp + 6 * k + t;
              const bool own = wp == wv && 6 * k + t == ln;
              const float g = wvalid ? gv[t] : (own ? 1.0f : 0.0f);
              T.k[c] = fmaf(scale, g, blk ? sM * Urow[t] : 0.0f);
              asm volatile("" : "+v"(T.k[c]));  // final here (no sinking into the Gauss-Jordan)
            }
          }
        }
#pragma unroll
        for (int c = 60 * W; c < 64 * W; ++c) T.k[c] = 0.0f;
      }
      if constexpr (W == 1)
        lit_invert(S, lxf, nw, T);  // (sM M)^-1
      else
        lit_invert2(S, wv, 6 * H, 6 * (N - H), T);
#pragma unroll
      for (int c = 0; c < 60 * W; ++c) T.k[c] *= sM;  // T = M^-1
      // a = W0^-1 D^-1 b and x~ = D^-1 (a - W0^-1 t): this lane's row of W0^-1
      // as leg-triple shifts (D^-1 applied elementwise around the two dots)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float wx, wy, wz;
        w0_inv_row(h, wx, wy, wz);
        const f4v wi = {wx, wy, wz, 0.0f};
        W1[h] = shift5(valid[h] ? wi.x : 0.0f, valid[h] ? wi.y : 0.0f, valid[h] ? wi.z : 0.0f, comp);
      }
    }
    bool refactor = false;

    for (;;) {
      int iter = ui(S.sc[wv].iter);
      const int ctm = ui(S.sc[wv].ctm), interval = ui(S.sc[wv].interval);
      if (iter < a.max_iter) {
        int next = a.max_iter;
        if (ctm) next = min(next, (iter / ctm + 1) * ctm);
        if (interval) next = min(next, (iter / interval + 1) * interval);
        const float rho = uf(S.sc[wv].rho);
        const float rho_s = rho;
        const float rvb_s = sgpr_f(1.0f / rho);
        const float zlo = a.fz_max > 0.0f ? a.fz_min / a.fz_max : 0.0f;  // z rows: lower = zlo upper
        QL_LIT_LANE_INDICES(lxi);
        // loop operands read here, per segment of iterations: none is a register
        // across the residual checks and factorisations
        const float alpha = uf(S.sc[wv].alpha), oma = uf(S.sc[wv].oma), sigma = uf(S.sc[wv].sigma),
                    dtm = uf(S.sc[wv].dtm);
        float qvr[2], Dinv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          qvr[h] = S.qvl[wv][h][lxi];
          Dinv[h] = valid[h] ? 1.0f / S.dr[wv][h][lxi] : 0.0f;
        }
        // wave-uniform trip count (a scalar loop, not an exec-masked one)
        iter = __builtin_amdgcn_readfirstlane(iter);
        next = __builtin_amdgcn_readfirstlane(next);
        for (; iter < next; ++iter) {
          asm volatile("" ::: "memory");
          const int par = W == 1 ? 0 : (iter & 1);  // two waves: broadcast rows double-buffered
          // rho vector (eq rows 1e3 rho) from the scalar rho each iteration: per-lane
          // selects instead of six loop-invariant registers
          float rr = rho_s, rvb = rvb_s;
          asm volatile("" : "+v"(rr), "+v"(rvb));
          const float rva[2][2] = {{eq0[0] ? 1e3f * rr : rr, rr}, {eq0[1] ? 1e3f * rr : rr, rr}};
          const float rvia[2] = {eq0[0] ? 1e-3f * rvb : rvb, eq0[1] ? 1e-3f * rvb : rvb};
          // rhs = sigma x - q + A'(rho z - y) per slot, then a = W0^-1 D^-1 rhs
          float av[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f4v arz = S.arz[wv][h][lxi];
            const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
            const f2v rv = {rva[h][0], rva[h][1]};
            const f2v w = __builtin_elementwise_fma(rv, z[h], -y[h]);
            const f2v aw = ra * w, zw = rz * w;
            const float tz = zw.x + zw.y;
            float rhs = fmaf(sigma, x[h], (aw.x + aw.y) - qvr[h]);
            {
              const float m2 = comp == 2 ? 1.0f : 0.0f;
              float u;
              asm("s_nop 1\n\t"
                  "v_add_f32_dpp %0, %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                  "s_nop 1\n\t"
                  "v_fmac_f32_dpp %1, %0, %3 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                  : "=&v"(u), "+v"(rhs)
                  : "v"(tz), "v"(m2));
            }
            av[h] = tdot(Dinv[h] * rhs, W1[h]);  // W0^-1 D^-1 rhs
            S.av[wv][h][lxi] = av[h];
          }
          lsync();
          // v = Vu a: wrench row (jr, sr) over its step's 12 variables
          float wr = 0.0f;
          {
            const int hh = jr >= 5 ? 1 : 0, base = 12 * (jr - 5 * hh);
            const f4v *src = reinterpret_cast<const f4v *>(&S.av[wv][hh][base]);
            const f4v u0 = src[0], u1 = src[1], u2 = src[2];
            const float uv[12] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w, u2.x, u2.y, u2.z, u2.w};
            const f4v *br = reinterpret_cast<const f4v *>(S.Bb[sr]);
            const f4v b0 = br[0], b1 = br[1], b2 = br[2];
            const float bv[12] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w};
            float w0 = 0.0f, w1 = 0.0f;
#pragma unroll
            for (int w = 0; w < 12; w += 2) {
              w0 = fmaf(bv[w], uv[w], w0);
              w1 = fmaf(bv[w + 1], uv[w + 1], w1);
            }
            wr = w0 + w1;
          }
          reinterpret_cast<float *>(&S.bc[par][wv][0])[lxi] = wr;
          bsync<W>();
          // s = T v (DPP broadcast matvec, 60 columns per half)
          float sv;
          {
            const f4v r0 = S.bc[par][0][lxi & 15];
            float acc0, acc1;
            QL_DPP_MATVEC60_2(acc0, acc1, r0, T.k, 0);
            if constexpr (W == 2) {
              const f4v r1 = S.bc[par][1][lxi & 15];
              float acc2, acc3;
              QL_DPP_MATVEC60_2(acc2, acc3, r1, T.k, 60);
              sv = (acc0 + acc1) + (acc2 + acc3);
            } else {
              sv = acc0 + acc1;
            }
          }
          S.wv[wv][lxi] = sv;
          lsync();
          // x~ = D^-1 a - D^-1 W0^-1 Vu' s, then update_x / update_z / update_y; the
          // variable's omega rows of B_d from LDS (a padding slot's are harmless:
          // its leg's B1 coefficients are zero)
          const float bw0 = S.Bb[0][lxi % 12], bw1 = S.Bb[1][lxi % 12], bw2 = S.Bb[2][lxi % 12];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float *gs = &S.wv[wv][6 * stepl[h]];
            const f2v s01 = *reinterpret_cast<const f2v *>(gs), s23 = *reinterpret_cast<const f2v *>(gs + 2);
            f2v s45 = *reinterpret_cast<const f2v *>(gs + 4);
            asm volatile("" : "+v"(s45));  // loaded by every lane (no exec-masked load)
            const float sf = comp == 0 ? s23.y : (comp == 1 ? s45.x : s45.y);
            const float tv = fmaf(bw0, s01.x, fmaf(bw1, s01.y, fmaf(bw2, s23.x, dtm * sf)));
            const float xt = Dinv[h] * (av[h] - tdot(tv, W1[h]));  // D^-1 (a - W0^-1 t)
            const f4v arz = S.arz[wv][h][lxi];
            const f2v ra = {arz.x, arz.y}, rz = {arz.z, arz.w};
            const float hi = S.zh[wv][h][lxi];
            const f2v bnd = {xy ? 0.0f : zlo * hi, hi};
            const float n1 = lane_next(xt), n2 = lane_next(n1);
            const float xtz = comp == 0 ? n2 : n1;
            x[h] = fmaf(alpha, xt, oma * x[h]);
            const f2v rv = {rva[h][0], rva[h][1]};
            const f2v rvi2 = {rvia[h], rvb};
            const f2v zt = __builtin_elementwise_fma(rz, (f2v)(xtz), ra * xt);
            const f2v zr = __builtin_elementwise_fma((f2v)(alpha), zt, oma * z[h]);
            const f2v v = __builtin_elementwise_fma(y[h], rvi2, zr);
            const f2v zn = {__builtin_amdgcn_fmed3f(v.x, bnd.x, bnd.y), __builtin_amdgcn_fmed3f(v.y, -INFINITY, 0.0f)};
            y[h] = __builtin_elementwise_fma(rv, zr - zn, y[h]);
            z[h] = zn;
          }
        }
      }
      iter = ui(iter);
      S.sc[wv].iter = iter;
      const bool fin = iter >= a.max_iter;
      const bool can_check = ctm && iter > 0 && (iter % ctm == 0);
      const bool do_rho = interval && iter > 0 && (iter % interval == 0);
      if (!(can_check || do_rho || fin)) continue;
      float o[6], r[6];
      residuals(o, r, do_rho);
      const float cinv = uf(S.sc[wv].cinv), qn0 = uf(S.sc[wv].qn0);
      const float pri_res = o[0], dua_res = cinv * o[3];
      if (can_check) {
        const float eps_p = a.eps_abs + a.eps_rel * fmaxf(o[1], o[2]);
        const float eps_d = a.eps_abs + a.eps_rel * cinv * fmaxf(fmaxf(qn0, o[4]), o[5]);
        if (pri_res < eps_p && dua_res < eps_d) {
          S.sc[wv].status = QLOCO_OK;
          break;
        }
      }
      if (do_rho) {  // compute_rho_estimate + adapt_rho
        const float pn = r[0] / (fmaxf(r[1], r[2]) + 1e-30f);
        const float dn = r[3] / (fmaxf(fmaxf(uf(S.sc[wv].qn1), r[4]), r[5]) + 1e-30f);
        const float rho = uf(S.sc[wv].rho);
        float rho_new = rho * sqrtf(pn / (dn + 1e-30f));
        rho_new = fminf(fmaxf(rho_new, 1e-6f), 1e6f);
        if (rho_new > rho * a.rho_tol || rho_new < rho / a.rho_tol) {
          const int nup = ui(S.sc[wv].rho_updates) + 1;
          S.sc[wv].rho = sgpr_f(rho_new);
          S.sc[wv].rho_updates = nup;
          if (!fin) {
            refactor = true;
            break;
          }
        }
      }
      if (fin) {
        float e_abs = a.eps_abs, e_rel = a.eps_rel;  // laundered: 10 eps is not hoisted into VGPRs
        asm volatile("" : "+v"(e_abs), "+v"(e_rel));
        const float ep = 10.f * e_abs + 10.f * e_rel * fmaxf(o[1], o[2]);
        const float ed = 10.f * e_abs + 10.f * e_rel * cinv * fmaxf(fmaxf(qn0, o[4]), o[5]);
        S.sc[wv].status = __builtin_amdgcn_readfirstlane((pri_res < ep && dua_res < ed) ? QLOCO_SOLVED_INACCURATE
                                                                                          : QLOCO_MAX_ITER);
        break;
      }
    }
    if (!refactor) break;
  }

  // ---------------- 7. outputs: unscale, objective, leg slots (A1RobotControl.cpp:593-599)
  const int lane_o = fresh_lane();
  const int tid_o = W == 1 ? lane_o : (int)threadIdx.x;
  float xu[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) xu[h] = valid[h] ? x[h] * S.dr[wv][h][lane_o] : 0.0f;
  // P~ x at the final iterate, recomputed (the last check's copy would be a
  // register live across every ADMM iteration; same operands, same result)
  float px[2];
  p_times_x(px);
  const float cinv = uf(S.sc[wv].cinv);
  int status = ui(S.sc[wv].status);
  float ob = 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h) ob += valid[h] ? cinv * (0.5f * x[h] * px[h] + S.qvl[wv][h][lane_o] * x[h]) : 0.0f;
  const float objp = bsum<W>(S, wsum(ob), wv);
  const bool bad = !isfinite(objp);
  if (bad) status = QLOCO_NAN;
  if (a.u) {
    float *uo = a.u + b * 12 * N + 12 * so;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (valid[h]) uo[60 * h + lane_o] = bad ? NAN : xu[h];
  }
  // u0: step-0 forces (variables 0..11 = wave 0's slot 0, lanes 0..11); optional body frame R' u
  {
    const float n1 = lane_next(xu[0]), n2 = lane_next(n1);
    const float p1 = lane_prev(xu[0]), p2 = lane_prev(p1);
    const float f0 = comp == 0 ? xu[0] : (comp == 1 ? p1 : p2);
    const float f1 = comp == 0 ? n1 : (comp == 1 ? xu[0] : p1);
    const float f2 = comp == 0 ? n2 : (comp == 1 ? n1 : xu[0]);
    if (tid_o < 12) {
      float o = xu[0];
      if (a.output_frame == 1) {  // R^T f with R = [[c,s,0],[-s,c,0],[0,0,1]], recomputed here
        const float yw = S.x0[2], cw = cosf(yw), sw = sinf(yw);
        o = comp == 0 ? (cw * f0 - sw * f1) : (comp == 1 ? (sw * f0 + cw * f1) : f2);
      }
      a.u0[b * 12 + lane_o] = bad ? NAN : o;
    }
  }
  if (prec) {  // the persistent record for the next call (layout QLOCO_SRBD_PERSIST_LEN)
    QL_LIT_LANE_INDICES(lxo);  // fresh indices: no address kept live from the warm start
    for (int k = tid_o; k < NP + 4; k += 64 * W)
      if (k < 84 * N || k >= 96 * N) prec[k] = 0.0f;  // [84 N, 96 N): q, written at the gradient
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!valid[h]) continue;
      const int vidx = 12 * step[h] + 3 * leg[h] + comp, rbase = 20 * step[h] + 5 * leg[h] + 2 * comp;
      prec[vidx] = x[h];
      prec[52 * N + vidx] = xu[h];
      prec[12 * N + rbase] = z[h].x;
      prec[32 * N + rbase] = y[h].x;
      const f2v e = row_e(h);
      prec[64 * N + rbase] = cinv * e.x * y[h].x;
      if (xy) {
        prec[12 * N + rbase + 1] = z[h].y;
        prec[32 * N + rbase + 1] = y[h].y;
        prec[64 * N + rbase + 1] = cinv * e.y * y[h].y;
      }
    }
    for (int k = tid_o; k < 4 * N; k += 64 * W) prec[96 * N + k] = S.ctf[k];
    if (tid_o == 0) {
      prec[NP] = S.sc[wv].rho;
      prec[NP + 1] = 1.0f;
    }
  }
  if (WS && a.warm_start == 1) {
    QL_LIT_LANE_INDICES(lxo);
    const int nu = 12 * N, ncn = 20 * N;
    float *wx = a.warm + b * (nu + ncn);
    float *wy = wx + nu;
    for (int k = tid_o; k < nu + ncn; k += 64 * W) wx[k] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!valid[h]) continue;
      wx[12 * step[h] + 3 * leg[h] + comp] = xu[h];
      const int rbase = 20 * step[h] + 5 * leg[h] + 2 * comp;
      const f2v e = row_e(h);
      wy[rbase] = cinv * e.x * y[h].x;
      if (xy) wy[rbase + 1] = cinv * e.y * y[h].y;
    }
  }
  if (tid_o == 0) {
    if (a.status) a.status[b] = status;
    if (a.iters) a.iters[b] = S.sc[wv].iter;
    if (a.rho_updates) a.rho_updates[b] = S.sc[wv].rho_updates;
    if (a.obj) a.obj[b] = objp;
  }
}

template <bool WS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kLitWpe)))
void srbd_lit_kernel(const SrbdArgs a) {
  __shared__ __attribute__((aligned(16))) LitLds<1> S;
  const int64_t i = blockIdx.x;
  if (i >= a.batch) return;
  srbd_lit_one<1, WS>(a, S, i);
}

template <bool WS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(kLit2Wpe)))
void srbd_lit2_kernel(const SrbdArgs a) {
  __shared__ __attribute__((aligned(16))) LitLds<2> S;
  const int64_t i = blockIdx.x;
  if (i >= a.batch) return;
  srbd_lit_one<2, WS>(a, S, i);
}

int srbd_lit_launch(const SrbdArgs &a, bool warm, hipStream_t stream) {
  const dim3 grid((unsigned)a.batch);
  if (a.N < 1 || a.N > kLitN2) return QLOCO_BAD_SIZE;
  if (a.N <= kLitN) {
    if (warm)
      hipLaunchKernelGGL(srbd_lit_kernel<true>, grid, dim3(64), 0, stream, a);
    else
      hipLaunchKernelGGL(srbd_lit_kernel<false>, grid, dim3(64), 0, stream, a);
    QLOCO_HIP_CHECK(hipGetLastError(), "srbd_lit_kernel launch");
  } else {
    if (warm)
      hipLaunchKernelGGL(srbd_lit2_kernel<true>, grid, dim3(128), 0, stream, a);
    else
      hipLaunchKernelGGL(srbd_lit2_kernel<false>, grid, dim3(128), 0, stream, a);
    QLOCO_HIP_CHECK(hipGetLastError(), "srbd_lit2_kernel launch");
  }
  return QLOCO_OK;
}

}  // namespace qloco
