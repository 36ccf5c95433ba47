// qloco_host.cpp -- C++ host shim (include/qloco.hpp) over the C ABI.
//
// Host code only: it stages reference-shaped host arrays to the device on a
// HIP stream and calls libqloco.so.  No solver arithmetic lives here except
// the reference's own input assembly for compute_grf
// (A1RobotControl.cpp:459-497), which is host-side in the reference too.
#include <algorithm>

#include "qloco.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

namespace qloco {

Error::Error(const std::string &what, int s) : std::runtime_error(what), status(s) {}

static void hip_ok(hipError_t e, const char *where) {
  if (e != hipSuccess)
    throw Error(std::string(where) + ": " + hipGetErrorString(e), QLOCO_ERR_DEVICE);
}
static void abi_ok(int s, const char *where) {
  if (s != QLOCO_OK)
    throw Error(std::string(where) + " failed: " + qloco_status_string(s) + " " +
                    qloco_last_error(),
                s);
}

// ---------------------------------------------------------------- DeviceArena
DeviceArena::DeviceArena() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    throw Error("qloco: no GPU visible (the solver has no CPU fallback)", QLOCO_ERR_NO_GPU);
  hipStream_t s;
  hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
}
DeviceArena::~DeviceArena() {
  for (void *p : blocks_) (void)hipFree(p);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}
void *DeviceArena::alloc(size_t bytes) {
  void *p = nullptr;
  hip_ok(hipMalloc(&p, bytes ? bytes : 16), "hipMalloc");
  blocks_.push_back(p);
  return p;
}
void DeviceArena::release(void *p) {
  if (!p) return;
  for (size_t i = 0; i < blocks_.size(); ++i)
    if (blocks_[i] == p) {
      (void)hipFree(p);
      blocks_[i] = blocks_.back();
      blocks_.pop_back();
      return;
    }
}
void DeviceArena::upload(void *dev, const void *host, size_t bytes) {
  if (bytes) hip_ok(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, (hipStream_t)stream_), "upload");
}
void DeviceArena::download(void *host, const void *dev, size_t bytes) {
  if (bytes) hip_ok(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream_), "download");
}
void DeviceArena::sync() { hip_ok(hipStreamSynchronize((hipStream_t)stream_), "hipStreamSynchronize"); }

template <class T>
static T *dalloc(DeviceArena &a, size_t n) {
  return static_cast<T *>(a.alloc(n * sizeof(T)));
}

// ---------------------------------------------------------------- QPsolverGpu
QPsolverGpu::QPsolverGpu(int max_batch) : max_batch_(max_batch < 1 ? 1 : max_batch) {}
QPsolverGpu::~QPsolverGpu() = default;

void QPsolverGpu::resize(const int &nVar, const int &nEq, const int &nIneq) {
  // QPBaseClass.cpp:111-112 asserts nVars <= 60, nIneq <= 300; the kernels
  // take n, p <= 64, m <= 320 (qloco_gi_limits)
  int32_t ln = 0, lp = 0, lm = 0;
  qloco_gi_limits(&ln, &lp, &lm);
  if (nVar < 1 || nVar > ln || nEq < 0 || nEq > lp || nIneq < 0 || nIneq > lm)
    throw Error("QPsolverGpu::resize: size out of range", QLOCO_BAD_SIZE);
  n_ = nVar;
  p_ = nEq;
  m_ = nIneq;
}

// Device blocks are reused while the batch and the (n, p, m) of the last
// resize fit the sizes they were allocated for; otherwise the old blocks are
// freed before the new ones are allocated (repeated resizeQP calls or a
// growing batch do not accumulate device memory).
void QPsolverGpu::ensure(int batch) {
  if (batch <= cap_ && n_ <= an_ && p_ <= ap_ && m_ <= am_) return;
  for (void *p : {(void *)dG_, (void *)dg0_, (void *)dCE_, (void *)dce0_, (void *)dCI_,
                  (void *)dci0_, (void *)dX_, (void *)df_, (void *)dst_, (void *)dit_})
    arena_.release(p);
  dG_ = dg0_ = dCE_ = dce0_ = dCI_ = dci0_ = dX_ = df_ = nullptr;
  dst_ = dit_ = nullptr;
  if (batch < cap_) batch = cap_;
  const size_t B = batch;
  dG_ = dalloc<double>(arena_, B * n_ * n_);
  dg0_ = dalloc<double>(arena_, B * n_);
  dCE_ = dalloc<double>(arena_, B * (p_ ? n_ * p_ : 1));
  dce0_ = dalloc<double>(arena_, B * (p_ ? p_ : 1));
  dCI_ = dalloc<double>(arena_, B * (m_ ? n_ * m_ : 1));
  dci0_ = dalloc<double>(arena_, B * (m_ ? m_ : 1));
  dX_ = dalloc<double>(arena_, B * n_);
  df_ = dalloc<double>(arena_, B);
  dst_ = dalloc<int32_t>(arena_, B);
  dit_ = dalloc<int32_t>(arena_, B);
  cap_ = batch;
  an_ = n_;
  ap_ = p_;
  am_ = m_;
}

void QPsolverGpu::solve_batch(int batch, const double *G, const double *g0, const double *CE,
                              const double *ce0, const double *CI, const double *ci0,
                              double *X, double *f, int32_t *status) {
  if (n_ == 0) throw Error("QPsolverGpu: resize() first", QLOCO_ERR_ARG);
  ensure(batch);
  const size_t B = batch;
  arena_.upload(dG_, G, sizeof(double) * B * n_ * n_);
  arena_.upload(dg0_, g0, sizeof(double) * B * n_);
  if (p_) {
    arena_.upload(dCE_, CE, sizeof(double) * B * n_ * p_);
    arena_.upload(dce0_, ce0, sizeof(double) * B * p_);
  }
  if (m_) {
    arena_.upload(dCI_, CI, sizeof(double) * B * n_ * m_);
    arena_.upload(dci0_, ci0, sizeof(double) * B * m_);
  }
  abi_ok(qloco_eiquadprog_solve(n_, p_, m_, batch, dG_, (int64_t)n_ * n_, dg0_, n_,
                                p_ ? dCE_ : nullptr, (int64_t)n_ * p_, p_ ? dce0_ : nullptr, p_,
                                m_ ? dCI_ : nullptr, (int64_t)n_ * m_, m_ ? dci0_ : nullptr, m_,
                                dX_, df_, dst_, dit_, arena_.stream()),
         "qloco_eiquadprog_solve");
  arena_.download(X, dX_, sizeof(double) * B * n_);
  std::vector<double> fh(B);
  std::vector<int32_t> sh(B), ih(B);
  arena_.download(fh.data(), df_, sizeof(double) * B);
  arena_.download(sh.data(), dst_, sizeof(int32_t) * B);
  arena_.download(ih.data(), dit_, sizeof(int32_t) * B);
  arena_.sync();
  if (f) std::memcpy(f, fh.data(), sizeof(double) * B);
  if (status) std::memcpy(status, sh.data(), sizeof(int32_t) * B);
  last_status_ = sh[B - 1];
  last_iters_ = ih[B - 1];
}

double QPsolverGpu::solve(const double *G, const double *g0, const double *CE, const double *ce0,
                          const double *CI, const double *ci0, double *X) {
  double f = 0.0;
  solve_batch(1, G, g0, CE, ce0, CI, ci0, X, &f, nullptr);
  return f;
}

void QPBaseClassGpu::resizeQP(const int &nv, const int &ne, const int &ni) {
  nVars = nv;
  nEq = ne;
  nIneq = ni;
  G.assign((size_t)nv * nv, 0.0);
  g0.assign(nv, 0.0);
  CE.assign((size_t)nv * ne, 0.0);
  ce0.assign(ne, 0.0);
  CI.assign((size_t)nv * ni, 0.0);
  ci0.assign(ni, 0.0);
  X.assign(nv, 0.0);
  solver_.resize(nv, ne, ni);
}

bool QPBaseClassGpu::solveQP() {  // QPBaseClass.cpp:126-152
  solver_.solve(G.data(), g0.data(), CE.data(), ce0.data(), CI.data(), ci0.data(), X.data());
  for (double v : X)
    if (std::isnan(v)) return false;
  return true;
}

// ---------------------------------------------------------------- Dynamiccclass
Dynamiccclass::Dynamiccclass(int batch, const qloco_force_params *params) : batch_(batch) {
  if (batch < 1) throw Error("Dynamiccclass: batch < 1", QLOCO_ERR_ARG);
  if (params) prm_ = *params;
  else qloco_force_params_default(&prm_);
  const size_t B = batch;
  grf_opt.assign(B * 12, 0.0);
  F_leg_ref.assign(B * 12, 0.0);
  F_leg_guess.assign(B * 12, 0.0);
  qp_solution.assign(B, 1);
  status.assign(B, 0);
  iters.assign(B, 0);
  h_com_.assign(B * 3, 0.0);
  h_leg_.assign(B * 12, 0.0);
  h_F_.assign(B * 6, 0.0);
  h_rf_.assign(B * 3, 0.0);
  h_lf_.assign(B * 3, 0.0);
  h_base_.assign(B * 3, 0.0);
  h_feet_.assign(B * 12, 0.0);
  h_FT_.assign(B * 6, 0.0);
  h_y_.assign(B, 0.0);
  h_mode_.assign(B, 0);
  h_rs_.assign(B, 2);
  d_com_ = dalloc<double>(arena_, B * 3);
  d_leg_ = dalloc<double>(arena_, B * 12);
  d_F_ = dalloc<double>(arena_, B * 6);
  d_rf_ = dalloc<double>(arena_, B * 3);
  d_lf_ = dalloc<double>(arena_, B * 3);
  d_base_ = dalloc<double>(arena_, B * 3);
  d_feet_ = dalloc<double>(arena_, B * 12);
  d_FT_ = dalloc<double>(arena_, B * 6);
  d_y_ = dalloc<double>(arena_, B);
  d_Fref_ = dalloc<double>(arena_, B * 12);
  d_grf_ = dalloc<double>(arena_, B * 12);
  d_guess_ = dalloc<double>(arena_, B * 12);
  d_mode_ = dalloc<int32_t>(arena_, B);
  d_rs_ = dalloc<int32_t>(arena_, B);
  d_qps_ = dalloc<int32_t>(arena_, B);
  d_st_ = dalloc<int32_t>(arena_, B);
  d_it_ = dalloc<int32_t>(arena_, B);
  // the grouped launch's workspace (previous iteration counts carried between calls)
  const size_t nord = (size_t)qloco_force_order_ws_len(batch);
  d_ord_ = dalloc<int32_t>(arena_, nord);
  hip_ok(hipMemsetAsync(d_ord_, 0, sizeof(int32_t) * nord, (hipStream_t)arena_.stream()), "order workspace");
  // member state starts at zero (Dynamiccclass ctor, dynmics_compute.cpp:29-100)
  arena_.upload(d_Fref_, F_leg_ref.data(), sizeof(double) * B * 12);
  arena_.upload(d_grf_, grf_opt.data(), sizeof(double) * B * 12);
  arena_.sync();
}

void Dynamiccclass::force_distribution(const double com_des[3], const double leg_des[12],
                                       const double F_force_des[6], int mode,
                                       double y_coefficient, const double rfoot_des[3],
                                       const double lfoot_des[3], int r) {
  if (r < 0 || r >= batch_) throw Error("Dynamiccclass: robot index", QLOCO_ERR_ARG);
  std::memcpy(&h_com_[r * 3], com_des, sizeof(double) * 3);
  std::memcpy(&h_leg_[r * 12], leg_des, sizeof(double) * 12);
  std::memcpy(&h_F_[r * 6], F_force_des, sizeof(double) * 6);
  std::memcpy(&h_rf_[r * 3], rfoot_des, sizeof(double) * 3);
  std::memcpy(&h_lf_[r * 3], lfoot_des, sizeof(double) * 3);
  h_mode_[r] = mode;
  h_y_[r] = y_coefficient;
}

void Dynamiccclass::force_opt(const double base_p[3], const double FR_p[3], const double FL_p[3],
                              const double RR_p[3], const double RL_p[3],
                              const double FT_total_des[6], int mode, int right_support,
                              double y_coefficient, int r) {
  if (r < 0 || r >= batch_) throw Error("Dynamiccclass: robot index", QLOCO_ERR_ARG);
  std::memcpy(&h_base_[r * 3], base_p, sizeof(double) * 3);
  std::memcpy(&h_feet_[r * 12 + 0], FR_p, sizeof(double) * 3);
  std::memcpy(&h_feet_[r * 12 + 3], FL_p, sizeof(double) * 3);
  std::memcpy(&h_feet_[r * 12 + 6], RR_p, sizeof(double) * 3);
  std::memcpy(&h_feet_[r * 12 + 9], RL_p, sizeof(double) * 3);
  std::memcpy(&h_FT_[r * 6], FT_total_des, sizeof(double) * 6);
  h_mode_[r] = mode;  // force_opt's own mode / y_coefficient arguments (:265)
  h_rs_[r] = right_support;
  h_y_[r] = y_coefficient;
  if (r == batch_ - 1) run();
}

void Dynamiccclass::run() {
  const size_t B = batch_;
  arena_.upload(d_com_, h_com_.data(), sizeof(double) * B * 3);
  arena_.upload(d_leg_, h_leg_.data(), sizeof(double) * B * 12);
  arena_.upload(d_F_, h_F_.data(), sizeof(double) * B * 6);
  arena_.upload(d_rf_, h_rf_.data(), sizeof(double) * B * 3);
  arena_.upload(d_lf_, h_lf_.data(), sizeof(double) * B * 3);
  arena_.upload(d_base_, h_base_.data(), sizeof(double) * B * 3);
  arena_.upload(d_feet_, h_feet_.data(), sizeof(double) * B * 12);
  arena_.upload(d_FT_, h_FT_.data(), sizeof(double) * B * 6);
  arena_.upload(d_y_, h_y_.data(), sizeof(double) * B);
  arena_.upload(d_mode_, h_mode_.data(), sizeof(int32_t) * B);
  arena_.upload(d_rs_, h_rs_.data(), sizeof(int32_t) * B);
  abi_ok(qloco_force_qp_solve_ordered(&prm_, batch_, d_com_, d_leg_, d_F_, d_rf_, d_lf_, d_base_,
                                      d_feet_, d_FT_, d_mode_, d_rs_, d_y_, d_Fref_, d_grf_, d_guess_,
                                      d_qps_, d_st_, d_it_, d_ord_, arena_.stream()),
         "qloco_force_qp_solve_ordered");
  arena_.download(grf_opt.data(), d_grf_, sizeof(double) * B * 12);
  arena_.download(F_leg_ref.data(), d_Fref_, sizeof(double) * B * 12);
  arena_.download(F_leg_guess.data(), d_guess_, sizeof(double) * B * 12);
  arena_.download(qp_solution.data(), d_qps_, sizeof(int32_t) * B);
  arena_.download(status.data(), d_st_, sizeof(int32_t) * B);
  arena_.download(iters.data(), d_it_, sizeof(int32_t) * B);
  arena_.sync();
}

void Dynamiccclass::compute_joint_torques(const double *Jaco, const int32_t *swing,
                                          const double *p_des, const double *p_est,
                                          const double *pv_des, const double *pv_est,
                                          double *tau) {
  const size_t B = batch_;
  if (!d_jt_) {
    d_jt_ = dalloc<double>(arena_, B * (36 + 48 + 12));
    d_sw_ = dalloc<int32_t>(arena_, B * 4);
  }
  double *dJ = d_jt_, *dp = d_jt_ + B * 36, *dtau = d_jt_ + B * 84;
  int32_t *dsw = d_sw_;
  arena_.upload(dJ, Jaco, sizeof(double) * B * 36);
  arena_.upload(dsw, swing, sizeof(int32_t) * B * 4);
  arena_.upload(dp, p_des, sizeof(double) * B * 12);
  arena_.upload(dp + B * 12, p_est, sizeof(double) * B * 12);
  arena_.upload(dp + B * 24, pv_des, sizeof(double) * B * 12);
  arena_.upload(dp + B * 36, pv_est, sizeof(double) * B * 12);
  abi_ok(qloco_joint_torques(batch_, dJ, dsw, dp, dp + B * 12, dp + B * 24, dp + B * 36, d_Fref_,
                             dtau, arena_.stream()),
         "qloco_joint_torques");
  arena_.download(tau, dtau, sizeof(double) * B * 12);
  arena_.sync();
}

// ---------------------------------------------------------------- PRMPCClass
PRMPCClass::PRMPCClass(int batch) : batch_(batch) {
  if (batch < 1) throw Error("PRMPCClass: batch < 1", QLOCO_ERR_ARG);
  const size_t B = batch;
  state.assign(B * QLOCO_BODY_STATE_LEN, 0.0);
  abi_ok(qloco_body_state_init_host(batch, state.data()), "qloco_body_state_init_host");
  d_state_ = dalloc<double>(arena_, B * QLOCO_BODY_STATE_LEN);
  d_in_ = dalloc<double>(arena_, B * (4 + 4 * 10 + 15));
  d_traj_ = dalloc<double>(arena_, B * 14);
  d_t_ = dalloc<double>(arena_, 1);
  d_i_ = dalloc<int32_t>(arena_, B);
  d_st_ = dalloc<int32_t>(arena_, B);
  d_j_ = dalloc<int32_t>(arena_, 1);
  arena_.upload(d_state_, state.data(), sizeof(double) * B * QLOCO_BODY_STATE_LEN);
  arena_.sync();
}

void PRMPCClass::body_theta_mpc_batch(const int32_t *i, const double *bs, const double *zmp,
                                      const double *ang, const double *rf, const double *lf,
                                      const double *acc, double *com_traj) {
  const size_t B = batch_;
  double *d_bs = d_in_, *d_zmp = d_bs + B * 4, *d_ang = d_zmp + B * 10, *d_rf = d_ang + B * 10,
         *d_lf = d_rf + B * 10, *d_acc = d_lf + B * 10;
  arena_.upload(d_i_, i, sizeof(int32_t) * B);
  arena_.upload(d_bs, bs, sizeof(double) * B * 4);
  arena_.upload(d_zmp, zmp, sizeof(double) * B * 10);
  arena_.upload(d_ang, ang, sizeof(double) * B * 10);
  arena_.upload(d_rf, rf, sizeof(double) * B * 10);
  arena_.upload(d_lf, lf, sizeof(double) * B * 10);
  arena_.upload(d_acc, acc, sizeof(double) * B * 15);
  abi_ok(qloco_body_mpc_step(batch_, d_i_, d_bs, d_zmp, d_ang, d_rf, d_lf, d_acc, d_state_,
                             d_traj_, d_st_, arena_.stream()),
         "qloco_body_mpc_step");
  arena_.download(com_traj, d_traj_, sizeof(double) * B * 14);
  arena_.download(state.data(), d_state_, sizeof(double) * B * QLOCO_BODY_STATE_LEN);
  arena_.sync();
}

std::array<double, 14> PRMPCClass::body_theta_mpc(int i, const double bodyangle_state[4],
                                                  const double zmp_ref[10],
                                                  const double angle_ref[10],
                                                  const double rfoot_ref[10],
                                                  const double lfoot_ref[10],
                                                  const double comacc_ref[15],
                                                  const double * /*Nrtfoorpr_gen*/) {
  if (batch_ != 1) throw Error("PRMPCClass::body_theta_mpc: use body_theta_mpc_batch", QLOCO_ERR_ARG);
  std::array<double, 14> out{};
  const int32_t ii = i;
  body_theta_mpc_batch(&ii, bodyangle_state, zmp_ref, angle_ref, rfoot_ref, lfoot_ref, comacc_ref,
                       out.data());
  return out;
}

int PRMPCClass::Indexfind(double goal_P) {
  int32_t j = 0;
  arena_.upload(d_t_, &goal_P, sizeof(double));
  abi_ok(qloco_body_indexfind(1, d_t_, d_j_, arena_.stream()), "qloco_body_indexfind");
  arena_.download(&j, d_j_, sizeof(int32_t));
  arena_.sync();
  return j;
}

// ---------------------------------------------------------------- ConvexMpcBatch
// argument check in the member-initialiser list: batch_ is declared before
// the DeviceArena, so a bad batch is refused before any device call
static int positive_batch(int batch, const char *who) {
  if (batch < 1) throw Error(std::string(who) + ": batch < 1", QLOCO_ERR_ARG);
  return batch;
}

ConvexMpcBatch::ConvexMpcBatch(int batch, const qloco_srbd_spec *sp)
    : batch_(positive_batch(batch, "ConvexMpcBatch")) {
  if (sp) {
    spec = *sp;
  } else {
    qloco_srbd_spec_default(&spec);
    spec.warm_start = 2;       // the reference's persistent member solver
    spec.literal_full_qp = 1;  // on its literal 12N-variable QP (update path every call)
  }
  if (spec.horizon < 1 || spec.horizon > 20)
    throw Error("ConvexMpcBatch: horizon outside 1..20", QLOCO_BAD_SIZE);
  if (spec.warm_start < 0 || spec.warm_start > 2)
    throw Error("ConvexMpcBatch: warm_start outside 0..2", QLOCO_ERR_ARG);
  // the device buffers (x_ref, the persistent record) are sized from these:
  // later edits of the public spec are checked against them on every call
  horizon_ = spec.horizon;
  warm_mode_ = spec.warm_start;
  spec.feet_per_step = 0;      // compute_grf passes one foot_pos_abs (:527-531)
  spec.contacts_per_step = 0;  // and one contacts[4] (ConvexMpc.cpp:232-249)
  spec.output_frame = 1;       // root_rot_mat' u (:596-599)
  const size_t B = batch, N = spec.horizon;
  d_x0_ = dalloc<float>(arena_, B * 13);
  d_xr_ = dalloc<float>(arena_, B * 13 * N);
  d_feet_ = dalloc<float>(arena_, B * 12);
  d_ct_ = dalloc<uint8_t>(arena_, B * 4);
  d_u0_ = dalloc<float>(arena_, B * 12);
  d_st_ = dalloc<int32_t>(arena_, B);
  d_it_ = dalloc<int32_t>(arena_, B);
  if (spec.warm_start == 2) {  // per-robot persistent solver record
    d_rec_ = dalloc<float>(arena_, B * QLOCO_SRBD_PERSIST_LEN(N));
    reset();
  }
  status.assign(B, 0);
  iters.assign(B, 0);
}

static int shard_count_of(int64_t total, int world, int rank, int mode) {
  int64_t count = 0;
  if (qloco_mgpu_shard(total, world, rank, mode, nullptr, &count, nullptr) != QLOCO_OK)
    throw Error("ConvexMpcBatch: invalid shard (total, world, rank, mode)", QLOCO_ERR_ARG);
  if (count < 1 || count > INT32_MAX)
    throw Error("ConvexMpcBatch: this rank's shard is empty or too large", QLOCO_BAD_SIZE);
  return (int)count;
}

ConvexMpcBatch::ConvexMpcBatch(int64_t total, int world, int rank, const uint8_t *comm_id,
                               int shard_mode, const qloco_srbd_spec *sp)
    : ConvexMpcBatch(shard_count_of(total, world, rank, shard_mode), sp) {
  abi_ok(qloco_mgpu_shard(total, world, rank, shard_mode, &shard_first, &shard_count, &shard_stride),
         "qloco_mgpu_shard");
  total_ = total;
  d_u0_all_ = dalloc<float>(arena_, (size_t)total * 12);
  d_st_all_ = dalloc<int32_t>(arena_, (size_t)total);
  d_it_all_ = dalloc<int32_t>(arena_, (size_t)total);
  all_forces_.assign((size_t)total * 12, 0.0);
  abi_ok(qloco_mgpu_init(&mg_, comm_id, world, rank, total, shard_mode), "qloco_mgpu_init");
}

ConvexMpcBatch::~ConvexMpcBatch() {
  if (mg_) qloco_mgpu_destroy(mg_);
}

void ConvexMpcBatch::check_spec() const {
  if (spec.horizon != horizon_)
    throw Error("ConvexMpcBatch: spec.horizon changed after construction (buffers sized for " +
                    std::to_string(horizon_) + ")", QLOCO_ERR_ARG);
  if (spec.warm_start != warm_mode_)
    throw Error("ConvexMpcBatch: spec.warm_start changed after construction", QLOCO_ERR_ARG);
}

void ConvexMpcBatch::reset() {
  if (!d_rec_) return;
  hip_ok(hipMemsetAsync(d_rec_, 0,
                        sizeof(float) * (size_t)batch_ * QLOCO_SRBD_PERSIST_LEN(horizon_),
                        (hipStream_t)arena_.stream()),
         "hipMemsetAsync");
}

void ConvexMpcBatch::solve_device(const float *x0, const float *x_ref, const float *feet,
                                  const uint8_t *contacts, float *u0, int32_t *st, int32_t *it) {
  check_spec();
  if (mg_)
    throw Error("ConvexMpcBatch::solve_device: a multi-GPU object solves through compute_grf "
                "(or qloco_mgpu_solve directly)", QLOCO_ERR_ARG);
  const int32_t legs = 4 * horizon_;  // constant contacts over the horizon: 4N worst case
  abi_ok(qloco_srbd_solve_ex(&spec, batch_, x0, x_ref, feet, contacts, u0, nullptr, st, it,
                             nullptr, nullptr, d_rec_, legs, arena_.stream()),
         "qloco_srbd_solve_ex");
}

void ConvexMpcBatch::compute_grf(const A1MpcState *s, double *forces) {
  check_spec();
  const size_t B = batch_, N = horizon_;
  const double dt = spec.dt;
  std::vector<float> x0(B * 13), xr(B * 13 * N), feet(B * 12);
  std::vector<uint8_t> ct(B * 4);
  int maxlegs = 0;
  for (size_t b = 0; b < B; ++b) {
    const A1MpcState &st = s[b];
    float *X = &x0[b * 13];  // mpc_states (:459-463)
    for (int k = 0; k < 3; ++k) {
      X[k] = (float)st.root_euler[k];
      X[3 + k] = (float)st.root_pos[k];
      X[6 + k] = (float)st.root_ang_vel[k];
      X[9 + k] = (float)st.root_lin_vel[k];
    }
    X[12] = -9.8f;
    // root_lin_vel_d_world = root_rot_mat * root_lin_vel_d (:479), before the
    // yaw overwrite of root_rot_mat (:502-510, done inside the kernel)
    double vw[3];
    for (int r = 0; r < 3; ++r)
      vw[r] = st.root_rot_mat[0 * 3 + r] * st.root_lin_vel_d[0] +
              st.root_rot_mat[1 * 3 + r] * st.root_lin_vel_d[1] +
              st.root_rot_mat[2 * 3 + r] * st.root_lin_vel_d[2];
    for (size_t i = 0; i < N; ++i) {  // mpc_states_d (:480-497)
      float *R = &xr[b * 13 * N + 13 * i];
      const double k = dt * (double)(i + 1);
      R[0] = (float)st.root_euler_d[0];
      R[1] = (float)st.root_euler_d[1];
      R[2] = (float)(st.root_euler[2] + st.root_ang_vel_d[2] * k);
      R[3] = (float)(st.root_pos[0] + vw[0] * k);
      R[4] = (float)(st.root_pos[1] + vw[1] * k);
      R[5] = (float)st.root_pos_d[2];
      R[6] = (float)st.root_ang_vel_d[0];
      R[7] = (float)st.root_ang_vel_d[1];
      R[8] = (float)st.root_ang_vel_d[2];
      R[9] = (float)vw[0];
      R[10] = (float)vw[1];
      R[11] = 0.0f;
      R[12] = -9.8f;
    }
    int legs = 0;
    for (int l = 0; l < 4; ++l) {
      for (int c = 0; c < 3; ++c) feet[b * 12 + 3 * l + c] = (float)st.foot_pos_abs[3 * l + c];
      ct[b * 4 + l] = st.contacts[l] ? 1 : 0;
      legs += st.contacts[l] ? 1 : 0;
    }
    if (legs * (int)N > maxlegs) maxlegs = legs * (int)N;
  }
  arena_.upload(d_x0_, x0.data(), sizeof(float) * B * 13);
  arena_.upload(d_xr_, xr.data(), sizeof(float) * B * 13 * N);
  arena_.upload(d_feet_, feet.data(), sizeof(float) * B * 12);
  arena_.upload(d_ct_, ct.data(), B * 4);
  if (mg_) {  // this rank's shard, then one all-gather of every robot's u0
    abi_ok(qloco_mgpu_solve(mg_, &spec, d_x0_, d_xr_, d_feet_, d_ct_, d_rec_, d_u0_all_, d_st_all_,
                            d_it_all_, maxlegs, arena_.stream()),
           "qloco_mgpu_solve");
    const size_t T = (size_t)total_;
    std::vector<float> ua(T * 12);
    std::vector<int32_t> sa(T), ia(T);
    arena_.download(ua.data(), d_u0_all_, sizeof(float) * T * 12);
    arena_.download(sa.data(), d_st_all_, sizeof(int32_t) * T);
    arena_.download(ia.data(), d_it_all_, sizeof(int32_t) * T);
    arena_.sync();
    for (size_t g = 0; g < T; ++g)
      for (int l = 0; l < 4; ++l) {
        const float *f = &ua[g * 12 + 3 * l];
        if (std::isnan(f[0]) || std::isnan(f[1]) || std::isnan(f[2])) continue;  // :597 guard
        for (int c = 0; c < 3; ++c) all_forces_[g * 12 + 3 * l + c] = f[c];
      }
    for (size_t b = 0; b < B; ++b) {
      const size_t g = (size_t)(shard_first + (int64_t)b * shard_stride);
      status[b] = sa[g];
      iters[b] = ia[g];
      for (int l = 0; l < 4; ++l) {
        const float *f = &ua[g * 12 + 3 * l];
        if (std::isnan(f[0]) || std::isnan(f[1]) || std::isnan(f[2])) continue;
        for (int c = 0; c < 3; ++c) forces[b * 12 + 3 * l + c] = f[c];
      }
    }
    return;
  }
  abi_ok(qloco_srbd_solve_ex(&spec, batch_, d_x0_, d_xr_, d_feet_, d_ct_, d_u0_, nullptr, d_st_,
                             d_it_, nullptr, nullptr, d_rec_, maxlegs, arena_.stream()),
         "qloco_srbd_solve_ex");
  std::vector<float> u0(B * 12);
  arena_.download(u0.data(), d_u0_, sizeof(float) * B * 12);
  arena_.download(status.data(), d_st_, sizeof(int32_t) * B);
  arena_.download(iters.data(), d_it_, sizeof(int32_t) * B);
  arena_.sync();
  for (size_t b = 0; b < B; ++b)
    for (int l = 0; l < 4; ++l) {
      const float *f = &u0[b * 12 + 3 * l];
      if (std::isnan(f[0]) || std::isnan(f[1]) || std::isnan(f[2])) continue;  // :597 guard
      for (int c = 0; c < 3; ++c) forces[b * 12 + 3 * l + c] = f[c];
    }
}


// ---------------------------------------------------------------- A1QpBatch
A1QpBatch::A1QpBatch(int batch, const qloco_a1_params *p)
    : batch_(positive_batch(batch, "A1QpBatch")) {
  if (p) params = *p;
  else qloco_a1_params_default(&params);
  const size_t B = batch;
  d_state_ = dalloc<double>(arena_, B * QLOCO_A1_STATE_LEN);
  d_forces_ = dalloc<double>(arena_, B * 12);
  d_ct_ = dalloc<uint8_t>(arena_, B * 4);
  d_st_ = dalloc<int32_t>(arena_, B);
  d_it_ = dalloc<int32_t>(arena_, B);
  status.assign(B, 0);
  iters.assign(B, 0);
}

void A1QpBatch::compute_grf(const A1QpState *s, double *forces) {
  const size_t B = batch_;
  std::vector<double> st(B * QLOCO_A1_STATE_LEN);
  std::vector<uint8_t> ct(B * 4);
  for (size_t b = 0; b < B; ++b) {  // the record layout of include/qloco.h section 9
    double *r = &st[b * QLOCO_A1_STATE_LEN];
    const double *src[8] = {s[b].root_pos,     s[b].root_pos_d,     s[b].root_euler,
                            s[b].root_euler_d, s[b].root_lin_vel,   s[b].root_lin_vel_d,
                            s[b].root_ang_vel, s[b].root_ang_vel_d};
    for (int f = 0; f < 8; ++f)
      for (int k = 0; k < 3; ++k) r[3 * f + k] = src[f][k];
    for (int k = 0; k < 9; ++k) {
      r[24 + k] = s[b].root_rot_mat[k];
      r[33 + k] = s[b].root_rot_mat_z[k];
    }
    for (int k = 0; k < 12; ++k) r[42 + k] = s[b].foot_pos_abs[k];
    for (int l = 0; l < 4; ++l) ct[b * 4 + l] = s[b].contacts[l] ? 1 : 0;
  }
  arena_.upload(d_state_, st.data(), sizeof(double) * st.size());
  arena_.upload(d_ct_, ct.data(), ct.size());
  abi_ok(qloco_a1_qp_solve(&params, batch_, d_state_, d_ct_, d_forces_, nullptr, d_st_, d_it_,
                           nullptr, nullptr, arena_.stream()),
         "qloco_a1_qp_solve");
  arena_.download(forces, d_forces_, sizeof(double) * B * 12);
  arena_.download(status.data(), d_st_, sizeof(int32_t) * B);
  arena_.download(iters.data(), d_it_, sizeof(int32_t) * B);
  arena_.sync();
}


// ------------------------------------------------------------------------
// Kinematicclass -> qloco_leg_fk / qloco_leg_ik
Kinematicclass::Kinematicclass(int max_legs) : cap_(0) {
  if (max_legs < 1) throw Error("Kinematicclass: max_legs < 1", QLOCO_ERR_ARG);
  ensure(max_legs);
}

void Kinematicclass::ensure(int n) {
  if (n <= cap_) return;
  const size_t N = n;
  d_a_ = dalloc<double>(arena_, N * 3);
  d_b_ = dalloc<double>(arena_, N * 3);
  d_p_ = dalloc<double>(arena_, N * 3);
  d_r_ = dalloc<double>(arena_, N * 3);
  d_q_ = dalloc<double>(arena_, N * 3);
  d_pos_ = dalloc<double>(arena_, N * 3);
  d_jac_ = dalloc<double>(arena_, N * 9);
  d_leg_ = dalloc<int32_t>(arena_, N);
  d_upd_ = dalloc<int32_t>(arena_, N);
  cap_ = n;
}

void Kinematicclass::forward_batch(int n, const double *q, const int32_t *leg,
                                   const double *body_p, const double *body_r, double *pos,
                                   double *jac) {
  if (n < 0 || (n > 0 && (!q || !leg || !pos)) || ((body_p == nullptr) != (body_r == nullptr)))
    throw Error("Kinematicclass::forward_batch: bad arguments", QLOCO_ERR_ARG);
  if (n == 0) return;
  ensure(n);
  const size_t N = n;
  const bool g = body_p != nullptr;
  arena_.upload(d_q_, q, sizeof(double) * N * 3);
  arena_.upload(d_leg_, leg, sizeof(int32_t) * N);
  if (g) {
    arena_.upload(d_p_, body_p, sizeof(double) * N * 3);
    arena_.upload(d_r_, body_r, sizeof(double) * N * 3);
  }
  abi_ok(qloco_leg_fk(n, d_q_, d_leg_, g ? d_p_ : nullptr, g ? d_r_ : nullptr, d_pos_,
                      jac ? d_jac_ : nullptr, arena_.stream()),
         "qloco_leg_fk");
  arena_.download(pos, d_pos_, sizeof(double) * N * 3);
  if (jac) arena_.download(jac, d_jac_, sizeof(double) * N * 9);
  arena_.sync();
}

void Kinematicclass::inverse_batch(int n, const double *pos_des, const double *q_ini,
                                   const int32_t *leg, const double *body_p,
                                   const double *body_r, double *q_out, double *pos_out,
                                   double *jac, int32_t *updates) {
  if (n < 0 || (n > 0 && (!pos_des || !q_ini || !leg || !q_out)) ||
      ((body_p == nullptr) != (body_r == nullptr)))
    throw Error("Kinematicclass::inverse_batch: bad arguments", QLOCO_ERR_ARG);
  if (n == 0) return;
  ensure(n);
  const size_t N = n;
  const bool g = body_p != nullptr;
  arena_.upload(d_a_, pos_des, sizeof(double) * N * 3);
  arena_.upload(d_b_, q_ini, sizeof(double) * N * 3);
  arena_.upload(d_leg_, leg, sizeof(int32_t) * N);
  if (g) {
    arena_.upload(d_p_, body_p, sizeof(double) * N * 3);
    arena_.upload(d_r_, body_r, sizeof(double) * N * 3);
  }
  abi_ok(qloco_leg_ik(n, d_a_, d_b_, d_leg_, g ? d_p_ : nullptr, g ? d_r_ : nullptr, d_q_, d_pos_,
                      d_jac_, d_upd_, arena_.stream()),
         "qloco_leg_ik");
  arena_.download(q_out, d_q_, sizeof(double) * N * 3);
  if (pos_out) arena_.download(pos_out, d_pos_, sizeof(double) * N * 3);
  if (jac) arena_.download(jac, d_jac_, sizeof(double) * N * 9);
  if (updates) arena_.download(updates, d_upd_, sizeof(int32_t) * N);
  arena_.sync();
}

std::array<double, 3> Kinematicclass::Forward_kinematics(const double q_joint[3], int feet_flag) {
  std::array<double, 3> p{};
  const int32_t leg = feet_flag;
  forward_batch(1, q_joint, &leg, nullptr, nullptr, p.data(), Jacobian_kin.data());
  return p;
}

std::array<double, 3> Kinematicclass::Forward_kinematics_g(const double body_P[3],
                                                           const double body_R[3],
                                                           const double q_joint[3],
                                                           int feet_flag) {
  std::array<double, 3> p{};
  const int32_t leg = feet_flag;
  forward_batch(1, q_joint, &leg, body_P, body_R, p.data(), Jacobian_kin.data());
  return p;
}

std::array<double, 3> Kinematicclass::Inverse_kinematics(const double pos_des[3],
                                                         const double q_ini[3], int feet_flag) {
  std::array<double, 3> q{};
  const int32_t leg = feet_flag;
  int32_t upd = 0;
  inverse_batch(1, pos_des, q_ini, &leg, nullptr, nullptr, q.data(), pos_cal.data(),
                Jacobian_kin.data(), &upd);
  last_updates = upd;
  return q;
}

std::array<double, 3> Kinematicclass::Inverse_kinematics_g(const double body_P[3],
                                                           const double body_R[3],
                                                           const double pos_des[3],
                                                           const double q_ini[3],
                                                           int feet_flag) {
  std::array<double, 3> q{};
  const int32_t leg = feet_flag;
  int32_t upd = 0;
  inverse_batch(1, pos_des, q_ini, &leg, body_P, body_R, q.data(), pos_cal.data(),
                Jacobian_kin.data(), &upd);
  last_updates = upd;
  return q;
}


// ---------------------------------------------------------------- RtMpcNode
RtMpcNode::RtMpcNode(int batch) : batch_(batch) {
  if (batch < 1) throw Error("RtMpcNode: batch < 1", QLOCO_ERR_ARG);
  const size_t B = batch;
  gait_.assign(B * QLOCO_GAIT_MSG_LEN, 0.0);  // low_mpc_gait.setZero() (gait_fast.cpp:387)
  ctrl_.assign(B * QLOCO_CTRL_MSG_LEN, 0.0);
  traj.assign(B * QLOCO_TRAJ_MSG_LEN, 0.0);
  nrt.assign(B * QLOCO_NRT_MSG_LEN, 0.0);
  sched.assign(B * QLOCO_RT_SCHED_LEN, 0);
  const int64_t ws = qloco_rt_workspace_bytes(batch);
  if (ws < 0) throw Error("qloco_rt_workspace_bytes", QLOCO_ERR_ARG);
  d_ws_ = arena_.alloc((size_t)ws);
  d_gait_ = dalloc<double>(arena_, B * QLOCO_GAIT_MSG_LEN);
  d_ctrl_ = dalloc<double>(arena_, B * QLOCO_CTRL_MSG_LEN);
  d_traj_ = dalloc<double>(arena_, B * QLOCO_TRAJ_MSG_LEN);
  d_nrt_ = dalloc<double>(arena_, B * QLOCO_NRT_MSG_LEN);
  d_sched_ = dalloc<int32_t>(arena_, B * QLOCO_RT_SCHED_LEN);
  abi_ok(qloco_rt_init(batch, d_ws_, arena_.stream()), "qloco_rt_init");
  arena_.sync();
}

void RtMpcNode::nrt_gait_sub_operation(const double msg[QLOCO_GAIT_MSG_LEN], int robot) {
  if (robot < 0 || robot >= batch_) throw Error("RtMpcNode: robot out of range", QLOCO_ERR_ARG);
  std::copy(msg, msg + QLOCO_GAIT_MSG_LEN, gait_.begin() + (size_t)robot * QLOCO_GAIT_MSG_LEN);
}

void RtMpcNode::control_gait_sub_operation(const double msg[QLOCO_CTRL_MSG_LEN], int robot) {
  if (robot < 0 || robot >= batch_) throw Error("RtMpcNode: robot out of range", QLOCO_ERR_ARG);
  std::copy(msg, msg + QLOCO_CTRL_MSG_LEN, ctrl_.begin() + (size_t)robot * QLOCO_CTRL_MSG_LEN);
}

void RtMpcNode::loop_once() {
  const size_t B = batch_;
  arena_.upload(d_gait_, gait_.data(), sizeof(double) * B * QLOCO_GAIT_MSG_LEN);
  arena_.upload(d_ctrl_, ctrl_.data(), sizeof(double) * B * QLOCO_CTRL_MSG_LEN);
  abi_ok(qloco_rt_tick(batch_, d_ws_, d_gait_, d_ctrl_, d_traj_, d_nrt_, nullptr, d_sched_,
                       arena_.stream()),
         "qloco_rt_tick");
  arena_.download(traj.data(), d_traj_, sizeof(double) * B * QLOCO_TRAJ_MSG_LEN);
  arena_.download(nrt.data(), d_nrt_, sizeof(double) * B * QLOCO_NRT_MSG_LEN);
  arena_.download(sched.data(), d_sched_, sizeof(int32_t) * B * QLOCO_RT_SCHED_LEN);
  arena_.sync();
}


// ---------------------------------------------------------------- ServoForceBlock
// double inputs, per robot: coma 3, com 3, rfoot 3, lfoot 3, body_p 3, foot 12,
// y 1, Jaco 36, rel_mea 12, v_est 12 (= 88); int inputs: rs, mode, count (3);
// double outputs: F_sum 6, FLR 6, grf 12, tau 12 (= 36); int outputs: swing 4, qps, status (6)
ServoForceBlock::ServoForceBlock(int batch, const qloco_force_params *params) : batch_(batch) {
  if (batch < 1) throw Error("ServoForceBlock: batch < 1", QLOCO_ERR_ARG);
  if (params) prm_ = *params;
  else qloco_force_params_default(&prm_);
  const size_t B = batch;
  F_sum.assign(B * 6, 0.0);
  Force_L_R.assign(B * 6, 0.0);
  grf_opt.assign(B * 12, 0.0);
  Legs_torque.assign(B * 12, 0.0);
  swing.assign(B * 4, 0);
  qp_solution.assign(B, 1);
  status.assign(B, 0);
  const int64_t ws = qloco_servo_workspace_bytes(batch);
  if (ws < 0) throw Error("qloco_servo_workspace_bytes", QLOCO_ERR_ARG);
  d_ws_ = arena_.alloc((size_t)ws);
  d_in_ = dalloc<double>(arena_, B * 88);
  d_out_ = dalloc<double>(arena_, B * 36);
  d_iin_ = dalloc<int32_t>(arena_, B * 3);
  d_iout_ = dalloc<int32_t>(arena_, B * 6);
  abi_ok(qloco_servo_init(batch, d_ws_, arena_.stream()), "qloco_servo_init");
  arena_.sync();
}

void ServoForceBlock::step(const double *coma_des, const double *com_des, const double *rfoot_des,
                           const double *lfoot_des, const double *body_p_des,
                           const double *foot_des, const int32_t *right_support,
                           const int32_t *gait_mode, const double *y_offset,
                           const int32_t *count_in_rt_loop, const double *Jaco,
                           const double *foot_rel_mea, const double *v_est_rel) {
  const size_t B = batch_;
  double *in = d_in_;
  double *coma = in, *com = coma + 3 * B, *rf = com + 3 * B, *lf = rf + 3 * B, *bp = lf + 3 * B,
         *ft = bp + 3 * B, *y = ft + 12 * B, *J = y + B, *rm = J + 36 * B, *ve = rm + 12 * B;
  int32_t *rs = d_iin_, *md = rs + B, *cnt = md + B;
  arena_.upload(coma, coma_des, sizeof(double) * 3 * B);
  arena_.upload(com, com_des, sizeof(double) * 3 * B);
  arena_.upload(rf, rfoot_des, sizeof(double) * 3 * B);
  arena_.upload(lf, lfoot_des, sizeof(double) * 3 * B);
  arena_.upload(bp, body_p_des, sizeof(double) * 3 * B);
  arena_.upload(ft, foot_des, sizeof(double) * 12 * B);
  arena_.upload(y, y_offset, sizeof(double) * B);
  arena_.upload(J, Jaco, sizeof(double) * 36 * B);
  arena_.upload(rm, foot_rel_mea, sizeof(double) * 12 * B);
  arena_.upload(ve, v_est_rel, sizeof(double) * 12 * B);
  arena_.upload(rs, right_support, sizeof(int32_t) * B);
  arena_.upload(md, gait_mode, sizeof(int32_t) * B);
  arena_.upload(cnt, count_in_rt_loop, sizeof(int32_t) * B);
  double *Fs = d_out_, *Fl = Fs + 6 * B, *g = Fl + 6 * B, *tau = g + 12 * B;
  int32_t *sw = d_iout_, *qps = sw + 4 * B, *st = qps + B;
  abi_ok(qloco_servo_force_block(&prm_, batch_, d_ws_, coma, com, rf, lf, bp, ft, rs, md, y, cnt,
                                 J, rm, ve, Fs, Fl, g, tau, sw, qps, st, arena_.stream()),
         "qloco_servo_force_block");
  arena_.download(F_sum.data(), Fs, sizeof(double) * 6 * B);
  arena_.download(Force_L_R.data(), Fl, sizeof(double) * 6 * B);
  arena_.download(grf_opt.data(), g, sizeof(double) * 12 * B);
  arena_.download(Legs_torque.data(), tau, sizeof(double) * 12 * B);
  arena_.download(swing.data(), sw, sizeof(int32_t) * 4 * B);
  arena_.download(qp_solution.data(), qps, sizeof(int32_t) * B);
  arena_.download(status.data(), st, sizeof(int32_t) * B);
  arena_.sync();
}

}  // namespace qloco
