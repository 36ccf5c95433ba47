// qloco_gen.cpp -- deterministic synthetic SRBD instances.
//
// Counter-based: every value is a pure function of (seed, instance id,
// field id), so any shard of the batch can be generated independently and
// every rank regenerates exactly its own slice.  Integer mixing plus IEEE
// double +,-,* only (no libm), compiled with -ffp-contract=off: the values
// are bit-identical on every x86-64 host.  The oracle carries an
// independent restatement (oracle/gen.c); tests compare the two.
#include <stdint.h>

#include "qloco.h"

namespace {

inline uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Stream {
  uint64_t key;
  double u(uint64_t field) const {
    const uint64_t h = mix64(key + field * 0xD1B54A32D192ED03ull);
    return static_cast<double>(h >> 11) * (1.0 / 9007199254740992.0);
  }
  double uniform(uint64_t field, double lo, double hi) const { return lo + (hi - lo) * u(field); }
  double normal(uint64_t field, double sigma) const {  // Irwin-Hall(12) - 6
    double s = 0.0;
    for (int j = 0; j < 12; ++j) s += u(1000 + field * 16 + j);
    return (s - 6.0) * sigma;
  }
};

// Go1 homing feet relative to the CoM (q = (0, 0.87, -1.5), Kinematics.cpp:124-126),
// ConvexMpc leg order FL, FR, RL, RR.
constexpr double kNominalFeet[4][3] = {{0.150786, 0.12675, -0.309458},
                                       {0.150786, -0.12675, -0.309458},
                                       {-0.225414, 0.12675, -0.309458},
                                       {-0.225414, -0.12675, -0.309458}};

constexpr uint8_t kTrot[2][4] = {{1, 0, 0, 1}, {0, 1, 1, 0}};  // {FL,RR} / {FR,RL}
constexpr uint8_t kPace[2][4] = {{1, 0, 1, 0}, {0, 1, 0, 1}};  // {FL,RL} / {FR,RR}

}  // namespace

extern "C" int qloco_gen_srbd_host_strided(uint64_t seed, int32_t N, float dt_f, int32_t gait,
                                           int64_t first, int64_t stride, int64_t count, float *x0,
                                           float *x_ref, float *feet, uint8_t *contacts) {
  if (N < 1 || count < 0 || stride < 1 || first < 0 || !x0 || !x_ref || !feet || !contacts)
    return QLOCO_ERR_ARG;
  const double dt = static_cast<double>(dt_f);
  for (int64_t t = 0; t < count; ++t) {
    const int64_t inst = first + t * stride;
    const Stream S{mix64(seed + 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(inst + 1))};
    const double roll = S.uniform(0, -0.1, 0.1), pitch = S.uniform(1, -0.1, 0.1);
    const double yaw = S.uniform(2, -3.141592653589793, 3.141592653589793);
    const double p[3] = {S.uniform(3, -1, 1), S.uniform(4, -1, 1), S.uniform(5, 0.27, 0.33)};
    const double w[3] = {S.normal(6, 0.3), S.normal(7, 0.3), S.normal(8, 0.3)};
    const double v[3] = {S.normal(9, 0.3), S.normal(10, 0.3), S.normal(11, 0.3)};
    const double vdx = S.uniform(24, -0.5, 0.5), vdy = S.uniform(25, -0.3, 0.3);
    const double wdz = S.uniform(26, -0.5, 0.5);
    float *X = x0 + 13 * t;
    const double xs[13] = {roll, pitch, yaw, p[0], p[1], p[2], w[0], w[1], w[2], v[0], v[1], v[2], -9.8};
    for (int k = 0; k < 13; ++k) X[k] = static_cast<float>(xs[k]);
    // desired trajectory, compute_grf layout (A1RobotControl.cpp:480-497)
    for (int k = 0; k < N; ++k) {
      float *R = x_ref + static_cast<int64_t>(13) * N * t + 13 * k;
      const double tk = dt * static_cast<double>(k + 1);
      const double r[13] = {0.0, 0.0, yaw + wdz * tk, p[0] + vdx * tk, p[1] + vdy * tk, 0.30,
                            0.0, 0.0, wdz, vdx, vdy, 0.0, -9.8};
      for (int s = 0; s < 13; ++s) R[s] = static_cast<float>(r[s]);
    }
    for (int leg = 0; leg < 4; ++leg)
      for (int c = 0; c < 3; ++c)
        feet[12 * t + 3 * leg + c] =
            static_cast<float>(kNominalFeet[leg][c] + S.uniform(12 + 3 * leg + c, -0.02, 0.02));
    uint8_t *C = contacts + static_cast<int64_t>(4) * N * t;
    if (gait == 0 || gait == 1) {
      const uint8_t *pat = (gait == 0 ? kTrot : kPace)[inst & 1];
      for (int k = 0; k < N; ++k)
        for (int i = 0; i < 4; ++i) C[4 * k + i] = pat[i];
    } else if (gait == 2) {
      // mixed schedules: trot or pace, random phase in a 16-step cycle with
      // all-stance windows [0,2) and [8,10) (double support at each switch)
      const bool pace = S.u(27) < 0.5;
      const int phase = static_cast<int>(S.u(28) * 16.0);
      const uint8_t *A = (pace ? kPace : kTrot)[0], *B = (pace ? kPace : kTrot)[1];
      for (int k = 0; k < N; ++k) {
        const int ph = (phase + k) % 16;
        for (int i = 0; i < 4; ++i)
          C[4 * k + i] = (ph < 2 || (ph >= 8 && ph < 10)) ? 1 : (ph < 8 ? A[i] : B[i]);
      }
    } else {
      for (int k = 0; k < 4 * N; ++k) C[k] = 1;
    }
  }
  return QLOCO_OK;
}

extern "C" int qloco_gen_srbd_host(uint64_t seed, int32_t N, float dt_f, int32_t gait, int64_t first,
                                   int64_t count, float *x0, float *x_ref, float *feet,
                                   uint8_t *contacts) {
  return qloco_gen_srbd_host_strided(seed, N, dt_f, gait, first, 1, count, x0, x_ref, feet,
                                     contacts);
}
