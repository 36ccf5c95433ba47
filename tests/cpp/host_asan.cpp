// host_asan.cpp -- the C++ shim (quadrupedal_loco_amd/host/qloco_host.cpp)
// under AddressSanitizer + UBSan on a machine WITHOUT a GPU (test
// infrastructure; tests/test_sanitizers.py builds and runs it).  What runs
// here is everything the shim does before device work: constructor argument
// checks, the "no GPU" refusal of every class (no CPU fallback), and the C
// ABI's argument validation of every entry point.
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "qloco.hpp"

static int g_fail = 0;
#define CHECK(c, msg)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
      ++g_fail;                                         \
    }                                                   \
  } while (0)

static int status_of(const std::function<void()> &f) {
  try {
    f();
  } catch (const qloco::Error &e) {
    return e.status;
  }
  return 0;
}

int main() {
  // every device-owning class refuses to come up without a GPU
  const int nogpu = QLOCO_ERR_NO_GPU;
  CHECK(status_of([] { qloco::ConvexMpcBatch m(4); }) == nogpu, "ConvexMpcBatch");
  CHECK(status_of([] { qloco::A1QpBatch m(4); }) == nogpu, "A1QpBatch");
  CHECK(status_of([] { qloco::Dynamiccclass d(4); }) == nogpu, "Dynamiccclass");
  CHECK(status_of([] { qloco::Kinematicclass k(4); }) == nogpu, "Kinematicclass");
  CHECK(status_of([] { qloco::QPBaseClassGpu q; }) == nogpu, "QPBaseClassGpu");
  // constructor argument checks come first
  CHECK(status_of([] { qloco::ConvexMpcBatch m(0); }) == QLOCO_ERR_ARG, "batch 0");
  CHECK(status_of([] { qloco::A1QpBatch m(-3); }) == QLOCO_ERR_ARG, "batch -3");
  // C ABI validation (no device work)
  qloco_srbd_spec sp;
  qloco_srbd_spec_default(&sp);
  CHECK(qloco_srbd_solve(&sp, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                         nullptr, nullptr, nullptr, nullptr) == QLOCO_OK, "empty batch");
  sp.polish = 1;
  float dummy[64] = {0};
  uint8_t ct[4] = {1, 0, 0, 1};
  CHECK(qloco_srbd_solve(&sp, 1, dummy, dummy, dummy, ct, dummy, nullptr, nullptr, nullptr,
                         nullptr, nullptr, nullptr) == QLOCO_ERR_ARG, "polish refused");
  sp.polish = 0;
  sp.warm_start = 3;
  CHECK(qloco_srbd_solve(&sp, 1, dummy, dummy, dummy, ct, dummy, nullptr, nullptr, nullptr,
                         nullptr, dummy, nullptr) == QLOCO_ERR_ARG, "warm_start 3 refused");
  qloco_a1_params ap;
  qloco_a1_params_default(&ap);
  CHECK(qloco_a1_qp_solve(&ap, -1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                          nullptr, nullptr) == QLOCO_ERR_ARG, "a1 batch -1");
  CHECK(qloco_eiquadprog_solve(65, 0, 8, 1, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, nullptr,
                               0, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                               nullptr) == QLOCO_BAD_SIZE, "eiquadprog n 65");
  CHECK(qloco_rt_workspace_bytes(-1) == -1, "rt ws");
  CHECK(qloco_servo_workspace_bytes(-1) == -1, "servo ws");
  CHECK(std::string(qloco_status_string(QLOCO_BAD_SIZE)).size() > 0, "status string");
  if (g_fail) {
    std::printf("%d FAILURES\n", g_fail);
    return 1;
  }
  std::printf("host_asan ALL OK\n");
  return 0;
}
