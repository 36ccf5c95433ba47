// qloco_capi.hip -- call-level helpers of the C ABI (status strings, errors).
#include <string.h>

#include "qloco_common.hpp"

namespace qloco {
static thread_local char g_last_error[256] = {0};
void set_last_error(const char *where, hipError_t e) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, hipGetErrorString(e));
}
void set_last_error_msg(const char *where, const char *what) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, what);
}
}  // namespace qloco

extern "C" const char *qloco_last_error(void) { return qloco::g_last_error; }
extern "C" int qloco_abi_version(void) { return QLOCO_ABI_VERSION; }

extern "C" const char *qloco_status_string(int s) {
  switch (s) {
    case QLOCO_OK: return "ok";
    case QLOCO_MAX_ITER: return "max_iter";
    case QLOCO_INFEASIBLE: return "infeasible";
    case QLOCO_NAN: return "nan";
    case QLOCO_BAD_SIZE: return "bad_size";
    case QLOCO_NOT_PD: return "not_pd";
    case QLOCO_DEGENERATE: return "degenerate";
    case QLOCO_UB_PATH: return "ub_path";
    case QLOCO_SOLVED_INACCURATE: return "solved_inaccurate";
    case QLOCO_ERR_ARG: return "err_arg";
    case QLOCO_ERR_DEVICE: return "err_device";
    case QLOCO_ERR_NO_GPU: return "err_no_gpu";
    default: return "unknown";
  }
}
