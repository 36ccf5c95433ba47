// qloco_mgpu.hip -- multi-GPU handles of the C ABI.
//
// The SRBD instances are independent, so the path shards with no exchange
// during the solve: each rank (one process or thread per GPU) owns a
// contiguous balanced range or the stride-interleaved ids of the global
// batch, solves them with qloco_srbd_solve_ex on its own device, and ONE
// RCCL all-gather over xGMI on the caller's stream leaves every rank with
// the whole batch's first-step forces in global instance order.  The
// reference has no distributed execution (its controllers are one process
// each, A1RobotControl.cpp:553-578); this is what lets a C++ caller of the
// batched solver shard without Python.
//
// RCCL is loaded on first use (dlopen of librccl.so.1), so libqloco.so has
// no link-time dependency on it and the single-GPU entry points never touch
// it.  The communicator id is made by rank 0 (qloco_mgpu_unique_id) and
// shipped to the other ranks by the caller, over whatever channel it has.
#include <dlfcn.h>
#include <string.h>

#include <mutex>

#include <rccl/rccl.h>

#include "qloco_common.hpp"

namespace qloco {

// ---------------------------------------------------------------- shards
// Owner rank and its position of global id g, and the rows of the gathered
// (world x P) buffer: shared by the device unpack and the host query.
__host__ __device__ inline void mgpu_owner(int64_t g, int64_t total, int world, int mode,
                                           int *rank, int64_t *k) {
  if (mode == QLOCO_SHARD_INTERLEAVED) {
    *rank = (int)(g % world);
    *k = g / world;
    return;
  }
  const int64_t base = total / world, extra = total % world;
  const int64_t big = extra * (base + 1);  // ranks < extra own base + 1 ids
  if (g < big) {
    *rank = (int)(g / (base + 1));
    *k = g % (base + 1);
  } else {
    *rank = (int)(extra + (g - big) / base);
    *k = (g - big) % base;
  }
}

__host__ __device__ inline int64_t mgpu_padded(int64_t total, int world) {
  return (total + world - 1) / world;
}

// [u0 (12) | status | iters] per instance into the send rows (width 14)
__global__ void mgpu_pack_kernel(int64_t count, const float *u0, const int32_t *status,
                                 const int32_t *iters, float *send) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count * 14) return;
  const int64_t b = i / 14;
  const int c = (int)(i - b * 14);
  float v;
  if (c < 12) v = u0[b * 12 + c];
  else if (c == 12) v = __int_as_float(status ? status[b] : 0);
  else v = __int_as_float(iters ? iters[b] : 0);
  send[i] = v;
}

// gathered (world x P x width) rows -> global id order
__global__ void mgpu_unpack_kernel(int64_t total, int world, int mode, int64_t P, int width,
                                   const float *stage, float *u0_all, int32_t *status_all,
                                   int32_t *iters_all) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total * 12) return;
  const int64_t g = i / 12;
  const int c = (int)(i - g * 12);
  int r;
  int64_t k;
  mgpu_owner(g, total, world, mode, &r, &k);
  const float *row = stage + ((int64_t)r * P + k) * width;
  u0_all[i] = row[c];
  if (c == 0 && width == 14) {
    if (status_all) status_all[g] = __float_as_int(row[12]);
    if (iters_all) iters_all[g] = __float_as_int(row[13]);
  }
}

// ---------------------------------------------------------------- RCCL
struct Rccl {
  void *so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};

static const Rccl *rccl() {
  static std::once_flag once;
  static Rccl r;
  std::call_once(once, [] {
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.so) break;
    }
    if (!r.so) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.so, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.so, "ncclCommInitRank"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(r.so, "ncclAllGather"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.so, "ncclCommDestroy"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.so, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string)
      r.so = nullptr;
  });
  if (!r.so) {
    set_last_error_msg("qloco_mgpu", "librccl.so.1 could not be loaded (RCCL is needed for the multi-GPU handles)");
    return nullptr;
  }
  return &r;
}

static int rccl_fail(const Rccl *r, const char *where, ncclResult_t e) {
  set_last_error_msg(where, r->error_string(e));
  return QLOCO_ERR_DEVICE;
}

}  // namespace qloco

using namespace qloco;

struct qloco_mgpu {
  int device = 0, world = 1, rank = 0, mode = 0;
  int64_t total = 0, first = 0, count = 0, stride = 1, P = 0;
  ncclComm_t comm = nullptr;
  float *u0_local = nullptr;
  int32_t *status_local = nullptr, *iters_local = nullptr;
  float *send = nullptr, *stage = nullptr;
};

extern "C" int qloco_mgpu_shard(int64_t total, int32_t world, int32_t rank, int32_t mode,
                                int64_t *first, int64_t *count, int64_t *stride) {
  if (total < 0 || world < 1 || rank < 0 || rank >= world) return QLOCO_ERR_ARG;
  if (mode != QLOCO_SHARD_CONTIGUOUS && mode != QLOCO_SHARD_INTERLEAVED) return QLOCO_ERR_ARG;
  int64_t f, c, s;
  if (mode == QLOCO_SHARD_INTERLEAVED) {
    f = rank;
    s = world;
    c = total > rank ? (total - rank + world - 1) / world : 0;
  } else {
    const int64_t base = total / world, extra = total % world;
    f = rank * base + (rank < extra ? rank : extra);
    c = base + (rank < extra ? 1 : 0);
    s = 1;
  }
  if (first) *first = f;
  if (count) *count = c;
  if (stride) *stride = s;
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_gather_rows(int64_t total, int32_t world, int32_t mode, int64_t *rows) {
  if (total < 0 || world < 1 || !rows) return QLOCO_ERR_ARG;
  if (mode != QLOCO_SHARD_CONTIGUOUS && mode != QLOCO_SHARD_INTERLEAVED) return QLOCO_ERR_ARG;
  const int64_t P = mgpu_padded(total, world);
  for (int64_t g = 0; g < total; ++g) {
    int r;
    int64_t k;
    mgpu_owner(g, total, world, mode, &r, &k);
    rows[g] = (int64_t)r * P + k;
  }
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_unique_id(uint8_t *id) {
  if (!id) return QLOCO_ERR_ARG;
  const Rccl *r = rccl();
  if (!r) return QLOCO_ERR_DEVICE;
  ncclUniqueId u;
  const ncclResult_t e = r->get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(r, "ncclGetUniqueId", e);
  memcpy(id, u.internal, QLOCO_MGPU_ID_BYTES);
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_destroy(qloco_mgpu *h) {
  if (!h) return QLOCO_OK;
  int rc = QLOCO_OK;
  if (h->comm) {
    const Rccl *r = rccl();
    if (r) {
      const ncclResult_t e = r->comm_destroy(h->comm);
      if (e != ncclSuccess) rc = rccl_fail(r, "ncclCommDestroy", e);
    }
  }
  (void)hipFree(h->u0_local);
  (void)hipFree(h->status_local);
  (void)hipFree(h->iters_local);
  (void)hipFree(h->send);
  (void)hipFree(h->stage);
  delete h;
  return rc;
}

extern "C" int qloco_mgpu_init(qloco_mgpu **out, const uint8_t *id, int32_t world, int32_t rank,
                               int64_t total, int32_t mode) {
  if (!out || !id) return QLOCO_ERR_ARG;
  *out = nullptr;
  int64_t first, count, stride;
  const int rc0 = qloco_mgpu_shard(total, world, rank, mode, &first, &count, &stride);
  if (rc0 != QLOCO_OK) return rc0;
  if (total < 1) return QLOCO_ERR_ARG;
  const Rccl *r = rccl();
  if (!r) return QLOCO_ERR_DEVICE;
  qloco_mgpu *h = new qloco_mgpu();
  if (hipGetDevice(&h->device) != hipSuccess) {
    delete h;
    return QLOCO_ERR_NO_GPU;
  }
  h->world = world;
  h->rank = rank;
  h->mode = mode;
  h->total = total;
  h->first = first;
  h->count = count;
  h->stride = stride;
  h->P = mgpu_padded(total, world);
  const int64_t P = h->P;
  if (hipMalloc(&h->u0_local, P * 12 * sizeof(float)) != hipSuccess ||
      hipMalloc(&h->status_local, P * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&h->iters_local, P * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&h->send, P * 14 * sizeof(float)) != hipSuccess ||
      hipMalloc(&h->stage, (int64_t)world * P * 14 * sizeof(float)) != hipSuccess) {
    set_last_error("qloco_mgpu_init: device buffers", hipErrorOutOfMemory);
    qloco_mgpu_destroy(h);
    return QLOCO_ERR_DEVICE;
  }
  // the padding rows of a short shard are gathered but never read: zero
  // them once so the exchanged bytes are deterministic
  if (hipMemset(h->u0_local, 0, P * 12 * sizeof(float)) != hipSuccess ||
      hipMemset(h->send, 0, P * 14 * sizeof(float)) != hipSuccess) {
    qloco_mgpu_destroy(h);
    return QLOCO_ERR_DEVICE;
  }
  ncclUniqueId u;
  memcpy(u.internal, id, QLOCO_MGPU_ID_BYTES);
  const ncclResult_t e = r->comm_init_rank(&h->comm, world, u, rank);
  if (e != ncclSuccess) {
    h->comm = nullptr;
    const int rc = rccl_fail(r, "ncclCommInitRank", e);
    qloco_mgpu_destroy(h);
    return rc;
  }
  *out = h;
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_info(const qloco_mgpu *h, int64_t *first, int64_t *count, int64_t *stride,
                               int64_t *padded) {
  if (!h) return QLOCO_ERR_ARG;
  if (first) *first = h->first;
  if (count) *count = h->count;
  if (stride) *stride = h->stride;
  if (padded) *padded = h->P;
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_solve(qloco_mgpu *h, const qloco_srbd_spec *spec, const float *x0,
                                const float *x_ref, const float *feet, const uint8_t *contacts,
                                float *warm, float *u0_all, int32_t *status_all,
                                int32_t *iters_all, int32_t max_stance_legs, void *stream) {
  if (!h || !spec || !u0_all) return QLOCO_ERR_ARG;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != h->device) {
    set_last_error_msg("qloco_mgpu_solve", "the current device is not the handle's device");
    return QLOCO_ERR_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  const bool stats = status_all || iters_all;
  // 1. this rank's shard (its inputs are the caller's count instances)
  if (h->count > 0) {
    const int rc = qloco_srbd_solve_ex(spec, h->count, x0, x_ref, feet, contacts, h->u0_local,
                                       nullptr, stats ? h->status_local : nullptr,
                                       stats ? h->iters_local : nullptr, nullptr, nullptr, warm,
                                       max_stance_legs, stream);
    if (rc != QLOCO_OK) return rc;
  }
  // 2. one all-gather of the padded shard rows
  const int width = stats ? 14 : 12;
  const float *sendbuf = h->u0_local;
  if (stats) {
    const int64_t n = h->count * 14;
    if (n > 0)
      hipLaunchKernelGGL(mgpu_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                         h->count, h->u0_local, h->status_local, h->iters_local, h->send);
    QLOCO_HIP_CHECK(hipGetLastError(), "mgpu_pack_kernel launch");
    sendbuf = h->send;
  }
  // contiguous equal shards of u0 alone: rank order is global order, so the
  // all-gather lands in the caller's buffer directly
  const bool direct = !stats && h->mode == QLOCO_SHARD_CONTIGUOUS && h->total % h->world == 0;
  float *recv = direct ? u0_all : h->stage;
  const Rccl *r = rccl();
  if (!r) return QLOCO_ERR_DEVICE;
  const ncclResult_t e = r->all_gather(sendbuf, recv, (size_t)(h->P * width), ncclFloat32, h->comm, st);
  if (e != ncclSuccess) return rccl_fail(r, "ncclAllGather", e);
  // 3. global id order
  if (!direct) return qloco_mgpu_reorder(h->total, h->world, h->mode, width, h->stage, u0_all,
                                         status_all, iters_all, stream);
  return QLOCO_OK;
}

extern "C" int qloco_mgpu_reorder(int64_t total, int32_t world, int32_t mode, int32_t width,
                                  const float *stage, float *u0_all, int32_t *status_all,
                                  int32_t *iters_all, void *stream) {
  if (total < 1 || world < 1 || (mode != QLOCO_SHARD_CONTIGUOUS && mode != QLOCO_SHARD_INTERLEAVED))
    return QLOCO_ERR_ARG;
  if ((width != 12 && width != 14) || !stage || !u0_all) return QLOCO_ERR_ARG;
  const int64_t n = total * 12;
  hipLaunchKernelGGL(mgpu_unpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, total, (int)world, (int)mode, mgpu_padded(total, world),
                     (int)width, stage, u0_all, status_all, iters_all);
  QLOCO_HIP_CHECK(hipGetLastError(), "mgpu_unpack_kernel launch");
  return QLOCO_OK;
}
