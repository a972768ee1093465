// libtrexhip.so -- the multi-GPU exchange of the sharded paths, for bindings
// that do not go through torch.distributed.
//
// C4 shards the tree batch and C5 the sites; each rank then holds a partial
// of one small fp32 buffer ([dC, loss] = Q*Q + 1 floats for C4, the N x N
// Gram for C5) and the only collective of either path is its sum over the
// ranks: trex_allreduce_sum, one RCCL all-reduce on the caller's stream
// (xGMI ring on one node).  RCCL is resolved with dlopen on first use, so the
// library has no link-time RCCL dependency and shares an RCCL already loaded
// in the process (torch's, when called from Python).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "trex_common.h"

namespace trex {
namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*err)(ncclResult_t) = nullptr;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.h) break;
    }
    if (!r.h) return;
    r.get_id = reinterpret_cast<decltype(r.get_id)>(dlsym(r.h, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(r.h, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(r.h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.h, "ncclAllReduce"));
    r.err = reinterpret_cast<decltype(r.err)>(dlsym(r.h, "ncclGetErrorString"));
  });
  if (!r.h || !r.get_id || !r.init_rank || !r.destroy || !r.all_reduce) return nullptr;
  return &r;
}

int rccl_fail(const char* fn, const Rccl* r, ncclResult_t e) {
  return set_error(TREX_E_HIP, "%s: RCCL error %d (%s)", fn, (int)e, r->err ? r->err(e) : "?");
}

}  // namespace
}  // namespace trex

using namespace trex;

// Switches the calling thread's current device for the duration of a call
// and restores the caller's on every return path (a process may drive
// several GPUs: torch, or a C caller).
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    ok_ = hipGetDevice(&prev_) == hipSuccess && hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
  bool ok_ = false;
};

extern "C" int trex_comm_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int trex_comm_get_unique_id(void* id) {
  const Rccl* r = rccl();
  if (!r) return set_error(TREX_E_UNSUPPORTED, "trex_comm_get_unique_id: RCCL not loadable");
  if (!id) return set_error(TREX_E_ARG, "trex_comm_get_unique_id: null id");
  ncclUniqueId u;
  if (ncclResult_t e = r->get_id(&u)) return rccl_fail("trex_comm_get_unique_id", r, e);
  std::memcpy(id, &u, sizeof u);
  return TREX_OK;
}

extern "C" int trex_comm_init(void** comm, int nranks, const void* id, int rank, int dev) {
  const char* fn = "trex_comm_init";
  const Rccl* r = rccl();
  if (!r) return set_error(TREX_E_UNSUPPORTED, "%s: RCCL not loadable", fn);
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks || dev < 0)
    return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  DeviceGuard guard(dev);
  if (!guard.ok()) return set_error(TREX_E_HIP, "%s: hipSetDevice(%d)", fn, dev);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t c = nullptr;
  if (ncclResult_t e = r->init_rank(&c, nranks, u, rank)) return rccl_fail(fn, r, e);
  *comm = c;
  return TREX_OK;
}

extern "C" int trex_comm_destroy(void* comm) {
  const Rccl* r = rccl();
  if (!r) return set_error(TREX_E_UNSUPPORTED, "trex_comm_destroy: RCCL not loadable");
  if (!comm) return TREX_OK;
  if (ncclResult_t e = r->destroy(static_cast<ncclComm_t>(comm)))
    return rccl_fail("trex_comm_destroy", r, e);
  return TREX_OK;
}

extern "C" int trex_allreduce_sum(float* buf, int count, int dev, void* comm, void* stream) {
  const char* fn = "trex_allreduce_sum";
  const Rccl* r = rccl();
  if (!r) return set_error(TREX_E_UNSUPPORTED, "%s: RCCL not loadable", fn);
  if (!buf || count < 0 || !comm || dev < 0) return set_error(TREX_E_ARG, "%s: bad arguments", fn);
  if (count == 0) return TREX_OK;
  DeviceGuard guard(dev);
  if (!guard.ok()) return set_error(TREX_E_HIP, "%s: hipSetDevice(%d)", fn, dev);
  if (ncclResult_t e = r->all_reduce(buf, buf, (size_t)count, ncclFloat32, ncclSum,
                                     static_cast<ncclComm_t>(comm), (hipStream_t)stream))
    return rccl_fail(fn, r, e);
  return TREX_OK;
}
