// Gradient exchange over RCCL (xGMI) for the data-parallel training step.
//
// The reference gets its gradient all-reduce from DDP's bucket hooks inside
// accelerator.backward (reference trainer.py:360).  Here the trainer's bucket
// all-reduces are issued on a communicator this library owns, enqueued on the
// caller's HIP stream — eagerly, or inside a HIP-graph capture of the
// backward.  No c10d work object, event or watchdog is involved, so nothing
// outside the capturing thread ever queries an event recorded during a
// capture (the failure mode of routing captured collectives through
// ProcessGroupNCCL: its watchdog polls work events while the capture is open).
//
// RCCL is resolved at run time (dlopen): the instance PyTorch already loaded
// when it is there (same soname, so one set of RCCL proxy threads per
// process), otherwise the ROCm one.  The library itself stays loadable on a
// host without RCCL; only these entry points then fail.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and enums only: nothing is linked, RCCL is dlopen'ed

#include <cstring>
#include <mutex>
#include <string>

#include "../../include/dv_hip.h"

namespace dv {
void set_error(const std::string& msg);
}

namespace {

// the ABI comes from the image's rccl.h (the resolved symbols are cast to the
// header's own prototypes); the unique id travels as 128 raw bytes through
// the torch.distributed store and the Python binding
static_assert(sizeof(ncclUniqueId) == 128 && NCCL_UNIQUE_ID_BYTES == 128,
              "dv_comm_unique_id hands out 128 bytes (include/dv_hip.h, trainer.GradComm)");
static_assert(ncclSuccess == 0, "status 0 is success");

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclCommGetAsyncError) comm_get_async_error = nullptr;
  decltype(&ncclGetErrorString) get_error_string = nullptr;
  std::string why;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // torch's bundled RCCL first (already mapped, soname librccl.so.1), then
    // the loader's search path (this library's RUNPATH: /opt/rocm/lib)
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    r.handle = h;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.comm_abort = (decltype(r.comm_abort))dlsym(h, "ncclCommAbort");
    r.comm_get_async_error = (decltype(r.comm_get_async_error))dlsym(h, "ncclCommGetAsyncError");
    r.get_error_string = (decltype(r.get_error_string))dlsym(h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy || !r.comm_abort ||
        !r.get_error_string) {
      r.why = "librccl.so.1 lacks an expected symbol";
      r.handle = nullptr;
    }
  });
  return r;
}

int fail(const char* what, ncclResult_t rc) {
  Rccl& r = rccl();
  dv::set_error(std::string(what) + ": " + (r.get_error_string ? r.get_error_string(rc) : "rccl error"));
  return DV_ERR_LAUNCH;
}

bool ready(const char* what) {
  Rccl& r = rccl();
  if (!r.handle) {
    dv::set_error(std::string(what) + ": " + r.why);
    return false;
  }
  return true;
}

}  // namespace

extern "C" int dv_comm_unique_id(void* id_out) {
  if (!id_out) {
    dv::set_error("dv_comm_unique_id: null pointer");
    return DV_ERR_INVALID;
  }
  if (!ready("dv_comm_unique_id")) return DV_ERR_UNSUPPORTED;
  ncclUniqueId id;
  ncclResult_t rc = rccl().get_unique_id(&id);
  if (rc != 0) return fail("ncclGetUniqueId", rc);
  std::memcpy(id_out, id.internal, sizeof(id.internal));
  return DV_OK;
}

extern "C" int dv_comm_init(const void* id, int nranks, int rank, int device, void** comm_out) {
  if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks) {
    dv::set_error("dv_comm_init: invalid arguments");
    return DV_ERR_INVALID;
  }
  if (!ready("dv_comm_init")) return DV_ERR_UNSUPPORTED;
  if (hipSetDevice(device) != hipSuccess) {
    dv::set_error("dv_comm_init: hipSetDevice failed");
    return DV_ERR_INVALID;
  }
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, sizeof(uid.internal));
  ncclComm_t comm = nullptr;
  ncclResult_t rc = rccl().comm_init_rank(&comm, nranks, uid, rank);
  if (rc != 0) return fail("ncclCommInitRank", rc);
  *comm_out = comm;
  return DV_OK;
}

extern "C" int dv_comm_allreduce(void* comm, void* buf, long long count, int dtype, int average,
                                 void* stream) {
  if (!comm || (!buf && count > 0) || count < 0 || (dtype != DV_F32 && dtype != DV_BF16)) {
    dv::set_error("dv_comm_allreduce: invalid arguments");
    return DV_ERR_INVALID;
  }
  if (count == 0) return DV_OK;
  if (!ready("dv_comm_allreduce")) return DV_ERR_UNSUPPORTED;
  ncclResult_t rc = rccl().all_reduce(buf, buf, (size_t)count, dtype == DV_F32 ? ncclFloat32 : ncclBfloat16,
                                      average ? ncclAvg : ncclSum, (ncclComm_t)comm, (hipStream_t)stream);
  if (rc != 0) return fail("ncclAllReduce", rc);
  return DV_OK;
}

extern "C" int dv_comm_async_error(void* comm) {
  if (!comm) {
    dv::set_error("dv_comm_async_error: null communicator");
    return DV_ERR_INVALID;
  }
  if (!ready("dv_comm_async_error")) return DV_ERR_UNSUPPORTED;
  if (!rccl().comm_get_async_error) return DV_OK;
  ncclResult_t st = ncclSuccess;
  ncclResult_t rc = rccl().comm_get_async_error((ncclComm_t)comm, &st);
  if (rc != ncclSuccess) return fail("ncclCommGetAsyncError", rc);
  if (st != ncclSuccess && st != ncclInProgress) return fail("communicator async error", st);
  return DV_OK;
}

extern "C" int dv_comm_destroy(void* comm) {
  if (!comm) {
    dv::set_error("dv_comm_destroy: null communicator");
    return DV_ERR_INVALID;
  }
  if (!ready("dv_comm_destroy")) return DV_ERR_UNSUPPORTED;
  ncclResult_t rc = rccl().comm_destroy((ncclComm_t)comm);
  if (rc != 0) return fail("ncclCommDestroy", rc);
  return DV_OK;
}

extern "C" int dv_comm_abort(void* comm) {
  if (!comm) {
    dv::set_error("dv_comm_abort: null communicator");
    return DV_ERR_INVALID;
  }
  if (!ready("dv_comm_abort")) return DV_ERR_UNSUPPORTED;
  ncclResult_t rc = rccl().comm_abort((ncclComm_t)comm);
  if (rc != 0) return fail("ncclCommAbort", rc);
  return DV_OK;
}
