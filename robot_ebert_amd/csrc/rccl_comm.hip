// An RCCL communicator for ebt_cosine_topk_sharded's all-gather (include/ebert.h ebt_comm), so
// a host drives the row-sharded step with no per-collective callback into its own runtime:
// comm.all_gather = ebt_rccl_all_gather, comm.ctx = the handle of ebt_rccl_comm_init. RCCL over
// xGMI is the node's collective fabric; the library does not link it: librccl.so.1 is opened
// at the first use (in a PyTorch process that is the copy torch already loaded, by soname).
// Reference: none (the reference runs one CPU process, /root/reference/src/backend/app/lib.py).
#include <dlfcn.h>

#include <cstring>

#include <mutex>

#include <rccl/rccl.h>

#include "common.h"

namespace ebt {
namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const RcclApi* rccl_api() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
    api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
    api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.all_reduce = (decltype(api.all_reduce))dlsym(h, "ncclAllReduce");
    api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
    api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_gather &&
             api.all_reduce && api.error_string;
  });
  return api.ok ? &api : nullptr;
}

int rccl_check(const RcclApi* a, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return EBT_OK;
  set_error("%s: %s", what, a->error_string(r));
  return EBT_EHIP;
}

}  // namespace
}  // namespace ebt

using namespace ebt;

extern "C" {

int ebt_rccl_unique_id(void* id_out, size_t bytes) {
  const RcclApi* a = rccl_api();
  if (!a) {
    set_error("ebt_rccl_unique_id: librccl.so.1 could not be loaded");
    return EBT_EUNSUPPORTED;
  }
  if (!id_out || bytes < sizeof(ncclUniqueId)) {
    set_error("ebt_rccl_unique_id: need %zu bytes", sizeof(ncclUniqueId));
    return EBT_EINVAL;
  }
  ncclUniqueId id;
  const int rc = rccl_check(a, a->get_unique_id(&id), "ncclGetUniqueId");
  if (!rc) memcpy(id_out, &id, sizeof(id));
  return rc;
}

int ebt_rccl_comm_init(const void* id, int32_t rank, int32_t world, void** comm_out) {
  const RcclApi* a = rccl_api();
  if (!a) {
    set_error("ebt_rccl_comm_init: librccl.so.1 could not be loaded");
    return EBT_EUNSUPPORTED;
  }
  if (!id || !comm_out || world < 1 || rank < 0 || rank >= world) {
    set_error("ebt_rccl_comm_init: bad arguments (rank %d of %d)", rank, world);
    return EBT_EINVAL;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  const int rc = rccl_check(a, a->comm_init_rank(&comm, world, uid, rank), "ncclCommInitRank");
  if (!rc) *comm_out = (void*)comm;
  return rc;
}

int ebt_rccl_comm_destroy(void* comm) {
  const RcclApi* a = rccl_api();
  if (!a || !comm) return EBT_OK;
  return rccl_check(a, a->comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
}

// ebt_allgather_fn over an ebt_rccl_comm_init handle: recv[r * bytes ..] <- rank r's send, on
// `stream` (stream-ordered: returns once enqueued)
int ebt_rccl_all_gather(void* comm, const void* send, void* recv, size_t bytes, void* stream) {
  const RcclApi* a = rccl_api();
  if (!a || !comm) {
    set_error("ebt_rccl_all_gather: no communicator");
    return EBT_EINVAL;
  }
  return rccl_check(a, a->all_gather(send, recv, bytes, ncclInt8, (ncclComm_t)comm,
                                     (hipStream_t)stream),
                    "ncclAllGather");
}

// ebt_allreduce_f64_fn over the same handle: buf <- the sum over ranks, in place, on `stream`
int ebt_rccl_all_reduce_f64(void* comm, double* buf, size_t count, void* stream) {
  const RcclApi* a = rccl_api();
  if (!a || !comm) {
    set_error("ebt_rccl_all_reduce_f64: no communicator");
    return EBT_EINVAL;
  }
  return rccl_check(a, a->all_reduce(buf, buf, count, ncclFloat64, ncclSum, (ncclComm_t)comm,
                                     (hipStream_t)stream),
                    "ncclAllReduce");
}

}  // extern "C"
