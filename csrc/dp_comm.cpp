// Single-process multi-GPU RCCL communicator for `-t DP` (SURVEY §2.4 "DP: RCCL broadcast and reduce
// from one process ... ncclCommInitAll and group calls"; reference path: torch.nn.DataParallel ->
// torch/nn/parallel/comm.py:67 broadcast_coalesced, :106-108 nccl.reduce, used by
// utils/train_utils.py:98,138-144).
//
// One clique of RCCL communicators, one per local device, created once; every collective is issued
// for all devices inside one ncclGroupStart/End from the calling thread, each on that device's
// compute stream (so it is ordered after the backward kernels that produced the gradients without
// any host synchronisation).  On the MI355X xGMI mesh RCCL runs the all-reduce of the flat gradient
// buffer over all 7 links of every GPU.
//
// Built as its own library (libdpa_comm.so) that resolves librccl.so.1 to the copy torch already
// loaded (same SONAME, rpath -> torch/lib), so the kernel library never depends on RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <vector>

#define DPA_API extern "C" __attribute__((visibility("default")))

namespace {

struct Clique {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
};

ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    default: return ncclNumTypes;
  }
}

ncclRedOp_t op_of(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
    default: return ncclNumOps;
  }
}

}  // namespace

// -> ncclResult_t; *out = opaque handle
DPA_API int dpa_dp_comm_init(int n, const int* devs, void** out) {
  if (n <= 0 || devs == nullptr || out == nullptr) return (int)ncclInvalidArgument;
  auto* c = new Clique;
  c->devs.assign(devs, devs + n);
  c->comms.resize(n);
  const ncclResult_t r = ncclCommInitAll(c->comms.data(), n, c->devs.data());
  if (r != ncclSuccess) {
    delete c;
    return (int)r;
  }
  *out = c;
  return (int)ncclSuccess;
}

DPA_API int dpa_dp_comm_destroy(void* h) {
  auto* c = static_cast<Clique*>(h);
  if (c == nullptr) return (int)ncclSuccess;
  ncclResult_t first = ncclSuccess;
  for (ncclComm_t cm : c->comms) {
    const ncclResult_t r = ncclCommDestroy(cm);
    if (first == ncclSuccess) first = r;
  }
  delete c;
  return (int)first;
}

DPA_API int dpa_dp_comm_size(void* h) { return h ? (int)static_cast<Clique*>(h)->comms.size() : 0; }

// In-place all-reduce of bufs[i] (count elements on device devs[i]) on streams[i].
DPA_API int dpa_dp_all_reduce(void* h, void* const* bufs, long long count, int dtype, int op, void* const* streams) {
  auto* c = static_cast<Clique*>(h);
  const ncclDataType_t dt = dtype_of(dtype);
  const ncclRedOp_t ro = op_of(op);
  if (c == nullptr || bufs == nullptr || streams == nullptr || count < 0 || dt == ncclNumTypes || ro == ncclNumOps)
    return (int)ncclInvalidArgument;
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    r = ncclAllReduce(bufs[i], bufs[i], (size_t)count, dt, ro, c->comms[i], (hipStream_t)streams[i]);
    if (r != ncclSuccess) break;
  }
  const ncclResult_t e = ncclGroupEnd();
  return (int)(r != ncclSuccess ? r : e);
}

// Broadcast bufs[root] into every bufs[i] (parameter / buffer replication, reference N6).
DPA_API int dpa_dp_broadcast(void* h, void* const* bufs, long long count, int dtype, int root, void* const* streams) {
  auto* c = static_cast<Clique*>(h);
  const ncclDataType_t dt = dtype_of(dtype);
  if (c == nullptr || bufs == nullptr || streams == nullptr || count < 0 || dt == ncclNumTypes || root < 0 ||
      root >= (int)c->comms.size())
    return (int)ncclInvalidArgument;
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    r = ncclBroadcast(bufs[i], bufs[i], (size_t)count, dt, root, c->comms[i], (hipStream_t)streams[i]);
    if (r != ncclSuccess) break;
  }
  const ncclResult_t e = ncclGroupEnd();
  return (int)(r != ncclSuccess ? r : e);
}

DPA_API const char* dpa_dp_error(int code) { return ncclGetErrorString((ncclResult_t)code); }

DPA_API int dpa_dp_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}
