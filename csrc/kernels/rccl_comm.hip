// Thin C ABI over RCCL for the framework's own data-parallel engine.
//
// The gradient bucketer (mlcomp_amd/parallel/ddp.py) issues collectives directly on a
// HIP stream of its choosing, so they are ordinary stream work: they overlap backward
// on a side stream via events and are captured into the step's HIP graph together with
// the compute kernels (no ProcessGroup work objects / watchdog involved).  The
// communicator is created once per process from a unique id exchanged through the
// torch.distributed TCP store.  Intra-node the transport is xGMI (all 8 MI355X are
// directly connected); RCCL's channel count decides how many of the 7 links a
// collective uses, so buckets are sized so each per-peer chunk stays >= ~1-4 MB.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#define MLC_EXPORT extern "C" __attribute__((visibility("default")))

MLC_EXPORT int mlc_comm_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

MLC_EXPORT int mlc_comm_get_unique_id(char* out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

// returns an opaque communicator handle (0 on failure; *err gets the ncclResult_t)
MLC_EXPORT void* mlc_comm_init(const char* id_bytes, int nranks, int rank, int device, int* err) {
  if (hipSetDevice(device) != hipSuccess) { *err = -1; return nullptr; }
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
  *err = (int)r;
  return r == ncclSuccess ? (void*)comm : nullptr;
}

MLC_EXPORT int mlc_comm_destroy(void* comm) {
  return comm ? (int)ncclCommDestroy((ncclComm_t)comm) : 0;
}

static ncclDataType_t dt(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt64;
    case 4: return ncclInt32;
    default: return ncclFloat32;
  }
}

static ncclRedOp_t op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclAvg;
    default: return ncclSum;
  }
}

MLC_EXPORT int mlc_allreduce(void* comm, const void* send, void* recv, long count, int dtype, int red,
                             hipStream_t st) {
  return (int)ncclAllReduce(send, recv, (size_t)count, dt(dtype), op(red), (ncclComm_t)comm, st);
}

MLC_EXPORT int mlc_broadcast(void* comm, const void* send, void* recv, long count, int dtype, int root,
                             hipStream_t st) {
  return (int)ncclBroadcast(send, recv, (size_t)count, dt(dtype), root, (ncclComm_t)comm, st);
}

// recvcount elements land on every rank
MLC_EXPORT int mlc_reduce_scatter(void* comm, const void* send, void* recv, long recvcount, int dtype,
                                  int red, hipStream_t st) {
  return (int)ncclReduceScatter(send, recv, (size_t)recvcount, dt(dtype), op(red), (ncclComm_t)comm, st);
}

MLC_EXPORT int mlc_allgather(void* comm, const void* send, void* recv, long sendcount, int dtype,
                             hipStream_t st) {
  return (int)ncclAllGather(send, recv, (size_t)sendcount, dt(dtype), (ncclComm_t)comm, st);
}

// all-to-all via grouped point-to-point (count elements per peer)
MLC_EXPORT int mlc_alltoall(void* comm, const void* send, void* recv, long count, int dtype, int elt_bytes,
                            int nranks, hipStream_t st) {
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (int p = 0; p < nranks; ++p) {
    ncclSend((const char*)send + (size_t)p * count * elt_bytes, (size_t)count, dt(dtype), p, (ncclComm_t)comm, st);
    ncclRecv((char*)recv + (size_t)p * count * elt_bytes, (size_t)count, dt(dtype), p, (ncclComm_t)comm, st);
  }
  return (int)ncclGroupEnd();
}
