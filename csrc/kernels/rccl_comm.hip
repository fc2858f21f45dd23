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
//
// Failure handling (what torch's ProcessGroupNCCL watchdog gives the reference through
// `init_process_group('nccl')`, `mlcomp/worker/executors/catalyst_/catalyst_.py:228-230`):
// the communicator is created NON-blocking (ncclCommInitRankConfig, blocking = 0), so
// init returns at once and the caller polls mlc_comm_async_error under a deadline
// (a peer that never joins -> ncclCommAbort, not a hang).  Every collective wrapper that
// gets ncclInProgress back (lazy connection setup) polls to completion before returning,
// so stream order is what a blocking communicator gives, bounded by g_comm_timeout_ms
// (kCommTimeout returned on expiry).  A watchdog thread on the Python side
// (mlcomp_amd/parallel/comm.py) polls async errors and step-completion events and calls
// mlc_comm_abort, which also makes RCCL kernels stuck on a dead peer exit.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <chrono>
#include <thread>

static long g_comm_timeout_ms = 600000;      // mlc_comm_set_timeout
constexpr int kCommTimeout = 1000;           // returned when an in-progress call outlives it

#define MLC_EXPORT extern "C" __attribute__((visibility("default")))

MLC_EXPORT int mlc_comm_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

MLC_EXPORT int mlc_comm_get_unique_id(char* out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

// returns an opaque communicator handle (0 on failure; *err gets the ncclResult_t).
// blocking == 0: the handle comes back at once with *err == ncclInProgress (7) while the
// ranks rendezvous; poll mlc_comm_async_error until it is no longer 7.
MLC_EXPORT void* mlc_comm_init(const char* id_bytes, int nranks, int rank, int device, int blocking, int* err) {
  if (hipSetDevice(device) != hipSuccess) { *err = -1; return nullptr; }
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = blocking ? 1 : 0;
  ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &cfg);
  *err = (int)r;
  return (r == ncclSuccess || r == ncclInProgress) ? (void*)comm : nullptr;
}

// ncclCommGetAsyncError: 0 ready, 7 still in progress, anything else a failed communicator
MLC_EXPORT int mlc_comm_async_error(void* comm) {
  if (!comm) return (int)ncclInvalidArgument;
  ncclResult_t st = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &st);
  return r != ncclSuccess ? (int)r : (int)st;
}

// tear the communicator down without waiting for peers (outstanding RCCL kernels exit)
MLC_EXPORT int mlc_comm_abort(void* comm) { return comm ? (int)ncclCommAbort((ncclComm_t)comm) : 0; }

MLC_EXPORT const char* mlc_comm_error_string(int code) {
  if (code == kCommTimeout) return "timed out";
  return ncclGetErrorString((ncclResult_t)code);
}

MLC_EXPORT const char* mlc_comm_last_error(void* comm) { return ncclGetLastError((ncclComm_t)comm); }

MLC_EXPORT void mlc_comm_set_timeout(long ms) { g_comm_timeout_ms = ms > 0 ? ms : 1; }

MLC_EXPORT int mlc_comm_destroy(void* comm) {
  return comm ? (int)ncclCommDestroy((ncclComm_t)comm) : 0;
}

// a call on a non-blocking communicator that returned ncclInProgress: wait (bounded) until
// the operation is issued, so the caller sees the ordering of a blocking communicator
static int settle(ncclComm_t comm, ncclResult_t r) {
  if (r != ncclInProgress) return (int)r;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t q = ncclCommGetAsyncError(comm, &st);
    if (q != ncclSuccess) return (int)q;
    if (st != ncclInProgress) return (int)st;
    const long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (ms > g_comm_timeout_ms) return kCommTimeout;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
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
  return settle((ncclComm_t)comm, ncclAllReduce(send, recv, (size_t)count, dt(dtype), op(red), (ncclComm_t)comm, st));
}

MLC_EXPORT int mlc_broadcast(void* comm, const void* send, void* recv, long count, int dtype, int root,
                             hipStream_t st) {
  return settle((ncclComm_t)comm, ncclBroadcast(send, recv, (size_t)count, dt(dtype), root, (ncclComm_t)comm, st));
}

// recvcount elements land on every rank
MLC_EXPORT int mlc_reduce_scatter(void* comm, const void* send, void* recv, long recvcount, int dtype,
                                  int red, hipStream_t st) {
  return settle((ncclComm_t)comm,
                ncclReduceScatter(send, recv, (size_t)recvcount, dt(dtype), op(red), (ncclComm_t)comm, st));
}

MLC_EXPORT int mlc_allgather(void* comm, const void* send, void* recv, long sendcount, int dtype,
                             hipStream_t st) {
  return settle((ncclComm_t)comm, ncclAllGather(send, recv, (size_t)sendcount, dt(dtype), (ncclComm_t)comm, st));
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
  return settle((ncclComm_t)comm, ncclGroupEnd());
}
