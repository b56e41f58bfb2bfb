// Collective boundary of the multi-GPU video-text step: clips are
// sharded by batch over one process per GPU, and the only exchange is the all-gather of every
// rank's pooled clip embeddings [b, D] into [world*b, D] on every rank (the `video_emb` of the
// reference's `video_emb @ text_emb.T`, README.md:81, verify_clip_models.py:84).  It runs on RCCL
// over xGMI: a communicator per process, bootstrapped from a unique id that rank 0 creates and
// the host distributes (videoprism/distributed.py sends it through torch.distributed's store).
// The gather is a few hundred KB per rank, latency-bound: one ncclAllGather on the caller's stream.
#include "../../include/videoprism_hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "vp_internal.h"

using namespace vpi;

struct vp_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1, device = 0;
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(VP_ECOMM, std::string(what) + ": " + ncclGetErrorString(r));
}

// the calling thread's current HIP device is restored when an entry point returns (the caller
// may drive another GPU from the same thread)
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

int vp_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int vp_comm_unique_id(uint8_t* id_out, int64_t nbytes) {
  if (!id_out || nbytes < (int64_t)sizeof(ncclUniqueId)) return fail(VP_EINVAL, "id buffer too small");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id_out, &id, sizeof(id));
  return VP_OK;
}

int vp_comm_init(const uint8_t* id, int64_t nbytes, int nranks, int rank, int device, vp_comm** out) {
  if (!id || !out || nbytes < (int64_t)sizeof(ncclUniqueId)) return fail(VP_EINVAL, "null argument / short id");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(VP_EINVAL, "rank out of range");
  DeviceGuard guard;
  VP_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  vp_comm* c = new vp_comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  return VP_OK;
}

int vp_comm_destroy(vp_comm* c) {
  if (!c) return VP_OK;
  DeviceGuard guard;
  (void)hipSetDevice(c->device);
  const ncclResult_t r = c->comm ? ncclCommDestroy(c->comm) : ncclSuccess;
  delete c;
  return r == ncclSuccess ? VP_OK : nccl_fail(r, "ncclCommDestroy");
}

int vp_allgather(vp_comm* c, const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (!c || !send || !recv || count < 1) return fail(VP_EINVAL, "bad argument");
  ncclDataType_t t;
  switch (dtype) {
    case VP_F32: t = ncclFloat32; break;
    case VP_BF16: t = ncclBfloat16; break;
    case VP_U8: t = ncclUint8; break;
    default: return fail(VP_EINVAL, "bad dtype");
  }
  DeviceGuard guard;
  VP_HIP(hipSetDevice(c->device));
  const ncclResult_t r = ncclAllGather(send, recv, (size_t)count, t, c->comm, static_cast<hipStream_t>(stream));
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
  return VP_OK;
}

}  // extern "C"
