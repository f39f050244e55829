// gwaoi_comm.hip — the X-strip halo exchange over RCCL (include/gwaoi_strips.h): one communicator per
// strip world (one rank per GPU), and one tick's exchange with both neighbours as ONE RCCL group of
// point-to-point sends/receives, enqueued on the caller's stream. Nothing is read back to the host:
// every message has a fixed size (the record count travels as its own one-word message, the records
// in a buffer of the select lists' capacity) and the receiver's absorb kernel reads the count from
// device memory, so select -> exchange -> absorb -> emit -> tick runs without a host round trip.
//
// xGMI is point-to-point (one link per neighbour pair on an 8-GPU node): a strip only ever talks to
// its two neighbours, ~two halo lists of 16-B records per tick, which is latency-bound, not bandwidth-
// bound.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "gwaoi.h"
#include "gwaoi_internal.h"
#include "gwaoi_strips.h"

static_assert(GWAOI_STRIP_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "communicator id size");

struct gwaoi_strip_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

#define NCHK(x)                                                                         \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      gw::set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_));   \
      return GWAOI_ERR_HIP;                                                             \
    }                                                                                   \
  } while (0)

// Inside an open ncclGroupStart: on a failure the group is closed before returning, so RCCL is never
// left in group state (a later collective on this thread would otherwise be folded into the dead group).
#define NCHK_GROUP(x)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      gw::set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_));   \
      (void)ncclGroupEnd();                                                             \
      return GWAOI_ERR_HIP;                                                             \
    }                                                                                   \
  } while (0)

extern "C" {

int gwaoi_strip_comm_id(uint8_t* id) {
  if (!id) return GWAOI_ERR_INVALID;
  ncclUniqueId u;
  NCHK(ncclGetUniqueId(&u));
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return GWAOI_OK;
}

int gwaoi_strip_comm_init(const uint8_t* id, int nranks, int rank, int device, gwaoi_strip_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) {
    gw::set_error("strip_comm_init: invalid argument");
    return GWAOI_ERR_INVALID;
  }
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) {
    gw::set_error("strip_comm_init: device %d", device);
    return GWAOI_ERR_HIP;
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  gwaoi_strip_comm* c = new (std::nothrow) gwaoi_strip_comm();
  if (!c) return GWAOI_ERR_NOMEM;
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    gw::set_error("strip_comm_init: ncclCommInitRank: %s", ncclGetErrorString(r));
    delete c;
    return GWAOI_ERR_HIP;
  }
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return GWAOI_OK;
}

int gwaoi_strip_comm_destroy(gwaoi_strip_comm* c) {
  if (!c) return GWAOI_OK;
  ncclResult_t r = ncclSuccess;
  if (c->comm) r = ncclCommDestroy(c->comm);
  delete c;
  if (r != ncclSuccess) {
    gw::set_error("strip_comm_destroy: %s", ncclGetErrorString(r));
    return GWAOI_ERR_HIP;
  }
  return GWAOI_OK;
}

int gwaoi_strip_exchange(gwaoi_strip_comm* c, void* stream, int left_peer, int right_peer, const uint32_t* d_left,
                         const uint32_t* d_right, const uint32_t* d_counts, uint32_t cap, uint32_t* d_left_in,
                         uint32_t* d_right_in, uint32_t* d_counts_in) {
  if (!c || !d_counts || !d_counts_in || left_peer >= c->nranks || right_peer >= c->nranks ||
      (left_peer >= 0 && (!d_left || !d_left_in)) || (right_peer >= 0 && (!d_right || !d_right_in))) {
    gw::set_error("strip_exchange: invalid argument");
    return GWAOI_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(c->device) != hipSuccess) return GWAOI_ERR_HIP;
  // a side without a neighbour receives nothing: its count is zeroed here, in stream order
  if (left_peer < 0 && hipMemsetAsync(d_counts_in, 0, sizeof(uint32_t), st) != hipSuccess) return GWAOI_ERR_HIP;
  if (right_peer < 0 && hipMemsetAsync(d_counts_in + 1, 0, sizeof(uint32_t), st) != hipSuccess) return GWAOI_ERR_HIP;
  const size_t words = (size_t)cap * 4;  // records are 4 x uint32
  NCHK(ncclGroupStart());
  if (left_peer >= 0) {  // sends and receives to one peer match in issue order: count, then records
    NCHK_GROUP(ncclSend(d_counts, 1, ncclUint32, left_peer, c->comm, st));
    NCHK_GROUP(ncclRecv(d_counts_in, 1, ncclUint32, left_peer, c->comm, st));
    NCHK_GROUP(ncclSend(d_left, words, ncclUint32, left_peer, c->comm, st));
    NCHK_GROUP(ncclRecv(d_left_in, words, ncclUint32, left_peer, c->comm, st));
  }
  if (right_peer >= 0) {
    NCHK_GROUP(ncclSend(d_counts + 1, 1, ncclUint32, right_peer, c->comm, st));
    NCHK_GROUP(ncclRecv(d_counts_in + 1, 1, ncclUint32, right_peer, c->comm, st));
    NCHK_GROUP(ncclSend(d_right, words, ncclUint32, right_peer, c->comm, st));
    NCHK_GROUP(ncclRecv(d_right_in, words, ncclUint32, right_peer, c->comm, st));
  }
  NCHK(ncclGroupEnd());
  return GWAOI_OK;
}

}  // extern "C"
