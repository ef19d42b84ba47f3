// RCCL entry points of the C ABI (comm_init, all_to_allv, all_reduce):
// the collectives of the row-sharded step for a host that binds the library directly (the
// Python engine reaches the same RCCL through torch.distributed, backend "nccl").  One
// communicator per rank / GPU; every call is stream-ordered and returns an RCCL error as
// 2000 + ncclResult_t with the message in dl_last_error().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/dlamd.h"

namespace dl {
void set_error(const char* fmt, ...);
}

#define DL_NCCL(call)                                                       \
  do {                                                                      \
    ncclResult_t r_ = (call);                                               \
    if (r_ != ncclSuccess) {                                                \
      ::dl::set_error("%s: %s", #call, ncclGetErrorString(r_));             \
      return 2000 + (int)r_;                                                \
    }                                                                       \
  } while (0)

extern "C" int dl_comm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int dl_comm_get_unique_id(void* id_out) {
  if (!id_out) {
    dl::set_error("dl_comm_get_unique_id: NULL argument");
    return 22;
  }
  ncclUniqueId id;
  DL_NCCL(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

extern "C" int dl_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm_out) {
  if (!unique_id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks) {
    dl::set_error("dl_comm_init: bad arguments (nranks %d, rank %d)", nranks, rank);
    return 22;
  }
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ncclComm_t c = nullptr;
  DL_NCCL(ncclCommInitRank(&c, nranks, id, rank));
  *comm_out = c;
  return 0;
}

extern "C" int dl_comm_destroy(void* comm) {
  if (!comm) return 0;
  DL_NCCL(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
  return 0;
}

// Variable all-to-all of fixed-size rows: peer p's rows are send[soff_p .. soff_p + send_counts[p])
// (offsets = prefix sums of the counts, rank order), received likewise into recv.  Counts are
// host arrays of nranks row counts (what the owner-count all-gather of the step provides).
extern "C" int dl_all_to_allv(void* comm, const void* send, const int64_t* send_counts, void* recv,
                              const int64_t* recv_counts, int64_t row_bytes, void* stream) {
  if (!comm || !send_counts || !recv_counts || row_bytes <= 0) {
    dl::set_error("dl_all_to_allv: bad arguments");
    return 22;
  }
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  int n = 0;
  DL_NCCL(ncclCommCount(c, &n));
  const char* s = reinterpret_cast<const char*>(send);
  char* r = reinterpret_cast<char*>(recv);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DL_NCCL(ncclGroupStart());
  int64_t so = 0, ro = 0;
  for (int p = 0; p < n; ++p) {
    if (send_counts[p] < 0 || recv_counts[p] < 0) {
      ncclGroupEnd();
      dl::set_error("dl_all_to_allv: negative count for peer %d", p);
      return 22;
    }
    // bytes as ncclChar: no element-size constraint on the rows.  A failed send/recv closes
    // the group before returning, so no later RCCL call of the thread is left grouped.
    ncclResult_t e = ncclSuccess;
    if (send_counts[p]) e = ncclSend(s + so * row_bytes, (size_t)(send_counts[p] * row_bytes), ncclChar, p, c, st);
    if (e == ncclSuccess && recv_counts[p])
      e = ncclRecv(r + ro * row_bytes, (size_t)(recv_counts[p] * row_bytes), ncclChar, p, c, st);
    if (e != ncclSuccess) {
      ncclGroupEnd();
      dl::set_error("dl_all_to_allv: peer %d: %s", p, ncclGetErrorString(e));
      return 2000 + (int)e;
    }
    so += send_counts[p];
    ro += recv_counts[p];
  }
  DL_NCCL(ncclGroupEnd());
  return 0;
}

// The sharded step's fixed-capacity exchange (shard.hip's block layout): for every array a,
// block_bytes[a] per block, 2W - 1 blocks from bases[a]; block p < W = what peer p sends this
// rank, block W + p - (p > rank) = this rank's side of its traffic with peer p.  dir 0 (requests
// and gradients to the owners): send the sender-side block to p, receive p's into block p;
// dir 1 (rows back to the senders): send block p to p, receive into the sender-side block.
// Every array's transfers with every peer in one group (one launch); this rank's own block
// never moves.  Sizes are fixed, so the call is captured into the step's hipGraph unchanged.
extern "C" int dl_shard_exchange(void* comm, int32_t n_arrays, void* const* bases, const int64_t* block_bytes,
                                 int32_t dir, void* stream) {
  if (!comm || n_arrays < 0 || (n_arrays && (!bases || !block_bytes)) || (dir != 0 && dir != 1)) {
    dl::set_error("dl_shard_exchange: bad arguments");
    return 22;
  }
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  int n = 0, me = 0;
  DL_NCCL(ncclCommCount(c, &n));
  DL_NCCL(ncclCommUserRank(c, &me));
  if (n == 1 || n_arrays == 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DL_NCCL(ncclGroupStart());
  for (int p = 0; p < n; ++p) {
    if (p == me) continue;
    const int64_t mine = n + p - (p > me ? 1 : 0);   // this rank's side of the traffic with p
    for (int a = 0; a < n_arrays; ++a) {
      char* base = reinterpret_cast<char*>(bases[a]);
      const int64_t bb = block_bytes[a];
      if (bb <= 0) continue;
      char* snd = base + (dir == 0 ? mine : p) * bb;
      char* rcv = base + (dir == 0 ? p : mine) * bb;
      ncclResult_t e = ncclSend(snd, (size_t)bb, ncclChar, p, c, st);
      if (e == ncclSuccess) e = ncclRecv(rcv, (size_t)bb, ncclChar, p, c, st);
      if (e != ncclSuccess) {
        ncclGroupEnd();
        dl::set_error("dl_shard_exchange: peer %d: %s", p, ncclGetErrorString(e));
        return 2000 + (int)e;
      }
    }
  }
  DL_NCCL(ncclGroupEnd());
  return 0;
}

// Sum all-reduce of n floats (in place when send == recv): the step's flat dense-gradient buffer.
extern "C" int dl_all_reduce_f32(void* comm, const float* send, float* recv, int64_t n, void* stream) {
  if (!comm || !send || !recv || n < 0) {
    dl::set_error("dl_all_reduce_f32: bad arguments");
    return 22;
  }
  if (n == 0) return 0;
  DL_NCCL(ncclAllReduce(send, recv, (size_t)n, ncclFloat32, ncclSum, reinterpret_cast<ncclComm_t>(comm),
                        reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

// All-gather of `bytes` per rank into recv [nranks][bytes] (the per-owner count matrix).
extern "C" int dl_all_gather(void* comm, const void* send, void* recv, int64_t bytes, void* stream) {
  if (!comm || !send || !recv || bytes < 0) {
    dl::set_error("dl_all_gather: bad arguments");
    return 22;
  }
  if (bytes == 0) return 0;
  DL_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclChar, reinterpret_cast<ncclComm_t>(comm),
                        reinterpret_cast<hipStream_t>(stream)));
  return 0;
}
