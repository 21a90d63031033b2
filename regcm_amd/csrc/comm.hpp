// comm.hpp -- inter-process halo transport over RCCL (xGMI) for the engine.
//
// Replaces the MPI point-to-point halo of mpplib (`exchange`, `exchange_lb`, `exchange_rt`,
// `exchange_bdy_lr/_bt`, Main/mpplib/mod_mppparam.F90:6065-13190).  The engine packs the
// owned edge boxes of all fields of one exchange point into one staging buffer per
// neighbour (k_pack_segs) and calls sendrecv(): one grouped ncclSend/ncclRecv per neighbour,
// each neighbour on its own xGMI link; tiles on the same device use device copies instead
// of this class with the identical staging layout.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rcmdyn.h"

namespace rcm {

struct Xfer {
  int peer;          // rank (= tile index)
  double* ptr;       // device staging pointer
  size_t count;      // doubles
};

class Comm {
 public:
  virtual ~Comm() = default;
  // one grouped ncclSend/ncclRecv (all peers) on stream s; sends[n] and recvs[n] to the same
  // peer are matched in issue order
  virtual void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) = 0;
  // in-place element-wise sum over all ranks (ncclAllReduce); the engine only reduces arrays
  // in which each element has one non-zero contributor, so the result is exact
  virtual void allreduce_sum(double* p, size_t count, hipStream_t s) = 0;
  // in-place maximum over all ranks: int32 words (the step error flags), doubles (cflmax)
  virtual void allreduce_max(int32_t* p, size_t count, hipStream_t s) = 0;
  virtual void allreduce_max_d(double* p, size_t count, hipStream_t s) = 0;
  virtual bool graph_safe() const = 0;
  virtual int rank() const = 0;
};

// one rank per tile: the communicator of the job (cfg.comm_rank / comm_size / unique id)
Comm* make_rccl_comm(const rcmdyn_config& cfg);
// a communicator of one rank that carries the halo messages between the tiles one engine
// holds, as RCCL sends and receives to itself (RCMDYN_FORCE_RCCL=1: exercises the RCCL
// transport, its grouping and its graph capture on a single GPU)
Comm* make_rccl_self_comm();
// "path (version)" of the librccl the engine's RCCL calls are bound to
std::string rccl_describe();
void comm_unique_id(uint8_t out[128]);

}  // namespace rcm
