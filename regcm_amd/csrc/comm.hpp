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
  virtual void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) = 0;
  // in-place element-wise sum over all ranks (ncclAllReduce); the engine only reduces arrays
  // in which each element has one non-zero contributor, so the result is exact
  virtual void allreduce_sum(double* p, size_t count) = 0;
  virtual bool graph_safe() const = 0;
};

Comm* make_rccl_comm(const rcmdyn_config& cfg, hipStream_t stream);
void comm_unique_id(uint8_t out[128]);

}  // namespace rcm
