// comm.hpp -- inter-process halo transport over RCCL (xGMI) for the engine.
//
// Replaces the MPI point-to-point halo of mpplib (`exchange`, `exchange_lb`, `exchange_rt`,
// `exchange_bdy_lr/_bt`, Main/mpplib/mod_mppparam.F90:6065-13190): every exchange packs the
// owned edge boxes of a field with one kernel, moves them with one grouped ncclSend/ncclRecv
// per neighbour (each neighbour sits on its own xGMI link) and unpacks into the ghost ring.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rcmdyn.h"
#include "engine.hpp"

namespace rcm {

class Comm {
 public:
  virtual ~Comm() = default;
  // sides: 0 all 8 neighbours, 1 receive left/bottom(+corner), 2 receive right/top(+corner)
  virtual void exchange(const Tile& t, double* field, int nk, int width, int sides) = 0;
  virtual void exchange_slices(const Tile& t, double* const* sl, long slen, int kz) = 0;
  virtual bool graph_safe() const = 0;
};

Comm* make_rccl_comm(const rcmdyn_config& cfg, hipStream_t stream);
void comm_unique_id(uint8_t out[128]);

}  // namespace rcm
