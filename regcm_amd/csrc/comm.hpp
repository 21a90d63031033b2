// comm.hpp -- inter-process halo transport over RCCL (xGMI) for the engine.
//
// Replaces the MPI point-to-point halo of mpplib (`exchange`, `exchange_lb`, `exchange_rt`,
// `exchange_bdy_lr/_bt`, Main/mpplib/mod_mppparam.F90:6065-13190).  The engine packs the
// owned edge boxes of all fields of one exchange point into one staging buffer per
// neighbour (k_pack_segs) and calls sendrecv(): one grouped ncclSend/ncclRecv per neighbour,
// each neighbour on its own xGMI link; tiles on the same device use device copies instead
// of this class with the identical staging layout.
//
// Channels: the engine issues exchanges on two HIP streams (the second carries the part of
// an exchange point that overlaps compute on the first).  Over RCCL both channels are the job's
// one communicator (shared_channels): the engine makes the second stream's grouped send/receive
// wait for the first stream's preceding one (fork_after_exchange / xch_join), so no two grouped
// calls on the communicator are in flight at once and it sees its operations in the same order
// on every rank.  The in-process loopback and the plan recorder keep two independent channels.
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
  uint64_t sig = 0;  // layout signature of the message (segment shapes), for plans and checks
};

constexpr int NCHAN = 2;

class Comm {
 public:
  virtual ~Comm() = default;
  // one grouped ncclSend/ncclRecv (all peers) on stream s over channel chan (0: the engine's
  // first stream, 1: its second); sends[n] and recvs[n] to the same peer are matched in
  // issue order within the channel
  virtual void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s,
                        int chan) = 0;
  // in-place element-wise sum over all ranks (ncclAllReduce, channel 0); the engine only
  // reduces arrays in which each element has one non-zero contributor, so the result is exact
  virtual void allreduce_sum(double* p, size_t count, hipStream_t s) = 0;
  // in-place maximum over all ranks: int32 words (the step error flags), doubles (cflmax)
  virtual void allreduce_max(int32_t* p, size_t count, hipStream_t s) = 0;
  virtual void allreduce_max_d(double* p, size_t count, hipStream_t s) = 0;
  virtual bool graph_safe() const = 0;
  virtual int rank() const = 0;
  // both channels go through one communicator: the engine then orders the second stream's
  // exchange after the first stream's preceding one (no two grouped calls in flight at once)
  virtual bool shared_channels() const { return false; }
};

// one rank per tile: the communicator of the job (cfg.comm_rank / comm_size / unique id),
// shared by both channels (the engine orders the two streams' exchanges)
Comm* make_rccl_comm(const rcmdyn_config& cfg);
// a communicator of one rank that carries the halo messages between the tiles one engine
// holds, as RCCL sends and receives to itself (RCMDYN_FORCE_RCCL=1: exercises the RCCL
// transport, its grouping and its graph capture on a single GPU)
Comm* make_rccl_self_comm();
// In-process loopback transport between engines of one process, one engine (one tile, one
// "rank") per host thread, all on one device (RCMDYN_LOCAL_COMM=<group>): a send posts the
// staging span with an event, the receiving rank copies it into its staging buffer on its own
// stream, and the sender's stream waits until its message was copied out, as MPI semantics
// require.  It runs the engine's remote-peer path (rank-addressed messages, the per-peer
// ordering, the collectives) on one GPU without a multi-GPU node; eager only (host rendezvous).
Comm* make_local_comm(const std::string& group, int rank, int size);
// The plan recorder of rcmdyn_exchange_plan: every call is logged, nothing moves.
struct PlanOp {
  int64_t seq;       // communication call number on this rank
  int64_t kind;      // 1 grouped send/recv, 2 allreduce sum (f64), 3 allreduce max (i32), 4 allreduce max (f64)
  int64_t chan;      // channel (0/1); collectives: 0
  int64_t dir;       // 0 send, 1 receive, -1 collective
  int64_t peer;      // peer rank (-1 for collectives)
  int64_t count;     // doubles (collectives: elements)
  int64_t sig;       // message layout signature (0 for collectives)
};
Comm* make_plan_comm(int rank, std::vector<PlanOp>* log);
// "path (version)" of the librccl the engine's RCCL calls are bound to
std::string rccl_describe();
void comm_unique_id(uint8_t out[128]);

}  // namespace rcm
