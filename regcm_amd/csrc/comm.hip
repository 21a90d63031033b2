// comm.hip -- RCCL halo transport (see comm.hpp).
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "comm.hpp"

namespace rcm {

namespace {

#define NCCLCHK(x)                                                                           \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

class RcclComm final : public Comm {
 public:
  RcclComm(const rcmdyn_config& cfg, hipStream_t s) : stream_(s) {
    const int ntiles = cfg.nproc_j * cfg.nproc_i;
    if (cfg.comm_size != ntiles || cfg.tile_count != 1 || cfg.tile_first != cfg.comm_rank)
      throw std::runtime_error("rcmdyn: RCCL mode needs one tile per rank (tile_first == comm_rank)");
    ncclUniqueId id;
    std::memcpy(id.internal, cfg.comm_unique_id, NCCL_UNIQUE_ID_BYTES);
    NCCLCHK(ncclCommInitRank(&comm_, cfg.comm_size, id, cfg.comm_rank));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) override {
    if (sends.empty() && recvs.empty()) return;
    NCCLCHK(ncclGroupStart());
    for (const Xfer& x : sends) NCCLCHK(ncclSend(x.ptr, x.count, ncclDouble, x.peer, comm_, stream_));
    for (const Xfer& x : recvs) NCCLCHK(ncclRecv(x.ptr, x.count, ncclDouble, x.peer, comm_, stream_));
    NCCLCHK(ncclGroupEnd());
  }
  void allreduce_sum(double* p, size_t count) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclSum, comm_, stream_));
  }
  bool graph_safe() const override { return false; }

 private:
  hipStream_t stream_;
  ncclComm_t comm_ = nullptr;
};

}  // namespace

Comm* make_rccl_comm(const rcmdyn_config& cfg, hipStream_t stream) { return new RcclComm(cfg, stream); }

void comm_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace rcm
