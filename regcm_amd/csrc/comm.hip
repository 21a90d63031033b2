// comm.hip -- RCCL halo transport (see comm.hpp).
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstdlib>
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
  explicit RcclComm(const rcmdyn_config& cfg) {
    const int ntiles = cfg.nproc_j * cfg.nproc_i;
    if (cfg.comm_size != ntiles || cfg.tile_count != 1 || cfg.tile_first != cfg.comm_rank)
      throw std::runtime_error("rcmdyn: RCCL mode needs one tile per rank (tile_first == comm_rank)");
    ncclUniqueId id;
    std::memcpy(id.internal, cfg.comm_unique_id, NCCL_UNIQUE_ID_BYTES);
    NCCLCHK(ncclCommInitRank(&comm_, cfg.comm_size, id, cfg.comm_rank));
    rank_ = cfg.comm_rank;
  }
  RcclComm() {                       // one rank: sends to itself
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    NCCLCHK(ncclCommInitRank(&comm_, 1, id, 0));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return;
    NCCLCHK(ncclGroupStart());
    for (const Xfer& x : sends) NCCLCHK(ncclSend(x.ptr, x.count, ncclDouble, x.peer, comm_, s));
    for (const Xfer& x : recvs) NCCLCHK(ncclRecv(x.ptr, x.count, ncclDouble, x.peer, comm_, s));
    NCCLCHK(ncclGroupEnd());
  }
  void allreduce_sum(double* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclSum, comm_, s));
  }
  void allreduce_max(int32_t* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclInt32, ncclMax, comm_, s));
  }
  void allreduce_max_d(double* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclMax, comm_, s));
  }
  // RCCL supports stream capture of its collectives and send/recv; RCMDYN_RCCL_EAGER=1 runs
  // decomposed steps eagerly instead
  bool graph_safe() const override { return std::getenv("RCMDYN_RCCL_EAGER") == nullptr; }
  int rank() const override { return rank_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0;
};

}  // namespace

Comm* make_rccl_comm(const rcmdyn_config& cfg) { return new RcclComm(cfg); }
Comm* make_rccl_self_comm() { return new RcclComm(); }

std::string rccl_describe() {
  Dl_info info{};
  std::string path = dladdr((void*)&ncclGetVersion, &info) && info.dli_fname ? info.dli_fname : "?";
  int v = 0;
  ncclGetVersion(&v);
  return path + " (" + std::to_string(v) + ")";
}

void comm_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace rcm
