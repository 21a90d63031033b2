// comm.hip -- halo transports of the engine (see comm.hpp): RCCL, the in-process loopback
// of the multi-rank tests, and the plan recorder.
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

#include "comm.hpp"

namespace rcm {

namespace {

#define NCCLCHK(x)                                                                           \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

#define HIPCHK_C(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

class RcclComm final : public Comm {
 public:
  explicit RcclComm(const rcmdyn_config& cfg) {
    const int ntiles = cfg.nproc_j * cfg.nproc_i;
    if (cfg.comm_size != ntiles || cfg.tile_count != 1 || cfg.tile_first != cfg.comm_rank)
      throw std::runtime_error("rcmdyn: RCCL mode needs one tile per rank (tile_first == comm_rank)");
    ncclUniqueId id;
    std::memcpy(id.internal, cfg.comm_unique_id, NCCL_UNIQUE_ID_BYTES);
    NCCLCHK(ncclCommInitRank(&comm_[0], cfg.comm_size, id, cfg.comm_rank));
    rank_ = cfg.comm_rank;
    second(cfg.comm_size);
  }
  RcclComm() {                       // one rank: sends to itself
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    NCCLCHK(ncclCommInitRank(&comm_[0], 1, id, 0));
    second(1);
  }
  ~RcclComm() override {            // the split communicator before its parent
    for (int q = NCHAN - 1; q >= 0; q--)
      if (comm_[q] && (q == 0 || comm_[q] != comm_[0])) ncclCommDestroy(comm_[q]);
  }
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s, int chan) override {
    if (sends.empty() && recvs.empty()) return;
    ncclComm_t c = comm_[chan];
    NCCLCHK(ncclGroupStart());
    for (const Xfer& x : sends) NCCLCHK(ncclSend(x.ptr, x.count, ncclDouble, x.peer, c, s));
    for (const Xfer& x : recvs) NCCLCHK(ncclRecv(x.ptr, x.count, ncclDouble, x.peer, c, s));
    NCCLCHK(ncclGroupEnd());
  }
  void allreduce_sum(double* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclSum, comm_[0], s));
  }
  void allreduce_max(int32_t* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclInt32, ncclMax, comm_[0], s));
  }
  void allreduce_max_d(double* p, size_t count, hipStream_t s) override {
    NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclMax, comm_[0], s));
  }
  // RCCL supports stream capture of its collectives and send/recv; RCMDYN_RCCL_EAGER=1 runs
  // decomposed steps eagerly instead
  bool graph_safe() const override { return std::getenv("RCMDYN_RCCL_EAGER") == nullptr; }
  int rank() const override { return rank_; }
  bool shared_channels() const override { return comm_[1] == comm_[0]; }

 private:
  // The second channel shares the first communicator; the engine orders the second stream's
  // exchange after the first stream's (shared_channels).  A second communicator per channel
  // (ncclCommInitRank on a broadcast unique id, or ncclCommSplit) crashed the first graph-
  // captured step under the RCCL 2.26 that torch bundles (a process that imported torch
  // before loading the engine binds torch's librccl.so.1, the soname of /opt/rocm's 2.27;
  // tools/rccl_dbg.py --torch-first) and was removed: one communicator runs under both.
  void second(int) { comm_[1] = comm_[0]; }
  ncclComm_t comm_[NCHAN] = {nullptr, nullptr};
  int rank_ = 0;
};

// ------------------------------------------------------------------ in-process loopback
struct MaxRanks { static constexpr int N = 64; };
struct RedArgs {
  const void* src[MaxRanks::N];
  int n;
};
__global__ void k_red_sum_d(double* out, RedArgs a, size_t count) {
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < count; q += (size_t)gridDim.x * blockDim.x) {
    double v = 0.0;
    for (int r = 0; r < a.n; r++) v += ((const double*)a.src[r])[q];
    out[q] = v;
  }
}
__global__ void k_red_max_d(double* out, RedArgs a, size_t count) {
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < count; q += (size_t)gridDim.x * blockDim.x) {
    double v = ((const double*)a.src[0])[q];
    for (int r = 1; r < a.n; r++) v = fmax(v, ((const double*)a.src[r])[q]);
    out[q] = v;
  }
}
__global__ void k_red_max_i(int32_t* out, RedArgs a, size_t count) {
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < count; q += (size_t)gridDim.x * blockDim.x) {
    int32_t v = ((const int32_t*)a.src[0])[q];
    for (int r = 1; r < a.n; r++) v = max(v, ((const int32_t*)a.src[r])[q]);
    out[q] = v;
  }
}

struct LocalMsg {
  const double* ptr;
  size_t count;
  uint64_t sig;
  hipEvent_t ready;                  // the staging span is packed (sender's stream)
  hipEvent_t consumed = nullptr;     // it was copied out (receiver's stream)
  bool done = false;
};

struct LocalGroup {
  int size;
  std::mutex m;
  std::condition_variable cv;
  // messages per (sender, receiver, channel), in issue order
  std::map<std::tuple<int, int, int>, std::deque<std::shared_ptr<LocalMsg>>> q;
  // collectives: per generation, each rank's staged input and its events
  struct Coll {
    std::vector<const void*> src;
    std::vector<hipEvent_t> ready, done;
    int posted = 0, finished = 0, left = 0, gone = 0;
  };
  std::map<long, Coll> coll;
  explicit LocalGroup(int n) : size(n) {}
};

std::mutex g_groups_m;
std::map<std::string, std::weak_ptr<LocalGroup>> g_groups;

class LocalComm final : public Comm {
 public:
  LocalComm(const std::string& name, int rank, int size) : rank_(rank), size_(size) {
    if (size < 1 || size > MaxRanks::N || rank < 0 || rank >= size)
      throw std::runtime_error("rcmdyn: local communicator: bad rank/size");
    std::lock_guard<std::mutex> lk(g_groups_m);
    auto& w = g_groups[name];
    grp_ = w.lock();
    if (!grp_) {
      grp_ = std::make_shared<LocalGroup>(size);
      w = grp_;
    }
    if (grp_->size != size) throw std::runtime_error("rcmdyn: local communicator: size mismatch in group " + name);
  }
  ~LocalComm() override {
    if (stage_) (void)hipFree(stage_);
  }
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s, int chan) override {
    if (sends.empty() && recvs.empty()) return;
    if (trace_) {
      std::fprintf(stderr, "[local %d] call %ld chan %d:", rank_, ncall_, chan);
      for (const Xfer& x : sends) std::fprintf(stderr, " s%d/%zu", x.peer, x.count);
      for (const Xfer& x : recvs) std::fprintf(stderr, " r%d/%zu", x.peer, x.count);
      std::fprintf(stderr, "\n");
    }
    ncall_++;
    std::vector<std::shared_ptr<LocalMsg>> mine;
    for (const Xfer& x : sends) {
      auto m = std::make_shared<LocalMsg>();
      m->ptr = x.ptr; m->count = x.count; m->sig = x.sig;
      HIPCHK_C(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
      HIPCHK_C(hipEventRecord(m->ready, s));
      mine.push_back(m);
      std::lock_guard<std::mutex> lk(grp_->m);
      grp_->q[{rank_, x.peer, chan}].push_back(m);
    }
    grp_->cv.notify_all();
    for (const Xfer& x : recvs) {
      std::shared_ptr<LocalMsg> m;
      {
        std::unique_lock<std::mutex> lk(grp_->m);
        auto& dq = grp_->q[{x.peer, rank_, chan}];
        grp_->cv.wait(lk, [&] { return !dq.empty(); });
        m = dq.front();
        dq.pop_front();
      }
      if (m->count != x.count || (m->sig && x.sig && m->sig != x.sig))
        throw std::runtime_error("rcmdyn: local communicator: message from rank " + std::to_string(x.peer) +
                                 " does not match the receive (count " + std::to_string(m->count) + " vs " +
                                 std::to_string(x.count) + ")");
      HIPCHK_C(hipStreamWaitEvent(s, m->ready, 0));
      HIPCHK_C(hipMemcpyAsync(x.ptr, m->ptr, x.count * sizeof(double), hipMemcpyDeviceToDevice, s));
      hipEvent_t ev;
      HIPCHK_C(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIPCHK_C(hipEventRecord(ev, s));
      {
        std::lock_guard<std::mutex> lk(grp_->m);
        m->consumed = ev;
        m->done = true;
      }
      grp_->cv.notify_all();
    }
    // the sender's later work (the next pack into the same staging) waits for the copies out
    for (auto& m : mine) {
      {
        std::unique_lock<std::mutex> lk(grp_->m);
        grp_->cv.wait(lk, [&] { return m->done; });
      }
      HIPCHK_C(hipStreamWaitEvent(s, m->consumed, 0));
      (void)hipEventDestroy(m->ready);
      (void)hipEventDestroy(m->consumed);
    }
  }
  void allreduce_sum(double* p, size_t count, hipStream_t s) override { coll(p, count * 8, s, 0, count); }
  void allreduce_max(int32_t* p, size_t count, hipStream_t s) override { coll(p, count * 4, s, 1, count); }
  void allreduce_max_d(double* p, size_t count, hipStream_t s) override { coll(p, count * 8, s, 2, count); }
  bool graph_safe() const override { return false; }
  int rank() const override { return rank_; }

 private:
  // every rank stages its input, all wait for all, each reduces the staged inputs in rank
  // order into its own buffer, and none reuses its stage before every rank has read it
  void coll(void* p, size_t bytes, hipStream_t s, int op, size_t count) {
    if (bytes > stage_cap_) {
      if (stage_) HIPCHK_C(hipFree(stage_));
      HIPCHK_C(hipMalloc(&stage_, bytes));
      stage_cap_ = bytes;
    }
    HIPCHK_C(hipMemcpyAsync(stage_, p, bytes, hipMemcpyDeviceToDevice, s));
    hipEvent_t ready, done;
    HIPCHK_C(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HIPCHK_C(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIPCHK_C(hipEventRecord(ready, s));
    const long gen = gen_++;
    LocalGroup::Coll* c;
    {
      std::unique_lock<std::mutex> lk(grp_->m);
      c = &grp_->coll[gen];
      if (c->src.empty()) { c->src.assign(size_, nullptr); c->ready.assign(size_, nullptr); c->done.assign(size_, nullptr); }
      c->src[rank_] = stage_;
      c->ready[rank_] = ready;
      c->posted++;
      grp_->cv.notify_all();
      grp_->cv.wait(lk, [&] { return c->posted == size_; });
    }
    RedArgs a{};
    a.n = size_;
    for (int r = 0; r < size_; r++) {
      a.src[r] = c->src[r];
      HIPCHK_C(hipStreamWaitEvent(s, c->ready[r], 0));
    }
    const int nb = (int)std::min<size_t>(1024, (count + 255) / 256);
    if (op == 0) hipLaunchKernelGGL(k_red_sum_d, dim3(nb), dim3(256), 0, s, (double*)p, a, count);
    else if (op == 1) hipLaunchKernelGGL(k_red_max_i, dim3(nb), dim3(256), 0, s, (int32_t*)p, a, count);
    else hipLaunchKernelGGL(k_red_max_d, dim3(nb), dim3(256), 0, s, (double*)p, a, count);
    HIPCHK_C(hipGetLastError());
    HIPCHK_C(hipEventRecord(done, s));
    {
      std::unique_lock<std::mutex> lk(grp_->m);
      c->done[rank_] = done;
      c->finished++;
      grp_->cv.notify_all();
      grp_->cv.wait(lk, [&] { return c->finished == size_; });
    }
    for (int r = 0; r < size_; r++) HIPCHK_C(hipStreamWaitEvent(s, c->done[r], 0));
    {
      // a rank destroys its events only once every rank has enqueued its waits on them; the
      // last rank out frees the generation's bookkeeping
      std::unique_lock<std::mutex> lk(grp_->m);
      c->left++;
      grp_->cv.notify_all();
      grp_->cv.wait(lk, [&] { return c->left == size_; });
      if (++c->gone == size_) grp_->coll.erase(gen);
    }
    (void)hipEventDestroy(ready);
    (void)hipEventDestroy(done);
  }
  std::shared_ptr<LocalGroup> grp_;
  int rank_, size_;
  long ncall_ = 0;
  const bool trace_ = std::getenv("RCMDYN_LOCAL_TRACE") != nullptr;
  long gen_ = 0;
  void* stage_ = nullptr;
  size_t stage_cap_ = 0;
};

// ------------------------------------------------------------------ plan recorder
class PlanComm final : public Comm {
 public:
  PlanComm(int rank, std::vector<PlanOp>* log) : rank_(rank), log_(log) {}
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t, int chan) override {
    if (sends.empty() && recvs.empty()) return;
    for (const Xfer& x : sends) log_->push_back({seq_, 1, chan, 0, x.peer, (int64_t)x.count, (int64_t)x.sig});
    for (const Xfer& x : recvs) log_->push_back({seq_, 1, chan, 1, x.peer, (int64_t)x.count, (int64_t)x.sig});
    seq_++;
  }
  void allreduce_sum(double*, size_t count, hipStream_t) override { coll(2, count); }
  void allreduce_max(int32_t*, size_t count, hipStream_t) override { coll(3, count); }
  void allreduce_max_d(double*, size_t count, hipStream_t) override { coll(4, count); }
  bool graph_safe() const override { return false; }
  int rank() const override { return rank_; }

 private:
  void coll(int kind, size_t count) { log_->push_back({seq_++, kind, 0, -1, -1, (int64_t)count, 0}); }
  int rank_;
  std::vector<PlanOp>* log_;
  int64_t seq_ = 0;
};

}  // namespace

Comm* make_rccl_comm(const rcmdyn_config& cfg) { return new RcclComm(cfg); }
Comm* make_rccl_self_comm() { return new RcclComm(); }
Comm* make_local_comm(const std::string& group, int rank, int size) { return new LocalComm(group, rank, size); }
Comm* make_plan_comm(int rank, std::vector<PlanOp>* log) { return new PlanComm(rank, log); }

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
