// comm.hip -- RCCL halo transport (see comm.hpp).
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "comm.hpp"

namespace rcm {

namespace {

#define NCCLCHK(x)                                                                           \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)
#define HIPCHK2(x)                                                                           \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct Box {
  int j1, j2, i1, i2;
  long off;   // offset in the staging buffer
};
struct Boxes {
  Box b[8];
  int n;
};

// direction d: 0 L, 1 R, 2 B, 3 T, 4 BL, 5 BR, 6 TL, 7 TR ; opposite(d)
constexpr int OPP[8] = {1, 0, 3, 2, 7, 6, 5, 4};
constexpr int DJ[8] = {-1, 1, 0, 0, -1, 1, -1, 1};
constexpr int DI[8] = {0, 0, -1, 1, -1, -1, 1, 1};

__global__ void k_pack(Geom g, const double* __restrict__ f, int nk, Boxes bx, double* buf) {
  const Box b = bx.b[blockIdx.z];
  const int nj = b.j2 - b.j1 + 1, ni = b.i2 - b.i1 + 1;
  const long n = (long)nj * ni * nk;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int j = b.j1 + (int)(q % nj);
    const int i = b.i1 + (int)((q / nj) % ni);
    const int k = (int)(q / ((long)nj * ni));
    buf[b.off + q] = f[(long)k * g.plane + g.ix(j, i)];
  }
}

__global__ void k_unpack(Geom g, double* f, int nk, Boxes bx, const double* __restrict__ buf) {
  const Box b = bx.b[blockIdx.z];
  const int nj = b.j2 - b.j1 + 1, ni = b.i2 - b.i1 + 1;
  const long n = (long)nj * ni * nk;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int j = b.j1 + (int)(q % nj);
    const int i = b.i1 + (int)((q / nj) % ni);
    const int k = (int)(q / ((long)nj * ni));
    f[(long)k * g.plane + g.ix(j, i)] = buf[b.off + q];
  }
}

class RcclComm final : public Comm {
 public:
  RcclComm(const rcmdyn_config& cfg, hipStream_t s) : stream_(s) {
    const int ntiles = cfg.nproc_j * cfg.nproc_i;
    if (cfg.comm_size != ntiles || cfg.tile_count != 1 || cfg.tile_first != cfg.comm_rank)
      throw std::runtime_error("rcmdyn: RCCL mode needs one tile per rank (tile_first == comm_rank)");
    ncclUniqueId id;
    std::memcpy(id.internal, cfg.comm_unique_id, NCCL_UNIQUE_ID_BYTES);
    NCCLCHK(ncclCommInitRank(&comm_, cfg.comm_size, id, cfg.comm_rank));
    const int lj = cfg.tile_first / cfg.nproc_i, li = cfg.tile_first % cfg.nproc_i;
    for (int d = 0; d < 8; d++) {
      const int nj = lj + DJ[d], ni = li + DI[d];
      peer_[d] = (nj >= 0 && nj < cfg.nproc_j && ni >= 0 && ni < cfg.nproc_i) ? nj * cfg.nproc_i + ni : -1;
    }
    cap_ = 0;
  }
  ~RcclComm() override {
    if (sbuf_) hipFree(sbuf_);
    if (rbuf_) hipFree(rbuf_);
    if (comm_) ncclCommDestroy(comm_);
  }

  // box of owned points sent toward direction d / ghost box received from direction d
  static Box send_box(const Geom& g, int d, int w) {
    Box b{g.jde1, g.jde2, g.ide1, g.ide2, 0};
    if (DJ[d] < 0) b.j2 = g.jde1 + w - 1;
    if (DJ[d] > 0) b.j1 = g.jde2 - w + 1;
    if (DI[d] < 0) b.i2 = g.ide1 + w - 1;
    if (DI[d] > 0) b.i1 = g.ide2 - w + 1;
    return b;
  }
  static Box recv_box(const Geom& g, int d, int w) {
    Box b{g.jde1, g.jde2, g.ide1, g.ide2, 0};
    if (DJ[d] < 0) { b.j1 = g.jde1 - w; b.j2 = g.jde1 - 1; }
    if (DJ[d] > 0) { b.j1 = g.jde2 + 1; b.j2 = g.jde2 + w; }
    if (DI[d] < 0) { b.i1 = g.ide1 - w; b.i2 = g.ide1 - 1; }
    if (DI[d] > 0) { b.i1 = g.ide2 + 1; b.i2 = g.ide2 + w; }
    return b;
  }
  static bool recv_dir(int sides, int d) {
    if (sides == 0) return true;
    if (sides == 1) return d == 0 || d == 2 || d == 4;   // left, bottom, bottom-left
    return d == 1 || d == 3 || d == 7;                    // right, top, top-right
  }

  void ensure(size_t n) {
    if (n <= cap_) return;
    if (sbuf_) hipFree(sbuf_);
    if (rbuf_) hipFree(rbuf_);
    HIPCHK2(hipMalloc(&sbuf_, n * sizeof(double)));
    HIPCHK2(hipMalloc(&rbuf_, n * sizeof(double)));
    cap_ = n;
  }

  void exchange(const Tile& t, double* field, int nk, int width, int sides) override {
    const Geom& g = t.g;
    Boxes sb{}, rb{};
    int sdir[8], rdir[8];
    long so = 0, ro = 0;
    for (int d = 0; d < 8; d++) {
      if (peer_[d] < 0) continue;
      // receive from d if d is a receive direction; send toward d if opposite(d) is one
      if (recv_dir(sides, OPP[d])) {
        Box b = send_box(g, d, width);
        b.off = so;
        so += (long)(b.j2 - b.j1 + 1) * (b.i2 - b.i1 + 1) * nk;
        sdir[sb.n] = d;
        sb.b[sb.n++] = b;
      }
      if (recv_dir(sides, d)) {
        Box b = recv_box(g, d, width);
        b.off = ro;
        ro += (long)(b.j2 - b.j1 + 1) * (b.i2 - b.i1 + 1) * nk;
        rdir[rb.n] = d;
        rb.b[rb.n++] = b;
      }
    }
    if (sb.n == 0 && rb.n == 0) return;
    ensure((size_t)std::max(so, ro) + 1);
    if (sb.n) hipLaunchKernelGGL(k_pack, dim3(64, 1, sb.n), dim3(256), 0, stream_, g, field, nk, sb, sbuf_);
    NCCLCHK(ncclGroupStart());
    for (int q = 0; q < sb.n; q++) {
      const Box& b = sb.b[q];
      const size_t cnt = (size_t)(b.j2 - b.j1 + 1) * (b.i2 - b.i1 + 1) * nk;
      NCCLCHK(ncclSend(sbuf_ + b.off, cnt, ncclDouble, peer_[sdir[q]], comm_, stream_));
    }
    for (int q = 0; q < rb.n; q++) {
      const Box& b = rb.b[q];
      const size_t cnt = (size_t)(b.j2 - b.j1 + 1) * (b.i2 - b.i1 + 1) * nk;
      NCCLCHK(ncclRecv(rbuf_ + b.off, cnt, ncclDouble, peer_[rdir[q]], comm_, stream_));
    }
    NCCLCHK(ncclGroupEnd());
    if (rb.n) hipLaunchKernelGGL(k_unpack, dim3(64, 1, rb.n), dim3(256), 0, stream_, g, field, nk, rb, rbuf_);
  }

  // exchange_bdy_lr (south/north slices, with left/right tiles) and exchange_bdy_bt
  // (west/east slices, with bottom/top tiles): width-1 ghost entries of every level.
  void exchange_slices(const Tile& t, double* const* sl, long slen, int kz) override {
    const Geom& g = t.g;
    std::vector<int> sidx;
    if (g.bt) for (int s : {10, 11, 14, 15}) sidx.push_back(s);
    if (g.bb) for (int s : {8, 9, 12, 13}) sidx.push_back(s);
    const bool lr = !sidx.empty();
    std::vector<int> sidy;
    if (g.bl) for (int s : {0, 1, 4, 5}) sidy.push_back(s);
    if (g.br) for (int s : {2, 3, 6, 7}) sidy.push_back(s);
    if (sidx.empty() && sidy.empty()) return;
    // Each slice is a [k][idx] array; use 1-row Geom views so k_pack/k_unpack can be reused.
    ensure((size_t)(sidx.size() + sidy.size()) * 4 * kz + 16);
    auto run = [&](const std::vector<int>& ids, int lo, int hi, int d_lo, int d_hi, int origin) {
      // lo/hi: first/last owned index along the slice; origin: frame origin of that index
      for (int s : ids) {
        Geom v{};
        v.j0 = origin; v.i0 = 0; v.pitch = (int)slen; v.plane = slen; v.nj = (int)slen; v.ni = 1;
        v.jde1 = lo; v.jde2 = hi; v.ide1 = 0; v.ide2 = 0;
        Boxes sb{}, rb{};
        int sd[2], rd[2];
        long so = 0, ro = 0;
        for (int side = 0; side < 2; side++) {
          const int d = side == 0 ? d_lo : d_hi;
          if (peer_[d] < 0) continue;
          Box s1{side == 0 ? lo : hi, side == 0 ? lo : hi, 0, 0, so};
          so += kz; sd[sb.n] = d; sb.b[sb.n++] = s1;
          Box r1{side == 0 ? lo - 1 : hi + 1, side == 0 ? lo - 1 : hi + 1, 0, 0, ro};
          ro += kz; rd[rb.n] = d; rb.b[rb.n++] = r1;
        }
        if (!sb.n) continue;
        hipLaunchKernelGGL(k_pack, dim3(1, 1, sb.n), dim3(64), 0, stream_, v, sl[s], kz, sb, sbuf_);
        NCCLCHK(ncclGroupStart());
        for (int q = 0; q < sb.n; q++) NCCLCHK(ncclSend(sbuf_ + sb.b[q].off, kz, ncclDouble, peer_[sd[q]], comm_, stream_));
        for (int q = 0; q < rb.n; q++) NCCLCHK(ncclRecv(rbuf_ + rb.b[q].off, kz, ncclDouble, peer_[rd[q]], comm_, stream_));
        NCCLCHK(ncclGroupEnd());
        hipLaunchKernelGGL(k_unpack, dim3(1, 1, rb.n), dim3(64), 0, stream_, v, sl[s], kz, rb, rbuf_);
      }
    };
    if (lr) run(sidx, g.jde1, g.jde2, 0, 1, g.j0);
    if (!sidy.empty()) run(sidy, g.ide1, g.ide2, 2, 3, g.i0);
  }

  bool graph_safe() const override { return false; }

 private:
  hipStream_t stream_;
  ncclComm_t comm_ = nullptr;
  int peer_[8];
  double* sbuf_ = nullptr;
  double* rbuf_ = nullptr;
  size_t cap_ = 0;
};

}  // namespace

Comm* make_rccl_comm(const rcmdyn_config& cfg, hipStream_t stream) { return new RcclComm(cfg, stream); }

void comm_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace rcm
