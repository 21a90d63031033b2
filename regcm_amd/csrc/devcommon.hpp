// devcommon.hpp -- device helpers shared by the hydrostatic (kernels.hip) and the
// non-hydrostatic (kernels_nh.hip) kernels: frame indexing, reference constants, psc2psd.
#pragma once
#include "engine.hpp"

namespace rcm {

#define F2(a, j, i) (a)[g.ix(j, i)]
#define F3(a, j, i, k) (a)[(long)((k) - 1) * g.plane + g.ix(j, i)]
#define SLI(s, i, k) (s)[(long)((k) - 1) * slen + ((i) - g.i0)]
#define SLJ(s, j, k) (s)[(long)((k) - 1) * slen + ((j) - g.j0)]
// byte-offset access
#define LD(a, o) (*(const double*)((const char*)(a) + (uint32_t)(o)))
#define ST(a, o, v) (*(double*)((char*)(a) + (uint32_t)(o)) = (v))
// neighbour offsets relative to the thread's point (o2: 2-D, o3: 3-D at level k)
#define O2(dj, di) (o2 + (uint32_t)((dj) * 8) + (uint32_t)(di) * P8)
#define O3(dj, di) (o3 + (uint32_t)((dj) * 8) + (uint32_t)(di) * P8)
#define O3K(dj, di, dk) (O3(dj, di) + (uint32_t)(dk) * L8)

static constexpr double d_zero = 0.0, d_one = 1.0, d_two = 2.0, d_four = 4.0;
static constexpr double d_half = 0.5, d_rfour = 0.25, d_1000 = 1000.0;
static constexpr double MINQQ = 1.0e-8, DLOWVAL = 1.0e-20;
static constexpr double z4_c1 = 1.0, z4_c2 = -4.0, z4_c3 = 12.0;
static constexpr double o4_c1 = 4.0 / 6.0, o4_c2 = 1.0 / 6.0, o4_c3 = -20.0 / 6.0;  // idiffu = 2
static constexpr double h4_c1 = 10.0, h4_c2 = -5.0, h4_c3 = 1.0;                   // idiffu = 3
static constexpr double T00PG = 287.0, P00PG = 101.325;   // ipgf = 1, Share/mod_constants.F90:359-360

__device__ __forceinline__ double dmax(double a, double b) { return (a > b) ? a : (b > a ? b : a); }
__device__ __forceinline__ double dmin(double a, double b) { return (a < b) ? a : (b < a ? b : a); }

__device__ __forceinline__ bool in(int v, int lo, int hi) { return v >= lo && v <= hi; }



// Block phase timing (build with -DRCM_PHASE_TIMING): thread 0 of every block records
// wall-clock marks (100 MHz) into a device buffer that rcm_phase_dump() (kernels.hip) writes
// to a file; the measurement behind the kernel structure notes in DESIGN.md.
#ifdef RCM_PHASE_TIMING
struct PtRec { int kid, bx, by, bz, n, pad; long long t[8]; };
constexpr int PT_CAP = 1 << 17;
static __device__ PtRec rcm_pt_buf[PT_CAP];
static __device__ int rcm_pt_count = 0;
#define PT_DECL long long pt_[8]; int pt_n_ = 0; pt_[pt_n_++] = wall_clock64();
#define PT_MARK() do { if (pt_n_ < 7) pt_[pt_n_++] = wall_clock64(); } while (0)
#define PT_PRINT(KID_)                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && threadIdx.y == 0) {                                                 \
      pt_[pt_n_++] = wall_clock64();                                                            \
      const int q_ = atomicAdd(&rcm_pt_count, 1);                                               \
      if (q_ < PT_CAP) {                                                                        \
        PtRec& r_ = rcm_pt_buf[q_];                                                             \
        r_.kid = KID_; r_.bx = blockIdx.x; r_.by = blockIdx.y; r_.bz = blockIdx.z; r_.n = pt_n_;  \
        for (int e_ = 0; e_ < pt_n_; e_++) r_.t[e_] = pt_[e_];                                  \
      }                                                                                         \
    }                                                                                           \
  } while (0)
#else
#define PT_DECL
#define PT_MARK() do { } while (0)
#define PT_PRINT(KID_) do { } while (0)
#endif

// XCD-aware block placement.  The workgroups of a launch go round-robin over the 8 XCDs, each
// with its own L2: in blockIdx order the four neighbours of a tile run on other XCDs, so every
// stencil halo is fetched again from beyond L2.  xcd_block() renumbers the blocks: launch-order
// block b takes tile start(b % 8) + b / 8 of the row-major tile order (x fastest, z slowest), so
// each XCD walks one contiguous band of tile rows and the rows above and below a tile are (but
// at the band edges) its own XCD's.
struct Blk3 {
  int x, y, z;
};
__device__ __forceinline__ Blk3 xcd_block() {
  const int nx = (int)gridDim.x, ny = (int)gridDim.y;
  const int n = nx * ny * (int)gridDim.z;
  const int b = ((int)blockIdx.z * ny + (int)blockIdx.y) * nx + (int)blockIdx.x;
  const int per = n >> 3, rem = n & 7, x = b & 7;
  const int t = x * per + (x < rem ? x : rem) + (b >> 3);
  return {t % nx, (t / nx) % ny, t / (nx * ny)};
}
// the same within one z slice: (x, y) renumbered so each XCD walks one contiguous band of the
// slice's rows; z (a level, say) keeps its launch order
__device__ __forceinline__ void xcd_tile2d(int& bx, int& by) {
  const int nx = (int)gridDim.x, n = nx * (int)gridDim.y;
  const int b = (int)blockIdx.y * nx + (int)blockIdx.x;
  const int per = n >> 3, rem = n & 7, x = b & 7;
  const int t = x * per + (x < rem ? x : rem) + (b >> 3);
  bx = t % nx;
  by = t / nx;
}
// the same over a range of the launch: the blocks B in [base, base + n) of the launch's linear
// (dispatch) order, renumbered 0..n-1 so that each XCD (B mod 8) takes one contiguous run; a
// kernel whose consecutive work items share operands (the levels of one column block, the rows
// of one column stripe) then finds them in its own XCD's L2
__device__ __forceinline__ int xcd_range(int B, int base, int n) {
  const int x = B & 7, b0 = base & 7;
  int t = 0;
  for (int y = 0; y < x; y++) {
    const int f = base + ((y - b0 + 8) & 7);        // first block of the range on XCD y
    t += f < base + n ? (base + n - 1 - f) / 8 + 1 : 0;
  }
  const int fx = base + ((x - b0 + 8) & 7);
  return t + (B - fx) / 8;
}
// THREAD_POINT over xcd_block()'s tile
#define THREAD_POINT_XCD(j1, i1)                                        \
  const Blk3 xb_ = xcd_block();                                         \
  const int j = (j1) + xb_.x * (int)blockDim.x + (int)threadIdx.x;      \
  const int i = (i1) + xb_.y * (int)blockDim.y + (int)threadIdx.y;      \
  const int k = xb_.z + 1;                                              \
  (void)k;

// thread -> (j, i, k) over a box starting at (j1, i1); k = blockIdx.z + 1
#define THREAD_POINT(j1, i1)                                   \
  const int j = (j1) + (int)(blockIdx.x * blockDim.x + threadIdx.x); \
  const int i = (i1) + (int)(blockIdx.y * blockDim.y + threadIdx.y); \
  const int k = (int)blockIdx.z + 1;                              \
  (void)k;

// The frame's rows start on 128-B lines (pitch of 16 doubles), but the index ranges start a
// few points in (jde1 = j0 + G): a 64-wide wavefront from jde1 touches five lines per field
// instead of four, and the fifth is fetched again by the neighbouring block (another XCD).
// ALIGN_J moves a box's first thread column down to the line boundary at or below j1 (those
// lanes idle: every such kernel rejects j < j1 by its own range test); jalign (engine.hpp) is
// the host's matching count of extra columns for the grid.
#define ALIGN_J(j1) ((j1) - jalign(g, j1))

// psc2psd at one dot point, Main/mpplib/mod_mppparam.F90:13811-13862.
__device__ __forceinline__ bool psc2psd_at(const Geom& g, const double* pc, int j, int i, double& v) {
  if (in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2)) {
    v = (F2(pc, j, i) + F2(pc, j, i - 1) + F2(pc, j - 1, i) + F2(pc, j - 1, i - 1)) * d_rfour;
    return true;
  }
  if (g.bt && i == g.ide2 && in(j, g.jdi1, g.jdi2)) { v = (F2(pc, j, g.ice2) + F2(pc, j - 1, g.ice2)) * d_half; return true; }
  if (g.bb && i == g.ide1 && in(j, g.jdi1, g.jdi2)) { v = (F2(pc, j, g.ice1) + F2(pc, j - 1, g.ice1)) * d_half; return true; }
  if (g.bl && j == g.jde1 && in(i, g.idi1, g.idi2)) { v = (F2(pc, g.jce1, i) + F2(pc, g.jce1, i - 1)) * d_half; return true; }
  if (g.br && j == g.jde2 && in(i, g.idi1, g.idi2)) { v = (F2(pc, g.jce2, i) + F2(pc, g.jce2, i - 1)) * d_half; return true; }
  if (g.bb && g.bl && j == g.jde1 && i == g.ide1) { v = F2(pc, g.jce1, g.ice1); return true; }
  if (g.bt && g.bl && j == g.jde1 && i == g.ide2) { v = F2(pc, g.jce1, g.ice2); return true; }
  if (g.bb && g.br && j == g.jde2 && i == g.ide1) { v = F2(pc, g.jce2, g.ice1); return true; }
  if (g.bt && g.br && j == g.jde2 && i == g.ide2) { v = F2(pc, g.jce2, g.ice2); return true; }
  return false;
}

// ---------------------------------------------------------------------------------------
// psc2psd at any dot point from the global domain extents (tile ghosts included),
// Main/mpplib/mod_mppparam.F90:13811-13862: 4-point mean inside, 2-point means on the domain
// edges, corner copies.  Equal to psc2psd_at on every owned point.
__device__ __forceinline__ double psc2psd_global(const Geom& g, const double* pc, int j, int i) {
  const int jx = g.gjx, iy = g.giy;
  const bool jin = g.band || (j >= 2 && j <= jx - 1), iin = g.crm || (i >= 2 && i <= iy - 1);   // a band: every j, CRM: every i
  if (jin && iin) return (F2(pc, j, i) + F2(pc, j, i - 1) + F2(pc, j - 1, i) + F2(pc, j - 1, i - 1)) * d_rfour;
  if (jin && i == iy) return (F2(pc, j, iy - 1) + F2(pc, j - 1, iy - 1)) * d_half;
  if (jin && i == 1) return (F2(pc, j, 1) + F2(pc, j - 1, 1)) * d_half;
  if (iin && j == 1) return (F2(pc, 1, i) + F2(pc, 1, i - 1)) * d_half;
  if (iin && j == jx) return (F2(pc, jx - 1, i) + F2(pc, jx - 1, i - 1)) * d_half;
  return F2(pc, (j == 1) ? 1 : jx - 1, (i == 1) ? 1 : iy - 1);
}

// idiffu = 3, the sixth-order flux-limited scheme (Main/mod_diffusion.F90:412-516 diffu_d,
// 736-785 diffu_x3d, 893-942 diffu_x4d3d).  The reference applies it on one column of each
// tile, j = jdi2 (dot) / jci2 (cross), every row of the interior, with neighbour indices
// clamped to the global domain (1..jx, 1..iy on dot points; 1..jx-1, 1..iy-1 on cross points).
// fv gives the field in the fluxes, lv the field over msfd in the limiter.
template <class FV, class LV>
__device__ __forceinline__ double diffu6_bracket(int j, int i, int jmax, int imax, FV fv, LV lv) {
  const int jm1 = max(j - 1, 1), jm2 = max(j - 2, 1), jm3 = max(j - 3, 1);
  const int jp1 = min(j + 1, jmax), jp2 = min(j + 2, jmax), jp3 = min(j + 3, jmax);
  const int im1 = max(i - 1, 1), im2 = max(i - 2, 1), im3 = max(i - 3, 1);
  const int ip1 = min(i + 1, imax), ip2 = min(i + 2, imax), ip3 = min(i + 3, imax);
  double x0 = h4_c1 * (fv(j, i) - fv(jm1, i)) + h4_c2 * (fv(jp1, i) - fv(jm2, i)) + h4_c3 * (fv(jp2, i) - fv(jm3, i));
  if (x0 * (lv(j, i) - lv(jm1, i)) <= d_zero) x0 = d_zero;
  double x1 = h4_c1 * (fv(jp1, i) - fv(j, i)) + h4_c2 * (fv(jp2, i) - fv(jm1, i)) + h4_c3 * (fv(jp3, i) - fv(jm2, i));
  if (x1 * (lv(jp1, i) - lv(j, i)) <= d_zero) x1 = d_zero;
  double y0 = h4_c1 * (fv(j, i) - fv(j, im1)) + h4_c2 * (fv(j, ip1) - fv(j, im2)) + h4_c3 * (fv(j, ip2) - fv(j, im3));
  if (y0 * (lv(j, i) - lv(j, im1)) <= d_zero) y0 = d_zero;
  double y1 = h4_c1 * (fv(j, ip1) - fv(j, i)) + h4_c2 * (fv(j, ip2) - fv(j, im1)) + h4_c3 * (fv(j, ip3) - fv(j, im2));
  if (y1 * (lv(j, ip1) - lv(j, i)) <= d_zero) y1 = d_zero;
  return (x1 - x0) + (y1 - y0);
}

// vadv4d ind = 3 (iuwvadv = 1 with ibltyp = 2, Main/mod_advection.F90:917-957): the hydrometeor
// interface value at interface kk (2..kz) before the svv factor.  The linear interpolation
// twt(kk,1) f(kk) + twt(kk,2) f(kk-1), replaced at kpb - 1 and kpb (kpb >= 4) by the PBL-top
// rule: a slope from the layer above the ambiguous one (levels kpb-3..kpb-1, zero unless f is
// monotone there), extended from f(kpb-2) to the interfaces; at kpb the extension is kept only
// if it does not overshoot f(kpb) by more than f(kpb-1) does.  fk(k) reads f at level k of the
// column (called only on the two replaced interfaces).
template <class FK>
__device__ __forceinline__ double uw_fg(const Consts* c, int kk, int kpb, double fkk, double fkm, FK fk) {
  if (kpb >= 4 && (kk == kpb - 1 || kk == kpb)) {
    const int k0 = kpb - 2;
    const double fp = fk(k0 + 1), f0 = fk(k0), fm = fk(k0 - 1), fb = fk(kpb);
    double slope;
    if ((fp - f0) > d_zero && (f0 - fm) > d_zero)
      slope = dmin((fp - f0) / (c->hsigma[k0 + 1] - c->hsigma[k0]), (f0 - fm) / (c->hsigma[k0] - c->hsigma[k0 - 1]));
    else if ((fp - f0) < d_zero && (f0 - fm) < d_zero)
      slope = dmax((fp - f0) / (c->hsigma[k0 + 1] - c->hsigma[k0]), (f0 - fm) / (c->hsigma[k0] - c->hsigma[k0 - 1]));
    else
      slope = d_zero;
    // f(kpb-2) = f0, f(kpb-1) = fp
    if (kk == kpb - 1) return f0 + slope * (c->sigma[kpb - 1] - c->hsigma[kpb - 2]);
    if (fabs(f0 + slope * (c->hsigma[kpb - 1] - c->hsigma[kpb - 2]) - fb) > fabs(fp - fb)) return fb;
    return f0 + slope * (c->sigma[kpb] - c->hsigma[kpb - 2]);
  }
  return c->twt1[kk] * fkk + c->twt2[kk] * fkm;
}

}  // namespace rcm
