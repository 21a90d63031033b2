// engine.hpp -- internal types of the MI355X dynamical-core engine (not part of the C-ABI).
//
// Data layout in HBM (DESIGN.md "Data layout"): every field of a tile lives on one 2-D frame
// covering the tile's dot-point extents plus a G-point ghost ring, rows j-fastest with a
// padded pitch (multiple of 16 doubles = 128 B), planes stacked by level k:
//   addr(j,i,k) = base + (k-1)*plane + (i-i0)*pitch + (j-j0),   j,i global Fortran indices.
// Cross-point fields use the same frame (their last row/column on the east/north tiles is
// unused), so every kernel indexes every field with the same affine map.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rcmdyn.h"

namespace rcm {

constexpr int G = 4;               // ghost ring of the frame: idif = 2 for idiffu = 1, plus
                                   // room for the width-3 p* exchange (even: 16-B pairs)
constexpr int MAXKZ = RCMDYN_MAXKZ;
constexpr int MAXSPLIT = RCMDYN_MAXSPLIT;
constexpr int MAXNSP = 256;        // max boundary-band width (nspgx)
constexpr int NQXH = 3;            // nqx = 5: the hydrometeors beyond qc (qi, qr, qs)

// Index ranges of one tile, Main/mod_atm_interface.F90:181-381 (global indices).
struct Geom {
  int jde1, jde2, jdi1, jdi2, jdii1, jdii2, ide1, ide2, idi1, idi2, idii1, idii2;
  int jce1, jce2, jci1, jci2, jcii1, jcii2, ice1, ice2, ici1, ici2, icii1, icii2;
  int jde1ga, jde2ga, ide1ga, ide2ga, jce1ga, jce2ga, ice1ga, ice2ga;
  int jci1ga, jci2ga, ici1ga, ici2ga;
  int jde1gb, jde2gb, ide1gb, ide2gb, jce1gb, jce2gb, ice1gb, ice2gb;
  int bl, br, bb, bt;              // has_bdyleft/right/bottom/top
  int band;                        // i_band = 1: periodic in j, no west/east boundary (bl = br = 0)
  int crm;                         // i_crm = 1 (with the band): periodic in i too (bb = bt = 0)
  int gjx, giy;                    // global dot-grid extents
  int j0, i0;                      // global index of frame origin
  int nj, ni;                      // frame size (nj <= pitch)
  int pitch;
  long plane;
  uint32_t P8, L8;                 // row and plane strides in bytes (all fields share them)
  __host__ __device__ __forceinline__ long ix(int j, int i) const {
    return (long)(i - i0) * pitch + (j - j0);
  }
  // byte offset of (j,i) in a 2-D field / of (j,i,k) in a 3-D field
  __host__ __device__ __forceinline__ uint32_t o2(int j, int i) const {
    return (uint32_t)((i - i0) * pitch + (j - j0)) * 8u;
  }
  __host__ __device__ __forceinline__ uint32_t o3(int j, int i, int k) const {
    return o2(j, i) + (uint32_t)(k - 1) * L8;
  }
  // The owned dot (d) and cross (c) ranges extended by the ghost ring toward neighbours (depth
  // 1).  The kernels of a decomposed hydrostatic step compute these rings exactly as their
  // owners do, in place of the halo exchanges the reference performs there.
  __host__ __device__ __forceinline__ int jdx1() const { return jde1 - (bl ? 0 : 1); }
  __host__ __device__ __forceinline__ int jdx2() const { return jde2 + (br ? 0 : 1); }
  __host__ __device__ __forceinline__ int idx1() const { return ide1 - (bb ? 0 : 1); }
  __host__ __device__ __forceinline__ int idx2() const { return ide2 + (bt ? 0 : 1); }
  __host__ __device__ __forceinline__ int jcx1() const { return jce1 - (bl ? 0 : 1); }
  __host__ __device__ __forceinline__ int jcx2() const { return jce2 + (br ? 0 : 1); }
  __host__ __device__ __forceinline__ int icx1() const { return ice1 - (bb ? 0 : 1); }
  __host__ __device__ __forceinline__ int icx2() const { return ice2 + (bt ? 0 : 1); }
  // Global index classes (Main/mod_atm_interface.F90:231-302 on one tile): equal to the tile
  // ranges jce/jci/jcii/jdi/jdii on owned points, and defined on ghost points.  In a band
  // (i_band = 1) every j is interior: the grid is periodic in j and both grids take all jx
  // points (Main/mpplib/mod_mppparam.F90:1131, 1351-1354); with CRM (i_crm = 1) every i too
  // (:1132, 1340-1342).
  __host__ __device__ __forceinline__ bool gce(int j, int i) const {
    return (band || (j >= 1 && j <= gjx - 1)) && (crm || (i >= 1 && i <= giy - 1));
  }
  __host__ __device__ __forceinline__ bool gci(int j, int i) const {
    return (band || (j >= 2 && j <= gjx - 2)) && (crm || (i >= 2 && i <= giy - 2));
  }
  __host__ __device__ __forceinline__ bool gcii(int j, int i) const {
    return (band || (j >= 3 && j <= gjx - 3)) && (crm || (i >= 3 && i <= giy - 3));
  }
  __host__ __device__ __forceinline__ bool gdi(int j, int i) const {
    return (band || (j >= 2 && j <= gjx - 1)) && (crm || (i >= 2 && i <= giy - 1));
  }
  __host__ __device__ __forceinline__ bool gdii(int j, int i) const {
    return (band || (j >= 3 && j <= gjx - 2)) && (crm || (i >= 3 && i <= giy - 2));
  }
  // global west / east boundary column tests (never in a band) and south / north row tests
  // (never with CRM)
  __host__ __device__ __forceinline__ bool gjeq(int j, int v) const { return !band && j == v; }
  __host__ __device__ __forceinline__ bool gieq(int i, int v) const { return !crm && i == v; }
  // the global cross grid (Main/mpplib/mod_mppparam.F90:1486-1516): njcross / nicross points,
  // and its interior range jci / ici over the whole domain (every point in a periodic direction)
  __host__ __device__ __forceinline__ int njcross() const { return band ? gjx : gjx - 1; }
  __host__ __device__ __forceinline__ int nicross() const { return crm ? giy : giy - 1; }
  __host__ __device__ __forceinline__ int gcj1() const { return band ? 1 : 2; }
  __host__ __device__ __forceinline__ int gcj2() const { return band ? gjx : gjx - 2; }
  __host__ __device__ __forceinline__ int gci1() const { return crm ? 1 : 2; }
  __host__ __device__ __forceinline__ int gci2() const { return crm ? giy : giy - 2; }
};
// the negative-moisture fix's row bitmap: words per (species, level) plane; the LDS (doubles) of
// its serial part (qxcommon.hpp): the row sweep's two interior rows and 13 per lane, or the
// wavefront's 4-slot ring per row; the wavefront's block: a thread per interior row
__host__ __device__ __forceinline__ int negfix_rowwords(const Geom& g) { return (g.ici2 - g.ici1 + 1 + 31) / 32; }
__host__ __device__ __forceinline__ int negfix_threads(const Geom& g) {
  const int r = (g.ici2 - g.ici1 + 1 + 63) / 64 * 64;
  return r < 64 ? 64 : (r > 512 ? 512 : r);
}
// the row sweep's LDS (one wavefront: two rows + 13 per lane)
__host__ __device__ __forceinline__ int negfix_sweep_lds(const Geom& g) { return 2 * (g.jci2 - g.jci1 + 1) + 64 * 13; }
// the LDS of a launch whose block per plane can run either path: the wavefront's 4-slot ring per
// row is added only when a negfix_threads block holds a thread per row (a tall tile
// then requests the sweep's LDS and keeps it, instead of failing the launch)
__host__ __device__ __forceinline__ int negfix_lds(const Geom& g) {
  const int a = negfix_sweep_lds(g), R = g.ici2 - g.ici1 + 1, b = R <= negfix_threads(g) ? 4 * R : 0;
  return a > b ? a : b;
}
// columns between j1 and the frame's 128-B line boundary at or below it (ALIGN_J, devcommon.hpp)
__host__ __device__ __forceinline__ int jalign(const Geom& g, int j1) { return (j1 - g.j0) & 15; }

// Run constants (read-only on device, one copy per engine).
struct Consts {
  int kz, nsplit, iboudy, nspgx, stability_enhance, present_qc, ipgf, idiffu;
  int isladvec, iqmsl;                 // semi-Lagrangian moisture advection (physicsparam)
  int ibltyp, iqxvadv;                 // 2: UW PBL TKE advected/diffused/filtered (tke.hip);
                                       // iqxvadv: vadv4d ind of the hydrometeors (3: ibltyp = 2
                                       // with iuwvadv = 1, Main/mod_tendency.F90:148-154; else 1)
  double nuk, tkemin;
  double pgfaa1;                       // ipgf = 1 reference-atmosphere exponent alam*rgas*regrav
  double dx, dx2, dx4, dx8, dx16, dxsq, rdxsq, ptop, ul, xkhmax, dydc, xkhz;
  double diff6;                     // idiffu = 3: diff_6th_coef (Main/mod_diffusion.F90:154)
  double gnu1, gnu2, dtsec, t_extrema, q_rel_extrema;
  double rgas, cpd, c287, ep1, regrav, rovcp;
  double sigma[MAXKZ + 2], hsigma[MAXKZ + 1], dsigma[MAXKZ + 1];
  double twt1[MAXKZ + 1], twt2[MAXKZ + 1], qcon[MAXKZ + 1], xds[MAXKZ + 1];
  double hefc[MAXNSP][MAXKZ + 1], hegc[MAXNSP][MAXKZ + 1];
  double fcx[MAXNSP], gcx[MAXNSP];
  double wgtx[MAXNSP], wgtd[MAXNSP];   // sponge weights (iboudy = 4)
  double zmatx[MAXSPLIT][MAXKZ], zmatxr[MAXSPLIT][MAXKZ], am[MAXSPLIT][MAXKZ];
  double tau[MAXSPLIT][MAXKZ];
  double an[MAXSPLIT], hbar[MAXSPLIT], aam[MAXSPLIT], dtau[MAXSPLIT];
  double pdlog[MAXSPLIT][MAXKZ + 2], eps1[MAXSPLIT][MAXKZ + 2], pd;
  // non-hydrostatic core (idynamic = 2): nonhydroparam and init_sound scalars
  int idynamic, ifupr, ifrayd, rayndamp;
  int crm;                     // i_crm = 1: the Rayleigh damping of u, v, pp toward 0, none of t, qv
  int negfix_mode;             // serial fix of a dense plane: 0 the wavefront, 1 the row sweep (tests)
  double rayalpha0, rayhd, nhbet, nhxkd, nh_dtsmax, nh_xmsf, xgamma, dds[MAXKZ + 2];
  // moisture species (physicsparam ipptls, Main/mod_params.F90:1358-1366): nqx = 2 (qv, qc)
  // or 5 (qv, qc, qi, qr, qs); nsp = nqx - 2 hydrometeors beyond qc
  int ipptls, nqx, nsp;
};

// rcm_timer state on the device, advanced by kernels so one captured step is replayable.
struct StepState {
  double dt;          // current leapfrog dt
  double xbctime;     // s since boundary interval start
  long long lcount;   // completed steps
  double ptntot, pt2tot;
  double cflmax;      // NH: max sigma-velocity CFL of the last acoustic sub-step
                      // (Main/mod_sound.F90:619-646); 0 for the hydrostatic core
  int nanflag;        // sticky: set when a step produced NaN ptntot
  int slflag;         // sticky: a semi-Lagrangian departure point beyond one cell
};

// Per-step copy of the step's error flags in host-mapped memory (k_flag_snapshot, the last
// launch of every tend): the host checks a step's flags once that step's event completed,
// without synchronising the stream.
struct FlagSnap {
  long long lcount;   // the clock after the step
  int nanflag, slflag;
};
constexpr int NFLAGSLOT = 16;       // ring of snapshots, slot (lcount - 1) % NFLAGSLOT

// Per-tile device buffers.
struct Tile {
  int index = 0;                   // tile number in the decomposition
  int lj = 0, li = 0;              // cartesian location
  Geom g{};
  int nbr[8];                      // neighbour tiles: L, R, B, T, BL, BR, TL, TR (-1 none)
  // prognostic state, ping-pong for the 3-D fields written by the fused update kernels
  double *a1u[2], *a1v[2], *a1t[2], *a1qv[2], *a1qc[2];
  double *a2u[2], *a2v[2], *a2t[2], *a2qv[2], *a2qc[2];
  double *psa_[2], *psb_[2];
  int cur = 0;
  int tq = 0;     // NH core: parity of t, qv, qc (the fused time filters ping-pong them)
  double *dstor, *hstor;
  // statics
  double *msfx, *msfd, *coriol, *ht, *xmsf, *dmsf, *hgfact, *mapf;
  int8_t *rgcr, *rgdt;
  int16_t *ibcr, *ibdt;
  // boundary data
  double *ub0, *ubt, *vb0, *vbt, *tb0, *tbt, *qb0, *qbt, *pb0, *pbt;
  // work
  // 2-D reciprocals of the decoupling (decouple / mkslice, recomputed on the fly from them)
  double *rpsa, *rpsb, *rpsda, *rpsdb, *psc, *psdota, *psdotb, *pten;
  double *qdot, *phi;
  double *slqv = nullptr, *slqc = nullptr;   // isladvec = 1: k_sladv output
  // idiffu = 3: the sixth-order terms of the tile's j = jdi2 / jci2 column (k_diffu6), frame
  // planes so one width-1 exchange hands the left neighbour's column to the ring: u, v, t, qv,
  // qc (and NH pp, w on kz + 1 planes)
  double* d6[7] = {};
  // ibltyp = 2: atm1/atm2 tke (decoupled, kz+1 levels), the forecast atmc%tke, and the UW
  // scheme's tendency (allocated on its first put)
  double *a1tke = nullptr, *a2tke = nullptr, *ctke = nullptr, *tkephy = nullptr;
  double* kpbl = nullptr;          // ibltyp = 2: the UW scheme's PBL-top level (put, 2-D)
  double *cqv, *cqc, *fqv, *fqc;
  // nqx = 5: the hydrometeors beyond qc (qi, qr, qs; species.hip), ping-pong like qc, their
  // forecasts / fixed values, the flagged planes of their negative fix, the semi-Lagrangian
  // tendency starts (isladvec = 1) and idiffu = 3 column terms
  double *a1qx[NQXH][2] = {}, *a2qx[NQXH][2] = {};
  double *cqx[NQXH] = {}, *fqx[NQXH] = {}, *slqx[NQXH] = {}, *d6qx[NQXH] = {};
  unsigned* depx = nullptr;          // nqx = 5: the species planes' row bitmaps (as depplane)
  unsigned* depxf = nullptr;         // nqx = 5: the species planes' row flags (k_qx_fix -> k_qx_serial)
  unsigned* depqf = nullptr;         // qfuse: the qv / qc planes' row flags (negfix_list -> the serial passes)
  unsigned *depplane;              // per (n,k) plane: bitmap of the rows with a serially dependent negative point
  int* negcnt = nullptr;           // hydrostatic qfuse: the negative forecasts k_scalars listed
  uint32_t* neglist = nullptr;
  double *deld, *delh, *ddsum, *dhsum, *uu, *vv;
  // diagnostics of the last tend
  double *tten, *uten, *vten, *qvten, *qcten, *omega, *xkcs;
  // boundary slices (Main/mod_bdycod.F90:58-61): [k][frame index]
  double *sl[16];
  // wide frame of the fused split step on a decomposed domain (2-D inputs, ghost depth SPH)
  Geom gw{};
  double *wdeld = nullptr, *wdelh = nullptr, *wpsa = nullptr, *wpsdota = nullptr;
  double *wmsfx = nullptr, *wmsfd = nullptr, *wmapf = nullptr;
  double *westore = nullptr;       // NH: estore of sound on the wide frame (6-deep halo)
  // physics coupling seam: pc_physic tendencies t, qv, qc, u, v, pp, w (allocated on the first
  // put of one of them) and the exported atms slice fields (allocated on the first
  // rcmdyn_tend_pre_physics), in rcmdyn_field order
  double *phy[7] = {};
  double *atms[22] = {};
  double *phyx[NQXH] = {}, *atmsx[NQXH] = {};   // nqx = 5: qxphy and the qxb3d export of qi, qr, qs
  // device bdyin: the raw record put by the host (u, v, t, qv, ps, pp, w) and the coupled
  // boundary data at the interval end (b1, same order), allocated on the first put of a
  // record field; NH: atm0%psdot (Pa) for the coupling of u, v
  double *bin[7] = {};
  double *bb1[7] = {};
  double *psdot0 = nullptr;
  // halo staging buffers
  double *sbuf = nullptr, *rbuf = nullptr;
  double *sbuf2 = nullptr, *rbuf2 = nullptr;   // of the exchange on the engine's second stream
  int red_off = 0, nred = 0;       // this tile's slice of the engine's reduction partials
  int ncolx = 0;                   // k_columns blocks per row
  // halo/compute overlap (Part, kernels.hpp): the rectangle R of points no exchange writes,
  // k_columns' part 1 / part 2 block counts (nint = 0: no split, part 0), and whether any
  // k_momentum / k_scalars block lies in R
  int rja = 0, rjb = -1, ria = 0, rib = -1, rnxb = 0, nint = 0, nring = 0;
  bool mom_in = false, sca_in = false;
  int mj0 = 0, sj0 = 0;         // the block-column origins of k_momentum / k_scalars in parts 1, 2
  long mom_p1 = 0, sca_p1 = 0;  // points their part-1 blocks compute (rcmdyn_overlap_shares)
  std::vector<void*> allocs;
};

}  // namespace rcm
