// kernels_nh.hpp -- device kernels of the non-hydrostatic step (kernels_nh.hip) and the
// argument block they share.
#pragma once
#include "engine.hpp"

namespace rcm {

// Every buffer of the non-hydrostatic step of one tile.  The NH core updates its state in
// place (no ping-pong), one kernel per reference loop nest or per column recurrence, with
// the intermediates the reference keeps in module arrays held in HBM.  Passed by value.
struct NHFields {
  // state (coupled with p*, as the reference stores it)
  double *a1u, *a1v, *a1t, *a1qv, *a1qc, *a2u, *a2v, *a2t, *a2qv, *a2qc;
  double *a1pp, *a2pp, *a1w, *a2w, *psa, *psb;
  // statics
  const double *msfx, *msfd, *coriol, *ht, *xmsf, *dmsf, *hgfact;
  const int8_t *rgcr, *rgdt;
  const int16_t *ibcr, *ibdt;
  const double *ps0, *pr0, *t0, *rho0, *z0, *pf0, *rhof0, *zf0, *dpsdxm, *dpsdym, *dprddx, *dprddy;
  const double *ef, *ddx, *ddy, *dmdx, *dmdy, *ex, *crx, *cry;
  // boundary data
  const double *ub0, *ubt, *vb0, *vbt, *tb0, *tbt, *qb0, *qbt, *ppb0, *ppbt, *wwb0, *wwbt;
  // 2-D reciprocals (k_surface_pressures)
  const double *rpsa, *rpsb, *rpsda, *rpsdb, *psdota, *psdotb;
  // decoupled / derived fields of the step
  double *ud, *vd, *pr1, *rho1, *xpr;
  double *th;                    // potential temperature atmx%t*(p00/atm1%pr)**rovcp (ithadv = 1)
  double *cr, *qdot;
  double *xkcr;
  // total tendencies (pc_total; pc_dynamic stays in the tendency kernels' registers)
  double *tten, *qvten, *qcten, *uten, *vten;
  double *ppten, *wten;
  // physics tendencies of the coupling seam (null: physics stubbed, the terms are 0)
  const double *tphy, *qvphy, *qcphy, *uphy, *vphy, *ppphy, *wphy;
  // semi-Lagrangian qv/qc tendency starts (isladvec = 1, k_sladv; null otherwise)
  const double *slqv, *slqc;
  // idiffu = 3: the column terms of k_nh_diffu6 (u, v, t, qv, qc, pp, w; null otherwise)
  double *d6u, *d6v, *d6t, *d6qv, *d6qc, *d6pp, *d6w;
  // iuwvadv = 1 (ibltyp = 2): the PBL-top level of vadv4d ind = 3 (null otherwise)
  const double* kpbl;
  // forecasts (atmc) and fixed moisture
  double *ct, *cqv, *cqc, *fqv, *fqc, *cu, *cv, *cpp, *cw, *cdt;
  unsigned* depplane;
  // sound work (Main/mod_sound.F90:40-60) that crosses a kernel boundary: the sweep's e, f
  // (k_nh_sound_bc -> k_nh_sound_cd), pi, the radiative condition's inputs and mask
  double *se, *sf, *spi, *estore, *astore, *tmask;
  unsigned long long* cfl;       // NH_CFL_SLOTS partial maxima of the step's CFL (non-negative
                                 // doubles as ordered bits), reduced by k_nh_advance
  unsigned long long* cfll;      // the same for the last acoustic sub-step alone (the value
                                 // the reference reports, Main/mod_sound.F90:634-646)
  // nqx = 5: atm1 qi, qr, qs (the water load of the adiabatic w term; null for nqx = 2)
  const double* qxa1[NQXH];
  // tfuse = 1: the time filters of t, qv, qc (Main/mod_tendency.F90:422-427) write the other
  // parity b* of those fields (k_nh_tend_c at non-negative forecasts, the negative-moisture fix
  // at the fixed points; k_nh_tend_c copies the points no filter writes); tfuse = 0: in place
  // in k_nh_tfilter_a1
  double *b1t, *b1qv, *b1qc, *b2t, *b2qv, *b2qc;
  int tfuse;
  // NH_NEGLIST: k_nh_tend_c lists its negative qv/qc forecasts (entry (k-1)*plane + ix, times 2,
  // plus the species bit) for k_nh_negfix, which visits the list instead of every point
  unsigned* neglist;
  int* negcnt;
};
constexpr int NH_CFL_SLOTS = 1024;
// block order of the NH tendency kernels: NH_ZFIRST = 1 launches them as (levels, tiles_j,
// tiles_i) grids, consecutive blocks on consecutive levels of one tile
// k_nh_tend_c block: TC_J x TC_I cross points of one level
#ifndef TC_J
#define TC_J 32
#endif
#ifndef TC_I
#define TC_I 8
#endif
// rows of dot points per k_nh_tend_d block (64 x TD_I threads)
#ifndef TD_I
#define TD_I 8
#endif
#ifndef NH_ZFIRST
#define NH_ZFIRST 1
#endif
// acoustic kernels: thread columns aligned to the frame's 128-B lines (ALIGN_J, devcommon.hpp).
// C5, alternating on one box (profiles/r05/c5_nh_align_ab.log): k_nh_sound_bc 762 -> 747 us;
// k_nh_sound_uv unchanged; k_nh_sound_cd 905-953 -> 981-1019 us (its 13th block column of
// mostly idle lanes lengthens a latency-bound column walk), so cd keeps the unaligned map
#ifndef NH_ALIGN
#define NH_ALIGN 1
#endif
#ifndef NH_ALIGN_CD
#define NH_ALIGN_CD 0
#endif
// NH_WRAP: the column kernels k_nh_sound_bc / k_nh_sound_cd on line-aligned block columns
// without the extra column of waves ALIGN_J adds (wrap_j): the lanes of block column 0 that
// fall below jci1 take the row's last columns instead, so a row of 768 columns is 12 waves,
// 11 of them on whole 128-B lines (was 12 misaligned, or 13 aligned)
#ifndef NH_WRAP
#define NH_WRAP 1
#endif
// the same line-aligned columns for the NH point and column kernels that start at jce1, jci1 or
// jde1 (k_nh_sound_uv, k_nh_omega, k_nh_coeff_raw, k_nh_a1_col, k_nh_negfix)
#ifndef NH_WRAP_PT
#define NH_WRAP_PT 1
#endif
#ifndef NH_NEGLIST
#define NH_NEGLIST 1
#endif
// k_nh_tend_c forms decouple's buoyancy helper atmx%pr (xpr) at k and k-1 from the operands it
// loads (decouple stops storing it, and reading t0, rho0 for it)
#ifndef NH_XPRFORM
#define NH_XPRFORM 1
#endif
// acoustic kernels: XCD-aware block placement (xcd_block, devcommon.hpp).  C5, alternating on
// one box (profiles/r05/rejected/c5_xcd_ab.log): k_nh_sound_bc unchanged, k_nh_sound_cd
// 884-894 -> 852-882 us, k_nh_sound_uv 519-521 -> 532-542 us, the step unchanged: off
#ifndef NH_XCD
#define NH_XCD 0
#endif
#if NH_XCD
#define NH_SOUND_POINT(j1, i1) THREAD_POINT_XCD(j1, i1)
#else
#define NH_SOUND_POINT(j1, i1) THREAD_POINT(j1, i1)
#endif
// k_nh_sound_uv forms atm0%dprddx / dprddy from atm0%pr where it reads them
// (Main/mod_params.F90:2676-2686: four-point sums, no rounding beyond the reference's)
#ifndef NH_DPRFORM
#define NH_DPRFORM 1
#endif
// decouple's ud, vd (atm1 u, v * 1/p*dot with the iboudy = 3/4 inflow/outflow rule) formed by
// their readers, k_nh_omega and k_nh_tend_d's staging, from the atm1 winds they load anyway
#ifndef NH_UDFORM
#define NH_UDFORM 1
#endif
// part A of acoustic sub-step 1 (tfuse) and calc_coeff's xkcr as column walks (one thread per
// column, k carried in registers) instead of one thread per point and level
#ifndef NH_A1COL
#define NH_A1COL 1
#endif
#ifndef NH_XKCOL
#define NH_XKCOL 1
#endif

struct QxArgs;
__global__ void k_nh_diffu6(Geom g, const Consts* __restrict__ c, NHFields f, QxArgs q);
__global__ void k_nh_decouple(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_omega(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_coeff_raw(Geom g, const Consts* __restrict__ c, NHFields f);
template <bool QX>
__global__ void k_nh_tend_c(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f, int wdiag, int istep);
__global__ void k_nh_tend_d(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f, int istep);
__global__ void k_nh_negfix(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_negfix_serial(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_tfilter_a1(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_a1_col(Geom g, const Consts* __restrict__ c, NHFields f);
__global__ void k_nh_check_dprd(Geom g, NHFields f, int* bad);
__global__ void k_nh_sound_uv(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f, int istep, int fin, int first, int part);
__global__ void k_nh_sound_bc(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f, int istep, int it);
__global__ void k_nh_tmask_gather(Geom g, const Consts* __restrict__ c, NHFields f, double* gbuf);
__global__ void k_nh_tmask(Geom g, const Consts* __restrict__ c, const double* __restrict__ gbuf, double* tmask);
__global__ void k_nh_sound_cd(Geom g, Geom ge, const double* __restrict__ est, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f, int istep, int last, int nexta);
__global__ void k_nh_sound_final(Geom g, const Consts* __restrict__ c, NHFields f);
int nh_frame_ring(const Geom& g);     // k_nh_sound_final's points per level
__global__ void k_nh_advance(const Consts* __restrict__ c, StepState* s, NHFields f);
__global__ void k_nh_bdyval(Geom g, int kz, const StepState* __restrict__ s, NHFields f);
__global__ void k_nh_bdyval_w1(Geom g, NHFields f);

}  // namespace rcm
