// tke.hpp -- UW PBL turbulent kinetic energy in the dyn step (ibltyp = 2), both cores.
#pragma once
#include "kernels.hpp"
#include "devcommon.hpp"

namespace rcm {

// xk: the full-level diffusion coefficient xkcf (non-hydrostatic core), or, for the
// hydrostatic core, xkc*rdxsq*psb on half levels (k_scalars' xkcs), which xkcf repeats one
// level down (Main/mod_diffusion.F90:232-235, 245): xkcf(1) = xkcs(1), xkcf(k+1) = xkcs(k).
struct TkeArgs {
  const double *a1u, *a1v, *msfd, *xmsf, *psa, *rpsa, *qdot, *xk, *tkephy;
  const double* xkpb;   // NH: xk is the unscaled xkcr, scaled here by rdxsq * p*(b) (xkcf)
  const double* psb;    // idiffu = 3: xkc = diff_6th_coef * p*b
  double *a1tke, *a2tke, *ctke;
  int xk_half;
};

__global__ void k_tke_tend(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, TkeArgs a);
__global__ void k_tke_filter(Geom g, const Consts* __restrict__ c, TkeArgs a);
__global__ void k_bdyval_tke(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, TkeArgs a,
                             Slices sl, long slen);

}  // namespace rcm
