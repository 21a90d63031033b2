// tke.hip -- UW PBL turbulent kinetic energy in the dyn step (ibltyp = 2), both cores.
//
// The reference advects (hadv3d ind = 1 of atm1%tke, vadv3d ind = 0 of tke*p*, Main/
// mod_tendency.F90:1414-1425), diffuses (diffu_x3df with nuk, :1545-1548), forecasts and
// filters (:515-544) the TKE the UW scheme produces; bdyval bounds it (Main/mod_bdycod.F90:
// 1166-1306, 2415-2530).  The TKE feeds no other dyn field, so these kernels stand apart from
// the fused step: k_tke_tend writes the forecast atmc%tke, k_tke_filter the Robert-Asselin
// filtered time levels, k_bdyval_tke the boundary lines after bdyval's slices are ready.
#include <hip/hip_runtime.h>

#include "tke.hpp"

namespace rcm {

// tkedyn + forecast, one thread per interior cross point and full level k = 1..kz+1.
// The accumulation order per point is the reference's: 0, hadv (k = 2..kz), the vadv flux
// through the level above (k-1, added) and below (k, subtracted), then the diffusion.
__global__ void k_tke_tend(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, TkeArgs a) {
  THREAD_POINT(g.jci1, g.ici1);
  if (j > g.jci2 || i > g.ici2) return;
  const int kz = c->kz;
  const double* f = a.a1tke;
  double ften = d_zero;
  auto umc = [&](int jj, int ii, int kk) { return F3(a.a1u, jj, ii, kk) * F2(a.msfd, jj, ii); };
  auto vmc = [&](int jj, int ii, int kk) { return F3(a.a1v, jj, ii, kk) * F2(a.msfd, jj, ii); };
  if (k >= 2 && k <= kz) {                  // hadv3d ind = 1, Main/mod_advection.F90:481-505
    const double uavg1 = umc(j, i + 1, k) + umc(j, i, k), uavg2 = umc(j + 1, i + 1, k) + umc(j + 1, i, k);
    const double vavg1 = vmc(j + 1, i, k) + vmc(j, i, k), vavg2 = vmc(j + 1, i + 1, k) + vmc(j, i + 1, k);
    const double uavg1m = umc(j, i + 1, k - 1) + umc(j, i, k - 1);
    const double uavg2m = umc(j + 1, i + 1, k - 1) + umc(j + 1, i, k - 1);
    const double vavg1m = vmc(j + 1, i, k - 1) + vmc(j, i, k - 1);
    const double vavg2m = vmc(j + 1, i + 1, k - 1) + vmc(j, i + 1, k - 1);
    const double t1 = c->twt1[k], t2 = c->twt2[k];
    const double uaz1 = (t1 * uavg1 + t2 * uavg1m), uaz2 = (t1 * uavg2 + t2 * uavg2m);
    const double vaz1 = (t1 * vavg1 + t2 * vavg1m), vaz2 = (t1 * vavg2 + t2 * vavg2m);
    const double ps = F2(a.psa, j, i), ul = c->ul;
    const double f1 = d_half * ul * (uavg2 + uavg1) / ps;
    const double f2 = d_half * ul * (vavg2 + vavg1) / ps;
    const double fc = F3(f, j, i, k);
    const double fx1 = (d_one + f1) * F3(f, j - 1, i, k) + (d_one - f1) * fc;
    const double fx2 = (d_one + f1) * fc + (d_one - f1) * F3(f, j + 1, i, k);
    const double fy1 = (d_one + f2) * F3(f, j, i - 1, k) + (d_one - f2) * fc;
    const double fy2 = (d_one + f2) * fc + (d_one - f2) * F3(f, j, i + 1, k);
    ften = ften - F2(a.xmsf, j, i) * (uaz2 * fx2 - uaz1 * fx1 + vaz2 * fy2 - vaz1 * fy1);
  }
  {                                         // vadv3d ind = 0, nk = kz+1, :756-765 on tke*p*
    const double ps = F2(a.psa, j, i);
    auto flux = [&](int kk) {               // through the interface between kk and kk+1
      const double qq = d_half * (F3(a.qdot, j, i, kk) + F3(a.qdot, j, i, kk + 1));
      return qq * ((F3(f, j, i, kk) * ps + F3(f, j, i, kk + 1) * ps));
    };
    if (k >= 2) ften = ften + flux(k - 1) * c->dds[k];
    if (k <= kz) ften = ften - flux(k) * c->dds[k];
  }
  {                                         // diffu_x3df(tkedyn, atm2%tke, nuk), :523-598
    const double* x = a.a2tke;
    const double xk = a.xkpb ? F3(a.xk, j, i, k > 1 ? k - 1 : 1) * c->rdxsq * F2(a.xkpb, j, i)
                    : a.xk_half ? F3(a.xk, j, i, k > 1 ? k - 1 : 1) : F3(a.xk, j, i, k);
    const double fac = c->nuk;
#define X(dj, di) F3(x, j + (dj), i + (di), k)
    if (c->idiffu == 3) {                   // :602-651, the tile's column j = jci2 only (fac * xkc)
      if (j == g.jci2) {
        auto fv = [&](int jj, int ii) { return F3(x, jj, ii, k); };
        auto lv = [&](int jj, int ii) { return F3(x, jj, ii, k) / F2(a.msfd, jj, ii); };
        ften = ften + fac * (c->diff6 * F2(a.psb, j, i)) * diffu6_bracket(j, i, g.gjx - 1, g.giy - 1, fv, lv);
      }
    } else if (c->idiffu == 2) {
      ften = ften + fac * xk * (o4_c1 * (X(1, 0) + X(-1, 0) + X(0, 1) + X(0, -1)) +
                                o4_c2 * (X(1, 1) + X(-1, -1) + X(-1, 1) + X(1, -1)) + o4_c3 * X(0, 0));
    } else {
      if (g.gcii(j, i))
        ften = ften - fac * xk * (z4_c1 * (X(2, 0) + X(-2, 0) + X(0, 2) + X(0, -2)) +
                                  z4_c2 * (X(1, 0) + X(-1, 0) + X(0, 1) + X(0, -1)) + z4_c3 * X(0, 0));
      const double lap2 = z4_c1 * (X(1, 0) + X(-1, 0) + X(0, 1) + X(0, -1)) + z4_c2 * X(0, 0);
      if (g.gjeq(j, 2)) ften = ften + fac * xk * lap2;
      if (g.gjeq(j, g.gjx - 2)) ften = ften + fac * xk * lap2;
      if (g.gieq(i, 2)) ften = ften + fac * xk * lap2;
      if (g.gieq(i, g.giy - 2)) ften = ften + fac * xk * lap2;
    }
#undef X
  }
  // tketen = (0 + tkedyn*rpsa) + tkephy, atmc%tke = max(tkemin, atm2%tke + dt*tketen)
  const double ten = (d_zero + ften * F2(a.rpsa, j, i)) + (a.tkephy ? F3(a.tkephy, j, i, k) : d_zero);
  const double v = F3(a.a2tke, j, i, k) + s->dt * ten;
  F3(a.ctke, j, i, k) = (v > c->tkemin) ? v : c->tkemin;
}

// filter_ra_3d(atm1%tke, atm2%tke, atmc%tke, gnu2), Main/mod_timefilter.F90:53-70
__global__ void k_tke_filter(Geom g, const Consts* __restrict__ c, TkeArgs a) {
  THREAD_POINT(g.jci1, g.ici1);
  if (j > g.jci2 || i > g.ici2) return;
  const double n1 = F3(a.a1tke, j, i, k), np = F3(a.ctke, j, i, k), nm = F3(a.a2tke, j, i, k);
  const double d = c->gnu2 * (np + nm - d_two * n1);
  F3(a.a2tke, j, i, k) = n1 + d;
  F3(a.a1tke, j, i, k) = np;
}

// bdyval for the TKE, one block per full level: atm2 = atm1 on the boundary lines while
// integrating (:1166-1306); then tkemin on every boundary line at the start, else (bdyflow)
// tkemin at k = 1 and, for the levels k+1 = 3..kz+1, tkemin at inflow and the first interior
// value at outflow (:2438-2509; level 2 is left as it is, as written).  West/east first: they
// read the south/north lines at jci1/jci2 before those are set.
__global__ void k_bdyval_tke(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, TkeArgs a,
                             Slices sl, long slen) {
  const int k = (int)blockIdx.x + 1, kz = c->kz;
  const double tmin = c->tkemin;
  double* t1 = a.a1tke;
  double* t2 = a.a2tke;
  const int tx = (int)threadIdx.x, nt = (int)blockDim.x;
  if (s->lcount > 0) {
    for (int i = g.ici1 + tx; i <= g.ici2; i += nt) {
      if (g.bl) F3(t2, g.jce1, i, k) = F3(t1, g.jce1, i, k);
      if (g.br) F3(t2, g.jce2, i, k) = F3(t1, g.jce2, i, k);
    }
    for (int j = g.jce1 + tx; j <= g.jce2; j += nt) {
      if (g.bb) F3(t2, j, g.ice1, k) = F3(t1, j, g.ice1, k);
      if (g.bt) F3(t2, j, g.ice2, k) = F3(t1, j, g.ice2, k);
    }
    __syncthreads();
  }
  if (s->lcount == 0) {                     // rcmtimer%start(): :2416-2431
    for (int i = g.ice1 + tx; i <= g.ice2; i += nt) {
      if (g.bl) { F3(t1, g.jce1, i, k) = tmin; F3(t2, g.jce1, i, k) = tmin; }
      if (g.br) { F3(t1, g.jce2, i, k) = tmin; F3(t2, g.jce2, i, k) = tmin; }
    }
    for (int j = g.jce1 + tx; j <= g.jce2; j += nt) {
      if (g.bt) { F3(t1, j, g.ice2, k) = tmin; F3(t2, j, g.ice2, k) = tmin; }
      if (g.bb) { F3(t1, j, g.ice1, k) = tmin; F3(t2, j, g.ice1, k) = tmin; }
    }
    return;
  }
  // level k = kk + 1 of the reference's loop kk = 2..kz reads the slices at kk and kk - 1
  const int kk = k - 1;
  for (int i = g.ice1 + tx; i <= g.ice2; i += nt) {
    if (g.bl) {
      if (k == 1) { F3(t1, g.jce1, i, 1) = tmin; F3(t2, g.jce1, i, 1) = tmin; }
      else if (kk >= 2 && kk <= kz) {
        const double tint = F3(t1, g.jci1, i, k);
        const double w = SLI(sl.s[0], i, kk) + SLI(sl.s[0], i + 1, kk) + SLI(sl.s[1], i, kk) + SLI(sl.s[1], i + 1, kk) +
                         SLI(sl.s[0], i, kk - 1) + SLI(sl.s[0], i + 1, kk - 1) + SLI(sl.s[1], i, kk - 1) +
                         SLI(sl.s[1], i + 1, kk - 1);
        F3(t1, g.jce1, i, k) = (w > d_zero) ? tmin : tint;
      }
    }
    if (g.br) {
      if (k == 1) { F3(t1, g.jce2, i, 1) = tmin; F3(t2, g.jce2, i, 1) = tmin; }
      else if (kk >= 2 && kk <= kz) {
        const double tint = F3(t1, g.jci2, i, k);
        const double w = SLI(sl.s[2], i, kk) + SLI(sl.s[2], i + 1, kk) + SLI(sl.s[3], i, kk) + SLI(sl.s[3], i + 1, kk) +
                         SLI(sl.s[2], i, kk - 1) + SLI(sl.s[2], i + 1, kk - 1) + SLI(sl.s[3], i, kk - 1) +
                         SLI(sl.s[3], i + 1, kk - 1);
        F3(t1, g.jce2, i, k) = (w < d_zero) ? tmin : tint;
      }
    }
  }
  __syncthreads();
  for (int j = g.jce1 + tx; j <= g.jce2; j += nt) {
    if (g.bb) {
      if (k == 1) { F3(t1, j, g.ice1, 1) = tmin; F3(t2, j, g.ice1, 1) = tmin; }
      else if (kk >= 2 && kk <= kz && in(j, g.jci1, g.jci2)) {
        const double tint = F3(t1, j, g.ici1, k);
        const double w = SLJ(sl.s[12], j, kk) + SLJ(sl.s[12], j + 1, kk) + SLJ(sl.s[13], j, kk) + SLJ(sl.s[13], j + 1, kk) +
                         SLJ(sl.s[12], j, kk - 1) + SLJ(sl.s[12], j + 1, kk - 1) + SLJ(sl.s[13], j, kk - 1) +
                         SLJ(sl.s[13], j + 1, kk - 1);
        F3(t1, j, g.ice1, k) = (w > d_zero) ? tmin : tint;
      }
    }
    if (g.bt) {
      if (k == 1) { F3(t1, j, g.ice2, 1) = tmin; F3(t2, j, g.ice2, 1) = tmin; }
      else if (kk >= 2 && kk <= kz && in(j, g.jci1, g.jci2)) {
        const double tint = F3(t1, j, g.ici2, k);
        const double w = SLJ(sl.s[14], j, kk) + SLJ(sl.s[14], j + 1, kk) + SLJ(sl.s[15], j, kk) + SLJ(sl.s[15], j + 1, kk) +
                         SLJ(sl.s[14], j, kk - 1) + SLJ(sl.s[14], j + 1, kk - 1) + SLJ(sl.s[15], j, kk - 1) +
                         SLJ(sl.s[15], j + 1, kk - 1);
        F3(t1, j, g.ice2, k) = (w < d_zero) ? tmin : tint;
      }
    }
  }
}

}  // namespace rcm
