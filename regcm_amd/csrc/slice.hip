// slice.hip -- device mkslice export for the physics coupling seam.
//
// The reference prepares the `atms` slice fields the physics reads in mkslice
// (Main/mod_slice.F90:102-358), called from tend before new_pressure (Main/mod_tendency.F90:
// 243).  The dyn kernels never store them (they form the decoupled products where they read
// them); rcmdyn_tend_pre_physics runs this kernel so a host running physics can fetch them.
// One thread per owned column walks the levels; every product and clamp is the reference's
// expression in its order (-ffp-contract=off), the powers/logs use the device libm.
#include "slice.hpp"

namespace rcm {

namespace {

constexpr double P00 = 1.0e5;                 // Share/mod_constants.F90:229
constexpr double TZERO = 273.15;              // :197
constexpr double EGRAV_S = 9.80665;           // :85

// pfesat / pfwsat, Share/pfesat.inc, Share/pfwsat.inc (Flatau et al. 1992 polynomials)
__device__ double pfwsat(double t, double p, double ep2) {
  double tl = t - TZERO;
  if (tl > 100.0) tl = 100.0;
  if (tl < -75.0) tl = -75.0;
  const double td = tl;
  double esat;
  if (td >= 0.0)
    esat = 6.11213476 + td * (0.444007856 + td * (0.143064234e-01 + td * (0.264461437e-03 + td * (0.305903558e-05 +
           td * (0.196237241e-07 + td * (0.892344772e-10 + td * (-0.373208410e-12 + td * 0.209339997e-15)))))));
  else
    esat = 6.11123516 + td * (0.503109514 + td * (0.188369801e-01 + td * (0.420547422e-03 + td * (0.614396778e-05 +
           td * (0.602780717e-07 + td * (0.387940929e-09 + td * (0.149436277e-11 + td * 0.262655803e-14)))))));
  const double es = esat * 100.0;
  return ep2 * (es / (p - es));
}

__device__ __forceinline__ double omega_hydro(const Geom& g, const Consts* c, const SliceArgs& a, int j, int i, int k) {
  // Main/mod_tendency.F90:1195-1214 (ud/vd = atm1 * (1/psdota), decouple :880-906)
#define UD(J, I) (F3(a.a1u, J, I, k) * F2(a.rpsda, J, I))
#define VD(J, I) (F3(a.a1v, J, I, k) * F2(a.rpsda, J, I))
  const double dummy = d_one / (c->dx8 * F2(a.msfx, j, i));
  const double ps = F2(a.psa, j, i);
  return d_half * (F3(a.qdot, j, i, k + 1) + F3(a.qdot, j, i, k)) * ps +
         c->hsigma[k] * (F2(a.pten, j, i) +
                         ((UD(j, i) + UD(j, i + 1) + UD(j + 1, i + 1) + UD(j + 1, i)) *
                              (F2(a.psa, j + 1, i) - F2(a.psa, j - 1, i)) +
                          (VD(j, i) + VD(j, i + 1) + VD(j + 1, i + 1) + VD(j + 1, i)) *
                              (F2(a.psa, j, i + 1) - F2(a.psa, j, i - 1))) * dummy);
#undef UD
#undef VD
}

}  // namespace

__global__ __launch_bounds__(256) void k_slice(Geom g, const Consts* __restrict__ c, SliceArgs a) {
  const int j = g.jde1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ide1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jde2 || i > g.ide2) return;
  const int kz = c->kz;
  const bool nh = c->idynamic == 2;
  const bool ce = in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
  const bool ci = in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2);
  const double rgas = c->rgas, ptop = c->ptop, ep1 = c->ep1;
  const double rovcp = rgas * (d_one / c->cpd), rovg = rgas / EGRAV_S, regrav = c->regrav;
  const double rpsb = F2(a.rpsb, j, i), rpsdb = F2(a.rpsdb, j, i), psb = F2(a.psb, j, i);
  // ps2d (:220-234): NH from atm0 and the lowest pp, hydrostatic from psb
  double ps2d;
  if (nh) ps2d = F2(a.ps0, j, i) + ptop * d_1000 + F3(a.a2pp, j, i, kz) * rpsb;
  else ps2d = (psb + ptop) * d_1000;
  if (ce) F2(a.ps2d, j, i) = ps2d;
  double wpx_m = 0.0, rhob_m = 1.0;
  for (int k = 1; k <= kz; k++) {
    // ubd3d/vbd3d (:171-174) on every dot point, ubx3d/vbx3d (:176-183) on cross points
    const double ubd = F3(a.a2u, j, i, k) * rpsdb, vbd = F3(a.a2v, j, i, k) * rpsdb;
    F3(a.ubd3d, j, i, k) = ubd;
    F3(a.vbd3d, j, i, k) = vbd;
    if (ce) {
#define UBD(J, I) (F3(a.a2u, J, I, k) * F2(a.rpsdb, J, I))
#define VBD(J, I) (F3(a.a2v, J, I, k) * F2(a.rpsdb, J, I))
      F3(a.ubx3d, j, i, k) = d_rfour * (UBD(j, i) + UBD(j, i + 1) + UBD(j + 1, i) + UBD(j + 1, i + 1));
      F3(a.vbx3d, j, i, k) = d_rfour * (VBD(j, i) + VBD(j, i + 1) + VBD(j + 1, i) + VBD(j + 1, i + 1));
#undef UBD
#undef VBD
    }
    // tb3d, qxb3d (:185-189) on jx1:jx2 (cross points and ghosts), tv3d (:199-202)
    if (!ce) continue;
    const double tb = F3(a.a2t, j, i, k) * rpsb;
    const double qvb = dmax(F3(a.a2qv, j, i, k) * rpsb, MINQQ);
    const double qcb = dmax(F3(a.a2qc, j, i, k) * rpsb, d_zero);
    F3(a.tb3d, j, i, k) = tb;
    F3(a.qvb3d, j, i, k) = qvb;
    F3(a.qcb3d, j, i, k) = qcb;
    for (int n = 0; n < c->nsp; n++) F3(a.qxb3d[n], j, i, k) = dmax(F3(a.a2qx[n], j, i, k) * rpsb, d_zero);
    const double tv = tb * (d_one + ep1 * qvb - qcb);
    F3(a.tv3d, j, i, k) = tv;
    // pb3d (:207-214 NH, :226-228 hydrostatic)
    double pb;
    if (nh) {
      const double ppb = F3(a.a2pp, j, i, k) * rpsb;
      pb = F3(a.pr0, j, i, k) + ppb;
      if (k == 1) pb = dmax(pb, ptop * d_1000 + 1.0);
    } else {
      pb = (c->hsigma[k] * psb + ptop) * d_1000;
    }
    F3(a.pb3d, j, i, k) = pb;
    // th3d (:244-247), rhob3d / tp3d (:248-252), qsb3d / rhb3d (:331-338)
    F3(a.th3d, j, i, k) = tb * pow(P00 / pb, rovcp);
    const double qs = pfwsat(tb, pb, a.ep2);
    F3(a.qsb3d, j, i, k) = qs;
    if (!ci) continue;
    const double rhob = pb / (rgas * tb);
    F3(a.rhob3d, j, i, k) = rhob;
    F3(a.tp3d, j, i, k) = tb * pow(ps2d / pb, rovcp);
    double rh = qvb / qs;
    rh = dmin(dmax(rh, a.rhmin), a.rhmax);
    F3(a.rhb3d, j, i, k) = rh;
    if (k == kz) F2(a.rhox2d, j, i) = ps2d / (rgas * tb);   // :240-242
    // wpx3d (:254-262): omega of compute_omega (Pa/s; the hydrostatic omega is in cb/s)
    double wpx;
    if (nh) {
      wpx = -d_half * EGRAV_S * F3(a.rho0, j, i, k) * rpsb * (F3(a.a2w, j, i, k) + F3(a.a2w, j, i, k + 1));
    } else {
      wpx = omega_hydro(g, c, a, j, i, k) * d_1000;
    }
    F3(a.wpx3d, j, i, k) = wpx;
    // hydrostatic wb3d (:266-271) from the level above
    if (!nh && k >= 2) F3(a.wb3d, j, i, k) = -d_half * regrav * (wpx_m / rhob_m + wpx / rhob);
    wpx_m = wpx;
    rhob_m = rhob;
  }
  if (nh) {
    // wb3d (:263-265) on jx1:jx2, pf3d (:215-225)
    if (!ce) return;
    for (int k = 1; k <= kz + 1; k++) F3(a.wb3d, j, i, k) = F3(a.a2w, j, i, k) * rpsb;
    F3(a.pf3d, j, i, 1) = ptop * d_1000;
    F3(a.pf3d, j, i, kz + 1) = ps2d;
    for (int k = 2; k <= kz; k++)
      F3(a.pf3d, j, i, k) = F3(a.pf0, j, i, k) + d_half * (F3(a.a2pp, j, i, k - 1) * rpsb + F3(a.a2pp, j, i, k) * rpsb);
    return;
  }
  if (!ce) return;
  for (int k = 1; k <= kz + 1; k++) F3(a.pf3d, j, i, k) = (c->sigma[k] * psb + ptop) * d_1000;
  // zq, za, dzq (:273-293): column recurrence from the top of the atmosphere down
  const double cell = ptop * rpsb;
  double zq = d_zero;
  F3(a.zq, j, i, kz + 1) = zq;
  for (int k = kz; k >= 1; k--) {
    const double tv = F3(a.tv3d, j, i, k);
    const double zk = zq + rovg * tv * log((c->sigma[k + 1] + cell) / (c->sigma[k] + cell));
    F3(a.zq, j, i, k) = zk;
    F3(a.za, j, i, k) = d_half * (zk + zq);
    F3(a.dzq, j, i, k) = zk - zq;
    zq = zk;
  }
}

}  // namespace rcm
