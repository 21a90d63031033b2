// kernels_nh.hip -- HIP/CDNA4 kernels of the non-hydrostatic (MM5-type) dynamical-core step
// (idynamic = 2): the NH branches of tend (Main/mod_tendency.F90), the acoustic sub-stepping
// of sound (Main/mod_sound.F90:163-718), Rayleigh damping (Main/mod_bdycod.F90:4953-5123)
// and the NH boundary values.  ithadv = 1 (the only NH temperature path of the reference,
// Main/mod_tendency.F90:98,128-129), ipptls = 1, i_crm = 0, physics stubbed.
//
// Every value is formed with the same floating-point operation order as oracle/rcm_oracle.c
// (compiled with -ffp-contract=off), so transcendental-free results are bit-identical.  The
// kernels fuse the reference's loop nests where that keeps each element's operation sequence:
// a chain of nests that each update only their own element becomes one thread's register
// accumulation (k_nh_tend_c / k_nh_tend_d), a column recurrence absorbs the level-parallel work
// that feeds it (k_nh_sound_bc / k_nh_sound_cd), and a decoupled product of a state field is
// formed where it is read instead of being stored.  The state is updated in place (the
// reference's own semantics); the intermediates that remain live in HBM (NHFields).  DESIGN.md
// section 4.2 lists the kernels with their roofline position.
#include "engine.hpp"
#include "kernels_nh.hpp"
#include "kernels.hpp"
#include "fastmath.hpp"
#include "devcommon.hpp"
#include "qxcommon.hpp"

namespace rcm {

// k_nh_tend_c is compiled in a translation unit of its own (kernels_nh_tc.hip includes this file
// with RCM_NH_TEND_C_TU defined) so that the Makefile can give it its own device scheduler; the
// other kernels are compiled here
#ifdef RCM_NH_TEND_C_TU
#define NH_OTHER_KERNELS 0
#else
#define NH_OTHER_KERNELS 1
#endif

static constexpr double EGRAV_NH = 9.80665;                 // Share/mod_constants.F90:85
static constexpr double REARTHRAD = 1.0 / 6.371229e6;       // :282-284
static constexpr double MATHPI = 3.1415926535897932384626433832795029;
static constexpr double P00 = 1.000000e5;                  // Share/mod_constants.F90:229

#define IN_CE(j, i) (in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2))
#define IN_CI(j, i) (in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2))
#define IN_DI(j, i) (in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2))
#define IN_DE(j, i) (in(j, g.jde1, g.jde2) && in(i, g.ide1, g.ide2))
// wrap_j (NH_WRAP): column of lane tx in block column bx over the n columns from j1, the block
// columns starting on the 128-B line at or below j1; lanes below j1 (block column 0 only) take
// the columns past the last of the ceil(n/64) block columns
__device__ __forceinline__ int wrap_j(const Geom& g, int j1, int n, int bx, int tx) {
  const int ja = j1 - jalign(g, j1);
  int j = ja + bx * 64 + tx;
  if (j < j1) j += ((n + 63) / 64) * 64;
  return j;
}
// thread -> (j, i, k) over the columns j1..j2 on wrap_j's block columns (64 x 4 blocks, grid3's
// count of block columns); NH_WRAP_PT = 0: THREAD_POINT from j1
#if NH_WRAP_PT
#define WRAP_POINT(j1, j2, i1)                                                        \
  const int j = wrap_j(g, j1, (j2) - (j1) + 1, (int)blockIdx.x, (int)threadIdx.x);   \
  const int i = (i1) + (int)(blockIdx.y * blockDim.y + threadIdx.y);                 \
  const int k = (int)blockIdx.z + 1;                                                  \
  (void)k;
#else
#define WRAP_POINT(j1, j2, i1) THREAD_POINT(j1, i1)
#endif
#if NH_ZFIRST
#define TBX ((int)blockIdx.y)
#define TBY ((int)blockIdx.z)
#define TBZ ((int)blockIdx.x)
#else
#define TBX ((int)blockIdx.x)
#define TBY ((int)blockIdx.y)
#define TBZ ((int)blockIdx.z)
#endif
__device__ __forceinline__ int j0c(const Geom& g) { return g.j0; }
__device__ __forceinline__ int i0c(const Geom& g) { return g.i0; }
#define FRAME_POINT()                                                  \
  THREAD_POINT(g.j0, g.i0);                                             \
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;

// decoupled boundary ud/vd with the iboudy = 3/4 inflow/outflow rule (see udvd_bdy in
// kernels.hip; Main/mod_tendency.F90:893-994)
__device__ double2 udvd_nh(const Geom& g, int iboudy, const double* a1u, const double* a1v, const double* rpsda,
                           int j, int i, int k) {
  auto base = [&](int jj, int ii) {
    const double r = F2(rpsda, jj, ii);
    return make_double2(F3(a1u, jj, ii, k) * r, F3(a1v, jj, ii, k) * r);
  };
  if (iboudy != 3 && iboudy != 4) return base(j, i);
  // global boundary lines (a ghost point on them carries the value its owner computes and
  // the reference exchanges)
  auto we = [&](int jj, int ii) {
    if (in(ii, 2, g.giy - 1)) {
      if (g.gjeq(jj, 1) && F3(a1u, jj, ii, k) <= d_zero) return base(2, ii);
      if (g.gjeq(jj, g.gjx) && F3(a1u, jj, ii, k) >= d_zero) return base(g.gjx - 1, ii);
    }
    return base(jj, ii);
  };
  if (g.band || in(j, 1, g.gjx)) {
    if (g.gieq(i, 1) && F3(a1v, j, i, k) >= d_zero) return we(j, 2);
    if (g.gieq(i, g.giy) && F3(a1v, j, i, k) <= d_zero) return we(j, g.giy - 1);
  }
  return we(j, i);
}

// ud, vd of one dot point from its atm1 u, v (au, av) and 1/p*dot (r), already loaded by the
// caller: udvd_nh's values (the inflow/outflow rule only on the global boundary lines)
__device__ __forceinline__ double2 udvd_nh_ld(const Geom& g, int iboudy, const NHFields& f, double au, double av,
                                              double r, int j, int i, int k) {
  if ((iboudy == 3 || iboudy == 4) && (g.gjeq(j, 1) || g.gjeq(j, g.gjx) || g.gieq(i, 1) || g.gieq(i, g.giy)))
    return udvd_nh(g, iboudy, f.a1u, f.a1v, f.rpsda, j, i, k);
  return make_double2(au * r, av * r);
}

// ---------------------------------------------------------------------------------------
// decouple NH (Main/mod_tendency.F90:852-1066): the decoupled winds ud, vd (with the iboudy
// inflow/outflow rule) on the dot frame; atm1 pr/rho, the buoyancy helper atmx%pr and the
// potential temperature th of ithadv = 1 (:1349-1353) on the cross frame with its ghost ring,
// the points exchange(th,1) fills: th is pointwise in atmx%t and atm1%pr, which are defined
// there.  The other decoupled fields -- umc, vmc, umd, vmd and atmx w, pp, qv, qc -- are one
// product (and clip) of a state field each and are formed by their readers.
#if NH_OTHER_KERNELS
__global__ void k_nh_decouple(Geom g, const Consts* __restrict__ c, NHFields f) {
  FRAME_POINT();
  const int kz = c->kz;
#if !NH_UDFORM
  if (k <= kz && in(j, g.jde1ga, g.jde2ga) && in(i, g.ide1ga, g.ide2ga)) {
    const double2 d = udvd_nh(g, c->iboudy, f.a1u, f.a1v, f.rpsda, j, i, k);
    F3(f.ud, j, i, k) = d.x;                           // umd = ud*msfd: formed by omega, tend_d
    F3(f.vd, j, i, k) = d.y;
  }
#endif
  if (!(in(j, g.jce1ga, g.jce2ga) && in(i, g.ice1ga, g.ice2ga))) return;
  const double rp = F2(f.rpsa, j, i);
  if (k > kz) return;
#if NH_NEGLIST
  if (j == g.jce1 && i == g.ice1 && k == 1) *f.negcnt = 0;      // k_nh_tend_c lists after this
#endif
  const double xt = F3(f.a1t, j, i, k) * rp;
  const double xqv = dmax(F3(f.a1qv, j, i, k) * rp, MINQQ);
  const double xtv = xt * (d_one + c->ep1 * xqv);
  const double xpp = F3(f.a1pp, j, i, k) * rp;
  const double pr1 = F3(f.pr0, j, i, k) + xpp;
  F3(f.pr1, j, i, k) = pr1;      // atmx t, tv, qv, qc, pp, w: formed by their readers
  F3(f.rho1, j, i, k) = pr1 / (c->rgas * xtv);
  F3(f.th, j, i, k) = xt * rcm_powpos(P00 / pr1, c->rovcp);
#if !NH_XPRFORM
  if (IN_CI(j, i))
    F3(f.xpr, j, i, k) = (xtv - F3(f.t0, j, i, k) - xpp / (c->cpd * F3(f.rho0, j, i, k))) / xt;
#endif
}
#endif

// compute_omega NH (:1157-1191), one thread per cross column: qdot from w and the terrain
// slopes of the reference p*, then the mass divergence with the qdot term
#if NH_OTHER_KERNELS
// 256-thread blocks at 3 waves/SIMD: the one-pass form needs 138 VGPRs (under the default
// 1 024-thread bound it spilled 44 B at 128); C5 321 -> 279 us (profiles/r05/c5_cd_omega_ab.log)
#ifndef NHOM_W
#define NHOM_W 3
#endif
__global__ __launch_bounds__(256, NHOM_W) void k_nh_omega(Geom g, const Consts* __restrict__ c, NHFields f) {
  WRAP_POINT(g.jce1, g.jce2, g.ice1);
  if (!IN_CE(j, i)) return;
  const int kz = c->kz;
  const double dummy = d_one / (c->dx2 * F2(f.msfx, j, i) * F2(f.msfx, j, i));
  // umd, vmd = ud, vd * msfd (decouple :893-994) at the four dot points of the column
  const double m00 = F2(f.msfd, j, i), m01 = F2(f.msfd, j, i + 1), m10 = F2(f.msfd, j + 1, i),
               m11 = F2(f.msfd, j + 1, i + 1);
  auto ucc = [&](int kk) {
    return F3(f.ud, j, i, kk) * m00 + F3(f.ud, j, i + 1, kk) * m01 + F3(f.ud, j + 1, i, kk) * m10 +
           F3(f.ud, j + 1, i + 1, kk) * m11;
  };
  auto vcc = [&](int kk) {
    return F3(f.vd, j, i, kk) * m00 + F3(f.vd, j, i + 1, kk) * m01 + F3(f.vd, j + 1, i, kk) * m10 +
           F3(f.vd, j + 1, i + 1, kk) * m11;
  };
  const double ps0 = F2(f.ps0, j, i), dx = F2(f.dpsdxm, j, i), dy = F2(f.dpsdym, j, i);
  F3(f.qdot, j, i, 1) = d_zero;
  F3(f.qdot, j, i, kz + 1) = d_zero;
#if NH_UDFORM
  // ud, vd formed here from atm1 u, v at the column's four dot points (decouple no longer
  // stores them), one pass over the levels: the level's winds give qdot(k) and, with
  // qdot(k-1), the mass divergence cr(k-1) (the same expressions as the two loops below)
  (void)ucc; (void)vcc;
  const double r00 = F2(f.rpsda, j, i), r01 = F2(f.rpsda, j, i + 1), r10 = F2(f.rpsda, j + 1, i),
               r11 = F2(f.rpsda, j + 1, i + 1);
  const int ib = c->iboudy;
  const double ps = F2(f.psa, j, i), rpa = F2(f.rpsa, j, i);
  struct W4 { double u00, u01, u10, u11, v00, v01, v10, v11; };
  auto ld = [&](int kk) {
    W4 a;
    a.u00 = F3(f.a1u, j, i, kk); a.u01 = F3(f.a1u, j, i + 1, kk); a.u10 = F3(f.a1u, j + 1, i, kk);
    a.u11 = F3(f.a1u, j + 1, i + 1, kk);
    a.v00 = F3(f.a1v, j, i, kk); a.v01 = F3(f.a1v, j, i + 1, kk); a.v10 = F3(f.a1v, j + 1, i, kk);
    a.v11 = F3(f.a1v, j + 1, i + 1, kk);
    return a;
  };
  auto dsum = [&](const W4& a, int kk, double& uk, double& vk) {     // ucc, vcc
    const double2 d00 = udvd_nh_ld(g, ib, f, a.u00, a.v00, r00, j, i, kk);
    const double2 d01 = udvd_nh_ld(g, ib, f, a.u01, a.v01, r01, j, i + 1, kk);
    const double2 d10 = udvd_nh_ld(g, ib, f, a.u10, a.v10, r10, j + 1, i, kk);
    const double2 d11 = udvd_nh_ld(g, ib, f, a.u11, a.v11, r11, j + 1, i + 1, kk);
    uk = d00.x * m00 + d01.x * m01 + d10.x * m10 + d11.x * m11;
    vk = d00.y * m00 + d01.y * m01 + d10.y * m10 + d11.y * m11;
  };
  auto crab = [&](const W4& a) {       // umc, vmc = atm1 u, v * msfd (decouple)
    const double x = a.u11 * m11 + a.u10 * m10 - a.u01 * m01 - a.u00 * m00;
    const double y = a.v11 * m11 + a.v01 * m01 - a.v10 * m10 - a.v00 * m00;
    return x + y;
  };
  W4 wa = ld(1);
  double um, vm;
  dsum(wa, 1, um, vm);
  double abm = crab(wa), qm = d_zero;
  for (int k = 2; k <= kz; k++) {
    const W4 wb = ld(k);
    double uk, vk;
    dsum(wb, k, uk, vk);
    const double qk = -F3(f.rhof0, j, i, k) * EGRAV_NH * (F3(f.a1w, j, i, k) * rpa) / ps0 -
                      c->sigma[k] * (dx * (c->twt1[k] * uk + c->twt2[k] * um) +
                                     dy * (c->twt1[k] * vk + c->twt2[k] * vm));
    F3(f.qdot, j, i, k) = qk;
    F3(f.cr, j, i, k - 1) = abm * dummy + (qk - qm) * ps / c->dsigma[k - 1];
    abm = crab(wb); qm = qk; um = uk; vm = vk;
  }
  F3(f.cr, j, i, kz) = abm * dummy + (d_zero - qm) * ps / c->dsigma[kz];
#else
  double um = ucc(1), vm = vcc(1);
  for (int k = 2; k <= kz; k++) {
    const double uk = ucc(k), vk = vcc(k);
    F3(f.qdot, j, i, k) = -F3(f.rhof0, j, i, k) * EGRAV_NH * (F3(f.a1w, j, i, k) * F2(f.rpsa, j, i)) / ps0 -
                          c->sigma[k] * (dx * (c->twt1[k] * uk + c->twt2[k] * um) +
                                         dy * (c->twt1[k] * vk + c->twt2[k] * vm));
    um = uk; vm = vk;
  }
  const double ps = F2(f.psa, j, i);
  for (int k = 1; k <= kz; k++) {
    // umc, vmc = atm1 u, v * msfd (decouple)
    const double a = F3(f.a1u, j + 1, i + 1, k) * m11 + F3(f.a1u, j + 1, i, k) * m10 -
                     F3(f.a1u, j, i + 1, k) * m01 - F3(f.a1u, j, i, k) * m00;
    const double b = F3(f.a1v, j + 1, i + 1, k) * m11 + F3(f.a1v, j, i + 1, k) * m01 -
                     F3(f.a1v, j + 1, i, k) * m10 - F3(f.a1v, j, i, k) * m00;
    F3(f.cr, j, i, k) = (a + b) * dummy + (F3(f.qdot, j, i, k + 1) - F3(f.qdot, j, i, k)) * ps / c->dsigma[k];
  }
#endif
}
#endif

// mkslice NH subset (Main/mod_slice.F90:163-183, 278-281): the b-level decoupled winds, t, q,
// pp and w (atm2 times 1/psdotb or 1/psb, q clipped at minqq / 0) are formed by their readers
// as they load them -- k_nh_coeff_raw and the LDS staging of k_nh_tend_c / k_nh_tend_d --
// so they never reach memory (the NH level pressures of :207-225 are formed by the
// physics-seam export, slice.hip, which is their only reader)
#define UBD(J, I, K) (F3(f.a2u, J, I, K) * F2(f.rpsdb, J, I))
#define VBD(J, I, K) (F3(f.a2v, J, I, K) * F2(f.rpsdb, J, I))

// calc_coeff NH (Main/mod_diffusion.F90:215-250): Smagorinsky coefficient with the
// vertical-velocity term, unscaled (xkcr) ...
#if NH_OTHER_KERNELS
#if NH_XKCOL
// one thread per cross frame column walking k = 1..kz: a2w * (1/p*b) of level k+1 is carried to
// the next level (the point form reads it again from the k+1 plane); the same values
__global__ void k_nh_coeff_raw(Geom g, const Consts* __restrict__ c, NHFields f) {
  WRAP_POINT(g.jce1, g.jce2, g.ice1);
  if (!IN_CE(j, i)) return;
  const double rpb = F2(f.rpsb, j, i), hg = F2(f.hgfact, j, i);
  const double r00 = F2(f.rpsdb, j, i), r10 = F2(f.rpsdb, j + 1, i), r01 = F2(f.rpsdb, j, i + 1),
               r11 = F2(f.rpsdb, j + 1, i + 1);
  const int kz = c->kz;
  double wk = F3(f.a2w, j, i, 1) * rpb;
#pragma unroll 2
  for (int kk = 1; kk <= kz; kk++) {
    const double u00 = F3(f.a2u, j, i, kk) * r00, u10 = F3(f.a2u, j + 1, i, kk) * r10,
                 u01 = F3(f.a2u, j, i + 1, kk) * r01, u11 = F3(f.a2u, j + 1, i + 1, kk) * r11;
    const double v00 = F3(f.a2v, j, i, kk) * r00, v10 = F3(f.a2v, j + 1, i, kk) * r10,
                 v01 = F3(f.a2v, j, i + 1, kk) * r01, v11 = F3(f.a2v, j + 1, i + 1, kk) * r11;
    const double wk1 = F3(f.a2w, j, i, kk + 1) * rpb;
    const double dudx = u10 + u11 - u00 - u01;
    const double dvdx = v10 + v11 - v00 - v01;
    const double dudy = u01 + u11 - u00 - u10;
    const double dvdy = v01 + v11 - v00 - v10;
    const double dwdz = wk - wk1;
    const double duv = sqrt(dmax((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy) - dwdz * dwdz, d_zero));
    F3(f.xkcr, j, i, kk) = dmin(hg + c->dydc * duv, c->xkhmax);
    wk = wk1;
  }
}
#else
__global__ void k_nh_coeff_raw(Geom g, const Consts* __restrict__ c, NHFields f) {
  WRAP_POINT(g.jce1, g.jce2, g.ice1);
  if (!IN_CE(j, i)) return;
  const double u00 = UBD(j, i, k), u10 = UBD(j + 1, i, k), u01 = UBD(j, i + 1, k), u11 = UBD(j + 1, i + 1, k);
  const double v00 = VBD(j, i, k), v10 = VBD(j + 1, i, k), v01 = VBD(j, i + 1, k), v11 = VBD(j + 1, i + 1, k);
  const double dudx = u10 + u11 - u00 - u01;
  const double dvdx = v10 + v11 - v00 - v01;
  const double dudy = u01 + u11 - u00 - u10;
  const double dvdy = v01 + v11 - v00 - v10;
  const double rpb = F2(f.rpsb, j, i);
  const double dwdz = F3(f.a2w, j, i, k) * rpb - F3(f.a2w, j, i, k + 1) * rpb;
  const double duv = sqrt(dmax((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy) - dwdz * dwdz, d_zero));
  F3(f.xkcr, j, i, k) = dmin(F2(f.hgfact, j, i) + c->dydc * duv, c->xkhmax);
}
#endif
#endif

// ... then scaled by rdxsq and p* (b) by their readers: xkc, xkcf (cross interior, full
// levels: xkcr of level k-1) in k_nh_tend_c, xkd (dot interior, the four-point mean) in
// k_nh_tend_d (Main/mod_diffusion.F90:236-250)

// upstream flux form of hadvt/hadvqv/hadvqx/hadv3d ind 0 at one cross point
// (Main/mod_advection.F90:337-386, 547-596, 639-653, 466-480) on the values of the advected
// field at the point and its west/east/south/north neighbours; limiter 0 none, 1 t, 2 q
__device__ __forceinline__ double hadv_v(const Consts* c, double fc, double fw, double fe, double fs, double fn,
                                         double u1, double u2, double v1, double v2, double xmf, double ps,
                                         int limiter) {
  const double f1 = d_half * c->ul * (u2 + u1) / ps;
  const double f2 = d_half * c->ul * (v2 + v1) / ps;
  const double fx1 = (d_one + f1) * fw + (d_one - f1) * fc;
  const double fx2 = (d_one + f1) * fc + (d_one - f1) * fe;
  const double fy1 = (d_one + f2) * fs + (d_one - f2) * fc;
  const double fy2 = (d_one + f2) * fc + (d_one - f2) * fn;
  double fg = -xmf * (u2 * fx2 - u1 * fx1 + v2 * fy2 - v1 * fy1);
  if (limiter && c->stability_enhance) {
    double den, thr;
    if (limiter == 1) { den = ps; thr = c->t_extrema; }
    else { den = dmax(fc, DLOWVAL); thr = c->q_rel_extrema; }
    if (fabs(fn + fs - d_two * fc) / den > thr) {
      if (fc > fn && fc > fs) fg = dmin(fg, d_zero);
      else if (fc < fn && fc < fs) fg = dmax(fg, d_zero);
    }
    if (fabs(fe + fw - d_two * fc) / den > thr) {
      if (fc > fe && fc > fw) fg = dmin(fg, d_zero);
      else if (fc < fe && fc < fw) fg = dmax(fg, d_zero);
    }
  }
  return fg;
}

__device__ __forceinline__ double nh_relax(double ften, double xf, double xg, double f0, double f1, double f2,
                                           double f3, double f4) {
  return ften + xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0);
}

// 4th-order (idiffu = 1) / 9-point (idiffu = 2) diffusion of one cross field at (j,i,k)
// (diffu_x3d / diffu_x3df / diffu_x4d3d, Main/mod_diffusion.F90:523-790)
__device__ __forceinline__ double diffx_at(const Geom& g, const Consts* c, double ften, const double* fa,
                                           const double* xk, int j, int i, int k) {
  if (c->idiffu == 2) {
    return ften + d_one * F3(xk, j, i, k) *
        (o4_c1 * (F3(fa, j + 1, i, k) + F3(fa, j - 1, i, k) + F3(fa, j, i + 1, k) + F3(fa, j, i - 1, k)) +
         o4_c2 * (F3(fa, j + 1, i + 1, k) + F3(fa, j - 1, i - 1, k) + F3(fa, j - 1, i + 1, k) + F3(fa, j + 1, i - 1, k)) +
         o4_c3 * F3(fa, j, i, k));
  }
  if (in(j, g.jcii1, g.jcii2) && in(i, g.icii1, g.icii2))
    ften = ften - d_one * F3(xk, j, i, k) *
        (z4_c1 * (F3(fa, j + 2, i, k) + F3(fa, j - 2, i, k) + F3(fa, j, i + 2, k) + F3(fa, j, i - 2, k)) +
         z4_c2 * (F3(fa, j + 1, i, k) + F3(fa, j - 1, i, k) + F3(fa, j, i + 1, k) + F3(fa, j, i - 1, k)) +
         z4_c3 * F3(fa, j, i, k));
  const double lap = z4_c1 * (F3(fa, j + 1, i, k) + F3(fa, j - 1, i, k) + F3(fa, j, i + 1, k) + F3(fa, j, i - 1, k)) +
                     z4_c2 * F3(fa, j, i, k);
  const int nb = (g.bl && j == g.jci1) + (g.br && j == g.jci2) + (g.bb && i == g.ici1) + (g.bt && i == g.ici2);
  for (int q = 0; q < nb; q++) ften = ften + d_one * F3(xk, j, i, k) * lap;
  return ften;
}

// idiffu = 3 (Main/mod_diffusion.F90:412-516, 602-651, 736-785, 893-942): the sixth-order
// terms of the tile's column, j = jdi2 for u, v and j = jci2 for t, qv, qc, pp (levels 1..kz)
// and w (1..kz+1; diffu_x3df reads xkc on level kz+1, one past its kz levels -- the
// coefficient is diff_6th_coef * p*b on every level, as xkcf holds it), from the decoupled
// atm2 fields of mkslice (Main/mod_slice.F90:163-183, 215-238).  blockIdx.z: 0 u and v, 1 t,
// 2 qv, 3 qc, 4 pp, 5 w, 6.. qi, qr, qs (nqx = 5); blockIdx.y = level.  k_nh_tend_c /
// k_nh_tend_d / k_nh_qx_tend add them in the reference's place of the diffusion term.
#if NH_OTHER_KERNELS
__global__ void k_nh_diffu6(Geom g, const Consts* __restrict__ c, NHFields f, QxArgs qx) {
  const int i = g.ide1 + (int)(blockIdx.x * blockDim.x + threadIdx.x), k = (int)blockIdx.y + 1;
  const int q0 = (int)blockIdx.z, kz = c->kz;
  const int q = q0 >= 6 ? 3 : q0;                  // the species take qc's clip and stencil
  const double* ps = f.psb;
  double* d6 = q0 >= 6 ? qx.d6[q0 - 6]
               : q == 0 ? f.d6u : q == 1 ? f.d6t : q == 2 ? f.d6qv : q == 3 ? f.d6qc : q == 4 ? f.d6pp : f.d6w;
  if (k > (q == 5 ? kz + 1 : kz)) return;
  if (q == 0) {
    const int j = g.jdi2;
    if (!in(i, g.idi1, g.idi2)) return;
    auto rd = [&](int jj, int ii) { return d_one / psc2psd_global(g, ps, jj, ii); };
    auto uu = [&](int jj, int ii) { return F3(f.a2u, jj, ii, k) * rd(jj, ii) / F2(f.msfd, jj, ii); };
    auto vv = [&](int jj, int ii) { return F3(f.a2v, jj, ii, k) * rd(jj, ii) / F2(f.msfd, jj, ii); };
    const double xkd = c->diff6 * psc2psd_global(g, ps, j, i);
    F3(d6, j, i, k) = xkd * diffu6_bracket(j, i, g.gjx, g.giy, uu, uu);
    F3(f.d6v, j, i, k) = xkd * diffu6_bracket(j, i, g.gjx, g.giy, vv, vv);
    return;
  }
  const int j = g.jci2;
  if (!in(i, g.ici1, g.ici2)) return;
  const double* a = q0 >= 6 ? qx.a2[q0 - 6] : q == 1 ? f.a2t : q == 2 ? f.a2qv : q == 3 ? f.a2qc : q == 4 ? f.a2pp : f.a2w;
  auto fv = [&](int jj, int ii) {
    const double v = F3(a, jj, ii, k) * (d_one / F2(ps, jj, ii));
    return q == 2 ? dmax(v, MINQQ) : (q == 3 ? dmax(v, d_zero) : v);
  };
  auto lv = [&](int jj, int ii) { return fv(jj, ii) / F2(f.msfd, jj, ii); };
  const double xkc = d_one * (c->diff6 * F2(ps, j, i));
  F3(d6, j, i, k) = xkc * diffu6_bracket(j, i, g.gjx - 1, g.giy - 1, fv, lv);
}
#endif
// the column term where k_nh_tend_c / k_nh_tend_d add diffusion
__device__ __forceinline__ double diff6_add(const Geom& g, double ften, const double* d6, int jc, int j, int i, int k) {
  return j == jc ? ften + F3(d6, j, i, k) : ften;
}

// tau, Main/mod_bdycod.F90:5115-5123
__device__ __forceinline__ double nh_tau(const Consts* c, double z, double zmax) {
  if (z > zmax - c->rayhd) {
    const double s = sin((MATHPI * d_half) * (d_one - (zmax - z) / c->rayhd));
    return c->rayalpha0 * (s * s);
  }
  return d_zero;
}

// diffx_at on a field staged in LDS: S[ti][tj] is the thread's point
template <int W>
__device__ __forceinline__ double diffx_l(const Geom& g, const Consts* c, double ften, const double (*S)[W],
                                          double xk, int j, int i, int ti, int tj) {
#define SA(dj, di) S[ti + (di)][tj + (dj)]
  if (c->idiffu == 2) {
    return ften + d_one * xk *
        (o4_c1 * (SA(1, 0) + SA(-1, 0) + SA(0, 1) + SA(0, -1)) +
         o4_c2 * (SA(1, 1) + SA(-1, -1) + SA(-1, 1) + SA(1, -1)) +
         o4_c3 * SA(0, 0));
  }
  if (in(j, g.jcii1, g.jcii2) && in(i, g.icii1, g.icii2))
    ften = ften - d_one * xk *
        (z4_c1 * (SA(2, 0) + SA(-2, 0) + SA(0, 2) + SA(0, -2)) +
         z4_c2 * (SA(1, 0) + SA(-1, 0) + SA(0, 1) + SA(0, -1)) +
         z4_c3 * SA(0, 0));
  const double lap = z4_c1 * (SA(1, 0) + SA(-1, 0) + SA(0, 1) + SA(0, -1)) + z4_c2 * SA(0, 0);
  const int nb = (g.bl && j == g.jci1) + (g.br && j == g.jci2) + (g.bb && i == g.ici1) + (g.bt && i == g.ici2);
  for (int q = 0; q < nb; q++) ften = ften + d_one * xk * lap;
  return ften;
#undef SA
}

// time filters of t (RA), qv and qc (RAW), Main/mod_tendency.F90:422-427 (p* is constant):
// o1, o2: atm1, atm2 before the filter; v: the forecast (for qv, qc fixed where negative);
// n1, n2: atm1, atm2 after it
__device__ __forceinline__ void nh_ra_t(const Consts* c, double o1, double o2, double v, double& n1, double& n2) {
  const double d = c->gnu1 * (v + o2 - d_two * o1);
  n2 = o1 + d;
  n1 = v;
}
__device__ __forceinline__ void nh_raw_qv(const Consts* c, double o1, double o2, double v, double psa, double psb,
                                          double& n1, double& n2) {
  const double beta = 0.53;
  const double d = c->gnu1 * (v + o2 - d_two * o1);
  n2 = dmax(o1 + beta * d, MINQQ * psa);
  n1 = dmax(v + (beta - d_one) * d, MINQQ * psb);
}
__device__ __forceinline__ void nh_raw_qc(const Consts* c, double o1, double o2, double v, double& n1, double& n2) {
  const double beta = 0.53;
  const double d = c->gnu2 * (v + o2 - d_two * o1);
  double m = o1 + beta * d, q = v + (beta - d_one) * d;
  if (m < d_zero) m = d_zero;
  if (q < d_zero) q = d_zero;
  n2 = m;
  n1 = q;
}
// tfuse: the RAW filter of qv (n = 0) or qc (n = 1) at one point into the other parity
__device__ __forceinline__ void nh_filter_q_to(const Geom& g, const Consts* c, const NHFields& f, int n, int j, int i, int k,
                                               double v) {
  double n1, n2;
  if (n == 0)
    nh_raw_qv(c, F3(f.a1qv, j, i, k), F3(f.a2qv, j, i, k), v, F2(f.psa, j, i), F2(f.psb, j, i), n1, n2);
  else
    nh_raw_qc(c, F3(f.a1qc, j, i, k), F3(f.a2qc, j, i, k), v, n1, n2);
  F3(n ? f.b1qc : f.b1qv, j, i, k) = n1;
  F3(n ? f.b2qc : f.b2qv, j, i, k) = n2;
}
// ---------------------------------------------------------------------------------------
// The tendency chain of the NH core as two point kernels.  For each variable the reference
// accumulates pc_dynamic over several loop nests -- advection (hadv/vadv), curvature or the
// adiabatic terms, the boundary relaxation, the diffusion -- and then sums pc_total + pc_dynamic
// + pc_physic in the forecast (Main/mod_tendency.F90:1227-1680, 285-411).  Every one of those
// nests updates the element of its own point only, and reads fields the chain never writes,
// so one thread can run the whole chain for its point and level in the reference's order,
// holding the running tendency in a register: the values are those of the separate nests,
// and pc_dynamic never reaches memory.
//   k_nh_tend_c, cross points, k = 1..kz+1: w, pp, t (ithadv = 1), qv, qc and the forecast of
//     t and moisture (atmc), with the t/qv Rayleigh damping; the ring of the cross frame
//     passes atm2 moisture to the forecasts;
//   k_nh_tend_d, dot points, k = 1..kz: u, v.
// The total tendencies (pc_total) are init_tendencies' zero except where the iboudy = 4
// sponges set them (band points).  tten/qvten/qcten are stored only with diagnostics on
// (wdiag): the step itself reads the forecasts.  The chains of u, v, pp and w end with the
// Rayleigh damping and decoupling of raydamp (:466-499; they read atm2 u, v, pp, w, which the
// time filters in between do not change) and with sound's scaling by the acoustic step
// (Main/mod_sound.F90:229-245): those are the tendencies sound reads.
constexpr int TCJ = TC_J, TCI = TC_I, TCW = TCJ + 4, TCH = TCI + 4, TCT = TCJ * TCI;   // block, staged tile
constexpr int TC_NF = 5;
#ifndef TC_W
#define TC_W 1      // 6 or 8 waves/SIMD measured slower (4.73, 5.35 ms against 3.82)
#endif
#ifndef TC_UV
#define TC_UV 1
#endif
#ifndef TD_X
#define TD_X 1
#endif
// relaxation and physics-tendency terms of k_nh_tend_c and k_nh_tend_d (#undef after k_nh_tend_d)
#define FG(b0, bt, a, J, I) ((F3(b0, J, I, k) + xt * F3(bt, J, I, k)) - F3(a, J, I, k))
#define RELAX5(x, b0, bt, a) \
  x = nh_relax(x, xf, xg, FG(b0, bt, a, j, i), FG(b0, bt, a, j - 1, i), FG(b0, bt, a, j + 1, i), \
               FG(b0, bt, a, j, i - 1), FG(b0, bt, a, j, i + 1))
#define PHY(p) (f.p ? F3(f.p, j, i, k) : 0.0)
#if !NH_OTHER_KERNELS
template <bool QX>
__global__ __launch_bounds__(TCT, TC_W) void k_nh_tend_c(Geom g, const Consts* __restrict__ c,
                                                   const StepState* __restrict__ s, NHFields f, int wdiag,
                                                   int istep) {
  // the horizontal stencil operands of this level for the 32 x 8 block and a 2-point halo,
  // staged in LDS once: the diffusion fields (13-point).  Staging the advected fields or the
  // relaxation differences as well measured slower at C5 (3.36 ms diffusion only, 3.66 ms
  // with the advected fields, 4.27 ms with both: LDS occupancy costs more than the L1 loads)
  __shared__ double sT[TC_NF][TCH][TCW];
  const int j = g.j0 + TBX * TCJ + (int)threadIdx.x, i = g.i0 + TBY * TCI + (int)threadIdx.y, k = TBZ + 1;
  const int kz = c->kz;
  const double xt = s->xbctime + s->dt;
  const bool inframe = j < g.j0 + g.nj && i < g.i0 + g.ni;
#if TC_UV
  // TC_UV: atm1 u, v of levels k and k - 1 at the block's (32 + 1) x (8 + 1) dot points, staged
  // too: the four-point wind averages of start_advect and the adiabatic term read them at every
  // cross point of the block (the same values, so the same bits)
  __shared__ double sU[2][TCI + 1][TCJ + 1], sV[2][TCI + 1][TCJ + 1];
  {
    const int J0 = g.j0 + TBX * TCJ, I0 = g.i0 + TBY * TCI;
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    constexpr int ND = (TCJ + 1) * (TCI + 1), NSU = (ND + TCT - 1) / TCT;
    double vu[NSU][4];
#pragma unroll
    for (int n = 0; n < NSU; n++) {
      const int q = tid + n * TCT, jg = J0 + q % (TCJ + 1), ig = I0 + q / (TCJ + 1);
      const bool okq = q < ND && jg < g.j0 + g.nj && ig < g.i0 + g.ni;
      const int jr = okq ? jg : g.j0, ir = okq ? ig : g.i0;
      vu[n][0] = (okq && k <= kz) ? F3(f.a1u, jr, ir, k) : 0.0;
      vu[n][1] = (okq && k <= kz) ? F3(f.a1v, jr, ir, k) : 0.0;
      vu[n][2] = (okq && k >= 2 && k - 1 <= kz) ? F3(f.a1u, jr, ir, k - 1) : 0.0;
      vu[n][3] = (okq && k >= 2 && k - 1 <= kz) ? F3(f.a1v, jr, ir, k - 1) : 0.0;
    }
#pragma unroll
    for (int n = 0; n < NSU; n++) {
      const int q = tid + n * TCT, jj = q % (TCJ + 1), ii = q / (TCJ + 1);
      if (q < ND) {
        sU[0][ii][jj] = vu[n][0]; sV[0][ii][jj] = vu[n][1];
        sU[1][ii][jj] = vu[n][2]; sV[1][ii][jj] = vu[n][3];
      }
    }
  }
#define A1U(dj, di, kk) sU[(kk) == k ? 0 : 1][(int)threadIdx.y + (di)][(int)threadIdx.x + (dj)]
#define A1V(dj, di, kk) sV[(kk) == k ? 0 : 1][(int)threadIdx.y + (di)][(int)threadIdx.x + (dj)]
#else
#define A1U(dj, di, kk) F3(f.a1u, j + (dj), i + (di), kk)
#define A1V(dj, di, kk) F3(f.a1v, j + (dj), i + (di), kk)
#endif
  {
    const int J0 = g.j0 + TBX * TCJ - 2, I0 = g.i0 + TBY * TCI - 2;
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    constexpr int NS = (TCW * TCH + TCT - 1) / TCT;
    double va[NS][TC_NF];
    bool ok[NS];
#pragma unroll
    for (int n = 0; n < NS; n++) {
      const int q = tid + n * TCT, jg = J0 + q % TCW, ig = I0 + q / TCW;
      ok[n] = q < TCW * TCH && jg >= g.j0 && jg < g.j0 + g.nj && ig >= g.i0 && ig < g.i0 + g.ni;
      const int jr = ok[n] ? jg : g.j0, ir = ok[n] ? ig : g.i0;
      for (int m = 0; m < TC_NF; m++) va[n][m] = 0.0;
      const double rpb = F2(f.rpsb, jr, ir);             // mkslice's products (:163-183)
      va[n][4] = F3(f.a2w, jr, ir, k) * rpb;
      if (k <= kz) {
        va[n][0] = F3(f.a2t, jr, ir, k) * rpb; va[n][1] = dmax(F3(f.a2qv, jr, ir, k) * rpb, MINQQ);
        va[n][2] = dmax(F3(f.a2qc, jr, ir, k) * rpb, d_zero); va[n][3] = F3(f.a2pp, jr, ir, k) * rpb;
      }
    }
#pragma unroll
    for (int n = 0; n < NS; n++) {
      const int q = tid + n * TCT, jj = q % TCW, ii = q / TCW;
      if (q < TCW * TCH)
        for (int m = 0; m < TC_NF; m++) sT[m][ii][jj] = ok[n] ? va[n][m] : 0.0;
    }
    __syncthreads();
  }
  if (!inframe) return;
  const int tj = (int)threadIdx.x + 2, ti = (int)threadIdx.y + 2;
  const double dt = s->dt;
  if (!IN_CI(j, i)) {
    if (k <= kz && IN_CE(j, i)) {
      F3(f.cqv, j, i, k) = F3(f.a2qv, j, i, k);
      F3(f.cqc, j, i, k) = F3(f.a2qc, j, i, k);
    }
    if (f.tfuse && k <= kz) {     // no filter here: the other parity keeps the values
      F3(f.b1t, j, i, k) = F3(f.a1t, j, i, k); F3(f.b2t, j, i, k) = F3(f.a2t, j, i, k);
      F3(f.b1qv, j, i, k) = F3(f.a1qv, j, i, k); F3(f.b2qv, j, i, k) = F3(f.a2qv, j, i, k);
      F3(f.b1qc, j, i, k) = F3(f.a1qc, j, i, k); F3(f.b2qc, j, i, k) = F3(f.a2qc, j, i, k);
    }
    return;
  }
  const double xmf = F2(f.xmsf, j, i), ps = F2(f.psa, j, i), ul = c->ul, pbs = F2(f.psb, j, i);
  const double m00 = F2(f.msfd, j, i), m01 = F2(f.msfd, j, i + 1), m10 = F2(f.msfd, j + 1, i),
               m11 = F2(f.msfd, j + 1, i + 1);
  // atmx of decouple (:852-1066) formed here: xw, xpp = atm1 w, pp * (1/p*), xqv, xqc the same
  // clipped at minqq / 0, at the point and its four neighbours (the 1/p* values of the five)
  const double r0 = F2(f.rpsa, j, i), rw = F2(f.rpsa, j - 1, i), re = F2(f.rpsa, j + 1, i),
               rs = F2(f.rpsa, j, i - 1), rn = F2(f.rpsa, j, i + 1);
  auto hadx = [&](const double* a, int clip, double u1, double u2, double v1, double v2, int lim) {
    double x[5] = {F3(a, j, i, k) * r0, F3(a, j - 1, i, k) * rw, F3(a, j + 1, i, k) * re, F3(a, j, i - 1, k) * rs,
                   F3(a, j, i + 1, k) * rn};
    if (clip)
      for (int q = 0; q < 5; q++) x[q] = dmax(x[q], clip == 1 ? MINQQ : d_zero);
    return hadv_v(c, x[0], x[1], x[2], x[3], x[4], u1, u2, v1, v2, xmf, ps, lim);
  };
  auto xqcat = [&](int kk) { return dmax(F3(f.a1qc, j, i, kk) * r0, d_zero); };
  // the water load qcd: qc, or with nqx = 5 the sum over iqfrst..iqlst (decouple, :1107-1115)
  auto xqload = [&](int kk) {
    if constexpr (QX) {
      double w = d_zero + xqcat(kk);
      for (int n = 0; n < NQXH; n++) w = w + dmax(F3(f.qxa1[n], j, i, kk) * r0, d_zero);
      return w;
    } else {
      return xqcat(kk);
    }
  };
  auto avg = [&](int kk, double& u1, double& u2, double& v1, double& v2) {   // start_advect :114-119
    u1 = A1U(0, 1, kk) * m01 + A1U(0, 0, kk) * m00;                         // umc = atm1 u * msfd
    u2 = A1U(1, 1, kk) * m11 + A1U(1, 0, kk) * m10;
    v1 = A1V(1, 0, kk) * m10 + A1V(0, 0, kk) * m00;
    v2 = A1V(1, 1, kk) * m11 + A1V(0, 1, kk) * m01;
  };
  // boundary relaxation (:1462-1501, Main/mod_bdycod.F90): nudging coefficients of the band
  const bool band = f.rgcr[g.ix(j, i)] > 0;
  const bool sponge = band && c->iboudy == 4;
  const bool nudge = band && c->iboudy != 4;
  const double dts = s->dt / (double)istep;
  const int kc = (k < kz) ? k : kz;
  double xf = d_zero, xg = d_zero, wsp = d_zero;
  if (band) {
    const int ib = f.ibcr[g.ix(j, i)];
    if (c->iboudy == 4) wsp = c->wgtx[ib];
    else if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; }
    else { xf = c->hefc[ib][kc]; xg = c->hegc[ib][kc]; }
  }
  // ================= w on full levels k = 1..kz+1
  {
    double wd = d_zero;
    if (k >= 2 && k <= kz) {                       // hadv3d ind = 1, Main/mod_advection.F90:486-507
      double u1, u2, v1, v2, pu1, pu2, pv1, pv2;
      avg(k, u1, u2, v1, v2);
      avg(k - 1, pu1, pu2, pv1, pv2);
      const double t1 = c->twt1[k], t2 = c->twt2[k];
      const double uaz1 = (t1 * u1 + t2 * pu1), uaz2 = (t1 * u2 + t2 * pu2);
      const double vaz1 = (t1 * v1 + t2 * pv1), vaz2 = (t1 * v2 + t2 * pv2);
      const double f1 = d_half * ul * (u2 + u1) / ps;
      const double f2 = d_half * ul * (v2 + v1) / ps;
      const double wc = F3(f.a1w, j, i, k) * r0, ww = F3(f.a1w, j - 1, i, k) * rw, we = F3(f.a1w, j + 1, i, k) * re;
      const double ws = F3(f.a1w, j, i - 1, k) * rs, wn = F3(f.a1w, j, i + 1, k) * rn;     // xw
      const double fx1 = (d_one + f1) * ww + (d_one - f1) * wc;
      const double fx2 = (d_one + f1) * wc + (d_one - f1) * we;
      const double fy1 = (d_one + f2) * ws + (d_one - f2) * wc;
      const double fy2 = (d_one + f2) * wc + (d_one - f2) * wn;
      wd = wd - xmf * (uaz2 * fx2 - uaz1 * fx1 + vaz2 * fy2 - vaz1 * fy1);
    }
    // vadv3d ind = 0, nk = kz+1 (w), :756-765: flux through the interface below level kk
    auto wflux = [&](int kk) {
      const double qq = d_half * (F3(f.qdot, j, i, kk) + F3(f.qdot, j, i, kk + 1));
      return qq * ((F3(f.a1w, j, i, kk) + F3(f.a1w, j, i, kk + 1)));
    };
    if (k >= 2) wd = wd + wflux(k - 1) * c->dds[k];
    if (k <= kz) wd = wd - wflux(k) * c->dds[k];
    if (k >= 2 && k <= kz) {                       // adiabatic NH, Main/mod_tendency.F90:1601-1671
      auto ucc = [&](int kk) { return A1U(0, 0, kk) + A1U(0, 1, kk) + A1U(1, 0, kk) + A1U(1, 1, kk); };
      auto vcc = [&](int kk) { return A1V(0, 0, kk) + A1V(0, 1, kk) + A1V(1, 0, kk) + A1V(1, 1, kk); };
      const double uk = ucc(k), vk = vcc(k), um = ucc(k - 1), vm = vcc(k - 1);
      const double rps = r0;
      const double ex = F2(f.ex, j, i), crx = F2(f.crx, j, i), cry = F2(f.cry, j, i);
      const double rofac = (c->dsigma[k - 1] * F3(f.rho0, j, i, k) + c->dsigma[k] * F3(f.rho0, j, i, k - 1)) /
                           (c->dsigma[k - 1] * F3(f.rho1, j, i, k) + c->dsigma[k] * F3(f.rho1, j, i, k - 1));
      const double uaq = d_rfour * (c->twt1[k] * uk + c->twt2[k] * um);
      const double vaq = d_rfour * (c->twt1[k] * vk + c->twt2[k] * vm);
#if NH_XPRFORM
      // decouple's atmx%pr (:1040-1048) at k and k-1, formed here as decouple formed it
      auto xprat = [&](int kk) {
        const double xt = F3(f.a1t, j, i, kk) * r0;
        const double xqv = dmax(F3(f.a1qv, j, i, kk) * r0, MINQQ);
        const double xtv = xt * (d_one + c->ep1 * xqv);
        const double xpp = F3(f.a1pp, j, i, kk) * r0;
        return (xtv - F3(f.t0, j, i, kk) - xpp / (c->cpd * F3(f.rho0, j, i, kk))) / xt;
      };
      const double xprm = xprat(k - 1), xprk = xprat(k);
#else
      const double xprm = F3(f.xpr, j, i, k - 1), xprk = F3(f.xpr, j, i, k);
#endif
      wd = wd +
          (c->twt2[k] * xprm + c->twt1[k] * xprk) * rofac * EGRAV_NH * ps +
          ex * (uaq * crx - vaq * cry) + (uaq * uaq + vaq * vaq) * REARTHRAD * rps +
          (F3(f.a1w, j, i, k) * r0) * (c->twt1[k] * F3(f.cr, j, i, k) + c->twt2[k] * F3(f.cr, j, i, k - 1));
      wd = wd - EGRAV_NH * ps * (c->twt2[k] * xqload(k - 1) + c->twt1[k] * xqload(k));
    }
    double wt0 = d_zero;
    if (sponge) wt0 = wsp * d_zero + (d_one - wsp) * F3(f.wwbt, j, i, k);
    if (nudge) RELAX5(wd, f.wwb0, f.wwbt, f.a2w);
    wd = c->idiffu == 3 ? diff6_add(g, wd, f.d6w, g.jci2, j, i, k)
                        : diffx_l(g, c, wd, sT[4], F3(f.xkcr, j, i, (k == 1) ? 1 : k - 1) * c->rdxsq * pbs, j, i, ti, tj);   // xkcf
    double wt = wt0 + wd + PHY(wphy);
    // raydamp3f and decoupling before sound (:466-499), sound's acoustic-step scaling (:229-245)
    if (c->ifrayd == 1 && k <= c->rayndamp)
      wt = wt + nh_tau(c, F3(f.zf0, j, i, k), F3(f.zf0, j, i, 1)) * (d_zero - F3(f.a2w, j, i, k));
    F3(f.wten, j, i, k) = (wt * F2(f.rpsa, j, i)) * dts;
  }
  if (k > kz) return;
  const double xkc = F3(f.xkcr, j, i, k) * c->rdxsq * pbs;      // calc_coeff's xkc
  double u1, u2, v1, v2;
  avg(k, u1, u2, v1, v2);
  const double cr = F3(f.cr, j, i, k);
  // ================= pp: hadv3d ind 0, vadv3d ind = 0 (nk = kz), adiabatic, boundary, diffusion
  {
    double pd = d_zero + hadx(f.a1pp, 0, u1, u2, v1, v2, 0);
    auto pflux = [&](int kk) {
      return F3(f.qdot, j, i, kk) * (c->twt1[kk] * F3(f.a1pp, j, i, kk) + c->twt2[kk] * F3(f.a1pp, j, i, kk - 1));
    };
    if (k >= 2) pd = pd + pflux(k) * c->xds[k];
    if (k + 1 <= kz) pd = pd - pflux(k + 1) * c->xds[k];
    pd = pd + (F3(f.a1pp, j, i, k) * r0) * cr;
    double pt0 = d_zero;
    if (sponge) pt0 = wsp * d_zero + (d_one - wsp) * F3(f.ppbt, j, i, k);
    if (nudge) RELAX5(pd, f.ppb0, f.ppbt, f.a2pp);
    pd = c->idiffu == 3 ? diff6_add(g, pd, f.d6pp, g.jci2, j, i, k) : diffx_l(g, c, pd, sT[3], xkc, j, i, ti, tj);
    double pt = pt0 + pd + PHY(ppphy);
    if (c->ifrayd == 1 && k <= c->rayndamp)       // raydamp3 (CRM: raydamp3f toward 0, :468-470),
      pt = pt + nh_tau(c, F3(f.z0, j, i, k), F3(f.z0, j, i, 1)) *  // decoupling, acoustic-step scaling
                    ((c->crm ? d_zero : F3(f.ppb0, j, i, k) + xt * F3(f.ppbt, j, i, k)) - F3(f.a2pp, j, i, k));
    F3(f.ppten, j, i, k) = (pt * F2(f.rpsa, j, i)) * dts;
  }
  const bool ray = c->ifrayd == 1 && k <= c->rayndamp && !c->crm;   // no t/qv damping in CRM mode (:359)
  const double tau = ray ? nh_tau(c, F3(f.z0, j, i, k), F3(f.z0, j, i, 1)) : d_zero;
  // ================= t, ithadv = 1 (:1347-1356, 1594-1600): thten = hadvt of th, then vadv3d
  // ind = 0 (nk = kz) of tha = th*p*, plus th*cr; tdyn = atm1%t*thten/tha
  {
    double thd = d_zero + hadv_v(c, F3(f.th, j, i, k), F3(f.th, j - 1, i, k), F3(f.th, j + 1, i, k),
                                 F3(f.th, j, i - 1, k), F3(f.th, j, i + 1, k), u1, u2, v1, v2, xmf, ps, 1);
    auto thflux = [&](int kk) {
      return F3(f.qdot, j, i, kk) *
             (c->twt1[kk] * (F3(f.th, j, i, kk) * ps) + c->twt2[kk] * (F3(f.th, j, i, kk - 1) * ps));
    };
    if (k >= 2) thd = thd + thflux(k) * c->xds[k];
    if (k + 1 <= kz) thd = thd - thflux(k + 1) * c->xds[k];
    const double th = F3(f.th, j, i, k);
    thd = thd + th * cr;
    double td = d_zero + F3(f.a1t, j, i, k) * thd / (th * ps);
    double tt0 = d_zero;
    if (sponge) tt0 = wsp * d_zero + (d_one - wsp) * F3(f.tbt, j, i, k);
    if (nudge) RELAX5(td, f.tb0, f.tbt, f.a2t);
    td = c->idiffu == 3 ? diff6_add(g, td, f.d6t, g.jci2, j, i, k) : diffx_l(g, c, td, sT[0], xkc, j, i, ti, tj);
    double tt = tt0 + td + PHY(tphy);
    tt = tt + 0.0;
    if (ray) tt = tt + tau * ((F3(f.tb0, j, i, k) + xt * F3(f.tbt, j, i, k)) - F3(f.a2t, j, i, k));
    if (wdiag) F3(f.tten, j, i, k) = tt;
    const double o2 = F3(f.a2t, j, i, k), ctv = o2 + dt * tt;
    if (f.tfuse) nh_ra_t(c, F3(f.a1t, j, i, k), o2, ctv, F3(f.b1t, j, i, k), F3(f.b2t, j, i, k));
    else F3(f.ct, j, i, k) = ctv;
  }
  // ================= qv: hadvqv (or the semi-Lagrangian start), vadvqv, adiabatic, boundary,
  // diffusion, forecast
  {
    double qd = d_zero + (c->isladvec ? F3(f.slqv, j, i, k)
                                      : hadx(f.a1qv, 1, u1, u2, v1, v2, 2));
    const double thr = MINQQ * ps;
    auto qflux = [&](int kk) {
      const double fk = F3(f.a1qv, j, i, kk), fkm = F3(f.a1qv, j, i, kk - 1);
      double fg = d_zero;
      if (fk > thr && fkm > thr) fg = fk * rcm_powpos(fkm / fk, c->qcon[kk]);
      return F3(f.qdot, j, i, kk) * fg;
    };
    if (k >= 2) qd = qd + qflux(k) * c->xds[k];
    if (k + 1 <= kz) qd = qd - qflux(k + 1) * c->xds[k];
    qd = qd + dmax(F3(f.a1qv, j, i, k) * r0, MINQQ) * cr;
    double qt0 = d_zero;
    if (sponge) qt0 = wsp * d_zero + (d_one - wsp) * F3(f.qbt, j, i, k);
    if (nudge) {
      const double nfac = 1.0e3, rfac = d_one / nfac;
#define FQ(J, I) (nfac * (F3(f.qb0, J, I, k) + xt * F3(f.qbt, J, I, k)) - nfac * F3(f.a2qv, J, I, k))
      const double q0 = FQ(j, i), q1 = FQ(j - 1, i), q2 = FQ(j + 1, i), q3 = FQ(j, i - 1), q4 = FQ(j, i + 1);
#undef FQ
      qd = qd + rfac * (xf * q0 - xg * (q1 + q2 + q3 + q4 - d_four * q0));
    }
    qd = c->idiffu == 3 ? diff6_add(g, qd, f.d6qv, g.jci2, j, i, k) : diffx_l(g, c, qd, sT[1], xkc, j, i, ti, tj);
    double qv = qt0 + qd + PHY(qvphy);
    qv = qv + 0.0;
    if (ray) qv = qv + tau * ((F3(f.qb0, j, i, k) + xt * F3(f.qbt, j, i, k)) - F3(f.a2qv, j, i, k));
    if (wdiag) F3(f.qvten, j, i, k) = qv;
    const double o2 = F3(f.a2qv, j, i, k), cq = o2 + dt * qv;
    F3(f.cqv, j, i, k) = cq;
    if (f.tfuse && !(cq < d_zero))      // a negative forecast: filtered after its fix
      nh_raw_qv(c, F3(f.a1qv, j, i, k), o2, cq, ps, pbs, F3(f.b1qv, j, i, k), F3(f.b2qv, j, i, k));
#if NH_NEGLIST
    if (cq < d_zero) f.neglist[atomicAdd(f.negcnt, 1)] = (unsigned)(((long)(k - 1) * g.plane + g.ix(j, i)) * 2);
#endif
  }
  // ================= qc: hadvqx (or the semi-Lagrangian start), vadv4d ind = 1, adiabatic,
  // diffusion, forecast
  {
    double cd = d_zero + (c->isladvec ? F3(f.slqc, j, i, k)
                                      : hadx(f.a1qc, 2, u1, u2, v1, v2, 0));
    const double thr = MINQQ * MINQQ * ps;
    const int kpb = f.kpbl ? (int)F2(f.kpbl, j, i) : 0;
    auto cflux = [&](int kk) {
      const double svv = F3(f.qdot, j, i, kk);
      const double fk = F3(f.a1qc, j, i, kk), fkm = F3(f.a1qc, j, i, kk - 1);
      // vadv4d ind = 3 (iuwvadv = 1): no threshold, the PBL-top rule at kpbl
      if (f.kpbl) return uw_fg(c, kk, kpb, fk, fkm, [&](int q) { return F3(f.a1qc, j, i, q); }) * svv;
      if (svv > d_zero) return (fkm > thr) ? svv * (c->twt1[kk] * fk + c->twt2[kk] * fkm) : d_zero;
      return (fk > thr) ? svv * (c->twt1[kk] * fk + c->twt2[kk] * fkm) : d_zero;
    };
    if (k >= 2) cd = cd + cflux(k) * c->xds[k];
    if (k + 1 <= kz) cd = cd - cflux(k + 1) * c->xds[k];
    cd = cd + xqcat(k) * cr;
    cd = c->idiffu == 3 ? diff6_add(g, cd, f.d6qc, g.jci2, j, i, k) : diffx_l(g, c, cd, sT[2], xkc, j, i, ti, tj);
    double qc = d_zero + cd + PHY(qcphy);
    qc = qc + 0.0;
    if (wdiag) F3(f.qcten, j, i, k) = qc;
    const double o2 = F3(f.a2qc, j, i, k), cq = o2 + dt * qc;
    F3(f.cqc, j, i, k) = cq;
    if (f.tfuse && !(cq < d_zero))
      nh_raw_qc(c, F3(f.a1qc, j, i, k), o2, cq, F3(f.b1qc, j, i, k), F3(f.b2qc, j, i, k));
#if NH_NEGLIST
    if (cq < d_zero) f.neglist[atomicAdd(f.negcnt, 1)] = (unsigned)(((long)(k - 1) * g.plane + g.ix(j, i)) * 2 + 1);
#endif
  }
}

#undef A1U
#undef A1V
template __global__ void k_nh_tend_c<false>(Geom, const Consts* __restrict__, const StepState* __restrict__, NHFields,
                                             int, int);
template __global__ void k_nh_tend_c<true>(Geom, const Consts* __restrict__, const StepState* __restrict__, NHFields,
                                            int, int);
#endif
#if NH_OTHER_KERNELS

// k_nh_tend_d stages its horizontal stencil operands of one level for a 64 x 4 block plus a
// 2-point halo in LDS, one load (and for ubd/msfd, vbd/msfd one division) per staged point:
// umc, vmc, ud, vd, cr (hadvuv) and the diffu_d operands; lanes outside the frame stage zero
constexpr int TDW = 64 + 4, TDH = TD_I + 4, TDT = 64 * TD_I;
__global__ __launch_bounds__(TDT) void k_nh_tend_d(Geom g, const Consts* __restrict__ c,
                                                   const StepState* __restrict__ s, NHFields f, int istep) {
  __shared__ double sUA[TDH][TDW], sVA[TDH][TDW], sU[TDH][TDW], sV[TDH][TDW], sCR[TDH][TDW];
  __shared__ double sBU[TDH][TDW], sBV[TDH][TDW];
  const int j = g.jdi1 + TBX * 64 + (int)threadIdx.x, i = g.idi1 + TBY * TD_I + (int)threadIdx.y, k = TBZ + 1;
#if TD_X
  // TD_X: the cross fields a dot point averages over its four cross points -- qdot at k and
  // k + 1 (vadvuv), atm1 w at k and k + 1 (the curvature terms) and xkcr at k (calc_coeff's xkd)
  // -- at the block's 65 x (TD_I + 1) cross points (j - 1 .. j + 63, i - 1 .. i + TD_I - 1)
  __shared__ double sQD[2][TD_I + 1][65], sWD[2][TD_I + 1][65], sXK[TD_I + 1][65];
  {
    const int J0 = g.jdi1 + TBX * 64 - 1, I0 = g.idi1 + TBY * TD_I - 1;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    constexpr int NC = 65 * (TD_I + 1), NSC = (NC + TDT - 1) / TDT;
    double vc[NSC][5];
#pragma unroll
    for (int n = 0; n < NSC; n++) {
      const int q = tid + n * TDT, jg = J0 + q % 65, ig = I0 + q / 65;
      const bool okq = q < NC && jg >= g.j0 && jg < g.j0 + g.nj && ig >= g.i0 && ig < g.i0 + g.ni;
      const int jr = okq ? jg : j0c(g), ir = okq ? ig : i0c(g);
      vc[n][0] = okq ? F3(f.qdot, jr, ir, k) : 0.0;
      vc[n][1] = okq ? F3(f.qdot, jr, ir, k + 1) : 0.0;
      vc[n][2] = okq ? F3(f.a1w, jr, ir, k) : 0.0;
      vc[n][3] = okq ? F3(f.a1w, jr, ir, k + 1) : 0.0;
      vc[n][4] = okq ? F3(f.xkcr, jr, ir, k) : 0.0;
    }
#pragma unroll
    for (int n = 0; n < NSC; n++) {
      const int q = tid + n * TDT, jj = q % 65, ii = q / 65;
      if (q < NC) {
        sQD[0][ii][jj] = vc[n][0]; sQD[1][ii][jj] = vc[n][1];
        sWD[0][ii][jj] = vc[n][2]; sWD[1][ii][jj] = vc[n][3]; sXK[ii][jj] = vc[n][4];
      }
    }
  }
#define QDC(dj, di, kk) sQD[(kk) == k ? 0 : 1][(int)threadIdx.y + 1 + (di)][(int)threadIdx.x + 1 + (dj)]
#define WDC(dj, di, kk) sWD[(kk) == k ? 0 : 1][(int)threadIdx.y + 1 + (di)][(int)threadIdx.x + 1 + (dj)]
#define XKC(dj, di) sXK[(int)threadIdx.y + 1 + (di)][(int)threadIdx.x + 1 + (dj)]
#else
#define QDC(dj, di, kk) F3(f.qdot, j + (dj), i + (di), kk)
#define WDC(dj, di, kk) F3(f.a1w, j + (dj), i + (di), kk)
#define XKC(dj, di) F3(f.xkcr, j + (dj), i + (di), k)
#endif
  {
    const int J0 = g.jdi1 + TBX * 64 - 2, I0 = g.idi1 + TBY * TD_I - 2;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    constexpr int NS = (TDW * TDH + TDT - 1) / TDT;
    double va[NS][7];
    bool ok[NS];
#pragma unroll
    for (int n = 0; n < NS; n++) {
      const int q = tid + n * TDT, jg = J0 + q % TDW, ig = I0 + q / TDW;
      ok[n] = q < TDW * TDH && jg >= g.j0 && jg < g.j0 + g.nj && ig >= g.i0 && ig < g.i0 + g.ni;
      const int jr = ok[n] ? jg : j0c(g), ir = ok[n] ? ig : i0c(g);
      const double m = F2(f.msfd, jr, ir);
#if NH_UDFORM
      // ud, vd formed from the atm1 winds loaded for umc, vmc (decouple no longer stores them)
      const double au = F3(f.a1u, jr, ir, k), av = F3(f.a1v, jr, ir, k);
      va[n][0] = au * m; va[n][1] = av * m;                                     // umc, vmc
      const double2 d = udvd_nh_ld(g, c->iboudy, f, au, av, F2(f.rpsda, jr, ir), jr, ir, k);
      va[n][2] = d.x; va[n][3] = d.y; va[n][4] = F3(f.cr, jr, ir, k);
#else
      va[n][0] = F3(f.a1u, jr, ir, k) * m; va[n][1] = F3(f.a1v, jr, ir, k) * m;   // umc, vmc
      va[n][2] = F3(f.ud, jr, ir, k); va[n][3] = F3(f.vd, jr, ir, k); va[n][4] = F3(f.cr, jr, ir, k);
#endif
      va[n][5] = UBD(jr, ir, k); va[n][6] = VBD(jr, ir, k);
      va[n][5] = va[n][5] / m; va[n][6] = va[n][6] / m;     // UM of diffu_d, Main/mod_diffusion.F90:281-411
    }
#pragma unroll
    for (int n = 0; n < NS; n++) {
      const int q = tid + n * TDT, jj = q % TDW, ii = q / TDW;
      if (q < TDW * TDH) {
        const bool o = ok[n];
        sUA[ii][jj] = o ? va[n][0] : 0.0; sVA[ii][jj] = o ? va[n][1] : 0.0;
        sU[ii][jj] = o ? va[n][2] : 0.0; sV[ii][jj] = o ? va[n][3] : 0.0; sCR[ii][jj] = o ? va[n][4] : 0.0;
        sBU[ii][jj] = o ? va[n][5] : 0.0; sBV[ii][jj] = o ? va[n][6] : 0.0;
      }
    }
    __syncthreads();
  }
  if (!IN_DI(j, i)) return;
  const int kz = c->kz;
  const int tj = (int)threadIdx.x + 2, ti = (int)threadIdx.y + 2;
#define L2(S, dj, di) S[ti + (di)][tj + (dj)]
  double ud, vd;
  // hadvuv NH upstream branch, Main/mod_advection.F90:235-264
  {
    const double ul = c->ul, dm = F2(f.dmsf, j, i);
    const double divd = d_rfour * (L2(sCR, 0, 0) + L2(sCR, 0, -1) + L2(sCR, -1, 0) + L2(sCR, -1, -1));
    const double ucmona = L2(sUA, 0, 1) + d_two * L2(sUA, 0, 0) + L2(sUA, 0, -1);
    double ucmonb = L2(sUA, 1, 1) + d_two * L2(sUA, 1, 0) + L2(sUA, 1, -1);
    double ucmonc = L2(sUA, -1, 1) + d_two * L2(sUA, -1, 0) + L2(sUA, -1, -1);
    const double vcmona = L2(sVA, 1, 0) + d_two * L2(sVA, 0, 0) + L2(sVA, -1, 0);
    double vcmonb = L2(sVA, 1, 1) + d_two * L2(sVA, 0, 1) + L2(sVA, -1, 1);
    double vcmonc = L2(sVA, 1, -1) + d_two * L2(sVA, 0, -1) + L2(sVA, -1, -1);
    const double diag = divd - dm * ((ucmonb - ucmonc) + (vcmonb - vcmonc));
    const double u0 = L2(sU, 0, 0), ue = L2(sU, 1, 0), uw = L2(sU, -1, 0);
    const double un = L2(sU, 0, 1), us = L2(sU, 0, -1);
    const double v0 = L2(sV, 0, 0), ve = L2(sV, 1, 0), vw = L2(sV, -1, 0);
    const double vn = L2(sV, 0, 1), vs = L2(sV, 0, -1);
    const double ff1 = ul * (ue + u0), ff2 = ul * (uw + u0);
    const double ff3 = ul * (vn + v0), ff4 = ul * (vs + v0);
    ucmonb = (d_one + ff1) * ucmona + (d_one - ff1) * ucmonb;
    ucmonc = (d_one + ff2) * ucmonc + (d_one - ff2) * ucmona;
    vcmonb = (d_one + ff3) * vcmona + (d_one - ff3) * vcmonb;
    vcmonc = (d_one + ff4) * vcmonc + (d_one - ff4) * vcmona;
    ud = d_zero + u0 * diag - dm * (ue * ucmonb - uw * ucmonc + un * vcmonb - us * vcmonc);
    vd = d_zero + v0 * diag - dm * (ve * ucmonb - vw * ucmonc + vn * vcmonb - vs * vcmonc);
  }
  // vadvuv (:286-299): the flux through interface kk reaches level kk (added) and kk-1
  // (subtracted), in the reference's loop order
  {
    auto flux = [&](int kk, double& uu, double& vv) {
      const double qq = d_rfour * (QDC(0, 0, kk) + QDC(0, -1, kk) + QDC(-1, 0, kk) + QDC(-1, -1, kk));
      uu = qq * (c->twt1[kk] * F3(f.a1u, j, i, kk) + c->twt2[kk] * F3(f.a1u, j, i, kk - 1));
      vv = qq * (c->twt1[kk] * F3(f.a1v, j, i, kk) + c->twt2[kk] * F3(f.a1v, j, i, kk - 1));
    };
    double uu, vv;
    if (k >= 2) {
      flux(k, uu, vv);
      ud = ud + uu * c->xds[k];
      vd = vd + vv * c->xds[k];
    }
    if (k + 1 <= kz) {
      flux(k + 1, uu, vv);
      ud = ud - uu * c->xds[k];
      vd = vd - vv * c->xds[k];
    }
  }
  // curvature NH (:1839-1879): horizontal and vertical Coriolis, horizontal and vertical curvature
  {
    const double wadot = 0.125 * (WDC(-1, -1, k) + WDC(-1, 0, k) + WDC(0, -1, k) + WDC(0, 0, k));
    const double wadotp1 = 0.125 * (WDC(-1, -1, k + 1) + WDC(-1, 0, k + 1) + WDC(0, -1, k + 1) + WDC(0, 0, k + 1));
    const double wabar = wadot + wadotp1;
    const double amfac = wabar * F2(f.rpsda, j, i) * REARTHRAD;
    const double uc = F3(f.a1u, j, i, k), vc = F3(f.a1v, j, i, k);
    const double duv = uc * F2(f.dmdy, j, i) - vc * F2(f.dmdx, j, i);
    const double cor = F2(f.coriol, j, i), ef = F2(f.ef, j, i);
    const double msd = F2(f.msfd, j, i);              // umd, vmd = ud, vd * msfd (decouple)
    ud = ud + cor * vc - ef * F2(f.ddx, j, i) * wabar + (L2(sV, 0, 0) * msd) * duv - uc * amfac;
    vd = vd - cor * uc + ef * F2(f.ddy, j, i) * wabar - (L2(sU, 0, 0) * msd) * duv - vc * amfac;
  }
  // boundary relaxation of u, v (nudgeuv) or the iboudy = 4 sponge of their total tendencies
  double ut0 = d_zero, vt0 = d_zero;
  if (f.rgdt[g.ix(j, i)] > 0) {
    const int ib = f.ibdt[g.ix(j, i)];
    if (c->iboudy == 4) {
      const double w = c->wgtd[ib];
      ut0 = w * d_zero + (d_one - w) * F3(f.ubt, j, i, k);
      vt0 = w * d_zero + (d_one - w) * F3(f.vbt, j, i, k);
    } else {
      const double xt = s->xbctime + s->dt;
      double xf, xg;
      if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; }
      else { xf = c->hefc[ib][k]; xg = c->hegc[ib][k]; }
      RELAX5(ud, f.ub0, f.ubt, f.a2u);
      RELAX5(vd, f.vb0, f.vbt, f.a2v);
    }
  }
  // diffu_d, Main/mod_diffusion.F90:281-411 (UM = ubd/msfd, vbd/msfd staged)
  {
#define UM(S, J, I) L2(S, (J) - j, (I) - i)
    const double xkd = d_rfour * (XKC(0, 0) + XKC(-1, -1) + XKC(-1, 0) + XKC(0, -1)) * c->rdxsq *
                       F2(f.psdotb, j, i);   // calc_coeff
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
      double (*b)[TDW] = pass ? sBV : sBU;
      double t = pass ? vd : ud;
      if (c->idiffu == 3) {                 // the column term of k_nh_diffu6
        t = diff6_add(g, t, pass ? f.d6v : f.d6u, g.jdi2, j, i, k);
      } else if (c->idiffu == 2) {
        t = t + xkd * (o4_c1 * (UM(b, j + 1, i) + UM(b, j - 1, i) + UM(b, j, i + 1) + UM(b, j, i - 1)) +
                       o4_c2 * (UM(b, j + 1, i + 1) + UM(b, j - 1, i - 1) + UM(b, j - 1, i + 1) + UM(b, j + 1, i - 1)) +
                       o4_c3 * (UM(b, j, i)));
      } else {
        if (in(j, g.jdii1, g.jdii2) && in(i, g.idii1, g.idii2))
          t = t - xkd * (z4_c1 * (UM(b, j + 2, i) + UM(b, j - 2, i) + UM(b, j, i + 2) + UM(b, j, i - 2)) +
                         z4_c2 * (UM(b, j + 1, i) + UM(b, j - 1, i) + UM(b, j, i + 1) + UM(b, j, i - 1)) +
                         z4_c3 * (UM(b, j, i)));
        const int nb = (g.bl && j == g.jdi1) + (g.br && j == g.jdi2) + (g.bb && i == g.idi1) + (g.bt && i == g.idi2);
        for (int q = 0; q < nb; q++)
          t = t + xkd * (z4_c1 * (UM(b, j + 1, i) + UM(b, j - 1, i) + UM(b, j, i + 1) + UM(b, j, i - 1)) +
                         z4_c2 * (UM(b, j, i)));
      }
      if (pass) vd = t; else ud = t;
    }
#undef UM
  }
#undef L2
  double ut = ut0 + ud + PHY(uphy);
  double vt = vt0 + vd + PHY(vphy);
  // Rayleigh damping and decoupling before sound (raydampuv, :466-499), then sound's scaling
  // by the acoustic step (Main/mod_sound.F90:229-236)
  if (c->ifrayd == 1 && k <= c->rayndamp) {
    const double xt = s->xbctime + s->dt;
    const double* z = f.z0;
    const double zz = d_rfour * (F3(z, j, i, k) + F3(z, j - 1, i, k) + F3(z, j, i - 1, k) + F3(z, j - 1, i - 1, k));
    const double zm = d_rfour * (F3(z, j, i, 1) + F3(z, j - 1, i, 1) + F3(z, j, i - 1, 1) + F3(z, j - 1, i - 1, 1));
    const double tau = nh_tau(c, zz, zm);
    // CRM: toward 0 (raydampuv_c with sval = d_zero, Main/mod_tendency.F90:467-469)
    ut = ut + tau * ((c->crm ? d_zero : F3(f.ub0, j, i, k) + xt * F3(f.ubt, j, i, k)) - F3(f.a2u, j, i, k));
    vt = vt + tau * ((c->crm ? d_zero : F3(f.vb0, j, i, k) + xt * F3(f.vbt, j, i, k)) - F3(f.a2v, j, i, k));
  }
  const double dts = s->dt / (double)istep;
  F3(f.uten, j, i, k) = (ut * F2(f.rpsda, j, i)) * dts;
  F3(f.vten, j, i, k) = (vt * F2(f.rpsda, j, i)) * dts;
}
#undef QDC
#undef WDC
#undef XKC
#undef PHY
#undef RELAX5
#undef FG

// negative-moisture fix (:382-393): see K6 in kernels.hip.  Parallel pass for the points
// whose sweep predecessors are non-negative, serial sweep of the flagged planes after it.
__device__ __forceinline__ double nh_negfix_sum(const Geom& g, const double* sv, const double* fx, int j, int i,
                                                int k, bool use_fixed) {
  double sum = 0.0;
  for (int ii = i - 1; ii <= i + 1; ii++)
    for (int jj = j - 1; jj <= j + 1; jj++) {
      double v = F3(sv, jj, ii, k);
      if (use_fixed) {
        const bool pred = (ii < i) || (ii == i && jj < j);
        if (pred && in(jj, g.jci1, g.jci2) && in(ii, g.ici1, g.ici2) && v < d_zero) v = F3(fx, jj, ii, k);
      }
      sum = sum + fabs(v);
    }
  return 0.01 * sum / 9.0;
}
// one negative forecast (species n) at an interior point: fixed in parallel when no sweep
// predecessor is negative, else its plane's row is marked for the serial sweep
__device__ __forceinline__ void nh_negfix_at(const Geom& g, const Consts* c, const NHFields& f, int n, int j, int i,
                                             int k) {
  const double* sv = n ? f.cqc : f.cqv;
  double* fx = n ? f.fqc : f.fqv;
  if (negfix_dependent(g, sv, j, i, k)) {
    negfix_mark(g, f.depplane, n * c->kz + (k - 1), i);
  } else {
    const double v = nh_negfix_sum(g, sv, fx, j, i, k, false);
    F3(fx, j, i, k) = v;
    if (f.tfuse) nh_filter_q_to(g, c, f, n, j, i, k, v);
  }
}
#if NH_NEGLIST
// NH_NEGLIST: the entries k_nh_tend_c listed, grid-stride (the list is unordered; every entry is
// an independent point, as in the point form below)
__global__ void k_nh_negfix(Geom g, const Consts* __restrict__ c, NHFields f) {
  const int cnt = *f.negcnt;
  for (int e = (int)(blockIdx.x * blockDim.x + threadIdx.x); e < cnt; e += (int)(gridDim.x * blockDim.x)) {
    const unsigned w = f.neglist[e];
    const int n = (int)(w & 1u);
    const long el = (long)(w >> 1);
    const int k = (int)(el / g.plane) + 1;
    const long r = el % g.plane;
    const int i = g.i0 + (int)(r / g.pitch), j = g.j0 + (int)(r % g.pitch);
    nh_negfix_at(g, c, f, n, j, i, k);
  }
}
#else
__global__ void k_nh_negfix(Geom g, const Consts* __restrict__ c, NHFields f) {
  WRAP_POINT(g.jci1, g.jci2, g.ici1);
  if (!IN_CI(j, i)) return;
  for (int n = 0; n < 2; n++)
    if (F3(n ? f.cqc : f.cqv, j, i, k) < d_zero) nh_negfix_at(g, c, f, n, j, i, k);
}
#endif

// one 64-lane block per (n, k) plane: the marked rows swept in the reference order
// (negfix_sweep, qxcommon.hpp; dynamic LDS negfix_lds(g))
// the filters of a fixed point (tfuse) from its atm1, atm2 (and p*a, p*b for qv) in x
struct NhQRaw {
  static constexpr int NI = 4;
  Geom g;
  const Consts* c;
  const double *a1, *a2, *psa, *psb;
  double *b1, *b2;
  int n, k, tfuse;
  __device__ void load(int j, int i, double* x) const {
    if (!tfuse) { x[0] = x[1] = x[2] = x[3] = 0.0; return; }
    x[0] = F3(a1, j, i, k); x[1] = F3(a2, j, i, k);
    x[2] = n == 0 ? F2(psa, j, i) : 0.0; x[3] = n == 0 ? F2(psb, j, i) : 0.0;
  }
  __device__ void apply(int j, int i, double v, const double* x) const {
    if (!tfuse) return;
    double n1, n2;
    if (n == 0) nh_raw_qv(c, x[0], x[1], v, x[2], x[3], n1, n2);
    else nh_raw_qc(c, x[0], x[1], v, n1, n2);
    F3(b1, j, i, k) = n1;
    F3(b2, j, i, k) = n2;
  }
};
__global__ __launch_bounds__(512) void k_nh_negfix_serial(Geom g, const Consts* __restrict__ c, NHFields f) {
  extern __shared__ double lds[];
  const int plane = blockIdx.x;
  const int kz = c->kz, n = plane / kz, k = plane % kz + 1;
  const NhQRaw acc{g, c, n ? f.a1qc : f.a1qv, n ? f.a2qc : f.a2qv, f.psa, f.psb, n ? f.b1qc : f.b1qv,
                   n ? f.b2qc : f.b2qv, n, k, f.tfuse};
  negfix_resolve(g, n ? f.cqc : f.cqv, n ? f.fqc : f.fqv, f.depplane, plane, k, lds, negfix_lds(g), acc,
                 [&](int jj, int i, double v) {
                   if (f.tfuse) nh_filter_q_to(g, c, f, n, jj, i, k, v);
                 }, c->negfix_mode);
}

// tfuse = 0: the three time filters in place at one interior cross point and level
__device__ __forceinline__ void nh_tfilter_at(const Geom& g, const Consts* c, const NHFields& f, int j, int i,
                                              int k) {
  nh_ra_t(c, F3(f.a1t, j, i, k), F3(f.a2t, j, i, k), F3(f.ct, j, i, k), F3(f.a1t, j, i, k), F3(f.a2t, j, i, k));
  {
    double v = F3(f.cqv, j, i, k);
    if (v < d_zero) v = F3(f.fqv, j, i, k);
    nh_raw_qv(c, F3(f.a1qv, j, i, k), F3(f.a2qv, j, i, k), v, F2(f.psa, j, i), F2(f.psb, j, i),
              F3(f.a1qv, j, i, k), F3(f.a2qv, j, i, k));
  }
  {
    double v = F3(f.cqc, j, i, k);
    if (v < d_zero) v = F3(f.fqc, j, i, k);
    nh_raw_qc(c, F3(f.a1qc, j, i, k), F3(f.a2qc, j, i, k), v, F3(f.a1qc, j, i, k), F3(f.a2qc, j, i, k));
  }
}

// ======================================================================= sound
// The initial arrays of the acoustic loop (Main/mod_sound.F90:217-228: atmc pp, w = atm2 *
// 1/psb on the cross frame, u, v = atm2 / psdotb on the dot frame) are formed by their first
// readers: part A of sub-step 1 (pp, w) and part B of sub-step 1 (u, v); the tendencies'
// scaling by the acoustic step (:229-245) ends the tendency kernels.

// part A of sub-step 1, one thread per cross point and level k = 1..kz+1: the loop's initial
// pp and w (:217-228, atm2 * 1/psb) and dp'/dp0 from that pp (:258-262)
__device__ __forceinline__ void nh_sound_a1_at(const Geom& g, const Consts* c, const NHFields& f, int j, int i,
                                               int k) {
  const int kz = c->kz;
  const double rpb = F2(f.rpsb, j, i);
  F3(f.cw, j, i, k) = F3(f.a2w, j, i, k) * rpb;
  if (k > kz) return;
  F3(f.cpp, j, i, k) = F3(f.a2pp, j, i, k) * rpb;
  const int kp1 = (kz < k + 1) ? kz : k + 1, km1 = (1 > k - 1) ? 1 : k - 1;
  F3(f.cdt, j, i, k) = (F3(f.a2pp, j, i, km1) * rpb - F3(f.a2pp, j, i, kp1) * rpb) /
                       (F3(f.pr0, j, i, km1) - F3(f.pr0, j, i, kp1));
}

// the filters of tend's end and part A of the first acoustic sub-step in one
// launch: independent point work over the cross frame, k = 1..kz+1
__global__ void k_nh_tfilter_a1(Geom g, const Consts* __restrict__ c, NHFields f) {
  THREAD_POINT(g.jce1, g.ice1);
  if (!IN_CE(j, i)) return;
  if (!f.tfuse && k <= c->kz && IN_CI(j, i)) nh_tfilter_at(g, c, f, j, i, k);
  nh_sound_a1_at(g, c, f, j, i, k);
}

// tfuse: the same part A as one column walk per cross frame column (k_nh_tfilter_a1 with tfuse
// does nothing else): each level's atm2 pp * (1/p*b) and atm0%pr are loaded once and carried to
// the levels above and below, where the point form reads them again from the k+-1 planes
// (the same products and differences, so the same bits)
__global__ void k_nh_a1_col(Geom g, const Consts* __restrict__ c, NHFields f) {
  WRAP_POINT(g.jce1, g.jce2, g.ice1);
  if (!IN_CE(j, i)) return;
  const int kz = c->kz;
  const double rpb = F2(f.rpsb, j, i);
  double pm = F3(f.a2pp, j, i, 1) * rpb, p0 = pm;          // pp at km1 = max(k-1, 1) and k
  double rm = F3(f.pr0, j, i, 1), r0 = rm;
#pragma unroll 4
  for (int kk = 1; kk <= kz; kk++) {
    const int kp1 = (kz < kk + 1) ? kz : kk + 1;
    const double pp = F3(f.a2pp, j, i, kp1) * rpb, rp = F3(f.pr0, j, i, kp1);
    F3(f.cw, j, i, kk) = F3(f.a2w, j, i, kk) * rpb;
    F3(f.cpp, j, i, kk) = p0;
    F3(f.cdt, j, i, kk) = (pm - pp) / (rm - rp);
    pm = p0; p0 = pp; rm = r0; r0 = rp;
  }
  F3(f.cw, j, i, kz + 1) = F3(f.a2w, j, i, kz + 1) * rpb;
}

// NH_DPRFORM: the acoustic u, v update forms dprddx / dprddy from atm0%pr; a host that puts
// them is checked once, after the put, to hold exactly those sums (Main/mod_params.F90:2676-2686)
// on the interior dot points the update reads (bad[0]: count of differing values)
__global__ void k_nh_check_dprd(Geom g, NHFields f, int* bad) {
  THREAD_POINT(g.jdi1, g.idi1);
  if (!IN_DI(j, i)) return;
  const double* pr = f.pr0;
  const double p00 = F3(pr, j, i, k), pm0 = F3(pr, j - 1, i, k), p0m = F3(pr, j, i - 1, k), pmm = F3(pr, j - 1, i - 1, k);
  const double dx = p00 - pm0 + p0m - pmm, dy = p00 - p0m + pm0 - pmm;
  const int n = (int)(__double_as_longlong(dx) != __double_as_longlong(F3(f.dprddx, j, i, k))) +
                (int)(__double_as_longlong(dy) != __double_as_longlong(F3(f.dprddy, j, i, k)));
  if (n) atomicAdd(bad, n);
}

// substep part B (:266-296): pressure-gradient update of u, v plus their tendencies
__device__ __forceinline__ void nh_sound_uv_at(const Geom& g, const Consts* __restrict__ c,
                                               const StepState* __restrict__ s, const NHFields& f, int istep,
                                               int fin, int first, int j, int i, int k) {
  // sub-step 1: the loop's initial u, v = atm2 / psdotb (:217-228), formed here; on the dot
  // frame's boundary ring they stay so for the whole loop
  auto init_u = [&](int jj, int ii) { return F3(f.a2u, jj, ii, k) / F2(f.psdotb, jj, ii); };
  auto init_v = [&](int jj, int ii) { return F3(f.a2v, jj, ii, k) / F2(f.psdotb, jj, ii); };
  if (!IN_DI(j, i)) {
    if (first && IN_DE(j, i)) {
      F3(f.cu, j, i, k) = init_u(j, i);
      F3(f.cv, j, i, k) = init_v(j, i);
    }
    return;
  }
  const double dts = s->dt / (double)istep;
  const double rho = d_rfour * (F3(f.rho1, j, i, k) + F3(f.rho1, j - 1, i, k) + F3(f.rho1, j, i - 1, k) +
                                F3(f.rho1, j - 1, i - 1, k));
  const double dppdp0 = d_rfour * (F3(f.cdt, j, i, k) + F3(f.cdt, j - 1, i, k) + F3(f.cdt, j, i - 1, k) +
                                   F3(f.cdt, j - 1, i - 1, k));
  const double chh = d_half * dts / (rho * c->dx) / F2(f.msfd, j, i);
  const double* pp = f.cpp;
#if NH_DPRFORM
  // atm0%dprddx / dprddy (Main/mod_params.F90:2678-2681), formed from atm0%pr as the reference
  // forms them once: the same four-point sums in the same order, so the same bits
  const double* pr = f.pr0;
  const double p00 = F3(pr, j, i, k), pm0 = F3(pr, j - 1, i, k), p0m = F3(pr, j, i - 1, k), pmm = F3(pr, j - 1, i - 1, k);
  const double dprx = p00 - pm0 + p0m - pmm, dpry = p00 - p0m + pm0 - pmm;
#else
  const double dprx = F3(f.dprddx, j, i, k), dpry = F3(f.dprddy, j, i, k);
#endif
  double u = (first ? init_u(j, i) : F3(f.cu, j, i, k)) - chh * (F3(pp, j, i, k) - F3(pp, j - 1, i, k) + F3(pp, j, i - 1, k) -
                                        F3(pp, j - 1, i - 1, k) - dprx * dppdp0);
  double v = (first ? init_v(j, i) : F3(f.cv, j, i, k)) - chh * (F3(pp, j, i, k) - F3(pp, j, i - 1, k) + F3(pp, j - 1, i, k) -
                                        F3(pp, j - 1, i - 1, k) - dpry * dppdp0);
  const double cu = u + F3(f.uten, j, i, k), cv = v + F3(f.vten, j, i, k);
  F3(f.cu, j, i, k) = cu;
  F3(f.cv, j, i, k) = cv;
  if (fin) {       // the last sub-step's u, v are final: the RA filters after the loop (:686-693)
    const double pd = F2(f.psdotb, j, i);
    const double uu = pd * cu, vv = pd * cv;
    double d = c->gnu1 * (uu + F3(f.a2u, j, i, k) - d_two * F3(f.a1u, j, i, k));
    F3(f.a2u, j, i, k) = F3(f.a1u, j, i, k) + d;
    F3(f.a1u, j, i, k) = uu;
    d = c->gnu1 * (vv + F3(f.a2v, j, i, k) - d_two * F3(f.a1v, j, i, k));
    F3(f.a2v, j, i, k) = F3(f.a1v, j, i, k) + d;
    F3(f.a1v, j, i, k) = vv;
  }
}

// Halo/compute overlap of the dp'/dp0, pp exchange: a dot point reads them at j-1 and i-1, so
// only the column j = jde1 and the row i = ide1 read ghost points (on sides with a neighbour).
// part 1 runs every other point while the exchange is in flight, part 2 that strip as a list
// (1-D blocks, blockIdx.y = level) after the join; part 0 every point.
__device__ __forceinline__ bool nh_uv_strip(const Geom& g, int j, int i) {
  return (!g.bl && j == g.jde1) || (!g.bb && i == g.ide1);
}
__global__ void k_nh_sound_uv(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f,
                              int istep, int fin, int first, int part) {
  if (part == 2) {
    const int ni = g.ide2 - g.ide1 + 1, nj = g.jde2 - g.jde1 + 1;
    const int ncol = g.bl ? 0 : ni, nrow = g.bb ? 0 : nj - (g.bl ? 0 : 1);
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x), k = (int)blockIdx.y + 1;
    if (q >= ncol + nrow) return;
    const int j = q < ncol ? g.jde1 : g.jde1 + (g.bl ? 0 : 1) + (q - ncol);
    const int i = q < ncol ? g.ide1 + q : g.ide1;
    nh_sound_uv_at(g, c, s, f, istep, fin, first, j, i, k);
    return;
  }
#if NH_WRAP_PT
  WRAP_POINT(g.jde1, g.jde2, g.ide1);
#else
  NH_SOUND_POINT(NH_ALIGN ? ALIGN_J(g.jde1) : g.jde1, g.ide1);
#endif
  if (part == 1 && nh_uv_strip(g, j, i)) return;
  nh_sound_uv_at(g, c, s, f, istep, fin, first, j, i, k);
}

// cu, cv at the dot points (j,i), (j+1,i), (j,i+1), (j+1,i+1) around a cross point, one level
struct NhQ { double u[4], v[4]; };
__device__ __forceinline__ NhQ nh_q_at(const Geom& g, const NHFields& f, int j, int i, int k) {
  NhQ q;
  q.u[0] = F3(f.cu, j, i, k); q.u[1] = F3(f.cu, j + 1, i, k); q.u[2] = F3(f.cu, j, i + 1, k); q.u[3] = F3(f.cu, j + 1, i + 1, k);
  q.v[0] = F3(f.cv, j, i, k); q.v[1] = F3(f.cv, j + 1, i, k); q.v[2] = F3(f.cv, j, i + 1, k); q.v[3] = F3(f.cv, j + 1, i + 1, k);
  return q;
}
struct NhB1 { double p, cc, cdd, cj, tk, ptend, rho0; };
// the level-parallel coefficients of level k (:297-399) from the column's rings: qm, q0, qp are
// cu/cv at km1 = k-1, k and kp1 = min(k+1, kz) (k = 1: levels 1 and 2 in q0, qp), pcm/pc/pcp
// pr0 of the column there; m[] msfd at the four dot points
__device__ __forceinline__ NhB1 nh_sound_b1_at(const Geom& g, const Consts* c, const NHFields& f, int j, int i,
                                               int k, int kz, int it, double dts, double msfx, double ps0,
                                               double rpb, const NhQ& qm, const NhQ& q0, const NhQ& qp,
                                               double pcm, double pc, double pcp, const double* m) {
  NhB1 r;
  const double xg = c->xgamma;
  const double* pr0 = f.pr0;
  r.p = F3(f.cpp, j, i, k);
  if (it > 1) r.p = r.p - c->nhxkd * F3(f.spi, j, i, k);
  const double pr1 = F3(f.pr1, j, i, k), rho0 = F3(f.rho0, j, i, k);
  r.rho0 = rho0;
  r.cc = xg * pr1 * dts / (c->dx * msfx);
  r.cdd = xg * pr1 * rho0 * EGRAV_NH * dts / (ps0 * c->dsigma[k]);
  r.cj = d_half * rho0 * EGRAV_NH * dts;
  r.tk = (d_half * ps0 * F3(f.t0, j, i, k)) / (xg * pc * F3(f.a2t, j, i, k) * rpb);
  double pxup, pyvp;
  if (k == 1) {
    pxup = 0.0625 * (F3(pr0, j + 1, i, 1) - F3(pr0, j - 1, i, 1)) *
        (q0.u[0] + q0.u[1] + q0.u[2] + q0.u[3] - qp.u[0] - qp.u[1] - qp.u[2] - qp.u[3]) / (pc - pcp);
    pyvp = 0.0625 * (F3(pr0, j, i + 1, 1) - F3(pr0, j, i - 1, 1)) *
        (q0.v[0] + q0.v[1] + q0.v[2] + q0.v[3] - qp.v[0] - qp.v[1] - qp.v[2] - qp.v[3]) / (pc - pcp);
  } else {
    pyvp = 0.125 * (F3(pr0, j, i + 1, k) - F3(pr0, j, i - 1, k)) *
        (qm.v[0] + qm.v[1] + qm.v[2] + qm.v[3] - qp.v[0] - qp.v[1] - qp.v[2] - qp.v[3]) / (pcm - pcp);
    pxup = 0.125 * (F3(pr0, j + 1, i, k) - F3(pr0, j - 1, i, k)) *
        (qm.u[0] + qm.u[1] + qm.u[2] + qm.u[3] - qp.u[0] - qp.u[1] - qp.u[2] - qp.u[3]) / (pcm - pcp);
    if (k == kz) { pyvp = pyvp * d_half; pxup = pxup * d_half; }
  }
  const double div = (q0.v[2] * m[2] - q0.v[0] * m[0] + q0.v[3] * m[3] - q0.v[1] * m[1] +
                      q0.u[1] * m[1] - q0.u[0] * m[0] + q0.u[3] * m[3] - q0.u[2] * m[2]) / msfx;
  r.ptend = F3(f.ppten, j, i, k) - d_half * r.cc * (div - d_two * (pyvp + pxup));
  return r;
}

// substep part C (:297-483) as one column kernel, one thread per interior cross column
// walking k = kz..1: the level-parallel coefficients of a level (undo of the divergence
// damping of pp, Ikawa cc/cdd/cj, the temperature factor tk, the horizontal pressure-advection
// terms and ptend, :297-399) are formed once, in registers, when the walk reaches the level,
// and feed the tridiagonal coefficients and right-hand side of the implicit w equation at the
// level below them (:400-457), the pp predictor (:458-464) and the sweep of the tridiagonal
// system (:468-476) in the same pass; the inputs of the upper radiative condition (:488-494)
// close the column.  cu/cv around the column and its pr0 are loaded once per level and kept
// in three-level rings.  Every value is the reference's expression; only se and sf (read by
// the downward sweep after the radiative condition's domain convolution) and the new pp, pi
// leave the column.
#ifndef NHBC_W
#define NHBC_W 2
#endif
__global__ __launch_bounds__(256, NHBC_W) void k_nh_sound_bc(Geom g, const Consts* __restrict__ c,
                                                             const StepState* __restrict__ s, NHFields f,
                                                             int istep, int it) {
#if NH_WRAP
  const int j = wrap_j(g, g.jci1, g.jci2 - g.jci1 + 1, (int)blockIdx.x, (int)threadIdx.x);
  const int i = g.ici1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
#else
  NH_SOUND_POINT(NH_ALIGN ? ALIGN_J(g.jci1) : g.jci1, g.ici1);
#endif
  if (!IN_CI(j, i)) return;
  const int kz = c->kz;
  const double dts = s->dt / (double)istep;
  const double msfx = F2(f.msfx, j, i), ps0 = F2(f.ps0, j, i), rpb = F2(f.rpsb, j, i);
  const double m[4] = {F2(f.msfd, j, i), F2(f.msfd, j + 1, i), F2(f.msfd, j, i + 1), F2(f.msfd, j + 1, i + 1)};
  const double bet = c->nhbet, bp = (d_one + bet) * d_half, bm = (d_one - bet) * d_half;
  const double bpxbp = bp * bp, bpxbm = bp * bm;
  const double* w = f.cw;                       // still the old w (wo) on levels 1..kz+1
  NhQ qb = nh_q_at(g, f, j, i, kz), qa = nh_q_at(g, f, j, i, kz - 1);   // levels kz, kz-1
  double pcb = F3(f.pr0, j, i, kz), pca = F3(f.pr0, j, i, kz - 1);
  // the sweep's start at the model top (:340-345)
  double e = d_zero;
  double ff = d_half * d_rfour * c->regrav *
      ((qb.v[2] + qb.v[0] + qb.v[3] + qb.v[1]) * (F2(f.ht, j, i + 1) - F2(f.ht, j, i - 1)) +
       (qb.u[2] + qb.u[0] + qb.u[3] + qb.u[1]) * (F2(f.ht, j + 1, i) - F2(f.ht, j - 1, i))) /
      (c->dx * msfx);
  F3(f.se, j, i, kz) = e;
  F3(f.sf, j, i, kz) = ff;
  NhB1 cur = nh_sound_b1_at(g, c, f, j, i, kz, kz, it, dts, msfx, ps0, rpb, qa, qb, qb, pca, pcb, pcb, m);
  double rho1k = F3(f.rho1, j, i, kz);
  double wk1 = F3(w, j, i, kz + 1), wk = F3(w, j, i, kz);
  double pnew = d_zero;
#if defined(NHBC_UNROLL) && NHBC_UNROLL == 2    // measured: no change at C5
#pragma unroll 2
#endif
  for (int k = kz; k >= 1; k--) {
    // rings: qb/pcb at k, qa/pca at k-1
    const double wkm = (k >= 2) ? F3(w, j, i, k - 1) : d_zero;
    NhB1 prv;
    double rho1m = d_zero;
    NhQ qc;
    double pcc = d_zero;
    if (k >= 2) {
      if (k >= 3) { qc = nh_q_at(g, f, j, i, k - 2); pcc = F3(f.pr0, j, i, k - 2); }
      else { qc = qa; pcc = pca; }                // unused by level 1's special form
      if (k - 1 == 1) prv = nh_sound_b1_at(g, c, f, j, i, 1, kz, it, dts, msfx, ps0, rpb, qa, qa, qb, pca, pca, pcb, m);
      else prv = nh_sound_b1_at(g, c, f, j, i, k - 1, kz, it, dts, msfx, ps0, rpb, qc, qa, qb, pcc, pca, pcb, m);
      rho1m = F3(f.rho1, j, i, k - 1);
      // tridiagonal coefficients and right-hand side at k (:400-457)
      const int km1 = k - 1;
      const double rofac = (c->dsigma[km1] * cur.rho0 + c->dsigma[k] * prv.rho0) /
                           (c->dsigma[km1] * rho1k + c->dsigma[k] * rho1m);
      const double ca = EGRAV_NH * dts / (pcb - pca) * rofac;
      const double g1 = d_one - c->dsigma[km1] * cur.tk;
      const double g2 = d_one + c->dsigma[k] * prv.tk;
      const double cdm = prv.cdd, cjm = prv.cj;
      const double cdk = cur.cdd, cjk = cur.cj;
      const double sc = -ca * (cdm - cjm) * g2 * bpxbp;
      const double sb = d_one + ca * (g1 * (cdk - cjk) + g2 * (cdm + cjm)) * bpxbp;
      const double saa = -ca * (cdk + cjk) * g1 * bpxbp;
      const double rhs = wk + F3(f.wten, j, i, k) + ca *
          (bpxbm * ((cdm - cjm) * g2 * wkm - ((cdm + cjm) * g2 + (cdk - cjk) * g1) * wk +
                    (cdk + cjk) * g1 * wk1) +
           (cur.p * g1 - prv.p * g2) +
           (g1 * cur.ptend - g2 * prv.ptend) * bp);
      // upward sweep (:468-476)
      const double denom = saa * e + sb;
      e = -sc / denom;
      ff = (rhs - ff * saa) / denom;
      F3(f.se, j, i, k - 1) = e;
      F3(f.sf, j, i, k - 1) = ff;
    }
    // pp predictor (:458-464)
    F3(f.spi, j, i, k) = cur.p;
    pnew = cur.p + cur.ptend + (cur.cj * (wk1 + wk) + cur.cdd * (wk1 - wk)) * bm;
    F3(f.cpp, j, i, k) = pnew;
    if (k >= 2) {
      cur = prv;
      rho1k = rho1m;
      wk1 = wk; wk = wkm;
      qb = qa; qa = qc; pcb = pca; pca = pcc;
    }
  }
  if (c->ifupr == 1) {          // cur: level 1; pnew: its predicted pp
    const double denom = (cur.cdd + cur.cj) * bp;
    F2(f.estore, j, i) = pnew + ff * denom;
    F2(f.astore, j, i) = denom * e + (cur.cj - cur.cdd) * bp;
  }
}

// upper radiative condition coefficients (:500-543), on the day alarm.  The domain means
// are sequential sums over the interior cross points in the reference's i-major order; each
// tile first scatters its points' terms into a global-indexed buffer (gbuf: astore, then
// rho*sqrt(N^2)), so every decomposition sums the same values in the same order.
__global__ void k_nh_tmask_gather(Geom g, const Consts* __restrict__ c, NHFields f, double* gbuf) {
  THREAD_POINT(g.jci1, g.ici1);
  if (!IN_CI(j, i)) return;
  const long q = (long)(i - 1) * g.gjx + (j - 1), n = (long)g.gjx * g.giy;
  const double ensq = EGRAV_NH * EGRAV_NH / c->cpd / (F3(f.a2t, j, i, 1) * F2(f.rpsb, j, i));
  gbuf[q] = F2(f.astore, j, i);
  gbuf[n + q] = F3(f.rho1, j, i, 1) * sqrt(ensq);
}

// The two sums stay sequential in the reference's order (one thread adds); the block stages
// the next TMC terms of both into LDS in parallel, so the adding thread reads LDS instead of
// waiting on one global load per term.
constexpr int TMC = 2048;
__global__ __launch_bounds__(256) void k_nh_tmask(Geom g, const Consts* __restrict__ c,
                                                  const double* __restrict__ gbuf, double* tmask) {
  __shared__ double sh[2];
  __shared__ double sA[TMC], sR[TMC];
  const long n = (long)g.gjx * g.giy;
  // the global interior cross points (j = 2..jx-2, i = 2..iy-2; every point of a periodic
  // direction: a band's j, CRM's i)
  const int j1 = g.gcj1(), i1 = g.gci1(), nj = g.gcj2() - j1 + 1, ni = g.gci2() - i1 + 1;
  const long total = (long)nj * ni;
  double atot = d_zero, rhontot = d_zero;
  for (long base = 0; base < total; base += TMC) {
    const int cnt = (int)((total - base) < TMC ? (total - base) : TMC);
    for (int t = threadIdx.x; t < cnt; t += blockDim.x) {
      const long p = base + t;                    // i-major, j-minor: the reference's loop order
      const int i = i1 + (int)(p / nj), j = j1 + (int)(p % nj);
      const long q = (long)(i - 1) * g.gjx + (j - 1);
      sA[t] = gbuf[q];
      sR[t] = gbuf[n + q];
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int t = 0; t < cnt; t++) { atot = atot + sA[t]; rhontot = rhontot + sR[t]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // init_sound's count, Main/mod_sound.F90:120: 1/((nicross-2)*(njcross-2)) (with CRM it
    // differs from the number of points summed, as in the reference)
    const double rnpts = d_one / (double)((g.nicross() - 2) * (g.njcross() - 2));
    sh[0] = atot * rnpts;
    sh[1] = rhontot * rnpts;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 169) return;
  const int jj = t / 13 - 6, ii = t % 13 - 6;       // tmask(jj, ii) stored at [jj+6][ii+6]
  const double abar = sh[0], rhon = sh[1];
  const double dxmsfb = d_two / c->dxsq / c->nh_xmsf;
  const double fi = (ii == -6 || ii == 6) ? d_half : d_one, fj = (jj == -6 || jj == 6) ? d_half : d_one;
  const double ri = (double)ii, rj = (double)jj;
  double acc = d_zero;
  for (int kk = 0; kk <= 6; kk++) {
    const double rkk = (double)kk, fk = (kk == 0 || kk == 6) ? d_one : d_two;
    for (int ll = 0; ll <= 6; ll++) {
      const double rll = (double)ll, fl = (ll == 0 || ll == 6) ? d_one : d_two;
      const double xkeff = dxmsfb * sin(MATHPI * rkk / 12.0) * cos(MATHPI * rll / 12.0);
      const double xleff = dxmsfb * sin(MATHPI * rll / 12.0) * cos(MATHPI * rkk / 12.0);
      const double xkleff = sqrt(xkeff * xkeff + xleff * xleff);
      acc = acc + (fi * fj * fk * fl) / 144.0 * cos(2.0 * MATHPI * rkk * ri / 12.0) *
                      cos(2.0 * MATHPI * rll * rj / 12.0) * xkleff / (rhon - abar * xkleff);
    }
  }
  tmask[t] = acc;
}

// substep part D (:488-685) as one kernel, 64 x 4 interior columns per block: the upper
// boundary value from the 13 x 13 convolution of estore (staged in LDS, clamped to the
// interior), then per column the downward sweep of w (:544-560) and, as each level's w(k+1)
// becomes known, the level's sigma-velocity CFL (:624-640), new pp (:661-674) and its
// temperature correction (:675-681); unless this is the last sub-step, part A of the next one
// (pp += xkd*pi and dp'/dp0, :250-262) follows on the column: the boundary ring's dp'/dp0 that
// part A also forms reads pp the sub-steps never change there, so it keeps its first-sub-step
// value.  The CFL maximum is reduced over the block (wavefront
// shuffles, one atomic per block; non-negative doubles order like their bit patterns and a NaN
// sorts above every finite value, raising the stop).
// estore is read from the frame ge (the tile frame, or on a decomposed domain the wide frame
// filled by a 6-deep exchange: the convolution reaches 6 points, clamped to the interior).
#ifdef NHCD_W
#define NHCD_LB __launch_bounds__(256, NHCD_W)
#else
#define NHCD_LB __launch_bounds__(256)
#endif
__global__ NHCD_LB void k_nh_sound_cd(Geom g, Geom ge, const double* __restrict__ est,
                                                     const Consts* __restrict__ c, const StepState* __restrict__ s,
                                                     NHFields f, int istep, int last, int nexta) {
  __shared__ double sE[4 + 12][64 + 12];
  __shared__ double sM[169];
  __shared__ unsigned long long sred[4];
  const int ilo = 2, ihi = g.nicross() - 1, jlo = 2, jhi = g.njcross() - 1;   // icross1+1 .. icross2-1
#if NH_XCD
  const Blk3 xb = xcd_block();
#else
  const Blk3 xb = {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
#endif
#if NH_WRAP
  // block column 0's lanes below jci1 take the row's tail columns (wrap_j): their 13 x 13
  // neighbourhoods come from a second staged tile, sT2, at the tail
  const int nci = g.jci2 - g.jci1 + 1, ja = g.jci1 - jalign(g, g.jci1);
  const int J0 = ja + xb.x * 64, JT = ja + ((nci + 63) / 64) * 64;
  __shared__ double sT2[4 + 12][16 + 12];
#else
  const int J0 = (NH_ALIGN_CD ? ALIGN_J(g.jci1) : g.jci1) + xb.x * 64;
#endif
  const int I0 = g.ici1 + xb.y * 4;
  const int tid = threadIdx.y * 64 + threadIdx.x;
  const bool upr = c->ifupr == 1;
  if (upr) {
    for (int q = tid; q < 16 * 76; q += 256) {
      const int jj = q % 76, ii = q / 76;
      int jn = J0 - 6 + jj, in_ = I0 - 6 + ii;
      jn = (jn < jlo) ? jlo : (jn > jhi ? jhi : jn);
      in_ = (in_ < ilo) ? ilo : (in_ > ihi ? ihi : in_);
      sE[ii][jj] = est[ge.ix(jn, in_)];
    }
#if NH_WRAP
    if (xb.x == 0 && J0 < g.jci1)
      for (int q = tid; q < 16 * 28; q += 256) {
        const int jj = q % 28, ii = q / 28;
        int jn = JT - 6 + jj, in_ = I0 - 6 + ii;
        jn = (jn < jlo) ? jlo : (jn > jhi ? jhi : jn);
        jn = (jn < ge.j0 + ge.nj) ? jn : ge.j0 + ge.nj - 1;     // an empty tail: stay in the frame
        in_ = (in_ < ilo) ? ilo : (in_ > ihi ? ihi : in_);
        sT2[ii][jj] = est[ge.ix(jn, in_)];
      }
#endif
    if (tid < 169) sM[tid] = f.tmask[tid];
    __syncthreads();
  }
#if NH_WRAP
  const bool tail = J0 + (int)threadIdx.x < g.jci1;
  const int j = tail ? JT + (J0 + (int)threadIdx.x - ja) : J0 + (int)threadIdx.x, i = I0 + (int)threadIdx.y;
  const double* tE = tail ? &sT2[0][0] : &sE[0][0];
  const int tW = tail ? 28 : 76, tJ = tail ? JT : J0;
#else
  const int j = J0 + (int)threadIdx.x, i = I0 + (int)threadIdx.y;
  const double* tE = &sE[0][0];
  const int tW = 76, tJ = J0;
#endif
  const bool active = IN_CI(j, i);
  unsigned long long cfl = 0ull;                       // bits of the column's CFL maximum
  if (active) {
    const int kz = c->kz;
    const double dt = s->dt, dts = dt / (double)istep;
    const double bp = (d_one + c->nhbet) * d_half;
    double wpval = d_zero;
    if (upr) {
      for (int nsi = -6; nsi <= 6; nsi++) {
        int inn = i + nsi; inn = (inn < ilo) ? ilo : (inn > ihi ? ihi : inn);
        for (int nsj = -6; nsj <= 6; nsj++) {
          int jnn = j + nsj; jnn = (jnn < jlo) ? jlo : (jnn > jhi ? jhi : jnn);
          wpval = wpval + tE[(inn - I0 + 6) * tW + (jnn - tJ + 6)] * sM[(nsj + 6) * 13 + (nsi + 6)];
        }
      }
    }
    double* w = f.cw;
    const double ps0 = F2(f.ps0, j, i), psb = F2(f.psb, j, i), rpsb = F2(f.rpsb, j, i);
    // last sub-step: the RA filters of pp and w after the loop (:694-702) follow on the column
    auto wfilt = [&](int kk, double wv) {
      if (!last) { F3(w, j, i, kk) = wv; return; }
      if (fabs(wv) < DLOWVAL) wv = d_zero;
      wv = psb * wv;
      const double d = c->gnu2 * (wv + F3(f.a2w, j, i, kk) - d_two * F3(f.a1w, j, i, kk));
      double a2 = F3(f.a1w, j, i, kk) + d, a1 = wv;
      F3(w, j, i, kk) = wv;
      if (fabs(a2) < DLOWVAL) a2 = d_zero;
      if (fabs(a1) < DLOWVAL) a1 = d_zero;
      F3(f.a2w, j, i, kk) = a2;
      F3(f.a1w, j, i, kk) = a1;
    };
    wfilt(1, wpval);
    const double dpx = F2(f.dpsdxm, j, i), dpy = F2(f.dpsdym, j, i);
    auto crs = [&](const double* a, int kk) {
      return F3(a, j, i, kk) + F3(a, j, i + 1, kk) + F3(a, j + 1, i, kk) + F3(a, j + 1, i + 1, kk);
    };
    double wm = wpval;
    double cum = d_zero, cvm = d_zero;          // crs(cu/cv, k-1)
    double pam = d_zero, pamm = d_zero, prm = d_zero, prmm = d_zero;   // next part A: pp, pr0 at k-1, k-2
#ifndef NHCD_UNROLL
#define NHCD_UNROLL 2      // two levels per iteration: 910 -> 861 us at C5 (A/B)
#endif
#if NHCD_UNROLL == 2
#pragma unroll 2
#endif
    for (int k = 1; k <= kz; k++) {
      const double wp = F3(f.se, j, i, k) * wm + F3(f.sf, j, i, k);
      wfilt(k + 1, wp);
      const double cuk = crs(f.cu, k), cvk = crs(f.cv, k);
      if (k >= 2) {
        const double sigdot = -F3(f.rhof0, j, i, k) * EGRAV_NH * wm / ps0 -
            c->sigma[k] * (dpx * (c->twt1[k] * cuk + c->twt2[k] * cum) +
                           dpy * (c->twt1[k] * cvk + c->twt2[k] * cvm));
        const unsigned long long b =
            (unsigned long long)__double_as_longlong(dmax(fabs(sigdot) * dt / (c->dsigma[k] + c->dsigma[k - 1]), d_zero));
        cfl = (b > cfl) ? b : cfl;
      }
      cum = cuk; cvm = cvk;
      const double ppold = F3(f.spi, j, i, k);
      const double rho0 = F3(f.rho0, j, i, k);
      const double cddtmp = c->xgamma * F3(f.pr1, j, i, k) * rho0 * EGRAV_NH * dts / (ps0 * c->dsigma[k]);
      const double cjtmp = rho0 * EGRAV_NH * dts * d_half;
      const double p = F3(f.cpp, j, i, k) + (cjtmp * (wp + wm) + cddtmp * (wp - wm)) * bp;
      const double spn = p - ppold - F3(f.ppten, j, i, k);
      F3(f.spi, j, i, k) = spn;
      const double cpm = c->cpd * (d_one + 0.80 * (F3(f.a2qv, j, i, k) * rpsb));   // qv = atm2 qv / p*b
      const double dpterm = psb * (p - ppold) / (cpm * F3(f.rho1, j, i, k));
      F3(f.a2t, j, i, k) = F3(f.a2t, j, i, k) + c->gnu1 * dpterm;
      F3(f.a1t, j, i, k) = F3(f.a1t, j, i, k) + dpterm;
      wm = wp;
      if (!nexta) {
        F3(f.cpp, j, i, k) = p;
        if (last) {
          const double pf = psb * p;
          const double d = c->gnu1 * (pf + F3(f.a2pp, j, i, k) - d_two * F3(f.a1pp, j, i, k));
          F3(f.a2pp, j, i, k) = F3(f.a1pp, j, i, k) + d;
          F3(f.a1pp, j, i, k) = pf;
        }
        continue;
      }
      // part A of the next sub-step on this column (:250-262): pp += xkd*pi, then dp'/dp0 at
      // the level above, whose neighbours k-2 (clamped to 1) and k are now known
      const double pa = p + c->nhxkd * spn;
      const double pr = F3(f.pr0, j, i, k);
      F3(f.cpp, j, i, k) = pa;
      if (k >= 2) {
        const double pk1 = (k >= 3) ? pamm : pam, rk1 = (k >= 3) ? prmm : prm;
        F3(f.cdt, j, i, k - 1) = (pk1 - pa) / (rk1 - pr);
      }
      if (k == kz) F3(f.cdt, j, i, kz) = (pam - pa) / (prm - pr);
      pamm = pam; prmm = prm; pam = pa; prm = pr;
    }
  }
  unsigned long long bits = cfl;
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(bits, off);
    bits = (o > bits) ? o : bits;
  }
  const int wv = threadIdx.y;                          // blockDim = 64 x 4: one wavefront per row
  if (threadIdx.x == 0) sred[wv] = bits;
  __syncthreads();
  if (threadIdx.x == 0 && wv == 0) {
    unsigned long long b = sred[0];
    for (int q = 1; q < 4; q++) b = (sred[q] > b) ? sred[q] : b;
    const unsigned slot = (blockIdx.x + blockIdx.y * gridDim.x) & (NH_CFL_SLOTS - 1);
    if (b != 0ull) {
      atomicMax(&f.cfl[slot], b);
      if (last) atomicMax(&f.cfll[slot], b);
    }
  }
}

// time filters after the acoustic loop (:686-702) off the interior cross columns: the last
// sub-step's k_nh_sound_uv filters u, v and its k_nh_sound_cd pp and w on the interior; what
// remains is the small-value clamp of w (the acoustic w, atm1/atm2 w) on the other frame
// points.  k = 1..kz+1.
// The frame points outside the interior as a list (nh_frame_ring: the rows below and above the
// interior over the frame's width, then the columns left and right of it), blockIdx.y = k - 1:
// a whole-frame grid spent 39 us at C5 on threads that return at once.
int nh_frame_ring(const Geom& g) {
  return (g.ici1 - g.i0 + g.i0 + g.ni - 1 - g.ici2) * g.nj + (g.ici2 - g.ici1 + 1) * (g.jci1 - g.j0 + g.j0 + g.nj - 1 - g.jci2);
}
__global__ void k_nh_sound_final(Geom g, const Consts* __restrict__ c, NHFields f) {
  (void)c;
  const int W = g.nj, wl = g.jci1 - g.j0, wr = g.j0 + g.nj - 1 - g.jci2;
  const int hb = g.ici1 - g.i0, ht = g.i0 + g.ni - 1 - g.ici2, hm = g.ici2 - g.ici1 + 1;
  int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int k = (int)blockIdx.y + 1;
  int j, i;
  if (q < hb * W) { i = g.i0 + q / W; j = g.j0 + q % W; }
  else if ((q -= hb * W) < ht * W) { i = g.ici2 + 1 + q / W; j = g.j0 + q % W; }
  else if ((q -= ht * W) < hm * (wl + wr)) {
    const int m = q % (wl + wr);
    i = g.ici1 + q / (wl + wr);
    j = m < wl ? g.j0 + m : g.jci2 + 1 + (m - wl);
  } else {
    return;
  }
  double w = F3(f.cw, j, i, k);
  if (fabs(w) < DLOWVAL) w = d_zero;
  F3(f.cw, j, i, k) = w;
  if (fabs(F3(f.a2w, j, i, k)) < DLOWVAL) F3(f.a2w, j, i, k) = d_zero;
  if (fabs(F3(f.a1w, j, i, k)) < DLOWVAL) F3(f.a1w, j, i, k) = d_zero;
}

// rcmtimer advance and the sound CFL stop (Main/mod_sound.F90:661-682,
// Main/mod_tendency.F90:608-616)
__global__ void k_nh_advance(const Consts* __restrict__ c, StepState* s, NHFields f) {
  __shared__ unsigned long long sm[256], sl[256];
  unsigned long long b = 0ull, bl = 0ull;
  for (int q = threadIdx.x; q < NH_CFL_SLOTS; q += blockDim.x) {
    const unsigned long long v = f.cfl[q], vl = f.cfll[q];
    b = (v > b) ? v : b;
    bl = (vl > bl) ? vl : bl;
    f.cfl[q] = 0ull;
    f.cfll[q] = 0ull;
  }
  sm[threadIdx.x] = b;
  sl[threadIdx.x] = bl;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sm[threadIdx.x] = (sm[threadIdx.x + w] > sm[threadIdx.x]) ? sm[threadIdx.x + w] : sm[threadIdx.x];
      sl[threadIdx.x] = (sl[threadIdx.x + w] > sl[threadIdx.x]) ? sl[threadIdx.x + w] : sl[threadIdx.x];
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double cfl = __longlong_as_double((long long)sm[0]);
  if (cfl > d_one || cfl != cfl) s->nanflag = 1;
  s->cflmax = __longlong_as_double((long long)sl[0]);
  s->lcount += 1;
  if (s->lcount == 2) s->dt = d_two * c->dtsec;
  s->ptntot = 0.0;
  s->pt2tot = 0.0;
}

// pp and w boundary values of bdyval (Main/mod_bdycod.F90:1150-1160, 1196-1206, 1242-1252,
// 1285-1295, 1707-1790).  A: copies and time interpolation, one thread per boundary cross
// point and level; B (one block): the w(k=1) copies W/E on ici, then S/N on jce (they read
// the W/E results at the corners).
__global__ void k_nh_bdyval(Geom g, int kz, const StepState* __restrict__ s, NHFields f) {
  const int nci = g.ici2 - g.ici1 + 1, ncj = g.jce2 - g.jce1 + 1;
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x), k = (int)blockIdx.y + 1;
  int j, i;
  if (p < nci) { if (!g.bl) return; j = g.jce1; i = g.ici1 + p; }
  else if (p < 2 * nci) { if (!g.br) return; j = g.jce2; i = g.ici1 + p - nci; }
  else if (p < 2 * nci + ncj) { if (!g.bb) return; j = g.jce1 + p - 2 * nci; i = g.ice1; }
  else if (p < 2 * nci + 2 * ncj) { if (!g.bt) return; j = g.jce1 + p - 2 * nci - ncj; i = g.ice2; }
  else return;
  const double xt = s->xbctime + s->dt;
  const bool integ = s->lcount > 0;
  if (k <= kz) {
    if (integ) F3(f.a2pp, j, i, k) = F3(f.a1pp, j, i, k);
    F3(f.a1pp, j, i, k) = F3(f.ppb0, j, i, k) + xt * F3(f.ppbt, j, i, k);
  }
  if (integ) F3(f.a2w, j, i, k) = F3(f.a1w, j, i, k);
  F3(f.a1w, j, i, k) = F3(f.wwb0, j, i, k) + xt * F3(f.wwbt, j, i, k);
}

__global__ void k_nh_bdyval_w1(Geom g, NHFields f) {
  const int nci = g.ici2 - g.ici1 + 1, ncj = g.jce2 - g.jce1 + 1;
  for (int t = threadIdx.x; t < nci; t += blockDim.x) {
    const int i = g.ici1 + t;
    if (g.bl) F3(f.a1w, g.jce1, i, 1) = F3(f.a1w, g.jci1, i, 1);
    if (g.br) F3(f.a1w, g.jce2, i, 1) = F3(f.a1w, g.jci2, i, 1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < ncj; t += blockDim.x) {
    const int j = g.jce1 + t;
    if (g.bb) F3(f.a1w, j, g.ice1, 1) = F3(f.a1w, j, g.ici1, 1);
    if (g.bt) F3(f.a1w, j, g.ice2, 1) = F3(f.a1w, j, g.ici2, 1);
  }
}

#endif  // NH_OTHER_KERNELS
}  // namespace rcm
