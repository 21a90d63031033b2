// kernels.hip -- HIP/CDNA4 kernels of the hydrostatic dynamical-core step (gfx950).
//
// Every kernel evaluates each output element with the same floating-point operation
// sequence as the reference loop nests it fuses (see oracle/rcm_oracle.c for the literal
// restatement and the Main/*.F90 file:line citations repeated below).  Contributions that the
// reference accumulates into one tendency element in several passes are accumulated here in
// the same order inside one thread, so transcendental-free results are bit-identical
// (compiled with -ffp-contract=off).
//
// Thread mapping: x -> j (west-east, unit stride, coalesced), y -> i, z -> k; blocks of
// 64 x 4.  Column recurrences (pten/qdot, phi, split projections) use one thread per
// (j,i) column with the k loop in registers.
#include "engine.hpp"
#include "kernels.hpp"

namespace rcm {

#define F2(a, j, i) (a)[g.ix(j, i)]
#define F3(a, j, i, k) (a)[(long)((k) - 1) * g.plane + g.ix(j, i)]
#define SLI(s, i, k) (s)[(long)((k) - 1) * slen + ((i) - g.i0)]
#define SLJ(s, j, k) (s)[(long)((k) - 1) * slen + ((j) - g.j0)]

static constexpr double d_zero = 0.0, d_one = 1.0, d_two = 2.0, d_four = 4.0;
static constexpr double d_half = 0.5, d_rfour = 0.25, d_1000 = 1000.0;
static constexpr double MINQQ = 1.0e-8, DLOWVAL = 1.0e-20;
static constexpr double z4_c1 = 1.0, z4_c2 = -4.0, z4_c3 = 12.0;

__device__ __forceinline__ double dmax(double a, double b) { return (a > b) ? a : (b > a ? b : a); }
__device__ __forceinline__ double dmin(double a, double b) { return (a < b) ? a : (b < a ? b : a); }

__device__ __forceinline__ bool in(int v, int lo, int hi) { return v >= lo && v <= hi; }

// thread -> (j, i, k) over a box starting at (j1, i1); k = blockIdx.z + kbase
#define THREAD_POINT(j1, i1)                                   \
  const int j = (j1) + (int)(blockIdx.x * blockDim.x + threadIdx.x); \
  const int i = (i1) + (int)(blockIdx.y * blockDim.y + threadIdx.y); \
  const int k = (int)blockIdx.z + 1;                              \
  (void)k;

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
// surface_pressures, Main/mod_tendency.F90:815-834 (both time levels in one pass)
__global__ void k_surface_pressures(Geom g, const double* __restrict__ psa, const double* __restrict__ psb,
                                    double* rpsa, double* rpsb, double* psdota, double* psdotb) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  if (in(j, g.jce1ga, g.jce2ga) && in(i, g.ice1ga, g.ice2ga)) F2(rpsa, j, i) = d_one / F2(psa, j, i);
  if (in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2)) F2(rpsb, j, i) = d_one / F2(psb, j, i);
  double v;
  if (psc2psd_at(g, psa, j, i, v)) F2(psdota, j, i) = v;
  if (psc2psd_at(g, psb, j, i, v)) F2(psdotb, j, i) = v;
}

// psdota only (splitf, Main/mod_split.F90:259-260)
__global__ void k_psc2psd(Geom g, const double* __restrict__ pc, double* pd) {
  THREAD_POINT(g.jde1, g.ide1);
  if (j > g.jde2 || i > g.ide2) return;
  double v;
  if (psc2psd_at(g, pc, j, i, v)) F2(pd, j, i) = v;
}

// ---------------------------------------------------------------------------------------
// decouple, Main/mod_tendency.F90:858-1025 (hydrostatic).  ud/vd are atm1*rpsda on the whole
// dot range: on the boundary rows this equals the reference's boundary-slice assignment
// (:895-994) because bdyval stores the identical value b0+xt*bt in both atm1 and the slice.
__global__ void k_decouple(Geom g, const double* __restrict__ a1u, const double* __restrict__ a1v,
                           const double* __restrict__ a1t, const double* __restrict__ a1qv,
                           const double* __restrict__ a1qc, const double* __restrict__ msfd,
                           const double* __restrict__ psdota, const double* __restrict__ rpsa,
                           double* rpsda, double* umc, double* vmc, double* ud, double* vd,
                           double* xt, double* xqv, double* xqc, double* xtv, double ep1) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  if (in(j, g.jde1ga, g.jde2ga) && in(i, g.ide1ga, g.ide2ga)) {
    const double r = d_one / F2(psdota, j, i);
    if (k == 1) F2(rpsda, j, i) = r;
    const double u = F3(a1u, j, i, k), v = F3(a1v, j, i, k), m = F2(msfd, j, i);
    F3(umc, j, i, k) = u * m;
    F3(vmc, j, i, k) = v * m;
    if (in(j, g.jde1, g.jde2) && in(i, g.ide1, g.ide2)) {
      F3(ud, j, i, k) = u * r;
      F3(vd, j, i, k) = v * r;
    }
  }
  if (in(j, g.jce1ga, g.jce2ga) && in(i, g.ice1ga, g.ice2ga)) {
    const double rp = F2(rpsa, j, i);
    const double t = F3(a1t, j, i, k) * rp;
    const double qv = dmax(F3(a1qv, j, i, k) * rp, MINQQ);
    const double qc = dmax(F3(a1qc, j, i, k) * rp, d_zero);
    F3(xt, j, i, k) = t;
    F3(xqv, j, i, k) = qv;
    F3(xqc, j, i, k) = qc;
    F3(xtv, j, i, k) = t * (d_one + ep1 * qv);
  }
}

// ---------------------------------------------------------------------------------------
// compute_omega column part, Main/mod_tendency.F90:1123-1156: pten and qdot (k-scan).
__device__ __forceinline__ double mass_div(const Geom& g, const double* umc, const double* vmc, int j, int i,
                                           int k, double dummy) {
  const double a = F3(umc, j + 1, i + 1, k) + F3(umc, j + 1, i, k) - F3(umc, j, i + 1, k) - F3(umc, j, i, k);
  const double b = F3(vmc, j + 1, i + 1, k) + F3(vmc, j, i + 1, k) - F3(vmc, j + 1, i, k) - F3(vmc, j, i, k);
  return (a + b) * dummy;
}

__global__ void k_omega_col(Geom g, const Consts* __restrict__ c, const double* __restrict__ umc,
                            const double* __restrict__ vmc, const double* __restrict__ msfx,
                            const double* __restrict__ rpsa, double* pten, double* qdot) {
  const int j = g.jde1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ide1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jde2 || i > g.ide2) return;
  const int kz = c->kz;
  if (!(in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2))) {
    for (int k = 1; k <= kz + 1; k++) F3(qdot, j, i, k) = d_zero;
    return;
  }
  const double mx = F2(msfx, j, i);
  const double dummy = d_one / (c->dx2 * mx * mx);
  double pt = d_zero;
  for (int k = 1; k <= kz; k++) pt = pt - mass_div(g, umc, vmc, j, i, k, dummy) * c->dsigma[k];
  F2(pten, j, i) = pt;
  const double rp = F2(rpsa, j, i);
  double q = d_zero;
  F3(qdot, j, i, 1) = d_zero;
  for (int k = 2; k <= kz; k++) {
    const double crm = mass_div(g, umc, vmc, j, i, k - 1, dummy);
    q = q - (pt + crm) * c->dsigma[k - 1] * rp;
    F3(qdot, j, i, k) = q;
  }
  F3(qdot, j, i, kz + 1) = d_zero;
}

// omega at one point, Main/mod_tendency.F90:1200-1214
__device__ __forceinline__ double omega_at(const Geom& g, const Consts* c, const double* qdot, const double* pten,
                                           const double* ud, const double* vd, const double* psa,
                                           const double* msfx, int j, int i, int k) {
  const double dummy = d_one / (c->dx8 * F2(msfx, j, i));
  const double su = F3(ud, j, i, k) + F3(ud, j, i + 1, k) + F3(ud, j + 1, i + 1, k) + F3(ud, j + 1, i, k);
  const double sv = F3(vd, j, i, k) + F3(vd, j, i + 1, k) + F3(vd, j + 1, i + 1, k) + F3(vd, j + 1, i, k);
  const double x = su * (F2(psa, j + 1, i) - F2(psa, j - 1, i)) + sv * (F2(psa, j, i + 1) - F2(psa, j, i - 1));
  return d_half * (F3(qdot, j, i, k + 1) + F3(qdot, j, i, k)) * F2(psa, j, i) +
         c->hsigma[k] * (F2(pten, j, i) + x * dummy);
}

// ---------------------------------------------------------------------------------------
// mkslice dyn subset, Main/mod_slice.F90:163-183
__global__ void k_mkslice(Geom g, const double* __restrict__ a2u, const double* __restrict__ a2v,
                          const double* __restrict__ a2t, const double* __restrict__ a2qv,
                          const double* __restrict__ a2qc, const double* __restrict__ psb,
                          const double* __restrict__ psdotb, double* ubd, double* vbd, double* tb3d,
                          double* qvb, double* qcb) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  if (in(j, g.jde1gb, g.jde2gb) && in(i, g.ide1gb, g.ide2gb)) {
    const double r = d_one / F2(psdotb, j, i);
    F3(ubd, j, i, k) = F3(a2u, j, i, k) * r;
    F3(vbd, j, i, k) = F3(a2v, j, i, k) * r;
  }
  if (in(j, g.jce1gb, g.jce2gb) && in(i, g.ice1gb, g.ice2gb)) {
    const double r = d_one / F2(psb, j, i);
    F3(tb3d, j, i, k) = F3(a2t, j, i, k) * r;
    F3(qvb, j, i, k) = dmax(F3(a2qv, j, i, k) * r, MINQQ);
    F3(qcb, j, i, k) = dmax(F3(a2qc, j, i, k) * r, d_zero);
  }
}

// ---------------------------------------------------------------------------------------
// generic relaxation contribution (nudge*, Main/mod_bdycod.F90:4262-4263)
__device__ __forceinline__ double relax(double ften, double xf, double xg, double f0, double f1, double f2,
                                        double f3, double f4) {
  return ften + xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0);
}
__device__ __forceinline__ void nudge_coef(const Consts* c, int ib, int k, double& xf, double& xg) {
  if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; }
  else { xf = c->hefc[ib][k]; xg = c->hegc[ib][k]; }
}

// new_pressure, Main/mod_tendency.F90:1428-1460 (+ nudge2d, Main/mod_bdycod.F90:4597-4766)
// plus per-block partial sums of the Bleck noise parameters.
__global__ void k_new_pressure(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s,
                               const double* __restrict__ psa, const double* __restrict__ psb,
                               const double* __restrict__ pb0, const double* __restrict__ pbt,
                               const int8_t* __restrict__ rgcr, const int16_t* __restrict__ ibcr,
                               const double* __restrict__ pten, double* ptenn, double* psc, double* rpsc,
                               double* red) {
  THREAD_POINT(g.jce1, g.ice1);
  const double dt = s->dt;
  const double xt = s->xbctime + dt;
  double a = 0.0, b = 0.0;
  if (j <= g.jce2 && i <= g.ice2) {
    double pt = F2(pten, j, i);
    if (in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2) && F2(rgcr, j, i) > 0) {
      double xf, xg;
      nudge_coef(c, F2(ibcr, j, i), c->kz, xf, xg);
#define FG1(J, I) ((F2(pb0, J, I) + xt * F2(pbt, J, I)) - F2(psb, J, I))
      pt = relax(pt, xf, xg, FG1(j, i), FG1(j - 1, i), FG1(j + 1, i), FG1(j, i - 1), FG1(j, i + 1));
#undef FG1
    }
    F2(ptenn, j, i) = pt;
    const double pc = F2(psb, j, i) + pt * dt;
    F2(psc, j, i) = pc;
    F2(rpsc, j, i) = d_one / pc;
    if (s->lcount > 0 && in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2)) {
      a = fabs(pt);
      b = fabs((pc + F2(psb, j, i) - d_two * F2(psa, j, i)) / (dt * dt * d_rfour));
    }
  }
  // deterministic block reduction (fixed tree order)
  __shared__ double sa[256], sb[256];
  const int t = threadIdx.y * blockDim.x + threadIdx.x;
  sa[t] = a; sb[t] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { sa[t] += sa[t + w]; sb[t] += sb[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    const int blk = blockIdx.y * gridDim.x + blockIdx.x;
    red[2 * blk] = sa[0];
    red[2 * blk + 1] = sb[0];
  }
}

__global__ void k_reduce_noise(const double* __restrict__ red, int nblk, StepState* s) {
  __shared__ double sa[256], sb[256];
  const int t = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int q = t; q < nblk; q += 256) { a += red[2 * q]; b += red[2 * q + 1]; }
  sa[t] = a; sb[t] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { sa[t] += sa[t + w]; sb[t] += sb[t + w]; }
    __syncthreads();
  }
  if (t == 0) {
    s->ptntot = sa[0];
    s->pt2tot = sb[0];
    if (sa[0] != sa[0]) s->nanflag = 1;
  }
}

// ---------------------------------------------------------------------------------------
// calc_coeff Smagorinsky part, Main/mod_diffusion.F90:194-210 (unscaled xkc on jce/ice)
__global__ void k_calc_coeff(Geom g, const Consts* __restrict__ c, const double* __restrict__ ubd,
                             const double* __restrict__ vbd, const double* __restrict__ hgfact, double* xkc) {
  THREAD_POINT(g.jce1, g.ice1);
  if (j > g.jce2 || i > g.ice2) return;
  const double dudx = F3(ubd, j + 1, i, k) + F3(ubd, j + 1, i + 1, k) - F3(ubd, j, i, k) - F3(ubd, j, i + 1, k);
  const double dvdx = F3(vbd, j + 1, i, k) + F3(vbd, j + 1, i + 1, k) - F3(vbd, j, i, k) - F3(vbd, j, i + 1, k);
  const double dudy = F3(ubd, j, i + 1, k) + F3(ubd, j + 1, i + 1, k) - F3(ubd, j, i, k) - F3(ubd, j + 1, i, k);
  const double dvdy = F3(vbd, j, i + 1, k) + F3(vbd, j + 1, i + 1, k) - F3(vbd, j, i, k) - F3(vbd, j + 1, i, k);
  const double duv = sqrt((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy));
  F3(xkc, j, i, k) = dmin(F2(hgfact, j, i) + c->dydc * duv, c->xkhmax);
}

// ---------------------------------------------------------------------------------------
// pressure_gradient_force geopotential column, Main/mod_tendency.F90:1966-1995, 2033-2097.
// alpha_hyd = 0 (Share/mod_constants.F90:319) makes td == tva bit-for-bit for finite input.
__global__ void k_phi_col(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1t,
                          const double* __restrict__ xqv, const double* __restrict__ xqc,
                          const double* __restrict__ psa, const double* __restrict__ rpsa,
                          const double* __restrict__ ht, double* phi) {
  const int j = g.jce1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ice1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jce2 || i > g.ice2) return;
  const int kz = c->kz;
  const double rp = F2(rpsa, j, i);
  const double ps = F2(psa, j, i);
  const double ptop = c->ptop, rgas = c->rgas, ep1 = c->ep1;
#define TD(K) (F3(a1t, j, i, K) * (d_one + ep1 * F3(xqv, j, i, K)))
#define TVFAC(K) (d_one / (d_one + F3(xqc, j, i, K) / (d_one + F3(xqv, j, i, K))))
  double tdk1 = TD(kz);
  const double tv = tdk1 * rp * TVFAC(kz);
  double ph = F2(ht, j, i) - rgas * tv * log((c->hsigma[kz] + ptop * rp) / (d_one + ptop * rp));
  F3(phi, j, i, kz) = ph;
  for (int lev = kz - 1; lev >= 1; lev--) {
    const double tdl = TD(lev);
    const double tvavg = ((tdl * c->dsigma[lev] + tdk1 * c->dsigma[lev + 1]) /
                          (ps * (c->dsigma[lev] + c->dsigma[lev + 1]))) * TVFAC(lev);
    ph = ph - rgas * tvavg * log((c->hsigma[lev] + ptop * rp) / (c->hsigma[lev + 1] + ptop * rp));
    F3(phi, j, i, lev) = ph;
    tdk1 = tdl;
  }
#undef TD
#undef TVFAC
}

// ---------------------------------------------------------------------------------------
// Momentum: hadvuv + vadvuv + curvature + nudgeuv + diffu_d + PGF, then the forecast and the
// Robert-Asselin filter (Main/mod_advection.F90:203-299, Main/mod_tendency.F90:1829-1838,
// Main/mod_bdycod.F90:3581-3823, Main/mod_diffusion.F90:281-385, Main/mod_tendency.F90:
// 1996-2025, 2103-2115, 404-411, 433-445; Main/mod_timefilter.F90 filter_ra_uv).
__global__ __launch_bounds__(256) void k_momentum(
    Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s,
    const double* __restrict__ a1u, const double* __restrict__ a1v,
    const double* __restrict__ a2u, const double* __restrict__ a2v,
    double* __restrict__ n1u, double* __restrict__ n1v, double* __restrict__ n2u, double* __restrict__ n2v,
    const double* __restrict__ umc, const double* __restrict__ vmc, const double* __restrict__ ud,
    const double* __restrict__ vd, const double* __restrict__ qdot, const double* __restrict__ coriol,
    const double* __restrict__ dmsf, const double* __restrict__ msfd,
    const double* __restrict__ ub0, const double* __restrict__ ubt, const double* __restrict__ vb0,
    const double* __restrict__ vbt, const int8_t* __restrict__ rgdt, const int16_t* __restrict__ ibdt,
    const double* __restrict__ xkc, const double* __restrict__ psdotb,
    const double* __restrict__ ubd, const double* __restrict__ vbd,
    const double* __restrict__ xtv, const double* __restrict__ psdota, const double* __restrict__ psa,
    const double* __restrict__ phi, double* uten, double* vten) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const long p = (long)(k - 1) * g.plane + g.ix(j, i);
  if (!(in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2))) {
    n1u[p] = a1u[p]; n1v[p] = a1v[p]; n2u[p] = a2u[p]; n2v[p] = a2v[p];
    return;
  }
  const int kz = c->kz;
  const double dt = s->dt;
  // hadvuv (upstream, hydrostatic)
  double ut, vt;
  {
    const double* ua = umc; const double* va = vmc;
    const double ucmona = F3(ua, j, i + 1, k) + d_two * F3(ua, j, i, k) + F3(ua, j, i - 1, k);
    double ucmonb = F3(ua, j + 1, i + 1, k) + d_two * F3(ua, j + 1, i, k) + F3(ua, j + 1, i - 1, k);
    double ucmonc = F3(ua, j - 1, i + 1, k) + d_two * F3(ua, j - 1, i, k) + F3(ua, j - 1, i - 1, k);
    const double vcmona = F3(va, j + 1, i, k) + d_two * F3(va, j, i, k) + F3(va, j - 1, i, k);
    double vcmonb = F3(va, j + 1, i + 1, k) + d_two * F3(va, j, i + 1, k) + F3(va, j - 1, i + 1, k);
    double vcmonc = F3(va, j + 1, i - 1, k) + d_two * F3(va, j, i - 1, k) + F3(va, j - 1, i - 1, k);
    const double u0 = F3(ud, j, i, k), ue = F3(ud, j + 1, i, k), uw = F3(ud, j - 1, i, k);
    const double un = F3(ud, j, i + 1, k), us = F3(ud, j, i - 1, k);
    const double v0 = F3(vd, j, i, k), ve = F3(vd, j + 1, i, k), vw = F3(vd, j - 1, i, k);
    const double vn = F3(vd, j, i + 1, k), vs = F3(vd, j, i - 1, k);
    const double ul = c->ul;
    const double ff1 = ul * (ue + u0), ff2 = ul * (uw + u0), ff3 = ul * (vn + v0), ff4 = ul * (vs + v0);
    ucmonb = (d_one + ff1) * ucmona + (d_one - ff1) * ucmonb;
    ucmonc = (d_one + ff2) * ucmonc + (d_one - ff2) * ucmona;
    vcmonb = (d_one + ff3) * vcmona + (d_one - ff3) * vcmonb;
    vcmonc = (d_one + ff4) * vcmonc + (d_one - ff4) * vcmona;
    const double dm = F2(dmsf, j, i);
    ut = d_zero - dm * ((ue + u0) * ucmonb - (u0 + uw) * ucmonc + (un + u0) * vcmonb - (u0 + us) * vcmonc);
    vt = d_zero - dm * ((ve + v0) * ucmonb - (v0 + vw) * ucmonc + (vn + v0) * vcmonb - (v0 + vs) * vcmonc);
  }
  // vadvuv: flux at interface k (from loop index k) then interface k+1 (loop index k+1)
  {
#define QQ(K) (d_rfour * (F3(qdot, j, i, K) + F3(qdot, j, i - 1, K) + F3(qdot, j - 1, i, K) + F3(qdot, j - 1, i - 1, K)))
    if (k >= 2) {
      const double qq = QQ(k);
      const double uu = qq * (c->twt1[k] * F3(a1u, j, i, k) + c->twt2[k] * F3(a1u, j, i, k - 1));
      const double vv = qq * (c->twt1[k] * F3(a1v, j, i, k) + c->twt2[k] * F3(a1v, j, i, k - 1));
      ut = ut + uu * c->xds[k];
      vt = vt + vv * c->xds[k];
    }
    if (k + 1 <= kz) {
      const double qq = QQ(k + 1);
      const double uu = qq * (c->twt1[k + 1] * F3(a1u, j, i, k + 1) + c->twt2[k + 1] * F3(a1u, j, i, k));
      const double vv = qq * (c->twt1[k + 1] * F3(a1v, j, i, k + 1) + c->twt2[k + 1] * F3(a1v, j, i, k));
      ut = ut - uu * c->xds[k];
      vt = vt - vv * c->xds[k];
    }
#undef QQ
  }
  // curvature (hydrostatic Coriolis)
  ut = ut + F2(coriol, j, i) * F3(a1v, j, i, k);
  vt = vt - F2(coriol, j, i) * F3(a1u, j, i, k);
  // nudgeuv
  if (F2(rgdt, j, i) > 0) {
    const double xt = s->xbctime + dt;
    double xf, xg;
    const int ib = F2(ibdt, j, i);
    if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; } else { xf = c->hefc[ib][k]; xg = c->hegc[ib][k]; }
#define FGU(J, I) ((F3(ub0, J, I, k) + xt * F3(ubt, J, I, k)) - F3(a2u, J, I, k))
#define FGV(J, I) ((F3(vb0, J, I, k) + xt * F3(vbt, J, I, k)) - F3(a2v, J, I, k))
    ut = relax(ut, xf, xg, FGU(j, i), FGU(j - 1, i), FGU(j + 1, i), FGU(j, i - 1), FGU(j, i + 1));
    vt = relax(vt, xf, xg, FGV(j, i), FGV(j - 1, i), FGV(j + 1, i), FGV(j, i - 1), FGV(j, i + 1));
#undef FGU
#undef FGV
  }
  // diffu_d (idiffu = 1); xkd from calc_coeff (Main/mod_diffusion.F90:237-248)
  {
    double xkd = d_rfour * (F3(xkc, j, i, k) + F3(xkc, j - 1, i - 1, k) + F3(xkc, j - 1, i, k) + F3(xkc, j, i - 1, k));
    xkd = xkd * c->rdxsq * F2(psdotb, j, i);
#define UM(a, J, I) (F3(a, J, I, k) / F2(msfd, J, I))
    if (in(j, g.jdii1, g.jdii2) && in(i, g.idii1, g.idii2)) {
      ut = ut - xkd * (z4_c1 * (UM(ubd, j + 2, i) + UM(ubd, j - 2, i) + UM(ubd, j, i + 2) + UM(ubd, j, i - 2)) +
                       z4_c2 * (UM(ubd, j + 1, i) + UM(ubd, j - 1, i) + UM(ubd, j, i + 1) + UM(ubd, j, i - 1)) +
                       z4_c3 * (UM(ubd, j, i)));
      vt = vt - xkd * (z4_c1 * (UM(vbd, j + 2, i) + UM(vbd, j - 2, i) + UM(vbd, j, i + 2) + UM(vbd, j, i - 2)) +
                       z4_c2 * (UM(vbd, j + 1, i) + UM(vbd, j - 1, i) + UM(vbd, j, i + 1) + UM(vbd, j, i - 1)) +
                       z4_c3 * (UM(vbd, j, i)));
    }
#define LAPD()                                                                                              \
  ut = ut + xkd * (z4_c1 * (UM(ubd, j + 1, i) + UM(ubd, j - 1, i) + UM(ubd, j, i + 1) + UM(ubd, j, i - 1)) + \
                   z4_c2 * (UM(ubd, j, i)));                                                                \
  vt = vt + xkd * (z4_c1 * (UM(vbd, j + 1, i) + UM(vbd, j - 1, i) + UM(vbd, j, i + 1) + UM(vbd, j, i - 1)) + \
                   z4_c2 * (UM(vbd, j, i)));
    if (g.bl && j == g.jdi1) { LAPD(); }
    if (g.br && j == g.jdi2) { LAPD(); }
    if (g.bb && i == g.idi1) { LAPD(); }
    if (g.bt && i == g.idi2) { LAPD(); }
#undef LAPD
#undef UM
  }
  // pressure gradient force, part 1 (ipgf = 0) and part 2 (geopotential gradient)
  {
    double rtbar = d_rfour * (F3(xtv, j - 1, i - 1, k) + F3(xtv, j - 1, i, k) + F3(xtv, j, i - 1, k) + F3(xtv, j, i, k));
    rtbar = c->rgas * rtbar * F2(psdota, j, i);
    const double hs = c->hsigma[k], pt = c->ptop;
    const double den = c->dx * F2(msfd, j, i);
    const double p00 = F2(psa, j, i), p0m = F2(psa, j, i - 1), pm0 = F2(psa, j - 1, i), pmm = F2(psa, j - 1, i - 1);
    ut = ut - rtbar * (log(d_half * (p00 + p0m) * hs + pt) - log(d_half * (pm0 + pmm) * hs + pt)) / den;
    vt = vt - rtbar * (log(d_half * (p00 + pm0) * hs + pt) - log(d_half * (pmm + p0m) * hs + pt)) / den;
    const double den2 = c->dx2 * F2(msfd, j, i);
    const double pd = F2(psdota, j, i);
    ut = ut - pd * (F3(phi, j, i, k) + F3(phi, j, i - 1, k) - F3(phi, j - 1, i, k) - F3(phi, j - 1, i - 1, k)) / den2;
    vt = vt - pd * (F3(phi, j, i, k) + F3(phi, j - 1, i, k) - F3(phi, j, i - 1, k) - F3(phi, j - 1, i - 1, k)) / den2;
  }
  // totals (uphy = 0), forecast, RA filter
  ut = (d_zero + ut) + d_zero;
  vt = (d_zero + vt) + d_zero;
  uten[p] = ut;
  vten[p] = vt;
  const double g1 = c->gnu1;
  const double u1 = a1u[p], u2 = a2u[p], v1 = a1v[p], v2 = a2v[p];
  const double cu = u2 + dt * ut, cv = v2 + dt * vt;
  double d = g1 * (cu + u2 - d_two * u1);
  n2u[p] = u1 + d;
  n1u[p] = cu;
  d = g1 * (cv + v2 - d_two * v1);
  n2v[p] = v1 + d;
  n1v[p] = cv;
}

// ---------------------------------------------------------------------------------------
// Scalar upstream flux-form advection (hadvt/hadvqv/hadvqx, Main/mod_advection.F90:337-386,
// 547-596, 639-653) for one point; limiter 0 none, 1 t_extrema, 2 q_rel_extrema.
__device__ __forceinline__ double hadv_point(const Geom& g, const Consts* c, const double* f, const double* umc,
                                             const double* vmc, const double* psa, const double* xmsf,
                                             int j, int i, int k, int limiter) {
  const double uavg1 = F3(umc, j, i + 1, k) + F3(umc, j, i, k);
  const double uavg2 = F3(umc, j + 1, i + 1, k) + F3(umc, j + 1, i, k);
  const double vavg1 = F3(vmc, j + 1, i, k) + F3(vmc, j, i, k);
  const double vavg2 = F3(vmc, j + 1, i + 1, k) + F3(vmc, j, i + 1, k);
  const double ps = F2(psa, j, i);
  const double ul = c->ul;
  const double f1 = d_half * ul * (uavg2 + uavg1) / ps;
  const double f2 = d_half * ul * (vavg2 + vavg1) / ps;
  const double fc = F3(f, j, i, k), fw = F3(f, j - 1, i, k), fe = F3(f, j + 1, i, k);
  const double fs = F3(f, j, i - 1, k), fn = F3(f, j, i + 1, k);
  const double fx1 = (d_one + f1) * fw + (d_one - f1) * fc;
  const double fx2 = (d_one + f1) * fc + (d_one - f1) * fe;
  const double fy1 = (d_one + f2) * fs + (d_one - f2) * fc;
  const double fy2 = (d_one + f2) * fc + (d_one - f2) * fn;
  double fg = -F2(xmsf, j, i) * (uavg2 * fx2 - uavg1 * fx1 + vavg2 * fy2 - vavg1 * fy1);
  if (limiter && c->stability_enhance) {
    double den, thr;
    if (limiter == 1) { den = ps; thr = c->t_extrema; } else { den = dmax(fc, DLOWVAL); thr = c->q_rel_extrema; }
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

// diffu_x (idiffu = 1) for one point, Main/mod_diffusion.F90:673-713 / 808-...
__device__ __forceinline__ double diffu_x_point(const Geom& g, double ften, double xkcs, const double* f,
                                                int j, int i, int k) {
  if (in(j, g.jcii1, g.jcii2) && in(i, g.icii1, g.icii2)) {
    ften = ften - d_one * xkcs *
        (z4_c1 * (F3(f, j + 2, i, k) + F3(f, j - 2, i, k) + F3(f, j, i + 2, k) + F3(f, j, i - 2, k)) +
         z4_c2 * (F3(f, j + 1, i, k) + F3(f, j - 1, i, k) + F3(f, j, i + 1, k) + F3(f, j, i - 1, k)) +
         z4_c3 * F3(f, j, i, k));
  }
#define LAP2() ften = ften + d_one * xkcs * \
    (z4_c1 * (F3(f, j + 1, i, k) + F3(f, j - 1, i, k) + F3(f, j, i + 1, k) + F3(f, j, i - 1, k)) + z4_c2 * F3(f, j, i, k))
  if (g.bl && j == g.jci1) { LAP2(); }
  if (g.br && j == g.jci2) { LAP2(); }
  if (g.bb && i == g.ici1) { LAP2(); }
  if (g.bt && i == g.ici2) { LAP2(); }
#undef LAP2
  return ften;
}

// Temperature: hadvt + vadv3d + adiabatic + nudge3d + diffu_x3d, forecast and RA filter
// (Main/mod_tendency.F90:1327-1341, 1561-1575, 1469, 1525, 285-287, 368-374, 422).
__global__ __launch_bounds__(256) void k_temperature(
    Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s,
    const double* __restrict__ a1t, const double* __restrict__ a2t, double* __restrict__ n1t,
    double* __restrict__ n2t, const double* __restrict__ xt, const double* __restrict__ umc,
    const double* __restrict__ vmc, const double* __restrict__ psa, const double* __restrict__ psb,
    const double* __restrict__ xmsf, const double* __restrict__ qdot, const double* __restrict__ pten,
    const double* __restrict__ ud, const double* __restrict__ vd, const double* __restrict__ msfx,
    const double* __restrict__ xqv, const double* __restrict__ xtv, const double* __restrict__ rpsa,
    const double* __restrict__ tb0, const double* __restrict__ tbt, const int8_t* __restrict__ rgcr,
    const int16_t* __restrict__ ibcr, const double* __restrict__ xkc, const double* __restrict__ tb3d,
    double* tten, double* omegad, double* xkcs_d) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const long p = (long)(k - 1) * g.plane + g.ix(j, i);
  if (!(in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2))) {
    n1t[p] = a1t[p]; n2t[p] = a2t[p];
    if (in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2)) xkcs_d[p] = xkc[p];
    return;
  }
  const int kz = c->kz;
  const double dt = s->dt;
  double td = d_zero + hadv_point(g, c, xt, umc, vmc, psa, xmsf, j, i, k, 1);
  // vadv3d ind = 1 (Main/mod_advection.F90:771-783): pf/pb from psb (mkslice :263-271)
  {
    const double pb = F2(psb, j, i), ptop = c->ptop, c287 = c->c287;
#define PF(K) ((c->sigma[K] * pb + ptop) * d_1000)
#define PB(K) ((c->hsigma[K] * pb + ptop) * d_1000)
#define DQ(K) (F3(qdot, j, i, K) * (c->twt1[K] * F3(a1t, j, i, K) * pow(PF(K) / PB(K), c287) + \
                                  c->twt2[K] * F3(a1t, j, i, (K) - 1) * pow(PF(K) / PB((K) - 1), c287)))
    if (k >= 2) td = td + DQ(k) * c->xds[k];
    if (k + 1 <= kz) td = td - DQ(k + 1) * c->xds[k];
#undef DQ
#undef PB
#undef PF
  }
  // adiabatic (hydrostatic), cpmf = cpd*(1+0.8 qv)
  const double om = omega_at(g, c, qdot, pten, ud, vd, psa, msfx, j, i, k);
  omegad[p] = om;
  {
    const double rovcpm = c->rgas / (c->cpd * (d_one + 0.80 * F3(xqv, j, i, k)));
    td = td + (om * rovcpm * F3(xtv, j, i, k)) / (c->ptop * F2(rpsa, j, i) + c->hsigma[k]);
  }
  // nudge3d
  if (F2(rgcr, j, i) > 0) {
    const double xtb = s->xbctime + dt;
    double xf, xg;
    nudge_coef(c, F2(ibcr, j, i), k, xf, xg);
#define FGT(J, I) ((F3(tb0, J, I, k) + xtb * F3(tbt, J, I, k)) - F3(a2t, J, I, k))
    td = relax(td, xf, xg, FGT(j, i), FGT(j - 1, i), FGT(j + 1, i), FGT(j, i - 1), FGT(j, i + 1));
#undef FGT
  }
  // diffu_x3d with xkc scaled as calc_coeff does (:241-243)
  const double xkcs = xkc[p] * c->rdxsq * F2(psb, j, i);
  xkcs_d[p] = xkcs;
  td = diffu_x_point(g, td, xkcs, tb3d, j, i, k);
  // totals (tphy = 0), forecast, RA filter
  const double tt = ((d_zero + td) + d_zero) + d_zero;
  tten[p] = tt;
  const double t1 = a1t[p], t2 = a2t[p];
  const double ct = t2 + dt * tt;
  const double d = c->gnu1 * (ct + t2 - d_two * t1);
  n2t[p] = t1 + d;
  n1t[p] = ct;
}

// Moisture tendencies and forecast (before the negative-value fix):
// hadvqv + vadvqv + nudge4d3d + diffu_x4d (qv); hadvqx + vadv4d(ind=1) + diffu_x4d (qc)
// (Main/mod_tendency.F90:1361-1392, 1470, 1526, 292-294, 332-349, 375-380).
__global__ __launch_bounds__(256) void k_moisture(
    Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s,
    const double* __restrict__ a1qv, const double* __restrict__ a1qc,
    const double* __restrict__ a2qv, const double* __restrict__ a2qc,
    const double* __restrict__ xqv, const double* __restrict__ xqc, const double* __restrict__ umc,
    const double* __restrict__ vmc, const double* __restrict__ psa, const double* __restrict__ psb,
    const double* __restrict__ xmsf, const double* __restrict__ qdot, const double* __restrict__ qb0,
    const double* __restrict__ qbt, const int8_t* __restrict__ rgcr, const int16_t* __restrict__ ibcr,
    const double* __restrict__ xkc, const double* __restrict__ qvb, const double* __restrict__ qcb,
    double* cqv, double* cqc, double* qvten, double* qcten) {
  THREAD_POINT(g.jce1, g.ice1);
  if (j > g.jce2 || i > g.ice2) return;
  const long p = (long)(k - 1) * g.plane + g.ix(j, i);
  if (!(in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2))) {
    cqv[p] = a2qv[p];
    cqc[p] = a2qc[p];
    return;
  }
  const int kz = c->kz;
  const double dt = s->dt;
  const double ps = F2(psa, j, i);
  // ---- qv
  double tq = d_zero + hadv_point(g, c, xqv, umc, vmc, psa, xmsf, j, i, k, 2);
  {
    const double thr = MINQQ * ps;
#define FGQ(K) ((F3(a1qv, j, i, K) > thr && F3(a1qv, j, i, (K) - 1) > thr) \
                ? F3(a1qv, j, i, K) * pow(F3(a1qv, j, i, (K) - 1) / F3(a1qv, j, i, K), c->qcon[K]) : d_zero)
    if (k >= 2) tq = tq + F3(qdot, j, i, k) * FGQ(k) * c->xds[k];
    if (k + 1 <= kz) tq = tq - F3(qdot, j, i, k + 1) * FGQ(k + 1) * c->xds[k];
#undef FGQ
  }
  if (F2(rgcr, j, i) > 0) {
    const double xtb = s->xbctime + dt;
    const double nfac = 1.0e3, rfac = d_one / nfac;
    double xf, xg;
    nudge_coef(c, F2(ibcr, j, i), k, xf, xg);
#define FGQ(J, I) (nfac * (F3(qb0, J, I, k) + xtb * F3(qbt, J, I, k)) - nfac * F3(a2qv, J, I, k))
    const double f0 = FGQ(j, i), f1 = FGQ(j - 1, i), f2 = FGQ(j + 1, i), f3 = FGQ(j, i - 1), f4 = FGQ(j, i + 1);
#undef FGQ
    tq = tq + rfac * (xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0));
  }
  const double xkcs = xkc[p] * c->rdxsq * F2(psb, j, i);
  tq = diffu_x_point(g, tq, xkcs, qvb, j, i, k);
  // ---- qc
  double tc = d_zero + hadv_point(g, c, xqc, umc, vmc, psa, xmsf, j, i, k, 0);
  {
    const double thr = MINQQ * MINQQ * ps;
#define FGC(K) ((F3(qdot, j, i, K) > d_zero)                                                        \
    ? ((F3(a1qc, j, i, (K) - 1) > thr) ? F3(qdot, j, i, K) * (c->twt1[K] * F3(a1qc, j, i, K) +       \
                                         c->twt2[K] * F3(a1qc, j, i, (K) - 1)) : d_zero)            \
    : ((F3(a1qc, j, i, K) > thr) ? F3(qdot, j, i, K) * (c->twt1[K] * F3(a1qc, j, i, K) +             \
                                   c->twt2[K] * F3(a1qc, j, i, (K) - 1)) : d_zero))
    if (k >= 2) tc = tc + FGC(k) * c->xds[k];
    if (k + 1 <= kz) tc = tc - FGC(k + 1) * c->xds[k];
#undef FGC
  }
  tc = diffu_x_point(g, tc, xkcs, qcb, j, i, k);
  tq = ((d_zero + tq) + d_zero) + d_zero;
  tc = ((d_zero + tc) + d_zero) + d_zero;
  qvten[p] = tq;
  qcten[p] = tc;
  cqv[p] = a2qv[p] + dt * tq;
  cqc[p] = a2qc[p] + dt * tc;
}

// filter_ra_2d on p*, Main/mod_timefilter.F90 (called at Main/mod_tendency.F90:420)
__global__ void k_ps_filter(Geom g, const Consts* __restrict__ c, double* psa, double* psb,
                            const double* __restrict__ psc) {
  THREAD_POINT(g.jci1, g.ici1);
  if (j > g.jci2 || i > g.ici2) return;
  const double d = c->gnu1 * (F2(psc, j, i) + F2(psb, j, i) - d_two * F2(psa, j, i));
  F2(psb, j, i) = F2(psa, j, i) + d;
  F2(psa, j, i) = F2(psc, j, i);
}

// Negative-moisture fix, Main/mod_tendency.F90:382-393.  The reference sweeps each (k,n)
// plane in i-major / j-minor order and a fixed point reads already-fixed predecessors.  A
// negative point whose four predecessors (j-1,i) (j-1,i-1) (j,i-1) (j+1,i-1) inside the
// sweep are all non-negative only ever reads original values and is fixed here in parallel;
// the rare others are flagged and resolved in sweep order by k_negfix_serial.
__device__ __forceinline__ double negfix_sum(const Geom& g, const double* sv, const double* fx, int j, int i, int k,
                                             bool use_fixed) {
  double sum = 0.0;
  for (int ii = i - 1; ii <= i + 1; ii++)
    for (int jj = j - 1; jj <= j + 1; jj++) {
      double v = F3(sv, jj, ii, k);
      if (use_fixed) {
        const bool pred = (ii < i) || (ii == i && jj < j);
        if (pred && in(jj, g.jci1, g.jci2) && in(ii, g.ici1, g.ici2)) v = F3(fx, jj, ii, k);
      }
      sum = sum + fabs(v);
    }
  return 0.01 * sum / 9.0;
}

__global__ void k_negfix(Geom g, int kz, const double* __restrict__ cqv, const double* __restrict__ cqc,
                         double* fqv, double* fqc, uint8_t* dep, int* depplane) {
  THREAD_POINT(g.jci1, g.ici1);
  if (j > g.jci2 || i > g.ici2) return;
  for (int n = 0; n < 2; n++) {
    const double* sv = n ? cqc : cqv;
    double* fx = n ? fqc : fqv;
    const long p = (long)(k - 1) * g.plane + g.ix(j, i);
    const double v = sv[p];
    uint8_t fl = 0;
    double out = v;
    if (v < d_zero) {
      bool negpred = false;
#define NEG(J, I) (in(J, g.jci1, g.jci2) && in(I, g.ici1, g.ici2) && F3(sv, J, I, k) < d_zero)
      negpred = NEG(j - 1, i) || NEG(j - 1, i - 1) || NEG(j, i - 1) || NEG(j + 1, i - 1);
#undef NEG
      if (negpred) {
        fl = 1;
        atomicOr(&depplane[n * kz + (k - 1)], 1);
      } else {
        out = negfix_sum(g, sv, fx, j, i, k, false);
      }
    }
    fx[p] = out;
    dep[(long)n * kz * g.plane + p] = fl;
  }
}

__global__ void k_negfix_serial(Geom g, int kz, const double* __restrict__ cqv, const double* __restrict__ cqc,
                                double* fqv, double* fqc, const uint8_t* __restrict__ dep, int* depplane) {
  const int plane_id = blockIdx.x;          // n*kz + (k-1)
  if (!depplane[plane_id]) return;
  const int n = plane_id / kz, k = plane_id % kz + 1;
  const double* sv = n ? cqc : cqv;
  double* fx = n ? fqc : fqv;
  const uint8_t* dp = dep + (long)n * kz * g.plane;
  for (int i = g.ici1; i <= g.ici2; i++) {
    for (int j0 = g.jci1; j0 <= g.jci2; j0 += 64) {
      const int j = j0 + (int)threadIdx.x;
      const bool flagged = (j <= g.jci2) && dp[(long)(k - 1) * g.plane + g.ix(j, i)];
      unsigned long long mask = __ballot(flagged);
      if (threadIdx.x == 0) {
        while (mask) {
          const int b = __ffsll((long long)mask) - 1;
          mask &= mask - 1;
          const int jj = j0 + b;
          F3(fx, jj, i, k) = negfix_sum(g, sv, fx, jj, i, k, true);
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) depplane[plane_id] = 0;
}

// RAW filter on qv (filter_raw_qv) and qc (filter_raw_4d), Main/mod_timefilter.F90;
// called at Main/mod_tendency.F90:424-427 with the already-filtered psa/psb.
__global__ void k_moisture_filter(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1qv,
                                  const double* __restrict__ a1qc, const double* __restrict__ a2qv,
                                  const double* __restrict__ a2qc, double* n1qv, double* n1qc, double* n2qv,
                                  double* n2qc, const double* __restrict__ fqv, const double* __restrict__ fqc,
                                  const double* __restrict__ psa, const double* __restrict__ psb) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const long p = (long)(k - 1) * g.plane + g.ix(j, i);
  if (!(in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2))) {
    n1qv[p] = a1qv[p]; n1qc[p] = a1qc[p]; n2qv[p] = a2qv[p]; n2qc[p] = a2qc[p];
    return;
  }
  const double beta = 0.53;
  double d = c->gnu1 * (fqv[p] + a2qv[p] - d_two * a1qv[p]);
  n2qv[p] = dmax(a1qv[p] + beta * d, MINQQ * F2(psa, j, i));
  n1qv[p] = dmax(fqv[p] + (beta - d_one) * d, MINQQ * F2(psb, j, i));
  d = c->gnu2 * (fqc[p] + a2qc[p] - d_two * a1qc[p]);
  double m = a1qc[p] + beta * d;
  double q = fqc[p] + (beta - d_one) * d;
  if (m < d_zero) m = d_zero;
  if (q < d_zero) q = d_zero;
  n2qc[p] = m;
  n1qc[p] = q;
}

// ---------------------------------------------------------------------------------------
// splitf projections, Main/mod_split.F90:254-409: one thread per (j,i) column builds deld/delh
// slots 1..3 and refreshes dstor/hstor.  slot(l, s) = base + ((s-1)*nsplit + l-1)*plane.
#define SLOT(a, l, s) ((a) + ((long)((s) - 1) * c->nsplit + ((l) - 1)) * g.plane)
__global__ void k_split_project(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1u,
                                const double* __restrict__ a1v, const double* __restrict__ a2u,
                                const double* __restrict__ a2v, const double* __restrict__ a1t,
                                const double* __restrict__ a2t, const double* __restrict__ psa,
                                const double* __restrict__ psb, const double* __restrict__ msfd,
                                const double* __restrict__ mapf, double* dstor, double* hstor, double* deld,
                                double* delh) {
  const int j = g.jde1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ide1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jde2 || i > g.ide2) return;
  const long q = g.ix(j, i);
  const bool ce = in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
  const double rdx2 = d_one / c->dx2;
  const int kz = c->kz;
  for (int l = 1; l <= c->nsplit; l++) {
    const double ds = dstor[(long)(l - 1) * g.plane + q];
    const double hs = hstor[(long)(l - 1) * g.plane + q];
    double d3 = d_zero, d2 = d_zero, h3 = d_zero, h2 = d_zero;
    if (ce) {
      const double mf = F2(mapf, j, i);
      const double m00 = F2(msfd, j, i), m10 = F2(msfd, j + 1, i), m01 = F2(msfd, j, i + 1), m11 = F2(msfd, j + 1, i + 1);
      for (int k = 1; k <= kz; k++) {
        const double zr = c->zmatxr[l - 1][k - 1];
#define DIV(U, V) (-(F3(U, j, i + 1, k) * m01) + (F3(U, j + 1, i + 1, k) * m11) - (F3(U, j, i, k) * m00) + \
                   (F3(U, j + 1, i, k) * m10) + (F3(V, j, i + 1, k) * m01) + (F3(V, j + 1, i + 1, k) * m11) - \
                   (F3(V, j, i, k) * m00) - (F3(V, j + 1, i, k) * m10))
        d3 = d3 + zr * rdx2 * mf * DIV(a1u, a1v);
        d2 = d2 + zr * rdx2 * mf * DIV(a2u, a2v);
#undef DIV
      }
      const double pa = F2(psa, j, i), pbv = F2(psb, j, i);
      h3 = c->pdlog[l - 1][kz + 1] + c->eps1[l - 1][kz + 1] * (pa - c->pd);
      h2 = c->pdlog[l - 1][kz + 1] + c->eps1[l - 1][kz + 1] * (pbv - c->pd);
      for (int k = 1; k <= kz; k++) {
        const double ta = c->tau[l - 1][k - 1], pdk = c->pdlog[l - 1][k], ek = c->eps1[l - 1][k];
        h3 = h3 + pdk + ta * F3(a1t, j, i, k) / pa + ek * (pa - c->pd);
        h2 = h2 + pdk + ta * F3(a2t, j, i, k) / pbv + ek * (pbv - c->pd);
      }
    }
    SLOT(deld, l, 1)[q] = ds - d2;
    SLOT(deld, l, 2)[q] = d2;
    SLOT(deld, l, 3)[q] = d3 - ds;
    SLOT(delh, l, 1)[q] = hs - h2;
    SLOT(delh, l, 2)[q] = h2;
    SLOT(delh, l, 3)[q] = h3 - hs;
    dstor[(long)(l - 1) * g.plane + q] = d2;
    hstor[(long)(l - 1) * g.plane + q] = h2;
  }
}

// spstep init, Main/mod_split.F90:475-492
__global__ void k_spstep_init(Geom g, const Consts* __restrict__ c, const double* __restrict__ deld,
                              const double* __restrict__ delh, double* ddsum, double* dhsum) {
  const int j = g.jde1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ide1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jde2 || i > g.ide2) return;
  const long q = g.ix(j, i);
  const bool ce = in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
  for (int l = 1; l <= c->nsplit; l++) {
    ddsum[(long)(l - 1) * g.plane + q] = ce ? SLOT(deld, l, 1)[q] : d_zero;
    dhsum[(long)(l - 1) * g.plane + q] = ce ? SLOT(delh, l, 1)[q] : d_zero;
  }
}

// spstep gradient of delh -> (uu, vv), Main/mod_split.F90:498-525
__global__ void k_spstep_grad(Geom g, const Consts* __restrict__ c, int l, int src,
                              const double* __restrict__ delh, const double* __restrict__ msfx,
                              const double* __restrict__ msfd, const double* __restrict__ psdota, double* uu,
                              double* vv) {
  const int j = g.jdi1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.idi1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jdi2 || i > g.idi2) return;
  const double* x = SLOT(delh, l, src);
  const double fac = c->dx2 * F2(msfx, j, i);
  double w1 = (F2(x, j, i) + F2(x, j, i - 1) - F2(x, j - 1, i) - F2(x, j - 1, i - 1)) / fac;
  double w2 = (F2(x, j, i) + F2(x, j - 1, i) - F2(x, j, i - 1) - F2(x, j - 1, i - 1)) / fac;
  w1 = w1 * F2(psdota, j, i);
  w2 = w2 * F2(psdota, j, i);
  F2(uu, j, i) = w1 * F2(msfd, j, i);
  F2(vv, j, i) = w2 * F2(msfd, j, i);
}

// spstep divergence + mode update + boundary extrapolation + sums, Main/mod_split.F90:530-573
// (forward step, leap = 0) and :614-658 (leapfrog, leap = 1).
__global__ void k_spstep_update(Geom g, const Consts* __restrict__ c, int l, int n0, int n1, int nn, int leap,
                                const double* __restrict__ uu, const double* __restrict__ vv,
                                const double* __restrict__ mapf, const double* __restrict__ psa, double* deld,
                                double* delh, double* ddsum, double* dhsum) {
  const int j = g.jce1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ice1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  if (j > g.jce2 || i > g.ice2) return;
  const long q = g.ix(j, i);
  double* D0 = SLOT(deld, l, n0); double* D1 = SLOT(deld, l, n1); double* DN = SLOT(deld, l, nn);
  double* H0 = SLOT(delh, l, n0); double* H1 = SLOT(delh, l, n1); double* HN = SLOT(delh, l, nn);
  const double* D3 = SLOT(deld, l, 3); const double* H3 = SLOT(delh, l, 3);
  const double aam = c->aam[l - 1], dtau = c->dtau[l - 1], hbar = c->hbar[l - 1];
  const bool ci = in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2);
  if (ci) {
    const double rdx2 = d_one / c->dx2;
    const double w3 = rdx2 * F2(mapf, j, i) *
        (-F2(uu, j, i + 1) + F2(uu, j + 1, i + 1) - F2(uu, j, i) + F2(uu, j + 1, i) +
         F2(vv, j, i + 1) + F2(vv, j + 1, i + 1) - F2(vv, j, i) - F2(vv, j + 1, i));
    if (!leap) {
      const double m2 = (double)((int)aam * 2);
      DN[q] = D0[q] - dtau * w3 + D3[q] / m2;
      HN[q] = H0[q] - dtau * hbar * D0[q] / F2(psa, j, i) + H3[q] / m2;
    } else {
      const double dtau2 = dtau * d_two;
      DN[q] = D0[q] - dtau2 * w3 + D3[q] / aam;
      HN[q] = H0[q] - dtau2 * hbar * D1[q] / F2(psa, j, i) + H3[q] / aam;
    }
  } else {
    bool bnd = (g.bl && j == g.jce1 && in(i, g.ici1, g.ici2)) || (g.br && j == g.jce2 && in(i, g.ici1, g.ici2)) ||
               (g.bb && i == g.ice1) || (g.bt && i == g.ice2);
    if (bnd) {
      if (!leap) HN[q] = H0[q] * ((aam - d_one) / aam);
      else HN[q] = d_two * H1[q] - H0[q];
    }
  }
  ddsum[(long)(l - 1) * g.plane + q] = ddsum[(long)(l - 1) * g.plane + q] + DN[q];
  dhsum[(long)(l - 1) * g.plane + q] = dhsum[(long)(l - 1) * g.plane + q] + HN[q];
}

// spstep fused, single-tile: every sub-step of one vertical mode in one launch (blockIdx.z =
// mode).  A workgroup owns SPB x SPB cross points plus a SPH-point halo held in LDS; each
// sub-step couples delh only within radius 1, so after m2 <= SPH sub-steps the owned block is
// exact (halo values are recomputed redundantly and the contaminated rim never reaches it).
// Per point the operations are those of k_spstep_grad/k_spstep_update, so results are
// bit-identical to the two-kernel-per-substep path (Main/mod_split.F90:463-669).
constexpr int SPR = SPB + 2 * SPH, SPP = SPR + 1;
__global__ __launch_bounds__(256) void k_spstep_fused(
    Geom g, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh,
    const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota,
    const double* __restrict__ mapf, const double* __restrict__ psa, double* ddsum, double* dhsum) {
  __shared__ double Ds[2][SPR][SPP], Hs[2][SPR][SPP], U[SPR][SPP], V[SPR][SPP];
  const int l = blockIdx.z + 1;
  const int J1 = g.jce1 + blockIdx.x * SPB, I1 = g.ice1 + blockIdx.y * SPB;
  const int jr0 = J1 - SPH, ir0 = I1 - SPH;          // region origin (global)
  const int tx = threadIdx.x, ty = threadIdx.y;        // 32 x 8
  const double aam = c->aam[l - 1], dtau = c->dtau[l - 1], hbar = c->hbar[l - 1];
  const int m2 = (int)aam * 2;
  const double dtau2 = dtau * d_two, rdx2 = d_one / c->dx2;
  const double* D1 = SLOT(deld, l, 1); const double* D2 = SLOT(deld, l, 2); const double* D3 = SLOT(deld, l, 3);
  const double* H1 = SLOT(delh, l, 1); const double* H2 = SLOT(delh, l, 2); const double* H3 = SLOT(delh, l, 3);
  // per-thread points: (tx, ty + 8 r), r = 0..3
  double d3[4], h3[4], ps[4], mf[4], ufac[4], msd[4], sd[4], sh[4];
  bool ce[4], ci[4], bnd[4], di[4], own[4];
  for (int r = 0; r < 4; r++) {
    const int lj = tx, li = ty + 8 * r, j = jr0 + lj, i = ir0 + li;
    ce[r] = in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
    ci[r] = in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2);
    di[r] = in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2);
    bnd[r] = ce[r] && !ci[r] &&
             ((g.bl && j == g.jce1 && in(i, g.ici1, g.ici2)) || (g.br && j == g.jce2 && in(i, g.ici1, g.ici2)) ||
              (g.bb && i == g.ice1) || (g.bt && i == g.ice2));
    own[r] = in(j, J1, J1 + SPB - 1) && in(i, I1, I1 + SPB - 1);
    const long q = ce[r] ? g.ix(j, i) : 0;
    Ds[0][li][lj] = ce[r] ? D1[q] : 0.0; Ds[1][li][lj] = ce[r] ? D2[q] : 0.0;
    Hs[0][li][lj] = ce[r] ? H1[q] : 0.0; Hs[1][li][lj] = ce[r] ? H2[q] : 0.0;
    U[li][lj] = 0.0; V[li][lj] = 0.0;
    d3[r] = ce[r] ? D3[q] : 0.0; h3[r] = ce[r] ? H3[q] : 0.0;
    ps[r] = ci[r] ? F2(psa, j, i) : 1.0;
    mf[r] = ci[r] ? F2(mapf, j, i) : 0.0;
    ufac[r] = di[r] ? c->dx2 * F2(msfx, j, i) : 1.0;
    msd[r] = di[r] ? F2(msfd, j, i) : 0.0;
    sd[r] = ce[r] ? Ds[0][li][lj] : 0.0;     // ddsum(ce) = deld(n0)
    sh[r] = ce[r] ? Hs[0][li][lj] : 0.0;
  }
  double pda[4];
  for (int r = 0; r < 4; r++) {
    const int j = jr0 + tx, i = ir0 + ty + 8 * r;
    pda[r] = di[r] ? F2(psdota, j, i) : 0.0;
  }
  __syncthreads();
  int n0 = 0, n1 = 1;                                   // slot indices (reference slots 1, 2)
  for (int n = 1; n <= m2; n++) {
    const int src = (n == 1) ? n0 : n1;
    // gradient of delh(src) at dot points -> (uu, vv)
    for (int r = 0; r < 4; r++) {
      const int lj = tx, li = ty + 8 * r;
      if (di[r] && lj >= 1 && li >= 1) {
        const double a = Hs[src][li][lj], b = Hs[src][li - 1][lj], cc = Hs[src][li][lj - 1], dd = Hs[src][li - 1][lj - 1];
        double w1 = (a + b - cc - dd) / ufac[r];
        double w2 = (a + cc - b - dd) / ufac[r];
        w1 = w1 * pda[r];
        w2 = w2 * pda[r];
        U[li][lj] = w1 * msd[r];
        V[li][lj] = w2 * msd[r];
      }
    }
    __syncthreads();
    const int nn = (n == 1) ? n1 : n0;                  // forward writes n1; leapfrog n2 = n0
    for (int r = 0; r < 4; r++) {
      const int lj = tx, li = ty + 8 * r;
      if (ci[r] && lj + 1 < SPR && li + 1 < SPR) {
        const double w3 = rdx2 * mf[r] *
            (-U[li + 1][lj] + U[li + 1][lj + 1] - U[li][lj] + U[li][lj + 1] +
             V[li + 1][lj] + V[li + 1][lj + 1] - V[li][lj] - V[li][lj + 1]);
        if (n == 1) {
          const double m2d = (double)m2;
          const double dn = Ds[n0][li][lj] - dtau * w3 + d3[r] / m2d;
          const double hn = Hs[n0][li][lj] - dtau * hbar * Ds[n0][li][lj] / ps[r] + h3[r] / m2d;
          Ds[nn][li][lj] = dn;
          Hs[nn][li][lj] = hn;
        } else {
          const double dn = Ds[n0][li][lj] - dtau2 * w3 + d3[r] / aam;
          const double hn = Hs[n0][li][lj] - dtau2 * hbar * Ds[n1][li][lj] / ps[r] + h3[r] / aam;
          Ds[nn][li][lj] = dn;
          Hs[nn][li][lj] = hn;
        }
      } else if (bnd[r]) {
        if (n == 1) Hs[nn][li][lj] = Hs[n0][li][lj] * ((aam - d_one) / aam);
        else Hs[nn][li][lj] = d_two * Hs[n1][li][lj] - Hs[n0][li][lj];
      }
      if (ce[r]) {
        sd[r] = sd[r] + Ds[nn][li][lj];
        sh[r] = sh[r] + Hs[nn][li][lj];
      }
    }
    __syncthreads();
    if (n >= 2) { const int t0 = n0; n0 = n1; n1 = t0; }
    else { /* forward step: n0 = 1, n1 = 2 stay; the leapfrog loop starts with n2 = n0 */ }
  }
  for (int r = 0; r < 4; r++) {
    const int j = jr0 + tx, i = ir0 + ty + 8 * r;
    if (own[r] && in(j, g.jde1, g.jde2) && in(i, g.ide1, g.ide2)) {
      const long q = (long)(l - 1) * g.plane + g.ix(j, i);
      ddsum[q] = ce[r] ? sd[r] : d_zero;
      dhsum[q] = ce[r] ? sh[r] : d_zero;
    }
  }
}

// splitf corrections, Main/mod_split.F90:417-457 (ps and t on ci, u and v on di)
__global__ void k_split_correct(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum,
                                const double* __restrict__ dhsum, const double* __restrict__ psdota,
                                const double* __restrict__ msfd, double* psa, double* psb, double* a1t,
                                double* a2t, double* a1u, double* a1v, double* a2u, double* a2v) {
  THREAD_POINT(g.jde1, g.ide1);
  if (j > g.jde2 || i > g.ide2) return;
  const long q = g.ix(j, i);
  const long p = (long)(k - 1) * g.plane + q;
  const double gnu1 = c->gnu1;
  const int ns = c->nsplit;
  if (in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2)) {
    if (k == 1) {
      double pa = psa[q], pb = psb[q];
      for (int l = 1; l <= ns; l++) {
        const double an = c->an[l - 1], dd = ddsum[(long)(l - 1) * g.plane + q];
        pa = pa - an * dd;
        pb = pb - gnu1 * an * dd;
      }
      psa[q] = pa; psb[q] = pb;
    }
    double t1 = a1t[p], t2 = a2t[p];
    for (int l = 1; l <= ns; l++) {
      const double am = c->am[l - 1][k - 1], dd = ddsum[(long)(l - 1) * g.plane + q];
      t1 = t1 + am * dd;
      t2 = t2 + gnu1 * am * dd;
    }
    a1t[p] = t1; a2t[p] = t2;
  }
  if (in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2)) {
    double u1 = a1u[p], v1 = a1v[p], u2 = a2u[p], v2 = a2v[p];
    const double fac = F2(psdota, j, i) / (c->dx2 * F2(msfd, j, i));
    for (int l = 1; l <= ns; l++) {
      const double* dh = dhsum + (long)(l - 1) * g.plane;
      const double zm = c->zmatx[l - 1][k - 1], gnuzm = gnu1 * zm;
      const double x = fac * (F2(dh, j, i) + F2(dh, j, i - 1) - F2(dh, j - 1, i) - F2(dh, j - 1, i - 1));
      const double y = fac * (F2(dh, j, i) - F2(dh, j, i - 1) + F2(dh, j - 1, i) - F2(dh, j - 1, i - 1));
      u1 = u1 - zm * x; v1 = v1 - zm * y; u2 = u2 - gnuzm * x; v2 = v2 - gnuzm * y;
    }
    a1u[p] = u1; a1v[p] = v1; a2u[p] = u2; a2v[p] = v2;
  }
}
#undef SLOT

// rcmtimer%advance + dt switch, Main/mod_tendency.F90:608-616
__global__ void k_advance_time(StepState* s, double dtsec) {
  s->lcount = s->lcount + 1;
  if (s->lcount == 2) s->dt = d_two * dtsec;
}

// ---------------------------------------------------------------------------------------
// bdyval, Main/mod_bdycod.F90:1109-1529 (+ bdyuv :896-1061).  Slice order:
// 0 wue 1 wui 2 eue 3 eui 4 wve 5 wvi 6 eve 7 evi (by i) / 8 sue 9 sui 10 nue 11 nui
// 12 sve 13 svi 14 nve 15 nvi (by j).


__global__ void k_bdyval_set(Geom g, const StepState* __restrict__ s, double* a1u, double* a1v, double* a1t,
                             double* a1qv, double* a1qc, double* a2u, double* a2v, double* a2t, double* a2qv,
                             double* a2qc, double* psa, double* psb, const double* __restrict__ ub0,
                             const double* __restrict__ ubt, const double* __restrict__ vb0,
                             const double* __restrict__ vbt, const double* __restrict__ tb0,
                             const double* __restrict__ tbt, const double* __restrict__ qb0,
                             const double* __restrict__ qbt, const double* __restrict__ pb0,
                             const double* __restrict__ pbt, Slices sl, long slen) {
  THREAD_POINT(g.jde1, g.ide1);
  if (j > g.jde2 || i > g.ide2) return;
  const long q = g.ix(j, i);
  const long p = (long)(k - 1) * g.plane + q;
  const double xt = s->xbctime + s->dt;
  const bool integ = s->lcount > 0;
  // dot-point boundary rows: left/right on idi, bottom/top on the whole jde range
  const bool dL = g.bl && j == g.jde1 && in(i, g.idi1, g.idi2);
  const bool dR = g.br && j == g.jde2 && in(i, g.idi1, g.idi2);
  const bool dB = g.bb && i == g.ide1;
  const bool dT = g.bt && i == g.ide2;
  if (dL || dR || dB || dT) {
    if (integ) { a2u[p] = a1u[p]; a2v[p] = a1v[p]; }
    a1u[p] = ub0[p] + xt * ubt[p];
    a1v[p] = vb0[p] + xt * vbt[p];
  }
  // cross-point boundary rows: left/right on ici, bottom/top on the jce range
  const bool cL = g.bl && j == g.jce1 && in(i, g.ici1, g.ici2);
  const bool cR = g.br && j == g.jce2 && in(i, g.ici1, g.ici2);
  const bool cB = g.bb && i == g.ice1 && in(j, g.jce1, g.jce2);
  const bool cT = g.bt && i == g.ice2 && in(j, g.jce1, g.jce2);
  if (cL || cR || cB || cT) {
    if (integ) {
      a2t[p] = a1t[p]; a2qv[p] = a1qv[p]; a2qc[p] = a1qc[p];
      if (k == 1) psb[q] = psa[q];
    }
    if (k == 1) psa[q] = pb0[q] + xt * pbt[q];
    a1t[p] = tb0[p] + xt * tbt[p];
    a1qv[p] = qb0[p] + xt * qbt[p];
  }
  // bdyuv slices (interior slice values are interior points: not modified above)
  if (g.bl && j == g.jde1 && in(i, g.idi1, g.idi2)) {
    SLI(sl.s[1], i, k) = F3(a1u, g.jdi1, i, k); SLI(sl.s[5], i, k) = F3(a1v, g.jdi1, i, k);
    SLI(sl.s[0], i, k) = ub0[p] + xt * ubt[p]; SLI(sl.s[4], i, k) = vb0[p] + xt * vbt[p];
  }
  if (g.br && j == g.jde2 && in(i, g.idi1, g.idi2)) {
    SLI(sl.s[3], i, k) = F3(a1u, g.jdi2, i, k); SLI(sl.s[7], i, k) = F3(a1v, g.jdi2, i, k);
    SLI(sl.s[2], i, k) = ub0[p] + xt * ubt[p]; SLI(sl.s[6], i, k) = vb0[p] + xt * vbt[p];
  }
  if (g.bb && i == g.ide1) {
    if (in(j, g.jdi1, g.jdi2)) { SLJ(sl.s[9], j, k) = F3(a1u, j, g.idi1, k); SLJ(sl.s[13], j, k) = F3(a1v, j, g.idi1, k); }
    SLJ(sl.s[8], j, k) = ub0[p] + xt * ubt[p]; SLJ(sl.s[12], j, k) = vb0[p] + xt * vbt[p];
  }
  if (g.bt && i == g.ide2) {
    if (in(j, g.jdi1, g.jdi2)) { SLJ(sl.s[11], j, k) = F3(a1u, j, g.idi2, k); SLJ(sl.s[15], j, k) = F3(a1v, j, g.idi2, k); }
    SLJ(sl.s[10], j, k) = ub0[p] + xt * ubt[p]; SLJ(sl.s[14], j, k) = vb0[p] + xt * vbt[p];
  }
}

// bdyuv corner fills, Main/mod_bdycod.F90:1030-1061
__global__ void k_bdyval_corners(Geom g, int kz, Slices sl, long slen) {
  const int k = 1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k > kz) return;
  if (g.bt && g.bl) {
    SLI(sl.s[1], g.ide2, k) = SLJ(sl.s[10], g.jdi1, k); SLI(sl.s[5], g.ide2, k) = SLJ(sl.s[14], g.jdi1, k);
    SLJ(sl.s[11], g.jde1, k) = SLI(sl.s[0], g.idi2, k); SLJ(sl.s[15], g.jde1, k) = SLI(sl.s[4], g.idi2, k);
  }
  if (g.bb && g.bl) {
    SLI(sl.s[1], g.ide1, k) = SLJ(sl.s[8], g.jdi1, k); SLI(sl.s[5], g.ide1, k) = SLJ(sl.s[12], g.jdi1, k);
    SLJ(sl.s[9], g.jde1, k) = SLI(sl.s[0], g.idi1, k); SLJ(sl.s[13], g.jde1, k) = SLI(sl.s[4], g.idi1, k);
  }
  if (g.bt && g.br) {
    SLI(sl.s[3], g.ide2, k) = SLJ(sl.s[10], g.jdi2, k); SLI(sl.s[7], g.ide2, k) = SLJ(sl.s[14], g.jdi2, k);
    SLJ(sl.s[11], g.jde2, k) = SLI(sl.s[2], g.idi2, k); SLJ(sl.s[15], g.jde2, k) = SLI(sl.s[6], g.idi2, k);
  }
  if (g.bb && g.br) {
    SLI(sl.s[3], g.ide1, k) = SLJ(sl.s[8], g.jdi2, k); SLI(sl.s[7], g.ide1, k) = SLJ(sl.s[12], g.jdi2, k);
    SLJ(sl.s[9], g.jde2, k) = SLI(sl.s[2], g.idi1, k); SLJ(sl.s[13], g.jde2, k) = SLI(sl.s[6], g.idi1, k);
  }
}

// qc inflow/outflow (present_qc = .false., bdyflow), Main/mod_bdycod.F90:2153-2220.
// west/east first (they read qc(jci1|jci2, ice1|ice2) before south/north rewrite it).
__global__ void k_bdyval_qc_we(Geom g, int kz, double* a1qc, const double* __restrict__ psa, Slices sl, long slen) {
  const int i = g.ice1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int k = 1 + (int)blockIdx.y;
  if (i > g.ice2) return;
  if (g.bl) {
    const double qxint = F3(a1qc, g.jci1, i, k) / F2(psa, g.jci1, i);
    const double w = SLI(sl.s[0], i, k) + SLI(sl.s[0], i + 1, k) + SLI(sl.s[1], i, k) + SLI(sl.s[1], i + 1, k);
    F3(a1qc, g.jce1, i, k) = (w > d_zero) ? d_zero : qxint * F2(psa, g.jce1, i);
  }
  if (g.br) {
    const double qxint = F3(a1qc, g.jci2, i, k) / F2(psa, g.jci2, i);
    const double w = SLI(sl.s[2], i, k) + SLI(sl.s[2], i + 1, k) + SLI(sl.s[3], i, k) + SLI(sl.s[3], i + 1, k);
    F3(a1qc, g.jce2, i, k) = (w < d_zero) ? d_zero : qxint * F2(psa, g.jce2, i);
  }
}

__global__ void k_bdyval_qc_sn(Geom g, int kz, double* a1qc, const double* __restrict__ psa, Slices sl, long slen) {
  const int j = g.jci1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int k = 1 + (int)blockIdx.y;
  if (j > g.jci2) return;
  if (g.bb) {
    const double qxint = F3(a1qc, j, g.ici1, k) / F2(psa, j, g.ici1);
    const double w = SLJ(sl.s[12], j, k) + SLJ(sl.s[12], j + 1, k) + SLJ(sl.s[13], j, k) + SLJ(sl.s[13], j + 1, k);
    F3(a1qc, j, g.ice1, k) = (w > d_zero) ? d_zero : qxint * F2(psa, j, g.ice1);
  }
  if (g.bt) {
    const double qxint = F3(a1qc, j, g.ici2, k) / F2(psa, j, g.ici2);
    const double w = SLJ(sl.s[14], j, k) + SLJ(sl.s[14], j + 1, k) + SLJ(sl.s[15], j, k) + SLJ(sl.s[15], j + 1, k);
    F3(a1qc, j, g.ice2, k) = (w < d_zero) ? d_zero : qxint * F2(psa, j, g.ice2);
  }
}

__global__ void k_bdyval_time(StepState* s, double dtsec) { s->xbctime = s->xbctime + dtsec; }

// ---------------------------------------------------------------------------------------
// static derived fields: Main/mod_params.F90:1993-2001 (xmsf, dmsf), Main/mod_diffusion.F90:
// 124-140 (hgfact), Main/mod_split.F90:99-101 (map)
__global__ void k_prepare_static(Geom g, const Consts* __restrict__ c, int diffu_hgtf,
                                 const double* __restrict__ msfx, const double* __restrict__ msfd,
                                 const double* __restrict__ ht, double* xmsf, double* dmsf, double* hgfact,
                                 double* mapf) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  if (in(j, g.jdi1, g.jdi2) && in(i, g.idi1, g.idi2)) {
    F2(dmsf, j, i) = d_one / (F2(msfd, j, i) * F2(msfd, j, i) * c->dx16);
    F2(xmsf, j, i) = d_one / (F2(msfx, j, i) * F2(msfx, j, i) * c->dx4);
  }
  if (in(j, g.jce1ga, g.jce2ga) && in(i, g.ice1ga, g.ice2ga)) {
    double hv = c->xkhz;
    if (diffu_hgtf == 1 && in(j, g.jci1ga, g.jci2ga) && in(i, g.ici1ga, g.ici2ga)) {
      const double h = F2(ht, j, i);
      const double hg1 = fabs((h - F2(ht, j, i - 1)) / c->dx);
      const double hg2 = fabs((h - F2(ht, j, i + 1)) / c->dx);
      const double hg3 = fabs((h - F2(ht, j - 1, i)) / c->dx);
      const double hg4 = fabs((h - F2(ht, j + 1, i)) / c->dx);
      const double hgmax = dmax(dmax(dmax(hg1, hg2), hg3), hg4) * c->regrav * 1.0e3;
      hv = c->xkhz / (d_one + hgmax * hgmax);
    }
    F2(hgfact, j, i) = hv;
  }
  if (in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2)) F2(mapf, j, i) = d_one / (F2(msfx, j, i) * F2(msfx, j, i));
}

// ---------------------------------------------------------------------------------------
// Halo staging: pack owned edge boxes / unpack ghost boxes of several fields in one launch.
// A segment addresses p + (k-1)*kstride + (i-i0)*pitch + (j-j0) over a box of nk levels and
// lands at buf[off + ((k-1)*ni + (i-i1))*nj + (j-j1)].  Used by every exchange, whether the
// peer tile is on this device (device copy) or on another rank (RCCL).
__global__ void k_pack_segs(SegList L, double* __restrict__ buf, int unpack) {
  const Seg sg = L.s[blockIdx.y];
  const int nj = sg.j2 - sg.j1 + 1, ni = sg.i2 - sg.i1 + 1;
  const long n = (long)nj * ni * sg.nk;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int j = sg.j1 + (int)(q % nj);
    const int i = sg.i1 + (int)((q / nj) % ni);
    const int k = (int)(q / ((long)nj * ni));
    double* a = sg.p + (long)k * sg.kstride + (long)(i - sg.i0) * sg.pitch + (j - sg.j0);
    if (unpack) *a = buf[sg.off + q];
    else buf[sg.off + q] = *a;
  }
}

}  // namespace rcm
