// qxcommon.hpp -- device helpers of the moisture species shared by the qv/qc kernels
// (kernels.hip) and the hydrometeors of nqx = 5 (species.hip): the upstream flux form, the
// negative-moisture fix, the RAW filters and bdyval's hydrometeor inflow/outflow lines.
#pragma once
#include "kernels.hpp"
#include "devcommon.hpp"

namespace rcm {

// negative-moisture fix helpers (K6 below)
__device__ __forceinline__ double negfix_sum(const Geom& g, const double* sv, const double* fx, int j, int i, int k,
                                             bool use_fixed) {
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

__device__ __forceinline__ bool negfix_dependent(const Geom& g, const double* sv, int j, int i, int k) {
#define NEG(J, I) (in(J, g.jci1, g.jci2) && in(I, g.ici1, g.ici2) && F3(sv, J, I, k) < d_zero)
  return NEG(j - 1, i) || NEG(j - 1, i - 1) || NEG(j, i - 1) || NEG(j + 1, i - 1);
#undef NEG
}

// RAW filters of one point (filter_raw_qv / filter_raw_4d) with the filtered p*
__device__ __forceinline__ void raw_filter(const Consts* c, int n, double fq, double o1, double o2v, double pa,
                                           double pb, double& n1, double& n2) {
  const double beta = 0.53;
  if (n == 0) {
    const double d = c->gnu1 * (fq + o2v - d_two * o1);
    n2 = dmax(o1 + beta * d, MINQQ * pa);
    n1 = dmax(fq + (beta - d_one) * d, MINQQ * pb);
  } else {
    const double d = c->gnu2 * (fq + o2v - d_two * o1);
    double m = o1 + beta * d;
    double q = fq + (beta - d_one) * d;
    if (m < d_zero) m = d_zero;
    if (q < d_zero) q = d_zero;
    n2 = m;
    n1 = q;
  }
}

// upstream flux-form advection of one scalar (hadvt/hadvqv/hadvqx, Main/mod_advection.F90:
// 337-386, 547-596, 639-653); limiter 0 none, 1 t_extrema, 2 q_rel_extrema
__device__ __forceinline__ double hadv_flux(const Consts* c, double xm, double ps, double uavg1, double uavg2,
                                            double vavg1, double vavg2, double fc, double fw, double fe, double fs,
                                            double fn, int limiter) {
  const double ul = c->ul;
  const double f1 = d_half * ul * (uavg2 + uavg1) / ps;
  const double f2 = d_half * ul * (vavg2 + vavg1) / ps;
  const double fx1 = (d_one + f1) * fw + (d_one - f1) * fc;
  const double fx2 = (d_one + f1) * fc + (d_one - f1) * fe;
  const double fy1 = (d_one + f2) * fs + (d_one - f2) * fc;
  const double fy2 = (d_one + f2) * fc + (d_one - f2) * fn;
  double fg = -xm * (uavg2 * fx2 - uavg1 * fx1 + vavg2 * fy2 - vavg1 * fy1);
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

// qc inflow/outflow (present_qc = .false., bdyflow), Main/mod_bdycod.F90:2153-2220, one
// block per level: west/east first (they read qc(jci1|jci2, ice1|ice2) before south/north
// rewrite it), then south/north.  The last tile's launch also advances the boundary clock
// xbctime += dtsec (Main/mod_bdycod.F90:2566): nothing here reads it.
template <class PS>
__device__ void bdyval_qc_level(const Geom& g, int do_qc, int do_qv, double* a1qc, double* a1qv, PS ps, const Slices& sl,
                                long slen, int k) {
  if (do_qv) {
    // qv inflow/outflow for iboudy = 3 or 4, Main/mod_bdycod.F90:1809-1950: west/east on ici,
    // then south/north on jce (reading the west/east results at the corners)
    for (int i = g.ici1 + (int)threadIdx.x; i <= g.ici2; i += (int)blockDim.x) {
      if (g.bl) {
        const double qext = F3(a1qv, g.jce1, i, k) / ps(g.jce1, i);
        const double qint = F3(a1qv, g.jci1, i, k) / ps(g.jci1, i);
        const double w = SLI(sl.s[0], i, k) + SLI(sl.s[0], i + 1, k) + SLI(sl.s[1], i, k) + SLI(sl.s[1], i + 1, k);
        F3(a1qv, g.jce1, i, k) = (w > d_zero) ? qext * ps(g.jce1, i) : qint * ps(g.jce1, i);
      }
      if (g.br) {
        const double qext = F3(a1qv, g.jce2, i, k) / ps(g.jce2, i);
        const double qint = F3(a1qv, g.jci2, i, k) / ps(g.jci2, i);
        const double w = SLI(sl.s[2], i, k) + SLI(sl.s[2], i + 1, k) + SLI(sl.s[3], i, k) + SLI(sl.s[3], i + 1, k);
        F3(a1qv, g.jce2, i, k) = (w < d_zero) ? qext * ps(g.jce2, i) : qint * ps(g.jce2, i);
      }
    }
    __syncthreads();
    for (int j = g.jce1 + (int)threadIdx.x; j <= g.jce2; j += (int)blockDim.x) {
      if (g.bb) {
        const double qext = F3(a1qv, j, g.ice1, k) / ps(j, g.ice1);
        const double qint = F3(a1qv, j, g.ici1, k) / ps(j, g.ici1);
        const double w = SLJ(sl.s[12], j, k) + SLJ(sl.s[12], j + 1, k) + SLJ(sl.s[13], j, k) + SLJ(sl.s[13], j + 1, k);
        F3(a1qv, j, g.ice1, k) = (w > d_zero) ? qext * ps(j, g.ice1) : qint * ps(j, g.ice1);
      }
      if (g.bt) {
        const double qext = F3(a1qv, j, g.ice2, k) / ps(j, g.ice2);
        const double qint = F3(a1qv, j, g.ici2, k) / ps(j, g.ici2);
        const double w = SLJ(sl.s[14], j, k) + SLJ(sl.s[14], j + 1, k) + SLJ(sl.s[15], j, k) + SLJ(sl.s[15], j + 1, k);
        F3(a1qv, j, g.ice2, k) = (w < d_zero) ? qext * ps(j, g.ice2) : qint * ps(j, g.ice2);
      }
    }
    __syncthreads();
  }
  if (!do_qc) return;
  // The west/east pass reads the interior columns jci1/jci2 on rows ice1..ice2 before the
  // south/north pass rewrites rows ice1/ice2 on jci1..jci2: the two passes share exactly the
  // four points (jci1|jci2, ice1|ice2), which are read here before any write.  Otherwise the
  // passes are independent (west/east writes columns jce1/jce2, which south/north never reads;
  // south/north reads rows ici1/ici2, which nothing writes), so every chunk of the loop below
  // may write as soon as it has read, whatever the tile's extent.
  const double c11 = F3(a1qc, g.jci1, g.ice1, k), c12 = F3(a1qc, g.jci1, g.ice2, k);
  const double c21 = F3(a1qc, g.jci2, g.ice1, k), c22 = F3(a1qc, g.jci2, g.ice2, k);
  __syncthreads();
  auto qcw = [&](int jc, int i) {
    if (i == g.ice1) return jc == g.jci1 ? c11 : c21;
    if (i == g.ice2) return jc == g.jci1 ? c12 : c22;
    return F3(a1qc, jc, i, k);
  };
  const int ni = g.ice2 - g.ice1 + 1, nj = g.jci2 - g.jci1 + 1, nx = max(ni, nj);
  for (int base = 0; base < nx; base += (int)blockDim.x) {
    const int x = base + (int)threadIdx.x;
    const int i = g.ice1 + x, j = g.jci1 + x;
    const bool wi = x < ni, sj = x < nj;
    double vw = 0.0, ve = 0.0, vs = 0.0, vn = 0.0;
    bool ow = false, oe = false, os = false, on = false;
    if (wi && g.bl) {
      const double qxint = qcw(g.jci1, i) / ps(g.jci1, i);
      const double w = SLI(sl.s[0], i, k) + SLI(sl.s[0], i + 1, k) + SLI(sl.s[1], i, k) + SLI(sl.s[1], i + 1, k);
      vw = (w > d_zero) ? d_zero : qxint * ps(g.jce1, i);
      ow = true;
    }
    if (wi && g.br) {
      const double qxint = qcw(g.jci2, i) / ps(g.jci2, i);
      const double w = SLI(sl.s[2], i, k) + SLI(sl.s[2], i + 1, k) + SLI(sl.s[3], i, k) + SLI(sl.s[3], i + 1, k);
      ve = (w < d_zero) ? d_zero : qxint * ps(g.jce2, i);
      oe = true;
    }
    if (sj && g.bb) {
      const double qxint = F3(a1qc, j, g.ici1, k) / ps(j, g.ici1);
      const double w = SLJ(sl.s[12], j, k) + SLJ(sl.s[12], j + 1, k) + SLJ(sl.s[13], j, k) + SLJ(sl.s[13], j + 1, k);
      vs = (w > d_zero) ? d_zero : qxint * ps(j, g.ice1);
      os = true;
    }
    if (sj && g.bt) {
      const double qxint = F3(a1qc, j, g.ici2, k) / ps(j, g.ici2);
      const double w = SLJ(sl.s[14], j, k) + SLJ(sl.s[14], j + 1, k) + SLJ(sl.s[15], j, k) + SLJ(sl.s[15], j + 1, k);
      vn = (w < d_zero) ? d_zero : qxint * ps(j, g.ice2);
      on = true;
    }
    if (ow) F3(a1qc, g.jce1, i, k) = vw;
    if (oe) F3(a1qc, g.jce2, i, k) = ve;
    if (os) F3(a1qc, j, g.ice1, k) = vs;
    if (on) F3(a1qc, j, g.ice2, k) = vn;
  }
}

}  // namespace rcm
