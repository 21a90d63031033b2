// kernels.hip -- HIP/CDNA4 kernels of the hydrostatic dynamical-core step (gfx950).
//
// Every kernel evaluates each output element with the same floating-point operation
// sequence as the reference loop nests it fuses (see oracle/rcm_oracle.c for the literal
// restatement and the Main/*.F90 file:line citations repeated below).  Contributions that the
// reference accumulates into one tendency element in several passes are accumulated here in
// the same order inside one thread, so transcendental-free results are bit-identical
// (compiled with -ffp-contract=off).
//
// The reference materialises decoupled copies of the state (decouple: umc, vmc, ud, vd, t,
// qv, qc, tv; mkslice: ubd3d, vbd3d, tb3d, qxb3d).  Each is one product of a state field with
// a 2-D factor, so the kernels here recompute them where they are read (the same product,
// hence the same bits) and only the 2-D reciprocals are stored: 13 3-D fields of HBM traffic
// and two launches per step disappear.
//
// Thread mapping: x -> j (west-east, unit stride, coalesced), y -> i, z -> k; blocks of
// 64 x 4.  All fields of a tile share one frame, so a point's 32-bit byte offset (plus
// shared neighbour offsets) addresses every field: loads are SGPR base + VGPR offset.
// Column recurrences (pten/qdot, phi, split projections) use one thread per (j,i) column.
#include "engine.hpp"
#include <cfloat>

#include "kernels.hpp"

#include <cstdio>
#include <vector>
#include "fastmath.hpp"
#include "devcommon.hpp"
#include "qxcommon.hpp"

namespace rcm {


// K1. surface_pressures, Main/mod_tendency.F90:815-834, and the 2-D reciprocals of decouple
// (rpsda, :868-875) and mkslice (1/psdotb, 1/psb, Main/mod_slice.F90:163-183), on the owned
// points and the ghost rings the consumers read: depth 2 for the atm1-derived ones and 3 for
// the atm2-derived ones (the stencils of the ghost-ring kernels), inside the global domain.
__device__ __forceinline__ void surface_pressures_at(const Geom& g, const Fields& f, int j, int i) {
  auto ring = [&](int d, int jhi, int ihi) {
    const bool jok = g.band ? in(j, g.jde1 - d, g.jde2 + d) : in(j, max(1, g.jde1 - d), min(jhi, g.jde2 + d));
    const bool iok = g.crm ? in(i, g.ide1 - d, g.ide2 + d) : in(i, max(1, g.ide1 - d), min(ihi, g.ide2 + d));
    return jok && iok;
  };
  if (ring(2, g.gjx - 1, g.giy - 1)) F2(f.rpsa, j, i) = d_one / F2(f.psa, j, i);
  if (ring(3, g.gjx - 1, g.giy - 1)) F2(f.rpsb, j, i) = d_one / F2(f.psb, j, i);
  if (ring(2, g.gjx, g.giy)) {
    const double v = psc2psd_global(g, f.psa, j, i);
    F2(f.psdota, j, i) = v;
    F2(f.rpsda, j, i) = d_one / v;
  }
  if (ring(3, g.gjx, g.giy)) {
    const double v = psc2psd_global(g, f.psb, j, i);
    F2(f.psdotb, j, i) = v;
    F2(f.rpsdb, j, i) = d_one / v;
  }
}
__global__ void k_surface_pressures(Geom g, Fields f) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  surface_pressures_at(g, f, j, i);
}

// generic relaxation contribution (nudge*, Main/mod_bdycod.F90:4262-4263)
__device__ __forceinline__ double relax(double ften, double xf, double xg, double f0, double f1, double f2,
                                        double f3, double f4) {
  return ften + xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0);
}
__device__ __forceinline__ void nudge_coef(const Consts* c, int ib, int k, double& xf, double& xg) {
  if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; }
  else { xf = c->hefc[ib][k]; xg = c->hegc[ib][k]; }
}

// qfuse: copies of the values at (j, i), levels k0, k0+dk, .. <= kz, that no update kernel of
// the step writes into the next buffers (k_qfilter's copies): u, v outside k_momentum's dot
// set, t outside k_scalars' cross set, qv, qc outside the owned interior (the moisture fix's
// set).  On a ghost point (the column box's one-point ring; k_columns runs before the atm2
// part of the prologue exchange has landed) only atm1 is copied: the atm2 ghost values this
// step still reads (a2 u, v on the boundary lines, in k_split_project's divergence) are read
// from the current buffers there (k_split_project), and the next step's exchange rewrites
// the rest before any read.
__device__ __forceinline__ void keep_point(const Geom& g, const Fields& f, int j, int i, int k0, int dk, int kz) {
  const bool own = in(j, g.jde1, g.jde2) && in(i, g.ide1, g.ide2);
  const int jd2 = g.br ? g.jdi2 : g.jde2 + 1, id2 = g.bt ? g.idi2 : g.ide2 + 1;
  const bool uvk = !(in(j, g.jdi1, jd2) && in(i, g.idi1, id2));
  const bool tk = !(in(i, g.icx1(), g.icx2()) && in(j, g.jcx1(), g.jcx2()) && g.gci(j, i));
  const bool qk = !(in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2));
  if (!uvk && !tk && !qk) return;
  for (int k = k0; k <= kz; k += dk) {
    const long p = (long)(k - 1) * g.plane + g.ix(j, i);
    if (uvk) { f.b1u[p] = f.a1u[p]; f.b1v[p] = f.a1v[p]; }
    if (tk) f.b1t[p] = f.a1t[p];
    if (qk) { f.b1qv[p] = f.a1qv[p]; f.b1qc[p] = f.a1qc[p]; }
    if (!own) continue;
    if (uvk) { f.b2u[p] = f.a2u[p]; f.b2v[p] = f.a2v[p]; }
    if (tk) f.b2t[p] = f.a2t[p];
    if (qk) { f.b2qv[p] = f.a2qv[p]; f.b2qc[p] = f.a2qc[p]; }
  }
}


// ---------------------------------------------------------------------------------------
// K2. Column work, 64 columns (j) of one row i per block:
//    compute_omega column part, Main/mod_tendency.F90:1123-1156 (pten, qdot k-scan),
//    new_pressure + nudge2d, :1428-1460 / Main/mod_bdycod.F90:4597-4766 (psc, nudged pten),
//    the geopotential of the PGF, :1966-1995, 2033-2097 (alpha_hyd = 0, td == tva),
//    and per-block partials of the Bleck noise sums (summed by k_split_correct).
//  A column block runs in two phases: all four wavefronts compute the independent per-level
//  terms (mass divergence, td, tvfac, the log ratios of the hypsometric equation) into LDS,
//  then wavefront 0 runs the pten sum / qdot scan / new_pressure and wavefront 1 the
//  geopotential recurrence, each in the reference's sequential order.
//  The same launch runs K1 (surface_pressures and the 2-D reciprocals): the column blocks on
//  their own columns, and `nsp` trailing blocks on the frame points outside the column box
//  (the deeper ghost rings of the reciprocals).  Nothing here reads those outputs elsewhere
//  than at the thread's own point, where rpsa = 1/psa is formed again (the same bits).
#ifndef COL_LB
#define COL_LB 6
#endif
// the column of lane tx in column block bb: part 0 the rows of the column box, part 1 the
// rows of R, part 2 the column box less R as one list (rows below R, the strips left and right
// of R, rows above R); false past the end
__device__ __forceinline__ bool column_of(const Geom& g, const Part& p, int bb, int tx, int nxb, int& j, int& i) {
  const int J1 = g.jdx1(), J2 = g.jdx2(), I1 = g.idx1(), I2 = g.idx2();
  if (p.part == 1) {
    j = p.ja + (bb % p.nxb) * COLW + tx;
    i = p.ia + bb / p.nxb;
    return j <= p.jb;
  }
  if (p.part == 2) {
    const int W = J2 - J1 + 1, wl = p.ja - J1, wm = wl + (J2 - p.jb);
    const int nb = (p.ia - I1) * W, nm = (p.ib - p.ia + 1) * wm, nt = (I2 - p.ib) * W;
    int q = bb * COLW + tx;
    j = J1; i = I1;
    if (q < nb) { i = I1 + q / W; j = J1 + q % W; return true; }
    q -= nb;
    if (q < nm) {
      const int c = q % wm;
      i = p.ia + q / wm;
      j = c < wl ? J1 + c : p.jb + 1 + (c - wl);
      return true;
    }
    q -= nm;
    if (q < nt) { i = p.ib + 1 + q / W; j = J1 + q % W; return true; }
    return false;
  }
  j = J1 + (bb % nxb) * COLW + tx;
  i = I1 + bb / nxb;
  return j <= J2;
}
// part 1 / part 2 membership of a block whose reads span [j1, j2] x [i1, i2]: true when this
// launch's part does not run it
__device__ __forceinline__ bool part_skip(const Part& p, int j1, int j2, int i1, int i2) {
  if (!p.part) return false;
  const bool inner = j1 >= p.ja && j2 <= p.jb && i1 >= p.ia && i2 <= p.ib;
  return inner != (p.part == 1);
}
#ifndef COL_KU
#define COL_KU 1
#endif
#ifndef COL_PF
#define COL_PF 1
#endif
// QX: nqx = 5, tvfac with the total water load (an instance of its own, so the nqx = 2 kernel
// keeps its code)
template <bool QX>
__global__ __launch_bounds__(COLT, COL_LB) void k_columns(Geom g, const Consts* __restrict__ c, StepState* s, Fields f,
                                                 int nxb, int ncol) {
  extern __shared__ double lds[];                        // 4 x kz x COLW
  PT_DECL
  const uint32_t P8 = g.P8, L8 = g.L8;
  const int bb = blockIdx.x;
  const int nsp = (g.nj * g.ni + COLT - 1) / COLT;
  if (bb >= ncol + nsp) {
    // qfuse: the copies of keep_point on the two outer rows and columns of the column box (every
    // point that has one), one (point, level) per thread; in blocks of their own so that the 2
    // in 3 column blocks with such points do not wait on them (+8 us at C3 when they did)
    const int J1 = g.jdx1(), J2 = g.jdx2(), I1 = g.idx1(), I2 = g.idx2();
    const int W = J2 - J1 + 1, H = I2 - I1 + 1;
    const int nb = 4 * W + 4 * (H > 4 ? H - 4 : 0);
    const int q = (bb - ncol - nsp) * COLT + (int)threadIdx.x;
    const int k = q / nb + 1, p = q % nb;
    if (k > c->kz) return;
    int jj, ii;
    if (p < 4 * W) {
      const int r = p / W;
      ii = r < 2 ? I1 + r : I2 - (3 - r);
      jj = J1 + p % W;
    } else {
      const int r = (p - 4 * W) % 4;
      ii = I1 + 2 + (p - 4 * W) / 4;
      jj = r < 2 ? J1 + r : J2 - (3 - r);
    }
    // a narrow box visits some points twice: the copies are idempotent
    if (in(jj, J1, J2) && in(ii, I1, I2)) keep_point(g, f, jj, ii, k, 1, k);
    return;
  }
  if (bb >= ncol) {
    // surface pressures (and with qfuse the copy of p*) on the frame points outside the column
    // box, all ghost points
    const int q = (bb - ncol) * COLT + (int)threadIdx.x;
    const int jj = g.j0 + q % g.nj, ii = g.i0 + q / g.nj;
    if (ii < g.i0 + g.ni && !(in(jj, g.jdx1(), g.jdx2()) && in(ii, g.idx1(), g.idx2()))) {
      surface_pressures_at(g, f, jj, ii);
      if (f.qfuse) { F2(f.bpsa, jj, ii) = F2(f.psa, jj, ii); F2(f.bpsb, jj, ii) = F2(f.psb, jj, ii); }
    }
    return;
  }
  // COL_XCD: the column blocks of one tile in XCD-contiguous runs of rows, so a block's i + 1
  // row (the dot points of its divergence) is the next row's block's own and a hit in the same
  // L2; the noise partial keeps the block's logical slot, so the sums are unchanged
  const int cb = (COL_XCD && f.pt.part == 0) ? xcd_range(bb, 0, ncol) : bb;
  // k_scalars appends after this (part 2 follows part 1 and the k_scalars blocks of part 1)
  if (f.qfuse && cb == 0 && threadIdx.x == 0 && f.pt.part != 2) *f.negcnt = 0;
  const int tx = (int)threadIdx.x % COLW, ty = (int)threadIdx.x / COLW;     // column, level group

  // Blocks cover the columns of the tile plus its ghost ring toward neighbours: the ghost
  // columns compute exactly what their owners do (qdot, phi, pten and the new p* there replace
  // the reference's exchanges of them).
  int j, i;
  const bool valid = column_of(g, f.pt, cb, tx, nxb, j, i);
  const bool own = valid && in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
  const bool ce = valid && in(j, g.jcx1(), g.jcx2()) && in(i, g.icx1(), g.icx2());
  const bool ci = ce && g.gci(j, i);
  const int kz = c->kz;
  double* sMD = lds;                                      // mass divergence, [k-1][tx]
  double* sTD = lds + kz * COLW;                            // td
  double* sTV = lds + 2 * kz * COLW;                        // tvfac
  double* sLG = lds + 3 * kz * COLW;                        // log ratio of the layer below level k
  const uint32_t o2 = valid ? g.o2(j, i) : 0u;
  const double ptop = c->ptop, rgas = c->rgas, ep1 = c->ep1;
  if (valid && ty == COLG - 1) surface_pressures_at(g, f, j, i);
  PT_MARK();
  double rp = 0.0;
  if (ce) {
    // phase 1: umc/vmc = atm1 * msfd (decouple :880-890); xqv/xqc decoupled moisture (:1000-1016)
    const double mx = LD(f.msfx, o2);
    const double dummy = d_one / (c->dx2 * mx * mx);
    const double m00 = LD(f.msfd, o2), m10 = LD(f.msfd, O2(1, 0));
    const double m01 = LD(f.msfd, O2(0, 1)), m11 = LD(f.msfd, O2(1, 1));
    const double psk = LD(f.psa, o2);
    rp = d_one / psk;                                    // rpsa (K1), the same division
    // two levels per thread and pass: every load of the pass is issued before any use
    constexpr int KU = COL_KU;
    for (int k0 = ty + 1; k0 <= kz; k0 += COLG * KU) {
      double u00[KU], u10[KU], u01[KU], u11[KU], v00[KU], v10[KU], v01[KU], v11[KU], tt[KU], qq[KU], cc[KU];
      double xq[KU][QX ? NQXH : 1];
#pragma unroll
      for (int n = 0; n < KU; n++) {
        const int kk = k0 + COLG * n;
        const uint32_t o3 = o2 + (uint32_t)((kk <= kz ? kk : kz) - 1) * L8;
        u00[n] = LD(f.a1u, o3); u10[n] = LD(f.a1u, O3(1, 0)); u01[n] = LD(f.a1u, O3(0, 1)); u11[n] = LD(f.a1u, O3(1, 1));
        v00[n] = LD(f.a1v, o3); v10[n] = LD(f.a1v, O3(1, 0)); v01[n] = LD(f.a1v, O3(0, 1)); v11[n] = LD(f.a1v, O3(1, 1));
        tt[n] = LD(f.a1t, o3); qq[n] = LD(f.a1qv, o3); cc[n] = LD(f.a1qc, o3);
        // nqx = 5: the species of the total water load, in the same round of loads
        if (QX)
#pragma unroll
          for (int q = 0; q < NQXH; q++) xq[n][q] = LD(f.qxa1[q], o3);
      }
#pragma unroll
      for (int n = 0; n < KU; n++) {
      const int k = k0 + COLG * n;
      if (k > kz) break;
      const double a = u11[n] * m11 + u10[n] * m10 - u01[n] * m01 - u00[n] * m00;
      const double bq = v11[n] * m11 + v01[n] * m01 - v10[n] * m10 - v00[n] * m00;
      sMD[(k - 1) * COLW + tx] = (a + bq) * dummy;
      const double qv = dmax(qq[n] * rp, MINQQ);
      const double qc = dmax(cc[n] * rp, d_zero);
      double tdk = tt[n] * (d_one + ep1 * qv);
      // ipgf = 1: minus the reference-atmosphere temperature (ttld, :1893-1964)
      if (c->ipgf == 1) tdk = tdk - psk * T00PG * rcm_powpos((c->hsigma[k] * psk + ptop) / P00PG, c->pgfaa1);
      sTD[(k - 1) * COLW + tx] = tdk;
      if (QX) {
        // nqx = 5: tvfac with the total water load qcd = ((0 + qc) + qi) + qr + qs (decouple
        // :1107-1115, each atmx%qx = max(atm1 * rpsa, 0); pressure_gradient_force :2037)
        double qcd = d_zero + qc;
#pragma unroll
        for (int q = 0; q < NQXH; q++) qcd = qcd + dmax(xq[n][q] * rp, d_zero);
        sTV[(k - 1) * COLW + tx] = d_one / (d_one + qcd / (d_one + qv));
      } else {
        sTV[(k - 1) * COLW + tx] = d_one / (d_one + qc / (d_one + qv));
      }
      }
    }
    PT_MARK();
    // the hypsometric log ratios in a loop of their own (no loads in flight there: the log's
    // polynomial constants stay in registers without spilling)
    for (int k = ty + 1; k <= kz; k += COLG)
      sLG[(k - 1) * COLW + tx] = (k < kz) ? rcm_log((c->hsigma[k] + ptop * rp) / (c->hsigma[k + 1] + ptop * rp))
                                        : rcm_log((c->hsigma[kz] + ptop * rp) / (d_one + ptop * rp));
    PT_MARK();
  }
  // the operands of new_pressure (scan wavefront) and of the geopotential column are loaded
  // before the barrier, so their latency overlaps the wait for the other level groups instead
  // of following the pten / qdot scan (COL_PF = 0: loaded where they are used)
  const int gwave = COLW == 32 ? 2 : 1;
#if COL_PF
  double psbv = 0.0, pav = 0.0, pbt0 = 0.0, dtv = 0.0, xbt = 0.0, fg1[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  int rgc = 0, ibc = 0;
  if (ce && ty == 0) {
    psbv = LD(f.psb, o2);
    pav = LD(f.psa, o2);
    rgc = f.rgcr[o2 >> 3];
    ibc = f.ibcr[o2 >> 3];
    dtv = s->dt;
    xbt = s->xbctime;
    if (ci) {
      pbt0 = LD(f.pbt, o2);
      const int dj[5] = {0, -1, 1, 0, 0}, di[5] = {0, 0, 0, -1, 1};
#pragma unroll
      for (int n = 0; n < 5; n++) {
        const uint32_t q = O2(dj[n], di[n]);
        fg1[n] = (LD(f.pb0, q) + (xbt + dtv) * LD(f.pbt, q)) - LD(f.psb, q);
      }
    }
  }
  double gps = 0.0, ght = 0.0;
  if (ce && ty == gwave) {
    gps = LD(f.psa, o2);
    ght = LD(f.ht, o2);
  }
#endif
  __syncthreads();
  PT_MARK();
  double na = 0.0, nb = 0.0;
  if (valid && ty == 0) {
    double pt = d_zero;
    if (!ce && f.qfuse) { ST(f.bpsa, o2, LD(f.psa, o2)); ST(f.bpsb, o2, LD(f.psb, o2)); }
    if (!ce) {
      for (int k = 1; k <= kz + 1; k++) ST(f.qdot, o2 + (uint32_t)(k - 1) * L8, d_zero);
    } else {
      for (int k = 1; k <= kz; k++) pt = pt - sMD[(k - 1) * COLW + tx] * c->dsigma[k];
      ST(f.pten, o2, pt);
      double q = d_zero;
      ST(f.qdot, o2, d_zero);
      for (int k = 2; k <= kz; k++) {
        q = q - (pt + sMD[(k - 2) * COLW + tx]) * c->dsigma[k - 1] * rp;
        ST(f.qdot, o2 + (uint32_t)(k - 1) * L8, q);
      }
      ST(f.qdot, o2 + (uint32_t)kz * L8, d_zero);
    }
    if (ce) {
      // new_pressure
#if COL_PF
      const double dt = dtv;
      if (ci && rgc > 0 && c->iboudy == 4) {
        // sponge2d, Main/mod_bdycod.F90:3065-3122
        pt = c->wgtx[ibc] * pt + (d_one - c->wgtx[ibc]) * pbt0;
      } else if (ci && rgc > 0) {
        double xf, xg;
        nudge_coef(c, ibc, kz, xf, xg);
        pt = relax(pt, xf, xg, fg1[0], fg1[1], fg1[2], fg1[3], fg1[4]);
      }
#else
      const double dt = s->dt;
      const double psbv = LD(f.psb, o2);
      if (ci && f.rgcr[o2 >> 3] > 0 && c->iboudy == 4) {
        // sponge2d, Main/mod_bdycod.F90:3065-3122
        const int ib = f.ibcr[o2 >> 3];
        pt = c->wgtx[ib] * pt + (d_one - c->wgtx[ib]) * LD(f.pbt, o2);
      } else if (ci && f.rgcr[o2 >> 3] > 0) {
        const double xt = s->xbctime + dt;
        double xf, xg;
        nudge_coef(c, f.ibcr[o2 >> 3], kz, xf, xg);
#define FG1(dj, di) ((LD(f.pb0, O2(dj, di)) + xt * LD(f.pbt, O2(dj, di))) - LD(f.psb, O2(dj, di)))
        pt = relax(pt, xf, xg, FG1(0, 0), FG1(-1, 0), FG1(1, 0), FG1(0, -1), FG1(0, 1));
#undef FG1
      }
#endif
      ST(f.ptenn, o2, pt);
      const double pc = psbv + pt * dt;
      ST(f.psc, o2, pc);
      if (f.qfuse) {
        // the RA filter of p* (Main/mod_tendency.F90:420, filter_ra_2d) into the next buffers
#if COL_PF
        const double pa = pav;
#else
        const double pa = LD(f.psa, o2);
#endif
        if (ci) {
          const double d = c->gnu1 * (pc + psbv - d_two * pa);
          ST(f.bpsb, o2, pa + d);
          ST(f.bpsa, o2, pc);
        } else {
          ST(f.bpsa, o2, pa);
          ST(f.bpsb, o2, psbv);
        }
      }
      if (s->lcount > 0 && ci && own) {
        na = fabs(pt);
#if COL_PF
        nb = fabs((pc + psbv - d_two * pav) / (dt * dt * d_rfour));
#else
        nb = fabs((pc + psbv - d_two * LD(f.psa, o2)) / (dt * dt * d_rfour));
#endif
      }
    }
  }
  // the geopotential column on another wavefront than the pten/qdot scan (COLW = 32: level
  // groups 2k and 2k+1 share wavefront k)
  if (ce && ty == gwave) {
    // geopotential column, bottom-up
#if COL_PF
    const double ps = gps;
    double top = ght;
#else
    const double ps = LD(f.psa, o2);
    double top = LD(f.ht, o2);
#endif
    double tdk1 = sTD[(kz - 1) * COLW + tx];
    const double tv = tdk1 * rp * sTV[(kz - 1) * COLW + tx];
    if (c->ipgf == 1) top = top + rgas * T00PG / c->pgfaa1 * rcm_powpos((ps + ptop) / P00PG, c->pgfaa1);  // :2045
    double ph = top - rgas * tv * sLG[(kz - 1) * COLW + tx];
    ST(f.phi, o2 + (uint32_t)(kz - 1) * L8, ph);
    for (int lev = kz - 1; lev >= 1; lev--) {
      const double tdl = sTD[(lev - 1) * COLW + tx];
      const double tvavg = ((tdl * c->dsigma[lev] + tdk1 * c->dsigma[lev + 1]) /
                            (ps * (c->dsigma[lev] + c->dsigma[lev + 1]))) * sTV[(lev - 1) * COLW + tx];
      ph = ph - rgas * tvavg * sLG[(lev - 1) * COLW + tx];
      ST(f.phi, o2 + (uint32_t)(lev - 1) * L8, ph);
      tdk1 = tdl;
    }
  }
  PT_MARK();
  // per-block partial of the noise sums (fixed tree); k_split_correct sums the partials.  Only
  // wavefront 0 holds non-zero terms, so the block's halving tree (a[t] += a[t + w], w = 256 ..
  // 1) reduces to wavefront 0's halving tree from w = 32 (adding the +0.0 terms of the other
  // wavefronts changes no bit): a shuffle reduction in registers, and no LDS for it (3 blocks
  // per CU fit the column LDS, so one round of blocks covers C3)
  if (threadIdx.x < 64) {         // wavefront 0 (COLW = 32: level groups 0 and 1, the latter's terms +0.0)
    for (int w = 32; w > 0; w >>= 1) {
      na = na + __shfl_down(na, w);
      nb = nb + __shfl_down(nb, w);
    }
    if (threadIdx.x == 0) {
      const int slot = f.red_off + (f.pt.part == 2 ? f.pt.rbase : 0) + cb;
      f.red[2 * slot] = na;
      f.red[2 * slot + 1] = nb;
    }
  }
  PT_PRINT(1);
}
template __global__ __launch_bounds__(COLT, COL_LB) void k_columns<false>(Geom, const Consts* __restrict__, StepState*,
                                                                        Fields, int, int);
template __global__ __launch_bounds__(COLT, COL_LB) void k_columns<true>(Geom, const Consts* __restrict__, StepState*,
                                                                       Fields, int, int);

// ---------------------------------------------------------------------------------------
// K3. Momentum: hadvuv + vadvuv + curvature + nudgeuv + diffu_d + PGF, then the forecast and
// the Robert-Asselin filter (Main/mod_advection.F90:203-299, Main/mod_tendency.F90:1829-1838,
// Main/mod_bdycod.F90:3581-3823, Main/mod_diffusion.F90:281-385, Main/mod_tendency.F90:
// 1996-2025, 2103-2115, 404-411, 433-445; Main/mod_timefilter.F90 filter_ra_uv).
// One block = MBJ x MBI dot points of the interior (jdi x idi) at one level.  Every stencil
// operand is first staged in LDS for the block plus its halo, with the decoupled products
// formed once per staged point (umc/vmc = atm1*msfd, ud/vd = atm1*rpsda, ubd3d/msfd =
// (atm2*(1/psdotb))/msfd, tv = t*(1+ep1*qv)): one round of independent global loads per
// block instead of dependent per-operand rounds, and one division per staged point instead
// of 13 per output.  Points outside jdi x idi keep their values (copied by k_qfilter).
// decoupled boundary ud/vd of decouple with the inflow/outflow rule of iboudy = 3/4
// (Main/mod_tendency.F90:893-994): an outflow boundary point takes the adjacent interior
// value.  W/E run on the idi columns first, then S/N on the full jde rows, so a corner row
// point copies the (possibly already replaced) W/E value.  The slice values the reference
// multiplies (wui, wue, ...) equal atm1 there (bdyuv), so the default is atm1 * rpsda.
__device__ double2 udvd_bdy(const Geom& g, const Fields& f, int j, int i, uint32_t kof) {
  auto base = [&](int jj, int ii) {
    const uint32_t q2 = g.o2(jj, ii);
    const double r = LD(f.rpsda, q2);
    return make_double2(LD(f.a1u, q2 + kof) * r, LD(f.a1v, q2 + kof) * r);
  };
  // global boundary lines (a ghost point on them carries the value its owner computes and
  // the reference exchanges)
  auto we = [&](int jj, int ii) {
    if (in(ii, 2, g.giy - 1)) {
      if (g.gjeq(jj, 1) && LD(f.a1u, g.o2(jj, ii) + kof) <= d_zero) return base(2, ii);
      if (g.gjeq(jj, g.gjx) && LD(f.a1u, g.o2(jj, ii) + kof) >= d_zero) return base(g.gjx - 1, ii);
    }
    return base(jj, ii);
  };
  if (g.band || in(j, 1, g.gjx)) {
    if (i == 1 && LD(f.a1v, g.o2(j, i) + kof) >= d_zero) return we(j, 2);
    if (i == g.giy && LD(f.a1v, g.o2(j, i) + kof) <= d_zero) return we(j, g.giy - 1);
  }
  return we(j, i);
}

// ---------------------------------------------------------------------------------------
// K_SL. Semi-Lagrangian horizontal advection of qv and qc (isladvec = 1),
// Main/mod_sladvection.F90: trajcalc_x (:121-229, adv_velocity(.false.) :91-114), slhadv_x4d
// of atm2 qx (:401-479) and hdvg_x4d of atm1 qx (:596-664), one thread per owned interior cross
// point and level.  The result is the start of qxdyn, (0 + sl) - hdvg, which k_scalars takes
// in place of hadvqv/hadvqx (Main/mod_tendency.F90:1361-1380).  ua/va = atmx%umd/vmd = ud*msfd
// (:998-1001); the departure points reach three points beyond (j, i), inside the exchanged
// atm2 ring.  A departure point more than one cell away sets the step flag (fatal
// 'SLADVECTION', :149-154, 184-189).
__global__ __launch_bounds__(256) void k_sladv(Geom g, const Consts* __restrict__ c, StepState* s, Fields f, QxArgs qx) {
  THREAD_POINT(g.jci1, g.ici1);
  if (j > g.jci2 || i > g.ici2) return;
  const uint32_t P8 = g.P8, L8 = g.L8, kof = (uint32_t)(k - 1) * L8;
  (void)P8;
  const bool ib4 = c->iboudy == 3 || c->iboudy == 4;     // inflow/outflow boundary winds
  auto ua = [&](int jj, int ii) {
    const uint32_t q2 = g.o2(jj, ii);
    double ud;
    if (ib4 && (g.gjeq(jj, 1) || g.gjeq(jj, g.gjx) || g.gieq(ii, 1) || g.gieq(ii, g.giy))) ud = udvd_bdy(g, f, jj, ii, kof).x;
    else ud = LD(f.a1u, q2 + kof) * LD(f.rpsda, q2);
    return ud * LD(f.msfd, q2);
  };
  auto va = [&](int jj, int ii) {
    const uint32_t q2 = g.o2(jj, ii);
    double vd;
    if (ib4 && (g.gjeq(jj, 1) || g.gjeq(jj, g.gjx) || g.gieq(ii, 1) || g.gieq(ii, g.giy))) vd = udvd_bdy(g, f, jj, ii, kof).y;
    else vd = LD(f.a1v, q2 + kof) * LD(f.rpsda, q2);
    return vd * LD(f.msfd, q2);
  };
  const double dt = s->dt, dtsq = dt * dt, dtcb = dt * dt * dt, ddx = c->dx, ddy = c->dx;
  const double mx = F2(f.msfx, j, i);
  const double u00 = ua(j, i), u01 = ua(j, i + 1), u11 = ua(j + 1, i + 1), u10 = ua(j + 1, i);
  const double v00 = va(j, i), v01 = va(j, i + 1), v11 = va(j + 1, i + 1), v10 = va(j + 1, i);
  const double uadvx = 0.25 * (u00 + u01 + u11 + u10) / mx;
  const double uadxp1 = 0.25 * (u10 + u11 + ua(j + 2, i + 1) + ua(j + 2, i)) / F2(f.msfx, j + 1, i);
  const double uadxm1 = 0.25 * (u00 + u01 + ua(j - 1, i + 1) + ua(j - 1, i)) / F2(f.msfx, j - 1, i);
  const double vadvy = 0.25 * (v00 + v01 + v11 + v10) / mx;
  const double vadyp1 = 0.25 * (v01 + v11 + va(j + 1, i + 2) + va(j, i + 2)) / F2(f.msfx, j, i + 1);
  const double vadym1 = 0.25 * (v00 + va(j, i - 1) + v10 + v10) / F2(f.msfx, j, i - 1);   // as written, :109-111
  const double ux = 0.5 * (uadxp1 - uadxm1) / ddx;
  const double uxx = (uadxp1 - 2.0 * uadvx + uadxm1) / (ddx * ddx);
  const double xdis = -(uadvx * dt) + 0.5 * (dtsq * uadvx * ux) - (dtcb * uadvx) * (ux * ux + uadvx * uxx) / 6.0;
  const double vy = 0.5 * (vadyp1 - vadym1) / ddy;
  const double vyy = (vadyp1 - 2.0 * vadvy + vadym1) / (ddy * ddy);
  const double ydis = -(vadvy * dt) + 0.5 * (dtsq * vadvy * vy) - (dtcb * vadvy) * (vy * vy + vadvy * vyy) / 6.0;
  const double xn = xdis / ddx, yn = ydis / ddy;
  if (!(fabs(xn) < 2.0) || !(fabs(yn) < 2.0)) {          // |int(xn)| > 1, or not a number
    s->slflag = 1;
    return;
  }
  const int xnp = (int)xn, ynp = (int)yn;
  const double alfax = fabs(((double)xnp * ddx - xdis) / ddx);
  const double betay = fabs(((double)ynp * ddy - ydis) / ddy);
  const int xsn = (int)copysign(1.0, xn), ysn = (int)copysign(1.0, yn);
  int xnd = j + xnp, xm1 = xnd + xsn, xm2 = xm1 + xsn, xp1 = xnd - xsn;
  int ynd = i + ynp, ym1 = ynd + ysn, ym2 = ym1 + ysn, yp1 = ynd - ysn;
  if (g.bl) { xnd = max(xnd, g.jce1); xm1 = max(xm1, g.jce1); xm2 = max(xm2, g.jce1); xp1 = max(xp1, g.jce1); }
  if (g.br) { xnd = min(xnd, g.jce2); xm1 = min(xm1, g.jce2); xm2 = min(xm2, g.jce2); xp1 = min(xp1, g.jce2); }
  if (g.bb) { ynd = max(ynd, g.ice1); ym1 = max(ym1, g.ice1); ym2 = max(ym2, g.ice1); yp1 = max(yp1, g.ice1); }
  if (g.bt) { ynd = min(ynd, g.ice2); ym1 = min(ym1, g.ice2); ym2 = min(ym2, g.ice2); yp1 = min(yp1, g.ice2); }
  const double alfm2 = -(alfax * (1.0 - alfax * alfax)) / 6.0;
  const double alfm1 = (alfax * (1.0 + alfax) * (2.0 - alfax)) / 2.0;
  const double alf0 = ((1.0 - alfax * alfax) * (2.0 - alfax)) / 2.0;
  const double alfp1 = -(alfax * (1.0 - alfax) * (2.0 - alfax)) / 6.0;
  const double betm2 = -(betay * (1.0 - betay * betay)) / 6.0;
  const double betm1 = (betay * (1.0 + betay) * (2.0 - betay)) / 2.0;
  const double bet0 = ((1.0 - betay * betay) * (2.0 - betay)) / 2.0;
  const double betp1 = -(betay * (1.0 - betay) * (2.0 - betay)) / 6.0;
  // hdvg_x4d divergence (:625-649)
  const double m11 = F2(f.msfd, j + 1, i + 1), m10 = F2(f.msfd, j + 1, i), m01 = F2(f.msfd, j, i + 1);
  const double m00 = F2(f.msfd, j, i);
  const double ucapf = (u11 * m11 + u10 * m10) * d_half;
  const double ucapi = (u01 * m01 + u00 * m00) * d_half;
  const double vcapf = (v11 * m11 + v01 * m01) * d_half;
  const double vcapi = (v10 * m10 + v00 * m00) * d_half;
  const double ducapdx = (ucapf - ucapi) / c->dx;
  const double dvcapdy = (vcapf - vcapi) / c->dx;
  const double hdvg = (ducapdx + dvcapdy) / (mx * mx);
  // qv, qc, then (nqx = 5) qi, qr, qs: slhadv_x4d / hdvg_x4d over n = iqfrst..iqlst
  for (int n = 0; n < 2 + qx.nsp; n++) {
    const double* var = n == 0 ? f.a2qv : n == 1 ? f.a2qc : qx.a2[n - 2];
#define V(J, I) F3(var, J, I, k)
    const double bl1 = alfax * V(xm1, yp1) + (d_one - alfax) * V(xnd, yp1);
    const double bl2 = alfax * V(xm1, ym2) + (d_one - alfax) * V(xnd, ym2);
    const double cb1 = alfm2 * V(xm2, ynd) + alfm1 * V(xm1, ynd) + alf0 * V(xnd, ynd) + alfp1 * V(xp1, ynd);
    const double cb2 = alfm2 * V(xm2, ym1) + alfm1 * V(xm1, ym1) + alf0 * V(xnd, ym1) + alfp1 * V(xp1, ym1);
    const double tbadp = betm2 * bl2 + betm1 * cb2 + bet0 * cb1 + betp1 * bl1;
    double tsla = tbadp;
    if (c->iqmsl == 1) {
      const double tbmax = fmax(fmax(fmax(V(xnd, ynd), V(xnd, ym1)), V(xm1, ynd)), V(xm1, ym1));
      const double tbmin = fmin(fmin(fmin(V(xnd, ynd), V(xnd, ym1)), V(xm1, ynd)), V(xm1, ym1));
      if (tbadp > tbmax) tsla = tbmax;
      else if (tbadp < tbmin) tsla = tbmin;
    }
    double ften = d_zero;
    if (fabs(tsla - V(j, i)) > DLOWVAL) ften = ften + (tsla - V(j, i)) / dt;
#undef V
    const double q1 = F3(n == 0 ? f.a1qv : n == 1 ? f.a1qc : qx.a1[n - 2], j, i, k);
    const double tatot = (q1 > DBL_EPSILON) ? q1 * hdvg : d_zero;
    F3(n == 0 ? f.slqv : n == 1 ? f.slqc : qx.sl[n - 2], j, i, k) = ften - tatot;
  }
}

constexpr int TW1 = MBJ + 2, TH1 = MBI + 2;   // halo 1 on every side
constexpr int TW2 = MBJ + 4, TH2 = MBI + 4;   // halo 2 on every side
constexpr int TW0 = MBJ + 1, TH0 = MBI + 1;   // halo 1 on the low sides (j-1, i-1)
// blocks per CU the register budget is sized for (LDS admits 2 of these blocks per CU)
#ifndef MO_LB
#define MO_LB 4
#endif
#ifndef SC_LB
#define SC_LB 4
#endif
// LDS of one k_momentum block
struct MomLDS {
  double sUMC[TH1][TW1], sVMC[TH1][TW1], sUD[TH1][TW1], sVD[TH1][TW1];
  double sUM[TH2][TW2], sVM[TH2][TW2];
  // ubd3d/vbd3d (consumed by xkc) share storage with the PGF log terms formed afterwards
  union {
    struct { double UB[TH2][TW2], VB[TH2][TW2]; } b;
    struct { double LU[MBI][TW0], LV[TH0][MBJ]; } l;
  } sX;
  double sTV[TH0][TW0], sQ0[TH0][TW0], sQ1[TH0][TW0], sPH[TH0][TW0], sPS[TH0][TW0], sXK[TH0][TW0];
};
// one k_momentum block (bx, by, bz) with its LDS (k_momentum, or the momentum blocks of k_update)
__device__ __forceinline__ void momentum_block(const Geom& g, const Consts* __restrict__ c,
                                               const StepState* __restrict__ s, const Fields& f, MomLDS& L,
                                               int bx, int by, int bz) {
  auto& sUMC = L.sUMC; auto& sVMC = L.sVMC; auto& sUD = L.sUD; auto& sVD = L.sVD;
  auto& sUM = L.sUM; auto& sVM = L.sVM; auto& sX = L.sX;
  auto& sTV = L.sTV; auto& sQ0 = L.sQ0; auto& sQ1 = L.sQ1; auto& sPH = L.sPH; auto& sPS = L.sPS; auto& sXK = L.sXK;
#define sUB sX.b.UB
#define sVB sX.b.VB
  const int tid = threadIdx.x;
  PT_DECL
  const int J0 = (f.pt.part ? f.pt.mj0 : g.jdi1) + bx * MBJ, I0 = g.idi1 + by * MBI;
  const int k = bz + 1;
  if (part_skip(f.pt, J0 - 2, J0 + MBJ + 1, I0 - 2, I0 + MBI + 1)) return;   // the staged halo-2 tile
  const uint32_t P8 = g.P8, L8 = g.L8;
  const uint32_t kof = (uint32_t)(k - 1) * L8;
  const int jlo = g.j0, jhi = g.j0 + g.nj - 1, ilo = g.i0, ihi = g.i0 + g.ni - 1;
  const int kz = c->kz;
  const double ep1 = c->ep1;
  // this thread's point and its point operands, loaded before the staging barrier so their
  // latency overlaps it (threads past the interior read a valid interior address)
  // the tile's jdi x idi points and its right/top ghost ring (k_split_project's divergence and
  // the bdyuv slices read the new u, v there); boundary branches test global indices
  const int tj = tid % MBJ, ti = tid / MBJ;
  const int j = J0 + tj, i = I0 + ti;
  const bool valid = j >= g.jdi1 && j <= (g.br ? g.jdi2 : g.jde2 + 1) && i <= (g.bt ? g.idi2 : g.ide2 + 1);
  const uint32_t o2 = valid ? g.o2(j, i) : g.o2(g.jdi1, g.idi1), o3 = o2 + kof;
  const double u1c = LD(f.a1u, o3), v1c = LD(f.a1v, o3), u2c = LD(f.a2u, o3), v2c = LD(f.a2v, o3);
  const double u1m = (k >= 2) ? LD(f.a1u, o3 - L8) : 0.0, v1m = (k >= 2) ? LD(f.a1v, o3 - L8) : 0.0;
  const double u1p = (k < kz) ? LD(f.a1u, o3 + L8) : 0.0, v1p = (k < kz) ? LD(f.a1v, o3 + L8) : 0.0;
  const double dmsf = LD(f.dmsf, o2), cor = LD(f.coriol, o2), pdotb = LD(f.psdotb, o2);
  const double pdota = LD(f.psdota, o2), mfd = LD(f.msfd, o2);
  const int rgd = f.rgdt[o2 >> 3];
  // ---- stage.  Every global load of the three staging sets (and hgfact for xkc) is issued
  // before the first LDS write: one memory latency per block.  Lanes past the tile or the frame
  // read this thread's own (valid) address and stage zero.
  constexpr int N1 = (TW1 * TH1 + MBT - 1) / MBT, N2 = (TW2 * TH2 + MBT - 1) / MBT;
  constexpr int N0 = (TW0 * TH0 + MBT - 1) / MBT;
  double au[N1], av[N1], am[N1], ar[N1];
  double br[N2], bm[N2], bu[N2], bv[N2];
  double crp[N0], ct[N0], cqv[N0], cq0[N0], cq1[N0], cph[N0], cps[N0], chg[N0];
  bool aok[N1], bok[N2], cok[N0];
#pragma unroll
  for (int n = 0; n < N1; n++) {
    const int t = tid + n * MBT, jg = J0 - 1 + t % TW1, ig = I0 - 1 + t / TW1;
    aok[n] = t < TW1 * TH1 && jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = aok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < TW1 * TH1) {          // waves wholly past the staged tile skip the loads
      au[n] = LD(f.a1u, q3); av[n] = LD(f.a1v, q3); am[n] = LD(f.msfd, q2); ar[n] = LD(f.rpsda, q2);
    } else {
      au[n] = av[n] = am[n] = ar[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < N2; n++) {
    const int t = tid + n * MBT, jg = J0 - 2 + t % TW2, ig = I0 - 2 + t / TW2;
    bok[n] = t < TW2 * TH2 && jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = bok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < TW2 * TH2) {          // waves wholly past the staged tile skip the loads
      br[n] = LD(f.rpsdb, q2); bm[n] = LD(f.msfd, q2); bu[n] = LD(f.a2u, q3); bv[n] = LD(f.a2v, q3);
    } else {
      br[n] = bm[n] = bu[n] = bv[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < N0; n++) {
    const int t = tid + n * MBT, jg = J0 - 1 + t % TW0, ig = I0 - 1 + t / TW0;
    cok[n] = t < TW0 * TH0 && jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = cok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < TW0 * TH0) {          // waves wholly past the staged tile skip the loads
      crp[n] = LD(f.rpsa, q2); ct[n] = LD(f.a1t, q3); cqv[n] = LD(f.a1qv, q3);
      cq0[n] = LD(f.qdot, q3); cq1[n] = LD(f.qdot, q3 + L8); cph[n] = LD(f.phi, q3); cps[n] = LD(f.psa, q2);
      chg[n] = LD(f.hgfact, q2);
    } else {
      crp[n] = ct[n] = cqv[n] = cq0[n] = cq1[n] = cph[n] = cps[n] = chg[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < N1; n++) {
    const int t = tid + n * MBT, jj = t % TW1, ii = t / TW1;
    if (t < TW1 * TH1) {
      const bool ok = aok[n];
      double ud = ok ? au[n] * ar[n] : 0.0, vd = ok ? av[n] * ar[n] : 0.0;
      if ((c->iboudy == 3 || c->iboudy == 4) && ok) {
        const int jg = J0 - 1 + jj, ig = I0 - 1 + ii;
        if (g.gjeq(jg, 1) || g.gjeq(jg, g.gjx) || ig == 1 || ig == g.giy) {
          const double2 bb = udvd_bdy(g, f, jg, ig, kof);
          ud = bb.x; vd = bb.y;
        }
      }
      sUMC[ii][jj] = ok ? au[n] * am[n] : 0.0; sVMC[ii][jj] = ok ? av[n] * am[n] : 0.0;
      sUD[ii][jj] = ud; sVD[ii][jj] = vd;
    }
  }
#pragma unroll
  for (int n = 0; n < N2; n++) {
    const int t = tid + n * MBT, jj = t % TW2, ii = t / TW2;
    if (t < TW2 * TH2) {
      const bool ok = bok[n];
      const double ub = bu[n] * br[n], vb = bv[n] * br[n];
      sUM[ii][jj] = ok ? ub / bm[n] : 0.0; sVM[ii][jj] = ok ? vb / bm[n] : 0.0;
      sUB[ii][jj] = ok ? ub : 0.0; sVB[ii][jj] = ok ? vb : 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < N0; n++) {
    const int t = tid + n * MBT, jj = t % TW0, ii = t / TW0;
    if (t < TW0 * TH0) {
      const bool ok = cok[n];
      const double rp = crp[n];
      const double tt = ct[n] * rp;
      const double qv = dmax(cqv[n] * rp, MINQQ);
      sTV[ii][jj] = ok ? tt * (d_one + ep1 * qv) : 0.0;
      sQ0[ii][jj] = ok ? cq0[n] : 0.0; sQ1[ii][jj] = ok ? cq1[n] : 0.0;
      sPH[ii][jj] = ok ? cph[n] : 0.0; sPS[ii][jj] = ok ? cps[n] : 0.0;
    }
  }
  __syncthreads();
  PT_MARK();
  // calc_coeff Smagorinsky xkc (Main/mod_diffusion.F90:194-210) at the low-halo tile points from
  // the staged ubd3d/vbd3d, over the cross points of the tile and its ghost ring toward
  // neighbouring tiles (the reference's exchanged xkc there is the same computation)
#pragma unroll
  for (int n = 0; n < N0; n++) {
    const int t = tid + n * MBT, jj = t % TW0, ii = t / TW0, jg = J0 - 1 + jj, ig = I0 - 1 + ii;
    if (t < TW0 * TH0) {
      double xk = 0.0;
      if (g.gce(jg, ig)) {
        const int y = ii + 1, x = jj + 1;            // (jg, ig) in the halo-2 tiles
        const double dudx = sUB[y][x + 1] + sUB[y + 1][x + 1] - sUB[y][x] - sUB[y + 1][x];
        const double dvdx = sVB[y][x + 1] + sVB[y + 1][x + 1] - sVB[y][x] - sVB[y + 1][x];
        const double dudy = sUB[y + 1][x] + sUB[y + 1][x + 1] - sUB[y][x] - sUB[y][x + 1];
        const double dvdy = sVB[y + 1][x] + sVB[y + 1][x + 1] - sVB[y][x] - sVB[y][x + 1];
        const double duv = sqrt((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy));
        xk = dmin(chg[n] + c->dydc * duv, c->xkhmax);
      }
      sXK[ii][jj] = xk;
    }
  }
  __syncthreads();
  PT_MARK();
#undef sUB
#undef sVB
  // PGF log terms (:1996-2025): the u term is LU(j,i) - LU(j-1,i), the v term LV(j,i) - LV(j,i-1),
  // LU(j,i) = log(0.5*(psa(j,i) + psa(j,i-1))*hs + ptop), LV(j,i) = log(0.5*(psa(j,i) + psa(j-1,i))*hs
  // + ptop): each log is formed once per staged point instead of twice per output
  {
    const double hs = c->hsigma[k], pt = c->ptop;
    for (int t = tid; t < TW0 * MBI; t += MBT) {
      const int jj = t % TW0, ii = t / TW0;                  // (J0-1+jj, I0+ii)
      sX.l.LU[ii][jj] = rcm_log(d_half * (sPS[ii + 1][jj] + sPS[ii][jj]) * hs + pt);
    }
    for (int t = tid; t < MBJ * TH0; t += MBT) {
      const int jj = t % MBJ, ii = t / MBJ;                  // (J0+jj, I0-1+ii)
      sX.l.LV[ii][jj] = rcm_log(d_half * (sPS[ii][jj + 1] + sPS[ii][jj]) * hs + pt);
    }
  }
  __syncthreads();
  PT_MARK();
  if (!valid) return;
  const double dt = s->dt;
  // tile coordinates of (j,i): halo-1 tiles (b1,a1), halo-2 (b2,a2), low-halo (b0,a0)
  const int b1 = tj + 1, a1 = ti + 1, b2 = tj + 2, a2 = ti + 2, b0 = tj + 1, a0 = ti + 1;
#define UMC(dj, di) sUMC[a1 + (di)][b1 + (dj)]
#define VMC(dj, di) sVMC[a1 + (di)][b1 + (dj)]
#define UD(dj, di) sUD[a1 + (di)][b1 + (dj)]
#define VD(dj, di) sVD[a1 + (di)][b1 + (dj)]
  // hadvuv (upstream, hydrostatic)
  double ut, vt;
  {
    const double ucmona = UMC(0, 1) + d_two * UMC(0, 0) + UMC(0, -1);
    double ucmonb = UMC(1, 1) + d_two * UMC(1, 0) + UMC(1, -1);
    double ucmonc = UMC(-1, 1) + d_two * UMC(-1, 0) + UMC(-1, -1);
    const double vcmona = VMC(1, 0) + d_two * VMC(0, 0) + VMC(-1, 0);
    double vcmonb = VMC(1, 1) + d_two * VMC(0, 1) + VMC(-1, 1);
    double vcmonc = VMC(1, -1) + d_two * VMC(0, -1) + VMC(-1, -1);
    const double u0 = UD(0, 0), ue = UD(1, 0), uw = UD(-1, 0), un = UD(0, 1), us = UD(0, -1);
    const double v0 = VD(0, 0), ve = VD(1, 0), vw = VD(-1, 0), vn = VD(0, 1), vs = VD(0, -1);
    const double ul = c->ul;
    const double ff1 = ul * (ue + u0), ff2 = ul * (uw + u0), ff3 = ul * (vn + v0), ff4 = ul * (vs + v0);
    ucmonb = (d_one + ff1) * ucmona + (d_one - ff1) * ucmonb;
    ucmonc = (d_one + ff2) * ucmonc + (d_one - ff2) * ucmona;
    vcmonb = (d_one + ff3) * vcmona + (d_one - ff3) * vcmonb;
    vcmonc = (d_one + ff4) * vcmonc + (d_one - ff4) * vcmona;
    const double dm = dmsf;
    ut = d_zero - dm * ((ue + u0) * ucmonb - (u0 + uw) * ucmonc + (un + u0) * vcmonb - (u0 + us) * vcmonc);
    vt = d_zero - dm * ((ve + v0) * ucmonb - (v0 + vw) * ucmonc + (vn + v0) * vcmonb - (v0 + vs) * vcmonc);
  }
#undef UMC
#undef VMC
#undef UD
#undef VD
  // vadvuv: flux at interface k (from loop index k) then interface k+1 (loop index k+1)
  {
#define QQ(S) (d_rfour * (S[a0][b0] + S[a0][b0 - 1] + S[a0 - 1][b0] + S[a0 - 1][b0 - 1]))
    if (k >= 2) {
      const double qq = QQ(sQ0);
      const double uu = qq * (c->twt1[k] * u1c + c->twt2[k] * u1m);
      const double vv = qq * (c->twt1[k] * v1c + c->twt2[k] * v1m);
      ut = ut + uu * c->xds[k];
      vt = vt + vv * c->xds[k];
    }
    if (k + 1 <= kz) {
      const double qq = QQ(sQ1);
      const double uu = qq * (c->twt1[k + 1] * u1p + c->twt2[k + 1] * u1c);
      const double vv = qq * (c->twt1[k + 1] * v1p + c->twt2[k + 1] * v1c);
      ut = ut - uu * c->xds[k];
      vt = vt - vv * c->xds[k];
    }
#undef QQ
  }
  // curvature (hydrostatic Coriolis)
  ut = ut + cor * v1c;
  vt = vt - cor * u1c;
  // nudgeuv (iboudy 1/5); the sponge of iboudy = 4 (spongeuv, Main/mod_bdycod.F90:2735-2813)
  // acts on the still-zero total tendency, so it enters as the first summand below
  double spu = d_zero, spv = d_zero;
  if (rgd > 0 && c->iboudy == 4) {
    const int ib = f.ibdt[o2 >> 3];
    spu = c->wgtd[ib] * d_zero + (d_one - c->wgtd[ib]) * LD(f.ubt, o3);
    spv = c->wgtd[ib] * d_zero + (d_one - c->wgtd[ib]) * LD(f.vbt, o3);
  } else if (rgd > 0) {
    const double xt = s->xbctime + dt;
    double xf, xg;
    const int ib = f.ibdt[o2 >> 3];
    if (c->iboudy == 1) { xf = c->fcx[ib]; xg = c->gcx[ib]; } else { xf = c->hefc[ib][k]; xg = c->hegc[ib][k]; }
#define FGU(dj, di) ((LD(f.ub0, O3(dj, di)) + xt * LD(f.ubt, O3(dj, di))) - LD(f.a2u, O3(dj, di)))
#define FGV(dj, di) ((LD(f.vb0, O3(dj, di)) + xt * LD(f.vbt, O3(dj, di))) - LD(f.a2v, O3(dj, di)))
    ut = relax(ut, xf, xg, FGU(0, 0), FGU(-1, 0), FGU(1, 0), FGU(0, -1), FGU(0, 1));
    vt = relax(vt, xf, xg, FGV(0, 0), FGV(-1, 0), FGV(1, 0), FGV(0, -1), FGV(0, 1));
#undef FGU
#undef FGV
  }
  // diffu_d (idiffu = 1); xkd from calc_coeff (Main/mod_diffusion.F90:237-248)
  if (c->idiffu == 3) {                     // the column term of k_diffu6
    if (j == g.jdi2 || (!g.bl && j == g.jde1 - 1)) {
      ut = ut + LD(f.d6u, o3);
      vt = vt + LD(f.d6v, o3);
    }
  } else {
    double xkd = d_rfour * (sXK[a0][b0] + sXK[a0 - 1][b0 - 1] + sXK[a0 - 1][b0] + sXK[a0][b0 - 1]);
    xkd = xkd * c->rdxsq * pdotb;
#define UM(S, dj, di) S[a2 + (di)][b2 + (dj)]
    if (c->idiffu == 2) {                   // 9-point scheme on jdi x idi, :386-411
      ut = ut + xkd * (o4_c1 * (UM(sUM, 1, 0) + UM(sUM, -1, 0) + UM(sUM, 0, 1) + UM(sUM, 0, -1)) +
                       o4_c2 * (UM(sUM, 1, 1) + UM(sUM, -1, -1) + UM(sUM, -1, 1) + UM(sUM, 1, -1)) +
                       o4_c3 * (UM(sUM, 0, 0)));
      vt = vt + xkd * (o4_c1 * (UM(sVM, 1, 0) + UM(sVM, -1, 0) + UM(sVM, 0, 1) + UM(sVM, 0, -1)) +
                       o4_c2 * (UM(sVM, 1, 1) + UM(sVM, -1, -1) + UM(sVM, -1, 1) + UM(sVM, 1, -1)) +
                       o4_c3 * (UM(sVM, 0, 0)));
    } else if (g.gdii(j, i)) {
      ut = ut - xkd * (z4_c1 * (UM(sUM, 2, 0) + UM(sUM, -2, 0) + UM(sUM, 0, 2) + UM(sUM, 0, -2)) +
                       z4_c2 * (UM(sUM, 1, 0) + UM(sUM, -1, 0) + UM(sUM, 0, 1) + UM(sUM, 0, -1)) +
                       z4_c3 * (UM(sUM, 0, 0)));
      vt = vt - xkd * (z4_c1 * (UM(sVM, 2, 0) + UM(sVM, -2, 0) + UM(sVM, 0, 2) + UM(sVM, 0, -2)) +
                       z4_c2 * (UM(sVM, 1, 0) + UM(sVM, -1, 0) + UM(sVM, 0, 1) + UM(sVM, 0, -1)) +
                       z4_c3 * (UM(sVM, 0, 0)));
    }
#define LAPD()                                                                                        \
  ut = ut + xkd * (z4_c1 * (UM(sUM, 1, 0) + UM(sUM, -1, 0) + UM(sUM, 0, 1) + UM(sUM, 0, -1)) +        \
                   z4_c2 * (UM(sUM, 0, 0)));                                                          \
  vt = vt + xkd * (z4_c1 * (UM(sVM, 1, 0) + UM(sVM, -1, 0) + UM(sVM, 0, 1) + UM(sVM, 0, -1)) +        \
                   z4_c2 * (UM(sVM, 0, 0)));
    if (c->idiffu == 1) {
      if (g.gjeq(j, 2)) { LAPD(); }
      if (g.gjeq(j, g.gjx - 1)) { LAPD(); }
      if (i == 2) { LAPD(); }
      if (i == g.giy - 1) { LAPD(); }
    }
#undef LAPD
#undef UM
  }
  // pressure gradient force, part 1 (ipgf = 0) and part 2 (geopotential gradient)
  {
    double rtbar = d_rfour * (sTV[a0 - 1][b0 - 1] + sTV[a0][b0 - 1] + sTV[a0 - 1][b0] + sTV[a0][b0]);
    if (c->ipgf == 1)                       // reference-atmosphere temperature, :1945-1946
      rtbar = rtbar - T00PG * rcm_powpos((c->hsigma[k] * pdota + c->ptop) / P00PG, c->pgfaa1);
    rtbar = c->rgas * rtbar * pdota;
    const double den = c->dx * mfd;
    ut = ut - rtbar * (sX.l.LU[ti][tj + 1] - sX.l.LU[ti][tj]) / den;
    vt = vt - rtbar * (sX.l.LV[ti + 1][tj] - sX.l.LV[ti][tj]) / den;
    const double den2 = c->dx2 * mfd;
    const double pd = pdota;
    const double f00 = sPH[a0][b0], f0m = sPH[a0 - 1][b0], fm0 = sPH[a0][b0 - 1], fmm = sPH[a0 - 1][b0 - 1];
    ut = ut - pd * (f00 + f0m - fm0 - fmm) / den2;
    vt = vt - pd * (f00 + fm0 - f0m - fmm) / den2;
  }
  // totals uten + udyn + uphy (Main/mod_tendency.F90:404-411), forecast, RA filter
  // (pc_physic of the coupling seam, loaded here to keep registers free: absent = 0)
  ut = (spu + ut) + (f.uphy ? LD(f.uphy, o3) : d_zero);
  vt = (spv + vt) + (f.vphy ? LD(f.vphy, o3) : d_zero);
  if (f.uten) { ST(f.uten, o3, ut); ST(f.vten, o3, vt); }
  const double g1 = c->gnu1;
  const double u2 = u2c, v2 = v2c;
  const double cu = u2 + dt * ut, cv = v2 + dt * vt;
  double d = g1 * (cu + u2 - d_two * u1c);
  ST(f.b2u, o3, u1c + d);
  ST(f.b1u, o3, cu);
  d = g1 * (cv + v2 - d_two * v1c);
  ST(f.b2v, o3, v1c + d);
  ST(f.b1v, o3, cv);
  PT_PRINT(2);
}
__global__ __launch_bounds__(MBT, MO_LB) void k_momentum(Geom g, const Consts* __restrict__ c,
                                                     const StepState* __restrict__ s, Fields f) {
  __shared__ MomLDS L;
  momentum_block(g, c, s, f, L, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// ---------------------------------------------------------------------------------------
// K4. Scalars at the cross points jce x ice, one level per block of SBJ x SBI points:
//  temperature: hadvt + vadv3d + omega + adiabatic + nudge3d + diffu_x3d, forecast and RA
//    filter (Main/mod_tendency.F90:1200-1214, 1327-1341, 1561-1575, 1469, 1525, 285-287,
//    368-374, 422);
//  moisture (before the negative-value fix): hadvqv + vadvqv + nudge4d3d + diffu_x4d (qv),
//    hadvqx + vadv4d(ind=1) + diffu_x4d (qc), forecast (:1361-1392, 1470, 1526, 292-294,
//    332-349, 375-380).
// The stencil operands are staged in LDS once for the block and its halo, with the decoupled
// products formed once per staged point: umc/vmc/ud/vd at the dot points (j..j+1, i..i+1),
// p*, t, qv, qc (atm1 * rpsa) with halo 1 and the mkslice fields atm2 * (1/psb) with halo 2.
// The interior ring (jce \ jci) only passes atm2 moisture to the forecast buffers.
constexpr int SDW = SBJ + 1, SDH = SBI + 1;    // dot points j..j+SBJ, i..i+SBI
constexpr int SW1 = SBJ + 2, SH1 = SBI + 2;    // halo 1
constexpr int SW2 = SBJ + 4, SH2 = SBI + 4;    // halo 2

// x**y for x > 0 as exp(y*log(x)) with the fdlibm-class routines of fastmath.hpp: about 70
// VALU instructions against 226 for OCML pow, within a few ulp of it for the arguments here
// (layer pressure ratios, adjacent-level humidity ratios); the reference's libm pow differs
// from OCML's by ulps anyway (tests/test_parity_gpu.py bounds)
__device__ __forceinline__ double powpos(double x, double y) { return rcm_powpos(x, y); }


// The column terms, once per tend (blockIdx.z: 0 u and v, 1 t, 2 qv, 3 qc, 4.. the hydrometeors
// of nqx = 5; blockIdx.y = level):
// the coefficient (calc_coeff, :174-183: diff_6th_coef * p*dotb on dot points, * p*b on cross
// points) times the bracket, from the decoupled atm2 fields mkslice forms (ubd3d = u * 1/p*dotb,
// tb3d = t * 1/p*b, qxb3d clamped; Main/mod_slice.F90:163-183) on the 3-deep ghost rings the
// exchange of width idif = 3 fills.  k_momentum / k_scalars add them at the column's points in
// the reference's place of the diffusion term.
__global__ void k_diffu6(Geom g, const Consts* __restrict__ c, Fields f, QxArgs qx) {
  const int i = g.ide1 + (int)(blockIdx.x * blockDim.x + threadIdx.x), k = (int)blockIdx.y + 1;
  const int q = (int)blockIdx.z;
  const double* ps = f.psb;
  if (q == 0) {
    const int j = g.jdi2;
    if (!in(i, g.idi1, g.idi2)) return;
    auto rd = [&](int jj, int ii) { return d_one / psc2psd_global(g, ps, jj, ii); };
    auto uu = [&](int jj, int ii) { return F3(f.a2u, jj, ii, k) * rd(jj, ii) / F2(f.msfd, jj, ii); };
    auto vv = [&](int jj, int ii) { return F3(f.a2v, jj, ii, k) * rd(jj, ii) / F2(f.msfd, jj, ii); };
    const double xkd = c->diff6 * psc2psd_global(g, ps, j, i);
    F3(f.d6u, j, i, k) = xkd * diffu6_bracket(j, i, g.gjx, g.giy, uu, uu);
    F3(f.d6v, j, i, k) = xkd * diffu6_bracket(j, i, g.gjx, g.giy, vv, vv);
    return;
  }
  const int j = g.jci2;
  if (!in(i, g.ici1, g.ici2)) return;
  const double* a = q == 1 ? f.a2t : (q == 2 ? f.a2qv : (q == 3 ? f.a2qc : qx.a2[q - 4]));
  const double lo = q == 2 ? MINQQ : d_zero;
  auto fv = [&](int jj, int ii) {
    const double v = F3(a, jj, ii, k) * (d_one / F2(ps, jj, ii));
    return q == 1 ? v : dmax(v, lo);
  };
  auto lv = [&](int jj, int ii) { return fv(jj, ii) / F2(f.msfd, jj, ii); };
  const double xkc = d_one * (c->diff6 * F2(ps, j, i));
  F3(q == 1 ? f.d6t : (q == 2 ? f.d6qv : (q == 3 ? f.d6qc : qx.d6[q - 4])), j, i, k) =
      xkc * diffu6_bracket(j, i, g.gjx - 1, g.giy - 1, fv, lv);
}

// diffu_x (idiffu = 1) at one point from a halo-2 LDS tile, Main/mod_diffusion.F90:673-713
#define H2T(S, dj, di) S[a2 + (di)][b2 + (dj)]
#define DIFFU_X(ften, S, D6)                                                                      \
  do {                                                                                            \
    if (c->idiffu == 3) {                   /* the column term of k_diffu6 */                     \
      if (j == g.jci2 || (!g.bl && j == g.jce1 - 1)) ften = ften + LD(D6, o3);                    \
      break;                                                                                      \
    }                                                                                             \
    if (c->idiffu == 2) {                   /* 9-point scheme, :726-735, 881-891 */               \
      ften = ften + d_one * xkcs *                                                                \
          (o4_c1 * (H2T(S, 1, 0) + H2T(S, -1, 0) + H2T(S, 0, 1) + H2T(S, 0, -1)) +                \
           o4_c2 * (H2T(S, 1, 1) + H2T(S, -1, -1) + H2T(S, -1, 1) + H2T(S, 1, -1)) +              \
           o4_c3 * H2T(S, 0, 0));                                                                 \
      break;                                                                                      \
    }                                                                                             \
    if (g.gcii(j, i))                                                                             \
      ften = ften - d_one * xkcs *                                                                \
          (z4_c1 * (H2T(S, 2, 0) + H2T(S, -2, 0) + H2T(S, 0, 2) + H2T(S, 0, -2)) +                \
           z4_c2 * (H2T(S, 1, 0) + H2T(S, -1, 0) + H2T(S, 0, 1) + H2T(S, 0, -1)) +                \
           z4_c3 * H2T(S, 0, 0));                                                                 \
    if (g.gjeq(j, 2)) ften = ften + d_one * xkcs * (z4_c1 * (H2T(S, 1, 0) + H2T(S, -1, 0) + \
        H2T(S, 0, 1) + H2T(S, 0, -1)) + z4_c2 * H2T(S, 0, 0));                                   \
    if (g.gjeq(j, g.gjx - 2)) ften = ften + d_one * xkcs * (z4_c1 * (H2T(S, 1, 0) + H2T(S, -1, 0) + \
        H2T(S, 0, 1) + H2T(S, 0, -1)) + z4_c2 * H2T(S, 0, 0));                                   \
    if (i == 2) ften = ften + d_one * xkcs * (z4_c1 * (H2T(S, 1, 0) + H2T(S, -1, 0) + \
        H2T(S, 0, 1) + H2T(S, 0, -1)) + z4_c2 * H2T(S, 0, 0));                                   \
    if (i == g.giy - 2) ften = ften + d_one * xkcs * (z4_c1 * (H2T(S, 1, 0) + H2T(S, -1, 0) + \
        H2T(S, 0, 1) + H2T(S, 0, -1)) + z4_c2 * H2T(S, 0, 0));                                   \
  } while (0)

// qfuse, k_scalars at an owned point: k_qfilter's work for one moisture forecast fq (n = 0 qv,
// 1 qc).  A non-negative forecast is final (the negative-moisture fix, Main/mod_tendency.F90:
// 382-393, rewrites negative ones only), so its RAW filter (:424-427) against the RA-filtered
// p* (:420: psc, psa + gnu1 (psc + psb - 2 psa)) is done here into the next buffers; a
// negative one is listed for k_split_project's fix-up blocks.  The atm1/atm2 values are
// loaded again here (lines the thread read before): holding them from the vertical fluxes on
// costs k_scalars registers.
__device__ __forceinline__ void scalars_qraw(const Consts* __restrict__ c, const Fields& f, int n, double fq,
                                          uint32_t o2, uint32_t o3, double ps, double pb) {
  if (fq < d_zero) {
    f.neglist[atomicAdd(f.negcnt, 1)] = (o3 >> 3) * 2u + (uint32_t)n;
    return;
  }
  const double psc = LD(f.psc, o2);
  const double pbn = ps + c->gnu1 * (psc + pb - d_two * ps);
  double n1, n2;
  raw_filter(c, n, fq, LD(n ? f.a1qc : f.a1qv, o3), LD(n ? f.a2qc : f.a2qv, o3), psc, pbn, n1, n2);
  ST(n ? f.b1qc : f.b1qv, o3, n1);
  ST(n ? f.b2qc : f.b2qv, o3, n2);
}

// LDS of one k_scalars block
struct ScaLDS {
  double sUMC[SDH][SDW], sVMC[SDH][SDW], sUD[SDH][SDW], sVD[SDH][SDW], sUB[SDH][SDW], sVB[SDH][SDW];
  double sPS[SH1][SW1], sXT[SH1][SW1], sXQV[SH1][SW1], sXQC[SH1][SW1];
  double sTB[SH2][SW2], sQVB[SH2][SW2], sQCB[SH2][SW2];
};
__device__ __forceinline__ void scalars_block(const Geom& g, const Consts* __restrict__ c,
                                              const StepState* __restrict__ s, const Fields& f, ScaLDS& L,
                                              int bx, int by, int bz) {
  auto& sUMC = L.sUMC; auto& sVMC = L.sVMC; auto& sUD = L.sUD; auto& sVD = L.sVD; auto& sUB = L.sUB;
  auto& sVB = L.sVB; auto& sPS = L.sPS; auto& sXT = L.sXT; auto& sXQV = L.sXQV; auto& sXQC = L.sXQC;
  auto& sTB = L.sTB; auto& sQVB = L.sQVB; auto& sQCB = L.sQCB;
  const int tid = threadIdx.x;
  PT_DECL
  // the tile's cross points and its ghost ring (k_qfilter's moisture fix reads the forecasts
  // there); boundary branches test global indices
  const int J0 = (f.pt.part ? f.pt.sj0 : g.jcx1()) + bx * SBJ, I0 = g.icx1() + by * SBI;
  const int k = bz + 1;
  if (part_skip(f.pt, J0 - 2, J0 + SBJ + 1, I0 - 2, I0 + SBI + 1)) return;   // the staged halo-2 tile
  const uint32_t P8 = g.P8, L8 = g.L8;
  const uint32_t kof = (uint32_t)(k - 1) * L8;
  const int jlo = g.j0, jhi = g.j0 + g.nj - 1, ilo = g.i0, ihi = g.i0 + g.ni - 1;
  const int kz = c->kz;
  (void)P8;
  // this thread's point and its point operands, loaded before the staging barrier
  const int tj = tid % SBJ, ti = tid / SBJ;
  const int j = J0 + tj, i = I0 + ti;
  const bool valid = j >= g.jcx1() && j <= g.jcx2() && i <= g.icx2();
  const uint32_t o2 = valid ? g.o2(j, i) : g.o2(g.jce1, g.ice1), o3 = o2 + kof;
  const double t1 = LD(f.a1t, o3), t2 = LD(f.a2t, o3), qv2 = LD(f.a2qv, o3), qc2 = LD(f.a2qc, o3);
  const double qv1 = LD(f.a1qv, o3), qc1 = LD(f.a1qc, o3);
  const double t1m = (k >= 2) ? LD(f.a1t, o3 - L8) : 0.0, qv1m = (k >= 2) ? LD(f.a1qv, o3 - L8) : 0.0;
  const double qc1m = (k >= 2) ? LD(f.a1qc, o3 - L8) : 0.0;
  const double t1p = (k < kz) ? LD(f.a1t, o3 + L8) : 0.0, qv1p = (k < kz) ? LD(f.a1qv, o3 + L8) : 0.0;
  const double qc1p = (k < kz) ? LD(f.a1qc, o3 + L8) : 0.0;
  const double q0 = LD(f.qdot, o3), q1 = LD(f.qdot, o3 + L8);
  const double xm = LD(f.xmsf, o2), rp = LD(f.rpsa, o2), pb = LD(f.psb, o2), mx = LD(f.msfx, o2);
  const double ptn = LD(f.pten, o2), hgf = LD(f.hgfact, o2);
  const int rgc = f.rgcr[o2 >> 3];
  // ---- stage.  Every global load of the three staging sets is issued before the first LDS
  // write, so the block waits one memory latency instead of one per set and slot; lanes past
  // the tile or the frame read this thread's own (valid) address and stage zero.
  constexpr int NA = (SDW * SDH + SBT - 1) / SBT, NB = (SW1 * SH1 + SBT - 1) / SBT;
  constexpr int NC = (SW2 * SH2 + SBT - 1) / SBT;
  double au[NA], av[NA], am[NA], ar[NA], arb[NA], au2[NA], av2[NA];
  double bps[NB], brp[NB], bt[NB], bqv[NB], bqc[NB];
  double crb[NC], ct2[NC], cqv[NC], cqc[NC];
  bool aok[NA], bok[NB], cok[NC];
#pragma unroll
  for (int n = 0; n < NA; n++) {
    const int t = tid + n * SBT, jg = J0 + t % SDW, ig = I0 + t / SDW;
    aok[n] = t < SDW * SDH && jg <= jhi && ig <= ihi;
    const uint32_t q2 = aok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < SDW * SDH) {          // waves wholly past the staged tile skip the loads
      au[n] = LD(f.a1u, q3); av[n] = LD(f.a1v, q3); am[n] = LD(f.msfd, q2); ar[n] = LD(f.rpsda, q2);
      arb[n] = LD(f.rpsdb, q2); au2[n] = LD(f.a2u, q3); av2[n] = LD(f.a2v, q3);
    } else {
      au[n] = av[n] = am[n] = ar[n] = arb[n] = au2[n] = av2[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < NB; n++) {
    const int t = tid + n * SBT, jg = J0 - 1 + t % SW1, ig = I0 - 1 + t / SW1;
    bok[n] = t < SW1 * SH1 && jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = bok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < SW1 * SH1) {          // waves wholly past the staged tile skip the loads
      bps[n] = LD(f.psa, q2); brp[n] = LD(f.rpsa, q2);
      bt[n] = LD(f.a1t, q3); bqv[n] = LD(f.a1qv, q3); bqc[n] = LD(f.a1qc, q3);
    } else {
      bps[n] = brp[n] = bt[n] = bqv[n] = bqc[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < NC; n++) {
    const int t = tid + n * SBT, jg = J0 - 2 + t % SW2, ig = I0 - 2 + t / SW2;
    cok[n] = t < SW2 * SH2 && jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = cok[n] ? g.o2(jg, ig) : o2, q3 = q2 + kof;
    if (t < SW2 * SH2) {          // waves wholly past the staged tile skip the loads
      crb[n] = LD(f.rpsb, q2); ct2[n] = LD(f.a2t, q3); cqv[n] = LD(f.a2qv, q3); cqc[n] = LD(f.a2qc, q3);
    } else {
      crb[n] = ct2[n] = cqv[n] = cqc[n] = 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < NA; n++) {
    const int t = tid + n * SBT, jj = t % SDW, ii = t / SDW;
    if (t < SDW * SDH) {
      const bool ok = aok[n];
      sUMC[ii][jj] = ok ? au[n] * am[n] : 0.0; sVMC[ii][jj] = ok ? av[n] * am[n] : 0.0;
      sUD[ii][jj] = ok ? au[n] * ar[n] : 0.0; sVD[ii][jj] = ok ? av[n] * ar[n] : 0.0;
      sUB[ii][jj] = ok ? au2[n] * arb[n] : 0.0; sVB[ii][jj] = ok ? av2[n] * arb[n] : 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < NB; n++) {
    const int t = tid + n * SBT, jj = t % SW1, ii = t / SW1;
    if (t < SW1 * SH1) {
      const bool ok = bok[n];
      const double rp = brp[n];
      sPS[ii][jj] = ok ? bps[n] : 0.0;
      sXT[ii][jj] = ok ? bt[n] * rp : 0.0;
      sXQV[ii][jj] = ok ? dmax(bqv[n] * rp, MINQQ) : 0.0;
      sXQC[ii][jj] = ok ? dmax(bqc[n] * rp, d_zero) : 0.0;
    }
  }
#pragma unroll
  for (int n = 0; n < NC; n++) {
    const int t = tid + n * SBT, jj = t % SW2, ii = t / SW2;
    if (t < SW2 * SH2) {
      const bool ok = cok[n];
      const double r = crb[n];
      sTB[ii][jj] = ok ? ct2[n] * r : 0.0;
      sQVB[ii][jj] = ok ? dmax(cqv[n] * r, MINQQ) : 0.0;
      sQCB[ii][jj] = ok ? dmax(cqc[n] * r, d_zero) : 0.0;
    }
  }
  __syncthreads();
  PT_MARK();
  if (!valid) return;
#define DT(S, dj, di) S[ti + (di)][tj + (dj)]
  // calc_coeff Smagorinsky xkc, Main/mod_diffusion.F90:194-210 (ubd3d/vbd3d = atm2 * (1/psdotb))
  double xkc;
  {
    const double dudx = DT(sUB, 1, 0) + DT(sUB, 1, 1) - DT(sUB, 0, 0) - DT(sUB, 0, 1);
    const double dvdx = DT(sVB, 1, 0) + DT(sVB, 1, 1) - DT(sVB, 0, 0) - DT(sVB, 0, 1);
    const double dudy = DT(sUB, 0, 1) + DT(sUB, 1, 1) - DT(sUB, 0, 0) - DT(sUB, 1, 0);
    const double dvdy = DT(sVB, 0, 1) + DT(sVB, 1, 1) - DT(sVB, 0, 0) - DT(sVB, 1, 0);
    const double duv = sqrt((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy));
    xkc = dmin(hgf + c->dydc * duv, c->xkhmax);
  }
  if (!g.gci(j, i)) {
    ST(f.cqv, o3, qv2);
    ST(f.cqc, o3, qc2);
    if (f.xkcs) ST(f.xkcs, o3, xkc);
    return;
  }
  const double dt = s->dt;
  const int b1 = tj + 1, a1 = ti + 1, b2 = tj + 2, a2 = ti + 2;
#define H1T(S, dj, di) S[a1 + (di)][b1 + (dj)]
  // mass fluxes of the cell (shared by the three scalars)
  const double uavg1 = DT(sUMC, 0, 1) + DT(sUMC, 0, 0);
  const double uavg2 = DT(sUMC, 1, 1) + DT(sUMC, 1, 0);
  const double vavg1 = DT(sVMC, 1, 0) + DT(sVMC, 0, 0);
  const double vavg2 = DT(sVMC, 1, 1) + DT(sVMC, 0, 1);
  const double ps = H1T(sPS, 0, 0);
  const double xkcs = xkc * c->rdxsq * pb;
  if (f.xkcs) ST(f.xkcs, o3, xkcs);
  // ================= temperature
#if RCM_SC_TIMING_PART == 2
  if (0)
#endif
  {
    double td = d_zero + hadv_flux(c, xm, ps, uavg1, uavg2, vavg1, vavg2, H1T(sXT, 0, 0), H1T(sXT, -1, 0),
                                   H1T(sXT, 1, 0), H1T(sXT, 0, -1), H1T(sXT, 0, 1), 1);
    // vadv3d ind = 1 (Main/mod_advection.F90:771-783): pf/pb from psb (mkslice :263-271)
    {
      const double ptop = c->ptop, c287 = c->c287;
#if RCM_SC_TIMING_PART >= 3
#define powpos(x, y) ((x) + 0.0 * (y))
#endif
#define PF(K) ((c->sigma[K] * pb + ptop) * d_1000)
#define PB(K) ((c->hsigma[K] * pb + ptop) * d_1000)
      if (k >= 2)
        td = td + (q0 * (c->twt1[k] * t1 * powpos(PF(k) / PB(k), c287) +
                         c->twt2[k] * t1m * powpos(PF(k) / PB(k - 1), c287))) * c->xds[k];
      if (k + 1 <= kz)
        td = td - (q1 * (c->twt1[k + 1] * t1p * powpos(PF(k + 1) / PB(k + 1), c287) +
                         c->twt2[k + 1] * t1 * powpos(PF(k + 1) / PB(k), c287))) * c->xds[k];
#undef PB
#undef PF
#if RCM_SC_TIMING_PART >= 3
#undef powpos
#endif
    }
    // omega, Main/mod_tendency.F90:1200-1214
    double om;
    {
      const double dummy = d_one / (c->dx8 * mx);
      const double su = DT(sUD, 0, 0) + DT(sUD, 0, 1) + DT(sUD, 1, 1) + DT(sUD, 1, 0);
      const double sv = DT(sVD, 0, 0) + DT(sVD, 0, 1) + DT(sVD, 1, 1) + DT(sVD, 1, 0);
      const double x = su * (H1T(sPS, 1, 0) - H1T(sPS, -1, 0)) + sv * (H1T(sPS, 0, 1) - H1T(sPS, 0, -1));
      om = d_half * (q1 + q0) * ps + c->hsigma[k] * (ptn + x * dummy);
    }
    if (f.omega) ST(f.omega, o3, om);
    // adiabatic (hydrostatic), cpmf = cpd*(1+0.8 qv)
    {
      const double qv = H1T(sXQV, 0, 0);
      const double tv = H1T(sXT, 0, 0) * (d_one + c->ep1 * qv);
      const double rovcpm = c->rgas / (c->cpd * (d_one + 0.80 * qv));
      td = td + (om * rovcpm * tv) / (c->ptop * rp + c->hsigma[k]);
    }
    // nudge3d (iboudy 1/5) or the sponge3d summand (iboudy 4, see k_momentum)
    double spt = d_zero;
    if (rgc > 0 && c->iboudy == 4) {
      const int ib = f.ibcr[o2 >> 3];
      spt = c->wgtx[ib] * d_zero + (d_one - c->wgtx[ib]) * LD(f.tbt, o3);
    } else if (rgc > 0) {
      const double xtb = s->xbctime + dt;
      double xf, xg;
      nudge_coef(c, f.ibcr[o2 >> 3], k, xf, xg);
#define FGT(dj, di) ((LD(f.tb0, O3(dj, di)) + xtb * LD(f.tbt, O3(dj, di))) - LD(f.a2t, O3(dj, di)))
      td = relax(td, xf, xg, FGT(0, 0), FGT(-1, 0), FGT(1, 0), FGT(0, -1), FGT(0, 1));
#undef FGT
    }
    DIFFU_X(td, sTB, f.d6t);
    // tten + tdyn + tphy (:285-288), then the SUBEX condensation term (:332-341, stubbed)
    // (pc_physic of the coupling seam, loaded here to keep registers free: absent = 0)
    const double tt = ((spt + td) + (f.tphy ? LD(f.tphy, o3) : d_zero)) + d_zero;
    if (f.tten) ST(f.tten, o3, tt);
    const double ct = t2 + dt * tt;
    const double d = c->gnu1 * (ct + t2 - d_two * t1);
    ST(f.b2t, o3, t1 + d);
    ST(f.b1t, o3, ct);
  }
#if RCM_SC_TIMING_PART == 1 || RCM_SC_TIMING_PART == 3
  return;
#endif
  // ================= qv
  // hadvqv, or the semi-Lagrangian start of qxdyn from k_sladv (isladvec = 1, :1361-1363)
  double tq = c->isladvec ? LD(f.slqv, o3)
                          : d_zero + hadv_flux(c, xm, ps, uavg1, uavg2, vavg1, vavg2, H1T(sXQV, 0, 0),
                                               H1T(sXQV, -1, 0), H1T(sXQV, 1, 0), H1T(sXQV, 0, -1),
                                               H1T(sXQV, 0, 1), 2);
  {
    const double thr = MINQQ * ps;
    const double qc0 = qv1;
    if (k >= 2) {
      const double qm = qv1m;
      tq = tq + q0 * ((qc0 > thr && qm > thr) ? qc0 * powpos(qm / qc0, c->qcon[k]) : d_zero) * c->xds[k];
    }
    if (k + 1 <= kz) {
      const double qp = qv1p;
      tq = tq - q1 * ((qp > thr && qc0 > thr) ? qp * powpos(qc0 / qp, c->qcon[k + 1]) : d_zero) * c->xds[k];
    }
  }
  double spq = d_zero;
  if (rgc > 0 && c->iboudy == 4) {
    const int ib = f.ibcr[o2 >> 3];
    spq = c->wgtx[ib] * d_zero + (d_one - c->wgtx[ib]) * LD(f.qbt, o3);
  } else if (rgc > 0) {
    const double xtb = s->xbctime + dt;
    const double nfac = 1.0e3, rfac = d_one / nfac;
    double xf, xg;
    nudge_coef(c, f.ibcr[o2 >> 3], k, xf, xg);
#define FGQ(dj, di) (nfac * (LD(f.qb0, O3(dj, di)) + xtb * LD(f.qbt, O3(dj, di))) - nfac * LD(f.a2qv, O3(dj, di)))
    const double f0 = FGQ(0, 0), f1 = FGQ(-1, 0), f2 = FGQ(1, 0), f3 = FGQ(0, -1), f4 = FGQ(0, 1);
#undef FGQ
    tq = tq + rfac * (xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0));
  }
  DIFFU_X(tq, sQVB, f.d6qv);
  // the qv sums and forecast (and with qfuse its RAW filter) before the qc chain, so the qv
  // operands are dead while it runs
  tq = ((spq + tq) + (f.qvphy ? LD(f.qvphy, o3) : d_zero)) + d_zero;
  if (f.qvten) ST(f.qvten, o3, tq);
  const bool qown = f.qfuse && in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2);
  {
    const double fcqv = qv2 + dt * tq;
    ST(f.cqv, o3, fcqv);
    if (qown) scalars_qraw(c, f, 0, fcqv, o2, o3, ps, pb);
  }
  // ================= qc
  // hadvqx, or the semi-Lagrangian start of qxdyn (:1378-1380)
  double tc = c->isladvec ? LD(f.slqc, o3)
                          : d_zero + hadv_flux(c, xm, ps, uavg1, uavg2, vavg1, vavg2, H1T(sXQC, 0, 0),
                                               H1T(sXQC, -1, 0), H1T(sXQC, 1, 0), H1T(sXQC, 0, -1),
                                               H1T(sXQC, 0, 1), 0);
  if (f.kpbl) {
    // vadv4d ind = 3 (iuwvadv = 1): no positivity threshold, the PBL-top rule at kpbl
    const int kpb = (int)LD(f.kpbl, o2);
    auto fk = [&](int kk) { return LD(f.a1qc, o2 + (uint32_t)(kk - 1) * L8); };
    if (k >= 2) tc = tc + (uw_fg(c, k, kpb, qc1, qc1m, fk) * q0) * c->xds[k];
    if (k + 1 <= kz) tc = tc - (uw_fg(c, k + 1, kpb, qc1p, qc1, fk) * q1) * c->xds[k];
  } else {
    const double thr = MINQQ * MINQQ * ps;
    const double c0 = qc1;
    if (k >= 2) {
      const double cm = qc1m;
      const double fl = (q0 > d_zero) ? ((cm > thr) ? q0 * (c->twt1[k] * c0 + c->twt2[k] * cm) : d_zero)
                                      : ((c0 > thr) ? q0 * (c->twt1[k] * c0 + c->twt2[k] * cm) : d_zero);
      tc = tc + fl * c->xds[k];
    }
    if (k + 1 <= kz) {
      const double cp = qc1p;
      const double fl = (q1 > d_zero) ? ((c0 > thr) ? q1 * (c->twt1[k + 1] * cp + c->twt2[k + 1] * c0) : d_zero)
                                      : ((cp > thr) ? q1 * (c->twt1[k + 1] * cp + c->twt2[k + 1] * c0) : d_zero);
      tc = tc - fl * c->xds[k];
    }
  }
  DIFFU_X(tc, sQCB, f.d6qc);
#undef DT
#undef H1T
  tc = ((d_zero + tc) + (f.qcphy ? LD(f.qcphy, o3) : d_zero)) + d_zero;
  if (f.qcten) ST(f.qcten, o3, tc);
  {
    const double fcqc = qc2 + dt * tc;
    ST(f.cqc, o3, fcqc);
    if (qown) scalars_qraw(c, f, 1, fcqc, o2, o3, ps, pb);
  }
  PT_PRINT(3);
}
__global__ __launch_bounds__(SBT, SC_LB) void k_scalars(Geom g, const Consts* __restrict__ c,
                                                    const StepState* __restrict__ s, Fields f) {
  __shared__ ScaLDS L;
  scalars_block(g, c, s, f, L, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// k_momentum and k_scalars in one launch: blockIdx.z < kz a scalars block of level z + 1, else
// a momentum block of level z - kz + 1 (x/y: the larger of the two grids; a block past its own
// grid exits).  Both read only k_columns' outputs and the state and write disjoint buffers, so
// the two block sets are independent; one launch drains one tail instead of two, and with the
// longer scalars blocks dispatched first the momentum blocks fill it (C3, alternating on one
// box: 203.5-212.1 us/step against 211.2-222.9 with the momentum blocks first, 222.3-224.1
// interleaved by level, 218.8-223.6 as two launches).
__global__ __launch_bounds__(SBT, SC_LB) void k_update(Geom g, const Consts* __restrict__ c,
                                                   const StepState* __restrict__ s, Fields fm, Fields fs,
                                                   int mnx, int mny, int snx, int sny, int xcd) {
  __shared__ union { MomLDS m; ScaLDS s; } L;
  const int kz = c->kz, bz = (int)blockIdx.z;
  int bx = (int)blockIdx.x, by = (int)blockIdx.y;
  if (xcd) xcd_tile2d(bx, by);
  const bool mom = bz >= kz;
  const int lz = mom ? bz - kz : bz;
  if (mom) {
    if (bx < mnx && by < mny) momentum_block(g, c, s, fm, L.m, bx, by, lz);
  } else if (bx < snx && by < sny) {
    scalars_block(g, c, s, fs, L.s, bx, by, lz);
  }
}
#undef DIFFU_X
#undef H2T

// ---------------------------------------------------------------------------------------
// K6. Negative-moisture fix + the RA filter of p* + the RAW filter of qv/qc, one pass
// (Main/mod_tendency.F90:382-393, 420, 424-427; Main/mod_timefilter.F90 filter_ra_2d,
// filter_raw_qv, filter_raw_4d).  The reference sweeps each (k,n) plane in i-major / j-minor
// order and a fixed point reads already-fixed predecessors.  A negative point whose four
// predecessors (j-1,i) (j-1,i-1) (j,i-1) (j+1,i-1) inside the sweep are all non-negative
// only ever reads original values and is fixed (and filtered) here in parallel; the rare
// others are flagged per plane and resolved in sweep order by the serial blocks of
// k_split_project (nothing in splitf reads moisture).  Fixed values are stored only for
// negative points: a fixed predecessor is (cq < 0 ? fq : cq).  p* is filtered on the fly by
// every thread and stored by the k = 1 threads into the next p* buffers.

// Two adjacent points (j, j+1) per thread with 16-byte accesses (rows start 128-B aligned and
// pairs start at even j - j0); the second point of a pair may fall in the row padding.
#define LD2(a, o) (*(const double2*)((const char*)(a) + (uint32_t)(o)))
#define ST2(a, o, v) (*(double2*)((char*)(a) + (uint32_t)(o)) = (v))
#ifndef QF_LB
#define QF_LB 1
#endif
__global__ __launch_bounds__(256, QF_LB) void k_qfilter(Geom g, const Consts* __restrict__ c, Fields f) {
  PT_DECL
  const int jp = g.j0 + 2 * (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.i0 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int k = (int)blockIdx.z + 1;
  if (jp >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const uint32_t o2 = g.o2(jp, i), o3 = o2 + (uint32_t)(k - 1) * g.L8;
  // owned points (the moisture fix and filters)
  const bool ici = in(i, g.ici1, g.ici2);
  const bool ci0 = ici && in(jp, g.jci1, g.jci2), ci1 = ici && in(jp + 1, g.jci1, g.jci2);
  // points k_scalars (cross ring) and k_momentum (dot, right/top ring) updated; p* is filtered
  // on the cross ring too (k_split_project's psdota and the split corrections read it there)
  const bool icx = in(i, g.icx1(), g.icx2()), idx = in(i, g.idi1, g.bt ? g.idi2 : g.ide2 + 1);
  const int jd2 = g.br ? g.jdi2 : g.jde2 + 1;
  const bool xi0 = icx && in(jp, g.jcx1(), g.jcx2()) && g.gci(jp, i);
  const bool xi1 = icx && in(jp + 1, g.jcx1(), g.jcx2()) && g.gci(jp + 1, i);
  const bool di0 = idx && in(jp, g.jdi1, jd2), di1 = idx && in(jp + 1, g.jdi1, jd2);
  // every operand is loaded before the first store (the buffers are not __restrict__, so a
  // store would otherwise order the later loads behind it: one memory latency per field)
  double2 pa = LD2(f.psa, o2), pb = LD2(f.psb, o2);
  const double2 psc = LD2(f.psc, o2);
  const double2 cvq[2] = {LD2(f.cqv, o3), LD2(f.cqc, o3)};
  const double2 o1q[2] = {LD2(f.a1qv, o3), LD2(f.a1qc, o3)};
  const double2 o2q[2] = {LD2(f.a2qv, o3), LD2(f.a2qc, o3)};
  // p* RA filter on the fly (k = 1 threads store it)
  if (xi0) { const double d = c->gnu1 * (psc.x + pb.x - d_two * pa.x); pb.x = pa.x + d; pa.x = psc.x; }
  if (xi1) { const double d = c->gnu1 * (psc.y + pb.y - d_two * pa.y); pb.y = pa.y + d; pa.y = psc.y; }
  if (k == 1) { ST2(f.bpsa, o2, pa); ST2(f.bpsb, o2, pb); }
  // points k_momentum / k_scalars do not update keep their values in the next buffers
  {
    double2 x;
#define KEEP(dst, src, upd) x = LD2(dst, o3); { const double2 y = LD2(src, o3);              \
    if (!upd##0) x.x = y.x; if (!upd##1) x.y = y.y; } ST2(dst, o3, x);
    if (!(di0 && di1)) { KEEP(f.b1u, f.a1u, di) KEEP(f.b1v, f.a1v, di) KEEP(f.b2u, f.a2u, di) KEEP(f.b2v, f.a2v, di) }
    if (!(xi0 && xi1)) { KEEP(f.b1t, f.a1t, xi) KEEP(f.b2t, f.a2t, xi) }
#undef KEEP
  }
  if (!ci0 && !ci1) {
    ST2(f.b1qv, o3, o1q[0]); ST2(f.b1qc, o3, o1q[1]);
    ST2(f.b2qv, o3, o2q[0]); ST2(f.b2qc, o3, o2q[1]);
    return;
  }
#pragma unroll
  for (int n = 0; n < 2; n++) {
    const double* sv = n ? f.cqc : f.cqv;
    double* fx = n ? f.fqc : f.fqv;
    const double2 cv = cvq[n], o1 = o1q[n], o2v = o2q[n];
    double2 n1, n2;
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int j = jp + q;
      const bool ci = q ? ci1 : ci0;
      const double a1 = q ? o1.y : o1.x, a2 = q ? o2v.y : o2v.x;
      double r1 = a1, r2 = a2;                  // ring points keep their values
      if (ci) {
        double v = q ? cv.y : cv.x;
        bool done = true;
        if (v < d_zero) {
          if (negfix_dependent(g, sv, j, i, k)) {
            negfix_mark(g, f.depplane, n * c->kz + (k - 1), i);
            done = false;                       // fixed and filtered by the serial sweep
          } else {
            v = negfix_sum(g, sv, fx, j, i, k, false);
            F3(fx, j, i, k) = v;
          }
        }
        if (done) raw_filter(c, n, v, a1, a2, q ? pa.y : pa.x, q ? pb.y : pb.x, r1, r2);
      }
      if (q) { n1.y = r1; n2.y = r2; } else { n1.x = r1; n2.x = r2; }
    }
    ST2(n ? f.b1qc : f.b1qv, o3, n1);
    ST2(n ? f.b2qc : f.b2qv, o3, n2);
  }
  PT_PRINT(4);
}

// serial sweep of one flagged (n,k) plane by one wavefront (see K6)
__device__ __forceinline__ void negfix_serial_plane(Geom g, const Consts* c, QFix q, int plane_id, double* lds) {
  const int kz = c->kz;
  const int n = plane_id / kz, k = plane_id % kz + 1;
  if (q.depf) {                        // the list pass's row flags (one wavefront calls this)
    negfix_collect(g, q.depf, q.depplane, plane_id, (int)threadIdx.x & 63, 64);
    wave_lds_sync();
  }
  const double* o1 = n ? q.o1qc : q.o1qv;
  const double* o2 = n ? q.o2qc : q.o2qv;
  double* n1p = n ? q.n1qc : q.n1qv;
  double* n2p = n ? q.n2qc : q.n2qv;
  negfix_sweep(g, n ? q.cqc : q.cqv, n ? q.fqc : q.fqv, q.depplane, plane_id, k, lds, [=](int jj, int i, double v) {
    // the RA-filtered p* of the step (Main/mod_tendency.F90:420), formed again from psc and the
    // step's p* (with qfuse k_split_correct corrects psa/psb beside this sweep)
    double n1, n2;
    const double pc = F2(q.psc, jj, i), po = F2(q.opsa, jj, i);
    raw_filter(c, n, v, F3(o1, jj, i, k), F3(o2, jj, i, k), pc, po + c->gnu1 * (pc + F2(q.opsb, jj, i) - d_two * po),
               n1, n2);
    F3(n1p, jj, i, k) = n1;
    F3(n2p, jj, i, k) = n2;
  });
}

// qfuse with nqx = 5: the qv / qc planes' serial fix in a launch of its own after the split
// corrections, a block per plane (negfix_resolve: the dense wavefront or the row sweep); the
// filter of a fixed point from its atm1, atm2 and the step's p* (x = o1, o2, psc, opsa, opsb)
struct QvRaw {
  static constexpr int NI = 5;
  Geom g;
  const Consts* c;
  const double *o1, *o2, *psc, *opsa, *opsb;
  double *n1p, *n2p;
  int n, k;
  __device__ void load(int j, int i, double* x) const {
    x[0] = F3(o1, j, i, k); x[1] = F3(o2, j, i, k);
    x[2] = F2(psc, j, i); x[3] = F2(opsa, j, i); x[4] = F2(opsb, j, i);
  }
  __device__ void apply(int j, int i, double v, const double* x) const {
    double n1, n2;
    const double pc = x[2], po = x[3];
    raw_filter(c, n, v, x[0], x[1], pc, po + c->gnu1 * (pc + x[4] - d_two * po), n1, n2);
    F3(n1p, j, i, k) = n1;
    F3(n2p, j, i, k) = n2;
  }
};
__global__ __launch_bounds__(512) void k_negfix_serial(Geom g, const Consts* __restrict__ c, QFix q) {
  extern __shared__ double lds[];
  const int plane = (int)blockIdx.x, kz = c->kz, n = plane / kz, k = plane % kz + 1;
  if (q.depf) {
    negfix_collect(g, q.depf, q.depplane, plane, (int)threadIdx.x, (int)blockDim.x);
    __syncthreads();
  }
  if (NEGFIX_POST) {
    negfix_resolve(g, n ? q.cqc : q.cqv, n ? q.fqc : q.fqv, q.depplane, plane, k, lds, negfix_lds(g), NoPost{},
                   [](int, int, double) {}, c->negfix_mode);
    return;
  }
  const QvRaw acc{g, c, n ? q.o1qc : q.o1qv, n ? q.o2qc : q.o2qv, q.psc, q.opsa, q.opsb,
                  n ? q.n1qc : q.n1qv, n ? q.n2qc : q.n2qv, n, k};
  negfix_resolve(g, n ? q.cqc : q.cqv, n ? q.fqc : q.fqv, q.depplane, plane, k, lds, negfix_lds(g), acc,
                 [=](int jj, int i, double v) {
                   double x[5];
                   acc.load(jj, i, x);
                   acc.apply(jj, i, v, x);
                 }, c->negfix_mode);
}

// NEGFIX_POST: the filters of the points k_negfix_serial fixed, a thread per interior point of
// a (qv | qc, level) plane (z = plane)
__global__ void k_negfix_post(Geom g, const Consts* __restrict__ c, QFix q) {
  const int j = g.jci1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ici1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int plane = (int)blockIdx.z, kz = c->kz, n = plane / kz, k = plane % kz + 1;
  if (j > g.jci2 || i > g.ici2) return;
  const double* sv = n ? q.cqc : q.cqv;
  if (!negfix_is_dependent(g, sv, j, i, k)) return;
  const QvRaw acc{g, c, n ? q.o1qc : q.o1qv, n ? q.o2qc : q.o2qv, q.psc, q.opsa, q.opsb,
                  n ? q.n1qc : q.n1qv, n ? q.n2qc : q.n2qv, n, k};
  double x[5];
  acc.load(j, i, x);
  acc.apply(j, i, F3(n ? q.fqc : q.fqv, j, i, k), x);
}

// qfuse: k_qfilter's fix of the negative forecasts k_scalars listed, one entry per thread
// (grid-stride over the list): an independent negative point (no negative sweep-predecessor)
// is fixed and RAW-filtered here, a dependent one flags its plane for the serial sweep
// (k_split_correct's extra blocks, after this launch)
__device__ __forceinline__ void negfix_list(Geom g, const Consts* c, QFix q, int t0, int stride) {
  const int cnt = *q.negcnt;
  for (int e = t0; e < cnt; e += stride) {
    const uint32_t w = q.neglist[e];
    const int n = (int)(w & 1u);
    const long el = (long)(w >> 1);
    const int k = (int)(el / g.plane) + 1;
    const long r = el % g.plane;
    const int i = g.i0 + (int)(r / g.pitch), j = g.j0 + (int)(r % g.pitch);
    const double* sv = n ? q.cqc : q.cqv;
    if (negfix_dependent(g, sv, j, i, k)) {
      if (q.depf) q.depf[(n * c->kz + (k - 1)) * (g.ici2 - g.ici1 + 1) + (i - g.ici1)] = 1u;
      else negfix_mark(g, q.depplane, n * c->kz + (k - 1), i);
      continue;
    }
    double* fx = n ? q.fqc : q.fqv;
    const double v = negfix_sum(g, sv, fx, j, i, k, false);
    F3(fx, j, i, k) = v;
    double n1, n2;
    raw_filter(c, n, v, F3(n ? q.o1qc : q.o1qv, j, i, k), F3(n ? q.o2qc : q.o2qv, j, i, k), F2(q.psa, j, i),
               F2(q.psb, j, i), n1, n2);
    F3(n ? q.n1qc : q.n1qv, j, i, k) = n1;
    F3(n ? q.n2qc : q.n2qv, j, i, k) = n2;
  }
}

// ---------------------------------------------------------------------------------------
// K7. splitf projections, Main/mod_split.F90:254-409, for 64 columns (j) of one row i per
// block: psdota (:259-260), deld/delh slots 1..3 and dstor/hstor refresh; slot(l, s) =
// base + ((s-1)*nsplit + l-1)*plane.  Phase 1: all four wavefronts compute each level's
// divergence of atm1/atm2 (shared by every vertical mode) and stage atm1/atm2 t in LDS;
// phase 2: one wavefront per (mode, divergence|geopotential) sum runs the k loop in the
// reference's order.  Blocks [nproj, nproj + 2 kz) run the serial negative-moisture sweeps
// (one plane each, usually an immediate exit).
#define SLOT(a, l, s) ((a) + ((long)((s) - 1) * c->nsplit + ((l) - 1)) * g.plane)
#ifndef SP_LB
#define SP_LB 5
#endif
#ifndef SP_KU
#define SP_KU 1
#endif
#ifndef SP_PF
#define SP_PF 1
#endif
__global__ __launch_bounds__(SPC * SPG, SP_LB) void k_split_project(
    Geom g, const Consts* __restrict__ c, const double* __restrict__ a1u, const double* __restrict__ a1v,
    const double* __restrict__ a2u, const double* __restrict__ a2v, const double* __restrict__ a1t,
    const double* __restrict__ a2t, const double* __restrict__ psa, const double* __restrict__ psb,
    const double* __restrict__ msfd, const double* __restrict__ mapf, double* dstor, double* hstor, double* deld,
    double* delh, double* psdota, int nxp, int nproj, QFix qf, Geom gw, double* wdeld, double* wdelh,
    double* wpsdota, double* wpsa, const double* __restrict__ o2u, const double* __restrict__ o2v) {
  extern __shared__ double lds[];                        // 4 x kz x SPC
  if ((int)blockIdx.x >= nproj) {
    const int b = blockIdx.x;
    if (qf.negcnt) negfix_list(g, c, qf, (b - nproj) * (int)blockDim.x + (int)threadIdx.x, ((int)gridDim.x - nproj) * (int)blockDim.x);
    else if (threadIdx.x < 64)
      negfix_serial_plane(g, c, qf, b - nproj, negfix_sweep_lds(g) <= 4 * c->kz * SPC ? lds : nullptr);
    return;
  }
  // SP_XCD: each XCD takes a contiguous run of column rows, so the i + 1 row of the u, v
  // divergence, which the next row's block loads as its own, is a hit in the same L2
  const int b = SP_XCD ? xcd_range((int)blockIdx.x, 0, nproj) : (int)blockIdx.x;
  PT_DECL
  const int tx = (int)threadIdx.x % SPC, ty = (int)threadIdx.x / SPC;
  // owned dot points, plus psdota on the right/top ghost ring (the split corrections of the
  // ghost-ring u, v read it there)
  const int j = g.jde1 + (b % nxp) * SPC + tx, i = g.ide1 + b / nxp;
  const bool valid = j <= g.jde2 && i <= g.ide2;
  const bool vpd = j <= g.jdx2() && i <= g.idx2();
  const bool ce = valid && in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2);
  const int kz = c->kz;
  double* sD1 = lds;
  double* sD2 = lds + kz * SPC;
  double* sT1 = lds + 2 * kz * SPC;
  double* sT2 = lds + 3 * kz * SPC;
  if (ty == 0) {
    double v;
    if (valid) {
      if (psc2psd_at(g, psa, j, i, v)) F2(psdota, j, i) = v;
    } else if (vpd) {
      F2(psdota, j, i) = psc2psd_global(g, psa, j, i);
    }
  }
  if (ce) {
    const double m00 = F2(msfd, j, i), m10 = F2(msfd, j + 1, i), m01 = F2(msfd, j, i + 1), m11 = F2(msfd, j + 1, i + 1);
    // qfuse: a ghost dot point k_momentum does not update (the boundary lines' ring points)
    // was not copied into the next atm2 buffers (keep_point): read it from the step's own
    const int jd2 = g.br ? g.jdi2 : g.jde2 + 1, id2 = g.bt ? g.idi2 : g.ide2 + 1;
    auto old_at = [&](int jj, int ii) {
      return qf.negcnt && !(in(jj, g.jde1, g.jde2) && in(ii, g.ide1, g.ide2)) &&
             !(in(jj, g.jdi1, jd2) && in(ii, g.idi1, id2));
    };
    const double* U01 = old_at(j, i + 1) ? o2u : a2u; const double* V01 = old_at(j, i + 1) ? o2v : a2v;
    const double* U11 = old_at(j + 1, i + 1) ? o2u : a2u; const double* V11 = old_at(j + 1, i + 1) ? o2v : a2v;
    const double* U10 = old_at(j + 1, i) ? o2u : a2u; const double* V10 = old_at(j + 1, i) ? o2v : a2v;
    // SP_KU levels per pass: every load of the pass is issued before any use
    for (int k0 = ty + 1; k0 <= kz; k0 += SPG * SP_KU) {
      double x[SP_KU][18];
#pragma unroll
      for (int n = 0; n < SP_KU; n++) {
        const int k = min(k0 + SPG * n, kz);
        x[n][0] = F3(a1u, j, i + 1, k); x[n][1] = F3(a1u, j + 1, i + 1, k);
        x[n][2] = F3(a1u, j, i, k); x[n][3] = F3(a1u, j + 1, i, k);
        x[n][4] = F3(a1v, j, i + 1, k); x[n][5] = F3(a1v, j + 1, i + 1, k);
        x[n][6] = F3(a1v, j, i, k); x[n][7] = F3(a1v, j + 1, i, k);
        x[n][8] = F3(U01, j, i + 1, k); x[n][9] = F3(U11, j + 1, i + 1, k);
        x[n][10] = F3(a2u, j, i, k); x[n][11] = F3(U10, j + 1, i, k);
        x[n][12] = F3(V01, j, i + 1, k); x[n][13] = F3(V11, j + 1, i + 1, k);
        x[n][14] = F3(a2v, j, i, k); x[n][15] = F3(V10, j + 1, i, k);
        x[n][16] = F3(a1t, j, i, k); x[n][17] = F3(a2t, j, i, k);
      }
#pragma unroll
      for (int n = 0; n < SP_KU; n++) {
        const int k = k0 + SPG * n;
        if (k > kz) break;
#define DIV(o) (-(x[n][o] * m01) + (x[n][o + 1] * m11) - (x[n][o + 2] * m00) + (x[n][o + 3] * m10) + \
                (x[n][o + 4] * m01) + (x[n][o + 5] * m11) - (x[n][o + 6] * m00) - (x[n][o + 7] * m10))
        sD1[(k - 1) * SPC + tx] = DIV(0);
        sD2[(k - 1) * SPC + tx] = DIV(8);
#undef DIV
        sT1[(k - 1) * SPC + tx] = x[n][16];
        sT2[(k - 1) * SPC + tx] = x[n][17];
      }
    }
  }
  // the 2-D operands of this thread's first (mode, sum) item are loaded before the barrier, so
  // their latency overlaps the wait instead of following it (SP_PF = 0: loaded where used)
  const int ns = c->nsplit;
  const long q = valid ? g.ix(j, i) : 0;
#if SP_PF
  double pf_st = 0.0, pf_a = 0.0, pf_b = 0.0;
  if (valid && ty < 2 * ns) {
    const int l = ty % ns + 1;
    if (ty < ns) {
      pf_st = dstor[(long)(l - 1) * g.plane + q];
      if (ce) pf_a = F2(mapf, j, i);
    } else {
      pf_st = hstor[(long)(l - 1) * g.plane + q];
      if (ce) { pf_a = F2(psa, j, i); pf_b = F2(psb, j, i); }
    }
  }
#endif
  __syncthreads();
  PT_MARK();
  if (!valid) return;
  const double rdx2 = d_one / c->dx2;
  // decomposed domain: the split step's inputs also go to the wide frame its exchange fills
  const long qw = wdeld ? gw.ix(j, i) : 0;
#define WSLOT(a, l, s) ((a) + ((long)((s) - 1) * c->nsplit + ((l) - 1)) * gw.plane)
  if (wdeld && ty == 0) {
    wpsa[qw] = F2(psa, j, i);
    wpsdota[qw] = F2(psdota, j, i);
  }
  for (int w = ty; w < 2 * ns; w += SPG) {
    const int l = w % ns + 1;
    const bool pf = SP_PF && w == ty;
    if (w < ns) {
      const double ds = pf ? pf_st : dstor[(long)(l - 1) * g.plane + q];
      double d3 = d_zero, d2 = d_zero;
      if (ce) {
        const double mf = pf ? pf_a : F2(mapf, j, i);
        for (int k = 1; k <= kz; k++) {
          const double zr = c->zmatxr[l - 1][k - 1];
          d3 = d3 + zr * rdx2 * mf * sD1[(k - 1) * SPC + tx];
          d2 = d2 + zr * rdx2 * mf * sD2[(k - 1) * SPC + tx];
        }
      }
      SLOT(deld, l, 1)[q] = ds - d2;
      SLOT(deld, l, 2)[q] = d2;
      SLOT(deld, l, 3)[q] = d3 - ds;
      if (wdeld) { WSLOT(wdeld, l, 1)[qw] = ds - d2; WSLOT(wdeld, l, 2)[qw] = d2; WSLOT(wdeld, l, 3)[qw] = d3 - ds; }
      dstor[(long)(l - 1) * g.plane + q] = d2;
    } else {
      const double hs = pf ? pf_st : hstor[(long)(l - 1) * g.plane + q];
      double h3 = d_zero, h2 = d_zero;
      if (ce) {
        const double pa = pf ? pf_a : F2(psa, j, i), pbv = pf ? pf_b : F2(psb, j, i);
        const double rpa = d_one / pa, rpbv = d_one / pbv;
        h3 = c->pdlog[l - 1][kz + 1] + c->eps1[l - 1][kz + 1] * (pa - c->pd);
        h2 = c->pdlog[l - 1][kz + 1] + c->eps1[l - 1][kz + 1] * (pbv - c->pd);
        for (int k = 1; k <= kz; k++) {
          const double ta = c->tau[l - 1][k - 1], pdk = c->pdlog[l - 1][k], ek = c->eps1[l - 1][k];
          h3 = h3 + pdk + div_by(ta * sT1[(k - 1) * SPC + tx], pa, rpa) + ek * (pa - c->pd);
          h2 = h2 + pdk + div_by(ta * sT2[(k - 1) * SPC + tx], pbv, rpbv) + ek * (pbv - c->pd);
        }
      }
      SLOT(delh, l, 1)[q] = hs - h2;
      SLOT(delh, l, 2)[q] = h2;
      SLOT(delh, l, 3)[q] = h3 - hs;
      if (wdeld) { WSLOT(wdelh, l, 1)[qw] = hs - h2; WSLOT(wdelh, l, 2)[qw] = h2; WSLOT(wdelh, l, 3)[qw] = h3 - hs; }
      hstor[(long)(l - 1) * g.plane + q] = h2;
    }
  }
#undef WSLOT
  PT_PRINT(5);
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
// One thread per region point (SPR x SPR = 1024): each sub-step is then one pass of the
// block with no per-thread loop over rows, the shortest chain of the m2 dependent sub-steps.
// (8 x 8 owned blocks on small tiles, a 24 x 24 region, measured no faster: the chain's
// latency is the sub-steps' barriers, not the region size.)
// Inputs (deld/delh slots, msfx, msfd, psdota, mapf, psa) are addressed through frame w, which
// for a tile of a decomposition is a wide frame whose ghost ring holds its neighbours' values
// to depth SPH (one width-SPH exchange per step instead of three per sub-step); the masks use
// global indices so ghost points evolve exactly as on their owning tile.  Outputs use frame g.
template <int SB>
__global__ __launch_bounds__((SB + 2 * SPH) * (SB + 2 * SPH)) void k_spstep_fused(
    Geom g, Geom w, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh,
    const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota,
    const double* __restrict__ mapf, const double* __restrict__ psa, double* ddsum, double* dhsum) {
  constexpr int SPB = SB, SPR = SB + 2 * SPH, SPP = SPR + 1;   // owned side, region side, LDS pitch
  __shared__ double Ds[2][SPR][SPP], Hs[2][SPR][SPP], U[SPR][SPP], V[SPR][SPP];
  const int l = blockIdx.z + 1;
  // owned blocks tile the tile's cross points plus its ghost ring (k_split_correct reads
  // ddsum/dhsum there; no dhsum exchange).  The ring's regions reach SPH + 1 points beyond the
  // tile, the depth of the wide exchange.
  const int J1 = g.jcx1() + blockIdx.x * SPB, I1 = g.icx1() + blockIdx.y * SPB;
  const int jr0 = J1 - SPH, ir0 = I1 - SPH;          // region origin (global)
  const int tx = threadIdx.x, ty = threadIdx.y;        // R x R, one region point each
  const double aam = c->aam[l - 1], dtau = c->dtau[l - 1], hbar = c->hbar[l - 1];
#ifdef RCM_SP_TIMING_M2      // timing-only builds (wrong results): the sub-step count capped
  const int m2 = min((int)aam * 2, RCM_SP_TIMING_M2);
#else
  const int m2 = (int)aam * 2;
#endif
  const double dtau2 = dtau * d_two, rdx2 = d_one / c->dx2;
#define WSLOT(a, l, s) ((a) + ((long)((s) - 1) * c->nsplit + ((l) - 1)) * w.plane)
  const double* D1 = WSLOT(deld, l, 1); const double* D2 = WSLOT(deld, l, 2); const double* D3 = WSLOT(deld, l, 3);
  const double* H1 = WSLOT(delh, l, 1); const double* H2 = WSLOT(delh, l, 2); const double* H3 = WSLOT(delh, l, 3);
#undef WSLOT
  const int gjx = g.gjx, giy = g.giy;
  // the thread's region point (tx, ty); d3/m2, h3/m2 (forward step) and d3/aam, h3/aam
  // (leapfrog) are loop-invariant and formed once
  constexpr int NR = 1;
  double d3f[NR], h3f[NR], d3l[NR], h3l[NR], ps[NR], mf[NR], ufac[NR], msd[NR], sd[NR], sh[NR];
  double rps[NR], rufac[NR];                            // 1/ps, 1/ufac for div_by
  bool ce[NR], ci[NR], bnd[NR], di[NR], own[NR];
  const double m2d = (double)m2;
  for (int r = 0; r < NR; r++) {
    const int lj = tx, li = ty + SPR * r, j = jr0 + lj, i = ir0 + li;
    // region points outside frame w (a partial last block) lie in the contaminated rim: they
    // are read as zero and never reach an output point
    const bool inw = in(j, w.j0, w.j0 + w.nj - 1) && in(i, w.i0, w.i0 + w.ni - 1);
    ce[r] = inw && g.gce(j, i);
    ci[r] = inw && g.gci(j, i);
    di[r] = inw && g.gdi(j, i);
    bnd[r] = ce[r] && !ci[r] &&
             (((g.gjeq(j, 1) || g.gjeq(j, gjx - 1)) && in(i, 2, giy - 2)) || i == 1 || i == giy - 1);
    own[r] = in(j, J1, J1 + SPB - 1) && in(i, I1, I1 + SPB - 1);
    const long q = ce[r] ? w.ix(j, i) : 0;
    Ds[0][li][lj] = ce[r] ? D1[q] : 0.0; Ds[1][li][lj] = ce[r] ? D2[q] : 0.0;
    Hs[0][li][lj] = ce[r] ? H1[q] : 0.0; Hs[1][li][lj] = ce[r] ? H2[q] : 0.0;
    U[li][lj] = 0.0; V[li][lj] = 0.0;
    const double d3 = ce[r] ? D3[q] : 0.0, h3 = ce[r] ? H3[q] : 0.0;
    d3f[r] = d3 / m2d; h3f[r] = h3 / m2d; d3l[r] = d3 / aam; h3l[r] = h3 / aam;
    ps[r] = ci[r] ? psa[w.ix(j, i)] : 1.0;
    mf[r] = ci[r] ? mapf[w.ix(j, i)] : 0.0;
    ufac[r] = di[r] ? c->dx2 * msfx[w.ix(j, i)] : 1.0;
    rufac[r] = d_one / ufac[r];
    rps[r] = d_one / ps[r];
    msd[r] = di[r] ? msfd[w.ix(j, i)] : 0.0;
    sd[r] = ce[r] ? Ds[0][li][lj] : 0.0;     // ddsum(ce) = deld(n0)
    sh[r] = ce[r] ? Hs[0][li][lj] : 0.0;
  }
  double pda[NR];
  for (int r = 0; r < NR; r++) {
    const int j = jr0 + tx, i = ir0 + ty + SPR * r;
    pda[r] = di[r] ? psdota[w.ix(j, i)] : 0.0;
  }
  __syncthreads();
  int n0 = 0, n1 = 1;                                   // slot indices (reference slots 1, 2)
  for (int n = 1; n <= m2; n++) {
    const int src = (n == 1) ? n0 : n1;
    // sub-step n must leave deld/delh valid within rho = m2 - n points of the owned block (the
    // owned points after the last): its update runs on that band only and its gradient on the
    // dot points the band reads; the rows outside are whole wavefronts (two region rows each)
    // that skip the sub-step's work
    const int rho = m2 - n, lo = SPH - rho, hi = SPH + SPB - 1 + rho;
    // gradient of delh(src) at dot points -> (uu, vv)
    for (int r = 0; r < NR; r++) {
      const int lj = tx, li = ty + SPR * r;
      if (di[r] && lj >= 1 && li >= 1 && in(li, lo, hi + 1) && in(lj, lo, hi + 1)) {
        const double a = Hs[src][li][lj], b = Hs[src][li - 1][lj], cc = Hs[src][li][lj - 1], dd = Hs[src][li - 1][lj - 1];
        double w1 = div_by(a + b - cc - dd, ufac[r], rufac[r]);
        double w2 = div_by(a + cc - b - dd, ufac[r], rufac[r]);
        w1 = w1 * pda[r];
        w2 = w2 * pda[r];
        U[li][lj] = w1 * msd[r];
        V[li][lj] = w2 * msd[r];
      }
    }
    __syncthreads();
    const int nn = (n == 1) ? n1 : n0;                  // forward writes n1; leapfrog n2 = n0
    for (int r = 0; r < NR; r++) {
      const int lj = tx, li = ty + SPR * r;
      if (!(in(li, lo, hi) && in(lj, lo, hi))) continue;
      if (ci[r] && lj + 1 < SPR && li + 1 < SPR) {
        const double w3 = rdx2 * mf[r] *
            (-U[li + 1][lj] + U[li + 1][lj + 1] - U[li][lj] + U[li][lj + 1] +
             V[li + 1][lj] + V[li + 1][lj + 1] - V[li][lj] - V[li][lj + 1]);
        if (n == 1) {
          const double dn = Ds[n0][li][lj] - dtau * w3 + d3f[r];
          const double hn = Hs[n0][li][lj] - div_by(dtau * hbar * Ds[n0][li][lj], ps[r], rps[r]) + h3f[r];
          Ds[nn][li][lj] = dn;
          Hs[nn][li][lj] = hn;
        } else {
          const double dn = Ds[n0][li][lj] - dtau2 * w3 + d3l[r];
          const double hn = Hs[n0][li][lj] - div_by(dtau2 * hbar * Ds[n1][li][lj], ps[r], rps[r]) + h3l[r];
          Ds[nn][li][lj] = dn;
          Hs[nn][li][lj] = hn;
        }
      } else if (bnd[r]) {
        if (n == 1) Hs[nn][li][lj] = Hs[n0][li][lj] * ((aam - d_one) / aam);
        else Hs[nn][li][lj] = d_two * Hs[n1][li][lj] - Hs[n0][li][lj];
      }
      if (ce[r] && own[r]) {          // only the owned points' sums are stored
        sd[r] = sd[r] + Ds[nn][li][lj];
        sh[r] = sh[r] + Hs[nn][li][lj];
      }
    }
    __syncthreads();
    if (n >= 2) { const int t0 = n0; n0 = n1; n1 = t0; }
    else { /* forward step: n0 = 1, n1 = 2 stay; the leapfrog loop starts with n2 = n0 */ }
  }
  for (int r = 0; r < NR; r++) {
    const int j = jr0 + tx, i = ir0 + ty + SPR * r;
    if (own[r] && in(j, g.jdx1(), g.jdx2()) && in(i, g.idx1(), g.idx2())) {
      const long q = (long)(l - 1) * g.plane + g.ix(j, i);
      ddsum[q] = ce[r] ? sd[r] : d_zero;
      dhsum[q] = ce[r] ? sh[r] : d_zero;
    }
  }
}
template __global__ __launch_bounds__(32 * 32) void k_spstep_fused<16>(Geom, Geom, const Consts* __restrict__,
    const double* __restrict__, const double* __restrict__, const double* __restrict__, const double* __restrict__,
    const double* __restrict__, const double* __restrict__, const double* __restrict__, double*, double*);
template __global__ __launch_bounds__(24 * 24) void k_spstep_fused<8>(Geom, Geom, const Consts* __restrict__,
    const double* __restrict__, const double* __restrict__, const double* __restrict__, const double* __restrict__,
    const double* __restrict__, const double* __restrict__, const double* __restrict__, double*, double*);

__device__ __forceinline__ void bdyval_point(const Geom& g, double xt, bool integ, const BdyArgs& a, int line, int x,
                                             int k, bool interior);
__device__ __forceinline__ int bdy_chunks_d(const Geom& g) { return (max(g.jde2 - g.jde1, g.ide2 - g.ide1) + 65) / 64; }

// splitf corrections, Main/mod_split.F90:417-457 (ps and t on ci, u and v on di).
// BDY (k_split_correct_bdy, rcmdyn_step): the step's bdyval (Main/mod_bdycod.F90:1109-1529 +
// bdyuv :896-1061, hydrostatic, after a tend: the integration branch) runs in the same launch.
// The corrections never touch a boundary-line point (ci and di exclude them), and with BDY the
// correcting threads store only the lanes they corrected, so extra blocks past the correction
// grid run bdyval's line loop (bdyval_point) concurrently: each bdyval write reads only its own
// point and the boundary data, except the slices' interior entries (u, v of the first interior
// row/column), which the thread correcting that interior point writes from its registers.
// The clock is advanced by k_bdyval_qc (advance = 2 here: noise sums only), so the bdyval time
// level is formed from the clock before the step's advance.
template <bool BDY, int NS>
__device__ __forceinline__ void split_correct_body(
    const Geom& g, const Consts* __restrict__ c, const double* __restrict__ ddsum, const double* __restrict__ dhsum,
    const double* __restrict__ psdota, const double* __restrict__ msfd, double* psa, double* psb, double* a1t,
    double* a2t, double* a1u, double* a1v, double* a2u, double* a2v, StepState* s, int advance,
    const double* __restrict__ red, int red_total, FlagSnap* ring, const BdyArgs& ba, const QFix& qf, int nser) {
  // qfuse: the serial sweeps of the planes k_split_project flagged, in trailing z slices (one
  // wavefront per plane)
  if (nser && (int)blockIdx.z >= (int)gridDim.z - nser) {
    const int plane = (((int)blockIdx.z - ((int)gridDim.z - nser)) * (int)gridDim.y + (int)blockIdx.y) *
                          (int)gridDim.x + (int)blockIdx.x;
    extern __shared__ double nlds[];            // negfix_sweep_lds(g) doubles when nser > 0 (the launch)
    if (threadIdx.y == 0 && plane < 2 * c->kz) negfix_serial_plane(g, c, qf, plane, nlds);
    return;
  }
  // bdyval blocks first: the leading z slices (blockIdx.z < zbdy) are dispatched before any
  // correction block, so their latency chain overlaps the corrections instead of trailing
  // them; 4 (line, chunk, level) items of 64 points per block
  const int kz = c->kz;
  const int zbdy = BDY ? (int)gridDim.z - nser - kz : 0;
  PT_DECL
  if (BDY && (int)blockIdx.z < zbdy) {
    const int nchunk = bdy_chunks_d(g);
    const int item = (((int)blockIdx.z * (int)gridDim.y + (int)blockIdx.y) * (int)gridDim.x + (int)blockIdx.x) * 4 +
                     (int)threadIdx.y;
    if (item >= 6 * nchunk * kz) return;
    const int line = item % 6, chunk = (item / 6) % nchunk, k = item / (6 * nchunk) + 1;
    const double xt = s->xbctime + ((s->lcount + 1 == 2) ? d_two * c->dtsec : s->dt);
    bdyval_point(g, xt, true, ba, line, chunk * 64 + (int)threadIdx.x, k, false);
    PT_PRINT(6);
    return;
  }
#if SCOR_FLAT
  // the (pair, row) points of a level flattened: every lane of a block has a point (no idle
  // second block column on a 192-wide tile), rows follow one another in the lanes
  const int npr = (g.jdx2() - g.jde1 + 2) / 2;
#if SCOR_XCD
  // the kz levels of one pair block run consecutively on one XCD: the 2-D sums, psdota and
  // msfd each level reads are fetched into that XCD's L2 once
  const int tq = xcd_range(((int)blockIdx.z * (int)gridDim.y + (int)blockIdx.y) * (int)gridDim.x + (int)blockIdx.x,
                           zbdy * (int)gridDim.x, kz * (int)gridDim.x);
  const int bxq = tq / kz, k = tq % kz + 1;
  const bool first = tq == 0;
#else
  const int bxq = (int)blockIdx.x, k = (int)blockIdx.z - zbdy + 1;
  const bool first = blockIdx.x == 0 && (int)blockIdx.z == zbdy;
#endif
  const int q = bxq * 256 + (int)threadIdx.y * 64 + (int)threadIdx.x;
  const int j = g.jde1 + q % npr;
  const int i = g.ide1 + q / npr;
#else
  const int j = g.jde1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ide1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int k = (int)blockIdx.z - zbdy + 1;
  const bool first = blockIdx.x == 0 && blockIdx.y == 0 && (int)blockIdx.z == zbdy;
#endif
  // last tile's launch, block 0: the Bleck noise sums of every tile (fixed-order tree over the
  // k_columns partials, Main/mod_tendency.F90:1449-1459), then rcmtimer%advance + dt switch
  // (:608-616); nothing else here reads the clock.  The same lane then copies the step's error
  // flags into the host-mapped ring (k_flag_snapshot's work; this is the step's last flag writer)
  if (advance && first) {
    __shared__ double sa[256], sb[256];
    const int t = threadIdx.y * blockDim.x + threadIdx.x;
    double a = 0.0, b = 0.0;
    for (int q = t; q < red_total; q += 256) { a += red[2 * q]; b += red[2 * q + 1]; }
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
    if (t == 0 && advance == 1) {
      s->lcount = s->lcount + 1;
      if (s->lcount == 2) s->dt = d_two * c->dtsec;
      const long long lc = s->lcount;
      FlagSnap& r = ring[(lc - 1 + NFLAGSLOT) % NFLAGSLOT];
      r.nanflag = s->nanflag;
      r.slflag = s->slflag;
      r.lcount = lc;
    }
  }
  // two adjacent points (jp, jp+1) per thread, 16-byte accesses (jp - j0 is even); owned points
  // and the right/top ghost ring (the bdyuv slices read the new u, v there)
  const int jp = g.jde1 + 2 * (j - g.jde1);
  if (jp > g.jdx2() || i > g.idx2()) return;
  const uint32_t o2 = g.o2(jp, i), o3 = o2 + (uint32_t)(k - 1) * g.L8;
  const double gnu1 = c->gnu1;
  constexpr int ns = NS;       // c->nsplit (the launch picks the instance)
  const int jd2 = g.br ? g.jdi2 : g.jde2 + 1, id2 = g.bt ? g.idi2 : g.ide2 + 1;
  const bool ici = in(i, g.ice1, g.icx2()), idi = in(i, g.idi1, id2);
  const bool ci0 = ici && in(jp, g.jce1, g.jcx2()) && g.gci(jp, i);
  const bool ci1 = ici && in(jp + 1, g.jce1, g.jcx2()) && g.gci(jp + 1, i);
  const bool di0 = idi && in(jp, g.jdi1, jd2), di1 = idi && in(jp + 1, g.jdi1, jd2);
  // every operand is loaded before the first store (the state buffers are not __restrict__:
  // a store would order the later loads behind it)
  const bool cx = ci0 || ci1, dx = di0 || di1;
  double dd[2][NS];
  double2 pa{}, pb{}, t1{}, t2{}, u1{}, v1{}, u2{}, v2{}, pd{}, md{};
  double2 h0[NS], hs[NS];
  double hw[NS], hsw[NS];
  if (cx) {
#pragma unroll
    for (int l = 1; l <= NS; l++) {
      const double2 d = LD2(ddsum, o2 + (uint32_t)(l - 1) * g.L8);
      dd[0][l - 1] = d.x; dd[1][l - 1] = d.y;
    }
    if (k == 1) { pa = LD2(psa, o2); pb = LD2(psb, o2); }
    t1 = LD2(a1t, o3); t2 = LD2(a2t, o3);
  }
  if (dx) {
    u1 = LD2(a1u, o3); v1 = LD2(a1v, o3); u2 = LD2(a2u, o3); v2 = LD2(a2v, o3);
    pd = LD2(psdota, o2); md = LD2(msfd, o2);
#pragma unroll
    for (int l = 1; l <= NS; l++) {
      const uint32_t lo = o2 + (uint32_t)(l - 1) * g.L8;
      // dhsum at (jp-1..jp+1, i-1..i)
      h0[l - 1] = LD2(dhsum, lo); hs[l - 1] = LD2(dhsum, lo - g.P8);
      hw[l - 1] = LD(dhsum, lo - 8u); hsw[l - 1] = LD(dhsum, lo - g.P8 - 8u);
    }
  }
  if (cx) {
    if (k == 1) {
      for (int l = 1; l <= ns; l++) {
        const double an = c->an[l - 1];
        if (ci0) { pa.x = pa.x - an * dd[0][l - 1]; pb.x = pb.x - gnu1 * an * dd[0][l - 1]; }
        if (ci1) { pa.y = pa.y - an * dd[1][l - 1]; pb.y = pb.y - gnu1 * an * dd[1][l - 1]; }
      }
      if (!BDY || (ci0 && ci1)) { ST2(psa, o2, pa); ST2(psb, o2, pb); }
      else if (ci0) { ST(psa, o2, pa.x); ST(psb, o2, pb.x); }
      else { ST(psa, o2 + 8u, pa.y); ST(psb, o2 + 8u, pb.y); }
    }
    for (int l = 1; l <= ns; l++) {
      const double am = c->am[l - 1][k - 1];
      if (ci0) { t1.x = t1.x + am * dd[0][l - 1]; t2.x = t2.x + gnu1 * am * dd[0][l - 1]; }
      if (ci1) { t1.y = t1.y + am * dd[1][l - 1]; t2.y = t2.y + gnu1 * am * dd[1][l - 1]; }
    }
    if (!BDY || (ci0 && ci1)) { ST2(a1t, o3, t1); ST2(a2t, o3, t2); }
    else if (ci0) { ST(a1t, o3, t1.x); ST(a2t, o3, t2.x); }
    else { ST(a1t, o3 + 8u, t1.y); ST(a2t, o3 + 8u, t2.y); }
  }
  if (dx) {
    const double fac0 = pd.x / (c->dx2 * md.x), fac1 = pd.y / (c->dx2 * md.y);
#pragma unroll
    for (int l = 1; l <= NS; l++) {
      const double zm = c->zmatx[l - 1][k - 1], gnuzm = gnu1 * zm;
      if (di0) {
        const double x = fac0 * (h0[l - 1].x + hs[l - 1].x - hw[l - 1] - hsw[l - 1]);
        const double y = fac0 * (h0[l - 1].x - hs[l - 1].x + hw[l - 1] - hsw[l - 1]);
        u1.x = u1.x - zm * x; v1.x = v1.x - zm * y; u2.x = u2.x - gnuzm * x; v2.x = v2.x - gnuzm * y;
      }
      if (di1) {
        const double x = fac1 * (h0[l - 1].y + hs[l - 1].y - h0[l - 1].x - hs[l - 1].x);
        const double y = fac1 * (h0[l - 1].y - hs[l - 1].y + h0[l - 1].x - hs[l - 1].x);
        u1.y = u1.y - zm * x; v1.y = v1.y - zm * y; u2.y = u2.y - gnuzm * x; v2.y = v2.y - gnuzm * y;
      }
    }
    if (!BDY || (di0 && di1)) { ST2(a1u, o3, u1); ST2(a1v, o3, v1); ST2(a2u, o3, u2); ST2(a2v, o3, v2); }
    else if (di0) { ST(a1u, o3, u1.x); ST(a1v, o3, v1.x); ST(a2u, o3, u2.x); ST(a2v, o3, v2.x); }
    else { ST(a1u, o3 + 8u, u1.y); ST(a1v, o3 + 8u, v1.y); ST(a2u, o3 + 8u, u2.y); ST(a2v, o3 + 8u, v2.y); }
  }
  PT_PRINT(7);
  if (!BDY) return;
  const Slices& sl = ba.sl;
  const long slen = ba.slen;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int jj = jp + r;
    // the slices' interior entries: this point's corrected u, v
    if (r ? di1 : di0) {
      const double uu = r ? u1.y : u1.x, vv = r ? v1.y : v1.x;
      if (g.bl && jj == g.jdi1) { SLI(sl.s[1], i, k) = uu; SLI(sl.s[5], i, k) = vv; }
      if (g.br && jj == g.jdi2) { SLI(sl.s[3], i, k) = uu; SLI(sl.s[7], i, k) = vv; }
      if (g.bb && i == g.idi1) { SLJ(sl.s[9], jj, k) = uu; SLJ(sl.s[13], jj, k) = vv; }
      if (g.bt && i == g.idi2) { SLJ(sl.s[11], jj, k) = uu; SLJ(sl.s[15], jj, k) = vv; }
    }
  }
}
#undef SLOT

#ifndef SCOR_LB
#define SCOR_LB 4
#endif
template <int NS>
__global__ __launch_bounds__(256, SCOR_LB) void k_split_correct(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum,
                                const double* __restrict__ dhsum, const double* __restrict__ psdota,
                                const double* __restrict__ msfd, double* psa, double* psb, double* a1t,
                                double* a2t, double* a1u, double* a1v, double* a2u, double* a2v, StepState* s,
                                int advance, const double* __restrict__ red, int red_total, FlagSnap* ring, QFix qf,
                                int nser) {
  split_correct_body<false, NS>(g, c, ddsum, dhsum, psdota, msfd, psa, psb, a1t, a2t, a1u, a1v, a2u, a2v, s, advance,
                            red, red_total, ring, BdyArgs{}, qf, nser);
}

// ---------------------------------------------------------------------------------------
// bdyval, Main/mod_bdycod.F90:1109-1529 (+ bdyuv :896-1061).  Slice order:
// 0 wue 1 wui 2 eue 3 eui 4 wve 5 wvi 6 eve 7 evi (by i) / 8 sue 9 sui 10 nue 11 nui
// 12 sve 13 svi 14 nve 15 nvi (by j).


// One boundary point (j, i) at level k: ghost = a point of the right/top ghost ring (only its
// slice entries are written).  interior: also write the slices' interior entries (u, v of the
// first interior row/column) from memory; the split-correct fusion writes them from the
// thread that corrects that point instead (k_split_correct_bdy).
__device__ __forceinline__ void bdyval_body(const Geom& g, double xt, bool integ, const BdyArgs& a, int j, int i,
                                            int k, bool ghost, bool interior);

__device__ __forceinline__ void bdyval_point(const Geom& g, double xt, bool integ, const BdyArgs& a, int line, int x,
                                             int k, bool interior) {
  // set_ps = 0 for the non-hydrostatic core, whose p* is the constant reference p*
  // (Main/mod_bdycod.F90:1150-1165, 1430-1451 are hydrostatic-only).
  // thread -> one point of the boundary lines: blockIdx.y 0..2 = rows i = ide1 (bottom),
  // ide2 (top), ice2 (top cross row) over jde; 3..5 = columns j = jde1, jde2, jce2 over ide
  // minus the points a row owns.  Every point the body modifies lies on these lines.
  // One point past the tile along each line (toward a neighbour) only writes the bdyuv slice
  // entry there, from the ghost-ring u, v and the boundary data: k_bdyval_qc reads it (the
  // reference exchanges the slices instead, exchange_bdy_lr/bt).
  int j, i;
  bool ghost = false;
  if (line < 3) {
    if (line == 0 ? !g.bb : !g.bt) return;
    i = (line == 0) ? g.ide1 : (line == 1) ? g.ide2 : g.ice2;
    j = g.jde1 + x;
    if (j > g.jdx2() || (j > g.jde2 && line == 2)) return;
    ghost = j > g.jde2;
  } else {
    if (line == 3 ? !g.bl : !g.br) return;
    j = (line == 3) ? g.jde1 : (line == 4) ? g.jde2 : g.jce2;
    i = g.ide1 + x;
    if (i > g.idx2() || (i > g.ide2 && line == 5)) return;
    ghost = i > g.ide2;
    if ((g.bb && i == g.ide1) || (g.bt && (i == g.ide2 || i == g.ice2))) return;
  }
  bdyval_body(g, xt, integ, a, j, i, k, ghost, interior);
}

__device__ __forceinline__ void bdyval_body(const Geom& g, double xt, bool integ, const BdyArgs& a, int j, int i,
                                            int k, bool ghost, bool interior) {
  double *a1u = a.a1u, *a1v = a.a1v, *a1t = a.a1t, *a1qv = a.a1qv, *a1qc = a.a1qc;
  double *a2u = a.a2u, *a2v = a.a2v, *a2t = a.a2t, *a2qv = a.a2qv, *a2qc = a.a2qc, *psa = a.psa, *psb = a.psb;
  const double *ub0 = a.ub0, *ubt = a.ubt, *vb0 = a.vb0, *vbt = a.vbt, *tb0 = a.tb0, *tbt = a.tbt;
  const double *qb0 = a.qb0, *qbt = a.qbt, *pb0 = a.pb0, *pbt = a.pbt;
  const Slices& sl = a.sl;
  const long slen = a.slen;
  const int set_ps = a.set_ps;
  const long q = g.ix(j, i);
  const long p = (long)(k - 1) * g.plane + q;
  // dot-point boundary rows: left/right on idi, bottom/top on the whole jde range
  const bool dL = g.bl && j == g.jde1 && in(i, g.idi1, g.idi2);
  const bool dR = g.br && j == g.jde2 && in(i, g.idi1, g.idi2);
  const bool dB = g.bb && i == g.ide1;
  const bool dT = g.bt && i == g.ide2;
  const bool dset = !ghost && (dL || dR || dB || dT);
  // cross-point boundary rows: left/right on ici, bottom/top on the jce range
  const bool cL = g.bl && j == g.jce1 && in(i, g.ici1, g.ici2);
  const bool cR = g.br && j == g.jce2 && in(i, g.ici1, g.ici2);
  const bool cB = g.bb && i == g.ice1 && in(j, g.jce1, g.jce2);
  const bool cT = g.bt && i == g.ice2 && in(j, g.jce1, g.jce2);
  const bool cset = !ghost && (cL || cR || cB || cT);
  const bool ps1 = cset && set_ps && k == 1;
  // bdyuv slices (the interior slice values are interior points, which nothing here modifies)
  const bool sW = g.bl && j == g.jde1 && (in(i, g.idi1, g.idi2) || ghost);
  const bool sE = g.br && j == g.jde2 && (in(i, g.idi1, g.idi2) || ghost);
  const bool sS = g.bb && i == g.ide1, sSi = sS && (in(j, g.jdi1, g.jdi2) || ghost);
  const bool sN = g.bt && i == g.ide2, sNi = sN && (in(j, g.jdi1, g.jdi2) || ghost);
  // ---- every operand first (no load waits behind a store of the same thread), then the stores
  double ubv = 0.0, vbv = 0.0, u1o = 0.0, v1o = 0.0, t1o = 0.0, qv1o = 0.0, qc1o = 0.0, pso = 0.0;
  double tbv = 0.0, qbv = 0.0, pbv = 0.0, su = 0.0, sv = 0.0;
  if (dset || sW || sE || sS || sN) { ubv = ub0[p] + xt * ubt[p]; vbv = vb0[p] + xt * vbt[p]; }
  if (dset && integ) { u1o = a1u[p]; v1o = a1v[p]; }
  if (cset) {
    if (integ) { t1o = a1t[p]; qv1o = a1qv[p]; qc1o = a1qc[p]; }
    if (ps1) { if (integ) pso = psa[q]; pbv = pb0[q] + xt * pbt[q]; }
    tbv = tb0[p] + xt * tbt[p];
    qbv = qb0[p] + xt * qbt[p];
  }
  if (!interior) { }
  else if (sW) { su = F3(a1u, g.jdi1, i, k); sv = F3(a1v, g.jdi1, i, k); }
  else if (sE) { su = F3(a1u, g.jdi2, i, k); sv = F3(a1v, g.jdi2, i, k); }
  else if (sSi) { su = F3(a1u, j, g.idi1, k); sv = F3(a1v, j, g.idi1, k); }
  else if (sNi) { su = F3(a1u, j, g.idi2, k); sv = F3(a1v, j, g.idi2, k); }
  // bdyuv corner fills, Main/mod_bdycod.F90:1030-1061: every corner slice entry is the
  // boundary value b0 + xt*bt of a known point, written by the thread of that tile corner
  const bool kTL = !ghost && g.bt && g.bl && j == g.jde1 && i == g.ide2;
  const bool kBL = !ghost && g.bb && g.bl && j == g.jde1 && i == g.ide1;
  const bool kTR = !ghost && g.bt && g.br && j == g.jde2 && i == g.ide2;
  const bool kBR = !ghost && g.bb && g.br && j == g.jde2 && i == g.ide1;
  double cu1 = 0.0, cv1 = 0.0, cu2 = 0.0, cv2 = 0.0;
#define UB(J, I) (F3(ub0, J, I, k) + xt * F3(ubt, J, I, k))
#define VB(J, I) (F3(vb0, J, I, k) + xt * F3(vbt, J, I, k))
  if (kTL) { cu1 = UB(g.jdi1, g.ide2); cv1 = VB(g.jdi1, g.ide2); cu2 = UB(g.jde1, g.idi2); cv2 = VB(g.jde1, g.idi2); }
  if (kBL) { cu1 = UB(g.jdi1, g.ide1); cv1 = VB(g.jdi1, g.ide1); cu2 = UB(g.jde1, g.idi1); cv2 = VB(g.jde1, g.idi1); }
  if (kTR) { cu1 = UB(g.jdi2, g.ide2); cv1 = VB(g.jdi2, g.ide2); cu2 = UB(g.jde2, g.idi2); cv2 = VB(g.jde2, g.idi2); }
  if (kBR) { cu1 = UB(g.jdi2, g.ide1); cv1 = VB(g.jdi2, g.ide1); cu2 = UB(g.jde2, g.idi1); cv2 = VB(g.jde2, g.idi1); }
#undef UB
#undef VB
  if (dset) {
    if (integ) { a2u[p] = u1o; a2v[p] = v1o; }
    a1u[p] = ubv;
    a1v[p] = vbv;
  }
  if (cset) {
    if (integ) {
      a2t[p] = t1o; a2qv[p] = qv1o; a2qc[p] = qc1o;
      if (ps1) psb[q] = pso;
    }
    if (ps1) psa[q] = pbv;
    a1t[p] = tbv;
    a1qv[p] = qbv;
  }
  if (sW) { if (interior) { SLI(sl.s[1], i, k) = su; SLI(sl.s[5], i, k) = sv; } SLI(sl.s[0], i, k) = ubv; SLI(sl.s[4], i, k) = vbv; }
  if (sE) { if (interior) { SLI(sl.s[3], i, k) = su; SLI(sl.s[7], i, k) = sv; } SLI(sl.s[2], i, k) = ubv; SLI(sl.s[6], i, k) = vbv; }
  if (sS) {
    if (sSi && interior) { SLJ(sl.s[9], j, k) = su; SLJ(sl.s[13], j, k) = sv; }
    SLJ(sl.s[8], j, k) = ubv; SLJ(sl.s[12], j, k) = vbv;
  }
  if (sN) {
    if (sNi && interior) { SLJ(sl.s[11], j, k) = su; SLJ(sl.s[15], j, k) = sv; }
    SLJ(sl.s[10], j, k) = ubv; SLJ(sl.s[14], j, k) = vbv;
  }
  if (kTL) { SLI(sl.s[1], g.ide2, k) = cu1; SLI(sl.s[5], g.ide2, k) = cv1; SLJ(sl.s[11], g.jde1, k) = cu2; SLJ(sl.s[15], g.jde1, k) = cv2; }
  if (kBL) { SLI(sl.s[1], g.ide1, k) = cu1; SLI(sl.s[5], g.ide1, k) = cv1; SLJ(sl.s[9], g.jde1, k) = cu2; SLJ(sl.s[13], g.jde1, k) = cv2; }
  if (kTR) { SLI(sl.s[3], g.ide2, k) = cu1; SLI(sl.s[7], g.ide2, k) = cv1; SLJ(sl.s[11], g.jde2, k) = cu2; SLJ(sl.s[15], g.jde2, k) = cv2; }
  if (kBR) { SLI(sl.s[3], g.ide1, k) = cu1; SLI(sl.s[7], g.ide1, k) = cv1; SLJ(sl.s[9], g.jde2, k) = cu2; SLJ(sl.s[13], g.jde2, k) = cv2; }
}


template <int NS>
__global__ __launch_bounds__(256, SCOR_LB) void k_split_correct_bdy(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum,
                                    const double* __restrict__ dhsum, const double* __restrict__ psdota,
                                    const double* __restrict__ msfd, StepState* s, int advance,
                                    const double* __restrict__ red, int red_total, BdyArgs a, QFix qf, int nser) {
  split_correct_body<true, NS>(g, c, ddsum, dhsum, psdota, msfd, a.psa, a.psb, a.a1t, a.a2t, a.a1u, a.a1v, a.a2u, a.a2v,
                           s, advance ? 2 : 0, red, red_total, nullptr, a, qf, nser);
}

// one instance per nsplit (1..MAXSPLIT): the mode loops unroll and only the split slots in
// use hold registers (114 -> fewer VGPRs at nsplit = 2)
#define RCM_SPLIT_INST(NS_)                                                                                   \
  template __global__ __launch_bounds__(256, SCOR_LB) void k_split_correct<NS_>(Geom, const Consts* __restrict__, const double* __restrict__, \
                                                const double* __restrict__, const double* __restrict__,       \
                                                const double* __restrict__, double*, double*, double*, double*, \
                                                double*, double*, double*, double*, StepState*, int,          \
                                                const double* __restrict__, int, FlagSnap*, QFix, int);      \
  template __global__ __launch_bounds__(256, SCOR_LB) void k_split_correct_bdy<NS_>(Geom, const Consts* __restrict__, const double* __restrict__, \
                                                    const double* __restrict__, const double* __restrict__,      \
                                                    const double* __restrict__, StepState*, int,                 \
                                                    const double* __restrict__, int, BdyArgs, QFix, int);
RCM_SPLIT_INST(1)
RCM_SPLIT_INST(2)
RCM_SPLIT_INST(3)
RCM_SPLIT_INST(4)
#undef RCM_SPLIT_INST

__global__ void k_bdyval_set(Geom g, const StepState* __restrict__ s, BdyArgs a) {
  const int x = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  bdyval_point(g, s->xbctime + s->dt, s->lcount > 0, a, (int)blockIdx.y, x, (int)blockIdx.z + 1, true);
}



__global__ void k_bdyval_qc(Geom g, int do_qc, int do_qv, double* a1qc, double* a1qv, const double* __restrict__ psa,
                            Slices sl, long slen, StepState* s, double dtsec, int advance, FlagSnap* ring) {
  const int k = (int)blockIdx.x + 1;
  if (advance && k == 1 && threadIdx.x == 0) {
    // every clock word is loaded before the first store (one memory latency, not one per word)
    const double xb = s->xbctime;
    const long long lc = s->lcount + 1;
    const int nanf = s->nanflag, slf = s->slflag;
    s->xbctime = xb + dtsec;
    if (advance == 2) {
      // the step clock of a fused step (k_split_correct_bdy): rcmtimer%advance + dt switch
      // (Main/mod_tendency.F90:608-616) and the step's flag snapshot
      s->lcount = lc;
      if (lc == 2) s->dt = d_two * dtsec;
      FlagSnap& r = ring[(lc - 1 + NFLAGSLOT) % NFLAGSLOT];
      r.nanflag = nanf;
      r.slflag = slf;
      r.lcount = lc;
    }
  }
  bdyval_qc_level(g, do_qc, do_qv, a1qc, a1qv, [&](int j, int i) { return F2(psa, j, i); }, sl, slen, k);
}

// the step's error flags into the host-mapped ring (one lane), after the clock advanced
__global__ void k_flag_snapshot(const StepState* __restrict__ s, FlagSnap* ring) {
  if (threadIdx.x != 0) return;
  const long long lc = s->lcount;
  FlagSnap& r = ring[(lc - 1 + NFLAGSLOT) % NFLAGSLOT];
  r.nanflag = s->nanflag;
  r.slflag = s->slflag;
  r.lcount = lc;
}

// the sticky error flags as one word for the RCCL max-reduction of a multi-rank job, and the
// reduced word into the host-mapped slot the host checks
__global__ void k_err_gather(const StepState* __restrict__ s, int32_t* derr) {
  if (threadIdx.x == 0) derr[0] = s->nanflag | (s->slflag << 1);
}
__global__ void k_err_publish(const int32_t* __restrict__ derr, int32_t* hslot) {
  if (threadIdx.x == 0) hslot[0] = derr[0];
}

// ---------------------------------------------------------------------------------------
// static derived fields: Main/mod_params.F90:1993-2001 (xmsf, dmsf), Main/mod_diffusion.F90:
// 124-140 (hgfact), Main/mod_split.F90:99-101 (map)
__global__ void k_prepare_static(Geom g, const Consts* __restrict__ c, int diffu_hgtf,
                                 const double* __restrict__ msfx, const double* __restrict__ msfd,
                                 const double* __restrict__ ht, double* xmsf, double* dmsf, double* hgfact,
                                 double* mapf) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  // dmsf/xmsf on the global dot interior of the tile and its 2-deep ghost ring (the map
  // factors' exchange depth): the ghost-ring kernels read them there
  if (g.gdi(j, i) && in(j, g.jde1 - 2, g.jde2 + 2) && in(i, g.ide1 - 2, g.ide2 + 2)) {
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

// Copy the owned points (jde x ide) of nplanes 2-D planes from frame g into frame w (the wide
// frame of the fused split step); plane strides sstride / dstride.
__global__ void k_copy_frame(Geom g, Geom w, int nplanes, const double* __restrict__ src, long sstride, double* dst,
                             long dstride) {
  THREAD_POINT(g.jde1, g.ide1);
  if (j > g.jde2 || i > g.ide2) return;
  for (int p = 0; p < nplanes; p++) dst[p * dstride + w.ix(j, i)] = src[p * sstride + g.ix(j, i)];
}

#ifdef RCM_PHASE_TIMING
// phase records of the launches since the last dump (see PT_DECL in devcommon.hpp)
extern "C" int rcm_phase_dump(const char* path) {
  int n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(rcm_pt_count), sizeof(int)) != hipSuccess) return -1;
  n = n < PT_CAP ? n : PT_CAP;
  std::vector<PtRec> v(n);
  if (n && hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(rcm_pt_buf), sizeof(PtRec) * n) != hipSuccess) return -1;
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return -1;
  std::fwrite(v.data(), sizeof(PtRec), n, fp);
  std::fclose(fp);
  const int zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(rcm_pt_count), &zero, sizeof(int)) != hipSuccess) return -1;
  return n;
}
#endif

}  // namespace rcm
