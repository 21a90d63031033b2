// species.hip -- the hydrometeors beyond qc (nqx = 5: qi, qr, qs; physicsparam ipptls >= 2,
// Main/mod_params.F90:1358-1366), gfx950.
//
// The reference runs every hydrometeor n = iqfrst..iqlst through qc's chain of the dyn step:
// hadvqx (Main/mod_advection.F90:607-662, Main/mod_tendency.F90:1382), vadv4d ind 1 or 3
// (:847-966, :1388), diffu_x4d (Main/mod_diffusion.F90:792-947, :1526), the sums with qxphy
// (:332-335), the forecast, the exchange of atmc%qx and the negative-moisture fix (:375-393),
// filter_raw_4d with the zero floor (:426-427), and bdyval's boundary copies (Main/mod_bdycod.F90:
// 1143-1284) and inflow/outflow lines (:2153-2220).  The species never feed back into the other
// prognostics except through the total water load (k_columns' tvfac, the NH water loading),
// so they run in kernels of their own after the qv/qc update, with qc's operation order:
//
//  k_qx_tend   one level per block of 64 x 8 cross points, the cell's mass fluxes and every
//              species' decoupled atm1 (halo 1) and mkslice atm2 (halo 2) staged in LDS; the
//              forecast atmc%qx into cq (atm2 on the ring jce \ jci);
//  k_qx_fix    the negative-value fix and the RAW filter into the next buffers (points with a
//              serially dependent negative predecessor flag their plane), and the copies of the
//              points the update does not write (qfuse's keep copies of qv, qc);
//  k_qx_serial one wavefront per flagged (species, level) plane: the sweep in the reference's
//              i-major, j-minor order;
//  k_bdyval_qx bdyval's atm2 = atm1 boundary copies, then the inflow/outflow lines.
//
// The non-hydrostatic core (k_nh_qx_tend) adds the atmx%qx * cr term of adiabatic
// (Main/mod_tendency.F90:1615-1617) and updates the state in place: k_qx_fix / k_qx_serial then
// filter into the same buffers (each thread reads and writes only its own point's levels).
//
// Transcendental-free: every result is bit-identical to the oracle's restatement
// (-ffp-contract=off).
#include "engine.hpp"
#include "kernels.hpp"
#include "kernels_nh.hpp"
#include "devcommon.hpp"
#include "qxcommon.hpp"

namespace rcm {

namespace {
// QBJ x QBI (kernels.hpp): the launch's grid and block come from the same constants
constexpr int QDW = QBJ + 1, QDH = QBI + 1;    // dot points j..j+QBJ, i..i+QBI
constexpr int QW1 = QBJ + 2, QH1 = QBI + 2;    // halo 1
constexpr int QW2 = QBJ + 4, QH2 = QBI + 4;    // halo 2
}  // namespace

// diffu_x4d of one point (Main/mod_diffusion.F90:673-713 idiffu = 1, 726-735 / 881-891
// idiffu = 2; idiffu = 3 adds k_diffu6's column term), f(dj, di) the mkslice field qxb3d
template <class FB>
__device__ __forceinline__ double qx_diffu(const Geom& g, const Consts* __restrict__ c, int j, int i, double ften,
                                           double xkcs, FB f, const double* d6, uint32_t o3) {
  if (c->idiffu == 3) {
    if (j == g.jci2 || (!g.bl && j == g.jce1 - 1)) ften = ften + LD(d6, o3);
    return ften;
  }
  if (c->idiffu == 2)
    return ften + d_one * xkcs *
                      (o4_c1 * (f(1, 0) + f(-1, 0) + f(0, 1) + f(0, -1)) +
                       o4_c2 * (f(1, 1) + f(-1, -1) + f(-1, 1) + f(1, -1)) + o4_c3 * f(0, 0));
  if (g.gcii(j, i))
    ften = ften - d_one * xkcs *
                      (z4_c1 * (f(2, 0) + f(-2, 0) + f(0, 2) + f(0, -2)) +
                       z4_c2 * (f(1, 0) + f(-1, 0) + f(0, 1) + f(0, -1)) + z4_c3 * f(0, 0));
  auto lap = [&](double x) {
    return x + d_one * xkcs * (z4_c1 * (f(1, 0) + f(-1, 0) + f(0, 1) + f(0, -1)) + z4_c2 * f(0, 0));
  };
  if (g.gjeq(j, 2)) ften = lap(ften);
  if (g.gjeq(j, g.gjx - 2)) ften = lap(ften);
  if (g.gieq(i, 2)) ften = lap(ften);
  if (g.gieq(i, g.giy - 2)) ften = lap(ften);
  return ften;
}

// K_QX1.  The tendencies and forecast of the hydrometeors beyond qc at the cross points of the
// tile and its ghost ring (jcx x icx, as k_scalars: the ring is what the exchange of atmc%qx
// would deliver), one level per block.  Reads the scaled diffusion coefficient k_scalars
// stored (xkc * rdxsq * p*b at the interior points) and qdot of k_columns.
__global__ __launch_bounds__(QBT) void k_qx_tend(Geom g, const Consts* __restrict__ c,
                                                 const StepState* __restrict__ s, Fields f, QxArgs q) {
  __shared__ double sUMC[QDH][QDW], sVMC[QDH][QDW];
  __shared__ double sX[NQXH][QH1][QW1];          // atmx%qx = max(atm1 * rpsa, 0), halo 1
  __shared__ double sB[NQXH][QH2][QW2];          // qxb3d = max(atm2 * (1/psb), 0), halo 2
  const int tid = threadIdx.x;
  const int J0 = g.jcx1() + (int)blockIdx.x * QBJ, I0 = g.icx1() + (int)blockIdx.y * QBI, k = (int)blockIdx.z + 1;
  const uint32_t P8 = g.P8, L8 = g.L8, kof = (uint32_t)(k - 1) * L8;
  (void)P8;
  const int jlo = g.j0, jhi = g.j0 + g.nj - 1, ilo = g.i0, ihi = g.i0 + g.ni - 1;
  const int kz = c->kz, nsp = q.nsp;
  const int tj = tid % QBJ, ti = tid / QBJ;
  const int j = J0 + tj, i = I0 + ti;
  const bool valid = j <= g.jcx2() && i <= g.icx2();
  const uint32_t o2 = valid ? g.o2(j, i) : g.o2(g.jce1, g.ice1), o3 = o2 + kof;
  // ---- stage (every load of a set before its LDS writes; lanes past the frame stage zero)
  for (int t = tid; t < QDW * QDH; t += QBT) {
    const int jj = t % QDW, ii = t / QDW, jg = J0 + jj, ig = I0 + ii;
    const bool ok = jg <= jhi && ig <= ihi;
    const uint32_t q2 = ok ? g.o2(jg, ig) : o2;
    const double m = LD(f.msfd, q2), u = LD(f.a1u, q2 + kof), v = LD(f.a1v, q2 + kof);
    sUMC[ii][jj] = ok ? u * m : 0.0;
    sVMC[ii][jj] = ok ? v * m : 0.0;
  }
  for (int t = tid; t < QW1 * QH1; t += QBT) {
    const int jj = t % QW1, ii = t / QW1, jg = J0 - 1 + jj, ig = I0 - 1 + ii;
    const bool ok = jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = ok ? g.o2(jg, ig) : o2;
    const double rp = LD(f.rpsa, q2);
    double x[NQXH];
#pragma unroll
    for (int n = 0; n < NQXH; n++) x[n] = n < nsp ? LD(q.a1[n], q2 + kof) : 0.0;
#pragma unroll
    for (int n = 0; n < NQXH; n++) sX[n][ii][jj] = ok ? dmax(x[n] * rp, d_zero) : 0.0;
  }
  for (int t = tid; t < QW2 * QH2; t += QBT) {
    const int jj = t % QW2, ii = t / QW2, jg = J0 - 2 + jj, ig = I0 - 2 + ii;
    const bool ok = jg >= jlo && jg <= jhi && ig >= ilo && ig <= ihi;
    const uint32_t q2 = ok ? g.o2(jg, ig) : o2;
    const double r = LD(f.rpsb, q2);
    double x[NQXH];
#pragma unroll
    for (int n = 0; n < NQXH; n++) x[n] = n < nsp ? LD(q.a2[n], q2 + kof) : 0.0;
#pragma unroll
    for (int n = 0; n < NQXH; n++) sB[n][ii][jj] = ok ? dmax(x[n] * r, d_zero) : 0.0;
  }
  __syncthreads();
  if (!valid) return;
  if (!g.gci(j, i)) {
    // the ring jce \ jci: atmc%qx = atm2%qx (:375-377)
    for (int n = 0; n < nsp; n++) ST(q.cq[n], o3, LD(q.a2[n], o3));
    return;
  }
  const double dt = s->dt;
  const double ps = LD(f.psa, o2), xm = LD(f.xmsf, o2), xkcs = LD(f.xkcs, o3);
  const double q0 = LD(f.qdot, o3), q1 = LD(f.qdot, o3 + L8);
  // start_advect's mass fluxes of the cell (Main/mod_advection.F90:111-120)
  const double uavg1 = sUMC[ti + 1][tj] + sUMC[ti][tj];
  const double uavg2 = sUMC[ti + 1][tj + 1] + sUMC[ti][tj + 1];
  const double vavg1 = sVMC[ti][tj + 1] + sVMC[ti][tj];
  const double vavg2 = sVMC[ti + 1][tj + 1] + sVMC[ti + 1][tj];
  const int kpb = f.kpbl ? (int)LD(f.kpbl, o2) : 0;
  for (int n = 0; n < nsp; n++) {
    const int b1 = tj + 1, a1 = ti + 1, b2 = tj + 2, a2 = ti + 2;
#define X1(dj, di) sX[n][a1 + (di)][b1 + (dj)]
    // hadvqx (:639-653), or the semi-Lagrangian start of qxdyn (:1378-1380)
    double tq = c->isladvec ? LD(q.sl[n], o3)
                            : d_zero + hadv_flux(c, xm, ps, uavg1, uavg2, vavg1, vavg2, X1(0, 0), X1(-1, 0),
                                                 X1(1, 0), X1(0, -1), X1(0, 1), 0);
#undef X1
    // vadv4d (:859-961): ind = 1, or 3 with iuwvadv = 1 (the PBL-top rule at kpbl)
    const double* qa = q.a1[n];
    const double c0 = LD(qa, o3);
    const double cm = (k >= 2) ? LD(qa, o3 - L8) : 0.0, cp = (k < kz) ? LD(qa, o3 + L8) : 0.0;
    if (f.kpbl) {
      auto fk = [&](int kk) { return LD(qa, o2 + (uint32_t)(kk - 1) * L8); };
      if (k >= 2) tq = tq + (uw_fg(c, k, kpb, c0, cm, fk) * q0) * c->xds[k];
      if (k + 1 <= kz) tq = tq - (uw_fg(c, k + 1, kpb, cp, c0, fk) * q1) * c->xds[k];
    } else {
      const double thr = MINQQ * MINQQ * ps;
      if (k >= 2) {
        const double fl = (q0 > d_zero) ? ((cm > thr) ? q0 * (c->twt1[k] * c0 + c->twt2[k] * cm) : d_zero)
                                        : ((c0 > thr) ? q0 * (c->twt1[k] * c0 + c->twt2[k] * cm) : d_zero);
        tq = tq + fl * c->xds[k];
      }
      if (k + 1 <= kz) {
        const double fl = (q1 > d_zero) ? ((c0 > thr) ? q1 * (c->twt1[k + 1] * cp + c->twt2[k + 1] * c0) : d_zero)
                                        : ((cp > thr) ? q1 * (c->twt1[k + 1] * cp + c->twt2[k + 1] * c0) : d_zero);
        tq = tq - fl * c->xds[k];
      }
    }
    tq = qx_diffu(g, c, j, i, tq, xkcs, [&](int dj, int di) { return sB[n][a2 + di][b2 + dj]; }, q.d6[n], o3);
    // qxten = (0 + qxdyn) + qxphy (:332-335); the forecast (:375-380)
    tq = (d_zero + tq) + (q.phy[n] ? LD(q.phy[n], o3) : d_zero);
    ST(q.cq[n], o3, LD(q.a2[n], o3) + dt * tq);
  }
}

// K_QX1 (non-hydrostatic).  The hydrometeor chains of k_nh_tend_c's qc (kernels_nh.hip) for
// qi, qr, qs at the interior cross points (owned points only, as the NH tendency kernels):
// hadvqx, vadv4d ind 1 / 3, + atmx%qx * cr (:1615-1617), diffu_x4d on the scaled xkcr, the
// sums with qxphy, the forecast; the ring jce \ jci takes atm2.
__global__ __launch_bounds__(256) void k_nh_qx_tend(Geom g, const Consts* __restrict__ c,
                                                    const StepState* __restrict__ s, NHFields f, QxArgs q) {
  THREAD_POINT(g.jce1, g.ice1);
  if (!(in(j, g.jce1, g.jce2) && in(i, g.ice1, g.ice2))) return;
  const int nsp = q.nsp, kz = c->kz;
  if (!(in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2))) {
    for (int n = 0; n < nsp; n++) F3(q.cq[n], j, i, k) = F3(q.a2[n], j, i, k);
    return;
  }
  const double dt = s->dt;
  const double xmf = F2(f.xmsf, j, i), ps = F2(f.psa, j, i), pbs = F2(f.psb, j, i);
  const double m00 = F2(f.msfd, j, i), m01 = F2(f.msfd, j, i + 1), m10 = F2(f.msfd, j + 1, i),
               m11 = F2(f.msfd, j + 1, i + 1);
  // start_advect's mass fluxes (umc = atm1 u * msfd)
  const double u1 = F3(f.a1u, j, i + 1, k) * m01 + F3(f.a1u, j, i, k) * m00;
  const double u2 = F3(f.a1u, j + 1, i + 1, k) * m11 + F3(f.a1u, j + 1, i, k) * m10;
  const double v1 = F3(f.a1v, j + 1, i, k) * m10 + F3(f.a1v, j, i, k) * m00;
  const double v2 = F3(f.a1v, j + 1, i + 1, k) * m11 + F3(f.a1v, j, i + 1, k) * m01;
  const double r0 = F2(f.rpsa, j, i), rw = F2(f.rpsa, j - 1, i), re = F2(f.rpsa, j + 1, i),
               rs = F2(f.rpsa, j, i - 1), rn = F2(f.rpsa, j, i + 1);
  const double cr = F3(f.cr, j, i, k);
  const double xkc = F3(f.xkcr, j, i, k) * c->rdxsq * pbs;      // calc_coeff's xkc
  const double thr = MINQQ * MINQQ * ps;
  const int kpb = f.kpbl ? (int)F2(f.kpbl, j, i) : 0;
  for (int n = 0; n < nsp; n++) {
    const double* a = q.a1[n];
    double cd;
    if (c->isladvec) {
      cd = d_zero + F3(q.sl[n], j, i, k);
    } else {
      const double xc = dmax(F3(a, j, i, k) * r0, d_zero), xw = dmax(F3(a, j - 1, i, k) * rw, d_zero);
      const double xe = dmax(F3(a, j + 1, i, k) * re, d_zero), xs = dmax(F3(a, j, i - 1, k) * rs, d_zero);
      const double xn = dmax(F3(a, j, i + 1, k) * rn, d_zero);
      cd = d_zero + hadv_flux(c, xmf, ps, u1, u2, v1, v2, xc, xw, xe, xs, xn, 0);
    }
    auto cflux = [&](int kk) {
      const double svv = F3(f.qdot, j, i, kk);
      const double fk = F3(a, j, i, kk), fkm = F3(a, j, i, kk - 1);
      if (f.kpbl) return uw_fg(c, kk, kpb, fk, fkm, [&](int qq) { return F3(a, j, i, qq); }) * svv;
      if (svv > d_zero) return (fkm > thr) ? svv * (c->twt1[kk] * fk + c->twt2[kk] * fkm) : d_zero;
      return (fk > thr) ? svv * (c->twt1[kk] * fk + c->twt2[kk] * fkm) : d_zero;
    };
    if (k >= 2) cd = cd + cflux(k) * c->xds[k];
    if (k + 1 <= kz) cd = cd - cflux(k + 1) * c->xds[k];
    cd = cd + dmax(F3(a, j, i, k) * r0, d_zero) * cr;
    if (c->idiffu == 3) {
      if (j == g.jci2) cd = cd + F3(q.d6[n], j, i, k);
    } else {
      // diffu_x4d on mkslice's qxb3d = max(atm2 * (1/psb), 0), Main/mod_diffusion.F90:792-947
      const double* b = q.a2[n];
      auto fb = [&](int dj, int di) {
        return dmax(F3(b, j + dj, i + di, k) * F2(f.rpsb, j + dj, i + di), d_zero);
      };
      if (c->idiffu == 2) {
        cd = cd + d_one * xkc * (o4_c1 * (fb(1, 0) + fb(-1, 0) + fb(0, 1) + fb(0, -1)) +
                                 o4_c2 * (fb(1, 1) + fb(-1, -1) + fb(-1, 1) + fb(1, -1)) + o4_c3 * fb(0, 0));
      } else {
        if (in(j, g.jcii1, g.jcii2) && in(i, g.icii1, g.icii2))
          cd = cd - d_one * xkc * (z4_c1 * (fb(2, 0) + fb(-2, 0) + fb(0, 2) + fb(0, -2)) +
                                   z4_c2 * (fb(1, 0) + fb(-1, 0) + fb(0, 1) + fb(0, -1)) + z4_c3 * fb(0, 0));
        const double lap = z4_c1 * (fb(1, 0) + fb(-1, 0) + fb(0, 1) + fb(0, -1)) + z4_c2 * fb(0, 0);
        const int nb = (g.bl && j == g.jci1) + (g.br && j == g.jci2) + (g.bb && i == g.ici1) + (g.bt && i == g.ici2);
        for (int r = 0; r < nb; r++) cd = cd + d_one * xkc * lap;
      }
    }
    const double qt = d_zero + cd + (q.phy[n] ? F3(q.phy[n], j, i, k) : d_zero);
    F3(q.cq[n], j, i, k) = F3(q.a2[n], j, i, k) + dt * qt;
  }
}

// K_QX2.  The negative-moisture fix (:382-393) and filter_raw_4d (:426-427, gnu2, the zero
// floor) of the hydrometeors beyond qc on the owned interior jci x ici, into the next buffers; the
// copies of the column box's other points (atm1, and atm2 on owned points: bdyval and the next
// step's exchange read them).  A negative point with a negative sweep-predecessor flags its
// (species, level) plane for k_qx_serial; the others read original values only.
__global__ void k_qx_fix(Geom g, const Consts* __restrict__ c, QxArgs q) {
  THREAD_POINT(g.jdx1(), g.idx1());
  if (j > g.jdx2() || i > g.idx2()) return;
  const uint32_t o3 = g.o3(j, i, k);
  const bool ci = in(j, g.jci1, g.jci2) && in(i, g.ici1, g.ici2);
  const bool own = in(j, g.jde1, g.jde2) && in(i, g.ide1, g.ide2);
  const double beta = 0.53;
  for (int n = 0; n < q.nsp; n++) {
    const double a1 = LD(q.a1[n], o3), a2 = LD(q.a2[n], o3);
    if (!ci) {
      if (q.b1[n] != q.a1[n]) {             // the NH core filters in place: nothing to keep
        ST(q.b1[n], o3, a1);
        if (own) ST(q.b2[n], o3, a2);
      }
      continue;
    }
    double v = LD(q.cq[n], o3);
    // a dependent point flags its row with a plain store (every writer stores the same 1, so
    // it holds for any block shape; the lanes of one row store one address, a single
    // transaction; device-scope atomics on the few bitmap words serialised at the memory side:
    // 190 of this kernel's 215 us at C3)
    const bool dp = v < d_zero && negfix_dependent(g, q.cq[n], j, i, k);
    if (dp) {
      q.depf[(n * c->kz + (k - 1)) * (g.ici2 - g.ici1 + 1) + (i - g.ici1)] = 1u;
      continue;
    }
    if (v < d_zero) {
      v = negfix_sum(g, q.cq[n], q.fq[n], j, i, k, false);
      ST(q.fq[n], o3, v);
    }
    const double d = c->gnu2 * (v + a2 - d_two * a1);
    double m = a1 + beta * d, x = v + (beta - d_one) * d;
    if (m < d_zero) m = d_zero;
    if (x < d_zero) x = d_zero;
    ST(q.b2[n], o3, m);
    ST(q.b1[n], o3, x);
  }
}

// K_QX3.  The serial sweep of one (species, level) plane by one wavefront (negfix_sweep,
// qxcommon.hpp): the marked rows' dependent negative points in i-major, j-minor order, each
// fixed from its already-fixed predecessors, then RAW-filtered; dynamic LDS negfix_lds(g)
// filter_raw_4d of a fixed point (gnu2, the zero floor) from its atm1, atm2 (x)
struct QxRaw {
  static constexpr int NI = 2;
  Geom g;
  const double *a1, *a2;
  double *b1, *b2;
  double gnu2;
  int k;
  __device__ void load(int j, int i, double* x) const { x[0] = F3(a1, j, i, k); x[1] = F3(a2, j, i, k); }
  __device__ void apply(int j, int i, double v, const double* x) const {
    const double beta = 0.53;
    const double d = gnu2 * (v + x[1] - d_two * x[0]);
    double m = x[0] + beta * d, y = v + (beta - d_one) * d;
    if (m < d_zero) m = d_zero;
    if (y < d_zero) y = d_zero;
    F3(b2, j, i, k) = m;
    F3(b1, j, i, k) = y;
  }
};
// one (species, level) plane of k_qx_serial (lds: negfix_lds(g) doubles)
__device__ __forceinline__ void qx_serial_plane(const Geom& g, const Consts* __restrict__ c, const QxArgs& q,
                                                int plane, double* lds) {
  const int kz = c->kz;
  if (plane >= q.nsp * kz) return;
  const int n = plane / kz, k = plane % kz + 1;
  {
    // k_qx_fix's row flags into this plane's bitmap words (negfix_resolve reads those), flags
    // cleared for the next step
    const int R = g.ici2 - g.ici1 + 1, T = (int)(blockDim.x * blockDim.y * blockDim.z);
    const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
    unsigned* fl = q.depf + plane * R;
    unsigned* words = q.dep + plane * negfix_rowwords(g);
    for (int b = 0; b < R; b += T) {
      const int r = b + tid;
      const bool f = r < R && fl[r] != 0u;
      if (f) fl[r] = 0u;
      const unsigned long long m = __ballot(f);
      if (r < R && (r & 31) == 0) words[r >> 5] = (unsigned)(m >> (r & 32));
    }
    __syncthreads();
  }
  if (NEGFIX_POST) {
    negfix_resolve(g, q.cq[n], q.fq[n], q.dep, plane, k, lds, negfix_lds(g), NoPost{}, [](int, int, double) {}, c->negfix_mode);
    return;
  }
  const QxRaw acc{g, q.a1[n], q.a2[n], q.b1[n], q.b2[n], c->gnu2, k};
  negfix_resolve(g, q.cq[n], q.fq[n], q.dep, plane, k, lds, negfix_lds(g), acc, [&](int jj, int i, double v) {
    double x[2];
    acc.load(jj, i, x);
    acc.apply(jj, i, v, x);
  }, c->negfix_mode);
}
__global__ __launch_bounds__(512) void k_qx_serial(Geom g, const Consts* __restrict__ c, QxArgs q) {
  extern __shared__ double lds[];
  qx_serial_plane(g, c, q, (int)blockIdx.x, lds);
}
// NEGFIX_POST, hydrostatic qfuse: the serial chains of the qv / qc planes (blocks [0, 2 kz), as
// k_negfix_serial) and of the species planes (k_qx_serial) in one launch after the split
// corrections: the two sets of planes are independent, so the launch takes the longer chain's
// time instead of the sum (k_qx_fix's flags wait for it; nothing of the split reads the species)
__global__ __launch_bounds__(512) void k_negfix_serial_qx(Geom g, const Consts* __restrict__ c, QFix qf, QxArgs q) {
  extern __shared__ double lds[];
  const int b = (int)blockIdx.x, kz = c->kz;
  if (b >= 2 * kz) {
    qx_serial_plane(g, c, q, b - 2 * kz, lds);
    return;
  }
  const int n = b / kz, k = b % kz + 1;
  if (qf.depf) {
    negfix_collect(g, qf.depf, qf.depplane, b, (int)threadIdx.x, (int)blockDim.x);
    __syncthreads();
  }
  negfix_resolve(g, n ? qf.cqc : qf.cqv, n ? qf.fqc : qf.fqv, qf.depplane, b, k, lds, negfix_lds(g), NoPost{},
                 [](int, int, double) {}, c->negfix_mode);
}

// NEGFIX_POST: filter_raw_4d of the points k_qx_serial fixed, a thread per interior point of a
// (species, level) plane (z = plane)
__global__ void k_qx_post(Geom g, const Consts* __restrict__ c, QxArgs q) {
  const int j = g.jci1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int i = g.ici1 + (int)(blockIdx.y * blockDim.y + threadIdx.y);
  const int plane = (int)blockIdx.z, kz = c->kz, n = plane / kz, k = plane % kz + 1;
  if (j > g.jci2 || i > g.ici2 || n >= q.nsp) return;
  if (!negfix_is_dependent(g, q.cq[n], j, i, k)) return;
  const QxRaw acc{g, q.a1[n], q.a2[n], q.b1[n], q.b2[n], c->gnu2, k};
  double x[2];
  acc.load(j, i, x);
  acc.apply(j, i, F3(q.fq[n], j, i, k), x);
}

// K_QX4.  bdyval for the hydrometeors beyond qc, one block per (level, species): while
// integrating, atm2 = atm1 on the cross boundary lines (Main/mod_bdycod.F90:1143-1284: west /
// east on ici, south / north on jce), then (not present_qc) the inflow/outflow lines of qc's
// rule (:2153-2220), which read the bdyuv slices and the boundary p* of this bdyval.
__global__ void k_bdyval_qx(Geom g, const StepState* __restrict__ s, QxArgs q, int integ, int do_qc,
                            const double* __restrict__ psa, Slices sl, long slen) {
  const int k = (int)blockIdx.x + 1, n = (int)blockIdx.y;
  if (n >= q.nsp) return;
  double* a1 = q.a1[n];
  double* a2 = q.a2[n];
  if (integ > 0 || (integ < 0 && s->lcount > 0)) {
    for (int i = g.ici1 + (int)threadIdx.x; i <= g.ici2; i += (int)blockDim.x) {
      if (g.bl) F3(a2, g.jce1, i, k) = F3(a1, g.jce1, i, k);
      if (g.br) F3(a2, g.jce2, i, k) = F3(a1, g.jce2, i, k);
    }
    for (int j = g.jce1 + (int)threadIdx.x; j <= g.jce2; j += (int)blockDim.x) {
      if (g.bb) F3(a2, j, g.ice1, k) = F3(a1, j, g.ice1, k);
      if (g.bt) F3(a2, j, g.ice2, k) = F3(a1, j, g.ice2, k);
    }
    __syncthreads();
  }
  bdyval_qc_level(g, do_qc, 0, a1, nullptr, [&](int j, int i) { return F2(psa, j, i); }, sl, slen, k);
}

}  // namespace rcm
