// bdyin.hip -- the ICBC boundary pipeline on the device:
// mod_bdycod::bdyin from read_icbc on (Main/mod_bdycod.F90:654-889).  The host reads the next
// record (its NetCDF I/O is unchanged) and puts it uncoupled; these kernels shift b1 into b0,
// convert and couple the record into b1 and form bt (timeint), in the reference's order with
// the two exchanges of b1 (p* before psc2psd, the coupled fields after) done by the engine.
// Every value is one product or difference of the reference's (-ffp-contract=off): exact.
#include "bdyin.hpp"

namespace rcm {

// b0 <- b1 over the whole frame (xub%b0(:,:,:) = xub%b1(:,:,:), :670-690)
__global__ void k_bdyin_shift(Geom g, BdyinArgs a) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const long q = (long)(k - 1) * g.plane + g.ix(j, i);
  if (k <= a.kz) {
    a.ub0[q] = a.ub1[q]; a.vb0[q] = a.vb1[q]; a.tb0[q] = a.tb1[q]; a.qb0[q] = a.qb1[q];
    if (a.nh) a.ppb0[q] = a.ppb1[q];
  }
  if (a.nh) a.wwb0[q] = a.wwb1[q];
  else if (k == 1) a.pb0[q] = a.pb1[q];
}

// p* of the record on the owned cross points: hydrostatic (ps*d_r10) - ptop (:757-760);
// non-hydrostatic xpsb%b1 = xpsb%b0 = atm0%ps*d_r1000 (:398-400)
__global__ void k_bdyin_ps(Geom g, BdyinArgs a) {
  THREAD_POINT(g.jce1, g.ice1);
  if (j > g.jce2 || i > g.ice2) return;
  F2(a.pb1, j, i) = a.nh ? F2(a.ps0, j, i) * 0.001 : (F2(a.rpb, j, i) * 0.1) - a.ptop;
}

// couple (:781-799, Main/mod_bdycod.F90:4938-4951): u, v with psdot on the owned dot points
// (psc2psd of the exchanged p*, :761; NH atm0%psdot*d_r1000, :399), t, qv, pp, w with p* on
// the owned cross points
__global__ void k_bdyin_couple(Geom g, BdyinArgs a) {
  THREAD_POINT(g.jde1, g.ide1);
  if (j > g.jde2 || i > g.ide2) return;
  const long q = (long)(k - 1) * g.plane + g.ix(j, i);
  if (k <= a.kz) {
    double psdot = 0.0;
    bool ok;
    if (a.nh) { psdot = F2(a.psdot0, j, i) * 0.001; ok = true; }
    else ok = psc2psd_at(g, a.pb1, j, i, psdot);
    if (ok) { a.ub1[q] = a.rub[q] * psdot; a.vb1[q] = a.rvb[q] * psdot; }
  }
  if (!in(j, g.jce1, g.jce2) || !in(i, g.ice1, g.ice2)) return;
  const double ps = F2(a.pb1, j, i);
  if (k <= a.kz) {
    a.tb1[q] = a.rtb[q] * ps;
    a.qb1[q] = a.rqb[q] * ps;
    if (a.nh) a.ppb1[q] = a.rppb[q] * ps;
  }
  if (a.nh) a.wwb1[q] = a.rwwb[q] * ps;
}

// timeint (:801-825, :5087-5113) on jde1ga:jde2ga x ide1ga:ide2ga (u, v) and the cross ga
// ranges (t, qv, p*, pp, w)
__global__ void k_bdyin_timeint(Geom g, BdyinArgs a) {
  THREAD_POINT(g.j0, g.i0);
  if (j >= g.j0 + g.nj || i >= g.i0 + g.ni) return;
  const int jd1 = g.jde1 - (g.bl ? 0 : 1), jd2 = g.jde2 + (g.br ? 0 : 1);
  const int id1 = g.ide1 - (g.bb ? 0 : 1), id2 = g.ide2 + (g.bt ? 0 : 1);
  const int jc1 = g.jce1 - (g.bl ? 0 : 1), jc2 = g.jce2 + (g.br ? 0 : 1);
  const int ic1 = g.ice1 - (g.bb ? 0 : 1), ic2 = g.ice2 + (g.bt ? 0 : 1);
  const long q = (long)(k - 1) * g.plane + g.ix(j, i);
  const double r = a.rdtbdy;
  if (k <= a.kz && in(j, jd1, jd2) && in(i, id1, id2)) {
    a.ubt[q] = (a.ub1[q] - a.ub0[q]) * r;
    a.vbt[q] = (a.vb1[q] - a.vb0[q]) * r;
  }
  if (!in(j, jc1, jc2) || !in(i, ic1, ic2)) return;
  if (k <= a.kz) {
    a.tbt[q] = (a.tb1[q] - a.tb0[q]) * r;
    a.qbt[q] = (a.qb1[q] - a.qb0[q]) * r;
    if (a.nh) a.ppbt[q] = (a.ppb1[q] - a.ppb0[q]) * r;
  }
  if (a.nh) a.wwbt[q] = (a.wwb1[q] - a.wwb0[q]) * r;
  else if (k == 1) a.pbt[q] = (a.pb1[q] - a.pb0[q]) * r;
}

}  // namespace rcm
