// bdyin.hpp -- argument block of the device bdyin kernels (bdyin.hip).
#pragma once
#include "devcommon.hpp"

namespace rcm {

// r*: the raw record (read_icbc units) put by the host; *0 / *1 / *t: the coupled boundary
// data at the interval start / end and its time tendency (v3dbound / v2dbound b0, b1, bt)
struct BdyinArgs {
  const double *rub, *rvb, *rtb, *rqb, *rpb, *rppb, *rwwb, *ps0, *psdot0;
  double *ub0, *ubt, *ub1, *vb0, *vbt, *vb1, *tb0, *tbt, *tb1, *qb0, *qbt, *qb1, *pb0, *pbt, *pb1;
  double *ppb0, *ppbt, *ppb1, *wwb0, *wwbt, *wwb1;
  double rdtbdy, ptop;
  int kz, nh;
};

__global__ void k_bdyin_shift(Geom g, BdyinArgs a);
__global__ void k_bdyin_ps(Geom g, BdyinArgs a);
__global__ void k_bdyin_couple(Geom g, BdyinArgs a);
__global__ void k_bdyin_timeint(Geom g, BdyinArgs a);

}  // namespace rcm
