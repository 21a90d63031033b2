// slice.hpp -- argument block of the mkslice export kernel (slice.hip).
#pragma once
#include "devcommon.hpp"

namespace rcm {

// inputs: the state at the start of the step and the 2-D reciprocals of k_surface_pressures;
// outputs: the atms fields of Main/mod_slice.F90 (rcmdyn_field ATMS_*)
struct SliceArgs {
  const double *a1u, *a1v, *a2u, *a2v, *a2t, *a2qv, *a2qc, *psa, *psb;
  const double *rpsb, *rpsdb, *rpsda, *msfx, *qdot, *pten;
  const double *a2pp, *a2w, *ps0, *pr0, *pf0, *rho0;       // non-hydrostatic core only
  double *ubx3d, *vbx3d, *ubd3d, *vbd3d, *tb3d, *qvb3d, *qcb3d, *tv3d, *pb3d, *pf3d, *ps2d, *rhox2d;
  double *th3d, *rhob3d, *tp3d, *wpx3d, *wb3d, *zq, *za, *dzq, *qsb3d, *rhb3d;
  double ep2, rhmin, rhmax;
  // nqx = 5: qxb3d of qi, qr, qs (Main/mod_slice.F90:193-195), from atm2 (null for nqx = 2)
  const double* a2qx[NQXH];
  double* qxb3d[NQXH];
};

__global__ void k_slice(Geom g, const Consts* __restrict__ c, SliceArgs a);

}  // namespace rcm
