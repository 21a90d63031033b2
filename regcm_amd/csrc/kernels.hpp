// kernels.hpp -- declarations of the device kernels in kernels.hip (generated list).
#pragma once
#include "engine.hpp"

namespace rcm {

// one halo staging segment (see k_pack_segs)
struct Seg {
  double* p;
  long kstride;
  int pitch, j0, i0, j1, j2, i1, i2, nk;
  long off;
};
constexpr int MAXSEG = 64;
// fused spstep tiling: SPB x SPB owned cross points + SPH halo (>= sub-steps per mode)
constexpr int SPB = 16, SPH = 8;
struct SegList {
  Seg s[MAXSEG];
  int n;
};

// boundary slices, order documented at k_bdyval_set
struct Slices { double* s[16]; };

__global__ void k_surface_pressures(Geom g, const double* __restrict__ psa, const double* __restrict__ psb, double* rpsa, double* rpsb, double* psdota, double* psdotb);
__global__ void k_psc2psd(Geom g, const double* __restrict__ pc, double* pd);
__global__ void k_decouple(Geom g, const double* __restrict__ a1u, const double* __restrict__ a1v, const double* __restrict__ a1t, const double* __restrict__ a1qv, const double* __restrict__ a1qc, const double* __restrict__ msfd, const double* __restrict__ psdota, const double* __restrict__ rpsa, double* rpsda, double* umc, double* vmc, double* ud, double* vd, double* xt, double* xqv, double* xqc, double* xtv, double ep1);
__global__ void k_omega_col(Geom g, const Consts* __restrict__ c, const double* __restrict__ umc, const double* __restrict__ vmc, const double* __restrict__ msfx, const double* __restrict__ rpsa, double* pten, double* qdot);
__global__ void k_mkslice(Geom g, const double* __restrict__ a2u, const double* __restrict__ a2v, const double* __restrict__ a2t, const double* __restrict__ a2qv, const double* __restrict__ a2qc, const double* __restrict__ psb, const double* __restrict__ psdotb, double* ubd, double* vbd, double* tb3d, double* qvb, double* qcb);
__global__ void k_new_pressure(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, const double* __restrict__ psa, const double* __restrict__ psb, const double* __restrict__ pb0, const double* __restrict__ pbt, const int8_t* __restrict__ rgcr, const int16_t* __restrict__ ibcr, const double* __restrict__ pten, double* ptenn, double* psc, double* rpsc, double* red);
__global__ void k_reduce_noise(const double* __restrict__ red, int nblk, StepState* s);
__global__ void k_calc_coeff(Geom g, const Consts* __restrict__ c, const double* __restrict__ ubd, const double* __restrict__ vbd, const double* __restrict__ hgfact, double* xkc);
__global__ void k_phi_col(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1t, const double* __restrict__ xqv, const double* __restrict__ xqc, const double* __restrict__ psa, const double* __restrict__ rpsa, const double* __restrict__ ht, double* phi);
__global__ void k_momentum(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, const double* __restrict__ a1u, const double* __restrict__ a1v, const double* __restrict__ a2u, const double* __restrict__ a2v, double* __restrict__ n1u, double* __restrict__ n1v, double* __restrict__ n2u, double* __restrict__ n2v, const double* __restrict__ umc, const double* __restrict__ vmc, const double* __restrict__ ud, const double* __restrict__ vd, const double* __restrict__ qdot, const double* __restrict__ coriol, const double* __restrict__ dmsf, const double* __restrict__ msfd, const double* __restrict__ ub0, const double* __restrict__ ubt, const double* __restrict__ vb0, const double* __restrict__ vbt, const int8_t* __restrict__ rgdt, const int16_t* __restrict__ ibdt, const double* __restrict__ xkc, const double* __restrict__ psdotb, const double* __restrict__ ubd, const double* __restrict__ vbd, const double* __restrict__ xtv, const double* __restrict__ psdota, const double* __restrict__ psa, const double* __restrict__ phi, double* uten, double* vten);
__global__ void k_temperature(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, const double* __restrict__ a1t, const double* __restrict__ a2t, double* __restrict__ n1t, double* __restrict__ n2t, const double* __restrict__ xt, const double* __restrict__ umc, const double* __restrict__ vmc, const double* __restrict__ psa, const double* __restrict__ psb, const double* __restrict__ xmsf, const double* __restrict__ qdot, const double* __restrict__ pten, const double* __restrict__ ud, const double* __restrict__ vd, const double* __restrict__ msfx, const double* __restrict__ xqv, const double* __restrict__ xtv, const double* __restrict__ rpsa, const double* __restrict__ tb0, const double* __restrict__ tbt, const int8_t* __restrict__ rgcr, const int16_t* __restrict__ ibcr, const double* __restrict__ xkc, const double* __restrict__ tb3d, double* tten, double* omegad, double* xkcs_d);
__global__ void k_moisture(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, const double* __restrict__ a1qv, const double* __restrict__ a1qc, const double* __restrict__ a2qv, const double* __restrict__ a2qc, const double* __restrict__ xqv, const double* __restrict__ xqc, const double* __restrict__ umc, const double* __restrict__ vmc, const double* __restrict__ psa, const double* __restrict__ psb, const double* __restrict__ xmsf, const double* __restrict__ qdot, const double* __restrict__ qb0, const double* __restrict__ qbt, const int8_t* __restrict__ rgcr, const int16_t* __restrict__ ibcr, const double* __restrict__ xkc, const double* __restrict__ qvb, const double* __restrict__ qcb, double* cqv, double* cqc, double* qvten, double* qcten);
__global__ void k_ps_filter(Geom g, const Consts* __restrict__ c, double* psa, double* psb, const double* __restrict__ psc);
__global__ void k_negfix(Geom g, int kz, const double* __restrict__ cqv, const double* __restrict__ cqc, double* fqv, double* fqc, uint8_t* dep, int* depplane);
__global__ void k_negfix_serial(Geom g, int kz, const double* __restrict__ cqv, const double* __restrict__ cqc, double* fqv, double* fqc, const uint8_t* __restrict__ dep, int* depplane);
__global__ void k_moisture_filter(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1qv, const double* __restrict__ a1qc, const double* __restrict__ a2qv, const double* __restrict__ a2qc, double* n1qv, double* n1qc, double* n2qv, double* n2qc, const double* __restrict__ fqv, const double* __restrict__ fqc, const double* __restrict__ psa, const double* __restrict__ psb);
__global__ void k_split_project(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1u, const double* __restrict__ a1v, const double* __restrict__ a2u, const double* __restrict__ a2v, const double* __restrict__ a1t, const double* __restrict__ a2t, const double* __restrict__ psa, const double* __restrict__ psb, const double* __restrict__ msfd, const double* __restrict__ mapf, double* dstor, double* hstor, double* deld, double* delh);
__global__ void k_spstep_init(Geom g, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh, double* ddsum, double* dhsum);
__global__ void k_spstep_grad(Geom g, const Consts* __restrict__ c, int l, int src, const double* __restrict__ delh, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota, double* uu, double* vv);
__global__ void k_spstep_update(Geom g, const Consts* __restrict__ c, int l, int n0, int n1, int nn, int leap, const double* __restrict__ uu, const double* __restrict__ vv, const double* __restrict__ mapf, const double* __restrict__ psa, double* deld, double* delh, double* ddsum, double* dhsum);
__global__ void k_split_correct(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum, const double* __restrict__ dhsum, const double* __restrict__ psdota, const double* __restrict__ msfd, double* psa, double* psb, double* a1t, double* a2t, double* a1u, double* a1v, double* a2u, double* a2v);
__global__ void k_advance_time(StepState* s, double dtsec);
__global__ void k_bdyval_set(Geom g, const StepState* __restrict__ s, double* a1u, double* a1v, double* a1t, double* a1qv, double* a1qc, double* a2u, double* a2v, double* a2t, double* a2qv, double* a2qc, double* psa, double* psb, const double* __restrict__ ub0, const double* __restrict__ ubt, const double* __restrict__ vb0, const double* __restrict__ vbt, const double* __restrict__ tb0, const double* __restrict__ tbt, const double* __restrict__ qb0, const double* __restrict__ qbt, const double* __restrict__ pb0, const double* __restrict__ pbt, Slices sl, long slen);
__global__ void k_bdyval_corners(Geom g, int kz, Slices sl, long slen);
__global__ void k_bdyval_qc_we(Geom g, int kz, double* a1qc, const double* __restrict__ psa, Slices sl, long slen);
__global__ void k_bdyval_qc_sn(Geom g, int kz, double* a1qc, const double* __restrict__ psa, Slices sl, long slen);
__global__ void k_bdyval_time(StepState* s, double dtsec);
__global__ void k_prepare_static(Geom g, const Consts* __restrict__ c, int diffu_hgtf, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ ht, double* xmsf, double* dmsf, double* hgfact, double* mapf);
__global__ void k_spstep_fused(Geom g, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota, const double* __restrict__ mapf, const double* __restrict__ psa, double* ddsum, double* dhsum);
__global__ void k_pack_segs(SegList L, double* __restrict__ buf, int unpack);

}  // namespace rcm
