/*
 * rcmdyn.h -- C-ABI of the MI355X-native RegCM4 dynamical-core step engine.
 *
 * Drop-in boundary for the reference hot path:
 *
 *   reference seam                                  replaced by
 *   ---------------------------------------------   -------------------------------
 *   call tend        Main/mod_regcm_interface.F90:189 rcmdyn_tend()
 *   call bdyval      Main/mod_regcm_interface.F90:208 rcmdyn_bdyval()
 *   tend+bdyval loop Main/mod_regcm_interface.F90:172-228   rcmdyn_step()
 *   module state     Main/mod_atm_interface.F90:39-70 rcmdyn_put()/rcmdyn_get()
 *   bdyin (b0,bt)    Main/mod_bdycod.F90:654-889      put XxB_B0/BT + rcmdyn_set_time(xbctime)
 *   mkslice -> physics -> sums  Main/mod_tendency.F90:243,271,285-411
 *                    rcmdyn_tend_pre_physics() + get ATMS_* / put *PHY + rcmdyn_tend_post_physics()
 *   rcmtimer/dt/xbctime Main/mpplib/mod_runparams.F90 rcmdyn_set_time()/get_time()
 *   exchange*        Main/mpplib/mod_mppparam.F90:6065-13190  internal (local copies / RCCL)
 *   fatal('CFL VIOLATION') Main/mod_tendency.F90:702  return code + rcmdyn_last_error()
 *
 * Conventions
 *  - Every entry point returns 0 on success, non-zero on failure; the message of the
 *    last failure is available from rcmdyn_last_error().
 *  - Host arrays cross the boundary in the reference's Fortran layout: column-major
 *    (j fastest, then i, then k), with explicit GLOBAL index bounds j1:j2, i1:i2, k1:k2
 *    (Fortran 1-based, as allocated by getmem*: Share/mod_memutil.F90).  In C/numpy
 *    terms that is a C-order [k][i][j] array.  The engine copies the intersection of
 *    the host box with the tiles it owns; it never keeps a host pointer.
 *  - All arithmetic is fp64 (rkx = rk8, Share/mod_realkinds.F90:44-55).
 *  - No torch / HIP types appear in any signature.
 */
#ifndef RCMDYN_H
#define RCMDYN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RCMDYN_ABI_VERSION 6
#define RCMDYN_MAXKZ 64
#define RCMDYN_MAXSPLIT 4

/* Run/grid configuration.  Scalars mirror the namelist / mod_runparams globals that
 * the reference dyn core reads (Share/mod_dynparam.F90:453-476, Main/mod_params.F90:85-170,
 * Main/mpplib/mod_runparams.F90:97-232).  Vertical-mode constants are the outputs of the
 * host-side init (spinit/vmodes, Main/mod_split.F90:75-239, Main/mod_vmodes.F90:86-594). */
typedef struct rcmdyn_config {
  int32_t abi_version;          /* = RCMDYN_ABI_VERSION */
  /* global grid: jx (west-east dot points), iy (south-north), kz (levels) */
  int32_t jx, iy, kz;
  /* 2-D decomposition in tiles (set_nproc rule, Main/mpplib/mod_mppparam.F90:1133-1186);
   * tile t has cartesian location (t / nproc_i, t % nproc_i) = (j-coord, i-coord). */
  int32_t nproc_j, nproc_i;
  /* tiles owned by this engine instance: [tile_first, tile_first + tile_count) */
  int32_t tile_first, tile_count;
  /* dynamics options (defaults in brackets) */
  int32_t idynamic;             /* [1] hydrostatic, 2 = non-hydrostatic (MM5-type, sound) */
  int32_t iboudy;               /* [5] exponential relaxation (1 = linear) */
  int32_t idiffu;               /* [1] 1: 4th-order, 2: 9-point, 3: 6th-order flux-limited on each
                                   tile's last interior column (Main/mod_diffusion.F90:412-942) */
  int32_t ipgf;                 /* [0] */
  int32_t nsplit;               /* [2] */
  int32_t nspgx, nspgd;         /* [12,12] boundary relaxation band width */
  int32_t diffu_hgtf;           /* [1] topographic diffusion reduction */
  int32_t upstream_mode;        /* [1] */
  int32_t stability_enhance;    /* [1] */
  int32_t present_qc;           /* [0] ICBC carries qc (Main/mod_bdycod.F90:306-310) */
  /* scalars */
  double ds;                    /* grid spacing, km */
  double dtsec;                 /* namelist dt, s */
  double ptop;                  /* model top, cb */
  double gnu1, gnu2;            /* Robert-Asselin [0.0625] */
  double uoffc;                 /* [0.25] */
  double t_extrema;             /* [5] */
  double q_rel_extrema;         /* [0.2] */
  double ckh, adyndif;          /* [1,1] */
  double high_nudge, medium_nudge, low_nudge; /* [3,2,1] */
  double bdy_nm, bdy_dm;        /* [-1,-1] -> derived from dt */
  double dtbdys;                /* boundary interval, s [6*3600] */
  /* vertical structure */
  double sigma[RCMDYN_MAXKZ + 1];          /* full sigma levels, k = 1..kz+1 */
  /* split-explicit constants (after spinit scaling), Fortran index order noted */
  double zmatx[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ];   /* zmatx(k,l) -> zmatx[l-1][k-1] */
  double zmatxr[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ];  /* zmatxr(l,k) -> zmatxr[l-1][k-1] */
  double am[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ];      /* am(k,l) -> am[l-1][k-1] */
  double tau[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ];     /* tau(l,k) -> tau[l-1][k-1] */
  double varpa1[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ + 1]; /* varpa1(l,k) -> varpa1[l-1][k-1] */
  double an[RCMDYN_MAXSPLIT];
  double hbar[RCMDYN_MAXSPLIT];
  double aam[RCMDYN_MAXSPLIT];
  double dtau[RCMDYN_MAXSPLIT];
  double sigmah[RCMDYN_MAXKZ + 1];
  double pd;                    /* vmodes reference p* (cb) */
  /* multi-process (RCCL) -- used only when tile_count < nproc_j*nproc_i */
  int32_t comm_rank, comm_size; /* process rank / size in the RCCL communicator */
  int32_t device;               /* HIP device ordinal, -1 = current */
  uint8_t comm_unique_id[128];  /* ncclUniqueId from rcmdyn_comm_unique_id() on rank 0 */
  /* non-hydrostatic core (idynamic = 2): nonhydroparam, Main/mod_params.F90:115-116,287-296 */
  int32_t ifupr;                /* [1] upper radiative boundary condition in sound */
  int32_t ifrayd;               /* [1] Rayleigh damping of the top levels */
  int32_t rayndamp;             /* [5] number of damped levels */
  int32_t nh_reserved;
  double nhbet, nhxkd;          /* [0.4, 0.1] Ikawa beta, divergence damping */
  double rayalpha0, rayhd;      /* [3e-4 1/s, 10000 m] */
  /* init_sound outputs (Main/mod_sound.F90:115-161), computed by the host once:
   * nh_dtsmax = dx / sqrt(gamma R max(t0)) / (1 + nhxkd), nh_xmsf = mean of msfx over the
   * interior cross points (the global sumall of :143-145) */
  double nh_dtsmax, nh_xmsf;
  /* cldparam relative-humidity clamps of the mkslice export (Main/mod_params.F90:331-332,
   * Main/mod_slice.F90:336-337) [rhmin 0.01, rhmax 1.01] */
  double rhmin, rhmax;
  /* physicsparam isladvec [0] (1 = semi-Lagrangian horizontal advection of the moisture,
   * Main/mod_sladvection.F90, both cores) and iqmsl [1] (its quasi-monotone limiter),
   * Main/mod_params.F90:100, 243-244 */
  int32_t isladvec, iqmsl;
  /* physicsparam ibltyp [1]: 2 = UW PBL, whose TKE the dyn step advects, diffuses, forecasts
   * and filters (Main/mod_tendency.F90:515-544, 1414-1425, 1545-1548) and bounds
   * (Main/mod_bdycod.F90:1166-1306, 2415-2530); uwparam nuk [5] (its diffusion factor,
   * Main/mod_params.F90:480); tkemin (uwtkemin = 1e-3, Main/pbllib/mod_pbl_uwtcm.F90:86,
   * Main/mod_pbl_interface.F90:68).  uwparam iuwvadv [0]: with ibltyp = 2, 1 selects the
   * PBL-aware vertical flux of the hydrometeors (vadv4d ind = 3, iqxvadv = 3,
   * Main/mod_tendency.F90:148-154, Main/mod_advection.F90:917-961), which reads the host's
   * KPBL field; ignored unless ibltyp = 2, as in the reference */
  int32_t ibltyp, iuwvadv;
  double nuk, tkemin;
  /* ABI 6.  physicsparam ipptls [1] and nqx, the number of moisture species param sets from
   * it (Main/mod_params.F90:1358-1366): nqx = 2 (qv, qc) for ipptls = 1 (SUBEX), nqx = 5 (qv,
   * qc, qi, qr, qs) for ipptls = 2 (WSM5 / Nogherotto-Tompkins).  Every hydrometeor
   * n = iqfrst..iqlst (qc and, with nqx = 5, qi, qr, qs) gets the qc chain of the dyn step:
   * hadvqx, vadv4d, diffu_x4d, the forecast and negative-value fix, filter_raw_4d with the zero
   * floor, bdyval's boundary copies and inflow/outflow lines; the total water load qcd (the sum
   * of the hydrometeors, Main/mod_tendency.F90:1107-1115) enters the geopotential's tvfac and
   * the NH water loading.  ipptls = 0 (no moisture scheme: the hydrometeor tendencies are never
   * summed, :331) and an nqx that does not match ipptls are refused. */
  int32_t ipptls, nqx;
  /* i_band = 1 (dimparam, hydrostatic core): the tropical band, periodic in j
   * (Main/mpplib/mod_mppparam.F90:1062, 1112-1114, 1131): no tile has a west or east boundary,
   * the tiles of the first and last tile column are neighbours (one tile in j is its own west
   * and east neighbour: its periodic exchange is a copy inside the tile), the cross grid takes
   * every j (:1351-1354: cross fields are defined on j = 1..jx), and only the south and north
   * rows relax to the boundary data (Main/mod_atm_interface.F90:435-457).  A put fills a band
   * tile's frame columns past either end of the period from the wrapped columns.  Refused for
   * idynamic = 2 and for values other than 0 and 1.
   * Options of the reference that this engine does not compute; a non-zero value is refused
   * at rcmdyn_create ('not supported'): i_crm = 1 (cloud-resolving, periodic in j and i,
   * Main/mpplib/mod_mppparam.F90:1063, 1132, 1224-1257); ichem = 1 (chemical tracers advected,
   * diffused and nudged by tend, Main/mod_tendency.F90:164, 198, 275, 548, 873). */
  int32_t i_band, i_crm, ichem;
} rcmdyn_config;

/* Field identifiers for put/get.  3-D fields have k = 1..kz unless noted. */
enum rcmdyn_field {
  /* prognostic state, coupled with p* exactly as the reference stores it */
  RCMDYN_ATM1_U = 0, RCMDYN_ATM1_V, RCMDYN_ATM1_T, RCMDYN_ATM1_QV, RCMDYN_ATM1_QC,
  RCMDYN_ATM2_U, RCMDYN_ATM2_V, RCMDYN_ATM2_T, RCMDYN_ATM2_QV, RCMDYN_ATM2_QC,
  RCMDYN_PSA, RCMDYN_PSB,                 /* 2-D (k1=k2=1) */
  RCMDYN_DSTOR, RCMDYN_HSTOR,             /* 2-D x nsplit (k = 1..nsplit) */
  /* static fields, as left by param (Main/mod_params.F90:1982-2002): map factors
   * already inverted, ht already converted to geopotential */
  RCMDYN_MSFX, RCMDYN_MSFD, RCMDYN_CORIOL, RCMDYN_HT,
  /* lateral boundary data (v3dbound / v2dbound b0, bt) */
  RCMDYN_XUB_B0, RCMDYN_XUB_BT, RCMDYN_XVB_B0, RCMDYN_XVB_BT,
  RCMDYN_XTB_B0, RCMDYN_XTB_BT, RCMDYN_XQB_B0, RCMDYN_XQB_BT,
  RCMDYN_XPSB_B0, RCMDYN_XPSB_BT,
  /* read-only diagnostics of the last tend */
  RCMDYN_PSC, RCMDYN_PTEN, RCMDYN_PSDOTA,
  RCMDYN_TTEN, RCMDYN_UTEN, RCMDYN_VTEN, RCMDYN_QVTEN, RCMDYN_QCTEN,
  RCMDYN_OMEGA, RCMDYN_QDOT /* k = 1..kz+1 */, RCMDYN_XKC, RCMDYN_PHI,
  /* non-hydrostatic state (coupled with p* like t): pressure perturbation (Pa), vertical
   * velocity on full levels (k = 1..kz+1), their boundary data */
  RCMDYN_ATM1_PP, RCMDYN_ATM2_PP, RCMDYN_ATM1_W, RCMDYN_ATM2_W,
  RCMDYN_XPPB_B0, RCMDYN_XPPB_BT, RCMDYN_XWWB_B0, RCMDYN_XWWB_BT,
  /* non-hydrostatic reference state and statics, as make_reference_atmosphere and
   * compute_full_coriolis_coefficients leave them (Main/mod_params.F90:2614-2741):
   * atm0 ps (2-D, p* in Pa), pr, t, rho, z (half levels), pf, rhof, zf (full levels, kz+1),
   * dpsdxm, dpsdym (2-D), dprddx, dprddy (dot, kz), ef, ddx, ddy, dmdx, dmdy (dot, 2-D),
   * ex, crx, cry (cross, 2-D) */
  RCMDYN_ATM0_PS, RCMDYN_ATM0_PR, RCMDYN_ATM0_T, RCMDYN_ATM0_RHO, RCMDYN_ATM0_Z,
  RCMDYN_ATM0_PF, RCMDYN_ATM0_RHOF, RCMDYN_ATM0_ZF,
  RCMDYN_DPSDXM, RCMDYN_DPSDYM, RCMDYN_DPRDDX, RCMDYN_DPRDDY,
  RCMDYN_EF, RCMDYN_DDX, RCMDYN_DDY, RCMDYN_DMDX, RCMDYN_DMDY, RCMDYN_EX, RCMDYN_CRX, RCMDYN_CRY,
  /* physics coupling (put): the pc_physic component of aten that the
   * host's physical_parametrizations produced (coupled with p*, like aten), added in tend's
   * sums exactly where the reference adds them (Main/mod_tendency.F90:285-314, 332-341,
   * 404-411).  Cross points for t, qv, qc, pp, w (w on kz+1 levels), dot points for u, v.
   * The engine holds no physics buffers until the first put of one of these; they then
   * persist (zero until put) and enter every later tend. */
  RCMDYN_TPHY, RCMDYN_QVPHY, RCMDYN_QCPHY, RCMDYN_UPHY, RCMDYN_VPHY, RCMDYN_PPPHY, RCMDYN_WPHY,
  /* atms slice fields (get, read-only) of mkslice, Main/mod_slice.F90:102-358, as the
   * physics reads them: filled by rcmdyn_tend_pre_physics from the state at the start of the
   * step; zero outside the index ranges the reference writes.  PF3D, WB3D, ZQ: kz+1 levels;
   * PS2D, RHOX2D: 2-D.  ZQ, ZA, DZQ only for idynamic = 1 (constant in the NH core). */
  RCMDYN_ATMS_UBX3D, RCMDYN_ATMS_VBX3D, RCMDYN_ATMS_UBD3D, RCMDYN_ATMS_VBD3D, RCMDYN_ATMS_TB3D,
  RCMDYN_ATMS_QVB3D, RCMDYN_ATMS_QCB3D, RCMDYN_ATMS_TV3D, RCMDYN_ATMS_PB3D, RCMDYN_ATMS_PF3D,
  RCMDYN_ATMS_PS2D, RCMDYN_ATMS_RHOX2D, RCMDYN_ATMS_TH3D, RCMDYN_ATMS_RHOB3D, RCMDYN_ATMS_TP3D,
  RCMDYN_ATMS_WPX3D, RCMDYN_ATMS_WB3D, RCMDYN_ATMS_ZQ, RCMDYN_ATMS_ZA, RCMDYN_ATMS_DZQ,
  RCMDYN_ATMS_QSB3D, RCMDYN_ATMS_RHB3D,
  /* device bdyin (put): the next ICBC record as read_icbc returns it
   * (Main/mod_bdycod.F90:469-480): u, v (m/s, dot), t (K), qv (kg/kg), ps (2-D, hPa; not read
   * for idynamic = 2), NH pp (Pa) and w (m/s, kz+1 levels), uncoupled; rcmdyn_bdyin converts
   * and couples it.  ATM0_PSDOT: atm0%psdot (2-D, Pa, dot points), the NH coupling factor of
   * u, v (:399). */
  RCMDYN_XUB_B1, RCMDYN_XVB_B1, RCMDYN_XTB_B1, RCMDYN_XQB_B1, RCMDYN_XPSB_B1, RCMDYN_XPPB_B1,
  RCMDYN_XWWB_B1, RCMDYN_ATM0_PSDOT,
  /* UW PBL turbulent kinetic energy (ibltyp = 2): atm1/atm2 tke, decoupled (m2/s2), kz+1
   * levels (Main/mod_atm_interface.F90), and the pc_physic tendency the UW scheme produces
   * (put, like the *PHY fields; added to the advective tendency, :530-531) */
  RCMDYN_ATM1_TKE, RCMDYN_ATM2_TKE, RCMDYN_TKEPHY,
  /* kpbl (put, ibltyp = 2): the PBL-top level index per cross point that the UW scheme sets
   * each step (Main/mod_atm_interface.F90:136, 1135: jci1:jci2 x ici1:ici2), as doubles
   * holding integers; read by the iuwvadv = 1 vertical flux.  A value above kz is refused
   * ('kpbl is greater than kz', Main/mod_advection.F90:923-925); below 4 the column keeps
   * the plain interpolated flux.  Zero until put. */
  RCMDYN_KPBL,
  /* ABI 6, nqx = 5 only (refused otherwise): the atm1/atm2 ice, rain and snow mixing ratios
   * qx(:,:,:,iqi|iqr|iqs), coupled with p* like qc; their pc_physic tendencies (put, like the
   * *PHY fields, :332-335); the mkslice export qxb3d(iqi|iqr|iqs) (get, like ATMS_QCB3D,
   * Main/mod_slice.F90:193-195) */
  RCMDYN_ATM1_QI, RCMDYN_ATM1_QR, RCMDYN_ATM1_QS, RCMDYN_ATM2_QI, RCMDYN_ATM2_QR, RCMDYN_ATM2_QS,
  RCMDYN_QIPHY, RCMDYN_QRPHY, RCMDYN_QSPHY,
  RCMDYN_ATMS_QXB3D_QI, RCMDYN_ATMS_QXB3D_QR, RCMDYN_ATMS_QXB3D_QS,
  RCMDYN_NFIELDS
};

typedef struct rcmdyn_engine rcmdyn_t;

/* Lifetime */
int rcmdyn_create(const rcmdyn_config* cfg, rcmdyn_t** out);
int rcmdyn_destroy(rcmdyn_t* h);
const char* rcmdyn_last_error(rcmdyn_t* h);    /* h may be NULL: last global error */

/* Decomposition (set_nproc, Main/mpplib/mod_mppparam.F90:1053-1371), host-only, no GPU:
 * fills cpus[2] = {cpus_j, cpus_i} for nproc ranks on a jx x iy grid. */
int rcmdyn_set_nproc(int32_t nproc, int32_t jx, int32_t iy, int32_t cpus[2]);
/* Tile extents in global indices: ext[8] = {jde1,jde2,ide1,ide2,jce1,jce2,ice1,ice2},
 * bdy[4] = {has_bdyleft, has_bdyright, has_bdybottom, has_bdytop}.  Host-only. */
int rcmdyn_tile_extent(int32_t jx, int32_t iy, int32_t nproc_j, int32_t nproc_i,
                       int32_t tile, int32_t ext[8], int32_t bdy[4]);
/* The same for the grid and decomposition of cfg (jx, iy, nproc_j, nproc_i), with the periodic
 * directions of i_band (j) and i_crm (i): a periodic direction has no boundary side and its
 * cross range takes every point (Main/mpplib/mod_mppparam.F90:1131-1132, 1340-1360), as the
 * engine's own tiles do.  rcmdyn_tile_extent is this call with i_band = i_crm = 0; a band or
 * CRM host picks its points with this one.  Returns non-zero for a tile or flag out of range,
 * and for i_crm = 1 without i_band = 1 (rcmdyn_create refuses that configuration).  Host-only. */
int rcmdyn_tile_extent_cfg(const rcmdyn_config* cfg, int32_t tile, int32_t ext[8], int32_t bdy[4]);

/* Communication plan of one rank, host-only (no GPU, no communicator): the halo messages and
 * collectives that rank cfg->comm_rank (one tile per rank: tile_first = comm_rank, tile_count
 * = 1, comm_size = nproc_j * nproc_i) issues for the first exchanges of the statics and the
 * boundary data, the initial bdyval after the state put (its slice exchange) and then nsteps x
 * (tend + bdyval), in issue order.  Record q is
 * ops[7q .. 7q+6] = {call, kind, channel, dir, peer, count, signature}: call = the rank's
 * communication call number; kind 1 = one grouped send/receive (one record per message), 2 =
 * all-reduce sum (f64), 3 = all-reduce max (i32), 4 = all-reduce max (f64); channel 0/1 = the
 * engine stream that issues it (over RCCL both share the job's communicator, the second
 * ordered after the first); dir 0 send, 1 receive, -1 collective; peer = rank
 * (-1 for collectives); count = doubles (collectives: elements); signature = hash of the
 * message's box shapes (0 for collectives).  *count = records in the plan (at most cap are
 * written).  Every message A sends B must be the receive B posts from A, in the same order on
 * the same channel, which a multi-rank job needs and tests check.  The plan models no put
 * between steps: a KPBL put (ibltyp = 2, iuwvadv = 1, hydrostatic) adds one width-1 exchange
 * of kpbl before the next tend, on every rank alike. */
int rcmdyn_exchange_plan(const rcmdyn_config* cfg, int32_t nsteps, int64_t* ops, int64_t cap, int64_t* count);
/* Halo/compute overlap of the hydrostatic step, host-only (no GPU): for each of the first cap
 * tiles this engine would own, out[6q .. 6q+5] = {k_columns points in the part-1 rectangle R,
 * k_columns points, k_momentum points of its part-1 blocks, k_momentum points, k_scalars points
 * of its part-1 blocks, k_scalars points}: the share of each kernel that runs beside the
 * prologue exchange (0 when the step does not overlap: one tile, NH, idiffu = 3). */
int rcmdyn_overlap_shares(const rcmdyn_config* cfg, int32_t* out, int32_t cap);

/* State transfer (host <-> device), Fortran layout, global index bounds. */
int rcmdyn_put(rcmdyn_t* h, int32_t field, const double* src,
               int32_t j1, int32_t j2, int32_t i1, int32_t i2, int32_t k1, int32_t k2);
int rcmdyn_get(rcmdyn_t* h, int32_t field, double* dst,
               int32_t j1, int32_t j2, int32_t i1, int32_t i2, int32_t k1, int32_t k2);
/* Step failures (CFL VIOLATION, SLADVECTION) are detected on the device.  rcmdyn_step and
 * rcmdyn_tend report a failed step at most 2 steps late (one-rank jobs) or one reduction
 * interval (8 steps) late (RCCL jobs), so they never wait for the stream per step;
 * rcmdyn_get and rcmdyn_diagnostics wait for the stream and report any failure of the steps
 * issued so far before copying anything (with RCCL: the job-wide words already reduced and
 * this rank's own flags; no collective is issued, so a rank may call them alone). */

/* rcm_timer state: lcount (steps done), dt (current leapfrog dt, s), xbctime (s since
 * the current boundary interval started). */
int rcmdyn_set_time(rcmdyn_t* h, int64_t lcount, double dt, double xbctime);
int rcmdyn_get_time(rcmdyn_t* h, int64_t* lcount, double* dt, double* xbctime);

/* The hot path. */
int rcmdyn_tend(rcmdyn_t* h);                  /* one mod_tendency::tend */
/* tend split at the reference's call of physical_parametrizations (Main/mod_tendency.F90:
 * 271): pre_physics runs surface_pressures, decouple, compute_omega, mkslice (device export
 * of the ATMS_* fields) and new_pressure; the host then runs its physics on the ATMS_*
 * fields, puts the *PHY tendencies, and post_physics runs the rest of tend.  pre + post is
 * bit-identical to rcmdyn_tend with the same *PHY contents. */
int rcmdyn_tend_pre_physics(rcmdyn_t* h);
int rcmdyn_tend_post_physics(rcmdyn_t* h);
int rcmdyn_bdyval(rcmdyn_t* h);                /* one mod_bdycod::bdyval */
/* mod_bdycod::bdyin from read_icbc on (Main/mod_bdycod.F90:654-889), on the device:
 * b0 <- b1; the record put into the XxB_B1 fields becomes the new b1 (p* = ps/10 - ptop,
 * exchange, psc2psd, couple u, v with p* on dot points and t, qv (pp, w) with p*, exchange);
 * bt = (b1 - b0)/dtbdys on the ga ranges (timeint); xbctime = 0.  The reference's init_bdy
 * (:280-650) reads b0 and b1: call rcmdyn_bdyin twice, with the record at the start and the
 * one dtbdys later. */
int rcmdyn_bdyin(rcmdyn_t* h);
int rcmdyn_step(rcmdyn_t* h, int32_t nsteps);  /* nsteps x (tend + bdyval), graph-replayed */
/* Waits for the device and reports a failure of any step issued so far.  In RCCL mode it is
 * COLLECTIVE (it max-reduces the step error flags over the job so that every rank stops at
 * the same call): every rank must call it, as every rank calls rcmdyn_step and
 * rcmdyn_reductions.  In RCCL mode a step failure (CFL / NaN / departure point) this rank's
 * own flags hold is sticky at the host read points (get, diagnostics): it is reported there
 * before the job-wide reduction carries it, and again at every later read, until
 * rcmdyn_set_time (the host's restart from a SAV state) clears the flags.  The reference's
 * fatal ends the job there (Main/abort.F90:20-36), as a host should. */
int rcmdyn_synchronize(rcmdyn_t* h);

/* Diagnostics of the last tend: out[0]=ptntot, out[1]=pt2tot (Bleck noise sums of the
 * owned tiles, Main/mod_tendency.F90:1449-1459), out[2]=1 if ptntot is NaN. */
int rcmdyn_diagnostics(rcmdyn_t* h, double out[4]);

/* The 3-hourly report of tend and sound (syncro_rep, Main/mod_tendency.F90:705-725,
 * Main/mod_sound.F90:634-646), reduced over every tile of the job (sumall / maxall: the
 * engine's own tiles, then RCCL across ranks; collective in RCCL mode -- every rank calls
 * it): out[0] = sum of |pten| (ptntot), out[1] = sum of the 2nd time derivative of p*
 * (pt2tot) over the interior points of the last step (the host multiplies both by its
 * rptn = 1/npoints, :715-716); out[2] = NH: the maximum sigma-velocity CFL of the last
 * acoustic sub-step (maxall(cfl), :637), 0 for the hydrostatic core. */
int rcmdyn_reductions(rcmdyn_t* h, double out[3]);

/* Which runtime libraries the engine's calls are bound to: "hip=<path>; rccl=<path>
 * (<version>)" into buf (NUL-terminated, at most len bytes).  In a PyTorch process the
 * already-loaded libamdhip64.so.7 / librccl.so.1 (torch's copies, same sonames) are the
 * ones bound when torch was imported first; otherwise ROCm's (/opt/rocm/lib). */
int rcmdyn_runtime_info(char* buf, int32_t len);

/* Multi-process: rank 0 creates the id, the host broadcasts it (MPI / torch.distributed),
 * every rank passes it in rcmdyn_config.comm_unique_id. */
int rcmdyn_comm_unique_id(uint8_t out[128]);

/* Wall-clock of device work: average ms per step of the last rcmdyn_step call measured
 * with HIP events on the engine's compute stream. */
int rcmdyn_last_step_ms(rcmdyn_t* h, double* ms);

/* Tendency diagnostics (TTEN..QCTEN, OMEGA, XKC of rcmdyn_field): off by default.  When on,
 * every tend also stores the per-point tendencies the reference accumulates in aten
 * (Main/mod_tendency.F90:259-400) for rcmdyn_get; when off those gets fail.  The prognostic
 * results are identical either way. */
int rcmdyn_set_diagnostics(rcmdyn_t* h, int32_t on);

/* Per-kernel device time (measurement hook, mirrors rocprofv3 --kernel-trace --stats):
 * runs nsteps steps (tend + bdyval, eagerly, no graph) with a HIP event pair around every
 * kernel launch on the engine's stream.  For each distinct kernel (at most cap) fills
 * names[q*48 .. q*48+47] (NUL-terminated), launches[q] and avg_ms[q] (mean duration per
 * launch); *count = kernels found.  The steps advance the model like rcmdyn_step. */
int rcmdyn_kernel_times(rcmdyn_t* h, int32_t nsteps, int32_t cap, char* names, int32_t* launches,
                        double* avg_ms, int32_t* count);

#ifdef __cplusplus
}
#endif
#endif /* RCMDYN_H */
