/*
 * rcm_oracle.c -- TEST INFRASTRUCTURE ONLY (see rcm_oracle.h).
 *
 * Plain-C restatement of the RegCM 4.7 hydrostatic dynamical-core step, written loop
 * nest by loop nest after the reference so that every floating-point expression is
 * evaluated in the reference's order (Fortran left-to-right, no reassociation, no FMA:
 * compile with -ffp-contract=off).  Each routine cites the reference file:line it
 * restates.  Physics is stubbed exactly as BASELINE configuration C2/C3 ("physics
 * stubbed"): every *phy tendency is zero (Main/mod_tendency.F90:1682-1820 with no-op
 * cumulus/microscheme/radiation/pbl and heatrt = 0).
 *
 * Scope (defaults assumed): idynamic=1, upstream_mode and
 * stability_enhance on, idiffu=1, iboudy=5 (or 1), ipgf=0, nsplit from config,
 * nqx = 2 (qv, qc) or 5 (qv, qc, qi, qr, qs: ipptls >= 2, Main/mod_params.F90:1358-1366),
 * isladvec=0/1, ibltyp=1/2 (iuwvadv 0/1), ichem=0, idiag=0, iboudy time-dependent.
 *
 * Parity unpinned: no execution of the reference is available (netCDF-Fortran absent),
 * no golden vectors exist in the reference tree.
 */
#include "rcm_oracle.h"
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

/* ---- constants: Share/mod_constants.F90 (evaluated exactly as written) ---- */
static const double d_zero = 0.0, d_one = 1.0, d_two = 2.0, d_four = 4.0;
static const double d_half = 0.5, d_rfour = 0.25, d_1000 = 1000.0;
#define EGRAV   9.80665                      /* :85  */
#define BOLTZK  1.3806504e-23                /* :92  */
#define NAVGDR  6.02214129e23                /* :94  */
#define AMD     28.96454                     /* :107 */
#define AMW     18.01528                     /* :109 */
#define MINQQ   1.0e-8                       /* :57  */
#define DLOWVAL 1.0e-20                      /* :68  */
#define VONKAR  0.4                          /* :296 */
static double c_rgas, c_cpd, c_c287, c_ep1, c_regrav, c_rovcp;
static const double alpha_hyd = 0.0;         /* :319 */
static const double beta_hyd = 1.0 - 2.0 * 0.0; /* :320 */
/* mod_diffusion.F90:69-71 */
static const double z4_c1 = 1.0, z4_c2 = -4.0, z4_c3 = 12.0;
/* second-order (9-point) scheme of idiffu = 2, Main/mod_diffusion.F90:63-65 */
static const double o4_c1 = 4.0 / 6.0, o4_c2 = 1.0 / 6.0, o4_c3 = -20.0 / 6.0;
/* sixth-order flux-limited scheme of idiffu = 3, Main/mod_diffusion.F90:75-78 */
static const double h4_c1 = 10.0, h4_c2 = -5.0, h4_c3 = 1.0, diff_6th_factor = 0.12;

/* reference-atmosphere constants of the ipgf = 1 pressure gradient, Share/mod_constants.F90:359-362 */
static const double T00PG = 287.0, P00PG = 101.325, ALAM = 6.5e-3;
static double c_pgfaa1;

static void init_constants(void) {
  double rgasmol = NAVGDR * BOLTZK;          /* :130 */
  c_c287 = rgasmol / AMD;                    /* :132 */
  c_rgas = c_c287 * 1000.0;                  /* :134 */
  c_cpd = 3.5 * c_rgas;                      /* :144 */
  c_ep1 = AMD / AMW - d_one;                 /* :303 */
  c_regrav = d_one / EGRAV;                  /* :182 */
  c_rovcp = c_rgas * (d_one / c_cpd);        /* :183-184, rovcp = rgas*rcpd */
  c_pgfaa1 = ALAM * c_rgas * c_regrav;       /* :362 */
}

#define NQ 5   /* moisture species at most: qv, qc, qi, qr, qs (iqv = 0 .. iqs = 4 here) */
#define GO 4   /* frame ghost width (covers ga/gb/gc halos and the isladvec = 1 exchange, 4 wide) */

struct orc {
  rcmdyn_config cfg;
  int jx, iy, kz, kzp1, nsplit, nqx;
  /* tile index ranges (global, Fortran), Main/mod_atm_interface.F90:181-381 */
  int jde1, jde2, jdi1, jdi2, jdii1, jdii2, ide1, ide2, idi1, idi2, idii1, idii2;
  int jce1, jce2, jci1, jci2, jcii1, jcii2, ice1, ice2, ici1, ici2, icii1, icii2;
  int jde1ga, jde2ga, ide1ga, ide2ga, jce1ga, jce2ga, ice1ga, ice2ga;
  int jci1ga, jci2ga, ici1ga, ici2ga;
  int jde1gb, jde2gb, ide1gb, ide2gb, jce1gb, jce2gb, ice1gb, ice2gb;
  int bl, br, bb, bt;                       /* has_bdyleft/right/bottom/top */
  /* frame */
  int j0, i0, nj, ni;
  size_t plane;
  /* time */
  long long lcount;
  double dt, dtsec, xbctime;
  /* derived constants */
  double dx, dx2, dx4, dx8, dx16, dxsq, rdxsq, ptop;
  double ul, xkhmax, dydc, xkhz, fnudge, gnudge;
  double sigma[RCMDYN_MAXKZ + 2], hsigma[RCMDYN_MAXKZ + 1], dsigma[RCMDYN_MAXKZ + 1];
  double twt1[RCMDYN_MAXKZ + 1], twt2[RCMDYN_MAXKZ + 1], qcon[RCMDYN_MAXKZ + 1];
  double xds[RCMDYN_MAXKZ + 1], dds[RCMDYN_MAXKZ + 2];
  double hefc[256][RCMDYN_MAXKZ + 1], hegc[256][RCMDYN_MAXKZ + 1]; /* (n,k), n=2..nspgx-1 */
  double fcx[256], gcx[256];
  double wgtx[256], wgtd[256];              /* sponge weights (iboudy = 4), :238-250 */
  double pdlog[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ + 2], eps1[RCMDYN_MAXSPLIT][RCMDYN_MAXKZ + 2];
  /* boundary masks: 0 none, 1 S, 2 N, 3 W, 4 E; ibnd */
  signed char *rg_cr, *rg_dt;
  int *ib_cr, *ib_dt;
  /* state */
  double *a1u, *a1v, *a1t, *a1q[NQ], *a2u, *a2v, *a2t, *a2q[NQ];
  double *psa, *psb, *psc, *psdota, *psdotb, *dstor, *hstor;
  double *msfx, *msfd, *xmsf, *dmsf, *coriol, *ht, *hgfact, *map;
  double *ub0, *ubt, *vb0, *vbt, *tb0, *tbt, *qb0, *qbt, *pb0, *pbt;
  /* work */
  double *rpsa, *rpsb, *rpsc, *rpsda, *srpsb, *rpsdotb;
  double *uc, *vc, *umc, *vmc, *ud, *vd, *xt, *xq[NQ], *xtv;
  double *qcd;                              /* nqx = 5: the total water load (decouple :1107-1115) */
  double *cr, *pten, *qdot, *omega, *dummy;
  double *ubd, *vbd, *tb3d, *qb3d[NQ], *pb3d, *pf3d;
  double *xkc, *xkd;
  double *tten, *tdyn, *uten, *udyn, *vten, *vdyn, *qten[NQ], *qdyn[NQ];
  double *fg, *uavg1, *uavg2, *vavg1, *vavg2, *dotqdot;
  double *fg1, *fg2;
  double *ct, *cq[NQ], *cu, *cv;
  double *td, *tvfac, *phi;
  double *deld, *delh, *ddsum, *dhsum, *xdelh, *work, *uu, *vv, *uuu, *vvv;
  /* boundary slices (Main/mod_bdycod.F90:58-61): indexed by frame j or i, then k */
  double *wue, *wui, *eue, *eui, *wve, *wvi, *eve, *evi;
  double *sue, *sui, *nue, *nui, *sve, *svi, *nve, *nvi;
  /* non-hydrostatic core (idynamic = 2) */
  int nh;
  double *a1pp, *a2pp, *a1w, *a2w, *ppb0, *ppbt, *wwb0, *wwbt;
  double *ps0, *pr0, *t0, *rho0, *z0, *pf0, *rhof0, *zf0, *dpsdxm, *dpsdym, *dprddx, *dprddy;
  double *ef, *ddx, *ddy, *dmdx, *dmdy, *ex, *crx, *cry;
  double *umd, *vmd, *xpp, *xw, *pr1, *rho1, *xpr, *ucc, *vcc, *ppb3d, *wb3d, *xkcf;
  double *th, *tha, *thten;                 /* potential temperature advection, ithadv = 1 */
  double *ppten, *ppdyn, *wten, *wdyn, *cpp, *cw, *cdt;
  double *s_wo, *s_e, *s_f, *s_aa, *s_b, *s_c, *s_rhs, *s_ca, *s_g1, *s_g2, *s_ptend, *s_pxup,
         *s_pyvp, *s_tk, *s_cc, *s_cdd, *s_cj, *s_pi, *s_ucrs, *s_vcrs;
  double *estore, *astore, *wpval;
  double tmask[13][13];                     /* tmask(nsj, nsi), nsj/nsi = -6..6 */
  int tmask_valid, nh_istep;
  double nh_cfl;
  /* physics coupling seam: pc_physic tendencies t, qv, qc, u, v, pp, w and the atms export
   * (rcmdyn_field TPHY.. and ATMS_UBX3D.. order) */
  double *phy[7], *atms[22];
  double *phyx[3], *atmsx[3];               /* nqx = 5: qi, qr, qs pc_physic tendencies, qxb3d export */
  /* UW PBL TKE (ibltyp = 2): atm1/atm2 tke, atmc%tke, tkedyn, tkeps, the pc_physic tendency */
  double *a1tke, *a2tke, *ctke, *tkedyn, *tkeps, *tkephy;
  double* kpbl;      /* ibltyp = 2: the UW scheme's PBL-top level (put; iuwvadv = 1 reads it) */
  int sound_probe;   /* test hook (orc_set_sound_probe): sound returns after this many sub-steps */
  int tend_probe;    /* test hook (orc_set_tend_probe): the hydrostatic tend returns at this stage */
  /* bdyin: raw record (u, v, t, qv, ps, pp, w), coupled b1 (same order), NH atm0%psdot */
  double *bin[7], *bb1[7], *psdot0;
  double rhmin, rhmax;
  /* diagnostics */
  double ptntot, pt2tot;
  /* exchange */
  orc_exchange_fn xfn;
  orc_exchange_bdy_fn bfn;
  orc_gather_fn gfn;
  void* xctx;
  double* s_tr;                             /* gather scratch of the day-alarm rho*N terms */
};

/* ---- indexing: frame [k][i][j], global Fortran indices ---- */
#define IX(j, i) ((size_t)((i) - o->i0) * (size_t)o->nj + (size_t)((j) - o->j0))
#define A2(a, j, i) (a)[IX(j, i)]
#define A3(a, j, i, k) (a)[((size_t)(k) - 1) * o->plane + IX(j, i)]
#define SJ(s, j, k) (s)[((size_t)(k) - 1) * (size_t)o->nj + (size_t)((j) - o->j0)]
#define SI(s, i, k) (s)[((size_t)(k) - 1) * (size_t)o->ni + (size_t)((i) - o->i0)]
#define DELD(j, i, n, s) o->deld[(((size_t)(s) - 1) * o->nsplit + ((n) - 1)) * o->plane + IX(j, i)]
#define DELH(j, i, n, s) o->delh[(((size_t)(s) - 1) * o->nsplit + ((n) - 1)) * o->plane + IX(j, i)]

static double* alloc3(orc_t* o, int nk) {
  return (double*)calloc((size_t)nk * o->plane, sizeof(double));
}
static double dmax(double a, double b) { return (a > b) ? a : (b > a ? b : a); }
static double dmin(double a, double b) { return (a < b) ? a : (b < a ? b : a); }

/* A band (i_band = 1) on one tile in j is its own west and east neighbour
 * (Main/mpplib/mod_mppparam.F90:1112-1114: ma%left = ma%right = myid): the exchange's band
 * branch (:6092-6140) copies the nex columns on each side around the period, rows ide1..ide2
 * (the box every exchange here moves); exchange_lb fills the left ghost columns only, _rt the
 * right ones. */
static void band_self_xch(orc_t* o, double* a, int nk, int nex, int sides) {
  const int jx = o->jx;
  for (int k = 1; k <= nk; k++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int w = 1; w <= nex; w++) {
        if (sides != 2) A3(a, o->jde1 - w, i, k) = A3(a, o->jde1 - w + jx, i, k);
        if (sides != 1) A3(a, o->jde2 + w, i, k) = A3(a, o->jde2 + w - jx, i, k);
      }
}
/* CRM (i_crm = 1, with the band) on one tile in i is its own south and north neighbour
 * (Main/mpplib/mod_mppparam.F90:1104-1108, 1132): the rows past either end of the period,
 * every column of the frame the j pass filled (so the corners wrap in both directions) */
static void crm_self_xch(orc_t* o, double* a, int nk, int nex, int sides) {
  const int iy = o->iy;
  const int j1 = o->cfg.nproc_j == 1 ? o->jde1 - nex : o->jde1, j2 = o->cfg.nproc_j == 1 ? o->jde2 + nex : o->jde2;
  for (int k = 1; k <= nk; k++)
    for (int w = 1; w <= nex; w++)
      for (int j = j1; j <= j2; j++) {
        if (sides != 2) A3(a, j, o->ide1 - w, k) = A3(a, j, o->ide1 - w + iy, k);
        if (sides != 1) A3(a, j, o->ide2 + w, k) = A3(a, j, o->ide2 + w - iy, k);
      }
}
static void xch(orc_t* o, double* a, int nk, int nex, int sides) {
  if (o->xfn) { o->xfn(o->xctx, a, nk, nex, sides); return; }
  if (o->cfg.i_band && o->cfg.nproc_j == 1) band_self_xch(o, a, nk, nex, sides);
  if (o->cfg.i_crm && o->cfg.nproc_i == 1) crm_self_xch(o, a, nk, nex, sides);
}
/* the boundary slices along j (south / north) exchange their entries one past the tile with
 * the left / right tiles (exchange_bdy_lr, Main/mod_bdycod.F90:1063-1089): around the period
 * on a band's single tile */
static void xchb(orc_t* o, double* s, int along) {
  if (o->bfn) o->bfn(o->xctx, s, o->kz, along);
  else if (o->cfg.i_band && o->cfg.nproc_j == 1 && along == 0)
    for (int k = 0; k < o->kz; k++) {
      double* r = s + (size_t)k * o->nj - o->j0;          /* r[j]: entry of column j */
      r[o->jde1 - 1] = r[o->jde2];
      r[o->jde2 + 1] = r[o->jde1];
    }
}

/* ---- set_nproc tile extents, Main/mpplib/mod_mppparam.F90:1295-1360 ---- */
static void tile_extent(int jx, int iy, int cj, int ci, int tile, int ext[8], int bdy[4], int band, int crm) {
  int lj = tile / ci, li = tile % ci;
  int jxp = jx / cj, iyp = iy / ci;
  int js = lj * jxp + 1, is = li * iyp + 1;
  if (jxp * cj < jx) {
    int imiss = jx - jxp * cj;
    if (lj < imiss) { js += lj; jxp += 1; } else { js += imiss; }
  }
  if (iyp * ci < iy) {
    int imiss = iy - iyp * ci;
    if (li < imiss) { is += li; iyp += 1; } else { is += imiss; }
  }
  int je = js + jxp - 1, ie = is + iyp - 1;
  ext[0] = js; ext[1] = je; ext[2] = is; ext[3] = ie;
  /* a band (i_band = 1) is periodic in j: no west/east boundary, and the cross grid takes every
   * j (global_cross_jend = global_dot_jend, Main/mpplib/mod_mppparam.F90:1351-1354) */
  ext[4] = js; ext[5] = (je == jx && !band) ? je - 1 : je;
  /* CRM (i_crm = 1): the same in i (dim_period(2), global_cross_iend = global_dot_iend, :1340-1342) */
  ext[6] = is; ext[7] = (ie == iy && !crm) ? ie - 1 : ie;
  bdy[0] = (lj == 0) && !band; bdy[1] = (lj == cj - 1) && !band;
  bdy[2] = (li == 0) && !crm; bdy[3] = (li == ci - 1) && !crm;
}

/* ---- setup_boundaries, Main/mod_atm_interface.F90:383-542 ---- */
static void setup_boundaries(orc_t* o, int ldot, signed char* rg, int* ib) {
  int jx = o->jx, iy = o->iy;
  int icx = ldot ? 0 : 1, icy = ldot ? 0 : 1;
  int nsp = ldot ? o->cfg.nspgd : o->cfg.nspgx;
  int igbb1 = 2, igbb2 = nsp - 1, jgbl1 = 2, jgbl2 = nsp - 1;
  int igbt1 = iy - icy - nsp + 2, igbt2 = iy - icy - 1;
  int jgbr1 = jx - icx - nsp + 2, jgbr2 = jx - icx - 1;
  for (int i = o->i0; i < o->i0 + o->ni; i++)
    for (int j = o->j0; j < o->j0 + o->nj; j++) { A2(rg, j, i) = 0; A2(ib, j, i) = -1; }
  if (o->cfg.i_crm) return;      /* CRM: no relaxation band at all (:434, "if (.not. ma%crmflag)") */
  if (o->cfg.i_band) {
    /* a band (:435-455): the south and north rows only, every j ("j < jgbl1 .and. j > jgbr2"
     * skips none) */
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        if (i >= igbb1 && i <= igbb2) { A2(ib, j, i) = i - igbb1 + 2; A2(rg, j, i) = 1; }
        if (i >= igbt1 && i <= igbt2) { A2(ib, j, i) = igbt2 - i + 2; A2(rg, j, i) = 2; }
      }
    return;
  }
  for (int i = o->ide1; i <= o->ide2; i++) {   /* South */
    if (i >= igbb1 && i <= igbb2)
      for (int j = o->jde1; j <= o->jde2; j++)
        if (j >= jgbl1 && j <= jgbr2) {
          if (j <= jgbl2 && i >= j) continue;
          if (j >= jgbr1 && i >= (jgbr2 - j + 2)) continue;
          A2(ib, j, i) = i - igbb1 + 2; A2(rg, j, i) = 1;
        }
  }
  for (int i = o->ide1; i <= o->ide2; i++) {   /* North */
    if (i >= igbt1 && i <= igbt2)
      for (int j = o->jde1; j <= o->jde2; j++)
        if (j >= jgbl1 && j <= jgbr2) {
          if (j <= jgbl2 && (igbt2 - i + 2) >= j) continue;
          if (j >= jgbr1 && (igbt2 - i) >= (jgbr2 - j)) continue;
          A2(ib, j, i) = igbt2 - i + 2; A2(rg, j, i) = 2;
        }
  }
  for (int i = o->ide1; i <= o->ide2; i++) {   /* West */
    if (i < igbb1 || i > igbt2) continue;
    for (int j = o->jde1; j <= o->jde2; j++)
      if (j >= jgbl1 && j <= jgbl2) {
        if (i < igbb2 && j > i) continue;
        if (i > igbt1 && j > (igbt2 - i + 2)) continue;
        A2(ib, j, i) = j - jgbl1 + 2; A2(rg, j, i) = 3;
      }
  }
  for (int i = o->ide1; i <= o->ide2; i++) {   /* East */
    if (i < igbb1 || i > igbt2) continue;
    for (int j = o->jde1; j <= o->jde2; j++)
      if (j >= jgbr1 && j <= jgbr2) {
        if (i < igbb2 && (jgbr2 - j + 2) > i) continue;
        if (i > igbt1 && (jgbr2 - j) > (igbt2 - i)) continue;
        A2(ib, j, i) = jgbr2 - j + 2; A2(rg, j, i) = 4;
      }
  }
}

static int atms_levels(int q, int kz) {
  int f = RCMDYN_ATMS_UBX3D + q;
  if (f == RCMDYN_ATMS_PF3D || f == RCMDYN_ATMS_WB3D || f == RCMDYN_ATMS_ZQ) return kz + 1;
  if (f == RCMDYN_ATMS_PS2D || f == RCMDYN_ATMS_RHOX2D) return 1;
  return kz;
}

orc_t* orc_create(const rcmdyn_config* cfg) {
  init_constants();
  if (cfg->tile_count != 1 || cfg->kz > RCMDYN_MAXKZ || cfg->nsplit > RCMDYN_MAXSPLIT)
    return NULL;
  /* a non-hydrostatic tile of a decomposition needs the whole-domain gather of sound's upper
   * radiative condition (Main/mod_sound.F90:496-497): orc_set_gather, before the first step */
  if (cfg->idynamic != 1 && cfg->idynamic != 2) return NULL;
  /* nqx from ipptls >= 1 (Main/mod_params.F90:1358-1366); a band (i_band = 1) for both cores;
   * CRM (i_crm = 1: periodic in i too, PreProc/CRM/crm_test.in) for the non-hydrostatic core
   * over the band, with iboudy = 0 (fixed lateral values: no boundary line exists) or any
   * other iboudy (none relaxes anything); chemistry not restated.  iboudy = 0 without CRM (the
   * b0-only branches of bdyval) is not restated either. */
  if (cfg->ipptls < 1 || cfg->nqx != (cfg->ipptls > 1 ? 5 : 2) || cfg->ichem) return NULL;
  if (cfg->i_band != 0 && cfg->i_band != 1) return NULL;
  if (cfg->i_crm && (cfg->i_crm != 1 || !cfg->i_band || cfg->idynamic != 2)) return NULL;
  if (cfg->iboudy == 0 && !cfg->i_crm) return NULL;
  orc_t* o = (orc_t*)calloc(1, sizeof(orc_t));
  o->sound_probe = -1;
  o->cfg = *cfg;
  o->jx = cfg->jx; o->iy = cfg->iy; o->kz = cfg->kz; o->kzp1 = cfg->kz + 1;
  o->nsplit = cfg->nsplit; o->nqx = cfg->nqx;
  int ext[8], bdy[4];
  tile_extent(o->jx, o->iy, cfg->nproc_j, cfg->nproc_i, cfg->tile_first, ext, bdy, cfg->i_band, cfg->i_crm);
  o->bl = bdy[0]; o->br = bdy[1]; o->bb = bdy[2]; o->bt = bdy[3];
  /* Main/mod_atm_interface.F90:231-302 */
  o->jde1 = o->jdi1 = o->jdii1 = ext[0]; o->jde2 = o->jdi2 = o->jdii2 = ext[1];
  o->ide1 = o->idi1 = o->idii1 = ext[2]; o->ide2 = o->idi2 = o->idii2 = ext[3];
  if (o->bl) { o->jdi1 = o->jde1 + 1; o->jdii1 = o->jde1 + 2; }
  if (o->br) { o->jdi2 = o->jde2 - 1; o->jdii2 = o->jde2 - 2; }
  if (o->bb) { o->idi1 = o->ide1 + 1; o->idii1 = o->ide1 + 2; }
  if (o->bt) { o->idi2 = o->ide2 - 1; o->idii2 = o->ide2 - 2; }
  o->jce1 = o->jci1 = o->jcii1 = ext[4]; o->jce2 = o->jci2 = o->jcii2 = ext[5];
  o->ice1 = o->ici1 = o->icii1 = ext[6]; o->ice2 = o->ici2 = o->icii2 = ext[7];
  if (o->bl) { o->jci1 = o->jce1 + 1; o->jcii1 = o->jce1 + 2; }
  if (o->br) { o->jci2 = o->jce2 - 1; o->jcii2 = o->jce2 - 2; }
  if (o->bb) { o->ici1 = o->ice1 + 1; o->icii1 = o->ice1 + 2; }
  if (o->bt) { o->ici2 = o->ice2 - 1; o->icii2 = o->ice2 - 2; }
  int gl = o->bl ? 0 : 1, gr = o->br ? 0 : 1, gbm = o->bb ? 0 : 1, gt = o->bt ? 0 : 1;
  o->jde1ga = o->jde1 - gl; o->jde2ga = o->jde2 + gr; o->ide1ga = o->ide1 - gbm; o->ide2ga = o->ide2 + gt;
  o->jce1ga = o->jce1 - gl; o->jce2ga = o->jce2 + gr; o->ice1ga = o->ice1 - gbm; o->ice2ga = o->ice2 + gt;
  o->jci1ga = o->jci1 - gl; o->jci2ga = o->jci2 + gr; o->ici1ga = o->ici1 - gbm; o->ici2ga = o->ici2 + gt;
  /* the slice frames: gb (2 deep), gc (3 deep) with idiffu = 3 (Main/mod_atm_interface.F90:1001-1028) */
  const int gs = cfg->idiffu == 3 ? 3 : 2;
  o->jde1gb = o->jde1 - gs * gl; o->jde2gb = o->jde2 + gs * gr; o->ide1gb = o->ide1 - gs * gbm; o->ide2gb = o->ide2 + gs * gt;
  o->jce1gb = o->jce1 - gs * gl; o->jce2gb = o->jce2 + gs * gr; o->ice1gb = o->ice1 - gs * gbm; o->ice2gb = o->ice2 + gs * gt;
  o->j0 = o->jde1 - GO; o->i0 = o->ide1 - GO;
  o->nj = (o->jde2 - o->jde1 + 1) + 2 * GO; o->ni = (o->ide2 - o->ide1 + 1) + 2 * GO;
  o->plane = (size_t)o->nj * (size_t)o->ni;

  /* derived run constants, Main/mod_params.F90:1628-1770, 2006-2011, 2208-2215 */
  o->dtsec = cfg->dtsec; o->dt = cfg->dtsec; o->lcount = 0; o->xbctime = 0.0;
  o->ptop = cfg->ptop;
  o->dx = cfg->ds * d_1000; o->dx2 = d_two * o->dx; o->dx4 = d_four * o->dx;
  o->dx8 = 8.0 * o->dx; o->dx16 = 16.0 * o->dx; o->dxsq = o->dx * o->dx;
  o->rdxsq = 1.0 / o->dxsq;
  int kz = o->kz;
  for (int k = 1; k <= kz + 1; k++) o->sigma[k] = cfg->sigma[k - 1];
  for (int k = 1; k <= kz; k++) {
    o->hsigma[k] = (o->sigma[k + 1] + o->sigma[k]) * d_half;
    o->dsigma[k] = (o->sigma[k + 1] - o->sigma[k]);
  }
  o->twt1[1] = 0; o->twt2[1] = 0; o->qcon[1] = 0;
  for (int k = 2; k <= kz; k++) {
    o->twt1[k] = (o->sigma[k] - o->hsigma[k - 1]) / (o->hsigma[k] - o->hsigma[k - 1]);
    o->twt2[k] = d_one - o->twt1[k];
    o->qcon[k] = (o->sigma[k] - o->hsigma[k]) / (o->hsigma[k - 1] - o->hsigma[k]);
  }
  /* init_advection, Main/mod_advection.F90:100-106 (dt == dtsec at init: quirk kept) */
  for (int k = 1; k <= kz; k++) o->xds[k] = d_one / o->dsigma[k];
  o->dds[1] = 0; o->dds[kz + 1] = 0;
  for (int k = 2; k <= kz; k++) o->dds[k] = d_one / (o->dsigma[k] + o->dsigma[k - 1]);
  o->ul = cfg->uoffc * d_half * o->dt / o->dx;
  /* initialize_diffusion, Main/mod_diffusion.F90:104-107 (idynamic = 1) */
  o->xkhmax = o->dxsq / (64.0 * o->dtsec);
  o->dydc = cfg->adyndif * VONKAR * VONKAR * o->dx * d_rfour;
  o->xkhz = cfg->ckh * 1.5e-3 * o->dxsq / o->dtsec;
  o->nh = (cfg->idynamic == 2);
  if (o->nh) {                                /* :108-113 (Xu et al. 2001) */
    o->xkhz = cfg->ckh * o->dx;
    o->xkhmax = d_two * o->xkhmax;
  }
  /* setup_bdycon, Main/mod_bdycod.F90:203-274 */
  o->fnudge = (cfg->bdy_nm > 0) ? cfg->bdy_nm : 0.1 / o->dt;
  o->gnudge = (cfg->bdy_dm > 0) ? cfg->bdy_dm : d_one / (o->dt * 50.0);
  for (int n = 2; n <= cfg->nspgx - 1 && n < 256; n++) {
    double xfun = (double)(cfg->nspgx - n) / (double)(cfg->nspgx - 2);
    o->fcx[n] = o->fnudge * xfun; o->gcx[n] = o->gnudge * xfun;
  }
  for (int k = 1; k <= kz; k++) {
    double an = (o->hsigma[k] < 0.4) ? cfg->high_nudge
              : (o->hsigma[k] < 0.8) ? cfg->medium_nudge : cfg->low_nudge;
    for (int n = 2; n <= cfg->nspgx - 1 && n < 256; n++) {
      double xfun = exp(-((double)(n - 2) / an));
      o->hefc[n][k] = o->fnudge * xfun; o->hegc[n][k] = o->gnudge * xfun;
    }
  }
  /* sponge weights, Main/mod_bdycod.F90:237-250 (iboudy = 4) */
  if (cfg->iboudy == 4) {
    o->wgtd[2] = 0.20; o->wgtd[3] = 0.55; o->wgtd[4] = 0.80; o->wgtd[5] = 0.95;
    for (int n = 6; n <= cfg->nspgd - 1 && n < 256; n++) o->wgtd[n] = d_one;
    o->wgtx[2] = 0.4; o->wgtx[3] = 0.7; o->wgtx[4] = 0.9;
    for (int n = 5; n <= cfg->nspgx - 1 && n < 256; n++) o->wgtx[n] = 1.0;
  }
  /* splitf scalar geopotential terms, Main/mod_split.F90:343-353 */
  for (int l = 1; l <= o->nsplit; l++)
    for (int k = 1; k <= kz + 1; k++) {
      double sh = cfg->sigmah[k - 1], va = cfg->varpa1[l - 1][k - 1];
      o->pdlog[l - 1][k] = va * log(sh * cfg->pd + o->ptop);
      o->eps1[l - 1][k] = va * sh / (sh * cfg->pd + o->ptop);
    }

  int kp = kz + 1;
  o->rg_cr = (signed char*)calloc(o->plane, 1); o->rg_dt = (signed char*)calloc(o->plane, 1);
  o->ib_cr = (int*)calloc(o->plane, sizeof(int)); o->ib_dt = (int*)calloc(o->plane, sizeof(int));
  setup_boundaries(o, 0, o->rg_cr, o->ib_cr);
  setup_boundaries(o, 1, o->rg_dt, o->ib_dt);
  o->a1u = alloc3(o, kz); o->a1v = alloc3(o, kz); o->a1t = alloc3(o, kz);
  o->a2u = alloc3(o, kz); o->a2v = alloc3(o, kz); o->a2t = alloc3(o, kz);
  for (int n = 0; n < o->nqx; n++) {
    o->a1q[n] = alloc3(o, kz); o->a2q[n] = alloc3(o, kz); o->xq[n] = alloc3(o, kz);
    o->qb3d[n] = alloc3(o, kz); o->qten[n] = alloc3(o, kz); o->qdyn[n] = alloc3(o, kz);
    o->cq[n] = alloc3(o, kz);
  }
  if (o->nqx > 2) {
    o->qcd = alloc3(o, kz);
    for (int q = 0; q < 3; q++) { o->phyx[q] = alloc3(o, kz); o->atmsx[q] = alloc3(o, kz); }
  }
  o->psa = alloc3(o, 1); o->psb = alloc3(o, 1); o->psc = alloc3(o, 1);
  o->psdota = alloc3(o, 1); o->psdotb = alloc3(o, 1);
  o->dstor = alloc3(o, o->nsplit); o->hstor = alloc3(o, o->nsplit);
  o->msfx = alloc3(o, 1); o->msfd = alloc3(o, 1); o->xmsf = alloc3(o, 1); o->dmsf = alloc3(o, 1);
  o->coriol = alloc3(o, 1); o->ht = alloc3(o, 1); o->hgfact = alloc3(o, 1); o->map = alloc3(o, 1);
  o->ub0 = alloc3(o, kz); o->ubt = alloc3(o, kz); o->vb0 = alloc3(o, kz); o->vbt = alloc3(o, kz);
  o->tb0 = alloc3(o, kz); o->tbt = alloc3(o, kz); o->qb0 = alloc3(o, kz); o->qbt = alloc3(o, kz);
  o->pb0 = alloc3(o, 1); o->pbt = alloc3(o, 1);
  o->rpsa = alloc3(o, 1); o->rpsb = alloc3(o, 1); o->rpsc = alloc3(o, 1); o->rpsda = alloc3(o, 1);
  o->srpsb = alloc3(o, 1); o->rpsdotb = alloc3(o, 1);
  o->uc = alloc3(o, kz); o->vc = alloc3(o, kz); o->umc = alloc3(o, kz); o->vmc = alloc3(o, kz);
  o->ud = alloc3(o, kz); o->vd = alloc3(o, kz); o->xt = alloc3(o, kz); o->xtv = alloc3(o, kz);
  o->cr = alloc3(o, kz); o->pten = alloc3(o, 1); o->qdot = alloc3(o, kp); o->omega = alloc3(o, kz);
  o->dummy = alloc3(o, 1);
  o->ubd = alloc3(o, kz); o->vbd = alloc3(o, kz); o->tb3d = alloc3(o, kz);
  o->pb3d = alloc3(o, kz); o->pf3d = alloc3(o, kp);
  o->xkc = alloc3(o, kz); o->xkd = alloc3(o, kz);
  o->tten = alloc3(o, kz); o->tdyn = alloc3(o, kz); o->uten = alloc3(o, kz); o->udyn = alloc3(o, kz);
  o->vten = alloc3(o, kz); o->vdyn = alloc3(o, kz);
  o->fg = alloc3(o, kz); o->uavg1 = alloc3(o, kz); o->uavg2 = alloc3(o, kz);
  o->vavg1 = alloc3(o, kz); o->vavg2 = alloc3(o, kz); o->dotqdot = alloc3(o, kz);
  o->fg1 = alloc3(o, kp); o->fg2 = alloc3(o, kz);
  o->ct = alloc3(o, kz); o->cu = alloc3(o, kz); o->cv = alloc3(o, kz);
  o->td = alloc3(o, kz); o->tvfac = alloc3(o, kz); o->phi = alloc3(o, kz);
  o->deld = alloc3(o, 3 * o->nsplit); o->delh = alloc3(o, 3 * o->nsplit);
  o->ddsum = alloc3(o, o->nsplit); o->dhsum = alloc3(o, o->nsplit);
  o->xdelh = alloc3(o, 1); o->work = alloc3(o, 3); o->uu = alloc3(o, 1); o->vv = alloc3(o, 1);
  o->uuu = alloc3(o, kz); o->vvv = alloc3(o, kz);
  if (o->nh) {
    o->a1pp = alloc3(o, kz); o->a2pp = alloc3(o, kz); o->a1w = alloc3(o, kp); o->a2w = alloc3(o, kp);
    o->ppb0 = alloc3(o, kz); o->ppbt = alloc3(o, kz); o->wwb0 = alloc3(o, kp); o->wwbt = alloc3(o, kp);
    o->ps0 = alloc3(o, 1); o->pr0 = alloc3(o, kz); o->t0 = alloc3(o, kz); o->rho0 = alloc3(o, kz);
    o->z0 = alloc3(o, kz); o->pf0 = alloc3(o, kp); o->rhof0 = alloc3(o, kp); o->zf0 = alloc3(o, kp);
    o->dpsdxm = alloc3(o, 1); o->dpsdym = alloc3(o, 1); o->dprddx = alloc3(o, kz); o->dprddy = alloc3(o, kz);
    o->ef = alloc3(o, 1); o->ddx = alloc3(o, 1); o->ddy = alloc3(o, 1); o->dmdx = alloc3(o, 1);
    o->dmdy = alloc3(o, 1); o->ex = alloc3(o, 1); o->crx = alloc3(o, 1); o->cry = alloc3(o, 1);
    o->umd = alloc3(o, kz); o->vmd = alloc3(o, kz); o->xpp = alloc3(o, kz); o->xw = alloc3(o, kp);
    o->pr1 = alloc3(o, kz); o->rho1 = alloc3(o, kz); o->xpr = alloc3(o, kz);
    o->ucc = alloc3(o, kz); o->vcc = alloc3(o, kz); o->ppb3d = alloc3(o, kz); o->wb3d = alloc3(o, kp);
    o->xkcf = alloc3(o, kp);
    o->th = alloc3(o, kz); o->tha = alloc3(o, kz); o->thten = alloc3(o, kz);
    o->ppten = alloc3(o, kz); o->ppdyn = alloc3(o, kz); o->wten = alloc3(o, kp); o->wdyn = alloc3(o, kp);
    o->cpp = alloc3(o, kz); o->cw = alloc3(o, kp); o->cdt = alloc3(o, kz);
    double** sc[] = {&o->s_wo, &o->s_e, &o->s_f, &o->s_aa, &o->s_b, &o->s_c, &o->s_rhs, &o->s_ca,
                     &o->s_g1, &o->s_g2, &o->s_ptend, &o->s_pxup, &o->s_pyvp, &o->s_tk, &o->s_cc,
                     &o->s_cdd, &o->s_cj, &o->s_pi, &o->s_ucrs, &o->s_vcrs};
    for (size_t q = 0; q < sizeof(sc) / sizeof(sc[0]); q++) *sc[q] = alloc3(o, kp);
    o->estore = alloc3(o, 1); o->astore = alloc3(o, 1); o->wpval = alloc3(o, 1);
  }
  for (int q = 0; q < 5; q++) o->phy[q] = alloc3(o, kz);
  if (cfg->ibltyp == 2) {
    o->a1tke = alloc3(o, kp); o->a2tke = alloc3(o, kp); o->ctke = alloc3(o, kp);
    o->tkedyn = alloc3(o, kp); o->tkeps = alloc3(o, kp); o->tkephy = alloc3(o, kp);
    o->kpbl = alloc3(o, 1);
  }
  if (!o->nh && (cfg->ibltyp == 2 || cfg->idiffu == 3)) o->xkcf = alloc3(o, kp);
  if (o->nh) { o->phy[5] = alloc3(o, kz); o->phy[6] = alloc3(o, kp); }
  for (int q = 0; q < 22; q++) o->atms[q] = alloc3(o, atms_levels(q, kz));
  for (int q = 0; q < 4; q++) { o->bin[q] = alloc3(o, kz); o->bb1[q] = alloc3(o, kz); }
  o->bin[4] = alloc3(o, 1); o->bb1[4] = alloc3(o, 1);
  if (o->nh) {
    o->bin[5] = alloc3(o, kz); o->bb1[5] = alloc3(o, kz);
    o->bin[6] = alloc3(o, kp); o->bb1[6] = alloc3(o, kp);
    o->psdot0 = alloc3(o, 1);
  }
  o->rhmin = cfg->rhmin; o->rhmax = cfg->rhmax;
  size_t sjn = (size_t)o->nj * kz, sin_ = (size_t)o->ni * kz;
  o->sue = calloc(sjn, 8); o->sui = calloc(sjn, 8); o->nue = calloc(sjn, 8); o->nui = calloc(sjn, 8);
  o->sve = calloc(sjn, 8); o->svi = calloc(sjn, 8); o->nve = calloc(sjn, 8); o->nvi = calloc(sjn, 8);
  o->wue = calloc(sin_, 8); o->wui = calloc(sin_, 8); o->eue = calloc(sin_, 8); o->eui = calloc(sin_, 8);
  o->wve = calloc(sin_, 8); o->wvi = calloc(sin_, 8); o->eve = calloc(sin_, 8); o->evi = calloc(sin_, 8);
  return o;
}

void orc_destroy(orc_t* o) {
  if (!o) return;
  double** ptrs[] = {
    &o->a1u, &o->a1v, &o->a1t, &o->a2u, &o->a2v, &o->a2t, &o->psa, &o->psb, &o->psc,
    &o->psdota, &o->psdotb, &o->dstor, &o->hstor, &o->msfx, &o->msfd, &o->xmsf, &o->dmsf,
    &o->coriol, &o->ht, &o->hgfact, &o->map, &o->ub0, &o->ubt, &o->vb0, &o->vbt, &o->tb0,
    &o->tbt, &o->qb0, &o->qbt, &o->pb0, &o->pbt, &o->rpsa, &o->rpsb, &o->rpsc, &o->rpsda,
    &o->srpsb, &o->rpsdotb, &o->uc, &o->vc, &o->umc, &o->vmc, &o->ud, &o->vd, &o->xt, &o->xtv,
    &o->cr, &o->pten, &o->qdot, &o->omega, &o->dummy, &o->ubd, &o->vbd, &o->tb3d, &o->pb3d,
    &o->pf3d, &o->xkc, &o->xkd, &o->tten, &o->tdyn, &o->uten, &o->udyn, &o->vten, &o->vdyn,
    &o->fg, &o->uavg1, &o->uavg2, &o->vavg1, &o->vavg2, &o->dotqdot, &o->fg1, &o->fg2, &o->ct,
    &o->cu, &o->cv, &o->td, &o->tvfac, &o->phi, &o->deld, &o->delh, &o->ddsum, &o->dhsum,
    &o->xdelh, &o->work, &o->uu, &o->vv, &o->uuu, &o->vvv, &o->sue, &o->sui, &o->nue, &o->nui,
    &o->sve, &o->svi, &o->nve, &o->nvi, &o->wue, &o->wui, &o->eue, &o->eui, &o->wve, &o->wvi,
    &o->eve, &o->evi};
  for (size_t p = 0; p < sizeof(ptrs) / sizeof(ptrs[0]); p++) free(*ptrs[p]);
  double** nhp[] = {
    &o->a1pp, &o->a2pp, &o->a1w, &o->a2w, &o->ppb0, &o->ppbt, &o->wwb0, &o->wwbt, &o->ps0, &o->pr0,
    &o->t0, &o->rho0, &o->z0, &o->pf0, &o->rhof0, &o->zf0, &o->dpsdxm, &o->dpsdym, &o->dprddx,
    &o->dprddy, &o->ef, &o->ddx, &o->ddy, &o->dmdx, &o->dmdy, &o->ex, &o->crx, &o->cry, &o->umd,
    &o->vmd, &o->xpp, &o->xw, &o->pr1, &o->rho1, &o->xpr, &o->ucc, &o->vcc, &o->ppb3d, &o->wb3d,
    &o->xkcf, &o->ppten, &o->ppdyn, &o->wten, &o->wdyn, &o->cpp, &o->cw, &o->cdt, &o->s_wo, &o->s_e,
    &o->s_f, &o->s_aa, &o->s_b, &o->s_c, &o->s_rhs, &o->s_ca, &o->s_g1, &o->s_g2, &o->s_ptend,
    &o->s_pxup, &o->s_pyvp, &o->s_tk, &o->s_cc, &o->s_cdd, &o->s_cj, &o->s_pi, &o->s_ucrs, &o->s_vcrs,
    &o->estore, &o->astore, &o->wpval, &o->th, &o->tha, &o->thten};
  for (size_t p = 0; p < sizeof(nhp) / sizeof(nhp[0]); p++) free(*nhp[p]);
  for (int q = 0; q < 7; q++) free(o->phy[q]);
  free(o->a1tke); free(o->a2tke); free(o->ctke); free(o->tkedyn); free(o->tkeps); free(o->tkephy);
  free(o->kpbl);
  /* xkcf (also allocated for the hydrostatic core with ibltyp = 2 or idiffu = 3) is in the list above */
  for (int q = 0; q < 22; q++) free(o->atms[q]);
  for (int q = 0; q < 7; q++) { free(o->bin[q]); free(o->bb1[q]); }
  free(o->psdot0);
  free(o->s_tr);
  for (int n = 0; n < NQ; n++) {
    free(o->a1q[n]); free(o->a2q[n]); free(o->xq[n]); free(o->qb3d[n]);
    free(o->qten[n]); free(o->qdyn[n]); free(o->cq[n]);
  }
  free(o->qcd);
  for (int q = 0; q < 3; q++) { free(o->phyx[q]); free(o->atmsx[q]); }
  free(o->rg_cr); free(o->rg_dt); free(o->ib_cr); free(o->ib_dt);
  free(o);
}

void orc_set_gather(orc_t* o, orc_gather_fn fn) {
  o->gfn = fn;
  if (fn && !o->s_tr) o->s_tr = alloc3(o, 1);
}

void orc_set_exchange(orc_t* o, orc_exchange_fn fn, orc_exchange_bdy_fn bfn, void* ctx) {
  o->xfn = fn; o->bfn = bfn; o->xctx = ctx;
}

void orc_frame_info(const orc_t* o, int info[16]) {
  info[0] = o->j0; info[1] = o->i0; info[2] = o->nj; info[3] = o->ni;
  info[4] = o->jde1; info[5] = o->jde2; info[6] = o->ide1; info[7] = o->ide2;
  info[8] = o->jce1; info[9] = o->jce2; info[10] = o->ice1; info[11] = o->ice2;
  info[12] = o->bl; info[13] = o->br; info[14] = o->bb; info[15] = o->bt;
}

void orc_set_time(orc_t* o, long long lcount, double dt, double xbctime) {
  o->lcount = lcount; o->dt = dt; o->xbctime = xbctime;
}
void orc_get_time(const orc_t* o, long long* lcount, double* dt, double* xbctime) {
  *lcount = o->lcount; *dt = o->dt; *xbctime = o->xbctime;
}
void orc_diagnostics(const orc_t* o, double out[4]) {
  out[0] = o->ptntot; out[1] = o->pt2tot; out[2] = isnan(o->ptntot) ? 1.0 : 0.0; out[3] = 0;
}

static double* field_ptr(orc_t* o, int f, int* nk) {
  *nk = o->kz;
  if (f >= RCMDYN_TPHY && f <= RCMDYN_WPHY) {
    if (f == RCMDYN_WPHY) *nk = o->kz + 1;
    return o->phy[f - RCMDYN_TPHY];
  }
  if (f >= RCMDYN_ATMS_UBX3D && f <= RCMDYN_ATMS_RHB3D) {
    *nk = atms_levels(f - RCMDYN_ATMS_UBX3D, o->kz);
    return o->atms[f - RCMDYN_ATMS_UBX3D];
  }
  if (f >= RCMDYN_XUB_B1 && f <= RCMDYN_XWWB_B1) {
    if (f == RCMDYN_XPSB_B1) *nk = 1;
    if (f == RCMDYN_XWWB_B1) *nk = o->kz + 1;
    return o->bin[f - RCMDYN_XUB_B1];
  }
  if (f == RCMDYN_ATM0_PSDOT) { *nk = 1; return o->psdot0; }
  if (f >= RCMDYN_ATM1_TKE && f <= RCMDYN_TKEPHY) {
    *nk = o->kz + 1;
    return f == RCMDYN_ATM1_TKE ? o->a1tke : f == RCMDYN_ATM2_TKE ? o->a2tke : o->tkephy;
  }
  if (f == RCMDYN_KPBL) { *nk = 1; return o->kpbl; }
  if (f >= RCMDYN_ATM1_QI && f <= RCMDYN_ATMS_QXB3D_QS) {     /* nqx = 5 only */
    if (o->nqx < 5) return NULL;
    if (f <= RCMDYN_ATM1_QS) return o->a1q[2 + f - RCMDYN_ATM1_QI];
    if (f <= RCMDYN_ATM2_QS) return o->a2q[2 + f - RCMDYN_ATM2_QI];
    if (f <= RCMDYN_QSPHY) return o->phyx[f - RCMDYN_QIPHY];
    return o->atmsx[f - RCMDYN_ATMS_QXB3D_QI];
  }
  switch (f) {
    case RCMDYN_ATM1_U: return o->a1u;   case RCMDYN_ATM1_V: return o->a1v;
    case RCMDYN_ATM1_T: return o->a1t;   case RCMDYN_ATM1_QV: return o->a1q[0];
    case RCMDYN_ATM1_QC: return o->a1q[1];
    case RCMDYN_ATM2_U: return o->a2u;   case RCMDYN_ATM2_V: return o->a2v;
    case RCMDYN_ATM2_T: return o->a2t;   case RCMDYN_ATM2_QV: return o->a2q[0];
    case RCMDYN_ATM2_QC: return o->a2q[1];
    case RCMDYN_XUB_B0: return o->ub0;   case RCMDYN_XUB_BT: return o->ubt;
    case RCMDYN_XVB_B0: return o->vb0;   case RCMDYN_XVB_BT: return o->vbt;
    case RCMDYN_XTB_B0: return o->tb0;   case RCMDYN_XTB_BT: return o->tbt;
    case RCMDYN_XQB_B0: return o->qb0;   case RCMDYN_XQB_BT: return o->qbt;
    case RCMDYN_TTEN: return o->tten;    case RCMDYN_UTEN: return o->uten;
    case RCMDYN_VTEN: return o->vten;    case RCMDYN_QVTEN: return o->qten[0];
    case RCMDYN_QCTEN: return o->qten[1];
    case RCMDYN_OMEGA: return o->omega;  case RCMDYN_XKC: return o->xkc;
    case RCMDYN_PHI: return o->phi;
    case RCMDYN_QDOT: *nk = o->kz + 1; return o->qdot;
    case RCMDYN_DSTOR: *nk = o->nsplit; return o->dstor;
    case RCMDYN_ATM1_PP: return o->a1pp;  case RCMDYN_ATM2_PP: return o->a2pp;
    case RCMDYN_XPPB_B0: return o->ppb0;  case RCMDYN_XPPB_BT: return o->ppbt;
    case RCMDYN_ATM0_PR: return o->pr0;   case RCMDYN_ATM0_T: return o->t0;
    case RCMDYN_ATM0_RHO: return o->rho0; case RCMDYN_ATM0_Z: return o->z0;
    case RCMDYN_DPRDDX: return o->dprddx; case RCMDYN_DPRDDY: return o->dprddy;
    case RCMDYN_ATM1_W: *nk = o->kz + 1; return o->a1w;
    case RCMDYN_ATM2_W: *nk = o->kz + 1; return o->a2w;
    case RCMDYN_XWWB_B0: *nk = o->kz + 1; return o->wwb0;
    case RCMDYN_XWWB_BT: *nk = o->kz + 1; return o->wwbt;
    case RCMDYN_ATM0_PF: *nk = o->kz + 1; return o->pf0;
    case RCMDYN_ATM0_RHOF: *nk = o->kz + 1; return o->rhof0;
    case RCMDYN_ATM0_ZF: *nk = o->kz + 1; return o->zf0;
    case RCMDYN_HSTOR: *nk = o->nsplit; return o->hstor;
    default: break;
  }
  *nk = 1;
  switch (f) {
    case RCMDYN_PSA: return o->psa;      case RCMDYN_PSB: return o->psb;
    case RCMDYN_MSFX: return o->msfx;    case RCMDYN_MSFD: return o->msfd;
    case RCMDYN_CORIOL: return o->coriol; case RCMDYN_HT: return o->ht;
    case RCMDYN_XPSB_B0: return o->pb0;  case RCMDYN_XPSB_BT: return o->pbt;
    case RCMDYN_PSC: return o->psc;      case RCMDYN_PTEN: return o->pten;
    case RCMDYN_PSDOTA: return o->psdota;
    case RCMDYN_ATM0_PS: return o->ps0;
    case RCMDYN_DPSDXM: return o->dpsdxm; case RCMDYN_DPSDYM: return o->dpsdym;
    case RCMDYN_EF: return o->ef;   case RCMDYN_DDX: return o->ddx;   case RCMDYN_DDY: return o->ddy;
    case RCMDYN_DMDX: return o->dmdx; case RCMDYN_DMDY: return o->dmdy;
    case RCMDYN_EX: return o->ex;   case RCMDYN_CRX: return o->crx;   case RCMDYN_CRY: return o->cry;
    default: return NULL;
  }
}

static void prepare_static(orc_t* o);

int orc_put(orc_t* o, int field, const double* src, int j1, int j2, int i1, int i2, int k1, int k2) {
  int nk; double* a = field_ptr(o, field, &nk);
  if (!a) return 1;
  int nj = j2 - j1 + 1, ni = i2 - i1 + 1;
  for (int k = k1; k <= k2; k++) {
    if (k < 1 || k > nk) continue;
    for (int i = i1; i <= i2; i++) {
      if (i < o->i0 || i >= o->i0 + o->ni) continue;
      for (int j = j1; j <= j2; j++) {
        if (j < o->j0 || j >= o->j0 + o->nj) continue;
        A3(a, j, i, k) = src[((size_t)(k - k1) * ni + (i - i1)) * nj + (j - j1)];
      }
      /* a band's frame columns past either end of the period take the wrapped column, as its
       * periodic exchange would give them */
      if (o->cfg.i_band)
        for (int j = o->j0; j < o->j0 + o->nj; j++) {
          const int jw = j < 1 ? j + o->jx : (j > o->jx ? j - o->jx : j);
          if (jw == j || jw < j1 || jw > j2) continue;
          A3(a, j, i, k) = src[((size_t)(k - k1) * ni + (i - i1)) * nj + (jw - j1)];
        }
    }
    /* CRM: the frame rows past either end of the period take the wrapped row (and column) */
    if (o->cfg.i_crm)
      for (int i = o->i0; i < o->i0 + o->ni; i++) {
        const int iw = i < 1 ? i + o->iy : (i > o->iy ? i - o->iy : i);
        if (iw == i || iw < i1 || iw > i2) continue;
        for (int j = o->j0; j < o->j0 + o->nj; j++) {
          const int jw = !o->cfg.i_band ? j : (j < 1 ? j + o->jx : (j > o->jx ? j - o->jx : j));
          if (jw < j1 || jw > j2) continue;
          A3(a, j, i, k) = src[((size_t)(k - k1) * ni + (iw - i1)) * nj + (jw - j1)];
        }
      }
  }
  if (field == RCMDYN_MSFX || field == RCMDYN_MSFD || field == RCMDYN_HT) prepare_static(o);
  return 0;
}

/* Test hook: a copy of one internal work array over the whole frame ([k][i][j], nk levels,
 * the layout of orc_frame_info), for the NumPy restatement checks of terms that no rcmdyn
 * field exports (the NH pp/w tendencies after tend, as sound leaves them).  Returns nk, or
 * 0 for an unknown name or a too small buffer. */
int orc_get_work(orc_t* o, const char* name, double* dst, size_t cap) {
  const double* a = NULL;
  int nk = o->kz;
  if (!strcmp(name, "uten")) a = o->uten;
  else if (!strcmp(name, "vten")) a = o->vten;
  else if (o->nh && !strcmp(name, "ppten")) a = o->ppten;
  else if (o->nh && !strcmp(name, "wten")) { a = o->wten; nk = o->kz + 1; }
  /* sound's state (atmc%u, v, pp, w, the pi of the last sub-step) and what it reads */
  else if (o->nh && !strcmp(name, "cu")) a = o->cu;
  else if (o->nh && !strcmp(name, "cv")) a = o->cv;
  else if (o->nh && !strcmp(name, "cpp")) a = o->cpp;
  else if (o->nh && !strcmp(name, "cw")) { a = o->cw; nk = o->kz + 1; }
  else if (o->nh && !strcmp(name, "pi")) a = o->s_pi;
  else if (o->nh && !strcmp(name, "pr1")) a = o->pr1;
  else if (o->nh && !strcmp(name, "rho1")) a = o->rho1;
  else if (!strcmp(name, "ct")) a = o->ct;
  else if (!strcmp(name, "qdynv")) a = o->qdyn[0];
  else if (!strcmp(name, "qdync")) a = o->qdyn[1];
  else if (!strcmp(name, "cqv")) a = o->cq[0];
  else if (!strcmp(name, "cqc")) a = o->cq[1];
  else if (o->nqx > 2 && !strcmp(name, "cqi")) a = o->cq[2];
  else if (o->nqx > 2 && !strcmp(name, "cqr")) a = o->cq[3];
  else if (o->nqx > 2 && !strcmp(name, "cqs")) a = o->cq[4];
  else if (o->nqx > 2 && !strcmp(name, "qcd")) a = o->qcd;
  else if (o->nqx > 2 && !strcmp(name, "qteni")) a = o->qten[2];   /* the total tendencies (sums) */
  else if (o->nqx > 2 && !strcmp(name, "qtenr")) a = o->qten[3];
  else if (o->nqx > 2 && !strcmp(name, "qtens")) a = o->qten[4];
  if (!a || cap < o->plane * (size_t)nk) return 0;
  memcpy(dst, a, sizeof(double) * o->plane * (size_t)nk);
  return nk;
}

void orc_set_sound_probe(orc_t* o, int nsub) { o->sound_probe = nsub; }
void orc_set_tend_probe(orc_t* o, int stage) { o->tend_probe = stage; }

int orc_get(orc_t* o, int field, double* dst, int j1, int j2, int i1, int i2, int k1, int k2) {
  int nk; double* a = field_ptr(o, field, &nk);
  if (!a) return 1;
  int nj = j2 - j1 + 1, ni = i2 - i1 + 1;
  for (int k = k1; k <= k2; k++) {
    if (k < 1 || k > nk) continue;
    for (int i = i1; i <= i2; i++) {
      if (i < o->ide1 || i > o->ide2) continue;
      for (int j = j1; j <= j2; j++) {
        if (j < o->jde1 || j > o->jde2) continue;
        dst[((size_t)(k - k1) * ni + (i - i1)) * nj + (j - j1)] = A3(a, j, i, k);
      }
    }
  }
  return 0;
}

/* Static derived fields: Main/mod_params.F90:1993-2001 (xmsf, dmsf),
 * Main/mod_diffusion.F90:124-140 (hgfact), Main/mod_split.F90:99-101 (map). */
static void prepare_static(orc_t* o) {
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++) {
      A2(o->dmsf, j, i) = d_one / (A2(o->msfd, j, i) * A2(o->msfd, j, i) * o->dx16);
      A2(o->xmsf, j, i) = d_one / (A2(o->msfx, j, i) * A2(o->msfx, j, i) * o->dx4);
    }
  for (int i = o->ice1ga; i <= o->ice2ga; i++)
    for (int j = o->jce1ga; j <= o->jce2ga; j++) A2(o->hgfact, j, i) = o->xkhz;
  if (o->cfg.diffu_hgtf == 1) {
    for (int i = o->ici1ga; i <= o->ici2ga; i++)
      for (int j = o->jci1ga; j <= o->jci2ga; j++) {
        double h = A2(o->ht, j, i);
        double hg1 = fabs((h - A2(o->ht, j, i - 1)) / o->dx);
        double hg2 = fabs((h - A2(o->ht, j, i + 1)) / o->dx);
        double hg3 = fabs((h - A2(o->ht, j - 1, i)) / o->dx);
        double hg4 = fabs((h - A2(o->ht, j + 1, i)) / o->dx);
        double hgmax = dmax(dmax(dmax(hg1, hg2), hg3), hg4) * c_regrav * 1.0e3;
        A2(o->hgfact, j, i) = o->xkhz / (d_one + hgmax * hgmax);
      }
  }
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++)
      A2(o->map, j, i) = d_one / (A2(o->msfx, j, i) * A2(o->msfx, j, i));
}

/* psc2psd, Main/mpplib/mod_mppparam.F90:13811-13862 */
static void psc2psd(orc_t* o, const double* pc, double* pd) {
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++)
      A2(pd, j, i) = (A2(pc, j, i) + A2(pc, j, i - 1) + A2(pc, j - 1, i) + A2(pc, j - 1, i - 1)) * d_rfour;
  if (o->bt) for (int j = o->jdi1; j <= o->jdi2; j++)
    A2(pd, j, o->ide2) = (A2(pc, j, o->ice2) + A2(pc, j - 1, o->ice2)) * d_half;
  if (o->bb) for (int j = o->jdi1; j <= o->jdi2; j++)
    A2(pd, j, o->ide1) = (A2(pc, j, o->ice1) + A2(pc, j - 1, o->ice1)) * d_half;
  if (o->bl) for (int i = o->idi1; i <= o->idi2; i++)
    A2(pd, o->jde1, i) = (A2(pc, o->jce1, i) + A2(pc, o->jce1, i - 1)) * d_half;
  if (o->br) for (int i = o->idi1; i <= o->idi2; i++)
    A2(pd, o->jde2, i) = (A2(pc, o->jce2, i) + A2(pc, o->jce2, i - 1)) * d_half;
  if (o->bb && o->bl) A2(pd, o->jde1, o->ide1) = A2(pc, o->jce1, o->ice1);
  if (o->bt && o->bl) A2(pd, o->jde1, o->ide2) = A2(pc, o->jce1, o->ice2);
  if (o->bb && o->br) A2(pd, o->jde2, o->ide1) = A2(pc, o->jce2, o->ice1);
  if (o->bt && o->br) A2(pd, o->jde2, o->ide2) = A2(pc, o->jce2, o->ice2);
}

/* the exchange width idif of the diffused fields (Main/mod_params.F90:1965-1977): 2 for
 * idiffu = 1, 3 for idiffu = 3; idiffu = 2 (idif = 1) keeps 2, a superset */
static int idw(const orc_t* o) { return o->cfg.idiffu == 3 ? 3 : 2; }

/* calc_coeff idiffu = 3 (Main/mod_diffusion.F90:174-183): diff_6th_coef * p*b on every level
 * (xkcf on kz + 1 of them), diff_6th_coef * p*dotb on the dot points; no exchange */
static void calc_coeff6(orc_t* o) {
  int kz = o->kz;
  const double coef = diff_6th_factor * 0.015625 / (2.0 * o->dtsec);   /* :154 */
  memset(o->xkc, 0, sizeof(double) * o->plane * kz);
  memset(o->xkd, 0, sizeof(double) * o->plane * kz);
  memset(o->xkcf, 0, sizeof(double) * o->plane * (kz + 1));
  for (int k = 1; k <= kz + 1; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        if (k <= kz) A3(o->xkc, j, i, k) = coef * A2(o->psb, j, i);
        A3(o->xkcf, j, i, k) = coef * A2(o->psb, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) A3(o->xkd, j, i, k) = coef * A2(o->psdotb, j, i);
}

/* the bracket ((fx_p1 - fx_p0) + (fy_p1 - fy_p0)) of the idiffu = 3 scheme at (j, i, k),
 * Main/mod_diffusion.F90:428-470 (dot, f / msfd in the fluxes and the limiter) and 618-648
 * (cross, f in the fluxes, f / msfd in the limiter); neighbours clamped to 1..jmax, 1..imax */
static double diffu6_bracket(orc_t* o, const double* f, int j, int i, int k, int jmax, int imax, int dot) {
  const double* m = o->msfd;
  const int jm1 = j - 1 < 1 ? 1 : j - 1, jm2 = j - 2 < 1 ? 1 : j - 2, jm3 = j - 3 < 1 ? 1 : j - 3;
  const int jp1 = j + 1 > jmax ? jmax : j + 1, jp2 = j + 2 > jmax ? jmax : j + 2, jp3 = j + 3 > jmax ? jmax : j + 3;
  const int im1 = i - 1 < 1 ? 1 : i - 1, im2 = i - 2 < 1 ? 1 : i - 2, im3 = i - 3 < 1 ? 1 : i - 3;
  const int ip1 = i + 1 > imax ? imax : i + 1, ip2 = i + 2 > imax ? imax : i + 2, ip3 = i + 3 > imax ? imax : i + 3;
#define FV(J, I) (dot ? A3(f, J, I, k) / A2(m, J, I) : A3(f, J, I, k))
#define LV(J, I) (A3(f, J, I, k) / A2(m, J, I))
  double x0 = h4_c1 * (FV(j, i) - FV(jm1, i)) + h4_c2 * (FV(jp1, i) - FV(jm2, i)) + h4_c3 * (FV(jp2, i) - FV(jm3, i));
  if (x0 * (LV(j, i) - LV(jm1, i)) <= d_zero) x0 = d_zero;
  double x1 = h4_c1 * (FV(jp1, i) - FV(j, i)) + h4_c2 * (FV(jp2, i) - FV(jm1, i)) + h4_c3 * (FV(jp3, i) - FV(jm2, i));
  if (x1 * (LV(jp1, i) - LV(j, i)) <= d_zero) x1 = d_zero;
  double y0 = h4_c1 * (FV(j, i) - FV(j, im1)) + h4_c2 * (FV(j, ip1) - FV(j, im2)) + h4_c3 * (FV(j, ip2) - FV(j, im3));
  if (y0 * (LV(j, i) - LV(j, im1)) <= d_zero) y0 = d_zero;
  double y1 = h4_c1 * (FV(j, ip1) - FV(j, i)) + h4_c2 * (FV(j, ip2) - FV(j, im1)) + h4_c3 * (FV(j, ip3) - FV(j, im2));
  if (y1 * (LV(j, ip1) - LV(j, i)) <= d_zero) y1 = d_zero;
#undef FV
#undef LV
  return (x1 - x0) + (y1 - y0);
}

/* diffu_x3d / diffu_x4d3d / diffu_x3df idiffu = 3 (Main/mod_diffusion.F90:602-651, 736-785,
 * 893-942): the tile's column j = jci2 only, levels 1..nk; fac multiplies the coefficient
 * (x3df; 1 for the other two).  x3df reads xkc on kz + 1 levels, one past its allocation; the
 * coefficient is diff_6th_coef * p*b on every level, which xkcf holds. */
static void diffu_x6(orc_t* o, double* ften, const double* f, int nk, double fac) {
  const int j = o->jci2;
  for (int k = 1; k <= nk; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      A3(ften, j, i, k) = A3(ften, j, i, k) + fac * A3(o->xkcf, j, i, k) *
          diffu6_bracket(o, f, j, i, k, o->jx - 1, o->iy - 1, 0);
}

/* surface_pressures, Main/mod_tendency.F90:815-834 */
static void surface_pressures(orc_t* o) {
  xch(o, o->psa, 1, 1, 0);
  for (int i = o->ice1ga; i <= o->ice2ga; i++)
    for (int j = o->jce1ga; j <= o->jce2ga; j++) A2(o->rpsa, j, i) = d_one / A2(o->psa, j, i);
  psc2psd(o, o->psa, o->psdota);
  xch(o, o->psdota, 1, 1, 0);
  xch(o, o->psb, 1, idw(o), 0);
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) A2(o->rpsb, j, i) = d_one / A2(o->psb, j, i);
  psc2psd(o, o->psb, o->psdotb);
  xch(o, o->psdotb, 1, idw(o), 0);
}

/* decouple, Main/mod_tendency.F90:852-1116 (hydrostatic branches) */
static void decouple(orc_t* o) {
  int kz = o->kz;
  for (int i = o->ide1ga; i <= o->ide2ga; i++)
    for (int j = o->jde1ga; j <= o->jde2ga; j++) A2(o->rpsda, j, i) = d_one / A2(o->psdota, j, i);
  xch(o, o->a1u, kz, 1, 0); xch(o, o->a1v, kz, 1, 0); xch(o, o->a1t, kz, 1, 0);
  for (int n = 0; n < o->nqx; n++) xch(o, o->a1q[n], kz, 1, 0);
  for (int k = 1; k <= kz; k++)                                   /* :879-884 */
    for (int i = o->ide1ga; i <= o->ide2ga; i++)
      for (int j = o->jde1ga; j <= o->jde2ga; j++) {
        A3(o->uc, j, i, k) = A3(o->a1u, j, i, k);
        A3(o->vc, j, i, k) = A3(o->a1v, j, i, k);
        A3(o->umc, j, i, k) = A3(o->a1u, j, i, k) * A2(o->msfd, j, i);
        A3(o->vmc, j, i, k) = A3(o->a1v, j, i, k) * A2(o->msfd, j, i);
      }
  for (int k = 1; k <= kz; k++)                                   /* :888-891 */
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->ud, j, i, k) = A3(o->a1u, j, i, k) * A2(o->rpsda, j, i);
        A3(o->vd, j, i, k) = A3(o->a1v, j, i, k) * A2(o->rpsda, j, i);
      }
  if (o->bl) {                                                    /* :895-907 */
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->ud, o->jdi1, i, k) = SI(o->wui, i, k) * A2(o->rpsda, o->jdi1, i);
        A3(o->vd, o->jdi1, i, k) = SI(o->wvi, i, k) * A2(o->rpsda, o->jdi1, i);
      }
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->ud, o->jde1, i, k) = SI(o->wue, i, k) * A2(o->rpsda, o->jde1, i);
        A3(o->vd, o->jde1, i, k) = SI(o->wve, i, k) * A2(o->rpsda, o->jde1, i);
      }
    if (o->cfg.iboudy == 3 || o->cfg.iboudy == 4)                    /* :908-918 */
      for (int k = 1; k <= kz; k++)
        for (int i = o->idi1; i <= o->idi2; i++)
          if (A3(o->a1u, o->jde1, i, k) <= d_zero) {
            A3(o->ud, o->jde1, i, k) = A3(o->ud, o->jdi1, i, k);
            A3(o->vd, o->jde1, i, k) = A3(o->vd, o->jdi1, i, k);
          }
  }
  if (o->br) {                                                    /* :920-932 */
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->ud, o->jdi2, i, k) = SI(o->eui, i, k) * A2(o->rpsda, o->jdi2, i);
        A3(o->vd, o->jdi2, i, k) = SI(o->evi, i, k) * A2(o->rpsda, o->jdi2, i);
      }
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->ud, o->jde2, i, k) = SI(o->eue, i, k) * A2(o->rpsda, o->jde2, i);
        A3(o->vd, o->jde2, i, k) = SI(o->eve, i, k) * A2(o->rpsda, o->jde2, i);
      }
    if (o->cfg.iboudy == 3 || o->cfg.iboudy == 4)                    /* :933-943 */
      for (int k = 1; k <= kz; k++)
        for (int i = o->idi1; i <= o->idi2; i++)
          if (A3(o->a1u, o->jde2, i, k) >= d_zero) {
            A3(o->ud, o->jde2, i, k) = A3(o->ud, o->jdi2, i, k);
            A3(o->vd, o->jde2, i, k) = A3(o->vd, o->jdi2, i, k);
          }
  }
  if (o->bb) {                                                    /* :945-957 */
    for (int k = 1; k <= kz; k++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->ud, j, o->idi1, k) = SJ(o->sui, j, k) * A2(o->rpsda, j, o->idi1);
        A3(o->vd, j, o->idi1, k) = SJ(o->svi, j, k) * A2(o->rpsda, j, o->idi1);
      }
    for (int k = 1; k <= kz; k++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->ud, j, o->ide1, k) = SJ(o->sue, j, k) * A2(o->rpsda, j, o->ide1);
        A3(o->vd, j, o->ide1, k) = SJ(o->sve, j, k) * A2(o->rpsda, j, o->ide1);
      }
    if (o->cfg.iboudy == 3 || o->cfg.iboudy == 4)                    /* :958-968 */
      for (int k = 1; k <= kz; k++)
        for (int j = o->jde1; j <= o->jde2; j++)
          if (A3(o->a1v, j, o->ide1, k) >= d_zero) {
            A3(o->ud, j, o->ide1, k) = A3(o->ud, j, o->idi1, k);
            A3(o->vd, j, o->ide1, k) = A3(o->vd, j, o->idi1, k);
          }
  }
  if (o->bt) {                                                    /* :970-982 */
    for (int k = 1; k <= kz; k++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->ud, j, o->idi2, k) = SJ(o->nui, j, k) * A2(o->rpsda, j, o->idi2);
        A3(o->vd, j, o->idi2, k) = SJ(o->nvi, j, k) * A2(o->rpsda, j, o->idi2);
      }
    for (int k = 1; k <= kz; k++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->ud, j, o->ide2, k) = SJ(o->nue, j, k) * A2(o->rpsda, j, o->ide2);
        A3(o->vd, j, o->ide2, k) = SJ(o->nve, j, k) * A2(o->rpsda, j, o->ide2);
      }
    if (o->cfg.iboudy == 3 || o->cfg.iboudy == 4)                    /* :983-993 */
      for (int k = 1; k <= kz; k++)
        for (int j = o->jde1; j <= o->jde2; j++)
          if (A3(o->a1v, j, o->ide2, k) <= d_zero) {
            A3(o->ud, j, o->ide2, k) = A3(o->ud, j, o->idi2, k);
            A3(o->vd, j, o->ide2, k) = A3(o->vd, j, o->idi2, k);
          }
  }
  {                                                              /* :995-1004 */
    int w = o->cfg.isladvec == 1 ? 2 : 1;
    xch(o, o->ud, kz, w, 0); xch(o, o->vd, kz, w, 0);
  }
  /* umd/vmd (:1005-1008) feed only non-hydrostatic terms: not needed for idynamic=1 */
  for (int k = 1; k <= kz; k++)                                   /* :1013-1025 */
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++) {
        double rp = A2(o->rpsa, j, i);
        A3(o->xt, j, i, k) = A3(o->a1t, j, i, k) * rp;
        A3(o->xq[0], j, i, k) = dmax(A3(o->a1q[0], j, i, k) * rp, MINQQ);
        for (int n = 1; n < o->nqx; n++)                          /* n = iqfrst .. iqlst */
          A3(o->xq[n], j, i, k) = dmax(A3(o->a1q[n], j, i, k) * rp, d_zero);
        A3(o->xtv, j, i, k) = A3(o->xt, j, i, k) * (d_one + c_ep1 * A3(o->xq[0], j, i, k));
      }
  /* atm1%pr/rho (:1037-1040) and atm2%pr (:1094-1096) feed only physics: skipped */
  xch(o, o->a2u, kz, idw(o), 0); xch(o, o->a2v, kz, idw(o), 0); xch(o, o->a2t, kz, idw(o), 0);
  if (o->cfg.ibltyp == 2) {                                      /* :871, 1079 */
    xch(o, o->a1tke, kz + 1, 1, 0); xch(o, o->a2tke, kz + 1, idw(o), 0);
  }
  {                                                              /* :1073-1077 */
    int w = o->cfg.isladvec == 1 ? 4 : idw(o);                    /* max(idif, 4) */
    for (int n = 0; n < o->nqx; n++) xch(o, o->a2q[n], kz, w, 0);
  }
  if (o->nqx > 2) {                                              /* total water load, :1107-1115 */
    memset(o->qcd, 0, sizeof(double) * o->plane * kz);
    for (int n = 1; n < o->nqx; n++)
      for (int k = 1; k <= kz; k++)
        for (int i = o->ice1; i <= o->ice2; i++)
          for (int j = o->jce1; j <= o->jce2; j++) A3(o->qcd, j, i, k) = A3(o->qcd, j, i, k) + A3(o->xq[n], j, i, k);
  }
}
/* qcd of decouple: the total hydrometeor load for nqx = 5, else an alias of atmx%qx(iqc)
 * (Main/mod_tendency.F90:117-121) */
static const double* qcd_of(const orc_t* o) { return o->nqx > 2 ? o->qcd : o->xq[1]; }

/* compute_omega, Main/mod_tendency.F90:1118-1215 (hydrostatic) */
static void compute_omega(orc_t* o) {
  int kz = o->kz;
  memset(o->qdot, 0, sizeof(double) * o->plane * (kz + 1));
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++)
      A2(o->dummy, j, i) = d_one / (o->dx2 * A2(o->msfx, j, i) * A2(o->msfx, j, i));
  memset(o->pten, 0, sizeof(double) * o->plane);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double a = A3(o->umc, j + 1, i + 1, k) + A3(o->umc, j + 1, i, k) - A3(o->umc, j, i + 1, k) - A3(o->umc, j, i, k);
        double b = A3(o->vmc, j + 1, i + 1, k) + A3(o->vmc, j, i + 1, k) - A3(o->vmc, j + 1, i, k) - A3(o->vmc, j, i, k);
        A3(o->cr, j, i, k) = (a + b) * A2(o->dummy, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A2(o->pten, j, i) = A2(o->pten, j, i) - A3(o->cr, j, i, k) * o->dsigma[k];
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++)
      for (int k = 2; k <= kz; k++)
        A3(o->qdot, j, i, k) = A3(o->qdot, j, i, k - 1) -
            (A2(o->pten, j, i) + A3(o->cr, j, i, k - 1)) * o->dsigma[k - 1] * A2(o->rpsa, j, i);
  xch(o, o->cr, kz, 1, 0);
  xch(o, o->qdot, kz + 1, 1, 0);
  memset(o->omega, 0, sizeof(double) * o->plane * kz);
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      A2(o->dummy, j, i) = d_one / (o->dx8 * A2(o->msfx, j, i));
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double su = A3(o->ud, j, i, k) + A3(o->ud, j, i + 1, k) + A3(o->ud, j + 1, i + 1, k) + A3(o->ud, j + 1, i, k);
        double sv = A3(o->vd, j, i, k) + A3(o->vd, j, i + 1, k) + A3(o->vd, j + 1, i + 1, k) + A3(o->vd, j + 1, i, k);
        double x = su * (A2(o->psa, j + 1, i) - A2(o->psa, j - 1, i)) +
                   sv * (A2(o->psa, j, i + 1) - A2(o->psa, j, i - 1));
        A3(o->omega, j, i, k) = d_half * (A3(o->qdot, j, i, k + 1) + A3(o->qdot, j, i, k)) * A2(o->psa, j, i) +
                                o->hsigma[k] * (A2(o->pten, j, i) + x * A2(o->dummy, j, i));
      }
}

/* mkslice, Main/mod_slice.F90:102-300 -- the subset the hydrostatic dyn core reads
 * (ubd3d, vbd3d, tb3d, qxb3d, pb3d, pf3d); the physics-only slices are not built. */
static void mkslice(orc_t* o) {
  int kz = o->kz;
  for (int i = o->ice1gb; i <= o->ice2gb; i++)
    for (int j = o->jce1gb; j <= o->jce2gb; j++) A2(o->srpsb, j, i) = d_one / A2(o->psb, j, i);
  for (int i = o->ide1gb; i <= o->ide2gb; i++)
    for (int j = o->jde1gb; j <= o->jde2gb; j++) A2(o->rpsdotb, j, i) = d_one / A2(o->psdotb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1gb; i <= o->ide2gb; i++)
      for (int j = o->jde1gb; j <= o->jde2gb; j++) {
        A3(o->ubd, j, i, k) = A3(o->a2u, j, i, k) * A2(o->rpsdotb, j, i);
        A3(o->vbd, j, i, k) = A3(o->a2v, j, i, k) * A2(o->rpsdotb, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1gb; i <= o->ice2gb; i++)
      for (int j = o->jce1gb; j <= o->jce2gb; j++) {
        double rp = A2(o->srpsb, j, i);
        A3(o->tb3d, j, i, k) = A3(o->a2t, j, i, k) * rp;
        A3(o->qb3d[0], j, i, k) = dmax(A3(o->a2q[0], j, i, k) * rp, MINQQ);
        for (int n = 1; n < o->nqx; n++) A3(o->qb3d[n], j, i, k) = dmax(A3(o->a2q[n], j, i, k) * rp, d_zero);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->pb3d, j, i, k) = (o->hsigma[k] * A2(o->psb, j, i) + o->ptop) * d_1000;
  for (int k = 1; k <= kz + 1; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->pf3d, j, i, k) = (o->sigma[k] * A2(o->psb, j, i) + o->ptop) * d_1000;
}

/* pfesat / pfwsat, Share/pfesat.inc:21-49, Share/pfwsat.inc:1-17 */
static double pfwsat(double t, double p) {
  double tl = t - 273.15;
  if (tl > 100.0) tl = 100.0;
  if (tl < -75.0) tl = -75.0;
  double td = tl, esat;
  if (td >= 0.0)
    esat = 6.11213476 + td * (0.444007856 + td * (0.143064234e-01 + td * (0.264461437e-03 + td * (0.305903558e-05 +
           td * (0.196237241e-07 + td * (0.892344772e-10 + td * (-0.373208410e-12 + td * 0.209339997e-15)))))));
  else
    esat = 6.11123516 + td * (0.503109514 + td * (0.188369801e-01 + td * (0.420547422e-03 + td * (0.614396778e-05 +
           td * (0.602780717e-07 + td * (0.387940929e-09 + td * (0.149436277e-11 + td * 0.262655803e-14)))))));
  double es = esat * 100.0;
  return (AMW / AMD) * (es / (p - es));
}

/* The rest of mkslice (Main/mod_slice.F90:163-338) as the physics reads it: the atms export
 * of the physics coupling seam (rcmdyn ATMS_* fields), after mkslice / nh_mkslice, on the
 * tile's owned points of each loop's range (zero elsewhere, as the reference's zero-filled
 * allocations). */
enum { S_UBX, S_VBX, S_UBD, S_VBD, S_TB, S_QVB, S_QCB, S_TV, S_PB, S_PF, S_PS2D, S_RHOX, S_TH, S_RHOB,
       S_TP, S_WPX, S_WB, S_ZQ, S_ZA, S_DZQ, S_QSB, S_RHB };
static void slice_export(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  double** s = o->atms;
  const double rovcp = c_rgas * (d_one / c_cpd), rovg = c_rgas / EGRAV, p00 = 1.0e5;
  for (int q = 0; q < 22; q++) memset(s[q], 0, sizeof(double) * o->plane * atms_levels(q, kz));
  for (int k = 1; k <= kz; k++)                                    /* :171-174 */
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(s[S_UBD], j, i, k) = A3(o->ubd, j, i, k);
        A3(s[S_VBD], j, i, k) = A3(o->vbd, j, i, k);
      }
  for (int k = 1; k <= kz; k++)                                    /* :176-183 */
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(s[S_UBX], j, i, k) = d_rfour * (A3(o->ubd, j, i, k) + A3(o->ubd, j, i + 1, k) +
                                           A3(o->ubd, j + 1, i, k) + A3(o->ubd, j + 1, i + 1, k));
        A3(s[S_VBX], j, i, k) = d_rfour * (A3(o->vbd, j, i, k) + A3(o->vbd, j, i + 1, k) +
                                           A3(o->vbd, j + 1, i, k) + A3(o->vbd, j + 1, i + 1, k));
      }
  for (int k = 1; k <= kz; k++)                                    /* :185-202 */
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double tb = A3(o->tb3d, j, i, k), qv = A3(o->qb3d[0], j, i, k), qc = A3(o->qb3d[1], j, i, k);
        A3(s[S_TB], j, i, k) = tb;
        A3(s[S_QVB], j, i, k) = qv;
        A3(s[S_QCB], j, i, k) = qc;
        A3(s[S_TV], j, i, k) = tb * (d_one + c_ep1 * qv - qc);
        A3(s[S_PB], j, i, k) = A3(o->pb3d, j, i, k);
        for (int n = 2; n < o->nqx; n++) A3(o->atmsx[n - 2], j, i, k) = A3(o->qb3d[n], j, i, k);
      }
  for (int k = 1; k <= kp; k++)                                    /* :215-234 */
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A3(s[S_PF], j, i, k) = A3(o->pf3d, j, i, k);
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++)
      A2(s[S_PS2D], j, i) = o->nh ? A2(o->ps0, j, i) + o->ptop * d_1000 + A3(o->ppb3d, j, i, kz)
                                  : (A2(o->psb, j, i) + o->ptop) * d_1000;
  for (int i = o->ici1; i <= o->ici2; i++)                         /* :236-238 */
    for (int j = o->jci1; j <= o->jci2; j++)
      A2(s[S_RHOX], j, i) = A2(s[S_PS2D], j, i) / (c_rgas * A3(o->tb3d, j, i, kz));
  for (int k = 1; k <= kz; k++)                                    /* :240-243 */
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(s[S_TH], j, i, k) = A3(o->tb3d, j, i, k) * pow(p00 / A3(o->pb3d, j, i, k), rovcp);
  for (int k = 1; k <= kz; k++)                                    /* :244-248 */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(s[S_RHOB], j, i, k) = A3(o->pb3d, j, i, k) / (c_rgas * A3(o->tb3d, j, i, k));
        A3(s[S_TP], j, i, k) = A3(o->tb3d, j, i, k) * pow(A2(s[S_PS2D], j, i) / A3(o->pb3d, j, i, k), rovcp);
      }
  if (o->nh) {                                                     /* :250-257 */
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) A3(s[S_WPX], j, i, k) = A3(o->omega, j, i, k);
    for (int k = 1; k <= kp; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) A3(s[S_WB], j, i, k) = A3(o->wb3d, j, i, k);
  } else {                                                         /* :258-272 */
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) A3(s[S_WPX], j, i, k) = A3(o->omega, j, i, k) * d_1000;
    for (int k = 2; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(s[S_WB], j, i, k) = -d_half * c_regrav *
              (A3(s[S_WPX], j, i, k - 1) / A3(s[S_RHOB], j, i, k - 1) + A3(s[S_WPX], j, i, k) / A3(s[S_RHOB], j, i, k));
    for (int k = kz; k >= 1; k--)                                  /* :273-293 */
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) {
          double cell = o->ptop * A2(o->srpsb, j, i);
          A3(s[S_ZQ], j, i, k) = A3(s[S_ZQ], j, i, k + 1) + rovg * A3(s[S_TV], j, i, k) *
                                 log((o->sigma[k + 1] + cell) / (o->sigma[k] + cell));
        }
    for (int k = 1; k <= kz; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) {
          A3(s[S_ZA], j, i, k) = d_half * (A3(s[S_ZQ], j, i, k) + A3(s[S_ZQ], j, i, k + 1));
          A3(s[S_DZQ], j, i, k) = A3(s[S_ZQ], j, i, k) - A3(s[S_ZQ], j, i, k + 1);
        }
  }
  for (int k = 1; k <= kz; k++)                                    /* :330-338 */
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(s[S_QSB], j, i, k) = pfwsat(A3(o->tb3d, j, i, k), A3(o->pb3d, j, i, k));
        if (j >= o->jci1 && j <= o->jci2 && i >= o->ici1 && i <= o->ici2) {
          double rh = A3(o->qb3d[0], j, i, k) / A3(s[S_QSB], j, i, k);
          A3(s[S_RHB], j, i, k) = dmin(dmax(rh, o->rhmin), o->rhmax);
        }
      }
}

/* generic relaxation step shared by nudge2d/3d/4d3d/uv, Main/mod_bdycod.F90:4218-4766 */
static inline double relax(double ften, double xf, double xg, double f0, double f1, double f2,
                           double f3, double f4) {
  return ften + xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0);
}
static void nudge_coef(orc_t* o, int ib, int k, double* xf, double* xg) {
  if (o->cfg.iboudy == 1) { *xf = o->fcx[ib]; *xg = o->gcx[ib]; }
  else { *xf = o->hefc[ib][k]; *xg = o->hegc[ib][k]; }
}

/* new_pressure, Main/mod_tendency.F90:1428-1460 (+ nudge2d :4597-4766, or sponge2d
 * Main/mod_bdycod.F90:3065-3122 for iboudy = 4) */
static void new_pressure(orc_t* o) {
  double xt = o->xbctime + o->dt;
  if (o->cfg.iboudy == 4) {
    for (int r = 1; r <= 4; r++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          int ib = A2(o->ib_cr, j, i);
          A2(o->pten, j, i) = o->wgtx[ib] * A2(o->pten, j, i) + (d_one - o->wgtx[ib]) * A2(o->pbt, j, i);
        }
    goto forecast;
  }
  if (o->cfg.iboudy == 2 || o->cfg.iboudy == 3) goto forecast;   /* no p* relaxation (:1434-1438) */
  for (int i = o->ice1ga; i <= o->ice2ga; i++)
    for (int j = o->jce1ga; j <= o->jce2ga; j++)
      A3(o->fg1, j, i, 1) = (A2(o->pb0, j, i) + xt * A2(o->pbt, j, i)) - A2(o->psb, j, i);
  for (int r = 1; r <= 4; r++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        if (A2(o->rg_cr, j, i) != r) continue;
        double xf, xg;
        nudge_coef(o, A2(o->ib_cr, j, i), o->kz, &xf, &xg);
        A2(o->pten, j, i) = relax(A2(o->pten, j, i), xf, xg, A3(o->fg1, j, i, 1), A3(o->fg1, j - 1, i, 1),
                                  A3(o->fg1, j + 1, i, 1), A3(o->fg1, j, i - 1, 1), A3(o->fg1, j, i + 1, 1));
      }
forecast:
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) {
      A2(o->psc, j, i) = A2(o->psb, j, i) + A2(o->pten, j, i) * o->dt;
      A2(o->rpsc, j, i) = d_one / A2(o->psc, j, i);
    }
  o->ptntot = 0; o->pt2tot = 0;
  if (o->lcount > 0)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        o->ptntot = o->ptntot + fabs(A2(o->pten, j, i));
        o->pt2tot = o->pt2tot + fabs((A2(o->psc, j, i) + A2(o->psb, j, i) - d_two * A2(o->psa, j, i)) /
                                     (o->dt * o->dt * d_rfour));
      }
}

/* calc_coeff, Main/mod_diffusion.F90:169-251 (idiffu = 1, idynamic = 1) */
static void calc_coeff(orc_t* o) {
  if (o->cfg.idiffu == 3) { calc_coeff6(o); return; }
  int kz = o->kz;
  memset(o->xkc, 0, sizeof(double) * o->plane * kz);
  memset(o->xkd, 0, sizeof(double) * o->plane * kz);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double dudx = A3(o->ubd, j + 1, i, k) + A3(o->ubd, j + 1, i + 1, k) - A3(o->ubd, j, i, k) - A3(o->ubd, j, i + 1, k);
        double dvdx = A3(o->vbd, j + 1, i, k) + A3(o->vbd, j + 1, i + 1, k) - A3(o->vbd, j, i, k) - A3(o->vbd, j, i + 1, k);
        double dudy = A3(o->ubd, j, i + 1, k) + A3(o->ubd, j + 1, i + 1, k) - A3(o->ubd, j, i, k) - A3(o->ubd, j + 1, i, k);
        double dvdy = A3(o->vbd, j, i + 1, k) + A3(o->vbd, j + 1, i + 1, k) - A3(o->vbd, j, i, k) - A3(o->vbd, j + 1, i, k);
        double duv = sqrt((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy));
        A3(o->xkc, j, i, k) = dmin(A2(o->hgfact, j, i) + o->dydc * duv, o->xkhmax);
      }
  xch(o, o->xkc, kz, 1, 0);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++)
        A3(o->xkd, j, i, k) = d_rfour * (A3(o->xkc, j, i, k) + A3(o->xkc, j - 1, i - 1, k) +
                                         A3(o->xkc, j - 1, i, k) + A3(o->xkc, j, i - 1, k));
  if (o->cfg.ibltyp == 2) {                   /* xkcf, Main/mod_diffusion.F90:232-235, 245 */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->xkcf, j, i, 1) = A3(o->xkc, j, i, 1);
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) A3(o->xkcf, j, i, k + 1) = A3(o->xkc, j, i, k);
    for (int k = 1; k <= kz + 1; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(o->xkcf, j, i, k) = A3(o->xkcf, j, i, k) * o->rdxsq * A2(o->psb, j, i);
  }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->xkc, j, i, k) = A3(o->xkc, j, i, k) * o->rdxsq * A2(o->psb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++)
        A3(o->xkd, j, i, k) = A3(o->xkd, j, i, k) * o->rdxsq * A2(o->psdotb, j, i);
}

/* ---- advection, Main/mod_advection.F90 ---- */
static void start_advect(orc_t* o) {                               /* :111-120 */
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->uavg1, j, i, k) = A3(o->umc, j, i + 1, k) + A3(o->umc, j, i, k);
        A3(o->uavg2, j, i, k) = A3(o->umc, j + 1, i + 1, k) + A3(o->umc, j + 1, i, k);
        A3(o->vavg1, j, i, k) = A3(o->vmc, j + 1, i, k) + A3(o->vmc, j, i, k);
        A3(o->vavg2, j, i, k) = A3(o->vmc, j + 1, i + 1, k) + A3(o->vmc, j, i + 1, k);
      }
}

static void hadvuv(orc_t* o) {                                     /* :203-233 */
  const double* ua = o->umc; const double* va = o->vmc;
  const double* u = o->ud; const double* v = o->vd;
  double ul = o->ul;
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double ucmona = A3(ua, j, i + 1, k) + d_two * A3(ua, j, i, k) + A3(ua, j, i - 1, k);
        double ucmonb = A3(ua, j + 1, i + 1, k) + d_two * A3(ua, j + 1, i, k) + A3(ua, j + 1, i - 1, k);
        double ucmonc = A3(ua, j - 1, i + 1, k) + d_two * A3(ua, j - 1, i, k) + A3(ua, j - 1, i - 1, k);
        double vcmona = A3(va, j + 1, i, k) + d_two * A3(va, j, i, k) + A3(va, j - 1, i, k);
        double vcmonb = A3(va, j + 1, i + 1, k) + d_two * A3(va, j, i + 1, k) + A3(va, j - 1, i + 1, k);
        double vcmonc = A3(va, j + 1, i - 1, k) + d_two * A3(va, j, i - 1, k) + A3(va, j - 1, i - 1, k);
        double ff1 = ul * (A3(u, j + 1, i, k) + A3(u, j, i, k));
        double ff2 = ul * (A3(u, j - 1, i, k) + A3(u, j, i, k));
        double ff3 = ul * (A3(v, j, i + 1, k) + A3(v, j, i, k));
        double ff4 = ul * (A3(v, j, i - 1, k) + A3(v, j, i, k));
        if (o->cfg.upstream_mode) {
          ucmonb = (d_one + ff1) * ucmona + (d_one - ff1) * ucmonb;
          ucmonc = (d_one + ff2) * ucmonc + (d_one - ff2) * ucmona;
          vcmonb = (d_one + ff3) * vcmona + (d_one - ff3) * vcmonb;
          vcmonc = (d_one + ff4) * vcmonc + (d_one - ff4) * vcmona;
        } else {                    /* centred, upstream_mode = .false. (:152-155, :183-186) */
          ucmonb = ucmona + ucmonb;
          ucmonc = ucmonc + ucmona;
          vcmonb = vcmona + vcmonb;
          vcmonc = vcmonc + vcmona;
        }
        double dm = A2(o->dmsf, j, i);
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) - dm *
            ((A3(u, j + 1, i, k) + A3(u, j, i, k)) * ucmonb - (A3(u, j, i, k) + A3(u, j - 1, i, k)) * ucmonc +
             (A3(u, j, i + 1, k) + A3(u, j, i, k)) * vcmonb - (A3(u, j, i, k) + A3(u, j, i - 1, k)) * vcmonc);
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - dm *
            ((A3(v, j + 1, i, k) + A3(v, j, i, k)) * ucmonb - (A3(v, j, i, k) + A3(v, j - 1, i, k)) * ucmonc +
             (A3(v, j, i + 1, k) + A3(v, j, i, k)) * vcmonb - (A3(v, j, i, k) + A3(v, j, i - 1, k)) * vcmonc);
      }
}

static void vadvuv(orc_t* o) {                                     /* :286-299 */
  for (int k = 2; k <= o->kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double qq = d_rfour * (A3(o->qdot, j, i, k) + A3(o->qdot, j, i - 1, k) +
                               A3(o->qdot, j - 1, i, k) + A3(o->qdot, j - 1, i - 1, k));
        double uu = qq * (o->twt1[k] * A3(o->uc, j, i, k) + o->twt2[k] * A3(o->uc, j, i, k - 1));
        double vv = qq * (o->twt1[k] * A3(o->vc, j, i, k) + o->twt2[k] * A3(o->vc, j, i, k - 1));
        A3(o->udyn, j, i, k - 1) = A3(o->udyn, j, i, k - 1) - uu * o->xds[k - 1];
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + uu * o->xds[k];
        A3(o->vdyn, j, i, k - 1) = A3(o->vdyn, j, i, k - 1) - vv * o->xds[k - 1];
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) + vv * o->xds[k];
      }
}

/* upstream flux form shared by hadvt/hadvqv/hadvqx (:337-351, :547-561, :639-653); the
 * centred form of upstream_mode = .false. (:322-335, :532-545, :624-637) */
static void hadv_scalar(orc_t* o, const double* f, double* ften, int limiter /*0 none,1 t,2 q*/) {
  double ul = o->ul;
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double ps = A2(o->psa, j, i);
        double f1 = d_half * ul * (A3(o->uavg2, j, i, k) + A3(o->uavg1, j, i, k)) / ps;
        double f2 = d_half * ul * (A3(o->vavg2, j, i, k) + A3(o->vavg1, j, i, k)) / ps;
        double fx1 = (d_one + f1) * A3(f, j - 1, i, k) + (d_one - f1) * A3(f, j, i, k);
        double fx2 = (d_one + f1) * A3(f, j, i, k) + (d_one - f1) * A3(f, j + 1, i, k);
        double fy1 = (d_one + f2) * A3(f, j, i - 1, k) + (d_one - f2) * A3(f, j, i, k);
        double fy2 = (d_one + f2) * A3(f, j, i, k) + (d_one - f2) * A3(f, j, i + 1, k);
        if (!o->cfg.upstream_mode) {  /* centred (:323-332, :414-423, :443-446, :533-542, :625-634) */
          fx1 = A3(f, j - 1, i, k) + A3(f, j, i, k);
          fx2 = A3(f, j, i, k) + A3(f, j + 1, i, k);
          fy1 = A3(f, j, i - 1, k) + A3(f, j, i, k);
          fy2 = A3(f, j, i, k) + A3(f, j, i + 1, k);
        }
        A3(o->fg, j, i, k) = -A2(o->xmsf, j, i) *
            (A3(o->uavg2, j, i, k) * fx2 - A3(o->uavg1, j, i, k) * fx1 +
             A3(o->vavg2, j, i, k) * fy2 - A3(o->vavg1, j, i, k) * fy1);
      }
  if (limiter && o->cfg.stability_enhance) {                       /* :359-386, :569-596 */
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double fc = A3(f, j, i, k);
          double fn = A3(f, j, i + 1, k), fs = A3(f, j, i - 1, k);
          double fe = A3(f, j + 1, i, k), fw = A3(f, j - 1, i, k);
          double den, thr;
          if (limiter == 1) { den = A2(o->psa, j, i); thr = o->cfg.t_extrema; }
          else { den = dmax(fc, DLOWVAL); thr = o->cfg.q_rel_extrema; }
          double* g = &A3(o->fg, j, i, k);
          if (fabs(fn + fs - d_two * fc) / den > thr) {
            if (fc > fn && fc > fs) *g = dmin(*g, d_zero);
            else if (fc < fn && fc < fs) *g = dmax(*g, d_zero);
          }
          if (fabs(fe + fw - d_two * fc) / den > thr) {
            if (fc > fe && fc > fw) *g = dmin(*g, d_zero);
            else if (fc < fe && fc < fw) *g = dmax(*g, d_zero);
          }
        }
  }
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(ften, j, i, k) = A3(ften, j, i, k) + A3(o->fg, j, i, k);
}

static void vadv3d_t(orc_t* o) {                                   /* :771-783, ind = 1 */
  const double* f = o->a1t;
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++) A3(o->dotqdot, j, i, 1) = d_zero;
  for (int k = 2; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double pf = A3(o->pf3d, j, i, k);
        A3(o->dotqdot, j, i, k) = A3(o->qdot, j, i, k) *
            (o->twt1[k] * A3(f, j, i, k) * pow(pf / A3(o->pb3d, j, i, k), c_c287) +
             o->twt2[k] * A3(f, j, i, k - 1) * pow(pf / A3(o->pb3d, j, i, k - 1), c_c287));
      }
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      for (int k = 2; k <= o->kz; k++) {
        A3(o->tdyn, j, i, k - 1) = A3(o->tdyn, j, i, k - 1) - A3(o->dotqdot, j, i, k) * o->xds[k - 1];
        A3(o->tdyn, j, i, k) = A3(o->tdyn, j, i, k) + A3(o->dotqdot, j, i, k) * o->xds[k];
      }
}

static void vadvqv(orc_t* o) {                                     /* :811-836 */
  const double* f = o->a1q[0];
  memset(o->fg, 0, sizeof(double) * o->plane * o->kz);
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      for (int k = 2; k <= o->kz; k++) {
        double thr = MINQQ * A2(o->psa, j, i);
        if (A3(f, j, i, k) > thr && A3(f, j, i, k - 1) > thr)
          A3(o->fg, j, i, k) = A3(f, j, i, k) * pow(A3(f, j, i, k - 1) / A3(f, j, i, k), o->qcon[k]);
      }
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      for (int k = 2; k <= o->kz; k++) {
        double* t = o->qdyn[0];
        A3(t, j, i, k - 1) = A3(t, j, i, k - 1) - A3(o->qdot, j, i, k) * A3(o->fg, j, i, k) * o->xds[k - 1];
        A3(t, j, i, k) = A3(t, j, i, k) + A3(o->qdot, j, i, k) * A3(o->fg, j, i, k) * o->xds[k];
      }
}

/* vadv4d ind = 3 (iqxvadv = 3: ibltyp = 2 with iuwvadv = 1, Main/mod_tendency.F90:148-154),
 * Main/mod_advection.F90:917-957: fg = twt-interpolated f on every interface, the PBL-top
 * rule at kpb - 1 and kpb, then fg * svv.  fg is zeroed by the caller (:860). */
static void vadv4d_qc_uw(orc_t* o, const double* f) {
  for (int i = o->ici1; i <= o->ici2; i++)                            /* :918-920 */
    for (int j = o->jci1; j <= o->jci2; j++)
      for (int k = 2; k <= o->kz; k++)
        A3(o->fg, j, i, k) = o->twt1[k] * A3(f, j, i, k) + o->twt2[k] * A3(f, j, i, k - 1);
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++) {
      const int kpb = (int)A2(o->kpbl, j, i);
      if (kpb > o->kz) {                                              /* :923-925 (refused at put) */
        fprintf(stderr, "oracle: kpbl is greater than kz\n");
        abort();
      }
      if (kpb >= 4) {                                                 /* :926-955 */
        double slope;
        int k = kpb - 2;
        if ((A3(f, j, i, k + 1) - A3(f, j, i, k)) > d_zero && (A3(f, j, i, k) - A3(f, j, i, k - 1)) > d_zero) {
          slope = dmin((A3(f, j, i, k + 1) - A3(f, j, i, k)) / (o->hsigma[k + 1] - o->hsigma[k]),
                        (A3(f, j, i, k) - A3(f, j, i, k - 1)) / (o->hsigma[k] - o->hsigma[k - 1]));
        } else if ((A3(f, j, i, k + 1) - A3(f, j, i, k)) < d_zero && (A3(f, j, i, k) - A3(f, j, i, k - 1)) < d_zero) {
          slope = dmax((A3(f, j, i, k + 1) - A3(f, j, i, k)) / (o->hsigma[k + 1] - o->hsigma[k]),
                        (A3(f, j, i, k) - A3(f, j, i, k - 1)) / (o->hsigma[k] - o->hsigma[k - 1]));
        } else {
          slope = d_zero;
        }
        k = kpb;
        A3(o->fg, j, i, k - 1) = A3(f, j, i, k - 2) + slope * (o->sigma[k - 1] - o->hsigma[k - 2]);
        if (fabs(A3(f, j, i, k - 2) + slope * (o->hsigma[k - 1] - o->hsigma[k - 2]) - A3(f, j, i, k)) >
            fabs(A3(f, j, i, k - 1) - A3(f, j, i, k))) {
          A3(o->fg, j, i, k) = A3(f, j, i, k);
        } else {
          A3(o->fg, j, i, k) = A3(f, j, i, k - 2) + slope * (o->sigma[k] - o->hsigma[k - 2]);
        }
      }
    }
  for (int k = 2; k <= o->kz; k++)                                    /* :957 */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->fg, j, i, k) = A3(o->fg, j, i, k) * A3(o->qdot, j, i, k);
}

static void vadv4d_qx(orc_t* o, int n) {      /* :859-961, ind = 1 (or 3: iuwvadv), one hydrometeor */
  const double* f = o->a1q[n];
  memset(o->fg, 0, sizeof(double) * o->plane * o->kz);
  if (o->cfg.ibltyp == 2 && o->cfg.iuwvadv == 1) vadv4d_qc_uw(o, f);
  else
  for (int k = 2; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double svv = A3(o->qdot, j, i, k);
        double thr = MINQQ * MINQQ * A2(o->psa, j, i);
        double fk = A3(f, j, i, k), fkm = A3(f, j, i, k - 1);
        if (svv > d_zero) {
          A3(o->fg, j, i, k) = (fkm > thr) ? svv * (o->twt1[k] * fk + o->twt2[k] * fkm) : d_zero;
        } else {
          A3(o->fg, j, i, k) = (fk > thr) ? svv * (o->twt1[k] * fk + o->twt2[k] * fkm) : d_zero;
        }
      }
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      for (int k = 2; k <= o->kz; k++) {
        double* t = o->qdyn[n];
        A3(t, j, i, k - 1) = A3(t, j, i, k - 1) - A3(o->fg, j, i, k) * o->xds[k - 1];
        A3(t, j, i, k) = A3(t, j, i, k) + A3(o->fg, j, i, k) * o->xds[k];
      }
}

/* advection driver, Main/mod_tendency.F90:1270-1392 (hydrostatic, isladvec = 0) */
/* Semi-Lagrangian horizontal advection of the moisture (isladvec = 1), Main/mod_sladvection.F90.
 * trajcalc_x (:121-229, adv_velocity(.false.) :91-114) for every interior cross point and
 * level, then slhadv_x4d (:401-479) of atm2 qx and hdvg_x4d (:596-664) of atm1 qx into qxdyn.
 * ua/va = atmx%umd/vmd = ud*msfd (Main/mod_tendency.F90:998-1001), mapfx/mapfd = msfx/msfd. */
#define UA(J, I) (A3(o->ud, J, I, k) * A2(o->msfd, J, I))
#define VA(J, I) (A3(o->vd, J, I, k) * A2(o->msfd, J, I))
static int sl_advection(orc_t* o) {
  int kz = o->kz, bad = 0;
  double ddx = o->dx, ddy = o->dx, dt = o->dt, dtsq = dt * dt, dtcb = dt * dt * dt;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double uadvx = 0.25 * (UA(j, i) + UA(j, i + 1) + UA(j + 1, i + 1) + UA(j + 1, i)) / A2(o->msfx, j, i);
        double uadxp1 = 0.25 * (UA(j + 1, i) + UA(j + 1, i + 1) + UA(j + 2, i + 1) + UA(j + 2, i)) / A2(o->msfx, j + 1, i);
        double uadxm1 = 0.25 * (UA(j, i) + UA(j, i + 1) + UA(j - 1, i + 1) + UA(j - 1, i)) / A2(o->msfx, j - 1, i);
        double vadvy = 0.25 * (VA(j, i) + VA(j, i + 1) + VA(j + 1, i + 1) + VA(j + 1, i)) / A2(o->msfx, j, i);
        double vadyp1 = 0.25 * (VA(j, i + 1) + VA(j + 1, i + 1) + VA(j + 1, i + 2) + VA(j, i + 2)) / A2(o->msfx, j, i + 1);
        /* as written at :109-111: va(j+1,i) twice */
        double vadym1 = 0.25 * (VA(j, i) + VA(j, i - 1) + VA(j + 1, i) + VA(j + 1, i)) / A2(o->msfx, j, i - 1);
        double ux = 0.5 * (uadxp1 - uadxm1) / ddx;
        double uxx = (uadxp1 - 2.0 * uadvx + uadxm1) / (ddx * ddx);
        double xdis = -(uadvx * dt) + 0.5 * (dtsq * uadvx * ux) - (dtcb * uadvx) * (ux * ux + uadvx * uxx) / 6.0;
        double xn = xdis / ddx;
        if (!(fabs(xn) < 2.0)) { bad = 1; continue; }
        int xnp = (int)xn;
        double alfax = fabs((xnp * ddx - xdis) / ddx);
        int xsn = (int)copysign(1.0, xn);
        int xnd = j + xnp, xm1 = xnd + xsn, xm2 = xm1 + xsn, xp1 = xnd - xsn;
        if (o->bl) { if (xnd < o->jce1) xnd = o->jce1; if (xm1 < o->jce1) xm1 = o->jce1;
                     if (xm2 < o->jce1) xm2 = o->jce1; if (xp1 < o->jce1) xp1 = o->jce1; }
        if (o->br) { if (xnd > o->jce2) xnd = o->jce2; if (xm1 > o->jce2) xm1 = o->jce2;
                     if (xm2 > o->jce2) xm2 = o->jce2; if (xp1 > o->jce2) xp1 = o->jce2; }
        double vy = 0.5 * (vadyp1 - vadym1) / ddy;
        double vyy = (vadyp1 - 2.0 * vadvy + vadym1) / (ddy * ddy);
        double ydis = -(vadvy * dt) + 0.5 * (dtsq * vadvy * vy) - (dtcb * vadvy) * (vy * vy + vadvy * vyy) / 6.0;
        double yn = ydis / ddy;
        if (!(fabs(yn) < 2.0)) { bad = 1; continue; }
        int ynp = (int)yn;
        double betay = fabs((ynp * ddy - ydis) / ddy);
        int ysn = (int)copysign(1.0, yn);
        int ynd = i + ynp, ym1 = ynd + ysn, ym2 = ym1 + ysn, yp1 = ynd - ysn;
        if (o->bb) { if (ynd < o->ice1) ynd = o->ice1; if (ym1 < o->ice1) ym1 = o->ice1;
                     if (ym2 < o->ice1) ym2 = o->ice1; if (yp1 < o->ice1) yp1 = o->ice1; }
        if (o->bt) { if (ynd > o->ice2) ynd = o->ice2; if (ym1 > o->ice2) ym1 = o->ice2;
                     if (ym2 > o->ice2) ym2 = o->ice2; if (yp1 > o->ice2) yp1 = o->ice2; }
        double alfm2 = -(alfax * (1.0 - alfax * alfax)) / 6.0;
        double alfm1 = (alfax * (1.0 + alfax) * (2.0 - alfax)) / 2.0;
        double alf0 = ((1.0 - alfax * alfax) * (2.0 - alfax)) / 2.0;
        double alfp1 = -(alfax * (1.0 - alfax) * (2.0 - alfax)) / 6.0;
        double betm2 = -(betay * (1.0 - betay * betay)) / 6.0;
        double betm1 = (betay * (1.0 + betay) * (2.0 - betay)) / 2.0;
        double bet0 = ((1.0 - betay * betay) * (2.0 - betay)) / 2.0;
        double betp1 = -(betay * (1.0 - betay) * (2.0 - betay)) / 6.0;
        /* hdvg_x4d divergence (:625-649) */
        double ucapf = (UA(j + 1, i + 1) * A2(o->msfd, j + 1, i + 1) + UA(j + 1, i) * A2(o->msfd, j + 1, i)) * d_half;
        double ucapi = (UA(j, i + 1) * A2(o->msfd, j, i + 1) + UA(j, i) * A2(o->msfd, j, i)) * d_half;
        double vcapf = (VA(j + 1, i + 1) * A2(o->msfd, j + 1, i + 1) + VA(j, i + 1) * A2(o->msfd, j, i + 1)) * d_half;
        double vcapi = (VA(j + 1, i) * A2(o->msfd, j + 1, i) + VA(j, i) * A2(o->msfd, j, i)) * d_half;
        double ducapdx = (ucapf - ucapi) / o->dx;
        double dvcapdy = (vcapf - vcapi) / o->dx;
        double hdvg = (ducapdx + dvcapdy) / (A2(o->msfx, j, i) * A2(o->msfx, j, i));
        for (int n = 0; n < o->nqx; n++) {
          const double* var = o->a2q[n];
#define V(J, I) A3(var, J, I, k)
          double bl1 = alfax * V(xm1, yp1) + (d_one - alfax) * V(xnd, yp1);
          double bl2 = alfax * V(xm1, ym2) + (d_one - alfax) * V(xnd, ym2);
          double cb1 = alfm2 * V(xm2, ynd) + alfm1 * V(xm1, ynd) + alf0 * V(xnd, ynd) + alfp1 * V(xp1, ynd);
          double cb2 = alfm2 * V(xm2, ym1) + alfm1 * V(xm1, ym1) + alf0 * V(xnd, ym1) + alfp1 * V(xp1, ym1);
          double tbadp = betm2 * bl2 + betm1 * cb2 + bet0 * cb1 + betp1 * bl1;
          double tsla = tbadp;
          if (o->cfg.iqmsl == 1) {
            double tbmax = fmax(fmax(fmax(V(xnd, ynd), V(xnd, ym1)), V(xm1, ynd)), V(xm1, ym1));
            double tbmin = fmin(fmin(fmin(V(xnd, ynd), V(xnd, ym1)), V(xm1, ynd)), V(xm1, ym1));
            if (tbadp > tbmax) tsla = tbmax;
            else if (tbadp < tbmin) tsla = tbmin;
          }
          if (fabs(tsla - V(j, i)) > DLOWVAL)
            A3(o->qdyn[n], j, i, k) = A3(o->qdyn[n], j, i, k) + (tsla - V(j, i)) / dt;
#undef V
          double q1 = A3(o->a1q[n], j, i, k);
          double tatot = (q1 > DBL_EPSILON) ? q1 * hdvg : d_zero;
          A3(o->qdyn[n], j, i, k) = A3(o->qdyn[n], j, i, k) - tatot;
        }
      }
  return bad;
}
#undef UA
#undef VA

static int advection(orc_t* o) {
  int bad = 0;
  start_advect(o);
  hadvuv(o);
  vadvuv(o);
  hadv_scalar(o, o->xt, o->tdyn, 1);      /* hadvt */
  vadv3d_t(o);
  if (o->cfg.isladvec == 1) {
    /* slhadv_x / hdvg_x of qv and the hydrometeors (:1361-1363, 1378-1380); the reference runs
     * the qv pass, then vadv of qv, then the qx pass: the passes touch disjoint qxdyn planes */
    bad = sl_advection(o);
    if (o->tend_probe == 3) return bad;     /* test hook: qxdyn holds the semi-Lagrangian terms only */
    vadvqv(o);
  } else {
    hadv_scalar(o, o->xq[0], o->qdyn[0], 2); /* hadvqv */
    vadvqv(o);                               /* all(icup /= 1) */
    for (int n = 1; n < o->nqx; n++)         /* hadvqx, n = iqfrst .. iqlst (:1382) */
      hadv_scalar(o, o->xq[n], o->qdyn[n], 0);
  }
  for (int n = 1; n < o->nqx; n++) vadv4d_qx(o, n);   /* vadv iqfrst .. iqlst (:1388) */
  return bad;
}

/* curvature, Main/mod_tendency.F90:1829-1838 */
static void curvature(orc_t* o) {
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + A2(o->coriol, j, i) * A3(o->vc, j, i, k);
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - A2(o->coriol, j, i) * A3(o->uc, j, i, k);
      }
}

/* adiabatic, Main/mod_tendency.F90:1561-1575; cpmf Share/cpmf.inc */
static void adiabatic(orc_t* o) {
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double rovcpm = c_rgas / (c_cpd * (d_one + 0.80 * A3(o->xq[0], j, i, k)));
        A3(o->tdyn, j, i, k) = A3(o->tdyn, j, i, k) +
            (A3(o->omega, j, i, k) * rovcpm * A3(o->xtv, j, i, k)) /
            (o->ptop * A2(o->rpsa, j, i) + o->hsigma[k]);
      }
}

/* boundary, Main/mod_tendency.F90:1462-1471 -> nudge3d/nudge4d3d/nudgeuv */
/* sponge3d / sponge4d / spongeuv, Main/mod_bdycod.F90:2591-2994 (iboudy = 4): applied to the
 * total tendencies (pc_total), which are still zero when boundary runs (init_tendencies);
 * the dynamic terms are added to them afterwards (:285-294). */
static void sponge_all(orc_t* o) {
  int kz = o->kz;
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          int ib = A2(o->ib_cr, j, i);
          A3(o->tten, j, i, k) = o->wgtx[ib] * A3(o->tten, j, i, k) + (d_one - o->wgtx[ib]) * A3(o->tbt, j, i, k);
        }
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          int ib = A2(o->ib_cr, j, i);
          A3(o->qten[0], j, i, k) = o->wgtx[ib] * A3(o->qten[0], j, i, k) + (d_one - o->wgtx[ib]) * A3(o->qbt, j, i, k);
        }
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          if (A2(o->rg_dt, j, i) != r) continue;
          int ib = A2(o->ib_dt, j, i);
          A3(o->uten, j, i, k) = o->wgtd[ib] * A3(o->uten, j, i, k) + (d_one - o->wgtd[ib]) * A3(o->ubt, j, i, k);
          A3(o->vten, j, i, k) = o->wgtd[ib] * A3(o->vten, j, i, k) + (d_one - o->wgtd[ib]) * A3(o->vbt, j, i, k);
        }
}

static void boundary(orc_t* o) {
  int kz = o->kz;
  double xt = o->xbctime + o->dt;
  if (o->cfg.iboudy == 4) { sponge_all(o); return; }
  if (o->cfg.iboudy == 2 || o->cfg.iboudy == 3) return;   /* no relaxation (:1464-1480) */
  /* nudge3d(atm2%t, xtb, tdyn), Main/mod_bdycod.F90:4218-4406 */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A3(o->fg1, j, i, k) = (A3(o->tb0, j, i, k) + xt * A3(o->tbt, j, i, k)) - A3(o->a2t, j, i, k);
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          double xf, xg; nudge_coef(o, A2(o->ib_cr, j, i), k, &xf, &xg);
          A3(o->tdyn, j, i, k) = relax(A3(o->tdyn, j, i, k), xf, xg, A3(o->fg1, j, i, k),
              A3(o->fg1, j - 1, i, k), A3(o->fg1, j + 1, i, k), A3(o->fg1, j, i - 1, k), A3(o->fg1, j, i + 1, k));
        }
  /* nudge4d3d(atm2%qx, xqb, qxdyn, iqv), :3206-3392 */
  const double nfac = 1.0e3, rfac = d_one / nfac;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A3(o->fg1, j, i, k) = nfac * (A3(o->qb0, j, i, k) + xt * A3(o->qbt, j, i, k)) - nfac * A3(o->a2q[0], j, i, k);
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          double xf, xg; nudge_coef(o, A2(o->ib_cr, j, i), k, &xf, &xg);
          double f0 = A3(o->fg1, j, i, k), f1 = A3(o->fg1, j - 1, i, k), f2 = A3(o->fg1, j + 1, i, k);
          double f3 = A3(o->fg1, j, i - 1, k), f4 = A3(o->fg1, j, i + 1, k);
          A3(o->qdyn[0], j, i, k) = A3(o->qdyn[0], j, i, k) + rfac * (xf * f0 - xg * (f1 + f2 + f3 + f4 - d_four * f0));
        }
  /* nudgeuv(atm2%u, atm2%v, xub, xvb, udyn, vdyn), :3581-3823 (iboudy=5 uses hefc/hegc) */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1ga; i <= o->ide2ga; i++)
      for (int j = o->jde1ga; j <= o->jde2ga; j++) {
        A3(o->fg1, j, i, k) = ((A3(o->ub0, j, i, k) + xt * A3(o->ubt, j, i, k)) - A3(o->a2u, j, i, k));
        A3(o->fg2, j, i, k) = ((A3(o->vb0, j, i, k) + xt * A3(o->vbt, j, i, k)) - A3(o->a2v, j, i, k));
      }
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          if (A2(o->rg_dt, j, i) != r) continue;
          int ib = A2(o->ib_dt, j, i);
          double xf, xg;
          if (o->cfg.iboudy == 1) { xf = o->fcx[ib]; xg = o->gcx[ib]; }  /* fcd==fcx when nspgd==nspgx */
          else { xf = o->hefc[ib][k]; xg = o->hegc[ib][k]; }
          A3(o->udyn, j, i, k) = relax(A3(o->udyn, j, i, k), xf, xg, A3(o->fg1, j, i, k),
              A3(o->fg1, j - 1, i, k), A3(o->fg1, j + 1, i, k), A3(o->fg1, j, i - 1, k), A3(o->fg1, j, i + 1, k));
          A3(o->vdyn, j, i, k) = relax(A3(o->vdyn, j, i, k), xf, xg, A3(o->fg2, j, i, k),
              A3(o->fg2, j - 1, i, k), A3(o->fg2, j + 1, i, k), A3(o->fg2, j, i - 1, k), A3(o->fg2, j, i + 1, k));
        }
}

/* diffusion, Main/mod_tendency.F90:1515-1526 -> diffu_d, diffu_x3d, diffu_x4d */
static void diffu_x(orc_t* o, double* ften, const double* f, double fac) {
  if (o->cfg.idiffu == 3) { diffu_x6(o, ften, f, o->kz, d_one); return; }
  if (o->cfg.idiffu == 2) {
    /* diffu_x3d / diffu_x4d3d idiffu = 2, Main/mod_diffusion.F90:726-735, 881-891 */
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(ften, j, i, k) = A3(ften, j, i, k) + fac * A3(o->xkc, j, i, k) *
              (o4_c1 * (A3(f, j + 1, i, k) + A3(f, j - 1, i, k) + A3(f, j, i + 1, k) + A3(f, j, i - 1, k)) +
               o4_c2 * (A3(f, j + 1, i + 1, k) + A3(f, j - 1, i - 1, k) + A3(f, j - 1, i + 1, k) +
                        A3(f, j + 1, i - 1, k)) +
               o4_c3 * A3(f, j, i, k));
    return;
  }
  /* diffu_x3d / diffu_x4d3d idiffu = 1, Main/mod_diffusion.F90:673-713, 808-... */
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->icii1; i <= o->icii2; i++)
      for (int j = o->jcii1; j <= o->jcii2; j++)
        A3(ften, j, i, k) = A3(ften, j, i, k) - fac * A3(o->xkc, j, i, k) *
            (z4_c1 * (A3(f, j + 2, i, k) + A3(f, j - 2, i, k) + A3(f, j, i + 2, k) + A3(f, j, i - 2, k)) +
             z4_c2 * (A3(f, j + 1, i, k) + A3(f, j - 1, i, k) + A3(f, j, i + 1, k) + A3(f, j, i - 1, k)) +
             z4_c3 * A3(f, j, i, k));
#define LAP2(J, I) \
  A3(ften, J, I, k) = A3(ften, J, I, k) + fac * A3(o->xkc, J, I, k) * \
      (z4_c1 * (A3(f, (J) + 1, I, k) + A3(f, (J) - 1, I, k) + A3(f, J, (I) + 1, k) + A3(f, J, (I) - 1, k)) + \
       z4_c2 * A3(f, J, I, k))
  if (o->bl) for (int k = 1; k <= o->kz; k++) for (int i = o->ici1; i <= o->ici2; i++) LAP2(o->jci1, i);
  if (o->br) for (int k = 1; k <= o->kz; k++) for (int i = o->ici1; i <= o->ici2; i++) LAP2(o->jci2, i);
  if (o->bb) for (int k = 1; k <= o->kz; k++) for (int j = o->jci1; j <= o->jci2; j++) LAP2(j, o->ici1);
  if (o->bt) for (int k = 1; k <= o->kz; k++) for (int j = o->jci1; j <= o->jci2; j++) LAP2(j, o->ici2);
#undef LAP2
}

static void diffu_d(orc_t* o) {                                    /* :281-385 */
  const double* m = o->msfd;
  if (o->cfg.idiffu == 3) {                                        /* :412-516, j = jdi2 */
    const int j = o->jdi2;
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + A3(o->xkd, j, i, k) *
            diffu6_bracket(o, o->ubd, j, i, k, o->jx, o->iy, 1);
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) + A3(o->xkd, j, i, k) *
            diffu6_bracket(o, o->vbd, j, i, k, o->jx, o->iy, 1);
      }
    return;
  }
#define UM(a, J, I) (A3(a, J, I, k) / A2(m, J, I))
  if (o->cfg.idiffu == 2) {                                        /* :386-411 */
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + A3(o->xkd, j, i, k) *
              (o4_c1 * (UM(o->ubd, j + 1, i) + UM(o->ubd, j - 1, i) + UM(o->ubd, j, i + 1) + UM(o->ubd, j, i - 1)) +
               o4_c2 * (UM(o->ubd, j + 1, i + 1) + UM(o->ubd, j - 1, i - 1) + UM(o->ubd, j - 1, i + 1) +
                        UM(o->ubd, j + 1, i - 1)) +
               o4_c3 * (UM(o->ubd, j, i)));
          A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) + A3(o->xkd, j, i, k) *
              (o4_c1 * (UM(o->vbd, j + 1, i) + UM(o->vbd, j - 1, i) + UM(o->vbd, j, i + 1) + UM(o->vbd, j, i - 1)) +
               o4_c2 * (UM(o->vbd, j + 1, i + 1) + UM(o->vbd, j - 1, i - 1) + UM(o->vbd, j - 1, i + 1) +
                        UM(o->vbd, j + 1, i - 1)) +
               o4_c3 * (UM(o->vbd, j, i)));
        }
    return;
  }
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->idii1; i <= o->idii2; i++)
      for (int j = o->jdii1; j <= o->jdii2; j++) {
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) - A3(o->xkd, j, i, k) *
            (z4_c1 * (UM(o->ubd, j + 2, i) + UM(o->ubd, j - 2, i) + UM(o->ubd, j, i + 2) + UM(o->ubd, j, i - 2)) +
             z4_c2 * (UM(o->ubd, j + 1, i) + UM(o->ubd, j - 1, i) + UM(o->ubd, j, i + 1) + UM(o->ubd, j, i - 1)) +
             z4_c3 * (UM(o->ubd, j, i)));
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - A3(o->xkd, j, i, k) *
            (z4_c1 * (UM(o->vbd, j + 2, i) + UM(o->vbd, j - 2, i) + UM(o->vbd, j, i + 2) + UM(o->vbd, j, i - 2)) +
             z4_c2 * (UM(o->vbd, j + 1, i) + UM(o->vbd, j - 1, i) + UM(o->vbd, j, i + 1) + UM(o->vbd, j, i - 1)) +
             z4_c3 * (UM(o->vbd, j, i)));
      }
#define LAPD(J, I) do { \
  A3(o->udyn, J, I, k) = A3(o->udyn, J, I, k) + A3(o->xkd, J, I, k) * \
      (z4_c1 * (UM(o->ubd, (J) + 1, I) + UM(o->ubd, (J) - 1, I) + UM(o->ubd, J, (I) + 1) + UM(o->ubd, J, (I) - 1)) + \
       z4_c2 * (UM(o->ubd, J, I))); \
  A3(o->vdyn, J, I, k) = A3(o->vdyn, J, I, k) + A3(o->xkd, J, I, k) * \
      (z4_c1 * (UM(o->vbd, (J) + 1, I) + UM(o->vbd, (J) - 1, I) + UM(o->vbd, J, (I) + 1) + UM(o->vbd, J, (I) - 1)) + \
       z4_c2 * (UM(o->vbd, J, I))); } while (0)
  if (o->bl) for (int k = 1; k <= o->kz; k++) for (int i = o->idi1; i <= o->idi2; i++) LAPD(o->jdi1, i);
  if (o->br) for (int k = 1; k <= o->kz; k++) for (int i = o->idi1; i <= o->idi2; i++) LAPD(o->jdi2, i);
  if (o->bb) for (int k = 1; k <= o->kz; k++) for (int j = o->jdi1; j <= o->jdi2; j++) LAPD(j, o->idi1);
  if (o->bt) for (int k = 1; k <= o->kz; k++) for (int j = o->jdi1; j <= o->jdi2; j++) LAPD(j, o->idi2);
#undef LAPD
#undef UM
}

/* pressure_gradient_force, Main/mod_tendency.F90:1965-2115 (ipgf = 0) */
static void pressure_gradient_force(orc_t* o) {
  int kz = o->kz;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double tva = A3(o->a1t, j, i, k) * (d_one + c_ep1 * A3(o->xq[0], j, i, k));
        double tvb = A3(o->a2t, j, i, k) * (d_one + c_ep1 * A3(o->a2q[0], j, i, k) * A2(o->rpsb, j, i));
        double tvc = A3(o->ct, j, i, k) * (d_one + c_ep1 * A3(o->cq[0], j, i, k) * A2(o->rpsc, j, i));
        A3(o->td, j, i, k) = alpha_hyd * (tvc + tvb) + beta_hyd * tva;
      }
#define TDB(J, I) A3(o->td, J, I, k) = A3(o->a1t, J, I, k) * (d_one + c_ep1 * A3(o->xq[0], J, I, k))
  if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) TDB(o->jce1, i);
  if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) TDB(o->jce2, i);
  if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) TDB(j, o->ice1);
  if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) TDB(j, o->ice2);
#undef TDB
  /* ipgf = 1 (:1893-1964, 2039-2067): td minus the reference-atmosphere temperature.  The
   * reference loops k = -1..kz over arrays allocated 1..kz (out of bounds below k = 1); the
   * defined part k = 1..kz is restated. */
  const int ipgf = o->cfg.ipgf;
  if (ipgf == 1)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++)
          A3(o->td, j, i, k) = A3(o->td, j, i, k) - A2(o->psa, j, i) * T00PG *
              pow((o->hsigma[k] * A2(o->psa, j, i) + o->ptop) / P00PG, c_pgfaa1);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double rtbar = d_rfour * (A3(o->xtv, j - 1, i - 1, k) + A3(o->xtv, j - 1, i, k) +
                                  A3(o->xtv, j, i - 1, k) + A3(o->xtv, j, i, k));
        if (ipgf == 1)
          rtbar = rtbar - T00PG * pow((o->hsigma[k] * A2(o->psdota, j, i) + o->ptop) / P00PG, c_pgfaa1);
        rtbar = c_rgas * rtbar * A2(o->psdota, j, i);
        double hs = o->hsigma[k], pt = o->ptop;
        double den = o->dx * A2(o->msfd, j, i);
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) - rtbar *
            (log(d_half * (A2(o->psa, j, i) + A2(o->psa, j, i - 1)) * hs + pt) -
             log(d_half * (A2(o->psa, j - 1, i) + A2(o->psa, j - 1, i - 1)) * hs + pt)) / den;
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - rtbar *
            (log(d_half * (A2(o->psa, j, i) + A2(o->psa, j - 1, i)) * hs + pt) -
             log(d_half * (A2(o->psa, j - 1, i - 1) + A2(o->psa, j, i - 1)) * hs + pt)) / den;
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->tvfac, j, i, k) = d_one / (d_one + A3(qcd_of(o), j, i, k) / (d_one + A3(o->xq[0], j, i, k)));
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) {
      double rp = A2(o->rpsa, j, i);
      double tv = A3(o->td, j, i, kz) * rp * A3(o->tvfac, j, i, kz);
      double top = A2(o->ht, j, i);
      if (ipgf == 1)
        top = top + c_rgas * T00PG / c_pgfaa1 * pow((A2(o->psa, j, i) + o->ptop) / P00PG, c_pgfaa1);
      A3(o->phi, j, i, kz) = top - c_rgas * tv *
          log((o->hsigma[kz] + o->ptop * rp) / (d_one + o->ptop * rp));
    }
  for (int k = 1; k <= kz - 1; k++) {
    int lev = kz - k;
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double rp = A2(o->rpsa, j, i);
        double tvavg = ((A3(o->td, j, i, lev) * o->dsigma[lev] + A3(o->td, j, i, lev + 1) * o->dsigma[lev + 1]) /
                        (A2(o->psa, j, i) * (o->dsigma[lev] + o->dsigma[lev + 1]))) * A3(o->tvfac, j, i, lev);
        A3(o->phi, j, i, lev) = A3(o->phi, j, i, lev + 1) - c_rgas * tvavg *
            log((o->hsigma[lev] + o->ptop * rp) / (o->hsigma[lev + 1] + o->ptop * rp));
      }
  }
  xch(o, o->phi, kz, 1, 1);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double den = o->dx2 * A2(o->msfd, j, i);
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) - A2(o->psdota, j, i) *
            (A3(o->phi, j, i, k) + A3(o->phi, j, i - 1, k) - A3(o->phi, j - 1, i, k) - A3(o->phi, j - 1, i - 1, k)) / den;
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - A2(o->psdota, j, i) *
            (A3(o->phi, j, i, k) + A3(o->phi, j - 1, i, k) - A3(o->phi, j, i - 1, k) - A3(o->phi, j - 1, i - 1, k)) / den;
      }
}

/* spstep, Main/mod_split.F90:463-669 */
static void sp_gradient_divergence(orc_t* o, int ns, int nsrc) {
  double rdx2 = d_one / o->dx2;
  for (int i = o->ide1; i <= o->ide2; i++)
    for (int j = o->jde1; j <= o->jde2; j++) A2(o->xdelh, j, i) = DELH(j, i, ns, nsrc);
  xch(o, o->xdelh, 1, 1, 1);
  double *w1 = o->work, *w2 = o->work + o->plane, *w3 = o->work + 2 * o->plane;
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++) {
      double fac = o->dx2 * A2(o->msfx, j, i);
      A2(w1, j, i) = (A2(o->xdelh, j, i) + A2(o->xdelh, j, i - 1) - A2(o->xdelh, j - 1, i) - A2(o->xdelh, j - 1, i - 1)) / fac;
      A2(w2, j, i) = (A2(o->xdelh, j, i) + A2(o->xdelh, j - 1, i) - A2(o->xdelh, j, i - 1) - A2(o->xdelh, j - 1, i - 1)) / fac;
    }
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++) A2(w1, j, i) = A2(w1, j, i) * A2(o->psdota, j, i);
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++) A2(w2, j, i) = A2(w2, j, i) * A2(o->psdota, j, i);
  for (int i = o->idi1; i <= o->idi2; i++)
    for (int j = o->jdi1; j <= o->jdi2; j++) {
      A2(o->uu, j, i) = A2(w1, j, i) * A2(o->msfd, j, i);
      A2(o->vv, j, i) = A2(w2, j, i) * A2(o->msfd, j, i);
    }
  xch(o, o->uu, 1, 1, 2); xch(o, o->vv, 1, 1, 2);
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++)
      A2(w3, j, i) = rdx2 * A2(o->map, j, i) *
          (-A2(o->uu, j, i + 1) + A2(o->uu, j + 1, i + 1) - A2(o->uu, j, i) + A2(o->uu, j + 1, i) +
           A2(o->vv, j, i + 1) + A2(o->vv, j + 1, i + 1) - A2(o->vv, j, i) - A2(o->vv, j + 1, i));
}

static void spstep(orc_t* o) {
  const rcmdyn_config* c = &o->cfg;
  double* w3 = o->work + 2 * o->plane;
  memset(o->ddsum, 0, sizeof(double) * o->plane * o->nsplit);
  memset(o->dhsum, 0, sizeof(double) * o->plane * o->nsplit);
  for (int ns = 1; ns <= o->nsplit; ns++) {
    double* dd = o->ddsum + (size_t)(ns - 1) * o->plane;
    double* dh = o->dhsum + (size_t)(ns - 1) * o->plane;
    int n0 = 1, n1 = 2, n2 = n0;
    double aam = c->aam[ns - 1], dtau = c->dtau[ns - 1], hbar = c->hbar[ns - 1];
    int m2 = (int)aam * 2;
    double dtau2 = dtau * d_two;
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) { A2(dd, j, i) = DELD(j, i, ns, n0); A2(dh, j, i) = DELH(j, i, ns, n0); }
    sp_gradient_divergence(o, ns, n0);
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        DELD(j, i, ns, n1) = DELD(j, i, ns, n0) - dtau * A2(w3, j, i) + DELD(j, i, ns, 3) / (double)m2;
        DELH(j, i, ns, n1) = DELH(j, i, ns, n0) - dtau * hbar * DELD(j, i, ns, n0) / A2(o->psa, j, i) +
                             DELH(j, i, ns, 3) / (double)m2;
      }
    double fac = (aam - d_one) / aam;
    if (o->bl) for (int i = o->ici1; i <= o->ici2; i++) DELH(o->jce1, i, ns, n1) = DELH(o->jce1, i, ns, n0) * fac;
    if (o->br) for (int i = o->ici1; i <= o->ici2; i++) DELH(o->jce2, i, ns, n1) = DELH(o->jce2, i, ns, n0) * fac;
    if (o->bb) for (int j = o->jce1; j <= o->jce2; j++) DELH(j, o->ice1, ns, n1) = DELH(j, o->ice1, ns, n0) * fac;
    if (o->bt) for (int j = o->jce1; j <= o->jce2; j++) DELH(j, o->ice2, ns, n1) = DELH(j, o->ice2, ns, n0) * fac;
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A2(dd, j, i) = A2(dd, j, i) + DELD(j, i, ns, n1);
        A2(dh, j, i) = A2(dh, j, i) + DELH(j, i, ns, n1);
      }
    for (int n = 2; n <= m2; n++) {
      sp_gradient_divergence(o, ns, n1);
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          DELD(j, i, ns, n2) = DELD(j, i, ns, n0) - dtau2 * A2(w3, j, i) + DELD(j, i, ns, 3) / aam;
          DELH(j, i, ns, n2) = DELH(j, i, ns, n0) - dtau2 * hbar * DELD(j, i, ns, n1) / A2(o->psa, j, i) +
                               DELH(j, i, ns, 3) / aam;
        }
      if (o->bl) for (int i = o->ici1; i <= o->ici2; i++)
        DELH(o->jce1, i, ns, n2) = d_two * DELH(o->jce1, i, ns, n1) - DELH(o->jce1, i, ns, n0);
      if (o->br) for (int i = o->ici1; i <= o->ici2; i++)
        DELH(o->jce2, i, ns, n2) = d_two * DELH(o->jce2, i, ns, n1) - DELH(o->jce2, i, ns, n0);
      if (o->bb) for (int j = o->jce1; j <= o->jce2; j++)
        DELH(j, o->ice1, ns, n2) = d_two * DELH(j, o->ice1, ns, n1) - DELH(j, o->ice1, ns, n0);
      if (o->bt) for (int j = o->jce1; j <= o->jce2; j++)
        DELH(j, o->ice2, ns, n2) = d_two * DELH(j, o->ice2, ns, n1) - DELH(j, o->ice2, ns, n0);
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) {
          A2(dd, j, i) = A2(dd, j, i) + DELD(j, i, ns, n2);
          A2(dh, j, i) = A2(dh, j, i) + DELH(j, i, ns, n2);
        }
      n0 = n1; n1 = n2; n2 = n0;
    }
  }
}

/* divergence projection used three times in splitf, Main/mod_split.F90:286-294 */
static void project_div(orc_t* o, const double* u, const double* v, int slot) {
  int kz = o->kz;
  double rdx2 = d_one / o->dx2;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->uuu, j, i, k) = A3(u, j, i, k) * A2(o->msfd, j, i);
        A3(o->vvv, j, i, k) = A3(v, j, i, k) * A2(o->msfd, j, i);
      }
  xch(o, o->uuu, kz, 1, 2); xch(o, o->vvv, kz, 1, 2);
  for (int l = 1; l <= o->nsplit; l++) {
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) DELD(j, i, l, slot) = d_zero;
    for (int k = 1; k <= kz; k++) {
      double zr = o->cfg.zmatxr[l - 1][k - 1];
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++)
          DELD(j, i, l, slot) = DELD(j, i, l, slot) + zr * rdx2 * A2(o->map, j, i) *
              (-A3(o->uuu, j, i + 1, k) + A3(o->uuu, j + 1, i + 1, k) - A3(o->uuu, j, i, k) + A3(o->uuu, j + 1, i, k) +
               A3(o->vvv, j, i + 1, k) + A3(o->vvv, j + 1, i + 1, k) - A3(o->vvv, j, i, k) - A3(o->vvv, j + 1, i, k));
    }
  }
}

static void project_geo(orc_t* o, const double* ps, const double* t, int slot) {
  int kz = o->kz;
  for (int l = 1; l <= o->nsplit; l++) {
    double pdl = o->pdlog[l - 1][kz + 1], e1 = o->eps1[l - 1][kz + 1];
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double eps = e1 * (A2(ps, j, i) - o->cfg.pd);
        DELH(j, i, l, slot) = pdl + eps;
      }
    for (int k = 1; k <= kz; k++) {
      double pdk = o->pdlog[l - 1][k], ek = o->eps1[l - 1][k], ta = o->cfg.tau[l - 1][k - 1];
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) {
          double eps = ek * (A2(ps, j, i) - o->cfg.pd);
          DELH(j, i, l, slot) = DELH(j, i, l, slot) + pdk + ta * A3(t, j, i, k) / A2(ps, j, i) + eps;
        }
    }
  }
}

/* splitf, Main/mod_split.F90:243-461 */
static void splitf(orc_t* o) {
  int kz = o->kz, nsp = o->nsplit;
  memset(o->deld, 0, sizeof(double) * o->plane * 3 * nsp);
  memset(o->delh, 0, sizeof(double) * o->plane * 3 * nsp);
  xch(o, o->psa, 1, 1, 0);
  psc2psd(o, o->psa, o->psdota);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        DELD(j, i, n, 1) = A3(o->dstor, j, i, n);
        DELH(j, i, n, 1) = A3(o->hstor, j, i, n);
      }
  project_div(o, o->a1u, o->a1v, 3);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) DELD(j, i, n, 3) = DELD(j, i, n, 3) - DELD(j, i, n, 1);
  project_div(o, o->a2u, o->a2v, 2);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) DELD(j, i, n, 1) = DELD(j, i, n, 1) - DELD(j, i, n, 2);
  project_geo(o, o->psa, o->a1t, 3);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) DELH(j, i, n, 3) = DELH(j, i, n, 3) - DELH(j, i, n, 1);
  project_geo(o, o->psb, o->a2t, 2);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) DELH(j, i, n, 1) = DELH(j, i, n, 1) - DELH(j, i, n, 2);
  for (int n = 1; n <= nsp; n++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->dstor, j, i, n) = DELD(j, i, n, 2);
        A3(o->hstor, j, i, n) = DELH(j, i, n, 2);
      }
  spstep(o);
  double gnu1 = o->cfg.gnu1;
  for (int l = 1; l <= nsp; l++) {
    double an = o->cfg.an[l - 1], gnuan = gnu1 * an;
    double* dd = o->ddsum + (size_t)(l - 1) * o->plane;
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A2(o->psa, j, i) = A2(o->psa, j, i) - an * A2(dd, j, i);
        A2(o->psb, j, i) = A2(o->psb, j, i) - gnuan * A2(dd, j, i);
      }
  }
  for (int l = 1; l <= nsp; l++) {
    double* dd = o->ddsum + (size_t)(l - 1) * o->plane;
    for (int k = 1; k <= kz; k++) {
      double am = o->cfg.am[l - 1][k - 1], gnuam = gnu1 * am;
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          A3(o->a1t, j, i, k) = A3(o->a1t, j, i, k) + am * A2(dd, j, i);
          A3(o->a2t, j, i, k) = A3(o->a2t, j, i, k) + gnuam * A2(dd, j, i);
        }
    }
  }
  xch(o, o->dhsum, nsp, 1, 1);
  for (int l = 1; l <= nsp; l++) {
    double* dh = o->dhsum + (size_t)(l - 1) * o->plane;
    for (int k = 1; k <= kz; k++) {
      double zm = o->cfg.zmatx[l - 1][k - 1], gnuzm = gnu1 * zm;
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          double fac = A2(o->psdota, j, i) / (o->dx2 * A2(o->msfd, j, i));
          double x = fac * (A2(dh, j, i) + A2(dh, j, i - 1) - A2(dh, j - 1, i) - A2(dh, j - 1, i - 1));
          double y = fac * (A2(dh, j, i) - A2(dh, j, i - 1) + A2(dh, j - 1, i) - A2(dh, j - 1, i - 1));
          A3(o->a1u, j, i, k) = A3(o->a1u, j, i, k) - zm * x;
          A3(o->a1v, j, i, k) = A3(o->a1v, j, i, k) - zm * y;
          A3(o->a2u, j, i, k) = A3(o->a2u, j, i, k) - gnuzm * x;
          A3(o->a2v, j, i, k) = A3(o->a2v, j, i, k) - gnuzm * y;
        }
    }
  }
}

/* ======================================================================================
 * Non-hydrostatic core (idynamic = 2): Main/mod_tendency.F90 NH branches, Main/mod_sound.F90,
 * raydamp (Main/mod_bdycod.F90:4953-5123).  ithadv = 1, ipptls = 1 (qcd aliases atmx%qx(iqc),
 * Main/mod_tendency.F90:117-121), i_crm = 0, physics stubbed.
 * ====================================================================================== */
#define NH_REARTHRAD (d_one / 6.371229e6)            /* Share/mod_constants.F90:282-284 */
#define NH_MATHPI 3.1415926535897932384626433832795029 /* :254-255 */
static double nh_xgamma(void) { return d_one / (d_one - c_rgas * (d_one / c_cpd)); } /* mod_sound:77 */

/* surface_pressures NH (:836-848): p* is the constant reference p*; psdota/psdotb as
 * mod_init leaves them (Main/mod_init.F90:174-178) */
static void nh_surface_pressures(orc_t* o) {
  /* the constant p* on dot points as mod_init leaves it, ghosts included
   * (Main/mod_init.F90:174-178) */
  psc2psd(o, o->psa, o->psdota);
  xch(o, o->psdota, 1, 1, 0);
  psc2psd(o, o->psb, o->psdotb);
  xch(o, o->psdotb, 1, idw(o), 0);
  for (int i = o->ice1ga; i <= o->ice2ga; i++)
    for (int j = o->jce1ga; j <= o->jce2ga; j++) A2(o->rpsa, j, i) = d_one / A2(o->psa, j, i);
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) A2(o->rpsb, j, i) = d_one / A2(o->psb, j, i);
  for (int i = o->ide1ga; i <= o->ide2ga; i++)
    for (int j = o->jde1ga; j <= o->jde2ga; j++) A2(o->rpsda, j, i) = d_one / A2(o->psdota, j, i);
}

/* decouple NH additions (:1005-1008, :1041-1066, :1081-1084) */
static void nh_decouple(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  decouple(o);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1ga; i <= o->ide2ga; i++)
      for (int j = o->jde1ga; j <= o->jde2ga; j++) {
        A3(o->umd, j, i, k) = A3(o->ud, j, i, k) * A2(o->msfd, j, i);
        A3(o->vmd, j, i, k) = A3(o->vd, j, i, k) * A2(o->msfd, j, i);
      }
  xch(o, o->a1pp, kz, 1, 0); xch(o, o->a1w, kp, 1, 0);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A3(o->xpp, j, i, k) = A3(o->a1pp, j, i, k) * A2(o->rpsa, j, i);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A3(o->xw, j, i, k) = A3(o->a1w, j, i, k) * A2(o->rpsa, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++) {
        A3(o->pr1, j, i, k) = A3(o->pr0, j, i, k) + A3(o->xpp, j, i, k);
        A3(o->rho1, j, i, k) = A3(o->pr1, j, i, k) / (c_rgas * A3(o->xtv, j, i, k));
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->xpr, j, i, k) = (A3(o->xtv, j, i, k) - A3(o->t0, j, i, k) -
                               A3(o->xpp, j, i, k) / (c_cpd * A3(o->rho0, j, i, k))) / A3(o->xt, j, i, k);
  xch(o, o->a2pp, kz, idw(o), 0); xch(o, o->a2w, kp, idw(o), 0);
}

/* compute_omega NH (:1157-1192, :1216-1223) */
static void nh_compute_omega(orc_t* o) {
  int kz = o->kz;
  memset(o->qdot, 0, sizeof(double) * o->plane * (kz + 1));
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++)
      A2(o->dummy, j, i) = d_one / (o->dx2 * A2(o->msfx, j, i) * A2(o->msfx, j, i));
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(o->ucc, j, i, k) = A3(o->umd, j, i, k) + A3(o->umd, j, i + 1, k) + A3(o->umd, j + 1, i, k) + A3(o->umd, j + 1, i + 1, k);
        A3(o->vcc, j, i, k) = A3(o->vmd, j, i, k) + A3(o->vmd, j, i + 1, k) + A3(o->vmd, j + 1, i, k) + A3(o->vmd, j + 1, i + 1, k);
      }
  for (int k = 2; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->qdot, j, i, k) = -A3(o->rhof0, j, i, k) * EGRAV * A3(o->xw, j, i, k) / A2(o->ps0, j, i) -
            o->sigma[k] * (A2(o->dpsdxm, j, i) * (o->twt1[k] * A3(o->ucc, j, i, k) + o->twt2[k] * A3(o->ucc, j, i, k - 1)) +
                           A2(o->dpsdym, j, i) * (o->twt1[k] * A3(o->vcc, j, i, k) + o->twt2[k] * A3(o->vcc, j, i, k - 1)));
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double a = A3(o->umc, j + 1, i + 1, k) + A3(o->umc, j + 1, i, k) - A3(o->umc, j, i + 1, k) - A3(o->umc, j, i, k);
        double b = A3(o->vmc, j + 1, i + 1, k) + A3(o->vmc, j, i + 1, k) - A3(o->vmc, j + 1, i, k) - A3(o->vmc, j, i, k);
        A3(o->cr, j, i, k) = (a + b) * A2(o->dummy, j, i) +
            (A3(o->qdot, j, i, k + 1) - A3(o->qdot, j, i, k)) * A2(o->psa, j, i) / o->dsigma[k];
      }
  xch(o, o->cr, kz, 1, 0);
  xch(o, o->qdot, kz + 1, 1, 0);
  memset(o->omega, 0, sizeof(double) * o->plane * kz);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->omega, j, i, k) = -d_half * EGRAV * A3(o->rho0, j, i, k) * A2(o->rpsb, j, i) *
                                (A3(o->a2w, j, i, k) + A3(o->a2w, j, i, k + 1));
}

/* mkslice NH subset the dyn core reads (Main/mod_slice.F90:163-183, 215-238, 278-281) */
static void nh_mkslice(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  mkslice(o);                              /* ubd, vbd, tb3d, qb3d (pb3d/pf3d overwritten below) */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1gb; i <= o->ice2gb; i++)
      for (int j = o->jce1gb; j <= o->jce2gb; j++)
        A3(o->ppb3d, j, i, k) = A3(o->a2pp, j, i, k) * A2(o->srpsb, j, i);
  for (int k = 2; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->pb3d, j, i, k) = A3(o->pr0, j, i, k) + A3(o->ppb3d, j, i, k);
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) {
      A3(o->pb3d, j, i, 1) = dmax(A3(o->pr0, j, i, 1) + A3(o->ppb3d, j, i, 1), o->ptop * d_1000 + 1.0);
      double ps2d = A2(o->ps0, j, i) + o->ptop * d_1000 + A3(o->ppb3d, j, i, kz);
      A3(o->pf3d, j, i, 1) = o->ptop * d_1000;
      A3(o->pf3d, j, i, kp) = ps2d;
    }
  for (int k = 2; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->pf3d, j, i, k) = A3(o->pf0, j, i, k) + d_half * (A3(o->ppb3d, j, i, k - 1) + A3(o->ppb3d, j, i, k));
  for (int k = 1; k <= kp; k++)
    for (int i = o->ice1gb; i <= o->ice2gb; i++)
      for (int j = o->jce1gb; j <= o->jce2gb; j++)
        A3(o->wb3d, j, i, k) = A3(o->a2w, j, i, k) * A2(o->srpsb, j, i);
}

/* calc_coeff NH (Main/mod_diffusion.F90:215-250) */
static void nh_calc_coeff(orc_t* o) {
  if (o->cfg.idiffu == 3) { calc_coeff6(o); return; }
  int kz = o->kz, kp = kz + 1;
  memset(o->xkc, 0, sizeof(double) * o->plane * kz);
  memset(o->xkd, 0, sizeof(double) * o->plane * kz);
  memset(o->xkcf, 0, sizeof(double) * o->plane * kp);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        double dudx = A3(o->ubd, j + 1, i, k) + A3(o->ubd, j + 1, i + 1, k) - A3(o->ubd, j, i, k) - A3(o->ubd, j, i + 1, k);
        double dvdx = A3(o->vbd, j + 1, i, k) + A3(o->vbd, j + 1, i + 1, k) - A3(o->vbd, j, i, k) - A3(o->vbd, j, i + 1, k);
        double dudy = A3(o->ubd, j, i + 1, k) + A3(o->ubd, j + 1, i + 1, k) - A3(o->ubd, j, i, k) - A3(o->ubd, j + 1, i, k);
        double dvdy = A3(o->vbd, j, i + 1, k) + A3(o->vbd, j + 1, i + 1, k) - A3(o->vbd, j, i, k) - A3(o->vbd, j + 1, i, k);
        double dwdz = A3(o->wb3d, j, i, k) - A3(o->wb3d, j, i, k + 1);
        double duv = sqrt(dmax((dudx - dvdy) * (dudx - dvdy) + (dvdx + dudy) * (dvdx + dudy) - dwdz * dwdz, d_zero));
        A3(o->xkc, j, i, k) = dmin(A2(o->hgfact, j, i) + o->dydc * duv, o->xkhmax);
      }
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++) A3(o->xkcf, j, i, 1) = A3(o->xkc, j, i, 1);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->xkcf, j, i, k + 1) = A3(o->xkc, j, i, k);
  xch(o, o->xkc, kz, 1, 0);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++)
        A3(o->xkd, j, i, k) = d_rfour * (A3(o->xkc, j, i, k) + A3(o->xkc, j - 1, i - 1, k) +
                                         A3(o->xkc, j - 1, i, k) + A3(o->xkc, j, i - 1, k));
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->xkc, j, i, k) = A3(o->xkc, j, i, k) * o->rdxsq * A2(o->psb, j, i);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->xkcf, j, i, k) = A3(o->xkcf, j, i, k) * o->rdxsq * A2(o->psb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++)
        A3(o->xkd, j, i, k) = A3(o->xkd, j, i, k) * o->rdxsq * A2(o->psdotb, j, i);
}

/* hadvuv NH upstream branch (Main/mod_advection.F90:235-264): flux form minus u*divergence */
static void nh_hadvuv(orc_t* o) {
  const double* ua = o->umc; const double* va = o->vmc;
  const double* u = o->ud; const double* v = o->vd;
  double ul = o->ul;
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double divd = d_rfour * (A3(o->cr, j, i, k) + A3(o->cr, j, i - 1, k) + A3(o->cr, j - 1, i, k) + A3(o->cr, j - 1, i - 1, k));
        double ucmona = A3(ua, j, i + 1, k) + d_two * A3(ua, j, i, k) + A3(ua, j, i - 1, k);
        double ucmonb = A3(ua, j + 1, i + 1, k) + d_two * A3(ua, j + 1, i, k) + A3(ua, j + 1, i - 1, k);
        double ucmonc = A3(ua, j - 1, i + 1, k) + d_two * A3(ua, j - 1, i, k) + A3(ua, j - 1, i - 1, k);
        double vcmona = A3(va, j + 1, i, k) + d_two * A3(va, j, i, k) + A3(va, j - 1, i, k);
        double vcmonb = A3(va, j + 1, i + 1, k) + d_two * A3(va, j, i + 1, k) + A3(va, j - 1, i + 1, k);
        double vcmonc = A3(va, j + 1, i - 1, k) + d_two * A3(va, j, i - 1, k) + A3(va, j - 1, i - 1, k);
        double dm = A2(o->dmsf, j, i);
        double diag = divd - dm * ((ucmonb - ucmonc) + (vcmonb - vcmonc));
        double ff1 = ul * (A3(u, j + 1, i, k) + A3(u, j, i, k));
        double ff2 = ul * (A3(u, j - 1, i, k) + A3(u, j, i, k));
        double ff3 = ul * (A3(v, j, i + 1, k) + A3(v, j, i, k));
        double ff4 = ul * (A3(v, j, i - 1, k) + A3(v, j, i, k));
        if (o->cfg.upstream_mode) {
          ucmonb = (d_one + ff1) * ucmona + (d_one - ff1) * ucmonb;
          ucmonc = (d_one + ff2) * ucmonc + (d_one - ff2) * ucmona;
          vcmonb = (d_one + ff3) * vcmona + (d_one - ff3) * vcmonb;
          vcmonc = (d_one + ff4) * vcmonc + (d_one - ff4) * vcmona;
        } else {                    /* centred, upstream_mode = .false. (:152-155, :183-186) */
          ucmonb = ucmona + ucmonb;
          ucmonc = ucmonc + ucmona;
          vcmonb = vcmona + vcmonb;
          vcmonc = vcmonc + vcmona;
        }
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + A3(u, j, i, k) * diag - dm *
            (A3(u, j + 1, i, k) * ucmonb - A3(u, j - 1, i, k) * ucmonc + A3(u, j, i + 1, k) * vcmonb - A3(u, j, i - 1, k) * vcmonc);
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) + A3(v, j, i, k) * diag - dm *
            (A3(v, j + 1, i, k) * ucmonb - A3(v, j - 1, i, k) * ucmonc + A3(v, j, i + 1, k) * vcmonb - A3(v, j, i - 1, k) * vcmonc);
      }
}

/* hadv3d ind = 1 upstream (Main/mod_advection.F90:486-507): w on full levels 2..kz */
static void nh_hadv3d_w(orc_t* o, const double* f, double* ften) {
  double ul = o->ul;
  for (int k = 2; k <= o->kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double t1 = o->twt1[k], t2 = o->twt2[k];
        double uaz1 = (t1 * A3(o->uavg1, j, i, k) + t2 * A3(o->uavg1, j, i, k - 1));
        double uaz2 = (t1 * A3(o->uavg2, j, i, k) + t2 * A3(o->uavg2, j, i, k - 1));
        double vaz1 = (t1 * A3(o->vavg1, j, i, k) + t2 * A3(o->vavg1, j, i, k - 1));
        double vaz2 = (t1 * A3(o->vavg2, j, i, k) + t2 * A3(o->vavg2, j, i, k - 1));
        double ps = A2(o->psa, j, i);
        double f1 = d_half * ul * (A3(o->uavg2, j, i, k) + A3(o->uavg1, j, i, k)) / ps;
        double f2 = d_half * ul * (A3(o->vavg2, j, i, k) + A3(o->vavg1, j, i, k)) / ps;
        double fx1 = (d_one + f1) * A3(f, j - 1, i, k) + (d_one - f1) * A3(f, j, i, k);
        double fx2 = (d_one + f1) * A3(f, j, i, k) + (d_one - f1) * A3(f, j + 1, i, k);
        double fy1 = (d_one + f2) * A3(f, j, i - 1, k) + (d_one - f2) * A3(f, j, i, k);
        double fy2 = (d_one + f2) * A3(f, j, i, k) + (d_one - f2) * A3(f, j, i + 1, k);
        if (!o->cfg.upstream_mode) {  /* centred (:323-332, :414-423, :443-446, :533-542, :625-634) */
          fx1 = A3(f, j - 1, i, k) + A3(f, j, i, k);
          fx2 = A3(f, j, i, k) + A3(f, j + 1, i, k);
          fy1 = A3(f, j, i - 1, k) + A3(f, j, i, k);
          fy2 = A3(f, j, i, k) + A3(f, j, i + 1, k);
        }
        A3(ften, j, i, k) = A3(ften, j, i, k) - A2(o->xmsf, j, i) * (uaz2 * fx2 - uaz1 * fx1 + vaz2 * fy2 - vaz1 * fy1);
      }
}

/* vadv3d ind = 0 (Main/mod_advection.F90:744-766): pp (nk = kz) and w (nk = kz+1) */
static void nh_vadv3d_lin(orc_t* o, const double* f, double* ften, int full) {
  int kz = o->kz;
  for (int i = o->ici1; i <= o->ici2; i++)
    for (int j = o->jci1; j <= o->jci2; j++) {
      if (!full) {
        for (int k = 2; k <= kz; k++) {
          double fx = A3(o->qdot, j, i, k) * (o->twt1[k] * A3(f, j, i, k) + o->twt2[k] * A3(f, j, i, k - 1));
          A3(ften, j, i, k - 1) = A3(ften, j, i, k - 1) - fx * o->xds[k - 1];
          A3(ften, j, i, k) = A3(ften, j, i, k) + fx * o->xds[k];
        }
      } else {
        for (int k = 1; k <= kz; k++) {
          double qq = d_half * (A3(o->qdot, j, i, k) + A3(o->qdot, j, i, k + 1));
          double fx = qq * ((A3(f, j, i, k) + A3(f, j, i, k + 1)));
          A3(ften, j, i, k + 1) = A3(ften, j, i, k + 1) + fx * o->dds[k + 1];
          A3(ften, j, i, k) = A3(ften, j, i, k) - fx * o->dds[k];
        }
      }
    }
}

/* potential temperature advection of the NH core, ithadv = 1 (Main/mod_tendency.F90:98,128-129:
 * ithadv is reset to 0 only for idynamic = 1, so every idynamic = 2 run takes this branch,
 * :1347-1356): th = atmx%t*(p00/atm1%pr)**rovcp, tha = th*p*, exchange(th,1), hadvt of th and
 * vadv3d ind = 0 of tha into thten */
#define NH_P00 1.000000e5                              /* Share/mod_constants.F90:229 */
static void nh_theta_advection(orc_t* o) {
  int kz = o->kz;
  memset(o->thten, 0, sizeof(double) * o->plane * kz);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(o->th, j, i, k) = A3(o->xt, j, i, k) * pow(NH_P00 / A3(o->pr1, j, i, k), c_rovcp);
        A3(o->tha, j, i, k) = A3(o->th, j, i, k) * A2(o->psa, j, i);
      }
  xch(o, o->th, kz, 1, 0);
  hadv_scalar(o, o->th, o->thten, 1);          /* hadv(thten,th) -> hadvt */
  nh_vadv3d_lin(o, o->tha, o->thten, 0);       /* vadv(thten,tha,kz,0) */
}

/* advection NH (Main/mod_tendency.F90:1270-1392) */
static int nh_advection(orc_t* o) {
  int bad = 0;
  start_advect(o);
  nh_hadvuv(o);
  vadvuv(o);
  hadv_scalar(o, o->xpp, o->ppdyn, 0);        /* hadv3d ind = 0 */
  nh_vadv3d_lin(o, o->a1pp, o->ppdyn, 0);
  nh_hadv3d_w(o, o->xw, o->wdyn);
  nh_vadv3d_lin(o, o->a1w, o->wdyn, 1);
  nh_theta_advection(o);                      /* ithadv = 1, :1347-1356 */
  if (o->cfg.isladvec == 1) {                 /* :1361-1363, 1378-1380, as in advection() */
    bad = sl_advection(o);
    if (o->tend_probe == 3) return bad;     /* test hook: qxdyn holds the semi-Lagrangian terms only */
    vadvqv(o);
  } else {
    hadv_scalar(o, o->xq[0], o->qdyn[0], 2);
    vadvqv(o);
    for (int n = 1; n < o->nqx; n++) hadv_scalar(o, o->xq[n], o->qdyn[n], 0);
  }
  for (int n = 1; n < o->nqx; n++) vadv4d_qx(o, n);
  return bad;
}

/* curvature NH (:1839-1879) */
static void nh_curvature(orc_t* o) {
  for (int k = 1; k <= o->kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double wadot = 0.125 * (A3(o->a1w, j - 1, i - 1, k) + A3(o->a1w, j - 1, i, k) +
                                A3(o->a1w, j, i - 1, k) + A3(o->a1w, j, i, k));
        double wadotp1 = 0.125 * (A3(o->a1w, j - 1, i - 1, k + 1) + A3(o->a1w, j - 1, i, k + 1) +
                                  A3(o->a1w, j, i - 1, k + 1) + A3(o->a1w, j, i, k + 1));
        double wabar = wadot + wadotp1;
        double amfac = wabar * A2(o->rpsda, j, i) * NH_REARTHRAD;
        double uc = A3(o->uc, j, i, k), vc = A3(o->vc, j, i, k);
        double duv = uc * A2(o->dmdy, j, i) - vc * A2(o->dmdx, j, i);
        A3(o->udyn, j, i, k) = A3(o->udyn, j, i, k) + A2(o->coriol, j, i) * vc -
            A2(o->ef, j, i) * A2(o->ddx, j, i) * wabar + A3(o->vmd, j, i, k) * duv - uc * amfac;
        A3(o->vdyn, j, i, k) = A3(o->vdyn, j, i, k) - A2(o->coriol, j, i) * uc +
            A2(o->ef, j, i) * A2(o->ddy, j, i) * wabar - A3(o->umd, j, i, k) * duv - vc * amfac;
      }
}

/* adiabatic NH (:1594-1600, 1606-1671), ithadv = 1, ipptls > 0 */
static void nh_adiabatic(orc_t* o) {
  int kz = o->kz;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->thten, j, i, k) = A3(o->thten, j, i, k) + A3(o->th, j, i, k) * A3(o->cr, j, i, k);
        A3(o->tdyn, j, i, k) = A3(o->tdyn, j, i, k) + A3(o->a1t, j, i, k) * A3(o->thten, j, i, k) / A3(o->tha, j, i, k);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->ppdyn, j, i, k) = A3(o->ppdyn, j, i, k) + A3(o->xpp, j, i, k) * A3(o->cr, j, i, k);
  for (int n = 0; n < o->nqx; n++)              /* :1615-1617, n = 1 .. nqx */
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(o->qdyn[n], j, i, k) = A3(o->qdyn[n], j, i, k) + A3(o->xq[n], j, i, k) * A3(o->cr, j, i, k);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(o->ucc, j, i, k) = A3(o->uc, j, i, k) + A3(o->uc, j, i + 1, k) + A3(o->uc, j + 1, i, k) + A3(o->uc, j + 1, i + 1, k);
        A3(o->vcc, j, i, k) = A3(o->vc, j, i, k) + A3(o->vc, j, i + 1, k) + A3(o->vc, j + 1, i, k) + A3(o->vc, j + 1, i + 1, k);
      }
  for (int k = 2; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double rofac = (o->dsigma[k - 1] * A3(o->rho0, j, i, k) + o->dsigma[k] * A3(o->rho0, j, i, k - 1)) /
                       (o->dsigma[k - 1] * A3(o->rho1, j, i, k) + o->dsigma[k] * A3(o->rho1, j, i, k - 1));
        double uaq = d_rfour * (o->twt1[k] * A3(o->ucc, j, i, k) + o->twt2[k] * A3(o->ucc, j, i, k - 1));
        double vaq = d_rfour * (o->twt1[k] * A3(o->vcc, j, i, k) + o->twt2[k] * A3(o->vcc, j, i, k - 1));
        A3(o->wdyn, j, i, k) = A3(o->wdyn, j, i, k) +
            (o->twt2[k] * A3(o->xpr, j, i, k - 1) + o->twt1[k] * A3(o->xpr, j, i, k)) * rofac * EGRAV * A2(o->psa, j, i) +
            A2(o->ex, j, i) * (uaq * A2(o->crx, j, i) - vaq * A2(o->cry, j, i)) +
            (uaq * uaq + vaq * vaq) * NH_REARTHRAD * A2(o->rpsa, j, i) +
            A3(o->xw, j, i, k) * (o->twt1[k] * A3(o->cr, j, i, k) + o->twt2[k] * A3(o->cr, j, i, k - 1));
      }
  const double* qcd = qcd_of(o);                /* water loading (:1662-1671): qcd, the load */
  for (int k = 2; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->wdyn, j, i, k) = A3(o->wdyn, j, i, k) - EGRAV * A2(o->psa, j, i) *
            (o->twt2[k] * A3(qcd, j, i, k - 1) + o->twt1[k] * A3(qcd, j, i, k));
}

/* nudge3d on nk levels (Main/mod_bdycod.F90:4218-4406; hefc(ib, min(k,kz)) for kz+1) */
static void nh_nudge3d(orc_t* o, const double* f, const double* b0, const double* bt, double* ften, int nk) {
  double xt = o->xbctime + o->dt;
  for (int k = 1; k <= nk; k++)
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A3(o->fg1, j, i, k) = (A3(b0, j, i, k) + xt * A3(bt, j, i, k)) - A3(f, j, i, k);
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= nk; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          double xf, xg; nudge_coef(o, A2(o->ib_cr, j, i), (k < o->kz) ? k : o->kz, &xf, &xg);
          A3(ften, j, i, k) = relax(A3(ften, j, i, k), xf, xg, A3(o->fg1, j, i, k),
              A3(o->fg1, j - 1, i, k), A3(o->fg1, j + 1, i, k), A3(o->fg1, j, i - 1, k), A3(o->fg1, j, i + 1, k));
        }
}

/* sponge3d on nk levels (Main/mod_bdycod.F90:2926-2994) */
static void nh_sponge3d(orc_t* o, const double* bt, double* ften, int nk) {
  for (int r = 1; r <= 4; r++)
    for (int k = 1; k <= nk; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          if (A2(o->rg_cr, j, i) != r) continue;
          int ib = A2(o->ib_cr, j, i);
          A3(ften, j, i, k) = o->wgtx[ib] * A3(ften, j, i, k) + (d_one - o->wgtx[ib]) * A3(bt, j, i, k);
        }
}

/* diffu_x3d / diffu_x3df on nk levels with coefficient xk (Main/mod_diffusion.F90:523-790) */
static void nh_diffu_xk(orc_t* o, double* ften, const double* f, const double* xk, int nk, double fac) {
  if (o->cfg.idiffu == 3) { diffu_x6(o, ften, f, nk, fac); return; }
  if (o->cfg.idiffu == 2) {
    for (int k = 1; k <= nk; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(ften, j, i, k) = A3(ften, j, i, k) + fac * A3(xk, j, i, k) *
              (o4_c1 * (A3(f, j + 1, i, k) + A3(f, j - 1, i, k) + A3(f, j, i + 1, k) + A3(f, j, i - 1, k)) +
               o4_c2 * (A3(f, j + 1, i + 1, k) + A3(f, j - 1, i - 1, k) + A3(f, j - 1, i + 1, k) + A3(f, j + 1, i - 1, k)) +
               o4_c3 * A3(f, j, i, k));
    return;
  }
  for (int k = 1; k <= nk; k++)
    for (int i = o->icii1; i <= o->icii2; i++)
      for (int j = o->jcii1; j <= o->jcii2; j++)
        A3(ften, j, i, k) = A3(ften, j, i, k) - fac * A3(xk, j, i, k) *
            (z4_c1 * (A3(f, j + 2, i, k) + A3(f, j - 2, i, k) + A3(f, j, i + 2, k) + A3(f, j, i - 2, k)) +
             z4_c2 * (A3(f, j + 1, i, k) + A3(f, j - 1, i, k) + A3(f, j, i + 1, k) + A3(f, j, i - 1, k)) +
             z4_c3 * A3(f, j, i, k));
#define LAP2(J, I) \
  A3(ften, J, I, k) = A3(ften, J, I, k) + fac * A3(xk, J, I, k) * \
      (z4_c1 * (A3(f, (J) + 1, I, k) + A3(f, (J) - 1, I, k) + A3(f, J, (I) + 1, k) + A3(f, J, (I) - 1, k)) + \
       z4_c2 * A3(f, J, I, k))
  if (o->bl) for (int k = 1; k <= nk; k++) for (int i = o->ici1; i <= o->ici2; i++) LAP2(o->jci1, i);
  if (o->br) for (int k = 1; k <= nk; k++) for (int i = o->ici1; i <= o->ici2; i++) LAP2(o->jci2, i);
  if (o->bb) for (int k = 1; k <= nk; k++) for (int j = o->jci1; j <= o->jci2; j++) LAP2(j, o->ici1);
  if (o->bt) for (int k = 1; k <= nk; k++) for (int j = o->jci1; j <= o->jci2; j++) LAP2(j, o->ici2);
#undef LAP2
}

/* the global cross grid (Main/mpplib/mod_mppparam.F90:1486-1516): njcross / nicross points, and
 * its interior jci / ici range (every point in a periodic direction) */
static int njcross(const orc_t* o) { return o->cfg.i_band ? o->jx : o->jx - 1; }
static int nicross(const orc_t* o) { return o->cfg.i_crm ? o->iy : o->iy - 1; }
static int gcj1(const orc_t* o) { return o->cfg.i_band ? 1 : 2; }
static int gcj2(const orc_t* o) { return o->cfg.i_band ? o->jx : o->jx - 2; }
static int gci1(const orc_t* o) { return o->cfg.i_crm ? 1 : 2; }
static int gci2(const orc_t* o) { return o->cfg.i_crm ? o->iy : o->iy - 2; }

/* tau, Main/mod_bdycod.F90:5115-5123 */
static double nh_tau(orc_t* o, double z, double zmax) {
  double rayhd = o->cfg.rayhd;
  if (z > zmax - rayhd) {
    double s = sin((NH_MATHPI * d_half) * (d_one - (zmax - z) / rayhd));
    return o->cfg.rayalpha0 * (s * s);
  }
  return d_zero;
}

/* raydamp3 / raydampqv (cross, coupled bounds) and raydamp3f (toward 0), :5021-5085 */
static void nh_raydamp_x(orc_t* o, const double* z, const double* var, double* vten,
                         const double* b0, const double* bt, int nk) {
  double xt = o->xbctime + o->dt;
  int kmax = (nk < o->cfg.rayndamp) ? nk : o->cfg.rayndamp;
  for (int k = 1; k <= kmax; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double bval = b0 ? (A3(b0, j, i, k) + xt * A3(bt, j, i, k)) : d_zero;
        A3(vten, j, i, k) = A3(vten, j, i, k) + nh_tau(o, A3(z, j, i, k), A3(z, j, i, 1)) * (bval - A3(var, j, i, k));
      }
}

/* raydampuv (dot points, z averaged from the four cross neighbours), :4953-4983 */
static void nh_raydamp_uv(orc_t* o) {
  double xt = o->xbctime + o->dt;
  const double* z = o->z0;
  int kmax = (o->kz < o->cfg.rayndamp) ? o->kz : o->cfg.rayndamp;
  for (int pass = 0; pass < 2; pass++) {
    const double* b0 = pass ? o->vb0 : o->ub0; const double* bt = pass ? o->vbt : o->ubt;
    const double* var = pass ? o->a2v : o->a2u; double* ten = pass ? o->vten : o->uten;
    for (int k = 1; k <= kmax; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          /* CRM: toward 0 (raydampuv_c with sval = d_zero, Main/mod_tendency.F90:467-469) */
          double bval = o->cfg.i_crm ? d_zero : A3(b0, j, i, k) + xt * A3(bt, j, i, k);
          double zz = d_rfour * (A3(z, j, i, k) + A3(z, j - 1, i, k) + A3(z, j, i - 1, k) + A3(z, j - 1, i - 1, k));
          double zm = d_rfour * (A3(z, j, i, 1) + A3(z, j - 1, i, 1) + A3(z, j, i - 1, 1) + A3(z, j - 1, i - 1, 1));
          A3(ten, j, i, k) = A3(ten, j, i, k) + nh_tau(o, zz, zm) * (bval - A3(var, j, i, k));
        }
  }
}

/* upper radiative boundary coefficients, Main/mod_sound.F90:500-543 (computed on the
 * day alarm at the first acoustic step) */
static void nh_tmask(orc_t* o, const double* rpsb) {
  double fi[13], fk[7];
  for (int n = 0; n < 13; n++) fi[n] = d_one;
  fi[0] = d_half; fi[12] = d_half;
  for (int n = 1; n <= 5; n++) fk[n] = d_two;
  fk[0] = d_one; fk[6] = d_one;
  double atot = d_zero, rhontot = d_zero;
  if (o->gfn) {
    /* decomposed: the per-point terms of every tile, summed over the global interior in the
     * single-tile order (i-major), so every tile gets the one-tile sums bit for bit */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double ensq = EGRAV * EGRAV / c_cpd / (A3(o->a2t, j, i, 1) * A2(rpsb, j, i));
        A2(o->s_tr, j, i) = A3(o->rho1, j, i, 1) * sqrt(ensq);
      }
    const double* ga = o->gfn(o->xctx, o->astore, 1);
    const double* gr = o->gfn(o->xctx, o->s_tr, 2);
    for (int i = gci1(o); i <= gci2(o); i++)
      for (int j = gcj1(o); j <= gcj2(o); j++) {
        atot = atot + ga[(size_t)(i - 1) * o->jx + (j - 1)];
        rhontot = rhontot + gr[(size_t)(i - 1) * o->jx + (j - 1)];
      }
  } else {
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        atot = atot + A2(o->astore, j, i);
        double ensq = EGRAV * EGRAV / c_cpd / (A3(o->a2t, j, i, 1) * A2(rpsb, j, i));
        rhontot = rhontot + A3(o->rho1, j, i, 1) * sqrt(ensq);
      }
  }
  /* rnpts = 1/((nicross-2)*(njcross-2)), init_sound :120 (nicross = iy in CRM, njcross = jx in
   * a band: the count then differs from the points summed, as in the reference) */
  double rnpts = d_one / (double)((nicross(o) - 2) * (njcross(o) - 2));
  double abar = atot * rnpts, rhon = rhontot * rnpts;
  double dxmsfb = d_two / o->dxsq / o->cfg.nh_xmsf;
  memset(o->tmask, 0, sizeof(o->tmask));
  for (int kk = 0; kk <= 6; kk++) {
    double rkk = (double)kk;
    for (int ll = 0; ll <= 6; ll++) {
      double rll = (double)ll;
      double xkeff = dxmsfb * sin(NH_MATHPI * rkk / 12.0) * cos(NH_MATHPI * rll / 12.0);
      double xleff = dxmsfb * sin(NH_MATHPI * rll / 12.0) * cos(NH_MATHPI * rkk / 12.0);
      double xkleff = sqrt(xkeff * xkeff + xleff * xleff);
      for (int ii = -6; ii <= 6; ii++) {
        double ri = (double)ii;
        for (int jj = -6; jj <= 6; jj++) {
          double rj = (double)jj;
          o->tmask[jj + 6][ii + 6] = o->tmask[jj + 6][ii + 6] +
              (fi[ii + 6] * fi[jj + 6] * fk[kk] * fk[ll]) / 144.0 *
              cos(2.0 * NH_MATHPI * rkk * ri / 12.0) * cos(2.0 * NH_MATHPI * rll * rj / 12.0) *
              xkleff / (rhon - abar * xkleff);
        }
      }
    }
  }
  o->tmask_valid = 1;
}

/* sound, Main/mod_sound.F90:163-718 */
static int nh_sound(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  const double xgamma = nh_xgamma();
  double dt = o->dt;
  int istep = (int)(dt / o->cfg.nh_dtsmax);
  if (istep < 2) istep = 2;
  if (o->lcount > 0 && istep < 4) istep = 4;
  o->nh_istep = istep;
  double dts = dt / (double)istep;
  double bet = o->cfg.nhbet, xkd = o->cfg.nhxkd;
  double bp = (d_one + bet) * d_half, bm = (d_one - bet) * d_half;
  double bpxbp = bp * bp, bpxbm = bp * bm;
  double* rpsb = o->srpsb;                     /* sound's own 1/psb (same values) */
  double* cu = o->cu; double* cv = o->cv;
  double* pp = o->cpp; double* w = o->cw;
  for (int i = o->ice1; i <= o->ice2; i++)
    for (int j = o->jce1; j <= o->jce2; j++) A2(rpsb, j, i) = d_one / A2(o->psb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(cu, j, i, k) = A3(o->a2u, j, i, k) / A2(o->psdotb, j, i);
        A3(cv, j, i, k) = A3(o->a2v, j, i, k) / A2(o->psdotb, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->uten, j, i, k) = A3(o->uten, j, i, k) * dts;
        A3(o->vten, j, i, k) = A3(o->vten, j, i, k) * dts;
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->cq[0], j, i, k) = A3(o->a2q[0], j, i, k) * A2(rpsb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A3(pp, j, i, k) = A3(o->a2pp, j, i, k) * A2(rpsb, j, i);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->ppten, j, i, k) = A3(o->ppten, j, i, k) * dts;
  for (int k = 1; k <= kp; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A3(w, j, i, k) = A3(o->a2w, j, i, k) * A2(rpsb, j, i);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->wten, j, i, k) = A3(o->wten, j, i, k) * dts;
  /* day alarm (Main/mpplib/mod_timer.F90:306-337): acts at the start and at the first step
   * whose start time reaches the next multiple of a day */
  double tnow = (double)o->lcount * o->dtsec;
  int day_alarm = (o->lcount == 0) || !o->tmask_valid ||
                  (floor(tnow / 86400.0) != floor((tnow - o->dtsec) / 86400.0));
  double cflmax = d_zero;
  if (o->sound_probe == 0) return 0;           /* test hook: the state at sub-step 1's start */
  double* e = o->s_e; double* f = o->s_f; double* wo = o->s_wo; double* spi = o->s_pi;
  double *aa = o->s_aa, *b = o->s_b, *c = o->s_c, *rhs = o->s_rhs, *ca = o->s_ca, *g1 = o->s_g1, *g2 = o->s_g2;
  double *ptend = o->s_ptend, *pxup = o->s_pxup, *pyvp = o->s_pyvp, *tk = o->s_tk, *cc = o->s_cc;
  double *cdd = o->s_cdd, *cj = o->s_cj;
  for (int it = 1; it <= istep; it++) {
    if (it > 1)
      for (int k = 1; k <= kz; k++)
        for (int i = o->ici1; i <= o->ici2; i++)
          for (int j = o->jci1; j <= o->jci2; j++) A3(pp, j, i, k) = A3(pp, j, i, k) + xkd * A3(spi, j, i, k);
    for (int k = 1; k <= kz; k++) {
      int kp1 = (kz < k + 1) ? kz : k + 1, km1 = (1 > k - 1) ? 1 : k - 1;
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++)
          A3(o->cdt, j, i, k) = (A3(pp, j, i, km1) - A3(pp, j, i, kp1)) / (A3(o->pr0, j, i, km1) - A3(o->pr0, j, i, kp1));
    }
    xch(o, o->cdt, kz, 1, 0); xch(o, pp, kz, 1, 0);
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          double rho = d_rfour * (A3(o->rho1, j, i, k) + A3(o->rho1, j - 1, i, k) + A3(o->rho1, j, i - 1, k) + A3(o->rho1, j - 1, i - 1, k));
          double dppdp0 = d_rfour * (A3(o->cdt, j, i, k) + A3(o->cdt, j - 1, i, k) + A3(o->cdt, j, i - 1, k) + A3(o->cdt, j - 1, i - 1, k));
          double chh = d_half * dts / (rho * o->dx) / A2(o->msfd, j, i);
          A3(cu, j, i, k) = A3(cu, j, i, k) - chh * (A3(pp, j, i, k) - A3(pp, j - 1, i, k) + A3(pp, j, i - 1, k) -
                                                     A3(pp, j - 1, i - 1, k) - A3(o->dprddx, j, i, k) * dppdp0);
          A3(cv, j, i, k) = A3(cv, j, i, k) - chh * (A3(pp, j, i, k) - A3(pp, j, i - 1, k) + A3(pp, j - 1, i, k) -
                                                     A3(pp, j - 1, i - 1, k) - A3(o->dprddy, j, i, k) * dppdp0);
        }
    for (int k = 1; k <= kz; k++)
      for (int i = o->idi1; i <= o->idi2; i++)
        for (int j = o->jdi1; j <= o->jdi2; j++) {
          A3(cu, j, i, k) = A3(cu, j, i, k) + A3(o->uten, j, i, k);
          A3(cv, j, i, k) = A3(cv, j, i, k) + A3(o->vten, j, i, k);
        }
    xch(o, cu, kz, 1, 0); xch(o, cv, kz, 1, 0);
    if (it > 1)
      for (int k = 1; k <= kz; k++)
        for (int i = o->ici1; i <= o->ici2; i++)
          for (int j = o->jci1; j <= o->jci2; j++) A3(pp, j, i, k) = A3(pp, j, i, k) - xkd * A3(spi, j, i, k);
    for (int k = 1; k <= kp; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) A3(wo, j, i, k) = A3(w, j, i, k);
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(w, j, i, kp) = d_half * d_rfour * c_regrav *
            ((A3(cv, j, i + 1, kz) + A3(cv, j, i, kz) + A3(cv, j + 1, i + 1, kz) + A3(cv, j + 1, i, kz)) *
                 (A2(o->ht, j, i + 1) - A2(o->ht, j, i - 1)) +
             (A3(cu, j, i + 1, kz) + A3(cu, j, i, kz) + A3(cu, j + 1, i + 1, kz) + A3(cu, j + 1, i, kz)) *
                 (A2(o->ht, j + 1, i) - A2(o->ht, j - 1, i))) /
            (o->dx * A2(o->msfx, j, i));
        A3(e, j, i, kz) = d_zero;
        A3(f, j, i, kz) = A3(w, j, i, kp);
      }
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double pr1 = A3(o->pr1, j, i, 1), rho0 = A3(o->rho0, j, i, 1), ps0 = A2(o->ps0, j, i);
        A3(cc, j, i, 1) = xgamma * pr1 * dts / (o->dx * A2(o->msfx, j, i));
        A3(cdd, j, i, 1) = xgamma * pr1 * rho0 * EGRAV * dts / (ps0 * o->dsigma[1]);
        A3(cj, j, i, 1) = d_half * rho0 * EGRAV * dts;
        A3(pxup, j, i, 1) = 0.0625 * (A3(o->pr0, j + 1, i, 1) - A3(o->pr0, j - 1, i, 1)) *
            (A3(cu, j, i, 1) + A3(cu, j + 1, i, 1) + A3(cu, j, i + 1, 1) + A3(cu, j + 1, i + 1, 1) -
             A3(cu, j, i, 2) - A3(cu, j + 1, i, 2) - A3(cu, j, i + 1, 2) - A3(cu, j + 1, i + 1, 2)) /
            (A3(o->pr0, j, i, 1) - A3(o->pr0, j, i, 2));
        A3(pyvp, j, i, 1) = 0.0625 * (A3(o->pr0, j, i + 1, 1) - A3(o->pr0, j, i - 1, 1)) *
            (A3(cv, j, i, 1) + A3(cv, j + 1, i, 1) + A3(cv, j, i + 1, 1) + A3(cv, j + 1, i + 1, 1) -
             A3(cv, j, i, 2) - A3(cv, j + 1, i, 2) - A3(cv, j, i + 1, 2) - A3(cv, j + 1, i + 1, 2)) /
            (A3(o->pr0, j, i, 1) - A3(o->pr0, j, i, 2));
        A3(ptend, j, i, 1) = A3(o->ppten, j, i, 1) - d_half * A3(cc, j, i, 1) *
            ((A3(cv, j, i + 1, 1) * A2(o->msfd, j, i + 1) - A3(cv, j, i, 1) * A2(o->msfd, j, i) +
              A3(cv, j + 1, i + 1, 1) * A2(o->msfd, j + 1, i + 1) - A3(cv, j + 1, i, 1) * A2(o->msfd, j + 1, i) +
              A3(cu, j + 1, i, 1) * A2(o->msfd, j + 1, i) - A3(cu, j, i, 1) * A2(o->msfd, j, i) +
              A3(cu, j + 1, i + 1, 1) * A2(o->msfd, j + 1, i + 1) - A3(cu, j, i + 1, 1) * A2(o->msfd, j, i + 1)) /
                 A2(o->msfx, j, i) - d_two * (A3(pyvp, j, i, 1) + A3(pxup, j, i, 1)));
        A3(tk, j, i, 1) = (d_half * ps0 * A3(o->t0, j, i, 1)) /
                          (xgamma * A3(o->pr0, j, i, 1) * A3(o->a2t, j, i, 1) * A2(rpsb, j, i));
      }
    for (int k = 2; k <= kz; k++) {
      int kp1 = (k + 1 < kz) ? k + 1 : kz, km1 = k - 1;
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double ps0 = A2(o->ps0, j, i);
          A3(tk, j, i, k) = (d_half * ps0 * A3(o->t0, j, i, k)) /
                            (xgamma * A3(o->pr0, j, i, k) * A3(o->a2t, j, i, k) * A2(rpsb, j, i));
          double rofac = (o->dsigma[km1] * A3(o->rho0, j, i, k) + o->dsigma[k] * A3(o->rho0, j, i, km1)) /
                         (o->dsigma[km1] * A3(o->rho1, j, i, k) + o->dsigma[k] * A3(o->rho1, j, i, km1));
          A3(cc, j, i, k) = xgamma * A3(o->pr1, j, i, k) * dts / (o->dx * A2(o->msfx, j, i));
          A3(cdd, j, i, k) = xgamma * A3(o->pr1, j, i, k) * A3(o->rho0, j, i, k) * EGRAV * dts / (ps0 * o->dsigma[k]);
          A3(cj, j, i, k) = d_half * A3(o->rho0, j, i, k) * EGRAV * dts;
          A3(ca, j, i, k) = EGRAV * dts / (A3(o->pr0, j, i, k) - A3(o->pr0, j, i, km1)) * rofac;
          A3(g1, j, i, k) = d_one - o->dsigma[km1] * A3(tk, j, i, k);
          A3(g2, j, i, k) = d_one + o->dsigma[k] * A3(tk, j, i, km1);
          A3(c, j, i, k) = -A3(ca, j, i, k) * (A3(cdd, j, i, km1) - A3(cj, j, i, km1)) * A3(g2, j, i, k) * bpxbp;
          A3(b, j, i, k) = d_one + A3(ca, j, i, k) * (A3(g1, j, i, k) * (A3(cdd, j, i, k) - A3(cj, j, i, k)) +
                                                      A3(g2, j, i, k) * (A3(cdd, j, i, km1) + A3(cj, j, i, km1))) * bpxbp;
          A3(aa, j, i, k) = -A3(ca, j, i, k) * (A3(cdd, j, i, k) + A3(cj, j, i, k)) * A3(g1, j, i, k) * bpxbp;
          A3(pyvp, j, i, k) = 0.125 * (A3(o->pr0, j, i + 1, k) - A3(o->pr0, j, i - 1, k)) *
              (A3(cv, j, i, km1) + A3(cv, j + 1, i, km1) + A3(cv, j, i + 1, km1) + A3(cv, j + 1, i + 1, km1) -
               A3(cv, j, i, kp1) - A3(cv, j + 1, i, kp1) - A3(cv, j, i + 1, kp1) - A3(cv, j + 1, i + 1, kp1)) /
              (A3(o->pr0, j, i, km1) - A3(o->pr0, j, i, kp1));
          A3(pxup, j, i, k) = 0.125 * (A3(o->pr0, j + 1, i, k) - A3(o->pr0, j - 1, i, k)) *
              (A3(cu, j, i, km1) + A3(cu, j + 1, i, km1) + A3(cu, j, i + 1, km1) + A3(cu, j + 1, i + 1, km1) -
               A3(cu, j, i, kp1) - A3(cu, j + 1, i, kp1) - A3(cu, j, i + 1, kp1) - A3(cu, j + 1, i + 1, kp1)) /
              (A3(o->pr0, j, i, km1) - A3(o->pr0, j, i, kp1));
        }
    }
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(pyvp, j, i, kz) = A3(pyvp, j, i, kz) * d_half;
        A3(pxup, j, i, kz) = A3(pxup, j, i, kz) * d_half;
      }
    for (int k = 2; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          A3(ptend, j, i, k) = A3(o->ppten, j, i, k) - d_half * A3(cc, j, i, k) *
              ((A3(cv, j, i + 1, k) * A2(o->msfd, j, i + 1) - A3(cv, j, i, k) * A2(o->msfd, j, i) +
                A3(cv, j + 1, i + 1, k) * A2(o->msfd, j + 1, i + 1) - A3(cv, j + 1, i, k) * A2(o->msfd, j + 1, i) +
                A3(cu, j + 1, i, k) * A2(o->msfd, j + 1, i) - A3(cu, j, i, k) * A2(o->msfd, j, i) +
                A3(cu, j + 1, i + 1, k) * A2(o->msfd, j + 1, i + 1) - A3(cu, j, i + 1, k) * A2(o->msfd, j, i + 1)) /
                   A2(o->msfx, j, i) - d_two * (A3(pyvp, j, i, k) + A3(pxup, j, i, k)));
          double cdm = A3(cdd, j, i, k - 1), cjm = A3(cj, j, i, k - 1), cdk = A3(cdd, j, i, k), cjk = A3(cj, j, i, k);
          double gg1 = A3(g1, j, i, k), gg2 = A3(g2, j, i, k);
          A3(rhs, j, i, k) = A3(w, j, i, k) + A3(o->wten, j, i, k) + A3(ca, j, i, k) *
              (bpxbm * ((cdm - cjm) * gg2 * A3(wo, j, i, k - 1) -
                        ((cdm + cjm) * gg2 + (cdk - cjk) * gg1) * A3(wo, j, i, k) +
                        (cdk + cjk) * gg1 * A3(wo, j, i, k + 1)) +
               (A3(pp, j, i, k) * gg1 - A3(pp, j, i, k - 1) * gg2) +
               (gg1 * A3(ptend, j, i, k) - gg2 * A3(ptend, j, i, k - 1)) * bp);
        }
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          A3(spi, j, i, k) = A3(pp, j, i, k);
          A3(pp, j, i, k) = A3(pp, j, i, k) + A3(ptend, j, i, k) +
              (A3(cj, j, i, k) * (A3(wo, j, i, k + 1) + A3(wo, j, i, k)) +
               A3(cdd, j, i, k) * (A3(wo, j, i, k + 1) - A3(wo, j, i, k))) * bm;
        }
    for (int k = kz; k >= 2; k--)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double denom = A3(aa, j, i, k) * A3(e, j, i, k) + A3(b, j, i, k);
          A3(e, j, i, k - 1) = -A3(c, j, i, k) / denom;
          A3(f, j, i, k - 1) = (A3(rhs, j, i, k) - A3(f, j, i, k) * A3(aa, j, i, k)) / denom;
        }
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A2(o->wpval, j, i) = d_zero;
    if (o->cfg.ifupr == 1) {
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double denom = (A3(cdd, j, i, 1) + A3(cj, j, i, 1)) * bp;
          A2(o->estore, j, i) = A3(pp, j, i, 1) + A3(f, j, i, 1) * denom;
          A2(o->astore, j, i) = denom * A3(e, j, i, 1) + (A3(cj, j, i, 1) - A3(cdd, j, i, 1)) * bp;
        }
      if (day_alarm && it == 1) nh_tmask(o, rpsb);
      int ilo = 2, ihi = nicross(o) - 1, jlo = 2, jhi = njcross(o) - 1;  /* icross1+1 .. icross2-1 */
      /* decomposed: the whole-domain estore (Main/mod_sound.F90:496-497) */
      const double* ge = o->gfn ? o->gfn(o->xctx, o->estore, 0) : NULL;
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double acc = A2(o->wpval, j, i);
          for (int nsi = -6; nsi <= 6; nsi++) {
            int inn = i + nsi; inn = (inn < ilo) ? ilo : (inn > ihi ? ihi : inn);
            for (int nsj = -6; nsj <= 6; nsj++) {
              int jnn = j + nsj; jnn = (jnn < jlo) ? jlo : (jnn > jhi ? jhi : jnn);
              const double ev = ge ? ge[(size_t)(inn - 1) * o->jx + (jnn - 1)] : A2(o->estore, jnn, inn);
              acc = acc + ev * o->tmask[nsj + 6][nsi + 6];
            }
          }
          A2(o->wpval, j, i) = acc;
        }
    }
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(w, j, i, 1) = A2(o->wpval, j, i);
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        for (int k = 1; k <= kz; k++)
          A3(w, j, i, k + 1) = A3(e, j, i, k) * A3(w, j, i, k) + A3(f, j, i, k);
    /* zero-gradient w on the boundary cross points (:586-617) */
    if (o->bb) {
      for (int k = 1; k <= kp; k++) for (int j = o->jci1; j <= o->jci2; j++) A3(w, j, o->ice1, k) = A3(w, j, o->ici1, k);
      if (o->bl) for (int k = 1; k <= kp; k++) A3(w, o->jce1, o->ice1, k) = A3(w, o->jci1, o->ici1, k);
      if (o->br) for (int k = 1; k <= kp; k++) A3(w, o->jce2, o->ice1, k) = A3(w, o->jci2, o->ici1, k);
    }
    if (o->bt) {
      for (int k = 1; k <= kp; k++) for (int j = o->jci1; j <= o->jci2; j++) A3(w, j, o->ice2, k) = A3(w, j, o->ici2, k);
      if (o->bl) for (int k = 1; k <= kp; k++) A3(w, o->jce1, o->ice2, k) = A3(w, o->jci1, o->ici2, k);
      if (o->br) for (int k = 1; k <= kp; k++) A3(w, o->jce2, o->ice2, k) = A3(w, o->jci2, o->ici2, k);
    }
    if (o->bl) for (int k = 1; k <= kp; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(w, o->jce1, i, k) = A3(w, o->jci1, i, k);
    if (o->br) for (int k = 1; k <= kp; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(w, o->jce2, i, k) = A3(w, o->jci2, i, k);
    /* CFL check (:622-682) */
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          A3(o->s_ucrs, j, i, k) = A3(cu, j, i, k) + A3(cu, j, i + 1, k) + A3(cu, j + 1, i, k) + A3(cu, j + 1, i + 1, k);
          A3(o->s_vcrs, j, i, k) = A3(cv, j, i, k) + A3(cv, j, i + 1, k) + A3(cv, j + 1, i, k) + A3(cv, j + 1, i + 1, k);
        }
    double cfl = d_zero;
    for (int k = kz; k >= 2; k--)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double sigdot = -A3(o->rhof0, j, i, k) * EGRAV * A3(w, j, i, k) / A2(o->ps0, j, i) -
              o->sigma[k] * (A2(o->dpsdxm, j, i) * (o->twt1[k] * A3(o->s_ucrs, j, i, k) + o->twt2[k] * A3(o->s_ucrs, j, i, k - 1)) +
                             A2(o->dpsdym, j, i) * (o->twt1[k] * A3(o->s_vcrs, j, i, k) + o->twt2[k] * A3(o->s_vcrs, j, i, k - 1)));
          double check = fabs(sigdot) * dt / (o->dsigma[k] + o->dsigma[k - 1]);
          cfl = dmax(check, cfl);
        }
    if (cfl > cflmax) cflmax = cfl;
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double ppold = A3(spi, j, i, k);
          double rho0 = A3(o->rho0, j, i, k);
          double cddtmp = xgamma * A3(o->pr1, j, i, k) * rho0 * EGRAV * dts / (A2(o->ps0, j, i) * o->dsigma[k]);
          double cjtmp = rho0 * EGRAV * dts * d_half;
          A3(pp, j, i, k) = A3(pp, j, i, k) +
              (cjtmp * (A3(w, j, i, k + 1) + A3(w, j, i, k)) + cddtmp * (A3(w, j, i, k + 1) - A3(w, j, i, k))) * bp;
          A3(spi, j, i, k) = A3(pp, j, i, k) - ppold - A3(o->ppten, j, i, k);
          double cpm = c_cpd * (d_one + 0.80 * A3(o->cq[0], j, i, k));
          double dpterm = A2(o->psb, j, i) * (A3(pp, j, i, k) - ppold) / (cpm * A3(o->rho1, j, i, k));
          A3(o->a2t, j, i, k) = A3(o->a2t, j, i, k) + o->cfg.gnu1 * dpterm;
          A3(o->a1t, j, i, k) = A3(o->a1t, j, i, k) + dpterm;
        }
    if (o->sound_probe == it) { o->nh_cfl = cflmax; return 0; }   /* test hook: stop here */
  }
  o->nh_cfl = cflmax;
  /* time filters (:686-702) */
  double g1f = o->cfg.gnu1, g2f = o->cfg.gnu2;
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(cu, j, i, k) = A2(o->psdotb, j, i) * A3(cu, j, i, k);
        A3(cv, j, i, k) = A2(o->psdotb, j, i) * A3(cv, j, i, k);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double d = g1f * (A3(cu, j, i, k) + A3(o->a2u, j, i, k) - d_two * A3(o->a1u, j, i, k));
        A3(o->a2u, j, i, k) = A3(o->a1u, j, i, k) + d;
        A3(o->a1u, j, i, k) = A3(cu, j, i, k);
        d = g1f * (A3(cv, j, i, k) + A3(o->a2v, j, i, k) - d_two * A3(o->a1v, j, i, k));
        A3(o->a2v, j, i, k) = A3(o->a1v, j, i, k) + d;
        A3(o->a1v, j, i, k) = A3(cv, j, i, k);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(pp, j, i, k) = A2(o->psb, j, i) * A3(pp, j, i, k);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g1f * (A3(pp, j, i, k) + A3(o->a2pp, j, i, k) - d_two * A3(o->a1pp, j, i, k));
        A3(o->a2pp, j, i, k) = A3(o->a1pp, j, i, k) + d;
        A3(o->a1pp, j, i, k) = A3(pp, j, i, k);
      }
  size_t nw = o->plane * (size_t)kp;
  for (size_t q = 0; q < nw; q++) if (fabs(w[q]) < DLOWVAL) w[q] = d_zero;
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(w, j, i, k) = A2(o->psb, j, i) * A3(w, j, i, k);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g2f * (A3(w, j, i, k) + A3(o->a2w, j, i, k) - d_two * A3(o->a1w, j, i, k));
        A3(o->a2w, j, i, k) = A3(o->a1w, j, i, k) + d;
        A3(o->a1w, j, i, k) = A3(w, j, i, k);
      }
  for (size_t q = 0; q < nw; q++) if (fabs(o->a2w[q]) < DLOWVAL) o->a2w[q] = d_zero;
  for (size_t q = 0; q < nw; q++) if (fabs(o->a1w[q]) < DLOWVAL) o->a1w[q] = d_zero;
  return (cflmax > d_one) ? 1 : 0;
}

/* The hydrometeors of nqx = 5 beyond qc (qi, qr, qs: n = 2 .. nqx-1 here): their sums
 * qxten + qxdyn + qxphy (Main/mod_tendency.F90:332-335, n = iqfrst..iqlst; qc's is summed with
 * t and qv at each core's place) */
static void qx_sums(orc_t* o) {
  for (int n = 2; n < o->nqx; n++)
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(o->qten[n], j, i, k) = A3(o->qten[n], j, i, k) + A3(o->qdyn[n], j, i, k) + A3(o->phyx[n - 2], j, i, k);
}
/* forecast of every species, the exchange of atmc%qx and the negative-moisture fix, :375-393 */
static void qx_forecast_fix(orc_t* o) {
  int kz = o->kz;
  for (int n = 0; n < o->nqx; n++) {
    for (int k = 1; k <= kz; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) A3(o->cq[n], j, i, k) = A3(o->a2q[n], j, i, k);
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          A3(o->cq[n], j, i, k) = A3(o->cq[n], j, i, k) + o->dt * A3(o->qten[n], j, i, k);
  }
  for (int n = 0; n < o->nqx; n++) xch(o, o->cq[n], kz, 1, 0);
  for (int n = 0; n < o->nqx; n++)
    for (int k = 1; k <= kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++)
          if (A3(o->cq[n], j, i, k) < d_zero) {
            double s = 0.0;
            for (int ii = i - 1; ii <= i + 1; ii++)
              for (int jj = j - 1; jj <= j + 1; jj++) s = s + fabs(A3(o->cq[n], jj, ii, k));
            A3(o->cq[n], j, i, k) = 0.01 * s / 9.0;
          }
}
/* filter_raw_4d of the hydrometeors n = iqfrst..iqlst with the zero floor, :426-427 */
static void qx_raw_filter(orc_t* o) {
  double g2 = o->cfg.gnu2, beta = 0.53;
  for (int n = 1; n < o->nqx; n++)
    for (int k = 1; k <= o->kz; k++)
      for (int i = o->ici1; i <= o->ici2; i++)
        for (int j = o->jci1; j <= o->jci2; j++) {
          double d = g2 * (A3(o->cq[n], j, i, k) + A3(o->a2q[n], j, i, k) - d_two * A3(o->a1q[n], j, i, k));
          A3(o->a2q[n], j, i, k) = A3(o->a1q[n], j, i, k) + beta * d;
          A3(o->a1q[n], j, i, k) = A3(o->cq[n], j, i, k) + (beta - d_one) * d;
          if (A3(o->a2q[n], j, i, k) < d_zero) A3(o->a2q[n], j, i, k) = d_zero;
          if (A3(o->a1q[n], j, i, k) < d_zero) A3(o->a1q[n], j, i, k) = d_zero;
        }
}

/* tend, non-hydrostatic (Main/mod_tendency.F90:212-616 with idynamic = 2) */
/* UW PBL TKE in tend (ibltyp = 2), both cores: hadv3d ind = 1 of atm1%tke and vadv3d of
 * tke*p* (Main/mod_tendency.F90:1414-1425, at the end of advection, with its uavg and the
 * start-of-step p*), diffu_x3df with nuk (:1545-1548), then tketen, the forecast with the
 * tkemin floor and filter_ra_3d (:515-544).  Nothing else in tend reads or writes the TKE, and
 * its inputs are unchanged between those points, so the three parts run here in sequence. */
static void tke_tend(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  memset(o->tkedyn, 0, sizeof(double) * o->plane * kp);
  nh_hadv3d_w(o, o->a1tke, o->tkedyn);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A3(o->tkeps, j, i, k) = A3(o->a1tke, j, i, k) * A2(o->psa, j, i);
  nh_vadv3d_lin(o, o->tkeps, o->tkedyn, 1);
  nh_diffu_xk(o, o->tkedyn, o->a2tke, o->xkcf, kp, o->cfg.nuk);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double ten = (d_zero + A3(o->tkedyn, j, i, k) * A2(o->rpsa, j, i)) + A3(o->tkephy, j, i, k);
        double v = A3(o->a2tke, j, i, k) + o->dt * ten;
        A3(o->ctke, j, i, k) = (v > o->cfg.tkemin) ? v : o->cfg.tkemin;
      }
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = o->cfg.gnu2 * (A3(o->ctke, j, i, k) + A3(o->a2tke, j, i, k) - d_two * A3(o->a1tke, j, i, k));
        A3(o->a2tke, j, i, k) = A3(o->a1tke, j, i, k) + d;
        A3(o->a1tke, j, i, k) = A3(o->ctke, j, i, k);
      }
}

static int nh_tend(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  size_t n3 = o->plane * (size_t)kz, n3p = o->plane * (size_t)kp;
  nh_surface_pressures(o);
  nh_decouple(o);
  nh_compute_omega(o);
  nh_mkslice(o);
  slice_export(o);
  nh_calc_coeff(o);
  memset(o->tten, 0, n3 * 8); memset(o->tdyn, 0, n3 * 8);
  memset(o->uten, 0, n3 * 8); memset(o->udyn, 0, n3 * 8);
  memset(o->vten, 0, n3 * 8); memset(o->vdyn, 0, n3 * 8);
  for (int n = 0; n < o->nqx; n++) { memset(o->qten[n], 0, n3 * 8); memset(o->qdyn[n], 0, n3 * 8); }
  memset(o->ppten, 0, n3 * 8); memset(o->ppdyn, 0, n3 * 8);
  memset(o->wten, 0, n3p * 8); memset(o->wdyn, 0, n3p * 8);
  int slbad = nh_advection(o);
  if (o->cfg.ibltyp == 2) tke_tend(o);
  nh_curvature(o);
  nh_adiabatic(o);
  /* boundary (:1462-1501) */
  if (o->cfg.iboudy == 4) {
    sponge_all(o);
    nh_sponge3d(o, o->ppbt, o->ppten, kz);
    nh_sponge3d(o, o->wwbt, o->wten, kp);
  } else if (o->cfg.iboudy == 1 || o->cfg.iboudy == 5) {   /* 2, 3: no relaxation (:1494-1500) */
    boundary(o);
    nh_nudge3d(o, o->a2pp, o->ppb0, o->ppbt, o->ppdyn, kz);
    nh_nudge3d(o, o->a2w, o->wwb0, o->wwbt, o->wdyn, kp);
  }
  /* diffusion (:1515-1538) */
  diffu_d(o);
  diffu_x(o, o->tdyn, o->tb3d, d_one);
  for (int n = 0; n < o->nqx; n++) diffu_x(o, o->qdyn[n], o->qb3d[n], d_one);   /* diffu_x4d 1..nqx */
  nh_diffu_xk(o, o->ppdyn, o->ppb3d, o->xkc, kz, d_one);
  nh_diffu_xk(o, o->wdyn, o->wb3d, o->xkcf, kp, d_one);
  /* sums (:285-314, 332-335) with the host's pc_physic tendencies (phy, 0 unless put) */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->tten, j, i, k) = A3(o->tten, j, i, k) + A3(o->tdyn, j, i, k) + A3(o->phy[0], j, i, k);
        A3(o->qten[0], j, i, k) = A3(o->qten[0], j, i, k) + A3(o->qdyn[0], j, i, k) + A3(o->phy[1], j, i, k);
      }
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->wten, j, i, k) = A3(o->wten, j, i, k) + A3(o->wdyn, j, i, k) + A3(o->phy[6], j, i, k);
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->ppten, j, i, k) = A3(o->ppten, j, i, k) + A3(o->ppdyn, j, i, k) + A3(o->phy[5], j, i, k);
        A3(o->qten[1], j, i, k) = A3(o->qten[1], j, i, k) + A3(o->qdyn[1], j, i, k) + A3(o->phy[2], j, i, k);
      }
  qx_sums(o);
  /* condtq (:336-350, ipptls = 1 only) is physics: stubbed, tphy = qxphy = 0 */
  if (o->cfg.ipptls == 1)
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->tten, j, i, k) = A3(o->tten, j, i, k) + 0.0;
        A3(o->qten[0], j, i, k) = A3(o->qten[0], j, i, k) + 0.0;
        A3(o->qten[1], j, i, k) = A3(o->qten[1], j, i, k) + 0.0;
      }
  if (o->cfg.ifrayd == 1 && !o->cfg.i_crm) {  /* :356-364 (not in CRM mode) */
    nh_raydamp_x(o, o->z0, o->a2t, o->tten, o->tb0, o->tbt, kz);
    nh_raydamp_x(o, o->z0, o->a2q[0], o->qten[0], o->qb0, o->qbt, kz);
  }
  /* forecast t, qx (:368-393) */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->ct, j, i, k) = A3(o->a2t, j, i, k) + o->dt * A3(o->tten, j, i, k);
  qx_forecast_fix(o);
  for (int k = 1; k <= kz; k++)                                     /* :404-411 */
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->uten, j, i, k) = A3(o->uten, j, i, k) + A3(o->udyn, j, i, k) + A3(o->phy[3], j, i, k);
        A3(o->vten, j, i, k) = A3(o->vten, j, i, k) + A3(o->vdyn, j, i, k) + A3(o->phy[4], j, i, k);
      }
  /* time filters t, qx (:422-427) */
  double g1 = o->cfg.gnu1, beta = 0.53;
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g1 * (A3(o->ct, j, i, k) + A3(o->a2t, j, i, k) - d_two * A3(o->a1t, j, i, k));
        A3(o->a2t, j, i, k) = A3(o->a1t, j, i, k) + d;
        A3(o->a1t, j, i, k) = A3(o->ct, j, i, k);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g1 * (A3(o->cq[0], j, i, k) + A3(o->a2q[0], j, i, k) - d_two * A3(o->a1q[0], j, i, k));
        A3(o->a2q[0], j, i, k) = dmax(A3(o->a1q[0], j, i, k) + beta * d, MINQQ * A2(o->psa, j, i));
        A3(o->a1q[0], j, i, k) = dmax(A3(o->cq[0], j, i, k) + (beta - d_one) * d, MINQQ * A2(o->psb, j, i));
      }
  qx_raw_filter(o);                                                 /* filter_raw_4d */
  /* Rayleigh damping of u, v, pp, w and decoupling of the tendencies (:466-499) */
  if (o->cfg.ifrayd == 1) {
    nh_raydamp_uv(o);
    /* CRM: pp toward 0 (raydamp3f, :468-470), else toward its boundary values (raydamp3) */
    if (o->cfg.i_crm) nh_raydamp_x(o, o->z0, o->a2pp, o->ppten, NULL, NULL, kz);
    else nh_raydamp_x(o, o->z0, o->a2pp, o->ppten, o->ppb0, o->ppbt, kz);
    nh_raydamp_x(o, o->zf0, o->a2w, o->wten, NULL, NULL, kp);
  }
  for (int k = 1; k <= kz; k++)
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->uten, j, i, k) = A3(o->uten, j, i, k) * A2(o->rpsda, j, i);
        A3(o->vten, j, i, k) = A3(o->vten, j, i, k) * A2(o->rpsda, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->ppten, j, i, k) = A3(o->ppten, j, i, k) * A2(o->rpsa, j, i);
  for (int k = 1; k <= kp; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) A3(o->wten, j, i, k) = A3(o->wten, j, i, k) * A2(o->rpsa, j, i);
  int err = nh_sound(o);
  /* atm2%pr (:507-513) feeds only physics: skipped */
  o->lcount += 1;
  if (o->lcount == 2) o->dt = d_two * o->dtsec;
  o->ptntot = 0; o->pt2tot = 0;
  if (err) return err;
  return slbad ? 2 : 0;
}

/* tend, Main/mod_tendency.F90:212-726 (hydrostatic, physics stubbed) */
int orc_tend(orc_t* o) {
  if (o->nh) return nh_tend(o);
  int kz = o->kz;
  size_t n3 = o->plane * (size_t)kz;
  surface_pressures(o);
  decouple(o);
  compute_omega(o);
  mkslice(o);
  slice_export(o);
  new_pressure(o);
  calc_coeff(o);
  /* init_tendencies, :1227-1268 (total/dynamic/physic components all zero) */
  memset(o->tten, 0, n3 * 8); memset(o->tdyn, 0, n3 * 8);
  memset(o->uten, 0, n3 * 8); memset(o->udyn, 0, n3 * 8);
  memset(o->vten, 0, n3 * 8); memset(o->vdyn, 0, n3 * 8);
  for (int n = 0; n < o->nqx; n++) { memset(o->qten[n], 0, n3 * 8); memset(o->qdyn[n], 0, n3 * 8); }
  int slbad = advection(o);
  if (o->tend_probe == 3 && o->cfg.isladvec == 1) return 0;
  if (o->cfg.ibltyp == 2) tke_tend(o);
  curvature(o);
  adiabatic(o);
  boundary(o);
  /* physical_parametrizations: the host's pc_physic tendencies (phy, 0 unless put) */
  diffu_d(o);
  diffu_x(o, o->tdyn, o->tb3d, d_one);
  for (int n = 0; n < o->nqx; n++) diffu_x(o, o->qdyn[n], o->qb3d[n], d_one);   /* diffu_x4d 1..nqx */
  /* sums, :285-294 and :332-349 (tphy, qxphy from the host; the SUBEX condtq terms = 0, ipptls = 1) */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        A3(o->tten, j, i, k) = A3(o->tten, j, i, k) + A3(o->tdyn, j, i, k) + A3(o->phy[0], j, i, k);
        A3(o->qten[0], j, i, k) = A3(o->qten[0], j, i, k) + A3(o->qdyn[0], j, i, k) + A3(o->phy[1], j, i, k);
        A3(o->qten[1], j, i, k) = A3(o->qten[1], j, i, k) + A3(o->qdyn[1], j, i, k) + A3(o->phy[2], j, i, k);
        if (o->cfg.ipptls == 1) {
          A3(o->tten, j, i, k) = A3(o->tten, j, i, k) + 0.0;
          A3(o->qten[0], j, i, k) = A3(o->qten[0], j, i, k) + 0.0;
          A3(o->qten[1], j, i, k) = A3(o->qten[1], j, i, k) + 0.0;
        }
      }
  qx_sums(o);
  /* forecast t, qx, :368-393 */
  for (int k = 1; k <= kz; k++)
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++)
        A3(o->ct, j, i, k) = A3(o->a2t, j, i, k) + o->dt * A3(o->tten, j, i, k);
  qx_forecast_fix(o);
  pressure_gradient_force(o);
  for (int k = 1; k <= kz; k++)                                     /* :404-411 */
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->uten, j, i, k) = A3(o->uten, j, i, k) + A3(o->udyn, j, i, k) + A3(o->phy[3], j, i, k);
        A3(o->vten, j, i, k) = A3(o->vten, j, i, k) + A3(o->vdyn, j, i, k) + A3(o->phy[4], j, i, k);
      }
  /* test hook: every tendency summed, the t / qx forecasts (and their negative fix) in ct / cq,
   * atm1 / atm2 and p* not yet filtered */
  if (o->tend_probe == 1) return 0;
  /* time filters, :419-427, Main/mod_timefilter.F90 */
  double g1 = o->cfg.gnu1, beta = 0.53;
  for (int i = o->ici1; i <= o->ici2; i++)                          /* filter_ra_2d */
    for (int j = o->jci1; j <= o->jci2; j++) {
      double d = g1 * (A2(o->psc, j, i) + A2(o->psb, j, i) - d_two * A2(o->psa, j, i));
      A2(o->psb, j, i) = A2(o->psa, j, i) + d;
      A2(o->psa, j, i) = A2(o->psc, j, i);
    }
  for (int k = 1; k <= kz; k++)                                     /* filter_ra_3d */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g1 * (A3(o->ct, j, i, k) + A3(o->a2t, j, i, k) - d_two * A3(o->a1t, j, i, k));
        A3(o->a2t, j, i, k) = A3(o->a1t, j, i, k) + d;
        A3(o->a1t, j, i, k) = A3(o->ct, j, i, k);
      }
  for (int k = 1; k <= kz; k++)                                     /* filter_raw_qv */
    for (int i = o->ici1; i <= o->ici2; i++)
      for (int j = o->jci1; j <= o->jci2; j++) {
        double d = g1 * (A3(o->cq[0], j, i, k) + A3(o->a2q[0], j, i, k) - d_two * A3(o->a1q[0], j, i, k));
        A3(o->a2q[0], j, i, k) = dmax(A3(o->a1q[0], j, i, k) + beta * d, MINQQ * A2(o->psa, j, i));
        A3(o->a1q[0], j, i, k) = dmax(A3(o->cq[0], j, i, k) + (beta - d_one) * d, MINQQ * A2(o->psb, j, i));
      }
  qx_raw_filter(o);                                                 /* filter_raw_4d */
  for (int k = 1; k <= kz; k++)                                     /* :433-440 */
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        A3(o->cu, j, i, k) = A3(o->a2u, j, i, k) + o->dt * A3(o->uten, j, i, k);
        A3(o->cv, j, i, k) = A3(o->a2v, j, i, k) + o->dt * A3(o->vten, j, i, k);
      }
  for (int k = 1; k <= kz; k++)                                     /* filter_ra_uv */
    for (int i = o->idi1; i <= o->idi2; i++)
      for (int j = o->jdi1; j <= o->jdi2; j++) {
        double d = g1 * (A3(o->cu, j, i, k) + A3(o->a2u, j, i, k) - d_two * A3(o->a1u, j, i, k));
        A3(o->a2u, j, i, k) = A3(o->a1u, j, i, k) + d;
        A3(o->a1u, j, i, k) = A3(o->cu, j, i, k);
        d = g1 * (A3(o->cv, j, i, k) + A3(o->a2v, j, i, k) - d_two * A3(o->a1v, j, i, k));
        A3(o->a2v, j, i, k) = A3(o->a1v, j, i, k) + d;
        A3(o->a1v, j, i, k) = A3(o->cv, j, i, k);
      }
  /* test hook: the state splitf starts from (every time filter applied) */
  if (o->tend_probe == 2) return 0;
  splitf(o);
  /* rcmtimer%advance and dt switch, :608-616 */
  o->lcount += 1;
  if (o->lcount == 2) o->dt = d_two * o->dtsec;
  /* NaN / CFL check, :624-703; departure point beyond one cell, Main/mod_sladvection.F90:149-154 */
  if (isnan(o->ptntot)) return 1;
  if (slbad) return 2;
  return 0;
}

/* bdyuv, Main/mod_bdycod.F90:896-1094 (time-dependent branch) */
static void bdyuv(orc_t* o, double xt) {
  int kz = o->kz;
  if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
    SI(o->wui, i, k) = A3(o->a1u, o->jdi1, i, k); SI(o->wvi, i, k) = A3(o->a1v, o->jdi1, i, k); }
  if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
    SI(o->eui, i, k) = A3(o->a1u, o->jdi2, i, k); SI(o->evi, i, k) = A3(o->a1v, o->jdi2, i, k); }
  if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jdi1; j <= o->jdi2; j++) {
    SJ(o->sui, j, k) = A3(o->a1u, j, o->idi1, k); SJ(o->svi, j, k) = A3(o->a1v, j, o->idi1, k); }
  if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jdi1; j <= o->jdi2; j++) {
    SJ(o->nui, j, k) = A3(o->a1u, j, o->idi2, k); SJ(o->nvi, j, k) = A3(o->a1v, j, o->idi2, k); }
  if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
    SI(o->wue, i, k) = (A3(o->ub0, o->jde1, i, k) + xt * A3(o->ubt, o->jde1, i, k));
    SI(o->wve, i, k) = (A3(o->vb0, o->jde1, i, k) + xt * A3(o->vbt, o->jde1, i, k)); }
  if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
    SI(o->eue, i, k) = (A3(o->ub0, o->jde2, i, k) + xt * A3(o->ubt, o->jde2, i, k));
    SI(o->eve, i, k) = (A3(o->vb0, o->jde2, i, k) + xt * A3(o->vbt, o->jde2, i, k)); }
  if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) {
    SJ(o->sue, j, k) = (A3(o->ub0, j, o->ide1, k) + xt * A3(o->ubt, j, o->ide1, k));
    SJ(o->sve, j, k) = (A3(o->vb0, j, o->ide1, k) + xt * A3(o->vbt, j, o->ide1, k)); }
  if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) {
    SJ(o->nue, j, k) = (A3(o->ub0, j, o->ide2, k) + xt * A3(o->ubt, j, o->ide2, k));
    SJ(o->nve, j, k) = (A3(o->vb0, j, o->ide2, k) + xt * A3(o->vbt, j, o->ide2, k)); }
  if (o->bt && o->bl) for (int k = 1; k <= kz; k++) {
    SI(o->wui, o->ide2, k) = SJ(o->nue, o->jdi1, k); SI(o->wvi, o->ide2, k) = SJ(o->nve, o->jdi1, k);
    SJ(o->nui, o->jde1, k) = SI(o->wue, o->idi2, k); SJ(o->nvi, o->jde1, k) = SI(o->wve, o->idi2, k); }
  if (o->bb && o->bl) for (int k = 1; k <= kz; k++) {
    SI(o->wui, o->ide1, k) = SJ(o->sue, o->jdi1, k); SI(o->wvi, o->ide1, k) = SJ(o->sve, o->jdi1, k);
    SJ(o->sui, o->jde1, k) = SI(o->wue, o->idi1, k); SJ(o->svi, o->jde1, k) = SI(o->wve, o->idi1, k); }
  if (o->bt && o->br) for (int k = 1; k <= kz; k++) {
    SI(o->eui, o->ide2, k) = SJ(o->nue, o->jdi2, k); SI(o->evi, o->ide2, k) = SJ(o->nve, o->jdi2, k);
    SJ(o->nui, o->jde2, k) = SI(o->eue, o->idi2, k); SJ(o->nvi, o->jde2, k) = SI(o->eve, o->idi2, k); }
  if (o->bb && o->br) for (int k = 1; k <= kz; k++) {
    SI(o->eui, o->ide1, k) = SJ(o->sue, o->jdi2, k); SI(o->evi, o->ide1, k) = SJ(o->sve, o->jdi2, k);
    SJ(o->sui, o->jde2, k) = SI(o->eue, o->idi1, k); SJ(o->svi, o->jde2, k) = SI(o->eve, o->idi1, k); }
  if (o->bt) { xchb(o, o->nue, 0); xchb(o, o->nui, 0); xchb(o, o->nve, 0); xchb(o, o->nvi, 0); }
  if (o->bb) { xchb(o, o->sue, 0); xchb(o, o->sui, 0); xchb(o, o->sve, 0); xchb(o, o->svi, 0); }
  if (o->bl) { xchb(o, o->wue, 1); xchb(o, o->wui, 1); xchb(o, o->wve, 1); xchb(o, o->wvi, 1); }
  if (o->br) { xchb(o, o->eue, 1); xchb(o, o->eui, 1); xchb(o, o->eve, 1); xchb(o, o->evi, 1); }
}

/* bdyval, Main/mod_bdycod.F90:1109-2571 (idynamic = 1, iboudy /= 0, bdyflow) */
/* bdyin from read_icbc on, Main/mod_bdycod.F90:654-889: b0 <- b1 (:670-690), the record in
 * bin converted and coupled into b1 (:757-799, couple :4938-4951), exchanges (:759, 800-815),
 * timeint on the ga ranges (:801-825, :5087-5113), xbctime = 0 (:666).  NH: xpsb%b1 =
 * atm0%ps*d_r1000, psdot = atm0%psdot*d_r1000 (:398-400). */
void orc_bdyin(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  size_t n3 = o->plane * (size_t)kz;
  double rdtbdy = d_one / o->cfg.dtbdys;
  o->xbctime = d_zero;
  memcpy(o->ub0, o->bb1[0], n3 * 8); memcpy(o->vb0, o->bb1[1], n3 * 8);
  memcpy(o->tb0, o->bb1[2], n3 * 8); memcpy(o->qb0, o->bb1[3], n3 * 8);
  if (o->nh) {
    memcpy(o->ppb0, o->bb1[5], n3 * 8); memcpy(o->wwb0, o->bb1[6], o->plane * (size_t)kp * 8);
  } else {
    memcpy(o->pb0, o->bb1[4], o->plane * 8);
  }
  double* pb1 = o->bb1[4];
  double* psdot = (double*)calloc(o->plane, sizeof(double));
  if (o->nh) {
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A2(pb1, j, i) = A2(o->ps0, j, i) * 0.001;
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) A2(psdot, j, i) = A2(o->psdot0, j, i) * 0.001;
  } else {
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) A2(pb1, j, i) = (A2(o->bin[4], j, i) * 0.1) - o->ptop;
    xch(o, pb1, 1, 1, 0);
    psc2psd(o, pb1, psdot);
  }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ide1; i <= o->ide2; i++)
      for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->bb1[0], j, i, k) = A3(o->bin[0], j, i, k) * A2(psdot, j, i);
        A3(o->bb1[1], j, i, k) = A3(o->bin[1], j, i, k) * A2(psdot, j, i);
      }
  for (int k = 1; k <= kz; k++)
    for (int i = o->ice1; i <= o->ice2; i++)
      for (int j = o->jce1; j <= o->jce2; j++) {
        A3(o->bb1[2], j, i, k) = A3(o->bin[2], j, i, k) * A2(pb1, j, i);
        A3(o->bb1[3], j, i, k) = A3(o->bin[3], j, i, k) * A2(pb1, j, i);
      }
  for (int q = 0; q < 4; q++) xch(o, o->bb1[q], kz, 1, 0);
  if (o->nh) {
    for (int k = 1; k <= kz; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) A3(o->bb1[5], j, i, k) = A3(o->bin[5], j, i, k) * A2(pb1, j, i);
    for (int k = 1; k <= kp; k++)
      for (int i = o->ice1; i <= o->ice2; i++)
        for (int j = o->jce1; j <= o->jce2; j++) A3(o->bb1[6], j, i, k) = A3(o->bin[6], j, i, k) * A2(pb1, j, i);
    xch(o, o->bb1[5], kz, 1, 0);
    xch(o, o->bb1[6], kp, 1, 0);
  }
  free(psdot);
  for (int k = 1; k <= kz; k++) {
    for (int i = o->ide1ga; i <= o->ide2ga; i++)
      for (int j = o->jde1ga; j <= o->jde2ga; j++) {
        A3(o->ubt, j, i, k) = (A3(o->bb1[0], j, i, k) - A3(o->ub0, j, i, k)) * rdtbdy;
        A3(o->vbt, j, i, k) = (A3(o->bb1[1], j, i, k) - A3(o->vb0, j, i, k)) * rdtbdy;
      }
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++) {
        A3(o->tbt, j, i, k) = (A3(o->bb1[2], j, i, k) - A3(o->tb0, j, i, k)) * rdtbdy;
        A3(o->qbt, j, i, k) = (A3(o->bb1[3], j, i, k) - A3(o->qb0, j, i, k)) * rdtbdy;
        if (o->nh) A3(o->ppbt, j, i, k) = (A3(o->bb1[5], j, i, k) - A3(o->ppb0, j, i, k)) * rdtbdy;
      }
  }
  if (o->nh) {
    for (int k = 1; k <= kp; k++)
      for (int i = o->ice1ga; i <= o->ice2ga; i++)
        for (int j = o->jce1ga; j <= o->jce2ga; j++)
          A3(o->wwbt, j, i, k) = (A3(o->bb1[6], j, i, k) - A3(o->wwb0, j, i, k)) * rdtbdy;
  } else {
    for (int i = o->ice1ga; i <= o->ice2ga; i++)
      for (int j = o->jce1ga; j <= o->jce2ga; j++)
        A2(o->pbt, j, i) = (A2(pb1, j, i) - A2(o->pb0, j, i)) * rdtbdy;
  }
}

/* bdyval for the UW TKE (ibltyp = 2): atm2 = atm1 on the boundary lines while integrating
 * (Main/mod_bdycod.F90:1166-1306, done first in bdyval), then tkemin on every line at the
 * start, else (bdyflow) tkemin at k = 1 and, for k+1 = 3..kz+1, tkemin at inflow and the first
 * interior value at outflow (:2415-2509; level 2 is left as it is, as written) */
static void bdyval_tke(orc_t* o) {
  int kz = o->kz, kp = kz + 1;
  double tmin = o->cfg.tkemin;
  double *t1 = o->a1tke, *t2 = o->a2tke;
  if (o->lcount > 0) {
    if (o->bl) for (int k = 1; k <= kp; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(t2, o->jce1, i, k) = A3(t1, o->jce1, i, k);
    if (o->br) for (int k = 1; k <= kp; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(t2, o->jce2, i, k) = A3(t1, o->jce2, i, k);
    if (o->bb) for (int k = 1; k <= kp; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(t2, j, o->ice1, k) = A3(t1, j, o->ice1, k);
    if (o->bt) for (int k = 1; k <= kp; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(t2, j, o->ice2, k) = A3(t1, j, o->ice2, k);
  }
  if (o->lcount == 0) {
    for (int k = 1; k <= kp; k++) {
      if (o->bl) for (int i = o->ice1; i <= o->ice2; i++) { A3(t1, o->jce1, i, k) = tmin; A3(t2, o->jce1, i, k) = tmin; }
      if (o->br) for (int i = o->ice1; i <= o->ice2; i++) { A3(t1, o->jce2, i, k) = tmin; A3(t2, o->jce2, i, k) = tmin; }
      if (o->bt) for (int j = o->jce1; j <= o->jce2; j++) { A3(t1, j, o->ice2, k) = tmin; A3(t2, j, o->ice2, k) = tmin; }
      if (o->bb) for (int j = o->jce1; j <= o->jce2; j++) { A3(t1, j, o->ice1, k) = tmin; A3(t2, j, o->ice1, k) = tmin; }
    }
    return;
  }
  if (o->bl) {
    for (int i = o->ice1; i <= o->ice2; i++) { A3(t1, o->jce1, i, 1) = tmin; A3(t2, o->jce1, i, 1) = tmin; }
    for (int k = 2; k <= kz; k++) for (int i = o->ice1; i <= o->ice2; i++) {
      double tint = A3(t1, o->jci1, i, k + 1);
      double w = SI(o->wue, i, k) + SI(o->wue, i + 1, k) + SI(o->wui, i, k) + SI(o->wui, i + 1, k) +
                 SI(o->wue, i, k - 1) + SI(o->wue, i + 1, k - 1) + SI(o->wui, i, k - 1) + SI(o->wui, i + 1, k - 1);
      A3(t1, o->jce1, i, k + 1) = (w > d_zero) ? tmin : tint; }
  }
  if (o->br) {
    for (int i = o->ice1; i <= o->ice2; i++) { A3(t1, o->jce2, i, 1) = tmin; A3(t2, o->jce2, i, 1) = tmin; }
    for (int k = 2; k <= kz; k++) for (int i = o->ice1; i <= o->ice2; i++) {
      double tint = A3(t1, o->jci2, i, k + 1);
      double w = SI(o->eue, i, k) + SI(o->eue, i + 1, k) + SI(o->eui, i, k) + SI(o->eui, i + 1, k) +
                 SI(o->eue, i, k - 1) + SI(o->eue, i + 1, k - 1) + SI(o->eui, i, k - 1) + SI(o->eui, i + 1, k - 1);
      A3(t1, o->jce2, i, k + 1) = (w < d_zero) ? tmin : tint; }
  }
  if (o->bb) {
    for (int j = o->jce1; j <= o->jce2; j++) { A3(t1, j, o->ice1, 1) = tmin; A3(t2, j, o->ice1, 1) = tmin; }
    for (int k = 2; k <= kz; k++) for (int j = o->jci1; j <= o->jci2; j++) {
      double tint = A3(t1, j, o->ici1, k + 1);
      double w = SJ(o->sve, j, k) + SJ(o->sve, j + 1, k) + SJ(o->svi, j, k) + SJ(o->svi, j + 1, k) +
                 SJ(o->sve, j, k - 1) + SJ(o->sve, j + 1, k - 1) + SJ(o->svi, j, k - 1) + SJ(o->svi, j + 1, k - 1);
      A3(t1, j, o->ice1, k + 1) = (w > d_zero) ? tmin : tint; }
  }
  if (o->bt) {
    for (int j = o->jce1; j <= o->jce2; j++) { A3(t1, j, o->ice2, 1) = tmin; A3(t2, j, o->ice2, 1) = tmin; }
    for (int k = 2; k <= kz; k++) for (int j = o->jci1; j <= o->jci2; j++) {
      double tint = A3(t1, j, o->ici2, k + 1);
      double w = SJ(o->nve, j, k) + SJ(o->nve, j + 1, k) + SJ(o->nvi, j, k) + SJ(o->nvi, j + 1, k) +
                 SJ(o->nve, j, k - 1) + SJ(o->nve, j + 1, k - 1) + SJ(o->nvi, j, k - 1) + SJ(o->nvi, j + 1, k - 1);
      A3(t1, j, o->ice2, k + 1) = (w < d_zero) ? tmin : tint; }
  }
}

void orc_bdyval(orc_t* o) {
  int kz = o->kz;
  double xt = o->xbctime + o->dt;
  if (o->lcount > 0) {                                              /* :1126-1310 */
    if (o->bl) {
      for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->a2u, o->jde1, i, k) = A3(o->a1u, o->jde1, i, k); A3(o->a2v, o->jde1, i, k) = A3(o->a1v, o->jde1, i, k); }
      for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2t, o->jce1, i, k) = A3(o->a1t, o->jce1, i, k);
      for (int n = 0; n < o->nqx; n++) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++)
        A3(o->a2q[n], o->jce1, i, k) = A3(o->a1q[n], o->jce1, i, k);
      if (o->nh) {
        for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2pp, o->jce1, i, k) = A3(o->a1pp, o->jce1, i, k);
        for (int k = 1; k <= kz + 1; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2w, o->jce1, i, k) = A3(o->a1w, o->jce1, i, k);
      } else
        for (int i = o->ici1; i <= o->ici2; i++) A2(o->psb, o->jce1, i) = A2(o->psa, o->jce1, i);
    }
    if (o->br) {
      for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) {
        A3(o->a2u, o->jde2, i, k) = A3(o->a1u, o->jde2, i, k); A3(o->a2v, o->jde2, i, k) = A3(o->a1v, o->jde2, i, k); }
      for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2t, o->jce2, i, k) = A3(o->a1t, o->jce2, i, k);
      for (int n = 0; n < o->nqx; n++) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++)
        A3(o->a2q[n], o->jce2, i, k) = A3(o->a1q[n], o->jce2, i, k);
      if (o->nh) {
        for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2pp, o->jce2, i, k) = A3(o->a1pp, o->jce2, i, k);
        for (int k = 1; k <= kz + 1; k++) for (int i = o->ici1; i <= o->ici2; i++) A3(o->a2w, o->jce2, i, k) = A3(o->a1w, o->jce2, i, k);
      } else
        for (int i = o->ici1; i <= o->ici2; i++) A2(o->psb, o->jce2, i) = A2(o->psa, o->jce2, i);
    }
    if (o->bb) {
      for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->a2u, j, o->ide1, k) = A3(o->a1u, j, o->ide1, k); A3(o->a2v, j, o->ide1, k) = A3(o->a1v, j, o->ide1, k); }
      for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2t, j, o->ice1, k) = A3(o->a1t, j, o->ice1, k);
      for (int n = 0; n < o->nqx; n++) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->a2q[n], j, o->ice1, k) = A3(o->a1q[n], j, o->ice1, k);
      if (o->nh) {
        for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2pp, j, o->ice1, k) = A3(o->a1pp, j, o->ice1, k);
        for (int k = 1; k <= kz + 1; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2w, j, o->ice1, k) = A3(o->a1w, j, o->ice1, k);
      } else
        for (int j = o->jce1; j <= o->jce2; j++) A2(o->psb, j, o->ice1) = A2(o->psa, j, o->ice1);
    }
    if (o->bt) {
      for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) {
        A3(o->a2u, j, o->ide2, k) = A3(o->a1u, j, o->ide2, k); A3(o->a2v, j, o->ide2, k) = A3(o->a1v, j, o->ide2, k); }
      for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2t, j, o->ice2, k) = A3(o->a1t, j, o->ice2, k);
      for (int n = 0; n < o->nqx; n++) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++)
        A3(o->a2q[n], j, o->ice2, k) = A3(o->a1q[n], j, o->ice2, k);
      if (o->nh) {
        for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2pp, j, o->ice2, k) = A3(o->a1pp, j, o->ice2, k);
        for (int k = 1; k <= kz + 1; k++) for (int j = o->jce1; j <= o->jce2; j++) A3(o->a2w, j, o->ice2, k) = A3(o->a1w, j, o->ice2, k);
      } else
        for (int j = o->jce1; j <= o->jce2; j++) A2(o->psb, j, o->ice2) = A2(o->psa, j, o->ice2);
    }
  }
  /* p* and p*u, p*v boundary values, :1430-1526 (p* only for the hydrostatic core) */
  if (!o->nh) {
  if (o->bl) for (int i = o->ici1; i <= o->ici2; i++) A2(o->psa, o->jce1, i) = A2(o->pb0, o->jce1, i) + xt * A2(o->pbt, o->jce1, i);
  if (o->br) for (int i = o->ici1; i <= o->ici2; i++) A2(o->psa, o->jce2, i) = A2(o->pb0, o->jce2, i) + xt * A2(o->pbt, o->jce2, i);
  if (o->bb) for (int j = o->jce1; j <= o->jce2; j++) A2(o->psa, j, o->ice1) = A2(o->pb0, j, o->ice1) + xt * A2(o->pbt, j, o->ice1);
  if (o->bt) for (int j = o->jce1; j <= o->jce2; j++) A2(o->psa, j, o->ice2) = A2(o->pb0, j, o->ice2) + xt * A2(o->pbt, j, o->ice2);
  }
#define UVB(J, I) do { \
  A3(o->a1u, J, I, k) = A3(o->ub0, J, I, k) + xt * A3(o->ubt, J, I, k); \
  A3(o->a1v, J, I, k) = A3(o->vb0, J, I, k) + xt * A3(o->vbt, J, I, k); } while (0)
  if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) UVB(o->jde1, i);
  if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->idi1; i <= o->idi2; i++) UVB(o->jde2, i);
  if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) UVB(j, o->ide1);
  if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jde1; j <= o->jde2; j++) UVB(j, o->ide2);
#undef UVB
  bdyuv(o, xt);
  /* p*t and p*qv boundary values, :1700-1805 */
#define TQB(J, I) do { \
  A3(o->a1t, J, I, k) = A3(o->tb0, J, I, k) + xt * A3(o->tbt, J, I, k); \
  A3(o->a1q[0], J, I, k) = A3(o->qb0, J, I, k) + xt * A3(o->qbt, J, I, k); } while (0)
  if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) TQB(o->jce1, i);
  if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) TQB(o->jce2, i);
  if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) TQB(j, o->ice1);
  if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) TQB(j, o->ice2);
#undef TQB
  if (o->nh) {                                                      /* :1707-1790 */
#define PPW(J, I, JI, II) do { \
  for (int k = 1; k <= kz; k++) A3(o->a1pp, J, I, k) = A3(o->ppb0, J, I, k) + xt * A3(o->ppbt, J, I, k); \
  for (int k = 1; k <= kz + 1; k++) A3(o->a1w, J, I, k) = A3(o->wwb0, J, I, k) + xt * A3(o->wwbt, J, I, k); } while (0)
    if (o->bl) {
      for (int i = o->ici1; i <= o->ici2; i++) PPW(o->jce1, i, 0, 0);
      for (int i = o->ici1; i <= o->ici2; i++) A3(o->a1w, o->jce1, i, 1) = A3(o->a1w, o->jci1, i, 1);
    }
    if (o->br) {
      for (int i = o->ici1; i <= o->ici2; i++) PPW(o->jce2, i, 0, 0);
      for (int i = o->ici1; i <= o->ici2; i++) A3(o->a1w, o->jce2, i, 1) = A3(o->a1w, o->jci2, i, 1);
    }
    if (o->bb) {
      for (int j = o->jce1; j <= o->jce2; j++) PPW(j, o->ice1, 0, 0);
      for (int j = o->jce1; j <= o->jce2; j++) A3(o->a1w, j, o->ice1, 1) = A3(o->a1w, j, o->ici1, 1);
    }
    if (o->bt) {
      for (int j = o->jce1; j <= o->jce2; j++) PPW(j, o->ice2, 0, 0);
      for (int j = o->jce1; j <= o->jce2; j++) A3(o->a1w, j, o->ice2, 1) = A3(o->a1w, j, o->ici2, 1);
    }
#undef PPW
  }
  /* qv inflow/outflow for iboudy = 3 or 4, :1809-1950: west/east on ici, then south/north on
   * jce (they read the west/east results at the corners) */
  if (o->cfg.iboudy == 3 || o->cfg.iboudy == 4) {
    double* q = o->a1q[0];
    if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) {
      double qext = A3(q, o->jce1, i, k) / A2(o->psa, o->jce1, i);
      double qint = A3(q, o->jci1, i, k) / A2(o->psa, o->jci1, i);
      double w = SI(o->wue, i, k) + SI(o->wue, i + 1, k) + SI(o->wui, i, k) + SI(o->wui, i + 1, k);
      A3(q, o->jce1, i, k) = (w > d_zero) ? qext * A2(o->psa, o->jce1, i) : qint * A2(o->psa, o->jce1, i); }
    if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->ici1; i <= o->ici2; i++) {
      double qext = A3(q, o->jce2, i, k) / A2(o->psa, o->jce2, i);
      double qint = A3(q, o->jci2, i, k) / A2(o->psa, o->jci2, i);
      double w = SI(o->eue, i, k) + SI(o->eue, i + 1, k) + SI(o->eui, i, k) + SI(o->eui, i + 1, k);
      A3(q, o->jce2, i, k) = (w < d_zero) ? qext * A2(o->psa, o->jce2, i) : qint * A2(o->psa, o->jce2, i); }
    if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) {
      double qext = A3(q, j, o->ice1, k) / A2(o->psa, j, o->ice1);
      double qint = A3(q, j, o->ici1, k) / A2(o->psa, j, o->ici1);
      double w = SJ(o->sve, j, k) + SJ(o->sve, j + 1, k) + SJ(o->svi, j, k) + SJ(o->svi, j + 1, k);
      A3(q, j, o->ice1, k) = (w > d_zero) ? qext * A2(o->psa, j, o->ice1) : qint * A2(o->psa, j, o->ice1); }
    if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jce1; j <= o->jce2; j++) {
      double qext = A3(q, j, o->ice2, k) / A2(o->psa, j, o->ice2);
      double qint = A3(q, j, o->ici2, k) / A2(o->psa, j, o->ici2);
      double w = SJ(o->nve, j, k) + SJ(o->nve, j + 1, k) + SJ(o->nvi, j, k) + SJ(o->nvi, j + 1, k);
      A3(q, j, o->ice2, k) = (w < d_zero) ? qext * A2(o->psa, j, o->ice2) : qint * A2(o->psa, j, o->ice2); }
  }
  /* qx inflow/outflow of n = iqfrst .. iqlst (not present_qc, bdyflow), :2153-2220 */
  if (!o->cfg.present_qc) for (int n = 1; n < o->nqx; n++) {
    double* q = o->a1q[n];
    if (o->bl) for (int k = 1; k <= kz; k++) for (int i = o->ice1; i <= o->ice2; i++) {
      double qxint = A3(q, o->jci1, i, k) / A2(o->psa, o->jci1, i);
      double w = SI(o->wue, i, k) + SI(o->wue, i + 1, k) + SI(o->wui, i, k) + SI(o->wui, i + 1, k);
      A3(q, o->jce1, i, k) = (w > d_zero) ? d_zero : qxint * A2(o->psa, o->jce1, i); }
    if (o->br) for (int k = 1; k <= kz; k++) for (int i = o->ice1; i <= o->ice2; i++) {
      double qxint = A3(q, o->jci2, i, k) / A2(o->psa, o->jci2, i);
      double w = SI(o->eue, i, k) + SI(o->eue, i + 1, k) + SI(o->eui, i, k) + SI(o->eui, i + 1, k);
      A3(q, o->jce2, i, k) = (w < d_zero) ? d_zero : qxint * A2(o->psa, o->jce2, i); }
    if (o->bb) for (int k = 1; k <= kz; k++) for (int j = o->jci1; j <= o->jci2; j++) {
      double qxint = A3(q, j, o->ici1, k) / A2(o->psa, j, o->ici1);
      double w = SJ(o->sve, j, k) + SJ(o->sve, j + 1, k) + SJ(o->svi, j, k) + SJ(o->svi, j + 1, k);
      A3(q, j, o->ice1, k) = (w > d_zero) ? d_zero : qxint * A2(o->psa, j, o->ice1); }
    if (o->bt) for (int k = 1; k <= kz; k++) for (int j = o->jci1; j <= o->jci2; j++) {
      double qxint = A3(q, j, o->ici2, k) / A2(o->psa, j, o->ici2);
      double w = SJ(o->nve, j, k) + SJ(o->nve, j + 1, k) + SJ(o->nvi, j, k) + SJ(o->nvi, j + 1, k);
      A3(q, j, o->ice2, k) = (w < d_zero) ? d_zero : qxint * A2(o->psa, j, o->ice2); }
  }
  if (o->cfg.ibltyp == 2) bdyval_tke(o);
  o->xbctime = o->xbctime + o->dtsec;                               /* :2566 */
}

int orc_step(orc_t* o, int nsteps) {
  for (int s = 0; s < nsteps; s++) {
    if (orc_tend(o)) return 1;
    orc_bdyval(o);
  }
  return 0;
}
