/*
 * rcm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64, no FMA contraction) of the RegCM 4.7 hydrostatic
 * dynamical-core step `tend` + `bdyval` (Main/mod_tendency.F90:212-2121,
 * Main/mod_bdycod.F90:896-2571 and the modules they call).  It is the checker the parity
 * tests compare the HIP engine against, and the `cpu_baseline` leg of bench.py.  Nothing
 * in the product path (regcm_amd/, include/) may link or call it.
 *
 * Parity status: "parity unpinned" against executions of the reference -- the reference
 * is Fortran that cannot be built in this image without stand-ins for netCDF-Fortran
 * (Share/mod_dynparam.F90:28 `use netcdf`), and it ships no golden vectors (SURVEY.md
 * section 4).  See DESIGN.md "Oracle".
 *
 * The oracle is tile-aware: it owns ONE tile of the set_nproc decomposition and calls a
 * user-supplied exchange callback wherever the reference calls mpplib `exchange*`, so a
 * multi-rank test can run it under torch.distributed (gloo).
 */
#ifndef RCM_ORACLE_H
#define RCM_ORACLE_H
#include <stddef.h>
#include "../include/rcmdyn.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc orc_t;

/* sides: 0 = all 8 neighbours (exchange), 1 = left/bottom (+bottom-left corner)
 * (exchange_lb), 2 = right/top (+top-right corner) (exchange_rt).
 * field points at a frame array of nk levels, layout [k][i][j] over the tile frame
 * (see orc_frame_info). */
typedef void (*orc_exchange_fn)(void* ctx, double* field, int nk, int nex, int sides);
/* boundary-slice exchange along the boundary (exchange_bdy_lr / _bt):
 * along = 0: slice indexed by j (south/north slices), exchanged with left/right tiles;
 * along = 1: slice indexed by i (west/east slices), exchanged with bottom/top tiles. */
typedef void (*orc_exchange_bdy_fn)(void* ctx, double* slice, int nk, int along);

/* whole-domain gather of a 2-D cross field (the NH upper radiative condition gathers estore
 * over the domain, Main/mod_sound.F90:496-497, and sums the day-alarm means over it): every
 * tile passes its frame array and gets back the global [iy][jx] array (i-major, 1-based indices
 * at [(i-1)*jx + (j-1)]) holding every tile's owned cross points.  Called by every tile at the
 * same point; slot selects one of the run's global buffers. */
typedef const double* (*orc_gather_fn)(void* ctx, const double* field, int slot);
void orc_set_gather(orc_t* o, orc_gather_fn fn);

/* config->tile_first selects the tile; tile_count must be 1. */
orc_t* orc_create(const rcmdyn_config* cfg);
void orc_destroy(orc_t* o);
void orc_set_exchange(orc_t* o, orc_exchange_fn fn, orc_exchange_bdy_fn bfn, void* ctx);
/* info[0..3] = j0, i0 (frame origin, global index), nj, ni (frame size);
 * info[4..11] = jde1,jde2,ide1,ide2,jce1,jce2,ice1,ice2; info[12..15] = bdy flags L,R,B,T */
void orc_frame_info(const orc_t* o, int info[16]);
int orc_put(orc_t* o, int field, const double* src, int j1, int j2, int i1, int i2, int k1, int k2);
int orc_get(orc_t* o, int field, double* dst, int j1, int j2, int i1, int i2, int k1, int k2);
/* test hook: copy of an internal work array ("uten", "vten", NH "ppten", "wten") over the
 * whole frame; returns its level count, 0 if unknown or cap (doubles) is too small */
int orc_get_work(orc_t* o, const char* name, double* dst, size_t cap);
/* test hook: the NH sound returns after nsub sub-steps (0: right after its set-up), before
 * the time filters, so a test can check one sub-step; -1 (default) runs sound whole */
void orc_set_sound_probe(orc_t* o, int nsub);
/* test hook: the hydrostatic tend returns early (without advancing the clock): 1 = after every
 * tendency is summed and the t / qx forecasts and their negative fix are formed (work arrays
 * "ct", "cqv", "cqc"), before any time filter; 2 = after the time filters, at the entry of
 * splitf; 3 (isladvec = 1) = right after the semi-Lagrangian pass, whose terms are then all the
 * qv / qc dynamic tendencies hold (work arrays "qdynv", "qdync"); 0 (default) runs tend whole */
void orc_set_tend_probe(orc_t* o, int stage);
void orc_set_time(orc_t* o, long long lcount, double dt, double xbctime);
void orc_get_time(const orc_t* o, long long* lcount, double* dt, double* xbctime);
int orc_tend(orc_t* o);     /* returns 1 on CFL violation (NaN ptntot) */
void orc_bdyval(orc_t* o);
/* bdyin from read_icbc on: the record put into the XxB_B1 fields becomes b1 (see rcmdyn_bdyin) */
void orc_bdyin(orc_t* o);
void orc_diagnostics(const orc_t* o, double out[4]);
/* OpenMP-free, single thread.  Runs nsteps x (tend + bdyval); returns first error. */
int orc_step(orc_t* o, int nsteps);

#ifdef __cplusplus
}
#endif
#endif
