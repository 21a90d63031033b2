/*
 * orc_par.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement run as set_nproc tiles on host
 * threads, the way the reference runs on MPI ranks (Main/mpplib/mod_mppparam.F90:1053-1371).
 *
 * Each tile is one orc_t (rcm_oracle.c) driven by its own OpenMP thread inside one parallel
 * region.  The oracle calls the exchange callbacks below at the points where the reference
 * calls mpplib `exchange*`.  As with MPI point-to-point messages, the n-th message from tile s
 * to its neighbour r matches r's n-th receive from s (tiles on the physical boundary skip
 * some exchanges, so there is no global barrier): the sender posts its array in the mailbox
 * of the pair, the receiver copies its ghost box straight out of the sender's frame (shared
 * memory in place of a message) and acknowledges, and the sender returns once every receiver
 * has acknowledged, so it never changes data a neighbour is still reading.  The box geometry
 * is the one of exchange / exchange_lb / exchange_rt / exchange_bdy_lr/_bt
 * (Main/mpplib/mod_mppparam.F90:6065-13190) and of tests/test_distributed_cpu.py.
 *
 * The hydrostatic step is decomposition-invariant, so a run on T
 * threads is bit-identical to the single-tile restatement; tests/test_oracle_cpu.py checks
 * that.  This is the all-cores CPU baseline of bench.py.
 */
#include <omp.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "rcm_oracle.h"

#define MAXT 256

struct orc_par {
  int ntiles, cj, ci, kz, jx, iy, band, crm;
  double* glob[3];                   /* whole-domain gathers of the NH radiative condition */
  orc_t* t[MAXT];
  int info[MAXT][16];
  /* mailbox of the message tile s sends toward direction d */
  double* volatile ptr[MAXT][8];
  atomic_int posted[MAXT][8], acked[MAXT][8];
  int sent[MAXT][8], rcvd[MAXT][8];   /* messages counted per pair (owner thread only) */
};
typedef struct orc_par orc_par_t;

static const int DJ[8] = {-1, 1, 0, 0, -1, 1, -1, 1};
static const int DI[8] = {0, 0, -1, 1, -1, -1, 1, 1};

static int recv_dir(int sides, int d) {
  if (sides == 0) return 1;
  if (sides == 1) return d == 0 || d == 2 || d == 4;     /* exchange_lb: from L, B, BL */
  return d == 1 || d == 3 || d == 7;                     /* exchange_rt: from R, T, TR */
}

/* a band (i_band = 1) is periodic in j (Main/mpplib/mod_mppparam.F90:1131 dim_period(1)),
 * CRM (i_crm = 1) in i as well (:1132 dim_period(2)) */
static int peer_of(const orc_par_t* p, int tile, int d) {
  int lj = tile / p->ci + DJ[d], li = tile % p->ci + DI[d];
  if (p->band) lj = (lj + p->cj) % p->cj;
  if (p->crm) li = (li + p->ci) % p->ci;
  return (lj >= 0 && lj < p->cj && li >= 0 && li < p->ci) ? lj * p->ci + li : -1;
}
/* offset from a ghost column's j to the same column in the frame of the tile across the
 * period (0 unless the message from direction d wraps around a band) */
static int jwrap(const orc_par_t* p, int tile, int d) {
  if (!p->band) return 0;
  const int lj = tile / p->ci;
  if (DJ[d] < 0 && lj == 0) return p->jx;
  if (DJ[d] > 0 && lj == p->cj - 1) return -p->jx;
  return 0;
}

/* the same for a ghost row across the CRM period in i */
static int iwrap(const orc_par_t* p, int tile, int d) {
  if (!p->crm) return 0;
  const int li = tile % p->ci;
  if (DI[d] < 0 && li == 0) return p->iy;
  if (DI[d] > 0 && li == p->ci - 1) return -p->iy;
  return 0;
}

static const int OPP[8] = {1, 0, 3, 2, 7, 6, 5, 4};

static void wait_ge(atomic_int* v, int n) {
  while (atomic_load_explicit(v, memory_order_acquire) < n) sched_yield();
}

/* post this tile's array toward every direction in `out` */
static void post(orc_par_t* p, int me, double* a, const int out[8]) {
  for (int d = 0; d < 8; d++)
    if (out[d]) {
      p->ptr[me][d] = a;
      atomic_store_explicit(&p->posted[me][d], ++p->sent[me][d], memory_order_release);
    }
}
/* wait until the message from direction d arrived; returns the sender's array */
static const double* arrived(orc_par_t* p, int me, int d, int* q) {
  *q = peer_of(p, me, d);
  const int n = ++p->rcvd[me][d];
  wait_ge(&p->posted[*q][OPP[d]], n);
  return p->ptr[*q][OPP[d]];
}
static void ack(orc_par_t* p, int me, int q, int d) {
  atomic_store_explicit(&p->acked[q][OPP[d]], p->rcvd[me][d], memory_order_release);
}
static void drain(orc_par_t* p, int me, const int out[8]) {
  for (int d = 0; d < 8; d++)
    if (out[d]) wait_ge(&p->acked[me][d], p->sent[me][d]);
}

static void xfn(void* ctx, double* a, int nk, int nex, int sides) {
  orc_par_t* p = (orc_par_t*)ctx;
  const int me = omp_get_thread_num();
  const int* f = p->info[me];
  int out[8];
  for (int d = 0; d < 8; d++) out[d] = peer_of(p, me, d) >= 0 && recv_dir(sides, OPP[d]);
  post(p, me, a, out);
  const size_t pl = (size_t)f[2] * f[3];
  for (int d = 0; d < 8; d++) {
    if (peer_of(p, me, d) < 0 || !recv_dir(sides, d)) continue;
    int q;
    const double* src = arrived(p, me, d, &q);
    const int* g = p->info[q];
    const size_t pq = (size_t)g[2] * g[3];
    const int sj = jwrap(p, me, d), si = iwrap(p, me, d);
    int j1 = f[4], j2 = f[5], i1 = f[6], i2 = f[7];      /* ghost box received from d */
    if (DJ[d] < 0) { j1 = f[4] - nex; j2 = f[4] - 1; }
    if (DJ[d] > 0) { j1 = f[5] + 1; j2 = f[5] + nex; }
    if (DI[d] < 0) { i1 = f[6] - nex; i2 = f[6] - 1; }
    if (DI[d] > 0) { i1 = f[7] + 1; i2 = f[7] + nex; }
    for (int k = 0; k < nk; k++)
      for (int i = i1; i <= i2; i++)
        for (int j = j1; j <= j2; j++)
          a[k * pl + (size_t)(i - f[1]) * f[2] + (j - f[0])] =
              src[k * pq + (size_t)(i + si - g[1]) * g[2] + (j + sj - g[0])];
    ack(p, me, q, d);
  }
  drain(p, me, out);
}

/* boundary slices: along 0 = indexed by j, exchanged with L/R; 1 = by i, with B/T */
static void bfn(void* ctx, double* s, int nk, int along) {
  orc_par_t* p = (orc_par_t*)ctx;
  const int me = omp_get_thread_num();
  const int* f = p->info[me];
  int out[8] = {0};
  for (int side = 0; side < 2; side++) {
    const int d = along == 0 ? side : 2 + side;
    out[d] = peer_of(p, me, d) >= 0;
  }
  post(p, me, s, out);
  const int n = along == 0 ? f[2] : f[3], o0 = along == 0 ? f[0] : f[1];
  const int lo = along == 0 ? f[4] : f[6], hi = along == 0 ? f[5] : f[7];
  for (int side = 0; side < 2; side++) {
    const int d = along == 0 ? side : 2 + side;
    if (!out[d]) continue;
    int q;
    const double* src = arrived(p, me, d, &q);
    const int* g = p->info[q];
    const int nq = along == 0 ? g[2] : g[3], oq = along == 0 ? g[0] : g[1];
    const int x = side == 0 ? lo - 1 : hi + 1;         /* owned by the peer */
    const int sx = along == 0 ? jwrap(p, me, d) : iwrap(p, me, d);
    for (int k = 0; k < nk; k++) s[(size_t)k * n + (x - o0)] = src[(size_t)k * nq + (x + sx - oq)];
    ack(p, me, q, d);
  }
  drain(p, me, out);
}

/* whole-domain gather (the NH upper radiative condition, Main/mod_sound.F90:496-497): a
 * barrier (nobody still reads the slot's previous contents), every tile copies its owned cross
 * points into the shared global array, a barrier, and every tile reads the whole array */
static const double* gfn(void* ctx, const double* a, int slot) {
  orc_par_t* p = (orc_par_t*)ctx;
  const int me = omp_get_thread_num();
  const int* f = p->info[me];
  double* gl = p->glob[slot];
#pragma omp barrier
  for (int i = f[10]; i <= f[11]; i++)
    for (int j = f[8]; j <= f[9]; j++)
      gl[(size_t)(i - 1) * p->jx + (j - 1)] = a[(size_t)(i - f[1]) * f[2] + (j - f[0])];
#pragma omp barrier
  return gl;
}

orc_par_t* orc_par_create(const rcmdyn_config* cfg) {
  const int nt = cfg->nproc_j * cfg->nproc_i;
  if (nt < 1 || nt > MAXT || (cfg->idynamic != 1 && cfg->idynamic != 2)) return NULL;
  orc_par_t* p = (orc_par_t*)calloc(1, sizeof(orc_par_t));
  p->ntiles = nt; p->cj = cfg->nproc_j; p->ci = cfg->nproc_i; p->kz = cfg->kz;
  p->jx = cfg->jx; p->iy = cfg->iy; p->band = cfg->i_band == 1; p->crm = cfg->i_crm == 1;
  if (cfg->idynamic == 2 && nt > 1)
    for (int q = 0; q < 3; q++) p->glob[q] = (double*)calloc((size_t)cfg->jx * cfg->iy, sizeof(double));
  for (int t = 0; t < nt; t++) {
    rcmdyn_config c = *cfg;
    c.tile_first = t; c.tile_count = 1;
    p->t[t] = orc_create(&c);
    if (!p->t[t]) {
      for (int u = 0; u < t; u++) orc_destroy(p->t[u]);
      free(p);
      return NULL;
    }
    orc_frame_info(p->t[t], p->info[t]);
    if (nt > 1) orc_set_exchange(p->t[t], xfn, bfn, p);
    if (nt > 1 && cfg->idynamic == 2) orc_set_gather(p->t[t], gfn);
  }
  return p;
}

void orc_par_destroy(orc_par_t* p) {
  if (!p) return;
  for (int t = 0; t < p->ntiles; t++) orc_destroy(p->t[t]);
  for (int q = 0; q < 3; q++) free(p->glob[q]);
  free(p);
}

int orc_par_ntiles(const orc_par_t* p) { return p->ntiles; }

int orc_par_put(orc_par_t* p, int field, const double* src, int j1, int j2, int i1, int i2, int k1, int k2) {
  int rc = 0;
  for (int t = 0; t < p->ntiles; t++) rc |= orc_put(p->t[t], field, src, j1, j2, i1, i2, k1, k2);
  return rc;
}

int orc_par_get(orc_par_t* p, int field, double* dst, int j1, int j2, int i1, int i2, int k1, int k2) {
  int rc = 0;
  for (int t = 0; t < p->ntiles; t++) rc |= orc_get(p->t[t], field, dst, j1, j2, i1, i2, k1, k2);
  return rc;
}

void orc_par_set_time(orc_par_t* p, long long lcount, double dt, double xbctime) {
  for (int t = 0; t < p->ntiles; t++) orc_set_time(p->t[t], lcount, dt, xbctime);
}

void orc_par_get_time(const orc_par_t* p, long long* lcount, double* dt, double* xbctime) {
  orc_get_time(p->t[0], lcount, dt, xbctime);
}

static int team_ok(const orc_par_t* p);

int orc_par_bdyval(orc_par_t* p) {
  if (!team_ok(p)) return -1;
#pragma omp parallel num_threads(p->ntiles)
  orc_bdyval(p->t[omp_get_thread_num()]);
  return 0;
}

/* nsteps x (tend + bdyval) on every tile.  orc_tend reports an error only after its last
 * exchange, so every tile finishes the step; the error then stops all of them together
 * (the reference's fatal aborts every rank).  Returns the error code. */
static int team_ok(const orc_par_t* p) {
  int got = 0;
#pragma omp parallel num_threads(p->ntiles)
  {
#pragma omp master
    got = omp_get_num_threads();
  }
  return got == p->ntiles;
}

int orc_par_step(orc_par_t* p, int nsteps) {
  int err = 0;
  if (!team_ok(p)) return -1;                /* one thread per tile, or the barriers deadlock */
#pragma omp parallel num_threads(p->ntiles)
  {
    orc_t* o = p->t[omp_get_thread_num()];
    for (int s = 0; s < nsteps; s++) {
      const int r = orc_tend(o);
      if (r) {
#pragma omp atomic write
        err = r;
      }
#pragma omp barrier
      int e;
#pragma omp atomic read
      e = err;
      if (e) break;
      orc_bdyval(o);
    }
  }
  return err;
}
