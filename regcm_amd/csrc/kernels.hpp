// kernels.hpp -- device kernels of kernels.hip and the argument blocks they share.
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
// k_split_project's extra blocks for the listed negative moisture forecasts (qfuse)
constexpr int NEGFIX_BLOCKS = 64;
// fused spstep tiling: SPB x SPB owned cross points + SPH halo (>= sub-steps per mode)
constexpr int SPB = 16, SPH = 8;
// the 8 x 8 form (k_spstep_fused<8>) below this many 16 x 16 blocks (engine.hip)
// timing-only builds (wrong results): the scalars blocks run 1 = the t chain only, 2 = the
// moisture chains only, 3 = the t chain only without the x**y of vadv3d, 4 = every chain
// without the x**y of vadv3d
#ifndef RCM_SC_TIMING_PART
#define RCM_SC_TIMING_PART 0
#endif
// k_update: XCD-aware tile placement within each level (xcd_tile2d, devcommon.hpp) on tiles of
// fewer points than this (rank tiles).  Alternating on one box (profiles/r05/tile_ab_uxcd.log,
// c3_uxcd_ab.log): 96x48 0.0792 -> 0.0773-0.0783 ms, 96x96 0.0962 -> 0.0936, 96x192 0.1325 ->
// 0.1310 ms; the 192x192 tile 2-5 us slower in k_update (99-101 -> 102-104 us), so off there
#ifndef UPD_XCD_BELOW
#define UPD_XCD_BELOW (192 * 192 / 2 + 1)
#endif
// k_split_correct(_bdy): the level's point pairs flattened over the blocks (1) or 64 x 4 pair
// tiles (0)
#ifndef SCOR_FLAT
#define SCOR_FLAT 1
#endif
#ifndef SP8_BELOW
#define SP8_BELOW 128
#endif
constexpr int SPR = SPB + 2 * SPH, SPP = SPR + 1;  // region side, LDS row pitch
// k_columns: COLW columns x 8 level groups per block (COLT threads, 4 x kz x COLW doubles of LDS;
// 32 measured 1-2 us slower at C3 than 64, profiles/r05/tile_ab_colw.log)
#ifndef RCM_COLW
#define RCM_COLW 64
#endif
#ifndef RCM_COLG
#define RCM_COLG 8
#endif
constexpr int COLW = RCM_COLW, COLG = RCM_COLG, COLT = COLW * COLG;   // COLG level groups
// k_split_project: SPC dot columns x SPG level groups per block (256 threads, 4 x kz x SPC
// doubles of LDS).  At C3 one row of 64 columns x 8 groups (512 threads) gave 576 blocks, a
// round and an eighth on 256 CUs at two blocks each; 32 x 8 gives 1 152 blocks of 23 KB, five
// per CU, one round (the kernel's time did not change: its block life, not the tail, sets it;
// profiles/r05/tile_ab_colw.log)
#ifndef RCM_SPC
#define RCM_SPC 32
#endif
constexpr int SPC = RCM_SPC, SPG = 8;
// k_split_project / k_split_correct(_bdy): XCD-contiguous block placement (xcd_range,
// devcommon.hpp): the rows a projection block shares with the next row's block, and the 2-D
// split sums every level of a correction block column reads, stay in one L2.  Round 6,
// alternating on one box (profiles/r06/tile_ab_split_xcd.log): k_split_project 24.4 -> 18.1-19.5
// us at C3, the C3 step 193.9-199.8 -> 186.0-189.9 us; the correction placement is neutral at
// C3 and takes the 96x48 rank tile's correction kernel 12.9 -> 10.9 us (step 0.0783-0.0788 ->
// 0.0771-0.0772 ms with both)
#ifndef SP_XCD
#define SP_XCD 1
#endif
#ifndef SCOR_XCD
#define SCOR_XCD 1
#endif
// k_columns: the same for its column blocks of a whole tile (part 0): the next row's column block,
// whose loads overlap this one's (atm1 at i + 1, p* at i +- 1), on the same XCD.  C3 k_columns
// 26.4-28.2 -> 24.3-25.6 us, the step 184.8 -> 183.7 us (3 alternations on one box), neutral on
// the 96 x 48 rank tile (profiles/r06/tile_ab_colx_spbdy.log)
#ifndef COL_XCD
#define COL_XCD 1
#endif
// depth of the wide exchange: SPH plus the ghost ring the fused split step also produces
constexpr int SPX = SPH + 1;
// LDS-tiled momentum block (dot points j x i at one level).  32 x 8 (256 threads, 39 KB of
// LDS: four blocks per CU): at C3 k_update 108 -> 97 us and the step 214 -> 200-203 us; on
// the 96-point rows of the scaling runs' tiles no half-idle second block column, and 96 x 48
// fits one round of blocks (step 88.6 -> 81.1 us); 64 x 8, 32 x 16 and 64 x 4 measured slower
// (round 5, alternating on one box: profiles/r05/tile_ab_w32.log)
#ifndef RCM_MBI
#define RCM_MBI 8
#endif
#ifndef RCM_MBJ
#define RCM_MBJ 32
#endif
constexpr int MBJ = RCM_MBJ, MBI = RCM_MBI, MBT = MBJ * MBI;
// LDS-tiled scalar (t, qv, qc) block (cross points j x i at one level)
#ifndef RCM_SBI
#define RCM_SBI 8
#endif
#ifndef RCM_SBJ
#define RCM_SBJ 32
#endif
constexpr int SBJ = RCM_SBJ, SBI = RCM_SBI, SBT = SBJ * SBI;
// k_update runs a momentum block or a scalars block in every workgroup of one launch, so the
// two block kinds must have the same thread count (their heights may differ only with it)
static_assert(MBT == SBT, "k_update launches momentum and scalars blocks with one block size");
// LDS-tiled species block of k_qx_tend (cross points j x i at one level).  Independent of the
// scalars tile: the launch in tend_post uses these constants, and the engine checks at create
// that the kernel was compiled for QBT threads (check_block_sizes, engine.hip)
#ifndef RCM_QBI
#define RCM_QBI 8
#endif
#ifndef RCM_QBJ
#define RCM_QBJ 64
#endif
constexpr int QBJ = RCM_QBJ, QBI = RCM_QBI, QBT = QBJ * QBI;
struct SegList {
  Seg s[MAXSEG];
  int n;
};

// boundary slices, order documented at k_bdyval_set
struct Slices { double* s[16]; };

// Halo/compute overlap of a decomposed tile: while the prologue exchange is in
// flight on the second stream, part 1 runs the blocks of k_columns / k_momentum / k_scalars
// whose reads all lie in R = [ja, jb] x [ia, ib], points no exchange writes and whose k_columns
// outputs part 1 itself forms; part 2 runs the others after the join; part 0 every block.
// k_columns maps its part 1 blocks onto the rows of R (nxb blocks of 64 columns per row) and
// its part 2 blocks onto the rest of the column box as one list (rbase: part 1's block count,
// so each block keeps its own noise partial).
// mj0 / sj0: the j origin of k_momentum's / k_scalars' 64-wide block columns in parts 1 and 2,
// shifted on narrow tiles so that one block column lies wholly in R (part 0: jdi1 / jcx1).
struct Part {
  int part, ja, jb, ia, ib, nxb, rbase, mj0, sj0;
};

// Every device buffer of one tile for one ping-pong parity: a* are the current time levels,
// b* the buffers the fused update kernels write the next time levels into.  Passed by value
// (kernel argument segment -> SGPRs); all fields share the frame, so one 32-bit byte offset
// per point addresses every one of them.  Diagnostic pointers are null when diagnostics are
// off (rcmdyn_set_diagnostics).
struct Fields {
  double *a1u, *a1v, *a1t, *a1qv, *a1qc, *a2u, *a2v, *a2t, *a2qv, *a2qc, *psa, *psb;
  double *b1u, *b1v, *b1t, *b1qv, *b1qc, *b2u, *b2v, *b2t, *b2qv, *b2qc, *bpsa, *bpsb;
  double *msfx, *msfd, *coriol, *ht, *xmsf, *dmsf, *hgfact, *mapf;
  const int8_t *rgcr, *rgdt;
  const int16_t *ibcr, *ibdt;
  double *ub0, *ubt, *vb0, *vbt, *tb0, *tbt, *qb0, *qbt, *pb0, *pbt;
  double *rpsa, *rpsb, *rpsda, *rpsdb, *psc, *psdota, *psdotb, *pten, *ptenn;
  double *qdot, *phi, *cqv, *cqc, *fqv, *fqc;
  double *slqv, *slqc;         // semi-Lagrangian qv/qc tendency starts (isladvec = 1, k_sladv)
  double *d6u, *d6v, *d6t, *d6qv, *d6qc;   // idiffu = 3 column terms (k_diffu6)
  unsigned* depplane;
  double *tten, *uten, *vten, *qvten, *qcten, *omega, *xkcs;
  // physics tendencies of the coupling seam (null: physics stubbed, the terms are 0)
  const double *tphy, *qvphy, *qcphy, *uphy, *vphy;
  const double* kpbl;          // iuwvadv = 1 (ibltyp = 2): the PBL-top level, vadv4d ind = 3 of qc
  // qfuse (the step without k_qfilter): k_columns filters p* into bpsa/bpsb and copies the
  // points the update kernels do not write into the next buffers; k_scalars RAW-filters the
  // non-negative moisture forecasts into b1q/b2q and appends the negative ones to neglist
  // (element offset * 2 + n) for k_split_project's fix-up blocks
  int qfuse;
  int* negcnt;
  uint32_t* neglist;
  // nqx = 5: atm1 of the hydrometeors beyond qc (k_columns: the total water load of tvfac)
  const double* qxa1[NQXH];
  double* red;                 // engine-wide noise-sum partials (k_columns -> k_split_correct)
  int red_off;                 // this tile's first partial
  Part pt;                     // the launch's overlap part (k_columns, k_momentum, k_scalars)
};

// nqx = 5: the hydrometeors beyond qc (qi, qr, qs) for the current (a*) and next (b*) time-level
// buffers (species.hip; the non-hydrostatic core updates a* in place and leaves b* null)
struct QxArgs {
  double *a1[NQXH], *a2[NQXH], *b1[NQXH], *b2[NQXH];
  double *cq[NQXH], *fq[NQXH];
  double *sl[NQXH], *d6[NQXH];
  const double* phy[NQXH];
  unsigned* dep;               // per (species, level) plane: row bitmap of the serially dependent negative points
  unsigned* depf;              // per (species, level) plane and row: k_qx_fix's flag of such a point (k_qx_serial
                               // turns the flags into the bitmap)
  int nsp;                     // hydrometeors beyond qc (0 for nqx = 2)
};

// serial negative-moisture fix-up of k_split_project's extra blocks: the q fields before
// (o*) and after (n*) the RAW filter, the unfiltered forecasts (c*) and fixed values (f*)
struct QFix {
  const double *cqv, *cqc;
  double *fqv, *fqc;
  const double *o1qv, *o1qc, *o2qv, *o2qc;
  double *n1qv, *n1qc, *n2qv, *n2qc;
  const double *psa, *psb;
  // the step's p* before its RA filter and psc: the serial sweep (in k_split_correct with
  // qfuse, beside the split corrections of psa/psb) forms the filtered p* from them
  const double *psc, *opsa, *opsb;
  unsigned* depplane;
  // qfuse: the negative forecasts k_scalars listed (k_split_project fixes the independent ones
  // in parallel; the serial sweeps of the flagged planes run in k_split_correct)
  const int* negcnt;
  const uint32_t* neglist;
  // qfuse: per (qv | qc, level) plane and row, the list pass's flag of a dependent point (a plain
  // store: atomics on the few bitmap words of a plane serialise at the memory side); the serial
  // passes OR the flags into depplane first (negfix_collect, qxcommon.hpp)
  unsigned* depf;
};

__global__ void k_surface_pressures(Geom g, Fields f);
template <bool QX>
__global__ void k_columns(Geom g, const Consts* __restrict__ c, StepState* s, Fields f, int nxb, int ncol);
__global__ void k_sladv(Geom g, const Consts* __restrict__ c, StepState* s, Fields f, QxArgs q);
__global__ void k_momentum(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, Fields f);
__global__ void k_diffu6(Geom g, const Consts* __restrict__ c, Fields f, QxArgs q);
__global__ void k_scalars(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, Fields f);
__global__ void k_update(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, Fields fm, Fields fs,
                         int mnx, int mny, int snx, int sny, int xcd);
__global__ void k_qfilter(Geom g, const Consts* __restrict__ c, Fields f);
// NEGFIX_POST (qxcommon.hpp): the serial fix passes resolve the chain, k_negfix_post / k_qx_post
// apply the filters of the points they fixed
#ifndef NEGFIX_POST
#define NEGFIX_POST 1
#endif
__global__ void k_negfix_serial(Geom g, const Consts* __restrict__ c, QFix q);
__global__ void k_negfix_post(Geom g, const Consts* __restrict__ c, QFix q);
__global__ void k_split_project(Geom g, const Consts* __restrict__ c, const double* __restrict__ a1u,
                                const double* __restrict__ a1v, const double* __restrict__ a2u,
                                const double* __restrict__ a2v, const double* __restrict__ a1t,
                                const double* __restrict__ a2t, const double* __restrict__ psa,
                                const double* __restrict__ psb, const double* __restrict__ msfd,
                                const double* __restrict__ mapf, double* dstor, double* hstor, double* deld,
                                double* delh, double* psdota, int nxp, int nproj, QFix qf, Geom gw,
                                double* wdeld, double* wdelh, double* wpsdota, double* wpsa,
                                const double* __restrict__ o2u, const double* __restrict__ o2v);
__global__ void k_spstep_init(Geom g, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh, double* ddsum, double* dhsum);
__global__ void k_spstep_grad(Geom g, const Consts* __restrict__ c, int l, int src, const double* __restrict__ delh, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota, double* uu, double* vv);
__global__ void k_spstep_update(Geom g, const Consts* __restrict__ c, int l, int n0, int n1, int nn, int leap, const double* __restrict__ uu, const double* __restrict__ vv, const double* __restrict__ mapf, const double* __restrict__ psa, double* deld, double* delh, double* ddsum, double* dhsum);
template <int SB>
__global__ void k_spstep_fused(Geom g, Geom w, const Consts* __restrict__ c, const double* __restrict__ deld, const double* __restrict__ delh, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ psdota, const double* __restrict__ mapf, const double* __restrict__ psa, double* ddsum, double* dhsum);
template <int NS>
__global__ __launch_bounds__(256) void k_split_correct(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum, const double* __restrict__ dhsum, const double* __restrict__ psdota, const double* __restrict__ msfd, double* psa, double* psb, double* a1t, double* a2t, double* a1u, double* a1v, double* a2u, double* a2v, StepState* s, int advance, const double* __restrict__ red, int red_total, FlagSnap* ring, QFix qf, int nser);
// pointers of bdyval (k_bdyval_set)
struct BdyArgs {
  double *a1u, *a1v, *a1t, *a1qv, *a1qc, *a2u, *a2v, *a2t, *a2qv, *a2qc, *psa, *psb;
  const double *ub0, *ubt, *vb0, *vbt, *tb0, *tbt, *qb0, *qbt, *pb0, *pbt;
  Slices sl;
  long slen;
  int set_ps;
};
__global__ void k_bdyval_set(Geom g, const StepState* __restrict__ s, BdyArgs a);
// 64-point chunks of the longest boundary line, one point past the tile included
inline int bdy_chunks(const Geom& g) { return (std::max(g.jde2 - g.jde1, g.ide2 - g.ide1) + 65) / 64; }
template <int NS>
__global__ __launch_bounds__(256) void k_split_correct_bdy(Geom g, const Consts* __restrict__ c, const double* __restrict__ ddsum, const double* __restrict__ dhsum, const double* __restrict__ psdota, const double* __restrict__ msfd, StepState* s, int advance, const double* __restrict__ red, int red_total, BdyArgs a, QFix qf, int nser);
__global__ void k_bdyval_qc(Geom g, int do_qc, int do_qv, double* a1qc, double* a1qv, const double* __restrict__ psa, Slices sl, long slen, StepState* s, double dtsec, int advance, FlagSnap* ring);
__global__ void k_flag_snapshot(const StepState* __restrict__ s, FlagSnap* ring);
__global__ void k_err_gather(const StepState* __restrict__ s, int32_t* derr);
__global__ void k_err_publish(const int32_t* __restrict__ derr, int32_t* hslot);
__global__ void k_prepare_static(Geom g, const Consts* __restrict__ c, int diffu_hgtf, const double* __restrict__ msfx, const double* __restrict__ msfd, const double* __restrict__ ht, double* xmsf, double* dmsf, double* hgfact, double* mapf);
__global__ void k_pack_segs(SegList L, double* __restrict__ buf, int unpack);
__global__ void k_copy_frame(Geom g, Geom w, int nplanes, const double* __restrict__ src, long sstride, double* dst, long dstride);

// species.hip: the hydrometeors beyond qc (nqx = 5), hydrostatic core (the ping-pong buffers)
__global__ void k_qx_tend(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, Fields f, QxArgs q);
__global__ void k_qx_fix(Geom g, const Consts* __restrict__ c, QxArgs q);
__global__ void k_qx_serial(Geom g, const Consts* __restrict__ c, QxArgs q);
__global__ void k_qx_post(Geom g, const Consts* __restrict__ c, QxArgs q);
__global__ void k_negfix_serial_qx(Geom g, const Consts* __restrict__ c, QFix qf, QxArgs q);
struct NHFields;
// the non-hydrostatic chains of the same hydrometeors (in place; k_qx_fix / k_qx_serial then
// run with b* = a*)
__global__ void k_nh_qx_tend(Geom g, const Consts* __restrict__ c, const StepState* __restrict__ s, NHFields f,
                             QxArgs q);
// bdyval's boundary copies and inflow/outflow of the hydrometeors beyond qc (both cores);
// integ: 1 integrating, 0 the initial call, -1 from the step clock (lcount > 0)
__global__ void k_bdyval_qx(Geom g, const StepState* __restrict__ s, QxArgs q, int integ, int do_qc,
                            const double* __restrict__ psa, Slices sl, long slen);

}  // namespace rcm
