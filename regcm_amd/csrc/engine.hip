// engine.hip -- host side of the MI355X dynamical-core engine and the extern "C" ABI
// (include/rcmdyn.h).
//
// One engine instance owns one or more tiles of the set_nproc decomposition
// (Main/mpplib/mod_mppparam.F90:1053-1371) on one GPU.  A step is the reference sequence
// tend + bdyval (Main/mod_regcm_interface.F90:189,208) issued as ~30 kernels on one HIP
// stream; rcmdyn_step captures one step per ping-pong parity into a hipGraph and replays it.
// Halo exchanges mirror every mpplib exchange the reference performs; tiles on the same
// device exchange through a ghost-fill kernel, tiles on other ranks through RCCL
// (comm.hip).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <csignal>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "comm.hpp"
#include "engine.hpp"
#include "kernels.hpp"
#include "kernels_nh.hpp"
#include "slice.hpp"
#include "bdyin.hpp"
#include "tke.hpp"

using namespace rcm;

namespace {

thread_local std::string g_last_error;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess)                                                                \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_) + " @" + std::to_string(__LINE__)); \
  } while (0)

// constants, Share/mod_constants.F90 (same expressions as oracle/rcm_oracle.c)
constexpr double EGRAV = 9.80665, BOLTZK = 1.3806504e-23, NAVGDR = 6.02214129e23;
constexpr double AMD = 28.96454, AMW = 18.01528, VONKAR = 0.4;

// band (i_band = 1): periodic in j, so no tile has a west/east boundary and the cross grid
// takes every j (global_cross_jend = global_dot_jend, Main/mpplib/mod_mppparam.F90:1351-1354);
// crm (i_crm = 1): the same in i (dim_period(2), :1132, 1340-1342)
void tile_extent(int jx, int iy, int cj, int ci, int tile, int ext[8], int bdy[4], int band = 0, int crm = 0) {
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
  ext[4] = js; ext[5] = (je == jx && !band) ? je - 1 : je;
  ext[6] = is; ext[7] = (ie == iy && !crm) ? ie - 1 : ie;
  bdy[0] = (lj == 0) && !band; bdy[1] = (lj == cj - 1) && !band;
  bdy[2] = (li == 0) && !crm; bdy[3] = (li == ci - 1) && !crm;
}

Geom make_geom(int jx, int iy, int cj, int ci, int tile, int gh = G, int band = 0, int crm = 0) {
  int ext[8], bdy[4];
  tile_extent(jx, iy, cj, ci, tile, ext, bdy, band, crm);
  Geom g{};
  g.bl = bdy[0]; g.br = bdy[1]; g.bb = bdy[2]; g.bt = bdy[3];
  g.band = band;
  g.crm = crm;
  g.gjx = jx; g.giy = iy;
  g.jde1 = g.jdi1 = g.jdii1 = ext[0]; g.jde2 = g.jdi2 = g.jdii2 = ext[1];
  g.ide1 = g.idi1 = g.idii1 = ext[2]; g.ide2 = g.idi2 = g.idii2 = ext[3];
  if (g.bl) { g.jdi1 = g.jde1 + 1; g.jdii1 = g.jde1 + 2; }
  if (g.br) { g.jdi2 = g.jde2 - 1; g.jdii2 = g.jde2 - 2; }
  if (g.bb) { g.idi1 = g.ide1 + 1; g.idii1 = g.ide1 + 2; }
  if (g.bt) { g.idi2 = g.ide2 - 1; g.idii2 = g.ide2 - 2; }
  g.jce1 = g.jci1 = g.jcii1 = ext[4]; g.jce2 = g.jci2 = g.jcii2 = ext[5];
  g.ice1 = g.ici1 = g.icii1 = ext[6]; g.ice2 = g.ici2 = g.icii2 = ext[7];
  if (g.bl) { g.jci1 = g.jce1 + 1; g.jcii1 = g.jce1 + 2; }
  if (g.br) { g.jci2 = g.jce2 - 1; g.jcii2 = g.jce2 - 2; }
  if (g.bb) { g.ici1 = g.ice1 + 1; g.icii1 = g.ice1 + 2; }
  if (g.bt) { g.ici2 = g.ice2 - 1; g.icii2 = g.ice2 - 2; }
  int gl = g.bl ? 0 : 1, gr = g.br ? 0 : 1, gb = g.bb ? 0 : 1, gt = g.bt ? 0 : 1;
  g.jde1ga = g.jde1 - gl; g.jde2ga = g.jde2 + gr; g.ide1ga = g.ide1 - gb; g.ide2ga = g.ide2 + gt;
  g.jce1ga = g.jce1 - gl; g.jce2ga = g.jce2 + gr; g.ice1ga = g.ice1 - gb; g.ice2ga = g.ice2 + gt;
  g.jci1ga = g.jci1 - gl; g.jci2ga = g.jci2 + gr; g.ici1ga = g.ici1 - gb; g.ici2ga = g.ici2 + gt;
  g.jde1gb = g.jde1 - 2 * gl; g.jde2gb = g.jde2 + 2 * gr; g.ide1gb = g.ide1 - 2 * gb; g.ide2gb = g.ide2 + 2 * gt;
  g.jce1gb = g.jce1 - 2 * gl; g.jce2gb = g.jce2 + 2 * gr; g.ice1gb = g.ice1 - 2 * gb; g.ice2gb = g.ice2 + 2 * gt;
  g.j0 = g.jde1 - gh; g.i0 = g.ide1 - gh;
  g.nj = (g.jde2 - g.jde1 + 1) + 2 * gh;
  g.ni = (g.ide2 - g.ide1 + 1) + 2 * gh;
  g.pitch = (g.nj + 15) / 16 * 16;
  g.plane = (long)g.pitch * g.ni;
  g.P8 = (uint32_t)g.pitch * 8u;
  g.L8 = (uint32_t)(g.plane * 8);
  return g;
}

// setup_boundaries, Main/mod_atm_interface.F90:383-542 (global indices).  A band (i_band = 1,
// :435-455) has the south and north bands only, over every j.
void setup_boundaries(const Geom& g, int jx, int iy, int nsp, bool ldot, std::vector<int8_t>& rg,
                      std::vector<int16_t>& ib) {
  int icx = ldot ? 0 : 1, icy = ldot ? 0 : 1;
  int igbb1 = 2, igbb2 = nsp - 1, jgbl1 = 2, jgbl2 = nsp - 1;
  int igbt1 = iy - icy - nsp + 2, igbt2 = iy - icy - 1;
  int jgbr1 = jx - icx - nsp + 2, jgbr2 = jx - icx - 1;
  rg.assign(g.plane, 0);
  ib.assign(g.plane, -1);
  auto set = [&](int j, int i, int r, int b) { rg[g.ix(j, i)] = (int8_t)r; ib[g.ix(j, i)] = (int16_t)b; };
  // every frame point of the global domain (owned and ghost): the masks are functions of the
  // global index, so ghost points carry their owners' values
  const int fi1 = std::max(1, g.i0), fi2 = std::min(iy, g.i0 + g.ni - 1);
  const int fj1 = std::max(1, g.j0), fj2 = std::min(jx, g.j0 + g.nj - 1);
  if (g.crm) return;            // CRM: no relaxation band at all (:434, "if (.not. ma%crmflag)")
  if (g.band) {
    // periodic ghosts carry the band rows too
    for (int i = fi1; i <= fi2; i++)
      for (int j = g.j0; j < g.j0 + g.nj; j++) {
        if (i >= igbb1 && i <= igbb2) set(j, i, 1, i - igbb1 + 2);
        if (i >= igbt1 && i <= igbt2) set(j, i, 2, igbt2 - i + 2);
      }
    return;
  }
  for (int i = fi1; i <= fi2; i++)
    if (i >= igbb1 && i <= igbb2)
      for (int j = fj1; j <= fj2; j++)
        if (j >= jgbl1 && j <= jgbr2) {
          if (j <= jgbl2 && i >= j) continue;
          if (j >= jgbr1 && i >= (jgbr2 - j + 2)) continue;
          set(j, i, 1, i - igbb1 + 2);
        }
  for (int i = fi1; i <= fi2; i++)
    if (i >= igbt1 && i <= igbt2)
      for (int j = fj1; j <= fj2; j++)
        if (j >= jgbl1 && j <= jgbr2) {
          if (j <= jgbl2 && (igbt2 - i + 2) >= j) continue;
          if (j >= jgbr1 && (igbt2 - i) >= (jgbr2 - j)) continue;
          set(j, i, 2, igbt2 - i + 2);
        }
  for (int i = fi1; i <= fi2; i++) {
    if (i < igbb1 || i > igbt2) continue;
    for (int j = fj1; j <= fj2; j++)
      if (j >= jgbl1 && j <= jgbl2) {
        if (i < igbb2 && j > i) continue;
        if (i > igbt1 && j > (igbt2 - i + 2)) continue;
        set(j, i, 3, j - jgbl1 + 2);
      }
  }
  for (int i = fi1; i <= fi2; i++) {
    if (i < igbb1 || i > igbt2) continue;
    for (int j = fj1; j <= fj2; j++)
      if (j >= jgbr1 && j <= jgbr2) {
        if (i < igbb2 && (jgbr2 - j + 2) > i) continue;
        if (i > igbt1 && (jgbr2 - j) > (igbt2 - i)) continue;
        set(j, i, 4, jgbr2 - j + 2);
      }
  }
}

// Launch with an optional HIP event pair around the kernel (rcmdyn_kernel_times).
#define KLAUNCH(kern, ...)                                  \
  do {                                                      \
    if (dry) break;                                         \
    hipEvent_t e0_ = prof ? prof->begin(stream) : nullptr;  \
    hipLaunchKernelGGL(kern, __VA_ARGS__);                  \
    if (prof) prof->end(stream, #kern, e0_);                \
  } while (0)
// a stream-path HIP call that a plan-only engine (rcmdyn_exchange_plan) skips
#define DHIPCHK(x)           \
  do {                       \
    if (!dry) HIPCHK(x);     \
  } while (0)

// per-launch event pairs, aggregated by kernel name after the run
struct KernelProf {
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> rec;
  hipEvent_t get() {
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("rcmdyn: hipEventCreate failed");
      pool.push_back(e);
    }
    return pool[used++];
  }
  hipEvent_t begin(hipStream_t s) {
    hipEvent_t e = get();
    (void)hipEventRecord(e, s);
    return e;
  }
  void end(hipStream_t s, const char* name, hipEvent_t e0) {
    hipEvent_t e1 = get();
    (void)hipEventRecord(e1, s);
    rec.push_back({name, {e0, e1}});
  }
  ~KernelProf() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

inline dim3 grid3(int nj, int ni, int nk) { return dim3((nj + 63) / 64, (ni + 3) / 4, nk); }
const dim3 BLK(64, 4, 1);

}  // namespace

// Buffers that exchanges refer to, resolved per tile.
enum class FK {
  A1U, A1V, A1T, A1QV, A1QC, A2U, A2V, A2T, A2QV, A2QC, PSA, PSB, PSDOTA, PSDOTB,
  RPSDA, RPSDB, QDOT, CQV, CQC, PHI, UU, VV, DHSUM, DELH, MSFX, MSFD, HT, CORIOL,
  UB0, UBT, VB0, VBT, TB0, TBT, QB0, QBT, PB0, PBT, DSTOR, HSTOR,
  // non-hydrostatic core
  A1PP, A2PP, A1W, A2W, NCR, NXKCR, NCDT, NCPP, NCU, NCV,
  // device bdyin: coupled boundary data at the interval end
  UB1, VB1, TB1, QB1, PB1, PPB1, WWB1,
  // semi-Lagrangian moisture tendency starts
  SLQV, SLQC,
  // UW PBL TKE (ibltyp = 2)
  A1TKE, A2TKE,
  // idiffu = 3 column terms
  D6U, D6V, D6T, D6QV, D6QC,
  // nqx = 5: the hydrometeors beyond qc (qi, qr, qs), each kind in species order
  A1QX0, A1QX1, A1QX2, A2QX0, A2QX1, A2QX2, CQX0, CQX1, CQX2, SLQX0, SLQX1, SLQX2, D6QX0, D6QX1, D6QX2,
  // iuwvadv = 1: the PBL-top level (2-D)
  KPBL
};
inline FK fkq(FK base, int n) { return (FK)((int)base + n); }

struct rcmdyn_engine {
  rcmdyn_config cfg{};
  Consts hc{};
  Consts* dc = nullptr;
  StepState* ds = nullptr;
  StepState hs{};            // host mirror of the time state
  int ntiles = 0;
  std::vector<Geom> all;     // every tile of the decomposition
  std::vector<Tile> tiles;   // tiles owned here
  hipStream_t stream = nullptr;
  hipGraphExec_t gexec[2] = {nullptr, nullptr};   // tend + bdyval, per ping-pong parity
  hipGraphExec_t gexec2[2] = {nullptr, nullptr};  // two steps (tend + bdyval) x 2, per parity
  // steps per replayed graph in rcmdyn_step (RCMDYN_GRAPH_STEPS, 1 or 2): two steps per launch
  // return to the same ping-pong parity and halve the graph launches
  const int graph_steps = std::getenv("RCMDYN_GRAPH_STEPS") ? std::max(1, std::min(2, std::atoi(std::getenv("RCMDYN_GRAPH_STEPS")))) : 2;
  hipGraphExec_t gtend[2] = {nullptr, nullptr};   // tend alone (the drop-in rcmdyn_tend)
  hipGraphExec_t gbdy[2] = {nullptr, nullptr};    // bdyval alone (rcmdyn_bdyval)
  hipGraphExec_t gbdyf[2] = {nullptr, nullptr};   // rcmdyn_bdyval with the deferred corrections
  // step error flags: host-mapped snapshot ring written by the last launch of every tend,
  // one event per slot; the host checks a step's flags once its event completed and keeps
  // at most FLAG_LAG steps unchecked, so no entry point synchronises the stream per step
  FlagSnap* hflags = nullptr;
  FlagSnap* dflags = nullptr;
  hipEvent_t fev[NFLAGSLOT] = {};
  std::deque<long long> pending;
  static constexpr int FLAG_LAG = 2;
  // with a communicator the flags are max-reduced over the ranks every GLOBAL_EVERY steps
  // (and at the end of every rcmdyn_step) and only the reduced word raises the error, so
  // every rank stops at the same step -- the reference's fatal aborts the whole job
  // (Main/abort.F90:20-36); a rank stopping alone would leave its neighbours waiting
  static constexpr int GLOBAL_EVERY = 8;
  int32_t* derr = nullptr;
  int32_t* hgerr = nullptr;
  int32_t* dgerr = nullptr;
  hipEvent_t gev[NFLAGSLOT] = {};
  std::deque<std::pair<long long, int>> gpending;   // (step, slot)
  int gslot = 0;
  bool statics_dirty = true;
  bool bdy_dirty = true;
  bool dprd_put = false;      // NH: a dprddx / dprddy check is pending (check_dprd); sticky until it passes
  bool dprd_any = false;      // NH: dprddx / dprddy were put (a later atm0%pr put re-arms the check)
  bool kpbl_dirty = false;    // kpbl put since the last tend: its ghost ring is stale
  bool ghosts_stale = true;   // state put since the last tend: ghost rings are not step results
  bool capturing = false;
  long slen = 0;
  long staging_cap = 0;
  double* red = nullptr;     // noise-sum partials of every tile (k_columns)
  int red_total = 0;
  bool halo = false;          // ghost rings come from exchanges: a decomposition, or a band (periodic in j)
  bool diag = false;         // write the per-tend diagnostic fields
  KernelProf* prof = nullptr;  // set while rcmdyn_kernel_times runs
  double last_ms = 0.0;
  // RCMDYN_NO_GRAPH=1 runs rcmdyn_step eagerly (the path of RCCL-decomposed runs), for timing
  const bool no_graph = std::getenv("RCMDYN_NO_GRAPH") != nullptr;
  // k_momentum and k_scalars as one launch (k_update); RCMDYN_NO_FUSE_UPDATE=1: two launches
  const bool fuse_update = std::getenv("RCMDYN_NO_FUSE_UPDATE") == nullptr;
  // NH: tend's time filters of t, qv, qc in k_nh_tend_c and the negative-moisture fix, into
  // the other parity (Tile::tq); RCMDYN_NH_NO_TFUSE=1: in place in k_nh_tfilter_a1
  const bool nh_tfuse = std::getenv("RCMDYN_NH_NO_TFUSE") == nullptr;
  // parity of t, qv, qc: the step's ping-pong (hydrostatic), Tile::tq (NH)
  int thp(const Tile& t) const { return cfg.idynamic == 2 ? t.tq : t.cur; }
  // the parity the step graphs are captured for
  int gpar() const { return thp(tiles[0]); }
  // rcmdyn_step's hydrostatic bdyval runs inside k_split_correct_bdy (RCMDYN_NO_FUSE_BDY: two
  // launches of its own, as after rcmdyn_tend)
  const bool no_fuse_bdy = [] {
    const char* v = std::getenv("RCMDYN_NO_FUSE_BDY");
    return v && *v && std::strcmp(v, "0") != 0;
  }();
  bool fuse_bdy = false;      // set by step_once for the tend + bdyval pair it runs
  // the drop-in pair (rcmdyn_tend, then rcmdyn_bdyval): tend leaves its split corrections
  // pending and bdyval launches them with its boundary lines (k_split_correct_bdy, the form of
  // rcmdyn_step); any other call in between launches them alone first (settle).
  // RCMDYN_NO_DEFER_CORR=1: tend launches them itself.
  const bool no_defer_corr = std::getenv("RCMDYN_NO_DEFER_CORR") != nullptr;
  bool defer_corr = false;    // set by tend_call / post_physics around the tend they run
  bool corr_pending = false;  // the last tend's corrections are not launched yet
  // lazy tend (drop-in pair): rcmdyn_tend does the host bookkeeping and leaves the launch to
  // the next call: rcmdyn_bdyval replays the one-step graph of tend + bdyval (rcmdyn_step's),
  // any other call (settle) replays tend's own graph first.  RCMDYN_NO_LAZY_TEND=1: off
  const bool lazy_tend = std::getenv("RCMDYN_NO_LAZY_TEND") == nullptr;
  bool tend_pending = false;
  // fault injection for the tests (RCMDYN_INJECT_LAUNCH_FAILURE=n at create): the n-th launch of
  // a lazy tend's graph fails before it is issued, as a failed hipGraphLaunch would
  int inject_fail = 0;
  void inject_launch_failure() {
    if (inject_fail > 0 && --inject_fail == 0) throw std::runtime_error("rcmdyn: injected launch failure");
  }
  int lazy_par = 0;
  // the hydrostatic step without k_qfilter (its work in k_columns, k_scalars and the extra
  // blocks of k_split_project / k_split_correct); RCMDYN_NO_QFUSE=1 launches k_qfilter
  const bool no_qfuse = [] {
    const char* v = std::getenv("RCMDYN_NO_QFUSE");
    return v && *v && std::strcmp(v, "0") != 0;
  }();
  bool qfuse() const { return cfg.idynamic != 2 && !no_qfuse; }
  // nqx = 5, hydrostatic qfuse: the species' serial fix joins the qv / qc one after the split
  // corrections (k_negfix_serial_qx)
  bool serial_with_corr() const { return NEGFIX_POST && qfuse() && hc.nsp > 0; }
  // halo/compute overlap of the hydrostatic prologue exchange (Part, kernels.hpp) on a
  // decomposed domain; RCMDYN_NO_OVERLAP=1: the atm1/p* part first, then the atm2 part beside
  // k_columns only
  const bool no_overlap = [] {
    const char* v = std::getenv("RCMDYN_NO_OVERLAP");
    return v && *v && std::strcmp(v, "0") != 0;
  }();
  // (idiffu = 3: the column terms are formed after the whole exchange, so no overlap)
  bool overlap() const { return halo && cfg.idynamic != 2 && cfg.idiffu != 3 && !no_overlap; }
  bool post_inner = false;    // tend_pre ran part 1 of k_momentum / k_scalars
  std::string err;
  std::unique_ptr<Comm> comm;
  // RCMDYN_FORCE_RCCL=1: the halo messages between tiles held by this engine travel as RCCL
  // sends/receives to itself (one-rank communicator), not as device copies
  const bool force_rccl = std::getenv("RCMDYN_FORCE_RCCL") != nullptr;
  int device = 0;
  // halo/compute overlap: the second stream carries the atm2 part of the prologue exchange
  // while the first computes what needs only atm1 and p* (xch_begin / xch_join)
  hipStream_t stream2 = nullptr;
  // two exchanges may be in flight on the second stream at once (joined separately, slot 0/1)
  hipEvent_t evfork = nullptr, evjoin[2] = {nullptr, nullptr};
  bool join_pending[2] = {false, false};
  bool on2 = false;           // an exchange is being issued on stream2 (its staging buffers)
  // plan-only engine (rcmdyn_exchange_plan): host logic only, no device call; the exchanges and
  // collectives a rank would issue are logged by a PlanComm
  bool dry = false;

  std::vector<NHFields> nhf;   // non-hydrostatic buffers of each owned tile (idynamic = 2)
  double* nh_gbuf = nullptr;   // global-indexed day-alarm terms of the radiative condition

  int nsplit() const { return cfg.nsplit; }

  // ------------------------------------------------------------------ setup
  void compute_constants() {
    Consts& c = hc;
    std::memset(&c, 0, sizeof(c));
    c.kz = cfg.kz; c.nsplit = cfg.nsplit; c.iboudy = cfg.iboudy; c.nspgx = cfg.nspgx;
    c.stability_enhance = cfg.stability_enhance; c.present_qc = cfg.present_qc;
    const double rgasmol = NAVGDR * BOLTZK;
    c.c287 = rgasmol / AMD; c.rgas = c.c287 * 1000.0; c.cpd = 3.5 * c.rgas;
    c.ep1 = AMD / AMW - 1.0; c.regrav = 1.0 / EGRAV;
    c.rovcp = c.rgas * (1.0 / c.cpd);                        // Share/mod_constants.F90:183-184
    c.ipgf = cfg.ipgf;
    c.isladvec = cfg.isladvec; c.iqmsl = cfg.iqmsl;
    c.idiffu = cfg.idiffu;
    c.pgfaa1 = 6.5e-3 * c.rgas * c.regrav;                  // Share/mod_constants.F90:359-362
    c.dx = cfg.ds * 1000.0; c.dx2 = 2.0 * c.dx; c.dx4 = 4.0 * c.dx; c.dx8 = 8.0 * c.dx;
    c.dx16 = 16.0 * c.dx; c.dxsq = c.dx * c.dx; c.rdxsq = 1.0 / c.dxsq;
    c.ptop = cfg.ptop; c.dtsec = cfg.dtsec; c.gnu1 = cfg.gnu1; c.gnu2 = cfg.gnu2;
    c.t_extrema = cfg.t_extrema; c.q_rel_extrema = cfg.q_rel_extrema;
    const int kz = cfg.kz;
    for (int k = 1; k <= kz + 1; k++) c.sigma[k] = cfg.sigma[k - 1];
    for (int k = 1; k <= kz; k++) {
      c.hsigma[k] = (c.sigma[k + 1] + c.sigma[k]) * 0.5;
      c.dsigma[k] = (c.sigma[k + 1] - c.sigma[k]);
    }
    for (int k = 2; k <= kz; k++) {                         // Main/mod_params.F90:2208-2215
      c.twt1[k] = (c.sigma[k] - c.hsigma[k - 1]) / (c.hsigma[k] - c.hsigma[k - 1]);
      c.twt2[k] = 1.0 - c.twt1[k];
      c.qcon[k] = (c.sigma[k] - c.hsigma[k]) / (c.hsigma[k - 1] - c.hsigma[k]);
    }
    for (int k = 1; k <= kz; k++) c.xds[k] = 1.0 / c.dsigma[k];  // Main/mod_advection.F90:100
    // :106 (init dt).  upstream_mode = .false. selects the centred branches of hadvuv, hadvt,
    // hadv3d, hadvqv, hadvqx (Main/mod_advection.F90:141-201, 322-335, 409-460, 532-545,
    // 624-637): each is the upstream expression with ul = 0, term for term -- (1 + 0) a +
    // (1 - 0) b evaluates to exactly a + b, f1 = f2 = ff1..ff4 = +-0 -- so ul = 0 is the
    // centred scheme bit for bit
    c.ul = cfg.upstream_mode ? cfg.uoffc * 0.5 * cfg.dtsec / c.dx : 0.0;
    c.xkhmax = c.dxsq / (64.0 * cfg.dtsec);                          // Main/mod_diffusion.F90:104
    c.dydc = cfg.adyndif * VONKAR * VONKAR * c.dx * 0.25;
    c.diff6 = 0.12 * 0.015625 / (2.0 * cfg.dtsec);                    // Main/mod_diffusion.F90:78, 154
    c.xkhz = cfg.ckh * 1.5e-3 * c.dxsq / cfg.dtsec;
    const double fnudge = (cfg.bdy_nm > 0) ? cfg.bdy_nm : 0.1 / cfg.dtsec;   // Main/mod_bdycod.F90:204-215
    const double gnudge = (cfg.bdy_dm > 0) ? cfg.bdy_dm : 1.0 / (cfg.dtsec * 50.0);
    for (int n = 2; n <= cfg.nspgx - 1 && n < MAXNSP; n++) {
      double xfun = (double)(cfg.nspgx - n) / (double)(cfg.nspgx - 2);
      c.fcx[n] = fnudge * xfun; c.gcx[n] = gnudge * xfun;
    }
    if (cfg.iboudy == 4) {                                  // Main/mod_bdycod.F90:237-250
      c.wgtd[2] = 0.20; c.wgtd[3] = 0.55; c.wgtd[4] = 0.80; c.wgtd[5] = 0.95;
      for (int n = 6; n <= cfg.nspgd - 1 && n < MAXNSP; n++) c.wgtd[n] = 1.0;
      c.wgtx[2] = 0.4; c.wgtx[3] = 0.7; c.wgtx[4] = 0.9;
      for (int n = 5; n <= cfg.nspgx - 1 && n < MAXNSP; n++) c.wgtx[n] = 1.0;
    }
    for (int k = 1; k <= kz; k++) {
      double an = (c.hsigma[k] < 0.4) ? cfg.high_nudge : (c.hsigma[k] < 0.8) ? cfg.medium_nudge : cfg.low_nudge;
      for (int n = 2; n <= cfg.nspgx - 1 && n < MAXNSP; n++) {
        double xfun = std::exp(-((double)(n - 2) / an));
        c.hefc[n][k] = fnudge * xfun; c.hegc[n][k] = gnudge * xfun;
      }
    }
    for (int l = 0; l < cfg.nsplit; l++) {
      for (int k = 0; k < kz; k++) {
        c.zmatx[l][k] = cfg.zmatx[l][k]; c.zmatxr[l][k] = cfg.zmatxr[l][k];
        c.am[l][k] = cfg.am[l][k]; c.tau[l][k] = cfg.tau[l][k];
      }
      c.an[l] = cfg.an[l]; c.hbar[l] = cfg.hbar[l]; c.aam[l] = cfg.aam[l]; c.dtau[l] = cfg.dtau[l];
      for (int k = 1; k <= kz + 1; k++) {                  // Main/mod_split.F90:343-353
        double sh = cfg.sigmah[k - 1], va = cfg.varpa1[l][k - 1];
        c.pdlog[l][k] = va * std::log(sh * cfg.pd + cfg.ptop);
        c.eps1[l][k] = va * sh / (sh * cfg.pd + cfg.ptop);
      }
    }
    c.pd = cfg.pd;
    // RCMDYN_NEGFIX_MODE=1 (tests): the row sweep for every marked plane, dense ones included
    c.negfix_mode = std::getenv("RCMDYN_NEGFIX_MODE") ? std::atoi(std::getenv("RCMDYN_NEGFIX_MODE")) : 0;
    // non-hydrostatic core: diffusion constants (Main/mod_diffusion.F90:108-113), sound
    c.idynamic = cfg.idynamic;
    if (cfg.idynamic == 2) {
      c.xkhz = cfg.ckh * c.dx;
      c.xkhmax = 2.0 * c.xkhmax;
      c.ifupr = cfg.ifupr; c.ifrayd = cfg.ifrayd; c.rayndamp = cfg.rayndamp; c.crm = cfg.i_crm;
      c.rayalpha0 = cfg.rayalpha0; c.rayhd = cfg.rayhd; c.nhbet = cfg.nhbet; c.nhxkd = cfg.nhxkd;
      c.nh_dtsmax = cfg.nh_dtsmax; c.nh_xmsf = cfg.nh_xmsf;
      c.xgamma = 1.0 / (1.0 - c.rgas * (1.0 / c.cpd));           // Main/mod_sound.F90:77
    }
    c.dds[1] = 0.0; c.dds[kz + 1] = 0.0;                            // Main/mod_advection.F90:101-105
    for (int k = 2; k <= kz; k++) c.dds[k] = 1.0 / (c.dsigma[k] + c.dsigma[k - 1]);
    c.ibltyp = cfg.ibltyp; c.nuk = cfg.nuk; c.tkemin = cfg.tkemin;
    c.iqxvadv = (cfg.ibltyp == 2 && cfg.iuwvadv == 1) ? 3 : 1;
    c.ipptls = cfg.ipptls; c.nqx = cfg.nqx; c.nsp = cfg.nqx - 2;
  }

  double* dalloc(Tile& t, size_t n) {
    if (dry) return nullptr;
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, n * sizeof(double)));
    HIPCHK(hipMemset(p, 0, n * sizeof(double)));
    t.allocs.push_back(p);
    return (double*)p;
  }
  template <class T>
  T* talloc(Tile& t, size_t n) {
    if (dry) return nullptr;
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, n * sizeof(T)));
    HIPCHK(hipMemset(p, 0, n * sizeof(T)));
    t.allocs.push_back(p);
    return (T*)p;
  }

  void setup_tile(Tile& t, int index) {
    t.index = index;
    t.lj = index / cfg.nproc_i; t.li = index % cfg.nproc_i;
    t.g = all[index];
    const Geom& g = t.g;
    const int kz = cfg.kz, ns = cfg.nsplit;
    const size_t P = g.plane, P3 = P * kz;
    // neighbours L, R, B, T, BL, BR, TL, TR
    const int dj[8] = {-1, 1, 0, 0, -1, 1, -1, 1}, di[8] = {0, 0, -1, 1, -1, -1, 1, 1};
    for (int d = 0; d < 8; d++) {
      int lj = t.lj + dj[d], li = t.li + di[d];
      if (cfg.i_band) lj = (lj + cfg.nproc_j) % cfg.nproc_j;      // periodic in j (a tile may be its own)
      if (cfg.i_crm) li = (li + cfg.nproc_i) % cfg.nproc_i;       // CRM: periodic in i too
      t.nbr[d] = (lj >= 0 && lj < cfg.nproc_j && li >= 0 && li < cfg.nproc_i) ? lj * cfg.nproc_i + li : -1;
    }
    for (int b = 0; b < 2; b++) {
      t.a1u[b] = dalloc(t, P3); t.a1v[b] = dalloc(t, P3); t.a1t[b] = dalloc(t, P3);
      t.a1qv[b] = dalloc(t, P3); t.a1qc[b] = dalloc(t, P3);
      t.a2u[b] = dalloc(t, P3); t.a2v[b] = dalloc(t, P3); t.a2t[b] = dalloc(t, P3);
      t.a2qv[b] = dalloc(t, P3); t.a2qc[b] = dalloc(t, P3);
    }
    for (int b = 0; b < 2; b++) { t.psa_[b] = dalloc(t, P); t.psb_[b] = dalloc(t, P); }
    t.dstor = dalloc(t, P * ns); t.hstor = dalloc(t, P * ns);
    t.msfx = dalloc(t, P); t.msfd = dalloc(t, P); t.coriol = dalloc(t, P); t.ht = dalloc(t, P);
    t.xmsf = dalloc(t, P); t.dmsf = dalloc(t, P); t.hgfact = dalloc(t, P); t.mapf = dalloc(t, P);
    t.rgcr = talloc<int8_t>(t, P); t.rgdt = talloc<int8_t>(t, P);
    t.ibcr = talloc<int16_t>(t, P); t.ibdt = talloc<int16_t>(t, P);
    t.ub0 = dalloc(t, P3); t.ubt = dalloc(t, P3); t.vb0 = dalloc(t, P3); t.vbt = dalloc(t, P3);
    t.tb0 = dalloc(t, P3); t.tbt = dalloc(t, P3); t.qb0 = dalloc(t, P3); t.qbt = dalloc(t, P3);
    t.pb0 = dalloc(t, P); t.pbt = dalloc(t, P);
    t.rpsa = dalloc(t, P); t.rpsb = dalloc(t, P); t.rpsda = dalloc(t, P); t.rpsdb = dalloc(t, P);
    t.psc = dalloc(t, P); t.psdota = dalloc(t, P); t.psdotb = dalloc(t, P); t.pten = dalloc(t, 2 * P);
    t.qdot = dalloc(t, P * (kz + 1));
    t.phi = dalloc(t, P3);
    if (cfg.isladvec == 1) { t.slqv = dalloc(t, P3); t.slqc = dalloc(t, P3); }
    if (cfg.idiffu == 3)
      for (int q = 0; q < (cfg.idynamic == 2 ? 7 : 5); q++) t.d6[q] = dalloc(t, P * (kz + 1));
    if (cfg.ibltyp == 2) {
      t.a1tke = dalloc(t, P * (kz + 1)); t.a2tke = dalloc(t, P * (kz + 1)); t.ctke = dalloc(t, P * (kz + 1));
      t.kpbl = dalloc(t, P);
    }
    t.cqv = dalloc(t, P3); t.cqc = dalloc(t, P3); t.fqv = dalloc(t, P3); t.fqc = dalloc(t, P3);
    for (int n = 0; n < hc.nsp; n++) {            // nqx = 5: qi, qr, qs (species.hip)
      for (int b = 0; b < (cfg.idynamic == 2 ? 1 : 2); b++) {     // the NH core: in place
        t.a1qx[n][b] = dalloc(t, P3);
        t.a2qx[n][b] = dalloc(t, P3);
      }
      t.cqx[n] = dalloc(t, P3); t.fqx[n] = dalloc(t, P3);
      if (cfg.isladvec == 1) t.slqx[n] = dalloc(t, P3);
      if (cfg.idiffu == 3) t.d6qx[n] = dalloc(t, P * (kz + 1));
    }
    if (hc.nsp) {
      t.depx = talloc<unsigned>(t, (size_t)hc.nsp * kz * negfix_rowwords(g));
      t.depxf = talloc<unsigned>(t, (size_t)hc.nsp * kz * (g.ici2 - g.ici1 + 1));
    }
    t.depplane = talloc<unsigned>(t, 2 * (size_t)kz * negfix_rowwords(g));
    t.depqf = talloc<unsigned>(t, 2 * (size_t)kz * (g.ici2 - g.ici1 + 1));
    if (cfg.idynamic != 2) {
      t.negcnt = talloc<int>(t, 1);
      t.neglist = talloc<uint32_t>(t, 2 * P3);     // every (point, level, qv|qc) at most once
    }
    t.deld = dalloc(t, P * 3 * ns); t.delh = dalloc(t, P * 3 * ns);
    t.ddsum = dalloc(t, P * ns); t.dhsum = dalloc(t, P * ns);
    t.uu = dalloc(t, P); t.vv = dalloc(t, P);
    t.tten = dalloc(t, P3); t.uten = dalloc(t, P3); t.vten = dalloc(t, P3);
    t.qvten = dalloc(t, P3); t.qcten = dalloc(t, P3); t.omega = dalloc(t, P3); t.xkcs = dalloc(t, P3);
    if (halo) {                       // wide frame of the fused split step
      t.gw = make_geom(cfg.jx, cfg.iy, cfg.nproc_j, cfg.nproc_i, index, SPH + G, cfg.i_band, cfg.i_crm);
      const size_t PW = t.gw.plane;
      t.wdeld = dalloc(t, PW * 3 * ns); t.wdelh = dalloc(t, PW * 3 * ns);
      t.wpsa = dalloc(t, PW); t.wpsdota = dalloc(t, PW);
      t.wmsfx = dalloc(t, PW); t.wmsfd = dalloc(t, PW); t.wmapf = dalloc(t, PW);
    }
    slen = std::max<long>(g.pitch, g.ni);
    for (int s = 0; s < 16; s++) t.sl[s] = dalloc(t, (size_t)slen * kz);
    // halo staging: 8 directions x widest exchange (the hydrostatic prologue: 5 fields 2 wide
    // + 5 fields 3 wide + p*; at most 32 field-widths of kz+1 levels; nqx = 5 adds 3 fields 2
    // wide + 3 fields 3 wide)
    staging_cap = std::max<long>(staging_cap, 8L * (std::max(g.nj, g.ni) + 2 * G) * (32 + 16 * (hc.nsp > 0)) * (kz + 1));
    t.sbuf = dalloc(t, staging_cap);
    t.rbuf = dalloc(t, staging_cap);
    if (halo) {
      t.sbuf2 = dalloc(t, staging_cap);
      t.rbuf2 = dalloc(t, staging_cap);
    }
    // column blocks of k_columns (one noise partial each)
    // k_columns blocks: 64 columns x one row, over the tile and its ghost ring
    t.ncolx = (g.jdx2() - g.jdx1() + COLW) / COLW;
    t.nred = t.ncolx * (g.idx2() - g.idx1() + 1);
    if (overlap()) setup_overlap(t);
    t.red_off = red_total;
    red_total += t.nred;
    if (cfg.idynamic == 2) setup_nh(t);
    // boundary masks
    std::vector<int8_t> rg;
    std::vector<int16_t> ib;
    if (dry) return;
    // iboudy = 2 (time-dependent) and 3 (inflow/outflow) relax nothing (Main/mod_tendency.F90:
    // 1434-1510): an empty band turns every nudging and sponge branch of the kernels off
    const bool band = cfg.iboudy != 2 && cfg.iboudy != 3;
    setup_boundaries(g, cfg.jx, cfg.iy, cfg.nspgx, false, rg, ib);
    if (!band) std::fill(rg.begin(), rg.end(), (int8_t)0);
    HIPCHK(hipMemcpy(t.rgcr, rg.data(), P, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.ibcr, ib.data(), P * 2, hipMemcpyHostToDevice));
    setup_boundaries(g, cfg.jx, cfg.iy, cfg.nspgd, true, rg, ib);
    if (!band) std::fill(rg.begin(), rg.end(), (int8_t)0);
    HIPCHK(hipMemcpy(t.rgdt, rg.data(), P, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.ibdt, ib.data(), P * 2, hipMemcpyHostToDevice));
  }

  // non-hydrostatic buffers (kernels_nh.hpp NHFields); shared hydrostatic buffers are
  // filled per call by nhfields()
  void setup_nh(Tile& t) {
    const size_t P = t.g.plane, P3 = P * cfg.kz, P4 = P * (cfg.kz + 1);
    NHFields f{};
    for (double** p : {&f.a1pp, &f.a2pp, &f.pr1, &f.rho1, &f.cr, &f.xkcr, &f.ppten, &f.ct, &f.cu, &f.cv,
                       &f.cpp, &f.cdt, &f.se, &f.sf, &f.spi, &f.th})
      *p = dalloc(t, P3);
    if (!NH_XPRFORM) f.xpr = dalloc(t, P3);
    if (!NH_UDFORM) { f.ud = dalloc(t, P3); f.vd = dalloc(t, P3); }
    if (NH_NEGLIST) {             // every interior point of both species at most once
      f.neglist = talloc<unsigned>(t, 2 * P3);
      f.negcnt = talloc<int>(t, 1);
    }
    for (double** p : {&f.a1w, &f.a2w, &f.wten, &f.cw})
      *p = dalloc(t, P4);
    f.ppb0 = dalloc(t, P3); f.ppbt = dalloc(t, P3); f.wwb0 = dalloc(t, P4); f.wwbt = dalloc(t, P4);
    f.pr0 = dalloc(t, P3); f.t0 = dalloc(t, P3); f.rho0 = dalloc(t, P3); f.z0 = dalloc(t, P3);
    f.dprddx = dalloc(t, P3); f.dprddy = dalloc(t, P3);
    f.pf0 = dalloc(t, P4); f.rhof0 = dalloc(t, P4); f.zf0 = dalloc(t, P4);
    f.ps0 = dalloc(t, P); f.dpsdxm = dalloc(t, P); f.dpsdym = dalloc(t, P);
    f.ef = dalloc(t, P); f.ddx = dalloc(t, P); f.ddy = dalloc(t, P); f.dmdx = dalloc(t, P); f.dmdy = dalloc(t, P);
    f.ex = dalloc(t, P); f.crx = dalloc(t, P); f.cry = dalloc(t, P);
    f.estore = dalloc(t, P); f.astore = dalloc(t, P);
    if (nhf.empty()) {                 // engine-wide: mask, CFL slots, day-alarm gather buffer
      f.tmask = dalloc(t, 169);
      f.cfl = talloc<unsigned long long>(t, NH_CFL_SLOTS);
      f.cfll = talloc<unsigned long long>(t, NH_CFL_SLOTS);
      nh_gbuf = dalloc(t, 2 * (size_t)cfg.jx * cfg.iy);
    } else {
      f.tmask = nhf[0].tmask;
      f.cfl = nhf[0].cfl;
      f.cfll = nhf[0].cfll;
    }
    if (halo) t.westore = dalloc(t, t.gw.plane);
    nhf.push_back(f);
  }

  TkeArgs tke_args(Tile& t) {
    const int c = t.cur;
    TkeArgs a{};
    a.a1u = t.a1u[c]; a.a1v = t.a1v[c]; a.msfd = t.msfd; a.xmsf = t.xmsf; a.psa = t.psa_[c]; a.rpsa = t.rpsa;
    a.qdot = t.qdot; a.tkephy = t.tkephy; a.a1tke = t.a1tke; a.a2tke = t.a2tke; a.ctke = t.ctke;
    a.psb = t.psb_[c];
    if (cfg.idynamic == 2) { a.xk = nhf[&t - tiles.data()].xkcr; a.xkpb = t.psb_[t.cur]; a.xk_half = 0; }
    else { a.xk = t.xkcs; a.xk_half = 1; }
    return a;
  }
  // the TKE forecast and filter of tend (Main/mod_tendency.F90:515-544), after the kernels
  // that produce qdot and the diffusion coefficients
  void tke_step() {
    if (cfg.ibltyp != 2) return;
    each([&](Tile& t) {
      const Geom& g = t.g;
      const dim3 grid = grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, cfg.kz + 1);
      KLAUNCH(k_tke_tend, grid, BLK, 0, stream, g, dc, ds, tke_args(t));
      KLAUNCH(k_tke_filter, grid, BLK, 0, stream, g, dc, tke_args(t));
    });
  }
  // the TKE boundary lines of bdyval, once the boundary-wind slices are current
  void tke_bdyval() {
    if (cfg.ibltyp != 2) return;
    each([&](Tile& t) {
      Slices sl;
      for (int q = 0; q < 16; q++) sl.s[q] = t.sl[q];
      KLAUNCH(k_bdyval_tke, dim3(cfg.kz + 1), dim3(256), 0, stream, t.g, dc, ds, tke_args(t), sl, slen);
    });
  }

  NHFields nhfields(Tile& t) {
    NHFields f = nhf[&t - tiles.data()];
    const int c = t.cur, q = thp(t), o = 1 - q;
    f.a1u = t.a1u[c]; f.a1v = t.a1v[c]; f.a1t = t.a1t[q]; f.a1qv = t.a1qv[q]; f.a1qc = t.a1qc[q];
    f.a2u = t.a2u[c]; f.a2v = t.a2v[c]; f.a2t = t.a2t[q]; f.a2qv = t.a2qv[q]; f.a2qc = t.a2qc[q];
    f.b1t = t.a1t[o]; f.b1qv = t.a1qv[o]; f.b1qc = t.a1qc[o];
    f.b2t = t.a2t[o]; f.b2qv = t.a2qv[o]; f.b2qc = t.a2qc[o];
    f.tfuse = nh_tfuse ? 1 : 0;
    f.psa = t.psa_[c]; f.psb = t.psb_[c];
    f.msfx = t.msfx; f.msfd = t.msfd; f.coriol = t.coriol; f.ht = t.ht; f.xmsf = t.xmsf; f.dmsf = t.dmsf;
    f.hgfact = t.hgfact; f.rgcr = t.rgcr; f.rgdt = t.rgdt; f.ibcr = t.ibcr; f.ibdt = t.ibdt;
    f.ub0 = t.ub0; f.ubt = t.ubt; f.vb0 = t.vb0; f.vbt = t.vbt; f.tb0 = t.tb0; f.tbt = t.tbt;
    f.qb0 = t.qb0; f.qbt = t.qbt;
    f.rpsa = t.rpsa; f.rpsb = t.rpsb; f.rpsda = t.rpsda; f.rpsdb = t.rpsdb; f.psdota = t.psdota;
    f.psdotb = t.psdotb; f.qdot = t.qdot;
    f.tten = t.tten; f.qvten = t.qvten; f.qcten = t.qcten; f.uten = t.uten; f.vten = t.vten;
    f.cqv = t.cqv; f.cqc = t.cqc; f.fqv = t.fqv; f.fqc = t.fqc; f.depplane = t.depplane;
    f.tphy = t.phy[0]; f.qvphy = t.phy[1]; f.qcphy = t.phy[2]; f.uphy = t.phy[3]; f.vphy = t.phy[4];
    f.ppphy = t.phy[5]; f.wphy = t.phy[6];
    f.slqv = t.slqv; f.slqc = t.slqc;
    f.d6u = t.d6[0]; f.d6v = t.d6[1]; f.d6t = t.d6[2]; f.d6qv = t.d6[3]; f.d6qc = t.d6[4];
    f.d6pp = t.d6[5]; f.d6w = t.d6[6];
    f.kpbl = hc.iqxvadv == 3 ? t.kpbl : nullptr;
    for (int n = 0; n < hc.nsp; n++) f.qxa1[n] = t.a1qx[n][c];
    return f;
  }

  // The LDS-tiled kernels stage a tile sized at compile time (their __launch_bounds__ = the
  // tile's thread count) and index it by threadIdx; their launches take grid and block from the
  // same kernels.hpp constants.  Check once that the code objects were built for those tiles, so
  // a block-size mismatch between a kernel and its launch fails here, not as unwritten points.
  void check_block_sizes() {
    struct K { const void* f; int threads; const char* name; };
    const K ks[] = {{(const void*)k_update, SBT, "k_update"},
                    {(const void*)k_momentum, MBT, "k_momentum"},
                    {(const void*)k_scalars, SBT, "k_scalars"},
                    {(const void*)k_qx_tend, QBT, "k_qx_tend"}};
    for (const K& k : ks) {
      hipFuncAttributes a{};
      HIPCHK(hipFuncGetAttributes(&a, k.f));
      if (a.maxThreadsPerBlock != k.threads)
        throw std::runtime_error(std::string("rcmdyn: ") + k.name + " was compiled for " +
                                 std::to_string(a.maxThreadsPerBlock) + " threads per block, launched with " +
                                 std::to_string(k.threads));
    }
  }

  // The dynamic LDS the launches request grows with the tile: the serial moisture fix's
  // (negfix_lds / negfix_sweep_lds, a row of the plane) and k_split_project's (4 x kz x SPC).
  // Check the owned tiles' requests against the device's limit at create, so a tile too large
  // for them is refused here rather than failing a launch inside a step.
  void check_lds() {
    int maxs = 0;
    HIPCHK(hipDeviceGetAttribute(&maxs, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
    for (int t = 0; t < cfg.tile_count; t++) {
      const Geom& g = all[cfg.tile_first + t];
      const size_t need = sizeof(double) * (size_t)std::max(negfix_lds(g), 4 * cfg.kz * SPC);
      if (need > (size_t)maxs)
        throw std::runtime_error("rcmdyn: tile " + std::to_string(cfg.tile_first + t) + " needs " + std::to_string(need) +
                                 " bytes of LDS per block, the device allows " + std::to_string(maxs));
    }
  }

  void create(const rcmdyn_config* c, std::vector<PlanOp>* plan = nullptr) {
    cfg = *c;
    dry = plan != nullptr;
    if (cfg.abi_version != RCMDYN_ABI_VERSION) throw std::runtime_error("rcmdyn: ABI version mismatch");
#if RCM_SC_TIMING_PART || defined(RCM_SP_TIMING_M2)
    // a timing-only build computes wrong results on purpose: never by accident
    if (!std::getenv("RCMDYN_TIMING_BUILD"))
      throw std::runtime_error("rcmdyn: this library is a timing-only build (set RCMDYN_TIMING_BUILD=1 to run it)");
#endif
    if (cfg.idynamic != 1 && cfg.idynamic != 2) throw std::runtime_error("rcmdyn: idynamic must be 1 or 2");
    if (cfg.idynamic == 2) {
      if (!(cfg.nh_dtsmax > 0.0) || !(cfg.nh_xmsf > 0.0))
        throw std::runtime_error("rcmdyn: nh_dtsmax / nh_xmsf (init_sound) must be set for idynamic=2");
    }
    if (cfg.idiffu < 1 || cfg.idiffu > 3) throw std::runtime_error("rcmdyn: idiffu must be 1, 2 or 3");
    if (cfg.ipgf != 0 && cfg.ipgf != 1) throw std::runtime_error("rcmdyn: ipgf must be 0 or 1");
    if (cfg.isladvec != 0 && cfg.isladvec != 1) throw std::runtime_error("rcmdyn: isladvec must be 0 or 1");
    if (cfg.ibltyp == 2 && !(cfg.tkemin >= 0.0))
      throw std::runtime_error("rcmdyn: ibltyp=2 needs tkemin (uwtkemin) >= 0");
    if (cfg.iuwvadv != 0 && cfg.iuwvadv != 1) throw std::runtime_error("rcmdyn: iuwvadv must be 0 or 1");
    if (cfg.iboudy < 0 || cfg.iboudy > 5) throw std::runtime_error("rcmdyn: iboudy must be 0 to 5");
    // iboudy = 0 (fixed lateral values): the b0-only branches of bdyval (Main/mod_bdycod.F90:944,
    // 1317, 1535) act on the boundary lines only, so with CRM, which has none, it is the empty
    // boundary of crm_test.in; on a limited area those branches are not built
    if (cfg.iboudy == 0 && cfg.i_crm != 1)
      throw std::runtime_error("rcmdyn: iboudy = 0 (fixed lateral values) is built for i_crm = 1 only");
    // physicsparam ipptls and the nqx param derives from it (Main/mod_params.F90:1358-1366)
    if (cfg.ipptls < 1 || cfg.ipptls > 2)
      throw std::runtime_error("rcmdyn: ipptls must be 1 or 2 (ipptls = 0 leaves the hydrometeor tendencies unsummed, "
                               "Main/mod_tendency.F90:331: not supported)");
    if (cfg.nqx != (cfg.ipptls > 1 ? 5 : 2))
      throw std::runtime_error("rcmdyn: nqx must be 2 for ipptls = 1 and 5 for ipptls = 2 (Main/mod_params.F90:1358-1366)");
    // periodic decompositions and chemical tracers are not built: refused, not ignored
    if (cfg.i_band != 0 && cfg.i_band != 1) throw std::runtime_error("rcmdyn: i_band must be 0 or 1");
    // CRM (i_crm = 1, PreProc/CRM/crm_test.in): periodic in j and i, for the non-hydrostatic
    // core over the band; CRM without the band decomposes differently on one rank and on
    // several in the reference (Main/mpplib/mod_mppparam.F90:1104-1108 against 1132)
    if (cfg.i_crm != 0 && cfg.i_crm != 1) throw std::runtime_error("rcmdyn: i_crm must be 0 or 1");
    if (cfg.i_crm == 1 && (cfg.i_band != 1 || cfg.idynamic != 2))
      throw std::runtime_error("rcmdyn: i_crm = 1 is built for the non-hydrostatic core over the band (i_band = 1)");
    if (cfg.i_band != 0 && cfg.idynamic == 2 && cfg.idiffu == 3)
      throw std::runtime_error("rcmdyn: idiffu = 3 on the non-hydrostatic band / CRM is not supported");
    if (cfg.ichem != 0) throw std::runtime_error("rcmdyn: ichem = 1 (chemical tracers) is not supported");
    if (const char* m = std::getenv("RCMDYN_RCCL_CHAN2"))   // the removed second-communicator modes
      if (std::string(m) != "one") throw std::runtime_error("rcmdyn: RCMDYN_RCCL_CHAN2 must be one (or unset)");
    // dynparam's upstream_mode (default .true., Main/mod_params.F90:646); .false. runs the
    // centred branches (Main/mod_advection.F90:141,322,409,532,624; see c.ul)
    if (cfg.upstream_mode != 0 && cfg.upstream_mode != 1)
      throw std::runtime_error("rcmdyn: upstream_mode must be 0 or 1");
    if (cfg.stability_enhance != 0 && cfg.stability_enhance != 1)
      throw std::runtime_error("rcmdyn: stability_enhance must be 0 or 1");
    if (cfg.kz < 2 || cfg.kz > MAXKZ) throw std::runtime_error("rcmdyn: kz out of range");
    if (cfg.nsplit < 1 || cfg.nsplit > MAXSPLIT) throw std::runtime_error("rcmdyn: nsplit out of range");
    if (cfg.nspgx >= MAXNSP || cfg.nspgd != cfg.nspgx) throw std::runtime_error("rcmdyn: nspgx/nspgd unsupported");
    ntiles = cfg.nproc_j * cfg.nproc_i;
    halo = ntiles > 1 || cfg.i_band != 0;
    if (ntiles < 1 || cfg.tile_first < 0 || cfg.tile_count < 1 || cfg.tile_first + cfg.tile_count > ntiles)
      throw std::runtime_error("rcmdyn: bad tile range");
    if (!dry) {
      if (cfg.device >= 0) HIPCHK(hipSetDevice(cfg.device));
      HIPCHK(hipGetDevice(&device));
    }
    for (int t = 0; t < ntiles; t++) {
      all.push_back(make_geom(cfg.jx, cfg.iy, cfg.nproc_j, cfg.nproc_i, t, G, cfg.i_band, cfg.i_crm));
      const Geom& g = all.back();
      if (g.jde2 - g.jde1 + 1 < 3 || g.ide2 - g.ide1 + 1 < 3)
        throw std::runtime_error("rcmdyn: Too much processors (tile < 3x3), mod_mppparam.F90:1365");
      // the NH radiative condition reaches 6 points: its halo must come from direct neighbours
      if (cfg.idynamic == 2 && cfg.nproc_j * cfg.nproc_i > 1 && (g.jde2 - g.jde1 + 1 < 6 || g.ide2 - g.ide1 + 1 < 6))
        throw std::runtime_error("rcmdyn: non-hydrostatic tiles must be at least 6x6 points");
    }
    compute_constants();
    if (dry) {
      if (cfg.tile_count != 1 || cfg.comm_size != ntiles || cfg.tile_first != cfg.comm_rank)
        throw std::runtime_error("rcmdyn_exchange_plan: one tile per rank (tile_first == comm_rank, comm_size = tiles)");
      hs = StepState{};
      hs.dt = cfg.dtsec;
      tiles.resize(1);
      setup_tile(tiles[0], cfg.tile_first);
      comm.reset(make_plan_comm(cfg.comm_rank, plan));
      return;
    }
    check_block_sizes();
    check_lds();
    if (const char* e = std::getenv("RCMDYN_INJECT_LAUNCH_FAILURE")) inject_fail = std::atoi(e);
    HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&dc, sizeof(Consts)));
    HIPCHK(hipMemcpy(dc, &hc, sizeof(Consts), hipMemcpyHostToDevice));
    hs = StepState{};
    hs.dt = cfg.dtsec; hs.xbctime = 0.0; hs.lcount = 0;
    HIPCHK(hipMalloc(&ds, sizeof(StepState)));
    HIPCHK(hipMemcpy(ds, &hs, sizeof(StepState), hipMemcpyHostToDevice));
    tiles.resize(cfg.tile_count);
    for (int t = 0; t < cfg.tile_count; t++) {
      const Geom& g = all[cfg.tile_first + t];
      if ((double)g.plane * 8.0 * (cfg.kz + 1) >= 4294967296.0)
        throw std::runtime_error("rcmdyn: tile too large for 32-bit field offsets");
      setup_tile(tiles[t], cfg.tile_first + t);
    }
    HIPCHK(hipMalloc(&red, sizeof(double) * 2 * (size_t)(red_total + 1)));
    HIPCHK(hipHostMalloc((void**)&hflags, sizeof(FlagSnap) * NFLAGSLOT, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(hflags, 0, sizeof(FlagSnap) * NFLAGSLOT);
    HIPCHK(hipHostGetDevicePointer((void**)&dflags, hflags, 0));
    for (auto& e : fev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (cfg.tile_count < ntiles) {
      // RCMDYN_LOCAL_COMM=<group>: the in-process loopback transport of the multi-rank tests
      const char* lg = std::getenv("RCMDYN_LOCAL_COMM");
      if (lg && *lg) {
        if (cfg.comm_size != ntiles || cfg.tile_count != 1 || cfg.tile_first != cfg.comm_rank)
          throw std::runtime_error("rcmdyn: local communicator mode needs one tile per rank (tile_first == comm_rank)");
        comm.reset(make_local_comm(lg, cfg.comm_rank, cfg.comm_size));
      } else {
        comm.reset(make_rccl_comm(cfg));
      }
    }
    else if (force_rccl && halo) comm.reset(make_rccl_self_comm());
    if (comm) {
      HIPCHK(hipMalloc(&derr, sizeof(int32_t)));
      HIPCHK(hipHostMalloc((void**)&hgerr, sizeof(int32_t) * NFLAGSLOT, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(hgerr, 0, sizeof(int32_t) * NFLAGSLOT);
      HIPCHK(hipHostGetDevicePointer((void**)&dgerr, hgerr, 0));
      for (auto& e : gev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (halo) {
      HIPCHK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&evfork, hipEventDisableTiming));
      for (hipEvent_t& e : evjoin) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
  }

  void destroy() {
    if (stream) (void)hipStreamSynchronize(stream);
    invalidate_graphs();
    for (auto& e : fev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : gev)
      if (e) (void)hipEventDestroy(e);
    if (hflags) (void)hipHostFree(hflags);
    if (hgerr) (void)hipHostFree(hgerr);
    if (derr) (void)hipFree(derr);
    for (auto& t : tiles)
      for (void* p : t.allocs) (void)hipFree(p);
    tiles.clear();
    comm.reset();
    if (dc) (void)hipFree(dc);
    if (ds) (void)hipFree(ds);
    if (red) (void)hipFree(red);

    if (evfork) (void)hipEventDestroy(evfork);
    for (hipEvent_t e : evjoin)
      if (e) (void)hipEventDestroy(e);
    if (stream2) (void)hipStreamDestroy(stream2);
    if (stream) (void)hipStreamDestroy(stream);
  }

  void invalidate_graphs() {
    for (hipGraphExec_t* g : {gexec, gexec2, gtend, gbdy, gbdyf})
      for (int p = 0; p < 2; p++)
        if (g[p]) { (void)hipGraphExecDestroy(g[p]); g[p] = nullptr; }
  }

  // ------------------------------------------------------------------ step error flags
  // a tend was issued whose clock is lc once it ran: remember its snapshot slot; with a
  // communicator, every GLOBAL_EVERY steps (or when `global`) issue the job-wide reduction
  void note_step(long long lc, bool global = false) {
    if (dry) {
      if (global || lc % GLOBAL_EVERY == 0) comm->allreduce_max(nullptr, 1, stream);
      return;
    }
    if (comm) {
      if (global || lc % GLOBAL_EVERY == 0) {
        if ((int)gpending.size() >= NFLAGSLOT - 1) check(0);
        const int slot = gslot++ % NFLAGSLOT;
        hipLaunchKernelGGL(k_err_gather, dim3(1), dim3(64), 0, stream, ds, derr);
        comm->allreduce_max(derr, 1, stream);
        hipLaunchKernelGGL(k_err_publish, dim3(1), dim3(64), 0, stream, derr, dgerr + slot);
        HIPCHK(hipEventRecord(gev[slot], stream));
        gpending.push_back({lc, slot});
      }
      return;
    }
    if ((int)pending.size() >= NFLAGSLOT - 1) check(0);
    HIPCHK(hipEventRecord(fev[(lc - 1 + NFLAGSLOT) % NFLAGSLOT], stream));
    pending.push_back(lc);
  }
  // a failure: the stream drains, the sticky device flags are cleared (reported once) and
  // the error is raised -- the reference's fatal (Main/mod_tendency.F90:702,
  // Main/mod_sound.F90:679-681, Main/mod_sladvection.F90:149-154).  keep: a rank-local report
  // (check_now with a communicator) leaves the flags set, so the next job-wide reduction still
  // carries the failure to the other ranks even if this rank's host catches the error.
  [[noreturn]] void fail(int sl, long long lc, const std::string& scope, bool keep = false) {
    HIPCHK(hipStreamSynchronize(stream));
    pending.clear();
    gpending.clear();
    if (!keep) {
      StepState st;
      HIPCHK(hipMemcpy(&st, ds, sizeof(st), hipMemcpyDeviceToHost));
      st.nanflag = 0; st.slflag = 0;
      HIPCHK(hipMemcpy(ds, &st, sizeof(st), hipMemcpyHostToDevice));
    }
    const std::string at = " (" + scope + std::to_string(lc) + ")";
    if (sl) throw std::runtime_error("SLADVECTION: departure point beyond one grid cell" + at);
    throw std::runtime_error("CFL VIOLATION" + at);
  }
  // check the flags of the oldest steps until at most `keep` stay unchecked (with a
  // communicator: the reduced words, one reduction interval behind unless keep = 0)
  void check(size_t keep) {
    if (comm) {
      const size_t gkeep = keep == 0 ? 0 : 1;
      while (gpending.size() > gkeep) {
        const auto [lc, slot] = gpending.front();
        HIPCHK(hipEventSynchronize(gev[slot]));
        gpending.pop_front();
        const int w = ((volatile int32_t*)hgerr)[slot];
        if (w) fail(w & 2, lc, "job, by step ");
      }
      return;
    }
    while (pending.size() > keep) {
      const long long lc = pending.front();
      const int slot = (int)((lc - 1 + NFLAGSLOT) % NFLAGSLOT);
      HIPCHK(hipEventSynchronize(fev[slot]));
      pending.pop_front();
      const volatile FlagSnap* f = hflags + slot;
      const int sl = f->slflag, nan = f->nanflag;
      if (sl || nan) fail(sl, lc, "step ");
    }
  }
  // at a host read point (get, diagnostics) with the stream idle: every step issued so far is
  // checked, so no field of a failed run leaves the engine (the reference's fatal stops before
  // any output).  With a communicator the reductions already issued are drained (no new
  // collective: a get need not be called by every rank) and this rank's own sticky flags are
  // read as well; a rank-local failure is reported to its host, which aborts the job as the
  // reference's fatal does (Main/abort.F90:20-36).
  void check_now() {
    check(0);
    if (!comm) return;
    StepState st;
    HIPCHK(hipMemcpy(&st, ds, sizeof(st), hipMemcpyDeviceToHost));
    if (st.nanflag || st.slflag) fail(st.slflag, hs.lcount, "this rank, by step ", true);
  }


  // ------------------------------------------------------------------ field access
  double* fptr(Tile& t, FK f) {
    const int c = t.cur, q = thp(t);
    switch (f) {
      case FK::A1U: return t.a1u[c]; case FK::A1V: return t.a1v[c]; case FK::A1T: return t.a1t[q];
      case FK::A1QV: return t.a1qv[q]; case FK::A1QC: return t.a1qc[q];
      case FK::A2U: return t.a2u[c]; case FK::A2V: return t.a2v[c]; case FK::A2T: return t.a2t[q];
      case FK::A2QV: return t.a2qv[q]; case FK::A2QC: return t.a2qc[q];
      case FK::PSA: return t.psa_[c]; case FK::PSB: return t.psb_[c];
      case FK::PSDOTA: return t.psdota; case FK::PSDOTB: return t.psdotb;
      case FK::RPSDA: return t.rpsda; case FK::RPSDB: return t.rpsdb; case FK::QDOT: return t.qdot;
      case FK::CQV: return t.cqv; case FK::CQC: return t.cqc;
      case FK::PHI: return t.phi; case FK::UU: return t.uu; case FK::VV: return t.vv;
      case FK::DHSUM: return t.dhsum; case FK::DELH: return t.delh;
      case FK::MSFX: return t.msfx; case FK::MSFD: return t.msfd; case FK::HT: return t.ht;
      case FK::CORIOL: return t.coriol;
      case FK::UB0: return t.ub0; case FK::UBT: return t.ubt; case FK::VB0: return t.vb0;
      case FK::VBT: return t.vbt; case FK::TB0: return t.tb0; case FK::TBT: return t.tbt;
      case FK::QB0: return t.qb0; case FK::QBT: return t.qbt; case FK::PB0: return t.pb0;
      case FK::PBT: return t.pbt; case FK::DSTOR: return t.dstor; case FK::HSTOR: return t.hstor;
      default: break;
    }
    switch (f) {
      case FK::UB1: return t.bb1[0]; case FK::VB1: return t.bb1[1]; case FK::TB1: return t.bb1[2];
      case FK::QB1: return t.bb1[3]; case FK::PB1: return t.bb1[4]; case FK::PPB1: return t.bb1[5];
      case FK::WWB1: return t.bb1[6];
      case FK::SLQV: return t.slqv; case FK::SLQC: return t.slqc;
      case FK::A1TKE: return t.a1tke; case FK::A2TKE: return t.a2tke;
      case FK::D6U: return t.d6[0]; case FK::D6V: return t.d6[1]; case FK::D6T: return t.d6[2];
      case FK::D6QV: return t.d6[3]; case FK::D6QC: return t.d6[4];
      case FK::KPBL: return t.kpbl;
      default: break;
    }
    if (f >= FK::A1QX0 && f <= FK::D6QX2) {
      const int r = (int)f - (int)FK::A1QX0, n = r % NQXH;
      switch (r / NQXH) {
        case 0: return t.a1qx[n][c];
        case 1: return t.a2qx[n][c];
        case 2: return t.cqx[n];
        case 3: return t.slqx[n];
        default: return t.d6qx[n];
      }
    }
    const NHFields& h = nhf[&t - tiles.data()];
    switch (f) {
      case FK::A1PP: return h.a1pp; case FK::A2PP: return h.a2pp; case FK::A1W: return h.a1w;
      case FK::A2W: return h.a2w; case FK::NCR: return h.cr; case FK::NXKCR: return h.xkcr;
      case FK::NCDT: return h.cdt; case FK::NCPP: return h.cpp; case FK::NCU: return h.cu; case FK::NCV: return h.cv;
      default: break;
    }
    return nullptr;
  }

  // public field id -> (pointer, levels)
  static int atms_levels(int q, int kz) {
    const int f = RCMDYN_ATMS_UBX3D + q;
    if (f == RCMDYN_ATMS_PF3D || f == RCMDYN_ATMS_WB3D || f == RCMDYN_ATMS_ZQ) return kz + 1;
    if (f == RCMDYN_ATMS_PS2D || f == RCMDYN_ATMS_RHOX2D) return 1;
    return kz;
  }
  double* field_ptr(Tile& t, int f, int& nk) {
    nk = cfg.kz;
    const int c = t.cur;
    if (f >= RCMDYN_TPHY && f <= RCMDYN_WPHY) {
      if (f == RCMDYN_WPHY) nk = cfg.kz + 1;
      return t.phy[f - RCMDYN_TPHY];
    }
    if (f >= RCMDYN_ATMS_UBX3D && f <= RCMDYN_ATMS_RHB3D) {
      nk = atms_levels(f - RCMDYN_ATMS_UBX3D, cfg.kz);
      return t.atms[f - RCMDYN_ATMS_UBX3D];
    }
    if (f >= RCMDYN_XUB_B1 && f <= RCMDYN_XWWB_B1) {
      if (f == RCMDYN_XPSB_B1) nk = 1;
      if (f == RCMDYN_XWWB_B1) nk = cfg.kz + 1;
      return t.bin[f - RCMDYN_XUB_B1];
    }
    if (f == RCMDYN_ATM0_PSDOT) { nk = 1; return t.psdot0; }
    if (f >= RCMDYN_ATM1_TKE && f <= RCMDYN_TKEPHY) {
      nk = cfg.kz + 1;
      return f == RCMDYN_ATM1_TKE ? t.a1tke : f == RCMDYN_ATM2_TKE ? t.a2tke : t.tkephy;
    }
    if (f == RCMDYN_KPBL) { nk = 1; return t.kpbl; }
    if (f >= RCMDYN_ATM1_QI && f <= RCMDYN_ATMS_QXB3D_QS) {      // nqx = 5 only
      if (hc.nsp == 0) return nullptr;
      if (f <= RCMDYN_ATM1_QS) return t.a1qx[f - RCMDYN_ATM1_QI][c];
      if (f <= RCMDYN_ATM2_QS) return t.a2qx[f - RCMDYN_ATM2_QI][c];
      if (f <= RCMDYN_QSPHY) return t.phyx[f - RCMDYN_QIPHY];
      return t.atmsx[f - RCMDYN_ATMS_QXB3D_QI];
    }
    if (f >= RCMDYN_ATM1_PP && f <= RCMDYN_CRY) {
      if (cfg.idynamic != 2) return nullptr;
      NHFields& h = nhf[&t - tiles.data()];
      auto cst = [](const double* p) { return const_cast<double*>(p); };
      switch (f) {
        case RCMDYN_ATM1_PP: return h.a1pp;  case RCMDYN_ATM2_PP: return h.a2pp;
        case RCMDYN_XPPB_B0: return cst(h.ppb0); case RCMDYN_XPPB_BT: return cst(h.ppbt);
        case RCMDYN_ATM0_PR: return cst(h.pr0); case RCMDYN_ATM0_T: return cst(h.t0);
        case RCMDYN_ATM0_RHO: return cst(h.rho0); case RCMDYN_ATM0_Z: return cst(h.z0);
        case RCMDYN_DPRDDX: return cst(h.dprddx); case RCMDYN_DPRDDY: return cst(h.dprddy);
        default: break;
      }
      nk = cfg.kz + 1;
      switch (f) {
        case RCMDYN_ATM1_W: return h.a1w;  case RCMDYN_ATM2_W: return h.a2w;
        case RCMDYN_XWWB_B0: return cst(h.wwb0); case RCMDYN_XWWB_BT: return cst(h.wwbt);
        case RCMDYN_ATM0_PF: return cst(h.pf0); case RCMDYN_ATM0_RHOF: return cst(h.rhof0);
        case RCMDYN_ATM0_ZF: return cst(h.zf0);
        default: break;
      }
      nk = 1;
      switch (f) {
        case RCMDYN_ATM0_PS: return cst(h.ps0);
        case RCMDYN_DPSDXM: return cst(h.dpsdxm); case RCMDYN_DPSDYM: return cst(h.dpsdym);
        case RCMDYN_EF: return cst(h.ef); case RCMDYN_DDX: return cst(h.ddx); case RCMDYN_DDY: return cst(h.ddy);
        case RCMDYN_DMDX: return cst(h.dmdx); case RCMDYN_DMDY: return cst(h.dmdy);
        case RCMDYN_EX: return cst(h.ex); case RCMDYN_CRX: return cst(h.crx); case RCMDYN_CRY: return cst(h.cry);
        default: return nullptr;
      }
    }
    switch (f) {
      case RCMDYN_ATM1_U: return t.a1u[c]; case RCMDYN_ATM1_V: return t.a1v[c];
      case RCMDYN_ATM1_T: return t.a1t[thp(t)]; case RCMDYN_ATM1_QV: return t.a1qv[thp(t)];
      case RCMDYN_ATM1_QC: return t.a1qc[thp(t)];
      case RCMDYN_ATM2_U: return t.a2u[c]; case RCMDYN_ATM2_V: return t.a2v[c];
      case RCMDYN_ATM2_T: return t.a2t[thp(t)]; case RCMDYN_ATM2_QV: return t.a2qv[thp(t)];
      case RCMDYN_ATM2_QC: return t.a2qc[thp(t)];
      case RCMDYN_XUB_B0: return t.ub0; case RCMDYN_XUB_BT: return t.ubt;
      case RCMDYN_XVB_B0: return t.vb0; case RCMDYN_XVB_BT: return t.vbt;
      case RCMDYN_XTB_B0: return t.tb0; case RCMDYN_XTB_BT: return t.tbt;
      case RCMDYN_XQB_B0: return t.qb0; case RCMDYN_XQB_BT: return t.qbt;
      case RCMDYN_TTEN: return t.tten; case RCMDYN_UTEN: return t.uten; case RCMDYN_VTEN: return t.vten;
      case RCMDYN_QVTEN: return t.qvten; case RCMDYN_QCTEN: return t.qcten;
      case RCMDYN_OMEGA: return t.omega; case RCMDYN_XKC: return t.xkcs; case RCMDYN_PHI: return t.phi;
      case RCMDYN_QDOT: nk = cfg.kz + 1; return t.qdot;
      case RCMDYN_DSTOR: nk = cfg.nsplit; return t.dstor;
      case RCMDYN_HSTOR: nk = cfg.nsplit; return t.hstor;
      default: break;
    }
    nk = 1;
    switch (f) {
      case RCMDYN_PSA: return t.psa_[c]; case RCMDYN_PSB: return t.psb_[c];
      case RCMDYN_MSFX: return t.msfx; case RCMDYN_MSFD: return t.msfd;
      case RCMDYN_CORIOL: return t.coriol; case RCMDYN_HT: return t.ht;
      case RCMDYN_XPSB_B0: return t.pb0; case RCMDYN_XPSB_BT: return t.pbt;
      case RCMDYN_PSC: return t.psc; case RCMDYN_PTEN: return t.pten + t.g.plane;
      case RCMDYN_PSDOTA: return t.psdota;
      default: return nullptr;
    }
  }

  void put(int f, const double* src, int j1, int j2, int i1, int i2, int k1, int k2) {
    settle();
    const bool qxf = f >= RCMDYN_ATM1_QI && f <= RCMDYN_QSPHY;
    const bool phyf = (f >= RCMDYN_TPHY && f <= RCMDYN_WPHY) || (f >= RCMDYN_QIPHY && f <= RCMDYN_QSPHY);
    const bool binf = f >= RCMDYN_XUB_B1 && f <= RCMDYN_ATM0_PSDOT;
    const bool tkef = (f >= RCMDYN_ATM1_TKE && f <= RCMDYN_TKEPHY) || f == RCMDYN_KPBL;
    if (f < 0 || f >= RCMDYN_NFIELDS || (f > RCMDYN_XPSB_BT && f < RCMDYN_ATM1_PP) ||
        (f > RCMDYN_CRY && !phyf && !binf && !tkef && !qxf))
      throw std::runtime_error("rcmdyn_put: field is read-only or unknown");
    if (qxf && hc.nsp == 0) throw std::runtime_error("rcmdyn_put: qi/qr/qs fields need nqx = 5 (ipptls = 2)");
    if (tkef && cfg.ibltyp != 2) throw std::runtime_error("rcmdyn_put: TKE/kpbl fields need ibltyp=2 (UW PBL)");
    if (f == RCMDYN_KPBL) {
      // vadv4d ind = 3 stops on a PBL top above the model (Main/mod_advection.F90:923-925)
      const size_t n = (size_t)(j2 - j1 + 1) * (i2 - i1 + 1) * std::max(1, k2 - k1 + 1);
      for (size_t q = 0; q < n; q++) {
        if (src[q] > cfg.kz) throw std::runtime_error("rcmdyn_put: kpbl is greater than kz");
        if (src[q] != std::floor(src[q])) throw std::runtime_error("rcmdyn_put: kpbl must hold integers");
      }
    }
    if (f == RCMDYN_TKEPHY && !tiles.empty() && !tiles[0].tkephy) {
      HIPCHK(hipStreamSynchronize(stream));
      for (auto& t : tiles) t.tkephy = dalloc(t, t.g.plane * (cfg.kz + 1));
      invalidate_graphs();
    }
    if (((f >= RCMDYN_ATM1_PP && f <= RCMDYN_CRY) || f == RCMDYN_PPPHY || f == RCMDYN_WPHY ||
         f == RCMDYN_XPPB_B1 || f == RCMDYN_XWWB_B1 || f == RCMDYN_ATM0_PSDOT) && cfg.idynamic != 2)
      throw std::runtime_error("rcmdyn_put: non-hydrostatic field on a hydrostatic engine");
    if (f == RCMDYN_XPSB_B1 && cfg.idynamic == 2)
      throw std::runtime_error("rcmdyn_put: the non-hydrostatic core reads no ps record (p* is atm0%ps)");
    if (phyf) enable_physics();
    if (binf) enable_bdyin();
    HIPCHK(hipStreamSynchronize(stream));
    const long nj = j2 - j1 + 1, ni = i2 - i1 + 1;
    for (auto& t : tiles) {
      int nk;
      double* d = field_ptr(t, f, nk);
      const Geom& g = t.g;
      std::vector<double> h((size_t)nk * g.plane);
      HIPCHK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
      for (int k = std::max(k1, 1); k <= std::min(k2, nk); k++)
        for (int i = g.i0; i <= g.i0 + g.ni - 1; i++) {
          // CRM: the frame rows past either end of the period take the wrapped row
          const int iw = !cfg.i_crm ? i : (i < 1 ? i + cfg.iy : (i > cfg.iy ? i - cfg.iy : i));
          if (iw < i1 || iw > i2) continue;
          for (int j = g.j0; j <= g.j0 + g.nj - 1; j++) {
            // a band's frame columns past either end of the period take the wrapped column
            const int jw = !cfg.i_band ? j : (j < 1 ? j + cfg.jx : (j > cfg.jx ? j - cfg.jx : j));
            if (jw < j1 || jw > j2) continue;
            h[(size_t)(k - 1) * g.plane + g.ix(j, i)] = src[((size_t)(k - k1) * ni + (iw - i1)) * nj + (jw - j1)];
          }
        }
      HIPCHK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    }
    if (f >= RCMDYN_MSFX && f <= RCMDYN_HT) statics_dirty = true;
    if ((f >= RCMDYN_XUB_B0 && f <= RCMDYN_XPSB_BT) || (f >= RCMDYN_XPPB_B0 && f <= RCMDYN_XWWB_BT)) bdy_dirty = true;
    // only the hydrostatic vadv4d ind = 3 (k_scalars, k_qx_tend) reads kpbl on the ghost ring;
    // the NH kernels read it at their own point
    if (f == RCMDYN_KPBL && hc.iqxvadv == 3 && cfg.idynamic != 2) kpbl_dirty = true;
    ghosts_stale = true;
    if (f >= RCMDYN_ATM0_PS && f <= RCMDYN_CRY) invalidate_graphs();
    if (f == RCMDYN_DPRDDX || f == RCMDYN_DPRDDY) dprd_any = true;
    if (f == RCMDYN_DPRDDX || f == RCMDYN_DPRDDY || (dprd_any && f == RCMDYN_ATM0_PR)) dprd_put = true;
  }

  // physics coupling seam: the pc_physic buffers exist from the first put of one of them on
  // (zero-filled), and every later tend adds them; the captured graphs held null pointers
  void enable_physics() {
    if (tiles.empty() || tiles[0].phy[0]) return;
    HIPCHK(hipStreamSynchronize(stream));
    for (auto& t : tiles) {
      const size_t P = t.g.plane;
      for (int q = 0; q < 5; q++) t.phy[q] = dalloc(t, P * cfg.kz);
      if (cfg.idynamic == 2) { t.phy[5] = dalloc(t, P * cfg.kz); t.phy[6] = dalloc(t, P * (cfg.kz + 1)); }
      for (int n = 0; n < hc.nsp; n++) t.phyx[n] = dalloc(t, P * cfg.kz);
    }
    invalidate_graphs();
  }

  // device bdyin buffers (raw record, coupled b1; NH atm0%psdot), zero-filled
  void enable_bdyin() {
    if (tiles.empty() || tiles[0].bin[0]) return;
    HIPCHK(hipStreamSynchronize(stream));
    const bool nh = cfg.idynamic == 2;
    for (auto& t : tiles) {
      const size_t P = t.g.plane, P3 = P * cfg.kz, P4 = P * (cfg.kz + 1);
      for (int q = 0; q < 4; q++) { t.bin[q] = dalloc(t, P3); t.bb1[q] = dalloc(t, P3); }
      t.bin[4] = dalloc(t, P); t.bb1[4] = dalloc(t, P);
      if (nh) {
        t.bin[5] = dalloc(t, P3); t.bb1[5] = dalloc(t, P3);
        t.bin[6] = dalloc(t, P4); t.bb1[6] = dalloc(t, P4);
        t.psdot0 = dalloc(t, P);
      }
    }
  }

  // mod_bdycod::bdyin from read_icbc on (bdyin.hip)
  void bdyin() {
    settle();
    if (tiles.empty() || !tiles[0].bin[0]) throw std::runtime_error("rcmdyn_bdyin: no ICBC record was put (XUB_B1 ..)");
    const int kz = cfg.kz;
    const bool nh = cfg.idynamic == 2;
    auto args = [&](Tile& t) {
      BdyinArgs a{};
      a.rub = t.bin[0]; a.rvb = t.bin[1]; a.rtb = t.bin[2]; a.rqb = t.bin[3]; a.rpb = t.bin[4];
      a.rppb = t.bin[5]; a.rwwb = t.bin[6]; a.psdot0 = t.psdot0;
      a.ub0 = t.ub0; a.ubt = t.ubt; a.ub1 = t.bb1[0]; a.vb0 = t.vb0; a.vbt = t.vbt; a.vb1 = t.bb1[1];
      a.tb0 = t.tb0; a.tbt = t.tbt; a.tb1 = t.bb1[2]; a.qb0 = t.qb0; a.qbt = t.qbt; a.qb1 = t.bb1[3];
      a.pb0 = t.pb0; a.pbt = t.pbt; a.pb1 = t.bb1[4];
      if (nh) {
        NHFields& h = nhf[&t - tiles.data()];
        a.ps0 = h.ps0;
        a.ppb0 = const_cast<double*>(h.ppb0); a.ppbt = const_cast<double*>(h.ppbt); a.ppb1 = t.bb1[5];
        a.wwb0 = const_cast<double*>(h.wwb0); a.wwbt = const_cast<double*>(h.wwbt); a.wwb1 = t.bb1[6];
      }
      a.rdtbdy = 1.0 / cfg.dtbdys;                        // Main/mod_bdycod.F90:203
      a.ptop = cfg.ptop; a.kz = kz; a.nh = nh ? 1 : 0;
      return a;
    };
    each([&](Tile& t) {
      KLAUNCH(k_bdyin_shift, grid3(t.g.nj, t.g.ni, kz + 1), BLK, 0, stream, t.g, args(t));
      KLAUNCH(k_bdyin_ps, grid3(t.g.jce2 - t.g.jce1 + 1, t.g.ice2 - t.g.ice1 + 1, 1), BLK, 0, stream, t.g, args(t));
    });
    xch({{FK::PB1, 1}}, 1, 0);                              // :759
    each([&](Tile& t) {
      KLAUNCH(k_bdyin_couple, grid3(t.g.jde2 - t.g.jde1 + 1, t.g.ide2 - t.g.ide1 + 1, kz + 1), BLK, 0, stream,
              t.g, args(t));
    });
    if (nh) xch({{FK::UB1, kz}, {FK::VB1, kz}, {FK::TB1, kz}, {FK::QB1, kz}, {FK::PPB1, kz}, {FK::WWB1, kz + 1}}, 1, 0);
    else xch({{FK::UB1, kz}, {FK::VB1, kz}, {FK::TB1, kz}, {FK::QB1, kz}}, 1, 0);   // :800-815
    each([&](Tile& t) {
      KLAUNCH(k_bdyin_timeint, grid3(t.g.nj, t.g.ni, kz + 1), BLK, 0, stream, t.g, args(t));
    });
    set_time(hs.lcount, hs.dt, 0.0);                        // xbctime = d_zero, :666
    bdy_dirty = true;                                       // b0/bt ghost rings (prepare)
  }

  // mkslice export (slice.hip) for the host physics, run by rcmdyn_tend_pre_physics
  void run_slice() {
    for (auto& t : tiles) {
      if (t.atms[0]) continue;
      for (int q = 0; q < 22; q++) t.atms[q] = dalloc(t, t.g.plane * (size_t)atms_levels(q, cfg.kz));
      for (int n = 0; n < hc.nsp; n++) t.atmsx[n] = dalloc(t, t.g.plane * (size_t)cfg.kz);
    }
    each([&](Tile& t) {
      const Geom& g = t.g;
      const int c = t.cur;
      SliceArgs a{};
      a.a1u = t.a1u[c]; a.a1v = t.a1v[c]; a.a2u = t.a2u[c]; a.a2v = t.a2v[c]; a.a2t = t.a2t[thp(t)];
      a.a2qv = t.a2qv[thp(t)]; a.a2qc = t.a2qc[thp(t)]; a.psa = t.psa_[c]; a.psb = t.psb_[c];
      a.rpsb = t.rpsb; a.rpsdb = t.rpsdb; a.rpsda = t.rpsda; a.msfx = t.msfx; a.qdot = t.qdot; a.pten = t.pten;
      if (cfg.idynamic == 2) {
        const NHFields& h = nhf[&t - tiles.data()];
        a.a2pp = h.a2pp; a.a2w = h.a2w; a.ps0 = h.ps0; a.pr0 = h.pr0; a.pf0 = h.pf0; a.rho0 = h.rho0;
      }
      double** o = t.atms;
      a.ubx3d = o[0]; a.vbx3d = o[1]; a.ubd3d = o[2]; a.vbd3d = o[3]; a.tb3d = o[4]; a.qvb3d = o[5];
      a.qcb3d = o[6]; a.tv3d = o[7]; a.pb3d = o[8]; a.pf3d = o[9]; a.ps2d = o[10]; a.rhox2d = o[11];
      a.th3d = o[12]; a.rhob3d = o[13]; a.tp3d = o[14]; a.wpx3d = o[15]; a.wb3d = o[16]; a.zq = o[17];
      a.za = o[18]; a.dzq = o[19]; a.qsb3d = o[20]; a.rhb3d = o[21];
      a.ep2 = AMW / AMD;                                  // Share/mod_constants.F90:306
      a.rhmin = cfg.rhmin; a.rhmax = cfg.rhmax;
      for (int n = 0; n < hc.nsp; n++) { a.a2qx[n] = t.a2qx[n][c]; a.qxb3d[n] = t.atmsx[n]; }
      KLAUNCH(k_slice, grid3(g.jde2 - g.jde1 + 1, g.ide2 - g.ide1 + 1, 1), BLK, 0, stream, g, dc, a);
    });
  }

  void get(int f, double* dst, int j1, int j2, int i1, int i2, int k1, int k2) {
    settle();
    if (!diag && (f == RCMDYN_TTEN || f == RCMDYN_UTEN || f == RCMDYN_VTEN || f == RCMDYN_QVTEN ||
                  f == RCMDYN_QCTEN || f == RCMDYN_OMEGA || f == RCMDYN_XKC))
      throw std::runtime_error("rcmdyn_get: tendency diagnostics are off (rcmdyn_set_diagnostics)");
    if (f >= RCMDYN_ATMS_UBX3D && f <= RCMDYN_ATMS_RHB3D) {
      if (!tiles[0].atms[0]) throw std::runtime_error("rcmdyn_get: no slice fields yet (rcmdyn_tend_pre_physics)");
      if (cfg.idynamic == 2 && (f == RCMDYN_ATMS_ZQ || f == RCMDYN_ATMS_ZA || f == RCMDYN_ATMS_DZQ))
        throw std::runtime_error("rcmdyn_get: zq/za/dzq are not computed by mkslice for idynamic=2");
    }
    if (f >= RCMDYN_TPHY && f <= RCMDYN_WPHY && !tiles[0].phy[0])
      throw std::runtime_error("rcmdyn_get: no physics tendencies were put");
    if (f >= RCMDYN_ATM1_QI && f <= RCMDYN_ATMS_QXB3D_QS) {
      if (hc.nsp == 0) throw std::runtime_error("rcmdyn_get: qi/qr/qs fields need nqx = 5 (ipptls = 2)");
      if (f >= RCMDYN_QIPHY && f <= RCMDYN_QSPHY && !tiles[0].phyx[0])
        throw std::runtime_error("rcmdyn_get: no physics tendencies were put");
      if (f >= RCMDYN_ATMS_QXB3D_QI && !tiles[0].atmsx[0])
        throw std::runtime_error("rcmdyn_get: no slice fields yet (rcmdyn_tend_pre_physics)");
    }
    if (((f >= RCMDYN_ATM1_TKE && f <= RCMDYN_TKEPHY) || f == RCMDYN_KPBL) && cfg.ibltyp != 2)
      throw std::runtime_error("rcmdyn_get: TKE/kpbl fields need ibltyp=2 (UW PBL)");
    if (f == RCMDYN_TKEPHY && !tiles[0].tkephy) throw std::runtime_error("rcmdyn_get: no TKE tendency was put");
    HIPCHK(hipStreamSynchronize(stream));
    check_now();
    const long nj = j2 - j1 + 1, ni = i2 - i1 + 1;
    for (auto& t : tiles) {
      int nk;
      double* d = field_ptr(t, f, nk);
      if (!d) throw std::runtime_error("rcmdyn_get: unknown field");
      const Geom& g = t.g;
      std::vector<double> h((size_t)nk * g.plane);
      HIPCHK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
      for (int k = std::max(k1, 1); k <= std::min(k2, nk); k++)
        for (int i = std::max(i1, g.ide1); i <= std::min(i2, g.ide2); i++)
          for (int j = std::max(j1, g.jde1); j <= std::min(j2, g.jde2); j++)
            dst[((size_t)(k - k1) * ni + (i - i1)) * nj + (j - j1)] = h[(size_t)(k - 1) * g.plane + g.ix(j, i)];
    }
  }

  // ------------------------------------------------------------------ halo exchange
  // Every exchange stages the owned edge boxes of its fields per neighbour direction
  // (0 L, 1 R, 2 B, 3 T, 4 BL, 5 BR, 6 TL, 7 TR) with k_pack_segs, moves each direction's
  // contiguous span to the peer (device copy for a tile on this GPU, RCCL for a remote one)
  // and unpacks the ghost boxes.  sides: 0 exchange, 1 exchange_lb, 2 exchange_rt.
  static constexpr int DJ[8] = {-1, 1, 0, 0, -1, 1, -1, 1};
  static constexpr int DI[8] = {0, 0, -1, 1, -1, -1, 1, 1};
  static constexpr int OPP[8] = {1, 0, 3, 2, 7, 6, 5, 4};
  static bool recv_dir(int sides, int d) {
    if (sides == 0) return true;
    if (sides == 1) return d == 0 || d == 2 || d == 4;
    return d == 1 || d == 3 || d == 7;
  }
  int peer_of(const Tile& t, int d) const {
    int lj = t.lj + DJ[d];
    int li = t.li + DI[d];
    if (cfg.i_band) lj = (lj + cfg.nproc_j) % cfg.nproc_j;       // periodic in j (may be t itself)
    if (cfg.i_crm) li = (li + cfg.nproc_i) % cfg.nproc_i;        // CRM: periodic in i too
    return (lj >= 0 && lj < cfg.nproc_j && li >= 0 && li < cfg.nproc_i) ? lj * cfg.nproc_i + li : -1;
  }
  Tile* local_tile(int idx) {
    int o = idx - cfg.tile_first;
    return (o >= 0 && o < (int)tiles.size()) ? &tiles[o] : nullptr;
  }
  struct XField { FK f; int nk; int width = 0; int sides = -1; };  // 0/-1: the call's default
  // (j1,j2,i1,i2) of the box sent toward d (send) or received from d (recv)
  static void box(const Geom& g, int d, int w, bool send, int b[4]) {
    b[0] = g.jde1; b[1] = g.jde2; b[2] = g.ide1; b[3] = g.ide2;
    if (send) {
      if (DJ[d] < 0) b[1] = g.jde1 + w - 1;
      if (DJ[d] > 0) b[0] = g.jde2 - w + 1;
      if (DI[d] < 0) b[3] = g.ide1 + w - 1;
      if (DI[d] > 0) b[2] = g.ide2 - w + 1;
    } else {
      if (DJ[d] < 0) { b[0] = g.jde1 - w; b[1] = g.jde1 - 1; }
      if (DJ[d] > 0) { b[0] = g.jde2 + 1; b[1] = g.jde2 + w; }
      if (DI[d] < 0) { b[2] = g.ide1 - w; b[3] = g.ide1 - 1; }
      if (DI[d] > 0) { b[2] = g.ide2 + 1; b[3] = g.ide2 + w; }
    }
  }
  // segment builder: appends the segments of direction d (send or recv) for tile t
  using SegFn = std::function<void(Tile&, int, bool, std::vector<Seg>&)>;
  struct Layout {
    std::vector<Seg> segs;
    long start[8], count[8];
    uint64_t sig[8];       // shape signature of each direction's message (FNV-1a of nk, nj, ni)
  };
  Layout layout(Tile& t, const SegFn& fn, bool send, const std::function<bool(int)>& dir_on) {
    Layout L;
    long off = 0;
    for (int d = 0; d < 8; d++) {
      L.start[d] = off; L.count[d] = 0;
      uint64_t h = 1469598103934665603ull;
      auto mix = [&h](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
      if (peer_of(t, d) < 0 || !dir_on(d)) { L.sig[d] = 0; continue; }
      std::vector<Seg> v;
      fn(t, d, send, v);
      for (Seg& s : v) {
        s.off = off;
        off += (long)(s.j2 - s.j1 + 1) * (s.i2 - s.i1 + 1) * s.nk;
        mix((uint64_t)s.nk); mix((uint64_t)(s.j2 - s.j1 + 1)); mix((uint64_t)(s.i2 - s.i1 + 1));
        L.segs.push_back(s);
      }
      L.count[d] = off - L.start[d];
      L.sig[d] = h & 0x7fffffffffffffffull;
    }
    if (off > staging_cap) throw std::runtime_error("rcmdyn: halo staging buffer too small");
    return L;
  }
  void launch_segs(const std::vector<Seg>& segs, double* buf, int unpack) {
    for (size_t a = 0; a < segs.size(); a += MAXSEG) {
      SegList L{};
      L.n = (int)std::min<size_t>(MAXSEG, segs.size() - a);
      for (int q = 0; q < L.n; q++) L.s[q] = segs[a + q];
      KLAUNCH(k_pack_segs, dim3(32, L.n), dim3(256), 0, stream, L, buf, unpack);
    }
  }
  void exchange_generic(const SegFn& fn, const std::function<bool(int)>& send_on,
                        const std::function<bool(int)>& recv_on) {
    if (!halo) return;
    // staging of the stream this exchange is issued on (the two streams' exchanges overlap)
    auto SB = [&](Tile& x) { return on2 ? x.sbuf2 : x.sbuf; };
    auto RB = [&](Tile& x) { return on2 ? x.rbuf2 : x.rbuf; };
    std::vector<Layout> S, R;
    for (auto& t : tiles) {
      S.push_back(layout(t, fn, true, send_on));
      R.push_back(layout(t, fn, false, recv_on));
    }
    for (size_t q = 0; q < tiles.size(); q++) launch_segs(S[q].segs, SB(tiles[q]), 0);
    std::vector<Xfer> sends, recvs;
    for (size_t q = 0; q < tiles.size(); q++) {
      Tile& t = tiles[q];
      for (int d = 0; d < 8; d++) {
        const int p = peer_of(t, d);
        if (p < 0) continue;
        Tile* pt = local_tile(p);
        if (S[q].count[d] && pt && force_rccl && comm) {
          // one-rank communicator: the n-th send to self matches the n-th receive
          const size_t pq = pt - tiles.data();
          if (R[pq].count[OPP[d]] != S[q].count[d]) throw std::runtime_error("rcmdyn: halo size mismatch");
          sends.push_back({comm->rank(), SB(t) + S[q].start[d], (size_t)S[q].count[d], S[q].sig[d]});
          recvs.push_back({comm->rank(), RB(*pt) + R[pq].start[OPP[d]], (size_t)S[q].count[d], R[pq].sig[OPP[d]]});
          continue;
        }
        if (S[q].count[d] && pt) {
          const size_t pq = pt - tiles.data();
          if (R[pq].count[OPP[d]] != S[q].count[d]) throw std::runtime_error("rcmdyn: halo size mismatch");
          DHIPCHK(hipMemcpyAsync(RB(*pt) + R[pq].start[OPP[d]], SB(t) + S[q].start[d],
                                 S[q].count[d] * sizeof(double), hipMemcpyDeviceToDevice, stream));
        }
        if (R[q].count[d] && !pt) recvs.push_back({p, RB(t) + R[q].start[d], (size_t)R[q].count[d], R[q].sig[d]});
      }
      // remote sends in the order of the receiver's directions: the n-th message between two
      // ranks matches the n-th receive, and in a band of two tiles in j one peer is both the
      // left and the right neighbour
      for (int e = 0; e < 8; e++) {
        const int d = OPP[e], p = peer_of(t, d);
        if (p < 0 || !S[q].count[d] || local_tile(p)) continue;
        sends.push_back({p, SB(t) + S[q].start[d], (size_t)S[q].count[d], S[q].sig[d]});
      }
    }
    if (!sends.empty() || !recvs.empty()) {
      if (!comm) throw std::runtime_error("rcmdyn: remote neighbour without a communicator");
      comm->sendrecv(sends, recvs, stream, on2 ? 1 : 0);
    }
    for (size_t q = 0; q < tiles.size(); q++) launch_segs(R[q].segs, RB(tiles[q]), 1);
  }

  Seg field_seg(Tile& t, double* p, int nk, int d, int w, bool send) {
    int b[4];
    box(t.g, d, w, send, b);
    Seg s{};
    s.p = p; s.kstride = t.g.plane; s.pitch = t.g.pitch; s.j0 = t.g.j0; s.i0 = t.g.i0;
    s.j1 = b[0]; s.j2 = b[1]; s.i1 = b[2]; s.i2 = b[3]; s.nk = nk;
    return s;
  }

  // exchange / exchange_lb / exchange_rt of several fields at once
  // One exchange point: every field travels in the same per-neighbour message, each with its
  // own width and sides (0 exchange, 1 exchange_lb, 2 exchange_rt).
  void xch(std::initializer_list<XField> fields, int width = 1, int sides = 0) {
    xchv(std::vector<XField>(fields), width, sides);
  }
  void xchv(std::vector<XField> fs, int width = 1, int sides = 0) {
    if (!halo) return;
    for (XField& x : fs) {
      if (x.width == 0) x.width = width;
      if (x.sides < 0) x.sides = sides;
    }
    auto fn = [&](Tile& t, int d, bool send, std::vector<Seg>& v) {
      for (const XField& x : fs)
        if (recv_dir(x.sides, send ? OPP[d] : d)) v.push_back(field_seg(t, fptr(t, x.f), x.nk, d, x.width, send));
    };
    auto all = [](int) { return true; };
    exchange_generic(fn, all, all);
  }

  // Halo/compute overlap (north star): issue an exchange point on the second
  // stream, forked from the first at this point of the step; the first stream goes on with
  // kernels that do not read these fields' ghost rings and waits for it in xch_join.  Both
  // streams' RCCL calls go to one communicator in the same order on every rank; captured
  // into the step graph as a fork/join.
  void fork_point() {
    if (!halo) return;
    DHIPCHK(hipEventRecord(evfork, stream));
  }
  // one communicator for both streams (RCMDYN_RCCL_CHAN2=one): the second stream's exchange
  // forks after the first stream's preceding exchange instead, so the two grouped calls are
  // never in flight together; the overlap with the kernels that follow stays
  void fork_after_exchange() {
    if (comm && comm->shared_channels()) fork_point();
  }
  void xch_begin(std::vector<XField> fs, int slot = 0) {
    if (!halo) return;
    DHIPCHK(hipStreamWaitEvent(stream2, evfork, 0));
    std::swap(stream, stream2);
    on2 = true;
    try {
      xchv(std::move(fs));
    } catch (...) {
      on2 = false;
      std::swap(stream, stream2);
      throw;
    }
    on2 = false;
    std::swap(stream, stream2);
    DHIPCHK(hipEventRecord(evjoin[slot], stream2));
    join_pending[slot] = true;
  }
  void xch_join(int slot = 0) {
    if (!join_pending[slot]) return;
    DHIPCHK(hipStreamWaitEvent(stream, evjoin[slot], 0));
    join_pending[slot] = false;
  }
  // The round-3 overlap form: every exchange stays on the engine's stream (RCCL calls are
  // captured on the capture's origin stream only; the RCCL 2.26 that torch bundles crashed a
  // captured step whose first exchange ran on the forked stream), and the kernels that read no
  // point of it run on the second stream: side_begin forks the second stream from the engine's
  // at this point and sends the following launches there, side_end records their completion
  // (slot) and sends launches back, side_join makes the engine's stream wait for them.
  void side_begin() {
    if (!halo) return;
    DHIPCHK(hipEventRecord(evfork, stream));
    DHIPCHK(hipStreamWaitEvent(stream2, evfork, 0));
    std::swap(stream, stream2);
  }
  void side_end(int slot) {
    if (!halo) return;
    DHIPCHK(hipEventRecord(evjoin[slot], stream));
    std::swap(stream, stream2);
    join_pending[slot] = true;
  }
  void side_join(int slot) { xch_join(slot); }

  // exchange_lb of xdelh = delh(:,:,l,src) (Main/mod_split.F90:498-499)
  void xch_delh_slot(int l, int src) {
    if (!halo) return;
    const long off = ((long)(src - 1) * cfg.nsplit + (l - 1));
    auto fn = [&](Tile& t, int d, bool send, std::vector<Seg>& v) {
      v.push_back(field_seg(t, t.delh + off * t.g.plane, 1, d, 1, send));
    };
    exchange_generic(fn, [&](int d) { return recv_dir(1, OPP[d]); }, [&](int d) { return recv_dir(1, d); });
  }

  // width-w exchange of 2-D planes held in the tiles' wide frames (fused split step)
  void xch_wide(std::initializer_list<std::pair<double* Tile::*, int>> fields, int w) {
    if (!halo) return;
    std::vector<std::pair<double* Tile::*, int>> fs(fields);
    auto fn = [&](Tile& t, int d, bool send, std::vector<Seg>& v) {
      int b[4];
      box(t.gw, d, w, send, b);
      for (auto& x : fs) {
        Seg sg{};
        sg.p = t.*(x.first); sg.kstride = t.gw.plane; sg.pitch = t.gw.pitch; sg.j0 = t.gw.j0; sg.i0 = t.gw.i0;
        sg.j1 = b[0]; sg.j2 = b[1]; sg.i1 = b[2]; sg.i2 = b[3]; sg.nk = x.second;
        v.push_back(sg);
      }
    };
    auto all = [](int) { return true; };
    exchange_generic(fn, all, all);
  }
  // the fused split step is exact on a decomposition when every tile is at least SPX wide
  // (its depth-SPX halo then comes from the direct neighbours only)
  bool wide_ok() const {
    if (!halo) return true;
    for (const Geom& g : all)
      if (g.jde2 - g.jde1 + 1 < SPX || g.ide2 - g.ide1 + 1 < SPX) return false;
    return true;
  }
  // The decomposed hydrostatic step runs without the post-prologue exchanges when the fused
  // split step applies (every tile at least SPX wide, every mode within SPH sub-steps): its
  // kernels then compute the ghost rings their consumers read.
  bool split_fused() const {
    bool f = wide_ok();
    for (int l = 1; l <= cfg.nsplit; l++) f = f && ((int)hc.aam[l - 1] * 2 <= SPH);
    return f;
  }
  void copy_wide(Tile& t, const double* src, double* dst, int nplanes) {
    KLAUNCH(k_copy_frame, grid3(t.g.jde2 - t.g.jde1 + 1, t.g.ide2 - t.g.ide1 + 1, 1), BLK, 0, stream, t.g, t.gw,
            nplanes, src, (long)t.g.plane, dst, (long)t.gw.plane);
  }

  // exchange_bdy_lr / exchange_bdy_bt of the bdyuv slices (Main/mod_bdycod.F90:1063-1089):
  // south/north slices (by j) with the left/right tiles, west/east slices (by i) with the
  // bottom/top tiles; width 1, every level.
  void xch_slices() {
    if (!halo) return;
    const int kz = cfg.kz;
    auto fn = [&](Tile& t, int d, bool send, std::vector<Seg>& v) {
      const Geom& g = t.g;
      std::vector<int> ids;
      int lo, hi, origin;
      if (d == 0 || d == 1) {
        if (g.bt) ids.insert(ids.end(), {10, 11, 14, 15});
        if (g.bb) ids.insert(ids.end(), {8, 9, 12, 13});
        lo = g.jde1; hi = g.jde2; origin = g.j0;
      } else {
        if (g.bl) ids.insert(ids.end(), {0, 1, 4, 5});
        if (g.br) ids.insert(ids.end(), {2, 3, 6, 7});
        lo = g.ide1; hi = g.ide2; origin = g.i0;
      }
      const bool low = (d == 0 || d == 2);
      const int x = send ? (low ? lo : hi) : (low ? lo - 1 : hi + 1);
      for (int s : ids) {
        Seg sg{};
        sg.p = t.sl[s]; sg.kstride = slen; sg.pitch = 0; sg.j0 = origin; sg.i0 = 0;
        sg.j1 = x; sg.j2 = x; sg.i1 = 0; sg.i2 = 0; sg.nk = kz;
        v.push_back(sg);
      }
    };
    auto on = [&](int d) { return d < 4; };
    exchange_generic(fn, on, on);
  }

  // NH_DPRFORM: the acoustic update forms dprddx / dprddy from atm0%pr as the reference
  // defines them (Main/mod_params.F90:2676-2686); values a host put must be exactly those, or
  // the engine would silently compute with others
  void check_dprd() {
    if (!NH_DPRFORM || cfg.idynamic != 2 || dry) { dprd_put = false; return; }
    int* bad = nullptr;
    HIPCHK(hipMalloc(&bad, sizeof(int)));
    HIPCHK(hipMemsetAsync(bad, 0, sizeof(int), stream));
    for (auto& t : tiles) {
      const Geom& g = t.g;
      KLAUNCH(k_nh_check_dprd, grid3(g.jdi2 - g.jdi1 + 1, g.idi2 - g.idi1 + 1, cfg.kz), BLK, 0, stream, g,
              nhf[&t - tiles.data()], bad);
    }
    int n = 0;
    HIPCHK(hipMemcpyAsync(&n, bad, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    HIPCHK(hipFree(bad));
    // a mismatch stays pending: every later call fails the same way until a put corrects it
    if (n) throw std::runtime_error("rcmdyn: DPRDDX/DPRDDY differ from atm0%pr's four-point differences at " +
                                    std::to_string(n) + " points (Main/mod_params.F90:2676-2686)");
    dprd_put = false;
  }

  // ------------------------------------------------------------------ the step
  template <class F>
  void each(F fn) { for (auto& t : tiles) fn(t); }

  void prepare() {
    if (statics_dirty) {
      xch({{FK::MSFX, 1}, {FK::MSFD, 1}, {FK::HT, 1}, {FK::CORIOL, 1}}, 2, 0);
      each([&](Tile& t) {
        KLAUNCH(k_prepare_static, grid3(t.g.nj, t.g.ni, 1), BLK, 0, stream, t.g, dc, cfg.diffu_hgtf,
                t.msfx, t.msfd, t.ht, t.xmsf, t.dmsf, t.hgfact, t.mapf);
      });
      if (halo) {
        each([&](Tile& t) {
          copy_wide(t, t.msfx, t.wmsfx, 1);
          copy_wide(t, t.msfd, t.wmsfd, 1);
          copy_wide(t, t.mapf, t.wmapf, 1);
        });
        xch_wide({{&Tile::wmsfx, 1}, {&Tile::wmsfd, 1}, {&Tile::wmapf, 1}}, SPX);
      }
      statics_dirty = false;
      invalidate_graphs();
    }
    if (dprd_put) check_dprd();
    if (bdy_dirty) {
      const int kz = cfg.kz;
      // width 2: the ghost-ring kernels relax at ghost points (stencil radius 1)
      xch({{FK::UB0, kz}, {FK::UBT, kz}, {FK::VB0, kz}, {FK::VBT, kz}}, 2, 0);
      xch({{FK::TB0, kz}, {FK::TBT, kz}, {FK::QB0, kz}, {FK::QBT, kz}, {FK::PB0, 1}, {FK::PBT, 1}}, 2, 0);
      bdy_dirty = false;
      invalidate_graphs();
    }
    if (kpbl_dirty) {
      // the physics puts kpbl on its own points (a rank puts its interior); vadv4d ind = 3 of
      // the fused hydrostatic step reads it on the ghost ring k_scalars computes in place of
      // the cqv/cqc exchange (Main/mod_advection.F90:898-925)
      xch({{FK::KPBL, 1}}, 1, 0);
      kpbl_dirty = false;
    }
  }

  // R of a tile: the column-box points whose k_columns work reads no ghost point toward a
  // neighbour (atm1 at j+1 / i+1, p* at +-1, psdot's j-1 / i-1), i.e. the owned points one in
  // from every side that has a neighbour; and the k_momentum / k_scalars blocks whose staged
  // halo-2 tile lies in R (their part-1 blocks, the same test as part_skip)
  void setup_overlap(Tile& t) {
    const Geom& g = t.g;
    t.rja = g.bl ? g.jdx1() : g.jde1 + 1;
    t.rjb = g.br ? g.jdx2() : g.jde2 - 1;
    t.ria = g.bb ? g.idx1() : g.ide1 + 1;
    t.rib = g.bt ? g.idx2() : g.ide2 - 1;
    if (t.rja > t.rjb || t.ria > t.rib) return;
    const long box = (long)(g.jdx2() - g.jdx1() + 1) * (g.idx2() - g.idx1() + 1);
    const long rin = (long)(t.rjb - t.rja + 1) * (t.rib - t.ria + 1);
    t.rnxb = (t.rjb - t.rja + COLW) / COLW;
    t.nint = t.rnxb * (t.rib - t.ria + 1);
    t.nring = (int)((box - rin + COLW - 1) / COLW);
    t.nred = t.nint + t.nring;
    auto inner = [&](int J0, int I0, int bj, int bi) {
      return J0 - 2 >= t.rja && J0 + bj + 1 <= t.rjb && I0 - 2 >= t.ria && I0 + bi + 1 <= t.rib;
    };
    // the block columns of k_momentum / k_scalars start at j1 or, shifted back by 64 - s, at
    // j1 + s - 64 (a partial first column): the origin that puts the most points of the tile in
    // blocks wholly inside R (on a 96-wide tile no default-aligned 64-wide block with its halo
    // fits, and part 1 would be empty)
    const int mj2 = g.br ? g.jdi2 : g.jde2 + 1, mi2 = g.bt ? g.idi2 : g.ide2 + 1;
    auto best = [&](int j1, int j2, int i1, int i2, int BJ, int BI, int& org, long& npts) {
      long top = 0;
      org = j1;
      for (int sft = 0; sft < BJ; sft++) {
        const int o = sft ? j1 + sft - BJ : j1;
        long pts = 0;
        for (int I0 = i1; I0 <= i2; I0 += BI)
          for (int J0 = o; J0 <= j2; J0 += BJ)
            if (inner(J0, I0, BJ, BI))
              pts += (long)(std::min(J0 + BJ - 1, j2) - std::max(J0, j1) + 1) * (std::min(I0 + BI - 1, i2) - I0 + 1);
        if (pts > top) { top = pts; org = o; }
      }
      npts = top;
      return top > 0;
    };
    t.mom_in = best(g.jdi1, mj2, g.idi1, mi2, MBJ, MBI, t.mj0, t.mom_p1);
    t.sca_in = best(g.jcx1(), g.jcx2(), g.icx1(), g.icx2(), SBJ, SBI, t.sj0, t.sca_p1);
  }
  Fields fields(Tile& t, int part) {
    Fields f = fields(t);
    f.pt = Part{part, t.rja, t.rjb, t.ria, t.rib, t.rnxb, t.nint, t.mj0, t.sj0};
    return f;
  }

  // dynamic LDS of the two-phase column kernels: 4 x kz x 64 doubles
  size_t col_lds() const { return sizeof(double) * 4 * COLW * (size_t)cfg.kz; }

  // all buffers of one tile for its current parity (see Fields)
  Fields fields(Tile& t) {
    const int c = t.cur, n = 1 - c, q = thp(t), o = 1 - q;
    Fields f{};
    f.a1u = t.a1u[c]; f.a1v = t.a1v[c]; f.a1t = t.a1t[q]; f.a1qv = t.a1qv[q]; f.a1qc = t.a1qc[q];
    f.a2u = t.a2u[c]; f.a2v = t.a2v[c]; f.a2t = t.a2t[q]; f.a2qv = t.a2qv[q]; f.a2qc = t.a2qc[q];
    f.psa = t.psa_[c]; f.psb = t.psb_[c];
    f.b1u = t.a1u[n]; f.b1v = t.a1v[n]; f.b1t = t.a1t[o]; f.b1qv = t.a1qv[o]; f.b1qc = t.a1qc[o];
    f.b2u = t.a2u[n]; f.b2v = t.a2v[n]; f.b2t = t.a2t[o]; f.b2qv = t.a2qv[o]; f.b2qc = t.a2qc[o];
    f.bpsa = t.psa_[n]; f.bpsb = t.psb_[n];
    f.msfx = t.msfx; f.msfd = t.msfd; f.coriol = t.coriol; f.ht = t.ht; f.xmsf = t.xmsf; f.dmsf = t.dmsf;
    f.hgfact = t.hgfact; f.mapf = t.mapf;
    f.rgcr = t.rgcr; f.rgdt = t.rgdt; f.ibcr = t.ibcr; f.ibdt = t.ibdt;
    f.ub0 = t.ub0; f.ubt = t.ubt; f.vb0 = t.vb0; f.vbt = t.vbt; f.tb0 = t.tb0; f.tbt = t.tbt;
    f.qb0 = t.qb0; f.qbt = t.qbt; f.pb0 = t.pb0; f.pbt = t.pbt;
    f.rpsa = t.rpsa; f.rpsb = t.rpsb; f.rpsda = t.rpsda; f.rpsdb = t.rpsdb; f.psc = t.psc;
    f.psdota = t.psdota; f.psdotb = t.psdotb; f.pten = t.pten; f.ptenn = t.pten + t.g.plane;
    f.qdot = t.qdot; f.phi = t.phi; f.slqv = t.slqv; f.slqc = t.slqc; f.cqv = t.cqv; f.cqc = t.cqc; f.fqv = t.fqv; f.fqc = t.fqc;
    f.d6u = t.d6[0]; f.d6v = t.d6[1]; f.d6t = t.d6[2]; f.d6qv = t.d6[3]; f.d6qc = t.d6[4];
    f.depplane = t.depplane;
    if (diag) {
      f.tten = t.tten; f.uten = t.uten; f.vten = t.vten; f.qvten = t.qvten; f.qcten = t.qcten;
      f.omega = t.omega; f.xkcs = t.xkcs;
    }
    if (cfg.ibltyp == 2) f.xkcs = t.xkcs;     // the TKE diffusion reads xkcf from it
    if (hc.iqxvadv == 3) f.kpbl = t.kpbl;    // vadv4d ind = 3 of qc
    f.tphy = t.phy[0]; f.qvphy = t.phy[1]; f.qcphy = t.phy[2]; f.uphy = t.phy[3]; f.vphy = t.phy[4];
    f.red = red; f.red_off = t.red_off;
    f.qfuse = qfuse() ? 1 : 0; f.negcnt = t.negcnt; f.neglist = t.neglist;
    for (int n = 0; n < hc.nsp; n++) f.qxa1[n] = t.a1qx[n][c];
    if (hc.nsp) f.xkcs = t.xkcs;              // k_qx_tend's diffusion reads the scaled xkc
    return f;
  }

  // the hydrometeors beyond qc (nqx = 5) for the current parity: a* current, b* next (the
  // hydrostatic ping-pong; the NH core updates a* in place)
  QxArgs qx_args(Tile& t, int par = -1) {
    const int c = par < 0 ? t.cur : par, n1 = 1 - c;
    QxArgs q{};
    q.nsp = hc.nsp;
    for (int n = 0; n < hc.nsp; n++) {
      q.a1[n] = t.a1qx[n][c]; q.a2[n] = t.a2qx[n][c];
      const bool nh = cfg.idynamic == 2;
      q.b1[n] = t.a1qx[n][nh ? c : n1]; q.b2[n] = t.a2qx[n][nh ? c : n1];
      q.cq[n] = t.cqx[n]; q.fq[n] = t.fqx[n]; q.sl[n] = t.slqx[n]; q.d6[n] = t.d6qx[n]; q.phy[n] = t.phyx[n];
    }
    q.dep = t.depx;
    q.depf = t.depxf;
    return q;
  }
  // the XField entries of the hydrometeors beyond qc for one kind (A1QX0 ..), width w
  void add_qx(std::vector<XField>& v, FK base, int nk, int w) const {
    for (int n = 0; n < hc.nsp; n++) v.push_back({fkq(base, n), nk, w});
  }

  // istep of sound (Main/mod_sound.F90:201-205) for the host time mirror
  int nh_istep() const {
    int istep = (int)(hs.dt / cfg.nh_dtsmax);
    if (istep < 2) istep = 2;
    if (hs.lcount > 0 && istep < 4) istep = 4;
    return istep;
  }
  // alarm_day (Main/mpplib/mod_timer.F90:277-337): active at the start and at the first step
  // whose start time reaches the next multiple of a day
  bool nh_day_alarm() const { return nh_day_alarm_at(hs.lcount); }
  bool nh_day_alarm_at(long long lc) const {
    const double tnow = (double)lc * cfg.dtsec;
    return lc == 0 || !nh_tmask_valid ||
           std::floor(tnow / 86400.0) != std::floor((tnow - cfg.dtsec) / 86400.0);
  }
  bool nh_tmask_valid = false;

  // tend, non-hydrostatic (Main/mod_tendency.F90:212-616 with idynamic = 2).  Exchange points
  // follow the reference's exchange calls: decouple (atm1 width 1, atm2 width idif, pp, w),
  // compute_omega (cr, qdot), calc_coeff (xkc), the moisture forecast (atmc%qx), and per
  // acoustic sub-step dp'/dp0 with pp, then u and v (Main/mod_sound.F90:262-263, 294-295);
  // the upper radiative condition's estore gather (:496-497) becomes a 6-deep halo.
  void nh_tend(int phase, bool slice) {
    const int kz = cfg.kz, kp = kz + 1;
    const int istep = nh_istep();
    const bool alarm = nh_day_alarm();
    // halo/compute overlap of a whole tend on a decomposed domain: the cr/qdot/xkcr exchange
    // on the second stream beside k_nh_tend_c (which reads them at its own point only), the
    // cqv/cqc exchange beside k_nh_tend_d (which does not read them)
    const bool ovl = halo && !no_overlap && phase == TEND_ALL && !slice && cfg.isladvec != 1;
    // ci1a: the interior cross columns from the 128-B line at or below jci1 (NH_ALIGN)
    struct Grids { dim3 fr, ce1, cek, ci1, cik, cik1, di1, dik, ci1a; };
    auto grids = [&](const Geom& g) {
      const int nce_j = g.jce2 - g.jce1 + 1, nce_i = g.ice2 - g.ice1 + 1;
      const int nci_j = g.jci2 - g.jci1 + 1, nci_i = g.ici2 - g.ici1 + 1;
      const int ndi_j = g.jdi2 - g.jdi1 + 1, ndi_i = g.idi2 - g.idi1 + 1;
      return Grids{grid3(g.nj, g.ni, kp), grid3(nce_j, nce_i, 1), grid3(nce_j, nce_i, kz),
                   grid3(nci_j, nci_i, 1), grid3(nci_j, nci_i, kz), grid3(nci_j, nci_i, kz - 1),
                   grid3(ndi_j, ndi_i, 1), grid3(ndi_j, ndi_i, kz),
                   grid3(nci_j + (NH_ALIGN ? jalign(g, g.jci1) : 0), nci_i, 1)};
    };
    if (phase & TEND_PRE) {
    // isladvec = 1: k_sladv forms ud*msfd two points out (the reference exchanges atmx%ud 2
    // wide, :995-997) and interpolates atm2 qx up to three points out (max(idif, 4), :1073-1075)
    // idiffu = 3: atm2 idif = 3 wide, p*b 4 wide (p*dotb on k_nh_diffu6's 3-deep dot rings)
    const int wd = cfg.idiffu == 3 ? 3 : 2;
    const int wu = cfg.isladvec == 1 ? 2 : 1, wq = std::max(cfg.isladvec == 1 ? 3 : 2, wd);
    // atm2 on the second stream, overlapped with decouple and compute_omega (atm1 only)
    std::vector<XField> pro{{FK::PSA, 1, 3}, {FK::PSB, 1, wd + 1}, {FK::A1U, kz, wu}, {FK::A1V, kz, wu}, {FK::A1T, kz},
                            {FK::A1QV, kz}, {FK::A1QC, kz}, {FK::A1PP, kz}, {FK::A1W, kp}};
    std::vector<XField> pro2{{FK::A2U, kz, wd}, {FK::A2V, kz, wd}, {FK::A2T, kz, wd}, {FK::A2QV, kz, wq},
                             {FK::A2QC, kz, wq}, {FK::A2PP, kz, wd}, {FK::A2W, kp, wd}};
    if (cfg.ibltyp == 2) { pro.push_back({FK::A1TKE, kp, 1}); pro2.push_back({FK::A2TKE, kp, wd}); }
    add_qx(pro, FK::A1QX0, kz, 1);
    add_qx(pro2, FK::A2QX0, kz, wq);
    fork_point();
    xchv(pro);
    fork_after_exchange();
    xch_begin(pro2);
    each([&](Tile& t) {
      const Geom& g = t.g;
      const NHFields f = nhfields(t);
      const Grids q = grids(g);
      KLAUNCH(k_surface_pressures, grid3(g.nj, g.ni, 1), BLK, 0, stream, g, fields(t));
      KLAUNCH(k_nh_decouple, q.fr, BLK, 0, stream, g, dc, f);
      KLAUNCH(k_nh_omega, q.ce1, BLK, 0, stream, g, dc, f);
    });
    xch_join();
    if (cfg.idiffu == 3)       // the tendency kernels compute owned points only: no exchange
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_nh_diffu6, dim3((g.ide2 - g.ide1 + 64) / 64, kp, 6 + hc.nsp), dim3(64), 0, stream, g, dc,
                nhfields(t), qx_args(t));
      });
    each([&](Tile& t) {
      const Geom& g = t.g;
      const NHFields f = nhfields(t);
      const Grids q = grids(g);
      KLAUNCH(k_nh_coeff_raw, NH_XKCOL ? q.ce1 : q.cek, BLK, 0, stream, g, dc, f);
    });
    // ovl: the exchange is issued in TEND_POST, after k_nh_tend_c went to the second stream
    if (!ovl) xch({{FK::NCR, kz}, {FK::QDOT, kp}, {FK::NXKCR, kz}});
    if (slice) run_slice();
    }
    if (!(phase & TEND_POST)) return;
    each([&](Tile& t) {
      const Geom& g = t.g;
      const NHFields f = nhfields(t);
      // init_tendencies (:1227-1240): the zero is the leading summand of each tendency's first
      // writer (k_nh_uv_adv, k_nh_scalar_adv, the iboudy = 4 sponges, k_nh_forecast), which
      // covers every point a later kernel reads.  With diagnostics on, the total tendencies
      // are also zeroed, so a get shows 0 at the points no kernel writes.
      if (diag) {
        const size_t b3 = sizeof(double) * g.plane * kz, b4 = sizeof(double) * g.plane * kp;
        for (double* p : {f.tten, f.qvten, f.qcten, f.uten, f.vten, f.ppten}) HIPCHK(hipMemsetAsync(p, 0, b3, stream));
        HIPCHK(hipMemsetAsync(f.wten, 0, b4, stream));
      }
      if (cfg.isladvec == 1)
        KLAUNCH(k_sladv, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, kz), BLK, 0, stream, g, dc, ds, fields(t),
                qx_args(t));
      // the tendency chains (advection, curvature/adiabatic, boundary, diffusion, forecast)
      if (!ovl) {
        tend_d_launch(t, f, istep);
        tend_c_launch(t, f, istep);
      }
    });
    if (ovl) {
      // second stream: k_nh_tend_c, then (after the cr/qdot/xkcr exchange) k_nh_tend_d; the
      // engine's stream: that exchange, then (after k_nh_tend_c) the cqv/cqc exchange
      side_begin();
      each([&](Tile& t) { tend_c_launch(t, nhfields(t), istep); });
      side_end(0);
      xch({{FK::NCR, kz}, {FK::QDOT, kp}, {FK::NXKCR, kz}});
      side_begin();
      each([&](Tile& t) { tend_d_launch(t, nhfields(t), istep); });
      side_end(1);
      side_join(0);
      xchv(cq_fields());
      side_join(1);
      tke_step();
    } else {
      tke_step();
      xchv(cq_fields());
    }
    each([&](Tile& t) {
      const Geom& g = t.g;
      const NHFields f = nhfields(t);
      const Grids q = grids(g);
      if (hc.nsp) {
        // the hydrometeors beyond qc: their fix and RAW filter in place (they feed nothing
        // else of the step; k_nh_tend_c read atm1 for the water load before)
        KLAUNCH(k_qx_fix, grid3(g.jdx2() - g.jdx1() + 1, g.idx2() - g.idx1() + 1, kz), BLK, 0, stream, g, dc,
                qx_args(t));      // the column box, as the hydrostatic launch: its jci x ici fix
        KLAUNCH(k_qx_serial, dim3(hc.nsp * kz), dim3(negfix_threads(g)), sizeof(double) * negfix_lds(g), stream, g, dc,
                qx_args(t));
        if (NEGFIX_POST)
          KLAUNCH(k_qx_post, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, hc.nsp * kz), BLK, 0, stream, g, dc,
                  qx_args(t));
      }
      if (NH_NEGLIST)
        KLAUNCH(k_nh_negfix, dim3(1024), dim3(256), 0, stream, g, dc, f);
      else
        KLAUNCH(k_nh_negfix, q.cik, BLK, 0, stream, g, dc, f);
      KLAUNCH(k_nh_negfix_serial, dim3(2 * kz), dim3(negfix_threads(g)), sizeof(double) * negfix_lds(g), stream, g, dc, f);
      // tend's time filters (tfuse = 0) with part A of the first acoustic sub-step (sound, :163-718)
      if (NH_A1COL && nh_tfuse)     // part A alone: one column walk per cross column
        KLAUNCH(k_nh_a1_col, q.ce1, BLK, 0, stream, g, dc, f);
      else
        KLAUNCH(k_nh_tfilter_a1, grid3(g.jce2 - g.jce1 + 1, g.ice2 - g.ice1 + 1, kp), BLK, 0, stream, g, dc, f);
    });
    if (nh_tfuse) for (auto& t : tiles) t.tq = 1 - t.tq;     // the filtered t, qv, qc
    // sound, Main/mod_sound.F90:163-718
    for (int it = 1; it <= istep; it++) {
      // part A: sub-step 1 in k_nh_tfilter_a1, the later ones in the previous k_nh_sound_cd
      // the dp'/dp0, pp exchange beside part 1 of k_nh_sound_uv (the points that read no ghost),
      // then the strip of the others
      auto sound_uv = [&](Tile& t, int part) {
        const Geom& g = t.g;
        const int fin = (int)(it == istep), first = (int)(it == 1);
        if (part == 2) {
          const int n = (g.bl ? 0 : g.ide2 - g.ide1 + 1) + (g.bb ? 0 : g.jde2 - g.jde1 + (g.bl ? 0 : 1));
          if (n > 0)
            KLAUNCH(k_nh_sound_uv, dim3((n + 127) / 128, kz), dim3(128), 0, stream, g, dc, ds, nhfields(t), istep,
                    fin, first, 2);
          return;
        }
        KLAUNCH(k_nh_sound_uv, grid3(g.jde2 - g.jde1 + 1 + (NH_ALIGN && !NH_WRAP_PT ? jalign(g, g.jde1) : 0), g.ide2 - g.ide1 + 1, kz),
                BLK, 0, stream, g, dc, ds, nhfields(t), istep, fin, first, part);
      };
      if (halo && !no_overlap) {
        side_begin();
        each([&](Tile& t) { sound_uv(t, 1); });
        side_end(0);
        xch({{FK::NCDT, kz}, {FK::NCPP, kz}});
        side_join(0);
        each([&](Tile& t) { sound_uv(t, 2); });
      } else {
        xch({{FK::NCDT, kz}, {FK::NCPP, kz}});
        each([&](Tile& t) { sound_uv(t, 0); });
      }
      xch({{FK::NCU, kz}, {FK::NCV, kz}});
      each([&](Tile& t) {
        const Geom& g = t.g;
        const NHFields f = nhfields(t);
        const Grids q = grids(g);
        KLAUNCH(k_nh_sound_bc, NH_WRAP ? q.ci1 : q.ci1a, BLK, 0, stream, g, dc, ds, f, istep, it);
      });
      if (cfg.ifupr == 1) {
        if (it == 1 && alarm) {
          each([&](Tile& t) {
            KLAUNCH(k_nh_tmask_gather, grids(t.g).ci1, BLK, 0, stream, t.g, dc, nhfields(t), nh_gbuf);
          });
          if (comm) comm->allreduce_sum(nh_gbuf, 2 * (size_t)cfg.jx * cfg.iy, stream);
          KLAUNCH(k_nh_tmask, dim3(1), dim3(256), 0, stream, tiles[0].g, dc, nh_gbuf, nhf[0].tmask);
          nh_tmask_valid = true;
        }
        if (halo) {
          each([&](Tile& t) { copy_wide(t, nhf[&t - tiles.data()].estore, t.westore, 1); });
          xch_wide({{&Tile::westore, 1}}, 6);
        }
      }
      each([&](Tile& t) {
        const Geom& g = t.g;
        const NHFields f = nhfields(t);
        const Grids q = grids(g);
        if (halo)
          KLAUNCH(k_nh_sound_cd, NH_ALIGN_CD && !NH_WRAP ? q.ci1a : q.ci1, BLK, 0, stream, g, t.gw, t.westore, dc, ds, f, istep, (int)(it == istep),
                  (int)(it < istep));
        else
          KLAUNCH(k_nh_sound_cd, NH_ALIGN_CD && !NH_WRAP ? q.ci1a : q.ci1, BLK, 0, stream, g, g, f.estore, dc, ds, f, istep, (int)(it == istep),
                  (int)(it < istep));
      });
    }
    each([&](Tile& t) {
      KLAUNCH(k_nh_sound_final, dim3((nh_frame_ring(t.g) + 255) / 256, kz + 1), dim3(256), 0, stream, t.g, dc,
              nhfields(t));
    });
    KLAUNCH(k_nh_advance, dim3(1), dim3(256), 0, stream, dc, ds, nhf[0]);
    hs.lcount += 1;
    if (hs.lcount == 2) hs.dt = 2.0 * cfg.dtsec;
  }

  void tend_d_launch(Tile& t, const NHFields& f, int istep) {
    const Geom& g = t.g;
    const dim3 gd((g.jdi2 - g.jdi1 + 64) / 64, (g.idi2 - g.idi1 + TD_I) / TD_I, cfg.kz);
    KLAUNCH(k_nh_tend_d, NH_ZFIRST ? dim3(gd.z, gd.x, gd.y) : gd, dim3(64, TD_I), 0, stream, g, dc, ds, f, istep);
  }
  void tend_c_launch(Tile& t, const NHFields& f, int istep) {
    const Geom& g = t.g;
    const dim3 gc((g.nj + TC_J - 1) / TC_J, (g.ni + TC_I - 1) / TC_I, cfg.kz + 1);
    if (hc.nsp) {
      KLAUNCH(k_nh_tend_c<true>, NH_ZFIRST ? dim3(gc.z, gc.x, gc.y) : gc, dim3(TC_J, TC_I), 0, stream, g, dc, ds, f,
              (int)diag, istep);
      // the chains of qi, qr, qs after it on the same stream
      KLAUNCH(k_nh_qx_tend, grid3(g.jce2 - g.jce1 + 1, g.ice2 - g.ice1 + 1, cfg.kz), BLK, 0, stream, g, dc, ds, f,
              qx_args(t));
    } else {
      KLAUNCH(k_nh_tend_c<false>, NH_ZFIRST ? dim3(gc.z, gc.x, gc.y) : gc, dim3(TC_J, TC_I), 0, stream, g, dc, ds, f,
              (int)diag, istep);
    }
  }
  // the forecasts exchanged after the tendency kernels (atmc%qx, :381)
  std::vector<XField> cq_fields() const {
    std::vector<XField> v{{FK::CQV, cfg.kz}, {FK::CQC, cfg.kz}};
    add_qx(v, FK::CQX0, cfg.kz, 1);
    return v;
  }

  // bdyval, non-hydrostatic: u, v, t, qv as the hydrostatic core (p* untouched), pp and w,
  // then the moisture inflow/outflow rules and the clock
  void nh_bdyval() {
    const int kz = cfg.kz;
    auto slices = [&](Tile& t) {
      Slices sl;
      for (int q = 0; q < 16; q++) sl.s[q] = t.sl[q];
      return sl;
    };
    each([&](Tile& t) {
      const Geom& g = t.g;
      KLAUNCH(k_bdyval_set, dim3((std::max(g.jde2 - g.jde1, g.ide2 - g.ide1) + 65) / 64, 6, kz), dim3(64), 0,
              stream, g, ds, bdy_args(t, 0));
      const int nperim = 2 * (g.ici2 - g.ici1 + 1) + 2 * (g.jce2 - g.jce1 + 1);
      KLAUNCH(k_nh_bdyval, dim3((nperim + 63) / 64, kz + 1), dim3(64), 0, stream, g, kz, ds, nhfields(t));
      KLAUNCH(k_nh_bdyval_w1, dim3(1), dim3(256), 0, stream, g, nhfields(t));
    });
    xch_slices();
    for (size_t q = 0; q < tiles.size(); q++) {
      Tile& t = tiles[q];
      const int c = t.cur;
      if (hc.nsp)
        KLAUNCH(k_bdyval_qx, dim3(kz, hc.nsp), dim3(256), 0, stream, t.g, ds, qx_args(t), -1, (int)!cfg.present_qc,
                t.psa_[c], slices(t), slen);
      KLAUNCH(k_bdyval_qc, dim3(kz), dim3(256), 0, stream, t.g, (int)!cfg.present_qc, (int)(cfg.iboudy == 3 || cfg.iboudy == 4),
              t.a1qc[thp(t)], t.a1qv[thp(t)], t.psa_[c], slices(t), slen, ds, cfg.dtsec, (int)(q + 1 == tiles.size()),
              dflags);
    }
    tke_bdyval();
    hs.xbctime = hs.xbctime + cfg.dtsec;
  }

  // tend in two phases split where the reference calls physical_parametrizations
  // (Main/mod_tendency.F90:271): TEND_PRE runs surface_pressures .. new_pressure (and the
  // mkslice export when `slice`), TEND_POST the rest; a step runs both.
  static constexpr int TEND_PRE = 1, TEND_POST = 2, TEND_ALL = 3;
  void tend(int phase = TEND_ALL, bool slice = false) {
    if (cfg.idynamic == 2) nh_tend(phase, slice);
    else {
      // part 1 of k_momentum / k_scalars beside the prologue exchange only in a whole tend (no
      // host work between) without the semi-Lagrangian pass that precedes them
      if (phase & TEND_PRE) tend_pre(slice, phase == TEND_ALL && !slice && cfg.isladvec != 1);
      if (phase & TEND_POST) tend_post();
    }
    // the hydrostatic step's snapshot is written by k_split_correct's clock lane
    if ((phase & TEND_POST) && cfg.idynamic == 2) KLAUNCH(k_flag_snapshot, dim3(1), dim3(64), 0, stream, ds, dflags);
  }

  void tend_pre(bool slice, bool with_post = false) {
    const int kz = cfg.kz;
    // One exchange point for the whole prologue (Main/mod_tendency.F90:815-1116,
    // Main/mod_slice.F90:102-300): the decoupled fields are recomputed where read, so their
    // exchanges become exchanges of atm1 (width 1) and atm2 (idif = 2); p* travels 3 wide so
    // psdot and its reciprocals are formed on the ghost ring locally (no psdot exchanges).
    // atm1 travels 2 wide and atm2 3 wide: one more than the reference's widths, for the
    // ghost rings the kernels below compute in place of the later exchanges.
    // Halo/compute overlap (overlap()): the exchange on the engine's stream, part 1 of
    // k_columns (and of k_momentum / k_scalars) on the second; RCMDYN_NO_OVERLAP: the atm2 part
    // on the second stream beside k_columns, which reads only atm1 and p*.
    // (idiffu = 3: p*b 4 wide, for p*dotb on k_diffu6's 3-deep dot ghost rings)
    std::vector<XField> pro{{FK::PSA, 1, 3}, {FK::PSB, 1, cfg.idiffu == 3 ? 4 : 3}, {FK::A1U, kz, 2}, {FK::A1V, kz, 2},
                            {FK::A1T, kz, 2}, {FK::A1QV, kz, 2}, {FK::A1QC, kz, 2}};
    std::vector<XField> pro2{{FK::A2U, kz, 3}, {FK::A2V, kz, 3}, {FK::A2T, kz, 3}, {FK::A2QV, kz, 3},
                             {FK::A2QC, kz, 3}};
    add_qx(pro, FK::A1QX0, kz, 2);        // nqx = 5: qi, qr, qs with qc
    add_qx(pro2, FK::A2QX0, kz, 3);
    // UW TKE: atm1 1 wide, atm2 idif wide (Main/mod_tendency.F90:871, 1079)
    if (cfg.ibltyp == 2) {
      pro.push_back({FK::A1TKE, kz + 1, 1});
      pro2.push_back({FK::A2TKE, kz + 1, cfg.idiffu == 3 ? 3 : 2});
    }
    // surface_pressures + 2-D reciprocals (:815-834), compute_omega columns, new_pressure,
    // geopotential in one launch (calc_coeff is formed where it is read, in k_momentum and
    // k_scalars)
    // ring: the trailing blocks too (the frame points outside the column box, then with qfuse
    // the copies of keep_point on the box's two outer rows and columns, every level)
    auto columns = [&](Tile& t, int part, int ncol, bool ring) {
      const Geom& g = t.g;
      int nsp = 0;
      if (ring) {
        const int W = g.jdx2() - g.jdx1() + 1, H = g.idx2() - g.idx1() + 1;
        const long nkeep = qfuse() ? (long)(4 * W + 4 * std::max(H - 4, 0)) * kz : 0;
        nsp = (int)((g.nj * (long)g.ni + COLT - 1) / COLT + (nkeep + COLT - 1) / COLT);
      }
      if (hc.nsp)
        KLAUNCH(k_columns<true>, dim3(ncol + nsp), dim3(COLT), col_lds(), stream, g, dc, ds, fields(t, part), t.ncolx, ncol);
      else
        KLAUNCH(k_columns<false>, dim3(ncol + nsp), dim3(COLT), col_lds(), stream, g, dc, ds, fields(t, part), t.ncolx, ncol);
    };
    if (overlap()) {
      // the whole exchange on the second stream; meanwhile part 1 of k_columns and, in a whole
      // step (k_momentum / k_scalars follow with no host work between), of k_momentum and
      // k_scalars; part 2 of each after the join
      pro.insert(pro.end(), pro2.begin(), pro2.end());
      side_begin();
      each([&](Tile& t) { if (t.nint) columns(t, 1, t.nint, false); });
      post_inner = with_post;
      if (with_post) each([&](Tile& t) { post_launch(t, 1); });
      side_end(0);
      xchv(pro);
      ghosts_stale = false;
      side_join(0);
      each([&](Tile& t) { columns(t, t.nint ? 2 : 0, t.nint ? t.nring : t.nred, true); });
    } else {
      fork_point();
      xchv(pro);
      fork_after_exchange();
      xch_begin(pro2);
      ghosts_stale = false;
      each([&](Tile& t) { columns(t, 0, t.nred, true); });
      xch_join();
    }
    if (cfg.idiffu == 3) diffu6();
    if (slice) run_slice();
  }

  // idiffu = 3: the column terms of every tile, then (decomposed) one width-1 exchange so the
  // ring k_momentum / k_scalars compute holds the left neighbour's column as it computes it
  void diffu6() {
    const int kz = cfg.kz;
    each([&](Tile& t) {
      const Geom& g = t.g;
      KLAUNCH(k_diffu6, dim3((g.ide2 - g.ide1 + 64) / 64, kz, 4 + hc.nsp), dim3(64), 0, stream, g, dc, fields(t),
              qx_args(t));
    });
    if (halo) {
      std::vector<XField> d6{{FK::D6U, kz}, {FK::D6V, kz}, {FK::D6T, kz}, {FK::D6QV, kz}, {FK::D6QC, kz}};
      add_qx(d6, FK::D6QX0, kz, 0);
      xchv(d6);
    }
  }

  // k_momentum and k_scalars of one tile: part 1 the blocks in R (when it has any), part 2 the
  // others; part 0 all
  void post_launch(Tile& t, int part) {
    const Geom& g = t.g;
    const int mj2 = g.br ? g.jdi2 : g.jde2 + 1, mi2 = g.bt ? g.idi2 : g.ide2 + 1;
    const int pm = part == 0 ? 0 : (t.nint && t.mom_in ? part : (part == 1 ? -1 : 0));
    const int ps = part == 0 ? 0 : (t.nint && t.sca_in ? part : (part == 1 ? -1 : 0));
    const int mo = pm > 0 ? t.mj0 : g.jdi1, so = ps > 0 ? t.sj0 : g.jcx1();     // block-column origins
    if (fuse_update && pm >= 0 && ps >= 0) {
      const int mnx = (mj2 - mo + MBJ) / MBJ, mny = (mi2 - g.idi1 + MBI) / MBI;
      const int snx = (g.jcx2() - so + SBJ) / SBJ, sny = (g.icx2() - g.icx1() + SBI) / SBI;
      KLAUNCH(k_update, dim3(std::max(mnx, snx), std::max(mny, sny), 2 * cfg.kz), dim3(SBT), 0, stream, g, dc, ds,
              fields(t, pm), fields(t, ps), mnx, mny, snx, sny,
              (int)((long)(g.jde2 - g.jde1 + 1) * (g.ide2 - g.ide1 + 1) < UPD_XCD_BELOW));
      return;
    }
    if (pm >= 0)
      KLAUNCH(k_momentum, dim3((mj2 - mo + MBJ) / MBJ, (mi2 - g.idi1 + MBI) / MBI, cfg.kz), dim3(MBT), 0,
              stream, g, dc, ds, fields(t, pm));
    if (ps >= 0)
      KLAUNCH(k_scalars, dim3((g.jcx2() - so + SBJ) / SBJ, (g.icx2() - g.icx1() + SBI) / SBI, cfg.kz),
              dim3(SBT), 0, stream, g, dc, ds, fields(t, ps));
  }

  void tend_post() {
    const int kz = cfg.kz, ns = cfg.nsplit;
    const bool fused = split_fused();
    // semi-Lagrangian moisture advection (isladvec = 1): owned points, then the ring k_scalars
    // also computes comes from the neighbours
    if (cfg.isladvec == 1) {
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_sladv, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, kz), BLK, 0, stream, g, dc, ds, fields(t),
                qx_args(t));
      });
      std::vector<XField> sl{{FK::SLQV, kz}, {FK::SLQC, kz}};
      add_qx(sl, FK::SLQX0, kz, 0);
      xchv(sl, 1, 0);
    }
    // fused tendencies + forecast + time filter (part 2 when tend_pre ran part 1)
    each([&](Tile& t) { post_launch(t, post_inner ? 2 : 0); });
    post_inner = false;
    tke_step();
    if (hc.nsp) {
      // nqx = 5: the hydrometeors beyond qc, their forecast (and ring), then the fix and filter
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_qx_tend, dim3((g.jcx2() - g.jcx1() + QBJ) / QBJ, (g.icx2() - g.icx1() + QBI) / QBI, kz), dim3(QBT),
                0, stream, g, dc, ds, fields(t), qx_args(t));
      });
      if (!fused) {
        std::vector<XField> cq;
        add_qx(cq, FK::CQX0, kz, 1);
        xchv(cq);
      }
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_qx_fix, grid3(g.jdx2() - g.jdx1() + 1, g.idx2() - g.idx1() + 1, kz), BLK, 0, stream, g, dc,
                qx_args(t));
        if (serial_with_corr()) return;          // the serial chains then run in launch_corrections
        KLAUNCH(k_qx_serial, dim3(hc.nsp * kz), dim3(negfix_threads(g)), sizeof(double) * negfix_lds(g), stream, g, dc,
                qx_args(t));
        if (NEGFIX_POST)
          KLAUNCH(k_qx_post, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, hc.nsp * kz), BLK, 0, stream, g, dc,
                  qx_args(t));
      });
    }
    if (!fused) xch({{FK::CQV, kz}, {FK::CQC, kz}});     // else k_scalars computed the ring
    // negative-moisture fix + p* RA filter + qv/qc RAW filter; then the new level is current
    // (qfuse: done by k_columns, k_scalars and the extra blocks below)
    each([&](Tile& t) {
      if (!qfuse()) KLAUNCH(k_qfilter, grid3((t.g.nj + 1) / 2, t.g.ni, kz), BLK, 0, stream, t.g, dc, fields(t));
      t.cur = 1 - t.cur;
    });
    // splitf, Main/mod_split.F90:243-461
    if (!fused) xch({{FK::PSA, 1}, {FK::A1U, kz, 1, 2}, {FK::A1V, kz, 1, 2}, {FK::A2U, kz, 1, 2}, {FK::A2V, kz, 1, 2}});
    const bool wide = fused && halo;     // k_split_project also fills the wide frames
    each([&](Tile& t) {
      const Geom& g = t.g;
      const int c = t.cur, o = 1 - c;
      const QFix q = qfix(t);
      const int nxp = (g.jdx2() - g.jde1 + SPC) / SPC, nproj = nxp * (g.idx2() - g.ide1 + 1);
      // extra blocks: qfuse the parallel fix of the listed negatives (grid-stride), else the
      // serial sweeps of the planes k_qfilter flagged
      const int nextra = qfuse() ? NEGFIX_BLOCKS * 512 / (SPC * SPG) : 2 * kz;   // 32 768 threads
      KLAUNCH(k_split_project, dim3(nproj + nextra), dim3(SPC * SPG), sizeof(double) * 4 * SPC * (size_t)kz, stream, g,
              dc, t.a1u[c], t.a1v[c],
                         t.a2u[c], t.a2v[c], t.a1t[c], t.a2t[c], t.psa_[c], t.psb_[c], t.msfd, t.mapf, t.dstor,
                         t.hstor, t.deld, t.delh, t.psdota, nxp, nproj, q, t.gw, wide ? t.wdeld : nullptr,
                         t.wdelh, t.wpsdota, t.wpsa, t.a2u[o], t.a2v[o]);
    });
    // spstep, :463-669: forward step then leapfrog, two time slots + forcing slot 3
    if (wide) {
      // one depth-SPX exchange of every split-step input instead of three per sub-step
      xch_wide({{&Tile::wdeld, 3 * ns}, {&Tile::wdelh, 3 * ns}, {&Tile::wpsa, 1}, {&Tile::wpsdota, 1}}, SPX);
    }
    if (fused) {
      each([&](Tile& t) {
        const Geom& g = t.g;
        // 16 x 16 owned points per block, or 8 x 8 when that leaves most CUs idle (a rank tile
        // of a multi-GPU run): the sub-step chain is the block's latency, and 8 x 8 blocks cut
        // it per block (576 region points instead of 1024) at the price of more halo points
        const int W = g.jcx2() - g.jcx1() + 1, H = g.icx2() - g.icx1() + 1;
        const bool small = (long)((W + 15) / 16) * ((H + 15) / 16) * ns < SP8_BELOW;
        const Geom& w = halo ? t.gw : g;
        const double *dd = halo ? t.wdeld : t.deld, *dh = halo ? t.wdelh : t.delh;
        const double *mx = halo ? t.wmsfx : t.msfx, *md = halo ? t.wmsfd : t.msfd;
        const double *pd = halo ? t.wpsdota : t.psdota, *mp = halo ? t.wmapf : t.mapf;
        const double* pa = halo ? t.wpsa : t.psa_[t.cur];
        if (small)
          KLAUNCH(k_spstep_fused<8>, dim3((W + 7) / 8, (H + 7) / 8, ns), dim3(8 + 2 * SPH, 8 + 2 * SPH), 0, stream, g, w,
                  dc, dd, dh, mx, md, pd, mp, pa, t.ddsum, t.dhsum);
        else
          KLAUNCH(k_spstep_fused<16>, dim3((W + 15) / 16, (H + 15) / 16, ns), dim3(16 + 2 * SPH, 16 + 2 * SPH), 0,
                  stream, g, w, dc, dd, dh, mx, md, pd, mp, pa, t.ddsum, t.dhsum);
      });
    } else {
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_spstep_init, grid3(g.jde2 - g.jde1 + 1, g.ide2 - g.ide1 + 1, 1), BLK, 0, stream, g,
                           dc, t.deld, t.delh, t.ddsum, t.dhsum);
      });
    }
    for (int l = 1; l <= ns && !fused; l++) {
      int n0 = 1, n1 = 2, n2 = n0;
      const int m2 = (int)hc.aam[l - 1] * 2;
      sp_substep(l, n0, n0, n0, n1, 0);
      for (int n = 2; n <= m2; n++) {
        sp_substep(l, n1, n0, n1, n2, 1);
        n0 = n1; n1 = n2; n2 = n0;
      }
    }
    // the fused split step also produced ddsum/dhsum on the left/bottom ghost ring
    if (!fused) xch({{FK::DHSUM, ns}}, 1, 1);
    // corrections + rcmtimer advance (last tile's launch); deferred to bdyval in the drop-in pair
    if (defer_corr && !fuse_bdy) corr_pending = true;
    else launch_corrections(fuse_bdy);
    hs.lcount += 1;
    if (hs.lcount == 2) hs.dt = 2.0 * cfg.dtsec;
  }

  // the split corrections + rcmtimer advance (last tile's launch); bdy: with bdyval's boundary
  // lines (k_split_correct_bdy; k_bdyval_qc then advances the clock)
  void launch_corrections(bool bdy) {
    const int kz = cfg.kz, ns = cfg.nsplit;
    for (size_t q = 0; q < tiles.size(); q++) {
      Tile& t = tiles[q];
      const Geom& g = t.g;
      const int c = t.cur;
      const long npts = (long)((g.jdx2() - g.jde1 + 2) / 2) * (g.idx2() - g.ide1 + 1);   // point pairs per level
      dim3 gr = SCOR_FLAT ? dim3((unsigned)((npts + 255) / 256), 1, kz)
                          : grid3((g.jdx2() - g.jde1 + 2) / 2, g.idx2() - g.ide1 + 1, kz);
      const int adv = (int)(q + 1 == tiles.size());
      // qfuse: trailing z slices run the serial sweeps of the flagged moisture planes
      const QFix qf = qfix(t);
      // (nqx = 5: in a launch of their own after the corrections, k_negfix_serial, whose block per
      // plane can run the dense wavefront; the patchy hydrometeor fields come with patchy qc)
      const bool own = hc.nsp > 0;
      const int nser = qfuse() && !own ? (int)((2 * kz + gr.x * gr.y - 1) / (gr.x * gr.y)) : 0;
      gr.z += nser;
      const size_t slds = nser ? sizeof(double) * negfix_sweep_lds(g) : 0;     // the sweeps' LDS (row sweeps only)
      if (bdy) {
        // the bdyval blocks: leading z slices of 6 lines x bdy_chunks 64-point chunks x kz
        // levels, 4 per block
        const unsigned per = 4 * gr.x * gr.y;
        gr.z += (6 * bdy_chunks(g) * kz + per - 1) / per;
        const BdyArgs ba = bdy_args(t, 1);
#define RCM_SCB(NS_) KLAUNCH(k_split_correct_bdy<NS_>, gr, BLK, slds, stream, g, dc, t.ddsum, t.dhsum, t.psdota, t.msfd, \
                             ds, adv, red, red_total, ba, qf, nser)
        switch (ns) { case 1: RCM_SCB(1); break; case 2: RCM_SCB(2); break; case 3: RCM_SCB(3); break; default: RCM_SCB(4); }
#undef RCM_SCB
      } else {
#define RCM_SC(NS_) KLAUNCH(k_split_correct<NS_>, gr, BLK, slds, stream, g, dc, t.ddsum, t.dhsum, t.psdota, t.msfd,   \
                            t.psa_[c], t.psb_[c], t.a1t[c], t.a2t[c], t.a1u[c], t.a1v[c], t.a2u[c], t.a2v[c], ds, adv, \
                            red, red_total, dflags, qf, nser)
        switch (ns) { case 1: RCM_SC(1); break; case 2: RCM_SC(2); break; case 3: RCM_SC(3); break; default: RCM_SC(4); }
#undef RCM_SC
      }
      if (serial_with_corr()) {
        // the qv / qc and the species planes' serial chains in one launch (the species' operands
        // of the step before tend_post's flip), then their filters
        const QxArgs qx = qx_args(t, 1 - t.cur);
        KLAUNCH(k_negfix_serial_qx, dim3((2 + hc.nsp) * kz), dim3(negfix_threads(g)), sizeof(double) * negfix_lds(g),
                stream, g, dc, qf, qx);
        KLAUNCH(k_negfix_post, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, 2 * kz), BLK, 0, stream, g, dc, qf);
        KLAUNCH(k_qx_post, grid3(g.jci2 - g.jci1 + 1, g.ici2 - g.ici1 + 1, hc.nsp * kz), BLK, 0, stream, g, dc, qx);
      } else if (qfuse() && own) {
        KLAUNCH(k_negfix_serial, dim3(2 * kz), dim3(negfix_threads(g)), sizeof(double) * negfix_lds(g), stream, g, dc,
                qf);
      }
    }
  }
  // not with a communicator: a rank-local call (a get) between tend and bdyval would then issue
  // the step's flag reduction on one rank only
  bool can_defer() const {
    return cfg.idynamic != 2 && !comm && !no_fuse_bdy && !no_defer_corr && (!halo || split_fused());
  }
  // a call other than rcmdyn_bdyval after a tend that deferred its corrections: launch them
  void settle() {
    if (tend_pending) {              // the lazy tend's own graph (captured with deferred corrections)
      inject_launch_failure();
      HIPCHK(hipGraphLaunch(gtend[lazy_par], stream));
      tend_pending = false;          // only once launched: a failed launch leaves the tend pending
      corr_pending = true;
    }
    if (!corr_pending) return;
    launch_corrections(false);     // if this throws, the corrections stay pending for the next call
    corr_pending = false;
    note_step(hs.lcount);
  }
  // rcmdyn_bdyval after a deferring tend: the corrections with the boundary lines, then the
  // rest of bdyval as rcmdyn_step runs it
  void fused_bdyval() {
    fuse_bdy = true;
    try {
      launch_corrections(true);
      corr_pending = false;
      bdyval();
    } catch (...) {
      fuse_bdy = false;
      throw;
    }
    fuse_bdy = false;
  }

  // one spstep substep: gradient of delh(src) -> (uu,vv) -> divergence -> mode update
  void sp_substep(int l, int src, int n0, int n1, int nn, int leap) {
    xch_delh_slot(l, src);
    each([&](Tile& t) {
      const Geom& g = t.g;
      KLAUNCH(k_spstep_grad, grid3(g.jdi2 - g.jdi1 + 1, g.idi2 - g.idi1 + 1, 1), BLK, 0, stream, g, dc, l,
                         src, t.delh, t.msfx, t.msfd, t.psdota, t.uu, t.vv);
    });
    xch({{FK::UU, 1}, {FK::VV, 1}}, 1, 2);
    each([&](Tile& t) {
      const Geom& g = t.g;
      KLAUNCH(k_spstep_update, grid3(g.jce2 - g.jce1 + 1, g.ice2 - g.ice1 + 1, 1), BLK, 0, stream, g, dc,
                         l, n0, n1, nn, leap, t.uu, t.vv, t.mapf, t.psa_[t.cur], t.deld, t.delh, t.ddsum, t.dhsum);
    });
  }

  // the moisture fix-up operands for the current parity (after the flip of tend_post): the
  // forecasts and fixed values, the old (o*) and new (n*) q buffers, the filtered p*
  QFix qfix(Tile& t) {
    const int c = t.cur, o = 1 - c;
    QFix q{t.cqv, t.cqc, t.fqv, t.fqc, t.a1qv[o], t.a1qc[o], t.a2qv[o], t.a2qc[o],
           t.a1qv[c], t.a1qc[c], t.a2qv[c], t.a2qc[c], t.psa_[c], t.psb_[c], t.psc, t.psa_[o], t.psb_[o],
           t.depplane, nullptr, nullptr, nullptr};
    if (qfuse()) { q.negcnt = t.negcnt; q.neglist = t.neglist; q.depf = t.depqf; }
    return q;
  }

  BdyArgs bdy_args(Tile& t, int set_ps) {
    const int c = t.cur, q = thp(t);
    BdyArgs a{};
    a.a1u = t.a1u[c]; a.a1v = t.a1v[c]; a.a1t = t.a1t[q]; a.a1qv = t.a1qv[q]; a.a1qc = t.a1qc[q];
    a.a2u = t.a2u[c]; a.a2v = t.a2v[c]; a.a2t = t.a2t[q]; a.a2qv = t.a2qv[q]; a.a2qc = t.a2qc[q];
    a.psa = t.psa_[c]; a.psb = t.psb_[c];
    a.ub0 = t.ub0; a.ubt = t.ubt; a.vb0 = t.vb0; a.vbt = t.vbt; a.tb0 = t.tb0; a.tbt = t.tbt;
    a.qb0 = t.qb0; a.qbt = t.qbt; a.pb0 = t.pb0; a.pbt = t.pbt;
    for (int q = 0; q < 16; q++) a.sl.s[q] = t.sl[q];
    a.slen = slen;
    a.set_ps = set_ps;
    return a;
  }

  void bdyval() {
    if (cfg.idynamic == 2) { nh_bdyval(); return; }
    const int kz = cfg.kz;
    // fused (step_once): the boundary lines and slices were set by k_split_correct_bdy, and
    // the clock advance of the step moves here (last tile's launch)
    if (!fuse_bdy) {
      each([&](Tile& t) {
        const Geom& g = t.g;
        KLAUNCH(k_bdyval_set, dim3((std::max(g.jde2 - g.jde1, g.ide2 - g.ide1) + 65) / 64, 6, kz), dim3(64), 0,
                stream, g, ds, bdy_args(t, 1));
      });
      // the ghost-ring step wrote the slice entries past the tile itself (k_bdyval_set)
      if (ghosts_stale || !split_fused()) xch_slices();
    }
    for (size_t q = 0; q < tiles.size(); q++) {
      Tile& t = tiles[q];
      const int adv = q + 1 == tiles.size() ? (fuse_bdy ? 2 : 1) : 0;
      if (hc.nsp)
        KLAUNCH(k_bdyval_qx, dim3(kz, hc.nsp), dim3(256), 0, stream, t.g, ds, qx_args(t), fuse_bdy ? 1 : -1,
                (int)!cfg.present_qc, t.psa_[t.cur], bdy_args(t, 1).sl, slen);
      KLAUNCH(k_bdyval_qc, dim3(kz), dim3(256), 0, stream, t.g, (int)!cfg.present_qc, (int)(cfg.iboudy == 3 || cfg.iboudy == 4),
              t.a1qc[t.cur], t.a1qv[t.cur], t.psa_[t.cur], bdy_args(t, 1).sl, slen, ds, cfg.dtsec, adv, dflags);
    }
    tke_bdyval();
    hs.xbctime = hs.xbctime + cfg.dtsec;
  }

  // one tend + bdyval of rcmdyn_step (no host work between them): the hydrostatic bdyval's
  // boundary lines and slices then run in k_split_correct_bdy, only its moisture
  // inflow/outflow pass in a launch of its own.  A decomposed domain needs no slice exchange
  // then (split_fused: every tile computes its ghost ring).
  void step_once() {
    fuse_bdy = cfg.idynamic != 2 && !no_fuse_bdy && (!halo || split_fused());
    try {
      tend();
      bdyval();
    } catch (...) {
      fuse_bdy = false;
      throw;
    }
    fuse_bdy = false;
  }

  // ------------------------------------------------------------------ graph replay
  // graph replay applies: not profiling, not an RCCL transport that cannot be captured, and
  // for NH not a step of another shape (istep on the first two steps, the day alarm's
  // radiative coefficients)
  bool graph_ok(int nsteps = 1) const {
    if (no_graph || prof || (comm && !comm->graph_safe())) return false;
    if (cfg.idynamic != 2) return true;
    for (int q = 0; q < nsteps; q++)
      if (hs.lcount + q < 2 || nh_day_alarm_at(hs.lcount + q)) return false;
    return true;
  }
  // host bookkeeping of a replayed tend / bdyval (what tend() and bdyval() do on the host)
  void replayed_tend() {
    if (cfg.idynamic != 2) for (auto& t : tiles) t.cur = 1 - t.cur;
    else if (nh_tfuse) for (auto& t : tiles) t.tq = 1 - t.tq;
    hs.lcount += 1;
    if (hs.lcount == 2) hs.dt = 2.0 * cfg.dtsec;
  }
  void replayed_bdyval() { hs.xbctime = hs.xbctime + cfg.dtsec; }

  void step(int n) {
    prepare();
    settle();
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, stream));
    for (int s = 0; s < n; s++) {
      check(FLAG_LAG);
      const int par = gpar();
      if (graph_steps == 2 && s + 1 < n && graph_ok(2)) {
        if (!gexec2[par]) capture(par, 3, 2);
        HIPCHK(hipGraphLaunch(gexec2[par], stream));
        replayed_tend();
        replayed_bdyval();
        note_step(hs.lcount);
        replayed_tend();
        replayed_bdyval();
        s++;
      } else if (graph_ok()) {
        if (!gexec[par]) capture(par, 3);
        HIPCHK(hipGraphLaunch(gexec[par], stream));
        replayed_tend();
        replayed_bdyval();
      } else {
        step_once();
      }
      note_step(hs.lcount, s == n - 1);
    }
    HIPCHK(hipEventRecord(e1, stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    last_ms = n > 0 ? (double)ms / n : 0.0;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    check(0);
  }

  // the drop-in call sequence of RCM_run (Main/mod_regcm_interface.F90:189,208): each call
  // replays its own captured graph and returns without synchronising the stream
  void tend_call() {
    prepare();
    settle();
    check(FLAG_LAG);
    const int par = gpar();
    defer_corr = can_defer();
    try {
      if (graph_ok()) {
        if (!gtend[par]) capture(par, 1);
        if (lazy_tend && defer_corr && !ghosts_stale) {
          if (!gexec[par]) {
            defer_corr = false;          // the step graph runs tend with its corrections
            capture(par, 3);
          }
          defer_corr = false;
          tend_pending = true;
          lazy_par = par;
          replayed_tend();               // the clock and parities as after the launch
          return;                        // note_step: at the launch
        }
        HIPCHK(hipGraphLaunch(gtend[par], stream));
        replayed_tend();
        corr_pending = defer_corr;
      } else {
        tend();
      }
    } catch (...) {
      defer_corr = false;
      throw;
    }
    defer_corr = false;
    if (!corr_pending) note_step(hs.lcount);     // else at the corrections' launch
  }
  void bdyval_call() {
    prepare();
    if (tend_pending) {              // the lazy tend and this bdyval: one step graph
      inject_launch_failure();
      HIPCHK(hipGraphLaunch(gexec[lazy_par], stream));
      tend_pending = false;          // only once launched: a failure keeps the step pending
      replayed_bdyval();
      note_step(hs.lcount);
      return;
    }
    const int par = gpar();
    if (corr_pending) {
      if (graph_ok() && !ghosts_stale) {
        if (!gbdyf[par]) capture(par, 4);
        HIPCHK(hipGraphLaunch(gbdyf[par], stream));
        corr_pending = false;
        replayed_bdyval();
      } else {
        fused_bdyval();
      }
      note_step(hs.lcount);
      return;
    }
    // after a put the ghost rings are not step results: bdyval runs eagerly (its slice
    // exchange depends on that, bdyval())
    if (graph_ok() && !ghosts_stale) {
      if (!gbdy[par]) capture(par, 2);
      HIPCHK(hipGraphLaunch(gbdy[par], stream));
      replayed_bdyval();
    } else {
      bdyval();
    }
  }

  // capture tend (what & 1) and/or bdyval (what & 2) for the current ping-pong parity; the
  // host bookkeeping done in tend()/bdyval() is rolled back, the replay redoes it per launch
  void capture(int par, int what, int nsteps = 1) {
    const StepState save = hs;
    const bool pend = corr_pending;
    std::vector<int> curs, tqs;
    for (auto& t : tiles) { curs.push_back(t.cur); tqs.push_back(t.tq); }
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    for (int q = 0; q < nsteps; q++) {
      if (what == 3) step_once();
      else if (what == 4) fused_bdyval();
      else if (what & 1) tend();
      else bdyval();
    }
    HIPCHK(hipStreamEndCapture(stream, &graph));
    hipGraphExec_t& x = nsteps == 2 ? gexec2[par] : what == 3 ? gexec[par] : what == 4 ? gbdyf[par]
                        : what == 1 ? gtend[par] : gbdy[par];
    HIPCHK(hipGraphInstantiate(&x, graph, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(graph));
    hs = save;
    corr_pending = pend;
    for (size_t q = 0; q < tiles.size(); q++) { tiles[q].cur = curs[q]; tiles[q].tq = tqs[q]; }
  }

  // rcmdyn_exchange_plan: the communication calls of put + bdyval + nsteps x (tend + bdyval),
  // the drop-in's start (the initial bdyval after the state put, with its slice exchange) and
  // the eager step sequence every rank runs (graph replay issues the same calls in the same order)
  void plan_run(int nsteps) {
    prepare();
    ghosts_stale = true;           // as after rcmdyn_put
    bdyval();
    for (int s = 0; s < nsteps; s++) {
      step_once();
      note_step(hs.lcount, s == nsteps - 1);
    }
  }

  void kernel_times(int nsteps, int cap, char* names, int32_t* launches, double* avg, int32_t* count) {
    prepare();
    settle();
    KernelProf kp;
    HIPCHK(hipStreamSynchronize(stream));
    prof = &kp;
    try {
      for (int s = 0; s < nsteps; s++) step_once();
    } catch (...) {
      prof = nullptr;
      throw;
    }
    prof = nullptr;
    HIPCHK(hipStreamSynchronize(stream));
    std::vector<std::string> order;
    std::vector<double> tot;
    std::vector<int> cnt;
    for (auto& r : kp.rec) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, r.second.first, r.second.second));
      size_t q = std::find(order.begin(), order.end(), r.first) - order.begin();
      if (q == order.size()) { order.push_back(r.first); tot.push_back(0.0); cnt.push_back(0); }
      tot[q] += ms;
      cnt[q] += 1;
    }
    const int n = std::min<int>(cap, (int)order.size());
    for (int q = 0; q < n; q++) {
      std::memset(names + 48 * q, 0, 48);
      std::strncpy(names + 48 * q, order[q].c_str(), 47);
      launches[q] = cnt[q];
      avg[q] = tot[q] / cnt[q];
    }
    *count = n;
  }

  void set_time(long long lcount, double dt, double xbctime) {
    settle();
    HIPCHK(hipStreamSynchronize(stream));
    pending.clear();
    gpending.clear();
    StepState st;
    HIPCHK(hipMemcpy(&st, ds, sizeof(st), hipMemcpyDeviceToHost));
    st.lcount = lcount; st.dt = dt; st.xbctime = xbctime; st.nanflag = 0; st.slflag = 0;
    HIPCHK(hipMemcpy(ds, &st, sizeof(st), hipMemcpyHostToDevice));
    hs.lcount = lcount; hs.dt = dt; hs.xbctime = xbctime;
  }

  void reductions(double out[3]) {
    settle();
    check(0);
    HIPCHK(hipStreamSynchronize(stream));
    StepState st;
    HIPCHK(hipMemcpy(&st, ds, sizeof(st), hipMemcpyDeviceToHost));
    out[0] = st.ptntot; out[1] = st.pt2tot; out[2] = cfg.idynamic == 2 ? st.cflmax : 0.0;
    if (comm && cfg.tile_count < ntiles) {        // sumall / maxall over the ranks
      double* d = nullptr;
      HIPCHK(hipMalloc(&d, 3 * sizeof(double)));
      double hv[3] = {out[0], out[1], out[2]};
      HIPCHK(hipMemcpy(d, hv, sizeof(hv), hipMemcpyHostToDevice));
      comm->allreduce_sum(d, 2, stream);
      comm->allreduce_max_d(d + 2, 1, stream);
      HIPCHK(hipStreamSynchronize(stream));
      HIPCHK(hipMemcpy(hv, d, sizeof(hv), hipMemcpyDeviceToHost));
      (void)hipFree(d);
      out[0] = hv[0]; out[1] = hv[1]; out[2] = hv[2];
    }
  }

  void diagnostics(double out[4]) {
    settle();
    HIPCHK(hipStreamSynchronize(stream));
    check_now();
    StepState st;
    HIPCHK(hipMemcpy(&st, ds, sizeof(st), hipMemcpyDeviceToHost));
    out[0] = st.ptntot; out[1] = st.pt2tot; out[2] = std::isnan(st.ptntot) ? 1.0 : 0.0; out[3] = st.nanflag;
  }
};

// ======================================================================== C-ABI
namespace {
template <class F>
int guard(rcmdyn_t* h, F fn) {
  try {
    fn();
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    if (h) h->err = e.what();
    return 1;
  }
}
}  // namespace

extern "C" {

// RCMDYN_SEGV_TRACE=1 (opt-in host debugging aid): print the native backtrace of a
// segmentation fault, then hand the signal to the handler that was installed before (Python's
// faulthandler, a host's own), or the default action
static struct sigaction g_prev_segv;
static void segv_trace(int sig, siginfo_t* info, void* uc) {
  void* bt[64];
  const int n = backtrace(bt, 64);
  const char msg[] = "rcmdyn: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(bt, n, 2);
  sigaction(sig, &g_prev_segv, nullptr);
  if (g_prev_segv.sa_flags & SA_SIGINFO) {
    if (g_prev_segv.sa_sigaction) { g_prev_segv.sa_sigaction(sig, info, uc); return; }
  } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
    g_prev_segv.sa_handler(sig);
    return;
  }
  std::raise(sig);
}
static void install_segv_trace() {
  static bool done = false;
  if (done || !std::getenv("RCMDYN_SEGV_TRACE")) return;
  done = true;
  void* warm[1];
  (void)backtrace(warm, 1);           // loads the unwinder now: backtrace's first call allocates
  struct sigaction sa {};
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO | SA_NODEFER;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}

int rcmdyn_create(const rcmdyn_config* cfg, rcmdyn_t** out) {
  if (!cfg || !out) { g_last_error = "rcmdyn_create: null argument"; return 1; }
  install_segv_trace();
  auto* h = new rcmdyn_engine();
  int rc = guard(h, [&] { h->create(cfg); });
  if (rc) {
    g_last_error = h->err;
    h->destroy();
    delete h;
    *out = nullptr;
    return rc;
  }
  *out = h;
  return 0;
}

int rcmdyn_exchange_plan(const rcmdyn_config* cfg, int32_t nsteps, int64_t* ops, int64_t cap, int64_t* count) {
  if (!cfg || !count || nsteps < 0 || cap < 0 || (cap > 0 && !ops)) {
    g_last_error = "rcmdyn_exchange_plan: bad argument";
    return 1;
  }
  std::vector<PlanOp> log;
  auto* h = new rcmdyn_engine();
  int rc = guard(h, [&] {
    h->create(cfg, &log);
    h->plan_run(nsteps);
  });
  if (rc) g_last_error = h->err;
  h->destroy();
  delete h;
  if (rc) return rc;
  *count = (int64_t)log.size();
  for (int64_t q = 0; q < std::min<int64_t>(cap, (int64_t)log.size()); q++) {
    const PlanOp& o = log[q];
    const int64_t v[7] = {o.seq, o.kind, o.chan, o.dir, o.peer, o.count, o.sig};
    std::memcpy(ops + 7 * q, v, sizeof(v));
  }
  return 0;
}

int rcmdyn_overlap_shares(const rcmdyn_config* cfg, int32_t* out, int32_t cap) {
  if (!cfg || !out || cap < 0) {
    g_last_error = "rcmdyn_overlap_shares: bad argument";
    return 1;
  }
  std::vector<PlanOp> log;
  auto* h = new rcmdyn_engine();
  int rc = guard(h, [&] {
    h->create(cfg, &log);
    for (size_t q = 0; q < h->tiles.size() && (int)q < cap; q++) {
      const Tile& t = h->tiles[q];
      const Geom& g = t.g;
      const int mj2 = g.br ? g.jdi2 : g.jde2 + 1, mi2 = g.bt ? g.idi2 : g.ide2 + 1;
      const bool ov = h->overlap() && t.rja <= t.rjb && t.ria <= t.rib;
      const int32_t v[6] = {
          ov ? (int32_t)((long)(t.rjb - t.rja + 1) * (t.rib - t.ria + 1)) : 0,
          (int32_t)((long)(g.jdx2() - g.jdx1() + 1) * (g.idx2() - g.idx1() + 1)),
          ov ? (int32_t)t.mom_p1 : 0, (int32_t)((long)(mj2 - g.jdi1 + 1) * (mi2 - g.idi1 + 1)),
          ov ? (int32_t)t.sca_p1 : 0, (int32_t)((long)(g.jcx2() - g.jcx1() + 1) * (g.icx2() - g.icx1() + 1))};
      std::memcpy(out + 6 * q, v, sizeof(v));
    }
  });
  if (rc) g_last_error = h->err;
  h->destroy();
  delete h;
  return rc;
}

int rcmdyn_destroy(rcmdyn_t* h) {
  if (!h) return 0;
  // a lazy tend (or deferred corrections) still pending is launched first, so the host's last
  // tend is not dropped without a word: its failure is this call's return code
  const int rc0 = guard(h, [&] { h->settle(); });
  const std::string err0 = h->err;
  const int rc = guard(h, [&] { h->destroy(); });
  if (rc0 || rc) g_last_error = rc0 ? err0 : h->err;      // h is gone: rcmdyn_last_error(NULL)
  delete h;
  return rc0 ? rc0 : rc;
}

const char* rcmdyn_last_error(rcmdyn_t* h) { return h ? h->err.c_str() : g_last_error.c_str(); }

int rcmdyn_set_nproc(int32_t nproc, int32_t jx, int32_t iy, int32_t cpus[2]) {
  // Main/mpplib/mod_mppparam.F90:1152-1186
  if (nproc < 1 || !cpus) return 1;
  if (nproc == 1) { cpus[0] = 1; cpus[1] = 1; return 0; }
  if (nproc < 4) { cpus[0] = nproc; cpus[1] = 1; return 0; }
  int cj = ((int)std::lround(std::sqrt((double)nproc)) / 2) * 2;
  if (iy > (int)(1.5 * (double)jx)) {
    cj -= 1;
    while (nproc % cj != 0) cj -= 1;
  } else if (jx > (int)(1.5 * (double)iy)) {
    cj += 1;
    while (nproc % cj != 0) cj += 1;
  } else {
    while (nproc % cj != 0) cj += 1;
  }
  cpus[0] = cj; cpus[1] = nproc / cj;
  return 0;
}

int rcmdyn_tile_extent(int32_t jx, int32_t iy, int32_t nproc_j, int32_t nproc_i, int32_t tile, int32_t ext[8],
                       int32_t bdy[4]) {
  if (tile < 0 || tile >= nproc_j * nproc_i) return 1;
  tile_extent(jx, iy, nproc_j, nproc_i, tile, ext, bdy);
  return 0;
}

int rcmdyn_tile_extent_cfg(const rcmdyn_config* cfg, int32_t tile, int32_t ext[8], int32_t bdy[4]) {
  if (!cfg || !ext || !bdy) return 1;
  if (tile < 0 || cfg->nproc_j < 1 || cfg->nproc_i < 1 || tile >= cfg->nproc_j * cfg->nproc_i) return 1;
  if ((cfg->i_band != 0 && cfg->i_band != 1) || (cfg->i_crm != 0 && cfg->i_crm != 1)) return 1;
  if (cfg->i_crm && !cfg->i_band) return 1;              // CRM is built over the band only (create refuses it)
  tile_extent(cfg->jx, cfg->iy, cfg->nproc_j, cfg->nproc_i, tile, ext, bdy, cfg->i_band, cfg->i_crm);
  return 0;
}

int rcmdyn_put(rcmdyn_t* h, int32_t field, const double* src, int32_t j1, int32_t j2, int32_t i1, int32_t i2,
               int32_t k1, int32_t k2) {
  return guard(h, [&] { h->put(field, src, j1, j2, i1, i2, k1, k2); });
}

int rcmdyn_get(rcmdyn_t* h, int32_t field, double* dst, int32_t j1, int32_t j2, int32_t i1, int32_t i2, int32_t k1,
               int32_t k2) {
  return guard(h, [&] { h->get(field, dst, j1, j2, i1, i2, k1, k2); });
}

int rcmdyn_set_time(rcmdyn_t* h, int64_t lcount, double dt, double xbctime) {
  return guard(h, [&] { h->set_time(lcount, dt, xbctime); });
}

int rcmdyn_get_time(rcmdyn_t* h, int64_t* lcount, double* dt, double* xbctime) {
  return guard(h, [&] {
    *lcount = h->hs.lcount; *dt = h->hs.dt; *xbctime = h->hs.xbctime;
  });
}

int rcmdyn_tend(rcmdyn_t* h) { return guard(h, [&] { h->tend_call(); }); }

int rcmdyn_tend_pre_physics(rcmdyn_t* h) {
  return guard(h, [&] {
    h->prepare();
    h->settle();
    h->check(rcmdyn_engine::FLAG_LAG);
    h->tend(rcmdyn_engine::TEND_PRE, true);
  });
}

int rcmdyn_tend_post_physics(rcmdyn_t* h) {
  return guard(h, [&] {
    h->prepare();
    h->settle();
    h->check(rcmdyn_engine::FLAG_LAG);
    h->defer_corr = h->can_defer();       // the corrections go with the next rcmdyn_bdyval
    try {
      h->tend(rcmdyn_engine::TEND_POST);
    } catch (...) {
      h->defer_corr = false;
      throw;
    }
    h->defer_corr = false;
    if (!h->corr_pending) h->note_step(h->hs.lcount);
  });
}

int rcmdyn_bdyin(rcmdyn_t* h) {
  return guard(h, [&] {
    h->bdyin();
    HIPCHK(hipStreamSynchronize(h->stream));
  });
}

int rcmdyn_bdyval(rcmdyn_t* h) { return guard(h, [&] { h->bdyval_call(); }); }

int rcmdyn_step(rcmdyn_t* h, int32_t nsteps) { return guard(h, [&] { h->step(nsteps); }); }

int rcmdyn_synchronize(rcmdyn_t* h) {
  return guard(h, [&] {
    h->settle();                                     // a deferred step's flags are checked here
    if (h->comm) h->note_step(h->hs.lcount, true);   // collective: every rank synchronizes
    HIPCHK(hipStreamSynchronize(h->stream));
    h->check(0);
  });
}

int rcmdyn_diagnostics(rcmdyn_t* h, double out[4]) { return guard(h, [&] { h->diagnostics(out); }); }

int rcmdyn_reductions(rcmdyn_t* h, double out[3]) { return guard(h, [&] { h->reductions(out); }); }

int rcmdyn_runtime_info(char* buf, int32_t len) {
  try {
    Dl_info info{};
    std::string hip = dladdr((void*)&hipGetDeviceCount, &info) && info.dli_fname ? info.dli_fname : "?";
    std::string s = "hip=" + hip + "; rccl=" + rccl_describe();
    if (buf && len > 0) {
      std::strncpy(buf, s.c_str(), (size_t)len - 1);
      buf[len - 1] = 0;
    }
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

int rcmdyn_comm_unique_id(uint8_t out[128]) {
  try {
    comm_unique_id(out);
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

int rcmdyn_last_step_ms(rcmdyn_t* h, double* ms) { return guard(h, [&] { *ms = h->last_ms; }); }

int rcmdyn_set_diagnostics(rcmdyn_t* h, int32_t on) {
  return guard(h, [&] {
    h->settle();                                     // a lazy tend replays its graph first
    HIPCHK(hipStreamSynchronize(h->stream));
    if (h->diag != (on != 0)) {
      h->diag = (on != 0);
      h->invalidate_graphs();
    }
  });
}

int rcmdyn_kernel_times(rcmdyn_t* h, int32_t nsteps, int32_t cap, char* names, int32_t* launches, double* avg_ms,
                        int32_t* count) {
  return guard(h, [&] { h->kernel_times(nsteps, cap, names, launches, avg_ms, count); });
}

}  // extern "C"
