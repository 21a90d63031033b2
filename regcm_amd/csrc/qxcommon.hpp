// qxcommon.hpp -- device helpers of the moisture species shared by the qv/qc kernels
// (kernels.hip) and the hydrometeors of nqx = 5 (species.hip): the upstream flux form, the
// negative-moisture fix, the RAW filters and bdyval's hydrometeor inflow/outflow lines.
#pragma once
#include "kernels.hpp"
#include "devcommon.hpp"
#include "fastmath.hpp"

namespace rcm {

// negative-moisture fix helpers (K6 below)
__device__ __forceinline__ double negfix_sum(const Geom& g, const double* sv, const double* fx, int j, int i, int k,
                                             bool use_fixed) {
  double sum = 0.0;
  for (int ii = i - 1; ii <= i + 1; ii++)
    for (int jj = j - 1; jj <= j + 1; jj++) {
      double v = F3(sv, jj, ii, k);
      if (use_fixed) {
        const bool pred = (ii < i) || (ii == i && jj < j);
        if (pred && in(jj, g.jci1, g.jci2) && in(ii, g.ici1, g.ici2) && v < d_zero) v = F3(fx, jj, ii, k);
      }
      sum = sum + fabs(v);
    }
  return 0.01 * sum / 9.0;
}

__device__ __forceinline__ bool negfix_dependent(const Geom& g, const double* sv, int j, int i, int k) {
#define NEG(J, I) (in(J, g.jci1, g.jci2) && in(I, g.ici1, g.ici2) && F3(sv, J, I, k) < d_zero)
  return NEG(j - 1, i) || NEG(j - 1, i - 1) || NEG(j, i - 1) || NEG(j + 1, i - 1);
#undef NEG
}

// ---- the serial part of the negative-moisture fix (Main/mod_tendency.F90:382-393)
// The parallel passes (k_qfilter / k_split_project's list blocks, k_qx_fix, k_nh_negfix) fix
// every negative point whose four sweep-predecessors are non-negative and mark, per (species,
// level) plane, the rows that hold a dependent one (a bitmap of negfix_rowwords words per
// plane).  negfix_sweep then resolves one plane in the reference's order with one wavefront:
// only the marked rows are visited; per chunk of 64 points every lane stages its point's nine
// neighbours (and the parallel pass's fixed values of its negative predecessors) in LDS in one
// round of loads, and lane 0 walks the chunk's dependent points in order on LDS alone, taking a
// dependent predecessor's value from the fixed values this sweep keeps for the current and
// the previous row.  Each value is the reference's expression (0.01 * the nine |q| summed in
// its order / 9), so the result is the sweep's, bit for bit.  The caller passes
// negfix_sweep_lds(g) doubles of LDS (lds), or null: then lane 0 reads every operand from memory.
__device__ __forceinline__ void negfix_mark(const Geom& g, unsigned* dep, int plane, int i) {
  const int r = i - g.ici1;
  atomicOr(&dep[plane * negfix_rowwords(g) + (r >> 5)], 1u << (r & 31));
}
// The row flags a parallel pass stored for plane `plane` (depf: R flags per plane, a plain
// store per dependent point) ORed into its bitmap words, the flags cleared for the next step:
// the tid-th of nt threads (nt a multiple of 64, whole wavefronts: a row chunk per wavefront
// and ballot); the caller synchronises before the words are read.
__device__ __forceinline__ void negfix_collect(const Geom& g, unsigned* depf, unsigned* dep, int plane, int tid, int nt) {
  const int R = g.ici2 - g.ici1 + 1;
  unsigned* fl = depf + plane * R;
  unsigned* words = dep + plane * negfix_rowwords(g);
  for (int b = 0; b < R; b += nt) {
    const int r = b + tid;
    const bool f = r < R && fl[r] != 0u;
    if (f) fl[r] = 0u;
    const unsigned long long m = __ballot(f);
    const unsigned w = (unsigned)(m >> (r & 32));
    if (r < R && (r & 31) == 0 && w) words[r >> 5] |= w;
  }
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// one wavefront (lane = threadIdx.x & 63) resolves plane `plane` (level k of sv / fx); post(j,
// i, v) writes what follows from a fixed value (the filters), on the lane of point (j, i)
template <class Post>
__device__ void negfix_sweep(const Geom& g, const double* sv, double* fx, unsigned* dep, int plane, int k,
                             double* lds, Post post) {
  const int lane = (int)threadIdx.x & 63;
  const int nw = negfix_rowwords(g), W = g.jci2 - g.jci1 + 1;
  unsigned* words = dep + plane * nw;
  const bool inlds = lds != nullptr;
  double(*pre)[13] = (double(*)[13])(lds + 2 * W);
  int last = -2, cur = 0;
  for (int w = 0; w < nw; w++) {
    unsigned bits = words[w];
    if (!bits) continue;
    while (bits) {
      const int r = __ffs((int)bits) - 1;
      bits &= bits - 1;
      const int i = g.ici1 + 32 * w + r;
      const bool pv = last == i - 1;
      cur ^= 1;
      // this sweep's fixed values of the current and the previous row (two LDS rows, alternating)
      double* rowc = lds + (cur ? W : 0);
      const double* rowp = lds + (cur ? 0 : W);
      if (inlds)
        for (int x = lane; x < W; x += 64) rowc[x] = -1.0;
      wave_lds_sync();
      for (int j0 = g.jci1; j0 <= g.jci2; j0 += 64) {
        const int j = j0 + lane;
        const bool fl = j <= g.jci2 && F3(sv, j, i, k) < d_zero && negfix_dependent(g, sv, j, i, k);
        const unsigned long long mask = __ballot(fl);
        if (!mask) continue;
        if (!inlds) {
          if (lane == 0) {
            unsigned long long m = mask;
            while (m) {
              const int b = __ffsll((long long)m) - 1;
              m &= m - 1;
              const double v = negfix_sum(g, sv, fx, j0 + b, i, k, true);
              F3(fx, j0 + b, i, k) = v;
              post(j0 + b, i, v);
            }
          }
          continue;
        }
        if (fl) {
          int s = 0;
          for (int ii = i - 1; ii <= i + 1; ii++)
            for (int jj = j - 1; jj <= j + 1; jj++, s++) {
              const double v = F3(sv, jj, ii, k);
              pre[lane][s] = v;
              if (s < 4)
                pre[lane][9 + s] =
                    (in(jj, g.jci1, g.jci2) && in(ii, g.ici1, g.ici2) && v < d_zero) ? F3(fx, jj, ii, k) : d_zero;
            }
        }
        wave_lds_sync();
        if (lane == 0) {
          unsigned long long m = mask;
          while (m) {
            const int b = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int jb = j0 + b;
            double sum = 0.0;
            int s = 0;
            for (int ii = i - 1; ii <= i + 1; ii++)
              for (int jj = jb - 1; jj <= jb + 1; jj++, s++) {
                double v = pre[b][s];
                if (s < 4 && in(jj, g.jci1, g.jci2) && in(ii, g.ici1, g.ici2) && v < d_zero) {
                  // a negative sweep-predecessor: this sweep's fixed value, or the parallel pass's
                  const double rv = s == 3 ? rowc[jj - g.jci1] : (pv ? rowp[jj - g.jci1] : -1.0);
                  v = rv >= d_zero ? rv : pre[b][9 + s];
                }
                sum = sum + fabs(v);
              }
            rowc[jb - g.jci1] = 0.01 * sum / 9.0;
          }
        }
        wave_lds_sync();
        if (fl) {
          const double v = rowc[j - g.jci1];
          F3(fx, j, i, k) = v;
          post(j, i, v);
        }
      }
      last = i;
    }
    if (lane == 0) words[w] = 0;
  }
}

// LDS-only block barrier: waits for this wave's LDS operations, not for its global loads in flight
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Dense planes (many marked rows): the sweep as a skewed wavefront.  Point (j, i) depends only
// on its sweep-predecessors (j-1, i) and (j-1..j+1, i-1), so with one thread per row and row i
// two steps behind row i-1 (step t = j - jci1 + 2 (i - ici1)) every dependency was resolved one
// or more steps earlier: W + 2 (R - 1) steps, one LDS barrier each, for the whole plane.  Each
// thread keeps the fixed value of its own previous point in a register and publishes its
// fixed values in a 4-slot LDS ring per row (ring: 4 R doubles) for the row below; it streams
// its 3 x 3 window of the original forecasts and the post inputs A::load of its row through a
// register queue loaded P steps ahead, so no step waits on memory.  Every negative point of
// the plane is evaluated (an independent one gives the parallel pass's value again); only the
// dependent ones are stored and post-processed (A::apply).  Needs R <= the block's threads.
template <class A>
__device__ void negfix_dense(const Geom& g, const double* sv, double* fx, int k, double* ring, const A& acc) {
  constexpr int P = 4, NQ = 3 + A::NI;
  const int r = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  const int R = g.ici2 - g.ici1 + 1, W = g.jci2 - g.jci1 + 1, S = W + 2 * (R - 1);
  const bool act = r < R;
  const int i = g.ici1 + r;
  auto qload = [&](int jc, double* q) {
    const bool ok = act && jc >= g.jci1 - 1 && jc <= g.jci2 + 1;
#pragma unroll
    for (int d = 0; d < 3; d++) q[d] = ok ? F3(sv, jc, i - 1 + d, k) : 0.0;
    if (act && in(jc, g.jci1, g.jci2)) acc.load(jc, i, q + 3);
    else
#pragma unroll
      for (int d = 3; d < NQ; d++) q[d] = 0.0;
  };
  int j = g.jci1 - 2 * r;                    // this row's column at step 0
  double w0[NQ], w1[NQ], w2[NQ], qa[P][NQ], qb[P][NQ];
  qload(j - 1, w0);
  qload(j, w1);
  qload(j + 1, w2);
#pragma unroll
  for (int u = 0; u < P; u++) qload(j + 2 + u, qa[u]);
  double prev = 0.0;                         // the fixed value of (j - 1, i)
  const bool up = r >= 1;                    // row i - 1 is interior
  for (int t0 = 0; t0 < S; t0 += P) {
#pragma unroll
    for (int u = 0; u < P; u++) qload(j + 2 + P + u, qb[u]);
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int jj = j + u;
      if (act && t0 + u < S && in(jj, g.jci1, g.jci2) && w1[1] < d_zero) {
        const bool p0 = up && jj - 1 >= g.jci1 && w0[0] < d_zero, p1 = up && w1[0] < d_zero;
        const bool p2 = up && jj + 1 <= g.jci2 && w2[0] < d_zero, p3 = jj - 1 >= g.jci1 && w0[1] < d_zero;
        const double* rp = ring + 4 * (r - 1);
        double sum = 0.0;
        sum = sum + fabs(p0 ? rp[(jj - 1) & 3] : w0[0]);
        sum = sum + fabs(p1 ? rp[jj & 3] : w1[0]);
        sum = sum + fabs(p2 ? rp[(jj + 1) & 3] : w2[0]);
        sum = sum + fabs(p3 ? prev : w0[1]);
        sum = sum + fabs(w1[1]);
        sum = sum + fabs(w2[1]);
        sum = sum + fabs(w0[2]);
        sum = sum + fabs(w1[2]);
        sum = sum + fabs(w2[2]);
        // / 9 as div_by (fastmath.hpp: the division's bits from the rounded reciprocal in three
        // dependent operations; the step's critical path runs through it), for normal operands
        const double xs = 0.01 * sum;
        const double v = xs >= 0x1p-960 ? div_by(xs, 9.0, 1.0 / 9.0) : xs / 9.0;
        ring[4 * r + (jj & 3)] = v;
        prev = v;
        if (p0 || p1 || p2 || p3) {
          F3(fx, jj, i, k) = v;
          acc.apply(jj, i, v, w1 + 3);
        }
      }
      lds_barrier();
#pragma unroll
      for (int d = 0; d < NQ; d++) { w0[d] = w1[d]; w1[d] = w2[d]; w2[d] = qa[u][d]; }
    }
#pragma unroll
    for (int u = 0; u < P; u++)
#pragma unroll
      for (int d = 0; d < NQ; d++) qa[u][d] = qb[u][d];
    j += P;
  }
}

// The same wavefront with the row-to-row hand-over in registers (NEGFIX_DPP): lane l of a
// wavefront holds row r = 64 w + l, and the value row r - 1 fixed in the previous step moves to
// lane l with one cross-lane shift (DPP wave_shr:1, or __shfl_up with NEGFIX_DPP = 2) instead of
// an LDS ring behind a block barrier every step.  Each lane keeps the three values of the row
// above that its window reads (columns jj - 1, jj, jj + 1) in registers.  Lane 0 of wavefront w > 0
// takes row 64 w - 1's values from an LDS ring written by lane 63 of wavefront w - 1, which runs
// SK steps ahead (wavefront w's rows start SK steps later than the two-per-row skew gives), so one
// block barrier every SK steps makes those writes visible: W + 2 (R - 1) + SK (nw - 1) steps.
// Every value is the same expression on the same operands as negfix_dense's, bit for bit.
#ifndef NEGFIX_DPP
#define NEGFIX_DPP 1
#endif
__device__ __forceinline__ double lane_shr1(double x) {      // lane l gets lane l - 1's x
#if NEGFIX_DPP == 2
  return __shfl_up(x, 1, 64);
#else
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x138, 0xf, 0xf, false);   // wave_shr:1
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
#endif
}
template <class A>
__device__ void negfix_dense_dpp(const Geom& g, const double* sv, double* fx, int k, double* ring, const A& acc) {
  constexpr int P = 4, NQ = 3 + A::NI, SK = 8;
  const int r = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  const int lane = r & 63, wv = r >> 6;
  const int R = g.ici2 - g.ici1 + 1, W = g.jci2 - g.jci1 + 1, nwv = (R + 63) >> 6;
  const int S = W + 2 * (R - 1) + SK * (nwv - 1);
  const bool act = r < R;
  const int i = g.ici1 + r;
  auto qload = [&](int jc, double* q) {
    const bool ok = act && jc >= g.jci1 - 1 && jc <= g.jci2 + 1;
#pragma unroll
    for (int d = 0; d < 3; d++) q[d] = ok ? F3(sv, jc, i - 1 + d, k) : 0.0;
    if (act && in(jc, g.jci1, g.jci2)) acc.load(jc, i, q + 3);
    else
#pragma unroll
      for (int d = 3; d < NQ; d++) q[d] = 0.0;
  };
  int j = g.jci1 - 2 * r - SK * wv;          // this row's column at step 0
  double w0[NQ], w1[NQ], w2[NQ], qa[P][NQ], qb[P][NQ];
  qload(j - 1, w0);
  qload(j, w1);
  qload(j + 1, w2);
#pragma unroll
  for (int u = 0; u < P; u++) qload(j + 2 + u, qa[u]);
  double prev = 0.0;                         // the fixed value of (j - 1, i)
  double pub = 0.0;                          // this lane's value of the last step (for row i + 1)
  double cm1 = 0.0, c0 = 0.0, cp1 = 0.0;     // row i - 1's values at columns jj - 1, jj, jj + 1
  const bool up = r >= 1;                    // row i - 1 is interior
  const bool from_ring = lane == 0 && wv > 0, to_ring = lane == 63 && wv < nwv - 1;
  for (int t0 = 0; t0 < S; t0 += P) {
#pragma unroll
    for (int u = 0; u < P; u++) qload(j + 2 + P + u, qb[u]);
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int t = t0 + u, jj = j + u;
      if ((t & (SK - 1)) == 0) lds_barrier();  // lane 63's ring writes of SK or more steps ago
      double recv = lane_shr1(pub);
      if (from_ring) recv = ring[(wv - 1) * 64 + ((jj + 1) & 63)];
      cm1 = c0; c0 = cp1; cp1 = recv;
      if (act && t < S && in(jj, g.jci1, g.jci2) && w1[1] < d_zero) {
        const bool p0 = up && jj - 1 >= g.jci1 && w0[0] < d_zero, p1 = up && w1[0] < d_zero;
        const bool p2 = up && jj + 1 <= g.jci2 && w2[0] < d_zero, p3 = jj - 1 >= g.jci1 && w0[1] < d_zero;
        double sum = 0.0;
        sum = sum + fabs(p0 ? cm1 : w0[0]);
        sum = sum + fabs(p1 ? c0 : w1[0]);
        sum = sum + fabs(p2 ? cp1 : w2[0]);
        sum = sum + fabs(p3 ? prev : w0[1]);
        sum = sum + fabs(w1[1]);
        sum = sum + fabs(w2[1]);
        sum = sum + fabs(w0[2]);
        sum = sum + fabs(w1[2]);
        sum = sum + fabs(w2[2]);
        const double xs = 0.01 * sum;
        const double v = xs >= 0x1p-960 ? div_by(xs, 9.0, 1.0 / 9.0) : xs / 9.0;
        pub = v;
        prev = v;
        if (p0 || p1 || p2 || p3) {
          F3(fx, jj, i, k) = v;
          acc.apply(jj, i, v, w1 + 3);
        }
      }
      if (to_ring) ring[wv * 64 + (jj & 63)] = pub;
#pragma unroll
      for (int d = 0; d < NQ; d++) { w0[d] = w1[d]; w1[d] = w2[d]; w2[d] = qa[u][d]; }
    }
#pragma unroll
    for (int u = 0; u < P; u++)
#pragma unroll
      for (int d = 0; d < NQ; d++) qa[u][d] = qb[u][d];
    j += P;
  }
}

// NEGFIX_POST (kernels.hpp): the serial pass resolves the chain only (the fixed values into fx)
// and a parallel launch afterwards (k_negfix_post, k_qx_post) applies the filters of the
// dependent points, so the wavefront's steps carry the forecasts alone: every load of the
// row-per-lane wavefront touches 64 lines, and the filters' inputs were 5 (qv/qc) or 2 (species)
// more such loads per step (C3, nqx = 5: k_negfix_serial 365 -> 175 us, k_qx_serial 295 -> 220)
struct NoPost {
  static constexpr int NI = 0;
  __device__ void load(int, int, double*) const {}
  __device__ void apply(int, int, double, const double*) const {}
};
// a dependent negative point of the plane (the serial pass fixed it): the post launches' test
__device__ __forceinline__ bool negfix_is_dependent(const Geom& g, const double* sv, int j, int i, int k) {
  return F3(sv, j, i, k) < d_zero && negfix_dependent(g, sv, j, i, k);
}

// One (species, level) plane's serial fix by a whole block: nothing when no row is marked, the
// wavefront when more than NEGFIX_SPARSE rows are and the block has a thread per row (and lds
// holds the ring), else the row sweep by wavefront 0.  lds: ldsn doubles (see negfix_lds);
// mode (Consts::negfix_mode, tests): 1 runs the row sweep on every marked plane.
constexpr int NEGFIX_SPARSE = 16;
template <class A, class Post>
__device__ void negfix_resolve(const Geom& g, const double* sv, double* fx, unsigned* dep, int plane, int k,
                               double* lds, int ldsn, const A& acc, Post post, int mode = 0) {
  const int nw = negfix_rowwords(g), R = g.ici2 - g.ici1 + 1;
  unsigned* words = dep + plane * nw;
  int nm = 0;
  for (int w = 0; w < nw; w++) nm += __popc(words[w]);
  if (nm == 0) return;
  const int T = (int)(blockDim.x * blockDim.y * blockDim.z);
  const int tid = (int)(threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z));
  if (mode == 0 && nm > NEGFIX_SPARSE && R <= T && 4 * R <= ldsn) {
    if (NEGFIX_DPP) negfix_dense_dpp(g, sv, fx, k, lds, acc);
    else negfix_dense(g, sv, fx, k, lds, acc);
    __syncthreads();                           // every wave read the bitmap before it is cleared
    for (int w = tid; w < nw; w += T) words[w] = 0;
    return;
  }
  if (tid < 64) negfix_sweep(g, sv, fx, dep, plane, k, negfix_sweep_lds(g) <= ldsn ? lds : nullptr, post);
}

// RAW filters of one point (filter_raw_qv / filter_raw_4d) with the filtered p*
__device__ __forceinline__ void raw_filter(const Consts* c, int n, double fq, double o1, double o2v, double pa,
                                           double pb, double& n1, double& n2) {
  const double beta = 0.53;
  if (n == 0) {
    const double d = c->gnu1 * (fq + o2v - d_two * o1);
    n2 = dmax(o1 + beta * d, MINQQ * pa);
    n1 = dmax(fq + (beta - d_one) * d, MINQQ * pb);
  } else {
    const double d = c->gnu2 * (fq + o2v - d_two * o1);
    double m = o1 + beta * d;
    double q = fq + (beta - d_one) * d;
    if (m < d_zero) m = d_zero;
    if (q < d_zero) q = d_zero;
    n2 = m;
    n1 = q;
  }
}

// upstream flux-form advection of one scalar (hadvt/hadvqv/hadvqx, Main/mod_advection.F90:
// 337-386, 547-596, 639-653); limiter 0 none, 1 t_extrema, 2 q_rel_extrema
__device__ __forceinline__ double hadv_flux(const Consts* c, double xm, double ps, double uavg1, double uavg2,
                                            double vavg1, double vavg2, double fc, double fw, double fe, double fs,
                                            double fn, int limiter) {
  const double ul = c->ul;
  const double f1 = d_half * ul * (uavg2 + uavg1) / ps;
  const double f2 = d_half * ul * (vavg2 + vavg1) / ps;
  const double fx1 = (d_one + f1) * fw + (d_one - f1) * fc;
  const double fx2 = (d_one + f1) * fc + (d_one - f1) * fe;
  const double fy1 = (d_one + f2) * fs + (d_one - f2) * fc;
  const double fy2 = (d_one + f2) * fc + (d_one - f2) * fn;
  double fg = -xm * (uavg2 * fx2 - uavg1 * fx1 + vavg2 * fy2 - vavg1 * fy1);
  if (limiter && c->stability_enhance) {
    double den, thr;
    if (limiter == 1) { den = ps; thr = c->t_extrema; } else { den = dmax(fc, DLOWVAL); thr = c->q_rel_extrema; }
    if (fabs(fn + fs - d_two * fc) / den > thr) {
      if (fc > fn && fc > fs) fg = dmin(fg, d_zero);
      else if (fc < fn && fc < fs) fg = dmax(fg, d_zero);
    }
    if (fabs(fe + fw - d_two * fc) / den > thr) {
      if (fc > fe && fc > fw) fg = dmin(fg, d_zero);
      else if (fc < fe && fc < fw) fg = dmax(fg, d_zero);
    }
  }
  return fg;
}

// qc inflow/outflow (present_qc = .false., bdyflow), Main/mod_bdycod.F90:2153-2220, one
// block per level: west/east first (they read qc(jci1|jci2, ice1|ice2) before south/north
// rewrite it), then south/north.  The last tile's launch also advances the boundary clock
// xbctime += dtsec (Main/mod_bdycod.F90:2566): nothing here reads it.
template <class PS>
__device__ void bdyval_qc_level(const Geom& g, int do_qc, int do_qv, double* a1qc, double* a1qv, PS ps, const Slices& sl,
                                long slen, int k) {
  if (do_qv) {
    // qv inflow/outflow for iboudy = 3 or 4, Main/mod_bdycod.F90:1809-1950: west/east on ici,
    // then south/north on jce (reading the west/east results at the corners)
    for (int i = g.ici1 + (int)threadIdx.x; i <= g.ici2; i += (int)blockDim.x) {
      if (g.bl) {
        const double qext = F3(a1qv, g.jce1, i, k) / ps(g.jce1, i);
        const double qint = F3(a1qv, g.jci1, i, k) / ps(g.jci1, i);
        const double w = SLI(sl.s[0], i, k) + SLI(sl.s[0], i + 1, k) + SLI(sl.s[1], i, k) + SLI(sl.s[1], i + 1, k);
        F3(a1qv, g.jce1, i, k) = (w > d_zero) ? qext * ps(g.jce1, i) : qint * ps(g.jce1, i);
      }
      if (g.br) {
        const double qext = F3(a1qv, g.jce2, i, k) / ps(g.jce2, i);
        const double qint = F3(a1qv, g.jci2, i, k) / ps(g.jci2, i);
        const double w = SLI(sl.s[2], i, k) + SLI(sl.s[2], i + 1, k) + SLI(sl.s[3], i, k) + SLI(sl.s[3], i + 1, k);
        F3(a1qv, g.jce2, i, k) = (w < d_zero) ? qext * ps(g.jce2, i) : qint * ps(g.jce2, i);
      }
    }
    __syncthreads();
    for (int j = g.jce1 + (int)threadIdx.x; j <= g.jce2; j += (int)blockDim.x) {
      if (g.bb) {
        const double qext = F3(a1qv, j, g.ice1, k) / ps(j, g.ice1);
        const double qint = F3(a1qv, j, g.ici1, k) / ps(j, g.ici1);
        const double w = SLJ(sl.s[12], j, k) + SLJ(sl.s[12], j + 1, k) + SLJ(sl.s[13], j, k) + SLJ(sl.s[13], j + 1, k);
        F3(a1qv, j, g.ice1, k) = (w > d_zero) ? qext * ps(j, g.ice1) : qint * ps(j, g.ice1);
      }
      if (g.bt) {
        const double qext = F3(a1qv, j, g.ice2, k) / ps(j, g.ice2);
        const double qint = F3(a1qv, j, g.ici2, k) / ps(j, g.ici2);
        const double w = SLJ(sl.s[14], j, k) + SLJ(sl.s[14], j + 1, k) + SLJ(sl.s[15], j, k) + SLJ(sl.s[15], j + 1, k);
        F3(a1qv, j, g.ice2, k) = (w < d_zero) ? qext * ps(j, g.ice2) : qint * ps(j, g.ice2);
      }
    }
    __syncthreads();
  }
  if (!do_qc) return;
  // The west/east pass reads the interior columns jci1/jci2 on rows ice1..ice2 before the
  // south/north pass rewrites rows ice1/ice2 on jci1..jci2: the two passes share exactly the
  // four points (jci1|jci2, ice1|ice2).  Otherwise the passes are independent (west/east writes
  // columns jce1/jce2, which south/north never reads; south/north reads rows ici1/ici2, which
  // nothing writes).  So the first chunk issues every load (its operands and the four shared
  // points) before one barrier and its stores: one memory round trip.  A later chunk (a tile
  // wider or taller than the block) reads the shared points of row ice2 from those first loads.
  const int ni = g.ice2 - g.ice1 + 1, nj = g.jci2 - g.jci1 + 1, nx = max(ni, nj);
  double c12 = 0.0, c22 = 0.0;
  for (int base = 0; base < nx; base += (int)blockDim.x) {
    const int x = base + (int)threadIdx.x;
    const int i = g.ice1 + x, j = g.jci1 + x;
    const bool wi = x < ni, sj = x < nj;
    const bool ow = wi && g.bl, oe = wi && g.br, os = sj && g.bb, on = sj && g.bt;
    if (base == 0) { c12 = F3(a1qc, g.jci1, g.ice2, k); c22 = F3(a1qc, g.jci2, g.ice2, k); }
    const bool late = base > 0 && i == g.ice2;       // (jci1|jci2, ice2) after the first chunk
    // operands (lanes without a line read their own row's valid address and discard it)
    const int ia = wi ? i : g.ice1, ja = sj ? j : g.jci1;
    const double qwi = late ? c12 : F3(a1qc, g.jci1, ia, k), pwi = ps(g.jci1, ia), pwe = ps(g.jce1, ia);
    const double qei = late ? c22 : F3(a1qc, g.jci2, ia, k), pei = ps(g.jci2, ia), pee = ps(g.jce2, ia);
    const double ww = SLI(sl.s[0], ia, k) + SLI(sl.s[0], ia + 1, k) + SLI(sl.s[1], ia, k) + SLI(sl.s[1], ia + 1, k);
    const double we = SLI(sl.s[2], ia, k) + SLI(sl.s[2], ia + 1, k) + SLI(sl.s[3], ia, k) + SLI(sl.s[3], ia + 1, k);
    const double qsi = F3(a1qc, ja, g.ici1, k), psi = ps(ja, g.ici1), pse = ps(ja, g.ice1);
    const double qni = F3(a1qc, ja, g.ici2, k), pni = ps(ja, g.ici2), pne = ps(ja, g.ice2);
    const double ws = SLJ(sl.s[12], ja, k) + SLJ(sl.s[12], ja + 1, k) + SLJ(sl.s[13], ja, k) + SLJ(sl.s[13], ja + 1, k);
    const double wn = SLJ(sl.s[14], ja, k) + SLJ(sl.s[14], ja + 1, k) + SLJ(sl.s[15], ja, k) + SLJ(sl.s[15], ja + 1, k);
    if (base == 0) __syncthreads();                  // every read of the shared points is done
    if (ow) F3(a1qc, g.jce1, i, k) = (ww > d_zero) ? d_zero : (qwi / pwi) * pwe;
    if (oe) F3(a1qc, g.jce2, i, k) = (we < d_zero) ? d_zero : (qei / pei) * pee;
    if (os) F3(a1qc, j, g.ice1, k) = (ws > d_zero) ? d_zero : (qsi / psi) * pse;
    if (on) F3(a1qc, j, g.ice2, k) = (wn < d_zero) ? d_zero : (qni / pni) * pne;
  }
}

}  // namespace rcm
