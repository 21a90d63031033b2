// fastmath.hpp -- fp64 log/exp for the positive, normal, moderate arguments of the dyn step.
//
// The step's transcendental calls (log in the hypsometric geopotential and the PGF,
// x**y in vadv3d/vadvqv) all take finite positive normal arguments, so the special-case
// handling of the general-purpose OCML routines (98 and 42 VALU instructions) is dead work in
// the dominant kernels.  These are the classic fdlibm algorithms (Sun, e_log.c / e_exp.c:
// argument reduction by ln 2, minimax polynomial with a division-based correction), error
// < 1 ulp, about 40 and 30 instructions.  tests/test_fastmath_cpu.py measures them against
// long-double references on the host (this header compiles for host and device).
//
// Domain: rcm_log(x) for finite x > 0 (normal); rcm_exp(x) for |x| < 700.
#pragma once
#include <cmath>

#if defined(__HIP__) || defined(__HIPCC__)
#define RCM_HD __host__ __device__ __forceinline__
#else
#define RCM_HD inline
#endif

namespace rcm {

// The device reads the polynomial coefficients from constant memory: scalar loads into SGPRs,
// where the compiler would otherwise materialise each 64-bit literal in a VGPR pair, hoist it
// out of the kernel's level loops and spill it (k_columns).
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ double rcm_fm_c[16] = {
    6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01,
    1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01, 1.66666666666666019037e-01,
    -2.77777777770155933842e-03, 6.61375632143793436117e-05, -1.65339022054652515390e-06,
    4.13813679705723846039e-08, 0.0, 0.0, 0.0, 0.0};
#define RCM_FMC(i, v) rcm_fm_c[i]
#else
#define RCM_FMC(i, v) (v)
#endif

RCM_HD double rcm_log(double x) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = RCM_FMC(0, 6.666666666666735130e-01), Lg2 = RCM_FMC(1, 3.999999999940941908e-01);
  const double Lg3 = RCM_FMC(2, 2.857142874366239149e-01), Lg4 = RCM_FMC(3, 2.222219843214978396e-01);
  const double Lg5 = RCM_FMC(4, 1.818357216161805012e-01), Lg6 = RCM_FMC(5, 1.531383769920937332e-01);
  const double Lg7 = RCM_FMC(6, 1.479819860511658591e-01);
  int e;
  double m = std::frexp(x, &e);                 // x = m * 2^e, m in [0.5, 1)
  if (m < 0.70710678118654752440) { m = m + m; e = e - 1; }   // m in [sqrt(1/2), sqrt(2))
  const double f = m - 1.0;                     // exact
  const double s = f / (2.0 + f);
  const double dk = (double)e;
  const double z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

RCM_HD double rcm_exp(double x) {
  constexpr double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
  constexpr double invln2 = 1.44269504088896338700e+00;
  const double P1 = RCM_FMC(7, 1.66666666666666019037e-01), P2 = RCM_FMC(8, -2.77777777770155933842e-03);
  const double P3 = RCM_FMC(9, 6.61375632143793436117e-05), P4 = RCM_FMC(10, -1.65339022054652515390e-06);
  const double P5 = RCM_FMC(11, 4.13813679705723846039e-08);
  const double k = std::rint(x * invln2);      // x = k ln2 + r, |r| <= ln2/2
  const double hi = x - k * ln2HI;             // k * ln2HI exact for |k| < 2^11
  const double lo = k * ln2LO;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return std::ldexp(y, (int)k);
}

// x**y for x > 0
RCM_HD double rcm_powpos(double x, double y) { return rcm_exp(y * rcm_log(x)); }

// x / y from r = 1.0 / y (an IEEE division formed once for a loop-invariant y): q = RN(x r) is
// faithful, the remainder x - q y is exact in an FMA, and RN(q + r (x - q y)) is the correctly
// rounded quotient (Markstein's theorem; finite normal operands), so the result has the bits of
// x / y in three dependent FMA-pipe operations instead of the ~10 of a full division.  A zero
// remainder means q = x / y exactly (and keeps the sign of a zero quotient).
// tests/test_fastmath_cpu.py checks the identity on the host over 10^7 operand pairs.
#ifndef RCM_MDIV
#define RCM_MDIV 1
#endif
RCM_HD double div_by(double x, double y, double r) {
#if RCM_MDIV
  const double q = x * r;
  const double e = __builtin_fma(-q, y, x);
  return e == 0.0 ? q : __builtin_fma(e, r, q);
#else
  (void)r;
  return x / y;
#endif
}

}  // namespace rcm
