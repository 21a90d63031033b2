// Host check of rcm::div_by (regcm_amd/csrc/fastmath.hpp): x / y from a precomputed 1 / y must
// have exactly the bits of the IEEE division.  Prints the number of mismatches over seeded
// operand pairs: the step's ranges (p*, map-factor scales, tendencies of any sign and size),
// random exponents, denominators near 1, and uniformly random mantissas (the hard cases).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <random>
#include "../../regcm_amd/csrc/fastmath.hpp"

int main() {
  std::mt19937_64 g(20261018);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  long bad = 0, n = 0;
  for (long it = 0; it < 10000000; it++) {
    double x, y;
    switch (it % 5) {
      case 0: y = 50.0 + 60.0 * u(g); x = (u(g) - 0.5) * std::pow(10.0, 12.0 * u(g) - 6.0); break;
      case 1: y = 2.0e3 * (0.9 + 0.2 * u(g)) * 3000.0; x = (u(g) - 0.5) * 1.0e3; break;
      case 2: y = std::ldexp(1.0 + u(g), (int)(40 * u(g)) - 20);
              x = std::ldexp(1.0 + u(g), (int)(80 * u(g)) - 40) * (u(g) < 0.5 ? -1.0 : 1.0); break;
      case 3: y = 1.0 + u(g) * 1.0e-3; x = u(g); break;
      default: {
        uint64_t a = g(), b = g();
        a = (a & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
        b = (b & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
        std::memcpy(&x, &a, 8); std::memcpy(&y, &b, 8);
        x = std::ldexp(x, (int)(20 * u(g)) - 10);
      }
    }
    const double r = 1.0 / y;
    const double q1 = rcm::div_by(x, y, r), q2 = x / y;
    n++;
    if (std::memcmp(&q1, &q2, 8)) bad++;
  }
  // zeros keep their sign
  const double z1 = rcm::div_by(-0.0, 3.0, 1.0 / 3.0), z2 = rcm::div_by(0.0, 3.0, 1.0 / 3.0);
  if (!std::signbit(z1) || std::signbit(z2)) bad++;
  std::printf("%ld %ld\n", n, bad);
  return 0;
}
