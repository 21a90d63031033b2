// Host accuracy check of regcm_amd/csrc/fastmath.hpp against long-double references:
// prints the maximum error in ulps of rcm_log, rcm_exp and rcm_powpos over seeded samples
// of the argument ranges the dyn step uses.
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <random>
#include "../../regcm_amd/csrc/fastmath.hpp"

static double ulp_err(double got, long double ref) {
  const double r = (double)ref;
  const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
  return (double)(std::fabs((long double)got - ref) / u);
}

int main() {
  std::mt19937_64 g(20261015);
  std::uniform_real_distribution<double> ulog(-14.0, 14.0), unear(0.8, 1.25), uexp(-8.0, 8.0);
  std::uniform_real_distribution<double> uy(0.05, 1.0);
  double elog = 0, eexp = 0, epow = 0;
  for (int n = 0; n < 4000000; n++) {
    const double x = (n & 1) ? std::exp(ulog(g)) : unear(g);
    elog = std::fmax(elog, ulp_err(rcm::rcm_log(x), logl((long double)x)));
    const double a = uexp(g);
    eexp = std::fmax(eexp, ulp_err(rcm::rcm_exp(a), expl((long double)a)));
    const double b = unear(g), y = uy(g);
    epow = std::fmax(epow, ulp_err(rcm::rcm_powpos(b, y), powl((long double)b, (long double)y)));
  }
  std::printf("%.3f %.3f %.3f\n", elog, eexp, epow);
  return 0;
}
