// Host build of the device Dirichlet sampler (csrc/az_random.h), test
// infrastructure for tests/test_dirichlet_cpu.py:
//   dirichlet_check funcs N         -> mismatches of glibc_log / glibc_pow
//                                      (the restatement) against this host's
//                                      glibc log / pow on N arguments of each
//                                      kind the gamma sampler passes them, and
//                                      general / subnormal-result ones
//   dirichlet_check draw SEED K ALPHA N -> N Dirichlet(ALPHA * ones(K)) draws
//                                      from MT19937(SEED), one per line, hex
// Built with -ffp-contract=off like the tree kernels that include the header.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "../../custom-alphazero_amd/csrc/az_random.h"

static double (*volatile g_log)(double) = log;
static double (*volatile g_pow)(double, double) = pow;

struct Mt {
  std::mt19937 m;
  uint32_t operator()() { return (uint32_t)m(); }
};

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "funcs")) {
    const long n = atol(argv[2]);
    Mt mt{std::mt19937(12345)};
    const double shape = 0.03, inv = 1.0 / shape;
    long bad_exp = 0, bad_pow = 0, bad_log2 = 0, bad_pow2 = 0, bad_gen = 0, bad_sub = 0;
    for (long i = 0; i < n; ++i) {
      const double u = az::legacy_double(mt), w = az::legacy_double(mt);
      // exponential: log(1 - u)
      if (az::glibc_log(1.0 - u) != g_log(1.0 - u)) ++bad_exp;
      // branch 1: pow(U, 1/shape), U <= 1 - shape
      const double U1 = u * (1.0 - shape);
      if (az::glibc_pow(U1, inv) != g_pow(U1, inv)) ++bad_pow;
      // branch 2: Y = -log((1 - U)/shape), pow(1 - shape + shape Y, 1/shape)
      const double U2 = 1.0 - shape + w * shape;
      const double a = (1.0 - U2) / shape;
      if (a > 0.0) {
        if (az::glibc_log(a) != g_log(a)) ++bad_log2;
        const double Y = -g_log(a);
        const double b = 1.0 - shape + shape * Y;
        if (az::glibc_pow(b, inv) != g_pow(b, inv)) ++bad_pow2;
      }
      // general arguments: x in (0, 4), exponents in (0.5, 40)
      const double x = 4.0 * u + 1e-300, p = 0.5 + 39.5 * w;
      if (az::glibc_pow(x, p) != g_pow(x, p) || az::glibc_log(x) != g_log(x)) ++bad_gen;
      // results near and below 2^-1022 (exp_inline's special case), x near 1
      // (log's second polynomial) and subnormal x
      const double xs = ldexp(0.5 + 0.5 * u, -(int)(w * 40.0)), ps = 1.0 / (0.01 + 0.04 * w) * 18.0;
      const double x1 = 1.0 + (u - 0.5) * 0x1p-3, xd = ldexp(u + 1e-9, -1060);
      if (az::glibc_pow(xs, ps) != g_pow(xs, ps) || az::glibc_log(x1) != g_log(x1) ||
          az::glibc_log(xd) != g_log(xd) || az::glibc_pow(xd, 0.5 + w) != g_pow(xd, 0.5 + w) ||
          az::glibc_pow(x1, 40.0 * w + 1.0) != g_pow(x1, 40.0 * w + 1.0))
        ++bad_sub;
    }
    printf("%ld %ld %ld %ld %ld %ld\n", bad_exp, bad_pow, bad_log2, bad_pow2, bad_gen, bad_sub);
    return 0;
  }
  if (argc >= 6 && !strcmp(argv[1], "draw")) {
    Mt mt{std::mt19937((uint32_t)strtoul(argv[2], nullptr, 10))};
    const int k = atoi(argv[3]);
    const double alpha = strtod(argv[4], nullptr);
    const long n = atol(argv[5]);
    double g[256];
    for (long i = 0; i < n; ++i) {
      double acc = 0.0;
      for (int j = 0; j < k; ++j) {
        g[j] = az::legacy_standard_gamma(mt, alpha);
        acc = acc + g[j];
      }
      const double invacc = 1.0 / acc;
      for (int j = 0; j < k; ++j) printf("%a%c", g[j] * invacc, j + 1 < k ? ' ' : '\n');
    }
    return 0;
  }
  fprintf(stderr, "usage\n");
  return 2;
}
