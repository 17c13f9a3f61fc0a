// az_random.h -- the reference's Dirichlet root noise draws (ConfigMCTS.
// enable_dirichlet_noise, mcts/mcts.py:70-85): numpy's LEGACY
// RandomState.dirichlet(alpha * ones(k)) on the game's MT19937 stream,
// restated for the device (and the host, for tests).
//
// numpy 1.x RandomState (mtrand.pyx dirichlet, legacy-distributions.c
// legacy_standard_gamma), which the reference's np.random.dirichlet is:
//   per component j: g_j = legacy_standard_gamma(alpha_j); acc += g_j
//   invacc = 1 / acc; d_j = g_j * invacc
//   legacy_standard_gamma(shape < 1), Johnk/Best rejection:
//     loop: U = legacy_double; V = -log(1 - legacy_double)
//       U <= 1 - shape: X = pow(U, 1/shape); accept if X <= V
//       else:           Y = -log((1 - U) / shape);
//                       X = pow(1 - shape + shape * Y, 1/shape); accept if X <= V + Y
//   shape == 1: -log(1 - legacy_double)
//   legacy_double = ((a >> 5) * 2^26 + (b >> 6)) / 2^53 of two MT19937 words
// Every float64 operation is the reference's, in its order (this header is
// only included by translation units built with -ffp-contract=off).  log and
// pow are evaluated in double-double arithmetic (~2^-100 relative) and
// rounded once: correctly rounded except within ~2^-45 of a rounding
// boundary; glibc's log/pow (what numpy calls) are within 0.52 ULP and round
// the same way everywhere else -- tests/test_dirichlet_cpu.py compares both
// on millions of the sampler's own arguments and the whole sampler against
// numpy's RandomState.dirichlet.
#pragma once
#include <math.h>
#include <stdint.h>

#include "az_device.h"

namespace az {

struct dd {
  double hi, lo;
};

AZ_HD dd dd_two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
AZ_HD dd dd_fast(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return {s, b - (s - a)};
}
AZ_HD dd dd_two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
AZ_HD dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
AZ_HD dd dd_add(dd a, dd b) {
  dd s = dd_two_sum(a.hi, b.hi);
  const dd t = dd_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_fast(s.hi, s.lo);
  s.lo += t.lo;
  return dd_fast(s.hi, s.lo);
}
AZ_HD dd dd_mul(dd a, dd b) {
  dd p = dd_two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return dd_fast(p.hi, p.lo);
}
AZ_HD dd dd_mul_d(dd a, double b) {
  dd p = dd_two_prod(a.hi, b);
  p.lo += a.lo * b;
  return dd_fast(p.hi, p.lo);
}
AZ_HD dd dd_div(dd a, dd b) {
  const double q1 = a.hi / b.hi;
  dd r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
  const double q2 = r.hi / b.hi;
  r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
  const double q3 = r.hi / b.hi;
  return dd_add(dd_fast(q1, q2), dd{q3, 0.0});
}

// ln 2 = kLn2[0] + kLn2[1] + kLn2[2]; kLn2[0] has 32 significant bits (k * it is exact)
#define AZ_LN2_0 0x1.62e42fee00000p-1
#define AZ_LN2_1 0x1.a39ef35793c76p-33
#define AZ_LN2_2 0x1.cc01f97b57a08p-87

// ln(x) as a double-double, x > 0 finite: x = m 2^e, m in [1/sqrt2, sqrt2),
// ln m = 2 atanh(s), s = (m - 1)/(m + 1) (|s| <= 0.1716), series to s^45
AZ_HD dd dd_log(double x) {
  // 1/(2k+1), k = 0..22, as double-doubles
  const double C[23][2] = {
      {0x1.0000000000000p+0, 0x0.0p+0},          {0x1.5555555555555p-2, 0x1.5555555555555p-56},
      {0x1.999999999999ap-3, -0x1.999999999999ap-57}, {0x1.2492492492492p-3, 0x1.2492492492492p-57},
      {0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58},  {0x1.745d1745d1746p-4, -0x1.745d1745d1746p-59},
      {0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58}, {0x1.1111111111111p-4, 0x1.1111111111111p-60},
      {0x1.e1e1e1e1e1e1ep-5, 0x1.e1e1e1e1e1e1ep-61},  {0x1.af286bca1af28p-5, 0x1.af286bca1af28p-59},
      {0x1.8618618618618p-5, 0x1.8618618618618p-59},  {0x1.642c8590b2164p-5, 0x1.642c8590b2164p-60},
      {0x1.47ae147ae147bp-5, -0x1.eb851eb851eb8p-61}, {0x1.2f684bda12f68p-5, 0x1.2f684bda12f68p-59},
      {0x1.1a7b9611a7b96p-5, 0x1.1a7b9611a7b96p-61},  {0x1.0842108421084p-5, 0x1.0842108421084p-60},
      {0x1.f07c1f07c1f08p-6, -0x1.f07c1f07c1f08p-61}, {0x1.d41d41d41d41dp-6, 0x1.0750750750750p-60},
      {0x1.bacf914c1bad0p-6, -0x1.bacf914c1bad0p-60}, {0x1.a41a41a41a41ap-6, 0x1.0690690690690p-60},
      {0x1.8f9c18f9c18fap-6, -0x1.f3831f3831f38p-61}, {0x1.7d05f417d05f4p-6, 0x1.7d05f417d05f4p-62},
      {0x1.6c16c16c16c17p-6, -0x1.f49f49f49f49fp-61}};
  int e = 0;
  double m = frexp(x, &e);  // [0.5, 1)
  if (m < 0x1.6a09e667f3bcdp-1) {
    m *= 2.0;
    e -= 1;
  }
  const dd num{m - 1.0, 0.0};  // exact (Sterbenz)
  const dd s = dd_div(num, dd_two_sum(m, 1.0));
  const dd s2 = dd_mul(s, s);
  dd acc{C[22][0], C[22][1]};
  for (int k = 21; k >= 0; --k) acc = dd_add(dd_mul(acc, s2), dd{C[k][0], C[k][1]});
  dd t = dd_mul(s, acc);
  t.hi *= 2.0;
  t.lo *= 2.0;
  const double ed = (double)e;
  dd el = dd_add(dd_fast(ed * AZ_LN2_0, 0.0), dd_two_prod(ed, AZ_LN2_1));
  el = dd_add(el, dd{ed * AZ_LN2_2, 0.0});
  return dd_add(el, t);
}

// exp(y), correctly rounded (up to ~2^-95 of a tie), y a double-double
AZ_HD double dd_exp_rn(dd y) {
  // 1/n!, n = 0..15
  const double F[16][2] = {
      {0x1.0000000000000p+0, 0x0.0p+0},          {0x1.0000000000000p+0, 0x0.0p+0},
      {0x1.0000000000000p-1, 0x0.0p+0},          {0x1.5555555555555p-3, 0x1.5555555555555p-57},
      {0x1.5555555555555p-5, 0x1.5555555555555p-59},  {0x1.1111111111111p-7, 0x1.1111111111111p-63},
      {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65}, {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73},
      {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},  {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
      {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76},  {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80},
      {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83}, {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
      {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92},  {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97}};
  if (y.hi != y.hi) return y.hi;
  if (y.hi > 710.0) return INFINITY;
  if (y.hi < -746.0) return 0.0;
  const double kd = rint(y.hi * 0x1.71547652b82fep+0);
  dd r = dd_add(y, dd{-kd * AZ_LN2_0, 0.0});  // k * LN2_0 exact
  r = dd_add(r, dd_neg(dd_two_prod(kd, AZ_LN2_1)));
  r = dd_add(r, dd{-kd * AZ_LN2_2, 0.0});
  // expm1(r / 32) by Taylor to r^15, then expm1(2z) = 2 expm1(z) + expm1(z)^2, five times
  r.hi *= 0x1p-5;
  r.lo *= 0x1p-5;
  dd p{F[15][0], F[15][1]};
  for (int n = 14; n >= 1; --n) p = dd_add(dd_mul(p, r), dd{F[n][0], F[n][1]});
  dd em = dd_mul(p, r);
  for (int i = 0; i < 5; ++i) em = dd_add(dd{2.0 * em.hi, 2.0 * em.lo}, dd_mul(em, em));
  const dd v = dd_add(dd{1.0, 0.0}, em);  // normalised: v.hi = round(v)
  const int k = (int)kd;
  int ev = 0;
  frexp(v.hi, &ev);
  if (k + ev - 1 >= -1022) return ldexp(v.hi, k);  // exact scaling (overflow -> inf)
  // subnormal result: round (v.hi + v.lo) 2^k on the 2^-1074 grid, ties to even
  const int sh = k + 1074;  // v * 2^sh units of 2^-1074 (< 2^53)
  if (sh < -2) return 0.0;
  const double a = ldexp(v.hi, sh), b = ldexp(v.lo, sh);
  double n = rint(a);
  const double d = (a - n) + b;
  if (d > 0.5 || (d == 0.5 && fmod(n, 2.0) != 0.0)) n += 1.0;
  else if (d < -0.5 || (d == -0.5 && fmod(n, 2.0) != 0.0)) n -= 1.0;
  return ldexp(n, -1074);
}

AZ_HD double rn_log(double x) {  // libm log for x > 0 finite; log(0) = -inf
  if (x == 0.0) return -INFINITY;
  if (x == 1.0) return 0.0;
  const dd l = dd_log(x);
  return l.hi;  // dd_add normalises: hi = round(hi + lo)
}

AZ_HD double rn_pow(double x, double p) {  // libm pow for x >= 0 finite, p > 0 finite
  if (x == 0.0) return 0.0;
  if (x == 1.0) return 1.0;
  return dd_exp_rn(dd_mul_d(dd_log(x), p));
}

// numpy legacy_double on a 32-bit word source
template <typename Next32>
AZ_HD double legacy_double(Next32& next) {
  const uint32_t a = next() >> 5;
  const uint32_t b = next() >> 6;
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

template <typename Next32>
AZ_HD double legacy_standard_exponential(Next32& next) {
  return -rn_log(1.0 - legacy_double(next));
}

// legacy_standard_gamma for 0 < shape <= 1 (the engine refuses larger shapes)
template <typename Next32>
AZ_HD double legacy_standard_gamma(Next32& next, double shape) {
  if (shape == 1.0) return legacy_standard_exponential(next);
  const double inv = 1.0 / shape;
  for (;;) {
    const double U = legacy_double(next);
    const double V = legacy_standard_exponential(next);
    if (U <= 1.0 - shape) {
      const double X = rn_pow(U, inv);
      if (X <= V) return X;
    } else {
      const double Y = -rn_log((1.0 - U) / shape);
      const double X = rn_pow(1.0 - shape + shape * Y, inv);
      if (X <= V + Y) return X;
    }
  }
}

}  // namespace az
