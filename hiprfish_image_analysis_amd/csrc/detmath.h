/* detmath.h -- exp / log / pow written out in IEEE double operations (+, *, /, fma, ldexp,
 * frexp, rint), so the device (hipcc, -ffp-contract=off) and the CPU restatement (gcc, oracle/)
 * compute them bit for bit alike.  The library functions are not: the device libm and glibc
 * round differently in the last ulp, and a one-ulp difference inside an iterative layout
 * (umap's refinement) grows into a different embedding.
 *
 * Accuracy: exp within ~1 ulp (Cody-Waite reduction, degree-13 Taylor polynomial), log within
 * ~1 ulp (atanh series on [sqrt(1/2), sqrt(2))), pow = exp(y log x) within ~|y log x| ulp.
 * Used where the reference's own arithmetic is unpinned (umap-learn is absent; its numba
 * code uses float32 state), so the choice of exp / pow is ours, and the same on both sides.
 *
 * Plain C (the oracle includes it) and HIP (host + device). */
#ifndef HRF_DETMATH_H
#define HRF_DETMATH_H

#include <math.h>

#ifdef __HIPCC__
#define HRF_DM_FN static inline __host__ __device__
#else
#define HRF_DM_FN static inline
#endif

HRF_DM_FN double hrf_det_exp(double x) {
  if (x != x) return x;
  if (x > 709.782712893384) return INFINITY;
  if (x < -745.2) return 0.0;
  const double k = rint(x * 1.4426950408889634);
  double r = fma(-k, 6.93147180369123816490e-01, x); /* ln2 hi */
  r = fma(-k, 1.90821492927058770002e-10, r);          /* ln2 lo */
  double p = 1.0 / 6227020800.0;                       /* 1/13! */
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)k);
}

HRF_DM_FN double hrf_det_log(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  int e = 0;
  double m = frexp(x, &e); /* x = m 2^e, m in [0.5, 1) */
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  /* log(m) = 2 atanh(s), s = (m - 1) / (m + 1), |s| < 0.1716 */
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double p = 1.0 / 25.0;
  p = fma(p, z, 1.0 / 23.0);
  p = fma(p, z, 1.0 / 21.0);
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  const double lm = fma(2.0 * s * z, p, 2.0 * s); /* 2s + 2s z p */
  const double de = (double)e;
  return fma(de, 6.93147180369123816490e-01, fma(de, 1.90821492927058770002e-10, lm));
}

/* x >= 0 (umap's squared distances): x^y */
HRF_DM_FN double hrf_det_pow(double x, double y) {
  if (x == 0.0) return y > 0.0 ? 0.0 : (y == 0.0 ? 1.0 : INFINITY);
  return hrf_det_exp(y * hrf_det_log(x));
}

#endif
