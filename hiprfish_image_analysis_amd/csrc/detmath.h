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
#define HRF_DM_TAB static constexpr
#else
#define HRF_DM_FN static inline
#define HRF_DM_TAB static const
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

/* ---- correctly rounded log / log10 -------------------------------------------------------
 * image_cn = log(sum + 1e-2) (ecoli measurement.py:72) feeds the KMeans thresholds and the
 * watershed priorities, so a last-ulp difference can move a pixel between clusters or reorder a
 * watershed contest.  numpy's own log is not a fixed function: its AVX-512 path (SVML) and glibc
 * differ in the last ulp on ~3e-4 of inputs, and neither is correctly rounded everywhere.  libhrf
 * and the oracle therefore both use the correctly rounded logarithm, computed in double-double
 * (relative error < 2^-100) from IEEE +, -, *, /, fma only, then rounded once: the two sides are
 * bit-identical by construction, and equal to the exact log rounded to nearest except for inputs
 * within 2^-100 of a rounding midpoint (none in the checks: tests/test_oracle_golden.py compares
 * against Python's decimal ln at 50 digits).
 *
 * x = m 2^e, m in [0.75, 1.5); c = k/128 the nearest multiple of 1/128 (exact, k in 96..192);
 * log m = log c + 2 atanh(s), s = (m - c) / (m + c), |s| < 2^-8.5; the series' s, s^3/3, s^5/5
 * in double-double, s^7/7 .. s^13/13 in double; log c and ln 2 from double-double tables. */
HRF_DM_FN void hrf_dd_two_sum(double a, double b, double *s, double *e) {
  const double t = a + b, bb = t - a;
  *e = (a - (t - bb)) + (b - bb);
  *s = t;
}
HRF_DM_FN void hrf_dd_fast(double a, double b, double *s, double *e) { /* |a| >= |b| or a == 0 */
  const double t = a + b;
  *e = b - (t - a);
  *s = t;
}
HRF_DM_FN void hrf_dd_add(double ah, double al, double bh, double bl, double *rh, double *rl) {
  double s, e, t, f;
  hrf_dd_two_sum(ah, bh, &s, &e);
  hrf_dd_two_sum(al, bl, &t, &f);
  e += t;
  hrf_dd_fast(s, e, &s, &e);
  e += f;
  hrf_dd_fast(s, e, rh, rl);
}
HRF_DM_FN void hrf_dd_mul(double ah, double al, double bh, double bl, double *rh, double *rl) {
  const double p = ah * bh;
  double e = fma(ah, bh, -p);
  e += ah * bl + al * bh;
  hrf_dd_fast(p, e, rh, rl);
}

/* BEGIN LOGTAB (gen_logtab.py) */
HRF_DM_TAB double hrf_logtab_hi[97] = {
  -0.2876820724517809, -0.27731928541623435, -0.26706278524904525, -0.2569104137850272,
  -0.24686007793152578, -0.2369097470783577, -0.22705745063534608, -0.2173012756899814,
  -0.2076393647782445, -0.1980699137620938, -0.18859116980755003, -0.179201429457711,
  -0.16989903679539747, -0.16068238169047347, -0.15154989812720093, -0.14250006260728304,
  -0.13353139262452263, -0.1246424452072766, -0.1158318155251217, -0.1070981355563671,
  -0.09844007281325252, -0.08985632912186105, -0.0813456394539524, -0.07290677080808779,
  -0.06453852113757118, -0.05623971832287608, -0.048009219186360606, -0.039845908547199674,
  -0.0317486983145803, -0.023716526617316044, -0.015748356968139168, -0.007843177461025893,
  0.0, 0.007782140442054949, 0.015504186535965254, 0.02316705928153438,
  0.030771658666753687, 0.0383188643021366, 0.0458095360312942, 0.053244514518812285,
  0.06062462181643484, 0.06795066190850775, 0.07522342123758753, 0.08244366921107459,
  0.08961215868968714, 0.09672962645855111, 0.10379679368164356, 0.11081436634029011,
  0.11778303565638346, 0.12470347850095724, 0.13157635778871926, 0.13840232285911913,
  0.1451820098444979, 0.15191604202584197, 0.15860503017663857, 0.16524957289530717,
  0.17185025692665923, 0.1784076574728183, 0.184922338494012, 0.19139485299962947,
  0.19782574332991987, 0.2042155414286909, 0.21056476910734964, 0.21687393830061436,
  0.22314355131420976, 0.22937410106484582, 0.2355660713127669, 0.24171993688714516,
  0.24783616390458127, 0.25391520998096345, 0.25995752443692605, 0.26596354849713794,
  0.27193371548364176, 0.2778684510034563, 0.2837681731306446, 0.28963329258304266,
  0.2954642128938359, 0.3012613305781618, 0.3070250352949119, 0.3127557100038969,
  0.3184537311185346, 0.324119468654212, 0.329753286372468, 0.3353555419211378,
  0.3409265869705932, 0.34646676734620857, 0.3519764231571782, 0.3574558889218038,
  0.3629054936893685, 0.3683255611587076, 0.37371640979358406, 0.37907835293496944,
  0.38441169891033206, 0.3897167511400252, 0.394993808240869, 0.4002431641270127,
  0.4054651081081644,
};
HRF_DM_TAB double hrf_logtab_lo[97] = {
  -2.607160616442564e-17, 7.44528405583513e-18, 7.32891532732017e-18, -2.502843296152504e-17,
  -1.361743371748368e-17, -1.9682402978398164e-18, -9.551415762738488e-18, -1.6168452453763015e-18,
  -1.2053243216686129e-17, -3.742843482461439e-18, 7.432164219196925e-18, 1.0785017454858423e-17,
  4.868008764439071e-19, 3.650183553047837e-18, -5.1669593684615594e-18, 9.926388234225749e-18,
  3.664457663660085e-18, 5.808912678940971e-18, -4.338484369808096e-18, 1.73705104015906e-18,
  4.439009633675136e-18, 6.273760163689594e-19, -5.07707635593117e-18, 6.306860257532778e-18,
  6.470486661692933e-18, 3.2835149805605613e-18, -1.4390903347292205e-18, 3.129547680315208e-18,
  -3.0382263084680858e-18, 1.5774243488668215e-18, -1.0021578630528974e-18, -2.764708154124904e-19,
  0.0, -1.2819179123343845e-20, -3.278321022892429e-19, -1.1769544932063305e-18,
  1.0431732029005968e-18, -2.357996157351286e-18, 1.902959866474257e-18, -1.665575816973663e-18,
  2.6424025938726934e-18, -1.2802141240611733e-18, -5.930604196293241e-18, 5.700437773813987e-18,
  -5.4268129336647135e-18, -5.597397486289965e-19, 5.47772415726659e-18, 1.183748342825649e-18,
  -1.1971685747593677e-18, -4.6522609636496624e-18, 1.1123000879729588e-17, 4.447777301357527e-18,
  8.242418783022475e-18, 6.4838631244022194e-18, 1.1257003872182592e-17, -1.0094935622322628e-17,
  -6.0224538210113705e-18, -1.2432553788701131e-17, 3.0236614153574064e-18, -1.2129496905792884e-17,
  1.2821194372980142e-17, 2.7338281018722773e-18, -4.249405314729895e-18, 4.551026193234283e-18,
  -9.091270597324799e-18, 9.927671823978025e-18, -2.3943371495187355e-18, 8.900990022166643e-18,
  -1.2432209578702523e-17, -8.048097394424201e-18, 2.069806938978935e-17, 5.3393802761314314e-18,
  7.83319637697442e-19, -9.16018294909263e-19, -2.032665581126656e-17, 2.0535953219858174e-17,
  -2.16461086040599e-17, -9.048511144048564e-18, -1.2319916200101964e-17, -1.451808353098951e-17,
  2.7114779367326236e-17, -7.958214381893813e-18, 2.122020616196946e-18, 1.834564437059473e-17,
  1.7467136443544747e-17, 1.028583585496265e-17, -1.2953893030191963e-17, -2.5136910072413547e-17,
  -2.1492361455310972e-17, 2.690672380132659e-17, 2.1836211281198184e-17, 1.587939415338447e-17,
  -1.612149700764673e-17, 2.734172667856699e-17, -1.5113724418336168e-17, -1.1349239205188711e-17,
  -2.8811380259626426e-18,
};
#define HRF_DD_LN2_HI 0.6931471805599453
#define HRF_DD_LN2_LO 2.3190468138462996e-17
#define HRF_DD_THIRD_HI 0.3333333333333333
#define HRF_DD_THIRD_LO 1.850371707708594e-17
#define HRF_DD_FIFTH_HI 0.2
#define HRF_DD_FIFTH_LO -1.1102230246251566e-17
#define HRF_DD_INVLN10_HI 0.4342944819032518
#define HRF_DD_INVLN10_LO 1.098319650216765e-17
/* END LOGTAB */

/* log(x) as a normalised double-double (x > 0 finite) */
HRF_DM_FN void hrf_dd_log(double x, double *rh, double *rl) {
  int e = 0;
  double m = frexp(x, &e); /* [0.5, 1) */
  if (m < 0.75) {
    m = m * 2.0;
    e -= 1;
  }
  const int k = (int)rint(m * 128.0);
  const double c = (double)k * 0.0078125;
  const double d = m - c; /* exact */
  double uh, ul;
  hrf_dd_two_sum(m, c, &uh, &ul);
  /* s = d / (uh + ul): the remainder of a correctly rounded quotient is exact under fma */
  const double q1 = d / uh;
  const double r = fma(-q1, uh, d) - q1 * ul;
  double sh, sl;
  hrf_dd_fast(q1, r / uh, &sh, &sl);
  double zh, zl, s3h, s3l, s5h, s5l, t3h, t3l, t5h, t5l;
  hrf_dd_mul(sh, sl, sh, sl, &zh, &zl);
  hrf_dd_mul(sh, sl, zh, zl, &s3h, &s3l);
  hrf_dd_mul(s3h, s3l, zh, zl, &s5h, &s5l);
  hrf_dd_mul(s3h, s3l, HRF_DD_THIRD_HI, HRF_DD_THIRD_LO, &t3h, &t3l);
  hrf_dd_mul(s5h, s5l, HRF_DD_FIFTH_HI, HRF_DD_FIFTH_LO, &t5h, &t5l);
  double p = fma(zh, 1.0 / 13.0, 1.0 / 11.0);
  p = fma(zh, p, 1.0 / 9.0);
  p = fma(zh, p, 1.0 / 7.0);
  const double tail = s5h * zh * p;
  double ah, al;
  hrf_dd_add(t5h, t5l, tail, 0.0, &ah, &al);
  hrf_dd_add(t3h, t3l, ah, al, &ah, &al);
  hrf_dd_add(sh, sl, ah, al, &ah, &al);
  ah *= 2.0;
  al *= 2.0;
  /* e ln2 + log c */
  const double de = (double)e;
  const double eh = de * HRF_DD_LN2_HI;
  double el = fma(de, HRF_DD_LN2_HI, -eh);
  el = fma(de, HRF_DD_LN2_LO, el);
  double bh, bl;
  hrf_dd_fast(eh, el, &bh, &bl);
  hrf_dd_add(bh, bl, hrf_logtab_hi[k - 96], hrf_logtab_lo[k - 96], &bh, &bl);
  hrf_dd_add(bh, bl, ah, al, rh, rl);
}

HRF_DM_FN double hrf_cr_log(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  double h, l;
  hrf_dd_log(x, &h, &l);
  return h + l;
}

HRF_DM_FN double hrf_cr_log10(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  double h, l;
  hrf_dd_log(x, &h, &l);
  hrf_dd_mul(h, l, HRF_DD_INVLN10_HI, HRF_DD_INVLN10_LO, &h, &l);
  return h + l;
}

/* x / d through its reciprocal r = 1.0 / d (correctly rounded), for x and d that are float32
 * values held as doubles, d finite and nonzero: q = x r, e = x - q d (exact under fma), q + e r
 * rounded once.  Equal to the IEEE quotient x / d: |x/d - q| <= 1.5 ulp, so the corrected sum is
 * within 2^-104 (relative) of x/d, while a quotient of two 24-bit significands is never within
 * 2^-78 of a double rounding midpoint (it would need m_d | m_x 2^54 with an odd multiplier).
 * The flat-field division of ecoli measurement.py:41 (image / calibration_norm) per calibrated
 * channel becomes one division per pixel plus three multiply-adds per channel.  Checked against
 * the division on random and directed float pairs (tests/test_oracle_golden.py). */
HRF_DM_FN double hrf_div_rcp(double x, double d, double r) {
  const double q = x * r;
  const double e = fma(-q, d, x);
  return fma(e, r, q);
}

/* BEGIN EXPTAB (gen_logtab.py) */
HRF_DM_TAB double hrf_exp2tab64[64] = {
  1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
  1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
  1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
  1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
  1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
  1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
  1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
  1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
  1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
  1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
  1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
  1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
  1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
  1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
  1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
  1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951,
};
#define HRF_EXP_INVL 92.33248261689366
#define HRF_EXP_L2HI 0.010830424696249145
#define HRF_EXP_L2LO 3.623510646634843e-19
/* END EXPTAB */

/* e^x for x in [-8, 0] (the NL-means weights, nlmeans.hip / oracle_nl_means): x = (64 m + j)
 * ln2/64 + r with k = rint(x * 64/ln2), |r| <= ln2/128 (Cody-Waite, two FMAs), then
 * 2^(j/64) (1 + q) with q = r + r^2/2 + ... + r^5/120 (truncation < 4e-17 relative) and an
 * exact scale by 2^m.  tab = hrf_exp2tab64 (the kernel passes its LDS copy).  Same operations
 * in the same order on both sides, so the kernel's weights equal the oracle's bit for bit. */
HRF_DM_FN double hrf_exp_neg_tab(double x, const double *tab) {
    const double k = rint(x * HRF_EXP_INVL);
    const int ki = (int)k;
    double r = fma(-k, HRF_EXP_L2HI, x);
    r = fma(-k, HRF_EXP_L2LO, r);
    double q = 1.0 / 120.0;
    q = fma(q, r, 1.0 / 24.0);
    q = fma(q, r, 1.0 / 6.0);
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = q * r;
    const double t = tab[ki & 63];
    return ldexp(fma(t, q, t), ki >> 6);
}

/* The same value for x in [-8, 0] from a widened table tabw[i] = 2^(-i/64), i = 0..739
 * (= ldexp(hrf_exp2tab64[-i & 63], -i >> 6), exact): fma(t 2^m, q, t 2^m) = 2^m fma(t, q, t)
 * exactly in the normal range, so the result equals hrf_exp_neg_tab's bit for bit without
 * the ldexp and the index split. */
#define HRF_EXP_WIDE_N 740
HRF_DM_FN double hrf_exp_neg_tabw(double x, const double *tabw) {
    const double k = rint(x * HRF_EXP_INVL);
    const int ki = (int)k;
    double r = fma(-k, HRF_EXP_L2HI, x);
    r = fma(-k, HRF_EXP_L2LO, r);
    double q = 1.0 / 120.0;
    q = fma(q, r, 1.0 / 24.0);
    q = fma(q, r, 1.0 / 6.0);
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = q * r;
    const double t = tabw[-ki];
    return fma(t, q, t);
}

/* x >= 0 (umap's squared distances): x^y */
HRF_DM_FN double hrf_det_pow(double x, double y) {
  if (x == 0.0) return y > 0.0 ? 0.0 : (y == 0.0 ? 1.0 : INFINITY);
  return hrf_det_exp(y * hrf_det_log(x));
}

#endif
