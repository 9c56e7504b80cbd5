/* orbx_sincos.h -- deterministic float sin/cos used by the rotated-BRIEF stage.
 *
 * The reference computes the sample rotation with glibc `sincosf`
 * (/root/reference/src/ORBextractor.cc:58-59: `cos(angle)`, `sin(angle)` on a
 * float, merged into one `sincosf` call by GCC -- SURVEY.md §0.3, App. A7).
 * glibc's single-precision sincosf is not correctly rounded, so a device
 * implementation cannot simply be "accurate": it must reproduce the host
 * library bit for bit wherever the difference would move a BRIEF sample.
 *
 * Strategy (identical on host and device):
 *   1. `orbx_sincos_core` evaluates sin/cos in double precision with only
 *      IEEE add/sub/mul (Cody-Waite pi/2 reduction + fdlibm kernel
 *      polynomials) and rounds to float.  Compiled with -ffp-contract=off on
 *      both gcc and hipcc, so host and device results are bit-identical.
 *   2. tools/gen_sincos_table.c enumerates EVERY float angle the extractor can
 *      produce (x in [0, f32(360*factorPI)]) against the host's glibc
 *      `sincosf`, and records the inputs where the two disagree AND the
 *      disagreement changes at least one of the 512 BRIEF sample positions.
 *      Those (x, sin, cos) triples are the exception table
 *      (sincos_exceptions.inc), looked up by `orbx_brief_sincos`.
 * Result: for every reachable angle, the 512 sample positions equal the ones
 * the reference computes with glibc sincosf.
 */
#ifndef ORBX_SINCOS_H
#define ORBX_SINCOS_H

#include <stdint.h>

#if defined(__HIPCC__)
#define ORBX_HD __host__ __device__
#else
#define ORBX_HD
#endif

/* pi/2 split for Cody-Waite reduction (fdlibm's PIO2_1 / PIO2_1T):
 * PIO2_1 has 33 significant bits, so k*PIO2_1 is exact for |k| < 2^20. */
#define ORBX_PIO2_1   1.57079632673412561417e+00
#define ORBX_PIO2_1T  6.07710050650619224932e-11
#define ORBX_INVPIO2  6.36619772367581382433e-01

static ORBX_HD inline double orbx_floor_d(double v) {
  /* exact floor without a library call (|v| < 2^52 here) */
  double t = (double)(int64_t)v;
  return (t > v) ? t - 1.0 : t;
}

static ORBX_HD inline double orbx_ksin(double r) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = r * r;
  double p = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return r + r * z * (S1 + z * p);
}

static ORBX_HD inline double orbx_kcos(double r) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = r * r;
  double p = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  return (1.0 - 0.5 * z) + z * p;
}

/* float sin/cos of a float argument, |x| < 1e5 */
static ORBX_HD inline void orbx_sincos_core(float x, float* s, float* c) {
  double xd = (double)x;
  double kd = orbx_floor_d(xd * ORBX_INVPIO2 + 0.5);
  int k = (int)kd;
  double r = (xd - kd * ORBX_PIO2_1) - kd * ORBX_PIO2_1T;
  double sr = orbx_ksin(r), cr = orbx_kcos(r);
  double sv, cv;
  switch (k & 3) {
    case 0: sv = sr; cv = cr; break;
    case 1: sv = cr; cv = -sr; break;
    case 2: sv = -sr; cv = -cr; break;
    default: sv = -cr; cv = sr; break;
  }
  *s = (float)sv;
  *c = (float)cv;
}

static ORBX_HD inline uint32_t orbx_f2u(float f) {
  union { float f; uint32_t u; } v;
  v.f = f;
  return v.u;
}

static ORBX_HD inline float orbx_u2f(uint32_t u) {
  union { float f; uint32_t u; } v;
  v.u = u;
  return v.f;
}

#endif /* ORBX_SINCOS_H */
