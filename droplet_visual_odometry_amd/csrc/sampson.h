// The RANSAC score's inlier test (EMEstimatorCallback::computeError +
// findInliers, reached from visual_odometry_v3.py:297), shared by the device
// code (geometry.hip) and the host checker tests/sampson_check.cpp, so the
// single-precision bound is exercised on the host with the same source.
// Compile with -ffp-contract=off (the f64 expressions mirror OpenCV's).
#pragma once
#include <math.h>
#include <float.h>
#ifdef __HIPCC__
#define DVO_HD __host__ __device__
#else
#define DVO_HD
#endif

namespace dvo {

// EMEstimatorCallback::computeError (five-point.cpp): err = (float)(num / den)
// with num = (x2' E x1)^2 and den = the four squared epipolar terms; the
// inlier test err <= t (ptsetreg.cpp findInliers), decided without the f64
// division for all but a sliver of points.  With nf = fl32(num),
// df = fl32(den), s = fl32(t * df) (relative errors <= 2^-24 each while the
// values are normal floats, which the range checks on t and s guarantee):
//   nf < fl32(s * (1 - 2^-20))  =>  num < t * den  =>  fl64(num / den) <= t (RN is
//                                   monotone and t is a double), so (float) <= t;
//   nf > fl32(s * (1 + 2^-20))  =>  num / den > t (1 + 2^-21)  =>  the double
//                                   quotient is past t's rounding midpoint
//                                   (half an ulp <= t 2^-24), so (float) > t.
// (nf zero, denormal or +inf only strengthens either inequality.)  Otherwise,
// and for NaN, the exact division decides.  Bit-identical inlier sets.
DVO_HD inline bool sampson_inlier(const double* E, double x1, double y1, double x2, double y2, float t,
                                               bool fast_ok) {
    double ex0 = E[0] * x1 + E[1] * y1 + E[2] * 1.;
    double ex1 = E[3] * x1 + E[4] * y1 + E[5] * 1.;
    double ex2 = E[6] * x1 + E[7] * y1 + E[8] * 1.;
    double et0 = E[0] * x2 + E[3] * y2 + E[6] * 1.;
    double et1 = E[1] * x2 + E[4] * y2 + E[7] * 1.;
    double x2tEx1 = x2 * ex0 + y2 * ex1 + 1. * ex2;
    double a = ex0 * ex0, b = ex1 * ex1, c = et0 * et0, d = et1 * et1;
    const double num = x2tEx1 * x2tEx1, den = a + b + c + d;
    if (fast_ok) {
        const float nf = (float)num, s = t * (float)den;
        if (s >= 1e-30f && s <= 1e30f) {
            if (nf < s * (1.f - 0x1p-20f)) return true;
            if (nf > s * (1.f + 0x1p-20f)) return false;
        }
    }
    return (float)(num / den) <= t;
}

// The same decision from single-precision estimates, for the batched score
// (ransac_score_kernel): it settles all but a sliver of the model-point pairs, and the
// rest (and every value outside the ranges below) take sampson_inlier.  Inputs
// rounded to f32 (relative error u = 2^-24 each), products and sums as FMAs.
// With A_i = |E_i0 x1| + |E_i1 y1| + |E_i2|, B_i the same for E^T x2, and
// S = |x2| A0 + |y2| A1 + A2, the running-error bounds of both evaluations give
//   |fr - r64| <= (7u + 7u_64) S         (r = x2' E x1; u_64 = 2^-53)
//   |df - den64| <= 12.01u D,  D = A0^2 + A1^2 + B0^2 + B1^2 <= 4 (M (2P + 1))^2
// (M = max |E_ij| of the model, P = max |coordinate| of the point).  The code
// bounds them by Er = 2^-21 S_f (S_f, computed from |f32 inputs| with FMAs, is
// >= S (1 - 6u)) and Edn = 2^-18 (1 + 2^-20) Q^2, Q = M_f (1 + 2^-19) (2 P_f + 1)
// (>= M (2P + 1) after the roundings).  Then
//   (|fr| + Er)^2 (1 + 2^-18) < t (df - Edn)          =>  num64 < t den64  (inlier)
//   (|fr| - Er)^2 > t (df + Edn) (1 + 2^-17), |fr| > Er  =>  num64 > t den64 (1 + 2^-21)  (outlier)
// as evaluated in f32 (the factors 1 + 2^-18 and 1 + 2^-17 absorb the
// comparisons' own roundings, < 8u); these are the two sufficient conditions of
// sampson_inlier's proof.  The ranges keep every intermediate a normal float.
struct SampsonF32 {
    float e[9], mk;
    bool ok;
    SampsonF32() = default;
    DVO_HD SampsonF32(const double* E, bool t_ok) {
        float M = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            e[k] = (float)E[k];
            M = fmaxf(M, fabsf(e[k]));
        }
        mk = M * (1.f + 0x1p-19f);
        ok = t_ok && M >= 1e-15f && M <= 1e15f;
    }
    // 1 inlier, 0 outlier, -1 undecided
    DVO_HD inline int decide(float X1, float Y1, float X2, float Y2, float t) const {
        const float fx0 = fmaf(e[0], X1, fmaf(e[1], Y1, e[2]));
        const float fx1 = fmaf(e[3], X1, fmaf(e[4], Y1, e[5]));
        const float fx2 = fmaf(e[6], X1, fmaf(e[7], Y1, e[8]));
        const float ft0 = fmaf(e[0], X2, fmaf(e[3], Y2, e[6]));
        const float ft1 = fmaf(e[1], X2, fmaf(e[4], Y2, e[7]));
        const float fr = fmaf(X2, fx0, fmaf(Y2, fx1, fx2));
        const float df = fmaf(fx0, fx0, fmaf(fx1, fx1, fmaf(ft0, ft0, ft1 * ft1)));
        const float aX1 = fabsf(X1), aY1 = fabsf(Y1);
        const float A0 = fmaf(fabsf(e[0]), aX1, fmaf(fabsf(e[1]), aY1, fabsf(e[2])));
        const float A1 = fmaf(fabsf(e[3]), aX1, fmaf(fabsf(e[4]), aY1, fabsf(e[5])));
        const float A2 = fmaf(fabsf(e[6]), aX1, fmaf(fabsf(e[7]), aY1, fabsf(e[8])));
        const float S = fmaf(fabsf(X2), A0, fmaf(fabsf(Y2), A1, A2));
        const float Pf = fmaxf(fmaxf(aX1, aY1), fmaxf(fabsf(X2), fabsf(Y2)));
        const float Q = mk * (2.f * Pf + 1.f);
        const float edn = 0x1p-18f * (1.f + 0x1p-20f) * Q * Q;
        const float Er = 0x1p-21f * S;
        const float ar = fabsf(fr);
        const float a = ar + Er, b = ar - Er;
        const float R = t * (df - edn);
        const float R2 = t * (df + edn) * (1.f + 0x1p-17f);
        const bool in_range = ok && S >= 1e-15f && S <= 1e15f && Pf <= 1e6f;
        if (in_range && R >= 1e-30f && a * a * (1.f + 0x1p-18f) < R) return 1;
        if (in_range && b > 0.f && R2 >= 1e-30f && R2 <= 1e30f && b * b > R2) return 0;
        return -1;
    }
};

}  // namespace dvo
