// Host checker of the RANSAC score's single-precision Sampson decision
// (droplet_visual_odometry_amd/csrc/sampson.h, the same source the device
// compiles): every decided point must match the f64 test.  Cases: realistic
// correspondences of random essential matrices, points placed at relative
// distances 1e-12 .. 1e-1 from the threshold on both sides, and extreme
// scales.  Prints "cases mismatches undecided realistic-cases realistic-undecided".  Build: g++ -O2 -ffp-contract=off.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../droplet_visual_odometry_amd/csrc/sampson.h"

using dvo::SampsonF32;
using dvo::sampson_inlier;

static void essential(std::mt19937_64& g, double E[9], double R[9], double t[3]) {
    std::normal_distribution<double> N(0, 1);
    std::uniform_real_distribution<double> U(0.01, 0.5);
    double a[3] = {N(g), N(g), N(g)};
    double n = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]), th = U(g);
    for (double& v : a) v /= n;
    const double c = std::cos(th), s = std::sin(th), C = 1 - c;
    const double Rm[9] = {c + a[0] * a[0] * C, a[0] * a[1] * C - a[2] * s, a[0] * a[2] * C + a[1] * s,
                          a[1] * a[0] * C + a[2] * s, c + a[1] * a[1] * C, a[1] * a[2] * C - a[0] * s,
                          a[2] * a[0] * C - a[1] * s, a[2] * a[1] * C + a[0] * s, c + a[2] * a[2] * C};
    double tv[3] = {N(g), N(g), N(g)};
    n = std::sqrt(tv[0] * tv[0] + tv[1] * tv[1] + tv[2] * tv[2]);
    for (double& v : tv) v /= n;
    const double T[9] = {0, -tv[2], tv[1], tv[2], 0, -tv[0], -tv[1], tv[0], 0};
    double f = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double v = 0;
            for (int k = 0; k < 3; ++k) v += T[3 * i + k] * Rm[3 * k + j];
            E[3 * i + j] = v;
            f += v * v;
        }
    for (int k = 0; k < 9; ++k) E[k] /= std::sqrt(f);
    for (int k = 0; k < 9; ++k) R[k] = Rm[k];
    for (int k = 0; k < 3; ++k) t[k] = tv[k];
}

static double sampson_err(const double E[9], const double q[4]) {
    const double ex0 = E[0] * q[0] + E[1] * q[1] + E[2], ex1 = E[3] * q[0] + E[4] * q[1] + E[5];
    const double ex2 = E[6] * q[0] + E[7] * q[1] + E[8];
    const double et0 = E[0] * q[2] + E[3] * q[3] + E[6], et1 = E[1] * q[2] + E[4] * q[3] + E[7];
    const double r = q[2] * ex0 + q[3] * ex1 + ex2;
    return r * r / (ex0 * ex0 + ex1 * ex1 + et0 * et0 + et1 * et1);
}

int main(int argc, char** argv) {
    const long models = argc > 1 ? atol(argv[1]) : 200;
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> U(0, 1);
    std::normal_distribution<double> N(0, 1);
    const float t = (float)((1.0 / 700.0) * (1.0 / 700.0));
    long cases = 0, bad = 0, und = 0, real_cases = 0, real_und = 0;
    auto check = [&](const double E[9], const double q[4], float tt) -> int {
        const SampsonF32 sf(E, tt >= FLT_MIN);
        const int d = sf.decide((float)q[0], (float)q[1], (float)q[2], (float)q[3], tt);
        const bool ex = sampson_inlier(E, q[0], q[1], q[2], q[3], tt, tt >= FLT_MIN);
        ++cases;
        if (d < 0) ++und;
        else if ((d == 1) != ex) {
            if (bad < 10)
                fprintf(stderr, "mismatch: E0 %.17g q %.17g %.17g %.17g %.17g t %.9g dec %d exact %d\n", E[0], q[0], q[1],
                        q[2], q[3], tt, d, (int)ex);
            ++bad;
        }
        return d;
    };
    for (long mi = 0; mi < models; ++mi) {
        double E[9], R[9], tv[3];
        essential(g, E, R, tv);
        for (int i = 0; i < 2000; ++i) {
            // a scene point seen by both cameras, with pixel noise, or an arbitrary pairing
            double q[4];
            const double X[3] = {-3 + 6 * U(g), -2 + 4 * U(g), 2 + 8 * U(g)};
            q[0] = X[0] / X[2];
            q[1] = X[1] / X[2];
            double Y[3];
            for (int k = 0; k < 3; ++k) Y[k] = R[3 * k] * X[0] + R[3 * k + 1] * X[1] + R[3 * k + 2] * X[2] + tv[k];
            q[2] = Y[0] / Y[2] + 0.002 * N(g);
            q[3] = Y[1] / Y[2] + 0.002 * N(g);
            if (i % 3 == 0)
                for (double& v : q) v = -1.2 + 2.4 * U(g);
            ++real_cases;
            real_und += check(E, q, t) < 0;
            // the same point moved along its epipolar line's normal to err = t (1 + rel)
            const double l0 = E[0] * q[0] + E[1] * q[1] + E[2], l1 = E[3] * q[0] + E[4] * q[1] + E[5];
            const double l2 = E[6] * q[0] + E[7] * q[1] + E[8], ln = std::sqrt(l0 * l0 + l1 * l1);
            const double n0 = l0 / ln, n1 = l1 / ln, off = (l0 * q[2] + l1 * q[3] + l2) / ln;
            const double b0 = q[2] - off * n0, b1 = q[3] - off * n1;  // on the line
            const double mag = std::pow(10.0, -12 + 11 * U(g)) * (U(g) < 0.5 ? -1 : 1);
            double dd = std::sqrt((double)t);
            for (int it = 0; it < 8; ++it) {
                double p[4] = {q[0], q[1], b0 + dd * n0, b1 + dd * n1};
                const double err = sampson_err(E, p);
                if (!(err > 0)) break;
                dd *= std::sqrt((double)t * (1 + mag) / err);
            }
            double p[4] = {q[0], q[1], b0 + dd * n0, b1 + dd * n1};
            check(E, p, t);
        }
        // extreme scales and exact zeros
        if (mi % 10 == 0) {
            const double sc[6][2] = {{1e-20, 1}, {1e20, 1}, {1, 1e-20}, {1, 1e12}, {1e-3, 1e3}, {0, 1}};
            for (auto& s : sc)
                for (int i = 0; i < 200; ++i) {
                    double Es[9], q[4] = {N(g), N(g), N(g), N(g)};
                    for (int k = 0; k < 9; ++k) Es[k] = E[k] * s[0];
                    for (double& v : q) v *= s[1];
                    if (i % 17 == 0) Es[2] = Es[5] = 0;
                    check(Es, q, t);
                    check(Es, q, 1e-12f);
                    check(Es, q, 0.5f);
                }
        }
    }
    printf("%ld %ld %ld %ld %ld\n", cases, bad, und, real_cases, real_und);
    return bad != 0;
}
