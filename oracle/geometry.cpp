// TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of the two-view
// geometry the reference calls in get_transformation_between_two_frames
// (scripts/visual_odometry_v3.py:293-345):
//   cv.findEssentialMat(p_prev, p_cur, K, RANSAC, 0.999, 1.0)   v3:297-300
//   cv.recoverPose(E, p_prev, p_cur, K)                          v3:303-306
//   cv.triangulatePoints(P_prev, P_cur, c_prev.T, c_cur.T)       v3:265
// following OpenCV 4.x calib3d five-point.cpp (EMEstimatorCallback,
// findEssentialMat, decomposeEssentialMat, recoverPose), ptsetreg.cpp
// (RANSACPointSetRegistrator, RANSACUpdateNumIters), triangulate.cpp
// (icvTriangulatePoints), core lapack.cpp (JacobiSVDImpl_, LUImpl) and
// mathfuncs.cpp (solvePoly, solveCubic), core RNG (multiply-with-carry).
//
// Restatement choices where OpenCV's exact source is not available here
// (documented in DESIGN.md §3): sums are evaluated sequentially in index order,
// no FMA contraction; hypot(a,b) = max*sqrt(1+(min/max)^2); the 10x20 Nister
// coefficient matrix is formed by explicit polynomial products (rows: the nine
// entries of 2EE^T E - tr(EE^T)E row-major, then det E; columns in Nister's
// monomial order, which OpenCV's B-matrix construction requires).
#include "oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Rng {  // cv::RNG
    uint64_t state;
    explicit Rng(uint64_t s) : state(s ? s : 0xffffffffULL) {}
    unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

double dvo_hypot(double a, double b) {
    a = std::fabs(a);
    b = std::fabs(b);
    if (a < b) std::swap(a, b);
    if (a == 0) return b;
    double r = b / a;
    return a * std::sqrt(1.0 + r * r);
}

// lapack.cpp JacobiSVDImpl_<double>(At, astep, W, Vt, vstep, m, n, n1, DBL_MIN, DBL_EPSILON*10).
// At: n rows (plus n1-n completion rows) of length m, row stride m.  Vt: n x n.
void jacobi_svd(double* At, double* _W, double* Vt, int m, int n, int n1) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    std::vector<double> W(n);
    int max_iter = std::max(m, 30);
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) {
            double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; ++k) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; ++iter) {
        bool changed = false;
        for (int i = 0; i < n - 1; ++i)
            for (int j = i + 1; j < n; ++j) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; ++k) p += Ai[k] * Aj[k];
                if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = dvo_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = std::sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = std::sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; ++k) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                double *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (int k = 0; k < n; ++k) {
                    double t0 = c * Vi[k] + s * Vj[k];
                    double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) {
            double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = std::sqrt(sd);
    }
    for (int i = 0; i < n - 1; ++i) {
        int j = i;
        for (int k = i + 1; k < n; ++k)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            std::swap(W[i], W[j]);
            for (int k = 0; k < m; ++k) std::swap(At[i * m + k], At[j * m + k]);
            for (int k = 0; k < n; ++k) std::swap(Vt[i * n + k], Vt[j * n + k]);
        }
    }
    for (int i = 0; i < n; ++i) _W[i] = W[i];
    Rng rng(0x12345678);
    for (int i = 0; i < n1; ++i) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; ++k) At[i * m + k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; ++k) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (int k = 0; k < m; ++k) {
                        double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += std::fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; ++k) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; ++k) {
                double t = At[i * m + k];
                sd += t * t;
            }
            sd = std::sqrt(sd);
        }
        double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; ++k) At[i * m + k] *= s;
    }
}

// lapack.cpp LUImpl<double>(A, m, b, n, DBL_EPSILON*100); returns 0 if singular.
int lu_solve(double* A, int m, double* b, int n) {
    const double eps = DBL_EPSILON * 100;
    int p = 1;
    for (int i = 0; i < m; i++) {
        int k = i;
        for (int j = i + 1; j < m; j++)
            if (std::fabs(A[j * m + i]) > std::fabs(A[k * m + i])) k = j;
        if (std::fabs(A[k * m + i]) < eps) return 0;
        if (k != i) {
            for (int j = i; j < m; j++) std::swap(A[i * m + j], A[k * m + j]);
            for (int j = 0; j < n; j++) std::swap(b[i * n + j], b[k * n + j]);
            p = -p;
        }
        double d = -1 / A[i * m + i];
        for (int j = i + 1; j < m; j++) {
            double alpha = A[j * m + i] * d;
            for (int c = i + 1; c < m; c++) A[j * m + c] += alpha * A[i * m + c];
            for (int c = 0; c < n; c++) b[j * n + c] += alpha * b[i * n + c];
        }
    }
    for (int i = m - 1; i >= 0; i--)
        for (int j = 0; j < n; j++) {
            double s = b[i * n + j];
            for (int k = i + 1; k < m; k++) s -= A[i * m + k] * b[k * n + j];
            b[i * n + j] = s / A[i * m + i];
        }
    return p;
}

struct Cx {
    double re, im;
};
inline Cx cmul(Cx a, Cx b) { return Cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
inline Cx cadd(Cx a, Cx b) { return Cx{a.re + b.re, a.im + b.im}; }
inline Cx csub(Cx a, Cx b) { return Cx{a.re - b.re, a.im - b.im}; }
inline Cx cdiv(Cx a, Cx b) {
    double t = 1. / (b.re * b.re + b.im * b.im);
    return Cx{(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
}
inline double cabs(Cx a) { return std::sqrt(a.re * a.re + a.im * a.im); }

// mathfuncs.cpp solveCubic, coefficients in descending order; returns x0.
int solve_cubic(const double* c, double* x) {
    double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3];
    double x0 = 0, x1 = 0, x2 = 0;
    int n;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0) n = a3 == 0 ? -1 : 0;
            else { x0 = -a3 / a2; n = 1; }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = std::sqrt(d);
                double q1 = (-a2 + d) * 0.5, q2 = (a2 + d) * -0.5;
                if (std::fabs(q1) > std::fabs(q2)) { x0 = q1 / a1; x1 = a3 / q1; }
                else { x0 = q2 / a1; x1 = a3 / q2; }
                n = d > 0 ? 2 : 1;
            } else n = 0;
        }
    } else {
        a0 = 1. / a0;
        a1 *= a0;
        a2 *= a0;
        a3 *= a0;
        double Q = (a1 * a1 - 3 * a2) * (1. / 9);
        double R = (2 * a1 * a1 * a1 - 9 * a1 * a2 + 27 * a3) * (1. / 54);
        double Qcubed = Q * Q * Q;
        double d = Qcubed - R * R;
        if (d > 0) {
            double theta = std::acos(R / std::sqrt(Qcubed));
            double sqrtQ = std::sqrt(Q);
            double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = a1 * (1. / 3);
            x0 = t0 * std::cos(t1) - t2;
            x1 = t0 * std::cos(t1 + (2. * M_PI / 3)) - t2;
            x2 = t0 * std::cos(t1 + (4. * M_PI / 3)) - t2;
            n = 3;
        } else if (d == 0) {
            if (R >= 0) { x0 = -2 * std::pow(R, 1. / 3) - a1 / 3; x1 = std::pow(R, 1. / 3) - a1 / 3; }
            else { x0 = 2 * std::pow(-R, 1. / 3) - a1 / 3; x1 = -std::pow(-R, 1. / 3) - a1 / 3; }
            x2 = 0;
            n = x0 == x1 ? 1 : 2;
            x1 = x0 == x1 ? 0 : x1;
        } else {
            d = std::sqrt(-d);
            double e = std::pow(d + std::fabs(R), 1. / 3);
            if (R > 0) e = -e;
            x0 = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    x[0] = x0; x[1] = x1; x[2] = x2;
    return n;
}

// mathfuncs.cpp solvePoly (Durand-Kerner, Gauss-Seidel order).  coeffs[0..n0]
// ascending.  Returns the working degree n; roots beyond it are not reported
// (OpenCV leaves them as uninitialised buffer contents).
// trace (analysis only, tools/dk_cycle_stats.py): a 64-bit hash of the roots' bits after each
// sweep, trace[max_iters] = the sweeps run (the maxDiff <= 0 exit or max_iters).
int solve_poly(const double* rc, int n0, int max_iters, Cx* roots, uint64_t* trace = nullptr) {
    std::vector<Cx> coeffs(n0 + 1);
    for (int i = 0; i <= n0; i++) coeffs[i] = Cx{rc[i], 0};
    int n = n0;
    for (; n > 1; n--)
        if (std::fabs(coeffs[n].re) + std::fabs(coeffs[n].im) > DBL_EPSILON) break;
    Cx p{1, 0}, r{1, 1};
    for (int i = 0; i < n; i++) {
        roots[i] = p;
        p = cmul(p, r);
    }
    max_iters = max_iters <= 0 ? 1000 : max_iters;
    for (int iter = 0; iter < max_iters; iter++) {
        double maxDiff = 0;
        for (int i = 0; i < n; i++) {
            p = roots[i];
            Cx num = coeffs[n], denom = coeffs[n];
            int num_same_root = 1;
            for (int j = 0; j < n; j++) {
                num = cadd(cmul(num, p), coeffs[n - j - 1]);
                if (j != i) {
                    Cx d = csub(p, roots[j]);
                    if (d.re == 0 && d.im == 0) num_same_root++;
                    else denom = cmul(denom, d);
                }
            }
            num = cdiv(num, denom);
            if (num_same_root > 1) {
                double ore = num.re, oim = num.im;
                int sq_times = num_same_root % 2 == 0 ? num_same_root / 2 : num_same_root / 2 - 1;
                for (int j = 0; j < sq_times; j++) {
                    num.re = ore * ore + oim * oim;
                    num.re = std::sqrt(num.re);
                    num.re += ore;
                    num.im = num.re - ore;
                    num.re /= 2;
                    num.re = std::sqrt(num.re);
                    num.im /= 2;
                    num.im = std::sqrt(num.im);
                    if (ore < 0) num.im = -num.im;
                }
                if (num_same_root % 2 != 0) {
                    double cc[4], cr[3];
                    cc[3] = -(std::pow(ore, 3));
                    cc[2] = -(15 * std::pow(ore, 2) + 27 * std::pow(oim, 2));
                    cc[1] = -48 * ore;
                    cc[0] = 64;
                    solve_cubic(cc, cr);
                    if (cr[0] >= 0) num.re = std::pow(cr[0], 1. / 3);
                    else num.re = -std::pow(-cr[0], 1. / 3);
                    num.im = std::sqrt(std::pow(num.re, 2) / 3 - ore / (3 * num.re));
                }
            }
            roots[i] = csub(p, num);
            maxDiff = std::max(maxDiff, cabs(num));
        }
        if (trace) {
            uint64_t hsh = 1469598103934665603ull;
            for (int i = 0; i < n; i++) {
                uint64_t a, b;
                std::memcpy(&a, &roots[i].re, 8);
                std::memcpy(&b, &roots[i].im, 8);
                hsh = (hsh ^ a) * 1099511628211ull;
                hsh = (hsh ^ b) * 1099511628211ull;
            }
            trace[iter] = hsh;
            trace[max_iters] = (uint64_t)(iter + 1);
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; i++)
        if (std::fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    return n;
}

// ---- Nister coefficient matrix by explicit polynomial products -------------
// Cubic monomials (x,y,z exponents), Nister / OpenCV column order.
const int CEXP[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                         {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                         {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
const int QEXP[10][3] = {{2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {1, 0, 0}, {0, 2, 0},
                         {0, 1, 1}, {0, 1, 0}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
const int LEXP[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};

struct PolyTables {
    int ll2q[4][4];
    int ql2c[10][4];
    PolyTables() {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int q = 0; q < 10; ++q)
                    if (QEXP[q][0] == LEXP[i][0] + LEXP[j][0] && QEXP[q][1] == LEXP[i][1] + LEXP[j][1] &&
                        QEXP[q][2] == LEXP[i][2] + LEXP[j][2])
                        ll2q[i][j] = q;
        for (int i = 0; i < 10; ++i)
            for (int j = 0; j < 4; ++j)
                for (int c = 0; c < 20; ++c)
                    if (CEXP[c][0] == QEXP[i][0] + LEXP[j][0] && CEXP[c][1] == QEXP[i][1] + LEXP[j][1] &&
                        CEXP[c][2] == QEXP[i][2] + LEXP[j][2])
                        ql2c[i][j] = c;
    }
};
const PolyTables PT;

void mul_ll(const double* a, const double* b, double* q) {
    for (int k = 0; k < 10; ++k) q[k] = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) q[PT.ll2q[i][j]] += a[i] * b[j];
}
void mul_ql(const double* q, const double* l, double* c) {
    for (int k = 0; k < 20; ++k) c[k] = 0;
    for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 4; ++j) c[PT.ql2c[i][j]] += q[i] * l[j];
}

void coeff_matrix(const double* X, const double* Y, const double* Z, const double* Wv, double* A /*10x20*/) {
    double E[9][4];
    for (int e = 0; e < 9; ++e) {
        E[e][0] = X[e];
        E[e][1] = Y[e];
        E[e][2] = Z[e];
        E[e][3] = Wv[e];
    }
    double EEt[9][10], t1[10], t2[10];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double* o = EEt[i * 3 + j];
            mul_ll(E[i * 3 + 0], E[j * 3 + 0], o);
            mul_ll(E[i * 3 + 1], E[j * 3 + 1], t1);
            for (int k = 0; k < 10; ++k) o[k] = o[k] + t1[k];
            mul_ll(E[i * 3 + 2], E[j * 3 + 2], t1);
            for (int k = 0; k < 10; ++k) o[k] = o[k] + t1[k];
        }
    double tr[10];
    for (int k = 0; k < 10; ++k) tr[k] = (EEt[0][k] + EEt[4][k]) + EEt[8][k];
    double c1[20], c2[20];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double* row = A + (i * 3 + j) * 20;
            mul_ql(EEt[i * 3 + 0], E[0 * 3 + j], row);
            mul_ql(EEt[i * 3 + 1], E[1 * 3 + j], c1);
            for (int k = 0; k < 20; ++k) row[k] = row[k] + c1[k];
            mul_ql(EEt[i * 3 + 2], E[2 * 3 + j], c1);
            for (int k = 0; k < 20; ++k) row[k] = row[k] + c1[k];
            mul_ql(tr, E[i * 3 + j], c1);
            for (int k = 0; k < 20; ++k) row[k] = 2.0 * row[k] - c1[k];
        }
    // det(E) = e00(e11e22 - e12e21) - e01(e10e22 - e12e20) + e02(e10e21 - e11e20)
    double* row = A + 9 * 20;
    mul_ll(E[4], E[8], t1);
    mul_ll(E[5], E[7], t2);
    for (int k = 0; k < 10; ++k) t1[k] = t1[k] - t2[k];
    mul_ql(t1, E[0], row);
    mul_ll(E[3], E[8], t1);
    mul_ll(E[5], E[6], t2);
    for (int k = 0; k < 10; ++k) t1[k] = t1[k] - t2[k];
    mul_ql(t1, E[1], c1);
    mul_ll(E[3], E[7], t1);
    mul_ll(E[4], E[6], t2);
    for (int k = 0; k < 10; ++k) t1[k] = t1[k] - t2[k];
    mul_ql(t1, E[2], c2);
    for (int k = 0; k < 20; ++k) row[k] = (row[k] - c1[k]) + c2[k];
}

void poly_mul(const double* a, int na, const double* b, int nb, double* r) {  // ascending coeffs
    for (int k = 0; k < na + nb - 1; ++k) r[k] = 0;
    for (int i = 0; i < na; ++i)
        for (int j = 0; j < nb; ++j) r[i + j] += a[i] * b[j];
}

// five-point.cpp EMEstimatorCallback::runKernel on 5 normalised correspondences.
thread_local double t_last_poly[11];  // the last five_point's degree-10 polynomial (analysis hook)

int five_point(const double* q1, const double* q2, double* models) {
    // Q (5x9), then SVD::compute(Q, W, U, Vt, MODIFY_A | FULL_UV): m<n so the
    // 5 rows are orthogonalised as At (m=9, n=5) and completed to 9 rows;
    // Vt(9x9) = that completed At, rows 5..8 span the null space.
    double At[9 * 9], W[5], Vt5[25];
    std::memset(At, 0, sizeof(At));
    for (int i = 0; i < 5; ++i) {
        double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double* r = At + i * 9;
        r[0] = x1 * x2;
        r[1] = y1 * x2;
        r[2] = x2 + 0.0;  // Q.col(2) = Q2.col(0) * 1.0  -> add(x, 0)
        r[3] = x1 * y2;
        r[4] = y1 * y2;
        r[5] = y2 + 0.0;
        r[6] = x1 + 0.0;
        r[7] = y1 + 0.0;
        r[8] = 1.0;
    }
    jacobi_svd(At, W, Vt5, 9, 5, 9);
    // EE = Vt.t().colRange(5, 9) * 1.0  -> add(x, 0)
    double EE[4][9];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 9; ++k) EE[r][k] = At[(5 + r) * 9 + k] + 0.0;
    const double *X = EE[0], *Y = EE[1], *Z = EE[2], *Wv = EE[3];
    double A[10 * 20];
    coeff_matrix(X, Y, Z, Wv, A);
    // A = A.colRange(0,10).inv() * A.colRange(10,20): OpenCV's MatExpr turns
    // inv(A1) * A2 into solve(A1, A2, DECOMP_LU) (MatOp_Invert::matmul).
    double L[100], G[100];
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 10; ++c) {
            L[r * 10 + c] = A[r * 20 + c];
            G[r * 10 + c] = A[r * 20 + 10 + c];
        }
    if (!lu_solve(L, 10, G, 10))
        for (int k = 0; k < 100; ++k) G[k] = 0;
    double b[3 * 13];
    for (int i = 0; i < 3; ++i) {
        const double* a1 = G + (i * 2 + 4) * 10;
        const double* a2 = G + (i * 2 + 5) * 10;
        // arow = A.row(.) * 1.0 and row.colRange(.) = arow.colRange(.) * 1.0: two add(x, 0)
        double row1[13] = {0}, row2[13] = {0};
        for (int k = 0; k < 3; ++k) row1[1 + k] = (a1[k] + 0.0) + 0.0;
        for (int k = 0; k < 3; ++k) row1[5 + k] = (a1[3 + k] + 0.0) + 0.0;
        for (int k = 0; k < 4; ++k) row1[9 + k] = (a1[6 + k] + 0.0) + 0.0;
        for (int k = 0; k < 3; ++k) row2[0 + k] = (a2[k] + 0.0) + 0.0;
        for (int k = 0; k < 3; ++k) row2[4 + k] = (a2[3 + k] + 0.0) + 0.0;
        for (int k = 0; k < 4; ++k) row2[8 + k] = (a2[6 + k] + 0.0) + 0.0;
        for (int k = 0; k < 13; ++k) b[i * 13 + k] = row1[k] - row2[k];
    }
    // c = det of the 3x3 polynomial matrix [px py pc] (ascending powers of z).
    double px[3][4], py[3][4], pc[3][5];
    for (int j = 0; j < 3; ++j) {
        const double* br = b + j * 13;
        for (int k = 0; k < 4; ++k) px[j][k] = br[3 - k];
        for (int k = 0; k < 4; ++k) py[j][k] = br[7 - k];
        for (int k = 0; k < 5; ++k) pc[j][k] = br[12 - k];
    }
    double u[8], v[8], m1[8], m2[8], m3[8], t1[11], t2[11], t3[11], c[11];
    poly_mul(py[1], 4, pc[2], 5, u);
    poly_mul(pc[1], 5, py[2], 4, v);
    for (int k = 0; k < 8; ++k) m1[k] = u[k] - v[k];
    poly_mul(px[1], 4, pc[2], 5, u);
    poly_mul(pc[1], 5, px[2], 4, v);
    for (int k = 0; k < 8; ++k) m2[k] = u[k] - v[k];
    poly_mul(px[1], 4, py[2], 4, u);
    poly_mul(py[1], 4, px[2], 4, v);
    for (int k = 0; k < 7; ++k) m3[k] = u[k] - v[k];
    poly_mul(px[0], 4, m1, 8, t1);
    poly_mul(py[0], 4, m2, 8, t2);
    poly_mul(pc[0], 5, m3, 7, t3);
    for (int k = 0; k < 11; ++k) c[k] = (t1[k] - t2[k]) + t3[k];

    std::memcpy(t_last_poly, c, sizeof(t_last_poly));
    Cx roots[10];
    int nr = solve_poly(c, 10, 300, roots);
    int count = 0;
    for (int i = 0; i < nr; ++i) {
        if (std::fabs(roots[i].im) > 1e-10) continue;
        double z1 = roots[i].re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double bz[9];
        for (int j = 0; j < 3; ++j) {
            const double* br = b + j * 13;
            bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        // SVD::solveZ(Bz): At = Bz^T, last row of Vt.
        double at3[9], w3[3], vt3[9];
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) at3[r * 3 + k] = bz[k * 3 + r];
        jacobi_svd(at3, w3, vt3, 3, 3, 0);
        const double* xy1 = vt3 + 6;
        if (std::fabs(xy1[2]) < 1e-10) continue;
        double xs = xy1[0] / xy1[2], ys = xy1[1] / xy1[2];
        double* e = models + count * 9;
        // addWeighted(X, xs, Y, ys, 0) -> scaleAdd(Z, zs, .) -> add(., W)
        for (int k = 0; k < 9; ++k) e[k] = (((X[k] * xs + Y[k] * ys) + 0.0) + Z[k] * z1) + Wv[k];
        // norm(Evec): normL2Sqr unrolled by 4, then sqrt; Evec /= n -> *= 1/n
        double s = 0;
        int k = 0;
        for (; k <= 9 - 4; k += 4) s += e[k] * e[k] + e[k + 1] * e[k + 1] + e[k + 2] * e[k + 2] + e[k + 3] * e[k + 3];
        for (; k < 9; ++k) s += e[k] * e[k];
        double inv_n = 1. / std::sqrt(s);
        for (k = 0; k < 9; ++k) e[k] = e[k] * inv_n + 0.0;  // convertTo(alpha = 1/n, beta = 0)
        count++;
    }
    return count;
}

// EMEstimatorCallback::computeError + RANSACPointSetRegistrator::findInliers
inline float sampson_err(const double* E, double x1, double y1, double x2, double y2) {
    double ex0 = E[0] * x1 + E[1] * y1 + E[2] * 1.;
    double ex1 = E[3] * x1 + E[4] * y1 + E[5] * 1.;
    double ex2 = E[6] * x1 + E[7] * y1 + E[8] * 1.;
    double et0 = E[0] * x2 + E[3] * y2 + E[6] * 1.;
    double et1 = E[1] * x2 + E[4] * y2 + E[7] * 1.;
    double x2tEx1 = x2 * ex0 + y2 * ex1 + 1. * ex2;
    double a = ex0 * ex0, b = ex1 * ex1, c = et0 * et0, d = et1 * et1;
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

int find_inliers(const double* E, const double* n1, const double* n2, int m, float t, uint8_t* mask) {
    int nz = 0;
    for (int i = 0; i < m; ++i) {
        float err = sampson_err(E, n1[2 * i], n1[2 * i + 1], n2[2 * i], n2[2 * i + 1]);
        int f = err <= t;
        if (mask) mask[i] = (uint8_t)f;
        nz += f;
    }
    return nz;
}

int ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = std::max(p, 0.);
    p = std::min(p, 1.);
    ep = std::max(ep, 0.);
    ep = std::min(ep, 1.);
    double num = std::max(1. - p, DBL_MIN);
    double denom = 1. - std::pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

void normalize_points(const double* p, int m, const double* K, double* out) {
    // findEssentialMat / recoverPose: col = (col - c) / f evaluated by OpenCV's
    // MatExpr as col * (1/f) + (-c * (1/f)).
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double ax = 1. / fx, ay = 1. / fy, bx = -cx * ax, by = -cy * ay;
    for (int i = 0; i < m; ++i) {
        out[2 * i] = p[2 * i] * ax + bx;
        out[2 * i + 1] = p[2 * i + 1] * ay + by;
    }
}

// triangulate.cpp icvTriangulatePoints for one correspondence.
void triangulate_one(const double* P1, const double* P2, double x1, double y1, double x2, double y2, double* X) {
    double A[16];
    for (int k = 0; k < 4; ++k) {
        A[0 * 4 + k] = x1 * P1[2 * 4 + k] - P1[0 * 4 + k];
        A[1 * 4 + k] = y1 * P1[2 * 4 + k] - P1[1 * 4 + k];
        A[2 * 4 + k] = x2 * P2[2 * 4 + k] - P2[0 * 4 + k];
        A[3 * 4 + k] = y2 * P2[2 * 4 + k] - P2[1 * 4 + k];
    }
    double At[16], W[4], Vt[16];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) At[r * 4 + k] = A[k * 4 + r];
    jacobi_svd(At, W, Vt, 4, 4, 0);
    for (int k = 0; k < 4; ++k) X[k] = Vt[12 + k];
}

double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

void matmul3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
}

}  // namespace

extern "C" {

int ora_jacobi_svd(double* At, int m, int n, int n1, double* W, double* Vt) {
    jacobi_svd(At, W, Vt, m, n, n1);
    return 0;
}

int ora_solve_poly(const double* coeffs, int n, int max_iters, double* roots) {
    std::vector<Cx> r(n);
    int nr = solve_poly(coeffs, n, max_iters, r.data());
    for (int i = 0; i < nr; ++i) {
        roots[2 * i] = r[i].re;
        roots[2 * i + 1] = r[i].im;
    }
    return nr;
}

int ora_ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    return ransac_update_num_iters(p, ep, model_points, max_iters);
}

int ora_five_point(const double* p1, const double* p2, double* models, int* n) {
    *n = five_point(p1, p2, models);
    return 0;
}

int ora_last_five_point_poly(double* c) {
    std::memcpy(c, t_last_poly, sizeof(t_last_poly));
    return 0;
}

int ora_solve_poly_trace(const double* coeffs, int n, int max_iters, uint64_t* trace) {
    std::vector<Cx> r(n);
    return solve_poly(coeffs, n, max_iters, r.data(), trace);
}

int ora_find_essential(const double* p1, const double* p2, int m, const double* K, double prob, double threshold,
                       int max_iters, double* E_out, int* rows, uint8_t* mask, int* iters_run) {
    *rows = 0;
    *iters_run = 0;
    const int model_points = 5;
    if (m < model_points) return -1;
    std::vector<double> n1(2 * m), n2(2 * m);
    normalize_points(p1, m, K, n1.data());
    normalize_points(p2, m, K, n2.data());
    double thr = threshold / ((K[0] + K[4]) / 2);
    if (m == model_points) {
        int k = five_point(n1.data(), n2.data(), E_out);
        if (k <= 0) return -2;
        *rows = 3 * k;
        if (mask) std::memset(mask, 1, m);
        return 0;
    }
    Rng rng((uint64_t)(int64_t)-1);
    int niters = std::max(max_iters, 1), max_good = 0;
    double best[9];
    std::vector<uint8_t> cur(m), bestmask(m, 0);
    const float t = (float)(thr * thr);
    double models[90], s1[10], s2[10];
    int iter;
    for (iter = 0; iter < niters; iter++) {
        int idx[5];
        for (int i = 0; i < model_points; ++i) {
            int idx_i;
            for (;;) {
                idx_i = idx[i] = rng.uniform(0, m);
                int j;
                for (j = 0; j < i; j++)
                    if (idx_i == idx[j]) break;
                if (j == i) break;
            }
            s1[2 * i] = n1[2 * idx_i];
            s1[2 * i + 1] = n1[2 * idx_i + 1];
            s2[2 * i] = n2[2 * idx_i];
            s2[2 * i + 1] = n2[2 * idx_i + 1];
        }
        int nmodels = five_point(s1, s2, models);
        if (nmodels <= 0) continue;
        for (int i = 0; i < nmodels; ++i) {
            int good = find_inliers(models + 9 * i, n1.data(), n2.data(), m, t, cur.data());
            if (good > std::max(max_good, model_points - 1)) {
                std::swap(cur, bestmask);
                std::memcpy(best, models + 9 * i, sizeof(best));
                max_good = good;
                niters = ransac_update_num_iters(prob, (double)(m - good) / m, model_points, niters);
            }
        }
    }
    *iters_run = iter;
    if (max_good <= 0) return -3;
    std::memcpy(E_out, best, sizeof(best));
    *rows = 3;
    if (mask) std::memcpy(mask, bestmask.data(), m);
    return 0;
}

// The subsets ora_find_essential draws: getSubset (ptsetreg.cpp) with
// cv::RNG((uint64)-1), n hypotheses of 5 distinct indices in [0, m).
int ora_ransac_subsets(int m, int n, int32_t* idx) {
    if (m < 6 || n < 0) return -1;
    Rng rng((uint64_t)(int64_t)-1);
    for (int h = 0; h < n; ++h)
        for (int i = 0; i < 5; ++i) {
            for (;;) {
                const int v = rng.uniform(0, m);
                int j;
                for (j = 0; j < i; ++j)
                    if (v == idx[h * 5 + j]) break;
                idx[h * 5 + i] = v;
                if (j == i) break;
            }
        }
    return 0;
}

// The bookkeeping of RANSACPointSetRegistrator::run (the loop of
// ora_find_essential) over given per-hypothesis model inlier counts:
// out = {iterations run, final niters, max good, best hypothesis, best model}.
int ora_ransac_replay(const int32_t* nmod, const int32_t* cnt, int n, int m, double prob, int max_iters, int32_t* out) {
    int niters = std::max(max_iters, 1), max_good = 0, best_h = -1, best_i = -1, iter;
    for (iter = 0; iter < niters && iter < n; iter++)
        for (int i = 0; i < nmod[iter]; ++i) {
            const int good = cnt[iter * 10 + i];
            if (good > std::max(max_good, 4)) {
                max_good = good;
                best_h = iter;
                best_i = i;
                niters = ransac_update_num_iters(prob, (double)(m - good) / m, 5, niters);
            }
        }
    out[0] = iter;
    out[1] = niters;
    out[2] = max_good;
    out[3] = best_h;
    out[4] = best_i;
    return 0;
}

int ora_recover_pose(const double* E, const double* p1, const double* p2, int m, const double* K, double dist_thresh,
                     const uint8_t* mask_in, double* R, double* t, uint8_t* mask_out, int* good_out) {
    std::vector<double> n1(2 * m), n2(2 * m);
    normalize_points(p1, m, K, n1.data());
    normalize_points(p2, m, K, n2.data());
    // decomposeEssentialMat: SVD::compute(E) (At = E^T), U = At^T, Vt.
    double At[9], W[3], Vt[9], U[9];
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) At[r * 3 + k] = E[k * 3 + r];
    jacobi_svd(At, W, Vt, 3, 3, 3);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) U[r * 3 + c] = At[c * 3 + r];
    if (det3(U) < 0)
        for (int k = 0; k < 9; ++k) U[k] *= -1.;
    if (det3(Vt) < 0)
        for (int k = 0; k < 9; ++k) Vt[k] *= -1.;
    const double Wm[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double UW[9], R1[9], R2[9], tv[3];
    matmul3(U, Wm, UW);
    matmul3(UW, Vt, R1);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, R2);
    for (int k = 0; k < 3; ++k) tv[k] = U[k * 3 + 2] + 0.0;  // t = U.col(2) * 1.0
    const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    double P[4][12];
    const double* Rs[4] = {R1, R2, R1, R2};
    for (int c = 0; c < 4; ++c)  // P(:, 0:3) = R * 1.0; P.col(3) = t * 1.0 | -t * 1.0
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) P[c][r * 4 + k] = Rs[c][r * 3 + k] + 0.0;
            P[c][r * 4 + 3] = c < 2 ? tv[r] + 0.0 : 0.0 - tv[r];
        }
    int good[4] = {0, 0, 0, 0};
    std::vector<uint8_t> masks(4 * (size_t)m);
    for (int c = 0; c < 4; ++c) {
        for (int i = 0; i < m; ++i) {
            double X[4];
            triangulate_one(P0, P[c], n1[2 * i], n1[2 * i + 1], n2[2 * i], n2[2 * i + 1], X);
            bool ok = X[2] * X[3] > 0;
            double q0 = X[0] / X[3], q1 = X[1] / X[3], q2 = X[2] / X[3], q3 = X[3] / X[3];
            ok = (q2 < dist_thresh) && ok;
            const double* Pr = P[c] + 8;
            double z = Pr[0] * q0 + Pr[1] * q1 + Pr[2] * q2 + Pr[3] * q3;
            ok = (z > 0) && ok;
            ok = (z < dist_thresh) && ok;
            if (mask_in && !mask_in[i]) ok = false;
            masks[(size_t)c * m + i] = ok ? 255 : 0;
            good[c] += ok;
        }
    }
    int pick;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) pick = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) pick = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) pick = 2;
    else pick = 3;
    std::memcpy(R, Rs[pick], 9 * sizeof(double));
    for (int k = 0; k < 3; ++k) t[k] = pick < 2 ? tv[k] : 0.0 - tv[k];  // t = -t -> subtract(0, t)
    if (mask_out) std::memcpy(mask_out, &masks[(size_t)pick * m], m);
    *good_out = good[pick];
    return 0;
}

int ora_triangulate(const double* P1, const double* P2, const double* x1, const double* x2, int k, double* X) {
    for (int i = 0; i < k; ++i) {
        double out[4];
        triangulate_one(P1, P2, x1[i], x1[k + i], x2[i], x2[k + i], out);
        for (int r = 0; r < 4; ++r) X[r * k + i] = out[r];
    }
    return 0;
}

}  // extern "C"
