// Two-view geometry for gfx950: the MI355X replacement of
//   cv.findEssentialMat(p_prev, p_cur, K, RANSAC, 0.999, 1.0)   visual_odometry_v3.py:297-300
//   cv.recoverPose(E, p_prev, p_cur, K)                          visual_odometry_v3.py:303-306
//   cv.triangulatePoints(P_prev, P_cur, c_prev.T, c_cur.T)       visual_odometry_v3.py:265
//
// ransac_kernel: one workgroup (256 threads) per frame pair.  RANSAC is
// evaluated in rounds of up to kChunk iterations: thread 0 draws the round's
// 5-point samples from cv::RNG((uint64)-1) exactly as getSubset does; every
// thread then solves one sample with the 5-point kernel (Jacobi SVD + RNG
// null-space completion, Nister coefficient matrix, LU solve, 10th-degree
// polynomial, Durand-Kerner, per-root 3x3 SVD); the waves score all models'
// Sampson errors over every correspondence (ballot popcounts); thread 0 then
// replays RANSACPointSetRegistrator::run's sequential best/niters logic over
// the round in iteration order, stopping where OpenCV would.  The result is
// identical to the sequential loop; only iterations past OpenCV's stop are
// wasted.
// pose_decompose/count/pick kernels (recoverPose): per pair decomposition, then one thread per
// (point, decomposition); formerly: one workgroup per pair; thread 0 decomposes E, all
// threads triangulate (4 poses x M points, one 4x4 Jacobi SVD per item).
//
// Every double expression mirrors oracle/geometry.cpp operation for operation
// (compiled with -ffp-contract=off), so E, R and t are bit-identical to it.
#include "dvo_internal.h"
#include "sampson.h"

#include <cfloat>

namespace dvo {


struct Cx {
    double re, im;
};
__device__ __forceinline__ Cx cmul(Cx a, Cx b) { return Cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ Cx cadd(Cx a, Cx b) { return Cx{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ Cx csub(Cx a, Cx b) { return Cx{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ Cx cdiv(Cx a, Cx b) {
    double t = 1. / (b.re * b.re + b.im * b.im);
    return Cx{(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
}
__device__ __forceinline__ double cabs_(Cx a) { return sqrt(a.re * a.re + a.im * a.im); }

struct Rng {  // cv::RNG multiply-with-carry
    uint64_t state;
    __device__ unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

__device__ __forceinline__ double dvo_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a < b) {
        double t = a;
        a = b;
        b = t;
    }
    if (a == 0) return b;
    double r = b / a;
    return a * sqrt(1.0 + r * r);
}

// lapack.cpp JacobiSVDImpl_ (see oracle/geometry.cpp jacobi_svd); compile-time
// sizes keep every array in registers.  At has R >= max(N, N1) rows of M.
template <int M, int N, int N1, int R>
__device__ __forceinline__ void jacobi_svd(double (&At)[R][M], double (&Wout)[N], double (&Vt)[N][N]) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            double t = At[i][k];
            sd += t * t;
        }
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < N; ++k) Vt[i][k] = 0;
        Vt[i][i] = 1;
    }
    constexpr int max_iter = M > 30 ? M : 30;
    for (int iter = 0; iter < max_iter; ++iter) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; ++i)
#pragma unroll
            for (int j = i + 1; j < N; ++j) {
                double a = W[i], p = 0, b = W[j];
#pragma unroll
                for (int k = 0; k < M; ++k) p += At[i][k] * At[j][k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = dvo_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    double t0 = c * At[i][k] + s * At[j][k];
                    double t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = t0;
                    At[j][k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    double t0 = c * Vt[i][k] + s * Vt[j][k];
                    double t1 = -s * Vt[i][k] + c * Vt[j][k];
                    Vt[i][k] = t0;
                    Vt[j][k] = t1;
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            double t = At[i][k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < N - 1; ++i) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k)
            if (wj < W[k]) {
                j = k;
                wj = W[k];
            }
#pragma unroll
        for (int kk = i + 1; kk < N; ++kk)
            if (j == kk) {
                double t = W[i];
                W[i] = W[kk];
                W[kk] = t;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    double u = At[i][k];
                    At[i][k] = At[kk][k];
                    At[kk][k] = u;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    double u = Vt[i][k];
                    Vt[i][k] = Vt[kk][k];
                    Vt[kk][k] = u;
                }
            }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) Wout[i] = W[i];
    if (N1 == 0) return;
    Rng rng{0x12345678ull};
#pragma unroll
    for (int i = 0; i < N1; ++i) {
        double sd = i < N ? W[i < N ? i : 0] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / M;
#pragma unroll
            for (int k = 0; k < M; ++k) At[i][k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
#pragma unroll
                for (int j = 0; j < i; j++) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) sd += At[i][k] * At[j][k];
                    double asum = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) {
                        double t = At[i][k] - sd * At[j][k];
                        At[i][k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) At[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < M; ++k) {
                double t = At[i][k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        double s = sd > minval ? 1 / sd : 0.;
#pragma unroll
        for (int k = 0; k < M; ++k) At[i][k] *= s;
    }
}

// ---- Nister coefficient matrix (index tables = oracle PolyTables) ----------
// Monomial index maps (linear x linear -> quadratic, quadratic x linear ->
// cubic) as compile-time functions so the unrolled products index registers.
__host__ __device__ constexpr int ll2q(int i, int j) {
    return i <= j ? i * 4 - i * (i - 1) / 2 + (j - i) : j * 4 - j * (j - 1) / 2 + (i - j);
}
struct QL2C {
    int v[10][4];
};
__host__ __device__ constexpr QL2C make_ql2c() {
    return QL2C{{{0, 2, 4, 5}, {2, 3, 8, 9}, {4, 8, 10, 11}, {5, 9, 11, 12}, {3, 1, 6, 7}, {8, 6, 13, 14},
                 {9, 7, 14, 15}, {10, 13, 16, 17}, {11, 14, 17, 18}, {12, 15, 18, 19}}};
}
template <int I, int J>
struct QL2CAt {
    static constexpr int value = make_ql2c().v[I][J];
};
static_assert(ll2q(0, 0) == 0 && ll2q(1, 2) == 5 && ll2q(3, 3) == 9 && ll2q(2, 1) == 5, "ll2q");

template <int I = 0, int J = 0>
__device__ __forceinline__ void mul_ql_acc(const double* q, const double* l, double* c) {
    if constexpr (I < 10) {
        c[QL2CAt<I, J>::value] += q[I] * l[J];
        if constexpr (J + 1 < 4) mul_ql_acc<I, J + 1>(q, l, c);
        else mul_ql_acc<I + 1, 0>(q, l, c);
    }
}
template <int I = 0, int J = 0>
__device__ __forceinline__ void mul_ll_acc(const double* a, const double* b, double* q) {
    if constexpr (I < 4) {
        q[ll2q(I, J)] += a[I] * b[J];
        if constexpr (J + 1 < 4) mul_ll_acc<I, J + 1>(a, b, q);
        else mul_ll_acc<I + 1, 0>(a, b, q);
    }
}

__device__ __forceinline__ void mul_ll(const double* a, const double* b, double* q) {
#pragma unroll
    for (int k = 0; k < 10; ++k) q[k] = 0;
    mul_ll_acc(a, b, q);  // (i, j) row-major, as the reference's loops
}
__device__ __forceinline__ void mul_ql(const double* q, const double* l, double* c) {
#pragma unroll
    for (int k = 0; k < 20; ++k) c[k] = 0;
    mul_ql_acc(q, l, c);
}

// Rows: the nine entries of 2 EE^T E - tr(EE^T) E (row-major), then det E;
// columns 0..9 go to L (the matrix OpenCV inverts), 10..19 to G (its RHS).
// Both are register arrays (the row loops are unrolled, so every index is a
// constant): the 1.6 KB per hypothesis never leaves the CU.  The null-space
// basis EE (4 x 9) is read from LDS (EL[(c * 9 + e) * 64] = EE[c][e]); E E^T
// entries are formed per row block i (the three diagonal ones first, for the
// trace); recomputed entries are bit-identical.
__device__ __forceinline__ void ee_entry(const double* EL, int e, double (&o)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = EL[(c * 9 + e) * 64];
}

__device__ __forceinline__ void eet_entry(const double* EL, int i, int j, double (&o)[10]) {
    double a[4], b[4], t1[10];
    ee_entry(EL, i * 3 + 0, a);
    ee_entry(EL, j * 3 + 0, b);
    mul_ll(a, b, o);
#pragma unroll
    for (int k = 1; k < 3; ++k) {
        ee_entry(EL, i * 3 + k, a);
        ee_entry(EL, j * 3 + k, b);
        mul_ll(a, b, t1);
#pragma unroll
        for (int q = 0; q < 10; ++q) o[q] = o[q] + t1[q];
    }
}

__device__ __forceinline__ void coeff_matrix(const double* EL, double (&L)[10][10], double (&G)[10][10]) {
    double tr[10];
    {
        double d0[10], d1[10], d2[10];
        eet_entry(EL, 0, 0, d0);
        eet_entry(EL, 1, 1, d1);
        eet_entry(EL, 2, 2, d2);
#pragma unroll
        for (int k = 0; k < 10; ++k) tr[k] = (d0[k] + d1[k]) + d2[k];
    }
    double row[20], c1[20], c2[20], t1[10], t2[10];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double Ei[3][10];
        eet_entry(EL, i, 0, Ei[0]);
        eet_entry(EL, i, 1, Ei[1]);
        eet_entry(EL, i, 2, Ei[2]);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double e0[4], e1[4], e2[4], eij[4];
            ee_entry(EL, 0 * 3 + j, e0);
            ee_entry(EL, 1 * 3 + j, e1);
            ee_entry(EL, 2 * 3 + j, e2);
            ee_entry(EL, i * 3 + j, eij);
            mul_ql(Ei[0], e0, row);
            mul_ql(Ei[1], e1, c1);
#pragma unroll
            for (int k = 0; k < 20; ++k) row[k] = row[k] + c1[k];
            mul_ql(Ei[2], e2, c1);
#pragma unroll
            for (int k = 0; k < 20; ++k) row[k] = row[k] + c1[k];
            mul_ql(tr, eij, c1);
            const int r = i * 3 + j;
#pragma unroll
            for (int k = 0; k < 10; ++k) L[r][k] = 2.0 * row[k] - c1[k];
#pragma unroll
            for (int k = 0; k < 10; ++k) G[r][k] = 2.0 * row[10 + k] - c1[10 + k];
        }
    }
    double ea[4], eb[4];
    auto det2 = [&](int a0, int b0, int a1, int b1) {  // t1 = E[a0] E[b0] - E[a1] E[b1]
        ee_entry(EL, a0, ea);
        ee_entry(EL, b0, eb);
        mul_ll(ea, eb, t1);
        ee_entry(EL, a1, ea);
        ee_entry(EL, b1, eb);
        mul_ll(ea, eb, t2);
#pragma unroll
        for (int k = 0; k < 10; ++k) t1[k] = t1[k] - t2[k];
    };
    det2(4, 8, 5, 7);
    ee_entry(EL, 0, ea);
    mul_ql(t1, ea, row);
    det2(3, 8, 5, 6);
    ee_entry(EL, 1, ea);
    mul_ql(t1, ea, c1);
    det2(3, 7, 4, 6);
    ee_entry(EL, 2, ea);
    mul_ql(t1, ea, c2);
#pragma unroll
    for (int k = 0; k < 10; ++k) L[9][k] = (row[k] - c1[k]) + c2[k];
#pragma unroll
    for (int k = 0; k < 10; ++k) G[9][k] = (row[10 + k] - c1[10 + k]) + c2[10 + k];
}

// LUImpl<double>(A, 10, b, 10, DBL_EPSILON*100) (matrix_decomp.cpp), split so
// the 10x10 A stays in registers: the factorisation records the pivot rows and
// keeps each elimination multiplier in A's (never again read) lower triangle;
// the right-hand side is then replayed one column at a time from LDS with the
// identical operation sequence.  Only solution rows 4..9 are consumed by the
// five-point solver and back substitution of row i reads rows > i only, so
// rows 0..3 are not back-substituted.
__device__ __forceinline__ bool lu10_factor(double (&A)[10][10], int (&piv)[10]) {
    const double eps = DBL_EPSILON * 100;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        int k = i;
        double amax = fabs(A[i][i]);
#pragma unroll
        for (int j = i + 1; j < 10; j++) {
            const double v = fabs(A[j][i]);
            if (v > amax) {
                k = j;
                amax = v;
            }
        }
        if (amax < eps) return false;
        piv[i] = k;
#pragma unroll
        for (int r = i + 1; r < 10; r++)
            if (r == k) {
#pragma unroll
                for (int j = i; j < 10; j++) {
                    const double t = A[i][j];
                    A[i][j] = A[r][j];
                    A[r][j] = t;
                }
            }
        const double d = -1 / A[i][i];
#pragma unroll
        for (int j = i + 1; j < 10; j++) {
            const double alpha = A[j][i] * d;
            A[j][i] = alpha;
#pragma unroll
            for (int c = i + 1; c < 10; c++) A[j][c] += alpha * A[i][c];
        }
    }
    return true;
}

// G: the right-hand side; solution rows 4..9 replace its rows 4..9.
__device__ __forceinline__ void lu10_solve_cols(const double (&A)[10][10], const int (&piv)[10], double (&G)[10][10]) {
#pragma unroll
    for (int c = 0; c < 10; c++) {
        double x[10];
#pragma unroll
        for (int r = 0; r < 10; r++) x[r] = G[r][c];
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int k = piv[i];
#pragma unroll
            for (int r = i + 1; r < 10; r++)
                if (r == k) {
                    const double t = x[i];
                    x[i] = x[r];
                    x[r] = t;
                }
#pragma unroll
            for (int j = i + 1; j < 10; j++) x[j] += A[j][i] * x[i];
        }
#pragma unroll
        for (int i = 9; i >= 4; i--) {
            double sacc = x[i];
#pragma unroll
            for (int k = i + 1; k < 10; k++) sacc -= A[i][k] * x[k];
            x[i] = sacc / A[i][i];
        }
#pragma unroll
        for (int r = 4; r < 10; r++) G[r][c] = x[r];
    }
}

__device__ __forceinline__ int solve_cubic(const double* c, double* x) {
    double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3];
    double x0 = 0, x1 = 0, x2 = 0;
    int n;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0) n = a3 == 0 ? -1 : 0;
            else {
                x0 = -a3 / a2;
                n = 1;
            }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = sqrt(d);
                double q1 = (-a2 + d) * 0.5, q2 = (a2 + d) * -0.5;
                if (fabs(q1) > fabs(q2)) {
                    x0 = q1 / a1;
                    x1 = a3 / q1;
                } else {
                    x0 = q2 / a1;
                    x1 = a3 / q2;
                }
                n = d > 0 ? 2 : 1;
            } else
                n = 0;
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
            double theta = acos(R / sqrt(Qcubed));
            double sqrtQ = sqrt(Q);
            double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = a1 * (1. / 3);
            x0 = t0 * cos(t1) - t2;
            x1 = t0 * cos(t1 + (2. * M_PI / 3)) - t2;
            x2 = t0 * cos(t1 + (4. * M_PI / 3)) - t2;
            n = 3;
        } else if (d == 0) {
            if (R >= 0) {
                x0 = -2 * pow(R, 1. / 3) - a1 / 3;
                x1 = pow(R, 1. / 3) - a1 / 3;
            } else {
                x0 = 2 * pow(-R, 1. / 3) - a1 / 3;
                x1 = -pow(-R, 1. / 3) - a1 / 3;
            }
            x2 = 0;
            n = x0 == x1 ? 1 : 2;
            x1 = x0 == x1 ? 0 : x1;
        } else {
            d = sqrt(-d);
            double e = pow(d + fabs(R), 1. / 3);
            if (R > 0) e = -e;
            x0 = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    x[0] = x0;
    x[1] = x1;
    x[2] = x2;
    return n;
}

__device__ __forceinline__ Cx same_root_step(Cx num, int num_same_root) {
    double ore = num.re, oim = num.im;
    int sq_times = num_same_root % 2 == 0 ? num_same_root / 2 : num_same_root / 2 - 1;
    for (int j = 0; j < sq_times; j++) {
        num.re = ore * ore + oim * oim;
        num.re = sqrt(num.re);
        num.re += ore;
        num.im = num.re - ore;
        num.re /= 2;
        num.re = sqrt(num.re);
        num.im /= 2;
        num.im = sqrt(num.im);
        if (ore < 0) num.im = -num.im;
    }
    if (num_same_root % 2 != 0) {
        double cc[4], cr[3];
        cc[3] = -(pow(ore, 3));
        cc[2] = -(15 * pow(ore, 2) + 27 * pow(oim, 2));
        cc[1] = -48 * ore;
        cc[0] = 64;
        solve_cubic(cc, cr);
        if (cr[0] >= 0) num.re = pow(cr[0], 1. / 3);
        else num.re = -pow(-cr[0], 1. / 3);
        num.im = sqrt(pow(num.re, 2) / 3 - ore / (3 * num.re));
    }
    return num;
}

// solvePoly, full degree 10: constant indices keep roots/coeffs in registers.
// One Gauss-Seidel sweep of solvePoly's Durand-Kerner iteration (mathfuncs.cpp)
// over the 10 roots; `moved` is the reference's maxDiff > 0.  kSameRoot=false
// leaves out the (register-hungry) coincident-root step and only reports it in
// `same`; the caller then redoes the polynomial with kSameRoot=true.
template <bool kSameRoot>
__device__ __forceinline__ void dk_sweep(const double (&c)[11], Cx (&roots)[10], bool& moved, bool& same) {
    moved = false;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const Cx p = roots[i];
        Cx num{c[10], 0}, denom{c[10], 0};
        int num_same_root = 1;
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const Cx t = cmul(num, p);
            num = Cx{t.re + c[10 - j - 1], t.im + 0.0};
            if (j != i) {
                Cx d = csub(p, roots[j]);
                if constexpr (kSameRoot) {
                    if (d.re == 0 && d.im == 0) num_same_root++;
                    else denom = cmul(denom, d);
                } else {
                    denom = cmul(denom, d);  // an exactly zero factor is caught below
                }
            }
        }
        if constexpr (!kSameRoot) {
            // A coincident root makes a factor exactly 0, so the unconditional
            // product is 0 or NaN: such polynomials, and the rare false alarms
            // (underflow, overflow), are redone exactly by the kSameRoot path.
            same |= !(denom.re != 0 || denom.im != 0) || denom.re != denom.re || denom.im != denom.im;
        }
        num = cdiv(num, denom);
        if constexpr (kSameRoot) {
            if (num_same_root > 1) num = same_root_step(num, num_same_root);
        }
        roots[i] = csub(p, num);
        // std::max(maxDiff, cv::abs(num)) > 0  <=>  re^2 + im^2 > 0 (sqrt is monotone, NaN stays out)
        moved |= (num.re * num.re + num.im * num.im) > 0;
    }
}

__device__ __forceinline__ void dk_init(Cx (&roots)[10]) {
    Cx p{1, 0}, r{1, 1};
#pragma unroll
    for (int i = 0; i < 10; i++) {
        roots[i] = p;
        p = cmul(p, r);
    }
}

__device__ __forceinline__ bool dk_same(const Cx (&a)[10], const Cx (&b)[10]) {
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 10; i++)
        eq &= (__double_as_longlong(a[i].re) == __double_as_longlong(b[i].re)) &
              (__double_as_longlong(a[i].im) == __double_as_longlong(b[i].im));
    return eq;
}

// Brent cycle detection on the sweep's state.  The sweep is a deterministic map
// S_k -> S_{k+1} of the 10 roots, so once S_k == S_a (a < k) the sequence is
// periodic with period k - a and S_300 = S_{k + (300 - k) mod (k - a)}: the
// iteration stops at that sweep with the roots the reference's 300 sweeps end
// on (or earlier at the reference's own maxDiff <= 0 exit).
// `saved` is a strided per-lane column (element k at saved[k * stride]) so the
// snapshot can live in LDS in the persistent kernel.
struct DkBrent {
    double* saved;
    int stride;
    int it, saved_it, power, target;
    __device__ void snap(const Cx (&roots)[10]) {
#pragma unroll
        for (int i = 0; i < 10; i++) {
            saved[(2 * i) * stride] = roots[i].re;
            saved[(2 * i + 1) * stride] = roots[i].im;
        }
    }
    __device__ void start(const Cx (&roots)[10]) {
        snap(roots);
        it = 0;
        saved_it = 0;
        power = 1;
        target = 300;
    }
    // after one sweep; true when the roots are final
    __device__ bool step(const Cx (&roots)[10], bool moved) {
        ++it;
        if (!moved || it >= target) return true;
        if (target == 300) {
            bool eq = true;
#pragma unroll
            for (int i = 0; i < 10; i++)
                eq &= (__double_as_longlong(roots[i].re) == __double_as_longlong(saved[(2 * i) * stride])) &
                      (__double_as_longlong(roots[i].im) == __double_as_longlong(saved[(2 * i + 1) * stride]));
            if (eq) {
                target = it + (300 - it) % (it - saved_it);
                return it >= target;
            }
            if (it - saved_it == power) {
                snap(roots);
                saved_it = it;
                power <<= 1;
            }
        }
        return false;
    }
};

__device__ __forceinline__ void dk_finish(Cx (&roots)[10]) {
#pragma unroll
    for (int i = 0; i < 10; i++)
        if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
}

// solvePoly for a degree-10 polynomial (single thread).
__device__ __forceinline__ void solve_poly10(const double (&c)[11], Cx (&roots)[10]) {
    dk_init(roots);
    double saved[20];
    DkBrent br;
    br.saved = saved;
    br.stride = 1;
    br.start(roots);
    for (;;) {
        bool moved, same = false;
        dk_sweep<true>(c, roots, moved, same);
        if (br.step(roots, moved)) break;
    }
    dk_finish(roots);
}

// solvePoly generic (leading coefficients trimmed; rare): scratch arrays.
__device__ int solve_poly_generic(const double* rc, int n0, Cx* roots) {
    Cx coeffs[11];
    for (int i = 0; i <= n0; i++) coeffs[i] = Cx{rc[i], 0};
    int n = n0;
    for (; n > 1; n--)
        if (fabs(coeffs[n].re) + fabs(coeffs[n].im) > DBL_EPSILON) break;
    Cx p{1, 0}, r{1, 1};
    for (int i = 0; i < n; i++) {
        roots[i] = p;
        p = cmul(p, r);
    }
    for (int iter = 0; iter < 300; iter++) {
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
            if (num_same_root > 1) num = same_root_step(num, num_same_root);
            roots[i] = csub(p, num);
            double an = cabs_(num);
            maxDiff = maxDiff < an ? an : maxDiff;
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; i++)
        if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    return n;
}

__device__ __forceinline__ void poly_mul(const double* a, int na, const double* b, int nb, double* r) {
#pragma unroll
    for (int k = 0; k < na + nb - 1; ++k) r[k] = 0;
#pragma unroll
    for (int i = 0; i < na; ++i)
#pragma unroll
        for (int j = 0; j < nb; ++j) r[i + j] += a[i] * b[j];
}

// five-point.cpp EMEstimatorCallback::runKernel; q: 5 x (x1, y1, x2, y2)
// normalised.  Writes up to 10 models (9 doubles each) and returns the count.
// Five-point solver (five-point.cpp, Nister via Stewenius' coefficient matrix)
// in three stages so the Durand-Kerner root finder can run as its own
// load-balanced kernel.  A hypothesis record R holds, element k at R[k * 64]:
//   [0, 11) polynomial coefficients c, [11, 50) the 3 x 13 matrix b,
//   [50, 86) the null-space basis EE (4 x 9), [86, 106) roots (re, im),
//   106: number of roots, 107: 1 when c[10] is negligible (generic solvePoly),
//   2 when two roots coincided exactly in the fast Durand-Kerner kernel.
constexpr int kRecC = 0, kRecB = 11, kRecEE = 50, kRecRoots = 86, kRecNr = 106, kRecGeneric = 107;
constexpr int kRecDoubles = 128;

// Stage A: Q -> null space (JacobiSVD) -> 10x20 coefficient matrix -> LU solve
// -> b -> degree-10 polynomial.  EL: this thread's LDS column of 36 doubles.
// The coefficient matrix and the solve stay in registers (L and G: 400 VGPRs
// at the peak, one wave per SIMD as before; round 2 kept them in a 1.6 KB
// global scratch column per hypothesis).
__device__ __forceinline__ void fp_stage_a(const double (&q)[5][4], double* EL, double* R) {
    double At[9][9], W[5], Vt[5][5];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < 9; ++k) At[i][k] = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        double x1 = q[i][0], y1 = q[i][1], x2 = q[i][2], y2 = q[i][3];
        At[i][0] = x1 * x2;
        At[i][1] = y1 * x2;
        At[i][2] = x2 + 0.0;
        At[i][3] = x1 * y2;
        At[i][4] = y1 * y2;
        At[i][5] = y2 + 0.0;
        At[i][6] = x1 + 0.0;
        At[i][7] = y1 + 0.0;
        At[i][8] = 1.0;
    }
    jacobi_svd<9, 5, 9, 9>(At, W, Vt);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const double v = At[5 + r][k] + 0.0;
            EL[(r * 9 + k) * 64] = v;
            R[(kRecEE + r * 9 + k) * 64] = v;
        }
    double b[3 * 13];
    {
        // A = A.colRange(0,10).inv() * A.colRange(10,20) == solve(A1, A2, DECOMP_LU)
        double L[10][10], G[10][10];
        int piv[10];
        coeff_matrix(EL, L, G);
        if (lu10_factor(L, piv)) {
            lu10_solve_cols(L, piv, G);
        } else {
#pragma unroll
            for (int r = 4; r < 10; ++r)
#pragma unroll
                for (int k = 0; k < 10; ++k) G[r][k] = 0;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double* a1 = G[i * 2 + 4];
            const double* a2 = G[i * 2 + 5];
            double row1[13], row2[13];
#pragma unroll
            for (int k = 0; k < 13; ++k) row1[k] = row2[k] = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) row1[1 + k] = (a1[k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) row1[5 + k] = (a1[3 + k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) row1[9 + k] = (a1[6 + k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) row2[0 + k] = (a2[k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) row2[4 + k] = (a2[3 + k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) row2[8 + k] = (a2[6 + k] + 0.0) + 0.0;
#pragma unroll
            for (int k = 0; k < 13; ++k) b[i * 13 + k] = row1[k] - row2[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 39; ++k) R[(kRecB + k) * 64] = b[k];
    double px[3][4], py[3][4], pc[3][5];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < 4; ++k) px[j][k] = b[j * 13 + 3 - k];
#pragma unroll
        for (int k = 0; k < 4; ++k) py[j][k] = b[j * 13 + 7 - k];
#pragma unroll
        for (int k = 0; k < 5; ++k) pc[j][k] = b[j * 13 + 12 - k];
    }
    double u[8], v[8], m1[8], m2[8], m3[8], t1[11], t2[11], t3[11];
    poly_mul(py[1], 4, pc[2], 5, u);
    poly_mul(pc[1], 5, py[2], 4, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m1[k] = u[k] - v[k];
    poly_mul(px[1], 4, pc[2], 5, u);
    poly_mul(pc[1], 5, px[2], 4, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m2[k] = u[k] - v[k];
    poly_mul(px[1], 4, py[2], 4, u);
    poly_mul(py[1], 4, px[2], 4, v);
#pragma unroll
    for (int k = 0; k < 7; ++k) m3[k] = u[k] - v[k];
    poly_mul(px[0], 4, m1, 8, t1);
    poly_mul(py[0], 4, m2, 8, t2);
    poly_mul(pc[0], 5, m3, 7, t3);
    double c10 = 0;
#pragma unroll
    for (int k = 0; k < 11; ++k) {
        const double ck = (t1[k] - t2[k]) + t3[k];
        R[(kRecC + k) * 64] = ck;
        c10 = ck;
    }
    R[kRecGeneric * 64] = fabs(c10) > DBL_EPSILON ? 0.0 : 1.0;
}

// Stage C: roots -> (x, y, z) by the 3x3 null space of B(z) -> E, normalised.
// Polynomials flagged generic (leading coefficient negligible) are solved here.
__device__ __forceinline__ void dk_store(double* R, Cx (&roots)[10]);
// The model of one real root z1 (five-point.cpp getModels, per root): x, y from
// the SVD of the 3x3 B(z1), E = x X + y Y + z W + Z normalised.  False when the
// root is rejected (|v22| < 1e-10).
__device__ __forceinline__ bool root_model(const double (&b)[39], const double (&EE)[36], double z1, double (&out)[9]) {
    double z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
    double bz[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double* br = b + j * 13;
        bz[j][0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
        bz[j][1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
        bz[j][2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
    }
    double at3[3][3], w3[3], vt3[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) at3[r][k] = bz[k][r];
    jacobi_svd<3, 3, 0, 3>(at3, w3, vt3);
    if (fabs(vt3[2][2]) < 1e-10) return false;
    double xs = vt3[2][0] / vt3[2][2], ys = vt3[2][1] / vt3[2][2];
    double e[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) e[k] = (((EE[k] * xs + EE[9 + k] * ys) + 0.0) + EE[18 + k] * z1) + EE[27 + k];
    double s = 0;
    s += e[0] * e[0] + e[1] * e[1] + e[2] * e[2] + e[3] * e[3];
    s += e[4] * e[4] + e[5] * e[5] + e[6] * e[6] + e[7] * e[7];
    s += e[8] * e[8];
    double inv_n = 1. / sqrt(s);
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = e[k] * inv_n + 0.0;
    return true;
}

// Roots of a polynomial stage A flagged for an exact solve (2: coincident roots
// in Durand-Kerner, other nonzero: the generic solver), stored in the record.
__device__ __forceinline__ void fp_exact_roots(double* R, bool store) {
    if (R[kRecGeneric * 64] == 2.0) {
        double c[11];
        Cx roots[10];
#pragma unroll
        for (int k = 0; k < 11; ++k) c[k] = R[(kRecC + k) * 64];
        solve_poly10(c, roots);
        if (store) dk_store(R, roots);
    } else if (R[kRecGeneric * 64] != 0.0) {
        double c[11];
        Cx roots[10];
#pragma unroll
        for (int k = 0; k < 11; ++k) c[k] = R[(kRecC + k) * 64];
        const int nr = solve_poly_generic(c, 10, roots);
        if (store) {
            for (int i = 0; i < nr; ++i) {
                R[(kRecRoots + 2 * i) * 64] = roots[i].re;
                R[(kRecRoots + 2 * i + 1) * 64] = roots[i].im;
            }
            R[kRecNr * 64] = nr;
        }
    }
}

__device__ __forceinline__ int fp_stage_c(double* R, double* models) {
    fp_exact_roots(R, true);
    double b[39], EE[36];
#pragma unroll
    for (int k = 0; k < 39; ++k) b[k] = R[(kRecB + k) * 64];
#pragma unroll
    for (int k = 0; k < 36; ++k) EE[k] = R[(kRecEE + k) * 64];
    const int nr = (int)R[kRecNr * 64];
    // the real roots first, as a mask: a wave then runs as many root models as its lane with the most
    // real roots, not one per root position any lane's real root sits at
    uint32_t real = 0;
    for (int i = 0; i < nr; ++i) real |= (fabs(R[(kRecRoots + 2 * i + 1) * 64]) > 1e-10 ? 0u : 1u) << i;
    int count = 0;
    while (real) {
        const int i = __builtin_ctz(real);
        real &= real - 1;
        double e[9];
        if (!root_model(b, EE, R[(kRecRoots + 2 * i) * 64], e)) continue;
        double* out = models + count * 9;
#pragma unroll
        for (int k = 0; k < 9; ++k) out[k] = e[k];
        count++;
    }
    return count;
}

__device__ __forceinline__ void dk_store(double* R, Cx (&roots)[10]) {
    dk_finish(roots);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        R[(kRecRoots + 2 * i) * 64] = roots[i].re;
        R[(kRecRoots + 2 * i + 1) * 64] = roots[i].im;
    }
    R[kRecNr * 64] = 10;
}

// All three stages in one thread (test hook).  R: a 128-double record column.
__device__ __forceinline__ int five_point(const double (&q)[5][4], double* models, double* EL, double* R) {
    fp_stage_a(q, EL, R);
    if (R[kRecGeneric * 64] == 0.0) {
        double c[11];
        Cx roots[10];
#pragma unroll
        for (int k = 0; k < 11; ++k) c[k] = R[(kRecC + k) * 64];
        solve_poly10(c, roots);
        dk_store(R, roots);
    }
    return fp_stage_c(R, models);
}

__device__ int ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, (double)model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : cv_round_d(num / denom);
}

// ---------------------------------------------------------------------------

__device__ __forceinline__ int pair_m(const GeomArgs& g, int p) { return g.m_arr ? g.m_arr[p] : g.m_const; }

// findEssentialMat/recoverPose: col = (col - c)/f as OpenCV's MatExpr evaluates
// it: col * (1/f) + (-c * (1/f)).
__global__ __launch_bounds__(256) void normalize_kernel(GeomArgs g) {
    const int p = blockIdx.y;
    const int m = pair_m(g, p);
    const double ax = 1. / g.fx, ay = 1. / g.fy, bx = -g.cx * ax, by = -g.cy * ay;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) {
        const int64_t o = ((int64_t)p * g.pts_stride + i) * 4;
        double x1, y1, x2, y2;
        if (g.pts_f) {
            x1 = g.pts_f[o];
            y1 = g.pts_f[o + 1];
            x2 = g.pts_f[o + 2];
            y2 = g.pts_f[o + 3];
        } else {
            x1 = g.pts_d[o];
            y1 = g.pts_d[o + 1];
            x2 = g.pts_d[o + 2];
            y2 = g.pts_d[o + 3];
        }
        g.npts[o] = x1 * ax + bx;
        g.npts[o + 1] = y1 * ay + by;
        g.npts[o + 2] = x2 * ax + bx;
        g.npts[o + 3] = y2 * ay + by;
    }
}

// ---- findEssentialMat RANSAC (ptsetreg.cpp RANSACPointSetRegistrator::run) ----
// The sequential loop "sample 5 -> five-point -> count inliers of each root ->
// keep the first model beating max(best, 4) and shrink niters" is split into
// batch-wide kernels.  Hypotheses only depend on the RNG stream, so a round
// samples a range of them (one thread per pair, sequential RNG), solves all of
// them in parallel (one thread per hypothesis), counts inliers of every root
// in parallel (one wave per model), then replays the sequential bookkeeping in
// order (one thread per pair).  niters never grows, so round 1 covers
// [0, min(64, niters)) and round 2 everything left, [64, niters)
// (kRansacBounds): the result is the sequential loop's, bit for bit.
constexpr int kSolveNT = 64;
#ifndef DVO_SCORE_CHUNK
#define DVO_SCORE_CHUNK 256  // points per LDS chunk: smaller chunks, more resident blocks (measured)
#endif
#ifndef DVO_SCORE_HYPS_CALL
#define DVO_SCORE_HYPS_CALL 2  // drop-in pairs/s (profiles/r02z_ab_dropin_score_hyps.txt): 1 620, 2 626, 4 611, 16 610
#endif
constexpr int kScoreNT = 256, kScoreHyps = 16, kScoreChunk = DVO_SCORE_CHUNK;
// Deferred f64 Sampson tests per score block: the (model, point) pairs the
// single-precision bounds leave undecided are listed in LDS while the waves
// stream the chunks, and the whole block runs their f64 tests once, after the
// last chunk (one latency round trip per block instead of one per wave-chunk
// that met an undecided point).  A full list falls back to the inline test.
constexpr int kScoreUnd = 1024;
// Early exit of a model that cannot matter: the replay changes state only at a count above
// max(maxgood, 4) of the rounds before (RANSACPointSetRegistrator::run's test, ptsetreg.cpp), so
// once a model's count so far plus its deferred tests plus the points not yet scored is <= that
// bound, its final count is too, and it stops being scored (the partial count it stores is <= the
// bound as well: the replay cannot tell the difference).  Round 2 starts from round 1's maxgood.
constexpr int kScoreHypsCall = DVO_SCORE_HYPS_CALL;

// getSubset (ptsetreg.cpp) for the round's hypotheses [h0, h1) of one pair,
// one wave per pair: idx[i] = rng.uniform(0, m) = rng.next() % m, redrawn
// while it repeats an earlier index of the subset.  The MWC stream itself is
// sequential, but a multiply-with-carry stream can be jumped ahead (below), the
// subsets are assembled 64 at a time: lane j takes the 5 states after the
// 5j consumed before it, which is exact unless an earlier lane drew a
// duplicate; the first such lane redoes its subset with the rejection loop
// (wave-uniform, ~1% of subsets) and the next 64 start after it.  The stream
// is staged 1,024 states at a time, 64 lanes jumping ahead (below).
constexpr int kSampleBuf = 1024;  // MWC states staged per refill

// Jump-ahead of cv::RNG's multiply-with-carry step s' = (u32)s * A + (s >> 32),
// A = 4164903690.  With m = A * 2^32 - 1, s' * 2^32 = s + (u32)s * m, so
// s' = s * A (mod m) (A = 2^-32 mod m), and a state below m stays below m: from
// the second state of a stream on (the seed ~0 is the only state >= m it
// meets), s_{n+k} = s_n * A^k mod m exactly.  Lane j of a refill starts from
// s_n * A^(16 j + 1), a Montgomery product (R = 2^64) with the table below,
// and steps 15 times; the buffer equals lane 0 running the stream sequentially.
constexpr uint64_t kMwcA = 4164903690ull;
constexpr uint64_t kMwcM = kMwcA * (1ull << 32) - 1;
constexpr uint64_t mwc_mprime() {  // -m^-1 mod 2^64 (Newton)
    uint64_t inv = kMwcM;
    for (int i = 0; i < 6; ++i) inv *= 2 - kMwcM * inv;
    return 0 - inv;
}
constexpr uint64_t kMwcMp = mwc_mprime();
struct MwcJump {
    uint64_t v[64];  // A^(16 j + 1) * 2^64 mod m
};
constexpr MwcJump mwc_jump() {
    MwcJump t{};
    unsigned __int128 p = kMwcA % kMwcM;  // A^1
    unsigned __int128 a16 = 1;
    for (int i = 0; i < 16; ++i) a16 = a16 * kMwcA % kMwcM;
    for (int j = 0; j < 64; ++j) {
        t.v[j] = (uint64_t)((p << 64) % kMwcM);
        p = p * a16 % kMwcM;
    }
    return t;
}
__constant__ MwcJump c_mwc_jump = mwc_jump();
static_assert(kMwcM % 2 == 1 && (uint64_t)(kMwcM * (0 - kMwcMp)) == 1, "Montgomery constants");

__device__ __forceinline__ uint64_t mwc_mont(uint64_t a, uint64_t bR) {  // a * b mod m, a < m, bR = b * 2^64 mod m
    const uint64_t lo = a * bR, hi = __umul64hi(a, bR);
    const uint64_t u = lo * kMwcMp;
    const uint64_t uh = __umul64hi(u, kMwcM);
    uint64_t t = hi + uh;
    const bool c1 = t < hi;
    const uint64_t c = lo != 0;  // lo + u * m = 0 mod 2^64, with a carry unless lo == 0
    const uint64_t t2 = t + c;
    const bool c2 = t2 < t;
    return (c1 || c2 || t2 >= kMwcM) ? t2 - kMwcM : t2;
}
// Launch pair p belongs to set p / F, which runs round spec.round[set] (-1: idle set, its pairs
// get an empty range); slots past the set's batch (npairs) start with m = 0 (nothing to do).
__global__ __launch_bounds__(64) void ransac_sample_kernel(GeomArgs g, RoundSpec spec) {
    const int p = blockIdx.x;
    const int set = p / spec.F, local = p - set * spec.F;
    if (set >= spec.nsets) return;
    const int lane = threadIdx.x;
    __shared__ uint64_t s_st[kSampleBuf];
    RansacState S = g.rs[p];
    int32_t* idx = g.subsets + (int64_t)p * g.hyp_cap * 5;
    const int round = spec.round[set];
    if (round < 0) {  // idle set: no hypotheses this launch
        S.h0 = S.h1;
        if (lane == 0) g.rs[p] = S;
        return;
    }
    const int bound = spec.bound[round];
    int h0, h1;
    if (round == 0) {
        S.m = local < spec.npairs[set] ? pair_m(g, p) : 0;
        S.rng = ~0ull;  // RNG rng((uint64)-1)
        S.niters = g.max_iters > 1 ? g.max_iters : 1;
        S.iter = 0;
        S.maxgood = 0;
        S.best_h = S.best_i = -1;
        h0 = 0;
        if (S.m < 5) {
            h1 = 0;
        } else if (S.m == 5) {  // count == modelPoints: one direct solve, no RANSAC
            if (lane < 5) idx[lane] = lane;
            h1 = 1;
        } else {
            h1 = min(bound, S.niters);
        }
        if (S.m <= 5) {
            S.h0 = h0;
            S.h1 = h1;
            if (lane == 0) g.rs[p] = S;
            return;
        }
    } else {
        h0 = S.h1;
        h1 = (S.m > 5 && S.iter < S.niters) ? min(S.niters, bound) : h0;
    }
    const unsigned m = (unsigned)S.m;
    // x % m by Lemire's fastmod (exact for every 32-bit x and m)
    const uint64_t M = ~0ull / m + 1;
    auto draw = [&](uint64_t st) { return (int)__umul64hi(M * (uint64_t)(uint32_t)st, (uint64_t)m); };
    uint64_t gen = S.rng;   // last generated state (lane 0's stream position)
    uint64_t last = S.rng;  // state after the last consumed draw
    int avail = 0, cur = 0;
    auto refill = [&]() {  // keep the unconsumed states, then extend the buffer to kSampleBuf
        const int keep = avail - cur;
        uint64_t tmp[kSampleBuf / 64];
#pragma unroll
        for (int k = 0; k < kSampleBuf / 64; ++k) tmp[k] = 64 * k + lane < keep ? s_st[cur + 64 * k + lane] : 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSampleBuf / 64; ++k)
            if (64 * k + lane < keep) s_st[64 * k + lane] = tmp[k];
        const int head = min(2, kSampleBuf - keep);  // sequential: the stream's first state may be >= m
        if (lane == 0) {
            uint64_t st = gen;
            for (int k = keep; k < keep + head; ++k) {
                st = (uint64_t)(uint32_t)st * kMwcA + (st >> 32);
                s_st[k] = st;
            }
        }
        __syncthreads();
        const int rest = kSampleBuf - keep - head;  // the remaining states by jump-ahead, 16 per lane
        if (16 * lane < rest) {
            const int k0 = keep + head + 16 * lane;
            uint64_t st = mwc_mont(s_st[keep + head - 1], c_mwc_jump.v[lane]);
            s_st[k0] = st;
            for (int q = 1; q < 16 && k0 + q < kSampleBuf; ++q) {
                st = (uint64_t)(uint32_t)st * kMwcA + (st >> 32);
                s_st[k0 + q] = st;
            }
        }
        __syncthreads();
        gen = s_st[kSampleBuf - 1];
        avail = kSampleBuf;
        cur = 0;
    };
    int h = h0;
    while (h < h1) {
        if (avail - cur < 5 * 64) refill();
        const int hj = h + lane;
        const bool act = hj < h1;
        int v[5];
        bool dup = false;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            v[i] = draw(s_st[cur + 5 * lane + i]);
#pragma unroll
            for (int j = 0; j < i; ++j) dup |= v[j] == v[i];
        }
        const unsigned long long bad = __ballot(act && dup);
        const int nact = min(64, h1 - h);
        const int nok = bad ? min(nact, (int)__builtin_ctzll(bad)) : nact;
        if (lane < nok) {
#pragma unroll
            for (int i = 0; i < 5; ++i) idx[(int64_t)hj * 5 + i] = v[i];
        }
        if (nok > 0) last = s_st[cur + 5 * nok - 1];
        h += nok;
        cur += 5 * nok;
        if (nok < nact) {  // hypothesis h drew a duplicate: its subset with the rejection loop (wave-uniform)
            int w[5];
            for (int i = 0; i < 5; ++i) {
                for (;;) {
                    if (cur == avail) refill();
                    last = s_st[cur++];
                    w[i] = draw(last);
                    bool d = false;
                    for (int j = 0; j < i; ++j) d |= w[j] == w[i];
                    if (!d) break;
                }
            }
            if (lane < 5) idx[(int64_t)h * 5 + lane] = w[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : lane == 3 ? 3 : 4];
            ++h;
        }
    }
    S.rng = last;
    S.h0 = h0;
    S.h1 = h1;
    if (lane == 0) g.rs[p] = S;
}

// The five-point record of hypothesis h of launch pair p: records exist for the round's
// hypotheses only, one per work item (dk_off[p] + h - h0), in blocks of 64 items (a wave of stage
// A / C / Durand-Kerner pass 0 = 64 consecutive items = one record block: coalesced).
__device__ __forceinline__ double* item_record(const GeomArgs& g, int64_t r) {
    return g.fprec + ((r >> 6) * kRecDoubles) * 64 + (r & 63);
}
__device__ __forceinline__ double* hyp_record(const GeomArgs& g, int p, int h) {
    return item_record(g, (int64_t)g.dk_off[p] + (h - g.rs[p].h0));
}

// Pair of a round work-list item: the p with off[p] <= item < off[p + 1] (off ascending).
__device__ __forceinline__ int pair_of(const int32_t* off, int pairs, int item) {
    int lo = 0, hi = pairs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= item) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Work list of the round for the Durand-Kerner kernel: exclusive prefix of the
// per-pair hypothesis counts, the total, and a reset queue head.
// and the same prefixes in 64-hypothesis blocks (stage A / C, five-point records) and in score
// blocks of sh hypotheses.  Wave prefix sums, one carry per 1024 pairs.
__global__ __launch_bounds__(1024) void ransac_plan_kernel(GeomArgs g, int pairs, int sh) {
    __shared__ int4 s_w[16];
    __shared__ int4 s_carry;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = make_int4(0, 0, 0, 0);
    for (int b0 = 0; b0 < pairs; b0 += 1024) {
        const int p = b0 + threadIdx.x;
        const int n = p < pairs ? max(0, g.rs[p].h1 - g.rs[p].h0) : 0;
        const int na = (n + 63) >> 6, ns = (n + sh - 1) / sh;
        int x = n, y = na, z = ns;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scans
            const int xo = __shfl_up(x, o), yo = __shfl_up(y, o), zo = __shfl_up(z, o);
            if (lane >= o) {
                x += xo;
                y += yo;
                z += zo;
            }
        }
        __syncthreads();
        if (lane == 63) s_w[wid] = make_int4(x, y, z, 0);
        __syncthreads();
        int4 c = s_carry;
        for (int w = 0; w < wid; ++w) {
            c.x += s_w[w].x;
            c.y += s_w[w].y;
            c.z += s_w[w].z;
        }
        if (p < pairs) {
            g.dk_off[p] = c.x + x - n;
            g.a_off[p] = c.y + y - na;
            g.s_off[p] = c.z + z - ns;
        }
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = make_int4(c.x + x, c.y + y, c.z + z, 0);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        g.dk_off[pairs] = s_carry.x;
        g.a_off[pairs] = s_carry.y;
        g.s_off[pairs] = s_carry.z;
        g.dk_ctl[0] = 0;
        g.dk_ctl[1] = s_carry.x;  // pass 0 items
        for (int k = 0; k < kDkMaxPasses; ++k) g.dk_ctl[2 + k] = 0;  // parked after pass k
    }
}

// The launch pair of work item e = e0 + lane (dk_off: the round's hypotheses of all pairs back to
// back), for the wave of items [e0, e0 + 64): the first item's pair by a wave-uniform binary search,
// then the pair boundaries inside the wave (typically one or two: a round gives a pair 32+
// hypotheses) by uniform loads, each lane counting those at or below its item (empty pairs repeat a
// boundary and are counted through).  Packing the items leaves no lane idle where a pair's
// hypotheses end (64-hypothesis blocks per pair left stage A at 0.61 and stage C at 0.24 of the
// VALU lanes active, profiles/r05zz_pmc_f64.json).  Past 8 boundaries (a run of empty pairs: pairs
// whose loop already stopped, idle sets) each lane finishes with a binary search up to the last
// pair of the wave, so no wave walks a long run of empty pairs one load at a time.
static_assert(kSolveNT == 64, "wave_item_pair assumes one wave of 64 items per block");
__device__ __forceinline__ int wave_item_pair(const int32_t* off, int pairs, int e0, int e) {
    int p = pair_of(off, pairs, e0);
    const int lim = min(pairs, p + 8);
    for (int k = p + 1; k <= lim; ++k) {
        const int b = off[k];
        if (b > e0 + 63) return p;
        p += e >= b;
    }
    if (lim == pairs || p < lim) return p;
    int lo = p, hi = pair_of(off, pairs, e0 + 63);
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Stage A of every hypothesis of the round (one thread each), a 1-D grid over the round's items.
__global__ __launch_bounds__(kSolveNT) void ransac_stage_a_kernel(GeomArgs g, int pairs) {
    const int e0 = blockIdx.x * kSolveNT;
    if (e0 >= g.dk_off[pairs]) return;
    const int e = e0 + threadIdx.x;
    const int p = wave_item_pair(g.dk_off, pairs, e0, e);
    __shared__ double lds_g[36 * kSolveNT];
    if (e >= g.dk_off[pairs]) return;
    const int h = g.rs[p].h0 + (e - g.dk_off[p]);
    const double* npts = g.npts + (int64_t)p * g.pts_stride * 4;
    const int32_t* idx = g.subsets + ((int64_t)p * g.hyp_cap + h) * 5;
    double q[5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double* src = npts + (int64_t)idx[i] * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[i][k] = src[k];
    }
    fp_stage_a(q, lds_g + threadIdx.x, hyp_record(g, p, h));
}

// Durand-Kerner for every polynomial of the round, in passes that shrink the
// set of waves holding the long tail.  A pass gives every listed polynomial
// one lane and at most `budget` sweeps; polynomials still running then (a long
// pre-period or period before Brent's exit, or no cycle within 300 sweeps:
// ~40% after 48 sweeps, ~20% after 128) park their state in their record -
// roots, Brent snapshot and counters - and join the next pass's list.  The
// sweeps are the same deterministic map whichever pass runs them, so the
// roots are bit-identical to one uninterrupted run; the tail just no longer
// keeps every wave of the round resident (it needed all of them for ~300
// sweeps before).
constexpr int kDkNT = 256;
// Sweeps of each pass but the last, which runs to the end; a zero ends the list.
// Between passes the unfinished polynomials are compacted, so the waves of the
// next pass are full.
#ifndef DVO_DK_B0
#define DVO_DK_B0 48
#endif
#ifndef DVO_DK_B1
#define DVO_DK_B1 80
#endif
#ifndef DVO_DK_B2
#define DVO_DK_B2 0
#endif
constexpr int kDkBudgets[kDkMaxPasses - 1] = {DVO_DK_B0, DVO_DK_B1, DVO_DK_B2};
constexpr int kDkPasses = DVO_DK_B0 == 0 ? 1 : DVO_DK_B1 == 0 ? 2 : DVO_DK_B2 == 0 ? 3 : 4;
constexpr int kRecSnap = 108;                     // parked: Brent snapshot (20 doubles)
#ifdef DVO_DK_STATS
// Measurement build only: per pass, the sweeps run by each lane (useful work) and the
// sweeps of each wave (its slowest lane: issued work), printed by dk_stats_kernel.
constexpr int kDkStatWaves = 1 << 16;
__device__ unsigned int g_dk_wave_max[kDkMaxPasses][kDkStatWaves];
__device__ unsigned long long g_dk_lane_sum[kDkMaxPasses];
__device__ __forceinline__ void dk_stat(int pass, int sweeps) {
    atomicAdd(&g_dk_lane_sum[pass], (unsigned long long)sweeps);
    const int w = (int)(blockIdx.x * (kDkNT / 64) + (threadIdx.x >> 6));
    if (w < kDkStatWaves) atomicMax(&g_dk_wave_max[pass][w], (unsigned)sweeps);
}
__global__ void dk_stats_kernel(int round, int nwaves) {
    for (int pass = 0; pass < kDkMaxPasses; ++pass) {
        unsigned long long ws = 0, nw = 0;
        for (int w = 0; w < min(nwaves, kDkStatWaves); ++w) {
            ws += g_dk_wave_max[pass][w];
            nw += g_dk_wave_max[pass][w] > 0;
            g_dk_wave_max[pass][w] = 0;
        }
        if (ws)
            printf("DKSTAT round %d pass %d lane_sweeps %llu wave_sweeps_x64 %llu waves %llu lane_eff %.4f\n", round, pass,
                   g_dk_lane_sum[pass], ws * 64, nw, (double)g_dk_lane_sum[pass] / (double)(ws * 64));
        g_dk_lane_sum[pass] = 0;
    }
}
#define DK_STAT(pass, n) dk_stat(pass, n)
#else
#define DK_STAT(pass, n) ((void)0)
#endif
// 3 waves per SIMD (130 VGPRs); 4 spills 14 VGPRs and measured -0.3 % (profiles/r05s_ab_replay_dk_waves.txt)
__global__ __launch_bounds__(kDkNT) __attribute__((amdgpu_waves_per_eu(3, 8)))
void ransac_dk_kernel(GeomArgs g, int pairs, int pass, int budget) {
    // pass 0: items [0, dk_ctl[1]) of the round's work list; pass k > 0: dk_list[k - 1][0, dk_ctl[1 + k])
    const int total = g.dk_ctl[1 + pass];
    if ((int)blockIdx.x * kDkNT >= total) return;
    __shared__ double s_saved[20 * kDkNT];
    const int e = blockIdx.x * kDkNT + threadIdx.x;
    if (e >= total) return;
    const int item = pass == 0 ? e : g.dk_list[(int64_t)(pass - 1) * g.dk_list_cap + e];
    double* R = item_record(g, item);  // the item's record (no pair lookup: records are per item)
    if (pass == 0 && R[kRecGeneric * 64] != 0.0) return;  // stage C runs the generic solver
    double c[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) c[k] = R[(kRecC + k) * 64];
    Cx roots[10];
    DkBrent br;
    br.saved = s_saved + threadIdx.x;
    br.stride = kDkNT;
    if (pass == 0) {
        dk_init(roots);
        br.start(roots);
    } else {
#pragma unroll
        for (int i = 0; i < 10; i++) roots[i] = Cx{R[(kRecRoots + 2 * i) * 64], R[(kRecRoots + 2 * i + 1) * 64]};
#pragma unroll
        for (int k = 0; k < 20; ++k) br.saved[k * br.stride] = R[(kRecSnap + k) * 64];
        const int pk = (int)R[kRecNr * 64];
        br.it = pk & 511;
        br.saved_it = (pk >> 9) & 511;
        br.power = 1 << ((pk >> 18) & 15);
        br.target = (pk >> 22) & 511;
    }
    for (int sweep = 0;; ++sweep) {
        if (sweep == budget) {  // park for the next pass
#pragma unroll
            for (int i = 0; i < 10; i++) {
                R[(kRecRoots + 2 * i) * 64] = roots[i].re;
                R[(kRecRoots + 2 * i + 1) * 64] = roots[i].im;
            }
#pragma unroll
            for (int k = 0; k < 20; ++k) R[(kRecSnap + k) * 64] = br.saved[k * br.stride];
            R[kRecNr * 64] = (double)(br.it | br.saved_it << 9 | (31 - __clz(br.power)) << 18 | br.target << 22);
            const int slot = atomicAdd(&g.dk_ctl[2 + pass], 1);
            g.dk_list[(int64_t)pass * g.dk_list_cap + slot] = item;
            DK_STAT(pass, sweep);
            return;
        }
        bool moved, same = false;
        dk_sweep<false>(c, roots, moved, same);
        if (same) {  // coincident roots: stage C redoes this polynomial exactly
            R[kRecGeneric * 64] = 2.0;
            DK_STAT(pass, sweep + 1);
            return;
        }
        if (br.step(roots, moved)) {
            dk_store(R, roots);
            DK_STAT(pass, sweep + 1);
            return;
        }
    }
}

// Durand-Kerner with one lane per root, for rounds with few polynomials (the
// per-call findEssentialMat of the drop-in surface: at most a few thousand
// polynomials, so the one-lane kernel's ~1,750-instruction sweep on a single
// wave per SIMD is the whole latency).  A 16-lane row holds one polynomial,
// lane r < 10 owns root r and keeps a copy of all ten.  A sweep is the same
// Gauss-Seidel order as dk_sweep: every lane forms its numerator (Horner at its
// still-old root) at once; then for t = 0..9 lane t completes its denominator
// with the old roots t+1..9, divides and updates, the new root t is broadcast
// to the row (DPP row_newbcast), and the lanes r > t multiply in their factor
// (z_r - z_t new) -- each lane's product is the reference's left-to-right chain
// over j = 0..9, j != r.  Bit-identical to dk_sweep; per sweep ~2x fewer
// instructions on the critical wave.  Runs a polynomial to the end (Brent exit,
// no parking), as pass 0 of a round.
template <int T>
__device__ __forceinline__ double row_bcast(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x150 + T, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x150 + T, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Only lane T's own work sits inside the masked block: its old-root factors
// d[j] = z_T - z_j (j > T, still old at step T) are formed by every lane at the
// start of the sweep, and the moved / zero tests run once after the sweep.
template <int T>
__device__ __forceinline__ void dkw_step(const Cx& num, Cx& den, Cx& mine, Cx (&roots)[10], const Cx (&d)[10], int r,
                                         Cx& q) {
    if constexpr (T < 10) {
        if (r == T) {
#pragma unroll
            for (int j = T + 1; j < 10; ++j) den = cmul(den, d[j]);
            q = cdiv(num, den);
            mine = csub(mine, q);
        }
        roots[T] = Cx{row_bcast<T>(mine.re), row_bcast<T>(mine.im)};
        if (r > T) den = cmul(den, csub(mine, roots[T]));
        dkw_step<T + 1>(num, den, mine, roots, d, r, q);
    }
}

__global__ __launch_bounds__(64) void ransac_dk_wide_kernel(GeomArgs g, int pairs) {
    const int lane = threadIdx.x, r = lane & 15, rowbase = lane & ~15;
    const int total = g.dk_ctl[1];
    const int item = blockIdx.x * 4 + (lane >> 4);
    bool active = item < total;
    double* R = nullptr;
    if (active) {
        R = item_record(g, item);
        active = R[kRecGeneric * 64] == 0.0;  // else stage C runs the generic solver
    }
    if (__ballot(active) == 0) return;
    double c[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) c[k] = active ? R[(kRecC + k) * 64] : 1.0;
    Cx roots[10];
    dk_init(roots);
    Cx mine = roots[0];
#pragma unroll
    for (int k = 1; k < 10; ++k)
        if (r == k) mine = roots[k];
    Cx saved = mine;  // DkBrent::start
    int it = 0, saved_it = 0, power = 1, target = 300;
    const unsigned long long own = 0x3FFull << rowbase;  // the row's root lanes
    for (;;) {
        if (__ballot(active) == 0) break;
        // one sweep (every lane runs it; finished rows' results are ignored)
        Cx num{c[10], 0};
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const Cx t = cmul(num, mine);
            num = Cx{t.re + c[10 - j - 1], t.im + 0.0};
        }
        Cx d[10];
#pragma unroll
        for (int j = 0; j < 10; j++) d[j] = csub(mine, roots[j]);
        Cx den{c[10], 0}, q{0, 0};
        dkw_step<0>(num, den, mine, roots, d, r, q);
        // lane r's den is final after its own step (later steps only touch lanes r > T)
        const bool zero_l = !(den.re != 0 || den.im != 0) || den.re != den.re || den.im != den.im;
        const bool moved_l = (q.re * q.re + q.im * q.im) > 0;
        const bool moved = (__ballot(moved_l && r < 10) & own) != 0;
        const bool same = (__ballot(zero_l && r < 10) & own) != 0;
        const bool eq_l = __builtin_bit_cast(long long, mine.re) == __builtin_bit_cast(long long, saved.re) &&
                          __builtin_bit_cast(long long, mine.im) == __builtin_bit_cast(long long, saved.im);
        const bool eq = (__ballot(eq_l || r >= 10) & own) == own;
        if (!active) continue;
        if (same) {  // coincident roots: stage C redoes this polynomial exactly
            if (r == 0) R[kRecGeneric * 64] = 2.0;
            active = false;
            continue;
        }
        // DkBrent::step, identical in the row's lanes
        ++it;
        bool done = !moved || it >= target;
        if (!done && target == 300) {
            if (eq) {
                target = it + (300 - it) % (it - saved_it);
                done = it >= target;
            } else if (it - saved_it == power) {
                saved = mine;
                saved_it = it;
                power <<= 1;
            }
        }
        if (done) {
            if (r < 10) {
                const double im = fabs(mine.im) < 1e-100 ? 0.0 : mine.im;  // dk_finish
                R[(kRecRoots + 2 * r) * 64] = mine.re;
                R[(kRecRoots + 2 * r + 1) * 64] = im;
            }
            if (r == 0) R[kRecNr * 64] = 10;
            active = false;
        }
    }
}

// Stage C of every hypothesis of the round: models and their count.
__global__ __launch_bounds__(kSolveNT) void ransac_stage_c_kernel(GeomArgs g, int pairs) {
    const int e0 = blockIdx.x * kSolveNT;
    if (e0 >= g.dk_off[pairs]) return;
    const int e = e0 + threadIdx.x;
    const int p = wave_item_pair(g.dk_off, pairs, e0, e);
    if (e >= g.dk_off[pairs]) return;
    const int h = g.rs[p].h0 + (e - g.dk_off[p]);
    g.nmod[(int64_t)p * g.hyp_cap + h] =
        fp_stage_c(hyp_record(g, p, h), g.models + ((int64_t)p * g.hyp_cap + h) * 90);
}

// Stage C for rounds with few hypotheses (the per-call findEssentialMat): one
// 16-lane row per hypothesis, lane i builds the model of root i, so a
// hypothesis costs one 3x3 SVD of latency instead of one per real root.  The
// models keep the root order of fp_stage_c (a ballot prefix over the row).
__global__ __launch_bounds__(64) void ransac_stage_c_row_kernel(GeomArgs g) {
    const int p = blockIdx.y;
    const RansacState& S = g.rs[p];
    const int lane = threadIdx.x, r = lane & 15, rowbase = lane & ~15;
    const int h = S.h0 + blockIdx.x * 4 + (lane >> 4);
    const bool act = h < S.h1;
    double* R = act ? hyp_record(g, p, h) : nullptr;
    int nr = 0;
    double zre = 0, zim = 0;
    if (act) {
        const double gen = R[kRecGeneric * 64];
        if (gen == 0.0) {
            nr = (int)R[kRecNr * 64];
            if (r < nr) {
                zre = R[(kRecRoots + 2 * r) * 64];
                zim = R[(kRecRoots + 2 * r + 1) * 64];
            }
        } else {  // every lane of the row solves (same inputs, same roots); lane 0 records them
            double c[11];
            Cx roots[10];
#pragma unroll
            for (int k = 0; k < 11; ++k) c[k] = R[(kRecC + k) * 64];
            if (gen == 2.0) {
                solve_poly10(c, roots);
                dk_finish(roots);
                nr = 10;
            } else {
                nr = solve_poly_generic(c, 10, roots);
            }
            for (int i = 0; i < nr; ++i)
                if (i == r) {
                    zre = roots[i].re;
                    zim = roots[i].im;
                }
            if (r == 0) {
                for (int i = 0; i < nr; ++i) {
                    R[(kRecRoots + 2 * i) * 64] = roots[i].re;
                    R[(kRecRoots + 2 * i + 1) * 64] = roots[i].im;
                }
                R[kRecNr * 64] = nr;
            }
        }
    }
    bool valid = false;
    double e[9];
    if (act && r < nr && !(fabs(zim) > 1e-10)) {
        double b[39], EE[36];
#pragma unroll
        for (int k = 0; k < 39; ++k) b[k] = R[(kRecB + k) * 64];
#pragma unroll
        for (int k = 0; k < 36; ++k) EE[k] = R[(kRecEE + k) * 64];
        valid = root_model(b, EE, zre, e);
    }
    const uint32_t rowbits = (uint32_t)(__ballot(valid) >> rowbase) & 0xFFFFu;
    if (valid) {
        double* out = g.models + ((int64_t)p * g.hyp_cap + h) * 90 + __popc(rowbits & ((1u << r) - 1u)) * 9;
#pragma unroll
        for (int k = 0; k < 9; ++k) out[k] = e[k];
    }
    if (act && r == 0) g.nmod[(int64_t)p * g.hyp_cap + h] = __popc(rowbits);
}

// Inlier counts of every root of HYPS hypotheses of one pair; the pair's
// normalised points stream through LDS in chunks, one wave per model.
// HYPS = kScoreHyps for batches; the per-call path (one pair) takes kScoreHypsCall
// so that its few blocks spread over more CUs (fewer models per wave in sequence).
template <int HYPS>
__global__ __launch_bounds__(kScoreNT) void ransac_score_kernel(GeomArgs g, int pairs) {
    const int b = blockIdx.x;
    if (b >= g.s_off[pairs]) return;
    const int p = pair_of(g.s_off, pairs, b);
    const RansacState& S = g.rs[p];
    const int hb = S.h0 + (b - g.s_off[p]) * HYPS;
    if (hb >= S.h1 || S.m <= 5) return;
    const int hn = min(HYPS, S.h1 - hb);
    const int m = S.m;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    __shared__ int s_pref[HYPS + 1];
    __shared__ int s_cnt[HYPS * 10];
    __shared__ float4 s_ptf[kScoreChunk];
    __shared__ float s_sf[HYPS * 10][12];  // SampsonF32 of each model: e[9], mk, ok
    __shared__ int s_moff[HYPS * 10];      // the model's offset in g.models (the f64 test)
    __shared__ uint32_t s_und[kScoreUnd];  // deferred f64 tests: model << 16 | point, ~0u = void slot
    __shared__ int s_nund;
    __shared__ int s_pend[HYPS * 10];      // deferred tests per model (possible inliers not yet counted)
    const int64_t hbase = (int64_t)p * g.hyp_cap + hb;
    static_assert(HYPS < 64, "one wave prefixes the model counts; lane hn (< 64) writes the total");
    if (tid < 64) {  // model counts of the block's hypotheses: one load each, a wave prefix sum
        const int c = tid < hn ? g.nmod[hbase + tid] : 0;
        int x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (tid <= hn) s_pref[tid] = x - c;
    }
    if (tid == 0) s_nund = 0;
    __syncthreads();
    const int T = s_pref[hn];
    for (int e = tid; e < T; e += kScoreNT) s_cnt[e] = 0;
    for (int e = tid; e < T; e += kScoreNT) s_pend[e] = 0;
    const int bail = max(S.maxgood, 4);  // a final count <= bail never changes the replay
    const double thr = g.threshold / ((g.fx + g.fy) / 2);
    const float t = (float)(thr * thr);
    const bool fast_ok = t >= FLT_MIN;  // the division-free test needs t normal
    for (int e = tid; e < T; e += kScoreNT) {  // once per model, not per chunk
        int h = 0;
        while (h + 1 < hn && s_pref[h + 1] <= e) ++h;
        const int off = (int)((hbase + h) * 90 + (e - s_pref[h]) * 9 - hbase * 90);
        s_moff[e] = off;
        double Ed[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) Ed[k] = g.models[hbase * 90 + off + k];
        const SampsonF32 sf(Ed, fast_ok);
#pragma unroll
        for (int k = 0; k < 9; ++k) s_sf[e][k] = sf.e[k];
        s_sf[e][9] = sf.mk;
        s_sf[e][10] = sf.ok ? 1.f : 0.f;
    }
    const double* npts = g.npts + (int64_t)p * g.pts_stride * 4;
    for (int c0 = 0; c0 < m; c0 += kScoreChunk) {
        const int cn = min(kScoreChunk, m - c0);
        __syncthreads();
        for (int e = tid; e < cn; e += kScoreNT) {
            const double* q = npts + (int64_t)(c0 + e) * 4;
            s_ptf[e] = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
        }
        __syncthreads();
        // one wave per model (2 or 4 models per wave pass over the chunk, reading each point
        // once, measured slower: 73.0 K vs 72.6 / 71.4 K frames/s, profiles/r02w_ab_score_dk.txt)
        for (int e = wid; e < T; e += kScoreNT / 64) {
            if (s_cnt[e] + s_pend[e] + (m - c0) <= bail) continue;  // wave-uniform: this wave's own model
            int cnt = 0;
            // undecided points (a sliver) are marked per lane and take the f64 test after the
            // chunk, only in the waves that have one
            SampsonF32 sf;
#pragma unroll
            for (int k = 0; k < 9; ++k) sf.e[k] = s_sf[e][k];
            sf.mk = s_sf[e][9];
            sf.ok = s_sf[e][10] != 0.f;
            uint32_t umask = 0;
#pragma unroll
            for (int k = 0; k < kScoreChunk / 64; ++k) {
                const int j = lane + 64 * k;
                if (64 * k >= cn) break;  // wave-uniform
                const float4 pf = s_ptf[min(j, cn - 1)];
                const int d = j < cn ? sf.decide(pf.x, pf.y, pf.z, pf.w, t) : 0;
                cnt += __popcll(__ballot(d == 1));
                umask |= (uint32_t)(d < 0) << k;
            }
            if (m <= 0x10000 && __ballot(umask != 0)) {  // list the chunk's undecided points for the block's f64 pass
#pragma unroll
                for (int k = 0; k < kScoreChunk / 64; ++k) {
                    const bool u = (umask >> k) & 1u;
                    const unsigned long long bits = __ballot(u);
                    if (bits == 0) continue;  // wave-uniform
                    const int n = __popcll(bits);
                    int base = 0;
                    if (lane == 0) base = atomicAdd(&s_nund, n);
                    base = __shfl(base, 0);
                    const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                               (uint32_t)(bits >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bits, 0u));
                    if (base + n <= kScoreUnd) {
                        if (u) s_und[pos] = (uint32_t)e << 16 | (uint32_t)(c0 + lane + 64 * k);
                        if (lane == 0) s_pend[e] += n;
                        umask &= ~(1u << k);
                    } else if (u && pos < kScoreUnd) {
                        s_und[pos] = ~0u;  // the reservation straddles the end: its slots stay void
                    }
                }
            }
            if (__ballot(umask != 0)) {
                double Ed[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) Ed[k] = g.models[hbase * 90 + s_moff[e] + k];
                for (int k = 0; k < kScoreChunk / 64; ++k) {  // the f64 model and coordinates from L2
                    if (__ballot((umask >> k) & 1u) == 0) continue;  // wave-uniform: usually one k has any
                    bool in = false;
                    if ((umask >> k) & 1u) {
                        const double* pt = npts + (int64_t)(c0 + lane + 64 * k) * 4;
                        in = sampson_inlier(Ed, pt[0], pt[1], pt[2], pt[3], t, fast_ok);
                    }
                    cnt += __popcll(__ballot(in));
                }
            }
            if (lane == 0) s_cnt[e] += cnt;
        }
    }
    __syncthreads();
    {  // the block's deferred f64 tests, all at once
        const int nu = min(s_nund, kScoreUnd);
        for (int u = tid; u < nu; u += kScoreNT) {
            const uint32_t w = s_und[u];
            if (w == ~0u) continue;
            const int e = (int)(w >> 16), j = (int)(w & 0xFFFFu);
            double Ed[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) Ed[k] = g.models[hbase * 90 + s_moff[e] + k];
            const double* pt = npts + (int64_t)j * 4;
            if (sampson_inlier(Ed, pt[0], pt[1], pt[2], pt[3], t, fast_ok)) atomicAdd(&s_cnt[e], 1);
        }
        __syncthreads();
    }
    for (int e = tid; e < T; e += kScoreNT) {
        int h = 0;
        while (h + 1 < hn && s_pref[h + 1] <= e) ++h;
        g.cnt[(hbase + h) * 10 + (e - s_pref[h])] = s_cnt[e];
    }
}

// The sequential bookkeeping of RANSACPointSetRegistrator::run over this
// round's hypotheses, in order:
//   for each hypothesis while iter < niters: for each of its models:
//     if count > max(maxgood, 4): best = it, maxgood = count,
//                                 niters = RANSACUpdateNumIters(p, (m - count) / m, 5, niters)
// A model can only change the state when its count beats the running maximum
// of every count before it (and 4), so the wave finds those events in
// parallel (a block of hypotheses per lane, an exclusive prefix max across
// lanes) and lane 0 replays only the events, in order, with the stop rule:
// nothing changes niters between events, so the loop ends at the first
// hypothesis at or past niters.  Identical to the per-hypothesis loop
// (which remains for rounds with more events than the event list holds).
// kReplayMax: hypotheses per LDS chunk.  A pipelined round holds at most 32 / 32 / 64 / 128 hypotheses
// per pair before the last one, so chunks of 256 (12 KB of LDS: 13 blocks per CU) rarely split a
// round, where 1024 (46 KB: 3 blocks per CU) left the replay at under a wave per SIMD (RANSAC stage
// 13.8 vs 13.9-14.5 ms per two-stream step, frames/s within noise: profiles/r05s_ab_replay_dk_waves.txt).
#ifndef DVO_REPLAY_MAX
#define DVO_REPLAY_MAX 256
#endif
constexpr int kReplayNT = 64, kReplayMax = DVO_REPLAY_MAX, kReplayEv = 256;
__global__ __launch_bounds__(kReplayNT) void ransac_replay_kernel(GeomArgs g) {
    const int p = blockIdx.x;
    RansacState* Sp = g.rs + p;
    const int h0 = Sp->h0, h1 = Sp->h1;
    if (Sp->m <= 5 || h1 <= h0) return;
    __shared__ int s_nmod[kReplayMax];
    __shared__ int s_cnt[kReplayMax * 10];
    __shared__ int s_ev[kReplayEv];  // events: h << 4 | model
    __shared__ RansacState s_S;      // the state between chunks
    const int lane = threadIdx.x;
    const int64_t base = (int64_t)p * g.hyp_cap;
    if (lane == 0) s_S = *Sp;
    for (int h0c = h0; h0c < h1; h0c += kReplayMax) {  // hyp_cap > kReplayMax: chunked
        const int hn = min(kReplayMax, h1 - h0c);
        __syncthreads();
        for (int e = lane; e < hn; e += kReplayNT) s_nmod[e] = g.nmod[base + h0c + e];
        for (int e = lane; e < hn * 10; e += kReplayNT) s_cnt[e] = g.cnt[(base + h0c) * 10 + e];
        __syncthreads();
        const RansacState S = s_S;
        // lane's contiguous block of hypotheses, its max count, exclusive prefix max over lanes
        const int per = (hn + kReplayNT - 1) / kReplayNT;
        const int b0 = min(hn, lane * per), b1 = min(hn, b0 + per);
        int bmax = 0;
        for (int h = b0; h < b1; ++h)
            for (int i = 0; i < s_nmod[h]; ++i) bmax = max(bmax, s_cnt[h * 10 + i]);
        int pre = bmax;  // inclusive scan, then shift
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(pre, o);
            if (lane >= o) pre = max(pre, t);
        }
        int excl = __shfl_up(pre, 1);  // (shuffles stay in wave-uniform control flow)
        if (lane == 0) excl = 0;
        excl = max(excl, max(S.maxgood, 4));
        int run = excl;
        int nev = 0;
        for (int h = b0; h < b1; ++h)
            for (int i = 0; i < s_nmod[h]; ++i) {
                const int c = s_cnt[h * 10 + i];
                if (c > run) {
                    run = c;
                    ++nev;
                }
            }
        int off = nev;  // exclusive prefix sum of the event counts
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(off, o);
            if (lane >= o) off += t;
        }
        const int total = __shfl(off, 63);
        off -= nev;
        if (total <= kReplayEv && nev > 0) {
            run = excl;
            for (int h = b0; h < b1; ++h)
                for (int i = 0; i < s_nmod[h]; ++i) {
                    const int c = s_cnt[h * 10 + i];
                    if (c > run) {
                        run = c;
                        s_ev[off++] = h << 4 | i;
                    }
                }
        }
        __syncthreads();
        if (lane == 0) {
            const int m = S.m;
            RansacState T = S;
            int niters = S.niters, maxgood = S.maxgood;
            int hdone = 0;  // hypotheses of this chunk processed
            if (total <= kReplayEv) {
                for (int e = 0; e < total; ++e) {
                    const int h = s_ev[e] >> 4, i = s_ev[e] & 15;
                    // niters is checked when a hypothesis starts, not between its models
                    if (h + 1 != hdone && S.iter + h >= niters) break;  // the loop ends before hypothesis h
                    const int good = s_cnt[h * 10 + i];
                    T.best_h = h0c + h;
                    T.best_i = i;
                    maxgood = good;
                    niters = ransac_update_num_iters(g.prob, (double)(m - good) / m, 5, niters);
                    hdone = h + 1;
                }
                hdone = max(hdone, min(hn, niters - S.iter));
            } else {
                int it = S.iter;
                for (int h = 0; h < hn && it < niters; ++h, ++it) {
                    for (int i = 0; i < s_nmod[h]; ++i) {
                        const int good = s_cnt[h * 10 + i];
                        if (good > (maxgood > 4 ? maxgood : 4)) {
                            T.best_h = h0c + h;
                            T.best_i = i;
                            maxgood = good;
                            niters = ransac_update_num_iters(g.prob, (double)(m - good) / m, 5, niters);
                        }
                    }
                }
                hdone = it - S.iter;
            }
            T.iter = S.iter + hdone;
            T.niters = niters;
            T.maxgood = maxgood;
            s_S = T;
            *Sp = T;
        }
    }
}

// E, info and the optional inlier mask of each pair.
__global__ __launch_bounds__(256) void ransac_finish_kernel(GeomArgs g) {
    const int p = blockIdx.x;
    const RansacState S = g.rs[p];
    int32_t* info = g.info + (int64_t)p * 4;
    double* E_out = g.E + (int64_t)p * 90;
    const int m = S.m;
    const int64_t base = (int64_t)p * g.hyp_cap;
    if (m < 5) {
        if (threadIdx.x == 0) {
            info[0] = info[1] = info[2] = 0;
            info[3] = DVO_EFEWPTS;
        }
        return;
    }
    if (m == 5) {
        const int k = g.nmod[base];
        if (threadIdx.x == 0) {
            info[0] = 3 * k;
            info[1] = k > 0 ? 5 : 0;
            info[2] = 1;
            info[3] = k > 0 ? DVO_OK : DVO_ENOMODEL;
        }
        for (int e = threadIdx.x; e < k * 9; e += 256) E_out[e] = g.models[base * 90 + e];
        if (g.mask && k > 0 && threadIdx.x < 5) g.mask[(int64_t)p * g.pts_stride + threadIdx.x] = 1;
        return;
    }
    const int maxgood = S.maxgood;
    if (threadIdx.x == 0) {
        info[0] = maxgood > 0 ? 3 : 0;
        info[1] = maxgood;
        info[2] = S.iter;
        info[3] = maxgood > 0 ? DVO_OK : DVO_ENOMODEL;
    }
    if (maxgood <= 0) return;
    const double* Eb = g.models + (base + S.best_h) * 90 + S.best_i * 9;
    if (threadIdx.x < 9) E_out[threadIdx.x] = Eb[threadIdx.x];
    if (g.mask) {
        double Ed[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) Ed[k] = Eb[k];
        const double thr = g.threshold / ((g.fx + g.fy) / 2);
        const float t = (float)(thr * thr);
        const double* npts = g.npts + (int64_t)p * g.pts_stride * 4;
        for (int j = threadIdx.x; j < m; j += 256) {
            const double* pt = npts + (int64_t)j * 4;
            g.mask[(int64_t)p * g.pts_stride + j] = sampson_inlier(Ed, pt[0], pt[1], pt[2], pt[3], t, t >= FLT_MIN);
        }
    }
}

// Upper bounds of one round's work (host): the hypotheses a set at round r can take are
// [bound[r-1], bound[r]) clamped to the cap, so the grids of a launch are sized from its spec.
struct RoundWork {
    int64_t items, ablocks, sblocks;
};
static RoundWork round_work(const RoundSpec& spec, int cap, int sh) {
    RoundWork w{0, 0, 0};
    for (int k = 0; k < spec.nsets; ++k) {
        const int r = spec.round[k];
        if (r < 0) continue;
        const int lo = r == 0 ? 0 : min(spec.bound[r - 1], cap), hi = min(spec.bound[r], cap);
        const int span = max(0, hi - lo);
        w.items += (int64_t)spec.npairs[k] * span;
        w.ablocks += (int64_t)spec.npairs[k] * ((span + 63) / 64);
        w.sblocks += (int64_t)spec.npairs[k] * ((span + sh - 1) / sh);
    }
    return w;
}

// A stream's round of the largest total work: one set at each round (Buffers::fprec, dk_list).
static RoundSpec full_spec(int F) {
    RoundSpec sp{};
    sp.nsets = kRansacRounds;
    sp.F = F;
    for (int r = 0; r < kRansacRounds; ++r) {
        sp.round[r] = r;
        sp.npairs[r] = F;
        sp.bound[r] = kRansacBounds[r];
    }
    return sp;
}
int64_t round_blocks_bound(int F, int hyp_cap) { return round_work(full_spec(F), hyp_cap, kScoreHyps).ablocks; }
int64_t round_items_bound(int F, int hyp_cap) { return round_work(full_spec(F), hyp_cap, kScoreHyps).items; }

// One RANSAC round over the launch pairs [0, nsets F): sample -> plan -> stage A ->
// Durand-Kerner -> stage C -> score -> replay.  one (the per-call path, kStageOneRound): a
// single pair leaves the GPU idle, so it takes one round over every hypothesis up to maxIters
// (one Durand-Kerner tail instead of several), solved with one lane per root
// (ransac_dk_wide_kernel), stage C by rows, and small score blocks.  Rounds only schedule the
// same hypotheses; the replay's result is the same.
static hipError_t launch_round(const GeomArgs& g, const RoundSpec& spec, bool one, hipStream_t s) {
    const int pairs = spec.nsets * spec.F;
    if (pairs <= 0) return hipSuccess;
    const int sh = one ? kScoreHypsCall : kScoreHyps;
    const RoundWork w = round_work(spec, g.hyp_cap, sh);
    hipLaunchKernelGGL(ransac_sample_kernel, dim3(pairs), dim3(64), 0, s, g, spec);
    if (w.items == 0) return hipGetLastError();  // no pair of the launch can have a hypothesis
    hipLaunchKernelGGL(ransac_plan_kernel, dim3(1), dim3(1024), 0, s, g, pairs, sh);
    const dim3 agrid((unsigned)((w.items + kSolveNT - 1) / kSolveNT));
    hipLaunchKernelGGL(ransac_stage_a_kernel, agrid, dim3(kSolveNT), 0, s, g, pairs);
    if (one) {
        hipLaunchKernelGGL(ransac_dk_wide_kernel, dim3((unsigned)((w.items + 3) / 4)), dim3(64), 0, s, g, pairs);
        int span = 0;  // the per-call path: one set, round 0 up to the cap
        for (int k = 0; k < spec.nsets; ++k) span = max(span, min(spec.bound[0], g.hyp_cap));
        hipLaunchKernelGGL(ransac_stage_c_row_kernel, dim3((span + 3) / 4, pairs), dim3(64), 0, s, g);
        hipLaunchKernelGGL(ransac_score_kernel<kScoreHypsCall>, dim3((unsigned)w.sblocks), dim3(kScoreNT), 0, s, g,
                           pairs);
    } else {
        const dim3 dgrid((unsigned)((w.items + kDkNT - 1) / kDkNT));
        for (int pass = 0; pass < kDkPasses; ++pass)
            hipLaunchKernelGGL(ransac_dk_kernel, dgrid, dim3(kDkNT), 0, s, g, pairs, pass,
                               pass + 1 < kDkPasses ? kDkBudgets[pass] : 1 << 30);
#ifdef DVO_DK_STATS
        hipLaunchKernelGGL(dk_stats_kernel, dim3(1), dim3(1), 0, s, spec.round[0], (int)dgrid.x * (kDkNT / 64));
#endif
        hipLaunchKernelGGL(ransac_stage_c_kernel, agrid, dim3(kSolveNT), 0, s, g, pairs);
        hipLaunchKernelGGL(ransac_score_kernel<kScoreHyps>, dim3((unsigned)w.sblocks), dim3(kScoreNT), 0, s, g,
                           pairs);
    }
    hipLaunchKernelGGL(ransac_replay_kernel, dim3(pairs), dim3(kReplayNT), 0, s, g);
    return hipGetLastError();
}

hipError_t launch_ransac_round(const GeomArgs& g_all, const RoundSpec& spec, hipStream_t s) {
    return launch_round(g_all, spec, false, s);
}

// Every round of a batch of `pairs` back to back (one set), then E and info.
static hipError_t launch_ransac(const GeomArgs& g, int pairs, bool one, hipStream_t s) {
    RoundSpec sp{};
    sp.nsets = 1;
    sp.F = pairs;
    sp.npairs[0] = pairs;
    if (one) {
        sp.round[0] = 0;
        sp.bound[0] = 1 << 30;
        hipError_t e = launch_round(g, sp, true, s);
        if (e != hipSuccess) return e;
    } else {
        for (int r = 0; r < kRansacRounds; ++r) sp.bound[r] = kRansacBounds[r];
        for (int r = 0; r < kRansacRounds; ++r) {
            sp.round[0] = r;
            hipError_t e = launch_round(g, sp, false, s);
            if (e != hipSuccess) return e;
        }
    }
    hipLaunchKernelGGL(ransac_finish_kernel, dim3(pairs), dim3(256), 0, s, g);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ double det3(const double (&M)[3][3]) {
    return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
           M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

__device__ __forceinline__ void matmul3(const double (&A)[3][3], const double (&B)[3][3], double (&C)[3][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}

// triangulate.cpp icvTriangulatePoints for one correspondence (P rows 3x4).
__device__ __forceinline__ void triangulate_one(const double* P1, const double* P2, double x1, double y1, double x2,
                                                double y2, double (&X)[4]) {
    double A[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        A[0][k] = x1 * P1[8 + k] - P1[k];
        A[1][k] = y1 * P1[8 + k] - P1[4 + k];
        A[2][k] = x2 * P2[8 + k] - P2[k];
        A[3][k] = y2 * P2[8 + k] - P2[4 + k];
    }
    double At[4][4], W[4], Vt[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) At[r][k] = A[k][r];
    jacobi_svd<4, 4, 0, 4>(At, W, Vt);
#pragma unroll
    for (int k = 0; k < 4; ++k) X[k] = Vt[3][k];
}

// recoverPose in three launches: decomposeEssentialMat per pair (one thread
// each), then one thread per (point, decomposition) - 4M DLT triangulations
// per pair, a 4x4 Jacobi SVD each, spread over the whole GPU instead of one
// workgroup per pair - with per-wave ballot counts added into the pair's four
// totals (integers: order-free), then the tie-ordered pick.
constexpr int kPNT = 256;
constexpr int kPoseRec = 72;  // per pair: 4 P (3x4), R1, R2, t

// P of decomposition c (row-major 3x4) from the pair's record: [R1|t], [R2|t], [R1|-t], [R2|-t]
__global__ __launch_bounds__(64) void pose_decompose_kernel(GeomArgs g, int pairs) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= pairs) return;
    const int32_t* info = g.info + (int64_t)p * 4;
    int32_t* cnt = g.pose_cnt + (int64_t)p * 5;
    const bool ok = info[3] == DVO_OK && info[0] == 3;
    cnt[0] = ok;
    for (int c = 0; c < 4; ++c) cnt[1 + c] = 0;
    if (!ok) return;
    const double* E = g.E + (int64_t)p * 90;
    double At[3][3], W[3], Vt[3][3], U[3][3];
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) At[r][k] = E[k * 3 + r];
    jacobi_svd<3, 3, 3, 3>(At, W, Vt);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) U[r][c] = At[c][r];
    if (det3(U) < 0)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) U[r][c] *= -1.;
    if (det3(Vt) < 0)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Vt[r][c] *= -1.;
    const double Wm[3][3] = {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}};
    const double Wt[3][3] = {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}};
    double UW[3][3], R1[3][3], R2[3][3];
    matmul3(U, Wm, UW);
    matmul3(UW, Vt, R1);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, R2);
    double* P = g.pose_P + (int64_t)p * kPoseRec;
    for (int k = 0; k < 9; ++k) {  // the unnormalised R1, R2, t recoverPose returns
        P[48 + k] = R1[k / 3][k % 3];
        P[57 + k] = R2[k / 3][k % 3];
    }
    for (int k = 0; k < 3; ++k) P[66 + k] = U[k][2] + 0.0;
    for (int c = 0; c < 4; ++c) {
        const double(&Rs)[3][3] = (c & 1) ? R2 : R1;
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) P[c * 12 + r * 4 + k] = Rs[r][k] + 0.0;
            const double tv = U[r][2] + 0.0;
            P[c * 12 + r * 4 + 3] = c < 2 ? tv + 0.0 : 0.0 - tv;
        }
    }
}

// One thread per (point, rotation c in {0, 1}): decompositions c ([R_c|t]) and c + 2 ([R_c|-t])
// from ONE triangulation (round 4: recoverPose 1.20 -> 0.62 ms one-stream,
// profiles/r04m_ab_pose_mirror.txt; tests/test_pose_mirror.py checks the identity on the
// oracle's Jacobi SVD).  Their DLT matrices differ only in column 3, negated
// (row 0-1 entries are zeros, t's entries are exact negations: t + 0.0 and 0.0 - t), and the
// Jacobi SVD keeps that mirror exactly: a rotation pairing column 3 with another sees -p, hence
// -s with the same c, and every later value is the exact negation (IEEE rounding is symmetric;
// only the signs of exact zeros can differ).  So the c + 2 null vector is sigma (X0, X1, X2, -X3),
// sigma = +-1, and its tests are those of c with X2 X3, q = X / X3 and z negated.  A zero X3
// (q infinite: a zero's sign would matter) or a zero component of t takes the c + 2 SVD itself.
__device__ __forceinline__ bool pose_tests(const double (&X)[4], const double* Pl, double dist, bool mirror) {
    if (!mirror) {
        bool ok = X[2] * X[3] > 0;
        const double q0 = X[0] / X[3], q1 = X[1] / X[3], q2 = X[2] / X[3], q3 = X[3] / X[3];
        ok = (q2 < dist) && ok;
        const double z = Pl[8] * q0 + Pl[9] * q1 + Pl[10] * q2 + Pl[11] * q3;
        ok = (z > 0) && ok;
        return (z < dist) && ok;
    }
    // X, Pl of the +t decomposition; the tests of the -t one (see above)
    bool ok = -(X[2] * X[3]) > 0;
    const double q0 = X[0] / X[3], q1 = X[1] / X[3], q2 = X[2] / X[3], q3 = X[3] / X[3];
    ok = (-q2 < dist) && ok;
    const double z = Pl[8] * q0 + Pl[9] * q1 + Pl[10] * q2 + Pl[11] * q3;
    ok = (-z > 0) && ok;
    return (-z < dist) && ok;
}

__global__ __launch_bounds__(kPNT) void pose_count_kernel(GeomArgs g) {
    const int p = blockIdx.y;
    int32_t* cnt = g.pose_cnt + (int64_t)p * 5;
    if (!cnt[0]) return;
    const int m = pair_m(g, p);
    const int w = blockIdx.x * kPNT + threadIdx.x;
    if ((int)blockIdx.x * kPNT >= 2 * m) return;
    const int c = w & 1, i = w >> 1;
    bool ok = false, ok2 = false;  // decompositions c and (mirror) c + 2
    if (i < m) {
        const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        const double* Pc = g.pose_P + (int64_t)p * kPoseRec + c * 12;
        double Pl[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) Pl[k] = Pc[k];
        const double* pt = g.npts + ((int64_t)p * g.pts_stride + i) * 4;
        double X[4];
        triangulate_one(P0, Pl, pt[0], pt[1], pt[2], pt[3], X);
        ok = pose_tests(X, Pl, g.dist_thresh, false);
        const int64_t mi = (int64_t)p * g.pts_stride + i;
        uint8_t mv = ok ? 255 : 0;
        if (g.mask_in) mv &= g.mask_in[mi];  // bitwise_and(mask, mask_c)
        ok = mv != 0;
        if (g.pose_mask) g.pose_mask[mi * 4 + c] = mv;
        if (X[3] != 0 && Pl[3] != 0 && Pl[7] != 0 && Pl[11] != 0) {
            ok2 = pose_tests(X, Pl, g.dist_thresh, true);
        } else {  // the c + 2 decomposition's own triangulation
#pragma unroll
            for (int k = 0; k < 12; ++k) Pl[k] = Pc[24 + k];
            triangulate_one(P0, Pl, pt[0], pt[1], pt[2], pt[3], X);
            ok2 = pose_tests(X, Pl, g.dist_thresh, false);
        }
        uint8_t mv2 = ok2 ? 255 : 0;
        if (g.mask_in) mv2 &= g.mask_in[mi];
        ok2 = mv2 != 0;
        if (g.pose_mask) g.pose_mask[mi * 4 + c + 2] = mv2;
    }
    const unsigned long long b0 = __ballot(ok), b2 = __ballot(ok2);  // lane l: decompositions l & 1, (l & 1) + 2
    const int lane = threadIdx.x & 63;
    if (lane < 4) {
        const unsigned long long bal = lane < 2 ? b0 : b2;
        const int n = __popcll(bal & (0x5555555555555555ull << (lane & 1)));
        if (n) atomicAdd(&cnt[1 + lane], n);
    }
}

__global__ __launch_bounds__(64) void pose_pick_kernel(GeomArgs g, int pairs) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= pairs) return;
    const int32_t* cnt = g.pose_cnt + (int64_t)p * 5;
    if (!cnt[0]) {
        g.good[p] = 0;
        if (g.pick) g.pick[p] = -1;
        return;
    }
    const int* gd = cnt + 1;
    int pick;
    if (gd[0] >= gd[1] && gd[0] >= gd[2] && gd[0] >= gd[3]) pick = 0;
    else if (gd[1] >= gd[0] && gd[1] >= gd[2] && gd[1] >= gd[3]) pick = 1;
    else if (gd[2] >= gd[0] && gd[2] >= gd[1] && gd[2] >= gd[3]) pick = 2;
    else pick = 3;
    const double* P = g.pose_P + (int64_t)p * kPoseRec;
    double* Rt = g.Rt + (int64_t)p * 12;
    for (int k = 0; k < 9; ++k) Rt[k] = P[(pick & 1 ? 57 : 48) + k];
    for (int k = 0; k < 3; ++k) Rt[9 + k] = pick < 2 ? P[66 + k] : 0.0 - P[66 + k];
    g.good[p] = gd[pick];
    if (g.pick) g.pick[p] = pick;
}

__global__ void triangulate_kernel(const double* P, const double* x, int k, double* X) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= k) return;
    double out[4];
    triangulate_one(P, P + 12, x[i], x[k + i], x[2 * k + i], x[3 * k + i], out);
#pragma unroll
    for (int r = 0; r < 4; ++r) X[r * k + i] = out[r];
}

// The frame-side values of each pair's record, kept with the pair's set (PairHeader).
__global__ void pair_header_kernel(StreamParams P, PairHeader* hdr) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= stream_pairs(P)) return;
    const int fp = pair_frame(P, p);  // the pair's frames are fp, fp + 1
    hdr[p] = PairHeader{P.buf.nkp[fp], P.buf.nkp[fp + 1], P.buf.status[fp] | P.buf.status[fp + 1], 0};
}

__global__ void records_kernel(GeomArgs g, const PairHeader* hdr, int pairs, dvo_pair_record* rec) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= pairs) return;
    dvo_pair_record r;
    const int32_t* info = g.info + (int64_t)p * 4;
    const double* E = g.E + (int64_t)p * 90;
    const double* Rt = g.Rt + (int64_t)p * 12;
    const PairHeader h = hdr[p];
    const bool ok = info[3] == DVO_OK && info[0] == 3;
    for (int k = 0; k < 9; ++k) r.R[k] = ok ? Rt[k] : 0.0;
    for (int k = 0; k < 3; ++k) r.t[k] = ok ? Rt[9 + k] : 0.0;
    for (int k = 0; k < 9; ++k) r.E[k] = info[0] >= 3 ? E[k] : 0.0;
    r.n_kp_prev = h.nkp_prev;
    r.n_kp_cur = h.nkp_cur;
    r.n_matches = g.m_arr[p];
    r.n_inliers = info[1];
    r.n_good = ok ? g.good[p] : 0;
    r.ransac_iters = info[2];
    // ECAP (a buffer overflowed) > ENOFEAT (an empty frame: the reference's
    // bf.match(None, ...) raises, v3:219) > the RANSAC / pose status.
    r.status = h.flags ? DVO_ECAP : (h.nkp_prev == 0 || h.nkp_cur == 0) ? DVO_ENOFEAT : info[3];
    r.n_models = info[0] / 3;
    r.n_hypotheses = g.rs[p].h1;  // hypotheses [0, h1) were sampled and solved
    r.pad0 = 0;
    for (int k = 0; k < 6; ++k) r.reserved[k] = 0.0;
    rec[p] = r;
}

// ---- pose tail (visual_odometry_v3.py:309-345, :367) -------------------------
// Gohlke euler_from_matrix(M, 'rxyz') -> (ax, ay, az); rxyz = (firstaxis 2,
// parity 1, repetition 0, frame 1): i=2, j=1, k=0.
__device__ void euler_from_matrix_rxyz(const double* R, double& ax, double& ay, double& az) {
    const int i = 2, j = 1, k = 0;
    auto M = [&](int r, int c) { return R[r * 3 + c]; };
    const double eps4 = 4.0 * DBL_EPSILON;
    double cy = sqrt(M(i, i) * M(i, i) + M(j, i) * M(j, i));
    if (cy > eps4) {
        ax = atan2(M(k, j), M(k, k));
        ay = atan2(-M(k, i), cy);
        az = atan2(M(j, i), M(i, i));
    } else {
        ax = atan2(-M(j, k), M(j, j));
        ay = atan2(-M(k, i), cy);
        az = 0.0;
    }
    ax = -ax;  // parity
    ay = -ay;
    az = -az;
    double t = ax;  // frame
    ax = az;
    az = t;
}

// Gohlke euler_matrix(ai, aj, ak, 'sxyz') (i=0, j=1, k=2, no parity/repetition/frame).
__device__ void euler_matrix_sxyz(double ai, double aj, double ak, double* M /*4x4*/) {
    double si = sin(ai), sj = sin(aj), sk = sin(ak);
    double ci = cos(ai), cj = cos(aj), ck = cos(ak);
    double cc = ci * ck, cs = ci * sk, sc = si * ck, ss = si * sk;
    for (int r = 0; r < 16; ++r) M[r] = (r % 5 == 0) ? 1.0 : 0.0;
    M[0 * 4 + 0] = cj * ck;
    M[0 * 4 + 1] = sj * sc - cs;
    M[0 * 4 + 2] = sj * cc + ss;
    M[1 * 4 + 0] = cj * sk;
    M[1 * 4 + 1] = sj * ss + cc;
    M[1 * 4 + 2] = sj * cs - sc;
    M[2 * 4 + 0] = -sj;
    M[2 * 4 + 1] = cj * si;
    M[2 * 4 + 2] = cj * ci;
}

__device__ void proj_of(const double* K, const double* Rt, double* P) {  // K . [R | t]
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) {
            const double a0 = c < 3 ? Rt[0 * 3 + c] : Rt[9 + 0];
            const double a1 = c < 3 ? Rt[1 * 3 + c] : Rt[9 + 1];
            const double a2 = c < 3 ? Rt[2 * 3 + c] : Rt[9 + 2];
            P[r * 4 + c] = K[r * 3 + 0] * a0 + K[r * 3 + 1] * a1 + K[r * 3 + 2] * a2;
        }
}

struct TailArgs {
    const dvo_pair_record* rec;  // R (9) and t (3) are the record's first 12 doubles: the [R | t] layout
    int pairs;
    int p0;          // pose_tail_kernel: pairs [p0, pairs) of rec, T_rel[p - p0] (0: the whole window)
    double K[9];
    const double* cprev;
    const double* ccur;
    int k;
    double L;
    double* carry;   // P_prev carry (12 doubles); null for a chain-only launch
    double* tcarry;  // T_abs carry (16 doubles): in = pose before the first pair, out = after the last
    double* T_rel;
    double* T_abs;
};

// A pair the reference gets through to the pose tail: findEssentialMat returned
// exactly one E and recoverPose ran (status DVO_OK, one model).  Every other
// record is a pair where the reference raises before v3:344.
__device__ inline bool rec_ok(const dvo_pair_record* rec, int p) {
    return rec[p].status == DVO_OK && rec[p].n_models == 1;
}
__device__ inline const double* rec_Rt(const dvo_pair_record* rec, int p) { return rec[p].R; }

// P_prev carry after a window of records: the projection of its last successful pair (unchanged
// when none succeeded), as pose_chain_kernel leaves it.
__global__ __launch_bounds__(1024) void pose_carry_kernel(TailArgs a) {
    __shared__ int s_last[16];
    int last_ok = -1;
    for (int p = a.pairs - 1 - (int)threadIdx.x; p >= 0 && last_ok < 0; p -= 1024)  // from the end
        if (rec_ok(a.rec, p)) last_ok = p;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) last_ok = max(last_ok, __shfl_xor(last_ok, o));
    if ((threadIdx.x & 63) == 0) s_last[threadIdx.x >> 6] = last_ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) last_ok = max(last_ok, s_last[w]);
        if (last_ok >= 0) proj_of(a.K, rec_Rt(a.rec, last_ok), a.carry);
    }
}

// The pose tail reads only the 256-B pair records (R, t, status), so a pose
// stream whose records were computed on several ranks and all-gathered gives
// the same result as one rank's (dvo_pose_tail_records).
__global__ void pose_tail_kernel(TailArgs a) {
    const int p = a.p0 + blockIdx.x * 64 + threadIdx.x;
    if (p >= a.pairs) return;
    double* Tr = a.T_rel + (int64_t)(p - a.p0) * 16;
    if (!rec_ok(a.rec, p)) {  // the reference would have raised here
        for (int r = 0; r < 16; ++r) Tr[r] = (r % 5 == 0) ? 1.0 : 0.0;
        return;
    }
    const double* Rt = rec_Rt(a.rec, p);
    double Pc[12], Pp[12];
    proj_of(a.K, Rt, Pc);
    // P_prev is the projection of the last pair that got through (the reference
    // sets previous_projection_matrix only at the end of a successful pair,
    // v3:344); the carry when no earlier pair of this batch did.
    int q = p - 1;
    while (q >= 0 && !rec_ok(a.rec, q)) --q;
    if (q < 0) {
        for (int r = 0; r < 12; ++r) Pp[r] = a.carry[r];
    } else {
        proj_of(a.K, rec_Rt(a.rec, q), Pp);
    }
    double X0[4], X1[4];
    const double* cp = a.cprev + (int64_t)p * a.k * 2;
    const double* cc = a.ccur + (int64_t)p * a.k * 2;
    triangulate_one(Pp, Pc, cp[0], cp[1], cc[0], cc[1], X0);
    triangulate_one(Pp, Pc, cp[2], cp[3], cc[2], cc[3], X1);
    const double dx = X0[0] - X1[0], dy = X0[1] - X1[1], dz = X0[2] - X1[2];
    const double d = sqrt(dx * dx + dy * dy + dz * dz);
    const double s = a.L / d;
    double ax, ay, az;
    euler_from_matrix_rxyz(Rt, ax, ay, az);
    double M[16];
    euler_matrix_sxyz(ax, ay, az, M);
    const double tx = Rt[9] * s, ty = Rt[10] * s, tz = Rt[11] * s;
    // translation_matrix(t) . M: rows 0..2 gain t * M[3][:] (M[3] = [0 0 0 1])
    for (int c = 0; c < 4; ++c) {
        Tr[0 * 4 + c] = M[0 * 4 + c] + tx * M[3 * 4 + c];
        Tr[1 * 4 + c] = M[1 * 4 + c] + ty * M[3 * 4 + c];
        Tr[2 * 4 + c] = M[2 * 4 + c] + tz * M[3 * 4 + c];
        Tr[3 * 4 + c] = M[3 * 4 + c];
    }
}

// Prefix product T_abs[p] = T_abs[p-1] . T_rel[p], in pair order, and the
// carry-out of P_prev / T_abs for the next batch.  The product is not
// associative in floating point, so the chain stays sequential (bit-identical
// to the scalar left-to-right 4x4 product); what is parallel is inside a step.
// Lane 4 r + c (of 16) keeps element (r, c) of the running pose; a step is that
// element's 4 products and 3 sums, ((t_r0 A_0c + t_r1 A_1c) + t_r2 A_2c) + t_r3 A_3c,
// with row r's four elements taken from the lane's quad by DPP quad_perm.  The
// dependency chain of a step is then one quad exchange and 4 dependent f64 ops
// (round 3 kept a whole row per lane: 28 f64 instructions issued per step).
// T_rel is staged through LDS 64 pairs at a time and read one step ahead.
// (Round 5, beside a full batch on the other streams: 1.5 us per step against 80 ns alone with
// LDS staging, wave priority 3 or registers only (profiles/r05j_*, r05k_*); rank 0 of a sharded
// run therefore chains on the host, dvo_pose_chain_host.)
template <int K>
__device__ __forceinline__ double quad_bcast(double v) {  // lane 4 q + K of the lane's quad
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    constexpr int ctl = K | (K << 2) | (K << 4) | (K << 6);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, ctl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), ctl, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
__global__ __launch_bounds__(64) void pose_chain_kernel(TailArgs a) {
    constexpr int kChunk = 64, kPer = kChunk * 16 / 64;  // T_rel doubles per lane and chunk
    __shared__ double tr[kChunk * 16];
    __shared__ double ob[kChunk * 16];  // the chunk's T_abs, stored to global memory coalesced
    const int lane = threadIdx.x;
    int last_ok = -1;
    if (a.rec) {
        for (int p = lane; p < a.pairs; p += 64)
            if (rec_ok(a.rec, p)) last_ok = p;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) last_ok = max(last_ok, __shfl_xor(last_ok, o));
    }
    const int e = lane & 15, c = e & 3;  // lanes 16..63 repeat lanes 0..15
    double t = a.tcarry[e];
    // the next chunk's T_rel in flight in registers while this chunk's steps run
    double nxt[kPer];
    auto fetch = [&](int p0) {
        const int n16 = min(kChunk, a.pairs - p0) * 16;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = lane + 64 * k;
            nxt[k] = i < n16 ? a.T_rel[(int64_t)p0 * 16 + i] : 0.0;
        }
    };
    if (a.pairs > 0) fetch(0);
    for (int p0 = 0; p0 < a.pairs; p0 += kChunk) {
        const int n = min(kChunk, a.pairs - p0);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; ++k) tr[lane + 64 * k] = nxt[k];
        __syncthreads();
        if (p0 + kChunk < a.pairs) fetch(p0 + kChunk);
        // software pipeline, unrolled by two so the two column buffers alternate without moves:
        // the column of step q + 1 is read from LDS while step q computes
        auto step = [&](int q, double C0, double C1, double C2, double C3) {
            const double t0 = quad_bcast<0>(t), t1 = quad_bcast<1>(t), t2 = quad_bcast<2>(t), t3 = quad_bcast<3>(t);
            t = t0 * C0 + t1 * C1 + t2 * C2 + t3 * C3;
            ob[q * 16 + e] = t;  // lanes e, e + 16, .. store the same value
        };
        double A0 = tr[c], A1 = tr[4 + c], A2 = tr[8 + c], A3 = tr[12 + c];
        int q = 0;
        for (; q + 1 < n; q += 2) {
            const int q1 = q + 1, q2 = min(q + 2, n - 1);
            const double B0 = tr[q1 * 16 + c], B1 = tr[q1 * 16 + 4 + c], B2 = tr[q1 * 16 + 8 + c],
                         B3 = tr[q1 * 16 + 12 + c];
            step(q, A0, A1, A2, A3);
            A0 = tr[q2 * 16 + c];
            A1 = tr[q2 * 16 + 4 + c];
            A2 = tr[q2 * 16 + 8 + c];
            A3 = tr[q2 * 16 + 12 + c];
            step(q1, B0, B1, B2, B3);
        }
        if (q < n) step(q, A0, A1, A2, A3);
        __syncthreads();
        for (int i = lane; i < n * 16; i += 64) a.T_abs[(int64_t)p0 * 16 + i] = ob[i];
    }
    if (lane < 16) a.tcarry[e] = t;
    if (lane == 0 && last_ok >= 0 && a.carry) proj_of(a.K, rec_Rt(a.rec, last_ok), a.carry);
}

__global__ void test_update_num_iters_kernel(double p, const double* ep, int n, int mp, int mi, int32_t* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = ransac_update_num_iters(p, ep[i], mp, mi);
}

__device__ double g_test_rec[kRecDoubles * 64];
__global__ __launch_bounds__(64) void test_five_point_kernel(const double* qin, double* models, int* n) {
    __shared__ double lds_g[36 * 64];
    if (threadIdx.x != 0) return;
    double q[5][4];
    for (int i = 0; i < 5; ++i)
        for (int k = 0; k < 4; ++k) q[i][k] = qin[i * 4 + k];
    *n = five_point(q, models, lds_g, g_test_rec);
}

hipError_t launch_geometry_args(const GeomArgs& g, int pairs, int stages, hipStream_t s) {
    if (pairs <= 0) return hipSuccess;
    if (stages & kStageNormalize) hipLaunchKernelGGL(normalize_kernel, dim3(4, pairs), dim3(256), 0, s, g);
    if (stages & kStageRansac) {
        hipError_t e = launch_ransac(g, pairs, (stages & kStageOneRound) != 0, s);
        if (e != hipSuccess) return e;
    }
    if (stages & kStagePose) {
        hipLaunchKernelGGL(pose_decompose_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, g, pairs);
        hipLaunchKernelGGL(pose_count_kernel, dim3((unsigned)((2 * g.pts_stride + kPNT - 1) / kPNT), pairs), dim3(kPNT), 0,
                           s, g);
        hipLaunchKernelGGL(pose_pick_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, g, pairs);
    }
    return hipGetLastError();
}

hipError_t launch_geometry(const StreamParams& P, const GeomArgs& g, dvo_pair_record* records, hipStream_t s,
                           hipEvent_t* ev, bool one_round) {
    const int pairs = stream_pairs(P);
    if (pairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(pair_header_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, P, P.buf.hdr);
    mark(ev, 6, 0, s);
    hipError_t e = launch_geometry_args(g, pairs, kStageNormalize | kStageRansac | (one_round ? kStageOneRound : 0), s);
    mark(ev, 6, 1, s);
    if (e != hipSuccess) return e;
    mark(ev, 7, 0, s);
    e = launch_geometry_args(g, pairs, kStagePose, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(records_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, g, P.buf.hdr, pairs, records);
    mark(ev, 7, 1, s);
    return hipGetLastError();
}

hipError_t launch_pair_header(const StreamParams& P, PairHeader* hdr, hipStream_t s) {
    const int pairs = stream_pairs(P);
    if (pairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(pair_header_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, P, hdr);
    return hipGetLastError();
}

// A set whose last round has run: E and info (findEssentialMat's result), recoverPose, the records.
hipError_t launch_retire(const GeomArgs& g_set, int pairs, const PairHeader* hdr, dvo_pair_record* records,
                         hipStream_t s) {
    if (pairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(ransac_finish_kernel, dim3(pairs), dim3(256), 0, s, g_set);
    hipError_t e = launch_geometry_args(g_set, pairs, kStagePose, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(records_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, g_set, hdr, pairs, records);
    return hipGetLastError();
}

hipError_t launch_triangulate(const double* d_P, const double* d_x, int k, double* d_X, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(triangulate_kernel, dim3((k + 255) / 256), dim3(256), 0, s, d_P, d_x, k, d_X);
    return hipGetLastError();
}

hipError_t launch_pose_tail(const dvo_pair_record* rec, int pairs, const double* K, const double* cprev,
                            const double* ccur, int k, double marker_length, double* carry, double* T_rel,
                            double* T_abs, hipStream_t s) {
    if (pairs <= 0) return hipSuccess;
    TailArgs a{};
    a.rec = rec;
    a.pairs = pairs;
    for (int i = 0; i < 9; ++i) a.K[i] = K[i];
    a.cprev = cprev;
    a.ccur = ccur;
    a.k = k;
    a.L = marker_length;
    a.carry = carry;
    a.tcarry = carry + 12;
    a.T_rel = T_rel;
    a.T_abs = T_abs;
    hipLaunchKernelGGL(pose_tail_kernel, dim3((pairs + 63) / 64), dim3(64), 0, s, a);
    hipLaunchKernelGGL(pose_chain_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pose_rel_range(const dvo_pair_record* rec, int pairs, int p0, int n, const double* K,
                                 const double* cprev, const double* ccur, int k, double marker_length, double* P_carry,
                                 double* T_rel, hipStream_t s) {
    TailArgs a{};
    a.rec = rec;
    a.pairs = p0 + n;
    a.p0 = p0;
    for (int i = 0; i < 9; ++i) a.K[i] = K[i];
    a.cprev = cprev;
    a.ccur = ccur;
    a.k = k;
    a.L = marker_length;
    a.carry = P_carry;
    a.T_rel = T_rel;
    if (n > 0) hipLaunchKernelGGL(pose_tail_kernel, dim3((n + 63) / 64), dim3(64), 0, s, a);
    a.pairs = pairs;  // the carry leaves the window at its last successful pair
    hipLaunchKernelGGL(pose_carry_kernel, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pose_chain(const double* T_rel, int n, double* T_carry, double* T_abs, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    TailArgs a{};
    a.pairs = n;
    a.tcarry = T_carry;
    a.T_rel = const_cast<double*>(T_rel);
    a.T_abs = T_abs;
    hipLaunchKernelGGL(pose_chain_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

// Test hooks: the sampler / replay kernels on one pair whose RansacState the
// caller set (api.cpp dvo_test_ransac_*).
hipError_t launch_test_ransac_sample(const GeomArgs& g, hipStream_t s) {
    RoundSpec sp{};  // one pair continuing (round 1) from the caller's state, no bound
    sp.nsets = 1;
    sp.F = 1;
    sp.round[0] = 1;
    sp.npairs[0] = 1;
    sp.bound[0] = sp.bound[1] = 1 << 30;
    hipLaunchKernelGGL(ransac_sample_kernel, dim3(1), dim3(64), 0, s, g, sp);
    return hipGetLastError();
}
hipError_t launch_test_ransac_replay(const GeomArgs& g, hipStream_t s) {
    hipLaunchKernelGGL(ransac_replay_kernel, dim3(1), dim3(kReplayNT), 0, s, g);
    return hipGetLastError();
}

hipError_t launch_test_update_num_iters(double p, const double* d_ep, int n, int model_points, int max_iters,
                                        int32_t* d_out, hipStream_t s) {
    hipLaunchKernelGGL(test_update_num_iters_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, d_ep, n, model_points,
                       max_iters, d_out);
    return hipGetLastError();
}

// SampsonF32 against sampson_inlier on one model and n points (test hook):
// dec[i] = the f32 decision (1 / 0 / -1 undecided), ex[i] = the f64 decision.
__global__ __launch_bounds__(256) void test_sampson_kernel(const double* E, const double* pts, int n, float t,
                                                           int8_t* dec, uint8_t* ex) {
    double Ed[9];
    for (int k = 0; k < 9; ++k) Ed[k] = E[k];
    const bool fast_ok = t >= FLT_MIN;
    const SampsonF32 sf(Ed, fast_ok);
    for (int i = threadIdx.x; i < n; i += 256) {
        const double* q = pts + (int64_t)i * 4;
        dec[i] = (int8_t)sf.decide((float)q[0], (float)q[1], (float)q[2], (float)q[3], t);
        ex[i] = sampson_inlier(Ed, q[0], q[1], q[2], q[3], t, fast_ok);
    }
}

hipError_t launch_test_sampson(const double* d_E, const double* d_pts, int n, float t, int8_t* d_dec, uint8_t* d_ex,
                               hipStream_t s) {
    hipLaunchKernelGGL(test_sampson_kernel, dim3(1), dim3(256), 0, s, d_E, d_pts, n, t, d_dec, d_ex);
    return hipGetLastError();
}

hipError_t launch_test_five_point(const double* d_q, double* d_models, int* d_n, hipStream_t s) {
    hipLaunchKernelGGL(test_five_point_kernel, dim3(1), dim3(64), 0, s, d_q, d_models, d_n);
    return hipGetLastError();
}

}  // namespace dvo
