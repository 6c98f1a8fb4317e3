// TEST INFRASTRUCTURE ONLY — CPU restatement of opencv_contrib's
// cv::xfeatures2d::SURF::detectAndCompute(img, None) with SURF_create(400)
// (hessianThreshold 400, nOctaves 4, nOctaveLayers 3, extended false, upright
// false): the detector of the reference's 'surf' mode
// (scripts/visual_odometry_v3.py:103-106, detectAndCompute at :373, knnMatch
// at :215).  Follows xfeatures2d/src/surf.cpp (integral, calcLayerDetAndTrace,
// findMaximaInLayer, interpolateKeypoint, KeypointGreater, SURFInvoker) and the
// INTER_AREA resize it calls (imgproc resize.cpp: computeResizeAreaTab,
// ResizeArea_Invoker, resizeAreaFast_Invoker with ResizeAreaFastVec).  Where
// OpenCV's result depends on the build this restatement fixes one definition,
// which the GPU kernels (csrc/surf.hip) follow operation for operation:
//   - float expressions unfused, left to right;
//   - getGaussianKernel = double exp, float taps, renormalised over the float
//     taps (the classic formula; OpenCV >= 4.2's bit-exact variant treats the
//     even n = 20 descriptor kernel as odd, opencv#15856);
//   - cv::phase / fastAtan2 = the scalar polynomial (no SIMD FMA);
//   - sin/cos of a float argument = double libm result rounded to float;
//   - INTER_AREA at an integer scale of 2 = (a + b + c + d + 2) >> 2 (the
//     ResizeAreaFastVec path), other integer scales cvRound(sum * (1.f/area)).
// Parity against OpenCV itself is unpinned (OpenCV is absent).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

constexpr int kOctaves = 4, kLayers = 3;        // nOctaves, nOctaveLayers
constexpr int kHaar0 = 9, kHaarInc = 6;         // SURF_HAAR_SIZE0, SURF_HAAR_SIZE_INC
constexpr int kOriRadius = 6, kOriWin = 60;     // SURFInvoker::ORI_RADIUS, ORI_WIN
constexpr int kOriInc = 5;                      // SURF_ORI_SEARCH_INC
constexpr float kOriSigma = 2.5f, kDescSigma = 3.3f;
constexpr int kPatch = 20;                      // PATCH_SZ

int cv_round(float v) { return (int)std::nearbyint(v); }
int cv_round_d(double v) { return (int)std::nearbyint(v); }
int cv_floor_d(double v) { return (int)std::floor(v); }
int cv_ceil_d(double v) { return (int)std::ceil(v); }

float fast_atan2_deg(float y, float x) {  // cv::fastAtan2, scalar
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

std::vector<float> gauss_kernel(int n, double sigma) {  // getGaussianKernel(n, sigma, CV_32F)
    std::vector<float> k(n);
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        k[i] = (float)std::exp(scale2X * x * x);
        sum += k[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) k[i] = (float)(k[i] * sum);
    return k;
}

struct HF {  // SurfHF
    int p0, p1, p2, p3;
    float w;
};

// resizeHaarPattern: a pattern defined at oldSize scaled to newSize
void resize_haar(const int src[][5], HF* dst, int n, int old_size, int new_size, int step) {
    const float ratio = (float)new_size / old_size;
    for (int k = 0; k < n; ++k) {
        const int dx1 = cv_round(ratio * src[k][0]), dy1 = cv_round(ratio * src[k][1]);
        const int dx2 = cv_round(ratio * src[k][2]), dy2 = cv_round(ratio * src[k][3]);
        dst[k].p0 = dy1 * step + dx1;
        dst[k].p1 = dy2 * step + dx1;
        dst[k].p2 = dy1 * step + dx2;
        dst[k].p3 = dy2 * step + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

float haar(const int32_t* o, const HF* f, int n) {  // calcHaarPattern
    double d = 0;
    for (int k = 0; k < n; ++k) d += (o[f[k].p0] + o[f[k].p3] - o[f[k].p1] - o[f[k].p2]) * f[k].w;
    return (float)d;
}

const int kDxS[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
const int kDyS[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
const int kDxyS[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};
const int kGxS[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
const int kGyS[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};

struct Layer {
    int size, step, rows, cols;
    std::vector<float> det, trace;
};

// calcLayerDetAndTrace; cells outside the sampled region stay 0 (OpenCV leaves
// them unwritten and never reads them)
void calc_layer(const std::vector<int32_t>& sum, int sw, int sh, Layer& L) {
    const int size = L.size, step = L.step;
    if (size > sh - 1 || size > sw - 1) return;
    HF Dx[3], Dy[3], Dxy[4];
    resize_haar(kDxS, Dx, 3, 9, size, sw);
    resize_haar(kDyS, Dy, 3, 9, size, sw);
    resize_haar(kDxyS, Dxy, 4, 9, size, sw);
    const int samples_i = 1 + (sh - 1 - size) / step, samples_j = 1 + (sw - 1 - size) / step;
    const int margin = (size / 2) / step;
    for (int i = 0; i < samples_i; ++i) {
        const int32_t* sp = sum.data() + (size_t)(i * step) * sw;
        for (int j = 0; j < samples_j; ++j, sp += step) {
            const float dx = haar(sp, Dx, 3), dy = haar(sp, Dy, 3), dxy = haar(sp, Dxy, 4);
            const size_t o = (size_t)(i + margin) * L.cols + (j + margin);
            L.det[o] = dx * dy - 0.81f * dxy * dxy;
            L.trace[o] = dx + dy;
        }
    }
}

// interpolateKeypoint: Matx33f(A).solve(b, DECOMP_LU) = Matx_FastSolveOp<3, 1>
bool interpolate(const float (&N9)[3][9], int dx, int dy, int ds, ora_keypoint& kp) {
    const float b0 = -(N9[1][5] - N9[1][3]) / 2, b1 = -(N9[1][7] - N9[1][1]) / 2, b2 = -(N9[2][4] - N9[0][4]) / 2;
    const float a00 = N9[1][3] - 2 * N9[1][4] + N9[1][5];
    const float a01 = (N9[1][8] - N9[1][6] - N9[1][2] + N9[1][0]) / 4;
    const float a02 = (N9[2][5] - N9[2][3] - N9[0][5] + N9[0][3]) / 4;
    const float a10 = a01;
    const float a11 = N9[1][1] - 2 * N9[1][4] + N9[1][7];
    const float a12 = (N9[2][7] - N9[2][1] - N9[0][7] + N9[0][1]) / 4;
    const float a20 = a02, a21 = a12;
    const float a22 = N9[0][4] - 2 * N9[1][4] + N9[2][4];
    float x0 = 0, x1 = 0, x2 = 0;
    float d = (float)(double)(a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11));
    if (d != 0) {
        d = 1 / d;
        x0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2));
        x1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) + a02 * (a10 * b2 - b1 * a20));
        x2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * (a10 * a21 - a11 * a20));
    }
    const bool ok = (x0 != 0 || x1 != 0 || x2 != 0) && std::abs(x0) <= 1 && std::abs(x1) <= 1 && std::abs(x2) <= 1;
    if (ok) {
        kp.x += x0 * dx;
        kp.y += x1 * dy;
        kp.size = (float)cv_round(kp.size + x2 * ds);
    }
    return ok;
}

bool kp_greater(const ora_keypoint& a, const ora_keypoint& b) {  // KeypointGreater
    if (a.response > b.response) return true;
    if (a.response < b.response) return false;
    if (a.size > b.size) return true;
    if (a.size < b.size) return false;
    if (a.octave > b.octave) return true;
    if (a.octave < b.octave) return false;
    if (a.y < b.y) return false;
    if (a.y > b.y) return true;
    return a.x < b.x;
}

// computeResizeAreaTab for one axis, as per-destination-cell runs:
// [left partial at s1 - 1] [full cells s1 .. s2-1] [right partial at s2]
struct AreaCell {
    int s1, s2, has_l, has_r;
    float al, af, ar;
};
void area_cells(int ssize, int dsize, double scale, AreaCell* c) {
    for (int dx = 0; dx < dsize; ++dx) {
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cell = std::min(scale, ssize - fsx1);
        int sx1 = cv_ceil_d(fsx1), sx2 = cv_floor_d(fsx2);
        sx2 = std::min(sx2, ssize - 1);
        sx1 = std::min(sx1, sx2);
        AreaCell& a = c[dx];
        a.s1 = sx1;
        a.s2 = sx2;
        a.has_l = sx1 - fsx1 > 1e-3;
        a.al = (float)((sx1 - fsx1) / cell);
        a.af = float(1.0 / cell);
        a.has_r = fsx2 - sx2 > 1e-3;
        a.ar = (float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell);
    }
}

// resize(win, patch, Size(21, 21), 0, 0, INTER_AREA) for a square 8-bit window
void resize_area21(const std::vector<uint8_t>& W, int n, uint8_t (*P)[kPatch + 1]) {
    constexpr int D = kPatch + 1;
    const double inv_scale = (double)D / n, scale = 1. / inv_scale;
    const int iscale = cv_round_d(scale);
    if (std::abs(scale - iscale) < DBL_EPSILON) {  // resizeAreaFast_
        const int area = iscale * iscale;
        const float fs = 1.f / area;
        for (int dy = 0; dy < D; ++dy)
            for (int dx = 0; dx < D; ++dx) {
                int s = 0;
                for (int sy = 0; sy < iscale; ++sy)
                    for (int sx = 0; sx < iscale; ++sx) s += W[(size_t)(dy * iscale + sy) * n + dx * iscale + sx];
                P[dy][dx] = iscale == 2 ? (uint8_t)((s + 2) >> 2)
                                        : (uint8_t)std::min(255, std::max(0, cv_round(s * fs)));
            }
        return;
    }
    AreaCell c[D];
    area_cells(n, D, scale, c);
    // the ResizeArea_Invoker loop over ytab entries (dy, sy, beta) in order
    for (int dy = 0; dy < D; ++dy) {
        float sum[D], buf[D];
        bool first = true;
        auto row = [&](int sy, float beta) {
            const uint8_t* S = W.data() + (size_t)sy * n;
            for (int dx = 0; dx < D; ++dx) {  // xtab entries in k order
                float b = 0;
                if (c[dx].has_l) b += S[c[dx].s1 - 1] * c[dx].al;
                for (int sx = c[dx].s1; sx < c[dx].s2; ++sx) b += S[sx] * c[dx].af;
                if (c[dx].has_r) b += S[c[dx].s2] * c[dx].ar;
                buf[dx] = b;
            }
            for (int dx = 0; dx < D; ++dx) {
                if (first) sum[dx] = beta * buf[dx];
                else sum[dx] += beta * buf[dx];
            }
            first = false;
        };
        if (c[dy].has_l) row(c[dy].s1 - 1, c[dy].al);
        for (int sy = c[dy].s1; sy < c[dy].s2; ++sy) row(sy, c[dy].af);
        if (c[dy].has_r) row(c[dy].s2, c[dy].ar);
        for (int dx = 0; dx < D; ++dx) P[dy][dx] = (uint8_t)std::min(255, std::max(0, cv_round(sum[dx])));
    }
}

}  // namespace

extern "C" int ora_surf_detect_and_compute(const uint8_t* img, int w, int h, int stride, double hessian_threshold,
                                           ora_keypoint* kps, float* desc, int cap, int* n_out) {
    if (!img || !n_out || w < 1 || h < 1 || stride < w || cap < 0 || (cap > 0 && (!kps || !desc))) return -1;
    *n_out = 0;
    // integral(img, sum, CV_32S)
    const int sw = w + 1, sh = h + 1;
    std::vector<int32_t> sum((size_t)sw * sh, 0);
    for (int y = 0; y < h; ++y) {
        int32_t row = 0;
        for (int x = 0; x < w; ++x) {
            row += img[(size_t)y * stride + x];
            sum[(size_t)(y + 1) * sw + x + 1] = sum[(size_t)y * sw + x + 1] + row;
        }
    }
    // fastHessianDetector
    const int ntot = (kLayers + 2) * kOctaves;
    std::vector<Layer> L(ntot);
    std::vector<int> middle;
    for (int o = 0, idx = 0, step = 1; o < kOctaves; ++o, step *= 2)
        for (int l = 0; l < kLayers + 2; ++l, ++idx) {
            Layer& q = L[idx];
            q.rows = (sh - 1) / step;
            q.cols = (sw - 1) / step;
            q.det.assign((size_t)q.rows * q.cols, 0.f);
            q.trace.assign((size_t)q.rows * q.cols, 0.f);
            q.size = (kHaar0 + kHaarInc * l) << o;
            q.step = step;
            if (0 < l && l <= kLayers) middle.push_back(idx);
        }
    for (Layer& q : L) calc_layer(sum, sw, sh, q);
    const float thr = (float)hessian_threshold;
    std::vector<ora_keypoint> K;
    for (size_t mi = 0; mi < middle.size(); ++mi) {  // findMaximaInLayer
        const int li = middle[mi], octave = (int)mi / kLayers;
        const Layer &A = L[li - 1], &B = L[li], &C = L[li + 1];
        const int size = B.size, step = B.step;
        const int rows = (sh - 1) / step, cols = (sw - 1) / step;
        const int margin = (C.size / 2) / step + 1;
        for (int i = margin; i < rows - margin; ++i)
            for (int j = margin; j < cols - margin; ++j) {
                const float v = B.det[(size_t)i * B.cols + j];
                if (!(v > thr)) continue;
                const int sum_i = step * (i - (size / 2) / step), sum_j = step * (j - (size / 2) / step);
                float N9[3][9];
                const Layer* LL[3] = {&A, &B, &C};
                for (int t = 0; t < 3; ++t)
                    for (int r = 0; r < 3; ++r)
                        for (int q = 0; q < 3; ++q) N9[t][r * 3 + q] = LL[t]->det[(size_t)(i + r - 1) * LL[t]->cols + (j + q - 1)];
                bool mx = true;
                for (int t = 0; t < 3; ++t)
                    for (int k = 0; k < 9; ++k)
                        if (!(t == 1 && k == 4)) mx = mx && v > N9[t][k];
                if (!mx) continue;
                const float center_i = sum_i + (size - 1) * 0.5f, center_j = sum_j + (size - 1) * 0.5f;
                const float tr = B.trace[(size_t)i * B.cols + j];
                ora_keypoint kp{center_j, center_i, (float)size, -1.f, v, octave, (tr > 0) - (tr < 0)};
                if (interpolate(N9, step, step, size - A.size, kp)) K.push_back(kp);
            }
    }
    std::sort(K.begin(), K.end(), kp_greater);
    // SURFInvoker: orientation and 64-d descriptor per keypoint
    const std::vector<float> Go = gauss_kernel(2 * kOriRadius + 1, kOriSigma), Gd = gauss_kernel(kPatch, kDescSigma);
    int apx[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)], apy[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)];
    float apw[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)];
    int nori = 0;
    for (int i = -kOriRadius; i <= kOriRadius; ++i)
        for (int j = -kOriRadius; j <= kOriRadius; ++j)
            if (i * i + j * j <= kOriRadius * kOriRadius) {
                apx[nori] = i;  // apt[n] = Point(i, j)
                apy[nori] = j;
                apw[nori++] = Go[i + kOriRadius] * Go[j + kOriRadius];
            }
    std::vector<float> D((size_t)K.size() * 64, 0.f);
    std::vector<uint8_t> win;
    for (size_t k = 0; k < K.size(); ++k) {
        ora_keypoint& kp = K[k];
        const float s = kp.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round(2 * s);
        if (sh < gws || sw < gws) {
            kp.size = -1;
            continue;
        }
        HF gx[2], gy[2];
        resize_haar(kGxS, gx, 2, 4, gws, sw);
        resize_haar(kGyS, gy, 2, 4, gws, sw);
        float X[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)], Y[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)];
        int nang = 0;
        for (int t = 0; t < nori; ++t) {
            const int x = cv_round(kp.x + apx[t] * s - (float)(gws - 1) / 2);
            const int y = cv_round(kp.y + apy[t] * s - (float)(gws - 1) / 2);
            if (y < 0 || y >= sh - gws || x < 0 || x >= sw - gws) continue;
            const int32_t* p = sum.data() + (size_t)y * sw + x;
            const float vx = haar(p, gx, 2), vy = haar(p, gy, 2);
            X[nang] = vx * apw[t];
            Y[nang] = vy * apw[t];
            nang++;
        }
        if (nang == 0) {
            kp.size = -1;
            continue;
        }
        float ang[(2 * kOriRadius + 1) * (2 * kOriRadius + 1)];
        for (int t = 0; t < nang; ++t) ang[t] = fast_atan2_deg(Y[t], X[t]);  // phase(X, Y, angle, true)
        float bestx = 0, besty = 0, best = 0;
        for (float i = 0; i < 360; i += kOriInc) {
            float sx = 0, sy = 0;
            for (int t = 0; t < nang; ++t) {
                const int d = (int)std::abs(cv_round(ang[t]) - i);
                if (d < kOriWin / 2 || d > 360 - kOriWin / 2) {
                    sx += X[t];
                    sy += Y[t];
                }
            }
            const float m = sx * sx + sy * sy;
            if (m > best) {
                best = m;
                bestx = sx;
                besty = sy;
            }
        }
        float dir = fast_atan2_deg(-besty, bestx);
        kp.angle = dir;
        // the rotated window of 20s, bilinear, then INTER_AREA down to 21 x 21
        const int n = (int)((kPatch + 1) * s);
        win.assign((size_t)n * n, 0);
        dir *= (float)(M_PI / 180);
        const float sin_dir = -(float)std::sin((double)dir), cos_dir = (float)std::cos((double)dir);
        const float off = -(float)(n - 1) / 2;
        float start_x = kp.x + off * cos_dir + off * sin_dir;
        float start_y = kp.y - off * sin_dir + off * cos_dir;
        const int nc1 = w - 1, nr1 = h - 1;
        for (int i = 0; i < n; ++i, start_x += sin_dir, start_y += cos_dir) {
            double px = start_x, py = start_y;
            for (int j = 0; j < n; ++j, px += cos_dir, py -= sin_dir) {
                const int ix = cv_floor_d(px), iy = cv_floor_d(py);
                uint8_t v;
                if ((unsigned)ix < (unsigned)nc1 && (unsigned)iy < (unsigned)nr1) {
                    const float a = (float)(px - ix), b = (float)(py - iy);
                    const uint8_t* q = img + (size_t)iy * stride + ix;
                    v = (uint8_t)cv_round(q[0] * (1.f - a) * (1.f - b) + q[1] * a * (1.f - b) + q[stride] * (1.f - a) * b +
                                          q[stride + 1] * a * b);
                } else {
                    const int x = std::min(std::max(cv_round_d(px), 0), nc1), y = std::min(std::max(cv_round_d(py), 0), nr1);
                    v = img[(size_t)y * stride + x];
                }
                win[(size_t)i * n + j] = v;
            }
        }
        uint8_t P[kPatch + 1][kPatch + 1];
        resize_area21(win, n, P);
        float DX[kPatch][kPatch], DY[kPatch][kPatch];
        for (int i = 0; i < kPatch; ++i)
            for (int j = 0; j < kPatch; ++j) {
                const float dw = Gd[i] * Gd[j];
                DX[i][j] = (P[i][j + 1] - P[i][j] + P[i + 1][j + 1] - P[i + 1][j]) * dw;
                DY[i][j] = (P[i + 1][j] - P[i][j] + P[i + 1][j + 1] - P[i][j + 1]) * dw;
            }
        float* vec = D.data() + k * 64;
        double mag = 0;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                for (int y = i * 5; y < i * 5 + 5; ++y)
                    for (int x = j * 5; x < j * 5 + 5; ++x) {
                        const float tx = DX[y][x], ty = DY[y][x];
                        vec[0] += tx;
                        vec[1] += ty;
                        vec[2] += (float)std::fabs(tx);
                        vec[3] += (float)std::fabs(ty);
                    }
                for (int q = 0; q < 4; ++q) mag += vec[q] * vec[q];
                vec += 4;
            }
        vec = D.data() + k * 64;
        const float sc = (float)(1. / (std::sqrt(mag) + FLT_EPSILON));
        for (int q = 0; q < 64; ++q) vec[q] *= sc;
    }
    // drop the keypoints marked size -1, in order
    int m = 0;
    for (size_t k = 0; k < K.size(); ++k) {
        if (!(K[k].size > 0)) continue;
        if (m < cap) {
            kps[m] = K[k];
            std::memcpy(desc + (size_t)m * 64, D.data() + k * 64, 64 * sizeof(float));
        }
        m++;
    }
    *n_out = m;
    return m > cap ? -5 : 0;  // -5: cap too small, *n_out = the count needed (as the SIFT entry)
}
