// TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's image
// pre-processing: visual_odometry_v3.py:117-135
//   new_K, roi = cv.getOptimalNewCameraMatrix(K, dist, (w, h), 1, (w, h))
//   undistorted = cv.undistort(gray, K, dist, None, new_K)
// restated from OpenCV 4.x (calibration.cpp cvGetOptimalNewCameraMatrix /
// icvGetRectangles, undistort.dispatch.cpp cvUndistortPointsInternal,
// cv::undistort, initUndistortRectifyMap, imgproc/imgwarp.cpp remapBilinear with
// the 32x32 fixed-point bilinear table).  OpenCV itself is absent here, so this
// path is "parity unpinned": the GPU is checked bit-exact against this file.
// Restatement choices:
//   * initUndistortRectifyMap follows the scalar per-row loop (x advanced by
//     repeated addition of ir[0]); OpenCV >= 4.x may take a SIMD line routine
//     whose rounding can differ in the last bit of u, v before the 1/32-pixel
//     quantisation.
//   * cv::undistort builds the map in stripes of min(max(1, 4096 / cols), rows)
//     rows with the principal point shifted by the stripe's first row.
//   * distortion models: k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]]; no tilt.
#include "oracle.h"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

struct Dist {
    double k[12] = {0};  // k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4
};

Dist load_dist(const double* d, int n) {
    Dist D;
    for (int i = 0; i < n && i < 12; ++i) D.k[i] = d[i];
    return D;
}

// cvUndistortPointsInternal, R = P = identity, TermCriteria(COUNT, 5, 0.01):
// float points in, normalised float points out.
void undistort_points(const float* in, float* out, int n, const double* A, const Dist& D) {
    const double* k = D.k;
    const double fx = A[0], fy = A[4], ifx = 1. / fx, ify = 1. / fy, cx = A[2], cy = A[5];
    for (int i = 0; i < n; ++i) {
        double x = in[2 * i], y = in[2 * i + 1];
        const double u = x, v = y;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;  // no tilt: invMatTilt = I, invProj = 1
        for (int j = 0; j < 5; ++j) {
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            if (icdist < 0) {
                x = (u - cx) * ifx;
                y = (v - cy) * ify;
                break;
            }
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        // R = I: xx = x, yy = y, ww = 1 / 1
        const double ww = 1. / (0. * x + 0. * y + 1.);
        out[2 * i] = (float)((1. * x + 0. * y + 0.) * ww);
        out[2 * i + 1] = (float)((0. * x + 1. * y + 0.) * ww);
    }
}

// 3x3 inverse by LU with partial pivoting (Mat::inv(DECOMP_LU) -> hal LU on [A | I]).
bool inv3_lu(const double* M, double* out) {
    double A[9], b[9];
    std::memcpy(A, M, sizeof(A));
    for (int i = 0; i < 9; ++i) b[i] = (i % 4 == 0) ? 1.0 : 0.0;
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < 3; i++) {
        int k = i;
        for (int j = i + 1; j < 3; j++)
            if (std::fabs(A[j * 3 + i]) > std::fabs(A[k * 3 + i])) k = j;
        if (std::fabs(A[k * 3 + i]) < eps) return false;
        if (k != i) {
            for (int j = i; j < 3; j++) std::swap(A[i * 3 + j], A[k * 3 + j]);
            for (int j = 0; j < 3; j++) std::swap(b[i * 3 + j], b[k * 3 + j]);
        }
        const double d = -1 / A[i * 3 + i];
        for (int j = i + 1; j < 3; j++) {
            const double alpha = A[j * 3 + i] * d;
            for (int c = i + 1; c < 3; c++) A[j * 3 + c] += alpha * A[i * 3 + c];
            for (int c = 0; c < 3; c++) b[j * 3 + c] += alpha * b[i * 3 + c];
        }
    }
    for (int i = 2; i >= 0; i--)
        for (int j = 0; j < 3; j++) {
            double s = b[i * 3 + j];
            for (int k = i + 1; k < 3; k++) s -= A[i * 3 + k] * b[k * 3 + j];
            b[i * 3 + j] = s / A[i * 3 + i];
        }
    std::memcpy(out, b, sizeof(b));
    return true;
}

int round_i(double v) { return (int)std::lrint(v); }

// initUndistortRectifyMapComputer, CV_16SC2 + CV_16UC1 maps, R = I.
void map_rows(const double* A, const Dist& D, const double* ir, int w, int rows, int16_t* xy, uint16_t* frac) {
    const double u0 = A[2], v0 = A[5], fx = A[0], fy = A[4];
    const double *k = D.k, k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7],
                 s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
    for (int i = 0; i < rows; ++i) {
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < w; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double ww = 1. / _w, x = _x * ww, y = _y * ww;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
            const double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
            // tilt matrix = I: vecTilt = (xd, yd, 1), invProj = 1
            const double u = fx * (1. * xd) + u0;
            const double v = fy * (1. * yd) + v0;
            const int iu = round_i(u * 32), iv = round_i(v * 32);
            xy[(i * w + j) * 2] = (int16_t)(iu >> 5);
            xy[(i * w + j) * 2 + 1] = (int16_t)(iv >> 5);
            frac[i * w + j] = (uint16_t)((iv & 31) * 32 + (iu & 31));
        }
    }
}

// remapBilinear<FixedPtCast<int, uchar, 15>, short> for one channel, BORDER_CONSTANT 0.
void remap_rows(const uint8_t* src, int sw, int sh, int sstride, const int16_t* xy, const uint16_t* frac, int w,
                int rows, uint8_t* dst, int dstride) {
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < w; ++j) {
            const int sx = xy[(i * w + j) * 2], sy = xy[(i * w + j) * 2 + 1];
            const int a = frac[i * w + j] & 1023, ty = a >> 5, tx = a & 31;
            const int w00 = (32 - ty) * (32 - tx) * 32, w01 = (32 - ty) * tx * 32, w10 = ty * (32 - tx) * 32,
                      w11 = ty * tx * 32;  // float table x 32768, exact (sum 32768)
            int v00, v01, v10, v11;
            if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
                const uint8_t* S = src + (size_t)sy * sstride + sx;
                v00 = S[0];
                v01 = S[1];
                v10 = S[sstride];
                v11 = S[sstride + 1];
            } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
                dst[(size_t)i * dstride + j] = 0;
                continue;
            } else {
                auto pix = [&](int x, int y) { return (x >= 0 && x < sw && y >= 0 && y < sh) ? src[(size_t)y * sstride + x] : 0; };
                v00 = pix(sx, sy);
                v01 = pix(sx + 1, sy);
                v10 = pix(sx, sy + 1);
                v11 = pix(sx + 1, sy + 1);
            }
            const int s = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
            const int r = (s + (1 << 14)) >> 15;
            dst[(size_t)i * dstride + j] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        }
}

}  // namespace

extern "C" {

int ora_get_optimal_new_camera_matrix(const double* K, const double* dist, int ndist, int w, int h, double alpha,
                                      int new_w, int new_h, double* newK) {
    const Dist D = load_dist(dist, ndist);
    if (new_w * new_h == 0) {
        new_w = w;
        new_h = h;
    }
    const int N = 9;
    std::vector<float> pts(2 * N * N);
    for (int y = 0, k = 0; y < N; y++)
        for (int x = 0; x < N; x++, k++) {
            pts[2 * k] = (float)x * w / (N - 1);
            pts[2 * k + 1] = (float)y * h / (N - 1);
        }
    undistort_points(pts.data(), pts.data(), N * N, K, D);
    float iX0 = -FLT_MAX, iX1 = FLT_MAX, iY0 = -FLT_MAX, iY1 = FLT_MAX;
    float oX0 = FLT_MAX, oX1 = -FLT_MAX, oY0 = FLT_MAX, oY1 = -FLT_MAX;
    for (int y = 0, k = 0; y < N; y++)
        for (int x = 0; x < N; x++, k++) {
            const float px = pts[2 * k], py = pts[2 * k + 1];
            oX0 = std::min(oX0, px);
            oX1 = std::max(oX1, px);
            oY0 = std::min(oY0, py);
            oY1 = std::max(oY1, py);
            if (x == 0) iX0 = std::max(iX0, px);
            if (x == N - 1) iX1 = std::min(iX1, px);
            if (y == 0) iY0 = std::max(iY0, py);
            if (y == N - 1) iY1 = std::min(iY1, py);
        }
    const float in_x = iX0, in_y = iY0, in_w = iX1 - iX0, in_h = iY1 - iY0;
    const float ou_x = oX0, ou_y = oY0, ou_w = oX1 - oX0, ou_h = oY1 - oY0;
    std::memcpy(newK, K, 9 * sizeof(double));
    const double fx0 = (new_w - 1) / in_w, fy0 = (new_h - 1) / in_h;
    const double cx0 = -fx0 * in_x, cy0 = -fy0 * in_y;
    const double fx1 = (new_w - 1) / ou_w, fy1 = (new_h - 1) / ou_h;
    const double cx1 = -fx1 * ou_x, cy1 = -fy1 * ou_y;
    newK[0] = fx0 * (1 - alpha) + fx1 * alpha;
    newK[4] = fy0 * (1 - alpha) + fy1 * alpha;
    newK[2] = cx0 * (1 - alpha) + cx1 * alpha;
    newK[5] = cy0 * (1 - alpha) + cy1 * alpha;
    return 0;
}

// cv::undistort(src, K, dist, newK): stripes of map + remap.  xy/frac (w*h)
// receive the concatenated stripe maps (test access).
int ora_undistort(const uint8_t* src, int w, int h, int stride, const double* K, const double* dist, int ndist,
                  const double* newK, uint8_t* dst, int dstride, int16_t* xy, uint16_t* frac) {
    const Dist D = load_dist(dist, ndist);
    double Ar[9];
    std::memcpy(Ar, newK ? newK : K, sizeof(Ar));
    const double v0 = Ar[5];
    const int stripe0 = std::min(std::max(1, (1 << 12) / std::max(w, 1)), h);
    for (int y = 0; y < h; y += stripe0) {
        const int rows = std::min(stripe0, h - y);
        Ar[5] = v0 - y;
        double ir[9];
        if (!inv3_lu(Ar, ir)) return -1;
        map_rows(K, D, ir, w, rows, xy + (size_t)y * w * 2, frac + (size_t)y * w);
        remap_rows(src, w, h, stride, xy + (size_t)y * w * 2, frac + (size_t)y * w, w, rows, dst + (size_t)y * dstride,
                   dstride);
    }
    return 0;
}

}  // extern "C"
