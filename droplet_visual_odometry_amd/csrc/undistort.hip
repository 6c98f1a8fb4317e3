// Image pre-processing of the reference's frame path on gfx950:
// cv.undistort(gray, K, dist, None, new_K) (scripts/visual_odometry_v3.py:120,
// called from ros_img_msg_to_opencv_image v3:110-135).  SURVEY.md §8f rank 1.
//
// undistort_map_kernel: OpenCV builds the remap table in stripes of
//   min(max(1, 4096 / cols), rows) rows, each with the principal point of new_K
//   shifted by the stripe's first row and its own LU inverse (host, per stripe).
//   One thread per output row walks the columns exactly like
//   initUndistortRectifyMap's scalar loop (x advanced by repeated addition),
//   in double, and stores the CV_16SC2 integer part and the CV_16UC1 1/32-pixel
//   fraction.  Built once per calibration and kept on the device.
// undistort_remap_kernel: remap(INTER_LINEAR, BORDER_CONSTANT 0) with the
//   fixed-point bilinear table (weights (32-ty)(32-tx)*32 ... summing to 2^15),
//   4 output pixels per thread stored as one word, any number of frames.
#include "dvo_internal.h"

namespace dvo {
namespace {

__global__ __launch_bounds__(64) void undistort_map_kernel(UndistortGeom U, const double* __restrict__ ir_stripes,
                                                           int16_t* __restrict__ xy, uint16_t* __restrict__ frac) {
    const int row = blockIdx.x * 64 + threadIdx.x;
    if (row >= U.h) return;
    const int s = row / U.stripe, i = row - s * U.stripe;
    const double* ir = ir_stripes + 9 * s;
    const double u0 = U.K[2], v0 = U.K[5], fx = U.K[0], fy = U.K[4];
    const double *k = U.dist, k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7],
                 s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    int16_t* m1 = xy + (int64_t)row * U.w * 2;
    uint16_t* m2 = frac + (int64_t)row * U.w;
    for (int j = 0; j < U.w; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double ww = 1. / _w, x = _x * ww, y = _y * ww;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
        const double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
        const double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
        const double u = fx * (1. * xd) + u0;
        const double v = fy * (1. * yd) + v0;
        const int iu = (int)rint(u * 32), iv = (int)rint(v * 32);
        m1[2 * j] = (int16_t)(iu >> 5);
        m1[2 * j + 1] = (int16_t)(iv >> 5);
        m2[j] = (uint16_t)((iv & 31) * 32 + (iu & 31));
    }
}

__device__ __forceinline__ uint32_t remap_px(const uint8_t* src, int sw, int sh, int sp, int sx, int sy, int a) {
    const int ty = a >> 5, tx = a & 31;
    const int w00 = (32 - ty) * (32 - tx) * 32, w01 = (32 - ty) * tx * 32, w10 = ty * (32 - tx) * 32, w11 = ty * tx * 32;
    int v00, v01, v10, v11;
    if ((unsigned)sx < (unsigned)(sw - 1) && (unsigned)sy < (unsigned)(sh - 1)) {
        const uint8_t* S = src + (int64_t)sy * sp + sx;
        v00 = S[0];
        v01 = S[1];
        v10 = S[sp];
        v11 = S[sp + 1];
    } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        return 0;
    } else {
        auto pix = [&](int x, int y) {
            return (x >= 0 && x < sw && y >= 0 && y < sh) ? (int)src[(int64_t)y * sp + x] : 0;
        };
        v00 = pix(sx, sy);
        v01 = pix(sx + 1, sy);
        v10 = pix(sx, sy + 1);
        v11 = pix(sx + 1, sy + 1);
    }
    const int r = (v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11 + (1 << 14)) >> 15;
    return (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

__global__ __launch_bounds__(256) void undistort_remap_kernel(UndistortGeom U, const int16_t* __restrict__ xy,
                                                              const uint16_t* __restrict__ frac,
                                                              const uint8_t* __restrict__ src, int64_t src_fstride,
                                                              int src_pitch, uint8_t* __restrict__ dst,
                                                              int64_t dst_fstride, int dst_pitch) {
    const int f = blockIdx.z;
    const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x0 >= U.w || y >= U.h) return;
    const uint8_t* s = src + (int64_t)f * src_fstride;
    uint8_t* d = dst + (int64_t)f * dst_fstride + (int64_t)y * dst_pitch;
    const int16_t* m1 = xy + ((int64_t)y * U.w + x0) * 2;
    const uint16_t* m2 = frac + (int64_t)y * U.w + x0;
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (x0 + j < U.w)
            word |= remap_px(s, U.w, U.h, src_pitch, m1[2 * j], m1[2 * j + 1], m2[j] & 1023) << (8 * j);
    if (x0 + 4 <= U.w && ((dst_pitch | (uintptr_t)d) & 3) == 0) {
        *reinterpret_cast<uint32_t*>(d + x0) = word;
    } else {
        for (int j = 0; j < 4 && x0 + j < U.w; ++j) d[x0 + j] = (uint8_t)(word >> (8 * j));
    }
}

}  // namespace

hipError_t launch_undistort_map(const UndistortGeom& U, const double* d_ir, int16_t* d_xy, uint16_t* d_frac,
                                hipStream_t s) {
    hipLaunchKernelGGL(undistort_map_kernel, dim3((U.h + 63) / 64), dim3(64), 0, s, U, d_ir, d_xy, d_frac);
    return hipGetLastError();
}

hipError_t launch_undistort_remap(const UndistortGeom& U, const int16_t* d_xy, const uint16_t* d_frac,
                                  const uint8_t* d_src, int n, int64_t src_fstride, int src_pitch, uint8_t* d_dst,
                                  int64_t dst_fstride, int dst_pitch, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    dim3 grid((U.w + 255) / 256, (U.h + 3) / 4, n);
    hipLaunchKernelGGL(undistort_remap_kernel, grid, dim3(256), 0, s, U, d_xy, d_frac, d_src, src_fstride, src_pitch,
                       d_dst, dst_fstride, dst_pitch);
    return hipGetLastError();
}

}  // namespace dvo
