// xfeatures2d::SURF_create(hessianThreshold).detectAndCompute on gfx950: the
// detector of the reference's 'surf' mode (scripts/visual_odometry_v3.py:103-106,
// detectAndCompute at :373), feeding the float k-NN matcher (match.hip, 64-d).
// Every float expression follows oracle/surf.cpp (the restatement of
// opencv_contrib surf.cpp and the INTER_AREA resize it calls) operation for
// operation, compiled with -ffp-contract=off, so keypoints and descriptors are
// bit-identical to it.
//
// Pipeline for one image (launch_surf):
//   row_scan / col_scan   integral(img, sum, CV_32S) (integer: any order)
//   hessian_kernel        calcLayerDetAndTrace of the 20 layers, thread per sample
//   extrema_kernel        findMaximaInLayer of the 12 middle layers, thread per
//                         sample: threshold, strict 3x3x3 maximum, interpolation
//   sort_kernel           KeypointGreater order (one workgroup, bitonic)
//   describe_kernel       one wave per keypoint: the 113-sample orientation disc
//                         (ballot-compacted in sample order), the 72 sliding
//                         windows one per lane; the rotated 20s window walked row
//                         by row (one row per lane, the row's double coordinate
//                         accumulated pixel by pixel as OpenCV does), each row
//                         folded into the INTER_AREA cells as it is produced and
//                         the rows combined per output row in ytab order; then
//                         the 4x4x4 sums
//   compact_kernel        drop the keypoints marked size -1, in order
#include <cfloat>

#include "dvo_internal.h"

namespace dvo {
namespace {

constexpr int kOriN = 113, kOriWin = 60, kOriInc = 5;
constexpr int kPatch = 20, kP1 = 21;
constexpr int kMaxWin = 768;  // window side: size <= 264 -> (int)(21 * 35.2) = 739
constexpr int kSortNT = 1024;

__device__ __forceinline__ int cv_ceil_d(double v) {
    const int i = (int)v;
    return i + (i < v);
}

__device__ __forceinline__ float atan2_deg(float y, float x) {  // cv::fastAtan2, scalar
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
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

__device__ __forceinline__ float haar(const int32_t* o, const SurfHaar* f, int n) {  // calcHaarPattern
    double d = 0;
    for (int k = 0; k < n; ++k) d += (double)((float)(o[f[k].p0] + o[f[k].p3] - o[f[k].p1] - o[f[k].p2]) * f[k].w);
    return (float)d;
}

__device__ __forceinline__ void resize_haar(const int (&src)[2][5], SurfHaar* dst, int old_size, int new_size, int step) {
    const float ratio = (float)new_size / old_size;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int dx1 = cv_round_f(ratio * src[k][0]), dy1 = cv_round_f(ratio * src[k][1]);
        const int dx2 = cv_round_f(ratio * src[k][2]), dy2 = cv_round_f(ratio * src[k][3]);
        dst[k].p0 = dy1 * step + dx1;
        dst[k].p1 = dy2 * step + dx1;
        dst[k].p2 = dy1 * step + dx2;
        dst[k].p3 = dy2 * step + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

// ---- integral image -------------------------------------------------------------
__global__ __launch_bounds__(256) void row_scan_kernel(SurfArgs a) {
    const int y = blockIdx.x;
    if (y >= a.h) return;
    const int sw = a.w + 1, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ int s_w[4];
    int carry = 0;
    for (int x0 = 0; x0 < a.w; x0 += 256) {
        const int x = x0 + threadIdx.x;
        const int v = x < a.w ? a.img[(size_t)y * a.pitch + x] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();
        int before = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            before += k < wid ? s_w[k] : 0;
            tot += s_w[k];
        }
        if (x < a.w) a.sum[(size_t)(y + 1) * sw + x + 1] = carry + before + incl;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.sum[(size_t)(y + 1) * sw] = 0;
}

__global__ __launch_bounds__(256) void col_scan_kernel(SurfArgs a) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int sw = a.w + 1;
    if (x > a.w) return;
    a.sum[x] = 0;
    int acc = 0, y = 1;
    for (; y + 8 <= a.h + 1; y += 8) {  // 8 rows of loads in flight, then the sequential sums
        int v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = a.sum[(size_t)(y + k) * sw + x];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc += v[k];
            a.sum[(size_t)(y + k) * sw + x] = acc;
        }
    }
    for (; y <= a.h; ++y) {
        acc += a.sum[(size_t)y * sw + x];
        a.sum[(size_t)y * sw + x] = acc;
    }
}

// ---- calcLayerDetAndTrace -------------------------------------------------------
__global__ __launch_bounds__(256) void hessian_kernel(SurfArgs a) {
    const int L = blockIdx.y, o = L / kSurfLayers;
    const int size = a.size[L], step = 1 << o;
    const int sw = a.w + 1, sh = a.h + 1;
    if (size > sh - 1 || size > sw - 1) return;
    const int si = 1 + (sh - 1 - size) / step, sj = 1 + (sw - 1 - size) / step;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)si * sj) return;
    const int i = (int)(t / sj), j = (int)(t - (int64_t)i * sj);
    const int margin = (size / 2) / step;
    const int32_t* sp = a.sum + (size_t)(i * step) * sw + j * step;
    const SurfHaar* H = a.haar + L * 10;
    const float dx = haar(sp, H, 3), dy = haar(sp, H + 3, 3), dxy = haar(sp, H + 6, 4);
    const int64_t off = a.off[L] + (int64_t)(i + margin) * a.cols[o] + (j + margin);
    a.det[off] = dx * dy - 0.81f * dxy * dxy;
    a.trace[off] = dx + dy;
}

// ---- findMaximaInLayer + interpolateKeypoint -------------------------------------
__global__ __launch_bounds__(256) void extrema_kernel(SurfArgs a) {
    const int m = blockIdx.y, o = m / 3, Li = o * kSurfLayers + m % 3 + 1;
    const int step = 1 << o, size = a.size[Li];
    const int rows = a.h / step, cols = a.w / step, C = a.cols[o];
    const int margin = (a.size[Li + 1] / 2) / step + 1;
    const int ni = rows - 2 * margin, nj = cols - 2 * margin;
    if (ni <= 0 || nj <= 0) return;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)ni * nj) return;
    const int i = margin + (int)(t / nj), j = margin + (int)(t % nj);
    const float* d2 = a.det + a.off[Li];
    const float v = d2[(int64_t)i * C + j];
    if (!(v > a.thr)) return;
    const float* Ls[3] = {a.det + a.off[Li - 1], d2, a.det + a.off[Li + 1]};
    float N9[3][9];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) N9[q][r * 3 + c] = Ls[q][(int64_t)(i + r - 1) * C + (j + c - 1)];
    bool mx = true;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if (!(q == 1 && k == 4)) mx = mx && v > N9[q][k];
    if (!mx) return;
    const int sum_i = step * (i - (size / 2) / step), sum_j = step * (j - (size / 2) / step);
    const float tr = a.trace[a.off[Li] + (int64_t)i * C + j];
    dvo_keypoint kp;
    kp.x = sum_j + (size - 1) * 0.5f;
    kp.y = sum_i + (size - 1) * 0.5f;
    kp.size = (float)size;
    kp.angle = -1.f;
    kp.response = v;
    kp.octave = o;
    kp.class_id = (tr > 0) - (tr < 0);
    // interpolateKeypoint: Matx33f(A).solve(b, DECOMP_LU) = Matx_FastSolveOp<3, 1>
    const int ds = size - a.size[Li - 1];
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
    float d = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
    if (d != 0) {
        d = 1 / d;
        x0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2));
        x1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) + a02 * (a10 * b2 - b1 * a20));
        x2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * (a10 * a21 - a11 * a20));
    }
    const bool ok = (x0 != 0 || x1 != 0 || x2 != 0) && fabsf(x0) <= 1 && fabsf(x1) <= 1 && fabsf(x2) <= 1;
    if (!ok) return;
    kp.x += x0 * step;
    kp.y += x1 * step;
    kp.size = (float)cv_round_f(kp.size + x2 * ds);
    const int slot = atomicAdd(a.nraw, 1);
    if (slot < a.kp_cap) a.raw[slot] = kp;
    else atomicOr(a.flags, 2);
}

// ---- std::sort(KeypointGreater) ---------------------------------------------------
__device__ __forceinline__ bool kp_greater(const dvo_keypoint& a, const dvo_keypoint& b) {
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

__global__ __launch_bounds__(kSortNT) void sort_kernel(SurfArgs a) {
    const int n = min(*a.nraw, a.kp_cap);
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    int32_t* idx = a.order;
    for (int i = threadIdx.x; i < n2; i += kSortNT) idx[i] = i < n ? i : -1;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += kSortNT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int p = idx[i], q = idx[ixj];
                    // q belongs before p (padding -1 sorts last)
                    const bool q_first = p < 0 ? q >= 0 : (q >= 0 && kp_greater(a.raw[q], a.raw[p]));
                    if (q_first == ((i & k) == 0)) {
                        idx[i] = q;
                        idx[ixj] = p;
                    }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < n; i += kSortNT) a.kps[i] = a.raw[idx[i]];
}

// ---- SURFInvoker: orientation + 64-d descriptor, one wave per keypoint ------------
struct AreaCell {
    int s1, s2, has_l, has_r;
    float al, af, ar;
};

__device__ __forceinline__ uint8_t win_sample(const SurfArgs& a, double px, double py) {
    const int ix = cv_floor_d(px), iy = cv_floor_d(py);
    if ((unsigned)ix < (unsigned)(a.w - 1) && (unsigned)iy < (unsigned)(a.h - 1)) {
        const float fa = (float)(px - ix), fb = (float)(py - iy);
        const uint8_t* q = a.img + (size_t)iy * a.pitch + ix;
        return (uint8_t)cv_round_f(q[0] * (1.f - fa) * (1.f - fb) + q[1] * fa * (1.f - fb) + q[a.pitch] * (1.f - fa) * fb +
                                   q[a.pitch + 1] * fa * fb);
    }
    const int x = min(max(cv_round_d(px), 0), a.w - 1), y = min(max(cv_round_d(py), 0), a.h - 1);
    return a.img[(size_t)y * a.pitch + x];
}

__global__ __launch_bounds__(64) void describe_kernel(SurfArgs a) {
    __shared__ float s_X[128], s_Y[128];
    __shared__ int s_A[128];
    __shared__ float s_sx[kMaxWin], s_sy[kMaxWin];        // window row starts
    __shared__ int16_t s_e0[kMaxWin], s_e1[kMaxWin];      // INTER_AREA cells a source column feeds
    __shared__ float s_a0[kMaxWin], s_a1[kMaxWin];
    __shared__ AreaCell s_cell[kP1];
    __shared__ int s_pre[kP1 + 1];
    __shared__ float s_buf[64][kP1 + 1];
    __shared__ int s_edy[64];
    __shared__ float s_ebeta[64];
    __shared__ uint8_t s_P[kP1][kP1];
    __shared__ float s_DX[kPatch * kPatch], s_DY[kPatch * kPatch];
    __shared__ float s_vec[64];
    const int lane = threadIdx.x;
    const int n_kp = min(*a.nraw, a.kp_cap);
    const int sw = a.w + 1, sh = a.h + 1;
    const int gx_s[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
    const int gy_s[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};
    for (int k = blockIdx.x; k < n_kp; k += gridDim.x) {
        dvo_keypoint kp = a.kps[k];
        const float s = kp.size * 1.2f / 9.0f;
        const int gws = 2 * cv_round_f(2 * s);
        if (sh < gws || sw < gws) {
            if (lane == 0) a.kps[k].size = -1;
            continue;
        }
        // ---- orientation: the disc's Haar responses, compacted in sample order
        SurfHaar gx[2], gy[2];
        resize_haar(gx_s, gx, 4, gws, sw);
        resize_haar(gy_s, gy, 4, gws, sw);
        int nang = 0;
        for (int t0 = 0; t0 < a.nori; t0 += 64) {
            const int t = t0 + lane;
            bool valid = false;
            float X = 0, Y = 0;
            if (t < a.nori) {
                const int x = cv_round_f(kp.x + a.apt[2 * t] * s - (float)(gws - 1) / 2);
                const int y = cv_round_f(kp.y + a.apt[2 * t + 1] * s - (float)(gws - 1) / 2);
                valid = !(y < 0 || y >= sh - gws || x < 0 || x >= sw - gws);
                if (valid) {
                    const int32_t* p = a.sum + (size_t)y * sw + x;
                    const float vx = haar(p, gx, 2), vy = haar(p, gy, 2);
                    X = vx * a.aptw[t];
                    Y = vy * a.aptw[t];
                }
            }
            const unsigned long long bal = __ballot(valid);
            if (valid) {
                const int slot = nang + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                s_X[slot] = X;
                s_Y[slot] = Y;
                s_A[slot] = cv_round_f(atan2_deg(Y, X));  // phase(X, Y, angle, true), then cvRound
            }
            nang += __popcll(bal);
        }
        __syncthreads();
        if (nang == 0) {
            if (lane == 0) a.kps[k].size = -1;
            __syncthreads();
            continue;
        }
        // the 72 sliding windows i = 0, 5, ..., 355: lane l takes i = 5l and (l < 8) 320 + 5l
        float bm = -1.f, bx = 0, by = 0;
        int bi = 1 << 30;
        for (int r = 0; r < 2; ++r) {
            const int wi = r == 0 ? 5 * lane : 320 + 5 * lane;
            if (r == 1 && lane >= 8) break;
            const float fi = (float)wi;
            float sx = 0, sy = 0;
            for (int t = 0; t < nang; ++t) {
                const int d = (int)fabsf(s_A[t] - fi);
                if (d < kOriWin / 2 || d > 360 - kOriWin / 2) {
                    sx += s_X[t];
                    sy += s_Y[t];
                }
            }
            const float m = sx * sx + sy * sy;
            if (m > 0 && m > bm) {  // the first window (smallest i) of a lane's best value
                bm = m;
                bx = sx;
                by = sy;
                bi = wi;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float om = __shfl_xor(bm, off), ox = __shfl_xor(bx, off), oy = __shfl_xor(by, off);
            const int oi = __shfl_xor(bi, off);
            if (om > bm || (om == bm && oi < bi)) {
                bm = om;
                bx = ox;
                by = oy;
                bi = oi;
            }
        }
        const float bestx = bm > 0 ? bx : 0.f, besty = bm > 0 ? by : 0.f;
        float dir = atan2_deg(-besty, bestx);
        kp.angle = dir;
        // ---- the rotated window of side n = (int)(21 s), INTER_AREA to 21 x 21
        const int n = (int)((kPatch + 1) * s);
        if (n > kMaxWin) {
            if (lane == 0) {
                a.kps[k].size = -1;
                atomicOr(a.flags, 4);
            }
            __syncthreads();
            continue;
        }
        dir *= (float)(M_PI / 180);
        const float sin_dir = -(float)sin((double)dir), cos_dir = (float)cos((double)dir);
        if (lane == 0) {  // start_x += sin_dir, start_y += cos_dir per row: a sequential float chain
            const float off = -(float)(n - 1) / 2;
            float start_x = kp.x + off * cos_dir + off * sin_dir;
            float start_y = kp.y - off * sin_dir + off * cos_dir;
            for (int i = 0; i < n; ++i, start_x += sin_dir, start_y += cos_dir) {
                s_sx[i] = start_x;
                s_sy[i] = start_y;
            }
        }
        const double inv_scale = (double)kP1 / n, scale = 1. / inv_scale;
        const int iscale = cv_round_d(scale);
        const bool fast = fabs(scale - iscale) < DBL_EPSILON;
        if (!fast) {
            if (lane < kP1) {  // computeResizeAreaTab, per destination cell
                const double fsx1 = lane * scale, fsx2 = fsx1 + scale;
                const double cell = fmin(scale, n - fsx1);
                int sx1 = cv_ceil_d(fsx1), sx2 = cv_floor_d(fsx2);
                sx2 = min(sx2, n - 1);
                sx1 = min(sx1, sx2);
                AreaCell c;
                c.s1 = sx1;
                c.s2 = sx2;
                c.has_l = sx1 - fsx1 > 1e-3;
                c.al = (float)((sx1 - fsx1) / cell);
                c.af = float(1.0 / cell);
                c.has_r = fsx2 - sx2 > 1e-3;
                c.ar = (float)(fmin(fmin(fsx2 - sx2, 1.), cell) / cell);
                s_cell[lane] = c;
            }
            for (int i = lane; i < n; i += 64) {
                s_e0[i] = -1;
                s_e1[i] = -1;
            }
            __syncthreads();
            if (lane == 0) {  // which cells each source column feeds, cell order
                auto put = [&](int sx, int dx, float al) {
                    if (s_e0[sx] < 0) {
                        s_e0[sx] = (int16_t)dx;
                        s_a0[sx] = al;
                    } else {
                        s_e1[sx] = (int16_t)dx;
                        s_a1[sx] = al;
                    }
                };
                int acc = 0;
                for (int dx = 0; dx < kP1; ++dx) {
                    const AreaCell c = s_cell[dx];
                    if (c.has_l) put(c.s1 - 1, dx, c.al);
                    for (int sx = c.s1; sx < c.s2; ++sx) put(sx, dx, c.af);
                    if (c.has_r) put(c.s2, dx, c.ar);
                    s_pre[dx] = acc;
                    acc += c.has_l + (c.s2 - c.s1) + c.has_r;
                }
                s_pre[kP1] = acc;
            }
        } else if (lane <= kP1) {
            s_pre[lane] = lane * iscale;  // output row dy takes source rows dy*iscale .. + iscale - 1
        }
        __syncthreads();
        const int total = s_pre[kP1];
        float fsum = 0;
        int isum = 0, cur = -1;
        for (int j0 = 0; j0 < total; j0 += 64) {
            const int j = j0 + lane;
            if (j < total) {
                int dy = 0;
                while (dy + 1 < kP1 && s_pre[dy + 1] <= j) ++dy;
                const int q = j - s_pre[dy];
                int sy;
                float beta = 1.f;
                if (fast) {
                    sy = dy * iscale + q;
                } else {
                    const AreaCell c = s_cell[dy];
                    if (c.has_l && q == 0) {
                        sy = c.s1 - 1;
                        beta = c.al;
                    } else {
                        const int qq = q - c.has_l;
                        sy = c.s1 + qq;
                        beta = qq < c.s2 - c.s1 ? c.af : c.ar;
                    }
                }
                s_edy[lane] = dy;
                s_ebeta[lane] = beta;
                float* buf = s_buf[lane];
                for (int dx = 0; dx < kP1; ++dx) buf[dx] = 0;
                double px = s_sx[sy], py = s_sy[sy];
                for (int x0 = 0; x0 < n; x0 += 8) {  // 8 samples' image reads in flight
                    uint8_t v[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        v[q] = x0 + q < n ? win_sample(a, px, py) : 0;
                        px += cos_dir;  // the reference's per-pixel accumulation (done for the
                        py -= sin_dir;  // padding samples too: they are never read back)
                    }
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int x = x0 + q;
                        if (x >= n) break;
                        if (fast) {
                            reinterpret_cast<int*>(buf)[x / iscale] += v[q];
                        } else {
                            const int e0 = s_e0[x], e1 = s_e1[x];
                            if (e0 >= 0) buf[e0] += v[q] * s_a0[x];
                            if (e1 >= 0) buf[e1] += v[q] * s_a1[x];
                        }
                    }
                }
            }
            __syncthreads();
            if (lane < kP1) {  // the ytab loop of ResizeArea_Invoker for column dx = lane
                const int cn = min(64, total - j0);
                for (int e = 0; e < cn; ++e) {
                    const int dy = s_edy[e];
                    if (fast) {
                        const int v = reinterpret_cast<const int*>(s_buf[e])[lane];
                        if (dy != cur) {
                            if (cur >= 0)
                                s_P[cur][lane] = iscale == 2 ? (uint8_t)((isum + 2) >> 2)
                                                             : (uint8_t)min(255, max(0, cv_round_f(isum * (1.f / (iscale * iscale)))));
                            isum = v;
                            cur = dy;
                        } else {
                            isum += v;
                        }
                    } else {
                        const float bv = s_ebeta[e] * s_buf[e][lane];
                        if (dy != cur) {
                            if (cur >= 0) s_P[cur][lane] = (uint8_t)min(255, max(0, cv_round_f(fsum)));
                            fsum = bv;
                            cur = dy;
                        } else {
                            fsum += bv;
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (lane < kP1 && cur >= 0)
            s_P[cur][lane] = fast ? (iscale == 2 ? (uint8_t)((isum + 2) >> 2)
                                                 : (uint8_t)min(255, max(0, cv_round_f(isum * (1.f / (iscale * iscale))))))
                                  : (uint8_t)min(255, max(0, cv_round_f(fsum)));
        __syncthreads();
        // ---- gradients with wavelets of size 2s, Gaussian weighted; the 4x4x4 sums
        for (int c = lane; c < kPatch * kPatch; c += 64) {
            const int i = c / kPatch, j = c - i * kPatch;
            const float dw = a.gdesc[i] * a.gdesc[j];
            s_DX[c] = (s_P[i][j + 1] - s_P[i][j] + s_P[i + 1][j + 1] - s_P[i + 1][j]) * dw;
            s_DY[c] = (s_P[i + 1][j] - s_P[i][j] + s_P[i + 1][j + 1] - s_P[i][j + 1]) * dw;
        }
        __syncthreads();
        if (lane < 16) {
            const int i = lane >> 2, j = lane & 3;
            float v0 = 0, v1 = 0, v2 = 0, v3 = 0;
            for (int y = i * 5; y < i * 5 + 5; ++y)
                for (int x = j * 5; x < j * 5 + 5; ++x) {
                    const float tx = s_DX[y * kPatch + x], ty = s_DY[y * kPatch + x];
                    v0 += tx;
                    v1 += ty;
                    v2 += fabsf(tx);
                    v3 += fabsf(ty);
                }
            s_vec[lane * 4 + 0] = v0;
            s_vec[lane * 4 + 1] = v1;
            s_vec[lane * 4 + 2] = v2;
            s_vec[lane * 4 + 3] = v3;
        }
        __syncthreads();
        double mag = 0;
        for (int q = 0; q < 64; ++q) mag += (double)(s_vec[q] * s_vec[q]);  // every lane: the same sequence
        const float sc = (float)(1. / (sqrt(mag) + FLT_EPSILON));
        a.dtmp[(size_t)k * 64 + lane] = s_vec[lane] * sc;
        if (lane == 0) a.kps[k].angle = kp.angle;
        __syncthreads();
    }
}

// ---- drop the keypoints marked size -1 (in order) ----------------------------------
__global__ __launch_bounds__(kSortNT) void compact_kernel(SurfArgs a) {
    const int n = min(*a.nraw, a.kp_cap);
    __shared__ int s_part[kSortNT];
    const int per = (n + kSortNT - 1) / kSortNT;
    const int i0 = min(n, (int)threadIdx.x * per), i1 = min(n, i0 + per);
    int cnt = 0;
    for (int i = i0; i < i1; ++i) cnt += a.kps[i].size > 0;
    s_part[threadIdx.x] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int t = 0; t < kSortNT; ++t) {
            const int v = s_part[t];
            s_part[t] = acc;
            acc += v;
        }
        *a.nout = acc;
    }
    __syncthreads();
    int pos = s_part[threadIdx.x];
    for (int i = i0; i < i1; ++i) {  // destination of each kept keypoint (order: a.order, free after the sort)
        const bool keep = a.kps[i].size > 0;
        a.order[i] = keep ? pos : -1;
        if (keep) a.out[pos++] = a.kps[i];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n * 64; e += kSortNT) {  // descriptors: flat, coalesced
        const int i = e >> 6, d = a.order[i];
        if (d >= 0) a.desc[(size_t)d * 64 + (e & 63)] = a.dtmp[e];
    }
}

}  // namespace

hipError_t launch_surf(const SurfArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(row_scan_kernel, dim3(a.h), dim3(256), 0, s, a);
    hipLaunchKernelGGL(col_scan_kernel, dim3((a.w + 1 + 255) / 256), dim3(256), 0, s, a);
    const int64_t samples0 = (int64_t)a.h * a.w;  // an upper bound of every layer's sample count
    hipLaunchKernelGGL(hessian_kernel, dim3((unsigned)((samples0 + 255) / 256), kSurfTot), dim3(256), 0, s, a);
    hipLaunchKernelGGL(extrema_kernel, dim3((unsigned)((samples0 + 255) / 256), kSurfOct * 3), dim3(256), 0, s, a);
    hipLaunchKernelGGL(sort_kernel, dim3(1), dim3(kSortNT), 0, s, a);
    hipLaunchKernelGGL(describe_kernel, dim3(4096), dim3(64), 0, s, a);
    hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(kSortNT), 0, s, a);
    return hipGetLastError();
}

}  // namespace dvo
