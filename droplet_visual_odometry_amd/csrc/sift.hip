// SIFT_create().detectAndCompute on gfx950: the detector of the reference's
// 'sift' / 'knn_sift' / 'flann' modes (scripts/visual_odometry_v3.py:99-103,
// detectAndCompute at :373), feeding the float k-NN matcher (match.hip).
// Every float expression follows oracle/sift.cpp (the restatement of OpenCV
// 4.x sift.dispatch.cpp / sift.simd.hpp) operation for operation, compiled
// with -ffp-contract=off, so keypoints and descriptors are bit-identical to it.
//
// Pipeline for one image (launch_sift):
//   up2_kernel         u8 -> float, 2x INTER_LINEAR (weights 0/.25/.75: exact)
//   blur_rows/cols     GaussianBlur: row pass sum_k k[k] S[x-r+k], symmetric
//                      column pass, REFLECT_101; taps computed on the host
//   down2_kernel       INTER_NEAREST half of layer 3 -> next octave's layer 0
//   dog_kernel         DoG layers of an octave
//   extrema_kernel     26-neighbour extrema of the DoG layers 1..3 -> candidates
//   refine_kernel      one wave per candidate: adjustLocalExtrema (wave-uniform
//                      scalar code), the 36-bin orientation histogram (samples in
//                      parallel, accumulated in sample order per bin), peaks
//   sort_kernel        KeyPoint12_LessThan order + removeDuplicatedSorted +
//                      firstOctave = -1 rescale (one workgroup, bitonic network)
//   descriptor_kernel  one wave per keypoint: calcSIFTDescriptor, the 360-bin
//                      trilinear histogram filled in sample order, normalised
#include <cfloat>
#include <climits>

#include "dvo_internal.h"

namespace dvo {
namespace {

constexpr int kLayers = 3;
constexpr float kContrast = 0.04f, kEdge = 10.f, kSigma = 1.6f;
constexpr int kBorderS = 5, kMaxInterp = 5, kOriBins = 36;
constexpr float kOriSigFctr = 1.5f, kOriRadius = 3 * kOriSigFctr, kOriPeak = 0.8f;
constexpr int kDW = 4, kDB = 8, kHistN = (kDW + 2) * (kDW + 2) * (kDB + 2);
constexpr float kDescSclFctr = 3.f, kDescMagThr = 0.2f, kIntDescFctr = 512.f;

__device__ const double c_exptab[64] = {
#include "../../data/sift_exp_tab.inc"
};

__device__ __forceinline__ int rnd(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int refl101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__device__ __forceinline__ float sift_exp(float x) {  // cv::hal::exp32f scalar path
    const double prescale = 1.4426950408889634073599246810019 * 64, postscale = 1. / 64, maxv = 3000. * 64;
    const float A0 = .9670371139572337719125840413672004409288e-2;
    const float A4 = (float)(1.000000000000002438532970795181890933776 / A0);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / A0);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / A0);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / A0);
    const float minval = (float)(-maxv / prescale), maxval = (float)(maxv / prescale);
    float x0 = fminf(fmaxf(x, minval), maxval);
    x0 *= (float)prescale;
    const int xi = rnd(x0);
    x0 = (x0 - (float)xi) * (float)postscale;
    int t = (xi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    const float b = __builtin_bit_cast(float, (uint32_t)t << 23);
    const float poly = (((x0 + A1) * x0 + A2) * x0 + A3) * x0 + A4;
    return b * (float)c_exptab[xi & 63] * poly;
}

__device__ __forceinline__ float atan2_deg(float y, float x) {  // cv::fastAtan2
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__device__ __forceinline__ const float* layer(const SiftArgs& A, int o, int l) { return A.gp + A.gp_off[o * 6 + l]; }
__device__ __forceinline__ const float* dogl(const SiftArgs& A, int o, int l) { return A.dog + A.dog_off[o * 5 + l]; }

__global__ __launch_bounds__(256) void up2_kernel(const uint8_t* src, int w, int h, int stride, float* dst) {
    const int W = 2 * w, H = 2 * h;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const int dy = i / W, dx = i - dy * W;
    float fx = (float)((dx + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    float fy = (float)((dy + 0.5) * 0.5 - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    if (sy < 0) fy = 0, sy = 0;
    if (sy >= h - 1) fy = 0, sy = h - 1;
    const int sy1 = min(sy + 1, h - 1);
    auto hrow = [&](int y) {
        const uint8_t* s = src + (int64_t)y * stride;
        return sx >= w - 1 ? (float)s[w - 1] : (float)s[sx] * (1.f - fx) + (float)s[sx + 1] * fx;
    };
    dst[i] = hrow(sy) * (1.f - fy) + hrow(sy1) * fy;
}

__global__ __launch_bounds__(256) void blur_rows_kernel(const float* src, float* dst, int w, int h, const float* k, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= w * h) return;
    const int y = i / w, x = i - y * w, r = n / 2;
    const float* s = src + (int64_t)y * w;
    float acc = k[0] * s[refl101(x - r, w)];
    for (int t = 1; t < n; ++t) acc += k[t] * s[refl101(x - r + t, w)];
    dst[i] = acc;
}

__global__ __launch_bounds__(256) void blur_cols_kernel(const float* src, float* dst, int w, int h, const float* k, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= w * h) return;
    const int y = i / w, x = i - y * w, r = n / 2;
    float acc = k[r] * src[i] + 0.f;
    for (int t = 1; t <= r; ++t)
        acc += k[r + t] * (src[(int64_t)refl101(y + t, h) * w + x] + src[(int64_t)refl101(y - t, h) * w + x]);
    dst[i] = acc;
}

__global__ __launch_bounds__(256) void down2_kernel(const float* src, int sw, float* dst, int w, int h) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= w * h) return;
    const int y = i / w, x = i - y * w;
    dst[i] = src[(int64_t)(2 * y) * sw + 2 * x];
}

__global__ __launch_bounds__(256) void dog_kernel(SiftArgs A, int o) {
    const int n = A.ow[o] * A.oh[o];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int l = blockIdx.y;
    A.dog[A.dog_off[o * 5 + l] + i] = layer(A, o, l + 1)[i] - layer(A, o, l)[i];
}

__global__ __launch_bounds__(256) void extrema_kernel(SiftArgs A, int o, int threshold) {
    const int w = A.ow[o], h = A.oh[o];
    const int iw = w - 2 * kBorderS, ih = h - 2 * kBorderS;
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int l = 1 + blockIdx.y;
    if (iw <= 0 || ih <= 0 || t >= iw * ih) return;
    const int r = kBorderS + t / iw, c = kBorderS + t % iw;
    const float* cur = dogl(A, o, l);
    const float* prv = dogl(A, o, l - 1);
    const float* nxt = dogl(A, o, l + 1);
    const float val = cur[r * w + c];
    if (!(fabsf(val) > (float)threshold)) return;
    bool ext = val != 0;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            const int q = (r + dy) * w + c + dx;
            if (val > 0) ext &= val >= cur[q] && val >= prv[q] && val >= nxt[q];
            else ext &= val <= cur[q] && val <= prv[q] && val <= nxt[q];
        }
    if (!ext) return;
    const int slot = atomicAdd(A.ncand, 1);
    if (slot < A.cand_cap) A.cand[slot] = make_int4(o, l, r, c);
    else atomicOr(A.flags, 1);
}

// adjustLocalExtrema (oracle/sift.cpp adjust); wave-uniform scalar code
__device__ bool adjust(const SiftArgs& A, dvo_keypoint& kpt, int octv, int& lay, int& r, int& c) {
    const float img_scale = 1.f / 255;
    const float deriv_scale = img_scale * 0.5f, second = img_scale, cross = img_scale * 0.25f;
    const int w = A.ow[octv], h = A.oh[octv];
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < kMaxInterp; i++) {
        const float* img = dogl(A, octv, lay);
        const float* prev = dogl(A, octv, lay - 1);
        const float* next = dogl(A, octv, lay + 1);
        auto I = [&](const float* p, int y, int x) { return p[y * w + x]; };
        const float dD0 = (I(img, r, c + 1) - I(img, r, c - 1)) * deriv_scale;
        const float dD1 = (I(img, r + 1, c) - I(img, r - 1, c)) * deriv_scale;
        const float dD2 = (I(next, r, c) - I(prev, r, c)) * deriv_scale;
        const float v2 = I(img, r, c) * 2;
        const float dxx = (I(img, r, c + 1) + I(img, r, c - 1) - v2) * second;
        const float dyy = (I(img, r + 1, c) + I(img, r - 1, c) - v2) * second;
        const float dss = (I(next, r, c) + I(prev, r, c) - v2) * second;
        const float dxy = (I(img, r + 1, c + 1) - I(img, r + 1, c - 1) - I(img, r - 1, c + 1) + I(img, r - 1, c - 1)) * cross;
        const float dxs = (I(next, r, c + 1) - I(next, r, c - 1) - I(prev, r, c + 1) + I(prev, r, c - 1)) * cross;
        const float dys = (I(next, r + 1, c) - I(next, r - 1, c) - I(prev, r + 1, c) + I(prev, r - 1, c)) * cross;
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys, a22 = dss;
        float X0 = 0, X1 = 0, X2 = 0;
        float d = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
        if (d != 0) {
            d = 1 / d;
            X0 = d * (dD0 * (a11 * a22 - a12 * a21) - a01 * (dD1 * a22 - a12 * dD2) + a02 * (dD1 * a21 - a11 * dD2));
            X1 = d * (a00 * (dD1 * a22 - a12 * dD2) - dD0 * (a10 * a22 - a12 * a20) + a02 * (a10 * dD2 - dD1 * a20));
            X2 = d * (a00 * (a11 * dD2 - dD1 * a21) - a01 * (a10 * dD2 - dD1 * a20) + dD0 * (a10 * a21 - a11 * a20));
        }
        xi = -X2;
        xr = -X1;
        xc = -X0;
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3))
            return false;
        c += rnd(xc);
        r += rnd(xr);
        lay += rnd(xi);
        if (lay < 1 || lay > kLayers || c < kBorderS || c >= w - kBorderS || r < kBorderS || r >= h - kBorderS) return false;
    }
    if (i >= kMaxInterp) return false;
    {
        const float* img = dogl(A, octv, lay);
        const float* prev = dogl(A, octv, lay - 1);
        const float* next = dogl(A, octv, lay + 1);
        auto I = [&](const float* p, int y, int x) { return p[y * w + x]; };
        const float dD0 = (I(img, r, c + 1) - I(img, r, c - 1)) * deriv_scale;
        const float dD1 = (I(img, r + 1, c) - I(img, r - 1, c)) * deriv_scale;
        const float dD2 = (I(next, r, c) - I(prev, r, c)) * deriv_scale;
        const float t = dD0 * xc + dD1 * xr + dD2 * xi;
        contr = I(img, r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * kLayers < kContrast) return false;
        const float v2 = I(img, r, c) * 2.f;
        const float dxx = (I(img, r, c + 1) + I(img, r, c - 1) - v2) * second;
        const float dyy = (I(img, r + 1, c) + I(img, r - 1, c) - v2) * second;
        const float dxy = (I(img, r + 1, c + 1) - I(img, r + 1, c - 1) - I(img, r - 1, c + 1) + I(img, r - 1, c - 1)) * cross;
        const float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * kEdge >= (kEdge + 1) * (kEdge + 1) * det) return false;
    }
    kpt.x = (c + xc) * (float)(1 << octv);
    kpt.y = (r + xr) * (float)(1 << octv);
    kpt.octave = octv + (lay << 8) + ((int)__builtin_rint((xi + 0.5) * 255) << 16);
    kpt.size = kSigma * (float)exp2((double)((lay + xi) / kLayers)) * (float)(1 << octv) * 2;
    kpt.response = fabsf(contr);
    kpt.angle = 0;
    kpt.class_id = -1;
    return true;
}

// One wave per candidate (grid-stride over the candidate list).
__global__ __launch_bounds__(64) void refine_kernel(SiftArgs A) {
    const int lane = threadIdx.x;
    const int ncand = min(*A.ncand, A.cand_cap);
    for (int e = blockIdx.x; e < ncand; e += gridDim.x) {
        const int4 cd = A.cand[e];
        const int o = cd.x;
        int lay = cd.y, r = cd.z, c = cd.w;
        dvo_keypoint kpt;
        if (!adjust(A, kpt, o, lay, r, c)) continue;
        // calcOrientationHist on the Gaussian layer, centre (c, r)
        const float scl_octv = kpt.size * 0.5f / (float)(1 << o);
        const int radius = rnd(kOriRadius * scl_octv);
        const float sigma = kOriSigFctr * scl_octv;
        const float expf_scale = -1.f / (2.f * sigma * sigma);
        const float* img = layer(A, o, lay);
        const int w = A.ow[o], h = A.oh[o];
        const int side = 2 * radius + 1, total = side * side;
        float th = 0.f;  // lane b < 36 holds temphist[b]
        for (int t0 = 0; t0 < total; t0 += 64) {
            const int t = t0 + lane;
            const int i = t / side - radius, j = t % side - radius;
            const int y = r + i, x = c + j;
            const bool ok = t < total && y > 0 && y < h - 1 && x > 0 && x < w - 1;
            int bin = 0;
            float v = 0.f;
            if (ok) {
                const float dx = img[y * w + x + 1] - img[y * w + x - 1];
                const float dy = img[(y - 1) * w + x] - img[(y + 1) * w + x];
                const float wt = sift_exp((float)(i * i + j * j) * expf_scale);
                const float ori = atan2_deg(dy, dx);
                const float mag = __builtin_sqrtf(dx * dx + dy * dy);
                bin = rnd((kOriBins / 360.f) * ori);
                if (bin >= kOriBins) bin -= kOriBins;
                if (bin < 0) bin += kOriBins;
                v = wt * mag;
            }
            // temphist[bin] += W * Mag in sample order: the owner lane of each bin adds
            unsigned long long m = __ballot(ok);
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                const int bk = __builtin_amdgcn_readlane(bin, k);
                const float vk = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
                if (lane == bk) th += vk;
            }
        }
        // smoothing with the circular neighbours, max, peaks
        auto th_at = [&](int b) { return __shfl(th, (b + kOriBins) % kOriBins); };
        const int b = lane < kOriBins ? lane : 0;
        const float tm2 = th_at(b - 2), tp2 = th_at(b + 2), tm1 = th_at(b - 1), tp1 = th_at(b + 1);
        const float hist = (tm2 + tp2) * (1.f / 16.f) + (tm1 + tp1) * (4.f / 16.f) + th * (6.f / 16.f);
        float mx = lane < kOriBins ? hist : -FLT_MAX;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
        const float mag_thr = mx * kOriPeak;
        const float hl = __shfl(hist, (b + kOriBins - 1) % kOriBins), hr = __shfl(hist, (b + 1) % kOriBins);
        if (lane < kOriBins && hist > hl && hist > hr && hist >= mag_thr) {
            float bn = (float)lane + 0.5f * (hl - hr) / (hl - 2 * hist + hr);
            bn = bn < 0 ? kOriBins + bn : bn >= kOriBins ? bn - kOriBins : bn;
            dvo_keypoint q = kpt;
            q.angle = 360.f - (360.f / kOriBins) * bn;
            if (fabsf(q.angle - 360.f) < FLT_EPSILON) q.angle = 0.f;
            const int slot = atomicAdd(A.nraw, 1);
            if (slot < A.kp_cap) A.raw[slot] = q;
            else atomicOr(A.flags, 2);
        }
    }
}

__device__ __forceinline__ bool kp_less(const dvo_keypoint& a, const dvo_keypoint& b) {  // KeyPoint12_LessThan
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    return a.octave > b.octave;
}

// removeDuplicatedSorted + the firstOctave = -1 rescale, one workgroup.
constexpr int kSortNT = 1024;
__global__ __launch_bounds__(kSortNT) void sort_kernel(SiftArgs A) {
    const int n = min(*A.nraw, A.kp_cap);
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    int32_t* idx = A.order;
    for (int i = threadIdx.x; i < n2; i += kSortNT) idx[i] = i < n ? i : -1;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += kSortNT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = idx[i], b = idx[ixj];
                    // -1 (padding) sorts last
                    const bool a_gt_b = a < 0 ? b >= 0 : (b >= 0 && kp_less(A.raw[b], A.raw[a]));
                    if (a_gt_b == ((i & k) == 0)) {
                        idx[i] = b;
                        idx[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    // keep[i] = the first of its (x, y, size, angle) run; compaction in order
    __shared__ int s_part[kSortNT];
    const int per = (n + kSortNT - 1) / kSortNT;
    const int i0 = min(n, (int)threadIdx.x * per), i1 = min(n, i0 + per);
    auto keep = [&](int i) {
        if (i == 0) return true;
        const dvo_keypoint &p = A.raw[idx[i - 1]], &q = A.raw[idx[i]];
        return p.x != q.x || p.y != q.y || p.size != q.size || p.angle != q.angle;
    };
    int cnt = 0;
    for (int i = i0; i < i1; ++i) cnt += keep(i);
    s_part[threadIdx.x] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int t = 0; t < kSortNT; ++t) {
            const int v = s_part[t];
            s_part[t] = acc;
            acc += v;
        }
        *A.nkp = acc;
    }
    __syncthreads();
    int pos = s_part[threadIdx.x];
    for (int i = i0; i < i1; ++i)
        if (keep(i)) {
            dvo_keypoint q = A.raw[idx[i]];
            q.x = q.x * 0.5f;
            q.y = q.y * 0.5f;
            q.size = q.size * 0.5f;
            q.octave = (q.octave & ~255) | ((q.octave - 1) & 255);
            A.kps[pos++] = q;
        }
}

// calcSIFTDescriptor, one wave per keypoint (grid-stride).
__global__ __launch_bounds__(64) void descriptor_kernel(SiftArgs A) {
    __shared__ float hist[kHistN];
    __shared__ int s_idx[64];
    __shared__ float s_v[64][8];
    const int lane = threadIdx.x;
    const int nk = *A.nkp;
    constexpr int d = kDW, n = kDB;
    const int off[8] = {0, 1, n + 2, n + 3, (d + 2) * (n + 2), (d + 2) * (n + 2) + 1, (d + 3) * (n + 2), (d + 3) * (n + 2) + 1};
    for (int e = blockIdx.x; e < nk; e += gridDim.x) {
        const dvo_keypoint kp = A.kps[e];
        const int ob = kp.octave & 255, lay = (kp.octave >> 8) & 255;
        const int octv = ob < 128 ? ob : (-128 | ob);
        const float scale = octv >= 0 ? 1.f / (float)(1 << octv) : (float)(1 << -octv);
        const float size = kp.size * scale;
        const float ptx = kp.x * scale, pty = kp.y * scale;
        float ori = 360.f - kp.angle;
        if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
        const float scl = size * 0.5f;
        const int o = octv + 1;
        const float* img = layer(A, o, lay);
        const int w = A.ow[o], h = A.oh[o];
        const int px = rnd(ptx), py = rnd(pty);
        const float ang = ori * (float)(M_PI / 180);
        double sd, cdv;
        sincos((double)ang, &sd, &cdv);
        float cos_t = (float)cdv, sin_t = (float)sd;
        const float bins_per_rad = n / 360.f;
        const float exp_scale = -1.f / (d * d * 0.5f);
        const float hist_width = kDescSclFctr * scl;
        int radius = rnd(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
        radius = min(radius, (int)sqrt(((double)w) * w + ((double)h) * h));
        cos_t /= hist_width;
        sin_t /= hist_width;
        for (int q = lane; q < kHistN; q += 64) hist[q] = 0.f;
        const int side = 2 * radius + 1;
        const int64_t total = (int64_t)side * side;
        for (int64_t t0 = 0; t0 < total; t0 += 64) {
            const int64_t t = t0 + lane;
            const int i = (int)(t / side) - radius, j = (int)(t % side) - radius;
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            float rbin = r_rot + d / 2 - 0.5f;
            float cbin = c_rot + d / 2 - 0.5f;
            const int r = py + i, c = px + j;
            const bool ok = t < total && rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < h - 1 && c > 0 &&
                            c < w - 1;
            __syncthreads();
            if (ok) {
                const float dx = img[r * w + c + 1] - img[r * w + c - 1];
                const float dy = img[(r - 1) * w + c] - img[(r + 1) * w + c];
                const float wt = sift_exp((c_rot * c_rot + r_rot * r_rot) * exp_scale);
                const float og = atan2_deg(dy, dx);
                const float m = __builtin_sqrtf(dx * dx + dy * dy);
                float obin = (og - ori) * bins_per_rad;
                const float mag = m * wt;
                const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                int o0 = (int)floorf(obin);
                rbin -= r0;
                cbin -= c0;
                obin -= o0;
                if (o0 < 0) o0 += n;
                if (o0 >= n) o0 -= n;
                const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
                const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
                const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
                const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
                const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
                const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
                const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
                s_idx[lane] = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
                s_v[lane][0] = v_rco000;
                s_v[lane][1] = v_rco001;
                s_v[lane][2] = v_rco010;
                s_v[lane][3] = v_rco011;
                s_v[lane][4] = v_rco100;
                s_v[lane][5] = v_rco101;
                s_v[lane][6] = v_rco110;
                s_v[lane][7] = v_rco111;
            }
            __syncthreads();
            // the samples' 8 bins each, in sample order; within a sample the 8 bins differ
            unsigned long long m = __ballot(ok);
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                if (lane < 8) {
                    const int q = s_idx[k] + off[lane];
                    hist[q] = hist[q] + s_v[k][lane];
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        // circular orientation wrap, then the 128 raw values
        __shared__ float raw[kDW * kDW * kDB];
        if (lane < d * d) {
            const int i = lane / d, j = lane % d;
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            hist[idx] = hist[idx] + hist[idx + n];
            hist[idx + 1] = hist[idx + 1] + hist[idx + n + 1];
            for (int k = 0; k < n; k++) raw[(i * d + j) * n + k] = hist[idx + k];
        }
        __syncthreads();
        __shared__ float s_scale[2];
        if (lane == 0) {
            float nrm2 = 0;
            for (int k = 0; k < d * d * n; k++) nrm2 += raw[k] * raw[k];
            const float thr = __builtin_sqrtf(nrm2) * kDescMagThr;
            nrm2 = 0;
            for (int k = 0; k < d * d * n; k++) {
                const float v = fminf(raw[k], thr);
                nrm2 += v * v;
            }
            s_scale[0] = thr;
            s_scale[1] = kIntDescFctr / fmaxf(__builtin_sqrtf(nrm2), FLT_EPSILON);
        }
        __syncthreads();
        for (int k = lane; k < d * d * n; k += 64) {
            const float v = fminf(raw[k], s_scale[0]);
            const int q = rnd(v * s_scale[1]);
            A.desc[(int64_t)e * 128 + k] = (float)min(max(q, 0), 255);
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_sift(const SiftArgs& A, const uint8_t* d_img, int w, int h, int stride, const float* d_taps,
                       const int* tap_off, const int* tap_n, hipStream_t s) {
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    float* base = A.gp + A.gp_off[0];
    hipLaunchKernelGGL(up2_kernel, grid((int64_t)A.ow[0] * A.oh[0]), dim3(256), 0, s, d_img, w, h, stride, base);
    auto blur = [&](const float* src, float* dst, int o, int which) {
        const int64_t npx = (int64_t)A.ow[o] * A.oh[o];
        hipLaunchKernelGGL(blur_rows_kernel, grid(npx), dim3(256), 0, s, src, A.tmp, A.ow[o], A.oh[o], d_taps + tap_off[which],
                           tap_n[which]);
        hipLaunchKernelGGL(blur_cols_kernel, grid(npx), dim3(256), 0, s, A.tmp, dst, A.ow[o], A.oh[o], d_taps + tap_off[which],
                           tap_n[which]);
    };
    blur(base, base, 0, 0);
    for (int o = 0; o < A.noct; ++o) {
        if (o > 0)
            hipLaunchKernelGGL(down2_kernel, grid((int64_t)A.ow[o] * A.oh[o]), dim3(256), 0, s, A.gp + A.gp_off[(o - 1) * 6 + 3],
                               A.ow[o - 1], A.gp + A.gp_off[o * 6], A.ow[o], A.oh[o]);
        for (int l = 1; l < 6; ++l) blur(A.gp + A.gp_off[o * 6 + l - 1], A.gp + A.gp_off[o * 6 + l], o, l);
        dim3 dg = grid((int64_t)A.ow[o] * A.oh[o]);
        dg.y = 5;
        hipLaunchKernelGGL(dog_kernel, dg, dim3(256), 0, s, A, o);
    }
    const int threshold = (int)floor(0.5 * kContrast / kLayers * 255);
    for (int o = 0; o < A.noct; ++o) {
        const int iw = A.ow[o] - 2 * kBorderS, ih = A.oh[o] - 2 * kBorderS;
        if (iw <= 0 || ih <= 0) continue;
        dim3 eg = grid((int64_t)iw * ih);
        eg.y = kLayers;
        hipLaunchKernelGGL(extrema_kernel, eg, dim3(256), 0, s, A, o, threshold);
    }
    hipLaunchKernelGGL(refine_kernel, dim3(4096), dim3(64), 0, s, A);
    hipLaunchKernelGGL(sort_kernel, dim3(1), dim3(kSortNT), 0, s, A);
    hipLaunchKernelGGL(descriptor_kernel, dim3(4096), dim3(64), 0, s, A);
    return hipGetLastError();
}

}  // namespace dvo
