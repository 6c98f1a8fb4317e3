// TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of
// cv::ORB::detectAndCompute as called at scripts/visual_odometry_v3.py:373 with
// the cv.ORB_create() defaults chosen at scripts/visual_odometry_v3.py:96
// (nfeatures=500, scaleFactor=1.2f, nlevels=8, edgeThreshold=31, firstLevel=0,
// WTA_K=2, HARRIS_SCORE, patchSize=31, fastThreshold=20).  Follows OpenCV 4.x
// modules/features2d/src/orb.cpp, fast.cpp, keypoint.cpp and
// imgproc resize.cpp (INTER_LINEAR_EXACT) / filter.cpp (8-bit separable path).
// Compiled with -ffp-contract=off: every float/double expression below is
// evaluated in source order without FMA contraction, as OpenCV's SSE2 baseline.
#include "oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

const int kPattern[256 * 4] = {
#include "../data/orb_bit_pattern_31.inc"
};

const int kOcv4 = 0, kOcv32 = 1;  // ora_*_v semantics: OpenCV 4.x (default) or 3.2
const double kScaleFactor = (double)1.2f;  // ORB_Impl::scaleFactor (double member set from 1.2f)
const int kEdgeThreshold = 31;
const int kPatchSize = 31;
const int kFastThreshold = 20;
const float kHarrisK = 0.04f;

inline int cv_round(float v) { return (int)lrintf(v); }    // cvRound(float): nearest-even
inline int cv_round(double v) { return (int)lrint(v); }    // cvRound(double)
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }

// orb.cpp getScale(level, firstLevel=0, scaleFactor)
inline float get_scale(int level) { return (float)std::pow(kScaleFactor, (double)level); }

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
};

struct KP {
    float x, y, size, angle, response;
    int octave;
};

// ---------------------------------------------------------------------------
// resize(INTER_LINEAR_EXACT): resize.cpp resize_bitExact<uchar, interpolationLinear<uchar>>.
// Coefficients are ufixedpoint16 (8 fractional bits), computed in softdouble
// (= IEEE double); horizontal pass keeps 8.8 sums, vertical pass rounds
// (sum + 2^15) >> 16.
struct LinCoeffs {
    std::vector<int> ofs;
    std::vector<uint16_t> c0, c1;
    int minofst = 0, maxofst = 0;
};

LinCoeffs linear_coeffs(int srcsize, int dstsize) {
    LinCoeffs lc;
    lc.ofs.assign(dstsize, 0);
    lc.c0.assign(dstsize, 0);
    lc.c1.assign(dstsize, 0);
    const double inv_scale = (double)dstsize / srcsize;   // resize(): inv_scale_x = dsize.width/ssize.width
    const double scale = 1.0 / inv_scale;                 // softdouble::one() / softdouble(inv_scale)
    lc.minofst = 0;
    lc.maxofst = dstsize;
    for (int val = 0; val < dstsize; ++val) {
        double fval = scale * ((double)val + 0.5) - 0.5;
        int ival = cv_floor(fval);
        if (ival >= 0 && srcsize > 1) {
            if (ival < srcsize - 1) {
                lc.ofs[val] = ival;
                uint16_t c1 = (uint16_t)cv_round((fval - (double)ival) * 256.0);
                lc.c1[val] = c1;
                lc.c0[val] = (uint16_t)(256 > c1 ? 256 - c1 : 0);
            } else {
                lc.ofs[val] = srcsize - 1;
                lc.maxofst = std::min(lc.maxofst, val);
            }
        } else {
            lc.minofst = std::max(lc.minofst, val + 1);
        }
    }
    return lc;
}

void resize_linear_exact(const Img& src, Img& dst, int dw, int dh) {
    dst.w = dw;
    dst.h = dh;
    dst.px.assign((size_t)dw * dh, 0);
    LinCoeffs cx = linear_coeffs(src.w, dw), cy = linear_coeffs(src.h, dh);
    auto hline = [&](int sy, std::vector<uint16_t>& out) {
        const uint8_t* s = &src.px[(size_t)sy * src.w];
        out.resize(dw);
        int i = 0;
        for (; i < cx.minofst; ++i) out[i] = (uint16_t)(s[0] << 8);
        for (; i < cx.maxofst; ++i) {
            const uint8_t* p = s + cx.ofs[i];
            out[i] = (uint16_t)(cx.c0[i] * p[0] + cx.c1[i] * p[1]);
        }
        uint16_t edge = (uint16_t)(s[cx.ofs[dw - 1]] << 8);
        for (; i < dw; ++i) out[i] = edge;
    };
    std::vector<uint16_t> h0, h1;
    for (int dy = 0; dy < dh; ++dy) {
        uint8_t* d = &dst.px[(size_t)dy * dw];
        if (dy < cy.minofst || dy >= cy.maxofst) {
            hline(dy < cy.minofst ? 0 : src.h - 1, h0);
            for (int i = 0; i < dw; ++i) d[i] = (uint8_t)std::min(255, (h0[i] + 128) >> 8);
            continue;
        }
        int iy = cy.ofs[dy];
        hline(iy, h0);
        hline(iy + 1, h1);
        uint32_t w0 = cy.c0[dy], w1 = cy.c1[dy];
        for (int i = 0; i < dw; ++i) {
            uint32_t v = (uint32_t)h0[i] * w0 + (uint32_t)h1[i] * w1;
            d[i] = (uint8_t)std::min<uint32_t>(255, (v + 32768) >> 16);
        }
    }
}

// resize(INTER_LINEAR) as OpenCV 3.2 ran it for ORB's pyramid (imgwarp.cpp
// resize -> resizeGeneric_ with HResizeLinear<uchar,int,short,2048> and
// VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,VResizeLinearVec_32s8u>;
// 4.x switched ORB to INTER_LINEAR_EXACT).  Per destination column:
//   fx = (float)((dx + 0.5) * scale_x - 0.5), sx = cvFloor(fx), fx -= sx,
//   clamped to sx = 0 / sx = W-1 (fx = 0) at the edges, and the 11-bit weights
//   saturate_cast<short>((1 - fx) * 2048), saturate_cast<short>(fx * 2048)
//   (each cvRound-ed on its own, so they may sum to 2047 or 2049);
// rows the same with the source rows clipped to [0, H-1].  The horizontal
// pass is exact int (S[sx] a0 + S[sx+1] a1; S[W-1] * 2048 past xmax).  The
// vertical pass has two forms on x86: the SSE2 VResizeLinearVec_32s8u for
// x < xs, ((mulhi(S0 >> 4, b0) + mulhi(S1 >> 4, b1) + 2) >> 2) in 16-bit
// lanes, and the scalar FixedPtCast (S0 b0 + S1 b1 + 2^21) >> 22 for the last
// columns; xs = where the 16-wide loop (x <= W-16) and then the 4-wide loop
// (x < W-4) stop.  Assumes a build without IPP (distribution packages of 3.2
// disable IPPICV).
int ocv32_simd_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

void resize_linear_32(const Img& src, Img& dst, int dw, int dh) {
    dst.w = dw;
    dst.h = dh;
    dst.px.assign((size_t)dw * dh, 0);
    const double scale_x = 1. / ((double)dw / src.w), scale_y = 1. / ((double)dh / src.h);
    auto sat_short = [](float v) { return (int)std::max(-32768, std::min(32767, cv_round(v))); };
    std::vector<int> xofs(dw), ia(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= src.w) {
            xmax = std::min(xmax, dx);
            if (sx >= src.w - 1) fx = 0, sx = src.w - 1;
        }
        xofs[dx] = sx;
        ia[2 * dx] = sat_short((1.f - fx) * 2048);
        ia[2 * dx + 1] = sat_short(fx * 2048);
    }
    auto hline = [&](int sy, std::vector<int>& out) {
        const uint8_t* S = &src.px[(size_t)sy * src.w];
        out.resize(dw);
        for (int dx = 0; dx < dw; ++dx)
            out[dx] = dx < xmax ? S[xofs[dx]] * ia[2 * dx] + S[xofs[dx] + 1] * ia[2 * dx + 1] : S[xofs[dx]] * 2048;
    };
    auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
    const int xs = ocv32_simd_end(dw);
    std::vector<int> h0, h1;
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        hline(clip(sy, 0, src.h), h0);
        hline(clip(sy + 1, 0, src.h), h1);
        uint8_t* d = &dst.px[(size_t)dy * dw];
        for (int x = 0; x < dw; ++x) {
            int v;
            if (x < xs)  // _mm_mulhi_epi16 = (a * b) >> 16; the 16-bit adds never saturate here
                v = ((((h0[x] >> 4) * b0) >> 16) + (((h1[x] >> 4) * b1) >> 16) + 2) >> 2;
            else
                v = (h0[x] * b0 + h1[x] * b1 + (1 << 21)) >> 22;
            d[x] = (uint8_t)std::min(255, std::max(0, v));
        }
    }
}

// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on a pyramid ROI (orb.cpp
// detectAndCompute).  ORB blurs a submatrix without BORDER_ISOLATED, so OpenCV
// (3.2 and 4.x alike) takes sepFilter2D's 8-bit fixed-point path: kernel =
// cvRound(256*g) = {18,34,49,55,49,34,18}, exact int row sums, and the column
// pass SymmColumnFilter<FixedPtCastEx<int,uchar>, SymmColumnVec_32s8u>.  Its
// vector op (SSE2 in 3.2, universal intrinsics in 4.x) covers every column up
// to the last multiple of 4 in float with the kernel scaled by 2^-16: all
// products and partial sums are exact there (< 2^24 units of 2^-16), so the
// result is the exact sum, rounded half to even (cvtps2dq / v_round).  Only
// the last w % 4 columns take the scalar FixedPtCastEx, (sum + 2^15) >> 16,
// which rounds ties up.  The reflect-101 border only feeds pixels the
// descriptor can never sample (keypoints are >= 31 px from the level edge,
// patch reach <= 19), so clamping vs. reflecting is immaterial; reflect-101
// is used for fidelity anyway.
void gaussian_blur7(const Img& src, Img& dst) {
    // getGaussianKernel(7, 2, CV_32F), then convertTo(CV_32S, 256) (= cvRound).
    double sum = 0;
    float g[7];
    for (int i = 0; i < 7; ++i) {
        double x = i - 3.0;
        g[i] = (float)std::exp(-0.5 / (2.0 * 2.0) * x * x);
        sum += g[i];
    }
    int k[7];
    for (int i = 0; i < 7; ++i) k[i] = cv_round((double)(float)(g[i] * (1.0 / sum)) * 256.0);
    const int w = src.w, h = src.h;
    auto refl = [](int p, int n) {
        if (n == 1) return 0;
        while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
        return p;
    };
    std::vector<int> rows((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int i = 0; i < 7; ++i) s += k[i] * src.at(refl(x + i - 3, w), y);
            rows[(size_t)y * w + x] = s;
        }
    dst.w = w;
    dst.h = h;
    dst.px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int i = 0; i < 7; ++i) s += k[i] * rows[(size_t)refl(y + i - 3, h) * w + x];
            const int half_even = x < (w & ~3) ? (s >> 16) & 1 : 1;
            int v = (s + (1 << 15) - 1 + half_even) >> 16;
            dst.px[(size_t)y * w + x] = (uint8_t)std::min(255, std::max(0, v));
        }
}

// ---------------------------------------------------------------------------
// FAST-9/16 (fast.cpp FAST_t<16>, cornerScore<16>) with nonmax suppression.
const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

int corner_score16(const uint8_t* ptr, const int* pixel, int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[N];
    for (int k = 0; k < N; ++k) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

void fast16(const uint8_t* img, int w, int h, int step, int threshold, std::vector<KP>& kps) {
    kps.clear();
    const int K = 8, N = 16 + K + 1;
    int pixel[25];
    for (int k = 0; k < 16; ++k) pixel[k] = kCircle[k][0] + kCircle[k][1] * step;
    for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; ++i) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    std::vector<uint8_t> buf((size_t)w * 3, 0);
    std::vector<int> cpbuf((size_t)(w + 1) * 3, 0);
    uint8_t* bufs[3] = {&buf[0], &buf[w], &buf[2 * w]};
    int* cps[3] = {&cpbuf[0], &cpbuf[w + 1], &cpbuf[2 * (w + 1)]};
    for (int i = 3; i < h - 2; ++i) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = bufs[(i - 3) % 3];
        int* cornerpos = cps[(i - 3) % 3] + 1;
        std::memset(curr, 0, w);
        int ncorners = 0;
        if (i < h - 3) {
            for (int j = 3; j < w - 3; ++j, ++ptr) {
                int v = ptr[0];
                const uint8_t* t = &tab[0] - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; ++k) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; ++k) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = bufs[(i - 4 + 3) % 3];
        const uint8_t* pprev = bufs[(i - 5 + 3) % 3];
        cornerpos = cps[(i - 4 + 3) % 3] + 1;
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; ++k) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1])
                kps.push_back(KP{(float)j, (float)(i - 1), 7.f, -1.f, (float)score, 0});
        }
    }
}

// keypoint.cpp KeyPointsFilter::runByImageBorder (Rect::contains, stable remove_if)
void run_by_image_border(std::vector<KP>& kps, int w, int h, int border) {
    if (h <= border * 2 || w <= border * 2) {
        kps.clear();
        return;
    }
    const float x0 = (float)border, y0 = (float)border;
    const float x1 = (float)(w - border), y1 = (float)(h - border);
    kps.erase(std::remove_if(kps.begin(), kps.end(),
                             [&](const KP& k) { return !(x0 <= k.x && k.x < x1 && y0 <= k.y && k.y < y1); }),
              kps.end());
}

// keypoint.cpp KeyPointsFilter::retainBest: nth_element + partition (libstdc++).
// OpenCV 4.x selects the n-th best (nth_element at begin + n - 1); OpenCV 3.2
// called nth_element at begin + n and then still read the boundary response
// at index n - 1 (semantics == kOcv32), which keeps a different set whenever
// responses tie at the boundary -- with FAST scores they usually do.
template <class T, class Resp>
void retain_best(std::vector<T>& kps, int n_points, Resp resp, int semantics = kOcv4) {
    if (n_points >= 0 && kps.size() > (size_t)n_points) {
        if (n_points == 0) {
            kps.clear();
            return;
        }
        std::nth_element(kps.begin(), kps.begin() + n_points - (semantics == kOcv32 ? 0 : 1), kps.end(),
                         [&](const T& a, const T& b) { return resp(a) > resp(b); });
        float amb = resp(kps[n_points - 1]);
        auto new_end = std::partition(kps.begin() + n_points, kps.end(),
                                      [&](const T& k) { return resp(k) >= amb; });
        kps.resize(new_end - kps.begin());
    }
}

// orb.cpp HarrisResponses(img, layerinfo, pts, blockSize=7, harris_k=0.04f)
void harris_responses(const Img& img, std::vector<KP>& pts, int begin, int end) {
    const int blockSize = 7, r = blockSize / 2;
    const float scale = 1.f / ((1 << 2) * blockSize * 255.f);
    const float scale_sq_sq = scale * scale * scale * scale;
    const int step = img.w;
    for (int p = begin; p < end; ++p) {
        int x0 = cv_round(pts[p].x), y0 = cv_round(pts[p].y);
        const uint8_t* ptr0 = &img.px[(size_t)(y0 - r) * step + (x0 - r)];
        int a = 0, b = 0, c = 0;
        for (int i = 0; i < blockSize; ++i)
            for (int j = 0; j < blockSize; ++j) {
                const uint8_t* ptr = ptr0 + i * step + j;
                int Ix = (ptr[1] - ptr[-1]) * 2 + (ptr[-step + 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[step - 1]);
                int Iy = (ptr[step] - ptr[-step]) * 2 + (ptr[step - 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[-step + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        pts[p].response = ((float)a * b - (float)c * c - kHarrisK * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
    }
}

// core fastAtan2 (mathfuncs_core atan_f32), degrees in [0, 360)
const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

std::vector<int> make_umax(int half) {
    std::vector<int> umax(half + 2);
    int v, v0, vmax = cv_floor(half * std::sqrt(2.f) / 2 + 1);
    int vmin = cv_ceil(half * std::sqrt(2.f) / 2);
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt((double)half * half - v * v));
    for (v = half, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    return umax;
}

// orb.cpp ICAngles
void ic_angles(const Img& img, std::vector<KP>& pts, int begin, int end, const std::vector<int>& umax, int half) {
    const int step = img.w;
    for (int p = begin; p < end; ++p) {
        const uint8_t* center = &img.px[(size_t)cv_round(pts[p].y) * step + cv_round(pts[p].x)];
        int m_01 = 0, m_10 = 0;
        for (int u = -half; u <= half; ++u) m_10 += u * center[u];
        for (int v = 1; v <= half; ++v) {
            int v_sum = 0, d = umax[v];
            for (int u = -d; u <= d; ++u) {
                int vp = center[u + v * step], vm = center[u - v * step];
                v_sum += (vp - vm);
                m_10 += u * (vp + vm);
            }
            m_01 += v * v_sum;
        }
        pts[p].angle = fast_atan2((float)m_01, (float)m_10);
    }
}

// orb.cpp computeOrbDescriptors (WTA_K == 2).  cos/sin: double-precision of
// the float angle, rounded to float (OpenCV `(float)cos(angle)`).
void orb_descriptor(const Img& blurred, const KP& kpt, float layer_scale, uint8_t* desc) {
    float scale = 1.f / layer_scale;
    float angle = kpt.angle;
    angle *= (float)(M_PI / 180.f);
    float a = (float)std::cos((double)angle), b = (float)std::sin((double)angle);
    const int step = blurred.w;
    const uint8_t* center = &blurred.px[(size_t)cv_round(kpt.y * scale) * step + cv_round(kpt.x * scale)];
    auto get = [&](int idx) {
        int px = kPattern[(idx >> 1) * 4 + (idx & 1) * 2], py = kPattern[(idx >> 1) * 4 + (idx & 1) * 2 + 1];
        float x = px * a - py * b;
        float y = px * b + py * a;
        int ix = cv_round(x), iy = cv_round(y);
        return (int)center[iy * step + ix];
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            int idx = i * 16 + bit * 2;
            int t0 = get(idx), t1 = get(idx + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

struct Pyramid {
    std::vector<Img> lv;
    std::vector<float> scale;
};

Pyramid build_pyramid(const uint8_t* img, int w, int h, int stride, int nlevels, int semantics) {
    Pyramid P;
    P.lv.resize(nlevels);
    P.scale.resize(nlevels);
    for (int l = 0; l < nlevels; ++l) {
        float s = get_scale(l);
        P.scale[l] = s;
        float inv = 1.0f / s;
        int lw = cv_round(w * inv), lh = cv_round(h * inv);
        if (l == 0) {
            P.lv[0].w = w;
            P.lv[0].h = h;
            P.lv[0].px.resize((size_t)w * h);
            for (int y = 0; y < h; ++y) std::memcpy(&P.lv[0].px[(size_t)y * w], img + (size_t)y * stride, w);
        } else {
            if (semantics == kOcv32)
                resize_linear_32(P.lv[l - 1], P.lv[l], lw, lh);
            else
                resize_linear_exact(P.lv[l - 1], P.lv[l], lw, lh);
        }
    }
    return P;
}

std::vector<int> features_per_level(int nfeatures, int nlevels) {
    std::vector<int> n(nlevels);
    float factor = (float)(1.0 / kScaleFactor);
    float ndesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        n[l] = cv_round(ndesired);
        sum += n[l];
        ndesired *= factor;
    }
    n[nlevels - 1] = std::max(nfeatures - sum, 0);
    return n;
}

// orb.cpp computeKeyPoints + detectAndCompute (no mask, useProvidedKeypoints=false)
int detect_and_compute(const uint8_t* img, int w, int h, int stride, int nfeatures, std::vector<KP>& out,
                       std::vector<uint8_t>& desc, int semantics) {
    const int nlevels = 8;
    Pyramid P = build_pyramid(img, w, h, stride, nlevels, semantics);
    std::vector<int> nper = features_per_level(nfeatures, nlevels);
    const int half = kPatchSize / 2;
    std::vector<int> umax = make_umax(half);
    std::vector<KP> all;
    std::vector<int> counters(nlevels);
    for (int l = 0; l < nlevels; ++l) {
        std::vector<KP> kps;
        fast16(P.lv[l].px.data(), P.lv[l].w, P.lv[l].h, P.lv[l].w, kFastThreshold, kps);
        run_by_image_border(kps, P.lv[l].w, P.lv[l].h, kEdgeThreshold);
        retain_best(kps, 2 * nper[l], [](const KP& k) { return k.response; }, semantics);
        counters[l] = (int)kps.size();
        float sf = P.scale[l];
        for (auto& k : kps) {
            k.octave = l;
            k.size = kPatchSize * sf;
        }
        all.insert(all.end(), kps.begin(), kps.end());
    }
    out.clear();
    if (all.empty()) {
        desc.clear();
        return 0;
    }
    {
        int off = 0;
        for (int l = 0; l < nlevels; ++l) {
            harris_responses(P.lv[l], all, off, off + counters[l]);
            off += counters[l];
        }
    }
    std::vector<KP> newall;
    int off = 0;
    for (int l = 0; l < nlevels; ++l) {
        std::vector<KP> kps(all.begin() + off, all.begin() + off + counters[l]);
        off += counters[l];
        retain_best(kps, nper[l], [](const KP& k) { return k.response; }, semantics);
        newall.insert(newall.end(), kps.begin(), kps.end());
    }
    all.swap(newall);
    // ICAngles per level (pts still in level coordinates)
    for (size_t i = 0; i < all.size(); ++i) ic_angles(P.lv[all[i].octave], all, (int)i, (int)i + 1, umax, half);
    for (auto& k : all) {
        float s = P.scale[k.octave];
        k.x *= s;
        k.y *= s;
    }
    // descriptors on the blurred pyramid
    std::vector<Img> blurred(nlevels);
    for (int l = 0; l < nlevels; ++l) gaussian_blur7(P.lv[l], blurred[l]);
    desc.assign(all.size() * 32, 0);
    for (size_t i = 0; i < all.size(); ++i)
        orb_descriptor(blurred[all[i].octave], all[i], P.scale[all[i].octave], &desc[i * 32]);
    out = all;
    return 0;
}

// ---- restated libstdc++ introselect (for pinning the GPU emulation) --------
struct Sel {
    std::vector<float>* v;
    std::vector<int32_t>* perm;
    bool comp(int i, int j) const { return (*v)[i] > (*v)[j]; }
    void swap(int i, int j) const {
        std::swap((*v)[i], (*v)[j]);
        std::swap((*perm)[i], (*perm)[j]);
    }
    void move_median_to_first(int result, int a, int b, int c) const {
        if (comp(a, b)) {
            if (comp(b, c)) swap(result, b);
            else if (comp(a, c)) swap(result, c);
            else swap(result, a);
        } else if (comp(a, c)) swap(result, a);
        else if (comp(b, c)) swap(result, c);
        else swap(result, b);
    }
    int unguarded_partition(int first, int last, int pivot) const {
        while (true) {
            while (comp(first, pivot)) ++first;
            --last;
            while (comp(pivot, last)) --last;
            if (!(first < last)) return first;
            swap(first, last);
            ++first;
        }
    }
    void adjust_heap(int first, int hole, int len, float val, int32_t pv) const {
        std::vector<float>& a = *v;
        std::vector<int32_t>& p = *perm;
        const int top = hole;
        int second = hole;
        while (second < (len - 1) / 2) {
            second = 2 * (second + 1);
            if (a[first + second] > a[first + second - 1]) second--;
            a[first + hole] = a[first + second];
            p[first + hole] = p[first + second];
            hole = second;
        }
        if ((len & 1) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            a[first + hole] = a[first + second - 1];
            p[first + hole] = p[first + second - 1];
            hole = second - 1;
        }
        int parent = (hole - 1) / 2;
        while (hole > top && a[first + parent] > val) {
            a[first + hole] = a[first + parent];
            p[first + hole] = p[first + parent];
            hole = parent;
            parent = (hole - 1) / 2;
        }
        a[first + hole] = val;
        p[first + hole] = pv;
    }
    void heap_select(int first, int middle, int last) const {
        int len = middle - first;
        if (len >= 2) {
            int parent = (len - 2) / 2;
            while (true) {
                adjust_heap(first, parent, len, (*v)[first + parent], (*perm)[first + parent]);
                if (parent == 0) break;
                parent--;
            }
        }
        for (int i = middle; i < last; ++i)
            if (comp(i, first)) {
                float val = (*v)[i];
                int32_t pv = (*perm)[i];
                (*v)[i] = (*v)[first];
                (*perm)[i] = (*perm)[first];
                adjust_heap(first, 0, len, val, pv);
            }
    }
    void insertion_sort(int first, int last) const {
        if (first == last) return;
        for (int i = first + 1; i != last; ++i) {
            float val = (*v)[i];
            int32_t pv = (*perm)[i];
            if (val > (*v)[first]) {
                for (int k = i; k > first; --k) {
                    (*v)[k] = (*v)[k - 1];
                    (*perm)[k] = (*perm)[k - 1];
                }
                (*v)[first] = val;
                (*perm)[first] = pv;
            } else {
                int k = i;
                while (val > (*v)[k - 1]) {
                    (*v)[k] = (*v)[k - 1];
                    (*perm)[k] = (*perm)[k - 1];
                    --k;
                }
                (*v)[k] = val;
                (*perm)[k] = pv;
            }
        }
    }
    void introselect(int first, int nth, int last, int depth) const {
        while (last - first > 3) {
            if (depth == 0) {
                heap_select(first, nth + 1, last);
                swap(first, nth);
                return;
            }
            --depth;
            int mid = first + (last - first) / 2;
            move_median_to_first(first, first + 1, mid, last - 1);
            int cut = unguarded_partition(first + 1, last, first);
            if (cut <= nth) first = cut;
            else last = cut;
        }
        insertion_sort(first, last);
    }
};

}  // namespace

extern "C" {

int ora_orb_level_sizes(int w, int h, int nlevels, int* sizes) {
    for (int l = 0; l < nlevels; ++l) {
        float inv = 1.0f / get_scale(l);
        sizes[2 * l] = l == 0 ? w : cv_round(w * inv);
        sizes[2 * l + 1] = l == 0 ? h : cv_round(h * inv);
    }
    return 0;
}

// getScale of levels 0..nlevels-1: the factor the oracle multiplies a level's
// keypoint coordinates and sizes by (orb.cpp computeKeyPoints / KeyPoint scaling).
int ora_orb_level_scales(int nlevels, float* out) {
    for (int l = 0; l < nlevels; ++l) out[l] = get_scale(l);
    return 0;
}

int ora_orb_features_per_level(int nfeatures, int nlevels, int* out) {
    std::vector<int> n = features_per_level(nfeatures, nlevels);
    for (int l = 0; l < nlevels; ++l) out[l] = n[l];
    return 0;
}

int ora_orb_pyramid(const uint8_t* img, int w, int h, int stride, int nlevels, int blurred, uint8_t* out) {
    return ora_orb_pyramid_v(img, w, h, stride, nlevels, blurred, kOcv4, out);
}

int ora_orb_pyramid_v(const uint8_t* img, int w, int h, int stride, int nlevels, int blurred, int semantics,
                      uint8_t* out) {
    Pyramid P = build_pyramid(img, w, h, stride, nlevels, semantics);
    size_t off = 0;
    for (int l = 0; l < nlevels; ++l) {
        Img b;
        const Img* src = &P.lv[l];
        if (blurred) {
            gaussian_blur7(P.lv[l], b);
            src = &b;
        }
        std::memcpy(out + off, src->px.data(), src->px.size());
        off += src->px.size();
    }
    return 0;
}

int ora_fast(const uint8_t* img, int w, int h, int stride, int threshold, int32_t* xys, int cap, int* n) {
    std::vector<KP> kps;
    fast16(img, w, h, stride, threshold, kps);
    *n = (int)kps.size();
    if ((int)kps.size() > cap) return -1;
    for (size_t i = 0; i < kps.size(); ++i) {
        xys[3 * i] = (int)kps[i].x;
        xys[3 * i + 1] = (int)kps[i].y;
        xys[3 * i + 2] = (int)kps[i].response;
    }
    return 0;
}

int ora_retain_best(const float* resp, int n, int n_points, int32_t* perm) {
    return ora_retain_best_v(resp, n, n_points, kOcv4, perm);
}

int ora_retain_best_v(const float* resp, int n, int n_points, int semantics, int32_t* perm) {
    struct E { float r; int32_t i; };
    std::vector<E> v(n);
    for (int i = 0; i < n; ++i) v[i] = E{resp[i], i};
    retain_best(v, n_points, [](const E& e) { return e.r; }, semantics);
    for (size_t i = 0; i < v.size(); ++i) perm[i] = v[i].i;
    return (int)v.size();
}

int ora_retain_best_depth(const float* resp, int n, int n_points, int depth, int32_t* perm) {
    return ora_retain_best_depth_v(resp, n, n_points, depth, kOcv4, perm);
}

int ora_retain_best_depth_v(const float* resp, int n, int n_points, int depth, int semantics, int32_t* perm) {
    std::vector<float> v(resp, resp + n);
    std::vector<int32_t> p(n);
    for (int i = 0; i < n; ++i) p[i] = i;
    if (!(n_points >= 0 && n > n_points)) {
        for (int i = 0; i < n; ++i) perm[i] = i;
        return n;
    }
    if (n_points == 0) return 0;
    Sel s{&v, &p};
    if (depth < 0) {
        int lg = 0;
        while ((2 << lg) <= n) ++lg;  // std::__lg(n)
        depth = 2 * lg;
    }
    s.introselect(0, n_points - (semantics == kOcv32 ? 0 : 1), n, depth);
    float amb = v[n_points - 1];
    // std::partition (bidirectional) on [n_points, n) with pred resp >= amb
    int first = n_points, last = n;
    while (true) {
        while (true) {
            if (first == last) goto done;
            if (v[first] >= amb) ++first;
            else break;
        }
        --last;
        while (true) {
            if (first == last) goto done;
            if (!(v[last] >= amb)) --last;
            else break;
        }
        s.swap(first, last);
        ++first;
    }
done:
    for (int i = 0; i < first; ++i) perm[i] = p[i];
    return first;
}

int ora_orb_detect_and_compute(const uint8_t* img, int w, int h, int stride, int nfeatures, ora_keypoint* kps,
                               uint8_t* desc, int cap, int* n_out) {
    return ora_orb_detect_and_compute_v(img, w, h, stride, nfeatures, kOcv4, kps, desc, cap, n_out);
}

int ora_orb_detect_and_compute_v(const uint8_t* img, int w, int h, int stride, int nfeatures, int semantics,
                                 ora_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
    if (semantics != kOcv4 && semantics != kOcv32) return -2;
    std::vector<KP> out;
    std::vector<uint8_t> d;
    detect_and_compute(img, w, h, stride, nfeatures, out, d, semantics);
    *n_out = (int)out.size();
    if ((int)out.size() > cap) return -1;
    for (size_t i = 0; i < out.size(); ++i) {
        kps[i].x = out[i].x;
        kps[i].y = out[i].y;
        kps[i].size = out[i].size;
        kps[i].angle = out[i].angle;
        kps[i].response = out[i].response;
        kps[i].octave = out[i].octave;
        kps[i].class_id = -1;
    }
    if (!d.empty()) std::memcpy(desc, d.data(), d.size());
    return 0;
}

}  // extern "C"
