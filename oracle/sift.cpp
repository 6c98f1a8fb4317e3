// TEST INFRASTRUCTURE ONLY — CPU restatement of OpenCV 4.x
// cv::SIFT::detectAndCompute(img, None) with SIFT_create()'s defaults, the
// detector of the reference's 'sift' / 'knn_sift' / 'flann' modes
// (scripts/visual_odometry_v3.py:99-103 SIFT_create(), :373 detectAndCompute).
// Follows sift.dispatch.cpp / sift.simd.hpp (createInitialImage,
// buildGaussianPyramid, buildDoGPyramid, findScaleSpaceExtrema,
// adjustLocalExtrema, calcOrientationHist, removeDuplicatedSorted,
// calcSIFTDescriptor) with their scalar formulas.  Where OpenCV's result
// depends on the build (SIMD/FMA paths of sepFilter2D, exp32f, magnitude,
// fastAtan2; libm sinf/cosf/powf), this restatement fixes one definition,
// which the GPU kernels (csrc/sift.hip) follow operation for operation:
//   - float expressions evaluated unfused, left to right;
//   - GaussianBlur = row pass sum_k kx[k] S[x-r+k] (k ascending) then the
//     symmetric column pass ky[r] C + sum_k ky[r+k] (U_k + D_k), REFLECT_101;
//   - exp32f = its scalar table path (data/sift_exp_tab.inc);
//   - cos/sin/pow of a float argument = double libm result rounded to float.
// Parity against OpenCV itself is unpinned (OpenCV is absent).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

constexpr int kLayers = 3;                // nOctaveLayers
constexpr float kContrast = 0.04f;        // contrastThreshold
constexpr float kEdge = 10.f;             // edgeThreshold
constexpr float kSigma = 1.6f;            // sigma as createInitialImage / adjustLocalExtrema see it (float)
constexpr double kSigmaD = 1.6;           // SIFT_Impl::sigma (double member), used by buildGaussianPyramid
constexpr int kFirstOctave = -1;          // the input is upscaled 2x
constexpr int kBorder = 5;                // SIFT_IMG_BORDER
constexpr int kMaxInterp = 5;             // SIFT_MAX_INTERP_STEPS
constexpr int kOriBins = 36;              // SIFT_ORI_HIST_BINS
constexpr float kOriSigFctr = 1.5f;       // SIFT_ORI_SIG_FCTR
constexpr float kOriRadius = 3 * kOriSigFctr;
constexpr float kOriPeak = 0.8f;          // SIFT_ORI_PEAK_RATIO
constexpr int kDescW = 4, kDescBins = 8;  // SIFT_DESCR_WIDTH, SIFT_DESCR_HIST_BINS
constexpr float kInitSigma = 0.5f;        // SIFT_INIT_SIGMA
constexpr float kDescSclFctr = 3.f;       // SIFT_DESCR_SCL_FCTR
constexpr float kDescMagThr = 0.2f;       // SIFT_DESCR_MAG_THR
constexpr float kIntDescFctr = 512.f;     // SIFT_INT_DESCR_FCTR

struct FImg {
    int w = 0, h = 0;
    std::vector<float> d;
    FImg() = default;
    FImg(int w_, int h_) : w(w_), h(h_), d((size_t)w_ * h_) {}
    float at(int y, int x) const { return d[(size_t)y * w + x]; }
};

int cv_round(float v) { return (int)std::nearbyint(v); }
int cv_round_d(double v) { return (int)std::nearbyint(v); }
int cv_floor(float v) { return (int)std::floor(v); }

int refl101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

// getGaussianKernel(n, sigma, CV_32F): double exp, float taps, renormalised
std::vector<float> gauss_kernel(double sigma) {
    const int n = cv_round_d(sigma * 4 * 2 + 1) | 1;  // GaussianBlur ksize for float images
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

FImg gauss_blur(const FImg& s, double sigma) {
    const std::vector<float> k = gauss_kernel(sigma);
    const int n = (int)k.size(), r = n / 2;
    FImg t(s.w, s.h), o(s.w, s.h);
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            float acc = k[0] * s.at(y, refl101(x - r, s.w));
            for (int i = 1; i < n; ++i) acc += k[i] * s.at(y, refl101(x - r + i, s.w));
            t.d[(size_t)y * s.w + x] = acc;
        }
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            float acc = k[r] * t.at(y, x) + 0.f;
            for (int i = 1; i <= r; ++i) acc += k[r + i] * (t.at(refl101(y + i, s.h), x) + t.at(refl101(y - i, s.h), x));
            o.d[(size_t)y * s.w + x] = acc;
        }
    return o;
}

// cv::hal::exp32f, scalar path
const double kExpTab[64] = {
#include "../data/sift_exp_tab.inc"
};
float sift_exp(float x) {
    const double prescale = 1.4426950408889634073599246810019 * 64, postscale = 1. / 64, maxv = 3000. * 64;
    const float A0 = .9670371139572337719125840413672004409288e-2;
    const float A4 = (float)(1.000000000000002438532970795181890933776 / A0);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / A0);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / A0);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / A0);
    const float minval = (float)(-maxv / prescale), maxval = (float)(maxv / prescale);
    float x0 = std::min(std::max(x, minval), maxval);
    x0 *= (float)prescale;
    const int xi = cv_round(x0);
    x0 = (x0 - (float)xi) * (float)postscale;
    int t = (xi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    uint32_t bits = (uint32_t)t << 23;
    float b;
    std::memcpy(&b, &bits, 4);
    const float poly = (((x0 + A1) * x0 + A2) * x0 + A3) * x0 + A4;
    return b * (float)kExpTab[xi & 63] * poly;
}

float fast_atan2_deg(float y, float x) {  // cv::fastAtan2 / hal::fastAtan32f
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

struct Kp {
    float x, y, size, angle, response;
    int octave;
};

// adjustLocalExtrema (sift.simd.hpp); false rejects the candidate
bool adjust(const std::vector<FImg>& dog, Kp& kpt, int octv, int& layer, int& r, int& c) {
    const float img_scale = 1.f / 255;
    const float deriv_scale = img_scale * 0.5f, second = img_scale, cross = img_scale * 0.25f;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < kMaxInterp; i++) {
        const int idx = octv * (kLayers + 2) + layer;
        const FImg &img = dog[idx], &prev = dog[idx - 1], &next = dog[idx + 1];
        const float dD0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
        const float dD1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
        const float dD2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
        const float v2 = img.at(r, c) * 2;
        const float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second;
        const float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second;
        const float dss = (next.at(r, c) + prev.at(r, c) - v2) * second;
        const float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) * cross;
        const float dxs = (next.at(r, c + 1) - next.at(r, c - 1) - prev.at(r, c + 1) + prev.at(r, c - 1)) * cross;
        const float dys = (next.at(r + 1, c) - next.at(r - 1, c) - prev.at(r + 1, c) + prev.at(r - 1, c)) * cross;
        // Matx33f(dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss).solve(dD, DECOMP_LU): Matx_FastSolveOp<3, 1>
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys, a22 = dss;
        float X0 = 0, X1 = 0, X2 = 0;
        float d = (float)(double)(a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11));
        if (d != 0) {
            d = 1 / d;
            X0 = d * (dD0 * (a11 * a22 - a12 * a21) - a01 * (dD1 * a22 - a12 * dD2) + a02 * (dD1 * a21 - a11 * dD2));
            X1 = d * (a00 * (dD1 * a22 - a12 * dD2) - dD0 * (a10 * a22 - a12 * a20) + a02 * (a10 * dD2 - dD1 * a20));
            X2 = d * (a00 * (a11 * dD2 - dD1 * a21) - a01 * (a10 * dD2 - dD1 * a20) + dD0 * (a10 * a21 - a11 * a20));
        }
        xi = -X2;
        xr = -X1;
        xc = -X0;
        if (std::abs(xi) < 0.5f && std::abs(xr) < 0.5f && std::abs(xc) < 0.5f) break;
        if (std::abs(xi) > (float)(INT_MAX / 3) || std::abs(xr) > (float)(INT_MAX / 3) || std::abs(xc) > (float)(INT_MAX / 3))
            return false;
        c += cv_round(xc);
        r += cv_round(xr);
        layer += cv_round(xi);
        if (layer < 1 || layer > kLayers || c < kBorder || c >= img.w - kBorder || r < kBorder || r >= img.h - kBorder)
            return false;
    }
    if (i >= kMaxInterp) return false;
    {
        const int idx = octv * (kLayers + 2) + layer;
        const FImg &img = dog[idx], &prev = dog[idx - 1], &next = dog[idx + 1];
        const float dD0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
        const float dD1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
        const float dD2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
        const float t = dD0 * xc + dD1 * xr + dD2 * xi;
        contr = img.at(r, c) * img_scale + t * 0.5f;
        if (std::abs(contr) * kLayers < kContrast) return false;
        const float v2 = img.at(r, c) * 2.f;
        const float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second;
        const float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second;
        const float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) * cross;
        const float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * kEdge >= (kEdge + 1) * (kEdge + 1) * det) return false;
    }
    kpt.x = (c + xc) * (float)(1 << octv);
    kpt.y = (r + xr) * (float)(1 << octv);
    kpt.octave = octv + (layer << 8) + (cv_round_d((xi + 0.5) * 255) << 16);
    kpt.size = kSigma * (float)std::exp2((double)((layer + xi) / kLayers)) * (float)(1 << octv) * 2;
    kpt.response = std::abs(contr);
    return true;
}

// calcOrientationHist: 36-bin smoothed gradient histogram, returns its maximum
float orientation_hist(const FImg& img, int px, int py, int radius, float sigma, float* hist) {
    const int n = kOriBins;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    float temp[kOriBins + 4] = {0};
    float* th = temp + 2;
    for (int i = -radius; i <= radius; i++) {
        const int y = py + i;
        if (y <= 0 || y >= img.h - 1) continue;
        for (int j = -radius; j <= radius; j++) {
            const int x = px + j;
            if (x <= 0 || x >= img.w - 1) continue;
            const float dx = img.at(y, x + 1) - img.at(y, x - 1);
            const float dy = img.at(y - 1, x) - img.at(y + 1, x);
            const float w = sift_exp((float)(i * i + j * j) * expf_scale);
            const float ori = fast_atan2_deg(dy, dx);
            const float mag = std::sqrt(dx * dx + dy * dy);
            int bin = cv_round((n / 360.f) * ori);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
            th[bin] += w * mag;
        }
    }
    th[-1] = th[n - 1];
    th[-2] = th[n - 2];
    th[n] = th[0];
    th[n + 1] = th[1];
    for (int i = 0; i < n; i++)
        hist[i] = (th[i - 2] + th[i + 2]) * (1.f / 16.f) + (th[i - 1] + th[i + 1]) * (4.f / 16.f) + th[i] * (6.f / 16.f);
    float maxval = hist[0];
    for (int i = 1; i < n; i++) maxval = std::max(maxval, hist[i]);
    return maxval;
}

// calcSIFTDescriptor (d = 4, n = 8) into 128 floats holding saturate_cast<uchar> values
void descriptor(const FImg& img, float ptx, float pty, float ori, float scl, float* dst) {
    const int d = kDescW, n = kDescBins;
    const int px = cv_round(ptx), py = cv_round(pty);
    const float a = ori * (float)(M_PI / 180);
    float cos_t = (float)std::cos((double)a), sin_t = (float)std::sin((double)a);
    const float bins_per_rad = n / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = kDescSclFctr * scl;
    int radius = cv_round(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    radius = std::min(radius, (int)std::sqrt(((double)img.w) * img.w + ((double)img.h) * img.h));
    cos_t /= hist_width;
    sin_t /= hist_width;
    float hist[(kDescW + 2) * (kDescW + 2) * (kDescBins + 2)] = {0};
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            float rbin = r_rot + d / 2 - 0.5f;
            float cbin = c_rot + d / 2 - 0.5f;
            const int r = py + i, c = px + j;
            if (!(rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < img.h - 1 && c > 0 && c < img.w - 1))
                continue;
            const float dx = img.at(r, c + 1) - img.at(r, c - 1);
            const float dy = img.at(r - 1, c) - img.at(r + 1, c);
            const float w = sift_exp((c_rot * c_rot + r_rot * r_rot) * exp_scale);
            const float o = fast_atan2_deg(dy, dx);
            const float m = std::sqrt(dx * dx + dy * dy);
            float obin = (o - ori) * bins_per_rad;
            const float mag = m * w;
            int r0 = cv_floor(rbin), c0 = cv_floor(cbin), o0 = cv_floor(obin);
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
            const int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
            hist[idx] += v_rco000;
            hist[idx + 1] += v_rco001;
            hist[idx + (n + 2)] += v_rco010;
            hist[idx + (n + 3)] += v_rco011;
            hist[idx + (d + 2) * (n + 2)] += v_rco100;
            hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
            hist[idx + (d + 3) * (n + 2)] += v_rco110;
            hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
        }
    float raw[kDescW * kDescW * kDescBins];
    for (int i = 0; i < d; i++)
        for (int j = 0; j < d; j++) {
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            hist[idx] += hist[idx + n];
            hist[idx + 1] += hist[idx + n + 1];
            for (int k = 0; k < n; k++) raw[(i * d + j) * n + k] = hist[idx + k];
        }
    const int len = d * d * n;
    float nrm2 = 0;
    for (int k = 0; k < len; k++) nrm2 += raw[k] * raw[k];
    const float thr = std::sqrt(nrm2) * kDescMagThr;
    nrm2 = 0;
    for (int k = 0; k < len; k++) {
        const float v = std::min(raw[k], thr);
        raw[k] = v;
        nrm2 += v * v;
    }
    nrm2 = kIntDescFctr / std::max(std::sqrt(nrm2), FLT_EPSILON);
    for (int k = 0; k < len; k++) {
        const int v = cv_round(raw[k] * nrm2);
        dst[k] = (float)std::min(std::max(v, 0), 255);
    }
}

bool kp_less(const Kp& a, const Kp& b) {  // KeyPoint12_LessThan (class_id is -1 for all)
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    return a.octave > b.octave;
}

}  // namespace

int ora_sift_detect_and_compute(const uint8_t* img, int w, int h, int stride, ora_keypoint* kps, float* desc, int cap,
                                int* n_out) {
    *n_out = 0;
    if (w < 1 || h < 1) return -1;
    // createInitialImage: float, resize 2x INTER_LINEAR (weights 0 / 0.25 / 0.75: exact), GaussianBlur
    FImg up(2 * w, 2 * h);
    {
        std::vector<float> hrow((size_t)2 * w * h);
        for (int y = 0; y < h; ++y)
            for (int dx = 0; dx < 2 * w; ++dx) {
                float fx = (float)((dx + 0.5) * 0.5 - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) fx = 0, sx = 0;
                const float* s = nullptr;
                (void)s;
                const float a = (float)img[(size_t)y * stride + sx];
                if (sx >= w - 1) {
                    hrow[(size_t)y * 2 * w + dx] = (float)img[(size_t)y * stride + (w - 1)];
                } else {
                    hrow[(size_t)y * 2 * w + dx] = a * (1.f - fx) + (float)img[(size_t)y * stride + sx + 1] * fx;
                }
            }
        for (int dy = 0; dy < 2 * h; ++dy) {
            float fy = (float)((dy + 0.5) * 0.5 - 0.5);
            int sy = (int)std::floor(fy);
            fy -= sy;
            if (sy < 0) fy = 0, sy = 0;
            if (sy >= h - 1) fy = 0, sy = h - 1;
            const int sy1 = std::min(sy + 1, h - 1);
            for (int dx = 0; dx < 2 * w; ++dx)
                up.d[(size_t)dy * 2 * w + dx] =
                    hrow[(size_t)sy * 2 * w + dx] * (1.f - fy) + hrow[(size_t)sy1 * 2 * w + dx] * fy;
        }
    }
    const float sig_diff = std::sqrt(std::max(kSigma * kSigma - kInitSigma * kInitSigma * 4, 0.01f));
    FImg base = gauss_blur(up, sig_diff);
    const int nOct = cv_round_d(std::log((double)std::min(base.w, base.h)) / std::log(2.) - 2) - kFirstOctave;
    // buildGaussianPyramid
    std::vector<double> sig(kLayers + 3);
    sig[0] = kSigmaD;
    const double k = std::pow(2., 1. / kLayers);
    for (int i = 1; i < kLayers + 3; i++) {
        // SIFT_Impl::buildGaussianPyramid: the double member sigma = 1.6 (createInitialImage and
        // adjustLocalExtrema take it as float, hence kSigma elsewhere)
        const double sig_prev = std::pow(k, (double)(i - 1)) * kSigmaD, sig_total = sig_prev * k;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    std::vector<FImg> gp((size_t)nOct * (kLayers + 3));
    for (int o = 0; o < nOct; o++)
        for (int i = 0; i < kLayers + 3; i++) {
            FImg& dst = gp[(size_t)o * (kLayers + 3) + i];
            if (o == 0 && i == 0) {
                dst = base;
            } else if (i == 0) {  // INTER_NEAREST half of layer nOctaveLayers of the octave below
                const FImg& src = gp[(size_t)(o - 1) * (kLayers + 3) + kLayers];
                dst = FImg(src.w / 2, src.h / 2);
                for (int y = 0; y < dst.h; ++y)
                    for (int x = 0; x < dst.w; ++x) dst.d[(size_t)y * dst.w + x] = src.at(2 * y, 2 * x);
            } else {
                dst = gauss_blur(gp[(size_t)o * (kLayers + 3) + i - 1], sig[i]);
            }
        }
    // buildDoGPyramid
    std::vector<FImg> dog((size_t)nOct * (kLayers + 2));
    for (int o = 0; o < nOct; o++)
        for (int i = 0; i < kLayers + 2; i++) {
            const FImg &a = gp[(size_t)o * (kLayers + 3) + i], &b = gp[(size_t)o * (kLayers + 3) + i + 1];
            FImg& dd = dog[(size_t)o * (kLayers + 2) + i];
            dd = FImg(a.w, a.h);
            for (size_t q = 0; q < dd.d.size(); ++q) dd.d[q] = b.d[q] - a.d[q];
        }
    // findScaleSpaceExtrema
    const int threshold = (int)std::floor(0.5 * kContrast / kLayers * 255);
    std::vector<Kp> found;
    float hist[kOriBins];
    for (int o = 0; o < nOct; o++)
        for (int i = 1; i <= kLayers; i++) {
            const int idx = o * (kLayers + 2) + i;
            const FImg &img = dog[idx], &prev = dog[idx - 1], &next = dog[idx + 1];
            for (int r = kBorder; r < img.h - kBorder; r++)
                for (int c = kBorder; c < img.w - kBorder; c++) {
                    const float val = img.at(r, c);
                    if (!(std::abs(val) > threshold)) continue;
                    bool ext = true;
                    if (val > 0) {
                        for (int dy = -1; dy <= 1 && ext; ++dy)
                            for (int dx = -1; dx <= 1; ++dx)
                                if (!(val >= img.at(r + dy, c + dx) && val >= prev.at(r + dy, c + dx) &&
                                      val >= next.at(r + dy, c + dx))) {
                                    ext = false;
                                    break;
                                }
                    } else if (val < 0) {
                        for (int dy = -1; dy <= 1 && ext; ++dy)
                            for (int dx = -1; dx <= 1; ++dx)
                                if (!(val <= img.at(r + dy, c + dx) && val <= prev.at(r + dy, c + dx) &&
                                      val <= next.at(r + dy, c + dx))) {
                                    ext = false;
                                    break;
                                }
                    } else {
                        ext = false;
                    }
                    if (!ext) continue;
                    int r1 = r, c1 = c, layer = i;
                    Kp kpt{};
                    if (!adjust(dog, kpt, o, layer, r1, c1)) continue;
                    const float scl_octv = kpt.size * 0.5f / (float)(1 << o);
                    const float omax = orientation_hist(gp[(size_t)o * (kLayers + 3) + layer], c1, r1,
                                                        cv_round(kOriRadius * scl_octv), kOriSigFctr * scl_octv, hist);
                    const float mag_thr = omax * kOriPeak;
                    for (int j = 0; j < kOriBins; j++) {
                        const int l = j > 0 ? j - 1 : kOriBins - 1, r2 = j < kOriBins - 1 ? j + 1 : 0;
                        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                            float bin = (float)j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                            bin = bin < 0 ? kOriBins + bin : bin >= kOriBins ? bin - kOriBins : bin;
                            kpt.angle = 360.f - (360.f / kOriBins) * bin;
                            if (std::abs(kpt.angle - 360.f) < FLT_EPSILON) kpt.angle = 0.f;
                            found.push_back(kpt);
                        }
                    }
                }
        }
    // removeDuplicatedSorted
    std::sort(found.begin(), found.end(), kp_less);
    std::vector<Kp> kp;
    for (const Kp& q : found)
        if (kp.empty() || q.x != kp.back().x || q.y != kp.back().y || q.size != kp.back().size || q.angle != kp.back().angle)
            kp.push_back(q);
    const int n = (int)kp.size();
    *n_out = n;
    if (n > cap) return -5;
    for (int i = 0; i < n; ++i) {
        Kp q = kp[i];
        // firstOctave = -1: octave field, pt and size back to input-image units
        const int oct = q.octave & 255, layer = (q.octave >> 8) & 255;
        ora_keypoint& out = kps[i];
        out.x = q.x * 0.5f;
        out.y = q.y * 0.5f;
        out.size = q.size * 0.5f;
        out.angle = q.angle;
        out.response = q.response;
        out.octave = (q.octave & ~255) | ((q.octave + kFirstOctave) & 255);
        out.class_id = -1;
        // calcDescriptors: unpackOctave, image of that octave / layer, angle flipped
        const int octv = (out.octave & 255) < 128 ? (out.octave & 255) : (-128 | (out.octave & 255));
        const float scale = octv >= 0 ? 1.f / (float)(1 << octv) : (float)(1 << -octv);
        const float size = out.size * scale;
        const float ptx = out.x * scale, pty = out.y * scale;
        float angle = 360.f - out.angle;
        if (std::abs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        descriptor(gp[(size_t)(octv - kFirstOctave) * (kLayers + 3) + layer], ptx, pty, angle, size * 0.5f,
                   desc + (size_t)i * 128);
        (void)oct;
    }
    return 0;
}
