// TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of
// cv::BFMatcher(NORM_HAMMING, crossCheck=True).match(query, train) as built at
// scripts/visual_odometry_v3.py:75 and called at :219 (query = previous frame,
// train = current frame).  Follows OpenCV 4.x matchers.cpp
// BFMatcher::knnMatchImpl(k=1) + core batchDistance(crosscheck):
//   forward  NN: for each query the first train index reaching the min distance
//   backward NN: for each train the first query index reaching the min distance
//   4.x keeps (q, t=fwd[q]) iff bwd[t] == q; 3.x (mode 2) keeps for every query
//   the first train t with bwd[t] == q at the smallest distance.
// Output order is queryIdx ascending (DescriptorMatcher::convertMatches).
#include "oracle.h"

#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

namespace {
inline int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}
}  // namespace

extern "C" int ora_bf_match_hamming(const uint8_t* dq, int nq, const uint8_t* dt, int nt, int mode,
                                    int32_t* qidx, int32_t* tidx, float* dist, int* m_out) {
    *m_out = 0;
    if (nq <= 0 || nt <= 0) return 0;
    std::vector<int> fwd(nq, -1), fwd_d(nq, INT_MAX), bwd(nt, -1), bwd_d(nt, INT_MAX);
    for (int q = 0; q < nq; ++q)
        for (int t = 0; t < nt; ++t) {
            int d = hamming32(dq + 32 * q, dt + 32 * t);
            if (d < fwd_d[q]) { fwd_d[q] = d; fwd[q] = t; }
            if (d < bwd_d[t]) { bwd_d[t] = d; bwd[t] = q; }
        }
    int m = 0;
    if (mode == 0) {
        for (int q = 0; q < nq; ++q) { qidx[m] = q; tidx[m] = fwd[q]; dist[m] = (float)fwd_d[q]; ++m; }
    } else if (mode == 1) {
        for (int q = 0; q < nq; ++q) {
            int t = fwd[q];
            if (t >= 0 && bwd[t] == q) { qidx[m] = q; tidx[m] = t; dist[m] = (float)fwd_d[q]; ++m; }
        }
    } else {
        // OpenCV 3.x: nidx[q] = argmin_{t: bwd[t]==q} d (first t on ties), dist = that d.
        std::vector<int> best(nq, -1), bestd(nq, INT_MAX);
        for (int t = 0; t < nt; ++t) {
            int q = bwd[t], d = bwd_d[t];
            if (d < bestd[q]) { bestd[q] = d; best[q] = t; }
        }
        for (int q = 0; q < nq; ++q)
            if (best[q] >= 0) { qidx[m] = q; tidx[m] = best[q]; dist[m] = (float)bestd[q]; ++m; }
    }
    *m_out = m;
    return 0;
}

// ---- BFMatcher(NORM_L1).knnMatch / FlannBasedMatcher stand-in (float) -------
// The SIFT/SURF branches of the reference (visual_odometry_v3.py:99-106 build
// BFMatcher(NORM_L1); :200-215 call .match / .knnMatch(k=2) / FLANN knnMatch,
// :223-228 apply the 0.75 ratio test).  Follows OpenCV 4.x
// BFMatcher::knnMatchImpl -> batchDistance(K=k): each query keeps its k
// smallest distances, a train j entering iff d < dist[k-1] and landing after
// every kept entry with dist <= d (so ties keep the lower train index first);
// dist starts at FLT_MAX, idx at -1.
//   norm 0 (L1): cv::normL1<float,float> (core/base.hpp), 4-way unrolled
//       s += |v0| + |v1| + |v2| + |v3|, then a scalar tail.
//   norm 1 (L2SQR): flann::L2<float> (the distance FlannBasedMatcher reports,
//       squared, 4-way unrolled result += d0*d0 + d1*d1 + d2*d2 + d3*d3).
// OpenCV's SIMD kernels sum in another order; for SIFT descriptors (integer
// values 0..255 stored as float) every partial sum is an integer below 2^24,
// so all orders give the same float and parity is order-independent there.
namespace {
inline float dist_l1(const float* a, const float* b, int n) {
    float s = 0.f;
    int i = 0;
    for (; i <= n - 4; i += 4) {
        float v0 = a[i] - b[i], v1 = a[i + 1] - b[i + 1], v2 = a[i + 2] - b[i + 2], v3 = a[i + 3] - b[i + 3];
        s += std::fabs(v0) + std::fabs(v1) + std::fabs(v2) + std::fabs(v3);
    }
    for (; i < n; ++i) s += std::fabs(a[i] - b[i]);
    return s;
}
inline float dist_l2sqr(const float* a, const float* b, int n) {
    float s = 0.f;
    int i = 0;
    for (; i <= n - 4; i += 4) {
        float d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1], d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        float p0 = d0 * d0, p1 = d1 * d1, p2 = d2 * d2, p3 = d3 * d3;
        s += ((p0 + p1) + p2) + p3;
    }
    for (; i < n; ++i) { float d = a[i] - b[i]; float p = d * d; s += p; }
    return s;
}
}  // namespace

extern "C" int ora_bf_knn_float(const float* dq, int nq, const float* dt, int nt, int dim, int k, int norm,
                                int32_t* tidx, float* dist) {
    if (nq < 0 || nt < 0 || dim <= 0 || k <= 0 || norm < 0 || norm > 1) return -1;
    for (int q = 0; q < nq; ++q) {
        float* bd = dist + (size_t)q * k;
        int32_t* bi = tidx + (size_t)q * k;
        for (int s = 0; s < k; ++s) { bd[s] = FLT_MAX; bi[s] = -1; }
        for (int t = 0; t < nt; ++t) {
            const float d = norm == 0 ? dist_l1(dq + (size_t)q * dim, dt + (size_t)t * dim, dim)
                                      : dist_l2sqr(dq + (size_t)q * dim, dt + (size_t)t * dim, dim);
            if (d < bd[k - 1]) {
                int s = k - 2;
                for (; s >= 0 && bd[s] > d; --s) { bd[s + 1] = bd[s]; bi[s + 1] = bi[s]; }
                bd[s + 1] = d;
                bi[s + 1] = t;
            }
        }
    }
    return 0;
}
