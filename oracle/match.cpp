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

#include <climits>
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
