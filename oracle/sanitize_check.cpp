// TEST INFRASTRUCTURE ONLY — drives every oracle entry point under
// AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile `sanitize`,
// tests/test_sanitize.py): a textured synthetic frame pair with a known
// camera motion, plus the edge cases the GPU tests cover (tiny and blank
// frames, empty descriptor sets, fewer than 5 correspondences, k > trains).
// Exit 0 = every call returned and no sanitizer report fired.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "oracle.h"

namespace {

std::vector<uint8_t> textured(int w, int h, uint32_t seed, double shift) {
    std::vector<uint8_t> img((size_t)w * h);
    std::mt19937 rng(seed);
    std::vector<double> cx(300), cy(300), r(300), v(300);
    for (int i = 0; i < 300; ++i) {
        cx[i] = rng() % w;
        cy[i] = rng() % h;
        r[i] = 2 + rng() % 9;
        v[i] = 40 + rng() % 180;
    }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s = 20 + 10 * std::sin(0.05 * x) * std::cos(0.07 * y);
            for (int i = 0; i < 300; ++i) {
                const double dx = x - cx[i] - shift, dy = y - cy[i];
                if (dx * dx + dy * dy < r[i] * r[i]) s = v[i];
            }
            img[(size_t)y * w + x] = (uint8_t)std::min(255.0, std::max(0.0, s));
        }
    return img;
}

int fails = 0;
#define EXPECT(c)                                                           \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            ++fails;                                                        \
        }                                                                   \
    } while (0)

}  // namespace

int main() {
    const int W = 320, H = 240, N = 300;
    auto a = textured(W, H, 7, 0.0), b = textured(W, H, 7, 3.0);
    std::vector<ora_keypoint> ka(N + 512), kb(N + 512);
    std::vector<uint8_t> da((N + 512) * 32), db((N + 512) * 32);
    int na = 0, nb = 0;
    EXPECT(ora_orb_detect_and_compute(a.data(), W, H, W, N, ka.data(), da.data(), N + 512, &na) == 0);
    EXPECT(ora_orb_detect_and_compute(b.data(), W, H, W, N, kb.data(), db.data(), N + 512, &nb) == 0);
    EXPECT(na > 50 && nb > 50);

    // pyramid, FAST, retainBest
    int sizes[16];
    ora_orb_level_sizes(W, H, 8, sizes);
    size_t total = 0;
    for (int l = 0; l < 8; ++l) total += (size_t)sizes[2 * l] * sizes[2 * l + 1];
    std::vector<uint8_t> pyr(total);
    EXPECT(ora_orb_pyramid(a.data(), W, H, W, 8, 1, pyr.data()) == 0);
    std::vector<int32_t> xys(3 * 20000);
    int nf = 0;
    EXPECT(ora_fast(a.data(), W, H, W, 20, xys.data(), 20000, &nf) == 0);
    std::vector<float> resp(1000);
    std::mt19937 rng(3);
    for (auto& r : resp) r = (float)(rng() % 50);  // many ties
    std::vector<int32_t> perm(1000);
    EXPECT(ora_retain_best(resp.data(), 1000, 100, perm.data()) >= 100);
    EXPECT(ora_retain_best_depth(resp.data(), 1000, 100, 0, perm.data()) >= 100);  // heap-select path

    // matching: every cross-check mode, empty sides
    std::vector<int32_t> qi(N + 512), ti(N + 512);
    std::vector<float> dist(N + 512);
    int m = 0;
    for (int mode = 0; mode < 3; ++mode)
        EXPECT(ora_bf_match_hamming(da.data(), na, db.data(), nb, mode, qi.data(), ti.data(), dist.data(), &m) == 0);
    int m0 = 0;
    ora_bf_match_hamming(da.data(), 0, db.data(), nb, 1, qi.data(), ti.data(), dist.data(), &m0);
    ora_bf_match_hamming(da.data(), na, db.data(), 0, 1, qi.data(), ti.data(), dist.data(), &m0);
    ora_bf_match_hamming(da.data(), na, db.data(), nb, 1, qi.data(), ti.data(), dist.data(), &m);

    // float k-NN, k above the train count
    std::vector<float> fq(40 * 128), ft(3 * 128);
    for (auto& v : fq) v = (float)(rng() % 256);
    for (auto& v : ft) v = (float)(rng() % 256);
    std::vector<int32_t> kidx(40 * 4);
    std::vector<float> kd(40 * 4);
    for (int norm = 0; norm < 2; ++norm) EXPECT(ora_bf_knn_float(fq.data(), 40, ft.data(), 3, 128, 4, norm, kidx.data(), kd.data()) == 0);

    // geometry on the detected matches
    const double K[9] = {300, 0, 160, 0, 300, 120, 0, 0, 1};
    std::vector<double> p1(2 * (size_t)std::max(m, 1)), p2(2 * (size_t)std::max(m, 1));
    for (int i = 0; i < m; ++i) {
        p1[2 * i] = ka[qi[i]].x;
        p1[2 * i + 1] = ka[qi[i]].y;
        p2[2 * i] = kb[ti[i]].x;
        p2[2 * i + 1] = kb[ti[i]].y;
    }
    std::vector<double> E(90);
    std::vector<uint8_t> mask(std::max(m, 1)), mask2(std::max(m, 1));
    int rows = 0, iters = 0, good = 0;
    double R[9], t[3];
    if (ora_find_essential(p1.data(), p2.data(), m, K, 0.999, 1.0, 1000, E.data(), &rows, mask.data(), &iters) == 0 &&
        rows == 3)
        ora_recover_pose(E.data(), p1.data(), p2.data(), m, K, 50.0, nullptr, R, t, mask2.data(), &good);
    EXPECT(ora_find_essential(p1.data(), p2.data(), 4, K, 0.999, 1.0, 1000, E.data(), &rows, mask.data(), &iters) != 0);
    ora_find_essential(p1.data(), p2.data(), 5, K, 0.999, 1.0, 1000, E.data(), &rows, mask.data(), &iters);  // k x 3 rows
    ora_find_essential(p1.data(), p2.data(), m, K, 0.999, 1.0, 4096, E.data(), &rows, mask.data(), &iters);
    const double P1[12] = {300, 0, 160, 0, 0, 300, 120, 0, 0, 0, 1, 0};
    const double P2[12] = {300, 0, 160, -30, 0, 300, 120, 0, 0, 0, 1, 0};
    const double x1[8] = {100, 150, 200, 250, 80, 90, 100, 110}, x2[8] = {95, 146, 196, 247, 80, 90, 100, 110};
    double X[16];
    EXPECT(ora_triangulate(P1, P2, x1, x2, 4, X) == 0);

    // RANSAC parts: the sampler past one 1024-state chunk, the replay
    {
        std::vector<int32_t> sub(5 * 300);
        EXPECT(ora_ransac_subsets(m > 5 ? m : 6, 300, sub.data()) == 0);
        std::vector<int32_t> nmod(4096), cnt(4096 * 10), out(8);  // counts: 10 slots per hypothesis
        for (int i = 0; i < 4096; ++i) nmod[i] = 1 + (int)(rng() % 3);
        for (auto& c : cnt) c = (int)(rng() % 200);
        ora_ransac_replay(nmod.data(), cnt.data(), 4096, 200, 0.999, 4096, out.data());
        ora_ransac_replay(nmod.data(), cnt.data(), 0, 200, 0.999, 1000, out.data());
    }

    // SURF, textured, a cap below the count and a tiny frame
    {
        std::vector<ora_keypoint> uk(8192);
        std::vector<float> ud(8192 * 64);
        int nu = 0;
        EXPECT(ora_surf_detect_and_compute(a.data(), W, H, W, 400.0, uk.data(), ud.data(), 8192, &nu) == 0 && nu > 0);
        ora_surf_detect_and_compute(a.data(), W, H, W, 400.0, uk.data(), ud.data(), 2, &nu);
        std::vector<uint8_t> tiny((size_t)12 * 9, 200);
        ora_surf_detect_and_compute(tiny.data(), 12, 9, 12, 0.0, uk.data(), ud.data(), 8192, &nu);
    }

    // SIFT, textured and blank
    {
        std::vector<ora_keypoint> sk(4000);
        std::vector<float> sd(4000 * 128);
        int ns = 0;
        EXPECT(ora_sift_detect_and_compute(a.data(), W, H, W, sk.data(), sd.data(), 4000, &ns) == 0 && ns > 0);
        std::vector<uint8_t> flat((size_t)64 * 48, 90);
        ora_sift_detect_and_compute(flat.data(), 64, 48, 64, sk.data(), sd.data(), 4000, &ns);
        ora_sift_detect_and_compute(a.data(), W, H, W, sk.data(), sd.data(), 3, &ns);  // cap below the count
    }

    // pre-processing
    const double dist5[5] = {0.14, -0.25, -0.005, -0.005, 0.0};
    double newK[9];
    EXPECT(ora_get_optimal_new_camera_matrix(K, dist5, 5, W, H, 1.0, W, H, newK) == 0);
    std::vector<uint8_t> und((size_t)W * H);
    std::vector<int16_t> mxy((size_t)W * H * 2);
    std::vector<uint16_t> mfr((size_t)W * H);
    EXPECT(ora_undistort(a.data(), W, H, W, K, dist5, 5, newK, und.data(), W, mxy.data(), mfr.data()) == 0);

    // tiny and blank frames
    for (int s : {8, 17, 40}) {
        auto tiny = textured(s, s, 11, 0.0);
        int nt = 0;
        ora_orb_detect_and_compute(tiny.data(), s, s, s, 500, ka.data(), da.data(), N + 512, &nt);
    }
    std::vector<uint8_t> blank((size_t)W * H, 128);
    int nbk = -1;
    EXPECT(ora_orb_detect_and_compute(blank.data(), W, H, W, N, ka.data(), da.data(), N + 512, &nbk) == 0 && nbk == 0);

    std::printf("sanitize_check: %d keypoints / %d keypoints, %d matches, E rows %d, %d RANSAC iterations, good %d; %d failed checks\n",
                na, nb, m, rows, iters, good, fails);
    return fails ? 1 : 0;
}
