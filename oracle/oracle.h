// TEST INFRASTRUCTURE ONLY — the CPU oracle for droplet_visual_odometry_amd.
//
// A plain C++17 restatement of the OpenCV operators the reference's hot path
// calls (scripts/visual_odometry_v3.py:373 detectAndCompute, :219 BFMatcher.match,
// :297 findEssentialMat, :303 recoverPose, :265 triangulatePoints).  OpenCV is a
// third-party dependency that is neither vendored in the reference nor installed
// here, so every function below restates OpenCV 4.x's published
// algorithm; each cites the reference call site it serves and the OpenCV routine
// it follows.  Parity status: PARTIALLY PINNED — see DESIGN.md §3 (KAT-1 keypoint
// arithmetic from scripts/back_up_files/frame_extraction_notes.txt:6-7, analytic
// geometry KATs); bit-level OpenCV parity is unpinned because OpenCV is absent.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library.  The product (droplet_visual_odometry_amd) never links it.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Same 28-byte layout as cv::KeyPoint's python-visible fields and dvo_keypoint.
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} ora_keypoint;

// ---- ORB (cv::ORB_create() defaults, nfeatures variable) -------------------
int ora_orb_level_sizes(int w, int h, int nlevels, int* sizes /*2*nlevels*/);
int ora_orb_features_per_level(int nfeatures, int nlevels, int* out);
int ora_orb_level_scales(int nlevels, float* out);
// Pyramid (unblurred when blurred==0, else after GaussianBlur(7x7, sigma 2)).
// out: levels packed back to back, each w_l*h_l bytes.
int ora_orb_pyramid(const uint8_t* img, int w, int h, int stride, int nlevels,
                    int blurred, uint8_t* out);
// FAST-9/16 with non-max suppression on one image: (x, y, score) triples in
// raster order.
int ora_fast(const uint8_t* img, int w, int h, int stride, int threshold,
             int32_t* xys, int cap, int* n);
// KeyPointsFilter::retainBest on a response array; perm gets the permutation
// applied (perm[i] = original index now at i); returns the new size.
int ora_retain_best(const float* resp, int n, int n_points, int32_t* perm);
// Restated libstdc++ introselect with an overridable depth limit (-1 = default);
// used to pin the GPU's parallel emulation including the heap-select path.
int ora_retain_best_depth(const float* resp, int n, int n_points, int depth, int32_t* perm);
int ora_orb_detect_and_compute(const uint8_t* img, int w, int h, int stride,
                               int nfeatures, ora_keypoint* kps, uint8_t* desc,
                               int cap, int* n_out);
// The same with a choice of OpenCV semantics (the reference
// most likely ran OpenCV 3.2): 0 = 4.x (INTER_LINEAR_EXACT pyramid, retainBest
// nth at n-1; the default everywhere), 1 = 3.2 (INTER_LINEAR 11-bit pyramid with
// the SSE2 vertical pass, retainBest nth at n).  The blur is the same in both.
int ora_orb_detect_and_compute_v(const uint8_t* img, int w, int h, int stride, int nfeatures, int semantics,
                                 ora_keypoint* kps, uint8_t* desc, int cap, int* n_out);
int ora_orb_pyramid_v(const uint8_t* img, int w, int h, int stride, int nlevels, int blurred, int semantics,
                      uint8_t* out);
int ora_retain_best_v(const float* resp, int n, int n_points, int semantics, int32_t* perm);
int ora_retain_best_depth_v(const float* resp, int n, int n_points, int depth, int semantics, int32_t* perm);

// ---- BFMatcher(NORM_HAMMING, crossCheck) ------------------------------------
// mode 0: no cross check, 1: OpenCV 4.x mutual check, 2: OpenCV 3.x reverse-only.
int ora_bf_match_hamming(const uint8_t* dq, int nq, const uint8_t* dt, int nt,
                         int mode, int32_t* qidx, int32_t* tidx, float* dist,
                         int* m_out);

// ---- BFMatcher(NORM_L1).knnMatch / FLANN stand-in on float descriptors ------
// norm 0: L1 (cv::normL1), 1: squared L2 (flann::L2).  tidx/dist: nq x k,
// -1 / FLT_MAX where fewer than k trains exist.
int ora_bf_knn_float(const float* dq, int nq, const float* dt, int nt, int dim, int k, int norm,
                     int32_t* tidx, float* dist);

// ---- FlannBasedMatcher(KDTREE trees, checks).knnMatch on float descriptors
// (flann.cpp; the 'flann' mode, visual_odometry_v3.py:206-212): index over the
// train set, squared L2 distances, k smallest (distance, index) among the
// checked points.  rng_state: cv::theRNG() state before (in) / after (out).
// -1 on bad arguments (OpenCV asserts k <= train size).
int ora_flann_knn(const float* dq, int nq, const float* dt, int nt, int dim, int k, int trees, int checks,
                  uint64_t* rng_state, int32_t* tidx, float* dist);
uint64_t ora_flann_rng_after(uint64_t state, const int32_t* n, int calls, int trees);

// ---- findEssentialMat(RANSAC) / recoverPose / triangulatePoints -------------
// E_out holds up to 10 stacked 3x3 models (only when m == 5); *rows = 3*k.
// Returns 0 on success, <0 on failure (E empty).
int ora_find_essential(const double* p1, const double* p2, int m, const double* K,
                       double prob, double threshold, int max_iters,
                       double* E_out, int* rows, uint8_t* mask, int* iters_run);
int ora_recover_pose(const double* E, const double* p1, const double* p2, int m,
                     const double* K, double dist_thresh, const uint8_t* mask_in,
                     double* R, double* t, uint8_t* mask_out, int* good);
// x1, x2: 2 x k row-major (row 0 = x, row 1 = y).  X: 4 x k row-major.
int ora_triangulate(const double* P1, const double* P2, const double* x1,
                    const double* x2, int k, double* X);
// The 5-point kernel on 5 normalised correspondences; models: up to 10 x 9.
int ora_five_point(const double* p1, const double* p2, double* models, int* n);
// Helpers exposed for unit KATs.
int ora_jacobi_svd(double* At, int m, int n, int n1, double* W, double* Vt);
int ora_solve_poly(const double* coeffs, int n, int max_iters, double* roots /*2n*/);
// Analysis hooks (tools/dk_cycle_stats.py): the polynomial of this thread's last
// ora_five_point, and solvePoly's per-sweep root-state hashes (trace[max_iters] = sweeps run).
int ora_last_five_point_poly(double* c /*11*/);
int ora_solve_poly_trace(const double* coeffs, int n, int max_iters, uint64_t* trace /*max_iters + 1*/);
int ora_ransac_update_num_iters(double p, double ep, int model_points, int max_iters);
// RANSAC pieces pinned separately: getSubset's draws (n x 5) and the sequential
// best / niters bookkeeping over per-hypothesis counts (cnt: n x 10);
// out = {iterations, niters, max good, best hypothesis, best model}.
int ora_ransac_subsets(int m, int n, int32_t* idx);
int ora_ransac_replay(const int32_t* nmod, const int32_t* cnt, int n, int m, double prob, int max_iters, int32_t* out);

// ---- SIFT_create().detectAndCompute (sift.cpp; the 'sift' / 'knn_sift' /
// 'flann' modes, visual_odometry_v3.py:99-103, :373).  kps sorted as
// removeDuplicatedSorted leaves them; desc: n x 128 floats (integer values).
int ora_sift_detect_and_compute(const uint8_t* img, int w, int h, int stride, ora_keypoint* kps, float* desc, int cap,
                                int* n_out);

// ---- SURF_create(hessian).detectAndCompute (surf.cpp; the 'surf' mode,
// visual_odometry_v3.py:103-106, :373): nOctaves 4, nOctaveLayers 3, 64-d.
// kps in KeypointGreater order; desc: n x 64 floats.  -5 when cap < n.
int ora_surf_detect_and_compute(const uint8_t* img, int w, int h, int stride, double hessian_threshold,
                                ora_keypoint* kps, float* desc, int cap, int* n_out);

/* Image pre-processing (undistort.cpp): cv::getOptimalNewCameraMatrix and
 * cv::undistort (striped initUndistortRectifyMap + remap INTER_LINEAR,
 * BORDER_CONSTANT).  xy / frac receive the 16SC2 / 16UC1 maps (w*h). */
int ora_get_optimal_new_camera_matrix(const double* K, const double* dist, int ndist, int w, int h, double alpha,
                                      int new_w, int new_h, double* newK);
int ora_undistort(const uint8_t* src, int w, int h, int stride, const double* K, const double* dist, int ndist,
                  const double* newK, uint8_t* dst, int dstride, int16_t* xy, uint16_t* frac);

#ifdef __cplusplus
}
#endif
