/* droplet_visual_odometry_amd — C ABI of the MI355X visual-odometry front end.
 *
 * This is the drop-in boundary underneath the reference's Python call surface
 * (scripts/visual_odometry_v3.py, scripts/pose_estimation_module.py).  Each
 * per-call entry point replaces exactly one OpenCV operator the reference
 * invokes on its hot path; the batched stream API runs the whole per-pair path
 * (v3:384-408) for many frames per launch.  All compute runs in hand-written
 * HIP kernels for gfx950; there is no CPU fallback.
 *
 * Conventions: plain pointers and sizes, caller-owned outputs, int status
 * (DVO_OK or a negative DVO_E* code, message via dvo_last_error).  No C++
 * exceptions cross this boundary.  One context per host thread.
 */
#ifndef DVO_H_
#define DVO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVO_OK 0
#define DVO_EINVAL (-1)   /* bad argument (cv2.error analogue)                     */
#define DVO_ENOFEAT (-2)  /* no descriptors where the reference would hit None     */
#define DVO_EFEWPTS (-3)  /* fewer than 5 correspondences: findEssentialMat empty  */
#define DVO_EHIP (-4)     /* HIP runtime failure                                   */
#define DVO_ECAP (-5)     /* caller buffer too small; *_out holds the needed size  */
#define DVO_ENOMODEL (-6) /* RANSAC found no model (E empty)                       */

typedef struct dvo_ctx dvo_ctx;
typedef struct dvo_stream dvo_stream;
typedef struct dvo_undistort dvo_undistort;

/* cv::KeyPoint as the reference's Python sees it (28 bytes). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} dvo_keypoint;

/* cv::DMatch (16 bytes). */
typedef struct {
    int32_t queryIdx, trainIdx, imgIdx;
    float distance;
} dvo_dmatch;

/* OpenCV version whose ORB / BFMatcher semantics the path reproduces.  The
 * reference pins none (package.xml:21-30); its Python 2.7 .pyc files and ROS
 * Melodic docs point at OpenCV 3.2.  4.x is the default.
 * DVO_OPENCV_32: the pyramid is resize(INTER_LINEAR) with 11-bit weights and
 * the SSE2 vertical pass (4.x: INTER_LINEAR_EXACT), and retainBest runs
 * nth_element at n instead of n - 1; everything else is common to both. */
#define DVO_OPENCV_4X 0
#define DVO_OPENCV_32 1

/* cv.ORB_create() parameters (visual_odometry_v3.py:96 uses the defaults).
 * Only the defaults other than nfeatures are implemented; others -> DVO_EINVAL. */
typedef struct {
    int32_t nfeatures;      /* 500   */
    float scale_factor;     /* 1.2f  */
    int32_t nlevels;        /* 8     */
    int32_t edge_threshold; /* 31    */
    int32_t first_level;    /* 0     */
    int32_t wta_k;          /* 2     */
    int32_t score_type;     /* 0 = HARRIS_SCORE */
    int32_t patch_size;     /* 31    */
    int32_t fast_threshold; /* 20    */
    int32_t opencv_semantics; /* DVO_OPENCV_4X (0) or DVO_OPENCV_32 */
} dvo_orb_params;

int dvo_version(void);
/* Source hash the library was built from (16 hex digits; build.py source_hash). */
const char* dvo_build_id(void);
int dvo_ctx_create(dvo_ctx** out, int device);
void dvo_ctx_destroy(dvo_ctx* ctx);
const char* dvo_last_error(const dvo_ctx* ctx);

/* Replaces cv::ORB::detectAndCompute(img, None) — visual_odometry_v3.py:373.
 * img: host mono8, `stride` bytes per row.  Writes up to `cap` keypoints and
 * cap*32 descriptor bytes; *n_out = number found (DVO_ECAP if > cap). */
int dvo_orb_detect_and_compute(dvo_ctx* ctx, const dvo_orb_params* params, const uint8_t* img, int w, int h,
                               int stride, dvo_keypoint* kps, uint8_t* desc, int cap, int* n_out);

/* Replaces cv::BFMatcher(NORM_HAMMING, crossCheck).match(query, train) —
 * visual_odometry_v3.py:75 (construction) and :219 (call).  Output in
 * queryIdx order, as OpenCV returns it.  cross_check: 0 off, 1 OpenCV 4.x
 * mutual nearest neighbour, 2 OpenCV 3.x reverse-pass semantics. */
int dvo_bf_match_hamming(dvo_ctx* ctx, const uint8_t* dq, int nq, const uint8_t* dt, int nt, int cross_check,
                         dvo_dmatch* out, int cap, int* m_out);

/* Replaces cv::BFMatcher(NORM_L1).knnMatch(query, train, k) (k = 1: .match) on
 * float descriptors — the SIFT/SURF modes, visual_odometry_v3.py:99-106
 * (construction) and :200-204, :214-215 (calls) — and, with DVO_NORM_L2SQR,
 * serves cv::FlannBasedMatcher(KDTREE).knnMatch (:206-212) by exact search
 * (FLANN reports squared L2; its randomized kd-trees are approximate, so
 * exact results are the FLANN result whenever FLANN finds the true
 * neighbours).  dq: nq x dim, dt: nt x dim floats, dim 64 (SURF) or 128
 * (SIFT), k 1..4.  Per query, train_idx/dist get k entries in OpenCV's
 * order (ascending distance, lower train index first on ties); -1 / FLT_MAX
 * pad queries with fewer than k trains. */
#define DVO_NORM_L1 0
#define DVO_NORM_L2SQR 1
int dvo_bf_knn_float(dvo_ctx* ctx, const float* dq, int nq, const float* dt, int nt, int dim, int k, int norm,
                     int32_t* train_idx, float* dist);

/* Replaces cv::FlannBasedMatcher(dict(algorithm=FLANN_INDEX_KDTREE, trees),
 * dict(checks)).knnMatch(query, train, k) on float descriptors — the 'flann'
 * mode, visual_odometry_v3.py:206-212 (trees 5, checks 50, k 2), whose ratio
 * test follows at :223-228.  OpenCV's randomized kd-forest (FLANN 1.6 as
 * bundled with OpenCV 4.x, restated in oracle/flann.cpp) is built over the
 * train set and searched approximately, on the device: the same trees, the
 * same visiting order, the same neighbours.  The trees are drawn from
 * cv::theRNG(), process state in the reference; *rng_state carries it: the
 * state before the call on entry (a fresh thread's is 0xFFFFFFFF) and after
 * it on return (advanced trees * (2 nt - 1) draws).  dist: squared L2 (as
 * FLANN reports it; FlannBasedMatcher returns its square root); per query k
 * entries ascending by (distance, train index).  dim a multiple of 4 up to
 * 256, k <= nt (else DVO_EINVAL, where FLANN asserts), nt <= 65536.  An empty
 * query or train set returns at once without touching the state. */
int dvo_flann_knn(dvo_ctx* ctx, const float* dq, int nq, const float* dt, int nt, int dim, int k, int trees,
                  int checks, uint64_t* rng_state, int32_t* train_idx, float* dist);

/* Replaces cv::xfeatures2d::SIFT_create().detectAndCompute(img, None) — the
 * detector of the 'sift' / 'knn_sift' / 'flann' modes, visual_odometry_v3.py:100
 * (construction) and :373 (call).  Default parameters (nfeatures 0, 3 octave
 * layers, contrast 0.04, edge 10, sigma 1.6, input upscaled 2x).  img: host
 * mono8.  kps: keypoints in OpenCV's removeDuplicatedSorted order; desc: n x
 * 128 floats (integer values 0..255).  *n_out = count (DVO_ECAP if > cap). */
int dvo_sift_detect_and_compute(dvo_ctx* ctx, const uint8_t* img, int w, int h, int stride, dvo_keypoint* kps,
                                float* desc, int cap, int* n_out);

/* Replaces cv::xfeatures2d::SURF_create(hessianThreshold).detectAndCompute(img,
 * None) — the detector of the 'surf' mode, visual_odometry_v3.py:104
 * (SURF_create(400)) and :373 (call).  Other parameters at their defaults
 * (nOctaves 4, nOctaveLayers 3, extended false, upright false).  img: host
 * mono8.  kps: keypoints in OpenCV's KeypointGreater order (response, size,
 * octave descending, then y descending, x ascending), class_id = sign of the
 * Hessian trace; desc: n x 64 floats, unit norm.  *n_out = count (DVO_ECAP if
 * > cap). */
int dvo_surf_detect_and_compute(dvo_ctx* ctx, const uint8_t* img, int w, int h, int stride, double hessian_threshold,
                                dvo_keypoint* kps, float* desc, int cap, int* n_out);

/* Replaces cv::findEssentialMat(points1, points2, K, RANSAC, prob, threshold,
 * maxIters) — visual_odometry_v3.py:297-300.  p1/p2: m x 2 doubles (pixel
 * coords, the float32 KeyPoint_convert output widened).  E receives 3 rows
 * (or 3*k rows when m == 5, as OpenCV); cap 90 doubles.  mask: m bytes 0/1. */
int dvo_find_essential_mat(dvo_ctx* ctx, const double* p1, const double* p2, int m, const double* K, double prob,
                           double threshold, int max_iters, double* E, int* e_rows, uint8_t* mask);

/* Replaces cv::recoverPose(E, points1, points2, K, distanceThresh=50, mask) —
 * visual_odometry_v3.py:303-306.  R row-major 3x3, t unit 3-vector,
 * mask_out m bytes 0/255, *good = cheirality count (the Python retval). */
int dvo_recover_pose(dvo_ctx* ctx, const double* E, int e_rows, const double* p1, const double* p2, int m,
                     const double* K, double dist_thresh, const uint8_t* mask_in, double* R, double* t,
                     uint8_t* mask_out, int* good);

/* Replaces cv::triangulatePoints(P1, P2, x1, x2) — visual_odometry_v3.py:265.
 * P1/P2 row-major 3x4; x1/x2 2 x k row-major; X 4 x k row-major. */
int dvo_triangulate_points(dvo_ctx* ctx, const double* P1, const double* P2, const double* x1, const double* x2,
                           int k, double* X);

/* ---------------------------------------------------------------------------
 * Image pre-processing of ros_img_msg_to_opencv_image (visual_odometry_v3.py:110-135).
 * dist: k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]] (ndist 0, 4, 5, 8 or 12). */

/* Replaces cv::getOptimalNewCameraMatrix(K, dist, (w, h), alpha, (new_w, new_h))
 * — visual_odometry_v3.py:117.  Host arithmetic; newK row-major 3x3. */
int dvo_get_optimal_new_camera_matrix(const double* K, const double* dist, int ndist, int w, int h, double alpha,
                                      int new_w, int new_h, double* newK);

/* Replaces cv::undistort(img, K, dist, None, newK) — visual_odometry_v3.py:120.
 * The remap table (OpenCV's striped initUndistortRectifyMap, CV_16SC2 + 1/32
 * fractions) is built once on the device; apply = remap(INTER_LINEAR,
 * BORDER_CONSTANT) of n device frames (dst may be a dvo_stream's input);
 * hip_stream NULL = the context's stream. newK NULL = K. */
int dvo_undistort_create(dvo_ctx* ctx, const double* K, const double* dist, int ndist, const double* newK, int w,
                         int h, dvo_undistort** out);
void dvo_undistort_destroy(dvo_undistort* u);
int dvo_undistort_apply(dvo_undistort* u, const uint8_t* d_src, int n, int64_t src_frame_stride, int src_pitch,
                        uint8_t* d_dst, int64_t dst_frame_stride, int dst_pitch, void* hip_stream);
/* Host image in, host image out (synchronous; the drop-in's cv.undistort). */
int dvo_undistort_image(dvo_undistort* u, const uint8_t* img, int stride, uint8_t* out, int out_stride);
/* Test hook: the device remap table (w*h*2 int16, w*h uint16). */
int dvo_undistort_get_map(dvo_undistort* u, int16_t* xy, uint16_t* frac);

/* ---------------------------------------------------------------------------
 * Batched frame stream: the whole per-pair path of visual_odometry_calculations
 * (v3:384-408: detect both frames, match, E/RANSAC, recoverPose) for n_frames
 * device-resident frames -> n_frames-1 pair records, one launch sequence on the
 * stream's HIP stream.  Each frame is detected once and its features serve both
 * pairs it belongs to (identical outputs to re-detecting, v3:387-392). */
typedef struct {
    int32_t width, height, max_frames;
    dvo_orb_params orb;
    double K[9];
    double prob;        /* 0.999 */
    double threshold;   /* 1.0   */
    int32_t max_iters;  /* 1000  */
    int32_t cross_check;/* 1     */
    double dist_thresh; /* 50.0  */
} dvo_stream_config;

/* One pair's result, 256 bytes, gathered across ranks by RCCL all-gather. */
typedef struct {
    double R[9];
    double t[3];
    double E[9];
    int32_t n_kp_prev, n_kp_cur, n_matches, n_inliers;
    int32_t n_good, ransac_iters, status, n_models;
    int32_t n_hypotheses;  /* 5-point samples solved on the device (>= ransac_iters: rounds overshoot) */
    int32_t pad0;
    double reserved[6];
} dvo_pair_record;

int dvo_stream_create(dvo_ctx* ctx, const dvo_stream_config* cfg, dvo_stream** out);
void dvo_stream_destroy(dvo_stream* s);
/* d_frames: device pointer, frame i at d_frames + i*frame_stride, rows `stride`
 * bytes apart.  d_records: device pointer to n_frames-1 records.  Asynchronous
 * on the stream's HIP stream; call dvo_stream_sync before reading results. */
int dvo_stream_process(dvo_stream* s, const uint8_t* d_frames, int n_frames, int64_t frame_stride, int stride,
                       dvo_pair_record* d_records);
int dvo_stream_sync(dvo_stream* s);
/* The reference's own schedule: visual_odometry_calculations (v3:384-408) runs
 * compute_current_image_elements on BOTH frames of every pair (v3:387-392), so
 * each frame is detected twice in a stream.  d_frames holds 2 n_pairs frames;
 * pair p is frames 2p (previous) and 2p + 1 (current), each detected on its own.
 * Records, matches and the pose tail are per pair exactly as after
 * dvo_stream_process (the pair's outputs are identical: detection is a function
 * of the frame).  2 n_pairs <= max_frames.  Used for the reference-equivalent
 * timing leg of bench.py. */
int dvo_stream_process_pairs(dvo_stream* s, const uint8_t* d_frames, int n_pairs, int64_t frame_stride, int stride,
                             dvo_pair_record* d_records);
/* Pipelined batches.  findEssentialMat's RANSAC loop (RANSACPointSetRegistrator::run,
 * the hot part of v3:297) runs in rounds of hypotheses, [0, 32), [32, 64), [64, 128),
 * [128, 256), then the rest up to the adaptive bound, each round stopping where the
 * sequential loop would (the result is the loop's, bit for bit, whatever the rounds).
 * dvo_stream_process runs a batch's rounds back to back.  dvo_stream_submit runs
 * detection and matching of its batch and then ONE merged round in which each of the
 * last dvo_pipeline_depth() submitted batches takes its next round; the batch whose last
 * round ran is retired (recoverPose, its records written), so a batch's records are
 * complete dvo_pipeline_depth() - 1 submits later, or after dvo_stream_drain.  The
 * records buffer and frames of every pending batch must stay allocated until then
 * (frames only until the submit's detection has run).  dvo_stream_retired lists the
 * batches the last submit / drain / process call retired, oldest first (their records
 * pointers and pair counts), returning how many; dvo_stream_pose_tail_batch runs the
 * pose tail over one of them.  Records are identical to dvo_stream_process's.
 * Footprint: the per-pair geometry (points, RANSAC models and state, pose buffers) is
 * held once per pair set, about 0.9 MB per pair at 1280x720, N 2000, maxIters 1000
 * (the models, max_iters x 720 B, dominate).  A stream is created with one set; its
 * first submit grows it to dvo_pipeline_depth() sets (synchronising the stream once),
 * so streams that only process / pair never pay for the pipeline. */
int dvo_pipeline_depth(void);
int dvo_stream_submit(dvo_stream* s, const uint8_t* d_frames, int n_frames, int64_t frame_stride, int stride,
                      dvo_pair_record* d_records);
int dvo_stream_submit_pairs(dvo_stream* s, const uint8_t* d_frames, int n_pairs, int64_t frame_stride, int stride,
                            dvo_pair_record* d_records);
int dvo_stream_drain(dvo_stream* s);
int dvo_stream_retired(dvo_stream* s, void** records, int* pairs, int cap);
/* One pair of HOST frames through the whole per-pair path in one synchronous
 * call: the device half of visual_odometry_calculations (v3:384-408) up to
 * recoverPose (v3:303) -- detectAndCompute of both frames (v3:387-392),
 * BFMatcher.match + crossCheck (v3:219), findEssentialMat(RANSAC, 0.999, 1.0)
 * (v3:297) and recoverPose (v3:303) -- returning the pair's record (R, t, E,
 * counts, status) in rec_out.  It replaces the drop-in's six separate operator
 * calls per pair (their host round trips and Python glue) with one; E, R and t
 * equal the operator-by-operator path's (the per-call RANSAC schedule: one
 * round, n_hypotheses as dvo_find_essential_mat).  reuse_prev = 1: the
 * previous frame is the last call's current frame, whose features the stream
 * kept on the device (prev_img may be NULL), so only cur_img is detected;
 * that cache is valid only after a call that returned DVO_OK (a failing call
 * invalidates it, and reuse_prev is then refused).  After a reuse_prev call,
 * dvo_stream_get_pyramid has frame 1 only (the previous frame's pyramid is not
 * kept); get_features has both frames.
 * Images: w x h mono8, rows `stride` bytes apart.  Needs max_frames >= 2. */
int dvo_stream_pair(dvo_stream* s, const uint8_t* prev_img, const uint8_t* cur_img, int stride, int reuse_prev,
                    dvo_pair_record* rec_out);
/* dvo_stream_process on undistorted frames: the n raw frames are remapped by u
 * into the stream's own frame slab first (same HIP stream), as the reference
 * undistorts every frame before detection (v3:120, v3:135). */
int dvo_stream_process_undistorted(dvo_stream* s, dvo_undistort* u, const uint8_t* d_frames, int n_frames,
                                   int64_t frame_stride, int stride, dvo_pair_record* d_records);
/* HIP stream the batch runs on (hipStream_t as void*; each dvo_stream owns
 * one, so batches on different dvo_streams may overlap on the device). */
void* dvo_stream_hip_stream(dvo_stream* s);
/* Pose tail of get_transformation_between_two_frames (v3:309-345) and
 * previous_current_matching (v3:367) for the pairs of the last
 * dvo_stream_process (read from that call's d_records, which must stay
 * allocated until the tail has run), on the device:
 *   P_cur = K [R | t];  X = triangulatePoints(P_prev, P_cur, c_prev, c_cur);
 *   d = |X[:3,0] - X[:3,1]| (homogeneous, not divided by W: D3);  s = L / d;
 *   T_rel = translation_matrix(t s) . euler_matrix(euler_from_matrix(R,'rxyz'),'sxyz');
 *   T_abs = T_abs_prev . T_rel.
 * P_prev / T_abs_prev carry over between calls on the device; set them with
 * dvo_stream_reset_pose (controlled mode: P0 = K [I | 0], v3:164-166).
 * d_corners_*: device [pairs][k][2] doubles (k >= 2).  Outputs device [pairs][16]. */
int dvo_stream_reset_pose(dvo_stream* s, const double* P0 /* host 12 */, const double* T0 /* host 16 */);
/* Make s use owner's pose carry, so batches alternating between streams (each
 * stream runs on its own HIP stream; batches overlap on the device) chain one
 * pose stream: pose tails on a shared carry run in call order via HIP events. */
int dvo_stream_share_pose(dvo_stream* s, dvo_stream* owner);
int dvo_stream_pose_tail(dvo_stream* s, const double* d_corners_prev, const double* d_corners_cur, int k,
                         double marker_length, double* d_T_rel, double* d_T_abs);
/* The same for a retired batch's records (pipelined submits; pairs = its pair count). */
int dvo_stream_pose_tail_batch(dvo_stream* s, const dvo_pair_record* d_records, int pairs, const double* d_corners_prev,
                               const double* d_corners_cur, int k, double marker_length, double* d_T_rel,
                               double* d_T_abs);

/* The same pose tail over caller-supplied pair records: the reassembly step of
 * one pose stream sharded across ranks.  Every rank computes
 * the records of its run of pairs (dvo_stream_process), the ranks all-gather
 * records and per-pair marker corners, and rank 0 runs this over the whole
 * window in pair order.  The tail reads only R, t, status and n_models of each
 * record (a pair counts as successful iff status == DVO_OK and n_models == 1,
 * as in dvo_stream_pose_tail), so P_prev of the first pair of a run is the
 * last successful pair's even when it lies on another rank: the result is
 * bit-identical to one rank running dvo_stream_pose_tail over the stream.
 * K: host 9 doubles.  d_carry: device 28 doubles, P_prev (3x4) | T_abs (4x4),
 * the state before the first pair on entry and after the last on return
 * (controlled mode: P0 = K [I | 0], v3:164-166).  Asynchronous on hip_stream
 * (NULL = the context's stream). */
int dvo_pose_tail_records(dvo_ctx* ctx, const dvo_pair_record* d_records, int pairs, const double* K,
                          const double* d_corners_prev, const double* d_corners_cur, int k, double marker_length,
                          double* d_carry, double* d_T_rel, double* d_T_abs, void* hip_stream);

/* The pair-parallel half of that tail on one rank's run of a gathered window:
 * T_rel of pairs [p0, p0 + n) of the window's `pairs` records (d_T_rel[0 .. n)),
 * each triangulating against the last successful pair before it in the window
 * (or d_P_carry, 12 doubles, when none is), then d_P_carry advanced past the
 * window (to its last successful pair's K [R | t]).  Every rank runs it over its
 * own pairs, rank 0 gathers the T_rel and runs dvo_pose_chain: the same values,
 * bit for bit, as dvo_pose_tail_records over the window on one rank.  Corner
 * arrays are the window's ([pairs][k][2]).  Asynchronous on hip_stream. */
int dvo_pose_rel_range(dvo_ctx* ctx, const dvo_pair_record* d_records, int pairs, int p0, int n, const double* K,
                       const double* d_corners_prev, const double* d_corners_cur, int k, double marker_length,
                       double* d_P_carry, double* d_T_rel, void* hip_stream);

/* The same chain on the host (host arrays; the device kernel's arithmetic, bit for bit): the
 * chain is one sequential product per pair, which a CPU core runs in ~50 ns per pair while
 * the GPU is busy with the next batches, where the one-wave kernel slows to ~1.5 us per pair
 * (round 5).  Rank 0 of a sharded stream chains the gathered T_rel here. */
int dvo_pose_chain_host(const double* T_rel, int n, double* T_carry, double* T_abs);

/* The absolute-pose chain of previous_current_matching (v3:367,
 * T_robot_cur = T_robot_prev . T_prev->cur) on its own, for pose streams
 * reassembled from sharded runs: rank 0 all-gathers every
 * rank's T_rel and chains them in pair order with the same arithmetic as
 * dvo_stream_pose_tail, so the result is bit-identical to one rank chaining the
 * whole stream.  d_T_rel: device [n][16]; d_T_carry: device 16 doubles, the pose
 * before the first pair on entry and after the last on return; d_T_abs: device
 * [n][16].  Asynchronous on hip_stream (NULL = the context's stream). */
int dvo_pose_chain(dvo_ctx* ctx, const double* d_T_rel, int n, double* d_T_carry, double* d_T_abs, void* hip_stream);

/* Per-stage device time via HIP events recorded on the stream's HIP stream
 * around each kernel group (0 pyramid, 1 blur, 2 fast, 3 select+harris,
 * 4 describe, 5 match, 6 ransac, 7 recoverPose+records, 8 pose tail).  Accumulated over
 * every dvo_stream_process since profiling was enabled. */
#define DVO_NSTAGES 9  /* ... 8 pose tail */
int dvo_stream_set_profiling(dvo_stream* s, int enable);
int dvo_stream_stage_times(dvo_stream* s, double* ms /* DVO_NSTAGES */, int* calls);

/* Host copies of intermediate results of the last dvo_stream_process (tests).
 * get_pyramid(blurred = 1): the detection path blurs only the 39 x 44 descriptor
 * windows inside the describe kernel, so the whole GaussianBlur of the level is
 * computed on this call from the last process's frames, which must still be
 * alive (device frames passed to dvo_stream_process, or the stream's own upload
 * slab). */
int dvo_stream_get_features(dvo_stream* s, int frame, dvo_keypoint* kps, uint8_t* desc, int cap, int* n);
int dvo_stream_get_matches(dvo_stream* s, int pair, dvo_dmatch* out, int cap, int* m);
int dvo_stream_get_pyramid(dvo_stream* s, int frame, int level, int blurred, uint8_t* out, int cap);

/* Test hooks: exercise one device algorithm in isolation. */
/* KeyPointsFilter::retainBest permutation on `n` float responses (GPU emulation
 * of libstdc++ nth_element + partition); depth < 0 = libstdc++ default. */
int dvo_test_retain_best(dvo_ctx* ctx, const float* resp, int n, int n_points, int depth, int semantics,
                         int32_t* perm, int* k_out);
/* RANSACUpdateNumIters on the device for a batch of (ep) values. */
int dvo_test_update_num_iters(dvo_ctx* ctx, double p, const double* ep, int n, int model_points, int max_iters,
                              int32_t* out);
/* findEssentialMat's RANSAC sampler (getSubset with cv::RNG((uint64)-1)) for
 * one pair of m >= 6 correspondences: idx gets n x 5 indices. */
int dvo_test_ransac_subsets(dvo_ctx* ctx, int m, int n, int32_t* idx);
/* The RANSAC bookkeeping (best model / niters / stop) over n hypotheses'
 * model counts (nmod: n, cnt: n x 10); out = {iterations, niters, max good,
 * best hypothesis, best model}. */
int dvo_test_ransac_replay(dvo_ctx* ctx, const int32_t* nmod, const int32_t* cnt, int n, int m, double prob,
                           int max_iters, int32_t* out);
/* 5-point kernel on one sample of 5 normalised correspondences. */
int dvo_test_five_point(dvo_ctx* ctx, const double* q1, const double* q2, double* models, int* n);
/* The batched RANSAC score's single-precision Sampson decision on one model E
 * (9 doubles) and n normalised correspondences (n x {x1, y1, x2, y2}) at the
 * squared threshold t: dec[i] = 1 inlier / 0 outlier / -1 left to the f64 test,
 * exact[i] = the f64 test (computeError, err <= t). */
int dvo_test_sampson(dvo_ctx* ctx, const double* E, const double* pts, int n, float t, int8_t* dec,
                     uint8_t* exact);

#ifdef __cplusplus
}
#endif
#endif /* DVO_H_ */
