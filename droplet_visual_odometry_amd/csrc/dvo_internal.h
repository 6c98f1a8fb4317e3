// Internal declarations shared by the HIP translation units of libdvo_hip.so.
//
// Numerics contract: every file is compiled with
// -ffp-contract=off and IEEE-correct f32/f64 division and sqrt, so each float
// expression is evaluated in source order exactly like the CPU restatement of
// OpenCV (no FMA contraction, round-to-nearest-even), which makes the device
// results bit-identical to the oracle, not merely close.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dvo.h"

namespace dvo {


constexpr int kMaxLevels = 8;
// OpenCV semantics of the ORB path (dvo_orb_params.opencv_semantics): 4.x or 3.2.
constexpr int kOcv4 = DVO_OPENCV_4X, kOcv32 = DVO_OPENCV_32;
// FAST tile height (output rows).  Two-stream bench, 1280x720, round 2 kernel: 16 rows
// 66.8-67.2 K frames/s, 20: 67.7 K, 24: 68.2-69.1 K, 28: 65.7-66.1 K, 32: 67.1-67.9 K.  Round 3
// (per-wave compass/segment/score, word candidate lists, no separate blur pass;
// profiles/r03p_ab_fast_band_rows.txt, r03q_*): 20 73.7 K, 24 75.0 K, 28 75.9 K, 32 77.9 K
// (26 KB of LDS, still 6 workgroups per CU), 40 77.8 K (5 per CU), 48 76.9 K, 64 75.7 K:
// taller tiles cost fewer barriers and carried rows per output row.
#ifndef DVO_BAND_ROWS
#define DVO_BAND_ROWS 32
#endif
constexpr int kBandRows = DVO_BAND_ROWS;
constexpr int kFastTW = 124;        // FAST tile width (output columns; score columns 126 = LDS words 1..32)
constexpr int kBorder = 31;         // edgeThreshold == runByImageBorder border
constexpr int kMaxW = 4096;         // keys pack x, y in 12 bits each
#ifndef DVO_BLUR_TH
#define DVO_BLUR_TH 96
#endif
constexpr int kBlurTW = 248, kBlurTH = DVO_BLUR_TH;  // blur tile: 62 lanes x 4 columns, 4 waves x kBlurTH / 4 rows

// Per-level geometry of one ORB plan (identical for every frame of a stream).
struct LevelGeom {
    int w, h;
    float scale;          // getScale(l) = (float)pow(double(1.2f), l)
    int nper;             // features per level
    int pitch;            // row pitch of level l (l >= 1) in the pyramid slab, multiple of 16
    int bpitch;           // row pitch of level l in the blurred slab, multiple of 16
    int64_t pyr_off;      // byte offset of level l (l >= 1) in a frame's pyramid slab
    int64_t blur_off;     // byte offset of level l in a frame's blurred slab
    int xcoef_off, ycoef_off;  // resize coefficient tables of level l (l >= 1) in Buffers::coef
    int nbands;           // FAST tile rows (kBandRows each) over rows [31, h-31)
    int ntx;              // FAST tile columns (kFastTW each) over columns [31, w-31)
    int band_base;        // first FAST tile of this level within a frame (tile = band * ntx + col)
    int strip_base;       // first FAST column strip of this level within a frame (strip = level's col)
    int band_cap;         // candidate capacity per FAST tile
    int64_t band_cand_off;// u32 offset of this level's first tile slot within a frame
    int cand_cap;         // candidate capacity of the level (>= sum of its band caps)
    int64_t cand_off;     // u32 offset of this level's gathered list within a frame
    int tile_base;        // first blur tile of this level within a frame
    int tiles_x, tiles_y; // blur tiling
    int l32_x, l32_y;     // OpenCV 3.2 INTER_LINEAR tables of level l (l >= 1) in Buffers::coef32 (int4 entries)
    int l32_xs;           // columns below this take 3.2's SSE2 vertical pass, the rest the scalar one
};

struct Plan {
    int w, h, nlevels, nfeatures, kp_cap, fast_threshold;
    LevelGeom L[kMaxLevels];
    int64_t pyr_stride;       // bytes per frame (levels 1..7)
    int64_t blur_stride;      // bytes per frame (levels 0..7)
    int total_bands;          // FAST tiles per frame
    int total_strips;         // FAST column strips per frame (one workgroup each)
    int64_t band_cand_stride; // u32 per frame
    int64_t cand_stride;      // u32 per frame
    int total_tiles;          // blur tiles per frame
    int coef_total;           // ints in the resize coefficient table
    int coef32_total;         // ints in the OpenCV 3.2 resize tables
    int semantics;            // kOcv4 / kOcv32
};

// Resize coefficient of one destination column/row (resize.cpp INTER_LINEAR_EXACT):
// bits 0..12 source offset, 13..21 c1 (0..256, c0 = 256 - c1), 22..23 mode
// (0 interior, 1 clamp to src[0], 2 clamp to src[last]).
__host__ __device__ inline int coef_ofs(int c) { return c & 0x1FFF; }
__host__ __device__ inline int coef_c1(int c) { return (c >> 13) & 0x1FF; }
__host__ __device__ inline int coef_mode(int c) { return (c >> 22) & 3; }

// Device buffers of one stream (all sized for max_frames).
// Per-pair RANSAC state carried between the batch-wide round kernels
// (geometry.hip: sample -> solve -> score -> replay, at most two rounds).
struct RansacState {
    uint64_t rng;      // cv::RNG state after the last sampled subset
    int32_t niters;    // current adaptive iteration bound
    int32_t iter;      // iterations replayed so far
    int32_t maxgood;   // best inlier count so far
    int32_t h0, h1;    // hypotheses sampled in the current round: [h0, h1)
    int32_t m;         // correspondences
    int32_t best_h, best_i;  // best model: hypothesis, root
    int32_t pad[2];
};
constexpr int kDkMaxPasses = 4;  // Durand-Kerner passes per round (geometry.hip kDkBudgets)
// RANSAC rounds of a stream batch: round r solves hypotheses [bound[r-1], min(bound[r], niters)),
// the last round everything left.  A batch's pairs take one round per dvo_stream_submit call
// (the rounds of kRansacRounds consecutive batches run as ONE merged launch sequence), so a
// round costs no extra Durand-Kerner tail; dvo_stream_process runs them back to back.
// Hypotheses solved per pair at 1280x720 / 2000 features (oracle replay, tools/ransac_schedule_sim.py,
// profiles/r05c_*): 64 | rest 177.8, 32 | 64 | 128 | 256 | rest 141.9, for 132.2 iterations used.
#ifndef DVO_RANSAC_BOUNDS
#define DVO_RANSAC_BOUNDS 32, 64, 128, 256
#endif
constexpr int kRansacBounds[] = {DVO_RANSAC_BOUNDS, 1 << 30};
constexpr int kRansacRounds = sizeof(kRansacBounds) / sizeof(int);
constexpr int kMaxSets = 8;  // pair sets (batches in flight) of a merged round
static_assert(kRansacRounds <= kMaxSets, "one pair set per round in flight");
// One merged RANSAC round: launch pairs [0, nsets F) are nsets sets of F pairs (set k = pairs
// [k F, (k + 1) F), one stream batch each); set k runs round[k] (-1: idle) over its first
// npairs[k] pairs.  Round 0 starts a set's pairs (RNG, niters = maxIters).
struct RoundSpec {
    int nsets, F;
    int round[kMaxSets];
    int npairs[kMaxSets];
    int bound[kMaxSets];  // hypotheses bound of round r (the last: 1 << 30)
};
// Per-pair values the record needs from the frames (records_kernel), kept with the pair's set
// because the frames' buffers are rewritten by the next batch before the set retires.
struct PairHeader {
    int32_t nkp_prev, nkp_cur, flags, pad;
};

struct Buffers {
    uint8_t* pyr;
    uint8_t* blur;
    int32_t* coef;        // resize coefficient tables (Plan::coef_total ints)
    int32_t* coef32;      // OpenCV 3.2 resize tables (Plan::coef32_total ints)
    int32_t* band_cnt;    // [F][total_bands][kBandRows] FAST keeps per tile row
    uint32_t* band_cand;
    uint32_t* cand;       // gathered candidate keys (score<<24 | y<<12 | x)
    float* resp;          // Harris responses parallel to cand
    int32_t* sel_tmp;     // 2 * cand_stride per frame (Lpos / Rasc)
    int32_t* cnt1;        // [F][8] after FAST retainBest
    int32_t* cnt2;        // [F][8] after Harris retainBest
    dvo_keypoint* kps;    // [F][kp_cap]
    uint8_t* desc;        // [F][kp_cap][32] (also the matcher's operands, expanded in registers)
    int32_t* nkp;         // [F]
    int32_t* nn;          // [2][F][kp_cap] packed (dist << 16 | idx), -1 none
    int32_t* mq;          // [F][kp_cap] match queryIdx (sorted by (dist, q))
    int32_t* mt;          // [F][kp_cap] match trainIdx
    float* md;            // [F][kp_cap] match distance
    int32_t* nmatch;      // [sets F]
    // per pair, one copy per pair set ([sets][F] pairs: a set holds one batch until it retires)
    float* pts;           // [sets F][kp_cap][4] (x1, y1, x2, y2) KeyPoint_convert pixel coords
    double* npts;         // [sets F][kp_cap][4] normalised coords for RANSAC / recoverPose
    double* models;       // [sets F][hyp_cap][10][9]
    int32_t* nmod;        // [sets F][hyp_cap]
    int32_t* rcnt;        // [sets F][hyp_cap][10]
    int32_t* subsets;     // [sets F][hyp_cap][5]
    RansacState* rs;      // [sets F]
    double* fprec;        // [round blocks][128][64] five-point records of one round (a_off)
    int32_t* dk_off;      // [sets F + 1] round work list: hypotheses before each pair
    int32_t* a_off;       // [sets F + 1] 64-hypothesis blocks before each pair (stage A / C, records)
    int32_t* s_off;       // [sets F + 1] score blocks before each pair
    PairHeader* hdr;      // [sets][F]
    int32_t* dk_ctl;      // [2 + kDkMaxPasses]
    int32_t* dk_list;     // [kDkMaxPasses - 1][F * hyp_cap] parked Durand-Kerner polynomials
    int32_t* status;      // [F] per-frame error flags
    double* E;            // [sets F][90]
    int32_t* info;        // [sets F][4] rows, inliers, iters, status
    double* Rt;           // [sets F][12]
    int32_t* good;        // [sets F]
    double* pose_P;       // [sets F][72] recoverPose decompositions (4 P, R1, R2, t)
    int32_t* pose_cnt;    // [sets F][5] decomposition valid flag, cheirality counts
};


struct StreamParams {   // passed by value to every batch kernel
    Plan plan;
    Buffers buf;
    const uint8_t* frames;
    int64_t frame_stride;
    int in_pitch;
    int nframes;
    // Pair layout: 1 = a stream (pair p is frames p, p+1: each frame detected once and shared by two
    // pairs); 2 = independent pairs (pair p is frames 2p, 2p+1), the reference's own schedule, which
    // detects both frames of every pair (visual_odometry_v3.py:387-392).
    int pair_step;
};

__host__ __device__ inline int stream_pairs(const StreamParams& P) {
    return P.pair_step == 2 ? P.nframes / 2 : P.nframes - 1;
}
__host__ __device__ inline int pair_frame(const StreamParams& P, int p) { return P.pair_step == 2 ? 2 * p : p; }

__host__ __device__ inline const uint8_t* level_ptr(const StreamParams& P, int f, int l) {
    return l == 0 ? P.frames + (int64_t)f * P.frame_stride : P.buf.pyr + (int64_t)f * P.plan.pyr_stride + P.plan.L[l].pyr_off;
}
__host__ __device__ inline int level_pitch(const StreamParams& P, int l) { return l == 0 ? P.in_pitch : P.plan.L[l].pitch; }
__host__ __device__ inline uint8_t* blur_ptr(const StreamParams& P, int f, int l) {
    return P.buf.blur + (int64_t)f * P.plan.blur_stride + P.plan.L[l].blur_off;
}

// ---- numerics helpers shared by device code ----------------------------------
__device__ __forceinline__ int cv_round_f(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int cv_round_d(double v) { return (int)__builtin_rint(v); }
__device__ __forceinline__ int cv_floor_d(double v) { int i = (int)v; return i - (i > v); }

__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Arguments of the geometry kernels (findEssentialMat / recoverPose), shared by
// the batched stream and the per-call C-ABI entry points.
struct GeomArgs {
    const float* pts_f;     // [pairs][pts_stride][4] pixel coords (x1, y1, x2, y2) or null
    const double* pts_d;    // same layout in double, or null
    const int32_t* m_arr;   // [pairs] correspondence counts (device) or null
    int m_const;
    int64_t pts_stride;
    double fx, fy, cx, cy;
    double prob, threshold;
    int max_iters;
    double dist_thresh;
    double* npts;           // [pairs][pts_stride][4] normalised
    double* models;         // [pairs][hyp_cap][10][9] hypothesis models
    int32_t* nmod;          // [pairs][hyp_cap] models per hypothesis
    int32_t* cnt;           // [pairs][hyp_cap][10] inlier counts
    int32_t* subsets;       // [pairs][hyp_cap][5] sampled point indices
    RansacState* rs;        // [pairs]
    double* fprec;          // [round blocks][128][64] five-point records of the round (block = a_off[p] + (h - h0) / 64)
    int32_t* dk_off;        // [pairs + 1] round work-list offsets
    int32_t* a_off;         // [pairs + 1] 64-hypothesis blocks of the round before each pair
    int32_t* s_off;         // [pairs + 1] score blocks of the round before each pair
    int32_t* dk_ctl;        // [2 + kDkMaxPasses] -, pass-0 items, parked after pass k
    int32_t* dk_list;       // [kDkMaxPasses - 1][dk_list_cap] parked polynomials (work-list items)
    int64_t dk_list_cap;    // >= pairs * hyp_cap
    int hyp_cap;            // max(max_iters, 1)
    double* E;              // [pairs][90]
    int32_t* info;          // [pairs][4] rows, inliers, iters, status
    uint8_t* mask;          // [pairs][pts_stride] findEssentialMat mask, or null
    const uint8_t* mask_in; // [pairs][pts_stride] recoverPose input mask, or null
    double* Rt;             // [pairs][12] R row-major then t
    int32_t* good;          // [pairs]
    int32_t* pick;          // [pairs] chosen decomposition 0..3, or null
    uint8_t* pose_mask;     // [pairs][pts_stride][4] per-decomposition masks, or null
    double* pose_P;         // [pairs][72] decompositions [R1|t], [R2|t], [R1|-t], [R2|-t]; R1, R2, t
    int32_t* pose_cnt;      // [pairs][5] valid flag, cheirality counts of the 4 decompositions
};

constexpr int kStageNormalize = 1, kStageRansac = 2, kStagePose = 4, kStageFinish = 16;
// kStageOneRound: the per-call findEssentialMat (one pair): a single RANSAC round
// over every hypothesis up to maxIters, solved with one lane per root.  Stream
// batches keep the two-round schedule, so their records (n_hypotheses) do not
// depend on how a stream is split into batches or shards.
constexpr int kStageOneRound = 8;

// SIFT_create().detectAndCompute of one image (sift.hip).  Octave o has
// size ow[o] x oh[o] (octave 0 = the 2x upscaled input); its Gaussian layer l
// (0..5) starts at gp + gp_off[o * 6 + l] and DoG layer l (0..4) at
// dog + dog_off[o * 5 + l] (floats, rows of ow[o]).
constexpr int kSiftMaxOct = 16;
struct SiftArgs {
    float* gp;
    float* dog;
    float* tmp;             // row-pass buffer, ow[0] * oh[0]
    int64_t gp_off[kSiftMaxOct * 6];
    int64_t dog_off[kSiftMaxOct * 5];
    int ow[kSiftMaxOct], oh[kSiftMaxOct];
    int noct;
    int4* cand;             // (octave, layer, row, col) extrema
    int* ncand;
    int cand_cap;
    dvo_keypoint* raw;      // refined, oriented keypoints (unsorted)
    int* nraw;
    int kp_cap;
    int32_t* order;         // sort scratch, next power of two >= kp_cap
    dvo_keypoint* kps;      // final keypoints (sorted, deduplicated, input-image units)
    int* nkp;
    float* desc;            // kp_cap x 128
    int* flags;             // 1: candidate overflow, 2: keypoint overflow
};

// SURF_create(hessianThreshold).detectAndCompute (surf.hip): nOctaves 4,
// nOctaveLayers 3, 64-d descriptors, orientation on.
constexpr int kSurfOct = 4, kSurfLayers = 5, kSurfTot = kSurfOct * kSurfLayers;
struct SurfHaar {  // resizeHaarPattern output: 4 corner offsets + weight (host-built)
    int p0, p1, p2, p3;
    float w;
};
struct SurfArgs {
    const uint8_t* img;     // device copy of the image (pitch)
    int w, h, pitch;
    int32_t* sum;           // integral image, (h + 1) x (w + 1)
    float* det;             // per layer: rows x cols of the layer's octave
    float* trace;
    int64_t off[kSurfTot];  // element offset of each layer in det / trace
    int size[kSurfTot];     // (9 + 6 layer) << octave
    int rows[kSurfOct], cols[kSurfOct];
    const SurfHaar* haar;   // [kSurfTot][10]: Dx (3), Dy (3), Dxy (4) of calcLayerDetAndTrace
    const int8_t* apt;      // 113 x (i, j): the orientation disc, apt[n] = Point(i, j)
    const float* aptw;      // 113 weights gori[i + 6] * gori[j + 6]
    float thr;              // hessianThreshold
    dvo_keypoint* raw;      // extrema after interpolation (unsorted)
    int* nraw;
    int kp_cap;
    int32_t* order;         // sort scratch, next power of two >= kp_cap
    dvo_keypoint* kps;      // sorted (KeypointGreater), then oriented; size -1 = dropped
    float* dtmp;            // kp_cap x 64, descriptors in sorted order
    dvo_keypoint* out;      // compacted keypoints
    float* desc;            // compacted descriptors
    int* nout;
    int* flags;             // 2: keypoint overflow
    int nori;               // samples in the orientation disc (113)
    float gdesc[20];        // getGaussianKernel(20, 3.3)
};

// ---- host entry points of the kernels (implemented in the .hip files) -------
// ev: optional table of 2*DVO_NSTAGES events recorded around each stage.
inline void mark(hipEvent_t* ev, int stage, int end, hipStream_t s) {
    if (ev) hipEventRecord(ev[2 * stage + end], s);
}
// group_ev: when the batch's detection runs in frame groups (orb_groups(F) > 0), 2 x 5 events per
// group (stages 0..4 of group g at group_ev[10 g ..]) instead of ev's stages 0..4.
hipError_t launch_orb(const StreamParams& P, hipStream_t s, hipEvent_t* ev = nullptr, hipEvent_t* group_ev = nullptr);
int orb_groups(int nframes);
// dvo_stream_pair's feature bookkeeping in one launch, per 4-byte word i of the frame-0 / frame-1 / cache
// feature arrays (keypoints, descriptors, count, status): rotate = 1 (frame 0 holds the new current
// frame): frame 1 <- frame 0, frame 0 <- cache, cache <- frame 0; rotate = 0: cache <- frame 1.
struct FeatSlots {
    uint32_t* a[3][4];  // [frame 0, frame 1, cache][kps, desc, count, status]
    int words[4];
};
hipError_t launch_feature_rotate(const FeatSlots& f, int rotate, hipStream_t s);
// GaussianBlur of every level into Buffers::blur, for dvo_stream_get_pyramid(blurred): the
// detection path blurs only the pixels describe_kernel samples.
hipError_t launch_blur(const StreamParams& P, hipStream_t s);
// tsplit > 1 splits every pair's train stages over tsplit workgroups (one pair alone fills the chip)
hipError_t launch_match(const StreamParams& P, int cross_check, hipStream_t s, hipEvent_t* ev = nullptr, int tsplit = 1);
// one_round: a single RANSAC round over every hypothesis up to maxIters on the 16-lane Durand-Kerner
// (kStageOneRound, the per-call schedule: E, R, t are the same, n_hypotheses differs)
hipError_t launch_geometry(const StreamParams& P, const GeomArgs& g, dvo_pair_record* records, hipStream_t s,
                           hipEvent_t* ev = nullptr, bool one_round = false);
hipError_t launch_geometry_args(const GeomArgs& g, int pairs, int stages, hipStream_t s);
// Stream batches (api.cpp dvo_stream_submit): the per-set pieces.  g_all spans every set (pairs
// [0, nsets F)); g_set is one set's view (geom_set).
hipError_t launch_pair_header(const StreamParams& P, PairHeader* hdr, hipStream_t s);
hipError_t launch_ransac_round(const GeomArgs& g_all, const RoundSpec& spec, hipStream_t s);
hipError_t launch_retire(const GeomArgs& g_set, int pairs, const PairHeader* hdr, dvo_pair_record* records,
                         hipStream_t s);
// five-point record blocks a merged round can need (sizes Buffers::fprec, dk_list)
int64_t round_blocks_bound(int F, int hyp_cap);
int64_t round_items_bound(int F, int hyp_cap);
// Undistortion (undistort.hip): camera K, distortion k1 k2 p1 p2 k3 k4 k5 k6 s1..s4.
struct UndistortGeom {
    int w, h, stripe;
    double K[9];
    double dist[12];
};
hipError_t launch_undistort_map(const UndistortGeom& U, const double* d_ir, int16_t* d_xy, uint16_t* d_frac,
                                hipStream_t s);
hipError_t launch_undistort_remap(const UndistortGeom& U, const int16_t* d_xy, const uint16_t* d_frac,
                                  const uint8_t* d_src, int n, int64_t src_fstride, int src_pitch, uint8_t* d_dst,
                                  int64_t dst_fstride, int dst_pitch, hipStream_t s);

// carry: device [12 P_prev | 16 T_abs_prev]; updated in place.
// rec: the pairs' records (R, t, status, n_models are read).
hipError_t launch_pose_tail(const dvo_pair_record* rec, int pairs, const double* K, const double* cprev, const double* ccur, int k, double marker_length,
                            double* carry, double* T_rel, double* T_abs, hipStream_t s);
// T_abs[p] = T_carry . T_rel[0] ... T_rel[p] in pair order (the pose_tail chain on
// its own: the reassembled pose stream of a sharded run); T_carry is updated.
hipError_t launch_pose_chain(const double* T_rel /*[n][16]*/, int n, double* T_carry /*16*/, double* T_abs,
                             hipStream_t s);
// The pair-parallel half of the pose tail for pairs [p0, p0 + n) of a window of `pairs` records
// (T_rel[0 .. n)), then P_carry (12 doubles) advanced past the whole window.
hipError_t launch_pose_rel_range(const dvo_pair_record* rec, int pairs, int p0, int n, const double* K,
                                 const double* cprev, const double* ccur, int k, double marker_length, double* P_carry,
                                 double* T_rel, hipStream_t s);
hipError_t launch_triangulate(const double* d_P /*24*/, const double* d_x /*4 x k*/, int k, double* d_X, hipStream_t s);
// Float-descriptor kNN (NORM_L1 / squared L2), dim 64 or 128, k 1..4, over
// `ranges` = knn_ranges(nq, nt, CU count) train ranges; d_part / d_pidx hold
// ranges * nq * k partial slots (unused when ranges == 1).
int knn_ranges(int nq, int nt, int cus);
// d_bytes: knn_bytes_size(nq, nt, dim) bytes of workspace for the byte-valued fast path.
size_t knn_bytes_size(int nq, int nt, int dim);
hipError_t launch_knn_float(const float* d_q, int nq, const float* d_t, int nt, int dim, int k, int norm, int ranges,
                            void* d_bytes, float* d_part, int32_t* d_pidx, float* d_dist, int32_t* d_idx,
                            hipStream_t s);
// One-pair Hamming match (dvo_bf_match_hamming) on the stream's MFMA matcher;
// d_work: match_pair_work_size(nq, nt) bytes.  Output in queryIdx order.
size_t match_pair_work_size(int nq, int nt);
// d_taps: the 6 Gaussian kernels (initial blur, layers 1..5) back to back.
hipError_t launch_sift(const SiftArgs& A, const uint8_t* d_img, int w, int h, int stride, const float* d_taps,
                       const int* tap_off, const int* tap_n, hipStream_t s);
hipError_t launch_surf(const SurfArgs& a, hipStream_t s);
hipError_t launch_match_pair(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int cross_check, void* d_work,
                             dvo_dmatch* d_out, int* d_m, hipStream_t s);
// FLANN randomized kd-tree k-NN (flann.hip; the 'flann' mode's FlannBasedMatcher).
struct FlannBuildArgs {
    const float* data;  // train set [n][dim]
    int n, dim;
    int* ind;           // [n]
    float* xv;          // [n]
    int* sl;            // [n]
    int* sr;            // [n]
    const uint32_t* R;  // [2n - 1] draws of the tree
    int4* nodes;        // [2n - 1] nodes of the tree
    int4* open0;        // [n] open nodes, even levels
    int4* open1;        // [n] open nodes, odd levels
    int* cnt;           // [n + 2] open nodes per level
};
struct FlannSearchArgs {
    const float* q;
    const float* t;
    const int4* nodes;  // [trees][2n - 1]
    int nq, n, dim, k, trees, checks;
    int32_t* idx;       // [nq][k]
    float* dist;        // [nq][k] squared L2
    int32_t* flag;      // [nq]
};
size_t flann_search_lds(int n);
hipError_t launch_flann_draws(const uint64_t* d_chunk_state, int nchunk, int total, uint32_t* d_R, hipStream_t s);
hipError_t launch_flann_shuffle(const uint32_t* d_R, int n, int* d_cnt, int* d_off, int* d_fill, int* d_list,
                                const int* d_ind, int* d_new_ind, hipStream_t s);
hipError_t launch_flann_root(const FlannBuildArgs& a, hipStream_t s);
hipError_t launch_flann_level(const FlannBuildArgs& a, int level, int max_open, hipStream_t s);
hipError_t launch_flann_search(const FlannSearchArgs& a, hipStream_t s);
hipError_t launch_flann_redo_list(const int32_t* d_flag, int nq, int32_t* d_list, int32_t* d_count, hipStream_t s);
hipError_t launch_flann_search_global(const FlannSearchArgs& a, const int32_t* d_list, int count, float* d_heap_d,
                                      int32_t* d_heap_n, hipStream_t s);
hipError_t launch_test_retain_best(float* d_resp, uint32_t* d_payload, int32_t* d_tmp, int n, int n_points, int depth,
                                   int semantics, int* d_k, hipStream_t s);
hipError_t launch_test_update_num_iters(double p, const double* d_ep, int n, int model_points, int max_iters,
                                        int32_t* d_out, hipStream_t s);
hipError_t launch_test_ransac_sample(const GeomArgs& g, hipStream_t s);
hipError_t launch_test_ransac_replay(const GeomArgs& g, hipStream_t s);
hipError_t launch_test_five_point(const double* d_q, double* d_models, int* d_n, hipStream_t s);
hipError_t launch_test_sampson(const double* d_E, const double* d_pts, int n, float t, int8_t* d_dec, uint8_t* d_ex,
                               hipStream_t s);

}  // namespace dvo
