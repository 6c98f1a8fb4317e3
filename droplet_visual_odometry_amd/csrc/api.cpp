// C-ABI of libdvo_hip.so (include/dvo.h): contexts, ORB plans, device buffers
// and the per-call entry points that replace the reference's OpenCV calls.
// Host code only sizes buffers and moves bytes; every computation runs in the
// HIP kernels of orb.hip, match.hip and geometry.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "dvo_internal.h"

using namespace dvo;

struct SiftPlanDev {  // per-size device buffers of dvo_sift_detect_and_compute
    int w = 0, h = 0;
    SiftArgs a{};
    float* taps = nullptr;
    int tap_off[6] = {0}, tap_n[6] = {0};
    uint8_t* img = nullptr;
    int pitch = 0;
    std::vector<void*> allocs;
};

struct SurfPlanDev {  // per-size device buffers of dvo_surf_detect_and_compute
    int w = 0, h = 0;
    SurfArgs a{};
    uint8_t* img = nullptr;
    std::vector<void*> allocs;
};

struct dvo_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    SiftPlanDev sift;
    SurfPlanDev surf;
    // grow-only scratch for the per-call entry points
    std::vector<std::pair<void*, size_t>> scratch;
    dvo_stream* call_stream = nullptr;  // cached plan for detectAndCompute
    int call_w = 0, call_h = 0, call_nf = 0;
    // grow-only pinned host staging of the synchronous per-call entry points
    uint8_t* pin = nullptr;
    size_t pin_cap = 0;
};

struct dvo_stream {
    dvo_ctx* ctx = nullptr;
    dvo_stream_config cfg{};
    Plan plan{};
    Buffers buf{};
    std::vector<void*> allocs;
    uint8_t* d_frames = nullptr;  // per-call upload slab (max_frames images)
    double* d_carry = nullptr;    // pose tail carry: P_prev (12) | T_abs_prev (16)
    hipEvent_t carry_ev = nullptr;  // recorded after every pose tail on this carry
    bool carry_ev_valid = false;
    dvo_stream* carry_owner = nullptr;  // stream whose carry this one uses (itself by default)
    bool own_hs = false;
    int last_nframes = 0;
    int last_pairs = 0;           // pairs of that call (n - 1 for a stream, n / 2 for independent pairs)
    bool last_has_pairs = false;  // the last call ran match + geometry
    const dvo_pair_record* last_rec = nullptr;  // the caller's records of that call (read by the pose tail)
    const uint8_t* last_frames = nullptr;       // the frames of that call (get_pyramid recomputes blurred levels)
    int64_t last_fstride = 0;
    int last_pitch = 0;
    hipStream_t hs = nullptr;
    // dvo_stream_pair: the last pair's current-frame features (the next pair's previous frame) and
    // the device record of one pair, allocated by the first call
    dvo_keypoint* fc_kps = nullptr;
    uint8_t* fc_desc = nullptr;
    int32_t* fc_n = nullptr;  // nkp, status
    dvo_pair_record* pair_rec = nullptr;
    bool fc_valid = false;
    bool last_reuse = false;  // the last call was dvo_stream_pair(reuse_prev): pyramid slot 0 holds frame 1
    // Pair sets (dvo_stream_submit): set k holds one batch's pairs from its submit until it
    // retires kRansacRounds - 1 submits later (or at a drain); every submit / drain step runs one
    // merged RANSAC round in which each occupied set takes its next round.
    struct PairSet {
        bool used = false;
        int round = 0;  // the round this set runs next
        int pairs = 0;
        dvo_pair_record* rec = nullptr;  // the caller's records of the batch
    };
    PairSet sets[kMaxSets];
    int nsets = 0;  // pair sets allocated: 1 until the first submit, then kRansacRounds (alloc_sets)
    std::vector<void*> set_allocs;  // their buffers (also in allocs)
    int next_set = 0;  // the set the next submit fills (sets are taken in ring order)
    int last_set = 0;  // the set of the last submitted batch (get_matches)
    int retired = 0;   // batches retired by the last submit / drain / process call
    int last_sub_pairs = 0;  // pairs of the last submitted batch (get_matches)
    dvo_pair_record* retired_rec[kMaxSets] = {};
    int retired_pairs[kMaxSets] = {};
    // profiling: event tables per in-flight call, accumulated on query
    bool profiling = false;
    std::vector<std::vector<hipEvent_t>> ev_pending;
    std::vector<int> ev_groups;  // per pending table: detection frame groups (orb_groups), 0 = none
    std::vector<std::vector<hipEvent_t>> ev_free;
    double stage_ms[DVO_NSTAGES] = {0};
    int prof_calls = 0;
};

namespace {

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            if (ctx) ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);       \
            return DVO_EHIP;                                                             \
        }                                                                                \
    } while (0)

int fail(dvo_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int cv_round_f(float v) { return (int)lrintf(v); }

// orb.cpp computeKeyPoints: features per level (float arithmetic as OpenCV).
void features_per_level(int nfeatures, int nlevels, int* out) {
    const double sf = (double)1.2f;
    float factor = (float)(1.0 / sf);
    float ndesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        out[l] = cv_round_f(ndesired);
        sum += out[l];
        ndesired *= factor;
    }
    out[nlevels - 1] = std::max(nfeatures - sum, 0);
}

// OpenCV 3.2 resize(INTER_LINEAR) on x86: VResizeLinearVec_32s8u (SSE2) covers
// the columns before the point where its 16-wide loop (x <= W - 16) and then
// its 4-wide loop (x < W - 4) stop; VResizeLinear's scalar loop does the rest.
int ocv32_simd_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {
    }
    for (; x < width - 4; x += 4) {
    }
    return x;
}

Plan make_plan(int w, int h, int nfeatures, int fast_threshold, int semantics) {
    Plan p{};
    p.semantics = semantics;
    p.w = w;
    p.h = h;
    p.nlevels = kMaxLevels;
    p.nfeatures = nfeatures;
    p.fast_threshold = fast_threshold;
    int nper[kMaxLevels];
    features_per_level(nfeatures, kMaxLevels, nper);
    int64_t pyr = 0, blur = 0, bcand = 0, cand = 0;
    int bands = 0, strips = 0, tiles = 0, coef = 0, coef32 = 0;
    for (int l = 0; l < kMaxLevels; ++l) {
        LevelGeom& G = p.L[l];
        G.scale = (float)std::pow((double)1.2f, (double)l);  // getScale
        float inv = 1.0f / G.scale;
        G.w = l == 0 ? w : cv_round_f(w * inv);
        G.h = l == 0 ? h : cv_round_f(h * inv);
        G.nper = nper[l];
        G.pitch = (G.w + 15) & ~15;
        G.bpitch = G.pitch;
        G.pyr_off = l == 0 ? 0 : pyr;
        if (l > 0) pyr += (int64_t)G.pitch * G.h;
        G.blur_off = blur;
        blur += (int64_t)G.bpitch * G.h;
        // x table padded to a multiple of 4 entries at a 16-byte aligned offset (one int4 per 4 columns)
        G.xcoef_off = l == 0 ? 0 : coef;
        G.ycoef_off = l == 0 ? 0 : coef + ((G.w + 3) & ~3);
        if (l > 0) coef += ((G.w + 3) & ~3) + ((G.h + 7) & ~7);  // y table padded to 8 rows (resize_level_lds_kernel)
        G.l32_x = l == 0 ? 0 : coef32;
        G.l32_y = l == 0 ? 0 : coef32 + 4 * G.w;
        if (l > 0) coef32 += 4 * (G.w + G.h);
        G.l32_xs = ocv32_simd_end(G.w);
        const bool usable = G.w > 2 * kBorder && G.h > 2 * kBorder;
        const int rows = usable ? G.h - 2 * kBorder : 0;
        const int wc = usable ? G.w - 2 * kBorder : 0;
        G.nbands = (rows + kBandRows - 1) / kBandRows;
        G.ntx = (wc + kFastTW - 1) / kFastTW;
        G.band_base = bands;
        bands += G.nbands * G.ntx;
        G.strip_base = strips;
        strips += G.nbands > 0 ? G.ntx : 0;
        G.band_cap = (kBandRows / 2) * (kFastTW / 2) + 4;  // strict NMS: <= 1 keep per 2x2
        G.band_cand_off = bcand;
        bcand += (int64_t)G.nbands * G.ntx * G.band_cap;
        G.cand_cap = (kBandRows / 2) * G.nbands * ((wc + 1) / 2) + 4;
        G.cand_off = cand;
        cand += G.cand_cap;
        G.tiles_x = (G.w + kBlurTW - 1) / kBlurTW;
        G.tiles_y = (G.h + kBlurTH - 1) / kBlurTH;
        G.tile_base = tiles;
        tiles += G.tiles_x * G.tiles_y;
    }
    p.pyr_stride = (pyr + 255) & ~(int64_t)255;
    p.blur_stride = (blur + 255) & ~(int64_t)255;
    p.total_bands = bands;
    p.total_strips = strips;
    p.band_cand_stride = (bcand + 63) & ~(int64_t)63;
    p.cand_stride = (cand + 63) & ~(int64_t)63;
    p.total_tiles = tiles;
    p.coef_total = coef;
    p.coef32_total = coef32;
    p.kp_cap = ((nfeatures + 256) + 63) & ~63;
    return p;
}

// resize.cpp INTER_LINEAR_EXACT coefficient of destination index `val` (double
// arithmetic as OpenCV's softdouble path; host and device agree bit for bit
// because both are IEEE double without contraction).  Clamped positions store
// the clamped source index with weight c1 = 0, so the kernel never branches on
// the mode: (h0 * 256 + h1 * 0 + 2^15) >> 16 == (h0 + 128) >> 8.
int lin_coef_packed(int val, int srcsize, int dstsize) {
    const double inv_scale = (double)dstsize / srcsize;
    const double scale = 1.0 / inv_scale;
    const double fval = scale * ((double)val + 0.5) - 0.5;
    const int ival = (int)std::floor(fval);
    if (ival >= 0 && srcsize > 1) {
        if (ival < srcsize - 1) {
            const int c1 = (int)std::nearbyint((fval - (double)ival) * 256.0);
            return ival | (c1 << 13);
        }
        return (srcsize - 1) | (2 << 22);
    }
    return 1 << 22;
}

std::vector<int32_t> resize_coefs(const Plan& p) {
    std::vector<int32_t> c(std::max(p.coef_total, 1));
    for (int l = 1; l < p.nlevels; ++l) {
        const LevelGeom &S = p.L[l - 1], &D = p.L[l];
        for (int x = 0; x < ((D.w + 3) & ~3); ++x) c[D.xcoef_off + x] = lin_coef_packed(std::min(x, D.w - 1), S.w, D.w);
        for (int y = 0; y < ((D.h + 7) & ~7); ++y) c[D.ycoef_off + y] = lin_coef_packed(std::min(y, D.h - 1), S.h, D.h);
    }
    return c;
}

// OpenCV 3.2 resize(INTER_LINEAR) tables (imgwarp.cpp resize; oracle/orb.cpp
// resize_linear_32): fx = (float)((d + 0.5) * scale - 0.5) in double rounded to
// float, sx = cvFloor(fx), weights saturate_cast<short>(w * 2048.f) each
// rounded half to even.  Columns: {sx, sx + 1, a0 | a1 << 16, 0}, the
// positions past xmax {W-1, W-1, 2048, 0}; rows: {clip(sy), clip(sy + 1),
// b0 | b1 << 16, 0}.
std::vector<int32_t> resize_coefs_32(const Plan& p) {
    std::vector<int32_t> c(std::max(p.coef32_total, 4));
    auto wgt = [](float v) { return (int32_t)std::max(-32768, std::min(32767, cv_round_f(v))); };
    for (int l = 1; l < p.nlevels; ++l) {
        const LevelGeom &S = p.L[l - 1], &D = p.L[l];
        const double sx_scale = 1. / ((double)D.w / S.w), sy_scale = 1. / ((double)D.h / S.h);
        int xmax = D.w;
        for (int dx = 0; dx < D.w; ++dx) {
            float fx = (float)((dx + 0.5) * sx_scale - 0.5);
            int sx = (int)std::floor(fx);
            fx -= (float)sx;
            if (sx < 0) fx = 0, sx = 0;
            if (sx + 1 >= S.w) {
                xmax = std::min(xmax, dx);
                if (sx >= S.w - 1) fx = 0, sx = S.w - 1;
            }
            int32_t* e = &c[D.l32_x + 4 * dx];
            if (dx < xmax) {
                e[0] = sx;
                e[1] = sx + 1;
                e[2] = (wgt((1.f - fx) * 2048) & 0xFFFF) | (wgt(fx * 2048) << 16);
            } else {
                e[0] = e[1] = sx;
                e[2] = 2048;
            }
            e[3] = 0;
        }
        auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
        for (int dy = 0; dy < D.h; ++dy) {
            float fy = (float)((dy + 0.5) * sy_scale - 0.5);
            const int sy = (int)std::floor(fy);
            fy -= (float)sy;
            int32_t* e = &c[D.l32_y + 4 * dy];
            e[0] = clip(sy, 0, S.h);
            e[1] = clip(sy + 1, 0, S.h);
            e[2] = (wgt((1.f - fy) * 2048) & 0xFFFF) | (wgt(fy * 2048) << 16);
            e[3] = 0;
        }
    }
    return c;
}

int check_orb_params(dvo_ctx* ctx, const dvo_orb_params* o) {
    if (!o) return fail(ctx, DVO_EINVAL, "null ORB parameters");
    if (o->nfeatures <= 0 || o->nfeatures > 7680) return fail(ctx, DVO_EINVAL, "nfeatures out of range (1..7680)");
    if (o->scale_factor != 1.2f || o->nlevels != 8 || o->edge_threshold != 31 || o->first_level != 0 || o->wta_k != 2 ||
        o->score_type != 0 || o->patch_size != 31)
        return fail(ctx, DVO_EINVAL,
                    "only cv.ORB_create() defaults (scaleFactor 1.2, nlevels 8, edgeThreshold 31, firstLevel 0, "
                    "WTA_K 2, HARRIS_SCORE, patchSize 31) are implemented");
    if (o->fast_threshold < 0 || o->fast_threshold > 255) return fail(ctx, DVO_EINVAL, "fastThreshold out of range");
    if (o->opencv_semantics != DVO_OPENCV_4X && o->opencv_semantics != DVO_OPENCV_32)
        return fail(ctx, DVO_EINVAL, "opencv_semantics must be DVO_OPENCV_4X or DVO_OPENCV_32");
    return DVO_OK;
}

template <class T>
int dalloc(dvo_stream* s, T** p, size_t n) {
    dvo_ctx* ctx = s->ctx;
    void* q = nullptr;
    HIP_TRY(hipMalloc(&q, n * sizeof(T) + 256));
    s->allocs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return DVO_OK;
}

// grow-only per-context scratch slot
// One synchronous per-call operation's host traffic through pinned memory: inputs are
// packed into the staging area and sent with asynchronous copies on the call's
// stream, outputs come back the same way, and the caller synchronises once (a
// pageable hipMemcpy is a blocking staged copy each: ~10-20 us apiece).
struct Staging {
    uint8_t* base = nullptr;
    size_t off = 0, cap = 0;
    hipStream_t s = nullptr;
    static size_t round(size_t n) { return (n + 63) & ~(size_t)63; }
    uint8_t* take(size_t n) {  // the next n staged bytes (64-byte aligned)
        uint8_t* h = base + off;
        off += round(n);
        if (off > cap) {  // a caller sized its staging() request wrong: never write past the area
            std::fprintf(stderr, "dvo: staging overflow (%zu > %zu)\n", off, cap);
            std::abort();
        }
        return h;
    }
    hipError_t send(void* dev, const uint8_t* h, size_t n) {  // host -> device of staged bytes
        return n ? hipMemcpyAsync(dev, h, n, hipMemcpyHostToDevice, s) : hipSuccess;
    }
    hipError_t put(void* dev, const void* src, size_t n) {
        uint8_t* h = take(n);
        if (n) std::memcpy(h, src, n);
        return send(dev, h, n);
    }
    hipError_t get(const void* dev, size_t n, uint8_t** h) {  // device -> host, valid after synchronising
        *h = take(n);
        return n ? hipMemcpyAsync(*h, dev, n, hipMemcpyDeviceToHost, s) : hipSuccess;
    }
};

static int staging(dvo_ctx* ctx, size_t bytes, hipStream_t s, Staging* st) {
    if (ctx->pin_cap < bytes) {
        if (ctx->pin) HIP_TRY(hipHostFree(ctx->pin));
        ctx->pin = nullptr;
        ctx->pin_cap = 0;
        const size_t nb = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
        HIP_TRY(hipHostMalloc((void**)&ctx->pin, nb, hipHostMallocDefault));
        ctx->pin_cap = nb;
    }
    st->base = ctx->pin;
    st->off = 0;
    st->cap = ctx->pin_cap;
    st->s = s;
    return DVO_OK;
}

int scratch(dvo_ctx* ctx, int slot, size_t bytes, void** out) {
    if ((int)ctx->scratch.size() <= slot) ctx->scratch.resize(slot + 1, {nullptr, 0});
    auto& e = ctx->scratch[slot];
    if (e.second < bytes) {
        if (e.first) HIP_TRY(hipFree(e.first));
        e.first = nullptr;
        e.second = 0;
        size_t nb = bytes < 4096 ? 4096 : bytes + bytes / 4;
        HIP_TRY(hipMalloc(&e.first, nb));
        e.second = nb;
    }
    *out = e.first;
    return DVO_OK;
}

StreamParams params_of(dvo_stream* s, const uint8_t* frames, int nframes, int64_t frame_stride, int pitch) {
    StreamParams P{};
    P.plan = s->plan;
    P.buf = s->buf;
    P.frames = frames;
    P.frame_stride = frame_stride;
    P.in_pitch = pitch;
    P.nframes = nframes;
    P.pair_step = 1;
    return P;
}

GeomArgs stream_geom(dvo_stream* s) {
    GeomArgs g{};
    const dvo_stream_config& c = s->cfg;
    g.pts_f = s->buf.pts;
    g.m_arr = s->buf.nmatch;
    g.pts_stride = s->plan.kp_cap;
    g.fx = c.K[0];
    g.fy = c.K[4];
    g.cx = c.K[2];
    g.cy = c.K[5];
    g.prob = c.prob;
    g.threshold = c.threshold;
    g.max_iters = c.max_iters;
    g.dist_thresh = c.dist_thresh;
    g.npts = s->buf.npts;
    g.models = s->buf.models;
    g.nmod = s->buf.nmod;
    g.cnt = s->buf.rcnt;
    g.subsets = s->buf.subsets;
    g.rs = s->buf.rs;
    g.fprec = s->buf.fprec;
    g.dk_off = s->buf.dk_off;
    g.a_off = s->buf.a_off;
    g.s_off = s->buf.s_off;
    g.dk_ctl = s->buf.dk_ctl;
    g.hyp_cap = c.max_iters > 1 ? c.max_iters : 1;
    g.dk_list = s->buf.dk_list;
    g.dk_list_cap = std::max<int64_t>(round_items_bound(s->cfg.max_frames, g.hyp_cap), g.hyp_cap);
    g.E = s->buf.E;
    g.info = s->buf.info;
    g.Rt = s->buf.Rt;
    g.good = s->buf.good;
    g.pose_P = s->buf.pose_P;
    g.pose_cnt = s->buf.pose_cnt;
    return g;
}

// Set k's view of the per-pair geometry arrays (pairs [k F, (k + 1) F) of the stream's sets).
GeomArgs geom_set(const GeomArgs& g, int k, int F, int64_t hc) {
    GeomArgs o = g;
    const int64_t p0 = (int64_t)k * F;
    o.pts_f = g.pts_f + p0 * g.pts_stride * 4;
    o.m_arr = g.m_arr + p0;
    o.npts = g.npts + p0 * g.pts_stride * 4;
    o.models = g.models + p0 * hc * 90;
    o.nmod = g.nmod + p0 * hc;
    o.cnt = g.cnt + p0 * hc * 10;
    o.subsets = g.subsets + p0 * hc * 5;
    o.rs = g.rs + p0;
    o.E = g.E + p0 * 90;
    o.info = g.info + p0 * 4;
    o.Rt = g.Rt + p0 * 12;
    o.good = g.good + p0;
    o.pose_P = g.pose_P + p0 * 72;
    o.pose_cnt = g.pose_cnt + p0 * 5;
    return o;
}

// Row pitch of the internal frame slab (word-aligned rows for the byte kernels).
int frame_pitch(const dvo_stream* s) { return (s->cfg.width + 15) & ~15; }

// The per-pair geometry, one copy per pair set.  A stream starts with one set: the
// drained calls (dvo_stream_process, _process_pairs, _pair) run a batch's rounds back to back
// in it.  The first dvo_stream_submit / _submit_pairs grows it to kRansacRounds sets (the
// pipeline depth); no set is occupied then, since every drained call retires what it started.
// At 1280x720, N 2000, maxIters 1000 a set costs about 0.9 MB per pair (models 720 KB of it).
int alloc_sets(dvo_stream* s, int nsets) {
    dvo_ctx* ctx = s->ctx;
    Buffers& b = s->buf;
    if (!s->set_allocs.empty()) {
        HIP_TRY(hipStreamSynchronize(s->hs));
        for (void* q : s->set_allocs) {
            hipFree(q);
            s->allocs.erase(std::find(s->allocs.begin(), s->allocs.end(), q));
        }
        s->set_allocs.clear();
    }
    const size_t first = s->allocs.size();
    const size_t SF = (size_t)nsets * s->cfg.max_frames;
    const int cap = s->plan.kp_cap;
    const size_t hc = (size_t)(s->cfg.max_iters > 1 ? s->cfg.max_iters : 1);
    int rc = DVO_OK;
    auto take = [&](auto*& ptr, size_t n) {
        if (!rc) rc = dalloc(s, &ptr, n);
    };
    take(b.nmatch, SF);
    take(b.pts, SF * cap * 4);
    take(b.npts, SF * cap * 4);
    take(b.models, SF * hc * 90);
    take(b.nmod, SF * hc);
    take(b.rcnt, SF * hc * 10);
    take(b.subsets, SF * hc * 5);
    take(b.rs, SF);
    take(b.hdr, SF);
    take(b.dk_off, SF + 1);
    take(b.a_off, SF + 1);
    take(b.s_off, SF + 1);
    take(b.E, SF * 90);
    take(b.info, SF * 4);
    take(b.Rt, SF * 12);
    take(b.good, SF);
    take(b.pose_P, SF * 72);
    take(b.pose_cnt, SF * 5);
    s->set_allocs.assign(s->allocs.begin() + first, s->allocs.end());
    s->nsets = rc ? 0 : nsets;
    return rc;
}

int stream_alloc(dvo_stream* s) {
    const int F = s->cfg.max_frames;
    const Plan& p = s->plan;
    Buffers& b = s->buf;
    const int cap = p.kp_cap;
    int rc;
#define A(ptr, n)                              \
    if ((rc = dalloc(s, &(ptr), (size_t)(n)))) \
        return rc;
    A(b.pyr, (size_t)F * p.pyr_stride);
    A(b.blur, (size_t)F * p.blur_stride);
    A(b.coef, (size_t)std::max(p.coef_total, 1));
    A(b.coef32, (size_t)std::max(p.coef32_total, 4));
    A(b.band_cnt, (size_t)F * (p.total_bands + 1) * kBandRows);
    A(b.band_cand, (size_t)F * p.band_cand_stride);
    A(b.cand, (size_t)F * p.cand_stride);
    A(b.resp, (size_t)F * p.cand_stride);
    A(b.sel_tmp, (size_t)F * 2 * p.cand_stride);
    A(b.cnt1, (size_t)F * kMaxLevels);
    A(b.cnt2, (size_t)F * kMaxLevels);
    A(b.kps, (size_t)F * cap);
    A(b.desc, (size_t)F * cap * 32);
    A(b.nkp, (size_t)F);
    A(b.nn, (size_t)2 * F * cap);
    A(b.mq, (size_t)F * cap);
    A(b.mt, (size_t)F * cap);
    A(b.md, (size_t)F * cap);
    const size_t hc = (size_t)(s->cfg.max_iters > 1 ? s->cfg.max_iters : 1);
    if ((rc = alloc_sets(s, 1))) return rc;
    // five-point records and parked Durand-Kerner lists of one merged round (a bound over any
    // number of sets: one set at each round)
    A(b.fprec, (size_t)std::max<int64_t>(round_blocks_bound(F, (int)hc), (int64_t)(hc + 63) / 64) * 128 * 64);
    A(b.dk_ctl, (size_t)2 + kDkMaxPasses);
    A(b.dk_list, (size_t)(kDkMaxPasses - 1) * std::max<int64_t>(round_items_bound(F, (int)hc), (int64_t)hc));
    A(b.status, (size_t)F);
    A(s->d_frames, (size_t)F * frame_pitch(s) * s->cfg.height);
    A(s->d_carry, (size_t)28);
#undef A
    return DVO_OK;
}

dvo_orb_params default_orb(int nfeatures) {
    dvo_orb_params o{};
    o.nfeatures = nfeatures;
    o.scale_factor = 1.2f;
    o.nlevels = 8;
    o.edge_threshold = 31;
    o.first_level = 0;
    o.wta_k = 2;
    o.score_type = 0;
    o.patch_size = 31;
    o.fast_threshold = 20;
    return o;
}

// A table: 2 events per stage, then 2 x 5 per detection frame group (launch_orb's group_ev).
int acquire_events(dvo_stream* s, int groups, hipEvent_t** ev) {
    dvo_ctx* ctx = s->ctx;
    std::vector<hipEvent_t> e;
    if (!s->ev_free.empty()) {
        e = std::move(s->ev_free.back());
        s->ev_free.pop_back();
    } else {
        e.resize(2 * DVO_NSTAGES + 10 * orb_groups(s->cfg.max_frames));
        for (auto& x : e) HIP_TRY(hipEventCreate(&x));
    }
    s->ev_pending.push_back(std::move(e));
    s->ev_groups.push_back(groups);
    *ev = s->ev_pending.back().data();
    return DVO_OK;
}

// Drain completed event tables into the per-stage totals (blocks on the last).
int collect_events(dvo_stream* s) {
    dvo_ctx* ctx = s->ctx;
    for (size_t i = 0; i < s->ev_pending.size(); ++i) {
        auto& e = s->ev_pending[i];
        const int groups = s->ev_groups[i];
        HIP_TRY(hipEventSynchronize(e[2 * DVO_NSTAGES - 1]));
        for (int st = 0; st < DVO_NSTAGES; ++st) {
            float ms = 0;
            if (st <= 4 && groups > 0) {  // detection in frame groups: the stage's time summed over them
                for (int g = 0; g < groups; ++g)
                    if (hipEventElapsedTime(&ms, e[2 * DVO_NSTAGES + 10 * g + 2 * st],
                                            e[2 * DVO_NSTAGES + 10 * g + 2 * st + 1]) == hipSuccess)
                        s->stage_ms[st] += ms;
            } else if (hipEventElapsedTime(&ms, e[2 * st], e[2 * st + 1]) == hipSuccess) {
                s->stage_ms[st] += ms;
            }
        }
        s->prof_calls++;
        s->ev_free.push_back(std::move(e));
    }
    s->ev_pending.clear();
    s->ev_groups.clear();
    return DVO_OK;
}

// One merged RANSAC round: every occupied set that has rounds left takes its next one.
int merged_round(dvo_stream* s) {
    dvo_ctx* ctx = s->ctx;
    RoundSpec sp{};
    sp.nsets = s->nsets;
    sp.F = s->cfg.max_frames;
    bool any = false;
    for (int r = 0; r < kRansacRounds; ++r) sp.bound[r] = kRansacBounds[r];  // indexed by round
    for (int k = 0; k < s->nsets; ++k) {
        auto& st = s->sets[k];
        const bool run = st.used && st.round < kRansacRounds;
        sp.round[k] = run ? st.round : -1;
        sp.npairs[k] = run ? st.pairs : 0;
        any |= run;
    }
    if (!any) return DVO_OK;
    HIP_TRY(launch_ransac_round(stream_geom(s), sp, s->hs));
    for (auto& st : s->sets)
        if (st.used && st.round < kRansacRounds) ++st.round;
    return DVO_OK;
}

// Retire the sets whose last round has run, oldest first: E, recoverPose, the records.
int retire_sets(dvo_stream* s) {
    dvo_ctx* ctx = s->ctx;
    const int F = s->cfg.max_frames;
    const GeomArgs g = stream_geom(s);
    // ring order from the oldest set (the one after the newest)
    for (int j = 1; j <= kRansacRounds; ++j) {
        const int k = (s->last_set + j) % kRansacRounds;
        auto& st = s->sets[k];
        if (!st.used || st.round < kRansacRounds) continue;
        HIP_TRY(launch_retire(geom_set(g, k, F, g.hyp_cap), st.pairs, s->buf.hdr + (size_t)k * F, st.rec, s->hs));
        s->retired_rec[s->retired] = st.rec;
        s->retired_pairs[s->retired] = st.pairs;
        ++s->retired;
        s->last_rec = st.rec;
        s->last_pairs = st.pairs;
        s->last_has_pairs = true;
        st = dvo_stream::PairSet{};
    }
    return DVO_OK;
}

bool sets_pending(const dvo_stream* s) {
    for (const auto& st : s->sets)
        if (st.used) return true;
    return false;
}

// Detection of n frames, then (unless detect_only) matching of their pairs into the next pair
// set and one merged RANSAC round; drain: rounds until every set is done, then retire them all
// (dvo_stream_process: this batch's records are complete when the call's work is).
int run_stream(dvo_stream* s, const uint8_t* d_frames, int n, int64_t fstride, int pitch, dvo_pair_record* d_rec,
               bool detect_only, int pair_step = 1, bool drain = true) {
    dvo_ctx* ctx = s->ctx;
    if (!detect_only && !drain && s->nsets < kRansacRounds) {  // the first pipelined submit: grow the sets
        // (before params_of: the parameter block carries the buffer pointers)
        if (sets_pending(s)) return fail(ctx, DVO_EINVAL, "pair sets occupied at the first submit");
        int rc = alloc_sets(s, kRansacRounds);
        if (rc) return rc;
        s->next_set = 0;
    }
    StreamParams P = params_of(s, d_frames, n, fstride, pitch);
    P.pair_step = pair_step;
    const int pairs = detect_only ? 0 : stream_pairs(P);
    hipEvent_t* ev = nullptr;
    const int groups = orb_groups(n);
    if (s->profiling && pairs >= 1) {
        int rc = acquire_events(s, groups, &ev);
        if (rc) return rc;
    }
    s->retired = 0;
    s->last_has_pairs = false;  // set again when a batch retires: the pose tail reads its records
    const int F = s->cfg.max_frames;
    const int k = s->next_set;
    if (pairs >= 1 && s->sets[k].used) {  // the ring is full (cannot happen in lockstep): finish its oldest
        int rc;
        while (s->sets[k].used && s->sets[k].round < kRansacRounds)
            if ((rc = merged_round(s))) return rc;
        if ((rc = retire_sets(s))) return rc;
    }
    HIP_TRY(hipMemsetAsync(s->buf.status, 0, sizeof(int32_t) * n, s->hs));
    HIP_TRY(launch_orb(P, s->hs, ev, ev && groups ? ev + 2 * DVO_NSTAGES : nullptr));
    s->last_nframes = n;
    s->last_reuse = false;
    s->last_frames = d_frames;
    s->last_fstride = fstride;
    s->last_pitch = pitch;
    s->last_sub_pairs = pairs;
    if (detect_only) return DVO_OK;
    if (pairs >= 1) {
        // match into set k (its KeyPoint_convert points and counts), the frame-side record values
        StreamParams Pk = P;
        Pk.buf.pts += (size_t)k * F * s->plan.kp_cap * 4;
        Pk.buf.nmatch += (size_t)k * F;
        HIP_TRY(launch_match(Pk, s->cfg.cross_check, s->hs, ev));
        HIP_TRY(launch_pair_header(P, s->buf.hdr + (size_t)k * F, s->hs));
        const GeomArgs g = stream_geom(s);
        HIP_TRY(launch_geometry_args(geom_set(g, k, F, g.hyp_cap), pairs, kStageNormalize, s->hs));
        s->sets[k] = dvo_stream::PairSet{true, 0, pairs, d_rec};
        s->last_set = k;
        s->next_set = (k + 1) % s->nsets;
    }
    if (pairs < 1 && !drain) return DVO_OK;
    int rc;
    mark(ev, 6, 0, s->hs);
    if ((rc = merged_round(s))) return rc;
    if (drain)
        while (sets_pending(s)) {
            bool left = false;
            for (const auto& st : s->sets) left |= st.used && st.round < kRansacRounds;
            if (!left) break;
            if ((rc = merged_round(s))) return rc;
        }
    mark(ev, 6, 1, s->hs);
    mark(ev, 7, 0, s->hs);
    if ((rc = retire_sets(s))) return rc;
    mark(ev, 7, 1, s->hs);
    mark(ev, 8, 0, s->hs);  // pose-tail pair defaults to 0 ms; dvo_stream_pose_tail re-records it
    mark(ev, 8, 1, s->hs);
    return DVO_OK;
}

}  // namespace

extern "C" {

int dvo_version(void) { return 1; }

#ifndef DVO_BUILD_ID
#define DVO_BUILD_ID "unstamped0000000"
#endif
// "DVO_BUILD_ID=" + 16 hex digits: build.py finds it in the file without loading it
static const char kBuildTag[] = "DVO_BUILD_ID=" DVO_BUILD_ID;
const char* dvo_build_id(void) { return kBuildTag + 13; }

int dvo_ctx_create(dvo_ctx** out, int device) {
    if (!out) return DVO_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DVO_EHIP;
    if (device < 0 || device >= n) return DVO_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return DVO_EHIP;
    dvo_ctx* ctx = new dvo_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return DVO_EHIP;
    }
    *out = ctx;
    return DVO_OK;
}

void dvo_ctx_destroy(dvo_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    for (void* p : ctx->sift.allocs) hipFree(p);
    for (void* p : ctx->surf.allocs) hipFree(p);
    if (ctx->call_stream) dvo_stream_destroy(ctx->call_stream);
    for (auto& e : ctx->scratch)
        if (e.first) hipFree(e.first);
    if (ctx->pin) hipHostFree(ctx->pin);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* dvo_last_error(const dvo_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dvo_stream_create(dvo_ctx* ctx, const dvo_stream_config* cfg, dvo_stream** out) {
    if (!ctx || !cfg || !out) return fail(ctx, DVO_EINVAL, "null argument");
    *out = nullptr;
    int rc = check_orb_params(ctx, &cfg->orb);
    if (rc) return rc;
    if (cfg->width < 8 || cfg->height < 8 || cfg->width >= kMaxW || cfg->height >= kMaxW)
        return fail(ctx, DVO_EINVAL, "frame size out of range (8..4095)");
    if (cfg->max_frames < 1) return fail(ctx, DVO_EINVAL, "max_frames < 1");
    if (cfg->cross_check < 0 || cfg->cross_check > 2) return fail(ctx, DVO_EINVAL, "cross_check must be 0, 1 or 2");
    HIP_TRY(hipSetDevice(ctx->device));
    auto s = std::make_unique<dvo_stream>();
    s->ctx = ctx;
    s->cfg = *cfg;
    s->plan = make_plan(cfg->width, cfg->height, cfg->orb.nfeatures, cfg->orb.fast_threshold, cfg->orb.opencv_semantics);
    if (s->plan.kp_cap > 65535) return fail(ctx, DVO_EINVAL, "too many features");
    if (hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) != hipSuccess)
        return fail(ctx, DVO_EHIP, "hipStreamCreate failed");
    s->own_hs = true;
    s->carry_owner = s.get();
    if (hipEventCreateWithFlags(&s->carry_ev, hipEventDisableTiming) != hipSuccess) {
        hipStreamDestroy(s->hs);
        return fail(ctx, DVO_EHIP, "hipEventCreate failed");
    }
    rc = stream_alloc(s.get());
    if (!rc) {
        const std::vector<int32_t> coefs = resize_coefs(s->plan), coefs32 = resize_coefs_32(s->plan);
        if (hipMemcpy(s->buf.coef, coefs.data(), coefs.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(s->buf.coef32, coefs32.data(), coefs32.size() * sizeof(int32_t), hipMemcpyHostToDevice) !=
                hipSuccess)
            rc = fail(ctx, DVO_EHIP, "coefficient upload failed");
    }
    if (rc) {
        for (void* p : s->allocs) hipFree(p);
        hipEventDestroy(s->carry_ev);
        hipStreamDestroy(s->hs);
        return rc;
    }
    *out = s.release();
    return DVO_OK;
}

void dvo_stream_destroy(dvo_stream* s) {
    if (!s) return;
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->hs);
    for (void* p : s->allocs) hipFree(p);
    for (auto* pool : {&s->ev_pending, &s->ev_free})
        for (auto& e : *pool)
            for (auto x : e) hipEventDestroy(x);
    hipEventDestroy(s->carry_ev);
    if (s->own_hs) hipStreamDestroy(s->hs);
    delete s;
}

int dvo_stream_reset_pose(dvo_stream* s, const double* P0, const double* T0) {
    if (!s || !P0 || !T0) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    dvo_stream* o = s->carry_owner;
    double c[28];
    std::memcpy(c, P0, 12 * sizeof(double));
    std::memcpy(c + 12, T0, 16 * sizeof(double));
    if (o->carry_ev_valid) HIP_TRY(hipStreamWaitEvent(s->hs, o->carry_ev, 0));
    HIP_TRY(hipMemcpyAsync(o->d_carry, c, sizeof(c), hipMemcpyHostToDevice, s->hs));
    HIP_TRY(hipEventRecord(o->carry_ev, s->hs));
    o->carry_ev_valid = true;
    HIP_TRY(hipStreamSynchronize(s->hs));
    return DVO_OK;
}

int dvo_stream_share_pose(dvo_stream* s, dvo_stream* owner) {
    if (!s || !owner || owner->carry_owner != owner) return DVO_EINVAL;
    s->carry_owner = owner;
    return DVO_OK;
}

int dvo_stream_pose_tail(dvo_stream* s, const double* d_corners_prev, const double* d_corners_cur, int k,
                         double marker_length, double* d_T_rel, double* d_T_abs) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (!s->last_has_pairs) return fail(ctx, DVO_EINVAL, "pose tail needs a preceding dvo_stream_process");
    return dvo_stream_pose_tail_batch(s, s->last_rec, s->last_pairs, d_corners_prev, d_corners_cur, k, marker_length,
                                      d_T_rel, d_T_abs);
}

int dvo_stream_pose_tail_batch(dvo_stream* s, const dvo_pair_record* d_records, int pairs, const double* d_corners_prev,
                               const double* d_corners_cur, int k, double marker_length, double* d_T_rel,
                               double* d_T_abs) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (k < 2 || !d_corners_prev || !d_corners_cur || !d_T_rel || !d_T_abs)
        return fail(ctx, DVO_EINVAL, "pose tail needs >= 2 corners per frame and output buffers");
    if (!d_records || pairs < 1) return fail(ctx, DVO_EINVAL, "pose tail needs records");
    HIP_TRY(hipSetDevice(ctx->device));
    hipEvent_t* ev = (s->profiling && !s->ev_pending.empty()) ? s->ev_pending.back().data() : nullptr;
    dvo_stream* o = s->carry_owner;  // pose tails on one carry run in call order, across streams
    if (o->carry_ev_valid) HIP_TRY(hipStreamWaitEvent(s->hs, o->carry_ev, 0));
    mark(ev, 8, 0, s->hs);
    HIP_TRY(launch_pose_tail(d_records, pairs, s->cfg.K, d_corners_prev, d_corners_cur, k, marker_length,
                             o->d_carry, d_T_rel, d_T_abs, s->hs));
    mark(ev, 8, 1, s->hs);
    HIP_TRY(hipEventRecord(o->carry_ev, s->hs));
    o->carry_ev_valid = true;
    return DVO_OK;
}

int dvo_pose_tail_records(dvo_ctx* ctx, const dvo_pair_record* d_records, int pairs, const double* K,
                          const double* d_corners_prev, const double* d_corners_cur, int k, double marker_length,
                          double* d_carry, double* d_T_rel, double* d_T_abs, void* hip_stream) {
    if (!ctx) return DVO_EINVAL;
    if (pairs < 0 || !K) return fail(ctx, DVO_EINVAL, "pose tail needs pairs >= 0 and K");
    if (pairs == 0) return DVO_OK;
    if (k < 2 || !d_records || !d_corners_prev || !d_corners_cur || !d_carry || !d_T_rel || !d_T_abs)
        return fail(ctx, DVO_EINVAL, "pose tail needs records, >= 2 corners per frame, the carry and output buffers");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(launch_pose_tail(d_records, pairs, K, d_corners_prev, d_corners_cur, k, marker_length, d_carry, d_T_rel,
                             d_T_abs, hip_stream ? (hipStream_t)hip_stream : ctx->stream));
    return DVO_OK;
}

int dvo_pose_rel_range(dvo_ctx* ctx, const dvo_pair_record* d_records, int pairs, int p0, int n, const double* K,
                       const double* d_corners_prev, const double* d_corners_cur, int k, double marker_length,
                       double* d_P_carry, double* d_T_rel, void* hip_stream) {
    if (!ctx) return DVO_EINVAL;
    if (pairs < 0 || p0 < 0 || n < 0 || p0 + n > pairs || !K)
        return fail(ctx, DVO_EINVAL, "pose range needs 0 <= p0 <= p0 + n <= pairs and K");
    if (pairs == 0) return DVO_OK;
    if (!d_records || !d_P_carry || (n > 0 && (k < 2 || !d_corners_prev || !d_corners_cur || !d_T_rel)))
        return fail(ctx, DVO_EINVAL, "pose range needs records, the P carry, >= 2 corners per frame and T_rel");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(launch_pose_rel_range(d_records, pairs, p0, n, K, d_corners_prev, d_corners_cur, k, marker_length,
                                  d_P_carry, d_T_rel, hip_stream ? (hipStream_t)hip_stream : ctx->stream));
    return DVO_OK;
}

// The chain on the host, in the device kernel's arithmetic order (pose_chain_kernel: element
// (r, c) = ((t_r0 A_0c + t_r1 A_1c) + t_r2 A_2c) + t_r3 A_3c; this file is built with
// -ffp-contract=off, so each product and sum rounds as written).
int dvo_pose_chain_host(const double* T_rel, int n, double* T_carry, double* T_abs) {
    if (n < 0 || (n > 0 && (!T_rel || !T_carry || !T_abs))) return DVO_EINVAL;
    if (n == 0) return DVO_OK;  // nothing to chain; T_carry may be NULL (as dvo_pose_chain)
    double t[16];
    std::memcpy(t, T_carry, sizeof(t));
    for (int p = 0; p < n; ++p) {
        const double* A = T_rel + (size_t)p * 16;
        double u[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                const double m0 = t[r * 4 + 0] * A[0 * 4 + c], m1 = t[r * 4 + 1] * A[1 * 4 + c];
                const double m2 = t[r * 4 + 2] * A[2 * 4 + c], m3 = t[r * 4 + 3] * A[3 * 4 + c];
                u[r * 4 + c] = ((m0 + m1) + m2) + m3;
            }
        std::memcpy(t, u, sizeof(t));
        std::memcpy(T_abs + (size_t)p * 16, t, sizeof(t));
    }
    std::memcpy(T_carry, t, sizeof(t));
    return DVO_OK;
}

int dvo_pose_chain(dvo_ctx* ctx, const double* d_T_rel, int n, double* d_T_carry, double* d_T_abs, void* hip_stream) {
    if (!ctx) return DVO_EINVAL;
    if (n < 0 || (n > 0 && (!d_T_rel || !d_T_carry || !d_T_abs)))
        return fail(ctx, DVO_EINVAL, "pose chain needs T_rel, the carry and an output buffer");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(launch_pose_chain(d_T_rel, n, d_T_carry, d_T_abs,
                              hip_stream ? (hipStream_t)hip_stream : ctx->stream));
    return DVO_OK;
}

int dvo_stream_set_profiling(dvo_stream* s, int enable) {
    if (!s) return DVO_EINVAL;
    int rc = collect_events(s);
    if (rc) return rc;
    s->profiling = enable != 0;
    for (double& v : s->stage_ms) v = 0;
    s->prof_calls = 0;
    return DVO_OK;
}

int dvo_stream_stage_times(dvo_stream* s, double* ms, int* calls) {
    if (!s || !ms) return DVO_EINVAL;
    int rc = collect_events(s);
    if (rc) return rc;
    for (int i = 0; i < DVO_NSTAGES; ++i) ms[i] = s->stage_ms[i];
    if (calls) *calls = s->prof_calls;
    return DVO_OK;
}

void* dvo_stream_hip_stream(dvo_stream* s) { return s ? (void*)s->hs : nullptr; }

static int process_frames(dvo_stream* s, const uint8_t* d_frames, int n_frames, int64_t frame_stride, int stride,
                   dvo_pair_record* d_records, int pair_step, bool drain = true) {
    dvo_ctx* ctx = s->ctx;
    if (!d_frames || stride < s->cfg.width) return fail(ctx, DVO_EINVAL, "bad frame buffer");
    HIP_TRY(hipSetDevice(ctx->device));
    if (((uintptr_t)d_frames | (uintptr_t)frame_stride | (uintptr_t)stride) & 3) {
        // the byte kernels read level 0 in 4-byte words: realign into the slab
        const int pw = frame_pitch(s);
        for (int i = 0; i < n_frames; ++i)
            HIP_TRY(hipMemcpy2DAsync(s->d_frames + (size_t)i * pw * s->cfg.height, pw, d_frames + i * frame_stride,
                                     stride, s->cfg.width, s->cfg.height, hipMemcpyDeviceToDevice, s->hs));
        return run_stream(s, s->d_frames, n_frames, (int64_t)pw * s->cfg.height, pw, d_records, false, pair_step,
                          drain);
    }
    return run_stream(s, d_frames, n_frames, frame_stride, stride, d_records, false, pair_step, drain);
}

int dvo_stream_process(dvo_stream* s, const uint8_t* d_frames, int n_frames, int64_t frame_stride, int stride,
                       dvo_pair_record* d_records) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (n_frames < 1 || n_frames > s->cfg.max_frames) return fail(ctx, DVO_EINVAL, "n_frames out of range");
    if (n_frames > 1 && !d_records) return fail(ctx, DVO_EINVAL, "null records");
    return process_frames(s, d_frames, n_frames, frame_stride, stride, d_records, 1);
}

int dvo_pipeline_depth(void) { return kRansacRounds; }

int dvo_stream_submit(dvo_stream* s, const uint8_t* d_frames, int n_frames, int64_t frame_stride, int stride,
                      dvo_pair_record* d_records) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (n_frames < 2 || n_frames > s->cfg.max_frames) return fail(ctx, DVO_EINVAL, "n_frames out of range (2..max)");
    if (!d_records) return fail(ctx, DVO_EINVAL, "null records");
    return process_frames(s, d_frames, n_frames, frame_stride, stride, d_records, 1, false);
}

int dvo_stream_submit_pairs(dvo_stream* s, const uint8_t* d_frames, int n_pairs, int64_t frame_stride, int stride,
                            dvo_pair_record* d_records) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (n_pairs < 1 || 2 * (int64_t)n_pairs > s->cfg.max_frames) return fail(ctx, DVO_EINVAL, "n_pairs out of range");
    if (!d_records) return fail(ctx, DVO_EINVAL, "null records");
    return process_frames(s, d_frames, 2 * n_pairs, frame_stride, stride, d_records, 2, false);
}

int dvo_stream_drain(dvo_stream* s) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    HIP_TRY(hipSetDevice(ctx->device));
    s->retired = 0;
    s->last_has_pairs = false;
    int rc;
    for (;;) {
        bool left = false;
        for (const auto& st : s->sets) left |= st.used && st.round < kRansacRounds;
        if (!left) break;
        if ((rc = merged_round(s))) return rc;
    }
    return retire_sets(s);
}

int dvo_stream_retired(dvo_stream* s, void** records, int* pairs, int cap) {
    if (!s || (cap > 0 && (!records || !pairs))) return DVO_EINVAL;
    for (int i = 0; i < s->retired && i < cap; ++i) {
        records[i] = s->retired_rec[i];
        pairs[i] = s->retired_pairs[i];
    }
    return s->retired;
}

int dvo_stream_process_pairs(dvo_stream* s, const uint8_t* d_frames, int n_pairs, int64_t frame_stride, int stride,
                             dvo_pair_record* d_records) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (n_pairs < 1 || 2 * (int64_t)n_pairs > s->cfg.max_frames) return fail(ctx, DVO_EINVAL, "n_pairs out of range");
    if (!d_records) return fail(ctx, DVO_EINVAL, "null records");
    return process_frames(s, d_frames, 2 * n_pairs, frame_stride, stride, d_records, 2);
}

// One pair of host frames through the whole per-pair path in one synchronous call
// (dvo.h dvo_stream_pair).  Slot 0 of the stream's frame slab / feature buffers is the
// previous frame, slot 1 the current one.  With reuse_prev the current frame is detected
// alone (as frame 0, the ORB kernels' per-call launch shapes), its features are moved
// to slot 1 and the cached ones of the last call's current frame to slot 0; then the
// matcher (train stages split over workgroups: one pair alone fills the chip), the
// per-call RANSAC schedule (one round, 16-lane Durand-Kerner), recoverPose and the
// record, and one device-to-host copy of the record.
int dvo_stream_pair(dvo_stream* s, const uint8_t* prev_img, const uint8_t* cur_img, int stride, int reuse_prev,
                    dvo_pair_record* rec_out) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    const int w = s->cfg.width, h = s->cfg.height;
    if (s->cfg.max_frames < 2) return fail(ctx, DVO_EINVAL, "dvo_stream_pair needs max_frames >= 2");
    if (!cur_img || !rec_out || stride < w || (!reuse_prev && !prev_img)) return fail(ctx, DVO_EINVAL, "bad image buffer");
    if (reuse_prev && !s->fc_valid) return fail(ctx, DVO_EINVAL, "reuse_prev needs a preceding dvo_stream_pair");
    if (sets_pending(s)) return fail(ctx, DVO_EINVAL, "dvo_stream_pair: submitted batches are pending (dvo_stream_drain)");
    // the feature cache is valid only after a call that succeeds (a failing call may have left
    // its frame half-way through the rotation)
    s->fc_valid = false;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t kc = (size_t)s->plan.kp_cap;
    if (!s->pair_rec) {  // each buffer once: a partial failure leaves the rest to the next call
        int rc;
        if ((!s->fc_kps && (rc = dalloc(s, &s->fc_kps, kc))) || (!s->fc_desc && (rc = dalloc(s, &s->fc_desc, kc * 32))) ||
            (!s->fc_n && (rc = dalloc(s, &s->fc_n, 2))) || (rc = dalloc(s, &s->pair_rec, 1)))
            return rc;
    }
    Staging st;
    const size_t img_bytes = (size_t)w * h;
    int rc = staging(ctx, Staging::round(sizeof(dvo_pair_record)) + (reuse_prev ? 1 : 2) * Staging::round(img_bytes),
                     s->hs, &st);
    if (rc) return rc;
    const int pw = frame_pitch(s);
    // host frames go through the pinned staging area: one host copy, one asynchronous DMA each
    auto upload = [&](uint8_t* dst, const uint8_t* img) -> hipError_t {
        uint8_t* hp = st.take(img_bytes);
        if (stride == w) {
            std::memcpy(hp, img, img_bytes);
        } else {
            for (int y = 0; y < h; ++y) std::memcpy(hp + (size_t)y * w, img + (size_t)y * stride, w);
        }
        return hipMemcpy2DAsync(dst, pw, hp, w, w, h, hipMemcpyHostToDevice, s->hs);
    };
    const int64_t fst = (int64_t)pw * h;
    const Buffers& b = s->buf;
    // after the first upload, an error drains the stream before returning: its DMAs read the
    // context's pinned staging area, which the next staging user rewrites (or frees to grow it)
    auto body = [&]() -> int {
    // the feature arrays of frame 0, frame 1 and the cache (the last current frame's), in 4-byte words
    FeatSlots fsl{};
    auto slot = [&](int k, void* kps, void* desc, int32_t* n, int32_t* stt) {
        fsl.a[k][0] = (uint32_t*)kps;
        fsl.a[k][1] = (uint32_t*)desc;
        fsl.a[k][2] = (uint32_t*)n;
        fsl.a[k][3] = (uint32_t*)stt;
    };
    slot(0, b.kps, b.desc, b.nkp, b.status);
    slot(1, b.kps + kc, b.desc + kc * 32, b.nkp + 1, b.status + 1);
    slot(2, s->fc_kps, s->fc_desc, s->fc_n, s->fc_n + 1);
    fsl.words[0] = (int)(kc * sizeof(dvo_keypoint) / 4);
    fsl.words[1] = (int)(kc * 32 / 4);
    fsl.words[2] = fsl.words[3] = 1;
    if (reuse_prev) {
        HIP_TRY(upload(s->d_frames, cur_img));
        if ((rc = run_stream(s, s->d_frames, 1, fst, pw, nullptr, true))) return rc;
        // frame 1 <- the new frame's features (frame 0), frame 0 <- the cached previous frame's, and the
        // cache <- the new frame's (the next pair's previous frame): one launch, element by element
        HIP_TRY(launch_feature_rotate(fsl, 1, s->hs));
    } else {
        HIP_TRY(upload(s->d_frames, prev_img));
        HIP_TRY(upload(s->d_frames + fst, cur_img));
        if ((rc = run_stream(s, s->d_frames, 2, fst, pw, nullptr, true))) return rc;
        HIP_TRY(launch_feature_rotate(fsl, 0, s->hs));  // the current frame's features are the next previous
    }
    StreamParams P = params_of(s, s->d_frames, 2, fst, pw);
    const int nqb = ((int)kc + 255) / 256, nst = ((int)kc + 63) / 64;
    int tsplit = 1;
    while (tsplit < 16 && nqb * tsplit * 2 <= 256 && nst >= tsplit * 8) tsplit *= 2;
    HIP_TRY(launch_match(P, s->cfg.cross_check, s->hs, nullptr, tsplit));
    HIP_TRY(launch_geometry(P, stream_geom(s), s->pair_rec, s->hs, nullptr, true));
    uint8_t* hr = nullptr;
    HIP_TRY(st.get(s->pair_rec, sizeof(dvo_pair_record), &hr));
    HIP_TRY(hipStreamSynchronize(s->hs));
    std::memcpy(rec_out, hr, sizeof(dvo_pair_record));
    return DVO_OK;
    };
    if ((rc = body())) {
        (void)hipStreamSynchronize(s->hs);
        return rc;
    }
    s->fc_valid = true;
    s->last_reuse = reuse_prev != 0;
    s->last_nframes = 2;
    s->last_pairs = 1;
    s->last_sub_pairs = 1;
    s->last_set = 0;
    s->last_has_pairs = true;
    s->last_rec = s->pair_rec;
    s->last_frames = s->d_frames;
    s->last_fstride = fst;
    s->last_pitch = pw;
    return DVO_OK;
}

int dvo_stream_sync(dvo_stream* s) {
    if (!s) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    HIP_TRY(hipStreamSynchronize(s->hs));
    HIP_TRY(hipGetLastError());
    return DVO_OK;
}

int dvo_stream_get_features(dvo_stream* s, int frame, dvo_keypoint* kps, uint8_t* desc, int cap, int* n) {
    if (!s || !n) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (frame < 0 || frame >= s->last_nframes) return fail(ctx, DVO_EINVAL, "frame out of range");
    HIP_TRY(hipStreamSynchronize(s->hs));
    int nk = 0, st = 0;
    HIP_TRY(hipMemcpy(&nk, s->buf.nkp + frame, sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&st, s->buf.status + frame, sizeof(int), hipMemcpyDeviceToHost));
    *n = nk;
    if (st) return fail(ctx, DVO_ECAP, "keypoint capacity exceeded (Harris ties)");
    if (nk > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    if (nk > 0) {
        if (kps)
            HIP_TRY(hipMemcpy(kps, s->buf.kps + (size_t)frame * s->plan.kp_cap, sizeof(dvo_keypoint) * nk,
                              hipMemcpyDeviceToHost));
        if (desc)
            HIP_TRY(hipMemcpy(desc, s->buf.desc + (size_t)frame * s->plan.kp_cap * 32, 32 * (size_t)nk,
                              hipMemcpyDeviceToHost));
    }
    return DVO_OK;
}

int dvo_stream_get_matches(dvo_stream* s, int pair, dvo_dmatch* out, int cap, int* m) {
    if (!s || !m) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (pair < 0 || pair >= s->last_sub_pairs) return fail(ctx, DVO_EINVAL, "pair out of range");
    HIP_TRY(hipStreamSynchronize(s->hs));
    int nm = 0;
    HIP_TRY(hipMemcpy(&nm, s->buf.nmatch + (size_t)s->last_set * s->cfg.max_frames + pair, sizeof(int),
                      hipMemcpyDeviceToHost));
    *m = nm;
    if (nm > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    std::vector<int32_t> q(nm), t(nm);
    std::vector<float> d(nm);
    const size_t off = (size_t)pair * s->plan.kp_cap;
    if (nm) {
        HIP_TRY(hipMemcpy(q.data(), s->buf.mq + off, 4 * (size_t)nm, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(t.data(), s->buf.mt + off, 4 * (size_t)nm, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(d.data(), s->buf.md + off, 4 * (size_t)nm, hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < nm; ++i) out[i] = dvo_dmatch{q[i], t[i], 0, d[i]};
    return DVO_OK;
}

int dvo_stream_get_pyramid(dvo_stream* s, int frame, int level, int blurred, uint8_t* out, int cap) {
    if (!s || !out) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (frame < 0 || frame >= s->last_nframes || level < 0 || level >= s->plan.nlevels)
        return fail(ctx, DVO_EINVAL, "frame/level out of range");
    int nfr = s->last_nframes;
    if (s->last_reuse) {  // dvo_stream_pair(reuse_prev) detected frame 1 alone, into pyramid slot 0
        if (frame == 0)
            return fail(ctx, DVO_EINVAL, "after dvo_stream_pair(reuse_prev) only frame 1's pyramid is kept");
        frame = 0;
        nfr = 1;
    }
    const LevelGeom& G = s->plan.L[level];
    if (cap < G.w * G.h) return fail(ctx, DVO_ECAP, "capacity too small");
    HIP_TRY(hipStreamSynchronize(s->hs));
    if (blurred) {
        // the detection path blurs only the descriptor windows (describe_kernel): the whole blurred
        // pyramid is recomputed here from the last call's frames, which must still be alive
        HIP_TRY(launch_blur(params_of(s, s->last_frames, nfr, s->last_fstride, s->last_pitch), s->hs));
        HIP_TRY(hipStreamSynchronize(s->hs));
    }
    if (blurred) {
        HIP_TRY(hipMemcpy2D(out, G.w, s->buf.blur + (size_t)frame * s->plan.blur_stride + G.blur_off, G.bpitch, G.w,
                            G.h, hipMemcpyDeviceToHost));
    } else {
        if (level == 0) return fail(ctx, DVO_EINVAL, "level 0 is the input frame");
        HIP_TRY(hipMemcpy2D(out, G.w, s->buf.pyr + (size_t)frame * s->plan.pyr_stride + G.pyr_off, G.pitch, G.w,
                            G.h, hipMemcpyDeviceToHost));
    }
    return DVO_OK;
}

// ---------------------------------------------------------------------------
int dvo_orb_detect_and_compute(dvo_ctx* ctx, const dvo_orb_params* params, const uint8_t* img, int w, int h,
                               int stride, dvo_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
    if (!ctx) return DVO_EINVAL;
    int rc = check_orb_params(ctx, params);
    if (rc) return rc;
    if (!img || !n_out || stride < w) return fail(ctx, DVO_EINVAL, "bad image buffer");
    if (w < 8 || h < 8 || w >= kMaxW || h >= kMaxW) return fail(ctx, DVO_EINVAL, "image size out of range (8..4095)");
    HIP_TRY(hipSetDevice(ctx->device));
    if (!ctx->call_stream || ctx->call_w != w || ctx->call_h != h || ctx->call_nf != params->nfeatures ||
        ctx->call_stream->cfg.orb.fast_threshold != params->fast_threshold ||
        ctx->call_stream->cfg.orb.opencv_semantics != params->opencv_semantics) {
        if (ctx->call_stream) dvo_stream_destroy(ctx->call_stream);
        ctx->call_stream = nullptr;
        dvo_stream_config cfg{};
        cfg.width = w;
        cfg.height = h;
        cfg.max_frames = 2;
        cfg.orb = *params;
        cfg.K[0] = cfg.K[4] = cfg.K[8] = 1.0;
        cfg.prob = 0.999;
        cfg.threshold = 1.0;
        cfg.max_iters = 1000;
        cfg.cross_check = 1;
        cfg.dist_thresh = 50.0;
        rc = dvo_stream_create(ctx, &cfg, &ctx->call_stream);
        if (rc) return rc;
        ctx->call_w = w;
        ctx->call_h = h;
        ctx->call_nf = params->nfeatures;
    }
    dvo_stream* s = ctx->call_stream;
    const int pw = frame_pitch(s);
    const size_t kc = (size_t)s->plan.kp_cap;
    Staging st;
    if ((rc = staging(ctx, 2 * Staging::round(4) + Staging::round(kc * sizeof(dvo_keypoint)) + Staging::round(kc * 32),
                      s->hs, &st)))
        return rc;
    HIP_TRY(hipMemcpy2DAsync(s->d_frames, pw, img, stride, w, h, hipMemcpyHostToDevice, s->hs));
    rc = run_stream(s, s->d_frames, 1, (int64_t)pw * h, pw, nullptr, true);
    if (rc) return rc;
    // dvo_stream_get_features of frame 0, with every list copied back at once (capacity-sized)
    uint8_t *hn, *hst, *hk = nullptr, *hd = nullptr;
    HIP_TRY(st.get(s->buf.nkp, sizeof(int), &hn));
    HIP_TRY(st.get(s->buf.status, sizeof(int), &hst));
    if (kps) HIP_TRY(st.get(s->buf.kps, kc * sizeof(dvo_keypoint), &hk));
    if (desc) HIP_TRY(st.get(s->buf.desc, kc * 32, &hd));
    HIP_TRY(hipStreamSynchronize(s->hs));
    int nk = 0, stt = 0;
    std::memcpy(&nk, hn, sizeof(int));
    std::memcpy(&stt, hst, sizeof(int));
    *n_out = nk;
    if (stt) return fail(ctx, DVO_ECAP, "keypoint capacity exceeded (Harris ties)");
    if (nk > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    if (nk > 0) {
        if (kps) std::memcpy(kps, hk, sizeof(dvo_keypoint) * nk);
        if (desc) std::memcpy(desc, hd, 32 * (size_t)nk);
    }
    return DVO_OK;
}

int dvo_bf_match_hamming(dvo_ctx* ctx, const uint8_t* dq, int nq, const uint8_t* dt, int nt, int cross_check,
                         dvo_dmatch* out, int cap, int* m_out) {
    if (!ctx || !m_out) return DVO_EINVAL;
    *m_out = 0;
    if (cross_check < 0 || cross_check > 2) return fail(ctx, DVO_EINVAL, "cross_check must be 0, 1 or 2");
    if (nq < 0 || nt < 0 || nq > 8192 || nt > 8192)
        return fail(ctx, DVO_EINVAL, "descriptor count out of range (0..8192)");
    if (nq == 0 || nt == 0) return DVO_OK;  // BFMatcher returns no matches
    if (!dq || !dt || !out) return fail(ctx, DVO_EINVAL, "null buffer");
    HIP_TRY(hipSetDevice(ctx->device));
    void *bq, *bt, *bnn, *bout, *bm;
    int rc;
    if ((rc = scratch(ctx, 0, (size_t)nq * 32, &bq)) || (rc = scratch(ctx, 1, (size_t)nt * 32, &bt)) ||
        (rc = scratch(ctx, 2, match_pair_work_size(nq, nt), &bnn)) ||
        (rc = scratch(ctx, 3, (size_t)nq * sizeof(dvo_dmatch), &bout)) ||
        (rc = scratch(ctx, 4, 64, &bm)))
        return rc;
    Staging st;
    if ((rc = staging(ctx, Staging::round((size_t)nq * 32) + Staging::round((size_t)nt * 32) + Staging::round(64) +
                               Staging::round((size_t)nq * sizeof(dvo_dmatch)), ctx->stream, &st)))
        return rc;
    HIP_TRY(st.put(bq, dq, (size_t)nq * 32));
    HIP_TRY(st.put(bt, dt, (size_t)nt * 32));
    HIP_TRY(launch_match_pair((const uint8_t*)bq, nq, (const uint8_t*)bt, nt, cross_check, bnn, (dvo_dmatch*)bout,
                              (int*)bm, ctx->stream));
    uint8_t *hm, *hout;
    HIP_TRY(st.get(bm, sizeof(int), &hm));
    HIP_TRY(st.get(bout, (size_t)nq * sizeof(dvo_dmatch), &hout));  // at most one match per query
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int m = 0;
    std::memcpy(&m, hm, sizeof(int));
    *m_out = m;
    if (m > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    if (m) std::memcpy(out, hout, (size_t)m * sizeof(dvo_dmatch));
    return DVO_OK;
}

int dvo_bf_knn_float(dvo_ctx* ctx, const float* dq, int nq, const float* dt, int nt, int dim, int k, int norm,
                     int32_t* train_idx, float* dist) {
    if (!ctx) return DVO_EINVAL;
    if (norm != DVO_NORM_L1 && norm != DVO_NORM_L2SQR) return fail(ctx, DVO_EINVAL, "norm must be DVO_NORM_L1 or DVO_NORM_L2SQR");
    if (dim != 64 && dim != 128) return fail(ctx, DVO_EINVAL, "descriptor length must be 64 (SURF) or 128 (SIFT)");
    if (k < 1 || k > 4) return fail(ctx, DVO_EINVAL, "k must be 1..4");
    if (nq < 0 || nt < 0 || nq > (1 << 20) || nt > (1 << 20))
        return fail(ctx, DVO_EINVAL, "descriptor count out of range (0..2^20)");
    if (nq == 0) return DVO_OK;
    if (!dq || !train_idx || !dist || (nt > 0 && !dt)) return fail(ctx, DVO_EINVAL, "null buffer");
    if (nt == 0) {  // batchDistance leaves every slot at (-1, FLT_MAX)
        for (size_t i = 0; i < (size_t)nq * k; ++i) {
            train_idx[i] = -1;
            dist[i] = FLT_MAX;
        }
        return DVO_OK;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const int ranges = knn_ranges(nq, nt, cus);
    const size_t out_n = (size_t)nq * k, part_n = ranges > 1 ? (size_t)ranges * nq * k : 1;
    void *bq, *bt, *bd, *bi, *bpd, *bpi, *bb;
    int rc;
    if ((rc = scratch(ctx, 27, (size_t)nq * dim * 4, &bq)) || (rc = scratch(ctx, 28, (size_t)nt * dim * 4, &bt)) ||
        (rc = scratch(ctx, 29, out_n * 4, &bd)) || (rc = scratch(ctx, 30, out_n * 4, &bi)) ||
        (rc = scratch(ctx, 31, part_n * 4, &bpd)) || (rc = scratch(ctx, 32, part_n * 4, &bpi)) ||
        (rc = scratch(ctx, 33, knn_bytes_size(nq, nt, dim), &bb)))
        return rc;
    HIP_TRY(hipMemcpyAsync(bq, dq, (size_t)nq * dim * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(bt, dt, (size_t)nt * dim * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_knn_float((const float*)bq, nq, (const float*)bt, nt, dim, k, norm, ranges, bb, (float*)bpd, (int32_t*)bpi,
                             (float*)bd, (int32_t*)bi, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dist, bd, out_n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(train_idx, bi, out_n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DVO_OK;
}

namespace {
// cv::theRNG()'s multiply-with-carry s' = (u32)s * A + (s >> 32) is s' = s * A mod m,
// m = A * 2^32 - 1, for every state below m (all but a few seeds): jump k steps ahead.
constexpr uint64_t kTheRngA = 4164903690ull;
uint64_t therng_jump(uint64_t s, uint64_t k) {
    const unsigned __int128 m = ((unsigned __int128)kTheRngA << 32) - 1;
    if (k > 0 && (unsigned __int128)s >= m) {  // a seed at or above m: one plain step lands below m
        s = (uint64_t)(uint32_t)s * kTheRngA + (s >> 32);
        --k;
    }
    unsigned __int128 r = s, b = kTheRngA;
    for (; k; k >>= 1) {
        if (k & 1) r = r * b % m;
        b = b * b % m;
    }
    return (uint64_t)r;
}
}  // namespace

// Replaces cv::FlannBasedMatcher(KDTREE, trees).knnMatch(query, train, k) with
// search checks (the 'flann' mode, visual_odometry_v3.py:206-212); flann.hip.
int dvo_flann_knn(dvo_ctx* ctx, const float* dq, int nq, const float* dt, int nt, int dim, int k, int trees,
                  int checks, uint64_t* rng_state, int32_t* train_idx, float* dist) {
    if (!ctx) return DVO_EINVAL;
    if (!rng_state) return fail(ctx, DVO_EINVAL, "null theRNG state");
    if (dim < 4 || dim > 256 || dim % 4) return fail(ctx, DVO_EINVAL, "dim must be a multiple of 4 in 4..256");
    if (k < 1 || k > 4) return fail(ctx, DVO_EINVAL, "k must be 1..4");
    if (trees < 1 || trees > 64 || checks < 1) return fail(ctx, DVO_EINVAL, "trees 1..64 and checks >= 1");
    if (nq < 0 || nt < 0 || nq > (1 << 20) || nt > (1 << 16))
        return fail(ctx, DVO_EINVAL, "descriptor counts out of range (queries 0..2^20, train 0..2^16)");
    // DescriptorMatcher::knnMatch returns before training on an empty query or train set
    if (nq == 0 || nt == 0) return DVO_OK;
    if (!dq || !dt || !train_idx || !dist) return fail(ctx, DVO_EINVAL, "null buffer");
    if (k > nt) return fail(ctx, DVO_EINVAL, "k exceeds the train set (FLANN asserts knn <= index size)");
    HIP_TRY(hipSetDevice(ctx->device));
    const int n = nt, draws = 2 * n - 1, nodes_per_tree = 2 * n - 1;
    constexpr int kChunks = 64;
    void *bq, *bt, *bR, *bcs, *bcnt, *boff, *bfill, *blist, *bind, *bind2, *bxv, *bsl, *bsr, *bnodes, *bopen, *blev,
        *bidx, *bdist, *bflag, *bredo;
    int rc;
    if ((rc = scratch(ctx, 40, (size_t)nq * dim * 4, &bq)) || (rc = scratch(ctx, 41, (size_t)nt * dim * 4, &bt)) ||
        (rc = scratch(ctx, 42, (size_t)draws * 4, &bR)) || (rc = scratch(ctx, 43, (size_t)trees * kChunks * 8, &bcs)) ||
        (rc = scratch(ctx, 44, (size_t)n * 4, &bcnt)) || (rc = scratch(ctx, 45, (size_t)(n + 1) * 4, &boff)) ||
        (rc = scratch(ctx, 46, (size_t)n * 4, &bfill)) || (rc = scratch(ctx, 47, (size_t)n * 4, &blist)) ||
        (rc = scratch(ctx, 48, (size_t)n * 4, &bind)) || (rc = scratch(ctx, 49, (size_t)n * 4, &bind2)) ||
        (rc = scratch(ctx, 50, (size_t)n * 4, &bxv)) || (rc = scratch(ctx, 51, (size_t)n * 4, &bsl)) ||
        (rc = scratch(ctx, 52, (size_t)n * 4, &bsr)) ||
        (rc = scratch(ctx, 53, (size_t)trees * nodes_per_tree * 16, &bnodes)) ||
        (rc = scratch(ctx, 54, (size_t)2 * n * 16, &bopen)) || (rc = scratch(ctx, 55, (size_t)(n + 2) * 4, &blev)) ||
        (rc = scratch(ctx, 56, (size_t)nq * k * 4, &bidx)) || (rc = scratch(ctx, 57, (size_t)nq * k * 4, &bdist)) ||
        (rc = scratch(ctx, 58, (size_t)nq * 4, &bflag)) || (rc = scratch(ctx, 59, (size_t)(nq + 1) * 4, &bredo)))
        return rc;
    hipStream_t s = ctx->stream;
    Staging st;
    if ((rc = staging(ctx, Staging::round((size_t)nq * dim * 4) + Staging::round((size_t)nt * dim * 4) +
                               Staging::round((size_t)trees * kChunks * 8) + 2 * Staging::round((size_t)nq * k * 4) +
                               2 * Staging::round(4),
                      s, &st)))
        return rc;
    // the multiply-with-carry state at the start of every draw chunk of every tree (tree t's draws
    // begin t (2n - 1) steps after the call's state)
    std::vector<uint64_t> cs((size_t)trees * kChunks);
    for (int t = 0; t < trees; ++t)
        for (int c = 0; c < kChunks; ++c)
            cs[(size_t)t * kChunks + c] =
                therng_jump(*rng_state, (uint64_t)t * draws + (uint64_t)((int64_t)draws * c / kChunks));
    HIP_TRY(st.put(bq, dq, (size_t)nq * dim * 4));
    HIP_TRY(st.put(bt, dt, (size_t)nt * dim * 4));
    HIP_TRY(st.put(bcs, cs.data(), cs.size() * 8));
    // ind = 0..n-1 once; every tree shuffles the previous tree's final order (KDTreeIndex::buildIndex)
    {
        std::vector<int32_t> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
        HIP_TRY(hipMemcpyAsync(bind, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));  // the pageable copy must finish before iota goes out of scope
    }
    int* ind = (int*)bind;
    int* ind2 = (int*)bind2;
    int32_t* hcnt = reinterpret_cast<int32_t*>(st.take(4));
    for (int t = 0; t < trees; ++t) {
        HIP_TRY(launch_flann_draws((const uint64_t*)bcs + (size_t)t * kChunks, kChunks, draws, (uint32_t*)bR, s));
        HIP_TRY(launch_flann_shuffle((const uint32_t*)bR, n, (int*)bcnt, (int*)boff, (int*)bfill, (int*)blist, ind, ind2,
                                     s));
        std::swap(ind, ind2);
        FlannBuildArgs a{(const float*)bt, n, dim, ind, (float*)bxv, (int*)bsl, (int*)bsr, (const uint32_t*)bR,
                         (int4*)bnodes + (size_t)t * nodes_per_tree, (int4*)bopen, (int4*)bopen + n, (int*)blev};
        HIP_TRY(hipMemsetAsync(blev, 0, (size_t)(n + 2) * 4, s));
        HIP_TRY(launch_flann_root(a, s));
        // level-synchronous divideTree: a level has at most min(2^d, n / 2) open nodes; levels go in
        // batches of 8, then the host reads whether the next level has any
        for (int d = 0; d < n; d += 8) {
            for (int e = d; e < d + 8 && e < n; ++e)
                HIP_TRY(launch_flann_level(a, e, (int)std::min<int64_t>(int64_t(1) << std::min(e, 20), n / 2 + 1), s));
            HIP_TRY(hipMemcpyAsync(hcnt, (int*)blev + std::min(d + 8, n + 1), 4, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (*hcnt == 0) break;
        }
    }
    FlannSearchArgs sa{(const float*)bq, (const float*)bt, (const int4*)bnodes, nq, n, dim, k, trees, checks,
                       (int32_t*)bidx, (float*)bdist, (int32_t*)bflag};
    HIP_TRY(launch_flann_search(sa, s));
    HIP_TRY(launch_flann_redo_list((const int32_t*)bflag, nq, (int32_t*)bredo + 1, (int32_t*)bredo, s));
    int32_t* hredo = reinterpret_cast<int32_t*>(st.take(4));
    HIP_TRY(hipMemcpyAsync(hredo, bredo, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int done = 0; done < *hredo;) {  // queries whose heap outgrew LDS, with the heap in global memory
        const int batch = std::min(*hredo - done, 256);
        void *bhd, *bhn;
        if ((rc = scratch(ctx, 60, (size_t)batch * n * 4, &bhd)) || (rc = scratch(ctx, 61, (size_t)batch * n * 4, &bhn)))
            return rc;
        HIP_TRY(launch_flann_search_global(sa, (const int32_t*)bredo + 1 + done, batch, (float*)bhd, (int32_t*)bhn, s));
        done += batch;
    }
    uint8_t *hi, *hd;
    HIP_TRY(st.get(bidx, (size_t)nq * k * 4, &hi));
    HIP_TRY(st.get(bdist, (size_t)nq * k * 4, &hd));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(train_idx, hi, (size_t)nq * k * 4);
    std::memcpy(dist, hd, (size_t)nq * k * 4);
    *rng_state = therng_jump(*rng_state, (uint64_t)trees * draws);
    return DVO_OK;
}

namespace {
// getGaussianKernel(ksize = cvRound(sigma * 8 + 1) | 1, sigma, CV_32F), as oracle/sift.cpp gauss_kernel
std::vector<float> sift_gauss_taps(double sigma) {
    const int n = (int)std::nearbyint(sigma * 4 * 2 + 1) | 1;
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

int sift_plan(dvo_ctx* ctx, int w, int h) {
    SiftPlanDev& P = ctx->sift;
    if (P.w == w && P.h == h) return DVO_OK;
    for (void* p : P.allocs) hipFree(p);
    P = SiftPlanDev{};
    SiftArgs& A = P.a;
    const int W = 2 * w, H = 2 * h;  // firstOctave = -1
    A.noct = (int)std::nearbyint(std::log((double)std::min(W, H)) / std::log(2.) - 2) + 1;
    A.noct = std::max(1, std::min(A.noct, kSiftMaxOct));
    int64_t gp = 0, dg = 0;
    for (int o = 0; o < A.noct; ++o) {
        A.ow[o] = o == 0 ? W : A.ow[o - 1] / 2;
        A.oh[o] = o == 0 ? H : A.oh[o - 1] / 2;
        if (A.ow[o] < 1 || A.oh[o] < 1) {  // as small as the pyramid goes
            A.noct = o;
            break;
        }
        const int64_t px = (int64_t)A.ow[o] * A.oh[o];
        for (int l = 0; l < 6; ++l) A.gp_off[o * 6 + l] = gp + l * px;
        for (int l = 0; l < 5; ++l) A.dog_off[o * 5 + l] = dg + l * px;
        gp += 6 * px;
        dg += 5 * px;
    }
    A.cand_cap = 1 << 18;
    A.kp_cap = 1 << 16;
    std::vector<float> taps;
    const double sig0 = std::sqrt(std::max(1.6f * 1.6f - 0.5f * 0.5f * 4, 0.01f));
    std::vector<double> sig(6);
    sig[0] = sig0;
    const double k = std::pow(2., 1. / 3);
    for (int i = 1; i < 6; ++i) {
        // buildGaussianPyramid uses SIFT_Impl's double member sigma (1.6, not 1.6f);
        // only createInitialImage and adjustLocalExtrema take it as float
        const double sig_prev = std::pow(k, (double)(i - 1)) * 1.6, sig_total = sig_prev * k;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    for (int i = 0; i < 6; ++i) {
        const std::vector<float> t = sift_gauss_taps(i == 0 ? (double)(float)sig0 : sig[i]);
        P.tap_off[i] = (int)taps.size();
        P.tap_n[i] = (int)t.size();
        taps.insert(taps.end(), t.begin(), t.end());
    }
    P.pitch = (w + 255) & ~255;
    auto A_ = [&](auto*& p, size_t bytes) {
        void* q = nullptr;
        if (hipMalloc(&q, bytes ? bytes : 16) != hipSuccess) return false;
        P.allocs.push_back(q);
        p = static_cast<std::remove_reference_t<decltype(p)>>(q);
        return true;
    };
    int order_n = 1;
    while (order_n < A.kp_cap) order_n <<= 1;
    int* counters = nullptr;
    if (!A_(A.gp, (size_t)gp * 4) || !A_(A.dog, (size_t)dg * 4) || !A_(A.tmp, (size_t)W * H * 4) ||
        !A_(A.cand, (size_t)A.cand_cap * sizeof(int4)) || !A_(A.raw, (size_t)A.kp_cap * sizeof(dvo_keypoint)) ||
        !A_(A.order, (size_t)order_n * 4) || !A_(A.kps, (size_t)A.kp_cap * sizeof(dvo_keypoint)) ||
        !A_(A.desc, (size_t)A.kp_cap * 128 * 4) || !A_(counters, 64) || !A_(P.taps, taps.size() * 4) ||
        !A_(P.img, (size_t)P.pitch * h)) {
        for (void* p : P.allocs) hipFree(p);
        P = SiftPlanDev{};
        return fail(ctx, DVO_EHIP, "SIFT buffers: hipMalloc failed");
    }
    A.ncand = counters;
    A.nraw = counters + 1;
    A.nkp = counters + 2;
    A.flags = counters + 3;
    if (hipMemcpy(P.taps, taps.data(), taps.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(ctx, DVO_EHIP, "SIFT taps upload failed");
    P.w = w;
    P.h = h;
    return DVO_OK;
}
}  // namespace

namespace {
// getGaussianKernel(n, sigma, CV_32F) as oracle/surf.cpp restates it
std::vector<float> surf_gauss(int n, double sigma) {
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

// resizeHaarPattern (surf.cpp) on the host: offsets in an integral image of row step `step`
void surf_haar(const int src[][5], SurfHaar* dst, int n, int old_size, int new_size, int step) {
    const float ratio = (float)new_size / old_size;
    for (int k = 0; k < n; ++k) {
        const int dx1 = (int)std::nearbyint(ratio * src[k][0]), dy1 = (int)std::nearbyint(ratio * src[k][1]);
        const int dx2 = (int)std::nearbyint(ratio * src[k][2]), dy2 = (int)std::nearbyint(ratio * src[k][3]);
        dst[k].p0 = dy1 * step + dx1;
        dst[k].p1 = dy2 * step + dx1;
        dst[k].p2 = dy1 * step + dx2;
        dst[k].p3 = dy2 * step + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

int surf_plan(dvo_ctx* ctx, int w, int h) {
    SurfPlanDev& P = ctx->surf;
    if (P.w == w && P.h == h) return DVO_OK;
    for (void* p : P.allocs) hipFree(p);
    P = SurfPlanDev{};
    SurfArgs& A = P.a;
    A.w = w;
    A.h = h;
    A.pitch = (w + 255) & ~255;
    const int sw = w + 1;
    static const int dx_s[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
    static const int dy_s[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
    static const int dxy_s[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};
    std::vector<SurfHaar> haar((size_t)kSurfTot * 10);
    int64_t cells = 0;
    for (int o = 0; o < kSurfOct; ++o) {
        const int step = 1 << o;
        A.rows[o] = h / step;
        A.cols[o] = w / step;
        for (int l = 0; l < kSurfLayers; ++l) {
            const int L = o * kSurfLayers + l;
            A.size[L] = (9 + 6 * l) << o;
            A.off[L] = cells;
            cells += (int64_t)A.rows[o] * A.cols[o];
            surf_haar(dx_s, &haar[L * 10], 3, 9, A.size[L], sw);
            surf_haar(dy_s, &haar[L * 10 + 3], 3, 9, A.size[L], sw);
            surf_haar(dxy_s, &haar[L * 10 + 6], 4, 9, A.size[L], sw);
        }
    }
    // SURF_ORI_SIGMA 2.5f, SURF_DESC_SIGMA 3.3f: float constants widened to double
    const std::vector<float> go = surf_gauss(13, (double)2.5f), gd = surf_gauss(20, (double)3.3f);
    std::vector<int8_t> apt;
    std::vector<float> aptw;
    for (int i = -6; i <= 6; ++i)
        for (int j = -6; j <= 6; ++j)
            if (i * i + j * j <= 36) {
                apt.push_back((int8_t)i);
                apt.push_back((int8_t)j);
                aptw.push_back(go[i + 6] * go[j + 6]);
            }
    A.nori = (int)aptw.size();
    for (int i = 0; i < 20; ++i) A.gdesc[i] = gd[i];
    A.kp_cap = std::max(4096, (w * h) / 64);
    int order_n = 1;
    while (order_n < A.kp_cap) order_n <<= 1;
    auto A_ = [&](auto*& p, size_t bytes) {
        void* q = nullptr;
        if (hipMalloc(&q, bytes ? bytes : 16) != hipSuccess) return false;
        P.allocs.push_back(q);
        p = static_cast<std::remove_reference_t<decltype(p)>>(q);
        return true;
    };
    int* counters = nullptr;
    SurfHaar* d_haar = nullptr;
    int8_t* d_apt = nullptr;
    float* d_aptw = nullptr;
    if (!A_(A.sum, (size_t)sw * (h + 1) * 4) || !A_(A.det, (size_t)cells * 4) || !A_(A.trace, (size_t)cells * 4) ||
        !A_(A.raw, (size_t)A.kp_cap * sizeof(dvo_keypoint)) || !A_(A.order, (size_t)order_n * 4) ||
        !A_(A.kps, (size_t)A.kp_cap * sizeof(dvo_keypoint)) || !A_(A.dtmp, (size_t)A.kp_cap * 64 * 4) ||
        !A_(A.out, (size_t)A.kp_cap * sizeof(dvo_keypoint)) || !A_(A.desc, (size_t)A.kp_cap * 64 * 4) ||
        !A_(counters, 64) || !A_(d_haar, haar.size() * sizeof(SurfHaar)) || !A_(d_apt, apt.size()) ||
        !A_(d_aptw, aptw.size() * 4) || !A_(P.img, (size_t)A.pitch * h)) {
        for (void* p : P.allocs) hipFree(p);
        P = SurfPlanDev{};
        return fail(ctx, DVO_EHIP, "SURF buffers: hipMalloc failed");
    }
    A.nraw = counters;
    A.nout = counters + 1;
    A.flags = counters + 2;
    A.haar = d_haar;
    A.apt = d_apt;
    A.aptw = d_aptw;
    A.img = P.img;
    if (hipMemcpy(d_haar, haar.data(), haar.size() * sizeof(SurfHaar), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_apt, apt.data(), apt.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_aptw, aptw.data(), aptw.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(ctx, DVO_EHIP, "SURF tables upload failed");
    P.w = w;
    P.h = h;
    return DVO_OK;
}
}  // namespace

int dvo_surf_detect_and_compute(dvo_ctx* ctx, const uint8_t* img, int w, int h, int stride, double hessian_threshold,
                                dvo_keypoint* kps, float* desc, int cap, int* n_out) {
    if (!ctx || !n_out) return DVO_EINVAL;
    *n_out = 0;
    if (!img || stride < w) return fail(ctx, DVO_EINVAL, "bad image buffer");
    if (w < 1 || h < 1 || w >= kMaxW || h >= kMaxW) return fail(ctx, DVO_EINVAL, "image size out of range (1..4095)");
    if (!(hessian_threshold >= 0)) return fail(ctx, DVO_EINVAL, "hessianThreshold must be >= 0");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = surf_plan(ctx, w, h);
    if (rc) return rc;
    SurfPlanDev& P = ctx->surf;
    P.a.thr = (float)hessian_threshold;
    HIP_TRY(hipMemsetAsync(P.a.nraw, 0, 16, ctx->stream));
    const int64_t cells = P.a.off[kSurfTot - 1] + (int64_t)P.a.rows[kSurfOct - 1] * P.a.cols[kSurfOct - 1];
    HIP_TRY(hipMemsetAsync(P.a.det, 0, (size_t)cells * 4, ctx->stream));
    HIP_TRY(hipMemsetAsync(P.a.trace, 0, (size_t)cells * 4, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(P.img, P.a.pitch, img, stride, w, h, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_surf(P.a, ctx->stream));
    int cnt[3];
    HIP_TRY(hipMemcpyAsync(cnt, P.a.nraw, 12, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (cnt[2]) return fail(ctx, DVO_ECAP, "SURF: more keypoints than the device lists hold");
    const int n = cnt[1];
    *n_out = n;
    if (n > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    if (n) {
        if (kps) HIP_TRY(hipMemcpyAsync(kps, P.a.out, (size_t)n * sizeof(dvo_keypoint), hipMemcpyDeviceToHost, ctx->stream));
        if (desc) HIP_TRY(hipMemcpyAsync(desc, P.a.desc, (size_t)n * 64 * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return DVO_OK;
}

int dvo_sift_detect_and_compute(dvo_ctx* ctx, const uint8_t* img, int w, int h, int stride, dvo_keypoint* kps,
                                float* desc, int cap, int* n_out) {
    if (!ctx || !n_out) return DVO_EINVAL;
    *n_out = 0;
    if (!img || stride < w) return fail(ctx, DVO_EINVAL, "bad image buffer");
    if (w < 1 || h < 1 || w >= kMaxW || h >= kMaxW) return fail(ctx, DVO_EINVAL, "image size out of range (1..4095)");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = sift_plan(ctx, w, h);
    if (rc) return rc;
    SiftPlanDev& P = ctx->sift;
    HIP_TRY(hipMemsetAsync(P.a.ncand, 0, 16, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(P.img, P.pitch, img, stride, w, h, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_sift(P.a, P.img, w, h, P.pitch, P.taps, P.tap_off, P.tap_n, ctx->stream));
    int cnt[4];
    HIP_TRY(hipMemcpyAsync(cnt, P.a.ncand, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (cnt[3]) return fail(ctx, DVO_ECAP, "SIFT: more extrema / keypoints than the device lists hold");
    const int n = cnt[2];
    *n_out = n;
    if (n > cap) return fail(ctx, DVO_ECAP, "caller capacity too small");
    if (n) {
        if (kps) HIP_TRY(hipMemcpyAsync(kps, P.a.kps, (size_t)n * sizeof(dvo_keypoint), hipMemcpyDeviceToHost, ctx->stream));
        if (desc) HIP_TRY(hipMemcpyAsync(desc, P.a.desc, (size_t)n * 128 * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return DVO_OK;
}

static int upload_points(dvo_ctx* ctx, Staging& st, const double* p1, const double* p2, int m, void** dpts) {
    int rc = scratch(ctx, 5, (size_t)(m > 0 ? m : 1) * 32, dpts);
    if (rc) return rc;
    double* h = reinterpret_cast<double*>(st.take((size_t)m * 32));
    for (int i = 0; i < m; ++i) {
        h[4 * i] = p1[2 * i];
        h[4 * i + 1] = p1[2 * i + 1];
        h[4 * i + 2] = p2[2 * i];
        h[4 * i + 3] = p2[2 * i + 1];
    }
    HIP_TRY(st.send(*dpts, reinterpret_cast<const uint8_t*>(h), (size_t)m * 32));
    return DVO_OK;
}

int dvo_find_essential_mat(dvo_ctx* ctx, const double* p1, const double* p2, int m, const double* K, double prob,
                           double threshold, int max_iters, double* E, int* e_rows, uint8_t* mask) {
    if (!ctx || !K || !E || !e_rows) return DVO_EINVAL;
    *e_rows = 0;
    if (m < 0 || (m > 0 && (!p1 || !p2))) return fail(ctx, DVO_EINVAL, "bad point arrays");
    if (!(prob > 0 && prob < 1)) return fail(ctx, DVO_EINVAL, "prob must be in (0, 1)");
    if (m < 5) return fail(ctx, DVO_EFEWPTS, "fewer than 5 correspondences");
    HIP_TRY(hipSetDevice(ctx->device));
    void *dpts, *dn, *dmod, *dE, *dinfo, *dmask, *dnmod, *dcnt, *dsub, *drs, *drec, *doff, *dctl, *dlist, *daoff, *dsoff;
    int rc;
    const size_t hc = (size_t)(max_iters > 1 ? max_iters : 1);
    Staging st;
    if ((rc = staging(ctx, Staging::round((size_t)m * 32) + Staging::round(16) + Staging::round(90 * 8) +
                               Staging::round((size_t)m), ctx->stream, &st)))
        return rc;
    if ((rc = scratch(ctx, 6, (size_t)m * 32, &dn)) ||
        (rc = scratch(ctx, 7, hc * 90 * 8, &dmod)) || (rc = scratch(ctx, 8, 90 * 8, &dE)) ||
        (rc = scratch(ctx, 9, 16, &dinfo)) || (rc = scratch(ctx, 10, (size_t)m, &dmask)) ||
        (rc = scratch(ctx, 16, hc * 4, &dnmod)) || (rc = scratch(ctx, 17, hc * 40, &dcnt)) ||
        (rc = scratch(ctx, 18, hc * 20, &dsub)) || (rc = scratch(ctx, 19, sizeof(RansacState), &drs)) ||
        (rc = scratch(ctx, 21, ((hc + 63) / 64) * 128 * 64 * 8, &drec)) || (rc = scratch(ctx, 22, 8, &doff)) ||
        (rc = scratch(ctx, 23, 4 * (2 + kDkMaxPasses), &dctl)) || (rc = scratch(ctx, 24, hc * 8, &dlist)) ||
        (rc = scratch(ctx, 62, 8, &daoff)) || (rc = scratch(ctx, 63, 8, &dsoff)) ||
        (rc = upload_points(ctx, st, p1, p2, m, &dpts)))
        return rc;
    GeomArgs g{};
    g.pts_d = (const double*)dpts;
    g.m_const = m;
    g.pts_stride = m;
    g.fx = K[0];
    g.fy = K[4];
    g.cx = K[2];
    g.cy = K[5];
    g.prob = prob;
    g.threshold = threshold;
    g.max_iters = max_iters;
    g.npts = (double*)dn;
    g.models = (double*)dmod;
    g.nmod = (int32_t*)dnmod;
    g.cnt = (int32_t*)dcnt;
    g.subsets = (int32_t*)dsub;
    g.rs = (RansacState*)drs;
    g.fprec = (double*)drec;
    g.dk_off = (int32_t*)doff;
    g.a_off = (int32_t*)daoff;
    g.s_off = (int32_t*)dsoff;
    g.dk_ctl = (int32_t*)dctl;
    g.dk_list = (int32_t*)dlist;
    g.dk_list_cap = (int64_t)hc;
    g.hyp_cap = (int)hc;
    g.E = (double*)dE;
    g.info = (int32_t*)dinfo;
    g.mask = (uint8_t*)dmask;
    HIP_TRY(launch_geometry_args(g, 1, kStageNormalize | kStageRansac | kStageOneRound, ctx->stream));
    uint8_t *hinfo, *hE, *hmask = nullptr;
    HIP_TRY(st.get(dinfo, 16, &hinfo));
    HIP_TRY(st.get(dE, 90 * 8, &hE));  // every row the kernel may write (<= 10 models)
    if (mask) HIP_TRY(st.get(dmask, (size_t)m, &hmask));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int info[4];
    std::memcpy(info, hinfo, sizeof(info));
    if (info[3] != DVO_OK) return fail(ctx, info[3], "findEssentialMat: no model (E is empty)");
    *e_rows = info[0];
    std::memcpy(E, hE, sizeof(double) * 3 * info[0]);
    if (mask) std::memcpy(mask, hmask, (size_t)m);
    return DVO_OK;
}

int dvo_recover_pose(dvo_ctx* ctx, const double* E, int e_rows, const double* p1, const double* p2, int m,
                     const double* K, double dist_thresh, const uint8_t* mask_in, double* R, double* t,
                     uint8_t* mask_out, int* good) {
    if (!ctx || !E || !K || !R || !t || !good) return DVO_EINVAL;
    if (e_rows != 3) return fail(ctx, DVO_EINVAL, "recoverPose: E must be 3x3 (decomposeEssentialMat reshape)");
    if (m < 0 || (m > 0 && (!p1 || !p2))) return fail(ctx, DVO_EINVAL, "bad point arrays");
    HIP_TRY(hipSetDevice(ctx->device));
    void *dpts, *dn, *dE, *dinfo, *dRt, *dgood, *dpick, *dpm, *dmin = nullptr;
    int rc;
    const int mm = m > 0 ? m : 1;
    Staging st;
    if ((rc = staging(ctx, Staging::round((size_t)m * 32) + Staging::round((size_t)m) + 2 * Staging::round(96) +
                               Staging::round(16) * 3 + Staging::round((size_t)m * 4), ctx->stream, &st)))
        return rc;
    if ((rc = scratch(ctx, 6, (size_t)mm * 32, &dn)) ||
        (rc = scratch(ctx, 8, 90 * 8, &dE)) || (rc = scratch(ctx, 9, 16, &dinfo)) ||
        (rc = scratch(ctx, 11, 12 * 8, &dRt)) || (rc = scratch(ctx, 12, 8, &dgood)) ||
        (rc = scratch(ctx, 13, 8, &dpick)) || (rc = scratch(ctx, 14, (size_t)mm * 4, &dpm)))
        return rc;
    if (mask_in && (rc = scratch(ctx, 15, (size_t)mm, &dmin))) return rc;
    void *dpP, *dpc;
    if ((rc = scratch(ctx, 25, 72 * sizeof(double), &dpP)) || (rc = scratch(ctx, 26, 5 * sizeof(int32_t), &dpc)) ||
        (rc = upload_points(ctx, st, p1, p2, m, &dpts)))
        return rc;
    if (mask_in) HIP_TRY(st.put(dmin, mask_in, (size_t)m));
    const int info[4] = {3, 0, 0, DVO_OK};
    HIP_TRY(st.put(dE, E, 9 * sizeof(double)));
    HIP_TRY(st.put(dinfo, info, sizeof(info)));
    GeomArgs g{};
    g.pts_d = (const double*)dpts;
    g.m_const = m;
    g.pts_stride = mm;
    g.fx = K[0];
    g.fy = K[4];
    g.cx = K[2];
    g.cy = K[5];
    g.dist_thresh = dist_thresh;
    g.npts = (double*)dn;
    g.E = (double*)dE;
    g.info = (int32_t*)dinfo;
    g.mask_in = (const uint8_t*)dmin;
    g.Rt = (double*)dRt;
    g.good = (int32_t*)dgood;
    g.pick = (int32_t*)dpick;
    g.pose_mask = (uint8_t*)dpm;
    g.pose_P = (double*)dpP;
    g.pose_cnt = (int32_t*)dpc;
    HIP_TRY(launch_geometry_args(g, 1, kStageNormalize | kStagePose, ctx->stream));
    uint8_t *hRt, *hgood, *hpick, *hpm = nullptr;
    HIP_TRY(st.get(dRt, 12 * sizeof(double), &hRt));
    HIP_TRY(st.get(dgood, sizeof(int), &hgood));
    HIP_TRY(st.get(dpick, sizeof(int), &hpick));
    if (mask_out && m > 0) HIP_TRY(st.get(dpm, (size_t)m * 4, &hpm));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::memcpy(R, hRt, 9 * sizeof(double));
    std::memcpy(t, hRt + 9 * sizeof(double), 3 * sizeof(double));
    int pick = 0;
    std::memcpy(good, hgood, sizeof(int));
    std::memcpy(&pick, hpick, sizeof(int));
    if (hpm)
        for (int i = 0; i < m; ++i) mask_out[i] = hpm[(size_t)i * 4 + pick];
    return DVO_OK;
}

int dvo_triangulate_points(dvo_ctx* ctx, const double* P1, const double* P2, const double* x1, const double* x2,
                           int k, double* X) {
    if (!ctx || !P1 || !P2 || !X || k < 0 || (k > 0 && (!x1 || !x2))) return DVO_EINVAL;
    if (k == 0) return DVO_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    void *dP, *dx, *dX;
    int rc;
    if ((rc = scratch(ctx, 16, 24 * 8, &dP)) || (rc = scratch(ctx, 17, (size_t)k * 32, &dx)) ||
        (rc = scratch(ctx, 18, (size_t)k * 32, &dX)))
        return rc;
    Staging st;
    if ((rc = staging(ctx, Staging::round(24 * 8) + Staging::round((size_t)k * 32) * 2, ctx->stream, &st))) return rc;
    uint8_t* hP = st.take(24 * 8);
    std::memcpy(hP, P1, 12 * sizeof(double));
    std::memcpy(hP + 12 * sizeof(double), P2, 12 * sizeof(double));
    HIP_TRY(st.send(dP, hP, 24 * 8));
    uint8_t* hx = st.take((size_t)k * 32);
    std::memcpy(hx, x1, (size_t)k * 16);
    std::memcpy(hx + (size_t)k * 16, x2, (size_t)k * 16);
    HIP_TRY(st.send(dx, hx, (size_t)k * 32));
    HIP_TRY(launch_triangulate((const double*)dP, (const double*)dx, k, (double*)dX, ctx->stream));
    uint8_t* hX;
    HIP_TRY(st.get(dX, (size_t)k * 32, &hX));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::memcpy(X, hX, (size_t)k * 32);
    return DVO_OK;
}

// ---------------------------------------------------------------------------
int dvo_test_retain_best(dvo_ctx* ctx, const float* resp, int n, int n_points, int depth, int semantics,
                         int32_t* perm, int* k_out) {
    if (!ctx || !resp || !perm || !k_out || n < 0) return DVO_EINVAL;
    if (semantics != DVO_OPENCV_4X && semantics != DVO_OPENCV_32) return fail(ctx, DVO_EINVAL, "bad semantics");
    HIP_TRY(hipSetDevice(ctx->device));
    void *dv, *dk, *dt, *dkk;
    int rc;
    if ((rc = scratch(ctx, 20, (size_t)(n + 1) * 4, &dv)) || (rc = scratch(ctx, 21, (size_t)(n + 1) * 4, &dk)) ||
        (rc = scratch(ctx, 22, (size_t)(2 * n + 2) * 4, &dt)) || (rc = scratch(ctx, 23, 8, &dkk)))
        return rc;
    std::vector<uint32_t> ids(n);
    for (int i = 0; i < n; ++i) ids[i] = (uint32_t)i;
    if (n) {
        HIP_TRY(hipMemcpy(dv, resp, (size_t)n * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(dk, ids.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    }
    HIP_TRY(launch_test_retain_best((float*)dv, (uint32_t*)dk, (int32_t*)dt, n, n_points, depth, semantics, (int*)dkk,
                                    ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int k = 0;
    HIP_TRY(hipMemcpy(&k, dkk, sizeof(int), hipMemcpyDeviceToHost));
    *k_out = k;
    if (k) HIP_TRY(hipMemcpy(perm, dk, (size_t)k * 4, hipMemcpyDeviceToHost));
    return DVO_OK;
}

int dvo_test_update_num_iters(dvo_ctx* ctx, double p, const double* ep, int n, int model_points, int max_iters,
                              int32_t* out) {
    if (!ctx || !ep || !out || n < 0) return DVO_EINVAL;
    if (n == 0) return DVO_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    void *de, *dout;
    int rc;
    if ((rc = scratch(ctx, 24, (size_t)n * 8, &de)) || (rc = scratch(ctx, 25, (size_t)n * 4, &dout))) return rc;
    HIP_TRY(hipMemcpy(de, ep, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_TRY(launch_test_update_num_iters(p, (const double*)de, n, model_points, max_iters, (int32_t*)dout, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost));
    return DVO_OK;
}

int dvo_test_ransac_subsets(dvo_ctx* ctx, int m, int n, int32_t* idx) {
    if (!ctx || !idx || m < 6 || n < 1) return DVO_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    void *drs, *dsub;
    int rc;
    if ((rc = scratch(ctx, 19, sizeof(RansacState), &drs)) || (rc = scratch(ctx, 18, (size_t)n * 20, &dsub))) return rc;
    RansacState S{};
    S.rng = ~0ull;
    S.m = m;
    S.niters = n;  // round 2 of the sampler covers [h1, niters) = [0, n)
    HIP_TRY(hipMemcpyAsync(drs, &S, sizeof(S), hipMemcpyHostToDevice, ctx->stream));
    GeomArgs g{};
    g.rs = (RansacState*)drs;
    g.subsets = (int32_t*)dsub;
    g.hyp_cap = n;
    g.m_const = m;
    HIP_TRY(launch_test_ransac_sample(g, ctx->stream));
    HIP_TRY(hipMemcpyAsync(idx, dsub, (size_t)n * 20, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DVO_OK;
}

int dvo_test_ransac_replay(dvo_ctx* ctx, const int32_t* nmod, const int32_t* cnt, int n, int m, double prob,
                           int max_iters, int32_t* out) {
    if (!ctx || !nmod || !cnt || !out || n < 1 || m < 6) return DVO_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    void *drs, *dn, *dc;
    int rc;
    if ((rc = scratch(ctx, 19, sizeof(RansacState), &drs)) || (rc = scratch(ctx, 16, (size_t)n * 4, &dn)) ||
        (rc = scratch(ctx, 17, (size_t)n * 40, &dc)))
        return rc;
    RansacState S{};
    S.m = m;
    S.niters = max_iters > 1 ? max_iters : 1;
    S.h0 = 0;
    S.h1 = n < S.niters ? n : S.niters;
    S.best_h = S.best_i = -1;
    HIP_TRY(hipMemcpyAsync(drs, &S, sizeof(S), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dn, nmod, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dc, cnt, (size_t)n * 40, hipMemcpyHostToDevice, ctx->stream));
    GeomArgs g{};
    g.rs = (RansacState*)drs;
    g.nmod = (int32_t*)dn;
    g.cnt = (int32_t*)dc;
    g.hyp_cap = n;
    g.prob = prob;
    HIP_TRY(launch_test_ransac_replay(g, ctx->stream));
    HIP_TRY(hipMemcpyAsync(&S, drs, sizeof(S), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    out[0] = S.iter;
    out[1] = S.niters;
    out[2] = S.maxgood;
    out[3] = S.best_h;
    out[4] = S.best_i;
    return DVO_OK;
}

int dvo_test_five_point(dvo_ctx* ctx, const double* q1, const double* q2, double* models, int* n) {
    if (!ctx || !q1 || !q2 || !models || !n) return DVO_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    void *dq, *dm, *dn;
    int rc;
    if ((rc = scratch(ctx, 26, 20 * 8, &dq)) || (rc = scratch(ctx, 27, 90 * 8, &dm)) || (rc = scratch(ctx, 28, 8, &dn)))
        return rc;
    double q[20];
    for (int i = 0; i < 5; ++i) {
        q[4 * i] = q1[2 * i];
        q[4 * i + 1] = q1[2 * i + 1];
        q[4 * i + 2] = q2[2 * i];
        q[4 * i + 3] = q2[2 * i + 1];
    }
    HIP_TRY(hipMemcpy(dq, q, sizeof(q), hipMemcpyHostToDevice));
    HIP_TRY(launch_test_five_point((const double*)dq, (double*)dm, (int*)dn, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(n, dn, sizeof(int), hipMemcpyDeviceToHost));
    if (*n > 0) HIP_TRY(hipMemcpy(models, dm, (size_t)*n * 72, hipMemcpyDeviceToHost));
    return DVO_OK;
}

int dvo_test_sampson(dvo_ctx* ctx, const double* E, const double* pts, int n, float t, int8_t* dec,
                     uint8_t* exact) {
    if (!ctx || !E || n < 0 || (n > 0 && (!pts || !dec || !exact))) return DVO_EINVAL;
    if (n == 0) return DVO_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    void *dE, *dp, *dd, *dx;
    int rc;
    if ((rc = scratch(ctx, 26, 9 * 8, &dE)) || (rc = scratch(ctx, 27, (size_t)n * 32, &dp)) ||
        (rc = scratch(ctx, 28, (size_t)n, &dd)) || (rc = scratch(ctx, 29, (size_t)n, &dx)))
        return rc;
    HIP_TRY(hipMemcpy(dE, E, 9 * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dp, pts, (size_t)n * 32, hipMemcpyHostToDevice));
    HIP_TRY(launch_test_sampson((const double*)dE, (const double*)dp, n, t, (int8_t*)dd, (uint8_t*)dx, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(dec, dd, (size_t)n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(exact, dx, (size_t)n, hipMemcpyDeviceToHost));
    return DVO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Image pre-processing: cv.getOptimalNewCameraMatrix / cv.undistort
// (visual_odometry_v3.py:110-135).
namespace {

int load_dist12(dvo_ctx* ctx, const double* dist, int ndist, double* k) {
    for (int i = 0; i < 12; ++i) k[i] = 0.0;
    if (ndist < 0 || (ndist > 0 && !dist)) return fail(ctx, DVO_EINVAL, "bad distortion coefficients");
    if (!(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8 || ndist == 12))
        return fail(ctx, DVO_EINVAL, "distortion must have 4, 5, 8 or 12 coefficients (tilt models unsupported)");
    for (int i = 0; i < ndist; ++i) k[i] = dist[i];
    return DVO_OK;
}

// undistort.dispatch.cpp cvUndistortPointsInternal (R = P = I, 5 iterations),
// float points in and out.
void undistort_points_f(float* pts, int n, const double* A, const double* k) {
    const double fx = A[0], fy = A[4], ifx = 1. / fx, ify = 1. / fy, cx = A[2], cy = A[5];
    for (int i = 0; i < n; ++i) {
        double x = pts[2 * i], y = pts[2 * i + 1];
        const double u = x, v = y;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; ++j) {
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            if (icdist < 0) {
                x = (u - cx) * ifx;
                y = (v - cy) * ify;
                break;
            }
            const double dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - dx) * icdist;
            y = (y0 - dy) * icdist;
        }
        const double ww = 1. / (0. * x + 0. * y + 1.);
        pts[2 * i] = (float)((1. * x + 0. * y + 0.) * ww);
        pts[2 * i + 1] = (float)((0. * x + 1. * y + 0.) * ww);
    }
}

// Mat::inv(DECOMP_LU) of a 3x3 (LU with partial pivoting on [A | I]).
bool inv3(const double* M, double* out) {
    double A[9], b[9];
    std::memcpy(A, M, sizeof(A));
    for (int i = 0; i < 9; ++i) b[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 3; i++) {
        int k = i;
        for (int j = i + 1; j < 3; j++)
            if (std::fabs(A[j * 3 + i]) > std::fabs(A[k * 3 + i])) k = j;
        if (std::fabs(A[k * 3 + i]) < DBL_EPSILON * 100) return false;
        if (k != i) {
            for (int j = i; j < 3; j++) std::swap(A[i * 3 + j], A[k * 3 + j]);
            for (int j = 0; j < 3; j++) std::swap(b[i * 3 + j], b[k * 3 + j]);
        }
        const double d = -1 / A[i * 3 + i];
        for (int j = i + 1; j < 3; j++) {
            const double alpha = A[j * 3 + i] * d;
            for (int c = i + 1; c < 3; c++) A[j * 3 + c] += alpha * A[i * 3 + c];
            for (int c = 0; c < 3; c++) b[j * 3 + c] += alpha * b[i * 3 + c];
        }
    }
    for (int i = 2; i >= 0; i--)
        for (int j = 0; j < 3; j++) {
            double s = b[i * 3 + j];
            for (int k = i + 1; k < 3; k++) s -= A[i * 3 + k] * b[k * 3 + j];
            b[i * 3 + j] = s / A[i * 3 + i];
        }
    std::memcpy(out, b, sizeof(b));
    return true;
}

}  // namespace

struct dvo_undistort {
    dvo_ctx* ctx = nullptr;
    UndistortGeom U{};
    double* d_ir = nullptr;
    int16_t* d_xy = nullptr;
    uint16_t* d_frac = nullptr;
};

int dvo_get_optimal_new_camera_matrix(const double* K, const double* dist, int ndist, int w, int h, double alpha,
                                      int new_w, int new_h, double* newK) {
    if (!K || !newK || w <= 0 || h <= 0) return DVO_EINVAL;
    double k[12];
    if (load_dist12(nullptr, dist, ndist, k)) return DVO_EINVAL;
    if (new_w * new_h == 0) {
        new_w = w;
        new_h = h;
    }
    // calibration.cpp icvGetRectangles: a 9 x 9 grid over the image, undistorted
    const int N = 9;
    float pts[2 * N * N];
    for (int y = 0, i = 0; y < N; y++)
        for (int x = 0; x < N; x++, i++) {
            pts[2 * i] = (float)x * w / (N - 1);
            pts[2 * i + 1] = (float)y * h / (N - 1);
        }
    undistort_points_f(pts, N * N, K, k);
    float iX0 = -FLT_MAX, iX1 = FLT_MAX, iY0 = -FLT_MAX, iY1 = FLT_MAX;
    float oX0 = FLT_MAX, oX1 = -FLT_MAX, oY0 = FLT_MAX, oY1 = -FLT_MAX;
    for (int y = 0, i = 0; y < N; y++)
        for (int x = 0; x < N; x++, i++) {
            const float px = pts[2 * i], py = pts[2 * i + 1];
            oX0 = std::min(oX0, px);
            oX1 = std::max(oX1, px);
            oY0 = std::min(oY0, py);
            oY1 = std::max(oY1, py);
            if (x == 0) iX0 = std::max(iX0, px);
            if (x == N - 1) iX1 = std::min(iX1, px);
            if (y == 0) iY0 = std::max(iY0, py);
            if (y == N - 1) iY1 = std::min(iY1, py);
        }
    const float in_w = iX1 - iX0, in_h = iY1 - iY0, ou_w = oX1 - oX0, ou_h = oY1 - oY0;
    std::memcpy(newK, K, 9 * sizeof(double));
    const double fx0 = (new_w - 1) / in_w, fy0 = (new_h - 1) / in_h, cx0 = -fx0 * iX0, cy0 = -fy0 * iY0;
    const double fx1 = (new_w - 1) / ou_w, fy1 = (new_h - 1) / ou_h, cx1 = -fx1 * oX0, cy1 = -fy1 * oY0;
    newK[0] = fx0 * (1 - alpha) + fx1 * alpha;
    newK[4] = fy0 * (1 - alpha) + fy1 * alpha;
    newK[2] = cx0 * (1 - alpha) + cx1 * alpha;
    newK[5] = cy0 * (1 - alpha) + cy1 * alpha;
    return DVO_OK;
}

int dvo_undistort_create(dvo_ctx* ctx, const double* K, const double* dist, int ndist, const double* newK, int w,
                         int h, dvo_undistort** out) {
    if (!ctx || !K || !out) return DVO_EINVAL;
    *out = nullptr;
    if (w < 2 || h < 2 || w >= 32768 || h >= 32768) return fail(ctx, DVO_EINVAL, "image size out of range");
    auto u = std::make_unique<dvo_undistort>();
    u->ctx = ctx;
    UndistortGeom& U = u->U;
    int rc = load_dist12(ctx, dist, ndist, U.dist);
    if (rc) return rc;
    U.w = w;
    U.h = h;
    std::memcpy(U.K, K, sizeof(U.K));
    // cv::undistort: stripes of min(max(1, 4096 / cols), rows) rows, principal
    // point of new_K shifted by the stripe's first row, one LU inverse each
    U.stripe = std::min(std::max(1, (1 << 12) / w), h);
    const int nstripes = (h + U.stripe - 1) / U.stripe;
    std::vector<double> ir((size_t)nstripes * 9);
    double Ar[9];
    std::memcpy(Ar, newK ? newK : K, sizeof(Ar));
    const double v0 = Ar[5];
    for (int s = 0; s < nstripes; ++s) {
        Ar[5] = v0 - (double)(s * U.stripe);
        if (!inv3(Ar, &ir[(size_t)s * 9])) return fail(ctx, DVO_EINVAL, "new camera matrix is singular");
    }
    HIP_TRY(hipSetDevice(ctx->device));
    bool ok = hipMalloc(&u->d_ir, ir.size() * sizeof(double)) == hipSuccess &&
              hipMalloc(&u->d_xy, (size_t)w * h * 2 * sizeof(int16_t)) == hipSuccess &&
              hipMalloc(&u->d_frac, (size_t)w * h * sizeof(uint16_t)) == hipSuccess;
    if (ok) ok = hipMemcpy(u->d_ir, ir.data(), ir.size() * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    if (ok) ok = launch_undistort_map(U, u->d_ir, u->d_xy, u->d_frac, ctx->stream) == hipSuccess;
    if (ok) ok = hipStreamSynchronize(ctx->stream) == hipSuccess;
    if (!ok) {
        hipFree(u->d_ir);
        hipFree(u->d_xy);
        hipFree(u->d_frac);
        return fail(ctx, DVO_EHIP, "undistort map construction failed");
    }
    *out = u.release();
    return DVO_OK;
}

void dvo_undistort_destroy(dvo_undistort* u) {
    if (!u) return;
    hipSetDevice(u->ctx->device);
    hipFree(u->d_ir);
    hipFree(u->d_xy);
    hipFree(u->d_frac);
    delete u;
}

int dvo_undistort_apply(dvo_undistort* u, const uint8_t* d_src, int n, int64_t src_frame_stride, int src_pitch,
                        uint8_t* d_dst, int64_t dst_frame_stride, int dst_pitch, void* hip_stream) {
    if (!u) return DVO_EINVAL;
    dvo_ctx* ctx = u->ctx;
    if (n < 0 || (n > 0 && (!d_src || !d_dst)) || src_pitch < u->U.w || dst_pitch < u->U.w)
        return fail(ctx, DVO_EINVAL, "bad frame buffers");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    HIP_TRY(launch_undistort_remap(u->U, u->d_xy, u->d_frac, d_src, n, src_frame_stride, src_pitch, d_dst,
                                   dst_frame_stride, dst_pitch, s));
    return DVO_OK;
}

int dvo_undistort_get_map(dvo_undistort* u, int16_t* xy, uint16_t* frac) {
    if (!u || !xy || !frac) return DVO_EINVAL;
    dvo_ctx* ctx = u->ctx;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpy(xy, u->d_xy, (size_t)u->U.w * u->U.h * 2 * sizeof(int16_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(frac, u->d_frac, (size_t)u->U.w * u->U.h * sizeof(uint16_t), hipMemcpyDeviceToHost));
    return DVO_OK;
}

int dvo_undistort_image(dvo_undistort* u, const uint8_t* img, int stride, uint8_t* out, int out_stride) {
    if (!u || !img || !out) return DVO_EINVAL;
    dvo_ctx* ctx = u->ctx;
    const int w = u->U.w, h = u->U.h;
    if (stride < w || out_stride < w) return fail(ctx, DVO_EINVAL, "bad strides");
    HIP_TRY(hipSetDevice(ctx->device));
    void *dsrc, *ddst;
    int rc;
    const int pw = (w + 15) & ~15;
    if ((rc = scratch(ctx, 24, (size_t)pw * h, &dsrc)) || (rc = scratch(ctx, 25, (size_t)pw * h, &ddst))) return rc;
    HIP_TRY(hipMemcpy2DAsync(dsrc, pw, img, stride, w, h, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_undistort_remap(u->U, u->d_xy, u->d_frac, (const uint8_t*)dsrc, 1, 0, pw, (uint8_t*)ddst, 0, pw,
                                   ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(out, out_stride, ddst, pw, w, h, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return DVO_OK;
}

int dvo_stream_process_undistorted(dvo_stream* s, dvo_undistort* u, const uint8_t* d_frames, int n_frames,
                                   int64_t frame_stride, int stride, dvo_pair_record* d_records) {
    if (!s || !u) return DVO_EINVAL;
    dvo_ctx* ctx = s->ctx;
    if (u->U.w != s->cfg.width || u->U.h != s->cfg.height) return fail(ctx, DVO_EINVAL, "undistort size != stream size");
    if (n_frames < 1 || n_frames > s->cfg.max_frames) return fail(ctx, DVO_EINVAL, "n_frames out of range");
    if (!d_frames || stride < s->cfg.width) return fail(ctx, DVO_EINVAL, "bad frame buffer");
    if (n_frames > 1 && !d_records) return fail(ctx, DVO_EINVAL, "null records");
    HIP_TRY(hipSetDevice(ctx->device));
    const int pw = frame_pitch(s);
    const int64_t fs = (int64_t)pw * s->cfg.height;
    HIP_TRY(launch_undistort_remap(u->U, u->d_xy, u->d_frac, d_frames, n_frames, frame_stride, stride, s->d_frames, fs,
                                   pw, s->hs));
    return run_stream(s, s->d_frames, n_frames, fs, pw, d_records, false);
}
