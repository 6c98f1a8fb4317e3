// ORB detect-and-compute for gfx950: the MI355X replacement of
// cv::ORB::detectAndCompute as called at scripts/visual_odometry_v3.py:373
// (cv.ORB_create() defaults chosen at v3:96).  Batched: every launch covers all
// frames of a stream batch (grid.y / grid.z = frame), so one batch of F frames
// runs 7 resize launches + 6 detect/describe launches regardless of F.
//
// Stages (DESIGN.md §4 lists the roofline of each):
//   resize_level_kernel   INTER_LINEAR_EXACT 8-bit fixed point, level l-1 -> l
//   blur_kernel           GaussianBlur 7x7 sigma 2, 8-bit fixed-point separable, of every level:
//                         only for dvo_stream_get_pyramid(blurred); describe_kernel blurs
//                         the pixels its own windows sample
//   fast_strip_kernel     FAST-9/16 + strict 3x3 NMS + border cut + per-row
//                         compaction, one column strip of one level per workgroup
//   select_fast_kernel    KeyPointsFilter::retainBest(2n) by FAST score: exact
//                         emulation of libstdc++ nth_element + partition
//   harris_kernel         HarrisResponses(blockSize 7, k 0.04)
//   select_harris_kernel  retainBest(n) by Harris response
//   describe_kernel       ICAngles + pt scaling + GaussianBlur of the 39 x 44 sample window
//                         + rBRIEF-256, one wave per keypoint
#include "dvo_internal.h"

#include <climits>
#include <type_traits>

namespace dvo {

namespace {

__constant__ int8_t c_pattern[256 * 4] = {
#include "../../data/orb_bit_pattern_31.inc"
};
// the same points as floats (x0, y0, x1, y1 per pair): describe_kernel's lanes load theirs as float4s
// instead of converting bytes per keypoint
__constant__ __attribute__((aligned(16))) float c_pattern_f[256 * 4] = {
#include "../../data/orb_bit_pattern_31.inc"
};

// ICAngles u_max for halfPatchSize 15 (orb.cpp computeKeyPoints): cvRound of
// sqrt(225 - v^2) for v <= 11, then the symmetry fix-up; pinned by a test.
constexpr int c_umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
// describe_kernel's ICAngles moments from whole LDS words, two lanes per window row (words 0..4
// and 5..9 of the row's 9; word 9 weighs nothing), v_dot4_u32_u8 against per-(alignment, row,
// word) weight words: byte weight u + 15 (in [0, 30]) inside the disk |u| <= umax(|v|), 0
// outside, and a 0/1 word for the plain sum.  m10 = sum (u + 15) I - 15 sum I, m01 = v sum I per
// row; integer sums, so the same m10 / m01 as orb.cpp's per-pixel loop (round 4: 6.36 -> 5.67 ms
// one-stream, profiles/r04n_ab_describe_ic.txt).  o = (kx - 15) & 3: the keypoint column's byte offset in
// the row's first word minus 15 (the window starts at the aligned (kx - 15) & ~3).
struct IcTable {
    uint32_t w[4][32][10][2];  // [o][row][word] = {weights u + 15, ones}; row 31 is the idle lanes' zeros
};
constexpr IcTable ic_table() {
    IcTable t{};
    for (int o = 0; o < 4; ++o)
        for (int r = 0; r < 31; ++r)
            for (int w = 0; w < 9; ++w) {
                uint32_t wu = 0, w1 = 0;
                for (int b = 0; b < 4; ++b) {
                    const int u = 4 * w + b - 15 - o, v = r - 15;
                    const int au = u < 0 ? -u : u, av = v < 0 ? -v : v;
                    if (au <= c_umax[av]) {
                        wu |= (uint32_t)(u + 15) << (8 * b);
                        w1 |= 1u << (8 * b);
                    }
                }
                t.w[o][r][w][0] = wu;
                t.w[o][r][w][1] = w1;
            }
    return t;
}
__constant__ IcTable c_ictab = ic_table();

// FAST 16-pixel Bresenham circle (dx, dy), fast.cpp makeOffsets.
constexpr int kCdx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kCdy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// ------------------------------------------------------------------------
// Level l from level l-1: resize.cpp resize_bitExact<uchar, interpolationLinear>
// (INTER_LINEAR_EXACT, 8-bit fixed point).  The per-column / per-row
// coefficients are computed once per plan on the host (api.cpp resize_coefs,
// same double arithmetic) and read from a table.  A lane produces 4 adjacent
// output pixels (one word) on kRsR consecutive output rows of its wave: the
// column taps come from one 16-byte table load, the row taps from scalar loads
// (rows are wave-uniform), and all source words of the kRsR rows are issued as
// buffer loads before any arithmetic (row offset in the scalar offset).  The
// source bytes of 4 output columns span at most 12 bytes from an aligned base
// (level ratio <= 1.5); wider ratios take a bytewise path.
constexpr int kRsR = 4;

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

__device__ __forceinline__ uint32_t byte_of(const uint32_t* w, int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFF; }

__global__ __launch_bounds__(256) void resize_level_kernel(StreamParams P, int l) {
    const int f = blockIdx.z;
    const LevelGeom& S = P.plan.L[l - 1];
    const LevelGeom& D = P.plan.L[l];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * 256 + 4 * lane;
    const int dy0 = (blockIdx.y * 4 + wid) * kRsR;
    if (dy0 >= D.h) return;
    const uint8_t* src = level_ptr(P, f, l - 1);
    const int sp = level_pitch(P, l - 1);
    uint8_t* dst = P.buf.pyr + (int64_t)f * P.plan.pyr_stride + D.pyr_off;
    // taps: (source index, weight of the next index); clamped positions carry weight 0 (api.cpp)
    const int4 cx = *reinterpret_cast<const int4*>(P.buf.coef + D.xcoef_off + min(x0, ((D.w + 3) & ~3) - 4));
    const int4 cy = *reinterpret_cast<const int4*>(P.buf.coef + D.ycoef_off + dy0);  // wave-uniform
    const int cxs[4] = {cx.x, cx.y, cx.z, cx.w}, cys[4] = {cy.x, cy.y, cy.z, cy.w};
    int i0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        i0[j] = coef_ofs(cxs[j]);
        c1[j] = coef_c1(cxs[j]);
    }
    const int base = i0[0] & ~3;
    const bool narrow = i0[3] + 1 - base < 12;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, S.h * sp, 0x00020000);
    int ry0[kRsR];
    uint32_t cy1[kRsR];
    uint32_t wa[kRsR][3], wb[kRsR][3];
#pragma unroll
    for (int rr = 0; rr < kRsR; ++rr) {
        ry0[rr] = coef_ofs(cys[rr]);
        cy1[rr] = coef_c1(cys[rr]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // row ry0 + 1 may lie past the level: weight 0, buffer reads 0
            wa[rr][k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, base + 4 * k, ry0[rr] * sp, 0);
            wb[rr][k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, base + 4 * k, (ry0[rr] + 1) * sp, 0);
        }
    }
    const bool full = x0 + 4 <= D.w;
#pragma unroll
    for (int rr = 0; rr < kRsR; ++rr) {
        const int dy = dy0 + rr;
        if (dy >= D.h) break;
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k1 = c1[j], k0 = 256 - k1;
            uint32_t a0, a1, b0, b1;
            if (narrow) {
                a0 = byte_of(wa[rr], i0[j] - base);
                a1 = byte_of(wa[rr], i0[j] + 1 - base);
                b0 = byte_of(wb[rr], i0[j] - base);
                b1 = byte_of(wb[rr], i0[j] + 1 - base);
            } else {  // generic ratio: byte gathers (weight-0 taps read an in-range byte)
                const int i1 = min(i0[j] + 1, S.w - 1), r1 = min(ry0[rr] + 1, S.h - 1);
                a0 = src[(int64_t)ry0[rr] * sp + i0[j]];
                a1 = src[(int64_t)ry0[rr] * sp + i1];
                b0 = src[(int64_t)r1 * sp + i0[j]];
                b1 = src[(int64_t)r1 * sp + i1];
            }
            const uint32_t h0 = k0 * a0 + k1 * a1;
            const uint32_t h1 = k0 * b0 + k1 * b1;
            const uint32_t v = (h0 * (256 - cy1[rr]) + h1 * cy1[rr] + 32768u) >> 16;
            word |= (v > 255 ? 255u : v) << (8 * j);
        }
        uint8_t* drow = dst + (int64_t)dy * D.pitch;
        if (full) {
            *reinterpret_cast<uint32_t*>(drow + x0) = word;
        } else {
            for (int j = 0; j < 4 && x0 + j < D.w; ++j) drow[x0 + j] = (uint8_t)(word >> (8 * j));
        }
    }
}

// LDS-staged variant for level ratios <= 1.25 (ORB's 1.2 pyramid): the
// workgroup's output tile (256 columns x 32 rows) needs at most kRsW source
// words x kRsRows source rows; each wave stages whole source rows with
// coalesced word loads (lane k <- word k), then every lane reads its 3 words
// per source row from LDS.  Same arithmetic as resize_level_kernel.
constexpr int kRsLR = 8;  // output rows per wave (32 per workgroup)
#ifndef DVO_RS_PIN
#define DVO_RS_PIN 1
#endif

constexpr int kRsW = 96, kRsLRows = 44;  // 32 * 1.25 + 2 source rows, padded to a multiple of 4

// 1-D grids of (frame, item) blocks, XCD-grouped: workgroups are dispatched
// round-robin over the 8 XCDs (block b on XCD b & 7), so XCD x takes frames
// x, x + 8, ... and one frame's items run on one XCD at about the same time.
// Neighbouring tiles / strips share the 128-B lines of their halo columns
// through that XCD's L2 instead of each XCD fetching its own copy.
// Grid: nitems * xcd_frames(F) blocks; blocks past the last frame return.
// Batches of fewer than 8 frames (the per-call surface: one frame) keep the plain
// frame-major order, or all of a frame's blocks would land on one XCD.
__host__ __device__ constexpr int xcd_frames(int F) { return F < 8 ? F : (F + 7) & ~7; }
__device__ __forceinline__ int xcd_frame_item(int nitems, int nframes, int& item) {
    if (nframes < 8) {
        const int f = blockIdx.x / nitems;
        item = blockIdx.x - f * nitems;
        return f;
    }
    const int q8 = blockIdx.x >> 3, fq = q8 / nitems;
    item = q8 - fq * nitems;
    return (blockIdx.x & 7) + 8 * fq;
}

// Per-lane constants of one destination word (4 pixels) of the LDS-staged resize: the staged
// source words it reads (wb0 .. wb0 + 2 of a window starting at source column sx0), the byte shift
// of its first tap, and per output pixel j a v_perm selector giving the u16 pair (src[o_j],
// src[o_j + 1]) and the pair of weights (256 - c1, c1) for v_dot2_u32_u16.  The 4 taps of a lane span
// <= 6 bytes at ratio <= 1.25.  x0: the word's first destination column; dw: the destination width;
// maxw: the staged row's word count (lanes past the level's right edge read any in-range words).
struct RsLane {
    int wb0, sh;
    uint32_t sel[4], kw[4];
};
__device__ __forceinline__ RsLane rs_lane(const int32_t* cxt, int x0, int dw, int sx0, int maxw) {
    const int4 cx = *reinterpret_cast<const int4*>(cxt + min(x0, ((dw + 3) & ~3) - 4));
    const int cxs[4] = {cx.x, cx.y, cx.z, cx.w};
    int i0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        i0[j] = coef_ofs(cxs[j]) - sx0;
        c1[j] = coef_c1(cxs[j]);
    }
    RsLane L;
    L.wb0 = min(i0[0] >> 2, maxw - 3);
    const int base = 4 * L.wb0;
    L.sh = min(i0[0] - base, 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t r = (uint32_t)min(max(i0[j] - base - L.sh, 0), 6);
        L.sel[j] = 0x0C000C00u | r | ((r + 1) << 16);
        L.kw[j] = (uint32_t)(256 - c1[j]) | ((uint32_t)c1[j] << 16);
    }
    return L;
}
// One destination word from two staged source rows a (ofs) and b (ofs + 1) and the row weights
// ky = (256 - cy1) | cy1 << 16: h = (256 - c1) s[o] + c1 s[o + 1] <= 65280 per row, then
// h0 (256 - cy1) + h1 cy1 + 2^15 < 2^24, whose byte 2 is the pixel (INTER_LINEAR_EXACT).
__device__ __forceinline__ uint32_t rs_word(const uint32_t* a, const uint32_t* b, const RsLane& L, uint32_t ky) {
    const uint32_t a0 = a[L.wb0], a1 = a[L.wb0 + 1], a2 = a[L.wb0 + 2];
    const uint32_t b0 = b[L.wb0], b1 = b[L.wb0 + 1], b2 = b[L.wb0 + 2];
    const uint32_t alo = __builtin_amdgcn_alignbyte(a1, a0, L.sh), ahi = __builtin_amdgcn_alignbyte(a2, a1, L.sh);
    const uint32_t blo = __builtin_amdgcn_alignbyte(b1, b0, L.sh), bhi = __builtin_amdgcn_alignbyte(b2, b1, L.sh);
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t h0 = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(ahi, alo, L.sel[j])),
                                                   as_u16x2(L.kw[j]), 0u, false);
        const uint32_t h1 = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(bhi, blo, L.sel[j])),
                                                   as_u16x2(L.kw[j]), 0u, false);
        v[j] = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(h1, h0, 0x05040100u)), as_u16x2(ky), 32768u,
                                      false);
    }
    return __builtin_amdgcn_perm(__builtin_amdgcn_perm(v[3], v[2], 0x0C0C0602u),
                                 __builtin_amdgcn_perm(v[1], v[0], 0x0C0C0602u), 0x05040100u);
}
__device__ __forceinline__ uint32_t rs_ky(int c) {
    const uint32_t cy1 = coef_c1(c);
    return (256u - cy1) | (cy1 << 16);
}

// OpenCV 3.2's resize(INTER_LINEAR) taps of one destination word (the 3.2 table, api.cpp
// resize_coefs_32: per column {sx, sx1, a0 | a1 << 16}): the same staged-window selectors as
// rs_lane, the 11-bit weight pair as the dot2 operand (a0, a1 <= 2048).  Past xmax the table has
// sx1 = sx, a1 = 0: the second byte is read and weighted 0.
__device__ __forceinline__ RsLane rs_lane32(const int32_t* cxt, int x0, int dw, int sx0, int maxw) {
    int i0[4];
    uint32_t kw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int4 c = *reinterpret_cast<const int4*>(cxt + 4 * min(x0 + j, dw - 1));
        i0[j] = c.x - sx0;
        kw[j] = (uint32_t)c.z;
    }
    RsLane L;
    L.wb0 = min(i0[0] >> 2, maxw - 3);
    const int base = 4 * L.wb0;
    L.sh = min(i0[0] - base, 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t r = (uint32_t)min(max(i0[j] - base - L.sh, 0), 6);
        L.sel[j] = 0x0C000C00u | r | ((r + 1) << 16);
        L.kw[j] = kw[j];
    }
    return L;
}
// One destination word in 3.2 semantics from staged source rows a (r0) and b (r1) and the row
// weights b0 | b1 << 16: h = a0 s[sx] + a1 s[sx1] (HResizeLinear, exact in 32 bits), then per
// column VResizeLinearVec_32s8u's SSE2 form ((mulhi(h0 >> 4, b0) + mulhi(h1 >> 4, b1) + 2) >> 2)
// before column xs, FixedPtCast<int, uchar, 22> from there (resize_level_ocv32_kernel's arithmetic).
__device__ __forceinline__ uint32_t rs_word32(const uint32_t* a, const uint32_t* b, const RsLane& L, uint32_t ky,
                                              int x0, int xs) {
    const uint32_t a0 = a[L.wb0], a1 = a[L.wb0 + 1], a2 = a[L.wb0 + 2];
    const uint32_t b0 = b[L.wb0], b1 = b[L.wb0 + 1], b2 = b[L.wb0 + 2];
    const uint32_t alo = __builtin_amdgcn_alignbyte(a1, a0, L.sh), ahi = __builtin_amdgcn_alignbyte(a2, a1, L.sh);
    const uint32_t blo = __builtin_amdgcn_alignbyte(b1, b0, L.sh), bhi = __builtin_amdgcn_alignbyte(b2, b1, L.sh);
    const int wy0 = (int)(ky & 0xFFFFu), wy1 = (int)(ky >> 16);
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int h0 = (int)__builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(ahi, alo, L.sel[j])),
                                                   as_u16x2(L.kw[j]), 0u, false);
        const int h1 = (int)__builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(bhi, blo, L.sel[j])),
                                                   as_u16x2(L.kw[j]), 0u, false);
        int v;
        if (x0 + j < xs)
            v = ((((h0 >> 4) * wy0) >> 16) + (((h1 >> 4) * wy1) >> 16) + 2) >> 2;
        else
            v = (int)(((uint32_t)h0 * (uint32_t)wy0 + (uint32_t)h1 * (uint32_t)wy1 + (1u << 21)) >> 22);
        out |= (uint32_t)min(255, max(0, v)) << (8 * j);
    }
    return out;
}

// kOcv32Sem: OpenCV 3.2's INTER_LINEAR pyramid (the 3.2 tables), same staging and tiles.
template <bool kOcv32Sem>
__global__ __launch_bounds__(256) void resize_level_lds_kernel(StreamParams P, int l, int gx) {
    __shared__ uint32_t tile[kRsLRows][kRsW];
    int item;
    const int f = xcd_frame_item(gx * ((P.plan.L[l].h + 4 * kRsLR - 1) / (4 * kRsLR)), P.nframes, item);
    if (f >= P.nframes) return;
    const int by = item / gx, bxi = item - by * gx;
    const LevelGeom& S = P.plan.L[l - 1];
    const LevelGeom& D = P.plan.L[l];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xa = bxi * 256;
    const int x0 = xa + 4 * lane;
    const int ty0 = by * (4 * kRsLR);
    const uint8_t* src = level_ptr(P, f, l - 1);
    const int sp = level_pitch(P, l - 1);
    uint8_t* dst = P.buf.pyr + (int64_t)f * P.plan.pyr_stride + D.pyr_off;
    const int32_t* cxt = kOcv32Sem ? P.buf.coef32 + D.l32_x : P.buf.coef + D.xcoef_off;
    const int32_t* cyt = kOcv32Sem ? P.buf.coef32 + D.l32_y : P.buf.coef + D.ycoef_off;
    // source window of the tile (wave-uniform)
    int sx0, sy0, nr;
    if constexpr (kOcv32Sem) {  // rows already clipped in the table
        sx0 = cxt[4 * xa] & ~3;
        sy0 = cyt[4 * ty0];
        nr = cyt[4 * min(ty0 + 4 * kRsLR - 1, D.h - 1) + 1] - sy0 + 1;
    } else {
        sx0 = coef_ofs(cxt[xa]) & ~3;
        sy0 = coef_ofs(cyt[ty0]);
        nr = min(coef_ofs(cyt[min(ty0 + 4 * kRsLR - 1, D.h - 1)]) + 1, S.h - 1) - sy0 + 1;
    }
#if DVO_RS_PIN
    // the lane's column taps and the wave's row taps are requested before the staging loads, so
    // their latency overlaps it (dy0 is a multiple of 8: a wave with rows reads inside the row
    // table's 8-row padding, an idle wave its last 8 rows)
    const RsLane L = kOcv32Sem ? rs_lane32(cxt, x0, D.w, sx0, kRsW) : rs_lane(cxt, x0, D.w, sx0, kRsW);
    const int dy0 = ty0 + wid * kRsLR;
    const int dyc = min(dy0, ((D.h + 7) & ~7) - 8);
    const int4 cy = *reinterpret_cast<const int4*>(cyt + dyc);
    const int4 cz = *reinterpret_cast<const int4*>(cyt + dyc + 4);
    int4 r32[kOcv32Sem ? kRsLR : 1];  // the 3.2 row table {r0, r1, b0 | b1 << 16} of the wave's rows
    if constexpr (kOcv32Sem) {
#pragma unroll
        for (int rr = 0; rr < kRsLR; ++rr) r32[rr] = *reinterpret_cast<const int4*>(cyt + 4 * min(dy0 + rr, D.h - 1));
    }
#endif
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, S.h * sp, 0x00020000);
    {  // kRsLRows / 4 rows per wave, all loads in flight (rows past nr re-read row nr - 1: unused)
        uint32_t v0[kRsLRows / 4], v1[kRsLRows / 4];
#pragma unroll
        for (int it = 0; it < kRsLRows / 4; ++it) {
            const int soff = (sy0 + min(wid + 4 * it, nr - 1)) * sp;
            v0[it] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, sx0 + 4 * lane, soff, 0);
            v1[it] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, sx0 + 4 * lane + 256, soff, 0);
        }
#if DVO_RS_PIN
        // keep every load in this one batch: the compiler otherwise sinks the first rows' second
        // words into the lane < 32 store branch, a second memory round trip per workgroup
#pragma unroll
        for (int it = 0; it < kRsLRows / 4; ++it) asm volatile("" ::"v"(v1[it]));
#endif
#pragma unroll
        for (int it = 0; it < kRsLRows / 4; ++it) {
            tile[wid + 4 * it][lane] = v0[it];
            if (lane + 64 < kRsW) tile[wid + 4 * it][lane + 64] = v1[it];
        }
    }
#if !DVO_RS_PIN
    // this lane's taps (their latency overlaps the staging)
    const RsLane L = kOcv32Sem ? rs_lane32(cxt, x0, D.w, sx0, kRsW) : rs_lane(cxt, x0, D.w, sx0, kRsW);
    const int dy0 = ty0 + wid * kRsLR;
#endif
    __syncthreads();
    if (dy0 >= D.h) return;
    const bool full = x0 + 4 <= D.w;
    if constexpr (kOcv32Sem) {
#pragma unroll
        for (int rr = 0; rr < kRsLR; ++rr) {
            const int dy = dy0 + rr;
#if DVO_RS_PIN
            if (dy < D.h) {  // (no break: the unrolled loop indexes r32 by constants)
                const int4 cy = r32[rr];
#else
            {
                if (dy >= D.h) break;
                const int4 cy = *reinterpret_cast<const int4*>(cyt + 4 * dy);  // wave-uniform
#endif
                const uint32_t word = rs_word32(tile[cy.x - sy0], tile[cy.y - sy0], L, (uint32_t)cy.z, x0, D.l32_xs);
                uint8_t* drow = dst + (int64_t)dy * D.pitch;
                if (full) {
                    *reinterpret_cast<uint32_t*>(drow + x0) = word;
                } else {
                    for (int j = 0; j < 4 && x0 + j < D.w; ++j) drow[x0 + j] = (uint8_t)(word >> (8 * j));
                }
            }
        }
        return;
    } else {
#if !DVO_RS_PIN
    const int4 cy = *reinterpret_cast<const int4*>(cyt + dy0);  // wave-uniform (table padded to 8 rows)
    const int4 cz = *reinterpret_cast<const int4*>(cyt + dy0 + 4);
#endif
    const int cys[kRsLR] = {cy.x, cy.y, cy.z, cy.w, cz.x, cz.y, cz.z, cz.w};
    static_assert(kRsLR == 8, "two int4 row-coefficient loads");
#pragma unroll
    for (int rr = 0; rr < kRsLR; ++rr) {
        const int dy = dy0 + rr;
        if (dy >= D.h) break;
        const int lr = coef_ofs(cys[rr]) - sy0;
        const int lr1 = min(lr + 1, kRsLRows - 1);  // weight-0 row past the window: any in-range row
        const uint32_t word = rs_word(tile[lr], tile[lr1], L, rs_ky(cys[rr]));
        uint8_t* drow = dst + (int64_t)dy * D.pitch;
        if (full) {
            *reinterpret_cast<uint32_t*>(drow + x0) = word;
        } else {
            for (int j = 0; j < 4 && x0 + j < D.w; ++j) drow[x0 + j] = (uint8_t)(word >> (8 * j));
        }
    }
    }
}

// ------------------------------------------------------------------------
// OpenCV 3.2 semantics (Plan::semantics == kOcv32): ORB's pyramid was
// resize(INTER_LINEAR), 11-bit weights, not INTER_LINEAR_EXACT (oracle/orb.cpp
// resize_linear_32 restates it).  Per-plan tables (api.cpp resize_coefs_32):
// per destination column {sx, sx1, a0 | a1 << 16} (past xmax: sx1 = sx, a0 =
// 2048, a1 = 0, the HResizeLinear tail S[sx] * 2048) and per row {r0, r1,
// b0 | b1 << 16} with the rows already clipped.  One thread per output pixel
// Tiny levels only (ratios past 1.25, where the staged tiles do not fit); the
// pyramid of ORB-sized frames runs through resize_level_lds_kernel<true>.
// The vertical pass takes the SSE2 form below column l32_xs, the scalar
// FixedPtCast form from there on.
__global__ __launch_bounds__(256) void resize_level_ocv32_kernel(StreamParams P, int l) {
    const int f = blockIdx.z;
    const LevelGeom& S = P.plan.L[l - 1];
    const LevelGeom& D = P.plan.L[l];
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= D.w || y >= D.h) return;
    const int4 cx = *reinterpret_cast<const int4*>(P.buf.coef32 + D.l32_x + 4 * x);
    const int4 cy = *reinterpret_cast<const int4*>(P.buf.coef32 + D.l32_y + 4 * y);
    const uint8_t* src = level_ptr(P, f, l - 1);
    const int sp = level_pitch(P, l - 1);
    const uint8_t* s0 = src + (int64_t)cy.x * sp;
    const uint8_t* s1 = src + (int64_t)cy.y * sp;
    const int a0 = cx.z & 0xFFFF, a1 = cx.z >> 16, b0 = cy.z & 0xFFFF, b1 = cy.z >> 16;
    const int h0 = s0[cx.x] * a0 + s0[cx.y] * a1;
    const int h1 = s1[cx.x] * a0 + s1[cx.y] * a1;
    int v;
    if (x < D.l32_xs)  // VResizeLinearVec_32s8u: _mm_mulhi_epi16 on h >> 4, then (t + 2) >> 2
        v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
    else               // FixedPtCast<int, uchar, 22>
        v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    uint8_t* dst = P.buf.pyr + (int64_t)f * P.plan.pyr_stride + D.pyr_off;
    dst[(int64_t)y * D.pitch + x] = (uint8_t)min(255, max(0, v));
}

// ------------------------------------------------------------------------
// GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) with the 8-bit kernel
// {18,34,49,55,49,34,18} over the 49 taps, sum / 2^16 rounded as OpenCV's
// column filter does (oracle/orb.cpp gaussian_blur7): half to even in every
// column up to the last multiple of 4 (its vector op: exact float sum, then
// cvtps2dq), half up, (sum + 2^15) >> 16, in the last w % 4 columns (the
// scalar FixedPtCastEx); saturated.  Half to even is (s + bit16(s)) >> 16
// with s = sum + 2^15 - 1: the two differ only at a tie above an odd value.
// Vertical first, in packed 16-bit lanes: a column sum of 7 bytes is at most
// 255 * 257 = 65535, so each lane keeps its 4 columns as two u16 pairs and
// forms the vertical sums with v_pk_mad_u16 over a rolling 7-row window (one
// word load per input row).  The horizontal taps then come from the
// neighbouring lanes' pairs (DPP wave_shr / wave_shl) through v_dot2_u32_u16.
// A wave covers 62 * 4 = 248 output columns (lanes 0 and 63 are the halo) and
// kBlurR output rows; border columns gather bytes through reflect-101.
__device__ __forceinline__ int refl101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__device__ __forceinline__ uint32_t dpp_from_left(uint32_t v) {  // lane i <- lane i-1 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_from_right(uint32_t v) {  // lane i <- lane i+1 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}
constexpr int kBlurR = kBlurTH / 4;  // output rows per wave

// One wave: kBlurR output rows from row yw, columns x0 .. x0+3 per lane.
// kInside: every lane's 4 columns lie inside the row (one word load per row);
// otherwise each lane gathers its 4 (reflect-101) columns col[0..3] bytewise.
// kSmall: fewer than 4 rows, rows need the general reflect-101 loop.
template <bool kInside, bool kSmall>
__device__ __forceinline__ void blur_wave(const uint8_t* __restrict__ src, int sp, uint8_t* __restrict__ dst,
                                          int dp, int w, int h, int yw, int x0, bool store, int col_base,
                                          uint32_t col_sel) {
    // the lane's 4 columns are all below w & ~3 (half to even) or all in the w % 4 tail (half up)
    const uint32_t he = x0 + 4 <= w ? 1u : 0u;
    const uint32_t R = he ? 0x7FFFu : 0x8000u;
    const u16x2 k18 = {18, 18}, k34 = {34, 34}, k49 = {49, 49}, k55 = {55, 55};
    // all input rows are loaded up front (rows past the bottom are read, reflected, but not stored)
    uint32_t wds[kBlurR + 6];
    // buffer loads: row offset in the scalar offset, column(s) in the vector offset
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, h * sp, 0x00020000);
#pragma unroll
    for (int r = 0; r < kBlurR + 6; ++r) {
        const int y = yw - 3 + r;
        const int ry = kSmall ? refl101(y, h) : min(abs(y), 2 * h - 2 - y);
        if (kInside) {
            wds[r] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, x0, ry * sp, 0);
        } else {  // the lane's 4 reflected columns lie in the 8 bytes at its aligned base (span <= 6)
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, col_base, ry * sp, 0);
            const uint32_t w1 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, col_base + 4, ry * sp, 0);
            wds[r] = __builtin_amdgcn_perm(w1, w0, col_sel);
        }
    }
    u16x2 lo[7], hi[7];
#pragma unroll
    for (int r = 0; r < kBlurR + 6; ++r) {
        const int y = yw - 3 + r;
        const uint32_t wd = wds[r];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            lo[k] = lo[k + 1];
            hi[k] = hi[k + 1];
        }
        lo[6] = as_u16x2(__builtin_amdgcn_perm(0u, wd, 0x0C010C00u));  // (b0, b1)
        hi[6] = as_u16x2(__builtin_amdgcn_perm(0u, wd, 0x0C030C02u));  // (b2, b3)
        if (r < 6) continue;
        const u16x2 a = k18 * (lo[0] + lo[6]) + k34 * (lo[1] + lo[5]) + k49 * (lo[2] + lo[4]) + k55 * lo[3];
        const u16x2 b = k18 * (hi[0] + hi[6]) + k34 * (hi[1] + hi[5]) + k49 * (hi[2] + hi[4]) + k55 * hi[3];
        const uint32_t A = __builtin_bit_cast(uint32_t, a), B = __builtin_bit_cast(uint32_t, b);
        const u16x2 al = as_u16x2(dpp_from_left(A)), bl = as_u16x2(dpp_from_left(B));
        const u16x2 ar = as_u16x2(dpp_from_right(A)), br = as_u16x2(dpp_from_right(B));
        uint32_t s0 = __builtin_amdgcn_udot2(al, (u16x2){0, 18}, R, false);
        s0 = __builtin_amdgcn_udot2(bl, (u16x2){34, 49}, s0, false);
        s0 = __builtin_amdgcn_udot2(a, (u16x2){55, 49}, s0, false);
        s0 = __builtin_amdgcn_udot2(b, (u16x2){34, 18}, s0, false);
        uint32_t s1 = __builtin_amdgcn_udot2(bl, (u16x2){18, 34}, R, false);
        s1 = __builtin_amdgcn_udot2(a, (u16x2){49, 55}, s1, false);
        s1 = __builtin_amdgcn_udot2(b, (u16x2){49, 34}, s1, false);
        s1 = __builtin_amdgcn_udot2(ar, (u16x2){18, 0}, s1, false);
        uint32_t s2 = __builtin_amdgcn_udot2(bl, (u16x2){0, 18}, R, false);
        s2 = __builtin_amdgcn_udot2(a, (u16x2){34, 49}, s2, false);
        s2 = __builtin_amdgcn_udot2(b, (u16x2){55, 49}, s2, false);
        s2 = __builtin_amdgcn_udot2(ar, (u16x2){34, 18}, s2, false);
        uint32_t s3 = __builtin_amdgcn_udot2(a, (u16x2){18, 34}, R, false);
        s3 = __builtin_amdgcn_udot2(b, (u16x2){49, 55}, s3, false);
        s3 = __builtin_amdgcn_udot2(ar, (u16x2){49, 34}, s3, false);
        s3 = __builtin_amdgcn_udot2(br, (u16x2){18, 0}, s3, false);
        s0 += __builtin_amdgcn_ubfe(s0, 16, he);
        s1 += __builtin_amdgcn_ubfe(s1, 16, he);
        s2 += __builtin_amdgcn_ubfe(s2, 16, he);
        s3 += __builtin_amdgcn_ubfe(s3, 16, he);
        // byte 2 of min(s, 2^24 - 1) == min(s >> 16, 255)
        s0 = min(s0, 0xFFFFFFu);
        s1 = min(s1, 0xFFFFFFu);
        s2 = min(s2, 0xFFFFFFu);
        s3 = min(s3, 0xFFFFFFu);
        const uint32_t word = __builtin_amdgcn_perm(__builtin_amdgcn_perm(s3, s2, 0x0C0C0602u),
                                                    __builtin_amdgcn_perm(s1, s0, 0x0C0C0602u), 0x05040100u);
        if (store && y - 3 < h) {
            uint8_t* drow = dst + (int64_t)(y - 3) * dp;
            if (kInside || x0 + 4 <= w) {
                *reinterpret_cast<uint32_t*>(drow + x0) = word;
            } else {
                for (int j = 0; j < 4 && x0 + j < w; ++j) drow[x0 + j] = (uint8_t)(word >> (8 * j));
            }
        }
    }
}

__global__ __launch_bounds__(256) void blur_kernel(StreamParams P) {
    int item;
    const int f = xcd_frame_item(P.plan.total_tiles, P.nframes, item);
    if (f >= P.nframes) return;
    int l = 0;
    while (l + 1 < P.plan.nlevels && item >= P.plan.L[l + 1].tile_base) ++l;
    const LevelGeom& G = P.plan.L[l];
    const int t = item - G.tile_base;
    const int ty = t / G.tiles_x, tx = t - ty * G.tiles_x;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = G.w, h = G.h;
    const int yw = ty * kBlurTH + wid * kBlurR;
    if (yw >= h) return;
    const int xw = tx * kBlurTW - 4;  // column of lane 0
    const int x0 = xw + 4 * lane;
    const uint8_t* src = level_ptr(P, f, l);
    const int sp = level_pitch(P, l);
    uint8_t* dst = blur_ptr(P, f, l);
    const bool store = lane >= 1 && lane <= 62 && x0 < w;
    // border lanes: v_perm selector of the 4 reflect-101 columns from 2 aligned words
    int col[4], cmin = INT_MAX;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        col[k] = refl101(min(x0 + k, w + 2), w);  // columns past w+2 are never used: clamp
        cmin = min(cmin, col[k]);
    }
    const int col_base = cmin & ~3;
    uint32_t col_sel = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) col_sel |= (uint32_t)(col[k] - col_base) << (8 * k);
    if (h < 4) {
        blur_wave<false, true>(src, sp, dst, G.bpitch, w, h, yw, x0, store, col_base, col_sel);
    } else if (xw >= 0 && xw + 256 <= w) {
        blur_wave<true, false>(src, sp, dst, G.bpitch, w, h, yw, x0, store, col_base, col_sel);
    } else {
        blur_wave<false, false>(src, sp, dst, G.bpitch, w, h, yw, x0, store, col_base, col_sel);
    }
}

// ------------------------------------------------------------------------
// FAST-9/16 over one band of kBandRows output rows.
constexpr int kFastNT = 256;
#ifndef DVO_FAST_SEG_CALL
#define DVO_FAST_SEG_CALL 8
#endif
// workgroups per strip: batches of fewer than 8 frames are latency-bound on the strip walk.
// Drop-in pairs/s at 1280x720 (tools/ab_dropin.sh): 1 segment 512, 2: 523, 4: 529, 8: 533.
__host__ __device__ constexpr int kFastSeg(int F) { return F < 8 ? DVO_FAST_SEG_CALL : 1; }

__device__ __forceinline__ int fast_score16(const int* c, int v, int threshold) {
    // fast.cpp cornerScore<16> (scalar form): d[k] = v - circle[k], k in [0, 25)
    int d[25];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - c[k];
#pragma unroll
    for (int k = 16; k < 25; ++k) d[k] = d[k - 16];
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(d[k + 1], d[k + 2]);
        b = max(b, d[k + 3]);
        b = max(b, d[k + 4]);
        b = max(b, d[k + 5]);
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// cornerScore<16> in packed 16-bit lanes: P[k] = (v - c_k, c_k - v).  The scalar form's second
// loop is its first with d -> -d and a0 -> -b0 (max(x) = -min(-x)), started from the first
// loop's result; max being associative, both loops run as one packed fold from (threshold,
// -inf) and the score is max(low, high) - 1.  The 8-wide window minima of both are shared:
// pairwise, 4-wide and 8-wide minima over P[1..22] (29 packed mins instead of 2 x 8 x 7).
// Checked against fast_score16 on 2e7 random and structured circles (host build of both).
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int fast_score16_pk(const uint8_t* p, int stride, int threshold) {
    const int v = p[0];
    i16x2 P[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int t = v - (int)p[kCdy[k] * stride + kCdx[k]];
        P[k] = (i16x2){(short)t, (short)-t};
    }
    auto pmin = [](i16x2 a, i16x2 b) { return __builtin_elementwise_min(a, b); };
    auto pmax = [](i16x2 a, i16x2 b) { return __builtin_elementwise_max(a, b); };
    // M2(i) = min(P[2i+1], P[2i+2]) (indices mod 16), M4(i) = min(M2(i), M2(i+1)),
    // M8(i) = min(M4(i), M4(i+2)) = min(d[2i+1 .. 2i+8]); rolled so few of them are live at once
    auto m2 = [&](int i) { return pmin(P[(2 * i + 1) & 15], P[(2 * i + 2) & 15]); };
    i16x2 acc = (i16x2){(short)threshold, (short)-32768};
    i16x2 a2 = m2(0), b2 = m2(1), c2 = m2(2), d2 = m2(3);
    i16x2 m4a = pmin(a2, b2), m4b = pmin(b2, c2), m4c = pmin(c2, d2);  // M4(i), M4(i+1), M4(i+2)
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // k = 2 i: window d[k+1 .. k+8] = M8(i), ends d[k], d[k+9]
        const i16x2 w8 = pmin(m4a, m4c);
        acc = pmax(acc, pmin(w8, P[2 * i]));
        acc = pmax(acc, pmin(w8, P[(2 * i + 9) & 15]));
        if (i < 7) {
            const i16x2 e2 = m2(i + 4);
            m4a = m4b;
            m4b = m4c;
            m4c = pmin(d2, e2);
            d2 = e2;
        }
    }
    return max((int)acc.x, (int)acc.y) - 1;
}

__device__ __forceinline__ bool has_run9(uint32_t m) {
    uint32_t m2 = m | (m << 16);
    uint32_t a = m2 & (m2 >> 1);  // runs >= 2
    a = a & (a >> 2);             // >= 4
    a = a & (a >> 4);             // >= 8
    a = a & (m2 >> 8);            // >= 9
    return (a & 0xFFFFu) != 0;
}

__device__ __forceinline__ int block_excl_scan(int v, int& total, int* lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    // inclusive scan within the wave
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        int c = lds[w];
        if (w < wid) off += c;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

__device__ __forceinline__ uint32_t byte_at(uint32_t lo, uint32_t hi, int k) {  // byte k of (hi:lo), k in [0, 8)
    return k < 4 ? (lo >> (8 * k)) & 0xFF : (hi >> (8 * (k - 4))) & 0xFF;
}

// FAST over one column strip of one level.  The workgroup walks the strip's
// tiles (kBandRows output rows x kFastTW (124) output columns) top to bottom.
// The image window of a tile (rows [r0-4, r0+kBandRows+4), 144 columns from the
// column bx = xs - 7) lives in LDS as words; the next tile's kBandRows new rows are loaded into
// registers while the current tile is processed (the load latency hides behind
// the compute), and its last 8 rows are carried to the top of the window, so
// every image byte is fetched from HBM once.  FAST scores are needed on the
// NMS neighbourhood, score rows [r0-1, r1] x score columns [xs-1, xs+125): the
// first tile computes all kBandRows+2 score rows, later tiles the kBandRows new ones and carry
// the two above (and the corners of the last one, an output row of the next
// tile, in a small list).  Per tile, each wave runs compass -> segment test ->
// score on its own rows with its own LDS list segment (no workgroup barrier
// in between: at ~6% candidates a wave's list is about one 64-lane round, as
// the concatenated list's share per wave was), then workgroup barriers
// separate NMS (which reads neighbours' scores) and the output:
//   compass  every pixel: a run of 9 on the 16-circle contains two adjacent
//            compass pixels (0,4 / 4,8 / 8,12 / 12,0) that are both brighter
//            or both darker: min(max(c0,c8), max(c4,c12)) > v+t, or the dual;
//            a lane tests the 4 pixels of one LDS word from 5 word reads
//            (centre row -1/0/+1 words, rows -3/+3), byte-permuted into packed
//            u16 pairs and compared with saturating v_pk ops;
//   segment  survivors (~6%): the 16 circle compares packed into bright/dark
//            masks with v_alignbit (sign bit shifted in), run-of-9 test;
//   score    corners (~1%): cornerScore<16> into the LDS score plane;
//   NMS      per corner: strict 3x3 maximum -> keep bit of its row;
//   output   keeps per tile row in column order, (offset << 16 | count) per
//            row; select_fast_kernel restores raster order across tiles.
// Minimum resident waves per SIMD requested of the compiler (VGPR budget).  With the corner list
// compacted into the candidate slots a workgroup needs ~18.4 KB of LDS, so 8 workgroups would fit a
// CU, but the kernel then spills (64 VGPRs + 64 B/lane scratch at 8, 72 + 32 B at 7).  Measured,
// whole default bench (profiles/r03e_ab_fast_occupancy.txt): 4 / 5 -> 70.5 K frames/s, 6 -> 73.0 K
// (79 VGPRs, no spill), 7 -> 69.1 K, 8 -> 67.3 K: the FAST stage gets faster with occupancy but
// starves the blur / describe kernels the other stream runs beside it.
#ifndef DVO_FAST_WAVES_PER_EU
#define DVO_FAST_WAVES_PER_EU 6
#endif
constexpr int kFtLW = 144;                      // LDS row stride of the image and score planes
constexpr int kFtRows = kBandRows + 8;          // staged image rows per tile: [r0-4, r0+kBandRows+4)
static_assert(kFastTW == 124 && (kBorder - 7) % 4 == 0, "FAST tiles: score columns = LDS words 1..32");
// per-wave list capacities: compass, row pairs wid, wid+4, .. of 64 lanes x 4 px; segment test, the
// concatenated candidates of the tile (<= (kBandRows + 2) x 126) in 64-lane rounds of the 4 waves
constexpr int kFtSegCand = ((kBandRows + 3) / 2 + 3) / 4 * 256;
constexpr int kFtWordCand = kFtSegCand / 4;  // compass word entries per wave (64 lanes x iterations)
constexpr int kFtWords = kFtLW / 4;             // words per staged row
constexpr int kFtNewW = kBandRows * kFtWords;   // words loaded per tile (rows r0+4 .. r0+kBandRows+4)
constexpr int kFtPf = (kFtNewW + kFastNT - 1) / kFastNT;
constexpr int kFtCarryW = 8 * kFtWords;         // image words carried (the window's last 8 rows -> top)
constexpr int kFtCarryR = (kFtCarryW + kFastNT - 1) / kFastNT;
constexpr int kFtCarryList = 128;               // corners of one score row
static_assert(kFtRows * kFtWords == kFtNewW + kFtCarryW, "staging covers the window");
// The compass pre-test of two pixels (packed u16 pairs): min(max(c0,c8), max(c4,c12)) - v > t or
// v - max(min(c0,c8), min(c4,c12)) > t, as saturating differences (t in [0, 255]); a nonzero
// half (<= 255) passes.
__device__ __forceinline__ uint32_t compass_pass(u16x2 v, u16x2 c0, u16x2 c8, u16x2 c4, u16x2 c12, uint32_t thr2) {
    const u16x2 X = __builtin_elementwise_min(__builtin_elementwise_max(c0, c8), __builtin_elementwise_max(c4, c12));
    const u16x2 Y = __builtin_elementwise_max(__builtin_elementwise_min(c0, c8), __builtin_elementwise_min(c4, c12));
    const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_sub_sat(X, v), __builtin_elementwise_sub_sat(v, Y));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(m, as_u16x2(thr2)));
}
__device__ __forceinline__ uint32_t lane_prefix(unsigned long long bal) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}
// index of entry e of the concatenation of the 4 per-wave segments of a list (counts cnt[0..3])
template <int kSeg>
__device__ __forceinline__ int seg_index(const int* cnt, int e) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool past = e >= cnt[k];
        e -= past ? cnt[k] : 0;
        s += past ? 1 : 0;
        if (!past) break;
    }
    return s * kSeg + e;
}
template <int kSeg>
__device__ __forceinline__ int seg_at(const uint16_t* list, const int* cnt, int e) {
    return list[seg_index<kSeg>(cnt, e)];
}
__global__ __launch_bounds__(kFastNT, DVO_FAST_WAVES_PER_EU) void fast_strip_kernel(StreamParams P, int nseg) {
    // nseg > 1 (batches of a few frames): a strip's tiles are walked by nseg workgroups,
    // segment k from tile k * ceil(nbands / nseg), each starting like tile 0 (2 more score rows)
    int it;
    const int f = xcd_frame_item(P.plan.total_strips * nseg, P.nframes, it);
    if (f >= P.nframes) return;
    const int strip = it / nseg, seg = it - strip * nseg;
    int l = 0;
    while (l + 1 < P.plan.nlevels && strip >= P.plan.L[l + 1].strip_base) ++l;
    const LevelGeom& G = P.plan.L[l];
    const int c = strip - G.strip_base;
    const int per_seg = (G.nbands + nseg - 1) / nseg;
    const int b_begin = seg * per_seg, b_end = min(G.nbands, b_begin + per_seg);
    if (b_begin >= b_end) return;
    const int w = G.w, h = G.h;
    const int xs = kBorder + c * kFastTW, xe = min(xs + kFastTW, w - kBorder);
    const int bx = xs - 7;  // image column of LDS column 0 (a multiple of 4: kBorder - 7 and kFastTW are)
    const int thr = P.plan.fast_threshold;
    const uint8_t* src = level_ptr(P, f, l);
    const int sp = level_pitch(P, l);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, h * sp, 0x00020000);
    __shared__ __attribute__((aligned(16))) uint8_t img[kFtRows * kFtLW];            // rows [r0-4, r0+kBandRows+4)
    __shared__ __attribute__((aligned(16))) uint8_t sc[(kBandRows + 2) * kFtLW];     // rows [r0-1, r0+kBandRows+1)
    // + 64 slots per wave that lanes without an entry store to (branch-free appends: no exec-mask SALU);
    // a wave's corners are compacted into its consumed candidate slots
    __shared__ uint16_t cand[4 * kFtSegCand + 256];
    __shared__ uint16_t wlist[4 * kFtWordCand + 256];  // per-wave word entries of the compass (+ spare slots)
    __shared__ uint16_t carry[2][kFtCarryList];  // corners of score row r0+16, as next-tile addresses
    __shared__ int ncorner[4], ncarry[2];
    __shared__ uint32_t keep[kBandRows][4];  // bit i <-> score column xs - 1 + i
    __shared__ int row_off[4][kBandRows];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xlast = min(xe, w - 4);  // last score column (xs - 1 >= 30 >= 3 on the left)
    // score columns [xs - 1, xlast] are LDS columns [6, xlast - bx + 1) <= [6, 132): the LDS words
    // 1..32 of a row; this lane's word and the mask of its score bytes
    const int c_col = 4 + 4 * (lane & 31), c_hi = xlast - bx + 1 - c_col;
    const uint32_t c_vm = (c_col == 4 ? 0xFFFF0000u : 0xFFFFFFFFu) &
                          (c_hi >= 4 ? 0xFFFFFFFFu : c_hi <= 0 ? 0u : (1u << (8 * c_hi)) - 1u);
    // the same as a 4-bit pixel mask (bit k <-> byte k)
    const uint32_t c_vm4 = (c_vm & 1u) | ((c_vm >> 7) & 2u) | ((c_vm >> 14) & 4u) | ((c_vm >> 21) & 8u);
    const uint32_t thr2 = (uint32_t)thr * 0x10001u;
    // Words past the row end are never read by the FAST tests (x + 3 <= w - 1): the buffer
    // load returns whatever lies there (or 0 past the level).  The row offset goes in the
    // per-lane offset: the rows of one wave's words differ (a scalar offset would be a waterfall).
    uint32_t creg[kFtCarryR], pf[kFtPf], screg = 0;
    // per-lane part of the prefetch addresses (row rr_k, word wd_k of word q = tid + k kFastNT): 32-bit,
    // the wave-uniform row base goes in the scalar offset
    int voff[kFtPf];
#pragma unroll
    for (int k = 0; k < kFtPf; ++k) {
        const int q = threadIdx.x + k * kFastNT;
        const int rr = q / kFtWords, wd = q - rr * kFtWords;
        voff[k] = 4 * wd + rr * sp;
    }
    {  // prologue: rows [r0-4, r0+4) into the carry registers, [r0+4, r0+kBandRows+4) into the prefetch registers
        const int ylo = kBorder + b_begin * kBandRows - 4;
#pragma unroll
        for (int k = 0; k < kFtCarryR; ++k) {
            const int q = threadIdx.x + k * kFastNT;
            creg[k] = q < kFtCarryW ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff[k], bx + ylo * sp, 0) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kFtPf; ++k) {
            const int q = threadIdx.x + k * kFastNT;
            pf[k] = q < kFtNewW ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff[k], bx + (ylo + 8) * sp, 0) : 0u;
        }
    }
    if (threadIdx.x == 0) ncarry[0] = 0;
    for (int b = b_begin; b < b_end; ++b) {
        const int par = (b - b_begin) & 1;
        const int r0 = kBorder + b * kBandRows;
        const int r1 = min(r0 + kBandRows, h - kBorder);
        const int nrows = r1 - r0;
        const int item = G.band_base + b * G.ntx + c;
        // ---- window: carried rows 0..7, new rows 8..kFtRows-1; score rows 0, 1 carried (tile 0: zero)
#pragma unroll
        for (int k = 0; k < kFtCarryR; ++k) {
            const int q = threadIdx.x + k * kFastNT;
            if (q < kFtCarryW) reinterpret_cast<uint32_t*>(img)[q] = creg[k];
        }
#pragma unroll
        for (int k = 0; k < kFtPf; ++k) {
            const int q = threadIdx.x + k * kFastNT;
            if (q < kFtNewW) reinterpret_cast<uint32_t*>(img)[kFtCarryW + q] = pf[k];
        }
        if (threadIdx.x < 2 * kFtWords) reinterpret_cast<uint32_t*>(sc)[threadIdx.x] = b == b_begin ? 0u : screg;
        for (int q = threadIdx.x; q < kBandRows * kFtLW / 16; q += kFastNT)
            reinterpret_cast<uint4*>(sc + 2 * kFtLW)[q] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x < kBandRows * 4) keep[threadIdx.x >> 2][threadIdx.x & 3] = 0;
        if (threadIdx.x == 0) ncarry[par ^ 1] = 0;
        __syncthreads();
        // ---- next tile: carried rows from LDS, new rows from HBM (in flight during this tile)
        if (b + 1 < b_end) {
#pragma unroll
            for (int k = 0; k < kFtCarryR; ++k) {
                const int q = threadIdx.x + k * kFastNT;
                creg[k] = q < kFtCarryW ? reinterpret_cast<const uint32_t*>(img)[kFtNewW + q] : 0u;
            }
            const int ynew = r0 + kBandRows + 4;
#pragma unroll
            for (int k = 0; k < kFtPf; ++k) {
                const int q = threadIdx.x + k * kFastNT;
                pf[k] = q < kFtNewW ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff[k], bx + ynew * sp, 0) : 0u;
            }
        }
        // ---- compass, segment test and score, each wave on its own rows, no workgroup barrier in
        // between: the window is in LDS, a wave's candidates and corners are its own list segment and
        // its scores land on its own score pixels.  Four score pixels per lane: lane -> LDS word
        // 1 + (lane & 31) of score row sr_lo + 2 (wid + 4 t) + (lane >> 5), t = 0, 1, ...
        const int nsr = nrows + 2;
        const int sr_lo = b == b_begin ? 0 : 2;
        const int seg_off = wid * kFtSegCand, spare_i = 4 * kFtSegCand + wid * 64 + lane;
        int ncw = 0;  // this wave's corners (wave-uniform), compacted to cand[seg_off, seg_off + ncw)
        {
            int n = 0, nw = 0;  // wave-uniform: pixel candidates, words with one
            const int wl_off = wid * kFtWordCand, wl_spare = 4 * kFtWordCand + wid * 64 + lane;
            for (int sr = sr_lo + 2 * wid + (lane >> 5); __builtin_amdgcn_readfirstlane(sr - (lane >> 5)) < nsr;
                 sr += 8) {
                const int base = (sr + 3) * kFtLW + c_col;  // centre-row byte address of the word
                const uint32_t* wp = reinterpret_cast<const uint32_t*>(img + base);
                const uint32_t wc = wp[0], wl = wp[-1], wr = wp[1];
                const uint32_t wu = wp[-3 * kFtWords], wd = wp[3 * kFtWords];
                // pixels 0, 2 in the low pair, 1, 3 in the high pair; c4 = columns +3, c12 = columns -3
                const uint32_t r0p = compass_pass(as_u16x2(__builtin_amdgcn_perm(0, wc, 0x0C020C00)),
                                                  as_u16x2(__builtin_amdgcn_perm(0, wu, 0x0C020C00)),
                                                  as_u16x2(__builtin_amdgcn_perm(0, wd, 0x0C020C00)),
                                                  as_u16x2(__builtin_amdgcn_perm(wr, wc, 0x0C050C03)),
                                                  as_u16x2(__builtin_amdgcn_perm(wc, wl, 0x0C030C01)), thr2);
                const uint32_t r1p = compass_pass(as_u16x2(__builtin_amdgcn_perm(0, wc, 0x0C030C01)),
                                                  as_u16x2(__builtin_amdgcn_perm(0, wu, 0x0C030C01)),
                                                  as_u16x2(__builtin_amdgcn_perm(0, wd, 0x0C030C01)),
                                                  as_u16x2(__builtin_amdgcn_perm(wr, wc, 0x0C060C04)),
                                                  as_u16x2(__builtin_amdgcn_perm(wc, wl, 0x0C040C02)), thr2);
                // bit k of msk <=> pixel k passes and is a score pixel of this tile: each half of
                // r0p (pixels 0, 2) and r1p (1, 3) is <= 255 and nonzero iff the pixel passes, so a
                // packed min with 1 gives its bit; (p0 | p1 << 1) in bits 0-1, (p2 | p3 << 1) in 16-17
                // (LLVM folds a packed min with 1 into per-half compares and selects: v_pk_min_u16
                // written out keeps it at one instruction per pair)
                uint32_t b0, b1;
                asm("v_pk_min_u16 %0, %1, %2" : "=v"(b0) : "v"(r0p), "v"(0x00010001u));
                asm("v_pk_min_u16 %0, %1, %2" : "=v"(b1) : "v"(r1p), "v"(0x00010001u));
                const uint32_t m2 = b0 | (b1 << 1);
                const uint32_t msk = (m2 | (m2 >> 14)) & (sr < nsr ? c_vm4 : 0u);
                // one entry per word with a passing pixel: (word index | mask << 12)
                const bool any = msk != 0;
                const unsigned long long bal = __ballot(any);
                const int to = wl_off + nw + (int)lane_prefix(bal);
                wlist[any ? to : wl_spare] = (uint16_t)((base >> 2) | (msk << 12));
                nw += __popcll(bal);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // word entries -> pixel entries: a lane's c = popc(mask) pixels go to its prefix of c
            // (from three ballots of c's bits) plus the rank of the pixel's bit in the mask
            for (int e0 = 0; e0 < nw; e0 += 64) {
                const int e = e0 + lane;
                const uint32_t ent = e < nw ? (uint32_t)wlist[wl_off + e] : 0u;
                const uint32_t msk = ent >> 12;
                const int a0 = (int)(ent & 0xFFFu) << 2;
                const uint32_t c = (uint32_t)__popc(msk);
                const unsigned long long b0 = __ballot(c & 1u), b1 = __ballot(c & 2u), b2 = __ballot(c & 4u);
                const int pre = n + (int)lane_prefix(b0) + 2 * (int)lane_prefix(b1) + 4 * (int)lane_prefix(b2);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool on = (msk >> k) & 1u;
                    const int to = seg_off + pre + __popc(msk & ((1u << k) - 1u));
                    if (on) cand[to] = (uint16_t)(a0 + k);
                }
                n += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // segment test over the wave's candidates in 64-lane rounds; its j-th corner overwrites its
            // j-th read entry (already consumed: j <= the entries read so far)
            for (int e0 = 0; e0 < n; e0 += 64) {
                const int e = e0 + lane;
                bool is_corner = false;
                int a = 0;
                if (e < n) {
                    a = cand[seg_off + e];
                    const uint8_t* p = img + a;
                    const int v = p[0];
                    const uint32_t hi = (uint32_t)(v + thr), lo = (uint32_t)(v - thr);
                    uint32_t br = 0, dk = 0;
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const uint32_t cv = p[kCdy[k] * kFtLW + kCdx[k]];
                        br = __builtin_amdgcn_alignbit(br, hi - cv, 31);  // bit <- (cv > v + thr)
                        dk = __builtin_amdgcn_alignbit(dk, cv - lo, 31);  // bit <- (cv < v - thr)
                    }
                    is_corner = has_run9(br) || has_run9(dk);
                }
                const unsigned long long bal = __ballot(is_corner);
                cand[is_corner ? seg_off + ncw + (int)lane_prefix(bal) : spare_i] = (uint16_t)a;
                ncw += __popcll(bal);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // scores of the wave's corners into the score plane
            for (int e = lane; e < ncw; e += 64) {
                const int a = cand[seg_off + e];
                sc[a - 3 * kFtLW] = (uint8_t)fast_score16_pk(img + a, kFtLW, thr);
            }
            if (lane == 0) ncorner[wid] = ncw;
        }
        __syncthreads();
        int cnt2[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) cnt2[k] = ncorner[k];
        const int ncorners = cnt2[0] + cnt2[1] + cnt2[2] + cnt2[3];
        const int nc = ncarry[par];
        // score rows kBandRows, kBandRows+1 for the next tile (final now)
        if (threadIdx.x < 2 * kFtWords) screg = reinterpret_cast<const uint32_t*>(sc)[kBandRows * kFtWords + threadIdx.x];
        // ---- strict 3x3 NMS of the carried and new corners; keeps lie in rows [r0, r1), columns [xs, xe).
        // New corners of score row kBandRows+1 (row r0 + kBandRows) are the next tile's row-1 corners.
        for (int e = threadIdx.x; e < nc + ncorners; e += kFastNT) {
            const int a = (e < nc ? (int)carry[par][e] : seg_at<kFtSegCand>(cand, cnt2, e - nc)) -
                          3 * kFtLW;  // score-plane address
            const int sr = a / kFtLW, x = bx + (a - sr * kFtLW);
            if (sr == kBandRows + 1) {
                const int slot = atomicAdd(&ncarry[par ^ 1], 1);
                carry[par ^ 1][slot] = (uint16_t)(a + 3 * kFtLW - kBandRows * kFtLW);
                continue;
            }
            if (sr < 1 || sr > nrows || x < xs || x >= xe) continue;
            const uint8_t* s = sc + a;
            const uint32_t v = s[0];
            const uint32_t nmax = max(max(max((uint32_t)s[-kFtLW - 1], (uint32_t)s[-kFtLW]),
                                          max((uint32_t)s[-kFtLW + 1], (uint32_t)s[-1])),
                                      max(max((uint32_t)s[1], (uint32_t)s[kFtLW - 1]),
                                          max((uint32_t)s[kFtLW], (uint32_t)s[kFtLW + 1])));
            if (v > nmax) {
                const int i_col = x - (xs - 1);
                atomicOr(&keep[sr - 1][i_col >> 5], 1u << (i_col & 31));
            }
        }
        __syncthreads();
        // ---- output: row counts and offsets (a 16-lane scan in every wave), then every kept corner
        // writes its key at row offset + kept columns before it: keys of a row land in column order
        uint32_t* outp = P.buf.band_cand + (int64_t)f * P.plan.band_cand_stride + G.band_cand_off +
                         (int64_t)(b * G.ntx + c) * G.band_cap;
        {
            int rc = 0;
            if (lane < kBandRows && lane < nrows)
                rc = __popc(keep[lane][0]) + __popc(keep[lane][1]) + __popc(keep[lane][2]) + __popc(keep[lane][3]);
            int incl = rc;
#pragma unroll
            for (int o = 1; o < kBandRows; o <<= 1) {
                const int y2 = __shfl_up(incl, o);
                if (lane >= o) incl += y2;
            }
            if (lane < kBandRows) {
                row_off[wid][lane] = incl - rc;
                if (wid == 0)
                    P.buf.band_cnt[((int64_t)f * P.plan.total_bands + item) * kBandRows + lane] = ((incl - rc) << 16) | rc;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (int e = threadIdx.x; e < nc + ncorners; e += kFastNT) {
            const int a = (e < nc ? (int)carry[par][e] : seg_at<kFtSegCand>(cand, cnt2, e - nc)) - 3 * kFtLW;
            const int sr = a / kFtLW, x = bx + (a - sr * kFtLW);
            if (sr < 1 || sr > nrows || x < xs || x >= xe) continue;
            const int i_col = x - (xs - 1), wq = i_col >> 5;
            const uint32_t* kr = keep[sr - 1];
            if (!((kr[wq] >> (i_col & 31)) & 1)) continue;
            int before = __popc(kr[wq] & ((1u << (i_col & 31)) - 1));
            for (int q = 0; q < wq; ++q) before += __popc(kr[q]);
            outp[row_off[wid][sr - 1] + before] = ((uint32_t)sc[a] << 24) | ((uint32_t)(r0 + sr - 1) << 12) | (uint32_t)x;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------
// KeyPointsFilter::retainBest — exact emulation of libstdc++'s introselect
// (median-of-3 + unguarded Hoare partition, heap-select fallback, final
// insertion sort) followed by the bidirectional std::partition.  Each Hoare
// partition step is computed in parallel: the k-th left stop is the k-th
// position (ascending) holding a value <= pivot, the k-th right stop the k-th
// position (descending) holding a value >= pivot; pairs are swapped while
// left < right, and the returned cut is min(L[k*], R[k*-1]).
struct FastKeys {
    uint32_t* key;
    struct Elem {
        uint32_t k;
    };
    __device__ int val(int i) const { return (int)(key[i] >> 24); }
    __device__ void swap(int i, int j) const {
        uint32_t t = key[i];
        key[i] = key[j];
        key[j] = t;
    }
    __device__ Elem get(int i) const { return Elem{key[i]}; }
    __device__ void put(int i, Elem e) const { key[i] = e.k; }
    __device__ static int ev(Elem e) { return (int)(e.k >> 24); }
};

struct HarrisVals {
    float* v;
    uint32_t* key;
    struct Elem {
        float v;
        uint32_t k;
    };
    __device__ float val(int i) const { return v[i]; }
    __device__ void swap(int i, int j) const {
        float t = v[i];
        v[i] = v[j];
        v[j] = t;
        uint32_t u = key[i];
        key[i] = key[j];
        key[j] = u;
    }
    __device__ Elem get(int i) const { return Elem{v[i], key[i]}; }
    __device__ void put(int i, Elem e) const {
        v[i] = e.v;
        key[i] = e.k;
    }
    __device__ static float ev(Elem e) { return e.v; }
};

__device__ __forceinline__ void block_excl_scan2(int fa, int fb, int& pa, int& pb, int& ta, int& tb, int* lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    unsigned long long ma = __ballot(fa), mb = __ballot(fb);
    unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    if (lane == 0) {
        lds[wid] = __popcll(ma);
        lds[32 + wid] = __popcll(mb);
    }
    __syncthreads();
    int oa = 0, ob = 0, sa = 0, sb = 0;
    for (int w = 0; w < nw; ++w) {
        int ca = lds[w], cb = lds[32 + w];
        if (w < wid) {
            oa += ca;
            ob += cb;
        }
        sa += ca;
        sb += cb;
    }
    __syncthreads();
    pa = oa + __popcll(ma & lt);
    pb = ob + __popcll(mb & lt);
    ta = sa;
    tb = sb;
}

__device__ __forceinline__ int block_sum(int v, int* lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    int s = 0;
    for (int w = 0; w < nw; ++w) s += lds[w];
    __syncthreads();
    return s;
}

template <class A, class V>
__device__ int partition_step(const A& a, int first, int last, V p, int32_t* Lpos, int32_t* Rasc, int* lds) {
    int nL = 0, nR = 0;
    for (int base = first; base < last; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const bool in = i < last;
        V v = in ? a.val(i) : p;
        int fl = in && i >= first + 1 && !(v > p);
        int fr = in && !(p > v);
        int pa, pb, ta, tb;
        block_excl_scan2(fl, fr, pa, pb, ta, tb, lds);
        if (fl) Lpos[nL + pa] = i;
        if (fr) Rasc[nR + pb] = i;
        nL += ta;
        nR += tb;
    }
    __syncthreads();
    const int K = min(nL, nR);
    int cnt = 0;
    for (int k = threadIdx.x; k < K; k += blockDim.x) cnt += Lpos[k] < Rasc[nR - 1 - k];
    const int kstar = block_sum(cnt, lds);
    for (int k = threadIdx.x; k < kstar; k += blockDim.x) a.swap(Lpos[k], Rasc[nR - 1 - k]);
    const int cl = kstar < nL ? Lpos[kstar] : INT_MAX;
    const int cr = kstar > 0 ? Rasc[nR - kstar] : INT_MAX;
    __syncthreads();
    return min(cl, cr);
}

// libstdc++ heap primitives, single thread (rare depth-limit fallback).
template <class A>
__device__ void adjust_heap(const A& a, int first, int hole, int len, typename A::Elem value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (a.val(first + second) > a.val(first + second - 1)) second--;
        a.put(first + hole, a.get(first + second));
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a.put(first + hole, a.get(first + second - 1));
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && a.val(first + parent) > A::ev(value)) {
        a.put(first + hole, a.get(first + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a.put(first + hole, value);
}

template <class A>
__device__ void heap_select(const A& a, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2) {
        int parent = (len - 2) / 2;
        while (true) {
            adjust_heap(a, first, parent, len, a.get(first + parent));
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; ++i)
        if (a.val(i) > a.val(first)) {
            typename A::Elem v = a.get(i);
            a.put(i, a.get(first));
            adjust_heap(a, first, 0, len, v);
        }
}

template <class A>
__device__ void insertion_sort(const A& a, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        typename A::Elem v = a.get(i);
        if (A::ev(v) > a.val(first)) {
            for (int k = i; k > first; --k) a.put(k, a.get(k - 1));
            a.put(first, v);
        } else {
            int k = i;
            while (A::ev(v) > a.val(k - 1)) {
                a.put(k, a.get(k - 1));
                --k;
            }
            a.put(k, v);
        }
    }
}

template <class A>
__device__ void move_median_to_first(const A& a, int result, int x, int y, int z) {
    if (a.val(x) > a.val(y)) {
        if (a.val(y) > a.val(z)) a.swap(result, y);
        else if (a.val(x) > a.val(z)) a.swap(result, z);
        else a.swap(result, x);
    } else if (a.val(x) > a.val(z)) a.swap(result, x);
    else if (a.val(y) > a.val(z)) a.swap(result, z);
    else a.swap(result, y);
}

// Returns the retained size; the first `result` entries hold the kept
// elements in libstdc++ order.  Must be called by the whole block.
// semantics kOcv32: OpenCV 3.2's retainBest ran nth_element at begin + n (not
// n - 1) and still read the boundary response at n - 1 (oracle retain_best).
template <class A>
__device__ int retain_best_block(const A& a, int n, int npoints, int depth, int32_t* Lpos, int32_t* Rasc, int* lds,
                                 int semantics = kOcv4) {
    if (npoints < 0 || n <= npoints) return n;
    if (npoints == 0) return 0;
    const int nth = semantics == kOcv32 ? npoints : npoints - 1;
    int first = 0, last = n;
    if (depth < 0) depth = 2 * (31 - __clz(n));
    bool heap_done = false;
    while (last - first > 3) {
        if (depth == 0) {
            if (threadIdx.x == 0) {
                heap_select(a, first, nth + 1, last);
                a.swap(first, nth);
            }
            heap_done = true;
            break;
        }
        --depth;
        if (threadIdx.x == 0) move_median_to_first(a, first, first + 1, first + (last - first) / 2, last - 1);
        __syncthreads();
        auto p = a.val(first);
        const int cut = partition_step(a, first, last, p, Lpos, Rasc, lds);
        if (cut <= first || cut >= last) break;  // impossible for a correct emulation; never loop unbounded
        if (cut <= nth) first = cut;
        else last = cut;
    }
    if (!heap_done && threadIdx.x == 0) insertion_sort(a, first, last);
    __syncthreads();
    // std::partition(begin+npoints, end, response >= ambiguous) (bidirectional)
    auto amb = a.val(npoints - 1);
    int nL = 0, nR = 0;
    for (int base = npoints; base < n; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const bool in = i < n;
        int fl = 0, fr = 0;
        if (in) {
            bool pr = a.val(i) >= amb;
            fl = !pr;
            fr = pr;
        }
        int pa, pb, ta, tb;
        block_excl_scan2(fl, fr, pa, pb, ta, tb, lds);
        if (fl) Lpos[nL + pa] = i;
        if (fr) Rasc[nR + pb] = i;
        nL += ta;
        nR += tb;
    }
    __syncthreads();
    const int K = min(nL, nR);
    int cnt = 0;
    for (int k = threadIdx.x; k < K; k += blockDim.x) cnt += Lpos[k] < Rasc[nR - 1 - k];
    const int kstar = block_sum(cnt, lds);
    for (int k = threadIdx.x; k < kstar; k += blockDim.x) a.swap(Lpos[k], Rasc[nR - 1 - k]);
    __syncthreads();
    return npoints + nR;
}

#ifndef DVO_SEL_NT
#define DVO_SEL_NT 128  // measured: 128 threads 0.81 ms, 256 0.82, 512 1.06, 1024 2.17 (select + Harris, 513 frames)
#endif
constexpr int kSelNT = DVO_SEL_NT;
// select_fast's level-0 blocks (a 1280x720 frame keeps ~15 K FAST corners there, the other levels a
// few thousand): each quickselect partition step scans the range NT at a time between barriers.  Level
// 0 in its own launch at 256 threads: two-stream 89.1-89.4 -> 90.3-90.5 K (192: 90.2-90.4, 512: +0.6 %,
// 1024: -2.4 %; profiles/r04s_ab_bounds_select.txt, r04t_ab_select_level0.txt); alone it is slower
// (select + Harris 3.73 -> 4.18 ms), beside the other stream the separate launch interleaves better.
#ifndef DVO_SEL_NT0
#define DVO_SEL_NT0 256
#endif
constexpr int kSelNT0 = DVO_SEL_NT0;
// Batches of a few frames (the per-call drop-in surface: one frame) are latency-bound:
// fewer, wider partition chunks.  Drop-in pairs/s at 1280x720 (tools/ab_dropin.sh):
// 128 threads 429, 256 441, 512 452, 1024 447.
#ifndef DVO_SEL_NT_CALL
#define DVO_SEL_NT_CALL 512
#endif
constexpr int kSelNTCall = DVO_SEL_NT_CALL, kSelCallFrames = 4;
// The per-call kernels (one block per level, nothing else on the GPU) run the
// selection on an LDS copy of the level's list when it fits: every partition
// step's reads, scans and swaps are then LDS round trips instead of HBM ones.
// Lists longer than this (very textured frames) take the global-memory path.
constexpr int kSelLdsCap = 8192;
#ifndef DVO_SEL_LDS_CALL
#define DVO_SEL_LDS_CALL 1
#endif
constexpr bool kSelLdsCall = DVO_SEL_LDS_CALL != 0;

template <int NT, bool kLds>
__global__ __launch_bounds__(NT) void select_fast_kernel(StreamParams P, int l0) {
    const int l = l0 + blockIdx.x, f = blockIdx.y;
    if (l >= P.plan.nlevels) return;
    const LevelGeom& G = P.plan.L[l];
    __shared__ int lds[64];
    __shared__ int s_carry;
    const int32_t* rc = P.buf.band_cnt + ((int64_t)f * P.plan.total_bands + G.band_base) * kBandRows;
    const uint32_t* bsrc = P.buf.band_cand + (int64_t)f * P.plan.band_cand_stride + G.band_cand_off;
    uint32_t* A = P.buf.cand + (int64_t)f * P.plan.cand_stride + G.cand_off;
    // raster order: segment (band b, row rr, tile column c) = s = (b * kBandRows + rr) * ntx + c.
    // Per call (kLds: one block per level, nothing else resident) thread t owns the contiguous
    // run of segments [t per, (t + 1) per): one pass sums its counts, one block scan places the
    // runs, a second pass copies -- one scan instead of one per NT segments.  Batches keep the
    // NT-segment rounds (coalesced count reads; the per-thread runs measured 0.75 -> 1.16 ms).
    if constexpr (kLds) {
        const int nseg = G.nbands * kBandRows * G.ntx;
        const int per = (nseg + NT - 1) / NT;
        const int s_begin = min(nseg, (int)threadIdx.x * per), s_end = min(nseg, s_begin + per);
        auto seg_word = [&](int sg) {
            const int cc = sg % G.ntx, br = sg / G.ntx;
            const int b = br / kBandRows, rr = br - b * kBandRows;
            const int tile = b * G.ntx + cc;
            return make_int2(tile, rc[(int64_t)tile * kBandRows + rr]);
        };
        constexpr int kG = 8;  // segment words requested together
        int mine = 0;
        for (int s0 = s_begin; s0 < s_end; s0 += kG) {
            int2 tv[kG];
#pragma unroll
            for (int k = 0; k < kG; ++k) tv[k] = s0 + k < s_end ? seg_word(s0 + k) : make_int2(0, 0);
#pragma unroll
            for (int k = 0; k < kG; ++k) mine += tv[k].y & 0xFFFF;
        }
        int tot;
        int o = block_excl_scan(mine, tot, lds);
        for (int s0 = s_begin; s0 < s_end; s0 += kG) {
            int2 tv[kG];
#pragma unroll
            for (int k = 0; k < kG; ++k) tv[k] = s0 + k < s_end ? seg_word(s0 + k) : make_int2(0, 0);
#pragma unroll
            for (int k = 0; k < kG; ++k) {
                const int cnt = tv[k].y & 0xFFFF, src_off = tv[k].x * G.band_cap + (tv[k].y >> 16);
                for (int i = 0; i < cnt; ++i) A[o + i] = bsrc[src_off + i];
                o += cnt;
            }
        }
        if (threadIdx.x == 0) s_carry = tot;
        __syncthreads();
    } else {
        const int nseg = G.nbands * kBandRows * G.ntx;
        if (threadIdx.x == 0) s_carry = 0;
        __syncthreads();
        for (int s0 = 0; s0 < nseg; s0 += NT) {
            const int sg = s0 + threadIdx.x;
            int cnt = 0, src_off = 0;
            if (sg < nseg) {
                const int cc = sg % G.ntx, br = sg / G.ntx;
                const int b = br / kBandRows, rr = br - b * kBandRows;
                const int tile = b * G.ntx + cc;
                const int v = rc[(int64_t)tile * kBandRows + rr];
                cnt = v & 0xFFFF;
                src_off = tile * G.band_cap + (v >> 16);
            }
            int tot;
            const int off = block_excl_scan(cnt, tot, lds);
            const int base = s_carry;
            for (int i = 0; i < cnt; ++i) A[base + off + i] = bsrc[src_off + i];
            __syncthreads();
            if (threadIdx.x == 0) s_carry = base + tot;
            __syncthreads();
        }
    }
    const int n = s_carry;
    __syncthreads();
    int32_t* Lpos = P.buf.sel_tmp + (int64_t)f * 2 * P.plan.cand_stride + 2 * G.cand_off;
    int32_t* Rasc = Lpos + G.cand_cap;
    int k;
    if constexpr (kLds) {
        __shared__ uint32_t s_key[kSelLdsCap];
        __shared__ int32_t s_L[kSelLdsCap], s_R[kSelLdsCap];
        if (n <= kSelLdsCap) {
            for (int i = threadIdx.x; i < n; i += NT) s_key[i] = A[i];
            __syncthreads();
            k = retain_best_block(FastKeys{s_key}, n, 2 * G.nper, -1, s_L, s_R, lds, P.plan.semantics);
            __syncthreads();
            for (int i = threadIdx.x; i < k; i += NT) A[i] = s_key[i];
        } else {
            k = retain_best_block(FastKeys{A}, n, 2 * G.nper, -1, Lpos, Rasc, lds, P.plan.semantics);
        }
    } else {
        k = retain_best_block(FastKeys{A}, n, 2 * G.nper, -1, Lpos, Rasc, lds, P.plan.semantics);
    }
    if (threadIdx.x == 0) P.buf.cnt1[f * kMaxLevels + l] = k;
}

// orb.cpp HarrisResponses(blockSize 7, k 0.04f) on the unblurred level.
// HarrisResponses (orb.cpp, blockSize 7, k 0.04, Sobel 3x3): 16 lanes per
// keypoint, 4 keypoints per wave.  The keypoint's 9 x 12 byte window (rows
// y-4..y+4, aligned columns) is fetched as 27 coalesced words into LDS, each lane
// forms Ix, Iy at 3-4 of the 49 block positions, and the integer sums a, b, c
// are reduced over the 16 lanes (integer: order-free), then the float response
// is formed exactly as the scalar code does.
// Harris grid width: sized for 2n per level (the FAST-retained list is >= 2n
// with ties, known only on the device), grid-stride beyond that
// kHG keypoint groups per wave: every group's window words are requested before
// any is used, so one load latency covers kHG groups (the kernel is latency-bound:
// one group per wave left each wave a single load round trip of work).
#ifndef DVO_HARRIS_GROUPS
#define DVO_HARRIS_GROUPS 2  // two-stream bench: 1 73.6 K, 2 74.7 K, 4 74.6 K frames/s (profiles/r02z_ab_harris_groups.txt)
#endif
constexpr int kHG = DVO_HARRIS_GROUPS;
__host__ __device__ inline int harris_blocks_x(const Plan& pl) {
    int hb = 0;
    for (int l = 0; l < pl.nlevels; ++l) hb = hb > 2 * pl.L[l].nper ? hb : 2 * pl.L[l].nper;
    return (hb + 16 * kHG - 1) / (16 * kHG) + 1;
}

__global__ __launch_bounds__(256) void harris_kernel(StreamParams P) {
    __shared__ uint32_t win[kHG][16][32];  // one 9 x 3-word window (+ padding) per 16-lane group
    const int l = blockIdx.y, f = blockIdx.z;
    const int hb = blockIdx.x, gdx = gridDim.x;
    const int n = P.buf.cnt1[f * kMaxLevels + l];
    const LevelGeom& G = P.plan.L[l];
    const uint8_t* img = level_ptr(P, f, l);
    const int step = level_pitch(P, l);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, j = lane & 15;
    const uint32_t* cand = P.buf.cand + (int64_t)f * P.plan.cand_stride + G.cand_off;
    float* resp = P.buf.resp + (int64_t)f * P.plan.cand_stride + G.cand_off;
    for (int base = (hb * 4 + wid) * 4 * kHG; base < n; base += gdx * 16 * kHG) {
        int x0[kHG], ax[kHG];
        uint32_t v0[kHG], v1[kHG];
#pragma unroll
        for (int u = 0; u < kHG; ++u) {  // group u: keypoints base + 4 u .. base + 4 u + 3
            const int i = min(base + 4 * u + g, n - 1);
            const uint32_t key = cand[i];
            x0[u] = key & 0xFFF;
            const int y0 = (key >> 12) & 0xFFF;
            ax[u] = (x0[u] - 4) & ~3;  // window columns ax .. ax+11 cover x0-4 .. x0+4
            const uint8_t* wp = img + (int64_t)(y0 - 4) * step + ax[u];
            const int e1 = min(j + 16, 26);
            v0[u] = *reinterpret_cast<const uint32_t*>(wp + (int64_t)(j / 3) * step + 4 * (j % 3));
            v1[u] = *reinterpret_cast<const uint32_t*>(wp + (int64_t)(e1 / 3) * step + 4 * (e1 % 3));
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < kHG; ++u) {
            win[u][wid * 4 + g][j] = v0[u];
            win[u][wid * 4 + g][j + 16] = v1[u];  // j + 16 >= 27: padding words
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < kHG; ++u) {
            const uint8_t* Wb = reinterpret_cast<const uint8_t*>(win[u][wid * 4 + g]);
            const int o = x0[u] - ax[u] - 3;  // window column of block column 0 (pixel x0 - 3)
            int a = 0, b = 0, c = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int pos = j + 16 * t;
                if (t < 3 || pos < 49) {
                    const int py = pos / 7, px = pos - 7 * py;
                    const uint8_t* q = Wb + (1 + py) * 12 + o + px;
                    const int Ix = (q[1] - q[-1]) * 2 + (q[-12 + 1] - q[-12 - 1]) + (q[12 + 1] - q[12 - 1]);
                    const int Iy = (q[12] - q[-12]) * 2 + (q[12 - 1] - q[-12 - 1]) + (q[12 + 1] - q[-12 + 1]);
                    a += Ix * Ix;
                    b += Iy * Iy;
                    c += Ix * Iy;
                }
            }
#pragma unroll
            for (int s2 = 8; s2 >= 1; s2 >>= 1) {
                a += __shfl_xor(a, s2);
                b += __shfl_xor(b, s2);
                c += __shfl_xor(c, s2);
            }
            if (j == 0 && base + 4 * u + g < n) {
                const float scale = 1.f / ((1 << 2) * 7 * 255.f);
                const float s4 = scale * scale * scale * scale;
                const float fa = (float)a, fb = (float)b, fc = (float)c;
                resp[base + 4 * u + g] = (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * s4;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int NT, bool kLds>
__global__ __launch_bounds__(NT) void select_harris_kernel(StreamParams P) {
    const int l = blockIdx.x, f = blockIdx.y;
    if (l >= P.plan.nlevels) return;
    const LevelGeom& G = P.plan.L[l];
    __shared__ int lds[64];
    const int n = P.buf.cnt1[f * kMaxLevels + l];
    uint32_t* A = P.buf.cand + (int64_t)f * P.plan.cand_stride + G.cand_off;
    float* R = P.buf.resp + (int64_t)f * P.plan.cand_stride + G.cand_off;
    int32_t* Lpos = P.buf.sel_tmp + (int64_t)f * 2 * P.plan.cand_stride + 2 * G.cand_off;
    int32_t* Rasc = Lpos + G.cand_cap;
    int k;
    if constexpr (kLds) {
        __shared__ float s_v[kSelLdsCap];
        __shared__ uint32_t s_key[kSelLdsCap];
        __shared__ int32_t s_L[kSelLdsCap], s_R[kSelLdsCap];
        if (n <= kSelLdsCap) {
            for (int i = threadIdx.x; i < n; i += NT) {
                s_v[i] = R[i];
                s_key[i] = A[i];
            }
            __syncthreads();
            k = retain_best_block(HarrisVals{s_v, s_key}, n, G.nper, -1, s_L, s_R, lds, P.plan.semantics);
            __syncthreads();
            for (int i = threadIdx.x; i < k; i += NT) {
                R[i] = s_v[i];
                A[i] = s_key[i];
            }
        } else {
            k = retain_best_block(HarrisVals{R, A}, n, G.nper, -1, Lpos, Rasc, lds, P.plan.semantics);
        }
    } else {
        k = retain_best_block(HarrisVals{R, A}, n, G.nper, -1, Lpos, Rasc, lds, P.plan.semantics);
    }
    if (threadIdx.x == 0) P.buf.cnt2[f * kMaxLevels + l] = k;
}

// core fastAtan2 polynomial (degrees), evaluated exactly as the CPU restatement.
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = fabsf(x), ay = fabsf(y);
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

// One wave per keypoint: ICAngles (integer moments, wave-reduced), then
// pt *= scale, size = 31*scale, and the 256 rBRIEF bits — lane j evaluates bits
// j, j+64, j+128, j+192 and a ballot assembles each 64-bit descriptor word.
// One wave per keypoint.  Everything the keypoint needs is requested at once:
// the 16 IC-angle row segments of the unblurred level (registers) and the
// blurred 39 x 44 window around it (word loads into LDS); the 512 rBRIEF
// samples are then LDS reads.
// pattern radius <= 13*sqrt(2) -> 19; rows of 64 bytes: a sample's offset is (iy << 6) + ix (phase 3)
constexpr int kDPR = 19, kDPH = 2 * kDPR + 1, kDPW = 64;
// keypoints per wave, the loads of all of them requested first.  Reading a blurred pyramid: 1 73.0 K,
// 2 73.6 K, 4 72.3 K frames/s (profiles/r02z_ab_describe_dkw.txt); blurring the windows here
// (16 raw rows per lane and keypoint): 1 74.8 K (51 VGPRs), 2 74.3 K (119 VGPRs), against 73.2 K
// for the separate blur pass (profiles/r03o_ab_describe_blur.txt)
#ifndef DVO_DKW
#define DVO_DKW 1
#endif
constexpr int kDKW = DVO_DKW;          // keypoints per wave
constexpr int kDKB = 4 * kDKW;         // keypoints per workgroup
constexpr int kICW = 36, kICR = 36;    // IC window: rows ky-15 .. ky+15 (+ padding) x 9 aligned words

// The GaussianBlur of the pixels the descriptor samples is computed here from the
// raw level instead of being read from a blurred copy of the pyramid (blur_kernel,
// which does not run on the detection path; round 3, and FAST writing the blurred
// tiles in round 4 lost 9 %, profiles/r04l_ab_fast_blur.txt).  A band's lanes hold
// raw words of the window row span around the keypoint (a halo word each side), 8
// output rows from 14 raw rows, the vertical 7-tap over a rolling window of u16
// pairs and the horizontal taps from the neighbouring lanes (wave_shr /
// wave_shl), with blur_wave's arithmetic and rounding rule (half to even below
// w & ~3, half up in the w % 4 tail).  Keypoints lie >= 31 pixels from every
// border and the window reaches 22, so no reflection is needed.
// Only the pixels the rotated pattern can sample are blurred: pattern points lie within
// r = 18.385 of the centre (|x|, |y| <= 13), so a sample rounds to |dy| <= 18 and, in row dy,
// |dx| <= floor(sqrt(r^2 - (|dy| - 1/2)^2) + 1/2) (r for dy = 0): 6, 8, 10, .. 18 .. 6 (equal to
// the extents of cvRound over a 2e5-step angle sweep).  Five bands of 8 patch rows
// (dy = -18 + 8s .. -11 + 8s) take 11, 12, 12, 12 and 9 lanes (the band's words at its largest
// |dx| for any keypoint alignment, plus a halo word each side): 56 lanes, 8 rows each, where the
// full 39 x 44 window needed 52 lanes x 10 rows.
constexpr int kDBRows = 8, kDBSeg = 5, kDBRaw = kDBRows + 6;  // output rows per band, bands, raw rows
constexpr int kDBRow0 = 1;                                     // patch row of band 0's first row (dy = -18)
constexpr int kDBBase[kDBSeg + 1] = {0, 11, 23, 35, 47, 56};    // first lane of each band
constexpr int kDBHalfW[kDBSeg] = {15, 18, 18, 18, 12};          // largest |dx| in the band

// Every stored word lies left of the level's last w % 4 columns (keypoints >= 31 pixels from the border,
// the window <= 22 + a word): the half-to-even rule throughout.  The rounded sums s >> 16 are <= 257
// (the 8-bit kernel sums to 257^2 > 2^16): v_sat_pk_u8_i16 saturates two of them to bytes.
__device__ __forceinline__ uint32_t sat_pk_u8(uint32_t v) {
    uint32_t d;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(d) : "v"(v));
    return d;
}
__device__ __forceinline__ void describe_blur_rows(const uint32_t (&raw)[kDBRaw], uint8_t* patch_slot, int s, int wc,
                                                   bool st) {
    const u16x2 k18 = {18, 18}, k34 = {34, 34}, k49 = {49, 49}, k55 = {55, 55};
    const uint32_t R = 0x7FFFu;
    u16x2 lo[7], hi[7];
#pragma unroll
    for (int r = 0; r < kDBRaw; ++r) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            lo[k] = lo[k + 1];
            hi[k] = hi[k + 1];
        }
        lo[6] = as_u16x2(__builtin_amdgcn_perm(0u, raw[r], 0x0C010C00u));  // (b0, b1)
        hi[6] = as_u16x2(__builtin_amdgcn_perm(0u, raw[r], 0x0C030C02u));  // (b2, b3)
        if (r < 6) continue;
        const u16x2 a = k18 * (lo[0] + lo[6]) + k34 * (lo[1] + lo[5]) + k49 * (lo[2] + lo[4]) + k55 * lo[3];
        const u16x2 b = k18 * (hi[0] + hi[6]) + k34 * (hi[1] + hi[5]) + k49 * (hi[2] + hi[4]) + k55 * hi[3];
        const uint32_t A = __builtin_bit_cast(uint32_t, a), B = __builtin_bit_cast(uint32_t, b);
        const u16x2 al = as_u16x2(dpp_from_left(A)), bl = as_u16x2(dpp_from_left(B));
        const u16x2 ar = as_u16x2(dpp_from_right(A)), br = as_u16x2(dpp_from_right(B));
        uint32_t s0 = __builtin_amdgcn_udot2(al, (u16x2){0, 18}, R, false);
        s0 = __builtin_amdgcn_udot2(bl, (u16x2){34, 49}, s0, false);
        s0 = __builtin_amdgcn_udot2(a, (u16x2){55, 49}, s0, false);
        s0 = __builtin_amdgcn_udot2(b, (u16x2){34, 18}, s0, false);
        uint32_t s1 = __builtin_amdgcn_udot2(bl, (u16x2){18, 34}, R, false);
        s1 = __builtin_amdgcn_udot2(a, (u16x2){49, 55}, s1, false);
        s1 = __builtin_amdgcn_udot2(b, (u16x2){49, 34}, s1, false);
        s1 = __builtin_amdgcn_udot2(ar, (u16x2){18, 0}, s1, false);
        uint32_t s2 = __builtin_amdgcn_udot2(bl, (u16x2){0, 18}, R, false);
        s2 = __builtin_amdgcn_udot2(a, (u16x2){34, 49}, s2, false);
        s2 = __builtin_amdgcn_udot2(b, (u16x2){55, 49}, s2, false);
        s2 = __builtin_amdgcn_udot2(ar, (u16x2){34, 18}, s2, false);
        uint32_t s3 = __builtin_amdgcn_udot2(a, (u16x2){18, 34}, R, false);
        s3 = __builtin_amdgcn_udot2(b, (u16x2){49, 55}, s3, false);
        s3 = __builtin_amdgcn_udot2(ar, (u16x2){49, 34}, s3, false);
        s3 = __builtin_amdgcn_udot2(br, (u16x2){18, 0}, s3, false);
        s0 += __builtin_amdgcn_ubfe(s0, 16, 1);
        s1 += __builtin_amdgcn_ubfe(s1, 16, 1);
        s2 += __builtin_amdgcn_ubfe(s2, 16, 1);
        s3 += __builtin_amdgcn_ubfe(s3, 16, 1);
        // (s0 >> 16, s1 >> 16) and (s2 >> 16, s3 >> 16) as 16-bit pairs, saturated to bytes
        const uint32_t word = sat_pk_u8(__builtin_amdgcn_perm(s1, s0, 0x07060302u)) |
                              (sat_pk_u8(__builtin_amdgcn_perm(s3, s2, 0x07060302u)) << 16);
        const int i = kDBRow0 + kDBRows * s + (r - 6);  // patch row
        if (st && s < kDBSeg && wc >= 1 && wc <= 11 && i < kDPH)
            reinterpret_cast<uint32_t*>(patch_slot + i * kDPW)[wc - 1] = word;
    }
}

// Sum over the wave by DPP (quad swaps, row shifts, row broadcasts; invalid source lanes read 0),
// the total read from lane 63: six DPP adds instead of six ds_bpermute rounds.
template <int kCtl, int kRowMask = 0xF>
__device__ __forceinline__ int dpp_or_zero(int v) {
    return __builtin_amdgcn_update_dpp(0, v, kCtl, kRowMask, 0xF, false);
}
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += dpp_or_zero<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_or_zero<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_or_zero<0x114>(v);  // row_shr:4
    v += dpp_or_zero<0x118>(v);  // row_shr:8  -> lane 15 of each row: the row's sum
    v += dpp_or_zero<0x142>(v);  // row_bcast:15
    v += dpp_or_zero<0x143>(v);  // row_bcast:31 -> lane 63: the wave's sum
    return __builtin_amdgcn_readlane(v, 63);
}

__global__ __launch_bounds__(256) void describe_kernel(StreamParams P) {
    __shared__ __attribute__((aligned(16))) uint8_t patch[kDKB][kDPH + 2][kDPW];  // + 2 padding rows
    __shared__ __attribute__((aligned(16))) uint8_t icw[4][kICR][kICW];
    __shared__ float s_ang[kDKB], s_ca[kDKB], s_sa[kDKB];
    __shared__ int s_pc[kDKB];  // offset of the keypoint's centre in its patch
    // 1-D grid: block b runs on XCD b & 7, and XCD x takes frames x, x + 8, ...
    // in turn, so one frame's keypoint windows meet in one L2 (and its
    // descriptors are written there for the matcher): 61.9-62.7 K -> 64.3 K frames/s
    const int nbx = (P.plan.kp_cap + kDKB - 1) / kDKB;
    int bxi;
    const int f = xcd_frame_item(nbx, P.nframes, bxi);
    if (f >= P.nframes) return;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int32_t* c2 = P.buf.cnt2 + f * kMaxLevels;
    int cnt[kMaxLevels];
    int total = 0;
#pragma unroll
    for (int q = 0; q < kMaxLevels; ++q) {  // all level counts in flight at once
        cnt[q] = q < P.plan.nlevels ? c2[q] : 0;
        total += cnt[q];
    }
    if (bxi == 0 && threadIdx.x == 0) {
        P.buf.nkp[f] = total;
        if (total > P.plan.kp_cap) atomicOr(&P.buf.status[f], 1);
    }
    const int nk = min(total, P.plan.kp_cap);
    if (bxi * kDKB >= nk) return;  // whole block idle (uniform)
    // rBRIEF pattern points of this lane's 4 bits (independent of the keypoint: issued first)
    float4 pat[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pat[q] = reinterpret_cast<const float4*>(c_pattern_f)[q * 64 + lane];
    // ICAngles disk membership of this lane's 16 samples (u = column, v = row): keypoint independent
    // keypoint (level, index, key) of this wave's 4 slots, keys requested together
    int lv[kDKW], ix[kDKW];
    uint32_t keys[kDKW];
    float resps[kDKW];
#pragma unroll
    for (int kk = 0; kk < kDKW; ++kk) {
        int l = 0, i = min(bxi * kDKB + wv * kDKW + kk, nk - 1);
#pragma unroll
        for (int q = 0; q + 1 < kMaxLevels; ++q)
            if (l == q && q + 1 < P.plan.nlevels && i >= cnt[q]) {
                i -= cnt[q];
                l = q + 1;
            }
        lv[kk] = l;
        ix[kk] = i;
        keys[kk] = P.buf.cand[(int64_t)f * P.plan.cand_stride + P.plan.L[l].cand_off + i];
        resps[kk] = P.buf.resp[(int64_t)f * P.plan.cand_stride + P.plan.L[l].cand_off + i];
    }
    // ---- phase 1: every keypoint of this wave requests both windows first (one load latency
    // covers the wave's kDKW keypoints), then each is staged in LDS and gets its IC angle
    constexpr int kIW = 31 * (kICW / 4);
    uint32_t ivs[kDKW][5], pvs[kDKW][kDBRaw];
    int db_s = 0;
#pragma unroll
    for (int q = 1; q < kDBSeg; ++q) db_s += lane >= kDBBase[q];
    const int db_k = lane - kDBBase[db_s];  // lanes >= 56: band 4 past its words (loads in range, no store)
    const int db_hw = db_s == 0 ? kDBHalfW[0] : db_s == 4 ? kDBHalfW[4] : kDBHalfW[1];
    const bool db_st = db_k >= 1 && db_k <= kDBBase[db_s + 1] - kDBBase[db_s] - 2;  // not a band halo word
    int db_wcs[kDKW];
#pragma unroll
    for (int kk = 0; kk < kDKW; ++kk) {  // slots past nk read the clamped last keypoint (unused)
        const int l = lv[kk];
        const LevelGeom& G = P.plan.L[l];
        const uint32_t key = keys[kk];
        const int kx = key & 0xFFF, ky = (key >> 12) & 0xFFF;
        const float scale = G.scale;
        const float sc = 1.f / scale;
        const int cxb = cv_round_f((float)kx * scale * sc), cyb = cv_round_f((float)ky * scale * sc);
        const int a0 = (cxb - kDPR) & ~3;
        const int ai = (kx - 15) & ~3;
        const int step = level_pitch(P, l);
        const uint8_t* img = level_ptr(P, f, l) + (int64_t)(ky - 15) * step + ai;
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const int ec = min(64 * t + lane, kIW - 1);
            const int rc = ec / (kICW / 4), wc = ec - rc * (kICW / 4);
            ivs[kk][t] = *reinterpret_cast<const uint32_t*>(img + (int64_t)rc * step + 4 * wc);
        }
        {  // raw rows cyb - 22 + 10 s .. + 15 of word db_wc of [a0 - 4, a0 + 48)
            const int sr = min(db_s, kDBSeg - 1);
            // the band's first word: the one left of the word holding cx - halfwidth (raw word
            // index ((x - a0) >> 2) + 1); <= 12 for every lane of the band
            const int db_wc = min(((cxb - db_hw - a0) >> 2) + db_k, 12);
            db_wcs[kk] = db_wc;
            const uint8_t* rw = level_ptr(P, f, l) + (int64_t)(cyb - kDPR - 3 + kDBRow0 + kDBRows * sr) * step +
                                a0 - 4 + 4 * db_wc;
#pragma unroll
            for (int t = 0; t < kDBRaw; ++t) pvs[kk][t] = *reinterpret_cast<const uint32_t*>(rw + (int64_t)t * step);
        }
    }
#pragma unroll
    for (int kk = 0; kk < kDKW; ++kk) {
        const int slot = wv * kDKW + kk;
        const int k = bxi * kDKB + slot;
        if (k >= nk) continue;  // wave-uniform
        const int l = lv[kk];
        const LevelGeom& G = P.plan.L[l];
        const uint32_t key = keys[kk];
        const int kx = key & 0xFFF, ky = (key >> 12) & 0xFFF;
        const float scale = G.scale;
        const float ptx = (float)kx * scale, pty = (float)ky * scale;
        const float sc = 1.f / scale;
        const int cxb = cv_round_f(ptx * sc);  // orb.cpp: center = &img(cvRound(pt*sc))
        const int a0 = (cxb - kDPR) & ~3;
        const int ai = (kx - 15) & ~3;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 5; ++t) reinterpret_cast<uint32_t*>(&icw[wv][0][0])[64 * t + lane] = ivs[kk][t];
        const int db_wc = db_wcs[kk];
        describe_blur_rows(pvs[kk], &patch[slot][0][0], db_s, db_wc, db_st);
        __builtin_amdgcn_wave_barrier();
        // m10 = sum u * I, m01 = sum v * I over the disk (integer: any order)
        int m10, m01;
        {
            const int r = lane >> 1, hh = lane & 1;  // window row (31: lanes 62, 63, zero weights), word half
            const uint32_t* rowp = reinterpret_cast<const uint32_t*>(&icw[wv][0][0]) + r * (kICW / 4) + 5 * hh;
            const uint2* tp = reinterpret_cast<const uint2*>(&c_ictab.w[(kx - 15) & 3][r][5 * hh][0]);
            uint32_t dU = 0, d1 = 0;
#pragma unroll
            for (int q = 0; q < 5; ++q) {  // word 9 (the next row's first) has zero weights
                const uint32_t I4 = rowp[q];
                const uint2 t = tp[q];
                dU = __builtin_amdgcn_udot4(I4, t.x, dU, false);
                d1 = __builtin_amdgcn_udot4(I4, t.y, d1, false);
            }
            m10 = (int)dU - 15 * (int)d1;
            m01 = (r - 15) * (int)d1;
        }
        (void)ai;
        m10 = wave_sum_dpp(m10);  // integer sums: the order does not matter
        m01 = wave_sum_dpp(m01);
        if (lane == 0) {
            const float angle = fast_atan2((float)m01, (float)m10);
            s_ang[slot] = angle;
            s_pc[slot] = kDPR * kDPW + (cxb - a0);
            dvo_keypoint kp;
            kp.x = ptx;
            kp.y = pty;
            kp.size = 31 * scale;
            kp.angle = angle;
            kp.response = resps[kk];
            kp.octave = l;
            kp.class_id = -1;
            P.buf.kps[(int64_t)f * P.plan.kp_cap + k] = kp;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // ---- phase 2: the workgroup's 16 rotations in one evaluation (orb.cpp: (float)cos / sin of
    // angle * (float)(CV_PI / 180))
    if (threadIdx.x < kDKB) {
        const float ang = s_ang[threadIdx.x] * (float)(M_PI / 180.f);
        double sd, cd;
        sincos((double)ang, &sd, &cd);
        s_ca[threadIdx.x] = (float)cd;
        s_sa[threadIdx.x] = (float)sd;
    }
    __syncthreads();
    // ---- phase 3: rBRIEF on the blurred level (orb.cpp computeOrbDescriptors, WTA_K 2).  cvRound of a
    // rotated coordinate v (|v| < 20) by the rounding constant M = 1.5 * 2^23: the float sum v + M is
    // M + cvRound(v) (round to nearest, ties to even, as cvRound), so its bit pattern is Mi + cvRound(v)
    // and (Y << 6) + X of a sample's two sums is its patch offset + 65 Mi (mod 2^32): two integer
    // operations per sample instead of two round-and-converts and a multiply.
    constexpr float kRoundM = 12582912.0f;
    constexpr uint32_t kRoundC = 65u * 0x4B400000u;  // 65 x the bit pattern of M, mod 2^32
    static_assert(sizeof(patch) < 65536, "patch offsets");
    const uint8_t* pbytes = &patch[0][0][0];
    for (int kk = 0; kk < kDKW; ++kk) {
        const int slot = wv * kDKW + kk;
        const int k = bxi * kDKB + slot;
        if (k >= nk) break;
        const float ca = s_ca[slot], sa = s_sa[slot];
        const uint32_t pc = (uint32_t)(slot * (kDPH + 2) * kDPW + s_pc[slot]) - kRoundC;
        // (x, y) = (px ca - py sa, px sa + py ca) as packed products and one packed sum (-(py sa) is
        // (-sa) py exactly), then + M
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 cs = {ca, sa}, nsc = {-sa, ca};
        const auto at = [&](float px, float py) {
            const f32x2 r = (cs * (f32x2){px, px} + nsc * (f32x2){py, py}) + (f32x2){kRoundM, kRoundM};
            const uint32_t X = __float_as_uint(r.x), Y = __float_as_uint(r.y);
            return (uint32_t)pbytes[(Y << 6) + X + pc];
        };
        uint32_t t0[4], t1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            t0[q] = at(pat[q].x, pat[q].y);
            t1[q] = at(pat[q].z, pat[q].w);
        }
        unsigned long long words[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) words[q] = __ballot(t0[q] < t1[q]);
        if (lane < 4) {
            unsigned long long* d = reinterpret_cast<unsigned long long*>(P.buf.desc + ((int64_t)f * P.plan.kp_cap + k) * 32);
            d[lane] = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
        }
    }
}

__global__ void test_retain_best_kernel(float* resp, uint32_t* payload, int32_t* tmp, int n, int npoints, int depth,
                                        int semantics, int* kout) {
    __shared__ int lds[64];
    int k = retain_best_block(HarrisVals{resp, payload}, n, npoints, depth, tmp, tmp + n + 1, lds, semantics);
    if (threadIdx.x == 0) *kout = k;
}

}  // namespace

hipError_t launch_blur(const StreamParams& P, hipStream_t s) {
    hipLaunchKernelGGL(blur_kernel, dim3(P.plan.total_tiles * xcd_frames(P.nframes)), dim3(256), 0, s, P);
    return hipGetLastError();
}


namespace {
hipError_t launch_orb_frames(const StreamParams& P, hipStream_t s, hipEvent_t* ev) {
    const Plan& pl = P.plan;
    const int F = P.nframes;
    mark(ev, 0, 0, s);
    // staged tiles fit when both ratios are <= 1.25: 256 * 1.25 + 12 bytes <= kRsW words,
    // 32 * 1.25 + 2 rows <= kRsRows
    auto lds_ok = [&](int l) { return 4 * pl.L[l - 1].w <= 5 * pl.L[l].w && 4 * pl.L[l - 1].h <= 5 * pl.L[l].h; };
    for (int l = 1; l < pl.nlevels; ++l) {
        const bool lds = lds_ok(l);
        if (pl.semantics == kOcv32) {
            if (lds)  // the 3.2 tables through the same staged tiles
                hipLaunchKernelGGL(resize_level_lds_kernel<true>,
                                   dim3((pl.L[l].w + 255) / 256 * ((pl.L[l].h + 4 * kRsLR - 1) / (4 * kRsLR)) *
                                        xcd_frames(F)),
                                   dim3(256), 0, s, P, l, (pl.L[l].w + 255) / 256);
            else
                hipLaunchKernelGGL(resize_level_ocv32_kernel, dim3((pl.L[l].w + 63) / 64, (pl.L[l].h + 3) / 4, F),
                                   dim3(256), 0, s, P, l);
            continue;
        }
        if (lds)
            hipLaunchKernelGGL(resize_level_lds_kernel<false>,
                               dim3((pl.L[l].w + 255) / 256 * ((pl.L[l].h + 4 * kRsLR - 1) / (4 * kRsLR)) * xcd_frames(F)),
                               dim3(256), 0, s, P, l, (pl.L[l].w + 255) / 256);
        else  // level pairs whose rounded sizes differ by more than 1.25x: tiny frames (8x8: levels 4->5, 6->7)
            hipLaunchKernelGGL(resize_level_kernel, dim3((pl.L[l].w + 255) / 256, (pl.L[l].h + 4 * kRsR - 1) / (4 * kRsR), F),
                               dim3(256), 0, s, P, l);
    }
    mark(ev, 0, 1, s);
    mark(ev, 1, 0, s);
    mark(ev, 1, 1, s);

    mark(ev, 2, 0, s);
    if (pl.total_strips > 0)
        hipLaunchKernelGGL(fast_strip_kernel, dim3(pl.total_strips * kFastSeg(F) * xcd_frames(F)), dim3(kFastNT), 0,
                           s, P, kFastSeg(F));
    mark(ev, 2, 1, s);
    mark(ev, 3, 0, s);
    if (F <= kSelCallFrames)
        hipLaunchKernelGGL((select_fast_kernel<kSelNTCall, kSelLdsCall>), dim3(pl.nlevels, F), dim3(kSelNTCall), 0, s, P, 0);
    else if (kSelNT0 != kSelNT) {  // level 0 (the longest lists) on wider blocks, the other levels as before
        hipLaunchKernelGGL((select_fast_kernel<kSelNT0, false>), dim3(1, F), dim3(kSelNT0), 0, s, P, 0);
        hipLaunchKernelGGL((select_fast_kernel<kSelNT, false>), dim3(pl.nlevels - 1, F), dim3(kSelNT), 0, s, P, 1);
    } else {
        hipLaunchKernelGGL((select_fast_kernel<kSelNT, false>), dim3(pl.nlevels, F), dim3(kSelNT), 0, s, P, 0);
    }
    hipLaunchKernelGGL(harris_kernel, dim3(harris_blocks_x(pl), pl.nlevels, F), dim3(256), 0, s, P);
    if (F <= kSelCallFrames)
        hipLaunchKernelGGL((select_harris_kernel<kSelNTCall, kSelLdsCall>), dim3(pl.nlevels, F), dim3(kSelNTCall), 0, s,
                           P);
    else
        hipLaunchKernelGGL((select_harris_kernel<kSelNT, false>), dim3(pl.nlevels, F), dim3(kSelNT), 0, s, P);
    mark(ev, 3, 1, s);
    mark(ev, 4, 0, s);
    hipLaunchKernelGGL(describe_kernel, dim3(xcd_frames(F) * ((pl.kp_cap + kDKB - 1) / kDKB)), dim3(256), 0, s, P);
    mark(ev, 4, 1, s);
    return hipGetLastError();
}

// Frames [f0, f0 + n) of P as a batch of their own: every per-frame buffer the detection
// kernels index by frame advanced by f0 frames.
StreamParams frame_group(const StreamParams& P, int f0, int n) {
    StreamParams Q = P;
    const Plan& pl = P.plan;
    const int64_t f = f0;
    Q.nframes = n;
    Q.frames = P.frames + f * P.frame_stride;
    Q.buf.pyr += f * pl.pyr_stride;
    Q.buf.blur += f * pl.blur_stride;
    Q.buf.band_cnt += f * pl.total_bands * kBandRows;
    Q.buf.band_cand += f * pl.band_cand_stride;
    Q.buf.cand += f * pl.cand_stride;
    Q.buf.resp += f * pl.cand_stride;
    Q.buf.sel_tmp += f * 2 * pl.cand_stride;
    Q.buf.cnt1 += f * kMaxLevels;
    Q.buf.cnt2 += f * kMaxLevels;
    Q.buf.kps += f * pl.kp_cap;
    Q.buf.desc += f * pl.kp_cap * 32;
    Q.buf.nkp += f;
    Q.buf.status += f;
    return Q;
}
}  // namespace

// DVO_ORB_GROUP > 0: a batch of more than that many frames runs its detection (pyramid -> FAST ->
// selections -> Harris -> describe) over ceil(F / DVO_ORB_GROUP) groups of equal size (+-1) in turn
// (the group's pyramid is still in the caches when Harris and describe
// re-read it).  Two-stream bench, whole batch 87.6-88.2 K; groups of 64 -8 %, 128 -2 %, 256
// +0.8 to +1.5 %, 512 / 1024 +-0 (profiles/r04o_ab_describe_sincos_groups.txt, r04p_ab*.txt,
// r04q_ab_orb_groups.txt); one stream alone is slower (small launches), two overlap better.  Re-swept
// at batch 3072 on the round-4 final kernels: 256 90.8 K, 384 91.7 K, 512 91.7 K, 768 92.0 K, none
// 90.6 K at C3; 137.1 / 139.0 / 140.4 / 141.1 / 139.7 K at C2 (profiles/r05b_ab_c3_orb_groups.txt,
// r05b_ab_c2_orb_groups.txt).  Stage events: one table of 2 x 5 per group (orb_groups), summed per
// stage.
#ifndef DVO_ORB_GROUP
#define DVO_ORB_GROUP 768
#endif
int orb_groups(int nframes) {
    const int grp = DVO_ORB_GROUP;
    return grp > 0 && nframes > grp ? (nframes + grp - 1) / grp : 0;
}
hipError_t launch_orb(const StreamParams& P, hipStream_t s, hipEvent_t* ev, hipEvent_t* group_ev) {
    const int F = P.nframes, G = orb_groups(F);
    if (G == 0) return launch_orb_frames(P, s, ev);
    for (int g = 0; g < G; ++g) {
        const int f0 = (int)((int64_t)F * g / G), f1 = (int)((int64_t)F * (g + 1) / G);
        const hipError_t e = launch_orb_frames(frame_group(P, f0, f1 - f0), s, group_ev ? group_ev + 10 * g : nullptr);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

namespace {
__global__ __launch_bounds__(256) void feature_rotate_kernel(FeatSlots f, int rotate) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < f.words[b]; i += gridDim.x * 256) {
            if (rotate) {
                const uint32_t cur = f.a[0][b][i], prev = f.a[2][b][i];
                f.a[1][b][i] = cur;
                f.a[0][b][i] = prev;
                f.a[2][b][i] = cur;
            } else {
                f.a[2][b][i] = f.a[1][b][i];
            }
        }
}
}  // namespace

hipError_t launch_feature_rotate(const FeatSlots& f, int rotate, hipStream_t s) {
    hipLaunchKernelGGL(feature_rotate_kernel, dim3(64), dim3(256), 0, s, f, rotate);
    return hipGetLastError();
}

hipError_t launch_test_retain_best(float* d_resp, uint32_t* d_payload, int32_t* d_tmp, int n, int n_points, int depth,
                                   int semantics, int* d_k, hipStream_t s) {
    hipLaunchKernelGGL(test_retain_best_kernel, dim3(1), dim3(kSelNT), 0, s, d_resp, d_payload, d_tmp, n, n_points,
                       depth, semantics, d_k);
    return hipGetLastError();
}

}  // namespace dvo
