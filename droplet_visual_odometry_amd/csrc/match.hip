// Brute-force Hamming matching for gfx950: the MI355X replacement of
// cv::BFMatcher(NORM_HAMMING, crossCheck=True).match(prev_desc, cur_desc)
// (scripts/visual_odometry_v3.py:75 and :219), followed by the reference's own
// `sorted(matches, key=lambda x: x.distance)` (v3:221, a stable sort, so the
// order is (distance, queryIdx)) and KeyPoint_convert of the matched keypoints
// (v3:355, v3:358).
//
// nn_mfma_kernel: forward and backward nearest neighbours of a pair on the
// matrix cores (block-scaled fp4 MFMA over descriptor bits as +-1.0), for the batched stream
// and, through a one-pair parameter block, for the per-call C-ABI.
// crosscheck_*_kernel: mutual-NN filter, then a bitonic sort of the unique
// keys (distance << 16 | queryIdx) in LDS, then the point gather.
#include <algorithm>
#include <cfloat>
#include <climits>

#include "dvo_internal.h"

namespace dvo {
namespace {

// Forward + backward nearest neighbours of one stream pair on the matrix cores.
// The operands are the packed 32-byte descriptors (P.buf.desc, as described;
// the per-call path's caller buffers), expanded in registers on the way in:
// every descriptor bit becomes an operand element, +1 on the query side and
// -1 on the train side when set (the opposite sign when clear), scaled so the
// accumulator is D = -4096 s where s = q.t = 256 - 2 * Hamming(q, t), exact
// (format below).  Then key = 2^20 + D + index =
// Hamming * 8192 + index (index < 8192): one add per element and direction,
// and the minimum key is OpenCV's nearest neighbour with its first-index tie
// rule.  A wave owns 64 queries (two 32-row strips, A fragments resident in
// VGPRs); the workgroup streams the trains through LDS 64 at a time (2 KB of
// packed rows per stage, 8 KB expanded), double-buffered (the next stage's
// global loads are in flight during this stage's MFMAs; one barrier per
// stage), 16-byte chunks XOR-swizzled by train so the b128 fragment reads are
// conflict-free.  Forward keys fold into a per-register running minimum (the
// lane's column changes, its rows do not); backward keys fold over the lane's
// 32 rows (v_min3), into LDS, then a global atomicMin per train in the
// (Hamming << 16 | index) form the cross check reads (the re-encoding is
// monotone, so the minimum is the same).  Workgroups are grouped by XCD
// (blocks b and b + 8 share one) so the query blocks of a pair stream its
// trains through one L2.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kMWaves = 4, kMQB = 64 * kMWaves, kMStage = 64;
constexpr int kKeyBase = 1 << 20;     // 256 * 4096

// Operand format: v_mfma_scale_f32_32x32x64_f8f6f4 on e2m1 (fp4) operands,
// +-1.0 per descriptor bit (a nibble each: 32 bits of a descriptor word = one
// 16-byte chunk), the train side's block scale 2^12, so the f32 accumulator is
// D = -4096 s exactly (integers < 2^21); keys are formed in f32 (exact below
// 2^24) and compared as the bit patterns of non-negative floats (ordered like
// the values).  Twice the K per clock of the i8 form (v_mfma_i32_32x32x32_i8 on
// +-64 bytes, round 3's first matcher) and half its LDS bytes per train.
constexpr int kMChunks = 8;   // 16-byte operand chunks per train
constexpr int kMKs = 4;       // MFMAs per 32x32 block
typedef v16f acc_t;
// 32 descriptor bits to 32 e2m1 nibbles (a permutation of the bit order that A
// and B share, so the dot product is unchanged): nibble-spread of byte k is
// L | H << 4, L / H the byte's low / high nibble spread to bytes by
// (n * 0x204081) & 0x01010101; bit 3 of a nibble is the e2m1 sign, so
// base ^ (spread << 3) is 0x2 (+1.0) or 0xA (-1.0).  Query base 0xAA.. (set ->
// +1), train base 0x22.. (set -> -1).
__device__ __forceinline__ v4i expand_chunk(uint32_t bits, uint32_t base) {
    v4i r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t L = (((bits >> (8 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
        const uint32_t H = (((bits >> (8 * k + 4)) & 0xFu) * 0x00204081u) & 0x01010101u;
        r[k] = (int)(base ^ (L << 3) ^ (H << 7));
    }
    return r;
}
constexpr uint32_t kExpQ = 0xAAAAAAAAu, kExpT = 0x22222222u;
__device__ __forceinline__ acc_t mfma_chunk(v4i a, v4i b, acc_t c) {
    const v8i A = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, B = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    // cbsz = blgp = 4 (e2m1); E8M0 scales 127 (1.0) for A, 139 (2^12) for B
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 4, 4, 0, 0x7F7F7F7F, 0, 0x8B8B8B8B);
}
// key bits of accumulator element a plus the exact integer c (both as f32)
__device__ __forceinline__ int key_add(float a, float c) { return __float_as_int(a + c); }
__device__ __forceinline__ int key_value(int kbits) { return (int)__int_as_float(kbits); }
constexpr int kKeyNone = 0x7F000000;  // bits of ~1.7e38f: above every key, not a NaN
constexpr int kChunkMask = kMChunks - 1;
__device__ __forceinline__ int key_old(int k) { return ((k >> 13) << 16) | (k & 8191); }

// One stage of 64 trains against the wave's 64 queries.  Backward key of
// register g of strip s: D + 2^20 + the query row (rowb = 2^20 + qs + 4h).
template <bool kFull>
__device__ __forceinline__ void nn_stage(const v4i* btc, int* cmin, const v4i (&A)[2][kMKs], int (&best)[2][16], int t0,
                                         int nt, int r, int h, int rowb, int nq) {
    // the accumulators start at the backward key base of their rows, 2^20 + row (exact,
    // loop-invariant: the MFMA's C input), so they end as backward keys; forward keys add the train
    // index and carry the row, a constant of each forward minimum, taken off at the end
    const float rbf = (float)rowb;
    acc_t rb0, rb1;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        const int goff = (g & 3) + 8 * (g >> 2);
        rb0[g] = rbf + (float)goff;
        rb1[g] = rbf + (float)(32 + goff);
    }
#pragma unroll 1
    for (int tt = 0; tt < kMStage / 32; ++tt) {
        const int j = t0 + 32 * tt + r;
        const float cf = (float)(j < nt ? j : (1 << 30));
        acc_t acc0 = rb0, acc1 = rb1;
#pragma unroll
        for (int ks = 0; ks < kMKs; ++ks) {
            const v4i B = btc[(32 * tt + r) * kMChunks + ((2 * ks + h) ^ (r & kChunkMask))];
            acc0 = mfma_chunk(A[0][ks], B, acc0);
            acc1 = mfma_chunk(A[1][ks], B, acc1);
        }
        int cm = 0x7FFFFFFF;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int goff = (g & 3) + 8 * (g >> 2);
            best[0][g] = min(best[0][g], key_add(acc0[g], cf));
            best[1][g] = min(best[1][g], key_add(acc1[g], cf));
            int k0 = __float_as_int(acc0[g]), k1 = __float_as_int(acc1[g]);
            if (!kFull) {
                k0 = rowb - kKeyBase + goff < nq ? k0 : kKeyNone;
                k1 = rowb - kKeyBase + 32 + goff < nq ? k1 : kKeyNone;
            }
            cm = min(cm, min(k0, k1));
        }
        if (j < nt) atomicMin(&cmin[32 * tt + r], cm);
    }
}

// Operands of one launch: pair p's queries are the rows at q0 + p * stride,
// its trains the rows at t0 + p * stride (32 bytes each); counts from nkp[p],
// nkp[p + 1] (the stream) or nq_fix / nt_fix (the per-call pair, >= 0).
struct NnOperands {
    const uint8_t* q0;
    const uint8_t* t0;
    int64_t stride;
    int nq_fix, nt_fix;
};

// tsplit > 1 (the per-call path: one pair, so a short grid) gives each
// workgroup a contiguous 1/tsplit of the train stages and folds the forward
// keys with atomicMin too (fwd pre-filled with 0x7F7F7F7F).
// Resident waves per SIMD asked of the compiler (165 VGPRs unconstrained = 3).
#ifndef DVO_MATCH_WAVES
#define DVO_MATCH_WAVES 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DVO_MATCH_WAVES)))
void nn_mfma_kernel(StreamParams P, NnOperands O, int pairs, int nqb, int tsplit) {
    __shared__ v4i bt[2][kMStage * kMChunks];
    __shared__ int colmin[2][kMStage];
    const int nwg = gridDim.x;  // a multiple of 8
    const int L0 = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
    const int L = L0 / tsplit, ts = L0 - L * tsplit;
    const int p = L / nqb, qb = L - p * nqb;
    if (p >= pairs) return;
    const int cap = P.plan.kp_cap;
    const int fp = pair_frame(P, p);  // the pair's previous frame; its current frame is fp + 1
    const int nq = O.nq_fix >= 0 ? O.nq_fix : min(P.buf.nkp[fp], cap);
    const int nt = O.nt_fix >= 0 ? O.nt_fix : min(P.buf.nkp[fp + 1], cap);
    const int qbase = qb * kMQB;
    if (qbase >= nq) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const uint4* XQ = reinterpret_cast<const uint4*>(O.q0 + fp * O.stride);
    const uint2* XT = reinterpret_cast<const uint2*>(O.t0 + fp * O.stride);
    int32_t* fwd = P.buf.nn + (int64_t)p * cap;
    int32_t* bwd = P.buf.nn + ((int64_t)P.nframes + p) * cap;
    const int qs = qbase + wid * 64;  // this wave's first query
    v4i A[2][kMKs];
    int best[2][16];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const int q = qs + 32 * s2 + r;
        const uint4 w0 = q < nq ? XQ[2 * (int64_t)q] : make_uint4(0, 0, 0, 0);
        const uint4 w1 = q < nq ? XQ[2 * (int64_t)q + 1] : make_uint4(0, 0, 0, 0);
        const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int ks = 0; ks < kMKs; ++ks) {  // chunk 2 ks + h; a zero fragment past nq
            const int ch = 2 * ks + h;
            const uint32_t bits = wd[ch];
            A[s2][ks] = q < nq ? expand_chunk(bits, kExpQ) : (v4i){0, 0, 0, 0};
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) best[s2][g] = 0x7FFFFFFF;
    }
    // backward key base of register g: 2^20 + row(g); rows past nq never win (partial waves only)
    const int rowb = kKeyBase + qs + 4 * h;
    const bool full = qs + 64 <= nq;
    const int nst_all = (nt + kMStage - 1) / kMStage;
    const int st0 = (int)((int64_t)nst_all * ts / tsplit), nst = (int)((int64_t)nst_all * (ts + 1) / tsplit);
    // a stage: 64 trains x 32 bytes, 8 bytes (chunks 4 qd .. 4 qd + 3) per thread
    const int tr = threadIdx.x >> 2, qd = threadIdx.x & 3;
    uint2 v;
    auto load_stage = [&](int st) { v = XT[(int64_t)min(st * kMStage + tr, nt - 1) * 4 + qd]; };  // clamped
    auto store_stage = [&](int st, int b) {
        const bool in = st * kMStage + tr < nt;  // zero operands past nt
        constexpr int kPer = kMChunks / 4;       // chunks of this thread's 8 bytes
#pragma unroll
        for (int c = 0; c < kPer; ++c) {
            const int ch = kPer * qd + c;
            const uint32_t bits = c == 0 ? v.x : v.y;
            bt[b][tr * kMChunks + (ch ^ (tr & kChunkMask))] = in ? expand_chunk(bits, kExpT) : (v4i){0, 0, 0, 0};
        }
        if (threadIdx.x < kMStage) colmin[b][threadIdx.x] = 0x7FFFFFFF;
    };
    if (st0 < nst) {
        load_stage(st0);
        store_stage(st0, 0);
    }
    __syncthreads();
    for (int st = st0; st < nst; ++st) {
        const int cur = (st - st0) & 1;
        if (st + 1 < nst) load_stage(st + 1);
        if (full) nn_stage<true>(bt[cur], colmin[cur], A, best, st * kMStage, nt, r, h, rowb, nq);
        else nn_stage<false>(bt[cur], colmin[cur], A, best, st * kMStage, nt, r, h, rowb, nq);
        if (st + 1 < nst) store_stage(st + 1, cur ^ 1);
        __syncthreads();
        const int t = st * kMStage + threadIdx.x;
        if (threadIdx.x < kMStage && t < nt && colmin[cur][threadIdx.x] != 0x7FFFFFFF)
            atomicMin(&bwd[t], key_old(key_value(colmin[cur][threadIdx.x])));
    }
    // forward: minimum over the 32 lanes of each half (they hold the 32 columns)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            int vv = best[s2][g];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) vv = min(vv, __shfl_xor(vv, o));
            const int qr = qs + 32 * s2 + (g & 3) + 8 * (g >> 2) + 4 * h;
            if (r == g && qr < nq) {
                if (tsplit > 1) {
                    if (st0 < nst) atomicMin(&fwd[qr], key_old(key_value(vv) - qr));
                } else {
                    fwd[qr] = nt > 0 ? key_old(key_value(vv) - qr) : -1;
                }
            }
        }
}

constexpr int kXNT = 1024;
constexpr int kMaxSort = 8192;

// Mutual-NN / legacy cross check + stable (distance, queryIdx) order.
// Writes m keys sorted ascending into keys[] (LDS) and returns m.
__device__ int crosscheck_sort(const int32_t* fwd, const int32_t* bwd, int nq, int nt, int mode, uint32_t* keys,
                               int* scan_lds) {
    __shared__ int s_m;
    if (threadIdx.x == 0) s_m = 0;
    __syncthreads();
    if (mode == 2) {
        // OpenCV 3.x: for each train t (reverse NN q = bwd[t]), keep per query the
        // train with the smallest distance, first t on ties.
        for (int q = threadIdx.x; q < nq; q += kXNT) keys[q] = 0xFFFFFFFFu;
        __syncthreads();
        for (int t = threadIdx.x; t < nt; t += kXNT) {
            int b = bwd[t];
            if (b < 0 || (b >> 16) > 256) continue;  // -1 or the untouched 0x7F7F7F7F fill
            int q = b & 0xFFFF, d = b >> 16;
            atomicMin(&keys[q], ((uint32_t)d << 16) | (uint32_t)t);
        }
        __syncthreads();
        // convert to (d << 16 | q) keys; the train index is recovered from bwd later
        for (int q = threadIdx.x; q < nq; q += kXNT) {
            uint32_t k = keys[q];
            keys[kMaxSort + q] = k;  // stash (d << 16 | t) in the upper half
        }
        __syncthreads();
        for (int q = threadIdx.x; q < nq; q += kXNT) {
            uint32_t k = keys[kMaxSort + q];
            keys[q] = 0xFFFFFFFFu;
            if (k != 0xFFFFFFFFu) {
                int slot = atomicAdd(&s_m, 1);
                keys[slot] = ((k >> 16) << 16) | (uint32_t)q;
            }
        }
    } else {
        for (int q = threadIdx.x; q < nq; q += kXNT) {
            int f = fwd[q];
            if (f < 0 || (f >> 16) > 256) continue;  // -1 or the untouched 0x7F7F7F7F fill (split trains, nt = 0)
            int t = f & 0xFFFF;
            if (mode == 1 && (bwd[t] & 0xFFFF) != q) continue;
            int slot = atomicAdd(&s_m, 1);
            keys[slot] = ((uint32_t)(f >> 16) << 16) | (uint32_t)q;
        }
    }
    __syncthreads();
    const int m = s_m;
    int n2 = 1;
    while (n2 < m) n2 <<= 1;
    for (int i = m + threadIdx.x; i < n2; i += kXNT) keys[i] = 0xFFFFFFFFu;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += kXNT) {
                int ixj = i ^ j;
                if (ixj > i) {
                    uint32_t a = keys[i], b = keys[ixj];
                    bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    (void)scan_lds;
    return m;
}

__global__ __launch_bounds__(kXNT) void crosscheck_stream_kernel(StreamParams P, int mode) {
    __shared__ uint32_t keys[2 * kMaxSort];
    __shared__ int scan_lds[32];
    const int p = blockIdx.x;
    const int cap = P.plan.kp_cap;
    const int fp = pair_frame(P, p);
    const int nq = min(P.buf.nkp[fp], cap), nt = min(P.buf.nkp[fp + 1], cap);
    const int32_t* fwd = P.buf.nn + (int64_t)p * cap;
    const int32_t* bwd = P.buf.nn + ((int64_t)P.nframes + p) * cap;
    const int m = crosscheck_sort(fwd, bwd, nq, nt, mode, keys, scan_lds);
    const dvo_keypoint* ka = P.buf.kps + (int64_t)fp * cap;
    const dvo_keypoint* kb = P.buf.kps + (int64_t)(fp + 1) * cap;
    int32_t* mq = P.buf.mq + (int64_t)p * cap;
    int32_t* mt = P.buf.mt + (int64_t)p * cap;
    float* md = P.buf.md + (int64_t)p * cap;
    float* pts = P.buf.pts + (int64_t)p * cap * 4;
    for (int i = threadIdx.x; i < m; i += kXNT) {
        const uint32_t k = keys[i];
        const int q = k & 0xFFFF;
        const int t = mode == 2 ? (int)(keys[kMaxSort + q] & 0xFFFF) : (fwd[q] & 0xFFFF);
        mq[i] = q;
        mt[i] = t;
        md[i] = (float)(k >> 16);
        pts[4 * i + 0] = ka[q].x;
        pts[4 * i + 1] = ka[q].y;
        pts[4 * i + 2] = kb[t].x;
        pts[4 * i + 3] = kb[t].y;
    }
    if (threadIdx.x == 0) P.buf.nmatch[p] = m;
}

// Single pair (C-ABI dvo_bf_match_hamming): output in queryIdx order like
// OpenCV's raw list (the caller's Python applies the stable distance sort), so
// no sort is needed: the kept queries are compacted in ascending q with a
// block-wide exclusive scan, 1024 queries per round.
__global__ __launch_bounds__(kXNT) void crosscheck_pair_kernel(const int32_t* fwd, const int32_t* bwd, int nq, int nt,
                                                               int mode, dvo_dmatch* out, int* m_out) {
    __shared__ uint32_t best[kMaxSort];  // mode 2: per query min (d << 16 | t) over the trains naming it
    __shared__ int s_wave[kXNT / 64];
    __shared__ int s_carry;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (mode == 2) {
        // OpenCV 3.x: for each train t (reverse NN q = bwd[t]), keep per query the
        // train with the smallest distance, first t on ties.
        for (int q = threadIdx.x; q < nq; q += kXNT) best[q] = 0xFFFFFFFFu;
        __syncthreads();
        for (int t = threadIdx.x; t < nt; t += kXNT) {
            const int b = bwd[t];
            if (b < 0 || (b >> 16) > 256) continue;  // -1 or the untouched 0x7F7F7F7F fill
            atomicMin(&best[b & 0xFFFF], ((uint32_t)(b >> 16) << 16) | (uint32_t)t);
        }
    }
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int q0 = 0; q0 < nq; q0 += kXNT) {
        const int q = q0 + threadIdx.x;
        bool keep = false;
        int t = 0, d = 0;
        if (q < nq) {
            if (mode == 2) {
                const uint32_t k = best[q];
                keep = k != 0xFFFFFFFFu;
                t = (int)(k & 0xFFFF);
                d = (int)(k >> 16);
            } else {
                const int f = fwd[q];
                if (f >= 0) {
                    t = f & 0xFFFF;
                    d = f >> 16;
                    keep = mode != 1 || (bwd[t] & 0xFFFF) == q;
                }
            }
        }
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) s_wave[wid] = __popcll(bal);
        __syncthreads();
        int off = s_carry, tot = 0;
        for (int w = 0; w < kXNT / 64; ++w) {
            const int c = s_wave[w];
            off += w < wid ? c : 0;
            tot += c;
        }
        off += __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (keep) out[off] = dvo_dmatch{q, t, 0, (float)d};
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *m_out = s_carry;
}

}  // namespace

hipError_t launch_match(const StreamParams& P, int cross_check, hipStream_t s, hipEvent_t* ev, int tsplit) {
    const int pairs = stream_pairs(P);
    if (pairs < 1) return hipSuccess;
    mark(ev, 5, 0, s);
    const int cap = P.plan.kp_cap;
    // backward keys (and, split, the forward keys) start at 0x7F7F7F7F ("none") and are lowered by atomicMin
    hipError_t e = tsplit > 1
                       ? hipMemsetAsync(P.buf.nn, 0x7F, sizeof(int32_t) * 2 * (size_t)P.nframes * cap, s)
                       : hipMemsetAsync(P.buf.nn + (int64_t)P.nframes * cap, 0x7F,
                                        sizeof(int32_t) * (size_t)P.nframes * cap, s);
    if (e != hipSuccess) return e;
    const int nqb = (cap + kMQB - 1) / kMQB;
    const int nwg = ((pairs * nqb * tsplit + 7) / 8) * 8;  // XCD grouping needs a multiple of 8 blocks
    const NnOperands O{P.buf.desc, P.buf.desc + (int64_t)cap * 32, (int64_t)cap * 32, -1, -1};
    hipLaunchKernelGGL(nn_mfma_kernel, dim3(nwg), dim3(256), 0, s, P, O, pairs, nqb, tsplit);
    hipLaunchKernelGGL(crosscheck_stream_kernel, dim3(pairs), dim3(kXNT), 0, s, P, cross_check);
    mark(ev, 5, 1, s);
    return hipGetLastError();
}

namespace {
int pair_cap(int nq, int nt) { return ((nq > nt ? nq : nt) + kMQB - 1) / kMQB * kMQB; }
}  // namespace

size_t match_pair_work_size(int nq, int nt) { return 3 * (size_t)pair_cap(nq, nt) * sizeof(int32_t); }

// One pair through the stream's matcher: a StreamParams whose two "frames" are
// the query and train sets (counts passed as nq_fix / nt_fix, operands the
// caller's packed descriptors, nn = fwd | unused | bwd), so nn_mfma_kernel
// runs unchanged, with the train stages split over tsplit workgroups per query
// block to fill more than nq / 256 CUs.
hipError_t launch_match_pair(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int cross_check, void* d_work,
                             dvo_dmatch* d_out, int* d_m, hipStream_t s) {
    const int cap = pair_cap(nq, nt);
    StreamParams P{};
    P.plan.kp_cap = cap;
    P.nframes = 2;
    P.pair_step = 1;
    P.buf.nn = static_cast<int32_t*>(d_work);
    int32_t* fwd = P.buf.nn;
    int32_t* bwd = P.buf.nn + 2 * (size_t)cap;
    hipError_t e = hipMemsetAsync(P.buf.nn, 0x7F, sizeof(int32_t) * 3 * (size_t)cap, s);
    if (e != hipSuccess) return e;
    const int nqb = cap / kMQB;
    const int nst = (nt + kMStage - 1) / kMStage;
    int tsplit = 1;
    while (tsplit < 16 && nqb * tsplit * 2 <= 256 && nst >= tsplit * 4) tsplit *= 2;  // <= 256 workgroups, >= 2 stages each
    const int nwg = ((nqb * tsplit + 7) / 8) * 8;
    const NnOperands O{d_q, d_t, 0, nq, nt};
    hipLaunchKernelGGL(nn_mfma_kernel, dim3(nwg), dim3(256), 0, s, P, O, 1, nqb, tsplit);
    hipLaunchKernelGGL(crosscheck_pair_kernel, dim3(1), dim3(kXNT), 0, s, fwd, bwd, nq, nt, cross_check, d_out, d_m);
    return hipGetLastError();
}

// ---- float descriptors: BFMatcher(NORM_L1).knnMatch / FLANN stand-in ---------
// The SIFT/SURF branches (visual_odometry_v3.py:99-106, :200-215).  One thread
// per query holds its descriptor in registers; a workgroup scans a contiguous
// train range, staging kKnnTC rows at a time in LDS, which every wave reads
// as wave-uniform (broadcast) ds_read_b128 through a software pipeline
// (scalar loads of the rows serialised on their latency: 13x off).  Grid:
// x = query blocks, y = train ranges, sized so the grid is about one round of
// resident workgroups (3 per CU at <= 168 VGPRs): a fixed 64-row split left a
// third round nearly empty.  Each (query, range) keeps its K best in OpenCV's
// batchDistance order (enter iff d < dist[K-1], land after entries with
// dist <= d), i.e. the K smallest (distance, train index) pairs in
// lexicographic order; a merge kernel folds the ranges with a wave per query
// (that order is total, so any merge tree gives the sequential scan's result;
// oracle ora_bf_knn_float).
namespace {

struct KnnBytes {  // byte-packed rows, squared norms, rejection flag (knn_pack_u8_kernel)
    uint32_t *q, *t, *qn, *tn;
    int* rejected;
};

constexpr int kKnnQ = 256;  // queries per workgroup (one per thread)
constexpr int kKnnTC = 64;  // train rows per LDS stage
constexpr int kKnnWgPerCu = 3;
#ifndef DVO_KNN_G
#define DVO_KNN_G 2
#endif
constexpr int kKnnG = DVO_KNN_G;  // float4 train pieces in flight per wave (software pipeline depth)

// One group of 4 descriptor elements into the running distance: cv::normL1
// (base.hpp: s += |v0| + |v1| + |v2| + |v3|) or flann::L2 (squared, same
// grouping); no contraction under -ffp-contract=off.
template <int NORM>
__device__ __forceinline__ void dist_group(float& s, float a0, float a1, float a2, float a3, const float4 tv) {
    const float d0 = a0 - tv.x, d1 = a1 - tv.y, d2 = a2 - tv.z, d3 = a3 - tv.w;
    if constexpr (NORM == 0) {
        s += ((fabsf(d0) + fabsf(d1)) + fabsf(d2)) + fabsf(d3);
    } else {
        s += ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3;
    }
}

template <int K>
__device__ __forceinline__ void knn_insert(float (&bd)[K], int (&bi)[K], float d, int j) {
    if (!(d < bd[K - 1])) return;
#pragma unroll
    for (int s = K - 1; s >= 0; --s) {
        // sorted ascending: slot s keeps its entry if <= d, else takes d (when
        // slot s-1 is <= d) or the entry shifted down from s-1
        if (bd[s] > d) {
            if (s > 0 && bd[s - 1] > d) {
                bd[s] = bd[s - 1];
                bi[s] = bi[s - 1];
            } else {
                bd[s] = d;
                bi[s] = j;
            }
        }
    }
}

template <int D, int NORM, int K>
__global__ __launch_bounds__(kKnnQ) void knn_float_kernel(const float* __restrict__ q, int nq,
                                                          const float* __restrict__ t, int nt, int range,
                                                          const int* __restrict__ u8_rejected,
                                                          float* __restrict__ odist, int32_t* __restrict__ oidx) {
    if (*u8_rejected == 0) return;  // knn_u8_kernel served this call (uniform)
    constexpr int R = D / 4;
    static_assert(R % kKnnG == 0, "pipeline depth must divide the row");
    __shared__ float4 st[kKnnTC * R];
    const int qi = blockIdx.x * kKnnQ + threadIdx.x;
    const int qs = qi < nq ? qi : nq - 1;  // clamped: spare lanes compute, never store
    float qv[D];
    const float4* q4 = reinterpret_cast<const float4*>(q + (size_t)qs * D);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const float4 v = q4[i];
        qv[4 * i] = v.x;
        qv[4 * i + 1] = v.y;
        qv[4 * i + 2] = v.z;
        qv[4 * i + 3] = v.w;
    }
    float bd[K];
    int bi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        bd[s] = FLT_MAX;
        bi[s] = -1;
    }
    const int r0 = blockIdx.y * range, r1 = min(nt, r0 + range);
    for (int j0 = r0; j0 < r1; j0 += kKnnTC) {
        const int nj = min(r1 - j0, kKnnTC);
        const float4* src = reinterpret_cast<const float4*>(t + (size_t)j0 * D);
        if (j0 != r0) __syncthreads();  // previous stage fully read
        for (int i = threadIdx.x; i < nj * R; i += kKnnQ) st[i] = src[i];
        __syncthreads();
        // software pipeline over the stage's float4 stream: the next kKnnG
        // pieces (of this row or the next) are read while the current ones
        // are consumed
        float4 cur[kKnnG];
#pragma unroll
        for (int e = 0; e < kKnnG; ++e) cur[e] = st[e];
        for (int j = 0; j < nj; ++j) {
            const float4* row = st + j * R;
            const float4* nrow = st + min(j + 1, nj - 1) * R;
            float s = 0.f;
#pragma unroll
            for (int g = 0; g < R; g += kKnnG) {
                float4 nxt[kKnnG];
                const float4* pf = g + kKnnG < R ? row + g + kKnnG : nrow;
#pragma unroll
                for (int e = 0; e < kKnnG; ++e) nxt[e] = pf[e];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int e = 0; e < kKnnG; ++e) {
                    const int i = 4 * (g + e);
                    dist_group<NORM>(s, qv[i], qv[i + 1], qv[i + 2], qv[i + 3], cur[e]);
                }
#pragma unroll
                for (int e = 0; e < kKnnG; ++e) cur[e] = nxt[e];
            }
            knn_insert<K>(bd, bi, s, j0 + j);
        }
    }
    if (qi < nq) {
        const size_t o = ((size_t)blockIdx.y * nq + qi) * K;
#pragma unroll
        for (int s = 0; s < K; ++s) {
            odist[o + s] = bd[s];
            oidx[o + s] = bi[s];
        }
    }
}

// ---- byte-valued descriptors (SIFT: integers 0..255 stored as float) --------
// Every partial sum of such a distance is an integer below 2^24, so any
// summation order gives the float the restated order gives (oracle
// ora_bf_knn_float).  knn_pack_u8_kernel packs each row into bytes and its
// squared norm, and flags any value that is not an integer in [0, 255]; when
// nothing is flagged, knn_u8_kernel computes the distances in integer
// arithmetic — L1 with v_sad_u8 (4 elements per instruction), squared L2 as
// |q|^2 + |t|^2 - 2 q.t with v_dot4_u32_u8 — kKnnU8Q queries per thread so
// each broadcast train read feeds several rows; otherwise knn_float_kernel runs.  Both
// fill the same (range, query) partial slots.
// one thread per 4 values (coalesced float4 reads); a row's dim/4 threads are
// consecutive lanes, which reduce its squared norm with xor shuffles
// One launch packs both sides: blocks [0, qblocks) take the queries, the rest the trains.
__global__ __launch_bounds__(256) void knn_pack_u8_kernel(const float* __restrict__ xq, int nq,
                                                          const float* __restrict__ xt, int nt, int dim, int qblocks,
                                                          KnnBytes u8) {
    const bool side_q = (int)blockIdx.x < qblocks;
    const float* __restrict__ x = side_q ? xq : xt;
    const int n = side_q ? nq : nt;
    uint32_t* __restrict__ out = side_q ? u8.q : u8.t;
    uint32_t* __restrict__ norm = side_q ? u8.qn : u8.tn;
    int* __restrict__ rejected = u8.rejected;
    const int wpr = dim / 4;  // 16 or 32: divides 64
    const int64_t id = (int64_t)(side_q ? blockIdx.x : blockIdx.x - qblocks) * 256 + threadIdx.x;
    const bool in = id < (int64_t)n * wpr;
    const float4 v = in ? reinterpret_cast<const float4*>(x)[id] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float e[4] = {v.x, v.y, v.z, v.w};
    uint32_t word = 0, ss = 0;
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        ok &= e[c] >= 0.f && e[c] <= 255.f && e[c] == __builtin_rintf(e[c]);  // NaN fails
        const uint32_t b = e[c] >= 0.f && e[c] <= 255.f ? (uint32_t)e[c] : 0u;
        word |= b << (8 * c);
        ss += b * b;
    }
    for (int o = 1; o < wpr; o <<= 1) ss += __shfl_xor(ss, o);
    if (in) {
        out[id] = word;
        if ((id & (wpr - 1)) == 0) norm[id / wpr] = ss;
    }
    if (__ballot(!ok) != 0 && (threadIdx.x & 63) == 0) atomicOr(rejected, 1);
}

#ifndef DVO_KNN_U8Q
#define DVO_KNN_U8Q 2
#endif
constexpr int kKnnU8Q = DVO_KNN_U8Q;  // queries per thread in knn_u8_kernel
// Queries per workgroup the train split is sized for.  The byte kernel runs
// 256 * kKnnU8Q = 512 per workgroup, but sizing the split for 512 (twice the
// ranges) left its time unchanged (59 / 30 us at 5000^2 / 2000^2) and slowed
// the merge (7.3 -> 10.8 us): profiles/r02_qb{256,512}_knn_kernel_stats.csv.
#ifndef DVO_KNN_RANGE_QB
#define DVO_KNN_RANGE_QB 256
#endif
constexpr int kKnnRangeQB = DVO_KNN_RANGE_QB;

template <int D, int NORM, int K>
__global__ __launch_bounds__(256) void knn_u8_kernel(const uint32_t* __restrict__ q, const uint32_t* __restrict__ qn,
                                                     int nq, const uint32_t* __restrict__ t,
                                                     const uint32_t* __restrict__ tn, int nt, int range,
                                                     const int* __restrict__ rejected, float* __restrict__ odist,
                                                     int32_t* __restrict__ oidx) {
    if (*rejected != 0) return;  // some value is not a byte: knn_float_kernel serves the call (uniform)
    constexpr int W = D / 16;    // uint4 per row
    __shared__ uint4 st[kKnnTC * W];
    __shared__ uint32_t stn[kKnnTC];
    int qi[kKnnU8Q];
    uint4 qv[kKnnU8Q][W];
    uint32_t qnv[kKnnU8Q];
    float bd[kKnnU8Q][K];
    int bi[kKnnU8Q][K];
#pragma unroll
    for (int u = 0; u < kKnnU8Q; ++u) {
        qi[u] = blockIdx.x * (256 * kKnnU8Q) + 256 * u + threadIdx.x;
        const int qs = qi[u] < nq ? qi[u] : nq - 1;
        const uint4* q4 = reinterpret_cast<const uint4*>(q + (size_t)qs * (D / 4));
#pragma unroll
        for (int g = 0; g < W; ++g) qv[u][g] = q4[g];
        qnv[u] = qn[qs];
#pragma unroll
        for (int s2 = 0; s2 < K; ++s2) {
            bd[u][s2] = FLT_MAX;
            bi[u][s2] = -1;
        }
    }
    const int r0 = blockIdx.y * range, r1 = min(nt, r0 + range);
    for (int j0 = r0; j0 < r1; j0 += kKnnTC) {
        const int nj = min(r1 - j0, kKnnTC);
        const uint4* src = reinterpret_cast<const uint4*>(t + (size_t)j0 * (D / 4));
        if (j0 != r0) __syncthreads();
        for (int i = threadIdx.x; i < nj * W; i += 256) st[i] = src[i];
        if (threadIdx.x < nj) stn[threadIdx.x] = tn[j0 + threadIdx.x];
        __syncthreads();
        uint4 cur[W];
#pragma unroll
        for (int g = 0; g < W; ++g) cur[g] = st[g];
        for (int j = 0; j < nj; ++j) {
            uint4 nxt[W];
            const uint4* nrow = st + min(j + 1, nj - 1) * W;
#pragma unroll
            for (int g = 0; g < W; ++g) nxt[g] = nrow[g];
            const uint32_t tnj = stn[j];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < kKnnU8Q; ++u) {
                uint32_t acc = 0;
#pragma unroll
                for (int g = 0; g < W; ++g) {
                    if constexpr (NORM == 0) {
                        acc = __builtin_amdgcn_sad_u8(qv[u][g].x, cur[g].x, acc);
                        acc = __builtin_amdgcn_sad_u8(qv[u][g].y, cur[g].y, acc);
                        acc = __builtin_amdgcn_sad_u8(qv[u][g].z, cur[g].z, acc);
                        acc = __builtin_amdgcn_sad_u8(qv[u][g].w, cur[g].w, acc);
                    } else {
                        acc = __builtin_amdgcn_udot4(qv[u][g].x, cur[g].x, acc, false);
                        acc = __builtin_amdgcn_udot4(qv[u][g].y, cur[g].y, acc, false);
                        acc = __builtin_amdgcn_udot4(qv[u][g].z, cur[g].z, acc, false);
                        acc = __builtin_amdgcn_udot4(qv[u][g].w, cur[g].w, acc, false);
                    }
                }
                const uint32_t d = NORM == 0 ? acc : qnv[u] + tnj - 2u * acc;  // exact: < 2^24
                knn_insert<K>(bd[u], bi[u], (float)d, j0 + j);
            }
#pragma unroll
            for (int g = 0; g < W; ++g) cur[g] = nxt[g];
        }
    }
#pragma unroll
    for (int u = 0; u < kKnnU8Q; ++u)
        if (qi[u] < nq) {
            const size_t o = ((size_t)blockIdx.y * nq + qi[u]) * K;
#pragma unroll
            for (int s2 = 0; s2 < K; ++s2) {
                odist[o + s2] = bd[u][s2];
                oidx[o + s2] = bi[u][s2];
            }
        }
}

// (d, i) lexicographic; empty slots are (FLT_MAX, INT_MAX) and sort last
__device__ __forceinline__ bool knn_less(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}

// K smallest of two sorted K-lists, in place into (ad, ai)
template <int K>
__device__ __forceinline__ void knn_merge2(float (&ad)[K], int (&ai)[K], const float (&bd)[K], const int (&bi)[K]) {
    float md[K];
    int mi[K];
    int pa = 0, pb = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) {
        float da = FLT_MAX, db = FLT_MAX;
        int ia = INT_MAX, ib = INT_MAX;
#pragma unroll
        for (int u = 0; u < K; ++u) {
            if (u == pa) { da = ad[u]; ia = ai[u]; }
            if (u == pb) { db = bd[u]; ib = bi[u]; }
        }
        const bool ta = knn_less(da, ia, db, ib);
        md[s] = ta ? da : db;
        mi[s] = ta ? ia : ib;
        pa += ta;
        pb += !ta;
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
        ad[s] = md[s];
        ai[s] = mi[s];
    }
}

// one wave per query: lane l folds ranges l, l+64, ... by sequential
// insertion, then a butterfly of sorted-list merges
template <int K>
__global__ __launch_bounds__(256) void knn_merge_kernel(const float* __restrict__ pdist, const int32_t* __restrict__ pidx,
                                                        int nq, int ranges, float* __restrict__ odist,
                                                        int32_t* __restrict__ oidx) {
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (qi >= nq) return;  // wave-uniform
    float bd[K];
    int bi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        bd[s] = FLT_MAX;
        bi[s] = INT_MAX;
    }
    for (int c = lane; c < ranges; c += 64) {
        const size_t o = ((size_t)c * nq + qi) * K;
        float cd[K];
        int ci[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const int i = pidx[o + s];
            cd[s] = i >= 0 ? pdist[o + s] : FLT_MAX;
            ci[s] = i >= 0 ? i : INT_MAX;
        }
        knn_merge2<K>(bd, bi, cd, ci);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        float od[K];
        int oi[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            od[s] = __shfl_xor(bd[s], m, 64);
            oi[s] = __shfl_xor(bi[s], m, 64);
        }
        knn_merge2<K>(bd, bi, od, oi);
    }
    if (lane < K) {
        float d = bd[0];
        int i = bi[0];
#pragma unroll
        for (int s = 1; s < K; ++s)
            if (lane == s) {
                d = bd[s];
                i = bi[s];
            }
        odist[(size_t)qi * K + lane] = i == INT_MAX ? FLT_MAX : d;
        oidx[(size_t)qi * K + lane] = i == INT_MAX ? -1 : i;
    }
}

template <int D, int NORM, int K>
hipError_t launch_knn_t(const float* d_q, int nq, const float* d_t, int nt, int ranges, const KnnBytes& u8,
                        float* d_part, int32_t* d_pidx, float* d_dist, int32_t* d_idx, hipStream_t s) {
    const int range = (nt + ranges - 1) / ranges;
    float* od = ranges == 1 ? d_dist : d_part;
    int32_t* oi = ranges == 1 ? d_idx : d_pidx;
    hipError_t e = hipMemsetAsync(u8.rejected, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    const int qblocks = (int)(((int64_t)nq * (D / 4) + 255) / 256), tblocks = (int)(((int64_t)nt * (D / 4) + 255) / 256);
    hipLaunchKernelGGL(knn_pack_u8_kernel, dim3(qblocks + tblocks), dim3(256), 0, s, d_q, nq, d_t, nt, D, qblocks, u8);
    hipLaunchKernelGGL((knn_u8_kernel<D, NORM, K>), dim3((nq + 256 * kKnnU8Q - 1) / (256 * kKnnU8Q), ranges), dim3(256), 0, s, u8.q, u8.qn, nq,
                       u8.t, u8.tn, nt, range, u8.rejected, od, oi);
    hipLaunchKernelGGL((knn_float_kernel<D, NORM, K>), dim3((nq + kKnnQ - 1) / kKnnQ, ranges), dim3(kKnnQ), 0, s, d_q,
                       nq, d_t, nt, range, u8.rejected, od, oi);
    if (ranges > 1)
        hipLaunchKernelGGL((knn_merge_kernel<K>), dim3((nq + 3) / 4), dim3(256), 0, s, d_part, d_pidx, nq, ranges,
                           d_dist, d_idx);
    return hipGetLastError();
}

template <int D, int NORM>
hipError_t launch_knn_k(int k, const float* d_q, int nq, const float* d_t, int nt, int ranges, const KnnBytes& u8,
                        float* d_part, int32_t* d_pidx, float* d_dist, int32_t* d_idx, hipStream_t s) {
    switch (k) {
        case 1: return launch_knn_t<D, NORM, 1>(d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
        case 2: return launch_knn_t<D, NORM, 2>(d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
        case 3: return launch_knn_t<D, NORM, 3>(d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
        case 4: return launch_knn_t<D, NORM, 4>(d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

int knn_ranges(int nq, int nt, int cus) {
    // about two rounds of resident workgroups of kKnnRangeQB queries, at least
    // 16 trains per range; the float and byte kernels share the split
    const int qblocks = (nq + kKnnRangeQB - 1) / kKnnRangeQB;
    int ranges = (cus * kKnnWgPerCu * 2) / qblocks;
    ranges = std::min(ranges, (nt + 15) / 16);
    ranges = std::max(ranges, 1);
    const int range = (nt + ranges - 1) / ranges;
    return (nt + range - 1) / range;  // no empty trailing range
}

size_t knn_bytes_size(int nq, int nt, int dim) { return (size_t)(nq + nt) * dim + 4 * (size_t)(nq + nt) + 16; }

hipError_t launch_knn_float(const float* d_q, int nq, const float* d_t, int nt, int dim, int k, int norm, int ranges,
                            void* d_bytes, float* d_part, int32_t* d_pidx, float* d_dist, int32_t* d_idx,
                            hipStream_t s) {
    if (nq <= 0 || nt <= 0) return hipSuccess;
    uint8_t* b = static_cast<uint8_t*>(d_bytes);  // packed rows (dim bytes each; dim % 64 == 0), norms, flag
    KnnBytes u8;
    u8.q = reinterpret_cast<uint32_t*>(b);
    u8.t = reinterpret_cast<uint32_t*>(b + (size_t)nq * dim);
    u8.qn = reinterpret_cast<uint32_t*>(b + (size_t)(nq + nt) * dim);
    u8.tn = u8.qn + nq;
    u8.rejected = reinterpret_cast<int*>(u8.tn + nt);
    if (dim == 128)
        return norm == 0 ? launch_knn_k<128, 0>(k, d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s)
                         : launch_knn_k<128, 1>(k, d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
    if (dim == 64)
        return norm == 0 ? launch_knn_k<64, 0>(k, d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s)
                         : launch_knn_k<64, 1>(k, d_q, nq, d_t, nt, ranges, u8, d_part, d_pidx, d_dist, d_idx, s);
    return hipErrorInvalidValue;
}

}  // namespace dvo
