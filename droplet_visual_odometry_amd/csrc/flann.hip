// FLANN randomized kd-tree k-NN for gfx950: the MI355X replacement of
// cv::FlannBasedMatcher(dict(algorithm=FLANN_INDEX_KDTREE, trees=5),
// dict(checks=50)).knnMatch(previous, current, k=2), the matcher of the
// reference's 'flann' mode (scripts/visual_odometry_v3.py:206-212).  The
// algorithm is OpenCV 4.x's bundled FLANN, restated in oracle/flann.cpp (see
// its header for the call chain); every step below reproduces it exactly:
//
//   draws      cv::theRNG() outputs of one tree: n shuffle draws, then one per
//              internal node in preorder (the host jumps the multiply-with-
//              carry state to each chunk's start: s_k = s_0 A^k mod m);
//   shuffle    cv::randShuffle(ind): for i = 0..n-1 swap(ind[r_i % n], ind[i]).
//              Sequential as written; here every output position is traced
//              backwards through the transpositions that touch it (step i
//              touches positions i and r_i % n; the steps with r_i % n = v
//              are bucketed by v), O(n log n) work in parallel;
//   divideTree level by level, one workgroup per open node: mean / variance
//              per dimension in float over the node's first min(101, count)
//              points in ind order (one thread per dimension, the sum in point
//              order), selectDivision's top-5 by (variance desc, index asc)
//              and rand_int(num) from the node's preorder draw, then
//              planeSplit's two Hoare passes as parallel pairings (the k-th
//              misplaced point from the left swaps with the k-th from the
//              right), and the split-point rule; node ids are preorder ids, so
//              the child ids follow from the left child's count;
//   search     one wave per query (getNeighbors with eps 0): descend every
//              tree, then pop branches from a binary heap in LDS (libstdc++'s
//              push_heap / pop_heap sift order, so ties pop as in OpenCV)
//              while fewer than `checks` leaves were checked or the result is
//              not full; the checked set is a bitset in LDS; flann::L2's
//              grouped sum ((d0^2 + d1^2) + d2^2) + d3^2 per lane, the groups
//              added in order; a KNNUniqueResultSet of (distance, index).
//              A query whose heap outgrows LDS is flagged and redone with its
//              heap in global memory (the heap holds up to n entries).
#include <cfloat>
#include <climits>

#include "dvo_internal.h"

namespace dvo {
namespace {

constexpr uint64_t kTheRngA = 4164903690ull;
constexpr int kFlNT = 256;         // build kernels
constexpr int kFlSample = 101;     // SAMPLE_MEAN + 1
constexpr int kFlHeapLds = 1024;   // heap entries per query wave in LDS

__global__ void flann_draws_kernel(const uint64_t* chunk_state, int nchunk, int total, uint32_t* R) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunk) return;
    const int b = (int)((int64_t)total * c / nchunk), e = (int)((int64_t)total * (c + 1) / nchunk);
    uint64_t st = chunk_state[c];
    for (int i = b; i < e; ++i) {
        st = (uint64_t)(uint32_t)st * kTheRngA + (st >> 32);
        R[i] = (uint32_t)st;
    }
}

__global__ void flann_bucket_count_kernel(const uint32_t* R, int n, int* cnt) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) atomicAdd(&cnt[R[s] % (uint32_t)n], 1);
}

// exclusive scan of cnt[0..n) into off[0..n], one workgroup (n <= 2^16)
__global__ __launch_bounds__(1024) void flann_bucket_scan_kernel(const int* cnt, int n, int* off, int* fill) {
    __shared__ int part[1024];
    const int per = (n + 1023) / 1024, b = threadIdx.x * per, e = min(n, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the per-thread sums
        const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = part[threadIdx.x] - s;
    for (int i = b; i < e; ++i) {
        off[i] = run;
        fill[i] = 0;
        run += cnt[i];
    }
    if (threadIdx.x == 1023) off[n] = part[1023];
}

__global__ void flann_bucket_fill_kernel(const uint32_t* R, int n, const int* off, int* fill, int* list) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int v = (int)(R[s] % (uint32_t)n);
    list[off[v] + atomicAdd(&fill[v], 1)] = s;  // bucket order is irrelevant: the trace takes a maximum
}

// new_ind[p] = ind[pos], pos = the position whose value the n transpositions move into p
__global__ void flann_shuffle_trace_kernel(const uint32_t* R, int n, const int* off, const int* list,
                                           const int* ind, int* new_ind) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    int pos = p, s = n - 1;
    while (s >= 0) {
        const int s1 = pos <= s ? pos : -1;
        int s2 = -1;
        for (int q = off[pos]; q < off[pos + 1]; ++q) {
            const int t = list[q];
            if (t <= s && t > s2) s2 = t;
        }
        const int st = max(s1, s2);
        if (st < 0) break;
        if (st == s1 && st == s2) {
        } else if (st == s1) {  // step st = pos: swap(ind[r % n], ind[pos]) brought ind[r % n] here
            pos = (int)(R[st] % (uint32_t)n);
        } else {  // step st put ind[st] at position r_st % n == pos
            pos = st;
        }
        s = st - 1;
    }
    new_ind[p] = ind[pos];
}

struct FlannBuild {
    const float* data;
    int n, dim;
    int* ind;            // [n], permuted in place by the splits
    float* xv;           // [n] split values along ind (per-node segment scratch)
    int* sl;             // [n] left stops
    int* sr;             // [n] right stops
    const uint32_t* R;   // the tree's draws: [0, n) shuffle, [n, 2n - 1) internal nodes in preorder
    int4* nodes;         // the tree's 2n - 1 nodes {divfeat, divval bits, child1, child2} (ids tree-local)
    int4* open[2];       // open nodes {segment start, count, node id, preorder internal index}
    int* cnt;            // [levels] open nodes per level
};

__device__ __forceinline__ int block_scan_excl(int v, int& total, int* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kFlNT / 64; ++w) {
        const int c = sh[w];
        off += w < wid ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

// One Hoare pass of planeSplit over [lo, hi) of the node segment: the points with !keep in
// [lo, mid) pair with the points with keep in [mid, hi), the k-th from the left with the k-th
// from the right (mid = lo + #keep in [lo, hi)).
template <class Keep>
__device__ void hoare_pass(const FlannBuild& B, int a, int lo, int mid, int hi, Keep keep, int* sh) {
    int nl = 0, nr = 0;
    for (int b0 = lo; b0 < hi; b0 += kFlNT) {
        const int i = b0 + threadIdx.x;
        const bool in = i < hi;
        const bool k = in && keep(B.xv[a + i]);
        const int fl = in && i < mid && !k, fr = in && i >= mid && k;
        int tl, tr;
        const int pl = block_scan_excl(fl, tl, sh);
        const int pr = block_scan_excl(fr, tr, sh + 8);
        if (fl) B.sl[a + lo + nl + pl] = i;
        if (fr) B.sr[a + lo + nr + pr] = i;
        nl += tl;
        nr += tr;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nl; q += kFlNT) {  // nl == nr
        const int i = B.sl[a + lo + q], j = B.sr[a + lo + nr - 1 - q];
        const int ti = B.ind[a + i];
        B.ind[a + i] = B.ind[a + j];
        B.ind[a + j] = ti;
        const float tx = B.xv[a + i];
        B.xv[a + i] = B.xv[a + j];
        B.xv[a + j] = tx;
    }
    __syncthreads();
}

__device__ __forceinline__ bool var_better(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia < ib);
}

__global__ __launch_bounds__(kFlNT) void flann_level_kernel(FlannBuild B, int level) {
    if ((int)blockIdx.x >= B.cnt[level]) return;
    const int4 e = B.open[level & 1][blockIdx.x];
    const int a = e.x, c = e.y, id = e.z, pre = e.w;
    __shared__ int s_ind[kFlSample];
    __shared__ float s_mean[256], s_var[256];
    __shared__ int sh[16];
    __shared__ int s_top[5], s_cnt[2];
    const int cnt = min(kFlSample, c);
    for (int j = threadIdx.x; j < cnt; j += kFlNT) s_ind[j] = B.ind[a + j];
    __syncthreads();
    const int k = threadIdx.x;
    if (k < B.dim) {  // meanSplit: float sums in point order, one thread per dimension
        float m = 0.f;
        for (int j = 0; j < cnt; ++j) m += B.data[(int64_t)s_ind[j] * B.dim + k];
        m /= (float)cnt;
        float v = 0.f;
        for (int j = 0; j < cnt; ++j) {
            const float d = B.data[(int64_t)s_ind[j] * B.dim + k] - m;
            v += d * d;
        }
        s_mean[k] = m;
        s_var[k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // selectDivision: the RAND_DIM = 5 largest variances, (var desc, index asc)
        const int lane = threadIdx.x;
        float v[4];
        int ix[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ix[q] = lane + 64 * q;
            v[q] = ix[q] < B.dim ? s_var[ix[q]] : -FLT_MAX;
            if (ix[q] >= B.dim) ix[q] = INT_MAX;
        }
        const int num = min(5, B.dim);
        for (int r = 0; r < num; ++r) {
            float bv = -FLT_MAX;
            int bi = INT_MAX;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (ix[q] != INT_MAX && (bi == INT_MAX || var_better(v[q], ix[q], bv, bi))) {
                    bv = v[q];
                    bi = ix[q];
                }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const float ov = __shfl_xor(bv, o);
                const int oi = __shfl_xor(bi, o);
                if (oi != INT_MAX && (bi == INT_MAX || var_better(ov, oi, bv, bi))) {
                    bv = ov;
                    bi = oi;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (ix[q] == bi) ix[q] = INT_MAX;  // taken
            if (lane == 0) s_top[r] = bi;
        }
        if (lane == 0) {
            const int rv = (int)(B.R[B.n + pre] & 0x7FFFFFFFu);
            const int rnd = (int)((double)num * (rv / (2147483647.0 + 1.0)));
            s_cnt[0] = s_top[rnd];
        }
    }
    __syncthreads();
    const int cutfeat = s_cnt[0];
    const float cutval = s_mean[cutfeat];
    // planeSplit: split values along the segment, then the two passes (< cutval, then <= cutval)
    int lim1 = 0, lim2 = 0;
    for (int b0 = 0; b0 < c; b0 += kFlNT) {
        const int i = b0 + threadIdx.x;
        int l1 = 0, l2 = 0;
        if (i < c) {
            const float x = B.data[(int64_t)B.ind[a + i] * B.dim + cutfeat];
            B.xv[a + i] = x;
            l1 = x < cutval;
            l2 = x <= cutval;
        }
        int t1, t2;
        block_scan_excl(l1, t1, sh);
        block_scan_excl(l2, t2, sh + 8);
        lim1 += t1;
        lim2 += t2;
    }
    __syncthreads();
    hoare_pass(B, a, 0, lim1, c, [&](float x) { return x < cutval; }, sh);
    hoare_pass(B, a, lim1, lim2, c, [&](float x) { return x <= cutval; }, sh);
    int index;
    if (lim1 > c / 2) index = lim1;
    else if (lim2 < c / 2) index = lim2;
    else index = c / 2;
    if (lim1 == c || lim2 == 0) index = c / 2;
    if (threadIdx.x == 0) {
        const int l_id = id + 1, r_id = id + 2 * index;
        B.nodes[id] = make_int4(cutfeat, __float_as_int(cutval), l_id, r_id);
        const int ca[2] = {a, a + index}, cc[2] = {index, c - index}, ci[2] = {l_id, r_id}, cp[2] = {pre + 1, pre + index};
        for (int h = 0; h < 2; ++h) {
            if (cc[h] == 1) {
                B.nodes[ci[h]] = make_int4(B.ind[ca[h]], 0, -1, -1);
            } else {
                const int slot = atomicAdd(&B.cnt[level + 1], 1);
                B.open[(level + 1) & 1][slot] = make_int4(ca[h], cc[h], ci[h], cp[h]);
            }
        }
    }
}

__global__ void flann_root_kernel(FlannBuild B) {
    if (threadIdx.x != 0) return;
    if (B.n == 1) {
        B.nodes[0] = make_int4(B.ind[0], 0, -1, -1);
        B.cnt[0] = 0;
    } else {
        B.open[0][0] = make_int4(0, B.n, 0, 0);
        B.cnt[0] = 1;
    }
}

// ---- search ------------------------------------------------------------------
struct FlannSearch {
    const float* q;        // [nq][dim]
    const float* t;        // [n][dim]
    const int4* nodes;     // [trees][2n - 1]
    int nq, n, dim, k, trees, checks, nodes_per_tree;
    int32_t* idx;          // [nq][k]
    float* dist;           // [nq][k]
    int32_t* flag;         // [nq]: heap outgrew LDS (redo with the global heap)
    const int32_t* redo;   // global-heap pass: the query of each workgroup
    float* gheap_d;        // global-heap pass: [workgroups][n]
    int32_t* gheap_n;
};

template <bool kGlobalHeap>
__global__ __launch_bounds__(64) void flann_search_kernel(FlannSearch S) {
    extern __shared__ uint32_t smem[];
    const int qi = kGlobalHeap ? S.redo[blockIdx.x] : (int)blockIdx.x;
    if (qi >= S.nq) return;
    const int lane = threadIdx.x;
    const int nwords = (S.n + 31) >> 5;
    uint32_t* checked = smem;
    float* hd = kGlobalHeap ? S.gheap_d + (int64_t)blockIdx.x * S.n : reinterpret_cast<float*>(smem + nwords);
    int* hn = kGlobalHeap ? S.gheap_n + (int64_t)blockIdx.x * S.n : reinterpret_cast<int*>(smem + nwords + kFlHeapLds);
    const int hcap = kGlobalHeap ? S.n : min(S.n, kFlHeapLds);
    for (int w = lane; w < nwords; w += 64) checked[w] = 0;
    const int ng = S.dim >> 2;  // groups of 4 (dim % 4 == 0)
    const float4 qv = lane < ng ? *reinterpret_cast<const float4*>(S.q + (int64_t)qi * S.dim + 4 * lane)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // result set (KNNUniqueResultSet), wave-uniform
    float rd[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    int ri[4] = {-1, -1, -1, -1};
    int rsize = 0;
    bool full = false;
    float worst = FLT_MAX;
    int check_count = 0, hs = 0;
    bool overflow = false;
    auto qval = [&](int f) {  // q[f], f wave-uniform
        const int src = f >> 2, comp = f & 3;
        const float x = comp == 0 ? qv.x : comp == 1 ? qv.y : comp == 2 ? qv.z : qv.w;
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src));
    };
    auto add_point = [&](float d, int index) {
        if (d >= worst) return;
        int pos = rsize;  // (distance, index) order; an index is checked once, so no duplicates
        while (pos > 0 && (rd[pos - 1] > d || (rd[pos - 1] == d && ri[pos - 1] > index))) --pos;
        for (int j = 3; j > 0; --j)
            if (j > pos) {
                rd[j] = rd[j - 1];
                ri[j] = ri[j - 1];
            }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j == pos) {
                rd[j] = d;
                ri[j] = index;
            }
        if (rsize < S.k) ++rsize;
        if (rsize == S.k) {
            full = true;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j == S.k - 1) worst = rd[j];
        }
    };
    // std::push_heap / __adjust_heap with CompareT(a, b) = b.mindist < a.mindist (a min-heap)
    auto heap_push = [&](int node, float md) {
        if (hs == S.n) return;  // Heap::insert drops when full (count == length)
        if (hs == hcap) {
            overflow = true;
            return;
        }
        int hole = hs, parent = (hole - 1) / 2;
        while (hole > 0 && md < hd[parent]) {
            if (lane == 0) {
                hd[hole] = hd[parent];
                hn[hole] = hn[parent];
            }
            hole = parent;
            parent = (hole - 1) / 2;
        }
        if (lane == 0) {
            hd[hole] = md;
            hn[hole] = node;
        }
        ++hs;
    };
    auto heap_pop = [&](int& node, float& md) {
        node = hn[0];
        md = hd[0];
        const int len = hs - 1;
        if (len > 0) {
            const float vd = hd[len];
            const int vn = hn[len];
            int hole = 0, second = 0;
            while (second < (len - 1) / 2) {
                second = 2 * (second + 1);
                if (hd[second - 1] < hd[second]) second--;
                if (lane == 0) {
                    hd[hole] = hd[second];
                    hn[hole] = hn[second];
                }
                hole = second;
            }
            if ((len & 1) == 0 && second == (len - 2) / 2) {
                second = 2 * (second + 1);
                if (lane == 0) {
                    hd[hole] = hd[second - 1];
                    hn[hole] = hn[second - 1];
                }
                hole = second - 1;
            }
            int parent = (hole - 1) / 2;
            while (hole > 0 && vd < hd[parent]) {
                if (lane == 0) {
                    hd[hole] = hd[parent];
                    hn[hole] = hn[parent];
                }
                hole = parent;
                parent = (hole - 1) / 2;
            }
            if (lane == 0) {
                hd[hole] = vd;
                hn[hole] = vn;
            }
        }
        hs = len;
    };
    auto descend = [&](int tree, int node, float mindist) {
        const int4* nodes = S.nodes + (int64_t)tree * S.nodes_per_tree;
        while (!overflow) {
            if (worst < mindist) return;
            const int4 nd = nodes[__builtin_amdgcn_readfirstlane(node)];
            if (nd.z < 0 && nd.w < 0) {  // leaf: check it once
                const int index = nd.x;
                const uint32_t bit = 1u << (index & 31);
                if ((checked[index >> 5] & bit) || (check_count >= S.checks && full)) return;
                if (lane == 0) checked[index >> 5] |= bit;
                ++check_count;
                float g = 0.f;
                if (lane < ng) {
                    const float4 tv = *reinterpret_cast<const float4*>(S.t + (int64_t)index * S.dim + 4 * lane);
                    const float d0 = tv.x - qv.x, d1 = tv.y - qv.y, d2 = tv.z - qv.z, d3 = tv.w - qv.w;
                    g = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
                }
                float d = 0.f;
                for (int j = 0; j < ng; ++j) d += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), j));
                add_point(d, index);
                return;
            }
            const float val = qval(nd.x);
            const float divval = __int_as_float(nd.y);
            const float diff = val - divval;
            const int best = diff < 0 ? nd.z : nd.w, other = diff < 0 ? nd.w : nd.z;
            const float new_distsq = mindist + (val - divval) * (val - divval);
            if (new_distsq * 1.0f < worst || !full) heap_push(tree * S.nodes_per_tree + other, new_distsq);
            node = best;
        }
    };
    for (int tr = 0; tr < S.trees && !overflow; ++tr) {
        descend(tr, 0, 0.f);
        if (check_count >= S.checks && full) break;
    }
    while (hs > 0 && !overflow) {
        int gnode;
        float md;
        heap_pop(gnode, md);
        if (!(check_count < S.checks || !full)) break;
        const int tr = gnode / S.nodes_per_tree;
        descend(tr, gnode - tr * S.nodes_per_tree, md);
    }
    if (lane == 0) {
        if (!kGlobalHeap) S.flag[qi] = overflow ? 1 : 0;
        if (!overflow)
            for (int j = 0; j < S.k; ++j) {
                S.idx[(int64_t)qi * S.k + j] = j < rsize ? ri[j] : -1;
                S.dist[(int64_t)qi * S.k + j] = j < rsize ? rd[j] : FLT_MAX;
            }
    }
}

__global__ void flann_redo_list_kernel(const int32_t* flag, int nq, int32_t* list, int32_t* count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq && flag[i]) list[atomicAdd(count, 1)] = i;
}

}  // namespace

size_t flann_search_lds(int n) { return ((size_t)(n + 31) / 32 + 2 * kFlHeapLds) * 4; }

hipError_t launch_flann_draws(const uint64_t* d_chunk_state, int nchunk, int total, uint32_t* d_R, hipStream_t s) {
    hipLaunchKernelGGL(flann_draws_kernel, dim3((nchunk + 63) / 64), dim3(64), 0, s, d_chunk_state, nchunk, total, d_R);
    return hipGetLastError();
}

hipError_t launch_flann_shuffle(const uint32_t* d_R, int n, int* d_cnt, int* d_off, int* d_fill, int* d_list,
                                const int* d_ind, int* d_new_ind, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_cnt, 0, sizeof(int) * n, s);
    if (e != hipSuccess) return e;
    const int g = (n + 255) / 256;
    hipLaunchKernelGGL(flann_bucket_count_kernel, dim3(g), dim3(256), 0, s, d_R, n, d_cnt);
    hipLaunchKernelGGL(flann_bucket_scan_kernel, dim3(1), dim3(1024), 0, s, d_cnt, n, d_off, d_fill);
    hipLaunchKernelGGL(flann_bucket_fill_kernel, dim3(g), dim3(256), 0, s, d_R, n, d_off, d_fill, d_list);
    hipLaunchKernelGGL(flann_shuffle_trace_kernel, dim3(g), dim3(256), 0, s, d_R, n, d_off, d_list, d_ind, d_new_ind);
    return hipGetLastError();
}

hipError_t launch_flann_root(const FlannBuildArgs& a, hipStream_t s) {
    FlannBuild B{a.data, a.n, a.dim, a.ind, a.xv, a.sl, a.sr, a.R, a.nodes, {a.open0, a.open1}, a.cnt};
    hipLaunchKernelGGL(flann_root_kernel, dim3(1), dim3(64), 0, s, B);
    return hipGetLastError();
}

hipError_t launch_flann_level(const FlannBuildArgs& a, int level, int max_open, hipStream_t s) {
    FlannBuild B{a.data, a.n, a.dim, a.ind, a.xv, a.sl, a.sr, a.R, a.nodes, {a.open0, a.open1}, a.cnt};
    hipLaunchKernelGGL(flann_level_kernel, dim3(max_open), dim3(kFlNT), 0, s, B, level);
    return hipGetLastError();
}

hipError_t launch_flann_search(const FlannSearchArgs& a, hipStream_t s) {
    FlannSearch S{a.q, a.t, a.nodes, a.nq, a.n, a.dim, a.k, a.trees, a.checks, 2 * a.n - 1,
                  a.idx, a.dist, a.flag, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL(flann_search_kernel<false>, dim3(a.nq), dim3(64), flann_search_lds(a.n), s, S);
    return hipGetLastError();
}

hipError_t launch_flann_redo_list(const int32_t* d_flag, int nq, int32_t* d_list, int32_t* d_count, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_count, 0, sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flann_redo_list_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, d_flag, nq, d_list, d_count);
    return hipGetLastError();
}

hipError_t launch_flann_search_global(const FlannSearchArgs& a, const int32_t* d_list, int count, float* d_heap_d,
                                      int32_t* d_heap_n, hipStream_t s) {
    FlannSearch S{a.q, a.t, a.nodes, a.nq, a.n, a.dim, a.k, a.trees, a.checks, 2 * a.n - 1,
                  a.idx, a.dist, a.flag, d_list, d_heap_d, d_heap_n};
    hipLaunchKernelGGL(flann_search_kernel<true>, dim3(count), dim3(64), ((size_t)(a.n + 31) / 32) * 4, s, S);
    return hipGetLastError();
}

}  // namespace dvo
