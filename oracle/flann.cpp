// TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of
// cv::FlannBasedMatcher(dict(algorithm=FLANN_INDEX_KDTREE, trees=5),
// dict(checks=50)).knnMatch(previous, current, k=2) as the reference's 'flann'
// mode builds and calls it (scripts/visual_odometry_v3.py:206-212; the 0.75
// ratio test follows at :223-228).  Follows OpenCV 4.x's bundled FLANN 1.6:
//   FlannBasedMatcher::knnMatch -> DescriptorMatcher::knnMatch clones the
//     matcher, adds the train set and trains: a new cv::flann::Index over the
//     train descriptors (cvflann::L2<float>, squared distances) every call;
//   KDTreeIndex::buildIndex: one index permutation ind = 0..n-1, and for each
//     of the `trees` trees cv::randShuffle(ind) (theRNG: j = rng.next() % n,
//     swap(ind[j], ind[i]) for i = 0..n-1) then divideTree(ind) -- which
//     permutes ind in place, so each tree's shuffle starts from the previous
//     tree's order;
//   divideTree / meanSplit: mean and (unnormalised) variance per dimension in
//     float over the first min(101, count) vectors of the node in ind order,
//     selectDivision = one of the RAND_DIM = 5 largest variances picked by
//     rand_int(num) = (int)(num * (rand() / (RAND_MAX + 1.0))) with
//     cvflann::rand() = theRNG().next() & INT_MAX (RAND_MAX == INT_MAX on
//     glibc), cutval = the mean there, planeSplit's two Hoare passes (< cutval,
//     then <= cutval), and the split point rule lim1 / lim2 / count / 2;
//   getNeighbors (eps 0, explore_all_trees false): descend every tree once
//     (searchLevel), then pop branches from a binary heap (std::push_heap /
//     pop_heap on mindist) while fewer than `checks` leaves were checked or the
//     result is not full; a leaf is checked once (DynamicBitset); the
//     unexplored child is pushed iff new_distsq < worstDist or the result is
//     not full, with new_distsq = mindist + (val - divval)^2 in float;
//   NNIndex::knnSearch keeps a KNNUniqueResultSet: the k smallest
//     (distance, index) pairs among the checked points, ascending.
// cv::theRNG() is process state in the reference: every call consumes
// trees * (n + (n - 1)) draws (n shuffle draws and one per internal node),
// so it is passed in and returned (rng_state) and the drop-in carries it.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <iterator>
#include <limits>
#include <set>
#include <vector>

#include "oracle.h"

namespace {

struct TheRng {  // cv::RNG (multiply-with-carry)
    uint64_t state;
    unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

inline int flann_rand(TheRng& r) { return (int)(r.next() & INT_MAX); }
inline int rand_int(TheRng& r, int high) { return (int)((double)high * (flann_rand(r) / (INT_MAX + 1.0))); }

struct Node {
    int divfeat;       // split dimension, or the point index of a leaf
    float divval;
    int child1, child2;  // -1 for a leaf
};

struct KDForest {
    const float* data;
    int n, dim;
    std::vector<Node> nodes;
    std::vector<int> roots;
    std::vector<float> mean, var;

    const float* vec(int i) const { return data + (size_t)i * dim; }

    int select_division(TheRng& rng) {
        const int kRandDim = 5;
        int num = 0;
        size_t topind[kRandDim];
        for (int i = 0; i < dim; ++i) {
            if (num < kRandDim || var[i] > var[topind[num - 1]]) {
                if (num < kRandDim) topind[num++] = i;
                else topind[num - 1] = i;
                int j = num - 1;
                while (j > 0 && var[topind[j]] > var[topind[j - 1]]) {
                    std::swap(topind[j], topind[j - 1]);
                    --j;
                }
            }
        }
        return (int)topind[rand_int(rng, num)];
    }

    void plane_split(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2) {
        int left = 0, right = count - 1;
        for (;;) {
            while (left <= right && vec(ind[left])[cutfeat] < cutval) ++left;
            while (left <= right && vec(ind[right])[cutfeat] >= cutval) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]);
            ++left;
            --right;
        }
        lim1 = left;
        right = count - 1;
        for (;;) {
            while (left <= right && vec(ind[left])[cutfeat] <= cutval) ++left;
            while (left <= right && vec(ind[right])[cutfeat] > cutval) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]);
            ++left;
            --right;
        }
        lim2 = left;
    }

    void mean_split(int* ind, int count, int& index, int& cutfeat, float& cutval, TheRng& rng) {
        std::fill(mean.begin(), mean.end(), 0.f);
        std::fill(var.begin(), var.end(), 0.f);
        const int cnt = std::min(100 + 1, count);  // SAMPLE_MEAN + 1
        for (int j = 0; j < cnt; ++j) {
            const float* v = vec(ind[j]);
            for (int k = 0; k < dim; ++k) mean[k] += v[k];
        }
        for (int k = 0; k < dim; ++k) mean[k] /= cnt;
        for (int j = 0; j < cnt; ++j) {
            const float* v = vec(ind[j]);
            for (int k = 0; k < dim; ++k) {
                const float d = v[k] - mean[k];
                var[k] += d * d;
            }
        }
        cutfeat = select_division(rng);
        cutval = mean[cutfeat];
        int lim1, lim2;
        plane_split(ind, count, cutfeat, cutval, lim1, lim2);
        if (lim1 > count / 2) index = lim1;
        else if (lim2 < count / 2) index = lim2;
        else index = count / 2;
        if (lim1 == count || lim2 == 0) index = count / 2;
    }

    int divide_tree(int* ind, int count, TheRng& rng) {
        const int id = (int)nodes.size();
        nodes.push_back(Node{0, 0.f, -1, -1});
        if (count == 1) {
            nodes[id].divfeat = *ind;
            return id;
        }
        int idx, cutfeat;
        float cutval;
        mean_split(ind, count, idx, cutfeat, cutval, rng);
        nodes[id].divfeat = cutfeat;
        nodes[id].divval = cutval;
        const int c1 = divide_tree(ind, idx, rng);
        const int c2 = divide_tree(ind + idx, count - idx, rng);
        nodes[id].child1 = c1;
        nodes[id].child2 = c2;
        return id;
    }

    void build(int trees, TheRng& rng) {
        std::vector<int> ind(n);
        for (int i = 0; i < n; ++i) ind[i] = i;
        mean.assign(dim, 0.f);
        var.assign(dim, 0.f);
        nodes.reserve((size_t)trees * 2 * n);
        for (int t = 0; t < trees; ++t) {
            for (unsigned i = 0; i < (unsigned)n; ++i) {  // cv::randShuffle(ind)
                const unsigned j = rng.next() % (unsigned)n;
                std::swap(ind[j], ind[i]);
            }
            roots.push_back(divide_tree(ind.data(), n, rng));
        }
    }

    // flann::L2<float>: 4-way grouped squared differences (exact for SIFT's integer values)
    float l2(const float* a, const float* b) const {
        float result = 0.f;
        int i = 0;
        for (; i + 3 < dim; i += 4) {
            const float d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1], d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
            result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        }
        for (; i < dim; ++i) {
            const float d0 = a[i] - b[i];
            result += d0 * d0;
        }
        return result;
    }
};

struct Branch {
    int node;
    float mindist;
};
// Heap<BranchSt>: std::push_heap / pop_heap with CompareT(a, b) = b < a on mindist (a min-heap)
struct BranchGreater {
    bool operator()(const Branch& a, const Branch& b) const { return b.mindist < a.mindist; }
};

struct KnnUnique {  // KNNUniqueResultSet
    unsigned capacity;
    std::set<std::pair<float, int>> s;  // DistIndex order: (dist, index)
    bool full_ = false;
    float worst = std::numeric_limits<float>::max();
    void add(float dist, int index) {
        if (dist >= worst) return;
        s.insert({dist, index});
        if (full_) {
            if (s.size() > capacity) {
                s.erase(std::prev(s.end()));
                worst = std::prev(s.end())->first;
            }
        } else if (s.size() == capacity) {
            full_ = true;
            worst = std::prev(s.end())->first;
        }
    }
};

struct Searcher {
    const KDForest& F;
    const float* q;
    int max_checks;
    int check_count = 0;
    std::vector<uint8_t> checked;
    std::vector<Branch> heap;
    KnnUnique* res;

    void search_level(int node, float mindist) {
        if (res->worst < mindist) return;
        const Node& nd = F.nodes[node];
        if (nd.child1 < 0 && nd.child2 < 0) {
            const int index = nd.divfeat;
            if (checked[index] || (check_count >= max_checks && res->full_)) return;
            checked[index] = 1;
            check_count++;
            res->add(F.l2(F.vec(index), q), index);
            return;
        }
        const float val = q[nd.divfeat];
        const float diff = val - nd.divval;
        const int best = diff < 0 ? nd.child1 : nd.child2;
        const int other = diff < 0 ? nd.child2 : nd.child1;
        const float new_distsq = mindist + (val - nd.divval) * (val - nd.divval);
        if (new_distsq * 1.0f < res->worst || !res->full_) {
            if ((int)heap.size() < F.n) {  // Heap(size_) never fills in practice; insert drops when full
                heap.push_back(Branch{other, new_distsq});
                std::push_heap(heap.begin(), heap.end(), BranchGreater());
            }
        }
        search_level(best, mindist);
    }

    void run() {
        for (size_t t = 0; t < F.roots.size(); ++t) {
            search_level(F.roots[t], 0.f);
            if (check_count >= max_checks && res->full_) break;
        }
        while (!heap.empty()) {
            std::pop_heap(heap.begin(), heap.end(), BranchGreater());
            const Branch b = heap.back();
            heap.pop_back();
            if (!(check_count < max_checks || !res->full_)) break;
            search_level(b.node, b.mindist);
        }
    }
};

}  // namespace

extern "C" int ora_flann_knn(const float* dq, int nq, const float* dt, int nt, int dim, int k, int trees, int checks,
                             uint64_t* rng_state, int32_t* tidx, float* dist) {
    if (nq < 0 || nt < 1 || dim <= 0 || k < 1 || k > nt || trees < 1 || checks < 1 || !rng_state) return -1;
    TheRng rng{*rng_state};
    KDForest F{dt, nt, dim, {}, {}, {}, {}};
    F.build(trees, rng);
    *rng_state = rng.state;
    for (int qi = 0; qi < nq; ++qi) {
        KnnUnique res{(unsigned)k};
        Searcher S{F, dq + (size_t)qi * dim, checks, 0, std::vector<uint8_t>(nt, 0), {}, &res};
        S.run();
        int s = 0;
        for (auto it = res.s.begin(); it != res.s.end() && s < k; ++it, ++s) {
            tidx[(size_t)qi * k + s] = it->second;
            dist[(size_t)qi * k + s] = it->first;
        }
        for (; s < k; ++s) {  // getNeighbors asserts a full result; unreachable for k <= nt
            tidx[(size_t)qi * k + s] = -1;
            dist[(size_t)qi * k + s] = std::numeric_limits<float>::max();
        }
    }
    return 0;
}

// The theRNG state after `calls` index builds over train sets of sizes n[i]
// (trees * (2 n - 1) draws each): what the drop-in carries between calls.
extern "C" uint64_t ora_flann_rng_after(uint64_t state, const int32_t* n, int calls, int trees) {
    TheRng r{state};
    for (int c = 0; c < calls; ++c)
        for (long long d = 0; d < (long long)trees * (2LL * n[c] - 1); ++d) r.next();
    return r.state;
}
