// bow.hip -- bag-of-words kernels: DBoW2 TemplatedVocabulary::transform,
// BowVector / FeatureVector assembly, and ORBmatcher::SearchByBoW.
//
//   bow_transform_kernel   one thread per descriptor walks the vocabulary
//                          tree (TemplatedVocabulary.h:1242-1283): Hamming
//                          distance to each child, first minimum wins, the
//                          node passed at level L-levelsup is the direct-index
//                          node, the leaf gives word id and weight.
//   bow_vectors_kernel     one block per frame: (node, feature) and (word,
//                          feature) keys sorted in LDS (bitonic) give the
//                          FeatureVector (FeatureVector::addFeature appends
//                          in feature order) and the BowVector (addWeight
//                          sums a word's weights in feature order, then
//                          normalize() divides by the L1/L2 norm summed over
//                          words in ascending order, TemplatedVocabulary.h:
//                          1151-1230, BowVector.cpp:34-90).
//   search_by_bow_kernel   one block per frame pair; DBoW2 direct-index nodes
//                          partition the features, so nodes are independent
//                          and one lane walks one common node sequentially
//                          (ORBmatcher.cpp:205-348, :604-743); the rotation
//                          histogram, ComputeThreeMaxima and the cull follow.
//   triangulation_kernel   ORBmatcher::SearchForTriangulation (ORBmatcher.cpp:
//                          755-951) in the same shape: one block per keyframe
//                          pair, one lane per common node, the reference's
//                          inner loop (TH_LOW gate, last passing candidate
//                          among equal distances, epipole distance for
//                          monocular pairs, CheckDistEpipolarLine :166-190).
#include "../../include/orbgpu_bow.h"
#include "bow_kernels.h"
#include "device_state.h"

namespace orbgpu {

namespace {

constexpr int kMaxStride = 4096;
constexpr int kHL = 30, kThLow = 50;

__global__ __launch_bounds__(256) void bow_transform_kernel(VocabDev V, int batch, const uint8_t* __restrict__ desc,
                                                            const int* __restrict__ counts, int stride, int levelsup,
                                                            int* __restrict__ word, int* __restrict__ node,
                                                            double* __restrict__ weight) {
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    const int f = (int)(g / stride), i = (int)(g - (long)f * stride);
    if (f >= batch || i >= counts[f]) return;
    const size_t slot = (size_t)f * stride + i;
    const uint8_t* d = desc + 32 * slot;
    unsigned long long q[4];
    for (int k = 0; k < 4; ++k) q[k] = reinterpret_cast<const unsigned long long*>(d)[k];
    const int nid_level = V.L - levelsup;
    int nid = 0, fin = 0, level = 0;
    do {
        ++level;
        const int cs = V.child_start[fin], cc = V.child_count[fin];
        int best = V.children[cs], best_d = 0x7FFFFFFF;
        for (int j = 0; j < cc; ++j) {
            const int c = V.children[cs + j];
            const unsigned long long* e = reinterpret_cast<const unsigned long long*>(V.desc + 32 * (size_t)c);
            const int dd = __popcll(q[0] ^ e[0]) + __popcll(q[1] ^ e[1]) + __popcll(q[2] ^ e[2]) + __popcll(q[3] ^ e[3]);
            if (dd < best_d) {
                best_d = dd;
                best = c;
            }
        }
        fin = best;
        if (level == nid_level) nid = fin;
    } while (V.child_count[fin] > 0);
    word[slot] = V.word_id[fin];
    node[slot] = nid;
    weight[slot] = V.weight[fin];
}

// ascending bitonic sort of n (power of two) keys in LDS, all threads
__device__ void bitonic_sort(unsigned long long* k, int n) {
    for (int size = 2; size <= n; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = k[lo], b = k[hi];
                if ((a > b) == up) {
                    k[lo] = b;
                    k[hi] = a;
                }
            }
        }
    __syncthreads();
}

// exclusive prefix sum of flags[0..n) (n <= kMaxStride) into pos[], total returned to all threads
__device__ int block_scan(const unsigned char* flags, int* pos, int n, int* s_tmp) {
    const int per = (n + blockDim.x - 1) / blockDim.x;
    const int b = threadIdx.x * per, e = min(b + per, n);
    int sum = 0;
    for (int i = b; i < e; ++i) sum += flags[i];
    s_tmp[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int t = 0; t < (int)blockDim.x; ++t) {
            const int v = s_tmp[t];
            s_tmp[t] = acc;
            acc += v;
        }
        s_tmp[blockDim.x] = acc;
    }
    __syncthreads();
    int acc = s_tmp[threadIdx.x];
    for (int i = b; i < e; ++i) {
        pos[i] = acc;
        acc += flags[i];
    }
    const int total = s_tmp[blockDim.x];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(1024) void bow_vectors_kernel(VocabDev V, const int* __restrict__ counts, int stride,
                                                           const int* __restrict__ word, const int* __restrict__ node,
                                                           const double* __restrict__ weight,
                                                           int* __restrict__ fv_nodes, int* __restrict__ fv_offsets,
                                                           int* __restrict__ fv_features, int* __restrict__ fv_n,
                                                           int* __restrict__ bow_words, double* __restrict__ bow_values,
                                                           int* __restrict__ bow_n) {
    __shared__ unsigned long long s_key[kMaxStride];  // later reused as the BowVector values
    __shared__ unsigned char s_flag[kMaxStride];
    __shared__ int s_pos[kMaxStride];
    __shared__ int s_tmp[1025];
    __shared__ int s_kept;
    __shared__ double s_norm;
    const int f = blockIdx.x;
    const int n = counts[f];
    const size_t base = (size_t)f * stride;
    if (n > stride) {  // rejected, never truncated
        if (threadIdx.x == 0) fv_n[f] = bow_n[f] = -1;
        return;
    }
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    if (threadIdx.x == 0) s_kept = 0;
    // ---- FeatureVector: (node, feature) for features with weight > 0
    int kept = 0;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const bool in = i < n && weight[base + i] > 0;
        kept += in;
        s_key[i] = in ? ((unsigned long long)(unsigned)node[base + i] << 32) | (unsigned)i : ~0ull;
    }
    __syncthreads();
    atomicAdd(&s_kept, kept);
    bitonic_sort(s_key, n2);
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        s_flag[i] = s_key[i] != ~0ull && (i == 0 || (s_key[i] >> 32) != (s_key[i - 1] >> 32));
    __syncthreads();
    const int nnodes = block_scan(s_flag, s_pos, n, s_tmp);
    int* FO = fv_offsets + (size_t)f * (stride + 1);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (s_key[i] == ~0ull) continue;
        fv_features[base + i] = (int)(s_key[i] & 0xFFFFFFFFu);
        if (s_flag[i]) {
            fv_nodes[base + s_pos[i]] = (int)(s_key[i] >> 32);
            FO[s_pos[i]] = i;
        }
    }
    if (threadIdx.x == 0) {
        FO[nnodes] = s_kept;
        fv_n[f] = nnodes;
    }
    __syncthreads();
    // ---- BowVector: (word, feature) for features with weight > 0
    for (int i = threadIdx.x; i < n2; i += blockDim.x)
        s_key[i] = (i < n && weight[base + i] > 0) ? ((unsigned long long)(unsigned)word[base + i] << 32) | (unsigned)i
                                                   : ~0ull;
    bitonic_sort(s_key, n2);
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        s_flag[i] = s_key[i] != ~0ull && (i == 0 || (s_key[i] >> 32) != (s_key[i - 1] >> 32));
    __syncthreads();
    const int nwords = block_scan(s_flag, s_pos, n, s_tmp);
    const bool tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (!s_flag[i]) continue;
        double v = weight[base + (s_key[i] & 0xFFFFFFFFu)];
        if (tf)  // the word's weights summed in feature order
            for (int j = i + 1; j < n && s_key[j] != ~0ull && (s_key[j] >> 32) == (s_key[i] >> 32); ++j)
                v += weight[base + (s_key[j] & 0xFFFFFFFFu)];
        bow_values[base + s_pos[i]] = v;
        bow_words[base + s_pos[i]] = (int)(s_key[i] >> 32);
    }
    __syncthreads();
    double* s_val = reinterpret_cast<double*>(s_key);
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) s_val[w] = bow_values[base + w];
    __syncthreads();
    // mustNormalize: every scoring but DOT_PRODUCT (5); L2 norm for L2_NORM (1)
    const bool must = V.scoring != 5;
    if (threadIdx.x == 0) {
        double norm = 0.0;
        if (must) {
            if (V.scoring == 1) {
                for (int w = 0; w < nwords; ++w) norm += s_val[w] * s_val[w];
                norm = sqrt(norm);
            } else {
                for (int w = 0; w < nwords; ++w) norm += fabs(s_val[w]);
            }
        }
        s_norm = norm;
        bow_n[f] = nwords;
    }
    __syncthreads();
    const double norm = s_norm;
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        double v = s_val[w];
        if (!must && tf) v /= (double)nwords;
        if (must && norm > 0.0) v /= norm;
        bow_values[base + w] = v;
    }
}

__device__ inline int find_node(const int* nodes, int n, int key) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int v = nodes[mid];
        if (v == key) return mid;
        if (v < key) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
}

// Staging (kStage): kStage >= 1 copies the candidate frame's descriptors,
// FeatureVector feature list and valid flags, and the match state, to LDS
// with coalesced loads first; kStage == 2 also the query frame's.  The node
// walks then cost LDS round trips instead of dependent HBM ones (the walk is
// latency bound: round 2 measured 136 us for one 1000-feature pair, most of
// it in chained global loads).  The level is the largest whose bytes for
// `stride` features fit the budget.
constexpr int kBowStageMaxLds = 128 * 1024;
__host__ __device__ inline size_t bow_stage_bytes(int stride, int level) {
    // per feature: descB 32, fvfB 4, match 4, common-node record 16, B node id 4, angleB 4, validB 1 (+ descA
    // 32, fvfA 4, angleA 4, validA 1 at level 2)
    return level == 0 ? 0
                      : (size_t)stride * (32 + 4 + 4 + 16 + 4 + 4 + 1) +
                            (level == 2 ? (size_t)stride * (32 + 4 + 4 + 1) : 0) + 128;
}

// block-wide copy of n elements with kBatch loads per thread issued before
// any store (a plain copy loop waits for each load: one memory latency per
// iteration)
template <class T, int kBatch = 8>
__device__ __forceinline__ void stage_copy(T* __restrict__ dst, const T* __restrict__ src, int n) {
    for (int base = threadIdx.x; base < n; base += kBatch * blockDim.x) {
        T v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = base + k * (int)blockDim.x;
            v[k] = src[i < n ? i : n - 1];
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = base + k * (int)blockDim.x;
            if (i < n) dst[i] = v[k];
        }
    }
}

// (first minimum key, second smallest distance) over the lane's 8-lane row:
// three DPP exchanges (quad xor 1, xor 2, then the other quad of the half
// row), all within the row, so a row-uniform branch leaves no source lane
// disabled; min / max are order-free, so every pattern gives the same result.
// (ds_bpermute here cost ~100 cycles per exchange on the sequential walk.)
template <int Ctrl>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, Ctrl, 0xF, 0xF, false);
}
__device__ __forceinline__ void row8_best2(uint32_t& k1, uint32_t& d2) {
    auto step = [&](uint32_t ok1, uint32_t od2) {
        d2 = min(min(d2, od2), max(k1 >> 16, ok1 >> 16));
        k1 = min(k1, ok1);
    };
    step(dpp_u32<0xB1>(k1), dpp_u32<0xB1>(d2));    // quad_perm [1,0,3,2]
    step(dpp_u32<0x4E>(k1), dpp_u32<0x4E>(d2));    // quad_perm [2,3,0,1]
    step(dpp_u32<0x141>(k1), dpp_u32<0x141>(d2));  // row_half_mirror
}

#ifdef BOW_STAMPS  // diagnostic build only: phase stamps of block 0 (tools/bow_stamps.py)
__device__ unsigned long long g_bow_stamps[32];
#define BOW_T(k)                                                                                 \
    do {                                                                                         \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                          \
            g_bow_stamps[(k) < 4 ? (k) : (k) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define BOW_T(k) ((void)0)
#endif

constexpr int kBowThreads = 1024;  // 128 rows of 8 lanes: ~one common node per row for a 1000-feature pair

template <int kStage>
__global__ __launch_bounds__(kBowThreads) void search_by_bow_kernel(int mode, const orbgpu_bow_frame* __restrict__ A_,
                                                            const orbgpu_bow_frame* __restrict__ B_, float nnratio,
                                                            int check_ori, int stride, int* __restrict__ match_g,
                                                            int* __restrict__ nmatches) {
    __shared__ unsigned int s_used[kMaxStride / 32];  // vbMatched2 (KF_KF)
    __shared__ signed char s_bin[kMaxStride];
    __shared__ int s_hist[kHL];
    __shared__ int s_ind[3];
    __shared__ int s_cnt;
    __shared__ int s_npairs;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    BOW_T(0);
    const orbgpu_bow_frame A = A_[blockIdx.x], B = B_[blockIdx.x];
    const int nout = mode == ORBGPU_BOW_KF_F ? B.n : A.n;
    int* match_out = match_g + (size_t)blockIdx.x * stride;
    if (A.n > stride || B.n > stride) {  // rejected, never truncated
        if (threadIdx.x == 0) nmatches[blockIdx.x] = -1;
        return;
    }
    if (A.n == 0 || B.n == 0 || A.fv_n == 0 || B.fv_n == 0) {  // no common node: nothing matches
        for (int i = threadIdx.x; i < nout; i += blockDim.x) match_out[i] = -1;
        if (threadIdx.x == 0) nmatches[blockIdx.x] = 0;
        return;
    }
    // LDS carve: descB[stride] (32 B) | descA[stride] (level 2) | common-node records (16 B) | fvfB | fvfA (2) |
    // match | B node ids | angleB | angleA (2) | validB | validA (2).  The angles are staged too: a match's
    // rotation bin read them from HBM inside the sequential node walk (two dependent global loads per match)
    ulonglong4* s_descB = reinterpret_cast<ulonglong4*>(s_dyn);
    ulonglong4* s_descA = s_descB + (kStage == 2 ? stride : 0);
    int4* s_pairs = reinterpret_cast<int4*>(s_descA + (kStage == 2 ? stride : 0));  // (a0, na, b0, nb)
    int* s_fvfB = reinterpret_cast<int*>(s_pairs + stride);
    int* s_fvfA = s_fvfB + stride;
    int* s_match = s_fvfA + (kStage == 2 ? stride : 0);
    int* s_nodesB = s_match + stride;
    float* s_angB = reinterpret_cast<float*>(s_nodesB + stride);
    float* s_angA = s_angB + stride;
    unsigned char* s_validB = reinterpret_cast<unsigned char*>(s_angA + (kStage == 2 ? stride : 0));
    unsigned char* s_validA = s_validB + stride;
    int* match = kStage ? s_match : match_out;
    for (int i = threadIdx.x; i < nout; i += blockDim.x) {
        match[i] = -1;
        s_bin[i] = -1;
    }
    if constexpr (kStage >= 1) {
        // every staged array's loads of a round issued before its stores (one memory latency per round)
        // native vectors (HIP's uint4 is a union wrapper, and arrays of it
        // were kept in scratch memory)
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u* gdB = reinterpret_cast<const v4u*>(B.desc);
        const v4u* gdA = reinterpret_cast<const v4u*>(A.desc);
        v4u* sdB = reinterpret_cast<v4u*>(s_descB);
        v4u* sdA = reinterpret_cast<v4u*>(s_descA);
        const int nA = kStage == 2 ? A.n : 0;
        const int nmax = max(max(B.n, nA), B.fv_n);
        constexpr int kR = 2;  // elements per thread per round: up to 2048 features in one round trip
        for (int base = threadIdx.x; base < nmax; base += kR * blockDim.x) {
            v4u db[2 * kR], da[2 * kR];
            int fb[kR], fa[kR], nd[kR];
            float gb[kR], ga[kR];
            unsigned char vb[kR], va[kR];
#pragma unroll
            for (int k = 0; k < kR; ++k) {  // clamped indices (every array is non-empty here)
                const int i = base + k * (int)blockDim.x;
                const int ib = min(i, B.n - 1), ia = min(i, nA - 1);
                db[2 * k] = gdB[2 * ib];
                db[2 * k + 1] = gdB[2 * ib + 1];
                fb[k] = B.fv_features[ib];
                gb[k] = check_ori ? B.angle[ib] : 0.f;  // angles may be absent without the orientation check
                vb[k] = B.valid[ib];
                nd[k] = B.fv_nodes[min(i, B.fv_n - 1)];
                if (kStage == 2) {
                    da[2 * k] = gdA[2 * ia];
                    da[2 * k + 1] = gdA[2 * ia + 1];
                    fa[k] = A.fv_features[ia];
                    ga[k] = check_ori ? A.angle[ia] : 0.f;
                    va[k] = A.valid[ia];
                }
            }
#pragma unroll
            for (int k = 0; k < kR; ++k) {
                const int i = base + k * (int)blockDim.x;
                if (i < B.n) {
                    sdB[2 * i] = db[2 * k];
                    sdB[2 * i + 1] = db[2 * k + 1];
                    s_fvfB[i] = fb[k];
                    s_angB[i] = gb[k];
                    s_validB[i] = vb[k];
                }
                if (i < B.fv_n) s_nodesB[i] = nd[k];
                if (kStage == 2 && i < nA) {
                    sdA[2 * i] = da[2 * k];
                    sdA[2 * i + 1] = da[2 * k + 1];
                    s_fvfA[i] = fa[k];
                    s_angA[i] = ga[k];
                    s_validA[i] = va[k];
                }
            }
        }
    }
    for (int i = threadIdx.x; i < kMaxStride / 32; i += blockDim.x) s_used[i] = 0;
    if (threadIdx.x < kHL) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        s_cnt = 0;
        s_npairs = 0;
    }
    __syncthreads();
    BOW_T(1);
    if constexpr (kStage >= 1) {
        // the common direct-index nodes and their feature ranges, found by
        // every thread at once (one binary search each, over B's node ids in
        // LDS) instead of by each row before its node
        for (int a = threadIdx.x; a < A.fv_n; a += blockDim.x) {
            const int b = find_node(s_nodesB, B.fv_n, A.fv_nodes[a]);
            if (b >= 0) {
                const int a0 = A.fv_offsets[a], b0 = B.fv_offsets[b];
                s_pairs[atomicAdd(&s_npairs, 1)] = make_int4(a0, A.fv_offsets[a + 1] - a0, b0, B.fv_offsets[b + 1] - b0);
            }
        }
        __syncthreads();
    }
    BOW_T(2);
    auto fvfA = [&](int k) { return kStage == 2 ? s_fvfA[k] : A.fv_features[k]; };
    auto validA = [&](int i) { return kStage == 2 ? s_validA[i] != 0 : A.valid[i] != 0; };
    auto descA = [&](int i) {
        return kStage == 2 ? s_descA[i] : *reinterpret_cast<const ulonglong4*>(A.desc + 32 * (size_t)i);
    };
    auto fvfB = [&](int k) { return kStage ? s_fvfB[k] : B.fv_features[k]; };
    auto descB = [&](int i) { return kStage ? s_descB[i] : *reinterpret_cast<const ulonglong4*>(B.desc + 32 * (size_t)i); };
    auto validB = [&](int i) { return kStage ? s_validB[i] != 0 : B.valid[i] != 0; };
    auto angA = [&](int i) { return kStage == 2 ? s_angA[i] : A.angle[i]; };
    auto angB = [&](int i) { return kStage ? s_angB[i] : B.angle[i]; };
    auto sync_match = [&] {  // lane 0's match / vbMatched2 update visible to its row before the next A feature
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    const float factor = (float)kHL / 360.0f;
    // One common direct-index node per 8-lane row (32 rows per block).  The
    // node's A features are taken in the reference's order (the match state
    // they leave feeds the next one); for each, the row's lanes scan the
    // node's B features (lane r: positions r, r + 8, ...) and the row
    // reduces (dist << 16 | position) -- the reference keeps the FIRST
    // minimum in node order -- and the second smallest distance of the
    // multiset (bestDist2: an equal second minimum counts).  A lane per node
    // (round 2) ran a whole skewed node serially.
    constexpr int kRow = 8;
    constexpr int kRegC = 4;  // candidates per lane held in registers (nodes of up to 32 B features)
    const int r16 = threadIdx.x & (kRow - 1), row = threadIdx.x / kRow, nrows = blockDim.x / kRow;
    const int nwork = kStage >= 1 ? s_npairs : A.fv_n;  // nodes are independent: any order
    for (int w = row; w < nwork; w += nrows) {
        int a0, a1, b0, nb;
        if constexpr (kStage >= 1) {
            const int4 pr = s_pairs[w];
            a0 = pr.x;
            a1 = pr.x + pr.y;
            b0 = pr.z;
            nb = pr.w;
        } else {
            const int b = find_node(B.fv_nodes, B.fv_n, A.fv_nodes[w]);
            if (b < 0) continue;
            a0 = A.fv_offsets[w];
            a1 = A.fv_offsets[w + 1];
            b0 = B.fv_offsets[b];
            nb = B.fv_offsets[b + 1] - b0;
        }
        if (nb <= kRow * kRegC) {
            // The node's B features are the same for all of its A features:
            // the row loads them once into registers (lane r: positions r, r +
            // 8, ...) with their skip flags, and keeps the flags current
            // itself (nodes partition B, so only this row changes them: a
            // match clears the matched candidate in its owner lane).  An A
            // feature then costs its own loads, the distances and the row
            // reduction, with no LDS round trip per candidate.
            ulonglong4 cd[kRegC];
            bool ok[kRegC];
#pragma unroll
            for (int c = 0; c < kRegC; ++c) {
                const int j = r16 + kRow * c;
                const int ib = fvfB(b0 + min(j, nb - 1));  // clamped: every slot loaded, unused ones flagged off
                cd[c] = descB(ib);
                ok[c] = j < nb && (mode == ORBGPU_BOW_KF_F ? match[ib] < 0
                                                           : !(((s_used[ib >> 5] >> (ib & 31)) & 1u) || !validB(ib)));
            }
            for (int ia_ = a0; ia_ < a1; ++ia_) {
                const int ia = fvfA(ia_);
                if (!validA(ia)) continue;
                const ulonglong4 qa = descA(ia);
                uint32_t k1 = 0xFFFFFFFFu, d2 = 0xFFFFu;
#pragma unroll
                for (int c = 0; c < kRegC; ++c) {  // predicated: cd[] stays in registers
                    if (c > 0 && !__any(r16 + kRow * c < nb)) break;  // no row of the wave has slot c
                    const uint32_t dist = __popcll(qa.x ^ cd[c].x) + __popcll(qa.y ^ cd[c].y) +
                                          __popcll(qa.z ^ cd[c].z) + __popcll(qa.w ^ cd[c].w);
                    const uint32_t key = ok[c] ? ((dist << 16) | (uint32_t)(r16 + kRow * c)) : 0xFFFFFFFFu;
                    const uint32_t dm = ok[c] ? dist : 0xFFFFu;
                    const bool lt = key < k1;
                    d2 = min(d2, lt ? (k1 >> 16) : dm);
                    k1 = lt ? key : k1;
                }
                row8_best2(k1, d2);
                const int best1 = k1 == 0xFFFFFFFFu ? 256 : (int)(k1 >> 16);
                const int best2 = d2 >= 256u ? 256 : (int)d2;
                const bool pass = mode == ORBGPU_BOW_KF_F ? best1 <= kThLow : best1 < kThLow;
                if (!pass || !((float)best1 < nnratio * (float)best2)) continue;  // row-uniform
                const int pos = (int)(k1 & 0xFFFFu);
#pragma unroll
                for (int c = 0; c < kRegC; ++c)
                    if (r16 + kRow * c == pos) ok[c] = false;  // matched: skipped by later A features
                if (r16 == 0) {
                    const int bidx = fvfB(b0 + pos);
                    int out;
                    if (mode == ORBGPU_BOW_KF_F) {
                        match[bidx] = ia;
                        out = bidx;
                    } else {
                        match[ia] = bidx;
                        atomicOr(&s_used[bidx >> 5], 1u << (bidx & 31));
                        out = ia;
                    }
                    if (check_ori) {
                        float rot = angA(ia) - angB(bidx);
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == kHL) bin = 0;
                        s_bin[out] = (signed char)bin;
                        atomicAdd(&s_hist[bin], 1);
                    }
                }
            }
            continue;
        }
        for (int ia_ = a0; ia_ < a1; ++ia_) {
            const int ia = fvfA(ia_);
            if (!validA(ia)) continue;
            const ulonglong4 qa = descA(ia);
            uint32_t k1 = 0xFFFFFFFFu;  // (dist << 16 | position) of the lane's first minimum
            uint32_t d2 = 0xFFFFu;      // the lane's second smallest distance
            for (int j = r16; j < nb; j += kRow) {
                const int ib = fvfB(b0 + j);
                const bool skip = mode == ORBGPU_BOW_KF_F ? match[ib] >= 0
                                                          : (((s_used[ib >> 5] >> (ib & 31)) & 1u) || !validB(ib));
                if (skip) continue;
                const ulonglong4 qb = descB(ib);
                const uint32_t dist = __popcll(qa.x ^ qb.x) + __popcll(qa.y ^ qb.y) + __popcll(qa.z ^ qb.z) +
                                      __popcll(qa.w ^ qb.w);
                const uint32_t key = (dist << 16) | (uint32_t)j;
                if (key < k1) {
                    d2 = min(d2, k1 >> 16);
                    k1 = key;
                } else {
                    d2 = min(d2, dist);
                }
            }
            row8_best2(k1, d2);  // row reduction within the row's 8 lanes
            const int best1 = k1 == 0xFFFFFFFFu ? 256 : (int)(k1 >> 16);
            const int best2 = d2 >= 256u ? 256 : (int)d2;
            const bool pass = mode == ORBGPU_BOW_KF_F ? best1 <= kThLow : best1 < kThLow;
            if (!pass || !((float)best1 < nnratio * (float)best2)) continue;  // row-uniform
            const int bidx = fvfB(b0 + (int)(k1 & 0xFFFFu));
            if (r16 == 0) {
                int out;
                if (mode == ORBGPU_BOW_KF_F) {
                    match[bidx] = ia;
                    out = bidx;
                } else {
                    match[ia] = bidx;
                    atomicOr(&s_used[bidx >> 5], 1u << (bidx & 31));
                    out = ia;
                }
                if (check_ori) {
                    float rot = angA(ia) - angB(bidx);
                    if (rot < 0.0f) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == kHL) bin = 0;
                    s_bin[out] = (signed char)bin;
                    atomicAdd(&s_hist[bin], 1);
                }
            }
            sync_match();
        }
    }
    BOW_T(8);  // slots 8..11: each wave's end of the node walk
    __syncthreads();
    BOW_T(3);
    if (check_ori && threadIdx.x == 0) {  // ComputeThreeMaxima (ORBmatcher.cpp:1792-1833)
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHL; ++i) {
            const int s = s_hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) ind3 = -1;
        s_ind[0] = ind1;
        s_ind[1] = ind2;
        s_ind[2] = ind3;
    }
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < nout; i += blockDim.x) {
        int m = match[i];
        if (m >= 0) {
            const int bin = s_bin[i];
            if (check_ori && bin != s_ind[0] && bin != s_ind[1] && bin != s_ind[2]) m = -1;
            else ++cnt;
        }
        match_out[i] = m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_cnt, cnt);  // one LDS atomic per wave, not per thread
    __syncthreads();
    if (threadIdx.x == 0) nmatches[blockIdx.x] = s_cnt;
#ifdef BOW_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0) g_bow_stamps[30] = __builtin_amdgcn_s_memtime();
#endif
}

#ifdef BOW_STAMPS
extern "C" int orbgpu_debug_bow_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bow_stamps), sizeof(g_bow_stamps)) == hipSuccess ? 0 : -2;
}
#endif

// ComputeThreeMaxima (ORBmatcher.cpp:1792-1833) over s_hist into s_ind[3]
__device__ inline void three_maxima(const int* s_hist, int* s_ind) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHL; ++i) {
        const int s = s_hist[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if ((float)max3 < 0.1f * (float)max1) ind3 = -1;
    s_ind[0] = ind1;
    s_ind[1] = ind2;
    s_ind[2] = ind3;
}

__global__ __launch_bounds__(256) void triangulation_kernel(const orbgpu_triangulation_pair* __restrict__ pairs,
                                                            int check_ori, int stride, int* __restrict__ match_g,
                                                            int* __restrict__ nmatches) {
    __shared__ unsigned int s_used[kMaxStride / 32];  // vbMatched2
    __shared__ signed char s_bin[kMaxStride];
    __shared__ int s_hist[kHL];
    __shared__ int s_ind[3];
    __shared__ int s_cnt;
    __shared__ float s_e[2];  // epipole (ex, ey)
    const orbgpu_triangulation_pair& P = pairs[blockIdx.x];
    const orbgpu_bow_frame& A = P.kf1;
    const orbgpu_bow_frame& B = P.kf2;
    int* match = match_g + (size_t)blockIdx.x * stride;
    if (A.n > stride || B.n > stride) {  // rejected, never truncated
        if (threadIdx.x == 0) nmatches[blockIdx.x] = -1;
        return;
    }
    for (int i = threadIdx.x; i < A.n; i += blockDim.x) {
        match[i] = -1;
        s_bin[i] = -1;
    }
    for (int i = threadIdx.x; i < kMaxStride / 32; i += blockDim.x) s_used[i] = 0;
    if (threadIdx.x < kHL) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        s_cnt = 0;
        // C2 = R2w*Cw + t2w (cv::Mat product accumulated in double), epipole (:763-770)
        float C2[3];
        for (int r = 0; r < 3; ++r)
            C2[r] = (float)((double)P.T2w[4 * r] * P.Cw1[0] + (double)P.T2w[4 * r + 1] * P.Cw1[1] +
                            (double)P.T2w[4 * r + 2] * P.Cw1[2]) + P.T2w[4 * r + 3];
        const float invz = 1.0f / C2[2];
        s_e[0] = P.fx2 * C2[0] * invz + P.cx2;
        s_e[1] = P.fy2 * C2[1] * invz + P.cy2;
    }
    __syncthreads();
    const float ex = s_e[0], ey = s_e[1];
    const float* F = P.F12;
    const float factor = (float)kHL / 360.0f;
    for (int a = threadIdx.x; a < A.fv_n; a += blockDim.x) {
        const int b = find_node(B.fv_nodes, B.fv_n, A.fv_nodes[a]);
        if (b < 0) continue;
        const int a0 = A.fv_offsets[a], a1 = A.fv_offsets[a + 1];
        const int b0 = B.fv_offsets[b], b1 = B.fv_offsets[b + 1];
        for (int ia_ = a0; ia_ < a1; ++ia_) {
            const int idx1 = A.fv_features[ia_];
            if (!A.valid[idx1]) continue;  // pKF1 already has a MapPoint there
            const bool stereo1 = P.u_right1 && P.u_right1[idx1] >= 0.0f;
            if (P.only_stereo && !stereo1) continue;
            const orbgpu_keypoint kp1 = P.kps1[idx1];
            // epipolar line of kp1 in KF2 (CheckDistEpipolarLine), the same for every candidate
            const float la = kp1.x * F[0] + kp1.y * F[3] + F[6];
            const float lb = kp1.x * F[1] + kp1.y * F[4] + F[7];
            const float lc = kp1.x * F[2] + kp1.y * F[5] + F[8];
            const float den = la * la + lb * lb;
            const ulonglong4 q1 = *reinterpret_cast<const ulonglong4*>(A.desc + 32 * (size_t)idx1);
            int bestDist = kThLow, bestIdx2 = -1;
            // four candidates per memory round trip (as in search_by_bow_kernel), then
            // the reference's tests in candidate order; vbMatched2 only changes after
            // this loop, in this lane
            for (int base = b0; base < b1; base += 4) {
              int ids[4];
              bool st2[4], skip[4];
              ulonglong4 q2[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) ids[u] = B.fv_features[min(base + u, b1 - 1)];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                  const int id = ids[u];
                  st2[u] = P.u_right2 && P.u_right2[id] >= 0.0f;
                  skip[u] = ((s_used[id >> 5] >> (id & 31)) & 1u) || !B.valid[id];
                  q2[u] = *reinterpret_cast<const ulonglong4*>(B.desc + 32 * (size_t)id);
              }
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int idx2 = ids[u];
                if (base + u >= b1 || skip[u]) continue;
                const bool stereo2 = st2[u];
                if (P.only_stereo && !stereo2) continue;
                const int dist = __popcll(q1.x ^ q2[u].x) + __popcll(q1.y ^ q2[u].y) + __popcll(q1.z ^ q2[u].z) +
                                 __popcll(q1.w ^ q2[u].w);
                if (dist > kThLow || dist > bestDist) continue;
                const orbgpu_keypoint kp2 = P.kps2[idx2];
                if (!stereo1 && !stereo2) {  // too close to the epipole: the point is too close to KF1
                    const float dx = ex - kp2.x, dy = ey - kp2.y;
                    if (dx * dx + dy * dy < 100 * P.scale_factors2[kp2.octave & 15]) continue;
                }
                if (den == 0.0f) continue;
                const float num = la * kp2.x + lb * kp2.y + lc;
                const float dsqr = num * num / den;
                if ((double)dsqr < 3.84 * (double)P.level_sigma2_2[kp2.octave & 15]) {
                    bestIdx2 = idx2;
                    bestDist = dist;
                }
              }
            }
            if (bestIdx2 < 0) continue;
            match[idx1] = bestIdx2;
            atomicOr(&s_used[bestIdx2 >> 5], 1u << (bestIdx2 & 31));
            if (check_ori) {
                float rot = A.angle[idx1] - B.angle[bestIdx2];
                if (rot < 0.0f) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == kHL) bin = 0;
                s_bin[idx1] = (signed char)bin;
                atomicAdd(&s_hist[bin], 1);
            }
        }
    }
    __syncthreads();
    if (check_ori && threadIdx.x == 0) three_maxima(s_hist, s_ind);
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < A.n; i += blockDim.x) {
        if (match[i] < 0) continue;
        const int bin = s_bin[i];
        if (check_ori && bin != s_ind[0] && bin != s_ind[1] && bin != s_ind[2]) {
            match[i] = -1;
            continue;
        }
        ++cnt;
    }
    atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0) nmatches[blockIdx.x] = s_cnt;
}

// DBoW2 GeneralScoring::score (ScoringObject.cpp:23-313) of the query
// BowVector against keyframe k's, one thread per keyframe: the reference's
// merge walk in ascending word order (lower_bound skips == stepping), the
// double sum in that order; plus the number of common words (the mnLoopWords /
// mnRelocWords counts of KeyFrameDatabase.cpp:107-125, 250-262).
__global__ __launch_bounds__(256) void bow_db_score_kernel(int scoring, const int* __restrict__ qw,
                                                           const double* __restrict__ qv, int nq, int nkf,
                                                           const int* __restrict__ off, const int* __restrict__ dw,
                                                           const double* __restrict__ dv, int* __restrict__ common,
                                                           double* __restrict__ score) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= nkf) return;
    const double LOG_EPS = log(2.220446049250313080847e-16);  // log(DBL_EPSILON)
    int i = 0, j = off[k];
    const int je = off[k + 1];
    double s = 0.0;
    int nc = 0;
    while (i < nq && j < je) {
        const int a = qw[i], b = dw[j];
        const double vi = qv[i], wi = dv[j];
        if (a == b) {
            ++nc;
            switch (scoring) {
                case 0: s += fabs(vi - wi) - fabs(vi) - fabs(wi); break;     // L1
                case 1: case 5: s += vi * wi; break;                         // L2, dot product
                case 2: if (vi + wi != 0.0) s += vi * wi / (vi + wi); break; // chi-square
                case 3: if (vi != 0 && wi != 0) s += vi * log(vi / wi); break;  // KL
                default: s += sqrt(vi * wi); break;                          // Bhattacharyya
            }
            ++i;
            ++j;
        } else if (a < b) {
            if (scoring == 3) s += vi * (log(vi) - LOG_EPS);  // KL walks every query word
            ++i;
        } else {
            ++j;
        }
    }
    if (scoring == 3)
        for (; i < nq; ++i)
            if (qv[i] != 0) s += qv[i] * (log(qv[i]) - LOG_EPS);
    if (scoring == 0) s = -s / 2.0;
    else if (scoring == 1) s = s >= 1 ? 1.0 : 1.0 - sqrt(1.0 - s);
    else if (scoring == 2) s = 2. * s;
    // common words count every query word once (the inverted-file loop visits each
    // (word, keyframe) entry once)
    if (scoring == 3) {  // the KL walk advanced i past non-common words too: count separately
        nc = 0;
        int ii = 0, jj = off[k];
        while (ii < nq && jj < je) {
            const int a = qw[ii], b = dw[jj];
            if (a == b) { ++nc; ++ii; ++jj; }
            else if (a < b) ++ii;
            else ++jj;
        }
    }
    common[k] = nc;
    score[k] = s;
}

}  // namespace

int bow_max_stride() { return kMaxStride; }

hipError_t launch_bow_transform(const VocabDev& V, int batch, const uint8_t* desc, const int* counts, int stride,
                                int levelsup, int* word, int* node, double* weight, int* fv_nodes, int* fv_offsets,
                                int* fv_features, int* fv_n, int* bow_words, double* bow_values, int* bow_n,
                                hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    const long total = (long)batch * stride;
    hipLaunchKernelGGL(bow_transform_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, V, batch,
                       desc, counts, stride, levelsup, word, node, weight);
    hipLaunchKernelGGL(bow_vectors_kernel, dim3(batch), dim3(1024), 0, stream, V, counts, stride, word, node, weight,
                       fv_nodes, fv_offsets, fv_features, fv_n, bow_words, bow_values, bow_n);
    return hipGetLastError();
}

hipError_t launch_search_by_bow(int mode, int batch, const orbgpu_bow_frame* a, const orbgpu_bow_frame* b,
                                float nnratio, int check_ori, int stride, int* match, int* nmatches,
                                hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    // the staged variants' LDS limit, once per device (device_state.h)
    static PerDeviceOnce attr_once;
    const hipError_t attr = attr_once.get([](int) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&search_by_bow_kernel<1>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kBowStageMaxLds);
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(&search_by_bow_kernel<2>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kBowStageMaxLds);
        return e;
    });
    if (attr != hipSuccess) return attr;
    if (bow_stage_bytes(stride, 2) <= (size_t)kBowStageMaxLds)
        hipLaunchKernelGGL(search_by_bow_kernel<2>, dim3(batch), dim3(kBowThreads), bow_stage_bytes(stride, 2), stream, mode,
                           a, b, nnratio, check_ori, stride, match, nmatches);
    else if (bow_stage_bytes(stride, 1) <= (size_t)kBowStageMaxLds)
        hipLaunchKernelGGL(search_by_bow_kernel<1>, dim3(batch), dim3(kBowThreads), bow_stage_bytes(stride, 1), stream, mode,
                           a, b, nnratio, check_ori, stride, match, nmatches);
    else
        hipLaunchKernelGGL(search_by_bow_kernel<0>, dim3(batch), dim3(kBowThreads), 0, stream, mode, a, b, nnratio,
                           check_ori, stride, match, nmatches);
    return hipGetLastError();
}

hipError_t launch_bow_db_score(int scoring, const int* qw, const double* qv, int nq, int nkf, const int* off,
                               const int* dw, const double* dv, int* common, double* score, hipStream_t stream) {
    if (nkf <= 0) return hipSuccess;
    hipLaunchKernelGGL(bow_db_score_kernel, dim3((nkf + 255) / 256), dim3(256), 0, stream, scoring, qw, qv, nq, nkf,
                       off, dw, dv, common, score);
    return hipGetLastError();
}

hipError_t launch_search_for_triangulation(int batch, const orbgpu_triangulation_pair* pairs, int check_ori, int stride,
                                          int* match, int* nmatches, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(triangulation_kernel, dim3(batch), dim3(256), 0, stream, pairs, check_ori, stride, match,
                       nmatches);
    return hipGetLastError();
}

}  // namespace orbgpu
