// octree.hip -- ORBextractor::DistributeOctTree (ORBextractor.cpp:541-770)
// for one (frame, level) per 256-thread workgroup.
//
// The reference mutates a std::list of quadtree nodes.  This kernel restates
// it as level-synchronous passes over flat arrays, keeping the list ORDER
// (which is the output order) exact:
//   * node array = the list in order; a pass writes the next list into a
//     ping-pong buffer: children of the divided nodes in reverse push order
//     (push_front), then the untouched nodes in their old order;
//   * main-loop pass (:610-669): every node with > 1 key is divided, in list
//     order;
//   * inner-loop pass (:681-743): the nodes with > 1 key (== the reference's
//     vSizeAndPointerToNode at that point) are divided in descending
//     (size, creation seq) order and the pass stops right after the division
//     that makes the list reach N -- found with a prefix sum of (children-1);
//   * each key carries its node index; a pass is two sweeps over the keys
//     (quadrant histogram via LDS atomics, then remap to the child/new slot);
//   * finally the max-response key per node (first in candidate order on
//     ties, :751-767) via one LDS atomicMax of (score << 24 | ~index).
// The reference breaks size ties by heap address (:690); here ties are
// broken by creation sequence number, the documented deviation,
// identical to the oracle.
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "group_sum.h"
#include <algorithm>
#include <type_traits>

namespace orbgpu {

namespace {

#ifndef ORBGPU_OCT_THREADS
#define ORBGPU_OCT_THREADS 256
#endif
#ifndef ORBGPU_OCT_AGG_HIST
#define ORBGPU_OCT_AGG_HIST 1
#endif
constexpr bool kAggHist = ORBGPU_OCT_AGG_HIST != 0;
constexpr int kThreads = ORBGPU_OCT_THREADS;  // large batches: 6 workgroups per CU at 640x480 (LDS-bound)
#ifndef ORBGPU_OCT_THREADS_SMALL
#define ORBGPU_OCT_THREADS_SMALL 1024
#endif
constexpr int kThreadsSmall = ORBGPU_OCT_THREADS_SMALL;  // a few frames: one workgroup per (frame, level) on its own CU
constexpr int kSmallBatch = 8;       // batches up to this size take kThreadsSmall

struct ONode {
    uint32_t r0;   // x0 | y0 << 16
    uint32_t r1;   // x1 | y1 << 16
    uint32_t cnt;  // keys in node
    uint32_t seq;  // creation sequence number
};

__device__ inline int node_quad(const ONode& n, uint32_t key) {
    const int x0 = n.r0 & 0xFFFF, y0 = n.r0 >> 16, x1 = n.r1 & 0xFFFF, y1 = n.r1 >> 16;
    const int mx = x0 + ((x1 - x0 + 1) >> 1);  // ceil((float)(UR.x-UL.x)/2), ExtractorNode::DivideNode :485
    const int my = y0 + ((y1 - y0 + 1) >> 1);
    return (key_x(key) < mx ? 0 : 1) + (key_y(key) < my ? 0 : 2);
}

__device__ inline ONode child_rect(const ONode& n, int q) {
    const int x0 = n.r0 & 0xFFFF, y0 = n.r0 >> 16, x1 = n.r1 & 0xFFFF, y1 = n.r1 >> 16;
    const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
    const int cx0 = (q & 1) ? mx : x0, cx1 = (q & 1) ? x1 : mx;
    const int cy0 = (q & 2) ? my : y0, cy1 = (q & 2) ? y1 : my;
    ONode c;
    c.r0 = (uint32_t)cx0 | ((uint32_t)cy0 << 16);
    c.r1 = (uint32_t)cx1 | ((uint32_t)cy1 << 16);
    c.cnt = 0;
    c.seq = 0;
    return c;
}

__device__ inline int wave_incl_scan(int v) { return wave_incl_scan_dpp(v); }

// In-place exclusive scan of a[0..n) in LDS by the whole block; returns total.
template <int NT>
__device__ int block_scan(int* a, int n, int* s_tmp) {
    const int per = (n + NT - 1) / NT;
    const int beg = min(n, (int)threadIdx.x * per), end = min(n, beg + per);
    int sum = 0;
    for (int i = beg; i < end; ++i) sum += a[i];
    const int incl = wave_incl_scan(sum);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) s_tmp[wave] = incl;
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const int t = s_tmp[w];
        if (w < wave) off += t;
        total += t;
    }
    int run = off + incl - sum;
    for (int i = beg; i < end; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// Key storage: LDS when the level's candidates fit, else an HBM scratch
// region.  Accessed through a uniform branch so that the LDS case compiles
// to ds_* instructions (a generic pointer would force flat_* accesses).
template <bool LDS>
struct KeyStore {
    uint32_t* keys;
    uint16_t* nodes;
    __device__ uint32_t key(int k) const { return keys[k]; }
    __device__ int node(int k) const { return (int)nodes[k]; }
    __device__ void set_key(int k, uint32_t v) const { keys[k] = v; }
    __device__ void set_node(int k, int v) const { nodes[k] = (uint16_t)v; }
};

// The quadrant histogram of each node (4 counters per node; after the push
// the counters hold the children's list positions).  With the keys in LDS a
// level has at most kcap (< 2^16) keys, so the counters are u16, bumped with
// a 32-bit LDS atomic on the pair's dword; the HBM-scratch path (any number
// of keys) keeps u32 counters, in the LDS region the keys would have used.
template <bool LDS>
struct QuadCounts;

template <>
struct QuadCounts<true> {
    uint16_t* h;
    __device__ void zero(int nodes, int tid, int nt) const {
        uint32_t* w = reinterpret_cast<uint32_t*>(h);
        for (int i = tid; i < nodes * 2; i += nt) w[i] = 0u;
    }
    __device__ void add(int i, int q, uint32_t n = 1u) const {
        atomicAdd(reinterpret_cast<uint32_t*>(h) + i * 2 + (q >> 1), n << ((q & 1) << 4));
    }
    __device__ uint32_t get(int i, int q) const { return h[i * 4 + q]; }
    __device__ void set(int i, int q, int v) const { h[i * 4 + q] = (uint16_t)v; }
    __device__ int nonzero(int i) const {  // children a divided node would have
        const uint2 v = reinterpret_cast<const uint2*>(h)[i];
        return ((v.x & 0xFFFFu) != 0) + ((v.x >> 16) != 0) + ((v.y & 0xFFFFu) != 0) + ((v.y >> 16) != 0);
    }
};

template <>
struct QuadCounts<false> {
    uint32_t* w;
    __device__ void zero(int nodes, int tid, int nt) const {
        for (int i = tid; i < nodes * 4; i += nt) w[i] = 0u;
    }
    __device__ void add(int i, int q, uint32_t n = 1u) const { atomicAdd(&w[i * 4 + q], n); }
    __device__ uint32_t get(int i, int q) const { return w[i * 4 + q]; }
    __device__ void set(int i, int q, int v) const { w[i * 4 + q] = (uint32_t)v; }
    __device__ int nonzero(int i) const {
        const uint4 v = reinterpret_cast<const uint4*>(w)[i];
        return (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
    }
};

__device__ inline int pow2ceil(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Diagnostic build (-DOCT_STAMPS): thread 0 of frame 0's workgroups records
// s_memtime at phase boundaries into the debug trace (ints 384.. of the
// level's 512-int record, 64-bit stamps); tools/octree_trace.py prints them.
#ifdef OCT_STAMPS
#define OCT_T(k)                                                                                      \
    do {                                                                                              \
        if (trace && f == 0 && threadIdx.x == 0 && (k) < 64) {                                        \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
            trace[l * 512 + 384 + 2 * (k)] = (int)(t_ & 0xFFFFFFFFu);                               \
            trace[l * 512 + 385 + 2 * (k)] = (int)(t_ >> 32);                                        \
        }                                                                                             \
    } while (0)
#else
#define OCT_T(k) ((void)0)
#endif

__device__ inline void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One pass over a list of nL <= 64 nodes by wave 0 alone (lane = node): the
// same ordering, push bases, kept-node positions and pushes as the block path
// below, with wave scans and ballots instead of block scans and barriers.
//   main pass (:610-669): every node with > 1 key is divided, in list order;
//   inner pass (:681-743): the nodes with > 1 key in descending (size, seq)
//   order, up to and including the division that makes the list reach N.
// Publishes C, S and an error code in s_misc[20..22], the children with > 1
// key in *s_nexp; s_flag / s_aux1 / the quadrant counters as the remap reads
// them.  (Inner-pass scratch: the sort keys in the next list's buffer, the
// rank-ordered child counts in s_aux1 and push bases in s_aux0 -- all read
// before the pushes and the kept positions overwrite them, in wave order.)
template <class QC>
__device__ void wave_small_pass(const ONode* old, ONode* nw, unsigned long long* s_sortk, const QC& qc, int* s_aux0,
                                int* s_aux1, uint8_t* s_flag, int* s_misc, int* s_nexp, int nL, int N, int ncap,
                                int nseq, bool inner, int lane) {
    const bool valid = lane < nL;
    ONode nd{};
    if (valid) nd = old[lane];
    const bool div = valid && nd.cnt > 1;
    const int nch = div ? qc.nonzero(lane) : 0;
    bool flag;
    int C, S, base, spos;
    if (!inner) {
        // (children << 16 | kept) scanned together, as the block path
        const int v = valid ? (div ? nch << 16 : 1) : 0;
        const int incl = wave_incl_scan_dpp(v);
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        C = tot >> 16;
        S = tot & 0xFFFF;
        flag = div;
        base = (incl - v) >> 16;
        spos = (incl - v) & 0xFFFF;
    } else {
        // descending (cnt, seq) rank among the dividing nodes (keys distinct:
        // they end in the node index)
        const unsigned long long key =
            div ? ((unsigned long long)min(nd.cnt, 0xFFFFFFu) << 40) | ((unsigned long long)(nd.seq & 0xFFFFFFFu) << 12) |
                      (unsigned)lane
                : 0ull;
        if (valid) s_sortk[lane] = key;
        wave_sync();
        int rank = 0;
        int j = 0;
#pragma unroll 4
        for (; j + 1 < nL; j += 2) {
            const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(s_sortk + j);
            rank += (kk.x > key) + (kk.y > key);
        }
        if (j < nL) rank += s_sortk[j] > key;
        const int m = __popcll(__ballot(div));
        // children per rank, their prefix; the first rank whose division makes
        // the list reach N (nL + sum of (children - 1) up to it >= N)
        if (div) s_aux1[rank] = nch;
        wave_sync();
        const int x = lane < m ? s_aux1[lane] : 0;
        const int incl = wave_incl_scan_dpp(x);
        const int ex = incl - x;
        const unsigned long long br = __ballot(lane < m && nL + (ex - lane) + x - 1 >= N);
        const int kstop = br ? (int)__builtin_ctzll(br) : m - 1;
        C = kstop >= 0 ? __builtin_amdgcn_readlane(incl, kstop) : 0;
        if (lane == 0) s_misc[24] = kstop;  // (the debug trace's kstop)
        if (lane < m) s_aux0[lane] = ex;
        wave_sync();
        flag = div && rank <= kstop;
        base = flag ? s_aux0[rank] : 0;
        const unsigned long long bs = __ballot(valid && !flag);
        S = __popcll(bs);
        spos = lanes_below(bs);
        wave_sync();  // (the rank scratch is read before the kept positions overwrite s_aux1)
    }
    const bool bad = C + S > ncap || nseq + C > 0x0FFFFFFF;
    if (lane == 0) {
        s_misc[20] = C;
        s_misc[21] = S;
        s_misc[22] = bad ? (C + S > ncap ? kErrNodeCap : kErrSeqCap) : 0;
    }
    int nexp = 0;  // this node's children with > 1 key
    if (!bad && valid) {
        s_flag[lane] = flag;
        if (flag) {
            int p = base;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = qc.get(lane, q);
                if (c > 0) {
                    const int pos = C - 1 - p;
                    ONode ch = child_rect(nd, q);
                    ch.cnt = c;
                    ch.seq = (uint32_t)(nseq + p);
                    nw[pos] = ch;
                    qc.set(lane, q, pos);
                    nexp += c > 1;
                    ++p;
                }
            }
        } else {
            const int pos = C + spos;
            nw[pos] = nd;
            s_aux1[lane] = pos;
        }
    }
    const int tot_exp = __popcll(__ballot(nexp >= 1)) + __popcll(__ballot(nexp >= 2)) + __popcll(__ballot(nexp >= 3)) +
                        __popcll(__ballot(nexp >= 4));
    if (lane == 0) *s_nexp = tot_exp;
    // the last pass (:673 / :740): the best-key words of the final list, in
    // s_aux0 (its scratch reads are behind, in this wave's order), zeroed here
    // so the remap sweep can take every key's response straight away
    const int nNew = C + S;
    if (!bad && (nNew >= N || nNew == nL))
        for (int i = lane; i < nNew; i += 64) s_aux0[i] = 0;
}

template <int NT, bool LDS>
__device__ void octree_body(const Geom& g, const LevelGeom& L, int l, int f, int nk, int ncells, int ncap, int ncap2,
                            const uint32_t* __restrict__ cand, uint32_t* __restrict__ out,
                            int* __restrict__ oct_count, int* __restrict__ err, int* __restrict__ trace,
                            KeyStore<LDS> ks, QuadCounts<LDS> qc, int* s_misc, ONode* s_node0, ONode* s_node1,
                            int* s_aux0, int* s_aux1, uint8_t* s_flag, int* s_cellofs) {
    const int tid = threadIdx.x;
    int* s_tmp = s_misc;

    const int N = L.nfeat;
    const int nini = L.nini;
    if (nini > ncap) {
        if (tid == 0) { atomicOr(err, kErrNodeCap); oct_count[f * kOcStride + l] = 0; }
        return;
    }

    // 2. roots (:545-587): keys -> root index (int)(x / hX).  The keys are
    // gathered from the FAST cell slots in candidate order: first every cell
    // writes its index over its key range (the node array as a key -> cell
    // map), then each thread loads its keys eight at a time, all eight loads in
    // flight before any is used (measured: the per-key binary search over
    // the cell offsets and one dependent load per key made this phase a
    // quarter of the workgroup's time).
    for (int i = tid; i < nini; i += NT) s_aux0[i] = 0;
    OCT_T(60);
    for (int c = tid; c < ncells; c += NT) {
        const int b = s_cellofs[c], e = s_cellofs[c + 1];
        for (int k = b; k < e; ++k) ks.set_node(k, c);
    }
    __syncthreads();
    OCT_T(61);
    const uint32_t* cbase = cand + (size_t)f * g.cand_frame + L.cand_offset;
    // one root (4:3 and narrower levels): every key's root is 0 and its count
    // nk -- no per-key LDS atomic on one address, no root remap sweep
    const bool one_root = nini == 1;
    constexpr int kGather = 8;
    for (int k0 = tid; k0 < nk; k0 += kGather * NT) {
        uint32_t key[kGather];
#pragma unroll
        for (int u = 0; u < kGather; ++u) {
            const int k = min(k0 + u * NT, nk - 1);
            const int c = ks.node(k);
            key[u] = cbase[(size_t)c * L.cell_cap + (k - s_cellofs[c])];
        }
#pragma unroll
        for (int u = 0; u < kGather; ++u) {
            const int k = k0 + u * NT;
            if (k < nk) {
                ks.set_key(k, key[u]);
                if (one_root) {
                    ks.set_node(k, 0);
                } else {
                    int r = (int)__fdiv_rn((float)key_x(key[u]), L.hx);
                    r = min(r, nini - 1);
                    ks.set_node(k, r);
                    atomicAdd(&s_aux0[r], 1);
                }
            }
        }
    }
    if (one_root && tid == 0) s_aux0[0] = nk;
    __syncthreads();
    OCT_T(1);
    // non-empty roots keep their order; empty ones are erased.  Computed by
    // thread r (no single-lane loop: see tools/check_scc.py for the ROCm 7.2
    // miscompile a uniform-address select in such a loop triggered).
    auto make_root = [&](int r, int c, int pos) {
        ONode nd;
        const int x0 = (int)(L.hx * (float)r), x1 = (int)(L.hx * (float)(r + 1));
        nd.r0 = (uint32_t)x0;
        nd.r1 = (uint32_t)x1 | ((uint32_t)(L.max_by - kBorder) << 16);
        nd.cnt = (uint32_t)c;
        nd.seq = (uint32_t)r;
        s_node0[pos] = nd;
    };
    int nroots;
    if (__builtin_amdgcn_readfirstlane(nini) <= 64) {
        // up to 64 roots (every level of 640x480 .. 1241x376): wave 0 alone
        // (lane = root), positions by ballot -- one block barrier
        if (tid < 64) {
            const int c = tid < nini ? s_aux0[tid] : 0;
            const unsigned long long b = __ballot(c > 0);
            const int pos = lanes_below(b);
            if (c > 0) make_root(tid, c, pos);
            if (tid < nini) s_aux1[tid] = c > 0 ? pos : -1;
            if (tid == 0) s_misc[23] = __popcll(b);
        }
        __syncthreads();
        nroots = s_misc[23];
    } else {
        for (int r = tid; r < nini; r += NT) s_aux1[r] = s_aux0[r] > 0 ? 1 : 0;
        __syncthreads();
        nroots = block_scan<NT>(s_aux1, nini, s_tmp);
        for (int r = tid; r < nini; r += NT) {
            const int c = s_aux0[r];
            const int pos = s_aux1[r];
            if (c > 0) make_root(r, c, pos);
            s_aux1[r] = c > 0 ? pos : -1;
        }
        __syncthreads();
    }
    if (!one_root)  // one root: root 0 is node 0 (when there are keys at all)
        for (int k = tid; k < nk; k += NT) ks.set_node(k, s_aux1[ks.node(k)]);
    __syncthreads();

    OCT_T(2);
    // 3. passes.  The pass state (list size, buffer, phase, next seq) is kept
    // in registers: every thread derives it from the same block-scan totals.
    int nL = nroots, cur = 0, nseq = nini;
    bool inner = false;
    uint32_t* s_best = reinterpret_cast<uint32_t*>(s_aux0);  // (step 4's words, in aux0)
    int best_state = 0;  // 1: zeroed by the last pass, 2: filled by its remap
    for (int guard = 0; guard < 4096; ++guard) {
        ONode* old = cur ? s_node1 : s_node0;
        ONode* nw = cur ? s_node0 : s_node1;
        // the inner pass's sort keys live in the next list's buffer: it is
        // written only after the last sort-key read (ncap2 <= 2 ncap keys fit)
        unsigned long long* s_sortk = reinterpret_cast<unsigned long long*>(nw);
        // quadrant histogram of every node with > 1 key; the counter of
        // children with > 1 key alternates between two slots, so this pass
        // resets its own while the previous pass's may still be read
        int* s_nexp = s_misc + 25 + (guard & 1);
        qc.zero(nL, tid, NT);
        if (tid == 0) *s_nexp = 0;
        __syncthreads();
        if constexpr (kAggHist && NT == kThreads) {
        // (the batch kernel: 256-thread workgroups, round 6 r6d: octree 0.1174 -> 0.1125 ms per
        // 512 frames; the 1024-thread single-frame kernel measured no faster with it)
        // a wave whose keys all sit in one node (the early passes: one root,
        // then its quadrants; keys are in candidate order, so spatially local)
        // adds its four quadrant counts with at most four atomics from one
        // lane instead of one atomic per key on the same two counter words
        for (int k0 = tid & ~63; k0 < nk; k0 += NT) {
            const int lane = tid & 63, k = k0 + lane;
            const bool valid = k < nk;
            const int i = valid ? ks.node(k) : -1;
            const int i0 = __builtin_amdgcn_readfirstlane(i);  // lane 0 is valid whenever the wave runs
            const bool uni = __ballot(valid && i != i0) == 0ull;
            const ONode nd = old[valid ? i : i0];
            const int q = valid && nd.cnt > 1 ? node_quad(nd, ks.key(k)) : -1;
            if (uni) {  // wave-uniform: every lane takes part in the ballots
                const unsigned long long b0 = __ballot(q == 0), b1 = __ballot(q == 1), b2 = __ballot(q == 2),
                                         b3 = __ballot(q == 3);
                if (lane == 0) {
                    if (b0) qc.add(i0, 0, (uint32_t)__popcll(b0));
                    if (b1) qc.add(i0, 1, (uint32_t)__popcll(b1));
                    if (b2) qc.add(i0, 2, (uint32_t)__popcll(b2));
                    if (b3) qc.add(i0, 3, (uint32_t)__popcll(b3));
                }
            } else if (q >= 0) {
                qc.add(i, q);
            }
        }
        } else {
        for (int k = tid; k < nk; k += NT) {
            const int i = ks.node(k);
            const ONode nd = old[i];
            if (nd.cnt > 1) qc.add(i, node_quad(nd, ks.key(k)));
        }
        }
        __syncthreads();
        OCT_T(3 + 4 * guard);
        // processing order and push bases
        int C, S;  // children pushed this pass, surviving nodes
        // (nL is block-uniform; read as a scalar so the branch is a scalar
        // compare: tools/check_scc.py)
        const bool small = __builtin_amdgcn_readfirstlane(nL) <= 64;
        if (small) {
            // a list of at most 64 nodes (every main pass of a 640x480 level
            // and most inner passes): wave 0 alone orders, scans and pushes
            // it, lane = node, with wave scans and ballots -- one block barrier
            // before the remap instead of a scan's and a phase's each
            if (tid < 64) wave_small_pass(old, nw, s_sortk, qc, s_aux0, s_aux1, s_flag, s_misc, s_nexp, nL, N, ncap,
                                          nseq, inner, tid);
            __syncthreads();
            C = s_misc[20];
            S = s_misc[21];
            if (s_misc[22]) {
                if (tid == 0) { atomicOr(err, s_misc[22]); oct_count[f * kOcStride + l] = 0; }
                return;
            }
        } else {
            if (!inner) {
                // one scan of (children << 16 | survives): push bases and survivor
                // positions together (C <= 4 nL and S <= nL stay below 2^16)
                for (int i = tid; i < nL; i += NT) {
                    const bool div = old[i].cnt > 1;
                    const int nch = qc.nonzero(i);
                    s_aux0[i] = div ? nch << 16 : 1;
                    s_flag[i] = div;
                }
                __syncthreads();
                const int tot = block_scan<NT>(s_aux0, nL, s_tmp);
                C = tot >> 16;
                S = tot & 0xFFFF;
            } else {
                // compact the nodes with > 1 key, sort descending by (cnt, seq)
                for (int i = tid; i < nL; i += NT) s_aux1[i] = old[i].cnt > 1;
                __syncthreads();
                const int m = block_scan<NT>(s_aux1, nL, s_tmp);
                const int P = pow2ceil(max(m, 1));
                constexpr int kRankPer = 2;  // up to 2 keys per thread: rank sort, else bitonic
                const bool by_rank = m <= kRankPer * NT;
                for (int i = tid; i < nL; i += NT)
                    if (old[i].cnt > 1)
                        s_sortk[s_aux1[i]] = ((unsigned long long)min(old[i].cnt, 0xFFFFFFu) << 40) |
                                             ((unsigned long long)(old[i].seq & 0xFFFFFFFu) << 12) | (unsigned)i;
                if (!by_rank)
                    for (int i = m + tid; i < P; i += NT) s_sortk[i] = 0ull;
                __syncthreads();
                if (by_rank) {
                    // descending order by rank = the number of larger keys (the keys
                    // are distinct: they end in the node index); every thread reads
                    // the same key per step (LDS broadcast), no barrier per step
                    unsigned long long mine[kRankPer];
                    int rank[kRankPer];
    #pragma unroll
                    for (int u = 0; u < kRankPer; ++u) {
                        mine[u] = s_sortk[min(tid + u * NT, max(m - 1, 0))];
                        rank[u] = 0;
                    }
                    // two keys per 16-byte read, several reads in flight; only the
                    // key slots that exist (the second when m > NT), and a wave
                    // whose threads hold no key skips the loop (wave-uniform)
                    auto rank_keys = [&](auto nu_c) {
                        constexpr int NU = decltype(nu_c)::value;
                        int j = 0;
    #pragma unroll 4
                        for (; j + 1 < m; j += 2) {
                            const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(s_sortk + j);
    #pragma unroll
                            for (int u = 0; u < NU; ++u) rank[u] += (kk.x > mine[u]) + (kk.y > mine[u]);
                        }
                        if (j < m) {
                            const unsigned long long kj = s_sortk[j];
    #pragma unroll
                            for (int u = 0; u < NU; ++u) rank[u] += kj > mine[u];
                        }
                    };
                    if ((tid & ~63) < m) {
                        if (m > NT) rank_keys(std::integral_constant<int, 2>{});
                        else rank_keys(std::integral_constant<int, 1>{});
                    }
                    __syncthreads();
    #pragma unroll
                    for (int u = 0; u < kRankPer; ++u)
                        if (tid + u * NT < m) s_sortk[rank[u]] = mine[u];
                    __syncthreads();
                } else {
                    for (int k = 2; k <= P; k <<= 1)
                        for (int j = k >> 1; j > 0; j >>= 1) {
                            for (int i = tid; i < P; i += NT) {
                                const int ixj = i ^ j;
                                if (ixj > i) {
                                    const unsigned long long a = s_sortk[i], b = s_sortk[ixj];
                                    const bool desc = (i & k) == 0;
                                    if (desc ? (a < b) : (a > b)) { s_sortk[i] = b; s_sortk[ixj] = a; }
                                }
                            }
                            __syncthreads();
                        }
                }
                // rank r -> (nch - 1); inclusive scan; first r reaching N
                for (int r = tid; r < m; r += NT) {
                    const int i = (int)(s_sortk[r] & 0xFFF);
                    s_aux1[r] = qc.nonzero(i) - 1;
                }
                if (tid == 0) s_misc[24] = m - 1;
                __syncthreads();
                block_scan<NT>(s_aux1, m, s_tmp);  // exclusive prefix of (nch-1)
                for (int r = tid; r < m; r += NT) {
                    const int i = (int)(s_sortk[r] & 0xFFF);
                    if (nL + s_aux1[r] + qc.nonzero(i) - 1 >= N) atomicMin(&s_misc[24], r);
                }
                for (int i = tid; i < nL; i += NT) { s_flag[i] = 0; s_aux0[i] = 0; }
                __syncthreads();
                const int kstop = s_misc[24];
                // push bases over ranks 0..kstop, scattered to node index
                for (int r = tid; r < m; r += NT) {
                    const int i = (int)(s_sortk[r] & 0xFFF);
                    s_aux1[r] = r <= kstop ? qc.nonzero(i) : 0;
                }
                __syncthreads();
                C = block_scan<NT>(s_aux1, m, s_tmp);
                for (int r = tid; r <= kstop && r < m; r += NT) {
                    const int i = (int)(s_sortk[r] & 0xFFF);
                    s_aux0[i] = s_aux1[r];
                    s_flag[i] = 1;
                }
                __syncthreads();
            }
            OCT_T(4 + 4 * guard);
            if (inner) {  // survivors keep their order after the C pushed children
                for (int i = tid; i < nL; i += NT) s_aux1[i] = s_flag[i] ? 0 : 1;
                __syncthreads();
                S = block_scan<NT>(s_aux1, nL, s_tmp);
            }
            if (C + S > ncap || nseq + C > 0x0FFFFFFF) {
                if (tid == 0) { atomicOr(err, C + S > ncap ? kErrNodeCap : kErrSeqCap); oct_count[f * kOcStride + l] = 0; }
                return;
            }
            for (int i = tid; i < nL; i += NT) {
                const ONode nd = old[i];
                const int pk = s_aux0[i];  // main pass: packed prefix; inner pass: push base
                if (s_flag[i]) {
                    int p = inner ? pk : pk >> 16;
    #pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t c = qc.get(i, q);
                        if (c > 0) {
                            const int pos = C - 1 - p;
                            ONode ch = child_rect(nd, q);
                            ch.cnt = c;
                            ch.seq = (uint32_t)(nseq + p);
                            nw[pos] = ch;
                            qc.set(i, q, pos);
                            if (c > 1) atomicAdd(s_nexp, 1);
                            ++p;
                        }
                    }
                } else {
                    const int pos = C + (inner ? s_aux1[i] : (pk & 0xFFFF));
                    nw[pos] = nd;
                    s_aux1[i] = pos;
                }
            }
            __syncthreads();
        }
        const int nNew = C + S;
        const bool done = nNew >= N || nNew == nL;  // :673 / :740
        OCT_T(5 + 4 * guard);
        if (done && small) {
            // the last pass after the wave path: the best-key words are zeroed,
            // so each key's response goes to its final node in the remap sweep
            for (int k = tid; k < nk; k += NT) {
                const int i = ks.node(k);
                const uint32_t key = ks.key(k);
                const int ni = s_flag[i] ? (int)qc.get(i, node_quad(old[i], key)) : s_aux1[i];
                ks.set_node(k, ni);
                atomicMax(&s_best[ni], ((uint32_t)key_s(key) << 24) | (0xFFFFFFu - (uint32_t)k));
            }
            best_state = 2;
        } else {
            for (int k = tid; k < nk; k += NT) {
                const int i = ks.node(k);
                ks.set_node(k, s_flag[i] ? (int)qc.get(i, node_quad(old[i], ks.key(k))) : s_aux1[i]);
            }
            if (done) {  // (s_aux0 is not read by the remap)
                for (int i = tid; i < nNew; i += NT) s_best[i] = 0;
                best_state = 1;
            }
        }
        __syncthreads();
        OCT_T(6 + 4 * guard);
        if (tid == 0 && trace && f == 0 && guard < 47) {  // below the stamp region (ints 384..)
            int* t = trace + l * 512 + 2 + guard * 8;
            t[0] = inner; t[1] = nL; t[2] = C; t[3] = S; t[4] = *s_nexp; t[5] = s_misc[24]; t[6] = nk; t[7] = N;
            trace[l * 512] = guard + 1;
        }
        const int nexp = *s_nexp;  // children with > 1 key (nToExpand)
        if (!inner && nNew + nexp * 3 > N) inner = true;  // :678
        nseq += C;
        cur ^= 1;
        nL = nNew;
        // no barrier here: the next pass first writes s_qc (last read by the
        // remap above, before its barrier) and the other nexp slot
        if (done) break;
    }

    // 4. best key per node (max response, first in candidate order); usually
    // zeroed (best_state 1) or filled (2) by the last pass already
    if (best_state == 0) {
        for (int i = tid; i < nL; i += NT) s_best[i] = 0;
        __syncthreads();
    }
    if (best_state < 2) {
        for (int k = tid; k < nk; k += NT)
            atomicMax(&s_best[ks.node(k)], ((uint32_t)key_s(ks.key(k)) << 24) | (0xFFFFFFu - (uint32_t)k));
        __syncthreads();
    }
    if (nL > L.ocap) {
        if (tid == 0) { atomicOr(err, kErrNodeCap); oct_count[f * kOcStride + l] = 0; }
        return;
    }
    for (int i = tid; i < nL; i += NT) out[i] = ks.key((int)(0xFFFFFFu - (s_best[i] & 0xFFFFFFu)));
    if (tid == 0) oct_count[f * kOcStride + l] = nL;
    OCT_T(63);
}

template <int NT>
__global__ __launch_bounds__(NT) void octree_kernel(Geom g, const uint32_t* __restrict__ cand,
                                                          const int* __restrict__ cell_counts,
                                                          uint32_t* __restrict__ gkeys,
                                                          uint16_t* __restrict__ gknode,
                                                          uint32_t* __restrict__ oct_out,
                                                          int* __restrict__ oct_count, int* __restrict__ err,
                                                          int* __restrict__ trace, OctreeGroup A, OctreeGroup B,
                                                          int batch) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // linear block index: group A's (frame, level) blocks first, then group B's, so B's
    // short workgroups fill the slots of A's finished ones inside one launch
    const int id = (int)blockIdx.x, na = A.nlev * batch;
    const bool inA = id < na;
    const OctreeGroup& G = inA ? A : B;
    const int j = inA ? id : id - na;
    const int f = j / G.nlev, l = G.level0 + (j - f * G.nlev);
    const int kcap = G.kcap, ncap = G.ncap;
    const int tid = threadIdx.x;
    const LevelGeom& L = g.lv[l];
    const int ncells = L.ncols * L.nrows;
    const int ncap2 = pow2ceil(ncap);
    OCT_T(0);

    // LDS carve (byte offsets must match octree_lds_bytes).  ncap is a
    // multiple of 16, so every region below starts 16-byte aligned.  Regions
    // shared by phases that never overlap: the cell offsets (roots phase
    // only) sit in node buffer 1, the inner pass's sort keys in the next
    // list's node buffer, the final best-key words in aux0, and the HBM-path
    // quadrant counters in the key region.
    const size_t o_node0 = 128;
    const size_t o_node1 = o_node0 + (size_t)ncap * 16;
    const size_t o_qc = o_node1 + std::max((size_t)ncap * 16, (((size_t)(g.max_cells_level + 1) * 4 + 15) & ~(size_t)15));
    const size_t o_aux0 = o_qc + (size_t)ncap * 8;
    const size_t o_aux1 = o_aux0 + (size_t)ncap * 4;
    const size_t o_flag = o_aux1 + (size_t)ncap * 4;
    const size_t o_keys = o_flag + (size_t)ncap;
    const size_t o_knode = o_keys + (size_t)kcap * 4;
    int* s_misc = reinterpret_cast<int*>(smem);
    ONode* s_node0 = reinterpret_cast<ONode*>(smem + o_node0);
    ONode* s_node1 = reinterpret_cast<ONode*>(smem + o_node1);
    int* s_aux0 = reinterpret_cast<int*>(smem + o_aux0);
    int* s_aux1 = reinterpret_cast<int*>(smem + o_aux1);
    uint8_t* s_flag = smem + o_flag;
    int* s_cellofs = reinterpret_cast<int*>(smem + o_node1);
    int* s_tmp = s_misc;  // [0..15] scan scratch (a wave total each), [24..25] scalars

    // 1. candidate order: cells row-major, within a cell FAST order (:797-838)
    const int* cc = cell_counts + (size_t)f * g.total_cells + L.cell_base;
    for (int i = tid; i < ncells; i += NT) s_cellofs[i] = cc[i];
    if (tid == 0) s_cellofs[ncells] = 0;
    __syncthreads();
    const int nk = block_scan<NT>(s_cellofs, ncells + 1, s_tmp);
    uint32_t* out = oct_out + (size_t)f * g.slots_frame + L.out_offset;
    if (nk <= kcap) {
        KeyStore<true> ks{reinterpret_cast<uint32_t*>(smem + o_keys), reinterpret_cast<uint16_t*>(smem + o_knode)};
        QuadCounts<true> qc{reinterpret_cast<uint16_t*>(smem + o_qc)};
        octree_body<NT, true>(g, L, l, f, nk, ncells, ncap, ncap2, cand, out, oct_count, err, trace, ks, qc, s_misc,
                              s_node0, s_node1, s_aux0, s_aux1, s_flag, s_cellofs);
    } else {  // too many candidates for LDS: the same algorithm on an HBM scratch region
        KeyStore<false> ks{gkeys + (size_t)f * g.cand_frame + L.cand_offset,
                           gknode + (size_t)f * g.cand_frame + L.cand_offset};
        QuadCounts<false> qc{reinterpret_cast<uint32_t*>(smem + o_keys)};
        octree_body<NT, false>(g, L, l, f, nk, ncells, ncap, ncap2, cand, out, oct_count, err, trace, ks, qc, s_misc,
                               s_node0, s_node1, s_aux0, s_aux1, s_flag, s_cellofs);
    }
}

}  // namespace

size_t octree_lds_bytes(const Geom& g, int kcap, int ncap) {
    // misc, node 0, node 1 (or the cell offsets), u16 quadrant counters,
    // aux0, aux1, flags, keys + key nodes (or u32 quadrant counters); ncap
    // is a multiple of 16 and kcap of 64 (see the kernel's carve)
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t n = (size_t)ncap;
    return r16(32 * 4) + r16(n * 16) + std::max(r16(n * 16), r16((size_t)(g.max_cells_level + 1) * 4)) +
           r16(n * 8) + 2 * r16(n * 4) + r16(n) +
           std::max(r16((size_t)kcap * 4) + r16((size_t)kcap * 2), r16(n * 16));
}

hipError_t launch_octree(const Geom& g, int batch, const uint32_t* cand, const int* cell_counts,
                         uint32_t* gkeys, uint16_t* gknode, uint32_t* oct_out, int* oct_count,
                         int* err, const OctreeGroup* groups, int ngroups, int* trace, hipStream_t stream) {
    // both level groups in one launch, LDS sized for the larger group: group B's short
    // workgroups start as group A's finish instead of after the last of them (two
    // launches: 0.278 ms per 512 frames, one: 0.184 ms)
    // a few frames leave most CUs idle: then every (frame, level) workgroup
    // gets 1024 threads, so its key sweeps, scans and sorts take a quarter of the steps
    const bool small = batch <= kSmallBatch;
    auto kernel = small ? &octree_kernel<kThreadsSmall> : &octree_kernel<kThreads>;
    const int nt = small ? kThreadsSmall : kThreads;
    if (ngroups == 2 && groups[0].nlev > 0 && groups[1].nlev > 0) {
        const size_t lds = std::max(octree_lds_bytes(g, groups[0].kcap, groups[0].ncap),
                                    octree_lds_bytes(g, groups[1].kcap, groups[1].ncap));
        hipLaunchKernelGGL(kernel, dim3((groups[0].nlev + groups[1].nlev) * batch), dim3(nt), lds,
                           stream, g, cand, cell_counts, gkeys, gknode, oct_out, oct_count, err, trace, groups[0],
                           groups[1], batch);
        return hipGetLastError();
    }
    // one launch per level group: the LDS (and so the workgroups per CU) sized for the group's levels
    for (int i = 0; i < ngroups; ++i) {
        const OctreeGroup& G = groups[i];
        if (G.nlev <= 0) continue;
        const size_t lds = octree_lds_bytes(g, G.kcap, G.ncap);
        hipLaunchKernelGGL(kernel, dim3(G.nlev * batch), dim3(nt), lds, stream, g, cand, cell_counts,
                           gkeys, gknode, oct_out, oct_count, err, trace, G, OctreeGroup{0, 0, 0, 0}, batch);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace orbgpu
