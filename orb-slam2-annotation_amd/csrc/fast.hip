// fast.hip -- the FAST part of ORBextractor::ComputeKeyPointsOctTree
// (ORBextractor.cpp:776-838): per 30-px cell window, cv::FAST(window, 20,
// nonmax=true), and if that finds nothing cv::FAST(window, 7, true).
//
// One wave per cell window (<= 72x72 px staged in LDS).  The FAST arc
// strength s (cornerScore + 1) is computed once per pixel; "corner at
// threshold t" is exactly s >= t+1 (a 9-arc with all |d| > t exists iff the
// best arc's min |d| >= t+1), so both threshold passes reuse one score tile.
// NMS is the cv::FAST 3x3 strict-> test among corners of the SAME window
// (non-corners and pixels outside the window's detection region count 0),
// and keypoints are emitted row-major through ballot/mbcnt compaction, which
// reproduces cv::FAST's emission order.  Output: packed (x, y, score) keys
// relative to (minBorderX, minBorderY), in the cell's fixed slot range.
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

#include <cstdlib>
#include <type_traits>

namespace orbgpu {

namespace {

#ifndef ORBGPU_FAST_BANDS
#define ORBGPU_FAST_BANDS 1
#endif
// survivor-list entries per cell wave: every pixel of a cell, or with
// ORBGPU_FAST_BANDS a list that keeps the wave's LDS within 4,864 B (32 waves
// per CU; at least 256 entries)
__host__ __device__ constexpr int fast_list_len(int P, int R, int det_max) {
    const int c = ((4864 - 2 * P * R - 16) / 2 - 1) & ~7;
    return !ORBGPU_FAST_BANDS || c >= det_max ? det_max : (c >= 256 ? c : det_max);
}

// a wave-uniform pointer held in scalar registers (loads then take the
// saddr + 32-bit vector offset form: no 64-bit vector address arithmetic)
__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (const uint8_t*)(((uint64_t)hi << 32) | lo);
}

// Window staging geometry (fast_cells_kernel): chunks of CB bytes, NC per
// P-byte row, RPI rows per pass of 64 lanes, kGroup passes' loads in flight.
template <int P>
struct FastStage {
    static constexpr int CB = P % 16 == 0 ? 16 : 4, NC = P / CB, RPI = 64 / NC, kGroup = CB == 16 ? 2 : 4;
};
// LDS rows the staging writes for windows of up to R rows (at most): its
// passes plus the row the lanes past RPI * NC stage; they must fit in the
// window and the score tile behind it, 2R rows
template <int P>
constexpr int fast_stage_rows(int R) {
    using S = FastStage<P>;
    return S::RPI * ((R + S::RPI - 1) / S::RPI + 1);
}

// The waves of a block work on different cells (their own LDS regions), so
// stages are ordered within the wave, never with a block barrier.  A wave's DS
// instructions execute in order, so its LDS writes are seen by its later LDS
// reads: only the compiler must keep memory operations on their side of this
// point (the asm's memory clobber), plus a wait for the wave's own LDS
// operations.  No VMEM wait: a workgroup-scope fence here waited for every
// outstanding global access (vmcnt(0)), stores included.
__device__ inline void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// a where this lane's bit of the mask m (scalar registers) is set, else b:
// one v_cndmask on the mask as it is (a bool built from it would be turned
// back into a vector value and compared again)
__device__ __forceinline__ int lane_select(unsigned long long m, int a, int b) {
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

struct CellTiles {
    const uint8_t* win;  // staged window, pitch P, column c <-> level x = xa + c
    uint8_t* sc;         // FAST arc strength of corners, 0 elsewhere
    uint16_t* la;        // tile offsets passing the compass pre-test
    uint16_t* lb;        // tile offsets of corners (row-major order); the same buffer as la: the
                         // corner list is compacted in place behind the survivors being read
    int dump;            // list index past the longest list: the compass's non-survivor lanes store there
};

// Compass pre-test, row-major over the detection region: LPR = 32 lanes
// per row when it fits (two rows per pass), else 64 (dw <= 64: host check).
// Two passes per iteration, evaluated together: the lane's two pixels (rows
// r and r + 64 / LPR of one column) are the two halves of packed u16 values,
// so every min/max/subtract below is one packed op for both (rows past the
// region read the rest of the wave's LDS area and are masked).
//   two adjacent compass points both darker than v - t <=> the smallest
//   pairwise max is; both brighter than v + t <=> the largest pairwise min
//   is; dark < v - t <=> sat(v - dark) > t, bright > v + t <=> sat(bright - v) > t
// Returns the number of survivors, listed (tile offsets, row-major) in T.la.
template <int P, int LPR, bool kBand = false>
__device__ int compass_pass(const CellTiles& T, int dw, int dh, int ox, int t, int lane, int row0 = 0, int start = 0,
                            int* row_end = nullptr) {
    constexpr int kStep = 64 / LPR;  // rows between a lane's two pixels
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto compass2 = [&](const uint8_t* p) -> uint32_t {
        auto ld = [&](int o) {
            u16x2 r;
            r.x = p[o];
            r.y = p[kStep * P + o];
            return r;
        };
        // Every pair of adjacent compass points is one of {c0, c8} with one of
        // {c4, c12} (a 4-cycle), so the smallest pairwise max is
        // max(min(c0, c8), min(c4, c12)) and the largest pairwise min is
        // min(max(c0, c8), max(c4, c12)): three ops each
        const u16x2 v = ld(0), c0 = ld(3 * P), c4 = ld(3), c8 = ld(-3 * P), c12 = ld(-3);
        const u16x2 dark = __builtin_elementwise_max(__builtin_elementwise_min(c0, c8), __builtin_elementwise_min(c4, c12));
        const u16x2 bright =
            __builtin_elementwise_min(__builtin_elementwise_max(c0, c8), __builtin_elementwise_max(c4, c12));
        const u16x2 x = __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, dark),
                                                  __builtin_elementwise_sub_sat(bright, v));
        const u16x2 tt = {(unsigned short)t, (unsigned short)t};
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(x, tt));  // a half nonzero <=> its pixel passes
    };
    auto below = [](unsigned long long m) {  // set bits of m in lanes below this one
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };
    // Lane masks are formed in scalar registers: the compass results by
    // v_cmp straight into a mask, the column and row ranges as wave-uniform
    // masks (rows r + rsub are in range for every lane while 2+ rows remain,
    // only the rsub = 0 half on the last row).  Every lane stores: a survivor
    // at its compacted position, the others into the dump slot past the list.
    const int rsub = LPR == 32 ? lane >> 5 : 0, col = lane & (LPR - 1);
    const unsigned long long colmask = __builtin_amdgcn_uicmp((uint32_t)col, (uint32_t)dw, 36 /* ult */);
    constexpr unsigned long long sub0 = LPR == 32 ? 0xFFFFFFFFull : ~0ull;  // lanes of row rsub = 0
    int o = (3 + rsub + row0) * P + 3 + ox + col;  // tile offset of the lane's first pixel
    int na = start;
    int rr = row0;
    for (; rr < dh; rr += 2 * kStep, o += 2 * kStep * P) {
        if (kBand && na + 128 > T.dump) break;  // a pass adds at most 128 entries: the band ends here
        const uint32_t y = compass2(T.win + o);
        const int rem = dh - rr;  // rows left, >= 1
        const unsigned long long rows0 = rem >= 2 ? ~0ull : sub0;
        const unsigned long long rows1 = rem > kStep + 1 ? ~0ull : (rem > kStep ? sub0 : 0ull);
        const unsigned long long m0 = __builtin_amdgcn_uicmp(y & 0xFFFFu, 0u, 33 /* ne */) & colmask & rows0;
        const unsigned long long m1 = __builtin_amdgcn_uicmp(y, 0x10000u, 35 /* uge */) & colmask & rows1;
        T.la[na + lane_select(m0, below(m0), T.dump - na)] = (uint16_t)o;
        na += __popcll(m0);
        T.la[na + lane_select(m1, below(m1), T.dump - na)] = (uint16_t)(o + kStep * P);
        na += __popcll(m1);
    }
    if (kBand) *row_end = rr;
    return na;
}

// The same compass pre-test on dword groups (ORBGPU_FAST_COMPASS_DW): a lane
// takes 4 adjacent pixels of a row -- the 4-aligned tile columns 4g .. 4g+3
// of the detection region's NG groups, RPI = 64 / NG rows per iteration, lanes
// row-major over (row, group) -- and reads its centre, c0 and c8 as one dword
// each and c4 / c12 from the dwords either side (v_alignbyte): 5 LDS reads per
// 4 pixels instead of 10 byte reads per 2.  Each dword splits into two packed
// u16 pairs (v_perm), so the test is the packed arithmetic above on bytes
// (0, 1) and (2, 3).  Survivors are listed row-major: a pixel's position is
// the survivors of the lanes below it (mbcnt over the four byte masks) plus
// those of the lower bytes of its own lane.  Pixels of a group outside the
// detection columns, and rows past the region, are masked.
__constant__ uint32_t c_ng_magic[18] = {0,     65536, 32769, 21846, 16385, 13108, 10923, 9363, 8193,
                                        7282,  6554,  5958,  5462,  5042,  4682,  4370,  4097, 3856};
// 64 / ng (a scalar load: the division took a VALU reciprocal sequence per pass)
__constant__ int c_ng_rpi[18] = {0, 64, 32, 21, 16, 12, 10, 9, 8, 7, 6, 5, 5, 4, 4, 4, 4, 3};
template <int P, bool kBand = false>
__device__ int compass_pass_dw(const CellTiles& T, int dw, int dh, int ox, int t, int lane, int row0 = 0,
                               int start = 0, int* row_end = nullptr) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const int c_lo = 3 + ox, c_hi = 3 + ox + dw;  // detection columns [c_lo, c_hi) of the tile
    const int g_lo = c_lo >> 2, ng = ((c_hi - 1) >> 2) - g_lo + 1;  // <= 17 (dw <= 64)
    const int rpi = c_ng_rpi[ng];                                     // 64 / ng, wave-uniform (scalar)
    const uint32_t magic = c_ng_magic[ng];
    const int rl = (int)(__umul24((uint32_t)lane, magic) >> 16), g = lane - rl * ng;  // lane / ng, lane % ng
    const int col0 = 4 * (g_lo + g);
    // per-byte column masks (lanes of the rpi rows whose byte b is a detection column)
    unsigned long long cm[4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
        cm[b] = __builtin_amdgcn_uicmp((uint32_t)(col0 + b - c_lo), (uint32_t)dw, 36 /* ult */) &
                __builtin_amdgcn_uicmp((uint32_t)rl, (uint32_t)rpi, 36);
    auto split = [](uint32_t x, bool hi) {  // bytes (0, 1) or (2, 3) of x as a packed u16 pair
        return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, x, hi ? 0x0C030C02u : 0x0C010C00u));
    };
    // the compass strength of both pixels (packed u16): a pixel passes iff its
    // half exceeds t (compared per half below: no packed subtract of t)
    auto test = [&](u16x2 v, u16x2 c0, u16x2 c4, u16x2 c8, u16x2 c12) -> u16x2 {
        const u16x2 dark = __builtin_elementwise_max(__builtin_elementwise_min(c0, c8), __builtin_elementwise_min(c4, c12));
        const u16x2 bright =
            __builtin_elementwise_min(__builtin_elementwise_max(c0, c8), __builtin_elementwise_max(c4, c12));
        return __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, dark), __builtin_elementwise_sub_sat(bright, v));
    };
    // c4 (pixel + 3) and c12 (pixel - 3) as packed pairs straight from the
    // neighbouring dwords by one v_perm each (no v_alignbyte first):
    // c4 = (V3, Vp0 | Vp1, Vp2), c12 = (Vm1, Vm2 | Vm3, V0)
    auto pick = [](uint32_t hi, uint32_t lo, uint32_t sel) {
        return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi, lo, sel));
    };
    const uint32_t tq = (uint32_t)t;
    auto addc = [](int a, unsigned long long m) {  // a + (this lane's bit of m)
        int r;
        unsigned long long co;
        asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(a), "s"(m));
        return r;
    };
    int o = (3 + row0 + rl) * P + col0;  // tile offset of the lane's byte 0
    int na = start;
    int rr = row0;
    const int per_iter = dw * rpi;  // most entries one iteration can add
    for (; rr < dh; rr += rpi, o += rpi * P) {
        if (kBand && na + per_iter > T.dump) break;  // the band ends here
        const uint8_t* p = T.win + o;
        const uint32_t V = *reinterpret_cast<const uint32_t*>(p), Vm = *reinterpret_cast<const uint32_t*>(p - 4),
                       Vp = *reinterpret_cast<const uint32_t*>(p + 4), D = *reinterpret_cast<const uint32_t*>(p + 3 * P),
                       U = *reinterpret_cast<const uint32_t*>(p - 3 * P);
        const u16x2 ylo = test(split(V, false), split(D, false), pick(Vp, V, 0x0C040C03u), split(U, false),
                               pick(V, Vm, 0x0C020C01u));
        const u16x2 yhi = test(split(V, true), split(D, true), pick(Vp, V, 0x0C060C05u), split(U, true),
                               pick(V, Vm, 0x0C040C03u));
        // rows past the region: only the last pass has any (cm[] already drops
        // the lanes past rpi rows), so the per-lane row compare runs there alone
        unsigned long long rows = ~0ull;
        if (dh - rr < rpi) rows = __builtin_amdgcn_uicmp((uint32_t)rl, (uint32_t)(dh - rr), 36 /* ult */);
        const unsigned long long m0 = __builtin_amdgcn_uicmp((uint32_t)ylo.x, tq, 34 /* ugt */) & cm[0] & rows;
        const unsigned long long m1 = __builtin_amdgcn_uicmp((uint32_t)ylo.y, tq, 34 /* ugt */) & cm[1] & rows;
        const unsigned long long m2 = __builtin_amdgcn_uicmp((uint32_t)yhi.x, tq, 34 /* ugt */) & cm[2] & rows;
        const unsigned long long m3 = __builtin_amdgcn_uicmp((uint32_t)yhi.y, tq, 34 /* ugt */) & cm[3] & rows;
        uint32_t s = 0u;
        s = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, s));
        s = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, s));
        s = __builtin_amdgcn_mbcnt_hi((uint32_t)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m2, s));
        s = __builtin_amdgcn_mbcnt_hi((uint32_t)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m3, s));
        const int p0 = na + (int)s, p1 = addc(p0, m0), p2 = addc(p1, m1), p3 = addc(p2, m2);
        T.la[lane_select(m0, p0, T.dump)] = (uint16_t)o;
        T.la[lane_select(m1, p1, T.dump)] = (uint16_t)(o + 1);
        T.la[lane_select(m2, p2, T.dump)] = (uint16_t)(o + 2);
        T.la[lane_select(m3, p3, T.dump)] = (uint16_t)(o + 3);
        na += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    }
    if (kBand) *row_end = rr;
    return na;
}
#ifndef ORBGPU_FAST_COMPASS_DW
#define ORBGPU_FAST_COMPASS_DW 1
#endif

// The 16 ring bytes and the centre of two survivors (top-left corners of
// their 7x7 neighbourhoods p0, p1) as packed pairs: survivor 0 in the low
// 16-bit half, survivor 1 in the high half (f16 denormal bit patterns).  One
// byte read per point: unaligned wide LDS reads (one dword for rows 0 and 6,
// 8 bytes for rows 1..5: 7 reads per survivor instead of 17) were correct on
// gfx950 but ran fast_cells in 1.485 ms instead of 0.500 (round 5, r5l).
typedef _Float16 fast_h2 __attribute__((ext_vector_type(2)));
template <int P>
__device__ __forceinline__ uint32_t ring_pairs(const uint8_t* p0, const uint8_t* p1, fast_h2 (&r)[16]) {
    // (each pair by one v_lshl_or: ds_read_u8_d16 / _d16_hi would assemble it in
    // the LDS unit, but with SRAM ECC enabled -- MI355X -- a D16 load zeroes the
    // other half instead of preserving it; round 6 measured the wrong results)
    const int ring_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int ring_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    auto pair = [&](int o) { return (uint32_t)p0[o] | ((uint32_t)p1[o] << 16); };
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = __builtin_bit_cast(fast_h2, pair((ring_dy[k] + 3) * P + ring_dx[k] + 3));
    return pair(3 * P + 3);
}

// One chunk of the arc pass: list entries base + lane and base + 64 + lane
// (one per 16-bit half) -> arc strength, corners at t appended to T.lb after
// nb (list order: the low halves' corners, then the high halves'), their
// scores into the score tile.  With d = v - ring, the arc strength max over
// arcs of max(min d, -max d) is
//   s = max(v - min_k max9_k(ring), max_k min9_k(ring) - v)
// (max9_k / min9_k over the 9-arc starting at ring position k); corner at
// t <=> s >= t + 1.  The ring bytes of both pixels sit in the two halves
// of a register as f16 denormals (order-preserving bit patterns; the
// kernel keeps f16 denormals, and minimum/maximum only select), so every
// 3-way min/max is one v_pk_minimum3_f16 / v_pk_maximum3_f16: a 9-arc is
// three 3-runs.  The corner appends take the lane masks as they are (one
// mbcnt pair each, exec-masked stores; a bool re-materialised into vcc and
// counted with masked popcounts cost 7 VALU per append).
template <int P>
__device__ __forceinline__ int arc_chunk(const CellTiles& T, int na, int base, int t, int lane, int nb) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    typedef short i16x2 __attribute__((ext_vector_type(2)));
    auto max3 = [](h2 x, h2 y, h2 z) { return __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z); };
    auto min3 = [](h2 x, h2 y, h2 z) { return __builtin_elementwise_minimum(__builtin_elementwise_minimum(x, y), z); };
    const int j0 = base + lane, j1 = j0 + 64;
    const int off0 = T.la[min(j0, na - 1)], off1 = T.la[min(j1, na - 1)];  // clamped: real pixels
    // ring reads from the circle's top-left corner: every read is the base
    // register plus a non-negative immediate
    // (one scalar base: the window's LDS offset less the circle's 3P+3 bias)
    const uint8_t* winb = T.win - (3 * P + 3);
    h2 r[16];
    const uint32_t vv = ring_pairs<P>(winb + off0, winb + off1, r);
    h2 hi3[16], lo3[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        hi3[k] = max3(r[k], r[(k + 1) & 15], r[(k + 2) & 15]);
        lo3[k] = min3(r[k], r[(k + 1) & 15], r[(k + 2) & 15]);
    }
    h2 hi9[16], lo9[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        hi9[k] = max3(hi3[k], hi3[(k + 3) & 15], hi3[(k + 6) & 15]);
        lo9[k] = min3(lo3[k], lo3[(k + 3) & 15], lo3[(k + 6) & 15]);
    }
    h2 A = min3(hi9[0], hi9[1], hi9[2]), B = max3(lo9[0], lo9[1], lo9[2]);
#pragma unroll
    for (int k = 3; k < 16; k += 2) {
        A = k + 1 < 16 ? min3(A, hi9[k], hi9[k + 1]) : __builtin_elementwise_minimum(A, hi9[k]);
        B = k + 1 < 16 ? max3(B, lo9[k], lo9[k + 1]) : __builtin_elementwise_maximum(B, lo9[k]);
    }
    const i16x2 v = __builtin_bit_cast(i16x2, vv), ia = __builtin_bit_cast(i16x2, A), ib = __builtin_bit_cast(i16x2, B);
    const i16x2 sc = __builtin_elementwise_max(v - ia, ib - v);  // arc strength (cornerScore + 1)
    const bool c0 = (j0 < na) & (sc.x > t), c1 = (j1 < na) & (sc.y > t);
    const unsigned long long m0 = __ballot(c0), m1 = __ballot(c1);
    auto below = [](unsigned long long m) {  // set bits of m in lanes below this one
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };
    const int p0 = nb + below(m0), nb1 = nb + __popcll(m0), p1 = nb1 + below(m1);
    if (c0) {
        T.sc[off0] = (uint8_t)sc.x;
        T.lb[p0] = (uint16_t)off0;
    }
    if (c1) {
        T.sc[off1] = (uint8_t)sc.y;
        T.lb[p1] = (uint16_t)off1;
    }
    return nb1 + __popcll(m1);
}

// FAST at threshold t on the cell's detection region: returns the number
// of corners, their tile offsets in lb[] (row-major) and scores in sc[].
// Stages are separated by wave compaction so each runs on dense lanes:
// compass pre-test on every pixel -> arc strength of the survivors, two per
// lane in packed 16-bit arithmetic (the corner test is s >= t + 1).
template <int P>
__device__ int fast_corners(const CellTiles& T, int dw, int dh, int ox, int t, int lane,
                            unsigned long long* stamp = nullptr) {
    const int na = ORBGPU_FAST_COMPASS_DW ? compass_pass_dw<P>(T, dw, dh, ox, t, lane)
                   : dw > 32              ? compass_pass<P, 64>(T, dw, dh, ox, t, lane)
                                          : compass_pass<P, 32>(T, dw, dh, ox, t, lane);
    wave_sync();
#ifdef FAST_STAMPS
    if (stamp) {
        stamp[0] = __builtin_amdgcn_s_memtime();
        stamp[1] = (unsigned long long)na;
    }
#endif
    // survivors -> corners, two per lane (arc_chunk), compacted in place
    // behind the survivors being read
    int nb = 0;
    for (int base = 0; base < na; base += 128) nb = arc_chunk<P>(T, na, base, t, lane, nb);
    wave_sync();
    return nb;
}

// 3x3 strict NMS among the corners (cv::FAST: non-corners and pixels outside
// the detection region count 0), emitted in lb order = row-major.
template <int P>
__device__ int nms_emit(const CellTiles& T, int nb, int ox, int t, int lane, int iniX, int iniY,
                        uint32_t* out, int cap, int* err, int jbeg = 0, int total = 0) {
    for (int base = jbeg; base < nb; base += 64) {
        const int j = base + lane;
        bool keep = false;
        int s = 0, off = 0;
        if (j < nb) {
            off = T.lb[j];
            int a = off - (P + 1);  // the 3x3 block's top-left: non-negative read offsets
            asm volatile("" : "+v"(a));
            const uint8_t* q = T.sc + a;
            s = q[P + 1];
            // all eight neighbours loaded without short-circuit branches (one
            // basic block: the loads issue together).  The tile holds 0 or a
            // score >= t + 1 (this pass's corners only), so cv::FAST's neighbour
            // term (v >= t + 1 ? v - 1 : 0) is max(v - 1, 0), and
            // s - 1 > max over the neighbours  <=>  s > max(vmax, 1)
            int v[8];
            int k = 0;
#pragma unroll
            for (int dy = 0; dy <= 2; ++dy)
#pragma unroll
                for (int dx = 0; dx <= 2; ++dx)
                    if (dx != 1 || dy != 1) v[k++] = q[dy * P + dx];
            const int vmax = max(max(max(max(v[0], v[1]), max(v[2], v[3])), max(max(v[4], v[5]), max(v[6], v[7]))), 1);
            keep = s > vmax;
        }
        const unsigned long long m = __ballot(keep);
        if (keep) {
            const int pos = total + __popcll(m & ((1ull << lane) - 1ull));
            const int r = off / P, c = off - r * P;
            if (pos < cap)
                out[pos] = pack_key(iniX + c - ox - kBorder, iniY + r - kBorder, s - 1);
            else
                atomicOr(err, kErrCellCap);
        }
        total += __popcll(m);
    }
    return total;
}

// FAST + NMS of one cell with a survivor list shorter than the detection
// region (ORBGPU_FAST_BANDS: less LDS per wave, more waves per CU).  The
// compass runs in row bands that fit the list after the pending corners;
// each band's survivors go through the arc pass (corners compacted behind the
// pending ones); when rows remain, the corners whose 3x3 neighbourhood is
// complete (region rows < row - 1) are emitted -- they lead the row-major
// list, so the emission order is cv::FAST's -- and the others move to the
// front.  Returns the keypoints emitted; *pending = corners left in the
// list, *dropped = whether emitted corners left the list (their scores stay
// in the tile).
template <int P>
__device__ int fast_cell_banded(const CellTiles& T, int dw, int dh, int ox, int t, int lane, int iniX, int iniY,
                                uint32_t* out, int cap, int* err, int* pending, bool* dropped) {
    int nb = 0, total = 0, row = 0;
    bool drop = false;
    while (true) {
        int row_end = dh;
        const int na = ORBGPU_FAST_COMPASS_DW ? compass_pass_dw<P, true>(T, dw, dh, ox, t, lane, row, nb, &row_end)
                       : dw > 32              ? compass_pass<P, 64, true>(T, dw, dh, ox, t, lane, row, nb, &row_end)
                                              : compass_pass<P, 32, true>(T, dw, dh, ox, t, lane, row, nb, &row_end);
        wave_sync();
        int nc = nb;
        for (int base = nb; base < na; base += 128) nc = arc_chunk<P>(T, na, base, t, lane, nc);
        wave_sync();
        nb = nc;
        row = row_end;
        // corners to emit now: all of them at the end, else those above row - 1
        int k = nb;
        if (row < dh) {
            const int lim = (3 + row - 1) * P;  // tile offsets of region rows < row - 1
            k = 0;
            for (int base = 0; base < nb; base += 64) {
                const int j = base + lane;
                k += __popcll(__ballot(j < nb && (int)T.lb[j] < lim));
            }
        }
        total = nms_emit<P>(T, k, ox, t, lane, iniX, iniY, out, cap, err, 0, total);
        if (row >= dh) break;
        if (k > 0) {  // the rest to the front (each chunk read before its writes; later chunks read above)
            for (int base = 0; base < nb - k; base += 64) {
                const int j = base + lane;
                const uint16_t e = j < nb - k ? T.lb[k + j] : 0;
                if (j < nb - k) T.lb[j] = e;
            }
            nb -= k;
            drop = true;
            wave_sync();
        }
    }
    *pending = nb;
    *dropped = drop;
    return total;
}

// Diagnostic build (-DFAST_STAMPS): every 16th cell's wave adds its phase
// durations (s_memtime cycles) to g_fast_stamps[phase] and its survivor /
// corner counts to [8] / [9]; [15] counts the sampled waves
// (tools/extract_stamps.py).
#ifdef FAST_STAMPS
__device__ unsigned long long g_fast_stamps[16];
#define FSTAMP(k) (stamp_on ? (ts[k] = __builtin_amdgcn_s_memtime()) : 0ull)
#else
#define FSTAMP(k) ((void)0)
#endif

#ifndef ORBGPU_FAST_CELL_WAVES
#define ORBGPU_FAST_CELL_WAVES 1
#endif
constexpr int kCellWaves = ORBGPU_FAST_CELL_WAVES;  // cells (one per wave) per block: 1 measured fastest (4: 0.839 ms, 2: 0.857, 1: 0.817 per 512 frames)

template <int P>
__global__ __launch_bounds__(64 * kCellWaves) void fast_cells_kernel(Geom g, int ncells_total,
                                                                     const uint8_t* __restrict__ img0, size_t row0,
                                                                     size_t frame0, const uint8_t* __restrict__ pyr,
                                                                     uint32_t* __restrict__ cand,
                                                                     int* __restrict__ cell_counts,
                                                                     int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int R = g.win_rows;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: metadata in SGPRs
    const size_t per_wave = (((size_t)2 * P * R + 2 * ((size_t)fast_list_len(P, R, g.det_max) + 1) + 15) & ~(size_t)15);
    uint8_t* ws = smem + wave * per_wave;
    CellTiles T;
    T.win = ws;
    T.sc = ws + P * R;
    T.la = reinterpret_cast<uint16_t*>(ws + 2 * P * R);
    T.lb = T.la;
    T.dump = fast_list_len(P, R, g.det_max);  // in-place: iteration `base` writes below base + 64 after reading la[base .. base + 64)
    uint8_t* s_win = ws;

    // one cell per wave; waves of a block take consecutive cells of a frame;
    // XCD-swizzled blocks keep a frame's cells (overlapping windows) on one L2
#if ORBGPU_FAST_SWIZZLE == 2
    // XCD-local runs: blocks are dealt round-robin over the 8 XCDs (b and b + 8
    // share one), so within each window of 64 consecutive blocks the 8 blocks
    // of one XCD take 8 consecutive cells -- horizontal neighbours of a cell
    // row, whose windows overlap by 6 px and share 64-B sectors -- and fetch
    // their shared lines into one L2 instead of up to three.  Dispatch order
    // over time is unchanged (a window's blocks are in flight together); the
    // last partial window keeps the plain order.
    const int b = (int)blockIdx.x, nfull = (int)gridDim.x & ~63;
    const int item = (b < nfull ? (b & ~63) | ((b & 7) << 3) | ((b >> 3) & 7) : b) * kCellWaves + wave;
#elif ORBGPU_FAST_SWIZZLE
    const int item = xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * kCellWaves + wave;
#else
    const int item = (int)blockIdx.x * kCellWaves + wave;
#endif
    if (item >= ncells_total) return;
#ifdef FAST_STAMPS
    const bool stamp_on = (item & 15) == 0;
    unsigned long long ts[8] = {};
#endif
    FSTAMP(0);
    const int f = (int)udiv40((uint32_t)item, g.cells_magic);  // item / total_cells
    const int gc = item - f * g.total_cells;
    // level and cell coordinates of the frame's cell gc: one scalar load
    const uint32_t ce = g.cell_tab[gc];
    const int l = (int)(ce & 15u), ci = (int)((ce >> 4) & 0x3FFFu), cj = (int)(ce >> 18);
    const LevelGeom& L = g.lv[l];
    const int c = ci * L.ncols + cj;
    int* cnt_out = cell_counts + (size_t)f * g.total_cells + gc;
    uint32_t* out = cand + (size_t)f * g.cand_frame + L.cand_offset + (size_t)c * L.cell_cap;

    // window (ORBextractor.cpp:797-814); all values are integral floats there
    const int iniY = kBorder + ci * L.hcell, iniX = kBorder + cj * L.wcell;
    if (iniY >= L.max_by - 3 || iniX >= L.max_bx - 6) {
        if (lane == 0) *cnt_out = 0;
        return;
    }
    const int maxY = min(iniY + L.hcell + 6, L.max_by), maxX = min(iniX + L.wcell + 6, L.max_bx);
    const int wh = maxY - iniY;
    const uint8_t* base = l == 0 ? img0 + (size_t)f * frame0 : pyr + L.offset + (size_t)f * L.frame_bytes;
    const uint32_t pitch = l == 0 ? (uint32_t)row0 : (uint32_t)L.pitch;  // < 2^24 (launcher check)

    // stage rows: bytes [xa - sh, maxX) at tile column 0.., xa = iniX & ~3, where the
    // shift sh puts the detection region's first column (iniX + 3) on a 4-aligned
    // tile column (4 or 8): the dword compass then needs ceil(dw / 4) groups per
    // row -- 8 for the 30-32 px cells, so 8 rows per pass on all 64 lanes instead
    // of 9 groups and 7 rows for about half of them (round 6).  The loads start
    // at any byte (one unaligned vector load each); maxX <= w - 16, so no over-read.
    const int xa = iniX & ~3, sh = (1 - (iniX - xa)) & 3, ox = iniX - xa + sh;  // ox: tile column of iniX
    // Every window row is staged as P bytes: NC chunks of CB bytes (16 when P is
    // a multiple of 16, else 4), so LDS chunk (r, q) sits at CB * (r * NC + q)
    // and a fixed lane -> (row rl, chunk q) map covers RPI = 64 / NC rows per
    // pass at LDS offset CB * lane + pass * RPI * P: the stores take immediate
    // offsets, and a load's address costs a row clamp and one 24-bit multiply-
    // add (the map is computed once per lane; round 4's per-load division and
    // offset arithmetic was ~16 VALU per load, 128 per wave).  Lanes past
    // RPI * NC map to row RPI with the same formula, i.e. they stage the next
    // pass's first row (the same bytes).  Chunks past the window's last needed
    // one re-read that chunk (column clamp: no read past maxX + 15 <= w - 1),
    // rows past the window re-read its last row; both land in LDS the detection
    // never reads: rows >= wh, inside the score tile (zeroed after; the
    // launcher checks the bound, fast_stage_rows).  A whole group's stores are
    // unconditional (no load is sunk behind a branch); the last partial group
    // stores only its passes.  All of a lane's loads of a group are issued
    // before any is stored.
#ifdef FAST_PROBE_SAMEWIN
    // latency probe (diagnostic build only; wrong results): every cell stages
    // its window from frame 0's level 0 at (16, 16) -- L2-resident after the first
    const uint8_t* wbase = uniform_ptr(img0 + (size_t)kBorder * row0 + kBorder);
    (void)base;
#else
    const uint8_t* wbase = uniform_ptr(base + (size_t)iniY * pitch + (xa - sh));
#endif
    {
        constexpr int CB = FastStage<P>::CB, NC = FastStage<P>::NC, RPI = FastStage<P>::RPI,
                      kGroup = FastStage<P>::kGroup;
        const int rl = lane / NC, q = lane - rl * NC;  // compile-time divisor
        const int ncneed = (maxX - xa + sh + CB - 1) / CB;
        const uint32_t col = (uint32_t)(CB * min(q, ncneed - 1));
        const int passes = (wh + RPI - 1) / RPI;  // wave-uniform
        uint8_t* dst = s_win + CB * lane;
        typedef typename std::conditional<CB == 16, uint4, uint32_t>::type Chunk;
        // one group of NG passes: all its loads issued, then its stores
        auto stage_group = [&](auto ngc, int p0) {
            constexpr int NG = decltype(ngc)::value;
            Chunk v[NG];
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const uint32_t r = (uint32_t)min(rl + RPI * (p0 + k), wh - 1);
#ifdef FAST_PROBE_SAMEWIN
                const uint8_t* src = wbase + (__umul24(r, (uint32_t)row0) + col);
#else
                const uint8_t* src = wbase + (__umul24(r, pitch) + col);
#endif
                if constexpr (CB == 16)
                    v[k] = load16_a1(src);
                else
                    v[k] = load4_a1(src);
            }
            if (p0 + NG <= passes) {  // a whole group (wave-uniform): unconditional stores
#pragma unroll
                for (int k = 0; k < NG; ++k) *reinterpret_cast<Chunk*>(dst + (p0 + k) * RPI * P) = v[k];
            } else {  // the last, partial group
#pragma unroll
                for (int k = 0; k < NG; ++k)
                    if (p0 + k < passes) *reinterpret_cast<Chunk*>(dst + (p0 + k) * RPI * P) = v[k];
            }
        };
#pragma unroll 1
        for (int p0 = 0; p0 < passes; p0 += kGroup) stage_group(std::integral_constant<int, kGroup>{}, p0);
    }
    // (T.sc is 16-byte aligned when P * R is: then 16-byte stores, else dwords)
    const int nz16 = (P * R) % 16 == 0 ? P * R / 16 : 0;
    for (int idx = lane; idx < nz16; idx += 64) reinterpret_cast<uint4*>(T.sc)[idx] = make_uint4(0u, 0u, 0u, 0u);
    for (int idx = nz16 * 4 + lane; idx < P * R / 4; idx += 64) reinterpret_cast<uint32_t*>(T.sc)[idx] = 0u;
    wave_sync();
    FSTAMP(1);

    // detection region of cv::FAST on the window: rows [3, wh-3), cols [3, ww-3)
    const int dw = maxX - iniX - 6, dh = wh - 6;
    int total = 0;
#ifdef FAST_STAMPS
    int st_nb = 0, st_retry = 0;
    unsigned long long cst[2] = {0, 0};
#endif
#if ORBGPU_FAST_BANDS
    if (dw > 0 && dh > 0) {
        int nb = 0;
        bool dropped = false;
        total = fast_cell_banded<P>(T, dw, dh, ox, g.ini_th, lane, iniX, iniY, out, L.cell_cap, err, &nb, &dropped);
        FSTAMP(2);
        FSTAMP(3);
#ifdef FAST_STAMPS
        st_nb = total;
        cst[0] = ts[2];  // (the banded path has no separate compass stamp)
#endif
        if (total == 0) {  // ORBextractor.cpp:821-825: retry the cell at minThFAST
#ifdef FAST_STAMPS
            st_retry = 1;
#endif
            if (!dropped)
                for (int j = lane; j < nb; j += 64) T.sc[T.lb[j]] = 0;
            else
                for (int idx = lane; idx < P * R / 4; idx += 64) reinterpret_cast<uint32_t*>(T.sc)[idx] = 0u;
            wave_sync();
            total = fast_cell_banded<P>(T, dw, dh, ox, g.min_th, lane, iniX, iniY, out, L.cell_cap, err, &nb, &dropped);
        }
    }
    if (false) {
#else
    if (dw > 0 && dh > 0) {
#endif
#ifdef FAST_STAMPS
        int nb = fast_corners<P>(T, dw, dh, ox, g.ini_th, lane, stamp_on ? cst : nullptr);
#else
        int nb = fast_corners<P>(T, dw, dh, ox, g.ini_th, lane);
#endif
        FSTAMP(2);
        total = nms_emit<P>(T, nb, ox, g.ini_th, lane, iniX, iniY, out, L.cell_cap, err);
        FSTAMP(3);
#ifdef FAST_STAMPS
        st_nb = nb;
#endif
        if (total == 0) {  // ORBextractor.cpp:821-825: retry the cell at minThFAST
#ifdef FAST_STAMPS
            st_retry = 1;
#endif
            for (int j = lane; j < nb; j += 64) T.sc[T.lb[j]] = 0;
            wave_sync();
            nb = fast_corners<P>(T, dw, dh, ox, g.min_th, lane);
            total = nms_emit<P>(T, nb, ox, g.min_th, lane, iniX, iniY, out, L.cell_cap, err);
        }
    }
    if (lane == 0) *cnt_out = min(total, L.cell_cap);
#ifdef FAST_STAMPS
    FSTAMP(4);
    if (stamp_on && lane == 0) {
        if (dw > 0 && dh > 0) {
            for (int k = 1; k <= 4; ++k) atomicAdd(&g_fast_stamps[k - 1], ts[k] - ts[k - 1]);
            atomicAdd(&g_fast_stamps[6], cst[0] - ts[1]);  // compass part of fast_corners
            atomicAdd(&g_fast_stamps[8], cst[1]);          // compass survivors
        } else
            atomicAdd(&g_fast_stamps[4], ts[4] - ts[0]);
        atomicAdd(&g_fast_stamps[5], ts[1] - ts[0]);
        atomicAdd(&g_fast_stamps[9], (unsigned long long)st_nb);
        atomicAdd(&g_fast_stamps[10], (unsigned long long)st_retry);
        atomicAdd(&g_fast_stamps[15], 1ull);
    }
#endif
}

}  // namespace

#ifdef FAST_STAMPS
extern "C" int orbgpu_debug_fast_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_stamps), sizeof(g_fast_stamps)) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fast_stamps), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif


hipError_t launch_fast_cells(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                             const uint8_t* pyr, uint32_t* cand, int* cell_counts, int* err,
                             hipStream_t stream) {
    const int items = g.total_cells * batch;
    if (row0 >= (1u << 24)) return hipErrorInvalidValue;  // row offsets by 24-bit multiplies
    if (items >= (1 << 24) || g.total_cells >= (1 << 16)) return hipErrorInvalidValue;  // udiv40's range
    const size_t per_wave =
        (((size_t)2 * g.win_pitch * g.win_rows + 2 * ((size_t)fast_list_len(g.win_pitch, g.win_rows, g.det_max) + 1) + 15) & ~(size_t)15);
    dim3 grid((items + kCellWaves - 1) / kCellWaves);
    const size_t lds = per_wave * kCellWaves;
#define ORBGPU_FAST_CASE(PP)                                                                                        \
    case PP:                                                                                                        \
        if (fast_stage_rows<PP>(g.win_rows) > 2 * g.win_rows) return hipErrorInvalidValue;                        \
        hipLaunchKernelGGL(fast_cells_kernel<PP>, grid, dim3(64 * kCellWaves), lds, stream, g, items, img0, row0, \
                           frame0, pyr, cand, cell_counts, err);                                                   \
        break;
    switch (g.win_pitch) {
        ORBGPU_FAST_CASE(40)
        ORBGPU_FAST_CASE(48)
        ORBGPU_FAST_CASE(56)
        ORBGPU_FAST_CASE(64)
        ORBGPU_FAST_CASE(72)
        default:
            return hipErrorInvalidValue;
    }
#undef ORBGPU_FAST_CASE
    return hipGetLastError();
}

}  // namespace orbgpu
