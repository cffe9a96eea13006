// pyramid.hip -- ORBextractor::ComputePyramid (ORBextractor.cpp:1123-1148):
// every level 1..L-1 of a batch of frames in ONE launch, each level written to
// HBM once and never read back.
//
// Level l = resize(level l-1, INTER_LINEAR) with OpenCV-2.4's 8U fixed-point
// arithmetic: Q11 horizontal taps (exact int), VResizeLinearVec_32s8u on
// x < simd_end and FixedPtCast<int,uchar,22> on the tail.  The x/y tap tables
// come from the host (orbgpu.cpp, build_resize_tables) exactly as resize()
// builds xofs/ialpha and yofs/ibeta.
//
// One block per frame, in ticks (plan: pyramid_plan.cpp).  Producer wave(s)
// stream level 0 into an LDS ring by LDS-DMA, one chunk of tk_t0 rows per
// tick, two chunks in flight; they never store to HBM, so their counted
// vmcnt waits cover only their own loads.  Compute lanes each own one
// (level, row group, 8-pixel column) entry (two when the levels are too wide
// for one block) and at tick k compute that column's rows the plan assigns to
// the group at the tick: rows whose two source rows were in LDS before it.  Each output quad goes to
// HBM and into its level's LDS ring for the next level; the compute waves
// issue no loads at all in the tick loop, so their HBM stores are never waited
// for.  One barrier per tick; HBM traffic = |P_0| + sum_{l>=1} |P_l| per frame.
//
// Per output quad and source row: one 12-byte window (three dwords) from
// LDS, v_perm_b32 spreads each pixel's tap pair into the high bytes of two
// 16-bit lanes and v_dot2_u32_u16 applies (16 ialpha0, 16 ialpha1): 4096 x
// the exact horizontal sum, whose high half is the (h >> 4) of the vertical
// pass.
// The vertical pass is four SDWA/op_sel instructions per pixel.
#include <algorithm>
#include <cstdlib>

#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

#ifndef ORBGPU_PYR_WAVES_EU
#define ORBGPU_PYR_WAVES_EU 4  // register budget hint: 4 measured 0.6-1.4 % faster than 5 (two 10-wave blocks per CU either way, 65-66 VGPRs)
#endif

#ifdef PYR_STAMPS  // diagnostic build only (tools/pyr_ticks.py): per-tick clock stamps of blocks 0..63
__device__ unsigned long long g_pyr_stamps[64 * 160 * 16];
__device__ __forceinline__ unsigned long long pyr_clock() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
// per block (all 512): realtime (100 MHz) at start and end, memtime at start and end, HW_ID, XCC_ID
__device__ unsigned long long g_pyr_blocks[1024 * 6];
#define PYR_BLOCK(slot, v)                                                                              \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 1024) g_pyr_blocks[(size_t)blockIdx.x * 6 + (slot)] = (v);  \
    } while (0)
#define PYR_STAMP(k, slot)                                                                              \
    do {                                                                                                \
        const unsigned long long t_ = pyr_clock();                                                      \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 64 && (k) < 160)                                   \
            g_pyr_stamps[((size_t)blockIdx.x * 160 + (k)) * 16 + (slot)] = t_;                           \
    } while (0)
#else
#define PYR_STAMP(k, slot) ((void)0)
#define PYR_BLOCK(slot, v) ((void)0)
#endif

// Column taps of a quad (host: build_geometry, 3 int4 per quad): the byte
// offset w0 of a 12-byte window in the source row, the four (16 ialpha0, 16
// ialpha1) weight pairs and the four v_perm_b32 selectors (pixels 0..2 from
// dwords (d1:d0), pixel 3 from (d2:d1)); each selector puts a pixel's two tap
// bytes in the high bytes of two 16-bit lanes.
struct Taps {
    int w0;
    uint32_t wt[4], sel[4];
};

// Horizontal pass of one source row for the quad: h[k] = 4096 x the exact
// Q11 sum of pixel k's two taps (HResizeLinear), so the high half of h[k] is
// the (h >> 4) VResizeLinearVec_32s8u multiplies (h <= 255 * 2049, so
// 4096 h < 2^32).  `row` = LDS byte offset of the source row.
__device__ __forceinline__ void hrow(uint32_t (&h)[4], const uint8_t* lds, const Taps& t, int row) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(lds + t.w0 + row);
    const uint32_t d0 = a[0], d1 = a[1], d2 = a[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = k < 3 ? __builtin_amdgcn_perm(d1, d0, t.sel[k]) : __builtin_amdgcn_perm(d2, d1, t.sel[k]);
        h[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p), __builtin_bit_cast(us2, t.wt[k]), 0u, false);
    }
}

// VResizeLinearVec_32s8u for one quad:
//   out = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2
// with (h >> 4) the high half of the 4096-scaled sums.  Per pixel:
// x = (h0>>4) b0 + 2^17 (v_mad_u32_u16, op_sel picks the high half; b0 is the
// low half of the packed taps), y = (h1>>4) b1 (SDWA WORD_1), then one SDWA
// add of the two high halves lands the rounded sum + 2 in a 16-bit lane; a
// packed shift and one v_perm_b32 give the four bytes.  No saturation is
// needed: with non-negative Q11 weights every partial sum is <= 1020.
__device__ __forceinline__ uint32_t vert_simd(const uint32_t (&h0)[4], const uint32_t (&h1)[4], uint32_t b0,
                                              uint32_t b1) {
    uint32_t x[4], y[4], s01, s23;
    const uint32_t two = 2u << 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(x[k]) : "v"(h0[k]), "v"(b0), "s"(two));
        asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
            : "=v"(y[k]) : "v"(h1[k]), "v"(b1));
    }
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
        : "=v"(s01) : "v"(x[0]), "v"(y[0]));
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
        : "+v"(s01) : "v"(x[1]), "v"(y[1]));
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
        : "=v"(s23) : "v"(x[2]), "v"(y[2]));
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
        : "+v"(s23) : "v"(x[3]), "v"(y[3]));
    // both halves shifted by 2: the inline constant feeds the high half only
    // through op_sel_hi (tools/sdwa_probe.hip)
    asm("v_pk_lshrrev_b16 %0, 2, %0 op_sel_hi:[0,1]" : "+v"(s01));
    asm("v_pk_lshrrev_b16 %0, 2, %0 op_sel_hi:[0,1]" : "+v"(s23));
    return __builtin_amdgcn_perm(s23, s01, 0x06040200u);
}

// FixedPtCast<int, uchar, 22> (the scalar tail of VResizeLinear):
// (S0*b0 + S1*b1 + 2^21) >> 22 with S = h = (4096 h) >> 12 < 2^20, b < 2^12.
__device__ __forceinline__ uint32_t vert_tail(const uint32_t (&h0)[4], const uint32_t (&h1)[4], uint32_t b0,
                                              uint32_t b1) {
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        out |= ((__umul24(h0[k] >> 12, b0) + __umul24(h1[k] >> 12, b1) + (1u << 21)) >> 22) << (8 * k);
    return out;
}

// One compute entry: two adjacent quads (8 pixels) of one level and row
// group, with everything the tick loop needs in registers (plan_pyramid
// writes 9 int4: range index, tail bits, record base, LDS pitch | LDS ring
// base, end, HBM pitch, HBM frame bytes | HBM offset of the column, its byte
// offset 8o | the 3 int4 of taps of each quad).
struct TickEnt {
    int rng, tail, rec, lpitch;
    int rbase, rend, hpitch, col8;
    uint32_t hoff;  // byte offset of the column in the pyramid buffer: level offset + 8o + f * frame bytes (< 4 GiB)
    Taps ta, tb;
};

__device__ __forceinline__ Taps load_taps(const int4& t0, const int4& t1, const int4& t2) {
    Taps t;
    t.w0 = t0.x;
    t.wt[0] = t0.y; t.wt[1] = t0.z; t.wt[2] = t0.w; t.wt[3] = t1.x;
    t.sel[0] = t1.y; t.sel[1] = t1.z; t.sel[2] = t1.w; t.sel[3] = t2.x;
    return t;
}

__device__ __forceinline__ TickEnt load_ent(const int4* __restrict__ ent, int f) {
    TickEnt e;
    const int4 a = ent[0], b = ent[1], c = ent[2];
    e.rng = a.x;
    e.tail = a.y;
    e.rec = a.z;
    e.lpitch = a.w;
    e.rbase = b.x;
    e.rend = b.y;
    e.hpitch = b.z;
    e.col8 = c.z;
    e.hoff = (uint32_t)c.x + (uint32_t)f * (uint32_t)b.w;
    e.ta = load_taps(ent[3], ent[4], ent[5]);
    e.tb = load_taps(ent[6], ent[7], ent[8]);
    return e;
}

// Both quads' horizontal passes of one source row.
struct HRow {
    uint32_t a[4], b[4];
};

__device__ __forceinline__ void hrow2(HRow& h, const uint8_t* lds, const TickEnt& e, int row) {
    hrow(h.a, lds, e.ta, row);
    hrow(h.b, lds, e.tb, row);
}

// Vertical pass of both quads.  A level's scalar-tail quad (the last quad of
// a row when w is not a multiple of 16: FixedPtCast form) is always quad B of
// its oct, and those octs fill waves of their own (plan_pyramid), so TAIL is
// wave-uniform and no lane evaluates both forms.
template <bool TAIL>
__device__ __forceinline__ uint2 vert2(const HRow& p, const HRow& q, uint32_t bp) {
    return uint2{vert_simd(p.a, q.a, bp, bp >> 16),
                 TAIL ? vert_tail(p.b, q.b, bp & 0xFFFFu, bp >> 16) : vert_simd(p.b, q.b, bp, bp >> 16)};
}

// The rows [ra, rb) of one entry at one tick.  rec[y] = (LDS offset / 16 of
// source row y0 | of y1 << 16, ibeta0 | ibeta1 << 16); d = LDS slot of row ra
// in the entry's ring (the last level: a sink, lpitch 0).  Consecutive output
// rows share source rows (~1.2x downscale), so the last source row's sums stay
// in registers (~1.2 horizontal passes per output row); two rows per step
// with the roles of P and Q swapped, so the carried row needs no moves.
template <bool TAIL>
__device__ __forceinline__ void tick_rows(const uint8_t* __restrict__ lds, uint8_t* __restrict__ ldsw,
                                          const int2* __restrict__ rec, const TickEnt& e, int ra, int rb, int d,
                                          uint8_t* __restrict__ pyr) {
    uint32_t hp = e.hoff + (uint32_t)ra * (uint32_t)e.hpitch;  // 32-bit offsets: saddr-form stores off the uniform base
    const uint32_t hpitch = (uint32_t)e.hpitch;
    auto advance = [&]() {
        d += e.lpitch;
        if (d == e.rend) d = e.rbase;
    };
    HRow P, Q;
    int cur = -1;  // LDS offset of the source row whose sums are in P
    int y = ra;
    for (; y + 1 < rb; y += 2) {
        const int2 r0 = rec[y], r1 = rec[y + 1];
        const int a0 = (r0.x & 0xFFFF) << 4, a1 = (int)((uint32_t)r0.x >> 16) << 4;
        const int c0 = (r1.x & 0xFFFF) << 4, c1 = (int)((uint32_t)r1.x >> 16) << 4;
        // the tail wave's lanes belong to different levels: no carried-row
        // branch there (it would diverge)
        if (TAIL || a0 != cur) hrow2(P, lds, e, a0);
        hrow2(Q, lds, e, a1);
        const uint2 o0 = vert2<TAIL>(P, Q, (uint32_t)r0.y);
        if (TAIL || c0 != a1) hrow2(Q, lds, e, c0);
        hrow2(P, lds, e, c1);
        const uint2 o1 = vert2<TAIL>(Q, P, (uint32_t)r1.y);
        cur = c1;
        *reinterpret_cast<uint2*>(ldsw + d) = o0;
        advance();
        *reinterpret_cast<uint2*>(ldsw + d) = o1;
        advance();
        *reinterpret_cast<uint2*>(pyr + hp) = o0;
        *reinterpret_cast<uint2*>(pyr + (hp + hpitch)) = o1;
        hp += 2 * hpitch;
    }
    if (y < rb) {
        const int2 r0 = rec[y];
        const int a0 = (r0.x & 0xFFFF) << 4, a1 = (int)((uint32_t)r0.x >> 16) << 4;
        if (TAIL || a0 != cur) hrow2(P, lds, e, a0);
        hrow2(Q, lds, e, a1);
        const uint2 o0 = vert2<TAIL>(P, Q, (uint32_t)r0.y);
        *reinterpret_cast<uint2*>(ldsw + d) = o0;
        *reinterpret_cast<uint2*>(pyr + hp) = o0;
    }
}

// One entry at one tick: its row run from the packed range (row ra: 11
// bits, row count: 5, LDS slot of row ra / 16: 16).
template <bool TAIL>
__device__ __forceinline__ void tick_entry(const uint8_t* __restrict__ lds, uint8_t* __restrict__ ldsw,
                                           const int2* __restrict__ s_tab, const uint32_t* __restrict__ rng,
                                           const TickEnt& e, uint8_t* __restrict__ pyr) {
    const uint32_t r = rng[e.rng];
    const int ra = (int)(r & 0x7FFu), n = (int)((r >> 11) & 31u);
    if (n == 0) return;
    // ldsw + 8o: the entry's column within its ring rows (hoff has it for HBM)
    tick_rows<TAIL>(lds, ldsw + e.col8, s_tab + e.rec, e, ra, ra + n, (int)(r >> 16) << 4, pyr);
}

// Producer waves: level-0 chunk c (rows [c T0, c T0 + T0)) -> its run of
// ring-0 slots, by LDS-DMA (global_load_lds_dwordx4: the 64 lanes of one
// instruction fill 1 KiB of LDS in lane order, each lane from its own
// address), NP instructions per wave per chunk.  The chunk's run is its T0
// rows back to back at the level-0 pitch (a multiple of 16), padded to whole
// instructions; pieces past the chunk land in the pad and pieces of rows past
// the frame re-read its last row.  Two chunks are in flight: the wait for
// chunk c+1 is a counted vmcnt(NP) that leaves chunk c+2's NP loads running,
// and the producer's barriers are raw s_barriers (no fence, so no vmcnt(0)).
typedef __attribute__((address_space(3))) void lds_void;

template <int NP>
__device__ __forceinline__ void pyr_issue(const uint8_t* __restrict__ fb, size_t row0, int c, uint8_t* lds_run,
                                          uint32_t pstep, const int (&prow)[NP], const int (&pcol)[NP], int T0, int K0,
                                          int H0) {
    c = min(c, K0 - 1);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int y = min(c * T0 + prow[j], H0 - 1);
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(fb + (size_t)y * row0 + pcol[j]),
                                         (lds_void*)(lds_run + pstep * (uint32_t)j), 16, 0, 0);
    }
}

// Two frames share each CU (two blocks), and the hardware issues by wave
// priority, then age: the older block's waves win every contended slot, so
// it finishes first (measured: 114 us vs 170 us for the two blocks of a CU,
// tools/pyr_ticks.py) and the younger one then runs alone, leaving the CU
// half used.  A priority that decreases with the tick index (3 at the
// start, 0 at the end) lets a block that is behind win over
// one that is ahead, so the two progress together.  The phases shrink
// towards the end (ticks [0, K/2), [K/2, 3K/4), [3K/4, 7K/8), [7K/8, K)):
// within a phase age decides again, so the last phase bounds how far apart
// the two blocks can finish.
__device__ __forceinline__ void prio_by_progress(int k, int K) {
    if (k == 0) __builtin_amdgcn_s_setprio(3);
    else if (k == K / 2) __builtin_amdgcn_s_setprio(2);
    else if (k == (3 * K) / 4) __builtin_amdgcn_s_setprio(1);
    else if (k == (7 * K) / 8) __builtin_amdgcn_s_setprio(0);
}

template <int NP>
__device__ __forceinline__ void pyr_producer(const Geom& g, const uint8_t* __restrict__ fb, size_t row0, int p,
                                             int P, uint8_t* s_mem) {
    const LevelGeom& V0 = g.lv[0];
    const int T0 = g.tk_t0, K0 = g.tk_k0, H0 = V0.h, K = g.tk_ticks;
    const int v4 = (V0.w + 15) >> 4, items = T0 * v4;
    const int NC = g.tk_nc0;
    // this wave's LDS-DMA base within a chunk run: piece j of lane i of wave w
    // is item m = j P + 64 w + i at byte 16 m of the run
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane((p & ~63) * 16);
    int prow[NP], pcol[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int m = min(p + j * P, items - 1);
        const int r = m / v4;
        prow[j] = r;
        pcol[j] = 16 * (m - r * v4);
    }
    // LDS byte address of chunk c's run + this wave's base; piece j is P*16 further
    auto run = [&](int c) { return s_mem + V0.tk_ring + (uint32_t)(c % NC) * (uint32_t)g.tk_cstride0 + wbase; };
    const uint32_t pstep = 16u * (uint32_t)P;
    pyr_issue<NP>(fb, row0, 0, run(0), pstep, prow, pcol, T0, K0, H0);
    pyr_issue<NP>(fb, row0, 1, run(1), pstep, prow, pcol, T0, K0, H0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NP) : "memory");  // chunk 0 landed, chunk 1 in flight
    pyr_issue<NP>(fb, row0, 2, run(2), pstep, prow, pcol, T0, K0, H0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's share of the plan-table copy
    __builtin_amdgcn_s_barrier();
    for (int k = 0; k < K; ++k) {
        prio_by_progress(k, K);
        // chunk k+1 lands before the barrier that ends tick k; chunk k+2 stays
        // in flight; chunk k+3 is issued as tick k+1 starts (plan_pyramid
        // sizes ring 0 for the two chunks written during a tick)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NP) : "memory");
        __builtin_amdgcn_s_barrier();
        pyr_issue<NP>(fb, row0, k + 3, run(k + 3), pstep, prow, pcol, T0, K0, H0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int E, int NP>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(ORBGPU_PYR_WAVES_EU))) void pyramid_tick_kernel(Geom g, const int4* __restrict__ ents,
                                                            const int2* __restrict__ tab,
                                                            const uint8_t* __restrict__ img0, size_t row0,
                                                            size_t frame0, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_mem[];
    int2* s_tab = reinterpret_cast<int2*>(s_mem + g.tk_lds_tab);
    const int tid = threadIdx.x;
    const int f = blockIdx.x;
    const int nthr = g.tk_threads;
#ifdef PYR_STAMPS
    PYR_BLOCK(0, __builtin_amdgcn_s_memrealtime());
    PYR_BLOCK(2, __builtin_amdgcn_s_memtime());
    {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        PYR_BLOCK(4, hw);
        PYR_BLOCK(5, xcc);
    }
#endif
    for (int i = tid; i < g.tk_tab_n; i += nthr) s_tab[i] = tab[i];
    const int K = g.tk_ticks;
    const int CL = 64 * g.tk_cwaves;
    if (tid >= CL) {
        pyr_producer<NP>(g, img0 + (size_t)f * frame0, row0, tid - CL, g.tk_threads - CL, s_mem);
        return;
    }
    // ---- compute lanes
    TickEnt en[E];
#pragma unroll
    for (int e = 0; e < E; ++e) en[e] = load_ent(ents + (size_t)(e * CL + tid) * 9, f);
    __syncthreads();
    const uint32_t* rng = reinterpret_cast<const uint32_t*>(s_tab) + g.tk_rng;
    // entries whose quad B is a scalar-tail quad fill whole waves (per entry
    // slot) from lane 0, padded with idle lanes, so lane 0 gives the wave's form
    bool tail[E];
#pragma unroll
    for (int e = 0; e < E; ++e) tail[e] = __builtin_amdgcn_readfirstlane(en[e].tail) != 0;
    for (int k = 0; k < K; ++k) {
        prio_by_progress(k, K);
        if (tid < 64) PYR_STAMP(k, 15);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (tail[e])
                tick_entry<true>(s_mem, s_mem, s_tab, rng, en[e], pyr);
            else
                tick_entry<false>(s_mem, s_mem, s_tab, rng, en[e], pyr);
        }
        PYR_STAMP(k, tid >> 6);
        rng += g.tk_rs;
        __syncthreads();
    }
    PYR_BLOCK(1, __builtin_amdgcn_s_memrealtime());
    PYR_BLOCK(3, __builtin_amdgcn_s_memtime());
}

template <int E>
hipError_t launch_e(const Geom& g, int batch, const int4* ents, const int2* tab, const uint8_t* img0, size_t row0,
                    size_t frame0, uint8_t* pyr, hipStream_t s, bool set_lds) {
    const void* fn = nullptr;
#define PYR_NP_CASE(N) \
    case N: fn = reinterpret_cast<const void*>(&pyramid_tick_kernel<E, N>); break;
    switch (g.tk_np) {
        PYR_NP_CASE(1) PYR_NP_CASE(2) PYR_NP_CASE(3) PYR_NP_CASE(4)
        PYR_NP_CASE(5) PYR_NP_CASE(6) PYR_NP_CASE(7) PYR_NP_CASE(8)
        default: return hipErrorInvalidValue;
    }
#undef PYR_NP_CASE
    if (set_lds) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, g.tk_lds_bytes);
    void* args[] = {const_cast<Geom*>(&g), &ents, &tab, &img0, &row0, &frame0, &pyr};
    return hipLaunchKernel(fn, dim3(batch), dim3(g.tk_threads), args, (size_t)g.tk_lds_bytes, s);
}

}  // namespace

#ifdef PYR_STAMPS
extern "C" int orbgpu_debug_pyr_stamps(unsigned long long* out, unsigned long long* blocks) {
    if (blocks && hipMemcpyFromSymbol(blocks, HIP_SYMBOL(g_pyr_blocks), sizeof(g_pyr_blocks)) != hipSuccess) return -2;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_stamps), sizeof(g_pyr_stamps)) == hipSuccess ? 0 : -2;
}
#endif

// ---- small batches (the drop-in Frame path): level by level over the whole chip ----
// The tick kernel runs one block per frame, so a single frame is 66 serial
// ticks on one CU.  For a few frames each level is instead one launch of
// quads over every row of every frame (level l-1 read from HBM/L2 in place),
// with the same arithmetic: exact Q11 horizontal sums, then
// VResizeLinearVec_32s8u for x < simd_end and FixedPtCast<int,uchar,22> on the
// tail.  Tables: xt[x] = (sx0 | sx1 << 16, a0 | a1 << 16) and
// yt[y] = (y0 | y1 << 16, b0 | b1 << 16) as build_resize_tables makes them.
constexpr int kLevelThreads = 64;

__global__ __launch_bounds__(kLevelThreads) void pyramid_level_kernel(const uint8_t* __restrict__ src, int spitch,
                                                                       size_t sframe, uint8_t* __restrict__ dst,
                                                                       int dpitch, size_t dframe, int dw,
                                                                       int simd_end, const int2* __restrict__ xt,
                                                                       const int2* __restrict__ yt) {
    const int q = blockIdx.x * kLevelThreads + threadIdx.x;
    const int y = blockIdx.y, f = blockIdx.z;
    if (4 * q >= dw) return;
    const int2 ty = yt[y];
    const uint32_t b0 = (uint32_t)ty.y & 0xFFFFu, b1 = (uint32_t)ty.y >> 16;
    const uint8_t* r0 = src + (size_t)f * sframe + (size_t)(ty.x & 0xFFFF) * spitch;
    const uint8_t* r1 = src + (size_t)f * sframe + (size_t)((uint32_t)ty.x >> 16) * spitch;
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = 4 * q + k;
        if (x >= dw) break;
        const int2 tx = xt[x];
        const int sx0 = tx.x & 0xFFFF, sx1 = (int)((uint32_t)tx.x >> 16);
        const uint32_t a0 = (uint32_t)tx.y & 0xFFFFu, a1 = (uint32_t)tx.y >> 16;
        const uint32_t h0 = r0[sx0] * a0 + r0[sx1] * a1, h1 = r1[sx0] * a0 + r1[sx1] * a1;
        const uint32_t v = x < simd_end ? ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2u) >> 2
                                        : (h0 * b0 + h1 * b1 + (1u << 21)) >> 22;
        out |= v << (8 * k);
    }
    // the level pitch is a multiple of 16 >= dw: the quad's dword lies inside the row
    *reinterpret_cast<uint32_t*>(dst + (size_t)f * dframe + (size_t)y * dpitch + 4 * q) = out;
}

hipError_t launch_pyramid_levels(const Geom& g, int batch, const int2* xtab, const int2* ytab, const uint8_t* img0,
                                 size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    for (int l = 1; l < g.nlevels; ++l) {
        const LevelGeom& v = g.lv[l];
        const LevelGeom& p = g.lv[l - 1];
        const uint8_t* src = l == 1 ? img0 : pyr + p.offset;
        const int spitch = l == 1 ? (int)row0 : p.pitch;
        const size_t sframe = l == 1 ? frame0 : p.frame_bytes;
        const int quads = (v.w + 3) / 4;
        hipLaunchKernelGGL(pyramid_level_kernel, dim3((quads + kLevelThreads - 1) / kLevelThreads, v.h, batch),
                           dim3(kLevelThreads), 0, stream, src, spitch, sframe, pyr + v.offset, v.pitch,
                           v.frame_bytes, v.w, v.simd_end, xtab + v.xtab_offset, ytab + v.ytab_offset);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---- small batches, one launch: row bands with every level in LDS ----
// The level-by-level launches cost a dependent launch each (7 x ~4.4 us at
// one 640x480 frame, measured, for ~1 us of work each).  Here g.bd_nb blocks
// per frame each own a band of rows of every level and compute all levels of
// it in one launch: level 0's rows the band needs are staged in LDS, then
// level l is computed from level l-1's LDS rows into LDS (levels < L-1) and
// its OWN rows are written to HBM.  A band needs, at level l, its own rows
// plus the source rows of the rows it needs at level l+1 (plan_pyramid_bands:
// a few rows of halo per level, recomputed by the neighbouring band with the
// same arithmetic, so the written rows are exactly the level kernel's).
constexpr int kBandThreads = 1024;  // 16 waves per CU: the per-level loads of one wave hide behind the others
constexpr int kBandMaxLds = 96 * 1024;
constexpr int kBandStage = 4;       // level-0 words per thread per staging round, all loads issued first

__device__ __forceinline__ uint32_t resize_quad(const uint8_t* r0, const uint8_t* r1, int x0, int dw, int simd_end,
                                                const int2* __restrict__ xt, uint32_t b0, uint32_t b1) {
    int2 tx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tx[k] = xt[min(x0 + k, dw - 1)];
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = x0 + k;
        if (x >= dw) break;
        const int sx0 = tx[k].x & 0xFFFF, sx1 = (int)((uint32_t)tx[k].x >> 16);
        const uint32_t a0 = (uint32_t)tx[k].y & 0xFFFFu, a1 = (uint32_t)tx[k].y >> 16;
        const uint32_t h0 = r0[sx0] * a0 + r0[sx1] * a1, h1 = r1[sx0] * a0 + r1[sx1] * a1;
        const uint32_t v = x < simd_end ? ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2u) >> 2
                                        : (h0 * b0 + h1 * b1 + (1u << 21)) >> 22;
        out |= v << (8 * k);
    }
    return out;
}

__global__ __launch_bounds__(kBandThreads) void pyramid_band_kernel(const Geom g, const int4* __restrict__ bands,
                                                                     const int2* __restrict__ xtab,
                                                                     const int2* __restrict__ ytab,
                                                                     const uint8_t* __restrict__ img0, size_t row0,
                                                                     size_t frame0, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_rows[];
    const int L = g.nlevels, tid = threadIdx.x, f = blockIdx.y;
    const int4* B = bands + (size_t)blockIdx.x * L;
    {  // stage level 0's rows [B[0].x, B[0].y)
        const LevelGeom& v = g.lv[0];
        const int4 r = B[0];
        const uint8_t* src = img0 + (size_t)f * frame0;
        uint8_t* dst = s_rows + v.bd_lds_off;
        if ((((uintptr_t)src | row0) & 3) == 0) {
            // whole words inside the row; the row's last partial word bytewise
            const int words = v.w >> 2, n = (r.y - r.x) * words;
            for (int i0 = 0; i0 < n; i0 += kBandThreads * kBandStage) {
                uint32_t w[kBandStage];
#pragma unroll
                for (int k = 0; k < kBandStage; ++k) {
                    const int i = min(i0 + k * kBandThreads + tid, n - 1), y = i / words, c = i - y * words;
                    w[k] = *reinterpret_cast<const uint32_t*>(src + (size_t)(r.x + y) * row0 + 4 * c);
                }
#pragma unroll
                for (int k = 0; k < kBandStage; ++k) {
                    const int i = i0 + k * kBandThreads + tid, y = i / words, c = i - y * words;
                    if (i < n) *reinterpret_cast<uint32_t*>(dst + y * v.bd_pitch + 4 * c) = w[k];
                }
            }
            const int tail = v.w & 3;
            if (tail)
                for (int y = tid; y < r.y - r.x; y += kBandThreads)
                    for (int k = 0; k < tail; ++k)
                        dst[y * v.bd_pitch + 4 * words + k] = src[(size_t)(r.x + y) * row0 + 4 * words + k];
        } else {
            const int n = (r.y - r.x) * v.w;
            for (int i = tid; i < n; i += kBandThreads) {
                const int y = i / v.w, c = i - y * v.w;
                dst[y * v.bd_pitch + c] = src[(size_t)(r.x + y) * row0 + c];
            }
        }
    }
    __syncthreads();
    for (int l = 1; l < L; ++l) {
        const LevelGeom& v = g.lv[l];
        const LevelGeom& p = g.lv[l - 1];
        const int4 r = B[l];
        const int src_lo = B[l - 1].x;
        const uint8_t* srow = s_rows + p.bd_lds_off;
        uint8_t* drow = s_rows + v.bd_lds_off;
        const bool keep = l + 1 < L;
        const int quads = (v.w + 3) >> 2, n = (r.y - r.x) * quads;
        // i / quads by a multiply-high with the host's ceil(2^32 / quads) (exact
        // while i * (quads - 1) < 2^32; quads >= 2: plan_pyramid_bands); the
        // per-element integer division was ~25 VALU on each level's chain
        const uint32_t qmagic = v.bd_qmagic;
        const int2* xt = xtab + v.xtab_offset;
        const int2* yt = ytab + v.ytab_offset;
        uint8_t* out = pyr + v.offset + (size_t)f * v.frame_bytes;
        for (int i = tid; i < n; i += kBandThreads) {
            const int yy = (int)__umulhi((uint32_t)i, qmagic), q = i - yy * quads, y = r.x + yy;
            const int2 ty = yt[y];
            const uint8_t* r0 = srow + ((ty.x & 0xFFFF) - src_lo) * p.bd_pitch;
            const uint8_t* r1 = srow + ((int)((uint32_t)ty.x >> 16) - src_lo) * p.bd_pitch;
            const uint32_t o = resize_quad(r0, r1, 4 * q, v.w, v.simd_end, xt, (uint32_t)ty.y & 0xFFFFu,
                                           (uint32_t)ty.y >> 16);
            if (keep) *reinterpret_cast<uint32_t*>(drow + yy * v.bd_pitch + 4 * q) = o;
            if (y >= r.z && y < r.w) *reinterpret_cast<uint32_t*>(out + (size_t)y * v.pitch + 4 * q) = o;
        }
        __syncthreads();
    }
}

hipError_t launch_pyramid(const Geom& g, int batch, const int4* ents, const int2* tab, const uint8_t* img0,
                          size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    if (g.nlevels < 2) return hipSuccess;
    return g.tk_e == 1 ? launch_e<1>(g, batch, ents, tab, img0, row0, frame0, pyr, stream, false)
                       : launch_e<2>(g, batch, ents, tab, img0, row0, frame0, pyr, stream, false);
}

hipError_t pyramid_set_lds_limit(const Geom& g) {
    if (g.nlevels < 2) return hipSuccess;
    if (g.bd_nb > 0) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_band_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, kBandMaxLds);
        if (e != hipSuccess) return e;
    }
    return g.tk_e == 1 ? launch_e<1>(g, 0, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, true)
                       : launch_e<2>(g, 0, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, true);
}

void plan_pyramid_bands(Geom& g, const std::vector<int2>& ytab, std::vector<int4>& bands) {
    const int L = g.nlevels;
    g.bd_nb = 0;
    g.bd_lds_bytes = 0;
    bands.clear();
    if (L < 2) return;
    auto src_rows = [&](int l, int lo, int hi) {  // level l-1 rows read by level-l rows [lo, hi)
        const int2* yt = ytab.data() + g.lv[l].ytab_offset;
        return int2{yt[lo].x & 0xFFFF, (int)((uint32_t)yt[hi - 1].x >> 16) + 1};
    };
    // the most bands (smallest halo share) whose rows fit the LDS budget; at
    // least one own row per band at every level.  At most 64 (ORBGPU_PYR_BANDS_MAX
    // overrides): a workgroup's level chain is latency bound, so more, smaller
    // bands finish sooner -- one 640x480 frame: 19.2 us at 32 bands, 16.3 us at
    // 64; 96 measured slower again (profiles/r06_notes_ab.txt r6k, r6m)
    static const int nb_max = [] {
        const char* s = std::getenv("ORBGPU_PYR_BANDS_MAX");
        return s ? std::atoi(s) : 64;
    }();
    for (int nb : {128, 96, 64, 48, 32, 24, 16, 8}) {
        if (nb > nb_max) continue;
        bool ok = true;
        for (int l = 1; l < L; ++l) ok = ok && g.lv[l].h >= nb && g.lv[l].w > 4;  // (the kernel's row division needs >= 2 quads)
        if (!ok) continue;
        std::vector<int4> b((size_t)nb * L);
        std::vector<int> cap(L, 0);
        for (int k = 0; k < nb; ++k) {
            int4* B = b.data() + (size_t)k * L;
            for (int l = 1; l < L; ++l) {
                const int h = g.lv[l].h;
                B[l] = int4{0, 0, (int)((long)k * h / nb), (int)((long)(k + 1) * h / nb)};
            }
            B[L - 1].x = B[L - 1].z;
            B[L - 1].y = B[L - 1].w;
            for (int l = L - 1; l >= 1; --l) {
                const int2 s = src_rows(l, B[l].x, B[l].y);
                if (l == 1) {
                    B[0] = int4{s.x, s.y, 0, 0};
                } else {
                    B[l - 1].x = std::min(B[l - 1].z, s.x);
                    B[l - 1].y = std::max(B[l - 1].w, s.y);
                }
            }
            for (int l = 0; l + 1 < L; ++l) cap[l] = std::max(cap[l], B[l].y - B[l].x);
        }
        for (int l = 1; l < L; ++l) {
            const uint64_t quads = (uint64_t)((g.lv[l].w + 3) >> 2);
            g.lv[l].bd_qmagic = (uint32_t)(((1ull << 32) + quads - 1) / quads);
        }
        int off = 0;
        for (int l = 0; l + 1 < L; ++l) {
            LevelGeom& v = g.lv[l];
            v.bd_pitch = (v.w + 15) & ~15;
            v.bd_lds_off = off;
            off += cap[l] * v.bd_pitch;
        }
        if (off > kBandMaxLds) continue;
        g.lv[L - 1].bd_pitch = 0;
        g.lv[L - 1].bd_lds_off = 0;
        g.bd_nb = nb;
        g.bd_lds_bytes = off;
        bands = std::move(b);
        return;
    }
}

hipError_t launch_pyramid_bands(const Geom& g, int batch, const int4* bands, const int2* xtab, const int2* ytab,
                                const uint8_t* img0, size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    if (g.nlevels < 2 || batch <= 0) return hipSuccess;
    if (g.bd_nb <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pyramid_band_kernel, dim3(g.bd_nb, batch), dim3(kBandThreads), (size_t)g.bd_lds_bytes, stream,
                       g, bands, xtab, ytab, img0, row0, frame0, pyr);
    return hipGetLastError();
}

}  // namespace orbgpu
