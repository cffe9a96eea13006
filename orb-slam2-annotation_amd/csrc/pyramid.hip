// pyramid.hip -- ORBextractor::ComputePyramid (ORBextractor.cpp:1123-1148)
// for all levels of a frame band in ONE launch.
//
// Level l = resize(level l-1, INTER_LINEAR) with OpenCV-2.4's 8U fixed-point
// arithmetic: Q11 horizontal taps (exact int), VResizeLinearVec_32s8u on
// x < simd_end and FixedPtCast<int,uchar,22> on the tail.  The x/y tap
// tables come from the host (orbgpu.cpp, build_resize_tables) exactly as
// resize() builds xofs/ialpha/yofs/ibeta.
//
// Fusion: a block owns one horizontal band of one frame and walks the levels
// bottom-up.  Each level's band rows (its owned rows plus the few halo rows
// the band's next level reads, planned on the host: plan_pyramid_bands) are
// computed from the previous level's rows held in LDS, written to LDS for the
// next level and to HBM (halo rows too: the neighbouring band writes the same
// bytes there).  The band's level-0 rows are staged into LDS once with 16-byte
// loads.  So no level is read back from HBM by this pass: HBM traffic is
// |P_0| + sum_l |P_l| (+ halo), while the
// algorithmic bytes of the reference's level-by-level pass
// (sum_l |P_{l-1}| + |P_l|) are larger.
//
// Per output quad and source row: one 12-byte window (three dwords), v_perm_b32
// spreads each pixel's tap pair into the high bytes of two 16-bit lanes and
// v_dot2_u32_u16 applies (16 ialpha0, 16 ialpha1): 4096 x the exact
// horizontal sum, whose high half is the (h >> 4) of the vertical pass.  Row
// groups walk runs of consecutive output rows and keep the last source row's
// sums in registers (~1.2 horizontal passes per output row).  The vertical
// pass is four SDWA/op_sel instructions per pixel (vert_simd).
#include <algorithm>

#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

#ifndef PYR_PROBE
#define PYR_PROBE 0  // timing probes for tuning only (tools/pyr_variants.sh): bit 0 = no level-0 loads, bit 2 = level 1 only, bit 3 = phase stamps, bit 5 = no HBM stores in the row loop, bit 6 = no window loads (frame kernel), bit 7 = no store drain before the level barrier (frame kernel, wrong results), bit 8 = band kernel setup only (no rows); 0 = the product
#endif
#ifndef PYR_THREADS
#define PYR_THREADS 1024
#endif
constexpr int kPyrThreads = PYR_THREADS;
#ifndef PYR_WAVES_EU
#define PYR_WAVES_EU 8  // frame kernel: waves per SIMD the register budget is sized for
#endif
constexpr int kPyrPre = 4;     // level-0 uint4 loads per thread per item (host checks the band fits)
constexpr int kPyrPreRec = 1;  // record int4 per thread per item (host checks pyr_rec_stride <= threads)

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

#if PYR_PROBE & 8
// diagnostic build only: per-block phase stamps (never read by the kernel)
__device__ unsigned long long g_pyr_stamps[8192 * 10];
__device__ __forceinline__ void pyr_stamp_at(int item, int slot) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (threadIdx.x == 0 && item < 8192) g_pyr_stamps[item * 10 + slot] = t;
}
#define PYR_STAMP(i) pyr_stamp_at(item, i)
__device__ unsigned long long g_pyr_wave[8192 * 8 * 16];
#else
#define PYR_STAMP(i) ((void)0)
#endif

// Column taps of a thread's quad (host: build_geometry, 3 int4 per quad):
// the byte offset w0 of a 12-byte window in the source row, the four
// (16 ialpha0, 16 ialpha1) weight pairs and the four v_perm_b32 selectors
// (pixels 0..2 from dwords (d1:d0), pixel 3 from (d2:d1)); each selector puts
// a pixel's two tap bytes in the high bytes of two 16-bit lanes.
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
// x = (h0>>4) b0 + 2^17 (v_mad_u32_u16, op_sel picks the high half), y =
// (h1>>4) b1 (SDWA WORD_1), then one SDWA add of the two high halves lands
// the rounded sum + 2 in a 16-bit lane; a packed shift and one v_perm_b32
// give the four bytes.  No saturation is needed: with non-negative Q11
// weights every partial sum is <= 1020.
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

// A thread's quad of one level: which quad and row group, and its column
// taps, loaded one level ahead (before the barrier that ends the previous
// level) so the table read's latency is hidden by the barrier wait.
struct QuadTaps {
    int4 a, b, c;
    int q, rg;
    int mode;  // 0 idle, 1 vector quad (1 .. qmain-1), 2 first quad, 3 scalar-tail quad
};

// Thread layout of a level: vector quads 1 .. qmain-1 fill threads
// [0, (qmain-1) * rgroups) (row group rg = t / (qmain-1) owns one run of
// consecutive rows); the edge wave starting at tail_base takes the first quad
// of every row on lanes 0..31 (its column window starts up to 8 bytes before
// the row) and the scalar-tail quad on lanes 32..63 (lane = row, rows lane,
// lane + 32, ...), so the main loop never meets either case.
__device__ __forceinline__ QuadTaps quad_taps(const LevelGeom& V, const int4* __restrict__ ptab) {
    QuadTaps tp;
    const int t = threadIdx.x;
    const int qv = V.qmain - 1;
    tp.mode = 0;
    tp.q = 0;
    tp.rg = 0;
    if (t < qv * V.rgroups) {
        tp.rg = (int)__umulhi((uint32_t)t, V.quad_magic);
        tp.q = 1 + t - tp.rg * qv;
        tp.mode = 1;
    } else if (t >= V.tail_base && t < V.tail_base + 32) {
        tp.rg = t - V.tail_base;
        tp.q = 0;
        tp.mode = 2;
    } else if (t >= V.tail_base + 32 && t < V.tail_base + 64 && 4 * V.qmain < V.w) {
        tp.rg = t - V.tail_base - 32;
        tp.q = V.qmain;
        tp.mode = 3;
    }
    if (tp.mode) {
        const int4* pt = ptab + V.ptab_offset + 3 * tp.q;
        tp.a = pt[0];
        tp.b = pt[1];
        tp.c = pt[2];
    }
    return tp;
}

// Band-kernel thread layout of a level: quads 0 .. qmain-1 (the first quad's
// window may start before the row: the LDS row buffers have 16 bytes in
// front) fill threads [0, qmain * brgroups), row group rg = t / qmain; the
// scalar-tail quad of row group rg is lane rg of the wave at btail_base, so
// it walks the same run of rows as its group.
__device__ __forceinline__ QuadTaps band_taps(const LevelGeom& V, const int4* __restrict__ ptab) {
    QuadTaps tp;
    const int t = threadIdx.x;
    tp.mode = 0;
    tp.q = 0;
    tp.rg = 0;
    if (t < V.qmain * V.brgroups) {
        tp.rg = (int)__umulhi((uint32_t)t, V.bquad_magic);
        tp.q = t - tp.rg * V.qmain;
        tp.mode = 1;
    } else if (t >= V.btail_base && t < V.btail_base + V.brgroups && 4 * V.qmain < V.w) {
        tp.rg = t - V.btail_base;
        tp.q = V.qmain;
        tp.mode = 3;
    }
    if (tp.mode) {
        const int4* pt = ptab + V.ptab_offset + 3 * tp.q;
        tp.a = pt[0];
        tp.b = pt[1];
        tp.c = pt[2];
    }
    return tp;
}

// One level's band rows [r0, r1) in runs of n rows per row group (n even,
// from the band record).  s_rows[r - r0] = (LDS offset of source row y0, of
// y1, ibeta0, ibeta1).  Stores go to the next level's LDS buffer (lds_dst, if
// any) and to HBM: every computed row, halo rows included -- a halo row is
// also an owned row of the neighbouring band, computed there from the same
// source rows with the same arithmetic, so the two writes carry identical
// bytes.  Bytes past V.w land in the row padding (LDS pitch and HBM pitch are
// multiples of 4 and 16).
//
// Rows of a ~1.2x downscale share source rows (y0 of row r+1 is mostly y1 of
// row r), so the last source row's sums stay in registers: about 1.2
// horizontal passes per output row.  Unrolled by two with the roles of P and
// Q swapped, so the carried row needs no register moves.
template <bool TAIL>
__device__ __forceinline__ void resize_rows(const uint8_t* __restrict__ lds, const LevelGeom& V, const QuadTaps& tp,
                                            int r0, int r1, int n, const int4* __restrict__ s_rows,
                                            uint8_t* __restrict__ lds_dst, uint8_t* __restrict__ hbm_dst) {
    Taps t;
    t.w0 = tp.a.x;
    t.wt[0] = tp.a.y; t.wt[1] = tp.a.z; t.wt[2] = tp.a.w; t.wt[3] = tp.b.x;
    t.sel[0] = tp.b.y; t.sel[1] = tp.b.z; t.sel[2] = tp.b.w; t.sel[3] = tp.c.x;
    const int q = tp.q;
    uint32_t P[4], Q[4];
    const uint32_t lpitch = (uint32_t)V.lds_pitch, hpitch = (uint32_t)V.pitch;
    auto vert = [&](const uint32_t (&a)[4], const uint32_t (&b)[4], const int4& y) {
        return TAIL ? vert_tail(a, b, (uint32_t)y.z, (uint32_t)y.w) : vert_simd(a, b, (uint32_t)y.z, (uint32_t)y.w);
    };
#if PYR_PROBE & 256
    const int ra = r0 + tp.rg * n, rb = ra + (((int)lpitch) >> 20);  // timing probe: setup only, no rows
#else
    const int ra = r0 + tp.rg * n, rb = min(ra + n, r1);
#endif
    if (ra >= rb) return;
    uint8_t* lp = lds_dst ? lds_dst + __umul24((uint32_t)(ra - r0), lpitch) + 4 * q : nullptr;
    uint8_t* hp = hbm_dst + __umul24((uint32_t)ra, hpitch) + 4 * q;
    const int4* rec = s_rows + (ra - r0);
    int cur = -1;  // LDS offset of the source row whose sums are in P
    int r = ra;
    for (; r + 1 < rb; r += 2) {
        const int4 y = rec[0];
        const int4 z = rec[1];
        rec += 2;
        if (y.x != cur) hrow(P, lds, t, y.x);
        hrow(Q, lds, t, y.y);
        const uint32_t o0 = vert(P, Q, y);
        if (z.x != y.y) hrow(Q, lds, t, z.x);
        hrow(P, lds, t, z.y);
        const uint32_t o1 = vert(Q, P, z);
        cur = z.y;
        if (lp) {
            *reinterpret_cast<uint32_t*>(lp) = o0;
            *reinterpret_cast<uint32_t*>(lp + lpitch) = o1;
            lp += 2 * lpitch;
        }
#if !(PYR_PROBE & 32)
        *reinterpret_cast<uint32_t*>(hp) = o0;
        *reinterpret_cast<uint32_t*>(hp + hpitch) = o1;
#endif
        hp += 2 * hpitch;
    }
    if (r < rb) {
        const int4 y = rec[0];
        if (y.x != cur) hrow(P, lds, t, y.x);
        hrow(Q, lds, t, y.y);
        const uint32_t o0 = vert(P, Q, y);
        if (lp) *reinterpret_cast<uint32_t*>(lp) = o0;
        *reinterpret_cast<uint32_t*>(hp) = o0;
    }
}

__device__ __forceinline__ void resize_band(const uint8_t* __restrict__ lds, const LevelGeom& V, const QuadTaps& tp,
                                            int r0, int r1, int n, const int4* __restrict__ s_rows,
                                            uint8_t* __restrict__ lds_dst, uint8_t* __restrict__ hbm_dst) {
    if (tp.mode == 1)
        resize_rows<false>(lds, V, tp, r0, r1, n, s_rows, lds_dst, hbm_dst);
    else if (tp.mode == 3)
        resize_rows<true>(lds, V, tp, r0, r1, n, s_rows, lds_dst, hbm_dst);
}

// ---------------------------------------------------------------------------
// Frame-per-block form (pyramid_frame_kernel): a 1024-thread block owns one
// frame and computes level l from level l-1 read straight from memory (level
// 0 = the caller's frame, levels >= 1 = this block's own writes of the
// previous level, L2/MALL-resident), so there is no band halo and no LDS
// staging, and every row group walks one long run of rows.  Source windows
// come through buffer loads: the hardware range check turns the few reads
// outside a level (the window of quad 0 starts up to 8 bytes before a row)
// into zeros instead of faults, and those bytes are never selected by a tap.
// Window loads run one row pair ahead of their use.
// ---------------------------------------------------------------------------
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

struct Win {
    uint32_t d0, d1, d2;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ Win ldwin(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
#if PYR_PROBE & 64
    return Win{voff, voff ^ soff, voff + soff};  // timing probe: no window loads
#else
    const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)voff, (int)soff, 0);
    return Win{v.x, v.y, v.z};
#endif
}

// hrow() on a window already in registers
__device__ __forceinline__ void hwin(uint32_t (&h)[4], const Win& w, const Taps& t) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = k < 3 ? __builtin_amdgcn_perm(w.d1, w.d0, t.sel[k]) : __builtin_amdgcn_perm(w.d2, w.d1, t.sel[k]);
        h[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p), __builtin_bit_cast(us2, t.wt[k]), 0u, false);
    }
}

// One level of one frame.  rec[r] = (y0 of output row r, ibeta0 | ibeta1 <<
// 16); the second source row is y0 + 1 (at the bottom clamp ibeta1 = 0, so
// whatever that row holds is multiplied by zero).  sp = source row pitch,
// src = buffer resource over the source level of this frame.
template <bool TAIL>
__device__ __forceinline__ void frame_rows(__amdgpu_buffer_rsrc_t src, uint32_t sp, const LevelGeom& V,
                                           const QuadTaps& tp, const int2* __restrict__ rec,
                                           uint8_t* __restrict__ dst) {
    Taps t;
    t.w0 = tp.a.x;
    t.wt[0] = tp.a.y; t.wt[1] = tp.a.z; t.wt[2] = tp.a.w; t.wt[3] = tp.b.x;
    t.sel[0] = tp.b.y; t.sel[1] = tp.b.z; t.sel[2] = tp.b.w; t.sel[3] = tp.c.x;
    const uint32_t dp = (uint32_t)V.pitch;
    const uint32_t q4 = 4u * (uint32_t)tp.q;
    const int rows = V.h;
    uint32_t P[4], Q[4];
    auto voff = [&](int y) { return __umul24((uint32_t)y, sp) + (uint32_t)t.w0; };
    if (TAIL) {  // edge wave: one row per lane, first quad (mode 2) or scalar tail (mode 3)
        // The first quad's window starts at w0 = -4 or -8: on row 0 that is
        // before the level, where a buffer load returns zeros for all three
        // dwords, so the load starts at 0 and the dwords move up instead.
        auto ld = [&](int o) {
            Win w = ldwin(src, (uint32_t)max(o, 0), 0);
            if (o == -4) {
                w.d2 = w.d1; w.d1 = w.d0; w.d0 = 0;
            } else if (o == -8) {
                w.d2 = w.d0; w.d1 = 0; w.d0 = 0;
            }
            return w;
        };
        for (int r = tp.rg; r < rows; r += 32) {
            const int2 y = rec[r];
            const int o = (int)voff(y.x);
            const Win w0 = ld(o), w1 = ld(o + (int)sp);
            hwin(P, w0, t);
            hwin(Q, w1, t);
            const uint32_t out = tp.mode == 2 ? vert_simd(P, Q, (uint32_t)y.y, (uint32_t)y.y >> 16)
                                              : vert_tail(P, Q, (uint32_t)y.y & 0xFFFFu, (uint32_t)y.y >> 16);
            *reinterpret_cast<uint32_t*>(dst + __umul24((uint32_t)r, dp) + q4) = out;
        }
        return;
    }
    // row group rg: run [ra, rb) of n rows (n a multiple of 4)
    const int R = V.rgroups;
    const int n = ((rows + R - 1) / R + 3) & ~3;
    const int ra = tp.rg * n;
    if (ra >= rows) return;
    const int rb = min(ra + n, rows);
    uint32_t ho = __umul24((uint32_t)ra, dp) + q4;
    int cur = -1;  // source row whose sums are in P
    int r = ra;
    // two output rows per step: (P, Q) for the first, (Q, P) for the second,
    // so the carried source row never moves between registers.  The y1 row's
    // window of every output row is loaded a pair ahead; the y0 row's only
    // when it is not the carried row (run start, or y0 advancing by 2), on
    // demand.
    auto pair = [&](const int2 ya, const int2 yb, const Win& a1, const Win& b1) {
        if (ya.x != cur) hwin(P, ldwin(src, voff(ya.x), 0), t);
        hwin(Q, a1, t);
        const uint32_t o0 = vert_simd(P, Q, (uint32_t)ya.y, (uint32_t)ya.y >> 16);
        if (yb.x != ya.x + 1) hwin(Q, ldwin(src, voff(yb.x), 0), t);
        hwin(P, b1, t);
        const uint32_t o1 = vert_simd(Q, P, (uint32_t)yb.y, (uint32_t)yb.y >> 16);
        cur = yb.x + 1;
#if !(PYR_PROBE & 32)
        *reinterpret_cast<uint32_t*>(dst + ho) = o0;
        *reinterpret_cast<uint32_t*>(dst + ho + dp) = o1;
#endif
        ho += 2 * dp;
    };
    if (rb - ra >= 4) {
        int2 ya = rec[r], yb = rec[r + 1];
        Win A1 = ldwin(src, voff(ya.x), sp), B1 = ldwin(src, voff(yb.x), sp);
        for (; r + 3 < rb; r += 4) {
            const int2 yc = rec[r + 2], yd = rec[r + 3];
            const Win C1 = ldwin(src, voff(yc.x), sp), D1 = ldwin(src, voff(yd.x), sp);
            pair(ya, yb, A1, B1);
            ya = rec[min(r + 4, rb - 1)];
            yb = rec[min(r + 5, rb - 1)];
            A1 = ldwin(src, voff(ya.x), sp);
            B1 = ldwin(src, voff(yb.x), sp);
            pair(yc, yd, C1, D1);
        }
    }
    for (; r < rb; ++r) {  // the last run's remainder (< 4 rows)
        const int2 y = rec[r];
        const Win w0 = ldwin(src, voff(y.x), 0), w1 = ldwin(src, voff(y.x), sp);
        if (y.x != cur) hwin(P, w0, t);
        hwin(Q, w1, t);
        const uint32_t o = vert_simd(P, Q, (uint32_t)y.y, (uint32_t)y.y >> 16);
        *reinterpret_cast<uint32_t*>(dst + ho) = o;
        ho += dp;
        cur = y.x + 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) P[k] = Q[k];
    }
}

__global__ __launch_bounds__(kPyrThreads) __attribute__((amdgpu_waves_per_eu(PYR_WAVES_EU, PYR_WAVES_EU))) void pyramid_frame_kernel(Geom g, const int2* __restrict__ yrec,
                                                                    const int4* __restrict__ ptab,
                                                                    const uint8_t* __restrict__ img0, size_t row0,
                                                                    size_t frame0, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) int2 s_y[];
    const int f = blockIdx.x;
    const int L = g.nlevels;
    for (int i = threadIdx.x; i < g.pyr_yrec_total; i += kPyrThreads) s_y[i] = yrec[i];
    QuadTaps tp = quad_taps(g.lv[1], ptab);
    __syncthreads();
    for (int l = 1; l < L; ++l) {
        const LevelGeom& V = g.lv[l];
        const LevelGeom& Sv = g.lv[l - 1];
        const uint8_t* src = l == 1 ? img0 + (size_t)f * frame0 : pyr + Sv.offset + (size_t)f * Sv.frame_bytes;
        const uint32_t sp = l == 1 ? (uint32_t)row0 : (uint32_t)Sv.pitch;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, sp * (uint32_t)Sv.h);
        uint8_t* dst = pyr + V.offset + (size_t)f * V.frame_bytes;
        if (tp.mode == 1)
            frame_rows<false>(rs, sp, V, tp, s_y + V.yrec_offset, dst);
        else if (tp.mode >= 2)
            frame_rows<true>(rs, sp, V, tp, s_y + V.yrec_offset, dst);
        if (l + 1 < L) tp = quad_taps(g.lv[l + 1], ptab);
        // level l must be in L2 before any wave reads it as level l+1's source
#if !(PYR_PROBE & 128)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Stream form (pyramid_stream_kernel, the default): one 1024-thread block per
// frame, as the frame kernel, but the source rows reach the row groups through
// LDS: row group g of level l owns output rows [g*run, (g+1)*run) and walks
// them in steps of 4; before step k the block stages, for every group, the 6
// source rows that group's 4 rows read (ystage[k][g] onwards), with
// coalesced 16-byte buffer loads -- 1 KiB per load instruction instead of one
// 12-byte window per lane -- double-buffered one step ahead.  The rows stay
// long runs (the carried source row in registers, no halo), and a level is
// read back from L2/MALL once, by whole-row loads.  The edge wave (first quad
// and scalar-tail quad of every row) reads its windows straight from memory.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t voff) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 0);
    return uint4{v.x, v.y, v.z, v.w};
}

// edge rows [r0, r1) of one level: first quad (mode 2) / scalar tail (mode 3),
// one row per lane of the half-wave, windows from memory
__device__ __forceinline__ void edge_rows(__amdgpu_buffer_rsrc_t src, uint32_t sp, const LevelGeom& V,
                                          const QuadTaps& tp, const int2* __restrict__ rec, uint8_t* __restrict__ dst,
                                          int r0, int r1) {
    Taps t;
    t.w0 = tp.a.x;
    t.wt[0] = tp.a.y; t.wt[1] = tp.a.z; t.wt[2] = tp.a.w; t.wt[3] = tp.b.x;
    t.sel[0] = tp.b.y; t.sel[1] = tp.b.z; t.sel[2] = tp.b.w; t.sel[3] = tp.c.x;
    const uint32_t dp = (uint32_t)V.pitch;
    const uint32_t q4 = 4u * (uint32_t)tp.q;
    uint32_t P[4], Q[4];
    // the first quad's window starts at w0 = -4 or -8: on row 0 that is before
    // the level, where a buffer load returns zeros for all three dwords, so
    // the load starts at 0 and the dwords move up instead
    auto ld = [&](int o) {
        Win w = ldwin(src, (uint32_t)max(o, 0), 0);
        if (o == -4) {
            w.d2 = w.d1; w.d1 = w.d0; w.d0 = 0;
        } else if (o == -8) {
            w.d2 = w.d0; w.d1 = 0; w.d0 = 0;
        }
        return w;
    };
    for (int r = r0 + tp.rg; r < r1; r += 32) {
        const int2 y = rec[r];
        const int o = (int)(__umul24((uint32_t)y.x, sp) + (uint32_t)t.w0);
        const Win w0 = ld(o), w1 = ld(o + (int)sp);
        hwin(P, w0, t);
        hwin(Q, w1, t);
        const uint32_t out = tp.mode == 2 ? vert_simd(P, Q, (uint32_t)y.y, (uint32_t)y.y >> 16)
                                          : vert_tail(P, Q, (uint32_t)y.y & 0xFFFFu, (uint32_t)y.y >> 16);
        *reinterpret_cast<uint32_t*>(dst + __umul24((uint32_t)r, dp) + q4) = out;
    }
}

__global__ __launch_bounds__(kPyrThreads) __attribute__((amdgpu_waves_per_eu(PYR_WAVES_EU, PYR_WAVES_EU))) void
pyramid_stream_kernel(Geom g, const int2* __restrict__ yrec, const int* __restrict__ ystage,
                      const int4* __restrict__ ptab, const uint8_t* __restrict__ img0, size_t row0, size_t frame0,
                      uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_mem[];
    int2* s_y = reinterpret_cast<int2*>(s_mem);
    int* s_ys = reinterpret_cast<int*>(s_mem + (size_t)g.pyr_yrec_total * sizeof(int2));
    uint8_t* s_buf = s_mem + g.pyr_lds_stage;
    const int f = blockIdx.x;
    const int L = g.nlevels;
    const int tid = threadIdx.x;
    for (int i = tid; i < g.pyr_yrec_total; i += kPyrThreads) s_y[i] = yrec[i];
    for (int i = tid; i < g.pyr_ystage_total; i += kPyrThreads) s_ys[i] = ystage[i];
    QuadTaps tp = quad_taps(g.lv[1], ptab);
    __syncthreads();
    const uint32_t SB = (uint32_t)g.pyr_stage_bytes;
    for (int l = 1; l < L; ++l) {
        const LevelGeom& V = g.lv[l];
        const LevelGeom& Sv = g.lv[l - 1];
        const uint8_t* src = l == 1 ? img0 + (size_t)f * frame0 : pyr + Sv.offset + (size_t)f * Sv.frame_bytes;
        const uint32_t spg = l == 1 ? (uint32_t)row0 : (uint32_t)Sv.pitch;  // source pitch in memory
        const uint32_t lp = ((uint32_t)Sv.w + 15u) & ~15u;                    // staged pitch in LDS
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, spg * (uint32_t)Sv.h);
        uint8_t* dst = pyr + V.offset + (size_t)f * V.frame_bytes;
        const int2* rec = s_y + V.yrec_offset;
        const int* ysl = s_ys + V.ystage_offset;
        const int R = V.rgroups, S = V.pyr_steps, run = V.pyr_run, h = V.h;
        // this thread's two staging chunks: (group, row j, 16-byte column c)
        const int cpr = (int)(lp >> 4), pg = 6 * cpr, total = R * pg;
        int sg[2], sgo[2], slo[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + u * kPyrThreads;
            const int gi = i / pg, rem = i - gi * pg, j = rem / cpr, c = rem - j * cpr;
            sg[u] = i < total ? gi : -1;
            sgo[u] = (int)(__umul24((uint32_t)j, spg) + 16u * (uint32_t)c);
            slo[u] = (int)((uint32_t)(gi * 6 + j) * lp + 16u * (uint32_t)c);
        }
        auto gload = [&](int k, int u) {
            uint4 v = uint4{0, 0, 0, 0};
            if (sg[u] >= 0) v = ld16(rs, __umul24((uint32_t)ysl[k * R + sg[u]], spg) + (uint32_t)sgo[u]);
            return v;
        };
        auto lstore = [&](int k, int u, const uint4& v) {
            if (sg[u] >= 0) *reinterpret_cast<uint4*>(s_buf + (uint32_t)(k & 1) * SB + (uint32_t)slo[u]) = v;
        };
        {
            const uint4 a = gload(0, 0), b = gload(0, 1);
            lstore(0, 0, a);
            lstore(0, 1, b);
        }
        __syncthreads();
        // compute state
        Taps t;
        t.w0 = tp.a.x;
        t.wt[0] = tp.a.y; t.wt[1] = tp.a.z; t.wt[2] = tp.a.w; t.wt[3] = tp.b.x;
        t.sel[0] = tp.b.y; t.sel[1] = tp.b.z; t.sel[2] = tp.b.w; t.sel[3] = tp.c.x;
        const uint32_t dp = (uint32_t)V.pitch;
        const int rg = tp.rg;
        const bool vec = tp.mode == 1 && rg * run < h;
        const int rend = min(rg * run + run, h);
        uint32_t ho = __umul24((uint32_t)(rg * run), dp) + 4u * (uint32_t)tp.q;
        uint32_t P[4], Q[4];
        int cur = -1;
        const int E = (h + S - 1) / S;  // edge rows per step
        for (int k = 0; k < S; ++k) {
            uint4 na = uint4{0, 0, 0, 0}, nb = uint4{0, 0, 0, 0};
            if (k + 1 < S) {
                na = gload(k + 1, 0);
                nb = gload(k + 1, 1);
            }
            if (vec) {
                const int o0 = rg * run + 4 * k;
                if (o0 < rend) {
                    const int ys = ysl[k * R + rg];
                    // LDS offset of staged row 0 of this group, minus ys rows
                    const int base = (int)((uint32_t)(k & 1) * SB + (uint32_t)(rg * 6) * lp) - ys * (int)lp;
                    auto row = [&](int y) { return base + y * (int)lp; };
#pragma unroll
                    for (int j = 0; j < 4; j += 2) {
                        const int o = o0 + j;
                        if (o < rend) {
                            const int2 ya = rec[o];
                            if (ya.x != cur) hrow(P, s_buf, t, row(ya.x));
                            hrow(Q, s_buf, t, row(ya.x + 1));
                            const uint32_t out0 = vert_simd(P, Q, (uint32_t)ya.y, (uint32_t)ya.y >> 16);
#if !(PYR_PROBE & 32)
                            *reinterpret_cast<uint32_t*>(dst + ho) = out0;
#endif
                            ho += dp;
                            cur = ya.x + 1;
                            if (o + 1 < rend) {
                                const int2 yb = rec[o + 1];
                                if (yb.x != cur) hrow(Q, s_buf, t, row(yb.x));
                                hrow(P, s_buf, t, row(yb.x + 1));
                                const uint32_t out1 = vert_simd(Q, P, (uint32_t)yb.y, (uint32_t)yb.y >> 16);
#if !(PYR_PROBE & 32)
                                *reinterpret_cast<uint32_t*>(dst + ho) = out1;
#endif
                                ho += dp;
                                cur = yb.x + 1;
                            } else {
#pragma unroll
                                for (int m = 0; m < 4; ++m) P[m] = Q[m];
                            }
                        }
                    }
                }
            } else if (tp.mode >= 2) {
                edge_rows(rs, spg, V, tp, rec, dst, k * E, min(k * E + E, h));
            }
            if (k + 1 < S) {
                lstore(k + 1, 0, na);
                lstore(k + 1, 1, nb);
            }
            __syncthreads();
        }
        tp = quad_taps(g.lv[l + 1 < L ? l + 1 : 1], ptab);
        // level l must be in L2 before the next level stages it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// Level-0 rows of a work item (one band of one frame) and its record, held
// in registers between the issue of their loads and their LDS write: the
// loads of item k+1 are issued right after item k's rows reach LDS and land
// while item k's levels are computed.
struct Prefetch {
    uint4 px[kPyrPre];
    int4 rec[kPyrPreRec];
};

__device__ __forceinline__ void prefetch_item(Prefetch& p, const Geom& g, const int4* __restrict__ recs,
                                              const uint8_t* __restrict__ img0, size_t row0, size_t frame0, int item) {
    const int S = g.pyr_bands;
    const int f = item / S, band = item - f * S;
    const int4* rec = recs + (size_t)band * g.pyr_rec_stride;
    const int y0 = __builtin_amdgcn_readfirstlane(rec[0].x), y1 = __builtin_amdgcn_readfirstlane(rec[0].y);
    const int v4 = (g.lv[0].w + 15) >> 4;
    const int n = (y1 - y0) * v4;
    const uint8_t* src = img0 + (size_t)f * frame0 + (size_t)y0 * row0;
    // unconditional loads (an index past the band re-reads chunk 0), so the
    // registers are written on every path
    auto ld = [&](int k) {
        int i = threadIdx.x + k * kPyrThreads;
        i = i < n ? i : 0;
        const int r = (int)__umulhi((uint32_t)i, g.lv[0].quad_magic);
        const int c = i - r * v4;
        return *reinterpret_cast<const uint4*>(src + (size_t)r * row0 + 16 * c);
    };
    static_assert(kPyrPre == 4 && kPyrPreRec == 1, "prefetch is written out for 4 + 1 loads");
    p.px[0] = ld(0);
    p.px[1] = ld(1);
    p.px[2] = ld(2);
    p.px[3] = ld(3);
    p.rec[0] = rec[(int)threadIdx.x < g.pyr_rec_stride ? threadIdx.x : 0];
}

// Persistent blocks: block i processes work items i, i + gridDim.x, ... of
// the batch (item = frame * pyr_bands + band), so the level-0 staging of the
// next item overlaps the current item's levels.
__global__ __launch_bounds__(kPyrThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void pyramid_kernel(Geom g, const int4* __restrict__ recs,
                                                              const int4* __restrict__ ptab,
                                                              const uint8_t* __restrict__ img0, size_t row0,
                                                              size_t frame0, uint8_t* __restrict__ pyr, int items) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_pyr[];
    const int S = g.pyr_bands;
    const int L = g.nlevels;
    int4* s_rec = reinterpret_cast<int4*>(s_pyr + g.pyr_lds_y);
    int item = blockIdx.x;
    Prefetch pf;
    prefetch_item(pf, g, recs, img0, row0, frame0, item);
    QuadTaps tp = band_taps(g.lv[1], ptab);
    const int v4 = (g.lv[0].w + 15) >> 4;
    for (; item < items; item += gridDim.x) {
        PYR_STAMP(0);
        const int f = item / S;
        const int band = item - f * S;
        // this item's level-0 rows and record (band entries + per-row source
        // offsets and y taps) from the prefetch registers into LDS
        {
            const int4* rec = recs + (size_t)band * g.pyr_rec_stride;
            const int y0 = __builtin_amdgcn_readfirstlane(rec[0].x), y1 = __builtin_amdgcn_readfirstlane(rec[0].y);
            const int n = (y1 - y0) * v4;
            uint8_t* dst = s_pyr + g.pyr_lds_b;
            auto st = [&](int k, const uint4& v) {
                const int i = threadIdx.x + k * kPyrThreads;
                if (i < n) {
                    const int r = (int)__umulhi((uint32_t)i, g.lv[0].quad_magic);
                    const int c = i - r * v4;
                    *reinterpret_cast<uint4*>(dst + r * g.lv[0].lds_pitch + 16 * c) = v;
                }
            };
            st(0, pf.px[0]);
            st(1, pf.px[1]);
            st(2, pf.px[2]);
            st(3, pf.px[3]);
            if ((int)threadIdx.x < g.pyr_rec_stride) s_rec[threadIdx.x] = pf.rec[0];
        }
        __syncthreads();
        if (item + (int)gridDim.x < items) prefetch_item(pf, g, recs, img0, row0, frame0, item + gridDim.x);
        PYR_STAMP(1);
        int yoff = L;
#if PYR_PROBE & 4
        for (int l = 1; l < 2; ++l) {
#else
        for (int l = 1; l < L; ++l) {
#endif
            const LevelGeom& V = g.lv[l];
            const int4 bv = s_rec[l];  // computed rows [x, y) (owned rows plus halo), run length z; uniform
            const int bx = __builtin_amdgcn_readfirstlane(bv.x), by = __builtin_amdgcn_readfirstlane(bv.y);
            const int bn = __builtin_amdgcn_readfirstlane(bv.z);
            uint8_t* dst_lds = l + 1 < L ? s_pyr + ((l & 1) ? g.pyr_lds_a : g.pyr_lds_b) : nullptr;
            uint8_t* dst_hbm = pyr + V.offset + (size_t)f * V.frame_bytes;
            resize_band(s_pyr, V, tp, bx, by, bn, s_rec + yoff, dst_lds, dst_hbm);
            yoff += by - bx;
#if PYR_PROBE & 8
            {
                __builtin_amdgcn_sched_barrier(0);
                unsigned long long t;
                asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
                __builtin_amdgcn_sched_barrier(0);
                if ((threadIdx.x & 63) == 0 && item < 8192) g_pyr_wave[(item * 8 + l) * 16 + threadIdx.x / 64] = t;
            }
#endif
            tp = band_taps(g.lv[l + 1 < L ? l + 1 : 1], ptab);
            __syncthreads();
            PYR_STAMP(1 + l);
        }
    }
}

}  // namespace

int pyr_threads() { return kPyrThreads; }
int pyr_prefetch_uint4() { return kPyrPre * kPyrThreads; }
int pyr_prefetch_rec() { return kPyrPreRec * kPyrThreads; }

hipError_t launch_pyramid(const Geom& g, int batch, const int4* recs, const int2* yrec, const int* ystage, const int4* ptab,
                          const uint8_t* img0, size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    if (g.nlevels < 2) return hipSuccess;
    if (g.pyr_mode == 2) {
        hipLaunchKernelGGL(pyramid_stream_kernel, dim3(batch), dim3(kPyrThreads), (size_t)pyr_stream_lds_bytes(g),
                           stream, g, yrec, ystage, ptab, img0, row0, frame0, pyr);
        return hipGetLastError();
    }
    if (g.pyr_mode == 1) {
        hipLaunchKernelGGL(pyramid_frame_kernel, dim3(batch), dim3(kPyrThreads), (size_t)g.pyr_yrec_total * sizeof(int2),
                           stream, g, yrec, ptab, img0, row0, frame0, pyr);
        return hipGetLastError();
    }
    // persistent grid: every resident block slot once (blocks loop over items)
    static int slots = 0, slots_lds = -1;
    if (slots_lds != g.pyr_lds_bytes) {
        int dev = 0, cus = 0, per_cu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&pyramid_kernel),
                                                             kPyrThreads, g.pyr_lds_bytes);
        if (e != hipSuccess) return e;
        slots = std::max(1, cus * std::max(1, per_cu));
        slots_lds = g.pyr_lds_bytes;
    }
    const int items = g.pyr_bands * batch;
#ifdef PYR_GRID_ALL
    slots = items;  // tuning: one block per item
#endif
    hipLaunchKernelGGL(pyramid_kernel, dim3(std::min(items, slots)), dim3(kPyrThreads), g.pyr_lds_bytes, stream, g,
                       recs, ptab, img0, row0, frame0, pyr, items);
    return hipGetLastError();
}

#if PYR_PROBE & 8
extern "C" int orbgpu_debug_pyr_waves(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_wave), (size_t)n * 8 * 16 * sizeof(unsigned long long)) == hipSuccess
               ? 0 : -2;
}
extern "C" int orbgpu_debug_pyr_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_stamps), (size_t)n * 10 * sizeof(unsigned long long)) == hipSuccess
               ? 0 : -2;
}
#endif

int pyr_stream_lds_bytes(const Geom& g) { return g.pyr_lds_stage + 2 * g.pyr_stage_bytes; }

hipError_t pyramid_set_lds_limit(const Geom& g) {
    if (g.pyr_mode == 0)
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, g.pyr_lds_bytes);
    if (g.pyr_mode == 2)
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_stream_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, pyr_stream_lds_bytes(g));
    return hipSuccess;
}

}  // namespace orbgpu
