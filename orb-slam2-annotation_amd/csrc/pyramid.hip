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
// next level and, for owned rows, to HBM.  The band's level-0 rows are staged
// into LDS once with 16-byte loads.  So every level is written to HBM once and never read back by
// this pass: HBM traffic is |P_0| (+ halo) + sum_l |P_l|, while the
// algorithmic bytes of the reference's level-by-level pass
// (sum_l |P_{l-1}| + |P_l|) are larger.
//
// Per output quad: one 8-byte window of each of the two source rows (one
// dword pair each), v_perm_b32 spreads each pixel's tap pair into 16-bit
// lanes and v_dot2_u32_u16 applies (ialpha0, ialpha1) -- the exact
// horizontal sum -- then the vertical rounding.  No saturation is needed: with non-negative
// Q11 weights summing to 2048 (+-1), every intermediate is in range
// (h <= 255*2048; the SIMD-path sum of the two >>16 products <= 1020).
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

#ifndef PYR_PROBE
#define PYR_PROBE 0  // timing probes for tuning only (tools/pyr_variants.sh): bit 0 = no level-0 loads, bit 2 = level 1 only, bit 3 = phase stamps; 0 = the product
#endif
#ifndef PYR_THREADS
#define PYR_THREADS 1024
#endif
constexpr int kPyrThreads = PYR_THREADS;

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

#if PYR_PROBE & 8
// diagnostic build only: per-block phase stamps (never read by the kernel)
__device__ unsigned long long g_pyr_stamps[8192 * 10];
__device__ __forceinline__ void pyr_stamp(int slot) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_pyr_stamps[blockIdx.x * 10 + slot] = t;
}
#define PYR_STAMP(i) pyr_stamp(i)
__device__ unsigned long long g_pyr_wave[8192 * 8 * 16];
#else
#define PYR_STAMP(i) ((void)0)
#endif

// 24 x 24 -> high 32 bits of the 48-bit product (v_mul_hi_u32_u24); both
// operands must be < 2^24
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

// out.byte[K] = s >> 2, other bytes preserved (SDWA destination select)
template <int K>
__device__ __forceinline__ void put_byte_shr2(uint32_t& out, uint32_t s) {
    static_assert(K >= 1 && K <= 3, "byte 0 is written by a plain shift");
    if (K == 1)
        asm("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(out) : "v"(s));
    else if (K == 2)
        asm("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(out) : "v"(s));
    else
        asm("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(out) : "v"(s));
}

// One level's band rows [r0, r1).  Thread layout: quad column q of 4 output
// pixels x row group rg walking rows r0+rg, r0+rg+rgroups, ..., so the
// column taps stay in registers for the whole level.  s_rows[r - r0] = (LDS
// offset of source row y0, of y1, ibeta0 << 12, ibeta1 << 12).
//
// Column taps per quad (ptab, 3 x int4), two layouts chosen for the whole
// pyramid on the host (Geom::pyr_win; the kernel is instantiated for each):
//  * window (WIN): all eight taps of the quad lie in one dword-aligned 8-byte
//    window of the source row (always true for scale factors <= 4/3):
//    (lo, wt0, wt1, wt2), (wt3, sel0, sel1, sel2), (sel3, -, -, -) -- one
//    ds_read2_b32 per source row serves the whole quad;
//  * pairs: (lo0, wt0, lo1, wt1), (lo2, wt2, lo3, wt3), (sel0..3) with lo_k
//    the dword pair holding taps sx_k, sx_k + 1.
// sel = the v_perm_b32 selector spreading a pixel's two taps into 16-bit
// lanes, wt = (ialpha0, ialpha1); v_dot2_u32_u16 forms the exact horizontal
// sum.  Rows are padded so reading past a row end is safe.
//
// Vertical pass, VResizeLinearVec_32s8u: ((h0>>4)*b0 >> 16) + ((h1>>4)*b1 >>
// 16) + 2 >> 2, each term as mulhi24(h & ~15, b << 12) = (16 (h>>4) b 2^12)
// >> 32.  h <= 255 * 2049 < 2^24 and b << 12 <= 2049 << 12 < 2^24.
//
// The last quad of every row is exactly the scalar tail (simd_end = 4 *
// (quads - 1), checked on the host; or there is no tail when w is a multiple
// of 16); its threads get a wave of their own (quad_taps).
// The source bytes one output row of a quad needs: rows y0 (a) and y1 (b),
// one dword pair per row (WIN) or per pixel.
// Horizontal pass of one source row for the quad: h[k] = the exact Q11 sum
// of pixel k's two taps (HResizeLinear), from the row at LDS offset `row`.
struct H4 {
    uint32_t h[4];
};

template <bool WIN>
__device__ __forceinline__ H4 hrow(const uint8_t* const (&col)[4], const uint32_t (&wt)[4], const uint32_t (&sel)[4],
                                   int row) {
    H4 r;
    uint32_t w[WIN ? 2 : 8];
#pragma unroll
    for (int k = 0; k < (WIN ? 1 : 4); ++k) {
        const uint32_t* a = reinterpret_cast<const uint32_t*>(col[k] + row);
        w[2 * k] = a[0];
        w[2 * k + 1] = a[1];
    }
#if PYR_PROBE & 16
    // timing probe: half the horizontal work (pixels 2, 3 reuse 0, 1)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#else
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#endif
        const int j = WIN ? 0 : 2 * k;
        const uint32_t p = __builtin_amdgcn_perm(w[j + 1], w[j], sel[k]);
        r.h[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p), __builtin_bit_cast(us2, wt[k]), 0u, false);
    }
#if PYR_PROBE & 16
    r.h[2] = r.h[0] ^ 1; r.h[3] = r.h[1] ^ 1;
#endif
    return r;
}

// Vertical pass of one output quad from its two source rows' sums.
template <bool TAIL>
__device__ __forceinline__ uint32_t vert(const H4& h0, const H4& h1, int4 yr) {
    uint32_t out;
    if (!TAIL) {
        const uint32_t B0 = (uint32_t)yr.z & 0xFFFFFFu, B1 = (uint32_t)yr.w & 0xFFFFFFu;
        uint32_t sum[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            sum[k] = mulhi24(h0.h[k] & 0xFFFFF0u, B0) + mulhi24(h1.h[k] & 0xFFFFF0u, B1) + 2u;
        out = sum[0] >> 2;
        put_byte_shr2<1>(out, sum[1]);
        put_byte_shr2<2>(out, sum[2]);
        put_byte_shr2<3>(out, sum[3]);
    } else {  // FixedPtCast<int, uchar, 22>: (S0*b0 + S1*b1 + 2^21) >> 22, < 2^31 (S < 2^24, b < 2^12)
        const uint32_t b0 = (uint32_t)yr.z >> 12, b1 = (uint32_t)yr.w >> 12;
        out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            out |= ((__umul24(h0.h[k], b0) + __umul24(h1.h[k], b1) + (1u << 21)) >> 22) << (8 * k);
    }
    return out;
}

// A thread's quad of one level: which quad and row group, and its column
// taps, loaded one level ahead (before the barrier that ends the previous
// level) so the table read's latency is hidden by the barrier wait.
struct QuadTaps {
    int4 a, b, c;
    int q, rg;
    int mode;  // 0 idle, 1 vector quad, 2 tail quad
};

// Thread layout of a level: vector quads fill threads [0, qmain * rgroups)
// (row group rg = t / qmain, rows rg, rg + rgroups, ...); the tail quad of
// every row goes to the wave starting at tail_base (lane = row, rows lane,
// lane + 64, ...) -- the tail formula then never shares a wave with the
// vector one, no wave runs both loops, and the tail wave needs one pass for
// bands up to 64 rows.
__device__ __forceinline__ QuadTaps quad_taps(const LevelGeom& V, const int4* __restrict__ ptab) {
    QuadTaps tp;
    const int t = threadIdx.x;
    tp.mode = 0;
    tp.q = 0;
    tp.rg = 0;
    if (t < V.qmain * V.rgroups) {
        tp.rg = (int)__umulhi((uint32_t)t, V.quad_magic);
        tp.q = t - tp.rg * V.qmain;
        tp.mode = 1;
    } else if (t >= V.tail_base && t < V.tail_base + 64 && 4 * V.qmain < V.w) {
        tp.rg = t - V.tail_base;
        tp.q = V.qmain;
        tp.mode = 2;
    }
    if (tp.mode) {
        const int4* pt = ptab + V.ptab_offset + 3 * tp.q;
        tp.a = pt[0];
        tp.b = pt[1];
        tp.c = pt[2];
    }
    return tp;
}

template <bool TAIL, bool WIN>
__device__ __forceinline__ void resize_rows(const uint8_t* __restrict__ lds, const LevelGeom& V, const QuadTaps& tp,
                                            int r0, int r1, int own0, int own1, const int4* __restrict__ s_rows,
                                            uint8_t* __restrict__ lds_dst, uint8_t* __restrict__ hbm_dst) {
    const int4 ta = tp.a, tb = tp.b, tc = tp.c;
    const int q = tp.q;
    const uint8_t* col[4];
    uint32_t wt[4], sel[4];
    if (WIN) {
        col[0] = col[1] = col[2] = col[3] = lds + ta.x;
        wt[0] = ta.y; wt[1] = ta.z; wt[2] = ta.w; wt[3] = tb.x;
        sel[0] = tb.y; sel[1] = tb.z; sel[2] = tb.w; sel[3] = tc.x;
    } else {
        col[0] = lds + ta.x; col[1] = lds + ta.z; col[2] = lds + tb.x; col[3] = lds + tb.z;
        wt[0] = ta.y; wt[1] = ta.w; wt[2] = tb.y; wt[3] = tb.w;
        sel[0] = tc.x; sel[1] = tc.y; sel[2] = tc.z; sel[3] = tc.w;
    }
    auto store = [&](int r, uint32_t out) {
        // bytes past V.w land in the row padding (LDS pitch and HBM pitch are
        // multiples of 4 and 16)
        if (lds_dst) *reinterpret_cast<uint32_t*>(lds_dst + (uint32_t)((r - r0) * V.lds_pitch + 4 * q)) = out;
        if (r >= own0 && r < own1) *reinterpret_cast<uint32_t*>(hbm_dst + (uint32_t)(r * V.pitch + 4 * q)) = out;
    };
    if (TAIL) {  // one row per lane (tail wave)
        for (int r = r0 + tp.rg; r < r1; r += 64) {
            const int4 y = s_rows[r - r0];
            store(r, vert<true>(hrow<WIN>(col, wt, sel, y.x), hrow<WIN>(col, wt, sel, y.y), y));
        }
        return;
    }
    // Row groups own pairs of consecutive output rows: (r, r+1) read source
    // rows (y0, y0+1) and (y0', y0'+1) with y0' = y0 + 1 for most pairs of a
    // ~1.2x downscale, so the shared source row's horizontal sums are
    // computed once (3 source rows per 2 output rows instead of 4).
    for (int r = r0 + 2 * tp.rg; r < r1; r += 2 * V.rgroups) {
        const bool two = r + 1 < r1;
        const int4 ya = s_rows[r - r0];
        const int4 yb = s_rows[(two ? r + 1 : r) - r0];
        const H4 hA = hrow<WIN>(col, wt, sel, ya.x);
        const H4 hB = hrow<WIN>(col, wt, sel, ya.y);
        H4 hC, hD;
        if (yb.x == ya.y) hC = hB; else hC = hrow<WIN>(col, wt, sel, yb.x);
        if (yb.y == ya.y) hD = hB; else hD = hrow<WIN>(col, wt, sel, yb.y);
        store(r, vert<false>(hA, hB, ya));
        if (two) store(r + 1, vert<false>(hC, hD, yb));
    }
}

template <bool WIN>
__device__ __forceinline__ void resize_band(const uint8_t* __restrict__ lds, const LevelGeom& V, const QuadTaps& tp,
                                            int r0, int r1, int own0, int own1, const int4* __restrict__ s_rows,
                                            uint8_t* __restrict__ lds_dst, uint8_t* __restrict__ hbm_dst) {
    if (tp.mode == 1)
        resize_rows<false, WIN>(lds, V, tp, r0, r1, own0, own1, s_rows, lds_dst, hbm_dst);
    else if (tp.mode == 2)
        resize_rows<true, WIN>(lds, V, tp, r0, r1, own0, own1, s_rows, lds_dst, hbm_dst);
}

template <bool WIN>
__global__ __launch_bounds__(kPyrThreads) void pyramid_kernel(Geom g, const int4* __restrict__ recs,
                                                              const int4* __restrict__ ptab,
                                                              const uint8_t* __restrict__ img0, size_t row0,
                                                              size_t frame0, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_pyr[];
    const int S = g.pyr_bands;
    const int f = blockIdx.x / S;
    const int band = blockIdx.x - f * S;
    const int L = g.nlevels;
    const int4* rec = recs + (size_t)band * g.pyr_rec_stride;
    int4* s_rec = reinterpret_cast<int4*>(s_pyr + g.pyr_lds_y);
    PYR_STAMP(0);
    QuadTaps tp = quad_taps(g.lv[1], ptab);
    // stage: this band's level-0 rows (16-byte loads; row0 is a multiple of
    // 16) and its record (band entries + per-row source offsets and y taps)
    {
        const int4 b = rec[0];
        const int v4 = (g.lv[0].w + 15) >> 4;
        const uint8_t* src = img0 + (size_t)f * frame0 + (size_t)b.x * row0;
        uint8_t* dst = s_pyr + g.pyr_lds_b;
        const int n = (b.y - b.x) * v4;
#if PYR_PROBE & 1
        if (n < 0)
#endif
        for (int i = threadIdx.x; i < n; i += kPyrThreads) {
            const int r = (int)__umulhi((uint32_t)i, g.lv[0].quad_magic);
            const int c = i - r * v4;
            *reinterpret_cast<uint4*>(dst + r * g.lv[0].lds_pitch + 16 * c) =
                *reinterpret_cast<const uint4*>(src + (size_t)r * row0 + 16 * c);
        }
        for (int i = threadIdx.x; i < g.pyr_rec_stride; i += kPyrThreads) s_rec[i] = rec[i];
    }
    __syncthreads();
    PYR_STAMP(1);
    int yoff = L;
#if PYR_PROBE & 4
    for (int l = 1; l < 2; ++l) {
#else
    for (int l = 1; l < L; ++l) {
#endif
        const LevelGeom& V = g.lv[l];
        const int4 bv = s_rec[l];  // need [x, y), owned [z, w); uniform
        const int bx = __builtin_amdgcn_readfirstlane(bv.x), by = __builtin_amdgcn_readfirstlane(bv.y);
        const int bz = __builtin_amdgcn_readfirstlane(bv.z), bw = __builtin_amdgcn_readfirstlane(bv.w);
        uint8_t* dst_lds = l + 1 < L ? s_pyr + ((l & 1) ? g.pyr_lds_a : g.pyr_lds_b) : nullptr;
        uint8_t* dst_hbm = pyr + V.offset + (size_t)f * V.frame_bytes;
        resize_band<WIN>(s_pyr, V, tp, bx, by, bz, bw, s_rec + yoff, dst_lds, dst_hbm);
        yoff += by - bx;
#if PYR_PROBE & 8
        {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if ((threadIdx.x & 63) == 0 && blockIdx.x < 8192) g_pyr_wave[(blockIdx.x * 8 + l) * 16 + threadIdx.x / 64] = t;
        }
#endif
        if (l + 1 < L) tp = quad_taps(g.lv[l + 1], ptab);
        __syncthreads();
        PYR_STAMP(1 + l);
    }
}

}  // namespace

int pyr_threads() { return kPyrThreads; }

hipError_t launch_pyramid(const Geom& g, int batch, const int4* recs, const int4* ptab, const uint8_t* img0,
                          size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream) {
    if (g.nlevels < 2) return hipSuccess;
    if (g.pyr_win)
        hipLaunchKernelGGL(pyramid_kernel<true>, dim3(g.pyr_bands * batch), dim3(kPyrThreads), g.pyr_lds_bytes,
                           stream, g, recs, ptab, img0, row0, frame0, pyr);
    else
        hipLaunchKernelGGL(pyramid_kernel<false>, dim3(g.pyr_bands * batch), dim3(kPyrThreads), g.pyr_lds_bytes,
                           stream, g, recs, ptab, img0, row0, frame0, pyr);
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

hipError_t pyramid_set_lds_limit(size_t bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel<false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace orbgpu
