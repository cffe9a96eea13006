// describe.hip -- per-keypoint tail of ORBextractor::operator():
//   IC_Angle on the unblurred level (ORBextractor.cpp:79-106, :474-481),
//   computeOrbDescriptor (:110-149) on the blurred level (blur.hip) and the
//   final keypoint fields (:847-857, :1107-1115).
//
// One wave per keypoint slot.  The keypoint's raw 43x43 neighbourhood is
// staged in LDS once (dword loads); the GaussianBlur of the level
// (ORBextractor.cpp:1097-1098) is computed for the 37x37 patch rBRIEF reads,
// right there, with the blur's own arithmetic (blur_device.h) -- the whole
// blurred levels are never written to or read from HBM.  IC_Angle's disc
// comes from the same staged patch; moments by a 64-lane reduction; 256 tests
// as 4 wave ballots (bit t of the descriptor = test t = lane t%64 of ballot
// t/64).  sin/cos of the angle use
// the glibc-2.35 sinf/cosf restatement (fp64 polynomial), pinned bit-exact
// against libm over every float in [0, 6.3].
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"
#include "blur_device.h"
#include "group_sum.h"
#include "../../include/orbgpu.h"

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <type_traits>

namespace orbgpu {

namespace {

constexpr signed char kPattern[1024] = {
#include "bit_pattern_31.inc"
};
// the pattern as floats, one float4 (x0, x1, y0, y1) per test: a lane's test
// is one 16-byte load, no per-coordinate conversions, and the two points'
// x and y coordinates are already the packed pairs the rotation uses
struct PatternF { float4 t[256]; };
constexpr PatternF make_pattern_f() {
    PatternF p{};
    for (int i = 0; i < 256; ++i)
        p.t[i] = float4{(float)kPattern[4 * i], (float)kPattern[4 * i + 2], (float)kPattern[4 * i + 1],
                        (float)kPattern[4 * i + 3]};
    return p;
}
__constant__ PatternF c_pattern = make_pattern_f();

// umax of the 31-px disc (ORBextractor.cpp:456-471; the oracle builds it the
// reference's way)
constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};

// raw patch row pitch (bytes; the staged rows are 48 columns wide).  A/B:
// 52 spreads the row pass's six row chunks over distinct LDS banks (48: the
// chunk stride 84 dwords = 20 mod 32 banks, 2-way conflicts)
#ifndef ORBGPU_DESC_RPITCH
#define ORBGPU_DESC_RPITCH 48
#endif
constexpr int kRPitchC = ORBGPU_DESC_RPITCH;  // = kRPitch, needed by the table below
constexpr int kRWidth = 48;                   // staged columns per row: xb-4 .. xb+43
static_assert(kRPitchC % 4 == 0 && kRPitchC >= kRWidth, "raw pitch");
constexpr int kDiscWords = 31 * 9, kDiscLoads = (kDiscWords + 63) / 64;
// IC_Angle's disc as staged-patch words.  Disc row v = r - 15 (r < 31)
// covers the 4-aligned window columns c = 4q .. 4q+3 (q < 9) starting at
// xd = (cx - 15) & ~3, so byte b of word (r, q) is u = 4q + b - od - 15
// (od = cx - 15 - xd) and it is in the disc iff |u| <= umax[|v|].  Per
// (od, word): byte weights 1, c and v + 15 of the bytes in the disc (0
// outside), so Σp, Σc·p and Σ(v+15)·p are three v_dot4 accumulations, and
// the word's LDS offset from the disc's top-left word.  Words past the disc
// (idx >= 279) weigh 0.
struct DiscWord { uint32_t m1, mc, mv, off; };
struct DiscLut { DiscWord w[4][kDiscLoads * 64]; };
constexpr DiscLut make_disc_lut() {
    DiscLut L{};
    for (int od = 0; od < 4; ++od)
        for (int idx = 0; idx < kDiscWords; ++idx) {
            const int r = idx / 9, q = idx % 9, v = r - 15, d = kUmax[v < 0 ? -v : v];
            DiscWord e{0u, 0u, 0u, (uint32_t)(r * kRPitchC + 4 * q)};
            for (int b = 0; b < 4; ++b) {
                const int u = 4 * q + b - od - 15;
                if (u >= -d && u <= d) {
                    e.m1 |= 1u << (8 * b);
                    e.mc |= (uint32_t)(4 * q + b) << (8 * b);
                    e.mv |= (uint32_t)(v + 15) << (8 * b);
                }
            }
            L.w[od][idx] = e;
        }
    return L;
}
__constant__ DiscLut c_disc = make_disc_lut();
// words 256.. of each od (the fifth load) as a table of their own: its own
// scalar base, as global immediate offsets stop at 4095
struct DiscTail { DiscWord w[4][64]; };
constexpr DiscTail make_disc_tail() {
    DiscTail T{};
    const DiscLut L = make_disc_lut();
    for (int od = 0; od < 4; ++od)
        for (int i = 0; i < 64; ++i) T.w[od][i] = L.w[od][256 + i];
    return T;
}
__constant__ DiscTail c_disc_tail = make_disc_tail();
static_assert(kDiscLoads == 5, "the disc loads are four from c_disc and one from c_disc_tail");

// OpenCV 2.4 fastAtan2 (mathfuncs.cpp); explicit _rn ops: never contracted.
__device__ inline float fast_atan2(float y, float x) {
    const float k = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float ax = fabsf(x), ay = fabsf(y);
    const float eps = (float)2.220446049250313080847e-16;  // (float)DBL_EPSILON
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, eps));
        c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, eps));
        c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// glibc 2.35 sinf/cosf (sysdeps/ieee754/flt-32, FMA variant), |y| < 120.
struct SinCosTab { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; };
__constant__ SinCosTab c_sc[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

__device__ inline uint32_t top12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

__device__ inline float sc_poly(double x, double x2, const SinCosTab* p, int n) {
    if ((n & 1) == 0) {
        const double x3 = __dmul_rn(x, x2);
        const double s1 = __fma_rn(x2, p->s3, p->s2);
        const double x7 = __dmul_rn(x3, x2);
        const double s = __fma_rn(x3, p->s1, x);
        return __double2float_rn(__fma_rn(x7, s1, s));
    }
    const double x4 = __dmul_rn(x2, x2);
    const double c2 = __fma_rn(x2, p->c4, p->c3);
    const double c1 = __fma_rn(x2, p->c1, p->c0);
    const double x6 = __dmul_rn(x4, x2);
    const double c = __fma_rn(x4, p->c2, c1);
    return __double2float_rn(__fma_rn(x6, c2, c));
}

__device__ inline void glibc_sincosf(float y, float* sinp, float* cosp) {
    double x = y;
    if (top12(y) < top12(0x1.921FB6p-1f)) {
        if (top12(y) < top12(0x1p-12f)) { *sinp = y; *cosp = 1.0f; return; }
        const double x2 = __dmul_rn(x, x);
        *sinp = sc_poly(x, x2, &c_sc[0], 0);
        *cosp = sc_poly(x, x2, &c_sc[0], 1);
        return;
    }
    const double r = __dmul_rn(x, c_sc[0].hpi_inv);
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = __fma_rn(-(double)n, c_sc[0].hpi, x);
    const double s = c_sc[0].sign[n & 3];
    const SinCosTab* p = (n & 2) ? &c_sc[1] : &c_sc[0];
    const double xs = __dmul_rn(x, s), x2 = __dmul_rn(x, x);
    *sinp = sc_poly(xs, x2, p, n);
    *cosp = sc_poly(xs, x2, p, n ^ 1);
}

// wave total of an unsigned int, wave-uniform: 16-lane row sums on DPP
// (quad xor 1, xor 2, half mirror, mirror; update_dpp with bound_ctrl so the
// compiler folds each move into its add: one v_add_u32_dpp per step), then
// the row totals combined by row broadcasts (integer: order-free, exact)
__device__ inline uint32_t wave_total(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor1, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor2, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppHalfMirror, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppMirror, 0xF, 0xF, true);
    // the four row totals into row 3 (row_bcast:15 into rows 1, 3, then
    // row_bcast:31 into rows 2, 3), one readlane: 3 VALU instead of 4 readlanes
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

constexpr int kBPitch = 40;      // 37-px blurred rows, from a 4-aligned column
constexpr int kRPitch = kRPitchC;  // raw patch rows: columns xb-4 .. xb+43 (12 dwords)
constexpr int kRawWords = kPatch * (kRWidth / 4);   // 43 rows x 12 dwords
constexpr int kQuads = kBPitch / 4;                 // 10 output quads per blurred row
constexpr int kColChunks = (kBlur + 6) / 7;         // 6 chunks of <= 7 blurred rows

// The waves of a block process different keypoints in LDS regions of their
// own: stages are ordered within the wave, never with a block barrier.  A
// wave's DS instructions execute in order, so only the compiler must keep
// memory operations on their side (the asm's memory clobber) and the wave's
// own LDS operations are waited for; no VMEM wait (a workgroup-scope fence
// here waited for every outstanding global access, vmcnt(0), stores included).
__device__ inline void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline int reflect101(int p, int n) { return p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p); }

// keypoints per wave (1, 2 or 4): the wave stages and blurs them one after
// the other, then runs ONE orientation chain for all (lane k: keypoint k)
#ifndef ORBGPU_DESC_KEYS
#define ORBGPU_DESC_KEYS 1
#endif
constexpr int kKeysPerWave = ORBGPU_DESC_KEYS;

// Diagnostic builds (-DDESC_LDS_PROBE=mask; wrong results by design): the
// LDS accesses of the phases in `mask` are redirected to conflict-free
// addresses (consecutive dwords per lane, or a coprime stride) with the same
// instructions, so SQ_LDS_BANK_CONFLICT of a probe build against the product
// build is that phase's share of the bank conflicts, and its time what they
// cost.  1: the rBRIEF test reads, 2: the blur's row-pass reads, 4: the
// moments' disc reads, 8: the blurred-patch stores.
#ifndef DESC_LDS_PROBE
#define DESC_LDS_PROBE 0
#endif
static_assert(kKeysPerWave == 1 || kKeysPerWave == 2 || kKeysPerWave == 4, "ORBGPU_DESC_KEYS: 1, 2 or 4");

// Per-wave LDS: the raw 43x48 neighbourhood (re-staged per keypoint) and one
// blurred 37x40 patch per keypoint of the wave.
// Every region starts on a 16-byte boundary: lanes past the raw patch dump
// their 16-byte staging chunk into the keypoint's blur region with a 128-bit
// store, so each blur slot is padded to 16 bytes (1480 -> 1488 at the default
// pitches; one slot per wave by default, where the struct's alignment already
// rounded it up).
constexpr int kRawBytes = (kPatch * kRPitch + 15) & ~15;
constexpr int kBlurSlotBytes = (kBlur * kBPitch + 15) & ~15;
struct alignas(16) DescLds {
    uint8_t raw[kRawBytes];
    uint8_t blur[kKeysPerWave][kBlurSlotBytes];
};
static_assert(offsetof(DescLds, blur) % 16 == 0 && kBlurSlotBytes % 16 == 0, "16-byte dump stores into blur[k]");

#ifndef ORBGPU_DESC_SCALAR_COUNTS
#define ORBGPU_DESC_SCALAR_COUNTS 1
#endif

// A keypoint slot of a frame: its level, index within the level and output
// position; false when the slot is past the level's octree count.
struct KeyRef {
    int l, i, before, cx, cy;
    uint32_t key;
};

__device__ bool key_ref(const Geom& g, int f, int slot, int lane, const uint32_t* __restrict__ oct_out,
                        const int* __restrict__ oct_count, int* __restrict__ counts, KeyRef& K) {
    // level and index of the slot: one scalar load; the frame's per-level
    // counts on lanes 0..15 (each 16-lane row holds them all), prefix sums by
    // DPP row shifts, the values this slot needs read out of lane l / 15
    // the three loads (slot table entry, the slot's key, the frame's per-level
    // counts) are independent: issued together, waited for once (the empty asm
    // uses them all, so the compiler can neither sink the key's load behind the
    // count test nor wait for each load in turn).  A slot past its level's
    // count reads a stale key that is never used; the counts record has
    // kOcStride = 16 entries, so every lane's read is in bounds.
    uint32_t se = g.slot_tab[slot];
    uint32_t key = oct_out[(size_t)f * g.slots_frame + slot];
#if ORBGPU_DESC_SCALAR_COUNTS
    // the frame's per-level counts as scalar loads (one s_load_dwordx16), the
    // level's start and count and the frame total by scalar adds: no VALU
    // (the vector form took a lane load, four DPP adds and the readlanes)
    (void)lane;
    se = (uint32_t)__builtin_amdgcn_readfirstlane((int)se);
    key = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
    const int l = (int)(se & 15u), i = (int)(se >> 4);
    const int* cr = oct_count + (size_t)f * kOcStride;
    int cv[kMaxLevels];  // all kOcStride entries (in bounds): one wide scalar load, then masked
#pragma unroll
    for (int j = 0; j < kMaxLevels; ++j) cv[j] = cr[j];
    int before = 0, mine = 0, total = 0;
#pragma unroll
    for (int j = 0; j < kMaxLevels; ++j) {
        const int cj = j < g.nlevels ? cv[j] : 0;
        before += j < l ? cj : 0;
        mine = j == l ? cj : mine;
        total += cj;
    }
    if (slot == 0 && lane == 0) counts[f] = total;
#else
    const int ll = lane & 15;
    int c = oct_count[(size_t)f * kOcStride + ll];
    se = (uint32_t)__builtin_amdgcn_readfirstlane((int)se);
    key = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
    asm volatile("" ::"s"(se), "s"(key), "v"(c));
    c = ll < g.nlevels ? c : 0;
    const int l = (int)(se & 15u), i = (int)(se >> 4);
    int sc = c;
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x111, 0xF, 0xF, true);  // row_shr:1
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x112, 0xF, 0xF, true);  // row_shr:2
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x114, 0xF, 0xF, true);  // row_shr:4
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x118, 0xF, 0xF, true);  // row_shr:8
    const int mine = __builtin_amdgcn_readlane(c, l);
    const int before = __builtin_amdgcn_readlane(sc, l) - mine;
    if (slot == 0 && lane == 0) counts[f] = __builtin_amdgcn_readlane(sc, 15);
#endif
    if (i >= mine) return false;
    K.l = l;
    K.i = i;
    K.before = before;
    K.key = key;
    K.cx = key_x(K.key) + kBorder;
    K.cy = key_y(K.key) + kBorder;
    return true;
}

// Stage the neighbourhood, IC_Angle's moments, the blurred patch into S.blur;
// returns (m10, m01), wave-uniform.
// rawbuf: the wave's raw-neighbourhood buffer (kPatch rows of kRPitch bytes).
__device__ int2 describe_patch(const Geom& g, int f, const KeyRef& K, int lane, uint8_t* rawbuf, uint8_t* blur_out,
                               const uint8_t* __restrict__ img0, size_t row0, size_t frame0,
                               const uint8_t* __restrict__ pyr) {
    const int l = K.l, cx = K.cx, cy = K.cy;
    const LevelGeom& L = g.lv[l];
#ifdef DESC_PROBE_SAMEFRAME
    // latency probe (diagnostic build only; wrong results): every keypoint's
    // neighbourhood comes from frame 0's level 0 (L2-resident)
    const uint8_t* raw = img0;
    const size_t rp = row0;
    (void)frame0;
#else
    const uint8_t* raw = l == 0 ? img0 + (size_t)f * frame0 : pyr + L.offset + (size_t)f * L.frame_bytes;
    const size_t rp = l == 0 ? row0 : (size_t)L.pitch;
#endif

    // 1. Stage the raw neighbourhood: rows cy-21 .. cy+21, columns xb-4 ..
    // xb+43 (xb = the blurred patch's 4-aligned first column), reflected at
    // the level border (BORDER_REFLECT_101 of GaussianBlur on the level
    // clone, ORBextractor.cpp:1097-1098).  Dwords inside the level are one
    // load each; a dword that crosses the border is assembled from reflected
    // bytes.  All loads of a lane are issued before any is stored.
    const int xb = (cx - kBlurR) & ~3, x0 = xb - 4;
    // a neighbourhood entirely inside the level (wave-uniform; most keypoints): three
    // 16-byte chunks per row, two loads per lane, no reflection
    if (x0 >= 0 && x0 + kRWidth <= L.w && cy - kPatchR >= 0 && cy + kPatchR < L.h) {
        constexpr int kChunks = kPatch * (kRWidth / 16);  // 129
        const uint8_t* top = raw + (size_t)(cy - kPatchR) * rp + x0;
        uint4 c[3];
        uint8_t* dst[3];
        // the dump for lanes past the patch: this keypoint's blurred patch,
        // written only after this staging
        uint8_t* const dump = blur_out;
        // r = idx / 3 by a 24-bit multiply (exact for idx < 4096), row offsets
        // by 24-bit multiplies (rp < 2^24: launcher check), unsigned 32-bit
        // offsets (no sign extension); lanes past the patch load its last row
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t idx = (uint32_t)(lane + 64 * k), r = __umul24(idx, 21846u) >> 16, q = idx - 3u * r;
            // chunk (r, q) at r * 48 + 16 q = 16 idx when the row pitch is 48 (three
            // chunks a row): no per-chunk multiply; chunks 0..127 (k = 0, 1) always
            // exist, so only k = 2 selects the dump (VALU-bound kernel: round 6)
            const uint32_t doff = kRPitch == 48 ? 16u * idx : __umul24(r, (uint32_t)kRPitch) + 16u * q;
            dst[k] = (k < 2 && 64 * 2 <= kChunks) || idx < (uint32_t)kChunks ? rawbuf + doff : dump;
            // the source offset r * rp + 16 q = r * (rp - 48) + 16 idx: one 24-bit
            // multiply-add (rp >= w >= 48 here), no quarter-rate v_mul_lo_u32 for
            // q; lanes past the patch load its last chunk (idx clamped to 128)
            const uint32_t idxc = k < 2 ? idx : min(idx, (uint32_t)kChunks - 1u), rc = __umul24(idxc, 21846u) >> 16;
            c[k] = load16_a4(top + (uint32_t)(__umul24(rc, (uint32_t)rp - 48u) + 16u * idxc));
        }
        // unconditional stores (lanes past the patch write into kDump): no
        // branch the loads could be sunk into
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if constexpr (kRPitch % 16 == 0) {
                *reinterpret_cast<uint4*>(dst[k]) = c[k];
            } else {
                uint32_t* d = reinterpret_cast<uint32_t*>(dst[k]);
                d[0] = c[k].x;
                d[1] = c[k].y;
                d[2] = c[k].z;
                d[3] = c[k].w;
            }
        }
    } else {
    constexpr int kLoads = (kRawWords + 63) / 64;
    uint32_t v[kLoads];
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
        const int idx = min(lane + 64 * k, kRawWords - 1), r = idx / 12, q = idx - r * 12;
        const uint8_t* row = raw + (size_t)reflect101(cy - kPatchR + r, L.h) * rp;
        const int col = x0 + 4 * q;
        if (col >= 0 && col + 3 < L.w) {
            v[k] = *reinterpret_cast<const uint32_t*>(row + col);
        } else {
            uint32_t w = 0;
            for (int j = 0; j < 4; ++j) w |= (uint32_t)row[reflect101(col + j, L.w)] << (8 * j);
            v[k] = w;
        }
    }
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
        const int idx = lane + 64 * k, r = idx / 12, q = idx - r * 12;
        if (idx < kRawWords) reinterpret_cast<uint32_t*>(rawbuf)[r * (kRPitch / 4) + q] = v[k];
    }
    }
    wave_sync();

    // 2. Intensity centroid (IC_Angle, ORBextractor.cpp:79-106) from the raw
    // patch: per disc word (c_disc: offset and byte weights for this od)
    // three v_dot4_u32_u8 accumulate Σp, Σc·p and Σ(v+15)·p; then
    // m10 = Σc·p - (od+15)Σp, m01 = Σ(v+15)·p - 15Σp.  Integer moments:
    // order-free, exact.
    const int xd = (cx - 15) & ~3, od = cx - 15 - xd;
    const uint8_t* disc = rawbuf + (kPatchR - 15) * kRPitch + (xd - x0);
    uint32_t sp = 0u, cp = 0u, vp = 0u;
    // uniform table bases + 32-bit lane offset: saddr loads, no per-load
    // 64-bit address arithmetic
    const __attribute__((address_space(1))) uint8_t* dtab =
        (const __attribute__((address_space(1))) uint8_t*)&c_disc.w[od][0];
    const __attribute__((address_space(1))) uint8_t* dtab4 =
        (const __attribute__((address_space(1))) uint8_t*)&c_disc_tail.w[od][0];
#pragma unroll
    for (int k = 0; k < kDiscLoads; ++k) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 t = *(const __attribute__((address_space(1))) u32x4*)((k < 4 ? dtab : dtab4) + 16u * (uint32_t)lane +
                                                                          1024u * (k % 4));
        const DiscWord e{t.x, t.y, t.z, t.w};
#if DESC_LDS_PROBE & 4
        const uint32_t w = *reinterpret_cast<const uint32_t*>(rawbuf + 4 * lane + 256 * k + (e.off & 0));
#else
        const uint32_t w = *reinterpret_cast<const uint32_t*>(disc + e.off);
#endif
        sp = __builtin_amdgcn_udot4(w, e.m1, sp, false);
        cp = __builtin_amdgcn_udot4(w, e.mc, cp, false);
        vp = __builtin_amdgcn_udot4(w, e.mv, vp, false);
    }
    // wave totals now (scalars): the blur below then has every VGPR
    // (the per-lane combinations first: two wave totals instead of three;
    // modulo-2^32 sums, exact since the totals fit)
    // (24-bit multiplies: sp <= 255 x 709 disc pixels)
    const int m10 = (int)wave_total(cp - __umul24((uint32_t)(od + 15), sp));
    const int m01 = (int)wave_total(vp - __umul24(15u, sp));

    // 3. Blur (blur_device.h, the arithmetic of blur.hip) of the 37x37 patch:
    // lane = (output quad q, chunk c of 7 blurred rows); row passes from the
    // raw patch in LDS, the column pass in registers, rounding per path (quad
    // columns x < 4*floor(w/4): the SIMD path).  No intermediate array, no
    // extra wave sync.
    const int simd_end = L.w & ~3;
    // c is the fastest lane index, so the chunk below a lane's is
    // the next lane: a lane runs the row pass of its chunk's first 8 raw rows
    // (7c .. 7c+7) and takes the 5 halo rows 7c+8 .. 7c+12 from lane + 1
    // (its rows 1..5) by whole-wave DPP shifts -- 8 row passes per 7 output
    // rows instead of 13.  Chunk 5 (rows 35..42) needs no halo: it outputs
    // rows 35 and 36 only.  All 64 lanes run the passes (lanes 60..63 repeat
    // quad 9 and store nothing), so every DPP source lane is active.
    // A patch whose every quad is on the SIMD path (xb + 36 < simd_end: all
    // but the keypoints at a level's right edge) takes a copy of the passes
    // that packs with v_cvt_pk_u8_f32 alone: with a per-lane path choice the
    // compiler evaluates both roundings and selects (16 VALU per output row).
    auto passes = [&](auto all_simd) {
        // lane / 6 by a 24-bit multiply (exact for lane < 64); LDS offsets as
        // 24-bit products (no quarter-rate v_mul_lo_u32 / v_mad_u64_u32)
        const int qq = (int)(__umul24((uint32_t)lane, 10923u) >> 16), c = lane - qq * kColChunks;
        const int q = min(qq, kQuads - 1), r0 = c * 7;
        const bool simd = xb + 4 * q < simd_end, store = qq < kQuads;
#if DESC_LDS_PROBE & 2
        const uint32_t raw0 = 12u * (uint32_t)lane + 0u * (uint32_t)(r0 + q);
#else
        const uint32_t raw0 = __umul24((uint32_t)r0, (uint32_t)kRPitch) + 4u * (uint32_t)q;
#endif
        const uint32_t out0 = __umul24((uint32_t)r0, (uint32_t)kBPitch) + 4u * (uint32_t)q;
        auto row = [&](int k, blurdev::f32x2& lo, blurdev::f32x2& hi) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(rawbuf + raw0 + k * kRPitch);
            blurdev::Raw3 R3;
            R3.a = w[0];
            R3.b = w[1];
            R3.c = w[2];
            blurdev::row_pass_raw_shifted(R3, lo, hi);
        };
        auto from_next = [](blurdev::f32x2 v) {  // the value of lane + 1 (DPP wave_shl:1)
            return blurdev::f32x2{
                __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.x), 0x130, 0xF, 0xF, false)),
                __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.y), 0x130, 0xF, 0xF, false))};
        };
        blurdev::f32x2 wl[13], wh[13];  // local rows 0..12 (8..12 from lane + 1)
#pragma unroll
        for (int k = 0; k < 8; ++k) row(k, wl[k], wh[k]);
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            if (j >= 2) {  // halo row 6 + j = next lane's row j - 1, fetched just before its first use
                wl[6 + j] = from_next(wl[j - 1]);
                wh[6 + j] = from_next(wh[j - 1]);
            }
            if (store && r0 + j < kBlur) {
                const blurdev::f32x2 lo =
                    blurdev::col_pass(wl[j], wl[j + 1], wl[j + 2], wl[j + 3], wl[j + 4], wl[j + 5], wl[j + 6]);
                const blurdev::f32x2 hi =
                    blurdev::col_pass(wh[j], wh[j + 1], wh[j + 2], wh[j + 3], wh[j + 4], wh[j + 5], wh[j + 6]);
#if DESC_LDS_PROBE & 8
                *reinterpret_cast<uint32_t*>(blur_out + ((4 * lane + 256 * j) & 1023) + (out0 & 0)) =
                    all_simd ? blurdev::pack4_simd(lo, hi) : blurdev::pack4(lo, hi, simd);
#else
                *reinterpret_cast<uint32_t*>(blur_out + out0 + j * kBPitch) =
                    all_simd ? blurdev::pack4_simd(lo, hi) : blurdev::pack4(lo, hi, simd);
#endif
            }
        }
    };
    if (xb + 4 * (kQuads - 1) < simd_end)
        passes(std::true_type{});
    else
        passes(std::false_type{});
    return int2{m10, m01};
}

// rBRIEF (computeOrbDescriptor, ORBextractor.cpp:110-149) on the blurred
// patch with the keypoint's rotation, and the output record.
__device__ void describe_tests(const Geom& g, int f, const KeyRef& K, int lane, const uint8_t* blur, float4 rot,
                               orbgpu_keypoint* __restrict__ kps, uint8_t* __restrict__ desc, int kp_cap) {
    const LevelGeom& L = g.lv[K.l];
    const int ob = K.cx - kBlurR - ((K.cx - kBlurR) & ~3);
    const float angle = rot.x, a = rot.y, b = rot.z;
    unsigned long long words[4];
    // cvRound of the rotated offsets by the float magic-number add: r + 1.5*2^23
    // rounds r to an integer half-to-even (the magic is even, |r| <= 19), and
    // the sum's bits are 0x4B400000 + round(r), whose low 24 bits 0x400000 +
    // round(r) feed one v_mad_u32_u24: ry_bits * 40 + rx_bits - kBias is the
    // blurred-patch offset from the centre
    constexpr float kMagic = 12582912.f;
    constexpr uint32_t kBias = 0x400000u * (uint32_t)kBPitch + 0x4B400000u;
    const uint32_t cb = (uint32_t)(kBlurR * kBPitch + kBlurR + ob) - kBias;  // wave-uniform
    // both points of a test at once on packed f32 pairs: every product and sum
    // is one IEEE single operation per component, as the reference's scalar
    // float code (no contraction: -ffp-contract=off)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 va = {a, a}, vb = {b, b}, vm = {kMagic, kMagic};
#pragma unroll
    for (int rnd = 0; rnd < 4; ++rnd) {
        const float4 pt = c_pattern.t[rnd * 64 + lane];
        const f2 px = {pt.x, pt.y}, py = {pt.z, pt.w};  // (x0, x1), (y0, y1)
        const f2 fy = px * vb + py * va;                 // x*b + y*a
        const f2 fx = px * va - py * vb;                 // x*a - y*b
        const f2 my = fy + vm, mx = fx + vm;
        int val[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const uint32_t iy = __float_as_uint(pp ? my.y : my.x), ix = __float_as_uint(pp ? mx.y : mx.x);
#if DESC_LDS_PROBE & 1
            val[pp] = blur[(int)(4u * (uint32_t)lane + (uint32_t)pp + ((__umul24(iy, (uint32_t)kBPitch) + ix + cb) & 0x300u))];
#else
            val[pp] = blur[(int)(__umul24(iy, (uint32_t)kBPitch) + ix + cb)];
#endif
        }
        words[rnd] = __ballot(val[0] < val[1]);
    }

    const size_t o = (size_t)f * kp_cap + K.before + K.i;
    if (lane == 0) {
        // the four ballot words (scalars) from lane 0 as two 16-byte stores of
        // 64-bit pairs (v_mov_b64 from the SGPR pairs), where selecting
        // words[lane] on lanes 0..3 took 17 VALU
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        auto vmov64 = [](unsigned long long x) {  // one v_mov_b64 (the compiler moved the halves apart)
            unsigned long long v;
            asm("v_mov_b64 %0, %1" : "=v"(v) : "s"(x));
            return v;
        };
        u64x2* d = reinterpret_cast<u64x2*>(desc + o * 32);
        d[0] = u64x2{vmov64(words[0]), vmov64(words[1])};
        d[1] = u64x2{vmov64(words[2]), vmov64(words[3])};
        orbgpu_keypoint kp;
        const float fx = (float)K.cx, fy = (float)K.cy;
        kp.x = K.l == 0 ? fx : __fmul_rn(fx, L.scale);
        kp.y = K.l == 0 ? fy : __fmul_rn(fy, L.scale);
        kp.size = (float)L.size_i;
        kp.angle = angle;
        kp.response = (float)key_s(K.key);
        kp.octave = K.l;
        kp.class_id = -1;
        kps[o] = kp;
    }
}

// Diagnostic build (-DDESC_STAMPS): every 64th item's wave adds its phase
// durations (s_memtime cycles) to g_desc_stamps[phase], and [15] counts the
// sampled waves; tools/extract_stamps.py prints the per-wave means.
#ifdef DESC_STAMPS
__device__ unsigned long long g_desc_stamps[16];
#define DSTAMP(k) (stamp_on ? (ts[k] = __builtin_amdgcn_s_memtime()) : 0ull)
#else
#define DSTAMP(k) ((void)0)
#endif

// keypoints (waves) per block: 2 since round 5 (with the 256-keypoint matcher beside
// describe: 396.1k vs 394.3k frames/s, describe 0.487 vs 0.492 ms; 1: 396.3k; 8: slower;
// profiles/r05_notes_ab.txt r6g/r6h)
#ifndef ORBGPU_DESC_WAVES
#define ORBGPU_DESC_WAVES 2
#endif
constexpr int kDescWaves = ORBGPU_DESC_WAVES;

// One wave per (frame, slot) item, kDescWaves items per block.  Blocks are
// XCD-swizzled so one frame's keypoints (whose neighbourhoods overlap) are
// described on one XCD and its level rows are fetched into one L2.
__global__ __launch_bounds__(64 * kDescWaves) void describe_kernel(Geom g, int items, int f0,
                                                                   const uint8_t* __restrict__ img0, size_t row0,
                                                                   size_t frame0, const uint8_t* __restrict__ pyr,
                                                                   const uint32_t* __restrict__ oct_out,
                                                                   const int* __restrict__ oct_count,
                                                                   orbgpu_keypoint* __restrict__ kps,
                                                                   uint8_t* __restrict__ desc,
                                                                   int* __restrict__ counts, int kp_cap,
                                                                   int* __restrict__ err_word,
                                                                   int* __restrict__ err_copy) {
    __shared__ DescLds s_lds[kDescWaves];
    // single-frame path: the error word of this extraction (FAST / octree ran
    // before on the stream) moves into the output block and is cleared, so
    // the host needs no extra copy and memset launches
    if (err_copy && blockIdx.x == 0 && threadIdx.x == 0) *err_copy = atomicExch(err_word, 0);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: metadata in SGPRs
#if ORBGPU_DESC_SWIZZLE
    const int blk = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
#else
    const int blk = (int)blockIdx.x;
#endif
    const int item = blk * kDescWaves + wave;  // the wave's keypoint slots: kKeysPerWave consecutive ones
#ifdef DESC_STAMPS
    const bool stamp_on = (item & 63) == 0;
    unsigned long long ts[8] = {};
#endif
    DSTAMP(0);
    const int per_frame = (g.slots_frame + kKeysPerWave - 1) / kKeysPerWave;
    const int fi = kKeysPerWave == 1 ? (int)udiv40((uint32_t)item, g.slots_magic) : item / per_frame;
    const int slot0 = (item - fi * per_frame) * kKeysPerWave;
    const int f = f0 + fi;  // frame of the whole batch (a chunk's launch starts at frame f0)
    if (item >= items) return;
    KeyRef K[kKeysPerWave];
    bool valid[kKeysPerWave];
    int nvalid = 0;
#pragma unroll
    for (int k = 0; k < kKeysPerWave; ++k) {
        valid[k] = slot0 + k < g.slots_frame && key_ref(g, f, slot0 + k, lane, oct_out, oct_count, counts, K[k]);
        nvalid += valid[k];
    }
    if (nvalid == 0) return;
    DSTAMP(1);
    // Each keypoint in turn: raw neighbourhood -> moments -> its blurred patch
    // (the raw buffer is re-staged, so a wave sync before the next keypoint's
    // staging); then ONE orientation chain for all of them (lane k computes
    // keypoint k's: the same instructions as for one), then the tests.
    // (a rolled loop: one copy of the staging / blur code, so the register
    // budget is the one-keypoint kernel's)
    // keypoint k of the wave in a rolled loop (k wave-uniform: the selects
    // below are scalar)
    auto key_at = [&](int k, KeyRef& Kk) {
        int l = K[0].l, i = K[0].i, before = K[0].before, cx = K[0].cx, cy = K[0].cy;
        uint32_t key = K[0].key;
        bool v = valid[0];
#pragma unroll
        for (int j = 1; j < kKeysPerWave; ++j) {
            const bool h = k == j;
            l = h ? K[j].l : l;
            i = h ? K[j].i : i;
            before = h ? K[j].before : before;
            cx = h ? K[j].cx : cx;
            cy = h ? K[j].cy : cy;
            key = h ? K[j].key : key;
            v = h ? valid[j] : v;
        }
        Kk = KeyRef{l, i, before, cx, cy, key};
        return v;
    };
    int mx = 0, my = 0;
#pragma unroll 1
    for (int k = 0; k < kKeysPerWave; ++k) {
        KeyRef Kk;
        if (!key_at(k, Kk)) continue;
        if (k > 0) wave_sync();  // the previous keypoint's blur has read the raw buffer
        int lane_k = lane;
        asm volatile("" : "+v"(lane_k));  // per iteration: no lane-derived invariant is hoisted out (VGPRs 82 -> 50)
        const int2 mm = describe_patch(g, f, Kk, lane_k, s_lds[wave].raw, s_lds[wave].blur[k], img0, row0, frame0, pyr);
        if (kKeysPerWave == 1 || lane == k) {  // one keypoint: wave-uniform moments, uniform branches below
            mx = mm.x;
            my = mm.y;
        }
    }
    DSTAMP(2);
    // the orientation: fastAtan2 + sincosf on lane k for keypoint k (a serial
    // chain; measured in round 3: sharing it across a block's waves through LDS
    // and barriers was slower, 0.574 -> 0.593 ms -- within a wave it is free)
    const float ang = fast_atan2((float)my, (float)mx);
    float sa, ca;
    glibc_sincosf(__fmul_rn(ang, (float)(M_PI / 180.f)), &sa, &ca);
    wave_sync();  // blurred patches complete
    DSTAMP(3);
#pragma unroll 1
    for (int k = 0; k < kKeysPerWave; ++k) {
        KeyRef Kk;
        if (!key_at(k, Kk)) continue;
        const float a_k = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ang), k));
        const float c_k = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ca), k));
        const float s_k = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sa), k));
        describe_tests(g, f, Kk, lane, s_lds[wave].blur[k], float4{a_k, c_k, s_k, 0.f}, kps, desc, kp_cap);
    }
#ifdef DESC_STAMPS
    DSTAMP(4);
    if (stamp_on && lane == 0) {
        for (int k = 1; k <= 4; ++k) atomicAdd(&g_desc_stamps[k - 1], ts[k] - ts[k - 1]);
        atomicAdd(&g_desc_stamps[15], 1ull);
    }
#endif
}

}  // namespace

#ifdef DESC_STAMPS
extern "C" int orbgpu_debug_desc_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_desc_stamps), sizeof(g_desc_stamps)) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_desc_stamps), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

hipError_t launch_describe(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                           const uint8_t* pyr, const uint32_t* oct_out, const int* oct_count,
                           orbgpu_keypoint* kps, uint8_t* desc, int* counts, int kp_cap,
                           hipStream_t stream, int* err_word, int* err_copy, int f0) {
    if (row0 >= (1u << 24)) return hipErrorInvalidValue;  // row offsets by 24-bit multiplies
    if ((size_t)g.slots_frame * batch >= (1u << 24) || g.slots_frame >= (1 << 16))
        return hipErrorInvalidValue;  // udiv40's range
    const int items = (g.slots_frame + kKeysPerWave - 1) / kKeysPerWave * batch;  // waves (frames f0 .. f0+batch-1)
    const int blocks = (items + kDescWaves - 1) / kDescWaves;
    hipLaunchKernelGGL(describe_kernel, dim3(blocks), dim3(64 * kDescWaves), 0, stream, g, items, f0, img0, row0, frame0,
                       pyr, oct_out, oct_count, kps, desc, counts, kp_cap, err_word, err_copy);
    return hipGetLastError();
}

}  // namespace orbgpu
