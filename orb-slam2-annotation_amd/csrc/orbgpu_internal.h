// orbgpu_internal.h -- geometry and buffer layout shared by the host driver
// (orbgpu.cpp) and the HIP kernels.  Everything here is precomputed once per
// extractor on the host (it depends only on the frame size and the
// ORBextractor parameters) and handed to kernels by value.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orbgpu {

constexpr int kMaxLevels = 16;
// per-frame stride of the octree's per-level counts (oct_count): one 64-byte
// record per frame, so a wave loads all of a frame's counts in one scalar load
constexpr int kOcStride = kMaxLevels;
constexpr int kEdge = 19;              // EDGE_THRESHOLD (ORBextractor.cpp:76)
constexpr int kBorder = kEdge - 3;     // minBorderX/Y (ORBextractor.cpp:781)
#ifndef ORBGPU_BLUR_STRIP
#define ORBGPU_BLUR_STRIP 63
#endif
constexpr int kBlurStrip = ORBGPU_BLUR_STRIP;  // blur.hip: output rows per thread (a multiple of its 7-row window rotation)
constexpr int kMaxWin = 72;            // FAST cell window <= (wCell+6) x (hCell+6)
constexpr int kPatchR = 21;            // raw patch radius for blur+rBRIEF
constexpr int kPatch = 2 * kPatchR + 1;  // 43
constexpr int kBlurR = 18;             // blurred patch radius (13*sqrt2 rounded)
constexpr int kBlur = 2 * kBlurR + 1;    // 37

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8
// XCDs (each with its own L2), so blocks b and b+8 share an L2.  Kernels whose
// consecutive blocks read the same frame's pixels use the remapped index, so
// one frame's blocks land on one XCD and its level rows are fetched into one
// L2, not eight.  Bijective for any nwg (MI355X_MICROARCH / cdna guide T1);
// a pure speed choice, never needed for correctness.
#ifndef ORBGPU_FAST_SWIZZLE
// FAST: 2 = XCD-local runs of 8 consecutive cells within each window of 64
// blocks (fast.hip; round 6: FETCH_SIZE 1,077 -> 383 MB per 512-frame launch,
// fast_cells 0.499 -> 0.497 ms, r6b); 1 = the whole-grid remap below (measured
// slower for FAST: 0.547 -> 0.573 ms, round 4); 0 = block order
#define ORBGPU_FAST_SWIZZLE 2
#endif
#ifndef ORBGPU_DESC_SWIZZLE
#define ORBGPU_DESC_SWIZZLE 1
#endif
__device__ inline int xcd_swizzle(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// 16 bytes read from a 4-byte-aligned address (level rows staged from a
// dword-aligned column): declaring the alignment keeps the dwordx4 load
// well-defined instead of promising the 16 bytes of uint4.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ inline uint4 load16_a4(const uint8_t* p) {
    const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 / 4 bytes from any byte address of global memory (gfx950 serves unaligned
// vector loads in one instruction; FAST's column-shifted window staging).  The
// pointer is cast to the global address space: a pointer rebuilt from scalars
// (uniform_ptr) is generic, and its loads were flat_load (counted in lgkmcnt too,
// 64-bit vector addresses) instead of global_load with a scalar base.
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32_a1 __attribute__((aligned(1)));
__device__ inline uint4 load16_a1(const uint8_t* p) {
    const u32x4_a1 v = *(const __attribute__((address_space(1))) u32x4_a1*)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline uint32_t load4_a1(const uint8_t* p) { return *(const __attribute__((address_space(1))) u32_a1*)(p); }

// Candidate key packing (FAST output, octree input/output):
//   bits 0..10  x relative to minBorderX (level x - 16)
//   bits 11..21 y relative to minBorderY
//   bits 22..29 FAST score (cornerScore, <= 254)
__host__ __device__ inline uint32_t pack_key(int x, int y, int s) {
    return (uint32_t)x | ((uint32_t)y << 11) | ((uint32_t)s << 22);
}
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0x7FF); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 11) & 0x7FF); }
__host__ __device__ inline int key_s(uint32_t k) { return (int)(k >> 22); }

// level of index `i` given a packed table of level start indices (entry 0 is
// 0, entries past the last level INT_MAX): compares only, wave-uniform
__host__ __device__ inline int level_of(const int (&base)[kMaxLevels], int i) {
    int l = 0;
#pragma unroll
    for (int k = 1; k < kMaxLevels; ++k) l += i >= base[k];
    return l;
}

struct LevelGeom {
    int w, h;                 // level size (ComputePyramid, ORBextractor.cpp:1128)
    int pitch;                // row pitch in the pyramid buffer (levels >= 1)
    int simd_end;             // resize: VResizeLinearVec_32s8u coverage
    int xtab_offset;          // resize column taps (per output column) in the level-by-level tables
    size_t frame_bytes;       // bytes per frame of this level in the pyramid buffer
    size_t offset;            // byte offset of this level's region (levels >= 1)
    float scale;              // mvScaleFactor[l]
    int size_i;               // (int)(PATCH_SIZE * mvScaleFactor[l])
    int nfeat;                // mnFeaturesPerLevel[l]
    // FAST cells (ORBextractor.cpp:781-814)
    int max_bx, max_by;       // maxBorderX/Y
    int ncols, nrows, wcell, hcell;
    int cell_base;            // first cell index of this level within a frame
    int cell_cap;             // candidate slots per cell
    size_t cand_offset;       // u32 offset of this level's candidate slots in a frame
    // DistributeOctTree roots (ORBextractor.cpp:545-565)
    int nini;
    float hx;
    int ocap;                 // output slots (max list size)
    int out_offset;           // slot offset of this level within a frame
    // resize tables (levels >= 1)
    int ytab_offset;
    // fused pyramid pass (pyramid.hip, plan_pyramid in pyramid_plan.cpp)
    int qmain;                // quads per row on VResizeLinearVec_32s8u's vector path (the rest is the tail quad)
    int ptab_offset;          // int4 offset of this level's per-quad column taps (3 int4 per quad)
    int tk_ring;              // LDS byte offset of the ring holding this level's latest rows (levels 0..L-2)
    int tk_ring_rows;         // rows in that ring (levels >= 1: row y lives in slot y mod tk_ring_rows; level 0: tk_nc0 * tk_t0)
    int tk_pitch;             // LDS pitch of the ring rows: w rounded up to 16
    int tk_rec;               // int2 index of row 0's record in the plan table (levels >= 1)
    // banded pyramid pass (small batches, pyramid.hip pyramid_band_kernel):
    // this level's rows of a band live in LDS at bd_lds_off with pitch bd_pitch
    // (levels 0..L-2)
    int bd_lds_off, bd_pitch;
    uint32_t bd_qmagic;       // ceil(2^32 / quads): row index of a band element by a multiply-high
    // blurred level (all levels, incl. 0): same row pitch as the pyramid
    size_t blur_offset, blur_frame_bytes;
    int blur_tiles_x, blur_tile_base;   // blur work items: 4-column x 64-row strips
};

// n / d for the divisor whose udiv40_magic(d) is m: exact for n * d < 2^40
// (m * d - 2^40 < d); the launchers keep n < 2^24 and d < 2^16
__host__ __device__ constexpr uint64_t udiv40_magic(uint32_t d) { return ((1ull << 40) + d - 1) / d; }
__host__ __device__ inline uint32_t udiv40(uint32_t n, uint64_t m) { return (uint32_t)(((uint64_t)n * m) >> 40); }

struct Geom {
    int nlevels;
    // level lookup tables, packed so one scalar load brings a whole table and the
    // level of an index is a count of compares (no dependent loads per level):
    // entry l = lv[l].cell_base / lv[l].out_offset, INT_MAX past the last level
    int lvl_cell_base[kMaxLevels];
    int lvl_out_offset[kMaxLevels];
    // per-index lookup tables in HBM (built once per geometry), one scalar load
    // per wave: cell_tab[gc] = level | ci << 4 | cj << 18 for the frame's cell gc
    // (FAST), slot_tab[slot] = level | i << 4 for octree output slot `slot`
    // (describe)
    const uint32_t* cell_tab;
    const uint32_t* slot_tab;
    int width, height;
    int ini_th, min_th;
    int total_cells;          // cells per frame over all levels
    size_t cand_frame;        // u32 candidate slots per frame
    int slots_frame;          // octree output slots per frame (= sum ocap)
    // n / total_cells and n / slots_frame as ((u64)n * magic) >> 40 (udiv40):
    // scalar multiplies instead of a VALU reciprocal sequence per wave
    uint64_t cells_magic, slots_magic;
    int max_cells_level;
    int win_pitch, win_rows;  // FAST LDS tile: max over levels of (wCell+9) rounded to 4, (hCell+6)
    int blur_tiles_frame;     // blur tiles per frame over all levels
    int det_max;              // max FAST detection-region pixels of a cell (wCell x hCell)
    // fused pyramid pass (pyramid.hip): one block per frame walks the frame in
    // ticks; the plan (pyramid_plan.cpp) fixes every row's tick and LDS slot
    int tk_t0;                // level-0 rows per chunk (one chunk enters LDS per tick)
    int tk_k0;                // level-0 chunks
    int tk_ticks;             // ticks per frame
    int tk_rs;                // ranges per tick (tk_groups + 1; the last is empty)
    int tk_groups;            // row-group slots per tick (each level's regular groups, then its tail groups)
    int tk_cwaves, tk_pwaves; // compute waves, producer (level-0 loader) waves
    int tk_np;                // 16-byte level-0 loads per producer lane per chunk
    int tk_e;                 // entries (level, quad, group) per compute lane
    int tk_threads;           // 64 * (tk_cwaves + tk_pwaves)
    int tk_lds_tab;           // LDS byte offset of the plan table (row records, then ranges)
    int tk_tab_n;             // int2 entries in the plan table
    int tk_rng;               // u32 index of the range table within the plan table (one packed u32 per range)
    int tk_lds_bytes;         // LDS per block
    int tk_nc0;               // level-0 chunk runs in ring 0 (row r: run (r / tk_t0) % tk_nc0, row r % tk_t0 in it)
    int tk_cstride0;          // bytes per chunk run (tk_t0 rows at the level-0 pitch, padded to whole LDS-DMA pieces)
    // banded pyramid pass (plan_pyramid_bands): bd_nb row bands per frame, one
    // block each; 0 when the geometry does not fit (the level-by-level launches run)
    int bd_nb;
    int bd_lds_bytes;
    LevelGeom lv[kMaxLevels];
};

}  // namespace orbgpu
