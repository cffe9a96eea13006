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
#define ORBGPU_FAST_SWIZZLE 0  // measured slower for FAST (1.193 vs 1.129 ms per 512 frames)
#endif
#ifndef ORBGPU_DESC_SWIZZLE
#define ORBGPU_DESC_SWIZZLE 1
#endif
__device__ inline int xcd_swizzle(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

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

struct LevelGeom {
    int w, h;                 // level size (ComputePyramid, ORBextractor.cpp:1128)
    int pitch;                // row pitch in the pyramid buffer (levels >= 1)
    int simd_end;             // resize: VResizeLinearVec_32s8u coverage
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
    // fused pyramid pass (pyramid.hip)
    int lds_pitch;            // LDS row pitch: w rounded up to 4 (level 0: to 16)
    int qmain;                // quads per row on VResizeLinearVec_32s8u's vector path (the rest is the tail quad)
    int dbg_level;            // = level index (diagnostic builds)
    uint32_t quad_magic;      // ceil(2^32 / d): i / d = umulhi(i, magic); d = qmain (level 0: ceil(w/16))
    int ptab_offset;          // int4 offset of this level's per-quad column taps (3 int4 per quad)
    int rgroups;              // row groups of a pyramid block (pyramid.hip quad_taps)
    int tail_base;            // first thread of the tail quads (a wave boundary)
    int yrec_offset;          // first row record of this level (pyramid_frame_kernel)
    int brgroups;             // band kernel: row groups (quads 0..qmain-1 per group)
    uint32_t bquad_magic;     // band kernel: ceil(2^32 / qmain)
    int btail_base;           // band kernel: first thread of the tail wave (lane = row group)
    int pyr_run;              // stream/frame kernels: output rows per row group (a multiple of 4)
    int pyr_steps;            // stream kernel: 4-row steps per level (pyr_run / 4)
    int ystage_offset;        // stream kernel: first staged-row base of this level ([step][group])
    // blurred level (all levels, incl. 0): same row pitch as the pyramid
    size_t blur_offset, blur_frame_bytes;
    int blur_tiles_x, blur_tile_base;   // blur work items: 4-column x 64-row strips
};

struct Geom {
    int nlevels;
    int width, height;
    int ini_th, min_th;
    int total_cells;          // cells per frame over all levels
    size_t cand_frame;        // u32 candidate slots per frame
    int slots_frame;          // octree output slots per frame (= sum ocap)
    int max_cells_level;
    int win_pitch, win_rows;  // FAST LDS tile: max over levels of (wCell+9) rounded to 4, (hCell+6)
    int blur_tiles_frame;     // blur tiles per frame over all levels
    int det_max;              // max FAST detection-region pixels of a cell (wCell x hCell)
    // fused pyramid pass (pyramid.hip): frame bands per frame and LDS layout
    int pyr_bands;
    int pyr_lds_a, pyr_lds_b, pyr_lds_y, pyr_lds_bytes;  // odd levels, even levels (incl. 0), y taps
    int pyr_rec_stride;       // int4s per band record (band entries + per-row source offsets)
    int pyr_mode;             // 0: band kernel (levels through LDS), 1: frame kernel (levels through L2), 2: stream kernel
    int pyr_yrec_total;       // row records of all levels >= 1 (frame kernel)
    int pyr_ystage_total;     // stream kernel: staged-row bases of all levels
    int pyr_stage_bytes;      // stream kernel: bytes of one staging buffer (max over levels)
    int pyr_lds_stage;        // stream kernel: LDS offset of the staging buffers (after the row tables)
    LevelGeom lv[kMaxLevels];
};

}  // namespace orbgpu
