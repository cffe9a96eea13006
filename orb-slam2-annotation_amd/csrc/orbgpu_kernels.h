// orbgpu_kernels.h -- host-side launchers of the HIP kernels (one per stage).
#pragma once

#include <vector>

#include "orbgpu_internal.h"

struct orbgpu_keypoint;
struct orbgpu_pack_desc;

namespace orbgpu {

// Fused pyramid pass (pyramid.hip) and its host plan (pyramid_plan.cpp).
struct PyrPlan {
    std::vector<int2> tab;  // row records of levels 1..L-1 (LDS offsets of the two source rows, ibeta pair), then per tick the row range of every (level, group)
    std::vector<int4> ent;  // per compute lane and entry: 6 int4 (pyramid.hip TickEnt)
};
// fills g.tk_* and g.lv[l].tk_* and the plan; ORBGPU_ERR_UNSUPPORTED when the
// geometry does not fit one block (message in orbgpu_last_error)
int plan_pyramid(Geom& g, const std::vector<int2>& ytab, const std::vector<int4>& ptab, int max_batch, PyrPlan& plan);
// LDS byte offset of row r of level l in its ring
int slot_offset(const Geom& g, int l, int r);
// the kernel's schedule run on the CPU with slot-ownership checks (levels[l]: w_l x h_l, tight)
int emulate_pyramid(const Geom& g, const std::vector<int2>& ytab, const PyrPlan& plan, const uint8_t* img, size_t row0,
                    std::vector<std::vector<uint8_t>>& levels);
// all pyramid levels 1..L-1 of `batch` frames (one block per frame)
// level-by-level pyramid for small batches (xtab / ytab: build_resize_tables per level)
hipError_t launch_pyramid_levels(const Geom& g, int batch, const int2* xtab, const int2* ytab, const uint8_t* img0,
                                 size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream);
// banded pyramid for small batches: g.bd_nb blocks per frame, every level of a
// row band in one launch (bands: per band and level (need_lo, need_hi,
// own_lo, own_hi) rows; level 0: the staged rows).  Fills g.bd_* and
// g.lv[l].bd_*; bd_nb = 0 when no band count fits the LDS budget.
void plan_pyramid_bands(Geom& g, const std::vector<int2>& ytab, std::vector<int4>& bands);
hipError_t launch_pyramid_bands(const Geom& g, int batch, const int4* bands, const int2* xtab, const int2* ytab,
                                const uint8_t* img0, size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream);
hipError_t launch_pyramid(const Geom& g, int batch, const int4* ents, const int2* tab, const uint8_t* img0,
                          size_t row0, size_t frame0, uint8_t* pyr, hipStream_t stream);
hipError_t pyramid_set_lds_limit(const Geom& g);

hipError_t launch_fast_cells(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                             const uint8_t* pyr, uint32_t* cand, int* cell_counts, int* err,
                             hipStream_t stream);

// level_from: blur levels level_from .. nlevels-1 only; 0 = every level (the debug API)
hipError_t launch_blur_levels(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                              const uint8_t* pyr, uint8_t* blur, hipStream_t stream, int level_from = 0);

size_t octree_lds_bytes(const Geom& g, int kcap, int ncap);
// levels [level0, level0 + nlev) in one launch: node arrays for ncap nodes,
// keys in LDS up to kcap (more: the HBM scratch path)
struct OctreeGroup {
    int level0, nlev, kcap, ncap;
};
hipError_t launch_octree(const Geom& g, int batch, const uint32_t* cand, const int* cell_counts,
                         uint32_t* gkeys, uint16_t* gknode, uint32_t* oct_out, int* oct_count,
                         int* err, const OctreeGroup* groups, int ngroups, int* trace, hipStream_t stream);

hipError_t launch_describe(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                           const uint8_t* pyr, const uint32_t* oct_out, const int* oct_count,
                           orbgpu_keypoint* kps, uint8_t* desc, int* counts, int kp_cap,
                           hipStream_t stream, int* err_word = nullptr, int* err_copy = nullptr, int f0 = 0);

// The stream form of SearchForInitialization (orbgpu_search_for_initialization_stream_device):
// with kps set, pair b takes F1 = frame b - 1 of the F1 arrays and pair 0 this frame
// (the one before the batch, read in place); kps == nullptr: pair b takes F1 frame b.
struct MatchFirstF1 {
    const orbgpu_keypoint* kps = nullptr;
    const uint8_t* desc = nullptr;
    const int* n = nullptr;
};

hipError_t launch_match_init(int batch, float minX, float maxX, float minY, float maxY,
                             const orbgpu_keypoint* kps1, const uint8_t* desc1, const int* n1, size_t stride1,
                             const orbgpu_keypoint* kps2, const uint8_t* desc2, const int* n2, size_t stride2,
                             float* prev_xy, int window, float nnratio, int flags,
                             int* matches12, int* nmatches, hipStream_t stream, size_t level0_bound = 0,
                             MatchFirstF1 first = MatchFirstF1());

hipError_t launch_hamming_pairs(const uint8_t* a, const uint8_t* b, int n, int* dist, hipStream_t stream);
hipError_t launch_pack_rows(int batch, int cap, int ntensors, const ::orbgpu_pack_desc* d, hipStream_t stream);
// nbytes (a multiple of 16, both pointers 16-byte aligned) from src to dst by a kernel;
// src may be pinned host memory
hipError_t launch_copy16(void* dst, const void* src, size_t nbytes, hipStream_t stream);
hipError_t launch_done_flag(unsigned long long* flag, unsigned long long v, hipStream_t stream);
// several such copies (each a multiple of 16 bytes, 16-byte aligned) in one launch
constexpr int kCopyList = 16;
struct CopyDesc16 {
    const void* src;
    void* dst;
    size_t bytes;
};
struct CopyList16 {
    CopyDesc16 d[kCopyList];
    int n;
};
hipError_t launch_copy16_list(const CopyList16& L, hipStream_t stream);

// error bits written to the device error word
enum : int {
    kErrCellCap = 1,     // FAST cell candidates overflowed cell_cap
    kErrNodeCap = 2,     // octree list exceeded ncap / ocap
    kErrKeyCap = 4,      // octree key count exceeded the scratch region
    kErrUnused8 = 8,     // (was the matcher capacity bit; now reported per pair)
    kErrSeqCap = 16,     // octree creation sequence overflow
};

}  // namespace orbgpu
