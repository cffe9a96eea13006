/*
 * orbgpu_debug.h -- stage-level accessors of the last extraction, used by the
 * parity tests to localise a divergence (pyramid / FAST cells / octree).
 * Not part of the drop-in surface.  Synchronous; host outputs.
 */
#ifndef ORBGPU_DEBUG_H
#define ORBGPU_DEBUG_H

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* FAST candidates of (frame, level) in vToDistributeKeys order (cells
 * row-major, FAST order inside a cell), as (x, y, score) relative to
 * (minBorderX, minBorderY).  Returns the count (writes at most cap). */
int orbgpu_debug_level_candidates(orbgpu_extractor* ex, int frame, int level, int* xys, int cap);

/* DistributeOctTree output of (frame, level) in list order, (x, y, score)
 * relative to the border.  Returns the count (writes at most cap). */
int orbgpu_debug_level_octree(orbgpu_extractor* ex, int frame, int level, int* xys, int cap);

/* The blurred level (GaussianBlur 7x7, sigma 2, REFLECT_101, as
 * ORBextractor.cpp:1097-1098) of (frame, level) of the last extraction,
 * copied row by row into dst (dst_step >= level width). */
int orbgpu_debug_level_blur(orbgpu_extractor* ex, int frame, int level, uint8_t* dst, size_t dst_step);

/* Per-pass trace of the octree kernel for frame 0 (enable before extracting;
 * out: per level 512 ints = [passes, 0, then 8 ints per pass: inner, nL, C,
 * S, nToExpand, kstop, nkeys, N]). */
int orbgpu_debug_octree_trace(orbgpu_extractor* ex, int enable, int* out, int cap);

/* CPU run of the fused pyramid pass's plan (pyramid_plan.cpp), no GPU
 * needed: builds the extractor geometry for these parameters and executes the
 * kernel's tick schedule on the host -- same LDS ring slots, row records,
 * per-lane column entries and fixed-point arithmetic -- checking that every
 * read finds its source row in its slot and that no write of a tick lands in
 * a slot read during it.  Writes levels 1..nlevels-1 tightly packed (w_l x
 * h_l each) into out (out_bytes), and, if info != NULL, info[0..7] = {ticks,
 * rows per chunk, compute waves, producer waves, loads per producer lane,
 * entries per compute lane, LDS bytes per block, level-0 ring rows}. */
int orbgpu_debug_pyramid_emulate(int nfeatures, float scale_factor, int nlevels, int width, int height,
                                 const uint8_t* img, size_t img_step, uint8_t* out, size_t out_bytes, int* info);

/* The fused pyramid plan's work per tick (no GPU; tools/pyr_plan_cost.py):
 * rows[k * lanes + i] = output rows compute lane i (entry 0, then entry 1 at
 * i + lanes / entries) computes at tick k, lane_info[i] = level | tail << 8
 * (level 0: an idle lane), dims[0..3] = {ticks, lanes, compute waves,
 * entries per lane}.  rows / lane_info may be NULL (dims only). */
int orbgpu_debug_pyramid_plan_rows(int nfeatures, float scale_factor, int nlevels, int width, int height, int* rows,
                                   size_t rows_n, int* lane_info, size_t lanes_n, int* dims);

/* PnPsolver::qr_solve (PnPsolver.cpp:955-1047) as the GPU's EPnP runs it
 * (csrc/epnp.h qr_solve_6x4), on n independent 6 x 4 systems in HBM: A (n x
 * 24 doubles, row-major), b (n x 6), X (n x 4, read as the initial x: a
 * singular system leaves it untouched, as the reference does).  Asynchronous
 * on `stream`. */
int orbgpu_debug_qr_solve_6x4_device(const double* A, const double* b, double* X, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif
