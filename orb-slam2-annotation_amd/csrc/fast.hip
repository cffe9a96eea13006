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

namespace orbgpu {

namespace {

__device__ inline bool has_run9(uint32_t m16) {
    uint32_t m = m16 | (m16 << 16);
    uint32_t r = m & (m >> 1);   // runs >= 2
    r &= r >> 2;                 // >= 4
    r &= r >> 4;                 // >= 8
    r &= m >> 8;                 // >= 9
    return r != 0;
}

// arc strength: max over the 16 arcs of 9 of max(min d, -max d), d = v - ring
__device__ inline int arc_strength(const int d[16]) {
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mn2[k] = min(d[k], d[(k + 1) & 15]);
        mx2[k] = max(d[k], d[(k + 1) & 15]);
    }
    int mn4[16], mx4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mn4[k] = min(mn2[k], mn2[(k + 2) & 15]);
        mx4[k] = max(mx2[k], mx2[(k + 2) & 15]);
    }
    int best = -1000;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int mn9 = min(min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
        const int mx9 = max(max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
        best = max(best, max(mn9, -mx9));
    }
    return best;
}

// q = n / d for n < 65536, 0 < d < 256 via one multiply (m = ceil(2^24/d))
__device__ inline int fast_div(int n, uint32_t m) { return (int)(((uint32_t)n * m) >> 24); }

// The waves of a block work on different cells, so stages are ordered with
// a wave-local LDS fence, never a block barrier.
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Wave-level stream compaction: lanes holding `pred` append `v` to list[]
// after `n` entries (order = lane order); returns the new length.
__device__ inline int wave_append(bool pred, uint16_t v, uint16_t* list, int n, int lane) {
    const unsigned long long m = __ballot(pred);
    if (pred) list[n + __popcll(m & ((1ull << lane) - 1ull))] = v;
    return n + __popcll(m);
}

struct CellTiles {
    const uint8_t* win;  // staged window, pitch P, column c <-> level x = xa + c
    uint8_t* sc;         // FAST arc strength of corners, 0 elsewhere
    uint16_t* la;        // tile offsets passing the compass pre-test
    uint16_t* lb;        // tile offsets of corners (row-major order)
};

// FAST at threshold t on the cell's detection region: returns the number
// of corners, their tile offsets in lb[] (row-major) and scores in sc[].
// Stages are separated by wave compaction so each runs on dense lanes:
// compass pre-test on every pixel -> 16-pixel contiguity test on survivors
// -> arc strength on corners.
__device__ int fast_corners(const CellTiles& T, int P, int dw, int dh, int ox, int t, int lane) {
    const uint32_t mdw = (1u << 24) / (uint32_t)dw + 1u;
    int na = 0;
    for (int base = 0; base < dw * dh; base += 64) {
        const int idx = base + lane;
        bool pass = false;
        int off = 0;
        if (idx < dw * dh) {
            const int rr = fast_div(idx, mdw);
            off = (3 + rr) * P + 3 + ox + (idx - rr * dw);
            const uint8_t* p = T.win + off;
            const int v = p[0], lo = v - t, hi = v + t;
            const int c0 = p[3 * P], c4 = p[3], c8 = p[-3 * P], c12 = p[-3];
            const uint32_t dk = (c0 < lo) | ((c4 < lo) << 1) | ((c8 < lo) << 2) | ((c12 < lo) << 3);
            const uint32_t br = (c0 > hi) | ((c4 > hi) << 1) | ((c8 > hi) << 2) | ((c12 > hi) << 3);
            pass = ((dk & ((dk >> 1) | (dk << 3))) | (br & ((br >> 1) | (br << 3)))) & 15;
        }
        na = wave_append(pass, (uint16_t)off, T.la, na, lane);
    }
    wave_sync();
    const int ring_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int ring_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    int nb = 0;
    for (int base = 0; base < na; base += 64) {
        const int j = base + lane;
        bool corner = false;
        int off = 0;
        if (j < na) {
            off = T.la[j];
            const uint8_t* p = T.win + off;
            const int v = p[0], lo = v - t, hi = v + t;
            uint32_t dark = 0, bright = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int q = p[ring_dy[k] * P + ring_dx[k]];
                dark |= (uint32_t)(q < lo) << k;
                bright |= (uint32_t)(q > hi) << k;
            }
            corner = has_run9(dark) || has_run9(bright);
        }
        nb = wave_append(corner, (uint16_t)off, T.lb, nb, lane);
    }
    wave_sync();
    for (int j = lane; j < nb; j += 64) {
        const int off = T.lb[j];
        const uint8_t* p = T.win + off;
        const int v = p[0];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = v - p[ring_dy[k] * P + ring_dx[k]];
        T.sc[off] = (uint8_t)min(arc_strength(d), 255);  // >= t + 1 for a corner
    }
    wave_sync();
    return nb;
}

// 3x3 strict NMS among the corners (cv::FAST: non-corners and pixels outside
// the detection region count 0), emitted in lb order = row-major.
__device__ int nms_emit(const CellTiles& T, int P, int nb, int ox, int t, int lane, int iniX, int iniY,
                        uint32_t* out, int cap, int* err) {
    const int t1 = t + 1;
    int total = 0;
    for (int base = 0; base < nb; base += 64) {
        const int j = base + lane;
        bool keep = false;
        int s = 0, off = 0;
        if (j < nb) {
            off = T.lb[j];
            const uint8_t* q = T.sc + off;
            s = q[0];
            keep = true;
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) {
                    if (dx == 0 && dy == 0) continue;
                    const int v = q[dy * P + dx];
                    keep = keep && (s - 1 > (v >= t1 ? v - 1 : 0));
                }
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

constexpr int kCellWaves = 4;  // cells (one per wave) in flight per block

__global__ __launch_bounds__(64 * kCellWaves) void fast_cells_kernel(Geom g, int ncells_total,
                                                                     const uint8_t* __restrict__ img0, size_t row0,
                                                                     size_t frame0, const uint8_t* __restrict__ pyr,
                                                                     uint32_t* __restrict__ cand,
                                                                     int* __restrict__ cell_counts,
                                                                     int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int P = g.win_pitch, R = g.win_rows;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t per_wave = ((size_t)2 * P * R + 4 * (size_t)g.det_max + 15) & ~(size_t)15;
    uint8_t* ws = smem + wave * per_wave;
    CellTiles T;
    T.win = ws;
    T.sc = ws + P * R;
    T.la = reinterpret_cast<uint16_t*>(ws + 2 * P * R);
    T.lb = T.la + g.det_max;
    uint8_t* s_win = ws;

    // one cell per wave; waves of a block take consecutive cells of a frame
    const int item = blockIdx.x * kCellWaves + wave;
    if (item >= ncells_total) return;
    const int f = item / g.total_cells;
    const int gc = item - f * g.total_cells;
    int l = 0;
    while (l + 1 < g.nlevels && gc >= g.lv[l + 1].cell_base) ++l;
    const LevelGeom& L = g.lv[l];
    const int c = gc - L.cell_base;
    const int ci = c / L.ncols, cj = c - ci * L.ncols;
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
    const size_t pitch = l == 0 ? row0 : (size_t)L.pitch;

    // stage rows: dwords covering [xa, maxX), xa = iniX & ~3 (row pitch and
    // frame base are 16-byte aligned; maxX <= w - 16, so no over-read)
    const int xa = iniX & ~3, ox = iniX - xa;
    const int nd = (maxX - xa + 3) >> 2;
    const uint32_t mnd = (1u << 24) / (uint32_t)nd + 1u;
    for (int idx = lane; idx < nd * wh; idx += 64) {
        const int r = fast_div(idx, mnd), q = idx - r * nd;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(base + (size_t)(iniY + r) * pitch + xa + 4 * q);
        *reinterpret_cast<uint32_t*>(s_win + r * P + 4 * q) = v;
    }
    for (int idx = lane; idx < P * R / 4; idx += 64) reinterpret_cast<uint32_t*>(T.sc)[idx] = 0u;
    wave_sync();

    // detection region of cv::FAST on the window: rows [3, wh-3), cols [3, ww-3)
    const int dw = maxX - iniX - 6, dh = wh - 6;
    int total = 0;
    if (dw > 0 && dh > 0) {
        int nb = fast_corners(T, P, dw, dh, ox, g.ini_th, lane);
        total = nms_emit(T, P, nb, ox, g.ini_th, lane, iniX, iniY, out, L.cell_cap, err);
        if (total == 0) {  // ORBextractor.cpp:821-825: retry the cell at minThFAST
            for (int j = lane; j < nb; j += 64) T.sc[T.lb[j]] = 0;
            wave_sync();
            nb = fast_corners(T, P, dw, dh, ox, g.min_th, lane);
            total = nms_emit(T, P, nb, ox, g.min_th, lane, iniX, iniY, out, L.cell_cap, err);
        }
    }
    if (lane == 0) *cnt_out = min(total, L.cell_cap);
}

}  // namespace

hipError_t launch_fast_cells(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                             const uint8_t* pyr, uint32_t* cand, int* cell_counts, int* err,
                             hipStream_t stream) {
    const int items = g.total_cells * batch;
    const size_t per_wave = ((size_t)2 * g.win_pitch * g.win_rows + 4 * (size_t)g.det_max + 15) & ~(size_t)15;
    dim3 grid((items + kCellWaves - 1) / kCellWaves);
    hipLaunchKernelGGL(fast_cells_kernel, grid, dim3(64 * kCellWaves), per_wave * kCellWaves, stream, g, items,
                       img0, row0, frame0, pyr, cand, cell_counts, err);
    return hipGetLastError();
}

}  // namespace orbgpu
