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

constexpr int W = kMaxWin;

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

__global__ __launch_bounds__(64) void fast_cells_kernel(Geom g, const uint8_t* __restrict__ img0, size_t row0,
                                                        size_t frame0, const uint8_t* __restrict__ pyr,
                                                        uint32_t* __restrict__ cand, int* __restrict__ cell_counts,
                                                        int* __restrict__ err) {
    // LDS tile: the cell window, re-based to a 4-byte aligned column so rows
    // are fetched with dword loads; column c <-> level x = xa + c.
    __shared__ __attribute__((aligned(16))) uint8_t s_win[W * W];
    __shared__ uint8_t s_sc[W * W];
    const int lane = threadIdx.x;
    const int f = blockIdx.y;
    const int gc = blockIdx.x;
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
    const int ww = maxX - iniX, wh = maxY - iniY;
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
        *reinterpret_cast<uint32_t*>(s_win + r * W + 4 * q) = v;
    }
    for (int idx = lane; idx < W * W / 4; idx += 64) reinterpret_cast<uint32_t*>(s_sc)[idx] = 0u;
    __syncthreads();

    // detection region of cv::FAST on the window: rows [3, wh-3), cols [3, ww-3)
    const int dw = ww - 6, dh = wh - 6;
    const int tmin = min(g.ini_th, g.min_th);
    const int ring_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int ring_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    if (dw > 0 && dh > 0) {
        const uint32_t mdw = (1u << 24) / (uint32_t)dw + 1u;
        for (int idx = lane; idx < dw * dh; idx += 64) {
            const int rr = fast_div(idx, mdw);
            const int r = 3 + rr, x = 3 + ox + (idx - rr * dw);
            const uint8_t* p = s_win + r * W + x;
            const int v = p[0];
            // compass pre-test (ring 0/4/8/12): a 9-arc covers two adjacent ones
            const int c0 = p[3 * W], c4 = p[3], c8 = p[-3 * W], c12 = p[-3];
            const int lo = v - tmin, hi = v + tmin;
            const uint32_t dk = (c0 < lo) | ((c4 < lo) << 1) | ((c8 < lo) << 2) | ((c12 < lo) << 3);
            const uint32_t br = (c0 > hi) | ((c4 > hi) << 1) | ((c8 > hi) << 2) | ((c12 > hi) << 3);
            const uint32_t dk2 = dk & ((dk >> 1) | (dk << 3)), br2 = br & ((br >> 1) | (br << 3));
            if ((dk2 | br2) & 15) {
                int d[16];
                uint32_t dark = 0, bright = 0;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int q = p[ring_dy[k] * W + ring_dx[k]];
                    d[k] = v - q;
                    dark |= (uint32_t)(q < lo) << k;
                    bright |= (uint32_t)(q > hi) << k;
                }
                if (has_run9(dark) || has_run9(bright)) {
                    const int sc = arc_strength(d);  // >= tmin + 1 here
                    s_sc[r * W + x] = (uint8_t)min(sc, 255);
                }
            }
        }
    }
    __syncthreads();

    int total = 0;
    for (int pass = 0; pass < 2 && total == 0 && dw > 0 && dh > 0; ++pass) {
        const int t1 = (pass == 0 ? g.ini_th : g.min_th) + 1;
        for (int r = 3; r < 3 + dh; ++r) {
            for (int x0 = 3; x0 < 3 + dw; x0 += 64) {
                const int x = x0 + lane;
                bool keep = false;
                int s = 0;
                if (x < 3 + dw) {
                    const uint8_t* q = s_sc + r * W + x + ox;
                    s = q[0];
                    if (s >= t1) {
                        keep = true;
#pragma unroll
                        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (dx == 0 && dy == 0) continue;
                                const int nb = q[dy * W + dx];
                                const int nbv = nb >= t1 ? nb - 1 : 0;
                                keep = keep && (s - 1 > nbv);
                            }
                    }
                }
                const unsigned long long m = __ballot(keep);
                if (keep) {
                    const int pos = total + __popcll(m & ((1ull << lane) - 1ull));
                    if (pos < L.cell_cap)
                        out[pos] = pack_key(iniX + x - kBorder, iniY + r - kBorder, s - 1);
                    else
                        atomicOr(err, kErrCellCap);
                }
                total += __popcll(m);
            }
        }
    }
    if (lane == 0) *cnt_out = min(total, L.cell_cap);
}

}  // namespace

hipError_t launch_fast_cells(const Geom& g, int batch, const uint8_t* img0, size_t row0, size_t frame0,
                             const uint8_t* pyr, uint32_t* cand, int* cell_counts, int* err,
                             hipStream_t stream) {
    dim3 grid(g.total_cells, batch);
    hipLaunchKernelGGL(fast_cells_kernel, grid, dim3(64), 0, stream, g, img0, row0, frame0, pyr, cand,
                       cell_counts, err);
    return hipGetLastError();
}

}  // namespace orbgpu
