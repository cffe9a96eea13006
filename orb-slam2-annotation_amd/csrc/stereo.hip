// stereo.hip -- Frame::ComputeStereoMatches (Frame.cpp:540-748) for batches
// of rectified stereo pairs extracted by one orbgpu_extractor (left = frame
// 2p, right = frame 2p+1 of the last batch extraction), or for one pair
// extracted by two extractors (the stereo Frame's mpORBextractorLeft/Right).
//
// S 1024-thread blocks per pair (S chosen so the launch fills every CU; a
// pair's left keypoints are dealt to its S blocks, wave w of block b taking
// iL = 16 b + w + 16 S k):
//  A. the right keypoints go to LDS with their row band [minr, maxr]
//     (Frame.cpp:562-576: r = 2 * scale[octave], ceil/floor of y +- r) and
//     are bucketed by floor(y) (CSR over the image rows);
//  B. one wave per left keypoint: lanes walk the right keypoints of the rows
//     that can contain vL, apply the reference's row, octave and u filters
//     (:599-629) and reduce (Hamming, index) -- the reference keeps the first
//     strict minimum in increasing right-index order (:634); then the 11x11
//     SAD search over 11 shifts on the keypoint's pyramid level (:656-691):
//     lanes = (shift, window row) pairs, per-shift sums reduced in LDS;
//     parabola fit, disparity and depth (:697-729) on lane 0;
//  C. (stereo_median_kernel, one block per pair, after all S blocks) the
//     median cut (:734-747): the (M/2)-th smallest SAD of the accepted
//     matches by a two-pass 8-bit radix select in LDS, then every match with
//     SAD >= 1.5f*1.4f*median is reset to -1.
// A and B write uRight/depth and the accepted SAD (scratch) once per left
// keypoint; C rewrites the rejected ones.
//
// Spec decisions where the reference is undefined: row-band
// rows outside the image are skipped; a SAD window that would leave the
// level makes the keypoint unmatched; no accepted match -> no cut.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>

#include "../../include/orbgpu.h"
#include "orbgpu_internal.h"
#include "stereo_kernels.h"
#include "device_state.h"
#include "group_sum.h"

namespace orbgpu {

namespace {

constexpr int kStThreads = 1024;
constexpr int kStWaves = kStThreads / 64;

// wave minimum, wave-uniform: 16-lane row minima on DPP (quad xor 1, xor 2,
// half mirror, mirror: VALU lane moves), then the four row minima by readlane
// (six ds_bpermute round trips before)
__device__ __forceinline__ int wave_min(int v) {
    v = min(v, __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, kDppMirror, 0xF, 0xF, false));
    return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// the SAD windows of one left keypoint in its wave's LDS scratch: the left
// 11x11 window and the right 11x21 band (rows iv-5..iv+5) as the aligned
// dwords that hold them (left: 4 dwords a row, right: 7 in an 8-dword row)
constexpr int kWinL = 16, kWinR = 32, kWinBytes = 11 * (kWinL + kWinR);

__global__ __launch_bounds__(kStThreads) void stereo_kernel(StereoArgs a, int S) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_mem[];
    const int p = blockIdx.x / S, sub = blockIdx.x - p * S;
    const int fl = 2 * p, fr = 2 * p + 1;
    const int N = a.counts[fl], Nr = a.counts[fr];
    const int H = a.lvl_h[0];
    const int cap = a.cap;
    // LDS carve (host: stereo_lds_bytes)
    float4* s_r = reinterpret_cast<float4*>(s_mem);                     // x, y, minr, maxr << 8 | octave (as int bits)
    int* s_cnt = reinterpret_cast<int*>(s_r + cap);                      // H + 1 row starts
    int* s_cur = s_cnt + (H + 1);                                        // H fill cursors
    uint16_t* s_ent = reinterpret_cast<uint16_t*>(s_cur + H);            // cap entries
    int* s_scr = reinterpret_cast<int*>(s_ent + ((cap + 1) & ~1));      // per wave 128 SAD partials
    uint8_t* s_win = reinterpret_cast<uint8_t*>(s_scr + kStWaves * 128);  // per wave the SAD windows
    int* s_wsum = reinterpret_cast<int*>(s_win + kStWaves * kWinBytes);   // row-scan wave totals
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const orbgpu_keypoint* kl = a.kps + (size_t)fl * cap;
    const orbgpu_keypoint* kr = a.kps + (size_t)fr * cap;
    const uint8_t* dl = a.desc + (size_t)fl * cap * 32;
    const uint8_t* dr = a.desc + (size_t)fr * cap * 32;

    // A. right keypoints, row bands, buckets
    float* g_ur = a.uright + (size_t)p * cap;
    float* g_dp = a.depth + (size_t)p * cap;
    int* g_sad = a.sad + (size_t)p * cap;
    const int first = sub * kStWaves, stride = S * kStWaves;  // this block's left keypoints
    for (int i = tid; i <= H; i += kStThreads) s_cnt[i] = 0;
    for (int i = first + wave; i < N; i += stride)
        if (lane == 0) {
            g_ur[i] = -1.f;
            g_dp[i] = -1.f;
            g_sad[i] = -1;
        }
    __syncthreads();
    for (int i = tid; i < Nr; i += kStThreads) {
        const orbgpu_keypoint k = kr[i];
        const float r = __fmul_rn(2.0f, a.scale[k.octave]);
        const int maxr = (int)ceilf(__fadd_rn(k.y, r));
        const int minr = (int)floorf(__fsub_rn(k.y, r));
        s_r[i] = make_float4(k.x, k.y, __int_as_float(minr), __int_as_float((maxr << 8) | (k.octave & 0xFF)));
        const int row = min(max((int)k.y, 0), H - 1);
        atomicAdd(&s_cnt[row], 1);
    }
    __syncthreads();
    // exclusive scan over the rows, 1024 rows per pass (wave scans + wave totals)
    int carry = 0;
    for (int base = 0; base < H; base += kStThreads) {
        const int i = base + tid;
        const int x = i < H ? s_cnt[i] : 0;
        const int v = wave_incl_scan_dpp(x);
        if (lane == 63) s_wsum[wave] = v;
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int w = 0; w < kStWaves; ++w) {
                const int t = s_wsum[w];
                s_wsum[w] = acc;
                acc += t;
            }
            s_wsum[kStWaves] = acc;
        }
        __syncthreads();
        const int ex = carry + s_wsum[wave] + v - x;
        if (i < H) {
            s_cnt[i] = ex;
            s_cur[i] = ex;
        }
        carry += s_wsum[kStWaves];
        __syncthreads();
    }
    if (tid == 0) s_cnt[H] = carry;
    __syncthreads();
    for (int i = tid; i < Nr; i += kStThreads) {
        const int row = min(max((int)s_r[i].y, 0), H - 1);
        s_ent[atomicAdd(&s_cur[row], 1)] = (uint16_t)i;
    }
    __syncthreads();

    // B. one wave per left keypoint
    int* scr = s_scr + wave * 128;
    for (int iL = first + wave; iL < N; iL += stride) {
        const orbgpu_keypoint k = kl[iL];
        const int lvl = k.octave;
        const float vL = k.y, uL = k.x;
        const int vi = (int)vL;
        if (vi >= H) continue;
        const float minU = __fsub_rn(uL, a.max_d);
        const float maxU = __fsub_rn(uL, 0.0f);
        if (maxU < 0.f) continue;
        const int ra = max(vi - a.rr, 0), rb = min(vi + a.rr, H - 1);
        const int e0 = s_cnt[ra], e1 = s_cnt[rb + 1];
        // left descriptor (same for all lanes)
        const uint4 L0 = *reinterpret_cast<const uint4*>(dl + (size_t)iL * 32);
        const uint4 L1 = *reinterpret_cast<const uint4*>(dl + (size_t)iL * 32 + 16);
        int best = 0x7FFFFFFF;
        for (int e = e0 + lane; e < e1; e += 64) {
            const int iR = s_ent[e];
            const float4 r = s_r[iR];
            const int minr = __float_as_int(r.z), mo = __float_as_int(r.w);
            const int maxr = mo >> 8, o = mo & 0xFF;
            if (vi < minr || vi > maxr) continue;
            if (o < lvl - 1 || o > lvl + 1) continue;
            if (!(r.x >= minU && r.x <= maxU)) continue;
            const uint4 R0 = *reinterpret_cast<const uint4*>(dr + (size_t)iR * 32);
            const uint4 R1 = *reinterpret_cast<const uint4*>(dr + (size_t)iR * 32 + 16);
            const int d = __popc(L0.x ^ R0.x) + __popc(L0.y ^ R0.y) + __popc(L0.z ^ R0.z) + __popc(L0.w ^ R0.w) +
                          __popc(L1.x ^ R1.x) + __popc(L1.y ^ R1.y) + __popc(L1.z ^ R1.z) + __popc(L1.w ^ R1.w);
            best = min(best, (d << 16) | iR);
        }
        best = wave_min(best);
        const int bestDist = best == 0x7FFFFFFF ? 0x7FFF : (best >> 16);
        if (bestDist >= 100 || bestDist >= a.th_orb) continue;  // TH_HIGH start (:610), thOrbDist (:645)
        const int bestR = best & 0xFFFF;
        // subpixel match by correlation on level lvl
        const float uR0 = s_r[bestR].x;
        const float sf = a.inv_scale[lvl];
        const float su = roundf(__fmul_rn(uL, sf));
        const float sv = roundf(__fmul_rn(vL, sf));
        const float sr = roundf(__fmul_rn(uR0, sf));
        const int lw = a.lvl_w[lvl], lh = a.lvl_h[lvl];
        const int iu = (int)su, iv = (int)sv, ir = (int)sr;
        if (iv - 5 < 0 || iv + 6 > lh || iu - 5 < 0 || iu + 6 > lw) continue;  // spec: IL inside the level
        const float iniu = __fadd_rn(sr, 0.0f), endu = __fadd_rn(sr, 11.0f);   // scaleduR0 + L - w, + L + w + 1
        if (iniu < 0.f || endu >= (float)lw) continue;                            // :668-671
        if (ir - 10 < 0) continue;                                                 // spec: IR inside the level
        // the windows into LDS by aligned dword loads, 121 of them over the wave
        // (24 byte loads per lane before: the address unit set the kernel's
        // time); a dword is loaded only when it holds a window byte, so every
        // load lies inside its row (pitches are multiples of 4)
        uint8_t* wl = s_win + wave * kWinBytes;
        uint8_t* wr = wl + 11 * kWinL;
        {
            const uint8_t* lb = a.lvl_base[lvl] + (size_t)p * a.lvl_pair[lvl];
            const uint8_t* rb = a.lvl_base_r[lvl] + (size_t)p * a.lvl_pair[lvl];
            const size_t pitch = (size_t)a.lvl_pitch[lvl];
            const int lx0 = (iu - 5) & ~3, rx0 = (ir - 10) & ~3;
            for (int t = lane; t < 121; t += 64) {
                if (t < 44) {
                    const int row = t >> 2, c = t & 3;
                    if (lx0 + 4 * c <= iu + 5)
                        *reinterpret_cast<uint32_t*>(wl + row * kWinL + 4 * c) =
                            load4_a1(lb + (size_t)(iv - 5 + row) * pitch + lx0 + 4 * c);
                } else {
                    const int u = t - 44, row = u / 7, c = u - row * 7;
                    if (rx0 + 4 * c <= ir + 10)
                        *reinterpret_cast<uint32_t*>(wr + row * kWinR + 4 * c) =
                            load4_a1(rb + (size_t)(iv - 5 + row) * pitch + rx0 + 4 * c);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the windows are in LDS
            __builtin_amdgcn_wave_barrier();
            wl += (iu - 5) - lx0;  // byte 0 = column iu - 5 / ir - 10
            wr += (ir - 10) - rx0;
        }
        const int cL = wl[5 * kWinL + 5];
        for (int c = lane; c < 121; c += 64) {
            const int inc = c / 11 - 5, rr = c - (c / 11) * 11;
            const int cR = wr[5 * kWinR + inc + 10];
            const uint8_t* lrow = wl + rr * kWinL;
            const uint8_t* rrow = wr + rr * kWinR + inc + 5;
            int s = 0;
#pragma unroll
            for (int col = 0; col < 11; ++col) s += abs(((int)lrow[col] - cL) - ((int)rrow[col] - cR));
            scr[c] = s;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's partials are in LDS
        __builtin_amdgcn_wave_barrier();
        int dsum = 0;
        if (lane < 11)
            for (int rr = 0; rr < 11; ++rr) dsum += scr[lane * 11 + rr];
        __builtin_amdgcn_wave_barrier();
        // the 11 shift sums, wave-uniform (readlane: no LDS round trip)
        int dists[11];
#pragma unroll
        for (int j = 0; j < 11; ++j) dists[j] = __builtin_amdgcn_readlane(dsum, j);
        if (lane == 0) {
            int bestSad = 0x7FFFFFFF, bestInc = 0;
#pragma unroll
            for (int j = 0; j < 11; ++j)
                if ((float)dists[j] < (float)bestSad) {  // float dist vs int bestDist (:681)
                    bestSad = dists[j];
                    bestInc = j - 5;
                }
            if (bestInc != -5 && bestInc != 5) {
                const float d1 = (float)dists[bestInc + 4], d2 = (float)dists[bestInc + 5],
                            d3 = (float)dists[bestInc + 6];
                const float deltaR =
                    __fdiv_rn(__fsub_rn(d1, d3), __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2))));
                if (!(deltaR < -1.f || deltaR > 1.f)) {
                    float bestuR = __fmul_rn(a.scale[lvl], __fadd_rn(__fadd_rn(sr, (float)bestInc), deltaR));
                    float disparity = __fsub_rn(uL, bestuR);
                    if (disparity >= 0.f && disparity < a.max_d) {
                        if (disparity <= 0.f) {
                            disparity = 0.01f;
                            bestuR = (float)__dsub_rn((double)uL, 0.01);
                        }
                        g_dp[iL] = __fdiv_rn(a.bf, disparity);
                        g_ur[iL] = bestuR;
                        g_sad[iL] = bestSad;
                    }
                }
            }
        }
    }
}

// C. median cut (Frame.cpp:734-747) of pair p: (M/2)-th smallest accepted SAD
// (< 2^16) by a two-pass 8-bit radix select, then every accepted match with
// SAD >= 1.5f*1.4f*median is reset to -1.
constexpr int kMedThreads = 256;

__global__ __launch_bounds__(kMedThreads) void stereo_median_kernel(StereoArgs a) {
    __shared__ int s_hist[256];
    __shared__ int s_tot[4];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int N = a.counts[2 * p], cap = a.cap;
    const int* sad = a.sad + (size_t)p * cap;
    s_hist[tid] = 0;
    if (tid == 0) s_tot[0] = 0;
    __syncthreads();
    int m = 0;
    for (int i = tid; i < N; i += kMedThreads)
        if (sad[i] >= 0) {
            atomicAdd(&s_hist[(sad[i] >> 8) & 0xFF], 1);
            ++m;
        }
    atomicAdd(&s_tot[0], m);
    __syncthreads();
    const int M = s_tot[0];
    if (M == 0) return;
    if (tid == 0) {
        int k = M / 2, acc = 0, b = 0;
        for (; b < 256; ++b) {
            if (acc + s_hist[b] > k) break;
            acc += s_hist[b];
        }
        s_tot[1] = b;
        s_tot[2] = k - acc;
    }
    __syncthreads();
    const int hb = s_tot[1];
    s_hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += kMedThreads)
        if (sad[i] >= 0 && ((sad[i] >> 8) & 0xFF) == hb) atomicAdd(&s_hist[sad[i] & 0xFF], 1);
    __syncthreads();
    if (tid == 0) {
        int k = s_tot[2], acc = 0, b = 0;
        for (; b < 256; ++b) {
            if (acc + s_hist[b] > k) break;
            acc += s_hist[b];
        }
        s_tot[3] = (hb << 8) | b;
    }
    __syncthreads();
    const float median = (float)s_tot[3];
    const float th = __fmul_rn(1.5f * 1.4f, median);
    for (int i = tid; i < N; i += kMedThreads)
        if (sad[i] >= 0 && !((float)sad[i] < th)) {
            a.uright[(size_t)p * cap + i] = -1.f;
            a.depth[(size_t)p * cap + i] = -1.f;
        }
}

}  // namespace

size_t stereo_lds_bytes(int cap, int H) {
    return (size_t)cap * 16 + (size_t)(2 * H + 1) * 4 + (size_t)((cap + 1) & ~1) * 2 + (size_t)kStWaves * 128 * 4 +
           (size_t)kStWaves * kWinBytes + (kStWaves + 4) * 4;
}

// blocks per pair at most (ORBGPU_STEREO_SPLIT_MAX overrides): a single pair
// (the stereo Frame's call) is dealt to this many blocks, whose waves then
// take about 1200 / (16 S) left keypoints each
int stereo_split_max() {
    static const int v = [] {
        const char* s = std::getenv("ORBGPU_STEREO_SPLIT_MAX");
        const int x = s ? std::atoi(s) : 32;
        return std::max(1, std::min(x, 256));
    }();
    return v;
}

hipError_t launch_stereo(const StereoArgs& a, int npairs, hipStream_t stream) {
    if (npairs <= 0) return hipSuccess;
    // the SAD windows are staged by aligned dword loads: 4-byte aligned rows
    for (int l = 0; l < kMaxLevels; ++l)
        if (a.lvl_base[l] && ((((uintptr_t)a.lvl_base[l] | (uintptr_t)a.lvl_base_r[l] | a.lvl_pair[l]) & 3) ||
                              (a.lvl_pitch[l] & 3)))
            return hipErrorInvalidValue;
    const size_t lds = stereo_lds_bytes(a.cap, a.lvl_h[0]);
    // per-device state (device_state.h; the drop-in calls this per frame, from
    // any thread, on any device): the kernel's LDS limit only grows, the CU
    // count is read once per device
    static PerDeviceLdsLimit lds_limit;
    {
        const hipError_t e = lds_limit.ensure(reinterpret_cast<const void*>(&stereo_kernel), lds);
        if (e != hipSuccess) return e;
    }
    const int ncu = current_device_cus();
    // blocks per pair: at least two 1024-thread blocks per CU over the launch
    const int S = std::min(stereo_split_max(), std::max(1, (2 * ncu + npairs - 1) / npairs));
    hipLaunchKernelGGL(stereo_kernel, dim3(npairs * S), dim3(kStThreads), lds, stream, a, S);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(stereo_median_kernel, dim3(npairs), dim3(kMedThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace orbgpu
