// pack.hip -- a batch's per-frame outputs trimmed to their counts and packed
// back to back, for delivery to the Tracking thread that consumes them
// (src/Tracking.cpp:280-317 reads one Frame's mvKeys / mDescriptors; the
// batch path keeps B frames x capacity rows in HBM).  One launch packs up to
// four row tensors (keypoints, descriptors, matches, ...): block (b, t) copies
// frame b's counts[t][b] rows of tensor t to the offset sum_{b' < b}
// counts[t][b'] -- a block-wide sum over the preceding frames' counts, then a
// dword copy (every row size here is a multiple of 4 bytes).  HBM-bound:
// each used row is read once and written once.
#include "../../include/orbgpu.h"
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

#include <algorithm>

namespace orbgpu {

namespace {

constexpr int kPackThreads = 256;

__global__ __launch_bounds__(kPackThreads) void pack_rows_kernel(orbgpu_pack_desc d0, orbgpu_pack_desc d1,
                                                                 orbgpu_pack_desc d2, orbgpu_pack_desc d3, int cap) {
    const int t = blockIdx.y;
    const orbgpu_pack_desc& D = t == 0 ? d0 : t == 1 ? d1 : t == 2 ? d2 : d3;
    const int b = blockIdx.x;
    __shared__ int s_part[kPackThreads / 64];
    // offset of frame b: the counts of frames 0 .. b-1 (B <= a few thousand), each
    // clamped to [0, cap] exactly as a frame's own row count below, so an
    // out-of-range count (an error sentinel) can leave neither gaps nor overlaps
    int part = 0;
    for (int j = threadIdx.x; j < b; j += kPackThreads) part += min(max(D.counts[j], 0), cap);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = part;
    __syncthreads();
    int off = 0;
#pragma unroll
    for (int w = 0; w < kPackThreads / 64; ++w) off += s_part[w];
    const int n = min(max(D.counts[b], 0), cap);
    const int words = D.row_bytes >> 2;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(D.rows + (size_t)b * cap * D.row_bytes);
    uint32_t* dst = reinterpret_cast<uint32_t*>(D.packed + (size_t)off * D.row_bytes);
    const int total = n * words;
    for (int k = threadIdx.x; k < total; k += kPackThreads) dst[k] = src[k];
}

// The single-frame upload: the frame's rows from pinned host memory to HBM
// by a kernel (16 bytes per thread, reads over PCIe), so the drop-in path
// has no copy-engine transfer and no copy-engine / compute-queue handoff
// (each cost ~8 us per transfer on the box, tools/dropin_timeline.py).
__global__ __launch_bounds__(256) void copy16_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, int n16) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

// The single-frame completion flag: launched after the extraction on its
// stream, so every output store of the call has completed (kernel boundary)
// when it publishes the call's sequence number to coherent pinned memory; the
// host spins on it instead of waking from hipStreamSynchronize.  The outputs
// it orders are in coherent (uncached) pinned memory too, so the store needs
// no release: a system-scope release wrote the whole L2 back first (3.9 us
// per call, profiles/r06_dropin_timeline_final.txt); relaxed at system scope
// it is one write-through store.
__global__ void done_flag_kernel(unsigned long long* flag, unsigned long long v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// up to kCopyList such copies in one launch (blockIdx.y = the copy)
__global__ __launch_bounds__(256) void copy16_list_kernel(CopyList16 L) {
    const CopyDesc16& d = L.d[blockIdx.y];
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(d.src);
    uint4* __restrict__ dst = reinterpret_cast<uint4*>(d.dst);
    const int n16 = (int)(d.bytes / 16);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

}  // namespace

hipError_t launch_done_flag(unsigned long long* flag, unsigned long long v, hipStream_t stream) {
    hipLaunchKernelGGL(done_flag_kernel, dim3(1), dim3(64), 0, stream, flag, v);
    return hipGetLastError();
}

hipError_t launch_copy16_list(const CopyList16& L, hipStream_t stream) {
    if (L.n <= 0) return hipSuccess;
    if (L.n > kCopyList) return hipErrorInvalidValue;
    size_t most = 0;
    for (int i = 0; i < L.n; ++i) {
        const CopyDesc16& d = L.d[i];
        if (d.bytes % 16 || ((uintptr_t)d.src & 15) || ((uintptr_t)d.dst & 15) || d.bytes / 16 > (size_t)INT32_MAX)
            return hipErrorInvalidValue;
        most = d.bytes > most ? d.bytes : most;
    }
    const int blocks = (int)std::min<size_t>((most / 16 + 255) / 256, 1024);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(copy16_list_kernel, dim3(blocks, L.n), dim3(256), 0, stream, L);
    return hipGetLastError();
}

hipError_t launch_copy16(void* dst, const void* src, size_t nbytes, hipStream_t stream) {
    if (nbytes % 16 || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15) || nbytes / 16 > (size_t)INT32_MAX)
        return hipErrorInvalidValue;
    const int n16 = (int)(nbytes / 16);
    if (n16 == 0) return hipSuccess;
    const int blocks = (n16 + 255) / 256;
    hipLaunchKernelGGL(copy16_kernel, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<uint4*>(dst),
                       reinterpret_cast<const uint4*>(src), n16);
    return hipGetLastError();
}

hipError_t launch_pack_rows(int batch, int cap, int ntensors, const orbgpu_pack_desc* d, hipStream_t stream) {
    if (batch <= 0 || ntensors <= 0) return hipSuccess;
    const orbgpu_pack_desc z{};
    hipLaunchKernelGGL(pack_rows_kernel, dim3(batch, ntensors), dim3(kPackThreads), 0, stream, d[0],
                       ntensors > 1 ? d[1] : z, ntensors > 2 ? d[2] : z, ntensors > 3 ? d[3] : z, cap);
    return hipGetLastError();
}

}  // namespace orbgpu
