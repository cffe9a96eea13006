// TA (address unit) cost per wave-instruction for the access shapes of the
// pyramid kernels (diagnostic tool, not part of the library).  Every CU runs
// 16 waves, each issuing N loads/stores of one shape over an L2-resident
// buffer; prints cycles per wave-instruction per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o ta_rate ta_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 256;

template <int SHAPE>
__global__ __launch_bounds__(1024) void k(unsigned* buf, unsigned* out, unsigned long long* cyc) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 1 << 20, 0x00020000);
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    unsigned acc = 0;
    __syncthreads();
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) {
        const int base = ((blockIdx.x * 16 + w) * 4096 + i * 384) & 0xFFFF0;
        if (SHAPE == 0) {  // dwordx3 per lane, lanes 4.8 B apart (pyramid windows)
            u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, base + (lane * 24 / 5 & ~3), 0, 0);
            acc += v.x ^ v.y ^ v.z;
        } else if (SHAPE == 1) {  // dwordx4 per lane, contiguous 1 KiB
            u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, base + lane * 16, 0, 0);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (SHAPE == 2) {  // dword per lane contiguous store (256 B)
            __builtin_amdgcn_raw_buffer_store_b32(acc + i, rs, base + lane * 4, 0, 0);
        } else if (SHAPE == 3) {  // dwordx3 loads, one lane in three active
            if (lane % 3 == 0) {
                u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, base + (lane * 24 / 5 & ~3), 0, 0);
                acc += v.x ^ v.y ^ v.z;
            }
        } else if (SHAPE == 4) {  // dwordx4 store contiguous 1 KiB
            __builtin_amdgcn_raw_buffer_store_b128((u32x4){acc, acc + 1, acc + 2, (unsigned)i}, rs, base + lane * 16, 0, 0);
        } else if (SHAPE == 5) {  // dword per lane load, lanes 4.8 B apart
            acc += __builtin_amdgcn_raw_buffer_load_b32(rs, base + (lane * 24 / 5 & ~3), 0, 0);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *buf, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&buf, 4 << 20);
    (void)hipMalloc(&out, 4096 * 4);
    (void)hipMalloc(&cyc, cus * 8);
    (void)hipMemset(buf, 1, 4 << 20);
    const char* names[] = {"b96 load, 4.8B lane stride", "b128 load, contiguous", "b32 store, contiguous",
                           "b96 load, 1/3 lanes", "b128 store, contiguous", "b32 load, 4.8B lane stride"};
    for (int s = 0; s < 6; ++s) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (s) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(cus), dim3(1024), 0, 0, buf, out, cyc); break;
            }
            (void)hipDeviceSynchronize();
        }
        unsigned long long h[1024];
        (void)hipMemcpy(h, cyc, cus * 8, hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < cus; ++i) m += (double)h[i];
        m /= cus;
        printf("%-28s %7.1f cycles per wave-instruction per CU (16 waves x %d)\n", names[s], m / (16.0 * N), N);
    }
    return 0;
}
