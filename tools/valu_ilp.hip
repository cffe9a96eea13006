// Microbenchmark: VALU issue cost vs waves per SIMD and independent chains
// per wave (dependent v_add_u32 / v_pk_fma_f32 chains).
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_ilp.hip -o tools/valu_ilp
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ __launch_bounds__(64) void k_add(unsigned* out, unsigned seed, int iters) {
    unsigned v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = seed * (c + 1) ^ threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed));
    }
    unsigned x = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) x ^= v[c];
    out[blockIdx.x * 64 + threadIdx.x] = x;
}

template <int CH>
__global__ __launch_bounds__(64) void k_pkfma(unsigned* out, unsigned seed, int iters) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = f2{(float)(seed + c), 1.f};
    const f2 k = {1.0001f, 0.9999f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v[c]) : "v"(k));
    }
    float x = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) x += v[c].x + v[c].y;
    out[blockIdx.x * 64 + threadIdx.x] = (unsigned)x;
}

#define OPK(NAME, ASM)                                                                       \
    __global__ __launch_bounds__(64) void NAME(unsigned* out, unsigned seed, int iters) {     \
        unsigned v0 = seed ^ threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7;                \
        for (int i = 0; i < iters; ++i) {                                                      \
            _Pragma("unroll") for (int r = 0; r < 8; ++r) {                                    \
                asm volatile(ASM : "+v"(v0) : "v"(seed));                                      \
                asm volatile(ASM : "+v"(v1) : "v"(seed));                                      \
                asm volatile(ASM : "+v"(v2) : "v"(seed));                                      \
                asm volatile(ASM : "+v"(v3) : "v"(seed));                                      \
            }                                                                                  \
        }                                                                                      \
        out[blockIdx.x * 64 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3;                                \
    }
OPK(k_cmpsel, "v_cmp_lt_i32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc")
OPK(k_min, "v_min_i32_e32 %0, %0, %1")
OPK(k_max3, "v_max3_i32 %0, %0, %1, %1")
OPK(k_lshl, "v_lshlrev_b32_e32 %0, 1, %0")
OPK(k_lshladd, "v_lshl_add_u32 %0, %0, 1, %1")
OPK(k_bfe, "v_bfe_u32 %0, %0, 3, 5")
OPK(k_cmpaddc, "v_cmp_lt_i32_e32 vcc, %0, %1\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc")
OPK(k_sub, "v_sub_u32_e32 %0, %0, %1")
OPK(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")

template <class F>
void run(const char* name, F f, int ch, int wps, int cus, unsigned* out) {
    const int iters = 2048;
    const int blocks = cus * 4 * wps;  // one wave per block, wps waves per SIMD
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 3u, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 3u, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double instr_per_simd = (double)wps * iters * 8 * ch;
    printf("%-14s chains %d waves/SIMD %d: %.2f cycles per instruction per SIMD\n", name, ch, wps,
           ms * 1e-3 * 2.4e9 / instr_per_simd);
}

int main() {
    int cus = 256;
    unsigned* out;
    (void)hipMalloc(&out, (size_t)cus * 4 * 8 * 64 * 4);
    {
        const char* names[] = {"cmp+cndmask(x2)", "v_min_i32", "v_max3_i32", "v_lshlrev", "v_lshl_add", "v_bfe_u32",
                               "cmp+addc(x2)", "v_sub_u32", "v_alignbyte"};
        void (*fs[])(unsigned*, unsigned, int) = {k_cmpsel, k_min, k_max3, k_lshl, k_lshladd, k_bfe, k_cmpaddc, k_sub,
                                                  k_alignbyte};
        for (int i = 0; i < 9; ++i) run(names[i], fs[i], 4, 8, cus, out);
    }
    for (int w : {1, 2, 4, 8}) {
        run("v_add_u32", k_add<1>, 1, w, cus, out);
        run("v_add_u32", k_add<2>, 2, w, cus, out);
        run("v_add_u32", k_add<4>, 4, w, cus, out);
        run("v_pk_fma_f32", k_pkfma<1>, 1, w, cus, out);
        run("v_pk_fma_f32", k_pkfma<2>, 2, w, cus, out);
        run("v_pk_fma_f32", k_pkfma<4>, 4, w, cus, out);
    }
    return 0;
}
