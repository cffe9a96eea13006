// Microbenchmark: issue cost of the VALU instructions the pyramid pass uses
// (wave64, 8 waves per SIMD, 8 independent chains per wave).
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP_KERNEL(NAME, ASM)                                                                  \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed, int iters) {    \
        unsigned v0 = seed ^ threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, \
                 v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19;                                     \
        const unsigned k = seed | 0x01010101u;                                                 \
        for (int i = 0; i < iters; ++i) {                                                      \
            asm volatile(ASM : "+v"(v0) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v1) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v2) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v3) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v4) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v5) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v6) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v7) : "v"(k));                                             \
        }                                                                                      \
        out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;          \
    }

OP_KERNEL(k_add, "v_add_u32 %0, %0, %1")
OP_KERNEL(k_and, "v_and_b32 %0, %0, %1")
OP_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
OP_KERNEL(k_dot2, "v_dot2_u32_u16 %0, %0, %1, 0")
OP_KERNEL(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1")
OP_KERNEL(k_mul24, "v_mul_u32_u24 %0, %0, %1")
OP_KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %1")
OP_KERNEL(k_sdwa, "v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD")
OP_KERNEL(k_add3, "v_add3_u32 %0, %0, %1, 2")
OP_KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %1")
OP_KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %1")
OP_KERNEL(k_pkmad16, "v_pk_mad_u16 %0, %0, %1, %1")
OP_KERNEL(k_pkadd16, "v_pk_add_u16 %0, %0, %1")
OP_KERNEL(k_cvtsdwa, "v_cvt_f32_u32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1")
OP_KERNEL(k_cvtpku8, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
OP_KERNEL(k_min3, "v_min3_i32 %0, %0, %1, %1")
// round 6: the ops FAST's compass / arc pass and describe's blur / moments issue most
OP_KERNEL(k_pkmaxu16, "v_pk_max_u16 %0, %0, %1")
OP_KERNEL(k_pksubu16, "v_pk_sub_u16 %0, %0, %1 clamp")
OP_KERNEL(k_pkmax3f16, "v_pk_maximum3_f16 %0, %0, %1, %1")
OP_KERNEL(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %0")
OP_KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
OP_KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 16, %1")
OP_KERNEL(k_mbcnt, "v_mbcnt_lo_u32_b32 %0, %1, %0")

// scalar ALU: 8 independent 64-bit chains per wave
__global__ __launch_bounds__(256) void k_salu(unsigned* out, unsigned seed, int iters) {
    unsigned long long a = seed, b = seed * 3ull, c = seed * 5ull, d = seed * 7ull, e = seed * 9ull, f = seed * 11ull,
                       g = seed * 13ull, h = seed * 15ull;
    const unsigned long long k = seed | 0x0101010101010101ull;
    for (int i = 0; i < iters; ++i) {
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(a) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(b) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(c) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(d) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(e) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(f) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(g) : "s"(k));
        asm volatile("s_and_b64 %0, %0, %1" : "+s"(h) : "s"(k));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a ^ b ^ c ^ d ^ e ^ f ^ g ^ h);
}

#define OP64_KERNEL(NAME, ASM)                                                                \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed, int iters) {    \
        typedef float f2 __attribute__((ext_vector_type(2)));                                  \
        f2 v0 = {(float)(seed ^ threadIdx.x), 1.f}, v1 = v0 * 3.f, v2 = v0 * 5.f, v3 = v0 * 7.f;  \
        const f2 k = {1.0001f, 0.9999f};                                                       \
        for (int i = 0; i < iters; ++i) {                                                      \
            asm volatile(ASM : "+v"(v0) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v1) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v2) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v3) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v0) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v1) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v2) : "v"(k));                                             \
            asm volatile(ASM : "+v"(v3) : "v"(k));                                             \
        }                                                                                      \
        f2 r = v0 + v1 + v2 + v3;                                                              \
        out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(r.x + r.y);                           \
    }
OP64_KERNEL(k_pkfma, "v_pk_fma_f32 %0, %0, %1, %1")
OP64_KERNEL(k_pkaddf, "v_pk_add_f32 %0, %0, %1")

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;  // 8 x 256 threads = 32 waves per CU = 8 per SIMD
    unsigned* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const int iters = 4096;
    struct K { const char* n; void (*f)(unsigned*, unsigned, int); } ks[] = {
        {"v_add_u32", k_add}, {"v_and_b32", k_and}, {"v_perm_b32", k_perm}, {"v_dot2_u32_u16", k_dot2},
        {"v_mul_hi_u32_u24", k_mulhi24}, {"v_mul_u32_u24", k_mul24}, {"v_mul_lo_u32", k_mullo},
        {"v_lshrrev_b32_sdwa", k_sdwa}, {"v_add3_u32", k_add3}, {"v_fma_f32", k_fma}, {"v_mad_u32_u24", k_mad24},
        {"v_pk_mad_u16", k_pkmad16}, {"v_pk_add_u16", k_pkadd16}, {"v_cvt_f32_u32_sdwa", k_cvtsdwa},
        {"v_cvt_pk_u8_f32", k_cvtpku8}, {"v_min3_i32", k_min3}, {"v_pk_max_u16", k_pkmaxu16}, {"v_pk_sub_u16 clamp", k_pksubu16},
        {"v_pk_maximum3_f16", k_pkmax3f16}, {"v_dot4_u32_u8", k_dot4}, {"v_alignbyte_b32", k_alignbyte},
        {"v_lshl_or_b32", k_lshlor}, {"v_mbcnt_lo_u32_b32", k_mbcnt}, {"v_pk_fma_f32", k_pkfma}, {"v_pk_add_f32", k_pkaddf}, {"s_and_b64 (SALU)", k_salu}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
        hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD = 8 waves * iters * 8
        const double per_simd = 8.0 * iters * 8;
        const double cyc = ms * 1e-3 * p.clockRate * 1e3;
        printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", k.n, ms, cyc / per_simd);
    }
    return 0;
}
