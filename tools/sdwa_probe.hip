// Probe of SDWA / op_sel semantics on gfx950 used by pyramid.hip (diagnostic
// tool, not part of the library): prints what each instruction form returns
// for fixed operands.  Build: hipcc --offload-arch=gfx950 -O2 -o sdwa_probe sdwa_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
    unsigned a = 0x12345678u, b = 0x00030005u, c = 0xAAAAAAAAu, d = 0, e = 0x0000BEEFu;
    unsigned x = 0;
    asm volatile("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(x) : "v"(a), "v"(b), "v"(e));
    o[0] = x;  // expect 0x1234*5 + 0xBEEF
    unsigned y = c;
    asm volatile("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
                 : "+v"(y) : "v"(a), "v"(b));
    o[1] = y;  // expect ((0x1234+3) << 16) | 0xAAAA
    unsigned z = c;
    asm volatile("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
                 : "+v"(z) : "v"(a), "v"(b));
    o[2] = z;  // expect 0x1237
    unsigned w = c;
    asm volatile("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t"
                 "s_nop 1\n\t"
                 "v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
                 : "+v"(w) : "v"(a), "v"(b));
    o[3] = w;  // expect ((0x5678+5) << 16) | 0x1237
    unsigned v = 0x00FF0102u;
    asm volatile("v_pk_lshrrev_b16 %0, 2, %0" : "+v"(v));
    o[4] = v;  // expect 0x003F0040
    unsigned m = 0;
    asm volatile("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
                 : "=v"(m) : "v"(a), "v"(b));
    o[5] = m;  // expect 0x1234 * 0x30005
    (void)d;
}
// raw buffer loads (stride 0) near the range limit: per-dword or whole-load
// zeroing?  buf holds 0x11111111, 0x22222222, ... ; num_records = 10 bytes
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
__global__ void kb(unsigned* o, unsigned* buf) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 10, 0x00020000);
    u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(rs, 0, 0, 0);    // bytes 0..12: dword 2 straddles 10
    u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(rs, -4, 0, 0);   // negative offset
    u32x3 c = __builtin_amdgcn_raw_buffer_load_b96(rs, 4, 0, 0);    // dwords 1..3
    if (threadIdx.x == 0) {
        o[0] = a.x; o[1] = a.y; o[2] = a.z;
        o[3] = b.x; o[4] = b.y; o[5] = b.z;
        o[6] = c.x; o[7] = c.y; o[8] = c.z;
    }
}
int main() {
    unsigned* o; (void)hipMalloc(&o, 64); (void)hipMemset(o, 0, 64);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
    unsigned h[6]; (void)hipMemcpy(h, o, 24, hipMemcpyDeviceToHost);
    const unsigned exp[6] = {0x1234u * 5 + 0xBEEFu, ((0x1234u + 3) << 16) | 0xAAAAu, 0x1237u,
                             ((0x5678u + 5) << 16) | 0x1237u, 0x003F0040u, 0x1234u * 0x30005u};
    for (int i = 0; i < 6; ++i) printf("%d got %08x expect %08x %s\n", i, h[i], exp[i], h[i] == exp[i] ? "ok" : "DIFF");
    unsigned* buf; (void)hipMalloc(&buf, 64);
    unsigned hb[16]; for (int i = 0; i < 16; ++i) hb[i] = 0x11111111u * (i + 1);
    (void)hipMemcpy(buf, hb, 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kb, dim3(1), dim3(64), 0, 0, o, buf);
    unsigned r[9]; (void)hipMemcpy(r, o, 36, hipMemcpyDeviceToHost);
    printf("buffer b96 @0  (num_records 10): %08x %08x %08x\n", r[0], r[1], r[2]);
    printf("buffer b96 @-4 (num_records 10): %08x %08x %08x\n", r[3], r[4], r[5]);
    printf("buffer b96 @4  (num_records 10): %08x %08x %08x\n", r[6], r[7], r[8]);
    return 0;
}
