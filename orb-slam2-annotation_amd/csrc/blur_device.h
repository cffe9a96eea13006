// blur_device.h -- the arithmetic of GaussianBlur(7x7, sigma 2) on 8-bit
// rows as OpenCV 2.4 does it (ORBextractor.cpp:1097-1098): integer kernel
// [18,34,49,55,49,34,18] (x256), exact int row pass, column pass rounded
// half-to-even on the SIMD columns (x < 4*floor(w/4), SymmColumnVec_32s8u)
// and half-up on the scalar tail (FixedPtCastEx<int,uchar>).  Shared by
// blur.hip (whole levels, the debug/blurred-level API) and describe.hip
// (the 37x37 neighbourhood of each keypoint, fused into the descriptor).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbgpu {
namespace blurdev {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Row pass of 4 adjacent columns: packed 16-bit arithmetic, two columns per
// register.  P[j] = (px[j], px[j+1]) with px[j] = column x0 - 3 + j.  The
// symmetric sum 18(a+g) + 34(b+f) + 49(c+e) + 55d of 8-bit inputs is at most
// 255 * 257 = 65535: exact in u16.  Returns the 4 sums as floats (exact).
__device__ __forceinline__ void row_pass(const uint32_t (&P)[9], f32x2& lo, f32x2& hi) {
    const u16x2* Q = reinterpret_cast<const u16x2*>(P);
    const u16x2 k18 = {18, 18}, k34 = {34, 34}, k49 = {49, 49}, k55 = {55, 55};
    const u16x2 r01 = (Q[0] + Q[6]) * k18 + (Q[1] + Q[5]) * k34 + (Q[2] + Q[4]) * k49 + Q[3] * k55;
    const u16x2 r23 = (Q[2] + Q[8]) * k18 + (Q[3] + Q[7]) * k34 + (Q[4] + Q[6]) * k49 + Q[5] * k55;
    lo = f32x2{(float)r01.x, (float)r01.y};
    hi = f32x2{(float)r23.x, (float)r23.y};
}

// Column pass over the 7-row window (w[i] = row y - 3 + i), two columns per
// packed-f32 op.  Every product and partial sum is an integer below 2^24
// unless the total is (then the result saturates to 255 either way), so the
// float arithmetic is exact.
__device__ __forceinline__ f32x2 col_pass(f32x2 w0, f32x2 w1, f32x2 w2, f32x2 w3, f32x2 w4, f32x2 w5, f32x2 w6) {
    // the taps carry the 1/65536 of the two passes' fixed-point scale: every
    // term is an integer below 2^24 times 2^-16, so the sums are still exact
    constexpr float kS = 1.f / 65536.f;
    const f32x2 k18 = {18.f * kS, 18.f * kS}, k34 = {34.f * kS, 34.f * kS}, k49 = {49.f * kS, 49.f * kS},
                k55 = {55.f * kS, 55.f * kS};
    f32x2 s = w3 * k55;
    s = __builtin_elementwise_fma(w2 + w4, k49, s);
    s = __builtin_elementwise_fma(w1 + w5, k34, s);
    return __builtin_elementwise_fma(w0 + w6, k18, s);
}

// 8-bit result of one column on the scalar tail (x >= 4*floor(w/4)):
// FixedPtCastEx rounds half up.  (The vector path, SymmColumnVec_32s8u,
// rounds half to even: v_cvt_pk_u8_f32 in store_row.)
__device__ __forceinline__ uint32_t to_u8(float v) {
    return (uint32_t)fminf(__builtin_floorf(v + 0.5f), 255.f);  // v + 0.5 exact (< 2^8, 16 frac bits)
}

// 8-bit packing of 4 filtered columns; v_cvt_pk_u8_f32 rounds to nearest
// even and saturates (the vector path), to_u8 rounds half up (the tail).
__device__ __forceinline__ uint32_t pack4_simd(f32x2 lo, f32x2 hi) {
    uint32_t packed = __builtin_amdgcn_cvt_pk_u8_f32(lo.x, 0, 0u);
    packed = __builtin_amdgcn_cvt_pk_u8_f32(lo.y, 1, packed);
    packed = __builtin_amdgcn_cvt_pk_u8_f32(hi.x, 2, packed);
    return __builtin_amdgcn_cvt_pk_u8_f32(hi.y, 3, packed);
}

__device__ __forceinline__ uint32_t pack4(f32x2 lo, f32x2 hi, bool simd) {
    if (simd) return pack4_simd(lo, hi);
    return to_u8(lo.x) | (to_u8(lo.y) << 8) | (to_u8(hi.x) << 16) | (to_u8(hi.y) << 24);
}

struct Raw3 {
    uint32_t a, b, c;  // level columns x0-4 .. x0+7
};

// Row pass of the 4 columns x0..x0+3 from the three raw words around them,
// with no byte shuffling: column x0 + m takes its 7 taps from the words as
// they are, against the kernel shifted by m bytes -- m = 0: a[1..3] b[0..3];
// m = 1: a[2..3] b c[0]; m = 2: a[3] b c[0..1]; m = 3: b c[0..2] -- ten
// v_dot4_u32_u8 in all (2 + 3 + 3 + 2), exact (at most 255 * 257 = 65535).
// The four sums as integers, each added to `acc`.
__device__ __forceinline__ void row_sums_shifted(const Raw3& R, uint32_t acc, uint32_t (&s)[4]) {
    constexpr uint32_t A0 = 0u | 18u << 8 | 34u << 16 | 49u << 24, B0 = 55u | 49u << 8 | 34u << 16 | 18u << 24;
    constexpr uint32_t A1 = 18u << 16 | 34u << 24, B1 = 49u | 55u << 8 | 49u << 16 | 34u << 24, C1 = 18u;
    constexpr uint32_t A2 = 18u << 24, B2 = 34u | 49u << 8 | 55u << 16 | 49u << 24, C2 = 34u | 18u << 8;
    constexpr uint32_t B3 = 18u | 34u << 8 | 49u << 16 | 55u << 24, C3 = 49u | 34u << 8 | 18u << 16;
    s[0] = __builtin_amdgcn_udot4(R.b, B0, __builtin_amdgcn_udot4(R.a, A0, acc, false), false);
    s[1] = __builtin_amdgcn_udot4(R.c, C1,
                                  __builtin_amdgcn_udot4(R.b, B1, __builtin_amdgcn_udot4(R.a, A1, acc, false), false),
                                  false);
    s[2] = __builtin_amdgcn_udot4(R.c, C2,
                                  __builtin_amdgcn_udot4(R.b, B2, __builtin_amdgcn_udot4(R.a, A2, acc, false), false),
                                  false);
    s[3] = __builtin_amdgcn_udot4(R.c, C3, __builtin_amdgcn_udot4(R.b, B3, acc, false), false);
}

__device__ __forceinline__ void row_pass_raw_shifted(const Raw3& R, f32x2& lo, f32x2& hi) {
    // the sums accumulate onto the bits of 2^23 (0x4B000000), so each is the
    // float 2^23 + s as it stands (s < 2^16); one packed subtract per two
    // columns (exact) replaces four integer-to-float conversions
    uint32_t s[4];
    row_sums_shifted(R, 0x4B000000u, s);
    const f32x2 m = {8388608.f, 8388608.f};
    lo = f32x2{__uint_as_float(s[0]), __uint_as_float(s[1])} - m;
    hi = f32x2{__uint_as_float(s[2]), __uint_as_float(s[3])} - m;
}

// The same sums with the windows cut out by v_alignbyte_b32 ([x-3, x]
// against (18, 34, 49, 55), [x+1, x+4) against (49, 34, 18, 0)): the form
// blur.hip's whole-level pass uses.
__device__ __forceinline__ void row_pass_raw(const Raw3& R, f32x2& lo, f32x2& hi) {
    constexpr uint32_t K1 = 18u | 34u << 8 | 49u << 16 | 55u << 24;  // taps x-3 .. x
    constexpr uint32_t K2 = 49u | 34u << 8 | 18u << 16;              // taps x+1 .. x+3
    const uint32_t w10 = __builtin_amdgcn_alignbyte(R.b, R.a, 1), w20 = __builtin_amdgcn_alignbyte(R.c, R.b, 1);
    const uint32_t w11 = __builtin_amdgcn_alignbyte(R.b, R.a, 2), w21 = __builtin_amdgcn_alignbyte(R.c, R.b, 2);
    const uint32_t w12 = __builtin_amdgcn_alignbyte(R.b, R.a, 3), w22 = __builtin_amdgcn_alignbyte(R.c, R.b, 3);
    const uint32_t s0 = __builtin_amdgcn_udot4(w20, K2, __builtin_amdgcn_udot4(w10, K1, 0u, false), false);
    const uint32_t s1 = __builtin_amdgcn_udot4(w21, K2, __builtin_amdgcn_udot4(w11, K1, 0u, false), false);
    const uint32_t s2 = __builtin_amdgcn_udot4(w22, K2, __builtin_amdgcn_udot4(w12, K1, 0u, false), false);
    const uint32_t s3 = __builtin_amdgcn_udot4(R.c, K2, __builtin_amdgcn_udot4(R.b, K1, 0u, false), false);
    lo = f32x2{(float)s0, (float)s1};
    hi = f32x2{(float)s2, (float)s3};
}

}  // namespace blurdev
}  // namespace orbgpu
