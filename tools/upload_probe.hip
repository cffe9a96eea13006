// Single-frame upload probe: how fast can one 640x480 frame get from a
// pageable host buffer into HBM for the extraction kernels?  Median over
// 300 repetitions of
//   A  memcpy into pinned (hipHostMalloc default) + copy kernel + sync
//   B  memcpy into pinned write-combined + copy kernel + sync
//   C  memcpy into pinned + hipMemcpyAsync H2D (copy engine) + sync
//   D  memcpy straight into fine-grained device memory (host-mapped VRAM) + a
//      kernel that reads it + sync
// plus the host memcpy alone into each destination.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/upload_probe tools/upload_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void copy16(uint4* dst, const uint4* src, int n16) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

__global__ void touch16(const uint4* src, int n16, unsigned* out) {
    unsigned acc = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) acc ^= src[i].x ^ src[i].w;
    if (acc == 0x12345678u) out[0] = acc;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F&& f, int reps = 300) {
    std::vector<double> t;
    for (int i = 0; i < 30; ++i) f();
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_us();
        f();
        t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t n = 640 * 480;
    const int n16 = (int)(n / 16), blocks = (n16 + 255) / 256;
    std::vector<uint8_t> src(n);
    for (size_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint8_t *pin, *pin_wc, *dimg, *fg;
    unsigned* dout;
    CK(hipHostMalloc((void**)&pin, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin_wc, n, hipHostMallocWriteCombined));
    CK(hipMalloc((void**)&dimg, n));
    CK(hipMalloc((void**)&dout, 64));
    auto kcopy = [&](const uint8_t* from) {
        hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s, (uint4*)dimg, (const uint4*)from, n16);
    };
    std::printf("memcpy into pinned default      %7.2f us\n", median_us([&] { std::memcpy(pin, src.data(), n); }));
    std::printf("memcpy into pinned WC           %7.2f us\n", median_us([&] { std::memcpy(pin_wc, src.data(), n); }));
    std::printf("A pinned + copy kernel + sync   %7.2f us\n", median_us([&] {
                    std::memcpy(pin, src.data(), n);
                    kcopy(pin);
                    (void)hipStreamSynchronize(s);
                }));
    std::printf("B WC + copy kernel + sync       %7.2f us\n", median_us([&] {
                    std::memcpy(pin_wc, src.data(), n);
                    kcopy(pin_wc);
                    (void)hipStreamSynchronize(s);
                }));
    std::printf("C pinned + H2D DMA + sync       %7.2f us\n", median_us([&] {
                    std::memcpy(pin, src.data(), n);
                    (void)hipMemcpyAsync(dimg, pin, n, hipMemcpyHostToDevice, s);
                    (void)hipStreamSynchronize(s);
                }));
    std::printf("kernel only (copy from pinned)  %7.2f us\n", median_us([&] {
                    kcopy(pin);
                    (void)hipStreamSynchronize(s);
                }));
    std::fflush(stdout);
    if (hipExtMallocWithFlags((void**)&fg, n, hipDeviceMallocFinegrained) == hipSuccess) {
        std::printf("fine-grained device memory allocated; host write next\n");
        std::fflush(stdout);
        std::printf("memcpy into fine-grained VRAM   %7.2f us\n", median_us([&] { std::memcpy(fg, src.data(), n); }, 50));
        std::printf("D fine-grained + kernel + sync  %7.2f us\n", median_us([&] {
                        std::memcpy(fg, src.data(), n);
                        hipLaunchKernelGGL(touch16, dim3(blocks), dim3(256), 0, s, (const uint4*)fg, n16, dout);
                        (void)hipStreamSynchronize(s);
                    }, 50));
    } else {
        std::printf("fine-grained device allocation refused\n");
    }
    std::printf("UPLOADPROBEDONE\n");
    return 0;
}
