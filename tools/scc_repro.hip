#include <hip/hip_runtime.h>
struct ONode { unsigned r0, r1, cnt, seq; };
struct G { float hx; int maxby; };
__global__ void k(int* out, int nini, G g) {
    __shared__ int a[16], b[16];
    __shared__ ONode nodes[16];
    if (threadIdx.x < 16) a[threadIdx.x] = (threadIdx.x % 3) * 7;
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = 0;
        for (int r = 0; r < nini; ++r) {
            const int c = a[r];
            b[r] = c > 0 ? n : -1;
            if (c > 0) {
                ONode nd;
                const int x0 = (int)(g.hx * (float)r), x1 = (int)(g.hx * (float)(r + 1));
                nd.r0 = (unsigned)x0;
                nd.r1 = (unsigned)x1 | ((unsigned)(g.maxby - 16) << 16);
                nd.cnt = (unsigned)c;
                nd.seq = (unsigned)r;
                nodes[n++] = nd;
            }
        }
        out[100] = n;
    }
    __syncthreads();
    if (threadIdx.x < 16) { out[threadIdx.x] = b[threadIdx.x]; out[16 + threadIdx.x] = nodes[threadIdx.x].cnt; }
}
int main() {
    int* d; hipMalloc(&d, 512 * 4); hipMemset(d, 0, 512*4);
    G g{302.25f, 376};
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, 9, g);
    int h[512]; hipMemcpy(h, d, 512*4, hipMemcpyDeviceToHost);
    printf("b:"); for (int i = 0; i < 9; ++i) printf(" %d", h[i]); printf("\ncnt:"); for (int i = 0; i < 9; ++i) printf(" %d", h[16+i]); printf("\nn=%d\n", h[100]);
    return 0;
}
