// D2H of decoded frames by a copy kernel storing straight into pinned host memory, against
// hipMemcpyAsync (SDMA), at frame-sized copies (dev tool):
//   hipcc --offload-arch=gfx950 -O3 tools/d2h_kernel_probe.hip -o /tmp/d2h_kernel_probe && /tmp/d2h_kernel_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            return 1;                                                           \
        }                                                                       \
    } while (0)

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// grid-stride 16-B copy; nt: nontemporal stores (streamed over PCIe without L2 allocation)
template <bool NT>
__global__ void __launch_bounds__(256) copy_k(const u4v* __restrict__ s, u4v* __restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u4v v = s[i];
        if (NT)
            __builtin_nontemporal_store(v, d + i);
        else
            d[i] = v;
    }
}

int main() {
    const size_t fb = 3133440, nf = 256, bytes = fb * nf;
    uint8_t *dev, *host;
    CK(hipMalloc(&dev, bytes));
    CK(hipHostMalloc((void**)&host, bytes, hipHostMallocDefault));
    CK(hipMemset(dev, 7, bytes));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;
    for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(a, st));
        for (size_t f = 0; f < nf; f++) CK(hipMemcpyAsync(host + f * fb, dev + f * fb, fb, hipMemcpyDeviceToHost, st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("{\"how\": \"hipMemcpyAsync per frame\", \"GBps\": %.2f}\n", bytes / (ms * 1e6));
    const int grids[] = {16, 32, 64, 128, 256, 1024};
    for (int nt = 0; nt < 2; nt++)
        for (int g : grids)
            for (int per_chunk : {1, 16}) {
                for (int rep = 0; rep < 2; rep++) {
                    CK(hipEventRecord(a, st));
                    for (size_t f = 0; f < nf; f += per_chunk) {
                        const size_t n16 = fb * per_chunk / 16;
                        if (nt)
                            copy_k<true><<<g, 256, 0, st>>>((const u4v*)(dev + f * fb), (u4v*)(host + f * fb), n16);
                        else
                            copy_k<false><<<g, 256, 0, st>>>((const u4v*)(dev + f * fb), (u4v*)(host + f * fb), n16);
                    }
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                }
                CK(hipGetLastError());
                printf("{\"how\": \"copy kernel\", \"nt\": %d, \"grid\": %d, \"frames_per_launch\": %d, \"GBps\": %.2f}\n",
                       nt, g, per_chunk, bytes / (ms * 1e6));
            }
    bool ok = true;
    for (size_t i = 0; i < bytes; i += 4099) ok = ok && host[i] == 7;
    printf("{\"check\": %s}\n", ok ? "true" : "false");
    return ok ? 0 : 1;
}
