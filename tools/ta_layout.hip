// ta_layout.hip — texture-address cost of the MC row-load lane layouts (dev tool).
//   hipcc -O3 --offload-arch=gfx950 tools/ta_layout.hip -o tools/ta_layout.bin && tools/ta_layout.bin
// One wave-instruction group = the loads one prediction direction of a 4-MB group issues for
// its 64 luma rows (4 MBs x 16 rows), from a reference plane of 2048-B rows; MB k's block sits at
// x = 16k + jitter_k (jitter: 0 = coherent vectors, else per-MB random in [-J, J] px, dword-aligned).
//   v8: lane = row*4 + k, dwordx4 at x + dwordx1 at x + 16 (one 16-px row per lane)
//   v9: lane = p*8 + h*4 + k, dwordx3 at x + 8h, rows 2p (pass 0) and 2p+1 (pass 1)
//   v9h: lane = p*8 + k*2 + h (halves of a row in adjacent lanes)
// Prints CU cycles per group (2048 WGs x 4 waves x ITER groups).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 128
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int L, int J>
__global__ __launch_bounds__(256) void kern(const uint8_t* __restrict__ buf, uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (int it = 0; it < ITER; it++) {
        const uint32_t gid = wave * ITER + it;
        const uint32_t y0 = (hash(gid) & 2047u) & ~15u;   // group's MB row in a 2048-row window
        const uint32_t x0 = (hash(gid * 3 + 1) & 1023u) & ~63u;
        auto mbx = [&](int k) -> uint32_t {
            const int j = J ? (int)(hash(gid * 7 + k) % (2 * J + 1)) - J : 0;
            return (uint32_t)((int)x0 + 16 * k + 64 + j) & ~3u;
        };
        if (L == 0) {
            const int k = lane & 3, row = lane >> 2;
            const uint32_t off = ((y0 + row) & 2047u) * 2048u + mbx(k);
            const uint4 v = *(const uint4*)(buf + off);
            const uint32_t w = *(const uint32_t*)(buf + off + 16);
            acc += v.x ^ v.y ^ v.z ^ v.w ^ w;
        } else {
            int k, h, p;
            if (L == 1) { k = lane & 3; h = (lane >> 2) & 1; p = lane >> 3; }
            else        { h = lane & 1; k = (lane >> 1) & 3; p = lane >> 3; }
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t off = ((y0 + 2 * p + j) & 2047u) * 2048u + mbx(k) + 8 * h;
                const uint3 v = *(const uint3*)(buf + off);
                acc += v.x ^ v.y ^ v.z;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int L, int J>
static int run(const char* name, const uint8_t* buf, uint32_t* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int blocks = 2048;
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((kern<L, J>), dim3(blocks), dim3(256), 0, 0, buf, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
    }
    const double groups_per_cu = (double)blocks * 4 * ITER / 256.0;
    printf("%-34s J=%-2d %8.3f ms  %7.1f CU cycles/group\n", name, J, ms, ms * 1e-3 * 2.4e9 / groups_per_cu);
    return 0;
}

int main() {
    uint8_t* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, 4 << 20));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, 4 << 20));
    run<0, 0>("v8 x4+x1, lane = row*4+k", buf, out);
    run<1, 0>("v9 x3 x2, lane = p*8+h*4+k", buf, out);
    run<2, 0>("v9h x3 x2, lane = p*8+k*2+h", buf, out);
    run<0, 8>("v8 x4+x1, lane = row*4+k", buf, out);
    run<1, 8>("v9 x3 x2, lane = p*8+h*4+k", buf, out);
    run<2, 8>("v9h x3 x2, lane = p*8+k*2+h", buf, out);
    run<0, 32>("v8 x4+x1, lane = row*4+k", buf, out);
    run<1, 32>("v9 x3 x2, lane = p*8+h*4+k", buf, out);
    run<2, 32>("v9h x3 x2, lane = p*8+k*2+h", buf, out);
    return 0;
}
