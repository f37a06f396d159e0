// ta_bench.hip — micro-benchmark of the vector-memory issue cost on gfx950 for the access
// patterns of the MC row loads (dev tool; results inform recon.hip's load layout).
//   hipcc -O3 --offload-arch=gfx950 tools/ta_bench.hip -o /tmp/ta_bench && /tmp/ta_bench
// Every pattern: 2048 workgroups x 256 threads, each wave issues ITER loads of one shape from
// an L2-resident 8 MB buffer; prints ns per wave-instruction per CU (= CU cycles / 2.4).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITER 256
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// pattern: 0 x4 row-per-lane, 1 x4 4-lanes-per-row, 2 x4 contiguous, 3 x1 row-per-lane,
// 4 x1 contiguous, 5 x4 16 rows + 48 lanes same address, 6 x4 16 rows + 48 lanes masked,
// 7 x3 row-per-lane, 8 x4 2 lanes per row (32 B), 9 x1 16 rows + 48 same
template <int P>
__global__ __launch_bounds__(256) void kern(const uint8_t* __restrict__ buf, uint32_t* __restrict__ out, uint32_t mask) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    uint32_t acc = 0;
    uint32_t base = (wave * 7919u) & mask;
    for (int it = 0; it < ITER; it++) {
        const uint32_t row = (base + it * 131u) & 2047u;  // rows of 2048 B, 4 MB window
        uint32_t off;
        if (P == 0 || P == 3 || P == 7) off = ((row + lane) & 2047u) * 2048u + (lane & 7) * 4;
        else if (P == 1) off = ((row + (lane >> 2)) & 2047u) * 2048u + (lane & 3) * 16;
        else if (P == 2) off = row * 2048u + lane * 16;
        else if (P == 4) off = row * 2048u + lane * 4;
        else if (P == 5 || P == 6 || P == 9) off = (lane < 16) ? ((row + lane) & 2047u) * 2048u + 8 : 64;
        else if (P == 10) off = ((row + (lane & 15)) & 2047u) * 2048u + (lane >> 4) * 16;  // 16 rows, MB k = lane >> 4
        else off = ((row + (lane >> 1)) & 2047u) * 2048u + (lane & 1) * 16;  // P == 8
        if (P == 3 || P == 4 || P == 9) {
            acc += *(const uint32_t*)(buf + off);
        } else if (P == 7) {
            const uint3 v = *(const uint3*)(buf + off);
            acc += v.x ^ v.y ^ v.z;
        } else if (P == 6) {
            if (lane < 16) {
                const uint4 v = *(const uint4*)(buf + off);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            }
        } else {
            const uint4 v = *(const uint4*)(buf + off);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int P>
static int run(const char* name, const uint8_t* buf, uint32_t* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int blocks = 2048;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, buf, out, 0xffffu);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
    }
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double waves_instr = (double)blocks * 4 * ITER;
    const double per_cu = waves_instr / 256.0;
    printf("%-34s %8.3f ms  %7.2f ns/wave-instr/CU  (%.1f cycles @2.4GHz)\n", name, ms, ms * 1e6 / per_cu,
           ms * 1e6 / per_cu * 2.4);
    return 0;
}

int main() {
    uint8_t* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, 8 << 20));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, 8 << 20));
    run<0>("x4  row per lane (64 lines)", buf, out);
    run<1>("x4  4 lanes per row (16 lines)", buf, out);
    run<8>("x4  2 lanes per row (32 lines)", buf, out);
    run<2>("x4  contiguous 1 KB", buf, out);
    run<7>("x3  row per lane", buf, out);
    run<3>("x1  row per lane", buf, out);
    run<4>("x1  contiguous 256 B", buf, out);
    run<5>("x4  16 rows + 48 lanes same addr", buf, out);
    run<6>("x4  16 rows, 48 lanes masked", buf, out);
    run<9>("x1  16 rows + 48 lanes same addr", buf, out);
    run<10>("x4  16 rows x 4 lanes, lanes 16 apart", buf, out);
    return 0;
}
