// mem_probe.hip — vector-memory cost of the MC load / store shapes on gfx950 (dev tool; informs
// the lane layout of recon.hip's reference-row loads).
//   hipcc -O3 --offload-arch=gfx950 tools/mem_probe.hip -o tools/mem_probe.bin && tools/mem_probe.bin
// Each pattern: 2048 workgroups x 256 threads; every wave issues ITER instructions of one shape
// through a raw buffer resource (as the kernel does) at random 2,048-B-stride rows of a window
// (4 MB: L2-resident; 256 MB: HBM / MALL); prints CU cycles per wave-instruction at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 128
#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);               \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

typedef uint32_t u3v __attribute__((ext_vector_type(3)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0xFFFFFF00u;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// P: 0 b128 row/lane | 1 b128 + b32(+16) row/lane | 2 b128 row/lane, lanes with (l&3) odd OOB |
//    3 b128 row/lane, 3 of 4 lanes OOB | 4 b128 all OOB | 5 b128 lane pairs per row (x, x+8) |
//    6 b64 4 lanes per row | 7 b96 row/lane | 8 b32 row/lane | 9 b128 row/lane exec-masked half |
//    10 b128 row/lane, the 4 lanes of a row-quad 4 rows apart in one line-group (row = y + (l>>2) + ...)
template <int P>
__global__ __launch_bounds__(256) void kload(const uint8_t* __restrict__ buf, uint32_t bytes, uint32_t rows_mask,
                                             uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, (int)bytes, 0x00020000);
    uint32_t acc = 0;
    for (int it = 0; it < ITER; it++) {
        const uint32_t h = hsh(wave * 1315423911u + it * 2654435761u + (uint32_t)(P == 5 ? lane >> 1 : (P == 6 ? lane >> 2 : lane)));
        const uint32_t row = h & rows_mask;
        uint32_t off = row * 2048u + ((h >> 20) & 0x1ffu) * 4u;  // dword-aligned x in [0, 2044)
        if (P == 5) off += (lane & 1) * 8u;
        if (P == 6) off += (lane & 3) * 8u;
        if (P == 2 && (lane & 1)) off = kOOB;
        if (P == 3 && (lane & 3)) off = kOOB;
        if (P == 4) off = kOOB;
        if (P == 0 || P == 2 || P == 3 || P == 4 || P == 5) {
            const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (P == 1) {
            const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(off + 16), 0, 0);
            acc += v.x ^ v.y ^ v.z ^ v.w ^ w;
        } else if (P == 6) {
            const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
            acc += v.x ^ v.y;
        } else if (P == 7) {
            const u3v v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)off, 0, 0);
            acc += v.x ^ v.y ^ v.z;
        } else if (P == 8) {
            acc += __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
        } else if (P == 9) {
            if (lane & 1) {
                const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// S: 0 b128, 16 rows x 4 adjacent lanes (64 B per row, the luma row store) | 1 b64, 16 rows x 4
//    lanes (32 B per row, chroma) | 2 b128 row/lane (64 rows) | 3 b32, 16 rows x 4 lanes
template <int S>
__global__ __launch_bounds__(256) void kstore(uint8_t* __restrict__ buf, uint32_t rows_mask) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    for (int it = 0; it < ITER; it++) {
        const uint32_t h = hsh(wave * 1315423911u + it * 2654435761u);
        const uint32_t base = (h & rows_mask & ~15u) * 2048u + ((h >> 24) & 15u) * 64u;
        uint32_t off;
        if (S == 2) off = ((h + lane) & rows_mask) * 2048u + ((h >> 24) & 15u) * 64u;
        else off = base + (lane >> 2) * 2048u + (lane & 3) * (S == 1 ? 8u : (S == 3 ? 4u : 16u));
        if (S == 0 || S == 2) *(uint4*)(buf + off) = make_uint4(it, lane, 0, 0);
        else if (S == 1) *(uint2*)(buf + off) = make_uint2(it, lane);
        else *(uint32_t*)(buf + off) = it;
    }
}

static double cyc(float ms) {
    const double per_cu = 2048.0 * 4 * ITER / 256.0;
    return ms * 1e6 / per_cu * 2.4;
}

template <int P>
static int runl(const char* name, const uint8_t* buf, uint32_t* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float ms[2];
    const uint32_t masks[2] = {2047u, 131071u};  // 4 MB, 256 MB windows
    for (int w = 0; w < 2; w++) {
        for (int rep = 0; rep < 2; rep++) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(kload<P>, dim3(2048), dim3(256), 0, 0, buf, 256u << 20, masks[w], out);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
        }
        CHECK(hipEventElapsedTime(&ms[w], a, b));
    }
    printf("load  %-44s L2 %7.1f cyc   HBM %7.1f cyc\n", name, cyc(ms[0]), cyc(ms[1]));
    return 0;
}

template <int S>
static int runs(const char* name, uint8_t* buf) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float ms[2];
    const uint32_t masks[2] = {2047u, 131071u};
    for (int w = 0; w < 2; w++) {
        for (int rep = 0; rep < 2; rep++) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(kstore<S>, dim3(2048), dim3(256), 0, 0, buf, masks[w]);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
        }
        CHECK(hipEventElapsedTime(&ms[w], a, b));
    }
    printf("store %-44s L2 %7.1f cyc   HBM %7.1f cyc\n", name, cyc(ms[0]), cyc(ms[1]));
    return 0;
}

int main() {
    uint8_t* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, (256u << 20) + 4096));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, (256u << 20) + 4096));
    runl<0>("b128 row/lane (64 lines)", buf, out);
    runl<1>("b128 + b32(+16) row/lane (2 instr)", buf, out);
    runl<2>("b128 row/lane, half lanes OOB", buf, out);
    runl<3>("b128 row/lane, 3/4 lanes OOB", buf, out);
    runl<4>("b128 all lanes OOB", buf, out);
    runl<9>("b128 row/lane, half lanes exec-masked", buf, out);
    runl<5>("b128 lane pair per row (x, x+8): 32 rows", buf, out);
    runl<6>("b64 4 lanes per row: 16 rows", buf, out);
    runl<7>("b96 row/lane", buf, out);
    runl<8>("b32 row/lane", buf, out);
    runs<0>("b128 16 rows x 4 lanes (64 B/row)", buf);
    runs<1>("b64 16 rows x 4 lanes (32 B/row)", buf);
    runs<3>("b32 16 rows x 4 lanes (16 B/row)", buf);
    runs<2>("b128 row/lane (64 rows)", buf);
    return 0;
}
