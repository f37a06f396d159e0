// unaligned_check.hip — do raw buffer loads at byte (non-dword) offsets return the bytes at that
// offset on gfx950, and what do they cost in the texture-address unit? (dev tool)
//   hipcc -O3 --offload-arch=gfx950 tools/unaligned_check.hip -o tools/unaligned_check.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void probe(const uint8_t* buf, uint32_t* out) {
    const int lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 4096, 0x00020000);
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, lane, 0, 0);  // byte offset = lane
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, lane + 16, 0, 0);
    out[lane * 5 + 0] = v.x; out[lane * 5 + 1] = v.y; out[lane * 5 + 2] = v.z; out[lane * 5 + 3] = v.w;
    out[lane * 5 + 4] = w;
}

#define ITER 256
template <int U>
__global__ __launch_bounds__(256) void cost(const uint8_t* __restrict__ buf, uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 8 << 20, 0x00020000);
    uint32_t acc = 0;
    uint32_t base = (wave * 7919u) & 0xffffu;
    for (int it = 0; it < ITER; it++) {
        const uint32_t row = (base + it * 131u) & 2047u;
        const uint32_t off = ((row + (lane >> 2)) & 2047u) * 2048u + (lane & 3) * 16 + (U ? ((lane * 7 + it) % 4) : 0);
        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U>
static int run(const char* name, const uint8_t* buf, uint32_t* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(cost<U>, dim3(2048), dim3(256), 0, 0, buf, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
    }
    printf("%-40s %8.3f ms\n", name, ms);
    return 0;
}

int main() {
    uint8_t* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, 8 << 20));
    CHECK(hipMalloc(&out, 64 * 5 * 4));
    uint8_t h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 37 + 11);
    CHECK(hipMemcpy(buf, h, 4096, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, out);
    CHECK(hipDeviceSynchronize());
    uint32_t o[64 * 5];
    CHECK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int d = 0; d < 5; d++) {
            uint32_t e = 0;
            for (int j = 0; j < 4; j++) e |= (uint32_t)h[l + 4 * d + j] << (8 * j);
            if (o[l * 5 + d] != e) {
                if (bad < 5) printf("lane %d dword %d got %08x want %08x\n", l, d, o[l * 5 + d], e);
                bad++;
            }
        }
    printf("unaligned buffer loads: %s (%d mismatches)\n", bad ? "NOT byte-exact" : "byte-exact", bad);
    run<0>("x4 4 lanes per row, aligned", buf, out);
    run<1>("x4 4 lanes per row, byte offsets 0-3", buf, out);
    return 0;
}
