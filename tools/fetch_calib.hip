// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes
// of the reconstruct kernel (dev tool; MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib.bin
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- tools/fetch_calib.bin   (and WRITE_SIZE, TCC_*)
// Every kernel touches a 1 GiB buffer (4x the Infinity Cache), each line at most once, after a
// 1 GiB scrub of a second buffer, so every access is an HBM miss:
//   k_stream:     coalesced 16 B / lane over 512 MiB                  -> bytes read = 512 MiB
//   k_rows:       one b128 + b32 (+16) per lane, the tap shape: 20 B of a distinct 2,048-B row
//                 per lane, inside one 128-B line (x = 0..108, dword aligned)   -> 262,144 lines
//   k_rows_x:     the same straddling two lines (x = 124: bytes 124..143)     -> 2 x 262,144 lines
//   k_rowstore:   16 rows x 64 B per store instruction (the luma row store), 256 MiB of rows
//                 written at a 2,048-B pitch, 64 B per row (half lines)     -> bytes written = 8 MiB x 16
//   k_linestore:  8 rows x 128 B per store instruction (whole lines)          -> same bytes
// It prints the byte / line counts each kernel moves; divide the PMC values by them.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__global__ void k_scrub(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(i, 0, 0, 0);
}

__global__ void k_stream(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int X>
__global__ void k_rows(const uint8_t* __restrict__ p, uint32_t* out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;  // one row per lane
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t x = X >= 0 ? (uint32_t)X : ((g * 2654435761u) >> 27) * 4u;  // 0..124 step 4
    const uint32_t off = g * 2048u + (X >= 0 ? x : (x > 108 ? 108 : x));
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(off + 16), 0, 0);
    if ((v.x ^ v.y ^ v.z ^ v.w ^ w) == 0x12345678u) out[0] = w;
}

template <int LANES_PER_ROW>
__global__ void k_store(uint8_t* __restrict__ p) {
    const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t rows = 64 / LANES_PER_ROW;
    const size_t off = ((size_t)wave * rows + lane / LANES_PER_ROW) * 2048u + (lane % LANES_PER_ROW) * 16u;
    *(uint4*)(p + off) = make_uint4(lane, wave, 1, 2);
}

int main() {
    const size_t GB = 1ull << 30;
    uint8_t *a, *b;
    uint32_t* out;
    (void)hipMalloc(&a, GB);
    (void)hipMalloc(&b, GB);
    (void)hipMalloc(&out, 64);
    auto scrub = [&]() {
        hipLaunchKernelGGL(k_scrub, dim3(8192), dim3(256), 0, 0, (uint4*)b, GB / 16);
        (void)hipDeviceSynchronize();
    };
    (void)hipMemset(a, 1, GB);
    scrub();
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)a, (512ull << 20) / 16, out);
    (void)hipDeviceSynchronize();
    printf("k_stream: %llu bytes read\n", 512ull << 20);
    scrub();
    const int nrows = 1 << 18;  // 262,144 rows x 2,048 B = 512 MiB
    hipLaunchKernelGGL(k_rows<-1>, dim3(nrows / 256), dim3(256), 0, 0, a, out);
    (void)hipDeviceSynchronize();
    printf("k_rows<-1>: %d lines (20 B each, one line per row)\n", nrows);
    scrub();
    hipLaunchKernelGGL(k_rows<124>, dim3(nrows / 256), dim3(256), 0, 0, a + (512ull << 20), out);
    (void)hipDeviceSynchronize();
    printf("k_rows<124>: %d lines (20 B straddling two lines per row)\n", 2 * nrows);
    scrub();
    // 4 lanes per row: 16 rows x 64 B per wave; 2^22 waves... keep 16 MiB of data
    const int waves4 = (16 << 20) / 1024;
    hipLaunchKernelGGL(k_store<4>, dim3(waves4 / 4), dim3(256), 0, 0, a);
    (void)hipDeviceSynchronize();
    printf("k_store<4>: %d bytes written (64 B per 2,048-B row)\n", 16 << 20);
    scrub();
    hipLaunchKernelGGL(k_store<8>, dim3(waves4 / 4), dim3(256), 0, 0, a + (256ull << 20));
    (void)hipDeviceSynchronize();
    printf("k_store<8>: %d bytes written (128 B per 2,048-B row)\n", 16 << 20);
    return 0;
}
