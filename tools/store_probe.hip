// store_probe.hip — what a row store costs beside the MC tap loads and VALU work (dev tool).
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe.bin
// Every wave runs ITER iterations of: 8 row-per-lane b128 tap loads (random rows of a 4 MB
// window, L2 hits; consumed next iteration), 800 VOP3 ops, and 2 store instructions of 1 KB each
// (64 lanes x 16 B) in shape S into a 256 MB output region (random 16-row block per iteration):
//   0 none | 1 16 rows x 64 B (4 lanes/row), pitch 2048 | 2 same, pitch 1920 (the 1080p stride)
//   3 8 rows x 128 B (8 lanes/row: whole lines), pitch 1920 | 4 4 rows x 256 B, pitch 1920
//   5 1 KB contiguous | 6 shape 2 nontemporal | 7 shape 2 into a 4 MB region (L2-resident)
//   8 shape 2, the two stores issued back to back after the loads (not after the VALU)
// 4 waves per workgroup, 4 workgroups per CU (LDS-padded), 4096 workgroups.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 64
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

template <int S>
__device__ __forceinline__ void row_store(uint8_t* obase, uint32_t h, int lane, int j, uint4 v) {
    if (S == 0) return;
    uint32_t pitch = S == 1 ? 2048u : 1920u;
    uint32_t region = S == 7 ? (4u << 20) : (240u << 20);
    uint32_t blk = (h % (region / (pitch * 16u))) * pitch * 16u;
    uint32_t off;
    if (S == 1 || S == 2 || S == 6 || S == 7 || S == 8) off = blk + (lane >> 2) * pitch + (lane & 3) * 16u + j * 8u * pitch;
    else if (S == 3) off = blk + (lane >> 3) * pitch + (lane & 7) * 16u + j * 8u * pitch;
    else if (S == 4) off = blk + (lane >> 4) * pitch + (lane & 15) * 16u + j * 8u * pitch;
    else off = (h % (region / 2048u)) * 2048u + lane * 16u + j * 1024u;
    if (S == 6) {
        u4v w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (u4v*)(obase + off));
    } else {
        *(uint4*)(obase + off) = v;
    }
}

template <int S>
__global__ __launch_bounds__(256) void kern(const uint8_t* __restrict__ buf, uint8_t* __restrict__ obuf,
                                            uint32_t* __restrict__ out) {
    __shared__ uint32_t pad[9000];
    const int lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 4 << 20, 0x00020000);
    uint32_t a[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i][0] = a[i][1] = a[i][2] = a[i][3] = lane;
    uint32_t x0 = lane * 0x01010101u, x1 = gw, x2 = x0 ^ 0x5a5a5a5a, x3 = x1 * 3u;
    for (int it = 0; it < ITER; it++) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) acc ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
        x1 ^= acc;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t h = hsh(gw * 977u + it * 131u + i * 7919u + lane);
            const uint32_t off = (h & 2047u) * 2048u + ((h >> 20) & 0x1ffu) * 4u;
            const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            a[i][0] = v.x; a[i][1] = v.y; a[i][2] = v.z; a[i][3] = v.w;
        }
        const uint32_t hs = hsh(gw * 31u + it);
        if (S == 8) {
            row_store<2>(obuf, hs, lane, 0, make_uint4(x0, x1, x2, x3));
            row_store<2>(obuf, hs, lane, 1, make_uint4(x3, x1, x2, x0));
        }
        for (int m = 0; m < 100; m++) {
            x0 = __builtin_amdgcn_alignbyte(x1, x0, m & 3);
            x2 = __builtin_amdgcn_alignbyte(x3, x2, (m + 1) & 3);
            x0 = __builtin_amdgcn_lerp(x0, x2, 0x01010101u);
            x2 = __builtin_amdgcn_lerp(x2, x1, 0x01010101u);
            x1 = __builtin_amdgcn_perm(x0, x1, 0x05040100u);
            x3 = __builtin_amdgcn_perm(x2, x3, 0x07060302u);
            x1 = __builtin_amdgcn_lerp(x1, x3, 0x01010101u);
            x3 = __builtin_amdgcn_alignbyte(x0, x3, 1);
        }
        if (S != 8) {
            row_store<S>(obuf, hs, lane, 0, make_uint4(x0, x1, x2, x3));
            row_store<S>(obuf, hs, lane, 1, make_uint4(x3, x1, x2, x0));
        }
    }
    uint32_t acc = x0 ^ x1 ^ x2 ^ x3;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (pad[(threadIdx.x + 1) & 255] == 0x12345678u) out[0] = acc;
}

template <int S>
static void run(const char* name, const uint8_t* buf, uint8_t* obuf, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(kern<S>, dim3(4096), dim3(256), 0, 0, buf, obuf, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    const double per_cu_store = 4096.0 * 4 * ITER * 2 / 256.0;
    printf("S%d %-52s %.3f ms\n", S, name, ms);
    (void)per_cu_store;
}

int main() {
    uint8_t *buf, *obuf;
    uint32_t* out;
    (void)hipMalloc(&buf, (4 << 20) + 4096);
    (void)hipMalloc(&obuf, (256u << 20));
    (void)hipMalloc(&out, 64);
    (void)hipMemset(buf, 1, 4 << 20);
    (void)hipMemset(obuf, 0, 256u << 20);
    run<0>("no stores", buf, obuf, out);
    run<1>("16 rows x 64 B, pitch 2048", buf, obuf, out);
    run<2>("16 rows x 64 B, pitch 1920", buf, obuf, out);
    run<3>("8 rows x 128 B (whole lines), pitch 1920", buf, obuf, out);
    run<4>("4 rows x 256 B, pitch 1920", buf, obuf, out);
    run<5>("1 KB contiguous", buf, obuf, out);
    run<6>("16 rows x 64 B, pitch 1920, nontemporal", buf, obuf, out);
    run<7>("16 rows x 64 B, pitch 1920, 4 MB region", buf, obuf, out);
    run<8>("16 rows x 64 B, pitch 1920, right after the loads", buf, obuf, out);
    return 0;
}
