// overlap_probe.hip — does row-per-lane tap traffic overlap with VALU work inside a CU when the
// same waves do both (as recon.hip does), vs when waves specialise? (dev tool)
//   hipcc -O3 --offload-arch=gfx950 tools/overlap_probe.hip -o tools/overlap_probe.bin
// Each wave runs ITER iterations; an iteration issues NL row-per-lane buffer loads (b128, random
// rows of a 4 MB window: L2 hits, 64 lines per instruction) whose data is consumed one iteration
// later, and NV rounds of dependent-pair VALU work (v_lerp_u8 / alignbyte chains, VOP3).
//   mode 0: loads only   1: VALU only   2: both in every wave   3: waves 0,1 of each workgroup
//   load-only, waves 2,3 VALU-only (same total work per workgroup as mode 2 with 2x per wave)
// 4 waves per workgroup, LDS-padded so 4 workgroups share a CU (16 waves, as the kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 64
#define CHECK(x)                                                            \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);     \
            return 1;                                                       \
        }                                                                   \
    } while (0)

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// EXTRA bits: 1 two row stores per iteration (16 rows x 4 lanes, 64 B/row), 2 sixteen ds_bpermute
// per iteration, 4 loads from a 64 MB window (MALL / HBM) instead of 4 MB, 8 LDS write+read round
// trip (ds_write_b32 + dependent ds_read_b32 x 8)
template <int MODE, int NL, int NV, int EXTRA>
__global__ __launch_bounds__(256) void kern(const uint8_t* __restrict__ buf, uint32_t* __restrict__ out) {
    __shared__ uint32_t pad[9000];  // ~36 KB: 4 workgroups per CU
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * 4 + wave;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 64 << 20, 0x00020000);
    const uint32_t rmask = (EXTRA & 4) ? 32767u : 2047u;
    bool do_load = MODE == 0 || MODE == 2 || (MODE == 3 && wave < 2);
    bool do_valu = MODE == 1 || MODE == 2 || (MODE == 3 && wave >= 2);
    const int mult = MODE == 3 ? 2 : 1;
    uint32_t a[NL][4];
#pragma unroll
    for (int i = 0; i < NL; i++) a[i][0] = a[i][1] = a[i][2] = a[i][3] = lane;
    uint32_t x0 = lane * 0x01010101u, x1 = gw, x2 = x0 ^ 0x5a5a5a5a, x3 = x1 * 3u;
    for (int it = 0; it < ITER; it++) {
        if (do_load) {
            for (int m = 0; m < mult; m++) {
                uint32_t acc = 0;
#pragma unroll
                for (int i = 0; i < NL; i++) acc ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
                x1 ^= acc;
#pragma unroll
                for (int i = 0; i < NL; i++) {
                    const uint32_t h = hsh(gw * 977u + (uint32_t)(it * mult + m) * 131u + i * 7919u + lane);
                    const uint32_t off = (h & rmask) * 2048u + ((h >> 20) & 0x1ffu) * 4u;
                    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
                    a[i][0] = v.x; a[i][1] = v.y; a[i][2] = v.z; a[i][3] = v.w;
                }
            }
        }
        if (do_valu) {
            for (int m = 0; m < mult * NV; m++) {
                // 8 VOP3 ops in two independent chains (like the prediction arithmetic)
                x0 = __builtin_amdgcn_alignbyte(x1, x0, m & 3);
                x2 = __builtin_amdgcn_alignbyte(x3, x2, (m + 1) & 3);
                x0 = __builtin_amdgcn_lerp(x0, x2, 0x01010101u);
                x2 = __builtin_amdgcn_lerp(x2, x1, 0x01010101u);
                x1 = __builtin_amdgcn_perm(x0, x1, 0x05040100u);
                x3 = __builtin_amdgcn_perm(x2, x3, 0x07060302u);
                x1 = __builtin_amdgcn_lerp(x1, x3, 0x01010101u);
                x3 = __builtin_amdgcn_alignbyte(x0, x3, 1);
            }
            if (EXTRA & 2) {
#pragma unroll
                for (int i = 0; i < 16; i++) x0 ^= (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + 4 + i) & 63) * 4, (int)x1);
            }
            if (EXTRA & 8) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    pad[(threadIdx.x * 8 + i) & 8191] = x2 + i;
                    __builtin_amdgcn_wave_barrier();
                    x1 += pad[(threadIdx.x * 8 + ((i + 3) & 7)) & 8191];
                }
            }
            if (EXTRA & 1) {
                const uint32_t h = hsh(gw * 31u + it);
                uint8_t* o = (uint8_t*)buf + (16u << 20) + ((h & 1023u) * 16u + (lane >> 2)) * 2048u + (lane & 3) * 16u;
                *(uint4*)o = make_uint4(x0, x1, x2, x3);
                *(uint4*)(o + 1024) = make_uint4(x3, x1, x2, x0);
            }
        }
    }
    uint32_t acc = x0 ^ x1 ^ x2 ^ x3;
#pragma unroll
    for (int i = 0; i < NL; i++) acc ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (pad[(threadIdx.x + 1) & 255] == 0x12345678u) out[0] = acc;
}

template <int MODE, int NL, int NV, int EXTRA>
static float run(const uint8_t* buf, uint32_t* out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(a);
        hipLaunchKernelGGL((kern<MODE, NL, NV, EXTRA>), dim3(4096), dim3(256), 0, 0, buf, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
    }
    return ms;
}

template <int NL, int NV, int EXTRA = 0>
static void sweep() {
    uint8_t* buf;
    uint32_t* out;
    hipMalloc(&buf, (64 << 20) + 4096);
    hipMalloc(&out, 64);
    hipMemset(buf, 1, 64 << 20);
    const float l = run<0, NL, NV, EXTRA>(buf, out), v = run<1, NL, NV, EXTRA>(buf, out), both = run<2, NL, NV, EXTRA>(buf, out),
                sp = run<3, NL, NV, EXTRA>(buf, out);
    printf("X%2d NL %2d NV %3d (VALU ops/iter %4d): loads %.3f ms  valu %.3f ms  sum %.3f  max %.3f | mixed %.3f  specialised %.3f\n",
           EXTRA, NL, NV, NV * 8, l, v, l + v, l > v ? l : v, both, sp);
    hipFree(buf);
    hipFree(out);
}

int main() {
    sweep<8, 100>();
    sweep<8, 100, 1>();
    sweep<8, 100, 2>();
    sweep<8, 100, 4>();
    sweep<8, 100, 8>();
    sweep<8, 100, 15>();
    sweep<8, 50, 15>();
    return 0;
}
