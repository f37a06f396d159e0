// valu_bench.hip — issue rate of the VALU ops the reconstruct kernel leans on (dev tool).
//   hipcc -O3 --offload-arch=gfx950 tools/valu_bench.hip -o tools/valu_bench.bin && tools/valu_bench.bin
// Each kernel runs 8 independent chains of one op per lane (2048 WGs x 256 threads); prints
// cycles per wave-instruction per SIMD at 2.4 GHz (2.0 = full rate for wave64 on SIMD32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N 2048
typedef short short2_t __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    const uint32_t k = seed ^ 0x5bd1e995u;
    for (int it = 0; it < N; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) v[i] = v[i] + k;                                               // v_add_u32
            if (OP == 1) v[i] = __builtin_amdgcn_perm(v[i], k, 0x05040100u);            // v_perm_b32
            if (OP == 2) v[i] = __builtin_amdgcn_alignbyte(v[i], k, v[(i + 1) & 7]);   // v_alignbyte_b32
            if (OP == 3) v[i] = __builtin_amdgcn_lerp(v[i], k, 0x01010101u);            // v_lerp_u8
            if (OP == 4) v[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(
                                    __builtin_bit_cast(short2_t, v[i]), __builtin_bit_cast(short2_t, k)));  // v_pk_add_i16 clamp
            if (OP == 5) v[i] = (uint32_t)(((int)(short)v[i] * (int)(short)k) >> 16);  // v_mul_i32_i24 + shift
            if (OP == 6) v[i] = v[i] ? v[i] : k;                                        // v_cndmask
            if (OP == 7) v[i] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(v[i] & 252), (int)v[i]);  // ds_bpermute
            if (OP == 8) v[i] = __builtin_amdgcn_ubfe(v[i], k & 31, 8);                 // v_bfe_u32
            if (OP == 9) v[i] = v[i] * v[(i + 1) & 7];                                  // v_mul_lo_u32
            if (OP == 10) v[i] = v[i] + v[(i + 3) & 7];                                 // v_add_u32 (no folding)
            if (OP == 11) v[i] = v[i] ^ v[(i + 3) & 7];                                 // v_xor_b32
            if (OP == 12) v[i] = __builtin_bit_cast(uint32_t, __builtin_fmaf(__builtin_bit_cast(float, v[i]), 1.0001f, __builtin_bit_cast(float, k)));  // v_fma_f32
            if (OP == 14) v[i] = __builtin_amdgcn_mov_dpp(v[i], 0x101, 0xf, 0xf, false);      // v_mov_b32_dpp row_shl:1
            if (OP == 15) v[i] = __builtin_amdgcn_mov_dpp(v[i], 0x153, 0xf, 0xf, false) ^ v[(i + 1) & 7];  // dpp newbcast + xor
            if (OP == 13) v[i] = __builtin_amdgcn_perm(v[i], v[(i + 3) & 7], 0x05040100u);  // v_perm, 2 VGPR operands
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r ^= v[i];
    if (r == 0x12345678u) out[0] = r;
}

template <int OP>
static void run(const char* name, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 2048;
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, 12345u + rep);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    const double instr_per_simd = (double)blocks * 4 * N * 8 / 1024.0;
    printf("%-28s %7.3f ms  %5.2f cycles/wave-instr/SIMD\n", name, ms, ms * 1e-3 * 2.4e9 / instr_per_simd);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 64);
    run<0>("v_add_u32", out);
    run<1>("v_perm_b32", out);
    run<2>("v_alignbyte_b32", out);
    run<3>("v_lerp_u8", out);
    run<4>("v_pk_add_i16 clamp", out);
    run<5>("mul i24 + shift", out);
    run<6>("v_cndmask", out);
    run<7>("ds_bpermute", out);
    run<8>("v_bfe_u32", out);
    run<9>("v_mul_lo_u32", out);
    run<10>("v_add_u32 (cross-chain)", out);
    run<11>("v_xor_b32 (cross-chain)", out);
    run<12>("v_fma_f32", out);
    run<13>("v_perm_b32 (2 VGPR srcs)", out);
    run<14>("v_mov_b32_dpp row_shl:1", out);
    run<15>("dpp row_newbcast + v_xor", out);
    return 0;
}
