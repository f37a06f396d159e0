// issue_bench.hip — SIMD issue cost of the VALU encodings the reconstruct loops use (dev tool).
//   hipcc -O3 --offload-arch=gfx950 tools/issue_bench.hip -o tools/issue_bench.bin && tools/issue_bench.bin
// Every kernel runs a loop of inline-asm blocks: 8 independent register chains, one instruction
// form (or a fixed mix of forms) per block, so the compiler can neither fold nor reorder them.
// Waves per SIMD = workgroups per CU (4-wave workgroups, grid = 256 CUs x W).  Cycles come from
// s_memtime around the loop in each wave (shader clock, MI355X_MICROARCH.md; s_memrealtime, 100 MHz,
// beside it gives that clock's rate), reported as SIMD
// cycles per wave64 instruction: (cycles per wave per instruction) / (waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 512

#define R8 "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
// one instruction form over the 8 chains; %8 = a VGPR constant, %9 = an SGPR constant
#define FORM8(ins) \
    ins(0) ins(1) ins(2) ins(3) ins(4) ins(5) ins(6) ins(7)

#define ADD_E32(i) "v_add_u32_e32 %" #i ", %8, %" #i "\n"
#define ADD_E64(i) "v_add_u32_e64 %" #i ", %8, %" #i "\n"
#define ADD_SG(i) "v_add_u32_e32 %" #i ", %9, %" #i "\n"
#define AND_LIT(i) "v_and_b32_e32 %" #i ", 0x7fff8, %" #i "\n"
#define XOR_E32(i) "v_xor_b32_e32 %" #i ", %8, %" #i "\n"
#define LSHL_E32(i) "v_lshlrev_b32_e32 %" #i ", 3, %" #i "\n"
#define MUL24_E32(i) "v_mul_u32_u24_e32 %" #i ", %8, %" #i "\n"
#define MULHI24_E32(i) "v_mul_hi_i32_i24_e32 %" #i ", %8, %" #i "\n"
#define MUL24_SDWA(i) "v_mul_i32_i24_sdwa %" #i ", sext(%" #i "), %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
#define ADD_SDWA(i) "v_add_u32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
#define CND_E32(i) "v_cndmask_b32_e32 %" #i ", %8, %" #i ", vcc\n"
#define CND_E64(i) "v_cndmask_b32_e64 %" #i ", %8, %" #i ", s[4:5]\n"
#define PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n"
#define ALIGNB(i) "v_alignbyte_b32 %" #i ", %" #i ", %8, %8\n"
#define LERP(i) "v_lerp_u8 %" #i ", %" #i ", %8, %9\n"
#define PKADD(i) "v_pk_add_i16 %" #i ", %" #i ", %8 clamp\n"
#define PKSUB(i) "v_pk_sub_i16 %" #i ", %" #i ", %8 clamp\n"
#define PKLSH(i) "v_pk_lshlrev_b16 %" #i ", 1, %" #i "\n"
#define ADD3(i) "v_add3_u32 %" #i ", %" #i ", %8, %8\n"
#define BFE(i) "v_bfe_u32 %" #i ", %" #i ", 8, 8\n"
#define ANDOR(i) "v_and_or_b32 %" #i ", %" #i ", %8, %8\n"
#define SATPK(i) "v_sat_pk_u8_i16_e32 %" #i ", %" #i "\n"
#define MOVDPP(i) "v_mov_b32_dpp %" #i ", %" #i " row_shl:1 row_mask:0xf bank_mask:0xf\n"
#define ADD_I16_E32(i) "v_add_u16_e32 %" #i ", %8, %" #i "\n"
#define MED3(i) "v_med3_i32 %" #i ", %" #i ", %8, %9\n"
#define ASHR_E32(i) "v_ashrrev_i32_e32 %" #i ", 16, %" #i "\n"
#define BFI(i) "v_bfi_b32 %" #i ", %8, %" #i ", %8\n"
#define LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 16, %8\n"
#define ADD_INL(i) "v_add_u32_e32 %" #i ", 3, %" #i "\n"
#define LSHL_VV(i) "v_lshlrev_b32_e32 %" #i ", %8, %" #i "\n"
#define LSHL_SG(i) "v_lshlrev_b32_e32 %" #i ", %9, %" #i "\n"
#define AND_VV(i) "v_and_b32_e32 %" #i ", %8, %" #i "\n"
#define AND_INL(i) "v_and_b32_e32 %" #i ", 64, %" #i "\n"
#define OR_LIT(i) "v_or_b32_e32 %" #i ", 0x12345, %" #i "\n"
#define MOV_VV(i) "v_mov_b32_e32 %" #i ", %8\n"
#define CMP_CND(i) "v_cmp_ne_u32_e32 vcc, %" #i ", %8\n v_cndmask_b32_e32 %" #i ", %8, %" #i ", vcc\n"
#define CND_E64V(i) "v_cndmask_b32_e64 %" #i ", %8, %" #i ", vcc\n"
#define OR3(i) "v_or3_b32 %" #i ", %" #i ", %8, %8\n"
#define SUB_VV(i) "v_sub_u32_e32 %" #i ", %8, %" #i "\n"
#define LSHR_INL(i) "v_lshrrev_b32_e32 %" #i ", 3, %" #i "\n"
#define ASHR_VV(i) "v_ashrrev_i32_e32 %" #i ", %8, %" #i "\n"
#define MUL24_INL(i) "v_mul_u32_u24_e32 %" #i ", 3, %" #i "\n"
// mixes: a VOP3 form and a VOP2 form alternating, and pairs
#define MIX_PERM_ADD(i) PERM(i) ADD_E32(i)
#define MIX_PKADD_ADD(i) PKADD(i) ADD_E32(i)
#define MIX_LERP_XOR(i) LERP(i) XOR_E32(i)

template <int F>
__device__ __forceinline__ void body(uint32_t& v0, uint32_t& v1, uint32_t& v2, uint32_t& v3, uint32_t& v4,
                                     uint32_t& v5, uint32_t& v6, uint32_t& v7, uint32_t k, uint32_t s) {
#define CASE(n, ins) \
    if constexpr (F == n) asm volatile(FORM8(ins) : R8 : "v"(k), "s"(s) : "vcc", "s4", "s5");
    CASE(0, ADD_E32)
    CASE(1, ADD_E64)
    CASE(2, ADD_SG)
    CASE(3, AND_LIT)
    CASE(4, XOR_E32)
    CASE(5, LSHL_E32)
    CASE(6, MUL24_E32)
    CASE(7, MULHI24_E32)
    CASE(8, MUL24_SDWA)
    CASE(9, ADD_SDWA)
    CASE(10, CND_E32)
    CASE(11, CND_E64)
    CASE(12, PERM)
    CASE(13, ALIGNB)
    CASE(14, LERP)
    CASE(15, PKADD)
    CASE(16, PKSUB)
    CASE(17, PKLSH)
    CASE(18, ADD3)
    CASE(19, BFE)
    CASE(20, ANDOR)
    CASE(21, SATPK)
    CASE(22, MOVDPP)
    CASE(23, ADD_I16_E32)
    CASE(24, MED3)
    CASE(25, ASHR_E32)
    CASE(26, BFI)
    CASE(27, LSHLOR)
    CASE(28, MIX_PERM_ADD)
    CASE(29, MIX_PKADD_ADD)
    CASE(30, MIX_LERP_XOR)
    CASE(31, ADD_INL)
    CASE(32, LSHL_VV)
    CASE(33, LSHL_SG)
    CASE(34, AND_VV)
    CASE(35, AND_INL)
    CASE(36, OR_LIT)
    CASE(37, MOV_VV)
    CASE(38, CMP_CND)
    CASE(39, CND_E64V)
    CASE(40, OR3)
    CASE(41, SUB_VV)
    CASE(42, LSHR_INL)
    CASE(43, ASHR_VV)
    CASE(44, MUL24_INL)
#undef CASE
}
constexpr int kForms = 45;
constexpr int kInstr[kForms] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 16, 16, 16,
                                8, 8, 8, 8, 8, 8, 8, 16, 8, 8, 8, 8, 8, 8};
const char* kName[kForms] = {"v_add_u32_e32 (VOP2)", "v_add_u32_e64 (VOP3 enc)", "v_add_u32_e32 sgpr src0", "v_and_b32_e32 literal",
                             "v_xor_b32_e32", "v_lshlrev_b32_e32 inline", "v_mul_u32_u24_e32", "v_mul_hi_i32_i24_e32",
                             "v_mul_i32_i24_sdwa", "v_add_u32_sdwa", "v_cndmask_b32_e32 vcc", "v_cndmask_b32_e64 sgpr",
                             "v_perm_b32", "v_alignbyte_b32", "v_lerp_u8", "v_pk_add_i16 clamp", "v_pk_sub_i16 clamp",
                             "v_pk_lshlrev_b16", "v_add3_u32", "v_bfe_u32", "v_and_or_b32", "v_sat_pk_u8_i16_e32",
                             "v_mov_b32_dpp row_shl", "v_add_u16_e32", "v_med3_i32", "v_ashrrev_i32_e32", "v_bfi_b32",
                             "v_lshl_or_b32", "mix perm + add_e32", "mix pk_add + add_e32", "mix lerp + xor_e32",
                             "v_add_u32_e32 inline 3", "v_lshlrev_b32_e32 vgpr", "v_lshlrev_b32_e32 sgpr", "v_and_b32_e32 vv",
                             "v_and_b32_e32 inline 64", "v_or_b32_e32 literal", "v_mov_b32_e32 v", "v_cmp_e32 + cndmask_e32",
                             "v_cndmask_b32_e64 vcc", "v_or3_b32", "v_sub_u32_e32 vv", "v_lshrrev_b32_e32 inline",
                             "v_ashrrev_i32_e32 vgpr", "v_mul_u32_u24_e32 inline"};

template <int F>
__global__ __launch_bounds__(256) void kern(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    uint32_t v0 = seed * (threadIdx.x + 1), v1 = v0 ^ 1, v2 = v0 ^ 2, v3 = v0 ^ 3, v4 = v0 ^ 4, v5 = v0 ^ 5, v6 = v0 ^ 6,
             v7 = v0 ^ 7;
    const uint32_t k = seed ^ 0x5bd1e995u;
    const uint32_t s = __builtin_amdgcn_readfirstlane(seed) | 0x01010101u;
    asm volatile("s_mov_b64 vcc, -1\n s_mov_b64 s[4:5], -1" ::: "vcc", "s4", "s5");
    uint64_t t0, r0;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0)::"memory");
    for (int it = 0; it < ITERS; it++) {
        body<F>(v0, v1, v2, v3, v4, v5, v6, v7, k, s);
        body<F>(v0, v1, v2, v3, v4, v5, v6, v7, k, s);
        body<F>(v0, v1, v2, v3, v4, v5, v6, v7, k, s);
        body<F>(v0, v1, v2, v3, v4, v5, v6, v7, k, s);
    }
    uint64_t t1, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
    const uint32_t r = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
    if (r == 0x12345678u) out[0] = r;
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(cyc, (unsigned long long)(t1 - t0));
        atomicAdd(cyc + 1, (unsigned long long)(r1 - r0));
    }
}

template <int F>
static void run(int waves_per_simd, unsigned long long* dcyc, uint32_t* out) {
    const int blocks = 256 * waves_per_simd;
    double cpi = 0, ghz = 0;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipMemset(dcyc, 0, 16);
        hipLaunchKernelGGL(kern<F>, dim3(blocks), dim3(256), 0, 0, dcyc, out, 12345u + rep);
        (void)hipDeviceSynchronize();
        unsigned long long cc[2] = {0, 0};
        (void)hipMemcpy(cc, dcyc, 16, hipMemcpyDeviceToHost);
        const unsigned long long c = cc[0];
        ghz = (double)cc[0] / (double)cc[1] * 0.1;  // s_memrealtime: 100 MHz
        const double waves = blocks * 4.0, instr = (double)ITERS * 4 * kInstr[F];
        cpi = (double)c / waves / instr / waves_per_simd;  // SIMD cycles per wave-instruction
    }
    printf("%-28s W=%d  %5.2f SIMD cycles/instr  (s_memtime %.2f GHz)\n", kName[F], waves_per_simd, cpi, ghz);
}

template <int F>
static void all(unsigned long long* dcyc, uint32_t* out) {
    for (int w : {1, 4})
        run<F>(w, dcyc, out);
    if constexpr (F + 1 < kForms) all<F + 1>(dcyc, out);
}

int main() {
    unsigned long long* dcyc;
    uint32_t* out;
    (void)hipMalloc(&dcyc, 16);
    (void)hipMalloc(&out, 64);
    all<0>(dcyc, out);
    return 0;
}
