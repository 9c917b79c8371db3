// valu_rate2.hip -- issue cost of a wider set of gfx950 VALU instructions
// (which 32-bit ops issue at the fast rate measured for v_add_u32 / v_xor_b32
// in profiles/r02_valu_rate.jsonl), to pick the instruction mix of the x87
// soft add.  Not part of the product: a probe for DESIGN.md 4.
// Each kernel: CH independent chains of one instruction per lane, WPS waves
// per SIMD on every CU; prints cycles per wave64 instruction per SIMD at the
// device's reported clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 2048
#define CH 8

// two-operand forms on a 32-bit chain: "op %0, %0, %1"
#define K32(NAME, ASM)                                                                \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, unsigned s)            \
    {                                                                                 \
        unsigned x[CH];                                                               \
        for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;                          \
        for (int it = 0; it < ITERS; it++) {                                          \
            _Pragma("unroll") for (int c = 0; c < CH; c++)                            \
                asm volatile(ASM : "+v"(x[c]) : "v"(s), "v"(s + 1u) : "vcc", "s8", "s9", "s10", "s11");                 \
        }                                                                             \
        unsigned a = 0;                                                               \
        for (int c = 0; c < CH; c++) a ^= x[c];                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a;                                      \
    }
#define K64(NAME, ASM)                                                                \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, unsigned s)            \
    {                                                                                 \
        unsigned long long x[CH];                                                     \
        for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;                          \
        const unsigned long long s64 = s;                                             \
        for (int it = 0; it < ITERS; it++) {                                          \
            _Pragma("unroll") for (int c = 0; c < CH; c++)                            \
                asm volatile(ASM : "+v"(x[c]) : "v"(s), "v"(s64) : "vcc", "s8", "s9", "s10", "s11");                    \
        }                                                                             \
        unsigned long long a = 0;                                                     \
        for (int c = 0; c < CH; c++) a ^= x[c];                                       \
        out[blockIdx.x * 256 + threadIdx.x] = (unsigned) (a ^ (a >> 32));             \
    }

K32(k_add, "v_add_u32 %0, %0, %1")
K32(k_sub, "v_sub_u32 %0, %0, %1")
K32(k_and, "v_and_b32 %0, %0, %1")
K32(k_or, "v_or_b32 %0, %0, %1")
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_not, "v_not_b32 %0, %0")
K32(k_mov, "v_mov_b32 %0, %1")
K32(k_min, "v_min_u32 %0, %0, %1")
K32(k_max, "v_max_u32 %0, %0, %1")
K32(k_shl, "v_lshlrev_b32 %0, %1, %0")
K32(k_shr, "v_lshrrev_b32 %0, %1, %0")
K32(k_ashr, "v_ashrrev_i32 %0, %1, %0")
K32(k_shl_imm, "v_lshlrev_b32 %0, 3, %0")
K32(k_add3, "v_add3_u32 %0, %0, %1, %2")
K32(k_or3, "v_or3_b32 %0, %0, %1, %2")
K32(k_lshl_or, "v_lshl_or_b32 %0, %0, %1, %2")
K32(k_lshl_add, "v_lshl_add_u32 %0, %0, %1, %2")
K32(k_add_lshl, "v_add_lshl_u32 %0, %0, %1, %2")
K32(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
K32(k_xad, "v_xad_u32 %0, %0, %1, %2")
K32(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
K32(k_bfe, "v_bfe_u32 %0, %0, %1, %2")
K32(k_align, "v_alignbit_b32 %0, %0, %1, %2")
K32(k_perm, "v_perm_b32 %0, %0, %1, %2")
K32(k_med3, "v_med3_u32 %0, %0, %1, %2")
K32(k_ffbh, "v_ffbh_u32 %0, %0")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
K32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
K32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_addco, "v_add_co_u32 %0, vcc, %0, %1")
K32(k_addc_vcc, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
K32(k_cnd_s, "v_cndmask_b32 %0, %0, %1, s[8:9]")
K32(k_cmp_s, "v_cmp_gt_u32 s[8:9], %0, %1")
K32(k_cmp_vcc, "v_cmp_gt_u32 vcc, %0, %1")
K32(k_cmpx, "v_cmp_gt_u32_e64 s[10:11], %0, %1\n\tv_cndmask_b32 %0, %0, %1, s[10:11]")
K32(k_subrev_co, "v_sub_co_u32 %0, vcc, %0, %1")
K32(k_pk_add16, "v_pk_add_u16 %0, %0, %1")
K32(k_sad, "v_sad_u32 %0, %0, %1, %2")
K32(k_add_f32, "v_add_f32 %0, %0, %1")
K32(k_cvt, "v_cvt_f32_u32 %0, %0")
K64(k_shl64, "v_lshlrev_b64 %0, %1, %0")
K64(k_shr64, "v_lshrrev_b64 %0, %1, %0")
K64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %2")
K64(k_cmp64, "v_cmp_gt_u64 s[8:9], %0, %2")
K64(k_add_f64, "v_add_f64 %0, %0, %2")
K64(k_fma_f64, "v_fma_f64 %0, %0, %2, %2")
K64(k_mad64, "v_mad_u64_u32 %0, s[8:9], %1, %1, %0")
K64(k_pkmov, "v_pk_mov_b32 %0, %2, %0 op_sel:[0,1]")

int main()
{
    hipDeviceProp_t p;
    (void) hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int wps = getenv("WPS") ? atoi(getenv("WPS")) : 8;
    const int blocks = cus * wps;  // wps waves per SIMD: wps blocks of 4 waves per CU
    unsigned *out;
    hipMalloc(&out, (size_t) blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char *name; void (*k)(unsigned *, unsigned); int per; } ks[] = {
#define E(K, N, PER) {N, K, PER}
        E(k_add, "v_add_u32", 1), E(k_sub, "v_sub_u32", 1), E(k_and, "v_and_b32", 1),
        E(k_or, "v_or_b32", 1), E(k_xor, "v_xor_b32", 1), E(k_not, "v_not_b32", 1),
        E(k_mov, "v_mov_b32", 1), E(k_min, "v_min_u32", 1), E(k_max, "v_max_u32", 1),
        E(k_shl, "v_lshlrev_b32", 1), E(k_shr, "v_lshrrev_b32", 1), E(k_ashr, "v_ashrrev_i32", 1),
        E(k_shl_imm, "v_lshlrev_b32 imm", 1), E(k_add3, "v_add3_u32", 1),
        E(k_or3, "v_or3_b32", 1), E(k_lshl_or, "v_lshl_or_b32", 1), E(k_lshl_add, "v_lshl_add_u32", 1),
        E(k_add_lshl, "v_add_lshl_u32", 1), E(k_and_or, "v_and_or_b32", 1), E(k_xad, "v_xad_u32", 1),
        E(k_bfi, "v_bfi_b32", 1), E(k_bfe, "v_bfe_u32", 1), E(k_align, "v_alignbit_b32", 1),
        E(k_perm, "v_perm_b32", 1), E(k_med3, "v_med3_u32", 1), E(k_ffbh, "v_ffbh_u32", 1),
        E(k_bitop3, "v_bitop3_b32", 1), E(k_mul_lo, "v_mul_lo_u32", 1), E(k_mul_hi, "v_mul_hi_u32", 1),
        E(k_mad24, "v_mad_u32_u24", 1), E(k_addco, "v_add_co_u32 (vcc out)", 1),
        E(k_addc_vcc, "v_addc_co_u32 (vcc in/out)", 1), E(k_cnd_s, "v_cndmask_b32 (sgpr pair)", 1),
        E(k_cmp_s, "v_cmp_gt_u32 -> sgpr pair", 1), E(k_cmp_vcc, "v_cmp_gt_u32 -> vcc", 1),
        E(k_cmpx, "v_cmp_e64 + v_cndmask (pair)", 2), E(k_subrev_co, "v_sub_co_u32 (vcc out)", 1),
        E(k_pk_add16, "v_pk_add_u16", 1), E(k_sad, "v_sad_u32", 1), E(k_add_f32, "v_add_f32", 1),
        E(k_cvt, "v_cvt_f32_u32", 1), E(k_shl64, "v_lshlrev_b64", 1), E(k_shr64, "v_lshrrev_b64", 1),
        E(k_lshladd64, "v_lshl_add_u64", 1), E(k_cmp64, "v_cmp_gt_u64 -> sgpr pair", 1),
        E(k_add_f64, "v_add_f64", 1), E(k_fma_f64, "v_fma_f64", 1), E(k_mad64, "v_mad_u64_u32", 1),
        E(k_pkmov, "v_pk_mov_b32", 1),
    };
    for (auto &k : ks) {
        float best = 1e30f;
        for (int r = 0; r < 4; r++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 3u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        const double ins = (double) wps * ITERS * CH * k.per;
        const double cyc = best * 1e-3 * p.clockRate * 1e3;  // clockRate in kHz
        printf("{\"instr\": \"%s\", \"cycles\": %.2f, \"ms\": %.4f, \"clock_MHz\": %d, \"waves_per_SIMD\": %d}\n",
               k.name, cyc / ins, best, p.clockRate / 1000, wps);
    }
    hipFree(out);
    return 0;
}
