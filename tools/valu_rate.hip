// valu_rate.hip -- issue cost of the VALU instructions the x87 soft-float
// leans on (64-bit shifts / adds / compares vs 32-bit ops), gfx950.  Not part
// of the product: a probe for DESIGN.md 4.  Each kernel runs 8 independent
// chains of one instruction per lane, 4 waves per SIMD, all CUs; prints the
// cycles per wave64 instruction per SIMD (clock from hipDeviceProp).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 4096
#define CH 8

#define KERNEL(NAME, DECL, BODY, SINK)                                          \
    __global__ __launch_bounds__(256) void NAME(unsigned long long *out, unsigned s) \
    {                                                                            \
        DECL;                                                                    \
        for (int it = 0; it < ITERS; it++) {                                     \
            _Pragma("unroll") for (int c = 0; c < CH; c++) { BODY; }             \
        }                                                                        \
        SINK;                                                                    \
    }

KERNEL(k_shl64,
       unsigned long long x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(x[c]) : "v"(s)),
       unsigned long long a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_add64,
       unsigned long long x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[c]) : "v"((unsigned long long) s)),
       unsigned long long a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_cmp64,
       unsigned long long x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_cmp_gt_u64 vcc, %0, %1" : : "v"(x[c]), "v"((unsigned long long) s) : "vcc"),
       unsigned long long a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_shl32,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_cnd32,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_addc32,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x[c]) : "v"(s) : "vcc"),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)

KERNEL(k_fma32,
       float x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[c]) : "v"((float) s)),
       float a = 0; for (int c = 0; c < CH; c++) a += x[c]; out[blockIdx.x * 256 + threadIdx.x] = (unsigned long long) a)
KERNEL(k_add32,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_xor32,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_cnds,
       unsigned x[CH]; unsigned long long m = __builtin_amdgcn_read_exec(); for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c,
       asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(s), "s"(m)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)

KERNEL(k_cndv,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;
       asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(threadIdx.x), "v"(s) : "vcc"),
       asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)
KERNEL(k_cnde,
       unsigned x[CH]; for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;
       asm volatile("s_mov_b64 vcc, exec" : : : "vcc"),
       asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(s)),
       unsigned a = 0; for (int c = 0; c < CH; c++) a ^= x[c]; out[blockIdx.x * 256 + threadIdx.x] = a)

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int wps = getenv("WPS") ? atoi(getenv("WPS")) : 4;
    const int blocks = cus * wps;  // wps waves per SIMD: wps blocks of 4 waves per CU
    unsigned long long *out;
    hipMalloc(&out, (size_t) blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char *name; void (*k)(unsigned long long *, unsigned); int per; } ks[] = {
        {"v_lshlrev_b64", k_shl64, 1}, {"v_lshl_add_u64", k_add64, 1}, {"v_cmp_gt_u64", k_cmp64, 1},
        {"v_lshlrev_b32", k_shl32, 1}, {"v_cndmask_b32 (vcc)", k_cnd32, 1},
        {"v_cndmask_b32 (sgpr pair)", k_cnds, 1},
        {"v_cndmask_b32 (vcc from v_cmp)", k_cndv, 1}, {"v_cndmask_b32 (vcc = exec)", k_cnde, 1}, {"v_fma_f32", k_fma32, 1}, {"v_add_u32", k_add32, 1},
        {"v_xor_b32", k_xor32, 1}, {"v_add_co+v_addc (pair)", k_addc32, 2}};
    for (auto &k : ks) {
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 3u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        // wave-instructions per SIMD: 4 waves * ITERS * CH * per
        const double ins = (double) wps * ITERS * CH * k.per;
        const double cyc = best * 1e-3 * p.clockRate * 1e3;  // clockRate in kHz
        printf("{\"instr\": \"%s\", \"ms\": %.4f, \"cycles_per_wave_instr_per_SIMD\": %.2f, \"clock_MHz\": %d, \"waves_per_SIMD\": %d}\n",
               k.name, best, cyc / ins, p.clockRate / 1000, wps);
    }
    hipFree(out);
    return 0;
}
