// Microbenchmark: issue cost of a few VALU instructions on gfx950 (wave64), 8 independent
// chains per lane, many waves per SIMD.  hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#define N 4096
#define OP(name, asmstr)                                                                 \
    __global__ void name(unsigned* o, unsigned s) {                                      \
        unsigned a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 ^ 4,   \
                 a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                                  \
        for (int i = 0; i < N; ++i) {                                                    \
            asm volatile(asmstr " %0, %0, %8\n" asmstr " %1, %1, %8\n" asmstr " %2, %2, %8\n" \
                         asmstr " %3, %3, %8\n" asmstr " %4, %4, %8\n" asmstr " %5, %5, %8\n" \
                         asmstr " %6, %6, %8\n" asmstr " %7, %7, %8\n"                  \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                           "+v"(a6), "+v"(a7)                                            \
                         : "v"(s));                                                      \
        }                                                                                \
        o[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
    }
#define OP3(name, asmstr)                                                                \
    __global__ void name(unsigned* o, unsigned s) {                                      \
        unsigned a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 ^ 4,   \
                 a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                                  \
        for (int i = 0; i < N; ++i) {                                                    \
            asm volatile(asmstr " %0, %0, %8, %9\n" asmstr " %1, %1, %8, %9\n" asmstr " %2, %2, %8, %9\n" \
                         asmstr " %3, %3, %8, %9\n" asmstr " %4, %4, %8, %9\n" asmstr " %5, %5, %8, %9\n" \
                         asmstr " %6, %6, %8, %9\n" asmstr " %7, %7, %8, %9\n"                  \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                           "+v"(a6), "+v"(a7)                                            \
                         : "v"(s), "v"(s + 1));                                          \
        }                                                                                \
        o[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
    }
#define OP1(name, asmstr)                                                                \
    __global__ void name(unsigned* o, unsigned s) {                                      \
        unsigned a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 ^ 4,   \
                 a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;                                  \
        for (int i = 0; i < N; ++i) {                                                    \
            asm volatile(asmstr " %0, %1\n" asmstr " %1, %2\n" asmstr " %2, %3\n"     \
                         asmstr " %3, %4\n" asmstr " %4, %5\n" asmstr " %5, %6\n"     \
                         asmstr " %6, %7\n" asmstr " %7, %0\n"                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                           "+v"(a6), "+v"(a7)                                            \
                         : "v"(s));                                                      \
        }                                                                                \
        o[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
    }
OP(k_xor, "v_xor_b32")
OP(k_or, "v_or_b32")
OP(k_lshl, "v_lshlrev_b32")
OP(k_ashr, "v_ashrrev_i32")
OP(k_addf, "v_add_f32")
OP1(k_mov, "v_mov_b32")
OP1(k_cvtfu, "v_cvt_f32_u32")
OP1(k_cvtuf, "v_cvt_u32_f32")
OP1(k_rndne, "v_rndne_f32")
OP1(k_ub0, "v_cvt_f32_ubyte0")
OP(k_addu16, "v_add_u16")
OP(k_minu16, "v_min_u16")
OP(k_subu16, "v_sub_u16")
OP(k_maxf, "v_max_f32")
OP(k_minf, "v_min_f32")
OP(k_mulhi, "v_mul_hi_u32")
OP(k_mullo, "v_mul_lo_u32")
OP3(k_cvtpk, "v_cvt_pk_u8_f32")
OP1(k_not, "v_not_b32")
OP1(k_bfrev, "v_bfrev_b32")
OP1(k_ffbl, "v_ffbl_b32")
OP3(k_fma, "v_fma_f32")
OP3(k_sad, "v_sad_u8")
OP3(k_msad, "v_msad_u8")
OP3(k_lerp, "v_lerp_u8")
OP3(k_andor, "v_and_or_b32")
OP3(k_or3, "v_or3_b32")
OP3(k_lshladd, "v_lshl_add_u32")
OP3(k_addlshl, "v_add_lshl_u32")
OP3(k_xad, "v_xad_u32")
OP3(k_sadu16, "v_sad_u16")
OP3(k_max3f, "v_max3_f32")
OP3(k_sadu32, "v_sad_u32")
OP(k_sub, "v_sub_u32")
OP(k_maxi, "v_max_i32")
OP(k_pksub, "v_pk_sub_u16")
OP(k_pkadd, "v_pk_add_u16")
OP(k_mul24, "v_mul_u32_u24")
OP(k_lshr, "v_lshrrev_b32")
OP(k_and, "v_and_b32")
OP(k_fmul, "v_mul_f32")
OP3(k_min3, "v_min3_u32")
OP3(k_med3, "v_med3_u32")
OP3(k_perm, "v_perm_b32")
OP3(k_align, "v_alignbyte_b32")
OP3(k_dot4, "v_dot4_u32_u8")
OP3(k_dot2, "v_dot2_u32_u16")
OP3(k_lshlor, "v_lshl_or_b32")
OP3(k_add3, "v_add3_u32")
OP3(k_bfe, "v_bfe_u32")
OP3(k_mad24, "v_mad_u32_u24")
OP(k_bcnt, "v_bcnt_u32_b32")
OP(k_add, "v_add_u32")
OP(k_min, "v_min_u32")
OP(k_pkmin, "v_pk_min_u16")


int main() {
    unsigned* o;
    hipMalloc(&o, 256 * 1024 * 4 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char* n; void (*k)(unsigned*, unsigned); } ks[] = {
        {"v_xor_b32", k_xor}, {"v_bcnt_u32_b32", k_bcnt}, {"v_add_u32", k_add},
        {"v_min_u32", k_min}, {"v_pk_min_u16", k_pkmin}, {"v_sub_u32", k_sub},
        {"v_max_i32", k_maxi}, {"v_pk_sub_u16", k_pksub}, {"v_pk_add_u16", k_pkadd},
        {"v_mul_u32_u24", k_mul24}, {"v_lshrrev_b32", k_lshr}, {"v_and_b32", k_and},
        {"v_mul_f32", k_fmul}, {"v_min3_u32", k_min3}, {"v_med3_u32", k_med3},
        {"v_perm_b32", k_perm}, {"v_alignbyte_b32", k_align}, {"v_dot4_u32_u8", k_dot4},
        {"v_dot2_u32_u16", k_dot2}, {"v_lshl_or_b32", k_lshlor}, {"v_add3_u32", k_add3},
        {"v_bfe_u32", k_bfe}, {"v_mad_u32_u24", k_mad24},
        {"v_or_b32", k_or}, {"v_lshlrev_b32", k_lshl}, {"v_ashrrev_i32", k_ashr}, {"v_add_f32", k_addf}, {"v_mov_b32", k_mov}, {"v_cvt_f32_u32", k_cvtfu}, {"v_cvt_u32_f32", k_cvtuf}, {"v_rndne_f32", k_rndne}, {"v_cvt_f32_ubyte0", k_ub0}, {"v_add_u16", k_addu16}, {"v_min_u16", k_minu16}, {"v_sub_u16", k_subu16}, {"v_max_f32", k_maxf}, {"v_min_f32", k_minf}, {"v_mul_hi_u32", k_mulhi}, {"v_mul_lo_u32", k_mullo}, {"v_cvt_pk_u8_f32", k_cvtpk}, {"v_not_b32", k_not}, {"v_bfrev_b32", k_bfrev}, {"v_ffbl_b32", k_ffbl}, {"v_fma_f32", k_fma}, {"v_sad_u8", k_sad}, {"v_msad_u8", k_msad}, {"v_lerp_u8", k_lerp}, {"v_and_or_b32", k_andor}, {"v_or3_b32", k_or3}, {"v_lshl_add_u32", k_lshladd}, {"v_add_lshl_u32", k_addlshl}, {"v_xad_u32", k_xad}, {"v_sad_u16", k_sadu16}, {"v_max3_f32", k_max3f}, {"v_sad_u32", k_sadu32}};
    const int blocks = 256 * 8, threads = 256;   // 8 waves per SIMD
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, o, 3u);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, o, 3u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double winstr = (double)blocks * (threads / 64) * N * 8;
        // cycles per wave-instruction per SIMD at 2.4 GHz, 1024 SIMDs
        printf("%-16s %.3f ms  %.2f cycles/wave-instr/SIMD\n", k.n, ms,
               ms * 1e-3 * 2.4e9 * 1024 / winstr);
    }
    return 0;
}
