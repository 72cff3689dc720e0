// VALU issue-rate microbenchmark for gfx950: cycles per wave-instruction per SIMD of
// the integer instructions the Goldilocks / BN254 arithmetic is built from, at 8 waves
// per SIMD (enough independent waves to saturate issue). Compare with v_add_f32 (2 cyc).
// Build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 512
#define BODY8(X) X X X X X X X X

#define K1(NAME, ASM)                                                            \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {     \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;    \
    uint32_t a4 = a0 + 11, a5 = a0 + 13, a6 = a0 + 17, a7 = a0 + 19;            \
    uint32_t b = seed | 1;                                                      \
    for (int i = 0; i < ITERS; ++i) {                                           \
      asm volatile(ASM(a0) ASM(a1) ASM(a2) ASM(a3) ASM(a4) ASM(a5) ASM(a6) ASM(a7) \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b) : "vcc");                                             \
    }                                                                           \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
  }

// each ASM(x) expands to one instruction on operand register %N; we index via stringized positions
#define I_ADDF(r) "v_add_f32 " r ", " r ", %8\n"
#define I_ADDU(r) "v_add_u32 " r ", " r ", %8\n"
#define I_ADDCO(r) "v_add_co_u32 " r ", vcc, " r ", %8\n"
#define I_ADDC(r) "v_addc_co_u32 " r ", vcc, " r ", %8, vcc\n"
#define I_MULLO(r) "v_mul_lo_u32 " r ", " r ", %8\n"
#define I_MULHI(r) "v_mul_hi_u32 " r ", " r ", %8\n"
#define I_CND(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define I_ADD3(r) "v_add3_u32 " r ", " r ", %8, " r "\n"
#define I_ALIGN(r) "v_alignbit_b32 " r ", " r ", %8, 7\n"
#define I_MOV(r) "v_mov_b32 " r ", %8\n"
#define I_MAD24(r) "v_mad_u32_u24 " r ", " r ", %8, " r "\n"
#define I_PERM(r) "v_perm_b32 " r ", " r ", %8, " r "\n"
#define I_LSHL(r) "v_lshlrev_b32 " r ", 3, " r "\n"
#define I_CMP(r) "v_cmp_lt_u32 vcc, " r ", %8\n"
#define I_SUBB(r) "v_subbrev_co_u32 " r ", vcc, 0, " r ", vcc\n"
#define I_XAD(r) "v_xad_u32 " r ", " r ", %8, " r "\n"
#define I_LSHLADD(r) "v_lshl_add_u32 " r ", " r ", 2, %8\n"
#define I_MADHI(r) "v_mul_hi_u32_u24 " r ", " r ", %8\n"


#define I_CNDS(r) "v_cndmask_b32_e64 " r ", " r ", %8, s[40:41]\n"
#define I_CMPCND(r) "v_cmp_lt_u32 vcc, " r ", %8\nv_cndmask_b32 " r ", " r ", %8, vcc\n"
#define I_AND(r) "v_and_b32 " r ", " r ", %8\n"
#define I_OR(r) "v_or_b32 " r ", " r ", %8\n"
#define I_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define I_SUBU(r) "v_sub_u32 " r ", " r ", %8\n"
#define I_MAXU(r) "v_max_u32 " r ", " r ", %8\n"
#define I_MINU(r) "v_min_u32 " r ", " r ", %8\n"
#define I_BFE(r) "v_bfe_u32 " r ", " r ", 3, 7\n"
#define I_LSHR(r) "v_lshrrev_b32 " r ", 3, " r "\n"
#define I_LSHLV(r) "v_lshlrev_b32 " r ", %8, " r "\n"
#define I_ASHR(r) "v_ashrrev_i32 " r ", 31, " r "\n"
#define I_ADDCO3(r) "v_add_co_u32_e64 " r ", s[40:41], " r ", %8\n"
#define I_ADDNC(r) "v_add_nc_u32 " r ", " r ", %8\n"
#define I_MULU24(r) "v_mul_u32_u24 " r ", " r ", %8\n"
#define I_FMAF(r) "v_fma_f32 " r ", " r ", %8, " r "\n"
#define I_MULF(r) "v_mul_f32 " r ", " r ", %8\n"
#define I_SUBREV(r) "v_subrev_u32 " r ", " r ", %8\n"
#define R0 "%0"
#define R1 "%1"
#define R2 "%2"
#define R3 "%3"
#define R4 "%4"
#define R5 "%5"
#define R6 "%6"
#define R7 "%7"
#define K(NAME, I)                                                                     \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {           \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;          \
    uint32_t a4 = a0 + 11, a5 = a0 + 13, a6 = a0 + 17, a7 = a0 + 19;                  \
    uint32_t b = seed | 1;                                                            \
    for (int i = 0; i < ITERS; ++i) {                                                 \
      asm volatile(I(R0) I(R1) I(R2) I(R3) I(R4) I(R5) I(R6) I(R7)                    \
                   I(R0) I(R1) I(R2) I(R3) I(R4) I(R5) I(R6) I(R7)                    \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b) : "vcc", "s40", "s41");                                                 \
    }                                                                                 \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
  }

// 64-bit operand kernels
#define J_LSHLADD64(r) "v_lshl_add_u64 " r ", " r ", 0, %8\n"
#define J_MAD64(r) "v_mad_u64_u32 " r ", s[40:41], %9, %9, " r "\n"
#define J_CMP64(r) "v_cmp_lt_u64 vcc, " r ", %8\n"
#define J_LSHL64(r) "v_lshlrev_b64 " r ", 3, " r "\n"
#define J_MOV64(r) "v_mov_b64 " r ", %8\n"
#define J_PKADD(r) "v_pk_add_f32 " r ", " r ", %8\n"
#define J_MADI64(r) "v_mad_i64_i32 " r ", s[40:41], %9, %9, " r "\n"
#define J_ASHR64(r) "v_ashrrev_i64 " r ", 3, " r "\n"
#define J_LSHR64(r) "v_lshrrev_b64 " r ", 3, " r "\n"
#define J_PKMOV(r) "v_pk_mov_b32 " r ", " r ", %8 op_sel:[0,1]\n"
#define K64(NAME, I)                                                                   \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {           \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;          \
    uint64_t a4 = a0 + 11, a5 = a0 + 13, a6 = a0 + 17, a7 = a0 + 19;                  \
    uint64_t b = seed | 1;                                                            \
    uint32_t c = seed * 7;                                                            \
    for (int i = 0; i < ITERS; ++i) {                                                 \
      asm volatile(I(R0) I(R1) I(R2) I(R3) I(R4) I(R5) I(R6) I(R7)                    \
                   I(R0) I(R1) I(R2) I(R3) I(R4) I(R5) I(R6) I(R7)                    \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b), "v"(c) : "vcc", "s40", "s41");                            \
    }                                                                                 \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }

K(k_add_f32, I_ADDF)
K(k_add_u32, I_ADDU)
K(k_add_co, I_ADDCO)
K(k_addc, I_ADDC)
K(k_mul_lo, I_MULLO)
K(k_mul_hi, I_MULHI)
K(k_cndmask, I_CND)
K(k_add3, I_ADD3)
K(k_alignbit, I_ALIGN)
K(k_mov, I_MOV)
K(k_mad24, I_MAD24)
K(k_perm, I_PERM)
K(k_lshl, I_LSHL)
K(k_cmp32, I_CMP)
K(k_subb, I_SUBB)
K(k_xad, I_XAD)
K(k_lshl_add32, I_LSHLADD)
K(k_mulhi24, I_MADHI)
K(k_cnds, I_CNDS)
K(k_cmpcnd, I_CMPCND)
K(k_and, I_AND)
K(k_or, I_OR)
K(k_xor, I_XOR)
K(k_subu, I_SUBU)
K(k_maxu, I_MAXU)
K(k_minu, I_MINU)
K(k_bfe, I_BFE)
K(k_lshr, I_LSHR)
K(k_lshlv, I_LSHLV)
K(k_ashr, I_ASHR)
K(k_addco3, I_ADDCO3)
K(k_mulu24, I_MULU24)
K(k_fmaf, I_FMAF)
K(k_mulf, I_MULF)
K(k_subrev, I_SUBREV)
K64(k_lshl_add64, J_LSHLADD64)
K64(k_mad64, J_MAD64)
K64(k_cmp64, J_CMP64)
K64(k_lshl64, J_LSHL64)
K64(k_mov64, J_MOV64)
K64(k_pk_add_f32, J_PKADD)
K64(k_pk_mov, J_PKMOV)
K64(k_madi64, J_MADI64)
K64(k_ashr64, J_ASHR64)
K64(k_lshr64, J_LSHR64)
#define I_DPP(r) "v_mov_b32_dpp " r ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define I_PL32(r) "v_permlane32_swap_b32 " r ", %8\n"
#define I_SUBCO(r) "v_sub_co_u32 " r ", vcc, " r ", %8\n"
#define I_LSHLOR(r) "v_lshl_or_b32 " r ", " r ", 3, %8\n"
#define I_ANDOR(r) "v_and_or_b32 " r ", " r ", %8, " r "\n"
#define I_BFI(r) "v_bfi_b32 " r ", " r ", %8, " r "\n"
#define I_ADDI(r) "v_add_i32 " r ", " r ", %8\n"
#define I_ASHRV(r) "v_ashrrev_i32 " r ", %8, " r "\n"
#define I_PKADDU16(r) "v_pk_add_u16 " r ", " r ", %8\n"
#define I_BFEI(r) "v_bfe_i32 " r ", " r ", 3, 7\n"
K(k_dpp, I_DPP)
K(k_subco, I_SUBCO)
K(k_lshlor, I_LSHLOR)
K(k_andor, I_ANDOR)
K(k_bfi, I_BFI)
K(k_addi, I_ADDI)
K(k_ashrv, I_ASHRV)
K(k_pkaddu16, I_PKADDU16)
K(k_bfei, I_BFEI)

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  struct { const char* name; kfn f; } ks[] = {
      {"v_add_f32", k_add_f32}, {"v_add_u32", k_add_u32}, {"v_add_co_u32", k_add_co}, {"v_addc_co_u32", k_addc},
      {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi}, {"v_cndmask_b32", k_cndmask}, {"v_add3_u32", k_add3},
      {"v_alignbit_b32", k_alignbit}, {"v_mov_b32", k_mov}, {"v_mad_u32_u24", k_mad24}, {"v_perm_b32", k_perm},
      {"v_lshlrev_b32", k_lshl}, {"v_cmp_lt_u32", k_cmp32}, {"v_subbrev_co_u32", k_subb}, {"v_xad_u32", k_xad},
      {"v_lshl_add_u32", k_lshl_add32}, {"v_mul_hi_u32_u24", k_mulhi24},
      {"v_cndmask_e64 sgpr", k_cnds}, {"v_cmp32+v_cndmask", k_cmpcnd}, {"v_and_b32", k_and}, {"v_or_b32", k_or},
      {"v_xor_b32", k_xor}, {"v_sub_u32", k_subu}, {"v_max_u32", k_maxu}, {"v_min_u32", k_minu}, {"v_bfe_u32", k_bfe},
      {"v_lshrrev_b32", k_lshr}, {"v_lshlrev_b32 vreg", k_lshlv}, {"v_ashrrev_i32", k_ashr}, {"v_add_co_u32_e64 sdst", k_addco3},
      {"v_mul_u32_u24", k_mulu24}, {"v_fma_f32", k_fmaf}, {"v_mul_f32", k_mulf}, {"v_subrev_u32", k_subrev},
      {"v_lshl_add_u64", k_lshl_add64}, {"v_mad_u64_u32", k_mad64}, {"v_cmp_lt_u64", k_cmp64},
      {"v_lshlrev_b64", k_lshl64}, {"v_mov_b64", k_mov64}, {"v_pk_add_f32", k_pk_add_f32}, {"v_pk_mov_b32", k_pk_mov}, {"v_mad_i64_i32", k_madi64}, {"v_ashrrev_i64", k_ashr64}, {"v_lshrrev_b64", k_lshr64}, {"v_mov_b32_dpp", k_dpp}, {"v_sub_co_u32", k_subco}, {"v_lshl_or_b32", k_lshlor}, {"v_and_or_b32", k_andor}, {"v_bfi_b32", k_bfi}, {"v_add_i32", k_addi}, {"v_ashrrev_i32 vreg", k_ashrv}, {"v_pk_add_u16", k_pkaddu16}, {"v_bfe_i32", k_bfei},
  };
  const int blocks = 256 * 8 * 4;  // 8 workgroups of 256 threads per CU resident = 8 waves/SIMD, x4 rounds
  uint32_t* out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double ref = 0;
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 12345u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 12345u + r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD: blocks*4 waves * ITERS*16 instr / (256 CUs * 4 SIMD) * 5 reps
    const double winst = (double)blocks * 4 * ITERS * 16 * 5 / (256.0 * 4);
    const double ns_per = ms * 1e6 / winst;
    if (ref == 0) ref = ns_per;
    printf("%-20s %7.3f ns/wave-instr/SIMD  = %5.2f x v_add_f32  (%.2f cyc @2.4GHz)\n", k.name, ns_per, ns_per / ref,
           ns_per * 2.4);
  }
  return 0;
}
