// valu_rate.hip -- VALU issue throughput per instruction type on gfx950 (MI355X): 8 independent
// accumulator chains per lane, 16 waves per CU, each loop iteration issues 8 instructions of one
// kind; reports wave-instructions per SIMD-cycle (clock from s_memtime inside the kernel).
//   build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 4096;

#define BODY8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define KERNEL(NAME, OP, INIT)                                                                      \
  __global__ __launch_bounds__(256) void NAME(uint32_t *out, unsigned long long *clk, uint32_t s) {  \
    uint32_t a0 = threadIdx.x + s, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11,   \
             a6 = a0 + 13, a7 = a0 + 17;                                                            \
    uint32_t k = INIT;                                                                              \
    const uint64_t sm = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);                               \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
    for (int i = 0; i < kIters; i++) { BODY8(OP) }                                                 \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                    \
    if (threadIdx.x == 0) atomicMax(clk, t1 - t0);                                                 \
  }

#define OP_ADDF(r) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_MULF(r) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_PKMULF(r) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(double *)&r) : "v"(*(double *)&k));
#define OP_ADDU(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_MAXI(r) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_PKMAXI16(r) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_BFI(r) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(r) : "v"(k));
#define OP_DPP(r) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(r));
#define OP_MAX3(r) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_MINI(r) asm volatile("v_min_i32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_SUBU(r) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_AND(r) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_OR(r) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_LSHL(r) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r) : "v"(k));
#define OP_CNDMASK(r) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(k));
#define OP_MED3(r) asm volatile("v_med3_i32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_PKADD16(r) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_PKSUB16(r) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_PERM(r) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_BFE(r) asm volatile("v_bfe_i32 %0, %0, %1, 1" : "+v"(r) : "v"(k));
#define OP_MOV(r) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(k));
#define OP_SUBF(r) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_FMAC(r) asm volatile("v_fmac_f32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_MAXF(r) asm volatile("v_max_f32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_ADDI16(r) asm volatile("v_add_u16 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_LSHLOR(r) asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(r) : "v"(k));
#define OP_XOR(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_CMPCND(r) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(k) : "vcc");
#define OP_CNDS(r) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(k), "s"(sm));
#define OP_CMP(r) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(r), "v"(k) : "vcc");
#define OP_MULF_DPP(r) asm volatile("v_mul_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
#define OP_MULF_ROR(r) asm volatile("v_mul_f32_dpp %0, %0, %1 wave_ror:1 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
#define OP_ADDF_DPP(r) asm volatile("v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
#define OP_ADDCO(r) asm volatile("v_add_co_u32 %0, vcc, -1, %0" : "+v"(r) : : "vcc");
#define OP_ADDC(r) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(r) : : "vcc");
#define OP_CARRYPAIR(r) asm volatile("v_add_co_u32 %0, vcc, -1, %1\n v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(r) : "v"(k) : "vcc");
#define OP_MINSDWA(r) asm volatile("v_min_u32_sdwa %0, %1, 1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(r) : "v"(k));
#define OP_MOVSDWA(r) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(r) : "v"(k));
#define OP_ORSDWA(r) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(r) : "v"(k));
#define OP_MULU24(r) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_MADU24(r) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_MINU(r) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_SUBREV(r) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define OP_ADD3(r) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_OR3(r) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
#define OP_BITOP3(r) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0xca" : "+v"(r) : "v"(k));
#define OP_ADDF64(r) asm volatile("v_add_f64 %0, %0, %1" : "+v"(*(double *)&r) : "v"(*(double *)&k));
#define OP_MULF64(r) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(*(double *)&r) : "v"(*(double *)&k));
#define OP_PKADDF(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&r) : "v"(*(double *)&k));
#define OP_PKFMAF(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(*(double *)&r) : "v"(*(double *)&k));

KERNEL(k_addf, OP_ADDF, 0x3f800000u)
KERNEL(k_mulf, OP_MULF, 0x3f800000u)
KERNEL(k_addu, OP_ADDU, 1u)
KERNEL(k_maxi, OP_MAXI, 1u)
KERNEL(k_pkmaxi16, OP_PKMAXI16, 0x00010001u)
KERNEL(k_bfi, OP_BFI, 0x0f0f0f0fu)
KERNEL(k_dpp, OP_DPP, 0u)
KERNEL(k_max3, OP_MAX3, 1u)
KERNEL(k_mini, OP_MINI, 1u)
KERNEL(k_subu, OP_SUBU, 1u)
KERNEL(k_and, OP_AND, 0xffffu)
KERNEL(k_or, OP_OR, 1u)
KERNEL(k_lshl, OP_LSHL, 1u)
KERNEL(k_cnd, OP_CNDMASK, 1u)
KERNEL(k_med3, OP_MED3, 1u)
KERNEL(k_pkadd16, OP_PKADD16, 0x00010001u)
KERNEL(k_pksub16, OP_PKSUB16, 0x00010001u)
KERNEL(k_perm, OP_PERM, 0x05040100u)
KERNEL(k_bfe, OP_BFE, 3u)
KERNEL(k_mov, OP_MOV, 1u)
KERNEL(k_subf, OP_SUBF, 0x3f800000u)
KERNEL(k_fmac, OP_FMAC, 0x3f800000u)
KERNEL(k_maxf, OP_MAXF, 0x3f800000u)
KERNEL(k_addi16, OP_ADDI16, 1u)
KERNEL(k_lshlor, OP_LSHLOR, 1u)
KERNEL(k_xor, OP_XOR, 1u)
KERNEL(k_cmpcnd, OP_CMPCND, 1u)
KERNEL(k_cnds, OP_CNDS, 1u)
KERNEL(k_cmp, OP_CMP, 1u)
KERNEL(k_mulf_dpp, OP_MULF_DPP, 0x3f800000u)
KERNEL(k_mulf_ror, OP_MULF_ROR, 0x3f800000u)
KERNEL(k_addf_dpp, OP_ADDF_DPP, 0x3f800000u)
KERNEL(k_addco, OP_ADDCO, 1u)
KERNEL(k_addc, OP_ADDC, 1u)
KERNEL(k_carrypair, OP_CARRYPAIR, 1u)
KERNEL(k_minsdwa, OP_MINSDWA, 1u)
KERNEL(k_movsdwa, OP_MOVSDWA, 1u)
KERNEL(k_orsdwa, OP_ORSDWA, 1u)
KERNEL(k_mulu24, OP_MULU24, 3u)
KERNEL(k_madu24, OP_MADU24, 3u)
KERNEL(k_minu, OP_MINU, 1u)
KERNEL(k_subrev, OP_SUBREV, 1u)
KERNEL(k_add3, OP_ADD3, 1u)
KERNEL(k_or3, OP_OR3, 1u)
KERNEL(k_bitop3, OP_BITOP3, 1u)

#define KERNEL64(NAME, OP)                                                                          \
  __global__ __launch_bounds__(256) void NAME(uint32_t *out, unsigned long long *clk, uint32_t s) {  \
    double a0 = threadIdx.x + s, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 9, a5 = a0 + 11,     \
           a6 = a0 + 13, a7 = a0 + 17;                                                              \
    double kd = 1.0;                                                                                \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
    for (int i = 0; i < kIters; i++) { BODY8(OP) }                                                 \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);        \
    if (threadIdx.x == 0) atomicMax(clk, t1 - t0);                                                 \
  }
#define OP64(INS) asm volatile(INS " %0, %0, %1" : "+v"(r) : "v"(kd));
#define OP_D_ADDF64(r) asm volatile("v_add_f64 %0, %0, %1" : "+v"(r) : "v"(kd));
#define OP_D_MULF64(r) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r) : "v"(kd));
#define OP_D_FMAF64(r) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(r) : "v"(kd));
#define OP_D_PKMULF(r) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(r) : "v"(kd));
#define OP_D_PKADDF(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"(kd));
#define OP_D_PKFMAF(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(r) : "v"(kd));
KERNEL64(k_addf64, OP_D_ADDF64)
KERNEL64(k_mulf64, OP_D_MULF64)
KERNEL64(k_fmaf64, OP_D_FMAF64)
KERNEL64(k_pkmulf, OP_D_PKMULF)
KERNEL64(k_pkaddf, OP_D_PKADDF)
KERNEL64(k_pkfmaf, OP_D_PKFMAF)

typedef void (*KFN)(uint32_t *, unsigned long long *, uint32_t);

int main() {
  uint32_t *out;
  unsigned long long *clk;
  const int cus = 256, waves_per_cu = 16, blocks = cus * waves_per_cu / 4;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CK(hipMalloc(&clk, 8));
  struct { const char *name; KFN fn; } ks[] = {{"v_add_f32", k_addf}, {"v_mul_f32", k_mulf}, {"v_add_u32", k_addu},
      {"v_max_i32", k_maxi}, {"v_pk_max_i16", k_pkmaxi16}, {"v_bfi_b32", k_bfi}, {"v_mov_b32_dpp", k_dpp},
      {"v_max3_i32", k_max3}, {"v_min_i32", k_mini}, {"v_sub_u32", k_subu}, {"v_and_b32", k_and},
      {"v_or_b32", k_or}, {"v_xor_b32", k_xor}, {"v_lshlrev_b32", k_lshl}, {"v_cndmask_b32", k_cnd},
      {"v_med3_i32", k_med3}, {"v_pk_add_u16", k_pkadd16}, {"v_pk_sub_i16", k_pksub16}, {"v_perm_b32", k_perm},
      {"v_bfe_i32", k_bfe}, {"v_mov_b32", k_mov}, {"v_sub_f32", k_subf}, {"v_fmac_f32", k_fmac},
      {"v_max_f32", k_maxf}, {"v_add_u16", k_addi16}, {"v_lshl_or_b32", k_lshlor},
      {"cmp+cndmask(vcc)x2", k_cmpcnd}, {"cndmask(sgpr)", k_cnds}, {"v_cmp(vcc)", k_cmp},
      {"v_mul_f32_dpp row_shr", k_mulf_dpp}, {"v_mul_f32_dpp wave_ror", k_mulf_ror}, {"v_add_f32_dpp row_shr", k_addf_dpp},
      {"v_add_co_u32(vcc)", k_addco}, {"v_addc_co_u32(vcc)", k_addc}, {"add_co+addc pair x2", k_carrypair},
      {"v_min_u32_sdwa byte", k_minsdwa}, {"v_mov_b32_sdwa word", k_movsdwa}, {"v_or_b32_sdwa byte", k_orsdwa},
      {"v_mul_u32_u24", k_mulu24}, {"v_mad_u32_u24", k_madu24}, {"v_min_u32", k_minu}, {"v_subrev_u32", k_subrev},
      {"v_add3_u32", k_add3}, {"v_or3_b32", k_or3}, {"v_bitop3_b32", k_bitop3},
      {"v_add_f64", k_addf64}, {"v_mul_f64", k_mulf64}, {"v_fma_f64", k_fmaf64}, {"v_pk_mul_f32", k_pkmulf},
      {"v_pk_add_f32", k_pkaddf}, {"v_pk_fma_f32", k_pkfmaf}};
  for (auto &k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipMemset(clk, 0, 8));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, clk, 3u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long c;
      CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
      // per SIMD: 4 waves (16 per CU), each 8 * kIters instructions, over c cycles (max wave span)
      const double per_simd = 4.0 * 8 * kIters / (double)c;
      if (rep) printf("%-14s %.3f wave-instr / SIMD-cycle (%.2f cycles each), kernel %.3f ms\n", k.name, per_simd, 1.0 / per_simd, ms);
      CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    }
  }
  return 0;
}
