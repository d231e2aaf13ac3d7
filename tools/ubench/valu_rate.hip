// Microbenchmark: wave-instruction throughput of the VALU forms the IDFT / decoder use (gfx950).
// Every CU runs 1, 2, 4 and 8 waves per SIMD of a loop of 16 independent chains x ITER of one
// instruction, plus encoding-size controls (the same op as VOP2 / VOP3).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048
#define OP_LOOP(ASM)                                                                        \
  for (int i = 0; i < ITER; i++) {                                                          \
    _Pragma("unroll") for (int k = 0; k < 16; k++) asm volatile(ASM : "+v"(r[k]) : "v"(b)); \
  }
#define KERNEL(NAME, ASM)                                                   \
  __global__ void __launch_bounds__(256) NAME(unsigned *out, unsigned b) {  \
    unsigned r[16];                                                         \
    for (int k = 0; k < 16; k++) r[k] = threadIdx.x * (k + 1);              \
    OP_LOOP(ASM)                                                            \
    unsigned s = 0;                                                         \
    if (threadIdx.x == 0 && blockIdx.x == 0) {}                             \
    for (int k = 0; k < 16; k++) s ^= r[k];                                 \
    if (s == 0x1234567u) out[0] = s;                                        \
  }
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_dot2, "v_dot2_i32_i16 %0, %0, %1, %0")
KERNEL(k_dot2z, "v_dot2_i32_i16 %0, %0, %1, 0")
KERNEL(k_cvtpk, "v_cvt_pk_i16_i32 %0, %0, %1")
KERNEL(k_pkadd_sat, "v_pk_add_i16 %0, %0, %1 clamp")
KERNEL(k_pkadd, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_pkmax, "v_pk_max_i16 %0, %0, %1")
KERNEL(k_ashr, "v_ashrrev_i32 %0, 15, %0")
KERNEL(k_pkashr, "v_pk_ashrrev_i16 %0, 1, %0")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 5")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")
KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_max3, "v_max3_i32 %0, %0, %1, %0")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
KERNEL(k_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KERNEL(k_addsdwa, "v_add_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0")
KERNEL(k_pkmaxsdwa, "v_max_i16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")

KERNEL(k_lshl, "v_lshlrev_b32 %0, 3, %0")
KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL(k_mul24, "v_mul_i32_i24 %0, %0, %1")
KERNEL(k_mulhi24, "v_mul_hi_i32_i24 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERNEL(k_lshladd, "v_lshl_add_u32 %0, %0, 2, %1")
KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 16, %1")
KERNEL(k_andor, "v_and_or_b32 %0, %0, %1, %0")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %0")
KERNEL(k_bfei, "v_bfe_i32 %0, %0, 3, 16")
KERNEL(k_med3, "v_med3_i32 %0, %0, %1, %0")
KERNEL(k_pkmullo, "v_pk_mul_lo_u16 %0, %0, %1 op_sel:[1,0] op_sel_hi:[0,1]")
KERNEL(k_mov, "v_mov_b32 %0, %1")
KERNEL(k_sub16, "v_sub_u16 %0, %0, %1")
KERNEL(k_addi32c, "v_add_i32 %0, %0, %1 clamp")
KERNEL(k_madi24, "v_mad_i32_i24 %0, %0, %1, %0")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 2")
KERNEL(k_max, "v_max_i32 %0, %0, %1")
KERNEL(k_pklshl, "v_pk_lshlrev_b16 %0, 1, %0")
KERNEL(k_lshr16, "v_lshrrev_b16 %0, 1, %0")
KERNEL(k_not, "v_not_b32 %0, %0")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %0")
KERNEL(k_addco, "v_add_co_u32 %0, vcc, %0, %1")
KERNEL(k_pksubsat, "v_pk_sub_i16 %0, %0, %1 clamp")
KERNEL(k_pksubsel, "v_pk_sub_i16 %0, %0, %1 op_sel:[1,1] op_sel_hi:[0,0] clamp")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %0")
KERNEL(k_addsdwa32, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
KERNEL(k_ashrsdwa, "v_ashrrev_i32_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_lshlor2, "v_lshl_or_b32 %0, %0, 1, %1")
KERNEL(k_dot2u, "v_dot2_u32_u16 %0, %0, %1, %0")
KERNEL(k_mulu24, "v_mul_u32_u24 %0, %0, %1")
// encoding-size controls: the full-rate VOP2 ops forced into the 8-byte VOP3 encoding, and
// half-rate ops that have a 4-byte VOP2 / VOP1 encoding (is the rate the op or the fetch?)
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL(k_and_e64, "v_and_b32_e64 %0, %0, %1")
KERNEL(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
KERNEL(k_mov_e64, "v_mov_b32_e64 %0, %1")
KERNEL(k_max_e32, "v_max_i32_e32 %0, %0, %1")
KERNEL(k_lshl_e32v, "v_lshlrev_b32_e32 %0, %1, %0")
KERNEL(k_mul24_e32, "v_mul_i32_i24_e32 %0, %0, %1")
KERNEL(k_maxu16_e32, "v_max_u16_e32 %0, %0, %1")
KERNEL(k_addf32_e32, "v_add_f32_e32 %0, %0, %1")

typedef void (*kfn)(unsigned *, unsigned);
int main() {
  struct { const char *n; kfn f; } ks[] = {
      {"v_add_u32", k_add}, {"v_dot2_i32_i16 (acc)", k_dot2}, {"v_dot2_i32_i16 (0)", k_dot2z},
      {"v_cvt_pk_i16_i32", k_cvtpk}, {"v_pk_add_i16 clamp", k_pkadd_sat}, {"v_pk_add_u16", k_pkadd},
      {"v_pk_max_i16", k_pkmax}, {"v_ashrrev_i32", k_ashr}, {"v_pk_ashrrev_i16", k_pkashr},
      {"v_alignbit_b32", k_alignbit}, {"v_perm_b32", k_perm}, {"v_mad_u32_u24", k_mad24},
      {"v_mul_lo_u32", k_mullo}, {"v_max3_i32", k_max3}, {"v_bitop3_b32", k_bitop3}, {"v_mov_b32_dpp", k_dpp},
      {"v_add_u16_sdwa", k_addsdwa}, {"v_max_i16_sdwa", k_pkmaxsdwa}, {"v_lshlrev_b32", k_lshl}, {"v_and_b32", k_and}, {"v_or_b32", k_or}, {"v_xor_b32", k_xor}, {"v_sub_u32", k_sub}, {"v_mul_i32_i24", k_mul24}, {"v_mul_hi_i32_i24", k_mulhi24}, {"v_add3_u32", k_add3}, {"v_lshl_add_u32", k_lshladd}, {"v_lshl_or_b32", k_lshlor}, {"v_and_or_b32", k_andor}, {"v_or3_b32", k_or3}, {"v_bfe_i32", k_bfei}, {"v_med3_i32", k_med3}, {"v_pk_mul_lo_u16 sel", k_pkmullo}, {"v_mov_b32", k_mov}, {"v_sub_u16", k_sub16}, {"v_add_i32", k_addi32c}, {"v_mad_i32_i24", k_madi24}, {"v_alignbyte_b32", k_alignbyte}, {"v_max_i32", k_max}, {"v_pk_lshlrev_b16", k_pklshl}, {"v_lshrrev_b16", k_lshr16}, {"v_not_b32", k_not}, {"v_bfi_b32", k_bfi}, {"v_add_co_u32", k_addco}, {"v_pk_sub_i16", k_pksubsat}, {"v_pk_sub_i16 sel", k_pksubsel}, {"v_xad_u32", k_xad}, {"v_add_u32_sdwa sdwa", k_addsdwa32}, {"v_ashrrev_i32_sdwa sdwa", k_ashrsdwa}, {"v_cndmask_b32", k_cndmask}, {"v_lshl_or_b32", k_lshlor2}, {"v_dot2_u32_u16", k_dot2u}, {"v_mul_u32_u24", k_mulu24},
      {"v_add_u32_e64 (VOP3)", k_add_e64}, {"v_and_b32_e64 (VOP3)", k_and_e64}, {"v_xor_b32_e64 (VOP3)", k_xor_e64},
      {"v_mov_b32_e64 (VOP3)", k_mov_e64}, {"v_max_i32_e32 (VOP2)", k_max_e32}, {"v_lshlrev_b32_e32 vv", k_lshl_e32v},
      {"v_mul_i32_i24_e32", k_mul24_e32}, {"v_max_u16_e32 (VOP2)", k_maxu16_e32}, {"v_add_f32_e32 (VOP2)", k_addf32_e32}};
  unsigned *d;
  hipMalloc(&d, 64);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wps : {1, 2, 4, 8}) {
  int blocks = cus * wps;   // 256-thread blocks: wps per CU = wps waves per SIMD
  printf("--- %d wave(s) per SIMD\n", wps);
  for (auto &k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, d, 3u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) {
        double winst = (double)blocks * 4 * ITER * 16;   // wave-instructions
        double per_simd = winst / (cus * 4);
        printf("%-22s %8.3f ms  %6.2f Gwave-inst/s/SIMD  -> %5.2f cycles @2.4GHz\n", k.n, ms,
               per_simd / (ms * 1e6), 2.4e9 * ms * 1e-3 / per_simd);
      }
    }
  }
  }
  return 0;
}
