// Microbenchmark: wave-instruction throughput of the VALU forms the IDFT / decoder use (gfx950).
// Every CU runs 8 waves per SIMD of a loop of 16 independent chains x ITER of one instruction.
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

typedef void (*kfn)(unsigned *, unsigned);
int main() {
  struct { const char *n; kfn f; } ks[] = {
      {"v_add_u32", k_add}, {"v_dot2_i32_i16 (acc)", k_dot2}, {"v_dot2_i32_i16 (0)", k_dot2z},
      {"v_cvt_pk_i16_i32", k_cvtpk}, {"v_pk_add_i16 clamp", k_pkadd_sat}, {"v_pk_add_u16", k_pkadd},
      {"v_pk_max_i16", k_pkmax}, {"v_ashrrev_i32", k_ashr}, {"v_pk_ashrrev_i16", k_pkashr},
      {"v_alignbit_b32", k_alignbit}, {"v_perm_b32", k_perm}, {"v_mad_u32_u24", k_mad24},
      {"v_mul_lo_u32", k_mullo}, {"v_max3_i32", k_max3}, {"v_bitop3_b32", k_bitop3}, {"v_mov_b32_dpp", k_dpp},
      {"v_add_u16_sdwa", k_addsdwa}, {"v_max_i16_sdwa", k_pkmaxsdwa}};
  unsigned *d;
  hipMalloc(&d, 64);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  int blocks = cus * 8;   // 256-thread blocks: 8 per CU = 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
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
  return 0;
}
