// Microbenchmark: scalar-ALU throughput per CU on gfx950 (is SALU issue shared by a CU's four SIMDs?).
// Every CU runs 1, 2, 4 and 8 waves per SIMD of a loop of 16 independent SGPR chains x ITER of
// s_add_u32; then the same with a VALU chain interleaved (does SALU issue steal VALU slots?).
// Scalar ALU only: no scalar memory instructions.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048

__global__ void __launch_bounds__(256) k_salu(unsigned *out, unsigned b)
{
  unsigned r[16];
  for (int k = 0; k < 16; k++) r[k] = __builtin_amdgcn_readfirstlane(blockIdx.x * (k + 1));
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) asm volatile("s_add_u32 %0, %0, %1" : "+s"(r[k]) : "s"(b) : "scc");
  }
  unsigned s = 0;
  for (int k = 0; k < 16; k++) s ^= r[k];
  if (s == 0x1234567u && threadIdx.x == 0) out[0] = s;
}

__global__ void __launch_bounds__(256) k_valu(unsigned *out, unsigned b)
{
  unsigned v[16];
  for (int k = 0; k < 16; k++) v[k] = threadIdx.x * (k + 1);
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[k]) : "v"(b));
  }
  unsigned s = 0;
  for (int k = 0; k < 16; k++) s ^= v[k];
  if (s == 0x1234567u) out[0] = s;
}

__global__ void __launch_bounds__(256) k_mixed(unsigned *out, unsigned b)
{
  unsigned r[16], v[16];
  for (int k = 0; k < 16; k++) {
    r[k] = __builtin_amdgcn_readfirstlane(blockIdx.x * (k + 1));
    v[k] = threadIdx.x * (k + 1);
  }
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      asm volatile("s_add_u32 %0, %0, %1" : "+s"(r[k]) : "s"(b) : "scc");
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[k]) : "v"(b));
    }
  }
  unsigned s = 0;
  for (int k = 0; k < 16; k++) s ^= r[k] ^ v[k];
  if (s == 0x1234567u) out[0] = s;
}

typedef void (*kfn)(unsigned *, unsigned);
int main()
{
  struct {
    const char *n;
    kfn f;
  } ks[] = {{"s_add_u32", k_salu}, {"v_add_u32", k_valu}, {"s_add + v_add", k_mixed}};
  unsigned *d;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  hipEvent_t a, e;
  hipEventCreate(&a);
  hipEventCreate(&e);
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = cus * wps;   // 256-thread blocks: wps per CU = wps waves per SIMD
    printf("--- %d wave(s) per SIMD\n", wps);
    for (auto &k : ks) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, d, 3u);
        hipEventRecord(e);
        hipEventSynchronize(e);
        float ms;
        hipEventElapsedTime(&ms, a, e);
        if (rep) {
          const double per_cu = (double)blocks * 4 * ITER * 16 / cus;   // instructions of the named kind per CU
          printf("%-16s %8.3f ms  %7.3f G inst/s per CU  -> %5.2f cycles per instruction per CU @2.4GHz\n", k.n, ms,
                 per_cu / (ms * 1e6), 2.4e9 * ms * 1e-3 / per_cu);
        }
      }
    }
  }
  return 0;
}
