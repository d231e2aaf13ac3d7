// LDS allocation granularity probe: occupancy (256-thread workgroups per CU) against dynamic LDS bytes
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k_lds(int *o)
{
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) o[blockIdx.x] = s[255];
}
int main()
{
  int prev = -1;
  for (size_t b = 12288; b <= 24576; b += 128) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lds, 256, b) != hipSuccess) return 1;
    if (occ != prev) printf("lds %zu B -> %d workgroups per CU\n", b, occ);
    prev = occ;
  }
  return 0;
}
