// Probe (development tool): which XCD / SE / CU each CU-mask bit selects.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_where(unsigned* out) {
  unsigned x, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) { out[0] = x; out[1] = hw; }
}
int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* d; hipMalloc(&d, 8);
  const int words = (ncu + 31) / 32;
  printf("CUs %d\n", ncu);
  for (int bit = 0; bit < ncu; ++bit) {
    std::vector<uint32_t> m(words, 0u);
    m[bit / 32] = 1u << (bit % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) { printf("mask fail\n"); return 1; }
    hipLaunchKernelGGL(k_where, dim3(1), dim3(64), 0, s, d);
    unsigned h[2];
    hipStreamSynchronize(s);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    // HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] ...
    printf("bit %3d -> xcc %u se %u sh %u cu %u\n", bit, h[0] & 7, (h[1] >> 13) & 7, (h[1] >> 12) & 1, (h[1] >> 8) & 15);
    hipStreamDestroy(s);
  }
  return 0;
}
