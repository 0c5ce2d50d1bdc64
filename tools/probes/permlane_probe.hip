// Ground truth for v_permlane16/32_swap as exposed by the clang builtins on gfx950: each lane writes
// the two results of swap(x, x) and swap(x, y) for x = lane, y = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  auto c = __builtin_amdgcn_permlane16_swap(l, l, false, false);
  auto d = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  out[l * 8 + 0] = a[0]; out[l * 8 + 1] = a[1];
  out[l * 8 + 2] = b[0]; out[l * 8 + 3] = b[1];
  out[l * 8 + 4] = c[0]; out[l * 8 + 5] = c[1];
  out[l * 8 + 6] = d[0]; out[l * 8 + 7] = d[1];
}
int main() {
  unsigned* d; unsigned h[64 * 8];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 15, 16, 17, 31, 32, 33, 47, 48, 63})
    printf("lane %2d: p32(x,x)=(%u,%u) p32(x,y)=(%u,%u) p16(x,x)=(%u,%u) p16(x,y)=(%u,%u)\n", l, h[l*8], h[l*8+1],
           h[l*8+2], h[l*8+3], h[l*8+4], h[l*8+5], h[l*8+6], h[l*8+7]);
  return 0;
}
