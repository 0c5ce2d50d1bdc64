// Per-CU fetch rate of L2-resident data: LDS-DMA (global_load_lds_dwordx4, the GEMMs' path) vs plain
// global_load_dwordx4 into VGPRs.  One workgroup per CU, every workgroup sweeps the same 2 MiB window
// (resident in each XCD's 4 MiB L2) 1 KiB per wave-instruction.  Prints bytes per clock per CU at the
// given clock (diagnostic only: tells whether the ~20 B/clk/CU the GEMM K loops reach is a property of the
// LDS-DMA path or of the CU's vector-memory path as a whole).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/fetch_probe.hip -o build/fetch_probe && build/fetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int WIN = 2 << 20;          // bytes swept by every workgroup
constexpr int ITERS = 2048;           // 8 KiB-per-wave batches per wave

typedef __attribute__((address_space(3))) void* lptr_t;

template <int MODE, int WAVES>
__global__ void __launch_bounds__(WAVES * 64, 1) probe(const char* __restrict__ src, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char lds[WAVES * 16384];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned base = (blockIdx.x * 65536u + wave * 8192u) % WIN;
  uint4 acc = {0, 0, 0, 0};
  for (int it = 0; it < ITERS; ++it) {
    const unsigned off = (base + (unsigned)it * (WAVES * 8192u)) % WIN;
    if (MODE == 0) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lptr_t)(lds + wave * 16384 + (it & 1) * 8192));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const char* p = src + off + j * 1024 + lane * 16;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(m0 + j * 1024)
                     : "memory");
      }
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // the previous batch landed; this one in flight
    } else {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const uint4*>(src + off + j * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) { acc.x ^= v[j].x; acc.y ^= v[j].y; acc.z ^= v[j].z; acc.w ^= v[j].w; }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 0) acc.x = reinterpret_cast<const unsigned*>(lds)[threadIdx.x];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int MODE, int WAVES>
void run(const char* src, unsigned* out, int ncu, double ghz) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<MODE, WAVES>), dim3(ncu), dim3(WAVES * 64), 0, 0, src, out);   // warm-up
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<MODE, WAVES>), dim3(ncu), dim3(WAVES * 64), 0, 0, src, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)reps * ncu * WAVES * ITERS * 8192.0;
  const double s = ms / 1e3;
  printf("%-14s waves/CU %d: %.3f ms  %.2f TB/s chip  %.1f B/clk/CU at %.2f GHz\n",
         MODE == 0 ? "LDS-DMA" : "global->VGPR", WAVES, ms / reps, bytes / s / 1e12, bytes / s / (ghz * 1e9) / ncu, ghz);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  char* src;
  unsigned* out;
  hipMalloc(&src, WIN + 65536);
  hipMemset(src, 0x5a, WIN + 65536);
  hipMalloc(&out, (size_t)ncu * 1024 * 4);
  const double ghz = 2.0;
  run<0, 4>(src, out, ncu, ghz);
  run<0, 8>(src, out, ncu, ghz);
  run<1, 4>(src, out, ncu, ghz);
  run<1, 8>(src, out, ncu, ghz);
  run<0, 4>(src, out, ncu, ghz);
  run<1, 4>(src, out, ncu, ghz);
  return 0;
}
