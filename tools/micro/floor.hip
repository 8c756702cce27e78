// Launch-floor microbenchmarks on MI355X: what a short kernel costs before it does any work.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty(int* p) {
  if (threadIdx.x == 1024) p[0] = 1;
}
// every workgroup copies `units` 16-B units (shared source, L2-resident) into LDS, one barrier
__global__ void k_stage(const uint4* src, int units, int* p) {
  extern __shared__ uint4 lds[];
  for (int i = threadIdx.x; i < units; i += 256) lds[i] = src[i];
  __syncthreads();
  if (lds[threadIdx.x].x == 0xdeadbeef) p[0] = 1;
}
// every workgroup reads its own `units` units (distinct addresses, HBM/MALL) into LDS
__global__ void k_stage_own(const uint4* src, int units, int* p) {
  extern __shared__ uint4 lds[];
  const uint4* s = src + (size_t)blockIdx.x * units;
  for (int i = threadIdx.x; i < units; i += 256) lds[i] = s[i];
  __syncthreads();
  if (lds[threadIdx.x].x == 0xdeadbeef) p[0] = 1;
}
// every workgroup writes 32 KB of output (like a conv epilogue)
__global__ void k_store(uint2* dst) {
  uint2* d = dst + (size_t)blockIdx.x * 4096;
  for (int i = threadIdx.x; i < 4096; i += 256) d[i] = make_uint2(i, blockIdx.x);
}

template <class F>
float timeit(F f, int reps = 50) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

int main() {
  int* p;
  uint4* src;
  uint2* dst;
  hipMalloc(&p, 64);
  hipMalloc(&src, (size_t)64 << 20);
  hipMalloc(&dst, (size_t)64 << 20);
  hipMemset(src, 1, (size_t)64 << 20);
  hipFuncSetAttribute((const void*)k_stage, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)k_stage_own, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int wgs : {256, 640, 1280, 2560}) {
    printf("wgs %5d: empty %.2f us", wgs, timeit([&] { hipLaunchKernelGGL(k_empty, dim3(wgs), dim3(256), 0, 0, p); }));
    for (int kb : {16, 48, 128}) {
      const int units = kb * 64;
      printf(" | stage %3dKB shared %.2f own %.2f", kb,
             timeit([&] { hipLaunchKernelGGL(k_stage, dim3(wgs), dim3(256), units * 16, 0, src, units, p); }),
             wgs * (size_t)units * 16 <= ((size_t)64 << 20)
                 ? timeit([&] { hipLaunchKernelGGL(k_stage_own, dim3(wgs), dim3(256), units * 16, 0, src, units, p); })
                 : -1.f);
    }
    printf(" | store32KB %.2f\n", wgs * 32768 <= (64 << 20) ? timeit([&] { hipLaunchKernelGGL(k_store, dim3(wgs), dim3(256), 0, 0, dst); }) : -1.f);
  }
  return 0;
}
