// Exhaustive check of a cheaper SiLU against the fp32 build's exact one (detector.hip silu<true>):
// for every float bit pattern v (NaNs skipped), exact = v / (1 + expf(-v)) with an IEEE division,
// fast = the same expf, then the quotient by a reciprocal and one fused correction step
//   r = rcp(d), q0 = v * r, e = fma(-d, q0, v), q = fma(e, r, q0)
// with the exact division kept for d >= 2^126 (rcp would be subnormal) or a non-finite v / d.
// Prints the mismatch count and the first mismatches.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/silu_exact.hip -o /tmp/silu_exact && /tmp/silu_exact
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ float silu_exact(float v) { return v / (1.0f + expf(-v)); }

__device__ __forceinline__ float silu_fast(float v) {
  const float d = 1.0f + expf(-v);
  if (!(d < 0x1p126f) || !(fabsf(v) < INFINITY)) return v / d;  // rare lanes: the IEEE division
  const float r = __builtin_amdgcn_rcpf(d);
  const float q0 = v * r;
  const float e = __builtin_fmaf(-d, q0, v);
  return __builtin_fmaf(e, r, q0);
}

__global__ void check(unsigned long long base, unsigned* count, unsigned* first) {
  const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > 0xffffffffull) return;
  const float v = __uint_as_float((unsigned)i);
  if (v != v) return;
  const float a = silu_exact(v), b = silu_fast(v);
  if (__float_as_uint(a) != __float_as_uint(b)) {
    const unsigned k = atomicAdd(count, 1u);
    if (k < 16) first[k] = (unsigned)i;
  }
}

int main() {
  unsigned *count, *first;
  hipMalloc(&count, 4);
  hipMalloc(&first, 64);
  hipMemset(count, 0, 4);
  hipMemset(first, 0, 64);
  const unsigned long long chunk = 1ull << 30;
  for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
    hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, count, first);
  unsigned c = 0, f[16];
  hipMemcpy(&c, count, 4, hipMemcpyDeviceToHost);
  hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
  printf("{\"mismatches\": %u, \"first\": [", c);
  for (unsigned k = 0; k < (c < 16 ? c : 16); ++k) printf("%s\"0x%08x\"", k ? ", " : "", f[k]);
  printf("]}\n");
  return c != 0;
}
