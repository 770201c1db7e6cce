// Microbenchmark: issue cost of v_pk_fma_f32 vs two v_fma_f32 (gfx950), one and two waves per
// SIMD.  8 independent accumulator chains per lane, N iterations; reports cycles per instruction.
// Build (not tracked):  hipcc --offload-arch=gfx950 -O3 -o tools/diag/pk_issue tools/diag/pk_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, float a, float b, int n, long long* cyc) {
  float s[16];
  for (int i = 0; i < 16; ++i) s[i] = threadIdx.x * 0.001f + i;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < n; ++it) {
    if (MODE == 0) {  // 16 scalar fma
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[i]) : "v"(a), "v"(b));
    } else if (MODE == 1) {  // 8 packed fma (same 16 results)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f2 v = {s[2 * i], s[2 * i + 1]};
        v = __builtin_elementwise_fma(v, f2{a, a}, f2{b, b});
        s[2 * i] = v.x; s[2 * i + 1] = v.y;
      }
    } else {  // 16 exp
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = __builtin_amdgcn_exp2f(s[i]);
    }
    asm volatile("" ::: "memory");
  }
  long long t1 = __builtin_readcyclecounter();
  float acc = 0.f;
  for (int i = 0; i < 16; ++i) acc += s[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float* o; long long* c; hipMalloc(&o, 1 << 24); hipMalloc(&c, 1 << 20);
  const int n = 4096;
  long long h[4096];
  for (int waves : {1024, 2048}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0) k<0><<<waves, 64>>>(o, 1.0001f, 0.5f, n, c);
        if (mode == 1) k<1><<<waves, 64>>>(o, 1.0001f, 0.5f, n, c);
        if (mode == 2) k<2><<<waves, 64>>>(o, 1.0001f, 0.5f, n, c);
      }
      hipMemcpy(h, c, waves * 8, hipMemcpyDeviceToHost);
      double m = 0; for (int i = 0; i < waves; ++i) m += h[i]; m /= waves;
      const int ninst = mode == 1 ? 8 : 16;
      printf("waves=%d mode=%s cycles/instr=%.2f (per 16 results %.1f)\n", waves, mode == 0 ? "fma" : mode == 1 ? "pk_fma" : "exp", m / n / ninst, m / n);
    }
  }
  return 0;
}
