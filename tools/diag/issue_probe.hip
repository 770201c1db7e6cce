// Microbenchmark: aggregate VALU issue rate of one SIMD against the number of resident waves
// (gfx950).  Every wave runs N iterations of a fixed instruction block; the kernel is launched
// with w * 1024 one-wave workgroups (w waves per SIMD, all resident: few registers, no LDS), and
// the wall time (hipEvent) gives SIMD cycles per wave-instruction at the measured clock
// (s_memtime deltas per wave give the wave's own view).  Blocks:
//   fma16   16 independent v_fma_f32 chains
//   pk8     8 independent v_pk_fma_f32 chains (16 fp32 results)
//   exp16   16 independent v_exp_f32
//   rcp16   16 independent v_rcp_f32
//   pair4   4 independent Ferro element pairs as fused4's v4_pair (6 transcendental + 7 packed)
//   dep     one dependent v_fma_f32 chain (latency)
//   deptr   one dependent exp -> add -> rcp chain (latency)
// Build (not tracked):  hipcc --offload-arch=gfx950 -O3 -o tools/diag/issue_probe tools/diag/issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void probe(float* out, float a, float b, int n, long long* cyc) {
  float s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = threadIdx.x * 0.001f + i * 0.01f;
  const f2 aa = {a, a}, bb = {b, b};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < n; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[i]) : "v"(a), "v"(b));
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f2 v = {s[2 * i], s[2 * i + 1]};
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(aa), "v"(bb));
        s[2 * i] = v.x;
        s[2 * i + 1] = v.y;
      }
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(s[i]));
    } else if constexpr (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_rcp_f32 %0, %0" : "+v"(s[i]));
    } else if constexpr (MODE == 4) {
      // 4 pairs: s = rcp(e*ep + 1); m = g*s + 1; z = kE*m + k2*x; th = 1 - 2 rcp(exp(z) + 1); acc += cp th
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f2 ep = {s[4 * p], s[4 * p + 1]}, acc = {s[4 * p + 2], s[4 * p + 3]};
        f2 t, m, z, k;
        asm volatile("v_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0]" : "=v"(t) : "v"(aa), "v"(ep));
        asm volatile("v_rcp_f32 %0, %1" : "=v"(t.x) : "v"(t.x));
        asm volatile("v_rcp_f32 %0, %1" : "=v"(t.y) : "v"(t.y));
        asm volatile("v_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0]" : "=v"(m) : "v"(bb), "v"(t));
        asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(k) : "v"(aa), "v"(ep));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(z) : "v"(ep), "v"(m), "v"(k));
        asm volatile("v_exp_f32 %0, %1" : "=v"(z.x) : "v"(z.x));
        asm volatile("v_exp_f32 %0, %1" : "=v"(z.y) : "v"(z.y));
        asm volatile("v_pk_add_f32 %0, %1, 1.0 op_sel_hi:[1,0]" : "=v"(z) : "v"(z));
        asm volatile("v_rcp_f32 %0, %1" : "=v"(z.x) : "v"(z.x));
        asm volatile("v_rcp_f32 %0, %1" : "=v"(z.y) : "v"(z.y));
        asm volatile("v_pk_fma_f32 %0, %1, -2.0, 1.0 op_sel_hi:[1,0,0]" : "=v"(z) : "v"(z));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(ep), "v"(z));
        s[4 * p + 2] = acc.x;
        s[4 * p + 3] = acc.y;
        s[4 * p] += 1e-30f * acc.x;  // keep ep live and changing (one v_fma per pair)
      }
    } else if constexpr (MODE == 5) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[0]) : "v"(a), "v"(b));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(s[0]));
        asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(s[0]));
        asm volatile("v_rcp_f32 %0, %0" : "+v"(s[0]));
      }
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += s[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*KFn)(float*, float, float, int, long long*);
int main() {
  float* o;
  long long* c;
  hipMalloc(&o, 8 * 1024 * 64 * 4);
  hipMalloc(&c, 8 * 1024 * 8);
  static long long h[8 * 1024];
  const char* names[] = {"fma16", "pk8", "exp16", "rcp16", "pair4", "dep", "deptr"};
  // wave-instructions per iteration, VALU issue model in quad-cycles (transcendental 2, else 1)
  const double insts[] = {16, 8, 16, 16, 4 * 14, 16, 12};
  const double model[] = {16, 8, 32, 32, 4 * (6 * 2 + 8), 16, 4 * (2 + 1 + 2)};
  KFn fns[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  printf("device clock attribute %d kHz\n", clk_khz);
  const int n = 2048;
  for (int mode = 0; mode < 7; ++mode) {
    for (int w : {1, 2, 3, 4, 6, 8}) {
      const int wgs = w * 1024;
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(fns[mode], dim3(wgs), dim3(64), 0, 0, o, 1.0000001f, 0.5f, n, c);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      hipMemcpy(h, c, wgs * 8, hipMemcpyDeviceToHost);
      double m = 0;
      for (int i = 0; i < wgs; ++i) m += h[i];
      m /= wgs;
      // SIMD cycles per wave-instruction from the wall time at 2.4 GHz and from the wave's own count
      const double tot_inst = (double)w * n * insts[mode];
      const double simd_cyc_wall = best * 1e-3 * 2.4e9 / tot_inst;
      const double wave_cyc = m / ((double)n * insts[mode]);
      const double quad_busy = (double)w * n * model[mode] * 4 / (best * 1e-3 * 2.4e9);
      printf("%-6s w=%d  ms=%8.3f  simd_cyc/inst(wall@2.4G)=%6.2f  wave_cyc/inst=%6.2f  quadmodel_busy=%5.2f\n",
             names[mode], w, best, simd_cyc_wall, wave_cyc, quad_busy);
    }
  }
  return 0;
}
