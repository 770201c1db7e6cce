// fetode_device.h — device helpers shared by the fetode kernels (gfx950 / CDNA4).
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit
// (__builtin_fmaf), so the stage-combine arithmetic keeps torchdiffeq's exact
// op order and rounding (rk_common.rk4_alt_step_func) while the field maths
// uses FMAs where we choose to.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FETODE_LOG2E 1.4426950408889634f

namespace fetode {

// v_exp_f32: 2^x (inf for large x, 0 for very negative x)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
// v_rcp_f32: 1/x to 1 ulp, rcp(inf) = 0
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float ffma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// logistic sigmoid of z given zl = -z*log2(e):  1/(1+2^zl)
__device__ __forceinline__ float sig_from_neg_l2(float zl) { return rcp(1.0f + ex2(zl)); }

// SiLU(x) = x * sigmoid(x)  (efficientkan base_activation = nn.SiLU)
__device__ __forceinline__ float silu(float x) { return x * sig_from_neg_l2(-x * FETODE_LOG2E); }

// Local-support Cox–de Boor (efficientkan.py:117-131) for one input value.
// g: NG knots, rk: reciprocal knot spans rk[(k-1)*(NG-1)+j] = 1/(g[j+k]-g[j]).
// Writes the NS = NG-1-SO level-SO bases to out[0..NS) (all zero outside
// [g0, g_{NG-1}) exactly like the half-open indicator at :122; NaN for non-finite x, as the
// reference's (x-g)/d*0 products give).
// Only the <= SO+1 non-zero bases of the active interval are evaluated; the
// recursion per entry is the reference's ((x-g_j)/d)*B + ((g_{j+k+1}-x)/d')*B'
// with the divisions replaced by the precomputed reciprocals.
template <int SO, typename KnotPtr, typename OutF>
__device__ __forceinline__ void bspline_local(float x, int NG, KnotPtr g, KnotPtr rk, OutF&& out) {
  const int NS = NG - 1 - SO;
  if (!__builtin_isfinite(x)) {  // reference: (x-g)/d * 0 = NaN for x = +-inf or NaN
    for (int c = 0; c < NS; ++c) out(c, __builtin_nanf(""));
    return;
  }
  int m = -1;
  for (int j = 0; j < NG; ++j) m += (x >= g[j]) ? 1 : 0;
  for (int c = 0; c < NS; ++c) out(c, 0.0f);
  if (m < 0 || m > NG - 2) return;
  float N[SO + 2];
#pragma unroll
  for (int r = 0; r < SO + 2; ++r) N[r] = 0.0f;
  N[SO] = 1.0f;
#pragma unroll
  for (int k = 1; k <= SO; ++k) {
    float M[SO + 2];
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.0f;
#pragma unroll
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= NG - 2 - k) {
        const float* rkk = &rk[(k - 1) * (NG - 1)];
        float left = ((x - g[j]) * rkk[j]) * N[r];
        float right = ((g[j + k + 1] - x) * rkk[j + 1]) * N[r + 1];
        M[r] = left + right;
      }
    }
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
#pragma unroll
  for (int r = 0; r <= SO; ++r) {
    const int j = m - SO + r;
    if (j >= 0 && j < NS) out(j, N[r]);
  }
}

// Exact-reference Cox–de Boor with true divisions (bitwise equal to the CPU
// reference when compiled without contraction): used by the standalone
// KANLinear.b_splines / forward kernels.
template <int SO, typename OutF>
__device__ __forceinline__ void bspline_local_div(float x, int NG, const float* __restrict__ g,
                                                  OutF&& out) {
  const int NS = NG - 1 - SO;
  if (!__builtin_isfinite(x)) {  // reference: (x-g)/d * 0 = NaN for x = +-inf or NaN
    for (int c = 0; c < NS; ++c) out(c, __builtin_nanf(""));
    return;
  }
  int m = -1;
  for (int j = 0; j < NG; ++j) m += (x >= g[j]) ? 1 : 0;
  for (int c = 0; c < NS; ++c) out(c, 0.0f);
  if (m < 0 || m > NG - 2) return;
  float N[SO + 2];
#pragma unroll
  for (int r = 0; r < SO + 2; ++r) N[r] = 0.0f;
  N[SO] = 1.0f;
#pragma unroll
  for (int k = 1; k <= SO; ++k) {
    float M[SO + 2];
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.0f;
#pragma unroll
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= NG - 2 - k) {
        float left = ((x - g[j]) / (g[j + k] - g[j])) * N[r];
        float right = ((g[j + k + 1] - x) / (g[j + k + 1] - g[j + 1])) * N[r + 1];
        M[r] = left + right;
      }
    }
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
#pragma unroll
  for (int r = 0; r <= SO; ++r) {
    const int j = m - SO + r;
    if (j >= 0 && j < NS) out(j, N[r]);
  }
}

// ---- cross-lane helpers (DPP) -------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                               false));
}
// the same with an undefined old value (no zero-init move): only for controls where every lane
// reads a valid source (row_newbcast)
template <int CTRL>
__device__ __forceinline__ float dppm(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over the 16 lanes of a row, result on every lane of the row
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0x128>(v);  // row_ror:8
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x122>(v);  // row_ror:2
  v += dpp<0x121>(v);  // row_ror:1
  return v;
}
// gfx950 lane swaps, in place: permlane32 swaps lanes 32-63 of p with lanes 0-31 of q; permlane16
// swaps the odd rows of p with the even rows of q.  Inline asm: this compiler's builtins for them
// treat the two results as one register.  The s_nop covers the VALU-write -> permlane-read hazard.
__device__ __forceinline__ void permlane32_swap(float& p, float& q) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(p), "+v"(q));
}
__device__ __forceinline__ void permlane16_swap(float& p, float& q) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p), "+v"(q));
}
}  // namespace fetode
