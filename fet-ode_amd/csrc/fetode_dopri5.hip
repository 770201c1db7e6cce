// fetode_dopri5.hip — device pieces of the Dormand–Prince 5(4) solver (torchdiffeq Dopri5Solver,
// rk_common._runge_kutta_step / interp._interp_fit / interp._interp_evaluate / misc._rms_norm).
// Call sites in the reference: train_ecg_kan_fet_nn_ode.py:558-565, :1034-1041 and every
// default-method odeint (train_kanfet_node_predprey.py:252).
#include <algorithm>

#include "fetode_common.h"

using namespace fetode;

namespace {

struct Coef8 {
  float c[8];
};

// out = (y0 ? y0 : 0) + sum_{j<m} k[j] * c[j]   (sequential j order, then + y0)
__global__ void lincomb_kernel(const float* __restrict__ y0, const float* __restrict__ k, int64_t kstride, Coef8 c,
                               int m, float* __restrict__ out, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float acc = k[t] * c.c[0];
  for (int j = 1; j < m; ++j) acc = acc + k[j * kstride + t] * c.c[j];
  out[t] = y0 ? y0[t] + acc : acc;
}

// ---- the stage combine under autograd (dopri5._CombFn): coefficients on the device ----
// _Dopri5Grad differentiates through dt (torchdiffeq's step-size control is a tensor expression), so
// the coefficients c_j = beta_j dt are device values with a gradient.  Forward: out = y0 + sum_j k_j c_j
// with every product rounded and the running sum in j order, then + y0 (the op order of the torch
// expression it replaces: ks[0] * c[0] + ks[1] * c[1] + ..., then y0 + acc; no contraction).
// Backward: d k_j = c_j g (rounded product, as torch's), d c_j = <g, k_j> (fp32 per-thread sums, then
// fixed-order block and grid sums: deterministic for a given n).
constexpr int kCombMax = 8;
constexpr int kCombThreads = 256;
constexpr int kCombMaxBlocks = 1024;

struct CombPtrs {
  const float* k[kCombMax];
  float* gk[kCombMax];
};

__global__ __launch_bounds__(kCombThreads) void comb_fwd_kernel(const float* __restrict__ y0, CombPtrs p,
                                                                const float* __restrict__ c, int m,
                                                                float* __restrict__ out, int64_t n) {
#pragma clang fp contract(off)
  float cj[kCombMax];
#pragma unroll
  for (int j = 0; j < kCombMax; ++j) cj[j] = j < m ? c[j] : 0.f;
  for (int64_t t = (int64_t)blockIdx.x * kCombThreads + threadIdx.x; t < n; t += (int64_t)gridDim.x * kCombThreads) {
    float acc = p.k[0][t] * cj[0];
#pragma unroll
    for (int j = 1; j < kCombMax; ++j)
      if (j < m) acc = acc + p.k[j][t] * cj[j];
    out[t] = y0 ? y0[t] + acc : acc;
  }
}

// part[block][j] = this block's share of <g, k_j> (when want_c)
__global__ __launch_bounds__(kCombThreads) void comb_bwd_kernel(const float* __restrict__ g, CombPtrs p,
                                                                const float* __restrict__ c, int m, int want_c,
                                                                float* __restrict__ part, int64_t n) {
#pragma clang fp contract(off)
  __shared__ float red[kCombMax][kCombThreads];
  float cj[kCombMax], dot[kCombMax];
#pragma unroll
  for (int j = 0; j < kCombMax; ++j) {
    cj[j] = j < m ? c[j] : 0.f;
    dot[j] = 0.f;
  }
  for (int64_t t = (int64_t)blockIdx.x * kCombThreads + threadIdx.x; t < n; t += (int64_t)gridDim.x * kCombThreads) {
    const float gv = g[t];
#pragma unroll
    for (int j = 0; j < kCombMax; ++j) {
      if (j < m) {
        if (p.gk[j]) p.gk[j][t] = gv * cj[j];
        if (want_c) dot[j] = dot[j] + gv * p.k[j][t];
      }
    }
  }
  if (!want_c) return;
#pragma unroll
  for (int j = 0; j < kCombMax; ++j) red[j][threadIdx.x] = dot[j];
  __syncthreads();
  for (int w = kCombThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
#pragma unroll
      for (int j = 0; j < kCombMax; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + w];
    }
    __syncthreads();
  }
  if ((int)threadIdx.x < kCombMax) part[(int64_t)blockIdx.x * kCombMax + threadIdx.x] = red[threadIdx.x][0];
}

// gc[j] = sum over blocks of part[b][j]: wave j, lane l sums blocks l, l + 64, ... in order, then a
// fixed tree over the lanes (a serial loop over 512 partials was 51 us of latency per call)
__global__ __launch_bounds__(64 * kCombMax) void comb_dot_kernel(const float* __restrict__ part, int nb, int m,
                                                                 float* __restrict__ gc) {
  __shared__ float red[kCombMax][64];
  const int j = threadIdx.x >> 6, l = threadIdx.x & 63;
  float s = 0.f;
  if (j < m)
    for (int b = l; b < nb; b += 64) s += part[(int64_t)b * kCombMax + j];
  red[j][l] = s;
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (l < w) red[j][l] += red[j][l + w];
    __syncthreads();
  }
  if (l == 0 && j < m) gc[j] = red[j][0];
}

// sum(((a - sub) / (atol + rtol * max(|y0|, |y1|)))^2), one workgroup, fp64 accumulation;
// RMS = true writes sqrt(sum / n) as fp32 (misc._rms_norm), false the raw fp64 sum
template <bool RMS>
__global__ void scaled_rms_kernel(const float* __restrict__ a, const float* __restrict__ sub,
                                  const float* __restrict__ y0, const float* __restrict__ y1, float rtol,
                                  float atol, int64_t n, void* __restrict__ out_) {
  __shared__ double red[1024];
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  double s = 0.0;
  int nf = 0;
  for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
    nf |= !__builtin_isfinite(y0[t]);
    const float v = sub ? a[t] - sub[t] : a[t];
    const float m = y1 ? fmaxf(fabsf(y0[t]), fabsf(y1[t])) : fabsf(y0[t]);
    const float tol = atol + rtol * m;
    const float q = v / tol;
    s += (double)q * (double)q;
  }
  red[threadIdx.x] = s;
  if (nf) atomicOr(&bad, 1);
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if constexpr (RMS) {
      float* out = static_cast<float*>(out_);
      out[0] = sqrtf((float)(red[0] / (double)n));
      out[1] = bad ? 1.0f : 0.0f;  // torchdiffeq asserts torch.isfinite(y0).all() every step
    } else {
      double* out = static_cast<double*>(out_);
      out[0] = red[0];
      out[1] = bad ? 1.0 : 0.0;
    }
  }
}

// The same sum over many workgroups (a single workgroup is load-latency-bound: 0.33 ms at n = 524 288,
// the ETT latent batch): workgroup g sums its contiguous slice [g S, (g + 1) S) (a strided loop per
// thread, then a fixed tree), writes an fp64 partial, and the last workgroup to arrive sums the
// partials in index order — deterministic, independent of arrival order.  ws: kRmsMaxGroups
// (partial, bad) pairs + one arrival counter (zero between calls: the last workgroup resets it).
constexpr int kRmsMaxGroups = 512;
constexpr int kRmsThreads = 256;
template <bool RMS>
__global__ __launch_bounds__(kRmsThreads) void scaled_rms_grid_kernel(
    const float* __restrict__ a, const float* __restrict__ sub, const float* __restrict__ y0,
    const float* __restrict__ y1, float rtol, float atol, int64_t n, int64_t slice, double* __restrict__ ws,
    void* __restrict__ out_) {
  __shared__ double red[kRmsThreads];
  __shared__ int bad, last;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * slice, hi = lo + slice < n ? lo + slice : n;
  double s = 0.0;
  int nf = 0;
  for (int64_t t = lo + threadIdx.x; t < hi; t += kRmsThreads) {
    nf |= !__builtin_isfinite(y0[t]);
    const float v = sub ? a[t] - sub[t] : a[t];
    const float m = y1 ? fmaxf(fabsf(y0[t]), fabsf(y1[t])) : fabsf(y0[t]);
    const float q = v / (atol + rtol * m);
    s += (double)q * (double)q;
  }
  red[threadIdx.x] = s;
  if (nf) atomicOr(&bad, 1);
  __syncthreads();
  for (int w = kRmsThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  unsigned* cnt = reinterpret_cast<unsigned*>(ws + 2 * kRmsMaxGroups);
  if (threadIdx.x == 0) {
    ws[2 * blockIdx.x] = red[0];
    ws[2 * blockIdx.x + 1] = bad ? 1.0 : 0.0;
    __threadfence();
    last = atomicAdd(cnt, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the last workgroup: partials in index order (thread i sums i, i + 256, ..; then the tree)
  double p = 0.0, b = 0.0;
  for (unsigned g = threadIdx.x; g < gridDim.x; g += kRmsThreads) {
    p += __hip_atomic_load(&ws[2 * g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_load(&ws[2 * g + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  red[threadIdx.x] = p;
  __syncthreads();
  for (int w = kRmsThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (b != 0.0) atomicOr(&bad, 1);   // (bad was this workgroup's own flag: OR the others' in)
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (RMS) {
      float* out = static_cast<float*>(out_);
      out[0] = sqrtf((float)(red[0] / (double)n));
      out[1] = bad ? 1.0f : 0.0f;
    } else {
      double* out = static_cast<double*>(out_);
      out[0] = red[0];
      out[1] = bad ? 1.0 : 0.0;
    }
    *cnt = 0u;   // ready for the next call on this workspace
  }
}

// interp._interp_fit with y_mid = y0 + k . (dt * mid); coeffs (5, n) = [e, d, c, b, a]
__global__ void interp_fit_kernel(const float* __restrict__ y0, const float* __restrict__ y1,
                                  const float* __restrict__ k, int64_t kstride, Coef8 mid, float dt,
                                  float* __restrict__ co, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float acc = k[t] * mid.c[0];
  for (int j = 1; j < 7; ++j) acc = acc + k[j * kstride + t] * mid.c[j];
  const float y0v = y0[t], y1v = y1[t];
  const float ym = y0v + acc;
  const float f0 = k[t], f1 = k[6 * kstride + t];
  const float a = ((2.0f * dt) * (f1 - f0) - 8.0f * (y1v + y0v)) + 16.0f * ym;
  const float b = ((dt * (5.0f * f0 - 3.0f * f1) + 18.0f * y0v) + 14.0f * y1v) - 32.0f * ym;
  const float c = ((dt * (f1 - 4.0f * f0) - 11.0f * y0v) - 5.0f * y1v) + 16.0f * ym;
  co[t] = y0v;
  co[n + t] = dt * f0;
  co[2 * n + t] = c;
  co[3 * n + t] = b;
  co[4 * n + t] = a;
}

__global__ void interp_eval_kernel(const float* __restrict__ co, float x, float* __restrict__ out, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float total = co[t] + x * co[n + t];
  float xp = x;
  for (int j = 2; j < 5; ++j) {
    xp = xp * x;
    total = total + xp * co[j * n + t];
  }
  out[t] = total;
}

template <bool RMS>
int scaled_norm(const float* a, const float* sub, const float* y0, const float* y1, double rtol, double atol,
                       int64_t n, void* out, void* workspace, hipStream_t s) {
  // small n or no workspace: one workgroup; else workgroups of >= 2048 elements, at most 512
  const int64_t groups = (n + 2047) / 2048;
  if (!workspace || groups <= 1) {
    hipLaunchKernelGGL(scaled_rms_kernel<RMS>, dim3(1), dim3(1024), 0, s, a, sub, y0, y1, (float)rtol, (float)atol, n,
                       out);
  } else {
    const int g = (int)(groups < kRmsMaxGroups ? groups : kRmsMaxGroups);
    const int64_t slice = (n + g - 1) / g;
    const int gg = (int)((n + slice - 1) / slice);
    hipLaunchKernelGGL(scaled_rms_grid_kernel<RMS>, dim3((unsigned)gg), dim3(kRmsThreads), 0, s, a, sub, y0, y1,
                       (float)rtol, (float)atol, n, slice, (double*)workspace, out);
  }
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // namespace

extern "C" {

int fetode_lincomb(const float* y0, const float* k, int64_t kstride, const float* c, int32_t m, float* out,
                   int64_t n, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!k || !c || !out || m < 1 || m > 8) return set_err(FETODE_EINVAL, "lincomb: bad arguments (m=%d)", m);
  Coef8 cc;
  for (int j = 0; j < 8; ++j) cc.c[j] = j < m ? c[j] : 0.f;
  hipLaunchKernelGGL(lincomb_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, y0, k, kstride, cc, m,
                     out, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_comb_workspace(int64_t n) {
  return (int64_t)sizeof(float) * kCombMax * std::max(1, std::min(kCombMaxBlocks, nblk(n, kCombThreads)));
}

int fetode_comb_forward(const float* y0, const float* const* k, int32_t m, const float* c, float* out, int64_t n,
                        void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!k || !c || !out || m < 1 || m > kCombMax) return set_err(FETODE_EINVAL, "comb_forward: bad arguments (m=%d)", m);
  CombPtrs p{};
  for (int j = 0; j < m; ++j) {
    if (!k[j]) return set_err(FETODE_EINVAL, "comb_forward: k[%d] is null", j);
    p.k[j] = k[j];
  }
  const int nb = std::min(kCombMaxBlocks, nblk(n, kCombThreads));
  hipLaunchKernelGGL(comb_fwd_kernel, dim3(nb), dim3(kCombThreads), 0, (hipStream_t)stream, y0, p, c, (int)m, out, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_comb_backward(const float* g, const float* const* k, int32_t m, const float* c, float* const* gk,
                         float* gc, void* workspace, int64_t n, void* stream) {
  if (n <= 0) {   // an empty state (as the forward accepts): d/d c = 0, nothing else to write
    if (m < 1 || m > kCombMax) return set_err(FETODE_EINVAL, "comb_backward: bad arguments (m=%d)", m);
    if (gc) HIP_CHECK_RET(hipMemsetAsync(gc, 0, sizeof(float) * (size_t)m, (hipStream_t)stream));
    return FETODE_OK;
  }
  if (!g || !k || !c || m < 1 || m > kCombMax || (gc && !workspace))
    return set_err(FETODE_EINVAL, "comb_backward: bad arguments (m=%d)", m);
  CombPtrs p{};
  for (int j = 0; j < m; ++j) {
    if (!k[j]) return set_err(FETODE_EINVAL, "comb_backward: k[%d] is null", j);
    p.k[j] = k[j];
    p.gk[j] = gk ? gk[j] : nullptr;
  }
  const int nb = std::min(kCombMaxBlocks, nblk(n, kCombThreads));
  hipLaunchKernelGGL(comb_bwd_kernel, dim3(nb), dim3(kCombThreads), 0, (hipStream_t)stream, g, p, c, (int)m,
                     gc ? 1 : 0, (float*)workspace, n);
  LAUNCH_CHECK();
  if (gc) {
    hipLaunchKernelGGL(comb_dot_kernel, dim3(1), dim3(64 * kCombMax), 0, (hipStream_t)stream, (const float*)workspace, nb,
                       (int)m, gc);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int64_t fetode_scaled_rms_workspace(int64_t n) {
  (void)n;
  return (int64_t)sizeof(double) * (2 * kRmsMaxGroups + 1);
}

int fetode_scaled_rms(const float* a, const float* sub, const float* y0, const float* y1, double rtol, double atol,
                      int64_t n, float* out, void* workspace, void* stream) {
  if (n <= 0 || !a || !y0 || !out) return set_err(FETODE_EINVAL, "scaled_rms: bad arguments");
  return scaled_norm<true>(a, sub, y0, y1, rtol, atol, n, out, workspace, (hipStream_t)stream);
}

int fetode_scaled_sumsq(const float* a, const float* sub, const float* y0, const float* y1, double rtol, double atol,
                        int64_t n, double* out, void* workspace, void* stream) {
  if (n < 0 || !out || (n > 0 && (!a || !y0))) return set_err(FETODE_EINVAL, "scaled_sumsq: bad arguments");
  if (n == 0) return hipMemsetAsync(out, 0, 2 * sizeof(double), (hipStream_t)stream) == hipSuccess
                         ? FETODE_OK
                         : set_err(FETODE_EHIP, "scaled_sumsq: memset failed");
  return scaled_norm<false>(a, sub, y0, y1, rtol, atol, n, out, workspace, (hipStream_t)stream);
}

int fetode_interp_fit(const float* y0, const float* y1, const float* k, int64_t kstride, const float* mid_dt,
                      float dt, float* coeffs, int64_t n, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!y0 || !y1 || !k || !mid_dt || !coeffs) return set_err(FETODE_EINVAL, "interp_fit: null pointer");
  Coef8 cc;
  for (int j = 0; j < 8; ++j) cc.c[j] = j < 7 ? mid_dt[j] : 0.f;
  hipLaunchKernelGGL(interp_fit_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, y0, y1, k, kstride,
                     cc, dt, coeffs, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_interp_eval(const float* coeffs, float x, float* out, int64_t n, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!coeffs || !out) return set_err(FETODE_EINVAL, "interp_eval: null pointer");
  hipLaunchKernelGGL(interp_eval_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, coeffs, x, out, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"
