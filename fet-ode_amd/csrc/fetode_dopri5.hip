// fetode_dopri5.hip — device pieces of the Dormand–Prince 5(4) solver (torchdiffeq Dopri5Solver,
// rk_common._runge_kutta_step / interp._interp_fit / interp._interp_evaluate / misc._rms_norm).
// Call sites in the reference: train_ecg_kan_fet_nn_ode.py:558-565, :1034-1041 and every
// default-method odeint (train_kanfet_node_predprey.py:252).
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
