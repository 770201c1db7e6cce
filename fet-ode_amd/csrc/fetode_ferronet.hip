// fetode_ferronet.hip — the elementwise stages of the ECG FerroElectricNet field KANFetODEFunc
// (train_ecg.py:986-1013, also compare_noise_ecg.py:1561-1588):
//     h  = h_bound * tanh(h / h_bound)            (:1002)
//     z  = tanh(fc1(h))                           (:1003-1004)
//     dh = clamp(nan_to_num(fc2(z), 0, 1e3, -1e3), -50, 50)   (:1005-1011)
// fc1 / fc2 are FerroelectricBasis layers (fetode_ferro_forward / _backward).  Forward and VJP
// follow torch's op order: mul(h_bound) . tanh . div(h_bound) and its autograd chain
// ((g * h_bound) * (1 - t^2)) / h_bound; tanh' = 1 - y^2; nan_to_num' = isfinite(x);
// clamp' = lo <= v <= hi.  Grid-stride loops; HBM-bound and tiny next to the Ferro layers.
#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kThreadsEw = 256;

__global__ __launch_bounds__(kThreadsEw) void tanh_bound_kernel(int64_t n, float hb, const float* __restrict__ x,
                                                               float* __restrict__ out, float* __restrict__ t_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float t = tanhf(x[i] / hb);
    out[i] = hb * t;
    if (t_out) t_out[i] = t;
  }
}

__global__ __launch_bounds__(kThreadsEw) void tanh_bound_bwd_kernel(int64_t n, float hb, const float* __restrict__ g,
                                                                   const float* __restrict__ t, float* __restrict__ gx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float tv = t[i];
    gx[i] = ((g[i] * hb) * (1.0f - tv * tv)) / hb;
  }
}

__global__ __launch_bounds__(kThreadsEw) void tanh_kernel(int64_t n, const float* __restrict__ x, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = tanhf(x[i]);
}

__global__ __launch_bounds__(kThreadsEw) void tanh_bwd_kernel(int64_t n, const float* __restrict__ g,
                                                             const float* __restrict__ y, float* __restrict__ gx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float yv = y[i];
    gx[i] = g[i] * (1.0f - yv * yv);
  }
}

__device__ __forceinline__ float nan_to_num(float v, float nan, float posinf, float neginf) {
  if (__builtin_isnan(v)) return nan;
  if (__builtin_isinf(v)) return v > 0.f ? posinf : neginf;
  return v;
}

__global__ __launch_bounds__(kThreadsEw) void nan_clamp_kernel(int64_t n, float nan, float posinf, float neginf, float lo,
                                                              float hi, const float* __restrict__ x,
                                                              float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = nan_to_num(x[i], nan, posinf, neginf);
    out[i] = fminf(fmaxf(v, lo), hi);
  }
}

__global__ __launch_bounds__(kThreadsEw) void nan_clamp_bwd_kernel(int64_t n, float nan, float posinf, float neginf,
                                                                  float lo, float hi, const float* __restrict__ g,
                                                                  const float* __restrict__ x, float* __restrict__ gx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = x[i];
    const float v = nan_to_num(xv, nan, posinf, neginf);
    const bool pass = __builtin_isfinite(xv) && v >= lo && v <= hi;
    gx[i] = pass ? g[i] : 0.0f;
  }
}

unsigned ew_grid(int64_t n) {
  const int64_t b = (n + kThreadsEw - 1) / kThreadsEw;
  return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

extern "C" {

int fetode_tanh_bound(int64_t n, float h_bound, const float* x, float* out, float* t_out, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!x || !out) return set_err(FETODE_EINVAL, "tanh_bound: null pointer");
  if (!(h_bound != 0.0f)) return set_err(FETODE_EINVAL, "tanh_bound: h_bound must be nonzero");
  hipLaunchKernelGGL(tanh_bound_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, h_bound, x, out,
                     t_out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_tanh_bound_backward(int64_t n, float h_bound, const float* g, const float* t, float* gx, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!g || !t || !gx) return set_err(FETODE_EINVAL, "tanh_bound backward: null pointer");
  hipLaunchKernelGGL(tanh_bound_bwd_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, h_bound, g, t,
                     gx);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_tanh(int64_t n, const float* x, float* out, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!x || !out) return set_err(FETODE_EINVAL, "tanh: null pointer");
  hipLaunchKernelGGL(tanh_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, x, out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_tanh_backward(int64_t n, const float* g, const float* y, float* gx, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!g || !y || !gx) return set_err(FETODE_EINVAL, "tanh backward: null pointer");
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, g, y, gx);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_nan_clamp(int64_t n, float nan, float posinf, float neginf, float lo, float hi, const float* x, float* out,
                     void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!x || !out) return set_err(FETODE_EINVAL, "nan_clamp: null pointer");
  hipLaunchKernelGGL(nan_clamp_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, nan, posinf, neginf,
                     lo, hi, x, out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_nan_clamp_backward(int64_t n, float nan, float posinf, float neginf, float lo, float hi, const float* g,
                              const float* x, float* gx, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!g || !x || !gx) return set_err(FETODE_EINVAL, "nan_clamp backward: null pointer");
  hipLaunchKernelGGL(nan_clamp_bwd_kernel, dim3(ew_grid(n)), dim3(kThreadsEw), 0, (hipStream_t)stream, n, nan, posinf,
                     neginf, lo, hi, g, x, gx);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"
