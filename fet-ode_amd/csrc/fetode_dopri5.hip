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

int fetode_scaled_rms(const float* a, const float* sub, const float* y0, const float* y1, double rtol, double atol,
                      int64_t n, float* out, void* stream) {
  if (n <= 0 || !a || !y0 || !out) return set_err(FETODE_EINVAL, "scaled_rms: bad arguments");
  hipLaunchKernelGGL(scaled_rms_kernel<true>, dim3(1), dim3(1024), 0, (hipStream_t)stream, a, sub, y0, y1,
                     (float)rtol, (float)atol, n, (void*)out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_scaled_sumsq(const float* a, const float* sub, const float* y0, const float* y1, double rtol, double atol,
                        int64_t n, double* out, void* stream) {
  if (n < 0 || !out || (n > 0 && (!a || !y0))) return set_err(FETODE_EINVAL, "scaled_sumsq: bad arguments");
  if (n == 0) return hipMemsetAsync(out, 0, 2 * sizeof(double), (hipStream_t)stream) == hipSuccess
                         ? FETODE_OK
                         : set_err(FETODE_EHIP, "scaled_sumsq: memset failed");
  hipLaunchKernelGGL(scaled_rms_kernel<false>, dim3(1), dim3(1024), 0, (hipStream_t)stream, a, sub, y0, y1,
                     (float)rtol, (float)atol, n, (void*)out);
  LAUNCH_CHECK();
  return FETODE_OK;
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
