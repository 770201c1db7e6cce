// fetode_generic.hip — standalone module kernels for any widths (the per-stage / drop-in path):
//   bsplines_kernel       efficientkan.KANLinear.b_splines (bitwise equal to the reference)
//   kanlinear_fwd_kernel  efficientkan.KANLinear.forward
//   ferro_fwd_kernel      ferro_class.FerroelectricBasis.forward (general branch_sign)
//   rk_combine_kernel     torchdiffeq stage combines (exact op order)
#include "fetode_common.h"

using namespace fetode;

// ---------------------------------------------------------------------------------------------
// generic kernels (any widths)
// ---------------------------------------------------------------------------------------------
template <int SO>
__global__ void bsplines_kernel(const float* __restrict__ x, const float* __restrict__ grid, int64_t B,
                                int in, int NG, float* __restrict__ bases) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * in) return;
  const int i = t % in;
  const int NS = NG - 1 - SO;
  float* o = bases + t * NS;
  bspline_local_div<SO>(x[t], NG, grid + (int64_t)i * NG, [&](int c, float v) { o[c] = v; });
}

// KANLinear.forward: thread per (b, o); features recomputed per o (generic path only).
template <int SO>
__global__ void kanlinear_fwd_kernel(fetode_kanlinear_t kl, const float* __restrict__ x, int64_t B,
                                     float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, outf = kl.out_features, NB = kl.num_logistic;
  const int NG = kl.grid_size + 2 * SO + 1, NS = kl.grid_size + SO;
  if (t >= B * outf) return;
  const int64_t b = t / outf;
  const int o = t % outf;
  const float lsc = (NB > 0 && kl.logistic_scaler) ? kl.logistic_scaler[o] : 1.0f;
  float base = 0.f, spl = 0.f, lgs = 0.f;
  for (int i = 0; i < in; ++i) {
    const float xi = x[b * in + i];
    // base branch: SiLU(x) . base_weight (efficientkan.py:166)
    base += (xi / (1.0f + expf(-xi))) * kl.base_weight[o * in + i];
    const float sc = kl.spline_scaler ? kl.spline_scaler[o * in + i] : 1.0f;
    const float* sw = kl.spline_weight + ((int64_t)o * in + i) * NS;
    bspline_local_div<SO>(xi, NG, kl.grid + (int64_t)i * NG,
                          [&](int c, float v) { spl += v * (sw[c] * sc); });
    for (int j = 0; j < NB; ++j) {
      const float a = kl.logistic_a[i * NB + j], bb = kl.logistic_b[i * NB + j];
      const float phi = 2.0f / (1.0f + expf(-a * (xi - bb)));  // efficientkan.py:24
      const float w = (kl.logistic_weight[(int64_t)o * in * NB + i * NB + j] * kl.scale_logistic) * lsc;
      lgs += phi * w;
    }
  }
  float r = base + spl;
  if (NB > 0) r = r + lgs;
  out[t] = r;
}

// FerroelectricBasis.forward, general branch_sign, thread per (b, o); reference formula verbatim.
__global__ void ferro_fwd_kernel(fetode_ferro_t fl, const float* __restrict__ x, int64_t B,
                                 const float* __restrict__ prev, int reinit, int accumulate,
                                 float* __restrict__ out, float* __restrict__ basis_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = fl.in_dim, outd = fl.out_dim, K = fl.num_basis;
  if (t >= B * outd) return;
  const int64_t b = t / outd;
  const int o = t % outd;
  const float gs = (float)fl.gate_slope, al = (float)fl.alpha, oma = (float)(1.0 - fl.alpha);
  // two-level sum (K bases of one input, then inputs): at production widths (64 x 12, 128 x 12
  // terms) one running fp32 sum loses ~5x the accuracy of the reference's reduction
  float acc = 0.f;
  for (int i = 0; i < in; ++i) {
    float acc_i = 0.f;
    const float xv = x[b * in + i];
    const float pv = reinit ? xv : prev[b * in + i];
    const float dx = xv - pv;
    const float up = 1.0f / (1.0f + expf(-(gs * dx)));
    for (int k = 0; k < K; ++k) {
      const int e = (i * outd + o) * K + k;
      const float Ec = fl.Ec[e];
      const float bs = fl.branch_sign ? fl.branch_sign[b * fl.branch_sign_bstride + e] : 1.0f;
      const float cp = 1.0f / (1.0f + expf(-(gs * (xv - Ec))));
      const float cn = 1.0f / (1.0f + expf(-(gs * (-xv - Ec))));
      const float su = up * cp, sl = (1.0f - up) * cn;
      const float tgt = (su * 1.0f + sl * (-1.0f)) + ((1.0f - su) - sl) * bs;
      const float mom = al * bs + oma * tgt;
      const float sh = xv + Ec * mom;
      const float bv = fl.Ps[e] * tanhf(fl.k[e] * sh) + fl.bias[e];
      if (basis_out) basis_out[((b * in + i) * outd + o) * K + k] = bv;
      acc_i += bv * fl.coef[e];
    }
    acc += acc_i;
  }
  out[t] = accumulate ? out[t] + acc : acc;
}

__global__ void rk_combine_kernel(int method, int stage, const float* __restrict__ y,
                                  const float* __restrict__ k1, const float* __restrict__ k2,
                                  const float* __restrict__ k3, const float* __restrict__ k4, float dt,
                                  float* __restrict__ out, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float third = 1.0f / 3.0f;
  const float yv = y[t];
  float r;
  if (method == FETODE_RK4) {
    if (stage == 1) r = yv + (dt * k1[t]) * third;
    else if (stage == 2) r = yv + dt * (k2[t] - k1[t] * third);
    else if (stage == 3) r = yv + dt * ((k1[t] - k2[t]) + k3[t]);
    else r = yv + (((k1[t] + 3.0f * (k2[t] + k3[t])) + k4[t]) * dt) * 0.125f;
  } else if (method == FETODE_RK4_CLASSIC && stage == 4) {
    // train_kan_fet_ett.py:76: z + (h/6) * (k1 + 2*k2 + 2*k3 + k4), dt = fp32(h/6)
    r = yv + dt * (((k1[t] + 2.0f * k2[t]) + 2.0f * k3[t]) + k4[t]);
  } else {
    r = yv + dt * k1[t];
  }
  out[t] = r;
}

__global__ void axpby_kernel(int64_t n, float a, const float* __restrict__ x, float b, const float* __restrict__ y,
                             float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = y ? a * x[t] + b * y[t] : a * x[t];
}

extern "C" {

int fetode_axpby(int64_t n, float a, const float* x, float b, const float* y, float* out, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!x || !out) return set_err(FETODE_EINVAL, "null pointer");
  hipLaunchKernelGGL(axpby_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, n, a, x, b, y, out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_kanlinear_forward(const fetode_kanlinear_t* kl, const float* x, int64_t B, float* out,
                             void* stream) {
  fetode_field_t f{1, kl, nullptr};
  int rc = validate_field(&f);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !out) return set_err(FETODE_EINVAL, "null pointer");
  const int64_t n = B * kl->out_features;
  switch (kl->spline_order) {
    case 1: hipLaunchKernelGGL(kanlinear_fwd_kernel<1>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, *kl, x, B, out); break;
    case 2: hipLaunchKernelGGL(kanlinear_fwd_kernel<2>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, *kl, x, B, out); break;
    default: hipLaunchKernelGGL(kanlinear_fwd_kernel<3>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, *kl, x, B, out); break;
  }
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_kanlinear_bsplines(const fetode_kanlinear_t* kl, const float* x, int64_t B, float* bases,
                              void* stream) {
  fetode_field_t f{1, kl, nullptr};
  int rc = validate_field(&f);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !bases) return set_err(FETODE_EINVAL, "null pointer");
  const int NG = kl->grid_size + 2 * kl->spline_order + 1;
  const int64_t n = B * kl->in_features;
  switch (kl->spline_order) {
    case 1: hipLaunchKernelGGL(bsplines_kernel<1>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, x, kl->grid, B, kl->in_features, NG, bases); break;
    case 2: hipLaunchKernelGGL(bsplines_kernel<2>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, x, kl->grid, B, kl->in_features, NG, bases); break;
    default: hipLaunchKernelGGL(bsplines_kernel<3>, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, x, kl->grid, B, kl->in_features, NG, bases); break;
  }
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_ferro_forward(const fetode_ferro_t* fl, const float* x, int64_t B, const float* prev,
                         int32_t reinit, int32_t accumulate, float* out, float* basis, float* prev_out,
                         void* stream) {
  if (!fl || fl->in_dim <= 0 || fl->out_dim <= 0 || fl->num_basis <= 0)
    return set_err(FETODE_EINVAL, "ferro: bad dims");
  if (!fl->k || !fl->Ec || !fl->Ps || !fl->bias || !fl->coef) return set_err(FETODE_EINVAL, "ferro: null param");
  if (B <= 0) return FETODE_OK;
  if (!x || !out || (!reinit && !prev)) return set_err(FETODE_EINVAL, "null pointer");
  const int64_t n = B * fl->out_dim;
  hipLaunchKernelGGL(ferro_fwd_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, *fl, x, B,
                     prev, reinit, accumulate, out, basis);
  LAUNCH_CHECK();
  if (prev_out)
    HIP_CHECK_RET(hipMemcpyAsync(prev_out, x, sizeof(float) * B * fl->in_dim, hipMemcpyDeviceToDevice,
                                 (hipStream_t)stream));
  return FETODE_OK;
}

int fetode_rk_combine(int32_t method, int32_t stage, const float* y, const float* k1, const float* k2,
                      const float* k3, const float* k4, float dt, float* out, int64_t n, void* stream) {
  if (n <= 0) return FETODE_OK;
  if (!y || !k1 || !out) return set_err(FETODE_EINVAL, "null pointer");
  if ((method == FETODE_RK4 && ((stage >= 2 && !k2) || (stage >= 3 && !k3) || (stage >= 4 && !k4))) ||
      (method == FETODE_RK4_CLASSIC && stage == 4 && (!k2 || !k3 || !k4)))
    return set_err(FETODE_EINVAL, "rk4 stage %d: missing k", stage);
  hipLaunchKernelGGL(rk_combine_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, method,
                     stage, y, k1, k2, k3, k4, dt, out, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"
