// fetode_generic.hip — standalone module kernels for any widths (the per-stage / drop-in path):
//   bsplines_kernel       efficientkan.KANLinear.b_splines (bitwise equal to the reference)
//   kanlinear_fwd_kernel  efficientkan.KANLinear.forward
//   ferro_fwd_kernel      ferro_class.FerroelectricBasis.forward (general branch_sign)
//   rk_combine_kernel     torchdiffeq stage combines (exact op order)
#include "fetode_common.h"

#include <cstdlib>

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

// KANLinear.forward for wide layers: a wave owns 64 rows (lane -> b) x kOB outputs, so the features
// of (b, i) — SiLU, the cubic B-spline bases, the logistic bases — are computed once per wave and
// reused for kOB outputs (the thread-per-(b, o) kernel recomputes them for every o), and every
// weight read is wave-uniform (scalar loads).  Per output the accumulation order is the thread
// kernel's (base, spline over c ascending incl. the zero bases, logistic over j), so the two agree
// bit for bit.
constexpr int kNBMax = 16;
template <int SO, int G, int kOB>
__global__ __launch_bounds__(256) void kanlinear_fwd_wave_kernel(fetode_kanlinear_t kl, const float* __restrict__ x,
                                                                int64_t B, float* __restrict__ out) {
  constexpr int NG = G + 2 * SO + 1, NS = G + SO;
  const int in = kl.in_features, outf = kl.out_features, NB = kl.num_logistic;
  const int lane = threadIdx.x & 63;
  const int o0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * kOB;
  if (o0 >= outf) return;
  const int64_t b = (int64_t)blockIdx.x * 64 + lane;
  const bool live = b < B;
  const int no = min(kOB, outf - o0);
  float base[kOB], spl[kOB], lgs[kOB], lsc[kOB];
#pragma unroll
  for (int q = 0; q < kOB; ++q) {
    base[q] = spl[q] = lgs[q] = 0.f;
    lsc[q] = (q < no && NB > 0 && kl.logistic_scaler) ? kl.logistic_scaler[o0 + q] : 1.0f;
  }
  for (int i = 0; i < in; ++i) {
    const float xi = live ? x[b * in + i] : 0.f;
    const float silu = xi / (1.0f + expf(-xi));
    float S[NS];
    bspline_local_div<SO>(xi, NG, kl.grid + (int64_t)i * NG, [&](int c, float v) {
#pragma unroll
      for (int cc = 0; cc < NS; ++cc)   // register select (no dynamically indexed private array)
        if (cc == c) S[cc] = v;
    });
    float phi[kNBMax];
#pragma unroll
    for (int j = 0; j < kNBMax; ++j) {
      if (j < NB) {
        const float a = kl.logistic_a[i * NB + j], bb = kl.logistic_b[i * NB + j];
        phi[j] = 2.0f / (1.0f + expf(-a * (xi - bb)));
      }
    }
#pragma unroll
    for (int q = 0; q < kOB; ++q) {
      if (q >= no) break;
      const int o = o0 + q;
      base[q] += silu * kl.base_weight[o * in + i];
      const float sc = kl.spline_scaler ? kl.spline_scaler[o * in + i] : 1.0f;
      const float* sw = kl.spline_weight + ((int64_t)o * in + i) * NS;
#pragma unroll
      for (int c = 0; c < NS; ++c) spl[q] += S[c] * (sw[c] * sc);
      const float* lw = kl.logistic_weight + (int64_t)o * in * NB + i * NB;
#pragma unroll
      for (int j = 0; j < kNBMax; ++j)
        if (j < NB) lgs[q] += phi[j] * ((lw[j] * kl.scale_logistic) * lsc[q]);
    }
  }
  if (!live) return;
#pragma unroll
  for (int q = 0; q < kOB; ++q) {
    if (q >= no) break;
    float r = base[q] + spl[q];
    if (NB > 0) r = r + lgs[q];
    out[b * outf + o0 + q] = r;
  }
}

// FerroelectricBasis.forward for wide layers with the constant branch_sign (the reference never
// updates it, ferro_class.py:377-378) and no activations output: a wave owns 64 rows (lane -> b)
// and one output o, so every parameter read is wave-uniform.  Inputs are walked in chunks of kFI:
// per chunk the block stages x, the hysteresis gate and e^{-gs x}, e^{gs x} of its (64 rows x kFI)
// tile in LDS ([i][row], conflict-free), and each wave stages P = e^{gs Ec} of its own output.
// The two coercive sigmoids then need no exponential per basis element:
//     sigma(gs (x - Ec)) = 1 / (1 + e^{-gs x} P),   sigma(gs (-x - Ec)) = 1 / (1 + e^{gs x} P)
// (inputs with |gs x| > 80 or parameters with |gs Ec| > 80 take the direct form, so no 0 * inf and
// no overflowed factor can appear); tanh z =
// 1 - 2 / (1 + e^{2z}) with v_exp_f32 / v_rcp_f32.  The gate sigmoid(gs (x - prev_x)) keeps the
// precise exp (it carries the fp32 conditioning of the hysteresis).  Two-level sum as the thread
// kernel (K bases of one input, then inputs).
constexpr int kFI = 32, kFKMax = 16;
template <int KT>  // KT > 0: the basis count as a compile-time constant (unrolled, batched scalar loads)
__global__ __launch_bounds__(256) void ferro_fwd_wide_kernel(fetode_ferro_t fl, const float* __restrict__ x, int64_t B,
                                                            const float* __restrict__ prev, int reinit,
                                                            int accumulate, float* __restrict__ out) {
  __shared__ float xs[kFI * 64], ups[kFI * 64], e1s[kFI * 64], e2s[kFI * 64];
  __shared__ float ps[4][kFI * kFKMax];
  const int in = fl.in_dim, outd = fl.out_dim, K = KT > 0 ? KT : fl.num_basis;
  const float gs = (float)fl.gate_slope, al = (float)fl.alpha, oma = (float)(1.0 - fl.alpha);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = blockIdx.y * 4 + w;
  const bool ovalid = o < outd;
  const int64_t b0 = (int64_t)blockIdx.x * 64;
  const int64_t b = b0 + lane;
  float acc = 0.f;
  for (int i0 = 0; i0 < in; i0 += kFI) {
    const int ni = min(kFI, in - i0);
    __syncthreads();  // the previous chunk is consumed
    for (int idx = threadIdx.x; idx < 64 * ni; idx += 256) {
      const int r = idx / ni, ii = idx - r * ni;
      const int64_t bb = b0 + r;
      float xv = 0.f, up = 0.f;
      if (bb < B) {
        xv = x[bb * in + i0 + ii];
        const float pv = reinit ? xv : prev[bb * in + i0 + ii];
        up = 1.0f / (1.0f + expf(-(gs * (xv - pv))));
      }
      const float gx = gs * xv;
      xs[ii * 64 + r] = xv;
      ups[ii * 64 + r] = up;
      e1s[ii * 64 + r] = __expf(-gx);
      e2s[ii * 64 + r] = __expf(gx);
    }
    bool big_ec = false;  // some |gs Ec| > 80 in this chunk of output o: P would over/underflow
    if (ovalid)
      for (int idx = lane; idx < ni * K; idx += 64) {
        const int ii = idx / K, k = idx - ii * K;
        const float gec = gs * fl.Ec[((i0 + ii) * outd + o) * K + k];
        big_ec |= fabsf(gec) > 80.0f;
        ps[w][idx] = __expf(gec);
      }
    big_ec = __any(big_ec);
    __syncthreads();
    if (!ovalid) continue;
    for (int ii = 0; ii < ni; ++ii) {
      const float xv = xs[ii * 64 + lane], up = ups[ii * 64 + lane];
      const float e1 = e1s[ii * 64 + lane], e2 = e2s[ii * 64 + lane];
      // the product form needs both factors finite and non-zero: |gs x| <= 80 and |gs Ec| <= 80
      // (then a product that overflows / underflows only does so where the sigmoid is saturated)
      const bool direct = big_ec || __any(fabsf(gs * xv) > 80.0f);   // wave-uniform: no divergent paths
      const float omu = 1.0f - up;
      const int e0 = ((i0 + ii) * outd + o) * K;
      const float* P = &ps[w][ii * K];
      float acc_i = 0.f;
#pragma unroll
      for (int k = 0; k < (KT > 0 ? KT : kFKMax); ++k) {
        if (KT == 0 && k >= K) break;
        const int e = e0 + k;
        const float Ec = fl.Ec[e];
        float cp, cn;
        if (direct) {
          cp = __builtin_amdgcn_rcpf(1.0f + __expf(-(gs * (xv - Ec))));
          cn = __builtin_amdgcn_rcpf(1.0f + __expf(-(gs * (-xv - Ec))));
        } else {
          cp = __builtin_amdgcn_rcpf(1.0f + e1 * P[k]);
          cn = __builtin_amdgcn_rcpf(1.0f + e2 * P[k]);
        }
        const float su = up * cp, sl = omu * cn;
        const float tgt = (su - sl) + ((1.0f - su) - sl);       // branch_sign = 1
        const float mom = al + oma * tgt;
        const float sh = xv + Ec * mom;
        const float th = 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * (fl.k[e] * sh)));
        const float bv = fl.Ps[e] * th + fl.bias[e];
        acc_i += bv * fl.coef[e];
      }
      acc += acc_i;
    }
  }
  if (ovalid && b < B) {
    const int64_t t = b * outd + o;
    out[t] = accumulate ? out[t] + acc : acc;
  }
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
  if (kl->out_features >= 16 && kl->num_logistic <= kNBMax && kl->grid_size == 5 && kl->spline_order == 3) {
    // outputs per wave: the largest of 8/4/2/1 that still gives >= 1024 workgroups (4 per CU); fewer
    // outputs per wave recompute the features more often but fill the chip at small batches
    static const int64_t min_blocks = [] {
      const char* e = getenv("FETODE_WAVE_MIN_BLOCKS");  // tuning knob (default 1024, measured r01_s5)
      return e ? (int64_t)atoll(e) : (int64_t)1024;
    }();
    const int64_t rb = (B + 63) / 64;
    int ob = 8;
    while (ob > 1 && rb * ((kl->out_features + 4 * ob - 1) / (4 * ob)) < min_blocks) ob >>= 1;
    const dim3 grid((unsigned)rb, (unsigned)((kl->out_features + 4 * ob - 1) / (4 * ob)));
    const hipStream_t st = (hipStream_t)stream;
    switch (ob) {
      case 8: hipLaunchKernelGGL((kanlinear_fwd_wave_kernel<3, 5, 8>), grid, dim3(256), 0, st, *kl, x, B, out); break;
      case 4: hipLaunchKernelGGL((kanlinear_fwd_wave_kernel<3, 5, 4>), grid, dim3(256), 0, st, *kl, x, B, out); break;
      case 2: hipLaunchKernelGGL((kanlinear_fwd_wave_kernel<3, 5, 2>), grid, dim3(256), 0, st, *kl, x, B, out); break;
      default: hipLaunchKernelGGL((kanlinear_fwd_wave_kernel<3, 5, 1>), grid, dim3(256), 0, st, *kl, x, B, out); break;
    }
    LAUNCH_CHECK();
    return FETODE_OK;
  }
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
  if (fl->in_dim >= 32 && fl->num_basis <= kFKMax && !fl->branch_sign && !basis) {
    const dim3 grid((unsigned)((B + 63) / 64), (unsigned)((fl->out_dim + 3) / 4));
    const hipStream_t st = (hipStream_t)stream;
    if (fl->num_basis == 10)
      hipLaunchKernelGGL(ferro_fwd_wide_kernel<10>, grid, dim3(256), 0, st, *fl, x, B, prev, reinit, accumulate, out);
    else if (fl->num_basis == 12)
      hipLaunchKernelGGL(ferro_fwd_wide_kernel<12>, grid, dim3(256), 0, st, *fl, x, B, prev, reinit, accumulate, out);
    else
      hipLaunchKernelGGL(ferro_fwd_wide_kernel<0>, grid, dim3(256), 0, st, *fl, x, B, prev, reinit, accumulate, out);
  } else {
    hipLaunchKernelGGL(ferro_fwd_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, *fl, x, B,
                       prev, reinit, accumulate, out, basis);
  }
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
