// fetode_ecg.hip — the ECG KAN-FET NODE vector field (BASELINE configs[2]):
// KANFeatureMixer(hysteretic LogisticBasis, Sigmoid) followed by a Linear head —
// No_MLP_KANODEFunc, train_ecg_kan_fet_nn_ode.py:483-509, LogisticBasis :54-133.
//
// Forward, one launch per evaluation: a workgroup owns kRows batch rows; its threads evaluate the
// (row, input, basis) features into LDS in the reference's op order (IEEE division, expf), then
// one thread per (row, output) forms the dot product with the head in a fixed order.  The
// hysteresis memory is the LAST row of the batch (:131-132): it is read by every workgroup and
// replaced by a second, one-block launch on the same stream, so no workgroup can see a
// half-updated state.
//
// Backward: the head's input gradient (phi-space), the basis VJP per (row, input) over its bases,
// and the parameter gradients reduced over the batch by one thread per parameter in a fixed order
// (no atomics, run-to-run identical).  branch_state is a comparison: no gradient flows through it,
// nor through the detached prev_x (:119-132).
#include <cstring>

#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kRows = 4;      // batch rows per forward workgroup
constexpr int kThreads = 256;

struct HL {  // device copy of fetode_hlogistic_t
  int in, nb;
  const float *k, *Ec, *Ps, *bias;
  float gs, bp;
};

__device__ __forceinline__ float ref_sigmoid(float z) { return 1.0f / (1.0f + expf(-z)); }

// the reference's up / down / gate for element (i, j) at input x (train_ecg_kan_fet_nn_ode.py:110-121)
struct HPoint {
  float su, sd, bs, basis;
};
__device__ __forceinline__ HPoint hpoint(const HL& L, float x, float pv, int q) {
  HPoint p;
  const float k = L.k[q], Ec = L.Ec[q], Ps = L.Ps[q];
  p.su = 1.0f / (1.0f + expf(-k * (x - Ec)));
  p.sd = 1.0f / (1.0f + expf(-k * (x + Ec)));
  const float up = Ps * p.su * 2.0f - Ps;
  const float down = Ps * p.sd * 2.0f - Ps;
  const float g = ref_sigmoid(L.gs * (x - pv));
  p.bs = g > L.bp ? 1.0f : 0.0f;
  p.basis = p.bs * up + (1.0f - p.bs) * down + L.bias[q];
  return p;
}

__global__ __launch_bounds__(kThreads) void mixer_fwd_kernel(HL L, const float* __restrict__ x, int64_t B,
                                                            const float* __restrict__ prev, int act_sigmoid,
                                                            const float* __restrict__ w, const float* __restrict__ bvec,
                                                            int n_out, float* __restrict__ phi_out,
                                                            float* __restrict__ out, float* __restrict__ branch) {
  extern __shared__ float s_phi[];  // kRows * in * nb
  const int F = L.in * L.nb;
  const int64_t b0 = (int64_t)blockIdx.x * kRows;
  const int rows = (int)(B - b0 < kRows ? B - b0 : kRows);
  for (int t = threadIdx.x; t < rows * F; t += blockDim.x) {
    const int r = t / F, q = t % F, i = q / L.nb;
    const int64_t b = b0 + r;
    const HPoint p = hpoint(L, x[b * L.in + i], prev[q], q);
    const float v = act_sigmoid ? ref_sigmoid(p.basis) : p.basis;
    s_phi[t] = v;
    if (phi_out) phi_out[b * F + q] = v;
    if (branch) branch[b * F + q] = p.bs;
  }
  if (!w) return;
  __syncthreads();
  for (int t = threadIdx.x; t < rows * n_out; t += blockDim.x) {
    const int r = t / n_out, o = t % n_out;
    const float* wr = w + (int64_t)o * F;
    const float* ph = s_phi + r * F;
    float acc = 0.f;
    for (int q = 0; q < F; ++q) acc = __builtin_fmaf(ph[q], wr[q], acc);
    out[(b0 + r) * n_out + o] = acc + (bvec ? bvec[o] : 0.f);
  }
}

// prev_x.copy_(x_exp[-1:]) (:131-132): every basis of input i remembers x[B-1, i]
__global__ void mixer_state_kernel(const float* __restrict__ x, int64_t B, int in, int nb, float* __restrict__ prev) {
  for (int q = threadIdx.x; q < in * nb; q += blockDim.x) prev[q] = x[(B - 1) * in + q / nb];
}

// g_phi[b, q] = sum_o g[b, o] w[o, q]   (the head's input gradient)
__global__ void head_gin_kernel(const float* __restrict__ g, const float* __restrict__ w, int64_t B, int n_out, int F,
                                float* __restrict__ gphi) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * F) return;
  const int64_t b = t / F;
  const int q = (int)(t % F);
  float acc = 0.f;
  for (int o = 0; o < n_out; ++o) acc = __builtin_fmaf(g[b * n_out + o], w[(int64_t)o * F + q], acc);
  gphi[t] = acc;
}

// d loss / d w[o, q] = sum_b g[b, o] phi[b, q];  d loss / d bias[o] = sum_b g[b, o]
__global__ void head_gw_kernel(const float* __restrict__ g, const float* __restrict__ phi, int64_t B, int n_out, int F,
                               float* __restrict__ gw, float* __restrict__ gb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n_out * F) {
    const int o = t / F, q = t % F;
    float acc = 0.f;
    for (int64_t b = 0; b < B; ++b) acc = __builtin_fmaf(g[b * n_out + o], phi[b * F + q], acc);
    if (gw) gw[t] = acc;
  } else if (t < n_out * F + n_out && gb) {
    const int o = t - n_out * F;
    float acc = 0.f;
    for (int64_t b = 0; b < B; ++b) acc += g[b * n_out + o];
    gb[o] = acc;
  }
}

// derivative pieces of element (b, i, j): d basis / d (x, k, Ec, Ps), gb = d loss / d basis
struct HGrad {
  float gb, dx, dk, dEc, dPs;
};
__device__ __forceinline__ HGrad hgrad(const HL& L, float x, float pv, int q, float gphi, float phi, int act_sigmoid) {
  const HPoint p = hpoint(L, x, pv, q);
  HGrad r;
  r.gb = act_sigmoid ? gphi * (phi * (1.0f - phi)) : gphi;
  const float k = L.k[q], Ec = L.Ec[q], Ps = L.Ps[q];
  const float cu = p.bs * 2.0f * Ps * p.su * (1.0f - p.su);          // d up / d z_up    (z = k (x - Ec))
  const float cd = (1.0f - p.bs) * 2.0f * Ps * p.sd * (1.0f - p.sd);  // d down / d z_down (z = k (x + Ec))
  r.dx = (cu + cd) * k;
  r.dk = cu * (x - Ec) + cd * (x + Ec);
  r.dEc = (cd - cu) * k;
  r.dPs = p.bs * (2.0f * p.su - 1.0f) + (1.0f - p.bs) * (2.0f * p.sd - 1.0f);
  return r;
}

__global__ void mixer_gx_kernel(HL L, const float* __restrict__ x, int64_t B, const float* __restrict__ prev,
                                const float* __restrict__ gphi, const float* __restrict__ phi, int act_sigmoid,
                                float* __restrict__ gx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * L.in) return;
  const int64_t b = t / L.in;
  const int i = (int)(t % L.in), F = L.in * L.nb;
  const float xv = x[t];
  float acc = 0.f;
  for (int j = 0; j < L.nb; ++j) {
    const int q = i * L.nb + j;
    const HGrad h = hgrad(L, xv, prev[q], q, gphi[b * F + q], phi[b * F + q], act_sigmoid);
    acc += h.gb * h.dx;
  }
  gx[t] = acc;
}

__global__ void mixer_gparam_kernel(HL L, const float* __restrict__ x, int64_t B, const float* __restrict__ prev,
                                    const float* __restrict__ gphi, const float* __restrict__ phi, int act_sigmoid,
                                    float* __restrict__ gk, float* __restrict__ gEc, float* __restrict__ gPs,
                                    float* __restrict__ gbias) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int F = L.in * L.nb;
  if (q >= F) return;
  const int i = q / L.nb;
  float sk = 0.f, sE = 0.f, sP = 0.f, sb = 0.f;
  for (int64_t b = 0; b < B; ++b) {
    const HGrad h = hgrad(L, x[b * L.in + i], prev[q], q, gphi[b * F + q], phi[b * F + q], act_sigmoid);
    sk = __builtin_fmaf(h.gb, h.dk, sk);
    sE = __builtin_fmaf(h.gb, h.dEc, sE);
    sP = __builtin_fmaf(h.gb, h.dPs, sP);
    sb += h.gb;
  }
  if (gk) gk[q] = sk;
  if (gEc) gEc[q] = sE;
  if (gPs) gPs[q] = sP;
  if (gbias) gbias[q] = sb;
}

int check_layer(const fetode_hlogistic_t* l) {
  if (!l || l->in_dim <= 0 || l->num_basis <= 0) return set_err(FETODE_EINVAL, "hlogistic: bad dims");
  if (!l->k || !l->Ec || !l->Ps || !l->bias) return set_err(FETODE_EINVAL, "hlogistic: null parameter");
  return FETODE_OK;
}

HL to_dev(const fetode_hlogistic_t* l) {
  HL L;
  L.in = l->in_dim;
  L.nb = l->num_basis;
  L.k = l->k;
  L.Ec = l->Ec;
  L.Ps = l->Ps;
  L.bias = l->bias;
  // gate_slope * dx with gate_slope a Python float: torch scales an fp32 tensor by it in fp32
  L.gs = (float)l->gate_slope;
  L.bp = (float)l->breaking_point;
  return L;
}

}  // namespace

extern "C" {

int fetode_hlogistic_mixer_forward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                   int32_t act_sigmoid, const float* w, const float* bias, int32_t n_out,
                                   float* phi, float* out, float* branch, float* prev_out, void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !prev || (w && (!out || n_out <= 0)) || (!w && !phi))
    return set_err(FETODE_EINVAL, "hlogistic mixer: null pointer");
  const HL L = to_dev(layer);
  const int F = L.in * L.nb;
  const size_t lds = sizeof(float) * kRows * F;
  if (lds > 64 * 1024) return set_err(FETODE_EINVAL, "hlogistic mixer: in*num_basis=%d too large", F);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mixer_fwd_kernel, dim3(nblk(B, kRows)), dim3(kThreads), lds, s, L, x, B, prev, act_sigmoid, w,
                     bias, n_out, phi, out, branch);
  LAUNCH_CHECK();
  if (prev_out) {
    hipLaunchKernelGGL(mixer_state_kernel, dim3(1), dim3(256), 0, s, x, B, L.in, L.nb, prev_out);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int64_t fetode_hlogistic_mixer_backward_workspace(const fetode_hlogistic_t* layer, int64_t B) {
  if (check_layer(layer) || B <= 0) return -1;
  return (int64_t)sizeof(float) * B * layer->in_dim * layer->num_basis;
}

int fetode_hlogistic_mixer_backward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                    int32_t act_sigmoid, const float* phi, const float* w, int32_t n_out,
                                    const float* g, float* gx, float* gw, float* gbias_head, float* gk, float* gEc,
                                    float* gPs, float* gbias, void* workspace, void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !prev || !phi || !g || (w && (n_out <= 0 || !workspace)))
    return set_err(FETODE_EINVAL, "hlogistic mixer backward: null pointer");
  const HL L = to_dev(layer);
  const int F = L.in * L.nb;
  hipStream_t s = (hipStream_t)stream;
  const float* gphi = g;  // without a head, g is already d loss / d phi
  if (w) {
    float* gp = (float*)workspace;
    hipLaunchKernelGGL(head_gin_kernel, dim3(nblk(B * F, 256)), dim3(256), 0, s, g, w, B, n_out, F, gp);
    LAUNCH_CHECK();
    if (gw || gbias_head) {
      hipLaunchKernelGGL(head_gw_kernel, dim3(nblk((int64_t)n_out * F + n_out, 256)), dim3(256), 0, s, g, phi, B,
                         n_out, F, gw, gbias_head);
      LAUNCH_CHECK();
    }
    gphi = gp;
  }
  if (gx) {
    hipLaunchKernelGGL(mixer_gx_kernel, dim3(nblk(B * L.in, 256)), dim3(256), 0, s, L, x, B, prev, gphi, phi,
                       act_sigmoid, gx);
    LAUNCH_CHECK();
  }
  if (gk || gEc || gPs || gbias) {
    hipLaunchKernelGGL(mixer_gparam_kernel, dim3(nblk(F, 64)), dim3(64), 0, s, L, x, B, prev, gphi, phi,
                       act_sigmoid, gk, gEc, gPs, gbias);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

}  // extern "C"
