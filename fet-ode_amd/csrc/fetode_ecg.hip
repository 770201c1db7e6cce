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

// =============================================================================================
// Device-resident dopri5 for the ECG field: the whole torchdiffeq solve —
// f0, _select_initial_step, 6 evaluations per attempt (FSAL), the global RMS error norm,
// accept/reject, _optimal_step_size, _interp_fit / _interp_evaluate — in ONE cooperative launch,
// with the same fp32/fp64 arithmetic as the host-driven path (dopri5.py + the kernels above).
//
// A workgroup owns kDR batch rows and, as a SHADOW row, the batch's last row: the hysteresis
// memory every evaluation reads is the last row's previous input (:131-132), so each workgroup
// evaluates that row itself and no evaluation needs data from another workgroup.  Only the
// error norms (one per attempt, three in the initial-step selection) are global: per-workgroup
// fp64 partial sums, a grid barrier, and the same fixed-order sum in every workgroup — so every
// workgroup takes the same accept/reject decisions and the same dt sequence.
// =============================================================================================
namespace {

constexpr int kDR = 3;                 // real rows per workgroup (+1 shadow)
constexpr int kDT = 64 * (kDR + 1);    // one thread per (row, state dim): state dim <= 64

struct DopriTab {
  float beta[6][6];  // torchdiffeq Dopri5 tableau rounded to fp32 (tableau.to(y0.dtype))
  float cerr[7];
  float cmid[7];
};

struct EcgDopriArgs {
  HL L;
  const float* wT;  // (F, D) head weight, transposed
  const float* bh;  // (D) head bias, nullable
  int D, F;
  const float* prev0;  // (F) prev_x before the solve
  const float* y0;     // (B, D)
  int64_t B;
  const double* t;  // (T) strictly increasing
  int T;
  float rtol, atol;
  double first_step;  // > 0: options["first_step"]; else _select_initial_step
  double safety, ifactor, dfactor, min_step, max_step;
  int max_steps;
  DopriTab tab;
  float* sol;         // (T, B, D)
  float* prev_out;    // (F)
  float* branch_out;  // (B, F) nullable: branch_state of the last evaluation
  double* part;       // (2, gridDim.x, 2) double-buffered partial sums
  unsigned* bar;      // 2 words, zeroed: arrival count, generation
  int* stats;         // [nfev, attempts, status]
  double* att;        // (max_att, 4): t0, dt, error ratio, accepted
  int max_att;
};

__device__ void grid_barrier(unsigned* bar, unsigned nblk) {
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* count = bar;
    unsigned* gen = bar + 1;
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblk - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float fast_sigmoid(float z) { return rcp(1.0f + ex2(-z * FETODE_LOG2E)); }

// misc._rms_norm over the WHOLE batch of sum_v (per-thread fp64 squares, real elements only):
// workgroup tree -> partial slot -> grid barrier -> the same fixed-order sum in every workgroup
struct GlobalNorm {
  double* red;  // LDS, kDT doubles
  int* bad_lds;
  double* tot;  // LDS, 2 doubles
  __device__ void run(const EcgDopriArgs& a, double v, int bad, int phase, int nvals, double* out_sum, int* out_bad) {
    const int tid = threadIdx.x;
    red[tid] = v;
    if (tid == 0) *bad_lds = 0;
    __syncthreads();
    if (bad) atomicOr(bad_lds, 1);
    for (int w = kDT / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    double* slot = a.part + ((int64_t)(phase & 1) * gridDim.x + blockIdx.x) * 2;
    if (tid == 0) {
      __hip_atomic_store(&slot[0], red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&slot[1], (double)*bad_lds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_barrier(a.bar, gridDim.x);
    double s = 0.0, fb = 0.0;
    for (int g = tid; g < (int)gridDim.x; g += kDT) {
      const double* o = a.part + ((int64_t)(phase & 1) * gridDim.x + g) * 2;
      s += __hip_atomic_load(&o[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      fb += __hip_atomic_load(&o[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    red[tid] = s;
    __syncthreads();
    for (int w = kDT / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    if (tid == 0) tot[0] = red[0];
    red[tid] = fb;
    __syncthreads();
    for (int w = kDT / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    if (tid == 0) tot[1] = red[0];
    __syncthreads();
    *out_sum = tot[0];
    *out_bad = tot[1] != 0.0;
    (void)nvals;
  }
};

__global__ __launch_bounds__(kDT) void ecg_dopri5_kernel(EcgDopriArgs a) {
  extern __shared__ float s_dyn[];  // phi (kDR+1) * F | prev F | prevold F
  __shared__ float xs[kDR + 1][64];
  __shared__ double red[kDT];
  __shared__ double tot[2];
  __shared__ int bad_lds;
  const int tid = threadIdx.x, r = tid / 64, d = tid % 64;
  const int D = a.D, F = a.F, nb = a.L.nb;
  float* phi = s_dyn;
  float* prev = phi + (kDR + 1) * F;
  float* prevold = prev + F;
  const bool dval = d < D;
  int64_t b = r < kDR ? (int64_t)blockIdx.x * kDR + r : a.B - 1;  // row kDR: the shadow last row
  const bool real = r < kDR && b < a.B && dval;
  if (b >= a.B) b = a.B - 1;  // padding rows mirror the last row; never stored or counted
  const int64_t BD = a.B * D;
  const double n_el = (double)BD;
  GlobalNorm gn{red, &bad_lds, tot};
  int phase = 0, nfev = 0, status = 0, n_att = 0;

  for (int q = tid; q < F; q += kDT) prev[q] = a.prev0[q];
  __syncthreads();

  // one field evaluation of this thread's element; all threads of the workgroup take part
  auto eval = [&](float xv) -> float {
    if (dval) xs[r][d] = xv;
    __syncthreads();
    for (int idx = tid; idx < (kDR + 1) * F; idx += kDT) {
      const int r2 = idx / F, q = idx - r2 * F, i = q / nb;
      const float x = xs[r2][i];
      const float kq = a.L.k[q], Ec = a.L.Ec[q], Ps = a.L.Ps[q];
      const float su = fast_sigmoid(kq * (x - Ec)), sd = fast_sigmoid(kq * (x + Ec));
      const float up = Ps * su * 2.0f - Ps, down = Ps * sd * 2.0f - Ps;
      const float bs = ref_sigmoid(a.L.gs * (x - prev[q])) > a.L.bp ? 1.0f : 0.0f;
      phi[idx] = fast_sigmoid(bs * up + (1.0f - bs) * down + a.L.bias[q]);
    }
    __syncthreads();
    for (int q = tid; q < F; q += kDT) {  // :131-132, the shadow row's input
      prevold[q] = prev[q];
      prev[q] = xs[kDR][q / nb];
    }
    float acc = 0.f;
    if (dval) {
      const float* ph = phi + r * F;
      for (int q = 0; q < F; ++q) acc = __builtin_fmaf(ph[q], a.wT[(int64_t)q * D + d], acc);
      acc += a.bh ? a.bh[d] : 0.f;
    }
    __syncthreads();
    ++nfev;
    return acc;
  };

  float y = dval ? a.y0[b * D + d] : 0.f;
  if (real) a.sol[b * D + d] = y;
  float f0 = eval(y);
  double dt;
  if (a.first_step > 0.0) {
    dt = a.first_step;
  } else {  // misc._select_initial_step in fp32 (dopri5.py select_initial_step)
    const float scale = a.atol + a.rtol * fabsf(y);
    double s;
    int bad;
    const float q0 = y / scale, q1 = f0 / scale;
    gn.run(a, real ? (double)q0 * q0 : 0.0, 0, phase++, 0, &s, &bad);
    const float d0 = fabsf(sqrtf((float)(s / n_el)));
    gn.run(a, real ? (double)q1 * q1 : 0.0, 0, phase++, 0, &s, &bad);
    const float d1 = fabsf(sqrtf((float)(s / n_el)));
    float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
    h0 = fabsf(h0);
    const float f1 = eval(y + f0 * h0);
    const float q2 = (f1 - f0) / scale;
    gn.run(a, real ? (double)q2 * q2 : 0.0, 0, phase++, 0, &s, &bad);
    const float d2 = fabsf(sqrtf((float)(s / n_el)) / h0);
    float h1;
    if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
    else h1 = powf(0.01f / fmaxf(d1, d2), 0.2f);
    dt = (double)fminf(100.0f * h0, fabsf(h1));
  }

  float co[5] = {y, 0.f, 0.f, 0.f, 0.f};
  double t0s = a.t[0], t1s = a.t[0];
  for (int i = 1; i < a.T && status == 0; ++i) {
    const double next_t = a.t[i];
    int n_steps = 0;
    while (next_t > t1s) {
      if (n_steps >= a.max_steps) { status = 3; break; }
      const double t0 = t1s;
      if (!(t0 + dt > t0)) { status = 2; break; }
      const float dt32 = (float)dt;
      const double t1 = t0 + dt;
      float k[7];
      k[0] = f0;
      float yi = y;
#pragma unroll
      for (int s = 0; s < 6; ++s) {  // rk_common._runge_kutta_step via fetode_lincomb's op order
        float acc = k[0] * (a.tab.beta[s][0] * dt32);
#pragma unroll
        for (int j = 1; j <= s; ++j) acc = acc + k[j] * (a.tab.beta[s][j] * dt32);
        yi = y + acc;
        k[s + 1] = eval(yi);
      }
      const float y1 = yi;
      float err = k[0] * (a.tab.cerr[0] * dt32);
#pragma unroll
      for (int j = 1; j < 7; ++j) err = err + k[j] * (a.tab.cerr[j] * dt32);
      const float tol = a.atol + a.rtol * fmaxf(fabsf(y), fabsf(y1));
      const float qe = err / tol;
      double s;
      int bad;
      gn.run(a, real ? (double)qe * qe : 0.0, real && !__builtin_isfinite(y), phase++, 0, &s, &bad);
      if (bad) { status = 1; break; }
      const float ratio = sqrtf((float)(s / n_el));
      const bool accept = ratio <= 1.0f;
      if (blockIdx.x == 0 && tid == 0 && n_att < a.max_att) {
        double* o = a.att + (int64_t)n_att * 4;
        o[0] = t0;
        o[1] = dt;
        o[2] = (double)ratio;
        o[3] = accept ? 1.0 : 0.0;
      }
      ++n_att;
      if (accept) {  // interp._interp_fit (fetode_interp_fit's op order)
        float acc = k[0] * (a.tab.cmid[0] * dt32);
#pragma unroll
        for (int j = 1; j < 7; ++j) acc = acc + k[j] * (a.tab.cmid[j] * dt32);
        const float ym = y + acc, fa = k[0], fb = k[6];
        co[4] = ((2.0f * dt32) * (fb - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
        co[3] = ((dt32 * (5.0f * fa - 3.0f * fb) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
        co[2] = ((dt32 * (fb - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
        co[1] = dt32 * fa;
        co[0] = y;
        y = y1;
        f0 = k[6];
        t0s = t0;
        t1s = t1;
      } else {
        t0s = t0;
      }
      // rk_common._optimal_step_size in fp64 (dopri5.py optimal_step)
      const double rr = (double)ratio;
      double nxt;
      if (rr == 0.0) {
        nxt = dt * a.ifactor;
      } else {
        const double dfac = rr < 1.0 ? 1.0 : a.dfactor;
        const double factor = __builtin_isnan(rr) ? rr : fmin(a.ifactor, fmax(a.safety / pow(rr, 1.0 / 5.0), dfac));
        nxt = dt * factor;
      }
      dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, a.min_step), a.max_step);
      ++n_steps;
    }
    if (status) break;
    const float x = (float)((next_t - t0s) / (t1s - t0s));  // interp._interp_evaluate
    float total = co[0] + x * co[1];
    float xp = x;
#pragma unroll
    for (int j = 2; j < 5; ++j) {
      xp = xp * x;
      total = total + xp * co[j];
    }
    if (real) a.sol[(int64_t)i * BD + b * D + d] = total;
  }
  // module state after the solve: prev_x = the last evaluation's last-row input; branch_state of
  // that evaluation for this workgroup's rows
  if (blockIdx.x == 0)
    for (int q = tid; q < F; q += kDT) a.prev_out[q] = prev[q];
  if (a.branch_out) {
    for (int idx = tid; idx < kDR * F; idx += kDT) {
      const int r2 = idx / F, q = idx - r2 * F;
      const int64_t b2 = (int64_t)blockIdx.x * kDR + r2;
      if (b2 < a.B)
        a.branch_out[b2 * F + q] = ref_sigmoid(a.L.gs * (xs[r2][q / nb] - prevold[q])) > a.L.bp ? 1.0f : 0.0f;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    a.stats[0] = nfev;
    a.stats[1] = n_att;
    a.stats[2] = status;
  }
}

}  // namespace

extern "C" {

int fetode_ecg_dopri5(const fetode_hlogistic_t* layer, const float* wT, const float* bias, int32_t D,
                      const float* prev, const float* y0, int64_t B, const double* t, int32_t T, double rtol,
                      double atol, const double* opts, const float* tableau, float* solution, float* prev_out,
                      float* branch_out, void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                      void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!wT || !prev || !y0 || !t || !opts || !tableau || !solution || !prev_out || !workspace || !stats)
    return set_err(FETODE_EINVAL, "ecg dopri5: null pointer");
  if (D != layer->in_dim || D > 64) return set_err(FETODE_EINVAL, "ecg dopri5: state dim %d (must equal in_dim, <= 64)", D);
  EcgDopriArgs a;
  memset(&a, 0, sizeof(a));
  a.L = to_dev(layer);
  a.wT = wT;
  a.bh = bias;
  a.D = D;
  a.F = a.L.in * a.L.nb;
  a.prev0 = prev;
  a.y0 = y0;
  a.B = B;
  a.t = t;
  a.T = T;
  a.rtol = (float)rtol;
  a.atol = (float)atol;
  a.first_step = opts[0];
  a.safety = opts[1];
  a.ifactor = opts[2];
  a.dfactor = opts[3];
  a.min_step = opts[4];
  a.max_step = opts[5];
  a.max_steps = opts[6] > 2e9 ? 2000000000 : (int)opts[6];
  memcpy(&a.tab, tableau, sizeof(DopriTab));
  a.sol = solution;
  a.prev_out = prev_out;
  a.branch_out = branch_out;
  const int64_t grid = (B + kDR - 1) / kDR;
  if (grid > 1024) return set_err(FETODE_EUNSUPPORTED, "ecg dopri5: batch %lld too large for one cooperative grid", (long long)B);
  a.bar = (unsigned*)workspace;
  a.part = (double*)((char*)workspace + 64);
  a.stats = stats;
  a.att = attempts;
  a.max_att = attempts ? max_attempts : 0;
  hipStream_t s = (hipStream_t)stream;
  HIP_CHECK_RET(hipMemsetAsync(workspace, 0, 64, s));
  const size_t lds = sizeof(float) * ((kDR + 1) * a.F + 2 * a.F);
  if (lds > 48 * 1024) return set_err(FETODE_EINVAL, "ecg dopri5: in*num_basis=%d too large", a.F);
  void* args[] = {&a};
  HIP_CHECK_RET(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(ecg_dopri5_kernel), dim3((unsigned)grid),
                                           dim3(kDT), args, (unsigned)lds, s));
  return FETODE_OK;
}

int64_t fetode_ecg_dopri5_workspace(int64_t B) {
  const int64_t grid = (B + kDR - 1) / kDR;
  return 64 + (int64_t)sizeof(double) * 2 * 2 * grid;
}

}  // extern "C"
