// fetode_fieldn_bwd.hip — the reverse sweep of fieldn_kernel's fixed-grid solve: training of the
// depth-2 [D, H, D] KAN / KAN-FET fields that have no specialised kernel (D <= 8, H <= 64; e.g.
// KANFET([2, 16, 2]) with K = 12, KAN([4, 32, 4])).
//
// What it replaces: loss.backward() through torchdiffeq's fixed-grid solve of such a field
// (train_kanfet_node_predprey.py:254-257 with other widths), i.e. autograd through every stage
// evaluation (KANLinear.forward efficientkan.py:160-182, FerroelectricBasis.forward
// ferro_class.py:368-420, prev_x detached :381-382), the stage combines and the outputs.
//
// Structure (two passes, no per-stage host work):
//   1. fieldn_adj_kernel — one wave per trajectory walks the evaluations backwards (the tape
//      holds both layers' inputs of every evaluation, fieldn_kernel) carrying the adjoints of y
//      and of the stage derivatives; per evaluation lane o (= hidden unit o) forms d loss / d h_o
//      from the layer-1 edges (o -> every output) and its share of d loss / d x_i from the
//      layer-0 edges (i -> o), summed over the lanes by a fixed-order butterfly.  Every
//      evaluation's output adjoint (D) and hidden adjoint (H) are recorded (two planes).
//   2. the parameter gradients: the per-module VJP kernels (fetode_grad.hip, fixed-order batch
//      sums) over all n_ev * B (evaluation, trajectory) rows at once — layer 1 on (h, d loss/d k),
//      layer 0 on (x, d loss/d h); the hysteresis input of evaluation ev is the tape row of ev - 1,
//      or the state before the solve for ev = 0 (so the Ferro VJP runs as two row ranges).
// Same per-element formulas as the forward's plan (fetode_common.h LayerPlan); results agree with
// the per-stage path to fp32 summation order.
#include <string.h>

#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kFbMaxD = 8, kFbMaxH = 64, kFbWaves = 4;
constexpr float kLn2 = 0.69314718f;

__device__ __forceinline__ float fb_sig(float zl) { return rcp(1.0f + ex2(zl)); }  // 1/(1+2^zl)
// one wave's LDS traffic lands in issue order: a compiler barrier + a wait replaces a block barrier
__device__ __forceinline__ void fb_wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float fb_wave_sum(float v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

// sum_{o in [o0, o0 + no)} go[o - o0] * d edge(o, i) / d x at x: the layer's edge (o, i) as the
// forward evaluates it (fieldn fn_edge) — SiLU base, logistic branch, spline cubic per knot
// interval, Ferro elements (o, i, k) with hysteresis input pv — differentiated in x
template <bool FERRO>
__device__ float fb_vjp_input(const float* __restrict__ plan, const LayerPlan& P, int i, float x, float pv,
                              const float* go, int o0, int no) {
  const float sx = fb_sig(-x * FETODE_LOG2E);
  const float dsx = sx * ffma(x, 1.0f - sx, 1.0f);  // SiLU'
  // knot interval as fn_interval; off the grid: the plan's zero row, u = 0 (NaN for non-finite x)
  const float* g = plan + P.knots + (int64_t)i * P.NG;
  int m = -1;
  for (int j = 0; j < P.NG; ++j) m += x >= g[j] ? 1 : 0;
  const bool fin = __builtin_isfinite(x);
  const int mfix = ((unsigned)m < (unsigned)P.NI && fin) ? m : P.NI;
  const float rhm = mfix < P.NI ? plan[P.rh + (int64_t)i * P.NI + mfix] : 0.f;
  const float u = mfix < P.NI ? (x - g[mfix]) * rhm : (fin ? 0.0f : __builtin_nanf(""));
  float acc = 0.f;
  for (int oo = 0; oo < no; ++oo) {
    const int o = o0 + oo;
    const float* kw = plan + P.kw + ((int64_t)o * P.in + i) * P.NFL;
    const float4 cf = *reinterpret_cast<const float4*>(plan + P.sp + (((int64_t)o * P.in + i) * (P.NI + 1) + mfix) * 4);
    const float dsp = ffma(u, ffma(3.0f * u, cf.w, 2.0f * cf.z), cf.y) * rhm;
    acc = ffma(go[oo], ffma(kw[0], dsx, dsp), acc);
  }
  // logistic branch: d/dx 1/(1 + 2^(a' x + b')) = -ln2 a' s (1 - s)
  const float* lg = plan + P.lg + 2 * (int64_t)i * P.NB;
  for (int j = 0; j < P.NB; ++j) {
    const float s = fb_sig(ffma(lg[2 * j], x, lg[2 * j + 1]));
    const float dj = (-kLn2 * lg[2 * j]) * (s * (1.0f - s));
    float wsum = 0.f;
    for (int oo = 0; oo < no; ++oo) wsum = ffma(go[oo], plan[P.kw + ((int64_t)(o0 + oo) * P.in + i) * P.NFL + 1 + j], wsum);
    acc = ffma(dj, wsum, acc);
  }
  if constexpr (FERRO) {
    // element (o, i, k): s = sigmoid(gs(-x - Ec)), m = 1 + w s with w = wc (1 - up),
    // up = sigmoid(gs(x - prev)); z = 2 log2e k (x + Ec m), th = tanh(z ln2 / 2).
    // dm/dx = -gs w s (1 + up - s);  d th/dx = (ln2 / 2)(1 - th^2)(k2 + k2Ec dm/dx)
    const float up = fb_sig(-P.gsl2e * (x - pv));
    const float w = ffma(up, -P.wc, P.wc);
    const float gw = (-kLn2 * P.gsl2e) * w;
    const float upp1 = 1.0f + up;
    for (int oo = 0; oo < no; ++oo) {
      const int64_t e0 = (int64_t)(o0 + oo) * P.in * P.K + (int64_t)i * P.K;
      const float* GEc = plan + P.fe_GEc + e0;
      const float* k2 = plan + P.fe_k2 + e0;
      const float* kE = plan + P.fe_k2Ec + e0;
      const float* cp = plan + P.fe_CPs2 + e0;
      float d = 0.f;
      for (int k = 0; k < P.K; ++k) {
        const float s = rcp(ex2(ffma(P.gsl2e, x, GEc[k])) + 1.0f);
        const float mm = ffma(w, s, 1.0f);
        const float z = ffma(kE[k], mm, k2[k] * x);
        const float th = ffma(rcp(ex2(z) + 1.0f), -2.0f, 1.0f);
        const float dm = gw * s * (upp1 - s);
        d = ffma(cp[k] * ffma(-th, th, 1.0f), ffma(kE[k], dm, k2[k]), d);
      }
      acc = ffma(go[oo] * (0.5f * kLn2), d, acc);
    }
  }
  return acc;
}

struct FbArgs {
  const float* plan;
  LayerPlan P0, P1;
  int32_t method;
  int64_t B;
  const float* step_coef;
  int32_t n_steps;
  const int32_t* out_step;
  const int32_t* out_mode;
  const float* out_slope;
  int32_t T;
  const float* gsol;    // (T, B, D)
  const float* tape;    // planes (n_ev, B, D) then (n_ev, B, H)
  const float* state0;  // hysteresis state before the solve, or null (every init bit set)
  uint32_t init_mask;
  float* gy0;           // (B, D) or null
  float* gadj;          // planes (n_ev, B, D) d loss / d k, then (n_ev, B, H) d loss / d h
};

// stage-combine coefficients of one step in the forward's fp32 arithmetic (odeint.py
// _combine_coefs): y1 = y + sum_j bc[j] k_j,  X_st = y + sum_{j<st} ac[st][j] k_j
__device__ void fb_coefs(int method, float dt, float hh, float h6, float bc[4], float ac[4][3]) {
  const float third = 1.0f / 3.0f;
  for (int i = 0; i < 4; ++i) {
    bc[i] = 0.f;
    for (int j = 0; j < 3; ++j) ac[i][j] = 0.f;
  }
  if (method == FETODE_RK4) {  // rk_common.rk4_alt_step_func (3/8 rule)
    bc[0] = dt * 0.125f;
    bc[1] = 3.0f * dt * 0.125f;
    bc[2] = 3.0f * dt * 0.125f;
    bc[3] = dt * 0.125f;
    ac[1][0] = dt * third;
    ac[2][0] = -dt * third;
    ac[2][1] = dt;
    ac[3][0] = dt;
    ac[3][1] = -dt;
    ac[3][2] = dt;
  } else if (method == FETODE_RK4_CLASSIC) {
    bc[0] = h6;
    bc[1] = 2.0f * h6;
    bc[2] = 2.0f * h6;
    bc[3] = h6;
    ac[1][0] = hh;
    ac[2][1] = hh;
    ac[3][2] = dt;
  } else if (method == FETODE_MIDPOINT) {
    bc[1] = dt;
    ac[1][0] = hh;
  } else {
    bc[0] = dt;
  }
}

template <bool FERRO>
__global__ __launch_bounds__(64 * kFbWaves) void fieldn_adj_kernel(FbArgs a) {
  __shared__ float s_x[kFbWaves][kFbMaxD], s_p[kFbWaves][kFbMaxD], s_gk[kFbWaves][kFbMaxD];
  __shared__ float s_ak[kFbWaves][4][kFbMaxD], s_ac[kFbWaves][4][3];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kFbWaves + wid;
  if (b >= a.B) return;  // whole waves only; no workgroup barriers below
  const LayerPlan& P0 = a.P0;
  const LayerPlan& P1 = a.P1;
  const int D = P0.in, H = P0.out;
  const float* __restrict__ plan = a.plan;
  const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  const int64_t n_ev = (int64_t)a.n_steps * ns;
  const float* X = a.tape;
  const float* Hh = a.tape + n_ev * a.B * D;
  float* GK = a.gadj;
  float* GH = a.gadj + n_ev * a.B * D;
  float* xs = s_x[wid];
  float* ps = s_p[wid];
  float* gk = s_gk[wid];
  float(&ak)[4][kFbMaxD] = s_ak[wid];
  float(&acs)[4][3] = s_ac[wid];
  const bool dl = lane < D, hl = lane < H;
  float ay1 = 0.f, ay = 0.f;  // adjoint of y at the end of the current step (lanes < D)
  int jj = a.T - 1;
  for (int s = a.n_steps - 1; s >= 0; --s) {
    float bc[4], ac[4][3];
    fb_coefs(a.method, a.step_coef[4 * s], a.step_coef[4 * s + 1], a.step_coef[4 * s + 2], bc, ac);
    float ay0x = 0.f;  // outputs produced in this step (y at step start, end, or interpolated)
    for (; jj >= 1 && a.out_step[jj] == s; --jj) {
      if (dl) {
        const float g = a.gsol[((int64_t)jj * a.B + b) * D + lane];
        const int mode = a.out_mode[jj];
        if (mode == 0) {
          ay0x += g;
        } else if (mode == 1) {
          ay1 += g;
        } else {
          const float slo = a.out_slope[jj];
          ay1 = ffma(slo, g, ay1);
          ay0x = ffma(1.0f - slo, g, ay0x);
        }
      }
    }
    if (dl) {
      for (int j = 0; j < ns; ++j) ak[j][lane] = bc[j] * ay1;
      ay = ay1 + ay0x;
    }
    if (lane == 0)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) acs[i][j] = ac[i][j];
    for (int st = ns - 1; st >= 0; --st) {
      const int64_t ev = (int64_t)s * ns + st;
      if (dl) {
        const float x = X[(ev * a.B + b) * D + lane];
        xs[lane] = x;
        ps[lane] = ev > 0 ? X[((ev - 1) * a.B + b) * D + lane]
                          : ((a.init_mask & 1u) ? x : (FERRO ? a.state0[b * D + lane] : 0.f));
        gk[lane] = ak[st][lane];
      }
      float h = 0.f, ph = 0.f;
      if (hl) {
        h = Hh[(ev * a.B + b) * H + lane];
        ph = ev > 0 ? Hh[((ev - 1) * a.B + b) * H + lane]
                    : ((a.init_mask & 2u) ? h : (FERRO ? a.state0[a.B * D + b * H + lane] : 0.f));
      }
      fb_wsync();
      // layer 1 (h -> k): d loss / d h_o on lane o
      const float gh = hl ? fb_vjp_input<FERRO>(plan, P1, lane, h, ph, gk, 0, D) : 0.f;
      if (dl) GK[(ev * a.B + b) * D + lane] = gk[lane];
      if (hl) GH[(ev * a.B + b) * H + lane] = gh;
      // layer 0 (x -> h): d loss / d x_i = sum over the lanes o of gh_o d edge(o, i) / d x_i
      float gx = 0.f;
      for (int i = 0; i < D; ++i) {
        const float one = 1.0f;
        const float c = hl ? gh * fb_vjp_input<FERRO>(plan, P0, i, xs[i], ps[i], &one, lane, 1) : 0.f;
        const float sum = fb_wave_sum(c);
        if (lane == i) gx = sum;
      }
      if (dl) {
        ay += gx;
        for (int j = 0; j < st; ++j) ak[j][lane] = ffma(acs[st][j], gx, ak[j][lane]);
      }
      fb_wsync();
    }
    ay1 = ay;
  }
  if (dl && a.gy0) a.gy0[b * D + lane] = ay1 + a.gsol[b * D + lane];  // solution[0] = y0
}

int64_t n_evals(int32_t method, int32_t n_steps) {
  return (int64_t)n_steps * (method == FETODE_RK4 || method == FETODE_RK4_CLASSIC ? 4 : method == FETODE_MIDPOINT ? 2 : 1);
}

int64_t align16(int64_t n) { return (n + 15) / 16 * 16; }

int zero_grads(const fetode_field_t* f, const fetode_kanlinear_grad_t* kg, const fetode_ferro_grad_t* fg, hipStream_t s) {
  for (int l = 0; l < 2; ++l) {
    const fetode_kanlinear_t& k = f->kan[l];
    const int64_t in = k.in_features, out = k.out_features, NS = k.grid_size + k.spline_order, NB = k.num_logistic;
    if (kg) {
      const fetode_kanlinear_grad_t& g = kg[l];
      float* p[7] = {g.base_weight, g.spline_weight, g.spline_scaler, g.logistic_a, g.logistic_b, g.logistic_weight,
                     g.logistic_scaler};
      const int64_t n[7] = {out * in, out * in * NS, out * in, in * NB, in * NB, out * in * NB, out};
      for (int q = 0; q < 7; ++q)
        if (p[q] && n[q] > 0) HIP_CHECK_RET(hipMemsetAsync(p[q], 0, sizeof(float) * n[q], s));
    }
    if (fg && f->ferro) {
      const fetode_ferro_grad_t& g = fg[l];
      float* p[5] = {g.k, g.Ec, g.Ps, g.bias, g.coef};
      const int64_t n = (int64_t)f->ferro[l].in_dim * f->ferro[l].out_dim * f->ferro[l].num_basis;
      for (int q = 0; q < 5; ++q)
        if (p[q]) HIP_CHECK_RET(hipMemsetAsync(p[q], 0, sizeof(float) * n, s));
    }
  }
  return FETODE_OK;
}

bool any_kan(const fetode_kanlinear_grad_t& g) {
  return g.base_weight || g.spline_weight || g.spline_scaler || g.logistic_a || g.logistic_b || g.logistic_weight ||
         g.logistic_scaler;
}
bool any_ferro(const fetode_ferro_grad_t& g) { return g.k || g.Ec || g.Ps || g.bias || g.coef; }

}  // namespace

int64_t fetode::fieldn_fixed_backward_workspace(const fetode_field_t* f, int32_t method, int32_t n_steps, int64_t B) {
  const int64_t D = f->kan[0].in_features, H = f->kan[0].out_features;
  const int64_t kw0 = fetode_kanlinear_backward_workspace(&f->kan[0]), kw1 = fetode_kanlinear_backward_workspace(&f->kan[1]);
  if (kw0 < 0 || kw1 < 0) return -1;
  return (int64_t)sizeof(float) * align16(n_evals(method, n_steps) * B * (D + H)) + (kw0 > kw1 ? kw0 : kw1);
}

int fetode::fieldn_fixed_backward(const fetode_field_t* f, const void* plan, int32_t method, int64_t B,
                                  const float* step_coef, int32_t n_steps, const int32_t* out_step,
                                  const int32_t* out_mode, const float* out_slope, int32_t T,
                                  const float* grad_solution, const float* tape, const float* state0,
                                  uint32_t init_mask, float* grad_y0, const fetode_kanlinear_grad_t* kan_grads,
                                  const fetode_ferro_grad_t* ferro_grads, void* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int D = f->kan[0].in_features, H = f->kan[0].out_features;
  if (D > kFbMaxD || H > kFbMaxH) return set_err(FETODE_EUNSUPPORTED, "fieldn backward: widths beyond [8, 64, 8]");
  const int64_t n_ev = n_evals(method, n_steps);
  float* gadj = (float*)workspace;
  void* kws = gadj + align16(n_ev * B * (D + H));
  FbArgs a;
  memset(&a, 0, sizeof(a));
  a.plan = (const float*)plan;
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  a.method = method;
  a.B = B;
  a.step_coef = step_coef;
  a.n_steps = n_steps;
  a.out_step = out_step;
  a.out_mode = out_mode;
  a.out_slope = out_slope;
  a.T = T;
  a.gsol = grad_solution;
  a.tape = tape;
  a.state0 = state0;
  a.init_mask = f->ferro ? init_mask : 3u;
  a.gy0 = grad_y0;
  a.gadj = gadj;
  hipLaunchKernelGGL(f->ferro ? fieldn_adj_kernel<true> : fieldn_adj_kernel<false>, dim3(nblk(B, kFbWaves)),
                     dim3(64 * kFbWaves), 0, s, a);
  LAUNCH_CHECK();
  if (n_ev == 0) return zero_grads(f, kan_grads, ferro_grads, s);
  // parameter gradients: the per-module VJPs over all n_ev * B rows (written, not accumulated)
  const int64_t R = n_ev * B;
  const float* Xp = tape;           // layer-0 inputs (R, D)
  const float* Hp = tape + R * D;   // layer-1 inputs (R, H)
  const float* GKp = gadj;          // layer-1 output adjoints (R, D)
  const float* GHp = gadj + R * D;  // layer-0 output adjoints (R, H)
  for (int l = 0; l < 2; ++l) {
    const float* x = l == 0 ? Xp : Hp;
    const float* g = l == 0 ? GHp : GKp;
    const int in = l == 0 ? D : H;
    if (kan_grads && any_kan(kan_grads[l])) {
      const int rc = fetode_kanlinear_backward(&f->kan[l], x, R, g, nullptr, &kan_grads[l], kws, 0, stream);
      if (rc) return rc;
    }
    if (f->ferro && ferro_grads && any_ferro(ferro_grads[l])) {
      // evaluation 0: the hysteresis input is the state before the solve (or x itself: reinit);
      // evaluations >= 1: the previous evaluation's row of the same plane
      const bool re = (init_mask >> l) & 1u;
      const float* p0 = re ? nullptr : state0 + (l == 0 ? 0 : B * D);
      int rc = fetode_ferro_backward(&f->ferro[l], x, B, p0, re ? 1 : 0, g, nullptr, &ferro_grads[l], 0, stream);
      if (rc) return rc;
      if (n_ev > 1) {
        rc = fetode_ferro_backward(&f->ferro[l], x + B * in, R - B, x, 0, g + B * (l == 0 ? H : D), nullptr,
                                   &ferro_grads[l], 1, stream);
        if (rc) return rc;
      }
    }
  }
  return FETODE_OK;
}
