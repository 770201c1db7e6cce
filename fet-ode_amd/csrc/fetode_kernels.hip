// fetode_kernels.hip — MI355X (gfx950) kernels of the KAN-FET Neural-ODE hot path
// and the C ABI declared in include/fetode.h.
//
// Kernels
//   plan_build_kernel       per-layer parameter transform, once per solve
//   fused_integrate_kernel  whole fixed-grid solve (rk4 3/8, classic rk4, euler, midpoint) of a
//                           depth-2 KAN / KAN-FET field in ONE launch; hysteresis state, stage
//                           values and the field's activations never leave the CU
//   kanlinear_fwd_kernel    efficientkan.KANLinear.forward, generic widths
//   bsplines_kernel         efficientkan.KANLinear.b_splines, generic widths (bitwise = reference)
//   ferro_fwd_kernel        ferro_class.FerroelectricBasis.forward, generic widths
//   rk_combine_kernel       torchdiffeq stage combines for the per-stage (generic func) path
//
// Mapping of the fused kernel: a trajectory is owned by a group of LPT=32
// lanes (two trajectories per wave, 8 per 256-thread workgroup).  Per field evaluation and per
// layer: phase A computes the per-input features (SiLU, local Cox–de Boor bases, logistic basis,
// hysteresis direction gate) into LDS; phase B gives each lane one (output o, chunk c) item that
// owns a fixed slice of the (input, basis) Ferro elements and of the KAN feature weights, held in
// VGPRs for the whole solve; phase C reduces the chunk partials per output.  The RK stage
// combine runs on lanes d < D in registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fetode.h"
#include "fetode_device.h"

using namespace fetode;

// ---------------------------------------------------------------------------------------------
// error handling
// ---------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_CHECK_RET(expr)                                                             \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return set_err(FETODE_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define LAUNCH_CHECK()                                                                  \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess) return set_err(FETODE_EHIP, "kernel launch: %s", hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------------------------------------
// plan layout (floats, per layer, concatenated over layers)
// ---------------------------------------------------------------------------------------------
struct LayerPlan {
  int in, out, K, NB, SO, NG, NF;  // NF = 1 + NS + NB features per input
  int64_t base;                    // float offset of this layer in the plan
  int64_t fe_GEc, fe_k2, fe_k2Ec, fe_CPs2, fconst, kw, lg, knots, rk, end;
  float gsl2e, wc;                 // gate_slope*log2e, -2*(1-alpha)
};

static void layer_plan(const fetode_kanlinear_t& kl, const fetode_ferro_t* fl, int64_t base,
                       LayerPlan* p) {
  p->in = kl.in_features;
  p->out = kl.out_features;
  p->K = fl ? fl->num_basis : 0;
  p->NB = kl.num_logistic;
  p->SO = kl.spline_order;
  p->NG = kl.grid_size + 2 * kl.spline_order + 1;
  p->NF = 1 + (kl.grid_size + kl.spline_order) + p->NB;
  const int64_t NE = (int64_t)p->in * p->out * p->K;
  p->base = base;
  int64_t o = base;
  p->fe_GEc = o; o += NE;
  p->fe_k2 = o; o += NE;
  p->fe_k2Ec = o; o += NE;
  p->fe_CPs2 = o; o += NE;
  p->fconst = o; o += p->out;
  p->kw = o; o += (int64_t)p->out * p->in * p->NF;
  p->lg = o; o += (int64_t)p->in * p->NB * 2;
  p->knots = o; o += (int64_t)p->in * p->NG;
  p->rk = o; o += (int64_t)p->in * p->SO * (p->NG - 1);
  o = (o + 3) & ~int64_t(3);
  p->end = o;
  // the reference multiplies by Python floats: (1.0 - alpha) is formed in double, then rounded
  p->gsl2e = fl ? (float)fl->gate_slope * FETODE_LOG2E : 0.f;
  p->wc = fl ? -2.0f * (float)(1.0 - fl->alpha) : 0.f;
}

static int validate_field(const fetode_field_t* f) {
  if (!f || f->n_layers <= 0 || !f->kan) return set_err(FETODE_EINVAL, "field: no layers");
  for (int l = 0; l < f->n_layers; ++l) {
    const fetode_kanlinear_t& k = f->kan[l];
    if (k.in_features <= 0 || k.out_features <= 0 || k.grid_size <= 0 || k.spline_order < 1 ||
        k.spline_order > 3 || k.num_logistic < 0)
      return set_err(FETODE_EINVAL, "layer %d: bad KANLinear dims", l);
    if (!k.grid || !k.base_weight || !k.spline_weight)
      return set_err(FETODE_EINVAL, "layer %d: null KANLinear parameter", l);
    if (k.num_logistic > 0 && (!k.logistic_a || !k.logistic_b || !k.logistic_weight))
      return set_err(FETODE_EINVAL, "layer %d: null logistic parameter", l);
    if (l > 0 && k.in_features != f->kan[l - 1].out_features)
      return set_err(FETODE_EINVAL, "layer %d: in_features %d != previous out %d", l,
                     k.in_features, f->kan[l - 1].out_features);
    if (f->ferro) {
      const fetode_ferro_t& r = f->ferro[l];
      if (r.in_dim != k.in_features || r.out_dim != k.out_features || r.num_basis <= 0)
        return set_err(FETODE_EINVAL, "layer %d: Ferro dims (%d,%d,%d) mismatch KANLinear", l,
                       r.in_dim, r.out_dim, r.num_basis);
      if (!r.k || !r.Ec || !r.Ps || !r.bias || !r.coef)
        return set_err(FETODE_EINVAL, "layer %d: null Ferro parameter", l);
    }
  }
  return FETODE_OK;
}

// ---------------------------------------------------------------------------------------------
// plan build
// ---------------------------------------------------------------------------------------------
__global__ void plan_build_kernel(LayerPlan P, fetode_kanlinear_t kl, fetode_ferro_t fl, int has_ferro,
                                  float* __restrict__ plan) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int in = P.in, out = P.out, K = P.K, NB = P.NB, NG = P.NG, SO = P.SO, NF = P.NF;
  const int NS = NG - 1 - SO;
  const float l2 = FETODE_LOG2E;
  // Ferro elements, reordered (o, i, k) so a (o, chunk) lane reads a contiguous run
  if (has_ferro) {
    const int NP = in * K;
    if (tid < out * NP) {
      const int o = tid / NP, p = tid % NP, i = p / K, k = p % K;
      const int src = (i * out + o) * K + k;
      const float kk = fl.k[src], Ec = fl.Ec[src], Ps = fl.Ps[src], co = fl.coef[src];
      plan[P.fe_GEc + tid] = P.gsl2e * Ec;
      const float k2 = 2.0f * l2 * kk;
      plan[P.fe_k2 + tid] = k2;
      plan[P.fe_k2Ec + tid] = k2 * Ec;
      plan[P.fe_CPs2 + tid] = -2.0f * co * Ps;
    }
    if (tid < out) {
      float s = 0.f;
      for (int i = 0; i < in; ++i)
        for (int k = 0; k < K; ++k) {
          const int src = (i * out + tid) * K + k;
          s += fl.coef[src] * (fl.Ps[src] + fl.bias[src]);
        }
      plan[P.fconst + tid] = s;
    }
  } else if (tid < out) {
    plan[P.fconst + tid] = 0.f;
  }
  // KAN feature weights W[o][i][f]
  if (tid < out * in * NF) {
    const int o = tid / (in * NF), r = tid % (in * NF), i = r / NF, f = r % NF;
    float w;
    if (f == 0) {
      w = kl.base_weight[o * in + i];
    } else if (f <= NS) {
      const float sc = kl.spline_scaler ? kl.spline_scaler[o * in + i] : 1.0f;
      w = kl.spline_weight[(o * in + i) * NS + (f - 1)] * sc;
    } else {
      const int j = f - 1 - NS;
      const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      w = 2.0f * ((kl.logistic_weight[o * (in * NB) + i * NB + j] * kl.scale_logistic) * ls);
    }
    plan[P.kw + tid] = w;
  }
  if (tid < in * NB) {
    const float a = kl.logistic_a[tid], b = kl.logistic_b[tid];
    plan[P.lg + 2 * tid + 0] = -a * l2;
    plan[P.lg + 2 * tid + 1] = (a * b) * l2;
  }
  if (tid < in * NG) plan[P.knots + tid] = kl.grid[tid];
  if (tid < in * SO * (NG - 1)) {
    const int i = tid / (SO * (NG - 1)), r = tid % (SO * (NG - 1));
    const int k = r / (NG - 1) + 1, j = r % (NG - 1);
    const float* g = kl.grid + i * NG;
    plan[P.rk + tid] = (j <= NG - 1 - k) ? 1.0f / (g[j + k] - g[j]) : 0.0f;
  }
}

// ---------------------------------------------------------------------------------------------
// fused depth-2 field: compile-time shapes
// ---------------------------------------------------------------------------------------------
template <int IN, int OUT, int K, int NB, int SO, int NG, int LPT>
struct LayerShape {
  static constexpr int NS = NG - 1 - SO;
  static constexpr int NF = 1 + NS + NB;
  static constexpr int C = LPT / OUT;           // chunks per output
  static constexpr int NP = IN * K;             // Ferro (input, basis) pairs
  static constexpr int NQ = IN * NF;            // KAN features
  static constexpr int EPL = K > 0 ? (NP + C - 1) / C : 0;
  static constexpr int FPL = (NQ + C - 1) / C;
  static constexpr int LJ = NB > 0 ? (IN * NB + LPT - 1) / LPT : 0;
  static constexpr int NRK = SO * (NG - 1);
  static_assert(C >= 1, "out_features must be <= lanes per trajectory");
};

// per-lane register-resident slice of one layer's parameters
template <class S>
struct LayerRegs {
  float GEc[S::EPL > 0 ? S::EPL : 1], k2[S::EPL > 0 ? S::EPL : 1], k2Ec[S::EPL > 0 ? S::EPL : 1],
      CPs2[S::EPL > 0 ? S::EPL : 1];
  float fw[S::FPL];
  float lna[S::LJ > 0 ? S::LJ : 1], lab[S::LJ > 0 ? S::LJ : 1];
  int o, c;
  bool active;

  __device__ void load(const float* __restrict__ plan, const LayerPlan& P, int lane) {
    o = lane / S::C;
    c = lane % S::C;
    active = lane < S::C * P.out;
    const int oo = active ? o : 0;
#pragma unroll
    for (int r = 0; r < S::EPL; ++r) {
      const int p = c + S::C * r;
      const bool ok = active && p < S::NP;
      const int64_t idx = (int64_t)oo * S::NP + (ok ? p : 0);
      GEc[r] = ok ? plan[P.fe_GEc + idx] : 0.f;
      k2[r] = ok ? plan[P.fe_k2 + idx] : 0.f;
      k2Ec[r] = ok ? plan[P.fe_k2Ec + idx] : 0.f;
      CPs2[r] = ok ? plan[P.fe_CPs2 + idx] : 0.f;
    }
#pragma unroll
    for (int f = 0; f < S::FPL; ++f) {
      const int q = c + S::C * f;
      const bool ok = active && q < S::NQ;
      fw[f] = ok ? plan[P.kw + (int64_t)oo * S::NQ + q] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < S::LJ; ++r) {
      const int job = lane + S::LPT_ * r;
      const bool ok = job < S::IN_NB;
      lna[r] = ok ? plan[P.lg + 2 * job] : 0.f;
      lab[r] = ok ? plan[P.lg + 2 * job + 1] : 0.f;
    }
  }
};

// Adds the two helper constants LayerRegs needs without widening LayerShape's public surface.
template <int IN, int OUT, int K, int NB, int SO, int NG, int LPT>
struct LayerShapeX : LayerShape<IN, OUT, K, NB, SO, NG, LPT> {
  static constexpr int IN_ = IN, OUT_ = OUT, K_ = K, NB_ = NB, SO_ = SO, NG_ = NG, LPT_ = LPT, IN_NB = IN * NB;
};

// Per-trajectory LDS scratch of one layer
template <class S>
struct LayerLds {
  float F[S::IN_ * S::NF];     // features
  float G[S::IN_ * 2];         // (x_i, w_i) gate inputs of the Ferro elements
  float prev[S::IN_];          // hysteresis prev_x (compact)
  float P[S::OUT_ * S::C];     // chunk partials
};

template <class S, bool FERRO>
__device__ __forceinline__ void layer_phase_A(const float* __restrict__ xin, LayerLds<S>& L,
                                              const LayerRegs<S>& R, const float* __restrict__ knots,
                                              const float* __restrict__ rk, const LayerPlan& P,
                                              int lane, bool reinit) {
  constexpr int LPT = S::LPT_;
  // logistic basis: phi'_{ij} = 1/(1+exp(-a(x-b)))  (efficientkan.py:24, factor 2 in weights)
#pragma unroll
  for (int r = 0; r < S::LJ; ++r) {
    const int job = lane + LPT * r;
    if (job < S::IN_NB) {
      const int i = job / S::NB_, j = job % S::NB_;
      const float x = xin[i];
      L.F[i * S::NF + 1 + S::NS + j] = rcp(1.0f + ex2(ffma(R.lna[r], x, R.lab[r])));
    }
  }
  // per input: SiLU, spline bases, hysteresis gate and state update
  for (int i = lane; i < S::IN_; i += LPT) {
    const float x = xin[i];
    L.F[i * S::NF] = silu(x);
    float* Fi = &L.F[i * S::NF + 1];
    bspline_local<S::SO_>(
        x, S::NG_, knots + i * S::NG_, rk + i * S::NRK, [&](int c, float v) { Fi[c] = v; });
    if constexpr (FERRO) {
      const float pv = reinit ? x : L.prev[i];
      const float dx = x - pv;
      // is_moving_up = sigmoid(gate_slope*dx) (ferro_class.py:387); w = -2(1-alpha)(1-u)
      const float u = rcp(1.0f + ex2(-P.gsl2e * dx));
      L.G[2 * i] = x;
      L.G[2 * i + 1] = P.wc * (1.0f - u);
      L.prev[i] = x;  // ferro_class.py:409
    }
  }
}

template <class S, bool FERRO>
__device__ __forceinline__ float layer_phase_B(const LayerLds<S>& L, const LayerRegs<S>& R,
                                               float gsl2e) {
  float acc = 0.f;
  if (!R.active) return acc;
  if constexpr (FERRO) {
    // Ferro element (ferro_class.py:384-414) with branch_sign == 1 (never written, F8):
    //   sl = (1-u) * sigmoid(gs(-x-Ec)),  m = alpha + (1-alpha)(1-2 sl) = 1 + w*s
    //   coef*(Ps*tanh(k(x+Ec m)) + bias) = coef(Ps+bias) - 2 coef Ps / (1+exp(2k(x+Ec m)))
#pragma unroll
    for (int r = 0; r < S::EPL; ++r) {
      const int p = R.c + S::C * r;
      if (p < S::NP) {
        const int i = p / S::K_;
        const float x = L.G[2 * i], w = L.G[2 * i + 1];
        const float s = rcp(1.0f + ex2(ffma(gsl2e, x, R.GEc[r])));
        const float m = ffma(w, s, 1.0f);
        const float z = ffma(R.k2Ec[r], m, R.k2[r] * x);
        const float t = rcp(1.0f + ex2(z));
        acc = ffma(R.CPs2[r], t, acc);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < S::FPL; ++f) {
    const int q = R.c + S::C * f;
    if (q < S::NQ) acc = ffma(R.fw[f], L.F[q], acc);
  }
  return acc;
}

struct FusedArgs {
  const float* plan;
  LayerPlan P0, P1;
  int32_t method;
  const float* y0;
  int64_t B;
  const float* step_coef;  // n_steps x 4 : dt, 0.5dt, dt/6, unused (time dtype -> fp32)
  int32_t n_steps;
  const int32_t* out_step;
  const int32_t* out_mode;
  const float* out_slope;
  int32_t T;
  float* solution;
  float* state;
  uint32_t init_mask;
  float* ckpt;
  int32_t single_eval;     // 1: out = field(y0) once (fetode_field_forward)
  float* eval_out;
};

template <int IN0, int H, int OUT, int K, int NB, int SO, int NG, bool FERRO, int LPT>
__global__ __launch_bounds__(256) void fused_integrate_kernel(FusedArgs a) {
  using S0 = LayerShapeX<IN0, H, FERRO ? K : 0, NB, SO, NG, LPT>;
  using S1 = LayerShapeX<H, OUT, FERRO ? K : 0, NB, SO, NG, LPT>;
  constexpr int TPB = 256 / LPT;  // trajectories per block
  constexpr int D = IN0;
  static_assert(IN0 == OUT, "ODE field must map R^D -> R^D");
  static_assert(D <= LPT && H <= LPT, "dims exceed lanes per trajectory");

  struct TrajLds {
    float x0[IN0];
    float h[H];
    float kout[OUT];
    LayerLds<S0> L0;
    LayerLds<S1> L1;
  };
  __shared__ float s_knots0[IN0 * NG], s_rk0[IN0 * S0::NRK];
  __shared__ float s_knots1[H * NG], s_rk1[H * S1::NRK];
  __shared__ float s_const0[H], s_const1[OUT];
  __shared__ TrajLds s_traj[TPB];

  const int tid = threadIdx.x;
  const int g = tid / LPT, lane = tid % LPT;
  const int64_t b = (int64_t)blockIdx.x * TPB + g;
  const bool valid = b < a.B;
  TrajLds& T = s_traj[g];

  // stage shared parameters
  for (int i = tid; i < IN0 * NG; i += 256) s_knots0[i] = a.plan[a.P0.knots + i];
  for (int i = tid; i < IN0 * S0::NRK; i += 256) s_rk0[i] = a.plan[a.P0.rk + i];
  for (int i = tid; i < H * NG; i += 256) s_knots1[i] = a.plan[a.P1.knots + i];
  for (int i = tid; i < H * S1::NRK; i += 256) s_rk1[i] = a.plan[a.P1.rk + i];
  for (int i = tid; i < H; i += 256) s_const0[i] = a.plan[a.P0.fconst + i];
  for (int i = tid; i < OUT; i += 256) s_const1[i] = a.plan[a.P1.fconst + i];

  LayerRegs<S0> R0;
  LayerRegs<S1> R1;
  R0.load(a.plan, a.P0, lane);
  R1.load(a.plan, a.P1, lane);

  constexpr int SW = FERRO ? IN0 + H : 0;  // state width
  if (FERRO) {
    for (int i = lane; i < IN0; i += LPT) T.L0.prev[i] = valid ? a.state[b * SW + i] : 0.f;
    for (int i = lane; i < H; i += LPT) T.L1.prev[i] = valid ? a.state[b * SW + IN0 + i] : 0.f;
  }
  bool re0 = FERRO && (a.init_mask & 1u), re1 = FERRO && (a.init_mask & 2u);

  // RK state lives in registers of lanes d < D
  const int d = lane;
  const bool own = d < D;
  float y = (own && valid) ? a.y0[b * D + d] : 0.f;
  if (!a.single_eval && own && valid) a.solution[b * D + d] = y;  // solution[0] = y0

  auto eval = [&](float xin) -> float {
    if (own) T.x0[d] = xin;
    __syncthreads();
    layer_phase_A<S0, FERRO>(T.x0, T.L0, R0, s_knots0, s_rk0, a.P0, lane, re0);
    re0 = false;
    __syncthreads();
    float acc0 = layer_phase_B<S0, FERRO>(T.L0, R0, a.P0.gsl2e);
    if (R0.active) T.L0.P[R0.o * S0::C + R0.c] = acc0;
    __syncthreads();
    for (int o = lane; o < H; o += LPT) {
      float s = s_const0[o];
#pragma unroll
      for (int c = 0; c < S0::C; ++c) s += T.L0.P[o * S0::C + c];
      T.h[o] = s;
    }
    __syncthreads();
    layer_phase_A<S1, FERRO>(T.h, T.L1, R1, s_knots1, s_rk1, a.P1, lane, re1);
    re1 = false;
    __syncthreads();
    float acc1 = layer_phase_B<S1, FERRO>(T.L1, R1, a.P1.gsl2e);
    if (R1.active) T.L1.P[R1.o * S1::C + R1.c] = acc1;
    __syncthreads();
    for (int o = lane; o < OUT; o += LPT) {
      float s = s_const1[o];
#pragma unroll
      for (int c = 0; c < S1::C; ++c) s += T.L1.P[o * S1::C + c];
      T.kout[o] = s;
    }
    __syncthreads();
    return own ? T.kout[d] : 0.f;
  };

  if (a.single_eval) {
    const float f = eval(y);
    if (own && valid) a.eval_out[b * OUT + d] = f;
  } else {
    int jj = 1;
    const float third = 1.0f / 3.0f;
    for (int s = 0; s < a.n_steps; ++s) {
      const float dt = a.step_coef[4 * s + 0];
      if (a.ckpt && valid) {
        // prev[i] is written and read by the same lane (i % LPT): no barrier needed
        const int64_t W = D + SW;
        float* ck = a.ckpt + ((int64_t)s * a.B + b) * W;
        if (own) ck[d] = y;
        if (FERRO) {
          for (int i = lane; i < IN0; i += LPT) ck[D + i] = T.L0.prev[i];
          for (int i = lane; i < H; i += LPT) ck[D + IN0 + i] = T.L1.prev[i];
        }
      }
      float y1;
      if (a.method == FETODE_RK4) {
        // rk_common.rk4_alt_step_func, exact op order (3/8 rule)
        const float k1 = eval(y);
        const float k2 = eval(y + (dt * k1) * third);
        const float k3 = eval(y + dt * (k2 - k1 * third));
        const float k4 = eval(y + dt * ((k1 - k2) + k3));
        y1 = y + (((k1 + 3.0f * (k2 + k3)) + k4) * dt) * 0.125f;
      } else if (a.method == FETODE_RK4_CLASSIC) {
        // train_kan_fet_ett.py:72-76 / train_ecg_kan_fet_nn_ode.py:699-703
        const float hh = a.step_coef[4 * s + 1], h6 = a.step_coef[4 * s + 2];
        const float k1 = eval(y);
        const float k2 = eval(y + hh * k1);
        const float k3 = eval(y + hh * k2);
        const float k4 = eval(y + dt * k3);
        y1 = y + h6 * (((k1 + 2.0f * k2) + 2.0f * k3) + k4);
      } else if (a.method == FETODE_MIDPOINT) {
        const float hh = a.step_coef[4 * s + 1];
        const float k1 = eval(y);
        const float k2 = eval(y + k1 * hh);
        y1 = y + dt * k2;
      } else {  // Euler
        const float k1 = eval(y);
        y1 = y + dt * k1;
      }
      while (jj < a.T && a.out_step[jj] == s) {
        const int mode = a.out_mode[jj];
        const float v = mode == 0 ? y : (mode == 1 ? y1 : y + a.out_slope[jj] * (y1 - y));
        if (own && valid) a.solution[((int64_t)jj * a.B + b) * D + d] = v;
        ++jj;
      }
      y = y1;
    }
  }
  if (FERRO) {
    __syncthreads();
    if (valid) {
      for (int i = lane; i < IN0; i += LPT) a.state[b * SW + i] = T.L0.prev[i];
      for (int i = lane; i < H; i += LPT) a.state[b * SW + IN0 + i] = T.L1.prev[i];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// fused-shape registry
// ---------------------------------------------------------------------------------------------
typedef void (*fused_fn)(FusedArgs);
struct FusedEntry {
  int in0, h, out, K, NB, SO, NG;
  bool ferro;
  fused_fn fn;
};
#define FUSED(IN0, H, OUT, K, NB, SO, NG, FE) \
  {IN0, H, OUT, K, NB, SO, NG, FE, fused_integrate_kernel<IN0, H, OUT, K, NB, SO, NG, FE, 32>}
static const FusedEntry kFused[] = {
    FUSED(2, 10, 2, 10, 10, 3, 12, true),   // LV KAN-FET [2,10,2], K=10 (train_kanfet_node_predprey.py:146)
    FUSED(2, 10, 2, 1, 10, 3, 12, false),   // LV KAN [2,10,2] (predator_prey.py:101)
};

static const FusedEntry* find_fused(const fetode_field_t* f) {
  if (f->n_layers != 2) return nullptr;
  const fetode_kanlinear_t &k0 = f->kan[0], &k1 = f->kan[1];
  if (k0.grid_size != k1.grid_size || k0.spline_order != k1.spline_order ||
      k0.num_logistic != k1.num_logistic)
    return nullptr;
  const int NG = k0.grid_size + 2 * k0.spline_order + 1;
  for (const FusedEntry& e : kFused) {
    if (e.in0 != k0.in_features || e.h != k0.out_features || e.out != k1.out_features) continue;
    if (e.NB != k0.num_logistic || e.SO != k0.spline_order || e.NG != NG) continue;
    if (e.ferro != (f->ferro != nullptr)) continue;
    if (f->ferro) {
      if (f->ferro[0].num_basis != e.K || f->ferro[1].num_basis != e.K) continue;
      if (f->ferro[0].branch_sign || f->ferro[1].branch_sign) continue;  // general-sign path: generic
    }
    return &e;
  }
  return nullptr;
}

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
  float acc = 0.f;
  for (int i = 0; i < in; ++i) {
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
      acc += bv * fl.coef[e];
    }
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
  } else {
    r = yv + dt * k1[t];
  }
  out[t] = r;
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
static inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

extern "C" {

const char* fetode_last_error(void) { return g_last_error.c_str(); }
int fetode_abi_version(void) { return FETODE_ABI_VERSION; }

int32_t fetode_state_width(const fetode_field_t* f) {
  if (!f || !f->ferro) return 0;
  int32_t w = 0;
  for (int l = 0; l < f->n_layers; ++l) w += f->ferro[l].in_dim;
  return w;
}

int64_t fetode_plan_bytes(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return -1;
  int64_t base = 0;
  for (int l = 0; l < f->n_layers; ++l) {
    LayerPlan p;
    layer_plan(f->kan[l], f->ferro ? &f->ferro[l] : nullptr, base, &p);
    base = p.end;
  }
  return base * (int64_t)sizeof(float);
}

int fetode_plan_build(const fetode_field_t* f, void* plan, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  if (!plan) return set_err(FETODE_EINVAL, "plan is NULL");
  int64_t base = 0;
  for (int l = 0; l < f->n_layers; ++l) {
    LayerPlan p;
    const fetode_ferro_t* fl = f->ferro ? &f->ferro[l] : nullptr;
    layer_plan(f->kan[l], fl, base, &p);
    int64_t n = std::max<int64_t>({(int64_t)p.out * p.in * std::max(p.K, 1), (int64_t)p.out * p.in * p.NF,
                                   (int64_t)p.in * p.SO * (p.NG - 1), (int64_t)p.in * p.NG,
                                   (int64_t)p.in * std::max(p.NB, 1), (int64_t)p.out});
    fetode_ferro_t dummy;
    memset(&dummy, 0, sizeof(dummy));
    hipLaunchKernelGGL(plan_build_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, p,
                       f->kan[l], fl ? *fl : dummy, fl ? 1 : 0, (float*)plan);
    LAUNCH_CHECK();
    base = p.end;
  }
  return FETODE_OK;
}

int fetode_fused_supported(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return 0;
  return find_fused(f) != nullptr;
}

static int launch_fused(const fetode_field_t* f, FusedArgs& a, void* stream) {
  const FusedEntry* e = find_fused(f);
  if (!e) return set_err(FETODE_EUNSUPPORTED, "no fused kernel for this field shape");
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  const int tpb = 256 / 32;
  hipLaunchKernelGGL(e->fn, dim3(nblk(a.B, tpb)), dim3(256), 0, (hipStream_t)stream, a);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_field_forward(const fetode_field_t* f, const void* plan, const float* x, int64_t B,
                         float* state, uint32_t init_mask, float* out, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!plan || !x || !out || (f->ferro && !state)) return set_err(FETODE_EINVAL, "null pointer");
  FusedArgs a;
  memset(&a, 0, sizeof(a));
  a.plan = (const float*)plan;
  a.y0 = x;
  a.B = B;
  a.state = state;
  a.init_mask = init_mask;
  a.single_eval = 1;
  a.eval_out = out;
  return launch_fused(f, a, stream);
}

int fetode_integrate_fixed(const fetode_field_t* f, const void* plan, int32_t method, const float* y0,
                           int64_t B, const float* step_coef, int32_t n_steps, const int32_t* out_step,
                           const int32_t* out_mode, const float* out_slope, int32_t T,
                           float* solution, float* state, uint32_t init_mask, float* ckpt,
                           void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  if (method < FETODE_EULER || method > FETODE_RK4_CLASSIC)
    return set_err(FETODE_EINVAL, "unknown method %d", method);
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!plan || !y0 || !solution || (n_steps > 0 && (!step_coef || !out_step || !out_mode || !out_slope)) ||
      (f->ferro && !state))
    return set_err(FETODE_EINVAL, "null pointer");
  if (f->kan[0].in_features != f->kan[f->n_layers - 1].out_features)
    return set_err(FETODE_EINVAL, "field is not R^D -> R^D");
  FusedArgs a;
  memset(&a, 0, sizeof(a));
  a.plan = (const float*)plan;
  a.method = method;
  a.y0 = y0;
  a.B = B;
  a.step_coef = step_coef;
  a.n_steps = n_steps;
  a.out_step = out_step;
  a.out_mode = out_mode;
  a.out_slope = out_slope;
  a.T = T;
  a.solution = solution;
  a.state = state;
  a.init_mask = init_mask;
  a.ckpt = ckpt;
  return launch_fused(f, a, stream);
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
  if (method == FETODE_RK4 && ((stage >= 2 && !k2) || (stage >= 3 && !k3) || (stage >= 4 && !k4)))
    return set_err(FETODE_EINVAL, "rk4 stage %d: missing k", stage);
  hipLaunchKernelGGL(rk_combine_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, method,
                     stage, y, k1, k2, k3, k4, dt, out, n);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"
