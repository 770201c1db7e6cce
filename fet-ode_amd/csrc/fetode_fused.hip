// fetode_fused.hip — the single-launch fixed-grid integrator of a depth-2 KAN / KAN-FET field.
//
// One launch integrates the whole t-grid (torchdiffeq FixedGridODESolver.integrate): every RK
// stage evaluation of the field, the hysteresis state updates in exact call order
// (ferro_class.py:409), the stage combines (rk_common.rk4_alt_step_func op order) and the
// output writes.  Nothing but y0, the parameters and the outputs touch HBM.
//
// Mapping.  A trajectory is owned by a group of LPT = 32 lanes (2 per wave).
// Per field evaluation and per layer:
//   phase A  per-input features into LDS: logistic basis (one (i,j) job per lane), and per input
//            SiLU, the knot interval m and local coordinate u of x, the hysteresis gate
//            w = -2(1-alpha)(1-sigmoid(gs*(x-prev))) and exp(gs*x); prev_x <- x.
//   phase B  lane (o, c) owns a fixed slice of the layer's (input, basis) Ferro elements and of
//            its feature weights, kept in VGPRs for the whole solve; the spline edge (o, i) is a
//            cubic in u per knot interval, read as one float4 from the LDS table; partial sums
//            are reduced over the C lanes of an output with cross-lane shuffles.
// The stage combine runs on lanes d < D, in registers.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fetode_common.h"

using namespace fetode;

#ifdef FETODE_ISA_MARKERS
#define FETODE_MARK(s) asm volatile("; MARK " s ::: "memory")
#else
#define FETODE_MARK(s)
#endif

namespace {

template <int IN_, int OUT_, int K_, int NB_, int NG_, int LPT_>
struct LS {
  static constexpr int IN = IN_, OUT = OUT_, K = K_, NB = NB_, NG = NG_, LPT = LPT_;
  static constexpr int NI = NG - 1;           // knot intervals
  static constexpr int NFL = 1 + NB;          // LDS features per input: SiLU + logistic
  static constexpr int C = LPT / OUT;         // lanes (chunks) per output
  static constexpr int NP = IN * K;           // Ferro (input, basis) pairs
  static constexpr int NQ = IN * NFL;         // feature weights per output
  static constexpr int EPL = K > 0 ? (NP + C - 1) / C : 0;
  static constexpr int FPL = (NQ + C - 1) / C;
  static constexpr int SPL = (IN + C - 1) / C;
  static constexpr int LJ = NB > 0 ? (IN * NB + LPT - 1) / LPT : 0;
  static constexpr int SPT = OUT * IN * (NI + 1) * 4;  // spline table floats
  static_assert(C >= 1, "out_features must be <= lanes per trajectory");
};

template <class S>
struct Regs {  // per-lane register-resident slice of one layer
  float ep[S::EPL > 0 ? S::EPL : 1];    // exp2(GEc) (factored gate) or GEc
  float k2[S::EPL > 0 ? S::EPL : 1], k2Ec[S::EPL > 0 ? S::EPL : 1], CPs2[S::EPL > 0 ? S::EPL : 1];
  float fw[S::FPL];
  float lna[S::LJ > 0 ? S::LJ : 1], lab[S::LJ > 0 ? S::LJ : 1];
  int o, c;
  bool active;

  __device__ void load(const float* __restrict__ plan, const LayerPlan& P, int lane, bool factored) {
    o = lane / S::C;
    c = lane % S::C;
    active = lane < S::C * S::OUT;
    const int oo = active ? o : 0;
#pragma unroll
    for (int r = 0; r < S::EPL; ++r) {
      const int p = c + S::C * r;
      const bool ok = active && p < S::NP;
      const int64_t idx = (int64_t)oo * S::NP + (ok ? p : 0);
      const float gec = ok ? plan[P.fe_GEc + idx] : 0.f;
      ep[r] = factored ? ex2(gec) : gec;
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
      const int job = lane + S::LPT * r;
      const bool ok = job < S::IN * S::NB;
      lna[r] = ok ? plan[P.lg + 2 * job] : 0.f;
      lab[r] = ok ? plan[P.lg + 2 * job + 1] : 0.f;
    }
  }
};

template <class S>
struct TrajLayer {        // per-trajectory LDS scratch of one layer
  float F[S::IN * S::NFL];  // SiLU, logistic features
  float G[S::IN * 4];       // x, w (gate factor), exp(gs x), u (spline coordinate)
  int M[S::IN];             // knot interval (NI = outside / non-finite -> zero table row)
  float prev[S::IN];        // compact prev_x
};

template <class S>
struct WgLayer {          // per-workgroup LDS copy of the shared tables of one layer
  float knots[S::IN * S::NG];
  float rh[S::IN * S::NI];
  float cst[S::OUT];
};

// sum over the C consecutive lanes of an output; valid on lane c == 0 (and on all for pow2 C)
template <int C>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr ((C & (C - 1)) == 0) {
#pragma unroll
    for (int k = C / 2; k >= 1; k >>= 1) v += __shfl_xor(v, k);
    return v;
  } else {
    float s = v;
#pragma unroll
    for (int d = 1; d < C; ++d) s += __shfl_down(v, d);
    return s;
  }
}

template <class S, bool FERRO>
__device__ __forceinline__ void phase_A(const float* xin, TrajLayer<S>& L, const WgLayer<S>& W, const Regs<S>& R,
                                        const LayerPlan& P, int lane, bool reinit) {
  // logistic basis phi'_{ij} = 1/(1+exp(-a(x-b)))  (efficientkan.py:24; the 2 is in the weights)
#pragma unroll
  for (int r = 0; r < S::LJ; ++r) {
    const int job = lane + S::LPT * r;
    if (job < S::IN * S::NB) {
      const int i = job / S::NB, j = job % S::NB;
      L.F[i * S::NFL + 1 + j] = rcp(1.0f + ex2(ffma(R.lna[r], xin[i], R.lab[r])));
    }
  }
  for (int i = lane; i < S::IN; i += S::LPT) {
    const float x = xin[i];
    L.F[i * S::NFL] = silu(x);
    // knot interval: half-open [g_m, g_{m+1}) as the order-0 indicator (efficientkan.py:122)
    const float* g = &W.knots[i * S::NG];
    int m = -1;
#pragma unroll
    for (int j = 0; j < S::NG; ++j) m += (x >= g[j]) ? 1 : 0;
    float u;
    if (!__builtin_isfinite(x)) {
      m = S::NI;
      u = __builtin_nanf("");  // the reference's bases are NaN for +-inf / NaN inputs
    } else if (m < 0 || m >= S::NI) {
      m = S::NI;               // zero row of the table: all bases vanish outside the grid
      u = 0.f;
    } else {
      u = (x - g[m]) * W.rh[i * S::NI + m];
    }
    L.M[i] = m;
    L.G[4 * i + 3] = u;
    if constexpr (FERRO) {
      const float pv = reinit ? x : L.prev[i];
      const float dx = x - pv;
      // is_moving_up = sigmoid(gate_slope*dx) (ferro_class.py:387); w = -2(1-alpha)(1-u)
      const float up = rcp(1.0f + ex2(-P.gsl2e * dx));
      L.G[4 * i + 0] = x;
      L.G[4 * i + 1] = P.wc * (1.0f - up);
      L.G[4 * i + 2] = ex2(P.gsl2e * x);
      L.prev[i] = x;  // ferro_class.py:409
    }
  }
}

// returns the output value on lanes with c == 0 (garbage elsewhere)
template <class S, bool FERRO, bool FACT>
__device__ __forceinline__ float phase_B(const TrajLayer<S>& L, const float* __restrict__ sp_lds,
                                         const Regs<S>& R, float gsl2e) {
  float acc = 0.f;
  if (R.active) {
    if constexpr (FERRO) {
      // Ferro element (ferro_class.py:384-414) with branch_sign == 1 (never written, F8):
      //   sl = (1-u) sigmoid(gs(-x-Ec)),  m = alpha + (1-alpha)(1-2 sl) = 1 + w s
      //   coef (Ps tanh(k(x+Ec m)) + bias), tanh(z) = 1 - 2/(1+exp(2z)); sum coef*bias is folded
      //   into the output constant.  The centred term coef*Ps*tanh keeps partial sums as small
      //   as the reference's (a folded coef*(Ps+bias) constant costs ~10x more rounding).
#pragma unroll
      for (int r = 0; r < S::EPL; ++r) {
        const int p = R.c + S::C * r;
        if (p < S::NP) {
          const int i = p / S::K;
          const float x = L.G[4 * i], w = L.G[4 * i + 1];
          float s;
          if constexpr (FACT) s = rcp(1.0f + L.G[4 * i + 2] * R.ep[r]);
          else s = rcp(1.0f + ex2(ffma(gsl2e, x, R.ep[r])));
          const float m = ffma(w, s, 1.0f);
          const float z = ffma(R.k2Ec[r], m, R.k2[r] * x);
          const float th = ffma(-2.0f, rcp(1.0f + ex2(z)), 1.0f);
          acc = ffma(R.CPs2[r], th, acc);
        }
      }
    }
#pragma unroll
    for (int f = 0; f < S::FPL; ++f) {
      const int q = R.c + S::C * f;
      if (q < S::NQ) acc = ffma(R.fw[f], L.F[q], acc);
    }
#pragma unroll
    for (int r = 0; r < S::SPL; ++r) {
      const int i = R.c + S::C * r;
      if (i < S::IN) {
        const float u = L.G[4 * i + 3];
        const float4 cf = *reinterpret_cast<const float4*>(
            &sp_lds[((R.o * S::IN + i) * (S::NI + 1) + L.M[i]) * 4]);
        acc += ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x);
      }
    }
  }
  return group_sum<S::C>(acc);
}

struct FusedArgs {
  const float* plan;
  LayerPlan P0, P1;
  int32_t method;
  const float* y0;
  int64_t B;
  const float* step_coef;  // n_steps x 4 : dt, 0.5dt, dt/6, 0 (time dtype -> fp32)
  int32_t n_steps;
  const int32_t* out_step;
  const int32_t* out_mode;
  const float* out_slope;
  int32_t T;
  float* solution;
  float* state;
  uint32_t init_mask;
  float* ckpt;
  int32_t single_eval;  // 1: eval_out = field(y0) once (fetode_field_forward)
  float* eval_out;
};

template <int IN0, int H, int OUT, int K, int NB, int NG, bool FERRO, int LPT, int NT>
__global__ __launch_bounds__(NT) void fused_integrate_kernel(FusedArgs a) {
  using S0 = LS<IN0, H, FERRO ? K : 0, NB, NG, LPT>;
  using S1 = LS<H, OUT, FERRO ? K : 0, NB, NG, LPT>;
  constexpr int TPB = NT / LPT;  // trajectories per block
  constexpr int D = IN0;
  static_assert(IN0 == OUT, "ODE field must map R^D -> R^D");
  static_assert(D <= LPT && H <= LPT, "dims exceed lanes per trajectory");

  struct Traj {
    float x0[IN0];
    float h[H];
    float kout[OUT];
    TrajLayer<S0> L0;
    TrajLayer<S1> L1;
  };
  __shared__ __attribute__((aligned(16))) float s_sp0[S0::SPT];
  __shared__ __attribute__((aligned(16))) float s_sp1[S1::SPT];
  __shared__ WgLayer<S0> s_w0;
  __shared__ WgLayer<S1> s_w1;
  __shared__ Traj s_traj[TPB];

  const int tid = threadIdx.x;
  const int g = tid / LPT, lane = tid % LPT;
  const int64_t b = (int64_t)blockIdx.x * TPB + g;
  const bool valid = b < a.B;
  Traj& T = s_traj[g];

  // stage the shared tables
  for (int i = tid; i < S0::SPT; i += NT) s_sp0[i] = a.plan[a.P0.sp + i];
  for (int i = tid; i < S1::SPT; i += NT) s_sp1[i] = a.plan[a.P1.sp + i];
  for (int i = tid; i < IN0 * NG; i += NT) s_w0.knots[i] = a.plan[a.P0.knots + i];
  for (int i = tid; i < H * NG; i += NT) s_w1.knots[i] = a.plan[a.P1.knots + i];
  for (int i = tid; i < IN0 * S0::NI; i += NT) s_w0.rh[i] = a.plan[a.P0.rh + i];
  for (int i = tid; i < H * S1::NI; i += NT) s_w1.rh[i] = a.plan[a.P1.rh + i];
  for (int i = tid; i < H; i += NT) s_w0.cst[i] = a.plan[a.P0.fconst + i];
  for (int i = tid; i < OUT; i += NT) s_w1.cst[i] = a.plan[a.P1.fconst + i];

  // factored gate exp only where it is exact in fp32 (fetode_common.h kFactorLimit)
  const bool fact = FERRO && a.plan[a.P0.flag] <= kFactorLimit && a.plan[a.P1.flag] <= kFactorLimit;
  Regs<S0> R0;
  Regs<S1> R1;
  R0.load(a.plan, a.P0, lane, fact);
  R1.load(a.plan, a.P1, lane, fact);

  constexpr int SW = FERRO ? IN0 + H : 0;  // state width
  if (FERRO) {
    for (int i = lane; i < IN0; i += LPT) T.L0.prev[i] = valid ? a.state[b * SW + i] : 0.f;
    for (int i = lane; i < H; i += LPT) T.L1.prev[i] = valid ? a.state[b * SW + IN0 + i] : 0.f;
  }
  bool re0 = FERRO && (a.init_mask & 1u), re1 = FERRO && (a.init_mask & 2u);

  const int d = lane;
  const bool own = d < D;
  float y = (own && valid) ? a.y0[b * D + d] : 0.f;
  if (!a.single_eval && own && valid) a.solution[b * D + d] = y;  // solution[0] = y0

  auto eval_body = [&](float xin, auto fact_tag) __attribute__((always_inline)) -> float {
    constexpr bool F_ = decltype(fact_tag)::value;
    if (own) T.x0[d] = xin;
    __syncthreads();
    FETODE_MARK("A0");
    phase_A<S0, FERRO>(T.x0, T.L0, s_w0, R0, a.P0, lane, re0);
    re0 = false;
    __syncthreads();
    FETODE_MARK("B0");
    const float v0 = phase_B<S0, FERRO, F_>(T.L0, s_sp0, R0, a.P0.gsl2e);
    if (R0.active && R0.c == 0) T.h[R0.o] = v0 + s_w0.cst[R0.o];
    __syncthreads();
    FETODE_MARK("A1");
    phase_A<S1, FERRO>(T.h, T.L1, s_w1, R1, a.P1, lane, re1);
    re1 = false;
    __syncthreads();
    FETODE_MARK("B1");
    const float v1 = phase_B<S1, FERRO, F_>(T.L1, s_sp1, R1, a.P1.gsl2e);
    if (R1.active && R1.c == 0) T.kout[R1.o] = v1 + s_w1.cst[R1.o];
    __syncthreads();
    FETODE_MARK("END");
    return own ? T.kout[d] : 0.f;
  };
  auto eval = [&](float xin) __attribute__((always_inline)) -> float {
    if (fact) return eval_body(xin, std::integral_constant<bool, true>{});
    return eval_body(xin, std::integral_constant<bool, false>{});
  };

  if (a.single_eval) {
    const float f = eval(y);
    if (own && valid) a.eval_out[b * OUT + d] = f;
  } else {
    const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4
                   : a.method == FETODE_MIDPOINT ? 2 : 1;
    const float third = 1.0f / 3.0f;
    int jj = 1;
    for (int s = 0; s < a.n_steps; ++s) {
      const float dt = a.step_coef[4 * s + 0], hh = a.step_coef[4 * s + 1], h6 = a.step_coef[4 * s + 2];
      if (a.ckpt && valid) {  // prev[i] is written and read by the same lane (i % LPT)
        const int64_t W = D + SW;
        float* ck = a.ckpt + ((int64_t)s * a.B + b) * W;
        if (own) ck[d] = y;
        if (FERRO) {
          for (int i = lane; i < IN0; i += LPT) ck[D + i] = T.L0.prev[i];
          for (int i = lane; i < H; i += LPT) ck[D + IN0 + i] = T.L1.prev[i];
        }
      }
      float k1 = 0.f, k2 = 0.f, k3 = 0.f, k4 = 0.f;
      for (int st = 0; st < ns; ++st) {
        float xin = y;
        if (a.method == FETODE_RK4) {
          // rk_common.rk4_alt_step_func, exact op order (3/8 rule)
          if (st == 1) xin = y + (dt * k1) * third;
          else if (st == 2) xin = y + dt * (k2 - k1 * third);
          else if (st == 3) xin = y + dt * ((k1 - k2) + k3);
        } else if (a.method == FETODE_RK4_CLASSIC) {
          // train_kan_fet_ett.py:72-75 / train_ecg_kan_fet_nn_ode.py:699-702
          if (st == 1) xin = y + hh * k1;
          else if (st == 2) xin = y + hh * k2;
          else if (st == 3) xin = y + dt * k3;
        } else if (a.method == FETODE_MIDPOINT) {
          if (st == 1) xin = y + k1 * hh;  // fixed_grid.Midpoint: y0 + f0 * half_dt
        }
        const float kk = eval(xin);
        if (st == 0) k1 = kk;
        else if (st == 1) k2 = kk;
        else if (st == 2) k3 = kk;
        else k4 = kk;
      }
      float y1;
      if (a.method == FETODE_RK4) y1 = y + (((k1 + 3.0f * (k2 + k3)) + k4) * dt) * 0.125f;
      else if (a.method == FETODE_RK4_CLASSIC) y1 = y + h6 * (((k1 + 2.0f * k2) + 2.0f * k3) + k4);
      else if (a.method == FETODE_MIDPOINT) y1 = y + dt * k2;
      else y1 = y + dt * k1;
      while (jj < a.T && a.out_step[jj] == s) {
        const int mode = a.out_mode[jj];
        const float v = mode == 0 ? y : (mode == 1 ? y1 : y + a.out_slope[jj] * (y1 - y));
        if (own && valid) a.solution[((int64_t)jj * a.B + b) * D + d] = v;
        ++jj;
      }
      y = y1;
    }
  }
  if (FERRO && valid) {
    for (int i = lane; i < IN0; i += LPT) a.state[b * SW + i] = T.L0.prev[i];
    for (int i = lane; i < H; i += LPT) a.state[b * SW + IN0 + i] = T.L1.prev[i];
  }
}

typedef void (*fused_fn)(FusedArgs);
struct FusedEntry {
  int in0, h, out, K, NB, NG;
  bool ferro;
  fused_fn fn;
  int nt, lpt;
};
#define FUSED(IN0, H, OUT, K, NB, NG, FE, LPT, NT) \
  {IN0, H, OUT, K, NB, NG, FE, fused_integrate_kernel<IN0, H, OUT, K, NB, NG, FE, LPT, NT>, NT, LPT}
const FusedEntry kFused[] = {
    // LV KAN-FET [2,10,2], K=10 (train_kanfet_node_predprey.py:146)
    FUSED(2, 10, 2, 10, 10, 12, true, 32, 64),
    FUSED(2, 10, 2, 10, 10, 12, true, 32, 256),
    FUSED(2, 10, 2, 10, 10, 12, true, 64, 64),
    FUSED(2, 10, 2, 10, 10, 12, true, 64, 256),
    // LV KAN [2,10,2] (predator_prey.py:101)
    FUSED(2, 10, 2, 1, 10, 12, false, 32, 64),
    FUSED(2, 10, 2, 1, 10, 12, false, 32, 256),
    FUSED(2, 10, 2, 1, 10, 12, false, 64, 64),
    FUSED(2, 10, 2, 1, 10, 12, false, 64, 256),
};

// workgroup size: 64 threads (one wave, 2 trajectories; its barriers cost almost nothing)
// unless FETODE_FUSED_NT says otherwise (measured: 64 >= 256 at B=4096 and 1.11x at B=65536)
int preferred_nt() {
  static int nt = [] {
    const char* e = getenv("FETODE_FUSED_NT");
    return e ? atoi(e) : 64;
  }();
  return nt;
}
// lanes per trajectory: 32 (2 trajectories per wave) unless FETODE_FUSED_LPT says otherwise
int preferred_lpt() {
  static int v = [] {
    const char* e = getenv("FETODE_FUSED_LPT");
    return e ? atoi(e) : 32;
  }();
  return v;
}

const FusedEntry* find_fused(const fetode_field_t* f) {
  if (f->n_layers != 2) return nullptr;
  const fetode_kanlinear_t &k0 = f->kan[0], &k1 = f->kan[1];
  if (k0.grid_size != k1.grid_size || k0.spline_order != k1.spline_order ||
      k0.num_logistic != k1.num_logistic)
    return nullptr;
  const int NG = k0.grid_size + 2 * k0.spline_order + 1;
  for (const FusedEntry& e : kFused) {
    if (e.in0 != k0.in_features || e.h != k0.out_features || e.out != k1.out_features) continue;
    if (e.NB != k0.num_logistic || e.NG != NG) continue;
    if (e.ferro != (f->ferro != nullptr)) continue;
    if (e.nt != preferred_nt() || e.lpt != preferred_lpt()) continue;
    if (f->ferro) {
      if (f->ferro[0].num_basis != e.K || f->ferro[1].num_basis != e.K) continue;
      if (f->ferro[0].branch_sign || f->ferro[1].branch_sign) continue;  // general sign: generic path
    }
    return &e;
  }
  return nullptr;
}

int launch_fused(const fetode_field_t* f, FusedArgs& a, void* stream) {
  const FusedEntry* e = find_fused(f);
  if (!e) return set_err(FETODE_EUNSUPPORTED, "no fused kernel for this field shape");
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  const int tpb = e->nt / e->lpt;
  hipLaunchKernelGGL(e->fn, dim3(nblk(a.B, tpb)), dim3(e->nt), 0, (hipStream_t)stream, a);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // namespace

extern "C" {

int fetode_fused_supported(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return 0;
  return find_fused(f) != nullptr;
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
                           const int32_t* out_mode, const float* out_slope, int32_t T, float* solution,
                           float* state, uint32_t init_mask, float* ckpt, void* stream) {
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

}  // extern "C"
