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

#include <cstdlib>

#include "fetode_common.h"
#include "fetode_fieldn_plan.h"

using namespace fetode;

namespace {

#include "fetode_gridsum.h"

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
// interval, Ferro elements (o, i, k) with hysteresis input pv — differentiated in x.  IMG: the
// plan's lane-contiguous LDS image (fetode_fieldn_plan.h), layer L (lanes: layer 0's outputs,
// layer 1's inputs)
template <bool FERRO, int UNR = 1, bool IMG = false, int L = 0>
__device__ float fb_vjp_input(const float* __restrict__ plan, const LayerPlan& P, int i, float x, float pv,
                              const float* go, int o0, int no) {
  using X = FnIdx<IMG, L>;
  const int st = X::stride(P);
  const float sx = fb_sig(-x * FETODE_LOG2E);
  const float dsx = sx * ffma(x, 1.0f - sx, 1.0f);  // SiLU'
  // knot interval as fn_interval; off the grid: the plan's zero row, u = 0 (NaN for non-finite x)
  const float* g = plan + X::knot(P, i, 0);
  const int gst = X::knot_stride(P);
  int m = -1;
  for (int j = 0; j < P.NG; ++j) m += x >= g[j * gst] ? 1 : 0;
  const bool fin = __builtin_isfinite(x);
  const int mfix = ((unsigned)m < (unsigned)P.NI && fin) ? m : P.NI;
  const float rhm = mfix < P.NI ? plan[X::rh(P, i, mfix)] : 0.f;
  const float u = mfix < P.NI ? (x - g[mfix * gst]) * rhm : (fin ? 0.0f : __builtin_nanf(""));
  float acc = 0.f;
  for (int oo = 0; oo < no; ++oo) {
    const int o = o0 + oo;
    const float* kw = plan + X::row(P, P.kw, o, i, P.NFL);
    const float4 cf = *reinterpret_cast<const float4*>(plan + X::sp(P, o, i, mfix));
    const float dsp = ffma(u, ffma(3.0f * u, cf.w, 2.0f * cf.z), cf.y) * rhm;
    acc = ffma(go[oo], ffma(kw[0], dsx, dsp), acc);
  }
  // logistic branch: d/dx 1/(1 + 2^(a' x + b')) = -ln2 a' s (1 - s)
  // UNR: as fn_edge — overlap the independent exp2 / rcp chains of consecutive basis functions
#pragma unroll UNR
  for (int j = 0; j < P.NB; ++j) {
    const float la = plan[X::lg(P, i, j, 0)];
    const float s = fb_sig(ffma(la, x, plan[X::lg(P, i, j, 1)]));
    const float dj = (-kLn2 * la) * (s * (1.0f - s));
    float wsum = 0.f;
    for (int oo = 0; oo < no; ++oo) wsum = ffma(go[oo], plan[X::row(P, P.kw, o0 + oo, i, P.NFL) + (1 + j) * st], wsum);
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
      const int64_t e0 = X::row(P, 0, o0 + oo, i, P.K);
      const float* GEc = plan + P.fe_GEc + e0;
      const float* k2 = plan + P.fe_k2 + e0;
      const float* kE = plan + P.fe_k2Ec + e0;
      const float* cp = plan + P.fe_CPs2 + e0;
      float d = 0.f;
#pragma unroll UNR
      for (int k = 0; k < P.K; ++k) {
        const float s = rcp(ex2(ffma(P.gsl2e, x, GEc[k * st])) + 1.0f);
        const float mm = ffma(w, s, 1.0f);
        const float z = ffma(kE[k * st], mm, k2[k * st] * x);
        const float th = ffma(rcp(ex2(z) + 1.0f), -2.0f, 1.0f);
        const float dm = gw * s * (upp1 - s);
        d = ffma(cp[k * st] * ffma(-th, th, 1.0f), ffma(kE[k * st], dm, k2[k * st]), d);
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

// LDSP: the plan of both layers staged in LDS once per workgroup (as fieldn_kernel<.., LDSP>)
constexpr int kFbWavesL = 8;
constexpr int kFbMaxT = 8;  // trajectories per wave at most
// unit lanes U = the smallest power of two >= max(H, D, 64 / kFbMaxT) and split factor SF as
// fieldn_kernel (fn_unit_lanes / fn_split): split group sg takes half the layer-1 outputs (a
// contiguous half) and the layer-0 inputs i = sg (mod 2)
__host__ __device__ inline int fb_unit_lanes(int D, int H) {
  int hp = 64 / kFbMaxT;
  while (hp < H || hp < D) hp <<= 1;
  return hp < 64 ? hp : 64;
}
__host__ __device__ inline int fb_split(int D, int H) { return (fb_unit_lanes(D, H) <= 32 && D >= 2) ? 2 : 1; }
__host__ __device__ inline int fb_lanes_per_traj(int D, int H) { return fb_unit_lanes(D, H) * fb_split(D, H); }
constexpr int64_t kFbLdsMax = 78 * 1024;
template <bool FERRO, bool LDSP = false>
__global__ __launch_bounds__(LDSP ? 64 * kFbWavesL : 64 * kFbWaves) void fieldn_adj_kernel(FbArgs a) {
  constexpr int NW = LDSP ? kFbWavesL : kFbWaves;
  // several trajectories per wave, as fieldn_kernel: lane = (slot t, unit o), HP lanes per slot
  __shared__ float s_x[NW][kFbMaxT][kFbMaxD], s_p[NW][kFbMaxT][kFbMaxD], s_gk[NW][kFbMaxT][kFbMaxD];
  __shared__ float s_ak[NW][kFbMaxT][4][kFbMaxD], s_ac[NW][4][3];
  extern __shared__ float s_plan[];
  if constexpr (LDSP) {
    fn_stage_image(s_plan, a.plan, a.P0, a.P1);  // the lane-contiguous image (fetode_fieldn_plan.h)
    __syncthreads();
  }
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const LayerPlan& P0 = a.P0;
  const LayerPlan& P1 = a.P1;
  const int D = P0.in, H = P0.out;
  const int U = fb_unit_lanes(D, H), SF = fb_split(D, H), HP = U * SF, TPW = 64 / HP;
  const int t = lane / HP, sg = (lane & (HP - 1)) / U, o = lane & (U - 1);
  const bool own = sg == 0;  // the group that owns the trajectory's adjoint state and writes
  const int dlo = SF == 2 ? (sg ? (D + 1) / 2 : 0) : 0, dn = SF == 2 ? (sg ? D / 2 : (D + 1) / 2) : D;
  const int64_t bw = ((int64_t)blockIdx.x * NW + wid) * TPW;
  if (bw >= a.B) return;  // whole waves only; no workgroup barriers below
  const int64_t b = bw + t;
  const bool live = b < a.B;  // a missing slot runs on zeros (its lanes still take part in the sums)
  const int64_t bi = live ? b : bw;
  const float* __restrict__ plan = LDSP ? s_plan : a.plan;
  const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  const int64_t n_ev = (int64_t)a.n_steps * ns;
  const float* X = a.tape;
  const float* Hh = a.tape + n_ev * a.B * D;
  float* GK = a.gadj;
  float* GH = a.gadj + n_ev * a.B * D;
  float* xs = s_x[wid][t];
  float* ps = s_p[wid][t];
  float* gk = s_gk[wid][t];
  float(&ak)[4][kFbMaxD] = s_ak[wid][t];
  float(&acs)[4][3] = s_ac[wid];
  const bool dl = own && o < D, hl = o < H;
  float ay1 = 0.f, ay = 0.f;  // adjoint of y at the end of the current step (lanes < D)
  int jj = a.T - 1;
  for (int s = a.n_steps - 1; s >= 0; --s) {
    float bc[4], ac[4][3];
    fb_coefs(a.method, a.step_coef[4 * s], a.step_coef[4 * s + 1], a.step_coef[4 * s + 2], bc, ac);
    float ay0x = 0.f;  // outputs produced in this step (y at step start, end, or interpolated)
    for (; jj >= 1 && a.out_step[jj] == s; --jj) {
      if (dl) {
        const float g = live ? a.gsol[((int64_t)jj * a.B + bi) * D + o] : 0.f;
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
      for (int j = 0; j < ns; ++j) ak[j][o] = bc[j] * ay1;
      ay = ay1 + ay0x;
    }
    if (lane == 0)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) acs[i][j] = ac[i][j];
    for (int st = ns - 1; st >= 0; --st) {
      const int64_t ev = (int64_t)s * ns + st;
      if (dl) {
        const float x = live ? X[(ev * a.B + bi) * D + o] : 0.f;
        xs[o] = x;
        ps[o] = !live ? 0.f
                : ev > 0 ? X[((ev - 1) * a.B + bi) * D + o]
                         : ((a.init_mask & 1u) ? x : (FERRO ? a.state0[bi * D + o] : 0.f));
        gk[o] = ak[st][o];
      }
      float h = 0.f, ph = 0.f;
      if (hl && live) {
        h = Hh[(ev * a.B + bi) * H + o];
        ph = ev > 0 ? Hh[((ev - 1) * a.B + bi) * H + o]
                    : ((a.init_mask & 2u) ? h : (FERRO ? a.state0[a.B * D + bi * H + o] : 0.f));
      }
      fb_wsync();
      // layer 1 (h -> k): d loss / d h_o on lane o
      // (split: each group its half of the outputs, then the two halves' sum on both)
      float gh = hl ? fb_vjp_input<FERRO, 4, LDSP, 1>(plan, P1, o, h, ph, gk + dlo, dlo, dn) : 0.f;
      if (SF == 2) gh += __shfl_xor(gh, U);
      if (live && dl) GK[(ev * a.B + b) * D + o] = gk[o];
      if (live && own && hl) GH[(ev * a.B + b) * H + o] = gh;
      // layer 0 (x -> h): d loss / d x_i = sum over the lanes o of gh_o d edge(o, i) / d x_i
      float gx = 0.f;
      for (int i = sg; i < D; i += SF) {  // group sg: the inputs i = sg (mod SF)
        const float one = 1.0f;
        const float c = hl ? gh * fb_vjp_input<FERRO, 4, LDSP, 0>(plan, P0, i, xs[i], ps[i], &one, o, 1) : 0.f;
        float sum = c;
        for (int m = U >> 1; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);  // within the group's lanes
        if (o == i) gx = sum;
        if (SF == 2) {  // the odd input's sum to its owner lane in group 0
          const float oth = __shfl_xor(sum, U);
          if (o == i + 1) gx = oth;
        }
      }
      if (dl) {
        ay += gx;
        for (int j = 0; j < st; ++j) ak[j][o] = ffma(acs[st][j], gx, ak[j][o]);
      }
      fb_wsync();
    }
    ay1 = ay;
  }
  if (live && dl && a.gy0) a.gy0[b * D + o] = ay1 + a.gsol[b * D + o];  // solution[0] = y0
}

// =============================================================================================
// The reverse sweep of fieldn's taped resident dopri5 solve (fieldn_kernel<FERRO, DOPRI, TAPE>):
// loss.backward() through odeint(..., method="dopri5") for these widths.  The control adjoint is
// the [2, 10, 2] sweep's (fetode_bwd.hip dopri_bwd_kernel: the step-size control, the error norm
// with one grid sum per attempt, the interpolant, _select_initial_step), one trajectory per wave;
// the per-evaluation VJP is fieldn_adj_kernel's, and every evaluation's layer inputs and output /
// hidden adjoints are written as planes for the row-batched parameter VJPs afterwards.
// =============================================================================================
struct FdArgs {
  FbArgs b;             // plan, layers, B, T, gsol, tape rows (n_ev, B, 2 D + H), state0, init_mask, gy0
  const double* att;    // (n_att, 4): t0, dt, error ratio, accepted
  int32_t n_att, n_ev, base;
  const double* t;
  const double* init_rec;
  float beta[6][6], cerr[7], cmid[7];
  float rtol, atol;
  double safety, ifactor, dfactor, min_step, max_step, n_el;
  DopriParams gp;
  int32_t* status;
  float *Xc, *Hc;       // planes (n_ev, B, D) / (n_ev, B, H): the layer inputs, for the parameter VJPs
};

template <bool FERRO>
__global__ __launch_bounds__(64 * kFbWaves) void fieldn_dopri_bwd_kernel(FdArgs da) {
  const FbArgs& a = da.b;
  __shared__ float s_x[kFbWaves][kFbMaxD], s_p[kFbWaves][kFbMaxD], s_g1[kFbWaves][kFbMaxD], s_gx[kFbWaves][kFbMaxD];
  __shared__ float s_k[kFbWaves][8][kFbMaxD], s_kb[kFbWaves][8][kFbMaxD];
  __shared__ double s_red[kFbWaves][2], s_res[2];
  __shared__ int s_ab;
  struct ElSt {
    double pd, pt;
    float yb0, yb1, dtb32;
    float ybc, fbc;
    float scb, f0bp;
  };
  __shared__ ElSt s_el[kFbWaves][kFbMaxD];
  struct WSc {
    double dtbar, tbar, dtb_base, h0b, d0b, d1b;
    float dt32, h0f;
    int jj, acc;
  };
  __shared__ WSc s_sc[kFbWaves];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const LayerPlan& P0 = a.P0;
  const LayerPlan& P1 = a.P1;
  const int D = P0.in, H = P0.out, TW = 2 * D + H;
  const float* __restrict__ plan = a.plan;
  const int64_t b = (int64_t)blockIdx.x * kFbWaves + wid;
  const bool live = b < a.B;
  const int64_t bi = live ? b : 0;
  const bool dl = lane < D, hl = lane < H, el = live && dl;
  float* xs = s_x[wid];
  float* ps = s_p[wid];
  float* g1s = s_g1[wid];
  float* gxs = s_gx[wid];
  float(&kk)[8][kFbMaxD] = s_k[wid];
  float(&kb)[8][kFbMaxD] = s_kb[wid];
  const int n_ev = da.n_ev, base = da.base;
  const int64_t tstride = a.B * TW;
  auto tx = [&](int ev) -> float { return a.tape[(int64_t)ev * tstride + bi * TW + lane]; };          // layer input
  auto tk = [&](int ev) -> float { return a.tape[(int64_t)ev * tstride + bi * TW + D + H + lane]; };  // output
  if (threadIdx.x == 0) s_ab = 0;
  __syncthreads();

  // the VJP of evaluation ev: g1s (d loss / d k) -> gxs (d loss / d layer-0 input), adjoints recorded
  auto vjp = [&](int ev) {
    float h = 0.f, ph = 0.f;
    if (live) {
      const float* row = a.tape + (int64_t)ev * tstride + bi * TW;
      const float* prow = ev > 0 ? row - tstride : nullptr;
      if (dl) {
        const float x = row[lane];
        xs[lane] = x;
        ps[lane] = prow ? prow[lane] : ((a.init_mask & 1u) ? x : (FERRO ? a.state0[bi * D + lane] : 0.f));
        da.Xc[((int64_t)ev * a.B + b) * D + lane] = x;
        a.gadj[((int64_t)ev * a.B + b) * D + lane] = g1s[lane];
      }
      if (hl) {
        h = row[D + lane];
        ph = prow ? prow[D + lane] : ((a.init_mask & 2u) ? h : (FERRO ? a.state0[a.B * D + bi * H + lane] : 0.f));
        da.Hc[((int64_t)ev * a.B + b) * H + lane] = h;
      }
    } else if (dl) {
      xs[lane] = 0.f;
      ps[lane] = 0.f;
    }
    fb_wsync();
    const float gh = (live && hl) ? fb_vjp_input<FERRO>(plan, P1, lane, h, ph, g1s, 0, D) : 0.f;
    if (live && hl) a.gadj[(int64_t)n_ev * a.B * D + ((int64_t)ev * a.B + b) * H + lane] = gh;
    float gx = 0.f;
    for (int i = 0; i < D; ++i) {
      const float one = 1.0f;
      const float c = (live && hl) ? gh * fb_vjp_input<FERRO>(plan, P0, i, xs[i], ps[i], &one, lane, 1) : 0.f;
      const float sum = fb_wave_sum(c);
      if (lane == i) gx = sum;
    }
    if (dl) gxs[lane] = gx;
    fb_wsync();
  };

  unsigned round = 0;
  auto gsum = [&](double v0, double v1, double& s0, double& s1) {
    v0 = xor_sum64(v0);
    v1 = xor_sum64(v1);
    if (lane == 0) {
      s_red[wid][0] = v0;
      s_red[wid][1] = v1;
    }
    __syncthreads();
    if (wid == 0) {
      double u0 = s_red[0][0], u1 = s_red[0][1];
      for (int w = 1; w < kFbWaves; ++w) {
        u0 += s_red[w][0];
        u1 += s_red[w][1];
      }
      double r0 = 0.0, r1 = 0.0;
      const bool ab = grid_sum2(da.gp, round, u0, u1, r0, r1);
      if (lane == 0) {
        s_res[0] = r0;
        s_res[1] = r1;
        if (ab) s_ab = 1;
      }
    }
    __syncthreads();
    s0 = s_res[0];
    s1 = s_res[1];
  };

  ElSt& E = s_el[wid][dl ? lane : 0];  // written by lanes < D only
  if (dl) {
    E.ybc = E.fbc = 0.f;
    E.scb = E.f0bp = 0.f;
  }
  WSc& C = s_sc[wid];
  C.dtbar = C.tbar = C.dtb_base = C.h0b = C.d0b = C.d1b = 0.0;
  C.jj = a.T - 1;
  C.dt32 = C.h0f = 0.f;
  C.acc = 0;
  const double* att = da.att;

  for (int ev = n_ev - 1; ev >= 0; --ev) {
    const bool in_att = ev >= base;
    const int n = in_att ? (ev - base) / 6 : -1, s = in_att ? 2 + (ev - base) % 6 : 0;
    if (in_att && s == 7) {
      const double t0 = att[4 * n], dt = att[4 * n + 1];
      const float ratio = (float)att[4 * n + 2];
      C.acc = att[4 * n + 3] != 0.0;
      int m = n - 1;  // the attempt whose stage 7 produced this attempt's y and f0
      while (m >= 0 && att[4 * m + 3] == 0.0) --m;
      const int fe = m >= 0 ? base + 6 * m + 5 : 0;
      const int e2 = base + 6 * n;
      C.dt32 = (float)dt;
      const double rr = (double)ratio;
      double rbar = 0.0, dtbb = 0.0;
      if (n + 1 < da.n_att) {  // rk_common._optimal_step_size's adjoint (the factor from the log)
        const double dtn1 = att[4 * (n + 1) + 1];
        const bool clamped = (da.min_step > 0.0 && dtn1 == da.min_step) || dtn1 == da.max_step;
        if (!clamped) {
          const double fac = dtn1 / dt;
          dtbb = C.dtbar * fac;
          if (rr > 0.0) {
            const double dfac = rr < 1.0 ? 1.0 : da.dfactor;
            const bool bound = fabs(fac - da.ifactor) <= 1e-12 * da.ifactor || fabs(fac - dfac) <= 1e-12 * dfac;
            if (!bound) rbar = C.dtbar * dt * (-0.2 * fac / rr);
          }
        }
      }
      C.dtb_base = dtbb;
      double pd = 0.0, pt = 0.0;
      float dtb32 = 0.f, yb0, yb1;
      const float ybc = dl ? E.ybc : 0.f, fbc = dl ? E.fbc : 0.f;
      float kv[8], kbv[8];
      for (int j = 0; j < 8; ++j) kv[j] = kbv[j] = 0.f;
      float y = 0.f, y1 = 0.f;
      if (el) {
        y = tx(fe);
        kv[1] = tk(fe);
        for (int j = 2; j <= 7; ++j) kv[j] = tk(e2 + j - 2);
        y1 = tx(e2 + 5);
      }
      float err = kv[1] * (da.cerr[0] * C.dt32), midv = kv[1] * (da.cmid[0] * C.dt32);
      for (int j = 2; j <= 7; ++j) {
        err = err + kv[j] * (da.cerr[j - 1] * C.dt32);
        midv = midv + kv[j] * (da.cmid[j - 1] * C.dt32);
      }
      float midb = 0.f, fab;
      if (C.acc) {
        yb1 = ybc;
        kbv[7] = fbc;
        yb0 = 0.f;
        fab = 0.f;
        const float ym = y + midv, fa = kv[1], fbk = kv[7];
        const float co1 = C.dt32 * fa;
        const float co2 = ((C.dt32 * (fbk - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
        const float co3 = ((C.dt32 * (5.0f * fa - 3.0f * fbk) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
        const float co4 = ((2.0f * C.dt32) * (fbk - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, c4 = 0.f;
        const double t1 = t0 + dt, dlt = t1 - t0;
        for (; C.jj >= 1 && da.t[C.jj] > t0; --C.jj) {  // outputs in (t0, t1]
          const float x = (float)((da.t[C.jj] - t0) / dlt);
          const float g = el ? a.gsol[((int64_t)C.jj * a.B + bi) * D + lane] : 0.f;
          const float x2 = x * x, x3 = x2 * x;
          c0 += g;
          c1 += g * x;
          c2 += g * x2;
          c3 += g * x3;
          c4 += g * (x3 * x);
          const float dsdx = co1 + 2.0f * x * co2 + 3.0f * x2 * co3 + 4.0f * x3 * co4;
          const double xb = (double)(g * dsdx);
          pt += xb * (-1.0 / dlt);
          pd += xb * (-(double)x / dlt);
        }
        yb0 += ((c0 - 11.0f * c2) + 18.0f * c3) - 8.0f * c4;
        yb1 += (-5.0f * c2 + 14.0f * c3) - 8.0f * c4;
        const float ymb = (16.0f * c2 - 32.0f * c3) + 16.0f * c4;
        fab += C.dt32 * (((c1 - 4.0f * c2) + 5.0f * c3) - 2.0f * c4);
        kbv[7] += C.dt32 * ((c2 - 3.0f * c3) + 2.0f * c4);
        dtb32 += ((c1 * fa + c2 * (fbk - 4.0f * fa)) + c3 * (5.0f * fa - 3.0f * fbk)) + c4 * (2.0f * (fbk - fa));
        yb0 += ymb;
        midb = ymb;
      } else {
        yb0 = ybc;
        fab = fbc;
        yb1 = 0.f;
      }
      kbv[1] = fab;
      float errb = 0.f;  // error ratio = rms(err / tol): d ratio / d qe = qe / (N ratio)
      if (rbar != 0.0 && ratio > 0.f) {
        const float tol = da.atol + da.rtol * fmaxf(fabsf(y), fabsf(y1));
        const float qe = err / tol;
        const float qb = (float)(rbar * (double)qe / (da.n_el * rr));
        errb = qb / tol;
        const float tolb = -qb * qe / tol, ay = fabsf(y), ay1 = fabsf(y1);
        const float sy = y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f), sy1 = y1 > 0.f ? 1.f : (y1 < 0.f ? -1.f : 0.f);
        const float wy = ay > ay1 ? 1.f : (ay < ay1 ? 0.f : 0.5f);
        yb0 += tolb * da.rtol * wy * sy;
        yb1 += tolb * da.rtol * (1.f - wy) * sy1;
      }
      float se = 0.f, sm = 0.f;
      for (int j = 1; j <= 7; ++j) {
        kbv[j] += errb * (da.cerr[j - 1] * C.dt32) + midb * (da.cmid[j - 1] * C.dt32);
        se += da.cerr[j - 1] * kv[j];
        sm += da.cmid[j - 1] * kv[j];
      }
      dtb32 += errb * se + midb * sm;
      if (dl) {
        for (int j = 1; j <= 7; ++j) {
          kk[j][lane] = kv[j];
          kb[j][lane] = kbv[j];
        }
        E.pd = pd;
        E.pt = pt;
        E.yb0 = yb0;
        E.yb1 = yb1;
        E.dtb32 = dtb32;
      }
    } else if (!in_att && ev == 1) {  // _select_initial_step (fp32): dt0 = min(100 h0, h1)
      const float d1 = (float)da.init_rec[1], d2 = (float)da.init_rec[2];
      const float h0 = (float)da.init_rec[3], h1 = (float)da.init_rec[4];
      C.h0f = h0;
      const double dtb = C.dtbar;
      double h1b = 0.0;
      C.h0b = 0.0;
      const float a100 = 100.0f * h0, ah1 = fabsf(h1), sh1 = h1 < 0.f ? -1.f : 1.f;
      if (a100 < ah1) C.h0b = 100.0 * dtb;
      else if (ah1 < a100) h1b = dtb * sh1;
      else {
        C.h0b = 50.0 * dtb;
        h1b = 0.5 * dtb * sh1;
      }
      double d2b = 0.0, d1b_ = 0.0;
      if (d1 <= 1e-15f && d2 <= 1e-15f) {
        const float v = h0 * 1e-3f;
        if (v > 1e-6f) C.h0b += 1e-3 * h1b;
        else if (v == 1e-6f) C.h0b += 0.5e-3 * h1b;
      } else {  // h1 = (0.01 / max(d1, d2)) ** (1/5); Python's max keeps d1 on a tie
        const bool take2 = d2 > d1;
        const double mx = take2 ? d2 : d1, bse = 0.01 / mx;
        const double mxb = -(h1b * 0.2 * (double)h1 / bse) * bse / mx;
        if (take2) d2b += mxb;
        else d1b_ += mxb;
      }
      const double r2 = (double)d2 * h0, r2b = d2b / h0;  // d2 = |rms((f1 - f0) / scale) / h0|
      C.h0b = C.h0b - d2b * d2 / h0;
      C.d1b = d1b_;
      float f1b = 0.f, f0bp = 0.f, scb = 0.f;
      if (el && r2 > 0.0) {
        const float y = tx(0), f0 = tk(0), f1 = tk(1);
        const float scale = da.atol + fabsf(y) * da.rtol;
        const float q2 = (f1 - f0) / scale;
        const float q2b = (float)(r2b * (double)q2 / (da.n_el * r2));
        f1b = q2b / scale;
        f0bp = -q2b / scale;
        scb = -q2b * q2 / scale;
      }
      if (dl) {
        kb[0][lane] = f1b;
        E.f0bp = f0bp;
        E.scb = scb;
      }
      C.d0b = 0.0;
    } else if (ev == 0) {
      if (base == 2) {  // the rest of _select_initial_step: d0 = rms(y0 / scale), d1 = rms(f0 / scale)
        const float d0 = (float)da.init_rec[0], d1 = (float)da.init_rec[1];
        if (el) {
          const float y = tx(0), f0 = tk(0);
          const float scale = da.atol + fabsf(y) * da.rtol;
          const float q0 = y / scale, q1 = f0 / scale;
          const float q0b = d0 > 0.f ? (float)(C.d0b * (double)q0 / (da.n_el * d0)) : 0.f;
          const float q1b = d1 > 0.f ? (float)(C.d1b * (double)q1 / (da.n_el * d1)) : 0.f;
          const float scb = E.scb - q0b * q0 / scale - q1b * q1 / scale;
          const float sy = y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f);
          E.ybc += q0b / scale + scb * da.rtol * sy;
          E.fbc += q1b / scale;
        }
      }
      if (dl) kb[0][lane] = el ? E.fbc : 0.f;
    }
    if (dl) g1s[lane] = in_att ? kb[s][lane] : kb[0][lane];
    fb_wsync();
    vjp(ev);
    const float xb = dl ? gxs[lane] : 0.f;
    if (in_att) {
      double v0 = 0.0, v1 = 0.0;
      if (dl) {
        const float X = xb + (s == 7 ? E.yb1 : 0.f);  // stage 7's input IS y1
        E.yb0 += X;
        float sb = 0.f;
        for (int j = 1; j < s; ++j) {  // tableau row s - 2
          const float c = da.beta[s - 2][j - 1];
          kb[j][lane] += (c * C.dt32) * X;
          sb += c * kk[j][lane];
        }
        E.dtb32 += X * sb;
        if (s == 2) {  // attempt n done: the carries
          E.ybc = el ? E.yb0 : 0.f;
          E.fbc = el ? kb[1][lane] : 0.f;
          v0 = el ? E.pd + (double)E.dtb32 : 0.0;
          v1 = el ? E.pt : 0.0;
        }
      }
      if (s == 2) {  // the grid sum of the attempt's d/d dt and d/d t0 terms
        double S0, S1;
        gsum(v0, v1, S0, S1);
        C.dtbar = C.dtb_base + (C.acc ? C.tbar : 0.0) + S0;
        C.tbar = C.tbar + S1;
      }
    } else if (ev == 1) {  // the probe: input y0 + h0 f0
      const float f0 = el ? tk(0) : 0.f;
      if (el) {
        E.ybc += xb;
        E.fbc += xb * C.h0f + E.f0bp;
      }
      double S0, S1;
      gsum(el ? (double)(xb * f0) : 0.0, 0.0, S0, S1);
      C.h0b = C.h0b + S0;
      const float d0 = (float)da.init_rec[0], d1 = (float)da.init_rec[1];
      if (!(d0 < 1e-5f || d1 < 1e-5f)) {  // h0 = |0.01 d0 / d1|
        C.d0b = C.h0b * 0.01 / d1;
        C.d1b = C.d1b - C.h0b * (double)C.h0f / d1;
      }
    } else {  // evaluation 0: f(y0)
      if (el) {
        E.ybc += xb;
        if (a.gy0) a.gy0[bi * D + lane] = E.ybc + a.gsol[bi * D + lane];  // solution[0] = y0
      }
    }
    fb_wsync();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    da.status[0] = (s_ab || __hip_atomic_load(dp_abort(da.gp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 4 : 0;
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

// ---- dopri5 ----
static int64_t fieldn_dopri_grid(int64_t B) { return (B + kFbWaves - 1) / kFbWaves; }

static int64_t fieldn_dopri_resident(bool ferro) {
  static int n_cu = 0, per_cu[2] = {0, 0};
  const int fi = ferro ? 0 : 1;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
  }
  if (!per_cu[fi] && hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         &per_cu[fi], ferro ? (const void*)fieldn_dopri_bwd_kernel<true> : (const void*)fieldn_dopri_bwd_kernel<false>,
                         64 * kFbWaves, 0) != hipSuccess)
    return -1;
  return (int64_t)per_cu[fi] * n_cu;
}

// workspace: grid-sum words and slots | output / hidden adjoint planes | layer-input planes | KAN VJP scratch
// the parameter-VJP scratch: the larger KANLinear workspace, or the Ferro row-split partials
static int64_t param_ws(int64_t kw0, int64_t kw1) {
  int64_t w = kw0 > kw1 ? kw0 : kw1;
  return w > ferro_param_rows_workspace() ? w : ferro_param_rows_workspace();
}

struct FdWs {
  int64_t bar, slot, gadj, xc, hc, kws, total;
};
static FdWs fieldn_dopri_ws(const fetode_field_t* f, int64_t B, int64_t n_ev) {
  const int64_t D = f->kan[0].in_features, H = f->kan[0].out_features, grid = fieldn_dopri_grid(B);
  const int64_t kw0 = fetode_kanlinear_backward_workspace(&f->kan[0]), kw1 = fetode_kanlinear_backward_workspace(&f->kan[1]);
  FdWs w;
  w.bar = 0;
  w.slot = (int64_t)sizeof(unsigned) * kDpBarWords;
  w.gadj = w.slot + (int64_t)sizeof(double) * (2 * grid + 4 * kDpGroups);
  w.xc = w.gadj + (int64_t)sizeof(float) * align16(n_ev * B * (D + H));
  w.hc = w.xc + (int64_t)sizeof(float) * align16(n_ev * B * D);
  w.kws = w.hc + (int64_t)sizeof(float) * align16(n_ev * B * H);
  w.total = w.kws + param_ws(kw0, kw1);
  return w;
}

// the row-batched parameter VJPs over all n_ev * B (evaluation, trajectory) rows (written, not
// accumulated): layer 1 on (h, d loss / d k), layer 0 on (x, d loss / d h); the Ferro VJP as two
// row ranges (evaluation 0's hysteresis input: the state before the solve, or the reinit rule)
static int fieldn_param_vjps(const fetode_field_t* f, int64_t B, int64_t n_ev, const float* Xp, const float* Hp,
                      const float* GKp, const float* GHp, const float* state0, uint32_t init_mask,
                      const fetode_kanlinear_grad_t* kan_grads, const fetode_ferro_grad_t* ferro_grads, void* kws,
                      void* stream) {
  const int D = f->kan[0].in_features;
  const int64_t R = n_ev * B;
  for (int l = 0; l < 2; ++l) {
    const float* x = l == 0 ? Xp : Hp;
    const float* g = l == 0 ? GHp : GKp;
    if (kan_grads && any_kan(kan_grads[l])) {
      const int rc = fetode_kanlinear_backward(&f->kan[l], x, R, g, nullptr, &kan_grads[l], kws, 0, stream);
      if (rc) return rc;
    }
    if (f->ferro && ferro_grads && any_ferro(ferro_grads[l])) {
      // one row-split launch over both hysteresis rules (evaluation 0: the state before the solve or
      // reinit; later evaluations: the previous one, B rows earlier)
      const bool re = (init_mask >> l) & 1u;
      const float* p0 = re ? nullptr : state0 + (l == 0 ? 0 : B * D);
      const int rc = ferro_param_rows(&f->ferro[l], x, R, p0, B, g, &ferro_grads[l], kws, 0, stream);
      if (rc) return rc;
    }
  }
  return FETODE_OK;
}

int64_t fetode::fieldn_fixed_backward_workspace(const fetode_field_t* f, int32_t method, int32_t n_steps, int64_t B) {
  const int64_t D = f->kan[0].in_features, H = f->kan[0].out_features;
  const int64_t kw0 = fetode_kanlinear_backward_workspace(&f->kan[0]), kw1 = fetode_kanlinear_backward_workspace(&f->kan[1]);
  if (kw0 < 0 || kw1 < 0) return -1;
  return (int64_t)sizeof(float) * align16(n_evals(method, n_steps) * B * (D + H)) + param_ws(kw0, kw1);
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
  const int64_t pbytes = (int64_t)sizeof(float) * a.P1.end;
  const int tpw = 64 / fb_lanes_per_traj(D, H);
  static const int lds_on = [] {  // FETODE_FIELDN_LDS=0: the plan read from global memory (A/B)
    const char* e = getenv("FETODE_FIELDN_LDS");
    return e ? atoi(e) : 1;
  }();
  if (lds_on && pbytes <= kFbLdsMax) {
    auto* kfn = f->ferro ? fieldn_adj_kernel<true, true> : fieldn_adj_kernel<false, true>;
    static bool attr[2] = {false, false};  // dynamic LDS beyond the 64 KB default
    if (!attr[f->ferro ? 1 : 0]) {
      HIP_CHECK_RET(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFbLdsMax));
      attr[f->ferro ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(kfn, dim3(nblk(B, kFbWavesL * tpw)), dim3(64 * kFbWavesL), (size_t)pbytes, s, a);
  } else {
    auto* kfn = f->ferro ? fieldn_adj_kernel<true, false> : fieldn_adj_kernel<false, false>;
    hipLaunchKernelGGL(kfn, dim3(nblk(B, kFbWaves * tpw)), dim3(64 * kFbWaves), 0, s, a);
  }
  LAUNCH_CHECK();
  if (n_ev == 0) return zero_grads(f, kan_grads, ferro_grads, s);
  // parameter gradients: the per-module VJPs over all n_ev * B rows (planes: tape = x then h,
  // gadj = d loss / d k then d loss / d h)
  const int64_t R = n_ev * B;
  return fieldn_param_vjps(f, B, n_ev, tape, tape + R * D, gadj, gadj + R * D, state0, f->ferro ? init_mask : 3u,
                           kan_grads, ferro_grads, kws, stream);
}

int64_t fetode::fieldn_dopri5_backward_max_batch(const fetode_field_t* f) {
  const int64_t w = fieldn_dopri_resident(f->ferro != nullptr);
  return w > 0 ? w * kFbWaves : 0;
}

int64_t fetode::fieldn_dopri5_backward_workspace(const fetode_field_t* f, int64_t B, int64_t n_ev) {
  if (fetode_kanlinear_backward_workspace(&f->kan[0]) < 0 || fetode_kanlinear_backward_workspace(&f->kan[1]) < 0) return -1;
  return fieldn_dopri_ws(f, B, n_ev).total;
}

int fetode::fieldn_dopri5_backward(const fetode_field_t* f, const void* plan, int64_t B, const double* t, int32_t T,
                                   double rtol, double atol, const double* opts, const float* tableau,
                                   const float* grad_solution, const float* tape, int32_t n_ev, const double* attempts,
                                   int32_t n_att, const double* init_rec, const float* state0, uint32_t init_mask,
                                   float* grad_y0, const fetode_kanlinear_grad_t* kan_grads,
                                   const fetode_ferro_grad_t* ferro_grads, void* workspace, int32_t* status,
                                   void* stream) {
  const int D = f->kan[0].in_features, H = f->kan[0].out_features;
  if (D > kFbMaxD || H > kFbMaxH) return set_err(FETODE_EUNSUPPORTED, "fieldn dopri5 backward: widths beyond [8, 64, 8]");
  const int64_t grid = fieldn_dopri_grid(B), resident = fieldn_dopri_resident(f->ferro != nullptr);
  if (resident < 0) return set_err(FETODE_EHIP, "fieldn dopri5 backward: occupancy query failed");
  if (grid > resident)
    return set_err(FETODE_EUNSUPPORTED, "fieldn dopri5 backward: batch %lld needs %lld workgroups, %lld resident",
                   (long long)B, (long long)grid, (long long)resident);
  hipStream_t s = (hipStream_t)stream;
  const FdWs w = fieldn_dopri_ws(f, B, n_ev);
  char* ws = (char*)workspace;
  FdArgs d;
  memset(&d, 0, sizeof(d));
  FbArgs& a = d.b;
  a.plan = (const float*)plan;
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  a.B = B;
  a.T = T;
  a.gsol = grad_solution;
  a.tape = tape;
  a.state0 = state0;
  a.init_mask = f->ferro ? init_mask : 3u;
  a.gy0 = grad_y0;
  a.gadj = (float*)(ws + w.gadj);
  d.Xc = (float*)(ws + w.xc);
  d.Hc = (float*)(ws + w.hc);
  d.att = attempts;
  d.n_att = n_att;
  d.n_ev = n_ev;
  d.base = opts[0] > 0.0 ? 1 : 2;
  d.t = t;
  d.init_rec = init_rec;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) d.beta[i][j] = tableau[i * 6 + j];
  for (int j = 0; j < 7; ++j) {
    d.cerr[j] = tableau[36 + j];
    d.cmid[j] = tableau[43 + j];
  }
  d.rtol = (float)rtol;
  d.atol = (float)atol;
  d.safety = opts[1];
  d.ifactor = opts[2];
  d.dfactor = opts[3];
  d.min_step = opts[4];
  d.max_step = opts[5];
  d.n_el = (double)B * D;
  d.gp.bar = (unsigned*)(ws + w.bar);
  d.gp.slot = (double*)(ws + w.slot);
  d.gp.xs = d.gp.slot + 2 * grid;
  dp_single_device(d.gp, grid);
  d.status = status;
  HIP_CHECK_RET(hipMemsetAsync(workspace, 0, sizeof(unsigned) * kDpBarWords, s));
  void* args[] = {&d};
  HIP_CHECK_RET(resident_launch(f->ferro ? (const void*)fieldn_dopri_bwd_kernel<true> : (const void*)fieldn_dopri_bwd_kernel<false>,
                                dim3((unsigned)grid), dim3(64 * kFbWaves), args, 0, s));
  if (n_ev == 0) return zero_grads(f, kan_grads, ferro_grads, s);
  const int64_t R = (int64_t)n_ev * B;
  return fieldn_param_vjps(f, B, n_ev, d.Xc, d.Hc, a.gadj, a.gadj + R * D, state0, a.init_mask, kan_grads,
                           ferro_grads, ws + w.kws, stream);
}
