// fetode_bwd.hip — the reverse sweep of the single-launch fixed-grid integrator (training).
//
// What it replaces: loss.backward() through torchdiffeq's fixed-grid solve of a KAN / KAN-FET
// field (train_kanfet_node_predprey.py:254-257), i.e. reverse-mode autograd through every stage
// evaluation (KANLinear.forward efficientkan.py:160-182, FerroelectricBasis.forward
// ferro_class.py:368-420 whose prev_x / branch_sign snapshots are detached, :381-382), the
// rk_common.rk4_alt_step_func stage combines and FixedGridODESolver's output interpolation.
//
// Data flow.  The forward kernel (fetode_fused.hip) records the two layer inputs of every
// evaluation on a "tape" (n_evals, B, D + H); the hysteresis input of evaluation ev is the tape
// row of ev - 1 (ferro_class.py:409), or the state before the solve for ev = 0.  So the sweep
// recomputes nothing but per-input features: one wave owns one trajectory and walks its
// evaluations backwards, carrying the adjoints of y and of the stage derivatives k_j.
//
// Per evaluation (layer 1 then layer 0, lanes = jobs):
//   features   per input: SiLU, SiLU', dense B-spline bases, knot interval/coordinate, the
//              hysteresis gate u = sigmoid(gs(x - prev)); per (input, basis): the logistic sigmoid
//   Ferro      per element (i, o, k): the element's forward quantities and its VJP; parameter
//              gradients are accumulated in three per-element sums A, C, E (see below)
//   KAN edges  per (o, i): base + spline-coefficient sums, d/dx via the plan's cubic tables
//   logistic   per (i, j): the logistic-weight sums and the a / b gradients
//   d out/d x  per-job contributions land in an LDS table and are summed per input in a fixed
//              order (segmented sum + xor shuffles): run-to-run deterministic, no atomics.
// The gradient sums live in VGPRs for the whole sweep (each lane owns fixed slots), are written
// once per block to a partial buffer, reduced over blocks in a fixed order (fp64), and turned
// into parameter gradients by one small kernel:
//   Ferro e = (i,o,k):  A = sum g_o th,  C = sum g_o (1-th^2) sh,  E = sum g_o (1-th^2)(m + Ec dm/dEc),
//                       G_o = sum g_o   ->  dk = coef Ps C, dEc = coef Ps k E, dPs = coef A,
//                       dbias = coef G_o, dcoef = Ps A + bias G_o
//   KAN (o,i):          base = sum g_o SiLU(x_i), spline_c = sum g_o B_c(x_i)
//   logistic (o,i,j):   sum g_o sigmoid_ij;  a_ij, b_ij directly.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fetode_common.h"

using namespace fetode;

namespace {

#include "fetode_gridsum.h"

constexpr int kSO = 3;  // spline order of the fused kernels (efficientkan default)
// FETODE_EXP_SKIP (phase-cost attribution: 1 Ferro, 2 edges, 4 logistic, 8 features, 16 d/dx
// reductions compiled out — results are wrong when set) exists only in the diagnostic build
// (make diag EXTRA=-DFETODE_EXP_SKIP=n); the product library is always built with 0.
#if defined(FETODE_EXP_SKIP) && !defined(FETODE_DIAG)
#error "FETODE_EXP_SKIP is a diagnostic knob: build it with make diag"
#endif
#ifndef FETODE_EXP_SKIP
#define FETODE_EXP_SKIP 0
#endif

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }
__device__ __forceinline__ f2 ex2x2(f2 v) { return f2{ex2(v.x), ex2(v.y)}; }
__device__ __forceinline__ f2 rcpx2(f2 v) { return f2{rcp(v.x), rcp(v.y)}; }

constexpr int pow2_floor(int v) {
  int p = 1;
  while (p * 2 <= v) p *= 2;
  return p;
}

// Layout of one layer's gradient sums in a partial row (host and device agree on it).
struct AccLayout {
  int E, NE, NL, NS, NTM;
  int oA, oC, oE, oG, oBase, oSpl, oLw, oLa, oLb, n;
};
__host__ __device__ constexpr AccLayout acc_layout(int in, int out, int K, int NB, int NS, bool ferro) {
  AccLayout L{};
  L.E = ferro ? in * out * K : 0;
  L.NE = in * out;
  L.NL = in * NB;
  L.NS = NS;
  L.NTM = (ferro ? out * K : 0) + out + NB;
  L.oA = 0;
  L.oC = L.E;
  L.oE = 2 * L.E;
  L.oG = 3 * L.E;
  L.oBase = L.oG + (ferro ? out : 0);
  L.oSpl = L.oBase + L.NE;
  L.oLw = L.oSpl + L.NE * NS;
  L.oLa = L.oLw + out * L.NL;
  L.oLb = L.oLa + L.NL;
  L.n = L.oLb + L.NL;
  return L;
}

template <int IN_, int OUT_, int K_, int NB_, int NG_, bool FERRO_>
struct BL {  // compile-time shape of one layer
  static constexpr int IN = IN_, OUT = OUT_, K = FERRO_ ? K_ : 0, NB = NB_, NG = NG_;
  static constexpr bool FERRO = FERRO_;
  static constexpr int NI = NG - 1, NS = NG - 1 - kSO, NFL = 1 + NB;
  static constexpr AccLayout AL = acc_layout(IN, OUT, K, NB, NS, FERRO);
  static constexpr int E = AL.E, NE = AL.NE, NL = AL.NL, NTM = AL.NTM;
  static constexpr int RF = (E + 63) / 64, RE = (NE + 63) / 64, RL = (NL + 63) / 64;
  static constexpr int RF1 = RF > 0 ? RF : 1, RL1 = RL > 0 ? RL : 1;
  static constexpr int EP = E / 2, RP = (EP + 63) / 64, RP1 = RP > 0 ? RP : 1;  // Ferro element pairs (k, k+1)
  static_assert(K % 2 == 0, "Ferro elements are walked in (k, k+1) pairs");
  static constexpr int LPI = pow2_floor(64 / IN);  // lanes per input in the d/dx segmented sum
  // cb row pitch: NTM rounded up to LPI mod 32, so the LPI-lane groups of one half-wave read
  // distinct LDS banks in reduce_gin (a pitch of 32 put all ten inputs of layer 1 on banks 0-3)
  // (extra padding of 4 / 12 / 16 floats measured within 1 %: the pitch is not a lever)
  static constexpr int NTMP = LPI >= 32 ? NTM : NTM + ((LPI - NTM % 32) % 32 + 32) % 32;
  static_assert(IN <= 64 && OUT <= 64, "layer widths up to 64");
  static_assert(NS >= 1, "grid too small for cubic splines");
};

// Per-block LDS tables of the whole field.  Per-INPUT tables are laid out over the combined input
// index t in [0, W): t < D are layer-0 inputs, t >= D layer-1 inputs (same knot count), so the
// feature phase is one code path for both layers.
template <int W, int NG, int NB>
struct BInTab {
  static constexpr int NI = NG - 1;
  // basis B_{m-3+r} on interval m as a cubic in u: [t][m][r] (power basis); one float4 of
  // padding per input so that lanes gathering different inputs' rows spread over the LDS banks
  static constexpr int BPS = NI * 4 + 1;
  float4 bp[W * BPS];
  __device__ static int bpi(int t, int m) { return t * BPS + m * 4; }
  float knots[W * NG];
  float rh[W * NI];       // 1/(g[m+1] - g[m])
  __attribute__((aligned(8))) float lg[NB > 0 ? 2 * W * NB : 1];  // (-a log2e, a b log2e) per (t, j)

  __device__ void stage(const float* __restrict__ plan, const LayerPlan& P0, const LayerPlan& P1, int D, int tid,
                        int nt) {
    for (int q = tid; q < W * NG; q += nt) {
      const int t = q / NG, j = q % NG;
      knots[q] = t < D ? plan[P0.knots + t * NG + j] : plan[P1.knots + (t - D) * NG + j];
    }
    for (int q = tid; q < W * NI; q += nt) {
      const int t = q / NI, m = q % NI;
      rh[q] = t < D ? plan[P0.rh + t * NI + m] : plan[P1.rh + (t - D) * NI + m];
    }
    for (int q = tid; q < 2 * W * NB; q += nt)
      lg[q] = q < 2 * D * NB ? plan[P0.lg + q] : plan[P1.lg + (q - 2 * D * NB)];
    // basis polynomials: Cox-de Boor (efficientkan.py:117-131) restricted to interval m, in
    // fp64 at u = 0, 1/3, 2/3, 1, converted to the power basis (exact for cubics)
    for (int q = tid; q < W * NI; q += nt) {
      const int t = q / NI, m = q % NI;
      const float* g = t < D ? plan + P0.knots + t * NG : plan + P1.knots + (t - D) * NG;
      const double h = (double)g[m + 1] - g[m];
      double v[4][kSO + 2];
      for (int s = 0; s < 4; ++s) {
        const double x = g[m] + h * (s / 3.0);
        double* N = v[s];
        for (int r = 0; r < kSO + 2; ++r) N[r] = 0.0;
        N[kSO] = 1.0;
        for (int k = 1; k <= kSO; ++k) {
          double M[kSO + 2];
          for (int r = 0; r < kSO + 2; ++r) M[r] = 0.0;
          for (int r = kSO - k; r <= kSO; ++r) {
            const int j = m - kSO + r;
            if (j >= 0 && j <= NG - 2 - k) {
              const double left = (x - g[j]) / ((double)g[j + k] - g[j]) * N[r];
              const double right = ((double)g[j + k + 1] - x) / ((double)g[j + k + 1] - g[j + 1]) * N[r + 1];
              M[r] = left + right;
            }
          }
          for (int r = 0; r < kSO + 2; ++r) N[r] = M[r];
        }
      }
      for (int r = 0; r <= kSO; ++r) {
        const double a0 = v[0][r], a1 = v[1][r], a2 = v[2][r], a3 = v[3][r];
        bp[bpi(t, m) + r] = make_float4((float)a0, (float)((-11.0 * a0 + 18.0 * a1 - 9.0 * a2 + 2.0 * a3) / 2.0),
                                    (float)(9.0 * (2.0 * a0 - 5.0 * a1 + 4.0 * a2 - a3) / 2.0),
                                    (float)(9.0 * (-a0 + 3.0 * a1 - 3.0 * a2 + a3) / 2.0));
      }
    }
  }
};

template <class L>
struct BTab {  // per-block LDS copy of one layer's edge tables
  // spline edge (o, i) as a cubic in u per interval (NI + 1 rows: the last is the zero row), rows
  // of one edge padded to SPS float4s (lanes gather different edges: spread over the banks)
  static constexpr int SPS = L::NI + 2;
  float4 sp[L::OUT * L::IN * SPS];
  float kw[L::OUT * L::IN * L::NFL];        // SiLU weight, 2 * scaled logistic weights
  float pa[L::NL > 0 ? L::NL : 1], pb[L::NL > 0 ? L::NL : 1];
  // Ferro element pair p = elements (2p, 2p + 1) = (i, o, k..k+1):
  //   fpa = (Ec, Ec', 2 log2e k, 2 log2e k'),  fpb = (coef Ps k, coef' Ps' k', gs log2e Ec, gs log2e Ec')
  float4 fpa[L::EP > 0 ? L::EP : 1], fpb[L::EP > 0 ? L::EP : 1];

  __device__ void stage(const fetode_kanlinear_t& kl, const fetode_ferro_t& fl, const float* __restrict__ plan,
                        const LayerPlan& P, int tid, int nt) {
    const float gl = L::FERRO ? P.gsl2e : 0.f, k2 = 2.0f * FETODE_LOG2E;
    for (int p = tid; p < L::EP; p += nt) {
      const int e = 2 * p;
      fpa[p] = make_float4(fl.Ec[e], fl.Ec[e + 1], k2 * fl.k[e], k2 * fl.k[e + 1]);
      fpb[p] = make_float4((fl.coef[e] * fl.Ps[e]) * fl.k[e], (fl.coef[e + 1] * fl.Ps[e + 1]) * fl.k[e + 1],
                           gl * fl.Ec[e], gl * fl.Ec[e + 1]);
    }
    const float4* src = reinterpret_cast<const float4*>(plan + P.sp);
    for (int q = tid; q < L::OUT * L::IN * (L::NI + 1); q += nt) sp[q / (L::NI + 1) * SPS + q % (L::NI + 1)] = src[q];
    for (int q = tid; q < L::OUT * L::IN * L::NFL; q += nt) kw[q] = plan[P.kw + q];
    for (int q = tid; q < L::NL; q += nt) {
      pa[q] = kl.logistic_a[q];
      pb[q] = kl.logistic_b[q];
    }
  }
};

template <int W, int NS, int NB, bool WIN = false>
struct BFeat {  // per-wave LDS features of both layers' inputs, combined index t
  // dense B-spline row of input t at bd[t * BDP + BD0 + c].  WIN: the interval's four bases are
  // written at c = m - 3 .. m into a filled row, so the rows carry kSO guard floats on either side
  // (BD0 keeps the data 16-byte aligned; BDP = 4 mod 8 spreads the inputs over the banks); without
  // WIN (the adjoint-only sweep, whose 4 waves per SIMD leave no LDS for guards) the row is dense
  static constexpr bool WINDOW = WIN;
  static constexpr int BD0 = WIN ? 4 : 0;
  static constexpr int BDP0 = (BD0 + NS + kSO + 3) / 4 * 4;
  static constexpr int BDP = !WIN ? NS : BDP0 % 8 == 0 ? BDP0 + 4 : BDP0;
  __device__ static int bdi(int t, int c) { return t * BDP + BD0 + c; }
  float4 g4[W];  // Ferro per-input terms: x, gate up, wo = wc (1 - up), -ln2 wo
  float x[W], pv[W], silu[W], dsilu[W], u[W], rhm[W];  // rhm: 1 / (knot step) of x's interval
  int m[W];
  __attribute__((aligned(16))) float bd[W * BDP];
  float sg[NB > 0 ? W * NB : 1];
};

template <class L>
struct BReg {  // per-lane register slice of one layer: its gradient sums
  f2 A[L::RP1], C[L::RP1], Ev[L::RP1];  // element pairs
  float G;
  float base[L::RE], spl[L::RE][L::NS];
  float lw[L::RL1][L::OUT], la[L::RL1], lb[L::RL1];

  __device__ void zero() {
#pragma unroll
    for (int r = 0; r < L::RP1; ++r) A[r] = C[r] = Ev[r] = splat(0.f);
    G = 0.f;
#pragma unroll
    for (int r = 0; r < L::RE; ++r) {
      base[r] = 0.f;
#pragma unroll
      for (int c = 0; c < L::NS; ++c) spl[r][c] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < L::RL1; ++r) {
      la[r] = lb[r] = 0.f;
#pragma unroll
      for (int o = 0; o < L::OUT; ++o) lw[r][o] = 0.f;
    }
  }

  // TPW > 1: job sets that fit in 64 / TPW lanes ran once per trajectory on lanes tt * LPT + job
  // (layer_jobs), so their sums are combined here, trajectories in order
  template <int TPW>
  __device__ void store(float* __restrict__ part, int lane) {
    constexpr AccLayout AL = L::AL;
    constexpr int LPT = 64 / TPW;
    auto comb = [&](float v) {
      float t = v;
#pragma unroll
      for (int k = 1; k < TPW; ++k) t += __shfl(v, lane + k * LPT);
      return t;
    };
    if constexpr (TPW > 1 && L::NE <= LPT) {
      base[0] = comb(base[0]);
#pragma unroll
      for (int c = 0; c < L::NS; ++c) spl[0][c] = comb(spl[0][c]);
    }
    if constexpr (TPW > 1 && L::NL <= LPT) {
#pragma unroll
      for (int o = 0; o < L::OUT; ++o) lw[0][o] = comb(lw[0][o]);
      la[0] = comb(la[0]);
      lb[0] = comb(lb[0]);
    }
#pragma unroll
    for (int r = 0; r < L::RP; ++r) {
      const int e = 2 * (lane + 64 * r);
      if (e < L::E) {
        part[AL.oA + e] = A[r].x;
        part[AL.oA + e + 1] = A[r].y;
        part[AL.oC + e] = C[r].x;
        part[AL.oC + e + 1] = C[r].y;
        part[AL.oE + e] = Ev[r].x;
        part[AL.oE + e + 1] = Ev[r].y;
      }
    }
    if (L::FERRO && lane < L::OUT) part[AL.oG + lane] = G;
#pragma unroll
    for (int r = 0; r < L::RE; ++r) {
      const int q = lane + 64 * r;
      if (q < L::NE) {
        part[AL.oBase + q] = base[r];
#pragma unroll
        for (int c = 0; c < L::NS; ++c) part[AL.oSpl + q * L::NS + c] = spl[r][c];
      }
    }
#pragma unroll
    for (int r = 0; r < L::RL; ++r) {
      const int q = lane + 64 * r;
      if (q < L::NL) {
#pragma unroll
        for (int o = 0; o < L::OUT; ++o) part[AL.oLw + o * L::NL + q] = lw[r][o];
        part[AL.oLa + q] = la[r];
        part[AL.oLb + q] = lb[r];
      }
    }
  }
};

__device__ __forceinline__ float sigm_l2(float zl) { return rcp(1.0f + ex2(zl)); }  // 1/(1+2^zl)

// The lanes of one wave exchange data only through that wave's private LDS region.  DS
// instructions of one wave execute in issue order, so a compiler barrier plus a wait for the
// wave's own LDS traffic replaces the workgroup barrier (global loads in flight — the tape
// prefetch — are not waited for).
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// sum over aligned groups of G lanes (G a power of two <= 32), result on every lane of the group
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (G >= 2) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  if constexpr (G >= 4) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  if constexpr (G == 8) v += __shfl_xor(v, 4);
  if constexpr (G >= 16) {  // row_ror 4 then 8: every lane of the 16-lane row holds the row sum
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  }
  if constexpr (G >= 32) v += __shfl_xor(v, 16);
  static_assert(G <= 32, "group up to 32 lanes");
  return v;
}

// features of combined input t (one lane): SiLU, SiLU', knot interval, u, dense bases, gate
template <int W, int NG, int NB, bool WIN>
__device__ __forceinline__ void feat_input(BFeat<W, NG - 1 - kSO, NB, WIN>& F, const BInTab<W, NG, NB>& Tb, int t,
                                           float gsl2e, float wc, float gs, int z) {
  constexpr int NI = NG - 1, NS = NG - 1 - kSO;
  const float x = F.x[t];
  const float sx = sigm_l2(-x * FETODE_LOG2E);
  F.silu[t] = x * sx;
  F.dsilu[t] = sx * ffma(x, 1.0f - sx, 1.0f);
  const float* g = &Tb.knots[t * NG + z];
  int m = -1;
  if constexpr (NG % 4 == 0) {  // the row as float4s: every knot read issued at once
    const float4* g4 = reinterpret_cast<const float4*>(g);
#pragma unroll
    for (int j = 0; j < NG / 4; ++j) {
      const float4 v = g4[j];
      m += ((x >= v.x) ? 1 : 0) + ((x >= v.y) ? 1 : 0) + ((x >= v.z) ? 1 : 0) + ((x >= v.w) ? 1 : 0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NG; ++j) m += (x >= g[j]) ? 1 : 0;
  }
  const bool fin = __builtin_isfinite(x);
  const bool in = fin && m >= 0 && m < NI;
  const int mc = in ? m : 0;
  const float rhm = Tb.rh[t * NI + mc + z];
  const float u = in ? (x - g[mc]) * rhm : (fin ? 0.f : __builtin_nanf(""));
  F.rhm[t] = rhm;
  F.m[t] = in ? m : NI;
  F.u[t] = u;
  using FB = BFeat<W, NS, NB, WIN>;
  float* bd = &F.bd[FB::bdi(t, 0)];
  // non-finite x: NaN bases like the reference's (x - g)/d * 0; outside the grid: all zero
  const float fill = fin ? 0.f : __builtin_nanf("");
  // the interval's four basis cubics, all reads issued before any use
  const float4* bp = &Tb.bp[Tb.bpi(t, mc) + z];
  float4 p[kSO + 1];
#pragma unroll
  for (int r = 0; r <= kSO; ++r) p[r] = bp[r];
  float v[kSO + 1];
#pragma unroll
  for (int r = 0; r <= kSO; ++r) v[r] = ffma(ffma(ffma(p[r].w, u, p[r].z), u, p[r].y), u, p[r].x);
  // dense row through the LDS window: the row filled, then bases m - 3 .. m written over it (one
  // wave's LDS writes land in issue order; c outside [0, NS) falls in the guards, and off the grid
  // mc = 0 puts the fill over c = 0 again)
  if constexpr (WIN) {
    if constexpr (NS % 4 == 0) {
#pragma unroll
      for (int c = 0; c < NS; c += 4) *reinterpret_cast<float4*>(&bd[c]) = make_float4(fill, fill, fill, fill);
    } else {
#pragma unroll
      for (int c = 0; c < NS; ++c) bd[c] = fill;
    }
#pragma unroll
    for (int r = 0; r <= kSO; ++r) bd[mc - kSO + r] = in ? v[r] : fill;
  } else {  // formed in registers (select chains) and written once
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      float b = fill;
#pragma unroll
      for (int r = 0; r <= kSO; ++r) b = (in && c == mc - kSO + r) ? v[r] : b;
      bd[c] = b;
    }
  }
  const float up = sigm_l2(-gsl2e * (x - F.pv[t]));
  const float wo = wc * (1.0f - up);
  F.g4[t] = make_float4(x, up, wo, -0.69314718f * wo);
}

// the VJP jobs of one layer (inputs at combined offset TB) for one evaluation of each of the
// wave's TPW trajectories (Fs[tt], gouts + tt * GS, cbs + tt * CBS): gradient sums into R (the
// lane's job slots, summed over the trajectories in order), d out/d x contributions into
// cb[i * NTMP + t]
template <class L, int TB, bool ACC, int TPW, int GS, int CBS, class FT>
__device__ __forceinline__ void layer_jobs(const FT* Fs, const float* __restrict__ gouts, const BTab<L>& Tb,
                                           const float* __restrict__ rhs, BReg<L>& R, float* __restrict__ cbs,
                                           float gsl2e, float wc, float gs, int lane, int z) {
  if constexpr (L::FERRO && !(FETODE_EXP_SKIP & 1)) {
    // element pairs (k, k+1) of one (i, o) on packed-fp32 ops; with wo = wc (1 - up), c' = c (1 - c):
    //   c = sigmoid(gs(-x - Ec)), m = 1 + wo c, sh = x + Ec m, th = tanh(k sh), q = g (1 - th^2)
    //   A += g th, C += q sh, E += q (m + Ec dm/dEc) with Ec dm/dEc = (-gs Ec) wo c'
    //   d out/d x = q coef Ps k (1 + Ec dm/dx) with dm/dx = -gs wo (up c + c');
    //   (-gs Ec) wo is formed once per pair as (gs log2e Ec)(-ln2 wo)
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)  // trajectories in turn, each one's rounds interleaved
#pragma unroll
    for (int r = 0; r < L::RP; ++r) {
      const int p = lane + 64 * r;
      if (p < L::EP) {
        const FT& F = Fs[tt];
        const float* gout = gouts + tt * GS;
        float* cb = cbs + tt * CBS;
        const int e = 2 * p, i = e / (L::OUT * L::K), ok_ = e % (L::OUT * L::K);
        const int o = ok_ / L::K;
        const float4 g = F.g4[TB + i];
        const float go = gout[o];
        const float4 fa = Tb.fpa[p + z], fb = Tb.fpb[p + z];
        const f2 Ec = f2{fa.x, fa.y}, k2 = f2{fa.z, fa.w}, cPk = f2{fb.x, fb.y}, Eg2 = f2{fb.z, fb.w};
        const f2 x = splat(g.x), wo = splat(g.z), gv = splat(go);
        const f2 cn = rcpx2(ex2x2(pfma(x, splat(gsl2e), Eg2)) + splat(1.0f));  // sigmoid(gs(-x - Ec))
        const f2 mm = pfma(wo, cn, splat(1.0f));                           // branch_mom, branch_sign = 1
        const f2 sh = pfma(Ec, mm, x);                                     // shifted_x
        const f2 th = pfma(splat(-2.0f), rcpx2(ex2x2(k2 * sh) + splat(1.0f)), splat(1.0f));  // tanh(k sh)
        const f2 q = gv * pfma(-th, th, splat(1.0f));
        const f2 dcn = pfma(-cn, cn, cn);
        const f2 ew = Eg2 * splat(g.w);  // (-gs Ec) wo
        if constexpr (ACC) {
          R.A[r] = pfma(gv, th, R.A[r]);
          R.C[r] = pfma(q, sh, R.C[r]);
          R.Ev[r] = pfma(q, pfma(ew, dcn, mm), R.Ev[r]);
        }
        // Ec dm/dx = ew (up c + c')
        *reinterpret_cast<f2*>(&cb[i * L::NTMP + ok_]) = (q * cPk) * pfma(ew, pfma(splat(g.y), cn, dcn), splat(1.0f));
      }
    }
    if constexpr (ACC)
      if (lane < L::OUT)
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt) R.G += gouts[tt * GS + lane];
  }
  // KAN edges (and below, logistic pairs): when one trajectory's jobs fit in 64 / TPW lanes, every
  // trajectory's jobs run in ONE round (lane = tt * 64 / TPW + job); the lane sums of one job are
  // combined across trajectories once, at store
  auto edge = [&](int tt, int q, int r) __attribute__((always_inline)) {
    {
      const FT& F = Fs[tt];
      float* cb = cbs + tt * CBS;
      const int o = q / L::IN, i = q % L::IN;
      const float go = gouts[tt * GS + o];
      if constexpr (ACC) {
        R.base[r] = ffma(go, F.silu[TB + i], R.base[r]);
#pragma unroll
        for (int c = 0; c < L::NS; ++c) R.spl[r][c] = ffma(go, F.bd[FT::bdi(TB + i, c)], R.spl[r][c]);
      }
      const int m = F.m[TB + i];
      const float u = F.u[TB + i];
      // (o, i, interval), q = o*IN + i; off the grid m = NI reads the zero row, so dsdx is 0 there
      // (u = 0) and NaN for non-finite inputs (u = NaN): the reference's NaN bases, branch-free
      const float4 cf = Tb.sp[q * BTab<L>::SPS + m + z];
      const float dsdx = ffma(u, ffma(3.0f * u, cf.w, 2.0f * cf.z), cf.y) * F.rhm[TB + i];
      const float wb = Tb.kw[o * (L::IN * L::NFL) + i * L::NFL + z];
      cb[i * L::NTMP + L::OUT * L::K + o] = go * ffma(wb, F.dsilu[TB + i], dsdx);
    }
  };
  constexpr int LPT = 64 / TPW;
  if constexpr (FETODE_EXP_SKIP & 2) {
  } else if constexpr (L::NE <= LPT) {
    if (lane % LPT < L::NE) edge(lane / LPT, lane % LPT, 0);
  } else {
#pragma unroll 1
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int r = 0; r < L::RE; ++r)
      if (lane + 64 * r < L::NE) edge(tt, lane + 64 * r, r);
  }
  auto logi = [&](int tt, int q, int r) __attribute__((always_inline)) {
    {
      const FT& F = Fs[tt];
      const float* gout = gouts + tt * GS;
      float* cb = cbs + tt * CBS;
      const int i = q / L::NB, j = q % L::NB;
      const float s = F.sg[TB * L::NB + q], ds = s * (1.0f - s), x = F.x[TB + i];
      float S = 0.f;
#pragma unroll
      for (int o = 0; o < L::OUT; ++o) {
        const float go = gout[o];
        S = ffma(go, Tb.kw[o * (L::IN * L::NFL) + i * L::NFL + 1 + j + z], S);
        if constexpr (ACC) R.lw[r][o] = ffma(go, s, R.lw[r][o]);
      }
      const float T = S * ds;  // kw holds 2 * scaled logistic weight: d(2 sigmoid) folded in
      const float pa = Tb.pa[q + z];
      if constexpr (ACC) {
        R.la[r] = ffma(T, x - Tb.pb[q + z], R.la[r]);
        R.lb[r] = ffma(-T, pa, R.lb[r]);
      }
      cb[i * L::NTMP + L::OUT * L::K + L::OUT + j] = T * pa;
    }
  };
  if constexpr (FETODE_EXP_SKIP & 4) {
  } else if constexpr (L::NL <= LPT) {
    if (lane % LPT < L::NL) logi(lane / LPT, lane % LPT, 0);
  } else {
#pragma unroll 1
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int r = 0; r < L::RL; ++r)
      if (lane + 64 * r < L::NL) logi(tt, lane + 64 * r, r);
  }
}

// gin[i] = sum_t cb[i * NTMP + t], fixed order: LPI lanes per input, each summing a contiguous
// run of float4 chunks, then a DPP tree; with TPW trajectories per wave each takes 64 / TPW lanes
// (cbs + tt * CBS -> gins + tt * GS)
template <class L, int TPW, int GS, int CBS>
__device__ __forceinline__ void reduce_gin(const float* __restrict__ cbs, float* gins, int lane) {
  if constexpr (FETODE_EXP_SKIP & 16) return;
  constexpr int HALF = 64 / TPW;
  constexpr int LPI0 = pow2_floor(HALF / L::IN);
  constexpr int LPI = LPI0 > 32 ? 32 : (L::LPI < LPI0 ? L::LPI : LPI0);
  constexpr int C4 = (L::NTM + 4 * LPI - 1) / (4 * LPI);  // float4 chunks per lane
  static_assert(L::NTM % 4 == 0 && L::NTMP % 4 == 0 && CBS % 4 == 0, "float4 rows of the cb table");
  const int tt = lane / HALF, sl = lane % HALF;
  const int i = sl / LPI, sub = sl % LPI;
  const float4* cb = reinterpret_cast<const float4*>(cbs + tt * CBS + i * L::NTMP);
  float s = 0.f;
  if (i < L::IN) {
#pragma unroll
    for (int k = 0; k < C4; ++k) {
      const int c = sub * C4 + k;
      if (4 * c < L::NTM) {
        const float4 v = cb[c];
        s += (v.x + v.y) + (v.z + v.w);
      }
    }
  }
  s = group_sum<LPI>(s);
  if (i < L::IN && sub == 0) gins[tt * GS + i] = s;
}

struct BwdArgs {
  const float* plan;
  LayerPlan P0, P1;
  fetode_kanlinear_t k0, k1;
  fetode_ferro_t f0, f1;
  int32_t method;
  int64_t B;
  const float* step_coef;
  int32_t n_steps;
  const int32_t* out_step;
  const int32_t* out_mode;
  const float* out_slope;
  int32_t T;
  const float* gsol;    // (T, B, D)
  const float* tape;    // (n_evals, B, D + H)
  const float* state0;  // hysteresis state before the solve (include/fetode.h layout)
  uint32_t init_mask;
  float* gy0;           // (B, D) or null
  float* part;          // (rows, nacc)
  int32_t nacc;
  float* gadj;          // (n_evals, B, D + H): d loss / d k (D) and d loss / d h (H) per evaluation
};

// stage-combine coefficients of one step in the forward's fp32 arithmetic (odeint.py
// _combine_coefs): y1 = y + sum_j bc[j] k_j,  X_st = y + sum_{j<st} ac[st][j] k_j
__device__ __forceinline__ void step_coefs(int method, float dt, float hh, float h6, float bc[4], float ac[4][3]) {
  const float third = 1.0f / 3.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bc[i] = 0.f;
#pragma unroll
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
  } else if (method == FETODE_RK4_CLASSIC) {  // train_kan_fet_ett.py:72-75
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

constexpr int kTPB = 4;  // trajectories (waves) per workgroup, sharing one copy of the tables
#ifndef FETODE_BWD_WAVES
#define FETODE_BWD_WAVES 2  // minimum waves per SIMD the register allocation must allow
#endif

// ACC = true: the whole reverse sweep in one kernel — adjoints and the parameter-gradient sums (in
// VGPRs, one partial row per wave).  ACC = false: the adjoint sweep only (no sums: 114 VGPRs, four
// waves per SIMD, all B = 4096 trajectories resident at once); it records every evaluation's
// output and hidden adjoints in a.gadj and param_sum_kernel forms the sums in parallel.
// TPW trajectories per wave: lane l serves trajectory tt = l / (64 / TPW) in the per-input phases
// (tape, features, d out/d x sums, adjoint scalars) and owns its job slots for all TPW of them in
// the VJP phases, so the gradient sums do not grow with TPW.  TPW = 2 halves the waves (B = 4096:
// 2 048 waves = every trajectory resident in one round at the sums' 2 waves per SIMD).
template <int D, int H, int K, int NB, int NG, bool FERRO, bool ACC, int TPW>
__global__ __launch_bounds__(64 * kTPB) __attribute__((amdgpu_waves_per_eu(ACC ? FETODE_BWD_WAVES : 4))) void fixed_bwd_kernel(BwdArgs a) {
  using L0 = BL<D, H, K, NB, NG, FERRO>;
  using L1 = BL<H, D, K, NB, NG, FERRO>;
  constexpr int W = D + H, NS = NG - 1 - kSO, HALF = 64 / TPW;
  constexpr int CB = L0::IN * L0::NTMP > L1::IN * L1::NTMP ? L0::IN * L0::NTMP : L1::IN * L1::NTMP;
  static_assert(CB % 2 == 0 && L0::NTMP % 2 == 0 && L1::NTMP % 2 == 0, "8-byte pair stores into the cb table");
  // PF: features are adjoint-free, so they are formed for two evaluations at once (ev on lanes
  // [0, FH) of a trajectory's half, ev - 1 on [FH, HALF)) every other evaluation, into LDS buffers
  // indexed by evaluation parity: the per-input phase's instructions serve twice the lanes.  Only
  // the Ferro sweep with sums pairs them (the others would lose occupancy to the second buffer).
  constexpr bool PF = FERRO && ACC && 2 * W <= HALF;
  constexpr int FH = PF ? HALF / 2 : HALF, NBUF = PF ? 2 : 1;
  static_assert(W <= FH && (TPW == 1 || TPW == 2 || TPW == 4), "one lane per input of each trajectory and evaluation");
  __shared__ BInTab<W, NG, NB> TI;
  __shared__ BTab<L0> T0;
  __shared__ BTab<L1> T1;
  using FB = BFeat<W, NS, NB, PF>;
  __shared__ FB sF[kTPB][NBUF][TPW];
  __shared__ __attribute__((aligned(16))) float s_cb[kTPB][TPW][CB];  // f2 stores (pairs)
  __shared__ float s_g1[kTPB][TPW][D], s_g0[kTPB][TPW][H], s_gx[kTPB][TPW][D];
  __shared__ float s_ak[kTPB][TPW][4][D], s_ay[kTPB][TPW][D], s_ac[kTPB][4][3];

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tt = lane / HALF, sl = lane % HALF;  // this lane's trajectory in the per-input phases
  const int fb = sl / FH, fsl = sl % FH;          // feature lanes: evaluation ev - fb, input fsl
  TI.stage(a.plan, a.P0, a.P1, D, threadIdx.x, 64 * kTPB);
  T0.stage(a.k0, a.f0, a.plan, a.P0, threadIdx.x, 64 * kTPB);
  T1.stage(a.k1, a.f1, a.plan, a.P1, threadIdx.x, 64 * kTPB);
  BReg<L0> R0;
  BReg<L1> R1;
  if constexpr (ACC) {
    R0.zero();
    R1.zero();
  }
  __syncthreads();  // tables staged; from here on every wave syncs only with itself

  float* cbs = &s_cb[wid][0][0];
  float* g1s = &s_g1[wid][0][0];  // layer-1 output adjoint = d loss / d k_stage
  float* g0s = &s_g0[wid][0][0];  // layer-0 output adjoint = d loss / d h
  float* gxs = &s_gx[wid][0][0];
  float(&ak)[4][D] = s_ak[wid][tt];
  float(&ay)[D] = s_ay[wid][tt];
  float(&acs)[4][3] = s_ac[wid];
  const float gs0 = (float)a.f0.gate_slope, gs1 = (float)a.f1.gate_slope;
  const float gl0 = a.P0.gsl2e, gl1 = a.P1.gsl2e, wc0 = a.P0.wc, wc1 = a.P1.wc;
  const float glane = fsl < D ? gl0 : gl1, wlane = fsl < D ? wc0 : wc1, slane = fsl < D ? gs0 : gs1;  // the feature lane's layer
  const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  const int64_t tstride = a.B * W;
  const int n_ev = a.n_steps * ns;

  for (int64_t b0 = ((int64_t)blockIdx.x * kTPB + wid) * TPW; b0 < a.B; b0 += (int64_t)gridDim.x * kTPB * TPW) {
    // this lane's trajectory; a missing partner (B odd) runs on zeros: finite inputs, zero
    // adjoints, exact-zero contributions to every sum
    const int64_t b = b0 + tt;
    const bool live = b < a.B;
    const int64_t bc_ = live ? b : b0;
    // the hysteresis input of evaluation ev is the layer input of ev - 1 (ferro_class.py:409)
    // (any ev < 0 reads the state before the solve: the paired feature lanes of a last pair (0, -1)
    // fill a buffer nothing reads)
    auto tape_at = [&](int ev) -> float {
      if (fsl >= W || !live) return 0.f;
      if (ev >= 0) return a.tape[(int64_t)ev * tstride + b * W + fsl];
      const float v = a.tape[b * W + fsl];  // before evaluation 0: the stored state / reinit rule
      if (fsl < D) return (a.init_mask & 1u) ? v : (FERRO ? a.state0[b * D + fsl] : 0.f);
      return (a.init_mask & 2u) ? v : (FERRO ? a.state0[a.B * D + b * H + (fsl - D)] : 0.f);
    };
    // this feature lane's layer input and hysteresis input, for evaluation ev - fb of the next pair
    float cur = tape_at(n_ev - 1 - fb), prv = tape_at(n_ev - 2 - fb);
    float ay1 = 0.f;  // adjoint of y at the end of the current step (lanes sl < D)
    int jj = a.T - 1;
    for (int s = a.n_steps - 1; s >= 0; --s) {
      float bc[4], ac[4][3];
      step_coefs(a.method, a.step_coef[4 * s], a.step_coef[4 * s + 1], a.step_coef[4 * s + 2], bc, ac);
      // outputs produced in this step (FixedGridODESolver: y at step start, end, or interpolated)
      float ay0x = 0.f;
      for (; jj >= 1 && a.out_step[jj] == s; --jj) {
        if (sl < D) {
          const float g = live ? a.gsol[((int64_t)jj * a.B + bc_) * D + sl] : 0.f;
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
      if (sl < D) {
        for (int j = 0; j < ns; ++j) ak[j][sl] = bc[j] * ay1;
        ay[sl] = ay1 + ay0x;
      }
      if (lane == 0) {  // through LDS: the stage index below is a runtime value
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acs[i][j] = ac[i][j];
      }
      for (int st = ns - 1; st >= 0; --st) {
        const int ev = s * ns + st;
        // table reads are re-issued every evaluation (an opaque zero offset stops the compiler
        // from hoisting ~100 loop-invariant LDS values into VGPRs, which halves occupancy)
        int z = 0;
        asm volatile("" : "+s"(z));
        // features of evaluations ev and ev - 1 (every other evaluation; wave-uniform)
        const bool fstep = !PF || ((n_ev - 1 - ev) & 1) == 0;
        float nx1 = 0.f, nx2 = 0.f;
        FB& FF = sF[wid][PF ? (ev - fb) & 1 : 0][tt];
        if (fstep) {
          if constexpr (PF) {  // prefetch: consumed by the next pair
            nx1 = tape_at(ev - fb - 2);
            nx2 = tape_at(ev - fb - 3);
          } else {  // the next evaluation's layer input is this one's hysteresis input
            nx1 = prv;
            nx2 = tape_at(ev - 2);
          }
          if (fsl < W) {
            FF.x[fsl] = cur;
            FF.pv[fsl] = prv;
          }
        }
        if (sl < D) g1s[tt * D + sl] = ak[st][sl];
        wsync();
        if (fstep) {
          // both layers' inputs on one code path over the combined input index
          if (!(FETODE_EXP_SKIP & 8) && fsl < W) feat_input<W, NG, NB, PF>(FF, TI, fsl, glane, wlane, slane, z);
          if (!(FETODE_EXP_SKIP & 8)) {
            constexpr int NSG = TPW * W * NB, RSG = (NSG + 63) / 64;
#pragma unroll
            for (int pb = 0; pb < NBUF; ++pb) {  // one parity buffer at a time (register pressure)
              FB* Fp = sF[wid][pb];
              float sa[RSG], sb[RSG], sx[RSG];
#pragma unroll
              for (int k = 0; k < RSG; ++k) {  // every round's operands read before any sigmoid
                const int q = lane + 64 * k, qc = q < NSG ? q : 0;
                const int qt = qc / (W * NB), qq = qc % (W * NB);
                const float2 ab = *reinterpret_cast<const float2*>(&TI.lg[2 * qq + z]);  // one 8-byte read
                sa[k] = ab.x;
                sb[k] = ab.y;
                sx[k] = Fp[qt].x[qq / NB];
              }
#pragma unroll
              for (int k = 0; k < RSG; ++k) {
                const int q = lane + 64 * k;
                if (q < NSG) {
                  const int qt = q / (W * NB), qq = q % (W * NB);
                  Fp[qt].sg[qq] = sigm_l2(ffma(sa[k], sx[k], sb[k]));
                }
              }
            }
          }
          wsync();
          cur = nx1;
          prv = nx2;
        }
        FB* Fs = sF[wid][PF ? ev & 1 : 0];
        layer_jobs<L1, D, ACC, TPW, D, CB>(Fs, g1s, T1, TI.rh, R1, cbs, gl1, wc1, gs1, lane, z);
        wsync();
        reduce_gin<L1, TPW, H, CB>(cbs, g0s, lane);  // d loss / d h
        wsync();
        if constexpr (!ACC) {  // this evaluation's adjoints for param_sum_kernel
          if (live) {
            float* gr = a.gadj + ((int64_t)ev * a.B + b) * W;
            if (sl < D) gr[sl] = g1s[tt * D + sl];
            else if (sl < W) gr[sl] = g0s[tt * H + sl - D];
          }
        }
        layer_jobs<L0, 0, ACC, TPW, H, CB>(Fs, g0s, T0, TI.rh, R0, cbs, gl0, wc0, gs0, lane, z);
        wsync();
        reduce_gin<L0, TPW, D, CB>(cbs, gxs, lane);
        wsync();
        if (sl < D) {
          const float ax = gxs[tt * D + sl];
          ay[sl] += ax;
          for (int j = 0; j < st; ++j) ak[j][sl] = ffma(acs[st][j], ax, ak[j][sl]);
        }
        wsync();
      }
      ay1 = sl < D ? ay[sl] : 0.f;
    }
    if (sl < D && live && a.gy0) a.gy0[b * D + sl] = ay1 + a.gsol[b * D + sl];  // solution[0] = y0
    wsync();
  }
  if constexpr (ACC) {
    float* part = a.part + ((int64_t)blockIdx.x * kTPB + wid) * a.nacc;
    R0.template store<TPW>(part, lane);
    R1.template store<TPW>(part + L0::AL.n, lane);
  }
}

// =============================================================================================
// The reverse sweep of the device-resident dopri5 solve: loss.backward() through the reference's
// own training call, odeint(calDeriv, X0, t_learn) with torchdiffeq's default dopri5
// (train_kanfet_node_predprey.py:252-257), i.e. reverse-mode autograd through every evaluation of
// every attempt (rejected ones included), the stage sums, the error norm and the step-size
// control (rk_common._runge_kutta_step / _optimal_step_size, misc._select_initial_step /
// _rms_norm, interp._interp_fit / _interp_evaluate — nothing in torchdiffeq detaches dt).
//
// Tape (fetode_integrate_dopri5_tape): per evaluation its two layer inputs (as the fixed-grid
// tape) and its output k; per attempt (t0, dt, error ratio, accepted); the initial-step scalars.
// Evaluation order: 0 = f(y0), 1 = the initial-step probe (absent with first_step), then six per
// attempt (stages 2..7; stage 7's input is the attempt's y1, its output the next f0).
//
// One wave owns TPW trajectories and walks the evaluations backwards exactly like
// fixed_bwd_kernel (same per-evaluation VJP, gradient sums in VGPRs); the lanes sl < D of a
// trajectory carry its state adjoints.  The adjoint of dt couples the batch (the error ratio is a
// norm over every element), so every attempt ends with one grid-wide fixed-order fp64 sum
// (grid_sum2) of the per-element d/d dt terms — the whole grid is resident.  Per attempt n, in
// reverse, with dt_{n+1}'s adjoint known:
//   control   dt_{n+1} = clamp(dt_n * min(ifactor, max(safety ratio^-1/5, dfactor)))
//             -> adjoint of ratio_n and dt_n's direct part
//   outputs   (accepted) every output t_i in (t0, t1]: the interpolant's coefficient adjoints and
//             d out/d x, x = (t_i - t0s)/(t1s - t0s) -> d/d t0, d/d dt (grid sums)
//   element   interp fit, error ratio (err / tol, tol = atol + rtol max(|y|, |y1|)) and the stage
//             sums -> adjoints of k_1..k_7, y and dt; evaluations 7..2 by VJP
//   carry     y's adjoint and f0's (= k_1's) to the attempt that produced them
// After attempt 0: _select_initial_step's adjoint (one more grid sum, through the probe).
// =============================================================================================
struct DopriBwdArgs {
  BwdArgs b;            // plan, layers, B, T, gsol, tape ((n_ev, B, 2 D + H): inputs, output), state0, ...
  const double* att;    // (n_att, 4): t0, dt, error ratio, accepted
  int32_t n_att, n_ev, base;  // base: evaluation index of attempt 0's stage 2 (1 with first_step, else 2)
  const double* t;      // (T) output times, fp64
  const double* init_rec;  // {d0, d1, d2, h0, h1}
  float beta[6][6], cerr[7], cmid[7];
  float rtol, atol;
  double safety, ifactor, dfactor, min_step, max_step, n_el;
  DopriParams gp;       // the grid-sum words and leaf layout (single device)
  int32_t* status;      // 0, or 4 when a grid sum timed out
};

// a wave-uniform value computed on the VALU (or read from LDS) into SGPRs: it stays live across
// the evaluations' VJPs without holding VGPRs
__device__ __forceinline__ float unif(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, v)));
}
__device__ __forceinline__ double uni(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

template <int D, int H, int K, int NB, int NG, bool FERRO, int TPW>
__global__ __launch_bounds__(64 * kTPB) __attribute__((amdgpu_waves_per_eu(FETODE_BWD_WAVES))) void dopri_bwd_kernel(DopriBwdArgs da) {
  const BwdArgs& a = da.b;
  using L0 = BL<D, H, K, NB, NG, FERRO>;
  using L1 = BL<H, D, K, NB, NG, FERRO>;
  constexpr int W = D + H, NS = NG - 1 - kSO, HALF = 64 / TPW;
  constexpr int CB = L0::IN * L0::NTMP > L1::IN * L1::NTMP ? L0::IN * L0::NTMP : L1::IN * L1::NTMP;
  constexpr bool PF = FERRO && 2 * W <= HALF;
  constexpr int FH = PF ? HALF / 2 : HALF, NBUF = PF ? 2 : 1;
  static_assert(W <= FH && (TPW == 1 || TPW == 2 || TPW == 4), "one lane per input of each trajectory and evaluation");
  __shared__ BInTab<W, NG, NB> TI;
  __shared__ BTab<L0> T0;
  __shared__ BTab<L1> T1;
  using FB = BFeat<W, NS, NB, PF>;
  __shared__ FB sF[kTPB][NBUF][TPW];
  __shared__ __attribute__((aligned(16))) float s_cb[kTPB][TPW][CB];
  __shared__ float s_g1[kTPB][TPW][D], s_g0[kTPB][TPW][H], s_gx[kTPB][TPW][D];
  __shared__ float s_k[kTPB][TPW][8][D], s_kb[kTPB][TPW][8][D];  // k_1..k_7 and their adjoints
  __shared__ double s_red[kTPB][2], s_res[2];
  __shared__ int s_ab;
  // the element lanes' carried adjoints, kept in LDS across the VJPs (register pressure)
  struct ElSt {
    double pd, pt;          // this attempt's d/d dt and d/d t0 terms of the outputs (+ d/d dt32 at the end)
    float yb0, yb1, dtb32;  // adjoints of the attempt's y, y1, dt32
    float ybc, fbc;         // carried: adjoints of the current y and f0
    float scb, f0bp;        // initial step: adjoint of scale, the probe's term of f0's adjoint
  };
  __shared__ ElSt s_el[kTPB][TPW][D];
  // the tableau in LDS: kernel-argument reads with constant indices would be hoisted into ~50
  // SGPRs for the whole loop (the VJP needs the SGPR file)
  __shared__ float s_beta[6][6], s_cerr[8], s_cmid[8];
  // the wave-uniform control scalars, per wave in LDS: they are touched once per attempt and would
  // otherwise hold registers across every VJP (adjoints of the next dt and of t1s, ...)
  struct WSc {
    double dtbar, tbar, dtb_base, h0b, d0b, d1b;
    float dt32, h0f;
    int jj, acc;
  };
  __shared__ WSc s_sc[kTPB];
  // the arguments the per-attempt code reads, in LDS: read from the kernel arguments inside the
  // loop they would be hoisted into SGPRs (and spilled) for the whole sweep
  struct RareArgs {
    const double* att;
    const double* t;
    const float* gsol;
    float* gy0;
    const double* init_rec;
    int64_t B;
    int base, n_att;
    float rtol, atol;
    double n_el, safety, ifactor, dfactor, min_step, max_step;
  };
  __shared__ RareArgs s_ra;

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tt = lane / HALF, sl = lane % HALF;
  const int fb = sl / FH, fsl = sl % FH;
  TI.stage(a.plan, a.P0, a.P1, D, threadIdx.x, 64 * kTPB);
  T0.stage(a.k0, a.f0, a.plan, a.P0, threadIdx.x, 64 * kTPB);
  T1.stage(a.k1, a.f1, a.plan, a.P1, threadIdx.x, 64 * kTPB);
  BReg<L0> R0;
  BReg<L1> R1;
  R0.zero();
  R1.zero();
  if (threadIdx.x == 0) {
    s_ab = 0;
    s_ra = RareArgs{da.att, da.t, a.gsol, a.gy0, da.init_rec, a.B, da.base, da.n_att, da.rtol, da.atol,
                    da.n_el, da.safety, da.ifactor, da.dfactor, da.min_step, da.max_step};
#pragma unroll
    for (int q = 0; q < 36; ++q) s_beta[q / 6][q % 6] = da.beta[q / 6][q % 6];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      s_cerr[q] = da.cerr[q];
      s_cmid[q] = da.cmid[q];
    }
  }
  __syncthreads();

  float* cbs = &s_cb[wid][0][0];
  float* g1s = &s_g1[wid][0][0];
  float* g0s = &s_g0[wid][0][0];
  float* gxs = &s_gx[wid][0][0];
  float(&kk)[8][D] = s_k[wid][tt];
  float(&kb)[8][D] = s_kb[wid][tt];
  const float gs0 = (float)a.f0.gate_slope, gs1 = (float)a.f1.gate_slope;
  const float gl0 = a.P0.gsl2e, gl1 = a.P1.gsl2e, wc0 = a.P0.wc, wc1 = a.P1.wc;
  const float glane = fsl < D ? gl0 : gl1, wlane = fsl < D ? wc0 : wc1, slane = fsl < D ? gs0 : gs1;
  constexpr int TW = 2 * D + H;  // tape row: layer-0 input, layer-1 input, output k
  const int64_t tstride = a.B * TW;
  const int n_ev = da.n_ev;
  const int64_t b0 = ((int64_t)blockIdx.x * kTPB + wid) * TPW;
  const int64_t b = b0 + tt;
  const bool live = b < a.B;
  const bool el = live && sl < D;  // this lane carries element (b, sl)
  // per-lane offsets in 32 bits, row bases uniform (scalar base + vector offset addressing)
  const int bi = live ? (int)b : 0;
  auto tape_at = [&](int ev) -> float {
    if (fsl >= W || !live) return 0.f;
    if (ev >= 0) return (a.tape + (int64_t)ev * tstride)[bi * TW + fsl];
    const float v = a.tape[bi * TW + fsl];
    if (fsl < D) return (a.init_mask & 1u) ? v : (FERRO ? a.state0[bi * D + fsl] : 0.f);
    return (a.init_mask & 2u) ? v : (FERRO ? (a.state0 + a.B * D)[bi * H + (fsl - D)] : 0.f);
  };
  auto tx = [&](int ev) -> float { return (a.tape + (int64_t)ev * tstride)[bi * TW + sl]; };      // layer input (el lanes)
  auto tk = [&](int ev) -> float { return (a.tape + (int64_t)ev * tstride)[bi * TW + W + sl]; };  // output (el lanes)
  float cur = tape_at(n_ev - 1 - fb), prv = tape_at(n_ev - 2 - fb);

  // the VJP of evaluation ev: g1s (d loss / d k) -> gxs (d loss / d layer-0 input); sums into R0, R1
  auto vjp = [&](int ev) {
    int z = 0;
    asm volatile("" : "+s"(z));
    const bool fstep = !PF || ((n_ev - 1 - ev) & 1) == 0;
    float nx1 = 0.f, nx2 = 0.f;
    FB& FF = sF[wid][PF ? (ev - fb) & 1 : 0][tt];
    if (fstep) {
      if constexpr (PF) {
        nx1 = tape_at(ev - fb - 2);
        nx2 = tape_at(ev - fb - 3);
      } else {
        nx1 = prv;
        nx2 = tape_at(ev - 2);
      }
      if (fsl < W) {
        FF.x[fsl] = cur;
        FF.pv[fsl] = prv;
      }
    }
    wsync();
    if (fstep) {
      if (fsl < W) feat_input<W, NG, NB, PF>(FF, TI, fsl, glane, wlane, slane, z);
      constexpr int NSG = TPW * W * NB, RSG = (NSG + 63) / 64;
#pragma unroll
      for (int pb = 0; pb < NBUF; ++pb) {
        FB* Fp = sF[wid][pb];
        float sa[RSG], sb[RSG], sx[RSG];
#pragma unroll
        for (int k = 0; k < RSG; ++k) {
          const int q = lane + 64 * k, qc = q < NSG ? q : 0;
          const int qt = qc / (W * NB), qq = qc % (W * NB);
          const float2 ab = *reinterpret_cast<const float2*>(&TI.lg[2 * qq + z]);
          sa[k] = ab.x;
          sb[k] = ab.y;
          sx[k] = Fp[qt].x[qq / NB];
        }
#pragma unroll
        for (int k = 0; k < RSG; ++k) {
          const int q = lane + 64 * k;
          if (q < NSG) {
            const int qt = q / (W * NB), qq = q % (W * NB);
            Fp[qt].sg[qq] = sigm_l2(ffma(sa[k], sx[k], sb[k]));
          }
        }
      }
      wsync();
      cur = nx1;
      prv = nx2;
    }
    FB* Fs = sF[wid][PF ? ev & 1 : 0];
    layer_jobs<L1, D, true, TPW, D, CB>(Fs, g1s, T1, TI.rh, R1, cbs, gl1, wc1, gs1, lane, z);
    wsync();
    reduce_gin<L1, TPW, H, CB>(cbs, g0s, lane);
    wsync();
    layer_jobs<L0, 0, true, TPW, H, CB>(Fs, g0s, T0, TI.rh, R0, cbs, gl0, wc0, gs0, lane, z);
    wsync();
    reduce_gin<L0, TPW, D, CB>(cbs, gxs, lane);
    wsync();
  };

  // grid-wide fixed-order sum of two per-lane fp64 values (every workgroup gets the same result)
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
#pragma unroll
      for (int w = 1; w < kTPB; ++w) {
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

  ElSt& E = s_el[wid][tt][sl < D ? sl : 0];  // written by lanes sl < D only
  if (sl < D) {
    E.ybc = E.fbc = 0.f;
    E.scb = E.f0bp = 0.f;
  }
  // wave-uniform scalars (SGPRs): adjoints of the next dt and of t1s, this attempt's control terms
  WSc& C = s_sc[wid];  // every lane writes the same values
  C.dtbar = C.tbar = C.dtb_base = C.h0b = C.d0b = C.d1b = 0.0;
  C.jj = a.T - 1;  // the last output not yet taken
  C.dt32 = C.h0f = 0.f;
  C.acc = 0;

  for (int ev = n_ev - 1; ev >= 0; --ev) {
    const bool in_att = ev >= s_ra.base;
    const int n = in_att ? (ev - s_ra.base) / 6 : -1, s = in_att ? 2 + (ev - s_ra.base) % 6 : 0;
    // ---------------- before the VJP: this evaluation's output adjoint ----------------
    if (in_att && s == 7) {
      const double t0 = s_ra.att[4 * n], dt = s_ra.att[4 * n + 1];
      const float ratio = (float)s_ra.att[4 * n + 2];
      C.acc = s_ra.att[4 * n + 3] != 0.0;
      int m = n - 1;  // the attempt whose stage 7 produced this attempt's y and f0
      while (m >= 0 && s_ra.att[4 * m + 3] == 0.0) --m;
      const int fe = m >= 0 ? s_ra.base + 6 * m + 5 : 0;
      const int e2 = s_ra.base + 6 * n;
      C.dt32 = ((float)dt);
      // control: dt_{n+1} = clamp(dt * min(ifactor, max(safety ratio^-1/5, dfac))) (rk_common.
      // _optimal_step_size, fp64).  The factor the forward took is dt_{n+1} / dt_n from the attempt
      // log, so no pow here: the middle term was taken unless the factor sits on a bound (or the
      // clamp did), and its derivative is -factor / (5 ratio).  The last attempt's next dt feeds
      // nothing (its adjoint is 0).
      const double rr = (double)ratio;
      double rbar = 0.0, dtbb = 0.0;
      if (n + 1 < s_ra.n_att) {
        const double dtn1 = s_ra.att[4 * (n + 1) + 1];
        const bool clamped = (s_ra.min_step > 0.0 && dtn1 == s_ra.min_step) || dtn1 == s_ra.max_step;
        if (!clamped) {
          const double fac = dtn1 / dt;
          dtbb = C.dtbar * fac;
          if (rr > 0.0) {
            const double dfac = rr < 1.0 ? 1.0 : s_ra.dfactor;
            const bool bound = fabs(fac - s_ra.ifactor) <= 1e-12 * s_ra.ifactor || fabs(fac - dfac) <= 1e-12 * dfac;
            if (!bound) rbar = C.dtbar * dt * (-0.2 * fac / rr);
          }
        }
      }
      C.dtb_base = dtbb;
      double pd = 0.0, pt = 0.0;
      float dtb32 = 0.f, yb0, yb1;
      const float ybc = sl < D ? E.ybc : 0.f, fbc = sl < D ? E.fbc : 0.f;
      float kv[8], kbv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kv[j] = kbv[j] = 0.f;
      float y = 0.f, y1 = 0.f;
      if (el) {
        y = tx(fe);
        kv[1] = tk(fe);
#pragma unroll
        for (int j = 2; j <= 7; ++j) kv[j] = tk(e2 + j - 2);
        y1 = tx(e2 + 5);
      }
      // err and mid in the forward's op order (fetode_fused.hip DOPRI)
      float err = kv[1] * (s_cerr[0] * C.dt32), midv = kv[1] * (s_cmid[0] * C.dt32);
#pragma unroll
      for (int j = 2; j <= 7; ++j) {
        err = err + kv[j] * (s_cerr[j - 1] * C.dt32);
        midv = midv + kv[j] * (s_cmid[j - 1] * C.dt32);
      }
      float midb = 0.f, fab;
      if (C.acc) {
        yb1 = ybc;
        kbv[7] = fbc;
        yb0 = 0.f;
        fab = 0.f;
        // interp._interp_fit (fetode_fused.hip's op order)
        const float ym = y + midv, fa = kv[1], fbk = kv[7];
        const float co1 = C.dt32 * fa;
        const float co2 = ((C.dt32 * (fbk - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
        const float co3 = ((C.dt32 * (5.0f * fa - 3.0f * fbk) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
        const float co4 = ((2.0f * C.dt32) * (fbk - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, c4 = 0.f;
        const double t1 = t0 + dt, dlt = t1 - t0;
        for (; C.jj >= 1 && s_ra.t[C.jj] > t0; --C.jj) {  // outputs in (t0, t1]: uniform over the grid
          const float x = (float)((s_ra.t[C.jj] - t0) / dlt);
          const float g = el ? (s_ra.gsol + (int64_t)C.jj * a.B * D)[bi * D + sl] : 0.f;
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
      // error ratio = rms(err / tol): d ratio / d qe = qe / (N ratio)
      float errb = 0.f;
      if (rbar != 0.0 && ratio > 0.f) {
        const float tol = s_ra.atol + s_ra.rtol * fmaxf(fabsf(y), fabsf(y1));
        const float qe = err / tol;
        const float qb = (float)(rbar * (double)qe / (s_ra.n_el * rr));
        errb = qb / tol;
        const float tolb = -qb * qe / tol, ay = fabsf(y), ay1 = fabsf(y1);
        const float sy = y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f), sy1 = y1 > 0.f ? 1.f : (y1 < 0.f ? -1.f : 0.f);
        const float wy = ay > ay1 ? 1.f : (ay < ay1 ? 0.f : 0.5f);
        yb0 += tolb * s_ra.rtol * wy * sy;
        yb1 += tolb * s_ra.rtol * (1.f - wy) * sy1;
      }
      float se = 0.f, sm = 0.f;
#pragma unroll
      for (int j = 1; j <= 7; ++j) {
        kbv[j] += errb * (s_cerr[j - 1] * C.dt32) + midb * (s_cmid[j - 1] * C.dt32);
        se += s_cerr[j - 1] * kv[j];
        sm += s_cmid[j - 1] * kv[j];
      }
      dtb32 += errb * se + midb * sm;
      if (sl < D) {
#pragma unroll
        for (int j = 1; j <= 7; ++j) {
          kk[j][sl] = kv[j];
          kb[j][sl] = kbv[j];
        }
        E.pd = pd;
        E.pt = pt;
        E.yb0 = yb0;
        E.yb1 = yb1;
        E.dtb32 = dtb32;
      }
    } else if (!in_att && ev == 1) {
      // _select_initial_step (dopri5.py select_initial_step, fp32): dt0 = min(100 h0, h1)
      const float d0 = (float)s_ra.init_rec[0], d1 = (float)s_ra.init_rec[1], d2 = (float)s_ra.init_rec[2];
      const float h0 = (float)s_ra.init_rec[3], h1 = (float)s_ra.init_rec[4];
      C.h0f = (h0);
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
      if (d1 <= 1e-15f && d2 <= 1e-15f) {  // h1 = max(1e-6, h0 1e-3)
        const float v = h0 * 1e-3f;
        if (v > 1e-6f) C.h0b += 1e-3 * h1b;
        else if (v == 1e-6f) C.h0b += 0.5e-3 * h1b;
      } else {  // h1 = (0.01 / max(d1, d2)) ** (1/5); Python's max keeps d1 on a tie
        const bool take2 = d2 > d1;
        const double mx = take2 ? d2 : d1, base = 0.01 / mx;
        const double mxb = -(h1b * 0.2 * (double)h1 / base) * base / mx;
        if (take2) d2b += mxb;
        else d1b_ += mxb;
      }
      // d2 = |rms((f1 - f0) / scale) / h0|
      const double r2 = (double)d2 * h0, r2b = d2b / h0;
      C.h0b = (C.h0b - d2b * d2 / h0);
      C.d1b = (d1b_);
      float f1b = 0.f, f0bp = 0.f, scb = 0.f;
      if (el && r2 > 0.0) {
        const float y = tx(0), f0 = tk(0), f1 = tk(1);
        const float scale = s_ra.atol + fabsf(y) * s_ra.rtol;
        const float q2 = (f1 - f0) / scale;
        const float q2b = (float)(r2b * (double)q2 / (s_ra.n_el * r2));
        f1b = q2b / scale;
        f0bp = -q2b / scale;
        scb = -q2b * q2 / scale;
      }
      if (sl < D) {
        kb[0][sl] = f1b;
        E.f0bp = f0bp;
        E.scb = scb;
      }
      C.d0b = 0.0;
      (void)d0;
    } else if (ev == 0) {
      if (s_ra.base == 2) {  // the rest of _select_initial_step: d0 = rms(y0 / scale), d1 = rms(f0 / scale)
        const float d0 = (float)s_ra.init_rec[0], d1 = (float)s_ra.init_rec[1];
        if (el) {
          const float y = tx(0), f0 = tk(0);
          const float scale = s_ra.atol + fabsf(y) * s_ra.rtol;
          const float q0 = y / scale, q1 = f0 / scale;
          const float q0b = d0 > 0.f ? (float)(C.d0b * (double)q0 / (s_ra.n_el * d0)) : 0.f;
          const float q1b = d1 > 0.f ? (float)(C.d1b * (double)q1 / (s_ra.n_el * d1)) : 0.f;
          const float scb = E.scb - q0b * q0 / scale - q1b * q1 / scale;
          const float sy = y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f);
          E.ybc += q0b / scale + scb * s_ra.rtol * sy;
          E.fbc += q1b / scale;
        }
      }
      if (sl < D) kb[0][sl] = el ? E.fbc : 0.f;
    }
    // this evaluation's output adjoint -> the layer-1 output slots
    if (sl < D) g1s[tt * D + sl] = in_att ? kb[s][sl] : kb[0][sl];
    vjp(ev);
    // ---------------- after the VJP: the input adjoint ----------------
    const float xb = sl < D ? gxs[tt * D + sl] : 0.f;
    if (in_att) {
      double v0 = 0.0, v1 = 0.0;
      if (sl < D) {
        const float X = xb + (s == 7 ? E.yb1 : 0.f);  // stage 7's input IS y1
        E.yb0 += X;
        float sb = 0.f;
        for (int j = 1; j < s; ++j) {  // tableau row s - 2
          const float c = s_beta[s - 2][j - 1];
          kb[j][sl] += (c * C.dt32) * X;
          sb += c * kk[j][sl];
        }
        E.dtb32 += X * sb;
        if (s == 2) {  // attempt n done: the carries
          E.ybc = el ? E.yb0 : 0.f;
          E.fbc = el ? kb[1][sl] : 0.f;
          v0 = el ? E.pd + (double)E.dtb32 : 0.0;
          v1 = el ? E.pt : 0.0;
        }
      }
      if (s == 2) {  // the grid sum of the attempt's d/d dt and d/d t0 terms
        double S0, S1;
        gsum(v0, v1, S0, S1);
        C.dtbar = (C.dtb_base + (C.acc ? C.tbar : 0.0) + S0);
        C.tbar = (C.tbar + S1);
      }
    } else if (ev == 1) {  // the probe: input y0 + h0 f0
      const float f0 = el ? tk(0) : 0.f;
      if (el) {
        E.ybc += xb;
        E.fbc += xb * C.h0f + E.f0bp;
      }
      double S0, S1;
      gsum(el ? (double)(xb * f0) : 0.0, 0.0, S0, S1);
      C.h0b = (C.h0b + S0);
      const float d0 = (float)s_ra.init_rec[0], d1 = (float)s_ra.init_rec[1];
      if (!(d0 < 1e-5f || d1 < 1e-5f)) {  // h0 = |0.01 d0 / d1|
        C.d0b = (C.h0b * 0.01 / d1);
        C.d1b = (C.d1b - C.h0b * (double)C.h0f / d1);
      }
    } else {  // evaluation 0: f(y0)
      if (el) {
        E.ybc += xb;
        if (s_ra.gy0) s_ra.gy0[bi * D + sl] = E.ybc + s_ra.gsol[bi * D + sl];  // solution[0] = y0
      }
    }
  }
  float* part = a.part + ((int64_t)blockIdx.x * kTPB + wid) * a.nacc;
  R0.template store<TPW>(part, lane);
  R1.template store<TPW>(part + L0::AL.n, lane);
  if (blockIdx.x == 0 && threadIdx.x == 0)
    da.status[0] = (s_ab || __hip_atomic_load(dp_abort(da.gp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 4 : 0;
}

// Parameter-gradient sums of one layer from the recorded adjoints (after fixed_bwd_kernel<ACC =
// false>): every sample (evaluation ev, trajectory b) is independent, so the sums are formed
// element-major — a thread owns fixed jobs of the layer (a Ferro element, a KAN edge, one or two
// logistic (input, basis) pairs) with their sums in a few VGPRs, and walks its block's samples in
// tiles of TS whose per-input features (SiLU, dense B-spline bases, hysteresis gate, logistic
// sigmoids) are computed once per tile into LDS.  The per-sample arithmetic is layer_jobs'; only
// the summation order differs (per block, samples in (ev, b) order; blocks in a fixed order).
// Jobs (256 threads): Ferro element e = tid (E = 200); edge q = tid - E (NE = 20; the i = 0 edge of
// output o also sums G_o); logistic (i, j) jobs tid - E - NE and, if NL exceeds what is left, a
// second one on threads 0.. (L1: 36 + 64 of 100).
// FE = false (after sweep7_kernel, which keeps the Ferro sums itself): the KAN sums only — no
// hysteresis inputs fetched, no Ferro jobs (edges on threads 0.., logistic jobs after them), the
// Ferro slots of the block's row written as zeros.
constexpr int kPsTS = 32;  // samples per tile
template <int D, int H, int K, int NB, int NG, int LAYER, bool FE = true>
__global__ __launch_bounds__(256) void param_sum_kernel(BwdArgs a) {
  using LA = BL<D, H, K, NB, NG, true>;
  using LB = BL<H, D, K, NB, NG, true>;
  using L = typename std::conditional<LAYER == 0, LA, LB>::type;
  constexpr int W = D + H, NS = NG - 1 - kSO, NI = NG - 1, TS = kPsTS;
  constexpr int IN = L::IN, OUT = L::OUT, E = L::E, NE = L::NE, NL = L::NL;
  constexpr int TB = LAYER == 0 ? 0 : D;          // the layer's inputs in a tape row
  constexpr int GB = LAYER == 0 ? D : 0;          // its output adjoints in a gadj row (h | k)
  constexpr int EJ = FE ? E : 0;                   // Ferro jobs of this launch
  constexpr int J1 = 256 - EJ - NE;                // logistic jobs of the first round
  static_assert(EJ + NE <= 256 && NL <= J1 + 64 && (NL <= J1 || NL - J1 <= EJ), "param_sum job map");
  constexpr AccLayout AL = L::AL;
  __shared__ BInTab<W, NG, NB> TI;
  __shared__ BTab<L> Tb;
  __shared__ float sx[TS][IN], sup[TS][IN], ssl[TS][IN], sgo[TS][OUT];
  __shared__ float sbd[TS][IN][NS + 1];            // +1: no bank aliasing between inputs
  __shared__ float ssg[TS][IN * NB];
  const int tid = threadIdx.x;
  const LayerPlan& P = LAYER == 0 ? a.P0 : a.P1;
  TI.stage(a.plan, a.P0, a.P1, D, tid, 256);
  Tb.stage(LAYER == 0 ? a.k0 : a.k1, LAYER == 0 ? a.f0 : a.f1, a.plan, P, tid, 256);
  const float gsl = P.gsl2e, wc = P.wc, gs = (float)(LAYER == 0 ? a.f0.gate_slope : a.f1.gate_slope);
  const uint32_t imask = (a.init_mask >> LAYER) & 1u;
  const int64_t N = (int64_t)a.n_steps * (a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4
                                          : a.method == FETODE_MIDPOINT ? 2 : 1) * a.B;
  const int64_t n0 = (int64_t)blockIdx.x * N / gridDim.x, n1 = (int64_t)(blockIdx.x + 1) * N / gridDim.x;
  __syncthreads();

  // this thread's jobs and their constants
  const bool fjob = tid < EJ;
  const int e = fjob ? tid : 0, fi = e / (OUT * K), fo = (e % (OUT * K)) / K;
  const float4 fpa = Tb.fpa[e >> 1];
  const float fEc = (e & 1) ? fpa.y : fpa.x, fk2 = (e & 1) ? fpa.w : fpa.z;  // Ec, 2 log2e k
  const bool ejob = tid >= EJ && tid < EJ + NE;
  const int q = ejob ? tid - EJ : 0, eo = q / IN, ei = q % IN;
  const int lq0 = tid - EJ - NE;
  const bool ljob0 = lq0 >= 0 && lq0 < NL;
  const bool ljob1 = NL > J1 && tid < NL - J1;
  const int l0 = ljob0 ? lq0 : 0, l1 = ljob1 ? J1 + tid : 0;
  float A = 0.f, C = 0.f, Ev = 0.f, G = 0.f, base = 0.f, spl[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c) spl[c] = 0.f;
  float lw0[OUT], lw1[OUT], la0 = 0.f, lb0 = 0.f, la1 = 0.f, lb1 = 0.f;
#pragma unroll
  for (int o = 0; o < OUT; ++o) lw0[o] = lw1[o] = 0.f;
  auto logistic = [&](int ql, int s, float* lw, float& la, float& lb) __attribute__((always_inline)) {
    const int i = ql / NB, j = ql % NB;
    const float sg = ssg[s][ql], ds = sg * (1.0f - sg), x = sx[s][i];
    float S = 0.f;
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const float go = sgo[s][o];
      S = ffma(go, Tb.kw[o * (IN * L::NFL) + i * L::NFL + 1 + j], S);
      lw[o] = ffma(go, sg, lw[o]);
    }
    const float T = S * ds;
    la = ffma(T, x - Tb.pb[ql], la);
    lb = ffma(-T, Tb.pa[ql], lb);
  };

  // the tile's raw inputs (x, prev, output adjoints) are fetched one tile ahead, into registers,
  // while the current tile's jobs run
  constexpr int KI = (TS * IN + 255) / 256, KO = (TS * OUT + 255) / 256;
  float px[KI], pp[KI], pg[KO];
  auto fetch = [&](int64_t tt) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int it = tid + 256 * k, s = it / IN, i = it % IN;
      const int64_t n = tt + s;
      px[k] = pp[k] = 0.f;
      if (it < TS * IN && n < n1) {
        const int64_t ev = n / a.B;
        px[k] = a.tape[n * W + TB + i];
        if (!FE) continue;  // no hysteresis input without the Ferro jobs
        if (ev > 0) pp[k] = a.tape[(n - a.B) * W + TB + i];
        else if (!imask) pp[k] = a.state0[(LAYER == 0 ? (n % a.B) * D : a.B * D + (n % a.B) * H) + i];
        else pp[k] = px[k];  // the tape_at(-1) rule: first call, dx = 0
      }
    }
#pragma unroll
    for (int k = 0; k < KO; ++k) {
      const int it = tid + 256 * k, s = it / OUT, o = it % OUT;
      pg[k] = (it < TS * OUT && tt + s < n1) ? a.gadj[(tt + s) * W + GB + o] : 0.f;
    }
  };
  fetch(n0);
  for (int64_t t0 = n0; t0 < n1; t0 += TS) {
    // ---- per-tile features (one thread per (sample, input)) ----
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int it = tid + 256 * k;
      if (it >= TS * IN) break;
      const int s = it / IN, i = it % IN, t = TB + i;
      const float x = px[k], pv = pp[k];
      // SiLU, interval, dense bases and gate: feat_input's arithmetic
      const float sx_ = sigm_l2(-x * FETODE_LOG2E);
      ssl[s][i] = x * sx_;
      int m = -1;
#pragma unroll
      for (int jj = 0; jj < NG; ++jj) m += (x >= TI.knots[t * NG + jj]) ? 1 : 0;
      const bool fin = __builtin_isfinite(x);
      const bool in = fin && m >= 0 && m < NI;
      const int mc = in ? m : 0;
      const float u = in ? (x - TI.knots[t * NG + mc]) * TI.rh[t * NI + mc] : (fin ? 0.f : __builtin_nanf(""));
      const float fill = fin ? 0.f : __builtin_nanf("");
      float bd[NS];
#pragma unroll
      for (int c = 0; c < NS; ++c) bd[c] = fill;
      if (in) {
#pragma unroll
        for (int r = 0; r <= kSO; ++r) {
          const int c = mc - kSO + r;
          const float4 p = TI.bp[TI.bpi(t, mc) + r];
          const float v = ffma(ffma(ffma(p.w, u, p.z), u, p.y), u, p.x);
#pragma unroll
          for (int cc = 0; cc < NS; ++cc) bd[cc] = cc == c ? v : bd[cc];
        }
      }
#pragma unroll
      for (int c = 0; c < NS; ++c) sbd[s][i][c] = bd[c];
      sx[s][i] = x;
      if (FE) sup[s][i] = sigm_l2(-gsl * (x - pv));
    }
#pragma unroll
    for (int k = 0; k < KO; ++k) {  // the layer's output adjoints
      const int it = tid + 256 * k;
      if (it < TS * OUT) sgo[it / OUT][it % OUT] = pg[k];
    }
    __syncthreads();  // sx of the tile (the logistic sigmoids read it)
    for (int it = tid; it < TS * IN * NB; it += 256) {
      const int s = it / (IN * NB), ql = it % (IN * NB), i = ql / NB;
      const int qq = (TB * NB) + ql;  // combined (t, j) index of the lg table
      ssg[s][ql] = sigm_l2(ffma(TI.lg[2 * qq], sx[s][i] , TI.lg[2 * qq + 1]));
    }
    __syncthreads();
    if (t0 + TS < n1) fetch(t0 + TS);
    // ---- jobs: each thread walks the tile's samples (all TS: samples past the block's range
    // have x = prev = 0 and zero adjoints, so they add exact zeros; unrolled for ILP) ----
    if (fjob) {
#pragma unroll 4
      for (int s = 0; s < TS; ++s) {  // layer_jobs' Ferro element VJP, sums only
        const float x = sx[s][fi], up = sup[s][fi], go = sgo[s][fo];
        const float Ec = fEc;
        const float cn = sigm_l2(gsl * (x + Ec));
        const float omu = 1.0f - up;
        const float mm = ffma(wc, omu * cn, 1.0f);
        const float sh = ffma(Ec, mm, x);
        const float th = ffma(-2.0f, sigm_l2(fk2 * sh), 1.0f);
        const float qv = go * ffma(-th, th, 1.0f);
        A = ffma(go, th, A);
        C = ffma(qv, sh, C);
        const float dcn = gs * cn * (1.0f - cn);
        const float dmdEc = -wc * omu * dcn;
        Ev = ffma(qv, ffma(Ec, dmdEc, mm), Ev);
      }
    }
    if (ejob) {
#pragma unroll 4
      for (int s = 0; s < TS; ++s) {
        const float go = sgo[s][eo];
        base = ffma(go, ssl[s][ei], base);
#pragma unroll
        for (int c = 0; c < NS; ++c) spl[c] = ffma(go, sbd[s][ei][c], spl[c]);
        G += go;  // read only on the i = 0 edge of each output
      }
    }
    if (ljob0) {
#pragma unroll 4
      for (int s = 0; s < TS; ++s) logistic(l0, s, lw0, la0, lb0);
    }
    if (ljob1) {
#pragma unroll 4
      for (int s = 0; s < TS; ++s) logistic(l1, s, lw1, la1, lb1);
    }
    __syncthreads();
  }
  // ---- this block's partial row (the layer's half; the other launch writes the other half) ----
  float* part = a.part + (int64_t)blockIdx.x * a.nacc + (LAYER == 0 ? 0 : LA::AL.n);
  if (!FE) {
    for (int i = tid; i < 3 * E; i += 256) part[AL.oA + i] = 0.f;  // (oA, oC, oE: contiguous)
  }
  if (fjob) {
    part[AL.oA + e] = A;
    part[AL.oC + e] = C;
    part[AL.oE + e] = Ev;
  }
  if (ejob) {
    if (ei == 0) part[AL.oG + eo] = G;
    part[AL.oBase + q] = base;
#pragma unroll
    for (int c = 0; c < NS; ++c) part[AL.oSpl + q * NS + c] = spl[c];
  }
  if (ljob0) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) part[AL.oLw + o * NL + l0] = lw0[o];
    part[AL.oLa + l0] = la0;
    part[AL.oLb + l0] = lb0;
  }
  if (ljob1) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) part[AL.oLw + o * NL + l1] = lw1[o];
    part[AL.oLa + l1] = la1;
    part[AL.oLb + l1] = lb1;
  }
}

// partial rows -> chunk sums (fp64), fixed order
__global__ void part_reduce_kernel(const float* __restrict__ part, int64_t nrows, int nacc, int64_t per,
                                   double* __restrict__ out) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= nacc) return;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = r0 + per < nrows ? r0 + per : nrows;
  double s = 0.0;
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) s += part[r * nacc + slot];
  out[(int64_t)blockIdx.y * nacc + slot] = s;
}

// chunk sums -> S: four waves per 64 columns each sum a quarter of the chunks (loads issued
// together), then the four partials are added in a fixed order
constexpr int kChunkWaves = 4;
__global__ __launch_bounds__(64 * kChunkWaves) void chunk_sum_kernel(const double* __restrict__ ch, int nch, int nacc,
                                                                     double* __restrict__ S) {
  __shared__ double ps[kChunkWaves][64];
  const int w = threadIdx.x / 64, lane = threadIdx.x % 64, slot = blockIdx.x * 64 + lane;
  const int per = (nch + kChunkWaves - 1) / kChunkWaves, c0 = w * per, c1 = c0 + per < nch ? c0 + per : nch;
  double s = 0.0;
  if (slot < nacc) {
#pragma unroll 8
    for (int c = c0; c < c1; ++c) s += ch[(int64_t)c * nacc + slot];
  }
  ps[w][lane] = s;
  __syncthreads();
  if (w == 0 && slot < nacc) {
    double t = ps[0][lane];
#pragma unroll
    for (int k = 1; k < kChunkWaves; ++k) t += ps[k][lane];
    S[slot] = t;
  }
}

struct ApplyLayer {
  fetode_kanlinear_t kl;
  fetode_ferro_t fl;
  int has_ferro;
  AccLayout AL;
  fetode_kanlinear_grad_t kg;
  fetode_ferro_grad_t fg;
};

__device__ __forceinline__ void put(float* p, int64_t i, double v) {
  if (p) p[i] = (float)v;
}

// work items of one layer in grad_apply_kernel: elements / edges / logistic weights / logistic
// (a, b) pairs, padded to whole waves, then one wave per output for the logistic scalers
__host__ __device__ inline int apply_items(const ApplyLayer& L) {
  const AccLayout& A = L.AL;
  const int out = L.kl.out_features;
  const int n = (A.E + A.NE + out * A.NL + A.NL + 63) / 64 * 64;
  return n + (A.NL && L.kl.logistic_scaler ? 64 * out : 0);
}

// gradient sums of both layers -> parameter gradients (reference parameter layouts); 64-thread
// blocks never straddle a layer (apply_items pads), so the layer choice is wave-uniform
__global__ __launch_bounds__(64) void grad_apply_kernel(const double* __restrict__ S_, ApplyLayer L0_, ApplyLayer L1_,
                                                        int n0) {
  int t = blockIdx.x * 64 + threadIdx.x;
  const bool second = t >= n0;
  const ApplyLayer& L = second ? L1_ : L0_;
  const double* S = S_ + (second ? L0_.AL.n : 0);
  if (second) t -= n0;
  const AccLayout& A = L.AL;
  const int out = L.kl.out_features, NS = A.NS;
  const int nitems = (A.E + A.NE + out * A.NL + A.NL + 63) / 64 * 64;
  if (t >= nitems) {  // logistic scaler of output o: one wave, lanes over the NL weights, fixed-order tree
    const int o = (t - nitems) / 64, lane = (t - nitems) % 64;
    const double sl = L.kl.scale_logistic;
    double g = 0.0;
    for (int q = lane; q < A.NL; q += 64)
      g += 2.0 * S[A.oLw + o * A.NL + q] * (double)L.kl.logistic_weight[(int64_t)o * A.NL + q] * sl;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) g += __shfl_xor(g, m);
    if (lane == 0) put(L.kg.logistic_scaler, o, g);
    return;
  }
  if (t < A.E) {  // Ferro element e = (i, o, k)
    const int K = L.fl.num_basis, o = (t / K) % out;
    const double co = L.fl.coef[t], Ps = L.fl.Ps[t], kk = L.fl.k[t], bi = L.fl.bias[t];
    const double sA = S[A.oA + t], sC = S[A.oC + t], sE = S[A.oE + t], sG = S[A.oG + o];
    put(L.fg.k, t, co * Ps * sC);
    put(L.fg.Ec, t, co * Ps * kk * sE);
    put(L.fg.Ps, t, co * sA);
    put(L.fg.bias, t, co * sG);
    put(L.fg.coef, t, Ps * sA + bi * sG);
    return;
  }
  t -= A.E;
  if (t < A.NE) {  // KAN edge (o, i)
    put(L.kg.base_weight, t, S[A.oBase + t]);
    const double ss = L.kl.spline_scaler ? (double)L.kl.spline_scaler[t] : 1.0;
    double gsc = 0.0;
    for (int c = 0; c < NS; ++c) {
      const double d = S[A.oSpl + t * NS + c];
      put(L.kg.spline_weight, (int64_t)t * NS + c, d * ss);
      gsc += d * (double)L.kl.spline_weight[(int64_t)t * NS + c];
    }
    if (L.kl.spline_scaler) put(L.kg.spline_scaler, t, gsc);
    return;
  }
  t -= A.NE;
  if (A.NL == 0) return;
  if (t < out * A.NL) {  // logistic weight (o, i*NB + j); the basis is 2 sigmoid
    const int o = t / A.NL;
    const double ls = L.kl.logistic_scaler ? (double)L.kl.logistic_scaler[o] : 1.0;
    put(L.kg.logistic_weight, t, 2.0 * S[A.oLw + t] * L.kl.scale_logistic * ls);
    return;
  }
  t -= out * A.NL;
  if (t < A.NL) {
    put(L.kg.logistic_a, t, S[A.oLa + t]);
    put(L.kg.logistic_b, t, S[A.oLb + t]);
  }
}

#include "fetode_sweep7.h"
#include "fetode_kansum.h"

typedef void (*bwd_fn)(BwdArgs);
typedef void (*dopri_bwd_fn)(DopriBwdArgs);
struct BwdEntry {
  int D, H, K, NB, NG;
  bool ferro;
  int tpw;                     // trajectories per wave of fn (and of dopri)
  bwd_fn fn;                   // the one-kernel sweep (sums in VGPRs)
  bwd_fn adj, sum0, sum1;      // the split: adjoint sweep + per-layer parameter sums (or null)
  dopri_bwd_fn dopri;          // the reverse sweep of the resident dopri5 solve
  int dtpw;                    // its trajectories per wave (the whole batch is resident)
  dopri_bwd_fn dopri1;         // the same, one trajectory per wave: half the VJP jobs per lane
                               // (latency) where the batch leaves the grid room (small B)
  bwd_fn fn1;                  // fn at one trajectory per wave (small B), or null
  bwd_fn v7, v7s;              // the lane-group sweep (two trajectories per wave): Ferro sums + the
                               // recorded adjoints (then ks), or every sum in the sweep; or null
  bwd_fn ks;                   // the KAN sums over all samples after v7 (kansum_kernel)
};
const BwdEntry kBwd[] = {
    // LV KAN-FET [2,10,2]: one kernel, two trajectories per wave (measured: TPW 1 / 2 / 4 = 1034 / 897 /
    // 1203 us at B = 4096); the split structure as the alternative
#ifdef FETODE_DIAG   // the split structure (measured slower) lives in the diagnostic build only
    {2, 10, 10, 10, 12, true, 2, fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 2>,
     fixed_bwd_kernel<2, 10, 10, 10, 12, true, false, 1>, param_sum_kernel<2, 10, 10, 10, 12, 0>,
     param_sum_kernel<2, 10, 10, 10, 12, 1>, dopri_bwd_kernel<2, 10, 10, 10, 12, true, 2>, 2,
     dopri_bwd_kernel<2, 10, 10, 10, 12, true, 1>, fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 1>,
#else
    {2, 10, 10, 10, 12, true, 2, fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 2>, nullptr, nullptr, nullptr,
     dopri_bwd_kernel<2, 10, 10, 10, 12, true, 2>, 2, dopri_bwd_kernel<2, 10, 10, 10, 12, true, 1>,
     fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 1>,
#endif
     sweep7_kernel<false>, sweep7_kernel<true>, kansum_kernel},
    // LV KAN [2,10,2] (126 VGPRs: four waves per SIMD already)
    {2, 10, 0, 10, 12, false, 1, fixed_bwd_kernel<2, 10, 1, 10, 12, false, true, 1>, nullptr, nullptr, nullptr,
     dopri_bwd_kernel<2, 10, 1, 10, 12, false, 2>, 2, dopri_bwd_kernel<2, 10, 1, 10, 12, false, 1>, nullptr,
     nullptr, nullptr, nullptr},
};
// Which path the KAN-FET sweep takes (fetode_backward_set_split; env FETODE_BWD_SPLIT).  Default:
// the one-kernel sweep — measured on MI355X at B = 4096, rk4, 34 steps: one kernel 1.06 ms vs the
// split 0.69 (adjoint sweep) + 0.25 + 0.31 (layer sums) ms (profiles/r02_split_pmc.txt).
int g_bwd_split = -1;
bool use_split(const BwdEntry* e) {
  if (g_bwd_split < 0) {
    const char* v = getenv("FETODE_BWD_SPLIT");
    g_bwd_split = v ? atoi(v) != 0 : 0;
  }
  return e->adj && g_bwd_split != 0;
}
constexpr int64_t kSumBlocks = 1024;  // param_sum_kernel blocks per layer (= partial rows)
// The lane-group sweep (sweep7_kernel; fetode_backward_set_v7, env FETODE_BWD_V7):
// 0 = off, 1 = where the one-kernel sweep would run two trajectories per wave (the default),
// 2 = at every batch; + 4: the sweep keeps the Ferro sums only and records each evaluation's
// adjoints, kansum_kernel forms the KAN sums over all samples afterwards (measured at B = 4096:
// 386 + 109 us vs 496 us with every sum in the sweep — kansum recomputes the features; kept as
// the alternative).
int g_bwd_v7 = -1;
int v7_mode() {
  if (g_bwd_v7 < 0) {
    const char* v = getenv("FETODE_BWD_V7");
    g_bwd_v7 = v ? atoi(v) : 1;
  }
  return g_bwd_v7;
}
int64_t n_evals_of(int32_t method, int32_t n_steps) {
  return (int64_t)n_steps * (method == FETODE_RK4 || method == FETODE_RK4_CLASSIC ? 4 : method == FETODE_MIDPOINT ? 2 : 1);
}

const BwdEntry* find_bwd(const fetode_field_t* f) {
  if (f->n_layers != 2) return nullptr;
  const fetode_kanlinear_t &k0 = f->kan[0], &k1 = f->kan[1];
  if (k0.spline_order != kSO || k1.spline_order != kSO || k0.grid_size != k1.grid_size ||
      k0.num_logistic != k1.num_logistic || k0.in_features != k1.out_features)
    return nullptr;
  const int NG = k0.grid_size + 2 * kSO + 1;
  for (const BwdEntry& e : kBwd) {
    if (e.D != k0.in_features || e.H != k0.out_features || e.NB != k0.num_logistic || e.NG != NG) continue;
    if (e.ferro != (f->ferro != nullptr)) continue;
    if (f->ferro) {
      if (f->ferro[0].num_basis != e.K || f->ferro[1].num_basis != e.K) continue;
      if (f->ferro[0].branch_sign || f->ferro[1].branch_sign) continue;
    }
    return &e;
  }
  return nullptr;
}

constexpr int64_t kMaxBwdRows = 8192;  // partial rows (one per wave)
constexpr int kChunks = 64;
// one partial row per wave: the grid's waves, a multiple of kTPB
int64_t bwd_rows(int64_t B, int tpw) {
  const int64_t nw = (B + tpw - 1) / tpw;  // waves the trajectories need
  const int64_t w = nw < kMaxBwdRows ? nw : kMaxBwdRows;
  return (w + kTPB - 1) / kTPB * kTPB;
}

void layouts(const fetode_field_t* f, AccLayout* L0, AccLayout* L1) {
  const int NS = f->kan[0].grid_size + kSO;
  const int K = f->ferro ? f->ferro[0].num_basis : 0;
  const bool fe = f->ferro != nullptr;
  *L0 = acc_layout(f->kan[0].in_features, f->kan[0].out_features, K, f->kan[0].num_logistic, NS, fe);
  *L1 = acc_layout(f->kan[1].in_features, f->kan[1].out_features, K, f->kan[1].num_logistic, NS, fe);
}


// gradient sums S -> parameter gradients in the reference layouts (grad_apply_kernel)
int apply_grads(const fetode_field_t* f, const double* S, const AccLayout& AL0, const AccLayout& AL1,
                const fetode_kanlinear_grad_t* kan_grads, const fetode_ferro_grad_t* ferro_grads, hipStream_t s) {
  if (!kan_grads && !ferro_grads) return FETODE_OK;
  ApplyLayer L[2];
  for (int l = 0; l < 2; ++l) {
    memset(&L[l], 0, sizeof(ApplyLayer));
    L[l].kl = f->kan[l];
    if (f->ferro) L[l].fl = f->ferro[l];
    L[l].has_ferro = f->ferro != nullptr;
    L[l].AL = l == 0 ? AL0 : AL1;
    if (kan_grads) L[l].kg = kan_grads[l];
    if (ferro_grads && f->ferro) L[l].fg = ferro_grads[l];
  }
  const int n0 = apply_items(L[0]), n1 = apply_items(L[1]);
  hipLaunchKernelGGL(grad_apply_kernel, dim3((unsigned)((n0 + n1) / 64)), dim3(64), 0, s, S, L[0], L[1], n0);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // namespace

extern "C" {

int fetode_backward_set_split(int32_t enable) {
#ifndef FETODE_DIAG
  if (enable > 0) {   // the split sweep is compiled into the diagnostic build only
    set_err(FETODE_EUNSUPPORTED, "the split backward is a diagnostic path (make diag)");
    return -2;
  }
  return 0;
#else
  use_split(&kBwd[0]);  // resolve the env default first
  const int prev = g_bwd_split;
  if (enable >= 0) g_bwd_split = enable != 0;
  return prev;
#endif
}

int fetode_backward_set_v7(int32_t mode) {
  const int prev = v7_mode();
  if (mode >= 0) g_bwd_v7 = mode;
  return prev;
}

int fetode_fused_backward_supported(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return 0;
  return find_bwd(f) != nullptr || fieldn_shape_supported(f);
}

// the one-kernel sweep at one trajectory per wave while those waves fit one resident round
// (latency-bound small batches: half the VJP jobs per lane), else e->tpw
int fixed_tpw(const BwdEntry* e, int64_t B) {
  if (!e->fn1) return e->tpw;
  static int64_t cap = -1;
  if (cap < 0 && getenv("FETODE_BWD_TPW1") && atoi(getenv("FETODE_BWD_TPW1")) == 0) cap = 0;  // A/B knob
  if (cap < 0) {
    int dev = 0, n_cu = 0, per = 0;
    cap = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
           hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, e->fn1, 64 * kTPB, 0) == hipSuccess)
              ? (int64_t)per * n_cu * kTPB : 0;
  }
  // measured (tools/diag/bwd_small_time.py, rk4 iteration): B = 512 0.73 vs 0.93 ms, B = 2048 0.79 vs
  // 0.75 ms — one trajectory per wave while at most half the resident waves are needed
  return 2 * B <= cap ? 1 : e->tpw;
}

bool use_v7(const BwdEntry* e, int64_t B) {
  if (!e->v7 || use_split(e)) return false;
  const int m = v7_mode() & 3;
  return m >= 2 || (m == 1 && fixed_tpw(e, B) == 2);
}
bool v7_offload(const BwdEntry* e, int64_t B) { return use_v7(e, B) && (v7_mode() & 4); }
// partial rows of the chosen path: one per wave (the one-kernel and lane-group sweeps) or per
// param_sum block (split)
int64_t sum_rows(const BwdEntry* e, int64_t B, int64_t n_ev) {
  if (use_v7(e, B)) return bwd_rows(B, 2) + (v7_offload(e, B) ? s7::kKsRows : 0);
  if (!use_split(e)) return bwd_rows(B, fixed_tpw(e, B));
  const int64_t tiles = (n_ev * B + kPsTS - 1) / kPsTS;
  return tiles < kSumBlocks ? (tiles > 0 ? tiles : 1) : kSumBlocks;
}

int64_t fetode_integrate_fixed_backward_workspace(const fetode_field_t* f, int32_t method, int32_t n_steps, int64_t B) {
  if (validate_field(f) != FETODE_OK || B <= 0 || n_steps < 0) return -1;
  if (!find_bwd(f)) return fieldn_shape_supported(f) ? fieldn_fixed_backward_workspace(f, method, n_steps, B) : -1;
  const BwdEntry* e = find_bwd(f);
  AccLayout L0, L1;
  layouts(f, &L0, &L1);
  const int64_t nacc = L0.n + L1.n;
  const int64_t n_ev = n_evals_of(method, n_steps);
  const int64_t nrow = sum_rows(e, B, n_ev);
  const int64_t nch = nrow < kChunks ? nrow : kChunks;
  const int64_t adj = use_split(e) || v7_offload(e, B) ? n_ev * B * (f->kan[0].in_features + f->kan[0].out_features) : 0;
  return (int64_t)sizeof(double) * nacc * (nch + 1) + (int64_t)sizeof(float) * (nrow * nacc + adj);
}

int fetode_integrate_fixed_backward(const fetode_field_t* f, const void* plan, int32_t method, int64_t B,
                                    const float* step_coef, int32_t n_steps, const int32_t* out_step,
                                    const int32_t* out_mode, const float* out_slope, int32_t T,
                                    const float* grad_solution, const float* tape, const float* state0,
                                    uint32_t init_mask, float* grad_y0, const fetode_kanlinear_grad_t* kan_grads,
                                    const fetode_ferro_grad_t* ferro_grads, void* workspace, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  const BwdEntry* e = find_bwd(f);
  const bool fieldn = !e && fieldn_shape_supported(f);  // other widths: fetode_fieldn_bwd.hip
  if (!e && !fieldn) return set_err(FETODE_EUNSUPPORTED, "no fused backward kernel for this field shape");
  if (method < FETODE_EULER || method > FETODE_RK4_CLASSIC) return set_err(FETODE_EINVAL, "unknown method %d", method);
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!plan || !grad_solution || !workspace || (n_steps > 0 && (!tape || !step_coef || !out_step || !out_mode ||
                                                                 !out_slope)) ||
      (f->ferro && !state0 && (init_mask & 3u) != 3u))
    return set_err(FETODE_EINVAL, "null pointer");
  if (fieldn)
    return fieldn_fixed_backward(f, plan, method, B, step_coef, n_steps, out_step, out_mode, out_slope, T,
                                 grad_solution, tape, state0, init_mask, grad_y0, kan_grads, ferro_grads, workspace,
                                 stream);
  hipStream_t s = (hipStream_t)stream;
  AccLayout AL0, AL1;
  layouts(f, &AL0, &AL1);
  const int nacc = AL0.n + AL1.n;
  const bool split = use_split(e);
  const int64_t n_ev = n_evals_of(method, n_steps);
  const int64_t nrow = sum_rows(e, B, n_ev);
  const int64_t nch = nrow < kChunks ? nrow : kChunks;
  double* S = (double*)workspace;
  double* chunks = S + nacc;
  float* part = (float*)(chunks + nch * nacc);
  float* gadj = part + nrow * nacc;  // (n_ev, B, D + H): the split and lane-group (+ kansum) paths

  BwdArgs a;
  memset(&a, 0, sizeof(a));
  a.plan = (const float*)plan;
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  a.k0 = f->kan[0];
  a.k1 = f->kan[1];
  if (f->ferro) {
    a.f0 = f->ferro[0];
    a.f1 = f->ferro[1];
  }
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
  a.part = part;
  a.nacc = nacc;
  a.gadj = gadj;
  if (use_v7(e, B)) {   // two trajectories per wave, one partial row per wave
    const bool off = v7_offload(e, B);
    const int64_t nw = bwd_rows(B, 2);
    hipLaunchKernelGGL(off ? e->v7 : e->v7s, dim3((unsigned)(nw / kTPB)), dim3(64 * kTPB), 0, s, a);
    LAUNCH_CHECK();
    if (off) {   // the KAN sums: kKsRows more partial rows (both layers' halves)
      BwdArgs a2 = a;
      a2.part = part + nw * nacc;
      hipLaunchKernelGGL(e->ks, dim3((unsigned)s7::kKsRows, 2), dim3(64 * s7::kKsWaves), 0, s, a2);
      LAUNCH_CHECK();
    }
  } else if (split) {
    // adjoint sweep: one wave per trajectory, every trajectory resident (grid-stride beyond)
    const int64_t blocks = (B + kTPB - 1) / kTPB;
    hipLaunchKernelGGL(e->adj, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(64 * kTPB), 0, s, a);
    LAUNCH_CHECK();
    if (n_ev > 0) {
      hipLaunchKernelGGL(e->sum0, dim3((unsigned)nrow), dim3(256), 0, s, a);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(e->sum1, dim3((unsigned)nrow), dim3(256), 0, s, a);
      LAUNCH_CHECK();
    } else {
      HIP_CHECK_RET(hipMemsetAsync(part, 0, sizeof(float) * nrow * nacc, s));
    }
  } else {
    // (an entry whose own sweep is one trajectory per wave has no fn1)
    hipLaunchKernelGGL((e->fn1 && fixed_tpw(e, B) == 1) ? e->fn1 : e->fn, dim3((unsigned)(nrow / kTPB)), dim3(64 * kTPB),
                       0, s, a);
    LAUNCH_CHECK();
  }
  const int64_t per = (nrow + nch - 1) / nch;
  hipLaunchKernelGGL(part_reduce_kernel, dim3(nblk(nacc, 64), (unsigned)nch), dim3(64), 0, s, part, nrow, nacc, per,
                     chunks);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(chunk_sum_kernel, dim3(nblk(nacc, 64)), dim3(64 * kChunkWaves), 0, s, chunks, (int)nch, nacc, S);
  LAUNCH_CHECK();
  return apply_grads(f, S, AL0, AL1, kan_grads, ferro_grads, s);
}

// ---- reverse sweep of the resident dopri5 solve ----
// every workgroup resident at once (one grid sum per attempt): the occupancy of the kernel
static int64_t dopri_bwd_resident_wgs(const BwdEntry* e, bool one = false) {
  static int n_cu = 0;
  static int per_cu[2][2] = {{0, 0}, {0, 0}};
  const int fi = e->ferro ? 0 : 1, v = one ? 1 : 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
  }
  if (!per_cu[fi][v] &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[fi][v], one ? e->dopri1 : e->dopri, 64 * kTPB, 0) != hipSuccess)
    return -1;
  return (int64_t)per_cu[fi][v] * n_cu;
}
// one trajectory per wave when that grid is resident (small batches), else e->dtpw
static int dopri_bwd_tpw(const BwdEntry* e, int64_t B) {
  // (as fixed_tpw: while the one-per-wave grid fills at most half of its resident capacity)
  if (e->dopri1 && 2 * ((B + kTPB - 1) / kTPB) <= dopri_bwd_resident_wgs(e, true)) return 1;
  return e->dtpw;
}
static int64_t dopri_bwd_grid(const BwdEntry* e, int64_t B) {
  const int tpw = dopri_bwd_tpw(e, B);
  return (B + kTPB * tpw - 1) / (kTPB * tpw);
}

int64_t fetode_integrate_dopri5_backward_max_batch(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return 0;
  const BwdEntry* e = find_bwd(f);
  if (!e && fieldn_shape_supported(f)) return fieldn_dopri5_backward_max_batch(f);
  if (!e || !e->dopri) return 0;
  const int64_t w = dopri_bwd_resident_wgs(e);
  return w > 0 ? w * kTPB * e->dtpw : 0;
}

int64_t fetode_integrate_dopri5_backward_workspace_ev(const fetode_field_t* f, int64_t B, int32_t n_ev) {
  if (validate_field(f) != FETODE_OK || B <= 0 || n_ev < 0) return -1;
  if (!find_bwd(f) && fieldn_shape_supported(f)) return fieldn_dopri5_backward_workspace(f, B, n_ev);
  return fetode_integrate_dopri5_backward_workspace(f, B);
}

int64_t fetode_integrate_dopri5_backward_workspace(const fetode_field_t* f, int64_t B) {
  if (validate_field(f) != FETODE_OK || B <= 0) return -1;
  const BwdEntry* e = find_bwd(f);
  if (!e || !e->dopri) return -1;
  AccLayout L0, L1;
  layouts(f, &L0, &L1);
  const int64_t nacc = L0.n + L1.n, grid = dopri_bwd_grid(e, B), nrow = grid * kTPB;
  const int64_t nch = nrow < kChunks ? nrow : kChunks;
  return (int64_t)sizeof(unsigned) * kDpBarWords + (int64_t)sizeof(double) * (2 * grid + 4 * kDpGroups) +
         (int64_t)sizeof(double) * nacc * (nch + 1) + (int64_t)sizeof(float) * nrow * nacc;
}

int fetode_integrate_dopri5_backward(const fetode_field_t* f, const void* plan, int64_t B, const double* t, int32_t T,
                                     double rtol, double atol, const double* opts, const float* tableau,
                                     const float* grad_solution, const float* tape, int32_t n_ev,
                                     const double* attempts, int32_t n_att, const double* init_rec,
                                     const float* state0, uint32_t init_mask, float* grad_y0,
                                     const fetode_kanlinear_grad_t* kan_grads, const fetode_ferro_grad_t* ferro_grads,
                                     void* workspace, int32_t* status, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  const BwdEntry* e = find_bwd(f);
  const bool fieldn = !e && fieldn_shape_supported(f);  // other widths: fetode_fieldn_bwd.hip
  if (!fieldn && (!e || !e->dopri)) return set_err(FETODE_EUNSUPPORTED, "no dopri5 backward kernel for this field shape");
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!plan || !t || !opts || !tableau || !grad_solution || !tape || !attempts || !init_rec || !workspace ||
      !status || (f->ferro && !state0 && (init_mask & 3u) != 3u))
    return set_err(FETODE_EINVAL, "dopri5 backward: null pointer");
  const int base = opts[0] > 0.0 ? 1 : 2;
  if (n_att < 0 || n_ev != base + 6 * n_att)
    return set_err(FETODE_EINVAL, "dopri5 backward: %d evaluations do not match %d attempts", n_ev, n_att);
  if (fieldn)
    return fieldn_dopri5_backward(f, plan, B, t, T, rtol, atol, opts, tableau, grad_solution, tape, n_ev, attempts,
                                  n_att, init_rec, state0, init_mask, grad_y0, kan_grads, ferro_grads, workspace, status,
                                  stream);
  const bool one = dopri_bwd_tpw(e, B) == 1;
  const int64_t resident = dopri_bwd_resident_wgs(e, one);
  if (resident < 0) return set_err(FETODE_EHIP, "dopri5 backward: occupancy query failed");
  const int64_t grid = dopri_bwd_grid(e, B);
  if (grid > resident)
    return set_err(FETODE_EUNSUPPORTED, "dopri5 backward: batch %lld needs %lld workgroups, %lld resident",
                   (long long)B, (long long)grid, (long long)resident);
  hipStream_t s = (hipStream_t)stream;
  AccLayout AL0, AL1;
  layouts(f, &AL0, &AL1);
  const int nacc = AL0.n + AL1.n;
  const int64_t nrow = grid * kTPB, nch = nrow < kChunks ? nrow : kChunks;
  unsigned* bar = (unsigned*)workspace;
  double* slot = (double*)((char*)workspace + sizeof(unsigned) * kDpBarWords);
  double* xs = slot + 2 * grid;
  double* S = xs + 4 * kDpGroups;
  double* chunks = S + nacc;
  float* part = (float*)(chunks + nch * nacc);

  DopriBwdArgs d;
  memset(&d, 0, sizeof(d));
  BwdArgs& a = d.b;
  a.plan = (const float*)plan;
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  a.k0 = f->kan[0];
  a.k1 = f->kan[1];
  if (f->ferro) {
    a.f0 = f->ferro[0];
    a.f1 = f->ferro[1];
  }
  a.B = B;
  a.T = T;
  a.gsol = grad_solution;
  a.tape = tape;
  a.state0 = state0;
  a.init_mask = f->ferro ? init_mask : 3u;
  a.gy0 = grad_y0;
  a.part = part;
  a.nacc = nacc;
  d.att = attempts;
  d.n_att = n_att;
  d.n_ev = n_ev;
  d.base = base;
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
  d.n_el = (double)B * f->kan[0].in_features;
  d.gp.bar = bar;
  d.gp.slot = slot;
  d.gp.xs = xs;
  dp_single_device(d.gp, grid);
  d.status = status;
  HIP_CHECK_RET(hipMemsetAsync(workspace, 0, sizeof(unsigned) * kDpBarWords, s));
  void* args[] = {&d};
  HIP_CHECK_RET(resident_launch((const void*)(one ? e->dopri1 : e->dopri), dim3((unsigned)grid), dim3(64 * kTPB), args,
                                0, s));
  const int64_t per = (nrow + nch - 1) / nch;
  hipLaunchKernelGGL(part_reduce_kernel, dim3(nblk(nacc, 64), (unsigned)nch), dim3(64), 0, s, part, nrow, nacc, per,
                     chunks);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(chunk_sum_kernel, dim3(nblk(nacc, 64)), dim3(64 * kChunkWaves), 0, s, chunks, (int)nch, nacc, S);
  LAUNCH_CHECK();
  return apply_grads(f, S, AL0, AL1, kan_grads, ferro_grads, s);
}

}  // extern "C"
