// fetode_sweep7.h — the v7 reverse sweep of the fused rk4 / fixed-grid solve of the KAN-FET
// [2, 10, 2] field (loss.backward() through train_kanfet_node_predprey.py:252-257), on the forward
// v7 lane map (fetode_fused.hip fused4_kernel).  Included inside fetode_bwd.hip's anonymous
// namespace (BwdArgs, BL / AccLayout, BInTab, step_coefs, kTPB, param_sum_kernel).
//
// Two trajectories per wave (lanes 0-31 / 32-63), on each half the group of 3 lanes of hidden
// unit o (lanes 3 (o % 5) .. +2 of row o / 5; lane 15 of a row idle) owns BOTH layers' work of o:
//   layer 1 (input o): h_o's features (4 rounds of SiLU / logistic jobs, the gate and 2^(gs log2e h)
//     on every lane), the Ferro elements (o, d, k) of both outputs as packed pairs (o, 0, k) /
//     (o, 1, k) fed by (g_0, g_1), the spline edges (o -> d) on lanes d = 0, 1; d loss / d h_o is a
//     group sum — the old sweep's LDS d out / d x table (64 % LDS-busy) is gone;
//   layer 0 (output o): g0_o = d loss / d h_o is already on the group; the Ferro elements (i, o, k)
//     as (i, k..k+1) pairs, the edges (o, i) on lanes i = 0, 1; the d / dx_i partials of all groups
//     fold into row i with one v_permlane16_swap and one row sum.
// The layer-0 input features (x_i on row i: one job per lane — logistic j, SiLU, gate, interval)
// go through LDS once per evaluation, written long before they are read.
//
// The parameter-gradient sums stay on the wave for the whole sweep: the Ferro sums (A, C, E of the
// 14 elements a lane owns) in VGPRs; the KAN sums (logistic weights / a / b, base, spline) in
// per-wave LDS slots [slot][lane] updated read-add-write once per evaluation (bank-conflict free;
// VGPRs for all of them took 256 + 40-60 spilled), the spline sums in one LDS row per edge with
// kSO guard floats either side (the interval's four bases added at m - 3 .. m).  One partial row
// per wave in fixed_bwd_kernel's layout (AccLayout): the reduction tail is shared.
#pragma once
#ifndef S7_SKIP
#define S7_SKIP 0   // diagnostic: bit 1 layer-1 logistic sums, 2 layer-1 spline, 4 layer-0 lw, 8 layer-0 a/b, 16 layer-0 spline/base
#endif

#ifndef S7_PRIO
// wave priority over the serial phases (as fetode_fused.hip PRIO_HI / PRIO_LO): the sweep runs two
// waves per SIMD; measured 0.558 -> 0.546 ms per B = 4096 backward (profiles/r06_s7prio_ab.log)
#define S7_PRIO 1
#endif
#if S7_PRIO
#define S7_HI() __builtin_amdgcn_s_setprio(1)
#define S7_LO() __builtin_amdgcn_s_setprio(0)
#else
#define S7_HI()
#define S7_LO()
#endif

namespace s7 {
constexpr int D = 2, H = 10, K = 10, NB = 10, NG = 12, NI = NG - 1, NS = NG - 1 - kSO, NFL = 1 + NB, KP = K / 2;
constexpr int W = D + H;
constexpr int NPL0 = (D * KP) / 3, NPL1 = K / 3;   // pair rounds per layer; the leftover as singles
static_assert(D * KP - 3 * NPL0 == 1 && K - 3 * NPL1 == 1, "one leftover pair (layer 0) / k (layer 1)");
constexpr int RF1 = (NFL + 2) / 3;                  // layer-1 feature rounds (SiLU + NB logistic)
constexpr int KT = (NG + 2) / 3;                    // knots per group lane
// spline-sum row: kSO guards, NS bases, kSO guards, one pad: an odd row stride puts the 20 edge rows
// of a half-wave on 20 different banks (an even one folds them onto 16)
constexpr int AR = NS + 2 * kSO + 1;
constexpr int SPR = NI + 2;                         // spline-table row stride (float4)
// KAN-sum LDS slots per lane
// KAN-sum LDS slot PAIRS per lane (both components of a pair are updated together, one
// ds_read_b64 / ds_write_b64 each): layer-0 logistic weights of outputs (2p, 2p + 1), layer-0
// (a, b), layer-1 round r's logistic weights of outputs (0, 1), layer-1 round r's (a, b)
constexpr int P_LW0 = 0, P_AB0 = H / 2, P_LW1 = P_AB0 + 1, P_AB1 = P_LW1 + RF1, NKP = P_AB1 + RF1;
constexpr int NSR = 2 * (H * D) + 1;                // spline rows per layer: (half, o, i) + a dummy row
// The element constants a lane reads are tabled per ROUND and LANE ([r][lane & 31]: both halves
// hold the same parameters): a round's reads are 32 consecutive entries, free of the bank conflicts
// the element-indexed tables had (lanes of different units on one 16-B slot: 2-way on most reads,
// 140 of the ~260 conflict cycles per evaluation, profiles/r06_sweep_pmc.txt), and the lanes keep
// no element indices in VGPRs.  Round NPL is the lane's single.
struct Tab {
  float4 fa0[NPL0 + 1][32], fb0[NPL0 + 1][32];  // layer-0 pairs: (Ec, Ec', k2, k2'), (cPk, cPk', Eg2, Eg2')
  f2 ee0[NPL0 + 1][32];                          // 2^(gs log2e Ec) (the factored coercive gate)
  float4 fa1[NPL1 + 1][32], fb1[NPL1 + 1][32];  // layer-1 pairs: elements (o, 0, k), (o, 1, k)
  f2 ee1[NPL1 + 1][32];
  // edge cubics by interval, one row of NI + 1 per edge padded to SPR float4: rows of different
  // edges start on different 16-B slots of the bank row (12: units 4 apart collide)
  float4 sp0[H * D * SPR], sp1[D * H * SPR];
  float kwT[D * NB * H];                                // layer-0 logistic weights by (i, j): the ten outputs
  float4 jf[RF1][32];   // layer-1 job (o, j = cc0 + 3 r): (-a log2e, a b log2e, a, b); SiLU (j = NB): (-log2e, 0, 1, 0)
  f2 jw[RF1][32];       // its weights for outputs 0, 1 (SiLU: the base weights)
};
// the lane map of sweep7_kernel (lane & 31): hidden unit o (idle lane 15: unit 0's constants, never
// used) and part cc0 of its group of 3; its element pair P = cc0 NPL + r of the unit
struct LaneMap {
  int row, q, o, cc0;
  __device__ explicit LaneMap(int l) : row(l >> 4), q(l & 15), o(q < 15 ? row * 5 + q / 3 : 0), cc0(q % 3) {}
  __device__ int p0(int r) const {   // layer-0 pair (i, o, 2 kp .. 2 kp + 1) as e / 2
    const int P = cc0 * NPL0 + r, i = P / KP, kp = P % KP;
    return (i * H + o) * KP + kp;
  }
  __device__ int ps0() const { return ((D - 1) * H + o) * KP + (KP - 1); }   // layer-0 single: (1, o, 8 + cc0)
  __device__ int p1(int r) const { return o * K + (cc0 + 3 * r); }         // layer-1 pair (o, k), both outputs
  __device__ int ps1() const { return o * K + (K - 1); }                     // layer-1 single: (o, cc0, 9)
};
struct Wv {
  float4 gx[2][D];   // per half, layer-0 input i: x, up, wo, 2^(gs log2e x)
  float4 fx[2][D];   // SiLU, SiLU', u, 1 / width
  float4 bx[2][D];   // the interval's four bases B_{m-3 .. m}(x_i)
  int mx[2][D];      // interval (NI: outside the grid / non-finite)
  float g0[2][H];    // d loss / d h of the evaluation
  f2 ks[NKP][64];                   // KAN sums, [pair][lane]
  float spl[2][NSR][AR];            // spline sums per layer and edge row
};
__device__ __forceinline__ float dcubic(float4 c, float u) { return ffma(u, ffma(3.0f * u, c.w, 2.0f * c.z), c.y); }
__device__ __forceinline__ int g3i(int v, int c) {
  const int s0 = v + __builtin_amdgcn_update_dpp(0, v, 0x101, 0xF, 0xF, false) +
                 __builtin_amdgcn_update_dpp(0, v, 0x102, 0xF, 0xF, false);
  const int b1 = __builtin_amdgcn_mov_dpp(s0, 0x111, 0xF, 0xF, false);
  const int b2 = __builtin_amdgcn_mov_dpp(s0, 0x112, 0xF, 0xF, false);
  return c == 0 ? s0 : (c == 1 ? b1 : b2);
}
__device__ __forceinline__ float g3f(float v, int c) {
  const float s0 = v + dpp<0x101>(v) + dpp<0x102>(v);
  const float b1 = dppm<0x111>(s0), b2 = dppm<0x112>(s0);
  return c == 0 ? s0 : (c == 1 ? b1 : b2);
}
__device__ __forceinline__ void pl16(float& p, float& q) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p), "+v"(q));
}
__device__ __forceinline__ float rs16(float v) {
  v += dpp<0x128>(v);
  v += dpp<0x124>(v);
  v += dpp<0x122>(v);
  v += dpp<0x121>(v);
  return v;
}
// lanes 0-31: the value of lane + 32 (v_permlane32_swap exchanges p's upper half with q's lower
// half, so q's lower half receives lanes 32-63; only lanes 0-31 store the combined sums)
__device__ __forceinline__ float partner(float v) {
  float p = v, q = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(p), "+v"(q));
  return q;
}
__device__ __forceinline__ void knots4(float x, const float* kn, int& cnt) {
  cnt = 0;
#pragma unroll
  for (int t = 0; t < KT; ++t)
    asm volatile("v_cmp_ge_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(cnt) : "v"(x), "v"(kn[t]) : "vcc");
}
// one Ferro element pair's VJP (ferro_class.py forward, differentiated; the element algebra of
// layer_jobs): sums A, C, E and the pair's d out / d x (both elements' sum)
template <bool FACT>
__device__ __forceinline__ float pair_vjp(float4 fa, float4 fb, f2 ee, f2 g, float x, float up, float wo, float E,
                                          float gsl2e, f2& A, f2& C, f2& Ev) {
  const f2 Ec = f2{fa.x, fa.y}, k2 = f2{fa.z, fa.w}, cPk = f2{fb.x, fb.y}, Eg2 = f2{fb.z, fb.w};
  f2 cn;
  if constexpr (FACT) cn = rcpx2(pfma(splat(E), ee, splat(1.0f)));          // sigmoid(gs(-x - Ec))
  else cn = rcpx2(ex2x2(pfma(splat(gsl2e), splat(x), Eg2)) + splat(1.0f));
  const f2 mm = pfma(splat(wo), cn, splat(1.0f));                            // branch_mom (bs = 1)
  const f2 sh = pfma(Ec, mm, splat(x));                                       // shifted_x
  const f2 th = pfma(splat(-2.0f), rcpx2(ex2x2(k2 * sh) + splat(1.0f)), splat(1.0f));  // tanh(k sh)
  const f2 q = g * pfma(-th, th, splat(1.0f));
  const f2 dcn = pfma(-cn, cn, cn);
  const f2 ew = Eg2 * splat(-0.69314718f * wo);                              // (-gs Ec) wo
  A = pfma(g, th, A);
  C = pfma(q, sh, C);
  Ev = pfma(q, pfma(ew, dcn, mm), Ev);
  const f2 dx = (q * cPk) * pfma(ew, pfma(splat(up), cn, dcn), splat(1.0f));  // Ec dm/dx = ew (up c + c')
  return dx.x + dx.y;
}
template <bool FACT>
__device__ __forceinline__ float single_vjp(float Ec, float k2, float cPk, float Eg2, float ee, float g, float x, float up,
                                            float wo, float E, float gsl2e, float& A, float& C, float& Ev) {
  float cn;
  if constexpr (FACT) cn = rcp(ffma(E, ee, 1.0f));
  else cn = rcp(ex2(ffma(gsl2e, x, Eg2)) + 1.0f);
  const float mm = ffma(wo, cn, 1.0f);
  const float sh = ffma(Ec, mm, x);
  const float th = ffma(-2.0f, rcp(ex2(k2 * sh) + 1.0f), 1.0f);
  const float q = g * ffma(-th, th, 1.0f);
  const float dcn = ffma(-cn, cn, cn);
  const float ew = Eg2 * (-0.69314718f * wo);
  A = ffma(g, th, A);
  C = ffma(q, sh, C);
  Ev = ffma(q, ffma(ew, dcn, mm), Ev);
  return (q * cPk) * ffma(ew, ffma(up, cn, dcn), 1.0f);
}
}  // namespace s7

// KS = true: the KAN sums as well (per-wave LDS slots, above); KS = false: the Ferro sums only, each
// evaluation's adjoints (g_0, g_1, d loss / d h) recorded in a.gadj for kansum_kernel
template <bool KS>
__global__ __launch_bounds__(64 * kTPB) __attribute__((amdgpu_waves_per_eu(2))) void sweep7_kernel(BwdArgs a) {
  using namespace s7;
  using L0 = BL<D, H, K, NB, NG, true>;
  using L1 = BL<H, D, K, NB, NG, true>;
  constexpr AccLayout A0L = L0::AL, A1L = L1::AL;
  // knots, 1 / widths, basis cubics [t][m][r] of all 12 inputs (no logistic table: the lanes hold
  // their logistic constants in registers / T.jf)
  __shared__ BInTab<W, NG, 0> TI;
  __shared__ Tab T;
  __shared__ Wv WV[kTPB];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int hh = lane >> 5, l = lane & 31, row = l >> 4, q = l & 15;
  const bool act = q < 15;
  const int o = act ? row * 5 + q / 3 : 0, cc0 = q % 3;
  Wv& V = WV[wid];
  const float k2c = 2.0f * FETODE_LOG2E;
  const float gl0 = a.P0.gsl2e, gl1 = a.P1.gsl2e, wc0 = a.P0.wc, wc1 = a.P1.wc;
  // ---- tables (once per workgroup) ----
  TI.stage(a.plan, a.P0, a.P1, D, tid, 64 * kTPB);
  for (int t = tid; t < (NPL0 + 1) * 32; t += 64 * kTPB) {   // layer 0: elements e = 2p, 2p + 1
    const int r = t / 32;
    const LaneMap lm(t % 32);
    const int e = 2 * (r < NPL0 ? lm.p0(r) : lm.ps0());
    const fetode_ferro_t& f = a.f0;
    T.fa0[r][t % 32] = make_float4(f.Ec[e], f.Ec[e + 1], k2c * f.k[e], k2c * f.k[e + 1]);
    T.fb0[r][t % 32] = make_float4((f.coef[e] * f.Ps[e]) * f.k[e], (f.coef[e + 1] * f.Ps[e + 1]) * f.k[e + 1],
                                   gl0 * f.Ec[e], gl0 * f.Ec[e + 1]);
    T.ee0[r][t % 32] = f2{ex2(gl0 * f.Ec[e]), ex2(gl0 * f.Ec[e + 1])};
  }
  for (int t = tid; t < (NPL1 + 1) * 32; t += 64 * kTPB) {   // layer 1: (o, 0, k), (o, 1, k)
    const int r = t / 32;
    const LaneMap lm(t % 32);
    const int p = r < NPL1 ? lm.p1(r) : lm.ps1();
    const int oo = p / K, k = p % K, e0 = (oo * D + 0) * K + k, e1 = (oo * D + 1) * K + k;
    const fetode_ferro_t& f = a.f1;
    T.fa1[r][t % 32] = make_float4(f.Ec[e0], f.Ec[e1], k2c * f.k[e0], k2c * f.k[e1]);
    T.fb1[r][t % 32] = make_float4((f.coef[e0] * f.Ps[e0]) * f.k[e0], (f.coef[e1] * f.Ps[e1]) * f.k[e1],
                                   gl1 * f.Ec[e0], gl1 * f.Ec[e1]);
    T.ee1[r][t % 32] = f2{ex2(gl1 * f.Ec[e0]), ex2(gl1 * f.Ec[e1])};
  }
  {
    const float4* s0 = reinterpret_cast<const float4*>(a.plan + a.P0.sp);
    const float4* s1 = reinterpret_cast<const float4*>(a.plan + a.P1.sp);
    for (int i = tid; i < H * D * (NI + 1); i += 64 * kTPB) {
      T.sp0[(i / (NI + 1)) * SPR + i % (NI + 1)] = s0[i];
      T.sp1[(i / (NI + 1)) * SPR + i % (NI + 1)] = s1[i];
    }
    for (int i = tid; i < D * NB * H; i += 64 * kTPB) {
      const int ij = i / H, oo = i % H, ii = ij / NB, j = ij % NB;
      T.kwT[i] = a.plan[a.P0.kw + (oo * D + ii) * NFL + 1 + j];
    }
    for (int t = tid; t < RF1 * 32; t += 64 * kTPB) {
      const LaneMap lm(t % 32);
      const int oo = lm.o, j = lm.cc0 + 3 * (t / 32);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      f2 w = f2{0.f, 0.f};
      if (j < NB) {
        v = make_float4(a.plan[a.P1.lg + 2 * (oo * NB + j)], a.plan[a.P1.lg + 2 * (oo * NB + j) + 1],
                        a.k1.logistic_a[oo * NB + j], a.k1.logistic_b[oo * NB + j]);
      } else if (j == NB) {
        v = make_float4(-FETODE_LOG2E, 0.f, 1.0f, 0.f);
      }
      if (j < NFL) {
        const int ff = j < NB ? 1 + j : 0;
        w = f2{a.plan[a.P1.kw + (0 * H + oo) * NFL + ff], a.plan[a.P1.kw + (1 * H + oo) * NFL + ff]};
      }
      T.jf[t / 32][t % 32] = v;
      T.jw[t / 32][t % 32] = w;
    }
  }
  for (int i = lane; i < NKP * 64; i += 64) (&V.ks[0][0])[i] = splat(0.f);
  for (int i = lane; i < 2 * NSR * AR; i += 64) (&V.spl[0][0][0])[i] = 0.f;
  const bool fact = a.plan[a.P0.flag] <= kFactorLimit && a.plan[a.P1.flag] <= kFactorLimit;

  // ---- per-lane constants ----
  // layer-0 feature job q of row i = row: logistic j = q (q < NB), SiLU + interval (NB), gate +
  // 2^(gs log2e x) (NB + 1), base r = q - (NB + 2) of the interval (12 .. 15)
  const int xi = row;
  float xna = 0.f, xab = 0.f, pa0 = 0.f, pb0 = 0.f;
  const float* kwo = &T.kwT[(xi * NB + (q < NB ? q : 0)) * H];
  const float kwm = q < NB ? 1.0f : 0.0f;   // (q >= NB: no logistic term)
  if (q < NB) {
    xna = a.plan[a.P0.lg + 2 * (xi * NB + q)];
    xab = a.plan[a.P0.lg + 2 * (xi * NB + q) + 1];
    pa0 = a.k0.logistic_a[xi * NB + q];
    pb0 = a.k0.logistic_b[xi * NB + q];
  } else if (q == NB) {
    xna = -FETODE_LOG2E;
  } else if (q == NB + 1) {
    xna = -gl0;   // the gate: 2^(-gs log2e (x - pv))
  }
  const int rb = q >= NB + 2 ? q - (NB + 2) : 0;   // base lanes
  const float xknot = q < NG ? a.plan[a.P0.knots + xi * NG + q] : __builtin_inff();
  const f2 mrow = xi == 0 ? f2{1.f, 0.f} : f2{0.f, 1.f};   // this row's component of (dx_0, dx_1)
  // layer-1 feature rounds of the group: job j = cc0 + 3 r, its constants in T.jf / T.jw [r][l]
  // (idle lane 15 reads group 0's, its results are never used)
  static_assert(NB % 3 == 1 && NFL <= 3 * RF1, "SiLU = job NB in the last round");
  const float4* hk4 = reinterpret_cast<const float4*>(&TI.knots[(D + o) * NG + KT * cc0]);   // 4 knots
  const bool sok = act && cc0 < 2;                 // single / edge lanes
  const f2 dsel = f2{(sok && cc0 == 0) ? 1.f : 0.f, (sok && cc0 == 1) ? 1.f : 0.f};
  const int ie = sok ? cc0 : 0;                        // edge input (layer 0) / output (layer 1)
  const int t1 = D + o;                                // combined input index of h_o
  const float4* sp1e = &T.sp1[(ie * H + o) * SPR];
  const float4* sp0e = &T.sp0[(o * D + ie) * SPR];
  const int srow = sok ? hh * (H * D) + o * D + ie : NSR - 1;   // this lane's spline-sum rows
  float* acc0 = &V.spl[0][srow][0];
  float* acc1 = &V.spl[1][srow][0];
  f2* ks = &V.ks[0][lane];                                    // pair k at ks[64 k]

  // ---- Ferro accumulators ----
  f2 A0[NPL0], C0[NPL0], E0[NPL0], A1[NPL1], C1[NPL1], E1[NPL1];
#pragma unroll
  for (int r = 0; r < NPL0; ++r) A0[r] = C0[r] = E0[r] = splat(0.f);
#pragma unroll
  for (int r = 0; r < NPL1; ++r) A1[r] = C1[r] = E1[r] = splat(0.f);
  float As0 = 0.f, Cs0 = 0.f, Es0 = 0.f, As1 = 0.f, Cs1 = 0.f, Es1 = 0.f;
  float G0 = 0.f, bs0 = 0.f;
  f2 G1 = splat(0.f);
  int nan0 = 0, nan1 = 0;
  __syncthreads();   // tables staged; from here on every wave syncs only with itself

  const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  const int64_t tstride = a.B * W;
  const int n_ev = a.n_steps * ns;
  auto run = [&](auto fact_tag) __attribute__((always_inline)) {
    constexpr bool F_ = decltype(fact_tag)::value;
    const float kbase0 = a.plan[a.P0.kw + (o * D + ie) * NFL];   // the edge's SiLU weight
    for (int64_t b0 = ((int64_t)blockIdx.x * kTPB + wid) * 2; b0 < a.B; b0 += (int64_t)gridDim.x * kTPB * 2) {
      const int64_t b = b0 + hh;
      const bool live = b < a.B;
      // tape column c of evaluation ev (ev < 0: the hysteresis state before the solve, or the
      // first input under the re-initialisation rule, ferro_class.py:373-378)
      auto tape_at = [&](int ev, int c) -> float {
        if (!live) return 0.f;
        if (ev >= 0) return a.tape[(int64_t)ev * tstride + b * W + c];
        const float v = a.tape[b * W + c];
        if (c < D) return (a.init_mask & 1u) ? v : a.state0[b * D + c];
        return (a.init_mask & 2u) ? v : a.state0[a.B * D + b * H + (c - D)];
      };
      float cx = tape_at(n_ev - 1, xi), ch = tape_at(n_ev - 1, D + o);
      float px = tape_at(n_ev - 2, xi), ph = tape_at(n_ev - 2, D + o);
      float ay1 = 0.f;   // adjoint of y (state dim `row`) at the end of the current step
      int jj = a.T - 1;
      // the next output's schedule entry and adjoint, and the next step's coefficients, fetched one
      // step ahead: their global round trips overlap the step's evaluations instead of heading its
      // chain (as the forward's output schedule, fetode_fused.hip)
      int pst = -1, pmd = 1;
      float psl = 0.f, pg = 0.f;
      auto fetch_out = [&]() __attribute__((always_inline)) {
        pst = jj >= 1 ? a.out_step[jj] : -1;
        if (jj >= 1) {
          pmd = a.out_mode[jj];
          psl = a.out_slope[jj];
          pg = live ? a.gsol[((int64_t)jj * a.B + b) * D + row] : 0.f;
        }
      };
      fetch_out();
      int sn = a.n_steps - 1;
      float sc0 = sn >= 0 ? a.step_coef[4 * sn] : 0.f, sc1 = sn >= 0 ? a.step_coef[4 * sn + 1] : 0.f;
      float sc2 = sn >= 0 ? a.step_coef[4 * sn + 2] : 0.f;
      for (int s = a.n_steps - 1; s >= 0; --s) {
        float bc[4], ac[4][3];
        step_coefs(a.method, sc0, sc1, sc2, bc, ac);
        if (s > 0) {
          sc0 = a.step_coef[4 * (s - 1)];
          sc1 = a.step_coef[4 * (s - 1) + 1];
          sc2 = a.step_coef[4 * (s - 1) + 2];
        }
        float ay0x = 0.f;
        while (pst == s) {
          const float g = pg;
          if (pmd == 0) {
            ay0x += g;
          } else if (pmd == 1) {
            ay1 += g;
          } else {
            ay1 = ffma(psl, g, ay1);
            ay0x = ffma(1.0f - psl, g, ay0x);
          }
          --jj;
          fetch_out();
        }
        float ak[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) ak[j] = bc[j] * ay1;
        float ay = ay1 + ay0x;
#pragma unroll
        for (int st = 3; st >= 0; --st) {
          if (st >= ns) continue;
          const int ev = s * ns + st;
          // prefetch evaluation ev - 2's inputs (the hysteresis inputs of ev - 1)
          const float nx = tape_at(ev - 2, xi), nh = tape_at(ev - 2, D + o);
          // this evaluation's output adjoint (g_0, g_1) on every lane
          float g0v = ak[st], g1v = ak[st];
          pl16(g0v, g1v);
          const f2 g01 = f2{g0v, g1v};
          // ---- (1) layer-0 input features: row xi, job q ----
          float sgx;
          {
            const float x = cx;
            const float e = ex2(ffma(xna, q == NB + 1 ? x - px : x, xab));
            sgx = rcp(1.0f + e);
            const uint64_t bal = __builtin_amdgcn_ballot_w64(x >= xknot);
            const int m = (int)__builtin_popcountll((bal >> (lane & 48)) & 0xFFFFull) - 1;
            if (q == NB) {
              const bool fin = __builtin_isfinite(x), in = fin && (unsigned)m < (unsigned)NI;
              const int mc = in ? m : 0;
              const float rhm = TI.rh[xi * NI + mc];
              const float u = in ? (x - TI.knots[xi * NG + mc]) * rhm : (fin ? 0.f : __builtin_nanf(""));
              V.fx[hh][xi] = make_float4(x * sgx, sgx * ffma(x, 1.0f - sgx, 1.0f), u, rhm);
              V.mx[hh][xi] = in ? m : NI;
            }
            if (q == NB + 1) {
              const float wo = wc0 * (1.0f - sgx);
              V.gx[hh][xi] = make_float4(x, sgx, wo, F_ ? ex2(gl0 * x) : 0.f);
            }
            if (KS && q >= NB + 2) {   // base rb of the interval (the row's sums: only on in-grid x)
              const bool fin = __builtin_isfinite(x), in = fin && (unsigned)m < (unsigned)NI;
              const int mc = in ? m : 0;
              const float u = in ? (x - TI.knots[xi * NG + mc]) * TI.rh[xi * NI + mc] : 0.f;
              const float4 c = TI.bp[TI.bpi(xi, mc) + rb];
              (&V.bx[hh][xi].x)[rb] = in ? ffma(ffma(ffma(c.w, u, c.z), u, c.y), u, c.x) : 0.f;
            }
          }
          // ---- (2) layer 1 on the group of hidden input o ----
          float dh = 0.f;
          {
            const float h = ch;
            // features: logistic j / SiLU, d out / d h through both outputs
#pragma unroll
            for (int r = 0; r < RF1; ++r) {
              const float4 jf = T.jf[r][l];
              const f2 jw = T.jw[r][l];
              const bool sl = r == RF1 - 1 && cc0 == 1;   // the SiLU job (NB = cc0 + 3 (RF1 - 1))
              const float sg = rcp(1.0f + ex2(ffma(jf.x, h, jf.y)));
              const float val = sl ? h * sg : sg;
              const float der = sl ? sg * ffma(h, 1.0f - sg, 1.0f) : ffma(-sg, sg, sg);
              const float Tt = ffma(g01.x, jw.x, g01.y * jw.y) * der;
              // sums: logistic weights of both outputs (SiLU job: base weights), a, b
              if (KS && !(S7_SKIP & 1)) {
              ks[64 * (P_LW1 + r)] = pfma(g01, splat(val), ks[64 * (P_LW1 + r)]);
              ks[64 * (P_AB1 + r)] = pfma(f2{Tt, -Tt}, f2{h - jf.w, jf.z}, ks[64 * (P_AB1 + r)]);
              }
              dh = ffma(Tt, jf.z, dh);
            }
            // gate and 2^(gs log2e h) of this input (every lane of the group)
            const float up = rcp(1.0f + ex2(-gl1 * (h - ph)));
            const float wo = wc1 * (1.0f - up);
            const float E = F_ ? ex2(gl1 * h) : 0.f;
            // interval of h (group count), the edge (o -> d = cc0): d out_d / d h
            int cnt;
            {
              const float4 kv = *hk4;
              const float kn[KT] = {kv.x, kv.y, kv.z, kv.w};
              knots4(h, kn, cnt);
            }
            const int m = g3i(cnt, cc0) - 1;
            const bool fin = __builtin_isfinite(h), in = fin && (unsigned)m < (unsigned)NI;
            const int mc = in ? m : 0;
            const float rhm = TI.rh[t1 * NI + mc];
            const float u = in ? (h - TI.knots[t1 * NG + mc]) * rhm : (fin ? 0.f : __builtin_nanf(""));
            const float4 cf = sp1e[in ? m : NI];
            const float ge = sok ? (cc0 == 0 ? g01.x : g01.y) : 0.f;
            dh = ffma(ge, dcubic(cf, u) * rhm, dh);
            if (KS && !(S7_SKIP & 2)) {   // spline sums of edge (o -> cc0): the interval's four bases
              const float4* bp = &TI.bp[TI.bpi(t1, mc)];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float4 c = bp[r];
                const float bv = in ? ffma(ffma(ffma(c.w, u, c.z), u, c.y), u, c.x) : 0.f;
                acc1[mc + r] = ffma(ge, bv, acc1[mc + r]);
              }
              nan1 |= fin ? 0 : 1;
            }
            // Ferro elements (o, d, k): pairs over both outputs, then the single (o, cc0, K - 1)
            S7_LO();
#pragma unroll
            for (int r = 0; r < NPL1; ++r)
              dh += pair_vjp<F_>(T.fa1[r][l], T.fb1[r][l], T.ee1[r][l], g01, h, up, wo, E, gl1, A1[r], C1[r], E1[r]);
            {
              const float4 fa = T.fa1[NPL1][l], fb = T.fb1[NPL1][l];
              const f2 ee = T.ee1[NPL1][l];
              const bool c1 = cc0 == 1;
              dh += single_vjp<F_>(c1 ? fa.y : fa.x, c1 ? fa.w : fa.z, c1 ? fb.y : fb.x, c1 ? fb.w : fb.z,
                                   c1 ? ee.y : ee.x, ge, h, up, wo, E, gl1, As1, Cs1, Es1);
            }
          }
          if (KS) G1 += g01;
          S7_HI();
          const float g0o = act ? g3f(dh, cc0) : 0.f;   // d loss / d h_o on the group (lane 15: none)
          if (act && cc0 == 0) V.g0[hh][o] = g0o;
          if (!KS && live) {   // this evaluation's adjoints for kansum_kernel
            float* gr = a.gadj + ((int64_t)ev * a.B + b) * W;
            if (q == 15) gr[row] = ak[st];
            if (act && cc0 == 0) gr[D + o] = g0o;
          }
          // ---- (3) layer 0 on the group of output o ----
          f2 dx01 = splat(0.f);
          {
            const f2 g2 = splat(g0o);
            S7_LO();
#pragma unroll
            for (int r = 0; r < NPL0; ++r) {
              const bool i1 = cc0 * NPL0 + r >= KP;   // the pair's input (LaneMap::p0)
              const float4 gx = V.gx[hh][i1 ? 1 : 0];
              const float d = pair_vjp<F_>(T.fa0[r][l], T.fb0[r][l], T.ee0[r][l], g2, gx.x, gx.y, gx.z, gx.w, gl0,
                                           A0[r], C0[r], E0[r]);
              dx01 = pfma(f2{i1 ? 0.f : 1.f, i1 ? 1.f : 0.f}, splat(d), dx01);
            }
            const float ge = sok ? g0o : 0.f;
            {
              const float4 gx = V.gx[hh][D - 1];
              const float4 fa = T.fa0[NPL0][l], fb = T.fb0[NPL0][l];
              const f2 ee = T.ee0[NPL0][l];
              const bool c1 = cc0 == 1;
              const float d = single_vjp<F_>(c1 ? fa.y : fa.x, c1 ? fa.w : fa.z, c1 ? fb.y : fb.x, c1 ? fb.w : fb.z,
                                             c1 ? ee.y : ee.x, ge, gx.x, gx.y, gx.z, gx.w, gl0, As0, Cs0, Es0);
              dx01.y += d;   // the layer-0 single is on input 1
            }
            // edge (o, ie): base and spline sums, d out_o / d x_ie (SiLU' base weight + spline')
            const float4 fx = V.fx[hh][ie], bx = V.bx[hh][ie];
            const int mx = V.mx[hh][ie];
            const int mc = mx < NI ? mx : 0;
            if (KS && !(S7_SKIP & 16)) {
            bs0 = ffma(ge, fx.x, bs0);
            acc0[mc + 0] = ffma(ge, bx.x, acc0[mc + 0]);
            acc0[mc + 1] = ffma(ge, bx.y, acc0[mc + 1]);
            acc0[mc + 2] = ffma(ge, bx.z, acc0[mc + 2]);
            acc0[mc + 3] = ffma(ge, bx.w, acc0[mc + 3]);
            }
            nan0 |= __builtin_isnan(fx.z) ? 1 : 0;
            const float4 cf = sp0e[mx];
            const float dxe = ge * ffma(kbase0, fx.y, dcubic(cf, fx.z) * fx.w);
            dx01 = pfma(dsel, splat(dxe), dx01);   // lane 0: input 0, lane 1: input 1, lane 2: 0
            if (KS) G0 += sok && cc0 == 0 ? g0o : 0.f;
          }
          // ---- (4) layer-0 logistic (i = xi, j = q) for all ten outputs: sums, d / dx_i ----
          {
            float S = 0.f;
#pragma unroll
            for (int oo = 0; oo < H; oo += 2) {
              const f2 gv = *reinterpret_cast<const f2*>(&V.g0[hh][oo]);
              const f2 kv = *reinterpret_cast<const f2*>(&kwo[oo]);
              S = ffma(gv.x, kv.x, S);
              S = ffma(gv.y, kv.y, S);
              if (KS && !(S7_SKIP & 4)) {
              ks[64 * (P_LW0 + oo / 2)] = pfma(gv, splat(sgx), ks[64 * (P_LW0 + oo / 2)]);
              }
            }
            const float Tt = (S * kwm) * ffma(-sgx, sgx, sgx);
            if (KS && !(S7_SKIP & 8)) {
            ks[64 * P_AB0] = pfma(f2{Tt, -Tt}, f2{cx - pb0, pa0}, ks[64 * P_AB0]);
            }
            dx01 = pfma(mrow, splat(Tt * pa0), dx01);
          }
          // ---- (5) d loss / d x: rows fold, row sum -> dx of state dim `row` on row `row` ----
          S7_HI();
          float r0 = dx01.x, r1 = dx01.y;
          pl16(r0, r1);
          const float dx = rs16(r0 + r1);
          ay += dx;
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if (j < st) ak[j] = ffma(ac[st][j], dx, ak[j]);
          cx = px;
          ch = ph;
          px = nx;
          ph = nh;
        }
        ay1 = ay;
      }
      if (q == 0 && live && a.gy0) a.gy0[b * D + row] = ay1 + a.gsol[b * D + row];   // solution[0] = y0
    }
  };
  using FT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;
  if (fact) run(FT{});
  else run(FF{});

  // ---- one partial row per wave: the two halves' (trajectories') sums, in order ----
  float* part = a.part + ((int64_t)blockIdx.x * kTPB + wid) * a.nacc;
  float* part1 = part + A0L.n;
  const bool lo = hh == 0;
  auto put = [&](float* base, int idx, float v) {
    const float t = v + partner(v);
    if (lo && act) base[idx] = t;
  };
  // Ferro sums
  const LaneMap lm(l);
#pragma unroll
  for (int r = 0; r < NPL0; ++r) {
    const int e = 2 * lm.p0(r);
    put(part, A0L.oA + e, A0[r].x); put(part, A0L.oA + e + 1, A0[r].y);
    put(part, A0L.oC + e, C0[r].x); put(part, A0L.oC + e + 1, C0[r].y);
    put(part, A0L.oE + e, E0[r].x); put(part, A0L.oE + e + 1, E0[r].y);
  }
#pragma unroll
  for (int r = 0; r < NPL1; ++r) {
    const int oo = lm.p1(r) / K, k = lm.p1(r) % K, e0 = (oo * D + 0) * K + k, e1 = (oo * D + 1) * K + k;
    put(part1, A1L.oA + e0, A1[r].x); put(part1, A1L.oA + e1, A1[r].y);
    put(part1, A1L.oC + e0, C1[r].x); put(part1, A1L.oC + e1, C1[r].y);
    put(part1, A1L.oE + e0, E1[r].x); put(part1, A1L.oE + e1, E1[r].y);
  }
  {
    const int es0 = 2 * lm.ps0() + cc0, es1 = (o * D + cc0) * K + (K - 1);
    const float a0 = As0 + partner(As0), c0 = Cs0 + partner(Cs0), x0 = Es0 + partner(Es0);
    const float a1 = As1 + partner(As1), c1 = Cs1 + partner(Cs1), x1 = Es1 + partner(Es1);
    if (lo && sok) {
      part[A0L.oA + es0] = a0; part[A0L.oC + es0] = c0; part[A0L.oE + es0] = x0;
      part1[A1L.oA + es1] = a1; part1[A1L.oC + es1] = c1; part1[A1L.oE + es1] = x1;
    }
  }
  if constexpr (!KS) {   // the KAN slots of both layers: kansum_kernel's rows hold them
    for (int i = 3 * A0L.E + lane; i < A0L.n; i += 64) part[i] = 0.f;
    for (int i = 3 * A1L.E + lane; i < A1L.n; i += 64) part1[i] = 0.f;
    return;
  }
  {
    const float g0t = G0 + partner(G0), g1x = G1.x + partner(G1.x), g1y = G1.y + partner(G1.y);
    if (lo && sok && cc0 == 0) part[A0L.oG + o] = g0t;
    if (lane == 0) {
      part1[A1L.oG + 0] = g1x;
      part1[A1L.oG + 1] = g1y;
    }
  }
  // edges: layer-0 base sums, both layers' spline sums (rows of the two halves added in order)
  {
    const float b0t = bs0 + partner(bs0);
    if (lo && sok) part[A0L.oBase + o * D + ie] = b0t;
    const int nf0 = nan0 | (int)partner((float)nan0), nf1 = nan1 | (int)partner((float)nan1);
    const float* r0a = &V.spl[0][o * D + ie][kSO];
    const float* r0b = &V.spl[0][H * D + o * D + ie][kSO];
    const float* r1a = &V.spl[1][o * D + ie][kSO];
    const float* r1b = &V.spl[1][H * D + o * D + ie][kSO];
    // (the nan flags of the two halves of one edge row: lanes of the same group, either half)
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      if (lo && sok) {
        part[A0L.oSpl + (o * D + ie) * NS + c] = nf0 ? __builtin_nanf("") : r0a[c] + r0b[c];
        part1[A1L.oSpl + (ie * H + o) * NS + c] = nf1 ? __builtin_nanf("") : r1a[c] + r1b[c];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RF1; ++r) {
    const int j = cc0 + 3 * r;
    const float vx = ks[64 * (P_LW1 + r)].x, vy = ks[64 * (P_LW1 + r)].y;
    const float va = ks[64 * (P_AB1 + r)].x, vb = ks[64 * (P_AB1 + r)].y;
    const float wx = vx + partner(vx), wy = vy + partner(vy), xa = va + partner(va), xb = vb + partner(vb);
    if (lo && act && j < NB) {
      part1[A1L.oLw + 0 * A1L.NL + o * NB + j] = wx;
      part1[A1L.oLw + 1 * A1L.NL + o * NB + j] = wy;
      part1[A1L.oLa + o * NB + j] = xa;
      part1[A1L.oLb + o * NB + j] = xb;
    } else if (lo && act && j == NB) {   // the SiLU job: base sums of edges (d, o)
      part1[A1L.oBase + 0 * H + o] = wx;
      part1[A1L.oBase + 1 * H + o] = wy;
    }
  }
#pragma unroll
  for (int oo = 0; oo < H; ++oo) {
    const float v = oo % 2 ? ks[64 * (P_LW0 + oo / 2)].y : ks[64 * (P_LW0 + oo / 2)].x;
    const float w = v + partner(v);
    if (lo && q < NB) part[A0L.oLw + oo * A0L.NL + xi * NB + q] = w;
  }
  {
    const float va = ks[64 * P_AB0].x, vb = ks[64 * P_AB0].y;
    const float xa = va + partner(va), xb = vb + partner(vb);
    if (lo && q < NB) {
      part[A0L.oLa + xi * NB + q] = xa;
      part[A0L.oLb + xi * NB + q] = xb;
    }
  }
}
