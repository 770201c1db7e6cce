// fetode_fused.hip — the single-launch fixed-grid integrator of the depth-2 LV KAN / KAN-FET field.
//
// One launch integrates the whole t-grid (torchdiffeq FixedGridODESolver.integrate): every RK
// stage evaluation of the field, the hysteresis state updates in exact call order
// (ferro_class.py:409), the stage combines (rk_common.rk4_alt_step_func op order) and the
// output writes.  Nothing but y0, the parameters and the outputs touch HBM.
//
// Kernel: fused4_kernel — one wave = two trajectories, packed-FP32 Ferro pairs,
// branch-free feature streams.  (Earlier variants v1-v3 and the one-trajectory-per-wave v5 were
// measured slower and removed from the library; they are in the git history before round 2.)
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fetode_common.h"
#include "fetode_fieldn_plan.h"
#if (defined(FETODE_EXP_NO_GRIDSUM) || defined(FETODE_EXP_NO_EVAL)) && !defined(FETODE_DIAG)
#error "FETODE_EXP_NO_GRIDSUM / FETODE_EXP_NO_EVAL are diagnostic knobs: build them with make diag"
#endif

using namespace fetode;

// In-kernel phase timing for the v4 kernel (diagnostic build only: make stamps).  Each wave
// accumulates s_memtime deltas per phase; the stamp waits for LDS (lgkmcnt(0)), so a stamped
// run attributes time, it does not reproduce the unstamped schedule exactly.
#ifdef FETODE_STAMPS
__device__ unsigned long long* g_fetode_stamps;
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_DECL            \
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long st_last = stamp_now();
#define STAMP(p)                                  \
  do {                                            \
    const unsigned long long st_t = stamp_now();  \
    st_acc[p] += st_t - st_last;                  \
    st_last = st_t;                               \
  } while (0)
#define STAMP_FLUSH()                                                                \
  do {                                                                               \
    if (threadIdx.x == 0 && g_fetode_stamps)                                         \
      for (int p_ = 0; p_ < 8; ++p_) g_fetode_stamps[blockIdx.x * 8 + p_] = st_acc[p_]; \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(p)
#define STAMP_FLUSH()
#endif

// Wave priority around an evaluation's serial phases (round 6).  At two trajectories per wave two
// waves share each SIMD and run the same instruction stream; the SIMD arbitrates their VALU issue by
// priority, then age.  The wave in a serial phase (the DPP / permlane reductions, the stage combine,
// the feature exchange) raises its priority so it gets through the dependent chain, and drops it for
// the Ferro pair rounds, whose independent instructions then fill the other wave's latency.
// Measured B = 4096: 159.9 -> 152.6 us per solve (tools/diag/fwd_ab.py, profiles/r06_prio_ab.log);
// at one wave per SIMD (TPW = 1, v8) there is no partner to yield to and it costs 2 %: TPW = 2 only.
#define PRIO_HI() \
  do {            \
    if constexpr (TPW == 2) __builtin_amdgcn_s_setprio(1); \
  } while (0)
#define PRIO_LO() \
  do {            \
    if constexpr (TPW == 2) __builtin_amdgcn_s_setprio(0); \
  } while (0)

#ifdef FETODE_ISA_MARKERS
#define FETODE_MARK(s) asm volatile("; MARK " s ::: "memory")
#else
#define FETODE_MARK(s)
#endif

namespace {

#include "fetode_gridsum.h"

#include "fetode_xrank.h"

// Trajectory-sharded solve (xr_world > 1): the rank sum of every grid reduction is formed by ONE
// extra workgroup (the last of the grid; the compute workgroups' path changes only in which counter
// they poll and where they read the result, so their registers do not grow).  Per round r it waits
// for the local top counter, sums the local leaf sums (the single-device order), writes this GPU's
// {s0, s1} into slot `rank` of every rank's inbox (remote stores over xGMI; its own by a local
// store), polls its own inbox until every rank's record of round r is there, sums them in rank
// order (the same order on every rank: every rank takes the same decisions) and publishes the
// result through xr_g and the ready-counter replicas the compute workgroups poll.  Inbox records are
// double-buffered by round parity: a rank writes round r + 2 into a peer's slot only after it has
// received that peer's round r + 1 record, which the peer sent after reading round r.  The loop
// ends when the compute workgroups post the solve's round count (dp_fin) or the abort word rises.
// Bounded spins; a timeout raises the abort word (status 4) and the peers time out in turn.
__device__ __forceinline__ unsigned* dp_fin(const DopriParams& P) { return P.bar + kDpLine * kDpGroups; }

__device__ void xrank_comm(const DopriParams& P) {
  const int lane = threadIdx.x & 63;
  const int W = P.xr_world;
  const unsigned nloc = (unsigned)P.n_leaf_local;
  unsigned* abw = dp_abort(P);
  for (unsigned r = 0;; ++r) {
    const unsigned par = r & 1u;
    // 1. this grid's leaves of round r (or the end of the solve)
    int stop = 0;
    if (lane == 0) {
      const unsigned want = nloc * (r + 1u);
      unsigned spins = 0;
      for (;;) {
        if ((int)(__hip_atomic_load(dp_top(P, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) >= 0) break;
        const unsigned fin = __hip_atomic_load(dp_fin(P), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((fin != 0u && fin <= r + 1u) || __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          stop = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (++spins == (P.spin_limit ? P.spin_limit : kXrSpinLimit)) {
          __hip_atomic_store(abw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stop = 1;
          break;
        }
      }
      dp_order();
    }
    if (__shfl(stop, 0)) return;
    const double* xs = P.xs + 2 * kDpGroups * par;
    double u0 = 0.0, u1 = 0.0;
    if ((unsigned)lane < nloc) dp_ld16(&xs[2 * (P.leaf_lo + lane)], u0, u1);
    // 2. send: the leaves themselves at their global leaf index (exact), or this grid's total at
    //    index `rank`; then the round's tag (after the payload stores have completed)
    if (P.xr_exact) {
      if ((unsigned)lane < nloc)
        for (int p = 0; p < W; ++p) xr_st16(xr_rec(P.xr_peers[p], par, P.leaf_lo + lane), u0, u1);
    } else {
      const double t0 = xor_sum64(u0), t1 = xor_sum64(u1);
      if (lane < W) xr_st16(xr_rec(P.xr_peers[lane], par, P.xr_rank), t0, t1);
    }
    const unsigned long long tag = ((unsigned long long)P.xr_epoch << 32) | (unsigned long long)(r + 1u);
    if (lane < W) xr_st_tag(xr_tagp(P.xr_peers[lane], par, P.xr_rank), tag);
    // 3. receive every rank's round-r tag, then the records
    int ab = 0;
    if (lane < W) {
      const double* tg = xr_tagp(P.xr_inbox, par, lane);
      unsigned spins = 0;
      while (xr_ld_tag(tg) != tag) {
        __builtin_amdgcn_s_sleep(2);
        if ((spins & 255u) == 255u && __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          ab = 1;
          break;
        }
        if (++spins == (P.spin_limit ? P.spin_limit : kXrSpinLimit)) {
          __hip_atomic_store(abw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ab = 1;
          break;
        }
      }
    }
    if (__any(ab)) return;
    double g0 = 0.0, g1 = 0.0;
    if (P.xr_exact) {   // the single device's final step: lane per leaf, xor tree
      double v0 = 0.0, v1 = 0.0;
      if (lane < P.n_leaf_global) xr_ld16(xr_rec(P.xr_inbox, par, lane), v0, v1);
      g0 = xor_sum64(v0);
      g1 = xor_sum64(v1);
    } else {            // rank totals in rank order (the same order on every rank)
      double v0 = 0.0, v1 = 0.0;
      if (lane < W) xr_ld16(xr_rec(P.xr_inbox, par, lane), v0, v1);
      for (int j = 0; j < W; ++j) {
        g0 += __shfl(v0, j);
        g1 += __shfl(v1, j);
      }
    }
    // 4. publish to this grid
    if (lane == 0) dp_st16(P.xr_g + 2 * par, g0, g1);
    dp_order();
    if (lane < kDpTopCopies) __hip_atomic_fetch_add(dp_ready(P, lane), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
  float* tape;            // (n_evals, B, D+H) layer inputs of every evaluation (training), or null
  int32_t single_eval;  // 1: eval_out = field(y0) once (fetode_field_forward)
  float* eval_out;
  float factor_limit;   // kFactorLimit (FETODE_FACTOR_LIMIT=-1 disables the factored gate: diagnostics)
  DopriParams dp;       // dp.on: the whole dopri5 solve in this launch (fetode_integrate_dopri5)
};

// integer version (knot counts)
__device__ __forceinline__ int group3_sum_i(int v, int c) {
  const int s0 = v + __builtin_amdgcn_update_dpp(0, v, 0x101, 0xF, 0xF, false) +
                 __builtin_amdgcn_update_dpp(0, v, 0x102, 0xF, 0xF, false);
  const int b1 = __builtin_amdgcn_mov_dpp(s0, 0x111, 0xF, 0xF, false);
  const int b2 = __builtin_amdgcn_mov_dpp(s0, 0x112, 0xF, 0xF, false);
  return c == 0 ? s0 : (c == 1 ? b1 : b2);
}
// knots <= x among this lane's N knots: one compare + one carry-in add per knot
template <int N>
__device__ __forceinline__ int knot_count(float x, const float* kn) {
  int cnt = 0;
#pragma unroll
  for (int t = 0; t < N; ++t)
    asm volatile("v_cmp_ge_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(cnt) : "v"(x), "v"(kn[t]) : "vcc");
  return cnt;
}

// sum over lanes 3k, 3k+1, 3k+2 of a row (k < 5), result on all three
__device__ __forceinline__ float group3_sum(float v, int c) {
  const float s0 = v + dpp<0x101>(v) + dpp<0x102>(v);  // row_shl:1, row_shl:2 -> valid at c == 0
  const float b1 = dppm<0x111>(s0);                     // row_shr:1 -> lane 3k+1 gets s0[3k]
  const float b2 = dppm<0x112>(s0);                     // row_shr:2 -> lane 3k+2 gets s0[3k]
  return c == 0 ? s0 : (c == 1 ? b1 : b2);
}

// =============================================================================================
// v4: packed-FP32 Ferro pairs, branch-free feature streams — same wave shape as v3.
//
// The field is VALU-issue bound: v3 spends ~320 VALU + ~60 transcendental
// instructions per evaluation per wave.  v4 keeps v3's trajectory/row mapping and cuts the
// VALU count:
//   * a lane evaluates its Ferro elements two at a time, (i, k) and (i, k+1) of one input, in
//     v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (two fp32 lanes per instruction) with the
//     input's x, gate factor and exp(gs x) broadcast from one ds_read_b128; only the
//     transcendentals stay one per element;
//   * feature weights are applied as packed FMAs over a contiguous 8-float LDS chunk;
//   * every feature job (logistic j, SiLU, gate sigmoid, exp(gs x)) is the same
//     sigmoid-of-affine instruction stream with per-lane constants, so the feature phases do
//     not diverge; the knot interval is a per-lane compare + DPP row count instead of a
//     12-step scan on one lane.
// =============================================================================================
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }
__device__ __forceinline__ f2 ex2x2(f2 v) { return f2{ex2(v.x), ex2(v.y)}; }
__device__ __forceinline__ f2 rcpx2(f2 v) { return f2{rcp(v.x), rcp(v.y)}; }

template <int IN, int FLEN>
struct V4Lds {
  float F[FLEN];  // per input NFP floats: SiLU, logistic 0..NB-1 (2x folded into weights), zero pad
  // per input {e = exp2(gs*log2e*x), w = wc*(1-up)} and {x, pad}: each packed operand of a pair is
  // the low or high half of a loaded register pair (op_sel broadcasts, no moves)
  float4 G[IN];
  int M[IN];      // knot interval (NI = zero table row)
  float sink;     // target of idle feature jobs
};
// the two register pairs of input i ({e, w}, {x, pad}); the empty asm keeps each a loaded pair
template <int IN, int FLEN>
__device__ __forceinline__ void v4_g(const V4Lds<IN, FLEN>& L, int i, f2& ew, f2& xp) {
  const f2* g2 = reinterpret_cast<const f2*>(&L.G[i]);
  ew = g2[0];
  xp = g2[1];
  asm volatile("" : "+v"(ew), "+v"(xp));
}

// one Ferro element pair of one input: acc += cps * tanh(k (x - Ec m)) for both
template <bool FACT>
__device__ __forceinline__ f2 v4_pair(f2 ew, f2 xp, f2 ep, f2 k2, f2 kE, f2 cp, f2 acc, float gsl2e) {
  f2 s;
  if constexpr (FACT) {
    s = rcpx2(pfma(splat(ew.x), ep, splat(1.0f)));              // sigma(gs(-x-Ec)), factored exp
  } else {
    s = rcpx2(ex2x2(pfma(splat(gsl2e), splat(xp.x), ep)) + splat(1.0f));
  }
  const f2 m = pfma(splat(ew.y), s, splat(1.0f));                 // 1 - 2(1-a)(1-u) sigma
  const f2 z = pfma(kE, m, k2 * splat(xp.x));                     // 2 log2e k (x - Ec m)
  const f2 th = pfma(rcpx2(ex2x2(z) + splat(1.0f)), splat(-2.0f), splat(1.0f));
  return pfma(cp, th, acc);
}

// one Ferro element (the single leftover of a layer's pair split): acc + cps * tanh(...)
template <bool FACT>
__device__ __forceinline__ float v4_single(f2 ew, f2 xp, float ep, float k2, float kE, float cp, float acc,
                                           float gsl2e) {
  float s;
  if constexpr (FACT) {
    s = rcp(ffma(ew.x, ep, 1.0f));
  } else {
    s = rcp(ex2(ffma(gsl2e, xp.x, ep)) + 1.0f);
  }
  const float m = ffma(ew.y, s, 1.0f);
  const float z = ffma(kE, m, k2 * xp.x);
  const float th = ffma(rcp(ex2(z) + 1.0f), -2.0f, 1.0f);
  return ffma(cp, th, acc);
}

// Ferro element split of one layer's output over a lane group: NPAIR element pairs (i, k), (i, k+1)
// over `lanes` lanes.  When the remainder of pairs is at most half a round, the full rounds stay
// pairs (NPL per lane) and the leftover pairs' elements go one per lane (NSL = 1: a single-element
// round costs about half a pair round); otherwise one more pair round (NSL = 0).
template <int NPAIR, int LANES>
struct FerroSplit {
  static constexpr int REM = NPAIR % LANES;
  static constexpr bool SPLIT = REM > 0 && 2 * REM <= LANES;
  static constexpr int NPL = SPLIT ? NPAIR / LANES : (NPAIR + LANES - 1) / LANES;
  static constexpr int NSL = SPLIT ? 1 : 0;
};

// the edge sum of one lane: NPL Ferro pairs (+ NSL single elements), FPL feature weights, and
// (spl) the spline edge of input `si` (sp_o = the layer's LDS cubic table at output o, kr = the
// layer's (knot, 1/width) table by (input, interval): u = (x - knot) / width is formed here, from
// the interval index the feature phase wrote; the zero row NI holds (0, 0): u = 0 for finite x and
// NaN otherwise, as the reference's bases)
// (round 6) x_si's knot interval comes from the feature phase's wave ballot `bal` (the trajectory's
// 16-bit row of input si starts at bit `bbase` + 16 si): every lane forms it in registers, so the
// spline table reads issue straight after the exchange instead of behind an LDS read of the interval.
// A non-finite x counts 0 or all knots (lanes >= NG hold +inf): the zero row, whose (x - 0) * 0 is the
// reference's NaN — no separate finiteness test.
template <int IN, int FLEN, int NI, int NPL, int NSL, int FPL, bool FERRO, bool FACT>
__device__ __forceinline__ float v4_edges(const V4Lds<IN, FLEN>& L, const float* sp_o, const f2* kr,
                                          const int* gi, const f2* ep, const f2* k2, const f2* kE, const f2* cp,
                                          const f2* fw, int fofs, bool spl, int si, float gsl2e, int gis, float eps,
                                          float k2s, float kEs, float cps, uint64_t bal, int bbase) {
  // spline operands first (table reads by interval), so their latency hides under the pairs
  const int mraw = (int)__builtin_popcountll((bal >> (bbase + 16 * si)) & 0xFFFFull) - 1;
  const int msi = (unsigned)mraw < (unsigned)NI ? mraw : NI;
  const float xsi = L.G[si].z;
  // the cubic tables' rows are NI + 2 float4 apart (NI + 1 entries and a pad, fused4_kernel)
  const float4 cf = *reinterpret_cast<const float4*>(&sp_o[(si * (NI + 2) + msi) * 4]);
  const f2 kw = kr[si * (NI + 1) + msi];
  f2 acc = splat(0.0f);
  float sgl = 0.0f;
  if constexpr (FERRO) {
    // the single element's dependent chain first: independent of the pairs, so its transcendental
    // latencies interleave with theirs
    if constexpr (NSL > 0) {
      f2 ew, xp;
      v4_g(L, gis, ew, xp);
      sgl = v4_single<FACT>(ew, xp, eps, k2s, kEs, cps, 0.0f, gsl2e);
    }
#pragma unroll
    for (int r = 0; r < NPL; ++r) {
      f2 ew, xp;
      v4_g(L, gi[r], ew, xp);
      acc = v4_pair<FACT>(ew, xp, ep[r], k2[r], kE[r], cp[r], acc, gsl2e);
    }
  }
  const float u = (xsi - kw.x) * kw.y;
  // feature weights after the pairs (measured: 191 vs 201 us per B = 4096 solve with them first)
  if constexpr (FPL % 4 == 0) {  // chunk offsets are 16-byte aligned: ds_read_b128
    const float4* Fp = reinterpret_cast<const float4*>(&L.F[fofs]);
#pragma unroll
    for (int f = 0; f < FPL / 4; ++f) {
      const float4 v = Fp[f];
      acc = pfma(fw[2 * f], f2{v.x, v.y}, acc);
      acc = pfma(fw[2 * f + 1], f2{v.z, v.w}, acc);
    }
  } else {  // 8-byte aligned chunks: ds_read_b64
    static_assert(FPL % 2 == 0, "feature chunks are float pairs");
    const f2* Fp = reinterpret_cast<const f2*>(&L.F[fofs]);
#pragma unroll
    for (int f = 0; f < FPL / 2; ++f) acc = pfma(fw[f], Fp[f], acc);
  }
  const float sv = ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x);
  return ((acc.x + acc.y) + sgl) + (spl ? sv : 0.0f);
}

// HOT = true: the rk4 (3/8) integrate path only, every stage inlined, outputs predicated;
// HOT = false: single evaluations and every other method.  At least 2 waves per SIMD in every
// variant: the resident dopri5 grid (DOPRI) needs B / 2 co-resident waves.
// TPW = 1 (inference, mid batches): ONE trajectory per wave — each hidden unit's group is 6 lanes, the
// 3 of the v7 map in each half-wave, and the halves split its Ferro pairs and feature rounds (per-lane
// constants: no divergence); the halves' partial sums meet with one v_permlane32_swap each (the same
// sum, in the same order, on both halves).  Half the pair rounds per lane: a shorter dependent chain
// per evaluation where the waves do not fill the SIMDs.
template <int H, int K_, int NB, int NG, bool FERRO, bool HOT, bool DOPRI = false, bool TAPE = false, int TPW = 2>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void fused4_kernel(FusedArgs a) {
  constexpr int D = 2, NI = NG - 1, NFL = 1 + NB, NFP = (NFL + 1) & ~1, K = FERRO ? K_ : 0;
  // feature jobs: logistic 0..NB-1, SiLU, [gate, exp(gs x)], then x / u / m stores
  constexpr int J_SILU = NB, J_GATE = NB + 1, J_EXP = NB + 2, J_X = FERRO ? NB + 3 : NB + 1;
  constexpr int J_M = J_X + 1;
  static_assert(J_M < 16 && NG <= 16, "v4 layout: NB logistic + SiLU (+ gate, exp) + x, m jobs on a row of 16 lanes");
  static_assert(H <= 10, "v4 layout: H <= 10 groups of 3 lanes");
  static_assert(!FERRO || K % 2 == 0, "v4 pairs Ferro elements (i, k), (i, k+1)");
  constexpr int KP = K / 2 > 0 ? K / 2 : 1;
  static_assert(TPW == 2 || (TPW == 1 && HOT && !DOPRI), "one trajectory per wave: the rk4 path");
  constexpr int NLG = TPW == 2 ? 3 : 6;                      // lanes per hidden unit
  // layer 0 (2 -> H): output o on a group of 3 lanes; layer 1 (H -> 2): hidden INPUT o on the
  // same group (v7): its features, its Ferro elements of both outputs (pairs (o, 0, k), (o, 1, k):
  // one packed pair feeds both output sums) and its two spline edges stay in the group's
  // registers — no LDS exchange between layer 0 and layer 1
  using FS0 = FerroSplit<D * KP, NLG>;
  static_assert(!FERRO || D == 2, "v7 layer 1 pairs the two outputs of an input");
  constexpr int REM1 = K % NLG;
  constexpr bool SPLIT1 = TPW == 2 && REM1 == 1;             // one k left: two singles (d = 0, 1)
  constexpr int NPL0 = FERRO ? FS0::NPL : 0, NPL1 = FERRO ? (SPLIT1 ? K / NLG : (K + NLG - 1) / NLG) : 0;
  constexpr int NSL0 = FERRO ? FS0::NSL : 0, NSL1 = (FERRO && SPLIT1) ? 1 : 0;
  constexpr int FPL0 = ((D * NFP + NLG - 1) / NLG + 3) & ~3;
  constexpr int RF1 = (NFL + NLG - 1) / NLG;                 // feature rounds of a hidden input (SiLU + NB)
  constexpr int FLEN0 = (NLG * FPL0 > D * NFP ? NLG * FPL0 : D * NFP);
  if constexpr (DOPRI) {
    if (a.dp.xr_world > 1 && blockIdx.x == gridDim.x - 1) {   // the cross-rank exchange workgroup
      xrank_comm(a.dp);
      return;
    }
  }
  constexpr int KT = (NG + 2) / 3;                   // knots per group lane
  static_assert(3 * KT >= NG, "knots per group lane");
  // edge cubic tables by interval, one row of NI + 1 float4 per edge padded to SPR: at a pitch of 12
  // float4 the rows of units 4 apart (layer 1) / of the same parity (layer 0) start on the same
  // 16-byte slot of the bank row and the lanes' interval reads collide (35 % of the kernel's LDS
  // cycles were conflicts, profiles/r06_lds_bench_nores.txt)
  constexpr int SPR = NI + 2, SPE = (NI + 1) * 4;
  constexpr int SPT0 = H * D * SPR * 4, SPT1 = D * H * SPR * 4;

  __shared__ __attribute__((aligned(16))) float s_sp0[SPT0];
  __shared__ __attribute__((aligned(16))) float s_sp1[SPT1];
  __shared__ __attribute__((aligned(8))) f2 s_kr0[D * (NI + 1)], s_kr1[H * SPR];
  __shared__ float s_c0[H], s_c1[D];
  __shared__ __attribute__((aligned(16))) V4Lds<D, FLEN0> s_L0[TPW];

  const int tid = threadIdx.x;
  const int hh = tid >> 5;                                   // half-wave
  const int g = TPW == 2 ? hh : 0, lane = tid & 31, row = lane >> 4, c1 = lane & 15;
  const int64_t b = (int64_t)blockIdx.x * TPW + g;
  const bool own = TPW == 2 || hh == 0;                      // TPW 1: half 0 stores
  const bool valid = b < a.B;
  V4Lds<D, FLEN0>& L0 = s_L0[g];

  for (int i = tid; i < H * D * SPE; i += 64) s_sp0[(i / SPE) * SPR * 4 + i % SPE] = a.plan[a.P0.sp + i];
  for (int i = tid; i < D * H * SPE; i += 64) s_sp1[(i / SPE) * SPR * 4 + i % SPE] = a.plan[a.P1.sp + i];
  for (int i = tid; i < D * (NI + 1); i += 64) {
    const int in = i / (NI + 1), m = i % (NI + 1);
    s_kr0[i] = m < NI ? f2{a.plan[a.P0.knots + in * NG + m], a.plan[a.P0.rh + in * NI + m]} : f2{0.f, 0.f};
  }
  for (int i = tid; i < H * (NI + 1); i += 64) {
    const int in = i / (NI + 1), m = i % (NI + 1);
    s_kr1[in * SPR + m] = m < NI ? f2{a.plan[a.P1.knots + in * NG + m], a.plan[a.P1.rh + in * NI + m]} : f2{0.f, 0.f};
  }
  for (int i = tid; i < H; i += 64) s_c0[i] = a.plan[a.P0.fconst + i];
  for (int i = tid; i < D; i += 64) s_c1[i] = a.plan[a.P1.fconst + i];
  for (int i = lane; i < FLEN0; i += 32) L0.F[i] = 0.f;  // pads stay zero (finite x zero weight)

  const bool fact = FERRO && a.plan[a.P0.flag] <= a.factor_limit && a.plan[a.P1.flag] <= a.factor_limit;
  const float l2 = FETODE_LOG2E;

  // ---- layer-0 edge lane: output o0 = 5 row + q/3, part cc0 ----
  const int q = c1;
  const int o0 = row * 5 + q / 3, cc0 = q % 3;
  const bool act0 = q < 15 && o0 < H;
  const int o0c = act0 ? o0 : 0;
  const int gl = TPW == 2 ? cc0 : cc0 + 3 * hh;              // lane within the hidden unit's group
  f2 ep0[NPL0 > 0 ? NPL0 : 1], k20[NPL0 > 0 ? NPL0 : 1], kE0[NPL0 > 0 ? NPL0 : 1], cp0[NPL0 > 0 ? NPL0 : 1];
  int gi0[NPL0 > 0 ? NPL0 : 1];
#pragma unroll
  for (int r = 0; r < NPL0; ++r) {
    const int P = gl * NPL0 + r;
    const bool ok = act0 && P < D * KP;
    int i = ok ? P / KP : 0;
    asm volatile("" : "+v"(i));  // keep in a VGPR (no per-evaluation rematerialisation)
    gi0[r] = i;
    float t[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t idx = (int64_t)o0c * (D * K) + i * K + (ok ? (P % KP) * 2 + h : 0);
      const float gec = ok ? a.plan[a.P0.fe_GEc + idx] : 0.f;
      t[0][h] = fact ? ex2(gec) : gec;
      t[1][h] = ok ? a.plan[a.P0.fe_k2 + idx] : 0.f;
      t[2][h] = ok ? a.plan[a.P0.fe_k2Ec + idx] : 0.f;
      t[3][h] = ok ? a.plan[a.P0.fe_CPs2 + idx] : 0.f;
    }
    ep0[r] = f2{t[0][0], t[0][1]};
    k20[r] = f2{t[1][0], t[1][1]};
    kE0[r] = f2{t[2][0], t[2][1]};
    cp0[r] = f2{t[3][0], t[3][1]};
  }
  // layer-0 single: leftover element q = cc0 of pair NPL0 * 3 + q / 2
  int gs0 = 0;
  float es0 = 0.f, k2s0 = 0.f, kEs0 = 0.f, cps0 = 0.f;
  if constexpr (NSL0 > 0) {
    const int Pl = NPL0 * NLG + gl / 2;
    const bool ok = act0 && gl < 2 * FS0::REM;
    const int i = ok ? Pl / KP : 0;
    const int64_t idx = (int64_t)o0c * (D * K) + i * K + (ok ? (Pl % KP) * 2 + gl % 2 : 0);
    const float gec = ok ? a.plan[a.P0.fe_GEc + idx] : 0.f;
    es0 = fact ? ex2(gec) : gec;
    k2s0 = ok ? a.plan[a.P0.fe_k2 + idx] : 0.f;
    kEs0 = ok ? a.plan[a.P0.fe_k2Ec + idx] : 0.f;
    cps0 = ok ? a.plan[a.P0.fe_CPs2 + idx] : 0.f;
    gs0 = i;
    asm volatile("" : "+v"(gs0));
  }
  f2 fw0[FPL0 / 2];
#pragma unroll
  for (int f = 0; f < FPL0; f += 2) {
    float w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int qq = gl * FPL0 + f + h, i = qq / NFP, ff = qq % NFP;
      w[h] = (act0 && i < D && ff < NFL) ? a.plan[a.P0.kw + (int64_t)o0c * (D * NFL) + i * NFL + ff] : 0.f;
    }
    fw0[f / 2] = f2{w[0], w[1]};
  }
  // ---- layer-1 (v7): hidden input o0 on its group; lane gl owns k = gl + NLG r ----
  // pair r: elements (o0, d = 0, k) and (o0, d = 1, k): .x feeds output 0, .y output 1
  f2 ep1[NPL1 > 0 ? NPL1 : 1], k21[NPL1 > 0 ? NPL1 : 1], kE1[NPL1 > 0 ? NPL1 : 1], cp1[NPL1 > 0 ? NPL1 : 1];
#pragma unroll
  for (int r = 0; r < NPL1; ++r) {
    const int k = gl + NLG * r;
    const bool ok = act0 && k < K;
    float t[4][2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int64_t idx = (int64_t)d * (H * K) + o0c * K + (ok ? k : 0);
      const float gec = ok ? a.plan[a.P1.fe_GEc + idx] : 0.f;
      t[0][d] = fact ? ex2(gec) : gec;   // padding: ep = 1 (fact) / 0, k = 0: th = 0, cp = 0
      t[1][d] = ok ? a.plan[a.P1.fe_k2 + idx] : 0.f;
      t[2][d] = ok ? a.plan[a.P1.fe_k2Ec + idx] : 0.f;
      t[3][d] = ok ? a.plan[a.P1.fe_CPs2 + idx] : 0.f;
    }
    ep1[r] = f2{t[0][0], t[0][1]};
    k21[r] = f2{t[1][0], t[1][1]};
    kE1[r] = f2{t[2][0], t[2][1]};
    cp1[r] = f2{t[3][0], t[3][1]};
  }
  // the single left over when K % 3 == 1: element (o0, d = cc0, K - 1) on lanes cc0 = 0, 1
  float es1 = 0.f, k2s1 = 0.f, kEs1 = 0.f, cps1 = 0.f;
  if constexpr (NSL1 > 0) {
    const bool ok = act0 && cc0 < D;
    const int64_t idx = (int64_t)(ok ? cc0 : 0) * (H * K) + o0c * K + (K - 1);
    const float gec = ok ? a.plan[a.P1.fe_GEc + idx] : 0.f;
    es1 = fact ? ex2(gec) : gec;
    k2s1 = ok ? a.plan[a.P1.fe_k2 + idx] : 0.f;
    kEs1 = ok ? a.plan[a.P1.fe_k2Ec + idx] : 0.f;
    cps1 = ok ? a.plan[a.P1.fe_CPs2 + idx] : 0.f;
  }
  // lane cc0 = d < 2 also owns the spline edge (o0 -> d): the single / spline value goes to output d
  const f2 dsel1 = f2{(act0 && gl == 0) ? 1.f : 0.f, (act0 && gl == 1) ? 1.f : 0.f};
  // feature rounds: job j = cc0 + 3 r (logistic j < NB, SiLU j == NB), its weights for both outputs
  float fna1[RF1], fab1[RF1], fml1[RF1];
  f2 fwt1[RF1];
#pragma unroll
  for (int r = 0; r < RF1; ++r) {
    const int j = gl + NLG * r;
    const bool ok = act0 && j < NFL;
    fna1[r] = 0.f; fab1[r] = 0.f; fml1[r] = 0.f;
    const int ff = j < NB ? 1 + j : 0;   // kw feature index: SiLU 0, logistic j at 1 + j
    if (ok && j < NB) {
      fna1[r] = a.plan[a.P1.lg + 2 * (o0 * NB + j)];
      fab1[r] = a.plan[a.P1.lg + 2 * (o0 * NB + j) + 1];
    } else if (ok) {
      fna1[r] = -l2;
      fml1[r] = 1.f;   // SiLU: h * sigmoid(h)
    }
    fwt1[r] = ok ? f2{a.plan[a.P1.kw + (int64_t)0 * (H * NFL) + o0 * NFL + ff],
                      a.plan[a.P1.kw + (int64_t)1 * (H * NFL) + o0 * NFL + ff]}
                 : f2{0.f, 0.f};
  }
  // ---- layer-0 feature stream: input d = row, job c1 ----
  float xna, xab, xmul, xadd;
  float* xdst;
  {
    const int j = c1;
    xna = 0.f; xab = 0.f; xmul = 1.f; xadd = 0.f;
    xdst = &L0.sink;
    if (j < NB) {
      xna = a.plan[a.P0.lg + 2 * (row * NB + j)];
      xab = a.plan[a.P0.lg + 2 * (row * NB + j) + 1];
      xdst = &L0.F[row * NFP + 1 + j];
    } else if (j == J_SILU) {
      xna = -l2;
      xdst = &L0.F[row * NFP];
    } else if (FERRO && j == J_GATE) {
      xna = -a.P0.gsl2e; xmul = -a.P0.wc; xadd = a.P0.wc;
      xdst = &L0.G[row].y;
    } else if (FERRO && j == J_EXP) {
      xna = a.P0.gsl2e;
      xdst = &L0.G[row].x;
    } else if (j == J_X) {
      xdst = &L0.G[row].z;
    }
  }
  const bool x_silu = c1 == J_SILU, x_gate = FERRO && c1 == J_GATE, x_exp = FERRO && c1 == J_EXP;
  const bool x_x = c1 == J_X;
  // knot interval: lane c1 holds knot c1 (and 1/(knot c1+1 - knot c1)); the lane whose knot
  // opens the interval writes u (no LDS round trip on the critical path)
  const float xknot = c1 < NG ? a.plan[a.P0.knots + row * NG + c1] : __builtin_inff();

  // knots of hidden input o0: lane cc0 holds knots KT cc0 .. KT cc0 + KT-1
  float hknot[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int kk = KT * cc0 + t;
    hknot[t] = (act0 && kk < NG) ? a.plan[a.P1.knots + o0 * NG + kk] : __builtin_inff();
  }
  // hysteresis state: prev_x of input `row` on the layer-0 gate lane, of input o0 on every lane
  // of its group (each forms the gate itself) (ferro_class.py:409); per-layer contiguous blocks
  // (include/fetode.h)
  float prev0 = 0.f, prev1 = 0.f;
  if (FERRO && valid) {
    if (x_gate) prev0 = a.state[b * D + row];
    if (act0) prev1 = a.state[a.B * D + b * H + o0];
  }
  bool re0 = FERRO && (a.init_mask & 1u), re1 = FERRO && (a.init_mask & 2u);

  float y = valid ? a.y0[b * D + row] : 0.f;   // state dim `row`, replicated over the row
  if (!a.single_eval && valid && own && c1 == 0) a.solution[b * D + row] = y;
  __syncthreads();  // tables staged

  STAMP_DECL
  const float c0o = s_c0[o0c], c1o = s_c1[row];  // per-output constants, held in registers
  const float* sp0_o = &s_sp0[o0c * D * SPR * 4];
  // layer 1: the cubic table of edge (o0 -> d = cc0) and the (knot, 1/width) rows of input o0
  const float* sp1_e = &s_sp1[((gl < D ? gl : 0) * H + o0c) * SPR * 4];
  const f2* kr1_o = &s_kr1[o0c * SPR];
  const int fofs0 = gl * FPL0;
  const bool spl0 = act0 && gl < D;  // lanes owning a layer-0 spline edge (input si)
  const int si0 = spl0 ? gl : 0;

  // training tape: the two layer inputs of evaluation `ev` at tape[(ev B + b)(D + H) + c]
  // TAPE = false (every inference instantiation) carries no tape code at all: the fixed-grid
  // training forward and the dopri5 driver have taped instantiations of their own
  bool taping = TAPE && a.tape != nullptr;
  // the dopri5 tape holds the first tape_cap evaluations (the host re-runs a longer solve)
  int64_t tape_left = DOPRI ? a.dp.tape_cap : 0;
  // dopri5 training rows also hold the evaluation's output k after the two layer inputs
  constexpr int TW = DOPRI ? 2 * D + H : D + H;
  float* tape_b = taping ? a.tape + (valid ? b : 0) * TW : nullptr;
  const int64_t tape_stride = a.B * TW;
  uint64_t bal0 = 0;   // the feature phase's knot ballot (both trajectories' rows of both inputs)
  auto eval_body = [&](float xin, auto fact_tag) __attribute__((always_inline)) -> float {
    constexpr bool F_ = decltype(fact_tag)::value;
    STAMP(6);
    FETODE_MARK("X_FEAT");
    {
      // (1) layer-0 features of input `row`: one sigmoid-of-affine job per lane
      const float pv = x_gate ? (re0 ? xin : prev0) : 0.f;
      const float e = ex2(ffma(xna, xin - pv, xab));
      const float sg = rcp(1.0f + e);
      float val = ffma(sg, x_silu ? xin : xmul, xadd);
      val = x_exp ? e : val;
      val = x_x ? xin : val;
      // knot intervals: lanes c1 < NG compare against their knot (the rest hold +inf); the edge
      // lanes count their input's row of this ballot themselves (v4_edges)
      bal0 = __builtin_amdgcn_ballot_w64(xin >= xknot);
      *xdst = val;
      if (FERRO) prev0 = xin;  // ferro_class.py:409 (meaningful on the gate lane)
      re0 = false;
    }
    STAMP(0);
    // the workgroup is this one wave: its LDS operations execute in order, so the edge reads see the
    // feature writes with no wait on them (a wave barrier only keeps the compiler from reordering)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    STAMP(0);
    FETODE_MARK("EDGES0");
    PRIO_LO();
    // (2) layer-0 edges -> h_o on the group of 3
    float h = v4_edges<D, FLEN0, NI, NPL0, NSL0, FPL0, FERRO, F_>(L0, sp0_o, s_kr0, gi0, ep0, k20, kE0, cp0, fw0,
                                                                  fofs0, spl0, si0, a.P0.gsl2e, gs0, es0, k2s0, kEs0,
                                                                  cps0, bal0, TPW == 2 ? 32 * g : 0);
    if constexpr (TPW == 1) {   // the two halves' partial edge sums (the same sum on both halves)
      float p = h, q2 = h;
      permlane32_swap(p, q2);
      h = p + q2;
    }
    PRIO_HI();
    h = group3_sum(h, cc0) + c0o;   // lane 15 of a row (no group) is never read by a group
    STAMP(2);
    FETODE_MARK("H_FEAT");
    // (3) layer 1 on the group of hidden input o0 (v7): partial sums of BOTH outputs in acc01
    f2 acc01 = splat(0.0f);
    {
      // knot interval of h: KT compares per lane, summed over the group
      // (a non-finite h counts 0 or all 12 knots: the zero row, no finiteness test needed)
      const int mm = group3_sum_i(knot_count<KT>(h, hknot), cc0) - 1;
      const int mfix = (unsigned)mm < (unsigned)NI ? mm : NI;
      // spline operands by interval (the zero row NI holds (0, 0): u = 0 for finite h, NaN
      // otherwise, as the reference's bases); their LDS latency hides under the pairs
      const float4 cf = *reinterpret_cast<const float4*>(&sp1_e[mfix * 4]);
      const f2 kw = kr1_o[mfix];
      float sgl = 0.0f;
      if constexpr (FERRO) {
        // every lane of the group forms the gate and exp(gs h) of its input itself (three
        // transcendentals: cheaper than broadcasting them across a group of 3 lanes)
        const float pv = re1 ? h : prev1;
        const float eg = ex2(ffma(-a.P1.gsl2e, h - pv, 0.0f));
        const float w = ffma(rcp(1.0f + eg), -a.P1.wc, a.P1.wc);   // wc (1 - up)
        const float e = F_ ? ex2(ffma(a.P1.gsl2e, h, 0.0f)) : 0.0f;
        prev1 = h;   // ferro_class.py:409
        re1 = false;
        const f2 ew = f2{e, w}, xp = f2{h, 0.0f};
        PRIO_LO();
        if constexpr (NSL1 > 0) sgl = v4_single<F_>(ew, xp, es1, k2s1, kEs1, cps1, 0.0f, a.P1.gsl2e);
#pragma unroll
        for (int r = 0; r < NPL1; ++r) acc01 = v4_pair<F_>(ew, xp, ep1[r], k21[r], kE1[r], cp1[r], acc01, a.P1.gsl2e);
      }
      // the group's features (SiLU + NB logistic), each weighted for both outputs
#pragma unroll
      for (int r = 0; r < RF1; ++r) {
        const float e = ex2(ffma(fna1[r], h, fab1[r]));
        const float sg = rcp(1.0f + e);
        const float val = fml1[r] != 0.0f ? h * sg : sg;   // SiLU h sigma(h) / logistic sigma
        acc01 = pfma(fwt1[r], splat(val), acc01);
      }
      const float u = (h - kw.x) * kw.y;
      const float sv = ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x);
      acc01 = pfma(dsel1, splat(sgl + sv), acc01);   // lane d < 2: single + spline onto output d
#ifndef FETODE_EXPERIMENT_NO_TAPE_STORE
      // the evaluation's tape row in ONE non-temporal store: h_o from the group's first lane, x_row
      // from the row's idle lane 15 (two plain stores cost the B = 4096 taped solve 23 us over none,
      // this one 15: profiles/r06_tape_store_ab.log; the sweep reads the rows long after)
      if (taping && valid && own && ((act0 && cc0 == 0) || q == 15))
        __builtin_nontemporal_store(q == 15 ? xin : h, tape_b + (q == 15 ? row : D + o0));
#endif
    }
    if (taping) {
      tape_b += tape_stride;
      if constexpr (DOPRI) taping = --tape_left > 0;
    }
    STAMP(3);
    // output sums over the half-wave: the permlane16 swap folds the two rows of each output into
    // row d (rows 0 / 2: output 0, rows 1 / 3: output 1), a row sum finishes: k_row on row `row`
    PRIO_HI();
    float p0 = acc01.x, p1 = acc01.y;
    if constexpr (TPW == 1) {   // the two halves' partials first (the same sums on both halves)
      float p = p0, q2 = p0;
      permlane32_swap(p, q2);
      p0 = p + q2;
      float r = p1, t = p1;
      permlane32_swap(r, t);
      p1 = r + t;
    }
    permlane16_swap(p0, p1);
    const float kr = row_sum16(p0 + p1) + c1o;
    STAMP(5);
    FETODE_MARK("END");
    return kr;
  };
  // the step / output schedule is staged through LDS in chunks: per-step global loads in the
  // loop would wait (vmcnt) behind the solution stores of the previous step
  constexpr int SCH = 32;
  __shared__ float s_dt[SCH], s_hh[SCH], s_h6[SCH], s_oslope[SCH];
  __shared__ int s_ostep[SCH], s_omode[SCH];
  auto load_steps = [&](int s0) {
    __syncthreads();
    for (int i = tid; i < SCH && s0 + i < a.n_steps; i += 64) {
      s_dt[i] = a.step_coef[4 * (s0 + i) + 0];
      s_hh[i] = a.step_coef[4 * (s0 + i) + 1];
      s_h6[i] = a.step_coef[4 * (s0 + i) + 2];
    }
    __syncthreads();
  };
  auto load_outs = [&](int j0) {
    __syncthreads();
    for (int i = tid; i < SCH; i += 64) {
      const bool in = j0 + i < a.T;
      s_ostep[i] = in ? a.out_step[j0 + i] : -1;
      s_omode[i] = in ? a.out_mode[j0 + i] : 1;
      s_oslope[i] = in ? a.out_slope[j0 + i] : 0.f;
    }
    __syncthreads();
  };

  auto out_write = [&](int j, float v) __attribute__((always_inline)) {
#ifndef FETODE_EXPERIMENT_NO_OUT
    if (valid && own && c1 == 0) a.solution[((int64_t)j * a.B + b) * D + row] = v;
#endif
  };
  using FT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;

  if constexpr (HOT) {
    // rk4 (torchdiffeq rk_common.rk4_alt_step_func op order); the step's first two output
    // slots are read before its stages and consumed after them, with predicated stores
    int sb = 0, jb = 1, jj = 1;
    load_steps(0);
    load_outs(1);
    auto run = [&](auto fact_tag) __attribute__((always_inline)) {
      const float third = 1.0f / 3.0f;
      for (int s = 0; s < a.n_steps; ++s) {
        if (s - sb == SCH) {
          sb = s;
          load_steps(s);
        }
        if (jj + 1 - jb >= SCH) {
          jb = jj;
          load_outs(jj);
        }
        const int sr = s - sb, jr = jj - jb;
        const float dt = s_dt[sr];
        const int os0 = s_ostep[jr], os1 = s_ostep[jr + 1], om0 = s_omode[jr];
        const float osl0 = s_oslope[jr];
        STAMP(7);
        const float k1 = eval_body(y, fact_tag);
        const float k2 = eval_body(y + (dt * k1) * third, fact_tag);
        const float k3 = eval_body(y + dt * (k2 - k1 * third), fact_tag);
        const float k4 = eval_body(y + dt * ((k1 - k2) + k3), fact_tag);
        const float y1 = y + (((k1 + 3.0f * (k2 + k3)) + k4) * dt) * 0.125f;
        if (os0 == s) {
          // mode / slope as opaque VGPRs: VALU selects instead of scalar branches on the mode
          int m0 = om0;
          float sl0 = osl0;
          asm volatile("" : "+v"(m0), "+v"(sl0));
          const float oip = y + sl0 * (y1 - y);
          const float o1 = m0 == 1 ? y1 : oip;
          out_write(jj, m0 == 0 ? y : o1);
          ++jj;
          if (os1 == s) {  // several outputs inside one step (step_size grids)
            while (jj < a.T) {
              if (jj - jb == SCH) {
                jb = jj;
                load_outs(jj);
              }
              if (s_ostep[jj - jb] != s) break;
              const int mode = s_omode[jj - jb];
              out_write(jj, mode == 0 ? y : (mode == 1 ? y1 : y + s_oslope[jj - jb] * (y1 - y)));
              ++jj;
            }
          }
        }
        STAMP(1);
        y = y1;
      }
    };
    if (fact) run(FT{});
    else run(FF{});
  } else {
    auto eval = [&](float xin) __attribute__((always_inline)) -> float {
      if (fact) return eval_body(xin, FT{});
      return eval_body(xin, FF{});
    };
    if constexpr (DOPRI) {
      // the whole driver once per coercive-gate form (as the rk4 path): the evaluations inline
      // one specialised field body, not a runtime choice between two per evaluation
      auto drive = [&](auto fact_tag) __attribute__((always_inline)) {
#ifndef FETODE_EXP_NO_EVAL
        auto eval = [&](float xin) __attribute__((always_inline)) -> float { return eval_body(xin, fact_tag); };
#else   // diagnostics only: a trivial field, the reductions and control as is
        auto eval = [&](float xin) -> float { return -0.5f * xin; };
#endif
        // ---- device-resident dopri5 (dopri5.py _Dopri5, lane (traj, dim = row) carries y_row) ----
        const DopriParams& P = a.dp;
        const bool real = valid && c1 == 0;  // one lane per (trajectory, state dim) in the sums
        const double n_el = P.n_total;   // B * D, or the global batch's in a sharded solve
        int nfev = 0, n_att = 0, status = 0;
        unsigned round = 0;
        auto gsum2 = [&](double v0, double v1, double& s0, double& s1) {
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            v0 += __shfl_xor(v0, o);
            v1 += __shfl_xor(v1, o);
          }
          if (grid_sum2(P, round, v0, v1, s0, s1)) status = 4;
        };
        // training: the output of evaluation nfev (the first tape_cap of them) next to its layer
        // inputs, in the row the evaluation just wrote (tape_b has moved past it)
        auto ktape = [&](float k) {
          if constexpr (TAPE)
            if (nfev < P.tape_cap && valid && c1 == 0) tape_b[D + H + row - tape_stride] = k;
        };
        float f0 = eval(y);
        ktape(f0);
        ++nfev;
        double dt;
        if (P.first_step > 0.0) {
          dt = P.first_step;
        } else {  // misc._select_initial_step in fp32 (dopri5.py select_initial_step)
          const float scale = P.atol + P.rtol * fabsf(y);
          const float q0 = y / scale, q1 = f0 / scale;
          double s, s1;
          gsum2(real ? (double)q0 * q0 : 0.0, real ? (double)q1 * q1 : 0.0, s, s1);
          const float d0 = fabsf(sqrtf((float)(s / n_el)));
          const float d1 = fabsf(sqrtf((float)(s1 / n_el)));
          float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
          h0 = fabsf(h0);
          const float f1 = eval(y + f0 * h0);
          ktape(f1);
          ++nfev;
          const float q2 = (f1 - f0) / scale;
          gsum2(real ? (double)q2 * q2 : 0.0, 0.0, s, s1);
          const float d2 = fabsf(sqrtf((float)(s / n_el)) / h0);
          float h1;
          if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
          else h1 = (float)pow((double)(0.01f / fmaxf(d1, d2)), (double)0.2f);  // fp64 pow rounded once: host == device
          dt = (double)fminf(100.0f * h0, fabsf(h1));
          if (TAPE && blockIdx.x == 0 && tid == 0) {
            P.init_rec[0] = d0;
            P.init_rec[1] = d1;
            P.init_rec[2] = d2;
            P.init_rec[3] = h0;
            P.init_rec[4] = h1;
          }
        }
        float co[5] = {y, 0.f, 0.f, 0.f, 0.f};
        double t0s = P.t[0], t1s = P.t[0];
        for (int i = 1; i < P.T && status == 0; ++i) {
          const double next_t = P.t[i];
          int n_steps = 0;
          while (next_t > t1s) {
            if (n_steps >= P.max_steps) { status = 3; break; }
            const double t0 = t1s;
            if (!(t0 + dt > t0)) { status = 2; break; }
            const float dt32 = (float)dt;
            const double t1 = t0 + dt;
            // rk_common._runge_kutta_step in fetode_lincomb's op order, accumulated as the stages
            // arrive: A[i] is stage s+1+i's sum k0 c0 + k1 c1 + ... (the same left-to-right sums)
            float A[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) A[q] = f0 * (P.stc[0][q] * dt32);
            float err = f0 * (P.stc[0][6] * dt32);
            float mid = f0 * (P.stc[0][7] * dt32);
            float yi = y, kn = f0;
#pragma unroll 1
            for (int st = 0; st < 6; ++st) {
              yi = y + A[0];
              // stage column st + 1 into SGPRs before the evaluation (the loads complete under it)
              float c[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) c[q] = P.stc[st + 1][q];
              kn = eval(yi);
              ktape(kn);
              ++nfev;
              // entries past the tableau (coefficient 0) are never read again
#pragma unroll
              for (int q = 0; q < 5; ++q) A[q] = A[q + 1] + kn * (c[q] * dt32);
              err = err + kn * (c[6] * dt32);
              mid = mid + kn * (c[7] * dt32);
              STAMP(6);
            }
            const float y1 = yi;
            const float tol = P.atol + P.rtol * fmaxf(fabsf(y), fabsf(y1));
            const float qe = err / tol;
            double s, nbad;
            gsum2(real ? (double)qe * qe : 0.0, (real && !__builtin_isfinite(y)) ? 1.0 : 0.0, s, nbad);
            STAMP(1);
            if (status) break;
            if (nbad != 0.0) { status = 1; break; }
            const float ratio = sqrtf((float)(s / n_el));
            const bool accept = ratio <= 1.0f;
            if (blockIdx.x == 0 && tid == 0 && n_att < P.max_att) {
              double* o = P.att + (int64_t)n_att * 4;
              o[0] = t0;
              o[1] = dt;
              o[2] = (double)ratio;
              o[3] = accept ? 1.0 : 0.0;
            }
            ++n_att;
            if (accept) {  // interp._interp_fit (fetode_interp_fit's op order)
              const float ym = y + mid, fa = f0, fb6 = kn;
              co[4] = ((2.0f * dt32) * (fb6 - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
              co[3] = ((dt32 * (5.0f * fa - 3.0f * fb6) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
              co[2] = ((dt32 * (fb6 - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
              co[1] = dt32 * fa;
              co[0] = y;
              y = y1;
              f0 = kn;
              t0s = t0;
              t1s = t1;
            } else {
              t0s = t0;
            }
            // rk_common._optimal_step_size in fp64 (dopri5.py optimal_step)
            const double rr = (double)ratio;
            double nxt;
            if (rr == 0.0) {
              nxt = dt * P.ifactor;
            } else {
              const double dfac = rr < 1.0 ? 1.0 : P.dfactor;
              const double factor = __builtin_isnan(rr) ? rr : fmin(P.ifactor, fmax(P.safety / pow(rr, 1.0 / 5.0), dfac));
              nxt = dt * factor;
            }
            dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, P.min_step), P.max_step);
            ++n_steps;
            STAMP(7);
          }
          if (status) break;
          const float xq = (float)((next_t - t0s) / (t1s - t0s));  // interp._interp_evaluate
          float total = co[0] + xq * co[1];
          float xp = xq;
#pragma unroll
          for (int j = 2; j < 5; ++j) {
            xp = xp * xq;
            total = total + xp * co[j];
          }
          out_write(i, total);
        }
        if (P.xr_world > 1 && blockIdx.x == 0 && tid == 0)   // the exchange workgroup may stop
          __hip_atomic_store(dp_fin(P), round + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (blockIdx.x == 0 && tid == 0) {
          P.stats[0] = nfev;
          P.stats[1] = n_att;
          P.stats[2] = __hip_atomic_load(P.bar + kDpLine * (kDpGroups + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 4 : status;
        }
      };
      if (fact) drive(FT{});
      else drive(FF{});
    } else if (a.single_eval) {
      const float f = eval(y);
      if (valid && c1 == 0) a.eval_out[b * D + row] = f;
    } else {
      const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4
                     : a.method == FETODE_MIDPOINT ? 2 : 1;
      const float third = 1.0f / 3.0f;
      int sb = 0, jb = 1, jj = 1;
      load_steps(0);
      load_outs(1);
      for (int s = 0; s < a.n_steps; ++s) {
        if (s - sb == SCH) {
          sb = s;
          load_steps(s);
        }
        const float dt = s_dt[s - sb], hh = s_hh[s - sb], h6 = s_h6[s - sb];
        float k1 = 0.f, k2 = 0.f, k3 = 0.f, k4 = 0.f;
        for (int st = 0; st < ns; ++st) {
          float xin = y;
          if (a.method == FETODE_RK4) {
            if (st == 1) xin = y + (dt * k1) * third;
            else if (st == 2) xin = y + dt * (k2 - k1 * third);
            else if (st == 3) xin = y + dt * ((k1 - k2) + k3);
          } else if (a.method == FETODE_RK4_CLASSIC) {
            if (st == 1) xin = y + hh * k1;
            else if (st == 2) xin = y + hh * k2;
            else if (st == 3) xin = y + dt * k3;
          } else if (a.method == FETODE_MIDPOINT) {
            if (st == 1) xin = y + k1 * hh;
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
        while (jj < a.T) {
          if (jj - jb == SCH) {
            jb = jj;
            load_outs(jj);
          }
          if (s_ostep[jj - jb] != s) break;
          const int mode = s_omode[jj - jb];
          out_write(jj, mode == 0 ? y : (mode == 1 ? y1 : y + s_oslope[jj - jb] * (y1 - y)));
          ++jj;
        }
        y = y1;
      }
    }
  }
  if (FERRO && valid && own) {
    if (x_gate) a.state[b * D + row] = prev0;
    if (act0 && cc0 == 0) a.state[a.B * D + b * H + o0] = prev1;
  }
  STAMP_FLUSH();
}

// =============================================================================================
// v6: one trajectory per 3-wave workgroup — the small-batch (strong-scaling) kernel.
//
// At B = 512 (an 8-GPU strong-scaled shard of the 4096 batch) v4 has 256 waves for 1024 SIMDs
// and every wave walks the whole evaluation chain of two trajectories (~0.17 ms per solve, lone
// wave).  v6 spreads ONE trajectory over 192 lanes so each lane's share of an evaluation is one
// short stream: row r (16 lanes) of the workgroup is layer-0 output r AND layer-1 input r
// (r < H = 10), so layer 0 -> layer 1 needs no exchange at all:
//   layer 0  the layer inputs x_0, x_1 are known to every lane; lane c takes the feature jobs
//            c and c + 16 of one sigmoid-of-affine stream (logistic, SiLU, gates, exp(gs x)),
//            the gates / exps reach the Ferro lanes by DPP row_newbcast, lanes c < 10 take one
//            packed Ferro pair (i, k..k+1) of output r, the lane whose knot opens x_i's interval
//            takes the spline edge; a DPP row sum leaves h_r on the 16 lanes of row r;
//   layer 1  row r evaluates the 13 feature jobs of h_r (one per lane), 10 Ferro pairs
//            (output o, k..k+1) and the two spline edges of input r; row sums, a readlane sum
//            over the wave's rows, and ONE workgroup barrier (per-wave partials in LDS, double-
//            buffered by evaluation parity) give k on every lane.
// The stage combines run redundantly on every lane in torchdiffeq's op order; thread 0 writes
// the outputs.  TAPE = true also records the training tapes (fixed-grid rows (x, h) and the
// dopri5 rows (x, h, k)) for B <= small_max(): the row owners write them
// (tests/test_gpu_grad.py::test_small_batch_tape_matches_v4 checks v6 vs v4 tapes and gradients).
// =============================================================================================
template <bool FERRO, bool HOT, bool DOPRI = false, bool TAPE = false>
__global__ __launch_bounds__(192) void small6_kernel(FusedArgs a) {
  constexpr int D = 2, H = 10, K = FERRO ? 10 : 0, KP = 5, NB = 10, NG = 12, NI = NG - 1, NFL = 1 + NB;
  __shared__ __attribute__((aligned(8))) f2 s_part[2][3];
  __shared__ double s_gs[2];  // dopri5: the grid sums, from wave 0
  __shared__ int s_gab;
  float* trow = nullptr;      // dopri5 training: this evaluation's tape row (x, h, k), or null
  constexpr int SCH = 32;
  __shared__ float s_dt[SCH], s_hh[SCH], s_h6[SCH], s_oslope[SCH];
  __shared__ int s_ostep[SCH], s_omode[SCH];

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = tid >> 4, c = tid & 15;
  const bool act = r < H;
  const int rr = act ? r : 0;
  const int64_t b = blockIdx.x;
  const float l2 = FETODE_LOG2E;
  const bool fact = FERRO && a.plan[a.P0.flag] <= a.factor_limit && a.plan[a.P1.flag] <= a.factor_limit;

  // ---- layer 0, row rr = output o: one Ferro pair (input i0, bases 2kp, 2kp+1) on lanes c < 10
  const int i0 = c >= KP ? 1 : 0;
  f2 ep0 = splat(0.f), k20 = splat(0.f), kE0 = splat(0.f), cp0 = splat(0.f);
  f2 ep1 = splat(0.f), k21 = splat(0.f), kE1 = splat(0.f), cp1 = splat(0.f);
  const int o1 = c >= KP ? 1 : 0;  // layer-1 pair lanes: output o1, bases 2 (c % 5) ..
  if constexpr (FERRO) {
    const bool pj = act && c < 2 * KP;
    float t0[4][2], t1[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t i0x = (int64_t)rr * (D * K) + i0 * K + (pj ? (c % KP) * 2 + h : 0);
      const float g0 = pj ? a.plan[a.P0.fe_GEc + i0x] : 0.f;
      t0[0][h] = fact ? ex2(g0) : g0;
      t0[1][h] = pj ? a.plan[a.P0.fe_k2 + i0x] : 0.f;
      t0[2][h] = pj ? a.plan[a.P0.fe_k2Ec + i0x] : 0.f;
      t0[3][h] = pj ? a.plan[a.P0.fe_CPs2 + i0x] : 0.f;
      const int64_t i1x = (int64_t)o1 * (H * K) + rr * K + (pj ? (c % KP) * 2 + h : 0);
      const float g1 = pj ? a.plan[a.P1.fe_GEc + i1x] : 0.f;
      t1[0][h] = fact ? ex2(g1) : g1;
      t1[1][h] = pj ? a.plan[a.P1.fe_k2 + i1x] : 0.f;
      t1[2][h] = pj ? a.plan[a.P1.fe_k2Ec + i1x] : 0.f;
      t1[3][h] = pj ? a.plan[a.P1.fe_CPs2 + i1x] : 0.f;
    }
    ep0 = f2{t0[0][0], t0[0][1]}; k20 = f2{t0[1][0], t0[1][1]}; kE0 = f2{t0[2][0], t0[2][1]}; cp0 = f2{t0[3][0], t0[3][1]};
    ep1 = f2{t1[0][0], t1[0][1]}; k21 = f2{t1[1][0], t1[1][1]}; kE1 = f2{t1[2][0], t1[2][1]}; cp1 = f2{t1[3][0], t1[3][1]};
  }
  // ---- layer 0 feature jobs q = c + 16 s:  logistic (0, j) | logistic (1, j) | SiLU_0, SiLU_1 |
  //      gate_0, gate_1 | exp_0, exp_1  (the last four only with FERRO)
  float fna[2], fab[2], fmul[2], fadd[2], fw[2];
  int fx[2];
  bool fsilu[2], fgate[2], fexp[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int q = c + 16 * s;
    fna[s] = 0.f; fab[s] = 0.f; fmul[s] = 1.f; fadd[s] = 0.f; fw[s] = 0.f; fx[s] = 0;
    fsilu[s] = fgate[s] = fexp[s] = false;
    if (q < 2 * NB) {
      const int i = q / NB, j = q % NB;
      fx[s] = i;
      fna[s] = a.plan[a.P0.lg + 2 * (i * NB + j)];
      fab[s] = a.plan[a.P0.lg + 2 * (i * NB + j) + 1];
      fw[s] = act ? a.plan[a.P0.kw + (int64_t)rr * (D * NFL) + i * NFL + 1 + j] : 0.f;
    } else if (q < 2 * NB + 2) {
      const int i = q - 2 * NB;
      fx[s] = i;
      fna[s] = -l2;
      fsilu[s] = true;
      fw[s] = act ? a.plan[a.P0.kw + (int64_t)rr * (D * NFL) + i * NFL] : 0.f;
    } else if (FERRO && q < 2 * NB + 4) {
      fx[s] = q - (2 * NB + 2);
      fna[s] = -a.P0.gsl2e; fmul[s] = -a.P0.wc; fadd[s] = a.P0.wc;
      fgate[s] = true;
    } else if (FERRO && q < 2 * NB + 6) {
      fx[s] = q - (2 * NB + 4);
      fna[s] = a.P0.gsl2e;
      fexp[s] = true;
    }
  }
  // Each lane computes ONE of them: even rows job c, odd rows job c + 16 (one permlane16 swap
  // per evaluation then gives every lane both values); the MAC weights stay per slot and row.
  const int so = r & 1;
  const float ona = so ? fna[1] : fna[0], oab = so ? fab[1] : fab[0];
  const float omul = so ? fmul[1] : fmul[0], oadd = so ? fadd[1] : fadd[0];
  const int ofx = so ? fx[1] : fx[0];
  const bool osilu = so ? fsilu[1] : fsilu[0], ogate = so ? fgate[1] : fgate[0], oexp = so ? fexp[1] : fexp[0];
  const bool fmac1 = !(fgate[1] || fexp[1]);  // slot-1 values to MAC (weight 0 elsewhere; never e)
  // knots of the two layer-0 inputs on lanes c < NG (every row holds the same)
  const float kn0 = c < NG ? a.plan[a.P0.knots + c] : __builtin_inff();
  const float kn1 = c < NG ? a.plan[a.P0.knots + NG + c] : __builtin_inff();
  const float rh0 = c < NI ? a.plan[a.P0.rh + c] : 0.f;
  const float rh1 = c < NI ? a.plan[a.P0.rh + NI + c] : 0.f;
  const float c0o = act ? a.plan[a.P0.fconst + rr] : 0.f;
  // the spline cubics live in registers: lane c holds knot interval c's cubic (c = NI: the zero
  // row) of its row's edges — layer 0 (r, 0), (r, 1), layer 1 (0, r), (1, r) — so the lane that
  // owns x's interval evaluates it with no LDS round trip on the evaluation's chain
  float4 cs0[D], cs1[D];
  {
    const bool hc = act && c <= NI;
    const float4* sp0 = reinterpret_cast<const float4*>(a.plan + a.P0.sp);
    const float4* sp1 = reinterpret_cast<const float4*>(a.plan + a.P1.sp);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      cs0[i] = hc ? sp0[(rr * D + i) * (NI + 1) + c] : make_float4(0.f, 0.f, 0.f, 0.f);
      cs1[i] = hc ? sp1[(i * H + rr) * (NI + 1) + c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // layer 0's two edges as packed pairs (input 0, input 1)
  const f2 s0x = f2{cs0[0].x, cs0[1].x}, s0y = f2{cs0[0].y, cs0[1].y};
  const f2 s0z = f2{cs0[0].z, cs0[1].z}, s0w = f2{cs0[0].w, cs0[1].w};
  const f2 nkn01 = f2{-kn0, -kn1}, rh01 = f2{rh0, rh1};
  auto cubic = [](float4 cf, float u) { return ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x); };

  // ---- layer 1, row rr = input i: feature job c (logistic j = c < 10, SiLU, gate, exp)
  float hna = 0.f, hab = 0.f, hmul = 1.f, hadd = 0.f, hw0 = 0.f, hw1 = 0.f;
  bool hsilu = false, hgate = false, hexp = false;
  if (act) {
    if (c < NB) {
      hna = a.plan[a.P1.lg + 2 * (rr * NB + c)];
      hab = a.plan[a.P1.lg + 2 * (rr * NB + c) + 1];
      hw0 = a.plan[a.P1.kw + (int64_t)0 * (H * NFL) + rr * NFL + 1 + c];
      hw1 = a.plan[a.P1.kw + (int64_t)1 * (H * NFL) + rr * NFL + 1 + c];
    } else if (c == NB) {
      hna = -l2;
      hsilu = true;
      hw0 = a.plan[a.P1.kw + (int64_t)0 * (H * NFL) + rr * NFL];
      hw1 = a.plan[a.P1.kw + (int64_t)1 * (H * NFL) + rr * NFL];
    } else if (FERRO && c == NB + 1) {
      hna = -a.P1.gsl2e; hmul = -a.P1.wc; hadd = a.P1.wc;
      hgate = true;
    } else if (FERRO && c == NB + 2) {
      hna = a.P1.gsl2e;
      hexp = true;
    }
  }
  // (idle rows read row 0's knots: finite u, zero cubics, zero weights -> they add exact zeros)
  const float knh = c < NG ? a.plan[a.P1.knots + rr * NG + c] : __builtin_inff();
  const float rhh = c < NI ? a.plan[a.P1.rh + rr * NI + c] : 0.f;
  const f2 hw = f2{hw0, hw1};
  const f2 psel = o1 ? f2{0.f, 1.f} : f2{1.f, 0.f};  // the lane's layer-1 Ferro pair feeds output o1
  const float c1o0 = a.plan[a.P1.fconst + 0], c1o1 = a.plan[a.P1.fconst + 1];

  // hysteresis state (ferro_class.py:409): both layer-0 inputs on every lane, input rr of layer 1
  // on its row
  // Each gate job keeps its own previous input (0 on every other job): pvs[s] for the layer-0
  // slots, pvh for layer 1.  The first evaluation is always at y0, so a fresh layer-0 state
  // (init_mask) starts from y0 directly; layer 1's first input is only known inside it (re1).
  const bool re0 = FERRO && (a.init_mask & 1u);
  bool re1 = FERRO && (a.init_mask & 2u);
  f2 y = f2{a.y0[b * D + 0], a.y0[b * D + 1]};
  float pvs = 0.f, pvh = 0.f;
  if (FERRO) {
    if (ogate) pvs = re0 ? (ofx ? y.y : y.x) : a.state[b * D + ofx];
    if (hgate) pvh = a.state[a.B * D + b * H + rr];
  }
  if (!a.single_eval && tid == 0) *reinterpret_cast<f2*>(&a.solution[b * D]) = y;
  int par = 0;
  STAMP_DECL

  auto eval_body = [&](f2 xin, auto fact_tag) __attribute__((always_inline)) -> f2 {
    constexpr bool F_ = decltype(fact_tag)::value;
    STAMP(6);
    const float x0 = xin.x, x1 = xin.y;
    // ---------------- layer 0 ----------------
    float acc, fv1;
    {
      const float x = ofx ? x1 : x0;
      const float e = ex2(ffma(ona, x - pvs, oab));
      if (FERRO) pvs = ogate ? x : 0.f;  // ferro_class.py:409
      const float sg = rcp(1.0f + e);
      const float v = ffma(sg, osilu ? x : omul, oadd);
      float f0 = oexp ? e : v, f1 = f0;
      permlane16_swap(f0, f1);  // f0: job c (the even rows' values), f1: job c + 16 (the odd rows')
      acc = fw[0] * f0;
      acc = ffma(fw[1], fmac1 ? f1 : 0.f, acc);  // gate / exp jobs carry weight 0: never MAC e (inf * 0)
      fv1 = f1;
    }
    STAMP(0);
    if constexpr (FERRO) {
      // gate_i / exp_i of the two inputs: slot 1, lanes 6..9 of every row (row_newbcast)
      const float g0 = dppm<0x156>(fv1), g1 = dppm<0x157>(fv1);
      const float e0 = dppm<0x158>(fv1), e1 = dppm<0x159>(fv1);
      const f2 ew = i0 ? f2{e1, g1} : f2{e0, g0}, xp = f2{i0 ? x1 : x0, 0.f};
      const f2 pr = v4_pair<F_>(ew, xp, ep0, k20, kE0, cp0, splat(0.0f), a.P0.gsl2e);
      acc += pr.x + pr.y;
    }
    // spline edges (r, 0), (r, 1): the lane whose knot opens the interval (ballot count over a
    // row), branch-free.  A non-finite x counts 0 or 16 knots (lanes >= NG hold +inf), so it
    // selects the zero row on lane NI, whose (x - knot) * 0 is NaN: the reference's NaN bases.
    {
      int m0 = (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(x0 >= kn0) & 0xFFFFull) - 1;
      int m1 = (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(x1 >= kn1) & 0xFFFFull) - 1;
      m0 = (unsigned)m0 < (unsigned)NI ? m0 : NI;
      m1 = (unsigned)m1 < (unsigned)NI ? m1 : NI;
      const f2 u = (xin + nkn01) * rh01;
      const f2 sv = pfma(pfma(pfma(s0w, u, s0z), u, s0y), u, s0x);
      acc += c == m0 ? sv.x : 0.0f;
      acc += c == m1 ? sv.y : 0.0f;
    }
    STAMP(1);
    const float h = row_sum16(acc) + c0o;
    STAMP(2);
    if constexpr (TAPE)
      if (trow && act && c == 0) trow[D + rr] = h;
    // ---------------- layer 1 (input h = h_rr) ----------------
    f2 acc01;
    {
      const float pv = re1 ? (hgate ? h : 0.f) : pvh;
      const float e = ex2(ffma(hna, h - pv, hab));
      const float sg = rcp(1.0f + e);
      float v = ffma(sg, hsilu ? h : hmul, hadd);
      acc01 = hw * splat(v);  // weight 0 on the gate / exp lanes: MAC the finite v before it becomes e
      v = hexp ? e : v;
      if constexpr (FERRO) {
        const float gt = dppm<0x15B>(v), ee = dppm<0x15C>(v);  // row_newbcast:11 / :12
        const f2 pr = v4_pair<F_>(f2{ee, gt}, f2{h, 0.f}, ep1, k21, kE1, cp1, splat(0.0f), a.P1.gsl2e);
        acc01 = pfma(psel, splat(pr.x + pr.y), acc01);  // 1 * ps onto output o1, 0 * ps (exact) onto the other
        pvh = hgate ? h : 0.f;
        re1 = false;
      }
    }
    STAMP(3);
    {
      const uint64_t bal = __builtin_amdgcn_ballot_w64(h >= knh);
      int m = (int)__builtin_popcountll((bal >> (lane & 48)) & 0xFFFFull) - 1;
      m = (unsigned)m < (unsigned)NI ? m : NI;  // non-finite h: 0 or 16 knots -> the zero row (NaN)
      const float u = (h - knh) * rhh;
      const f2 sab = f2{cubic(cs1[0], u), cubic(cs1[1], u)};
      acc01 += c == m ? sab : splat(0.0f);
    }
    // the wave's sums of both outputs in one pass: the permlane32 swap folds rows (0, 2), (1, 3)
    // of acc0 into lanes 0-31 and of acc1 into lanes 32-63, the permlane16 swap folds the two
    // remaining rows of each half, a row sum finishes (lane 0: output 0, lane 32: output 1)
    {
      float p = acc01.x, q = acc01.y;
      permlane32_swap(p, q);
      float r = p + q, t = r;
      permlane16_swap(r, t);
      const float sv = row_sum16(r + t);
      if ((lane & 31) == 0) reinterpret_cast<float*>(&s_part[par][w])[lane >> 5] = sv;
    }
    STAMP(4);
    __syncthreads();
    const f2 p0 = s_part[par][0], p1 = s_part[par][1], p2 = s_part[par][2];
    par ^= 1;
    STAMP(5);
    return f2{((p0.x + p1.x) + p2.x) + c1o0, ((p0.y + p1.y) + p2.y) + c1o1};
  };

  auto load_steps = [&](int s0) {
    __syncthreads();
    for (int i = tid; i < SCH && s0 + i < a.n_steps; i += 192) {
      s_dt[i] = a.step_coef[4 * (s0 + i) + 0];
      s_hh[i] = a.step_coef[4 * (s0 + i) + 1];
      s_h6[i] = a.step_coef[4 * (s0 + i) + 2];
    }
    __syncthreads();
  };
  auto load_outs = [&](int j0) {
    __syncthreads();
    for (int i = tid; i < SCH; i += 192) {
      const bool in = j0 + i < a.T;
      s_ostep[i] = in ? a.out_step[j0 + i] : -1;
      s_omode[i] = in ? a.out_mode[j0 + i] : 1;
      s_oslope[i] = in ? a.out_slope[j0 + i] : 0.f;
    }
    __syncthreads();
  };
  auto out_write = [&](int j, f2 v) __attribute__((always_inline)) {
    if (tid == 0) *reinterpret_cast<f2*>(&a.solution[((int64_t)j * a.B + b) * D]) = v;
  };
  auto interp = [](int mode, f2 y0v, f2 y1v, float sl) -> f2 {
    return mode == 0 ? y0v : (mode == 1 ? y1v : y0v + splat(sl) * (y1v - y0v));
  };
  // fixed-grid training tape (v6 at small batches): evaluation ev's row (x, h) of (n_evals, B, D + H)
  auto tape_at = [&](int ev, f2 xin) __attribute__((always_inline)) {
    if constexpr (TAPE && !DOPRI) {
      trow = a.tape + ((int64_t)ev * a.B + b) * (D + H);
      if (tid == 0) *reinterpret_cast<f2*>(trow) = xin;
    }
  };
  using FT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;

  const f2 third = splat(1.0f / 3.0f);
  if constexpr (HOT) {
    int sb = 0, jb = 1, jj = 1;
    // the step's outputs from the schedule entries read at its start (os1: a second output inside
    // the same step, step_size grids: the rest from LDS)
    auto out_step = [&](int s, int os0, int os1, int om0, float osl0, f2 y, f2 y1) __attribute__((always_inline)) {
      if (os0 != s) return;
      out_write(jj, interp(om0, y, y1, osl0));
      ++jj;
      if (os1 != s) return;
      while (jj < a.T) {
        if (jj - jb == SCH) {
          jb = jj;
          load_outs(jj);
        }
        if (s_ostep[jj - jb] != s) break;
        out_write(jj, interp(s_omode[jj - jb], y, y1, s_oslope[jj - jb]));
        ++jj;
      }
    };
    load_steps(0);
    load_outs(1);
    auto run = [&](auto fact_tag) __attribute__((always_inline)) {
      for (int s = 0; s < a.n_steps; ++s) {
        if (s - sb == SCH) {
          sb = s;
          load_steps(s);
        }
        if (jj + 1 - jb >= SCH) {
          jb = jj;
          load_outs(jj);
        }
        const f2 dt = splat(s_dt[s - sb]);
        // this step's output schedule read up front (as small6): its LDS round trips overlap the
        // four evaluations instead of following them on the wave's chain
        const int jr = jj - jb;
        const int os0 = s_ostep[jr], os1 = s_ostep[jr + 1], om0 = s_omode[jr];
        const float osl0 = s_oslope[jr];
        tape_at(4 * s, y);
        const f2 k1 = eval_body(y, fact_tag);
        const f2 x2 = y + (dt * k1) * third;
        tape_at(4 * s + 1, x2);
        const f2 k2 = eval_body(x2, fact_tag);
        const f2 x3 = y + dt * (k2 - k1 * third);
        tape_at(4 * s + 2, x3);
        const f2 k3 = eval_body(x3, fact_tag);
        const f2 x4 = y + dt * ((k1 - k2) + k3);
        tape_at(4 * s + 3, x4);
        const f2 k4 = eval_body(x4, fact_tag);
        const f2 y1 = y + (((k1 + splat(3.0f) * (k2 + k3)) + k4) * dt) * splat(0.125f);
        out_step(s, os0, os1, om0, osl0, y, y1);
        y = y1;
        STAMP(7);
      }
    };
    if (fact) run(FT{});
    else run(FF{});
  } else {
    auto eval = [&](f2 xin) __attribute__((always_inline)) -> f2 {
      if (fact) return eval_body(xin, FT{});
      return eval_body(xin, FF{});
    };
    if constexpr (DOPRI) {
      // ---- device-resident dopri5 on v6 (one trajectory per workgroup; the small batches: the
      // reference's own X0 (1, 2)).  fused4's driver in f2 arithmetic (both state dims on every
      // lane, the same fp32 ops per component), one grid sum per norm issued by wave 0 ----
      const DopriParams& P = a.dp;
      const double n_el = P.n_total;
      int nfev = 0, n_att = 0, status = 0;
      unsigned round = 0;
      auto gsum2 = [&](double v0, double v1, double& s0, double& s1) {
        if (w == 0) {
          double r0 = 0.0, r1 = 0.0;
          const bool ab = grid_sum2(P, round, v0, v1, r0, r1);
          if (lane == 0) {
            s_gs[0] = r0;
            s_gs[1] = r1;
            s_gab = ab ? 1 : 0;
          }
        }
        __syncthreads();
        s0 = s_gs[0];
        s1 = s_gs[1];
        if (s_gab) status = 4;
      };
      auto tape_eval = [&](f2 xin) -> f2 {  // the evaluation, and its tape row (x, h, k) in training
        if constexpr (TAPE) trow = nfev < P.tape_cap ? a.tape + ((int64_t)nfev * a.B + b) * (2 * D + H) : nullptr;
        const f2 k = eval(xin);
        if constexpr (TAPE) {
          if (trow && tid == 0) {
            *reinterpret_cast<f2*>(trow) = xin;
            *reinterpret_cast<f2*>(trow + D + H) = k;
          }
        }
        ++nfev;
        return k;
      };
      auto sq = [](f2 q) { return (double)q.x * q.x + (double)q.y * q.y; };
      f2 f0 = tape_eval(y);
      double dt;
      if (P.first_step > 0.0) {
        dt = P.first_step;
      } else {  // misc._select_initial_step in fp32
        const f2 scale = splat(P.atol) + splat(P.rtol) * f2{fabsf(y.x), fabsf(y.y)};
        const f2 q0 = y / scale, q1 = f0 / scale;
        double s, s1;
        gsum2(sq(q0), sq(q1), s, s1);
        const float d0 = fabsf(sqrtf((float)(s / n_el)));
        const float d1 = fabsf(sqrtf((float)(s1 / n_el)));
        float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
        h0 = fabsf(h0);
        const f2 f1 = tape_eval(y + f0 * splat(h0));
        const f2 q2 = (f1 - f0) / scale;
        gsum2(sq(q2), 0.0, s, s1);
        const float d2 = fabsf(sqrtf((float)(s / n_el)) / h0);
        float h1;
        if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
        else h1 = (float)pow((double)(0.01f / fmaxf(d1, d2)), (double)0.2f);
        dt = (double)fminf(100.0f * h0, fabsf(h1));
        if (TAPE && blockIdx.x == 0 && tid == 0) {
          P.init_rec[0] = d0;
          P.init_rec[1] = d1;
          P.init_rec[2] = d2;
          P.init_rec[3] = h0;
          P.init_rec[4] = h1;
        }
      }
      f2 co[5] = {y, splat(0.f), splat(0.f), splat(0.f), splat(0.f)};
      double t0s = P.t[0], t1s = P.t[0];
      for (int i = 1; i < P.T && status == 0; ++i) {
        const double next_t = P.t[i];
        int n_steps = 0;
        while (next_t > t1s) {
          if (n_steps >= P.max_steps) { status = 3; break; }
          const double t0 = t1s;
          if (!(t0 + dt > t0)) { status = 2; break; }
          const float dt32 = (float)dt;
          const double t1 = t0 + dt;
          f2 A[6];
#pragma unroll
          for (int q = 0; q < 6; ++q) A[q] = f0 * splat(P.stc[0][q] * dt32);
          f2 err = f0 * splat(P.stc[0][6] * dt32);
          f2 mid = f0 * splat(P.stc[0][7] * dt32);
          f2 yi = y, kn = f0;
#pragma unroll 1
          for (int st = 0; st < 6; ++st) {
            yi = y + A[0];
            float c[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) c[q] = P.stc[st + 1][q];
            kn = tape_eval(yi);
#pragma unroll
            for (int q = 0; q < 5; ++q) A[q] = A[q + 1] + kn * splat(c[q] * dt32);
            err = err + kn * splat(c[6] * dt32);
            mid = mid + kn * splat(c[7] * dt32);
          }
          const f2 y1 = yi;
          const f2 tol = splat(P.atol) + splat(P.rtol) * f2{fmaxf(fabsf(y.x), fabsf(y1.x)), fmaxf(fabsf(y.y), fabsf(y1.y))};
          const f2 qe = err / tol;
          double s, nbad;
          gsum2(sq(qe), (__builtin_isfinite(y.x) && __builtin_isfinite(y.y)) ? 0.0 : 1.0, s, nbad);
          if (status) break;
          if (nbad != 0.0) { status = 1; break; }
          const float ratio = sqrtf((float)(s / n_el));
          const bool accept = ratio <= 1.0f;
          if (blockIdx.x == 0 && tid == 0 && n_att < P.max_att) {
            double* o = P.att + (int64_t)n_att * 4;
            o[0] = t0;
            o[1] = dt;
            o[2] = (double)ratio;
            o[3] = accept ? 1.0 : 0.0;
          }
          ++n_att;
          if (accept) {  // interp._interp_fit (fused4's op order)
            const f2 ym = y + mid, fa = f0, fb6 = kn, dtv = splat(dt32);
            co[4] = ((splat(2.0f * dt32)) * (fb6 - fa) - splat(8.0f) * (y1 + y)) + splat(16.0f) * ym;
            co[3] = ((dtv * (splat(5.0f) * fa - splat(3.0f) * fb6) + splat(18.0f) * y) + splat(14.0f) * y1) - splat(32.0f) * ym;
            co[2] = ((dtv * (fb6 - splat(4.0f) * fa) - splat(11.0f) * y) - splat(5.0f) * y1) + splat(16.0f) * ym;
            co[1] = dtv * fa;
            co[0] = y;
            y = y1;
            f0 = kn;
            t0s = t0;
            t1s = t1;
          } else {
            t0s = t0;
          }
          const double rr_ = (double)ratio;
          double nxt;
          if (rr_ == 0.0) {
            nxt = dt * P.ifactor;
          } else {
            const double dfac = rr_ < 1.0 ? 1.0 : P.dfactor;
            const double factor = __builtin_isnan(rr_) ? rr_ : fmin(P.ifactor, fmax(P.safety / pow(rr_, 1.0 / 5.0), dfac));
            nxt = dt * factor;
          }
          dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, P.min_step), P.max_step);
          ++n_steps;
        }
        if (status) break;
        const float xq = (float)((next_t - t0s) / (t1s - t0s));
        f2 total = co[0] + splat(xq) * co[1];
        float xp = xq;
#pragma unroll
        for (int j = 2; j < 5; ++j) {
          xp = xp * xq;
          total = total + splat(xp) * co[j];
        }
        out_write(i, total);
      }
      if (blockIdx.x == 0 && tid == 0) {
        P.stats[0] = nfev;
        P.stats[1] = n_att;
        P.stats[2] = __hip_atomic_load(P.bar + kDpLine * (kDpGroups + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 4 : status;
      }
    } else if (a.single_eval) {

      const f2 f = eval(y);
      if (tid == 0) *reinterpret_cast<f2*>(&a.eval_out[b * D]) = f;
    } else {
      const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
      int sb = 0, jb = 1, jj = 1;
      load_steps(0);
      load_outs(1);
      for (int s = 0; s < a.n_steps; ++s) {
        if (s - sb == SCH) {
          sb = s;
          load_steps(s);
        }
        const f2 dt = splat(s_dt[s - sb]), hh = splat(s_hh[s - sb]), h6 = splat(s_h6[s - sb]);
        f2 k1 = splat(0.f), k2 = splat(0.f), k3 = splat(0.f), k4 = splat(0.f);
        for (int st = 0; st < ns; ++st) {
          f2 xin = y;
          if (a.method == FETODE_RK4) {
            if (st == 1) xin = y + (dt * k1) * third;
            else if (st == 2) xin = y + dt * (k2 - k1 * third);
            else if (st == 3) xin = y + dt * ((k1 - k2) + k3);
          } else if (a.method == FETODE_RK4_CLASSIC) {
            if (st == 1) xin = y + hh * k1;
            else if (st == 2) xin = y + hh * k2;
            else if (st == 3) xin = y + dt * k3;
          } else if (a.method == FETODE_MIDPOINT) {
            if (st == 1) xin = y + k1 * hh;
          }
          tape_at(s * ns + st, xin);
          const f2 kk = eval(xin);
          if (st == 0) k1 = kk;
          else if (st == 1) k2 = kk;
          else if (st == 2) k3 = kk;
          else k4 = kk;
        }
        f2 y1;
        if (a.method == FETODE_RK4) y1 = y + (((k1 + splat(3.0f) * (k2 + k3)) + k4) * dt) * splat(0.125f);
        else if (a.method == FETODE_RK4_CLASSIC) y1 = y + h6 * (((k1 + splat(2.0f) * k2) + splat(2.0f) * k3) + k4);
        else if (a.method == FETODE_MIDPOINT) y1 = y + dt * k2;
        else y1 = y + dt * k1;
        while (jj < a.T) {
          if (jj - jb == SCH) {
            jb = jj;
            load_outs(jj);
          }
          if (s_ostep[jj - jb] != s) break;
          out_write(jj, interp(s_omode[jj - jb], y, y1, s_oslope[jj - jb]));
          ++jj;
        }
        y = y1;
      }
    }
  }
  STAMP_FLUSH();
  if (FERRO && (DOPRI || a.single_eval || a.n_steps > 0)) {  // no evaluation: the state stays as it was
    if (r == 1 && ogate) a.state[b * D + ofx] = pvs;
    if (act && hgate) a.state[a.B * D + b * H + rr] = pvh;
  }
}

// =============================================================================================
// v8: one trajectory per TWO-wave workgroup — the strong-scaling shard kernel (rk4 inference).
//
// At B = 512 (the 8-way shard of the 4096 batch) v7 at one trajectory per wave leaves half the
// SIMDs idle and each wave walks the whole evaluation (~1 500 cycles: ~170 VALU + 33
// transcendentals issued by one wave, plus ~40 % of its cycles waiting on LDS round trips,
// profiles/r06_shard_pmc.txt).  v8 gives each trajectory two waves (B = 512 -> 1 024 waves, one
// per SIMD) and keeps LDS off the evaluation's chain except for ONE exchange of two partial sums:
//   * wave w owns hidden units o = 5w .. 5w+4; unit u of the wave is 12 lanes, 3 in each of the
//     4 rows (lanes 16r + 3u + j), lane index c = 3r + j in the unit;
//   * layer 0: every lane knows x (both state dims, f2); lane c < 10 takes Ferro pair c of output o
//     (input c / 5, elements 2(c % 5), +1) and forms its input's gate and exp(gs x) itself; lane c
//     forms feature slots 2c, 2c+1 of the 24 (input c / 6: SiLU, 10 logistic, pad) and applies
//     their weights; lane c holds knot interval c's spline cubics of edges (o, 0), (o, 1)
//     (c = NI: the zero row) and the lane that owns x_i's interval adds edge (o, i) — interval
//     from one wave ballot against the knots held one per unit lane; a group-of-3 DPP sum and two
//     lane folds (permlane32 / permlane16 swaps) leave h_o on the unit's 12 lanes;
//   * layer 1 (input h_o): lane c < 10 takes the element pair (o, d = 0 / 1, k = c), lane c < 11
//     feature job c (logistic c, SiLU at c = NB) weighted for both outputs, the lane owning h_o's
//     interval the two spline edges (o -> 0, 1), each lane the gate / exp(gs h_o) itself;
//   * the wave's partial sums of both outputs (permlane32 swap, permlane16 fold, row sum) meet the
//     other wave's through LDS and ONE workgroup barrier (double-buffered by evaluation parity);
//     every lane of both waves forms k = (S_w0 + S_w1) + c in the same order, so both waves carry
//     bitwise the same state and the stage combines run redundantly on every lane (torchdiffeq's
//     op order, rk_common.rk4_alt_step_func).
// Each butterfly / swap sum gives bitwise the same value on every lane it leaves it on (a + b and
// b + a round alike), so no lane's copy of h_o or k drifts from another's.
// =============================================================================================
// TPB trajectories per workgroup (two waves each): TPB = 2 makes the workgroup four waves, which the
// dispatcher spreads over a CU's four SIMDs — one wave per SIMD at B = 512 (with two-wave workgroups
// two of them may share a SIMD pair).
template <bool FERRO, int TPB>
__global__ __launch_bounds__(128 * TPB) void v8_kernel(FusedArgs a) {
  constexpr int D = 2, H = 10, K = FERRO ? 10 : 0, KP = 5, NB = 10, NG = 12, NI = NG - 1, NFL = 1 + NB;
  constexpr int NFP = NFL + 1;  // feature slots per input: SiLU, NB logistic, pad
  static_assert(D * NFP == 2 * 12 && NG == 12, "v8: 12 lanes per unit = 12 knots = 24 feature slots / 2");
  __shared__ __attribute__((aligned(16))) float s_part[TPB][2][2][2];   // [traj][parity][wave][output]
  constexpr int SCH = 32;
  __shared__ float s_dt[SCH], s_oslope[SCH];
  __shared__ int s_ostep[SCH], s_omode[SCH];

  const int tid = threadIdx.x, tj = tid >> 7, w = (tid >> 6) & 1, lane = tid & 63, r = lane >> 4, q = lane & 15;
  const bool act = q < 15;
  const int u = act ? q / 3 : 0, c = 3 * r + (q % 3);   // unit in the wave, lane index in the unit
  const int o = 5 * w + u;                              // hidden unit (layer-0 output, layer-1 input)
  const int64_t b0 = (int64_t)blockIdx.x * TPB + tj;
  const bool valid = b0 < a.B;          // an idle trajectory slot still takes part in the barriers
  const int64_t b = valid ? b0 : 0;
  const bool lead = valid && (tid & 127) == 0;
  const float l2 = FETODE_LOG2E;
  const bool fact = FERRO && a.plan[a.P0.flag] <= a.factor_limit && a.plan[a.P1.flag] <= a.factor_limit;
  // the unit's 12 lanes (3 per row) as a ballot mask; layer 0's knots are the same on every unit:
  // unit 0's lanes give its count as a uniform
  const uint64_t umask = (0x0007000700070007ull << (3 * u));
  constexpr uint64_t kMask0 = 0x0007000700070007ull;

  // ---- layer 0, unit lane c: Ferro pair c (input ip, elements 2 kp, 2 kp + 1) ----
  const bool pj = FERRO && act && c < 2 * KP;
  const int ip = c >= KP ? 1 : 0;
  f2 ep0 = splat(0.f), k20 = splat(0.f), kE0 = splat(0.f), cp0 = splat(0.f);
  f2 ep1 = splat(0.f), k21 = splat(0.f), kE1 = splat(0.f), cp1 = splat(0.f);
  if constexpr (FERRO) {
    float t0[4][2], t1[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t i0x = (int64_t)o * (D * K) + ip * K + (pj ? (c % KP) * 2 + h : 0);
      const float g0 = pj ? a.plan[a.P0.fe_GEc + i0x] : 0.f;
      t0[0][h] = fact ? ex2(g0) : g0;
      t0[1][h] = pj ? a.plan[a.P0.fe_k2 + i0x] : 0.f;
      t0[2][h] = pj ? a.plan[a.P0.fe_k2Ec + i0x] : 0.f;
      t0[3][h] = pj ? a.plan[a.P0.fe_CPs2 + i0x] : 0.f;
      // layer 1: element (o, d = h, k = c)
      const int64_t i1x = (int64_t)h * (H * K) + o * K + (pj ? c : 0);
      const float g1 = pj ? a.plan[a.P1.fe_GEc + i1x] : 0.f;
      t1[0][h] = fact ? ex2(g1) : g1;
      t1[1][h] = pj ? a.plan[a.P1.fe_k2 + i1x] : 0.f;
      t1[2][h] = pj ? a.plan[a.P1.fe_k2Ec + i1x] : 0.f;
      t1[3][h] = pj ? a.plan[a.P1.fe_CPs2 + i1x] : 0.f;
    }
    ep0 = f2{t0[0][0], t0[0][1]}; k20 = f2{t0[1][0], t0[1][1]}; kE0 = f2{t0[2][0], t0[2][1]}; cp0 = f2{t0[3][0], t0[3][1]};
    ep1 = f2{t1[0][0], t1[0][1]}; k21 = f2{t1[1][0], t1[1][1]}; kE1 = f2{t1[2][0], t1[2][1]}; cp1 = f2{t1[3][0], t1[3][1]};
  }
  // ---- layer 0 feature slots 2c, 2c+1 of input fi = c / 6 (slot f: 0 SiLU, 1..NB logistic f-1, pad) ----
  const int fi = c >= 6 ? 1 : 0;
  float fna[2], fab[2], fml[2], fwv[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int f = (2 * c + s) % NFP;
    fna[s] = 0.f; fab[s] = 0.f; fml[s] = 0.f; fwv[s] = 0.f;
    if (act && f == 0) {
      fna[s] = -l2;
      fml[s] = 1.f;
      fwv[s] = a.plan[a.P0.kw + (int64_t)o * (D * NFL) + fi * NFL];
    } else if (act && f <= NB) {
      fna[s] = a.plan[a.P0.lg + 2 * (fi * NB + f - 1)];
      fab[s] = a.plan[a.P0.lg + 2 * (fi * NB + f - 1) + 1];
      fwv[s] = a.plan[a.P0.kw + (int64_t)o * (D * NFL) + fi * NFL + f];
    }
  }
  const f2 fw0 = f2{fwv[0], fwv[1]};
  // ---- layer 0 splines: knot c of both inputs (the interval count), interval c's (knot, 1/width)
  //      and cubics of edges (o, 0), (o, 1) (c = NI: the zero row: u = 0 for finite x, NaN otherwise)
  const float kn0 = act ? a.plan[a.P0.knots + c] : __builtin_inff();
  const float kn1 = act ? a.plan[a.P0.knots + NG + c] : __builtin_inff();
  const bool ci = act && c < NI;
  const f2 nukn0 = f2{ci ? -a.plan[a.P0.knots + c] : 0.f, ci ? -a.plan[a.P0.knots + NG + c] : 0.f};
  const f2 urh0 = f2{ci ? a.plan[a.P0.rh + c] : 0.f, ci ? a.plan[a.P0.rh + NI + c] : 0.f};
  float4 cs0[D], cs1[D];
  {
    const float4* sp0 = reinterpret_cast<const float4*>(a.plan + a.P0.sp);
    const float4* sp1 = reinterpret_cast<const float4*>(a.plan + a.P1.sp);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      cs0[i] = act ? sp0[(o * D + i) * (NI + 1) + c] : make_float4(0.f, 0.f, 0.f, 0.f);
      cs1[i] = act ? sp1[(i * H + o) * (NI + 1) + c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const f2 s0x = f2{cs0[0].x, cs0[1].x}, s0y = f2{cs0[0].y, cs0[1].y};
  const f2 s0z = f2{cs0[0].z, cs0[1].z}, s0w = f2{cs0[0].w, cs0[1].w};
  const f2 s1x = f2{cs1[0].x, cs1[1].x}, s1y = f2{cs1[0].y, cs1[1].y};
  const f2 s1z = f2{cs1[0].z, cs1[1].z}, s1w = f2{cs1[0].w, cs1[1].w};
  const float c0o = act ? a.plan[a.P0.fconst + o] : 0.f;
  // ---- layer 1 (input h_o): feature job c (logistic c < NB, SiLU at NB), weights for both outputs
  float hna = 0.f, hab = 0.f, hml = 0.f;
  f2 hw = splat(0.f);
  if (act && c < NB) {
    hna = a.plan[a.P1.lg + 2 * (o * NB + c)];
    hab = a.plan[a.P1.lg + 2 * (o * NB + c) + 1];
    hw = f2{a.plan[a.P1.kw + (int64_t)0 * (H * NFL) + o * NFL + 1 + c], a.plan[a.P1.kw + (int64_t)1 * (H * NFL) + o * NFL + 1 + c]};
  } else if (act && c == NB) {
    hna = -l2;
    hml = 1.f;
    hw = f2{a.plan[a.P1.kw + (int64_t)0 * (H * NFL) + o * NFL], a.plan[a.P1.kw + (int64_t)1 * (H * NFL) + o * NFL]};
  }
  const float knh = act ? a.plan[a.P1.knots + o * NG + c] : __builtin_inff();
  const float nukh = ci ? -a.plan[a.P1.knots + o * NG + c] : 0.f;
  const float urhh = ci ? a.plan[a.P1.rh + o * NI + c] : 0.f;
  const float c1o0 = a.plan[a.P1.fconst + 0], c1o1 = a.plan[a.P1.fconst + 1];

  // hysteresis state (ferro_class.py:409): both layer-0 inputs on every lane, unit o's on its lanes
  // the first evaluation is always at y0, so a fresh layer-0 state starts from y0 directly; layer 1's
  // first input is only known inside it (re1)
  bool re1 = FERRO && (a.init_mask & 2u);
  f2 y = f2{a.y0[b * D + 0], a.y0[b * D + 1]};
  f2 prev0 = splat(0.f);
  float prev1 = 0.f;
  if (FERRO) {
    prev0 = (a.init_mask & 1u) ? y : f2{a.state[b * D + 0], a.state[b * D + 1]};
    if (act) prev1 = a.state[a.B * D + b * H + o];
  }
  if (!a.single_eval && lead) *reinterpret_cast<f2*>(&a.solution[b * D]) = y;
  int par = 0;
  auto cubic2 = [](f2 x, f2 y_, f2 z, f2 w_, f2 uu) { return pfma(pfma(pfma(w_, uu, z), uu, y_), uu, x); };
  auto interval = [](uint64_t bal, int cnt_extra, bool fin) {
    constexpr int NI = NG - 1;
    const int m = (int)__builtin_popcountll(bal) - 1 + cnt_extra;
    return ((unsigned)m < (unsigned)NI && fin) ? m : NI;
  };
  STAMP_DECL

  auto eval_body = [&](f2 xin, auto fact_tag) __attribute__((always_inline)) -> f2 {
    constexpr bool F_ = decltype(fact_tag)::value;
    STAMP(6);
    // ---------------- layer 0 -> h_o on the unit's 12 lanes ----------------
    float acc;
    {
      const float xf = fi ? xin.y : xin.x;   // this lane's feature input
      float val[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float e = ex2(ffma(fna[s], xf, fab[s]));
        const float sg = rcp(1.0f + e);
        val[s] = fml[s] != 0.0f ? xf * sg : sg;
      }
      f2 pr = splat(0.0f);
      if constexpr (FERRO) {
        const float xg = ip ? xin.y : xin.x;
        const float pv = ip ? prev0.y : prev0.x;
        const float eg = ex2(ffma(-a.P0.gsl2e, xg - pv, 0.0f));
        const float wg = ffma(rcp(1.0f + eg), -a.P0.wc, a.P0.wc);          // wc (1 - up)
        const float e = F_ ? ex2(ffma(a.P0.gsl2e, xg, 0.0f)) : 0.0f;
        pr = v4_pair<F_>(f2{e, wg}, f2{xg, 0.0f}, ep0, k20, kE0, cp0, splat(0.0f), a.P0.gsl2e);
        prev0 = xin;   // ferro_class.py:409
      }
      STAMP(0);
      pr = pfma(fw0, f2{val[0], val[1]}, pr);
      // the two spline edges (o, 0), (o, 1): the lane owning x_i's knot interval
      const int m0 = interval(__builtin_amdgcn_ballot_w64(xin.x >= kn0) & kMask0, 0, __builtin_isfinite(xin.x));
      const int m1 = interval(__builtin_amdgcn_ballot_w64(xin.y >= kn1) & kMask0, 0, __builtin_isfinite(xin.y));
      const f2 uu = (xin + nukn0) * urh0;
      const f2 sv = cubic2(s0x, s0y, s0z, s0w, uu);
      acc = (pr.x + pr.y) + ((c == m0 ? sv.x : 0.0f) + (c == m1 ? sv.y : 0.0f));
    }
    STAMP(1);
    // unit sum: group of 3 in the row, then rows (0, 2), (1, 3) and (0, 1)
    float hs = group3_sum(acc, q % 3);
    {
      float p = hs, t = hs;
      permlane32_swap(p, t);
      hs = p + t;
      float p2 = hs, t2 = hs;
      permlane16_swap(p2, t2);
      hs = p2 + t2;
    }
    const float h = hs + c0o;
    STAMP(2);
    // ---------------- layer 1 (input h = h_o) ----------------
    f2 acc01;
    {
      const int m = interval(__builtin_amdgcn_ballot_w64(h >= knh) & umask, 0, __builtin_isfinite(h));
      const float e = ex2(ffma(hna, h, hab));
      const float sg = rcp(1.0f + e);
      const float v = hml != 0.0f ? h * sg : sg;
      acc01 = splat(0.0f);
      if constexpr (FERRO) {
        const float pv = re1 ? h : prev1;
        const float eg = ex2(ffma(-a.P1.gsl2e, h - pv, 0.0f));
        const float wg = ffma(rcp(1.0f + eg), -a.P1.wc, a.P1.wc);
        const float eh = F_ ? ex2(ffma(a.P1.gsl2e, h, 0.0f)) : 0.0f;
        acc01 = v4_pair<F_>(f2{eh, wg}, f2{h, 0.0f}, ep1, k21, kE1, cp1, splat(0.0f), a.P1.gsl2e);
        prev1 = h;   // ferro_class.py:409
        re1 = false;
      }
      acc01 = pfma(hw, splat(v), acc01);
      const float uh = (h + nukh) * urhh;
      const f2 sab = cubic2(s1x, s1y, s1z, s1w, splat(uh));
      acc01 += c == m ? sab : splat(0.0f);
    }
    STAMP(3);
    // the wave's sums of both outputs: lanes 0-31 output 0, lanes 32-63 output 1
    float sw;
    {
      float p = acc01.x, t = acc01.y;
      permlane32_swap(p, t);
      float s = p + t, s2 = s;
      permlane16_swap(s, s2);
      sw = row_sum16(s + s2);
    }
    STAMP(4);
    if ((lane & 31) == 0) s_part[tj][par][w][lane >> 5] = sw;
    __syncthreads();
    const float4 pp = *reinterpret_cast<const float4*>(&s_part[tj][par][0][0]);
    par ^= 1;
    STAMP(5);
    return f2{(pp.x + pp.z) + c1o0, (pp.y + pp.w) + c1o1};
  };

  auto load_steps = [&](int s0) {
    __syncthreads();
    for (int i = tid; i < SCH && s0 + i < a.n_steps; i += 128 * TPB) s_dt[i] = a.step_coef[4 * (s0 + i) + 0];
    __syncthreads();
  };
  auto load_outs = [&](int j0) {
    __syncthreads();
    for (int i = tid; i < SCH; i += 128 * TPB) {
      const bool in = j0 + i < a.T;
      s_ostep[i] = in ? a.out_step[j0 + i] : -1;
      s_omode[i] = in ? a.out_mode[j0 + i] : 1;
      s_oslope[i] = in ? a.out_slope[j0 + i] : 0.f;
    }
    __syncthreads();
  };
  auto out_write = [&](int j, f2 v) __attribute__((always_inline)) {
    if (lead) *reinterpret_cast<f2*>(&a.solution[((int64_t)j * a.B + b) * D]) = v;
  };
  auto interp = [](int mode, f2 y0v, f2 y1v, float sl) -> f2 {
    return mode == 0 ? y0v : (mode == 1 ? y1v : y0v + splat(sl) * (y1v - y0v));
  };
  using FT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;
  const f2 third = splat(1.0f / 3.0f);
  int sb = 0, jb = 1, jj = 1;
  load_steps(0);
  load_outs(1);
  auto run = [&](auto fact_tag) __attribute__((always_inline)) {
    for (int s = 0; s < a.n_steps; ++s) {
      if (s - sb == SCH) {
        sb = s;
        load_steps(s);
      }
      if (jj + 1 - jb >= SCH) {
        jb = jj;
        load_outs(jj);
      }
      const f2 dt = splat(s_dt[s - sb]);
      // the step's output schedule read up front (as small6 / fused4): off the evaluation chain
      const int jr = jj - jb;
      const int os0 = s_ostep[jr], os1 = s_ostep[jr + 1], om0 = s_omode[jr];
      const float osl0 = s_oslope[jr];
      const f2 k1 = eval_body(y, fact_tag);
      const f2 k2 = eval_body(y + (dt * k1) * third, fact_tag);
      const f2 k3 = eval_body(y + dt * (k2 - k1 * third), fact_tag);
      const f2 k4 = eval_body(y + dt * ((k1 - k2) + k3), fact_tag);
      const f2 y1 = y + (((k1 + splat(3.0f) * (k2 + k3)) + k4) * dt) * splat(0.125f);
      if (os0 == s) {
        out_write(jj, interp(om0, y, y1, osl0));
        ++jj;
        if (os1 == s) {  // several outputs inside one step (step_size grids)
          while (jj < a.T) {
            if (jj - jb == SCH) {
              jb = jj;
              load_outs(jj);
            }
            if (s_ostep[jj - jb] != s) break;
            out_write(jj, interp(s_omode[jj - jb], y, y1, s_oslope[jj - jb]));
            ++jj;
          }
        }
      }
      y = y1;
      STAMP(7);
    }
  };
  if (fact) run(FT{});
  else run(FF{});
  STAMP_FLUSH();
  if (FERRO && valid && a.n_steps > 0) {  // no evaluation: the state stays as it was
    if (lead) *reinterpret_cast<f2*>(&a.state[b * D]) = prev0;
    if (act && c == 0) a.state[a.B * D + b * H + o] = prev1;   // each wave its own units
  }
}


typedef void (*fused_fn)(FusedArgs);
struct FusedEntry {
  int in0, h, out, K, NB, NG;
  bool ferro;
  fused_fn fn;        // v4: single evaluations and every fixed-grid method
  fused_fn fn_rk4;    // v4: the rk4 (3/8) integrate path, all four stages inlined
  fused_fn small;     // v6 (one trajectory per workgroup): generic
  fused_fn small_rk4; // v6: rk4
  fused_fn dopri;     // v4 with the device-resident dopri5 driver
  fused_fn dopri_tape;  // the same, recording the training tape
  fused_fn small_dopri, small_dopri_tape;  // v6 with the dopri5 driver (small batches)
  fused_fn small_tape, small_rk4_tape;     // v6 recording the fixed-grid training tape
  fused_fn fn_rk4_1;  // v7 rk4 at one trajectory per wave (inference, mid batches)
  fused_fn rk4_v8;    // v8 rk4 at two waves per trajectory (inference, the strong-scaling shards)
  fused_fn rk4_v8x2;  // the same, two trajectories per four-wave workgroup
  fused_fn fn_tape, fn_rk4_tape, fn_rk4_1_tape;  // v4 / v7 recording the fixed-grid training tape
};
const FusedEntry kFused[] = {
    // LV KAN-FET [2,10,2], K=10 (train_kanfet_node_predprey.py:146)
    {2, 10, 2, 10, 10, 12, true, fused4_kernel<10, 10, 10, 12, true, false>, fused4_kernel<10, 10, 10, 12, true, true>,
     small6_kernel<true, false>, small6_kernel<true, true>, fused4_kernel<10, 10, 10, 12, true, false, true>,
     fused4_kernel<10, 10, 10, 12, true, false, true, true>, small6_kernel<true, false, true, false>,
     small6_kernel<true, false, true, true>, small6_kernel<true, false, false, true>,
     small6_kernel<true, true, false, true>, fused4_kernel<10, 10, 10, 12, true, true, false, false, 1>,
     v8_kernel<true, 1>, v8_kernel<true, 2>, fused4_kernel<10, 10, 10, 12, true, false, false, true>,
     fused4_kernel<10, 10, 10, 12, true, true, false, true>, fused4_kernel<10, 10, 10, 12, true, true, false, true, 1>},
    // LV KAN [2,10,2] (predator_prey.py:101)
    {2, 10, 2, 1, 10, 12, false, fused4_kernel<10, 2, 10, 12, false, false>, fused4_kernel<10, 2, 10, 12, false, true>,
     small6_kernel<false, false>, small6_kernel<false, true>, fused4_kernel<10, 2, 10, 12, false, false, true>,
     fused4_kernel<10, 2, 10, 12, false, false, true, true>, small6_kernel<false, false, true, false>,
     small6_kernel<false, false, true, true>, small6_kernel<false, false, false, true>,
     small6_kernel<false, true, false, true>, fused4_kernel<10, 2, 10, 12, false, true, false, false, 1>,
     v8_kernel<false, 1>, v8_kernel<false, 2>, fused4_kernel<10, 2, 10, 12, false, false, false, true>,
     fused4_kernel<10, 2, 10, 12, false, true, false, true>, fused4_kernel<10, 2, 10, 12, false, true, false, true, 1>},
};

// Batches up to kSmallMax take v6 (one trajectory per 3-wave workgroup, latency-bound chain split
// over 160 lanes), larger ones v4 (two trajectories per wave, issue-bound); training tapes are v4
// only.  FETODE_SMALL_MAX overrides the switch point (diagnostics / tuning).
int64_t g_small_max = [] {
  const char* e = getenv("FETODE_SMALL_MAX");
  return e ? (int64_t)atoll(e) : (int64_t)512;  // measured switch point (tools/diag/batch_sweep.py)
}();
int64_t small_max() { return g_small_max; }
// Inference rk4 batches in (g_tpw1_lo, g_tpw1_hi] take v7 at one trajectory per wave (before the
// v6 / v4 choice; env FETODE_TPW1_LO / FETODE_TPW1_HI).  Measured (tools/diag/batch_sweep.py,
// profiles/r05_t1w_sweep*.log, us per 34-step solve, v6 / one / two per wave): B = 256 77 / 93 / 114,
// 384 98 / 97 / 114,
// 512 101 / 97 / 113, 768 129 / 97 / 119, 1024 146 / 99 / 119, 1536 202 / 133 / 117.
int64_t g_tpw1_lo = [] {
  const char* e = getenv("FETODE_TPW1_LO");
  return e ? (int64_t)atoll(e) : (int64_t)320;
}();
int64_t g_tpw1_hi = [] {
  const char* e = getenv("FETODE_TPW1_HI");
  return e ? (int64_t)atoll(e) : (int64_t)1024;
}();
// Inference rk4 batches in (g_v8_lo, g_v8_hi] take v8 (two waves per trajectory), before every other
// choice (env FETODE_V8_LO / FETODE_V8_HI).
// Measured (tools/diag/batch_sweep.py, profiles/r06_v8_sweep.log, us per 34-step solve, v6 / v7 one
// per wave / v8 at two trajectories per four-wave workgroup): B = 256 77 / 93 / 84, 320 94 / 92 / 84,
// 448 96 / 93 / 84, 512 97 / 93 / 85, 576 124 / 93 / 112 (v8 past one wave per SIMD), 1024 140 / 98 / 112.
int64_t g_v8_lo = [] {
  const char* e = getenv("FETODE_V8_LO");
  return e ? (int64_t)atoll(e) : (int64_t)256;
}();
int64_t g_v8_hi = [] {
  const char* e = getenv("FETODE_V8_HI");
  return e ? (int64_t)atoll(e) : (int64_t)512;
}();
int g_v8_tpb = [] {   // trajectories per v8 workgroup (1: two waves, 2: four waves); env FETODE_V8_TPB
  const char* e = getenv("FETODE_V8_TPB");
  return e ? atoi(e) : 2;
}();
uint32_t g_dp_spin_limit = 0;   // fetode_dopri5_set_spin_limit (0: the built-in limits)

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
    if (f->ferro) {
      if (f->ferro[0].num_basis != e.K || f->ferro[1].num_basis != e.K) continue;
      if (f->ferro[0].branch_sign || f->ferro[1].branch_sign) continue;  // general sign: generic path
    }
    return &e;
  }
  return nullptr;
}

// =============================================================================================
// fieldn: the single-launch integrator for depth-2 fields of OTHER widths — [D, H, D] with
// D <= 8, H <= 64 (KAN or KAN-FET, any K / NB, cubic splines): one trajectory per wave, lane o =
// hidden unit o.  Per evaluation, lane o forms h_o from the D layer inputs (their features are
// recomputed on every lane: D is small) and then its own input's features and contributions to
// all D outputs; a butterfly sum over the lanes gives k.  The arithmetic is the fused kernels'
// (the same plan and element formulas), the sums run in another order.  Training: the
// launch records both layers' inputs of every evaluation (two tape planes); the reverse sweep is
// fieldn_adj_kernel + the per-module parameter VJPs over every (evaluation, trajectory) row
// (fetode_fieldn_bwd.hip).  The resident dopri5 exists for the specialised [2, 10, 2] shapes only.
// =============================================================================================
constexpr int kFnMaxD = 8, kFnMaxH = 64;
constexpr int kFnWaves = 4;
// one wave's LDS traffic lands in issue order: a compiler barrier + a wait replaces the workgroup barrier
__device__ __forceinline__ void fn_wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float fn_sig_l2(float zl) { return rcp(1.0f + ex2(zl)); }  // 1/(1+2^zl)

// KAN edge (o, i) + the Ferro elements (o, i, k) of one layer at input x (gate weight w); IMG: the
// plan is read in its lane-contiguous LDS image (fetode_fieldn_plan.h), layer L
template <bool FERRO, int UNR, bool IMG, int L>
__device__ __forceinline__ float fn_edge(const float* __restrict__ plan, const LayerPlan& P, int o, int i, float x,
                                         float sx, float w, int mfix, float u) {
  using X = FnIdx<IMG, L>;
  const int st = X::stride(P);
  const float* kw = plan + X::row(P, P.kw, o, i, P.NFL);
  float v = kw[0] * sx;
  // UNR: the packed fixed-grid launch runs ~one wave per SIMD, so the independent exp2 / rcp chains
  // of consecutive basis functions must overlap within the lane (the sums stay in order); the
  // resident dopri5 keeps its register budget (occupancy = the batch one grid holds)
#pragma unroll UNR
  for (int j = 0; j < P.NB; ++j)
    v = ffma(kw[(1 + j) * st], fn_sig_l2(ffma(plan[X::lg(P, i, j, 0)], x, plan[X::lg(P, i, j, 1)])), v);
  const float4 cf = *reinterpret_cast<const float4*>(plan + X::sp(P, o, i, mfix));
  v += ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x);
  if constexpr (FERRO) {
    const int64_t e0 = X::row(P, 0, o, i, P.K);
    const float* GEc = plan + P.fe_GEc + e0;
    const float* k2 = plan + P.fe_k2 + e0;
    const float* kE = plan + P.fe_k2Ec + e0;
    const float* cp = plan + P.fe_CPs2 + e0;
#pragma unroll UNR
    for (int k = 0; k < P.K; ++k) {
      const float s = rcp(ex2(ffma(P.gsl2e, x, GEc[k * st])) + 1.0f);  // sigma(gs(-x - Ec)), one rounding as v4
      const float m = ffma(w, s, 1.0f);                    // branch momentum (branch_sign = 1)
      const float z = ffma(kE[k * st], m, k2[k * st] * x);
      const float th = ffma(rcp(ex2(z) + 1.0f), -2.0f, 1.0f);
      v = ffma(cp[k * st], th, v);
    }
  }
  return v;
}

// knot interval of x on input i's grid (m = NI: off the grid, the zero row) and its coordinate u
template <bool IMG, int L>
__device__ __forceinline__ void fn_interval(const float* __restrict__ plan, const LayerPlan& P, int i, float x, int& mfix,
                                            float& u) {
  using X = FnIdx<IMG, L>;
  const float* g = plan + X::knot(P, i, 0);
  const int gs = X::knot_stride(P);
  int m = -1;
  for (int j = 0; j < P.NG; ++j) m += x >= g[j * gs] ? 1 : 0;
  const bool fin = __builtin_isfinite(x);
  mfix = ((unsigned)m < (unsigned)P.NI && fin) ? m : P.NI;
  u = mfix < P.NI ? (x - g[mfix * gs]) * plan[X::rh(P, i, mfix)] : (fin ? 0.0f : __builtin_nanf(""));
}

// DOPRI: the whole dopri5 solve in this launch (fetode_integrate_dopri5 for these shapes), one
// trajectory per one-wave workgroup, every workgroup resident (grid sums of the error norms)
// TAPE (with DOPRI): training — every evaluation's row (x, h, k) of (tape_cap, B, 2 D + H), the rows
// fetode_integrate_dopri5_tape writes for the [2, 10, 2] fields too, and the initial-step scalars
// LDSP: the whole plan (both layers) is staged in LDS once per workgroup of kFnWavesL waves and read
// from there (every element constant, edge weight, knot and spline cubic is read per evaluation:
// from global memory each read is an L2 round trip on the evaluation's chain); plans up to
// kFnLdsMax bytes (e.g. KANFET([2, 16, 2], K = 12): 31 KB, KAN([4, 32, 4]): 67 KB — two 8-wave
// workgroups per CU still fit the 160 KB)
constexpr int kFnWavesL = 8;
constexpr int kFnMaxT = 8;  // trajectories per wave at most (H, D <= 8)
// unit lanes of a trajectory: the smallest power of two U >= max(H, D, 64 / kFnMaxT); split factor
// SF = 2 when a wave still holds two or more such groups and D >= 2: group sg of the trajectory's
// U * SF lanes takes the layer-0 inputs i = sg (mod 2) and the layer-1 outputs d = sg (mod 2), so
// each lane runs half the edges and the launch has twice the waves (the fixed-grid launch is
// latency-bound at ~one wave per SIMD otherwise).  Host and device agree on both.
__host__ __device__ inline int fn_unit_lanes(int D, int H) {
  int hp = 64 / kFnMaxT;
  while (hp < H || hp < D) hp <<= 1;
  return hp < 64 ? hp : 64;
}
__host__ __device__ inline int fn_split(int D, int H) {
  static_assert(kFnMaxT >= 2, "");
  return (fn_unit_lanes(D, H) <= 32 && D >= 2) ? 2 : 1;
}
__host__ __device__ inline int fn_lanes_per_traj(int D, int H) { return fn_unit_lanes(D, H) * fn_split(D, H); }
constexpr int64_t kFnLdsMax = 78 * 1024;
template <bool FERRO, bool DOPRI = false, bool TAPE = false, bool LDSP = false>
__global__ __launch_bounds__(DOPRI ? 64 : (LDSP ? 64 * kFnWavesL : 64 * kFnWaves)) void fieldn_kernel(FusedArgs a) {
  constexpr int NW = DOPRI ? 1 : (LDSP ? kFnWavesL : kFnWaves);
  extern __shared__ float s_plan[];
  if constexpr (LDSP) {
    fn_stage_image(s_plan, a.plan, a.P0, a.P1);  // the lane-contiguous image of both layers' plans
    __syncthreads();
  }
  if constexpr (DOPRI) {
    if (a.dp.xr_world > 1 && blockIdx.x == gridDim.x - 1) {  // the cross-rank exchange workgroup
      xrank_comm(a.dp);
      return;
    }
  }
  // trajectories per wave: lane = (slot t, split group sg, unit o) with U = pow2 >= max(H, D) unit
  // lanes and SF split groups per slot (KANFET([2, 16, 2]): two trajectories per wave, 2 x 16
  // lanes each); the resident dopri5 keeps one trajectory per wave (SF groups of 64 / SF lanes)
  constexpr int MT = DOPRI ? 1 : kFnMaxT;
  __shared__ float s_x[NW][MT][kFnMaxD], s_k[NW][MT][kFnMaxD], s_p0[NW][MT][kFnMaxD];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const LayerPlan& P0 = a.P0;
  const LayerPlan& P1 = a.P1;
  const int D = P0.in, H = P0.out;
  // the resident dopri5 keeps one trajectory per wave but splits it as well: SF groups of 64 / SF
  // lanes (lanes o >= H of a group add exact zeros to its butterfly, so the sums are the fixed-grid
  // launch's bit for bit — the host-loop and resident solves stay comparable)
  const int SF = fn_split(D, H), U = DOPRI ? 64 / SF : fn_unit_lanes(D, H), HP = U * SF, TPW = 64 / HP;
  const int t = lane / HP, sg = (lane & (HP - 1)) / U, o = lane & (U - 1);
  const bool own = sg == 0;  // the group that owns the trajectory's state and writes
  const int64_t b = ((int64_t)blockIdx.x * NW + wid) * TPW + t;
  const bool valid = b < a.B;
  const float* __restrict__ plan = LDSP ? s_plan : a.plan;
  float* xs = s_x[wid][t];
  float* ks = s_k[wid][t];
  float* p0 = s_p0[wid][t];
  const bool hl = o < H;  // this lane's hidden unit
  float prev1 = 0.f;
  if (FERRO && valid) {
    if (own && o < D) p0[o] = a.state[b * D + o];
    if (hl) prev1 = a.state[a.B * D + b * H + o];
  }
  bool re0 = FERRO && (a.init_mask & 1u), re1 = FERRO && (a.init_mask & 2u);
  const float c0o = hl ? plan[P0.fconst + o] : 0.f;
  // training tapes.  Fixed grid (fieldn_adj_kernel, fetode_fieldn_bwd.hip): two planes, the layer-0
  // inputs (n_ev, B, D) then the layer-1 inputs (n_ev, B, H).  dopri5 (TAPE): rows (x, h, k) of
  // (tape_cap, B, 2 D + H) for the first tape_cap evaluations
  const int nst = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  float* tx = (!DOPRI && a.tape && !a.single_eval) ? a.tape : nullptr;
  float* th_ = tx ? tx + (int64_t)a.n_steps * nst * a.B * D : nullptr;
  float* trow = nullptr;  // TAPE: this evaluation's row, or null past tape_cap
  int64_t ev = 0;
  auto eval = [&](void) {  // xs -> ks (all lanes), hysteresis states updated
    fn_wsync();
    if constexpr (TAPE) {
      trow = (ev < a.dp.tape_cap && valid) ? a.tape + (ev * a.B + b) * (2 * D + H) : nullptr;
      if (trow && own && o < D) trow[o] = xs[o];
    }
    if (tx && valid && own && o < D) tx[(ev * a.B + b) * D + o] = xs[o];
    // layer 0: h_o = c0 + (sum over the even inputs + sum over the odd inputs), each in input order
    // (one order for every split: the split groups hold one parity each and swap their sums)
    float h = 0.f;
    if (hl) {
      float pe = 0.f, po = 0.f;
      for (int i = sg; i < D; i += SF) {
        const float x = xs[i];
        const float sx = x * fn_sig_l2(-x * FETODE_LOG2E);
        float w = 0.f;
        if constexpr (FERRO) w = ffma(fn_sig_l2(-P0.gsl2e * (x - (re0 ? x : p0[i]))), -P0.wc, P0.wc);
        int mfix;
        float u;
        fn_interval<LDSP, 0>(plan, P0, i, x, mfix, u);
        const float e = fn_edge<FERRO, DOPRI ? 1 : 4, LDSP, 0>(plan, P0, o, i, x, sx, w, mfix, u);
        if (i & 1) po += e;
        else pe += e;
      }
      if (SF == 2) {
        const float other = __shfl_xor(sg ? po : pe, U);  // each group sends its own parity's sum
        if (sg) pe = other;
        else po = other;
      }
      h = c0o + (pe + po);
    }
    if (tx && valid && own && hl) th_[(ev * a.B + b) * H + o] = h;
    if (TAPE && trow && own && hl) trow[D + o] = h;
    ++ev;
    fn_wsync();
    if (FERRO && own && o < D) p0[o] = xs[o];  // ferro_class.py:409
    re0 = false;
    // layer 1: lane o's contributions to every output, then the sum over the lanes
    float w1 = 0.f, sh = 0.f, u1 = 0.f;
    int m1 = 0;
    if (hl) {
      sh = h * fn_sig_l2(-h * FETODE_LOG2E);
      if constexpr (FERRO) w1 = ffma(fn_sig_l2(-P1.gsl2e * (h - (re1 ? h : prev1))), -P1.wc, P1.wc);
      fn_interval<LDSP, 1>(plan, P1, o, h, m1, u1);
    }
    if (FERRO) prev1 = h;
    re1 = false;
    for (int d = sg; d < D; d += SF) {  // group sg: the outputs d = sg (mod SF)
      float v = hl ? fn_edge<FERRO, DOPRI ? 1 : 4, LDSP, 1>(plan, P1, d, o, h, sh, w1, m1, u1) : 0.f;
      for (int s = U >> 1; s >= 1; s >>= 1) v += __shfl_xor(v, s);  // within the group's U lanes
      if (o == 0) ks[d] = v + plan[P1.fconst + d];
    }
    fn_wsync();
  };
  // lane d < D carries state dim d
  const bool dl = own && o < D;
  float y = (valid && dl) ? a.y0[b * D + o] : 0.f;
  if constexpr (DOPRI) {
    // ---- device-resident dopri5: fused4's driver (dopri5.py _Dopri5's control arithmetic) with
    // lane d < D of the trajectory's wave carrying y_d; one grid sum per norm ----
    const DopriParams& P = a.dp;
    const bool real = valid && dl;  // one lane per (trajectory, state dim) in the sums
    const double n_el = P.n_total;
    int nfev = 0, n_att = 0, status = 0;
    unsigned round = 0;
    auto gsum2 = [&](double v0, double v1, double& s0, double& s1) {
      v0 = xor_sum64(v0);
      v1 = xor_sum64(v1);
      if (grid_sum2(P, round, v0, v1, s0, s1)) status = 4;
    };
    auto f = [&](float xin) -> float {
      if (dl) xs[o] = xin;
      eval();
      const float k = dl ? ks[o] : 0.f;
      if (TAPE && trow && dl) trow[D + H + o] = k;
      return k;
    };
    if (real) a.solution[b * D + o] = y;
    float f0 = f(y);
    ++nfev;
    double dt;
    if (P.first_step > 0.0) {
      dt = P.first_step;
    } else {  // misc._select_initial_step in fp32 (dopri5.py select_initial_step)
      const float scale = P.atol + P.rtol * fabsf(y);
      const float q0 = y / scale, q1 = f0 / scale;
      double s0, s1;
      gsum2(real ? (double)q0 * q0 : 0.0, real ? (double)q1 * q1 : 0.0, s0, s1);
      const float d0 = fabsf(sqrtf((float)(s0 / n_el)));
      const float d1 = fabsf(sqrtf((float)(s1 / n_el)));
      float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
      h0 = fabsf(h0);
      const float f1 = f(y + f0 * h0);
      ++nfev;
      const float q2 = (f1 - f0) / scale;
      gsum2(real ? (double)q2 * q2 : 0.0, 0.0, s0, s1);
      const float d2 = fabsf(sqrtf((float)(s0 / n_el)) / h0);
      float h1;
      if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
      else h1 = (float)pow((double)(0.01f / fmaxf(d1, d2)), (double)0.2f);  // fp64 pow rounded once
      dt = (double)fminf(100.0f * h0, fabsf(h1));
      if (TAPE && blockIdx.x == 0 && threadIdx.x == 0) {
        P.init_rec[0] = d0;
        P.init_rec[1] = d1;
        P.init_rec[2] = d2;
        P.init_rec[3] = h0;
        P.init_rec[4] = h1;
      }
    }
    float co[5] = {y, 0.f, 0.f, 0.f, 0.f};
    double t0s = P.t[0], t1s = P.t[0];
    for (int i = 1; i < P.T && status == 0; ++i) {
      const double next_t = P.t[i];
      int n_steps = 0;
      while (next_t > t1s) {
        if (n_steps >= P.max_steps) { status = 3; break; }
        const double t0 = t1s;
        if (!(t0 + dt > t0)) { status = 2; break; }
        const float dt32 = (float)dt;
        const double t1 = t0 + dt;
        // rk_common._runge_kutta_step in fetode_lincomb's op order, accumulated as the stages
        // arrive: A[q] is stage s + 1 + q's sum k0 c0 + k1 c1 + ... (left-to-right sums)
        float A[6];
        for (int q = 0; q < 6; ++q) A[q] = f0 * (P.stc[0][q] * dt32);
        float err = f0 * (P.stc[0][6] * dt32);
        float mid = f0 * (P.stc[0][7] * dt32);
        float yi = y, kn = f0;
        for (int st = 0; st < 6; ++st) {
          yi = y + A[0];
          kn = f(yi);
          ++nfev;
          for (int q = 0; q < 5; ++q) A[q] = A[q + 1] + kn * (P.stc[st + 1][q] * dt32);
          err = err + kn * (P.stc[st + 1][6] * dt32);
          mid = mid + kn * (P.stc[st + 1][7] * dt32);
        }
        const float y1 = yi;
        const float tol = P.atol + P.rtol * fmaxf(fabsf(y), fabsf(y1));
        const float qe = err / tol;
        double sq, nbad;
        gsum2(real ? (double)qe * qe : 0.0, (real && !__builtin_isfinite(y)) ? 1.0 : 0.0, sq, nbad);
        if (status) break;
        if (nbad != 0.0) { status = 1; break; }
        const float ratio = sqrtf((float)(sq / n_el));
        const bool accept = ratio <= 1.0f;
        if (blockIdx.x == 0 && threadIdx.x == 0 && n_att < P.max_att) {
          double* o = P.att + (int64_t)n_att * 4;
          o[0] = t0;
          o[1] = dt;
          o[2] = (double)ratio;
          o[3] = accept ? 1.0 : 0.0;
        }
        ++n_att;
        if (accept) {  // interp._interp_fit (fetode_interp_fit's op order)
          const float ym = y + mid, fa = f0, fb6 = kn;
          co[4] = ((2.0f * dt32) * (fb6 - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
          co[3] = ((dt32 * (5.0f * fa - 3.0f * fb6) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
          co[2] = ((dt32 * (fb6 - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
          co[1] = dt32 * fa;
          co[0] = y;
          y = y1;
          f0 = kn;
          t0s = t0;
          t1s = t1;
        } else {
          t0s = t0;
        }
        // rk_common._optimal_step_size in fp64 (dopri5.py optimal_step)
        const double rr = (double)ratio;
        double nxt;
        if (rr == 0.0) {
          nxt = dt * P.ifactor;
        } else {
          const double dfac = rr < 1.0 ? 1.0 : P.dfactor;
          const double factor = __builtin_isnan(rr) ? rr : fmin(P.ifactor, fmax(P.safety / pow(rr, 1.0 / 5.0), dfac));
          nxt = dt * factor;
        }
        dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, P.min_step), P.max_step);
        ++n_steps;
      }
      if (status) break;
      const float xq = (float)((next_t - t0s) / (t1s - t0s));  // interp._interp_evaluate
      float total = co[0] + xq * co[1];
      float xp = xq;
      for (int j = 2; j < 5; ++j) {
        xp = xp * xq;
        total = total + xp * co[j];
      }
      if (real) a.solution[((int64_t)i * a.B + b) * D + o] = total;
    }
    if (P.xr_world > 1 && blockIdx.x == 0 && threadIdx.x == 0)  // the exchange workgroup may stop
      __hip_atomic_store(dp_fin(P), round + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      P.stats[0] = nfev;
      P.stats[1] = n_att;
      P.stats[2] = __hip_atomic_load(P.bar + kDpLine * (kDpGroups + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 4 : status;
    }
  } else if (a.single_eval) {
    if (dl) xs[o] = y;
    eval();
    if (valid && dl) a.eval_out[b * D + o] = ks[o];
  } else {
    if (valid && dl) a.solution[b * D + o] = y;
    const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
    const float third = 1.0f / 3.0f;
    int jj = 1;
    for (int s = 0; s < a.n_steps; ++s) {
      const float dt = a.step_coef[4 * s], hh = a.step_coef[4 * s + 1], h6 = a.step_coef[4 * s + 2];
      float k1 = 0.f, k2 = 0.f, k3 = 0.f, k4 = 0.f;
      for (int st = 0; st < ns; ++st) {  // fused4's generic path, same op order
        float xin = y;
        if (a.method == FETODE_RK4) {
          if (st == 1) xin = y + (dt * k1) * third;
          else if (st == 2) xin = y + dt * (k2 - k1 * third);
          else if (st == 3) xin = y + dt * ((k1 - k2) + k3);
        } else if (a.method == FETODE_RK4_CLASSIC) {
          if (st == 1) xin = y + hh * k1;
          else if (st == 2) xin = y + hh * k2;
          else if (st == 3) xin = y + dt * k3;
        } else if (a.method == FETODE_MIDPOINT) {
          if (st == 1) xin = y + k1 * hh;
        }
        if (dl) xs[o] = xin;
        eval();
        const float kk = dl ? ks[o] : 0.f;
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
      for (; jj < a.T && a.out_step[jj] == s; ++jj) {
        const int mode = a.out_mode[jj];
        const float v = mode == 0 ? y : (mode == 1 ? y1 : y + a.out_slope[jj] * (y1 - y));
        if (valid && dl) a.solution[((int64_t)jj * a.B + b) * D + o] = v;
      }
      y = y1;
    }
  }
  if (FERRO && valid) {
    if (dl) a.state[b * D + o] = p0[o];
    if (own && hl) a.state[a.B * D + b * H + o] = prev1;
  }
}

// the shapes fieldn serves (any other depth-2 [D, H, D] field of the fused kernels' basis shape)
bool fieldn_supported(const fetode_field_t* f) {
  static const bool on = [] {  // FETODE_FIELDN=0: these shapes take the per-stage path (A/B diagnostics)
    const char* e = getenv("FETODE_FIELDN");
    return !e || atoi(e) != 0;
  }();
  if (!on || f->n_layers != 2) return false;
  const fetode_kanlinear_t &k0 = f->kan[0], &k1 = f->kan[1];
  if (k0.in_features < 1 || k0.in_features > kFnMaxD || k1.out_features != k0.in_features ||
      k1.in_features != k0.out_features || k0.out_features < 1 || k0.out_features > kFnMaxH)
    return false;
  if (k0.spline_order != 3 || k1.spline_order != 3 || k0.grid_size != k1.grid_size) return false;
  if (f->ferro && (f->ferro[0].branch_sign || f->ferro[1].branch_sign)) return false;
  return true;
}

int launch_fused(const fetode_field_t* f, FusedArgs& a, void* stream) {
  const FusedEntry* e = find_fused(f);
  if (!e) {  // other widths: the generic single-launch kernel (inference and single evaluations)
    if (!fieldn_supported(f)) return set_err(FETODE_EUNSUPPORTED, "no fused kernel for this field shape");
    layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
    layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
    const int64_t pbytes = (int64_t)sizeof(float) * a.P1.end;
    const int tpw = 64 / fn_lanes_per_traj(a.P0.in, a.P0.out);
    static const int lds_on = [] {  // FETODE_FIELDN_LDS=0: the plan read from global memory (A/B)
      const char* e = getenv("FETODE_FIELDN_LDS");
      return e ? atoi(e) : 1;
    }();
    if (lds_on && pbytes <= kFnLdsMax) {
      auto* kfn = f->ferro ? fieldn_kernel<true, false, false, true> : fieldn_kernel<false, false, false, true>;
      static bool attr[2] = {false, false};  // dynamic LDS beyond the 64 KB default
      if (!attr[f->ferro ? 1 : 0]) {
        HIP_CHECK_RET(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFnLdsMax));
        attr[f->ferro ? 1 : 0] = true;
      }
      hipLaunchKernelGGL(kfn, dim3(nblk(a.B, (int64_t)kFnWavesL * tpw)), dim3(64 * kFnWavesL), (size_t)pbytes,
                         (hipStream_t)stream, a);
    } else
      hipLaunchKernelGGL(f->ferro ? fieldn_kernel<true> : fieldn_kernel<false>, dim3(nblk(a.B, (int64_t)kFnWaves * tpw)),
                         dim3(64 * kFnWaves), 0, (hipStream_t)stream, a);
    LAUNCH_CHECK();
    return FETODE_OK;
  }
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  static const float limit = [] {
    const char* e = getenv("FETODE_FACTOR_LIMIT");
    return e ? (float)atof(e) : kFactorLimit;
  }();
  a.factor_limit = limit;
  const bool rk4 = !a.single_eval && a.method == FETODE_RK4;
  if (rk4 && !a.tape && a.B > g_v8_lo && a.B <= g_v8_hi) {   // v8, two waves per trajectory
    if (g_v8_tpb == 2)
      hipLaunchKernelGGL(e->rk4_v8x2, dim3(nblk(a.B, 2)), dim3(256), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(e->rk4_v8, dim3((unsigned)a.B), dim3(128), 0, (hipStream_t)stream, a);
  } else if (rk4 && a.B > g_tpw1_lo && a.B <= g_tpw1_hi) {   // v7, one trajectory per wave (tapes too)
    hipLaunchKernelGGL(a.tape ? e->fn_rk4_1_tape : e->fn_rk4_1, dim3((unsigned)a.B), dim3(64), 0, (hipStream_t)stream, a);
  } else if (a.B <= small_max()) {  // v6: one trajectory per 192-thread workgroup (training tapes too)
    const fused_fn fn = a.tape ? (rk4 ? e->small_rk4_tape : e->small_tape) : (rk4 ? e->small_rk4 : e->small);
    hipLaunchKernelGGL(fn, dim3((unsigned)a.B), dim3(192), 0, (hipStream_t)stream, a);
  } else {                              // v4: two trajectories per one-wave workgroup
    const fused_fn fn = a.tape ? (rk4 ? e->fn_rk4_tape : e->fn_tape) : (rk4 ? e->fn_rk4 : e->fn);
    hipLaunchKernelGGL(fn, dim3(nblk(a.B, 2)), dim3(64), 0, (hipStream_t)stream, a);
  }
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // namespace

bool fetode::fieldn_shape_supported(const fetode_field_t* f) { return find_fused(f) == nullptr && fieldn_supported(f); }

extern "C" {

#ifdef FETODE_STAMPS
int fetode_debug_stamp_buffer(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fetode_stamps), &p, sizeof(p)) == hipSuccess ? FETODE_OK : FETODE_EHIP;
}
#endif

uint32_t fetode_dopri5_set_spin_limit(uint32_t polls) {
  const uint32_t prev = g_dp_spin_limit;
  g_dp_spin_limit = polls;
  return prev;
}

int64_t fetode_fused_set_small_batch_max(int64_t b) {
  const int64_t prev = g_small_max;
  if (b >= 0) g_small_max = b;
  return prev;
}

int64_t fetode_fused_set_tpw1_range(int64_t lo, int64_t hi) {
  const int64_t prev = g_tpw1_hi;
  if (lo >= 0) g_tpw1_lo = lo;
  if (hi >= 0) g_tpw1_hi = hi;
  return prev;
}

int64_t fetode_fused_set_v8_range(int64_t lo, int64_t hi) {
  const int64_t prev = g_v8_hi;
  if (lo >= 0) g_v8_lo = lo;
  if (hi >= 0) g_v8_hi = hi;
  return prev;
}

int fetode_fused_get_batch_ranges(int64_t* out) {
  if (!out) return set_err(FETODE_EINVAL, "fetode_fused_get_batch_ranges: null output");
  out[0] = g_small_max;
  out[1] = g_tpw1_lo;
  out[2] = g_tpw1_hi;
  out[3] = g_v8_lo;
  out[4] = g_v8_hi;
  return FETODE_OK;
}

int fetode_fused_supported(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return 0;
  return find_fused(f) != nullptr || fieldn_supported(f);
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

int64_t fetode_integrate_dopri5_workspace(int64_t B) {
  const int64_t grid = B;  // v6 (one trajectory per workgroup) at small batches, v4 (two) beyond
  return (int64_t)sizeof(unsigned) * kDpBarWords + (int64_t)sizeof(double) * (2 * grid + 4 * kDpGroups + 4);
}

// every workgroup must be resident at once (grid reductions): one-wave workgroups of two
// trajectories, as many as the occupancy of the DOPRI instantiation admits (-1: query failed)
// v6's dopri5 driver: one 192-thread workgroup per trajectory, every one resident
static int64_t dopri5_small_resident_wgs(const FusedEntry* e, bool ferro) {
  static int n_cu = 0, per_cu[2] = {0, 0};
  const int fi = ferro ? 0 : 1;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
  }
  if (!per_cu[fi] && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[fi], e->small_dopri, 192, 0) != hipSuccess)
    return -1;
  return (int64_t)per_cu[fi] * n_cu;
}

static int64_t dopri5_resident_wgs(const FusedEntry* e, bool ferro) {
  static int n_cu = 0, per_cu[2] = {0, 0};
  const int fi = ferro ? 0 : 1;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
  }
  if (!per_cu[fi] && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[fi], e->dopri, 64, 0) != hipSuccess) return -1;
  return (int64_t)per_cu[fi] * n_cu;
}

// fieldn's dopri5 driver: one trajectory per one-wave workgroup, every one resident
static const void* fieldn_dopri_fn(bool ferro, bool tape) {
  return ferro ? (tape ? (const void*)fieldn_kernel<true, true, true> : (const void*)fieldn_kernel<true, true, false>)
               : (tape ? (const void*)fieldn_kernel<false, true, true> : (const void*)fieldn_kernel<false, true, false>);
}
static int64_t dopri5_fieldn_resident_wgs(bool ferro, bool tape = false) {
  static int n_cu = 0, per_cu[2][2] = {{0, 0}, {0, 0}};
  const int fi = ferro ? 0 : 1, ti = tape ? 1 : 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
  }
  if (!per_cu[fi][ti] && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[fi][ti], fieldn_dopri_fn(ferro, tape), 64, 0) !=
                             hipSuccess)
    return -1;
  return (int64_t)per_cu[fi][ti] * n_cu;
}

int64_t fetode_integrate_dopri5_max_batch(const fetode_field_t* f, int32_t sharded) {
  if (validate_field(f) != FETODE_OK) return 0;
  const FusedEntry* e = find_fused(f);
  if (!e && fieldn_supported(f)) {  // the taped variant's grid bounds training solves too
    const int64_t w0 = dopri5_fieldn_resident_wgs(f->ferro != nullptr), w1 = dopri5_fieldn_resident_wgs(f->ferro != nullptr, true);
    const int64_t w = (w0 < w1 ? w0 : w1) - (sharded ? 1 : 0);
    return w > 0 ? w : 0;
  }
  if (!e) return 0;
  const int64_t w = dopri5_resident_wgs(e, f->ferro != nullptr) - (sharded ? 1 : 0);
  return w > 0 ? 2 * w : 0;
}

static int dopri5_launch(const fetode_field_t* f, const void* plan, const float* y0, int64_t B, const double* t,
                         int32_t T, double rtol, double atol, const double* opts, const float* tableau,
                         float* solution, float* state, uint32_t init_mask, void* workspace, int32_t* stats,
                         double* attempts, int32_t max_attempts, const fetode_xrank_t* xr, int64_t B_total,
                         float* tape, int64_t tape_cap, double* init_rec, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!plan || !y0 || !t || !opts || !tableau || !solution || !workspace || !stats || (f->ferro && !state))
    return set_err(FETODE_EINVAL, "dopri5: null pointer");
  if (f->kan[0].in_features != f->kan[f->n_layers - 1].out_features)
    return set_err(FETODE_EINVAL, "field is not R^D -> R^D");
  const FusedEntry* e = find_fused(f);
  // other widths: fieldn's driver, one trajectory per one-wave workgroup
  const bool fn = !e && fieldn_supported(f);
  if (!e && !fn) return set_err(FETODE_EUNSUPPORTED, "no fused dopri5 kernel for this field shape");
  const bool sharded = xr && xr->world > 1;
  // small batches (the reference's own X0 (1, 2); the strong-scaled shard): v6, one trajectory per
  // workgroup, when the whole grid is resident; else v4, two per one-wave workgroup
  const int64_t res6 = (!fn && !sharded && B <= small_max()) ? dopri5_small_resident_wgs(e, f->ferro != nullptr) : -1;
  const bool use6 = res6 >= B;
  const int64_t resident = fn ? dopri5_fieldn_resident_wgs(f->ferro != nullptr, tape_cap > 0)
                              : use6 ? res6 : dopri5_resident_wgs(e, f->ferro != nullptr);
  if (resident < 0) return set_err(FETODE_EHIP, "dopri5: occupancy query failed");
  const int per = fn ? 1 : 2;  // trajectories per workgroup (v6: one, never sharded)
  const int64_t grid = (use6 || fn) ? B : nblk(B, 2);
  const int64_t lgrid = grid + (sharded ? 1 : 0);   // + the cross-rank exchange workgroup
  if (lgrid > resident)
    return set_err(FETODE_EUNSUPPORTED, "dopri5: batch %lld needs %lld workgroups, %lld resident", (long long)B,
                   (long long)lgrid, (long long)resident);
  FusedArgs a;
  memset(&a, 0, sizeof(a));
  a.plan = (const float*)plan;
  a.method = FETODE_RK4;
  a.y0 = y0;
  a.B = B;
  a.T = T;
  a.solution = solution;
  a.state = state;
  a.init_mask = init_mask;
  a.tape = tape_cap > 0 ? tape : nullptr;
  DopriParams& P = a.dp;
  P.on = 1;
  P.spin_limit = g_dp_spin_limit;
  P.tape_cap = tape_cap;
  P.init_rec = init_rec;
  P.t = t;
  P.T = T;
  P.rtol = (float)rtol;
  P.atol = (float)atol;
  P.first_step = opts[0];
  P.safety = opts[1];
  P.ifactor = opts[2];
  P.dfactor = opts[3];
  P.min_step = opts[4];
  P.max_step = opts[5];
  P.max_steps = opts[6] > 2e9 ? 2000000000 : (int)opts[6];
  for (int j = 0; j < 7; ++j) {  // tableau = beta (6 x 6, row i = stage i + 1), c_error (7), c_mid (7)
    for (int q = 0; q < 6; ++q) P.stc[j][q] = (j < 6 && j + q < 6) ? tableau[(j + q) * 6 + j] : 0.0f;
    P.stc[j][6] = tableau[36 + j];
    P.stc[j][7] = tableau[43 + j];
  }
  P.bar = (unsigned*)workspace;
  double* d = (double*)((char*)workspace + sizeof(unsigned) * kDpBarWords);
  P.slot = d;
  P.xs = d + 2 * grid;
  P.stats = stats;
  P.att = attempts;
  P.max_att = attempts ? max_attempts : 0;
  P.xr_g = P.xs + 4 * kDpGroups;
  P.n_total = (double)B_total * f->kan[0].in_features;
  // leaves: runs of L workgroups; exact when this rank's workgroups are whole leaves of the
  // single-device grid over the global batch (two trajectories per workgroup everywhere)
  auto cdiv = [](int64_t a_, int64_t b_) { return (a_ + b_ - 1) / b_; };
  auto lshift = [&](int64_t nb) {   // the smallest power-of-two leaf that needs <= kDpGroups leaves
    int sh = 0;
    while ((int64_t)kDpGroups << sh < nb) ++sh;
    return sh;
  };
  // leaves of `n` workgroups from a block boundary: full blocks of 8 leaves, then the last block's
  // leaves that have at least one workgroup (a prefix of its 8)
  auto nleaves = [&](int64_t n, int sh) -> int64_t {
    const int64_t blk = (int64_t)8 << sh, nb = cdiv(n, blk);
    return nb == 0 ? 0 : 8 * (nb - 1) + std::min<int64_t>(8, n - (nb - 1) * blk);
  };
  P.xr_exact = 0;
  P.wg_off = 0;
  P.nblk_global = (int32_t)grid;
  P.leaf_shift = lshift(grid);
  if (sharded) {
    P.xr_rank = xr->rank;
    P.xr_world = xr->world;
    P.xr_epoch = xr->epoch;
    P.xr_peers = (double* const*)xr->peers;
    P.xr_inbox = (double*)xr->inbox;
    const int64_t gg = cdiv(B_total, per), shg = lshift(gg), Bk = (int64_t)8 << shg, off = xr->b_offset / per;
    const bool last = xr->b_offset + B == B_total;
    if (xr->b_offset % per == 0 && (B % per == 0 || last) && off % Bk == 0 && ((off + grid) % Bk == 0 || last)) {
      P.xr_exact = 1;
      P.wg_off = (int32_t)off;
      P.nblk_global = (int32_t)gg;
      P.leaf_shift = (int32_t)shg;
    }
  } else {
    P.xr_world = 1;
  }
  P.leaf_lo = (P.wg_off >> (P.leaf_shift + 3)) * 8;
  P.n_leaf_local = (int32_t)nleaves(grid, P.leaf_shift);
  P.n_leaf_global = (int32_t)nleaves(P.nblk_global, P.leaf_shift);
  layer_plan(f->kan[0], f->ferro ? &f->ferro[0] : nullptr, 0, &a.P0);
  layer_plan(f->kan[1], f->ferro ? &f->ferro[1] : nullptr, a.P0.end, &a.P1);
  a.factor_limit = kFactorLimit;
  hipStream_t s = (hipStream_t)stream;
  HIP_CHECK_RET(hipMemsetAsync(workspace, 0, sizeof(unsigned) * kDpBarWords, s));
  void* args[] = {&a};
  const void* kfn = fn ? fieldn_dopri_fn(f->ferro != nullptr, a.tape != nullptr)
                   : use6 ? (const void*)(a.tape ? e->small_dopri_tape : e->small_dopri)
                          : (const void*)(a.tape ? e->dopri_tape : e->dopri);
  HIP_CHECK_RET(resident_launch(kfn, dim3((unsigned)lgrid), dim3(use6 ? 192 : 64), args, 0, s));
  return FETODE_OK;
}

int fetode_integrate_dopri5(const fetode_field_t* f, const void* plan, const float* y0, int64_t B, const double* t,
                            int32_t T, double rtol, double atol, const double* opts, const float* tableau,
                            float* solution, float* state, uint32_t init_mask, void* workspace, int32_t* stats,
                            double* attempts, int32_t max_attempts, void* stream) {
  return dopri5_launch(f, plan, y0, B, t, T, rtol, atol, opts, tableau, solution, state, init_mask, workspace, stats,
                       attempts, max_attempts, nullptr, B, nullptr, 0, nullptr, stream);
}

int fetode_integrate_dopri5_tape(const fetode_field_t* f, const void* plan, const float* y0, int64_t B, const double* t,
                                 int32_t T, double rtol, double atol, const double* opts, const float* tableau,
                                 float* solution, float* state, uint32_t init_mask, void* workspace, int32_t* stats,
                                 double* attempts, int32_t max_attempts, float* tape, int64_t tape_cap,
                                 double* init_rec, void* stream) {
  if (tape_cap <= 0 || !tape || !init_rec || !attempts)
    return set_err(FETODE_EINVAL, "dopri5 tape: null tape / init record / attempt log, or tape_cap <= 0");
  return dopri5_launch(f, plan, y0, B, t, T, rtol, atol, opts, tableau, solution, state, init_mask, workspace, stats,
                       attempts, max_attempts, nullptr, B, tape, tape_cap, init_rec, stream);
}

int fetode_integrate_dopri5_xrank(const fetode_field_t* f, const void* plan, const float* y0, int64_t B,
                                  int64_t B_total, const double* t, int32_t T, double rtol, double atol,
                                  const double* opts, const float* tableau, float* solution, float* state,
                                  uint32_t init_mask, void* workspace, int32_t* stats, double* attempts,
                                  int32_t max_attempts, const fetode_xrank_t* xr, void* stream) {
  if (!xr || xr->world < 1 || xr->rank < 0 || xr->rank >= xr->world || xr->world > 64)
    return set_err(FETODE_EINVAL, "dopri5 xrank: bad rank / world");
  if (xr->world > 1 && (!xr->peers || !xr->inbox)) return set_err(FETODE_EINVAL, "dopri5 xrank: null inbox / peers");
  if (B_total < B || xr->b_offset < 0 || xr->b_offset + B > B_total)
    return set_err(FETODE_EINVAL, "dopri5 xrank: shard [%lld, %lld) outside the global batch %lld",
                   (long long)xr->b_offset, (long long)(xr->b_offset + B), (long long)B_total);
  return dopri5_launch(f, plan, y0, B, t, T, rtol, atol, opts, tableau, solution, state, init_mask, workspace, stats,
                       attempts, max_attempts, xr, B_total, nullptr, 0, nullptr, stream);
}

int64_t fetode_xrank_inbox_bytes(int32_t world) {
  if (world < 1 || world > 64) return -1;
  return (int64_t)sizeof(double) * (2 * 2 * 64 + 2 * 64);   // (2, 64) records + (2, 64) tags
}

int fetode_xrank_alloc(int64_t bytes, void** dev_ptr, void* handle) {
  if (bytes <= 0 || !dev_ptr || !handle) return set_err(FETODE_EINVAL, "xrank alloc: bad argument");
  void* p = nullptr;
  // fine-grained device memory: coherent for the system-scope stores / loads of the exchange.  No
  // coarse-grained fallback: a peer spinning on coarse-grained IPC memory is not guaranteed to see
  // remote stores, so without it the caller declines the resident sharded path on every rank
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained) != hipSuccess || !p) {
    const hipError_t e = hipGetLastError();
    return set_err(FETODE_EUNSUPPORTED, "xrank alloc: no fine-grained device memory (%s)", hipGetErrorString(e));
  }
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess) {
    const hipError_t e = hipGetLastError();
    (void)hipFree(p);
    return set_err(FETODE_EHIP, "xrank alloc: hipMemset: %s", hipGetErrorString(e));
  }
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return set_err(FETODE_EHIP, "hipIpcGetMemHandle: %s", hipGetErrorString(e));
  }
  memcpy(handle, &h, sizeof(h) < 64 ? sizeof(h) : 64);
  *dev_ptr = p;
  return FETODE_OK;
}

int fetode_xrank_open(const void* handle, void** dev_ptr) {
  if (!handle || !dev_ptr) return set_err(FETODE_EINVAL, "xrank open: bad argument");
  hipIpcMemHandle_t h;
  memset(&h, 0, sizeof(h));
  memcpy(&h, handle, sizeof(h) < 64 ? sizeof(h) : 64);
  HIP_CHECK_RET(hipIpcOpenMemHandle(dev_ptr, h, hipIpcMemLazyEnablePeerAccess));
  return FETODE_OK;
}

int fetode_xrank_close(void* dev_ptr) {
  if (dev_ptr) HIP_CHECK_RET(hipIpcCloseMemHandle(dev_ptr));
  return FETODE_OK;
}

int fetode_xrank_free(void* dev_ptr) {
  if (dev_ptr) HIP_CHECK_RET(hipFree(dev_ptr));
  return FETODE_OK;
}

int fetode_integrate_fixed(const fetode_field_t* f, const void* plan, int32_t method, const float* y0,
                           int64_t B, const float* step_coef, int32_t n_steps, const int32_t* out_step,
                           const int32_t* out_mode, const float* out_slope, int32_t T, float* solution,
                           float* state, uint32_t init_mask, float* tape, void* stream) {
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
  a.tape = tape;
  return launch_fused(f, a, stream);
}

}  // extern "C"
