// fetode_wide.hip — one KAN-FET layer at production widths (64..128 in / out) in ONE launch:
//   out[b, o] = KANLinear(x)[b, o] + FerroelectricBasis(x)[b, o]          (KANFET layer, A9)
// or either half alone (KANLinear.forward / FerroelectricBasis.forward with the constant
// branch_sign, no activations).  BASELINE configs[3] runs KANFET([64, 128, 64], K = 10) this way,
// two launches per field evaluation (train_kan_fet_ett.py:136-197 with the KAN-FET field;
// efficientkan.py:160-182; ferro_class.py:368-420).
//
// Workgroup = 8 waves = a tile of 64 rows x 16 outputs; the inputs are walked in chunks of kCh = 8:
//   staging   one (row, input) item per thread: the hysteresis gate w = -2(1-alpha)(1-sigma(gs(x -
//             prev))) and e = e^{gs x} for the Ferro elements, and the 20 KAN features (SiLU, the 8
//             cubic B-spline bases by the reference's Cox-de Boor, 10 logistic bases) into LDS;
//   Ferro     wave w owns outputs 2w, 2w+1 for all 64 rows (lane = row), so every Ferro constant
//             is wave-uniform (scalar loads into SGPR operands, no LDS traffic): per element
//               s = 1/(1 + e P),  m = 1 + w s,  z = 2 log2e k (x + Ec m),  th = 1 - 2/(1 + 2^z)
//             (P = e^{gs Ec} packed once; branch_sign = 1 makes the crossing gate cp drop out, as in
//             the fused LV kernel), 7 VALU + 3 transcendental instructions;
//   KAN       the (64 x 16) x (in * 20) contraction on v_mfma_f32_16x16x4_f32: wave w owns rows
//             16 (w % 4).. and the chunk inputs of parity w / 4, A = the staged features (LDS, pitch
//             = 2 mod 32: conflict-free), B = the packed weights (global, L2-resident, loaded at the
//             chunk start), two accumulators alternating per input (half the dependent MFMA chain).
// Epilogue: the two K-halves and the Ferro sums (lane = row) meet the MFMA tile in LDS, fixed order.
//
// Factored gate: s = 1/(1 + e P) with e = 2^{gs log2e x} staged per (row, input) and P =
// 2^{gs log2e Ec} per element.  With |gs Ec| <= 60 for every element of an (output, input), e
// overflowing (gs x > 88.7) or flushing (gs x < -87.3) only happens where the fp32 sigmoid is
// already saturated (|gs (x + Ec)| > 27), and inf * P / 0 * P give its limits, so no bound on x
// is needed.  An (output, input) with some |gs Ec| > 60 evaluates s = 1/(1 + 2^{gs log2e (x +
// Ec)}) directly, one more exponential per element.
#include <algorithm>
#include <cstdlib>

#include "fetode_common.h"

using namespace fetode;

namespace {

#include "fetode_xrank.h"

constexpr float kWideFactorLimit = 60.0f;  // |gs Ec| bound of the factored gate (header comment)
#ifndef WIDE_FOLD
#define WIDE_FOLD 0   // 1: the folded tanh (rounds 3-5; diagnostics / A-B)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }
__device__ __forceinline__ f2 ex2x2(f2 v) { return f2{ex2(v.x), ex2(v.y)}; }
__device__ __forceinline__ f2 rcpx2(f2 v) { return f2{rcp(v.x), rcp(v.y)}; }

constexpr int kWF = 20;       // KAN features per input: SiLU, B_0..B_7, phi_0..phi_9, 0
constexpr int kNS = 8, kNB = 10, kNG = 12;
constexpr int kRows = 64, kOuts = 16, kChMax = 8, kWaves = 8, kThreads = 64 * kWaves;
constexpr int kJ = kOuts / kWaves;      // Ferro outputs per wave
// LDS pitch of a row of staged features: = 2 (mod 32), so the MFMA A-operand reads are conflict-free
constexpr int pitch_of(int ch) { return ((ch * kWF + 29) / 32) * 32 + 2; }

// packed plan of one layer (offsets in floats)
struct WideLayout {
  int in, out, K;
  bool kan, ferro;
  int64_t fe4;     // (out, in, K) float4 {P = 2^{gs log2e Ec}, 2 log2e k, 2 log2e k Ec, coef Ps}
  int64_t gec;     // (out, in, K) gs log2e Ec (direct form)
  int64_t dflag;   // (out, in) 1 if some |gs Ec| > kWideFactorLimit for (o, i)
  int64_t fconst;  // (out) sum_{i,k} coef bias (WIDE_FOLD: + coef Ps, the folded tanh's constant part)
  int64_t wp;      // (in, 20, out) packed KAN weights
  int64_t lg;      // (in, NB, 2) (-a log2e, a b log2e)
  int64_t knots;   // (in, 12) knot grid (efficientkan.py:55-61 buffer)
  int64_t rh;      // (in, 11) 1 / (g[m+1] - g[m])
  int64_t bt;      // (in, 12, 8) float4: basis c on knot interval m as a cubic in u (m = 11: zero)
  int64_t par;     // (in, 64): knots (12) | 1 / (g[j+1] - g[j]) (11) | 0 | logistic (-a log2e, a b log2e) (20)
                   //           | 1 / (g[j+2] - g[j]) (10) | 1 / (g[j+3] - g[j]) (9) | 0
  int64_t end;
  float gsl2e, gs, wc;
};

WideLayout wide_layout(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl) {
  WideLayout L{};
  L.kan = kl != nullptr;
  L.ferro = fl != nullptr;
  L.in = kl ? kl->in_features : fl->in_dim;
  L.out = kl ? kl->out_features : fl->out_dim;
  L.K = fl ? fl->num_basis : 0;
  int64_t o = 0;
  if (L.ferro) {
    const int64_t NE = (int64_t)L.out * L.in * L.K;
    L.fe4 = o; o += 4 * NE;
    L.gec = o; o += NE;
    L.dflag = o; o += (int64_t)L.out * L.in;
  }
  L.fconst = o; o += L.out;
  o = (o + 3) & ~int64_t(3);
  if (L.kan) {
    L.wp = o; o += (int64_t)L.in * kWF * L.out;
    L.lg = o; o += (int64_t)L.in * kNB * 2;
    L.knots = o; o += (int64_t)L.in * kNG;
    L.rh = o; o += (int64_t)L.in * (kNG - 1);
    o = (o + 3) & ~int64_t(3);
    L.bt = o; o += (int64_t)L.in * kNG * kNS * 4;
    L.par = o; o += (int64_t)L.in * 64;
  }
  L.end = (o + 3) & ~int64_t(3);
  L.gs = fl ? (float)fl->gate_slope : 0.f;
  L.gsl2e = L.gs * FETODE_LOG2E;
  L.wc = fl ? -2.0f * (float)(1.0 - fl->alpha) : 0.f;
  return L;
}

bool wide_supported(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl) {
  if (!kl && !fl) return false;
  if (kl && (kl->grid_size != 5 || kl->spline_order != 3 || kl->num_logistic != kNB || !kl->grid || !kl->base_weight ||
             !kl->spline_weight || !kl->logistic_a || !kl->logistic_b || !kl->logistic_weight))
    return false;
  if (fl && (fl->num_basis != 10 && fl->num_basis != 12)) return false;
  if (fl && (fl->branch_sign || !fl->k || !fl->Ec || !fl->Ps || !fl->bias || !fl->coef)) return false;
  if (kl && fl && (kl->in_features != fl->in_dim || kl->out_features != fl->out_dim)) return false;
  const int in = kl ? kl->in_features : fl->in_dim, out = kl ? kl->out_features : fl->out_dim;
  return in >= 16 && out >= 16 && out % kOuts == 0 && in % kChMax == 0;
}

// ---- packing (once per parameter version) ------------------------------------------------------
// Cox-de Boor (efficientkan.py:117-131) in fp64 restricted to knot interval m: the cubic bases
// B_{m-3..m} that are non-zero on [g_m, g_{m+1}) at x.
__device__ void bases_on_interval(double x, int m, const float* g, double* N) {
  constexpr int SO = 3;
  for (int r = 0; r < SO + 2; ++r) N[r] = 0.0;
  N[SO] = 1.0;
  for (int k = 1; k <= SO; ++k) {
    double M[SO + 2];
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.0;
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= kNG - 2 - k) {
        const double left = (x - g[j]) / ((double)g[j + k] - g[j]) * N[r];
        const double right = ((double)g[j + k + 1] - x) / ((double)g[j + k + 1] - g[j + 1]) * N[r + 1];
        M[r] = left + right;
      }
    }
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
}

__global__ void wide_pack_kernel(fetode_kanlinear_t kl, fetode_ferro_t fl, WideLayout L, float* __restrict__ plan) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = L.in, out = L.out, K = L.K;
  const float l2 = FETODE_LOG2E;
  if (L.ferro && t < (int64_t)out * in * K) {
    const int o = (int)(t / ((int64_t)in * K)), r = (int)(t % ((int64_t)in * K)), i = r / K, k = r % K;
    const int src = (i * out + o) * K + k;  // reference layout (in, out, K)
    const float kk = fl.k[src], Ec = fl.Ec[src], Ps = fl.Ps[src], co = fl.coef[src];
    const float gec = L.gsl2e * Ec;
    const float k2 = 2.0f * l2 * kk;
    float* d = plan + L.fe4 + 4 * t;
    d[0] = ex2(gec);
    d[1] = k2;
    d[2] = k2 * Ec;
#if WIDE_FOLD
    d[3] = -2.0f * (co * Ps);
#else
    d[3] = co * Ps;
#endif
    plan[L.gec + t] = gec;
  }
  if (L.ferro && t < (int64_t)out * in) {
    const int o = (int)(t / in), i = (int)(t % in);
    float f = 0.f;
    for (int k = 0; k < K; ++k) f = fabsf(L.gs * fl.Ec[(i * out + o) * K + k]) > kWideFactorLimit ? 1.0f : f;
    plan[L.dflag + t] = f;
  }
  if (L.kan && t < (int64_t)in * kWF * out) {
    const int o = (int)(t % out), f = (int)((t / out) % kWF), i = (int)(t / ((int64_t)out * kWF));
    float v = 0.f;
    if (f == 0) {
      v = kl.base_weight[(int64_t)o * in + i];
    } else if (f <= kNS) {
      const float sc = kl.spline_scaler ? kl.spline_scaler[(int64_t)o * in + i] : 1.0f;
      v = kl.spline_weight[((int64_t)o * in + i) * kNS + (f - 1)] * sc;
    } else if (f <= kNS + kNB) {
      const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      // phi = 2 sigma(a (x - b)) (efficientkan.py:24): the 2 lives in the weight
      v = 2.0f * ((kl.logistic_weight[(int64_t)o * (in * kNB) + i * kNB + (f - 1 - kNS)] * kl.scale_logistic) * ls);
    }
    plan[L.wp + t] = v;
  }
  if (L.kan && t < (int64_t)in * kNB) {
    const float a = kl.logistic_a[t], b = kl.logistic_b[t];
    plan[L.lg + 2 * t + 0] = -a * l2;
    plan[L.lg + 2 * t + 1] = (a * b) * l2;
  }
  if (L.kan && t < (int64_t)in * 64) {  // the per-input block the layer tile stages per chunk
    const int i = (int)(t / 64), q = (int)(t % 64);
    const float* g = kl.grid + (int64_t)i * kNG;
    float v = 0.f;
    if (q < kNG) v = g[q];
    else if (q < 2 * kNG - 1) v = 1.0f / (g[q - kNG + 1] - g[q - kNG]);
    else if (q >= 24 && q < 24 + 2 * kNB) {
      const int j = (q - 24) >> 1;
      const float a = kl.logistic_a[(int64_t)i * kNB + j], b = kl.logistic_b[(int64_t)i * kNB + j];
      v = (q & 1) ? (a * b) * l2 : -a * l2;
    } else if (q >= 44 && q < 54) {
      v = 1.0f / (g[q - 44 + 2] - g[q - 44]);
    } else if (q >= 54 && q < 63) {
      v = 1.0f / (g[q - 54 + 3] - g[q - 54]);
    }
    plan[L.par + t] = v;
  }
  if (L.kan && t < (int64_t)in * kNG) {
    const int i = (int)(t / kNG), j = (int)(t % kNG);
    const float* g = kl.grid + (int64_t)i * kNG;
    plan[L.knots + t] = g[j];
    if (j < kNG - 1) plan[L.rh + (int64_t)i * (kNG - 1) + j] = 1.0f / (g[j + 1] - g[j]);
  }
}

// basis table: thread per (input i, knot interval m, basis c): B_c on [g_m, g_{m+1}) as a cubic
// in u = (x - g_m) / (g_{m+1} - g_m), fitted in fp64 through u = 0, 1/3, 2/3, 1 (exact: each basis
// is a cubic on the interval); m = 11 (outside the grid) and bases not supported there: zero
__global__ void wide_basis_kernel(fetode_kanlinear_t kl, WideLayout L, float* __restrict__ plan) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!L.kan || t >= (int64_t)L.in * kNG * kNS) return;
  const int c = (int)(t % kNS), m = (int)((t / kNS) % kNG), i = (int)(t / (kNS * kNG));
  const float* g = kl.grid + (int64_t)i * kNG;
  const int r = c - m + 3;  // slot of basis c among the interval's B_{m-3..m}
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  if (m < kNG - 1 && r >= 0 && r <= 3) {
    const double h = (double)g[m + 1] - g[m];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double N[5];
      bases_on_interval(g[m] + h * (q / 3.0), m, g, N);
      const double v = r == 0 ? N[0] : r == 1 ? N[1] : r == 2 ? N[2] : N[3];
      if (q == 0) v0 = v;
      else if (q == 1) v1 = v;
      else if (q == 2) v2 = v;
      else v3 = v;
    }
  }
  float* d = plan + L.bt + t * 4;
  d[0] = (float)v0;
  d[1] = (float)((-11.0 * v0 + 18.0 * v1 - 9.0 * v2 + 2.0 * v3) / 2.0);
  d[2] = (float)(9.0 * (2.0 * v0 - 5.0 * v1 + 4.0 * v2 - v3) / 2.0);
  d[3] = (float)(9.0 * (-v0 + 3.0 * v1 - 3.0 * v2 + v3) / 2.0);
}

// per-output constant sum_{i,k} coef * bias: one wave per output, fixed order
__global__ void wide_const_kernel(fetode_ferro_t fl, WideLayout L, float* __restrict__ plan) {
  const int o = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  if (L.ferro)
    for (int p = lane; p < L.in * L.K; p += 64) {
      const int i = p / L.K, k = p % L.K;
      const int src = (i * L.out + o) * L.K + k;
#if WIDE_FOLD
      s += fl.coef[src] * fl.bias[src] + fl.coef[src] * fl.Ps[src];
#else
      s += fl.coef[src] * fl.bias[src];
#endif
    }
  for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) plan[L.fconst + o] = s;
}

struct WideArgs {
  const float* plan;
  WideLayout L;
  const float* x;
  const float* prev;
  const float* grid;  // (in, 12) knots
  int64_t B;
  int reinit;
  int nslice;  // input slices (wide_slices): blockIdx.z takes 1 / nslice of the inputs
  float* out;
  // resident solver only (wide_tile<.., RES = true>): the layer input / its hysteresis memory as the
  // fixed-order sum ((s0 + s1) + s2) + .. of nxs / nps input-sliced partial slabs, xss / pss floats apart
  int nxs, nps;
  int64_t xss, pss;
};

// Input slices of a layer launch: with few (row, output) tiles the CUs are short of waves (and at
// small batches one tile's walk over all inputs is the whole latency), so the inputs are split over
// up to 8 workgroups per tile, each walking in / nslice of them (whole chunks of 8).  The partial
// sums meet in a fixed order — slab 0 + slab 1 (+ slab 2 ..), left to right — in both the per-layer
// launch (two slices: vector atomics into a zeroed out, 0 + a + b; more: slabs + wide_slab_sum_kernel)
// and the resident solver (the consumer sums the slabs), so the two paths agree bit for bit.
constexpr int kMaxSlices = 16;
int wide_slices(int64_t wgs, int in) {
  int S = 1;
  while (S < kMaxSlices && wgs * S <= 2 * 256 && (in / (2 * S)) % kChMax == 0 && in % (2 * S) == 0) S *= 2;
  return S;
}

// One slice stores; two add into a zeroed out with vector atomics: 0 + a + b in either order is the
// same fp32 value (addition commutes), so the split stays bitwise deterministic.
__device__ __forceinline__ void store_out(float* p, float v, int nslice) {
  if (nslice != 2) *p = v;  // whole, or this slice's own slab
  else atomicAdd(p, v);
}

// out = ((s0 + s1) + s2) + .. of the slabs (slice s at s * n)
__global__ void wide_slab_sum_kernel(const float* __restrict__ slab, int S, int64_t n, float* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float v = slab[j];
  for (int s = 1; s < S; ++s) v = v + slab[s * n + j];
  out[j] = v;
}

// grow-only per-device scratch for the slabs of > 2 input slices (the per-layer launch's ABI has no
// workspace argument); reallocated outside any stream work only when a larger batch first needs it
float* slab_scratch(size_t floats) {
  static float* buf[64] = {};
  static size_t cap[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (cap[dev] < floats) {
    if (buf[dev]) {
      (void)hipDeviceSynchronize();
      (void)hipFree(buf[dev]);
    }
    buf[dev] = nullptr;
    cap[dev] = 0;
    if (hipMalloc(&buf[dev], floats * sizeof(float)) != hipSuccess) return nullptr;
    cap[dev] = floats;
  }
  return buf[dev];
}

// ---- the layer --------------------------------------------------------------------------------
typedef __attribute__((address_space(4))) const float kconst_f;
typedef __attribute__((address_space(4))) const float4 kconst_f4;

// One tile (row block bx, output block by, input slice bz) of the layer.  The per-layer launch
// (wide_layer_kernel) runs one per workgroup; the device-resident dopri5 solver (wide_dopri5_kernel)
// walks every tile of a layer phase with its persistent grid.  RES: the input and the hysteresis
// memory may be the sum of input-sliced partial slabs (nxs / nps), and every output goes through `epi`
// (a write-through store, or the solver's per-element stage combine) instead of store_out.
template <int K, bool KAN, bool FERRO, int kCh, bool RES, class Epi>
__device__ __forceinline__ void wide_tile(const WideArgs& a, const int bx, const int by, const int bz, Epi&& epi) {
  constexpr int kPitch = pitch_of(kCh);
  static_assert(kCh * kRows <= kThreads && (kCh & 1) == 0, "one staging item per thread, even chunks");
  static_assert(!FERRO || K % 2 == 0, "Ferro elements in (k, k+1) pairs");
  // staged per (input, row) at si * kRP + sr: the pitch kRows + 4 puts a half-wave's 8 inputs x 4 rows
  // on 32 different banks (at kRows the 8 inputs of a row shared one: 8-way, round 6)
  constexpr int kRP = kRows + 4;
  __shared__ float s_x[kCh * kRP], s_w[kCh * kRP], s_e[kCh * kRP];
  __shared__ float s_dfl[kOuts * kCh];
  // the chunk's per-input KAN parameters (knots | 1 / spans | logistic (-a log2e, a b log2e)), staged
  // one chunk ahead and double-buffered by chunk parity: the staging items read them from LDS instead
  // of a dependent L2 round trip per item before the basis-table gather (the KANLinear part of the
  // layer 98 -> 52 us with the loads taken away entirely)
  // In LDS each input's block sits at a pitch of kParL = 68 floats: at 64 (one 256-byte bank row) the
  // 8 inputs a half-wave reads at once all hit the same bank — the layer's LDS was 65 % conflict
  // cycles (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r06_lds_wide.txt)
  constexpr int kPar = 64, kParL = 68, kPK = 0, kPR = 12, kPL = 24, kP2 = 44, kP3 = 54;
  __shared__ __attribute__((aligned(16))) float s_par[KAN ? 2 : 1][KAN ? kCh * kParL : 1];
  // KAN features of the chunk (MFMA A operand); the epilogue reuses the space for the Ferro sums
  // and the second K-half of the MFMA tile
  constexpr int kPhi = KAN ? kRows * kPitch : 0, kFer = 2 * kRows * (kOuts + 1);
  __shared__ __attribute__((aligned(16))) float s_phi[kPhi > kFer ? kPhi : kFer];
  float* s_fer = s_phi;
  float* s_kc = s_phi + kRows * (kOuts + 1);
  const WideLayout& L = a.L;
  const int in = L.in, out = L.out;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b0 = (int64_t)bx * kRows;
  const int o0 = by * kOuts;
  const float* __restrict__ plan = a.plan;
  const float gsl2e = L.gsl2e, wc = L.wc, l2 = FETODE_LOG2E;

  float facc[kJ];  // Ferro: row = lane, output o0 + kJ w + j
#pragma unroll
  for (int j = 0; j < kJ; ++j) facc[j] = 0.f;
  f32x4 kacc0 = {0.f, 0.f, 0.f, 0.f}, kacc1 = {0.f, 0.f, 0.f, 0.f};  // KAN: rows 16 (w % 4) + 4 (lane >> 4) + v
  const int kr = lane & 15, kq = lane >> 4, rt = w & 3, kh = w >> 2;

  // staging item of this thread: row sr, chunk input si
  const int sr = tid / kCh, si = tid % kCh;
  const int64_t sb = b0 + sr;
  const bool stager = tid < kCh * kRows;
  const bool slive = stager && sb < a.B;

  // the staging item's x / prev_x, loaded one chunk ahead (their HBM latency hides under the
  // previous chunk's work)
  const int ibeg = bz * (in / a.nslice), iend = ibeg + in / a.nslice;
  auto ldx = [&](int64_t i) -> float {
    float v = a.x[i];
    if constexpr (RES)
      for (int s = 1; s < a.nxs; ++s) v = v + a.x[i + s * a.xss];   // slab 0 + slab 1 + ..: the launch path's order
    return v;
  };
  auto ldp = [&](int64_t i) -> float {
    float v = a.prev[i];
    if constexpr (RES)
      for (int s = 1; s < a.nps; ++s) v = v + a.prev[i + s * a.pss];
    return v;
  };
  float xn = slive ? ldx(sb * in + ibeg + si) : 0.f;
  float pn = (FERRO && slive && !a.reinit) ? ldp(sb * in + ibeg + si) : 0.f;
  // thread t < kCh * kPar loads word t of a chunk's parameter block (issued at the chunk's start,
  // written to LDS just before its staging barrier: the load's latency hides under the staging)
  const bool pld = KAN && tid < kCh * kPar;
  auto ld_par = [&](int i0c) -> float {   // the plan's per-input blocks are contiguous: word tid of the chunk
    return (pld && i0c < iend) ? plan[L.par + (int64_t)i0c * kPar + tid] : 0.f;
  };
  if constexpr (KAN) {
    const float p0 = ld_par(ibeg);
    if (pld) s_par[0][(tid / kPar) * kParL + tid % kPar] = p0;  // read after the first chunk's barrier
  }
  int pbuf = 0;
  for (int i0 = ibeg; i0 < iend; i0 += kCh) {
    const float x = xn, pvl = pn;
    if (i0 + kCh < iend) {
      xn = slive ? ldx(sb * in + i0 + kCh + si) : 0.f;
      pn = (FERRO && slive && !a.reinit) ? ldp(sb * in + i0 + kCh + si) : 0.f;
    }
    __syncthreads();  // the previous chunk is consumed
    // chunk i0 + kCh's parameters: loaded now, stored into the other buffer before the staging
    // barrier, read after the next chunk's barrier
    float parn = 0.f;
    if constexpr (KAN) parn = ld_par(i0 + kCh);
    if constexpr (FERRO) {
      const float pv = a.reinit ? x : pvl;
      if (stager) {
      // is_moving_up = sigmoid(gate_slope (x - prev_x)) (ferro_class.py:387), w = wc (1 - up)
      const float up = rcp(1.0f + ex2(-gsl2e * (x - pv)));
      s_x[si * kRP + sr] = x;
      s_w[si * kRP + sr] = wc * (1.0f - up);
      s_e[si * kRP + sr] = ex2(gsl2e * x);
      }
      if (tid < kOuts * kCh) s_dfl[tid] = plan[L.dflag + (int64_t)(o0 + tid / kCh) * in + i0 + tid % kCh];
    }
    if (KAN && stager) {
      const float sil = x * rcp(1.0f + ex2(-x * l2));  // SiLU (efficientkan.py:166)
      // cubic B-spline bases (efficientkan.py:117-131): the knot interval m by the half-open order-0
      // indicator, then the Cox-de Boor recursion restricted to the interval's triangle (the four
      // bases B_{m-3..m} that can be non-zero) on the staged knots and reciprocal spans, all from LDS
      // (no per-item gather of fitted tables: the layer's staging waited on those L2 round trips)
      const float* P = &s_par[KAN ? pbuf : 0][si * kParL];
      const float* g = P + kPK;
      int m = -1;
#pragma unroll
      for (int j = 0; j < kNG; ++j) m += (x >= g[j]) ? 1 : 0;
      const bool fin = __builtin_isfinite(x);
      const bool ing = fin && (unsigned)m < (unsigned)(kNG - 1);  // inside the grid
      const int mc = ing ? m : 0;
      // knots / spans outside the grid only enter bases B_{<0} or B_{>7}, which are dropped (clamped reads)
      auto G = [&](int j) { return g[j < 0 ? 0 : (j > kNG - 1 ? kNG - 1 : j)]; };
      auto R = [&](int off, int j, int n) { return P[off + (j < 0 ? 0 : (j > n - 1 ? n - 1 : j))]; };
      const float gm = G(mc), gm1 = G(mc + 1), gmm1 = G(mc - 1), gm2 = G(mc + 2), gmm2 = G(mc - 2), gm3 = G(mc + 3);
      const float r1 = P[kPR + mc];
      const float n10 = (gm1 - x) * r1, n11 = (x - gm) * r1;                        // B_{m-1,1}, B_{m,1}
      const float t0 = n10 * R(kP2, mc - 1, 10), t1 = n11 * R(kP2, mc, 10);
      const float n20 = (gm1 - x) * t0, n21 = (x - gmm1) * t0 + (gm2 - x) * t1, n22 = (x - gm) * t1;
      const float s0 = n20 * R(kP3, mc - 2, 9), s1 = n21 * R(kP3, mc - 1, 9), s2 = n22 * R(kP3, mc, 9);
      const float nb[4] = {(gm1 - x) * s0, (x - gmm2) * s0 + (gm2 - x) * s1, (x - gmm1) * s1 + (gm3 - x) * s2,
                           (x - gm) * s2};                                                // B_{m-3..m, 3}
      const float z = fin ? 0.f : __builtin_nanf("");  // non-finite x: NaN bases, as (x - g) / d * B
      float* d = &s_phi[sr * kPitch + si * kWF];
      *reinterpret_cast<float2*>(d) = make_float2(sil, z);
#pragma unroll
      for (int q = 2; q < kNS; q += 2) *reinterpret_cast<float2*>(d + q) = make_float2(z, z);
      const float f8 = z;  // (B_7's slot is written with phi_0 below; the interval's bases land after)
      // the logistic bases straight into the row, their parameters from LDS a pair at a time (few live
      // VGPRs: the whole block hoisted at once spilled the fused layer)
      const float4* lg = reinterpret_cast<const float4*>(P + kPL);
      float prev = f8;  // B_7 pairs with phi_0: the row is written as aligned float2s
#pragma unroll 1
      for (int j = 0; j < kNB; j += 2) {
        const float4 ab = lg[j / 2];  // (-a log2e, a b log2e) of bases j, j + 1
        const float p0 = rcp(1.0f + ex2(ffma(ab.x, x, ab.y))), p1 = rcp(1.0f + ex2(ffma(ab.z, x, ab.w)));
        *reinterpret_cast<float2*>(d + kNS + j) = make_float2(prev, p0);
        prev = p1;
      }
      *reinterpret_cast<float2*>(d + kNS + kNB) = make_float2(prev, 0.f);
      if (ing) {  // the interval's bases over the zeros (same thread, in order)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = m - 3 + r;
          if (c >= 0 && c < kNS) d[1 + c] = nb[r];
        }
      }
    }
    if constexpr (KAN) {
      if (pld) s_par[pbuf ^ 1][(tid / kPar) * kParL + tid % kPar] = parn;
    }
    __syncthreads();
    if constexpr (KAN) pbuf ^= 1;
    // KAN weights of this wave's chunk inputs (ii = 2 q + kh) for the MFMA B operand (L2-resident;
    // issued here so their latency hides under the Ferro work, and not live across the staging)
    float wb[KAN ? kCh / 2 * 5 : 1];
    if constexpr (KAN) {
#pragma unroll
      for (int q = 0; q < kCh / 2; ++q)
#pragma unroll
        for (int s = 0; s < 5; ++s)
          wb[q * 5 + s] = plan[L.wp + ((int64_t)(i0 + 2 * q + kh) * kWF + 4 * s + kq) * out + o0 + kr];
    }
    if constexpr (FERRO) {
      constexpr int kIU = K <= 10 ? 2 : 1;  // two inputs in flight at K = 10; K = 12 would spill
#pragma unroll kIU
      for (int ii = 0; ii < kCh; ++ii) {
        const int i = i0 + ii;
        const float xv = s_x[ii * kRP + lane], wg = s_w[ii * kRP + lane], e = s_e[ii * kRP + lane];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          const int jo = kJ * w + j;
          // the element constants are wave-uniform: scalar loads (s_load, SGPR operands) — through
          // LDS they cost a ds_read_b128 per element (Ferro alone 270 -> 230 us at 64 -> 128)
          // (read through the constant address space: the plan is never written during a launch, so the
          // loads stay scalar whatever precedes them — the resident solver's tile loop, the chunk
          // loop's vector loads of the staged parameters)
          const float4* par = reinterpret_cast<const float4*>(plan + L.fe4) + ((int64_t)(o0 + jo) * in + i) * K;
          auto pk = [&](int k) -> float4 {
#if defined(__HIP_DEVICE_COMPILE__)
            const kconst_f4* pc = (const kconst_f4*)(uintptr_t)(par + k);
            return make_float4(pc->x, pc->y, pc->z, pc->w);
#else
            return par[k];
#endif
          };
          float acc = 0.f;
          if (s_dfl[jo * kCh + ii] == 0.f) {  // wave-uniform
            // elements (k, k+1) in the two halves of packed-fp32 VALU ops (v_pk_fma / mul / add:
            // 3.5 instead of 7 non-transcendental issues per element); even and odd k sum apart
            f2 acc2 = splat(0.0f);
#pragma unroll
            for (int k = 0; k < K; k += 2) {
              const float4 p0 = pk(k), p1 = pk(k + 1);  // {P, k2, k2Ec, cps}, same address on every lane
              const f2 sg = rcpx2(pfma(splat(e), f2{p0.x, p1.x}, splat(1.0f)));
              const f2 mm = pfma(splat(wg), sg, splat(1.0f));
              const f2 z = pfma(f2{p0.z, p1.z}, mm, f2{p0.y, p1.y} * splat(xv));
#if WIDE_FOLD
              // coef Ps tanh z = coef Ps - 2 coef Ps / (1 + 2^z): the constant part lives in fconst
              acc2 = pfma(f2{p0.w, p1.w}, rcpx2(ex2x2(z) + splat(1.0f)), acc2);
#else
              // coef Ps tanh z, tanh z = 1 - 2 / (1 + 2^z): the terms keep the size of the
              // reference's (round 6: the fold above summed terms of size coef Ps whatever tanh was,
              // and over the 380 stateful steps of the ETT forecast its cancellation cost ~4x the
              // reference's own fp32 error)
              acc2 = pfma(f2{p0.w, p1.w}, pfma(rcpx2(ex2x2(z) + splat(1.0f)), splat(-2.0f), splat(1.0f)), acc2);
#endif
            }
            acc = acc2.x + acc2.y;
          } else {
            const float* gec = plan + L.gec + ((int64_t)(o0 + jo) * in + i) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const float4 p = pk(k);
              const float sg = rcp(1.0f + ex2(ffma(gsl2e, xv, gec[k])));
              const float mm = ffma(wg, sg, 1.0f);
              const float z = ffma(p.z, mm, p.y * xv);
#if WIDE_FOLD
              acc = ffma(p.w, rcp(ex2(z) + 1.0f), acc);
#else
              acc = ffma(p.w, ffma(rcp(ex2(z) + 1.0f), -2.0f, 1.0f), acc);
#endif
            }
          }
          facc[j] += acc;  // K bases of one input first, then inputs (the reference's two-level sum)
        }
      }
    }
    if constexpr (KAN) {
      const float* arow = &s_phi[(16 * rt + kr) * kPitch + kq];
#pragma unroll
      for (int q = 0; q < kCh / 2; ++q) {
        const int ii = 2 * q + kh;
#pragma unroll
        for (int s = 0; s < 5; ++s) {
          if (q & 1) kacc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[ii * kWF + 4 * s], wb[q * 5 + s], kacc1, 0, 0, 0);
          else kacc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[ii * kWF + 4 * s], wb[q * 5 + s], kacc0, 0, 0, 0);
        }
      }
    }
  }
  // epilogue: the Ferro sums (+ sum coef bias) and the second K-half meet the KAN tile in LDS
  __syncthreads();
  if constexpr (FERRO) {
#pragma unroll
    for (int j = 0; j < kJ; ++j)
      s_fer[lane * (kOuts + 1) + kJ * w + j] = facc[j] + (bz == 0 ? plan[L.fconst + o0 + kJ * w + j] : 0.f);
  }
  if constexpr (KAN) {
    if (kh == 1)
#pragma unroll
      for (int v = 0; v < 4; ++v) s_kc[(16 * rt + 4 * kq + v) * (kOuts + 1) + kr] = kacc0[v] + kacc1[v];
  }
  __syncthreads();
  if constexpr (KAN) {
    if (kh == 0)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int r = 16 * rt + 4 * kq + v;
        const int64_t b = b0 + r;
        const float kv = (kacc0[v] + kacc1[v]) + s_kc[r * (kOuts + 1) + kr];
        if (b < a.B) epi(b, o0 + kr, FERRO ? kv + s_fer[r * (kOuts + 1) + kr] : kv);
      }
  } else {
    for (int t = tid; t < kRows * kOuts; t += kThreads) {
      const int r = t / kOuts, c = t % kOuts;
      const int64_t b = b0 + r;
      if (b < a.B) epi(b, o0 + c, s_fer[r * (kOuts + 1) + c]);
    }
  }
}

template <int K, bool KAN, bool FERRO, int kCh>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6))) void wide_layer_kernel(WideArgs a) {
  const int out = a.L.out, ns = a.nslice;
  float* const o = a.out + (ns > 2 ? (int64_t)blockIdx.z * a.B * out : 0);
  wide_tile<K, KAN, FERRO, kCh, false>(a, blockIdx.x, blockIdx.y, blockIdx.z,
                                       [&](int64_t b, int c, float v) { store_out(&o[b * out + c], v, ns); });
}

typedef void (*wide_fn)(WideArgs);
template <int CH>
wide_fn pick_ch(int K, bool kan, bool ferro) {
  if (kan && !ferro) return wide_layer_kernel<10, true, false, CH>;
  if (K == 12) return kan ? wide_layer_kernel<12, true, true, CH> : wide_layer_kernel<12, false, true, CH>;
  return kan ? wide_layer_kernel<10, true, true, CH> : wide_layer_kernel<10, false, true, CH>;
}
// inputs per staged chunk: 8 (fewer barriers) or 4 (less LDS, more resident workgroups);
// FETODE_WIDE_CH picks (tuning knob, default 8)
wide_fn pick(int K, bool kan, bool ferro) {
  static const int ch = [] {
    const char* e = getenv("FETODE_WIDE_CH");
    return e && atoi(e) == 4 ? 4 : 8;
  }();
  return ch == 4 ? pick_ch<4>(K, kan, ferro) : pick_ch<8>(K, kan, ferro);
}



// ---- the Ferro layer's VJP at production widths (ferro_class.py:368-414 under autograd) ----------
// d loss / d x and the five parameter gradients of FerroelectricBasis (constant branch_sign) from the
// output adjoint g, in one pass over the element evaluations.  With branch_sign = 1 (never written,
// ferro_class.py:366) the crossing gate cp carries a zero coefficient and
//   cn = sigma(gs (-x - Ec)) = 1 / (1 + e^{gs x} P),  m = 1 + wc (1 - up) cn,   wc = -2 (1 - alpha)
//   th = tanh(k (x + Ec m)),  out = sum coef (Ps th + bias)
// with up = sigma(gs (x - prev)) (prev detached, ferro_class.py:381-387), so per element
//   gP = g coef;  gcoef = g P;  gPs = gP th;  gbias = gP;  gz = gP Ps (1 - th^2);  gk = gz (x + Ec m)
//   (1 - th^2 = 4 r (1 - r) with th = 1 - 2 r: no cancellation where th saturates)
//   gsh = gz k;  gm = gsh Ec;  dcn = gs cn (1 - cn)
//   gx += gsh - gm wc ((1 - up) dcn + cn gs up (1 - up));   gEc = gsh m - gm wc (1 - up) dcn.
// Mapping: a wave = 4 rows x (3 outputs x 5 pairs) at K = 10 (2 x 6 at K = 12): lane (q, o, kp) of
// 16-lane quarter q evaluates elements (i, o, 2kp), (i, o, 2kp + 1) of row b + q on packed fp32, so
// the parameter sums stay in the lane's registers over the whole row range and d/dx of a row is one
// 16-lane DPP row sum.  A wave walks OGW output groups for its input i and rows [r0, r1).  Partials:
// d/dx per (output-group block, row, input) and the parameter sums per row segment, both reduced in
// a fixed order afterwards (run-to-run identical).
// output groups per wave: 2 (default; 4 holds ~220 VGPRs, two waves per SIMD); FETODE_FERRO_BWD_OGW
// = 1 | 2 | 4 picks (tuning knob)
int ferro_bwd_ogw() {
  static const int v = [] {
    const char* e = getenv("FETODE_FERRO_BWD_OGW");
    const int x = e ? atoi(e) : 2;
    return x == 1 || x == 4 ? x : 2;
  }();
  return v;
}

struct WideFerroBwdArgs {
  const float* plan;
  WideLayout L;
  const float* k, *Ec, *Ps, *bias, *coef;  // reference layout (in, out, K)
  const float4* U;    // (B, in): {x, e = 2^{gs log2e x}, 1 - up, gs up (1 - up)}
  const float* g;     // (B, out)
  int64_t B;
  int n_og, n_ogb, rs, seg;   // output groups (of OPG outputs), group blocks (of ferro_bwd_ogw()), row segments, rows/segment
  float* gxp;         // (n_ogb, B, in)
  float* pp;          // (rs, in, out, K, 5)
};

__global__ void wide_ferro_prep_kernel(const float* __restrict__ x, const float* __restrict__ prev, int reinit,
                                       int64_t n, float gsl2e, float gs, float4* __restrict__ U) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float xv = x[t], pv = reinit ? xv : prev[t];
  const float up = rcp(1.0f + ex2(-gsl2e * (xv - pv)));   // the forward's gate (wide_layer_kernel)
  const float omu = 1.0f - up;
  U[t] = make_float4(xv, ex2(gsl2e * xv), omu, gs * up * omu);
}

template <int K, int kBwdOGW>
__global__ __launch_bounds__(256) void wide_ferro_bwd_kernel(WideFerroBwdArgs a) {
  constexpr int KP = K / 2, OPG = 16 / KP;   // pairs per output, outputs per 16-lane group (3 | 2)
  const WideLayout& L = a.L;
  const int in = L.in, out = L.out;
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ogb = (int)(task % a.n_ogb);
  const int64_t rest = task / a.n_ogb;
  const int i = (int)(rest % in), sgi = (int)(rest / in);
  if (sgi >= a.rs) return;
  const int64_t r0 = (int64_t)sgi * a.seg, r1 = r0 + a.seg < a.B ? r0 + a.seg : a.B;
  const bool act = c < OPG * KP;
  const int ol = act ? c / KP : 0, kp = act ? c % KP : 0;
  const float gs = L.gs, wc = L.wc, gsl2e = L.gsl2e;
  // this lane's element pairs in the kBwdOGW output groups of the block.  The parameter gradients are
  // linear in three per-element sums and one per-output sum (as the LV sweep's):
  //   A = sum g th,  C = sum g r (1 - r) sh,  E = sum gsh (m + Ec dm/dEc),  G = sum g
  //   dPs = coef A, dbias = coef G, dcoef = Ps A + bias G, dk = 4 coef Ps C, dEc = E
  // with gsh = g coef Ps 4 r (1 - r) k = g r (1 - r) cPk4 (1 - th^2 = 4 r (1 - r), th = 1 - 2 r:
  // no cancellation where th saturates), so the row loop carries no coef / Ps / bias products.
  f2 Pf[kBwdOGW], k2[kBwdOGW], Ecv[kBwdOGW], cPk4[kBwdOGW], gec[kBwdOGW];
  int oo[kBwdOGW];
  bool ok[kBwdOGW], dir[kBwdOGW];
  f2 sA[kBwdOGW], sC[kBwdOGW], sE[kBwdOGW];
  float sG[kBwdOGW];
#pragma unroll
  for (int j = 0; j < kBwdOGW; ++j) {
    const int og = ogb * kBwdOGW + j;
    const int o = og * OPG + ol;
    ok[j] = act && og < a.n_og && o < out;
    oo[j] = ok[j] ? o : 0;
    const int64_t e0 = ((int64_t)i * out + oo[j]) * K + 2 * kp;                 // reference layout
    const int64_t p0 = ((int64_t)oo[j] * in + i) * K + 2 * kp;                   // plan layout (o, i, k)
    const float4 a0 = ok[j] ? reinterpret_cast<const float4*>(a.plan + L.fe4)[p0] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 a1 = ok[j] ? reinterpret_cast<const float4*>(a.plan + L.fe4)[p0 + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    Pf[j] = f2{a0.x, a1.x};
    k2[j] = f2{a0.y, a1.y};
    Ecv[j] = ok[j] ? f2{a.Ec[e0], a.Ec[e0 + 1]} : splat(0.f);
    cPk4[j] = ok[j] ? f2{4.0f * a.coef[e0] * a.Ps[e0] * a.k[e0], 4.0f * a.coef[e0 + 1] * a.Ps[e0 + 1] * a.k[e0 + 1]}
                    : splat(0.f);
    gec[j] = ok[j] ? f2{a.plan[L.gec + p0], a.plan[L.gec + p0 + 1]} : splat(0.f);
    dir[j] = ok[j] && a.plan[L.dflag + (int64_t)oo[j] * in + i] != 0.f;
    sA[j] = sC[j] = sE[j] = splat(0.f);
    sG[j] = 0.f;
  }
  bool anydir = false;
#pragma unroll
  for (int j = 0; j < kBwdOGW; ++j) anydir |= __builtin_amdgcn_ballot_w64(dir[j]) != 0;
  // the next row group's U and g are loaded while this one computes (each row group's loads were
  // a full global-memory round trip on the wave's chain); out-of-range rows read row r0 (valid).
  // Row pointers advance by 4 rows per step (the 64-bit row products per step were ~20 of the
  // loop's ~150 instructions)
  const float4* const u_r0 = a.U + r0 * in + i;
  const float* const g_r0 = a.g + r0 * out;
  const int64_t du = 4 * (int64_t)in, dg = 4 * (int64_t)out;
  const float4* up = r0 + q < r1 ? u_r0 + q * (int64_t)in : u_r0;
  const float* gp = r0 + q < r1 ? g_r0 + q * (int64_t)out : g_r0;
  float* gxrow = a.gxp + (int64_t)ogb * a.B * in + (r0 + q) * in + i;
  auto ld = [&](float4& u, float* go) __attribute__((always_inline)) {
    u = *up;
#pragma unroll
    for (int j = 0; j < kBwdOGW; ++j) go[j] = gp[oo[j]];
  };
  float4 un;
  float gn[kBwdOGW];
  ld(un, gn);
  for (int64_t b0 = r0; b0 < r1; b0 += 4, gxrow += du) {
    const int64_t b = b0 + q;
    const bool live = b < r1;
    const float4 u = live ? un : make_float4(0.f, 0.f, 0.f, 0.f);
    float gcur[kBwdOGW];
#pragma unroll
    for (int j = 0; j < kBwdOGW; ++j) gcur[j] = gn[j];
    const bool nx = b + 4 < r1;
    up = nx ? up + du : u_r0;
    gp = nx ? gp + dg : g_r0;
    ld(un, gn);
    const float xv = u.x, e = u.y, omu = u.z, dup = u.w;
    // per row: m = 1 + wco cn; dm/dx = a1 cn + a2 cn (1 - cn); dm/dEc = a2 cn (1 - cn)
    const float wco = wc * omu, a1 = -wc * dup, a2 = -gs * wco;
    f2 dxacc = splat(0.0f);
#pragma unroll
    for (int j = 0; j < kBwdOGW; ++j) {
      const float go = (live && ok[j]) ? gcur[j] : 0.f;
      f2 cn;
      if (anydir && dir[j]) cn = rcpx2(ex2x2(pfma(splat(gsl2e), splat(xv), gec[j])) + splat(1.0f));
      else cn = rcpx2(pfma(splat(e), Pf[j], splat(1.0f)));
      const f2 m = pfma(splat(wco), cn, splat(1.0f));
      const f2 sh = pfma(Ecv[j], m, splat(xv));                     // x + Ec m
      const f2 r = rcpx2(ex2x2(k2[j] * sh) + splat(1.0f));          // 2^{2 log2e k sh}
      const f2 th = pfma(splat(-2.0f), r, splat(1.0f));             // tanh = 1 - 2 / (1 + e^{2 k sh})
      sA[j] = pfma(splat(go), th, sA[j]);
      sG[j] += go;
      const f2 w = splat(go) * (r * (splat(1.0f) - r));             // g (1 - th^2) / 4
      sC[j] = pfma(w, sh, sC[j]);
      const f2 gsh = w * cPk4[j];
      const f2 t = splat(a2) * (cn * (splat(1.0f) - cn));           // dm/dEc
      sE[j] = pfma(gsh, pfma(Ecv[j], t, m), sE[j]);
      const f2 dq = pfma(Ecv[j], pfma(splat(a1), cn, t), splat(1.0f));   // d sh/dx = 1 + Ec dm/dx
      dxacc = ok[j] ? pfma(gsh, dq, dxacc) : dxacc;                 // idle lanes: e = inf times P = 0 is NaN
    }
    const float row = row_sum16(dxacc.x + dxacc.y);
    if (c == 0 && live) *gxrow = row;
  }
  // the four row quarters hold the same elements: quarters (0 + 2) + (1 + 3) onto lanes 0..15, then
  // the sums -> this row segment's parameter-gradient partials (reference layout)
  float* pp = a.pp + (int64_t)sgi * in * out * K * 5;
  auto qsum = [&](float p) __attribute__((always_inline)) {
    float qq = p;
    permlane32_swap(p, qq);
    float s2 = p + qq, s3 = s2;
    permlane16_swap(s2, s3);
    return s2 + s3;
  };
#pragma unroll
  for (int j = 0; j < kBwdOGW; ++j) {
    const float G = qsum(sG[j]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float A = qsum(h ? sA[j].y : sA[j].x), C = qsum(h ? sC[j].y : sC[j].x), E = qsum(h ? sE[j].y : sE[j].x);
      if (lane < 16 && ok[j]) {
        const int64_t el = ((int64_t)i * out + oo[j]) * K + 2 * kp + h;
        const float co = a.coef[el], ps = a.Ps[el], bi = a.bias[el];
        float* d = pp + el * 5;
        d[0] = 4.0f * co * ps * C;   // k
        d[1] = E;                    // Ec
        d[2] = co * A;               // Ps
        d[3] = co * G;               // bias
        d[4] = ps * A + bi * G;      // coef
      }
    }
  }
}

// d/dx: the output-group blocks in order (+ the existing gx when accumulating); parameters: the row
// segments in order, written in the reference layout (+ accumulate)
__global__ void wide_ferro_gx_reduce_kernel(const float* __restrict__ gxp, int n_ogb, int64_t n, float* __restrict__ gx,
                                            int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float s = 0.f;
  for (int j = 0; j < n_ogb; ++j) s += gxp[(int64_t)j * n + t];
  gx[t] = accumulate ? gx[t] + s : s;
}

__global__ void wide_ferro_gp_reduce_kernel(const float* __restrict__ pp, int rs, int64_t ne, fetode_ferro_grad_t gr,
                                            int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ne * 5) return;
  const int64_t e = t / 5;
  const int which = (int)(t % 5);
  float s = 0.f;
  for (int j = 0; j < rs; ++j) s += pp[(int64_t)j * ne * 5 + t];
  float* dst = which == 0 ? gr.k : which == 1 ? gr.Ec : which == 2 ? gr.Ps : which == 3 ? gr.bias : gr.coef;
  if (dst) dst[e] = accumulate ? dst[e] + s : s;
}

struct FerroBwdPlan {
  int n_og, n_ogb, rs, seg;
  int64_t tasks;
};

template <int K, int kBwdOGW>
__global__ __launch_bounds__(256) void wide_ferro_bwd_kernel(WideFerroBwdArgs a);

// resident waves of wide_ferro_bwd_kernel on the device (CUs x 4 waves x blocks per CU), 0 unknown
int ferro_bwd_slots(int K) {
  static int slots[2] = {-1, -1};
  int& v = slots[K == 12 ? 1 : 0];
  if (v < 0) {
    v = 0;
    int dev = 0, n_cu = 0, per = 0;
    const int ogw = ferro_bwd_ogw();
    const void* fn = K == 12 ? (ogw == 1 ? (const void*)wide_ferro_bwd_kernel<12, 1>
                                : ogw == 4 ? (const void*)wide_ferro_bwd_kernel<12, 4> : (const void*)wide_ferro_bwd_kernel<12, 2>)
                             : (ogw == 1 ? (const void*)wide_ferro_bwd_kernel<10, 1>
                                : ogw == 4 ? (const void*)wide_ferro_bwd_kernel<10, 4> : (const void*)wide_ferro_bwd_kernel<10, 2>);
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0) == hipSuccess)
      v = n_cu * per * 4;
  }
  return v;
}

FerroBwdPlan ferro_bwd_plan(int in, int out, int K, int64_t B) {
  FerroBwdPlan p{};
  const int kBwdOGW = ferro_bwd_ogw();
  const int OPG = 16 / (K / 2);
  p.n_og = (out + OPG - 1) / OPG;
  p.n_ogb = (p.n_og + kBwdOGW - 1) / kBwdOGW;
  // row segments.  Every wave walks seg rows, so the kernel takes (waves / resident slots, rounded
  // up) rounds of seg / 4 row steps: rs minimises rounds x (seg / 4 + a per-wave setup of ~16 steps)
  // over segments of >= 64 rows (~8 waves per SIMD, >= 256 rows each, was 3 rounds of 342 rows at
  // the ETT widths for 2.06 rounds of work: 8448 waves on 4096 slots).  FETODE_FERRO_BWD_RS = n
  // fixes it (tuning knob).
  const int64_t base = (int64_t)p.n_ogb * in;
  const int64_t rmax = std::max<int64_t>(1, std::min<int64_t>(64, (B + 63) / 64));
  static const int rs_env = [] {
    const char* e = getenv("FETODE_FERRO_BWD_RS");
    return e ? atoi(e) : 0;
  }();
  int64_t rs = 1;
  const int slots = ferro_bwd_slots(K);
  if (rs_env > 0) {
    rs = std::min<int64_t>(rs_env, (B + 3) / 4);
  } else if (slots > 0) {
    double best = 1e300;
    for (int64_t r = 1; r <= rmax; ++r) {
      const int64_t rounds = (base * r + slots - 1) / slots;
      const double cost = (double)rounds * ((double)((B + r - 1) / r) / 4.0 + 16.0);
      if (cost < best * 0.999) {
        best = cost;
        rs = r;
      }
    }
  } else {
    rs = std::min<int64_t>((8 * 1024 + base - 1) / base, (B + 255) / 256);
  }
  p.rs = (int)(rs > 0 ? rs : 1);
  p.seg = (int)(((B + p.rs - 1) / p.rs + 3) / 4 * 4);
  p.rs = (int)((B + p.seg - 1) / p.seg);
  p.tasks = base * p.rs;
  return p;
}

// ---- the KANLinear VJP at production widths (efficientkan.py:160-182 under autograd) -----------
// With the packed weights Wp (in, 20, out) of the plan and the 20 staged features phi(x) of the
// forward (SiLU, 8 cubic B-spline bases, 10 logistic sigmoids), the layer is out = phi(x) Wp, so
//   gphi = g Wp^T            (B x in*20, K = out)   -> d/dx = sum_f gphi phi'_f, and the logistic
//                                                       a / b sums (sum_b gphi sigma' (x - b), -a ...)
//   dWp  = phi^T g           (in*20 x out, K = B)  -> the parameter gradients by the chain rule of
//                                                       the packing (spline scaler, logistic scales)
// both on v_mfma_f32_16x16x4_f32.  wide_kan_gx_kernel: a wave = 16 rows x 4 inputs (80 feature
// columns; one (row, input) item per lane); A = g rows, B = Wp columns, both straight from global
// memory (L2-resident) with the contraction index permuted so each lane reads 4-float runs
// (o = kg * out/4 + q for lane group kg, k-step q: the MFMA sums over k in any order); gphi meets
// the per-lane features through a wave-private LDS tile.  It also writes phi (B, in*20) for
// wide_kan_gw_kernel: a wave = 16 feature columns x 64 outputs over a row segment.  Partials
// (row segments) add in a fixed order: run-to-run identical.
constexpr int kKF = kWF;   // features per input (the plan's packing, last one zero)

__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct WideKanBwdArgs {
  const float* plan;
  WideLayout L;
  const float* la, *lb;   // logistic a, b (in, NB)
  const float* x, *g;
  int64_t B;
  float* gx;
  int accumulate;
  float* F;       // (B, in * 20) features
  float* abp;     // (n_rg, in, NB, 2) logistic a / b partial sums
  int n_rg, t16;  // row groups, 16-row tiles per group
};

template <int OUT4>
__global__ __launch_bounds__(256) void wide_kan_gx_kernel(WideKanBwdArgs a) {
  constexpr int OUT = 4 * OUT4, kPitch = 4 * kKF + 1;
  __shared__ float s_gp[4][16 * kPitch];
  const WideLayout& L = a.L;
  const int in = L.in, nch = in / 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t task = (int64_t)blockIdx.x * 4 + wv;
  const int c = (int)(task % nch);
  const int rg = (int)(task / nch);
  if (rg >= a.n_rg) return;
  const int kg = lane >> 4, n = lane & 15;
  const int ii = lane >> 4, r = lane & 15, i = c * 4 + ii;   // the lane's (row, input) item
  float* gp = s_gp[wv];
  const float* __restrict__ plan = a.plan;
  const float l2 = FETODE_LOG2E;
  float ga[kNB], gb[kNB];
#pragma unroll
  for (int j = 0; j < kNB; ++j) ga[j] = gb[j] = 0.f;
  const int64_t nt = (a.B + 15) / 16;
  const int64_t t_lo = (int64_t)rg * a.t16, t_hi = t_lo + a.t16 < nt ? t_lo + a.t16 : nt;
  for (int64_t t = t_lo; t < t_hi; ++t) {
    const int64_t b0 = t * 16;
    // gphi (16 rows x 80 columns): A = g rows (row b0 + n, k-group kg), B = Wp columns
    float4 ar[OUT4 / 4];
    {
      const bool ok = b0 + n < a.B;
      const float4* gr = reinterpret_cast<const float4*>(a.g + (b0 + n) * OUT + kg * OUT4);
#pragma unroll
      for (int q = 0; q < OUT4 / 4; ++q) ar[q] = ok ? gr[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int ct = 0; ct < 5; ++ct) {
      const float4* wr = reinterpret_cast<const float4*>(plan + L.wp + ((int64_t)c * 4 * kKF + ct * 16 + n) * OUT + kg * OUT4);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < OUT4 / 4; ++q) {
        const float4 w = wr[q];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[q].x, w.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[q].y, w.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[q].z, w.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[q].w, w.w, acc, 0, 0, 0);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) gp[(4 * kg + v) * kPitch + ct * 16 + n] = acc[v];
    }
    // the lane's item: features and their derivatives (the forward's staging, wide_layer_kernel)
    const int64_t b = b0 + r;
    const bool live = b < a.B;
    const float xv = live ? a.x[b * in + i] : 0.f;
    float f[kKF], d[kKF];
    {
      const float sg = rcp(1.0f + ex2(-xv * l2));
      f[0] = xv * sg;
      d[0] = sg * (1.0f + xv * (1.0f - sg));
      const float* kn = plan + L.knots + (int64_t)i * kNG;
      int m = -1;
#pragma unroll
      for (int j = 0; j < kNG; ++j) m += (xv >= kn[j]) ? 1 : 0;
      const bool fin = __builtin_isfinite(xv);
      const int mi = ((unsigned)m < (unsigned)(kNG - 1) && fin) ? m : kNG - 1;
      const float rh = mi < kNG - 1 ? plan[L.rh + (int64_t)i * (kNG - 1) + mi] : 0.f;
      const float u = mi < kNG - 1 ? (xv - kn[mi]) * rh : 0.f;
      const float4* bt = reinterpret_cast<const float4*>(plan + L.bt) + ((int64_t)i * kNG + mi) * kNS;
#pragma unroll
      for (int cc = 0; cc < kNS; ++cc) {
        const float4 cf = bt[cc];
        f[1 + cc] = fin ? ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x) : __builtin_nanf("");
        d[1 + cc] = fin ? ffma(ffma(3.0f * cf.w, u, 2.0f * cf.z), u, cf.y) * rh : __builtin_nanf("");
      }
      const float* lg = plan + L.lg + (int64_t)i * kNB * 2;
#pragma unroll
      for (int j = 0; j < kNB; ++j) {
        const float sj = rcp(1.0f + ex2(ffma(lg[2 * j], xv, lg[2 * j + 1])));
        f[1 + kNS + j] = sj;
        d[1 + kNS + j] = sj * (1.0f - sj);   // sigma'; times a for d/dx
      }
      f[kKF - 1] = 0.f;
      d[kKF - 1] = 0.f;
    }
    if (live) {
      float4* fr = reinterpret_cast<float4*>(a.F + b * (int64_t)in * kKF + (int64_t)i * kKF);
#pragma unroll
      for (int q = 0; q < kKF / 4; ++q) fr[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
    }
    wsync();
    const float* gq = gp + r * kPitch + ii * kKF;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q <= kNS; ++q) s = ffma(gq[q], d[q], s);
#pragma unroll
    for (int j = 0; j < kNB; ++j) {
      const float aj = a.la[i * kNB + j], bj = a.lb[i * kNB + j];
      const float gz = gq[1 + kNS + j] * d[1 + kNS + j];
      s = ffma(gz, aj, s);
      ga[j] = ffma(gz, xv - bj, ga[j]);
      gb[j] = ffma(gz, -aj, gb[j]);
    }
    if (live) a.gx[b * in + i] = a.accumulate ? a.gx[b * in + i] + s : s;
    wsync();   // the tile is read before the next one is written
  }
  // the 16 rows of an input are one DPP row
#pragma unroll
  for (int j = 0; j < kNB; ++j) {
    const float sa = row_sum16(ga[j]), sb = row_sum16(gb[j]);
    if (r == 0) {
      float* o = a.abp + (((int64_t)rg * in + i) * kNB + j) * 2;
      o[0] = sa;
      o[1] = sb;
    }
  }
}

// dWp partials: a wave = 16 feature columns x 64 outputs over rows [s * seg, (s + 1) * seg)
__global__ __launch_bounds__(256) void wide_kan_gw_kernel(const float* __restrict__ F, const float* __restrict__ g,
                                                          int64_t B, int ncol, int out, int rs, int64_t seg,
                                                          float* __restrict__ pw) {
  const int lane = threadIdx.x & 63, kg = lane >> 4, n = lane & 15;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nct = ncol / 16, nog = out / 64;
  const int ct = (int)(task % nct), og = (int)((task / nct) % nog), sgi = (int)(task / ((int64_t)nct * nog));
  if (sgi >= rs) return;
  const int64_t r0 = (int64_t)sgi * seg, r1 = r0 + seg < B ? r0 + seg : B;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* fa = F + ct * 16 + n;
  const float* gb = g + og * 64 + n;
  for (int64_t rr = r0; rr < r1; rr += 16) {
    float av[4], bv[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t b = rr + 4 * u + kg;
      const bool ok = b < r1;
      av[u] = ok ? fa[b * ncol] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) bv[u][t] = ok ? gb[b * out + 16 * t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u][t], acc[t], 0, 0, 0);
  }
  float* o = pw + ((int64_t)sgi * ncol + ct * 16) * out + og * 64 + n;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int v = 0; v < 4; ++v) o[(int64_t)(4 * kg + v) * out + 16 * t] = acc[t][v];
}

__device__ __forceinline__ void put_grad(float* p, float v, int accumulate) {
  if (p) *p = accumulate ? *p + v : v;
}

// a block = 64 consecutive (input i, output o) pairs (o fastest); wave w sums the row segments of
// features w, w + 4, ... in order (a thread per pair summing all 19 x rs partials ran 128 waves,
// 48 us of load latency at B = 2048), then wave 0 applies the packing's chain rule from LDS
// (wide_pack_kernel: base_weight; spline_weight * spline_scaler; 2 logistic_weight scale_logistic
// logistic_scaler) and writes the d/d(2 sigma) sums d_wl for the logistic_scaler pass
__global__ __launch_bounds__(256) void wide_kan_grad_kernel(fetode_kanlinear_t kl, const float* __restrict__ pw, int rs,
                                                            fetode_kanlinear_grad_t gr, float* __restrict__ d_wl,
                                                            int accumulate) {
  __shared__ float sv[kKF - 1][64];
  const int in = kl.in_features, out = kl.out_features;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  const bool live = t < (int64_t)in * out;
  const int o = live ? (int)(t % out) : 0, i = live ? (int)(t / out) : 0;
  const int64_t ncol = (int64_t)in * kKF, oi = (int64_t)o * in + i;
  for (int f = wv; f < kKF - 1; f += 4) {
    float s = 0.f;
    const float* src = pw + (int64_t)i * kKF * out + (int64_t)f * out + o;
#pragma unroll 4
    for (int q = 0; q < rs; ++q) s += src[(int64_t)q * ncol * out];
    sv[f][lane] = s;
  }
  __syncthreads();
  if (wv != 0 || !live) return;
  float v[kKF - 1];
#pragma unroll
  for (int f = 0; f < kKF - 1; ++f) v[f] = sv[f][lane];
  put_grad(gr.base_weight ? gr.base_weight + oi : nullptr, v[0], accumulate);
  const float sc = kl.spline_scaler ? kl.spline_scaler[oi] : 1.0f;
  float dsc = 0.f;
#pragma unroll
  for (int c = 0; c < kNS; ++c) {
    put_grad(gr.spline_weight ? gr.spline_weight + oi * kNS + c : nullptr, v[1 + c] * sc, accumulate);
    dsc += v[1 + c] * kl.spline_weight[oi * kNS + c];
  }
  if (kl.spline_scaler) put_grad(gr.spline_scaler ? gr.spline_scaler + oi : nullptr, dsc, accumulate);
  const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
#pragma unroll
  for (int j = 0; j < kNB; ++j) {
    const int64_t w = (int64_t)o * in * kNB + (int64_t)i * kNB + j;
    const float dw = 2.0f * v[1 + kNS + j];
    d_wl[w] = dw;
    put_grad(gr.logistic_weight ? gr.logistic_weight + w : nullptr, (dw * ls) * kl.scale_logistic, accumulate);
  }
}

// logistic a / b: a block = 64 (input, basis) sums, wave w adds row groups w, w + 16, ... in order,
// then wave 0 the 16 wave sums in order (one thread per sum over all row groups ran 10 waves: 30 us
// of load latency at B = 2048); logistic_scaler: one wave per output, fixed-order sums
constexpr int kAbWaves = 16;
__global__ __launch_bounds__(64 * kAbWaves) void wide_kan_ab_ls_kernel(fetode_kanlinear_t kl, const float* __restrict__ abp,
                                                                       int n_rg, const float* __restrict__ d_wl,
                                                                       fetode_kanlinear_grad_t gr, int accumulate) {
  __shared__ float sab[kAbWaves][2][64];
  const int in = kl.in_features, out = kl.out_features;
  const int nab = in * kNB;
  const int nabb = (nab + 63) / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if ((int)blockIdx.x < nabb) {
    const int t = blockIdx.x * 64 + lane;
    float sa = 0.f, sb = 0.f;
    if (t < nab)
      for (int q = wv; q < n_rg; q += kAbWaves) {
        const float2 v = *reinterpret_cast<const float2*>(&abp[((int64_t)q * nab + t) * 2]);
        sa += v.x;
        sb += v.y;
      }
    sab[wv][0][lane] = sa;
    sab[wv][1][lane] = sb;
    __syncthreads();
    if (wv != 0 || t >= nab) return;
    sa = sb = 0.f;
    for (int u = 0; u < kAbWaves; ++u) {
      sa += sab[u][0][lane];
      sb += sab[u][1][lane];
    }
    put_grad(gr.logistic_a ? gr.logistic_a + t : nullptr, sa, accumulate);
    put_grad(gr.logistic_b ? gr.logistic_b + t : nullptr, sb, accumulate);
    return;
  }
  if (!kl.logistic_scaler) return;
  const int o = ((int)blockIdx.x - nabb) * kAbWaves + wv;
  if (o >= out) return;
  float s = 0.f;
  for (int q = lane; q < nab; q += 64)
    s += d_wl[(int64_t)o * nab + q] * (kl.logistic_weight[(int64_t)o * nab + q] * kl.scale_logistic);
  for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) put_grad(gr.logistic_scaler ? gr.logistic_scaler + o : nullptr, s, accumulate);
}

struct KanBwdPlan {
  int n_rg, t16, rs;
  int64_t seg, tasks_gx, tasks_gw;
  int64_t off_F, off_abp, off_pw, off_dwl, off_gxs, end;   // floats
};

KanBwdPlan kan_bwd_plan(int in, int out, int64_t B) {
  KanBwdPlan p{};
  const int64_t nt = (B + 15) / 16, nch = in / 4;
  // ~4 k waves for the gx pass; the gw pass: segments of >= 256 rows, at most 16
  int64_t t16 = (nt * nch + 4095) / 4096;
  p.t16 = (int)(t16 > 0 ? t16 : 1);
  p.n_rg = (int)((nt + p.t16 - 1) / p.t16);
  p.tasks_gx = (int64_t)p.n_rg * nch;
  int64_t rs = (B + 255) / 256;
  rs = rs < 16 ? rs : 16;
  p.rs = (int)(rs > 0 ? rs : 1);
  p.seg = ((B + p.rs - 1) / p.rs + 15) / 16 * 16;
  p.rs = (int)((B + p.seg - 1) / p.seg);
  const int64_t ncol = (int64_t)in * kKF;
  p.tasks_gw = (ncol / 16) * (out / 64) * p.rs;
  int64_t o = 0;
  p.off_F = o; o += B * ncol;
  p.off_abp = o; o += (int64_t)p.n_rg * in * kNB * 2;
  p.off_pw = o; o += (int64_t)p.rs * ncol * out;
  p.off_dwl = o; o += (int64_t)out * in * kNB;
  p.off_gxs = o; o += B * in;   // d/dx when the caller wants only parameter gradients
  p.end = o;
  return p;
}

bool kan_bwd_wide_ok(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl) {
  return kl && wide_supported(kl, fl) && (kl->out_features == 64 || kl->out_features == 128) &&
         kl->spline_weight && kl->base_weight;
}


// =============================================================================================
// Device-resident dopri5 for a two-layer wide KAN-FET field: the ETT forecaster's own latent solve,
// odeint(self.dynamics, z0, t_fut, method="dopri5") at torchdiffeq's defaults
// (train_kan_fet_ett.py:192, :858, :879) with the KAN-FET field KANFET([64, 128, 64]).
//
// The host-driven solver (dopri5.py _Dopri5) pays per evaluation two wide-layer launches plus the
// combines, and per attempt a device->host read of the error ratio.  Here ONE launch runs the whole
// solve with a persistent grid that walks the layers' tiles (wide_tile, the per-layer launch's own
// body) phase by phase:
//   L0     tiles (64 rows x 16 hidden, input slice s) of layer 0: x = the stage input, prev = the
//          previous evaluation's input (ferro_class.py:409), out -> hidden slab hs[e & 1][s]
//   L1     tiles of layer 1: x = the hidden slabs summed in a fixed order (slab 0 + slab 1: the
//          per-layer launch's 0 + a + b), out -> k; whole (one slice) layers fold the Dormand-Prince
//          stage combine into the tile epilogue, sliced ones add a combine pass after a barrier
// A grid barrier separates the phases; stage inputs and hidden slabs are written through (sc1)
// and read after the barrier's agent-scope acquire (MI355X_MICROARCH.md, valid hand-off forms).
// Per-element solver state (y, f0, the running stage sums, err, mid, the interpolation
// coefficients) lives in HBM and is touched only by the element's owner thread: layer-1 tile t
// belongs to workgroup t % G, and its element (row, dim) to the epilogue thread that stores it —
// so none of it crosses workgroups.  The one global quantity per attempt is the RMS error ratio,
// summed in an order that depends on the batch alone (not on the grid): per layer-1 TILE an fp64
// partial (its owner threads, fixed order), then leaves of `leafL` consecutive tiles summed tile by
// tile, then an xor tree over the <= 64 leaves — every workgroup forms the same value, so all take
// the same decisions.  Control arithmetic: the host-driven path's (fp32 stage sums in
// fetode_lincomb's order, fp64 step control, fetode_interp_fit / _eval), so the solution equals the
// host loop's bit for bit up to the norms' fp64 summation order.
// Trajectory-sharded (fetode_wide_dopri5_xrank, SURVEY §8e caveat 2): each rank's grid owns the
// tiles of its rows; the norms are exchanged between the ranks' kernels through IPC-mapped inboxes
// (fetode_xrank.h).  When every rank's rows are whole leaves of the global tile sequence (and the
// input slices are the global batch's), the ranks exchange the leaf sums themselves and every rank
// forms the single device's xor tree: solution, steps and memory are bitwise the single device's on
// the global batch; otherwise the ranks exchange their totals and sum them in rank order.
// =============================================================================================
constexpr int kEs = 17;  // per-element state rows: y, f0, A0..A5, err, mid, co0..co4, y1, k_last
enum { kEY = 0, kEF0 = 1, kEA = 2, kEErr = 8, kEMid = 9, kECo = 10, kEY1 = 15, kEKl = 16 };
constexpr int kWBarWords = 64 * 10;  // 8 XCD counters, top counter, generation | abort (256 B apart)
constexpr unsigned kWSpinLimit = 1u << 22;
constexpr int kWideDopriMaxGrid = 256 * 8;  // the persistent grid's cap (2 workgroups per CU)
constexpr unsigned kXrSpinLimitW = 1u << 24;  // cross-rank polls: ranks may start seconds apart

struct WideDopriArgs {
  WideArgs l0, l1;  // plan + layout of each layer; x / prev / nslice are set per phase
  int64_t B;
  int D, H, S0, S1, reinit0, reinit1, nT0, nT1, nOT0, nOT1;
  const float* y0;
  const float* prev0;  // (B, D) hysteresis memory of layer 0 before the solve (unused when reinit0)
  const float* prev1;  // (B, H)
  float* st0;          // (B, D) / (B, H): the memory after the solve (the last evaluation's inputs)
  float* st1;
  float* xin;  // (2, B, D) stage inputs by evaluation parity
  float* hs;   // (2, S0, B, H) hidden slabs by evaluation parity
  float* ks;   // (S1, B, D) k slabs (S1 == 2)
  float* es;   // (kEs, B, D)
  float* sol;  // (T, B, D)
  const double* t;
  int T;
  float rtol, atol;
  double first_step, safety, ifactor, dfactor, min_step, max_step;
  int max_steps;
  float stc[7][8];  // tableau columns (DopriParams.stc)
  unsigned* bar;
  double* slot;  // (nT1, 2) per-tile norm partials
  int32_t* stats;
  double* att;
  int max_att;
  // the norm's summation structure and the cross-rank exchange
  double n_el;                 // element count of the norms: B_global * D
  int leafL, n_leaf;           // tiles per leaf (power of two), leaves of the global tile sequence (<= 64)
  int xr_rank, xr_world, xr_exact, leaf_lo, n_leaf_local;
  unsigned xr_epoch;
  double* const* xr_peers;     // (dev) every rank's inbox as mapped here (peers[rank] = own)
  double* xr_inbox;
};

__device__ __forceinline__ void st_wt(float* p, float v) {  // write-through (sc1) store
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef unsigned wd_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wd_st16(double* p, double v0, double v1) {
  const unsigned long long x = __double_as_longlong(v0), y = __double_as_longlong(v1);
  const wd_u32x4 v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y, (unsigned)(y >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void wd_ld16(const double* p, double& v0, double& v1) {
  wd_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  v0 = __longlong_as_double(((unsigned long long)v.y << 32) | v.x);
  v1 = __longlong_as_double(((unsigned long long)v.w << 32) | v.z);
}

// Grid barrier with a hand-off: every wave drains its write-through stores, the workgroup arrives
// (XCD-hierarchical counters as fetode_ecg.hip grid_barrier: per-XCD counter, its last arriver on
// the top counter, the last of those bumps the generation), polls the generation relaxed, then ONE
// agent-scope acquire (this CU's L1 dropped) before any wave loads what other workgroups wrote.
// Bounded spins: a grid that is not co-resident raises the abort word and every barrier returns.
__device__ bool wide_barrier(unsigned* bar) {
  __shared__ int s_ab;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nblk = gridDim.x;
    const unsigned x = blockIdx.x & 7u;
    const unsigned nx = (nblk + 7u - x) / 8u, nxcd = nblk < 8u ? nblk : 8u;
    unsigned* cnt = bar + 64 * x;
    unsigned* top = bar + 64 * 8;
    unsigned* gen = bar + 64 * 9;
    unsigned* abw = gen + 1;
    int ab = __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (!ab) {
      const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nx - 1u) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nxcd - 1u) {
          __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if ((spins & 15u) == 15u && __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          ab = 1;
          break;
        }
        if (++spins == kWSpinLimit) {
          __hip_atomic_store(abw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ab = 1;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_ab = ab;
  }
  __syncthreads();
  return s_ab != 0;
}

__device__ __forceinline__ double wd_xor_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// The owner threads' two fp64 values of one layer-1 tile -> the tile's partial (xor tree per wave,
// waves 0..3 in order), stored write-through at slot[t].  Every thread of the workgroup calls it.
__device__ void wide_tile_partial(double* slot, int t, double v0, double v1) {
  __shared__ double s_red[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v0 = wd_xor_sum(v0);
  v1 = wd_xor_sum(v1);
  if (lane == 0 && w < 4) {
    s_red[w][0] = v0;
    s_red[w][1] = v1;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    wd_st16(slot + 2 * t, ((s_red[0][0] + s_red[1][0]) + s_red[2][0]) + s_red[3][0],
            ((s_red[0][1] + s_red[1][1]) + s_red[2][1]) + s_red[3][1]);
  __syncthreads();
}

// leaf j's sum: its tiles [j L, (j + 1) L) of `nt` (read from slot, local tile numbering) in order
__device__ __forceinline__ void wide_leaf(const double* slot, int j, int L, int nt, double& a0, double& a1) {
  a0 = 0.0;
  a1 = 0.0;
  const int e = min((j + 1) * L, nt);
  for (int t = j * L; t < e; ++t) {
    double u0, u1;
    wd_ld16(slot + 2 * t, u0, u1);
    a0 += u0;
    a1 += u1;
  }
}

// The grid-wide (and, sharded, rank-wide) sum of the tile partials, returned to every workgroup in
// the same fixed order.  Contains a grid barrier.  `round` counts the calls (the same in every
// workgroup and on every rank: every rank takes the same decisions).
__device__ bool wide_norm(const WideDopriArgs& a, unsigned& round, double& s0, double& s1) {
  __shared__ double s_out[2];
  __shared__ int s_ab;
  if (wide_barrier(a.bar)) return true;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned* abw = a.bar + 64 * 9 + 1;
  if (w == 0) {
    double g0 = 0.0, g1 = 0.0;
    int ab = 0;
    if (a.xr_world <= 1) {  // one device: every workgroup sums the leaves itself
      double v0 = 0.0, v1 = 0.0;
      if (lane < a.n_leaf) wide_leaf(a.slot, lane, a.leafL, a.nT1, v0, v1);
      g0 = wd_xor_sum(v0);
      g1 = wd_xor_sum(v1);
    } else {
      const unsigned r = round, par = r & 1u;
      const int W = a.xr_world;
      if (blockIdx.x == 0) {  // send: this rank's leaves at their global index (exact), or its total
        double v0 = 0.0, v1 = 0.0;
        if (lane < a.n_leaf_local) wide_leaf(a.slot, lane, a.leafL, a.nT1, v0, v1);
        if (a.xr_exact) {
          if (lane < a.n_leaf_local)
            for (int q = 0; q < W; ++q) xr_st16(xr_rec(a.xr_peers[q], par, a.leaf_lo + lane), v0, v1);
        } else {
          const double t0 = wd_xor_sum(v0), t1 = wd_xor_sum(v1);
          if (lane < W) xr_st16(xr_rec(a.xr_peers[lane], par, a.xr_rank), t0, t1);
        }
        const unsigned long long tag = ((unsigned long long)a.xr_epoch << 32) | (unsigned long long)(r + 1u);
        if (lane < W) xr_st_tag(xr_tagp(a.xr_peers[lane], par, a.xr_rank), tag);
      }
      // receive: every rank's round-r tag in this device's inbox, then the records
      const unsigned long long tag = ((unsigned long long)a.xr_epoch << 32) | (unsigned long long)(r + 1u);
      if (lane < W) {
        const double* tg = xr_tagp(a.xr_inbox, par, lane);
        unsigned spins = 0;
        while (xr_ld_tag(tg) != tag) {
          __builtin_amdgcn_s_sleep(2);
          if ((spins & 255u) == 255u && __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            ab = 1;
            break;
          }
          if (++spins == kXrSpinLimitW) {
            __hip_atomic_store(abw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ab = 1;
            break;
          }
        }
      }
      ab = __any(ab) ? 1 : 0;
      if (!ab) {
        double v0 = 0.0, v1 = 0.0;
        if (a.xr_exact) {  // the single device's xor tree over the global leaves
          if (lane < a.n_leaf) xr_ld16(xr_rec(a.xr_inbox, par, lane), v0, v1);
          g0 = wd_xor_sum(v0);
          g1 = wd_xor_sum(v1);
        } else {  // rank totals in rank order
          if (lane < W) xr_ld16(xr_rec(a.xr_inbox, par, lane), v0, v1);
          for (int j = 0; j < W; ++j) {
            g0 += __shfl(v0, j);
            g1 += __shfl(v1, j);
          }
        }
      }
    }
    if (lane == 0) {
      s_out[0] = g0;
      s_out[1] = g1;
      s_ab = ab;
    }
  }
  ++round;
  __syncthreads();
  s0 = s_out[0];
  s1 = s_out[1];
  return s_ab != 0;
}

enum { kCmbF0 = 0, kCmbF1 = 1, kCmbStage = 2 };

// The solver's uniform state lives in LDS: thread 0 takes every decision, the other threads read
// it after a workgroup barrier, so none of it is live in registers across a layer phase (the tile
// body alone fills the SGPR file with its scalar-cache constants).
struct WdCtl {
  double dt, t0, t1, t0s, t1s;
  float h0, d1, dt32, fit_dt32;
  int nev, nfev, n_att, iout, n_steps, stg, kind, status;
  int fit, io_lo, io_hi, next;  // after a decision: accept fit?, outputs [io_lo, io_hi), next input
  float cc[8];                  // tableau column of the stage just evaluated (k_{stg+1})
};
enum { kNextNone = 0, kNextProbe = 1, kNextAttempt = 2 };

template <int K>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void wide_dopri5_kernel(WideDopriArgs a) {
  __shared__ WdCtl ctl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int G = (int)gridDim.x;
  const int64_t B = a.B, BD = B * a.D, BH = B * a.H;
  const int D = a.D, H = a.H;
  const double n_el = a.n_el;
  // element ownership: the layer-1 tile epilogue's storing threads (waves 0-3: row 16 (w % 4) +
  // 4 (lane / 16) + v, dim lane % 16), layer-1 tile t < nT1 on workgroup t % G
  const bool owner = w < 4;
  const int rt = w & 3, kq = lane >> 4, kr = lane & 15;
  auto for_owned = [&](auto&& f) {
    if (!owner) return;
    for (int t = blockIdx.x; t < a.nT1; t += G) {
      const int64_t b0 = (int64_t)(t / a.nOT1) * kRows;
      const int d = (t % a.nOT1) * kOuts + kr;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t b = b0 + 16 * rt + 4 * kq + v;
        if (b < B) f(b * D + d);
      }
    }
  };
  float* const es = a.es;
  unsigned nround = 0;  // norm rounds (wide_norm)

  for_owned([&](int64_t i) {
    const float y = a.y0[i];
    es[kEY * BD + i] = y;
    a.sol[i] = y;
  });
  if (tid == 0) {
    ctl.dt = a.first_step;
    ctl.t0 = ctl.t1 = 0.0;
    ctl.t0s = ctl.t1s = a.t[0];
    ctl.h0 = ctl.d1 = ctl.dt32 = 0.f;
    ctl.nev = ctl.nfev = ctl.n_att = ctl.n_steps = ctl.stg = 0;
    ctl.iout = 1;
    ctl.kind = kCmbF0;
    ctl.status = -1;
  }
  __syncthreads();
  int status = -1;
#pragma unroll 1
  for (;;) {
    // ---- one field evaluation: L0 phase | barrier | L1 phase | barrier ----
    const int e = ctl.nev, p = e & 1;
    if (e > 0 && wide_barrier(a.bar)) {  // the stage input came from other workgroups
      status = 4;
      break;
    }
    bool ab = false;
#pragma unroll 1
    for (int l = 0; l < 2 && !ab; ++l) {
      WideArgs L = l ? a.l1 : a.l0;
      const int nT = l ? a.nT1 : a.nT0, nOT = l ? a.nOT1 : a.nOT0, S = l ? a.S1 : a.S0;
      if (l == 0) {
        L.x = e == 0 ? a.y0 : a.xin + p * BD;
        L.nxs = L.nps = 1;
        L.reinit = e == 0 ? a.reinit0 : 0;
        L.prev = e == 0 ? a.prev0 : (e == 1 ? a.y0 : a.xin + (p ^ 1) * BD);
      } else {
        L.x = a.hs + (int64_t)p * a.S0 * BH;
        L.nxs = a.S0;
        L.xss = BH;
        L.reinit = e == 0 ? a.reinit1 : 0;
        L.prev = e == 0 ? a.prev1 : a.hs + (int64_t)(p ^ 1) * a.S0 * BH;
        L.nps = e == 0 ? 1 : a.S0;
        L.pss = BH;
      }
      L.nslice = S;
      const int ow = l ? D : H;
      float* const ob = l ? a.ks : a.hs + (int64_t)p * a.S0 * BH;  // k slabs | this parity's hidden slabs
      const int64_t sl = l ? BD : BH;
      for (int t = blockIdx.x; t < nT * S; t += G) {
        const int bz = t / nT, r = t % nT;
        float* const o = ob + bz * sl;
        wide_tile<K, true, true, kChMax, true>(L, r / nOT, r % nOT, bz,
                                               [&](int64_t b, int c, float v) { st_wt(&o[b * ow + c], v); });
      }
      ab = wide_barrier(a.bar);
    }
    if (ab) {
      status = 4;
      break;
    }
    // ---- the per-element combine of k (the host loop's fetode_lincomb / scaled_rms order) ----
    {
      const int kind = ctl.kind, stg = ctl.stg, pn = (e + 1) & 1;
      const float dt32 = ctl.dt32;
      float c[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) c[q] = ctl.cc[q];
      const int S1 = a.S1;
      // norm terms: per layer-1 tile (wide_tile_partial) when this evaluation ends in a reduction
      const bool red = (kind == kCmbF0 && !(a.first_step > 0.0)) || kind == kCmbF1 || (kind == kCmbStage && stg == 5);
      double acc0 = 0.0, acc1 = 0.0;
      auto elem = [&](int64_t i) {
        float k = a.ks[i];
        for (int s = 1; s < S1; ++s) k = k + a.ks[s * BD + i];  // slab 0 + slab 1 + ..: the launch path's order
        const float y = es[kEY * BD + i];
        if (kind == kCmbF0) {  // f0 = f(t0, y0); _select_initial_step's d0 / d1 terms
          es[kEF0 * BD + i] = k;
          const float scale = a.atol + a.rtol * fabsf(y);
          const float q0 = y / scale, q1 = k / scale;
          acc0 += (double)q0 * q0;
          acc1 += (double)q1 * q1;
        } else if (kind == kCmbF1) {  // d2 term: (f1 - f0) / scale
          const float scale = a.atol + a.rtol * fabsf(y);
          const float q2 = (k - es[kEF0 * BD + i]) / scale;
          acc0 += (double)q2 * q2;
        } else {  // Dormand-Prince stage stg (k = k_{stg + 1}): the running sums take k's column
          float a0 = 0.f;
#pragma unroll
          for (int q = 0; q < 5; ++q) {
            const float v = es[(kEA + q + 1) * BD + i] + k * (c[q] * dt32);
            es[(kEA + q) * BD + i] = v;
            if (q == 0) a0 = v;
          }
          const float err = es[kEErr * BD + i] + k * (c[6] * dt32);
          es[kEErr * BD + i] = err;
          es[kEMid * BD + i] = es[kEMid * BD + i] + k * (c[7] * dt32);
          if (stg < 5) {
            const float yi = y + a0;
            st_wt(a.xin + pn * BD + i, yi);
            es[kEY1 * BD + i] = yi;
          } else {  // FSAL: k is f(t1, y1); the error ratio's term and torchdiffeq's finiteness assert
            es[kEKl * BD + i] = k;
            const float y1 = es[kEY1 * BD + i];
            const float tol = a.atol + a.rtol * fmaxf(fabsf(y), fabsf(y1));
            const float qe = err / tol;
            acc0 += (double)qe * qe;
            acc1 += __builtin_isfinite(y) ? 0.0 : 1.0;
          }
        }
      };
      for (int t = blockIdx.x; t < a.nT1; t += G) {
        if (owner) {
          const int64_t b0 = (int64_t)(t / a.nOT1) * kRows;
          const int d = (t % a.nOT1) * kOuts + kr;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int64_t b = b0 + 16 * rt + 4 * kq + v;
            if (b < B) elem(b * D + d);
          }
        }
        if (red) {
          wide_tile_partial(a.slot, t, acc0, acc1);
          acc0 = acc1 = 0.0;
        }
      }
    }
    // ---- the decision (thread 0) ----
    const int kind = ctl.kind, stg = ctl.stg;
    const bool reduce = !(kind == kCmbF0 && a.first_step > 0.0) && !(kind == kCmbStage && stg < 5);
    double s0 = 0.0, s1 = 0.0;
    if (reduce && wide_norm(a, nround, s0, s1)) {
      status = 4;
      break;
    }
    __syncthreads();  // every wave has read this evaluation's control words before thread 0 rewrites them
    if (tid == 0) {
      ctl.nev = e + 1;
      ++ctl.nfev;
      ctl.fit = 0;
      ctl.next = kNextNone;
      ctl.io_lo = ctl.io_hi = ctl.iout;
      bool sched = false;  // outputs due, then the next attempt
      if (kind == kCmbStage && stg < 5) {
        ctl.stg = stg + 1;
        ctl.next = kNextNone;  // the combine already wrote the next stage input
      } else if (kind == kCmbF0 && !(a.first_step > 0.0)) {  // misc._select_initial_step in fp32
        const float d0 = fabsf(sqrtf((float)(s0 / n_el)));
        const float d1 = fabsf(sqrtf((float)(s1 / n_el)));
        float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
        ctl.h0 = fabsf(h0);
        ctl.d1 = d1;
        ctl.kind = kCmbF1;
        ctl.next = kNextProbe;
      } else if (kind == kCmbF1) {
        const float h0 = ctl.h0, d1 = ctl.d1;
        const float d2 = fabsf(sqrtf((float)(s0 / n_el)) / h0);
        float h1;
        if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
        else h1 = (float)pow((double)(0.01f / fmaxf(d1, d2)), (double)0.2f);  // fp64 pow rounded once: host == device
        ctl.dt = (double)fminf(100.0f * h0, fabsf(h1));
        sched = true;
      } else if (kind == kCmbF0) {  // first_step given
        sched = true;
      } else {  // the attempt's error ratio, accept / reject, rk_common._optimal_step_size
        if (s1 != 0.0) {
          ctl.status = 1;
        } else {
          const float ratio = sqrtf((float)(s0 / n_el));
          const bool accept = ratio <= 1.0f;
          const double dt = ctl.dt;
          if (blockIdx.x == 0 && ctl.n_att < a.max_att) {
            double* o = a.att + (int64_t)ctl.n_att * 4;
            o[0] = ctl.t0;
            o[1] = dt;
            o[2] = (double)ratio;
            o[3] = accept ? 1.0 : 0.0;
          }
          ++ctl.n_att;
          if (accept) {
            ctl.fit = 1;
            ctl.fit_dt32 = ctl.dt32;  // the accepted attempt's step (dt32 is about to take the next one)
            ctl.t0s = ctl.t0;
            ctl.t1s = ctl.t1;
          } else {
            ctl.t0s = ctl.t0;
          }
          const double rr = (double)ratio;
          double nxt;
          if (rr == 0.0) {
            nxt = dt * a.ifactor;
          } else {
            const double dfac = rr < 1.0 ? 1.0 : a.dfactor;
            const double factor = __builtin_isnan(rr) ? rr : fmin(a.ifactor, fmax(a.safety / pow(rr, 1.0 / 5.0), dfac));
            nxt = dt * factor;
          }
          ctl.dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, a.min_step), a.max_step);
          ++ctl.n_steps;
          sched = true;
        }
      }
      if (sched) {
        // outputs due (interp._interp_evaluate of the last accepted step), then the next attempt
        int io = ctl.iout;
        while (io < a.T && !(a.t[io] > ctl.t1s)) {
          ++io;
          ctl.n_steps = 0;
        }
        ctl.io_hi = io;
        ctl.iout = io;
        if (io >= a.T) {
          ctl.status = 0;
        } else if (ctl.n_steps >= a.max_steps) {
          ctl.status = 3;
        } else {
          const double t0 = ctl.t1s, dt = ctl.dt;
          if (!(t0 + dt > t0)) {
            ctl.status = 2;
          } else {
            ctl.t0 = t0;
            ctl.t1 = t0 + dt;
            ctl.dt32 = (float)dt;
            ctl.kind = kCmbStage;
            ctl.stg = 0;
            ctl.next = kNextAttempt;
          }
        }
      }
      // the tableau column of the next stage evaluation's k (static indices: kernel-argument reads)
#pragma unroll
      for (int j = 1; j < 7; ++j)
        if (j == ctl.stg + 1) {
#pragma unroll
          for (int q = 0; q < 8; ++q) ctl.cc[q] = a.stc[j][q];
        }
    }
    __syncthreads();
    // ---- the decision's element passes (owner threads only: no hand-off) ----
    if (ctl.fit) {  // interp._interp_fit (fetode_interp_fit's op order); y <- y1, f0 <- k7
      const float dtc = ctl.fit_dt32;
      for_owned([&](int64_t i) {
        const float y = es[kEY * BD + i], y1 = es[kEY1 * BD + i];
        const float fa = es[kEF0 * BD + i], fb = es[kEKl * BD + i];
        const float ym = y + es[kEMid * BD + i];
        es[(kECo + 4) * BD + i] = ((2.0f * dtc) * (fb - fa) - 8.0f * (y1 + y)) + 16.0f * ym;
        es[(kECo + 3) * BD + i] = ((dtc * (5.0f * fa - 3.0f * fb) + 18.0f * y) + 14.0f * y1) - 32.0f * ym;
        es[(kECo + 2) * BD + i] = ((dtc * (fb - 4.0f * fa) - 11.0f * y) - 5.0f * y1) + 16.0f * ym;
        es[(kECo + 1) * BD + i] = dtc * fa;
        es[kECo * BD + i] = y;
        es[kEY * BD + i] = y1;
        es[kEF0 * BD + i] = fb;
      });
    }
    for (int j = ctl.io_lo; j < ctl.io_hi; ++j) {
      const float xq = (float)((a.t[j] - ctl.t0s) / (ctl.t1s - ctl.t0s));
      float* const so = a.sol + (int64_t)j * BD;
      for_owned([&](int64_t i) {
        float total = es[kECo * BD + i] + xq * es[(kECo + 1) * BD + i];
        float xp = xq;
#pragma unroll
        for (int q = 2; q < 5; ++q) {
          xp = xp * xq;
          total = total + xp * es[(kECo + q) * BD + i];
        }
        so[i] = total;
      });
    }
    if (ctl.status >= 0) {
      status = ctl.status;
      break;
    }
    const int pw = (e + 1) & 1;
    if (ctl.next == kNextProbe) {  // y0 + f0 h0 (fetode_lincomb with k[0] = f0)
      const float hh = ctl.h0;
      for_owned([&](int64_t i) { st_wt(a.xin + pw * BD + i, es[kEY * BD + i] + es[kEF0 * BD + i] * hh); });
    } else if (ctl.next == kNextAttempt) {  // the attempt's running sums from f0, its first stage input
      const float dtc = ctl.dt32;
      for_owned([&](int64_t i) {
        const float f0 = es[kEF0 * BD + i];
        float a0 = 0.f;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const float v = f0 * (a.stc[0][q] * dtc);
          es[(kEA + q) * BD + i] = v;
          if (q == 0) a0 = v;
        }
        es[kEErr * BD + i] = f0 * (a.stc[0][6] * dtc);
        es[kEMid * BD + i] = f0 * (a.stc[0][7] * dtc);
        const float yi = es[kEY * BD + i] + a0;
        st_wt(a.xin + pw * BD + i, yi);
        es[kEY1 * BD + i] = yi;
      });
    }
  }
  const int nev = ctl.nev;
  if (status != 4 && nev > 0) {
    // the hysteresis memory after the solve: the last evaluation's layer inputs (ferro_class.py:409)
    const int el = nev - 1, pl = el & 1;
    const float* x0 = el == 0 ? a.y0 : a.xin + pl * BD;
    const float* h0 = a.hs + (int64_t)pl * a.S0 * BH;
    const int64_t nthr = (int64_t)G * kThreads;
    for (int64_t j = (int64_t)blockIdx.x * kThreads + tid; j < BH; j += nthr) {
      float v = h0[j];
      for (int s = 1; s < a.S0; ++s) v = v + h0[s * BH + j];
      a.st1[j] = v;
      if (j < BD) a.st0[j] = x0[j];
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    a.stats[0] = ctl.nfev;
    a.stats[1] = ctl.n_att;
    a.stats[2] = __hip_atomic_load(a.bar + 64 * 9 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 4 : status;
  }
}

struct WideDopriShape {
  int S0, S1, nT0, nT1, nOT0, nOT1;
  int64_t off_slot, off_xin, off_hs, off_ks, off_es, bytes;  // byte offsets in the workspace
};

// input slices per layer: the per-layer launch's rule (fetode_wide_layer_forward) over the batch
// B_slices (the local batch: the host-driven loop's sums; a sharded solve that must be bitwise the
// single device: the global batch)
WideDopriShape wide_dopri_shape(int64_t B, int D, int H, int64_t B_slices = 0) {
  WideDopriShape s{};
  const int64_t rows = (B + kRows - 1) / kRows;
  const int64_t rows_s = ((B_slices > 0 ? B_slices : B) + kRows - 1) / kRows;
  s.nOT0 = H / kOuts;
  s.nOT1 = D / kOuts;
  s.nT0 = (int)(rows * s.nOT0);
  s.nT1 = (int)(rows * s.nOT1);
  s.S0 = wide_slices(rows_s * s.nOT0, D);
  s.S1 = wide_slices(rows_s * s.nOT1, H);
  auto al = [](int64_t v) { return (v + 255) & ~int64_t(255); };
  int64_t o = al((int64_t)sizeof(unsigned) * kWBarWords);
  s.off_slot = o;
  o = al(o + (int64_t)sizeof(double) * 2 * s.nT1);
  s.off_xin = o;
  o = al(o + (int64_t)sizeof(float) * 2 * B * D);
  s.off_hs = o;
  o = al(o + (int64_t)sizeof(float) * 2 * s.S0 * B * H);
  s.off_ks = o;
  o = al(o + (int64_t)sizeof(float) * s.S1 * B * D);
  s.off_es = o;
  o = al(o + (int64_t)sizeof(float) * kEs * B * D);
  s.bytes = o;
  return s;
}

}  // namespace

extern "C" {

int fetode_wide_layer_supported(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl) {
  return wide_supported(kl, fl) ? 1 : 0;
}

int64_t fetode_wide_layer_plan_bytes(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl) {
  if (!wide_supported(kl, fl)) return -1;
  return wide_layout(kl, fl).end * (int64_t)sizeof(float);
}

int fetode_wide_layer_plan_build(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl, void* plan, void* stream) {
  if (!wide_supported(kl, fl)) return set_err(FETODE_EUNSUPPORTED, "wide layer: unsupported shape / parameters");
  if (!plan) return set_err(FETODE_EINVAL, "wide layer: null plan");
  const WideLayout L = wide_layout(kl, fl);
  const fetode_kanlinear_t k0 = kl ? *kl : fetode_kanlinear_t{};
  const fetode_ferro_t f0 = fl ? *fl : fetode_ferro_t{};
  const int64_t n = std::max<int64_t>({(int64_t)L.out * L.in * std::max(L.K, 1), (int64_t)L.in * kWF * L.out});
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wide_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k0, f0, L, (float*)plan);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_const_kernel, dim3((unsigned)L.out), dim3(64), 0, s, f0, L, (float*)plan);
  LAUNCH_CHECK();
  if (L.kan) {
    const int64_t nb = (int64_t)L.in * kNG * kNS;
    hipLaunchKernelGGL(wide_basis_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, k0, L, (float*)plan);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int fetode_wide_layer_forward(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl, const void* plan, const float* x,
                              int64_t B, const float* prev, int32_t reinit, float* out, void* stream) {
  if (!wide_supported(kl, fl)) return set_err(FETODE_EUNSUPPORTED, "wide layer: unsupported shape / parameters");
  if (B <= 0) return FETODE_OK;
  if (!plan || !x || !out || (fl && !reinit && !prev)) return set_err(FETODE_EINVAL, "wide layer: null pointer");
  if (x == out) return set_err(FETODE_EINVAL, "wide layer: out must not alias x");
  WideArgs a{};
  a.plan = (const float*)plan;
  a.L = wide_layout(kl, fl);
  a.x = x;
  a.prev = prev;
  a.grid = kl ? kl->grid : nullptr;
  a.B = B;
  a.reinit = reinit;
  a.out = out;
  const int64_t tiles = (B + kRows - 1) / kRows;
  if (tiles > 0x7fffffff) return set_err(FETODE_EINVAL, "wide layer: batch too large");
  // Few tiles (e.g. 128 -> 64 at B = 8192: 512 workgroups for 256 CUs x 3 resident) leave the CUs
  // short of waves to hide the staging latency: split the inputs over two workgroups per tile.
  const int64_t wgs = tiles * (a.L.out / kOuts);
  a.nslice = wide_slices(wgs, a.L.in);
  a.nxs = a.nps = 1;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)tiles, (unsigned)(a.L.out / kOuts), (unsigned)a.nslice);
  if (a.nslice == 2) HIP_CHECK_RET(hipMemsetAsync(out, 0, sizeof(float) * B * a.L.out, st));
  if (a.nslice <= 2) {
    hipLaunchKernelGGL(pick(a.L.K, a.L.kan, a.L.ferro), grid, dim3(kThreads), 0, st, a);
  } else {  // slabs (slice s at s * B * out), then their fixed-order sum into out
    const int64_t n = B * a.L.out;
    float* slab = slab_scratch((size_t)a.nslice * n);
    if (!slab) return set_err(FETODE_EHIP, "wide layer: slab scratch allocation failed");
    a.out = slab;
    hipLaunchKernelGGL(pick(a.L.K, a.L.kan, a.L.ferro), grid, dim3(kThreads), 0, st, a);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(wide_slab_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const float*)slab,
                       a.nslice, n, out);
  }
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_ferro_backward_wide_workspace(const fetode_ferro_t* fl, int64_t B) {
  if (!fl || !wide_supported(nullptr, fl)) return -1;
  if (B <= 0) return 0;
  const FerroBwdPlan p = ferro_bwd_plan(fl->in_dim, fl->out_dim, fl->num_basis, B);
  const int64_t nU = B * fl->in_dim * 4, ngx = (int64_t)p.n_ogb * B * fl->in_dim,
                npp = (int64_t)p.rs * fl->in_dim * fl->out_dim * fl->num_basis * 5;
  return (nU + ngx + npp) * (int64_t)sizeof(float) + 256;
}

int fetode_ferro_backward_wide(const fetode_ferro_t* fl, const void* plan, const float* x, int64_t B, const float* prev,
                               int32_t reinit, const float* g, float* gx, const fetode_ferro_grad_t* grads,
                               int32_t accumulate, void* workspace, void* stream) {
  if (!fl || !wide_supported(nullptr, fl)) return set_err(FETODE_EUNSUPPORTED, "ferro wide backward: unsupported shape / parameters");
  if (B <= 0) return FETODE_OK;
  if (!plan || !x || !g || !workspace || (!reinit && !prev)) return set_err(FETODE_EINVAL, "ferro wide backward: null pointer");
  if (!gx && !grads) return FETODE_OK;
  const int in = fl->in_dim, out = fl->out_dim, K = fl->num_basis;
  const FerroBwdPlan p = ferro_bwd_plan(in, out, K, B);
  if ((p.tasks + 3) / 4 > 0x7fffffff) return set_err(FETODE_EINVAL, "ferro wide backward: batch too large");
  const hipStream_t s = (hipStream_t)stream;
  const WideLayout L = wide_layout(nullptr, fl);
  const uintptr_t base = ((uintptr_t)workspace + 255) & ~(uintptr_t)255;
  float4* U = reinterpret_cast<float4*>(base);
  float* gxp = reinterpret_cast<float*>(U + B * in);
  float* pp = gxp + (int64_t)p.n_ogb * B * in;
  const int64_t n = B * in;
  hipLaunchKernelGGL(wide_ferro_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, prev, (int)reinit,
                     n, L.gsl2e, L.gs, U);
  LAUNCH_CHECK();
  WideFerroBwdArgs a;
  a.plan = (const float*)plan;
  a.L = L;
  a.k = fl->k;
  a.Ec = fl->Ec;
  a.Ps = fl->Ps;
  a.bias = fl->bias;
  a.coef = fl->coef;
  a.U = U;
  a.g = g;
  a.B = B;
  a.n_og = p.n_og;
  a.n_ogb = p.n_ogb;
  a.rs = p.rs;
  a.seg = p.seg;
  a.gxp = gxp;
  a.pp = pp;
  const int ogw = ferro_bwd_ogw();
  void (*kern)(WideFerroBwdArgs) =
      K == 12 ? (ogw == 1 ? wide_ferro_bwd_kernel<12, 1> : ogw == 4 ? wide_ferro_bwd_kernel<12, 4> : wide_ferro_bwd_kernel<12, 2>)
              : (ogw == 1 ? wide_ferro_bwd_kernel<10, 1> : ogw == 4 ? wide_ferro_bwd_kernel<10, 4> : wide_ferro_bwd_kernel<10, 2>);
  hipLaunchKernelGGL(kern, dim3((unsigned)((p.tasks + 3) / 4)),
                     dim3(256), 0, s, a);
  LAUNCH_CHECK();
  if (gx) {
    hipLaunchKernelGGL(wide_ferro_gx_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, gxp, p.n_ogb, n,
                       gx, (int)accumulate);
    LAUNCH_CHECK();
  }
  if (grads) {
    const int64_t ne = (int64_t)in * out * K;
    hipLaunchKernelGGL(wide_ferro_gp_reduce_kernel, dim3((unsigned)((ne * 5 + 255) / 256)), dim3(256), 0, s, pp, p.rs,
                       ne, *grads, (int)accumulate);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int64_t fetode_kanlinear_backward_wide_workspace(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl, int64_t B) {
  if (!kan_bwd_wide_ok(kl, fl)) return -1;
  if (B <= 0) return 0;
  return kan_bwd_plan(kl->in_features, kl->out_features, B).end * (int64_t)sizeof(float) + 256;
}

int fetode_kanlinear_backward_wide(const fetode_kanlinear_t* kl, const fetode_ferro_t* fl, const void* plan, const float* x,
                                   int64_t B, const float* g, float* gx, const fetode_kanlinear_grad_t* grads,
                                   int32_t accumulate, void* workspace, void* stream) {
  if (!kan_bwd_wide_ok(kl, fl)) return set_err(FETODE_EUNSUPPORTED, "kanlinear wide backward: unsupported shape / parameters");
  if (B <= 0) return FETODE_OK;
  if (!plan || !x || !g || !workspace) return set_err(FETODE_EINVAL, "kanlinear wide backward: null pointer");
  if ((uintptr_t)g & 15) return set_err(FETODE_EINVAL, "kanlinear wide backward: g must be 16-byte aligned");
  if (!gx && !grads) return FETODE_OK;
  const int in = kl->in_features, out = kl->out_features;
  const KanBwdPlan p = kan_bwd_plan(in, out, B);
  if ((p.tasks_gx + 3) / 4 > 0x7fffffff || (p.tasks_gw + 3) / 4 > 0x7fffffff)
    return set_err(FETODE_EINVAL, "kanlinear wide backward: batch too large");
  const hipStream_t s = (hipStream_t)stream;
  float* ws = reinterpret_cast<float*>(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  WideKanBwdArgs a;
  a.plan = (const float*)plan;
  a.L = wide_layout(kl, fl);
  a.la = kl->logistic_a;
  a.lb = kl->logistic_b;
  a.x = x;
  a.g = g;
  a.B = B;
  // d/dx is always formed (the pass also writes the features); without gx it goes to scratch
  a.gx = gx ? gx : ws + p.off_gxs;
  a.accumulate = gx ? (int)accumulate : 0;
  a.F = ws + p.off_F;
  a.abp = ws + p.off_abp;
  a.n_rg = p.n_rg;
  a.t16 = p.t16;
  hipLaunchKernelGGL(out == 128 ? wide_kan_gx_kernel<32> : wide_kan_gx_kernel<16>, dim3((unsigned)((p.tasks_gx + 3) / 4)),
                     dim3(256), 0, s, a);
  LAUNCH_CHECK();
  if (!grads) return FETODE_OK;
  const int ncol = in * kKF;
  hipLaunchKernelGGL(wide_kan_gw_kernel, dim3((unsigned)((p.tasks_gw + 3) / 4)), dim3(256), 0, s, (const float*)a.F, g, B,
                     ncol, out, p.rs, p.seg, ws + p.off_pw);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_kan_grad_kernel, dim3((unsigned)(((int64_t)in * out + 63) / 64)), dim3(256), 0, s, *kl,
                     (const float*)(ws + p.off_pw), p.rs, *grads, ws + p.off_dwl, (int)accumulate);
  LAUNCH_CHECK();
  const int nabb = (in * kNB + 63) / 64;
  hipLaunchKernelGGL(wide_kan_ab_ls_kernel, dim3((unsigned)(nabb + (out + kAbWaves - 1) / kAbWaves)), dim3(64 * kAbWaves), 0, s, *kl,
                     (const float*)a.abp, p.n_rg, (const float*)(ws + p.off_dwl), *grads, (int)accumulate);
  LAUNCH_CHECK();
  return FETODE_OK;
}


}  // extern "C"

namespace {
// the norm's leaves: L tiles each (the smallest power of two with <= 64 leaves over nt tiles)
int wide_leaf_len(int64_t nt) {
  int L = 1;
  while ((nt + L - 1) / L > 64) L *= 2;
  return L;
}
// a sharded solve is bitwise the single device's when this rank's rows are whole leaves of the
// global tile sequence (tiles are 64-row blocks x output blocks, row-block-major)
bool wide_xr_exact(int64_t B, int64_t B_total, int64_t b_off, int D) {
  const int nOT1 = D / kOuts;
  if (b_off % kRows) return false;
  const int64_t nT1g = (B_total + kRows - 1) / kRows * nOT1, L = wide_leaf_len(nT1g);
  const int64_t t_lo = b_off / kRows * nOT1, nT1 = (B + kRows - 1) / kRows * nOT1;
  const bool last = b_off + B == B_total;
  return t_lo % L == 0 && (nT1 % L == 0 || last) && (B % kRows == 0 || last);
}

int wide_dopri5_launch(const fetode_kanlinear_t* kan0, const fetode_ferro_t* fer0, const void* plan0,
                       const fetode_kanlinear_t* kan1, const fetode_ferro_t* fer1, const void* plan1, const float* y0,
                       int64_t B, const float* prev0, const float* prev1, uint32_t reinit_mask, const double* t,
                       int32_t T, double rtol, double atol, const double* opts, const float* tableau, float* solution,
                       float* state0, float* state1, void* workspace, int32_t* stats, double* attempts,
                       int32_t max_attempts, const fetode_xrank_t* xr, int64_t B_total, void* stream) {
  if (!kan0 || !fer0 || !kan1 || !fer1) return set_err(FETODE_EUNSUPPORTED, "wide dopri5: needs two KAN-FET layers");
  if (!wide_supported(kan0, fer0) || !wide_supported(kan1, fer1))
    return set_err(FETODE_EUNSUPPORTED, "wide dopri5: a layer has no wide kernel");
  const int D = kan0->in_features, H = kan0->out_features;
  if (kan1->in_features != H || kan1->out_features != D)
    return set_err(FETODE_EINVAL, "wide dopri5: layer 1 must map %d -> %d", H, D);
  if (fer0->num_basis != fer1->num_basis) return set_err(FETODE_EUNSUPPORTED, "wide dopri5: layers with different K");
  if (B <= 0 || T < 1) return set_err(FETODE_EINVAL, "wide dopri5: B and T must be positive");
  if (!plan0 || !plan1 || !y0 || !t || !opts || !tableau || !solution || !state0 || !state1 || !workspace || !stats)
    return set_err(FETODE_EINVAL, "wide dopri5: null pointer");
  if ((!(reinit_mask & 1u) && !prev0) || (!(reinit_mask & 2u) && !prev1))
    return set_err(FETODE_EINVAL, "wide dopri5: null hysteresis state");
  const bool sharded = xr && xr->world > 1;
  const bool exact = sharded && wide_xr_exact(B, B_total, xr->b_offset, D);
  const WideDopriShape sh = wide_dopri_shape(B, D, H, exact ? B_total : 0);
  if ((int64_t)sh.nT0 * sh.S0 > 0x7fffffff / 2) return set_err(FETODE_EINVAL, "wide dopri5: batch too large");
  const int K = fer0->num_basis;
  const void* fn = K == 12 ? (const void*)wide_dopri5_kernel<12> : (const void*)wide_dopri5_kernel<10>;
  // persistent grid: every workgroup resident at once (the phases meet at grid barriers)
  static int per_cu[2] = {0, 0}, n_cu = 0;
  const int fi = K == 12 ? 1 : 0;
  if (!n_cu) {
    int dev = 0;
    HIP_CHECK_RET(hipGetDevice(&dev));
    HIP_CHECK_RET(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (!per_cu[fi]) HIP_CHECK_RET(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[fi], fn, kThreads, 0));
  const int64_t want = std::max<int64_t>((int64_t)sh.nT0 * sh.S0, (int64_t)sh.nT1 * sh.S1);
  int64_t grid = std::min<int64_t>({want, (int64_t)per_cu[fi] * n_cu, (int64_t)kWideDopriMaxGrid});
  static const int64_t grid_cap = [] {  // diagnostics: cap the persistent grid (FETODE_WIDE_DOPRI_GRID)
    const char* e = getenv("FETODE_WIDE_DOPRI_GRID");
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  if (grid_cap > 0) grid = std::min(grid, grid_cap);
  if (grid < 1) return set_err(FETODE_EHIP, "wide dopri5: no resident workgroup");
  WideDopriArgs a{};
  a.l0.plan = (const float*)plan0;
  a.l0.L = wide_layout(kan0, fer0);
  a.l0.grid = kan0->grid;
  a.l0.B = B;
  a.l1.plan = (const float*)plan1;
  a.l1.L = wide_layout(kan1, fer1);
  a.l1.grid = kan1->grid;
  a.l1.B = B;
  a.B = B;
  a.D = D;
  a.H = H;
  a.S0 = sh.S0;
  a.S1 = sh.S1;
  a.nT0 = sh.nT0;
  a.nT1 = sh.nT1;
  a.nOT0 = sh.nOT0;
  a.nOT1 = sh.nOT1;
  a.reinit0 = (reinit_mask & 1u) ? 1 : 0;
  a.reinit1 = (reinit_mask & 2u) ? 1 : 0;
  a.y0 = y0;
  a.prev0 = prev0;
  a.prev1 = prev1;
  a.st0 = state0;
  a.st1 = state1;
  char* ws = (char*)workspace;
  a.bar = (unsigned*)ws;
  a.slot = (double*)(ws + sh.off_slot);
  a.xin = (float*)(ws + sh.off_xin);
  a.hs = (float*)(ws + sh.off_hs);
  a.ks = (float*)(ws + sh.off_ks);
  a.es = (float*)(ws + sh.off_es);
  a.sol = solution;
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
  for (int j = 0; j < 7; ++j) {  // tableau = beta (6 x 6, row i = stage i + 1), c_error (7), c_mid (7)
    for (int q = 0; q < 6; ++q) a.stc[j][q] = (j < 6 && j + q < 6) ? tableau[(j + q) * 6 + j] : 0.0f;
    a.stc[j][6] = tableau[36 + j];
    a.stc[j][7] = tableau[43 + j];
  }
  a.stats = stats;
  a.att = attempts;
  a.max_att = attempts ? max_attempts : 0;
  a.n_el = (double)(sharded ? B_total : B) * D;
  if (exact) {  // leaves of the global tile sequence; this rank's are [leaf_lo, leaf_lo + n_leaf_local)
    const int64_t nT1g = (B_total + kRows - 1) / kRows * sh.nOT1;
    a.leafL = wide_leaf_len(nT1g);
    a.n_leaf = (int)((nT1g + a.leafL - 1) / a.leafL);
    a.leaf_lo = (int)(xr->b_offset / kRows * sh.nOT1 / a.leafL);
  } else {
    a.leafL = wide_leaf_len(sh.nT1);
    a.n_leaf = (sh.nT1 + a.leafL - 1) / a.leafL;
    a.leaf_lo = 0;
  }
  a.n_leaf_local = (sh.nT1 + a.leafL - 1) / a.leafL;
  a.xr_world = sharded ? xr->world : 1;
  if (sharded) {
    a.xr_rank = xr->rank;
    a.xr_exact = exact ? 1 : 0;
    a.xr_epoch = xr->epoch;
    a.xr_peers = (double* const*)xr->peers;
    a.xr_inbox = (double*)xr->inbox;
  }
  hipStream_t s = (hipStream_t)stream;
  HIP_CHECK_RET(hipMemsetAsync(workspace, 0, sizeof(unsigned) * kWBarWords, s));
  void* args[] = {&a};
  HIP_CHECK_RET(resident_launch(fn, dim3((unsigned)grid), dim3(kThreads), args, 0, s));
  return FETODE_OK;
}
}  // namespace

extern "C" {

int64_t fetode_wide_dopri5_workspace(int64_t B, int32_t D, int32_t H) {
  if (B <= 0 || D < 16 || H < 16) return -1;
  return wide_dopri_shape(B, D, H).bytes;
}

int64_t fetode_wide_dopri5_xrank_workspace(int64_t B, int64_t B_total, int64_t b_offset, int32_t D, int32_t H) {
  if (B <= 0 || D < 16 || H < 16 || B_total < B || b_offset < 0 || b_offset + B > B_total) return -1;
  return wide_dopri_shape(B, D, H, wide_xr_exact(B, B_total, b_offset, D) ? B_total : 0).bytes;
}

int fetode_wide_dopri5(const fetode_kanlinear_t* kan0, const fetode_ferro_t* fer0, const void* plan0,
                       const fetode_kanlinear_t* kan1, const fetode_ferro_t* fer1, const void* plan1, const float* y0,
                       int64_t B, const float* prev0, const float* prev1, uint32_t reinit_mask, const double* t,
                       int32_t T, double rtol, double atol, const double* opts, const float* tableau, float* solution,
                       float* state0, float* state1, void* workspace, int32_t* stats, double* attempts,
                       int32_t max_attempts, void* stream) {
  return wide_dopri5_launch(kan0, fer0, plan0, kan1, fer1, plan1, y0, B, prev0, prev1, reinit_mask, t, T, rtol, atol,
                            opts, tableau, solution, state0, state1, workspace, stats, attempts, max_attempts, nullptr,
                            B, stream);
}

int fetode_wide_dopri5_xrank(const fetode_kanlinear_t* kan0, const fetode_ferro_t* fer0, const void* plan0,
                             const fetode_kanlinear_t* kan1, const fetode_ferro_t* fer1, const void* plan1,
                             const float* y0, int64_t B, int64_t B_total, const float* prev0, const float* prev1,
                             uint32_t reinit_mask, const double* t, int32_t T, double rtol, double atol,
                             const double* opts, const float* tableau, float* solution, float* state0, float* state1,
                             void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                             const fetode_xrank_t* xr, void* stream) {
  if (!xr || xr->world < 1 || xr->rank < 0 || xr->rank >= xr->world || xr->world > 64)
    return set_err(FETODE_EINVAL, "wide dopri5 xrank: bad rank / world");
  if (xr->world > 1 && (!xr->peers || !xr->inbox)) return set_err(FETODE_EINVAL, "wide dopri5 xrank: null inbox / peers");
  if (B_total < B || xr->b_offset < 0 || xr->b_offset + B > B_total)
    return set_err(FETODE_EINVAL, "wide dopri5 xrank: shard [%lld, %lld) outside the global batch %lld",
                   (long long)xr->b_offset, (long long)(xr->b_offset + B), (long long)B_total);
  return wide_dopri5_launch(kan0, fer0, plan0, kan1, fer1, plan1, y0, B, prev0, prev1, reinit_mask, t, T, rtol, atol,
                            opts, tableau, solution, state0, state1, workspace, stats, attempts, max_attempts, xr,
                            B_total, stream);
}
}  // extern "C"
