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

constexpr float kWideFactorLimit = 60.0f;  // |gs Ec| bound of the factored gate (header comment)

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
  int64_t fe4;     // (out, in, K) float4 {P = 2^{gs log2e Ec}, 2 log2e k, 2 log2e k Ec, -2 coef Ps}
  int64_t gec;     // (out, in, K) gs log2e Ec (direct form)
  int64_t dflag;   // (out, in) 1 if some |gs Ec| > kWideFactorLimit for (o, i)
  int64_t fconst;  // (out) sum_{i,k} coef (bias + Ps): coef Ps tanh = coef Ps - 2 coef Ps / (1 + e^{2z})
  int64_t wp;      // (in, 20, out) packed KAN weights
  int64_t lg;      // (in, NB, 2) (-a log2e, a b log2e)
  int64_t knots;   // (in, 12) knot grid (efficientkan.py:55-61 buffer)
  int64_t rh;      // (in, 11) 1 / (g[m+1] - g[m])
  int64_t bt;      // (in, 12, 8) float4: basis c on knot interval m as a cubic in u (m = 11: zero)
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
    d[3] = -2.0f * (co * Ps);
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
      s += fl.coef[src] * fl.bias[src] + fl.coef[src] * fl.Ps[src];
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
  int nslice;  // 1, or 2: blockIdx.z takes half of the inputs and adds into a zeroed out
  float* out;
};

// One slice stores; two add into a zeroed out with vector atomics: 0 + a + b in either order is the
// same fp32 value (addition commutes), so the split stays bitwise deterministic.
__device__ __forceinline__ void store_out(float* p, float v, int nslice) {
  if (nslice == 1) *p = v;
  else atomicAdd(p, v);
}

// ---- the layer --------------------------------------------------------------------------------
template <int K, bool KAN, bool FERRO, int kCh>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6))) void wide_layer_kernel(WideArgs a) {
  constexpr int kPitch = pitch_of(kCh);
  static_assert(kCh * kRows <= kThreads && (kCh & 1) == 0, "one staging item per thread, even chunks");
  static_assert(!FERRO || K % 2 == 0, "Ferro elements in (k, k+1) pairs");
  __shared__ float s_x[kCh * kRows], s_w[kCh * kRows], s_e[kCh * kRows];
  __shared__ float s_dfl[kOuts * kCh];
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
  const int64_t b0 = (int64_t)blockIdx.x * kRows;
  const int o0 = blockIdx.y * kOuts;
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
  const int ibeg = blockIdx.z * (in / a.nslice), iend = ibeg + in / a.nslice;
  float xn = slive ? a.x[sb * in + ibeg + si] : 0.f;
  float pn = (FERRO && slive && !a.reinit) ? a.prev[sb * in + ibeg + si] : 0.f;
  for (int i0 = ibeg; i0 < iend; i0 += kCh) {
    const float x = xn, pvl = pn;
    if (i0 + kCh < iend) {
      xn = slive ? a.x[sb * in + i0 + kCh + si] : 0.f;
      pn = (FERRO && slive && !a.reinit) ? a.prev[sb * in + i0 + kCh + si] : 0.f;
    }
    __syncthreads();  // the previous chunk is consumed
    if constexpr (FERRO) {
      const float pv = a.reinit ? x : pvl;
      if (stager) {
      // is_moving_up = sigmoid(gate_slope (x - prev_x)) (ferro_class.py:387), w = wc (1 - up)
      const float up = rcp(1.0f + ex2(-gsl2e * (x - pv)));
      s_x[si * kRows + sr] = x;
      s_w[si * kRows + sr] = wc * (1.0f - up);
      s_e[si * kRows + sr] = ex2(gsl2e * x);
      }
      if (tid < kOuts * kCh) s_dfl[tid] = plan[L.dflag + (int64_t)(o0 + tid / kCh) * in + i0 + tid % kCh];
    }
    if (KAN && stager) {
      const int i = i0 + si;
      float f[kWF];
      f[0] = x * rcp(1.0f + ex2(-x * l2));  // SiLU (efficientkan.py:166)
      // cubic B-spline bases (efficientkan.py:117-131): knot interval m by the half-open order-0
      // indicator, then the 8 bases as cubics of u from the fp64-fitted table (zero outside the grid)
      const float* g = plan + L.knots + (int64_t)i * kNG;
      int m = -1;
#pragma unroll
      for (int j = 0; j < kNG; ++j) m += (x >= g[j]) ? 1 : 0;
      const bool fin = __builtin_isfinite(x);
      const int mi = ((unsigned)m < (unsigned)(kNG - 1) && fin) ? m : kNG - 1;
      const float u = mi < kNG - 1 ? (x - g[mi]) * plan[L.rh + (int64_t)i * (kNG - 1) + mi] : 0.f;
      const float4* bt = reinterpret_cast<const float4*>(plan + L.bt) + ((int64_t)i * kNG + mi) * kNS;
#pragma unroll
      for (int c = 0; c < kNS; ++c) {
        const float4 cf = bt[c];
        f[1 + c] = fin ? ffma(ffma(ffma(cf.w, u, cf.z), u, cf.y), u, cf.x) : __builtin_nanf("");
      }
      const float* lg = plan + L.lg + (int64_t)i * kNB * 2;
#pragma unroll
      for (int j = 0; j < kNB; ++j) f[1 + kNS + j] = rcp(1.0f + ex2(ffma(lg[2 * j], x, lg[2 * j + 1])));
      f[kWF - 1] = 0.f;
      float* d = &s_phi[sr * kPitch + si * kWF];
#pragma unroll
      for (int q = 0; q < kWF; q += 2) *reinterpret_cast<float2*>(d + q) = make_float2(f[q], f[q + 1]);
    }
    __syncthreads();
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
#pragma unroll 2
      for (int ii = 0; ii < kCh; ++ii) {
        const int i = i0 + ii;
        const float xv = s_x[ii * kRows + lane], wg = s_w[ii * kRows + lane], e = s_e[ii * kRows + lane];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          const int jo = kJ * w + j;
          // the element constants are wave-uniform: scalar loads (s_load, SGPR operands) — through
          // LDS they cost a ds_read_b128 per element (Ferro alone 270 -> 230 us at 64 -> 128)
          const float4* par = reinterpret_cast<const float4*>(plan + L.fe4) + ((int64_t)(o0 + jo) * in + i) * K;
          float acc = 0.f;
          if (s_dfl[jo * kCh + ii] == 0.f) {  // wave-uniform
            // elements (k, k+1) in the two halves of packed-fp32 VALU ops (v_pk_fma / mul / add:
            // 3.5 instead of 7 non-transcendental issues per element); even and odd k sum apart
            f2 acc2 = splat(0.0f);
#pragma unroll
            for (int k = 0; k < K; k += 2) {
              const float4 p0 = par[k], p1 = par[k + 1];  // {P, k2, k2Ec, cps}, same address on every lane
              const f2 sg = rcpx2(pfma(splat(e), f2{p0.x, p1.x}, splat(1.0f)));
              const f2 mm = pfma(splat(wg), sg, splat(1.0f));
              const f2 z = pfma(f2{p0.z, p1.z}, mm, f2{p0.y, p1.y} * splat(xv));
              // coef Ps tanh z = coef Ps - 2 coef Ps / (1 + 2^z): the constant part lives in fconst
              acc2 = pfma(f2{p0.w, p1.w}, rcpx2(ex2x2(z) + splat(1.0f)), acc2);
            }
            acc = acc2.x + acc2.y;
          } else {
            const float* gec = plan + L.gec + ((int64_t)(o0 + jo) * in + i) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const float4 p = par[k];
              const float sg = rcp(1.0f + ex2(ffma(gsl2e, xv, gec[k])));
              const float mm = ffma(wg, sg, 1.0f);
              const float z = ffma(p.z, mm, p.y * xv);
              acc = ffma(p.w, rcp(ex2(z) + 1.0f), acc);
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
      s_fer[lane * (kOuts + 1) + kJ * w + j] = facc[j] + (blockIdx.z == 0 ? plan[L.fconst + o0 + kJ * w + j] : 0.f);
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
        if (b < a.B) store_out(&a.out[b * out + o0 + kr], FERRO ? kv + s_fer[r * (kOuts + 1) + kr] : kv, a.nslice);
      }
  } else {
    for (int t = tid; t < kRows * kOuts; t += kThreads) {
      const int r = t / kOuts, c = t % kOuts;
      const int64_t b = b0 + r;
      if (b < a.B) store_out(&a.out[b * out + o0 + c], s_fer[r * (kOuts + 1) + c], a.nslice);
    }
  }
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
  // this lane's element pairs in the kBwdOGW output groups of the block
  f2 Pf[kBwdOGW], k2[kBwdOGW], kk[kBwdOGW], Ecv[kBwdOGW], Psv[kBwdOGW], cov[kBwdOGW], bsv[kBwdOGW];
  f2 gec[kBwdOGW];
  int oo[kBwdOGW];
  bool ok[kBwdOGW], dir[kBwdOGW];
  f2 sk[kBwdOGW], sE[kBwdOGW], sPs[kBwdOGW], sb[kBwdOGW], sc[kBwdOGW];
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
    kk[j] = ok[j] ? f2{a.k[e0], a.k[e0 + 1]} : splat(0.f);
    Ecv[j] = ok[j] ? f2{a.Ec[e0], a.Ec[e0 + 1]} : splat(0.f);
    Psv[j] = ok[j] ? f2{a.Ps[e0], a.Ps[e0 + 1]} : splat(0.f);
    cov[j] = ok[j] ? f2{a.coef[e0], a.coef[e0 + 1]} : splat(0.f);
    bsv[j] = ok[j] ? f2{a.bias[e0], a.bias[e0 + 1]} : splat(0.f);
    gec[j] = ok[j] ? f2{a.plan[L.gec + p0], a.plan[L.gec + p0 + 1]} : splat(0.f);
    dir[j] = ok[j] && a.plan[L.dflag + (int64_t)oo[j] * in + i] != 0.f;
    sk[j] = sE[j] = sPs[j] = sb[j] = sc[j] = splat(0.f);
  }
  bool anydir = false;
#pragma unroll
  for (int j = 0; j < kBwdOGW; ++j) anydir |= __builtin_amdgcn_ballot_w64(dir[j]) != 0;
  float* gxp = a.gxp + (int64_t)ogb * a.B * in;
  for (int64_t b0 = r0; b0 < r1; b0 += 4) {
    const int64_t b = b0 + q;
    const bool live = b < r1;
    const float4 u = live ? a.U[b * in + i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float xv = u.x, e = u.y, omu = u.z, dup = u.w;
    float dx = 0.f;
#pragma unroll
    for (int j = 0; j < kBwdOGW; ++j) {
      const float go = (live && ok[j]) ? a.g[b * out + oo[j]] : 0.f;
      f2 cn;
      if (anydir && dir[j]) cn = rcpx2(ex2x2(pfma(splat(gsl2e), splat(xv), gec[j])) + splat(1.0f));
      else cn = rcpx2(pfma(splat(e), Pf[j], splat(1.0f)));
      const f2 m = pfma(splat(wc * omu), cn, splat(1.0f));
      const f2 sh = pfma(Ecv[j], m, splat(xv));                     // x + Ec m
      const f2 r = rcpx2(ex2x2(k2[j] * sh) + splat(1.0f));          // 2^{2 log2e k sh}
      const f2 th = pfma(splat(-2.0f), r, splat(1.0f));             // tanh = 1 - 2 / (1 + e^{2 k sh})
      const f2 gP = splat(go) * cov[j];
      sc[j] = pfma(splat(go), pfma(Psv[j], th, bsv[j]), sc[j]);
      sPs[j] = pfma(gP, th, sPs[j]);
      sb[j] = sb[j] + gP;
      const f2 gz = gP * Psv[j] * (splat(4.0f) * r * (splat(1.0f) - r));   // 1 - th^2 without cancellation
      sk[j] = pfma(gz, sh, sk[j]);
      const f2 gsh = gz * kk[j];
      const f2 gm = gsh * Ecv[j];
      const f2 dcn = splat(gs) * cn * (splat(1.0f) - cn);
      const f2 t1 = splat(omu) * dcn;
      sE[j] = pfma(gsh, m, sE[j]) - splat(wc) * gm * t1;
      const f2 dxp = gsh - splat(wc) * gm * pfma(cn, splat(dup), t1);
      dx += ok[j] ? dxp.x + dxp.y : 0.f;   // idle lanes: e = inf times P = 0 is NaN
    }
    const float row = row_sum16(dx);
    if (c == 0 && live) gxp[b * in + i] = row;
  }
  // the four row quarters hold the same elements: quarters (0 + 2) + (1 + 3) onto lanes 0..15
  float* pp = a.pp + (int64_t)sgi * in * out * K * 5;
#pragma unroll
  for (int j = 0; j < kBwdOGW; ++j) {
    f2 v[5] = {sk[j], sE[j], sPs[j], sb[j], sc[j]};
#pragma unroll
    for (int t = 0; t < 5; ++t) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float p = h ? v[t].y : v[t].x, qq = p;
        permlane32_swap(p, qq);
        float s2 = p + qq, s3 = s2;
        permlane16_swap(s2, s3);
        const float tot = s2 + s3;
        if (lane < 16 && ok[j]) pp[(((int64_t)i * out + oo[j]) * K + 2 * kp + h) * 5 + t] = tot;
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

FerroBwdPlan ferro_bwd_plan(int in, int out, int K, int64_t B) {
  FerroBwdPlan p{};
  const int kBwdOGW = ferro_bwd_ogw();
  const int OPG = 16 / (K / 2);
  p.n_og = (out + OPG - 1) / OPG;
  p.n_ogb = (p.n_og + kBwdOGW - 1) / kBwdOGW;
  // row segments: enough waves to fill the chip (~8 per SIMD), each at least 256 rows
  const int64_t base = (int64_t)p.n_ogb * in;
  int64_t rs = (8 * 1024 + base - 1) / base;
  const int64_t rmax = (B + 255) / 256;
  rs = rs < rmax ? rs : rmax;
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

// thread per (input i, output o): the row segments in order, then the packing's chain rule
// (wide_pack_kernel: base_weight; spline_weight * spline_scaler; 2 logistic_weight scale_logistic
// logistic_scaler); the d/d(2 sigma) sums d_wl for the logistic_scaler pass
__global__ void wide_kan_grad_kernel(fetode_kanlinear_t kl, const float* __restrict__ pw, int rs,
                                     fetode_kanlinear_grad_t gr, float* __restrict__ d_wl, int accumulate) {
  const int in = kl.in_features, out = kl.out_features;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)in * out) return;
  const int o = (int)(t % out), i = (int)(t / out);
  const int64_t ncol = (int64_t)in * kKF, oi = (int64_t)o * in + i;
  float v[kKF - 1];
#pragma unroll
  for (int f = 0; f < kKF - 1; ++f) {
    float s = 0.f;
    for (int q = 0; q < rs; ++q) s += pw[((int64_t)q * ncol + (int64_t)i * kKF + f) * out + o];
    v[f] = s;
  }
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

// logistic a / b: the row groups in order; logistic_scaler: one wave per output, fixed-order sums
__global__ void wide_kan_ab_ls_kernel(fetode_kanlinear_t kl, const float* __restrict__ abp, int n_rg,
                                      const float* __restrict__ d_wl, fetode_kanlinear_grad_t gr, int accumulate) {
  const int in = kl.in_features, out = kl.out_features;
  const int nab = in * kNB;
  const int nabb = (nab + 255) / 256;
  if ((int)blockIdx.x < nabb) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nab) return;
    float sa = 0.f, sb = 0.f;
    for (int q = 0; q < n_rg; ++q) {
      sa += abp[((int64_t)q * nab + t) * 2];
      sb += abp[((int64_t)q * nab + t) * 2 + 1];
    }
    put_grad(gr.logistic_a ? gr.logistic_a + t : nullptr, sa, accumulate);
    put_grad(gr.logistic_b ? gr.logistic_b + t : nullptr, sb, accumulate);
    return;
  }
  if (!kl.logistic_scaler) return;
  const int o = ((int)blockIdx.x - nabb) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
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
  WideArgs a;
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
  a.nslice = (wgs <= 2 * 256 && (a.L.in / 2) % kChMax == 0) ? 2 : 1;
  if (a.nslice == 2) HIP_CHECK_RET(hipMemsetAsync(out, 0, sizeof(float) * B * a.L.out, (hipStream_t)stream));
  hipLaunchKernelGGL(pick(a.L.K, a.L.kan, a.L.ferro), dim3((unsigned)tiles, (unsigned)(a.L.out / kOuts), (unsigned)a.nslice),
                     dim3(kThreads), 0, (hipStream_t)stream, a);
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
  hipLaunchKernelGGL(wide_kan_grad_kernel, dim3((unsigned)(((int64_t)in * out + 255) / 256)), dim3(256), 0, s, *kl,
                     (const float*)(ws + p.off_pw), p.rs, *grads, ws + p.off_dwl, (int)accumulate);
  LAUNCH_CHECK();
  const int nabb = (in * kNB + 255) / 256;
  hipLaunchKernelGGL(wide_kan_ab_ls_kernel, dim3((unsigned)(nabb + (out + 3) / 4)), dim3(256), 0, s, *kl,
                     (const float*)a.abp, p.n_rg, (const float*)(ws + p.off_dwl), *grads, (int)accumulate);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"

