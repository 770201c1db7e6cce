// fetode_grad.hip — vector-Jacobian products of KANLinear and FerroelectricBasis (any widths).
//
// These are the backward counterparts of the reference's autograd through
//   efficientkan.KANLinear.forward  (efficient_kan/efficientkan.py:160-182)
//   ferro_class.FerroelectricBasis.forward (ferro_class.py:368-420)
// used by the per-stage path (any func) and by the backward of the fused solve
// (train_kanfet_node_predprey.py:254-257: loss.backward() through every RK stage).
// The hysteresis state is a detached snapshot in the reference (:381-382), so no gradient
// flows through prev_x.  Parameter gradients are reduced over the batch inside one
// workgroup per parameter group (fixed order, no atomics): results are run-to-run identical.
#include <cstring>

#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int RB = 256;  // reduction block

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + expf(-z)); }
#ifndef FETODE_GXAB_FAST
#define FETODE_GXAB_FAST 1
#endif

template <int N>
__device__ __forceinline__ void block_sum(float (&v)[N], float* red /* RB*N */) {
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < N; ++q) red[q * RB + t] = v[q];
  __syncthreads();
  for (int s = RB / 2; s > 0; s >>= 1) {
    if (t < s) {
#pragma unroll
      for (int q = 0; q < N; ++q) red[q * RB + t] += red[q * RB + t + s];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < N; ++q) v[q] = red[q * RB];
}

// a workgroup barrier over LDS only: __syncthreads() is also a workgroup-scope fence, which waits
// for every outstanding global load (vmcnt(0)) — including a prefetch meant to cross the barrier
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void put(float* dst, float v, int accumulate) {
  if (dst) *dst = accumulate ? *dst + v : v;
}

// B-spline values and x-derivatives of the SO+1 bases that are non-zero at x (reference
// recursion with divisions; derivative = sum over the recursion of the (x-g)/d factors, i.e.
// SO*(B_{j,SO-1}/(g_{j+SO}-g_j) - B_{j+1,SO-1}/(g_{j+SO+1}-g_{j+1}))).  Returns m (or -1 if
// x is outside the grid; -2 if x is not finite -> NaN everywhere, as the reference's autograd).
template <int SO>
__device__ int bspline_vals_derivs(float x, int NG, const float* __restrict__ g, float* val, float* der) {
#pragma unroll
  for (int r = 0; r <= SO; ++r) val[r] = der[r] = 0.f;
  if (!__builtin_isfinite(x)) {
    for (int r = 0; r <= SO; ++r) val[r] = der[r] = __builtin_nanf("");
    return -2;
  }
  int m = -1;
  for (int j = 0; j < NG; ++j) m += (x >= g[j]) ? 1 : 0;
  if (m < 0 || m > NG - 2) return -1;
  float N[SO + 2];
#pragma unroll
  for (int r = 0; r < SO + 2; ++r) N[r] = 0.f;
  N[SO] = 1.f;
  float P[SO + 2];  // level SO-1
#pragma unroll
  for (int r = 0; r < SO + 2; ++r) P[r] = 0.f;
#pragma unroll
  for (int k = 1; k <= SO; ++k) {
    if (k == SO) {
#pragma unroll
      for (int r = 0; r < SO + 2; ++r) P[r] = N[r];
    }
    float M[SO + 2];
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.f;
#pragma unroll
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= NG - 2 - k) {
        M[r] = ((x - g[j]) / (g[j + k] - g[j])) * N[r] + ((g[j + k + 1] - x) / (g[j + k + 1] - g[j + 1])) * N[r + 1];
      }
    }
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
#pragma unroll
  for (int r = 0; r <= SO; ++r) {
    const int j = m - SO + r;
    val[r] = N[r];
    if (j >= 0 && j <= NG - 2 - SO) {
      const float a = P[r] / (g[j + SO] - g[j]);
      const float b = (r + 1 <= SO) ? P[r + 1] / (g[j + SO + 1] - g[j + 1]) : 0.f;
      der[r] = SO * (a - b);
    }
  }
  return m;
}

// bspline_vals_derivs with the divisions replaced by reciprocal knot spans
// rk[(k-1)*(NG-1)+j] = 1/(g[j+k]-g[j]) (as bspline_local does for the forward head)
template <int SO>
__device__ int bspline_vals_derivs_rk(float x, int NG, const float* __restrict__ g, const float* __restrict__ rk,
                                      float* val, float* der) {
#pragma unroll
  for (int r = 0; r <= SO; ++r) val[r] = der[r] = 0.f;
  if (!__builtin_isfinite(x)) {
    for (int r = 0; r <= SO; ++r) val[r] = der[r] = __builtin_nanf("");
    return -2;
  }
  int m = -1;
  for (int j = 0; j < NG; ++j) m += (x >= g[j]) ? 1 : 0;
  if (m < 0 || m > NG - 2) return -1;
  const int S = NG - 1;
  float N[SO + 2], P[SO + 2];
#pragma unroll
  for (int r = 0; r < SO + 2; ++r) N[r] = P[r] = 0.f;
  N[SO] = 1.f;
#pragma unroll
  for (int k = 1; k <= SO; ++k) {
    if (k == SO) {
#pragma unroll
      for (int r = 0; r < SO + 2; ++r) P[r] = N[r];
    }
    float M[SO + 2];
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.f;
#pragma unroll
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= NG - 2 - k)
        M[r] = ((x - g[j]) * rk[(k - 1) * S + j]) * N[r] + ((g[j + k + 1] - x) * rk[(k - 1) * S + j + 1]) * N[r + 1];
    }
#pragma unroll
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
#pragma unroll
  for (int r = 0; r <= SO; ++r) {
    const int j = m - SO + r;
    val[r] = N[r];
    if (j >= 0 && j <= NG - 2 - SO) {
      const float a = P[r] * rk[(SO - 1) * S + j];
      const float b = (r + 1 <= SO) ? P[r + 1] * rk[(SO - 1) * S + j + 1] : 0.f;
      der[r] = SO * (a - b);
    }
  }
  return m;
}

// ------------------------------------------------------------------------------------------
// KANLinear
// ------------------------------------------------------------------------------------------

constexpr int kMaxLogistic = 16;
// gx[b,i] (+)= sum_o g[b,o] d out[b,o] / d x[b,i]
template <int SO>
__global__ void kan_gx_kernel(fetode_kanlinear_t kl, const float* __restrict__ x, const float* __restrict__ g,
                              int64_t B, float* __restrict__ gx, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, out = kl.out_features, NB = kl.num_logistic;
  const int NG = kl.grid_size + 2 * SO + 1, NS = kl.grid_size + SO;
  if (t >= B * in) return;
  const int64_t b = t / in;
  const int i = t % in;
  const float xv = x[t];
  const float sg = sigm(xv);
  const float dsilu = sg * (1.0f + xv * (1.0f - sg));
  float val[SO + 1], der[SO + 1];
  const int m = bspline_vals_derivs<SO>(xv, NG, kl.grid + (int64_t)i * NG, val, der);
  float dphi[kMaxLogistic];  // d phi_j / d x, once per (b, i) rather than per output
  for (int j = 0; j < NB && j < kMaxLogistic; ++j) {
    const float a = kl.logistic_a[i * NB + j], bb = kl.logistic_b[i * NB + j];
    const float sj = sigm(a * (xv - bb));
    dphi[j] = 2.0f * sj * (1.0f - sj) * a;
  }
  float acc = 0.f;
  for (int o = 0; o < out; ++o) {
    const float go = g[b * out + o];
    float d = kl.base_weight[o * in + i] * dsilu;
    const float sc = kl.spline_scaler ? kl.spline_scaler[o * in + i] : 1.0f;
    const float* sw = kl.spline_weight + ((int64_t)o * in + i) * NS;
    if (m >= 0) {
      for (int r = 0; r <= SO; ++r) {
        const int j = m - SO + r;
        if (j >= 0 && j < NS) d += (sw[j] * sc) * der[r];
      }
    } else if (m == -2) {
      d = __builtin_nanf("");
    }
    if (NB > 0) {
      const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      for (int j = 0; j < NB; ++j) {
        const float w = (kl.logistic_weight[(int64_t)o * in * NB + i * NB + j] * kl.scale_logistic) * ls;
        float dj;
        if (j < kMaxLogistic) {
          dj = dphi[j];
        } else {
          const float a = kl.logistic_a[i * NB + j], bb = kl.logistic_b[i * NB + j];
          const float sj = sigm(a * (xv - bb));
          dj = 2.0f * sj * (1.0f - sj) * a;
        }
        d += w * dj;
      }
    }
    acc += go * d;
  }
  gx[t] = accumulate ? gx[t] + acc : acc;
}

// one block per (o, i, f): f = 0 base weight, 1..NS scaled spline weight c = f-1, NS+1.. W' (logistic)
template <int SO>
__global__ void kan_gw_kernel(fetode_kanlinear_t kl, const float* __restrict__ x, const float* __restrict__ g,
                              int64_t B, float* __restrict__ d_scaled /* (out,in,NS) scratch */,
                              float* __restrict__ d_wl /* (out,in*NB) scratch */, fetode_kanlinear_grad_t gr,
                              int accumulate) {
  __shared__ float red[RB];
  const int in = kl.in_features, out = kl.out_features, NB = kl.num_logistic;
  const int NG = kl.grid_size + 2 * SO + 1, NS = kl.grid_size + SO, NF = 1 + NS + NB;
  const int blk = blockIdx.x;
  const int o = blk / (in * NF), r = blk % (in * NF), i = r / NF, f = r % NF;
  float s[1] = {0.f};
  for (int64_t b = threadIdx.x; b < B; b += RB) {
    const float xv = x[b * in + i], go = g[b * out + o];
    float v;
    if (f == 0) {
      v = xv * sigm(xv);
    } else if (f <= NS) {
      float val[SO + 1], der[SO + 1];
      const int m = bspline_vals_derivs<SO>(xv, NG, kl.grid + (int64_t)i * NG, val, der);
      const int c = f - 1;
      v = 0.f;
      if (m == -2) v = __builtin_nanf("");
#pragma unroll
      for (int rr = 0; rr <= SO; ++rr)
        if (m >= 0 && m - SO + rr == c) v = val[rr];
    } else {
      const int j = f - 1 - NS;
      v = 2.0f / (1.0f + expf(-kl.logistic_a[i * NB + j] * (xv - kl.logistic_b[i * NB + j])));
    }
    s[0] += go * v;
  }
  block_sum(s, red);
  if (threadIdx.x == 0) {
    if (f == 0) put(gr.base_weight ? gr.base_weight + o * in + i : nullptr, s[0], accumulate);
    else if (f <= NS) d_scaled[((int64_t)o * in + i) * NS + (f - 1)] = s[0];
    else d_wl[(int64_t)o * in * NB + i * NB + (f - 1 - NS)] = s[0];
  }
}


// ------------------------------------------------------------------------------------------
// Wide layers (the MNIST head, 1568 -> 10; fetode_kanlinear_wide_supported): the weight
// gradients are one contraction over the batch, D[i, f, o] = sum_b feat_f(x[b, i]) g[b, o], on
// v_mfma_f32_16x16x4_f32 — A = features (lane (f, row-quad)), B = g (lane (row-quad, o)) — with
// the 17 features of each (row, input) computed once into LDS (the generic kan_gw_kernel computes
// them per (o, i, f) block: 170x).  A workgroup owns 4 inputs and a quarter of the batch (64-row
// chunks); the quarters add in a fixed order in wide_gw_reduce_kernel.
// ------------------------------------------------------------------------------------------
constexpr int kGwSplit = 4, kGwNS = 8, kGwNB = 8, kGwF = 1 + kGwNS + kGwNB, kGwNG = 12;
typedef float gw_f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void wide_gw_kernel(fetode_kanlinear_t kl, const float* __restrict__ x,
                                                     const float* __restrict__ g, int64_t B,
                                                     float* __restrict__ dpart) {
  // feature rows at a pitch of 66: the MFMA A operand reads Fs[wv][m][col] for the 16 features m of
  // a half-wave at once — at a pitch of 64 all 16 hit one bank (16-way; 64 % of the kernel's LDS
  // cycles were conflicts, profiles/r06_lds_bench_nores.txt); at 66, 2 m + col covers 32 banks
  __shared__ float Fs[4][kGwF][66];
  __shared__ float gs[64][16];
  __shared__ float gk[4][kGwNG];
  __shared__ float rk[4][3 * (kGwNG - 1)];  // 1 / (g[j+k] - g[j]) (bspline_local)
  __shared__ float lab[4][2 * kGwNB];       // -a log2(e) | b
  const int in = kl.in_features, out = kl.out_features;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i0 = blockIdx.x * 4;
  const int sp = blockIdx.y;
  const int64_t nch = (B + 63) / 64;
  const int64_t c0 = sp * nch / kGwSplit, c1 = (sp + 1) * nch / kGwSplit;
  const bool lg = kl.num_logistic != 0;
  if (tid < 4 * kGwNG) gk[tid / kGwNG][tid % kGwNG] = kl.grid[(int64_t)i0 * kGwNG + tid];
  if (tid < 4 * 3 * (kGwNG - 1)) {
    const int ii = tid / (3 * (kGwNG - 1)), q = tid % (3 * (kGwNG - 1)), k = q / (kGwNG - 1) + 1, j = q % (kGwNG - 1);
    const float* gg = kl.grid + (int64_t)(i0 + ii) * kGwNG;
    rk[ii][q] = j + k < kGwNG ? 1.0f / (gg[j + k] - gg[j]) : 0.f;
  }
  if (lg && tid < 4 * kGwNB) {
    lab[tid / kGwNB][tid % kGwNB] = -kl.logistic_a[(int64_t)i0 * kGwNB + tid] * FETODE_LOG2E;
    lab[tid / kGwNB][kGwNB + tid % kGwNB] = kl.logistic_b[(int64_t)i0 * kGwNB + tid];
  }
  gw_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  // the next chunk's x and g tile are fetched into registers while the current chunk computes
  float gnx[4], xnx = 0.f;
  auto fetch = [&](int64_t c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = tid + 256 * k, rr = t / 16, o = t % 16;
      const int64_t bb = c * 64 + rr;
      gnx[k] = (bb < B && o < out) ? g[bb * out + o] : 0.f;
    }
    const int64_t bl = c * 64 + lane;
    xnx = bl < B ? x[bl * in + i0 + wv] : 0.f;
  };
  if (c0 < c1) fetch(c0);
  for (int64_t c = c0; c < c1; ++c) {
    const int64_t b = c * 64 + lane;
    __syncthreads();
    const float xcur = xnx;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = tid + 256 * k;
      gs[t / 16][t % 16] = gnx[k];
    }
    if (c + 1 < c1) fetch(c + 1);
    {  // features of (row b, input i0 + wv)
      const bool ok = b < B;
      const float xv = xcur;
      // the forward head's feature forms (fetode_mnist.hip wide_fwd_kernel): v_exp / v_rcp, spans
      Fs[wv][0][lane] = ok ? silu(xv) : 0.f;   // the reference's base branch SiLU(x)
      // the spline rows written in place (zeros, then the active bases over them)
      bspline_local<3>(xv, kGwNG, &gk[wv][0], &rk[wv][0], [&](int cc, float v) { Fs[wv][1 + cc][lane] = ok ? v : 0.f; });
#pragma unroll
      for (int j = 0; j < kGwNB; ++j)
        Fs[wv][1 + kGwNS + j][lane] =
            (ok && lg) ? 2.0f * sig_from_neg_l2((xv - lab[wv][kGwNB + j]) * lab[wv][j]) : 0.f;
    }
    __syncthreads();
    const int m = lane & 15, kq = lane >> 4;
#pragma unroll 4
    for (int kt = 0; kt < 16; ++kt) {
      const float bo = gs[4 * kt + kq][m];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Fs[wv][m][4 * kt + kq], bo, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(m == 0 ? Fs[wv][16][4 * kt + kq] : 0.f, bo, acc1, 0, 0, 0);
    }
  }
  // D: lane holds rows (features) 4 (lane >> 4) + v, column (output) lane & 15
  const int o = lane & 15, i = i0 + wv;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int f = 4 * (lane >> 4) + v;
    dpart[(((int64_t)sp * in + i) * kGwF + f) * 16 + o] = acc0[v];
    if (f == 0) dpart[(((int64_t)sp * in + i) * kGwF + 16) * 16 + o] = acc1[v];
  }
}


// d x and d (logistic a, b) of a wide layer in one pass over the batch: per (row, input)
// G_f = sum_o g[b, o] W_f[i, o] (the packed weights of 4 inputs staged in LDS, one input per
// wave: broadcast reads), then d x = sum_f G_f d feat_f / d x and the logistic bases' a / b sums
// (per-lane partials -> wave sum in a fixed order -> per-split slots -> wide_ab_reduce_kernel).
// NO: outputs walked per (row, input) — 12 when out <= 12 (the MNIST head's 10), else 16
template <int NO>
__global__ __launch_bounds__(256) void wide_gxab_kernel(fetode_kanlinear_t kl, const float* __restrict__ x,
                                                       const float* __restrict__ g, int64_t B, float* __restrict__ gx,
                                                       float* __restrict__ abpart, int accumulate) {
  __shared__ float wts[4][kGwF][16];
  __shared__ float gs[64][17];
  __shared__ float gk[4][kGwNG];
  __shared__ float rk[4][3 * (kGwNG - 1)];  // reciprocal knot spans (bspline_vals_derivs_rk)
  __shared__ float lab[4][2 * kGwNB];
  const int in = kl.in_features, out = kl.out_features;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i0 = blockIdx.x * 4, i = i0 + wv;
  const int sp = blockIdx.y;
  const int64_t nch = (B + 63) / 64;
  const int64_t c0 = sp * nch / kGwSplit, c1 = (sp + 1) * nch / kGwSplit;
  const bool lg = kl.num_logistic != 0;
  for (int t = tid; t < 4 * kGwF * 16; t += 256) {
    const int ii = t / (kGwF * 16), f = (t / 16) % kGwF, o = t % 16;
    const int iv = i0 + ii;
    float v = 0.f;
    if (o < out) {
      if (f == 0) {
        v = kl.base_weight[(int64_t)o * in + iv];
      } else if (f <= kGwNS) {
        const float sc = kl.spline_scaler ? kl.spline_scaler[(int64_t)o * in + iv] : 1.0f;
        v = kl.spline_weight[((int64_t)o * in + iv) * kGwNS + (f - 1)] * sc;
      } else if (lg) {
        const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
        v = (kl.logistic_weight[(int64_t)o * in * kGwNB + iv * kGwNB + (f - 1 - kGwNS)] * kl.scale_logistic) * ls;
      }
    }
    wts[ii][f][o] = v;
  }
  if (tid < 4 * kGwNG) gk[tid / kGwNG][tid % kGwNG] = kl.grid[(int64_t)i0 * kGwNG + tid];
  if (tid < 4 * 3 * (kGwNG - 1)) {
    const int ii = tid / (3 * (kGwNG - 1)), q = tid % (3 * (kGwNG - 1)), k = q / (kGwNG - 1) + 1, j = q % (kGwNG - 1);
    const float* gg = kl.grid + (int64_t)(i0 + ii) * kGwNG;
    rk[ii][q] = j + k < kGwNG ? 1.0f / (gg[j + k] - gg[j]) : 0.f;
  }
  if (lg && tid < 4 * kGwNB) {
    lab[tid / kGwNB][tid % kGwNB] = kl.logistic_a[(int64_t)i0 * kGwNB + tid];
    lab[tid / kGwNB][kGwNB + tid % kGwNB] = kl.logistic_b[(int64_t)i0 * kGwNB + tid];
  }
  float ga[kGwNB], gb[kGwNB];
#pragma unroll
  for (int j = 0; j < kGwNB; ++j) ga[j] = gb[j] = 0.f;
  // the next chunk's g tile (4 values per thread) and x are loaded while the current chunk is
  // computed (their global-load latency was exposed once per chunk: ~half the wave cycles waiting)
  float gnx[4], xnx = 0.f;
  auto fetch = [&](int64_t c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = tid + 256 * k, rr = t / 16, o = t % 16;
      const int64_t bb = c * 64 + rr;
      gnx[k] = (bb < B && o < out) ? g[bb * out + o] : 0.f;
    }
    const int64_t bl = c * 64 + lane;
    xnx = bl < B ? x[bl * in + i] : 0.f;
  };
  if (c0 < c1) fetch(c0);
  for (int64_t c = c0; c < c1; ++c) {
    __syncthreads();  // the previous chunk's tile is consumed
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = tid + 256 * k;
      gs[t / 16][t % 16] = gnx[k];
    }
    const float xv = xnx;
    if (c + 1 < c1) fetch(c + 1);
    __syncthreads();
    const int64_t b = c * 64 + lane;
    if (b >= B) continue;
    float go[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) go[o] = gs[lane][o];
    // G_f = sum_o g[b, o] W_f[i, o] for the SiLU and logistic features; of the spline features only
    // the (at most 4) bases active at x are formed, below (the others multiply a zero derivative)
    auto gdot = [&](int f) __attribute__((always_inline)) {
      float acc = 0.f;
#pragma unroll
      for (int o = 0; o < NO; ++o) acc = __builtin_fmaf(go[o], wts[wv][f][o], acc);
      return acc;
    };
    float G[kGwF];
    G[0] = gdot(0);
#pragma unroll
    for (int f = 1 + kGwNS; f < kGwF; ++f) G[f] = gdot(f);
#if FETODE_GXAB_FAST  // v_exp / v_rcp sigmoids (1 ulp), as the forward head (wide_fwd_kernel)
    const float sg = sig_from_neg_l2(-xv * FETODE_LOG2E);
#else
    const float sg = sigm(xv);
#endif
    float d = G[0] * (sg * (1.0f + xv * (1.0f - sg)));
    float val[4], der[4];
    const int m = bspline_vals_derivs_rk<3>(xv, kGwNG, gk[wv], rk[wv], val, der);
    if (m >= 0) {
#pragma unroll
      for (int r = 0; r <= 3; ++r) {
        const int cc = m - 3 + r;   // spline basis cc, when 0 <= cc < NS
        if ((unsigned)cc < (unsigned)kGwNS) d += gdot(1 + cc) * der[r];
      }
    } else if (m == -2) {
      d = __builtin_nanf("");
    }
    if (lg) {
#pragma unroll
      for (int j = 0; j < kGwNB; ++j) {
        const float a = lab[wv][j], bj = lab[wv][kGwNB + j];
#if FETODE_GXAB_FAST
        const float sj = sig_from_neg_l2((a * (xv - bj)) * -FETODE_LOG2E);
#else
        const float sj = sigm(a * (xv - bj));
#endif
        const float dz = G[1 + kGwNS + j] * (2.0f * sj * (1.0f - sj));
        d += dz * a;
        ga[j] += dz * (xv - bj);
        gb[j] += dz * (-a);
      }
    }
    if (gx) gx[b * in + i] = accumulate ? gx[b * in + i] + d : d;
  }
  if (abpart && lg) {
#pragma unroll
    for (int j = 0; j < kGwNB; ++j) {
      float va = ga[j], vb = gb[j];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        va += __shfl_xor(va, o);
        vb += __shfl_xor(vb, o);
      }
      if (lane == 0) {
        abpart[(((int64_t)sp * in + i) * kGwNB + j) * 2 + 0] = va;
        abpart[(((int64_t)sp * in + i) * kGwNB + j) * 2 + 1] = vb;
      }
    }
  }
}

__global__ void wide_ab_reduce_kernel(fetode_kanlinear_t kl, const float* __restrict__ abpart, fetode_kanlinear_grad_t gr,
                                      int accumulate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features;
  if (t >= in * kGwNB) return;
  float va = abpart[(int64_t)t * 2], vb = abpart[(int64_t)t * 2 + 1];
  for (int sp = 1; sp < kGwSplit; ++sp) {
    va = va + abpart[((int64_t)sp * in * kGwNB + t) * 2];
    vb = vb + abpart[((int64_t)sp * in * kGwNB + t) * 2 + 1];
  }
  put(gr.logistic_a ? gr.logistic_a + t : nullptr, va, accumulate);
  put(gr.logistic_b ? gr.logistic_b + t : nullptr, vb, accumulate);
}

// the splits in order -> base-weight gradient, d_scaled (spline), d_wl (logistic) as kan_gw_kernel
__global__ void wide_gw_reduce_kernel(fetode_kanlinear_t kl, const float* __restrict__ dpart, float* __restrict__ d_scaled,
                                      float* __restrict__ d_wl, fetode_kanlinear_grad_t gr, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, out = kl.out_features;
  if (t >= (int64_t)out * in * kGwF) return;
  const int f = (int)(t % kGwF);
  const int64_t oi = t / kGwF;
  const int o = (int)(oi / in), i = (int)(oi % in);
  float v = dpart[(((int64_t)0 * in + i) * kGwF + f) * 16 + o];
  for (int sp = 1; sp < kGwSplit; ++sp) v = v + dpart[(((int64_t)sp * in + i) * kGwF + f) * 16 + o];
  if (f == 0) put(gr.base_weight ? gr.base_weight + (int64_t)o * in + i : nullptr, v, accumulate);
  else if (f <= kGwNS) d_scaled[((int64_t)o * in + i) * kGwNS + (f - 1)] = v;
  else if (kl.num_logistic) d_wl[(int64_t)o * in * kGwNB + i * kGwNB + (f - 1 - kGwNS)] = v;
}

// chain rule of the scaled weights: spline_weight, spline_scaler, logistic_weight, logistic_scaler
__global__ void kan_scale_grads_kernel(fetode_kanlinear_t kl, const float* __restrict__ d_scaled,
                                       const float* __restrict__ d_wl, fetode_kanlinear_grad_t gr, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, out = kl.out_features, NB = kl.num_logistic;
  const int NS = kl.grid_size + kl.spline_order;
  if (t < (int64_t)out * in) {
    const int o = t / in, i = t % in;
    const float sc = kl.spline_scaler ? kl.spline_scaler[t] : 1.0f;
    float dsc = 0.f;
    for (int c = 0; c < NS; ++c) {
      const float ds = d_scaled[(int64_t)t * NS + c];
      put(gr.spline_weight ? gr.spline_weight + (int64_t)t * NS + c : nullptr, ds * sc, accumulate);
      dsc += ds * kl.spline_weight[(int64_t)t * NS + c];
    }
    if (kl.spline_scaler) put(gr.spline_scaler ? gr.spline_scaler + t : nullptr, dsc, accumulate);
    (void)o;
    (void)i;
  }
  if (NB > 0 && t < (int64_t)out * in * NB) {   // one thread per logistic weight
    const int o = (int)(t / ((int64_t)in * NB));
    const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
    put(gr.logistic_weight ? gr.logistic_weight + t : nullptr, (d_wl[t] * ls) * kl.scale_logistic, accumulate);
  }
}

// d logistic_scaler[o] = sum_q dW'[o, q] (W[o, q] scale): a fixed-order sum per output
__global__ void kan_scale_ls_kernel(fetode_kanlinear_t kl, const float* __restrict__ d_wl, fetode_kanlinear_grad_t gr,
                                    int accumulate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, NB = kl.num_logistic;
  if (t >= kl.out_features) return;
  float dls = 0.f;
  for (int q = 0; q < in * NB; ++q)
    dls += d_wl[(int64_t)t * in * NB + q] * (kl.logistic_weight[(int64_t)t * in * NB + q] * kl.scale_logistic);
  put(gr.logistic_scaler ? gr.logistic_scaler + t : nullptr, dls, accumulate);
}

// The cubic B-spline bases of one input as per-interval polynomials in u = (x - g[m]) / (g[m+1] -
// g[m]): bp[m * 4 + r] = the power-basis coefficients of B_{m-3+r} on interval m — Cox-de Boor
// (efficientkan.py:117-131) restricted to interval m, evaluated in fp64 at u = 0, 1/3, 2/3, 1 and
// converted (exact for cubics; fetode_bwd.hip BInTab builds the same tables).  A row's four
// bases are then four float4 reads at its interval and a Horner each, instead of the recursion's
// chain of knot reads.  Entry q of the NI x 4 table (one thread per entry).
__device__ float4 bpoly_entry(const float* __restrict__ g, int NG, int q) {
  constexpr int SO = 3;
  const int m = q / 4, r = q % 4;
  const double h = (double)g[m + 1] - g[m];
  double v[4];
  for (int s = 0; s < 4; ++s) {
    const double x = g[m] + h * (s / 3.0);
    double N[SO + 2];
    for (int t = 0; t < SO + 2; ++t) N[t] = 0.0;
    N[SO] = 1.0;
    for (int k = 1; k <= SO; ++k) {
      double M[SO + 2];
      for (int t = 0; t < SO + 2; ++t) M[t] = 0.0;
      for (int t = SO - k; t <= SO; ++t) {
        const int j = m - SO + t;
        if (j >= 0 && j <= NG - 2 - k)
          M[t] = (x - g[j]) / ((double)g[j + k] - g[j]) * N[t] +
                 ((double)g[j + k + 1] - x) / ((double)g[j + k + 1] - g[j + 1]) * N[t + 1];
      }
      for (int t = 0; t < SO + 2; ++t) N[t] = M[t];
    }
    v[s] = N[r];
  }
  return make_float4((float)v[0], (float)((-11.0 * v[0] + 18.0 * v[1] - 9.0 * v[2] + 2.0 * v[3]) / 2.0),
                     (float)(9.0 * (2.0 * v[0] - 5.0 * v[1] + 4.0 * v[2] - v[3]) / 2.0),
                     (float)(9.0 * (-v[0] + 3.0 * v[1] - 3.0 * v[2] + v[3]) / 2.0));
}

// every input's table once per launch (the many-row kernels stage their inputs' rows from it)
__global__ void bpoly_build_kernel(fetode_kanlinear_t kl, float4* __restrict__ tab) {
  const int NG = kl.grid_size + 2 * kl.spline_order + 1, per = (NG - 1) * 4;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < kl.in_features * per) tab[t] = bpoly_entry(kl.grid + (int64_t)(t / per) * NG, NG, t % per);
}

// a row's interval m (-1: off the grid, -2: not finite) and its four basis values from the tables
__device__ __forceinline__ int bpoly_vals(float x, int NG, const float* __restrict__ kn, const float* __restrict__ rh,
                                          const float4* __restrict__ bp, float* val) {
  constexpr int SO = 3;
#pragma unroll
  for (int r = 0; r <= SO; ++r) val[r] = 0.f;
  if (!__builtin_isfinite(x)) {
#pragma unroll
    for (int r = 0; r <= SO; ++r) val[r] = __builtin_nanf("");
    return -2;
  }
  int m = -1;
  for (int j = 0; j < NG; ++j) m += (x >= kn[j]) ? 1 : 0;
  if (m < 0 || m > NG - 2) return -1;
  const float u = (x - kn[m]) * rh[m];
  float4 p[SO + 1];
#pragma unroll
  for (int r = 0; r <= SO; ++r) p[r] = bp[m * 4 + r];
#pragma unroll
  for (int r = 0; r <= SO; ++r) val[r] = ffma(ffma(ffma(p[r].w, u, p[r].z), u, p[r].y), u, p[r].x);
  return m;
}

// ------------------------------------------------------------------------------------------
// Parameter sums over many rows (B >= kPsMinRows: the fieldn training pass runs them over every
// (evaluation, trajectory) row, fetode_fieldn_bwd.hip): workgroup (input group, row split s) walks
// tiles of kPsTile rows.  Every thread forms the NF features of one (row, input) of the group ONCE
// (kan_gw_kernel forms them once per (o, i, f) block: out * NF times) while the NEXT tile's x and
// g are already in flight (the walk is latency-bound otherwise: two dependent global round trips
// per tile); then every thread sums a 4 x 4 block of (feature, output) products of one input over
// its share of the tile's rows; the logistic a / b sums ride along per (row, input).  Per-thread
// partials -> fixed-order workgroup sums -> per-split slots -> kan_psum_reduce_kernel sums the
// splits in order (run-to-run identical).
// ------------------------------------------------------------------------------------------
constexpr int kPsTile = 64, kPsMaxNF = 40, kPsMaxOut = 64, kPsMinRows = 2048, kPsBlocks = 2048, kPsMaxIG = 4;
constexpr int kPsGReg = kPsTile / 4;  // g values a thread stages per tile (a column of every 4th row)
// inputs per workgroup: up to 4, as long as the (input, feature block, output block) triples fit 256 threads
__host__ __device__ inline int ps_ig(int in, int NF, int out) {
  const int fo = ((NF + 3) / 4) * ((out + 3) / 4);
  int ig = in < kPsMaxIG ? in : kPsMaxIG;
  while (ig > 1 && ig * fo > 256) --ig;
  return ig;
}
int ps_nf(const fetode_kanlinear_t* kl) { return 1 + kl->grid_size + kl->spline_order + kl->num_logistic; }
int ps_groups(const fetode_kanlinear_t* kl) {
  const int ig = ps_ig(kl->in_features, ps_nf(kl), kl->out_features);
  return (kl->in_features + ig - 1) / ig;
}
int ps_smax(const fetode_kanlinear_t* kl) { return kPsBlocks / ps_groups(kl) > 1 ? kPsBlocks / ps_groups(kl) : 1; }
int ps_splits(const fetode_kanlinear_t* kl, int64_t B) {
  int64_t S = ps_smax(kl);
  const int64_t tiles = (B + kPsTile - 1) / kPsTile;
  if (S > tiles) S = tiles;
  return S < 1 ? 1 : (int)S;
}
size_t ps_lds_bytes(const fetode_kanlinear_t* kl) {
  const int NF = ps_nf(kl), out = kl->out_features, ig = ps_ig(kl->in_features, NF, out);
  const int NG = kl->grid_size + 2 * kl->spline_order + 1;
  const int64_t n = (int64_t)ig * (NG - 1) * 16 + (int64_t)ig * kPsTile * (NF | 1) + (int64_t)kPsTile * (out | 1) +
                    (int64_t)ig * out * ((kl->num_logistic + 3) & ~3) + (int64_t)ig * (NG + (NG - 1) + 3 * kl->num_logistic);
  return sizeof(float) * (size_t)(n > 256 * 16 ? n : 256 * 16);
}

template <int SO, bool LOG>
__global__ __launch_bounds__(256) void kan_psum_kernel(fetode_kanlinear_t kl, const float* __restrict__ x,
                                                      const float* __restrict__ g, int64_t B,
                                                      const float4* __restrict__ bpt /* (in, NG - 1, 4) */,
                                                      float* __restrict__ part /* (S, in, NF, out) */,
                                                      float* __restrict__ abpart /* (S, in, NB, 2) */) {
  extern __shared__ float ps_lds[];
  const int in = kl.in_features, out = kl.out_features, NB = LOG ? kl.num_logistic : 0;
  const int NG = kl.grid_size + 2 * SO + 1, NS = kl.grid_size + SO, NF = 1 + NS + NB;
  const int IG = ps_ig(in, NF, out), i0 = blockIdx.x * IG, ni = in - i0 < IG ? in - i0 : IG;
  const int s = blockIdx.y, S = gridDim.y, tid = threadIdx.x;
  // odd row strides: a thread per row reads its row's g (logistic a / b) without bank conflicts
  const int FS = NF | 1, GS = out | 1;
  const int NBP = (NB + 3) & ~3;                   // W' rows padded to float4s
  float4* bp = reinterpret_cast<float4*>(ps_lds);  // [IG][NG - 1][4] basis cubics (bpoly_entry)
  float* wl = ps_lds + IG * (NG - 1) * 16;     // [IG][out][NBP] (16-byte aligned rows)
  float* ft = wl + IG * out * NBP;             // [IG * kPsTile][FS]: (input, row) features
  float* gt = ft + IG * kPsTile * FS;          // [kPsTile][GS]
  float* kn = gt + kPsTile * GS;               // [IG][NG] knots
  float* rh = kn + IG * NG;                    // [IG][NG - 1] 1 / knot steps
  float* lab = rh + IG * (NG - 1);             // [IG][NB][3] logistic (-a log2e, b, a)
  float* red = ps_lds;                         // the workgroup sums, after the walk
  const int64_t tiles = (B + kPsTile - 1) / kPsTile;
  const int64_t t0 = s * tiles / S, t1 = (s + 1) * tiles / S;
  // the logistic weights W'[o, (i, j)] of the group's inputs (a / b sums)
  for (int q = tid; LOG && q < ni * out * NBP; q += 256) {
    const int ig = q / (out * NBP), o = (q / NBP) % out, j = q % NBP;
    const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
    wl[q] = j < NB ? (kl.logistic_weight[(int64_t)o * in * NB + (i0 + ig) * NB + j] * kl.scale_logistic) * ls : 0.f;
  }
  // the group's knots, 1 / knot steps, basis cubics (bpoly_entry, from the launch's table) and
  // logistic parameters
  for (int q = tid; q < ni * NG; q += 256) kn[q] = kl.grid[(int64_t)(i0 + q / NG) * NG + q % NG];
  for (int q = tid; q < ni * (NG - 1); q += 256) {
    const float* gg = kl.grid + (int64_t)(i0 + q / (NG - 1)) * NG;
    rh[q] = 1.0f / (gg[q % (NG - 1) + 1] - gg[q % (NG - 1)]);
  }
  for (int q = tid; q < ni * (NG - 1) * 4; q += 256) bp[q] = bpt[(int64_t)i0 * (NG - 1) * 4 + q];
  for (int q = tid; LOG && q < ni * NB; q += 256) {
    lab[3 * q] = -kl.logistic_a[i0 * NB + q] * FETODE_LOG2E;
    lab[3 * q + 1] = kl.logistic_b[i0 * NB + q];
    lab[3 * q + 2] = kl.logistic_a[i0 * NB + q];
  }
  // feature role: (input fig, row frr) of each tile
  const int fig = tid / kPsTile, frr = tid % kPsTile;
  const bool fe = fig < ni;
  const int fin = i0 + (fe ? fig : 0);
  const float* gi = kn + (fe ? fig : 0) * NG;
  const float* rhi = rh + (fe ? fig : 0) * (NG - 1);
  const float4* bpi = bp + (fe ? fig : 0) * (NG - 1) * 4;
  const float* labi = lab + (fe ? fig : 0) * 3 * NB;
  // sum role: a (input, feature block, output block) triple and a share of the tile's rows
  const int FBK = (NF + 3) / 4, OBK = (out + 3) / 4, P = ni * FBK * OBK, Q = P < 256 ? 256 / P : 1;
  const int p = tid % P, q = tid / P;
  const bool act = tid < P * Q;
  const int pig = p / (FBK * OBK), f0 = 4 * ((p / OBK) % FBK), o0 = 4 * (p % OBK);
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = 0.f;
  constexpr int NL = LOG ? kMaxLogistic : 1;
  float la[NL], lb[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) la[j] = lb[j] = 0.f;
  // the next tile's x (this thread's row / input) and g (its share of the tile) in registers
  float xn = 0.f, gn[kPsGReg];
  const int gc = tid & 63, gr0 = tid >> 6;  // g staging: column gc of rows gr0, gr0 + 4, ...
  auto fetch = [&](int64_t tl) {
    const int64_t r0 = tl * kPsTile;
    xn = (fe && r0 + frr < B) ? x[(r0 + frr) * in + fin] : 0.f;
#pragma unroll
    for (int k = 0; k < kPsGReg; ++k) {  // row gr0 + 4 k, column gc
      const int64_t r = r0 + gr0 + 4 * k;
      gn[k] = (gc < out && r < B) ? g[r * out + gc] : 0.f;
    }
  };
  if (t0 < t1) fetch(t0);
  for (int64_t tl = t0; tl < t1; ++tl) {
    const int64_t r0 = tl * kPsTile;
    const bool live = fe && r0 + frr < B;
    const float xv = xn;
    lds_barrier();  // the previous tile's reads are done (the next tile's loads stay in flight)
#pragma unroll
    for (int k = 0; k < kPsGReg; ++k)
      if (gc < out) gt[(gr0 + 4 * k) * GS + gc] = gn[k];
    if (tl + 1 < t1) fetch(tl + 1);
    if (fe) {  // row r0 + frr, input fin: the features as kan_gw_kernel forms them
      float* fr = ft + (fig * kPsTile + frr) * FS;
      // the forward's exp2 / rcp forms (fn_edge): SiLU, logistic 2 / (1 + 2^(-a log2e (x - b)))
      fr[0] = live ? xv * rcp(1.0f + ex2(-xv * FETODE_LOG2E)) : 0.f;
      float val[SO + 1];
      const int m = bpoly_vals(xv, NG, gi, rhi, bpi, val);
      for (int c = 0; c < NS; ++c) {
        float v = (live && m == -2) ? __builtin_nanf("") : 0.f;
#pragma unroll
        for (int rr = 0; rr <= SO; ++rr)
          if (live && m >= 0 && m - SO + rr == c) v = val[rr];
        fr[1 + c] = v;
      }
      for (int j = 0; j < NB; ++j)
        fr[1 + NS + j] = live ? 2.0f * rcp(1.0f + ex2(labi[3 * j] * (xv - labi[3 * j + 1]))) : 0.f;
    }
    lds_barrier();
    if (LOG && live) {  // logistic a / b: d phi_j through the row's g
      const float* fr = ft + (fig * kPsTile + frr) * FS;
      float gph[NL];
#pragma unroll
      for (int j = 0; j < NL; ++j) gph[j] = 0.f;
      for (int o = 0; o < out; ++o) {  // d loss / d phi_j = sum_o g[o] W'[o, (i, j)], W' row as float4s
        const float go = gt[frr * GS + o];
        const float4* wr = reinterpret_cast<const float4*>(wl + (fig * out + o) * NBP);
#pragma unroll
        for (int jq = 0; jq < NL / 4; ++jq) {
          if (4 * jq < NB) {
            const float4 w4 = wr[jq];
            gph[4 * jq] += go * w4.x;
            gph[4 * jq + 1] += go * w4.y;
            gph[4 * jq + 2] += go * w4.z;
            gph[4 * jq + 3] += go * w4.w;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        if (j >= NB) break;
        const float gphi = gph[j];
        const float a = labi[3 * j + 2], bb = labi[3 * j + 1];
        const float sg = 0.5f * fr[1 + NS + j];  // sigm(a (x - b))
        const float dz = gphi * 2.0f * sg * (1.0f - sg);
        la[j] += dz * (xv - bb);
        lb[j] += dz * (-a);
      }
    }
    if (act) {
      const float* fb = ft + pig * kPsTile * FS;
      for (int rr = q; rr < kPsTile; rr += Q) {
        float fv[4], gv[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) fv[a] = f0 + a < NF ? fb[rr * FS + f0 + a] : 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) gv[c] = o0 + c < out ? gt[rr * GS + o0 + c] : 0.f;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[a][c] = ffma(fv[a], gv[c], acc[a][c]);
      }
    }
  }
  // workgroup sums in a fixed order: the Q row groups of each triple, then the tile rows' a / b
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[tid * 16 + a * 4 + c] = acc[a][c];
  __syncthreads();
  for (int e = tid; e < P * 16; e += 256) {
    const int pp = e / 16, ac = e % 16, a = ac / 4, c = ac % 4;
    const int ig = pp / (FBK * OBK);
    const int f = 4 * ((pp / OBK) % FBK) + a, o = 4 * (pp % OBK) + c;
    float v = 0.f;
    for (int qq = 0; qq < Q; ++qq) v += red[(qq * P + pp) * 16 + ac];
    if (f < NF && o < out) part[(((int64_t)s * in + i0 + ig) * NF + f) * out + o] = v;
  }
  if (LOG) {
    for (int j = 0; j < NB && j < NL; ++j) {
      __syncthreads();
      if (fe) {
        red[tid * 2] = la[j];
        red[tid * 2 + 1] = lb[j];
      }
      __syncthreads();
      if (tid < 2 * ni) {
        const int ig = tid / 2, c = tid % 2;
        float v = 0.f;
        for (int rr = 0; rr < kPsTile; ++rr) v += red[(ig * kPsTile + rr) * 2 + c];
        abpart[(((int64_t)s * in + i0 + ig) * NB + j) * 2 + c] = v;
      }
    }
  }
}

// Narrow layers (out <= 4: a field's last layer, in -> D): the tile kernel above stages features
// and g rows in LDS for a handful of products per row.  Here a thread owns rows of ONE input and
// keeps every (feature, output) sum in registers — (1 + NS + NB) x OUT of them — so a row is its x,
// its g row (OUT floats, the next row's already in flight), the features in registers and
// (1 + NS + NB) x OUT FMAs; the logistic a / b sums ride along.  The only LDS is the input's
// tables (broadcast reads) and the final fixed-order sums (wave butterflies, then the 4 waves in
// order), written in the tile kernel's per-split layout for kan_psum_reduce_kernel.
constexpr int kPrNS = 8, kPrNB = 12, kPrMaxOut = 4;
bool pr_ok(const fetode_kanlinear_t* kl) {
  return kl->spline_order == 3 && kl->out_features <= kPrMaxOut && kl->grid_size + 3 <= kPrNS &&
         kl->num_logistic <= kPrNB;
}
int pr_splits(const fetode_kanlinear_t* kl, int64_t B) {
  int64_t S = kPsBlocks / kl->in_features;
  const int64_t rs = (B + 1023) / 1024;  // at least ~4 rows per thread
  if (S > rs) S = rs;
  if (S > ps_smax(kl)) S = ps_smax(kl);
  return S < 1 ? 1 : (int)S;
}

// NBM >= NB sizes the register sums: 10 (efficient_kan's default num_basis) or kPrNB
template <int OUT, int NBM>
__global__ __launch_bounds__(256) void kan_psum_rows_kernel(fetode_kanlinear_t kl, const float* __restrict__ x,
                                                           const float* __restrict__ g, int64_t B,
                                                           const float4* __restrict__ bpt /* (in, NG - 1, 4) */,
                                                           float* __restrict__ part /* (S, in, NF, out) */,
                                                           float* __restrict__ abpart /* (S, in, NB, 2) */) {
  constexpr int SO = 3, NV = (1 + kPrNS + NBM) * OUT + 2 * NBM;
  __shared__ float wl[OUT * NBM], kn[kPrNS + SO + 1], rh[kPrNS + SO], lab[3 * NBM];
  __shared__ float4 bp[(kPrNS + SO) * 4];
  __shared__ float red[4][NV];
  const int in = kl.in_features, NB = kl.num_logistic;
  const int NG = kl.grid_size + 2 * SO + 1, NS = kl.grid_size + SO, NF = 1 + NS + NB;
  const int i = blockIdx.x, sp = blockIdx.y, S = gridDim.y, tid = threadIdx.x;
  // input i's tables: W'[o, (i, j)], knots, 1 / knot steps, basis cubics (bpoly_entry), logistic
  for (int q = tid; q < OUT * NB; q += 256) {
    const int o = q / NB, j = q % NB;
    const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
    wl[o * NBM + j] = (kl.logistic_weight[(int64_t)o * in * NB + i * NB + j] * kl.scale_logistic) * ls;
  }
  const float* gg = kl.grid + (int64_t)i * NG;
  for (int q = tid; q < NG; q += 256) kn[q] = gg[q];
  for (int q = tid; q < NG - 1; q += 256) rh[q] = 1.0f / (gg[q + 1] - gg[q]);
  for (int q = tid; q < (NG - 1) * 4; q += 256) bp[q] = bpt[(int64_t)i * (NG - 1) * 4 + q];
  for (int j = tid; j < NB; j += 256) {
    lab[3 * j] = -kl.logistic_a[i * NB + j] * FETODE_LOG2E;
    lab[3 * j + 1] = kl.logistic_b[i * NB + j];
    lab[3 * j + 2] = kl.logistic_a[i * NB + j];
  }
  __syncthreads();
  float ab[OUT], spl[kPrNS][OUT], lw[NBM][OUT], la[NBM], lb[NBM];
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    ab[o] = 0.f;
#pragma unroll
    for (int c = 0; c < kPrNS; ++c) spl[c][o] = 0.f;
#pragma unroll
    for (int j = 0; j < NBM; ++j) lw[j][o] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < NBM; ++j) la[j] = lb[j] = 0.f;
  const int64_t r0 = sp * B / S, r1 = (sp + 1) * B / S;
  float xn = 0.f, gn[OUT];
#pragma unroll
  for (int o = 0; o < OUT; ++o) gn[o] = 0.f;
  if (r0 + tid < r1) {
    xn = x[(r0 + tid) * in + i];
#pragma unroll
    for (int o = 0; o < OUT; ++o) gn[o] = g[(r0 + tid) * OUT + o];
  }
  for (int64_t r = r0 + tid; r < r1; r += 256) {
    const float xv = xn;
    float gv[OUT];
#pragma unroll
    for (int o = 0; o < OUT; ++o) gv[o] = gn[o];
    if (r + 256 < r1) {  // the next row in flight while this one is summed
      xn = x[(r + 256) * in + i];
#pragma unroll
      for (int o = 0; o < OUT; ++o) gn[o] = g[(r + 256) * OUT + o];
    }
    const float silu = xv * rcp(1.0f + ex2(-xv * FETODE_LOG2E));
    float val[SO + 1];
    const int m = bpoly_vals(xv, NG, kn, rh, bp, val);
#pragma unroll
    for (int o = 0; o < OUT; ++o) ab[o] = ffma(gv[o], silu, ab[o]);
#pragma unroll
    for (int c = 0; c < kPrNS; ++c) {
      float v = m == -2 ? __builtin_nanf("") : 0.f;  // non-finite x: NaN bases (the tile kernel's rule)
#pragma unroll
      for (int q = 0; q <= SO; ++q)
        if (m >= 0 && m - SO + q == c) v = val[q];
      if (c < NS)
#pragma unroll
        for (int o = 0; o < OUT; ++o) spl[c][o] = ffma(gv[o], v, spl[c][o]);
    }
#pragma unroll
    for (int j = 0; j < NBM; ++j) {
      if (j < NB) {
        const float phi = 2.0f * rcp(1.0f + ex2(lab[3 * j] * (xv - lab[3 * j + 1])));
        float gphi = 0.f;
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          lw[j][o] = ffma(gv[o], phi, lw[j][o]);
          gphi += gv[o] * wl[o * NBM + j];
        }
        const float sg = 0.5f * phi;  // sigm(a (x - b))
        const float dz = gphi * 2.0f * sg * (1.0f - sg);
        la[j] += dz * (xv - lab[3 * j + 1]);
        lb[j] += dz * (-lab[3 * j + 2]);
      }
    }
  }
  // fixed-order sums: a butterfly per wave, then the four waves in order
  const int wid = tid >> 6, lane = tid & 63;
  auto wsum = [&](float v) {
#pragma unroll
    for (int mm = 32; mm >= 1; mm >>= 1) v += __shfl_xor(v, mm);
    return v;
  };
  int q = 0;
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    const float v = wsum(ab[o]);
    if (lane == 0) red[wid][q] = v;
    ++q;
  }
#pragma unroll
  for (int c = 0; c < kPrNS; ++c)
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const float v = c < NS ? wsum(spl[c][o]) : 0.f;
      if (lane == 0) red[wid][q] = v;
      ++q;
    }
#pragma unroll
  for (int j = 0; j < NBM; ++j) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const float v = j < NB ? wsum(lw[j][o]) : 0.f;
      if (lane == 0) red[wid][q] = v;
      ++q;
    }
    const float va = j < NB ? wsum(la[j]) : 0.f, vb = j < NB ? wsum(lb[j]) : 0.f;
    if (lane == 0) {
      red[wid][q] = va;
      red[wid][q + 1] = vb;
    }
    q += 2;
  }
  __syncthreads();
  // slot order above: base (OUT), spline c-major (kPrNS x OUT), then per j: lw (OUT), a, b
  for (int e = tid; e < NV; e += 256) {
    const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    if (e < OUT) {
      part[(((int64_t)sp * in + i) * NF + 0) * OUT + e] = v;
    } else if (e < OUT + kPrNS * OUT) {
      const int c = (e - OUT) / OUT, o = (e - OUT) % OUT;
      if (c < NS) part[(((int64_t)sp * in + i) * NF + 1 + c) * OUT + o] = v;
    } else {
      const int t = e - OUT - kPrNS * OUT, j = t / (OUT + 2), k = t % (OUT + 2);
      if (j < NB) {
        if (k < OUT) part[(((int64_t)sp * in + i) * NF + 1 + NS + j) * OUT + k] = v;
        else abpart[(((int64_t)sp * in + i) * NB + j) * 2 + (k - OUT)] = v;
      }
    }
  }
}

// the splits in order -> base-weight gradient, d_scaled, d_wl, logistic a / b: one wave per output
// (lane l sums splits l, l + 64, ...; then a fixed butterfly: run-to-run identical)
__device__ __forceinline__ float split_sum64(const float* __restrict__ p, int S, int64_t stride, int lane) {
  float v = 0.f;
  for (int sp = lane; sp < S; sp += 64) v += p[(int64_t)sp * stride];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__global__ __launch_bounds__(256) void kan_psum_reduce_kernel(fetode_kanlinear_t kl, const float* __restrict__ part,
                                                             const float* __restrict__ abpart, int S,
                                                             float* __restrict__ d_scaled, float* __restrict__ d_wl,
                                                             fetode_kanlinear_grad_t gr, int accumulate) {
  const int64_t t = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int in = kl.in_features, out = kl.out_features, NB = kl.num_logistic;
  const int NS = kl.grid_size + kl.spline_order, NF = 1 + NS + NB;
  const int64_t nw = (int64_t)out * in * NF;
  if (t < nw) {
    const int f = (int)(t % NF);
    const int64_t oi = t / NF;
    const int o = (int)(oi / in), i = (int)(oi % in);
    const float v = split_sum64(part + ((int64_t)i * NF + f) * out + o, S, (int64_t)in * NF * out, lane);
    if (lane) return;
    if (f == 0) put(gr.base_weight ? gr.base_weight + (int64_t)o * in + i : nullptr, v, accumulate);
    else if (f <= NS) d_scaled[((int64_t)o * in + i) * NS + (f - 1)] = v;
    else d_wl[(int64_t)o * in * NB + i * NB + (f - 1 - NS)] = v;
  } else if (t < nw + (int64_t)in * NB) {
    const int q = (int)(t - nw);  // (i, j)
    const float va = split_sum64(abpart + (int64_t)q * 2, S, (int64_t)in * NB * 2, lane);
    const float vb = split_sum64(abpart + (int64_t)q * 2 + 1, S, (int64_t)in * NB * 2, lane);
    if (lane) return;
    put(gr.logistic_a ? gr.logistic_a + q : nullptr, va, accumulate);
    put(gr.logistic_b ? gr.logistic_b + q : nullptr, vb, accumulate);
  }
}

// logistic basis parameters a, b: one block per (i, j)
__global__ void kan_gab_kernel(fetode_kanlinear_t kl, const float* __restrict__ x, const float* __restrict__ g,
                               int64_t B, fetode_kanlinear_grad_t gr, int accumulate) {
  __shared__ float red[2 * RB];
  const int in = kl.in_features, out = kl.out_features, NB = kl.num_logistic;
  const int i = blockIdx.x / NB, j = blockIdx.x % NB;
  const float a = kl.logistic_a[i * NB + j], bb = kl.logistic_b[i * NB + j];
  float s[2] = {0.f, 0.f};
  for (int64_t b = threadIdx.x; b < B; b += RB) {
    const float xv = x[b * in + i];
    float gphi = 0.f;
    for (int o = 0; o < out; ++o) {
      const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      gphi += g[b * out + o] * ((kl.logistic_weight[(int64_t)o * in * NB + i * NB + j] * kl.scale_logistic) * ls);
    }
    const float sg = sigm(a * (xv - bb));
    const float dz = gphi * 2.0f * sg * (1.0f - sg);
    s[0] += dz * (xv - bb);
    s[1] += dz * (-a);
  }
  block_sum(s, red);
  if (threadIdx.x == 0) {
    put(gr.logistic_a ? gr.logistic_a + i * NB + j : nullptr, s[0], accumulate);
    put(gr.logistic_b ? gr.logistic_b + i * NB + j : nullptr, s[1], accumulate);
  }
}

// ------------------------------------------------------------------------------------------
// FerroelectricBasis (general branch_sign), reference formula differentiated by hand
// ------------------------------------------------------------------------------------------
struct FerroPoint {  // forward values of one (b, i, o, k) element
  float th, m, u, cp, cn, bs, P;
};

__device__ __forceinline__ FerroPoint ferro_point(const fetode_ferro_t& fl, float xv, float pv, int e, int64_t b) {
  FerroPoint q;
  const float gs = (float)fl.gate_slope, al = (float)fl.alpha, oma = (float)(1.0 - fl.alpha);
  const float Ec = fl.Ec[e];
  q.bs = fl.branch_sign ? fl.branch_sign[b * fl.branch_sign_bstride + e] : 1.0f;
  q.u = sigm(gs * (xv - pv));
  q.cp = sigm(gs * (xv - Ec));
  q.cn = sigm(gs * (-xv - Ec));
  const float su = q.u * q.cp, sl = (1.0f - q.u) * q.cn;
  const float tgt = (su * 1.0f + sl * (-1.0f)) + ((1.0f - su) - sl) * q.bs;
  q.m = al * q.bs + oma * tgt;
  q.th = tanhf(fl.k[e] * (xv + Ec * q.m));
  q.P = fl.Ps[e] * q.th + fl.bias[e];
  return q;
}

// given g on the element output (g_out[b,o]), contributions to dx and to the 5 parameters
__device__ __forceinline__ void ferro_point_vjp(const fetode_ferro_t& fl, const FerroPoint& q, float xv, int e,
                                                float go, float* gx, float* gk, float* gEc, float* gPs,
                                                float* gbias, float* gcoef) {
  const float gs = (float)fl.gate_slope, oma = (float)(1.0 - fl.alpha);
  const float Ec = fl.Ec[e], kk = fl.k[e], Ps = fl.Ps[e], co = fl.coef[e];
  *gcoef = go * q.P;
  const float gP = go * co;
  *gPs = gP * q.th;
  *gbias = gP;
  const float gz = gP * Ps * (1.0f - q.th * q.th);
  const float sh = xv + Ec * q.m;
  *gk = gz * sh;
  const float gsh = gz * kk;
  const float gm = gsh * Ec;
  const float gt = gm * oma;
  const float gsu = gt * (1.0f - q.bs), gsl = gt * (-1.0f - q.bs);
  const float gu = gsu * q.cp - gsl * q.cn;
  const float gcp = gsu * q.u, gcn = gsl * (1.0f - q.u);
  const float dcp = gs * q.cp * (1.0f - q.cp), dcn = gs * q.cn * (1.0f - q.cn), du = gs * q.u * (1.0f - q.u);
  *gx = gsh + gu * du + gcp * dcp - gcn * dcn;
  *gEc = gsh * q.m - gcp * dcp - gcn * dcn;
}

__global__ void ferro_gx_kernel(fetode_ferro_t fl, const float* __restrict__ x, const float* __restrict__ prev,
                                int reinit, const float* __restrict__ g, int64_t B, float* __restrict__ gx,
                                int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = fl.in_dim, out = fl.out_dim, K = fl.num_basis;
  if (t >= B * in) return;
  const int64_t b = t / in;
  const int i = t % in;
  const float xv = x[t], pv = reinit ? xv : prev[t];
  float acc = 0.f;
  for (int o = 0; o < out; ++o) {
    const float go = g[b * out + o];
    for (int k = 0; k < K; ++k) {
      const int e = (i * out + o) * K + k;
      const FerroPoint q = ferro_point(fl, xv, pv, e, b);
      float dx, d1, d2, d3, d4, d5;
      ferro_point_vjp(fl, q, xv, e, go, &dx, &d1, &d2, &d3, &d4, &d5);
      acc += dx;
    }
  }
  gx[t] = accumulate ? gx[t] + acc : acc;
}

// one block per element (i, o, k)
__global__ void ferro_gp_kernel(fetode_ferro_t fl, const float* __restrict__ x, const float* __restrict__ prev,
                                int reinit, const float* __restrict__ g, int64_t B, fetode_ferro_grad_t gr,
                                int accumulate) {
  __shared__ float red[5 * RB];
  const int in = fl.in_dim, out = fl.out_dim, K = fl.num_basis;
  const int e = blockIdx.x;
  const int i = e / (out * K), o = (e / K) % out;
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t b = threadIdx.x; b < B; b += RB) {
    const float xv = x[b * in + i], pv = reinit ? xv : prev[b * in + i];
    const FerroPoint q = ferro_point(fl, xv, pv, e, b);
    float dx, gk, gEc, gPs, gb, gc;
    ferro_point_vjp(fl, q, xv, e, g[b * out + o], &dx, &gk, &gEc, &gPs, &gb, &gc);
    s[0] += gk;
    s[1] += gEc;
    s[2] += gPs;
    s[3] += gb;
    s[4] += gc;
  }
  block_sum(s, red);
  if (threadIdx.x == 0) {
    put(gr.k ? gr.k + e : nullptr, s[0], accumulate);
    put(gr.Ec ? gr.Ec + e : nullptr, s[1], accumulate);
    put(gr.Ps ? gr.Ps + e : nullptr, s[2], accumulate);
    put(gr.bias ? gr.bias + e : nullptr, s[3], accumulate);
    put(gr.coef ? gr.coef + e : nullptr, s[4], accumulate);
  }
}

// The Ferro parameter sums over many rows (the fieldn training pass: every (evaluation,
// trajectory) row): ferro_gp_kernel gives each element ONE workgroup walking all rows (in * out * K
// workgroups — 384 for [2, 16, 2] K=12 — each a serial chain of a few thousand rows); here element
// e's rows are split S ways (~8 K workgroups), per-split sums land in the workspace and
// ferro_gp_reduce_kernel adds the splits in order (run-to-run identical).  The hysteresis input of
// row r: rows < n0 read p0 (or reinit: x itself), later rows the row n0 earlier (the previous
// evaluation of the same trajectory, fieldn's tape layout (n_ev, B, in)).
constexpr int kFgTarget = 8192, kFgChunk = 6;  // workgroups per launch; elements per workgroup
int fg_units(const fetode_ferro_t* fl) {
  return fl->in_dim * fl->out_dim * ((fl->num_basis + kFgChunk - 1) / kFgChunk);
}
int fg_splits(const fetode_ferro_t* fl, int64_t R) {
  int64_t S = kFgTarget / fg_units(fl);
  const int64_t rs = (R + 1023) / 1024;  // at least ~4 rows per thread
  if (S > rs) S = rs;
  return S < 1 ? 1 : (int)S;
}

// workgroup (i, o, chunk of kFgChunk elements k, split): per row the shared sigmoid of the
// hysteresis gate once, then per element the forward's exp2 / rcp forms (fieldn's plan: branch
// sign 1, so m = 1 + w s with w = -2 (1 - alpha)(1 - u), s = sigmoid(gs(-x - Ec)));
// d P / d (k, Ec, Ps, bias, coef) as ferro_point_vjp with that m
__global__ __launch_bounds__(RB) void ferro_gp_split_kernel(fetode_ferro_t fl, const float* __restrict__ x,
                                                           int64_t R, const float* __restrict__ p0, int64_t n0,
                                                           const float* __restrict__ g, float* __restrict__ part) {
  __shared__ float red[5 * kFgChunk * RB];
  const int in = fl.in_dim, out = fl.out_dim, K = fl.num_basis, NC = (K + kFgChunk - 1) / kFgChunk;
  const int io = blockIdx.x / NC, kc = blockIdx.x % NC, sp = blockIdx.y, S = gridDim.y;
  const int i = io / out, o = io % out;
  const int e0 = io * K + kc * kFgChunk, ne = K - kc * kFgChunk < kFgChunk ? K - kc * kFgChunk : kFgChunk;
  const int64_t r0 = sp * R / S, r1 = (sp + 1) * R / S;
  const float gs = (float)fl.gate_slope, gs2 = gs * FETODE_LOG2E, wc = (float)(-2.0 * (1.0 - fl.alpha));
  float Ec[kFgChunk], kk[kFgChunk], Ps[kFgChunk], bi[kFgChunk], co[kFgChunk], GE[kFgChunk], k2[kFgChunk];
#pragma unroll
  for (int j = 0; j < kFgChunk; ++j) {
    const bool on = j < ne;
    Ec[j] = on ? fl.Ec[e0 + j] : 0.f;
    kk[j] = on ? fl.k[e0 + j] : 0.f;
    Ps[j] = on ? fl.Ps[e0 + j] : 0.f;
    bi[j] = on ? fl.bias[e0 + j] : 0.f;
    co[j] = on ? fl.coef[e0 + j] : 0.f;
    GE[j] = gs2 * Ec[j];
    k2[j] = 2.0f * FETODE_LOG2E * kk[j];
  }
  float acc[5 * kFgChunk];
#pragma unroll
  for (int q = 0; q < 5 * kFgChunk; ++q) acc[q] = 0.f;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += RB) {
    const float xv = x[r * in + i];
    const float pv = r >= n0 ? x[(r - n0) * in + i] : (p0 ? p0[r * in + i] : xv);
    const float go = g[r * out + o];
    const float u = rcp(1.0f + ex2(-gs2 * (xv - pv)));
    const float w = wc * (1.0f - u);
#pragma unroll
    for (int j = 0; j < kFgChunk; ++j) {
      const float sg = rcp(1.0f + ex2(ffma(gs2, xv, GE[j])));  // sigmoid(gs(-x - Ec))
      const float m = ffma(w, sg, 1.0f);
      const float sh = ffma(Ec[j], m, xv);
      const float th = ffma(rcp(1.0f + ex2(k2[j] * sh)), -2.0f, 1.0f);  // tanh(k sh)
      const float gP = go * co[j];
      const float gz = gP * Ps[j] * ffma(-th, th, 1.0f);
      acc[0 * kFgChunk + j] = ffma(gz, sh, acc[0 * kFgChunk + j]);                       // k
      const float dmdE = -(w * gs) * (sg * (1.0f - sg));                                // d m / d Ec
      acc[1 * kFgChunk + j] = ffma(gz * kk[j], ffma(Ec[j], dmdE, m), acc[1 * kFgChunk + j]);  // Ec
      acc[2 * kFgChunk + j] = ffma(gP, th, acc[2 * kFgChunk + j]);                       // Ps
      acc[3 * kFgChunk + j] += gP;                                                       // bias
      acc[4 * kFgChunk + j] = ffma(go, ffma(Ps[j], th, bi[j]), acc[4 * kFgChunk + j]);   // coef
    }
  }
  block_sum(acc, red);
  if (threadIdx.x < 5 * ne) {
    const int c = threadIdx.x / ne, j = threadIdx.x % ne;
    part[((int64_t)sp * in * out * K + e0 + j) * 5 + c] = acc[c * kFgChunk + j];
  }
}

__global__ __launch_bounds__(256) void ferro_gp_reduce_kernel(fetode_ferro_t fl, const float* __restrict__ part, int S,
                                                             fetode_ferro_grad_t gr, int accumulate) {
  const int E = fl.in_dim * fl.out_dim * fl.num_basis;
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (t >= E * 5) return;
  const int e = t / 5, c = t % 5;
  const float v = split_sum64(part + (int64_t)e * 5 + c, S, (int64_t)E * 5, lane);
  if (lane) return;
  float* dst = c == 0 ? gr.k : c == 1 ? gr.Ec : c == 2 ? gr.Ps : c == 3 ? gr.bias : gr.coef;
  put(dst ? dst + e : nullptr, v, accumulate);
}

bool ps_ok(const fetode_kanlinear_t* kl) {
  const int NF = 1 + kl->grid_size + kl->spline_order + kl->num_logistic;
  return kl->spline_order == 3 && NF <= kPsMaxNF && kl->out_features <= kPsMaxOut && kl->num_logistic <= kMaxLogistic;
}

}  // namespace

extern "C" {

int64_t fetode_kanlinear_backward_workspace(const fetode_kanlinear_t* kl) {
  if (!kl) return -1;
  const int NS = kl->grid_size + kl->spline_order;
  int64_t n = (int64_t)kl->out_features * kl->in_features * (NS + kl->num_logistic);
  if (fetode_kanlinear_wide_supported(kl))   // MFMA partials + logistic a / b partials
    n += (int64_t)kGwSplit * kl->in_features * (kGwF * 16 + 2 * kGwNB);
  else if (ps_ok(kl))                        // kan_psum_kernel's per-split partials + basis tables
    n += (int64_t)ps_smax(kl) * kl->in_features *
         ((int64_t)(1 + NS + kl->num_logistic) * kl->out_features + 2 * kl->num_logistic) +
         4 + (int64_t)kl->in_features * (kl->grid_size + 2 * kl->spline_order) * 16;
  return (int64_t)sizeof(float) * n;
}

int fetode_kanlinear_backward(const fetode_kanlinear_t* kl, const float* x, int64_t B, const float* g,
                              float* gx, const fetode_kanlinear_grad_t* grads, void* workspace,
                              int32_t accumulate, void* stream) {
  fetode_field_t f{1, kl, nullptr};
  int rc = validate_field(&f);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !g) return set_err(FETODE_EINVAL, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int in = kl->in_features, out = kl->out_features, NB = kl->num_logistic, SO = kl->spline_order;
  const int NS = kl->grid_size + SO;
  const bool wide = fetode_kanlinear_wide_supported(kl) && B >= 256;
  if (wide && (gx || (grads && NB > 0))) {   // d x and d (a, b) in one pass over the batch
    if (grads && !workspace) return set_err(FETODE_EINVAL, "kanlinear backward: workspace required for parameter grads");
    float* abpart = (grads && NB > 0)
                        ? (float*)workspace + (int64_t)out * in * (NS + NB) + (int64_t)kGwSplit * in * kGwF * 16
                        : nullptr;
    if (kl->out_features <= 12)
      hipLaunchKernelGGL(wide_gxab_kernel<12>, dim3(in / 4, kGwSplit), dim3(256), 0, s, *kl, x, g, B, gx, abpart, accumulate);
    else
      hipLaunchKernelGGL(wide_gxab_kernel<16>, dim3(in / 4, kGwSplit), dim3(256), 0, s, *kl, x, g, B, gx, abpart, accumulate);
    LAUNCH_CHECK();
    if (abpart) {
      hipLaunchKernelGGL(wide_ab_reduce_kernel, dim3(nblk((int64_t)in * NB, 256)), dim3(256), 0, s, *kl, abpart, *grads,
                         accumulate);
      LAUNCH_CHECK();
    }
  } else if (gx) {
    const int64_t n = B * in;
#define KGX(S) hipLaunchKernelGGL(kan_gx_kernel<S>, dim3(nblk(n, 256)), dim3(256), 0, s, *kl, x, g, B, gx, accumulate)
    if (SO == 1) KGX(1); else if (SO == 2) KGX(2); else KGX(3);
#undef KGX
    LAUNCH_CHECK();
  }
  if (grads) {
    if (!workspace) return set_err(FETODE_EINVAL, "kanlinear backward: workspace required for parameter grads");
    float* d_scaled = (float*)workspace;
    float* d_wl = d_scaled + (int64_t)out * in * NS;
    if (wide) {   // MFMA contraction over the batch
      float* dpart = d_wl + (int64_t)out * in * NB;
      hipLaunchKernelGGL(wide_gw_kernel, dim3(in / 4, kGwSplit), dim3(256), 0, s, *kl, x, g, B, dpart);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(wide_gw_reduce_kernel, dim3(nblk((int64_t)out * in * kGwF, 256)), dim3(256), 0, s, *kl, dpart,
                         d_scaled, d_wl, *grads, accumulate);
      LAUNCH_CHECK();
    } else if (B >= kPsMinRows && ps_ok(kl)) {   // many rows: features once per (row, input)
      const bool rows = pr_ok(kl);   // narrow layers: the row-owner form (sums in registers)
      const int S = rows ? pr_splits(kl, B) : ps_splits(kl, B);
      float* part = d_wl + (int64_t)out * in * NB;
      float* abpart = part + (int64_t)ps_smax(kl) * in * (1 + NS + NB) * out;
      float4* bpt = reinterpret_cast<float4*>(((uintptr_t)(abpart + (int64_t)ps_smax(kl) * in * NB * 2) + 15) & ~uintptr_t(15));
      const int NG = kl->grid_size + 2 * SO + 1;
      hipLaunchKernelGGL(bpoly_build_kernel, dim3(nblk((int64_t)in * (NG - 1) * 4, 64)), dim3(64), 0, s, *kl, bpt);
      LAUNCH_CHECK();
      if (rows) {
        auto* kfn = NB <= 10 ? (out == 1 ? kan_psum_rows_kernel<1, 10> : out == 2 ? kan_psum_rows_kernel<2, 10>
                               : out == 3 ? kan_psum_rows_kernel<3, 10> : kan_psum_rows_kernel<4, 10>)
                             : (out == 1 ? kan_psum_rows_kernel<1, kPrNB> : out == 2 ? kan_psum_rows_kernel<2, kPrNB>
                               : out == 3 ? kan_psum_rows_kernel<3, kPrNB> : kan_psum_rows_kernel<4, kPrNB>);
        hipLaunchKernelGGL(kfn, dim3(in, S), dim3(256), 0, s, *kl, x, g, B, bpt, part, abpart);
      } else {
        auto* kfn = NB > 0 ? kan_psum_kernel<3, true> : kan_psum_kernel<3, false>;
        hipLaunchKernelGGL(kfn, dim3(ps_groups(kl), S), dim3(256), ps_lds_bytes(kl), s, *kl, x, g, B, bpt, part, abpart);
      }
      LAUNCH_CHECK();
      const int64_t nt = (int64_t)out * in * (1 + NS + NB) + (int64_t)in * NB;
      hipLaunchKernelGGL(kan_psum_reduce_kernel, dim3(nblk(nt, 4)), dim3(256), 0, s, *kl, part, abpart, S, d_scaled,
                         d_wl, *grads, accumulate);
      LAUNCH_CHECK();
    } else {
      const int nblocks = out * in * (1 + NS + NB);
#define KGW(S) hipLaunchKernelGGL(kan_gw_kernel<S>, dim3(nblocks), dim3(RB), 0, s, *kl, x, g, B, d_scaled, d_wl, *grads, accumulate)
      if (SO == 1) KGW(1); else if (SO == 2) KGW(2); else KGW(3);
#undef KGW
      LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(kan_scale_grads_kernel, dim3(nblk((int64_t)out * in * (NB > 1 ? NB : 1), 128)), dim3(128), 0, s,
                       *kl, d_scaled, d_wl, *grads, accumulate);
    LAUNCH_CHECK();
    if (NB > 0 && kl->logistic_scaler) {
      hipLaunchKernelGGL(kan_scale_ls_kernel, dim3(nblk(out, 64)), dim3(64), 0, s, *kl, d_wl, *grads, accumulate);
      LAUNCH_CHECK();
    }
    if (NB > 0 && !wide && !(B >= kPsMinRows && ps_ok(kl))) {
      hipLaunchKernelGGL(kan_gab_kernel, dim3(in * NB), dim3(RB), 0, s, *kl, x, g, B, *grads, accumulate);
      LAUNCH_CHECK();
    }
  }
  return FETODE_OK;
}

int fetode_ferro_backward(const fetode_ferro_t* fl, const float* x, int64_t B, const float* prev, int32_t reinit,
                          const float* g, float* gx, const fetode_ferro_grad_t* grads, int32_t accumulate,
                          void* stream) {
  if (!fl || fl->in_dim <= 0 || fl->out_dim <= 0 || fl->num_basis <= 0)
    return set_err(FETODE_EINVAL, "ferro: bad dims");
  if (B <= 0) return FETODE_OK;
  if (!x || !g || (!reinit && !prev)) return set_err(FETODE_EINVAL, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (gx) {
    const int64_t n = B * fl->in_dim;
    hipLaunchKernelGGL(ferro_gx_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, *fl, x, prev, reinit, g, B, gx,
                       accumulate);
    LAUNCH_CHECK();
  }
  if (grads) {
    hipLaunchKernelGGL(ferro_gp_kernel, dim3(fl->in_dim * fl->out_dim * fl->num_basis), dim3(RB), 0, s, *fl, x,
                       prev, reinit, g, B, *grads, accumulate);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

}  // extern "C"

int64_t fetode::ferro_param_rows_workspace() { return (int64_t)sizeof(float) * kFgTarget * kFgChunk * 5; }

int fetode::ferro_param_rows(const fetode_ferro_t* fl, const float* x, int64_t R, const float* p0, int64_t n0,
                             const float* g, const fetode_ferro_grad_t* grads, void* workspace, int32_t accumulate,
                             void* stream) {
  if (!fl || fl->in_dim <= 0 || fl->out_dim <= 0 || fl->num_basis <= 0) return set_err(FETODE_EINVAL, "ferro: bad dims");
  if (fl->branch_sign) return set_err(FETODE_EUNSUPPORTED, "ferro row sums: branch_sign");
  if (R <= 0 || !grads) return FETODE_OK;
  if (!x || !g || !workspace) return set_err(FETODE_EINVAL, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int E = fl->in_dim * fl->out_dim * fl->num_basis;
  const int S = fg_splits(fl, R);
  float* part = (float*)workspace;
  hipLaunchKernelGGL(ferro_gp_split_kernel, dim3(fg_units(fl), S), dim3(RB), 0, s, *fl, x, R, p0, n0, g, part);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(ferro_gp_reduce_kernel, dim3(nblk((int64_t)E * 5, 4)), dim3(256), 0, s, *fl, part, S, *grads,
                     accumulate);
  LAUNCH_CHECK();
  return FETODE_OK;
}
