// fetode_mnist.hip — the Kuramoto front end of the MNIST classifier (mnist_kuramoto_kan.py:145-199,
// SURVEY §8f rank 3): theta = pi (2 x - 1), then `steps` explicit Euler steps
//     theta += dt (omega + K (cos(theta) S - sin(theta) C)),
// S / C the 4-neighbour sums of sin / cos (the reference's fixed 3x3 cross kernel, zero padding),
// and the features [cos(theta) | sin(theta)] (B, 2 H W).
//
// One workgroup per image: theta, sin and cos of the whole image live in LDS for all steps, so an
// image costs one read of its pixels and one write of its features (HBM-bound at 12 B per pixel
// plus the optional tape).  The backward walks the steps in reverse from a tape of theta_0..T
// (written by the training forward), forming d theta_s from d theta_{s+1} with the stencil's
// transpose; d omega and d K are per-image partial sums reduced over the batch in a fixed order
// (no atomics: run-to-run identical).
#include <cstdlib>

#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kKThreads = 256;

#ifndef FETODE_KURA_FAST
#define FETODE_KURA_FAST 1
#endif
// sin and cos of one phase.  Fast form: a two-constant Cody-Waite reduction of theta to
// r in [-pi, pi] (k = rint(theta / 2 pi); 2 pi = hi + lo), then v_sin_f32 / v_cos_f32 of r / 2 pi
// revolutions — 4 VALU + 2 transcendentals instead of OCML's two full sinf / cosf (the phases
// stay within a few periods; the hardware functions' error is ~1e-7 absolute there).
__device__ __forceinline__ void phase_sincos(float t, float& sn, float& cs) {
  if constexpr (FETODE_KURA_FAST) {
    constexpr float inv2pi = 0.159154943091895336f, hi = 6.28318548202514648f, lo = -1.74845553146951715e-07f;
    const float k = __builtin_rintf(t * inv2pi);
    const float r = __builtin_fmaf(-k, lo, __builtin_fmaf(-k, hi, t));
    const float rv = r * inv2pi;
    sn = __builtin_amdgcn_sinf(rv);
    cs = __builtin_amdgcn_cosf(rv);
  } else {
    sincosf(t, &sn, &cs);
  }
}
constexpr int kMaxPix = 3072;  // H * W: the backward keeps 4 * H * W floats in LDS (< 64 KB)

// 4-neighbour sum in the cross kernel's tap order: up (0,1), left (1,0), right (1,2), down (2,1)
__device__ __forceinline__ float nsum(const float* a, int p, int r, int c, int H, int W) {
  float s = 0.f;
  if (r > 0) s += a[p - W];
  if (c > 0) s += a[p - 1];
  if (c < W - 1) s += a[p + 1];
  if (r < H - 1) s += a[p + W];
  return s;
}

__global__ __launch_bounds__(kKThreads) void kuramoto_fwd_kernel(const float* __restrict__ x, int H, int W, int steps,
                                                                float dt, const float* __restrict__ Kp,
                                                                const float* __restrict__ omega,
                                                                float* __restrict__ feat, float* __restrict__ tape) {
  extern __shared__ float sm[];  // theta | sin | cos, HW each
  const int HW = H * W;
  float* th = sm;
  float* sn = sm + HW;
  float* cs = sm + 2 * HW;
  const int64_t b = blockIdx.x;
  const float K = *Kp;
  const float pi = 3.14159265358979323846f;
  for (int p = threadIdx.x; p < HW; p += kKThreads) th[p] = pi * (2.0f * x[b * HW + p] - 1.0f);
  for (int s = 0; s < steps; ++s) {
    __syncthreads();
    for (int p = threadIdx.x; p < HW; p += kKThreads) {
      const float t = th[p];
      if (tape) tape[(b * (steps + 1) + s) * HW + p] = t;
      phase_sincos(t, sn[p], cs[p]);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < HW; p += kKThreads) {
      const int r = p / W, c = p - r * W;
      const float sin_n = nsum(sn, p, r, c, H, W), cos_n = nsum(cs, p, r, c, H, W);
      const float coupling = cs[p] * sin_n - sn[p] * cos_n;
      th[p] = th[p] + dt * (omega[p] + K * coupling);
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += kKThreads) {
    const float t = th[p];
    if (tape) tape[(b * (steps + 1) + steps) * HW + p] = t;
    float sv, cv;
    phase_sincos(t, sv, cv);
    feat[b * 2 * HW + p] = cv;
    feat[b * 2 * HW + HW + p] = sv;
  }
}

// ---- lane-per-column kernels (W < 32, H = HM rows): no LDS, no barriers ---------------------------
// A wave holds two images: lanes 32 i + c (c < W) own column c of image 2 w + i, the column's H
// phases (and omega) in registers.  Vertical neighbours are the neighbouring registers; horizontal
// ones come from the neighbouring lanes by DPP wave shifts (wave_shr:1 = lane - 1, wave_shl:1 =
// lane + 1; lanes c >= W hold zero sin / cos / g and bound_ctrl gives zero past the wave's ends, so
// a missing tap adds +0 — the same sum as skipping it).  Rows are walked top to bottom with a
// three-row window: row r's update needs rows r - 1 .. r + 1 of the step's OLD values, and row
// r + 1's are formed before row r is overwritten.  Same tap order (up, left, right, down) and
// per-pixel arithmetic as the LDS kernels (kuramoto_fwd_kernel / _bwd_kernel).
constexpr int kLaneWaves = 4;  // waves per workgroup (2 images each)
__device__ __forceinline__ float dpp_left(float v) {  // lane - 1's value (0 at lane 0)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_right(float v) {  // lane + 1's value (0 at lane 63)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

template <int H>
__global__ __launch_bounds__(64 * kLaneWaves) void kuramoto_fwd_lanes_kernel(
    const float* __restrict__ x, int64_t B, int W, int steps, float dt, const float* __restrict__ Kp,
    const float* __restrict__ omega, float* __restrict__ feat, float* __restrict__ tape) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kLaneWaves + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool act = c < W && b < B;
  const int HW = H * W;
  const float K = *Kp;
  const float pi = 3.14159265358979323846f;
  const float* xb = x + (act ? b * HW + c : 0);
  const float* ob = omega + (act ? c : 0);
  float th[H], om[H];
#pragma unroll
  for (int r = 0; r < H; ++r) {
    th[r] = pi * (2.0f * xb[r * W] - 1.0f);
    om[r] = ob[r * W];
  }
  float* tpb = tape ? tape + (act ? b * (int64_t)(steps + 1) * HW + c : 0) : nullptr;
  for (int st = 0; st < steps; ++st) {
    if (tpb && act) {
#pragma unroll
      for (int r = 0; r < H; ++r) tpb[st * HW + r * W] = th[r];
    }
    float su = 0.f, cu = 0.f, sm, cm, sd = 0.f, cd = 0.f;  // rows r - 1 (up), r, r + 1 (down)
    phase_sincos(th[0], sm, cm);
    sm = act ? sm : 0.f;
    cm = act ? cm : 0.f;
#pragma unroll
    for (int r = 0; r < H; ++r) {
      if (r + 1 < H) {
        phase_sincos(th[r + 1], sd, cd);
        sd = act ? sd : 0.f;
        cd = act ? cd : 0.f;
      }
      float sn_n = 0.f, cs_n = 0.f;
      if (r > 0) {
        sn_n += su;
        cs_n += cu;
      }
      sn_n += dpp_left(sm);
      cs_n += dpp_left(cm);
      sn_n += dpp_right(sm);
      cs_n += dpp_right(cm);
      if (r + 1 < H) {
        sn_n += sd;
        cs_n += cd;
      }
      const float coupling = cm * sn_n - sm * cs_n;
      th[r] = th[r] + dt * (om[r] + K * coupling);
      su = sm;
      cu = cm;
      sm = sd;
      cm = cd;
    }
  }
  if (!act) return;
  float* fb = feat + b * 2 * HW + c;
#pragma unroll
  for (int r = 0; r < H; ++r) {
    if (tpb) tpb[steps * HW + r * W] = th[r];
    float sv, cv;
    phase_sincos(th[r], sv, cv);
    fb[r * W] = cv;
    fb[HW + r * W] = sv;
  }
}

// The VJP on the same layout (kuramoto_bwd_kernel's per-pixel arithmetic and tap order): g, the
// d omega accumulator and the step's tape phases in registers (each row's phase slot is refilled
// with step st - 1's once its sin / cos are formed); per row a window of rows r - 1 .. r + 1 of the
// step's sin / cos and OLD g (row r - 1's new g is written back after row r has read the old one).
// d K: this lane's sum over its pixels and steps, then the image's 32 lanes by an xor tree.
template <int H>
__global__ __launch_bounds__(64 * kLaneWaves) void kuramoto_bwd_lanes_kernel(
    int64_t B, int W, int steps, float dt, const float* __restrict__ Kp, const float* __restrict__ tape,
    const float* __restrict__ gfeat, float* __restrict__ gx, float* __restrict__ gK_part,
    float* __restrict__ gom_part) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kLaneWaves + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool act = c < W && b < B;
  const int HW = H * W;
  const float K = *Kp;
  // inactive lanes read image 0 / column 0 (valid memory) and mask the values: no branches in the
  // unrolled row loops (per-row branches made the register allocator copy the arrays at every join)
  const float* tb = tape + (act ? b * (int64_t)(steps + 1) * HW + c : 0);
  const float* gf = gfeat + (act ? b * 2 * HW + c : 0);
  const int sp = steps > 0 ? steps - 1 : 0;
  float g[H], go[H], th[H];
  float gk = 0.f;
#pragma unroll
  for (int r = 0; r < H; ++r) {
    go[r] = 0.f;
    float sv, cv;
    phase_sincos(tb[steps * HW + r * W], sv, cv);
    const float gv = (-sv) * gf[r * W] + cv * gf[HW + r * W];
    g[r] = act ? gv : 0.f;
    th[r] = tb[sp * HW + r * W];
  }
  for (int st = steps - 1; st >= 0; --st) {
    const float* tn = tb + (st > 0 ? st - 1 : 0) * HW;   // step st - 1 (step 0 again at the last: unused)
    float su = 0.f, cu = 0.f, gu = 0.f, sm, cm, sd = 0.f, cd = 0.f;
    float gnew_prev = 0.f;
    phase_sincos(th[0], sm, cm);
    sm = act ? sm : 0.f;
    cm = act ? cm : 0.f;
    th[0] = tn[0];
#pragma unroll
    for (int r = 0; r < H; ++r) {
      if (r + 1 < H) {
        phase_sincos(th[r + 1], sd, cd);
        sd = act ? sd : 0.f;
        cd = act ? cd : 0.f;
        th[r + 1] = tn[(r + 1) * W];
      }
      const float gm = g[r], gd = (r + 1 < H) ? g[r + 1] : 0.f;
      float S = 0.f, C = 0.f;  // tap order up, left, right, down
      if (r > 0) {
        S += su;
        C += cu;
      }
      const float sl = dpp_left(sm), cl = dpp_left(cm), gl = dpp_left(gm);
      const float sr = dpp_right(sm), cr = dpp_right(cm), gr = dpp_right(gm);
      S += sl;
      C += cl;
      S += sr;
      C += cr;
      if (r + 1 < H) {
        S += sd;
        C += cd;
      }
      const float coupling = cm * S - sm * C;
      gk += gm * coupling;
      go[r] += gm;
      float acc = gm * (-(sm * S + cm * C));
      if (r > 0) acc += gu * (cu * cm + su * sm);
      acc += gl * (cl * cm + sl * sm);   // a missing neighbour has g = sin = cos = 0: + 0
      acc += gr * (cr * cm + sr * sm);
      if (r + 1 < H) acc += gd * (cd * cm + sd * sm);
      if (r > 0) g[r - 1] = gnew_prev;  // row r - 1's old g was last read above
      gnew_prev = act ? gm + (dt * K) * acc : 0.f;
      su = sm;
      cu = cm;
      gu = gm;
      sm = sd;
      cm = cd;
    }
    g[H - 1] = gnew_prev;
  }
  const float pi = 3.14159265358979323846f;
  if (act && gx) {
#pragma unroll
    for (int r = 0; r < H; ++r) gx[b * HW + r * W + c] = (g[r] * pi) * 2.0f;  // theta_0 = pi (2 x - 1)
  }
  if (act && gom_part) {
#pragma unroll
    for (int r = 0; r < H; ++r) gom_part[b * HW + r * W + c] = dt * go[r];
  }
  if (gK_part) {  // the image's d K: xor tree over its 32 lanes (inactive lanes add 0)
    float v = act ? gk : 0.f;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (c == 0 && b < B) gK_part[b] = dt * v;
  }
}

// VJP through the steps.  g = d loss / d theta_{s+1}; with c_p = cos_p S_p - sin_p C_p:
//   d c_p / d theta_p = -(sin_p S_p + cos_p C_p),  d c_p / d theta_q = cos_p cos_q + sin_p sin_q (q ~ p)
//   d theta_s[q] = g[q] + dt K (g[q] dc_q/dtheta_q + sum_{p ~ q} g[p] dc_p/dtheta_q)
//   d omega[p] += dt g[p];  d K += dt sum_p g[p] c_p
__global__ __launch_bounds__(kKThreads) void kuramoto_bwd_kernel(int H, int W, int steps, float dt,
                                                                const float* __restrict__ Kp,
                                                                const float* __restrict__ tape,
                                                                const float* __restrict__ gfeat,
                                                                float* __restrict__ gx, float* __restrict__ gK_part,
                                                                float* __restrict__ gom_part) {
  extern __shared__ float sm[];  // g | sin | cos | dgo (d omega accumulator), HW each
  __shared__ float red[kKThreads];
  const int HW = H * W;
  float* g = sm;
  float* sn = sm + HW;
  float* cs = sm + 2 * HW;
  float* go = sm + 3 * HW;
  const int64_t b = blockIdx.x;
  const float K = *Kp;
  const float* tb = tape + b * (steps + 1) * HW;
  float gk = 0.f;
  for (int p = threadIdx.x; p < HW; p += kKThreads) {
    const float t = tb[steps * HW + p];
    // feat = [cos, sin]: d theta_T = -sin g_cos + cos g_sin
    float sv, cv;
    phase_sincos(t, sv, cv);
    g[p] = (-sv) * gfeat[b * 2 * HW + p] + cv * gfeat[b * 2 * HW + HW + p];
    go[p] = 0.f;
  }
  // the phases of step s - 1 are fetched into registers while step s runs (a global-load round
  // trip per step was exposed after the barrier)
  constexpr int kPP = kMaxPix / kKThreads;
  float tn[kPP];
#pragma unroll
  for (int j = 0; j < kPP; ++j) {
    const int q = threadIdx.x + j * kKThreads;
    tn[j] = (steps > 0 && q < HW) ? tb[(steps - 1) * HW + q] : 0.f;
  }
  for (int s = steps - 1; s >= 0; --s) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPP; ++j) {
      const int q = threadIdx.x + j * kKThreads;
      if (q < HW) phase_sincos(tn[j], sn[q], cs[q]);
    }
    if (s > 0) {
#pragma unroll
      for (int j = 0; j < kPP; ++j) {
        const int q = threadIdx.x + j * kKThreads;
        tn[j] = q < HW ? tb[(s - 1) * HW + q] : 0.f;
      }
    }
    __syncthreads();
    float gnew[kMaxPix / kKThreads];
#pragma unroll
    for (int j = 0; j < kMaxPix / kKThreads; ++j) {
      const int q = threadIdx.x + j * kKThreads;
      gnew[j] = 0.f;
      if (q >= HW) continue;
      const int r = q / W, c = q - r * W;
      const float S = nsum(sn, q, r, c, H, W), C = nsum(cs, q, r, c, H, W);
      const float gq = g[q];
      const float coupling = cs[q] * S - sn[q] * C;
      gk += gq * coupling;
      go[q] += gq;
      float acc = gq * (-(sn[q] * S + cs[q] * C));
      if (r > 0) acc += g[q - W] * (cs[q - W] * cs[q] + sn[q - W] * sn[q]);
      if (c > 0) acc += g[q - 1] * (cs[q - 1] * cs[q] + sn[q - 1] * sn[q]);
      if (c < W - 1) acc += g[q + 1] * (cs[q + 1] * cs[q] + sn[q + 1] * sn[q]);
      if (r < H - 1) acc += g[q + W] * (cs[q + W] * cs[q] + sn[q + W] * sn[q]);
      gnew[j] = gq + (dt * K) * acc;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kMaxPix / kKThreads; ++j) {
      const int q = threadIdx.x + j * kKThreads;
      if (q < HW) g[q] = gnew[j];
    }
  }
  __syncthreads();
  const float pi = 3.14159265358979323846f;
  for (int p = threadIdx.x; p < HW; p += kKThreads) {
    if (gx) gx[b * HW + p] = (g[p] * pi) * 2.0f;  // theta_0 = pi (2 x - 1)
    if (gom_part) gom_part[b * HW + p] = dt * go[p];
  }
  if (gK_part) {
    red[threadIdx.x] = gk;
    __syncthreads();
    for (int w = kKThreads / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) gK_part[b] = dt * red[0];
  }
}

// out[j] = sum_b part[b, j] in a fixed order, two levels: 64 row slices x 4 row phases per column
// block (64 columns wide, coalesced), fp64 partials, then the 64 slices in order
constexpr int kColSlices = 64;
__global__ __launch_bounds__(256) void column_sum_part_kernel(const float* __restrict__ part, int64_t B, int n,
                                                              double* __restrict__ mid) {
  __shared__ double red[4][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  const int sl = blockIdx.y;
  const int64_t b0 = sl * B / kColSlices, b1 = (sl + 1) * B / kColSlices;
  double s = 0.0;
  if (j < n)
    for (int64_t b = b0 + ph; b < b1; b += 4) s += (double)part[b * n + j];
  red[ph][c] = s;
  __syncthreads();
  if (ph == 0 && j < n) mid[(int64_t)sl * n + j] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

__global__ void column_sum_final_kernel(const double* __restrict__ mid, int n, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int sl = 0; sl < kColSlices; ++sl) s += mid[(int64_t)sl * n + j];
  out[j] = (float)s;
}


// =============================================================================================
// Wide KANLinear head on MFMA (mnist_kuramoto_kan.py:127-142 at in = 1568, out = 10; SURVEY §8f
// rank 3: "the only place MFMA is justified").  out[b, o] = sum_i sum_f feat_f(x[b, i]) Wp[i, f, o]
// with the F = 1 + 8 + 8 features of one input — SiLU, the 8 cubic B-spline bases (4 nonzero),
// the 8 logistic bases — computed ONCE per (row, input) (the generic kernel recomputes them per
// output) and contracted on v_mfma_f32_16x16x4_f32: an exact f32 fma chain in k order.
//   A (16 rows x 4 k): lane (r = l & 15, kq = l >> 4) holds feature f of input 4 g + kq of row r;
//   B (4 k x 16 outputs): lane (kq, o) holds Wp[4 g + kq, f, o] (o >= out: 0), read from LDS;
//   one MFMA per (input group g, feature f).
// A 256-thread workgroup = 4 waves x 16 rows; the inputs are split over gridDim.y (split-K) into
// fixed chunks whose packed weights (and knots, reciprocal knot spans, logistic -a log2(e) / b)
// are staged in LDS for all 64 rows.  Partials (S, B, 16) are added in split order by a second
// kernel with the logistic bias.
// The features run on the transcendental unit directly (v_exp_f32, v_rcp_f32; 1 ulp each) and the
// Cox-de Boor divisions are products with the staged reciprocal spans: IEEE expf and divisions
// made ~650 VALU instructions per (row, input) and the head 385 us at B = 8192 (rocprofv3,
// profiles/r02_mnist_pmc.txt); the feature error stays ~1e-7 relative, far inside the 1e-5 test
// bar on the 1568 x 17-term sums.
// =============================================================================================
// FETODE_WIDE_SKIP (timing attribution; results wrong when set): diagnostic build only (make diag)
#if defined(FETODE_WIDE_SKIP) && !defined(FETODE_DIAG)
#error "FETODE_WIDE_SKIP is a diagnostic knob: build it with make diag"
#endif
#ifndef FETODE_WIDE_SKIP
#define FETODE_WIDE_SKIP 0
#endif
#ifndef FETODE_WIDE_CH
#define FETODE_WIDE_CH 8
#endif
constexpr int kWideCh = FETODE_WIDE_CH;  // inputs per staged chunk
constexpr int kWideNS = 8, kWideNB = 8, kWideNG = 12, kWideNI = kWideNG - 1;
constexpr int kWideF = 1 + kWideNS + kWideNB;
#ifndef FETODE_WIDE_WGS
#define FETODE_WIDE_WGS 2048
#endif
#ifndef FETODE_WIDE_ROWS
#define FETODE_WIDE_ROWS 64
#endif
constexpr int kWideRows = FETODE_WIDE_ROWS;  // rows per workgroup (16 per wave): the staged chunk serves them all
constexpr int kWideThreads = kWideRows * 4;
constexpr int kWideTab = kWideNI * 5;  // float4s per input of the basis table
constexpr int kWinStride = 20;         // per-lane dense-basis window (floats; b128 reads conflict-free)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Pack = [in][F][16] weights (f = 0 base, 1 + c scaled spline, 1 + NS + j 2 x scaled logistic:
// the basis is 2 sigmoid) followed by the per-input basis table [in][interval m][5] float4s: the
// four non-zero cubic B-splines B_{m-3+r} of interval m as power-basis cubics in u = (x - g_m) / h_m
// (fit in fp64 from the Cox-de Boor recursion restricted to the interval, efficientkan.py:117-131),
// then (g_m, 1 / h_m, 0, 0).
__global__ void wide_pack_kernel(fetode_kanlinear_t kl, float* __restrict__ wp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int in = kl.in_features, outf = kl.out_features;
  if (t >= (int64_t)in * kWideF * 16) return;
  const int o = t % 16, f = (t / 16) % kWideF, i = (int)(t / (16 * kWideF));
  float v = 0.f;
  if (o < outf) {
    if (f == 0) {
      v = kl.base_weight[(int64_t)o * in + i];
    } else if (f <= kWideNS) {
      const float sc = kl.spline_scaler ? kl.spline_scaler[(int64_t)o * in + i] : 1.0f;
      v = kl.spline_weight[((int64_t)o * in + i) * kWideNS + (f - 1)] * sc;
    } else if (kl.num_logistic) {
      const float lsc = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      v = 2.0f * ((kl.logistic_weight[(int64_t)o * in * kWideNB + i * kWideNB + (f - 1 - kWideNS)] * kl.scale_logistic) * lsc);
    }
  }
  wp[t] = v;
}

__global__ void wide_table_kernel(fetode_kanlinear_t kl, float4* __restrict__ tab) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kl.in_features * kWideNI) return;
  const int i = t / kWideNI, m = t % kWideNI;
  const float* g = kl.grid + (int64_t)i * kWideNG;
  const double h = (double)g[m + 1] - g[m];
  double v[4][4];
  for (int s = 0; s < 4; ++s) {  // the interval's bases at u = s / 3
    const double x = g[m] + h * (s / 3.0);
    double N[5] = {0, 0, 0, 1, 0};
    for (int k = 1; k <= 3; ++k) {
      double M[5] = {0, 0, 0, 0, 0};
      for (int r = 3 - k; r <= 3; ++r) {
        const int j = m - 3 + r;
        if (j >= 0 && j <= kWideNG - 2 - k)
          M[r] = (x - g[j]) / ((double)g[j + k] - g[j]) * N[r] +
                 ((double)g[j + k + 1] - x) / ((double)g[j + k + 1] - g[j + 1]) * N[r + 1];
      }
      for (int r = 0; r < 5; ++r) N[r] = M[r];
    }
    for (int r = 0; r < 4; ++r) v[s][r] = N[r];
  }
  float4* out = tab + (int64_t)t * 5;
  for (int r = 0; r < 4; ++r) {  // cubic through (0, v0), (1/3, v1), (2/3, v2), (1, v3) in power basis
    const double a0 = v[0][r], a1 = v[1][r], a2 = v[2][r], a3 = v[3][r];
    out[r] = make_float4((float)a0, (float)((-11.0 * a0 + 18.0 * a1 - 9.0 * a2 + 2.0 * a3) / 2.0),
                         (float)(9.0 * (2.0 * a0 - 5.0 * a1 + 4.0 * a2 - a3) / 2.0),
                         (float)(9.0 * (-a0 + 3.0 * a1 - 3.0 * a2 + a3) / 2.0));
  }
  out[4] = make_float4(g[m], 1.0f / (g[m + 1] - g[m]), 0.f, 0.f);
}

// Per (row, input) the 17 features are formed once and contracted on v_mfma_f32_16x16x4_f32:
//   SiLU; the knot interval m (12 compares), u, the 4 non-zero bases as Horner cubics from the
//   table, placed into the dense 8 through the lane's LDS window (4 b32 writes at m + r, two b128
//   reads, 4 zeroing writes: runtime-indexed placement without select chains); the 8 logistic
//   sigmoids as 1 / (1 + 2^(-a log2e x + a b log2e)) (the 2 is in the packed weights).
__global__ __launch_bounds__(kWideThreads) void wide_fwd_kernel(fetode_kanlinear_t kl, const float* __restrict__ wp,
                                                      const float* __restrict__ x, int64_t B, int nch,
                                                      float* __restrict__ part) {
  __shared__ float ws[kWideCh * kWideF * 16];   // packed weights of the chunk
  __shared__ float xs[kWideRows][kWideCh + 1];  // the rows' inputs of the chunk
  __shared__ float4 gk[kWideCh][kWideNG / 4];   // knots
  __shared__ float4 tb[kWideCh * kWideTab];     // basis tables of the chunk's inputs
  __shared__ float2 lab[kWideCh][kWideNB];      // logistic (-a log2e, a b log2e)
  __shared__ __attribute__((aligned(16))) float win[kWideThreads * kWinStride];  // per-lane dense-basis window
  const int in = kl.in_features;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * kWideRows;
  const int S = gridDim.y, s = blockIdx.y;
  const int c0 = s * nch / S, c1 = (s + 1) * nch / S;
  const bool lg = kl.num_logistic != 0;
  const float4* wtab = reinterpret_cast<const float4*>(wp + (int64_t)in * kWideF * 16);
  float* mywin = win + tid * kWinStride;  // [0, 16): window slot m + r + 1 holds B_{m-3+r}; dense c at 4 + c
  for (int q = 0; q < kWinStride; ++q) mywin[q] = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // chunk c's global data is fetched into registers while chunk c - 1 is contracted
  constexpr int PW = (kWideCh * kWideF * 16 + kWideThreads - 1) / kWideThreads, PX = (kWideRows * kWideCh + kWideThreads - 1) / kWideThreads;
  constexpr int PT = (kWideCh * kWideTab + kWideThreads - 1) / kWideThreads, PG = (kWideCh * kWideNG + kWideThreads - 1) / kWideThreads;
  constexpr int PL = (kWideCh * kWideNB + kWideThreads - 1) / kWideThreads;
  float rw[PW], rx[PX], rg[PG], ra[PL], rb[PL];
  float4 rt[PT];
  auto fetch = [&](int c) __attribute__((always_inline)) {
    const int i0 = c * kWideCh, ni = min(kWideCh, in - i0);
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      const int t = tid + kWideThreads * k;
      rw[k] = t < ni * kWideF * 16 ? wp[(int64_t)i0 * kWideF * 16 + t] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int t = tid + kWideThreads * k, rr = t / kWideCh, ii = t - rr * kWideCh;
      rx[k] = (t < kWideRows * kWideCh && row0 + rr < B && ii < ni) ? x[(row0 + rr) * in + i0 + ii] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int t = tid + kWideThreads * k;
      rt[k] = t < ni * kWideTab ? wtab[(int64_t)i0 * kWideTab + t] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < PG; ++k) {
      const int t = tid + kWideThreads * k;
      rg[k] = t < ni * kWideNG ? kl.grid[(int64_t)i0 * kWideNG + t] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int t = tid + kWideThreads * k;
      const bool ok = lg && t < ni * kWideNB;
      ra[k] = ok ? kl.logistic_a[(int64_t)i0 * kWideNB + t] : 0.f;
      rb[k] = ok ? kl.logistic_b[(int64_t)i0 * kWideNB + t] : 0.f;
    }
  };
  if (c0 < c1) fetch(c0);
  for (int c = c0; c < c1; ++c) {
    const int i0 = c * kWideCh, ni = min(kWideCh, in - i0);
    __syncthreads();  // the previous chunk's contraction is done with the LDS copies
#pragma unroll
    for (int k = 0; k < PW; ++k)
      if (tid + kWideThreads * k < kWideCh * kWideF * 16) ws[tid + kWideThreads * k] = rw[k];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int t = tid + kWideThreads * k, rr = t / kWideCh, ii = t - rr * kWideCh;
      if (t < kWideRows * kWideCh) xs[rr][ii] = rx[k];
    }
#pragma unroll
    for (int k = 0; k < PT; ++k)
      if (tid + kWideThreads * k < kWideCh * kWideTab) tb[tid + kWideThreads * k] = rt[k];
#pragma unroll
    for (int k = 0; k < PG; ++k)
      if (tid + kWideThreads * k < kWideCh * kWideNG) reinterpret_cast<float*>(&gk[0][0])[tid + kWideThreads * k] = rg[k];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int t = tid + kWideThreads * k;
      if (t < kWideCh * kWideNB) lab[t / kWideNB][t % kWideNB] = make_float2(-ra[k] * FETODE_LOG2E, (ra[k] * rb[k]) * FETODE_LOG2E);
    }
    __syncthreads();
    if (c + 1 < c1) fetch(c + 1);
    for (int g = 0; g < ni / 4; ++g) {
      const int il = 4 * g + kq;
      const float xi = xs[wv * 16 + r][il];
      float feat[kWideF];
#if FETODE_WIDE_SKIP & 2  // diagnostics: MFMAs only
#pragma unroll
      for (int f = 0; f < kWideF; ++f) feat[f] = xi * (float)(f + 1);
      if (0)
#endif
      {
      feat[0] = silu(xi);  // SiLU, efficientkan.py:166 / mnist :131
      int m = -1;
#pragma unroll
      for (int j = 0; j < kWideNG / 4; ++j) {
        const float4 v = gk[il][j];
        m += ((xi >= v.x) ? 1 : 0) + ((xi >= v.y) ? 1 : 0) + ((xi >= v.z) ? 1 : 0) + ((xi >= v.w) ? 1 : 0);
      }
      const bool fin = __builtin_isfinite(xi), ing = fin && m >= 0 && m < kWideNI;
      const float4* tm = &tb[il * kWideTab + (ing ? m : 0) * 5];
      const float4 gr = tm[4];
      const float u = (xi - gr.x) * gr.y;
      if (ing) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 p = tm[q];
          mywin[m + q + 1] = ffma(ffma(ffma(p.w, u, p.z), u, p.y), u, p.x);
        }
      }
      asm volatile("" ::: "memory");  // the window writes stay before the vector reads
      {
        const float4 d0 = *reinterpret_cast<const float4*>(mywin + 4), d1 = *reinterpret_cast<const float4*>(mywin + 8);
        const float nf = fin ? 0.f : __builtin_nanf("");  // non-finite x: NaN bases, as (x - g) / d * 0
        feat[1] = d0.x + nf; feat[2] = d0.y + nf; feat[3] = d0.z + nf; feat[4] = d0.w + nf;
        feat[5] = d1.x + nf; feat[6] = d1.y + nf; feat[7] = d1.z + nf; feat[8] = d1.w + nf;
      }
      asm volatile("" ::: "memory");
      if (ing) {
#pragma unroll
        for (int q = 0; q < 4; ++q) mywin[m + q + 1] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < kWideNB; ++j) {  // 2 sigmoid(a (x - b)), mnist_kuramoto_kan.py:22 (2 in the weights)
        const float2 ab = lab[il][j];
        feat[1 + kWideNS + j] = lg ? rcp(1.0f + ex2(ffma(ab.x, xi, ab.y))) : 0.f;
      }
      }
      const float* wrow = ws + (il * kWideF) * 16 + r;   // lane (kq, o = r): Wp[i, f, o]
#if FETODE_WIDE_SKIP & 1  // diagnostics: features only
#pragma unroll
      for (int f = 0; f < kWideF; ++f) acc[f & 3] += feat[f] * wrow[f * 16];
#else
#pragma unroll
      for (int f = 0; f < kWideF; ++f) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(feat[f], wrow[f * 16], acc, 0, 0, 0);
#endif
    }
  }
  // D: lane l holds rows 4 (l >> 4) + v, column l & 15
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int64_t row = row0 + wv * 16 + 4 * kq + v;
    if (row < B) part[((int64_t)s * B + row) * 16 + r] = acc[v];
  }
}

// wide_fwd4_kernel (the default): the same contraction, each wave on FOUR 16-row tiles (64 rows; a
// 256-thread workgroup = 256 rows).  Per input group the lane's per-input data — its knots,
// logistic (a, b) and the 17 B operands Wp[4 g + kq, f, r] — is read from LDS once and serves the
// four tiles (per-(row, input) LDS operations 44 -> 23), the four tiles' features are formed first
// and the MFMAs issued round-robin over four independent accumulators.  Same chunks, splits and
// per-tile accumulation order as wide_fwd_kernel: bitwise the same partials.  Measured B = 8192
// (tools/diag/mnist_head_time.py): 147.0 -> 140.6 us per head forward; PMC
// (profiles/r04_h_pmc_issue.json): LDS-busy 0.59 -> 0.29, VALU-busy 0.36, MFMA-busy 0.32, 47 % of
// wave cycles issue-stalled — the head is bound by its VALU feature work and MFMAs taking turns,
// not by LDS; a software-pipelined variant (tile t + 1's features between tile t's MFMAs, branch-
// free window) measured 142.7 us and was not kept.
constexpr int kW4Rows = 256;
__global__ __launch_bounds__(256) void wide_fwd4_kernel(fetode_kanlinear_t kl, const float* __restrict__ wp,
                                                       const float* __restrict__ x, int64_t B, int nch,
                                                       float* __restrict__ part) {
  __shared__ float ws[kWideCh * kWideF * 16];
  __shared__ float xs[kW4Rows][kWideCh + 1];
  __shared__ float4 gk[kWideCh][kWideNG / 4];
  __shared__ float4 tb[kWideCh * kWideTab];
  __shared__ float2 lab[kWideCh][kWideNB];
  // per-lane dense-basis window, position-major ([pos][tid]): a lane's writes at its interval's
  // positions m + 1 .. m + 4 hit bank tid % 32 whatever m is (lane-major at a 20-float stride they
  // collided: 45 % of the head's LDS cycles were conflicts, profiles/r06_lds_mnist.txt)
  constexpr int kWinPos = 16;   // positions 0 .. 15: slot m + r + 1 holds B_{m-3+r}; dense c at 4 + c
  __shared__ float win[kWinPos * 256];
  const int in = kl.in_features;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * kW4Rows;
  const int S = gridDim.y, s = blockIdx.y;
  const int c0 = s * nch / S, c1 = (s + 1) * nch / S;
  const bool lg = kl.num_logistic != 0;
  const float4* wtab = reinterpret_cast<const float4*>(wp + (int64_t)in * kWideF * 16);
  float* mywin = win + tid;   // position q at mywin[256 q]
  for (int q = 0; q < kWinPos; ++q) mywin[256 * q] = 0.f;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PW = (kWideCh * kWideF * 16 + 255) / 256, PX = (kW4Rows * kWideCh + 255) / 256;
  constexpr int PT = (kWideCh * kWideTab + 255) / 256, PG = (kWideCh * kWideNG + 255) / 256;
  constexpr int PL = (kWideCh * kWideNB + 255) / 256;
  float rw[PW], rx[PX], rg[PG], ra[PL], rb[PL];
  float4 rt[PT];
  auto fetch = [&](int c) __attribute__((always_inline)) {
    const int i0 = c * kWideCh, ni = min(kWideCh, in - i0);
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      const int t = tid + 256 * k;
      rw[k] = t < ni * kWideF * 16 ? wp[(int64_t)i0 * kWideF * 16 + t] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int t = tid + 256 * k, rr = t / kWideCh, ii = t - rr * kWideCh;
      rx[k] = (t < kW4Rows * kWideCh && row0 + rr < B && ii < ni) ? x[(row0 + rr) * in + i0 + ii] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int t = tid + 256 * k;
      rt[k] = t < ni * kWideTab ? wtab[(int64_t)i0 * kWideTab + t] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < PG; ++k) {
      const int t = tid + 256 * k;
      rg[k] = t < ni * kWideNG ? kl.grid[(int64_t)i0 * kWideNG + t] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int t = tid + 256 * k;
      const bool ok = lg && t < ni * kWideNB;
      ra[k] = ok ? kl.logistic_a[(int64_t)i0 * kWideNB + t] : 0.f;
      rb[k] = ok ? kl.logistic_b[(int64_t)i0 * kWideNB + t] : 0.f;
    }
  };
  if (c0 < c1) fetch(c0);
  for (int c = c0; c < c1; ++c) {
    const int ni = min(kWideCh, in - c * kWideCh);
    __syncthreads();  // the previous chunk's contraction is done with the LDS copies
#pragma unroll
    for (int k = 0; k < PW; ++k)
      if (tid + 256 * k < kWideCh * kWideF * 16) ws[tid + 256 * k] = rw[k];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int t = tid + 256 * k, rr = t / kWideCh, ii = t - rr * kWideCh;
      if (t < kW4Rows * kWideCh) xs[rr][ii] = rx[k];
    }
#pragma unroll
    for (int k = 0; k < PT; ++k)
      if (tid + 256 * k < kWideCh * kWideTab) tb[tid + 256 * k] = rt[k];
#pragma unroll
    for (int k = 0; k < PG; ++k)
      if (tid + 256 * k < kWideCh * kWideNG) reinterpret_cast<float*>(&gk[0][0])[tid + 256 * k] = rg[k];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int t = tid + 256 * k;
      if (t < kWideCh * kWideNB) lab[t / kWideNB][t % kWideNB] = make_float2(-ra[k] * FETODE_LOG2E, (ra[k] * rb[k]) * FETODE_LOG2E);
    }
    __syncthreads();
    if (c + 1 < c1) fetch(c + 1);
    for (int g = 0; g < ni / 4; ++g) {
      const int il = 4 * g + kq;
      // the lane's input: knots, logistic (a, b), B operands — once for the four row tiles
      float4 gr4[kWideNG / 4];
#pragma unroll
      for (int j = 0; j < kWideNG / 4; ++j) gr4[j] = gk[il][j];
      float2 ab[kWideNB];
#pragma unroll
      for (int j = 0; j < kWideNB; ++j) ab[j] = lab[il][j];
      float wb[kWideF];
      const float* wrow = ws + (il * kWideF) * 16 + r;  // lane (kq, o = r): Wp[i, f, o]
#pragma unroll
      for (int f = 0; f < kWideF; ++f) wb[f] = wrow[f * 16];
      const float4* tbi = &tb[il * kWideTab];
      // features of row tile t (lane row 16 t + r, input il) into feat[]
      auto feats = [&](int t, float* feat) __attribute__((always_inline)) {
        const float xi = xs[wv * 64 + 16 * t + r][il];
        feat[0] = silu(xi);  // SiLU, efficientkan.py:166 / mnist :131
        // knot count: one v_cmp + one carry-in add per knot (no select + add)
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < kWideNG / 4; ++j) {
          const float kv[4] = {gr4[j].x, gr4[j].y, gr4[j].z, gr4[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            asm volatile("v_cmp_ge_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(cnt) : "v"(xi), "v"(kv[q]) : "vcc");
        }
        const int m = cnt - 1;
        const bool fin = __builtin_isfinite(xi), ing = fin && m >= 0 && m < kWideNI;
        const float4* tm = tbi + (ing ? m : 0) * 5;
        const float4 gq = tm[4];
        const float u = (xi - gq.x) * gq.y;
        if (ing) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 p = tm[q];
            mywin[256 * (m + q + 1)] = ffma(ffma(ffma(p.w, u, p.z), u, p.y), u, p.x);
          }
        }
        if (!fin) {   // non-finite x (rare): NaN bases, as (x - g) / d * 0 in the reference
#pragma unroll
          for (int q = 4; q < 12; ++q) mywin[256 * q] = __builtin_nanf("");
        }
        asm volatile("" ::: "memory");  // the window writes stay before the vector reads
#pragma unroll
        for (int c = 0; c < kWideNS; ++c) feat[1 + c] = mywin[256 * (4 + c)];
        asm volatile("" ::: "memory");
        if (ing) {
#pragma unroll
          for (int q = 0; q < 4; ++q) mywin[256 * (m + q + 1)] = 0.f;
        }
        if (!fin) {
#pragma unroll
          for (int q = 4; q < 12; ++q) mywin[256 * q] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < kWideNB; ++j)  // 2 sigmoid(a (x - b)), mnist_kuramoto_kan.py:22 (2 in the weights)
        feat[1 + kWideNS + j] = lg ? rcp(1.0f + ex2(ffma(ab[j].x, xi, ab[j].y))) : 0.f;
      };
      // tiles whose features are held at once (measured, tools/diag/mnist_head_time.py: 4 / 2 / 1 =
      // 136 / 135 / 144 us; forcing 3 waves per SIMD spills 27-48 VGPRs: 167-202 us)
      constexpr int TP = 4;
#pragma unroll
      for (int t0 = 0; t0 < 4; t0 += TP) {
        float ft[TP][kWideF];   // TP tiles' features first: then TP independent MFMA chains
#pragma unroll
        for (int t = 0; t < TP; ++t) feats(t0 + t, ft[t]);
#pragma unroll
        for (int f = 0; f < kWideF; ++f)
#pragma unroll
          for (int t = 0; t < TP; ++t)
            acc[t0 + t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ft[t][f], wb[f], acc[t0 + t], 0, 0, 0);
      }
    }
  }
  // D of tile t: lane l holds rows 16 t + 4 (l >> 4) + v, column l & 15
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t row = row0 + wv * 64 + 16 * t + 4 * kq + v;
      if (row < B) part[((int64_t)s * B + row) * 16 + r] = acc[t][v];
    }
}

__global__ void wide_reduce_kernel(const float* __restrict__ part, int S, int64_t B, int outf,
                                   const float* __restrict__ bias, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * outf) return;
  const int64_t b = t / outf;
  const int o = t % outf;
  float v = part[b * 16 + o];
  for (int s = 1; s < S; ++s) v = v + part[((int64_t)s * B + b) * 16 + o];
  out[t] = bias ? v + bias[o] : v;
}

// the LDS (workgroup-per-image) Kuramoto kernels for every shape: FETODE_KURA_LDS=1 (A/B and the
// cross-check test), or fetode_kuramoto_set_lds(1)
int g_kura_lds = [] {
  const char* e = getenv("FETODE_KURA_LDS");
  return e ? atoi(e) : 0;
}();
bool kura_lds_forced() { return g_kura_lds != 0; }

int wide_supported(const fetode_kanlinear_t* kl) {
  return kl && kl->spline_order == 3 && kl->grid_size == 5 && (kl->num_logistic == 0 || kl->num_logistic == kWideNB) &&
         kl->out_features >= 1 && kl->out_features <= 16 && kl->in_features >= 4 && kl->in_features % 4 == 0 &&
         kl->grid && kl->base_weight && kl->spline_weight && (kl->num_logistic == 0 ||
         (kl->logistic_a && kl->logistic_b && kl->logistic_weight));
}

int wide_splits(const fetode_kanlinear_t* kl, int64_t B) {
  const int nch = (kl->in_features + kWideCh - 1) / kWideCh;
  const int64_t tiles = (B + kWideRows - 1) / kWideRows;
  int64_t S = (FETODE_WIDE_WGS + tiles - 1) / tiles;   // aim at >= FETODE_WIDE_WGS workgroups
  if (S > nch) S = nch;
  return (int)(S < 1 ? 1 : S);
}

}  // namespace

extern "C" {

int fetode_kuramoto_forward(const float* x, int64_t B, int32_t H, int32_t W, int32_t steps, float dt, const float* K,
                            const float* omega, float* feat, float* tape, void* stream) {
  if (B <= 0) return FETODE_OK;
  if (!x || !K || !omega || !feat) return set_err(FETODE_EINVAL, "kuramoto: null pointer");
  if (H <= 0 || W <= 0 || H * W > kMaxPix || steps < 0)
    return set_err(FETODE_EINVAL, "kuramoto: H*W=%d (1..%d), steps=%d", H * W, kMaxPix, steps);
  if (H == 28 && W < 32 && !kura_lds_forced()) {  // lane per column (MNIST 28 x 28); lane 31 of each image stays empty
    const unsigned grid = (unsigned)((B + 2 * kLaneWaves - 1) / (2 * kLaneWaves));
    hipLaunchKernelGGL(kuramoto_fwd_lanes_kernel<28>, dim3(grid), dim3(64 * kLaneWaves), 0, (hipStream_t)stream, x, B,
                       W, steps, dt, K, omega, feat, tape);
    LAUNCH_CHECK();
    return FETODE_OK;
  }
  const size_t lds = sizeof(float) * 3 * H * W;
  hipLaunchKernelGGL(kuramoto_fwd_kernel, dim3((unsigned)B), dim3(kKThreads), lds, (hipStream_t)stream, x, H, W, steps,
                     dt, K, omega, feat, tape);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int fetode_kuramoto_set_lds(int on) {
  const int prev = g_kura_lds;
  if (on >= 0) g_kura_lds = on;
  return prev;
}

int64_t fetode_kuramoto_backward_workspace(int64_t B, int32_t H, int32_t W) {
  // per-image partials (d omega, d K) + fp64 slice sums of both
  return (int64_t)sizeof(float) * B * ((int64_t)H * W + 1) + (int64_t)sizeof(double) * kColSlices * ((int64_t)H * W + 1) + 16;
}

int fetode_kuramoto_backward(int64_t B, int32_t H, int32_t W, int32_t steps, float dt, const float* K,
                             const float* tape, const float* gfeat, float* gx, float* gK, float* gomega,
                             void* workspace, void* stream) {
  if (B <= 0) return FETODE_OK;
  if (!K || !tape || !gfeat) return set_err(FETODE_EINVAL, "kuramoto backward: null pointer");
  if (H <= 0 || W <= 0 || H * W > kMaxPix || steps < 0)
    return set_err(FETODE_EINVAL, "kuramoto backward: H*W=%d (1..%d), steps=%d", H * W, kMaxPix, steps);
  if ((gK || gomega) && !workspace) return set_err(FETODE_EINVAL, "kuramoto backward: workspace required");
  const int HW = H * W;
  float* gom_part = gomega ? (float*)workspace : nullptr;
  float* gK_part = gK ? (float*)workspace + B * HW : nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (H == 28 && W < 32 && !kura_lds_forced()) {
    const unsigned grid = (unsigned)((B + 2 * kLaneWaves - 1) / (2 * kLaneWaves));
    hipLaunchKernelGGL(kuramoto_bwd_lanes_kernel<28>, dim3(grid), dim3(64 * kLaneWaves), 0, s, B, W, steps, dt, K, tape,
                       gfeat, gx, gK_part, gom_part);
  } else {
    const size_t lds = sizeof(float) * 4 * HW;
    hipLaunchKernelGGL(kuramoto_bwd_kernel, dim3((unsigned)B), dim3(kKThreads), lds, s, H, W, steps, dt, K, tape, gfeat,
                       gx, gK_part, gom_part);
  }
  LAUNCH_CHECK();
  // fp64 slice sums, 8-byte aligned after the float partials
  const int64_t fl = B * ((int64_t)HW + 1);
  double* mid = (double*)((char*)workspace + ((sizeof(float) * fl + 15) & ~(size_t)15));
  if (gomega) {
    hipLaunchKernelGGL(column_sum_part_kernel, dim3((HW + 63) / 64, kColSlices), dim3(256), 0, s, gom_part, B, HW, mid);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(column_sum_final_kernel, dim3((HW + 255) / 256), dim3(256), 0, s, mid, HW, gomega);
    LAUNCH_CHECK();
  }
  if (gK) {
    double* midk = mid + (int64_t)kColSlices * HW;
    hipLaunchKernelGGL(column_sum_part_kernel, dim3(1, kColSlices), dim3(256), 0, s, gK_part, B, 1, midk);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(column_sum_final_kernel, dim3(1), dim3(256), 0, s, midk, 1, gK);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int fetode_kanlinear_wide_supported(const fetode_kanlinear_t* kl) { return wide_supported(kl); }

int64_t fetode_kanlinear_wide_pack_bytes(const fetode_kanlinear_t* kl) {
  return kl ? (int64_t)sizeof(float) * kl->in_features * (kWideF * 16 + 4 * kWideTab) : 0;
}

int fetode_kanlinear_wide_pack(const fetode_kanlinear_t* kl, float* wpack, void* stream) {
  if (!wide_supported(kl)) return set_err(FETODE_EUNSUPPORTED, "kanlinear wide: unsupported layer");
  if (!wpack) return set_err(FETODE_EINVAL, "kanlinear wide: null pack");
  const int64_t n = (int64_t)kl->in_features * kWideF * 16;
  hipLaunchKernelGGL(wide_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *kl, wpack);
  LAUNCH_CHECK();
  const int nt = kl->in_features * kWideNI;
  hipLaunchKernelGGL(wide_table_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *kl,
                     reinterpret_cast<float4*>(wpack + n));
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_kanlinear_wide_workspace(const fetode_kanlinear_t* kl, int64_t B) {
  if (!kl || B <= 0) return 0;
  return (int64_t)sizeof(float) * wide_splits(kl, B) * B * 16;
}

int fetode_kanlinear_wide_forward(const fetode_kanlinear_t* kl, const float* wpack, const float* bias, const float* x,
                                  int64_t B, float* out, void* workspace, void* stream) {
  if (!wide_supported(kl)) return set_err(FETODE_EUNSUPPORTED, "kanlinear wide: unsupported layer");
  if (B <= 0) return FETODE_OK;
  if (!wpack || !x || !out || !workspace) return set_err(FETODE_EINVAL, "kanlinear wide: null pointer");
  const int S = wide_splits(kl, B);
  const int nch = (kl->in_features + kWideCh - 1) / kWideCh;
  const int64_t tiles = (B + kWideRows - 1) / kWideRows;
  if (tiles > 0x7fffffff) return set_err(FETODE_EINVAL, "kanlinear wide: batch too large");
  hipStream_t s = (hipStream_t)stream;
  static const int v1 = [] {  // FETODE_WIDE_V=1: wide_fwd_kernel, one tile per wave (A/B, bitwise the same)
    const char* e = getenv("FETODE_WIDE_V");
    return e ? atoi(e) : 0;
  }();
  if (v1 == 1) {
    hipLaunchKernelGGL(wide_fwd_kernel, dim3((unsigned)tiles, (unsigned)S), dim3(kWideThreads), 0, s, *kl, wpack, x, B,
                       nch, (float*)workspace);
  } else {
    const int64_t t4 = (B + kW4Rows - 1) / kW4Rows;
    hipLaunchKernelGGL(wide_fwd4_kernel, dim3((unsigned)t4, (unsigned)S),
                       dim3(256), 0, s, *kl, wpack, x, B, nch, (float*)workspace);
  }
  LAUNCH_CHECK();
  const int64_t n = B * kl->out_features;
  hipLaunchKernelGGL(wide_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)workspace, S, B,
                     kl->out_features, bias, out);
  LAUNCH_CHECK();
  return FETODE_OK;
}

}  // extern "C"
