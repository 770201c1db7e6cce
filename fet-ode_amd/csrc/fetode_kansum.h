// fetode_kansum.h — the KAN parameter-gradient sums of the [2, 10, 2] KAN-FET reverse sweep, formed
// after sweep7_kernel<KS = false> over all (evaluation, trajectory) samples in parallel.  Included
// inside fetode_bwd.hip's anonymous namespace after fetode_sweep7.h (namespace s7's shape).
//
// The KAN sums are linear in the layer's output adjoints and need only the layer's input, both of
// which the sweep leaves behind: the tape row (x | h) and the gadj row (g_0, g_1 | d loss / d h).
// Per sample s and layer input t with output adjoints g_d (efficientkan.py:160-182 differentiated,
// the sums fixed_bwd_kernel keeps per lane):
//   G_d += g_d,  base(d, t) += g_d SiLU(x_t),  spline(d, t, c) += g_d B_c(x_t),
//   lw(d, t, j) += g_d s_tj,  s_tj = sigmoid(a_tj (x_t - b_tj)),
//   T_tj = s_tj (1 - s_tj) sum_d g_d kw(d, t, j):  la(t, j) += T_tj (x_t - b_tj),  lb(t, j) += -a_tj T_tj
// (la, lb kept as P = sum T x and Q = sum T: la = P - b Q, lb = -a Q at the end).
// One workgroup = 10 waves over one sample range; blockIdx.y = the layer.  Layer 1: wave o = hidden
// input o, outputs d = 0, 1.  Layer 0: wave (i, p) = input i, outputs 2p, 2p + 1 (the T sums of a
// pair of outputs are partial: the five pairs' are added in LDS in order).  A lane walks every 64th
// sample of the range with its 62 sums in VGPRs; the interval's four basis values reach the dense
// eight through a per-lane LDS window (as the MNIST head, fetode_mnist.hip).  The per-wave lane sums
// (DPP row sums, then the four rows in order) go to the block's partial row in the AccLayout of
// fixed_bwd_kernel; the block writes zeros into its layer's Ferro slots (the sweep's rows hold them).
#pragma once

namespace s7 {
constexpr int kKsWaves = 10;       // waves per workgroup
constexpr int kKsRows = 256;       // workgroups per layer (= partial rows; both layers share them)
constexpr int kKsWin = 20;         // per-lane window pitch (floats): bases at [4, 12), b128 reads
}  // namespace s7

__global__ __launch_bounds__(64 * s7::kKsWaves) void kansum_kernel(BwdArgs a) {
  using namespace s7;
  using L0 = BL<D, H, K, NB, NG, true>;
  using L1 = BL<H, D, K, NB, NG, true>;
  constexpr AccLayout A0L = L0::AL, A1L = L1::AL;
  __shared__ BInTab<W, NG, NB> TI;
  __shared__ __attribute__((aligned(16))) float win[64 * kKsWaves * kKsWin];
  __shared__ float red[kKsWaves][2 * NB];          // layer 0: the output pairs' P, Q partials
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int layer = blockIdx.y;
  TI.stage(a.plan, a.P0, a.P1, D, tid, 64 * kKsWaves);
  float* mw = &win[tid * kKsWin];
#pragma unroll
  for (int q = 0; q < kKsWin; ++q) mw[q] = 0.f;
  // this wave's input (combined tape column t) and output pair
  const int wu = __builtin_amdgcn_readfirstlane(wv);
  const int t = layer == 1 ? D + wu : wu / (H / 2);        // layer 0: waves 0-4 input 0, 5-9 input 1
  const int pr = layer == 1 ? 0 : wu % (H / 2);            // layer 0: output pair (2 pr, 2 pr + 1)
  const int gcol = layer == 1 ? 0 : D + 2 * pr;            // the pair's adjoints in a gadj row
  const LayerPlan& P = layer == 1 ? a.P1 : a.P0;
  const int ti = layer == 1 ? t - D : t;                   // input index within the layer
  const int IN = layer == 1 ? H : D;
  // the pair's logistic weights kw(d, t, j) (plan layout [out][in][NFL], 1 + j)
  float kwp[2][NB];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int oo = layer == 1 ? d : 2 * pr + d;
      kwp[d][j] = a.plan[P.kw + (oo * IN + ti) * NFL + 1 + j];
    }
  __syncthreads();

  const int ns = a.method == FETODE_RK4 || a.method == FETODE_RK4_CLASSIC ? 4 : a.method == FETODE_MIDPOINT ? 2 : 1;
  const int64_t N = (int64_t)a.n_steps * ns * a.B;
  const int64_t n0 = (int64_t)blockIdx.x * N / gridDim.x, n1 = (int64_t)(blockIdx.x + 1) * N / gridDim.x;
  float G[2] = {0.f, 0.f}, bs[2] = {0.f, 0.f}, sp[2][NS], lw[2][NB], Pq[NB], Qq[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) lw[0][j] = lw[1][j] = Pq[j] = Qq[j] = 0.f;
#pragma unroll
  for (int c = 0; c < NS; ++c) sp[0][c] = sp[1][c] = 0.f;
  const float* kn = &TI.knots[t * NG];
  for (int64_t n = n0 + lane; n < n1; n += 64) {
    const float x = a.tape[n * W + t];
    const float g0 = a.gadj[n * W + gcol], g1 = a.gadj[n * W + gcol + 1];
    G[0] += g0;
    G[1] += g1;
    // SiLU
    const float sx = rcp(1.0f + ex2(-x * FETODE_LOG2E));
    const float silu = x * sx;
    bs[0] = ffma(g0, silu, bs[0]);
    bs[1] = ffma(g1, silu, bs[1]);
    // interval and the four bases through the window
    int m = -1;
#pragma unroll
    for (int jj = 0; jj < NG; ++jj) m += x >= kn[jj] ? 1 : 0;
    const bool fin = __builtin_isfinite(x), in = fin && (unsigned)m < (unsigned)NI;
    const int mc = in ? m : 0;
    const float u = (x - kn[mc]) * TI.rh[t * NI + mc];
    const float4* bp = &TI.bp[TI.bpi(t, mc)];
    if (in) {
#pragma unroll
      for (int r = 0; r <= kSO; ++r) {
        const float4 c = bp[r];
        mw[mc + 1 + r] = ffma(ffma(ffma(c.w, u, c.z), u, c.y), u, c.x);   // basis m - 3 + r at [4 + m - 3 + r]
      }
    }
    asm volatile("" ::: "memory");
    {
      const float4 d0 = *reinterpret_cast<const float4*>(mw + 4), d1 = *reinterpret_cast<const float4*>(mw + 8);
      const float nf = fin ? 0.f : __builtin_nanf("");   // non-finite x: NaN bases (the reference's)
      const float bv[NS] = {d0.x + nf, d0.y + nf, d0.z + nf, d0.w + nf, d1.x + nf, d1.y + nf, d1.z + nf, d1.w + nf};
#pragma unroll
      for (int c = 0; c < NS; ++c) {
        sp[0][c] = ffma(g0, bv[c], sp[0][c]);
        sp[1][c] = ffma(g1, bv[c], sp[1][c]);
      }
    }
    asm volatile("" ::: "memory");
    if (in) {
#pragma unroll
      for (int r = 0; r <= kSO; ++r) mw[mc + 1 + r] = 0.f;
    }
    // logistic bases
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const float2 ab = *reinterpret_cast<const float2*>(&TI.lg[2 * (t * NB + j)]);
      const float sg = rcp(1.0f + ex2(ffma(ab.x, x, ab.y)));
      lw[0][j] = ffma(g0, sg, lw[0][j]);
      lw[1][j] = ffma(g1, sg, lw[1][j]);
      const float T = ffma(g0, kwp[0][j], g1 * kwp[1][j]) * ffma(-sg, sg, sg);
      Pq[j] = ffma(T, x, Pq[j]);
      Qq[j] += T;
    }
  }
  static_assert(NS == 8 && NFL == NB + 1, "kansum_kernel layout");

  // ---- the wave's sums (64 lanes, fixed order) -> this block's partial row ----
  auto wsum = [&](float v) {
    v += dpp<0x128>(v);
    v += dpp<0x124>(v);
    v += dpp<0x122>(v);
    v += dpp<0x121>(v);   // each lane: its row's sum
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return ((r0 + r1) + r2) + r3;
  };
  float* row = a.part + (int64_t)blockIdx.x * a.nacc + (layer == 1 ? A0L.n : 0);
  const AccLayout AL = layer == 1 ? A1L : A0L;
  for (int i = tid; i < 3 * AL.E; i += 64 * kKsWaves) row[AL.oA + i] = 0.f;   // the Ferro slots
  // (every sum is reduced by all lanes; lane 0 stores)
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const int oo = layer == 1 ? d : 2 * pr + d;               // the output
    const float vg = wsum(G[d]), vb = wsum(bs[d]);
    if (lane == 0) {
      if (ti == 0) row[AL.oG + oo] = vg;                       // one wave per output
      row[AL.oBase + oo * IN + ti] = vb;
    }
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      const float v = wsum(sp[d][c]);
      if (lane == 0) row[AL.oSpl + (oo * IN + ti) * NS + c] = v;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const float v = wsum(lw[d][j]);
      if (lane == 0) row[AL.oLw + oo * AL.NL + ti * NB + j] = v;
    }
  }
  // la = P - b Q, lb = -a Q (layer 0: the five output pairs' P, Q added in order first)
  float Pw[NB], Qw[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    Pw[j] = wsum(Pq[j]);
    Qw[j] = wsum(Qq[j]);
  }
  const float* la_ = layer == 1 ? a.k1.logistic_a : a.k0.logistic_a;
  const float* lb_ = layer == 1 ? a.k1.logistic_b : a.k0.logistic_b;
  if (layer == 1) {
    if (lane < NB) {
      float pv = 0.f, qv = 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        pv = lane == j ? Pw[j] : pv;
        qv = lane == j ? Qw[j] : qv;
      }
      const int q = ti * NB + lane;
      row[AL.oLa + q] = pv - lb_[q] * qv;
      row[AL.oLb + q] = -la_[q] * qv;
    }
  } else {
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        red[wv][j] = Pw[j];
        red[wv][NB + j] = Qw[j];
      }
    }
    __syncthreads();
    if (tid < D * NB) {   // (input i, basis j): the five pairs of input i in order
      const int i = tid / NB, j = tid % NB;
      float pv = 0.f, qv = 0.f;
      for (int p = 0; p < H / 2; ++p) {
        pv += red[i * (H / 2) + p][j];
        qv += red[i * (H / 2) + p][NB + j];
      }
      const int q = i * NB + j;
      row[AL.oLa + q] = pv - lb_[q] * qv;
      row[AL.oLb + q] = -la_[q] * qv;
    }
  }
}
