// fetode_kanrnn.hip — the ETT KAN-RNN encoder (train_kan_fet_ett.py:741-818) on gfx950.
//
// KANRNNEncoder.forward (:809-818) runs FullyNonlinearKANCell (:780-795) over a 96-step context:
//   h_t = sigmoid(cat(phi_x(x_t), phi_h(h_{t-1})))[:, :H],  phi(v)[i,k] = 2 / (1 + exp(-a (v_i - b)))
// and projects z0 = to_latent(h_T).  One wave owns one batch row: lane j owns hidden column j (its
// basis parameters live in registers for the whole recurrence), h_{t-1} and x_t sit in a per-wave LDS
// slot, so the recurrence never leaves the CU; to_latent runs in the same launch with W^T in LDS.
//
// The truncated cat makes most of the recurrence dead: column j < F*nb reads x_t only, column
// j >= F*nb reads h_{t-1} through column (j - F*nb)/nb < j, so a chain of dependencies that reaches
// h_T is at most depth = max_j d(j) steps long (d(j) = 0 for j < F nb, else 1 + d((j - F nb)/nb)).
// Without a tape the forward evaluates only the last depth+1 steps (at F = 7, nb = 10, H = 64:
// depth 0, i.e. the last step); the value is the reference's exactly, NaN / inf included, because
// nothing outside the cone can reach h_T.  With a tape (autograd) every step is evaluated.
//
// The backward reproduces the reference autograd's IEEE behaviour (tests/golden/ett_kanrnn_*.npz):
// the columns the cat drops (and live columns with a zero adjoint) get a zero gradient, which the
// exp backward multiplies by exp(z) — NaN when exp(z) is inf or NaN.  Dropped columns therefore only
// need z = -a (v - b) and one compare (z NaN or exp(z) overflowing); their NaN reaches the basis
// parameters and the input the column reads, and through h_{t-1} the earlier steps.
#include "fetode_common.h"

namespace fetode {
namespace {

constexpr int kWaves = 4;         // waves (rows in flight) per workgroup
constexpr int kMaxH = 256;        // hidden columns (4 per lane)
constexpr int kMaxF = 64;         // input features
constexpr int kMaxQ = 2048;       // combined basis columns (F + H) * nb, 32 per lane
constexpr int kMaxW = 16384;      // (latent + 1) * H floats of W^T in LDS (64 KiB)
constexpr int kBwdWaves = 4096;   // waves of the backward (rows are strided over them)
constexpr int kFwdGroups = 1024;  // forward workgroups (4 waves each)
constexpr int kRedChunks = 32;    // first-pass chunks of the fixed-order partial reduction
// expf(z) is finite iff z <= 88.72283172607421875f (the next float, 0x42B17218, overflows)
constexpr float kExpFinite = 88.72283172607421875f;

__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct RnnArgs {
  int F, H, nb, latent, Fnb, Q;
  const float *ax, *bx, *ah, *bh, *w, *bias;
  const float* x;
  int64_t B;
  int T, t_first;
  const float* h0;
  float *hout, *z0, *tape;
};

// the reference basis column phi = reciprocal(1 + exp(-a (v - b))) * 2 in torch's op order
// (`2 / t` is Tensor.__rtruediv__ = reciprocal(t) * 2), and the cell's sigmoid of it
__device__ __forceinline__ void basis_col(float v, float na, float b, float& e, float& r, float& d1) {
  d1 = v - b;
  const float z = na * d1;
  e = expf(z);
  r = 1.0f / (1.0f + e);
}
__device__ __forceinline__ float cell_col(float v, float na, float b, float& e, float& r, float& d1) {
  basis_col(v, na, b, e, r, d1);
  const float phi = r * 2.0f;
  return 1.0f / (1.0f + expf(-phi));
}

__device__ __forceinline__ void col_params(const RnnArgs& a, int c, float& na, float& b, int& src, bool& isx) {
  if (c < a.Fnb) {
    na = -a.ax[c];
    b = a.bx[c];
    src = c / a.nb;
    isx = true;
  } else {
    const int q = c - a.Fnb;
    na = -a.ah[q];
    b = a.bh[q];
    src = q / a.nb;
    isx = false;
  }
}

template <int MC>
__global__ __launch_bounds__(256) void kanrnn_fwd_kernel(RnnArgs a) {
  // W^T (H, latent) when projecting, rows at a pitch of latent + 1: the staging writes of 32
  // consecutive j (one row each) land on 32 banks instead of one (37 % of the kernel's LDS cycles
  // were conflicts at pitch latent = 64, profiles/r06_lds_enc.txt)
  extern __shared__ float s_w[];
  __shared__ float s_x[kWaves][kMaxF];
  __shared__ float s_h[kWaves][2][kMaxH];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool proj = a.z0 != nullptr;
  if (proj) {
    for (int e = threadIdx.x; e < a.latent * a.H; e += blockDim.x) {
      const int o = e / a.H, j = e - o * a.H;
      s_w[j * (a.latent + 1) + o] = a.w[e];
    }
    __syncthreads();
  }
  float na[MC], bb[MC];
  int src[MC];
  bool isx[MC];
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    const int c = lane + 64 * m;
    na[m] = 0.f, bb[m] = 0.f, src[m] = 0, isx[m] = true;
    if (c < a.H) col_params(a, c, na[m], bb[m], src[m], isx[m]);
  }
  for (int64_t row = (int64_t)blockIdx.x * kWaves + wv; row < a.B; row += (int64_t)gridDim.x * kWaves) {
  // h_{t_first - 1}: h0 when the cone reaches the start, else anything (no chain reads it)
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    const int c = lane + 64 * m;
    if (c < a.H) s_h[wv][0][c] = (a.t_first == 0 && a.h0) ? a.h0[row * a.H + c] : 0.0f;
  }
  int cur = 0;
  const float* xr = a.x + row * (int64_t)a.T * a.F;
  float xn = (lane < a.F && a.t_first < a.T) ? xr[(int64_t)a.t_first * a.F + lane] : 0.0f;
  for (int t = a.t_first; t < a.T; ++t) {
    if (lane < a.F) s_x[wv][lane] = xn;
    if (t + 1 < a.T && lane < a.F) xn = xr[(int64_t)(t + 1) * a.F + lane];   // prefetch x_{t+1}
    wsync();
#pragma unroll
    for (int m = 0; m < MC; ++m) {
      const int c = lane + 64 * m;
      if (c < a.H) {
        const float v = isx[m] ? s_x[wv][src[m]] : s_h[wv][cur][src[m]];
        float e, r, d1;
        const float s = cell_col(v, na[m], bb[m], e, r, d1);
        s_h[wv][cur ^ 1][c] = s;
        if (a.tape) a.tape[(row * a.T + t) * a.H + c] = s;
      }
    }
    wsync();
    cur ^= 1;
  }
  const float* h = s_h[wv][cur];
  if (a.hout) {
#pragma unroll
    for (int m = 0; m < MC; ++m) {
      const int c = lane + 64 * m;
      if (c < a.H) a.hout[row * a.H + c] = h[c];
    }
  }
  if (proj) {
    for (int o = lane; o < a.latent; o += 64) {
      float acc = 0.0f;
      for (int j = 0; j < a.H; ++j) acc = __builtin_fmaf(h[j], s_w[j * (a.latent + 1) + o], acc);
      a.z0[row * a.latent + o] = acc + a.bias[o];
    }
  }
  wsync();   // the next row overwrites this wave's LDS slots
  }
}

struct BwdArgs {
  RnnArgs f;
  const float* g_h;   // (B, H)
  float* g_x;         // (B, T, F)
  float* g_h0;        // (B, H)
  float* part;        // (n_waves, 2 Q)
  int n_waves;
};

template <int MQ, int MCL>   // MQ column slots per lane (Q <= 64 MQ), MCL of them can be live (H <= 64 MCL)
__global__ __launch_bounds__(256) void kanrnn_bwd_kernel(BwdArgs A) {
  const RnnArgs& a = A.f;
  constexpr int kIn = kMaxF + kMaxH;              // staged inputs: x_t at [0, F), h_{t-1} at [kMaxF, kMaxF + H)
  __shared__ float s_in[kWaves][kIn];
  __shared__ float s_cg[kWaves][kMaxH + 16];      // d loss / d (v - b) of the live columns (+ read padding)
  __shared__ float s_gn[kWaves][kMaxH];           // d loss / d h_{t-1}
  __shared__ int s_bad[kWaves][kIn];              // a dropped column reading this input gave NaN
  __shared__ float s_thr[kIn];                    // per input slot: |v| below it keeps every dropped column finite
  extern __shared__ float4 s_par[];               // per combined column {-a, b, input slot, 0}
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * kWaves + wv;
  for (int c = threadIdx.x; c < a.Q; c += blockDim.x) {
    float na, b;
    int src;
    bool isx;
    col_params(a, c, na, b, src, isx);
    s_par[c] = make_float4(na, b, __int_as_float(isx ? src : kMaxF + src), 0.0f);
  }
  // The dropped columns (c >= H) only ever contribute a NaN, when exp(na (v - b)) overflows.  With
  // |na (v - b)| <= |na| (|v| + |b|) (1 + 2 eps), |v| < kExpFinite / |na| (1 - 1e-5) - |b| (1 + 1e-5)
  // keeps every dropped column of the input finite: a step whose staged inputs all pass skips their
  // checks (bitwise the same sums: they add nothing then).  A NaN bound (an infinite b) is -inf.
  const int NU = a.F + a.H;   // inputs: x_t (F) and h_{t-1} (H)
  for (int u = threadIdx.x; u < NU; u += blockDim.x) {
    const bool ux = u < a.F;
    const int c0 = ux ? u * a.nb : a.Fnb + (u - a.F) * a.nb;
    float T = __builtin_inff();
    for (int c = c0; c < c0 + a.nb; ++c) {
      if (c < a.H || c >= a.Q) continue;   // live, or no column
      float na, b;
      int src;
      bool isx;
      col_params(a, c, na, b, src, isx);
      const float t = kExpFinite / fabsf(na) * (1.0f - 1e-5f) - fabsf(b) * (1.0f + 1e-5f);
      T = (t != t) ? -__builtin_inff() : (t < T ? t : T);
    }
    s_thr[ux ? u : kMaxF + u - a.F] = T;
  }
  __syncthreads();
  const float thr_x = lane < a.F ? s_thr[lane] : __builtin_inff();
  float thr_h[MCL];
#pragma unroll
  for (int m = 0; m < MCL; ++m) {
    const int c = lane + 64 * m;
    thr_h[m] = c < a.H ? s_thr[kMaxF + c] : __builtin_inff();
  }
  float ga[MQ], gb[MQ];
#pragma unroll
  for (int m = 0; m < MQ; ++m) ga[m] = 0.f, gb[m] = 0.f;
  bool bad_dirty = true;   // s_bad may hold flags (a step that checked its dropped columns, or LDS garbage)
  for (int64_t row = gw; row < a.B; row += A.n_waves) {
    const float* xr = a.x + row * (int64_t)a.T * a.F;
    const float* tr = A.f.tape + row * (int64_t)a.T * a.H;
    float g[MCL], sv[MCL], hp[MCL];
#pragma unroll
    for (int m = 0; m < MCL; ++m) {
      const int c = lane + 64 * m;
      g[m] = (c < a.H) ? A.g_h[row * a.H + c] : 0.0f;
      sv[m] = (c < a.H) ? tr[(int64_t)(a.T - 1) * a.H + c] : 0.0f;
    }
    auto load_hp = [&](int t, float* dst) {   // h_{t-1} for step t
#pragma unroll
      for (int m = 0; m < MCL; ++m) {
        const int c = lane + 64 * m;
        float v = 0.0f;
        if (c < a.H) v = t > 0 ? tr[(int64_t)(t - 1) * a.H + c] : (a.h0 ? a.h0[row * a.H + c] : 0.0f);
        dst[m] = v;
      }
    };
    load_hp(a.T - 1, hp);
    float xv = lane < a.F ? xr[(int64_t)(a.T - 1) * a.F + lane] : 0.0f;
    for (int t = a.T - 1; t >= 0; --t) {
      // stage x_t and h_{t-1}; prefetch step t-1's
#pragma unroll
      for (int m = 0; m < MCL; ++m) {
        const int c = lane + 64 * m;
        if (c < a.H) s_in[wv][kMaxF + c] = hp[m];
      }
      if (lane < a.F) s_in[wv][lane] = xv;
      if (bad_dirty)
        for (int u = lane; u < NU; u += 64) s_bad[wv][u < a.F ? u : kMaxF + u - a.F] = 0;
      float hpn[MCL], xn = 0.0f;
      if (t > 0) {
        load_hp(t - 1, hpn);
        if (lane < a.F) xn = xr[(int64_t)(t - 1) * a.F + lane];
      }
      // every staged input inside its dropped columns' finite range: the step skips their checks
      bool risky = lane < a.F && !(fabsf(xv) < thr_x);
#pragma unroll
      for (int m = 0; m < MCL; ++m) risky |= !(fabsf(hp[m]) < thr_h[m]);
      const bool check_dropped = __builtin_amdgcn_ballot_w64(risky) != 0;
      bad_dirty = check_dropped;   // only a checking step writes flags
      wsync();
#pragma unroll
      for (int m = 0; m < MQ; ++m) {
        const int c = lane + 64 * m;
        if (c >= a.Q) continue;
        const bool live = m < MCL && c < a.H;
        if (!live && !check_dropped) continue;
        const float4 pc = s_par[c];
        const int u = __float_as_int(pc.z);
        const float v = s_in[wv][u];
        if (live) {
          // live column: torch's autograd of sigmoid(reciprocal(1 + exp(na * (v - b))) * 2)
          float e, r, d1;
          basis_col(v, pc.x, pc.y, e, r, d1);
          const float sg = sv[m < MCL ? m : 0];
          const float gphi = g[m < MCL ? m : 0] * (1.0f - sg) * sg;   // sigmoid_backward
          const float gr = gphi * 2.0f;
          const float gden = -gr * (r * r);                            // reciprocal backward
          const float gz = gden * e;                                   // exp backward
          const float gna = gz * d1, gd1 = gz * pc.x;
          ga[m] += -gna;                                               // neg backward
          gb[m] += -gd1;                                               // sub backward (other)
          s_cg[wv][c] = gd1;
        } else {
          // dropped column: zero gradient; NaN iff exp(z) is not finite
          const float z = pc.x * (v - pc.y);
          if (!(z <= kExpFinite)) {
            const float qnan = __builtin_nanf("");
            ga[m] += qnan;
            gb[m] += qnan;
            s_bad[wv][u] = 1;
          }
        }
      }
      wsync();
      // d loss / d v per input: its live columns in k order (+ NaN from a dropped one); the reads
      // of one input are independent (unrolled), so the sum waits for one LDS round trip
      for (int u = lane; u < NU; u += 64) {
        const bool ux = u < a.F;
        const int i = ux ? u : u - a.F;
        const int c0 = ux ? i * a.nb : a.Fnb + i * a.nb;   // first column reading input u
        const int live = a.H - c0;
        const int cnt = live < 0 ? 0 : live < a.nb ? live : a.nb;
        float sum = 0.0f;
        if (cnt > 0) {
          if (a.nb <= 16) {
            float vals[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) vals[k] = s_cg[wv][c0 + k];
#pragma unroll
            for (int k = 0; k < 16; ++k)
              if (k < cnt) sum += vals[k];
          } else {
            for (int k = 0; k < cnt; ++k) sum += s_cg[wv][c0 + k];
          }
        }
        if (check_dropped && s_bad[wv][ux ? u : kMaxF + i]) sum += __builtin_nanf("");
        if (ux) {
          if (A.g_x) A.g_x[(row * a.T + t) * a.F + i] = sum;
        } else {
          s_gn[wv][i] = sum;
        }
      }
      wsync();
      if (t == 0) {
        if (A.g_h0)
          for (int i = lane; i < a.H; i += 64) A.g_h0[row * a.H + i] = s_gn[wv][i];
        break;
      }
#pragma unroll
      for (int m = 0; m < MCL; ++m) {
        const int c = lane + 64 * m;
        if (c < a.H) {
          g[m] = s_gn[wv][c];
          sv[m] = hp[m];   // h_{t-1} is the output of step t-1
          hp[m] = hpn[m];
        }
      }
      xv = xn;
      wsync();
    }
  }
  if (gw < A.n_waves) {
    float* p = A.part + (int64_t)gw * 2 * a.Q;
#pragma unroll
    for (int m = 0; m < MQ; ++m) {
      const int c = lane + 64 * m;
      if (c < a.Q) {
        p[c] = ga[m];
        p[a.Q + c] = gb[m];
      }
    }
  }
}

// fixed-order column sums of a (nrows, ncols) fp32 matrix: chunk sums in fp64, then the chunks in order
__global__ void colsum_pass1(const float* __restrict__ rows, int64_t nrows, int ncols, int64_t per, double* tmp) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= ncols) return;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = r0 + per < nrows ? r0 + per : nrows;
  double s = 0.0;
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    const float v0 = rows[r * ncols + col], v1 = rows[(r + 1) * ncols + col];
    const float v2 = rows[(r + 2) * ncols + col], v3 = rows[(r + 3) * ncols + col];
    s += (double)v0;
    s += (double)v1;
    s += (double)v2;
    s += (double)v3;
  }
  for (; r < r1; ++r) s += (double)rows[r * ncols + col];
  tmp[(int64_t)blockIdx.y * ncols + col] = s;
}

struct Segs {
  int begin[4];
  float* ptr[4];
};

__global__ void colsum_pass2(const double* __restrict__ tmp, int nch, int ncols, Segs segs) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= ncols) return;
  double s = 0.0;
  for (int c = 0; c < nch; ++c) s += tmp[(int64_t)c * ncols + col];
  int g = 0;
  while (g < 3 && segs.ptr[g + 1] != nullptr && col >= segs.begin[g + 1]) ++g;
  if (segs.ptr[g]) segs.ptr[g][col - segs.begin[g]] = (float)s;
}

int colsum(const float* rows, int64_t nrows, int ncols, double* tmp, const Segs& segs, hipStream_t s) {
  const int nch = nrows < kRedChunks ? (int)(nrows > 0 ? nrows : 1) : kRedChunks;
  const int64_t per = (nrows + nch - 1) / nch;
  hipLaunchKernelGGL(colsum_pass1, dim3((unsigned)nblk(ncols, 256), (unsigned)nch), dim3(256), 0, s, rows, nrows,
                     ncols, per > 0 ? per : 1, tmp);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_pass2, dim3((unsigned)nblk(ncols, 256)), dim3(256), 0, s, tmp, nch, ncols, segs);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int depth_of(int F, int H, int nb) {
  const int Fnb = F * nb;
  int D = 0;
  for (int j = 0; j < H; ++j) {
    int d = 0;
    for (int c = j; c >= Fnb; c = (c - Fnb) / nb) ++d;
    D = d > D ? d : D;
  }
  return D;
}

int check_rnn(const fetode_kanrnn_t* m) {
  if (!m) return set_err(FETODE_EINVAL, "kanrnn: null descriptor");
  if (m->num_features < 1 || m->num_features > kMaxF || m->hidden < 1 || m->hidden > kMaxH || m->num_basis < 1)
    return set_err(FETODE_EUNSUPPORTED, "kanrnn: F=%d H=%d nb=%d (supported F <= %d, H <= %d)", m->num_features,
                   m->hidden, m->num_basis, kMaxF, kMaxH);
  if ((int64_t)(m->num_features + m->hidden) * m->num_basis > kMaxQ)
    return set_err(FETODE_EUNSUPPORTED, "kanrnn: (F + H) * nb = %d > %d", (m->num_features + m->hidden) * m->num_basis,
                   kMaxQ);
  if (!m->ax || !m->bx || !m->ah || !m->bh) return set_err(FETODE_EINVAL, "kanrnn: null basis parameter");
  if (m->latent < 0) return set_err(FETODE_EINVAL, "kanrnn: latent < 0");
  return FETODE_OK;
}

RnnArgs rnn_args(const fetode_kanrnn_t* m) {
  RnnArgs a{};
  a.F = m->num_features, a.H = m->hidden, a.nb = m->num_basis, a.latent = m->latent;
  a.Fnb = a.F * a.nb, a.Q = (a.F + a.H) * a.nb;
  a.ax = m->ax, a.bx = m->bx, a.ah = m->ah, a.bh = m->bh, a.w = m->w, a.bias = m->bias;
  return a;
}

template <int MQ>
void launch_bwd(const BwdArgs& A, int grid, hipStream_t s) {
  const size_t lds = sizeof(float4) * A.f.Q;
  if (A.f.H <= 64)
    hipLaunchKernelGGL((kanrnn_bwd_kernel<MQ, 1>), dim3((unsigned)grid), dim3(64 * kWaves), lds, s, A);
  else if constexpr (MQ >= 4)
    hipLaunchKernelGGL((kanrnn_bwd_kernel<MQ, 4>), dim3((unsigned)grid), dim3(64 * kWaves), lds, s, A);
}

}  // namespace
}  // namespace fetode

using namespace fetode;

extern "C" {

int32_t fetode_kanrnn_depth(int32_t F, int32_t H, int32_t nb) {
  if (F < 1 || H < 1 || nb < 1) return -1;
  return depth_of(F, H, nb);
}

int fetode_kanrnn_forward(const fetode_kanrnn_t* m, const float* x, int64_t B, int32_t T, const float* h0,
                          float* h_out, float* z0, float* tape, int32_t full, void* stream) {
  if (int rc = check_rnn(m)) return rc;
  if (B < 0 || T < 0) return set_err(FETODE_EINVAL, "kanrnn: B=%lld T=%d", (long long)B, T);
  if (B == 0) return FETODE_OK;
  if (T > 0 && !x) return set_err(FETODE_EINVAL, "kanrnn: null x");
  if (T == 0) return set_err(FETODE_EINVAL, "kanrnn: T = 0 (h_T = h0; nothing to run)");
  if (z0 && (m->latent < 1 || !m->w || !m->bias)) return set_err(FETODE_EINVAL, "kanrnn: z0 needs latent, w, bias");
  if (z0 && (int64_t)(m->latent + 1) * m->hidden > kMaxW)
    return set_err(FETODE_EUNSUPPORTED, "kanrnn: (latent + 1) * H = %d > %d (project outside)",
                   (m->latent + 1) * m->hidden, kMaxW);
  if (z0 && m->latent > 256) return set_err(FETODE_EUNSUPPORTED, "kanrnn: latent > 256");
  if (B > (int64_t)0x7fffffff * kWaves) return set_err(FETODE_EINVAL, "kanrnn: batch too large");
  RnnArgs a = rnn_args(m);
  a.x = x, a.B = B, a.T = T, a.h0 = h0, a.hout = h_out, a.z0 = z0, a.tape = tape;
  const int D = depth_of(a.F, a.H, a.nb);
  a.t_first = (full || tape || T - 1 - D <= 0) ? 0 : T - 1 - D;
  // enough workgroups to fill the chip; rows are strided over the waves (W^T is staged once per workgroup)
  const int64_t nwg = (B + kWaves - 1) / kWaves;
  const unsigned grid = (unsigned)(nwg < kFwdGroups ? nwg : kFwdGroups);
  const size_t lds = z0 ? sizeof(float) * (size_t)(m->latent + 1) * m->hidden : 0;
  hipStream_t s = (hipStream_t)stream;
  if (a.H <= 64)
    hipLaunchKernelGGL(kanrnn_fwd_kernel<1>, dim3(grid), dim3(64 * kWaves), lds, s, a);
  else if (a.H <= 128)
    hipLaunchKernelGGL(kanrnn_fwd_kernel<2>, dim3(grid), dim3(64 * kWaves), lds, s, a);
  else
    hipLaunchKernelGGL(kanrnn_fwd_kernel<4>, dim3(grid), dim3(64 * kWaves), lds, s, a);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_kanrnn_backward_workspace(const fetode_kanrnn_t* m, int64_t B) {
  if (check_rnn(m)) return -1;
  const int64_t Q = (int64_t)(m->num_features + m->hidden) * m->num_basis;
  const int64_t nw = B < kBwdWaves ? (B > 0 ? B : 1) : kBwdWaves;
  const int64_t nwr = (nw + kWaves - 1) / kWaves * kWaves;
  return (int64_t)sizeof(float) * nwr * 2 * Q + (int64_t)sizeof(double) * kRedChunks * 2 * Q + 256;
}

int fetode_kanrnn_backward(const fetode_kanrnn_t* m, const float* x, int64_t B, int32_t T, const float* h0,
                           const float* tape, const float* g_h, float* g_x, float* g_h0, float* g_ax, float* g_bx,
                           float* g_ah, float* g_bh, void* workspace, void* stream) {
  if (int rc = check_rnn(m)) return rc;
  if (B <= 0 || T <= 0) return B == 0 ? FETODE_OK : set_err(FETODE_EINVAL, "kanrnn backward: B=%lld T=%d", (long long)B, T);
  if (!x || !tape || !g_h || !workspace) return set_err(FETODE_EINVAL, "kanrnn backward: null pointer");
  BwdArgs A{};
  A.f = rnn_args(m);
  A.f.x = x, A.f.B = B, A.f.T = T, A.f.h0 = h0, A.f.tape = const_cast<float*>(tape);
  A.g_h = g_h, A.g_x = g_x, A.g_h0 = g_h0;
  const int64_t nw = B < kBwdWaves ? B : kBwdWaves;
  const int grid = (int)((nw + kWaves - 1) / kWaves);
  A.n_waves = grid * kWaves;
  A.part = (float*)workspace;
  const int Q = A.f.Q;
  double* tmp = (double*)(((uintptr_t)(A.part + (int64_t)A.n_waves * 2 * Q) + 15) & ~(uintptr_t)15);
  hipStream_t s = (hipStream_t)stream;
  const int mq = (Q + 63) / 64;
  if (mq <= 2 && A.f.H <= 64) launch_bwd<2>(A, grid, s);
  else if (mq <= 4) launch_bwd<4>(A, grid, s);
  else if (mq <= 8) launch_bwd<8>(A, grid, s);
  else if (mq <= 12) launch_bwd<12>(A, grid, s);
  else if (mq <= 16) launch_bwd<16>(A, grid, s);
  else if (mq <= 24) launch_bwd<24>(A, grid, s);
  else launch_bwd<32>(A, grid, s);
  LAUNCH_CHECK();
  // parameter gradients: partial columns [ga (Q) | gb (Q)], combined column c -> ax (c < F nb) / ah
  Segs segs{};
  segs.begin[0] = 0, segs.ptr[0] = g_ax;
  segs.begin[1] = A.f.Fnb, segs.ptr[1] = g_ah;
  segs.begin[2] = Q, segs.ptr[2] = g_bx;
  segs.begin[3] = Q + A.f.Fnb, segs.ptr[3] = g_bh;
  if (!g_ax && !g_ah && !g_bx && !g_bh) return FETODE_OK;
  if (!g_ax || !g_ah || !g_bx || !g_bh)
    return set_err(FETODE_EINVAL, "kanrnn backward: the four parameter gradients come together");
  return colsum(A.part, A.n_waves, 2 * Q, tmp, segs, s);
}

// ---------------------------------------------------------------------------------------------
// LogisticBasis alone (train_kan_fet_ett.py:741-749): phi (B, in, nb)
// ---------------------------------------------------------------------------------------------

}  // extern "C"

namespace fetode {
namespace {

__global__ void lbasis_fwd_kernel(const float* __restrict__ x, int64_t n, int in, int nb, const float* __restrict__ A,
                                  const float* __restrict__ Bp, float* __restrict__ phi) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int q = (int)(e % ((int64_t)in * nb));
  const int64_t b = e / ((int64_t)in * nb);
  const float v = x[b * in + q / nb];
  float ee, r, d1;
  d1 = v - Bp[q];
  ee = expf(-A[q] * d1);
  r = 1.0f / (1.0f + ee);
  phi[e] = r * 2.0f;
}

// per (b, i): g_x = sum_k g_d1 (k order); per-element parameter contributions into rows (B, 2 in nb)
__global__ void lbasis_bwd_kernel(const float* __restrict__ x, int64_t B, int in, int nb, const float* __restrict__ A,
                                  const float* __restrict__ Bp, const float* __restrict__ g, float* __restrict__ gx,
                                  float* __restrict__ rows) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * in) return;
  const int i = (int)(e % in);
  const int64_t b = e / in;
  const float v = x[e];
  float sum = 0.0f;
  const int Q = in * nb;
  for (int k = 0; k < nb; ++k) {
    const int q = i * nb + k;
    const float na = -A[q];
    const float d1 = v - Bp[q];
    const float ee = expf(na * d1);
    const float r = 1.0f / (1.0f + ee);
    const float gr = g[b * Q + q] * 2.0f;
    const float gz = (-gr * (r * r)) * ee;
    const float gna = gz * d1, gd1 = gz * na;
    sum += gd1;
    if (rows) {
      rows[b * 2 * Q + q] = -gna;
      rows[b * 2 * Q + Q + q] = -gd1;
    }
  }
  if (gx) gx[e] = sum;
}

}  // namespace
}  // namespace fetode

extern "C" {

int fetode_logistic_basis_forward(const float* x, int64_t B, int32_t in, int32_t nb, const float* a, const float* b,
                                  float* phi, void* stream) {
  if (B < 0 || in < 1 || nb < 1) return set_err(FETODE_EINVAL, "logistic basis: B=%lld in=%d nb=%d", (long long)B, in, nb);
  if (B == 0) return FETODE_OK;
  if (!x || !a || !b || !phi) return set_err(FETODE_EINVAL, "logistic basis: null pointer");
  const int64_t n = B * in * nb;
  hipLaunchKernelGGL(lbasis_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n, in,
                     nb, a, b, phi);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_logistic_basis_backward_workspace(int32_t in, int32_t nb, int64_t B) {
  if (in < 1 || nb < 1 || B < 0) return -1;
  const int64_t Q = (int64_t)in * nb;
  return (int64_t)sizeof(float) * (B > 0 ? B : 1) * 2 * Q + (int64_t)sizeof(double) * kRedChunks * 2 * Q + 256;
}

int fetode_logistic_basis_backward(const float* x, int64_t B, int32_t in, int32_t nb, const float* a, const float* b,
                                   const float* g_phi, float* g_x, float* g_a, float* g_b, void* workspace,
                                   void* stream) {
  if (B < 0 || in < 1 || nb < 1) return set_err(FETODE_EINVAL, "logistic basis backward: bad shape");
  if (B == 0) return FETODE_OK;
  if (!x || !a || !b || !g_phi) return set_err(FETODE_EINVAL, "logistic basis backward: null pointer");
  const bool params = g_a || g_b;
  if (params && !workspace) return set_err(FETODE_EINVAL, "logistic basis backward: null workspace");
  const int Q = in * nb;
  float* rows = params ? (float*)workspace : nullptr;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(lbasis_bwd_kernel, dim3((unsigned)((B * in + 255) / 256)), dim3(256), 0, s, x, B, in, nb, a, b,
                     g_phi, g_x, rows);
  LAUNCH_CHECK();
  if (!params) return FETODE_OK;
  double* tmp = (double*)(((uintptr_t)(rows + B * 2 * Q) + 15) & ~(uintptr_t)15);
  Segs segs{};
  segs.begin[0] = 0, segs.ptr[0] = g_a;
  segs.begin[1] = Q, segs.ptr[1] = g_b;
  if (!g_a || !g_b) return set_err(FETODE_EINVAL, "logistic basis backward: g_a and g_b come together");
  return colsum(rows, B, 2 * Q, tmp, segs, s);
}

}  // extern "C"
