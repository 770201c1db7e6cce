// fetode_ecg.hip — the ECG KAN-FET NODE vector field (BASELINE configs[2]):
// KANFeatureMixer(hysteretic LogisticBasis, Sigmoid) followed by a Linear head —
// No_MLP_KANODEFunc, train_ecg_kan_fet_nn_ode.py:483-509, LogisticBasis :54-133.
//
// Forward, one launch per evaluation: a workgroup owns kRows batch rows; its threads evaluate the
// (row, input, basis) features into LDS in the reference's op order (IEEE division, expf), then
// one thread per (row, output) forms the dot product with the head in a fixed order.  The
// hysteresis memory is the LAST row of the batch (:131-132): it is read by every workgroup and
// replaced by a second, one-block launch on the same stream, so no workgroup can see a
// half-updated state.
//
// Backward: the head's input gradient (phi-space), the basis VJP per (row, input) over its bases,
// and the parameter gradients reduced over the batch by one thread per parameter in a fixed order
// (no atomics, run-to-run identical).  branch_state is a comparison: no gradient flows through it,
// nor through the detached prev_x (:119-132).
#include <algorithm>
#include <cstring>

#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kRows = 4;      // batch rows per forward workgroup
constexpr int kThreads = 256;

struct HL {  // device copy of fetode_hlogistic_t
  int in, nb;
  const float *k, *Ec, *Ps, *bias;
  float gs, bp;
};

__device__ __forceinline__ float ref_sigmoid(float z) { return 1.0f / (1.0f + expf(-z)); }

// The head's fp32 summation order, shared by every kernel that evaluates it: q in [0, F) splits
// into kHeadParts = 32 consecutive parts of head_part(F) (a multiple of 4) indices; each part P_p
// is an FMA chain from 0 in increasing q; groups of four add as S_w = (P_4w + P_4w+1) +
// (P_4w+2 + P_4w+3), and the eight S_w add left to right.  (The resident dopri5 gives each wave
// one group, a quarter-wave per part, and combines a group with two lane shuffles.)
constexpr int kHeadParts = 32;
constexpr int kHeadGroups = kHeadParts / 4;
__host__ __device__ __forceinline__ int head_part(int F) { return (((F + 3) & ~3) + 4 * kHeadParts - 1) / (4 * kHeadParts) * 4; }

// the reference's up / down / gate for element (i, j) at input x (train_ecg_kan_fet_nn_ode.py:110-121)
struct HPoint {
  float su, sd, bs, basis;
};
__device__ __forceinline__ HPoint hpoint(const HL& L, float x, float pv, int q) {
  HPoint p;
  const float k = L.k[q], Ec = L.Ec[q], Ps = L.Ps[q];
  p.su = 1.0f / (1.0f + expf(-k * (x - Ec)));
  p.sd = 1.0f / (1.0f + expf(-k * (x + Ec)));
  const float up = Ps * p.su * 2.0f - Ps;
  const float down = Ps * p.sd * 2.0f - Ps;
  const float g = ref_sigmoid(L.gs * (x - pv));
  p.bs = g > L.bp ? 1.0f : 0.0f;
  p.basis = p.bs * up + (1.0f - p.bs) * down + L.bias[q];
  return p;
}

__global__ __launch_bounds__(kThreads) void mixer_fwd_kernel(HL L, const float* __restrict__ x, int64_t B,
                                                            const float* __restrict__ prev, int act_sigmoid,
                                                            const float* __restrict__ w, const float* __restrict__ bvec,
                                                            int n_out, float* __restrict__ phi_out,
                                                            float* __restrict__ out, float* __restrict__ branch) {
  extern __shared__ float s_phi[];  // kRows * in * nb
  const int F = L.in * L.nb;
  const int64_t b0 = (int64_t)blockIdx.x * kRows;
  const int rows = (int)(B - b0 < kRows ? B - b0 : kRows);
  for (int t = threadIdx.x; t < rows * F; t += blockDim.x) {
    const int r = t / F, q = t % F, i = q / L.nb;
    const int64_t b = b0 + r;
    const HPoint p = hpoint(L, x[b * L.in + i], prev[q], q);
    const float v = act_sigmoid ? ref_sigmoid(p.basis) : p.basis;
    s_phi[t] = v;
    if (phi_out) phi_out[b * F + q] = v;
    if (branch) branch[b * F + q] = p.bs;
  }
  if (!w) return;
  __syncthreads();
  for (int t = threadIdx.x; t < rows * n_out; t += blockDim.x) {
    const int r = t / n_out, o = t % n_out;
    const float* wr = w + (int64_t)o * F;
    const float* ph = s_phi + r * F;
    const int PS = head_part(F);
    float tot = 0.f;
    for (int w = 0; w < kHeadGroups; ++w) {
      float P[4];
      for (int c = 0; c < 4; ++c) {
        const int p = 4 * w + c;
        float acc = 0.f;
        const int q1 = min(F, (p + 1) * PS);
        for (int q = p * PS; q < q1; ++q) acc = __builtin_fmaf(ph[q], wr[q], acc);
        P[c] = acc;
      }
      const float S = (P[0] + P[1]) + (P[2] + P[3]);
      tot = w == 0 ? S : tot + S;
    }
    out[(b0 + r) * n_out + o] = tot + (bvec ? bvec[o] : 0.f);
  }
}

// prev_x.copy_(x_exp[-1:]) (:131-132): every basis of input i remembers x[B-1, i]
__global__ void mixer_state_kernel(const float* __restrict__ x, int64_t B, int in, int nb, float* __restrict__ prev) {
  for (int q = threadIdx.x; q < in * nb; q += blockDim.x) prev[q] = x[(B - 1) * in + q / nb];
}

// g_phi[b, q] = sum_o g[b, o] w[o, q]   (the head's input gradient)
__global__ void head_gin_kernel(const float* __restrict__ g, const float* __restrict__ w, int64_t B, int n_out, int F,
                                float* __restrict__ gphi) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * F) return;
  const int64_t b = t / F;
  const int q = (int)(t % F);
  float acc = 0.f;
  for (int o = 0; o < n_out; ++o) acc = __builtin_fmaf(g[b * n_out + o], w[(int64_t)o * F + q], acc);
  gphi[t] = acc;
}

// d loss / d w[o, q] = sum_b g[b, o] phi[b, q];  d loss / d bias[o] = sum_b g[b, o]
__global__ void head_gw_kernel(const float* __restrict__ g, const float* __restrict__ phi, int64_t B, int n_out, int F,
                               float* __restrict__ gw, float* __restrict__ gb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n_out * F) {
    const int o = t / F, q = t % F;
    float acc = 0.f;
    for (int64_t b = 0; b < B; ++b) acc = __builtin_fmaf(g[b * n_out + o], phi[b * F + q], acc);
    if (gw) gw[t] = acc;
  } else if (t < n_out * F + n_out && gb) {
    const int o = t - n_out * F;
    float acc = 0.f;
    for (int64_t b = 0; b < B; ++b) acc += g[b * n_out + o];
    gb[o] = acc;
  }
}

// derivative pieces of element (b, i, j): d basis / d (x, k, Ec, Ps), gb = d loss / d basis
struct HGrad {
  float gb, dx, dk, dEc, dPs;
};
__device__ __forceinline__ HGrad hgrad(const HL& L, float x, float pv, int q, float gphi, float phi, int act_sigmoid) {
  const HPoint p = hpoint(L, x, pv, q);
  HGrad r;
  r.gb = act_sigmoid ? gphi * (phi * (1.0f - phi)) : gphi;
  const float k = L.k[q], Ec = L.Ec[q], Ps = L.Ps[q];
  const float cu = p.bs * 2.0f * Ps * p.su * (1.0f - p.su);          // d up / d z_up    (z = k (x - Ec))
  const float cd = (1.0f - p.bs) * 2.0f * Ps * p.sd * (1.0f - p.sd);  // d down / d z_down (z = k (x + Ec))
  r.dx = (cu + cd) * k;
  r.dk = cu * (x - Ec) + cd * (x + Ec);
  r.dEc = (cd - cu) * k;
  r.dPs = p.bs * (2.0f * p.su - 1.0f) + (1.0f - p.bs) * (2.0f * p.sd - 1.0f);
  return r;
}

__global__ void mixer_gx_kernel(HL L, const float* __restrict__ x, int64_t B, const float* __restrict__ prev,
                                const float* __restrict__ gphi, const float* __restrict__ phi, int act_sigmoid,
                                float* __restrict__ gx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * L.in) return;
  const int64_t b = t / L.in;
  const int i = (int)(t % L.in), F = L.in * L.nb;
  const float xv = x[t];
  float acc = 0.f;
  for (int j = 0; j < L.nb; ++j) {
    const int q = i * L.nb + j;
    const HGrad h = hgrad(L, xv, prev[q], q, gphi[b * F + q], phi[b * F + q], act_sigmoid);
    acc += h.gb * h.dx;
  }
  gx[t] = acc;
}

__global__ void mixer_gparam_kernel(HL L, const float* __restrict__ x, int64_t B, const float* __restrict__ prev,
                                    const float* __restrict__ gphi, const float* __restrict__ phi, int act_sigmoid,
                                    float* __restrict__ gk, float* __restrict__ gEc, float* __restrict__ gPs,
                                    float* __restrict__ gbias) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int F = L.in * L.nb;
  if (q >= F) return;
  const int i = q / L.nb;
  float sk = 0.f, sE = 0.f, sP = 0.f, sb = 0.f;
  for (int64_t b = 0; b < B; ++b) {
    const HGrad h = hgrad(L, x[b * L.in + i], prev[q], q, gphi[b * F + q], phi[b * F + q], act_sigmoid);
    sk = __builtin_fmaf(h.gb, h.dk, sk);
    sE = __builtin_fmaf(h.gb, h.dEc, sE);
    sP = __builtin_fmaf(h.gb, h.dPs, sP);
    sb += h.gb;
  }
  if (gk) gk[q] = sk;
  if (gEc) gEc[q] = sE;
  if (gPs) gPs[q] = sP;
  if (gbias) gbias[q] = sb;
}

int check_layer(const fetode_hlogistic_t* l) {
  if (!l || l->in_dim <= 0 || l->num_basis <= 0) return set_err(FETODE_EINVAL, "hlogistic: bad dims");
  if (!l->k || !l->Ec || !l->Ps || !l->bias) return set_err(FETODE_EINVAL, "hlogistic: null parameter");
  return FETODE_OK;
}

HL to_dev(const fetode_hlogistic_t* l) {
  HL L;
  L.in = l->in_dim;
  L.nb = l->num_basis;
  L.k = l->k;
  L.Ec = l->Ec;
  L.Ps = l->Ps;
  L.bias = l->bias;
  // gate_slope * dx with gate_slope a Python float: torch scales an fp32 tensor by it in fp32
  L.gs = (float)l->gate_slope;
  L.bp = (float)l->breaking_point;
  return L;
}

}  // namespace

extern "C" {

int fetode_hlogistic_mixer_forward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                   int32_t act_sigmoid, const float* w, const float* bias, int32_t n_out,
                                   float* phi, float* out, float* branch, float* prev_out, void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !prev || (w && (!out || n_out <= 0)) || (!w && !phi))
    return set_err(FETODE_EINVAL, "hlogistic mixer: null pointer");
  const HL L = to_dev(layer);
  const int F = L.in * L.nb;
  const size_t lds = sizeof(float) * kRows * F;
  if (lds > 64 * 1024) return set_err(FETODE_EINVAL, "hlogistic mixer: in*num_basis=%d too large", F);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mixer_fwd_kernel, dim3(nblk(B, kRows)), dim3(kThreads), lds, s, L, x, B, prev, act_sigmoid, w,
                     bias, n_out, phi, out, branch);
  LAUNCH_CHECK();
  if (prev_out) {
    hipLaunchKernelGGL(mixer_state_kernel, dim3(1), dim3(256), 0, s, x, B, L.in, L.nb, prev_out);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

int64_t fetode_hlogistic_mixer_backward_workspace(const fetode_hlogistic_t* layer, int64_t B) {
  if (check_layer(layer) || B <= 0) return -1;
  return (int64_t)sizeof(float) * B * layer->in_dim * layer->num_basis;
}

int fetode_hlogistic_mixer_backward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                    int32_t act_sigmoid, const float* phi, const float* w, int32_t n_out,
                                    const float* g, float* gx, float* gw, float* gbias_head, float* gk, float* gEc,
                                    float* gPs, float* gbias, void* workspace, void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0) return FETODE_OK;
  if (!x || !prev || !phi || !g || (w && (n_out <= 0 || !workspace)))
    return set_err(FETODE_EINVAL, "hlogistic mixer backward: null pointer");
  const HL L = to_dev(layer);
  const int F = L.in * L.nb;
  hipStream_t s = (hipStream_t)stream;
  const float* gphi = g;  // without a head, g is already d loss / d phi
  if (w) {
    float* gp = (float*)workspace;
    hipLaunchKernelGGL(head_gin_kernel, dim3(nblk(B * F, 256)), dim3(256), 0, s, g, w, B, n_out, F, gp);
    LAUNCH_CHECK();
    if (gw || gbias_head) {
      hipLaunchKernelGGL(head_gw_kernel, dim3(nblk((int64_t)n_out * F + n_out, 256)), dim3(256), 0, s, g, phi, B,
                         n_out, F, gw, gbias_head);
      LAUNCH_CHECK();
    }
    gphi = gp;
  }
  if (gx) {
    hipLaunchKernelGGL(mixer_gx_kernel, dim3(nblk(B * L.in, 256)), dim3(256), 0, s, L, x, B, prev, gphi, phi,
                       act_sigmoid, gx);
    LAUNCH_CHECK();
  }
  if (gk || gEc || gPs || gbias) {
    hipLaunchKernelGGL(mixer_gparam_kernel, dim3(nblk(F, 64)), dim3(64), 0, s, L, x, B, prev, gphi, phi,
                       act_sigmoid, gk, gEc, gPs, gbias);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

}  // extern "C"

// =============================================================================================
// Device-resident dopri5 for the ECG field: the whole torchdiffeq solve —
// f0, _select_initial_step, 6 evaluations per attempt (FSAL), the global RMS error norm,
// accept/reject, _optimal_step_size, _interp_fit / _interp_evaluate — in ONE cooperative launch,
// with the same fp32/fp64 arithmetic as the host-driven path (dopri5.py + the kernels above).
//
// A workgroup owns R-1 batch rows and, as a SHADOW row, the batch's last row: the hysteresis
// memory every evaluation reads is the last row's previous input (:131-132), so each workgroup
// evaluates that row itself and no evaluation needs data from another workgroup.  Only the
// error norms (one per attempt, three in the initial-step selection) are global: per-workgroup
// fp64 partial sums, a grid barrier, and the same fixed-order sum in every workgroup — so every
// workgroup takes the same accept/reject decisions and the same dt sequence.
//
// Everything an evaluation reads stays on chip for the whole solve.  The head weight W^T (F x D,
// 160 KB at latent 64) is split: its first QL rows sit in LDS as float4 groups [q/4][d] (all the
// LDS phi leaves), the remaining <= kTail rows in registers of the threads that own output d.
// The head is then one fp32 FMA chain over q per (row, output) — the mixer kernel's order — fed
// by ds_read_b128 instead of L2 round trips.  The feature parameters (k, Ec, Ps, bias) and the
// hysteresis memory prev_x live in registers of the thread that owns input-basis index q.
// =============================================================================================
namespace {

constexpr int kMaxF = 768;          // in * num_basis (in <= 64, num_basis <= 12)
constexpr int kLdsBytes = 163840;   // gfx950: one workgroup may declare all 160 KiB

struct DopriTab {
  float beta[6][6];  // torchdiffeq Dopri5 tableau rounded to fp32 (tableau.to(y0.dtype))
  float cerr[7];
  float cmid[7];
};

struct EcgDopriArgs {
  HL L;
  const float* wT;  // (F, D) head weight, transposed
  const float* bh;  // (D) head bias, nullable
  int D, F;
  int Fp;              // F rounded up to 4 (phi rows are zero-padded)
  int PS;              // head_part(F): q indices per head part
  int QL;              // head-weight rows per part kept in LDS (multiple of 4); the rest in registers
  const float* prev0;  // (F) prev_x before the solve
  const float* y0;     // (B, D)
  int64_t B;
  const double* t;  // (T) strictly increasing
  int T;
  float rtol, atol;
  double first_step;  // > 0: options["first_step"]; else _select_initial_step
  double safety, ifactor, dfactor, min_step, max_step;
  int max_steps;
  DopriTab tab;
  float* sol;         // (T, B, D)
  float* prev_out;    // (F)
  float* branch_out;  // (B, F) nullable: branch_state of the last evaluation
  double* part;       // (2, gridDim.x, 2) double-buffered partial sums
  unsigned* bar;      // kBarWords, zeroed: per-XCD and top arrival counters, generation
  int* stats;         // [nfev, attempts, status]
  double* att;        // (max_att, 4): t0, dt, error ratio, accepted
  int max_att;
  long long* stamps;  // debug (fetode_debug_ecg_stamps): workgroup 0's 100 MHz ticks per phase
};

// phase timer of workgroup 0 in the diagnostic build only (make stamps, tools/diag/ecg_time.py):
// other, features, head, partials, norms in 100 MHz ticks; the kernel's s_memtime total
#ifdef FETODE_STAMPS
#define STAMP(i)                                               \
  do {                                                         \
    if (stamping) {                                            \
      const long long now_ = __builtin_amdgcn_s_memrealtime(); \
      st_acc[i] += now_ - st_last;                             \
      st_last = now_;                                          \
    }                                                          \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

__device__ __forceinline__ float fast_sigmoid(float z) { return rcp(1.0f + ex2(-z * FETODE_LOG2E)); }

// Grid barrier, XCD-hierarchical (MI355X_MICROARCH.md "barrier-xcd"): workgroup i runs on XCD
// i % 8, so each XCD's workgroups arrive on their own counter (256 B apart); the last arriver of an
// XCD arrives on the top counter, the last of those bumps the generation every workgroup polls.
// The only data shared across workgroups (the partial slots) moves through agent-scope atomics,
// coherent across the XCDs' L2s by themselves, so the ordering needed is a vector-memory wait
// before arriving and after the poll — not agent-scope fences, which would also write back and
// invalidate the whole L2 (buffer_wbl2 / buffer_inv sc1) at every barrier (fetode_fused.hip
// dp_order).  Counters reset themselves; the words are zeroed once per launch.
constexpr int kBarWords = 64 * 10;  // 8 XCD counters, top counter, generation (256 B each)
// Every spin is bounded (MI355X_MICROARCH.md: a stranded workgroup must not hang the device): after
// 2^20 polls (about a second) the barrier gives up and raises the abort word 64*9+1.  Once that word
// is set every barrier returns at once (entering or spinning) and reports it: the solver then stops
// (status 4) instead of running on with counters that were never reset.
constexpr unsigned kSpinLimit = 1u << 20;
__device__ bool grid_barrier(unsigned* bar, unsigned nblk) {
  __shared__ int s_abort;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned x = blockIdx.x & 7u;
    const unsigned nx = (nblk + 7u - x) / 8u, nxcd = nblk < 8u ? nblk : 8u;
    unsigned* cnt = bar + 64 * x;
    unsigned* top = bar + 64 * 8;
    unsigned* gen = bar + 64 * 9;
    unsigned* abort_word = gen + 1;
    int ab = __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (!ab) {
      const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot stores have landed
      if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nx - 1u) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // reset lands before the release
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nxcd - 1u) {
          __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          ab = 1;
          break;
        }
        if (++spins == kSpinLimit) {
          __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ab = 1;
          break;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_abort = ab;
  }
  __syncthreads();
  return s_abort != 0;
}

// NT = 512 threads, R rows per workgroup (R-1 real + the shadow).  Solver thread (r, d) = tid for
// tid < 64 R carries state element d of row r.
// Features: the R * F (row, basis) elements of an evaluation are dealt round-robin to all threads
// (<= EPT each); their parameters sit in LDS as float4 {k, Ec, Ps, bias}.  prev_x is constant over
// the bases of one input after the first call (:131-132 expands the last row's x), so it is kept per
// input, double-buffered by evaluation parity; the first evaluation reads the module's prev_x.
// Head: wave w owns head group w = parts 4w..4w+3, a quarter-wave per part; lane l16 of a quarter
// forms the part's sums for outputs l16 + 16c (c < 4) of every row.  The part's W^T rows sit in
// LDS as [part][q/4][64] float4 (the first QL) and in registers (the rest, <= TAIL).  Two lane
// shuffles combine the four parts of a group; the solver threads add the eight groups.
constexpr int kResThreads = 512;
template <int R, int TAIL>
__global__ __launch_bounds__(kResThreads) void ecg_dopri5_kernel(EcgDopriArgs a) {
  constexpr int NT = kResThreads, NR = R - 1, EPT = (R * kMaxF + NT - 1) / NT;
  constexpr int FU = R <= 4 ? EPT : 2;  // feature-loop unroll (R = 8: registers)
  static_assert(NT / 64 == kHeadGroups, "one head group per wave");
  static_assert(R % 4 == 0, "the head runs four rows at a time");
  // dynamic LDS: W^T [kHeadParts][QL/4][64] float4 | prm [F] float4 | pv0 [Fp] | phi (R, Fp) | hs
  extern __shared__ float4 s_dyn4[];
  __shared__ float xs[R][64];
  __shared__ float pvx[2][64];
  __shared__ double red[NT / 64][2];
  __shared__ double tot[2];
  const int tid = threadIdx.x, lane = tid % 64, wv = tid / 64;
  const int r = wv, d = lane;  // solver view (rows r < R)
  const int D = a.D, F = a.F, Fp = a.Fp, PS = a.PS, QL = a.QL, G = a.QL / 4, nb = a.L.nb;
  float4* prm = s_dyn4 + (int64_t)kHeadParts * G * 64;
  float* pv0 = reinterpret_cast<float*>(prm + F);  // the module's prev_x before the solve (F)
  float* phi = pv0 + Fp;                            // (R, Fp)
  float* hs = phi + R * Fp;                          // (kHeadGroups, R, 64) group sums
  const bool solver = tid < 64 * R;
  const bool dval = solver && d < D;
  int64_t b = r < NR ? (int64_t)blockIdx.x * NR + r : a.B - 1;  // row NR: the shadow last row
  const bool real = r < NR && b < a.B && dval;
  if (b >= a.B) b = a.B - 1;  // padding rows mirror the last row; never stored or counted
  const int64_t BD = a.B * D;
  const double n_el = (double)BD;
  int phase = 0, nfev = 0, status = 0, n_att = 0;
#ifdef FETODE_STAMPS
  const bool stamping = a.stamps != nullptr && blockIdx.x == 0 && tid == 0;
  long long st_acc[5] = {0, 0, 0, 0, 0}, st_last = stamping ? __builtin_amdgcn_s_memrealtime() : 0;
  const long long st_clk0 = stamping ? __builtin_amdgcn_s_memtime() : 0, st_rt0 = st_last;
#endif

  // misc._rms_norm numerators over the WHOLE batch, two at once (per-thread fp64 terms, real
  // elements only): wave sums -> workgroup sum in wave order -> partial slot -> grid barrier ->
  // the same fixed-order sum of the slots in every workgroup
  auto global_sum2 = [&](double v0, double v1, double& s0, double& s1) {
    STAMP(0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      v0 += __shfl_xor(v0, o);
      v1 += __shfl_xor(v1, o);
    }
    if (lane == 0) {
      red[wv][0] = v0;
      red[wv][1] = v1;
    }
    __syncthreads();
    double* slot = a.part + ((int64_t)(phase & 1) * gridDim.x + blockIdx.x) * 2;
    if (tid == 0) {
      double w0 = red[0][0], w1 = red[0][1];
      for (int w = 1; w < NT / 64; ++w) {
        w0 += red[w][0];
        w1 += red[w][1];
      }
      __hip_atomic_store(&slot[0], w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&slot[1], w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (grid_barrier(a.bar, gridDim.x)) status = 4;  // aborted: every loop below checks status
    if (wv == 0) {  // one wave sums the slots: lane-strided then a fixed butterfly
      double u0 = 0.0, u1 = 0.0;
      for (int g = lane; g < (int)gridDim.x; g += 64) {
        const double* o = a.part + ((int64_t)(phase & 1) * gridDim.x + g) * 2;
        u0 += __hip_atomic_load(&o[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        u1 += __hip_atomic_load(&o[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        u0 += __shfl_xor(u0, o);
        u1 += __shfl_xor(u1, o);
      }
      if (lane == 0) {
        tot[0] = u0;
        tot[1] = u1;
      }
    }
    __syncthreads();
    s0 = tot[0];
    s1 = tot[1];
    ++phase;
    STAMP(4);
  };

  // stage the head weight and the feature parameters; zero phi's padding
  const int qtr = lane >> 4, l16 = lane & 15, part = 4 * wv + qtr;
  const int qp0 = part * PS, qend = min(F, qp0 + PS);
  for (int idx = tid; idx < kHeadParts * G * 64; idx += NT) {
    const int pg = idx / 64, dd = idx - pg * 64, pp = pg / G, g = pg - pp * G;
    const int q = pp * PS + 4 * g, qe = min(F, (pp + 1) * PS);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (dd < D) {
      v.x = q + 0 < qe ? a.wT[(int64_t)(q + 0) * D + dd] : 0.f;
      v.y = q + 1 < qe ? a.wT[(int64_t)(q + 1) * D + dd] : 0.f;
      v.z = q + 2 < qe ? a.wT[(int64_t)(q + 2) * D + dd] : 0.f;
      v.w = q + 3 < qe ? a.wT[(int64_t)(q + 3) * D + dd] : 0.f;
    }
    s_dyn4[idx] = v;
  }
  for (int q = tid; q < F; q += NT) {
    prm[q] = make_float4(a.L.k[q], a.L.Ec[q], a.L.Ps[q], a.L.bias[q]);
    pv0[q] = a.prev0[q];
  }
  for (int idx = tid; idx < R * Fp; idx += NT) phi[idx] = 0.f;
  float wt[TAIL][4];
#pragma unroll
  for (int j = 0; j < TAIL; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int q = qp0 + QL + j, dd = l16 + 16 * c;
      wt[j][c] = (dd < D && q < qend) ? a.wT[(int64_t)q * D + dd] : 0.f;
    }
  const int gcount = max(0, min(G, (qend - qp0 + 3) / 4));            // LDS groups of this part
  const int ntail = max(0, min(TAIL, ((qend - qp0 + 3) & ~3) - QL));  // register rows of this part
  const float bhd = (dval && a.bh) ? a.bh[d] : 0.f;
  // this thread's first element (row e0 / F, basis e0 % F), then every NT-th; i = q / nb by a
  // 16-bit reciprocal (exact for q < 768, nb <= 64)
  const int e_r0 = tid / F, e_q0 = tid - e_r0 * F;
  const unsigned inv_nb = (65536u + (unsigned)nb - 1u) / (unsigned)nb;
  const float gs = a.L.gs, bp = a.L.bp;
  __syncthreads();

  // one field evaluation of the solver thread's element; every thread of the workgroup takes part
  auto eval = [&](float xv) -> float {
    if (dval) xs[r][d] = xv;
    __syncthreads();
    STAMP(0);
    const int n = nfev;
    int q = e_q0, r2 = e_r0;
#pragma unroll FU
    for (int j = 0; j < EPT; ++j) {
      if (r2 < R) {  // hpoint's op order (train_ecg_kan_fet_nn_ode.py:110-121)
        const int i = (int)(((unsigned)q * inv_nb) >> 16);
        const float x = xs[r2][i];
        const float4 pr = prm[q];
        const float pq = n == 0 ? pv0[q] : pvx[n & 1][i];
        const float k = pr.x, Ec = pr.y, Ps = pr.z;
        // the smooth logistics on v_exp / v_rcp (1-ulp class); the hard gate in the reference's
        // rounding (expf, IEEE division), so it flips exactly where the mixer kernel's does
        const float su = fast_sigmoid(k * (x - Ec));
        const float sd = fast_sigmoid(k * (x + Ec));
        const float up = Ps * su * 2.0f - Ps;
        const float down = Ps * sd * 2.0f - Ps;
        const float bs = ref_sigmoid(gs * (x - pq)) > bp ? 1.0f : 0.0f;
        phi[r2 * Fp + q] = fast_sigmoid(bs * up + (1.0f - bs) * down + pr.w);
      }
      q += NT;
      while (q >= F) {
        q -= F;
        ++r2;
      }
    }
    __syncthreads();
    STAMP(1);
    if (tid < D) pvx[(n + 1) & 1][tid] = xs[NR][tid];  // :131-132, the shadow row's input
    // this quarter-wave's part of every row's head sums, outputs l16 + 16 c, four rows at a time
    const float4* W4 = s_dyn4 + (int64_t)part * G * 64 + l16;
    const float* ph0 = phi + qp0;
#pragma unroll
    for (int rc = 0; rc < R; rc += 4) {
      float acc[4][4];
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r2][c] = 0.f;
#pragma unroll 2
      for (int g = 0; g < gcount; ++g) {
        float4 w[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = W4[g * 64 + 16 * c];
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          const float4 p = *reinterpret_cast<const float4*>(ph0 + (rc + r2) * Fp + 4 * g);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            acc[r2][c] = __builtin_fmaf(p.x, w[c].x, acc[r2][c]);
            acc[r2][c] = __builtin_fmaf(p.y, w[c].y, acc[r2][c]);
            acc[r2][c] = __builtin_fmaf(p.z, w[c].z, acc[r2][c]);
            acc[r2][c] = __builtin_fmaf(p.w, w[c].w, acc[r2][c]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TAIL; j += 4) {
        if (j < ntail) {
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const float4 p = *reinterpret_cast<const float4*>(ph0 + (rc + r2) * Fp + QL + j);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              acc[r2][c] = __builtin_fmaf(p.x, wt[j][c], acc[r2][c]);
              acc[r2][c] = __builtin_fmaf(p.y, wt[j + 1][c], acc[r2][c]);
              acc[r2][c] = __builtin_fmaf(p.z, wt[j + 2][c], acc[r2][c]);
              acc[r2][c] = __builtin_fmaf(p.w, wt[j + 3][c], acc[r2][c]);
            }
          }
        }
      }
      // S_w = (P_4w + P_4w+1) + (P_4w+2 + P_4w+3): quarter 0 meets quarter 1, then the pairs meet
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          acc[r2][c] = acc[r2][c] + __shfl_xor(acc[r2][c], 16);
          acc[r2][c] = acc[r2][c] + __shfl_xor(acc[r2][c], 32);
        }
      if (qtr == 0)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2)
#pragma unroll
          for (int c = 0; c < 4; ++c) hs[(wv * R + rc + r2) * 64 + l16 + 16 * c] = acc[r2][c];
    }
    __syncthreads();
    STAMP(2);
    float out = 0.f;
    if (dval) {
      out = hs[r * 64 + d];
#pragma unroll
      for (int w = 1; w < kHeadGroups; ++w) out = out + hs[(w * R + r) * 64 + d];
      out = out + bhd;
    }
    // no trailing barrier: the next evaluation writes xs, then waits before phi / hs are rewritten
    ++nfev;
    return out;
  };

  float y = dval ? a.y0[b * D + d] : 0.f;
  if (real) a.sol[b * D + d] = y;
  float f0 = eval(y);
  double dt;
  if (a.first_step > 0.0) {
    dt = a.first_step;
  } else {  // misc._select_initial_step in fp32 (dopri5.py select_initial_step)
    const float scale = a.atol + a.rtol * fabsf(y);
    double s;
    const float q0 = y / scale, q1 = f0 / scale;
    double s1;
    global_sum2(real ? (double)q0 * q0 : 0.0, real ? (double)q1 * q1 : 0.0, s, s1);
    const float d0 = fabsf(sqrtf((float)(s / n_el)));
    const float d1 = fabsf(sqrtf((float)(s1 / n_el)));
    float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
    h0 = fabsf(h0);
    const float f1 = eval(y + f0 * h0);
    const float q2 = (f1 - f0) / scale;
    global_sum2(real ? (double)q2 * q2 : 0.0, 0.0, s, s1);
    const float d2 = fabsf(sqrtf((float)(s / n_el)) / h0);  // (status 4: the loop below is skipped)
    float h1;
    if (d1 <= 1e-15f && d2 <= 1e-15f) h1 = fmaxf(1e-6f, h0 * 1e-3f);
    else h1 = (float)pow((double)(0.01f / fmaxf(d1, d2)), (double)0.2f);  // fp64 pow rounded once: host == device
    dt = (double)fminf(100.0f * h0, fabsf(h1));
  }

  float co[5] = {y, 0.f, 0.f, 0.f, 0.f};
  double t0s = a.t[0], t1s = a.t[0];
  for (int i = 1; i < a.T && status == 0; ++i) {
    const double next_t = a.t[i];
    int n_steps = 0;
    while (next_t > t1s) {
      if (n_steps >= a.max_steps) { status = 3; break; }
      const double t0 = t1s;
      if (!(t0 + dt > t0)) { status = 2; break; }
      const float dt32 = (float)dt;
      const double t1 = t0 + dt;
      // rk_common._runge_kutta_step via fetode_lincomb's op order, accumulated as the stages
      // arrive: A[i] is stage s+1+i's sum k0*b0 + k1*b1 + ... (the same left-to-right sums), so
      // the stage loop keeps one copy of the evaluation and no indexed register array
      float A[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) A[i] = f0 * (a.tab.beta[i][0] * dt32);
      float err = f0 * (a.tab.cerr[0] * dt32);
      float mid = f0 * (a.tab.cmid[0] * dt32);
      float yi = y, kn = f0;
#pragma unroll 1
      for (int s = 0; s < 6; ++s) {
        yi = y + A[0];
        kn = eval(yi);
        const int j = s + 1;
#pragma unroll
        for (int i = 0; i < 5; ++i) A[i] = (j + i <= 5) ? A[i + 1] + kn * (a.tab.beta[j + i][j] * dt32) : 0.f;
        err = err + kn * (a.tab.cerr[j] * dt32);
        mid = mid + kn * (a.tab.cmid[j] * dt32);
      }
      const float y1 = yi;
      const float tol = a.atol + a.rtol * fmaxf(fabsf(y), fabsf(y1));
      const float qe = err / tol;
      double s, nbad;
      global_sum2(real ? (double)qe * qe : 0.0, (real && !__builtin_isfinite(y)) ? 1.0 : 0.0, s, nbad);
      if (status) break;
      if (nbad != 0.0) { status = 1; break; }
      const float ratio = sqrtf((float)(s / n_el));
      const bool accept = ratio <= 1.0f;
      if (blockIdx.x == 0 && tid == 0 && n_att < a.max_att) {
        double* o = a.att + (int64_t)n_att * 4;
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
        nxt = dt * a.ifactor;
      } else {
        const double dfac = rr < 1.0 ? 1.0 : a.dfactor;
        const double factor = __builtin_isnan(rr) ? rr : fmin(a.ifactor, fmax(a.safety / pow(rr, 1.0 / 5.0), dfac));
        nxt = dt * factor;
      }
      dt = __builtin_isnan(nxt) ? nxt : fmin(fmax(nxt, a.min_step), a.max_step);
      ++n_steps;
    }
    if (status) break;
    const float x = (float)((next_t - t0s) / (t1s - t0s));  // interp._interp_evaluate
    float total = co[0] + x * co[1];
    float xp = x;
#pragma unroll
    for (int j = 2; j < 5; ++j) {
      xp = xp * x;
      total = total + xp * co[j];
    }
    if (real) a.sol[(int64_t)i * BD + b * D + d] = total;
  }
  // module state after the solve: prev_x = the last evaluation's last-row input; branch_state of
  // that evaluation for this workgroup's rows (xs still holds its inputs)
  const int nl = nfev - 1;  // the last evaluation
  for (int q = tid; q < F; q += NT) {
    const int i = q / nb;
    if (blockIdx.x == 0) a.prev_out[q] = xs[NR][i];
    if (a.branch_out) {
      const float pq = nl == 0 ? pv0[q] : pvx[nl & 1][i];
      for (int r2 = 0; r2 < NR; ++r2) {
        const int64_t b2 = (int64_t)blockIdx.x * NR + r2;
        if (b2 < a.B) a.branch_out[b2 * F + q] = ref_sigmoid(gs * (xs[r2][i] - pq)) > bp ? 1.0f : 0.0f;
      }
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    a.stats[0] = nfev;
    a.stats[1] = n_att;
    a.stats[2] = __hip_atomic_load(a.bar + 64 * 9 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 4 : status;
#ifdef FETODE_STAMPS
    if (stamping) {
      for (int i = 0; i < 5; ++i) a.stamps[i] += st_acc[i];
      a.stamps[5] += __builtin_amdgcn_s_memtime() - st_clk0;
      a.stamps[6] += __builtin_amdgcn_s_memrealtime() - st_rt0;
    }
#endif
  }
}

long long* g_ecg_stamps = nullptr;  // fetode_debug_ecg_stamps

// one instantiation of the resident kernel: rows per workgroup and the register tail per part
struct EcgVariant {
  const void* fn;
  int rows, tail;
};
const EcgVariant kEcgVariants[] = {
    {reinterpret_cast<const void*>(ecg_dopri5_kernel<4, 8>), 4, 8},
    {reinterpret_cast<const void*>(ecg_dopri5_kernel<8, 8>), 8, 8},
};

}  // namespace

extern "C" {

int fetode_ecg_dopri5(const fetode_hlogistic_t* layer, const float* wT, const float* bias, int32_t D,
                      const float* prev, const float* y0, int64_t B, const double* t, int32_t T, double rtol,
                      double atol, const double* opts, const float* tableau, float* solution, float* prev_out,
                      float* branch_out, void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                      void* stream) {
  int rc = check_layer(layer);
  if (rc) return rc;
  if (B <= 0 || T <= 0) return FETODE_OK;
  if (!wT || !prev || !y0 || !t || !opts || !tableau || !solution || !prev_out || !workspace || !stats)
    return set_err(FETODE_EINVAL, "ecg dopri5: null pointer");
  if (D != layer->in_dim || D > 64) return set_err(FETODE_EINVAL, "ecg dopri5: state dim %d (must equal in_dim, <= 64)", D);
  const int F = layer->in_dim * layer->num_basis;
  if (F > kMaxF) return set_err(FETODE_EUNSUPPORTED, "ecg dopri5: in*num_basis=%d > %d", F, kMaxF);
  EcgDopriArgs a;
  memset(&a, 0, sizeof(a));
  a.L = to_dev(layer);
  a.wT = wT;
  a.bh = bias;
  a.D = D;
  a.F = F;
  a.Fp = (F + 3) & ~3;
  a.prev0 = prev;
  a.y0 = y0;
  a.B = B;
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
  memcpy(&a.tab, tableau, sizeof(DopriTab));
  a.sol = solution;
  a.prev_out = prev_out;
  a.branch_out = branch_out;
  a.bar = (unsigned*)workspace;
  a.part = (double*)((char*)workspace + sizeof(unsigned) * kBarWords);
  a.stats = stats;
  a.att = attempts;
  a.max_att = attempts ? max_attempts : 0;
  a.stamps = g_ecg_stamps;
  // per-variant launch facts, queried once (static LDS, the dynamic-LDS cap) and per LDS size
  // (occupancy): the launch path does no runtime queries on repeat calls
  static int n_cu_of[64] = {0};
  static struct {
    int static_lds = -1;
    size_t lds = 0;
    int per_cu = 0;
  } vstate[sizeof(kEcgVariants) / sizeof(kEcgVariants[0])];
  int dev = 0;
  HIP_CHECK_RET(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return set_err(FETODE_EINVAL, "ecg dopri5: device %d", dev);
  if (!n_cu_of[dev]) HIP_CHECK_RET(hipDeviceGetAttribute(&n_cu_of[dev], hipDeviceAttributeMultiprocessorCount, dev));
  const int n_cu = n_cu_of[dev];
  a.PS = head_part(F);
  // the smallest workgroup whose grid is co-resident (one cooperative grid) and whose head
  // weight fits LDS + its register tail
  for (size_t vi = 0; vi < sizeof(kEcgVariants) / sizeof(kEcgVariants[0]); ++vi) {
    const EcgVariant& v = kEcgVariants[vi];
    auto& vs = vstate[vi];
    if (vs.static_lds < 0) {
      hipFuncAttributes fa;
      HIP_CHECK_RET(hipFuncGetAttributes(&fa, v.fn));
      vs.static_lds = (int)fa.sharedSizeBytes;
    }
    // phi (R, Fp) + the (groups, R, 64) head sums; feature parameters; W^T in the rest
    const int64_t phi_bytes = (int64_t)sizeof(float) * v.rows * (a.Fp + 64 * kHeadGroups);
    const int64_t prm_bytes = (int64_t)sizeof(float) * (4 * F + a.Fp);  // + prev_x before the solve
    const int64_t w_floats = (kLdsBytes - (int64_t)vs.static_lds - phi_bytes - prm_bytes) / (int64_t)sizeof(float);
    if (w_floats < 0) continue;
    const int QL = (int)std::min<int64_t>(a.PS, (w_floats / ((int64_t)kHeadParts * 64)) & ~(int64_t)3);
    if (a.PS - QL > v.tail) continue;
    const size_t lds = (size_t)kHeadParts * QL * 64 * sizeof(float) + (size_t)(prm_bytes + phi_bytes);
    if (vs.lds != lds) {
      HIP_CHECK_RET(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      int per_cu = 0;
      HIP_CHECK_RET(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v.fn, kResThreads, lds));
      vs.lds = lds;
      vs.per_cu = per_cu;
    }
    const int64_t grid = (B + v.rows - 2) / (v.rows - 1);
    // one workgroup per CU below the API's answer when it admits several (it can be one too high)
    const int per_cu = vs.per_cu > 1 ? vs.per_cu - 1 : vs.per_cu;
    if (per_cu <= 0 || grid > (int64_t)per_cu * n_cu) continue;
    a.QL = QL;
    hipStream_t s = (hipStream_t)stream;
    HIP_CHECK_RET(hipMemsetAsync(workspace, 0, sizeof(unsigned) * kBarWords, s));
    void* args[] = {&a};
    HIP_CHECK_RET(resident_launch(v.fn, dim3((unsigned)grid), dim3(kResThreads), args, lds, s));
    return FETODE_OK;
  }
  return set_err(FETODE_EUNSUPPORTED, "ecg dopri5: batch %lld x in*num_basis %d does not fit one resident grid",
                 (long long)B, F);
}

#ifdef FETODE_STAMPS
void fetode_debug_ecg_stamps(void* p) { g_ecg_stamps = (long long*)p; }
#endif

int64_t fetode_ecg_dopri5_workspace(int64_t B) {
  const int64_t grid = (B + 2) / 3;  // the most workgroups any variant launches (3 real rows each)
  return (int64_t)sizeof(unsigned) * kBarWords + (int64_t)sizeof(double) * 2 * 2 * grid;
}

}  // extern "C"
