// fetode_common.hip — errors, shape validation and the parameter plan.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "fetode_common.h"

namespace fetode {

static thread_local std::string g_last_error;

// -1: not yet read from the environment
int g_resident_mode = -1;
int resident_mode() {
  if (g_resident_mode < 0) {
    const char* v = getenv("FETODE_COOPERATIVE");
    g_resident_mode = v && atoi(v) != 0;
  }
  return g_resident_mode;
}

hipError_t resident_launch(const void* fn, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s) {
  if (resident_mode()) return hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)lds, s);
  return hipLaunchKernel(fn, grid, block, args, lds, s);
}

int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

void layer_plan(const fetode_kanlinear_t& kl, const fetode_ferro_t* fl, int64_t base, LayerPlan* p) {
  p->in = kl.in_features;
  p->out = kl.out_features;
  p->K = fl ? fl->num_basis : 0;
  p->NB = kl.num_logistic;
  p->SO = kl.spline_order;
  p->NG = kl.grid_size + 2 * kl.spline_order + 1;
  p->NI = p->NG - 1;
  p->NFL = 1 + p->NB;
  const int64_t NE = (int64_t)p->in * p->out * p->K;
  p->base = base;
  int64_t o = base;
  p->fe_GEc = o; o += NE;
  p->fe_k2 = o; o += NE;
  p->fe_k2Ec = o; o += NE;
  p->fe_CPs2 = o; o += NE;
  p->fconst = o; o += p->out;
  p->kw = o; o += (int64_t)p->out * p->in * p->NFL;
  p->lg = o; o += (int64_t)p->in * p->NB * 2;
  p->knots = o; o += (int64_t)p->in * p->NG;
  p->rh = o; o += (int64_t)p->in * p->NI;
  o = (o + 3) & ~int64_t(3);  // 16-B aligned float4 table
  p->sp = o; o += (int64_t)p->out * p->in * (p->NI + 1) * 4;
  p->flag = o; o += 1;
  o = (o + 3) & ~int64_t(3);
  p->end = o;
  // the reference multiplies by Python floats: (1.0 - alpha) is formed in double, then rounded
  p->gsl2e = fl ? (float)fl->gate_slope * FETODE_LOG2E : 0.f;
  p->wc = fl ? -2.0f * (float)(1.0 - fl->alpha) : 0.f;
}

int validate_field(const fetode_field_t* f) {
  if (!f || f->n_layers <= 0 || !f->kan) return set_err(FETODE_EINVAL, "field: no layers");
  for (int l = 0; l < f->n_layers; ++l) {
    const fetode_kanlinear_t& k = f->kan[l];
    if (k.in_features <= 0 || k.out_features <= 0 || k.grid_size <= 0 || k.spline_order < 1 ||
        k.spline_order > 3 || k.num_logistic < 0)
      return set_err(FETODE_EINVAL, "layer %d: bad KANLinear dims", l);
    if (!k.grid || !k.base_weight || !k.spline_weight)
      return set_err(FETODE_EINVAL, "layer %d: null KANLinear parameter", l);
    if (k.num_logistic > 0 && (!k.logistic_a || !k.logistic_b || !k.logistic_weight))
      return set_err(FETODE_EINVAL, "layer %d: null logistic parameter", l);
    if (l > 0 && k.in_features != f->kan[l - 1].out_features)
      return set_err(FETODE_EINVAL, "layer %d: in_features %d != previous out %d", l,
                     k.in_features, f->kan[l - 1].out_features);
    if (f->ferro) {
      const fetode_ferro_t& r = f->ferro[l];
      if (r.in_dim != k.in_features || r.out_dim != k.out_features || r.num_basis <= 0)
        return set_err(FETODE_EINVAL, "layer %d: Ferro dims (%d,%d,%d) mismatch KANLinear", l,
                       r.in_dim, r.out_dim, r.num_basis);
      if (!r.k || !r.Ec || !r.Ps || !r.bias || !r.coef)
        return set_err(FETODE_EINVAL, "layer %d: null Ferro parameter", l);
    }
  }
  return FETODE_OK;
}

// Cox–de Boor restricted to knot interval m (double precision, plan build only): the SO+1
// bases B_{m-SO+r} that are non-zero on [g_m, g_{m+1}), as polynomials evaluated at x.
template <int SO>
__device__ void bspline_on_interval(double x, int m, int NG, const float* g, double* N) {
  for (int r = 0; r < SO + 2; ++r) N[r] = 0.0;
  N[SO] = 1.0;
  for (int k = 1; k <= SO; ++k) {
    double M[SO + 2];
    for (int r = 0; r < SO + 2; ++r) M[r] = 0.0;
    for (int r = SO - k; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j <= NG - 2 - k) {
        double left = (x - g[j]) / ((double)g[j + k] - g[j]) * N[r];
        double right = ((double)g[j + k + 1] - x) / ((double)g[j + k + 1] - g[j + 1]) * N[r + 1];
        M[r] = left + right;
      }
    }
    for (int r = 0; r < SO + 2; ++r) N[r] = M[r];
  }
}

template <int SO>
__device__ void spline_interval_poly(const fetode_kanlinear_t& kl, const LayerPlan& P, int o, int i, int m,
                                     float* dst) {
  if (m >= P.NI) {
    dst[0] = dst[1] = dst[2] = dst[3] = 0.f;
    return;
  }
  const float* g = kl.grid + (int64_t)i * P.NG;
  const int NS = P.NG - 1 - SO;
  const float sc = kl.spline_scaler ? kl.spline_scaler[o * P.in + i] : 1.0f;
  const float* sw = kl.spline_weight + ((int64_t)o * P.in + i) * NS;
  const double h = (double)g[m + 1] - g[m];
  double v[4];
  for (int s = 0; s < 4; ++s) {
    const double x = g[m] + h * (s / 3.0);
    double N[SO + 2];
    bspline_on_interval<SO>(x, m, P.NG, g, N);
    double acc = 0.0;
    for (int r = 0; r <= SO; ++r) {
      const int j = m - SO + r;
      if (j >= 0 && j < NS) acc += N[r] * ((double)sw[j] * sc);
    }
    v[s] = acc;
  }
  // cubic through u = 0, 1/3, 2/3, 1 in power basis
  dst[0] = (float)v[0];
  dst[1] = (float)((-11.0 * v[0] + 18.0 * v[1] - 9.0 * v[2] + 2.0 * v[3]) / 2.0);
  dst[2] = (float)(9.0 * (2.0 * v[0] - 5.0 * v[1] + 4.0 * v[2] - v[3]) / 2.0);
  dst[3] = (float)(9.0 * (-v[0] + 3.0 * v[1] - 3.0 * v[2] + v[3]) / 2.0);
}

__device__ void plan_build_layer(const LayerPlan& P, const fetode_kanlinear_t& kl, const fetode_ferro_t& fl,
                                 int has_ferro, float* __restrict__ plan, int tid) {
  const int in = P.in, out = P.out, K = P.K, NB = P.NB, NG = P.NG, NI = P.NI, NFL = P.NFL;
  const float l2 = FETODE_LOG2E;
  if (has_ferro) {
    const int NP = in * K;
    if (tid < out * NP) {
      const int o = tid / NP, p = tid % NP, i = p / K, k = p % K;
      const int src = (i * out + o) * K + k;
      const float kk = fl.k[src], Ec = fl.Ec[src], Ps = fl.Ps[src], co = fl.coef[src];
      const float gec = P.gsl2e * Ec;
      plan[P.fe_GEc + tid] = gec;
      const float k2 = 2.0f * l2 * kk;
      plan[P.fe_k2 + tid] = k2;
      plan[P.fe_k2Ec + tid] = k2 * Ec;
      plan[P.fe_CPs2 + tid] = co * Ps;
    }
  } else if (tid < out) {
    plan[P.fconst + tid] = 0.f;
  }
  if (tid < out * in * NFL) {
    const int o = tid / (in * NFL), r = tid % (in * NFL), i = r / NFL, f = r % NFL;
    float w;
    if (f == 0) {
      w = kl.base_weight[o * in + i];
    } else {
      const int j = f - 1;
      const float ls = kl.logistic_scaler ? kl.logistic_scaler[o] : 1.0f;
      w = 2.0f * ((kl.logistic_weight[(int64_t)o * (in * NB) + i * NB + j] * kl.scale_logistic) * ls);
    }
    plan[P.kw + tid] = w;
  }
  if (tid < in * NB) {
    const float a = kl.logistic_a[tid], b = kl.logistic_b[tid];
    plan[P.lg + 2 * tid + 0] = -a * l2;
    plan[P.lg + 2 * tid + 1] = (a * b) * l2;
  }
  if (tid < in * NG) plan[P.knots + tid] = kl.grid[tid];
  if (tid < in * NI) {
    const int i = tid / NI, m = tid % NI;
    const float* g = kl.grid + (int64_t)i * NG;
    plan[P.rh + tid] = 1.0f / (g[m + 1] - g[m]);
  }
  if (tid < out * in * (NI + 1)) {
    const int o = tid / (in * (NI + 1)), r = tid % (in * (NI + 1)), i = r / (NI + 1), m = r % (NI + 1);
    float* dst = plan + P.sp + (int64_t)tid * 4;
    if (P.SO == 1) spline_interval_poly<1>(kl, P, o, i, m, dst);
    else if (P.SO == 2) spline_interval_poly<2>(kl, P, o, i, m, dst);
    else spline_interval_poly<3>(kl, P, o, i, m, dst);
  }
}

constexpr int kPlanMaxLayers = 8;
constexpr int kPlanBlock = 128;
struct PlanBatch {
  int n_layers;
  int blk_begin[kPlanMaxLayers + 1];  // item blocks of layer l: [blk_begin[l], blk_begin[l+1])
  LayerPlan P[kPlanMaxLayers];
  fetode_kanlinear_t kl[kPlanMaxLayers];
  fetode_ferro_t fl[kPlanMaxLayers];
  int has_ferro[kPlanMaxLayers];
};

__device__ inline float wave_sum(float v) {
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ inline float wave_max(float v) {
  for (int m = 32; m > 0; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// One launch for every layer: item blocks, then one tail block per Ferro layer that computes
// the per-output constant sum_{i,k} coef*bias (one wave per output, fixed order) and the
// factored-exp guard word max |gate_slope*log2e*Ec| — no atomics, no memset, deterministic.
__global__ __launch_bounds__(kPlanBlock) void plan_build_kernel(PlanBatch pb, float* __restrict__ plan) {
  constexpr int kWaves = kPlanBlock / 64;
  __shared__ float red[kWaves];
  const int blk = blockIdx.x;
  const int nitem = pb.blk_begin[pb.n_layers];
  if (blk < nitem) {
    int l = 0;
    while (blk >= pb.blk_begin[l + 1]) ++l;
    plan_build_layer(pb.P[l], pb.kl[l], pb.fl[l], pb.has_ferro[l], plan,
                     (blk - pb.blk_begin[l]) * kPlanBlock + threadIdx.x);
    return;
  }
  const int l = blk - nitem;
  const LayerPlan& P = pb.P[l];
  if (!pb.has_ferro[l]) {
    if (threadIdx.x == 0) plan[P.flag] = 0.f;
    return;
  }
  const fetode_ferro_t& fl = pb.fl[l];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int NIK = P.in * P.K;
  for (int o = wave; o < P.out; o += kWaves) {
    float s = 0.f;
    for (int p = lane; p < NIK; p += 64) {
      const int i = p / P.K, k = p % P.K;
      const int src = (i * P.out + o) * P.K + k;
      s += fl.coef[src] * fl.bias[src];
    }
    s = wave_sum(s);
    if (lane == 0) plan[P.fconst + o] = s;
  }
  const int NE = P.in * P.out * P.K;
  float mx = 0.f;
  for (int e = threadIdx.x; e < NE; e += kPlanBlock) mx = fmaxf(mx, fabsf(P.gsl2e * fl.Ec[e]));
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kWaves; ++w) mx = fmaxf(mx, red[w]);
    plan[P.flag] = mx;
  }
}

}  // namespace fetode

using namespace fetode;

extern "C" {

const char* fetode_last_error(void) { return g_last_error.c_str(); }

int32_t fetode_resident_launch_mode(int32_t mode) {
  const int32_t prev = fetode::resident_mode();
  if (mode >= 0) fetode::g_resident_mode = mode != 0;
  return prev;
}
int fetode_abi_version(void) { return FETODE_ABI_VERSION; }

int32_t fetode_state_width(const fetode_field_t* f) {
  if (!f || !f->ferro) return 0;
  int32_t w = 0;
  for (int l = 0; l < f->n_layers; ++l) w += f->ferro[l].in_dim;
  return w;
}

int64_t fetode_plan_bytes(const fetode_field_t* f) {
  if (validate_field(f) != FETODE_OK) return -1;
  int64_t base = 0;
  for (int l = 0; l < f->n_layers; ++l) {
    LayerPlan p;
    layer_plan(f->kan[l], f->ferro ? &f->ferro[l] : nullptr, base, &p);
    base = p.end;
  }
  return base * (int64_t)sizeof(float);
}

int fetode_plan_build(const fetode_field_t* f, void* plan, void* stream) {
  int rc = validate_field(f);
  if (rc) return rc;
  if (!plan) return set_err(FETODE_EINVAL, "plan is NULL");
  int64_t base = 0;
  for (int l0 = 0; l0 < f->n_layers; l0 += kPlanMaxLayers) {
    PlanBatch pb;
    memset(&pb, 0, sizeof(pb));
    pb.n_layers = std::min(kPlanMaxLayers, f->n_layers - l0);
    int blocks = 0;
    for (int j = 0; j < pb.n_layers; ++j) {
      const int l = l0 + j;
      const fetode_ferro_t* fl = f->ferro ? &f->ferro[l] : nullptr;
      LayerPlan& p = pb.P[j];
      layer_plan(f->kan[l], fl, base, &p);
      base = p.end;
      pb.kl[j] = f->kan[l];
      if (fl) pb.fl[j] = *fl;
      pb.has_ferro[j] = fl ? 1 : 0;
      const int64_t n = std::max<int64_t>({(int64_t)p.out * p.in * std::max(p.K, 1), (int64_t)p.out * p.in * p.NFL,
                                           (int64_t)p.in * p.NG, (int64_t)p.in * std::max(p.NB, 1),
                                           (int64_t)p.out * p.in * (p.NI + 1), (int64_t)p.out});
      pb.blk_begin[j] = blocks;
      blocks += nblk(n, kPlanBlock);
    }
    pb.blk_begin[pb.n_layers] = blocks;
    hipLaunchKernelGGL(plan_build_kernel, dim3(blocks + pb.n_layers), dim3(kPlanBlock), 0, (hipStream_t)stream, pb,
                       (float*)plan);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

}  // extern "C"
