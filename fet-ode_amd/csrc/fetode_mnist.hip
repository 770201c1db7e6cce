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
#include "fetode_common.h"

using namespace fetode;

namespace {

constexpr int kKThreads = 256;
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
      sn[p] = sinf(t);
      cs[p] = cosf(t);
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
    feat[b * 2 * HW + p] = cosf(t);
    feat[b * 2 * HW + HW + p] = sinf(t);
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
    g[p] = (-sinf(t)) * gfeat[b * 2 * HW + p] + cosf(t) * gfeat[b * 2 * HW + HW + p];
    go[p] = 0.f;
  }
  for (int s = steps - 1; s >= 0; --s) {
    __syncthreads();
    for (int p = threadIdx.x; p < HW; p += kKThreads) {
      const float t = tb[s * HW + p];
      sn[p] = sinf(t);
      cs[p] = cosf(t);
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

// out[j] (+)= sum_b part[b, j], b in increasing order in fp64: one thread per column
__global__ void column_sum_kernel(const float* __restrict__ part, int64_t B, int n, float* __restrict__ out,
                                  int accumulate) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int64_t b = 0; b < B; ++b) s += (double)part[b * n + j];
  out[j] = accumulate ? out[j] + (float)s : (float)s;
}

}  // namespace

extern "C" {

int fetode_kuramoto_forward(const float* x, int64_t B, int32_t H, int32_t W, int32_t steps, float dt, const float* K,
                            const float* omega, float* feat, float* tape, void* stream) {
  if (B <= 0) return FETODE_OK;
  if (!x || !K || !omega || !feat) return set_err(FETODE_EINVAL, "kuramoto: null pointer");
  if (H <= 0 || W <= 0 || H * W > kMaxPix || steps < 0)
    return set_err(FETODE_EINVAL, "kuramoto: H*W=%d (1..%d), steps=%d", H * W, kMaxPix, steps);
  const size_t lds = sizeof(float) * 3 * H * W;
  hipLaunchKernelGGL(kuramoto_fwd_kernel, dim3((unsigned)B), dim3(kKThreads), lds, (hipStream_t)stream, x, H, W, steps,
                     dt, K, omega, feat, tape);
  LAUNCH_CHECK();
  return FETODE_OK;
}

int64_t fetode_kuramoto_backward_workspace(int64_t B, int32_t H, int32_t W) {
  return (int64_t)sizeof(float) * B * ((int64_t)H * W + 1);
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
  const size_t lds = sizeof(float) * 4 * HW;
  hipLaunchKernelGGL(kuramoto_bwd_kernel, dim3((unsigned)B), dim3(kKThreads), lds, s, H, W, steps, dt, K, tape, gfeat,
                     gx, gK_part, gom_part);
  LAUNCH_CHECK();
  if (gomega) {
    hipLaunchKernelGGL(column_sum_kernel, dim3((HW + 255) / 256), dim3(256), 0, s, gom_part, B, HW, gomega, 0);
    LAUNCH_CHECK();
  }
  if (gK) {
    hipLaunchKernelGGL(column_sum_kernel, dim3(1), dim3(256), 0, s, gK_part, B, 1, gK, 0);
    LAUNCH_CHECK();
  }
  return FETODE_OK;
}

}  // extern "C"
