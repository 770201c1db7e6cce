// fetode_fieldn_plan.h — where fieldn's kernels find a plan entry: in the plan itself (global
// memory, or its verbatim LDS copy) or in the lane-contiguous LDS IMAGE of it.
//
// The plan (fetode_common.h LayerPlan) stores every per-edge table output-major: entry (o, i, c)
// of layer L at ((o * in + i) * C + c).  fieldn's lanes run over layer 0's OUTPUTS (lane = o) and
// layer 1's INPUTS (lane = i), so in the plan one wave's reads of one entry are in * C (layer 0)
// or C (layer 1) words apart — LDS bank conflicts on every edge table read (PMC: 0.6 extra cycles
// per LDS-array cycle in the KAN([4, 32, 4]) solve).  The image permutes each table inside its own
// segment so that the lane index is innermost:
//   layer 0 (lane o):  (i, c, o) -> ((i * C + c) * out + o)
//   layer 1 (lane i):  (o, c, i) -> ((o * C + c) * in + i), and the per-input tables (logistic
//                      (-a log2e, a b log2e) pairs, knots, 1/knot steps) as (c, i) -> c * in + i
// Spline cubics keep their float4 granularity (C = interval, the float4 per lane contiguous).
// Segment offsets are the plan's, so only the index arithmetic differs (IMG below).
#pragma once

#include "fetode_common.h"

namespace fetode {

// where source entry q of layer L's segment lands in the image (32-bit arithmetic: an image is
// at most kFnLdsMax bytes, and 64-bit division is a long software sequence on the GPU)
template <int L>
__device__ __forceinline__ int fn_img_dst(const LayerPlan& P, int q) {
  const int in = P.in, out = P.out, K = P.K, NFL = P.NFL, NI1 = P.NI + 1;
  const int NE = in * out * K;
  const int fe = (int)P.fe_GEc, fc = (int)P.fconst, kw = (int)P.kw, lg = (int)P.lg, kn = (int)P.knots,
            rh = (int)P.rh, sp = (int)P.sp, fl = (int)P.flag;
  if (NE > 0 && q >= fe && q < fc) {  // the four Ferro element arrays (o, i, k)
    const int a0 = fe + ((q - fe) / NE) * NE, r = q - a0;
    const int k = r % K, oi = r / K, o = oi / in, i = oi % in;
    return a0 + (L == 0 ? (i * K + k) * out + o : (o * K + k) * in + i);
  }
  if (q >= kw && q < lg) {  // (o, i, c): SiLU weight, logistic weights
    const int r = q - kw, c = r % NFL, oi = r / NFL, o = oi / in, i = oi % in;
    return kw + (L == 0 ? (i * NFL + c) * out + o : (o * NFL + c) * in + i);
  }
  if (q >= sp && q < fl) {  // (o, i, interval) float4s
    const int r = q - sp, c = r % 4, t = r / 4, m = t % NI1, oi = t / NI1, o = oi / in, i = oi % in;
    return sp + (L == 0 ? (i * NI1 + m) * out + o : (o * NI1 + m) * in + i) * 4 + c;
  }
  if constexpr (L == 1) {
    if (q >= lg && q < kn) {  // (i, j, 2) -> (j, 2, i)
      const int r = q - lg, c = r % 2, ij = r / 2, i = ij / P.NB, j = ij % P.NB;
      return lg + (j * 2 + c) * in + i;
    }
    if (q >= kn && q < rh) {  // (i, j) -> (j, i)
      const int r = q - kn;
      return kn + (r % P.NG) * in + r / P.NG;
    }
    if (q >= rh && q < rh + in * P.NI) {  // (i, m) -> (m, i)
      const int r = q - rh;
      return rh + (r % P.NI) * in + r / P.NI;
    }
  }
  return q;  // fconst, flag, alignment padding
}

// the image of both layers in LDS (every thread of the workgroup; a barrier follows)
__device__ __forceinline__ void fn_stage_image(float* __restrict__ dst, const float* __restrict__ plan,
                                               const LayerPlan& P0, const LayerPlan& P1) {
  const int n0 = (int)P0.end, n = (int)P1.end;
  for (int q = threadIdx.x; q < n; q += blockDim.x) dst[q < n0 ? fn_img_dst<0>(P0, q) : fn_img_dst<1>(P1, q)] = plan[q];
}

// edge (o, i) of layer L: the base of its table row and the stride between its entries
template <bool IMG, int L>
struct FnIdx {
  // per-edge tables (kw, Ferro arrays): entry c of edge (o, i) of a table of C entries per edge
  __device__ static __forceinline__ int64_t row(const LayerPlan& P, int64_t off, int o, int i, int C) {
    if constexpr (!IMG) return off + ((int64_t)o * P.in + i) * C;
    else if constexpr (L == 0) return off + (int64_t)i * C * P.out + o;
    else return off + (int64_t)o * C * P.in + i;
  }
  __device__ static __forceinline__ int stride(const LayerPlan& P) {
    if constexpr (!IMG) return 1;
    else if constexpr (L == 0) return P.out;
    else return P.in;
  }
  // the spline cubic of edge (o, i) on interval m (float index of its float4)
  __device__ static __forceinline__ int64_t sp(const LayerPlan& P, int o, int i, int m) {
    if constexpr (!IMG) return P.sp + (((int64_t)o * P.in + i) * (P.NI + 1) + m) * 4;
    else if constexpr (L == 0) return P.sp + (((int64_t)i * (P.NI + 1) + m) * P.out + o) * 4;
    else return P.sp + (((int64_t)o * (P.NI + 1) + m) * P.in + i) * 4;
  }
  // per-input tables: knot j, 1 / step of interval m, logistic pair entry (j, c)
  __device__ static __forceinline__ int64_t knot(const LayerPlan& P, int i, int j) {
    if constexpr (IMG && L == 1) return P.knots + (int64_t)j * P.in + i;
    else return P.knots + (int64_t)i * P.NG + j;
  }
  __device__ static __forceinline__ int knot_stride(const LayerPlan& P) {
    if constexpr (IMG && L == 1) return P.in;
    else return 1;
  }
  __device__ static __forceinline__ int64_t rh(const LayerPlan& P, int i, int m) {
    if constexpr (IMG && L == 1) return P.rh + (int64_t)m * P.in + i;
    else return P.rh + (int64_t)i * P.NI + m;
  }
  __device__ static __forceinline__ int64_t lg(const LayerPlan& P, int i, int j, int c) {
    if constexpr (IMG && L == 1) return P.lg + ((int64_t)j * 2 + c) * P.in + i;
    else return P.lg + 2 * ((int64_t)i * P.NB + j) + c;
  }
};

}  // namespace fetode
