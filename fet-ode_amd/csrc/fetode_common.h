// fetode_common.h — shared host/device declarations of libfetode (plan layout, errors).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fetode.h"
#include "fetode_device.h"

namespace fetode {

int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIP_CHECK_RET(expr)                                                                        \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return ::fetode::set_err(FETODE_EHIP, "%s: %s", #expr, hipGetErrorString(e_));              \
  } while (0)

#define LAUNCH_CHECK()                                                                             \
  do {                                                                                             \
    hipError_t e_ = hipGetLastError();                                                             \
    if (e_ != hipSuccess)                                                                          \
      return ::fetode::set_err(FETODE_EHIP, "kernel launch: %s", hipGetErrorString(e_));           \
  } while (0)

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

// Packed per-layer "plan" (parameters pre-transformed once per solve).
// All offsets are in floats from the start of the plan buffer.
struct LayerPlan {
  int in, out, K, NB, SO, NG, NI, NFL;  // NI = NG-1 knot intervals, NFL = 1 + NB LDS features/input
  int64_t base;
  int64_t fe_GEc;   // (out, in*K)  gate_slope*log2e*Ec            (Ferro element order o, i, k)
  int64_t fe_k2;    // (out, in*K)  2*log2e*k
  int64_t fe_k2Ec;  // (out, in*K)  2*log2e*k*Ec
  int64_t fe_CPs2;  // (out, in*K)  coef*Ps
  int64_t fconst;   // (out)        sum_{i,k} coef*bias
  int64_t kw;       // (out, in*NFL) SiLU weight, 2*scaled logistic weights
  int64_t lg;       // (in*NB, 2)   (-a*log2e, a*b*log2e)
  int64_t knots;    // (in, NG)
  int64_t rh;       // (in, NI)     1/(g[m+1]-g[m])
  int64_t sp;       // (out, in, NI+1, 4) spline contribution as a cubic in u per interval
  int64_t flag;     // 1 word: max |gate_slope*log2e*Ec| (float bits) -> factored-exp guard
  int64_t end;
  float gsl2e;      // gate_slope*log2e
  float wc;         // -2*(1-alpha)
};

void layer_plan(const fetode_kanlinear_t& kl, const fetode_ferro_t* fl, int64_t base, LayerPlan* p);
int validate_field(const fetode_field_t* f);

// depth-2 fields of other widths served by fieldn_kernel (fetode_fused.hip), and their reverse
// sweep (fetode_fieldn_bwd.hip): arguments and workspace as fetode_integrate_fixed_backward
bool fieldn_shape_supported(const fetode_field_t* f);
// Ferro parameter sums over R rows split across workgroups (fetode_grad.hip; E * S <= 8192 partial
// slots of the fixed-size workspace): the hysteresis input of row r is p0[r] (or x[r] when p0 is
// null) for r < n0 and x[r - n0] after
int64_t ferro_param_rows_workspace();
int ferro_param_rows(const fetode_ferro_t* fl, const float* x, int64_t R, const float* p0, int64_t n0, const float* g,
                     const fetode_ferro_grad_t* grads, void* workspace, int32_t accumulate, void* stream);
int64_t fieldn_fixed_backward_workspace(const fetode_field_t* f, int32_t method, int32_t n_steps, int64_t B);
int fieldn_fixed_backward(const fetode_field_t* f, const void* plan, int32_t method, int64_t B, const float* step_coef,
                          int32_t n_steps, const int32_t* out_step, const int32_t* out_mode, const float* out_slope,
                          int32_t T, const float* grad_solution, const float* tape, const float* state0,
                          uint32_t init_mask, float* grad_y0, const fetode_kanlinear_grad_t* kan_grads,
                          const fetode_ferro_grad_t* ferro_grads, void* workspace, void* stream);
// the reverse sweep of fieldn's taped resident dopri5 solve (arguments as fetode_integrate_dopri5_backward)
int64_t fieldn_dopri5_backward_max_batch(const fetode_field_t* f);
int64_t fieldn_dopri5_backward_workspace(const fetode_field_t* f, int64_t B, int64_t n_ev);
int fieldn_dopri5_backward(const fetode_field_t* f, const void* plan, int64_t B, const double* t, int32_t T, double rtol,
                           double atol, const double* opts, const float* tableau, const float* grad_solution,
                           const float* tape, int32_t n_ev, const double* attempts, int32_t n_att,
                           const double* init_rec, const float* state0, uint32_t init_mask, float* grad_y0,
                           const fetode_kanlinear_grad_t* kan_grads, const fetode_ferro_grad_t* ferro_grads,
                           void* workspace, int32_t* status, void* stream);

// Launch of a grid that must be co-resident (the device-resident solvers' grid reductions).  The
// callers size the grid by occupancy; by default it is an ordinary launch (bounded spins turn a
// grid that is not co-resident into status 4), or hipLaunchCooperativeKernel when switched on
// (fetode_resident_launch_mode(1), env FETODE_COOPERATIVE=1).
hipError_t resident_launch(const void* fn, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s);
int resident_mode();
extern int g_resident_mode;

// The factored gate exp(gs(x+Ec)) = exp(gs x) * exp(gs Ec) is used only when
// |gs*log2e*Ec| <= kFactorLimit everywhere in the layer: then exp(gs x) overflowing /
// underflowing can only happen where the fp32 sigmoid is already saturated at 0 / 1.
constexpr float kFactorLimit = 60.0f;

}  // namespace fetode
