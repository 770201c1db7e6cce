/*
 * fetode.h — C ABI of libfetode.so, the MI355X (gfx950) hot path of the
 * KAN-FET Neural-ODE integrator.
 *
 * The reference (sallywang147/FET-ODE) is pure Python; it has no FFI.  Its
 * drop-in boundary on this path is the Python surface
 *   torchdiffeq.odeint(func, y0, t, rtol, atol, method, options)
 *       call sites: train_kanfet_node_predprey.py:252,260, predator_prey.py:142,149
 *   efficientkan.KANLinear.forward / .b_splines   efficient_kan/efficientkan.py:117-182
 *   ferro_class.FerroelectricBasis.forward          ferro_class.py:368-420
 * Each entry point below replaces one of those; the Python package
 * (fet-ode_amd/) binds them with ctypes (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - every pointer marked (dev) is device memory on the current HIP device;
 *     (host) pointers are host memory read synchronously before return.
 *   - tensors are fp32, C-contiguous, shapes in comments.
 *   - all work is enqueued on `stream` (a hipStream_t, may be NULL = default
 *     stream); nothing is allocated and nothing synchronises the host.
 *   - return 0 on success, otherwise a FETODE_E* code; fetode_last_error()
 *     returns a thread-local message for the last failure.
 */
#ifndef FETODE_H_
#define FETODE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FETODE_ABI_VERSION 2

enum {
  FETODE_OK = 0,
  FETODE_EINVAL = 1,       /* bad shape / argument */
  FETODE_EUNSUPPORTED = 2, /* no fused kernel for this field shape; use the per-stage path */
  FETODE_EHIP = 3          /* HIP runtime error (message in fetode_last_error) */
};

/* integration methods (torchdiffeq names) */
enum {
  FETODE_EULER = 0,     /* fixed_grid.Euler */
  FETODE_MIDPOINT = 1,  /* fixed_grid.Midpoint */
  FETODE_RK4 = 2,       /* fixed_grid.RK4 -> rk_common.rk4_alt_step_func (3/8 rule) */
  FETODE_RK4_CLASSIC = 3 /* classic 1/6 weights: train_ecg_kan_fet_nn_ode.py:693-705 */
};

/* One efficientkan.KANLinear (efficient_kan/efficientkan.py:27-90).  (dev) pointers. */
typedef struct fetode_kanlinear {
  int32_t in_features, out_features;
  int32_t grid_size, spline_order;  /* grid has grid_size + 2*spline_order + 1 knots per input */
  int32_t num_logistic;             /* logistic branch basis count; 0 = branch disabled */
  int32_t base_act;                 /* 0 = SiLU (the only activation on the path) */
  const float* grid;                /* (in, grid_size+2*spline_order+1) buffer :55-61 */
  const float* base_weight;         /* (out, in) */
  const float* spline_weight;       /* (out, in, grid_size+spline_order) */
  const float* spline_scaler;       /* (out, in), NULL if enable_standalone_scale_spline=False */
  const float* logistic_a;          /* (in, nb)  LogisticBasis.a :17 */
  const float* logistic_b;          /* (in, nb)  LogisticBasis.b :18 */
  const float* logistic_weight;     /* (out, in*nb) */
  const float* logistic_scaler;     /* (out), NULL if enable_standalone_scale_logistic=False */
  float scale_logistic;             /* :45 */
} fetode_kanlinear_t;

/* One ferro_class.FerroelectricBasis (ferro_class.py:329-424).  (dev) pointers. */
typedef struct fetode_ferro {
  int32_t in_dim, out_dim, num_basis;
  const float *k, *Ec, *Ps, *bias, *coef; /* each (in, out, K) :358-362 */
  double gate_slope, alpha;               /* :347 defaults 10.0, 0.8 (Python floats) */
  /* branch_sign buffer (:366).  The reference never writes it after (re)initialising it to
   * ones (:377-378), so NULL means "all ones" (fast path).  Otherwise a (Bs, in, out, K) tensor
   * with batch stride branch_sign_bstride elements (0 = broadcast one slice). */
  const float* branch_sign;
  int64_t branch_sign_bstride;
} fetode_ferro_t;

/* A vector field: a stack of layers, layer l = kan[l](x) (+ ferro[l](x) when present).
 * KANFET (build-defined): both present.  efficientkan.KAN: ferro == NULL.
 * (host) arrays of n_layers descriptors. */
typedef struct fetode_field {
  int32_t n_layers;
  const fetode_kanlinear_t* kan;  /* n_layers entries */
  const fetode_ferro_t* ferro;    /* n_layers entries or NULL (no hysteresis layers) */
} fetode_field_t;

/* Hysteresis state of a field: for every Ferro layer l a compact prev_x of shape (B, in_l)
 * (the reference stores x.expand(B,in,out,K), ferro_class.py:372,409 — constant over out,K).
 * Layout: one contiguous (B, in_l) block per Ferro layer, blocks concatenated in layer order:
 * element (l, b, i) at state[B*off_l + b*in_l + i], off_l = sum of in over earlier Ferro layers
 * (so every layer's prev_x is itself a contiguous (B, in_l) tensor); total B*state_width.
 * init_mask bit l set  =>  the reference's re-initialisation rule fires on the first call
 * (prev_x := x, i.e. dx = 0, ferro_class.py:373-375); clear => use the stored prev_x. */

const char* fetode_last_error(void);
/* How the device-resident solvers (fetode_integrate_dopri5, fetode_ecg_dopri5) launch their grid,
 * which is sized by occupancy to be co-resident: 0 (default) an ordinary launch, 1
 * hipLaunchCooperativeKernel (env FETODE_COOPERATIVE=1).  A grid that is not co-resident ends
 * in status 4 (bounded spins), never a hang.  mode < 0 queries.  Returns the previous mode. */
int32_t fetode_resident_launch_mode(int32_t mode);
/* Test knob of the resident dopri5 solvers (fetode_integrate_dopri5[_xrank|_tape]): polls of one
 * grid-reduction / cross-rank spin before it gives up with status 4 (0 = the built-in limits,
 * ~1 s single device, ~16 s across ranks).  A tiny limit forces the timeout path on a healthy
 * grid (tests/test_gpu_dopri5.py: the pre-solve hysteresis state is restored).  Returns the
 * previous value.  Process-wide. */
uint32_t fetode_dopri5_set_spin_limit(uint32_t polls);
int fetode_abi_version(void);

/* Size in bytes of the packed "plan" (pre-transformed parameters). */
int64_t fetode_plan_bytes(const fetode_field_t* field);
/* Build the plan from the parameters; enqueue on stream.  plan: (dev) fetode_plan_bytes bytes. */
int fetode_plan_build(const fetode_field_t* field, void* plan, void* stream);

/* Row length of the compact hysteresis state of `field` (sum of Ferro in_l). */
int32_t fetode_state_width(const fetode_field_t* field);

/* 1 if a fused (single-launch) integrator kernel exists for this field shape. */
int fetode_fused_supported(const fetode_field_t* field);

/* Kernel choice of the fused integrator: batches B <= this value (default 512, env
 * FETODE_SMALL_MAX) take the small-batch kernel (one trajectory per 3-wave workgroup: the
 * strong-scaling shard size), larger ones and every training tape the two-trajectories-per-wave
 * kernel.  Sets the value when b >= 0; returns the previous one.  Process-wide tuning knob. */
int64_t fetode_fused_set_small_batch_max(int64_t b);
/* Inference rk4 batches lo < B <= hi run the v7 kernel at ONE trajectory per wave (each hidden
 * unit's lane group split over both half-waves: half the Ferro rounds per lane — the latency-bound
 * batches of a strong-scaled shard), ahead of the small-batch switch above; training tapes too.
 * Defaults (320, 1024], below the v8 range (env FETODE_TPW1_LO / FETODE_TPW1_HI).  Sets lo / hi when >= 0; returns the
 * previous hi.  Process-wide tuning knob. */
int64_t fetode_fused_set_tpw1_range(int64_t lo, int64_t hi);
/* Inference rk4 batches lo < B <= hi run the v8 kernel: ONE trajectory per TWO-wave workgroup
 * (each wave five hidden units, 12 lanes per unit; one LDS exchange of two partial sums per
 * evaluation; two trajectories per four-wave workgroup) — the 8-way strong-scaled shard, ahead of
 * every other choice above.  Default (256, 512] (env FETODE_V8_LO / FETODE_V8_HI).  Sets lo / hi
 * when >= 0; returns the previous hi. */
int64_t fetode_fused_set_v8_range(int64_t lo, int64_t hi);
/* The current switch points, out[5] = {small_batch_max, tpw1_lo, tpw1_hi, v8_lo, v8_hi} (so a
 * caller can save and restore every knob above). */
int fetode_fused_get_batch_ranges(int64_t* out);

/* One stateful field evaluation out = field(x) — KANFET.forward / KAN.forward.
 * x (B, in0), out (B, out_last), state (B*state_width, layout above) updated in place. */
int fetode_field_forward(const fetode_field_t* field, const void* plan, const float* x, int64_t B,
                         float* state, uint32_t init_mask, float* out, void* stream);

/* Fixed-grid integration in ONE launch (torchdiffeq FixedGridODESolver.integrate).
 *   y0 (B, D) ; step_coef (dev) n_steps x 4 floats per step s, each formed in the time
 *   dtype then rounded to fp32 as torch does for a 0-dim time tensor times an fp32 state:
 *   [dt = grid[s+1]-grid[s], 0.5*dt, dt/6, 0] (0.5*dt: Midpoint / classic rk4; dt/6: classic rk4);
 *   outputs j = 1..T-1: out_step[j] (dev int32) = step after which solution[j] is produced,
 *   out_mode[j] (dev int32) 0: y(step start), 1: y(step end), 2: linear interp with out_slope[j];
 *   solution (T, B, D): row 0 is written from y0.
 *   state/init_mask as in fetode_field_forward (final state written back).
 *   tape (dev, nullable): n_evals * B * (D + H) floats, the inputs of both layers of every field
 *   evaluation (n_evals = n_steps * stages), recorded for fetode_integrate_fixed_backward
 *   (training): rows (n_evals, B, D + H) for the specialised [2, 10, 2] fields; two planes
 *   (n_evals, B, D) then (n_evals, B, H) for the other widths (fieldn).
 * Returns FETODE_EUNSUPPORTED when no fused kernel exists for this field shape. */
int fetode_integrate_fixed(const fetode_field_t* field, const void* plan, int32_t method,
                           const float* y0, int64_t B, const float* step_coef, int32_t n_steps,
                           const int32_t* out_step, const int32_t* out_mode, const float* out_slope,
                           int32_t T, float* solution, float* state, uint32_t init_mask,
                           float* tape, void* stream);

/* One KAN-FET layer at production widths in ONE launch (ETT KANFET[64,128,64], ECG FerroNet):
 *   out = KANLinear(x) + FerroelectricBasis(x)   (layer = KANFETLayer), or either
 *   half alone (layer / ferro NULL) — efficientkan.py:160-182, ferro_class.py:368-420 with the
 *   constant branch_sign and no activations.  Supported: grid_size 5, spline_order 3, 10 logistic
 *   bases; Ferro K = 10 or 12; in >= 16, in % 4 == 0, out % 16 == 0 (fetode_wide_layer_supported).
 *   The plan (fetode_wide_layer_plan_bytes, built once per parameter version) packs the Ferro
 *   constants and the KAN weights for the MFMA contraction.  prev (B, in) is read (ignored when
 *   reinit); the caller stores the new prev_x = x afterwards (ferro_class.py:409).  out must not
 *   alias x.  Replaces: KANFETLayer.forward / KANLinear.forward / FerroelectricBasis.forward. */
int fetode_wide_layer_supported(const fetode_kanlinear_t* layer, const fetode_ferro_t* ferro);
int64_t fetode_wide_layer_plan_bytes(const fetode_kanlinear_t* layer, const fetode_ferro_t* ferro);
int fetode_wide_layer_plan_build(const fetode_kanlinear_t* layer, const fetode_ferro_t* ferro, void* plan,
                                 void* stream);
int fetode_wide_layer_forward(const fetode_kanlinear_t* layer, const fetode_ferro_t* ferro, const void* plan,
                              const float* x, int64_t B, const float* prev, int32_t reinit, float* out,
                              void* stream);

/* The whole dopri5 solve of a two-layer wide KAN-FET field (KANFET([D, H, D]) with both layers
 * fetode_wide_layer_supported, KAN + Ferro, the same K) in ONE launch: the ETT forecaster's latent
 * solve odeint(self.dynamics, z0, t_fut, method="dopri5") (train_kan_fet_ett.py:192, :858, :879; the
 * dynamics' field KANFET([latent, hidden, latent]), BASELINE configs[3]).  A persistent grid walks
 * the wide-layer tiles phase by phase (layer 0 | grid barrier | layer 1 | grid barrier | stage
 * combine) with the host-driven loop's arithmetic: each layer's input slices as
 * fetode_wide_layer_forward picks them, fetode_lincomb's stage sums, fetode_scaled_rms's error ratio
 * (fp64, over the whole batch), _optimal_step_size in fp64, _interp_fit / _interp_evaluate — so the
 * attempts, nfev and solution are the host loop's.  Every evaluation (rejected attempts' too) sees
 * and advances the hysteresis memory (ferro_class.py:409).
 *   plan0 / plan1: fetode_wide_layer_plan_build of each layer (KAN + Ferro); y0 (B, D);
 *   prev0 (B, D) / prev1 (B, H): each layer's prev_x before the solve, unread where reinit_mask bit
 *   0 / 1 is set (first call: prev = x); t (dev, fp64, T) strictly increasing; opts / tableau as
 *   fetode_integrate_dopri5; solution (T, B, D); state0 (B, D) / state1 (B, H) receive the prev_x
 *   after the solve (may alias prev0 / prev1); workspace: fetode_wide_dopri5_workspace(B, D, H) bytes;
 *   stats / attempts as fetode_integrate_dopri5.  Replaces: the host loop of dopri5.py over
 *   KANFETDynamics (two fetode_wide_layer_forward per evaluation, a read-back per attempt). */
int fetode_wide_dopri5(const fetode_kanlinear_t* kan0, const fetode_ferro_t* ferro0, const void* plan0,
                       const fetode_kanlinear_t* kan1, const fetode_ferro_t* ferro1, const void* plan1,
                       const float* y0, int64_t B, const float* prev0, const float* prev1, uint32_t reinit_mask,
                       const double* t, int32_t T, double rtol, double atol, const double* opts,
                       const float* tableau, float* solution, float* state0, float* state1, void* workspace,
                       int32_t* stats, double* attempts, int32_t max_attempts, void* stream);
int64_t fetode_wide_dopri5_workspace(int64_t B, int32_t D, int32_t H);

/* The whole dopri5 solve of a fused-shape field (the LV KAN / KAN-FET [2,10,2] fields) in ONE
 * cooperative launch — torchdiffeq's default method of every reference odeint without `method`
 * (train_kanfet_node_predprey.py:252,260, rtol 1e-7 / atol 1e-9): f0, misc._select_initial_step
 * (unless opts[0] = first_step > 0), 6 evaluations per attempt incl. rejected ones (the hysteresis
 * state sees every call, ferro_class.py:409), the global RMS error norm, accept/reject,
 * _optimal_step_size, _interp_fit/_interp_evaluate at every output time, in the arithmetic of the
 * host-driven path (fetode_lincomb / fetode_scaled_rms / fetode_interp_*).
 *   y0 (B, D); t (dev, fp64, T) strictly increasing; opts / tableau as fetode_ecg_dopri5;
 *   solution (T, B, D); state / init_mask as fetode_field_forward (final state written back);
 *   workspace: fetode_integrate_dopri5_workspace(B) bytes; stats (dev, 3 ints) = nfev, attempts,
 *   status (0 ok, 1 non-finite state, 2 dt underflow, 3 max_num_steps, 4 a grid reduction timed
 *   out); attempts (dev, nullable) (max_attempts, 4) doubles: t0, dt, error ratio, accepted.
 * FETODE_EUNSUPPORTED when the shape has no fused kernel or B needs more workgroups than can be
 * resident at once (B <= 4096 on MI355X); the caller then takes the host-driven loop. */
int fetode_integrate_dopri5(const fetode_field_t* field, const void* plan, const float* y0, int64_t B,
                            const double* t, int32_t T, double rtol, double atol, const double* opts,
                            const float* tableau, float* solution, float* state, uint32_t init_mask,
                            void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                            void* stream);
int64_t fetode_integrate_dopri5_workspace(int64_t B);

/* Training through the resident dopri5 solve (train_kanfet_node_predprey.py:252-257: the
 * reference's loss.backward() through odeint's default dopri5).  _tape: fetode_integrate_dopri5
 * that also records, for the first tape_cap evaluations, the two layer inputs and the output of
 * every evaluation (tape (tape_cap, B, 2 D + H): x, h, k) and the initial-step scalars {d0, d1,
 * d2, h0, h1} (init_rec, 5 doubles).  The caller checks stats[0] (nfev) <= tape_cap and stats[1] <=
 * max_attempts (else re-runs from the same state with larger buffers). */
int fetode_integrate_dopri5_tape(const fetode_field_t* field, const void* plan, const float* y0, int64_t B,
                                 const double* t, int32_t T, double rtol, double atol, const double* opts,
                                 const float* tableau, float* solution, float* state, uint32_t init_mask,
                                 void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                                 float* tape, int64_t tape_cap, double* init_rec, void* stream);

/* Trajectory-sharded device-resident dopri5 (one process per GPU, the global batch split into
 * contiguous shards; SURVEY §8e caveat 2): torchdiffeq's error ratio is an RMS over the WHOLE
 * batch, so every norm of the solve (the two initial-step norms, each attempt's error norm and
 * non-finite flag) is summed over the ranks inside the launch: workgroup 0 of each rank writes its
 * GPU's partial into slot `rank` of every rank's inbox (IPC-mapped device memory, remote stores
 * over xGMI) and sums the world's records in rank order, so all ranks take the same steps as one
 * device would on the global batch.  When every rank's shard is whole leaves of the single-device
 * reduction tree (e.g. equal even shards of 2^k batches) the ranks exchange the leaf sums and the
 * norms are bitwise the single device's: the same attempts, steps and solution.  Replaces the host loop's per-attempt read-back + all-reduce
 * (dist.odeint_sharded, norm_group).  Every rank calls it with the same t / tolerances / options
 * and the same `epoch` (a per-solve counter); B_total = the global batch. */
typedef struct fetode_xrank {
  int32_t rank, world;
  uint32_t epoch;        /* distinct per solve, equal on every rank */
  void* inbox;           /* (dev) this rank's inbox (fetode_xrank_alloc) */
  void* const* peers;    /* (dev) array of `world` inbox pointers as mapped in this process */
  int64_t b_offset;      /* global index of this rank's first trajectory (contiguous shards) */
} fetode_xrank_t;
int fetode_integrate_dopri5_xrank(const fetode_field_t* field, const void* plan, const float* y0, int64_t B,
                                  int64_t B_total, const double* t, int32_t T, double rtol, double atol,
                                  const double* opts, const float* tableau, float* solution, float* state,
                                  uint32_t init_mask, void* workspace, int32_t* stats, double* attempts,
                                  int32_t max_attempts, const fetode_xrank_t* xr, void* stream);
/* inbox bytes for a world; allocate + export (handle: 64 bytes, hipIpcMemHandle_t), open a peer's
 * handle in this process, close / free.  Host calls (synchronous). */
int64_t fetode_xrank_inbox_bytes(int32_t world);
/* The wide KAN-FET field's resident dopri5 over this rank's shard [xr->b_offset, + B) of a
 * trajectory-sharded global batch B_total (the ETT forecaster's solve, train_kan_fet_ett.py:192,
 * sharded 8x: BASELINE configs[3]; dist.odeint_sharded).  Every error norm is the global batch's:
 * the ranks' kernels exchange them through the inboxes (no host round trip); every rank takes the
 * same attempts.  When the shard's rows are whole leaves of the global tile sequence the result is
 * bitwise fetode_wide_dopri5 on the global batch.  Arguments as fetode_wide_dopri5; workspace:
 * fetode_wide_dopri5_xrank_workspace(B, B_total, b_offset, D, H) bytes.  Replaces: the host loop's
 * one all-reduce + read-back per attempt under dist.odeint_sharded. */
int fetode_wide_dopri5_xrank(const fetode_kanlinear_t* kan0, const fetode_ferro_t* ferro0, const void* plan0,
                             const fetode_kanlinear_t* kan1, const fetode_ferro_t* ferro1, const void* plan1,
                             const float* y0, int64_t B, int64_t B_total, const float* prev0, const float* prev1,
                             uint32_t reinit_mask, const double* t, int32_t T, double rtol, double atol,
                             const double* opts, const float* tableau, float* solution, float* state0,
                             float* state1, void* workspace, int32_t* stats, double* attempts,
                             int32_t max_attempts, const fetode_xrank_t* xr, void* stream);
int64_t fetode_wide_dopri5_xrank_workspace(int64_t B, int64_t B_total, int64_t b_offset, int32_t D, int32_t H);
/* the largest batch one resident dopri5 launch takes on this device (sharded = 1: with the exchange
 * workgroup), 0 if the field has no resident kernel.  Host call (occupancy query, cached). */
int64_t fetode_integrate_dopri5_max_batch(const fetode_field_t* field, int32_t sharded);
int fetode_xrank_alloc(int64_t bytes, void** dev_ptr, void* handle);
int fetode_xrank_open(const void* handle, void** dev_ptr);
int fetode_xrank_close(void* dev_ptr);
int fetode_xrank_free(void* dev_ptr);

/* Standalone module kernels (generic widths). */
/* KANLinear.forward (efficientkan.py:160-182): x (B,in) -> out (B,out). */
int fetode_kanlinear_forward(const fetode_kanlinear_t* layer, const float* x, int64_t B, float* out,
                             void* stream);
/* KANLinear.b_splines (efficientkan.py:117-131): x (B,in) -> bases (B,in,grid_size+spline_order). */
int fetode_kanlinear_bsplines(const fetode_kanlinear_t* layer, const float* x, int64_t B,
                              float* bases, void* stream);
/* FerroelectricBasis.forward (ferro_class.py:368-420).  prev (B,in) is read (ignored when
 * reinit != 0, which applies the :373-375 rule dx = 0); after the kernel prev_out (nullable,
 * may alias prev) receives x (:409).  basis (nullable): (B,in,out,K) activations (:417-418).
 * accumulate != 0: out += ferro(x) (a KAN-FET layer adds it to the KANLinear output). */
int fetode_ferro_forward(const fetode_ferro_t* layer, const float* x, int64_t B, const float* prev,
                         int32_t reinit, int32_t accumulate, float* out, float* basis,
                         float* prev_out, void* stream);

/* Stage combines of the per-stage (generic func) path, exact torchdiffeq op order, n elements.
 *   rk4 (3/8, rk_common.rk4_alt_step_func):
 *     stage 1: out = y + (dt*k1)*(1/3)     stage 2: out = y + dt*(k2 - k1*(1/3))
 *     stage 3: out = y + dt*(k1 - k2 + k3) stage 4: out = y + ((k1 + 3*(k2+k3)) + k4)*dt*0.125
 *   rk4_classic stage 4: out = y + dt*(((k1 + 2*k2) + 2*k3) + k4) with dt = fp32(h/6);
 *   any other (method, stage): out = y + dt*k1 (Euler / Midpoint / classic-rk4 stage inputs).
 *   k2..k4 may be NULL when unused. */
int fetode_rk_combine(int32_t method, int32_t stage, const float* y, const float* k1,
                      const float* k2, const float* k3, const float* k4, float dt, float* out,
                      int64_t n, void* stream);

/* out = a*x + b*y  (y nullable -> out = a*x), n elements: adjoints of the stage combines. */
int fetode_axpby(int64_t n, float a, const float* x, float b, const float* y, float* out, void* stream);

/* ---- dopri5 pieces (torchdiffeq Dopri5Solver; train_ecg_kan_fet_nn_ode.py:558-565) ---------
 * k: (m, n) stage derivatives with row stride kstride; c: (host) m <= 8 fp32 coefficients.   */
/* out = (y0 ? y0 : 0) + sum_{j<m} k[j]*c[j]  — rk_common._runge_kutta_step stage inputs/error */
int fetode_lincomb(const float* y0, const float* k, int64_t kstride, const float* c, int32_t m,
                   float* out, int64_t n, void* stream);
/* The stage combine under autograd (dopri5._CombFn, _Dopri5Grad: rk_common._runge_kutta_step's
 * torch.stack(k).matmul(beta * dt) with dt a differentiable device value).  k: host array of m <= 8
 * device pointers (n floats each); c: m DEVICE fp32 coefficients.
 * forward: out = (y0 ? y0 : 0) + ((k0*c0 + k1*c1) + ...), every product and sum rounded in that order.
 * backward: gk[j] = c[j] * g (gk or gk[j] NULL: not written); gc (nullable, device, m floats) =
 * <g, k_j> in fp32, summed in a fixed order (deterministic for a given n); workspace:
 * fetode_comb_workspace(n) bytes when gc is given. */
int fetode_comb_forward(const float* y0, const float* const* k, int32_t m, const float* c, float* out,
                        int64_t n, void* stream);
int fetode_comb_backward(const float* g, const float* const* k, int32_t m, const float* c, float* const* gk,
                         float* gc, void* workspace, int64_t n, void* stream);
int64_t fetode_comb_workspace(int64_t n);
/* out[0] (dev) = sqrt(mean(((a - sub) / (atol + rtol*max(|y0|,|y1|)))^2)) — misc._rms_norm of the
 * scaled error (sub, y1 nullable: _select_initial_step's scale = atol + |y0|*rtol);
 * out[1] = 1 if y0 holds a non-finite value (torchdiffeq's per-step assertion), else 0. */
int fetode_scaled_rms(const float* a, const float* sub, const float* y0, const float* y1,
                      double rtol, double atol, int64_t n, float* out, void* workspace, void* stream);
/* workspace for both norms (zeroed once by the caller, kept zero by the kernel): the sum then runs
 * over up to 512 workgroups with a fixed-order combination (NULL: one workgroup). */
int64_t fetode_scaled_rms_workspace(int64_t n);
/* The same scaled error as fetode_scaled_rms, unreduced across devices: out[0] (dev, fp64) =
 * sum of squares, out[1] = non-finite flag.  A trajectory-sharded dopri5 all-reduces these two
 * words so every rank takes the global-batch RMS norm of torchdiffeq (SURVEY §8e caveat 2). */
int fetode_scaled_sumsq(const float* a, const float* sub, const float* y0, const float* y1,
                        double rtol, double atol, int64_t n, double* out, void* workspace, void* stream);
/* interp._interp_fit: coeffs (5, n) = [e, d, c, b, a]; y_mid = y0 + k . mid_dt (7 host floats). */
int fetode_interp_fit(const float* y0, const float* y1, const float* k, int64_t kstride,
                      const float* mid_dt, float dt, float* coeffs, int64_t n, void* stream);
/* interp._interp_evaluate at fractional position x in [0, 1]. */
int fetode_interp_eval(const float* coeffs, float x, float* out, int64_t n, void* stream);

/* ---- backward (vector-Jacobian products) -------------------------------------------------
 * Gradients of the reference's autograd through KANLinear.forward (efficientkan.py:160-182)
 * and FerroelectricBasis.forward (ferro_class.py:368-420; prev_x is a detached snapshot,
 * :381-382, so it receives no gradient).  Gradient buffers are (dev) pointers shaped like the
 * parameters; NULL members are skipped.  accumulate != 0: grad += result, else grad = result.
 * Parameter gradients are reduced over the batch in a fixed order (no atomics). */
typedef struct fetode_kanlinear_grad {
  float *base_weight, *spline_weight, *spline_scaler, *logistic_a, *logistic_b, *logistic_weight,
      *logistic_scaler;
} fetode_kanlinear_grad_t;

typedef struct fetode_ferro_grad {
  float *k, *Ec, *Ps, *bias, *coef;
} fetode_ferro_grad_t;

/* Workspace bytes needed by fetode_kanlinear_backward when grads != NULL. */
int64_t fetode_kanlinear_backward_workspace(const fetode_kanlinear_t* layer);
/* g (B,out) -> gx (B,in) (nullable) and parameter grads (nullable). */
int fetode_kanlinear_backward(const fetode_kanlinear_t* layer, const float* x, int64_t B, const float* g,
                              float* gx, const fetode_kanlinear_grad_t* grads, void* workspace,
                              int32_t accumulate, void* stream);
/* fetode_kanlinear_backward at production widths (fetode_wide_layer_supported(layer, plan_ferro),
 * out = 64 or 128): with the plan's packed weights Wp (in, 20, out), gphi = g Wp^T and dWp =
 * phi(x)^T g on MFMA, d/dx and the logistic a / b sums from gphi and the feature derivatives, the
 * parameter gradients from dWp by the packing's chain rule; fixed-order reductions.  plan = a
 * wide-layer plan built for (layer, plan_ferro) (plan_ferro = NULL: KANLinear alone).  Replaces the
 * autograd VJP of KANLinear.forward (efficientkan.py:160-182) in the reference's training loops
 * (train_kan_fet_ett.py:333).  g must be 16-byte aligned. */
int64_t fetode_kanlinear_backward_wide_workspace(const fetode_kanlinear_t* layer, const fetode_ferro_t* plan_ferro,
                                                 int64_t B);
int fetode_kanlinear_backward_wide(const fetode_kanlinear_t* layer, const fetode_ferro_t* plan_ferro,
                                   const void* plan, const float* x, int64_t B, const float* g, float* gx,
                                   const fetode_kanlinear_grad_t* grads, int32_t accumulate, void* workspace,
                                   void* stream);
/* prev/reinit exactly as the forward call that is being differentiated used them. */
int fetode_ferro_backward(const fetode_ferro_t* layer, const float* x, int64_t B, const float* prev,
                          int32_t reinit, const float* g, float* gx, const fetode_ferro_grad_t* grads,
                          int32_t accumulate, void* stream);
/* fetode_ferro_backward at production widths (fetode_wide_layer_supported(NULL, layer)): the element
 * evaluations once, d/dx and the five parameter sums from the same pass (packed fp32, the
 * parameter sums held per lane over a row segment), reduced in a fixed order.  plan = a wide-layer
 * plan built for this Ferro layer (alone or inside its KANFET layer: the Ferro part is laid out the
 * same).  Replaces the autograd VJP of FerroelectricBasis.forward (ferro_class.py:368-414; prev_x
 * detached :381-382) that the reference's training loops run (train_kan_fet_ett.py:333). */
int64_t fetode_ferro_backward_wide_workspace(const fetode_ferro_t* layer, int64_t B);
int fetode_ferro_backward_wide(const fetode_ferro_t* layer, const void* plan, const float* x, int64_t B,
                               const float* prev, int32_t reinit, const float* g, float* gx,
                               const fetode_ferro_grad_t* grads, int32_t accumulate, void* workspace,
                               void* stream);

/* ---- reverse sweep of fetode_integrate_fixed (training) -----------------------------------
 * loss.backward() through a fused fixed-grid solve (train_kanfet_node_predprey.py:254-257):
 * reverse-mode through every stage evaluation (efficientkan.py:160-182, ferro_class.py:368-420,
 * detached prev_x :381-382), the stage combines and the output interpolation.
 * 1 if a fused backward exists for this field shape: the specialised [2, 10, 2] sweeps, and for
 * the other depth-2 widths the fieldn sweep (an adjoint kernel + the per-module parameter VJPs over
 * every (evaluation, trajectory) row, fetode_fieldn_bwd.hip). */
int fetode_fused_backward_supported(const fetode_field_t* field);
/* The KAN-FET sweep's structure: 0 = one kernel (adjoints and parameter-gradient sums together,
 * the default), 1 = split (an adjoint sweep that records every evaluation's adjoints, then the
 * parameter sums of each layer in parallel over the samples).  Same results up to fp32 summation
 * order.  Returns the previous setting; enable < 0 only queries.  Call before sizing workspaces. */
int fetode_backward_set_split(int32_t enable);
/* The [2, 10, 2] KAN-FET sweep on the forward's lane groups (sweep7_kernel: the adjoints and every
 * parameter-gradient sum in one launch):
 * 0 = off (the one-kernel sweep), 1 = where the one-kernel sweep would run two trajectories per wave
 * (the default), 2 = at every batch; + 4 = the sweep keeps the Ferro sums only and a second launch
 * forms the KAN sums over every recorded (evaluation, trajectory) sample.  Same results up to fp32
 * summation order.  Returns the previous setting; mode < 0 only queries.  Call before sizing
 * workspaces. */
int fetode_backward_set_v7(int32_t mode);
/* Workspace bytes for fetode_integrate_fixed_backward of a (method, n_steps) forward at batch B
 * (the split path records every evaluation's adjoints: n_evals * B * (D + H) floats of it). */
int64_t fetode_integrate_fixed_backward_workspace(const fetode_field_t* field, int32_t method, int32_t n_steps,
                                                  int64_t B);
/* The schedule arguments are the forward's.  grad_solution (T, B, D) = d loss / d solution;
 * tape = the forward's tape; state0 (B*state_width) = the hysteresis state BEFORE the forward
 * solve (nullable when every init_mask bit is set), init_mask = the forward's.
 * Outputs: grad_y0 (B, D) (nullable) and the parameter gradients, written (not accumulated):
 * kan_grads / ferro_grads are (host) arrays of n_layers descriptors of (dev) buffers shaped like
 * the parameters (NULL members skipped; ferro_grads NULL for KAN fields).  Gradient sums are
 * reduced over the batch in a fixed order (fp64): results are run-to-run identical. */
int fetode_integrate_fixed_backward(const fetode_field_t* field, const void* plan, int32_t method, int64_t B,
                                    const float* step_coef, int32_t n_steps, const int32_t* out_step,
                                    const int32_t* out_mode, const float* out_slope, int32_t T,
                                    const float* grad_solution, const float* tape, const float* state0,
                                    uint32_t init_mask, float* grad_y0, const fetode_kanlinear_grad_t* kan_grads,
                                    const fetode_ferro_grad_t* ferro_grads, void* workspace, void* stream);

/* The reverse sweep of a taped solve, ONE resident launch (+ the fixed-order parameter-sum
 * reduction): reverse-mode autograd through every evaluation (rejected attempts included), the
 * stage sums, the interpolant, the error norm and the step-size control (rk_common._runge_kutta_step,
 * _optimal_step_size, misc._select_initial_step, interp._interp_fit / _interp_evaluate — torchdiffeq
 * detaches none of them), one grid-wide sum per attempt for the batch-coupled adjoint of dt.
 *   t / T / rtol / atol / opts / tableau: those of the forward; grad_solution (T, B, D); tape /
 *   attempts / init_rec: the forward's records, n_ev = stats[0], n_att = stats[1];
 *   state0 / init_mask: the hysteresis state before the solve; grad_y0 (B, D) nullable; the
 *   gradients as fetode_integrate_fixed_backward (overwritten); status (dev, 1 int): 0, or 4 when a
 *   grid sum timed out (not co-resident).
 * Replaces: dopri5.py _Dopri5Grad (host-driven autograd through every stage of every attempt).
 * FETODE_EUNSUPPORTED beyond fetode_integrate_dopri5_backward_max_batch. */
int fetode_integrate_dopri5_backward(const fetode_field_t* field, const void* plan, int64_t B, const double* t,
                                     int32_t T, double rtol, double atol, const double* opts, const float* tableau,
                                     const float* grad_solution, const float* tape, int32_t n_ev,
                                     const double* attempts, int32_t n_att, const double* init_rec,
                                     const float* state0, uint32_t init_mask, float* grad_y0,
                                     const fetode_kanlinear_grad_t* kan_grads, const fetode_ferro_grad_t* ferro_grads,
                                     void* workspace, int32_t* status, void* stream);
int64_t fetode_integrate_dopri5_backward_workspace(const fetode_field_t* field, int64_t B);
/* The workspace of a solve with n_ev evaluations: the other depth-2 widths' sweep (fieldn) records
 * every evaluation's adjoints and layer inputs for its row-batched parameter VJPs, so its workspace
 * grows with n_ev; for the [2, 10, 2] fields the same as fetode_integrate_dopri5_backward_workspace. */
int64_t fetode_integrate_dopri5_backward_workspace_ev(const fetode_field_t* field, int64_t B, int32_t n_ev);
int64_t fetode_integrate_dopri5_backward_max_batch(const fetode_field_t* field);

/* ---- ECG KAN-FET NODE field (BASELINE configs[2]) -----------------------
 * The hysteretic LogisticBasis of train_ecg_kan_fet_nn_ode.py:54-133 (hard branch switch:
 * branch_state = sigmoid(gate_slope (x - prev_x)) > breaking_point; prev_x remembers the LAST
 * batch row of the previous call, :131-132).  (dev) pointers. */
typedef struct fetode_hlogistic {
  int32_t in_dim, num_basis;
  const float *k, *Ec, *Ps, *bias;  /* (in, nb) :84-88 (coef :88 is unused by forward) */
  double gate_slope, breaking_point; /* :71,74 defaults 5.0, 0.5 */
} fetode_hlogistic_t;

/* KANFeatureMixer (:408-421): phi = act(basis(x)) flattened (B, in*nb), act = sigmoid when
 * act_sigmoid != 0 else identity; with w != NULL also the Linear head of No_MLP_KANODEFunc
 * (:483-509): out = phi w^T + bias, w (n_out, in*nb), bias (n_out) nullable.
 * x (B, in); prev (in*nb) = prev_x as read by this call; phi (B, in*nb) nullable when w != NULL;
 * branch (B, in*nb) nullable = the rebound branch_state buffer (:119); prev_out (in*nb) nullable
 * receives x[B-1] broadcast over the bases, written by a second launch on the same stream (may
 * alias prev). */
int fetode_hlogistic_mixer_forward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                   int32_t act_sigmoid, const float* w, const float* bias, int32_t n_out,
                                   float* phi, float* out, float* branch, float* prev_out, void* stream);
/* Workspace bytes of fetode_hlogistic_mixer_backward (the head's input gradient). */
int64_t fetode_hlogistic_mixer_backward_workspace(const fetode_hlogistic_t* layer, int64_t B);
/* VJP of the mixer (+ head).  x, prev, phi, w: as in (and produced by) the forward being
 * differentiated; g (B, n_out) with a head, else (B, in*nb).  Outputs (nullable, written):
 * gx (B, in), gw (n_out, in*nb), gbias_head (n_out), gk/gEc/gPs/gbias (in, nb).  Batch reductions
 * in a fixed order (no atomics). */
int fetode_hlogistic_mixer_backward(const fetode_hlogistic_t* layer, const float* x, int64_t B, const float* prev,
                                    int32_t act_sigmoid, const float* phi, const float* w, int32_t n_out,
                                    const float* g, float* gx, float* gw, float* gbias_head, float* gk, float* gEc,
                                    float* gPs, float* gbias, void* workspace, void* stream);

/* The whole dopri5 solve of dh/dt = No_MLP_KANODEFunc(h) (train_ecg_kan_fet_nn_ode.py:558-565 with
 * the field :483-509) in ONE cooperative launch: f0, misc._select_initial_step (unless
 * opts[0] = first_step > 0), 6 evaluations per attempt incl. rejected ones (the hysteresis memory
 * sees every call, :131-132), the global RMS error norm, accept/reject, _optimal_step_size,
 * _interp_fit/_interp_evaluate at every output time — the arithmetic of the host-driven path
 * (fetode_lincomb / fetode_scaled_rms / fetode_interp_*) on the device.
 *   layer/wT (in*nb, D) transposed head weight /bias (D, nullable), D = in_dim <= 64;
 *   prev (in*nb) prev_x before the solve; y0 (B, D); t (dev, fp64, T) strictly increasing;
 *   opts (host, 7 doubles): first_step (<= 0: select), safety, ifactor, dfactor, min_step,
 *   max_step, max_num_steps; tableau (host, 50 floats): beta[6][6], c_err[7], c_mid[7] in fp32;
 *   solution (T, B, D); prev_out (in*nb, may alias prev: prev is read before the first
 *   evaluation, prev_out written after the last) = prev_x after the solve;
 *   branch_out (B, in*nb, nullable) = branch_state of the last evaluation;
 *   workspace: fetode_ecg_dopri5_workspace(B) bytes; stats (dev, 3 ints) = nfev, attempts,
 *   status (0 ok, 1 non-finite state, 2 dt underflow, 3 max_num_steps, 4 a grid barrier timed
 *   out: the grid was not co-resident and the outputs are invalid);
 *   attempts (dev, nullable) (max_attempts, 4) doubles: t0, dt, error ratio, accepted.
 * FETODE_EUNSUPPORTED when B or in*nb need more than one co-resident grid (B > 7 * 256 at
 * in*nb = 640 on MI355X: 3 rows + a shadow row per 512-thread workgroup up to B = 768, 7 + 1
 * beyond); the caller then takes the host-driven loop. */
int fetode_ecg_dopri5(const fetode_hlogistic_t* layer, const float* wT, const float* bias, int32_t D,
                      const float* prev, const float* y0, int64_t B, const double* t, int32_t T, double rtol,
                      double atol, const double* opts, const float* tableau, float* solution, float* prev_out,
                      float* branch_out, void* workspace, int32_t* stats, double* attempts, int32_t max_attempts,
                      void* stream);
int64_t fetode_ecg_dopri5_workspace(int64_t B);

/* Elementwise stages of the ECG FerroElectricNet field KANFetODEFunc (train_ecg.py:986-1013; the
 * two FerroelectricBasis layers are fetode_ferro_forward / _backward), in torch's op order:
 *   fetode_tanh_bound: out = h_bound * tanh(x / h_bound) (:1002); t_out (nullable) keeps the tanh
 *   for the backward, gx = ((g * h_bound) * (1 - t^2)) / h_bound;
 *   fetode_tanh: nn.Tanh between the layers (:1004), gx = g * (1 - y^2);
 *   fetode_nan_clamp: clamp(nan_to_num(x, nan, posinf, neginf), lo, hi) (:1008-1011),
 *   gx = g where x is finite and lo <= nan_to_num(x) <= hi, else 0. */
int fetode_tanh_bound(int64_t n, float h_bound, const float* x, float* out, float* t_out, void* stream);
int fetode_tanh_bound_backward(int64_t n, float h_bound, const float* g, const float* t, float* gx, void* stream);
int fetode_tanh(int64_t n, const float* x, float* out, void* stream);
int fetode_tanh_backward(int64_t n, const float* g, const float* y, float* gx, void* stream);
int fetode_nan_clamp(int64_t n, float nan, float posinf, float neginf, float lo, float hi, const float* x, float* out,
                     void* stream);
int fetode_nan_clamp_backward(int64_t n, float nan, float posinf, float neginf, float lo, float hi, const float* g,
                              const float* x, float* gx, void* stream);

/* Kuramoto2D.forward (mnist_kuramoto_kan.py:179-199): x (B, H*W) pixels in [0, 1] -> feat (B, 2*H*W)
 * = [cos(theta) | sin(theta)] after `steps` Euler steps of theta += dt (omega + K coupling);
 * K (1 float) and omega (H*W) are device pointers; H*W <= 3072.  tape (nullable,
 * (B, steps + 1, H*W)) records theta_0..theta_steps for the backward.
 * fetode_kuramoto_backward: from the tape and gfeat (B, 2*H*W), gx (nullable, (B, H*W)), gK
 * (nullable, 1 float) and gomega (nullable, H*W), reduced over the batch in a fixed order;
 * workspace: fetode_kuramoto_backward_workspace(B, H, W) bytes when gK or gomega is wanted. */
int fetode_kuramoto_forward(const float* x, int64_t B, int32_t H, int32_t W, int32_t steps, float dt, const float* K,
                            const float* omega, float* feat, float* tape, void* stream);
int64_t fetode_kuramoto_backward_workspace(int64_t B, int32_t H, int32_t W);
/* 1: the workgroup-per-image LDS kernels for every shape (else lane-per-column register kernels for
 * W, H <= 32); -1 queries.  Returns the previous setting.  A/B and cross-check knob. */
int fetode_kuramoto_set_lds(int on);
int fetode_kuramoto_backward(int64_t B, int32_t H, int32_t W, int32_t steps, float dt, const float* K,
                             const float* tape, const float* gfeat, float* gx, float* gK, float* gomega,
                             void* workspace, void* stream);

/* Wide KANLinear forward on MFMA (the MNIST head, mnist_kuramoto_kan.py:127-142, KANLinear(1568 -> 10)):
 * out (B, out) = SiLU / B-spline / logistic features of each input contracted with the weights on
 * v_mfma_f32_16x16x4_f32, + bias (nullable: the MNIST logistic_bias).  Supported: grid_size 5,
 * spline_order 3, num_logistic 0 or 8, out <= 16, in % 4 == 0 (fetode_kanlinear_wide_supported);
 * otherwise FETODE_EUNSUPPORTED (fetode_kanlinear_forward serves every shape).  wpack
 * (fetode_kanlinear_wide_pack_bytes) holds the weights in the MFMA layout, filled by
 * fetode_kanlinear_wide_pack (re-pack after a weight update); workspace:
 * fetode_kanlinear_wide_workspace(layer, B) bytes. */
int fetode_kanlinear_wide_supported(const fetode_kanlinear_t* layer);
int64_t fetode_kanlinear_wide_pack_bytes(const fetode_kanlinear_t* layer);
int fetode_kanlinear_wide_pack(const fetode_kanlinear_t* layer, float* wpack, void* stream);
int64_t fetode_kanlinear_wide_workspace(const fetode_kanlinear_t* layer, int64_t B);
int fetode_kanlinear_wide_forward(const fetode_kanlinear_t* layer, const float* wpack, const float* bias, const float* x,
                                  int64_t B, float* out, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------------
 * ETT KAN-RNN encoder (train_kan_fet_ett.py:741-818; the encoder of
 * KAN_FET_LatentODE_DiffusionForecaster, :822-837).  One cell step (FullyNonlinearKANCell.forward,
 * :790-795) is h_t = sigmoid(cat(phi_x(x_t), phi_h(h_{t-1})))[:, :H] with
 * phi(v)[i, k] = 2 / (1 + exp(-a[i,k] (v[i] - b[i,k]))) (LogisticBasis.forward, :747-749);
 * KANRNNEncoder.forward (:809-818) runs the cell over the context from h = 0 and projects
 * z0 = to_latent(h_T).  (dev) pointers: ax, bx (F, nb); ah, bh (H, nb); w (latent, H); bias (latent).
 * -------------------------------------------------------------------------------------------- */
typedef struct fetode_kanrnn {
  int32_t num_features, hidden, num_basis, latent; /* latent = 0: no projection */
  const float *ax, *bx, *ah, *bh;                  /* rnn_cell.{input,hidden}_basis.{a,b} */
  const float *w, *bias;                           /* to_latent.weight / .bias (NULL if latent = 0) */
} fetode_kanrnn_t;

/* h_T of the recurrence over x (B, T, F) from h0 (B, H) (NULL = zeros) in ONE launch, h on chip.
 * h_out (B, H) (nullable), z0 (B, latent) = to_latent(h_T) (nullable; needs latent*H <= 16384).
 * tape (B, T, H) (nullable): every h_t, for fetode_kanrnn_backward; a tape forces the full
 * recurrence.  full = 0 evaluates only the steps whose outputs can reach h_T: column j of h_t reads
 * h_{t-1} only through column (j - F nb) / nb (the truncated cat), so every dependency chain is at
 * most depth(H, F, nb) steps long (exact, NaN included).  H <= 256, F <= 64. */
int fetode_kanrnn_forward(const fetode_kanrnn_t* m, const float* x, int64_t B, int32_t T, const float* h0,
                          float* h_out, float* z0, float* tape, int32_t full, void* stream);
/* the number of steps before h_T that can influence it (the cone depth) */
int32_t fetode_kanrnn_depth(int32_t num_features, int32_t hidden, int32_t num_basis);
/* VJP of the recurrence with the reference autograd's IEEE semantics (a dropped column's zero
 * gradient times an overflowing exp is NaN, as torch computes it).  g_h (B, H) = d loss / d h_T;
 * tape from fetode_kanrnn_forward; outputs (nullable): g_x (B, T, F), g_h0 (B, H), and the parameter
 * gradients g_ax, g_bx (F, nb), g_ah, g_bh (H, nb) (overwritten, reduced in a fixed order: run-to-run
 * identical).  workspace: fetode_kanrnn_backward_workspace(m, B) bytes. */
int64_t fetode_kanrnn_backward_workspace(const fetode_kanrnn_t* m, int64_t B);
int fetode_kanrnn_backward(const fetode_kanrnn_t* m, const float* x, int64_t B, int32_t T, const float* h0,
                           const float* tape, const float* g_h, float* g_x, float* g_h0, float* g_ax, float* g_bx,
                           float* g_ah, float* g_bh, void* workspace, void* stream);
/* LogisticBasis.forward (:747-749) alone: x (B, in) -> phi (B, in, nb), and its VJP
 * (g_x (B, in), g_a, g_b (in, nb); nullable; g_a / g_b reduced over the batch in a fixed order;
 * workspace fetode_logistic_basis_backward_workspace(in, nb, B) bytes). */
int fetode_logistic_basis_forward(const float* x, int64_t B, int32_t in, int32_t nb, const float* a, const float* b,
                                  float* phi, void* stream);
int64_t fetode_logistic_basis_backward_workspace(int32_t in, int32_t nb, int64_t B);
int fetode_logistic_basis_backward(const float* x, int64_t B, int32_t in, int32_t nb, const float* a,
                                   const float* b, const float* g_phi, float* g_x, float* g_a, float* g_b,
                                   void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FETODE_H_ */
