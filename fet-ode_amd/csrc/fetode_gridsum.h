// fetode_gridsum.h — the device-resident dopri5 solvers' control parameters and their grid-wide
// fixed-order fp64 reduction (shared by the forward solve, fetode_fused.hip, and its reverse
// sweep, fetode_bwd.hip).  Device code only; included inside each file's anonymous namespace.
#pragma once
// Device-resident dopri5 (torchdiffeq Dopri5Solver, the default method of every reference odeint
// without `method`, train_kanfet_node_predprey.py:252): the control arithmetic of the host-driven
// path (fet-ode_amd/dopri5.py _Dopri5 with fetode_lincomb / fetode_scaled_rms / fetode_interp_*).
struct DopriParams {
  int32_t on;
  const double* t;  // (T) output times, fp64, strictly increasing
  int32_t T;
  float rtol, atol;
  double first_step, safety, ifactor, dfactor, min_step, max_step;
  int32_t max_steps;
  // tableau in fp32 (RKAdaptiveStepsizeODESolver casts it to y0's dtype), by stage column j:
  // stc[j][q] = beta[j + q][j] (q < 6, 0 past the tableau), stc[j][6] = c_error[j], stc[j][7] = c_mid[j]
  float stc[7][8];
  unsigned* bar;    // grid-reduction words (zeroed before the launch)
  double* slot;     // (grid, 2) per-workgroup partial sums
  double* xs;       // (2, kDpGroups, 2) leaf sums, double-buffered by round parity
  int32_t* stats;   // nfev, attempts, status
  double* att;      // (max_att, 4): t0, dt, error ratio, accepted
  int32_t max_att;
  // trajectory-sharded solve (fetode_integrate_dopri5_xrank): every norm is the sum over all ranks
  double n_total;              // global element count of the norms (B_global * D)
  int32_t xr_rank, xr_world;   // xr_world <= 1: single device
  uint32_t xr_epoch;           // per-solve tag (the same on every rank)
  double* const* xr_peers;     // (dev) xr_world inbox base pointers as mapped here (peers[rank] = own)
  double* xr_inbox;            // (dev) own inbox: (2, world) records {v0, v1, tag, pad}
  double* xr_g;                // (2, 2) the global sums of the round, double-buffered by parity
  // leaves of the grid reduction: contiguous runs of leaf_len workgroups in GLOBAL workgroup numbers
  // (this grid's workgroup b is global workgroup wg_off + b); this grid owns leaves
  // [leaf_lo, leaf_lo + n_leaf_local) of n_leaf_global.  xr_exact: every rank owns whole leaves of
  // the single-device grid, so the rank-summed result is bitwise the single device's
  int32_t leaf_shift, wg_off, leaf_lo, n_leaf_local, n_leaf_global, nblk_global, xr_exact;  // leaf_len = 1 << leaf_shift
  // training (fetode_integrate_dopri5_tape): FusedArgs::tape rows (tape_cap, B, 2 D + H) hold the
  // two layer inputs and the output of the first tape_cap evaluations; the initial-step scalars
  int64_t tape_cap;
  double* init_rec;    // {d0, d1, d2, h0, h1} of _select_initial_step, or null
  // polls before a spin gives up (status 4); 0 = kDpSpinLimit / kXrSpinLimit.  A test knob
  // (fetode_dopri5_set_spin_limit): a tiny limit forces the timeout path on a healthy grid
  uint32_t spin_limit;
};

// the smallest power-of-two leaf length that needs <= kDpGroups leaves over nb workgroups
inline int dp_leaf_shift(int64_t nb);
// leaves of n workgroups from a block boundary: full blocks of 8 leaves, then the last block's
// leaves that have at least one workgroup (a prefix of its 8)
inline int64_t dp_n_leaves(int64_t n, int sh) {
  const int64_t blk = (int64_t)8 << sh, nbk = (n + blk - 1) / blk;
  return nbk == 0 ? 0 : 8 * (nbk - 1) + ((n - (nbk - 1) * blk) < 8 ? (n - (nbk - 1) * blk) : 8);
}

// Grid-wide sum of two fp64 values, one per workgroup (valid on every lane of a one-wave
// workgroup), returned to every workgroup in the same fixed summation order.  Round r:
//   1. each workgroup stores its partial and arrives on one of kDpGroups leaf counters
//      (blockIdx % kDpGroups, ~32 arrivals each at the 2048-workgroup grid: same-address atomics
//      serialise at the memory side, ~25 ns each);
//   2. the leaf's last arriver sums its leaf's partials (lane per partial, xor tree), stores the
//      leaf sum in the round's buffer (r & 1) and bumps the monotonic top counter (kDpTopCopies
//      replicas, one lane each);
//   3. every workgroup polls its replica of the top counter until all leaves of round r have arrived, then sums
//      the kDpGroups leaf sums itself (lane per leaf, xor tree: the same order everywhere).
// Round r + 2 may overwrite buffer r & 1 only after every workgroup has arrived at round r + 1,
// i.e. after it finished reading round r.  dp_order() between dependent steps.  Every spin is
// bounded: after ~1 s the abort word is raised and every later reduction returns at once (the
// grid was not co-resident); the caller reports status 4.
constexpr unsigned kDpSpinLimit = 1u << 20;
constexpr int kDpGroups = 64;
constexpr int kDpLine = 64;  // words per counter line
constexpr int kDpTopCopies = 8;  // replicas of the top counter: ~256 pollers per address, not 2048
constexpr int kDpBarWords = kDpLine * (kDpGroups + 2 + 2 * kDpTopCopies);
inline int dp_leaf_shift(int64_t nb) {
  int sh = 0;
  while ((int64_t)kDpGroups << sh < nb) ++sh;
  return sh;
}
// single-device leaf layout of a grid of `grid` workgroups
inline void dp_single_device(DopriParams& P, int64_t grid) {
  P.xr_world = 1;
  P.xr_exact = 0;
  P.wg_off = 0;
  P.nblk_global = (int32_t)grid;
  P.leaf_shift = dp_leaf_shift(grid);
  P.leaf_lo = 0;
  P.n_leaf_local = P.n_leaf_global = (int32_t)dp_n_leaves(grid, P.leaf_shift);
}
// replicas of the cross-rank "global sum ready" counter (after the top-counter replicas)
__device__ __forceinline__ unsigned* dp_ready(const DopriParams& P, unsigned c) {
  return P.bar + kDpLine * (kDpGroups + 2 + kDpTopCopies + c);
}
constexpr unsigned kXrSpinLimit = 1u << 24;   // cross-rank polls: ranks may start seconds apart
__device__ __forceinline__ unsigned* dp_cnt(const DopriParams& P, unsigned x) { return P.bar + kDpLine * x; }
__device__ __forceinline__ unsigned* dp_top(const DopriParams& P, unsigned c) {
  return P.bar + kDpLine * (kDpGroups + 2 + c);
}
__device__ __forceinline__ unsigned* dp_abort(const DopriParams& P) { return P.bar + kDpLine * (kDpGroups + 1); }

// Ordering between the reduction's atomics.  Every word the reduction shares between workgroups
// (partials, leaf sums, counters) is accessed only through agent-scope atomics, which are coherent
// across the XCDs' L2s by themselves (sc1 loads / stores); what the protocol needs is only that a
// store has landed before the arrival that publishes it, and that the reads after an arrival or a
// poll start after it — a wait on the vector memory counter.  An agent-scope fence (or an
// acquire / release atomic) would ALSO write back and invalidate the XCD's whole L2
// (buffer_wbl2 / buffer_inv sc1) for plain loads and stores this protocol never shares: with 2048
// workgroups arriving that cost ~50 us per reduction and evicted the field's parameters from L2.
__device__ __forceinline__ void dp_order() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One 16-byte {v0, v1} record per write-through (sc1) store / load: the hand-off forms of
// MI355X_MICROARCH.md's table (16-B sc1 payload, vmcnt(0), then the counter add; loads only after
// the add returned / the poll matched).  The load waits inside the asm (invisible to the compiler).
typedef unsigned dp_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void dp_st16(double* p, double v0, double v1) {
  const unsigned long long a = __double_as_longlong(v0), b = __double_as_longlong(v1);
  const dp_u32x4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void dp_ld16(const double* p, double& v0, double& v1) {
  dp_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  v0 = __longlong_as_double(((unsigned long long)v.y << 32) | v.x);
  v1 = __longlong_as_double(((unsigned long long)v.w << 32) | v.z);
}

__device__ __forceinline__ double xor_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ inline bool grid_sum2(const DopriParams& P, unsigned& round, double v0, double v1, double& s0, double& s1) {
#ifdef FETODE_EXP_NO_GRIDSUM  // diagnostics only: per-workgroup control, no synchronisation
  s0 = v0 * gridDim.x;
  s1 = v1 * gridDim.x;
  return false;
#endif
  const bool xr = P.xr_world > 1;   // the last workgroup is the cross-rank exchange (xrank_comm)
  const unsigned blk = blockIdx.x, nblk = gridDim.x - (xr ? 1u : 0u);
  if (nblk == 1u && !xr) {  // one workgroup: the sums below would return v0, v1 exactly
    s0 = v0;
    s1 = v1;
    return false;
  }
  // leaves in GLOBAL workgroup numbers: blocks of 8 L consecutive workgroups, each split by
  // workgroup % 8 into 8 leaves of L — a leaf's workgroups all run on one XCD (workgroups are dealt
  // to the 8 XCDs round-robin; rank offsets are multiples of 8 L), so its partials and counter stay
  // in that XCD's L2, and a block is whole on one rank in a sharded solve
  const unsigned sh = (unsigned)P.leaf_shift, L = 1u << sh, gb = blk + (unsigned)P.wg_off;
  const unsigned x = ((gb >> (sh + 3u)) << 3u) | (gb & 7u);
  const unsigned first = ((x >> 3u) << (sh + 3u)) + (x & 7u);
  const unsigned nx = min(L, ((unsigned)P.nblk_global - first + 7u) >> 3u);
  const unsigned ngrp = (unsigned)P.n_leaf_local;
  const unsigned r = round++;
  double* xs = P.xs + 2 * kDpGroups * (r & 1u);
  unsigned* abw = dp_abort(P);
  const int lane = threadIdx.x & 63;
  int ab = 0, leader = 0;
  if (lane == 0) {
    ab = __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    dp_st16(&P.slot[2 * blk], v0, v1);
    dp_order();
    if (!ab)
      leader = __hip_atomic_fetch_add(dp_cnt(P, x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nx * (r + 1u) - 1u;
  }
  ab = __shfl(ab, 0);
  leader = __shfl(leader, 0);
  if (!ab && leader) {
    dp_order();
    double a0 = 0.0, a1 = 0.0;
    for (unsigned j = lane; j < nx; j += 64) {
      double u0, u1;
      dp_ld16(&P.slot[2 * (first + (j << 3u) - (unsigned)P.wg_off)], u0, u1);
      a0 += u0;
      a1 += u1;
    }
    a0 = xor_sum64(a0);
    a1 = xor_sum64(a1);
    if (lane == 0) dp_st16(&xs[2 * x], a0, a1);
    dp_order();
    if (lane < kDpTopCopies) __hip_atomic_fetch_add(dp_top(P, lane), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0 && !ab) {
    // single device: all leaves of round r; sharded: the exchange workgroup's rank sum of round r
    const unsigned want = xr ? r + 1u : ngrp * (r + 1u);
    unsigned spins = 0;
    // wrap-safe: (int)(top - want) < 0 while fewer than `want` leaf arrivals have landed
    unsigned* top = xr ? dp_ready(P, blk % kDpTopCopies) : dp_top(P, blk % kDpTopCopies);
    while ((int)(__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((spins & 15u) == 15u && __hip_atomic_load(abw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        ab = 1;
        break;
      }
      if (++spins == (P.spin_limit ? P.spin_limit : (xr ? kXrSpinLimit : kDpSpinLimit))) {
        __hip_atomic_store(abw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab = 1;
        break;
      }
    }
    dp_order();
  }
  ab = __shfl(ab, 0);
  if (xr) {
    if (!ab) dp_ld16(P.xr_g + 2 * (r & 1u), s0, s1);
    return ab != 0;
  }
  double u0 = 0.0, u1 = 0.0;
  if ((unsigned)lane < ngrp && !ab) dp_ld16(&xs[2 * lane], u0, u1);   // one device: leaves 0 .. ngrp-1
  s0 = xor_sum64(u0);
  s1 = xor_sum64(u1);
  return ab != 0;
}
