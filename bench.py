"""Benchmark: RK4 steps/s of the batch-4096, 2-state Lotka-Volterra KAN-FET Neural ODE.

Workload (BASELINE.json configs[1]): KANFET([2,10,2], grid_size=5, K=10) as the
vector field (train_kanfet_node_predprey.py:146), torch.manual_seed(0) weights, y0 = 0.5 +
2.5*U[0,1)^(4096x2), t = linspace(0, 3.5, 35) float64 (t_learn, :155), method='rk4' (torchdiffeq
3/8 rule).  One bench "step" = one odeint solve = 34 RK4 steps of the batch, inputs resident in HBM.

Scaling: the path partitions by trajectory with no data-path collective.  The contract line is
STRONG scaling (--scaling strong, default; SURVEY §8d "strong (global 4096) is primary"): the
global seed-0 batch of 4096 cut into contiguous per-rank blocks (fet_ode_amd.dist.shard_bounds),
value = RK4 steps/s of that ONE job.  At N > 1 the same run also times WEAK scaling (every rank
solves its own batch of 4096, seed = rank; value summed over the ranks) and reports it as
`weak_scaling`; --scaling weak makes that the contract value instead.

Launch: python bench.py [--gpus N --steps K --warmup W]; N>1 via torch.distributed.run.
Prints ONE JSON line on rank 0.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from fet_ode_amd.autograd_ops import build_plan, make_handle, pack_state  # noqa: E402
from fet_ode_amd.odeint import get_schedule  # noqa: E402

B = 4096
T = 35
STEPS_PER_SOLVE = T - 1
METRIC = "RK4 steps/sec, batch-4096 2-state LV KAN-FET NODE @1/2/4/8 GPU; traj MSE vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector (= f32 MFMA) peak
PARAM_FLOATS = 3052 + 144      # trainable params + grid buffers of KANFET [2,10,2]
STATE_IN = 2 + 10              # sum of Ferro in_l


_T_START = time.perf_counter()


def progress(msg):
    """One line per bench leg on stderr (the JSON line stays the only stdout line): a long leg is
    visibly alive (the GPU harness kills a command that writes nothing for minutes)."""
    print(f"[bench +{time.perf_counter() - _T_START:6.1f}s] {msg}", file=sys.stderr, flush=True)


def alg_bytes_per_step(b):
    """y read+write (16 B) + compact prev_x r/w per Ferro layer (8*sum in_l) per
    trajectory, + parameters once:  112*B + 12784."""
    return b * (16 + 8 * STATE_IN) + 4 * PARAM_FLOATS


ALG_FLOPS_PER_TRAJ_STEP = 50_000   # ~50k flops (+5.8k transcendentals) per RK4 step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the GPU's clocks settle within ~100 back-to-back solves (the first 100 average 181 us,
    # every later block of 100 170.0-170.7 us: tools/diag/clock_ramp.py, profiles/r05_clock_ramp.log),
    # so 200 untimed solves (~35 ms) precede 500 timed ones (~85 ms)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--settle-s", type=float, default=0.25,
                    help="before the W warm-up solves: back-to-back solves for this many seconds so the GPU's "
                         "clocks reach their loaded state (DESIGN.md §3; 0 disables)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: global batch 4096 split over the ranks (the contract line); "
                         "weak: 4096 trajectories per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dopri5", action="store_true", help="skip the LV dopri5 (torchdiffeq defaults) line")
    ap.add_argument("--no-ecg", action="store_true", help="skip the ECG dopri5 (configs[2]) line")
    ap.add_argument("--no-mnist", action="store_true", help="skip the MNIST Kuramoto + KANLinear line")
    ap.add_argument("--no-ett", action="store_true", help="skip the ETT KAN-FET latent-ODE forecaster line")
    ap.add_argument("--ett-batch", type=int, default=8192)
    ap.add_argument("--ett-ref-iters", type=int, default=1,
                    help="iterations of the reference's own ETT training step (rtol 1e-7, ~1 min each); 0 skips")
    ap.add_argument("--cpu-solves", type=int, default=5, help="CPU baseline: median over this many solves")
    ap.add_argument("--train-iters", type=int, default=50, help="0 skips the training-rate line")
    return ap.parse_args()


def make_problem(rank, world, scaling, dev):
    """Seed-0 weights on every rank; y0: strong = this rank's block of the seed-0 global batch,
    weak = a full batch of its own (seed = rank)."""
    import fet_ode_amd.dist as D
    torch.manual_seed(0)
    model = F.KANFET([2, 10, 2], grid_size=5)
    if world > 1:   # one model for the job: the efficient_kan init is not reproducible across processes
        D.broadcast_parameters(model)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev)
    if scaling == "strong":
        y0g = lv_y0(B, 0)
        lo, hi = D.shard_bounds(B, rank, world)
        y0 = y0g[lo:hi].clone()
    else:
        y0g = y0 = lv_y0(B, rank)
    t = torch.tensor(np.linspace(0, 3.5, T))
    return model, sd, y0, y0g, t


def lv_y0(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (0.5 + 2.5 * torch.rand(n, 2, generator=g)).to(torch.float32)


def kernel_time_ms(model, y0d, t, reps=20):
    """Average duration of the fused integrate launch alone (HIP events on its stream) for the
    batch y0d."""
    dev = y0d.device
    Bl = y0d.shape[0]
    lib = _lib.load()
    sched = get_schedule(t.to(torch.float64) if t.dtype == torch.float64 else t, None, False)
    handle = make_handle(model, Bl, dev)
    plan = build_plan(model, handle, dev)
    state, mask = pack_state(model, Bl, dev)
    _, coef, ostep, omode, oslope = sched.device_arrays(dev)
    sol = torch.empty(sched.T, Bl, 2, device=dev)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream

    def launch():
        _lib.check(lib.fetode_integrate_fixed(handle.ref, plan.data_ptr(), _lib.RK4, y0d.data_ptr(), Bl,
                                              coef.data_ptr(), sched.n_steps, ostep.data_ptr(),
                                              omode.data_ptr(), oslope.data_ptr(), sched.T, sol.data_ptr(),
                                              state.data_ptr(), mask, None, h), "integrate")
    for _ in range(3):
        launch()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for r in range(reps):
        ev[2 * r].record(stream)
        launch()
        ev[2 * r + 1].record(stream)
    torch.cuda.synchronize(dev)
    return float(np.mean([ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps)]))


def solve_ms(model, y0d, t, reps=30):
    """Host wall time of one whole odeint call (what a caller sees), median of `reps`."""
    func = F.autonomous(model)
    dev = y0d.device
    with torch.no_grad():
        for _ in range(3):
            F.odeint(func, y0d, t, method="rk4")
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            F.odeint(func, y0d, t, method="rk4")
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def solve_stream_ms(model, y0d, t, reps=50):
    """(per-call wall, per-call host issue) of `reps` odeint calls issued back to back and drained
    once — how a caller that streams solves sees them (the headline steps are timed this way too);
    the host's per-call work overlaps the previous call's kernel when it is the shorter of the two."""
    func = F.autonomous(model)
    dev = y0d.device
    with torch.no_grad():
        for _ in range(3):
            F.odeint(func, y0d, t, method="rk4")
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            F.odeint(func, y0d, t, method="rk4")
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
    return (t2 - t0) / reps * 1e3, (t1 - t0) / reps * 1e3


def pmc_traffic_per_launch():
    """HBM bytes per fused launch from the newest committed rocprofv3 PMC summary, corrected as
    MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE x2 on gfx950; WRITE_SIZE as is; KiB units)."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic*.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], REPO)


def pmc_issue(kernel_key):
    """VALU-/LDS-busy fractions of a kernel from the newest committed issue summary
    (tools/pmc_issue.py over a rocprofv3 PMC pass: SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_LDS against
    GRBM_GUI_ACTIVE; the issue model 2 quad-cycles per transcendental, 1 per other VALU instruction
    reproduces SQ_ACTIVE_INST_VALU)."""
    files = sorted(f for f in glob.glob(os.path.join(REPO, "profiles", "*pmc_issue.json")) if "raw" not in f)
    if not files:
        return None
    d = json.load(open(files[-1]))
    v = d.get(kernel_key)
    if v is None:
        return None
    return {"valu_busy_frac": v["valu_busy_frac"], "lds_busy_frac": v["lds_busy_frac"],
            "valu_insts_per_wave": v["valu_insts_per_wave"], "source": os.path.relpath(files[-1], REPO)}


def pmc_mfma(kernel_key):
    """MFMA-busy fraction of the SIMDs' cycles and MFMA TFLOP/s against the dense fp32 MFMA peak of
    one kernel, from the newest committed issue summary (SQ_INSTS_MFMA, SQ_VALU_MFMA_BUSY_CYCLES,
    the pass's kernel-trace duration)."""
    files = sorted(f for f in glob.glob(os.path.join(REPO, "profiles", "*pmc_issue.json")) if "raw" not in f)
    for f in reversed(files):
        v = json.load(open(f)).get(kernel_key)
        if v and "mfma_busy_frac" in v:
            return {"mfma_busy_frac": v["mfma_busy_frac"], "mfma_tflops": v.get("mfma_tflops"),
                    "peak_tflops": FP32_PEAK_TFLOPS, "frac_of_peak": v.get("mfma_frac_of_fp32_peak"),
                    "mfma_per_launch": v.get("mfma_per_launch"), "source": os.path.relpath(f, REPO)}
    return None


def train_rate(model, y0d, t, iters, warmup, world, strong=True):
    """One training iteration = forward rk4 solve with autograd (one launch that also records the
    layer inputs of every evaluation) + backward (one reverse-sweep launch + fixed-order gradient
    reduction) + gradient all-reduce (RCCL when world > 1) + Adam.  Adam runs as
    torch's fused multi-tensor kernel (same update rule as the reference's torch.optim.Adam).
    On one GPU the iteration is captured once and replayed as ONE HIP graph
    (fet_ode_amd.training.CapturedStep: bitwise the eager iterations); `eager` times the same
    iteration issued op by op from Python (host-bound on a slow host).  N > 1 stays eager (the
    all-reduce is not captured)."""
    import copy
    import fet_ode_amd.dist as D
    from fet_ode_amd.training import CapturedStep
    dev = y0d.device
    target = torch.zeros(T, y0d.shape[0], 2, device=dev)

    def make(m, capturable):
        func = F.autonomous(m)
        opt = torch.optim.Adam(m.parameters(), lr=1e-4, fused=True, capturable=capturable)

        def it():
            # the reference's optimizer.zero_grad() (set_to_none=True, torch's default): autograd
            # then keeps the fused backward's gradient views as .grad (no per-parameter add kernels)
            opt.zero_grad(set_to_none=True)
            sol = F.odeint(func, y0d, t, method="rk4")
            loss = (sol - target).square().mean()
            loss.backward()
            D.allreduce_gradients(list(m.parameters()))
            opt.step()
        return it

    def timed(fn, n):
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            nccl = torch.distributed.get_backend() == "nccl"
            tt = torch.tensor([el], device=dev if nccl else "cpu", dtype=torch.float64)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            el = tt.item()
        return el

    eager_model = copy.deepcopy(model) if world == 1 else model
    it = make(eager_model, False)
    for _ in range(warmup):
        it()
    el_eager = timed(it, iters)
    scale = (1 if strong else world) * iters * STEPS_PER_SOLVE
    out = {"unit": "RK4 steps/s trained (fwd+bwd+allreduce+Adam) of the batch-4096 job", "iters": iters,
           "eager": {"value": scale / el_eager, "ms_per_iter": el_eager / iters * 1e3,
                     "path": "host-issued: fetode_integrate_fixed with tape + fetode_integrate_fixed_backward "
                             "+ loss ops + fused Adam, op by op"}}
    if world == 1:
        step = CapturedStep(make(copy.deepcopy(model), True), warmup=warmup, device=dev)
        el = timed(step, iters)
        out.update({"value": scale / el, "ms_per_iter": el / iters * 1e3,
                    "path": "one HIP graph replay per iteration (fet_ode_amd.training.CapturedStep) of the same "
                            "launches: fetode_integrate_fixed with tape + fetode_integrate_fixed_backward + loss + "
                            "fused Adam"})
    else:
        out.update({"value": out["eager"]["value"], "ms_per_iter": out["eager"]["ms_per_iter"],
                    "path": out["eager"]["path"]})
    return out


def lv_dopri5_rate(sd, y0d, t, reps=3, rtol=1e-7, atol=1e-9):
    """The north-star call as the reference makes it: torchodeint(calDeriv, X0, t_learn) with
    torchdiffeq's defaults (dopri5, rtol 1e-7, atol 1e-9; train_kanfet_node_predprey.py), B = 4096,
    the 35-point grid, no_grad.  The whole adaptive solve is one cooperative launch
    (fetode_integrate_dopri5: field, error norm and step control on the device)."""
    from fet_ode_amd.dopri5 import ResidentSolve
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(y0d.device)
    func = F.autonomous(m)
    with torch.no_grad():
        F.odeint(func, y0d, t, rtol=rtol, atol=atol)
        torch.cuda.synchronize(y0d.device)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            sol = F.odeint(func, y0d, t, rtol=rtol, atol=atol)
            torch.cuda.synchronize(y0d.device)
            ts.append(time.perf_counter() - t0)
    s = F.dopri5.dopri5_solve.last
    el = float(np.median(ts))
    acc = sum(1 for a in s.attempts if a[3])   # of the logged attempts (all of them below 16384)
    return {"value": 1.0 / el, "unit": f"dopri5 solves/s (B={y0d.shape[0]}, rtol {rtol:g}, atol {atol:g}, "
                                       "t=linspace(0,3.5,35))",
            "ms_per_solve": el * 1e3, "attempts": s.n_attempts, "accepted": acc, "nfev": s.nfev,
            "field_evals_per_s": s.nfev / el, "rk4_equiv_steps_per_s": s.nfev / 4 / el,
            "resident": isinstance(s, ResidentSolve), "finite": bool(torch.isfinite(sol).all()),
            "path": "fetode_integrate_dopri5: fused4_kernel DOPRI instantiation, one launch"}


def lv_dopri5_train_rate(sd, y0d, t, iters=3, rtol=1e-3, atol=1e-4, resident=True, target=None):
    """The reference's training iteration on its default method: odeint(calDeriv, X0, t_learn) with
    dopri5, then loss.backward() and Adam (train_kanfet_node_predprey.py:252-257).  torchdiffeq's
    direct backprop differentiates every stage of every attempt AND the step-size control (d dt /
    d theta through the error ratios, the initial step, the output times).  resident: the taped
    resident solve + one resident reverse sweep (fetode_integrate_dopri5_tape / _backward,
    DESIGN.md §4.10); else _Dopri5Grad (host-driven attempts, per-stage HIP kernels + HIP VJPs
    under autograd)."""
    from fet_ode_amd.dopri5 import ResidentSolve, set_resident_dopri5_training
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(y0d.device)
    func = F.autonomous(m)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    if target is None:
        target = torch.zeros(t.numel(), y0d.shape[0], 2, device=y0d.device)

    def it():
        opt.zero_grad()
        sol = F.odeint(func, y0d, t, rtol=rtol, atol=atol)
        loss = (sol - target).square().mean()
        loss.backward()
        opt.step()
        return loss

    prev = set_resident_dopri5_training(resident)
    try:
        it()
        torch.cuda.synchronize(y0d.device)
        t0 = time.perf_counter()
        for _ in range(iters):
            loss = it()
        torch.cuda.synchronize(y0d.device)
    finally:
        set_resident_dopri5_training(prev)
    el = (time.perf_counter() - t0) / iters
    s = F.dopri5.dopri5_solve.last
    B = y0d.shape[0]
    return {"value": 1.0 / el, "unit": f"dopri5 training iterations/s (B={B}, rtol {rtol:g}, atol {atol:g}, "
                                       f"t=linspace(0,3.5,{t.numel()}))",
            "ms_per_iter": el * 1e3, "attempts": s.n_attempts, "nfev": s.nfev,
            "finite": bool(torch.isfinite(loss).item()),
            "path": ("taped resident solve (fetode_integrate_dopri5_tape) + resident reverse sweep "
                     "(fetode_integrate_dopri5_backward): 2 launches + the parameter-sum reduction"
                     if isinstance(s, ResidentSolve) else
                     "_Dopri5Grad: host-driven attempts, per-stage HIP field kernels + HIP VJPs under autograd "
                     "(direct backprop incl. the step-size control)")}


def lv_dopri5_sharded_rate(sd, y0d, t, world, B_global, reps=3):
    """The north-star default call sharded over the ranks (dist.odeint_sharded): each rank solves
    its block of the global batch in ONE resident launch whose exchange workgroup sums every error
    norm across the ranks (fetode_integrate_dopri5_xrank), so all ranks take the global batch's
    steps.  Time = max over ranks between barriers."""
    import torch.distributed as dist
    import fet_ode_amd.dist as D
    from fet_ode_amd.dopri5 import ResidentSolve
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(y0d.device)
    func = F.autonomous(m)
    fallback = None
    with torch.no_grad():
        # the resident exchange must not cost the line: a timed-out resident solve (status 4:
        # grids not co-resident, or a peer's stores not seen) raises after restoring the
        # hysteresis state; every rank then agrees to rerun the leg on the host-driven loop
        err = None
        try:
            D.odeint_sharded(func, y0d, t)
            torch.cuda.synchronize(y0d.device)
        except RuntimeError as e:
            err = str(e)
        bad = torch.tensor([1.0 if err else 0.0], dtype=torch.float64,
                           device=y0d.device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item() > 0:
            fallback = err or "a peer rank's resident solve timed out"
            D.set_resident_sharded(False)
            m.load_state_dict(sd)   # hysteresis buffers back to the checkpoint's
            D.odeint_sharded(func, y0d, t)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(y0d.device)
            dist.barrier()
            t0 = time.perf_counter()
            sol = D.odeint_sharded(func, y0d, t)
            torch.cuda.synchronize(y0d.device)
            ts.append(time.perf_counter() - t0)
        if fallback is not None:
            D.set_resident_sharded(True)
    el = torch.tensor([float(np.median(ts))], dtype=torch.float64,
                      device=y0d.device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    s = F.dopri5.dopri5_solve.last
    return {"value": 1.0 / el, "unit": f"dopri5 solves/s (global B={B_global} over {world} GPUs, rtol 1e-7, "
                                       "atol 1e-9, t=linspace(0,3.5,35))",
            "ms_per_solve": el * 1e3, "attempts": s.n_attempts, "nfev": s.nfev,
            "resident": isinstance(s, ResidentSolve), "finite": bool(torch.isfinite(sol).all()),
            "path": ("fetode_integrate_dopri5_xrank: one launch per rank, norms exchanged between the kernels"
                     if isinstance(s, ResidentSolve) else
                     "host-driven loop: one field launch per evaluation, one norm all-reduce per attempt"),
            "resident_fallback": fallback}


def plain_closure_rate(model, y0d, t, reps=3):
    """The literal drop-in: the reference's `calDeriv(t, X) = kan_fet_model(X)` closure unchanged
    (train_kanfet_node_predprey.py:159-161).  odeint recognises the closure as
    the module call it is (fet_ode_amd.odeint.closure_field) and integrates it in one launch; the
    `per_stage` sub-line times the same closure with the recognition switched off (one fused
    single-evaluation launch + one stage-combine launch per stage, 272 per solve) — the path any
    closure that does more than call the module takes."""
    def calDeriv(t, X):
        dXdt = model(X)
        return dXdt

    def rate(fuse, n):
        with torch.no_grad(), F.closure_fusion(fuse):
            F.odeint(calDeriv, y0d, t, method="rk4")
            torch.cuda.synchronize(y0d.device)
            t0 = time.perf_counter()
            for _ in range(n):
                F.odeint(calDeriv, y0d, t, method="rk4")
            torch.cuda.synchronize(y0d.device)
            return (time.perf_counter() - t0) / n

    el, el_ps = rate(True, 20), rate(False, reps)
    return {"value": STEPS_PER_SOLVE / el, "unit": "RK4 steps/s of the batch-4096 job, plain calDeriv closure",
            "ms_per_solve": el * 1e3, "path": "fused: the closure recognised as the module call (one launch per solve)",
            "per_stage": {"value": STEPS_PER_SOLVE / el_ps, "ms_per_solve": el_ps * 1e3,
                          "path": "closure_fusion(False): fetode_field_forward + fetode_rk_combine per stage"}}


def synthetic_ecg(batch, T=96, seed=0):
    """Synthetic ECG200-shaped series (the dataset is not in the image): a seeded sum of two
    sinusoids + noise per row, z-normalised like the UCR files."""
    g = torch.Generator().manual_seed(seed)
    tt = torch.linspace(0, 1, T, dtype=torch.float64)
    f = 1.0 + 3.0 * torch.rand(batch, 1, generator=g, dtype=torch.float64)
    ph = 6.283185307179586 * torch.rand(batch, 1, generator=g, dtype=torch.float64)
    x = torch.sin(6.283185307179586 * f * tt + ph) + 0.3 * torch.sin(18.84955592153876 * f * tt)
    x = x + 0.1 * torch.randn(batch, T, generator=g, dtype=torch.float64)
    x = (x - x.mean(dim=1, keepdim=True)) / x.std(dim=1, keepdim=True)
    return x.to(torch.float32)


def synthetic_mnist(batch, H=28, W=28, seed=0):
    """Synthetic MNIST-shaped images in [0, 1] (the dataset is not in the image): a seeded ring per
    image plus noise."""
    g = torch.Generator().manual_seed(seed)
    yy = torch.linspace(-1, 1, H, dtype=torch.float64).view(1, H, 1)
    xx = torch.linspace(-1, 1, W, dtype=torch.float64).view(1, 1, W)
    c = (torch.rand(batch, 2, 1, 1, generator=g, dtype=torch.float64) - 0.5)
    r = 0.2 + 0.3 * torch.rand(batch, 1, 1, generator=g, dtype=torch.float64)
    d = ((yy - c[:, 0]) ** 2 + (xx - c[:, 1]) ** 2).sqrt()
    img = torch.exp(-((d - r) / 0.12) ** 2) + 0.05 * torch.rand(batch, H, W, generator=g, dtype=torch.float64)
    return img.clamp(0, 1).to(torch.float32).unsqueeze(1)


def ecg_rate(dev, reps=50, cpu_seconds=5.0, with_cpu=True, rtol=1e-3, atol=1e-4):
    """BASELINE configs[2] (train_ecg_kan_fet_nn_ode.py:512-572): KanFet_NODE.eval() forward on a
    batch of 200 synthetic ECG200-shaped series (T = 96; the dataset is not in the image), latent
    64, 10 bases, dopri5 on [0, 1] at the class defaults rtol 1e-3 / atol 1e-4 (:512-530) or, for
    the `rtol_1e-2` leg, the __main__'s rtol 1e-2 / atol 1e-3 (:1196-1197).  Under no_grad the whole
    dopri5 solve is one device-resident launch (fetode_ecg_dopri5); the encoder / classifier are one
    launch each."""
    from fet_ode_amd import ecg
    torch.manual_seed(0)
    m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10, rtol=rtol, atol=atol)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).eval()
    x = synthetic_ecg(200, seed=1)
    xd = x.to(dev)
    with torch.no_grad():
        for _ in range(20):   # clocks settle over the first back-to-back solves
            m(xd)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            m(xd)
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / reps
    s = m.last_solve
    out = {"value": 1.0 / el, "unit": "KanFet_NODE forward solves/s (B=200, dopri5)", "ms_per_solve": el * 1e3,
           "nfev": s.nfev, "attempts": len(s.attempts), "field_evals_per_s": s.nfev / el,
           "workload": f"KanFet_NODE(T=96, 2 classes, latent 64, nb 10), dopri5 rtol {rtol:g} atol {atol:g}, "
                       "t=[0,1], B=200 synthetic series, eval mode"}
    if with_cpu:   # the oracle is the CPU leg only
        from oracle import ecg_ref as E
        cores, _ = cpu_cores()
        torch.set_num_threads(cores)
        n, t0 = 0, time.perf_counter()
        with torch.no_grad():
            while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 20):
                E.ECGNodeRef({k: v.clone() for k, v in sd.items()}, rtol=rtol, atol=atol)(x)
                n += 1
        cel = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": 1.0 / cel, "unit": out["unit"], "cores": cores, "kind": "port",
                               "sample": f"{n} full forward(s) of the same workload with oracle/ecg_ref.py "
                                         f"(reference op order, torch CPU fp32), {cel * n:.1f} s"}
    return out


def mnist_rate(dev, batch=8192, reps=10, cpu_seconds=5.0, with_cpu=True):
    """The MNIST config (mnist_kuramoto_kan.py:202-221): KuramotoKANClassifier on 28 x 28 synthetic
    images (the dataset is not in the image), 10 Kuramoto steps, KANLinear(1568 -> 10, 8 logistic
    bases).  Forward images/s under no_grad and training images/s (forward + cross-entropy +
    backward of every parameter) on one GPU."""
    from fet_ode_amd import mnist
    torch.manual_seed(0)
    m = mnist.KuramotoKANClassifier()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = synthetic_mnist(batch, seed=3)
    xd = x.to(dev)
    y = (torch.arange(batch) % 10).to(dev)

    def timed(fn, n):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n

    with torch.no_grad():
        fwd = timed(lambda: m(xd), reps)

    def train_step():
        m.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(xd), y).backward()

    trn = timed(train_step, reps)
    out = {"value": batch / fwd, "unit": "images/s forward (KuramotoKANClassifier 28x28, 1 GPU)",
           "ms_per_batch": fwd * 1e3, "train_images_per_s": batch / trn, "train_ms_per_batch": trn * 1e3,
           "workload": f"KuramotoKANClassifier(28x28, 10 Kuramoto steps, KANLinear 1568->10, nb 8), batch {batch}, "
                       "synthetic images"}
    if with_cpu:   # the oracle is the CPU leg only
        from oracle import mnist_ref as M
        cores, _ = cpu_cores()
        torch.set_num_threads(cores)
        ref = M.ClassifierRef(sd)
        xs = x[:256]
        n, t0 = 0, time.perf_counter()
        with torch.no_grad():
            while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 20):
                ref(xs)
                n += 1
        cel = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": 256 / cel, "unit": out["unit"].replace("1 GPU", "CPU"), "cores": cores,
                               "kind": "port", "sample": f"{n} forward(s) of 256 of the images with "
                                                         f"oracle/mnist_ref.py (torch CPU fp32), {cel * n:.1f} s"}
    return out


def ett_rate(dev, batch=8192, reps=2, substeps=4, cpu_seconds=5.0, with_cpu=True):
    """The ETT config (train_kan_fet_ett.py:155-197, BASELINE configs[3]): LatentNeuralODEForecaster
    on 96 -> 96 windows of a 7-column synthetic ETTh1-shaped series (the dataset is not in the
    image), latent 64, KAN-FET latent field [64, 128, 64] (K=10), odeint_rk4 with the reference
    TrainConfig's rk4_substeps=4 over t_fut = 0..95.  Forward windows/s under no_grad on one GPU.
    The untrained field is scaled by 0.1 (coef, KAN weights; as the training line) so the latent
    state stays bounded over the 95 time units instead of diverging, and the first call's forecasts
    of 8 windows are checked against the CPU oracle's (`parity`, the windows the CPU leg times)."""
    from fet_ode_amd import ett
    c = p = 96
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=p, latent_dim=64, solver="rk4")
    with torch.no_grad():
        for n, p_ in m.dynamics.net.named_parameters():
            if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
                p_.mul_(0.1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(batch + c + p, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], c, p, device=dev)
    xb, _ = ds.batch(torch.arange(batch, device=dev))
    t_fut = torch.linspace(0.0, float(p - 1), steps=p, device=dev)
    with torch.no_grad():
        first = m(xb, t_fut, rk4_substeps=substeps)
        finite = bool(torch.isfinite(first).all())
        first8 = first[:8].double().cpu()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            m(xb, t_fut, rk4_substeps=substeps)
        torch.cuda.synchronize(dev)
    fwd = (time.perf_counter() - t0) / reps
    steps = (p - 1) * substeps
    out = {"value": batch / fwd, "unit": "forecast windows/s forward (96->96, 1 GPU)", "ms_per_batch": fwd * 1e3,
           "rk4_steps_per_s": batch * steps / fwd, "finite": finite,
           "workload": f"LatentNeuralODEForecaster(7 features, 96->96, latent 64, KANFET[64,128,64] K=10, field x0.1), "
                       f"odeint_rk4 x{substeps} substeps ({steps} steps), batch {batch}, synthetic series"}
    if with_cpu:
        from oracle import ett_ref as E
        from oracle import torch_ref as O
        cores, _ = cpu_cores()
        torch.set_num_threads(cores)
        field = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sd.items()
                                             if k.startswith("dynamics.net.")}, 2)
        ref = E.ForecasterRef(sd, lambda tt, zz: field(zz))
        xs = xb[:8].cpu()
        tc = t_fut.cpu()
        n, t0 = 0, time.perf_counter()
        with torch.no_grad():
            while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 5):
                field.reset_state()
                r = ref(xs, tc, rk4_substeps=substeps)
                if n == 0:
                    ref8 = r.double()
                n += 1
        cel = (time.perf_counter() - t0) / n
        # the fp64 oracle on the same windows: the reference's own fp32 spread beside the GPU's
        sd64 = {k: v.double() for k, v in sd.items()}
        field64 = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sd64.items()
                                               if k.startswith("dynamics.net.")}, 2)
        with torch.no_grad():
            ref64 = E.ForecasterRef(sd64, lambda tt, zz: field64(zz))(xs.double(), tc.double(), rk4_substeps=substeps)
        # three equally valid fp32 re-roundings of the parameters (oracle/parity.py's controls): one
        # fp32 rounding is one draw of the 380-step error
        gen = torch.Generator().manual_seed(0)
        ctrl = []
        for _ in range(3):
            sdp = {k: (v * (1 + 6e-8 * torch.randn(v.shape, generator=gen)) if v.is_floating_point()
                       and k.startswith("dynamics.net.") and not k.endswith(("grid", "prev_x", "branch_sign"))
                       else v) for k, v in sd.items()}
            fp = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sdp.items()
                                              if k.startswith("dynamics.net.")}, 2)
            with torch.no_grad():
                ctrl.append(E.ForecasterRef(sdp, lambda tt, zz: fp(zz))(xs, tc, rk4_substeps=substeps).double())
        d = (first8 - ref8).abs()
        scale = float(ref64.abs().max())
        err64, spread = float((first8 - ref64).abs().max()), float((ref8 - ref64).abs().max())
        cspread = [float((c_ - ref64).abs().max()) for c_ in ctrl]
        yard = max([spread] + cspread)
        out["parity"] = {"windows": 8, "max_abs_vs_oracle": float(d.max()),
                         "max_rel_vs_oracle": float(d.max() / ref8.abs().max().clamp_min(1e-30)),
                         "forecast_max_abs": float(ref8.abs().max()),
                         "gpu_vs_fp64_max_rel": err64 / scale, "ref_fp32_vs_fp64_max_rel": spread / scale,
                         "control_fp32_vs_fp64_max_rel": [c_ / scale for c_ in cspread],
                         "envelope_ok": err64 <= 4 * yard + 1e-5 * scale,
                         "note": "first call (fresh hysteresis state) of the GPU forecaster on the full batch, windows "
                                 "0-7, vs oracle/ett_ref.py on those windows (torch CPU fp32, and fp64: the "
                                 "reference's own fp32 spread, and three re-roundings of its parameters; envelope "
                                 "rule |gpu-fp64| <= 4 max|ref32-fp64| + 1e-5 scale, "
                                 "tests/test_gpu_production_oracle.py)"}
        out["cpu_baseline"] = {"value": 8 / cel, "unit": out["unit"].replace("1 GPU", "CPU"), "cores": cores,
                               "kind": "port", "sample": f"{n} forward(s) of 8 of the windows with oracle/ett_ref.py "
                                                         f"+ torch_ref.py (torch CPU fp32), {cel * n:.1f} s"}
    return out


def ett_dopri5_rate(dev, batch=8192, rtol=1e-3, atol=1e-4, small=(256, 1024)):
    """The reference forecaster's own solver call, odeint(dynamics, z0, t_fut, method="dopri5")
    (train_kan_fet_ett.py:192), with the KAN-FET latent field [64, 128, 64] (K = 10) on B = 8192
    96 -> 96 windows.  At torchdiffeq's default rtol 1e-7 / atol 1e-9 the fp32 KAN-FET field needs
    ~160 k attempts per forward (measured at B = 256: 159 373 attempts, 956 k evaluations, 184 s
    on the host loop), so the line runs at rtol 1e-3 / atol 1e-4.  The forward's
    solve is ONE launch (fetode_wide_dopri5: persistent grid over the wide-layer tiles, DESIGN.md
    §4.8); `host_loop` times the host-driven loop on the same inputs (two wide-layer launches per
    evaluation, one read-back per attempt; bitwise the same solution), `b256` / `b1024` both at
    those batches (VERDICT r4 asked for B = 1024 beside 8192)."""
    from fet_ode_amd import dopri5 as D
    from fet_ode_amd import ett
    c = p = 96

    sds = {}

    def run(B, resident):
        # one model per batch for both paths (the efficient_kan init is not bitwise reproducible
        # from a seed): the second run loads the first one's weights
        torch.manual_seed(0)
        m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=p, latent_dim=64, solver="dopri5",
                                          rtol=rtol, atol=atol)
        if B in sds:
            m.load_state_dict(sds[B])
        else:
            sds[B] = {k: v.clone() for k, v in m.state_dict().items()}
        m = m.to(dev)
        g = torch.Generator().manual_seed(4)
        series = torch.cumsum(torch.randn(B + c + p, 7, generator=g), 0) * 0.05
        ds = ett.EnergyWindowDataset(series, series[:, -1], c, p, device=dev)
        xb, _ = ds.batch(torch.arange(B, device=dev))
        t_fut = torch.linspace(0.0, float(p - 1), steps=p, device=dev)
        prev = D.set_wide_resident_dopri5(resident)
        try:
            with torch.no_grad():
                z0 = m.encoder(xb)
                for _ in range(2):
                    m.dynamics(0.0, z0)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(10):
                    m.dynamics(0.0, z0)
                torch.cuda.synchronize(dev)
                ev = (time.perf_counter() - t0) / 10
                m.dynamics.net.reset_state()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                y = m(xb, t_fut)
                torch.cuda.synchronize(dev)
                wall = time.perf_counter() - t0
        finally:
            D.set_wide_resident_dopri5(prev)
        s = D.dopri5_solve.last
        return {"value": B / wall, "ms_per_batch": wall * 1e3, "attempts": s.n_attempts, "nfev": s.nfev,
                "field_eval_ms": ev * 1e3, "eval_share": s.nfev * ev / wall, "finite": bool(torch.isfinite(y).all())}, y

    res, yr = run(batch, True)
    host, yh = run(batch, False)
    out = {"value": res["value"], "unit": "forecast windows/s forward, dopri5 (96->96, 1 GPU)", **res,
           "rtol": rtol, "atol": atol,
           "workload": f"LatentNeuralODEForecaster(7 features, 96->96, latent 64, KANFET[64,128,64] K=10), dopri5 "
                       f"rtol {rtol:g} atol {atol:g}, batch {batch}, synthetic series",
           "path": "fetode_wide_dopri5: the whole solve in one launch (persistent grid over the wide-layer tiles)",
           "host_loop": {**host, "same_solution": bool(torch.equal(yr, yh)),
                         "path": "dopri5 host loop: 2 fetode_wide_layer_forward per evaluation, a read-back per attempt"}}
    for sb in small or ():
        rs, ys = run(sb, True)
        hs, yhs = run(sb, False)
        out[f"b{sb}"] = {"resident": rs, "host_loop": hs, "same_solution": bool(torch.equal(ys, yhs)),
                         "speedup": hs["ms_per_batch"] / rs["ms_per_batch"]}
    return out


def ett_dopri5_train_rate(dev, batch=2048, P=24, tscale=0.05, iters=4, rtol=1e-3, atol=1e-4):
    """Training through the reference forecaster's own dopri5 call (train_kan_fet_ett.py:192, the
    loop at :320-335: forward, MSE, loss.backward(), Adam) with the KAN-FET latent field [64, 128, 64].
    torchdiffeq's direct backprop runs through every stage, the error ratios and the step sizes; here
    the attempts are host-driven (dopri5._Dopri5Grad: one read-back per attempt) and every field
    evaluation and VJP is the wide HIP kernels (_WideLayerFlatFn: one launch forward, the Ferro and
    KANLinear VJPs backward, the layer's parameters as one flat autograd input) and every stage
    combine one HIP launch each way (_CombFn, d/d dt kept).  The untrained synthetic field is scaled by 0.1 (coef, KAN weights) and
    the 24 outputs span 1.15 time units so the latent state stays where the reference's own logistic
    basis has finite gradients (exp overflow x zero adjoint is NaN in its autograd beyond)."""
    from fet_ode_amd import ett
    import fet_ode_amd.dopri5  # noqa: F401
    c = 96
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=P, latent_dim=64, solver="dopri5",
                                      rtol=rtol, atol=atol)
    with torch.no_grad():
        for n, p_ in m.dynamics.net.named_parameters():
            if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
                p_.mul_(0.1)
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(batch + c + P, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], c, P, device=dev)
    xb, yb = ds.batch(torch.arange(batch, device=dev))
    t_fut = torch.linspace(0.0, float(P - 1) * tscale, steps=P, device=dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    fwd, bwd, fin = [], [], True
    for it in range(iters + 1):
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        loss = torch.nn.functional.mse_loss(m(xb, t_fut), yb)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        loss.backward()
        opt.step()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        fin = fin and bool(torch.isfinite(loss)) and all(bool(torch.isfinite(p_.grad).all())
                                                         for p_ in m.parameters() if p_.grad is not None)
        if it > 0:
            fwd.append(t1 - t0)
            bwd.append(t2 - t1)
    s = F.dopri5.dopri5_solve.last
    el = float(np.mean(fwd) + np.mean(bwd))
    return {"value": batch / el, "unit": f"training windows/s (fwd + bwd + Adam, dopri5 rtol {rtol:g}, B={batch})",
            "ms_per_iter": el * 1e3, "fwd_ms": float(np.mean(fwd)) * 1e3, "bwd_ms": float(np.mean(bwd)) * 1e3,
            "attempts": s.n_attempts, "nfev": s.nfev, "finite": fin,
            "workload": f"LatentNeuralODEForecaster(7 features, 96->{P}, latent 64, KANFET[64,128,64] K=10, field x0.1), "
                        f"t_fut = linspace(0, {(P - 1) * tscale:g}, {P}), dopri5 rtol {rtol:g} atol {atol:g}, batch {batch}",
            "path": "dopri5._Dopri5Grad: host-driven attempts (torchdiffeq's direct backprop incl. the step-size "
                    "control; one read-back per attempt), the wide HIP layer kernel per evaluation, the wide "
                    "Ferro / KANLinear VJPs, stage combines as fetode_comb_forward / _backward"}


def ett_reference_iteration_rate(dev, batch=64, ctx=32, P=8, iters=2, rtol=1e-7, atol=1e-9, field_scale=0.1):
    """The reference's OWN training iteration (train_kan_fet_ett.py:258-260 TrainConfig, :312-335
    run_epoch): batch_size 64, context 32 -> pred 8, t_fut = linspace(0, 7, 8), the forecaster's
    odeint(..., method="dopri5") at torchdiffeq's defaults (rtol 1e-7 / atol 1e-9), MSE, backward,
    clip_grad_norm_(1.0), AdamW(lr 1e-3, weight_decay 1e-4) — with the KAN-FET latent field
    [64, 128, 64] (config 4's substitution) scaled by `field_scale` (untrained weights,
    synthetic 7-column series: the dataset is not in the image).  Host-driven dopri5 under autograd
    (dopri5._Dopri5Grad), the wide HIP layer / VJP kernels."""
    from fet_ode_amd import ett
    import fet_ode_amd.dopri5  # noqa: F401
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=ctx, pred_len=P, latent_dim=64, solver="dopri5",
                                      rtol=rtol, atol=atol)
    with torch.no_grad():
        for n, p_ in m.dynamics.net.named_parameters():
            if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
                p_.mul_(field_scale)
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(batch + ctx + P, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], ctx, P, device=dev)
    xb, yb = ds.batch(torch.arange(batch, device=dev))
    t_fut = torch.linspace(0.0, float(P - 1), steps=P, device=dev)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    its, fin, att, nfev = [], True, [], []
    for it in range(iters):
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        loss = torch.nn.functional.mse_loss(m(xb, t_fut), yb)
        s = F.dopri5.dopri5_solve.last
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        torch.cuda.synchronize(dev)
        its.append(time.perf_counter() - t0)
        att.append(s.n_attempts)
        nfev.append(s.nfev)
        fin = fin and bool(torch.isfinite(loss))
    el = float(np.mean(its))
    return {"value": batch / el, "unit": f"training windows/s (the reference's iteration, B={batch})",
            "ms_per_iter": el * 1e3, "attempts": att, "nfev": nfev, "finite": fin,
            "workload": f"LatentNeuralODEForecaster(7 features, {ctx}->{P}, latent 64, KANFET[64,128,64] K=10, field "
                        f"x{field_scale:g}), t_fut = linspace(0, {P - 1}, {P}), dopri5 rtol {rtol:g} atol {atol:g}, "
                        f"MSE, clip_grad_norm 1.0, AdamW(1e-3, wd 1e-4), batch {batch}",
            "path": "dopri5._Dopri5Grad (host-driven attempts under autograd), wide HIP layer + VJP kernels"}


def ett_encoder_rate(dev, batch=8192, ctx=96, reps=20, with_cpu=True, cpu_seconds=5.0):
    """The encoder of the reference's KAN-FET ETT model (KAN_FET_LatentODE_DiffusionForecaster,
    train_kan_fet_ett.py:822-837): KANRNNEncoder(7 features, hidden 64, latent 64, 10 bases) over
    96-step contexts (:798-818), B = 8192 windows of a synthetic series.  Forward (no_grad: one
    launch; only the steps that can reach h_T run), the full 96-step recurrence
    (the same launch with full = 1), and a training step (forward with tape + HIP VJP + the
    to_latent GEMMs)."""
    from fet_ode_amd import ett, _lib as L
    torch.manual_seed(0)
    enc = ett.KANRNNEncoder(7, 64, 64, 10)
    sd = {k: v.clone() for k, v in enc.state_dict().items()}
    enc = enc.to(dev)
    g = torch.Generator().manual_seed(6)
    series = torch.cumsum(torch.randn(batch + ctx, 7, generator=g), 0) * 0.05
    x = series.unfold(0, ctx, 1)[:batch].transpose(1, 2).contiguous()      # (B, 96, 7) windows
    xd = x.to(dev)
    lib = L.load()
    keep = []
    d = ett._rnn_desc(enc.rnn_cell, enc.to_latent, keep)
    z0 = torch.empty(batch, 64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch(full):
        L.check(lib.fetode_kanrnn_forward(L.ctypes.byref(d), xd.data_ptr(), batch, ctx, None, None, z0.data_ptr(),
                                          None, full, stream.cuda_stream), "kanrnn")

    def ev_time(fn, n):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(n):
            fn()
        b.record(stream)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / n

    k_cone = ev_time(lambda: launch(0), reps)
    k_full = ev_time(lambda: launch(1), reps)
    with torch.no_grad():
        for _ in range(2):
            enc(xd)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            enc(xd)
        torch.cuda.synchronize(dev)
        fwd = (time.perf_counter() - t0) / reps
    gz = torch.randn(batch, 64, device=dev)

    def step():
        enc.zero_grad(set_to_none=True)
        enc(xd).backward(gz)

    for _ in range(2):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    trn = (time.perf_counter() - t0) / reps
    depth = lib.fetode_kanrnn_depth(7, 64, 10)
    # algorithmic bytes: the cone reads x of the last depth+1 steps (7 floats each) and writes z0;
    # the full recurrence reads the whole context
    cone_bytes = batch * 4 * ((depth + 1) * 7 + 64)
    full_bytes = batch * 4 * (ctx * 7 + 64)
    out = {"value": batch / fwd, "unit": "windows/s encoded (KANRNNEncoder forward, 1 GPU)", "ms_per_batch": fwd * 1e3,
           "kernel_ms_cone": k_cone, "kernel_ms_full_recurrence": k_full, "cone_depth": depth,
           "full_recurrence_windows_per_s": batch / (k_full * 1e-3),
           "train_windows_per_s": batch / trn, "train_ms_per_batch": trn * 1e3,
           "roofline_full": {"bound": "transcendental (4 exp/rcp per hidden unit per step)",
                             "alg_bytes": full_bytes, "achieved_GBs": full_bytes / (k_full * 1e-3) / 1e9},
           "roofline_cone": {"alg_bytes": cone_bytes, "achieved_GBs": cone_bytes / (k_cone * 1e-3) / 1e9},
           "workload": f"KANRNNEncoder(7, hidden 64, latent 64, nb 10), context {ctx}, batch {batch}, synthetic series",
           "path": "fetode_kanrnn_forward (one launch, to_latent fused) / fetode_kanrnn_backward"}
    if with_cpu:
        from oracle import ett_ref as E
        cores, _ = cpu_cores()
        torch.set_num_threads(cores)
        ref = E.KANRNNEncoderRef(sd)
        xs = x[:1024]
        n, t0 = 0, time.perf_counter()
        with torch.no_grad():
            while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 20):
                ref(xs)
                n += 1
        cel = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": 1024 / cel, "unit": "windows/s encoded (CPU)", "cores": cores, "kind": "port",
                               "sample": f"{n} forward(s) of 1024 of the windows with oracle/ett_ref.py "
                                         f"KANRNNEncoderRef (reference op order, all 96 steps, torch CPU fp32), "
                                         f"{cel * n:.1f} s"}
    return out


def cpu_cores():
    """(threads used, physical cores of this host from lscpu).  The threads are the physical cores,
    capped at the process's CPU share: the GPU box allots 16 cores per GPU (OMP_NUM_THREADS = 16
    there, which its operators ask jobs to keep) and the affinity mask may be narrower still."""
    phys = None
    try:
        import subprocess
        out = subprocess.run(["lscpu", "-p=core,socket"], capture_output=True, text=True, timeout=10).stdout
        phys = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")})
    except Exception:
        pass
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    try:
        share = min(share, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    return max(1, min(phys or share, share)), phys


def _median_solves(fn, n):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def cpu_baseline(sd, y0, t, n_solves):
    """The CPU oracle (restatement of the reference, reference op order, verified bitwise against
    the reference modules) on this host: the full bench workload (B = 4096, 34 rk4 steps), median
    of `n_solves` fresh-state solves on the physical cores, plus one solve on 1 thread."""
    from oracle import torch_ref as O
    cores, phys = cpu_cores()
    sol = None

    def solve():
        nonlocal sol
        ref = O.KANFETRef.from_state_dict(sd, 2)
        sol = O.odeint(lambda tt, yy: ref(yy), y0, t, method="rk4")

    with torch.no_grad():
        torch.set_num_threads(cores)
        O.odeint(lambda tt, yy: O.KANFETRef.from_state_dict(sd, 2)(yy), y0[:64], t[:2], method="rk4")  # warm-up
        med, ts = _median_solves(solve, n_solves)
        first = sol
        torch.set_num_threads(1)
        med1, ts1 = _median_solves(solve, 1)
        torch.set_num_threads(cores)
    return {"value": STEPS_PER_SOLVE / med, "unit": "RK4 steps/s (batch 4096)", "cores": cores,
            "physical_cores": phys, "kind": "port",
            "spread": {"best": STEPS_PER_SOLVE / min(ts), "worst": STEPS_PER_SOLVE / max(ts)},
            # the host's cores are shared with other jobs: the median measures contention as much as
            # the reference, so the uncontended best solve is reported beside it
            "best_of_n": {"value": STEPS_PER_SOLVE / min(ts), "n": len(ts),
                          "note": "fastest of the timed solves (least host contention); value is their median"},
            "threads_note": f"{cores} threads = this process's CPU share on the GPU box (16 cores per GPU, "
                            f"OMP_NUM_THREADS; the host has {phys} physical cores shared with other jobs)",
            "sample": f"median of {n_solves} full solves of the bench workload (B=4096, 34 rk4 steps) with "
                      f"oracle/torch_ref.py (reference op order, torch CPU fp32) on {cores} threads: "
                      + ", ".join(f"{x:.2f}" for x in ts) + " s",
            "one_thread": {"value": STEPS_PER_SOLVE / med1, "cores": 1,
                           "per_core_scaled": STEPS_PER_SOLVE / med1 * cores,
                           "sample": f"1 full solve of the bench workload on 1 thread: {ts1[0]:.2f} s"}}, first


def cpu_dopri5_baseline(sd, y0, t, rtol, atol, n_solves=3):
    """The CPU oracle's dopri5 solve (restated torchdiffeq, reference op order) of the LV bench
    workload, measured: B = 4096 at rtol 1e-3 (~1 200 field evaluations; the reference's default
    rtol 1e-7 needs ~35 000, about 10 min on this CPU share), median of `n_solves`."""
    from oracle import torch_ref as O
    cores, phys = cpu_cores()
    torch.set_num_threads(cores)
    ts, nfev = [], None
    with torch.no_grad():
        for _ in range(n_solves):
            ref = O.KANFETRef.from_state_dict(sd, 2)
            tr = O.Dopri5Trace()
            t0 = time.perf_counter()
            O.odeint(lambda tt, yy: ref(yy), y0, t, rtol=rtol, atol=atol, trace=tr)
            ts.append(time.perf_counter() - t0)
            nfev = tr.nfev
    med = float(np.median(ts))
    return {"value": 1.0 / med, "unit": f"dopri5 solves/s (B={y0.shape[0]}, rtol {rtol:g}, atol {atol:g})",
            "cores": cores, "physical_cores": phys, "kind": "port", "nfev": nfev,
            "field_evals_per_s": nfev / med,
            "sample": f"median of {n_solves} full dopri5 solves (B={y0.shape[0]}, rtol {rtol:g}, {nfev} evaluations) "
                      f"with oracle/torch_ref.py (torch CPU fp32) on {cores} threads: "
                      + ", ".join(f"{x:.2f}" for x in ts) + " s"}


def cpu_train_baseline(sd, y0, t, n_iters):
    """The CPU oracle's training iteration (forward with autograd + backward of an MSE over the
    whole (35, 4096, 2) trajectory) on the FULL bench batch, median of `n_iters`.  The Adam update
    (3 052 parameters) is left out."""
    from oracle import torch_ref as O
    cores, phys = cpu_cores()
    torch.set_num_threads(cores)
    target = torch.zeros(T, y0.shape[0], 2)

    def it():
        ps = {k: v.clone().requires_grad_(v.is_floating_point() and "grid" not in k) for k, v in sd.items()}
        ref = O.KANFETRef.from_state_dict(ps, 2)
        sol = O.odeint(lambda tt, yy: ref(yy), y0, t, method="rk4")
        (sol - target).square().mean().backward()

    med, ts = _median_solves(it, n_iters)
    return {"value": STEPS_PER_SOLVE / med, "unit": "RK4 steps/s trained (fwd+bwd, batch 4096)",
            "cores": cores, "physical_cores": phys, "kind": "port",
            "sample": f"median of {n_iters} fwd+bwd iterations of the full bench batch (B=4096, 34 rk4 steps) "
                      f"with oracle/torch_ref.py autograd (torch CPU fp32): " + ", ".join(f"{x:.2f}" for x in ts) + " s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; FETODE_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # fewer GPUs (ranks share devices round-robin; timings are not meaningful then)
    backend = os.environ.get("FETODE_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    strong = args.scaling == "strong"
    model, sd, y0, y0g, t = make_problem(rank, world, args.scaling, dev)
    y0d = y0.to(dev)
    Bl = y0d.shape[0]
    func = F.autonomous(model)

    def solve():
        return F.odeint(func, y0d, t, method="rk4")

    progress(f"headline: rk4 B={Bl} x {args.steps} solves (warm-up {args.warmup})")
    with torch.no_grad():
        # clock settle: the GPU raises its clocks over the first ~100 back-to-back solves (~20 ms:
        # 181 -> 170 us per solve, profiles/r05_clock_ramp.log); a fixed wall time of untimed solves
        # first, so a short warm-up (the driver's W = 5) times the loaded clock like a long one
        settle_n, ts = 0, time.perf_counter()
        while time.perf_counter() - ts < args.settle_s:
            for _ in range(10):
                solve()
            settle_n += 10
            torch.cuda.synchronize(dev)
        settle_s = time.perf_counter() - ts
        for _ in range(args.warmup):
            solve()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sol = solve()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        k_ms = kernel_time_ms(model, y0d, t)
    progress("train")
    train = train_rate(model, y0d, t, args.train_iters, 5, world, strong) if args.train_iters > 0 else None
    other_line = None
    if world > 1:
        # the other scaling mode from the same run: strong = the global seed-0 batch of 4096 split
        # over the ranks; weak = a batch of 4096 per rank (seed = rank)
        import fet_ode_amd.dist as D
        lo, hi = D.shard_bounds(B, rank, world)
        y0s = (lv_y0(B, rank) if strong else lv_y0(B, 0)[lo:hi]).to(dev)
        with torch.no_grad():
            for _ in range(args.warmup):
                F.odeint(func, y0s, t, method="rk4")
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                F.odeint(func, y0s, t, method="rk4")
            torch.cuda.synchronize(dev)
            dist.barrier()
            els = time.perf_counter() - t0
        tt = torch.tensor([els], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        els = tt.item()
        if strong:
            other_line = {"value": world * args.steps * STEPS_PER_SOLVE / els, "ms_per_step": els / args.steps * 1e3,
                          "batch_per_gpu": B, "unit": "RK4 steps/s of the batch-4096 job (4096 per GPU, summed)",
                          "scaling": "weak"}
        else:
            other_line = {"value": args.steps * STEPS_PER_SOLVE / els, "ms_per_step": els / args.steps * 1e3,
                          "batch_per_gpu": hi - lo, "unit": "RK4 steps/s of ONE batch-4096 job split over the GPUs",
                          "scaling": "strong"}
    dp5_sharded = None
    if world > 1 and not args.no_dopri5:
        dp5_sharded = lv_dopri5_sharded_rate(sd, y0d, t, world, B if strong else B * world)
    ms_per_step = el / args.steps * 1e3
    # strong: every solve covers the global batch once; weak: each rank's solve is a batch of its own
    value = (1 if strong else world) * args.steps * STEPS_PER_SOLVE / el

    if rank == 0:
        bytes_launch = alg_bytes_per_step(Bl) * STEPS_PER_SOLVE
        achieved = bytes_launch / (k_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic_per_launch() if Bl == B else (None, None)
        flops_launch = ALG_FLOPS_PER_TRAJ_STEP * Bl * STEPS_PER_SOLVE
        tflops = flops_launch / (k_ms * 1e-3) / 1e12
        out = {
            "metric": METRIC, "value": value,
            "unit": "RK4 steps/s of the batch-4096 job" + (" (global batch split over GPUs)" if strong
                                                          else " (4096 per GPU, summed over GPUs)"),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "clock_settle": {"solves": settle_n, "s": settle_s,
                             "note": "untimed back-to-back solves before the warm-up (GPU clock ramp, DESIGN.md §3)"},
            # a bench "step" is one 34-step odeint solve; per RK4 step of the batch:
            "ms_per_rk4_step": ms_per_step / STEPS_PER_SOLVE,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded y0, torch.manual_seed(0) weights; no dataset)",
            "config": {"workload": "LV KAN-FET NODE: KANFET[2,10,2] G=5 k=3 nb=10 K=10, rk4 (3/8), "
                                   + (f"global B=4096 split {world} ways" if strong else "B=4096 per GPU")
                                   + ", t=linspace(0,3.5,35) -> 34 steps per solve",
                       "batch_per_gpu": Bl, "global_batch": B if strong else B * world,
                       "rk4_steps_per_solve": STEPS_PER_SOLVE,
                       "parallelism": f"trajectory-sharded x{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ("fused4_kernel<10,10,10,12,true,true,false,false,2> (v7 rk4, two trajectories per wave)"
                                    if Bl > 1024 else
                                    "fused4_kernel<10,10,10,12,true,true,false,false,1> (v7 rk4, one trajectory per wave)"
                                    if Bl > 512 else
                                    "v8_kernel<true,2> (v8 rk4, one trajectory per two waves, two per workgroup)"
                                    if Bl > 256 else "small6_kernel<true,true,false,false> (v6 small-batch rk4 path)"),
                         "kernel_ms": k_ms, "alg_bytes_per_launch": bytes_launch,
                         "traffic_source": traffic_src,
                         "valu": {"achieved_tflops": tflops, "peak_tflops": FP32_PEAK_TFLOPS,
                                  "frac": tflops / FP32_PEAK_TFLOPS,
                                  "alg_flops_per_launch": flops_launch},
                         # the kernel's actual bound: the SIMDs' VALU issue (PMC, committed profile)
                         "issue": (pmc_issue("fused4_kernel<10, 10, 10, 12, true, true, false, false, 2>")
                                   or pmc_issue("fused4_kernel<10, 10, 10, 12, true, true, false, false>")) if Bl > 1024
                                  else pmc_issue("fused4_kernel<10, 10, 10, 12, true, true, false, false, 1>") if Bl > 512
                                  else pmc_issue("v8_kernel<true, 2>") if Bl > 256
                                  else pmc_issue("small6_kernel<true, true, false, false>")},
            # north_star: "MFMA utilisation against chip peak" — the path's MFMA kernels (the LV field
            # itself has no GEMM-shaped work): the ETT wide KAN-FET layer and the MNIST
            # KANLinear head, from the committed PMC pass (tools/pmc_issue.py)
            "mfma": {k: pmc_mfma(k) for k in ("wide_layer_kernel<10, true, true, 8>", "wide_fwd4_kernel")},
        }
        if world == 1:
            # strong-scaling proxy on one GPU: the per-GPU block of an 8-GPU strong-scaled job
            y512 = y0d[:B // 8].contiguous()
            kb = kernel_time_ms(model, y512, t)
            out["strong_proxy_ms_b512"] = kb
            st_wall, st_issue = solve_stream_ms(model, y512, t)
            out["strong_proxy"] = {"kernel_ms_b4096": k_ms, "kernel_ms_b512": kb, "ratio_b512_over_b4096": kb / k_ms,
                                   "solve_ms_b4096": solve_ms(model, y0d, t), "solve_ms_b512": solve_ms(model, y512, t),
                                   "solve_ms_b512_streamed": st_wall, "host_issue_ms_b512": st_issue,
                                   "note": "B=512 = the per-GPU block of the 8-GPU strong-scaled job; kernel by HIP "
                                           "events, solve = host wall of one synchronised odeint call (median); "
                                           "streamed = per-call wall of 50 calls issued back to back and drained "
                                           "once, host_issue = the host's own time per call in that stream"}
        if other_line is not None:
            out[other_line["scaling"] + "_scaling"] = other_line
        if train is not None:
            out["train"] = train
        if world == 1:
            progress("plain closure")
            out["lv_plain_closure"] = plain_closure_rate(model, y0d, t)
        if world == 1 and not args.no_dopri5:
            progress("lv dopri5")
            out["lv_dopri5"] = lv_dopri5_rate(sd, y0d, t)
            out["lv_dopri5"]["rtol_1e-3"] = lv_dopri5_rate(sd, y0d, t, reps=5, rtol=1e-3, atol=1e-4)
            progress("lv dopri5 training")
            tr = lv_dopri5_train_rate(sd, y0d, t)
            tr["host_autograd"] = lv_dopri5_train_rate(sd, y0d, t, iters=1, resident=False)
            tr["speedup_vs_host_autograd"] = tr["value"] / tr["host_autograd"]["value"]
            # the reference's defaults (rtol 1e-7 / atol 1e-9): B = 4096, and its own iteration's
            # shape, one trajectory from X0 = (1, 1) (train_kanfet_node_predprey.py:49,149,252-257;
            # synthetic zero target)
            tr["default_tol_b4096"] = lv_dopri5_train_rate(sd, y0d, t, iters=2, rtol=1e-7, atol=1e-9)
            tr["reference_iteration"] = lv_dopri5_train_rate(
                sd, torch.tensor([[1.0, 1.0]], device=y0d.device), t, iters=5, rtol=1e-7, atol=1e-9)
            out["lv_dopri5"]["train"] = tr
        if dp5_sharded is not None:
            out["lv_dopri5"] = dp5_sharded
        if world == 1 and not args.no_ecg:
            progress("ecg")
            out["ecg"] = ecg_rate(dev, with_cpu=not args.no_cpu_baseline)
            out["ecg"]["rtol_1e-2"] = ecg_rate(dev, with_cpu=False, rtol=1e-2, atol=1e-3)
        if world == 1 and not args.no_mnist:
            progress("mnist")
            out["mnist"] = mnist_rate(dev, with_cpu=not args.no_cpu_baseline)
        if world == 1 and not args.no_ett:
            progress("ett rk4 forecaster")
            out["ett"] = ett_rate(dev, batch=args.ett_batch, with_cpu=not args.no_cpu_baseline)
            progress("ett encoder")
            out["ett"]["encoder"] = ett_encoder_rate(dev, with_cpu=not args.no_cpu_baseline)
            progress("ett dopri5")
            out["ett"]["dopri5"] = ett_dopri5_rate(dev, batch=args.ett_batch)
            progress("ett dopri5 training")
            out["ett"]["dopri5"]["train"] = ett_dopri5_train_rate(dev)
            if args.ett_ref_iters > 0:
                progress("ett reference iteration (dopri5 rtol 1e-7, ~1 min)")
                out["ett"]["dopri5"]["train"]["reference_iteration"] = ett_reference_iteration_rate(
                    dev, iters=args.ett_ref_iters)
        if world == 1 and not args.no_cpu_baseline:
            progress("cpu baseline + parity")
            cb, ref_sol = cpu_baseline(sd, y0, t, args.cpu_solves)
            out["cpu_baseline"] = cb
            if "lv_dopri5" in out:
                # measured on the same workload at rtol 1e-3 (the default rtol 1e-7 solve is ~35 000
                # evaluations, ~10 min on the CPU share); the GPU line at rtol 1e-3 sits beside it
                out["lv_dopri5"]["rtol_1e-3"]["cpu_baseline"] = cpu_dopri5_baseline(sd, y0, t, 1e-3, 1e-4)
            if train is not None:
                out["train"]["cpu_baseline"] = cpu_train_baseline(sd, y0, t, 3)
            fresh = F.KANFET([2, 10, 2], grid_size=5)
            fresh.load_state_dict(sd)          # fresh hysteresis state, as the CPU solve had
            with torch.no_grad():
                sol = F.odeint(F.autonomous(fresh.to(dev)), y0d, t, method="rk4")
                from oracle import torch_ref as O
                r64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
                e64 = O.odeint(lambda tt, yy: r64(yy), y0.double(), t, method="rk4")
            from oracle import parity as P
            runs = P.perturbed_solves(sd, y0, t, 5)
            robust = P.robust_parity(sol.cpu(), ref_sol, e64, runs[:3], runs[3:])
            g = sol.cpu().double()
            r = ref_sol.double()
            out["parity"] = {
                "traj_mse_vs_cpu_ref": ((g - r) ** 2).mean().item(),
                "max_slice_rel_vs_cpu_ref": ((g - r).reshape(T, -1).norm(dim=1)
                                             / r.reshape(T, -1).norm(dim=1)).max().item(),
                "cpu_ref_fp32_vs_fp64_max_slice_rel": ((r - e64).reshape(T, -1).norm(dim=1)
                                                       / e64.reshape(T, -1).norm(dim=1)).max().item(),
                "robust_subset": robust,
                "robust_subset_ok": P.robust_parity_ok(robust),
                "robust_subset_at_1e-5_ok": P.robust_parity_at_tol_ref_ok(robust),
                "note": "KAN-FET is ill-conditioned in fp32: the CPU reference's own fp32 solve departs from "
                        "fp64 by the per-slice error above, and which trajectories stay within 1e-5 depends on "
                        "the rounding; the 1e-5 bar is checked on the trajectories every equally valid "
                        "reference rounding keeps within 1e-5 (robust_subset, oracle/parity.py; DESIGN.md §2)",
            }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
