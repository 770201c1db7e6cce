"""Trajectory-sharded data parallelism over the GPUs of one node.

The reference runs one process on one device and never communicates.  Here the
batch of trajectories is split into contiguous blocks, one per rank (one process per GPU,
``torch.distributed`` with the "nccl" backend = RCCL over xGMI).  The forward solve needs no
communication: every trajectory and its hysteresis state (ferro_class.py:373-378, per sample)
live on one rank.  Training adds ONE all-reduce per iteration: all parameter gradients
flattened into a single fp32 bucket (12.2 KB for KANFET [2,10,2]) — a latency-bound message
on xGMI, so one fused bucket and no pipelining.

Adaptive solves (dopri5) shard too, with one exchange: the error ratio torchdiffeq tests is the
RMS over the WHOLE batch, so ``odeint_sharded`` all-reduces two fp64 words (sum of squares,
non-finite flag) per norm — 3 in the initial step selection, 1 per attempt — and every rank
takes the step sequence a single device would take on the global batch (SURVEY §8e caveat 2).
Under autograd the backward all-reduces those norms' adjoints too (the gradient through the
adaptive step sizes has cross-rank terms).

Caveat kept from the reference semantics: a fresh FerroelectricBasis re-initialises prev_x
(dx = 0) on its first call unless the batch is 1 (ferro_class.py:373-375).  Sharding a global
batch B > 1 into shards of size 1 would flip that rule, so ``shard_bounds`` refuses it.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(global_batch: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) block of the global batch for ``rank`` (sizes differ by at most 1)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("bad rank/world")
    base, rem = divmod(global_batch, world_size)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    if global_batch > 1 and (hi - lo) == 1:
        raise ValueError("a shard of 1 trajectory would flip FerroelectricBasis' first-call rule "
                         "(ferro_class.py:373-375); use fewer ranks or a larger batch")
    if hi <= lo:
        raise ValueError("more ranks than trajectories")
    return lo, hi


def shard(x: torch.Tensor, rank: Optional[int] = None, world_size: Optional[int] = None, dim: int = 0):
    r, w = world()
    rank = r if rank is None else rank
    world_size = w if world_size is None else world_size
    lo, hi = shard_bounds(x.shape[dim], rank, world_size)
    return x.narrow(dim, lo, hi - lo)


def allreduce_gradients(params: Iterable[torch.nn.Parameter], average: bool = True,
                        weights: Optional[float] = None) -> None:
    """Sum (or average) the gradients of ``params`` over ranks in ONE flat all-reduce.

    ``weights``: this rank's share of the global batch (e.g. B_local / B_global) when the loss
    is a per-rank mean over unequal shards; the result is then the global-mean gradient.
    """
    _, w = world()
    grads: List[torch.Tensor] = [p.grad for p in params if p.grad is not None]
    if w == 1 or not grads:
        return
    flat = _shared_flat(grads)
    views = flat is not None   # the gradients already are views of one buffer (fused backward)
    if not views:
        flat = torch._utils._flatten_dense_tensors(grads)
    if weights is not None:
        flat.mul_(weights)
    # RCCL ("nccl") reduces device buffers in place; gloo (CPU tests, several ranks on one GPU)
    # reduces a host copy
    host = flat.is_cuda and dist.get_backend() != "nccl"
    buf = flat.cpu() if host else flat
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    if host:
        flat.copy_(buf)
    if weights is None and average:
        flat.div_(w)
    if not views:
        for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
            g.copy_(f)


def _shared_flat(grads: List[torch.Tensor]) -> Optional[torch.Tensor]:
    """A flat view of the one storage run the gradients tile exactly, in order, or None.

    Compared by storage, not by ``._base``: AccumulateGrad stores ``new_grad.detach()``, whose
    ``_base`` is None although it still aliases the fused backward's flat buffer.
    """
    g0 = grads[0]
    st = g0.untyped_storage()
    start = off = g0.storage_offset()
    for g in grads:
        if (g.dtype != g0.dtype or g.device != g0.device or not g.is_contiguous()
                or g.untyped_storage().data_ptr() != st.data_ptr() or g.storage_offset() != off):
            return None
        off += g.numel()
    return g0.new_empty(0).set_(st, start, (off - start,))


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank's parameters and persistent buffers rank `src`'s, in place (what DDP does
    at construction).  Needed before data-parallel training: the efficient_kan init the drop-ins
    reproduce (curve2coeff's lstsq) is not bitwise reproducible across processes even with the
    same seed, so ranks that each construct the model start from slightly different weights.

    Non-persistent buffers are per-rank state and are NOT broadcast: FerroelectricBasis' compact
    hysteresis memory (`_prev`, `_bsign`, shape (B_local, in)) belongs to this rank's own
    trajectories, and unequal shards would give the collective mismatched sizes.  Persistent
    buffers a module lists in ``_rank_local_buffers`` are batch state too (the ECG hysteretic
    LogisticBasis' prev_x / branch_state, rebound to (B, in, nb) per call) and stay local."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    shared = list(module.parameters())
    for mod in module.modules():
        skip = set(mod._non_persistent_buffers_set) | set(getattr(mod, "_rank_local_buffers", ()))
        shared += [b for n, b in mod.named_buffers(recurse=False) if n not in skip and b is not None]
    with torch.no_grad():
        for t in shared:
            buf = t.detach() if t.device == dev else t.detach().to(dev)
            dist.broadcast(buf, src=src, group=group)
            if buf is not t:
                t.copy_(buf)


class XRank:
    """The cross-rank exchange of a trajectory-sharded device-resident dopri5
    (fetode_integrate_dopri5_xrank): this rank's inbox (device memory, IPC-exported) and every
    peer's inbox mapped into this process, as a device array of pointers the kernel's exchange
    workgroup writes through (remote stores over xGMI).  One per (group, device); created
    collectively (all_gather of the 64-byte IPC handles) the first time a sharded resident solve
    runs.  Mappings live until the process exits.

    Fail-safe: the inbox must be fine-grained device memory (fetode_xrank_alloc refuses a
    coarse-grained fallback) and every peer's inbox must map.  Both outcomes are agreed over the
    group, so ``ok`` is the same on every rank: when it is False every rank declines the resident
    sharded path and takes the host-driven loop (one all-reduce per attempt) together."""

    _cache: dict = {}

    @classmethod
    def get(cls, group, device) -> "XRank":
        key = (id(group) if group is not None else None, torch.device(device).index)
        x = cls._cache.get(key)
        if x is None:
            x = cls._cache[key] = cls(group, device)
        return x

    def __init__(self, group, device):
        import ctypes
        from . import _lib
        lib = _lib.load()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        nbytes = lib.fetode_xrank_inbox_bytes(self.world)
        if nbytes < 0:
            raise ValueError(f"sharded resident dopri5: world size {self.world} not supported")
        ptr = ctypes.c_void_p()
        handle = (ctypes.c_uint8 * 64)()
        self.ok, self.reason = False, None
        self.inbox, self.peers, self.epoch = None, None, 0
        with torch.cuda.device(device):
            rc = lib.fetode_xrank_alloc(nbytes, ctypes.byref(ptr), handle)
            mine = bytes(handle) if rc == _lib.FETODE_OK else None
            if mine is None:
                self.reason = _lib.last_error()
            handles = [None] * self.world
            dist.all_gather_object(handles, mine, group=group)   # reached by every rank, failed or not
            opened, ok_open = [], mine is not None and all(h is not None for h in handles)
            if ok_open:
                for j, h in enumerate(handles):
                    if j == self.rank:
                        opened.append(ptr.value)
                        continue
                    hb = (ctypes.c_uint8 * 64).from_buffer_copy(h)
                    q = ctypes.c_void_p()
                    if lib.fetode_xrank_open(hb, ctypes.byref(q)) != _lib.FETODE_OK:
                        self.reason = _lib.last_error()
                        ok_open = False
                        break
                    opened.append(q.value)
            flags = [None] * self.world
            dist.all_gather_object(flags, bool(ok_open), group=group)
            if not all(flags):
                # release what this rank holds: the peer mappings opened so far and its own inbox
                # (the failed XRank stays cached with ok = False for the life of the process)
                for j, q in enumerate(opened):
                    if j != self.rank and q:
                        lib.fetode_xrank_close(ctypes.c_void_p(q))
                if ptr.value:
                    lib.fetode_xrank_free(ptr)
        if not all(flags):
            self.reason = self.reason or "a peer could not allocate or map its inbox"
            return
        self.ok = True
        self.inbox = ptr.value
        self.peers = torch.tensor(opened, dtype=torch.int64, device=device)

    def desc(self, b_offset: int):
        from . import _lib
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF or 1
        return _lib.XRankDesc(self.rank, self.world, self.epoch, self.inbox, self.peers.data_ptr(), int(b_offset))


import os as _os

# FETODE_RESIDENT_SHARDED=0: the host-driven loop (e.g. when several ranks share ONE GPU, whose
# resident grids together would not be co-resident)
_RESIDENT_SHARDED = [_os.environ.get("FETODE_RESIDENT_SHARDED", "1") != "0"]


def set_resident_sharded(enabled: bool) -> bool:
    """Sharded dopri5 solves of fused fields in one launch per rank with the in-kernel cross-rank
    exchange (default), or the host-driven loop with one all-reduce per attempt."""
    prev, _RESIDENT_SHARDED[0] = _RESIDENT_SHARDED[0], bool(enabled)
    return prev


def resident_agreement(group, device, local_batch: int, ok: bool) -> Optional[Tuple[int, int]]:
    """One all-gather: (global batch, this rank's offset in it), or None unless every rank can take
    the resident path (all ranks must take the same one: their kernels exchange with each other)."""
    cpu = dist.get_backend(group) != "nccl"
    t = torch.tensor([float(local_batch), 1.0 if ok else 0.0], dtype=torch.float64,
                     device="cpu" if cpu else device)
    w = dist.get_world_size(group)
    out = [torch.empty_like(t) for _ in range(w)]
    dist.all_gather(out, t, group=group)
    rows = [o.tolist() for o in out]
    if not all(int(r[1]) for r in rows):
        return None
    r = dist.get_rank(group)
    return int(sum(x[0] for x in rows)), int(sum(x[0] for x in rows[:r]))


def odeint_sharded(func, y0_local: torch.Tensor, t: torch.Tensor, *, rtol=1e-7, atol=1e-9, method=None,
                   options: Optional[dict] = None, group=None):
    """odeint over this rank's shard of a trajectory-sharded batch.  Fixed-grid methods need no
    communication; adaptive ones use the global-batch error norm (all ranks, same steps).

    Without autograd, a fused field (fet_ode_amd.autonomous / the plain calDeriv closure) solves
    in ONE launch per rank with the norms exchanged between the ranks' kernels
    (fetode_integrate_dopri5_xrank, XRank); otherwise the host-driven loop all-reduces them.

    Training through dopri5: the norm's gradient is all-reduced in the backward
    (dopri5._NormAllReduce), so rank r's parameter gradient holds its trajectories' share of
    every cross-rank term.  Write the loss as this shard's share of the GLOBAL loss (e.g.
    ``sum_local / N_global`` for a global mean) and sum with ``allreduce_gradients(average=False)``;
    for equal shards a per-rank mean with ``weights=B_local / B`` is the same thing."""
    from .odeint import odeint
    opts = dict(options or {})
    _, w = world()
    if w > 1 and (method is None or method == "dopri5"):
        opts["norm_group"] = "world" if group is None else group
    return odeint(func, y0_local, t, rtol=rtol, atol=atol, method=method, options=opts)
