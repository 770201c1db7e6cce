"""Data-parallel training of the MNIST and ETT models (SURVEY §8e caveat 4, BASELINE configs[3] and
[4] "sharded 8x"): 2 ranks on cuda:0, gloo carrying the collectives (the driver's 8-GPU node runs
RCCL).  Each rank takes its contiguous shard of the global batch (fet_ode_amd.dist.shard), runs the
forward and backward on its own HIP kernels, and all-reduces the gradients in ONE flat bucket
(allreduce_gradients with this shard's share of the global mean); every rank must then hold the
single-device gradient of the global batch, and one Adam step must leave the ranks' weights equal.

* MNIST KuramotoKANClassifier (mnist_kuramoto_kan.py:202-283): 28 x 28 synthetic images, cross
  entropy — the ~307 k-parameter gradient bucket (1.2 MB) that SURVEY §8e caveat 4 names;
* the ETT LatentNeuralODEForecaster (train_kan_fet_ett.py:155-197, 320-335) with the KAN-FET latent
  field at the production widths (latent 64, KANFET[64, 128, 64]) through odeint_rk4, MSE loss.

Tolerance: the sharded gradient sums the same per-row terms in another order (per rank, then the
all-reduce), so it equals the single-device one to fp32 summation noise: 1e-5 relative (flat norm)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu

N_MNIST, N_ETT = 64, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mnist(dev):
    from fet_ode_amd import mnist
    torch.manual_seed(0)
    m = mnist.KuramotoKANClassifier()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(N_MNIST, 1, 28, 28, generator=g)
    y = torch.arange(N_MNIST) % 10
    return m, x, y


def _ett(dev):
    from fet_ode_amd import ett
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=24, pred_len=4, latent_dim=64, solver="rk4")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N_ETT, 24, 7, generator=g) * 0.5
    y = torch.randn(N_ETT, 4, generator=g)
    return m, x, y


def _loss(case, m, x, y, dev):
    if case == "mnist":
        return torch.nn.functional.cross_entropy(m(x.to(dev)), y.to(dev))
    t = torch.linspace(0.0, 0.3, steps=4, device=dev)
    return torch.mean((m(x.to(dev), t, rk4_substeps=2) - y.to(dev)) ** 2)


def _flat_grads(m):
    return torch.cat([p.grad.detach().double().cpu().reshape(-1) for p in m.parameters()])


def _worker(rank, world, port, q, case, sd):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import fet_ode_amd.dist as D
        dev = torch.device("cuda:0")
        m, x, y = (_mnist if case == "mnist" else _ett)(dev)
        m.load_state_dict(sd)          # the parent's weights (the efficient_kan init is per-process)
        m = m.to(dev)
        D.broadcast_parameters(m)
        xs, ys = D.shard(x), D.shard(y)
        loss = _loss(case, m, xs, ys, dev)
        loss.backward()
        D.allreduce_gradients(list(m.parameters()), weights=xs.shape[0] / x.shape[0])
        g = _flat_grads(m)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        opt.step()
        w = torch.cat([p.detach().double().cpu().reshape(-1) for p in m.parameters()])
        q.put((rank, g.numpy(), w.numpy()))   # numpy: the worker may exit before the parent reads
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["mnist", "ett"])
def test_data_parallel_training_matches_single_device(dev, case):
    m, x, y = (_mnist if case == "mnist" else _ett)(dev)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    _loss(case, m, x, y, dev).backward()
    ref = _flat_grads(m)
    assert torch.isfinite(ref).all() and ref.norm() > 0
    if case == "mnist":
        assert ref.numel() > 300_000      # the ~307 k-parameter bucket of SURVEY §8e caveat 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, case, sd)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, w0), (_, g1, w1) = [(r, torch.from_numpy(a), torch.from_numpy(b)) for r, a, b in res]
    assert torch.equal(g0, g1) and torch.equal(w0, w1)     # every rank: the same gradient and step
    rel = ((g0 - ref).norm() / ref.norm()).item()
    assert rel <= 1e-5, rel
