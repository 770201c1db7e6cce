"""Sharded resident dopri5 determinism check (2 ranks on cuda:0): the single-device solve twice, the
sharded solve twice per rank; prints the first attempt where any two differ."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
B = int(os.environ.get("B", 2048))
RTOL = float(os.environ.get("RTOL", 1e-7))


def problem(F):
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to("cuda:0")
    g = torch.Generator().manual_seed(0)
    y0 = (0.5 + 2.5 * torch.rand(B, 2, generator=g)).to(torch.float32)
    return m, y0, torch.tensor(np.linspace(0, 3.5, 35))


def solve(F, m, y0, t, sharded):
    import fet_ode_amd.dist as D
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    outs = []
    for _ in range(2):
        m.load_state_dict(sd)
        with torch.no_grad():
            if sharded:
                sol = D.odeint_sharded(F.autonomous(m), D.shard(y0).to("cuda:0"), t, rtol=RTOL, atol=RTOL * 1e-2)
            else:
                sol = F.odeint(F.autonomous(m), y0.to("cuda:0"), t, rtol=RTOL, atol=RTOL * 1e-2)
        s = F.dopri5.dopri5_solve.last
        outs.append((sol.cpu().numpy(), [tuple(a) for a in s.attempts], s.nfev))
    return outs


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    return None if len(a) == len(b) else (min(len(a), len(b)), "len", (len(a), len(b)))


def worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import fet_ode_amd as F
    m, y0, t = problem(F)
    q.put((rank, solve(F, m, y0, t, True)))
    dist.destroy_process_group()


if __name__ == "__main__":
    import fet_ode_amd as F
    m, y0, t = problem(F)
    single = solve(F, m, y0, t, False)
    print("single run-to-run:", first_diff(single[0][1], single[1][1]), "attempts", len(single[0][1]))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        print(f"rank {r} run-to-run:", first_diff(res[r][0][1], res[r][1][1]))
    print("rank0 vs rank1:", first_diff(res[0][0][1], res[1][0][1]))
    print("sharded vs single:", first_diff(res[0][0][1], single[0][1]))
    sol = np.concatenate([res[0][0][0], res[1][0][0]], 1)
    print("solution bitwise equal:", np.array_equal(sol, single[0][0]),
          "max abs diff", float(np.abs(sol - single[0][0]).max()))
