"""World-size-2 (and 3) gloo rehearsal of the slab decomposition on CPU.

Each rank owns planes [Lz*r/P, Lz*(r+1)/P) plus two ghost planes, exchanges
faces with its z-neighbours exactly as the RCCL path does (send top -> up,
send bottom -> down, recv lower ghost <- down, recv upper ghost <- up;
periodic wrap), and steps its slab with the oracle's slab update.  After k
steps the gathered field must equal the single-process run bit for bit: the
noise is keyed by the global site and step, so the decomposition cannot
change a single bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, shape, steps, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    sys.path.insert(0, os.path.dirname(here))
    import torch
    import oracle
    from stochquant_amd.decomp import slab_bounds, neighbours
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Lx, Ly, Lz = shape
        p = oracle.phi4_params(shape, 0.02, 0.5, 1.0, 11)
        full = oracle.phi4_init(p, 0.8)
        z0, z1 = slab_bounds(Lz, world, rank)
        nz = z1 - z0
        pad = np.zeros((nz + 2, Ly, Lx), np.float32)
        pad[1:-1] = full[z0:z1]
        up, dn = neighbours(world, rank)
        for s in range(steps):
            top = torch.from_numpy(pad[nz].copy())
            bot = torch.from_numpy(pad[1].copy())
            lo = torch.empty_like(top)
            hi = torch.empty_like(top)
            if world == 1:
                lo.copy_(top)
                hi.copy_(bot)
            else:
                ops = [dist.P2POp(dist.isend, top, up), dist.P2POp(dist.isend, bot, dn),
                       dist.P2POp(dist.irecv, lo, dn), dist.P2POp(dist.irecv, hi, up)]
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
            pad[0] = lo.numpy()
            pad[nz + 1] = hi.numpy()
            pad[1:-1] = oracle.phi4_step_slab(p, pad, z0, s)
        gathered = [torch.zeros(1) for _ in range(world)]
        dist.all_gather_object(gathered, (z0, pad[1:-1].copy()))
        if rank == 0:
            gathered.sort(key=lambda t: t[0])
            q.put(np.concatenate([g[1] for g in gathered]))
    finally:
        dist.destroy_process_group()


def _monolithic(shape, steps):
    import oracle
    p = oracle.phi4_params(shape, 0.02, 0.5, 1.0, 11)
    phi = oracle.phi4_init(p, 0.8)
    for s in range(steps):
        phi = oracle.phi4_step(p, phi, s)
    return phi


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_slab_exchange_bitwise(world, oracle_mod):
    shape, steps = (16, 8, 12), 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(got, _monolithic(shape, steps))


def test_slab_bounds_cover_lattice():
    from stochquant_amd.decomp import slab_bounds
    for Lz in (1, 7, 256, 1024):
        for P in range(1, min(Lz, 9) + 1):
            b = [slab_bounds(Lz, P, r) for r in range(P)]
            assert b[0][0] == 0 and b[-1][1] == Lz
            assert all(b[i][1] == b[i + 1][0] for i in range(P - 1))
            assert all(z1 > z0 for z0, z1 in b)
