"""bench.py's transport fallback (open_with_fallback) on a gloo world of 2-3
CPU ranks: when the primary transport (RCCL) fails to come up on ANY rank,
every rank closes what it opened and opens the fallback (P2P) together, and
each reports why; when it comes up everywhere, nobody falls back.  The
"lattices" are stand-ins that record what happened to them."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Fake:
    def __init__(self, kind):
        self.kind, self.closed = kind, False

    def close(self):
        self.closed = True


def _worker(rank, world, port, failing, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    opened = []

    def primary():
        if rank in failing:
            raise RuntimeError(f"rank {rank}: comm init timed out")
        f = _Fake("rccl")
        opened.append(f)
        return f

    try:
        lat, why = bench.open_with_fallback(primary, lambda: _Fake("p2p"), world, dist)
        q.put((rank, lat.kind, why, [f.closed for f in opened]))
    finally:
        dist.destroy_process_group()


def _run(world, failing):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, failing, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return sorted(q.get(timeout=5) for _ in range(world))


@pytest.mark.parametrize("world,failing", [(2, {1}), (3, {0}), (3, {0, 2})])
def test_one_failing_rank_moves_every_rank_to_the_fallback(world, failing):
    for rank, kind, why, closed in _run(world, failing):
        assert kind == "p2p"
        if rank in failing:
            assert "timed out" in why and closed == []
        else:
            assert why == "the primary transport failed on another rank" and closed == [True]


def test_no_failure_keeps_the_primary():
    for rank, kind, why, closed in _run(2, set()):
        assert kind == "rccl" and why is None and closed == [False]
