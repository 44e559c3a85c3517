"""Multi-rank CPU rehearsal (gloo, world size 1-3) of the product's deep-halo
slab exchange.

Each rank owns planes [Lz*r/P, Lz*(r+1)/P) plus a ghost zone of G planes on
either side in two padded ping-pong buffers, exactly as create_phi4 lays them
out, and executes the product's own schedule (`sq_phi4_block_plan`, the list
phi4_block in csrc/sq_api.cpp runs on the GPU):

* EXCHANGE: the G top planes to rank r+1, the G bottom planes to rank r-1,
  lower ghosts from r-1, upper ghosts from r+1, in the product's ncclSend /
  ncclRecv order (with P = 2 both neighbours are the same peer);
* STEP ranges that shrink through the ghost zone, the step-0 core/rim split,
  the last step's edge planes first;
* PAIR: two steps in one launch (phi4_tb2_kernel) over [lo, hi) reading
  [lo-2, hi+2) -- rehearsed as step s on [lo-1, hi+1) into a scratch slab
  and step s+1 on [lo, hi);
* the ghost depth chosen by the max-reduced trial times (one all-reduce, then
  sq_phi4_pick_ghost on every rank).

Every plane outside what the schedule writes starts as NaN, so a range that
reads a stale or never-written plane shows up as a clamped site.  After the
steps the gathered field must equal the single-process oracle run bit for
bit: the noise is keyed by global site and step, so the decomposition cannot
change a single bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

SHAPE = (16, 8, 36)
DT, M2, LAM, SEED = 0.02, 0.5, 1.0, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exchange(bufs, cur, nz, G, world, up, dn):
    """The product's halo exchange (sq_api.cpp phi4_block, RCCL branch)."""
    import torch
    b = bufs[cur]
    top = torch.from_numpy(b[G + nz - G:G + nz].copy())   # my top G planes -> up
    bot = torch.from_numpy(b[G:2 * G].copy())             # my bottom G planes -> down
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
    b[0:G] = lo.numpy()
    b[G + nz:G + nz + G] = hi.numpy()


def _ranges(op):
    r = [(op["lo"], op["hi"])]
    if op["lo2"] < op["hi2"]:
        r.append((op["lo2"], op["hi2"]))
    return r


def _run_block(oracle, p, plan, bufs, cur, nz, G, z0, step0, world, up, dn):
    """Execute one block's schedule as phi4_block does: consecutive STEP or
    PAIR ops of one step form a group that reads the latest buffer and writes
    the other; returns the buffer holding the result."""
    inb, flip, gstep, gkind = cur, False, -1, None
    for op in plan:
        k = op["op"]
        if k == "exchange":
            _exchange(bufs, cur, nz, G, world, up, dn)
        elif k in ("step", "pair"):
            if op["step"] != gstep or k != gkind:
                if flip:
                    inb ^= 1
                flip, gstep, gkind = True, op["step"], k
            s = step0 + op["step"]
            for lo, hi in _ranges(op):
                if k == "step":
                    oracle.phi4_step_range(p, bufs[inb], bufs[inb ^ 1], G, lo, hi, z0, s)
                else:   # two steps in one launch: step s on [lo-1, hi+1) into scratch, s+1 on [lo, hi)
                    mid = np.full_like(bufs[inb], np.nan)
                    oracle.phi4_step_range(p, bufs[inb], mid, G, lo - 1, hi + 1, z0, s)
                    oracle.phi4_step_range(p, mid, bufs[inb ^ 1], G, lo, hi, z0, s + 1)
        else:
            assert k in ("wait_exchange", "edges_done", "wait_staged")
    return inb ^ 1 if flip else inb


def _worker(rank, world, port, steps, fuse2, edge_first, gpad, q, core_pairs=1):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    sys.path.insert(0, os.path.dirname(here))
    import torch
    import oracle
    from stochquant_amd.decomp import block_plan, neighbours, pick_ghost, slab_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Lx, Ly, Lz = SHAPE
        p = oracle.phi4_params(SHAPE, DT, M2, LAM, SEED)
        full = oracle.phi4_init(p, 0.8)
        z0, z1 = slab_bounds(Lz, world, rank)
        nz = z1 - z0
        up, dn = neighbours(world, rank)
        # ghost-depth trial: per-rank times differ; the max over ranks picks one G everywhere
        cands = [g for g in (1, 2, 4, 8) if g <= gpad]
        ms = torch.tensor([1.0 / g + 0.01 * g + 0.001 * ((rank * 7 + i) % 3) for i, g in enumerate(cands)],
                          dtype=torch.float64)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        G = cands[pick_ghost(ms.tolist())]
        # padded ping-pong slabs: allocated depth gpad, active depth G (the product keeps
        # the allocation and uses the first G planes either side); NaN where nothing valid is
        bufs = [np.full((nz + 2 * G, Ly, Lx), np.nan, np.float32) for _ in range(2)]
        bufs[0][G:G + nz] = full[z0:z1]
        cur, done = 0, 0
        while done < steps:
            g = min(G, steps - done)
            plan = block_plan(nz, G, g, fuse2, edge_first, core_pairs)
            cur = _run_block(oracle, p, plan, bufs, cur, nz, G, z0, done, world, up, dn)
            done += g
        gathered = [None for _ in range(world)]
        dist.all_gather_object(gathered, (z0, G, bufs[cur][G:G + nz].copy()))
        if rank == 0:
            gathered.sort(key=lambda t: t[0])
            q.put(([g[1] for g in gathered], np.concatenate([g[2] for g in gathered])))
    finally:
        dist.destroy_process_group()


def _monolithic(steps):
    import oracle
    p = oracle.phi4_params(SHAPE, DT, M2, LAM, SEED)
    phi = oracle.phi4_init(p, 0.8)
    for s in range(steps):
        phi = oracle.phi4_step(p, phi, s)
    return phi


@pytest.mark.parametrize("world,steps,fuse2,edge_first,gpad,core_pairs", [
    (2, 11, True, True, 4, 1),    # P = 2: both neighbours the same peer; partial last block (11 = 4+4+3)
    (3, 11, True, True, 4, 1),
    (2, 9, False, True, 4, 1),    # per-step inner launches
    (3, 8, True, False, 4, 1),    # edges not first
    (2, 9, True, True, 8, 1),     # deeper zone: pairs over 2 ghost planes
    (2, 12, True, True, 2, 1),    # G = 2: blocks of one core/rim step and one edges-first step
    (3, 10, True, True, 8, 1),    # G = 8 over slabs of 12 planes: rims of 8 planes, no edge split
    (1, 7, True, True, 4, 1),     # single rank, self-exchange
    (2, 17, True, True, 8, 2),    # two core pairs ahead of the exchange
    (2, 19, True, True, 8, 4),    # every pair of the block split into core and rim
    (3, 11, True, False, 8, 3),   # three core pairs, slabs of 12 planes (the core shrinks to 4)
])
def test_gloo_deep_halo_blocks_bitwise(world, steps, fuse2, edge_first, gpad, core_pairs, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, fuse2, edge_first, gpad, q, core_pairs))
             for r in range(world)]
    for p in procs:
        p.start()
    ghosts, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(set(ghosts)) == 1, f"ranks picked different ghost depths {ghosts}"
    ref = _monolithic(steps)
    assert not np.isnan(got).any()
    assert np.array_equal(got, ref), f"max diff {np.nanmax(np.abs(got - ref))}"


def test_block_plan_shapes():
    """The schedule's ranges: fused blocks pair every step --
    a core pair overlapping the exchange, a rim pair after it, pairs over the
    shrinking ghost range, the last pair edges first; unfused blocks split
    step 0 into core and rim and run the rest one step per launch."""
    from stochquant_amd.decomp import block_plan
    ops = block_plan(64, 16, 16)
    assert [o["op"] for o in ops[:4]] == ["exchange", "pair", "wait_exchange", "pair"]
    assert (ops[1]["step"], ops[1]["lo"], ops[1]["hi"]) == (0, 2, 62)
    assert (ops[3]["lo"], ops[3]["hi"], ops[3]["lo2"], ops[3]["hi2"]) == (-14, 2, 62, 78)
    inner = [o for o in ops[4:] if o["op"] == "pair" and 0 < o["step"] < 14]
    assert [(o["step"], o["lo"], o["hi"]) for o in inner] == [(s, -(14 - s), 64 + 14 - s) for s in range(2, 14, 2)]
    tail = [o for o in ops if o["step"] == 14]
    assert [(o["op"], o["lo"], o["hi"], o["lo2"], o["hi2"]) for o in tail] == [
        ("pair", 0, 16, 48, 64), ("edges_done", 0, 0, 0, 0), ("pair", 16, 48, 0, 0)]
    # odd g: the last step single, edges first
    ops = block_plan(40, 4, 3)
    assert [(o["op"], o["step"], o["lo"], o["hi"], o["lo2"], o["hi2"]) for o in ops] == [
        ("exchange", 0, 0, 0, 0, 0), ("pair", 0, 2, 38, 0, 0), ("wait_exchange", 0, 0, 0, 0, 0),
        ("pair", 0, -1, 2, 38, 41), ("step", 2, 0, 4, 36, 40), ("edges_done", 2, 0, 0, 0, 0),
        ("step", 2, 4, 36, 0, 0)]
    # K core pairs run ahead of the exchange; their rims follow it, then the rest
    ops = block_plan(64, 8, 8, core_pairs=2)
    assert [(o["op"], o["step"], o["lo"], o["hi"], o["lo2"], o["hi2"]) for o in ops] == [
        ("exchange", 0, 1, 0, 0, 0), ("pair", 0, 2, 62, 0, 0), ("wait_staged", 0, 0, 0, 0, 0),
        ("pair", 2, 4, 60, 0, 0),
        ("wait_exchange", 0, 0, 0, 0, 0), ("pair", 0, -6, 2, 62, 70), ("pair", 2, -4, 4, 60, 68),
        ("pair", 4, -2, 66, 0, 0), ("pair", 6, 0, 8, 56, 64), ("edges_done", 6, 0, 0, 0, 0),
        ("pair", 6, 8, 56, 0, 0)]
    ops = block_plan(64, 8, 8, core_pairs=4)   # every pair split: the last rims are the edges
    assert [o["op"] for o in ops].count("pair") == 8 and ops[-1]["op"] == "edges_done"
    assert (ops[-2]["lo"], ops[-2]["hi"], ops[-2]["lo2"], ops[-2]["hi2"]) == (0, 8, 56, 64)
    # unfused: every step 1..g-1 covered once, the last one ghost-free
    ops = block_plan(12, 4, 3, fuse2=False, edge_first=False)
    steps = [(o["step"], o["lo"], o["hi"]) for o in ops if o["op"] == "step"]
    assert steps == [(0, 1, 11), (0, -2, 1), (1, -1, 13), (2, 0, 12)]
    assert ops[-1]["op"] == "edges_done"


def test_slab_bounds_cover_lattice():
    from stochquant_amd.decomp import slab_bounds
    for Lz in (1, 7, 256, 1024):
        for P in range(1, min(Lz, 9) + 1):
            b = [slab_bounds(Lz, P, r) for r in range(P)]
            assert b[0][0] == 0 and b[-1][1] == Lz
            assert all(b[i][1] == b[i + 1][0] for i in range(P - 1))
            assert all(z1 > z0 for z0, z1 in b)
