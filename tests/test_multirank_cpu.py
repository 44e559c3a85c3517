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


def _stream_order(plan, prefer):
    """A sequential order of the block's ops that respects what the product's
    two streams guarantee: each stream runs its ops in list order, a WAIT runs
    after its SIGNAL, WAIT_EXCHANGE / WAIT_STAGED after the exchange.  `prefer`
    "A" runs stream A whenever it can (the interior as far ahead of the
    exchange and the rims as the waits allow), "B" the other way round, "list"
    the list order itself.  A plan that lets one stream read what the other
    has not written yet then reads NaN (or a stale step) and fails the test."""
    if prefer == "list":
        return list(plan)
    queues = {"A": [op for op in plan if op["stream"] == "A"], "B": [op for op in plan if op["stream"] == "B"]}
    done, out = set(), []

    def ready(op):
        k = op["op"]
        if k in ("wait_exchange", "wait_staged"):
            return "exchange" in done
        if k == "wait":
            return ("signal", op["lo"]) in done
        return True

    while queues["A"] or queues["B"]:
        for name in (prefer, "B" if prefer == "A" else "A"):
            if queues[name] and ready(queues[name][0]):
                op = queues[name].pop(0)
                out.append(op)
                done.add(("signal", op["lo"]) if op["op"] == "signal" else op["op"])
                break
        else:
            raise AssertionError("block plan deadlocks: " + repr([q[0] for q in queues.values() if q]))
    return out


def _run_block(oracle, p, plan, bufs, cur, nz, G, z0, step0, world, up, dn, prefer="list"):
    """Execute one block's schedule as phi4_block does, in one sequential order
    of its two streams (_stream_order): a launch group (the STEP / PAIR ops of
    one first step) reads the buffer the group before it wrote; returns the
    buffer holding the result."""
    starts = sorted({op["step"] for op in plan if op["op"] in ("step", "pair")})
    for op in _stream_order(plan, prefer):
        k = op["op"]
        if k == "exchange":
            _exchange(bufs, cur, nz, G, world, up, dn)
        elif k in ("step", "pair"):
            inb = cur ^ (starts.index(op["step"]) & 1)
            s = step0 + op["step"]
            for lo, hi in _ranges(op):
                if k == "step":
                    oracle.phi4_step_range(p, bufs[inb], bufs[inb ^ 1], G, lo, hi, z0, s)
                else:   # two steps in one launch: step s on [lo-1, hi+1) into scratch, s+1 on [lo, hi)
                    mid = np.full_like(bufs[inb], np.nan)
                    oracle.phi4_step_range(p, bufs[inb], mid, G, lo - 1, hi + 1, z0, s)
                    oracle.phi4_step_range(p, mid, bufs[inb ^ 1], G, lo, hi, z0, s + 1)
        else:
            assert k in ("wait_exchange", "edges_done", "wait_staged", "signal", "wait")
    return cur ^ (len(starts) & 1)


def _worker(rank, world, port, steps, fuse2, edge_first, gpad, q, core_pairs=1, prefer="list", rims_b=False):
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
            plan = block_plan(nz, G, g, fuse2, edge_first, core_pairs, rims_b)
            cur = _run_block(oracle, p, plan, bufs, cur, nz, G, z0, done, world, up, dn, prefer)
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


@pytest.mark.parametrize("world,steps,fuse2,edge_first,gpad,core_pairs,prefer,rims_b", [
    (2, 11, True, True, 4, 1, "list", False),  # P = 2: both neighbours one peer; partial last block (4+4+3)
    (3, 11, True, True, 4, 1, "A", True),      # interior as far ahead as the waits allow
    (3, 11, True, True, 4, 1, "B", True),      # exchange and rims as far ahead as the waits allow
    (3, 11, True, True, 4, 1, "A", False),
    (2, 9, False, True, 4, 1, "A", True),      # per-step inner launches
    (2, 9, False, True, 4, 0, "B", False),     # ... without a core/rim split
    (3, 8, True, False, 4, 1, "list", False),  # edges not first
    (2, 9, True, True, 8, 1, "B", True),       # deeper zone: pairs over 2 ghost planes
    (2, 12, True, True, 2, 1, "A", False),     # G = 2: blocks of one core/rim step and one edges-first step
    (3, 10, True, True, 8, 1, "list", True),   # G = 8 over slabs of 12 planes: rims of 8 planes, no edge split
    (1, 7, True, True, 4, 1, "B", False),      # single rank, self-exchange
    (2, 13, True, True, 8, 0, "A", False),     # no core/rim split: the first pair waits for the exchange
    (2, 17, True, True, 8, 2, "A", True),      # two core pairs ahead of the exchange
    (2, 17, True, True, 8, 2, "B", True),
    (2, 17, True, True, 8, 2, "B", False),
    (2, 19, True, True, 8, 4, "A", True),      # every pair of the block split into core and rim
    (3, 11, True, False, 8, 3, "B", True),     # three core pairs, slabs of 12 planes (the core shrinks to 4)
    (8, 9, True, True, 2, 1, "list", False),   # the driver's N = 8: slabs of 4-5 planes, G = 2
    (8, 9, True, True, 2, 1, "B", True),
])
def test_gloo_deep_halo_blocks_bitwise(world, steps, fuse2, edge_first, gpad, core_pairs, prefer, rims_b, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, fuse2, edge_first, gpad, q, core_pairs, prefer,
                                               rims_b)) for r in range(world)]
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
    """The schedule's ranges and streams: fused blocks pair
    every step -- a core pair on stream A overlapping the exchange, the rim pair
    on stream B right behind the exchange, stream A waiting for the rims before
    the pairs over the shrinking ghost range, the last pair edges first;
    unfused blocks split step 0 into core (A) and rim (B) and run the rest one
    step per launch on A."""
    from stochquant_amd.decomp import block_plan

    def sig(ops):
        return [(o["op"], o["step"], o["lo"], o["hi"], o["lo2"], o["hi2"], o["stream"]) for o in ops]

    ops = block_plan(64, 16, 16)
    assert sig(ops[:4]) == [
        ("exchange", 0, 0, 0, 0, 0, "B"), ("pair", 0, 2, 62, 0, 0, "A"), ("wait_exchange", 0, 0, 0, 0, 0, "A"),
        ("pair", 0, -14, 2, 62, 78, "A")]
    assert sig(block_plan(64, 16, 16, rims_b=True)[:6]) == [
        ("exchange", 0, 0, 0, 0, 0, "B"), ("pair", 0, 2, 62, 0, 0, "A"), ("wait_exchange", 0, 0, 0, 0, 0, "B"),
        ("pair", 0, -14, 2, 62, 78, "B"), ("signal", 0, 15, 0, 0, 0, "B"), ("wait", 0, 15, 0, 0, 0, "A")]
    assert sig(block_plan(64, 16, 16, core_pairs=0)[:3]) == [
        ("exchange", 0, 0, 0, 0, 0, "B"), ("wait_exchange", 0, 0, 0, 0, 0, "A"), ("pair", 0, -14, 78, 0, 0, "A")]
    inner = [o for o in ops[4:] if o["op"] == "pair" and 0 < o["step"] < 14]
    assert [(o["step"], o["lo"], o["hi"], o["stream"]) for o in inner] == [
        (s, -(14 - s), 64 + 14 - s, "A") for s in range(2, 14, 2)]
    tail = [o for o in ops if o["step"] == 14]
    assert sig(tail) == [("pair", 14, 0, 16, 48, 64, "A"), ("edges_done", 14, 0, 0, 0, 0, "A"),
                         ("pair", 14, 16, 48, 0, 0, "A")]
    # odd g: the last step single, edges first
    ops = block_plan(40, 4, 3)
    assert sig(ops) == [
        ("exchange", 0, 0, 0, 0, 0, "B"), ("pair", 0, 2, 38, 0, 0, "A"), ("wait_exchange", 0, 0, 0, 0, 0, "A"),
        ("pair", 0, -1, 2, 38, 41, "A"),
        ("step", 2, 0, 4, 36, 40, "A"), ("edges_done", 2, 0, 0, 0, 0, "A"), ("step", 2, 4, 36, 0, 0, "A")]
    # K core pairs run ahead of the exchange on A (the second after the staged
    # copy); their rims follow the exchange on B, rim j after core j-1
    ops = block_plan(64, 8, 8, core_pairs=2, rims_b=True)
    assert sig(ops) == [
        ("exchange", 0, 1, 0, 0, 0, "B"), ("pair", 0, 2, 62, 0, 0, "A"), ("signal", 0, 0, 0, 0, 0, "A"),
        ("wait_staged", 0, 0, 0, 0, 0, "A"), ("pair", 2, 4, 60, 0, 0, "A"),
        ("wait_exchange", 0, 0, 0, 0, 0, "B"), ("pair", 0, -6, 2, 62, 70, "B"), ("wait", 2, 0, 0, 0, 0, "B"),
        ("pair", 2, -4, 4, 60, 68, "B"), ("signal", 0, 15, 0, 0, 0, "B"), ("wait", 0, 15, 0, 0, 0, "A"),
        ("pair", 4, -2, 66, 0, 0, "A"), ("pair", 6, 0, 8, 56, 64, "A"), ("edges_done", 6, 0, 0, 0, 0, "A"),
        ("pair", 6, 8, 56, 0, 0, "A")]
    ops = block_plan(64, 8, 8, core_pairs=4, rims_b=True)   # every pair split: the last rims are the edges
    assert [o["op"] for o in ops].count("pair") == 8 and ops[-1]["op"] == "edges_done"
    last_rim = [o for o in ops if o["op"] == "pair" and o["stream"] == "B"][-1]
    assert (last_rim["lo"], last_rim["hi"], last_rim["lo2"], last_rim["hi2"]) == (0, 8, 56, 64)
    # unfused: every step 1..g-1 covered once, the last one ghost-free
    ops = block_plan(12, 4, 3, fuse2=False, edge_first=False)
    steps = [(o["step"], o["lo"], o["hi"], o["stream"]) for o in ops if o["op"] == "step"]
    assert steps == [(0, 1, 11, "A"), (0, -2, 1, "A"), (1, -1, 13, "A"), (2, 0, 12, "A")]
    assert ops[-1]["op"] == "edges_done"


def test_slab_bounds_cover_lattice():
    from stochquant_amd.decomp import slab_bounds
    for Lz in (1, 7, 256, 1024):
        for P in range(1, min(Lz, 9) + 1):
            b = [slab_bounds(Lz, P, r) for r in range(P)]
            assert b[0][0] == 0 and b[-1][1] == Lz
            assert all(b[i][1] == b[i + 1][0] for i in range(P - 1))
            assert all(z1 > z0 for z0, z1 in b)
