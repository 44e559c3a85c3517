"""SQ_COMM_P2P: the peer-pointer halo transport, run as real separate rank
processes on one MI355X (RCCL refuses two ranks on one GPU; IPC peer
pointers do not), bit-identical to the monolithic single-slab run.

Each rank is its own process with its own HIP context, maps its neighbours'
staging buffers and mailboxes through IPC handles, and orders itself against
them only through stream-ordered flag writes/waits -- the same
code path a rank per GPU runs over xGMI.  Covered: P = 1 (own buffers), P = 2
(both neighbours one peer), P = 3 and 4, uneven slabs, partial blocks, the
fused two-step pairs with core pairs ahead of the exchange, the ghost-depth
trials max-reduced across ranks, frames (guard flag, stability records,
rollback) and the correlator's slice-sum all-reduce over peer memory.
"""
import numpy as np
import pytest

from conftest import rank_context

pytestmark = pytest.mark.gpu

TIMEOUT = 45


def _lat(shape, **kw):
    from stochquant_amd import Phi4Lattice
    return Phi4Lattice(shape, **kw)


def _mono(shape, kw, script):
    """The same script on one periodic slab in this process."""
    out = {}
    with _lat(shape, **kw) as L:
        for op, arg in script:
            if op == "upload":
                L.upload(arg)
            elif op == "upload_r0":   # arg = (field, nranks): rank 0's planes of field, the rest as they are
                from stochquant_amd.decomp import slab_bounds
                f = L.download()
                z0, z1 = slab_bounds(shape[2], arg[1], 0)
                f[z0:z1] = arg[0][z0:z1]
                L.upload(f)
            elif op == "step":
                L.step(arg)
            elif op == "frame":
                out.setdefault("stable", []).append(bool(L.run_frame()))
                out.setdefault("dtau", []).append(L.dtau)
                st = L.stability()
                out.setdefault("fired", []).append(st["fired"])
                out.setdefault("TV", []).append((float(st["T"]), float(st["V"])))
            elif op == "field":
                out.setdefault("field", []).append(L.download())
            elif op == "correlator":
                out["correlator"] = L.correlator(arg)
        out["step_counter"] = L.step_counter
    return out


def run_ranks(nranks, shape, kw, script, env=None):
    """Fork `nranks` rank processes, relay the handle blobs, return their outputs."""
    from p2p_ranks import rank_main
    ctx = rank_context()
    procs, conns = [], []
    try:
        for r in range(nranks):
            a, b = ctx.Pipe()
            p = ctx.Process(target=rank_main, args=(b, r, nranks, shape, kw, dict(env or {}), script), daemon=True)
            p.start()
            b.close()
            procs.append(p)
            conns.append(a)
        blobs = []
        for r, c in enumerate(conns):
            assert c.poll(TIMEOUT), f"rank {r} sent no handle"
            tag, val = c.recv()
            assert tag == "blob", f"rank {r}: {val}"
            blobs.append(val)
        for c in conns:
            c.send(blobs)
        outs = []
        for r, c in enumerate(conns):
            assert c.poll(TIMEOUT), f"rank {r} did not finish"
            tag, val = c.recv()
            assert tag == "ok", f"rank {r}: {val}"
            outs.append(val)
        for p in procs:
            p.join(TIMEOUT)
            assert p.exitcode == 0
        return outs
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(5)


def _field0(shape, amp=0.5, seed=77):
    rng = np.random.default_rng(seed)
    return (amp * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)


def _assemble(outs, k=-1):
    return np.concatenate([o["field"][k] for o in sorted(outs, key=lambda o: o["z0"])], axis=0)


KW = dict(dtau=0.02, m2=0.5, lam=1.0, seed=1234, C=1.0)


def test_p2p_single_rank_in_process(gpu):
    """P = 1: the exchange pulls from its own staged copy (no IPC mapping)."""
    shape = (64, 16, 24)
    phi0 = _field0(shape)
    script = [("upload", phi0), ("step", 13), ("field", None)]
    mono = _mono(shape, KW, script)
    with _lat(shape, comm="p2p", nranks=1, rank=0, **KW) as L:
        L.p2p_connect([L.p2p_handle()])
        L.upload(phi0)
        L.step(13)
        assert np.array_equal(L.download(), mono["field"][0])


@pytest.mark.parametrize("on_a", ["0", "1"])
@pytest.mark.parametrize("ghost", ["4", "16"])
def test_p2p_single_rank_kernel_staged(gpu, monkeypatch, ghost, on_a):
    """P = 1 with SQ_P2P_KSTAGE=1: several step calls (each block's last pair
    stages the next exchange, across calls too), an upload in between (the
    staged edges are dropped and re-staged by copy), a frame (frames stage by
    copy) and more steps: bit-identical to the single periodic slab."""
    shape = (256, 16, 48)
    phi0, phi1 = _field0(shape), _field0(shape, seed=3)
    kw = dict(KW, loops=6)
    script = [("upload", phi0), ("step", 20), ("step", 13), ("field", None), ("upload", phi1), ("step", 9),
              ("frame", None), ("step", 24), ("field", None)]
    mono = _mono(shape, kw, script)
    monkeypatch.setenv("SQ_P2P_KSTAGE", "1")
    monkeypatch.setenv("SQ_XCHG_ON_A", on_a)
    monkeypatch.setenv("SQ_GHOST", ghost)
    got = []
    with _lat(shape, comm="p2p", nranks=1, rank=0, **kw) as L:
        L.p2p_connect([L.p2p_handle()])
        for op, arg in script:
            if op == "upload":
                L.upload(arg)
            elif op == "step":
                L.step(arg)
            elif op == "frame":
                assert bool(L.run_frame()) == mono["stable"][0]
            elif op == "field":
                got.append(L.download())
    for a, b in zip(got, mono["field"]):
        assert np.array_equal(a, b)


def test_p2p_unconnected_context_refuses_to_step(gpu):
    from stochquant_amd import StochQuantError
    with _lat((64, 16, 24), comm="p2p", nranks=2, rank=0, **KW) as L:
        with pytest.raises(StochQuantError, match="not connected"):
            L.step(1)
        blob = L.p2p_handle()
        with pytest.raises(StochQuantError, match="rank order"):
            L.p2p_connect([blob, blob])


@pytest.mark.parametrize("nranks,shape,steps,env", [
    (2, (64, 16, 24), 13, {"SQ_GHOST": "4"}),                      # P = 2: one peer on both sides
    (3, (64, 8, 40), 22, {"SQ_GHOST": "3"}),                        # uneven slabs (13/13/14), partial block
    (4, (32, 8, 32), 9, {"SQ_GHOST": "2"}),
    (2, (256, 16, 64), 21, {"SQ_GHOST": "8"}),                      # fused pairs, odd tail
    (3, (256, 16, 96), 40, {"SQ_GHOST": "8", "SQ_CORE_PAIRS": "2"}),  # core pairs ahead of the exchange
    (3, (256, 16, 96), 40, {"SQ_GHOST": "8", "SQ_CORE_PAIRS": "2", "SQ_RIMS_B": "1"}),  # rims on stream B
    (2, (256, 16, 64), 30, {"SQ_GHOST": "16", "SQ_CORE_PAIRS": "0"}),  # no core/rim split
    # the driver's N = 8 shape: eight rank processes, each
    # slab's two peers distinct ranks, fused pairs and core pairs
    (8, (64, 8, 64), 17, {"SQ_GHOST": "4"}),
    (8, (256, 16, 256), 40, {"SQ_GHOST": "8", "SQ_CORE_PAIRS": "2"}),
    # the last pair of each block writes the next exchange's staging slot and
    # counts its blocks (SQ_P2P_KSTAGE=1, phi4_tb2_stage_kernel)
    (2, (256, 16, 64), 21, {"SQ_GHOST": "8", "SQ_P2P_KSTAGE": "1"}),
    (3, (256, 16, 96), 40, {"SQ_GHOST": "8", "SQ_CORE_PAIRS": "2", "SQ_P2P_KSTAGE": "1"}),
    (2, (256, 16, 64), 30, {"SQ_GHOST": "16", "SQ_CORE_PAIRS": "0", "SQ_P2P_KSTAGE": "1"}),
    (8, (256, 16, 256), 40, {"SQ_GHOST": "8", "SQ_CORE_PAIRS": "2", "SQ_P2P_KSTAGE": "1"}),
    (4, (256, 8, 20), 33, {"SQ_GHOST": "4", "SQ_P2P_KSTAGE": "1"}),  # slabs of 5 planes: edges overlap
    # the exchange in order on the interior stream (SQ_XCHG_ON_A=1), by copy or kernel-staged
    (2, (256, 16, 64), 21, {"SQ_GHOST": "8", "SQ_XCHG_ON_A": "1"}),
    (4, (32, 8, 32), 9, {"SQ_GHOST": "2", "SQ_XCHG_ON_A": "1"}),
    (3, (256, 16, 96), 40, {"SQ_GHOST": "8", "SQ_XCHG_ON_A": "1", "SQ_P2P_KSTAGE": "1"}),
    (8, (256, 16, 256), 40, {"SQ_GHOST": "16", "SQ_XCHG_ON_A": "1", "SQ_P2P_KSTAGE": "1"}),
])
def test_p2p_ranks_bitwise_vs_single_slab(gpu, nranks, shape, steps, env):
    phi0 = _field0(shape)
    script = [("upload", phi0), ("step", steps), ("field", None)]
    mono = _mono(shape, KW, script)
    outs = run_ranks(nranks, shape, KW, script, env)
    got = _assemble(outs)
    assert np.array_equal(got, mono["field"][0]), f"max diff {np.max(np.abs(got - mono['field'][0]))}"
    assert all(o["step_counter"] == steps for o in outs)
    assert all(o["perf"]["halo_bytes"] > 0 for o in outs)


def test_p2p_ghost_trials_agree_across_ranks(gpu):
    """Multi-rank P2P contexts time G in {4, 8, 16} and the core-pair / rim
    schedules and max-reduce the trial times over peer memory: every rank keeps
    the same schedule, and the trial steps are ordinary steps."""
    shape = (256, 16, 128)
    phi0 = _field0(shape)
    script = [("upload", phi0), ("step", 430), ("ghost", None), ("field", None)]
    mono = _mono(shape, KW, script)
    outs = run_ranks(2, shape, KW, script)
    assert outs[0]["ghost"] == outs[1]["ghost"] and outs[0]["ghost"][0] in (4, 8, 16)
    assert outs[0]["schedule"] == outs[1]["schedule"] and outs[0]["schedule"]["tuned"]
    assert np.array_equal(_assemble(outs), mono["field"][0])


def test_p2p_frames_rollback_and_correlator(gpu):
    """Frames over peer-memory collectives: guard flag, stability records and
    the rollback decision agree with the single slab (dtau = 0.2 diverges and
    is rolled back, then dtau shrinks until frames pass), and the correlator's
    slice sums are all-reduced exactly."""
    shape = (64, 16, 48)
    kw = dict(KW, dtau=0.2, m2=1.0, C=0.0, loops=12)
    phi0 = _field0(shape, amp=0.05)
    script = [("upload", phi0), ("frame", None), ("frame", None), ("field", None),
              ("correlator", 8)]
    mono = _mono(shape, kw, script)
    assert not mono["stable"][0]
    outs = run_ranks(3, shape, kw, script, {"SQ_GHOST": "4"})
    for o in outs:
        assert o["stable"] == mono["stable"] and o["fired"] == mono["fired"]
        assert o["TV"] == mono["TV"] and o["dtau"] == mono["dtau"]
        assert o["step_counter"] == mono["step_counter"]
        np.testing.assert_allclose(o["correlator"], mono["correlator"], rtol=1e-12, atol=1e-12)
    assert np.array_equal(_assemble(outs), mono["field"][0])


def test_p2p_rollback_after_one_rank_uploads_nan(gpu):
    """rank 0 uploads a NaN on its top plane, next to rank 1's ghost
    zone, while rank 1 re-uploads its own finite slab (uploads are collective,
    stochquant.h); the ranks agree that the field is unguarded before the
    frame captures the state its rollback restores, so both rolled-back frames
    clamp the NaN on rank 1's ghost copies too: verdicts, dtau and the field
    equal the single slab's."""
    shape = (64, 16, 24)
    kw = dict(KW, loops=4)
    phi0 = _field0(shape)
    bad = _field0(shape, seed=5)
    bad[11, 3, 7] = np.nan
    script = [("upload", phi0), ("step", 4), ("upload_r0", (bad, 2)), ("frame", None), ("frame", None),
              ("field", None)]
    mono = _mono(shape, kw, script)
    assert mono["stable"] == [False, False]
    outs = run_ranks(2, shape, kw, script, {"SQ_GHOST": "4"})
    for o in outs:
        assert o["stable"] == mono["stable"] and o["dtau"] == mono["dtau"] and o["TV"] == mono["TV"]
    # both frames rolled back: the field is the upload again, NaN included (compare bits)
    assert np.array_equal(_assemble(outs).view(np.uint32), mono["field"][0].view(np.uint32))


def test_p2p_frames_with_noise(gpu):
    shape = (256, 16, 64)
    kw = dict(KW, dtau=0.01, m2=1.0, loops=10)
    phi0 = _field0(shape, amp=0.3)
    script = [("upload", phi0), ("frame", None), ("step", 7), ("frame", None), ("field", None)]
    mono = _mono(shape, kw, script)
    outs = run_ranks(2, shape, kw, script, {"SQ_GHOST": "4"})
    for o in outs:
        assert o["stable"] == mono["stable"] == [True, True]
        assert o["TV"] == mono["TV"]
    assert np.array_equal(_assemble(outs), mono["field"][0])
    # the same with the kernel-staged exchange between the frames
    outs = run_ranks(2, shape, kw, script, {"SQ_GHOST": "4", "SQ_P2P_KSTAGE": "1"})
    for o in outs:
        assert o["stable"] == mono["stable"] == [True, True]
        assert o["TV"] == mono["TV"]
    assert np.array_equal(_assemble(outs), mono["field"][0])


def _bench(args, timeout=240):
    """bench.py in a child of the fork server; returns its JSON line."""
    import json
    import os
    import sys
    from conftest import ROOT
    from p2p_ranks import run_cmd
    ctx = rank_context()
    a, b = ctx.Pipe()
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = ctx.Process(target=run_cmd, args=(b, [sys.executable, os.path.join(ROOT, "bench.py")] + args, env,
                                          timeout), daemon=True)
    p.start()
    b.close()
    assert a.poll(timeout + 30), "bench.py did not finish"
    rc, out, err = a.recv()
    p.join(10)
    assert rc == 0, err[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("corrupt", [False, True])
def test_bench_multi_rank_check(gpu, corrupt):
    """bench.py's self-check of a multi-rank run (stochquant_amd/verify.py): two
    P2P rank processes of the bench's own spawn -> gloo -> connect path on one
    GPU run the check protocol and compare each slab's digest with the golden
    single-GPU run of the 256 x 256 x 512 lattice: "pass"; with one value of
    rank 1's slab flipped: "fail"."""
    args = ["--gpus", "2", "--comm", "p2p", "--same-device", "--steps", "4", "--warmup", "2",
            "--settle-ms", "0", "--no-cpu-baseline", "--no-c3"]
    if corrupt:
        args += ["--corrupt-rank", "1"]
    d = _bench(args)
    assert d["n_gpus"] == 2 and d["config"]["lattice"] == [256, 256, 512]
    assert d["multi_rank_check"] == ("fail" if corrupt else "pass")
