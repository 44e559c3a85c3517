"""Slab decomposition of the 3-D lattice along z (the slowest axis).

Mirrors create_phi4() / phi4_block() in csrc/sq_api.cpp: rank r
of P owns global planes [Lz*r//P, Lz*(r+1)//P) plus a ghost zone of G planes
on either side (G = steps per halo exchange).  Every G steps one exchange
sends the G top planes to rank r+1 and the G bottom planes to rank r-1 and
receives the lower ghosts from r-1 and the upper ghosts from r+1 (periodic
wrap), in that order, so that with P = 2 (both neighbours the same peer) the
k-th send still pairs with the k-th receive.  Step s of the block then updates
the shrinking range [-(G-1-s), nz+G-1-s), recomputing ghost-zone sites
redundantly (bit-identical: the noise is keyed by global site and step).

`block_plan` returns the product's own launch schedule of one block (the list
phi4_block executes, from libstochquant.so's pure-host sq_phi4_block_plan), so
the multi-rank CPU rehearsal (tests/test_multirank_cpu.py) runs exactly the
ranges, pairs and edge ordering the GPU path runs.
"""
import ctypes

from . import _lib


def slab_bounds(Lz, nranks, rank):
    """Global [z0, z1) of `rank`'s slab."""
    if not (1 <= nranks <= Lz and 0 <= rank < nranks):
        raise ValueError("need 1 <= nranks <= Lz and 0 <= rank < nranks")
    return Lz * rank // nranks, Lz * (rank + 1) // nranks


def neighbours(nranks, rank):
    """(up, down) = ranks owning the planes above / below this slab."""
    return (rank + 1) % nranks, (rank + nranks - 1) % nranks


def halo_bytes_per_step(Lx, Ly, dtype_bytes=4):
    """Bytes one rank sends per step (two faces; G faces every G steps)."""
    return 2 * Lx * Ly * dtype_bytes


OP_NAMES = {_lib.SQ_OP_EXCHANGE: "exchange", _lib.SQ_OP_STEP: "step", _lib.SQ_OP_PAIR: "pair",
            _lib.SQ_OP_WAIT_EXCHANGE: "wait_exchange", _lib.SQ_OP_EDGES_DONE: "edges_done",
            _lib.SQ_OP_WAIT_STAGED: "wait_staged", _lib.SQ_OP_SIGNAL: "signal", _lib.SQ_OP_WAIT: "wait"}


def block_plan(nz, ghost, g, fuse2=True, edge_first=True, core_pairs=1, rims_b=False):
    """The schedule of one deep-halo block of g <= ghost steps on a slab of nz
    planes: a list of dicts {op, step, lo, hi, lo2, hi2, stream} (stream "A" or "B")."""
    cap = 64
    ops = (_lib.SqBlockOp * cap)()
    n = ctypes.c_int()
    _lib.call("sq_phi4_block_plan", int(nz), int(ghost), int(g), 1 if fuse2 else 0, 1 if edge_first else 0,
              int(core_pairs), 1 if rims_b else 0, ops, cap, ctypes.byref(n))
    return [{"op": OP_NAMES[o.kind], "step": o.step, "lo": o.lo, "hi": o.hi, "lo2": o.lo2, "hi2": o.hi2,
             "stream": "AB"[o.stream]} for o in ops[:n.value]]


def pick_ghost(ms):
    """Index of the fastest ghost-depth candidate of the (rank-max-reduced) per-step times."""
    a = (ctypes.c_double * len(ms))(*ms)
    return _lib.load().sq_phi4_pick_ghost(a, len(ms))
