"""Slab decomposition of the 3-D lattice along z (the slowest axis).

Mirrors create_phi4() / phi4_one_step() in csrc/sq_api.cpp: rank r of P owns
global planes [Lz*r//P, Lz*(r+1)//P) plus two ghost planes; every step it
sends its top plane to rank r+1 and its bottom plane to rank r-1 and receives
its lower ghost from r-1 and its upper ghost from r+1 (periodic wrap), in
that order, so that with P = 2 (both neighbours the same peer) the k-th send
still pairs with the k-th receive.
"""


def slab_bounds(Lz, nranks, rank):
    """Global [z0, z1) of `rank`'s slab."""
    if not (1 <= nranks <= Lz and 0 <= rank < nranks):
        raise ValueError("need 1 <= nranks <= Lz and 0 <= rank < nranks")
    return Lz * rank // nranks, Lz * (rank + 1) // nranks


def neighbours(nranks, rank):
    """(up, down) = ranks owning the planes above / below this slab."""
    return (rank + 1) % nranks, (rank + nranks - 1) % nranks


def halo_bytes_per_step(Lx, Ly, dtype_bytes=4):
    """Bytes one rank sends per step (two faces)."""
    return 2 * Lx * Ly * dtype_bytes
