"""The P2P exchange protocol of round 6 (phi4_block in csrc/sq_api.cpp,
DESIGN.md §8.2), modelled on the CPU and checked under random interleavings.

Each rank's exchange stream B runs, per exchange e = 1, 2, ...:
    copy my edge planes into my staging slot e & 1
    write "staged e" into both neighbours' mailboxes
    wait until my mailbox's word from the lower neighbour is >= e
    pull the lower neighbour's slot e & 1
    wait until the word from the upper neighbour is >= e
    pull the upper neighbour's slot e & 1
with no acknowledgement in between (rounds 2-5 waited for both neighbours'
"read e - 1" first and wrote "read e" after the pulls).  The claim that lets
the acknowledgements go: when a rank overwrites slot e & 1 at exchange e, both
neighbours have finished pulling exchange e - 2 from it, because each wrote its
"staged e - 1" behind that pull and this rank waited for both of those flags
during exchange e - 1.  Here every rank is a program of those operations;
an adversarial scheduler advances any rank whose next operation is enabled
(waits block), a staging copy records which exchange a slot holds, and a pull
must find exactly the exchange it expects -- for P = 1 (a rank is its own
neighbour), P = 2 (both neighbours one peer) and larger rings, thousands of
schedules each.  The same model with ONE slot fails, which shows the checker
can see the hazard the second slot removes.

The same program covers round 6's later forms: with the exchange in order on
the interior stream (SQ_XCHG_ON_A) every operation is on that one stream in
this order, and with the staged last pair (SQ_P2P_KSTAGE) the "copy" of
exchange e is the block's last pair writing slot e & 1, which that stream runs
after the pulls of exchange e - 1 (the exchange stream's form: its hand-shake
waits for the pair's block count, and the pair follows the rim pair that
waited for those pulls) -- the order the model checks."""
import random

import pytest


def _program(r, P, n_exchanges, slots):
    up, dn = (r + 1) % P, (r - 1) % P
    ops = []
    for e in range(1, n_exchanges + 1):
        s = e % slots
        ops += [("copy", s, e), ("write", up, "dn", e), ("write", dn, "up", e),
                ("wait", "dn", e), ("pull", dn, s, e), ("wait", "up", e), ("pull", up, s, e)]
    return ops


def _run(P, n_exchanges, slots, rng):
    progs = [_program(r, P, n_exchanges, slots) for r in range(P)]
    pc = [0] * P
    slot = [[0] * slots for _ in range(P)]          # which exchange each staging slot holds
    mbox = [{"dn": 0, "up": 0} for _ in range(P)]   # staged flags: from my lower / upper neighbour
    while True:
        ready = []
        for r in range(P):
            if pc[r] == len(progs[r]):
                continue
            op = progs[r][pc[r]]
            if op[0] == "wait" and mbox[r][op[1]] < op[2]:
                continue
            ready.append(r)
        if not ready:
            assert all(pc[r] == len(progs[r]) for r in range(P)), "deadlock"
            return
        r = rng.choice(ready)
        op = progs[r][pc[r]]
        pc[r] += 1
        if op[0] == "copy":
            slot[r][op[1]] = op[2]
        elif op[0] == "write":
            # peer `op[1]` receives it in the word for the neighbour this rank is to it
            mbox[op[1]][op[2]] = max(mbox[op[1]][op[2]], op[3])
        elif op[0] == "pull":
            got = slot[op[1]][op[2]]
            assert got == op[3], f"rank {r} pulled exchange {got} from rank {op[1]} slot {op[2]}, wanted {op[3]}"


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_two_parity_slots_never_overwrite_an_unread_copy(P):
    rng = random.Random(1000 + P)
    for _ in range(2000 if P <= 4 else 500):
        _run(P, 6, slots=2, rng=rng)


def test_one_slot_without_acknowledgements_is_caught():
    rng = random.Random(7)
    with pytest.raises(AssertionError, match="pulled exchange"):
        for _ in range(2000):
            _run(3, 6, slots=1, rng=rng)
