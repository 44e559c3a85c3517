"""The multi-rank self-check's host logic (stochquant_amd/verify.py), on CPU."""
import numpy as np

from stochquant_amd import verify


def test_digest_is_content_and_order_sensitive():
    a = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    b = a.copy()
    assert verify.slab_digest(a) == verify.slab_digest(b)
    b[1, 2, 3] = np.nextafter(b[1, 2, 3], np.float32(100))
    assert verify.slab_digest(a) != verify.slab_digest(b)
    assert verify.slab_digest(a) != verify.slab_digest(a[::-1])


def test_check_pass_fail_and_missing():
    g = {verify.golden_key((4, 4, 8), 2): {"slabs": ["aa", "bb"]}}
    assert verify.check(["aa", "bb"], (4, 4, 8), 2, g) == "pass"
    assert verify.check(["aa", "bc"], (4, 4, 8), 2, g) == "fail"
    assert verify.check(["aa"], (4, 4, 8), 2, g) == "fail"
    assert verify.check(["aa", "bb"], (4, 4, 16), 2, g) == "no golden"


def test_committed_golden_covers_the_driver_configs():
    """Weak 256^3 per GPU and strong 1024^3 at N = 1, 2, 4, 8, one digest per rank."""
    g = verify.load_golden()
    for n in (1, 2, 4, 8):
        assert len(g[verify.golden_key((256, 256, 256 * n), n)]["slabs"]) == n
        assert len(g[verify.golden_key((1024, 1024, 1024), n)]["slabs"]) == n
        assert g[verify.golden_key((256, 256, 256 * n), n)]["steps"] == verify.CHECK_STEPS
