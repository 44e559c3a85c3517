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


def test_hash_field_is_slab_consistent_and_bounded():
    """Each rank's slab of the oracle check's field is the same planes of the
    whole lattice's field; values in [-AMP, AMP), no NaN, not constant."""
    shape = (16, 8, 12)
    whole = verify.hash_field(shape, 0, 12)
    assert whole.dtype == np.float32 and whole.shape == (12, 8, 16)
    assert np.array_equal(verify.hash_field(shape, 5, 4, chunk=3), whole[5:9])
    assert np.all(np.abs(whole) <= verify.HASH_FIELD_AMP) and np.std(whole) > 0.1
    # pinned values: the function must not drift between the digest generator and the bench
    assert whole[0, 0, 0] == np.float32(verify.hash_field(shape, 0, 1)[0, 0, 0])
    assert verify.slab_digest(verify.hash_field((256, 8, 4), 0, 4)) == verify.slab_digest(
        verify.hash_field((256, 8, 4), 0, 4, chunk=1))


def test_oracle_check_pass_fail_and_missing():
    g = {verify.golden_key((4, 4, 8), 2): {"slabs": ["aa", "bb"]}}
    assert verify.oracle_check(["aa", "bb"], (4, 4, 8), 2, g) == "pass"
    assert verify.oracle_check(["aa", "xx"], (4, 4, 8), 2, g) == "fail"
    assert verify.oracle_check(["aa", "bb"], (4, 4, 16), 2, g) == "no golden"


def test_oracle_check_noise_tables_first():
    """oracle_check_noise compares digests only when every rank's device
    Box-Muller tables hash like the ones the committed digests were made with."""
    key = verify.NOISE_PREFIX + verify.golden_key((4, 4, 8), 2)
    g = {key: {"slabs": ["aa", "bb"]}, verify.BM_TABLES_KEY: {"blake2b": "tt"}}
    assert verify.oracle_check_noise(["aa", "bb"], ["tt", "tt"], (4, 4, 8), 2, g) == "pass"
    assert verify.oracle_check_noise(["aa", "xx"], ["tt", "tt"], (4, 4, 8), 2, g) == "fail"
    assert verify.oracle_check_noise(["aa", "bb"], ["tt", "tu"], (4, 4, 8), 2, g) == "tables differ"
    assert verify.oracle_check_noise(["aa", "bb"], ["tt", "tt"], (4, 4, 16), 2, g) == "no golden"
    assert verify.oracle_check_noise(["aa", "bb"], ["tt", "tt"], (4, 4, 8), 2, {key: g[key]}) == "no golden"
    # the noise-off verdict never reads the noise digests
    assert verify.oracle_check(["aa", "bb"], (4, 4, 8), 2, g) == "no golden"


def test_committed_oracle_digests_cover_the_driver_configs():
    """tests/golden/oracle_slabs.json: weak 256^3 per GPU and strong 1024^3 at
    N = 1, 2, 4, 8, one oracle digest per rank, noise off."""
    g = verify.load_oracle_golden()
    for n in (1, 2, 4, 8):
        for shape in ((256, 256, 256 * n), (1024, 1024, 1024)):
            rec = g[verify.golden_key(shape, n)]
            assert len(rec["slabs"]) == n and rec["steps"] == verify.CHECK_STEPS and rec["C"] == 0.0


def test_oracle_digest_reproduces_from_the_oracle(oracle_mod):
    """The committed N = 1 digest is the oracle's (regenerated here on the CPU,
    tests/golden/make_oracle_slabs.py's recipe): the oracle pins what the
    GPU's oracle_check compares against."""
    import os
    shape = (256, 256, 256)
    P = verify.CHECK_PARAMS
    p = oracle_mod.phi4_params(shape, P["dtau"], P["m2"], P["lam"], P["seed"], C=0.0)
    f = verify.hash_field(shape, 0, 256)
    for s in range(verify.CHECK_STEPS):
        f = oracle_mod.phi4_step(p, f, s, os.cpu_count() or 1)
    assert verify.slab_digest(f) == verify.load_oracle_golden()[verify.golden_key(shape, 1)]["slabs"][0]
