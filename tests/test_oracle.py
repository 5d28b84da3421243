"""CPU: the oracle (oracle/nw_oracle.c) pinned against the reference's own outputs.

Golden vectors come from the unmodified reference sources compiled by
oracle/Makefile and run by tests/golden/make_golden.py.
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN

SCHEMES = oracle.SCHEMES
TINY = ["small", "small_rev", "t", "debug"]


@pytest.mark.parametrize("scheme", list(SCHEMES))
@pytest.mark.parametrize("name", TINY)
def test_full_table_matches_reference(pair, scheme, name):
    s1, s2 = pair(name)
    want = np.load(f"{GOLDEN}/table_{scheme}_{name}.npy")
    got = oracle.fill(s1, s2, SCHEMES[scheme])
    assert got.shape == (s2.size + 1, s1.size + 1)
    np.testing.assert_array_equal(got, want)


def test_small_table_is_survey_appendix_a(pair):
    """SURVEY.md Appendix A prints the small1 x small2 table (scheme 1,0,-1)."""
    s1, s2 = pair("small")
    t = oracle.fill(s1, s2)
    assert t[-1, -1] == 2
    assert list(t[3]) == [-3, -1, 0, 1, 1, 0, -1]
    assert list(t[:, 0]) == [-i for i in range(11)]


@pytest.mark.parametrize("name", ["small", "t", "debug", "smid", "2gb", "4gb"])
def test_scores_match_reference(golden, pair, name):
    s1, s2 = pair(name)
    for scheme, want in golden["pairs"][name]["scores"].items():
        assert oracle.score(s1, s2, SCHEMES[scheme]) == want, (name, scheme)


@pytest.mark.parametrize("scheme", list(SCHEMES))
@pytest.mark.parametrize("name", ["smid", "2gb"])
def test_rows_match_reference(pair, scheme, name):
    s1, s2 = pair(name)
    ref = np.load(f"{GOLDEN}/rows_{scheme}_{name}.npz")
    sc, lr, lc, rs, rw = oracle.score(s1, s2, SCHEMES[scheme], want_rows=True)
    np.testing.assert_array_equal(lr, ref["last_row"])
    np.testing.assert_array_equal(lc, ref["last_col"])
    np.testing.assert_array_equal(rs, ref["row_sum"])
    np.testing.assert_array_equal(rw, ref["row_wsum"])


def test_reference_mt_fills_agree(golden):
    """sentinel-mt / idxarray-mt (reference) produced tables equal to serial."""
    for name, e in golden["pairs"].items():
        for scheme, d in e.get("mt_table_equal", {}).items():
            assert all(d.values()), (name, scheme, d)


def _random_pair(rng, n1, n2, alphabet):
    if alphabet == "dna":
        return (rng.integers(1, 5, n1).astype(np.int8), rng.integers(1, 5, n2).astype(np.int8))
    return (rng.integers(-128, 128, n1).astype(np.int8), rng.integers(-128, 128, n2).astype(np.int8))


@pytest.mark.parametrize("shape", [(0, 0), (0, 5), (5, 0), (1, 1), (7, 3), (64, 64), (65, 129), (300, 257)])
@pytest.mark.parametrize("alphabet", ["dna", "bytes"])
def test_score_equals_full_fill(shape, alphabet):
    rng = np.random.default_rng(hash((shape, alphabet)) & 0xFFFF)
    s1, s2 = _random_pair(rng, *shape, alphabet)
    for scheme in SCHEMES.values():
        t = oracle.fill(s1, s2, scheme)
        sc, lr, lc, rs, rw = oracle.score(s1, s2, scheme, want_rows=True)
        assert sc == t[-1, -1]
        np.testing.assert_array_equal(lr, t[-1])
        np.testing.assert_array_equal(lc, t[:, -1])
        ers, erw = oracle.row_checksums(t)
        np.testing.assert_array_equal(rs, ers)
        np.testing.assert_array_equal(rw, erw)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("shape", [(0, 0), (0, 3), (4, 0), (1, 1), (33, 70), (129, 64), (500, 311)])
def test_oracle_vs_reference_random(shape):
    """Random inputs, including arbitrary signed bytes (the reference never validates)."""
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    for alphabet in ("dna", "bytes"):
        s1, s2 = _random_pair(rng, *shape, alphabet)
        for scheme, libname in (("shipped", "libref_serial.so"), ("mm1", "libref_serial_mm1.so"),
                                ("p3", "libref_serial_p3.so")):
            np.testing.assert_array_equal(oracle.fill(s1, s2, SCHEMES[scheme]),
                                          oracle.ref_fill(s1, s2, libname))


@pytest.mark.parametrize("shape", [(1, 1), (40, 90), (257, 100)])
def test_idxarray_restatement(shape):
    rng = np.random.default_rng(7)
    s1, s2 = _random_pair(rng, *shape, "dna")
    for nt in (1, 3, 8):
        np.testing.assert_array_equal(oracle.fill_idxarray(s1, s2, (1, -1, -1), nt),
                                      oracle.fill(s1, s2, (1, -1, -1)))


@pytest.mark.parametrize("n2", [0, 1, 7, 8, 9, 63, 100])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_band_partition_composes(n2, P):
    """mpi-horz row bands (mpi-horz-driver.cpp:31-32, mpi-horz.cpp:16): bands
    stitched through their halo rows reproduce the full table."""
    if n2 + 1 < P:
        pytest.skip("reference requires >= 1 row per band")
    rng = np.random.default_rng(n2 * 10 + P)
    s1, s2 = _random_pair(rng, 37, n2, "dna")
    full = oracle.fill(s1, s2, (1, -1, -1))
    rows, halo, covered = [], None, 0
    for r in range(P):
        nr, st = oracle.band_layout(n2, P, r)
        band = oracle.fill_band(s1, s2, P, r, halo, (1, -1, -1))
        assert band.shape == (nr, s1.size + 1)
        np.testing.assert_array_equal(band, full[st:st + nr])
        rows.append(band if r == 0 else band[1:])
        halo = band[-1]
        covered += nr - (r > 0)
    assert covered == n2 + 1
    np.testing.assert_array_equal(np.concatenate(rows), full)


@pytest.mark.skipif(not oracle.ref_available("libref_idxarray_emb_mt.so"),
                    reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("name", TINY + ["smid"])
def test_emb_layout_matches_reference(pair, name):
    """oracle.fill_emb (the restatement the GPU emb path is checked against) equals the
    reference's own idxarray-emb-mt fill (src/idxarray/idxarray-emb-mt.cpp:4-65,
    driver2.cpp:20-22 layout), progress column included."""
    s1, s2 = pair(name)
    want = oracle.ref_fill(s1, s2, "libref_idxarray_emb_mt.so", extra_cols=1)
    np.testing.assert_array_equal(oracle.fill_emb(s1, s2), want)
