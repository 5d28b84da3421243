"""GPU parity of the row-scan PANEL kernel (nw_params.kernel = NW_KERNEL_PANELS,
csrc/nw_rows.hip) against the oracle and the golden vectors.

The panel kernel computes the same table as the reference fills
(src/serial/serial.cpp:21-33) as a prefix maximum per row; every test goes
through the C ABI and compares bit-exact int32 cells.
"""
import numpy as np
import pytest

import nwhip
import oracle
from conftest import big_rows

pytestmark = pytest.mark.gpu
SCHEMES = oracle.SCHEMES
P = nwhip.KERNEL_PANELS
# every supported panel shape (C columns per lane, NW compute waves per panel)
PANEL_SHAPES = [(4, 4), (4, 2), (2, 4), (4, 1), (2, 2), (1, 4)]


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    return _t


@pytest.fixture(scope="module")
def ctx(torch):
    c = nwhip.Context(0)
    yield c
    c.close()


SHAPES = [(0, 0), (0, 1), (1, 0), (1, 1), (2, 3), (63, 65), (64, 64), (127, 1), (1, 127),
          (255, 257), (1000, 37), (37, 1000), (1500, 1100), (3000, 700), (5000, 130)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("alphabet", ["dna", "bytes"])
@pytest.mark.parametrize("panel", PANEL_SHAPES)
@pytest.mark.parametrize("form", ["table", "compare"])
def test_panel_random_vs_oracle(shape, alphabet, panel, form):
    """Both substitution forms (v_perm tables; byte compares, also reached on the
    device when s1 has more distinct characters than a table covers) for every
    panel shape; the wide shapes cross several panels (granule hand-offs)."""
    rng = np.random.default_rng(shape[0] * 7919 + shape[1] + (alphabet == "bytes"))
    lo, hi = (1, 5) if alphabet == "dna" else (-128, 128)
    s1 = rng.integers(lo, hi, shape[0]).astype(np.int8)
    s2 = rng.integers(lo, hi, shape[1]).astype(np.int8)
    flags = nwhip.FLAG_NO_PROFILE if form == "compare" else 0
    for scheme in SCHEMES.values():
        t, r = nwhip.fill(s1, s2, scheme, substrips=panel[0], strip_waves=panel[1], flags=flags, kernel=P)
        assert (r.substrips, r.strip_waves, r.kernel) == (panel[0], panel[1], P)
        np.testing.assert_array_equal(t, oracle.fill(s1, s2, scheme), err_msg=str((shape, scheme, panel, form)))


def alloc_aligned_table(torch, n1, n2):
    rows, pitch = nwhip.table_rows(n2), nwhip.table_pitch(n1)
    flat = torch.empty(rows * pitch + 64, dtype=torch.int32, device="cuda")
    shift = (-(flat.data_ptr() // 4)) % 64
    return flat[shift:shift + rows * pitch].view(rows, pitch)


@pytest.mark.parametrize("shape", [(0, 5), (1, 1), (63, 70), (256, 256), (1023, 77), (2049, 333)])
@pytest.mark.parametrize("panel", [(4, 4), (2, 4), (4, 1), (1, 4)])
def test_panel_origin_column0(torch, ctx, shape, panel):
    """A 256-byte aligned base sweeps column 0 with the panels (no left column:
    the lane holding column 0 takes t[i][0] = t[i-1][0] + GAP from the up term)."""
    rng = np.random.default_rng(shape[0] + 3 * shape[1])
    s1 = rng.integers(1, 5, shape[0]).astype(np.int8)
    s2 = rng.integers(1, 5, shape[1]).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    for scheme in SCHEMES.values():
        for tab in (nwhip.Context.alloc_table(s1.size, s2.size), alloc_aligned_table(torch, s1.size, s2.size)):
            r = ctx.fill(d1, d2, tab, scheme, substrips=panel[0], strip_waves=panel[1], kernel=P)
            assert r.status == 0
            np.testing.assert_array_equal(tab[:s2.size + 1, :s1.size + 1].cpu().numpy(),
                                          oracle.fill(s1, s2, scheme))


@pytest.mark.parametrize("waves", [1, 2, 3, 5])
@pytest.mark.parametrize("panel", [(4, 4), (2, 2), (1, 4)])
def test_panel_worker_count(torch, ctx, waves, panel):
    """Fewer persistent workers than panels: tickets, granule slots (M = workers
    + 1) and repeated launches on one context (fresh tags each launch)."""
    rng = np.random.default_rng(waves)
    s1 = rng.integers(1, 5, 9000).astype(np.int8)
    s2 = rng.integers(1, 5, 700).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    want = oracle.fill(s1, s2, (1, -1, -1))
    tab = nwhip.Context.alloc_table(s1.size, s2.size)
    for _ in range(2):
        tab.fill_(-7)
        r = ctx.fill(d1, d2, tab, (1, -1, -1), waves=waves, substrips=panel[0], strip_waves=panel[1], kernel=P)
        assert r.status == 0 and r.waves == waves
        np.testing.assert_array_equal(tab[:s2.size + 1, :s1.size + 1].cpu().numpy(), want)


@pytest.mark.parametrize("scheme", [(1, -1, -1), (1, 0, -1), (2, -1, -2)])
@pytest.mark.parametrize("panel", [(4, 4), (2, 4), (4, 1), (1, 4), (2, 2)])
@pytest.mark.parametrize("n1,n2,alpha", [(1, 1, 4), (63, 64, 4), (300, 1000, 4), (1500, 1100, 4),
                                         (1000, 300, 20), (4100, 513, 4)])
def test_panel_sw_vs_oracle(torch, ctx, scheme, panel, n1, n2, alpha):
    """Smith-Waterman (parity unpinned: the oracle is the build's restatement):
    tables, best cell and the traceback from it."""
    rng = np.random.default_rng(n1 * 3 + n2 + alpha)
    s1 = rng.integers(1, alpha + 1, n1).astype(np.int8)
    s2 = rng.integers(1, alpha + 1, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n1, n2)
    r = ctx.fill(d1, d2, tab, scheme, substrips=panel[0], strip_waves=panel[1], mode=nwhip.MODE_SW, kernel=P)
    assert r.status == 0
    want = oracle.sw_fill(s1, s2, scheme)
    np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), want)
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)
    al, ops = ctx.sw_traceback(d1, d2, tab, (r.end_i, r.end_j), scheme)
    wops, bi, bj = oracle.sw_traceback(s1, s2, want, (r.end_i, r.end_j), scheme)
    np.testing.assert_array_equal(ops, wops)


@pytest.mark.slow
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1)])
@pytest.mark.parametrize("panel", [(0, 0), (4, 1), (2, 2), (1, 4)])
def test_panel_64k_every_row(torch, ctx, scheme, panel):
    """65536 x 65536: every row's (sum, weighted sum) checksums, the last row and
    column, 32 whole rows (scheme (1, 0, -1)) and the score against the pinned
    linear-memory oracle's vectors."""
    from test_gpu_parity import device_row_checksums
    n = 65536
    g = big_rows(n, n, scheme)
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    r = ctx.fill(s1, s2, tab, scheme, substrips=panel[0], strip_waves=panel[1], kernel=P)
    assert r.status == 0 and r.score == g["score"]
    np.testing.assert_array_equal(tab[n, :n + 1].cpu().numpy(), g["last_row"])
    np.testing.assert_array_equal(tab[:n + 1, n].cpu().numpy(), g["last_col"])
    rs, rw = device_row_checksums(torch, tab, n + 1, n + 1)
    np.testing.assert_array_equal(rs, g["row_sum"])
    np.testing.assert_array_equal(rw, g["row_wsum"])
    from test_full_size import check_full_rows
    check_full_rows(torch, tab, n, n, scheme)  # exact cells where the fixture has rows
