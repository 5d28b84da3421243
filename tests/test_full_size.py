"""Parity at BASELINE's full sizes (configs 3 and 4), against row-level golden
vectors from the pinned oracle (tests/golden/make_big_rows.py; the reference
itself cannot hold these tables in host RAM -- SURVEY.md 8(c)).

Every row of the device table is compared through its (sum, column-weighted sum)
checksum; the last row and the last column exactly; ~32 whole rows per table
(rows 1, 63, 64, 65, 255, 256, n2, band boundaries, seeded random rows;
make_big_rows.py FULL_JOBS) cell by cell; the final score against
synth_scores.json.  Recurrence: src/serial/serial.cpp:21-33; band partition:
src/mpi/mpi-horz-driver.cpp:31-32, mpi-horz.cpp:16-40.

CPU (-m "not gpu"): the golden files decode consistently, agree with
synth_scores.json, and the 64k file matches the oracle recomputed here.
GPU (-m gpu): config 3 (262144^2, 275 GB table, one MI355X) under both schemes,
the 64k/128k squares, and a 524288 x 32767 table split as config 4 is on 8 GPUs:
8 row bands of 4096 rows (LocalBands) and 8 column bands of 256 strips
(LocalColBands, mpi-vert.cpp:4-109).
"""
import json
import os

import numpy as np
import pytest

import nwhip
import oracle
from conftest import GOLDEN, big_full_rows, big_rows

SQUARES = [(65536, (1, 0, -1)), (65536, (1, -1, -1)), (131072, (1, 0, -1)), (131072, (1, -1, -1)),
           (262144, (1, 0, -1)), (262144, (1, -1, -1))]


def synth_scores():
    with open(os.path.join(GOLDEN, "synth_scores.json")) as f:
        return json.load(f)


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("n,scheme", SQUARES)
def test_golden_rows_consistent(n, scheme):
    g = big_rows(n, n, scheme)
    assert g["last_row"].size == n + 1 and g["last_col"].size == n + 1
    assert g["row_sum"].size == n + 1 and g["row_wsum"].size == n + 1
    assert g["score"] == g["last_row"][-1] == g["last_col"][-1]
    assert g["score"] == synth_scores()[f"{n}:{','.join(map(str, scheme))}"]
    # row 0 is the boundary j*GAP (serial.cpp:16); column n1 of row i continues it
    gap = scheme[2]
    want = sum(j * gap for j in range(n + 1)) % (1 << 64)
    assert int(g["row_sum"][0]) == want
    assert g["last_col"][0] == n * gap


def test_golden_band_geometry_consistent():
    g = big_rows(524288, 32767, (1, 0, -1))
    assert g["last_row"].size == 524289 and g["row_sum"].size == 32768
    assert g["score"] == g["last_row"][-1] == g["last_col"][-1]


FULL = [(65536, 65536, (1, 0, -1)), (262144, 262144, (1, 0, -1)), (262144, 262144, (1, -1, -1)),
        (524288, 32767, (1, 0, -1))]


@pytest.mark.parametrize("n1,n2,scheme", FULL)
def test_golden_full_rows_consistent(n1, n2, scheme):
    """The exact-row fixtures agree with the row-level vectors: each row's
    checksums, and the last row where it is among them."""
    rows, t = big_full_rows(n1, n2, scheme)
    g = big_rows(n1, n2, scheme)
    assert t.shape == (rows.size, n1 + 1) and rows.size >= 32 and rows[-1] == n2
    assert {1, 63, 64, 65, 255, 256} <= set(rows.tolist())
    rs, rw = oracle.row_checksums(t)
    np.testing.assert_array_equal(rs, g["row_sum"][rows])
    np.testing.assert_array_equal(rw, g["row_wsum"][rows])
    np.testing.assert_array_equal(t[-1], g["last_row"])
    np.testing.assert_array_equal(t[:, n1], g["last_col"][rows])


def test_golden_64k_full_rows_match_oracle():
    """Re-derive the 64k exact rows with the oracle here (a few seconds)."""
    n, scheme = 65536, (1, 0, -1)
    rows, t = big_full_rows(n, n, scheme)
    np.testing.assert_array_equal(oracle.rows(oracle.synth(1, n), oracle.synth(2, n), scheme, rows), t)


def test_golden_64k_rows_match_oracle():
    """Re-derive the 64k golden file with the oracle here (17 s)."""
    n, scheme = 65536, (1, 0, -1)
    g = big_rows(n, n, scheme)
    sc, lr, lc, rs, rw = oracle.score(oracle.synth(1, n), oracle.synth(2, n), scheme, want_rows=True)
    assert sc == g["score"]
    np.testing.assert_array_equal(lr, g["last_row"])
    np.testing.assert_array_equal(lc, g["last_col"])
    np.testing.assert_array_equal(rs, g["row_sum"])
    np.testing.assert_array_equal(rw, g["row_wsum"])


# ------------------------------------------------------------------ GPU
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


def row_checksums(torch, tab, rows, n_cols, chunk=256, col_first=0, col_base=0):
    """(sum, column-weighted sum) per row mod 2^64 (oracle.row_checksums) on the device,
    `rows` = the table rows to check, in chunks (a few hundred MB of temporaries next
    to a 275 GB table).  Columns col_first .. n_cols-1 of `tab`, local column k being
    global column col_base + k (a column band's part of the sums)."""
    w = torch.arange(col_base + col_first + 1, col_base + n_cols + 1, dtype=torch.int64, device=tab.device)
    rs, rw = [], []
    for r0 in range(0, rows, chunk):
        r1 = min(rows, r0 + chunk)
        t64 = tab[r0:r1, col_first:n_cols].to(torch.int64)
        rs.append(t64.sum(dim=1).cpu())
        rw.append((t64 * w).sum(dim=1).cpu())
        del t64
    return (torch.cat(rs).numpy().view(np.uint64), torch.cat(rw).numpy().view(np.uint64))


def check_full_rows(torch, tab, n1, n2, scheme, row0=0, col_base=0, ncols=None, nrows=None):
    """Cell-by-cell comparison of the fixture's exact rows that fall in this
    table (global rows row0 .. row0 + nrows - 1, global columns col_base ..
    col_base + ncols - 1)."""
    fr = big_full_rows(n1, n2, scheme)
    if fr is None:
        return 0
    rows, want = fr
    ncols = n1 + 1 if ncols is None else ncols
    nrows = n2 + 1 - row0 if nrows is None else nrows
    sel = [k for k, r in enumerate(rows) if row0 <= r < row0 + nrows]
    for k in sel:
        got = tab[int(rows[k]) - row0, :ncols].cpu().numpy()
        exp = want[k, col_base:col_base + ncols]
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, (f"row {rows[k]}: {bad.size} cells differ, first col "
                               f"{col_base + bad[0]} got {got[bad[0]]} want {exp[bad[0]]} ({scheme})")
    return len(sel)


def check_square(torch, ctx, n, schemes, substrips=0, strip_waves=0, kernel=0):
    torch.cuda.empty_cache()
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    try:
        for scheme in schemes:
            g = big_rows(n, n, scheme)
            r = ctx.fill(s1, s2, tab, scheme, substrips=substrips, strip_waves=strip_waves, kernel=kernel)
            assert r.status == 0
            assert r.score == g["score"]
            np.testing.assert_array_equal(tab[n, :n + 1].cpu().numpy(), g["last_row"])
            np.testing.assert_array_equal(tab[:n + 1, n].cpu().numpy(), g["last_col"])
            rs, rw = row_checksums(torch, tab, n + 1, n + 1)
            bad = np.flatnonzero((rs != g["row_sum"]) | (rw != g["row_wsum"]))
            assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5].tolist()} ({scheme})"
            check_full_rows(torch, tab, n, n, scheme)
    finally:
        del tab
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("kernel", [nwhip.KERNEL_AUTO, nwhip.KERNEL_STRIPS])
def test_config3_256k_every_row(torch, ctx, kernel):
    """BASELINE config 3: 262144 x 262144 on one MI355X, both schemes, every row,
    the auto choice (the panels on a 256-CU MI355X) and the strips."""
    check_square(torch, ctx, 262144, [(1, 0, -1), (1, -1, -1)], kernel=kernel)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("n", [65536, 131072])
def test_squares_every_row(torch, ctx, n):
    check_square(torch, ctx, n, [(1, 0, -1), (1, -1, -1)])


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("strip", [(2, 2), (1, 4), (4, 1)])
def test_128k_every_row_by_strip_shape(torch, ctx, strip):
    check_square(torch, ctx, 131072, [(1, 0, -1)], substrips=strip[0], strip_waves=strip[1])


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("sweep", ["vertical", "horizontal"])
def test_config4_band_geometry(torch, sweep):
    """BASELINE config 4's row bands (524288 columns, 8 bands, mpi-horz partition) with
    4096 rows per band, concurrently on one device through the in-kernel halo hand-off
    (the 8-GPU run uses the same kernels with the halo in peer HBM), swept in vertical
    strips (LocalBands, the bench's `rows_contiguous` leg) and in horizontal strips
    (LocalTBands, the `rows_horizontal` leg): every row of every band against the
    whole-table golden rows."""
    import nw_bands
    n1, n2, P = 524288, 32767, 8
    g = big_rows(n1, n2, (1, 0, -1))
    torch.cuda.empty_cache()
    lb = nw_bands.LocalBands(n1, n2, P) if sweep == "vertical" else nw_bands.LocalTBands(n1, n2, P)
    try:
        score = lb.fill(torch.from_numpy(nwhip.synth(1, n1)).cuda(),
                        torch.from_numpy(nwhip.synth(2, n2)).cuda())
        assert score == g["score"]
        for r, (rows, start) in enumerate(lb.layout):
            tab = lb.tables[r]
            rs, rw = row_checksums(torch, tab, rows, n1 + 1)
            np.testing.assert_array_equal(rs, g["row_sum"][start:start + rows], err_msg=f"band {r}")
            np.testing.assert_array_equal(rw, g["row_wsum"][start:start + rows], err_msg=f"band {r}")
            np.testing.assert_array_equal(tab[:rows, n1].cpu().numpy(), g["last_col"][start:start + rows])
            check_full_rows(torch, tab, n1, n2, (1, 0, -1), row0=start, nrows=rows)
        rows, _ = lb.layout[-1]
        np.testing.assert_array_equal(lb.tables[-1][rows - 1, :n1 + 1].cpu().numpy(), g["last_row"])
    finally:
        lb.close()
        del lb
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.slow
def test_config4_colband_geometry(torch):
    """The same 524288 x 32767 table as 8 column bands (mpi-vert partition, the bench's
    default multi-GPU one), concurrently on one device through the in-kernel feed
    hand-off: every row's checksums assembled over the bands (each band's shared left
    column counted once), the last row and last column against the golden rows."""
    import nw_bands
    n1, n2, P = 524288, 32767, 8
    g = big_rows(n1, n2, (1, 0, -1))
    torch.cuda.empty_cache()
    lb = nw_bands.LocalColBands(n1, n2, P)
    try:
        score = lb.fill(torch.from_numpy(nwhip.synth(1, n1)).cuda(),
                        torch.from_numpy(nwhip.synth(2, n2)).cuda())
        assert score == g["score"]
        rs_all = np.zeros(n2 + 1, np.uint64)
        rw_all = np.zeros(n2 + 1, np.uint64)
        for r, (sf, sc, start, ncols) in enumerate(lb.layout):
            tab = lb.tables[r]
            rs, rw = row_checksums(torch, tab, n2 + 1, ncols, col_first=1 if r else 0, col_base=start)
            rs_all += rs
            rw_all += rw
            np.testing.assert_array_equal(tab[n2, :ncols].cpu().numpy(), g["last_row"][start:start + ncols],
                                          err_msg=f"band {r}")
            assert check_full_rows(torch, tab, n1, n2, (1, 0, -1), col_base=start, ncols=ncols) >= 32
        np.testing.assert_array_equal(rs_all, g["row_sum"])
        np.testing.assert_array_equal(rw_all, g["row_wsum"])
        np.testing.assert_array_equal(lb.tables[-1][:n2 + 1, lb.layout[-1][3] - 1].cpu().numpy(), g["last_col"])
    finally:
        lb.close()
        del lb
        torch.cuda.empty_cache()
