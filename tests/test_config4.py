"""BASELINE config 4's real per-rank workload on one MI355X.

Config 4 is the 524288 x 524288 table split into 8 contiguous row bands across 8
GPUs (src/mpi/mpi-horz-driver.cpp:31-32: base = (n2+1)/8 = 65536 rows, band r > 0
starts at its halo row 65536 r - 1, the last band takes the remainder row; the
score is the last band's last cell, :88-90).  One rank's band is 65537-65538 rows
x 524289 columns = 137 GB of int32 -- it fits one MI355X.  Here a rank's band is
filled ALONE, with its halo row pre-published from the pinned oracle's fixture
(tests/golden/make_config4.py) exactly as the upstream rank's kernel would publish
it: {tag, value} granules, raw table values for the vertical sweep
(nw_fill_band_async), w-form values for the horizontal one (nw_fill_tband_async).
The band's own published boundary is captured and compared with the next band's
halo row, so both ends of the multi-GPU hand-off are checked at full size.

CPU: the fixture decodes consistently (score, boundary rows, sums).
GPU: ranks 3 and 7 in both sweeps: every row's checksums, the last column, the
boundary rows and the fixture's rows inside the band cell by cell, the published
last row, and (rank 7) the final score 214685.
"""
import json
import os

import numpy as np
import pytest

import nwhip
import oracle
from conftest import GOLDEN, config4_golden

N, P, SCHEME = 524288, 8, (1, 0, -1)
GAP = SCHEME[2]


@pytest.fixture(scope="module")
def g():
    out = config4_golden()
    if out is None:
        pytest.skip("tests/golden/config4_524288_shipped.npz not generated")
    return out


def full_row(g, r: int) -> np.ndarray:
    k = int(np.searchsorted(g["rows"], r))
    assert g["rows"][k] == r, f"row {r} is not in the fixture"
    return g["full"][k]


# ------------------------------------------------------------------ CPU
def test_fixture_consistent(g):
    with open(os.path.join(GOLDEN, "synth_scores.json")) as f:
        assert g["score"] == json.load(f)[f"{N}:1,0,-1"] == 214685
    assert g["full"].shape == (g["rows"].size, N + 1)
    assert g["full"][-1, -1] == g["score"] == g["last_col"][-1] and g["rows"][-1] == N
    assert g["last_col"].size == N + 1 and g["last_col"][0] == N * GAP
    for r in range(1, P):  # every band's halo row and first computed row
        _, st = nwhip.band_layout(N, P, r)
        assert st == 65536 * r - 1 and {st, st + 1} <= set(g["rows"].tolist())
    for k, r in enumerate(g["rows"]):  # exact rows agree with the last column
        assert g["full"][k, N] == g["last_col"][r]
    for b in g["cs_bands"]:
        rows, st = nwhip.band_layout(N, P, b)
        assert g["row_sum"][b].size == rows
        sel = [k for k, r in enumerate(g["rows"]) if st <= r < st + rows]
        assert len(sel) >= 6
        rs, rw = oracle.row_checksums(g["full"][sel])
        np.testing.assert_array_equal(rs, g["row_sum"][b][g["rows"][sel] - st])
        np.testing.assert_array_equal(rw, g["row_wsum"][b][g["rows"][sel] - st])


def test_fixture_row1_matches_oracle(g):
    """Row 1 re-derived here (one row of the recurrence, instant)."""
    np.testing.assert_array_equal(oracle.rows(oracle.synth(1, N), oracle.synth(2, N), SCHEME, [1])[0],
                                  full_row(g, 1))


def test_band_layout_matches_oracle():
    for r in range(P):
        assert nwhip.band_layout(N, P, r) == oracle.band_layout(N, P, r)


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    return _t


def granules(torch, values: np.ndarray, tag: int, size: int):
    """{tag, value} granules (tag in the high word) as an int64 CUDA tensor of `size`:
    the values, then padding granules carrying the tag (a producer publishes whole
    64-granule blocks; the consumer takes them 16 at a time)."""
    v = values.astype(np.int64) & 0xFFFFFFFF
    out = np.full(size, np.int64(tag) << 32, np.int64)
    out[:v.size] |= v
    return torch.from_numpy(out).cuda()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("sweep", ["vertical", "horizontal"])
@pytest.mark.parametrize("rank", [3, 7])
def test_config4_rank_band_alone(torch, g, rank, sweep):
    from test_full_size import row_checksums
    rows, start = nwhip.band_layout(N, P, rank)
    last = rank == P - 1
    tag = 11
    torch.cuda.empty_cache()
    ctx = nwhip.Context(0)
    tab = nwhip.Context.alloc_table(N, rows - 1)  # 137 GB
    try:
        d1 = torch.from_numpy(nwhip.synth(1, N)).cuda()
        d2 = torch.from_numpy(nwhip.synth(2, N)[start:start + rows - 1].copy()).cuda()
        halo_row = full_row(g, start)
        j = np.arange(N + 1, dtype=np.int64)
        if sweep == "vertical":
            hin = granules(torch, halo_row, tag, N + 1)
            hout = None if last else torch.zeros(N + 1, dtype=torch.int64, device="cuda")
            ctx.fill_band(d1, d2, tab, halo_in=hin, halo_out=hout, tag=tag, row0=start)
        else:
            fsize = nwhip.feed_bytes(N) // 8
            hin = granules(torch, halo_row.astype(np.int64) - GAP * (j + start), tag, fsize)
            hout = None if last else torch.zeros(fsize, dtype=torch.int64, device="cuda")
            ctx.fill_tband(d1, d2, tab, row0=start, feed_in=hin, feed_out=hout, tag=tag)
        st = ctx.status()
        assert st == nwhip.NW_OK, f"status {st}, first failure {ctx.debug_failure()}"
        want_last = full_row(g, start + rows - 1)
        np.testing.assert_array_equal(tab[rows - 1, :N + 1].cpu().numpy(), want_last)
        np.testing.assert_array_equal(tab[:rows, N].cpu().numpy(), g["last_col"][start:start + rows])
        np.testing.assert_array_equal(tab[0, :N + 1].cpu().numpy(), halo_row)
        for k, r in enumerate(g["rows"]):
            if start <= r < start + rows:
                got = tab[int(r) - start, :N + 1].cpu().numpy()
                bad = np.flatnonzero(got != g["full"][k])
                assert bad.size == 0, f"row {r}: {bad.size} cells differ, first col {bad[0]}"
        if rank in g["cs_bands"]:
            rs, rw = row_checksums(torch, tab, rows, N + 1)
            bad = np.flatnonzero((rs != g["row_sum"][rank]) | (rw != g["row_wsum"][rank]))
            assert bad.size == 0, f"{bad.size} rows differ, first {(bad[:5] + start).tolist()}"
        if last:
            assert int(tab[rows - 1, N].item()) == g["score"] == 214685
        else:  # what the next rank would receive
            pub = hout.cpu().numpy()[:N + 1]
            assert np.all((pub >> 32) == tag)
            vals = (pub & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
            if sweep == "horizontal":
                vals = vals + GAP * (j + start + rows - 1)
            np.testing.assert_array_equal(vals, want_last)
    finally:
        del tab
        ctx.close()
        torch.cuda.empty_cache()
