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
GPU: ranks 0 (no halo: it seeds row 0 and only publishes), 3 and 7 in both
sweeps: every row's checksums, the last column, the boundary rows and the
fixture's rows inside the band cell by cell, the published last row, and (rank
7) the final score 214685.  And the real hand-off at full size: ranks 6 and 7
(274.9 GB together, as much as the 256k table) filled CONCURRENTLY on one GPU,
each on half the CUs, band 6's halo from the fixture and band 7's from band 6's
kernel, in both sweeps.
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


def halo_granules(torch, g, start: int, sweep: str, tag: int):
    """Band (start)'s halo row from the fixture as its upstream rank's kernel would
    publish it: raw values (vertical sweep, nw_fill_band_async) or w-form values
    w = t - GAP (start + j) (horizontal sweep's feed, nw_fill_tband_async)."""
    row = full_row(g, start)
    if sweep == "vertical":
        return granules(torch, row, tag, N + 1)
    j = np.arange(N + 1, dtype=np.int64)
    return granules(torch, row.astype(np.int64) - GAP * (j + start), tag, nwhip.feed_bytes(N) // 8)


def out_buffer(torch, sweep: str):
    return torch.zeros(N + 1 if sweep == "vertical" else nwhip.feed_bytes(N) // 8, dtype=torch.int64,
                       device="cuda")


def check_band(torch, g, tab, rank: int):
    """Band `rank`'s table against the fixture: its first (halo / boundary) and last
    rows, its last column, every fixture row inside it cell by cell, every row's
    checksums where the fixture has them, and (last rank) the score."""
    from test_full_size import row_checksums
    rows, start = nwhip.band_layout(N, P, rank)
    want_last = full_row(g, start + rows - 1)
    np.testing.assert_array_equal(tab[rows - 1, :N + 1].cpu().numpy(), want_last)
    np.testing.assert_array_equal(tab[:rows, N].cpu().numpy(), g["last_col"][start:start + rows])
    want_first = full_row(g, start) if start > 0 else GAP * np.arange(N + 1, dtype=np.int32)  # serial.cpp:16
    np.testing.assert_array_equal(tab[0, :N + 1].cpu().numpy(), want_first)
    for k, r in enumerate(g["rows"]):
        if start <= r < start + rows:
            got = tab[int(r) - start, :N + 1].cpu().numpy()
            bad = np.flatnonzero(got != g["full"][k])
            assert bad.size == 0, f"band {rank} row {r}: {bad.size} cells differ, first col {bad[0]}"
    if rank in g["cs_bands"]:
        rs, rw = row_checksums(torch, tab, rows, N + 1)
        bad = np.flatnonzero((rs != g["row_sum"][rank]) | (rw != g["row_wsum"][rank]))
        assert bad.size == 0, f"band {rank}: {bad.size} rows differ, first {(bad[:5] + start).tolist()}"
    if rank == P - 1:
        assert int(tab[rows - 1, N].item()) == g["score"] == 214685


def check_published(hout, g, rank: int, sweep: str, tag: int):
    """What band `rank` published for the next rank: its last row, every granule tagged."""
    rows, start = nwhip.band_layout(N, P, rank)
    pub = hout.cpu().numpy()[:N + 1]
    assert np.all((pub >> 32) == tag)
    vals = (pub & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
    if sweep == "horizontal":
        vals = vals + GAP * (np.arange(N + 1, dtype=np.int64) + start + rows - 1)
    np.testing.assert_array_equal(vals, full_row(g, start + rows - 1))


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("sweep", ["vertical", "horizontal"])
@pytest.mark.parametrize("rank", [0, 3, 7])
def test_config4_rank_band_alone(torch, g, rank, sweep):
    rows, start = nwhip.band_layout(N, P, rank)
    last = rank == P - 1
    tag = 11
    torch.cuda.empty_cache()
    ctx = nwhip.Context(0)
    tab = nwhip.Context.alloc_table(N, rows - 1)  # 137 GB
    try:
        d1 = torch.from_numpy(nwhip.synth(1, N)).cuda()
        d2 = torch.from_numpy(nwhip.synth(2, N)[start:start + rows - 1].copy()).cuda()
        hin = halo_granules(torch, g, start, sweep, tag) if rank > 0 else None  # rank 0: row 0 = boundary
        hout = None if last else out_buffer(torch, sweep)
        if sweep == "vertical":
            ctx.fill_band(d1, d2, tab, halo_in=hin, halo_out=hout, tag=tag, row0=start)
        else:
            ctx.fill_tband(d1, d2, tab, row0=start, feed_in=hin, feed_out=hout, tag=tag)
        st = ctx.status()
        assert st == nwhip.NW_OK, f"status {st}, first failure {ctx.debug_failure()}"
        check_band(torch, g, tab, rank)
        if not last:
            check_published(hout, g, rank, sweep, tag)
    finally:
        del tab
        ctx.close()
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("sweep", ["vertical", "horizontal"])
def test_config4_bands_6_7_handoff(torch, g, sweep):
    """the producer -> consumer hand-off at config-4 size.  Ranks 6 and 7
    (65537 + 65538 rows x 524289 = 274.9 GB) run CONCURRENTLY on one GPU, each on
    its own stream and context with half the resident workers (so both are
    co-resident and band 7 streams band 6's last row while band 6 still fills);
    band 6's halo is the fixture's row 393215, band 7's is published by band 6's
    kernel (the multi-GPU path's protocol, in local memory).  Both bands are
    checked against the fixture, band 7 through its score 214685."""
    import nw_bands
    tag = 13
    torch.cuda.empty_cache()
    lay = [nwhip.band_layout(N, P, r) for r in (6, 7)]
    ctxs = [nwhip.Context(0) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    tabs = [nwhip.Context.alloc_table(N, rows - 1) for rows, _ in lay]  # 2 x 137 GB
    try:
        d1 = torch.from_numpy(nwhip.synth(1, N)).cuda()
        s2 = nwhip.synth(2, N)
        d2 = [torch.from_numpy(s2[st:st + rows - 1].copy()).cuda() for rows, st in lay]
        hin = halo_granules(torch, g, lay[0][1], sweep, tag)
        link = out_buffer(torch, sweep)  # band 6 -> band 7
        if sweep == "vertical":
            waves = max(1, nw_bands.resident_waves(0, *nw_bands.band_shape(N, lay[1][0] - 1)) // 2)
        else:
            waves = max(1, nw_bands.resident_waves(0, 4, 1) // 2)
        torch.cuda.synchronize()
        for k, ((rows, st), stream) in enumerate(zip(lay, streams)):
            kw = dict(halo_in=hin if k == 0 else link, halo_out=link if k == 0 else None)
            if sweep == "vertical":
                ctxs[k].fill_band(d1, d2[k], tabs[k], tag=tag, row0=st, waves=waves, stream=stream, **kw)
            else:
                ctxs[k].fill_tband(d1, d2[k], tabs[k], row0=st, feed_in=kw["halo_in"], feed_out=kw["halo_out"],
                                   tag=tag, waves=waves, stream=stream)
        for k, stream in enumerate(streams):
            st = ctxs[k].status(stream)
            assert st == nwhip.NW_OK, f"band {6 + k}: status {st}, first failure {ctxs[k].debug_failure()}"
        torch.cuda.synchronize()
        check_published(link, g, 6, sweep, tag)
        check_band(torch, g, tabs[0], 6)
        check_band(torch, g, tabs[1], 7)
    finally:
        del tabs
        for c in ctxs:
            c.close()
        torch.cuda.empty_cache()
