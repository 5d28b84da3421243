"""Row bands in horizontal strips (nw_fill_tband_async): the mpi-horz contract
(src/mpi/mpi-horz.cpp:4-99, mpi-horz-driver.cpp:31-32,88-90) with each band swept
as 256-row strips along the columns, band r-1's last row fed to band r column by
column.

CPU (-m "not gpu"): the transposition contract the sweep rests on, with the
oracle's band restatements.
GPU (-m gpu): LocalTBands -- several bands concurrently on one device through
the in-kernel feed hand-off -- bit-exact against the oracle's whole table (the
serial.cpp:4-36 restatement) on ragged shapes, every scheme form, repeated
launches, a 32k config-2 score and every row of a config-4-width band set; the
argument refusals.  The multi-process leg is covered by test_bands.py's
shared-GPU bench test.
"""
import ctypes
import sys

import numpy as np
import pytest

import nwhip
import oracle
from conftest import PKG

sys.path.insert(0, PKG)
import nw_bands  # noqa: E402


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


# ------------------------------------------------------------------ contract (CPU)
@pytest.mark.parametrize("n1,n2,P", [(300, 200, 2), (129, 1000, 5), (7, 64, 3), (1000, 777, 8)])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1), (2, -1, -2), (1, -1, 0)])
def test_row_band_is_the_transposed_column_band(n1, n2, P, scheme):
    """What nw_fill_tband_async computes: row band r of the table of (s1, s2) -- its row 0
    the previous band's last row (mpi-horz.cpp:28-40) -- is the transpose of the column band
    of the table of (s2, s1) over the same global indices with that row as its left column
    (mpi-vert.cpp:4-109's contract), the scores being symmetric (serial.cpp:23-30).  Checked
    with the oracle's own band restatements, band by band against the whole table."""
    rng = np.random.default_rng(n1 + 7 * n2 + P)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    full = oracle.fill(s1, s2, scheme)
    np.testing.assert_array_equal(oracle.fill(s2, s1, scheme).T, full)
    for r in range(P):
        rows, start = oracle.band_layout(n2, P, r)
        halo = full[start] if r > 0 else None
        band_t = oracle.fill_colband(s2, s1, start, rows, halo, scheme)  # (n1 + 1) x rows
        np.testing.assert_array_equal(band_t.T, full[start:start + rows], err_msg=f"band {r}")
        np.testing.assert_array_equal(oracle.fill_band(s1, s2, P, r, halo, scheme), full[start:start + rows])


SHAPES = [(4, 1), (2, 2)]  # the horizontal strip shapes (256 rows each)


def _check(torch, n1, n2, P, scheme, seed, alphabet=4, shape=(4, 1), dense=False):
    rng = np.random.default_rng(seed)
    s1 = rng.integers(1, alphabet + 1, n1).astype(np.int8)
    s2 = rng.integers(1, alphabet + 1, n2).astype(np.int8)
    tb = nw_bands.LocalTBands(n1, n2, P, shape=shape, dense_polls=dense)
    try:
        score = tb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda(), scheme)
        full = oracle.fill(s1, s2, scheme)
        for r, (rows, start) in enumerate(tb.layout):
            got = tb.tables[r][:rows, :n1 + 1].cpu().numpy()
            np.testing.assert_array_equal(got, full[start:start + rows], err_msg=f"band {r}")
        assert score == full[-1, -1]
    finally:
        tb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,P", [(300, 200, 1), (300, 200, 2), (1000, 777, 3), (640, 130, 4),
                                     (129, 40, 1), (64 * 37 + 5, 999, 5), (5, 600, 3), (4100, 1300, 2),
                                     (33, 257, 1), (1, 513, 2), (2000, 20, 8), (97, 1025, 4)])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1), (2, -1, -2)])
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_local_tbands_vs_oracle(torch_gpu, n1, n2, P, scheme, shape):
    """Partial first/last strips, bands of a few rows, 1-column tables, widths that are
    not a multiple of the 32-column store batch; the v_perm form (scores - 2 GAP
    in int8) and the compare forms (UNIT: match - mismatch == 1, GEN: (2,-1,-2)); both
    strip shapes ((2, 2): the band's last row may sit in either compute wave's ring)."""
    _check(torch_gpu, n1, n2, P, scheme, n1 * 31 + n2 + P, shape=shape)


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,P", [(300, 200, 2), (1000, 777, 3), (64 * 37 + 5, 999, 5), (1, 513, 2),
                                     (2000, 20, 8)])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (2, -1, -2)])
def test_local_tbands_dense_polls(torch_gpu, n1, n2, P, scheme):
    """NW_TBAND_DENSE_POLLS (the long-chain poll policy, s_sleep 1 between polls): the same
    bands, bit-exact."""
    _check(torch_gpu, n1, n2, P, scheme, n1 * 17 + n2 + P, dense=True)


def test_dense_poll_policy():
    """bench.py --tband-polls auto: dense from chains of DENSE_POLL_STRIPS strips of 256 rows
    (N >= 2 at 65536 rows per GPU), sparse below; explicit choices win."""
    import argparse
    a = argparse.Namespace(tband_polls="auto")
    assert nw_bands.tband_dense(a, 2 * 65536) and nw_bands.tband_dense(a, 4 * 65536)
    assert not nw_bands.tband_dense(a, 65536) and not nw_bands.tband_dense(a, 65536 + 65535)
    assert nw_bands.tband_dense(a, 8 * 65536) and not nw_bands.tband_dense(a, 65536)
    assert nw_bands.tband_dense(argparse.Namespace(tband_polls="dense"), 256)
    assert not nw_bands.tband_dense(argparse.Namespace(tband_polls="sparse"), 8 * 65536)
    assert nw_bands.tband_dense(argparse.Namespace(), 2 * 65536) and not nw_bands.tband_dense(argparse.Namespace(), 65536)
    with pytest.raises(ValueError):
        nw_bands.tband_dense(argparse.Namespace(tband_polls="fast"), 1)


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", [(1, 0, -1), (3, -2, -1), (1, -1, 0), (2, 1, 1)])
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_local_tbands_alphabets_and_schemes(torch_gpu, scheme, shape):
    """More than kMaxPerm distinct row characters (the compare fallback), gap 0 and a
    positive gap."""
    _check(torch_gpu, 700, 900, 3, scheme, 5, alphabet=20, shape=shape)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_local_tbands_repeated_launches(torch_gpu, shape):
    """Tags advance per launch; stale feed granules of earlier launches are never taken."""
    torch = torch_gpu
    n1, n2, P = 2000, 1500, 3
    tb = nw_bands.LocalTBands(n1, n2, P, shape=shape)
    try:
        for seed in range(4):
            rng = np.random.default_rng(seed)
            s1 = rng.integers(1, 5, n1).astype(np.int8)
            s2 = rng.integers(1, 5, n2).astype(np.int8)
            score = tb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda())
            full = oracle.fill(s1, s2)
            assert score == full[-1, -1]
            for r, (rows, start) in enumerate(tb.layout):
                np.testing.assert_array_equal(tb.tables[r][:rows, :n1 + 1].cpu().numpy(),
                                              full[start:start + rows])
    finally:
        tb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_local_tbands_32k_score(torch_gpu, shape):
    """BASELINE config-2 inputs split into 4 concurrent horizontal-strip bands."""
    torch = torch_gpu
    n = 32768
    s1, s2 = nwhip.synth(1, n), nwhip.synth(2, n)
    tb = nw_bands.LocalTBands(n, n, 4, shape=shape)
    try:
        score = tb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda())
        assert score == 13394  # reference serial.cpp on the same inputs (synth_scores.json)
        sc, lr, lc, rs, rw = oracle.score(s1, s2, want_rows=True)
        for r, (rows, start) in enumerate(tb.layout):
            sums, wsums = oracle.row_checksums(tb.tables[r][:rows, :n + 1].cpu().numpy())
            np.testing.assert_array_equal(sums, rs[start:start + rows], err_msg=f"band {r} sums")
            np.testing.assert_array_equal(wsums, rw[start:start + rows], err_msg=f"band {r} wsums")
        rows, _ = tb.layout[-1]
        np.testing.assert_array_equal(tb.tables[-1][rows - 1, :n + 1].cpu().numpy(), lr)
    finally:
        tb.close()


@pytest.mark.gpu
def test_tband_refusals(torch_gpu):
    torch = torch_gpu
    n1, n2 = 300, 200
    s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
    ctx = nwhip.Context(0)
    tab = nwhip.Context.alloc_table(n1, n2)
    feed = nwhip.Feed(n1, 0)
    try:
        with pytest.raises(nwhip.NwError) as e:  # a band below row 0 needs its feed
            ctx.fill_tband(s1, s2, tab, row0=5)
        assert e.value.status == nwhip.NW_ERR_ARG
        with pytest.raises(nwhip.NwError) as e:  # band 0 has no feed
            ctx.fill_tband(s1, s2, tab, row0=0, feed_in=feed.ptr)
        assert e.value.status == nwhip.NW_ERR_ARG
        with pytest.raises(nwhip.NwError) as e:  # tag 0 is never a launch tag
            ctx.fill_tband(s1, s2, tab, tag=0)
        assert e.value.status == nwhip.NW_ERR_ARG
        big = nwhip.Context.alloc_table(n1, n2 + 64)
        rows = nwhip.table_rows(n2)
        with pytest.raises(nwhip.NwError) as e:  # misaligned table base (column 1 off its 256-B line)
            ctx.fill_tband(s1, s2, big.view(-1)[1:1 + rows * big.shape[1]].view(rows, big.shape[1]))
        assert e.value.status == nwhip.NW_ERR_ARG
        with pytest.raises(nwhip.NwError) as e:  # Smith-Waterman is the single-table path's
            lib_p = nwhip.params((1, -1, -1), mode=nwhip.MODE_SW)
            st = nwhip.lib().nw_fill_tband_async(ctx._h, ctypes.c_void_p(s1.data_ptr()), n1,
                                                 ctypes.c_void_p(s2.data_ptr()), n2, ctypes.byref(lib_p),
                                                 ctypes.byref(nwhip.NwTBand(None, None, 1, 0, 0)),
                                                 ctypes.c_void_p(tab.data_ptr()), tab.shape[1], None)
            if st != nwhip.NW_OK:
                raise nwhip.NwError(st, "nw_fill_tband_async")
        assert e.value.status == nwhip.NW_ERR_UNSUPPORTED
        with pytest.raises(nwhip.NwError) as e:  # unknown nw_tband.flags bits
            lib_p = nwhip.params((1, 0, -1))
            st = nwhip.lib().nw_fill_tband_async(ctx._h, ctypes.c_void_p(s1.data_ptr()), n1,
                                                 ctypes.c_void_p(s2.data_ptr()), n2, ctypes.byref(lib_p),
                                                 ctypes.byref(nwhip.NwTBand(None, None, 1, 2, 0)),
                                                 ctypes.c_void_p(tab.data_ptr()), tab.shape[1], None)
            if st != nwhip.NW_OK:
                raise nwhip.NwError(st, "nw_fill_tband_async")
        assert e.value.status == nwhip.NW_ERR_ARG
        for sub, nc in [(1, 4), (2, 1), (1, 1), (2, 4), (4, 2)]:  # 256-row (4, 1) / (2, 2) strips only
            with pytest.raises(nwhip.NwError) as e:
                ctx.fill_tband(s1, s2, tab, substrips=sub, strip_waves=nc)
            assert e.value.status in (nwhip.NW_ERR_UNSUPPORTED, nwhip.NW_ERR_ARG), (sub, nc)
        torch.cuda.synchronize()
        ctx.fill_tband(s1, s2, tab)  # and the context still works
        torch.cuda.synchronize()
        assert ctx.status() == nwhip.NW_OK
        assert int(tab[n2, n1].item()) == oracle.score(nwhip.synth(1, n1), nwhip.synth(2, n2))
    finally:
        feed.free()
        ctx.close()


# ------------------------------------------------------------------ the row-scan finisher
def _tband_chain(torch, s1, s2, P, scheme, waves, flags=0, row_split=None, shape=(4, 1)):
    """P bands of the (s1, s2) table, each filled by its own nw_fill_tband_async with
    `waves` workers, one after the other on one stream (band r's feed_out is band r+1's
    feed_in).  Returns (band tables, [published feed of band r]) as numpy."""
    n1, n2 = s1.size, s2.size
    ctx = nwhip.Context(0)
    d1 = torch.from_numpy(s1).cuda()
    fsize = nwhip.feed_bytes(n1) // 8
    feeds = [torch.zeros(fsize, dtype=torch.int64, device="cuda") for _ in range(P - 1)]
    out, pub = [], []
    try:
        for r in range(P):
            rows, start = oracle.band_layout(n2, P, r) if row_split is None else row_split[r]
            tab = nwhip.Context.alloc_table(n1, rows - 1)
            tab.fill_(-0x5A5A5A5)  # (torch.empty may hand back an earlier table's memory)
            d2 = torch.from_numpy(s2[start:start + rows - 1].copy()).cuda()
            ctx.fill_tband(d1, d2, tab, row0=start, feed_in=feeds[r - 1] if r > 0 else None,
                           feed_out=feeds[r] if r + 1 < P else None, tag=5, scheme=scheme, waves=waves,
                           flags=flags, substrips=shape[0], strip_waves=shape[1])
            torch.cuda.synchronize()
            assert ctx.status() == nwhip.NW_OK, f"band {r}: {ctx.debug_failure()}"
            out.append(tab[:rows, :n1 + 1].cpu().numpy())
            if r + 1 < P:
                pub.append(feeds[r].cpu().numpy()[:n1 + 1])
        return out, pub
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n1", [1, 100, 2047, 2048, 2049, 5000])
@pytest.mark.parametrize("waves,extra", [(1, 1), (2, 7), (2, 64), (3, 200), (1, 256), (4, 129)])
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_tband_finisher_rows(torch_gpu, n1, waves, extra, shape):
    """A band whose last strip would run alone as one more pass over all columns
    (strips = k * workers + 1) leaves that strip's rows (`extra` of them) to the
    row-scan finisher (nw_finish.hip): one prefix-max scan per row across the width,
    chunks of 2048 columns chained by a decoupled look-back.  Bit-exact against the
    oracle under three scheme forms, with and without a halo row above it, and the
    feed it publishes for the next band equals its last row (w form)."""
    torch = torch_gpu
    R = 256 * waves + extra  # strips = waves + 1
    rng = np.random.default_rng(n1 * 7 + waves * 131 + extra)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, 2 * R + 1).astype(np.int8)
    for scheme in [(1, 0, -1), (1, -1, -1), (2, -1, -2)]:
        full = oracle.fill(s1, s2, scheme)
        split = [(R + 1, 0), (R + 1, R)]  # two bands of R computed rows each, the second below a halo
        tabs, pub = _tband_chain(torch, s1, s2, 2, scheme, waves, row_split=split, shape=shape)
        for r, (rows, start) in enumerate(split):
            np.testing.assert_array_equal(tabs[r], full[start:start + rows], err_msg=f"band {r} {scheme}")
        gap = scheme[2]
        vals = (pub[0] & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        np.testing.assert_array_equal(vals + gap * (np.arange(n1 + 1) + R), full[R], err_msg=f"feed {scheme}")
        assert np.all((pub[0] >> 32) == 5)


@pytest.mark.gpu
@pytest.mark.parametrize("n1", [100, 8191, 8192, 8193, 20000])
def test_tband_finisher_wide_chunks(torch_gpu, n1, monkeypatch):
    """the finisher's K = 32 instantiation (8192-column chunks, its own
    vector-store and tail code) is chosen only above ~4.2M columns; forced here with
    NW_DEBUG_FINISH_WIDE=1 on small widths (one and several chunks, ragged tails) and
    checked bit-exactly, with the feed it publishes."""
    monkeypatch.setenv("NW_DEBUG_FINISH_WIDE", "1")
    torch = torch_gpu
    waves, extra = 2, 37
    R = 256 * waves + extra
    rng = np.random.default_rng(n1 + 5)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, 2 * R + 1).astype(np.int8)
    for scheme in [(1, 0, -1), (2, -1, -2)]:
        full = oracle.fill(s1, s2, scheme)
        split = [(R + 1, 0), (R + 1, R)]
        tabs, pub = _tband_chain(torch, s1, s2, 2, scheme, waves, row_split=split)
        for r, (rows, start) in enumerate(split):
            np.testing.assert_array_equal(tabs[r], full[start:start + rows], err_msg=f"band {r} {scheme}")
        vals = (pub[0] & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        np.testing.assert_array_equal(vals + scheme[2] * (np.arange(n1 + 1) + R), full[R])
        assert np.all((pub[0] >> 32) == 5)


@pytest.mark.gpu
def test_tband_finisher_matches_full_pass(torch_gpu):
    """The finisher's rows equal the strip kernel's own second pass (NW_FLAG_NO_FINISH)."""
    torch = torch_gpu
    n1, waves = 3000, 2
    R = 256 * waves * 2 + 3  # strips = 2 * waves + 1
    rng = np.random.default_rng(9)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, R).astype(np.int8)
    a, _ = _tband_chain(torch, s1, s2, 1, (1, 0, -1), waves)
    b, _ = _tband_chain(torch, s1, s2, 1, (1, 0, -1), waves, flags=nwhip.FLAG_NO_FINISH)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[0], oracle.fill(s1, s2))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=["4x1", "2x2"])
def test_local_tbands_leftover_row(torch_gpu, shape):
    """The mpi-horz partition's leftover row (bands after the first carry their halo
    row, the last one the remainder): 2 bands sharing the GPU (each 1/2 of the workers),
    the second sweeping 32769 rows = 129 strips on 128 workers -- the configuration that
    ran a second full pass before the finisher."""
    _check(torch_gpu, 300, 65537, 2, (1, 0, -1), 3, shape=shape)
