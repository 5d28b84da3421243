"""GPU parity: the gfx950 fill vs the reference's own outputs and the oracle.

Everything here calls through the C ABI (libnwhip.so) -- the host path
(nw_fill, reference table layout) and the device-resident path
(nw_fill_device, table kept in HBM).  Bar: bit-exact int32.
"""
import os
import subprocess

import numpy as np
import pytest

import nwhip
import oracle
from conftest import GOLDEN, PKG, ROOT, bdna_path

pytestmark = pytest.mark.gpu
SCHEMES = oracle.SCHEMES
TINY = ["small", "small_rev", "t", "debug"]


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


# every supported (columns per lane C, compute waves per strip NC)
STRIP_SHAPES = [(4, 1), (2, 1), (1, 1), (2, 2), (1, 2), (1, 4)]


def alloc_aligned_table(torch, n1, n2):
    """A table whose base is 256-byte aligned (strip origin column 0: the boundary
    column is swept like any other), instead of alloc_table's column-1 alignment."""
    rows, pitch = nwhip.table_rows(n2), nwhip.table_pitch(n1)
    flat = torch.empty(rows * pitch + 64, dtype=torch.int32, device="cuda")
    shift = (-(flat.data_ptr() // 4)) % 64
    return flat[shift:shift + rows * pitch].view(rows, pitch)


def device_fill(torch, ctx, s1, s2, scheme=(1, 0, -1), waves=0, substrips=0, strip_waves=0,
                col0=1, kernel=nwhip.KERNEL_AUTO):
    d1 = torch.from_numpy(np.ascontiguousarray(s1)).cuda()
    d2 = torch.from_numpy(np.ascontiguousarray(s2)).cuda()
    if col0 == 1:
        tab = nwhip.Context.alloc_table(s1.size, s2.size)
    else:
        tab = alloc_aligned_table(torch, s1.size, s2.size)
    r = ctx.fill(d1, d2, tab, scheme, waves=waves, substrips=substrips, strip_waves=strip_waves, kernel=kernel)
    assert r.status == 0
    return tab, r


def device_row_checksums(torch, tab, n_rows, n_cols, chunk=1024):
    """(sum, column-weighted sum) per row, mod 2^64 -- oracle.row_checksums on the GPU."""
    w = torch.arange(1, n_cols + 1, dtype=torch.int64, device=tab.device)
    rs, rw = [], []
    for r0 in range(0, n_rows, chunk):
        r1 = min(n_rows, r0 + chunk)
        t64 = tab[r0:r1, :n_cols].to(torch.int64)
        rs.append(t64.sum(dim=1).cpu())
        rw.append((t64 * w).sum(dim=1).cpu())
    return (torch.cat(rs).numpy().view(np.uint64), torch.cat(rw).numpy().view(np.uint64))


# ------------------------------------------------------------------ golden (reference)
@pytest.mark.parametrize("scheme", list(SCHEMES))
@pytest.mark.parametrize("name", TINY)
def test_full_table_vs_reference(pair, scheme, name):
    s1, s2 = pair(name)
    t, r = nwhip.fill(s1, s2, SCHEMES[scheme])
    np.testing.assert_array_equal(t, np.load(f"{GOLDEN}/table_{scheme}_{name}.npy"))
    assert r.score == t[-1, -1]


@pytest.mark.parametrize("name", ["small", "t", "debug", "smid", "2gb", "4gb", "8gb", "mid", "big"])
def test_score_vs_reference(golden, pair, name):
    s1, s2 = pair(name)
    for scheme, want in golden["pairs"][name]["scores"].items():
        assert nwhip.score(s1, s2, SCHEMES[scheme]) == want, (name, scheme)


@pytest.mark.parametrize("scheme", list(SCHEMES))
@pytest.mark.parametrize("name", ["smid", "2gb"])
def test_rows_vs_reference(torch, ctx, pair, scheme, name):
    s1, s2 = pair(name)
    ref = np.load(f"{GOLDEN}/rows_{scheme}_{name}.npz")
    tab, r = device_fill(torch, ctx, s1, s2, SCHEMES[scheme])
    n_rows, n_cols = s2.size + 1, s1.size + 1
    np.testing.assert_array_equal(tab[n_rows - 1, :n_cols].cpu().numpy(), ref["last_row"])
    np.testing.assert_array_equal(tab[:n_rows, n_cols - 1].cpu().numpy(), ref["last_col"])
    rs, rw = device_row_checksums(torch, tab, n_rows, n_cols)
    np.testing.assert_array_equal(rs, ref["row_sum"])
    np.testing.assert_array_equal(rw, ref["row_wsum"])
    assert r.score == ref["last_row"][-1]


# ------------------------------------------------------------------ oracle, random shapes
SHAPES = [(0, 0), (0, 1), (1, 0), (1, 1), (2, 3), (63, 63), (64, 64), (65, 65), (63, 65),
          (127, 1), (1, 127), (128, 129), (129, 128), (191, 200), (255, 257), (1000, 37),
          (37, 1000), (640, 640), (1500, 1100)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("alphabet", ["dna", "bytes"])
@pytest.mark.parametrize("strip", STRIP_SHAPES)
@pytest.mark.parametrize("form", ["table", "compare"])
def test_random_vs_oracle(shape, alphabet, strip, form):
    """Both substitution forms: per-lane v_perm score tables (default; the "bytes"
    alphabet has more distinct column characters than a table covers and falls
    back on the device) and byte compares (NW_FLAG_NO_PROFILE), for every strip
    shape (C columns per lane, NC chained compute waves)."""
    rng = np.random.default_rng(shape[0] * 7919 + shape[1] + (alphabet == "bytes"))
    lo, hi = (1, 5) if alphabet == "dna" else (-128, 128)
    s1 = rng.integers(lo, hi, shape[0]).astype(np.int8)
    s2 = rng.integers(lo, hi, shape[1]).astype(np.int8)
    flags = nwhip.FLAG_NO_PROFILE if form == "compare" else 0
    for scheme in SCHEMES.values():
        t, r = nwhip.fill(s1, s2, scheme, substrips=strip[0], strip_waves=strip[1], flags=flags)
        assert (r.substrips, r.strip_waves) == strip
        np.testing.assert_array_equal(t, oracle.fill(s1, s2, scheme),
                                      err_msg=str((shape, scheme, strip, form)))


@pytest.mark.parametrize("shape", [(0, 5), (1, 1), (63, 70), (255, 300), (256, 256), (257, 100),
                                   (511, 77), (1000, 333)])
@pytest.mark.parametrize("strip", STRIP_SHAPES)
def test_strip_origin_column0(torch, ctx, shape, strip):
    """A 256-byte aligned table base sweeps column 0 with the strips (origin 0);
    alloc_table's base (column 1 aligned) stores the boundary column apart
    (origin 1).  Both give the reference table."""
    rng = np.random.default_rng(shape[0] + 31 * shape[1])
    s1 = rng.integers(1, 5, shape[0]).astype(np.int8)
    s2 = rng.integers(1, 5, shape[1]).astype(np.int8)
    for col0 in (0, 1):
        for scheme in [(1, 0, -1), (2, -1, -2)]:
            tab, r = device_fill(torch, ctx, s1, s2, scheme, substrips=strip[0],
                                 strip_waves=strip[1], col0=col0)
            np.testing.assert_array_equal(tab[:s2.size + 1, :s1.size + 1].cpu().numpy(),
                                          oracle.fill(s1, s2, scheme), err_msg=str((col0, scheme)))


@pytest.mark.parametrize("ndistinct", [1, 2, 6, 7, 8, 40])
def test_table_count_boundary(ndistinct):
    """Up to 7 distinct column characters use the v_perm score tables, more fall
    back to compares inside the kernel; the table is the same either way.  Row
    characters outside the column alphabet (never matching) are included."""
    rng = np.random.default_rng(ndistinct)
    alphabet = rng.choice(np.arange(-128, 128), ndistinct, replace=False)
    s1 = rng.choice(alphabet, 900).astype(np.int8)
    s1[:ndistinct] = alphabet  # every character present
    s2 = rng.integers(-128, 128, 650).astype(np.int8)
    s2[::3] = rng.choice(alphabet, s2[::3].size)
    for scheme in [(1, 0, -1), (2, -1, -2), (7, -5, 3)]:
        t, _ = nwhip.fill(s1, s2, scheme)
        np.testing.assert_array_equal(t, oracle.fill(s1, s2, scheme), err_msg=str(scheme))


@pytest.mark.parametrize("scheme", [(3, -2, -2), (1, 1, -1), (0, -1, -3), (5, 0, 0), (2, -3, 1),
                                    (150, -10, -1), (-5, -200, 3), (4095, -4095, -4095)])
def test_other_schemes_vs_oracle(scheme):
    """Runtime scores beyond the reference's #defines (incl. gap 0, a positive gap,
    and scores whose s - GAP leaves int8, which take the compare form)."""
    rng = np.random.default_rng(11)
    s1 = rng.integers(1, 5, 700).astype(np.int8)
    s2 = rng.integers(1, 5, 333).astype(np.int8)
    t, _ = nwhip.fill(s1, s2, scheme)
    np.testing.assert_array_equal(t, oracle.fill(s1, s2, scheme))


def test_score_range_refused():
    """The kernel holds w = t - GAP*(i+j) in int32: a scheme/size whose
    (max|score| + |GAP|) * (n1 + n2 + 2) reaches 2^28 is refused (NW_ERR_ARG),
    never silently wrapped; just below the bound it fills."""
    s = nwhip.synth(1, 16400)
    with pytest.raises(nwhip.NwError) as e:
        nwhip.score(s, s, (4095, -4095, -4095))
    assert e.value.status == nwhip.NW_ERR_ARG
    small = s[:1000]
    assert nwhip.score(small, small, (4095, -4095, -4095)) == oracle.score(small, small, (4095, -4095, -4095))


@pytest.mark.parametrize("flags", [nwhip.FLAG_DEBUG_NO_STORE, nwhip.FLAG_DEBUG_DRAIN, nwhip.FLAG_DEBUG_STAGGER,
                                   1 << 20, 8])
def test_unknown_or_debug_flags_refused(flags):
    """Flag bits are checked: unknown bits, and the compute-pace probes (which leave
    the table unwritten) without NW_FLAG_TIMING_ONLY, are refused (NW_ERR_ARG).
    (Round 4 shared bits 4 / 8 between NW_FLAG_NO_FINISH and the probes.)"""
    s = nwhip.synth(1, 300)
    with pytest.raises(nwhip.NwError) as e:
        nwhip.fill(s, s, (1, 0, -1), flags=flags)
    assert e.value.status == nwhip.NW_ERR_ARG


@pytest.mark.gpu
def test_no_chain_probe_refused_on_bands(torch, ctx):
    """The store-pattern probe (NW_FLAG_DEBUG_NO_CHAIN: strips unchained, no fill) is
    refused wherever a band would hand its rows on, and accepted on a whole table."""
    n1, rows = 1000, 100
    d1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
    d2 = torch.from_numpy(nwhip.synth(2, rows)).cuda()
    tab = nwhip.Context.alloc_table(n1, rows)
    halo = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")
    with pytest.raises(nwhip.NwError) as e:
        ctx.fill_band(d1, d2, tab, halo_in=halo, tag=1, row0=5000, flags=nwhip.FLAG_DEBUG_NO_CHAIN)
    assert e.value.status == nwhip.NW_ERR_ARG
    ctx.fill(d1, d2, tab, flags=nwhip.FLAG_DEBUG_NO_CHAIN | nwhip.FLAG_DEBUG_STAGGER, kernel=nwhip.KERNEL_STRIPS)
    #  Smith-Waterman: an unchained table has no meaningful best cell
    for fl in (nwhip.FLAG_DEBUG_NO_CHAIN, nwhip.FLAG_DEBUG_NO_CHAIN | nwhip.FLAG_TIMING_ONLY):
        with pytest.raises(nwhip.NwError) as e:
            ctx.fill(d1, d2, tab, scheme=(1, -1, -1), mode=nwhip.MODE_SW, flags=fl, kernel=nwhip.KERNEL_STRIPS)
        assert e.value.status == nwhip.NW_ERR_ARG
    torch.cuda.synchronize()


def test_band_score_range_refused(torch, ctx):
    """A band's halo row carries global values: the range check uses the band's global
    row (nw_band.row0), so a band of a table the whole-table path refuses is refused too."""
    n1, rows = 1000, 100
    d1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
    d2 = torch.from_numpy(nwhip.synth(2, rows)).cuda()
    tab = nwhip.Context.alloc_table(n1, rows)
    halo = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")
    scheme = (4095, -4095, -4095)  # (4095 + 4095) * (n1 + row0 + rows + 2) >= 2^28 from row0 ~ 31k
    with pytest.raises(nwhip.NwError) as e:
        ctx.fill_band(d1, d2, tab, halo_in=halo, tag=1, scheme=scheme, row0=40000)
    assert e.value.status == nwhip.NW_ERR_ARG
    ctx.fill_band(d1, d2, tab, halo_in=None, tag=1, scheme=scheme, row0=0)  # accepted
    torch.cuda.synchronize()


@pytest.mark.parametrize("strip", [(2, 2), (1, 4)])
def test_watchdog_reports_timeout(torch, strip):
    """A band whose halo never arrives (its tag is never written) must not hang the
    device: every bounded wait gives up after nw_params.timeout_ms, the launch
    reports NW_ERR_TIMEOUT, and the control words name the wait (code 2: halo wait,
    site 4, the tag it needed).  Afterwards the same context fills correctly."""
    c = nwhip.Context(0)
    try:
        n1, rows = 64 * 40 + 5, 300
        s1 = nwhip.synth(3, n1)
        s2 = nwhip.synth(4, rows)
        d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
        tab = nwhip.Context.alloc_table(n1, rows)
        halo = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")  # tag 0 everywhere
        import time
        t0 = time.time()
        c.fill_band(d1, d2, tab, halo_in=halo, tag=7, timeout_ms=200,
                    substrips=strip[0], strip_waves=strip[1])
        assert c.status() == nwhip.NW_ERR_TIMEOUT
        assert time.time() - t0 < 30
        w = c.debug_ctrl()
        assert w[1] == 2                 # halo wait gave up (nw_fill.hip give_up code 2)
        assert (w[2] >> 24) == 4         # site 4: the halo wait at the start of a strip
        assert w[3] == 7                 # the tag it needed
        # the context recovers: a normal fill right after is exact
        tab2, r = device_fill(torch, c, s1, s2, (1, 0, -1), substrips=strip[0], strip_waves=strip[1])
        assert r.status == 0
        np.testing.assert_array_equal(tab2[:rows + 1, :n1 + 1].cpu().numpy(), oracle.fill(s1, s2))
    finally:
        c.close()


@pytest.mark.parametrize("kernel", [nwhip.KERNEL_STRIPS, nwhip.KERNEL_PANELS])
def test_failure_is_sticky_across_launches(torch, kernel):
    """a watchdog trip in launch k of a back-to-back sweep must survive
    the launches after it.  Launch 1 waits for a halo that never comes (200 ms
    bound); launches 2 and 3 are enqueued behind it with no status read between:
    they start poisoned and give up at once (no 20 s wait each, no halo published),
    and the one status read afterwards reports NW_ERR_TIMEOUT with launch 1's
    diagnosis (code 2 halo wait, tag 7) and 3 failed launches.  The read clears the
    record: the next fill is exact."""
    import time
    c = nwhip.Context(0)
    try:
        n1, rows = 64 * 40 + 5, 300
        s1, s2 = nwhip.synth(3, n1), nwhip.synth(4, rows)
        d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
        tab = nwhip.Context.alloc_table(n1, rows)
        halo = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")  # tag 0 everywhere
        out = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")
        t0 = time.time()
        c.fill_band(d1, d2, tab, halo_in=halo, tag=7, timeout_ms=200, kernel=kernel)
        torch.cuda.synchronize()
        t1 = time.time()
        for tag in (8, 9):  # a normal band fill (no halo in), publishing its last row
            c.fill_band(d1, d2, tab, halo_out=out, tag=tag, timeout_ms=20000, kernel=kernel)
        torch.cuda.synchronize()
        assert time.time() - t1 < 5, "poisoned launches must give up at once"
        assert t1 - t0 < 30
        assert int((out >> 32).count_nonzero()) == 0, "a poisoned launch published its halo"
        code, site, need, seen, nfail = c.debug_failure()
        # strips: the halo wait at a strip's start (code 2, site 4, the tag); panels:
        # both the compute waves (code 2, site 4) and the feeder-in wave (granule
        # wait, code 1, site 13) wait on the halo -- whichever expires first records
        wants = [(2, 4)] if kernel == nwhip.KERNEL_STRIPS else [(2, 4), (1, 13)]
        assert (code, site >> 24) in wants and nfail == 3  # launch 1 + the two poisoned ones
        if (code, site >> 24) == (2, 4):
            assert need == 7
        assert c.status() == nwhip.NW_ERR_TIMEOUT
        assert c.debug_failure()[0] == code  # as the status read cleared it
        assert c.debug_failure()[4] == 3
        assert c.status() == nwhip.NW_OK  # cleared
        tab2, r = device_fill(torch, c, s1, s2, (1, 0, -1), kernel=kernel)
        assert r.status == 0
        np.testing.assert_array_equal(tab2[:rows + 1, :n1 + 1].cpu().numpy(), oracle.fill(s1, s2))
    finally:
        c.close()


def test_link_wait_timeout_poisons_the_producer(torch):
    """a producer whose consumer never releases a buffer (its link word
    never reaches the launch) must not rewrite that buffer.  The expired
    nw_link_wait_ctx_async records code 4 in the producer's context, so its next
    band fill publishes nothing, and the context's status reports the failure."""
    c = nwhip.Context(0)
    link = nwhip.Link(0)
    try:
        n1, rows = 64 * 40 + 5, 300
        d1 = torch.from_numpy(nwhip.synth(3, n1)).cuda()
        d2 = torch.from_numpy(nwhip.synth(4, rows)).cuda()
        tab = nwhip.Context.alloc_table(n1, rows)
        out = torch.zeros(n1 + 1, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream()
        nwhip.link_wait(link.ptr, 5, st, timeout_ms=100, ctx=c)  # nobody signals 5
        c.fill_band(d1, d2, tab, halo_out=out, tag=3)
        torch.cuda.synchronize()
        assert link.status() == 5
        assert int((out >> 32).count_nonzero()) == 0
        code, site, need, seen, nfail = c.debug_failure()
        assert (code, site >> 24, need, seen) == (4, 20, 5, 0)
        assert c.status() == nwhip.NW_ERR_TIMEOUT and c.status() == nwhip.NW_OK
    finally:
        link.free()
        c.close()


@pytest.mark.parametrize("waves", [1, 2, 3, 5, 8, 17, 64])
@pytest.mark.parametrize("strip", STRIP_SHAPES)
def test_worker_count_independent(torch, ctx, waves, strip):
    """Few persistent workers -> many strips per worker and hand-off slot reuse
    (slot = strip % (waves + 1)); results must not depend on it."""
    rng = np.random.default_rng(waves)
    s1 = rng.integers(1, 5, 64 * 40 + 17).astype(np.int8)
    s2 = rng.integers(1, 5, 900).astype(np.int8)
    want = oracle.fill(s1, s2, (1, -1, -1))
    tab, r = device_fill(torch, ctx, s1, s2, (1, -1, -1), waves=waves, substrips=strip[0],
                         strip_waves=strip[1])
    np.testing.assert_array_equal(tab[:s2.size + 1, :s1.size + 1].cpu().numpy(), want)
    assert r.waves == min(waves, r.strips)


def test_repeated_launches_and_shapes(torch, ctx):
    """The hand-off tags advance per launch; stale granules of earlier launches
    (other shapes, same buffers) must never be taken for fresh ones."""
    rng = np.random.default_rng(5)
    shapes = [(2000, 300), (300, 2000), (2000, 300), (777, 777), (64 * 50, 128), (2000, 300)]
    for n1, n2 in shapes:
        s1 = rng.integers(1, 5, n1).astype(np.int8)
        s2 = rng.integers(1, 5, n2).astype(np.int8)
        tab, _ = device_fill(torch, ctx, s1, s2, (1, 0, -1), waves=7)
        np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), oracle.fill(s1, s2))


@pytest.mark.parametrize("strip", [(4, 1), (2, 1), (2, 2), (1, 4)])
def test_config2_32k_vs_oracle(torch, ctx, strip):
    """BASELINE config 2: 32k x 32k synthetic (seeds 1, 2), full table in HBM;
    every row checked through (sum, weighted sum), last row/column exactly."""
    n = 32768
    s1, s2 = nwhip.synth(1, n), nwhip.synth(2, n)
    tab, r = device_fill(torch, ctx, s1, s2, (1, 0, -1), substrips=strip[0], strip_waves=strip[1])
    sc, lr, lc, rs, rw = oracle.score(s1, s2, (1, 0, -1), want_rows=True)
    assert r.score == sc
    np.testing.assert_array_equal(tab[n, :n + 1].cpu().numpy(), lr)
    np.testing.assert_array_equal(tab[:n + 1, n].cpu().numpy(), lc)
    grs, grw = device_row_checksums(torch, tab, n + 1, n + 1)
    np.testing.assert_array_equal(grs, rs)
    np.testing.assert_array_equal(grw, rw)


# ------------------------------------------------------------------ emb layout
@pytest.mark.parametrize("scheme", list(SCHEMES))
@pytest.mark.parametrize("name", TINY + ["smid"])
def test_emb_layout_vs_oracle(pair, scheme, name):
    """nw_fill_emb: the driver2.cpp / idxarray-emb-mt table (n1+2 columns, progress
    column 0 = n1+2, columns 1.. = serial), bit-exact."""
    s1, s2 = pair(name)
    import ctypes
    t = np.full((s2.size + 1, s1.size + 2), -7, dtype=np.int32)
    p = nwhip.params(SCHEMES[scheme])
    L = nwhip.lib()
    L.nw_fill_emb.argtypes = L.nw_fill.argtypes
    i8 = ctypes.POINTER(ctypes.c_int8)
    a, b = np.ascontiguousarray(s1), np.ascontiguousarray(s2)
    st = L.nw_fill_emb(a.ctypes.data_as(i8), a.size, b.ctypes.data_as(i8), b.size, ctypes.byref(p),
                       t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), None)
    assert st == nwhip.NW_OK
    np.testing.assert_array_equal(t, oracle.fill_emb(s1, s2, SCHEMES[scheme]))


@pytest.mark.parametrize("name", ["small", "t", "debug", "smid"])
def test_dropin_driver_emb_cli(golden, name):
    """build/nw_driver_emb: driver2.cpp's stdout is the wall milliseconds only (no
    newline, no score), exit status 0."""
    e = golden["pairs"][name]
    out = subprocess.run([os.path.join(PKG, "build", "nw_driver_emb"), bdna_path(e["argv1"]),
                          bdna_path(e["argv2"])], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.isdigit()


# ------------------------------------------------------------------ drop-in CLI
@pytest.mark.parametrize("drv,name,want", [("nw_driver", "small", 2), ("nw_driver", "t", 17),
                                           ("nw_driver", "debug", 27), ("nw_driver", "smid", 5839),
                                           ("nw_driver_mm1", "small", 2), ("nw_driver_mm1", "t", 6),
                                           ("nw_driver_mm1", "smid", 3955)])
def test_dropin_driver_cli(golden, drv, name, want):
    e = golden["pairs"][name]
    out = subprocess.run([os.path.join(PKG, "build", drv), bdna_path(e["argv1"]),
                          bdna_path(e["argv2"])], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().split("\n")
    assert len(lines) == 2 and lines[0].isdigit()          # "<ms>" (driver.cpp:33)
    assert lines[1] == f"Score: {want}"                      # driver.cpp:35


@pytest.mark.gpu
@pytest.mark.parametrize("name,want", [("small", 2), ("t", 17), ("debug", 27), ("smid", 5839)])
def test_reference_driver_links_the_dropin(golden, name, want):
    """The reference's OWN, unmodified driver.cpp + helper.cpp (compiled in the build
    container by oracle/Makefile ref-dropin into oracle/_ref/ref_driver_hip) linked
    against the drop-in TU: the genuine caller of the plugin symbol runs the HIP fill."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_driver_hip")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/ref_driver_hip not built (needs the reference tree at build time)")
    e = golden["pairs"][name]
    out = subprocess.run([exe, bdna_path(e["argv1"]), bdna_path(e["argv2"])], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().split("\n")
    assert len(lines) == 2 and lines[0].isdigit()
    assert lines[1] == f"Score: {want}"
