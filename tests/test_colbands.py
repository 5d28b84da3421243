"""Column bands (multi-GPU path for n1 >> n2, mpi-vert contract:
src/mpi/mpi-vert.cpp:4-109, mpi-vert-driver.cpp:35-38).

CPU (-m "not gpu"): the oracle's restatement of a column band against the whole
table; the C ABI's strip-aligned layout (nw_colband_layout) tiles the columns
like mpi-vert's (one shared column between neighbours); the band / feed contract
over real world_size-2 and -3 gloo process groups (each rank fills its band with
the oracle, the left column travels rank to rank as the GPU path's feed granules
do), for both the reference's layout and the strip-aligned one.
GPU (-m gpu): LocalColBands -- several column bands concurrently on one device,
fed through the in-kernel feed hand-off -- bit-exact against the oracle, repeated
launches, refusals, and the multi-process bench path (--partition cols, 2 ranks
sharing the GPU) against the oracle's score.
"""
import datetime
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import nwhip
import oracle
from conftest import PKG, ROOT

sys.path.insert(0, PKG)
import nw_bands  # noqa: E402


# ------------------------------------------------------------------ layouts (CPU)
@pytest.mark.parametrize("n1,P", [(10, 2), (100, 3), (1000, 7), (524288, 8), (17, 8), (65535, 4)])
def test_oracle_colband_layout_tiles(n1, P):
    """mpi-vert: band r > 0 starts on band r-1's last column; the last band ends on n1."""
    lay = [oracle.colband_layout(n1, P, r) for r in range(P)]
    assert lay[0][1] == 0
    for (nc_a, st_a), (nc_b, st_b) in zip(lay, lay[1:]):
        assert st_b == st_a + nc_a - 1
    nc, st = lay[-1]
    assert st + nc - 1 == n1


@pytest.mark.parametrize("n1,n2,P,shape", [(1000, 50, 2, (1, 1)), (64 * 37 + 5, 999, 5, (2, 2)),
                                           (524287, 524288, 8, (0, 0)), (4096, 10, 4, (4, 1)),
                                           (300, 300, 1, (2, 1))])
def test_capi_colband_layout_tiles(n1, n2, P, shape):
    """nw_colband_layout: whole strips (W = 64 * C * NC columns from column 1) split
    over the bands, neighbouring local tables sharing one column as in mpi-vert."""
    sub, nc = nwhip.strip_shape(shape[0], shape[1], n1, n2)
    W = 64 * sub * nc
    S = -(-n1 // W)
    lay = [nwhip.colband_layout(n1, n2, P, r, shape[0], shape[1]) for r in range(P)]
    assert lay[0][0] == 0 and lay[0][2] == 0
    assert sum(x[1] for x in lay) == S and max(x[1] for x in lay) - min(x[1] for x in lay) <= 1
    for (sf_a, sc_a, st_a, nc_a), (sf_b, sc_b, st_b, nc_b) in zip(lay, lay[1:]):
        assert sf_b == sf_a + sc_a and st_b == sf_b * W and st_b == st_a + nc_a - 1
    sf, sc, st, ncols = lay[-1]
    assert st + ncols - 1 == n1


def test_capi_colband_layout_refuses_more_bands_than_strips():
    with pytest.raises(nwhip.NwError):
        nwhip.colband_layout(100, 100, 3, 0, 2, 2)  # one 256-column strip


@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1), (2, -1, -2)])
def test_oracle_colbands_reassemble_table(scheme):
    rng = np.random.default_rng(5)
    n1, n2 = 333, 121
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    full = oracle.fill(s1, s2, scheme)
    for P in (1, 2, 3, 7):
        left = None
        for r in range(P):
            nc, st = oracle.colband_layout(n1, P, r)
            band = oracle.fill_colband(s1, s2, st, nc, left, scheme)
            np.testing.assert_array_equal(band, full[:, st:st + nc], err_msg=f"P={P} r={r}")
            left = band[:, -1].copy()


# ------------------------------------------------------------------ gloo ranks (CPU)
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n1, n2, scheme, layout, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))  # fail, never hang
    s1, s2 = oracle.synth(21, n1), oracle.synth(22, n2)
    if layout == "reference":
        nc, st = oracle.colband_layout(n1, world, rank)
    else:
        _, _, st, nc = nwhip.colband_layout(n1, n2, world, rank, 1, 1)
    left = None
    if rank > 0:  # column 0 = rank-1's last column (mpi-vert.cpp:54-59)
        h = torch.empty(n2 + 1, dtype=torch.int32)
        dist.recv(h, src=rank - 1)
        left = h.numpy()
    band = oracle.fill_colband(s1, s2, st, nc, left, scheme)
    if rank + 1 < world:
        dist.send(torch.from_numpy(band[:, -1].copy()), dst=rank + 1)
    np.save(os.path.join(outdir, f"cb{rank}.npy"), band)
    np.save(os.path.join(outdir, f"cb{rank}_start.npy"), np.array([st]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("layout", ["reference", "strips"])
@pytest.mark.timeout(240)
def test_gloo_colbands_reassemble_the_table(tmp_path, world, layout):
    import torch.multiprocessing as mp
    n1, n2, scheme = 64 * 7 + 3, 211, (1, -1, -1)
    mp.spawn(_rank_main, args=(world, _free_port(), n1, n2, scheme, layout, str(tmp_path)),
             nprocs=world, join=True)
    full = oracle.fill(oracle.synth(21, n1), oracle.synth(22, n2), scheme)
    for r in range(world):
        band = np.load(tmp_path / f"cb{r}.npy")
        st = int(np.load(tmp_path / f"cb{r}_start.npy")[0])
        np.testing.assert_array_equal(band, full[:, st:st + band.shape[1]])
    # final score on the last rank's last cell (mpi-vert-driver.cpp)
    assert np.load(tmp_path / f"cb{world - 1}.npy")[-1, -1] == full[-1, -1]


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _check_local(torch, n1, n2, P, scheme, shape, seed):
    rng = np.random.default_rng(seed)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    lb = nw_bands.LocalColBands(n1, n2, P, substrips=shape[0], strip_waves=shape[1])
    try:
        score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda(), scheme)
        full = oracle.fill(s1, s2, scheme)
        assert score == full[-1, -1]
        for r, (sf, sc, st, ncols) in enumerate(lb.layout):
            got = lb.tables[r][:n2 + 1, :ncols].cpu().numpy()
            np.testing.assert_array_equal(got, full[:, st:st + ncols], err_msg=f"band {r}")
    finally:
        lb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,P,shape", [(1000, 300, 2, (1, 1)), (64 * 37 + 5, 999, 5, (1, 2)),
                                           (3000, 130, 3, (2, 2)), (4096 + 7, 64, 4, (4, 1)),
                                           (2500, 1777, 2, (1, 4)), (1100, 5, 4, (2, 1)),
                                           (9000, 2000, 8, (0, 0))])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1), (2, -1, -2)])
def test_local_colbands_vs_oracle(torch_gpu, n1, n2, P, shape, scheme):
    _check_local(torch_gpu, n1, n2, P, scheme, shape, n1 * 7 + n2 + P)


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,P", [(2000, 300, 2), (3000, 777, 3), (8191, 130, 4), (1100, 1500, 4)])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1)])
@pytest.mark.parametrize("panel", [(0, 0), (4, 1), (1, 4)])
def test_local_colbands_panels_vs_oracle(torch_gpu, n1, n2, P, scheme, panel):
    """Column bands with the row-scan panel kernel: a band's first panel takes the
    left band's last column from feed_in (its feeder-in wave), the band's last panel
    publishes into feed_out (its feeder-out wave)."""
    torch = torch_gpu
    rng = np.random.default_rng(n1 + 7 * n2 + P)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    lb = nw_bands.LocalColBands(n1, n2, P, substrips=panel[0], strip_waves=panel[1], kernel=nwhip.KERNEL_PANELS)
    try:
        score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda(), scheme)
        full = oracle.fill(s1, s2, scheme)
        assert score == full[-1, -1]
        for r, (sf, sc, start, ncols) in enumerate(lb.layout):
            got = lb.tables[r][:n2 + 1, :ncols].cpu().numpy()
            np.testing.assert_array_equal(got, full[:, start:start + ncols], err_msg=f"band {r}")
    finally:
        lb.close()


@pytest.mark.gpu
def test_local_colbands_repeated_launches(torch_gpu):
    """Tags advance per launch; stale feed granules of earlier launches are never taken."""
    torch = torch_gpu
    n1, n2, P = 3000, 1500, 3
    lb = nw_bands.LocalColBands(n1, n2, P, substrips=2, strip_waves=2)
    try:
        for seed in range(4):
            rng = np.random.default_rng(seed)
            s1 = rng.integers(1, 5, n1).astype(np.int8)
            s2 = rng.integers(1, 5, n2).astype(np.int8)
            score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda())
            full = oracle.fill(s1, s2)
            assert score == full[-1, -1]
            for r, (sf, sc, st, ncols) in enumerate(lb.layout):
                np.testing.assert_array_equal(lb.tables[r][:n2 + 1, :ncols].cpu().numpy(),
                                              full[:, st:st + ncols])
    finally:
        lb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [nwhip.KERNEL_STRIPS, nwhip.KERNEL_PANELS])
def test_colband_then_whole_fill_on_one_context(torch_gpu, kernel):
    """A column band r > 0 (global strips strip0 .. of the table's sweep, tags
    tagbase + p + 1 with p the GLOBAL strip) followed by whole-table fills on the
    SAME context: the whole fill must never take a granule the band left behind
    (tagbase moves past strip0 + nstrips; nw_capi.cpp launch_fill)."""
    torch = torch_gpu
    n1, n2, P = 6000, 700, 3
    rng = np.random.default_rng(77)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    full = oracle.fill(s1, s2)
    sh = (1, 1) if kernel == nwhip.KERNEL_STRIPS else (4, 1)
    lay = [nwhip.colband_layout(n1, n2, P, r, sh[0], sh[1], kernel=kernel) for r in range(P)]
    ctx, ctx0 = nwhip.Context(0), nwhip.Context(0)
    feeds = [nwhip.Feed(n2, 0) for _ in range(P - 1)]
    try:
        for it in range(2):
            tabs = [nwhip.Context.alloc_table(ncols - 1, n2) for (_, _, _, ncols) in lay]
            # band 0 on its own context, bands 1 .. on the shared one, in order
            for r in range(P):
                (ctx0 if r == 0 else ctx).fill_colband(
                    d1, d2, tabs[r], P, r, feed_in=feeds[r - 1].ptr if r else None,
                    feed_out=feeds[r].ptr if r + 1 < P else None, tag=it + 1,
                    substrips=sh[0], strip_waves=sh[1], kernel=kernel)
                torch.cuda.synchronize()
            for r, (_, _, st, ncols) in enumerate(lay):
                np.testing.assert_array_equal(tabs[r][:n2 + 1, :ncols].cpu().numpy(), full[:, st:st + ncols])
            tab = nwhip.Context.alloc_table(n1, n2)
            res = ctx.fill(d1, d2, tab, substrips=sh[0], strip_waves=sh[1], kernel=kernel)
            assert res.status == 0
            np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), full, err_msg=f"iteration {it}")
    finally:
        for f in feeds:
            f.free()
        ctx.close()
        ctx0.close()


@pytest.mark.gpu
def test_local_colbands_32k_score(torch_gpu):
    """BASELINE config-2 inputs split into 4 concurrent column bands on one GPU."""
    torch = torch_gpu
    n = 32768
    s1, s2 = nwhip.synth(1, n), nwhip.synth(2, n)
    lb = nw_bands.LocalColBands(n, n, 4)
    try:
        assert lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()) == 13394
        sc, lr, lc, rs, rw = oracle.score(s1, s2, want_rows=True)
        np.testing.assert_array_equal(lb.tables[-1][:n + 1, lb.layout[-1][3] - 1].cpu().numpy(), lc)
    finally:
        lb.close()


@pytest.mark.gpu
def test_colband_refusals(torch_gpu):
    torch = torch_gpu
    ctx = nwhip.Context(0)
    try:
        n1, n2 = 1000, 100
        d1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        d2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
        sf, sc, st, ncols = nwhip.colband_layout(n1, n2, 2, 1, 1, 1)
        tab = nwhip.Context.alloc_table(ncols - 1, n2)
        feed = nwhip.Feed(n2, 0)
        cases = [dict(r=1, feed_in=None),                      # band r > 0 needs its feed
                 dict(r=0, feed_in=feed.ptr),                  # the first band has none
                 dict(r=1, feed_in=feed.ptr, tag=0),           # tags are > 0
                 dict(r=1, feed_in=feed.ptr + 4)]              # misaligned granules
        for kw in cases:
            kw.setdefault("tag", 1)
            with pytest.raises(nwhip.NwError) as e:
                ctx.fill_colband(d1, d2, tab, 2, substrips=1, strip_waves=1, **kw)
            assert e.value.status == nwhip.NW_ERR_ARG, kw
        with pytest.raises(nwhip.NwError) as e:  # local alignment: single tables only
            p = nwhip.params((1, -1, -1), substrips=1, strip_waves=1, mode=nwhip.MODE_SW)
            b = nwhip.NwColBand(None, None, 1, 1, 0, 0)
            import ctypes
            st = nwhip.lib().nw_fill_colband_async(ctx._h, ctypes.c_void_p(d1.data_ptr()), n1,
                                                   ctypes.c_void_p(d2.data_ptr()), n2, ctypes.byref(p),
                                                   ctypes.byref(b), ctypes.c_void_p(tab.data_ptr()),
                                                   tab.shape[1], None)
            if st != nwhip.NW_OK:
                raise nwhip.NwError(st)
        assert e.value.status == nwhip.NW_ERR_UNSUPPORTED
        feed.free()
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [1, 2])
def test_two_process_colbands_shared_gpu(torch_gpu, kernel):
    """The bench's column-band path as `value` end to end on one GPU: 2 ranks,
    IPC-mapped feed buffers by launch parity, in-kernel feed stores."""
    width, n2 = 1500, 1300
    env = dict(os.environ, PYTHONPATH=PKG)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--share-gpu", "--partition", "cols", "--alt-partition", "none", "--col-width", str(width),
           "--col-rows", str(n2), "--kernel", str(kernel), "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    n1 = 2 * width
    want = oracle.score(nwhip.synth(1, n1), nwhip.synth(2, n2))
    assert res["score"] == want and res["n_gpus"] == 2 and res["config"]["n1"] == n1


# ------------------------------------------------------------------ shape model (CPU)
def test_colband_shape_model():
    """The modelled critical path picks the fast-pace shape for a short strip chain and the
    short-hop shape for a long one (DESIGN.md 'Multi-GPU'); an explicit shape is kept."""
    n2 = 524288
    assert nw_bands.colband_shape(65536, n2) == (1, 4)
    assert nw_bands.colband_shape(8 * 65536, n2) == (4, 1)
    assert nw_bands.colband_shape(8 * 65536, n2, 2, 2) == (2, 2)
    for shape in nw_bands.COLBAND_PACE_NS:
        c, nc = shape
        assert 64 * c * nc == 256  # one strip width: every band boundary is a strip boundary
        # monotone in the table width (more strips -> longer chain)
        assert nw_bands.colband_model_ms(65536, n2, shape) < nw_bands.colband_model_ms(131072, n2, shape)
