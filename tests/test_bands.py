"""Row bands (multi-GPU path, mpi-horz contract: src/mpi/mpi-horz.cpp:4-99,
mpi-horz-driver.cpp:31-32,88-90).

CPU (-m "not gpu"): the band layout of the C ABI against the oracle; the band /
halo contract over a real world_size-2 and -3 gloo process group (each rank fills
its band with the oracle, the halo row travels rank to rank as the GPU path's
halo granules do), checked against the whole-table oracle.
GPU (-m gpu): LocalBands -- several bands concurrently on one device through the
in-kernel halo hand-off -- bit-exact against the oracle's bands; and the
multi-process bench path (2 ranks sharing the one GPU: IPC halo buffers, gloo
control plane) checked against the oracle's score.
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


# ------------------------------------------------------------------ layout (CPU)
@pytest.mark.parametrize("n2,P", [(0, 1), (7, 8), (10, 2), (63, 4), (100, 3), (1000, 7),
                                  (524288, 8), (262144, 4), (131072, 2), (65535, 8)])
def test_band_layout_matches_oracle(n2, P):
    for r in range(P):
        assert nwhip.band_layout(n2, P, r) == oracle.band_layout(n2, P, r)


@pytest.mark.parametrize("n2,P", [(10, 2), (100, 3), (1000, 7), (524288, 8), (17, 8)])
def test_bands_tile_the_rows(n2, P):
    """Band r>0 starts on band r-1's last row (the halo); the last band ends on row n2."""
    lay = nw_bands.plan(n2, P)
    assert lay[0][1] == 0
    for (rows_a, st_a), (rows_b, st_b) in zip(lay, lay[1:]):
        assert st_b == st_a + rows_a - 1
    rows, st = lay[-1]
    assert st + rows - 1 == n2


# ------------------------------------------------------------------ gloo ranks (CPU)
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n1, n2, scheme, outdir):
    import torch.distributed as dist
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))  # fail, never hang
    s1, s2 = oracle.synth(11, n1), oracle.synth(12, n2)
    rows, start = nwhip.band_layout(n2, world, rank)
    halo = None
    if rank > 0:  # halo row = rank-1's last row (mpi-horz.cpp:28-40)
        h = torch.empty(n1 + 1, dtype=torch.int32)
        dist.recv(h, src=rank - 1)
        halo = h.numpy()
    band = oracle.fill_band(s1, s2, world, rank, halo, scheme)
    assert band.shape == (rows, n1 + 1)
    if rank + 1 < world:
        dist.send(torch.from_numpy(band[-1].copy()), dst=rank + 1)
    np.save(os.path.join(outdir, f"band{rank}.npy"), band)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.timeout(240)
def test_gloo_bands_reassemble_the_table(tmp_path, world):
    import torch.multiprocessing as mp
    n1, n2, scheme = 301, 257, (1, -1, -1)
    mp.spawn(_rank_main, args=(world, _free_port(), n1, n2, scheme, str(tmp_path)),
             nprocs=world, join=True)
    full = oracle.fill(oracle.synth(11, n1), oracle.synth(12, n2), scheme)
    for r in range(world):
        rows, start = nwhip.band_layout(n2, world, r)
        band = np.load(tmp_path / f"band{r}.npy")
        np.testing.assert_array_equal(band, full[start:start + rows])
    # final score on the last rank's last cell (mpi-horz-driver.cpp:88-90)
    assert np.load(tmp_path / f"band{world - 1}.npy")[-1, -1] == full[-1, -1]


# Synthetic per-rank (start, end) stamps of 3 fills, in ns: rank r starts late by
# 100 r us, the last rank ends last; fill 2 has a rank that ends first but started
# earliest -- the latency is still max end - min start over the ranks
_STAMPS = {
    0: [(1_000_000, 51_000_000), (100_000_000, 140_000_000), (200_000_000, 230_000_000)],
    1: [(1_100_000, 52_500_000), (100_200_000, 141_000_000), (199_000_000, 228_000_000)],
    2: [(1_200_000, 53_000_000), (100_100_000, 150_500_000), (200_300_000, 261_000_000)],
}


def _expected(world):
    st = [_STAMPS[r] for r in range(world)]
    return [(max(s[k][1] for s in st) - min(s[k][0] for s in st)) / 1e6 for k in range(3)]


def test_fill_latencies_min_start_max_end():
    """The per-fill latency of mpi-horz-driver.cpp:38-83: earliest start -> latest end."""
    got = nw_bands.fill_latencies([_STAMPS[r] for r in range(3)])
    assert got["ms"] == pytest.approx([52.0, 50.5, 62.0])
    assert got["start_skew_ms"] == pytest.approx([0.2, 0.2, 1.3])
    with pytest.raises(ValueError):
        nw_bands.fill_latencies([_STAMPS[0], _STAMPS[1][:2]])
    with pytest.raises(ValueError):
        nw_bands.fill_latencies([[(5, 4)]])


def _gather_main(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    got = nw_bands.gather_fill_latencies(_STAMPS[rank], world)
    with open(os.path.join(outdir, f"fills{rank}.json"), "w") as f:
        json.dump(got, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.timeout(240)
def test_gloo_gather_fill_latencies(tmp_path, world):
    """The cross-rank gather of the bench's N>1 timing over a real gloo world: every
    rank gets the same per-fill latencies, min start -> max end over ALL ranks."""
    import torch.multiprocessing as mp
    mp.spawn(_gather_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = _expected(world)
    for r in range(world):
        got = json.load(open(tmp_path / f"fills{r}.json"))
        assert got["ms"] == pytest.approx(want)


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,P", [(300, 200, 2), (1000, 777, 3), (640, 130, 4), (129, 7, 8),
                                     (64 * 37 + 5, 999, 5)])
@pytest.mark.parametrize("scheme", [(1, 0, -1), (1, -1, -1), (2, -1, -2)])
@pytest.mark.parametrize("kernel", [1, 2])
def test_local_bands_vs_oracle(torch_gpu, n1, n2, P, scheme, kernel):
    """Both kernel families: strips (1) and row-scan panels (2) take the halo row
    from halo_in granules and publish their last row into halo_out."""
    torch = torch_gpu
    rng = np.random.default_rng(n1 * 31 + n2 + P)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    lb = nw_bands.LocalBands(n1, n2, P, kernel=kernel)
    try:
        score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda(), scheme)
        full = oracle.fill(s1, s2, scheme)
        assert score == full[-1, -1]
        for r, (rows, start) in enumerate(lb.layout):
            got = lb.tables[r][:rows, :n1 + 1].cpu().numpy()
            np.testing.assert_array_equal(got, full[start:start + rows], err_msg=f"band {r}")
    finally:
        lb.close()


@pytest.mark.gpu
def test_local_bands_repeated_launches(torch_gpu):
    """Tags advance per launch; stale halo granules of earlier launches are never taken."""
    torch = torch_gpu
    n1, n2, P = 2000, 1500, 3
    lb = nw_bands.LocalBands(n1, n2, P)
    try:
        for seed in range(4):
            rng = np.random.default_rng(seed)
            s1 = rng.integers(1, 5, n1).astype(np.int8)
            s2 = rng.integers(1, 5, n2).astype(np.int8)
            score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda())
            full = oracle.fill(s1, s2)
            assert score == full[-1, -1]
            for r, (rows, start) in enumerate(lb.layout):
                np.testing.assert_array_equal(lb.tables[r][:rows, :n1 + 1].cpu().numpy(),
                                              full[start:start + rows])
    finally:
        lb.close()


@pytest.mark.gpu
def test_local_bands_32k_score(torch_gpu):
    """BASELINE config-2 inputs split into 4 concurrent bands on one GPU."""
    torch = torch_gpu
    n = 32768
    s1, s2 = nwhip.synth(1, n), nwhip.synth(2, n)
    lb = nw_bands.LocalBands(n, n, 4)
    try:
        score = lb.fill(torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda())
        assert score == 13394  # reference serial.cpp on the same inputs (synth_scores.json)
        sc, lr, lc, rs, rw = oracle.score(s1, s2, want_rows=True)
        rows, start = lb.layout[-1]
        np.testing.assert_array_equal(lb.tables[-1][rows - 1, :n + 1].cpu().numpy(), lr)
    finally:
        lb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,blocks,sweep", [(1, 1, "horizontal"), (1, 1, "vertical"), (2, 1, "vertical"),
                                                 (1, 4, "horizontal")])
def test_two_process_bands_shared_gpu(torch_gpu, kernel, blocks, sweep):
    """The bench's multi-process path end to end on one GPU: 2 ranks (torch.distributed.run,
    gloo control plane), IPC-mapped halo / feed buffers alternating by launch parity,
    link-word flow control between back-to-back launches, in-kernel halo stores; the
    row-band leg (`value`: contiguous, or block-cyclic with 4 blocks per rank, where
    the last rank also feeds rank 0) and the alternate legs (`alt_partitions`: the
    contiguous rows, the column bands) all against the oracle, both kernel families."""
    n1, rows = 4096 + 17, 704
    width, crows = 1500, 1300
    env = dict(os.environ, PYTHONPATH=PKG)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--share-gpu", "--partition", "rows", "--band-rows", str(rows), "--band-blocks", str(blocks),
           "--band-cols", str(n1), "--col-width", str(width), "--col-rows", str(crows),
           "--kernel", str(kernel), "--band-sweep", sweep, "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    n2 = 2 * rows
    want = oracle.score(nwhip.synth(1, n1), nwhip.synth(2, n2))
    assert res["score"] == want and res["n_gpus"] == 2 and res["config"]["n2"] == n2
    alts = res["alt_partitions"]
    # the per-fill latency is `value` (mpi-horz-driver.cpp:38-83); the back-to-back
    # throughput is reported beside it, in every leg
    for leg in [res] + list(alts.values()):
        assert len(leg["per_fill_ms"]) == 3 and leg["pipelined_ms_per_fill"] > 0
        assert leg["ms_per_step"] == pytest.approx(float(np.mean(leg["per_fill_ms"])), abs=2e-3)
    assert res["config"].get("blocks_per_gpu", 1) == blocks
    if blocks > 1 or (sweep == "horizontal" and kernel == 1):
        assert alts["rows_contiguous"]["score"] == want and res["rows_legs_agree"]
    if kernel == 1:  # the horizontal sweep of the same bands: main leg or alternate
        hz = res if (sweep == "horizontal" and blocks == 1) else alts["rows_horizontal"]
        assert hz["score"] == want and "horizontal strips" in hz["config"]["parallelism"]
    assert alts["cols"]["score"] == oracle.score(nwhip.synth(1, 2 * width), nwhip.synth(2, crows))
    assert alts["cols"]["config"]["n1"] == 2 * width


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,withhold,extra", [
    (2, 0, ["--band-sweep", "vertical"]), (2, 0, ["--band-sweep", "horizontal"]),
    (3, 1, ["--band-sweep", "vertical"]), (2, 0, ["--partition", "cols"])])
def test_withheld_producer_fails_fast(torch_gpu, nproc, withhold, extra):
    """the driver's multi-GPU run must fail fast.  A producer that never
    publishes its boundary (--debug-withhold-rank) makes its consumer's warmup wait
    give up after --warmup-timeout-ms; every rank then exits non-zero within seconds,
    naming the band, the watchdog site and the control words, and no JSON line is
    printed.  (The pre-flight peer-store ping passes: the buffers are mapped.)"""
    import time
    env = dict(os.environ, PYTHONPATH=PKG)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "3", "--warmup", "2",
           "--share-gpu", "--band-rows", "704", "--band-cols", "4113", "--col-width", "1500", "--col-rows", "1300",
           "--alt-partition", "none", "--no-cpu-baseline", "--warmup-timeout-ms", "2000",
           "--debug-withhold-rank", str(withhold)] + extra
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    dt = time.time() - t0
    assert out.returncode != 0
    assert dt < 60, f"took {dt:.0f} s"
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert f"band {withhold + 1}: " in out.stderr and "warmup" in out.stderr, out.stderr[-3000:]


@pytest.mark.parametrize("kw,want", [
    ({}, ["rows_horizontal", "rows_contiguous", "rows_cyclic", "cols"]),
    ({"band_sweep": "horizontal"}, ["rows_horizontal", "rows_contiguous", "rows_cyclic", "cols"]),
    ({"band_sweep": "vertical"}, ["rows_contiguous", "rows_horizontal", "rows_cyclic", "cols"]),
    ({"band_blocks": 4}, ["rows_cyclic", "rows_horizontal", "rows_contiguous", "cols"]),
    ({"kernel": 2}, ["rows_contiguous", "cols"]),
    ({"partition": "cols"}, ["cols", "rows_horizontal"]),
    ({"alt_partition": "none"}, ["rows_horizontal"]),
    ({"band_rows": 704}, ["rows_horizontal", "rows_contiguous", "cols"]),
    ({"band_rows": 704, "band_sweep": "vertical"}, ["rows_contiguous", "rows_horizontal", "cols"]),
])
def test_bench_legs(kw, want):
    """bench.py --gpus N: the row-band leg that is `value` (config 4: contiguous mpi-horz bands,
    horizontal strips unless --band-sweep vertical, the panel kernel or --band-blocks m > 1) and
    the alternates."""
    import argparse
    a = dict(partition="rows", kernel=0, band_blocks=1, band_sweep="auto", alt_partition=None,
             band_rows=65536)
    a.update(kw)
    assert [name for name, _, _ in nw_bands.legs_for(argparse.Namespace(**a))] == want


def test_launch_schedule_never_rewrites_an_unread_buffer():
    """The back-to-back launch schedule of nw_bands._sweep, simulated: launch k uses
    buffer k % 2; the producer's launch k waits for the consumer's "done with k - 2"
    signal.  Under every interleaving the simulation explores, a buffer is never
    rewritten before the consumer launch that reads it has finished."""
    import itertools
    rng = np.random.default_rng(0)
    K = 12
    for _ in range(200):
        done_c = 0          # consumer launches finished
        started_p = 0       # producer launches started
        written = {}        # buffer -> producer launch that last wrote it
        read_ok = True
        for step in itertools.count():
            if done_c >= K:
                break
            # the producer may start launch k+1 if the link word allows it
            k = started_p + 1
            can_p = k <= K and (k < 3 or done_c >= k - 2)
            # the consumer may finish launch done_c+1 once the producer wrote it
            can_c = done_c + 1 <= started_p
            if can_p and (not can_c or rng.random() < 0.5):
                b = k % 2
                prev = written.get(b)
                if prev is not None and prev > done_c:  # rewriting a buffer not yet consumed
                    read_ok = False
                written[b] = k
                started_p = k
            elif can_c:
                kk = done_c + 1
                read_ok &= written.get(kk % 2) == kk  # reads exactly launch kk's data
                done_c = kk
            assert step < 10 * K
        assert read_ok
