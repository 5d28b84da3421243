"""Block-cyclic row bands (nw_fill_band_cycle_async, nw_bands.LocalCycleBands).

The multi-GPU row-band partition with the rows dealt to the ranks in blocks:
global block g = k * P + r is rank r's block k, its row 0 the previous block's
last row (the mpi-horz contract, src/mpi/mpi-horz.cpp:16-40, per block).  Every
block's table is checked against the oracle (small tables) or against the
committed 524288-column golden rows (config 4's width), through the same
kernels and halo protocol as the multi-GPU run, with P ranks sharing one GPU.
P = 1 runs a rank's blocks as ONE launch (the multi-block kernel path, chained
through its own halo buffer); P > 1 runs one launch per block in global block
order (nw_bands.LocalCycleBands: one process cannot keep P launches that wait on
each other co-resident); one process per rank is bench.py --share-gpu.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import nw_bands  # noqa: E402
import nwhip  # noqa: E402
import oracle  # noqa: E402  (checker only)

SCHEMES = [(1, 0, -1), (1, -1, -1), (2, -1, -2)]


def test_cycle_layout():
    assert nw_bands.cycle_layout(24, 3, 2) == 4
    with pytest.raises(ValueError):
        nw_bands.cycle_layout(25, 3, 2)
    s2 = np.arange(24, dtype=np.int8)
    # rank 1 of 3, blocks g = 1, 4 of 4 rows: s2[4:8] and s2[16:20]
    np.testing.assert_array_equal(nw_bands.cycle_side_chars(s2, 4, 3, 2, 1),
                                  np.r_[np.arange(4, 8), np.arange(16, 20)].astype(np.int8))


# ------------------------------------------------------------------ gloo ranks (CPU)
def _block_rows(s1, s2_blk, top, row0, scheme):
    """Rows row0 .. row0 + h of the table given row row0 (`top`): the serial
    recurrence (serial.cpp:21-33), each row as a running maximum in the w form
    w = t - GAP * j (numpy restatement for the contract test)."""
    match, mismatch, gap = scheme
    h, n1 = s2_blk.size, s1.size
    t = np.empty((h + 1, n1 + 1), np.int64)
    t[0] = top
    j = np.arange(n1 + 1, dtype=np.int64)
    for i in range(1, h + 1):
        sub = np.where(s1 == s2_blk[i - 1], match, mismatch)
        c = np.empty(n1 + 1, np.int64)
        c[0] = (row0 + i) * gap
        c[1:] = np.maximum(t[i - 1, :-1] + sub, t[i - 1, 1:] + gap)
        t[i] = np.maximum.accumulate(c - gap * j) + gap * j
    return t.astype(np.int32)


def _cycle_rank_main(rank, world, port, n1, m, h, scheme, outdir):
    import datetime
    import torch.distributed as dist
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    s1, s2 = oracle.synth(11, n1), oracle.synth(12, world * m * h)
    for k in range(m):
        g = k * world + rank
        if g == 0:
            top = np.arange(n1 + 1, dtype=np.int64) * scheme[2]  # serial.cpp:16
        else:  # the previous block's last row, from rank g-1 mod world (mpi-horz.cpp:28-40 per block)
            buf = torch.empty(n1 + 1, dtype=torch.int32)
            dist.recv(buf, src=(rank - 1) % world)
            top = buf.numpy()
        blk = _block_rows(s1, s2[g * h:(g + 1) * h], top, g * h, scheme)
        if g + 1 < world * m:
            dist.send(torch.from_numpy(blk[-1].copy()), dst=(rank + 1) % world)
        np.save(os.path.join(outdir, f"block{g}.npy"), blk)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.timeout(240)
def test_gloo_cycles_reassemble_the_table(tmp_path, world):
    """The block-cyclic contract over a real gloo world: rank r fills blocks
    g = k * world + r from the halo row rank g-1 sends (the last rank feeding rank
    0's next block); the blocks tile the serial table."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    n1, m, h, scheme = 301, 3, 9, (1, -1, -1)
    mp.spawn(_cycle_rank_main, args=(world, port, n1, m, h, scheme, str(tmp_path)), nprocs=world, join=True)
    n2 = world * m * h
    full = oracle.fill(oracle.synth(11, n1), oracle.synth(12, n2), scheme)
    for g in range(world * m):
        np.testing.assert_array_equal(np.load(tmp_path / f"block{g}.npy"), full[g * h:(g + 1) * h + 1])


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    return _t


def check_blocks(lb, want):
    for g in range(lb.P * lb.m):
        tab, row0 = lb.block(g)
        got = tab[:lb.h + 1, :lb.n1 + 1].cpu().numpy()
        np.testing.assert_array_equal(got, want[row0:row0 + lb.h + 1], err_msg=f"block {g}")


@pytest.mark.gpu
@pytest.mark.parametrize("P,m", [(1, 3), (1, 16), (2, 2), (3, 2), (8, 2)])
@pytest.mark.parametrize("n1,h", [(300, 7), (1000, 64), (1537, 100)])
@pytest.mark.parametrize("shape", [(2, 2), (4, 1), (1, 4)])
def test_cycles_vs_oracle(torch, P, m, n1, h, shape):
    rng = np.random.default_rng(P * 1000 + m * 100 + n1 + h)
    n2 = P * m * h
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    lb = nw_bands.LocalCycleBands(n1, n2, P, m, substrips=shape[0], strip_waves=shape[1])
    try:
        d1 = torch.from_numpy(s1).cuda()
        for scheme in SCHEMES:
            want = oracle.fill(s1, s2, scheme)
            assert lb.fill(d1, s2, scheme) == want[-1, -1]
            check_blocks(lb, want)
    finally:
        lb.close()


@pytest.mark.gpu
def test_cycles_repeat_and_refusals(torch):
    """Back-to-back launches on the same buffers (new tag each), and the panel
    kernel refused for block cycles."""
    rng = np.random.default_rng(5)
    n1, P, m, h = 777, 1, 9, 33
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, P * m * h).astype(np.int8)
    lb = nw_bands.LocalCycleBands(n1, P * m * h, P, m)
    try:
        d1 = torch.from_numpy(s1).cuda()
        want = oracle.fill(s1, s2, (1, -1, -1))
        for _ in range(4):
            assert lb.fill(d1, s2, (1, -1, -1)) == want[-1, -1]
        check_blocks(lb, want)
        with pytest.raises(nwhip.NwError) as e:
            lb.ctxs[0].fill_band_cycle(d1, torch.from_numpy(s2[:m * h].copy()).cuda(), h, lb.tables[0],
                                       halo_in=lb.halos[0].ptr, halo_out=lb.halos[0].ptr, tag=99,
                                       kernel=nwhip.KERNEL_PANELS)
        assert e.value.status == nwhip.NW_ERR_UNSUPPORTED
        torch.cuda.synchronize()
    finally:
        lb.close()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("P,m", [(1, 24), (8, 3)])
def test_config4_width_cycles(torch, P, m):
    """Config 4's width (524288 columns) as block-cyclic row bands: the first
    32761 rows of the 524288 x 32767 golden table (rows depend only on the rows
    above), every row's checksums, the last column and the golden full rows."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_full_size import big_rows, check_full_rows, row_checksums
    n1, n2 = 524288, 32760
    g = big_rows(n1, 32767, (1, 0, -1))
    torch.cuda.empty_cache()
    lb = nw_bands.LocalCycleBands(n1, n2, P, m)
    try:
        lb.fill(torch.from_numpy(nwhip.synth(1, n1)).cuda(), nwhip.synth(2, 32767)[:n2].copy())
        for blk in range(P * m):
            tab, row0 = lb.block(blk)
            rows = lb.h + 1
            rs, rw = row_checksums(torch, tab, rows, n1 + 1)
            np.testing.assert_array_equal(rs, g["row_sum"][row0:row0 + rows], err_msg=f"block {blk}")
            np.testing.assert_array_equal(rw, g["row_wsum"][row0:row0 + rows], err_msg=f"block {blk}")
            np.testing.assert_array_equal(tab[:rows, n1].cpu().numpy(), g["last_col"][row0:row0 + rows])
            check_full_rows(torch, tab, n1, 32767, (1, 0, -1), row0=row0, nrows=rows)
    finally:
        lb.close()
        del lb
        torch.cuda.empty_cache()
