#!/usr/bin/env python3
"""Row-level golden vectors for the full-size synthetic workloads (BASELINE configs
3 and 4), too large for any host table here.

For each (n1, n2, scheme) the pinned linear-memory oracle (oracle/nw_oracle.c
nw_oracle_score, restating src/serial/serial.cpp:21-33; pinned to the reference
binaries on every fixture pair by tests/test_oracle.py) produces
  last_row  t[n2][0..n1]            (int32)
  last_col  t[0..n2][n1]            (int32)
  row_sum   sum_j t[i][j]           (per row, mod 2^64)
  row_wsum  sum_j (j+1) * t[i][j]   (per row, mod 2^64)
with s1 = synth(seed 1, n1), s2 = synth(seed 2, n2).  Stored
delta-encoded (np.diff, wrapping) in tests/golden/big_rows_<n1>x<n2>_<scheme>.npz;
tests/conftest.py big_rows() decodes them.

Exact cells: for the FULL_JOBS below, ~32 whole rows (nw_oracle_rows) -- rows 1,
63, 64, 65, 255, 256, n2, the band boundaries of the 8-band split where the
geometry is config 4's, and seeded random rows -- each stored as its column 0
plus int8 differences along the row, in big_fullrows_<n1>x<n2>_<scheme>.npz
(tests/conftest.py big_full_rows() decodes them).

  config 3 : 262144 x 262144 (and the 65536 / 131072 steps below it)
  config 4 : 524288 columns x 32767 rows -- the row-band geometry of the 8-GPU
             case (524288 columns, 8 bands of 4096 rows; mpi-horz-driver.cpp:31-32)
"""
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

NAMES = {(1, 0, -1): "shipped", (1, -1, -1): "mm1"}
JOBS = [(65536, 65536, (1, 0, -1)), (65536, 65536, (1, -1, -1)),
        (131072, 131072, (1, 0, -1)), (131072, 131072, (1, -1, -1)),
        (262144, 262144, (1, 0, -1)), (262144, 262144, (1, -1, -1)),
        (524288, 32767, (1, 0, -1))]

FULL_JOBS = [(65536, 65536, (1, 0, -1)), (262144, 262144, (1, 0, -1)), (262144, 262144, (1, -1, -1)),
             (524288, 32767, (1, 0, -1))]
FULL_ROWS = 32


def path(n1, n2, scheme):
    return os.path.join(HERE, f"big_rows_{n1}x{n2}_{NAMES[tuple(scheme)]}.npz")


def encode(a):
    a = np.asarray(a)
    with np.errstate(over="ignore"):
        return np.concatenate([a[:1], np.diff(a)])


def job(n1, n2, scheme):
    import oracle
    s1, s2 = oracle.synth(1, n1), oracle.synth(2, n2)
    t0 = time.time()
    sc, lr, lc, rs, rw = oracle.score(s1, s2, scheme, want_rows=True)
    np.savez_compressed(path(n1, n2, scheme), score=np.int64(sc), last_row=encode(lr),
                        last_col=encode(lc), row_sum=encode(rs), row_wsum=encode(rw))
    return n1, n2, scheme, sc, time.time() - t0


def full_path(n1, n2, scheme):
    return os.path.join(HERE, f"big_fullrows_{n1}x{n2}_{NAMES[tuple(scheme)]}.npz")


def pick_rows(n1, n2):
    """Rows 1, 63, 64, 65, 255, 256, n2; for config 4's geometry the boundaries of
    its 8 row bands (oracle band layout); then seeded random rows up to FULL_ROWS."""
    import oracle
    want = {r for r in (1, 63, 64, 65, 255, 256, n2) if r <= n2}
    if n1 == 524288:
        for b in range(1, 8):
            _, st = oracle.band_layout(n2, 8, b)
            want |= {st - 1, st, st + 1}
    rng = np.random.default_rng(n1 * 1000003 + n2)
    while len(want) < FULL_ROWS:
        want.add(int(rng.integers(0, n2 + 1)))
    return np.array(sorted(want), dtype=np.int64)


def full_job(n1, n2, scheme):
    import oracle
    t0 = time.time()
    rows = pick_rows(n1, n2)
    t = oracle.rows(oracle.synth(1, n1), oracle.synth(2, n2), scheme, rows)
    d = np.diff(t, axis=1)
    assert np.abs(d).max() < 128
    np.savez_compressed(full_path(n1, n2, scheme), rows=rows, first=t[:, 0].copy(), d=d.astype(np.int8))
    return n1, n2, scheme, rows.size, time.time() - t0


def main():
    todo = [(job, j) for j in JOBS if not os.path.exists(path(*j))]
    todo += [(full_job, j) for j in FULL_JOBS if not os.path.exists(full_path(*j))]
    with ProcessPoolExecutor(max_workers=min(5, max(1, len(todo)))) as ex:
        futs = [ex.submit(f, *j) for f, j in todo]
        for fu in futs:
            print(*fu.result()[:4], f"{fu.result()[4]:.0f}s", flush=True)


if __name__ == "__main__":
    main()
