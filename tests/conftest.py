"""Shared test setup.

Markers: `gpu` = needs a real MI355X (run with -m gpu on the GPU box);
everything else runs on CPU (-m "not gpu").
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fast-needleman-wunsch_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "oracle"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running (large tables)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def bdna_path(name: str) -> str:
    return os.path.join(GOLDEN, "bdna", name)


def read_bdna(name: str):
    import numpy as np
    with open(bdna_path(name), "rb") as f:
        return np.frombuffer(f.read(), dtype=np.int8).copy()


@pytest.fixture(scope="session")
def pair(golden):
    """pair(name) -> (s1, s2) int8 arrays (argv1 across the top, argv2 down the side)."""
    cache = {}

    def get(name):
        if name not in cache:
            e = golden["pairs"][name]
            cache[name] = (read_bdna(e["argv1"]), read_bdna(e["argv2"]))
        return cache[name]
    return get


def big_rows(n1: int, n2: int, scheme):
    """Row-level golden vectors of a full-size synthetic workload
    (tests/golden/make_big_rows.py): dict with score, last_row, last_col,
    row_sum, row_wsum -- decoded from the delta-encoded npz."""
    import numpy as np
    name = {(1, 0, -1): "shipped", (1, -1, -1): "mm1"}[tuple(scheme)]
    z = np.load(os.path.join(GOLDEN, f"big_rows_{n1}x{n2}_{name}.npz"))
    out = {"score": int(z["score"])}
    with np.errstate(over="ignore"):
        for k in ("last_row", "last_col", "row_sum", "row_wsum"):
            d = z[k]
            out[k] = np.cumsum(d, dtype=d.dtype)
    return out


def big_full_rows(n1: int, n2: int, scheme):
    """Exact whole rows of a full-size synthetic workload (make_big_rows.py
    FULL_JOBS): (row indices, (k, n1+1) int32 rows), or None without a fixture."""
    import numpy as np
    name = {(1, 0, -1): "shipped", (1, -1, -1): "mm1"}[tuple(scheme)]
    path = os.path.join(GOLDEN, f"big_fullrows_{n1}x{n2}_{name}.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)
    t = np.concatenate([z["first"][:, None].astype(np.int32), z["d"].astype(np.int32)], axis=1)
    return z["rows"], np.cumsum(t, axis=1, dtype=np.int32)
