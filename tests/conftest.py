"""Shared test setup.

Markers: `gpu` = needs a real MI355X (run with -m gpu on the GPU box);
everything else runs on CPU (-m "not gpu").
"""
import json
import os
import sys

import pytest

# The idxarray-mt fills (the reference's own, and the oracle's restatement) spin on
# per-row progress counters (src/idxarray/idxarray-mt.cpp:50-56) without yielding:
# with more OpenMP threads than free cores a descheduled producer stalls every
# spinner behind it for whole time slices.  Keep the default team at half the
# host's CPUs (set before libgomp first loads, i.e. before any oracle call).
os.environ.setdefault("OMP_NUM_THREADS", str(max(1, min(4, (os.cpu_count() or 2) // 2))))

# Default time bound of every test (pytest-timeout, thread method: it also ends a
# test stuck inside a C call -- an OpenMP spin, a GPU wait -- and names it).
# Tests marked `slow` (full-size tables) get the longer bound.
DEFAULT_TIMEOUT_S, SLOW_TIMEOUT_S = 600, 1500

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fast-needleman-wunsch_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "oracle"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running (large tables)")


def pytest_collection_modifyitems(config, items):
    """Every test without its own timeout marker gets the default bound (unless the
    command line already sets --timeout)."""
    if config.pluginmanager.hasplugin("timeout") and not config.getoption("timeout", None):
        for item in items:
            if item.get_closest_marker("timeout") is None:
                t = SLOW_TIMEOUT_S if item.get_closest_marker("slow") is not None else DEFAULT_TIMEOUT_S
                item.add_marker(pytest.mark.timeout(t, method="thread"))


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


def config4_golden():
    """BASELINE config 4's per-rank vectors (tests/golden/make_config4.py): dict with
    score, rows (global row indices) and full (their whole rows, int32), last_col,
    and for the bands in cs_bands their rows' row_sum / row_wsum (dict band -> array);
    None without the fixture."""
    import numpy as np
    path = os.path.join(GOLDEN, "config4_524288_shipped.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)
    t = np.concatenate([z["first"][:, None].astype(np.int32), z["d"].astype(np.int32)], axis=1)
    out = {"score": int(z["score"]), "rows": z["rows"], "full": np.cumsum(t, axis=1, dtype=np.int32),
           "cs_bands": [int(b) for b in z["cs_bands"]], "row_sum": {}, "row_wsum": {}}
    with np.errstate(over="ignore"):
        d = z["last_col"]
        out["last_col"] = np.cumsum(d, dtype=d.dtype)
        for b in out["cs_bands"]:
            for k in ("row_sum", "row_wsum"):
                d = z[f"{k}_{b}"]
                out[k][b] = np.cumsum(d, dtype=d.dtype)
    return out
