"""CPU checks of the measurement tools the DESIGN's multi-GPU model rests on
(tools/n8_model.py): on a synthetic one-band timeline whose answer is known in
closed form, the N-band vertical pipeline model must reproduce it."""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_model(tmp_path, start, end, waves, n1=524288, n2=65536, bands="1,2,4,8", halo=3.0, wait=None):
    p = tmp_path / "trace.npz"
    extra = {} if wait is None else {"wait": np.asarray(wait, float)}
    np.savez(p, start=np.asarray(start, float), end=np.asarray(end, float), waves=waves, n1=n1, n2=n2,
             kernel_ms=float(max(end)) / 1e3, substrips=2, strip_waves=2, **extra)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "n8_model.py"), str(p), "--bands", bands,
                          "--halo-us", str(halo)], capture_output=True, text=True, check=True).stdout
    return {int(m.group(1)): float(m.group(2)) for m in re.finditer(r"bands (\d+): step ([0-9.]+) ms", out)}


def test_one_pass_chain(tmp_path):
    """S strips on S workers started together, strip k waiting k h for its left
    neighbour (recorded as `wait`) and working d: one band takes d + (S-1) h; band r's
    strip k waits for band r-1's strip k, so P bands take P d + (S-1) h + (P-1) halo."""
    S, d, h, halo = 64, 1000.0, 10.0, 3.0
    start = np.zeros(S)
    end = d + h * np.arange(S)
    t = run_model(tmp_path, start, end, waves=S, halo=halo, wait=h * np.arange(S))
    for P, ms in t.items():
        want = (P * d + (S - 1) * h + (P - 1) * halo) / 1e3
        assert abs(ms - want) < 0.01 + 1e-3 * want, (P, ms, want)


def test_one_pass_chain_without_waits_is_pessimistic(tmp_path):
    """The same timeline without the recorded waits: each band repeats the whole
    measured durations (the chain's waits counted again), P (d + (S-1) h) + (P-1) halo."""
    S, d, h, halo = 64, 1000.0, 10.0, 3.0
    start = np.zeros(S)
    end = d + h * np.arange(S)
    t = run_model(tmp_path, start, end, waves=S, halo=halo)
    for P, ms in t.items():
        want = (P * (d + (S - 1) * h) + (P - 1) * halo) / 1e3
        assert abs(ms - want) < 0.01 + 1e-3 * want, (P, ms, want)


def test_two_passes_share_workers(tmp_path):
    """2 S strips on S workers (two passes of duration d, no lag): one band 2 d; the
    band below starts pass k of strip k when the band above has finished it, so P
    bands take (P + 1) d + (P - 1) halo."""
    S, d, halo = 32, 500.0, 3.0
    start = np.concatenate([np.zeros(S), np.full(S, d)])
    end = start + d
    t = run_model(tmp_path, start, end, waves=S, halo=halo)
    for P, ms in t.items():
        want = ((P + 1) * d + (P - 1) * halo) / 1e3
        assert abs(ms - want) < 0.01 + 1e-3 * want, (P, ms, want)


def _n8_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("n8_model", os.path.join(ROOT, "tools", "n8_model.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_family_bounds_closed_form():
    """tools/n8_model.py --families on synthetic inputs: a horizontal
    family is D + (S-1) h with D = max(band bytes / store rate, n1 x its sweep pace), a
    vertical one max(7 tau + bytes / rate, (n1 / W - 1) h + 8 tau), and the bare hop
    is NC x 63 steps of skew + (NC-1) LDS hand-offs + one memory hand-off."""
    m = _n8_module()
    inp = {"clock_ghz": 2.0, "store_tbps": 6.0, "gran_rows": 16, "mem_handoff_us": 3.0, "lds_handoff_us": 0.5,
           "step_cycles": {"4,1": 100.0, "2,2": 60.0},
           "infill": {"4,1": {"hop_us": 10.0, "leader_ns_per_row": 50.0, "follower_ns_per_row": 40.0}},
           "panel_row_ns": {"bare": 100.0, "infill": 100.0}, "scan_step_ns_1wave": {"bare": 90.0, "infill": 90.0}}
    d_store = m.band_bytes() / 6.0e12 * 1e3
    bare = {f: t for f, _, t, _ in m.family_bounds(inp, "bare")}
    h41 = (63 * 50.0 + 16 * 50.0) * 1e-3 + 3.0          # step 50 ns
    assert abs(bare["H(4,1)"] - (max(d_store, 524288 * 50e-6) + 2047 * h41 * 1e-3)) < 1e-9
    h22 = (2 * 63 * 30.0 + (16 * 30.0) * 2) * 1e-3 + 0.5 + 3.0  # step 30 ns, one LDS hand-off
    assert abs(bare["H(2,2)"] - (d_store + 2047 * h22 * 1e-3)) < 1e-9
    tau = 65536 * 30.0 * 1e-6
    assert abs(bare["V(2,2)"] - max(7 * tau + d_store, 2047 * h22 * 1e-3 + 8 * tau)) < 1e-9
    fill = {f: t for f, _, t, _ in m.family_bounds(inp, "infill")}
    assert abs(fill["H(4,1)"] - (max(d_store, 524288 * 40e-6) + 2047 * 10.0e-3)) < 1e-9
    assert abs(fill["V(4,1)"] - max(7 * 65536 * 50e-6 + d_store, 2047 * 10.0e-3 + 8 * 65536 * 50e-6)) < 1e-9
    assert abs(m.target_ms(45.064) - 30.04) < 0.01


def test_family_table_runs_on_committed_inputs():
    """The committed inputs (profiles/n8_inputs.json, every number with its source) give
    the table DESIGN.md section 5 quotes: no in-fill family reaches the 6x line."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "n8_model.py"), "--families"],
                         capture_output=True, text=True, check=True).stdout
    assert "needs <= 30.04 ms per fill" in out
    rows = re.findall(r"^(\S+)\s+.*?\s([0-9.]+)ms\s+([0-9.]+)ms", out, re.M)
    assert len(rows) >= 12
    assert min(float(r[2]) for r in rows) > 30.04
