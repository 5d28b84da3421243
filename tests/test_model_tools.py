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
