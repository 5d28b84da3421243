"""Debug: the panel kernel's compare (GEN) path on a small case vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import nwhip, oracle
for alpha, flags in (("bytes", 0), ("dna", nwhip.FLAG_NO_PROFILE), ("dna", 0)):
    for shape in ((63, 65), (5, 3), (300, 20)):
        rng = np.random.default_rng(shape[0] * 7919 + shape[1] + (alpha == "bytes"))
        lo, hi = (1, 5) if alpha == "dna" else (-128, 128)
        s1 = rng.integers(lo, hi, shape[0]).astype(np.int8)
        s2 = rng.integers(lo, hi, shape[1]).astype(np.int8)
        for panel in ((4, 4), (4, 1), (1, 4)):
            t, r = nwhip.fill(s1, s2, (1, 0, -1), substrips=panel[0], strip_waves=panel[1], flags=flags, kernel=2)
            o = oracle.fill(s1, s2, (1, 0, -1))
            bad = np.argwhere(t != o)
            print(alpha, flags, shape, panel, "mismatches", len(bad), "first", bad[:3].tolist(),
                  "row1 got", t[1, :8].tolist(), "want", o[1, :8].tolist(), flush=True)
