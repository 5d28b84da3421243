#!/usr/bin/env python3
"""Golden vectors for Smith-Waterman + traceback (BASELINE config 5).

PARITY UNPINNED: the reference has no local alignment (README.md:2), so these
come from the build's own CPU restatement (oracle/nw_oracle.c nw_oracle_sw_*,
cross-checked in tests/test_oracle.py against an independent pure-Python
restatement on small pairs).  Conventions: 0 floor, best cell = first
row-major maximum, traceback diag > up > left.

For each case: score, best cell, traceback begin, number of ops and the
sha256 of the ops bytes (path order begin -> end; 0 diag, 1 up, 2 left).
  * the reference's bdna fixture pairs small/t/debug/smid;
  * the synthetic 65536 x 65536 workload (seeds 1/2) -- config 5 -- whose full
    17 GB table the oracle fills in host RAM here.
Writes tests/golden/sw_golden.json.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

SCHEMES = [(1, -1, -1), (1, 0, -1), (2, -1, -2)]


def case(s1, s2, scheme):
    t0 = time.time()
    t = oracle.sw_fill(s1, s2, scheme)
    sc, ei, ej = oracle.sw_best(s1, s2, scheme)
    assert int(t[ei, ej]) == sc
    ops, bi, bj = oracle.sw_traceback(s1, s2, t, (ei, ej), scheme)
    del t
    assert oracle.sw_path_score(s1, s2, ops, (bi, bj), scheme) == sc
    return {"score": sc, "end": [ei, ej], "begin": [bi, bj], "n_ops": int(ops.size),
            "ops_sha256": hashlib.sha256(ops.tobytes()).hexdigest(),
            "ops_counts": [int((ops == k).sum()) for k in range(3)], "secs": round(time.time() - t0, 1)}


def main():
    golden = json.load(open(os.path.join(HERE, "golden.json")))
    out = {"conventions": "0 floor; best = first row-major max; traceback diag > up > left; "
                          "ops begin->end 0 diag 1 up 2 left", "pairs": {}, "synth": {}}
    for name in ["small", "t", "debug", "smid"]:
        e = golden["pairs"][name]
        rd = lambda f: np.fromfile(os.path.join(HERE, "bdna", f), dtype=np.int8)
        s1, s2 = rd(e["argv1"]), rd(e["argv2"])
        for sch in SCHEMES:
            out["pairs"][f"{name}:{','.join(map(str, sch))}"] = case(s1, s2, sch)
    n = 65536
    s1, s2 = oracle.synth(1, n), oracle.synth(2, n)
    for sch in SCHEMES[:2]:
        r = case(s1, s2, sch)
        print(n, sch, r, flush=True)
        out["synth"][f"{n}:{','.join(map(str, sch))}"] = r
    json.dump(out, open(os.path.join(HERE, "sw_golden.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
