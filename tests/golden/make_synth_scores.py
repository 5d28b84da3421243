#!/usr/bin/env python3
"""Golden final scores for the seeded synthetic N x N workloads (SURVEY.md 8(d):
s1 = synth(seed 1), s2 = synth(seed 2), i.i.d. uniform {1,2,3,4}).

  32k, 64k : the reference's serial fill itself (oracle/_ref, full host table),
             cross-checked against the oracle restatement;
  >= 128k  : the oracle's linear-memory restatement (nw_oracle_score), which is
             pinned to the reference on every fixture pair (tests/test_oracle.py);
             the reference itself would need a 69 GB .. 1.1 TB host table.
Rectangular tables (RECT): the multi-GPU bench's weak-scaling legs below N = 8
(bench.py --gpus 2 / 4: row bands of 65536 rows per GPU over 524288 columns, and
column bands of 65536 columns per GPU over 524288 rows; N = 8 is the 524288 square
above; 524288 x 65536 is the one-GPU rehearsal of the row bands -- 2 local bands, and
bench.py --share-gpu with 2, 4 or 8 ranks of 65536 / N rows), from the oracle, keyed
"<n1>x<n2>:<scheme>" (nw_bands._golden).
Writes tests/golden/synth_scores.json: {"<n>:<match>,<mismatch>,<gap>": score}.
"""
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SCHEMES = {(1, 0, -1): "libref_serial.so", (1, -1, -1): "libref_serial_mm1.so"}
SIZES = [32768, 65536, 131072, 262144, 524288]
RECT = [(524288, 65536), (524288, 131072), (524288, 262144), (131072, 524288), (262144, 524288)]


def rect_job(n1, n2, scheme):
    import oracle
    t0 = time.time()
    sc = oracle.score(oracle.synth(1, n1), oracle.synth(2, n2), scheme)
    return f"{n1}x{n2}:{','.join(map(str, scheme))}", sc, "oracle", time.time() - t0


def job(n, scheme):
    import oracle
    s1, s2 = oracle.synth(1, n), oracle.synth(2, n)
    t0 = time.time()
    sc = oracle.score(s1, s2, scheme)
    src = "oracle"
    if n <= 65536 and oracle.ref_available(SCHEMES[scheme]):
        t = oracle.ref_fill(s1, s2, SCHEMES[scheme])
        assert int(t[-1, -1]) == sc, (n, scheme, int(t[-1, -1]), sc)
        src = "reference"
        del t
    return f"{n}:{','.join(map(str, scheme))}", sc, src, time.time() - t0


def main():
    out_path = os.path.join(HERE, "synth_scores.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    src = res.pop("_source", {})
    jobs = [(job, (n, s)) for n in SIZES for s in SCHEMES if f"{n}:{','.join(map(str, s))}" not in res]
    jobs += [(rect_job, (n1, n2, (1, 0, -1))) for n1, n2 in RECT if f"{n1}x{n2}:1,0,-1" not in res]
    with ProcessPoolExecutor(max_workers=4) as ex:
        futs = [ex.submit(f, *a) for f, a in jobs]
        for key, sc, how, dt in (fu.result() for fu in futs):
            res[key] = sc
            src[key] = how
            print(key, sc, how, f"{dt:.0f}s", flush=True)
            json.dump(dict(res, _source=src), open(out_path, "w"), indent=1, sort_keys=True)
    json.dump(dict(res, _source=src), open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
