#!/usr/bin/env python3
"""CPU baseline leg of bench.py -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

Times one CPU fill of the reference on an n x n sample of the bench workload
(synthetic seeds 1/2) and prints one JSON object.  Runs as its
own process so that OMP_NUM_THREADS / OMP_PROC_BIND=close reach the OpenMP
runtime before it starts (bench.py sets them).

  --fill serial       src/serial/serial.cpp:4-36 (1 thread)
  --fill idxarray-mt  src/idxarray/idxarray-mt.cpp:4-70 (OpenMP team of
                      OMP_NUM_THREADS threads, progress counters per row)

kind "reference": the reference's own sources compiled unmodified into
oracle/_ref/ (oracle/Makefile `make ref`); kind "port": the C restatement
oracle/nw_oracle.c (nw_oracle_fill / nw_oracle_fill_idxarray) when _ref is absent.
Timing scope = the fill call only, as src/common/driver.cpp:26-30 (the table is
allocated and its pages touched before the timer, driver.cpp:22-23).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle  # noqa: E402

REF = {("serial", (1, 0, -1)): "libref_serial.so", ("serial", (1, -1, -1)): "libref_serial_mm1.so",
       ("serial", (2, -1, -2)): "libref_serial_p3.so",
       ("idxarray-mt", (1, 0, -1)): "libref_idxarray_mt.so",
       ("idxarray-mt", (1, -1, -1)): "libref_idxarray_mt_mm1.so"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fill", choices=["serial", "idxarray-mt"], default="serial")
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--scheme", default="1,0,-1")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    scheme = tuple(int(x) for x in args.scheme.split(","))
    n = args.n
    s1, s2 = oracle.synth(1, n), oracle.synth(2, n)
    lib_name = REF.get((args.fill, scheme))
    kind = "reference" if lib_name and oracle.ref_available(lib_name) else "port"
    threads = int(os.environ.get("OMP_NUM_THREADS", "1")) if args.fill == "idxarray-mt" else 1
    t = np.ones((n + 1, n + 1), dtype=np.int32)  # pages touched (driver.cpp:23)
    tp = t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    a, b = np.ascontiguousarray(s1), np.ascontiguousarray(s2)
    if kind == "reference":
        L = ctypes.CDLL(os.path.join(oracle.REF_DIR, lib_name))
        fn = getattr(L, "_Z15needlemanWunsch8dnaArrayS_Pi")
        fn.argtypes = [oracle.DnaArray, oracle.DnaArray, ctypes.POINTER(ctypes.c_int32)]
        fn.restype = None
        i8 = ctypes.POINTER(ctypes.c_int8)
        run = lambda: fn(oracle.DnaArray(n, a.ctypes.data_as(i8)), oracle.DnaArray(n, b.ctypes.data_as(i8)), tp)
    else:
        L = oracle.lib()
        i8 = ctypes.POINTER(ctypes.c_int8)
        if args.fill == "serial":
            run = lambda: L.nw_oracle_fill(a.ctypes.data_as(i8), n, b.ctypes.data_as(i8), n, *scheme, tp, n + 1)
        else:
            run = lambda: L.nw_oracle_fill_idxarray(a.ctypes.data_as(i8), n, b.ctypes.data_as(i8), n,
                                                    *scheme, tp, threads)
    secs = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        run()
        secs.append(time.perf_counter() - t0)
    med = statistics.median(secs)
    print(json.dumps({"fill": args.fill, "kind": kind, "n": n, "threads": threads,
                      "gcups": round(n * n / med / 1e9, 4), "seconds": [round(x, 3) for x in secs],
                      "score": int(t[n, n])}))


if __name__ == "__main__":
    main()
