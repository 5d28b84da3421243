#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE ITSELF.

Run in the build container (where /root/reference exists):

    make -C oracle all ref && python tests/golden/make_golden.py

What it does
  * copies a selection of the reference's own input files (bdna/*.bdna: raw
    bytes, data only) into tests/golden/bdna/ so tests can run where the
    reference tree is absent (the GPU box);
  * runs the reference's serial fill (src/serial/serial.cpp, compiled unmodified
    into oracle/_ref/ by oracle/Makefile) under three scoring schemes and
    records: full tables for the tiny pairs (.npy), and for the larger pairs the
    final score, last row, last column and per-row checksums (.npz);
  * cross-checks the reference's sentinel-mt and idxarray-mt fills
    (src/sentinel/sentinel-mt.cpp, src/idxarray/idxarray-mt.cpp) on the small
    pairs, recording their scores too.

Nothing here is imported by the product or by the GPU tests; the GPU tests only
read the files this script writes.
"""
from __future__ import annotations

import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

REF_BDNA = "/root/reference/bdna"
OUT_BDNA = os.path.join(HERE, "bdna")

# (name, argv1 file, argv2 file): argv1 = s1 "across the top", argv2 = s2 "down the side"
PAIRS = [
    ("small", "small1.bdna", "small2.bdna"),
    ("small_rev", "small2.bdna", "small1.bdna"),
    ("t", "t1.bdna", "t2.bdna"),
    ("debug", "debug1.bdna", "debug2.bdna"),
    ("smid", "smid1.bdna", "smid2.bdna"),
    ("2gb", "2gb-1.bdna", "2gb-2.bdna"),
    ("4gb", "4gb-1.bdna", "4gb-2.bdna"),
    ("8gb", "8gb-1.bdna", "8gb-2.bdna"),
    ("mid", "mid1.bdna", "mid2.bdna"),
    ("big", "big1.bdna", "big2.bdna"),
]
FULL_TABLE = {"small", "small_rev", "t", "debug"}
ROW_DATA = {"smid", "2gb"}
SCHEME_LIB = {"shipped": "libref_serial.so", "mm1": "libref_serial_mm1.so", "p3": "libref_serial_p3.so"}
MT_LIBS = {"shipped": ["libref_sentinel_mt.so", "libref_idxarray_mt.so"],
           "mm1": ["libref_sentinel_mt_mm1.so", "libref_idxarray_mt_mm1.so"]}
# the 40 GB `big` table and the p3 scheme on the largest pairs are skipped to bound host RAM/time
SKIP = {("big", "p3"), ("mid", "p3"), ("8gb", "p3")}


def read_bdna(path: str) -> np.ndarray:
    """readSequence semantics (src/common/helper.cpp:3-25): every byte, no stripping."""
    with open(path, "rb") as f:
        return np.frombuffer(f.read(), dtype=np.int8).copy()


def main() -> None:
    if not os.path.isdir(REF_BDNA) or not oracle.ref_available():
        sys.exit("needs /root/reference and `make -C oracle ref`")
    os.makedirs(OUT_BDNA, exist_ok=True)
    golden = {"source": "reference serial.cpp compiled unmodified (oracle/Makefile)",
              "schemes": oracle.SCHEMES, "pairs": {}}
    for name, f1, f2 in PAIRS:
        for f in (f1, f2):
            shutil.copyfile(os.path.join(REF_BDNA, f), os.path.join(OUT_BDNA, f))
        s1 = read_bdna(os.path.join(REF_BDNA, f1))
        s2 = read_bdna(os.path.join(REF_BDNA, f2))
        entry = {"argv1": f1, "argv2": f2, "n1": int(s1.size), "n2": int(s2.size), "scores": {}}
        for scheme, libname in SCHEME_LIB.items():
            if (name, scheme) in SKIP:
                continue
            t = oracle.ref_fill(s1, s2, libname)
            entry["scores"][scheme] = int(t[-1, -1])
            if name in FULL_TABLE:
                np.save(os.path.join(HERE, f"table_{scheme}_{name}.npy"), t)
            if name in ROW_DATA:
                rs, rw = oracle.row_checksums(t)
                np.savez_compressed(os.path.join(HERE, f"rows_{scheme}_{name}.npz"),
                                    last_row=t[-1].copy(), last_col=t[:, -1].copy(),
                                    row_sum=rs, row_wsum=rw)
            if name in FULL_TABLE or name == "smid":
                for mt in MT_LIBS.get(scheme, []):
                    tm = oracle.ref_fill(s1, s2, mt)
                    entry.setdefault("mt_scores", {}).setdefault(scheme, {})[mt] = int(tm[-1, -1])
                    entry.setdefault("mt_table_equal", {}).setdefault(scheme, {})[mt] = bool(
                        np.array_equal(tm, t))
            del t
            print(name, scheme, entry["scores"][scheme], flush=True)
        golden["pairs"][name] = entry
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
