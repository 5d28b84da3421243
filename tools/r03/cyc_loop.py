"""Repeat one LocalCycleBands case (diagnosing an intermittent watchdog)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
if len(sys.argv) > 5:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[5]
import numpy as np
import torch
import nw_bands, nwhip, oracle
P, m, n1, h = (int(x) for x in sys.argv[1:5])
n2 = P * m * h
rng = np.random.default_rng(1)
s1 = rng.integers(1, 5, n1).astype(np.int8)
s2 = rng.integers(1, 5, n2).astype(np.int8)
want = oracle.fill(s1, s2, (1, 0, -1))
for it in range(6):
    lb = nw_bands.LocalCycleBands(n1, n2, P, m, substrips=2, strip_waves=2)
    t0 = time.time()
    try:
        sc = lb.fill(torch.from_numpy(s1).cuda(), s2, (1, 0, -1), timeout_ms=2000)
        print(it, "ok", sc == want[-1, -1], round(time.time() - t0, 3), flush=True)
    except Exception as e:
        print(it, "FAIL", e, flush=True)
    lb.close()
