"""Debug: small fills of every strip shape / origin vs the oracle, with status."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402
import oracle  # noqa: E402

ctx = nwhip.Context(0)
shapes = [tuple(int(v) for v in x.split(":")) for x in (sys.argv[1] if len(sys.argv) > 1 else "4:1,2:1,1:1,2:2,1:2,1:4").split(",")]
sizes = [(300, 200), (1000, 777), (5000, 3000)]
for c, nc in shapes:
    for n1, n2 in sizes:
        rng = np.random.default_rng(n1 + n2)
        s1 = rng.integers(1, 5, n1).astype(np.int8)
        s2 = rng.integers(1, 5, n2).astype(np.int8)
        t0 = time.time()
        try:
            d1 = torch.from_numpy(s1).cuda()
            d2 = torch.from_numpy(s2).cuda()
            tab = nwhip.Context.alloc_table(n1, n2)
            r = ctx.fill(d1, d2, tab, (1, 0, -1), substrips=c, strip_waves=nc)
            got = tab[:n2 + 1, :n1 + 1].cpu().numpy()
            want = oracle.fill(s1, s2)
            bad = np.argwhere(got != want)
            print(f"C={c} NC={nc} {n1}x{n2}: status {r.status} strips {r.strips} waves {r.waves} "
                  f"mismatches {len(bad)} first {bad[:3].tolist()} {time.time() - t0:.2f}s", flush=True)
        except Exception as e:  # noqa: BLE001
            import ctypes
            w = (ctypes.c_uint32 * 8)()
            nwhip.lib().nw_debug_ctrl(ctx._h, w)
            site = w[2] >> 24
            print(f"C={c} NC={nc} {n1}x{n2}: EXC {e} {time.time() - t0:.2f}s ctrl={list(w)} "
                  f"site={site} wave={(w[2] >> 16) & 255} off={w[2] & 0xFFFF:#x} need={w[3]} "
                  f"seen={w[4]}", flush=True)
            ctx.close()
            ctx = nwhip.Context(0)
