"""Quick parity check of one strip shape against the oracle (experiment builds:
NWHIP_LIB=.../libnwhip_<variant>.so python tools/check_shape.py --sub 1 --nc 4)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402
import oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sub", type=int, default=1)
ap.add_argument("--nc", type=int, default=4)
ap.add_argument("--big", type=int, default=32768)
args = ap.parse_args()
ctx = nwhip.Context(0)
rng = np.random.default_rng(7)
shapes = [(1, 1), (5, 3), (63, 64), (64, 63), (65, 65), (255, 257), (256, 256), (257, 255),
          (300, 1000), (1000, 300), (1023, 1025), (1500, 1100), (4096, 777)]
bad = 0
for scheme in [(1, 0, -1), (1, -1, -1), (2, -1, -2)]:
    for (n1, n2) in shapes:
        for alpha in (4, 20):
            s1 = rng.integers(1, alpha + 1, n1).astype(np.int8)
            s2 = rng.integers(1, alpha + 1, n2).astype(np.int8)
            for col0 in (1, 0):
                d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
                if col0:
                    tab = nwhip.Context.alloc_table(n1, n2)
                else:
                    rows, pitch = nwhip.table_rows(n2), nwhip.table_pitch(n1)
                    flat = torch.empty(rows * pitch + 64, dtype=torch.int32, device="cuda")
                    sh = (-(flat.data_ptr() // 4)) % 64
                    tab = flat[sh:sh + rows * pitch].view(rows, pitch)
                r = ctx.fill(d1, d2, tab, scheme, substrips=args.sub, strip_waves=args.nc)
                got = tab[: n2 + 1, : n1 + 1].cpu().numpy()
                want = oracle.fill(s1, s2, scheme)
                if r.status != 0 or not np.array_equal(got, want):
                    bad += 1
                    idx = np.argwhere(got != want)
                    print("MISMATCH", scheme, n1, n2, alpha, col0, r.status, idx[:3].tolist(), flush=True)
print("small shapes:", "ok" if bad == 0 else f"{bad} bad", flush=True)
n = args.big
s1, s2 = oracle.synth(1, n), oracle.synth(2, n)
d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
tab = nwhip.Context.alloc_table(n, n)
for scheme in [(1, 0, -1), (1, -1, -1)]:
    r = ctx.fill(d1, d2, tab, scheme, substrips=args.sub, strip_waves=args.nc)
    sc, lr, lc, rs, rw = oracle.score(s1, s2, scheme, want_rows=True)
    got_lr = tab[n, : n + 1].cpu().numpy()
    got_lc = tab[: n + 1, n].cpu().numpy()
    t64 = tab[: n + 1, : n + 1].to(torch.int64)
    w = torch.arange(1, n + 2, dtype=torch.int64, device="cuda")
    gs = t64.sum(dim=1).cpu().numpy().view(np.uint64)
    gw = (t64 * w).sum(dim=1).cpu().numpy().view(np.uint64)
    ok = r.score == sc and np.array_equal(got_lr, lr) and np.array_equal(got_lc, lc) and \
        np.array_equal(gs, rs) and np.array_equal(gw, rw)
    print(f"{n}x{n} {scheme}: score {r.score} vs {sc} rows {'ok' if ok else 'MISMATCH'} "
          f"kernel {r.kernel_ms:.3f} ms", flush=True)
