import sys, numpy as np, torch
sys.path.insert(0, "fast-needleman-wunsch_amd"); sys.path.insert(0, "oracle")
import nwhip, oracle
ctx = nwhip.Context(0)
bad = 0
for (n1, n2) in [(1,1),(63,64),(64,1),(255,33),(256,256),(1000,777),(1500,1100),(70,2000),(3000,95)]:
    rng = np.random.default_rng(n1*7+n2)
    s1 = rng.integers(1,5,n1).astype(np.int8); s2 = rng.integers(1,5,n2).astype(np.int8)
    for sch in [(1,0,-1),(1,-1,-1),(2,-1,-2)]:
        for mode in (nwhip.MODE_NW, nwhip.MODE_SW):
            d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
            tab = nwhip.Context.alloc_table(n1, n2)
            r = ctx.fill(d1, d2, tab, sch, substrips=1, strip_waves=4, mode=mode)
            want = oracle.fill(s1, s2, sch) if mode == nwhip.MODE_NW else oracle.sw_fill(s1, s2, sch)
            ok = np.array_equal(tab[:n2+1,:n1+1].cpu().numpy(), want)
            bad += not ok
            if not ok: print("MISMATCH", n1, n2, sch, mode)
print("bad", bad)
