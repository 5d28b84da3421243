"""Row-band partition of one Needleman-Wunsch table over several GPUs.

Reference contract: src/mpi/mpi-horz.cpp:4-99 with src/mpi/mpi-horz-driver.cpp:31-32,88-90.
Rank r owns a contiguous band of rows; for r > 0 the band's row 0 is rank r-1's last
row (the halo), streamed while rank r-1 is still filling; the final score is the last
rank's last cell.  The reference sends the halo in 1280-column MPI chunks
(mpi-horz.cpp:28-40,72-84).

MI355X design ("Multi-GPU"): one process per GPU.  Each rank's persistent
fill kernel (nw_fill_band_async) waits, strip by strip, for its halo granules
({tag, value}, one per column) and publishes its own last row, strip by strip, straight
into the next rank's halo buffer in peer HBM over xGMI (system-scope stores from the
kernel; the buffer is mapped with HIP IPC).  The halo therefore advances at strip
granularity (one strip: 64 * C * NC columns, C columns per lane, NC chained compute
waves) with no host round trip and no copy engine, collective or
stream-ordered gating on the data path.  torch.distributed (gloo) is the control plane
only: handle exchange, the per-step barrier and the max-over-ranks timing.

`LocalBands` runs P bands concurrently on ONE device (same kernels, same halo
protocol, local instead of peer memory): an API for band-sized fills and the
single-GPU parity vehicle for the multi-GPU path.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

import nwhip

HBM_PEAK_GBPS = 8000.0  # per GPU, MI355X_MICROARCH.md
LDS_PER_CU = 160 * 1024


def plan(n2: int, nbands: int):
    """[(rows incl. halo row, global row of row 0)] per band (mpi-horz-driver.cpp:31-32)."""
    return [nwhip.band_layout(n2, nbands, r) for r in range(nbands)]


def resident_waves(device: int = 0, substrips: int = 0, strip_waves: int = 0) -> int:
    """Persistent strip workgroups that fit on the device at once (LDS-bound:
    nw_strip_lds_bytes per workgroup, 160 KiB per CU)."""
    import torch
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    return cus * (LDS_PER_CU // nwhip.strip_lds_bytes(*nwhip.strip_shape(substrips, strip_waves)))


class LocalBands:
    """P row bands of one (n2+1) x (n1+1) table on one device, filled concurrently:
    band r on its own stream and context, halo r-1 -> r through a device buffer.
    Each band gets at most 1/P of the resident workers so that all bands are
    co-resident (a band waiting for its halo never blocks its producer)."""

    def __init__(self, n1: int, n2: int, nbands: int, device: int = 0, substrips: int = 0,
                 strip_waves: int = 0):
        import torch
        self.n1, self.n2, self.P, self.device = n1, n2, nbands, device
        self.layout = plan(n2, nbands)
        # one shape for every band (auto: the tuned shape for a band of this size)
        self.substrips, self.strip_waves = nwhip.strip_shape(
            substrips, strip_waves, n1, max(rows for rows, _ in self.layout) - 1)
        if any(rows < 1 for rows, _ in self.layout):
            raise ValueError(f"{nbands} bands need at least {nbands} rows (n2+1 = {n2 + 1})")
        self.tables = [nwhip.Context.alloc_table(n1, rows - 1) for rows, _ in self.layout]
        self.halos = [None] + [nwhip.Halo(n1, device) for _ in range(nbands - 1)]
        self.ctxs = [nwhip.Context(device) for _ in range(nbands)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nbands)]
        self.waves = max(1, resident_waves(device, self.substrips, self.strip_waves) // nbands)
        self.tag = 0

    def fill(self, d_s1, d_s2, scheme=(1, 0, -1), flags: int = 0, timeout_ms: int = 0) -> int:
        """Fill every band; returns the final score t[n2][n1] (last band's last cell)."""
        import torch
        assert int(d_s1.numel()) == self.n1 and int(d_s2.numel()) == self.n2
        self.tag += 1
        cur = torch.cuda.current_stream(self.device)
        for r, ((rows, start), st) in enumerate(zip(self.layout, self.streams)):
            st.wait_stream(cur)
            self.ctxs[r].fill_band(
                d_s1, d_s2[start:start + rows - 1], self.tables[r],
                halo_in=self.halos[r].ptr if r > 0 else None,
                halo_out=self.halos[r + 1].ptr if r + 1 < self.P else None,
                tag=self.tag, scheme=scheme, waves=self.waves, stream=st, flags=flags,
                substrips=self.substrips, strip_waves=self.strip_waves, row0=start,
                timeout_ms=timeout_ms)
        for r, st in enumerate(self.streams):
            s = self.ctxs[r].status(st)
            if s != nwhip.NW_OK:
                raise nwhip.NwError(s, f"band {r}")
            cur.wait_stream(st)
        rows, _ = self.layout[-1]
        return int(self.tables[-1][rows - 1, self.n1].item())

    def close(self):
        for h in self.halos:
            if h is not None:
                h.free()
        for c in self.ctxs:
            c.close()


# Per-row pace (ns) of a strip in a store-saturated sweep, per strip shape (C, NC):
# tools/rect_time.py on 65536 x 524288 (one pass of 256 strips): T = pace *
# (n2 + 255 * 64 * NC) gives (4,1) 35.7 ms -> 66.1, (2,2) 37.0 -> 66.4, (1,4) 29.7 -> 50.3
# (gpurun_out/rect_cb2.log, this round's final kernel).  The three shapes share the
# strip width W = 256 columns.
COLBAND_PACE_NS = {(4, 1): 66.1, (2, 2): 66.4, (1, 4): 50.3}


def colband_model_ms(n1: int, n2: int, shape) -> float:
    """Critical path of a column-band sweep (multi-GPU model): strip p
    starts one hop (64 * NC rows of the anti-diagonal skew) after strip p-1, so the
    last of S strips starts (S-1) hops in and then runs all n2 rows."""
    c, nc = shape
    strips = -(-n1 // (64 * c * nc))
    return COLBAND_PACE_NS[shape] * ((strips - 1) * 64 * nc + n2 + 1) * 1e-6


def colband_shape(n1: int, n2: int, substrips: int = 0, strip_waves: int = 0):
    """The strip shape of a column-band fill: the caller's, else the one of the
    W = 256 shapes whose modelled critical path is shortest (a chain of many strips
    wants the short hop of (4,1), a short chain the fast pace of (1,4))."""
    if substrips or strip_waves:
        return nwhip.strip_shape(substrips, strip_waves, n1, n2)
    return min(COLBAND_PACE_NS, key=lambda sh: colband_model_ms(n1, n2, sh))


class LocalColBands:
    """P column bands of one (n2+1) x (n1+1) table on one device, filled concurrently
    (src/mpi/mpi-vert.cpp's partition, the bands being whole strips of the table's
    sweep): band r's table holds global columns [start_r, start_r + n_cols_r), its
    local column 0 is band r-1's last column, fed to band r's first strip through a
    feed buffer as band r-1's last strip produces it.  Each band gets 1/P of the
    resident workers so that all bands are co-resident."""

    def __init__(self, n1: int, n2: int, nbands: int, device: int = 0, substrips: int = 0,
                 strip_waves: int = 0):
        import torch
        self.n1, self.n2, self.P, self.device = n1, n2, nbands, device
        # one shape for every band (auto: colband_shape)
        self.substrips, self.strip_waves = colband_shape(n1, n2, substrips, strip_waves)
        self.layout = [nwhip.colband_layout(n1, n2, nbands, r, self.substrips, self.strip_waves)
                       for r in range(nbands)]
        self.tables = [nwhip.Context.alloc_table(nc - 1, n2) for _, _, _, nc in self.layout]
        self.feeds = [None] + [nwhip.Feed(n2, device) for _ in range(nbands - 1)]
        self.ctxs = [nwhip.Context(device) for _ in range(nbands)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nbands)]
        self.waves = max(1, resident_waves(device, self.substrips, self.strip_waves) // nbands)
        self.tag = 0

    def fill(self, d_s1, d_s2, scheme=(1, 0, -1), flags: int = 0, timeout_ms: int = 0) -> int:
        """Fill every band; returns the final score t[n2][n1] (last band's last cell)."""
        import torch
        assert int(d_s1.numel()) == self.n1 and int(d_s2.numel()) == self.n2
        self.tag += 1
        cur = torch.cuda.current_stream(self.device)
        for r, st in enumerate(self.streams):
            st.wait_stream(cur)
            self.ctxs[r].fill_colband(
                d_s1, d_s2, self.tables[r], self.P, r,
                feed_in=self.feeds[r].ptr if r > 0 else None,
                feed_out=self.feeds[r + 1].ptr if r + 1 < self.P else None,
                tag=self.tag, scheme=scheme, waves=self.waves, stream=st, flags=flags,
                substrips=self.substrips, strip_waves=self.strip_waves, timeout_ms=timeout_ms)
        for r, st in enumerate(self.streams):
            s = self.ctxs[r].status(st)
            if s != nwhip.NW_OK:
                raise nwhip.NwError(s, f"column band {r}")
            cur.wait_stream(st)
        return int(self.tables[-1][self.n2, self.layout[-1][3] - 1].item())

    def close(self):
        for f in self.feeds:
            if f is not None:
                f.free()
        for c in self.ctxs:
            c.close()


# ----------------------------------------------------------------------- multi-process
def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _golden(n1: int, n2: int, scheme):
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "tests", "golden", "synth_scores.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        g = json.load(f)
    sch = ",".join(str(x) for x in scheme)
    key = f"{n1}:{sch}" if n1 == n2 else f"{n1}x{n2}:{sch}"
    return g.get(key)


def run_bands(args) -> dict | None:
    """bench.py --gpus N (N > 1) under torch.distributed.run: one rank per GPU, rank r
    fills band r of an n1 x (N * band_rows) table (weak scaling: per-GPU band fixed;
    at N = 8 with the defaults this is BASELINE config 4, 512k x 512k).
    Prints and returns the JSON line on rank 0."""
    import torch
    import torch.distributed as dist

    rank, world = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1)
    local = _env_int("LOCAL_RANK", rank)
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise RuntimeError("run_bands needs a GPU (there is no CPU fallback)")
    dev = 0 if args.share_gpu else local % ndev
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world)
    scheme = tuple(int(x) for x in args.scheme.split(","))
    cols = getattr(args, "partition", "rows") == "cols"
    ctx = nwhip.Context(dev)
    stream = torch.cuda.current_stream()
    if cols:
        # column bands (mpi-vert): rank r owns ~col_width columns of every row
        n1, n2 = world * args.col_width, args.col_rows
        sub, nc = colband_shape(n1, n2, args.substrips, args.strip_waves)
        sf, scount, start, ncols = nwhip.colband_layout(n1, n2, world, rank, sub, nc)
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
        table = nwhip.Context.alloc_table(ncols - 1, n2)
        link_in = nwhip.Feed(n2, dev) if rank > 0 else None
        rows = n2 + 1
    else:
        n1 = args.band_cols
        n2 = world * args.band_rows
        rows, start = nwhip.band_layout(n2, world, rank)
        # synthetic inputs, identical on every rank (seeds 1 / 2); this rank's side chars only
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n2)[start:start + rows - 1].copy()).cuda()
        table = nwhip.Context.alloc_table(n1, rows - 1)
        link_in = nwhip.Halo(n1, dev) if rank > 0 else None
        sub, nc = nwhip.strip_shape(args.substrips, args.strip_waves, n1, rows - 1)
    # each rank exports its incoming buffer; rank r-1 maps it and stores into it
    handles = [None] * world
    dist.all_gather_object(handles, nwhip.ipc_get_handle(link_in.ptr) if link_in else None)
    link_out = nwhip.ipc_open_handle(handles[rank + 1]) if rank + 1 < world else None
    waves = args.waves
    if args.share_gpu and waves == 0:
        waves = max(1, resident_waves(dev, sub, nc) // world)
    tag = 0

    def step(ev=None):
        nonlocal tag
        tag += 1
        if ev is not None:
            ev[0].record(stream)
        if cols:
            ctx.fill_colband(s1, s2, table, world, rank, feed_in=link_in.ptr if link_in else None,
                             feed_out=link_out, tag=tag, scheme=scheme, waves=waves, stream=stream,
                             substrips=sub, strip_waves=nc)
        else:
            ctx.fill_band(s1, s2, table, halo_in=link_in.ptr if link_in else None,
                          halo_out=link_out, tag=tag, scheme=scheme, waves=waves, stream=stream,
                          substrips=sub, strip_waves=nc, row0=start)
        if ev is not None:
            ev[1].record(stream)
        torch.cuda.synchronize()
        # no rank starts launch k+1 (which rewrites its neighbour's halo / feed)
        # before every rank has finished launch k
        dist.barrier()

    for _ in range(args.warmup):
        step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    status = ctx.status()
    kms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    st_all = [None] * world
    dist.all_gather_object(st_all, (status, kms, rows, start))
    last_col = (ncols - 1) if cols else n1
    score = int(table[rows - 1, last_col].item()) if rank == world - 1 else None
    scores = [None] * world
    dist.all_gather_object(scores, score)
    if link_out is not None:
        nwhip.ipc_close_handle(link_out)
    dist.barrier()
    if link_in is not None:
        link_in.free()
    ctx.close()
    if any(s[0] != 0 for s in st_all):
        raise RuntimeError(f"band status per rank: {[s[0] for s in st_all]}")
    if rank != 0:
        return None
    score = scores[-1]
    want = _golden(n1, n2, scheme)
    wall_s = float(wall.item())
    cells = n1 * n2
    ms_step = wall_s / args.steps * 1e3
    value = cells * args.steps / wall_s / 1e9
    table_bytes = 4.0 * (n1 + 1) * (n2 + 1)
    per_gpu_bytes = table_bytes / world
    achieved = per_gpu_bytes / (ms_step * 1e6)  # GB/s per GPU, whole step (incl. pipeline ramp)
    out = {
        "metric": "GCUPS (DP cell updates/s) on NxN NW fill, bit-exact score",
        "value": round(value, 2),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (i.i.d. uniform {1,2,3,4}, seeds 1/2)",
        "config": ({"workload": f"nw_fill_colbands_{n2}x{n1}", "n1": n1, "n2": n2,
                    "scheme": list(scheme), "col_width": args.col_width, "bands": world,
                    "table_bytes": int(table_bytes), "parallelism": f"column bands x{world}",
                    "halo": "in-kernel xGMI peer stores of the band's right column, 64 rows at a time",
                    "strip_shape": [sub, nc],
                    "control_plane": "torch.distributed gloo",
                    "shared_gpu": bool(args.share_gpu)} if cols else
                   {"workload": f"nw_fill_rowbands_{n2}x{n1}", "n1": n1, "n2": n2,
                    "scheme": list(scheme), "band_rows": args.band_rows, "bands": world,
                    "table_bytes": int(table_bytes), "parallelism": f"row bands x{world}",
                    "halo": f"in-kernel xGMI peer stores, one strip ({64 * sub * nc} columns) at a time",
                    "strip_shape": [sub, nc],
                    "control_plane": "torch.distributed gloo",
                    "shared_gpu": bool(args.share_gpu)}),
        "score": score,
        "score_golden": want,
        "score_ok": (want == score) if want is not None else None,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": None, "basis": "per GPU: band table bytes / ms_per_step",
                     "kernel_ms_avg_per_rank": [round(s[1], 3) for s in st_all]},
        "cpu_baseline": None,
        "kernel": nwhip.version(),
    }
    print(json.dumps(out), flush=True)
    return out
