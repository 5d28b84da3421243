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


def resident_waves(device: int = 0, substrips: int = 0, strip_waves: int = 0, kernel: int = 0) -> int:
    """Persistent strip / panel workgroups that fit on the device at once
    (LDS-bound: nw_strip_lds_bytes / nw_panel_lds_bytes per workgroup, 160 KiB per
    CU; a panel workgroup of 2 * NW waves also counts against 32 waves per CU)."""
    import torch
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    if kernel == nwhip.KERNEL_PANELS:
        return cus  # one panel workgroup per CU (nw_capi.cpp make_shape)
    return cus * (LDS_PER_CU // nwhip.strip_lds_bytes(*nwhip.strip_shape(substrips, strip_waves)))


def panel_shape_for(cols: int, cus: int = 256):
    """Panel shape (C, NW) for a sweep of `cols` columns on `cus` CUs: the widest
    panel that still gives every CU one (nw_capi.cpp panel_auto)."""
    if cols >= cus * 1024:
        return 4, 4
    if cols >= cus * 512:
        return 2, 4
    return 4, 1


def band_shape(n1: int, n2_band: int, substrips: int = 0, strip_waves: int = 0, kernel: int = 0):
    """Shape of a row-band fill: the caller's, else strips: the tuned shape for
    a band of this size; panels: panel_shape_for(n1)."""
    if kernel == nwhip.KERNEL_PANELS:
        return (substrips, strip_waves) if (substrips or strip_waves) else panel_shape_for(n1 + 1)
    return nwhip.strip_shape(substrips, strip_waves, n1, n2_band)


class LocalBands:
    """P row bands of one (n2+1) x (n1+1) table on one device, filled concurrently:
    band r on its own stream and context, halo r-1 -> r through a device buffer.
    Each band gets at most 1/P of the resident workers so that all bands are
    co-resident (a band waiting for its halo never blocks its producer)."""

    def __init__(self, n1: int, n2: int, nbands: int, device: int = 0, substrips: int = 0,
                 strip_waves: int = 0, kernel: int = 0):
        import torch
        self.n1, self.n2, self.P, self.device, self.kernel = n1, n2, nbands, device, kernel
        self.layout = plan(n2, nbands)
        # one shape for every band (auto: the tuned shape for a band of this size)
        self.substrips, self.strip_waves = band_shape(
            n1, max(rows for rows, _ in self.layout) - 1, substrips, strip_waves, kernel)
        if any(rows < 1 for rows, _ in self.layout):
            raise ValueError(f"{nbands} bands need at least {nbands} rows (n2+1 = {n2 + 1})")
        self.tables = [nwhip.Context.alloc_table(n1, rows - 1) for rows, _ in self.layout]
        self.halos = [None] + [nwhip.Halo(n1, device) for _ in range(nbands - 1)]
        self.ctxs = [nwhip.Context(device) for _ in range(nbands)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nbands)]
        self.waves = max(1, resident_waves(device, self.substrips, self.strip_waves, kernel) // nbands)
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
                timeout_ms=timeout_ms, kernel=self.kernel)
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


def colband_shape(n1: int, n2: int, substrips: int = 0, strip_waves: int = 0, kernel: int = 0,
                  nbands: int = 1):
    """The shape of a column-band fill: the caller's, else for panels the panel
    that gives each CU one panel of its band (n1 / nbands columns), for strips the
    W = 256 shape whose modelled critical path is shortest (a chain of many strips
    wants the short hop of (4,1), a short chain the fast pace of (1,4))."""
    if kernel == nwhip.KERNEL_PANELS:
        return (substrips, strip_waves) if (substrips or strip_waves) else panel_shape_for(n1 // max(1, nbands))
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
                 strip_waves: int = 0, kernel: int = 0):
        import torch
        self.n1, self.n2, self.P, self.device, self.kernel = n1, n2, nbands, device, kernel
        # one shape for every band (auto: colband_shape)
        self.substrips, self.strip_waves = colband_shape(n1, n2, substrips, strip_waves, kernel, nbands)
        self.layout = [nwhip.colband_layout(n1, n2, nbands, r, self.substrips, self.strip_waves, kernel)
                       for r in range(nbands)]
        self.tables = [nwhip.Context.alloc_table(nc - 1, n2) for _, _, _, nc in self.layout]
        self.feeds = [None] + [nwhip.Feed(n2, device) for _ in range(nbands - 1)]
        self.ctxs = [nwhip.Context(device) for _ in range(nbands)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nbands)]
        self.waves = max(1, resident_waves(device, self.substrips, self.strip_waves, kernel) // nbands)
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
                substrips=self.substrips, strip_waves=self.strip_waves, timeout_ms=timeout_ms,
                kernel=self.kernel)
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


def _sweep(args, partition: str, rank: int, world: int, dev: int, scheme) -> dict:
    """One multi-rank band sweep: `warmup` + `steps` fills enqueued back to back on
    this rank's stream, halo / feed buffers alternating by launch parity, the
    producer's stream waiting on the consumer's "done with launch k" link word
    (nw_link_*) before it rewrites that launch's buffer -- no host round trip
    between launches.  Returns this rank's measurements (wall time of the timed
    launches between a barrier + synchronize on both sides)."""
    import torch
    import torch.distributed as dist

    cols = partition == "cols"
    kernel = getattr(args, "kernel", 0)
    ctx = nwhip.Context(dev)
    stream = torch.cuda.current_stream()
    if cols:
        # column bands (mpi-vert): rank r owns ~col_width columns of every row
        n1, n2 = world * args.col_width, args.col_rows
        sub, nc = colband_shape(n1, n2, args.substrips, args.strip_waves, kernel, world)
        sf, scount, start, ncols = nwhip.colband_layout(n1, n2, world, rank, sub, nc, kernel=kernel)
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
        table = nwhip.Context.alloc_table(ncols - 1, n2)
        links_in = [nwhip.Feed(n2, dev) for _ in range(2)] if rank > 0 else None
        rows = n2 + 1
    else:
        # row bands (mpi-horz, BASELINE config 4): rank r owns band_rows rows
        n1 = args.band_cols
        n2 = world * args.band_rows
        rows, start = nwhip.band_layout(n2, world, rank)
        # synthetic inputs, identical on every rank (seeds 1 / 2); this rank's side chars only
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n2)[start:start + rows - 1].copy()).cuda()
        table = nwhip.Context.alloc_table(n1, rows - 1)
        links_in = [nwhip.Halo(n1, dev) for _ in range(2)] if rank > 0 else None
        sub, nc = band_shape(n1, rows - 1, args.substrips, args.strip_waves, kernel)
        ncols = n1 + 1
    # rank r exports its two incoming buffers and (r < world-1) the link word its
    # consumer r+1 signals into; rank r maps r+1's buffers and r-1's word
    link_word = nwhip.Link(dev) if rank + 1 < world else None
    mine = ([nwhip.ipc_get_handle(b.ptr) for b in links_in] if links_in else None,
            nwhip.ipc_get_handle(link_word.ptr) if link_word else None)
    handles = [None] * world
    dist.all_gather_object(handles, mine)
    out_bufs = [nwhip.ipc_open_handle(h) for h in handles[rank + 1][0]] if rank + 1 < world else None
    prod_word = nwhip.ipc_open_handle(handles[rank - 1][1]) if rank > 0 else None
    waves = args.waves
    if args.share_gpu and waves == 0:
        waves = max(1, resident_waves(dev, sub, nc, kernel) // world)

    def launch(k: int, ev=None):
        """Launch k (tag k >= 1) on this rank's stream, buffers k % 2."""
        b = k % 2
        if out_bufs is not None and k >= 3:
            nwhip.link_wait(link_word.ptr, k - 2, stream)  # consumer done with launch k-2
        if ev is not None:
            ev[0].record(stream)
        kw = dict(tag=k, scheme=scheme, waves=waves, stream=stream, substrips=sub, strip_waves=nc,
                  kernel=kernel)
        if cols:
            ctx.fill_colband(s1, s2, table, world, rank, feed_in=links_in[b].ptr if links_in else None,
                             feed_out=out_bufs[b] if out_bufs else None, **kw)
        else:
            ctx.fill_band(s1, s2, table, halo_in=links_in[b].ptr if links_in else None,
                          halo_out=out_bufs[b] if out_bufs else None, row0=start, **kw)
        if ev is not None:
            ev[1].record(stream)
        if prod_word is not None:
            nwhip.link_signal(prod_word, k, stream)  # done reading launch k's buffer

    for k in range(1, args.warmup + 1):
        launch(k)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, e in enumerate(evs):
        launch(args.warmup + 1 + i, e)
    torch.cuda.synchronize()
    dist.barrier()
    wall = time.perf_counter() - t0
    status = ctx.status()
    link_status = link_word.status() if link_word else 0
    kms = float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else 0.0
    score = int(table[rows - 1, ncols - 1].item()) if rank == world - 1 else None
    dist.barrier()
    if out_bufs:
        for x in out_bufs:
            nwhip.ipc_close_handle(x)
    if prod_word is not None:
        nwhip.ipc_close_handle(prod_word)
    dist.barrier()
    for x in (links_in or []) + ([link_word] if link_word else []):
        x.free()
    ctx.close()
    del table
    torch.cuda.empty_cache()
    return {"wall": wall, "status": status, "link_status": link_status, "kms": kms, "score": score,
            "n1": n1, "n2": n2, "shape": [sub, nc], "kernel": kernel, "rows": rows, "start": start}


def run_bands(args) -> dict | None:
    """bench.py --gpus N (N > 1) under torch.distributed.run: one rank per GPU.
    `value` = row bands (BASELINE config 4, mpi-horz): rank r fills band r of an
    n1 x (N * band_rows) table (weak scaling: per-GPU band fixed; at N = 8 with the
    defaults this is 512k x 512k).  The other partition (column bands, mpi-vert:
    N * col_width columns x col_rows rows) runs after it as `alt_partition` unless
    --alt-partition none.  Prints and returns the JSON line on rank 0."""
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
    main = getattr(args, "partition", "rows")
    alt = getattr(args, "alt_partition", None)
    if alt is None:
        alt = "cols" if main == "rows" else "rows"
    legs = {}
    for part in [main] + ([alt] if alt not in ("none", main) else []):
        m = _sweep(args, part, rank, world, dev, scheme)
        allm = [None] * world
        dist.all_gather_object(allm, m)
        legs[part] = allm
    if rank != 0:
        return None
    out = _line(args, world, scheme, main, legs[main])
    if alt in legs:
        a = _line(args, world, scheme, alt, legs[alt])
        out["alt_partition"] = {k: a[k] for k in ("value", "ms_per_step", "config", "score", "score_golden",
                                                  "score_ok", "roofline")}
    if cpu_baseline_fn is not None and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_fn(args.cpu_n, scheme)
    print(json.dumps(out), flush=True)
    bad = [(p, [m["status"] for m in legs[p]], [m["link_status"] for m in legs[p]]) for p in legs
           if any(m["status"] != 0 or m["link_status"] != 0 for m in legs[p])]
    if bad:
        raise RuntimeError(f"band status per rank (fill, link): {bad}")
    return out


cpu_baseline_fn = None  # bench.py installs its cpu_baseline (rank 0 only reports it)


def _line(args, world: int, scheme, part: str, ms: list) -> dict:
    """The bench JSON line of one partition from every rank's _sweep result."""
    cols = part == "cols"
    m0, ml = ms[0], ms[-1]
    n1, n2 = m0["n1"], m0["n2"]
    wall_s = max(m["wall"] for m in ms)  # max over ranks
    score = ml["score"]
    want = _golden(n1, n2, scheme)
    cells = n1 * n2
    ms_step = wall_s / args.steps * 1e3
    value = cells * args.steps / wall_s / 1e9
    table_bytes = 4.0 * (n1 + 1) * (n2 + 1)
    per_gpu_bytes = table_bytes / world
    achieved = per_gpu_bytes / (ms_step * 1e6)  # GB/s per GPU, whole step (incl. pipeline ramp)
    kern = {0: "auto", 1: "strips", 2: "panels"}[m0["kernel"]]
    common = {"n1": n1, "n2": n2, "scheme": list(scheme), "bands": world, "table_bytes": int(table_bytes),
              "kernel": kern, "shape": m0["shape"], "control_plane": "torch.distributed gloo (setup, barriers)",
              "launches": "back to back, buffers by launch parity, link-word flow control (nw_link_*)",
              "shared_gpu": bool(args.share_gpu)}
    if cols:
        cfg = {"workload": f"nw_fill_colbands_{n2}x{n1}", "col_width": args.col_width,
               "parallelism": f"column bands x{world} (mpi-vert)",
               "halo": "in-kernel xGMI peer stores of the band's right column, 16 rows at a time", **common}
    else:
        cfg = {"workload": f"nw_fill_rowbands_{n2}x{n1}", "band_rows": args.band_rows,
               "parallelism": f"row bands x{world} (mpi-horz, BASELINE config 4)",
               "halo": "in-kernel xGMI peer stores of the band's last row, as each strip/panel finishes",
               **common}
    return {
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
        "config": cfg,
        "score": score,
        "score_golden": want,
        "score_ok": (want == score) if want is not None else None,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": None, "basis": "per GPU: band table bytes / ms_per_step (whole step)",
                     "kernel_ms_avg_per_rank": [round(m["kms"], 3) for m in ms]},
        "cpu_baseline": None,
        "kernel": nwhip.version(),
    }
