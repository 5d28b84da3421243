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

The bench's `value` sweeps each band in HORIZONTAL strips (nw_fill_tband_async: 256-row
strips running along the columns, the halo a feed of one granule per column written by
the band's last strip's store waves), so that band r+1 starts a strip hop after band r
rather than after band r's whole height; the vertical sweep above, block-cyclic bands and
column bands run as alternate legs.  Every N > 1 number is the
per-fill latency of mpi-horz-driver.cpp:38-83 (fill_latencies), with the back-to-back
throughput reported beside it.

`LocalBands` / `LocalTBands` run P bands concurrently on ONE device (same kernels,
same halo protocol, local instead of peer memory): an API for band-sized fills and
the single-GPU parity vehicles for the multi-GPU path.
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


class LocalTBands:
    """P row bands of one (n2+1) x (n1+1) table on one device in HORIZONTAL strips
    (nw_fill_tband_async): the mpi-horz partition and row-major band tables of
    LocalBands, each band swept as 256-row strips along the columns, band r-1's
    last row fed to band r column by column through a Feed(n1) buffer.  Each band
    gets 1/P of the resident workers so that all bands are co-resident.  shape: the
    strip shape (C, NC), TBAND_SHAPE by default ((4, 1) or (2, 2))."""

    def __init__(self, n1: int, n2: int, nbands: int, device: int = 0, shape=None, dense_polls: bool = False):
        import torch
        self.n1, self.n2, self.P, self.device = n1, n2, nbands, device
        self.shape = tuple(shape) if shape else TBAND_SHAPE
        self.dense_polls = dense_polls
        self.layout = plan(n2, nbands)
        if any(rows < 2 for rows, _ in self.layout):
            raise ValueError(f"{nbands} horizontal-strip bands need at least one row below each halo")
        self.tables = [nwhip.Context.alloc_table(n1, rows - 1) for rows, _ in self.layout]
        self.feeds = [None] + [nwhip.Feed(n1, device) for _ in range(nbands - 1)]
        self.ctxs = [nwhip.Context(device) for _ in range(nbands)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nbands)]
        self.waves = max(1, resident_waves(device, *self.shape) // nbands)
        self.tag = 0

    def fill(self, d_s1, d_s2, scheme=(1, 0, -1), flags: int = 0, timeout_ms: int = 0) -> int:
        """Fill every band; returns the final score t[n2][n1] (last band's last cell)."""
        import torch
        assert int(d_s1.numel()) == self.n1 and int(d_s2.numel()) == self.n2
        self.tag += 1
        cur = torch.cuda.current_stream(self.device)
        for r, ((rows, start), st) in enumerate(zip(self.layout, self.streams)):
            st.wait_stream(cur)
            self.ctxs[r].fill_tband(
                d_s1, d_s2[start:start + rows - 1], self.tables[r], row0=start,
                feed_in=self.feeds[r].ptr if r > 0 else None,
                feed_out=self.feeds[r + 1].ptr if r + 1 < self.P else None,
                tag=self.tag, scheme=scheme, waves=self.waves, stream=st, flags=flags, timeout_ms=timeout_ms,
                substrips=self.shape[0], strip_waves=self.shape[1], dense_polls=self.dense_polls)
        for r, st in enumerate(self.streams):
            s = self.ctxs[r].status(st)
            if s != nwhip.NW_OK:
                raise nwhip.NwError(s, f"horizontal-strip band {r}")
            cur.wait_stream(st)
        rows, _ = self.layout[-1]
        return int(self.tables[-1][rows - 1, self.n1].item())

    def close(self):
        for f in self.feeds:
            if f is not None:
                f.free()
        for c in self.ctxs:
            c.close()


def cycle_layout(n2: int, nranks: int, nblk: int):
    """Block-cyclic row bands (nw_fill_band_cycle_async): the n2 rows below row 0
    cut into nranks * nblk blocks of h rows, global block g = k * nranks + r being
    rank r's block k, its row 0 = global row g * h (the previous block's last row).
    Returns h; n2 must be a multiple of nranks * nblk."""
    nb = nranks * nblk
    if nranks < 1 or nblk < 1 or n2 < nb or n2 % nb:
        raise ValueError(f"block-cyclic bands need n2 = {n2} to be a positive multiple of {nb} blocks")
    return n2 // nb


def cycle_side_chars(s2, h: int, nranks: int, nblk: int, r: int):
    """Rank r's side characters, block k's h of them at [k*h, (k+1)*h): global
    rows g*h + 1 .. (g+1)*h use s2[g*h : (g+1)*h], g = k * nranks + r."""
    return np.concatenate([s2[(k * nranks + r) * h:(k * nranks + r + 1) * h] for k in range(nblk)])


class LocalCycleBands:
    """Block-cyclic row bands of one (n2+1) x (n1+1) table on ONE device, P ranks
    (contexts, 1/P of the resident workers each) of nblk blocks, halo regions
    r -> r+1 (and P-1 -> 0 for the next block) through device buffers -- the
    single-GPU parity vehicle of the multi-GPU block-cyclic partition.

    P = 1: the rank's nblk blocks in ONE launch (nw_fill_band_cycle_async chains
    them through its own halo buffer: the multi-block kernel path).  P > 1: one
    launch per block, enqueued in global block order on its rank's stream (the
    same kernel and halo regions; per-rank launches of all blocks need the P
    launches co-resident, which one process cannot promise: HIP maps its streams
    onto a few hardware queues, and rank 0 -- waiting on rank P-1 -- must not sit
    in front of it in one.  One process per GPU has no such limit: bench.py
    --share-gpu under torch.distributed.run rehearses that)."""

    def __init__(self, n1: int, n2: int, nranks: int, nblk: int, device: int = 0, substrips: int = 0,
                 strip_waves: int = 0):
        import torch
        self.n1, self.n2, self.P, self.m, self.device = n1, n2, nranks, nblk, device
        self.h = cycle_layout(n2, nranks, nblk)
        self.substrips, self.strip_waves = band_shape(n1, self.h, substrips, strip_waves)
        self.tables = [nwhip.Context.alloc_cycle_tables(n1, self.h, nblk) for _ in range(nranks)]
        self.halos = [nwhip.Halo(n1, device, regions=nblk) for _ in range(nranks)]
        self.ctxs = [nwhip.Context(device) for _ in range(nranks)]
        self.streams = [torch.cuda.Stream(device) for _ in range(nranks)]
        self.waves = max(1, resident_waves(device, self.substrips, self.strip_waves) // nranks)
        self.region = 8 * (n1 + 1)  # bytes per halo region (nw_halo_bytes)
        self.tag = 0

    def block(self, g: int):
        """(table of global block g, global row of its row 0)."""
        return self.tables[g % self.P][g // self.P], g * self.h

    def fill(self, d_s1, s2: np.ndarray, scheme=(1, 0, -1), flags: int = 0, timeout_ms: int = 0) -> int:
        """Fill every block; returns the final score t[n2][n1] (the last block's last cell)."""
        import torch
        assert int(d_s1.numel()) == self.n1 and s2.size == self.n2
        self.tag += 1
        P, m, h = self.P, self.m, self.h
        cur = torch.cuda.current_stream(self.device)
        sides = [torch.from_numpy(cycle_side_chars(s2, h, P, m, r)).cuda(self.device) for r in range(P)]
        for st in self.streams:
            st.wait_stream(cur)
        kw = dict(tag=self.tag, scheme=scheme, waves=self.waves, flags=flags, substrips=self.substrips,
                  strip_waves=self.strip_waves, timeout_ms=timeout_ms)
        if P == 1:
            self.ctxs[0].fill_band_cycle(d_s1, sides[0], h, self.tables[0], halo_in=self.halos[0].ptr,
                                         halo_out=self.halos[0].ptr, hin_first=False, hout_shift=1,
                                         row0_max=(m - 1) * h, stream=self.streams[0], **kw)
        else:
            for g in range(P * m):
                r, k = g % P, g // P
                nxt = (r + 1) % P  # block g + 1 lives on rank nxt, as its block k (or k + 1 after the wrap)
                kn = k + 1 if r == P - 1 else k
                self.ctxs[r].fill_band_cycle(
                    d_s1, sides[r][k * h:(k + 1) * h], h, self.tables[r][k:k + 1],
                    halo_in=self.halos[r].ptr + k * self.region, hin_first=g > 0,
                    halo_out=self.halos[nxt].ptr + kn * self.region if g + 1 < P * m else None,
                    hout_shift=0, row0_max=g * h, stream=self.streams[r], **kw)
        for r, st in enumerate(self.streams):
            s = self.ctxs[r].status(st)
            if s != nwhip.NW_OK:
                diag = [c.debug_ctrl() for c in self.ctxs]
                raise nwhip.NwError(s, f"cyclic bands, rank {r} (control words per rank: {diag})")
            cur.wait_stream(st)
        torch.cuda.synchronize(self.device)
        del sides
        return int(self.tables[P - 1][m - 1, h, self.n1].item())

    def close(self):
        for hb in self.halos:
            hb.free()
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


def _sweep(args, partition: str, rank: int, world: int, dev: int, scheme, blocks: int = 1) -> dict:
    """One multi-rank band sweep: `warmup` fills enqueued back to back, then `steps`
    timed fills EACH ALONE (barrier + synchronize around each; the per-fill latency
    of mpi-horz-driver.cpp:38-83, gathered by gather_fill_latencies), then `steps`
    more back to back (the pipelined throughput, reported separately).  Halo / feed
    buffers alternate by launch parity, the producer's stream waiting on the
    consumer's "done with launch k" link word (nw_link_*) before it rewrites that
    launch's buffer -- no host round trip between back-to-back launches.
    partition: "rows" (mpi-horz: contiguous row bands, or block-cyclic ones with
    args.band_blocks > 1 blocks per rank), "hrows" (the same bands in horizontal
    strips), "cols" (mpi-vert).  Returns this rank's measurements."""
    import torch
    import torch.distributed as dist

    cols = partition == "cols"
    hrows = partition == "hrows"  # row bands in horizontal strips (nw_fill_tband_async)
    kernel = getattr(args, "kernel", 0) if not hrows else nwhip.KERNEL_STRIPS
    m = max(1, blocks) if partition == "rows" else 1
    cyc = m > 1
    dense = False  # (horizontal strips: follower polls, tband_dense)
    ctx = nwhip.Context(dev)
    stream = torch.cuda.current_stream()
    h = 0
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
    elif cyc:
        # block-cyclic row bands: rank r owns blocks g = k * world + r of h rows
        n1, n2 = args.band_cols, world * args.band_rows
        h = cycle_layout(n2, world, m)
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(cycle_side_chars(nwhip.synth(2, n2), h, world, m, rank)).cuda()
        table = nwhip.Context.alloc_cycle_tables(n1, h, m)
        links_in = [nwhip.Halo(n1, dev, regions=m) for _ in range(2)]
        sub, nc = band_shape(n1, h, args.substrips, args.strip_waves)
        rows, start, ncols = h + 1, ((m - 1) * world + rank) * h, n1 + 1
    elif hrows:
        # row bands (mpi-horz, BASELINE config 4) swept in horizontal strips: the
        # halo is a feed of one granule per column
        n1 = args.band_cols
        n2 = world * args.band_rows
        rows, start = nwhip.band_layout(n2, world, rank)
        s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n2)[start:start + rows - 1].copy()).cuda()
        table = nwhip.Context.alloc_table(n1, rows - 1)
        links_in = [nwhip.Feed(n1, dev) for _ in range(2)] if rank > 0 else None
        sub, nc = tband_shape(args)
        dense = tband_dense(args, n2)
        ncols = n1 + 1
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
    # the chain: rank r feeds r+1 (and, block-cyclic, the last rank feeds rank 0's
    # next block).  Rank r exports its two incoming buffers and the link word its
    # consumer signals into; it maps its consumer's buffers and its producer's word.
    consumer = (rank + 1) % world if (rank + 1 < world or cyc) else None
    producer = (rank - 1) % world if (rank > 0 or cyc) else None
    link_word = nwhip.Link(dev) if consumer is not None else None
    mine = ([nwhip.ipc_get_handle(b.ptr) for b in links_in] if links_in else None,
            nwhip.ipc_get_handle(link_word.ptr) if link_word else None)
    handles = [None] * world
    dist.all_gather_object(handles, mine)
    out_bufs = [nwhip.ipc_open_handle(x) for x in handles[consumer][0]] if consumer is not None else None
    prod_word = nwhip.ipc_open_handle(handles[producer][1]) if producer is not None else None
    waves = args.waves
    if args.share_gpu and waves == 0:
        waves = max(1, resident_waves(dev, sub, nc, kernel) // world)
    # --debug-withhold-rank r: rank r publishes its boundary into a private buffer of
    # its own instead of its consumer's (the fail-fast test)
    withhold = getattr(args, "debug_withhold_rank", -1) == rank and out_bufs is not None
    if withhold:
        decoys = [nwhip.Feed(n2, dev) if cols else nwhip.Feed(n1, dev) if hrows else
                  nwhip.Halo(n1, dev, regions=m) for _ in range(2)]
    warm_tmo = int(getattr(args, "warmup_timeout_ms", 5000))
    clean = False
    try:
        preflight(rank, world, stream, links_in, out_bufs, link_word, prod_word)

        def launch(k: int, ev=None, timeout_ms: int = 0):
            """Launch k (tag k >= 1) on this rank's stream, buffers k % 2."""
            b = k % 2
            if out_bufs is not None and k >= 3:
                # consumer done with launch k-2; a wait that expires fails this context, so
                # launch k gives up instead of rewriting the buffer the consumer still reads
                nwhip.link_wait(link_word.ptr, k - 2, stream, timeout_ms=timeout_ms, ctx=ctx)
            if ev is not None:
                ev[0].record(stream)
            hout = (decoys[b].ptr if withhold else out_bufs[b]) if out_bufs is not None else None
            kw = dict(tag=k, scheme=scheme, waves=waves, stream=stream, substrips=sub, strip_waves=nc,
                      kernel=kernel, timeout_ms=timeout_ms)
            if cols:
                ctx.fill_colband(s1, s2, table, world, rank, feed_in=links_in[b].ptr if links_in else None,
                                 feed_out=hout, **kw)
            elif hrows:
                ctx.fill_tband(s1, s2, table, row0=start, feed_in=links_in[b].ptr if links_in else None,
                               feed_out=hout, tag=k, scheme=scheme, waves=waves, stream=stream,
                               timeout_ms=timeout_ms, substrips=sub, strip_waves=nc, dense_polls=dense)
            elif cyc:
                ctx.fill_band_cycle(s1, s2, h, table, halo_in=links_in[b].ptr, halo_out=hout,
                                    hin_first=rank > 0, hout_shift=int(rank == world - 1), row0_max=start, **kw)
            else:
                ctx.fill_band(s1, s2, table, halo_in=links_in[b].ptr if links_in else None,
                              halo_out=hout, row0=start, **kw)
            if ev is not None:
                ev[1].record(stream)
            if prod_word is not None:
                nwhip.link_signal(prod_word, k, stream)  # done reading launch k's buffer

        # warmup: every rank starts together (barrier) and every wait is bounded by
        # warm_tmo, so a halo / feed that never becomes visible (e.g. peer memory that
        # behaves differently across devices) fails the run in seconds, naming the band
        dist.barrier()
        for k in range(1, args.warmup + 1):
            launch(k, timeout_ms=warm_tmo)
        torch.cuda.synchronize()
        check_ranks(ctx, link_word, rank, world, f"{partition} warmup ({args.warmup} launches, "
                    f"{warm_tmo} ms bound)")
        # (1) per-fill latency, the reference's metric (mpi-horz-driver.cpp:38-83: the
        # earliest rank's start to the last rank's end of ONE fill): each timed fill
        # alone, every rank between a barrier + synchronize before it and a synchronize
        # after it, stamped on the host's CLOCK_MONOTONIC (one clock for every process
        # of the node); fill_latencies() takes min start -> max end over the ranks
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        stamps = []
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, e in enumerate(evs):
            dist.barrier()
            torch.cuda.synchronize()
            a = time.monotonic_ns()
            launch(args.warmup + 1 + i, e)
            torch.cuda.synchronize()
            stamps.append((a, time.monotonic_ns()))
        dist.barrier()
        wall = time.perf_counter() - t0
        # (2) the same fills back to back (link-word flow control only, no barrier
        # between them): fill k+1 runs on the upper bands while the lower ones still
        # finish fill k, so wall / steps is a THROUGHPUT -- per-fill time minus most of
        # the pipeline ramp -- reported separately as pipelined_ms_per_fill
        dist.barrier()
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for i in range(args.steps):
            launch(args.warmup + args.steps + 1 + i)
        torch.cuda.synchronize()
        dist.barrier()
        wall_pipe = time.perf_counter() - tp
        # any launch of the timed sweep that gave up (the record is sticky across launches)
        status = ctx.status()
        link_status = link_word.status() if link_word else 0
        failure = ctx.debug_failure() if status != nwhip.NW_OK else None
        kms = float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else 0.0
        fills = gather_fill_latencies(stamps, world)
        last = table[m - 1] if cyc else table
        score = int(last[rows - 1, ncols - 1].item()) if rank == world - 1 else None
        del last
        clean = True
    finally:
        # after a failure on any rank, leave at once (no collective: the ranks may
        # have failed at different points); torch.distributed.run then ends the
        # others, and the buffers go with the processes
        if not clean:
            print(f"rank {rank}: band sweep ({partition}) failed", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dist.barrier()
    if out_bufs:
        for x in out_bufs:
            nwhip.ipc_close_handle(x)
    if prod_word is not None:
        nwhip.ipc_close_handle(prod_word)
    dist.barrier()
    for x in (links_in or []) + ([link_word] if link_word else []) + (decoys if withhold else []):
        x.free()
    ctx.close()
    del table
    torch.cuda.empty_cache()
    return {"wall": wall, "wall_pipe": wall_pipe, "fills": fills, "status": status, "link_status": link_status,
            "failure": failure, "kms": kms, "score": score, "n1": n1, "n2": n2, "shape": [sub, nc], "kernel": kernel,
            "dense_polls": dense, "rows": rows,
            "start": start, "blocks": m, "block_rows": h}


def fill_latencies(stamps_per_rank) -> dict:
    """Per-fill latency as mpi-horz-driver.cpp:38-83 defines it: for each timed fill,
    the LATEST end over the ranks minus the EARLIEST start over the ranks.
    stamps_per_rank[r][k] = (start_ns, end_ns) of fill k on rank r (one host clock).
    Returns {"ms": [per fill], "start_skew_ms": [max - min start per fill]}."""
    nfill = len(stamps_per_rank[0])
    if any(len(s) != nfill for s in stamps_per_rank):
        raise ValueError("every rank must report the same number of fills")
    ms, skew = [], []
    for k in range(nfill):
        starts = [s[k][0] for s in stamps_per_rank]
        ends = [s[k][1] for s in stamps_per_rank]
        if any(e < a for a, e in zip(starts, ends)):
            raise ValueError(f"fill {k}: an end stamp precedes its start")
        ms.append((max(ends) - min(starts)) / 1e6)
        skew.append((max(starts) - min(starts)) / 1e6)
    return {"ms": ms, "start_skew_ms": skew}


def gather_fill_latencies(stamps, world: int) -> dict:
    """All-gather every rank's (start, end) stamps over the control plane and reduce
    them with fill_latencies (every rank gets the same answer)."""
    import torch.distributed as dist
    allst = [None] * world
    dist.all_gather_object(allst, [(int(a), int(b)) for a, b in stamps])
    return fill_latencies(allst)


CLOCK = "CLOCK_MONOTONIC (time.monotonic_ns), every rank on one host"


def same_host(hosts) -> bool:
    """True when every rank reported the same host name (fill_latencies compares
    CLOCK_MONOTONIC stamps across ranks, which is meaningful on one host only; the
    reference's epoch milliseconds, mpi-horz-driver.cpp:39-50, would need synchronised
    node clocks instead -- multi-node runs are out of scope)."""
    return len(set(hosts)) <= 1


def check_one_host(world: int) -> None:
    """All-gather the host names and refuse a multi-host world (see same_host)."""
    import socket
    import torch.distributed as dist
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname())
    if not same_host(hosts):
        raise RuntimeError(f"ranks span several hosts {sorted(set(hosts))}: the per-fill timing compares "
                           "CLOCK_MONOTONIC stamps across ranks and is single-node only")


PING = 0x5A5A0000  # pre-flight marker (never a launch tag: tags count launches from 1)


def preflight(rank: int, world: int, stream, links_in, out_bufs, link_word, prod_word, timeout_ms: int = 1000):
    """Before any fill: every producer stores one word into its consumer's incoming
    buffer (the halo / feed path, peer memory over xGMI) and every consumer stores
    one into its producer's link word (the flow-control path); each side polls its
    own copy with a `timeout_ms` bound (nw_link_wait).  A store that never becomes
    visible fails every rank at once, naming the pair, instead of the first fill
    waiting out its watchdog.  The marker words are cleared again before the
    barrier that precedes the first launch."""
    import torch
    import torch.distributed as dist
    dist.barrier()
    if out_bufs is not None:
        nwhip.link_signal(out_bufs[0], PING | 1, stream)       # granule 0, value word of consumer's buffer 0
    if prod_word is not None:
        nwhip.link_signal(prod_word + 8, PING | 2, stream)     # word 2 of the producer's link pair
    fails = []
    if links_in is not None:
        nwhip.link_wait(links_in[0].ptr, PING | 1, stream, timeout_ms=timeout_ms)
    if link_word is not None:
        nwhip.link_wait(link_word.ptr + 8, PING | 2, stream, timeout_ms=timeout_ms)
    torch.cuda.synchronize()
    if links_in is not None and nwhip.link_status_at(links_in[0].ptr) != 0:
        fails.append(f"rank {rank} never saw its producer's store into its incoming buffer")
    if link_word is not None and nwhip.link_status_at(link_word.ptr + 8) != 0:
        fails.append(f"rank {rank} never saw its consumer's store into its link word")
    # clear the markers (granule 0 back to {tag 0, value 0}; link words 2, 3)
    if links_in is not None:
        for w in (0, 4):
            nwhip.link_signal(links_in[0].ptr + w, 0, stream)
    if link_word is not None:
        for w in (8, 12):
            nwhip.link_signal(link_word.ptr + w, 0, stream)
    torch.cuda.synchronize()
    allf = [None] * world
    dist.all_gather_object(allf, fails)
    bad = [f for fs in allf for f in fs]
    if bad:
        raise RuntimeError(f"pre-flight peer-store check failed ({timeout_ms} ms bound): " + "; ".join(bad))
    dist.barrier()


def check_ranks(ctx, link_word, rank: int, world: int, what: str) -> None:
    """Every rank's fill status (sticky over the launches since the last check) and
    link status, gathered; raise on every rank if any failed, naming the band, the
    watchdog site and the recorded words."""
    import torch.distributed as dist
    st = ctx.status()
    ls = link_word.status() if link_word else 0
    mine = None
    if st != nwhip.NW_OK or ls != 0:
        code, site, need, seen, nfail = ctx.debug_failure()
        mine = {"rank": rank, "status": nwhip.strerror(st) if st else "ok", "link_status": ls,
                "code": code, "site": site >> 24, "wave": (site >> 16) & 0xFF, "need": need, "seen": seen,
                "failed_launches": nfail, "debug_ctrl": ctx.debug_ctrl()}
    allm = [None] * world
    dist.all_gather_object(allm, mine)
    bad = [m for m in allm if m is not None]
    if bad:
        raise RuntimeError(f"band fill failed during the {what}: " + "; ".join(
            f"band {m['rank']}: {m['status']}, code {m['code']} (1 granule / finisher look-back, 2 halo, 3 LDS counter, 4 link wait) "
            f"at site {m['site']} wave {m['wave']}, needed {m['need']} saw {m['seen']}, "
            f"{m['failed_launches']} failed launches, link status {m['link_status']}, debug_ctrl {m['debug_ctrl']}"
            for m in bad))


# Block-cyclic row bands on one GPU's share of config 4 (524288 x 65536), one launch
# of m chained blocks against the plain fill (tools/cycle_time.py, profiles/
# r03p_cycle_time.txt): m = 1 32.3 ms, 2 41.1, 4 58.2, 8 110.1.  Strips are claimed
# in (block, strip) order and a block's strips start one hop (64 * NC rows of the
# anti-diagonal skew + the hand-off, ~6.5 us for (4, 1)) apart, so a block of h
# rows keeps only ~h * pace / hop strips busy: short blocks starve the workers.
# The multi-GPU model therefore keeps contiguous bands as the
# main leg and measures 2 blocks per GPU (the only count the model finds no worse)
# as an alternate.
CYCLE_ALT_BLOCKS = 2


# Follower polls of the horizontal sweep (NW_TBAND_DENSE_POLLS; DESIGN.md section 5,
# profiles/r06l_poll_sleep.txt, r06n_lead_dense.txt): s_sleep 1 polls (which need no leader
# throttle) give a mean strip-to-strip lag of 10.0 us at a leader of 28.0-28.5 ms, against
# 12.2-12.5 us at 26.8-27.2 ms for s_sleep 64 with the throttled leader: they pay for chains
# longer than the break-even of ~1.25 ms / 2.4 us = ~520 strips of 256 rows -- from N = 2
# (512 strips: even) on; a band alone (256 strips) keeps sparse polls.
DENSE_POLL_STRIPS = 512


def tband_dense(args, n2: int) -> bool:
    """Dense polls for a horizontal sweep of n2 rows in all: --tband-polls dense / sparse, or
    auto (the default) = the chain of n2 / 256 strips is at least DENSE_POLL_STRIPS long."""
    v = getattr(args, "tband_polls", None) or "auto"
    if v not in ("auto", "dense", "sparse"):
        raise ValueError(f"--tband-polls {v}: auto, dense or sparse")
    if v != "auto":
        return v == "dense"
    return n2 // HSTRIP_ROWS >= DENSE_POLL_STRIPS


# Strip shape of the horizontal sweep (nw_fill_tband_async): (4, 1) or (2, 2), both
# 256 rows; bench.py --tband-shape overrides it.
TBAND_SHAPE = (4, 1)


def tband_shape(args) -> tuple:
    """(C, NC) of the horizontal-strip row bands: --tband-shape "C,NC" or TBAND_SHAPE."""
    v = getattr(args, "tband_shape", None)
    if not v:
        return TBAND_SHAPE
    c, nc = (int(x) for x in str(v).split(","))
    if (c, nc) not in ((4, 1), (2, 2)):
        raise ValueError(f"--tband-shape {v}: horizontal strips take (4, 1) or (2, 2)")
    return c, nc


# A horizontal sweep runs its strips side by side along the whole width: a band of
# fewer than 256 strips of 256 rows leaves CUs idle for the full n1-column sweep
# (2 ranks sharing one GPU with 16384-row bands: 32.0 ms against 19.8 for the
# vertical sweep, profiles/r03h_share2_bench.json).
HSTRIP_ROWS, HSTRIP_CUS = 256, 256


def legs_for(args) -> list:
    """[(name, partition, blocks per rank)] of a multi-GPU bench: the main one
    first (its value is the line's), then the alternates (--alt-partition).
    Row bands (BASELINE config 4, mpi-horz's contiguous partition) are swept in
    horizontal strips by default (--band-sweep auto): band r+1's first strip trails
    band r's last strip by a strip hop.  The vertical sweep of the same bands (band
    r+1's strip k starts when band r's strip k reaches its last row), the
    block-cyclic rows and the column bands run as alternates."""
    main = getattr(args, "partition", "rows")
    kernel = getattr(args, "kernel", 0)
    m = max(1, getattr(args, "band_blocks", 1))
    if kernel == nwhip.KERNEL_PANELS:
        m = 1  # (no block-cyclic launch for the panel kernel)
    horiz_ok = kernel != nwhip.KERNEL_PANELS  # (horizontal strips: the (4, 1) strip kernel)
    sweep = getattr(args, "band_sweep", "auto")
    if sweep == "auto":
        # horizontal: band r+1's first strip trails band r's last strip by one hop,
        # so the node's step is one strip sweep + 256 N - 1 hops (DESIGN.md section 5,
        # measured inputs, profiles/r04f_*: N = 8 modelled at ~53 ms against ~74-80 ms
        # for the vertical sweep, whose bands wait for the band above's strips to reach
        # its last row).  At N = 2 both measure alike: 2 bands of 524288 x 32768 on one
        # GPU 31.4 ms horizontal / 30.7 vertical (one process), 37.8 / 36.8 ms in two
        # processes sharing it.  (Round 3's horizontal sweep ran the last band's leftover
        # row as a second full pass and published the band's last row from the compute
        # wave; the row-scan finisher and the store-wave publish fixed both.)
        sweep = "horizontal" if horiz_ok else "vertical"
    horiz = horiz_ok and sweep == "horizontal"
    rows_h = ("rows_horizontal", "hrows", 1)
    rows_v = ("rows_contiguous", "rows", 1)
    rows_main = ("rows_cyclic", "rows", m) if m > 1 else rows_h if horiz else rows_v
    legs = [rows_main] if main == "rows" else [("cols", "cols", 1)]
    alt = getattr(args, "alt_partition", None)
    if alt == "none":
        return legs
    cyc_ok = kernel != nwhip.KERNEL_PANELS and args.band_rows % CYCLE_ALT_BLOCKS == 0
    if main == "rows":
        if alt in (None, "rows"):
            cands = ([rows_h] if horiz_ok else []) + [rows_v]
            if cyc_ok and args.band_rows >= 65536:
                cands.append(("rows_cyclic", "rows", CYCLE_ALT_BLOCKS))
            legs += [c for c in cands if c[0] != rows_main[0]]
        if alt in (None, "cols"):
            legs.append(("cols", "cols", 1))
    elif alt in (None, "rows"):
        legs.append(rows_main)
    return legs


def run_bands(args) -> dict | None:
    """bench.py --gpus N (N > 1) under torch.distributed.run: one rank per GPU.
    `value` = row bands (BASELINE config 4: an n1 x (N * band_rows) table, weak
    scaling, 512k x 512k at N = 8 with the defaults), contiguous as mpi-horz lays
    them out (or block-cyclic with --band-blocks m > 1); block-cyclic rows with
    CYCLE_ALT_BLOCKS blocks per rank and the column bands (mpi-vert, N * col_width
    columns x col_rows rows) run after it as `alt_partitions` unless
    --alt-partition none.  Prints and returns the JSON line on rank 0."""
    import torch
    import torch.distributed as dist

    rank, world = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1)
    local = _env_int("LOCAL_RANK", rank)
    if world != args.gpus:
        raise RuntimeError(f"run_bands: WORLD_SIZE={world} but --gpus {args.gpus} (bench.py refuses this)")
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise RuntimeError("run_bands needs a GPU (there is no CPU fallback)")
    if not args.share_gpu and ndev < world:
        raise RuntimeError(f"run_bands: {world} ranks but {ndev} visible GPU(s) and no --share-gpu")
    dev = 0 if args.share_gpu else local % ndev
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        # a bounded control plane: a rank that dies leaves the others' collectives
        # failing within minutes rather than gloo's default half hour
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    check_one_host(world)
    scheme = tuple(int(x) for x in args.scheme.split(","))
    legs = {}
    plan_ = legs_for(args)
    for name, part, m in plan_:
        r = _sweep(args, part, rank, world, dev, scheme, m)
        allm = [None] * world
        dist.all_gather_object(allm, r)
        legs[name] = (part, allm)
    if rank != 0:
        return None
    name0 = plan_[0][0]
    out = _line(args, world, scheme, *legs[name0])
    alts = {}
    for name, _, _ in plan_[1:]:
        a = _line(args, world, scheme, *legs[name])
        alts[name] = {k: a[k] for k in ("value", "ms_per_step", "per_fill_ms", "pipelined_ms_per_fill",
                                        "pipelined_value", "config", "score", "score_golden", "score_ok",
                                        "roofline")}
    if alts:
        out["alt_partitions"] = alts
        rows_legs = [out["score"]] + [alts[k]["score"] for k in ("rows_horizontal", "rows_cyclic", "rows_contiguous")
                                      if k in alts]
        if plan_[0][1] in ("rows", "hrows"):  # the same table under every row partition
            out["rows_legs_agree"] = len(set(rows_legs)) == 1 if len(rows_legs) > 1 else None
    # no value is published from a sweep whose watchdog or flow control tripped in
    # any launch (the fill status is sticky over the launches of a sweep)
    bad = [(p, [m["status"] for m in ms], [m["link_status"] for m in ms], [m["failure"] for m in ms])
           for p, (_, ms) in legs.items() if any(m["status"] != 0 or m["link_status"] != 0 for m in ms)]
    if bad:
        raise RuntimeError(f"band status per rank (fill, link, first failure [code, site, need, seen, "
                           f"launches]): {bad}")
    if cpu_baseline_fn is not None and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_fn(args.cpu_n, scheme)
    print(json.dumps(out), flush=True)
    return out


cpu_baseline_fn = None  # bench.py installs its cpu_baseline (rank 0 only reports it)


def band_traffic(n1: int, rows: int, sweep: str):
    """HBM bytes per launch of one GPU's row-band kernel (WRITE_SIZE + 2 x FETCH_SIZE)
    from the committed rocprofv3 PMC record of that band filled alone on one GPU
    (profiles/pmc_traffic.json, tools/profile_lease.sh: config 4's last band, 65538 x
    524289), and where it came from; (None, None) for a geometry without a record."""
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    key = f"nw_fill_rowband_{rows}x{n1 + 1}:{sweep}"
    e = d.get(key)
    if not e:
        return None, None
    return e["hbm_bytes_per_launch"], (f"profiles/pmc_traffic.json [{key}], {e.get('round', '?')} "
                                       f"{e.get('date', '')}: the band filled alone on one GPU, its kernel's "
                                       f"WRITE_SIZE + 2 x FETCH_SIZE")


def _line(args, world: int, scheme, part: str, ms: list) -> dict:
    """The bench JSON line of one partition from every rank's _sweep result."""
    cols = part == "cols"
    m0, ml = ms[0], ms[-1]
    n1, n2 = m0["n1"], m0["n2"]
    wall_s = max(m["wall"] for m in ms)  # max over ranks (the per-fill region, barriers included)
    pipe_s = max(m["wall_pipe"] for m in ms)
    fills = m0["fills"]  # the same on every rank (gather_fill_latencies)
    score = ml["score"]
    want = _golden(n1, n2, scheme)
    cells = n1 * n2
    # `value` / `ms_per_step`: the mean per-fill latency (earliest start -> latest end
    # over the ranks, each fill alone: mpi-horz-driver.cpp:38-83), NOT the back-to-back
    # throughput, which hides most of the pipeline ramp (pipelined_ms_per_fill)
    ms_step = float(np.mean(fills["ms"]))
    value = cells / (ms_step * 1e-3) / 1e9
    pipe_ms = pipe_s / args.steps * 1e3
    table_bytes = 4.0 * (n1 + 1) * (n2 + 1)
    per_gpu_bytes = table_bytes / world
    achieved = per_gpu_bytes / (ms_step * 1e6)  # GB/s per GPU over one whole fill (incl. pipeline ramp)
    kern = {0: "auto", 1: "strips", 2: "panels"}[m0["kernel"]]
    # per-GPU HBM traffic of the largest band (the last one) where a PMC record exists
    traffic, traffic_src = (band_traffic(n1, ml["rows"], "horizontal" if part == "hrows" else "vertical")
                            if part in ("rows", "hrows") and ml["blocks"] == 1 else (None, None))
    common = {"n1": n1, "n2": n2, "scheme": list(scheme), "bands": world, "table_bytes": int(table_bytes),
              "kernel": kern, "shape": m0["shape"], "control_plane": "torch.distributed gloo (setup, barriers)",
              "launches": "buffers by launch parity, link-word flow control (nw_link_*); timed fills one at a time, "
                           "then back to back for pipelined_ms_per_fill",
              "shared_gpu": bool(args.share_gpu)}
    if cols:
        cfg = {"workload": f"nw_fill_colbands_{n2}x{n1}", "col_width": args.col_width,
               "parallelism": f"column bands x{world} (mpi-vert)",
               "halo": "in-kernel xGMI peer stores of the band's right column, 16 rows at a time", **common}
    elif part == "hrows":
        cfg = {"workload": f"nw_fill_rowbands_{n2}x{n1}", "band_rows": args.band_rows,
               "parallelism": f"row bands x{world}, contiguous (mpi-horz, BASELINE config 4), each band swept in "
                              "horizontal strips of 256 rows (nw_fill_tband_async)",
               "halo": "in-kernel xGMI peer stores of the band's last row, 16 columns at a time, as the band's "
                       "last strip produces it",
               "polls": ("dense (s_sleep 1)" if m0.get("dense_polls") else "sparse (s_sleep 64)") +
                        ", the chain's leader throttled",
               **common}
    elif m0["blocks"] > 1:
        cfg = {"workload": f"nw_fill_rowbands_{n2}x{n1}", "band_rows": args.band_rows,
               "blocks_per_gpu": m0["blocks"], "block_rows": m0["block_rows"],
               "parallelism": f"row bands x{world}, block-cyclic: {m0['blocks']} blocks of {m0['block_rows']} rows "
                              f"per GPU, block g on GPU g mod {world} (mpi-horz halo contract per block, "
                              "BASELINE config 4)",
               "halo": "in-kernel xGMI peer stores of each block's last row into the next GPU's halo region, "
                       "as each strip finishes (the last GPU feeds GPU 0's next block)",
               **common}
    else:
        cfg = {"workload": f"nw_fill_rowbands_{n2}x{n1}", "band_rows": args.band_rows,
               "parallelism": f"row bands x{world}, contiguous (mpi-horz, BASELINE config 4)",
               "halo": "in-kernel xGMI peer stores of the band's last row, as each strip/panel finishes",
               **common}
    return {
        "metric": "GCUPS (DP cell updates/s) on NxN NW fill, bit-exact score",
        "value": round(value, 2),
        "unit": "GCUPS",
        "n_gpus": world,
        "requested_gpus": args.gpus,
        "launcher": os.environ.get("NW_BENCH_LAUNCHER", "external"),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "timing": "per fill: each timed fill alone (barrier + synchronize around it), earliest rank start -> "
                  "latest rank end on the host's CLOCK_MONOTONIC (mpi-horz-driver.cpp:38-83); value = cells / "
                  "mean per-fill time",
        "clock": CLOCK,
        "per_fill_ms": [round(x, 3) for x in fills["ms"]],
        "start_skew_ms_max": round(max(fills["start_skew_ms"]), 3),
        "timed_region_ms_per_step": round(wall_s / args.steps * 1e3, 3),
        "pipelined_ms_per_fill": round(pipe_ms, 3),
        "pipelined_value": round(cells / (pipe_ms * 1e-3) / 1e9, 2),
        "pipelined_note": "the same fills enqueued back to back (link-word flow control only): the upper bands "
                          "start fill k+1 while the lower ones finish fill k, so this is a throughput that hides "
                          "most of the pipeline ramp -- not the reference's metric",
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
                     "traffic": traffic, "traffic_source": traffic_src,
                     "basis": "per GPU: band table bytes / ms_per_step (one whole fill, pipeline ramp included)",
                     "kernel_ms_avg_per_rank": [round(m["kms"], 3) for m in ms]},
        "cpu_baseline": None,
        "kernel": nwhip.version(),
    }
