"""ctypes binding of libnwhip.so (include/nw_hip.h) -- the MI355X NW fill.

This is the Python-side mirror of the reference's fill plugin interface
(`needlemanWunsch(dnaArray s1, dnaArray s2, int* t)`, src/serial/serial.cpp:4):
`fill(s1, s2)` returns the full (n2+1) x (n1+1) int32 table in the reference
layout, `score(s1, s2)` only t[n2][n1] (what src/common/driver.cpp:35 prints).
Device-resident variants take torch tensors and never leave HBM.

There is no CPU fallback: if build/libnwhip.so is missing or no gfx950 device is
visible, every call raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NWHIP_LIB selects an alternative in-tree build (tuning variants from `make variant`)
LIB_PATH = os.environ.get("NWHIP_LIB") or os.path.join(HERE, "build", "libnwhip.so")

NW_OK, NW_ERR_ARG, NW_ERR_HIP, NW_ERR_OOM, NW_ERR_TIMEOUT, NW_ERR_NODEVICE, NW_ERR_UNSUPPORTED = range(7)
MODE_NW, MODE_SW = 0, 1  # nw_params.mode: global (the reference fills) / Smith-Waterman local
# nw_params.kernel: auto / anti-diagonal strips (nw_fill.hip) / row-scan panels (nw_rows.hip)
KERNEL_AUTO, KERNEL_STRIPS, KERNEL_PANELS = 0, 1, 2

# every symbol include/nw_hip.h declares (checked by tests/test_host.py)
EXPORTS = ["nw_params_default", "nw_strerror", "nw_version", "nw_fill", "nw_table_pitch",
           "nw_table_bytes", "nw_table_offset", "nw_strip_lds_bytes", "nw_panel_lds_bytes", "nw_ctx_create", "nw_ctx_destroy", "nw_ctx_workspace_bytes",
           "nw_fill_device", "nw_fill_device_async", "nw_ctx_status", "nw_read_bdna", "nw_free",
           "nw_synth_bdna", "nw_band_layout", "nw_halo_bytes", "nw_fill_band_async",
           "nw_ipc_get_handle", "nw_ipc_open_handle", "nw_ipc_close_handle", "nw_halo_alloc",
           "nw_halo_free", "nw_fill_emb", "nw_sw_align", "nw_sw_traceback", "nw_tuned_shape", "nw_auto_shape", "nw_debug_ctrl", "nw_debug_set_trace",
           "nw_debug_trace_words", "nw_colband_layout", "nw_feed_bytes", "nw_feed_alloc",
           "nw_fill_colband_async", "nw_link_alloc", "nw_link_wait_async", "nw_link_signal_async",
           "nw_link_status", "nw_host_warmup", "nw_host_release", "nw_halo_alloc_regions",
           "nw_fill_band_cycle_async", "nw_fill_tband_async", "nw_link_wait_ctx_async", "nw_debug_failure"]
IPC_HANDLE_BYTES = 64


class NwParams(ctypes.Structure):
    _fields_ = [("match", ctypes.c_int32), ("mismatch", ctypes.c_int32), ("gap", ctypes.c_int32),
                ("mode", ctypes.c_int32), ("waves", ctypes.c_int32), ("device", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("substrips", ctypes.c_int32),
                ("strip_waves", ctypes.c_int32), ("timeout_ms", ctypes.c_int32),
                ("kernel", ctypes.c_int32)]


class NwResult(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int32), ("status", ctypes.c_int32), ("cells", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("table_bytes", ctypes.c_double),
                ("strips", ctypes.c_int32), ("waves", ctypes.c_int32),
                ("substrips", ctypes.c_int32), ("strip_waves", ctypes.c_int32),
                ("end_i", ctypes.c_int64), ("end_j", ctypes.c_int64),
                ("kernel", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class NwAlignment(ctypes.Structure):
    """nw_alignment (include/nw_hip.h): a Smith-Waterman alignment."""
    _fields_ = [("score", ctypes.c_int32), ("status", ctypes.c_int32), ("begin_i", ctypes.c_int64),
                ("begin_j", ctypes.c_int64), ("end_i", ctypes.c_int64), ("end_j", ctypes.c_int64),
                ("n_ops", ctypes.c_int64), ("fill_ms", ctypes.c_double), ("traceback_ms", ctypes.c_double)]


class NwBand(ctypes.Structure):
    """nw_band (include/nw_hip.h): halo granule buffers of one row band."""
    _fields_ = [("halo_in", ctypes.c_void_p), ("halo_out", ctypes.c_void_p),
                ("tag", ctypes.c_uint32), ("row0", ctypes.c_uint32)]


class NwBandCycle(ctypes.Structure):
    """nw_band_cycle (include/nw_hip.h): one rank's blocks of block-cyclic row bands."""
    _fields_ = [("halo_in", ctypes.c_void_p), ("halo_out", ctypes.c_void_p), ("nblk", ctypes.c_int32),
                ("hin_first", ctypes.c_int32), ("hout_shift", ctypes.c_int32), ("tag", ctypes.c_uint32),
                ("row0_max", ctypes.c_int64), ("t_stride", ctypes.c_int64)]


class NwColBand(ctypes.Structure):
    """nw_colband (include/nw_hip.h): feed granule buffers of one column band."""
    _fields_ = [("feed_in", ctypes.c_void_p), ("feed_out", ctypes.c_void_p), ("tag", ctypes.c_uint32),
                ("nbands", ctypes.c_int32), ("r", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class NwTBand(ctypes.Structure):
    """nw_tband (include/nw_hip.h): feed granule buffers of one row band in horizontal strips."""
    _fields_ = [("feed_in", ctypes.c_void_p), ("feed_out", ctypes.c_void_p), ("tag", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("row0", ctypes.c_int64)]


TBAND_DENSE_POLLS = 1  # nw_tband.flags NW_TBAND_DENSE_POLLS


class NwError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"libnwhip {what}: {strerror(status)} ({status})")


_lib = None
_i8p = ctypes.POINTER(ctypes.c_int8)
_i32p = ctypes.POINTER(ctypes.c_int32)


def lib() -> ctypes.CDLL:
    """Load build/libnwhip.so (raises if it has not been built).

    torch (when installed) is imported first: torch and libnwhip share one HIP
    runtime (libamdhip64.so.7, deduplicated by SONAME), and torch must be the one
    that loads it or its own device initialisation fails."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C fast-needleman-wunsch_amd` "
                                "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.nw_params_default.argtypes = [ctypes.POINTER(NwParams)]
    L.nw_params_default.restype = None
    L.nw_strerror.argtypes = [ctypes.c_int]
    L.nw_strerror.restype = ctypes.c_char_p
    L.nw_version.restype = ctypes.c_char_p
    L.nw_fill.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.POINTER(NwParams),
                          _i32p, ctypes.POINTER(NwResult)]
    L.nw_fill_emb.argtypes = L.nw_fill.argtypes
    _u8p = ctypes.POINTER(ctypes.c_uint8)
    L.nw_sw_align.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.POINTER(NwParams), _u8p,
                              ctypes.c_int64, ctypes.POINTER(NwAlignment)]
    L.nw_sw_traceback.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                  ctypes.c_int64, ctypes.POINTER(NwParams), ctypes.c_void_p, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_int64, _u8p, ctypes.c_int64,
                                  ctypes.POINTER(NwAlignment)]
    L.nw_table_pitch.argtypes = [ctypes.c_int64]
    L.nw_table_pitch.restype = ctypes.c_int64
    L.nw_table_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.nw_table_bytes.restype = ctypes.c_int64
    L.nw_table_offset.argtypes = []
    L.nw_table_offset.restype = ctypes.c_int64
    L.nw_strip_lds_bytes.argtypes = [ctypes.c_int32, ctypes.c_int32]
    L.nw_strip_lds_bytes.restype = ctypes.c_int64
    L.nw_panel_lds_bytes.argtypes = [ctypes.c_int32, ctypes.c_int32]
    L.nw_panel_lds_bytes.restype = ctypes.c_int64
    L.nw_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_ctx_destroy.argtypes = [ctypes.c_void_p]
    L.nw_ctx_destroy.restype = None
    L.nw_ctx_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]
    L.nw_ctx_workspace_bytes.restype = ctypes.c_int64
    dev_args = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                ctypes.POINTER(NwParams), ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.nw_fill_device.argtypes = dev_args + [ctypes.POINTER(NwResult)]
    L.nw_fill_device_async.argtypes = dev_args
    L.nw_ctx_status.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.nw_read_bdna.argtypes = [ctypes.c_char_p, ctypes.POINTER(_i8p), ctypes.POINTER(ctypes.c_int64)]
    L.nw_free.argtypes = [ctypes.c_void_p]
    L.nw_free.restype = None
    L.nw_synth_bdna.argtypes = [ctypes.c_uint64, ctypes.c_int64, _i8p]
    L.nw_synth_bdna.restype = None
    L.nw_band_layout.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.nw_band_layout.restype = None
    L.nw_halo_bytes.argtypes = [ctypes.c_int64]
    L.nw_halo_bytes.restype = ctypes.c_int64
    L.nw_fill_band_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(NwParams),
                                     ctypes.POINTER(NwBand), ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_void_p]
    L.nw_ipc_get_handle.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.nw_ipc_open_handle.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_ipc_close_handle.argtypes = [ctypes.c_void_p]
    L.nw_halo_alloc.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_halo_free.argtypes = [ctypes.c_void_p]
    L.nw_halo_alloc_regions.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_fill_band_cycle_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.POINTER(NwParams), ctypes.POINTER(NwBandCycle),
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.nw_tuned_shape.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int32)]
    L.nw_tuned_shape.restype = None
    L.nw_auto_shape.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    L.nw_auto_shape.restype = None
    _i64p = ctypes.POINTER(ctypes.c_int64)
    L.nw_colband_layout.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(NwParams), _i64p, _i64p, _i64p, _i64p]
    L.nw_feed_bytes.argtypes = [ctypes.c_int64]
    L.nw_feed_bytes.restype = ctypes.c_int64
    L.nw_feed_alloc.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_fill_colband_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_int64, ctypes.POINTER(NwParams), ctypes.POINTER(NwColBand),
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.nw_fill_tband_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.POINTER(NwParams), ctypes.POINTER(NwTBand),
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.nw_link_alloc.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.nw_link_wait_async.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]
    L.nw_link_wait_ctx_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32,
                                         ctypes.c_void_p]
    L.nw_debug_failure.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    L.nw_link_signal_async.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.nw_link_status.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    L.nw_host_warmup.argtypes = [ctypes.c_int]
    L.nw_host_release.argtypes = [ctypes.c_int]
    L.nw_host_release.restype = None
    L.nw_debug_ctrl.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    L.nw_debug_set_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.nw_debug_trace_words.argtypes = []
    L.nw_debug_trace_words.restype = ctypes.c_int32
    _lib = L
    return L


def strerror(status: int) -> str:
    try:
        return lib().nw_strerror(status).decode()
    except FileNotFoundError:
        return str(status)


def version() -> str:
    return lib().nw_version().decode()


@dataclass
class Scheme:
    """Runtime replacement of needleman-wunsch.hpp:11-13 (MATCH, MISMATCH, GAP)."""
    match: int = 1
    mismatch: int = 0
    gap: int = -1


def params(scheme=(1, 0, -1), waves: int = 0, device: int = -1, flags: int = 0,
           substrips: int = 0, strip_waves: int = 0, timeout_ms: int = 0, mode: int = MODE_NW,
           kernel: int = KERNEL_AUTO) -> NwParams:
    if isinstance(scheme, Scheme):
        scheme = (scheme.match, scheme.mismatch, scheme.gap)
    p = NwParams()
    lib().nw_params_default(ctypes.byref(p))
    p.match, p.mismatch, p.gap = (int(x) for x in scheme)
    p.waves = int(waves)
    p.device = int(device)
    p.flags = int(flags)
    p.substrips = int(substrips)
    p.strip_waves = int(strip_waves)
    p.timeout_ms = int(timeout_ms)
    p.mode = int(mode)
    p.kernel = int(kernel)
    return p


def sw_align(s1, s2, scheme=(1, -1, -1), device: int = -1, substrips: int = 0, strip_waves: int = 0,
             kernel: int = KERNEL_AUTO):
    """Smith-Waterman local alignment on the device (nw_sw_align): returns
    (NwAlignment, ops) with ops a uint8 array in path order (0 diag, 1 up, 2 left)."""
    a, b = _seq(s1), _seq(s2)
    ops = np.empty(a.size + b.size + 1, dtype=np.uint8)
    out = NwAlignment()
    p = params(scheme, device=device, substrips=substrips, strip_waves=strip_waves, mode=MODE_SW, kernel=kernel)
    st = lib().nw_sw_align(a.ctypes.data_as(_i8p), a.size, b.ctypes.data_as(_i8p), b.size, ctypes.byref(p),
                           ops.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ops.size, ctypes.byref(out))
    if st != NW_OK:
        raise NwError(st, "nw_sw_align")
    return out, ops[:out.n_ops].copy()


def _seq(s) -> np.ndarray:
    if isinstance(s, (bytes, bytearray)):
        return np.frombuffer(bytes(s), dtype=np.int8).copy()
    return np.ascontiguousarray(np.asarray(s, dtype=np.int8))


FLAG_TIMING_ONLY, FLAG_NO_PROFILE, FLAG_NO_FINISH = 1, 2, 4  # nw_params.flags (include/nw_hip.h)
FLAG_DEBUG_DRAIN, FLAG_DEBUG_NO_STORE = 0x100, 0x200  # compute-pace probes, with FLAG_TIMING_ONLY only
FLAG_DEBUG_NO_CHAIN = 0x400  # store-pattern probe: strips unchained, HBM stores kept, no fill
FLAG_DEBUG_STAGGER = 0x800   # with NO_CHAIN: strip p starts p * 11.5 us after its claim


def fill(s1, s2, scheme=(1, 0, -1), waves: int = 0, device: int = -1, substrips: int = 0,
         flags: int = 0, strip_waves: int = 0, kernel: int = KERNEL_AUTO):
    """Full table in the reference layout ((n2+1) x (n1+1) int32) + NwResult."""
    a, b = _seq(s1), _seq(s2)
    t = np.empty((b.size + 1, a.size + 1), dtype=np.int32)
    r = NwResult()
    p = params(scheme, waves, device, flags=flags, substrips=substrips, strip_waves=strip_waves, kernel=kernel)
    st = lib().nw_fill(a.ctypes.data_as(_i8p), a.size, b.ctypes.data_as(_i8p), b.size,
                       ctypes.byref(p), t.ctypes.data_as(_i32p), ctypes.byref(r))
    if st != NW_OK:
        raise NwError(st, "nw_fill")
    return t, r


def score(s1, s2, scheme=(1, 0, -1), waves: int = 0, device: int = -1, substrips: int = 0,
          strip_waves: int = 0, kernel: int = KERNEL_AUTO) -> int:
    a, b = _seq(s1), _seq(s2)
    r = NwResult()
    p = params(scheme, waves, device, substrips=substrips, strip_waves=strip_waves, kernel=kernel)
    st = lib().nw_fill(a.ctypes.data_as(_i8p), a.size, b.ctypes.data_as(_i8p), b.size,
                       ctypes.byref(p), None, ctypes.byref(r))
    if st != NW_OK:
        raise NwError(st, "nw_fill")
    return int(r.score)


def host_release(device: int = -1) -> None:
    """Free the per-device state of the host-buffer calls (nw_host_release)."""
    lib().nw_host_release(device)


def trace_words() -> int:
    """uint64 words per strip of the debug trace (nw_debug_trace_words)."""
    return int(lib().nw_debug_trace_words())


def table_pitch(n1: int) -> int:
    return int(lib().nw_table_pitch(n1))


def table_rows(n2: int) -> int:
    return (n2 + 1 + 63) // 64 * 64


def table_offset() -> int:
    """Element offset of the table base from a 256-byte aligned allocation that
    puts column 1 on a 256-byte line (nw_table_offset)."""
    return int(lib().nw_table_offset())


def tuned_shape(n1: int, n2: int) -> tuple[int, int]:
    """(C, NC) an auto-shaped fill of an n1 x n2 table uses (nw_tuned_shape)."""
    c, nc = ctypes.c_int32(), ctypes.c_int32()
    lib().nw_tuned_shape(n1, n2, ctypes.byref(c), ctypes.byref(nc))
    return int(c.value), int(nc.value)


def auto_shape(n1: int, n2: int, cus: int = 256) -> tuple[int, int, int]:
    """(kernel, C, NC) a global fill with kernel = substrips = strip_waves = 0 uses
    for an n1 x n2 table on a device of `cus` CUs (nw_auto_shape)."""
    k, c, nc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    lib().nw_auto_shape(n1, n2, cus, ctypes.byref(k), ctypes.byref(c), ctypes.byref(nc))
    return int(k.value), int(c.value), int(nc.value)


def strip_shape(substrips: int = 0, strip_waves: int = 0, n1: int = -1, n2: int = -1) -> tuple[int, int]:
    """(C, NC) the library uses for these nw_params values (0 = auto), as
    make_shape in nw_capi.cpp: auto = the tuned shape for the table size (n1, n2;
    (2, 2) when no size is given); C alone implies 256-column strips."""
    if substrips <= 0 and strip_waves <= 0:
        return tuned_shape(n1, n2) if n1 >= 0 and n2 >= 0 else (2, 2)
    c = substrips if substrips > 0 else 2
    if strip_waves > 0:
        return c, strip_waves
    return c, {1: 4, 2: 2, 4: 1}[c]


def strip_lds_bytes(substrips: int, strip_waves: int) -> int:
    """LDS bytes of one strip workgroup of this shape (-1: unsupported shape)."""
    return int(lib().nw_strip_lds_bytes(substrips, strip_waves))


def panel_lds_bytes(substrips: int, strip_waves: int) -> int:
    """LDS bytes of one panel workgroup of this shape (-1: unsupported shape)."""
    return int(lib().nw_panel_lds_bytes(substrips, strip_waves))


def read_bdna(path: str) -> np.ndarray:
    """readSequence semantics (src/common/helper.cpp:3-25)."""
    buf = _i8p()
    n = ctypes.c_int64()
    st = lib().nw_read_bdna(path.encode(), ctypes.byref(buf), ctypes.byref(n))
    if st != NW_OK:
        raise FileNotFoundError(path)
    out = np.ctypeslib.as_array(buf, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int8)
    lib().nw_free(buf)
    return out


def band_layout(n2: int, nbands: int, r: int):
    """(rows incl. the halo row, global index of row 0) of band r -- the row
    partition of src/mpi/mpi-horz-driver.cpp:31-32 / mpi-horz.cpp:16."""
    rows, start = ctypes.c_int64(), ctypes.c_int64()
    lib().nw_band_layout(n2, nbands, r, ctypes.byref(rows), ctypes.byref(start))
    return int(rows.value), int(start.value)


def colband_layout(n1: int, n2: int, nbands: int, r: int, substrips: int = 0, strip_waves: int = 0,
                   kernel: int = KERNEL_AUTO):
    """(strip_first, strip_count, start, n_cols) of column band r: its strips of the
    whole table's sweep and the global columns [start, start + n_cols) of its local
    table, local column 0 = band r-1's last column (src/mpi/mpi-vert.cpp:17,
    mpi-vert-driver.cpp:35-36, at strip granularity)."""
    p = params(substrips=substrips, strip_waves=strip_waves, kernel=kernel)
    out = [ctypes.c_int64() for _ in range(4)]
    st = lib().nw_colband_layout(n1, n2, nbands, r, ctypes.byref(p), *[ctypes.byref(x) for x in out])
    if st != NW_OK:
        raise NwError(st, "nw_colband_layout")
    return tuple(int(x.value) for x in out)


def feed_bytes(n2: int) -> int:
    return int(lib().nw_feed_bytes(n2))


def halo_bytes(n1: int) -> int:
    return int(lib().nw_halo_bytes(n1))


class Halo:
    """A zeroed halo granule buffer (regions x (n1+1) {tag, value}) in its own
    allocation (one region per row block for block-cyclic bands)."""

    def __init__(self, n1: int, device: int = -1, regions: int = 1):
        ptr = ctypes.c_void_p()
        st = lib().nw_halo_alloc_regions(device, n1, regions, ctypes.byref(ptr))
        if st != NW_OK:
            raise NwError(st, "nw_halo_alloc_regions")
        self.ptr, self.n1, self.regions = int(ptr.value), n1, regions

    def free(self):
        if self.ptr:
            lib().nw_halo_free(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Feed(Halo):
    """A zeroed column-band feed granule buffer (n2+1 rows, padded to 64, x {tag, value})."""

    def __init__(self, n2: int, device: int = -1):
        ptr = ctypes.c_void_p()
        st = lib().nw_feed_alloc(device, n2, ctypes.byref(ptr))
        if st != NW_OK:
            raise NwError(st, "nw_feed_alloc")
        self.ptr, self.n2 = int(ptr.value), n2


class Link(Halo):
    """A zeroed launch-to-launch flow-control word pair (nw_link_alloc): the
    consumer band signals into it (peer store), the producer's stream waits on it."""

    def __init__(self, device: int = -1):
        ptr = ctypes.c_void_p()
        st = lib().nw_link_alloc(device, ctypes.byref(ptr))
        if st != NW_OK:
            raise NwError(st, "nw_link_alloc")
        self.ptr = int(ptr.value)

    def status(self) -> int:
        out = ctypes.c_uint32()
        st = lib().nw_link_status(ctypes.c_void_p(self.ptr), ctypes.byref(out))
        if st != NW_OK:
            raise NwError(st, "nw_link_status")
        return int(out.value)


def link_wait(ptr: int, value: int, stream, timeout_ms: int = 0, ctx: "Context | None" = None) -> None:
    """Stream-ordered wait until the link word at `ptr` is >= value (nw_link_wait_async).
    With `ctx` (nw_link_wait_ctx_async) a wait that gives up also fails that context:
    its next fill gives up at once instead of rewriting a buffer still being read."""
    st = lib().nw_link_wait_ctx_async(ctx._h if ctx is not None else None, ctypes.c_void_p(ptr),
                                      int(value) & 0xFFFFFFFF, int(timeout_ms), ctypes.c_void_p(stream.cuda_stream))
    if st != NW_OK:
        raise NwError(st, "nw_link_wait_ctx_async")


def link_status_at(ptr: int) -> int:
    """Word [1] of the word pair at `ptr` (nw_link_status): what a nw_link_wait on
    `ptr` records when it gives up, 0 otherwise."""
    out = ctypes.c_uint32()
    st = lib().nw_link_status(ctypes.c_void_p(ptr), ctypes.byref(out))
    if st != NW_OK:
        raise NwError(st, "nw_link_status")
    return int(out.value)


def link_signal(ptr: int, value: int, stream) -> None:
    """Stream-ordered store of `value` into the link word at `ptr` (may be peer memory)."""
    st = lib().nw_link_signal_async(ctypes.c_void_p(ptr), int(value) & 0xFFFFFFFF,
                                    ctypes.c_void_p(stream.cuda_stream))
    if st != NW_OK:
        raise NwError(st, "nw_link_signal_async")


def ipc_get_handle(ptr: int) -> bytes:
    """Export a device allocation (e.g. a halo buffer) to another process."""
    buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    st = lib().nw_ipc_get_handle(ctypes.c_void_p(ptr), buf)
    if st != NW_OK:
        raise NwError(st, "nw_ipc_get_handle")
    return buf.raw


def ipc_open_handle(handle: bytes) -> int:
    """Map a peer process's exported allocation into this device's address space."""
    ptr = ctypes.c_void_p()
    st = lib().nw_ipc_open_handle(handle, ctypes.byref(ptr))
    if st != NW_OK:
        raise NwError(st, "nw_ipc_open_handle")
    return int(ptr.value)


def ipc_close_handle(ptr: int) -> None:
    st = lib().nw_ipc_close_handle(ctypes.c_void_p(ptr))
    if st != NW_OK:
        raise NwError(st, "nw_ipc_close_handle")


def synth(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int8)
    lib().nw_synth_bdna(seed, n, out.ctypes.data_as(_i8p))
    return out


class Context:
    """Device-resident fills on torch tensors (table stays in HBM)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        st = lib().nw_ctx_create(device, ctypes.byref(self._h))
        if st != NW_OK:
            raise NwError(st, "nw_ctx_create")
        self.device = device

    def close(self):
        if self._h:
            lib().nw_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def alloc_table(n1: int, n2: int, device="cuda", pitch: int = 0):
        """(table_rows(n2), table_pitch(n1)) int32 view whose base sits
        table_offset() elements into a 256-byte aligned allocation, so that column
        1 of every row starts a 256-byte line (the fill then sweeps columns 1..n1
        in whole strips; include/nw_hip.h, nw_table_offset).  `pitch` (a
        multiple of 64 >= table_pitch(n1)) overrides the row pitch."""
        import torch
        rows = table_rows(n2)
        pitch = pitch or table_pitch(n1)
        assert pitch % 64 == 0 and pitch >= table_pitch(n1)
        off = table_offset() if n1 >= 1 else 0  # (no column 1 when n1 = 0)
        flat = torch.empty(rows * pitch + 64, dtype=torch.int32, device=device)
        shift = (-(flat.data_ptr() // 4) + off) % 64  # torch allocations are 512-B aligned
        return flat[shift:shift + rows * pitch].view(rows, pitch)

    @staticmethod
    def alloc_cycle_tables(n1: int, n2_blk: int, nblk: int, device="cuda"):
        """(nblk, table_rows(n2_blk), table_pitch(n1)) int32 view: nblk block tables
        laid out like alloc_table's, back to back (t_stride = rows * pitch)."""
        import torch
        rows, pitch = table_rows(n2_blk), table_pitch(n1)
        off = table_offset() if n1 >= 1 else 0
        flat = torch.empty(nblk * rows * pitch + 64, dtype=torch.int32, device=device)
        shift = (-(flat.data_ptr() // 4) + off) % 64
        return flat[shift:shift + nblk * rows * pitch].view(nblk, rows, pitch)

    def fill(self, d_s1, d_s2, table, scheme=(1, 0, -1), waves: int = 0, stream=None,
             sync: bool = True, flags: int = 0, substrips: int = 0, strip_waves: int = 0,
             timeout_ms: int = 0, mode: int = MODE_NW, kernel: int = KERNEL_AUTO):
        """d_s1/d_s2: int8/uint8 CUDA tensors; table: from alloc_table.  Returns NwResult
        when sync, else None (launch only)."""
        import torch
        n1, n2 = int(d_s1.numel()), int(d_s2.numel())
        assert table.dtype == torch.int32 and table.is_contiguous()
        assert table.shape[0] >= table_rows(n2) and table.shape[1] >= n1 + 1 and table.shape[1] % 64 == 0
        if stream is None:
            stream = torch.cuda.current_stream(table.device)
        sp = ctypes.c_void_p(stream.cuda_stream)
        p = params(scheme, waves, self.device, flags, substrips, strip_waves, timeout_ms, mode, kernel)
        args = (self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                ctypes.c_void_p(d_s2.data_ptr() if n2 else 0), n2, ctypes.byref(p),
                ctypes.c_void_p(table.data_ptr()), table.shape[1], sp)
        if sync:
            r = NwResult()
            st = lib().nw_fill_device(*args, ctypes.byref(r))
            if st != NW_OK:
                raise NwError(st, "nw_fill_device")
            return r
        st = lib().nw_fill_device_async(*args)
        if st != NW_OK:
            raise NwError(st, "nw_fill_device_async")
        return None

    def fill_band_cycle(self, d_s1, d_s2_blocks, n2_blk: int, tables, halo_in=None, halo_out=None,
                        hin_first: bool = False, hout_shift: int = 0, tag: int = 1, row0_max: int = 0,
                        scheme=(1, 0, -1), waves: int = 0, stream=None, flags: int = 0, substrips: int = 0,
                        strip_waves: int = 0, timeout_ms: int = 0, kernel: int = KERNEL_AUTO) -> None:
        """Launch one rank's blocks of block-cyclic row bands (asynchronous,
        nw_fill_band_cycle_async).  d_s2_blocks: the blocks' side characters, block
        k at [k * n2_blk, (k+1) * n2_blk); tables: alloc_cycle_tables(n1, n2_blk,
        nblk) (block k = tables[k]); halo_in / halo_out: raw device addresses of
        nblk-region halo buffers (Halo(..., regions=nblk).ptr or peer memory)."""
        import torch
        n1 = int(d_s1.numel())
        nblk = int(tables.shape[0])
        assert tables.dtype == torch.int32 and tables.is_contiguous() and tables.dim() == 3
        assert int(d_s2_blocks.numel()) == nblk * n2_blk
        assert tables.shape[1] >= table_rows(n2_blk) and tables.shape[2] >= n1 + 1 and tables.shape[2] % 64 == 0
        if stream is None:
            stream = torch.cuda.current_stream(tables.device)
        cy = NwBandCycle(halo_in, halo_out, nblk, int(bool(hin_first)), int(hout_shift), int(tag), int(row0_max),
                         int(tables.stride(0)))
        p = params(scheme, waves, self.device, flags, substrips, strip_waves, timeout_ms, kernel=kernel)
        st = lib().nw_fill_band_cycle_async(self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                                            ctypes.c_void_p(d_s2_blocks.data_ptr() if n2_blk else 0), n2_blk,
                                            ctypes.byref(p), ctypes.byref(cy), ctypes.c_void_p(tables.data_ptr()),
                                            tables.shape[2], ctypes.c_void_p(stream.cuda_stream))
        if st != NW_OK:
            raise NwError(st, "nw_fill_band_cycle_async")

    def fill_band(self, d_s1, d_s2_band, table, halo_in=None, halo_out=None, tag: int = 1,
                  scheme=(1, 0, -1), waves: int = 0, stream=None, flags: int = 0,
                  substrips: int = 0, strip_waves: int = 0, row0: int = 0,
                  timeout_ms: int = 0, kernel: int = KERNEL_AUTO) -> None:
        """Launch one row band (asynchronous).  d_s2_band: the band's side
        characters (len = band rows - 1); table: alloc_table(n1, len(d_s2_band)),
        row 0 = the halo row, global row `row0` (nw_band_layout start).  halo_in /
        halo_out: int64 CUDA tensors of n1+1 granules or raw device addresses (peer
        memory from ipc_open_handle)."""
        import torch
        n1, n2 = int(d_s1.numel()), int(d_s2_band.numel())
        assert table.dtype == torch.int32 and table.is_contiguous()
        assert table.shape[0] >= table_rows(n2) and table.shape[1] >= n1 + 1 and table.shape[1] % 64 == 0

        def addr(x):
            if x is None:
                return None
            if isinstance(x, int):
                return x
            assert x.dtype == torch.int64 and x.numel() >= n1 + 1
            return x.data_ptr()
        if stream is None:
            stream = torch.cuda.current_stream(table.device)
        b = NwBand(addr(halo_in), addr(halo_out), int(tag), int(row0))
        p = params(scheme, waves, self.device, flags, substrips, strip_waves, timeout_ms, kernel=kernel)
        st = lib().nw_fill_band_async(self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                                      ctypes.c_void_p(d_s2_band.data_ptr() if n2 else 0), n2,
                                      ctypes.byref(p), ctypes.byref(b),
                                      ctypes.c_void_p(table.data_ptr()), table.shape[1],
                                      ctypes.c_void_p(stream.cuda_stream))
        if st != NW_OK:
            raise NwError(st, "nw_fill_band_async")

    def fill_colband(self, d_s1, d_s2, table, nbands: int, r: int, feed_in=None, feed_out=None,
                     tag: int = 1, scheme=(1, 0, -1), waves: int = 0, stream=None, flags: int = 0,
                     substrips: int = 0, strip_waves: int = 0, timeout_ms: int = 0,
                     kernel: int = KERNEL_AUTO) -> None:
        """Launch column band r of nbands (asynchronous).  d_s1 / d_s2: the WHOLE
        sequences; table: alloc_table(n_cols - 1, n2) for the band's colband_layout
        n_cols; feed_in / feed_out: Feed buffers' addresses (raw ints, e.g. peer
        memory from ipc_open_handle) or None at the ends."""
        import torch
        n1, n2 = int(d_s1.numel()), int(d_s2.numel())
        assert table.dtype == torch.int32 and table.is_contiguous()
        if stream is None:
            stream = torch.cuda.current_stream(table.device)
        b = NwColBand(feed_in, feed_out, int(tag), int(nbands), int(r), 0)
        p = params(scheme, waves, self.device, flags, substrips, strip_waves, timeout_ms, kernel=kernel)
        st = lib().nw_fill_colband_async(self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                                         ctypes.c_void_p(d_s2.data_ptr() if n2 else 0), n2, ctypes.byref(p),
                                         ctypes.byref(b), ctypes.c_void_p(table.data_ptr()), table.shape[1],
                                         ctypes.c_void_p(stream.cuda_stream))
        if st != NW_OK:
            raise NwError(st, "nw_fill_colband_async")

    def fill_tband(self, d_s1, d_s2_band, table, row0: int = 0, feed_in=None, feed_out=None, tag: int = 1,
                   scheme=(1, 0, -1), waves: int = 0, stream=None, flags: int = 0,
                   timeout_ms: int = 0, substrips: int = 0, strip_waves: int = 0,
                   dense_polls: bool = False) -> None:
        """Launch one row band in horizontal strips (asynchronous, nw_fill_tband_async):
        the nw_fill_band contract (table: alloc_table(n1, len(d_s2_band)), row 0 =
        global row `row0` = the previous band's last row) with the band's rows swept
        as 256-row strips along the columns.  feed_in / feed_out: Feed(n1) buffers'
        addresses (raw ints, e.g. peer memory from ipc_open_handle), int64 CUDA tensors
        of feed_bytes(n1) / 8 granules, or None at the ends.  (substrips, strip_waves):
        the strip shape, (4, 1) (default) or (2, 2).  dense_polls: NW_TBAND_DENSE_POLLS
        (waiting strips poll with s_sleep 1: for chains of 1000+ strips)."""
        import torch
        n1, n2 = int(d_s1.numel()), int(d_s2_band.numel())
        assert table.dtype == torch.int32 and table.is_contiguous()
        assert table.shape[0] >= table_rows(n2) and table.shape[1] >= n1 + 1 and table.shape[1] % 64 == 0

        def addr(x):
            if x is None or isinstance(x, int):
                return x
            assert x.dtype == torch.int64 and x.numel() * 8 >= feed_bytes(n1)
            return x.data_ptr()
        if stream is None:
            stream = torch.cuda.current_stream(table.device)
        b = NwTBand(addr(feed_in), addr(feed_out), int(tag), TBAND_DENSE_POLLS if dense_polls else 0, int(row0))
        p = params(scheme, waves, self.device, flags, substrips, strip_waves, timeout_ms)
        st = lib().nw_fill_tband_async(self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                                       ctypes.c_void_p(d_s2_band.data_ptr() if n2 else 0), n2, ctypes.byref(p),
                                       ctypes.byref(b), ctypes.c_void_p(table.data_ptr()), table.shape[1],
                                       ctypes.c_void_p(stream.cuda_stream))
        if st != NW_OK:
            raise NwError(st, "nw_fill_tband_async")

    def sw_traceback(self, d_s1, d_s2, table, end, scheme=(1, -1, -1)):
        """Traceback of a device SW table (filled with mode=MODE_SW) from end = (i, j):
        (NwAlignment, ops) as sw_align."""
        n1, n2 = int(d_s1.numel()), int(d_s2.numel())
        ops = np.empty(end[0] + end[1] + 1, dtype=np.uint8)
        out = NwAlignment()
        p = params(scheme, device=self.device, mode=MODE_SW)
        st = lib().nw_sw_traceback(self._h, ctypes.c_void_p(d_s1.data_ptr() if n1 else 0), n1,
                                   ctypes.c_void_p(d_s2.data_ptr() if n2 else 0), n2, ctypes.byref(p),
                                   ctypes.c_void_p(table.data_ptr()), table.shape[1], int(end[0]), int(end[1]),
                                   ops.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ops.size,
                                   ctypes.byref(out))
        if st != NW_OK:
            raise NwError(st, "nw_sw_traceback")
        return out, ops[:out.n_ops].copy()

    def set_trace(self, trace_tensor) -> None:
        """Debug: per-strip timeline (start, end, waits, ...: tools/trace_strips.py) into
        a uint64/int64 CUDA tensor of at least strips * trace_words() elements (None = off)."""
        if trace_tensor is not None:
            assert trace_tensor.element_size() == 8
        lib().nw_debug_set_trace(self._h, ctypes.c_void_p(trace_tensor.data_ptr() if trace_tensor is not None else 0))

    def debug_ctrl(self) -> list[int]:
        """The 8 control words of the last launch (include/nw_hip.h nw_debug_ctrl)."""
        out = (ctypes.c_uint32 * 8)()
        st = lib().nw_debug_ctrl(self._h, out)
        if st != NW_OK:
            raise NwError(st, "nw_debug_ctrl")
        return list(out)

    def debug_failure(self) -> list[int]:
        """The first failure recorded on this context (include/nw_hip.h nw_debug_failure):
        [code, site word, need, seen, failed launches], pending or as the last status() cleared it."""
        out = (ctypes.c_uint32 * 5)()
        st = lib().nw_debug_failure(self._h, out)
        if st != NW_OK:
            raise NwError(st, "nw_debug_failure")
        return list(out)

    def status(self, stream=None) -> int:
        """NW_ERR_TIMEOUT if any launch on this context since the last call gave up
        (nw_ctx_status: read and cleared), else NW_OK."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream()
        return int(lib().nw_ctx_status(self._h, ctypes.c_void_p(stream.cuda_stream)))
