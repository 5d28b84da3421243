"""ctypes binding for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg import this module.  The product path never does.

Wraps oracle/liboracle.so (the C restatement in oracle/nw_oracle.c) and, when
present, the reference's own fills compiled into oracle/_ref/ by
oracle/Makefile (those export the reference C++ entry point
`needlemanWunsch(dnaArray, dnaArray, int*)`, src/serial/serial.cpp:4).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")

# scheme name -> (match, mismatch, gap); "shipped" = needleman-wunsch.hpp:11-13
SCHEMES = {"shipped": (1, 0, -1), "mm1": (1, -1, -1), "p3": (2, -1, -2)}

_i8p = ctypes.POINTER(ctypes.c_int8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.nw_oracle_fill.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     _i32p, ctypes.c_int64]
        L.nw_oracle_fill.restype = None
        L.nw_oracle_score.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      _i32p, _i32p, _u64p, _u64p]
        L.nw_oracle_score.restype = ctypes.c_int32
        L.nw_oracle_rows.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                     ctypes.c_int64, _i32p]
        L.nw_oracle_rows.restype = None
        L.nw_oracle_fill_idxarray.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64,
                                              ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                              _i32p, ctypes.c_int]
        L.nw_oracle_fill_idxarray.restype = None
        L.nw_oracle_band_layout.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_int64)]
        L.nw_oracle_fill_band.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int, ctypes.c_int, _i32p, _i32p]
        L.nw_oracle_colband_layout.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.nw_oracle_fill_colband.argtypes = [_i8p, _i8p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _i32p, _i32p]
        L.nw_oracle_synth.argtypes = [ctypes.c_uint64, ctypes.c_int64, _i8p]
        L.nw_oracle_sw_fill.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_int32, _i32p]
        L.nw_oracle_sw_fill.restype = None
        _i64p = ctypes.POINTER(ctypes.c_int64)
        L.nw_oracle_sw_best.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_int32, _i64p, _i64p]
        L.nw_oracle_sw_best.restype = ctypes.c_int32
        L.nw_oracle_sw_traceback.argtypes = [_i8p, ctypes.c_int64, _i8p, ctypes.c_int64, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, _i32p, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int64,
                                             _i64p, _i64p]
        L.nw_oracle_sw_traceback.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _seq(s) -> np.ndarray:
    a = np.ascontiguousarray(np.frombuffer(bytes(s), dtype=np.int8) if isinstance(s, (bytes, bytearray))
                             else np.asarray(s, dtype=np.int8))
    if a.size == 0:
        a = np.zeros(1, dtype=np.int8)[:0]
    return a


def fill(s1, s2, scheme=(1, 0, -1)) -> np.ndarray:
    """Full table, reference layout (n2+1, n1+1) int32 (serial.cpp:4-36)."""
    a, b = _seq(s1), _seq(s2)
    t = np.empty((b.size + 1, a.size + 1), dtype=np.int32)
    lib().nw_oracle_fill(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme, _p(t, _i32p), a.size + 1)
    return t


def fill_emb(s1, s2, scheme=(1, 0, -1)) -> np.ndarray:
    """The emb layout of src/idxarray/idxarray-emb-mt.cpp:4-65 (caller driver2.cpp:20-22):
    (n2+1) x (n1+2); column 0 = the rows' progress counters at their final value
    n1+2 (:36 row 0, :49 rows >= 1), columns 1.. = the serial table."""
    t = fill(s1, s2, scheme)
    out = np.empty((t.shape[0], t.shape[1] + 1), dtype=np.int32)
    out[:, 0] = t.shape[1] + 1
    out[:, 1:] = t
    return out


def fill_idxarray(s1, s2, scheme=(1, 0, -1), nthreads=8) -> np.ndarray:
    a, b = _seq(s1), _seq(s2)
    t = np.empty((b.size + 1, a.size + 1), dtype=np.int32)
    lib().nw_oracle_fill_idxarray(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme, _p(t, _i32p), nthreads)
    return t


def score(s1, s2, scheme=(1, 0, -1), want_rows=False):
    """Linear-memory score.  With want_rows: (score, last_row, last_col, row_sum, row_wsum)."""
    a, b = _seq(s1), _seq(s2)
    L = lib()
    if not want_rows:
        return int(L.nw_oracle_score(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme,
                                     None, None, None, None))
    lr = np.empty(a.size + 1, dtype=np.int32)
    lc = np.empty(b.size + 1, dtype=np.int32)
    rs = np.empty(b.size + 1, dtype=np.uint64)
    rw = np.empty(b.size + 1, dtype=np.uint64)
    sc = L.nw_oracle_score(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme,
                           _p(lr, _i32p), _p(lc, _i32p), _p(rs, _u64p), _p(rw, _u64p))
    return int(sc), lr, lc, rs, rw


def rows(s1, s2, scheme, which) -> np.ndarray:
    """Whole rows `which` (sorted, unique) of the table, (len(which), n1+1) int32,
    in O(n1) memory (nw_oracle_rows; the recurrence of serial.cpp:21-33)."""
    a, b = _seq(s1), _seq(s2)
    w = np.ascontiguousarray(np.asarray(which, dtype=np.int64))
    assert np.all(np.diff(w) > 0) and (w.size == 0 or (w[0] >= 0 and w[-1] <= b.size))
    out = np.empty((w.size, a.size + 1), dtype=np.int32)
    lib().nw_oracle_rows(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme,
                         w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), w.size, _p(out, _i32p))
    return out


def band_layout(n2: int, P: int, r: int):
    nr, st = ctypes.c_int64(), ctypes.c_int64()
    lib().nw_oracle_band_layout(n2, P, r, ctypes.byref(nr), ctypes.byref(st))
    return nr.value, st.value


def fill_band(s1, s2, P, r, halo, scheme=(1, 0, -1)) -> np.ndarray:
    a, b = _seq(s1), _seq(s2)
    nr, _ = band_layout(b.size, P, r)
    t = np.empty((nr, a.size + 1), dtype=np.int32)
    h = np.ascontiguousarray(halo, dtype=np.int32) if halo is not None else np.zeros(a.size + 1, np.int32)
    lib().nw_oracle_fill_band(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme, P, r,
                              _p(h, _i32p), _p(t, _i32p))
    return t


def colband_layout(n1: int, P: int, r: int):
    """(n_cols, start) of column band r (mpi-vert-driver.cpp:35-36, mpi-vert.cpp:17)."""
    nc, st = ctypes.c_int64(), ctypes.c_int64()
    lib().nw_oracle_colband_layout(n1, P, r, ctypes.byref(nc), ctypes.byref(st))
    return nc.value, st.value


def fill_colband(s1, s2, start: int, n_cols: int, left, scheme=(1, 0, -1)) -> np.ndarray:
    """Global columns [start, start + n_cols) given column `start` (`left`, n2+1
    values; None for the first band) -- mpi-vert.cpp:4-109."""
    a, b = _seq(s1), _seq(s2)
    assert 0 <= start and start + n_cols <= a.size + 1
    t = np.empty((b.size + 1, n_cols), dtype=np.int32)
    lp = None
    if left is not None:
        left = np.ascontiguousarray(left, dtype=np.int32)
        assert left.size == b.size + 1
        lp = _p(left, _i32p)
    lib().nw_oracle_fill_colband(_p(a, _i8p), _p(b, _i8p), b.size, *scheme, start, n_cols, lp, _p(t, _i32p))
    return t


# ------------------------------------------------------------------ Smith-Waterman
# (config 5; no reference counterpart -- parity unpinned, nw_oracle.c documents the
# conventions: 0 floor, first row-major best cell, traceback diag > up > left)
def sw_fill(s1, s2, scheme=(1, -1, -1)) -> np.ndarray:
    a, b = _seq(s1), _seq(s2)
    t = np.empty((b.size + 1, a.size + 1), dtype=np.int32)
    lib().nw_oracle_sw_fill(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme, _p(t, _i32p))
    return t


def sw_best(s1, s2, scheme=(1, -1, -1)):
    """(score, end_i, end_j) in linear memory."""
    a, b = _seq(s1), _seq(s2)
    ei, ej = ctypes.c_int64(), ctypes.c_int64()
    sc = lib().nw_oracle_sw_best(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme,
                                 ctypes.byref(ei), ctypes.byref(ej))
    return int(sc), int(ei.value), int(ej.value)


def sw_traceback(s1, s2, t, end, scheme=(1, -1, -1)):
    """(ops uint8 array begin -> end, begin_i, begin_j) from a full SW table."""
    a, b = _seq(s1), _seq(s2)
    t = np.ascontiguousarray(t, dtype=np.int32)
    ops = np.empty(a.size + b.size + 1, dtype=np.uint8)
    bi, bj = ctypes.c_int64(), ctypes.c_int64()
    k = lib().nw_oracle_sw_traceback(_p(a, _i8p), a.size, _p(b, _i8p), b.size, *scheme, _p(t, _i32p),
                                     end[0], end[1], ops.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                     ops.size, ctypes.byref(bi), ctypes.byref(bj))
    if k < 0:
        raise ValueError(f"sw_traceback failed ({k})")
    return ops[:k].copy(), int(bi.value), int(bj.value)


def sw_path_score(s1, s2, ops, begin, scheme=(1, -1, -1)) -> int:
    """Score of an alignment path (a size-independent property of a traceback):
    the sum of the substitution / gap scores along ops from `begin`."""
    a, b = _seq(s1), _seq(s2)
    ops = np.asarray(ops, dtype=np.uint8)
    m, mm, g = scheme
    i, j = begin
    di = np.where(ops == 2, 0, 1).cumsum()
    dj = np.where(ops == 1, 0, 1).cumsum()
    ii, jj = i + di, j + dj  # cell reached by each op
    diag = ops == 0
    eq = a[jj[diag] - 1] == b[ii[diag] - 1]
    return int(np.where(eq, m, mm).sum() + g * int((~diag).sum()))


def synth(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int8)
    lib().nw_oracle_synth(seed, n, _p(out, _i8p))
    return out


def row_checksums(t: np.ndarray):
    """(sum, column-weighted sum) per row, mod 2^64 -- same definition as nw_oracle_score."""
    t64 = t.astype(np.int64).view(np.uint64)
    w = np.arange(1, t.shape[1] + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return t64.sum(axis=1, dtype=np.uint64), (t64 * w).sum(axis=1, dtype=np.uint64)


# ---------------------------------------------------------------- reference (_ref)
class DnaArray(ctypes.Structure):
    """src/common/helper.hpp:9-12 -- {int size; int8_t* dna;} passed by value."""
    _fields_ = [("size", ctypes.c_int), ("dna", _i8p)]


def ref_available(name: str = "libref_serial.so") -> bool:
    return os.path.exists(os.path.join(REF_DIR, name))


def ref_fill(s1, s2, lib_name="libref_serial.so", extra_cols=0) -> np.ndarray:
    """Run the reference's own needlemanWunsch (compiled from its sources) on s1 x s2
    (extra_cols=1 for the emb-layout fills: n1+2 columns, driver2.cpp:20-22).  The
    table starts zeroed (idxarray-emb-mt.cpp:13-15 reads t[1] before writing it)."""
    L = ctypes.CDLL(os.path.join(REF_DIR, lib_name))
    fn = getattr(L, "_Z15needlemanWunsch8dnaArrayS_Pi")
    fn.argtypes = [DnaArray, DnaArray, _i32p]
    fn.restype = None
    a, b = _seq(s1), _seq(s2)
    a_buf = np.ascontiguousarray(a) if a.size else np.zeros(1, np.int8)
    b_buf = np.ascontiguousarray(b) if b.size else np.zeros(1, np.int8)
    t = np.zeros((b.size + 1, a.size + 1 + extra_cols), dtype=np.int32)
    fn(DnaArray(a.size, _p(a_buf, _i8p)), DnaArray(b.size, _p(b_buf, _i8p)), _p(t, _i32p))
    return t
