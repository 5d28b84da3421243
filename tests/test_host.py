"""CPU: the C-ABI library builds, loads and exports every symbol include/nw_hip.h
declares; host helpers match the oracle; no silent CPU fallback without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

import nwhip
import oracle
from conftest import ROOT, bdna_path, read_bdna

HEADER = os.path.join(ROOT, "include", "nw_hip.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(nw_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_api():
    assert header_functions() == sorted(nwhip.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", nwhip.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in header_functions() if s not in syms]
    assert not missing, missing
    lib = nwhip.lib()
    for s in header_functions():
        assert hasattr(lib, s)


def test_kernel_code_object_is_gfx950():
    data = open(nwhip.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_dropin_driver_exports_reference_plugin_symbol():
    drv = os.path.join(ROOT, "fast-needleman-wunsch_amd", "build", "nw_driver")
    out = subprocess.run(["nm", drv], capture_output=True, text=True, check=True).stdout
    # the reference fills' entry point, src/serial/serial.cpp:4
    assert "_Z15needlemanWunsch8dnaArrayS_Pi" in out


def test_pitch_and_bytes():
    # multiple of 64 holding nCols = n1 + 1 plus 3 columns of slack (the 16-byte
    # store holding column n1 must stay inside the row when strips start at column 1)
    assert nwhip.table_pitch(0) == 64
    assert nwhip.table_pitch(60) == 64
    assert nwhip.table_pitch(61) == 128
    assert nwhip.table_pitch(63) == 128
    assert nwhip.table_pitch(64) == 128
    assert nwhip.table_pitch(262144) == 262208
    assert nwhip.lib().nw_table_bytes(262144, 262144) == (262145 + 63) // 64 * 64 * 262208 * 4
    assert nwhip.table_offset() == 63  # column 1 of every row on a 256-byte line


def test_strip_shapes_lds():
    """Every supported strip shape fits a CU's 160 KiB of LDS; others are refused.
    (2, 4) fits only with its half-word rings (Smith-Waterman only)."""
    for c, nc in [(4, 1), (2, 1), (1, 1), (2, 2), (1, 2), (1, 4), (2, 4)]:
        b = nwhip.strip_lds_bytes(c, nc)
        assert 0 < b <= 160 * 1024, (c, nc, b)
    assert nwhip.strip_lds_bytes(4, 2) == -1 and nwhip.strip_lds_bytes(3, 1) == -1
    assert nwhip.strip_shape() == (2, 2)
    assert nwhip.strip_shape(4) == (4, 1) and nwhip.strip_shape(1) == (1, 4)
    assert nwhip.strip_shape(2, 1) == (2, 1)


def test_default_params_are_reference_constants():
    p = nwhip.params()
    assert (p.match, p.mismatch, p.gap) == (1, 0, -1)   # needleman-wunsch.hpp:11-13


@pytest.mark.parametrize("seed,n", [(1, 0), (1, 1000), (2, 4097), (12345, 10)])
def test_synth_matches_oracle(seed, n):
    a = nwhip.synth(seed, n)
    np.testing.assert_array_equal(a, oracle.synth(seed, n))
    if n:
        assert set(np.unique(a)) <= {1, 2, 3, 4}


@pytest.mark.parametrize("name", ["small1.bdna", "t2.bdna", "smid1.bdna"])
def test_read_bdna_is_readsequence(name):
    np.testing.assert_array_equal(nwhip.read_bdna(bdna_path(name)), read_bdna(name))


def test_read_bdna_missing_file():
    with pytest.raises(FileNotFoundError):
        nwhip.read_bdna("/nonexistent/x.bdna")


def test_read_bdna_keeps_every_byte(tmp_path):
    p = tmp_path / "x.bdna"
    raw = bytes([1, 2, 10, 0, 255, 3, 13])   # newline / zero / 0xFF are kept (helper.cpp:9-13)
    p.write_bytes(raw)
    np.testing.assert_array_equal(nwhip.read_bdna(str(p)), np.frombuffer(raw, np.int8))


def _gpu_visible():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-device path")
def test_no_device_fails_loudly():
    with pytest.raises(nwhip.NwError) as ei:
        nwhip.score([1, 2, 3], [1, 2])
    assert ei.value.status == nwhip.NW_ERR_NODEVICE


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-device path")
def test_dropin_driver_fails_loudly_without_device():
    drv = os.path.join(ROOT, "fast-needleman-wunsch_amd", "build", "nw_driver")
    r = subprocess.run([drv, bdna_path("small1.bdna"), bdna_path("small2.bdna")],
                       capture_output=True, text=True)
    assert r.returncode == 2
    assert "libnwhip" in r.stderr


def test_driver_cli_argument_errors():
    drv = os.path.join(ROOT, "fast-needleman-wunsch_amd", "build", "nw_driver")
    r = subprocess.run([drv, "only-one"], capture_output=True, text=True)
    assert r.returncode == 1 and "incorrect number of arguments" in r.stdout
    r = subprocess.run([drv, "/nonexistent/a", "/nonexistent/b"], capture_output=True, text=True)
    assert r.returncode == 1 and "ERROR: no such file /nonexistent/a" in r.stdout


def test_tuned_shape_is_supported():
    """nw_tuned_shape (the tuner's table, csrc/nw_tuned.h) only ever names supported
    strip shapes, for every size class."""
    for n in [0, 1, 100, 4096, 32768, 65536, 131072, 262144, 524288]:
        c, nc = nwhip.tuned_shape(n, n)
        assert nwhip.strip_lds_bytes(c, nc) > 0, (n, c, nc)
        assert nwhip.strip_shape(0, 0, n, n) == (c, nc)


def test_auto_shape_picks_supported_kernels():
    """nw_auto_shape: the tuner's table picks the kernel family too; a panel entry
    applies only when every CU gets a panel in one pass, else the strip entry."""
    for n in [0, 1, 100, 4096, 32768, 65536, 131072, 262144, 524288]:
        k, c, nc = nwhip.auto_shape(n, n, 256)
        assert k in (nwhip.KERNEL_STRIPS, nwhip.KERNEL_PANELS), (n, k)
        if k == nwhip.KERNEL_PANELS:
            assert nwhip.panel_lds_bytes(c, nc) > 0 and n + 1 >= 256 * 64 * c * nc, (n, c, nc)
        else:
            assert nwhip.strip_lds_bytes(c, nc) > 0, (n, c, nc)
    # a tall table with as many cells as the 256k square but narrow: strips
    assert nwhip.auto_shape(65535, 1 << 20, 256)[0] == nwhip.KERNEL_STRIPS
    # the panel rule scales with the device's CUs: on 512 CUs the 256k entry's panels no
    # longer give every CU one, so an earlier entry applies -- strips, or narrower panels
    # that still do (the round-6 table: (2,4) panels, 512 columns each)
    k, c, nc = nwhip.auto_shape(262144, 262144, 256)
    if k == nwhip.KERNEL_PANELS:
        assert 262145 >= 256 * 64 * c * nc
        k2, c2, nc2 = nwhip.auto_shape(262144, 262144, 512)
        if k2 == nwhip.KERNEL_PANELS:
            assert (c2, nc2) != (c, nc) and 262145 >= 512 * 64 * c2 * nc2, (c2, nc2)
        else:
            assert nwhip.strip_lds_bytes(c2, nc2) > 0, (c2, nc2)


def test_trace_words_exported():
    assert nwhip.trace_words() >= 16
