"""Host-side sanitizer runs (CPU only; GPU sanitizers are not available on the pool).

* oracle/san_check.c under AddressSanitizer + UndefinedBehaviorSanitizer: every
  entry point of the C restatement on small ragged shapes (empty included),
  cross-checked against each other (serial fill, score-only rows/checksums, row
  and column bands, SW fill / best cell / traceback replay).
* the idxarray-mt restatement (nw_oracle.c, idxarray-mt.cpp:4-70 semantics) under
  ThreadSanitizer, built with LLVM's libomp + Archer so that OpenMP's own
  synchronisation is visible to TSan (libgomp is not instrumented: its barriers
  show up as false races).
* the product's .bdna reader / synthetic generator (csrc/nw_bdna.cpp, host
  code of the drop-in helper.cpp:3-25) under ASan + UBSan on every fixture, an
  empty file and a missing file.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
LLVM = "/opt/rocm/lib/llvm"
BDNA_DIR = os.path.join(ROOT, "tests", "golden", "bdna")


def _run(cmd, env=None, timeout=120):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)


def _need(tool):
    if shutil.which(tool) is None and not os.path.exists(tool):
        pytest.skip(f"{tool} not available")


def test_oracle_asan_ubsan(tmp_path):
    _need("gcc")
    exe = str(tmp_path / "asan")
    r = _run(["gcc", "-std=c11", "-O1", "-g", "-fopenmp", "-fsanitize=address,undefined",
              "-fno-sanitize-recover=all", "-o", exe,
              os.path.join(ORACLE, "san_check.c"), os.path.join(ORACLE, "nw_oracle.c")])
    assert r.returncode == 0, r.stderr
    r = _run([exe, "all"])
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert "runtime error" not in r.stderr, r.stderr


def test_oracle_idxarray_tsan(tmp_path):
    clang = os.path.join(LLVM, "bin", "clang")
    _need(clang)
    if not os.path.exists(os.path.join(LLVM, "lib", "libarcher.so")):
        pytest.skip("LLVM OpenMP Archer not available")
    exe = str(tmp_path / "tsan")
    r = _run([clang, "-std=c11", "-O1", "-g", "-fopenmp", "-fsanitize=thread", "-o", exe,
              os.path.join(ORACLE, "san_check.c"), os.path.join(ORACLE, "nw_oracle.c"),
              "-L" + os.path.join(LLVM, "lib"), "-Wl,-rpath," + os.path.join(LLVM, "lib")])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="ignore_noninstrumented_modules=1 halt_on_error=1",
               OMP_NUM_THREADS="4")
    r = _run([exe, "threads"], env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert "ThreadSanitizer" not in r.stderr, r.stderr


BDNA_MAIN = r"""
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "nw_hip.h"
int main(int argc, char **argv) {
    // argv[1..]: paths; prints "<n> <sum>" or "err <code>" per path
    for (int a = 1; a < argc; ++a) {
        int8_t *p = nullptr; int64_t n = -1;
        int rc = nw_read_bdna(argv[a], &p, &n);
        if (rc != 0) { std::printf("err %d\n", rc); continue; }
        long long s = 0;
        for (int64_t i = 0; i < n; ++i) s += p[i];
        std::printf("%lld %lld\n", (long long)n, s);
        nw_free(p);
    }
    int8_t buf[1000];
    nw_synth_bdna(7, 1000, buf);
    for (int i = 0; i < 1000; ++i) if (buf[i] < 1 || buf[i] > 4) return 3;
    return 0;
}
"""


def test_bdna_reader_asan(tmp_path):
    _need("g++")
    src = tmp_path / "bdna_main.cpp"
    src.write_text(BDNA_MAIN)
    exe = str(tmp_path / "bdna_asan")
    r = _run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
              "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"), "-o", exe, str(src),
              os.path.join(ROOT, "fast-needleman-wunsch_amd", "csrc", "nw_bdna.cpp")])
    assert r.returncode == 0, r.stderr
    fixtures = sorted(os.path.join(BDNA_DIR, f) for f in os.listdir(BDNA_DIR) if f.endswith(".bdna"))
    assert fixtures
    empty = tmp_path / "empty.bdna"
    empty.write_bytes(b"")
    paths = fixtures + [str(empty), str(tmp_path / "missing.bdna")]
    r = _run([exe] + paths)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == len(paths)
    for path, line in zip(fixtures, lines):
        data = open(path, "rb").read()
        n, s = map(int, line.split())
        assert n == len(data) and s == sum(int.from_bytes(bytes([b]), "little", signed=True) for b in data)
    assert lines[-2].split()[0] in ("0", "err")
    assert lines[-1].startswith("err")
