"""Smith-Waterman + on-device traceback (BASELINE config 5).

PARITY UNPINNED: the reference has no local alignment (README.md:2 states the
intent only).  The checker is the build's CPU restatement (oracle/nw_oracle.c
nw_oracle_sw_*), itself cross-checked here against an independent pure-Python
restatement.  Conventions (include/nw_hip.h nw_sw_align): 0 floor, row/column 0
all zero, best cell = first row-major maximum, traceback while t > 0 preferring
diag > up > left (the order of serial.cpp:24-30's max).

CPU: the two restatements agree (tables, best cell, ops); the golden file is
self-consistent.  GPU: device tables bit-exact vs the oracle for every SW strip
shape (the (2, 4) half-word rings also where cells reach 2^16, through the corner
fix-up); nw_sw_align against the golden vectors (bdna pairs, and the 65536 x 65536
synthetic workload = config 5) including the ops' sha256; the score of the
returned path equals the table maximum (a size-independent property).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import nwhip
import oracle
from conftest import GOLDEN

SCHEMES = [(1, -1, -1), (1, 0, -1), (2, -1, -2)]
SW_SHAPES = [(2, 2), (1, 4), (4, 1), (2, 1), (2, 4)]  # (2, 4): 512-column strips, half-word rings


def sw_golden():
    with open(os.path.join(GOLDEN, "sw_golden.json")) as f:
        return json.load(f)


def py_sw(s1, s2, scheme):
    """Independent pure-Python restatement (small inputs only): table, best, ops."""
    m, mm, g = scheme
    n1, n2 = len(s1), len(s2)
    t = [[0] * (n1 + 1) for _ in range(n2 + 1)]
    best, bi, bj = 0, 0, 0
    for i in range(1, n2 + 1):
        for j in range(1, n1 + 1):
            d = t[i - 1][j - 1] + (m if s1[j - 1] == s2[i - 1] else mm)
            v = max(0, d, t[i - 1][j] + g, t[i][j - 1] + g)
            t[i][j] = v
            if v > best:
                best, bi, bj = v, i, j
    ops, i, j = [], bi, bj
    while i > 0 and j > 0 and t[i][j] > 0:
        v = t[i][j]
        if v == t[i - 1][j - 1] + (m if s1[j - 1] == s2[i - 1] else mm):
            ops.append(0)
            i, j = i - 1, j - 1
        elif v == t[i - 1][j] + g:
            ops.append(1)
            i -= 1
        else:
            assert v == t[i][j - 1] + g
            ops.append(2)
            j -= 1
    return np.array(t, dtype=np.int32), (best, bi, bj), np.array(ops[::-1], dtype=np.uint8), (i, j)


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("scheme", SCHEMES)
@pytest.mark.parametrize("shape", [(1, 1), (5, 9), (40, 33), (120, 97)])
def test_sw_oracle_matches_independent_restatement(scheme, shape):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    s1 = rng.integers(1, 5, shape[0]).astype(np.int8)
    s2 = rng.integers(1, 5, shape[1]).astype(np.int8)
    t, best, ops, begin = py_sw(list(s1), list(s2), scheme)
    np.testing.assert_array_equal(oracle.sw_fill(s1, s2, scheme), t)
    assert oracle.sw_best(s1, s2, scheme) == best
    got, bi, bj = oracle.sw_traceback(s1, s2, t, best[1:], scheme)
    np.testing.assert_array_equal(got, ops)
    assert (bi, bj) == begin
    assert oracle.sw_path_score(s1, s2, got, (bi, bj), scheme) == best[0]


def test_sw_golden_self_consistent():
    g = sw_golden()
    for key, e in list(g["pairs"].items()) + list(g["synth"].items()):
        assert sum(e["ops_counts"]) == e["n_ops"]
        di = e["ops_counts"][0] + e["ops_counts"][1]
        dj = e["ops_counts"][0] + e["ops_counts"][2]
        assert e["end"][0] - e["begin"][0] == di and e["end"][1] - e["begin"][1] == dj, key


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def torch():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    return _t


@pytest.fixture(scope="module")
def ctx(torch):
    c = nwhip.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("strip", SW_SHAPES)
@pytest.mark.parametrize("scheme", SCHEMES)
@pytest.mark.parametrize("n1,n2,alpha", [(1, 1, 4), (63, 64, 4), (300, 1000, 4), (1500, 1100, 4),
                                         (1000, 300, 20), (257, 513, 4)])
def test_sw_table_and_best_vs_oracle(torch, ctx, strip, scheme, n1, n2, alpha):
    rng = np.random.default_rng(n1 * 3 + n2 + alpha)
    s1 = rng.integers(1, alpha + 1, n1).astype(np.int8)
    s2 = rng.integers(1, alpha + 1, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n1, n2)
    r = ctx.fill(d1, d2, tab, scheme, substrips=strip[0], strip_waves=strip[1], mode=nwhip.MODE_SW)
    assert r.status == 0
    want = oracle.sw_fill(s1, s2, scheme)
    np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), want)
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)
    al, ops = ctx.sw_traceback(d1, d2, tab, (r.end_i, r.end_j), scheme)
    wops, bi, bj = oracle.sw_traceback(s1, s2, want, (r.end_i, r.end_j), scheme)
    np.testing.assert_array_equal(ops, wops)
    assert (al.begin_i, al.begin_j, al.score) == (bi, bj, r.score)


@pytest.mark.gpu
@pytest.mark.parametrize("band,maxwin", [(1, 4096), (3, 1), (17, 3), (128, 2), (128, 4096)])
@pytest.mark.parametrize("scheme", SCHEMES + [(2, -1, 0)])
@pytest.mark.parametrize("n1,n2,alpha", [(1500, 1100, 4), (1000, 300, 20), (300, 1000, 4), (2000, 2000, 2)])
def test_sw_traceback_windows_vs_oracle(torch, ctx, monkeypatch, band, maxwin, scheme, n1, n2, alpha):
    """The windowed traceback (nw_sw.hip) with narrow bands and short rounds: paths
    that leave the band and rounds that end in mid-table restart re-centred, and
    the ops still equal the oracle's walk."""
    monkeypatch.setenv("NW_TB_BAND", str(band))
    monkeypatch.setenv("NW_TB_MAXWIN", str(maxwin))
    rng = np.random.default_rng(n1 + 7 * n2 + alpha + band)
    s1 = rng.integers(1, alpha + 1, n1).astype(np.int8)
    s2 = rng.integers(1, alpha + 1, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n1, n2)
    r = ctx.fill(d1, d2, tab, scheme, mode=nwhip.MODE_SW)
    want = oracle.sw_fill(s1, s2, scheme)
    al, ops = ctx.sw_traceback(d1, d2, tab, (r.end_i, r.end_j), scheme)
    wops, bi, bj = oracle.sw_traceback(s1, s2, want, (r.end_i, r.end_j), scheme)
    np.testing.assert_array_equal(ops, wops)
    assert (al.begin_i, al.begin_j, al.score, al.n_ops) == (bi, bj, r.score, len(wops))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small", "t", "debug", "smid"])
@pytest.mark.parametrize("scheme", SCHEMES)
def test_sw_align_bdna_vs_golden(pair, name, scheme):
    e = sw_golden()["pairs"][f"{name}:{','.join(map(str, scheme))}"]
    s1, s2 = pair(name)
    al, ops = nwhip.sw_align(s1, s2, scheme)
    assert al.score == e["score"]
    assert [al.end_i, al.end_j] == e["end"] and [al.begin_i, al.begin_j] == e["begin"]
    assert al.n_ops == e["n_ops"] and hashlib.sha256(ops.tobytes()).hexdigest() == e["ops_sha256"]


@pytest.mark.gpu
def test_sw_no_positive_cell(torch):
    """Disjoint alphabets: every cell is 0, the best cell is (0, 0), no ops."""
    al, ops = nwhip.sw_align(np.full(300, 1, np.int8), np.full(200, 2, np.int8), (1, -1, -1))
    assert al.score == 0 and (al.end_i, al.end_j) == (0, 0) and al.n_ops == 0 and ops.size == 0


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("scheme", [(1, -1, -1), (1, 0, -1)])
def test_config5_sw_64k_vs_golden(torch, scheme):
    """BASELINE config 5: Smith-Waterman + on-device traceback, 65536 x 65536."""
    n = 65536
    e = sw_golden()["synth"][f"{n}:{','.join(map(str, scheme))}"]
    s1, s2 = nwhip.synth(1, n), nwhip.synth(2, n)
    torch.cuda.empty_cache()
    al, ops = nwhip.sw_align(s1, s2, scheme)
    assert al.score == e["score"]
    assert [al.end_i, al.end_j] == e["end"] and [al.begin_i, al.begin_j] == e["begin"]
    assert al.n_ops == e["n_ops"] and hashlib.sha256(ops.tobytes()).hexdigest() == e["ops_sha256"]
    assert oracle.sw_path_score(s1, s2, ops, (al.begin_i, al.begin_j), scheme) == al.score


@pytest.mark.gpu
def test_sw_range_refused(torch, ctx):
    """Smith-Waterman cells live in the w form too (w = t - GAP*(i+j), the
    floor z = -GAP*(i+j)), so the NW bound (max|score| + |GAP|) * (n1 + n2 + 2) < 2^28
    applies: a long, thin table with a large gap is refused, not wrapped."""
    s1, s2 = nwhip.synth(1, 600000), nwhip.synth(2, 1000)
    with pytest.raises(nwhip.NwError) as e:
        nwhip.sw_align(s1, s2, (1, -1, -4000))
    assert e.value.status == nwhip.NW_ERR_ARG
    # the same shape with the unit scheme is inside the bound and exact
    al, ops = nwhip.sw_align(s1[:20000], s2[:300], (1, -1, -1))
    assert (al.score, al.end_i, al.end_j) == oracle.sw_best(s1[:20000], s2[:300], (1, -1, -1))


@pytest.mark.gpu
def test_sw_refusals(torch, ctx):
    """SW with a positive gap, or on a row band, is refused rather than mis-computed."""
    s = nwhip.synth(1, 100)
    with pytest.raises(nwhip.NwError) as e:
        nwhip.sw_align(s, s, (1, -1, 1))
    assert e.value.status == nwhip.NW_ERR_ARG


def _half_word_pair(n, mutate, seed):
    rng = np.random.default_rng(seed)
    s1 = rng.integers(1, 5, n).astype(np.int8)
    s2 = s1.copy()
    pos = rng.random(n) < mutate
    s2[pos] = (s2[pos] % 4) + 1  # a different character
    return s1, s2


@pytest.mark.gpu
@pytest.mark.parametrize("n,mutate", [(660, 0.0), (661, 0.03), (700, 0.0)])
def test_sw_half_word_corner(torch, ctx, n, mutate):
    """(2, 4) keeps the low 16 bits of each cell in its LDS rings (nw_strips.h
    Lay::kHalf).  With match 100 the cells with min(i, j) >= 656 may reach 2^16
    (identical sequences: up to 66000 at n = 660); that corner -- 25 / 36 cells
    here -- is recomputed exactly after the fill (nw_sw.hip nw_sw_fixup), so the
    whole table, the best cell and the path equal the oracle's.  At n = 700 the
    corner (45 x 45 cells) exceeds the fix-up's bound: refused, and the auto shape
    still fills it exactly."""
    scheme = (100, -100, -1)
    s1, s2 = _half_word_pair(n, mutate, n)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    want = oracle.sw_fill(s1, s2, scheme)
    if n == 700:
        assert want.max() >= 65536
        with pytest.raises(nwhip.NwError) as e:
            ctx.fill(d1, d2, tab, scheme, substrips=2, strip_waves=4, mode=nwhip.MODE_SW)
        assert e.value.status == nwhip.NW_ERR_UNSUPPORTED
        r = ctx.fill(d1, d2, tab, scheme, mode=nwhip.MODE_SW)
    else:
        assert (want.max() >= 65536) == (mutate == 0.0)
        tab.fill_(-0x5A5A5A5)
        r = ctx.fill(d1, d2, tab, scheme, substrips=2, strip_waves=4, mode=nwhip.MODE_SW)
    np.testing.assert_array_equal(tab[:n + 1, :n + 1].cpu().numpy(), want)
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)
    al, ops = ctx.sw_traceback(d1, d2, tab, (r.end_i, r.end_j), scheme)
    wops, bi, bj = oracle.sw_traceback(s1, s2, want, (r.end_i, r.end_j), scheme)
    np.testing.assert_array_equal(ops, wops)


@pytest.mark.gpu
def test_sw_half_word_timing_only_leaves_table_alone(torch, ctx):
    """ NW_FLAG_TIMING_ONLY on the (2, 4) half-word path: the strips store
    into a scratch tile, so the corner fix-up must not run on the caller's (unwritten)
    table either -- every byte of it stays as it was, corner included."""
    scheme = (100, -100, -1)
    n = 660
    s1, s2 = _half_word_pair(n, 0.0, n)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    tab.fill_(-0x5A5A5A5)
    ctx.fill(d1, d2, tab, scheme, substrips=2, strip_waves=4, mode=nwhip.MODE_SW, flags=nwhip.FLAG_TIMING_ONLY)
    torch.cuda.synchronize()
    assert bool((tab == -0x5A5A5A5).all())


@pytest.mark.gpu
def test_sw_half_word_shape_is_sw_only(torch, ctx):
    """The half-word rings hold Smith-Waterman cells only: an NW fill with (2, 4) is
    refused rather than wrapped."""
    s = torch.from_numpy(nwhip.synth(1, 2000)).cuda()
    tab = nwhip.Context.alloc_table(2000, 2000)
    with pytest.raises(nwhip.NwError) as e:
        ctx.fill(s, s, tab, (1, 0, -1), substrips=2, strip_waves=4)
    assert e.value.status == nwhip.NW_ERR_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("strip", [(2, 2), (2, 4)])
@pytest.mark.parametrize("n1,n2", [(660, 657), (1537, 300), (5, 9)])
def test_sw_strip_origin_column0(torch, ctx, strip, n1, n2):
    """A 256-byte aligned table base sweeps column 0 with the strips (origin 0), also
    for the half-word rings and their corner fix-up (match 100: cells reach 2^16 where
    the sequences agree; the corner's strip words are indexed from origin 0)."""
    scheme = (100, -100, -1)
    rng = np.random.default_rng(n1 + 3 * n2)
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = s1[:n2].copy() if n2 <= n1 else rng.integers(1, 5, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    rows, pitch = nwhip.table_rows(n2), nwhip.table_pitch(n1)
    flat = torch.empty(rows * pitch + 64, dtype=torch.int32, device="cuda")
    shift = (-(flat.data_ptr() // 4)) % 64
    tab = flat[shift:shift + rows * pitch].view(rows, pitch)
    tab.fill_(-0x5A5A5A5)
    want = oracle.sw_fill(s1, s2, scheme)
    r = ctx.fill(d1, d2, tab, scheme, substrips=strip[0], strip_waves=strip[1], mode=nwhip.MODE_SW)
    np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), want)
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", [(2, -1, 0), (-1, 3, -2), (0, -1, -1), (7, -5, -3)])
@pytest.mark.parametrize("n1,n2", [(1100, 700), (513, 1024)])
def test_sw_half_word_schemes(torch, ctx, scheme, n1, n2):
    """(2, 4) half-word rings under gap 0, a mismatch above the match (the corner bound
    uses max(match, mismatch)), no positive score at all, and a wide scheme: tables,
    best cell and path equal the oracle's (all corners empty at these sizes)."""
    rng = np.random.default_rng(n1 + n2 + sum(scheme))
    s1 = rng.integers(1, 5, n1).astype(np.int8)
    s2 = rng.integers(1, 5, n2).astype(np.int8)
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(n1, n2)
    tab.fill_(-0x5A5A5A5)
    r = ctx.fill(d1, d2, tab, scheme, substrips=2, strip_waves=4, mode=nwhip.MODE_SW)
    want = oracle.sw_fill(s1, s2, scheme)
    np.testing.assert_array_equal(tab[:n2 + 1, :n1 + 1].cpu().numpy(), want)
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)
    al, ops = ctx.sw_traceback(d1, d2, tab, (r.end_i, r.end_j), scheme)
    wops, bi, bj = oracle.sw_traceback(s1, s2, want, (r.end_i, r.end_j), scheme)
    np.testing.assert_array_equal(ops, wops)
