"""The strip kernel's kinds (nw_strips.h launch_c, round 6): NW unit (match - mismatch = 1),
NW generic, Smith-Waterman -- each a kernel of its own -- and the TRACE build of the
generic and SW kinds that a launch takes when a debug trace buffer is set
(nw_debug_set_trace).  Every kind, traced and untraced, against the oracle (the
restatement of serial.cpp:21-33, pinned to the reference build in test_oracle.py),
including the table form (<= 7 distinct column characters) and the compare forms (20
letters).  Bar: bit-exact int32."""
import numpy as np
import pytest

import nwhip
import oracle

pytestmark = pytest.mark.gpu

# (scheme, kind the untraced launch takes)
SCHEMES = [((1, 0, -1), "unit"), ((1, -1, -1), "generic"), ((2, -1, -2), "generic")]
SHAPES = [(4, 1), (2, 2), (1, 4), (2, 1)]


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
    c.set_trace(None)
    c.close()


def _seqs(n1, n2, alpha, seed):
    rng = np.random.default_rng(seed)
    return (rng.integers(1, alpha + 1, n1).astype(np.int8), rng.integers(1, alpha + 1, n2).astype(np.int8))


def _fill(torch, ctx, s1, s2, scheme, shape, traced, mode=nwhip.MODE_NW):
    d1, d2 = torch.from_numpy(s1).cuda(), torch.from_numpy(s2).cuda()
    tab = nwhip.Context.alloc_table(s1.size, s2.size)
    tab.fill_(-7)
    strips = -(-(s1.size + 1) // (64 * shape[0] * shape[1])) + 1
    tr = torch.zeros(strips * nwhip.trace_words(), dtype=torch.int64, device="cuda") if traced else None
    ctx.set_trace(tr)
    try:
        r = ctx.fill(d1, d2, tab, scheme, substrips=shape[0], strip_waves=shape[1], mode=mode,
                     kernel=nwhip.KERNEL_STRIPS)
    finally:
        ctx.set_trace(None)
    assert r.status == 0
    return tab[:s2.size + 1, :s1.size + 1].cpu().numpy(), r, tr


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("scheme,kind", SCHEMES)
@pytest.mark.parametrize("alpha", [4, 20])
@pytest.mark.parametrize("traced", [False, True])
def test_nw_kinds_vs_oracle(torch, ctx, shape, scheme, kind, alpha, traced):
    s1, s2 = _seqs(1500, 700, alpha, 31 * alpha + shape[0])
    got, r, tr = _fill(torch, ctx, s1, s2, scheme, shape, traced)
    np.testing.assert_array_equal(got, oracle.fill(s1, s2, scheme))
    if traced:
        # strip 0's compute wave stamped its start (word 0) and its last wave its end (word 1)
        t = tr.cpu().numpy().view(np.uint64)
        assert t[1] > t[0] > 0


@pytest.mark.parametrize("shape", [(2, 2), (4, 1), (1, 4)])
@pytest.mark.parametrize("alpha", [4, 20])
@pytest.mark.parametrize("traced", [False, True])
def test_sw_kind_vs_oracle(torch, ctx, shape, alpha, traced):
    scheme = (1, -1, -1)
    s1, s2 = _seqs(1200, 900, alpha, 7 * alpha + shape[1])
    got, r, _ = _fill(torch, ctx, s1, s2, scheme, shape, traced, mode=nwhip.MODE_SW)
    np.testing.assert_array_equal(got, oracle.sw_fill(s1, s2, scheme))
    assert (r.score, r.end_i, r.end_j) == oracle.sw_best(s1, s2, scheme)


def test_trace_off_after_traced_fill(torch, ctx):
    """set_trace(None) returns the launch to the untraced kernel: the trace buffer of an
    earlier fill is not written again."""
    s1, s2 = _seqs(700, 300, 4, 5)
    _, _, tr = _fill(torch, ctx, s1, s2, (1, 0, -1), (4, 1), True)
    before = tr.clone()
    got, _, _ = _fill(torch, ctx, s1, s2, (1, 0, -1), (4, 1), False)
    assert torch.equal(before, tr)
    np.testing.assert_array_equal(got, oracle.fill(s1, s2, (1, 0, -1)))
