"""CPU tier: the exact=None default's choice (pipeline.auto_exact) -- the
exact path for aligned runs of fewer than AUTO_EXACT_FRAMES frames, where one
f32 rounding flip of the frame-parallel path can exceed the north star's
1e-6 A (bound ulp(x)/sqrt(N); profiles/r06_workloads/fuzz_fewframes_50seeds.txt)."""
import math

import pytest

from rmsf_amd import pipeline as PL


def test_threshold_covers_the_flip_bound():
    # one flip moves an RMSF by at most ulp(x)/sqrt(N); for |x| < 256 A the
    # f32 ulp is <= 2^-16 = 1.53e-5 A: below 1e-6 A from the threshold on
    assert 2.0 ** -16 / math.sqrt(PL.AUTO_EXACT_FRAMES) < 1e-6
    assert 2.0 ** -16 / math.sqrt(PL.AUTO_EXACT_FRAMES // 2) > 1e-6 * 0.5


@pytest.mark.parametrize("align,n,kw,want", [
    ("average", 10, {}, True), ("frame0", 255, {}, True), ("frame0", 256, {}, False),
    (None, 10, {}, False), ("average", 0, {}, False),
    ("average", 10, {"n_splits": 4}, False), ("average", 10, {"merge_scatter": True}, False),
    ("frame0", 10, {"merge_slabs": 2}, False), ("frame0", 10, {"merge_slabs": 1}, True)])
def test_auto_exact_rule(monkeypatch, align, n, kw, want):
    monkeypatch.delenv("RMSF_AUTO_EXACT_FRAMES", raising=False)
    assert PL.auto_exact(align, n, **kw) is want


def test_auto_exact_env(monkeypatch):
    monkeypatch.setenv("RMSF_AUTO_EXACT_FRAMES", "0")
    assert not PL.auto_exact("average", 3)
    monkeypatch.setenv("RMSF_AUTO_EXACT_FRAMES", "5000")
    assert PL.auto_exact("frame0", 4999)
