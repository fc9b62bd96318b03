"""Host logic of the merge slabs (rmsf_amd.pipeline._slab_bounds): the chunk
ranges of the flat balanced plan that become atom slabs at N > 1."""
import pytest

from rmsf_amd.pipeline import SLAB_MIN_ATOMS, SLABS_AUTO, _slab_bounds


@pytest.mark.parametrize("n_chunks", [6, 7, 8, 12, 100, 2930, 29297])
@pytest.mark.parametrize("k", [2, 3, 4, 8])
def test_slab_bounds_cover_whole_atoms(n_chunks, k):
    b = _slab_bounds(n_chunks, k)
    assert b[0][0] == 0 and b[-1][1] == n_chunks
    assert all(c0 < c1 for c0, c1 in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    # inner cuts at multiples of 3 chunks = 3 x 1024 coordinates = whole atoms
    assert all(c1 % 3 == 0 for _, c1 in b[:-1])
    assert 1 <= len(b) <= k
    if n_chunks >= 3 * k:
        assert len(b) == k
        sizes = [c1 - c0 for c0, c1 in b]
        assert max(sizes) - min(sizes) <= 6  # near-equal slabs


def test_auto_policy():
    # C4's 1M-atom share: 2930 chunks, 2 slabs by default
    assert SLAB_MIN_ATOMS == 1_000_000 and SLABS_AUTO == 2
    assert _slab_bounds(2930, SLABS_AUTO) == [(0, 1464), (1464, 2930)]
