"""RMSF.py:141-146's reduce order, pinned by the reference's own statements.

``tests/golden/reduce_exec.npz`` (tests/golden/make_reduce_vectors.py) holds
RMSF.py's exact=True computation -- each rank's RMSF.py:137-138 loop over
its RMSF.py:66-69 block, S of :140, RMSF of :146 -- with the reference's own
``second_order_moments`` applied in two orders: mpi4py's default object
reduce (``tree``: PyMPI_reduce_p2p's binomial tree, the order RMSF.py:143's
``comm.reduce`` runs; mpi4py is upstream and restated, not verified, here)
and rank order (``rank``).  They coincide at 2-3 ranks and differ in bits at
4, 5 and 8.  Also the reference function with an empty partial.

CPU tier: the oracle's reduce restatements and the C-ABI schedule
(rmsf_chan_reduce_steps, host-only).  GPU tier: rmsf_chan_reduce,
rmsf_chan_merge_pair, second_order_moments, RMSF(exact=True) under torchrun
gloo ranks, ``gpus=[0]*P`` and the context ABI's RMSF_PUSH_EXACT +
rmsf_multi_chan_merge_exact -- every one bit for bit with the vectors.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import rmsf_oracle as O
from oracle import synth as SY

PS = (2, 3, 4, 5, 8)


@pytest.fixture(scope="module")
def red():
    return np.load(os.path.join(GOLDEN, "reduce_exec.npz"))


def _traj(red):
    return SY.frames(int(red["seed"]), int(red["n_atoms"]), 0, int(red["n_frames"]))


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.uint64)


def _same(got, want, what):
    np.testing.assert_array_equal(_bits(got).reshape(-1), _bits(want).reshape(-1), err_msg=what)


# -- CPU tier ------------------------------------------------------------------

def test_orders_differ_from_four_ranks(red):
    for P in PS:
        same = np.array_equal(_bits(red[f"tree_m2_P{P}"]), _bits(red[f"rank_m2_P{P}"]))
        assert same == (P <= 3), P


@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("order,key", [("mpi4py", "tree"), ("rank", "rank")])
def test_oracle_reduce_vs_reference(red, P, order, key):
    """The oracle's rmsf_script(align=None, size=P, merge_order=...) equals the
    reference statements reduced in that order, bit for bit."""
    sel = red["sel"]
    r = O.rmsf_script(_traj(red), sel, None, size=P, align=None, merge_order=order)
    _same(r["rmsf"], red[f"{key}_rmsf_P{P}"], "rmsf")
    _same(r["mean"], red[f"{key}_mean_P{P}"], "mean")
    _same(r["m2"], red[f"{key}_m2_P{P}"], "m2")


def test_oracle_empty_partial_vs_reference(red):
    """RMSF.py:36-41 with an empty side: (3 mu) / 3, not mu (0.1 ->
    0.10000000000000002)."""
    z = np.zeros_like(red["empty_mu"])
    _, mu, M = O.second_order_moments((0, z, z), (3, red["empty_mu"], red["empty_M"]))
    _same(mu, red["empty_left_mu"], "empty left mu")
    _same(M, red["empty_left_M"], "empty left M")
    assert red["empty_left_mu"][0, 0] == 0.10000000000000002
    S = O.chan_fold([(0, z, z), (3, red["empty_mu"], red["empty_M"])])
    _same(S[1], red["empty_left_mu"], "chan_fold with an empty rank 0")


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 13, 16, 100])
def test_abi_schedule_is_mpi4py_tree(P):
    """rmsf_chan_reduce_steps (host-only C ABI) against an independent
    simulation of PyMPI_reduce_p2p's messages: every rank starts with its
    object; at each mask the ranks with the bit set send to rank & ~mask."""
    from rmsf_amd._lib import reduce_steps
    steps = reduce_steps(P, "mpi4py")
    # simulate the message passing: which rank's subtree each op combines
    holds = {r: (r,) for r in range(P)}
    expect = []
    active = set(range(P))
    mask = 1
    while mask < P:
        for r in sorted(active):
            if r & mask:
                dst = r & ~mask
                expect.append((dst, r))
                holds[dst] = holds[dst] + holds[r]
        active = {r for r in active if not r & mask}
        mask <<= 1
    assert sorted(steps) == sorted(expect)
    assert holds[0] == tuple(sorted(holds[0])) and len(holds[0]) == P
    assert reduce_steps(P, "rank") == [(0, i) for i in range(1, P)]
    with pytest.raises(ValueError):
        reduce_steps(P, "tree")


# -- GPU tier ------------------------------------------------------------------

def _states(red, P):
    """Each rank's exact S (RMSF.py:140), computed with the oracle's
    rank_sweep2 (itself bit-equal to the reference, test above)."""
    traj, sel = _traj(red), red["sel"]
    return [O.rank_sweep2(traj, sel, None, b.start, b.stop) for b in O.block_ranges(traj.shape[0], P)]


@pytest.mark.gpu
@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("order,key", [("mpi4py", "tree"), ("rank", "rank")])
def test_hip_chan_reduce_vs_reference(red, P, order, key):
    import torch

    from rmsf_amd.engine import Engine
    eng = Engine()
    parts = _states(red, P)
    n = parts[0][1].size
    mp = torch.tensor(np.stack([p[1].reshape(-1) for p in parts]), device=eng.device)
    qp = torch.tensor(np.stack([p[2].reshape(-1) for p in parts]), device=eng.device)
    mean, m2 = eng.empty(n), eng.empty(n)
    eng.chan_reduce(mp, qp, [p[0] for p in parts], n, mean, m2, order)
    rm = eng.empty(n // 3)
    eng.finalize(m2, n // 3, sum(p[0] for p in parts), rm)
    torch.cuda.synchronize()
    _same(mean.cpu().numpy(), red[f"{key}_mean_P{P}"], "mean")
    _same(m2.cpu().numpy(), red[f"{key}_m2_P{P}"], "m2")
    _same(rm.cpu().numpy(), red[f"{key}_rmsf_P{P}"], "rmsf")
    if order == "rank":   # the const-parts fold, same order
        mp = torch.tensor(np.stack([p[1].reshape(-1) for p in parts]), device=eng.device)
        qp = torch.tensor(np.stack([p[2].reshape(-1) for p in parts]), device=eng.device)
        eng.chan_merge(mp, qp, [p[0] for p in parts], n, mean, m2)
        torch.cuda.synchronize()
        _same(m2.cpu().numpy(), red["rank_m2_P%d" % P], "rmsf_chan_merge m2")


@pytest.mark.gpu
def test_hip_second_order_moments_empty_partial(red):
    """rmsf_amd.second_order_moments (k_chan_merge) with an empty side gives
    RMSF.py:36-41's values, not a copy of the other side."""
    from rmsf_amd import second_order_moments
    z = np.zeros_like(red["empty_mu"])
    T, mu, M = second_order_moments((0, z, z), (3, red["empty_mu"], red["empty_M"]))
    assert T == 3
    _same(mu, red["empty_left_mu"], "empty left mu")
    _same(M, red["empty_left_M"], "empty left M")
    assert mu[0, 0] == 0.10000000000000002
    T, mu, M = second_order_moments((3, red["empty_mu"], red["empty_M"]), (0, z, z))
    _same(mu, red["empty_right_mu"], "empty right mu")
    _same(M, red["empty_right_M"], "empty right M")
    with pytest.raises(ZeroDivisionError):
        second_order_moments((0, z, z), (0, z, z))


@pytest.mark.gpu
def test_hip_chan_merge_pair_and_reduce_empties():
    """rmsf_chan_merge_pair / rmsf_chan_reduce with empty partials: an empty
    side is (0, zeros, zeros) whatever its memory holds (NaN here), an
    empty-empty step is skipped, all-empty is RMSF_EEMPTY."""
    import torch

    from rmsf_amd.engine import Engine
    eng = Engine()
    rng = np.random.default_rng(3)
    n = 9
    counts = [0, 0, 0, 4, 0, 2, 0, 0]
    mu = rng.normal(10, 2, (8, n))
    M = rng.uniform(0, 3, (8, n))
    mu[[0, 1, 2, 4, 6, 7]] = np.nan   # empty ranks' memory is never read
    M[[0, 1, 2, 4, 6, 7]] = np.nan
    for order in ("mpi4py", "rank"):
        parts = [(c, mu[i] if c else np.zeros(n), M[i] if c else np.zeros(n)) for i, c in enumerate(counts)]
        want = O.chan_fold(parts, order)
        mp, qp = torch.tensor(mu, device=eng.device), torch.tensor(M, device=eng.device)
        mean, m2 = eng.empty(n), eng.empty(n)
        eng.chan_reduce(mp, qp, counts, n, mean, m2, order)
        torch.cuda.synchronize()
        _same(mean.cpu().numpy(), want[1], f"{order} mean")
        _same(m2.cpu().numpy(), want[2], f"{order} m2")
    a_mu, a_M = torch.tensor(mu[3], device=eng.device), torch.tensor(M[3], device=eng.device)
    b_mu, b_M = torch.full((n,), float("nan"), device=eng.device, dtype=torch.float64), eng.zeros(n)
    eng.chan_merge_pair(a_mu, a_M, 4, b_mu, b_M, 0)
    torch.cuda.synchronize()
    _, wmu, wM = O.second_order_moments((4, mu[3], M[3]), (0, np.zeros(n), np.zeros(n)))
    _same(a_mu.cpu().numpy(), wmu, "pair mu")
    _same(a_M.cpu().numpy(), wM, "pair M")
    with pytest.raises(ZeroDivisionError):
        eng.chan_merge_pair(a_mu, a_M, 0, b_mu, b_M, 0)
    with pytest.raises(ZeroDivisionError):
        eng.chan_reduce(torch.tensor(mu, device=eng.device), torch.tensor(M, device=eng.device), [0] * 8, n,
                        eng.empty(n), eng.empty(n))


def _exact_worker(rank, size, init, order, root, q):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import RMSF
        red = np.load(os.path.join(GOLDEN, "reduce_exec.npz"))
        r = RMSF(_traj(red), select=red["sel"], exact=True, merge_root=root, merge_order=order).run().results
        q.put((rank, r.rmsf, r.mean, r.sumsquares))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("P,root", [(4, 0), (5, None), (8, 3)])
@pytest.mark.parametrize("order,key", [("mpi4py", "tree"), ("rank", "rank")])
def test_rmsf_exact_torchrun_ranks(red, P, root, order, key):
    """RMSF(exact=True) on P gloo ranks sharing the GPU (the torchrun shape):
    each rank's block through the sequential Welford, the reduce point to
    point in mpi4py's tree (send / recv) or gathered in rank order -- the
    reference statements' values bit for bit on the root."""
    from conftest import spawn_ranks
    out = spawn_ranks(_exact_worker, P, lambda r, init, q: (r, P, init, order, root, q), timeout=200)
    for rank, rmsf, mean, m2 in sorted(out, key=lambda o: o[0]):
        assert not isinstance(rmsf, str), rmsf
        if root is not None and rank != root:
            assert rmsf is None
            continue
        _same(rmsf, red[f"{key}_rmsf_P{P}"], f"rank {rank} rmsf")
        _same(mean, red[f"{key}_mean_P{P}"], f"rank {rank} mean")
        _same(m2, red[f"{key}_m2_P{P}"], f"rank {rank} m2")


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 5, 8])
@pytest.mark.parametrize("order,key", [("mpi4py", "tree"), ("rank", "rank")])
@pytest.mark.parametrize("inp", ["host", "shards"])
def test_rmsf_exact_gpus_list(red, P, order, key, inp):
    """RMSF(gpus=[0]*P, exact=True): P contexts on the one device, the
    states reduced device to device by rmsf_multi_chan_merge_exact."""
    import torch

    from rmsf_amd import RMSF, parallel
    traj = _traj(red)
    x = traj if inp == "host" else [torch.tensor(traj[b0:b1], device="cuda")
                                    for b0, b1 in parallel.blocks(traj.shape[0], P)]
    r = RMSF(x, select=red["sel"], exact=True, gpus=[0] * P, merge_order=order, batch_frames=5).run().results
    _same(r.rmsf, red[f"{key}_rmsf_P{P}"], "rmsf")
    _same(r.mean, red[f"{key}_mean_P{P}"], "mean")
    _same(r.sumsquares, red[f"{key}_m2_P{P}"], "sumsquares")


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 5, 8])
@pytest.mark.parametrize("root", [None, 0, 2])
def test_context_exact_push_and_merge(red, P, root):
    """The torch-free boundary: P contexts (context i = rank i) push their
    RMSF.py:65-69 blocks with RMSF_PUSH_EXACT, rmsf_multi_chan_merge_exact
    reduces them in mpi4py's order: the result on root (or everywhere) is
    the reference statements' bit for bit; the other contexts refuse."""
    from rmsf_amd import RmsfError
    from rmsf_amd.context import PUSH_EXACT, Context
    traj, sel = _traj(red), red["sel"]
    ctxs = [Context(traj.shape[1], sel=sel) for _ in range(P)]
    try:
        for c, b in zip(ctxs, O.block_ranges(traj.shape[0], P)):
            c.set_staging(batch_frames=4, n_slots=2, n_threads=2)
            if len(b):
                c.push(traj[b.start:b.stop], PUSH_EXACT)
        Context.multi_chan_merge_exact(ctxs, root=root)
        for i, c in enumerate(ctxs):
            if root is not None and i != root:
                with pytest.raises(RmsfError):
                    c.rmsf()
                continue
            n, mean, m2 = c.partial()
            assert n == traj.shape[0]
            _same(mean, red[f"tree_mean_P{P}"], f"context {i} mean")
            _same(m2, red[f"tree_m2_P{P}"], f"context {i} m2")
            _same(c.rmsf(), red[f"tree_rmsf_P{P}"], f"context {i} rmsf")
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("root", [None, 2])
def test_context_reuse_right_after_exact_merge(red, root):
    """ADVICE r5 (write-after-read across streams): the exact merge's peer
    copies read other contexts' states on the reader's stream; every source
    context's stream now waits for those copies.  Resetting and pushing new
    frames into context 0 and a merged-away source straight after the merge
    (no synchronisation) leaves the receivers' results the script's bits."""
    from rmsf_amd.context import PUSH_EXACT, Context
    P = 4
    traj, sel = _traj(red), red["sel"]
    ctxs = [Context(traj.shape[1], sel=sel) for _ in range(P)]
    try:
        for c, b in zip(ctxs, O.block_ranges(traj.shape[0], P)):
            if len(b):
                c.push(traj[b.start:b.stop], PUSH_EXACT)
        Context.multi_chan_merge_exact(ctxs, root=root)
        reused = [0, 1] if root is not None else [0]
        noise = np.ascontiguousarray(traj[::-1][:7] + np.float32(3.0))
        for i in reused:  # overwrite the states the merge read, at once
            ctxs[i].reset()
            ctxs[i].push(noise, PUSH_EXACT)
        check = [root] if root is not None else [1, 2, 3]
        for i in check:
            n, mean, m2 = ctxs[i].partial()
            assert n == traj.shape[0]
            _same(mean, red[f"tree_mean_P{P}"], f"context {i} mean")
            _same(m2, red[f"tree_m2_P{P}"], f"context {i} m2")
        for i in reused:  # and the reused contexts hold their new frames alone
            n, _, _ = ctxs[i].partial()
            assert n == 7
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8, 9, 16, 33])
def test_abi_schedule_drives_oracle_fold(P):
    """The C ABI's schedule (rmsf_chan_reduce_steps), applied on the host
    with RMSF.py's second_order_moments and the kernels' empty-state rules
    (T = 0 skipped, an empty side as zeros), equals the oracle's
    chan_fold(order) bit for bit on random partials with empty ranks -- the
    device schedule and the Python restatement of mpi4py agree."""
    from rmsf_amd._lib import reduce_steps
    rng = np.random.default_rng(P)
    counts = [int(c) if rng.random() > 0.3 else 0 for c in rng.integers(1, 50, P)]
    if sum(counts) == 0:
        counts[-1] = 7
    parts = [(c, rng.normal(20, 5, (6, 3)) if c else np.zeros((6, 3)), rng.uniform(0, 9, (6, 3)) if c
              else np.zeros((6, 3))) for c in counts]
    for order in ("mpi4py", "rank"):
        S = list(parts)
        for d, s in reduce_steps(P, order):
            if S[d][0] + S[s][0] > 0:
                S[d] = O.second_order_moments(S[d], S[s])
        want = O.chan_fold(parts, order)
        _same(S[0][1], want[1], f"{order} mean")
        _same(S[0][2], want[2], f"{order} m2")
        assert S[0][0] == want[0] == sum(counts)
