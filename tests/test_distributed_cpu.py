"""CPU tier: the N>1 path (RMSF.py:59-72 blocks, :110 Allreduce, :143 reduce)
with world_size-2/3 gloo process groups.

Each rank computes its block's partial with the oracle (standing in for the
HIP kernels, which need a GPU) and then runs the *product's* cross-rank code
(``rmsf_amd.parallel``): the all-reduce sum of sweep 1 and the exact k-way
Chan merge.  The element-wise steps of the merge are injected through an
``ops`` object -- here the oracle's numpy restatement of the two kernels."""
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import PKG, ROOT


class OracleOps:
    """numpy restatement of k_chan_weight / k_chan_deviation (tests only)."""

    @staticmethod
    def chan_weight(mean_k, w, out):
        out.copy_(torch.from_numpy(w * mean_k.numpy()))

    @staticmethod
    def chan_deviation(mean_k, m2_k, mean, n_k, out):
        d = mean_k.numpy() - mean.numpy()
        out.copy_(torch.from_numpy(m2_k.numpy() + n_k * (d * d)))

    # k_chan_shift_pack / k_chan_shift_finish (the one-all-reduce merge)
    @staticmethod
    def _c(shift, off3, n):
        c = shift.numpy().astype(np.float64)[:n]
        return c + np.tile(off3.numpy(), n // 3) if off3 is not None else c

    @staticmethod
    def chan_shift_pack(mean_k, m2_k, shift, off3, n_k, out):
        n = mean_k.numel()
        d = mean_k.numpy() - OracleOps._c(shift, off3, n)
        out.copy_(torch.from_numpy(np.concatenate([n_k * d, m2_k.numpy() + n_k * (d * d)])))

    @staticmethod
    def chan_shift_pack_sliced(mean_k, m2_k, shift, off3, n_k, sc, out):
        """the atom-sliced layout: slice r = [T1 | T2] of coordinates
        [r sc, (r+1) sc) at out[2 r sc:]"""
        nn = mean_k.numel()
        d = mean_k.numpy() - OracleOps._c(shift, off3, nn)
        t1, t2 = n_k * d, m2_k.numpy() + n_k * (d * d)
        o = out.numpy()
        for r in range(-(-nn // sc)):
            a, b = r * sc, min(nn, (r + 1) * sc)
            o[2 * r * sc:2 * r * sc + b - a] = t1[a:b]
            o[2 * r * sc + sc:2 * r * sc + sc + b - a] = t2[a:b]

    @staticmethod
    def chan_shift_finish_slice(t, sc, shift, off3, n_sel, n, mean, m2, rmsf):
        c = OracleOps._c(shift, off3, 3 * n_sel)
        t1, t2 = t.numpy()[:3 * n_sel], t.numpy()[sc:sc + 3 * n_sel]
        q = np.maximum(t2 - t1 * (t1 / n), 0.0)
        mean.copy_(torch.from_numpy(c + t1 / n))
        m2.copy_(torch.from_numpy(q))
        rmsf[:n_sel].copy_(torch.from_numpy(np.sqrt(q.reshape(-1, 3).sum(axis=1) / n)))

    @staticmethod
    def chan_merge(means, m2s, counts, n, mean_out, m2_out):
        """k_chan_merge: second_order_moments (RMSF.py:36-41) folded over the
        parts in rank order (the oracle's chan_fold, order "rank")."""
        from oracle import rmsf_oracle as O
        S = O.chan_fold([(c, means[i].numpy(), m2s[i].numpy()) for i, c in enumerate(counts)], "rank")
        mean_out.copy_(torch.from_numpy(np.asarray(S[1])))
        m2_out.copy_(torch.from_numpy(np.asarray(S[2])))

    @staticmethod
    def chan_merge_pair(mean1, m21, n1, mean2, m22, n2):
        """k_chan_pair: (mean1, m21) = second_order_moments(S1, S2) in place,
        an empty side being RMSF.py's (0, zeros, zeros)."""
        from oracle import rmsf_oracle as O
        z = np.zeros(mean1.numel())
        a = (n1, mean1.numpy().copy(), m21.numpy().copy()) if n1 else (0, z, z)
        b = (n2, mean2.numpy(), m22.numpy()) if n2 else (0, z, z)
        _, mu, M = O.second_order_moments(a, b)
        mean1.copy_(torch.from_numpy(np.asarray(mu)))
        m21.copy_(torch.from_numpy(np.asarray(M)))

    @staticmethod
    def chan_shift_finish(t, shift, off3, n_sel, n, mean, m2, rmsf):
        c = OracleOps._c(shift, off3, 3 * n_sel)
        t1, t2 = t.numpy()[:3 * n_sel], t.numpy()[3 * n_sel:6 * n_sel]
        q = np.maximum(t2 - t1 * (t1 / n), 0.0)
        mean.copy_(torch.from_numpy(c + t1 / n))
        m2.copy_(torch.from_numpy(q))
        rmsf.copy_(torch.from_numpy(np.sqrt(q.reshape(-1, 3).sum(axis=1) / n)))


def _worker(rank, size, port, n_frames, q, merge="two", order="mpi4py"):
    sys.path[:0] = [ROOT, PKG]
    from conftest import init_gloo
    init_gloo(port, rank, size)
    try:
        from oracle import rmsf_oracle as O
        from oracle import synth as SY
        from rmsf_amd import parallel
        from rmsf_amd.synth import motion_table

        traj = SY.frames(8, 60, 0, n_frames, motion_table(9, n_frames))
        sel = np.arange(0, 60, 3)
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        assert parallel.world() == (rank, size)
        # sweep 1 (RMSF.py:89-111): per-rank sums + product all-reduce
        ref_com, ref_c = O.centred_reference(traj[0][sel])
        s = torch.from_numpy(O.rank_sweep1(traj, sel, None, b0, b1, ref_c, ref_com).reshape(-1).copy())
        parallel.allreduce_sum_(s)
        avg = s.numpy().reshape(-1, 3) / float(n_frames)
        ref_com2, ref_c2 = O.centred_reference(avg)
        # sweep 2 (RMSF.py:120-140) + product k-way Chan (replaces :143)
        n_k, mean_k, m2_k = O.rank_sweep2(traj, sel, None, b0, b1, ref_c2, ref_com2)
        mean_k = torch.from_numpy(mean_k.reshape(-1).copy())
        m2_k = torch.from_numpy(m2_k.reshape(-1).copy())
        if merge == "two":
            mean, m2 = parallel.global_chan(OracleOps, mean_k, m2_k, n_k, n_frames)
            rmsf = np.sqrt(m2.numpy().reshape(-1, 3).sum(axis=1) / n_frames)
        elif merge in ("exact", "exact_root"):
            # exact=True's merge: every rank's S gathered, folded in rank order
            counts = [b - a for a, b in parallel.blocks(n_frames, size)]
            mean, m2 = parallel.global_chan_exact(OracleOps, mean_k, m2_k, counts,
                                                  root=1 % size if merge == "exact_root" else None, order=order)
            rmsf = None if m2 is None else np.sqrt(m2.numpy().reshape(-1, 3).sum(axis=1) / n_frames)
        else:
            # the pipeline's one-all-reduce merge, shifted by the sweep-2
            # reference (f64 centred + COM: align="frame0"'s form), by the
            # sweep-1 average (f64: align="average"), or by frame 0 (f32,
            # broadcast by the owner of block 0: no alignment)
            if merge in ("ref", "root", "scatter"):
                shift, off3, work = torch.from_numpy(ref_c2.reshape(-1).copy()), torch.from_numpy(ref_com2), None
            elif merge == "average":
                shift, off3, work = torch.from_numpy(avg.reshape(-1).copy()), None, None
            else:
                owner = next(r for r, (a, b) in enumerate(parallel.blocks(n_frames, size)) if b > a)
                shift = torch.zeros(3 * len(sel), dtype=torch.float32)
                if rank == owner:
                    shift.copy_(torch.from_numpy(traj[0][sel].reshape(-1)))
                off3, work = None, parallel.broadcast_async(shift, owner)
            if merge == "scatter":  # reduce-scatter by atom slices, RMSF gathered to rank 0
                rmsf_t, mean_s, m2_s, (a0, a1) = parallel.global_chan_scatter(OracleOps, mean_k, m2_k, n_k, n_frames,
                                                                             shift, off3, work, root=0)
                mean_r, m2_r, _ = parallel.global_chan_shifted(OracleOps, mean_k, m2_k, n_k, n_frames, shift, off3)
                # this rank's slice of the merged statistics: those of the all-reduce form
                np.testing.assert_allclose(mean_s.numpy(), mean_r.numpy()[3 * a0:3 * a1], rtol=1e-14, atol=1e-14)
                np.testing.assert_allclose(m2_s.numpy(), m2_r.numpy()[3 * a0:3 * a1], rtol=1e-12, atol=1e-14)
            else:
                mean, m2, rmsf_t = parallel.global_chan_shifted(OracleOps, mean_k, m2_k, n_k, n_frames, shift, off3,
                                                                work, root=0 if merge == "root" else None)
            rmsf = None if rmsf_t is None else rmsf_t.numpy()
        q.put((rank, rmsf, avg))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("merge", ["two", "ref", "average", "frame0", "root", "scatter", "exact", "exact_root"])
@pytest.mark.parametrize("size,n_frames", [(2, 40), (3, 40), (2, 1), (3, 2)])
def test_gloo_two_sweep_merge(size, n_frames, merge):
    """world_size 2/3, including ranks with empty blocks (n_frames < size);
    the two-all-reduce Chan merge and the one-all-reduce shifted form with
    each of the pipeline's shifts; "root": the reduce to rank 0 of
    RMSF.py:143 (the other ranks get no result); "scatter": the
    reduce-scatter by atom slices (20 atoms over 3 ranks: a padded last
    slice), each rank's slice of mean/M2 equal to the all-reduce form's and
    the RMSF gathered to rank 0."""
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table

    from conftest import spawn_ranks
    out = spawn_ranks(_worker, size, lambda r, init, q: (r, size, init, n_frames, q, merge))
    traj = SY.frames(8, 60, 0, n_frames, motion_table(9, n_frames))
    ref = O.rmsf_script(traj, np.arange(0, 60, 3), None, size=1, align="average")
    # the exact merge: RMSF.py under mpirun -n size reduced in rank order, bit for bit
    ref_p = O.rmsf_script(traj, np.arange(0, 60, 3), None, size=size, align="average")
    for rank, rmsf, avg in out:
        if (merge in ("root", "scatter") and rank != 0) or (merge == "exact_root" and rank != 1 % size):
            assert rmsf is None
        elif merge.startswith("exact"):
            np.testing.assert_array_equal(rmsf.view(np.uint64), ref_p["rmsf"].view(np.uint64))
        else:
            np.testing.assert_allclose(rmsf, ref["rmsf"], atol=1e-9)
        np.testing.assert_allclose(avg, ref["average"], atol=1e-9)


def test_scatter_layout_single_process():
    """The atom-sliced layout of the reduce-scatter merge, one process: the
    pad coordinates of the last slices are zeroed, and the merge equals the
    one-all-reduce form (the oracle's ops; size 1 = no collective)."""
    from rmsf_amd import parallel
    t = torch.full((2 * 9 * 3,), 7.0, dtype=torch.float64)
    parallel.zero_slice_padding(t, n=20, sc=9, size=3)   # slices of 9 coordinates, 20 real
    t = t.numpy()
    assert (t[:36] == 7).all()                             # slices 0 and 1 full
    assert (t[36:38] == 7).all() and (t[38:45] == 0).all()  # slice 2: T1 has 2 real coordinates
    assert (t[45:47] == 7).all() and (t[47:] == 0).all()    # ... and so has T2
    rng = np.random.default_rng(5)
    mean_k = torch.from_numpy(rng.normal(50, 3, 3 * 7))
    m2_k = torch.from_numpy(rng.uniform(0, 2, 3 * 7))
    shift = torch.from_numpy(rng.normal(50, 3, 3 * 7).astype(np.float32))
    rmsf, mean_s, m2_s, sl = parallel.global_chan_scatter(OracleOps, mean_k, m2_k, 11, 11, shift)
    mean, m2, rmsf2 = parallel.global_chan_shifted(OracleOps, mean_k, m2_k, 11, 11, shift)
    assert sl == (0, 7)
    np.testing.assert_array_equal(rmsf.numpy(), rmsf2.numpy())
    np.testing.assert_array_equal(mean_s.numpy(), mean.numpy())
    np.testing.assert_array_equal(m2_s.numpy(), m2.numpy())


@pytest.mark.parametrize("order", ["mpi4py", "rank"])
@pytest.mark.parametrize("size,n_frames,to_root", [(4, 41, False), (5, 53, True), (4, 3, True), (5, 23, False),
                                                   (6, 40, False), (7, 5, True)])
def test_gloo_exact_merge_order(size, n_frames, to_root, order):
    """RMSF.py:143's comm.reduce at 4-7 ranks through the product's
    exact merge (parallel.global_chan_exact): order "mpi4py" runs mpi4py's
    binomial tree point to point (send / recv between the gloo ranks),
    "rank" gathers and folds in rank order; each equals the oracle's
    rmsf_script with that order bit for bit, on the root (or every rank).
    3 frames on 4 ranks: empty ranks 0-2 (a skipped empty-empty merge); 5
    frames on 7 ranks: only the last rank holds frames (empty subtrees)."""
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table

    from conftest import spawn_ranks
    out = spawn_ranks(_worker, size, lambda r, init, q: (r, size, init, n_frames, q,
                                                         "exact_root" if to_root else "exact", order))
    traj = SY.frames(8, 60, 0, n_frames, motion_table(9, n_frames))
    want = O.rmsf_script(traj, np.arange(0, 60, 3), None, size=size, align="average", merge_order=order)
    other = O.rmsf_script(traj, np.arange(0, 60, 3), None, size=size, align="average",
                          merge_order="rank" if order == "mpi4py" else "mpi4py")
    got_root = 1 % size if to_root else None
    for rank, rmsf, _ in out:
        if got_root is not None and rank != got_root:
            assert rmsf is None
            continue
        np.testing.assert_array_equal(rmsf.view(np.uint64), want["rmsf"].view(np.uint64))
    if n_frames > size:   # the two orders differ in bits here (the option matters)
        assert not np.array_equal(want["m2"].view(np.uint64), other["m2"].view(np.uint64))
