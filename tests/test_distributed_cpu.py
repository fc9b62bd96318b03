"""CPU tier: the N>1 path (RMSF.py:59-72 blocks, :110 Allreduce, :143 reduce)
with world_size-2/3 gloo process groups.

Each rank computes its block's partial with the oracle (standing in for the
HIP kernels, which need a GPU) and then runs the *product's* cross-rank code
(``rmsf_amd.parallel``): the all-reduce sum of sweep 1 and the exact k-way
Chan merge.  The element-wise steps of the merge are injected through an
``ops`` object -- here the oracle's numpy restatement of the two kernels."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, n_frames, q):
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
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
        mean, m2 = parallel.global_chan(OracleOps, torch.from_numpy(mean_k.reshape(-1).copy()),
                                        torch.from_numpy(m2_k.reshape(-1).copy()), n_k, n_frames)
        rmsf = np.sqrt(m2.numpy().reshape(-1, 3).sum(axis=1) / n_frames)
        q.put((rank, rmsf, avg))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_frames", [(2, 40), (3, 40), (2, 1), (3, 2)])
def test_gloo_two_sweep_merge(size, n_frames):
    """world_size 2/3, including ranks with empty blocks (n_frames < size)."""
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, n_frames, q)) for r in range(size)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    traj = SY.frames(8, 60, 0, n_frames, motion_table(9, n_frames))
    ref = O.rmsf_script(traj, np.arange(0, 60, 3), None, size=1, align="average")
    for rank, rmsf, avg in out:
        np.testing.assert_allclose(rmsf, ref["rmsf"], atol=1e-9)
        np.testing.assert_allclose(avg, ref["average"], atol=1e-9)
