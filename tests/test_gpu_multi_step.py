"""GPU tier: the one-process multi-context step (rmsf_multi_push_frames +
rmsf_multi_chan_merge_root), the torchrun rank step's shape in one process:
every context's push enqueued from its own host thread, the merge as ONE
collective of moments about a common shift -- frame 0 of the frame list for
unaligned state (rmsf_set_merge_shift_frame), the reference for aligned --
optionally reduced to one context (RMSF.py:143), and the atom-slab merge
from 1M atoms.  Contexts share device 0 here (the in-process host fold, or
RCCL over one device); against the oracle's ``mpirun -n P`` emulation of
RMSF.py and against each other bit for bit where the arithmetic is the same.
"""
import numpy as np
import pytest
import torch

from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _blocks(x, P):
    from rmsf_amd.parallel import blocks
    return [x[b0:b1].contiguous() for b0, b1 in blocks(x.shape[0], P)]


@pytest.fixture(scope="module")
def traj():
    from rmsf_amd.synth import motion_table
    return SY.frames(31, 2000, 0, 53, motion_table(9, 53))


def _ctxs(n_atoms, P, sel=None):
    from rmsf_amd.context import Context
    return [Context(n_atoms, sel=sel) for _ in range(P)]


@pytest.mark.parametrize("P,root", [(1, None), (2, None), (3, 0), (4, 2), (8, 5)])
def test_unaligned_shift_frame_merge(traj, P, root):
    """Unaligned: frame 0 as every context's merge shift -> one collective;
    root=r leaves the result on context r only (the others refuse rmsf());
    equal bit for bit to the all-reduce form and within 1e-6 A of RMSF.py's
    P-rank merge."""
    from rmsf_amd import RmsfError
    from rmsf_amd.context import PUSH_WELFORD, Context
    x = torch.tensor(traj, device="cuda")
    f0 = [x[0]] * P
    exp = O.rmsf_script(traj, None, None, size=P, align=None)
    got = {}
    for r in (None, root):
        ctxs = _ctxs(traj.shape[1], P)
        Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_WELFORD, shift_frames=f0 if P > 1 else None)
        Context.multi_chan_merge(ctxs, root=r)
        home = ctxs[r or 0]
        got[r] = (home.rmsf(), *home.partial())
        if r is not None and P > 1:
            other = ctxs[(r + 1) % P]
            with pytest.raises(RmsfError, match="root"):
                other.rmsf()
        for c in ctxs:
            c.close()
    for a, b in zip(got[None], got[root]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(got[root][0], exp["rmsf"], rtol=0, atol=TOL)
    assert got[root][1] == 53


@pytest.mark.parametrize("align", ["frame0", "average"])
@pytest.mark.parametrize("P,root", [(2, 0), (5, 3)])
def test_aligned_multi_push(traj, align, P, root):
    """Aligned pushes with per-context reference frames (rmsf_multi_push_frames'
    d_ref_frames) and RMSF.py's two sweeps, merged about the common reference,
    reduced to one context."""
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, Context
    x = torch.tensor(traj, device="cuda")
    ctxs = _ctxs(traj.shape[1], P)
    bl = _blocks(x, P)
    ref = [x[0]] * P
    if align == "average":
        Context.multi_push_frames(ctxs, bl, PUSH_ALIGN_SUM, ref_frames=ref)
        Context.multi_allreduce_sum(ctxs)
        for c in ctxs:
            c.set_reference_average()
        Context.multi_push_frames(ctxs, bl, PUSH_ALIGN_WELFORD)
    else:
        Context.multi_push_frames(ctxs, bl, PUSH_ALIGN_WELFORD, ref_frames=ref)
    Context.multi_chan_merge(ctxs, root=root)
    exp = O.rmsf_script(traj, None, None, size=P, align=align)["rmsf"]
    np.testing.assert_allclose(ctxs[root].rmsf(), exp, rtol=0, atol=TOL)
    for c in ctxs:
        c.close()


def test_shift_frame_vs_two_pass_and_pipeline(traj):
    """The same blocks merged three ways: the one-collective merge about
    frame 0 (contexts), the two-pass merge (contexts without a shift frame),
    and the torchrun pipeline's own arithmetic (run_pipeline of one rank
    plus the same shifted merge over the same T1/T2): equal to rounding."""
    from rmsf_amd.context import PUSH_WELFORD, Context
    P = 3
    x = torch.tensor(traj, device="cuda")
    out = []
    for shift in (True, False):
        ctxs = _ctxs(traj.shape[1], P)
        Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_WELFORD, shift_frames=[x[0]] * P if shift else None)
        Context.multi_chan_merge(ctxs)
        out.append(ctxs[0].rmsf())
        for c in ctxs:
            c.close()
    np.testing.assert_allclose(out[0], out[1], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(out[0], O.rmsf_two_pass(traj), rtol=0, atol=1e-9)


def test_mismatched_shift_frames_fall_back_to_two_pass(traj):
    """Contexts holding DIFFERENT shift frames must not take the one-collective
    merge (T1 needs one shift): the digests differ and the two-pass form runs."""
    from rmsf_amd.context import PUSH_WELFORD, Context
    P = 2
    x = torch.tensor(traj, device="cuda")
    ctxs = _ctxs(traj.shape[1], P)
    Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_WELFORD, shift_frames=[x[0], x[7]])
    Context.multi_chan_merge(ctxs, root=0)   # two-pass: every context gets the result
    exp = O.rmsf_two_pass(traj)
    for c in ctxs:
        np.testing.assert_allclose(c.rmsf(), exp, rtol=0, atol=1e-9)
        c.close()


def test_rccl_reduce_to_root_single_device(traj):
    """ncclReduce (the reduce-to-root collective) through a one-device
    communicator: the shifted merge of one context over RCCL equals the
    pipeline's N=1 result."""
    from rmsf_amd import RMSF
    from rmsf_amd.context import PUSH_WELFORD, Context
    x = torch.tensor(traj, device="cuda")
    ctxs = _ctxs(traj.shape[1], 1)
    Context.init_all(ctxs)
    Context.multi_push_frames(ctxs, [x], PUSH_WELFORD, shift_frames=[x[0]])
    Context.multi_chan_merge(ctxs, root=0)
    np.testing.assert_allclose(ctxs[0].rmsf(), RMSF(x).run().results.rmsf, rtol=1e-13, atol=1e-13)
    ctxs[0].close()


@pytest.mark.parametrize("transport", ["fold", "rccl"])
def test_slab_merge_1m_atoms(transport):
    """From 1M atoms the multi push records the (unaligned, one-batch) sweep
    and the merge streams it in 2 atom slabs, each slab's collective issued
    on a communicator stream beside the next slab (RCCL) or in turn (host
    fold).  Bit for bit the unslabbed merge (merge_slabs=1); the accumulate
    launches are the slabs'; sampled atoms against a CPU two-pass variance."""
    from rmsf_amd.context import PUSH_WELFORD, Context
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    n_atoms, nf = 1_000_000, 33
    P = 1 if transport == "rccl" else 2
    x = generate(Engine(), n_atoms, 0, nf, seed=21)
    torch.cuda.synchronize()
    res = {}
    for slabs in (1, 0, 3):
        ctxs = _ctxs(n_atoms, P)
        if transport == "rccl":
            Context.init_all(ctxs)
        for c in ctxs:
            c.set_timing(True)
        Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_WELFORD, shift_frames=[x[0]] * P, merge_slabs=slabs)
        Context.multi_chan_merge(ctxs, root=0)
        k = ctxs[0].kernel_time("accumulate")[0]
        res[slabs] = (ctxs[0].rmsf(), *ctxs[0].partial()[1:], k)
        for c in ctxs:
            c.close()
    assert res[1][3] == 1 and res[0][3] == 2 and res[3][3] == 3
    for k in (0, 3):
        for a, b in zip(res[1][:3], res[k][:3]):
            np.testing.assert_array_equal(a, b)
    atoms = np.sort(np.random.default_rng(4).choice(n_atoms, 40, replace=False))
    host = SY.frames(21, n_atoms, 0, nf, atoms=atoms)
    np.testing.assert_allclose(res[0][0][atoms], O.rmsf_two_pass(host), rtol=0, atol=1e-9)


def test_noop_transport_and_lazy_reset(traj):
    """The no-op transport (host-cost rehearsal) moves nothing: one context
    is still exact; and a reset context that pushes nothing contributes zeros
    (the lazily-zeroed state is materialised when the merge reads it)."""
    from rmsf_amd.context import PUSH_WELFORD, TRANSPORT_NOOP, Context
    x = torch.tensor(traj, device="cuda")
    c = _ctxs(traj.shape[1], 1)
    Context.multi_set_transport(c, TRANSPORT_NOOP)
    Context.multi_push_frames(c, [x], PUSH_WELFORD, shift_frames=[x[0]])
    Context.multi_chan_merge(c, root=0)
    np.testing.assert_allclose(c[0].rmsf(), O.rmsf_two_pass(traj), rtol=0, atol=1e-9)
    c[0].close()
    # an empty context in the group: the other block is the whole result
    ctxs = _ctxs(traj.shape[1], 2)
    for ctx in ctxs:
        ctx.push(x[:5], PUSH_WELFORD)
        ctx.reset()
    Context.multi_push_frames(ctxs, [x, x[:0]], PUSH_WELFORD, shift_frames=[x[0], x[0]])
    Context.multi_chan_merge(ctxs)
    np.testing.assert_allclose(ctxs[1].rmsf(), O.rmsf_two_pass(traj), rtol=0, atol=1e-9)
    for ctx in ctxs:
        ctx.close()


@pytest.mark.parametrize("align", [None, "frame0"])
def test_multi_push_selection_and_masses(traj, align):
    """The one-process step over contexts with an atom selection (gathered in
    the kernels; the shift frame is gathered to the selection too) and, when
    aligned, heterogeneous masses (RMSF.py:84's mass-weighted COM): against
    the oracle's 3-rank RMSF.py."""
    from rmsf_amd.context import PUSH_ALIGN_WELFORD, PUSH_WELFORD, Context
    P = 3
    sel = np.sort(np.random.default_rng(7).choice(traj.shape[1], 321, replace=False))
    masses = np.random.default_rng(8).uniform(1, 16, len(sel)) if align else None
    x = torch.tensor(traj, device="cuda")
    ctxs = [Context(traj.shape[1], sel=sel, masses=masses) for _ in range(P)]
    if align:
        Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_ALIGN_WELFORD, ref_frames=[x[0]] * P)
    else:
        Context.multi_push_frames(ctxs, _blocks(x, P), PUSH_WELFORD, shift_frames=[x[0]] * P)
    Context.multi_chan_merge(ctxs, root=1)
    exp = O.rmsf_script(traj, sel, masses, size=P, align=align)["rmsf"]
    np.testing.assert_allclose(ctxs[1].rmsf(), exp, rtol=0, atol=TOL)
    for c in ctxs:
        c.close()


def test_long_device_push_launch_groups():
    """A device push longer than one launch group (16,384 frames): each
    group's fold is deferred to the next group's launch and the last one to
    the merge (fused with the pack); the result equals the pipeline's one
    batch and the CPU two-pass variance."""
    from rmsf_amd import RMSF
    from rmsf_amd.context import PUSH_WELFORD, Context
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    n_atoms, nf = 96, 40_001
    x = generate(Engine(), n_atoms, 0, nf, seed=33)
    torch.cuda.synchronize()
    ctxs = _ctxs(n_atoms, 2)
    Context.multi_push_frames(ctxs, [x[:20_000].contiguous(), x[20_000:].contiguous()], PUSH_WELFORD,
                              shift_frames=[x[0], x[0]])
    Context.multi_chan_merge(ctxs, root=0)
    got = ctxs[0].rmsf()
    for c in ctxs:
        c.close()
    np.testing.assert_allclose(got, RMSF(x).run().results.rmsf, rtol=1e-12, atol=1e-13)
    host = SY.frames(33, n_atoms, 0, nf)
    np.testing.assert_allclose(got, O.rmsf_two_pass(host), rtol=0, atol=1e-9)
