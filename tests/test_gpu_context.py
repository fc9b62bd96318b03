"""GPU tier: the context ABI (rmsf_ctx_* / rmsf_push_* / rmsf_multi_*), i.e. the
torch-free boundary a C / MPI / ctypes host binds, vs the oracle restatement
of RMSF.py and the committed golden vectors (1e-6 A absolute, the north
star's tolerance).

Covered: the three modes, host (stager) and device pushes, chunked pushes
(running Chan fold), gathered selections and masses, explicit references,
checkpoint restore (set_partial), XTC pushes, P contexts of one process
merged on the host and over RCCL (ncclCommInitAll on one device), the
callback transport across two processes (gloo), the plain-C host program,
and the error contract."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG, ROOT
from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def c1():
    d = np.load(os.path.join(GOLDEN, "c1_synth.npz"))
    traj = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, int(d["n_frames"]), d["motion"])
    return d, traj


def _script(ctx, traj, align, mode_push, device=False, chunks=1):
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, PUSH_WELFORD
    x = torch.tensor(traj, device="cuda") if device else traj
    parts = np.array_split(np.arange(len(traj)), chunks)
    if align:
        ctx.set_reference_frame(x[0])
    if align == "average":
        for p in parts:
            ctx.push(x[p[0]:p[-1] + 1], PUSH_ALIGN_SUM)
        ctx.allreduce_sum()
        ctx.set_reference_average()
    for p in parts:
        ctx.push(x[p[0]:p[-1] + 1], PUSH_ALIGN_WELFORD if align else PUSH_WELFORD)
    ctx.chan_merge()
    return ctx.rmsf()


@pytest.mark.parametrize("align,tag", [(None, "none"), ("frame0", "frame0"), ("average", "average")])
@pytest.mark.parametrize("device", [False, True])
def test_context_modes_vs_golden(c1, align, tag, device):
    from rmsf_amd.context import Context
    d, traj = c1
    with Context(traj.shape[1], sel=d["sel"]) as ctx:
        rmsf = _script(ctx, traj, align, None, device=device)
        np.testing.assert_allclose(rmsf, d[f"rmsf_{tag}_P1"], rtol=0, atol=TOL)
        n, mean, m2 = ctx.partial()
        assert n == 98
        np.testing.assert_allclose(mean, d[f"mean_{tag}"], rtol=0, atol=1e-6)
        if align == "average":
            np.testing.assert_allclose(ctx.average(), d["average"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("chunks", [2, 7, 98])
def test_context_chunked_pushes(c1, chunks):
    """Pushes of any size fold into the same running state (Chan, RMSF.py:36-41)."""
    from rmsf_amd.context import Context
    d, traj = c1
    with Context(traj.shape[1], sel=d["sel"]) as ctx:
        rmsf = _script(ctx, traj, "average", None, chunks=chunks)
    np.testing.assert_allclose(rmsf, d["rmsf_average_P1"], rtol=0, atol=TOL)


def test_context_masses_staging_and_step(c1):
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, Context
    d, traj = c1
    exp = O.rmsf_script(traj, d["sel"], d["masses"], size=1, align="average", start=0, stop=98, step=3)["rmsf"]
    with Context(traj.shape[1], sel=d["sel"], masses=d["masses"]) as ctx:
        ctx.set_staging(batch_frames=4, n_slots=1, n_threads=2)
        ctx.set_reference_frame(traj[0])
        ctx.push(traj, PUSH_ALIGN_SUM, step=3)
        ctx.allreduce_sum()
        ctx.set_reference_average()
        ctx.push(traj, PUSH_ALIGN_WELFORD, step=3)
        np.testing.assert_allclose(ctx.rmsf(), exp, rtol=0, atol=TOL)


def test_context_explicit_reference_and_contiguous_selection():
    """rmsf_set_reference with a caller's centred reference == the frame form;
    no selection = atoms 0..n_sel-1 (the contiguous path)."""
    from rmsf_amd.context import PUSH_ALIGN_WELFORD, Context
    from rmsf_amd.synth import motion_table
    traj = SY.frames(4, 900, 0, 37, motion_table(5, 37))
    com, ref = O.centred_reference(traj[5][:600])
    exp = O.rmsf_script(traj[:, :600], None, None, size=1, align="frame0", ref_frame=5)["rmsf"]
    with Context(900, n_sel=600) as ctx:
        ctx.set_reference(ref, com)
        ctx.push(traj, PUSH_ALIGN_WELFORD)
        np.testing.assert_allclose(ctx.rmsf(), exp, rtol=0, atol=TOL)
        ctx.reset()
        ctx.set_reference_frame(traj[5])
        ctx.push(torch.tensor(traj, device="cuda"), PUSH_ALIGN_WELFORD)
        np.testing.assert_allclose(ctx.rmsf(), exp, rtol=0, atol=TOL)


def test_context_set_partial_restores_state(c1):
    from rmsf_amd.context import PUSH_WELFORD, Context
    d, traj = c1
    with Context(traj.shape[1], sel=d["sel"]) as a, Context(traj.shape[1], sel=d["sel"]) as b:
        a.push(traj[:40], PUSH_WELFORD)
        n, mean, m2 = a.partial()
        b.set_partial(n, mean, m2)   # checkpoint -> restore
        b.push(traj[40:], PUSH_WELFORD)
        np.testing.assert_allclose(b.rmsf(), d["rmsf_none_P1"], rtol=0, atol=TOL)


@pytest.mark.parametrize("P", [2, 3, 8, 120])
@pytest.mark.parametrize("align", ["average", None])
def test_context_group_in_process(c1, P, align):
    """P contexts of one process, RMSF.py:65-69 blocks, merged by the
    in-process host fold (P > n_frames leaves empty ranks)."""
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, PUSH_WELFORD, Context
    from rmsf_amd.parallel import blocks
    d, traj = c1
    if P == 120 and align is None:
        pytest.skip("one empty-rank case is enough")
    import os
    print(f"\n[P={P}] process threads before: {len(os.listdir('/proc/self/task'))}", flush=True)
    ctxs = [Context(traj.shape[1], sel=d["sel"]) for _ in range(P)]
    bl = blocks(98, P)
    if align:
        for c in ctxs:
            c.set_reference_frame(traj[0])
        for c, (b0, b1) in zip(ctxs, bl):
            c.push(traj[b0:b1], PUSH_ALIGN_SUM)
        Context.multi_allreduce_sum(ctxs)
        for c in ctxs:
            c.set_reference_average()
    for c, (b0, b1) in zip(ctxs, bl):
        c.push(traj[b0:b1], PUSH_ALIGN_WELFORD if align else PUSH_WELFORD)
    Context.multi_chan_merge(ctxs)
    exp = O.rmsf_script(traj, d["sel"], None, size=P, align=align)["rmsf"]
    for c in ctxs:
        np.testing.assert_allclose(c.rmsf(), exp, rtol=0, atol=TOL)
        c.close()


def test_context_rccl_single_device(c1):
    """The RCCL transport: ncclCommInitAll over one device, and
    ncclCommInitRank from a unique id (nranks = 1) -- the same collectives a
    multi-GPU run issues, on the one device this box has."""
    from rmsf_amd.context import Context
    d, traj = c1
    a = Context(traj.shape[1], sel=d["sel"])
    Context.init_all([a])
    np.testing.assert_allclose(_script(a, traj, "average", None), d["rmsf_average_P1"], rtol=0, atol=TOL)
    b = Context(traj.shape[1], sel=d["sel"])
    b.init_rccl(Context.unique_id(), 1, 0)
    np.testing.assert_allclose(_script(b, traj, "frame0", None), d["rmsf_frame0_P1"], rtol=0, atol=TOL)
    a.close()
    b.close()


def test_context_push_xtc(tmp_path):
    from oracle import xtc_py
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, Context
    from rmsf_amd.synth import motion_table
    from rmsf_amd.xtc import XTCFile, write_xtc
    traj = SY.frames(8, 500, 0, 30, motion_table(9, 30))
    path = str(tmp_path / "t.xtc")
    write_xtc(path, traj)
    q = xtc_py.read_xtc(path)
    sel = np.arange(3, 500, 4)
    exp = O.rmsf_script(q, sel, None, size=1, align="average", start=2, stop=29, step=2)["rmsf"]
    with XTCFile(path) as x, Context(500, sel=sel) as ctx:
        ctx.set_staging(batch_frames=5)
        ctx.set_reference_frame(q[0])
        ctx.push_xtc(x, 2, 29, 2, PUSH_ALIGN_SUM)
        ctx.allreduce_sum()
        ctx.set_reference_average()
        ctx.push_xtc(x, 2, 29, 2, PUSH_ALIGN_WELFORD)
        np.testing.assert_allclose(ctx.rmsf(), exp, rtol=0, atol=TOL)


def test_context_errors(c1):
    from rmsf_amd import RmsfEmptyError, RmsfError
    from rmsf_amd.context import PUSH_ALIGN_WELFORD, Context
    d, traj = c1
    with pytest.raises(RmsfError, match="out of range"):
        Context(10, sel=[0, 10])
    with Context(traj.shape[1], sel=d["sel"]) as ctx:
        with pytest.raises(RmsfError, match="before a reference"):
            ctx.push(traj[:3], PUSH_ALIGN_WELFORD)
        with pytest.raises(RmsfEmptyError):
            ctx.rmsf()
        with pytest.raises(RmsfEmptyError):
            ctx.set_reference_average()
        with pytest.raises(RmsfEmptyError):
            ctx.chan_merge()
        with pytest.raises(RmsfError, match="bad mode"):
            ctx.push(traj[:3], 9)


def test_plain_c_host_program(c1, tmp_path):
    """mdanalysis-mpi_amd/lib/rmsf_demo: RMSF.py's script written against the
    C ABI alone, P contexts, host pushes in halves; --device: the blocks in
    HBM and the one-process step (rmsf_multi_push_frames +
    rmsf_multi_chan_merge_root); exact: RMSF_PUSH_EXACT and
    rmsf_multi_chan_merge_exact, the script's own bits."""
    d, traj = c1
    exe = os.path.join(PKG, "lib", "rmsf_demo")
    f = tmp_path / "traj.f32"
    s = tmp_path / "sel.i64"
    traj.astype(np.float32).tofile(f)
    d["sel"].astype(np.int64).tofile(s)
    for P, mode, tag, extra in [(1, "average", "rmsf_average_P1", []), (2, "average", "rmsf_average_P2", []),
                                (8, "frame0", "rmsf_frame0_P8", []), (2, "none", "rmsf_none_P2", []),
                                (1, "average", "rmsf_average_P1", ["--rccl"]),
                                # the one-process step on HBM blocks: multi push + reduce to context 0
                                (2, "none", "rmsf_none_P2", ["--device"]), (8, "frame0", "rmsf_frame0_P8", ["--device"]),
                                (2, "average", "rmsf_average_P2", ["--device"]),
                                (1, "none", "rmsf_none_P1", ["--device", "--rccl"])]:
        out = tmp_path / f"rmsf_{P}_{mode}.f64"
        r = subprocess.run([exe, str(f), "98", str(traj.shape[1]), str(s), "214", str(P), mode, str(out)] + extra,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout.count("Process:") == P
        np.testing.assert_allclose(np.fromfile(out, dtype=np.float64), d[tag], rtol=0, atol=TOL)
    # exact: RMSF_PUSH_EXACT + rmsf_multi_chan_merge_exact (mpi4py's order), bit for bit
    for P in (1, 4, 5):
        out = tmp_path / f"rmsf_{P}_exact.f64"
        r = subprocess.run([exe, str(f), "98", str(traj.shape[1]), str(s), "214", str(P), "exact", str(out)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        want = O.rmsf_script(traj, d["sel"], None, size=P, align=None, merge_order="mpi4py")["rmsf"]
        np.testing.assert_array_equal(np.fromfile(out, dtype=np.float64).view(np.uint64), want.view(np.uint64))


# ---- callback transport across processes (gloo on cuda:0) -------------------
def _cb_worker(rank, size, port, q, shifted=False):
    sys.path[:0] = [ROOT, PKG]
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(port, rank, size)
    try:
        from oracle import synth as SY2
        from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, Context
        from rmsf_amd.parallel import blocks
        from rmsf_amd.synth import motion_table
        traj = SY2.frames(2, 700, 0, 41, motion_table(3, 41))
        sel = np.arange(5, 700, 3)
        b0, b1 = blocks(41, size)[rank]
        with Context(700, sel=sel) as c:
            c.set_reference_frame(traj[0])
            c.push(traj[b0:b1], PUSH_ALIGN_SUM)
            c.allreduce_sum()          # rmsf_ctx_allreduce_sum + torch.distributed callback
            c.set_reference_average()
            c.push(traj[b0:b1], PUSH_ALIGN_WELFORD)
            c.chan_merge(shifted=shifted)  # rmsf_ctx_chan_merge[_shifted] + callback
            q.put((rank, c.rmsf(), c.partial()[0]))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shifted", [False, True])
@pytest.mark.parametrize("size", [2, 3])
def test_context_callback_transport_processes(size, shifted):
    from conftest import spawn_ranks
    from rmsf_amd.synth import motion_table
    out = spawn_ranks(_cb_worker, size, lambda r, init, q: (r, size, init, q, shifted), timeout=100)
    traj = SY.frames(2, 700, 0, 41, motion_table(3, 41))
    exp = O.rmsf_script(traj, np.arange(5, 700, 3), None, size=size, align="average")["rmsf"]
    for rank, rmsf, n in out:
        assert n == 41, rmsf
        np.testing.assert_allclose(rmsf, exp, rtol=0, atol=TOL)


def test_multi_merge_contexts_with_different_references():
    """rmsf_multi_chan_merge over contexts aligned to DIFFERENT references
    (each to a frame of its own block): the one-all-reduce shifted merge
    would use one context's shift for all of them, so the reference digests
    differ and the exact two-pass Chan merge runs (RMSF.py:36-41 over the
    contexts' own partials); with equal references the shifted form runs and
    agrees with the same fold."""
    from rmsf_amd.context import PUSH_ALIGN_WELFORD, Context
    from rmsf_amd.synth import motion_table
    traj = SY.frames(6, 400, 0, 30, motion_table(7, 30))
    sel = np.arange(1, 400, 3)
    for refs in ([0, 10, 20], [4, 4, 4]):
        ctxs = [Context(400, sel=sel) for _ in range(3)]
        parts = []
        for c, r, (b0, b1) in zip(ctxs, refs, [(0, 10), (10, 20), (20, 30)]):
            c.set_reference_frame(traj[r])
            c.push(traj[b0:b1], PUSH_ALIGN_WELFORD)
            n, mean, m2 = c.partial()
            parts.append([n, mean, m2])
        Context.multi_chan_merge(ctxs)
        T, mu, M = O.chan_fold(parts)
        exp = np.sqrt(M.sum(axis=1) / T)
        for c in ctxs:
            np.testing.assert_allclose(c.rmsf(), exp, rtol=0, atol=1e-9)
            n, mean, _ = c.partial()
            assert n == 30
            np.testing.assert_allclose(mean, mu, rtol=0, atol=1e-9)
            c.close()


def test_shifted_merge_needs_a_reference():
    """rmsf_ctx_chan_merge_shifted refuses a context that holds no reference
    (its shift); the in-process rmsf_multi_chan_merge then keeps the
    two-pass form by itself."""
    import ctypes

    from rmsf_amd import RmsfError
    from rmsf_amd.context import PUSH_WELFORD, Context
    from rmsf_amd._lib import call
    traj = SY.frames(3, 200, 0, 9)

    @ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p)
    def noop(buf, count, stream, user):  # a one-rank "all-reduce"
        return 0

    with Context(200) as c:
        c.push(traj, PUSH_WELFORD)
        with pytest.raises(RmsfError):
            call("rmsf_ctx_chan_merge_shifted", c._h, ctypes.cast(noop, ctypes.c_void_p), None)
    with Context(200) as a, Context(200) as b:
        a.push(traj[:4], PUSH_WELFORD)
        b.push(traj[4:], PUSH_WELFORD)
        Context.multi_chan_merge([a, b])
        exp = O.rmsf_script(traj, None, None, size=2, align=None)["rmsf"]
        np.testing.assert_allclose(a.rmsf(), exp, rtol=0, atol=TOL)
