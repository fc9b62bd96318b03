"""bench.py's argument handling (no GPU): strong scaling of one trajectory
by default, weak scaling on request, and a one-process ``--gpus N`` that
fails loudly when fewer devices are visible unless it is a labelled
rehearsal."""
import pytest

import bench


def test_default_is_strong_scaling_of_c2():
    a = bench.parse(["--gpus", "8"])
    wl = bench.resolve(a, 8)
    assert wl["scaling"] == "strong" and wl["n_total"] == 20_000 and wl["n_atoms"] == 100_000
    assert wl["align"] is None
    assert bench.resolve(bench.parse([]), 1)["n_total"] == 20_000
    # the N = 1 modes: 3 untimed steps before their 3 timed ones
    d = bench.parse([])
    assert d.mode_warmup == 3 and d.mode_steps == 3


def test_weak_scaling_and_c4():
    wl = bench.resolve(bench.parse(["--scaling", "weak"]), 4)
    assert wl["scaling"] == "weak" and wl["n_total"] == 80_000
    wl = bench.resolve(bench.parse(["--workload", "c4"]), 8)
    assert wl["scaling"] == "weak" and wl["n_total"] == 20_000 and wl["n_atoms"] == 1_000_000
    wl = bench.resolve(bench.parse(["--frames-per-gpu", "100"]), 2)
    assert wl["scaling"] == "weak" and wl["n_total"] == 200


def test_too_few_frames_for_the_gpus():
    with pytest.raises(SystemExit):
        bench.resolve(bench.parse(["--frames", "3"]), 4)


def test_device_plan():
    assert bench.device_plan(2, 8, False) == ([0, 1], False)
    assert bench.device_plan(1, 1, False) == ([0], False)
    with pytest.raises(SystemExit, match="2 devices but 1"):
        bench.device_plan(2, 1, False)
    assert bench.device_plan(3, 1, True) == ([0, 0, 0], True)
    with pytest.raises(SystemExit):
        bench.device_plan(2, 0, True)


def test_roofline_sums_bytes_over_launch_time():
    # 3 launches of different sizes: sum(bytes) / sum(time), never > the data
    r = bench.roofline("k", 3, 3.0, 3.0e8)
    assert r["achieved"] == pytest.approx(12 * 3.0e8 / 3.0e-3 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0)
    assert r["algorithmic_bytes_per_launch"] == pytest.approx(12 * 1.0e8)


def test_rank_roofline_describes_every_rank():
    # rank 1 is slower: the line keeps sum(bytes)/sum(time) and names it
    rows = [(2, 1.0, 2.0e8), (2, 1.25, 2.0e8), (2, 1.0, 2.0e8)]
    r = bench.rank_roofline("k_welford_flat_sk", rows)
    assert r["ranks"] == 3 and r["launches"] == 6
    assert r["achieved"] == pytest.approx(12 * 6.0e8 / 3.25e-3 / 1e9)
    assert r["per_device_gbs"] == pytest.approx([2400.0, 1920.0, 2400.0])
    assert r["per_device_launches"] == [2, 2, 2]
    assert r["slowest_rank"] == 1 and r["slowest_rank_gbs"] == pytest.approx(1920.0)
    assert r["slowest_rank_frac"] == pytest.approx(1920.0 / 8000.0)
    one = bench.rank_roofline("k", [(3, 3.0, 3.0e8)])
    assert one["ranks"] == 1 and one["slowest_rank"] == 0 and one["achieved"] == pytest.approx(1200.0)


def _gather_worker(rank, size, init, q):
    from conftest import init_gloo
    import torch.distributed as dist

    init_gloo(init, rank, size)
    rows = bench.gather_rank_rows([rank + 1, 0.5 * (rank + 1), 1.0e6 * (rank + 1)])
    r = bench.rank_roofline("k", rows)
    q.put((rank, rows, r["slowest_rank"], r["launches"]))
    dist.destroy_process_group()


def test_gather_rank_rows_gloo_two_ranks():
    """The N>1 bench line is built from every rank's KernelTimer totals,
    all-reduced in rank order before rank 0 prints (gloo, world size 2)."""
    from conftest import spawn_ranks
    out = sorted(spawn_ranks(_gather_worker, 2, lambda r, init, q: (r, 2, init, q)))
    for rank, rows, slow, launches in out:
        assert rows == [[1.0, 0.5, 1.0e6], [2.0, 1.0, 2.0e6]]
        assert launches == 3 and slow in (0, 1)


def test_merge_defaults_to_reduce_to_root():
    # RMSF.py:143's comm.reduce(root=0) is the bench's N>1 merge; --merge all
    # is the all-reduce, --merge-root the older spelling of the default
    assert bench.parse([]).merge == "root"
    assert bench.parse(["--merge", "all"]).merge == "all"
    assert bench.parse(["--merge", "all", "--merge-root"]).merge == "root"


def test_merge_scatter_and_rehearsal_transport_flags():
    a = bench.parse(["--merge", "scatter", "--gpus", "8", "--rehearse", "--rehearse-transport", "noop"])
    assert a.merge == "scatter" and a.rehearse and a.rehearse_transport == "noop"
    assert bench.parse([]).rehearse_transport == "fold"


def test_script_exact_needs_unaligned_root_or_all():
    """rmsf_mi355x.py --exact is RMSF.py:120-146's own arithmetic: refused
    with alignment or the reduce-scatter merge, before any device work."""
    import subprocess
    import sys

    from conftest import ROOT
    script = f"{ROOT}/mdanalysis-mpi_amd/rmsf_mi355x.py"
    for extra in ([], ["--align", "frame0"], ["--align", "none", "--merge", "scatter"]):
        r = subprocess.run([sys.executable, script, "--synthetic", "10", "5", "--exact", *extra],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 2 and "--exact needs --align none" in r.stderr, (extra, r.stderr[-500:])


def test_script_file_input_forwards_merge_scatter_and_order(tmp_path, monkeypatch):
    """rmsf_mi355x.py with file input passes --merge scatter (and
    --merge-order) on to RMSF, as the --synthetic branch passes them to the
    pipeline (recorded by a stand-in RMSF; CPU only, no device work)."""
    import sys
    import types

    import numpy as np
    import torch

    from conftest import PKG, ROOT
    sys.path[:0] = [PKG]
    import rmsf_amd
    from rmsf_amd.topology import write_gro
    seen = {}

    class FakeRMSF:
        def __init__(self, inp, **kw):
            seen.update(kw, inp=inp)

        def run(self):
            return types.SimpleNamespace(results=types.SimpleNamespace(rmsf=np.ones(2)))

    monkeypatch.setattr(rmsf_amd, "RMSF", FakeRMSF)
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: None)
    gro = str(tmp_path / "t.gro")
    write_gro(gro, np.array([1, 1, 2, 2]), np.array(["ALA"] * 4), np.array(["N", "CA", "N", "CA"]),
              np.zeros((4, 3), np.float32))
    sys.path.insert(0, f"{ROOT}/mdanalysis-mpi_amd")
    import importlib
    script = importlib.import_module("rmsf_mi355x")
    assert script.main(["--topology", gro, "--trajectory", str(tmp_path / "t.xtc"), "--merge", "scatter",
                        "--merge-order", "rank"]) == 0
    assert seen["merge_scatter"] is True and seen["merge_root"] == 0 and seen["merge_order"] == "rank"
    assert script.main(["--topology", gro, "--trajectory", str(tmp_path / "t.xtc"), "--merge", "all"]) == 0
    assert seen["merge_scatter"] is False and seen["merge_root"] is None and seen["merge_order"] == "mpi4py"
