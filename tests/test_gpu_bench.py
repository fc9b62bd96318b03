"""bench.py on the GPU at small sizes: the JSON line keeps the driver's
contract, the roofline is computed from the bytes of the timed launches
(never above the data's own bytes), and the one-process multi-device form
(``--gpus N`` without a launcher; a labelled rehearsal on a one-GPU box)
computes the same RMSF as the oracle's ``mpirun -n N`` emulation."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("align", ["none", "frame0", "average"])
def test_single_process_rehearsal_matches_oracle(align, capsys):
    a = bench.parse(["--gpus", "3", "--rehearse", "--n-atoms", "1500", "--frames", "61", "--steps", "2",
                     "--warmup", "1", "--no-cpu-baseline", "--align", align])
    wl = bench.resolve(a, 3)
    bench.main_single_process(a, wl, None)
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["n_gpus"] == 3 and line["rehearsal"] is True and line["devices"] == [0, 0, 0]
    assert line["scaling"] == "strong" and line["config"]["n_frames_total"] == 61
    assert line["roofline"]["launches"] == 3 * 2 * (2 if align == "average" else 1)
    assert 0 < line["roofline"]["frac"] < 1.0
    # the one-process N > 1 line reports its merge, per device
    mt = line["merge_timing"]
    assert len(mt["per_device_ms_per_step"]) == 3 and mt["max_ms_per_step"] == max(mt["per_device_ms_per_step"])
    assert all(v > 0 for v in mt["per_device_ms_per_step"])
    assert len(line["roofline"]["per_device_gbs"]) == 3
    assert line["sanity"]["ok"]
    from rmsf_amd.synth import motion_table

    mt = motion_table(1, 61) if align != "none" else None
    traj = SY.frames(0, 1500, 0, 61, mt)
    exp = O.rmsf_script(traj, None, None, size=3, align=None if align == "none" else align)["rmsf"]
    assert abs(line["rmsf_checksum"] - float(exp.sum())) < 1e-6 * len(exp)


def test_io_modes_small(capsys):
    """modes.c4_share / modes.c5_xtc at reduced sizes: the one-process slab
    step's timings and the XTC stream's figures, each with its sanity check
    (rmsf_amd.synth.rmsf_sanity) passing."""
    from rmsf_amd.engine import Engine
    eng = Engine()
    a = bench.parse(["--mode-steps", "2"])
    c4 = bench.c4_share_mode(eng, a, 3.6, n_atoms=1_000_000, nf=33)
    assert c4["accumulate_launches_per_step"] == 2          # two atom slabs
    assert c4["sanity"]["ok"] and c4["ms_per_step"] > 0 and 0 < c4["accumulate_frac"] < 1
    assert c4["exposed_merge_ms_per_step"] > 0
    c5 = bench.c5_xtc_mode(eng, a, n_atoms=20000, nf=300)
    assert c5["sanity"]["ok"] and c5["decode_kernel"]["all_frames_ok"]
    assert c5["frames_per_s"] > 0 and c5["h2d_gbs"] > 0 and c5["decode_kernel"]["avg_ms"] > 0


def test_bench_cli_small_json_line():
    cmd = [sys.executable, "bench.py", "--n-atoms", "20000", "--frames", "300", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--mode-steps", "1", "--no-io-modes"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["scaling"] == "strong"
    rf = line["roofline"]
    assert rf["launches"] == 3 and 0 < rf["frac"] < 1.0
    assert rf["algorithmic_bytes_per_launch"] == 12 * 20000 * 300
    m = line["modes"]
    for name in ("c3_frame0", "rmsf_py_average"):
        assert 0 < m[name]["accumulate_hbm_gbs"] < 8000 and 0 < m[name]["superpose_hbm_gbs"] < 8000
    x = m["c2_exact"]
    assert x["kernel"] == "k_welford_seq" and 0 < x["hbm_frac"] < 1.0
    assert x["max_abs_rmsf_diff_vs_headline"] < 1e-12


def test_bench_batched_launches_roofline_below_peak():
    # several launches per step of different sizes: bytes are charged per launch
    cmd = [sys.executable, "bench.py", "--n-atoms", "20000", "--frames", "1000", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-modes", "--align", "frame0", "--batch-frames", "300"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rf = json.loads(r.stdout.strip().splitlines()[-1])["roofline"]
    assert rf["launches"] == 2 * 4  # 300+300+300+100 per step
    assert rf["algorithmic_bytes_per_launch"] == pytest.approx(12 * 20000 * 250)
    assert 0 < rf["frac"] < 1.0


@pytest.mark.parametrize("align", ["none", "frame0"])
def test_one_process_form_at_one_gpu_matches_n1_line(align):
    """Verdict r5 item 5: ``bench.py --gpus 1 --one-process`` runs the
    one-process context form (main_single_process) on one real device -- a
    one-rank ncclCommInitAll communicator and the RCCL merge path over it, no
    peer setup -- and its line agrees with the N = 1 pipeline line: the same
    RMSF checksum, a roofline below peak, no merge_timing (one device)."""
    base = [sys.executable, "bench.py", "--gpus", "1", "--n-atoms", "20000", "--frames", "300", "--steps", "3",
            "--warmup", "1", "--no-cpu-baseline", "--no-modes", "--align", align]
    lines = {}
    for form, extra in (("pipeline", []), ("contexts", ["--one-process"])):
        r = subprocess.run(base + extra, cwd=ROOT, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines[form] = json.loads(r.stdout.strip().splitlines()[-1])
    p, c = lines["pipeline"], lines["contexts"]
    assert c["devices"] == [0] and c["rehearsal"] is False and "RCCL" in c["config"]["parallelism"]
    assert "merge_timing" not in c and "merge_timing" not in p
    for ln in (p, c):
        assert ln["n_gpus"] == 1 and 0 < ln["roofline"]["frac"] < 1.0 and ln["sanity"]["ok"]
    assert c["roofline"]["algorithmic_bytes_per_launch"] == p["roofline"]["algorithmic_bytes_per_launch"]
    assert abs(c["rmsf_checksum"] - p["rmsf_checksum"]) <= 1e-11 * abs(p["rmsf_checksum"])


def test_single_process_refuses_missing_devices():
    import torch

    n = torch.cuda.device_count() + 1
    with pytest.raises(SystemExit, match="visible"):
        bench.device_plan(n, torch.cuda.device_count(), False)
    np.testing.assert_equal(bench.device_plan(n, torch.cuda.device_count(), True)[0], [0] * n)


def _free_port() -> int:
    """A TCP port on 127.0.0.1 that was free a moment ago (bind to port 0)."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("align", ["none", "frame0", "average"])
def test_torchrun_two_ranks_same_result_as_one_gpu(align):
    """The driver's multi-GPU form (torch.distributed.run, one process per
    rank; gloo ranks sharing the one GPU here, RCCL on a node): strong
    scaling of one trajectory over 2 ranks gives the 1-GPU run's RMSF (the
    one-all-reduce merge vs the single-device fold), and the oracle's."""
    common = ["--n-atoms", "6000", "--frames", "301", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--no-modes", "--align", align]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    one = subprocess.run([sys.executable, "bench.py"] + common, cwd=ROOT, capture_output=True, text=True,
                         timeout=300, env=env)
    assert one.returncode == 0, one.stderr[-2000:]
    for _ in range(3):  # a port the kernel just handed out; retried if taken meanwhile
        two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                              "--gpus", "2", "--backend", "gloo"] + common, cwd=ROOT, capture_output=True, text=True,
                             timeout=300, env=env)
        if two.returncode == 0 or "EADDRINUSE" not in two.stderr:
            break
    assert two.returncode == 0, two.stderr[-2000:]
    l1 = json.loads(one.stdout.strip().splitlines()[-1])
    l2 = json.loads(two.stdout.strip().splitlines()[-1])
    assert l2["n_gpus"] == 2 and l2["config"]["n_frames_per_gpu"] == 150
    assert l2["config"]["merge"] == "reduce to rank 0 (RMSF.py:143)"  # the default, RMSF.py:143's reduce
    # the roofline describes both ranks (KernelTimer totals all-reduced)
    rf = l2["roofline"]
    sweeps = 2 if align == "average" else 1
    assert rf["ranks"] == 2 and rf["launches"] == 2 * 2 * sweeps and rf["per_device_launches"] == [2 * sweeps] * 2
    assert len(rf["per_device_gbs"]) == 2 and all(0 < g < 8000 for g in rf["per_device_gbs"])
    assert rf["slowest_rank"] in (0, 1) and rf["slowest_rank_gbs"] == min(rf["per_device_gbs"])
    assert min(rf["per_device_gbs"]) <= rf["achieved"] <= max(rf["per_device_gbs"])
    if align != "none":
        assert len(l2["superpose"]["per_device_hbm_gbs"]) == 2
    assert l1["rmsf_checksum"] == pytest.approx(l2["rmsf_checksum"], rel=1e-12)
    from rmsf_amd.synth import motion_table

    mt = motion_table(1, 301) if align != "none" else None
    traj = SY.frames(0, 6000, 0, 301, mt)
    exp = O.rmsf_script(traj, None, None, size=2, align=None if align == "none" else align)["rmsf"]
    assert abs(l2["rmsf_checksum"] - float(exp.sum())) < 1e-6 * len(exp)


def test_torchrun_merge_slabs_same_checksum():
    """The driver's N>1 form with the final sweep in atom slabs (C4's
    merge overlap, forced at 300k atoms where the flat plan is chunk-aligned):
    2 gloo ranks on the GPU, slabbed and unslabbed give the same RMSF bit for
    bit (two ranks: the sum of two partials is order-free), and the line
    records the slab count."""
    common = ["--n-atoms", "300000", "--frames", "130", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--no-modes", "--gpus", "2", "--backend", "gloo"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    lines = {}
    for k in ("2", "0"):
        for _ in range(3):
            r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                                "--merge-slabs", k] + common, cwd=ROOT, capture_output=True, text=True, timeout=300,
                               env=env)
            if r.returncode == 0 or "EADDRINUSE" not in r.stderr:
                break
        assert r.returncode == 0, r.stderr[-2000:]
        lines[k] = json.loads(r.stdout.strip().splitlines()[-1])
    assert lines["2"]["config"]["merge_slabs"] == 2 and lines["0"]["config"]["merge_slabs"] == 0
    assert lines["2"]["rmsf_checksum"] == lines["0"]["rmsf_checksum"]
    assert lines["2"]["roofline"]["launches"] == 2 * 2 * 2  # 2 ranks x 2 steps x 2 slabs


def test_torchrun_merge_all_same_checksum():
    """``--merge all`` (an all-reduce leaving the result on every rank) and the
    default reduce to rank 0 (RMSF.py:143) give the same RMSF bit for bit
    with two ranks (the sum of two packed partials is order-free)."""
    common = ["--n-atoms", "6000", "--frames", "301", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--no-modes", "--gpus", "2", "--backend", "gloo"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    lines = {}
    for m in ("root", "all"):
        for _ in range(3):
            r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                                "--merge", m] + common, cwd=ROOT, capture_output=True, text=True, timeout=300,
                               env=env)
            if r.returncode == 0 or "EADDRINUSE" not in r.stderr:
                break
        assert r.returncode == 0, r.stderr[-2000:]
        lines[m] = json.loads(r.stdout.strip().splitlines()[-1])
    assert lines["root"]["config"]["merge"].startswith("reduce") and lines["all"]["config"]["merge"] == "all-reduce"
    assert lines["root"]["rmsf_checksum"] == lines["all"]["rmsf_checksum"]


def test_torchrun_merge_scatter_same_checksum():
    """bench --merge scatter (reduce-scatter by atom slices, RMSF gathered to
    rank 0) under the driver's torchrun form, 2 gloo ranks on the GPU: the
    checksum of --merge root, bit for bit (2 ranks: a + b either way)."""
    common = ["--steps", "2", "--warmup", "1", "--n-atoms", "20001", "--frames", "301", "--no-cpu-baseline",
              "--no-modes", "--gpus", "2", "--backend", "gloo"]
    res = {}
    for merge in ("root", "scatter"):
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                            "bench.py", "--merge", merge] + common, cwd=ROOT, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        res[merge] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["scatter"]["config"]["merge"].startswith("reduce-scatter")
    assert res["scatter"]["rmsf_checksum"] == res["root"]["rmsf_checksum"]
    for r in res.values():  # the merge's time on every rank's stream, per step
        mt = r["merge_timing"]
        assert len(mt["per_rank_ms_per_step"]) == 2 and 0 < mt["max_ms_per_step"] < r["ms_per_step"]
