"""pytest config: the ``gpu`` marker and import paths.

``-m "not gpu"`` runs everywhere (oracle vs golden vectors, host logic, the
C-ABI library's symbol table, gloo world_size-2 merges); ``-m gpu`` needs a
MI355X and exercises the HIP kernels through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mdanalysis-mpi_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The product's default (exact=None) runs aligned runs of fewer than 256
# frames through the exact path (pipeline.AUTO_EXACT_FRAMES).  The suite's
# many small aligned cases were written for the frame-parallel kernels, so
# they keep testing those (0 = never; inherited by spawned ranks);
# tests/test_gpu_exact_aligned.py checks the default itself.
os.environ["RMSF_AUTO_EXACT_FRAMES"] = "0"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def spawn_ranks(target, size: int, args_fn, timeout: float = 120.0) -> list:
    """Run ``target`` in ``size`` spawned processes (one torch.distributed
    rank each) and return what they put on the queue.  Ranks rendezvous
    through a fresh file (``init`` = file:// URL: no TCP port to collide
    with), and every child still alive when this returns -- a rank stuck in a
    collective after its peer failed -- is terminated, so a failing case can
    never leave the test run waiting on a hung child.
    ``args_fn(rank, init, q)`` builds each process's arguments."""
    import tempfile

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    d = tempfile.mkdtemp(prefix="rmsf_rdv_")
    init = "file://" + os.path.join(d, "store")
    procs = [ctx.Process(target=target, args=args_fn(r, init, q), daemon=True) for r in range(size)]
    try:
        for p in procs:
            p.start()
        return [q.get(timeout=timeout) for _ in range(size)]
    finally:
        for p in procs:
            p.join(timeout=30)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)


def init_gloo(init: str, rank: int, size: int) -> None:
    """gloo process group over a file rendezvous (see spawn_ranks)."""
    from datetime import timedelta

    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=size, timeout=timedelta(seconds=120))
