"""GPU XTC decode throughput (not product code): rmsf_xtc_decode_records on
250k-atom frames, one wave per frame.  K distinct frames are written once;
the record table points at them cyclically so N frames decode from device
memory.  (Round 1 also measured one LANE per frame, 1-64 frames per wave:
slower below ~8k frames -- profiles/r01_workloads/ubench_xtc_decode.txt.)
    python tools/ubench_xtc.py [N ...]"""
import ctypes
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from oracle import synth as SY  # noqa: E402
from rmsf_amd._lib import call, load  # noqa: E402
from rmsf_amd.xtc import XTCFile, write_xtc  # noqa: E402


def water_like(rng, n_atoms, n_frames):
    w = n_atoms // 3
    o = rng.uniform(0, 150, (w, 3))
    base = np.repeat(o, 3, axis=0) + rng.normal(0, 0.8, (3 * w, 3))
    base = np.concatenate([base, rng.uniform(0, 150, (n_atoms - 3 * w, 3))])
    return np.stack([base + rng.normal(0, 0.3, base.shape) for _ in range(n_frames)]).astype(np.float32)


def protein_like(rng, n_atoms, n_frames):
    """Chains of bonded atoms (1.5 A steps): frequent runs and flag bits,
    the hard case for the decoder's clean-group scan (~18 % flagged groups)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_xtc import _protein_like
    return _protein_like(rng, n_atoms, n_frames)


def main():
    ns = [int(a) for a in sys.argv[1:]] or [400, 4096]
    lib = load()
    n_atoms, K = 250_000, 32
    dev = torch.device("cuda")
    for kind in os.environ.get("UB_KINDS", "uniform,water,protein").split(","):
        rng = np.random.default_rng(1)
        x = (SY.frames(0, n_atoms, 0, K) if kind == "uniform" else
             water_like(rng, n_atoms, K) if kind == "water" else protein_like(rng, n_atoms, K))
        path = os.path.join(tempfile.mkdtemp(), "u.xtc")
        write_xtc(path, x)
        with XTCFile(path) as f:
            rec = [f.record(i) for i in range(f.n_frames)]
        words = torch.as_tensor(np.fromfile(path, dtype=np.uint32).view(np.int32)).to(dev)
        print(f"{kind}: {os.path.getsize(path) / K / n_atoms:.2f} B/atom compressed", flush=True)
        for N in ns:
            off = torch.as_tensor(np.array([rec[i % K][0] // 4 for i in range(N)], dtype=np.int64)).to(dev)
            ln = torch.as_tensor(np.array([rec[i % K][1] // 4 for i in range(N)], dtype=np.int64)).to(dev)
            out = torch.empty((N, n_atoms, 3), dtype=torch.float32, device=dev)
            st = torch.empty(N, dtype=torch.int32, device=dev)
            ref = None
            for mode in (0,):
                def go():
                    rc = lib.rmsf_xtc_decode_records(
                        ctypes.c_void_p(words.data_ptr()), ctypes.c_void_p(off.data_ptr()),
                        ctypes.c_void_p(ln.data_ptr()), ctypes.c_int64(N), ctypes.c_int64(n_atoms),
                        ctypes.c_void_p(out.data_ptr()), ctypes.c_int64(3 * n_atoms), ctypes.c_void_p(st.data_ptr()),
                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0
                go()
                torch.cuda.synchronize()
                t = time.perf_counter()
                go()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                ok = bool((st == 0).all())
                if ref is None:
                    ref = out[:K].clone()
                same = bool(torch.equal(out[:K], ref))
                print(f"  N={N:5d} mode={mode:3d}: {dt * 1e3:8.1f} ms  {N / dt:9.0f} frames/s  "
                      f"{N * n_atoms / dt:.3e} atoms/s  ok={ok} same={same}", flush=True)
            del out


if __name__ == "__main__":
    main()
