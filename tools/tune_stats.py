#!/usr/bin/env python3
"""Times rmsf_superpose (k_frame_stats + k_qcp_frames) on C3 data, 100k atoms
x 20k frames, HIP events on the launch stream (not product code).  Run in the
same gpurun call as tools/ubench_stats (UB_SET=O) to compare on one box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def motion_table_dev(eng, nf):
    from rmsf_amd.synth import motion_table
    global _mt
    _mt = torch.as_tensor(motion_table(1, nf)).to(eng.device)
    return _mt.data_ptr()


def main():
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    eng = Engine()
    n, nf = 100_000, 20_000
    if os.environ.get("TS_ALLOC") == "hip":  # plain hipMalloc instead of torch's caching allocator
        import ctypes
        from rmsf_amd._lib import call
        ptr = ctypes.c_void_p()
        call("rmsf_malloc", ctypes.byref(ptr), 12 * n * nf)

        class _Raw:  # the minimal tensor face generate()/superpose use
            def __init__(self, p):
                self.p = p

            def data_ptr(self):
                return self.p
        traj = _Raw(ptr.value)
        call("rmsf_synth_frames", ptr.value, 3 * n, n, 0, nf, 0,
             motion_table_dev(eng, nf), eng.stream)
    else:
        traj = generate(eng, n, 0, nf, seed=0, motion=motion_table(1, nf))
    ref, info = eng.reference_setup(n, frame_ptr=traj.data_ptr())
    xf = eng.empty(nf, 16)
    wk = eng.empty(eng.workspace_bytes(n, nf) // 8 + 1)
    s = torch.cuda.current_stream()
    kind = os.environ.get("TS_DATA", "synth")
    if kind != "synth":  # same allocation, other bit patterns (data-dependence probe)
        if kind == "const":
            traj.view(torch.int32).fill_(0x3f3f3f3f)
        else:
            traj.uniform_(0.0, 100.0)
        ref, info = eng.reference_setup(n, frame_ptr=traj.data_ptr())
        torch.cuda.synchronize()
    print("data:", kind, flush=True)
    for rep in range(3):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(s)
            eng.superpose(traj.data_ptr(), 3 * n, nf, n, None, None, ref, info, xf, wk)
            b.record(s)
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) for a, b in ev]
        print(f"rmsf_superpose 100k x 20k: median {np.median(t):.3f} ms  min {min(t):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
