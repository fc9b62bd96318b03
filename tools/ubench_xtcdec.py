"""Host side of the GPU XTC pipeline (not product code): time per
rmsf_xtcdec_decode call (pread into the pinned slot + async H2D + launch) vs
the whole pass, for a 250k-atom file.
    python tools/ubench_xtcdec.py [frames] [batch] [slots] [threads]"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from oracle import synth as SY  # noqa: E402
from rmsf_amd.sources import XtcDecoder  # noqa: E402
from rmsf_amd.xtc import XTCFile, write_xtc  # noqa: E402


def main():
    nf, batch, slots, threads = ([int(a) for a in sys.argv[1:]] + [2048, 715, 4, 16][len(sys.argv) - 1:])[:4]
    n_atoms = 250_000
    path = os.path.join(tempfile.mkdtemp(), "c5.xtc")
    for f in range(0, nf, 256):
        write_xtc(path, SY.frames(0, n_atoms, f, min(256, nf - f)), append=f > 0)
    size = os.path.getsize(path)
    x = XTCFile(path)
    torch.cuda.init()
    s = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    with open(path, "rb") as fh:
        while fh.read(1 << 28):
            pass
    print(f"file {size / 1e9:.2f} GB; plain python read {size / (time.perf_counter() - t0) / 1e9:.1f} GB/s")
    for rep in range(3):
        dec = XtcDecoder(x, batch, slots, threads)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        calls = []
        for f in range(0, nf, batch):
            n = min(batch, nf - f)
            t = time.perf_counter()
            slot, _ = dec.decode(f, n, 1, s)
            calls.append(time.perf_counter() - t)
            dec.release(slot, s)
        t_issue = time.perf_counter() - t0
        dec.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {rep}: pass {dt * 1e3:.0f} ms = {nf / dt:.0f} frames/s; host issue {t_issue * 1e3:.0f} ms "
              f"(per call {', '.join(f'{c * 1e3:.0f}' for c in calls)} ms; {size / sum(calls) / 1e9:.1f} GB/s)")
        dec.close()


if __name__ == "__main__":
    main()
