# Times RMSF(host array, align="average", gpus=[0]) with the block staged into HBM once vs streamed twice (not product code).
import sys, time
sys.path[:0] = [".", "mdanalysis-mpi_amd"]
import numpy as np, torch
from rmsf_amd import RMSF
from rmsf_amd import multi
rng = np.random.default_rng(0)
x = (rng.random((1000, 250000, 3), dtype=np.float32) * 100).astype(np.float32)
for label, fit in (("staged", multi._blocks_fit), ("streamed", lambda *a: False)):
    multi._blocks_fit = fit
    RMSF(x[:50], align="average", gpus=[0]).run()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); r = RMSF(x, align="average", gpus=[0]).run(); ts.append(time.perf_counter() - t0)
    print(label, "gpus=[0] average 250k x 1000 host frames: %.1f ms (min of 3)" % (1e3 * min(ts)), flush=True)
