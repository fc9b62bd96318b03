"""Device-backed ``second_order_moments`` (RMSF.py:36-41).

``S = (n, mean[N,3], M2[N,3])``; the merge runs in the Chan kernel
(``rmsf_chan_merge``) with T = n1+n2, mu = (n1 mu1 + n2 mu2)/T,
M = M1 + M2 + (n1 n2 / T)(mu2 - mu1)^2.  Accepts numpy arrays (copied to the
device and back) or HIP torch tensors (stays on device).  Merging two empty
partials raises ZeroDivisionError, as the reference does at RMSF.py:39.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import Engine


def second_order_moments(S1, S2):
    n1, mu1, m1 = S1
    n2, mu2, m2 = S2
    on_device = isinstance(mu1, torch.Tensor) and mu1.device.type == "cuda"
    eng = Engine(mu1.device if on_device else None)

    def dev(x):
        t = torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor) else x)
        return t.to(eng.device, torch.float64).contiguous()

    shape = tuple(mu1.shape)
    a_mu, a_m2, b_mu, b_m2 = dev(mu1), dev(m1), dev(mu2), dev(m2)
    if a_mu.shape != b_mu.shape or a_m2.shape != a_mu.shape or b_m2.shape != a_mu.shape:
        raise ValueError("second_order_moments: mean/M2 shapes differ")
    n = a_mu.numel()
    means = torch.stack([a_mu.reshape(-1), b_mu.reshape(-1)])
    m2s = torch.stack([a_m2.reshape(-1), b_m2.reshape(-1)])
    mean_out = eng.empty(n)
    m2_out = eng.empty(n)
    eng.chan_merge(means, m2s, [int(n1), int(n2)], n, mean_out, m2_out)
    T = int(n1) + int(n2)
    if on_device:
        return T, mean_out.view(shape), m2_out.view(shape)
    torch.cuda.current_stream(eng.device).synchronize()
    return T, mean_out.cpu().numpy().reshape(shape), m2_out.cpu().numpy().reshape(shape)
