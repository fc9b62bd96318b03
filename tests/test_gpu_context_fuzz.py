"""GPU tier: a randomised state-machine test of one context's running state.

Round 4 made the context lazier: a push's fold is deferred until the state
is next used (so a merge can fold and pack in one launch), a reset only marks
the state, and a recorded slab push runs at the merge or whole at the next
other call.  Every entry point that touches the running state must therefore
see exactly what the eager context would have held.  This drives one context
through random sequences of

  push (host or device frames, Welford or sum), reset (Welford / sum / both),
  get_partial, get_sum, rmsf, set_partial, the one-context merge (with or
  without a shift frame, root or all-reduce), multi push of one context,

and checks every read against a numpy model of RMSF.py's statistics (Chan's
merge of the pushed blocks, RMSF.py:36-41 and :137-138; the f64 sum of
:103), within 1e-9 (the device folds in a different order).
"""
import numpy as np
import pytest
import torch

from oracle import synth as SY

pytestmark = pytest.mark.gpu


class Model:
    """(n, mean, M2) and (n, sum) of the pushed frames, merged in f64."""

    def __init__(self, n_coord):
        self.nc = n_coord
        self.reset(3)

    def reset(self, what):
        if what & 1:
            self.n, self.mean, self.m2 = 0, np.zeros(self.nc), np.zeros(self.nc)
        if what & 2:
            self.ns, self.sum = 0, np.zeros(self.nc)

    def welford(self, x):  # x [f, n_coord] f64
        f = len(x)
        if not f:
            return
        mu2 = x.mean(axis=0)
        M2b = ((x - mu2) ** 2).sum(axis=0)
        if self.n == 0:
            self.n, self.mean, self.m2 = f, mu2, M2b
            return
        n = self.n + f
        d = mu2 - self.mean
        self.m2 = self.m2 + M2b + d * d * self.n * f / n
        self.mean = self.mean + d * f / n
        self.n = n

    def add_sum(self, x):
        self.ns += len(x)
        self.sum = self.sum + x.sum(axis=0)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_context_state_machine(seed):
    from rmsf_amd import RmsfEmptyError, RmsfError
    from rmsf_amd.context import PUSH_SUM, PUSH_WELFORD, Context
    rng = np.random.default_rng(seed)
    n_atoms = int(rng.integers(3, 400))
    sel = np.sort(rng.choice(n_atoms, int(rng.integers(1, n_atoms + 1)), replace=False)) if seed % 2 else None
    traj = SY.frames(40 + seed, n_atoms, 0, 300)
    dev = torch.tensor(traj, device="cuda")
    cols = np.arange(n_atoms) if sel is None else sel
    sel_rows = traj[:, cols].reshape(300, -1).astype(np.float64)
    n_sel = len(cols)
    c = Context(n_atoms, sel=sel)
    m = Model(3 * n_sel)
    merged_away = False
    tol = dict(rtol=1e-9, atol=1e-9)
    for step in range(160):
        op = rng.choice(["push_w", "push_w", "push_s", "reset", "partial", "sum", "rmsf", "set_partial",
                         "merge", "multi"])
        f0 = int(rng.integers(0, 300))
        f1 = int(rng.integers(f0, min(300, f0 + 60) + 1))
        on_dev = bool(rng.integers(0, 2))
        if op in ("push_w", "push_s"):
            x = dev[f0:f1] if on_dev else traj[f0:f1]
            c.push(x, PUSH_WELFORD if op == "push_w" else PUSH_SUM)
            (m.welford if op == "push_w" else m.add_sum)(sel_rows[f0:f1])
            if op == "push_w":
                merged_away = False
        elif op == "reset":
            what = int(rng.integers(1, 4))
            c.reset(welford=bool(what & 1), sum=bool(what & 2))
            m.reset(what)
            if what & 1:
                merged_away = False
        elif op == "partial":
            if merged_away:
                with pytest.raises(RmsfError):
                    c.partial()
                continue
            n, mean, m2 = c.partial()
            assert n == m.n, (step, op)
            np.testing.assert_allclose(mean.reshape(-1), m.mean, **tol, err_msg=f"step {step}")
            np.testing.assert_allclose(m2.reshape(-1), m.m2, **tol, err_msg=f"step {step}")
        elif op == "sum":
            n, s = c.sum()
            assert n == m.ns
            np.testing.assert_allclose(s.reshape(-1), m.sum, **tol, err_msg=f"step {step}")
        elif op == "rmsf":
            if merged_away:
                with pytest.raises(RmsfError):
                    c.rmsf()
            elif m.n == 0:
                with pytest.raises(RmsfEmptyError):
                    c.rmsf()
            else:
                np.testing.assert_allclose(c.rmsf(), np.sqrt(m.m2.reshape(-1, 3).sum(axis=1) / m.n), **tol,
                                           err_msg=f"step {step}")
        elif op == "set_partial":
            n = int(rng.integers(0, 50))
            mean = rng.normal(50, 5, 3 * n_sel)
            m2 = rng.uniform(0, 10, 3 * n_sel) if n else np.zeros(3 * n_sel)
            c.set_partial(n, mean, m2)
            m.n, m.mean, m.m2 = n, (mean if n else np.zeros(3 * n_sel)), m2
            merged_away = False
        elif op == "merge":
            if m.n == 0 or merged_away:
                continue
            if rng.integers(0, 2):
                c.set_merge_shift_frame(dev[int(rng.integers(0, 300))] if on_dev else traj[int(rng.integers(0, 300))])
            Context.multi_chan_merge([c], root=0 if rng.integers(0, 2) else None)
            # one context: the merge leaves its own statistics (to rounding)
        elif op == "multi":
            # the one-process step on one context: reset + push (+ shift frame) in one call
            x = dev[f0:max(f1, f0 + 1)]
            shift = [dev[int(rng.integers(0, 300))]] if rng.integers(0, 2) else None
            Context.multi_push_frames([c], [x], PUSH_WELFORD, shift_frames=shift)
            m.reset(1)
            m.welford(sel_rows[f0:max(f1, f0 + 1)])
            merged_away = False
    c.close()
