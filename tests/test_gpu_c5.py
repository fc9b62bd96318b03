"""Config C5 at its size (BASELINE.json configs[4]): a 250k-atom XTC
trajectory streamed from the host -- the frame source of RMSF.py:56,92,124.

  * the GPU decoder (kernel-level ``rmsf_xtc_decode_records`` and the
    pinned-slot ``XtcSource(decode="gpu")`` pipeline) is bit-exact against
    the host codec, on the bench's synthetic frames and on protein-like
    frames (chains + water clusters: the run-length and water-swap paths);
  * ``RMSF(path, align="average")`` -- RMSF.py's two sweeps -- matches the
    oracle on a sampled selection within 1e-6 A, and GPU-decoded equals
    host-decoded bit for bit."""
import numpy as np
import pytest

from test_xtc import _protein_like

pytestmark = pytest.mark.gpu

N_ATOMS = 250_000
N_FRAMES = 8
TOL = 1e-6  # Angstrom, north star


def _frames(kind):
    if kind == "synthetic":
        from oracle import synth as SY
        from rmsf_amd.synth import motion_table

        return SY.frames(0, N_ATOMS, 0, N_FRAMES, motion_table(1, N_FRAMES))
    return _protein_like(np.random.default_rng(5), N_ATOMS, N_FRAMES)


@pytest.fixture(scope="module", params=["synthetic", "protein"])
def c5file(request, tmp_path_factory):
    from rmsf_amd.xtc import XTCFile, write_xtc

    p = str(tmp_path_factory.mktemp("c5") / f"{request.param}.xtc")
    write_xtc(p, _frames(request.param))
    with XTCFile(p) as f:
        assert (f.n_atoms, f.n_frames) == (N_ATOMS, N_FRAMES)
        host = f.read(n_threads=8)
    return p, host


def test_kernel_decode_bit_exact(c5file):
    import torch

    from rmsf_amd._lib import call
    from rmsf_amd.xtc import XTCFile

    p, host = c5file
    with XTCFile(p) as f:
        rec = [f.record(i) for i in range(f.n_frames)]
    words = np.fromfile(p, dtype=np.uint32)
    off = np.array([o // 4 for o, _ in rec], dtype=np.int64)
    ln = np.array([n // 4 for _, n in rec], dtype=np.int64)
    dev = torch.device("cuda")
    d_words = torch.as_tensor(words.view(np.int32)).to(dev)
    d_off, d_ln = torch.as_tensor(off).to(dev), torch.as_tensor(ln).to(dev)
    out = torch.empty((N_FRAMES, N_ATOMS, 3), dtype=torch.float32, device=dev)
    st = torch.full((N_FRAMES,), -1, dtype=torch.int32, device=dev)
    call("rmsf_xtc_decode_records", d_words.data_ptr(), d_off.data_ptr(), d_ln.data_ptr(), N_FRAMES, N_ATOMS,
         out.data_ptr(), 3 * N_ATOMS, st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(out.cpu().numpy(), host)


@pytest.mark.parametrize("batch", [3, 8])
def test_pinned_slot_decoder_bit_exact(c5file, batch):
    """XtcSource(decode="gpu"): records pread into pinned slots, copied and
    decompressed in HBM, several batches in flight -- every decoded frame
    (kept in the HBM cache) equals the host codec's."""
    from rmsf_amd import RMSF
    from rmsf_amd.sources import XtcSource

    p, host = c5file
    src = XtcSource(p, None, batch_frames=batch, decode="gpu", cache=True)
    assert src.cache is not None
    RMSF(src).run()
    assert src._cached.all()
    np.testing.assert_array_equal(src.cache.cpu().numpy(), host)


def test_rmsf_average_vs_oracle(c5file):
    from oracle import rmsf_oracle as O
    from rmsf_amd import RMSF
    from rmsf_amd.sources import XtcSource

    p, host = c5file
    sel = np.sort(np.random.default_rng(3).choice(N_ATOMS, 4096, replace=False))
    got = RMSF(p, select=sel, align="average").run().results
    exp = O.rmsf_script(host, sel, None, size=1, align="average")
    assert np.abs(got.rmsf - exp["rmsf"]).max() < TOL
    assert np.abs(got.average - exp["average"]).max() < TOL
    # GPU-decoded and host-decoded (frame-parallel on host threads, then the
    # pinned stager) give the same frames, hence the same bits
    g = RMSF(XtcSource(p, sel, batch_frames=3, decode="gpu"), align="average").run().results.rmsf
    h = RMSF(XtcSource(p, sel, batch_frames=3, decode="host"), align="average").run().results.rmsf
    np.testing.assert_array_equal(g, h)
    assert np.abs(g - exp["rmsf"]).max() < TOL
