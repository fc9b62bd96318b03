"""The GPU XTC decoder (csrc/xtc_gpu.hip).

CPU tier: the decoder's own code, run on the host (rmsf_xtc_decode_records_host),
is bit-identical to the host codec (csrc/xtc.cpp, itself cross-checked against
the independent Python decoder in test_xtc.py) on every compression path:
raw (<= 9 atoms), runs + water swap, packed triples wider than 52 bits (byte
long division), per-axis bit sizes (large range) and small-integer indices
up to the end of the magicints table; corrupt records are rejected.
GPU tier: the device kernel and the pinned-slot decoder give the same bytes,
and RMSF from a GPU-decoded XTC equals RMSF from the host-decoded one."""

import numpy as np
import pytest

from test_xtc import _protein_like


def _records(path):
    """(uint32 words of the whole file, word offsets, word lengths)."""
    from rmsf_amd.xtc import XTCFile
    with XTCFile(path) as f:
        rec = [f.record(i) for i in range(f.n_frames)]
        n_atoms = f.n_atoms
    words = np.fromfile(path, dtype=np.uint32)
    off = np.array([o // 4 for o, _ in rec], dtype=np.int64)
    ln = np.array([n // 4 for _, n in rec], dtype=np.int64)
    return words, off, ln, n_atoms


def _host_decode(words, off, ln, n_atoms):
    from rmsf_amd._lib import call
    out = np.empty((len(off), n_atoms, 3), dtype=np.float32)
    st = np.empty(len(off), dtype=np.int32)
    call("rmsf_xtc_decode_records_host", words.ctypes.data, off.ctypes.data, ln.ctypes.data, len(off), n_atoms,
         out.ctypes.data, 3 * n_atoms, st.ctypes.data)
    return out, st


def _cases():
    rng = np.random.default_rng(11)
    wide = rng.uniform(0, 9000, (3, 600, 3)).astype(np.float32)  # 20-bit axes: 60-bit packed triples
    clusters = _protein_like(rng, 400, 2)
    clusters[:, 200:] += np.float32(8e5)
    clusters[:, :200] -= np.float32(8e4)
    return {
        "protein": (_protein_like(rng, 3341, 6), 1000.0),
        "coarse": (_protein_like(rng, 1000, 3), 100.0),
        "fine": (_protein_like(rng, 2000, 3), 10000.0),
        "raw9": (rng.uniform(-50, 50, (4, 9, 3)).astype(np.float32), 1000.0),
        "ten": (rng.uniform(-50, 50, (3, 10, 3)).astype(np.float32), 1000.0),
        "wide60": (wide, 1000.0),
        "large_range": (clusters, 1000.0),
        "no_close_pairs": (rng.uniform(-4e5, 4e5, (2, 300, 3)).astype(np.float32), 1000.0),
    }


@pytest.mark.parametrize("case", sorted(_cases()))
def test_device_code_on_host_matches_host_codec(tmp_path, case):
    from rmsf_amd.xtc import XTCFile, write_xtc
    x, prec = _cases()[case]
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x, precision=prec)
    words, off, ln, n_atoms = _records(p)
    got, st = _host_decode(words, off, ln, n_atoms)
    assert (st == 0).all()
    with XTCFile(p) as f:
        np.testing.assert_array_equal(got, f.read())


def test_corrupt_records_are_rejected(tmp_path):
    from rmsf_amd.xtc import write_xtc
    p = str(tmp_path / "t.xtc")
    write_xtc(p, _protein_like(np.random.default_rng(2), 500, 3))
    words, off, ln, n_atoms = _records(p)
    bad = words.copy()
    bad[off[0]] = 0                                   # frame 0: magic
    bad[off[1] + 1] = bad[off[1] + 1] ^ 0x01000000    # frame 1: atom count
    ln2 = ln.copy()
    ln2[2] = 30                                       # frame 2: truncated record
    _, st = _host_decode(bad, off, ln2, n_atoms)
    assert st[0] != 0 and st[1] != 0 and st[2] != 0
    # garbage compressed bytes never crash the decoder, and it accepts exactly
    # what the host codec (xtc.cpp, sequential) accepts, with the same atoms
    from rmsf_amd import RmsfError
    from rmsf_amd.xtc import XTCFile
    rng = np.random.default_rng(0)
    n_ok = 0
    for t in range(60):
        g = words.copy()
        lo = off[0] + 24 + (t % 5) * 40  # corrupt from a few depths into the stream
        g[lo:off[0] + ln[0]] = rng.integers(0, 2**32, off[0] + ln[0] - lo, dtype=np.uint64).astype(np.uint32)
        got, st = _host_decode(g, off[:1], ln[:1], n_atoms)
        pg = str(tmp_path / f"g{t}.xtc")
        g.tofile(pg)
        try:
            with XTCFile(pg) as f:
                ref = f.read(0, 1)
        except RmsfError:
            ref = None
        assert (st[0] == 0) == (ref is not None), t
        if ref is not None:
            n_ok += 1
            np.testing.assert_array_equal(got[0], ref[0])
    assert 0 < n_ok < 60  # both outcomes exercised


# -- GPU tier ------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(_cases()))
def test_device_kernel_matches_host(tmp_path, case):
    import torch

    from rmsf_amd._lib import call
    from rmsf_amd.xtc import write_xtc
    x, prec = _cases()[case]
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x, precision=prec)
    words, off, ln, n_atoms = _records(p)
    ref, _ = _host_decode(words, off, ln, n_atoms)
    dev = torch.device("cuda")
    d_words = torch.as_tensor(words.view(np.int32)).to(dev)
    d_off, d_ln = torch.as_tensor(off).to(dev), torch.as_tensor(ln).to(dev)
    out = torch.empty((len(off), n_atoms, 3), dtype=torch.float32, device=dev)
    st = torch.full((len(off),), -1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    call("rmsf_xtc_decode_records", d_words.data_ptr(), d_off.data_ptr(), d_ln.data_ptr(), len(off), n_atoms,
         out.data_ptr(), 3 * n_atoms, st.data_ptr(), s)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
def test_device_kernel_flags_corrupt_frames(tmp_path):
    import torch

    from rmsf_amd._lib import call
    from rmsf_amd.xtc import write_xtc
    p = str(tmp_path / "t.xtc")
    write_xtc(p, _protein_like(np.random.default_rng(2), 500, 3))
    words, off, ln, n_atoms = _records(p)
    words = words.copy()
    words[off[1]] = 7
    dev = torch.device("cuda")
    d_words = torch.as_tensor(words.view(np.int32)).to(dev)
    out = torch.zeros((3, n_atoms, 3), dtype=torch.float32, device=dev)
    st = torch.full((3,), -1, dtype=torch.int32, device=dev)
    d_off, d_ln = torch.as_tensor(off).to(dev), torch.as_tensor(ln).to(dev)  # keep alive across the launch
    call("rmsf_xtc_decode_records", d_words.data_ptr(), d_off.data_ptr(), d_ln.data_ptr(), 3, n_atoms,
         out.data_ptr(), 3 * n_atoms, st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert st.cpu().tolist()[0] == 0 and st.cpu().tolist()[1] != 0 and st.cpu().tolist()[2] == 0
    assert torch.isnan(out[1]).all() and not torch.isnan(out[0]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("align", [None, "frame0", "average"])
@pytest.mark.parametrize("batch,step", [(4, 1), (7, 2), (64, 1)])
def test_rmsf_from_gpu_decoded_xtc(tmp_path, align, batch, step):
    from rmsf_amd import RMSF
    from rmsf_amd.sources import XtcSource
    from rmsf_amd.xtc import write_xtc
    x = _protein_like(np.random.default_rng(4), 3341, 23)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    sel = np.sort(np.random.default_rng(1).choice(3341, 214, replace=False))
    host = RMSF(XtcSource(p, sel, batch_frames=batch, decode="host"), align=align).run(step=step).results.rmsf
    gpu = RMSF(XtcSource(p, sel, batch_frames=batch, decode="gpu"), align=align).run(step=step).results.rmsf
    np.testing.assert_array_equal(gpu, host)


@pytest.mark.gpu
def test_xtc_decoder_reports_corrupt_frame(tmp_path):
    from rmsf_amd import RMSF, RmsfError
    from rmsf_amd.sources import XtcSource
    from rmsf_amd.xtc import write_xtc
    x = _protein_like(np.random.default_rng(4), 500, 6)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    words, off, ln, _ = _records(p)
    words = words.copy()
    words[off[3] + 14 + 7] = np.array([200], ">u4").view(np.uint32)[0]  # frame 3: smallidx out of the table
    words.tofile(p)
    with pytest.raises(RmsfError, match="frame 3"):
        RMSF(XtcSource(p, None, batch_frames=2, decode="gpu")).run()


@pytest.mark.gpu
@pytest.mark.parametrize("step", [1, 3])
def test_hbm_cache_two_sweeps(tmp_path, step):
    """RMSF.py's two sweeps over a GPU-decoded XTC with the decoded frames kept
    in HBM: bit-identical to decoding twice, and to host decoding."""
    from rmsf_amd import RMSF
    from rmsf_amd.sources import XtcSource
    from rmsf_amd.xtc import write_xtc
    x = _protein_like(np.random.default_rng(8), 3341, 31)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    sel = np.sort(np.random.default_rng(2).choice(3341, 214, replace=False))
    cached = XtcSource(p, sel, batch_frames=5, cache=True)
    assert cached.cache is not None
    a = RMSF(cached, align="average").run(step=step).results
    assert cached._cached[::step].all()
    b = RMSF(cached, align="average").run(step=step).results  # all frames served from HBM
    c = RMSF(XtcSource(p, sel, batch_frames=5), align="average").run(step=step).results
    d = RMSF(XtcSource(p, sel, batch_frames=5, decode="host"), align="average").run(step=step).results
    for r in (b, c, d):
        np.testing.assert_array_equal(a.rmsf, r.rmsf)
        np.testing.assert_array_equal(a.average, r.average)
    # the path form caches in average mode (default batch size: another
    # Chan merge order, so equal to rounding only)
    e = RMSF(p, select=sel, align="average").run(step=step).results
    np.testing.assert_allclose(a.rmsf, e.rmsf, rtol=0, atol=1e-12)


@pytest.mark.gpu
def test_hbm_cache_forgets_corrupt_frames(tmp_path):
    from rmsf_amd import RMSF, RmsfError
    from rmsf_amd.sources import XtcSource
    from rmsf_amd.xtc import write_xtc
    x = _protein_like(np.random.default_rng(4), 500, 6)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    words, off, ln, _ = _records(p)
    words = words.copy()
    words[off[3] + 14 + 7] = np.array([200], ">u4").view(np.uint32)[0]
    words.tofile(p)
    src = XtcSource(p, None, batch_frames=2, cache=True)
    with pytest.raises(RmsfError, match="frame 3"):
        RMSF(src, align="average").run()
    assert not src._cached.any()


@pytest.mark.gpu
def test_decode_list_bit_exact(tmp_path):
    """rmsf_xtcdec_decode_list: scattered records (any order, repeats) in one
    batch, frame k of the list at k -- bit-exact against the host codec."""
    import torch

    from rmsf_amd._lib import call
    from rmsf_amd.sources import XtcDecoder
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = _protein_like(np.random.default_rng(9), 2000, 12)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    lst = np.array([7, 1, 1, 11, 0, 4], dtype=np.int64)
    with XTCFile(p) as f:
        ref = f.read()[lst]
        dec = XtcDecoder(f, batch_frames=8, n_slots=2, n_threads=4)
        s = torch.cuda.current_stream().cuda_stream
        slot, ptr = dec.decode_list(lst, s)
        out = np.empty((len(lst), 2000, 3), dtype=np.float32)
        call("rmsf_memcpy_d2h", out.ctypes.data, ptr, out.nbytes, s)
        call("rmsf_stream_synchronize", s)
        dec.release(slot, s)
        dec.synchronize()
        dec.close()
    np.testing.assert_array_equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cache", [False, True])
@pytest.mark.parametrize("align", [None, "average"])
def test_scattered_frames_batched_decode(tmp_path, cache, align):
    """run(frames=scattered list) over a GPU-decoded XTC reads the records as
    full batches (decode_list), with and without the HBM cache; equal to the
    host-decoded run to rounding and to the oracle within 1e-6 A."""
    from oracle import rmsf_oracle as O
    from rmsf_amd import RMSF
    from rmsf_amd.sources import XtcSource
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = _protein_like(np.random.default_rng(6), 1500, 40)
    p = str(tmp_path / "t.xtc")
    write_xtc(p, x)
    sel = np.arange(0, 1500, 3)
    idx = np.array([0, 2, 3, 9, 10, 17, 18, 25, 31, 33, 38])
    src = XtcSource(p, sel, batch_frames=4, cache=cache)
    got = RMSF(src, align=align).run(frames=idx).results.rmsf
    if cache:  # (the reference read also pre-decodes the batches after frame 0)
        assert src._cached[idx].all()
    host = RMSF(XtcSource(p, sel, batch_frames=4, decode="host"), align=align).run(frames=idx).results.rmsf
    # the same frames (decode_list is bit-exact, test above); the batches
    # differ (4-frame lists vs runs), so the Chan folds round differently
    np.testing.assert_allclose(got, host, rtol=0, atol=1e-12)
    with XTCFile(p) as f:
        dec = f.read()
    exp = O.rmsf_script(dec[idx], sel, None, size=1, align=align)["rmsf"]  # idx[0] = 0: frame 0 is the reference
    np.testing.assert_allclose(got, exp, rtol=0, atol=1e-6)
