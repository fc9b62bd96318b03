"""CPU tier: the C-ABI library loads and exports exactly what include/rmsf_hip.h
declares.  Only host-side integer entry points are called (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rmsf_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(rmsf_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_parses():
    names = declared_functions()
    assert "rmsf_accumulate" in names and "rmsf_superpose" in names and "rmsf_stager_stage" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    from rmsf_amd import _lib
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"symbols declared in rmsf_hip.h but not exported: {missing}"
    # and the ctypes signature table covers the header exactly
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_library_is_gfx950():
    path = os.path.join(ROOT, "mdanalysis-mpi_amd", "lib", "librmsf_hip.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_block_range():
    from rmsf_amd import _lib
    from rmsf_amd.engine import block_range
    from rmsf_amd.parallel import blocks
    assert _lib.load().rmsf_abi_version() == _lib.ABI_VERSION
    for n, size in [(98, 2), (3, 8), (20000, 8), (0, 3), (11, 1)]:
        py = blocks(n, size)
        for r in range(size):
            assert block_range(n, size, r) == py[r]


def test_block_range_rejects_bad_args():
    from rmsf_amd import _lib
    a, b = ctypes.c_int64(), ctypes.c_int64()
    lib = _lib.load()
    assert lib.rmsf_block_range(10, 0, 0, ctypes.byref(a), ctypes.byref(b)) == _lib.RMSF_EINVAL
    assert b"rmsf_block_range" in lib.rmsf_last_error()
    with pytest.raises(_lib.RmsfError):
        _lib.call("rmsf_block_range", 10, 2, 5, ctypes.byref(a), ctypes.byref(b))


def test_split_count_partitions_frames():
    from rmsf_amd import _lib
    lib = _lib.load()
    for n, s in [(20000, 56), (98, 7), (5, 5), (1, 1)]:
        counts = [lib.rmsf_split_count(n, s, i) for i in range(s)]
        assert sum(counts) == n and max(counts) - min(counts) <= 1
    # auto split choice keeps splits <= 4096 frames (the constant Welford table)
    for n_sel, n in [(100_000, 20_000), (1_000_000, 2_500), (214, 98), (10, 1_000_000)]:
        s = lib.rmsf_accumulate_splits(n_sel, n, 0)
        assert 1 <= s <= 65535 and -(-n // s) <= 4096


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from rmsf_amd.engine import Engine
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Engine()


def test_context_create_fails_cleanly_without_gpu():
    """rmsf_ctx_create reports (does not crash, does not fall back) when no
    device is visible; argument checks come first."""
    import torch
    from rmsf_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.rmsf_ctx_create(0, 10, 10, None, None, 1, ctypes.byref(h)) == _lib.RMSF_EINVAL
    assert b"flags" in lib.rmsf_last_error()
    assert lib.rmsf_ctx_create(0, 10, 11, None, None, 0, ctypes.byref(h)) == _lib.RMSF_EINVAL
    assert lib.rmsf_ctx_destroy(None) == _lib.RMSF_OK
    assert lib.rmsf_get_rmsf(None, None) == _lib.RMSF_EINVAL
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    rc = lib.rmsf_ctx_create(0, 10, 10, None, None, 0, ctypes.byref(h))
    assert rc < 0 and not h.value


def test_python_constants_match_header():
    """Every #define the ctypes layer mirrors has the header's value."""
    from rmsf_amd import _lib
    src = open(HEADER).read()
    defines = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(RMSF_[A-Z0-9_]+)\s+\(?(-?\d+)\)?", src)}
    mirrored = [n for n in defines if hasattr(_lib, n)]
    assert {"RMSF_XFORM_DOUBLES", "RMSF_REFINFO_DOUBLES", "RMSF_MAX_SPLIT_FRAMES", "RMSF_OK", "RMSF_EINVAL",
            "RMSF_MODE_SUM"} <= set(mirrored)
    for n in mirrored:
        assert getattr(_lib, n) == defines[n], n


def test_multi_device_list_and_input_errors():
    """rmsf_amd.multi host logic (no device touched): ``gpus=`` parsing and
    the inputs a one-process multi-device run refuses before any context."""
    import numpy as np
    import torch
    from rmsf_amd import multi
    assert multi.device_list(3) == [0, 1, 2]
    assert multi.device_list([2, 0, 0]) == [2, 0, 0]
    for bad in (0, [], [-1]):
        with pytest.raises(ValueError):
            multi.device_list(bad)
    with pytest.raises(TypeError):
        multi._frames_of(torch.zeros(2, 3, 3), None, None)
    with pytest.raises(ValueError):
        multi._frames_of("traj.nc", None, None)
    with pytest.raises(ValueError):
        multi._frames_of(np.zeros((2, 3, 3), np.float64), None, None)
    with pytest.raises(IndexError):
        multi._frames_of(np.zeros((2, 3, 3), np.float32), [0, 3], None)
