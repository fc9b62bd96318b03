"""Pure-Python XTC decoder -- TEST INFRASTRUCTURE ONLY.

An independent restatement (Python integers, no shared code) of the published
xdrfile xdr3dfcoord decompression, used to cross-check the native reader in
csrc/xtc.cpp.  MDAnalysis' XTCReader (libxdrfile, not vendored in
/root/reference and not installed here) is the upstream this mirrors; no
real XTC file exists in this environment, so the format itself is UNPINNED.
"""
from __future__ import annotations

import struct

import numpy as np

MAGICINTS = [0, 0, 0, 0, 0, 0, 0, 0, 0, 8, 10, 12, 16, 20, 25, 32, 40, 50, 64, 80, 101, 128, 161, 203, 256, 322,
             406, 512, 645, 812, 1024, 1290, 1625, 2048, 2580, 3250, 4096, 5060, 6501, 8192, 10321, 13003, 16384,
             20642, 26007, 32768, 41285, 52015, 65536, 82570, 104031, 131072, 165140, 208063, 262144, 330280,
             416127, 524287, 660561, 832255, 1048576, 1321122, 1664510, 2097152, 2642245, 3329021, 4194304,
             5284491, 6658042, 8388607, 10568983, 13316085, 16777216]
FIRSTIDX = 9


class _Bits:
    """MSB-first bit stream (the xdrfile receivebits convention)."""

    def __init__(self, data: bytes):
        self.data = data
        self.pos = 0  # bit position

    def bits(self, n: int) -> int:
        v = 0
        for _ in range(n):
            byte = self.data[self.pos >> 3]
            v = (v << 1) | ((byte >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def ints(self, nbits: int, sizes) -> list[int]:
        # whole bytes little-endian first, then the remaining high bits
        nbytes_full, rem = divmod(nbits, 8)
        if rem == 0 and nbytes_full > 0:
            nbytes_full -= 1
            rem = 8
        val = 0
        for k in range(nbytes_full):
            val |= self.bits(8) << (8 * k)
        if rem:
            val |= self.bits(rem) << (8 * nbytes_full)
        out = [0, 0, 0]
        for i in (2, 1):
            val, out[i] = divmod(val, sizes[i])
        out[0] = val
        return out


def _sizeofint(size: int) -> int:
    return max(0, int(size).bit_length()) if size > 0 else 0


def _sizeofints(sizes) -> int:
    # xdrfile sizeofints: the bit length of the product of the sizes
    prod = 1
    for s in sizes:
        prod *= s
    return prod.bit_length()


def _f32(x):
    return np.float32(x)


def read_xtc(path: str):
    """Decode every frame: returns float32 [n_frames, n_atoms, 3] in Angstrom
    (MDAnalysis rounding f32(f32(f32(i) * f32(1/prec)) * 10))."""
    data = open(path, "rb").read()
    off = 0
    frames = []
    while off + 56 <= len(data):
        magic, natoms, step, time = struct.unpack(">iiif", data[off:off + 16])
        assert magic == 1995, "bad magic"
        off += 16 + 36
        (lsize,) = struct.unpack(">i", data[off:off + 4])
        off += 4
        assert lsize == natoms
        if natoms <= 9:
            xyz = np.frombuffer(data[off:off + 12 * natoms], dtype=">f4").astype(np.float32).reshape(natoms, 3)
            off += 12 * natoms
            frames.append((xyz * np.float32(10.0)).astype(np.float32))
            continue
        (prec,) = struct.unpack(">f", data[off:off + 4])
        minint = struct.unpack(">iii", data[off + 4:off + 16])
        maxint = struct.unpack(">iii", data[off + 16:off + 28])
        (smallidx,) = struct.unpack(">i", data[off + 28:off + 32])
        (nbytes,) = struct.unpack(">i", data[off + 32:off + 36])
        off += 36
        bs = _Bits(data[off:off + nbytes])
        off += (nbytes + 3) & ~3
        sizeint = [maxint[i] - minint[i] + 1 for i in range(3)]
        large = (sizeint[0] | sizeint[1] | sizeint[2]) > 0xFFFFFF
        bitsizeint = [_sizeofint(s) for s in sizeint]
        bitsize = 0 if large else _sizeofints(sizeint)
        smaller = MAGICINTS[max(FIRSTIDX, smallidx - 1)] // 2
        smallnum = MAGICINTS[smallidx] // 2
        sizesmall = [MAGICINTS[smallidx]] * 3
        inv = np.float32(1.0 / np.float64(prec))
        out = []
        run = 0
        i = 0
        while i < natoms:
            if large:
                cur = [bs.bits(bitsizeint[k]) for k in range(3)]
            else:
                cur = bs.ints(bitsize, sizeint)
            i += 1
            cur = [cur[k] + minint[k] for k in range(3)]
            prev = list(cur)
            is_smaller = 0
            if bs.bits(1):
                run = bs.bits(5)
                is_smaller = run % 3
                run -= is_smaller
                is_smaller -= 1
            if run > 0:
                for k in range(0, run, 3):
                    t = bs.ints(smallidx, sizesmall)
                    i += 1
                    t = [t[j] + prev[j] - smallnum for j in range(3)]
                    if k == 0:
                        t, prev = prev, t  # undo the writer's water swap
                        out.append(prev)
                    else:
                        prev = list(t)
                    out.append(t)
            else:
                out.append(cur)
            smallidx += is_smaller
            if is_smaller < 0:
                smallnum = smaller
                smaller = MAGICINTS[smallidx - 1] // 2 if smallidx > FIRSTIDX else 0
            elif is_smaller > 0:
                smaller = smallnum
                smallnum = MAGICINTS[smallidx] // 2
            sizesmall = [MAGICINTS[smallidx]] * 3
        ints = np.array(out, dtype=np.int64)
        nm = ints.astype(np.float32) * inv
        frames.append((nm * np.float32(10.0)).astype(np.float32))
    return np.stack(frames) if frames else np.zeros((0, 0, 3), np.float32)


def quantize_expected(xyz_angstrom: np.ndarray, precision: float = 1000.0) -> np.ndarray:
    """What a write -> read round trip must return, bit for bit: the writer's
    nm = f32(x * 0.1f), i = trunc(f32(nm*prec) +/- 0.5f), then the reader's
    f32(f32(f32(i) * f32(1/prec)) * 10)."""
    x = np.asarray(xyz_angstrom, dtype=np.float32)
    nm = x * np.float32(0.1)
    p = np.float32(precision)
    sp = nm * p
    lf = np.where(nm >= 0, sp + np.float32(0.5), sp - np.float32(0.5)).astype(np.float32)
    i = np.trunc(lf).astype(np.int64)
    inv = np.float32(1.0 / np.float64(p))
    if x.shape[-2] <= 9:
        return (nm * np.float32(10.0)).astype(np.float32)
    return ((i.astype(np.float32) * inv) * np.float32(10.0)).astype(np.float32)
