"""Film output writers: PNG / PFM from host buffers, decoded independently
with the Python standard library (zlib, struct) and numpy."""
import struct
import zlib

import numpy as np
import pytest


def read_png(path):
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(b):
        n, = struct.unpack(">I", b[pos:pos + 4])
        typ, data = b[pos + 4:pos + 8], b[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", b[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + data) & 0xFFFFFFFF
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", data)
        elif typ == b"IDAT":
            idat += data
        pos += 12 + n
    w, h, depth, ctype = ihdr[:4]
    assert (depth, ctype) == (8, 2)
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert np.all(raw[:, 0] == 0)
    return raw[:, 1:].reshape(h, w, 3)


def read_pfm(path):
    b = open(path, "rb").read()
    head = b.split(b"\n", 3)
    assert head[0] == b"PF"
    w, h = map(int, head[1].split())
    assert float(head[2]) < 0  # little endian
    a = np.frombuffer(head[3], "<f4").reshape(h, w, 3)
    return a[::-1]  # PFM stores bottom row first


@pytest.mark.parametrize("w,h", [(1, 1), (37, 5), (300, 250)])
def test_png_roundtrip(mcpt_mod, tmp_path, w, h):
    rng = np.random.default_rng(w * h)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    p = tmp_path / "a.png"
    mcpt_mod.write_png(p, img)
    assert np.array_equal(read_png(p), img[..., :3])


def test_pfm_roundtrip(mcpt_mod, tmp_path):
    rng = np.random.default_rng(3)
    img = rng.normal(size=(7, 11, 3)).astype(np.float32)
    img[0, 0] = [np.inf, -0.0, 1e-40]
    p = tmp_path / "a.pfm"
    mcpt_mod.write_pfm(p, img)
    assert np.array_equal(read_pfm(p).view(np.uint32), img.view(np.uint32))
