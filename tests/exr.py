"""Minimal OpenEXR scanline reader (NONE / ZIPS / ZIP, HALF / FLOAT channels).

Test infrastructure: decodes the reference's Mitsuba goldens
(renderer/Media/reference/*.exr, ZIP-compressed half RGB) the way
loadReferenceImage does (renderer/Renderer.mm:162-253), without OpenEXR.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_COMP_LINES = {0: 1, 2: 1, 3: 16}


def _read_header(buf: bytes):
    if struct.unpack_from("<I", buf, 0)[0] != 20000630:
        raise ValueError("not an OpenEXR file")
    pos = 8
    attrs = {}
    while True:
        end = buf.index(b"\0", pos)
        name = buf[pos:end].decode()
        pos = end + 1
        if not name:
            break
        end = buf.index(b"\0", pos)
        typ = buf[pos:end].decode()
        pos = end + 1
        size = struct.unpack_from("<i", buf, pos)[0]
        pos += 4
        attrs[name] = (typ, buf[pos:pos + size])
        pos += size
    return attrs, pos


def _channels(raw: bytes):
    out, pos = [], 0
    while raw[pos] != 0:
        end = raw.index(b"\0", pos)
        name = raw[pos:end].decode()
        pos = end + 1
        ptype, _plin, _r0, _r1, _r2, xs, ys = struct.unpack_from("<iBBBBii", raw, pos)
        pos += 16
        out.append((name, ptype))
    return out


def read_exr(path: str) -> dict[str, np.ndarray]:
    """Returns {channel: float32 array [H, W]} with row 0 = TOP of the image."""
    buf = open(path, "rb").read()
    attrs, pos = _read_header(buf)
    chans = _channels(attrs["channels"][1])
    comp = attrs["compression"][1][0]
    if comp not in _COMP_LINES:
        raise ValueError(f"unsupported EXR compression {comp}")
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"][1])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    lpb = _COMP_LINES[comp]
    nblocks = (H + lpb - 1) // lpb
    offsets = struct.unpack_from(f"<{nblocks}Q", buf, pos)
    bpp = {1: 2, 2: 4, 0: 4}  # HALF, FLOAT, UINT
    out = {name: np.zeros((H, W), np.float32) for name, _ in chans}
    for off in offsets:
        y, size = struct.unpack_from("<ii", buf, off)
        data = buf[off + 8: off + 8 + size]
        nlines = min(lpb, y1 - y + 1)
        raw_size = sum(bpp[t] for _, t in chans) * W * nlines
        if comp != 0 and size < raw_size:
            t = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int32)
            t = (np.cumsum(t - 128) + 128) & 0xFF  # undo the predictor (t[0] kept)
            t[0] = np.frombuffer(zlib.decompress(data), np.uint8)[0]
            t = t.astype(np.uint8)
            half = (len(t) + 1) // 2
            d = np.empty_like(t)
            d[0::2] = t[:half]
            d[1::2] = t[half:]
            data = d.tobytes()
        p = 0
        for ly in range(nlines):
            row = y - y0 + ly
            for name, typ in chans:
                n = bpp[typ] * W
                dt = {1: "<f2", 2: "<f4", 0: "<u4"}[typ]
                out[name][row] = np.frombuffer(data, dt, count=W, offset=p).astype(np.float32)
                p += n
    return out


def read_rgb(path: str) -> np.ndarray:
    """[H, W, 3] float32, row 0 = top."""
    ch = read_exr(path)
    return np.stack([ch["R"], ch["G"], ch["B"]], axis=-1)
