"""H.261 bitstream layer over include/p64stream.h (host C in libp64gpu.so).

Writer turns the GPU's per-macroblock records into the reference's .p64 bytes
(WritePictureHeader/WriteGOBHeader/WriteMBHeader marker.c:103-357, EncodeDC/
EncodeAC/CBPEncodeAC codec.c:96-352, the trailing header p64.c:608-610);
Reader parses a .p64 back into records for p64gpu_decode_recon
(p64DecodeSequence p64.c:1022, ReadMBHeader marker.c:372, DecodeAC codec.c:215).
Macroblock arrays are in raster order, as the GPU path produces them.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import MB_DTYPE, P64GpuError, _check, lib

QCIF, CIF, NTSC = 0, 1, 2


def geometry(fmt: int) -> tuple[int, int, int]:
    """(width, height, number of GOBs) of a format."""
    w, h, g = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().p64s_geometry(fmt, ctypes.byref(w), ctypes.byref(h), ctypes.byref(g)))
    return w.value, h.value, g.value


def format_of(width: int, height: int) -> int:
    f = lib().p64s_format_of(width, height)
    if f < 0:
        _check(f)
    return f


class _Info(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("format", "width", "height", "ngob", "tr", "ptype", "pspare", "coded_mbs")]


@dataclass
class Picture:
    """One decoded picture's records (raster order)."""
    tr: int
    mb: np.ndarray        # [nmb] MB_DTYPE
    quant_mb: np.ndarray  # [nmb] uint8 UseQuant
    coded: np.ndarray     # [nmb] uint8, 1 = present in the stream
    coef: np.ndarray      # [nmb, 6, 64] int16 zigzag levels


class Writer:
    """Incremental .p64 writer: write_picture() per picture, then end()."""

    def __init__(self, fmt: int):
        self.fmt = fmt
        self.width, self.height, self.ngob = geometry(fmt)
        self.nmb = self.ngob * 33
        self._h = ctypes.c_void_p()
        _check(lib().p64s_writer_open(ctypes.byref(self._h)))

    def write_picture(self, tr: int, mb, coef, gquant, quant_mb=None) -> None:
        mb = np.ascontiguousarray(mb)
        if mb.dtype != MB_DTYPE:
            mb = np.ascontiguousarray(np.asarray(mb, np.int8).reshape(-1, 4)).view(MB_DTYPE).reshape(-1)
        coef = np.ascontiguousarray(coef, dtype=np.int16)
        if mb.size != self.nmb or coef.size != self.nmb * 384:
            raise P64GpuError("records do not match the picture format")
        gq = np.ascontiguousarray(np.broadcast_to(np.asarray(gquant, np.uint8), (self.ngob,)))
        qm = None if quant_mb is None else np.ascontiguousarray(quant_mb, dtype=np.uint8)
        if qm is not None and qm.size != self.nmb:
            raise P64GpuError("quant_mb must hold one value per macroblock")
        _check(lib().p64s_write_picture(self._h, self.fmt, tr, gq.ctypes.data,
                                        qm.ctypes.data if qm is not None else None,
                                        mb.ctypes.data, coef.ctypes.data))

    def bits(self) -> int:
        n, b = ctypes.c_size_t(), ctypes.c_int64()
        lib().p64s_writer_data(self._h, ctypes.byref(n), ctypes.byref(b))
        return b.value

    def end(self, tr: int) -> bytes:
        _check(lib().p64s_write_end(self._h, self.fmt, tr))
        return self.data()

    def data(self) -> bytes:
        n = ctypes.c_size_t()
        p = lib().p64s_writer_data(self._h, ctypes.byref(n), None)
        return ctypes.string_at(p, n.value) if n.value else b""

    def close(self):
        if self._h:
            lib().p64s_writer_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Reader:
    """Iterates the pictures of a .p64 byte string; `end_tr` is set once the
    stream is exhausted (temporal reference of the trailing picture header)."""

    def __init__(self, data: bytes):
        self._buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._h = ctypes.c_void_p()
        _check(lib().p64s_reader_open(self._buf, len(data), ctypes.byref(self._h)))
        info = _Info()
        _check(lib().p64s_reader_info(self._h, ctypes.byref(info)))
        self.fmt, self.width, self.height, self.ngob = info.format, info.width, info.height, info.ngob
        self.nmb = self.ngob * 33
        self.end_tr = None

    def read(self) -> Picture | None:
        info = _Info()
        mb = np.empty(self.nmb, MB_DTYPE)
        qm = np.empty(self.nmb, np.uint8)
        coded = np.empty(self.nmb, np.uint8)
        coef = np.empty((self.nmb, 6, 64), np.int16)
        s = lib().p64s_read_picture(self._h, ctypes.byref(info), mb.ctypes.data, qm.ctypes.data,
                                    coded.ctypes.data, coef.ctypes.data)
        if s < 0:
            _check(s)
        if s == 0:
            self.end_tr = info.tr
            return None
        return Picture(info.tr, mb, qm, coded, coef)

    def __iter__(self):
        while True:
            p = self.read()
            if p is None:
                return
            yield p

    def close(self):
        if self._h:
            lib().p64s_reader_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def output_schedule(trs: list[int], end_tr: int, start_frame: int = 0) -> list[int]:
    """How many times the decoder writes out each decoded picture
    (p64DecodeSequence p64.c:1047-1056): picture i is repeated until the frame
    counter, offset by the first picture's TR, reaches the next TR (mod 32)."""
    if not trs:
        return []
    cur = start_frame
    offset = _cmod(trs[0] - cur, 32)
    nxt = trs[1:] + [end_tr]
    counts = []
    for t in nxt:
        n = 0
        while _cmod(cur + offset, 32) != t:
            n += 1
            cur += 1
            if n > 32:
                raise P64GpuError("temporal references never meet")
        counts.append(n)
    return counts


def _cmod(a: int, m: int) -> int:
    """C's % (truncating division) for the reference's TR arithmetic."""
    r = abs(a) % m
    return -r if a < 0 else r


# ---------------------------------------------------------------------------
# whole-sequence helpers: GPU hot path + host bitstream (the CLI's two modes)

def encode_sequence(frames, width: int, height: int, *, quant: int = 8, me_mode: int = 0,
                    search_limit: int = 15, first: int = 0, skip: int = 1,
                    device: int = 0) -> bytes:
    """p64EncodeSequence (p64.c:524): frames[i] is coded as frame first+i*skip
    (TR mod 32), the first intra, then closed-loop inter on the GPU."""
    from . import Encoder
    fmt = format_of(width, height)
    enc = Encoder(width, height, me_mode=me_mode, search_limit=search_limit, device=device)
    w = Writer(fmt)
    cur = first
    try:
        for i, f in enumerate(frames):
            coef, mb, _, _ = enc.frame(f, intra=(i == 0), quant=quant)
            w.write_picture(cur % 32, mb, coef, quant)
            cur += skip
        return w.end(cur % 32)  # trailer, p64.c:606-610
    finally:
        enc.close()
        w.close()


def decode_sequence(data: bytes, start_frame: int = 0) -> list[np.ndarray]:
    """p64DecodeSequence (p64.c:1022): host parse + GPU reconstruction; returns
    the output frames (Y|U|V bytes) in the order the reference writes them."""
    import torch

    from . import decode_recon
    r = Reader(data)
    w, h, nmb = r.width, r.height, r.nmb
    pic = w * h * 3 // 2
    bufs = [torch.zeros(pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    pics, trs = [], []
    prev = 0
    for p in r:
        ref, rec = bufs[prev], bufs[prev ^ 1]
        rec.copy_(ref)  # MBs absent from the stream keep the previous picture
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        decode_recon(ref, rec, dev(p.coef), dev(p.mb.view(np.int8)), dev(p.quant_mb),
                     dev(p.coded), width=w, height=h)
        pics.append(rec.cpu().numpy())
        trs.append(p.tr)
        prev ^= 1
    counts = output_schedule(trs, r.end_tr, start_frame)
    return [pic for pic, n in zip(pics, counts) for _ in range(n)]
