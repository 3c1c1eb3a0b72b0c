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

    def write_bits(self, data, bits: int, phase: int) -> None:
        """Appends a picture coded on the GPU (vlc_pictures) at bit `phase` of
        data[0]: phase must be this writer's phase(), bits counts the phase
        bits too (p64s_write_bits)."""
        buf = np.frombuffer(bytes(data[:(bits + 7) // 8]), np.uint8)
        _check(lib().p64s_write_bits(self._h, buf.ctypes.data if buf.size else None, int(bits), int(phase)))

    def phase(self) -> int:
        """The stream's position within its current byte (0..7)."""
        return int(lib().p64s_writer_phase(self._h))

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

    def __init__(self, data: bytes, force_cif: bool = False):
        self._buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._h = ctypes.c_void_p()
        _check(lib().p64s_reader_open(self._buf, len(data), ctypes.byref(self._h)))
        if force_cif:  # -c ForceCIF (p64.c:308-310, 1071-1072)
            _check(lib().p64s_reader_force_cif(self._h))
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

class SeqConfig(ctypes.Structure):
    """p64seq_config (include/p64seq.h)."""
    _fields_ = [(n, ctypes.c_int) for n in
                ("format", "me_mode", "search_limit", "quant", "rate", "file_size_bits",
                 "start_frame", "last_frame", "frame_skip", "frame_rate", "frame_rate_div",
                 "device")] + [("program", ctypes.c_void_p), ("host_vlc", ctypes.c_int),
                               ("verbose", ctypes.c_int)]


class ProgSettings(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("quantization", "search_limit", "frame_rate", "frame_skip", "image_type",
                 "abort_code")]


class Program:
    """The -o program interpreter (include/p64prog.h, lexer.l): loading runs the
    top-level statements; programs 0 (MTYPE) and 1 (quantiser) are then called
    by the sequence encoder."""

    def __init__(self, text: str | bytes):
        data = text.encode() if isinstance(text, str) else bytes(text)
        self._h = ctypes.c_void_p()
        _check(lib().p64prog_load(data, len(data), None, ctypes.byref(self._h)))
        st = ProgSettings()
        _check(lib().p64prog_settings_get(self._h, ctypes.byref(st)))
        self.settings = st

    def memory(self):
        return np.ctypeslib.as_array(lib().p64prog_memory(self._h), shape=(1024,))

    def execute(self, n: int) -> None:
        _check(lib().p64prog_execute(self._h, n))

    def reads(self, n: int, loc: int) -> bool:
        return bool(lib().p64prog_reads(self._h, n, loc))

    def defined(self, n: int) -> bool:
        return bool(lib().p64prog_defined(self._h, n))

    def close(self):
        if self._h:
            lib().p64prog_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SeqStats(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_int), ("next_frame", ctypes.c_int), ("gquant", ctypes.c_int),
                ("rate", ctypes.c_int), ("bits", ctypes.c_int64), ("last_bits", ctypes.c_int64),
                ("first_frame_bits", ctypes.c_int64), ("overflows", ctypes.c_int),
                ("mtype_hist", ctypes.c_int * 10)]


class SequenceEncoder:
    """p64EncodeSequence (p64.c:524) over include/p64seq.h: GPU per-macroblock
    compute, host VLC and the reference's rate control (-r / -x)."""

    def __init__(self, width: int, height: int, *, quant: int = 0, me_mode: int = 0,
                 search_limit: int = 15, first: int = 0, last: int | None = None, skip: int = 1,
                 rate: int = 0, file_size_bits: int = 0, frame_rate: int = 30000,
                 frame_rate_div: int = 1001, device: int = 0, nframes: int | None = None,
                 program: "Program | str | bytes | None" = None, host_vlc: bool = False,
                 verbose: bool = False):
        L = lib()
        if program is not None and not isinstance(program, Program):
            program = Program(program)
        self.program = program  # kept alive for the encoder's lifetime
        if program is not None:  # top-level settings override the arguments (p64.c:409-413)
            ps = program.settings
            if ps.quantization >= 0:
                quant = ps.quantization
            if ps.search_limit >= 0:
                search_limit = ps.search_limit
            if ps.frame_rate >= 0:
                frame_rate, frame_rate_div = ps.frame_rate, 1
            if ps.frame_skip >= 0:
                skip = ps.frame_skip
        c = SeqConfig()
        L.p64seq_default_config(ctypes.byref(c))
        c.format = format_of(width, height)
        c.me_mode, c.search_limit, c.quant = me_mode, search_limit, quant
        c.rate, c.file_size_bits = rate, file_size_bits
        c.start_frame = first
        c.last_frame = last if last is not None else first + skip * ((nframes or 1) - 1)
        c.frame_skip, c.frame_rate, c.frame_rate_div, c.device = skip, frame_rate, frame_rate_div, device
        c.program = program._h if program is not None else None
        c.host_vlc = int(bool(host_vlc))
        c.verbose = int(bool(verbose))
        self.width, self.height = width, height
        self._h = ctypes.c_void_p()
        _check(L.p64seq_open(ctypes.byref(c), ctypes.byref(self._h)))
        self._chunks = []

    def more(self) -> bool:
        return bool(lib().p64seq_more(self._h))

    def encode(self, picture) -> None:
        pic = np.ascontiguousarray(picture, dtype=np.uint8)
        if pic.size != self.width * self.height * 3 // 2:
            raise P64GpuError("picture has the wrong size")
        _check(lib().p64seq_encode(self._h, pic.ctypes.data))
        self._drain()

    def finish(self) -> bytes:
        _check(lib().p64seq_finish(self._h))
        self._drain()
        return b"".join(self._chunks)

    def stats(self) -> SeqStats:
        st = SeqStats()
        _check(lib().p64seq_get_stats(self._h, ctypes.byref(st)))
        return st

    def _drain(self):
        L = lib()
        w = L.p64seq_writer(self._h)
        n = ctypes.c_size_t()
        p = L.p64s_writer_data(w, ctypes.byref(n), None)
        if n.value:
            self._chunks.append(ctypes.string_at(p, n.value))
            _check(L.p64s_writer_consume(w, n.value))

    def close(self):
        if self._h:
            lib().p64seq_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode_sequence(frames, width: int, height: int, *, quant: int = 0, me_mode: int = 0,
                    search_limit: int = 15, first: int = 0, skip: int = 1, rate: int = 0,
                    file_size_bits: int = 0, device: int = 0, program=None,
                    host_vlc: bool = False) -> bytes:
    """Encode frames[i] as frame first+i*skip: the reference CLI's `-a first
    -b last -k skip [-q] [-r|-x]` over the same pictures."""
    frames = list(frames)
    enc = SequenceEncoder(width, height, quant=quant, me_mode=me_mode, search_limit=search_limit,
                          first=first, skip=skip, rate=rate, file_size_bits=file_size_bits,
                          device=device, nframes=len(frames), program=program,
                          host_vlc=host_vlc)
    try:
        for f in frames:
            if not enc.more():
                break
            enc.encode(f)
        return enc.finish()
    finally:
        enc.close()


def pack_levels(fmt: int, mb, coded, coef):
    """p64s_pack_levels: the packed level layout of decode_recon_packed from
    the reader's dense output of one or more pictures (mb [n, nmb] records,
    coded [n, nmb], coef [n, nmb, 6, 64]).  Returns (levels [k, 64] int16,
    index [groups, 4] uint32)."""
    _, _, ngob = geometry(fmt)
    nmb = ngob * 33
    mbv = np.ascontiguousarray(mb)
    if mbv.dtype != MB_DTYPE:
        mbv = np.ascontiguousarray(np.asarray(mb, np.int8).reshape(-1, 4)).view(MB_DTYPE).reshape(-1)
    cd = np.ascontiguousarray(coded, dtype=np.uint8).reshape(-1)
    cf = np.ascontiguousarray(coef, dtype=np.int16).reshape(-1)
    n = cd.size // nmb
    if mbv.size != n * nmb or cf.size != n * nmb * 384:
        raise P64GpuError("pack_levels: arrays do not match the picture format")
    levels = np.empty((n * nmb * 6, 64), np.int16)
    index = np.empty(((n * 6 * nmb + 63) // 64, 4), np.uint32)  # groups of 64 blocks of the batch
    k = int(lib().p64s_pack_levels(fmt, n, mbv.ctypes.data, cd.ctypes.data, cf.ctypes.data,
                                   levels.ctypes.data, index.ctypes.data))
    _check(k if k < 0 else 0)
    return levels[:k], index


def decode_sequence(data: bytes, start_frame: int = 0, force_cif: bool = False,
                    packed: bool = True) -> list[np.ndarray]:
    """p64DecodeSequence (p64.c:1022): host parse + GPU reconstruction; returns
    the output frames (Y|U|V bytes) in the order the reference writes them.
    force_cif: the -c flag (CIF geometry whatever the stream's PTYPE says).
    packed: the reader's levels packed (pack_levels) for decode_recon_packed
    (ABI v3, the default); else the dense layout through decode_recon."""
    import torch

    from . import decode_recon, decode_recon_packed
    r = Reader(data, force_cif=force_cif)
    w, h, nmb = r.width, r.height, r.nmb
    pic = w * h * 3 // 2
    bufs = [torch.zeros(pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    pics, trs = [], []
    prev = 0
    for p in r:
        ref, rec = bufs[prev], bufs[prev ^ 1]
        rec.copy_(ref)  # MBs absent from the stream keep the previous picture
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        if packed:
            lv, ix = pack_levels(r.fmt, p.mb, p.coded, p.coef)
            lvd = dev(lv) if len(lv) else torch.zeros((1, 64), dtype=torch.int16, device="cuda")
            decode_recon_packed(ref, rec, lvd, len(lv), dev(ix.view(np.int32)), dev(p.mb.view(np.int8)),
                                dev(p.quant_mb), dev(p.coded), width=w, height=h)
        else:
            decode_recon(ref, rec, dev(p.coef), dev(p.mb.view(np.int8)), dev(p.quant_mb),
                         dev(p.coded), width=w, height=h)
        pics.append(rec.cpu().numpy())
        trs.append(p.tr)
        prev ^= 1
    counts = output_schedule(trs, r.end_tr, start_frame)
    return [pic for pic, n in zip(pics, counts) for _ in range(n)]


# ---------------------------------------------------------------------------
# entropy coding on the device (p64gpu_vlc_pictures, p64vlc.hip)

class VlcArgs(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("nframes", ctypes.c_int),
                ("flags", ctypes.c_int), ("mb", ctypes.c_void_p), ("coef", ctypes.c_void_p),
                ("gquant", ctypes.c_void_p), ("mquant", ctypes.c_void_p), ("tr", ctypes.c_void_p),
                ("phase", ctypes.c_void_p), ("out", ctypes.c_void_p), ("out_stride", ctypes.c_int64),
                ("bits", ctypes.c_void_p), ("scratch", ctypes.c_void_p), ("blk_bits", ctypes.c_void_p),
                ("seq_bits", ctypes.c_void_p), ("max_bits", ctypes.c_void_p)]


def vlc_buffers(n: int, width: int, height: int):
    """Device buffers for vlc_pictures over n pictures: (out, bits, scratch)."""
    import torch

    _, _, ngob = geometry(format_of(width, height))
    nmb = ngob * 33
    stride = (int(lib().p64gpu_vlc_max_bytes(width, height)) + 3) // 4 * 4
    return (torch.empty((n, stride), dtype=torch.uint8, device="cuda"),
            torch.empty(n, dtype=torch.int32, device="cuda"),
            torch.empty(6 * n * nmb, dtype=torch.int32, device="cuda"))


def vlc_pictures(mb, coef, gquant, tr, *, width: int, height: int, phase=None, mquant=None,
                 buffers=None, host_bits: bool = True, blk_bits=None, seq_bits=None, max_bits=None):
    """H.261 bits of a batch of pictures on the GPU.  All inputs are CUDA(HIP)
    tensors: mb [n, nmb, 4] int8, coef [n, nmb, 6, 64] int16, gquant [n, ngob]
    uint8, tr [n] int32, phase [n] uint8 or None, mquant [n, nmb] uint8 or None.
    buffers: (out, bits, scratch) from vlc_buffers, reused across calls.
    blk_bits: int16 [n, nmb, 8] from the encoder (FrameBatchOut.vlc_bits of the
    same records and levels): the coder skips its count pass.
    seq_bits: int64 [n], the sequences' running bit counts: each picture
    starts at phase seq_bits & 7 (phase is not read) and seq_bits advances by
    its bits, on the device.  max_bits: int32 [1], set to the longest
    picture's bit count.
    Returns (out [n, stride] uint8 tensor, bits [n] list of ints) -- or, with
    host_bits=False, the device bits tensor (no synchronisation)."""
    import torch

    from . import _stream, _torch
    _torch()
    L = lib()
    n = int(tr.numel())
    _, _, ngob = geometry(format_of(width, height))
    nmb = ngob * 33
    if blk_bits is not None and (blk_bits.numel() < n * nmb * 8 or blk_bits.dtype != torch.int16):
        raise P64GpuError("vlc_pictures: blk_bits must be int16 [n, nmb, 8]")
    if mb.numel() != n * nmb * 4 or coef.numel() != n * nmb * 384 or gquant.numel() != n * ngob:
        raise P64GpuError("vlc_pictures: buffer sizes do not match the picture format")
    out, bits, scratch = buffers if buffers is not None else vlc_buffers(n, width, height)
    stride = int(out.shape[1])
    if out.shape[0] < n or bits.numel() < n or scratch.numel() < 6 * n * nmb or \
            stride < int(L.p64gpu_vlc_max_bytes(width, height)):
        raise P64GpuError("vlc_pictures: buffers smaller than the batch")
    a = VlcArgs(width=width, height=height, nframes=n, flags=0, mb=mb.data_ptr(),
                coef=coef.data_ptr(), gquant=gquant.data_ptr(),
                mquant=mquant.data_ptr() if mquant is not None else None, tr=tr.data_ptr(),
                phase=phase.data_ptr() if phase is not None else None, out=out.data_ptr(),
                out_stride=stride, bits=bits.data_ptr(), scratch=scratch.data_ptr(),
                blk_bits=blk_bits.data_ptr() if blk_bits is not None else None,
                seq_bits=seq_bits.data_ptr() if seq_bits is not None else None,
                max_bits=max_bits.data_ptr() if max_bits is not None else None)
    _check(L.p64gpu_vlc_pictures(ctypes.byref(a), _stream(torch)))
    if not host_bits:
        return out, bits[:n]
    b = [int(x) & 0xFFFFFFFF for x in bits[:n].cpu().tolist()]
    if any(x == 0xFFFFFFFF for x in b):
        raise P64GpuError("vlc_pictures: invalid macroblock record or buffer overflow")
    return out, b


def prepare_vlc(mb, coef, gquant, tr, *, width: int, height: int, buffers, blk_bits=None, seq_bits=None,
                max_bits=None, mquant=None, phase=None, stream=None):
    """vlc_pictures' launch checked and packed once (host_bits=False): the
    returned function issues it again with the same buffers, without the
    per-call Python checks (bench.py's fed path).  The tensors must outlive
    it.  Returns (launch, bits tensor)."""
    import torch

    from . import _stream, _torch
    _torch()
    n = int(tr.numel())
    _, _, ngob = geometry(format_of(width, height))
    nmb = ngob * 33
    out, bits, scratch = buffers
    if mb.numel() != n * nmb * 4 or coef.numel() != n * nmb * 384 or gquant.numel() != n * ngob or \
            out.shape[0] < n or bits.numel() < n or scratch.numel() < 6 * n * nmb:
        raise P64GpuError("prepare_vlc: buffer sizes do not match the picture format")
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    a = VlcArgs(width=width, height=height, nframes=n, flags=0, mb=mb.data_ptr(), coef=coef.data_ptr(),
                gquant=gquant.data_ptr(), mquant=p(mquant), tr=tr.data_ptr(), phase=p(phase), out=out.data_ptr(),
                out_stride=int(out.shape[1]), bits=bits.data_ptr(), scratch=scratch.data_ptr(),
                blk_bits=p(blk_bits), seq_bits=p(seq_bits), max_bits=p(max_bits))
    st = ctypes.c_void_p((stream or torch.cuda.current_stream()).cuda_stream) if stream is not None else _stream(torch)
    L, ref_a = lib(), ctypes.byref(a)

    def launch():
        _check(L.p64gpu_vlc_pictures(ref_a, st))
    launch.args = a
    return launch, bits[:n]


class BitAssembler:
    """Concatenates pictures coded at a bit phase (vlc_pictures) into one
    stream, and closes it like p64s_write_end (trailer header + ones)."""

    def __init__(self):
        self.buf = bytearray()
        self.nbits = 0

    @property
    def phase(self) -> int:
        return self.nbits % 8

    def append(self, data: bytes, bits: int) -> None:
        """data was produced at phase == self.phase; bits includes the phase."""
        p = self.phase
        nbytes = (bits + 7) // 8
        chunk = bytes(data[:nbytes])
        if p:
            self.buf[-1] |= chunk[0]
            chunk = chunk[1:]
        self.buf += chunk
        self.nbits += bits - p

    def end(self, fmt: int, tr: int) -> bytes:
        hdr = (0x10 << 12) | ((tr & 31) << 7) | ((0 if fmt == QCIF else 4) << 1)
        n = 32
        if fmt == NTSC:
            hdr = (hdr >> 1 << 10) | (0x18c << 1)
            n = 41
        v, nb = hdr, n
        pad = (-(self.nbits + nb)) % 8
        v = (v << pad) | ((1 << pad) - 1)
        nb += pad
        p = self.phase
        total = p + nb
        word = v  # place at bit phase p within (p + nb) bits
        data = word.to_bytes(total // 8, "big")
        if p:
            self.buf[-1] |= data[0]
            data = data[1:]
        self.buf += data
        self.nbits += nb
        return bytes(self.buf)
