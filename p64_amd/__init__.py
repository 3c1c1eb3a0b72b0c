"""p64_amd -- MI355X-native PVRG-P64 macroblock encode hot path.

Python mirror of the reference's hot-path interface over the C ABI in
include/p64gpu.h (libp64gpu.so, hand-written HIP for gfx950).  Names follow the
reference (/root/reference):

    ChenDct / ChenIDct                       chendct.c:97 / :217
    CCITTQuantize / CCITTFlatQuantize        transform.c:271 / :317
    ICCITTQuantize / ICCITTFlatQuantize      transform.c:400 / :359
    BoundDctMatrix / BoundIDctMatrix         transform.c:460 / :483
    FlatBoundQuantizeMatrix / BoundQuantizeMatrix   transform.c:502 / :526
    ZigzagMatrix / IZigzagMatrix             transform.c:561 / :546
    MotionEstimation                         me.c:340 (StepBME :255 / FastBME :187)
    encode_frames                            p64.c:622-1013 per-MB compute, batched
    Encoder                                  p64EncodeSequence/p64EncodeFrame loop
                                             (closed loop, reconstruction on device)
    stream.Writer / stream.Reader            the H.261 bitstream either side of the
                                             GPU records (marker.c, codec.c, huffman.c)

Block functions take/return int32 tensors of shape [..., 64] (row-major 8x8
blocks) on a CUDA(HIP) device; the reference works on one `int[64]` at a time,
these work on a batch.  There is no CPU fallback: if the HIP library is missing
or no device is present the calls raise.  PyTorch is used only for device
memory and the stream handle.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# P64GPU_LIB lets development A/B runs point at an alternative build.
LIB_PATH = os.environ.get("P64GPU_LIB", os.path.join(_HERE, "libp64gpu.so"))

ABI_VERSION = 3  # include/p64gpu.h P64GPU_ABI_VERSION
ME_TSS = 0
ME_FULL = 1

OP_DCT, OP_IDCT, OP_QUANT_INTRA, OP_QUANT_INTER, OP_IQUANT_INTRA, OP_IQUANT_INTER = range(6)
OP_BOUND_DCT, OP_BOUND_IDCT, OP_BOUND_QFLAT, OP_BOUND_QUANT, OP_ZIGZAG, OP_IZIGZAG = range(6, 12)

# coding-control tables, p64.c:217-222
QUANT_MTYPE = (0, 1, 0, 1, 0, 0, 1, 0, 0, 1)
CBP_MTYPE = (0, 0, 1, 1, 0, 1, 1, 0, 1, 1)
INTRA_MTYPE = (1, 1, 0, 0, 0, 0, 0, 0, 0, 0)
MF_MTYPE = (0, 0, 0, 0, 1, 1, 1, 1, 1, 1)
FILTER_MTYPE = (0, 0, 0, 0, 0, 0, 0, 1, 1, 1)
TCOEFF_MTYPE = (1, 1, 1, 1, 0, 1, 1, 0, 1, 1)


class P64GpuError(RuntimeError):
    pass


class MeRec(ctypes.Structure):
    """p64_me_rec: one MB of MeX/MeY/MeVal/MeOVal/MeVAR/MeVAROR/MeMWOR (me.c:49-60)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("mx", "my", "sad", "sad0", "var", "varor", "mwor")]


class MbRec(ctypes.Structure):
    """p64_mb_rec: MType, CBP, MVDH, MVDV as written by WriteMBHeader (marker.c:288)."""
    _fields_ = [(n, ctypes.c_int8) for n in ("mtype", "cbp", "mvx", "mvy")]


class EncodeArgs(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("nframes", ctypes.c_int32),
        ("intra", ctypes.c_int32), ("quant", ctypes.c_int32), ("me_mode", ctypes.c_int32),
        ("search_limit", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("frame_stride", ctypes.c_int64),
        ("cur", ctypes.c_void_p), ("ref", ctypes.c_void_p), ("recon", ctypes.c_void_p),
        ("last_intra", ctypes.c_void_p), ("quant_mb", ctypes.c_void_p),
        ("mtype_override", ctypes.c_void_p), ("coef", ctypes.c_void_p),
        ("mb", ctypes.c_void_p), ("me", ctypes.c_void_p), ("nzmask", ctypes.c_void_p),
        ("vlc_bits", ctypes.c_void_p),
    ]


# numpy views of the record arrays (field order matches include/p64gpu.h)
P64GPU_FLAG_ME_GIVEN = 1  # include/p64gpu.h
P64GPU_FLAG_SEARCH_ONLY = 2
ME_DTYPE = np.dtype([(n, "<i4") for n in ("mx", "my", "sad", "sad0", "var", "varor", "mwor")])
MB_DTYPE = np.dtype([(n, "i1") for n in ("mtype", "cbp", "mvx", "mvy")])

_lib = None


def lib() -> ctypes.CDLL:
    """Load libp64gpu.so (built by `make` / __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise P64GpuError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch bundles its own libamdhip64 (SONAME
    # libamdhip64.so.7).  Loading torch first lets our DT_NEEDED resolve to that
    # already-mapped copy, so device pointers and streams are shared with torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    _check_single_runtime()
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.p64gpu_abi_version.restype = i32
    L.p64gpu_strerror.restype = ctypes.c_char_p
    L.p64gpu_strerror.argtypes = [i32]
    L.p64gpu_last_error.restype = ctypes.c_char_p
    L.p64gpu_device_count.argtypes = [ctypes.POINTER(i32)]
    L.p64gpu_set_device.argtypes = [i32]
    L.p64gpu_synchronize.argtypes = [vp]
    L.p64gpu_block_op.argtypes = [i32, vp, vp, i64, i32, i32, vp]
    L.p64gpu_motion_estimation.argtypes = [i32, i32, i32, i64, vp, vp, i32, i32, vp, vp]
    L.p64gpu_encode_frames.argtypes = [ctypes.POINTER(EncodeArgs), vp]
    L.p64gpu_decode_recon.argtypes = [i32, i32, i32, i64, vp, vp, vp, vp, vp, vp, vp]
    L.p64gpu_decode_recon_packed.argtypes = [i32, i32, i32, i64, vp, vp, vp, i64, vp, vp, vp, vp, vp]
    L.p64s_pack_levels.argtypes = [i32, i32, vp, vp, vp, vp, vp]
    L.p64s_pack_levels.restype = i64
    L.p64gpu_release_scratch.argtypes = []
    L.p64gpu_encoder_open.argtypes = [i32, i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.p64gpu_encoder_frame.argtypes = [vp, vp, i32, i32, vp, vp, vp, vp, vp]
    L.p64gpu_encoder_close.argtypes = [vp]
    L.p64gpu_encoder_close.restype = None
    L.p64gpu_synth_frames.argtypes = [i32, i32, ctypes.c_uint32, i32, i32, i32, i64, vp, vp]
    L.p64gpu_synth_content.argtypes = [i32, i32, i32, ctypes.c_uint32, i32, i32, i32, i64, vp, vp]
    L.p64_synth_frame_content.argtypes = [i32, ctypes.c_uint32, i32, i32, i32, vp]
    L.p64gpu_clock_probe.argtypes = [i32, ctypes.POINTER(i32), vp]
    L.p64_synth_frame.argtypes = [ctypes.c_uint32, i32, i32, i32, vp]
    L.p64_synth_frame.restype = None
    L.p64_synth_motion.argtypes = [ctypes.c_uint32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.p64_synth_motion.restype = None
    # H.261 bitstream layer (include/p64stream.h), host C
    L.p64s_geometry.argtypes = [i32, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.p64s_format_of.argtypes = [i32, i32]
    L.p64s_writer_open.argtypes = [ctypes.POINTER(vp)]
    L.p64s_writer_close.argtypes = [vp]
    L.p64s_writer_close.restype = None
    L.p64s_write_picture.argtypes = [vp, i32, i32, vp, vp, vp, vp]
    L.p64s_write_end.argtypes = [vp, i32, i32]
    L.p64s_writer_data.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(i64)]
    L.p64s_writer_data.restype = vp
    L.p64s_writer_consume.argtypes = [vp, ctypes.c_size_t]
    L.p64s_write_bits.argtypes = [vp, vp, i64, i32]
    L.p64s_writer_phase.argtypes = [vp]
    L.p64s_reader_open.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    L.p64s_reader_close.argtypes = [vp]
    L.p64s_reader_close.restype = None
    L.p64s_reader_info.argtypes = [vp, vp]
    L.p64s_reader_force_cif.argtypes = [vp]
    L.p64s_read_picture.argtypes = [vp, vp, vp, vp, vp, vp]
    # sequence encoder (include/p64seq.h), host C over the GPU path
    L.p64seq_default_config.argtypes = [vp]
    L.p64seq_default_config.restype = None
    L.p64seq_open.argtypes = [vp, ctypes.POINTER(vp)]
    L.p64seq_close.argtypes = [vp]
    L.p64seq_close.restype = None
    L.p64seq_more.argtypes = [vp]
    L.p64seq_encode.argtypes = [vp, vp]
    L.p64seq_finish.argtypes = [vp]
    L.p64seq_writer.argtypes = [vp]
    L.p64seq_writer.restype = vp
    L.p64seq_get_stats.argtypes = [vp, vp]
    L.p64gpu_encode_mb_list.argtypes = [ctypes.POINTER(EncodeArgs), vp, i32, vp]
    L.p64gpu_vlc_max_bytes.argtypes = [i32, i32]
    L.p64gpu_vlc_max_bytes.restype = i64
    L.p64gpu_vlc_pictures.argtypes = [vp, vp]
    # -o program interpreter (include/p64prog.h), host C
    L.p64prog_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.POINTER(vp)]
    L.p64prog_free.argtypes = [vp]
    L.p64prog_free.restype = None
    L.p64prog_settings_get.argtypes = [vp, vp]
    L.p64prog_defined.argtypes = [vp, i32]
    L.p64prog_reads.argtypes = [vp, i32, i32]
    L.p64prog_execute.argtypes = [vp, i32]
    L.p64prog_memory.argtypes = [vp]
    L.p64prog_memory.restype = ctypes.POINTER(ctypes.c_double)
    if L.p64gpu_abi_version() != ABI_VERSION:
        raise P64GpuError("libp64gpu.so ABI version mismatch")
    _lib = L
    return L


def _check_single_runtime() -> None:
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                paths.add(os.path.realpath(line.split()[-1]))
    if len(paths) > 1:
        raise P64GpuError(f"two HIP runtimes mapped in this process: {sorted(paths)}; "
                          "import torch before loading libp64gpu.so")


def _check(status: int) -> None:
    if status != 0:
        L = lib()
        raise P64GpuError(f"{L.p64gpu_strerror(status).decode()}: {L.p64gpu_last_error().decode()}")


# ---------------------------------------------------------------------------
# synthetic input (host, integer-only; identical bytes for GPU and CPU legs)

def picture_bytes(width: int, height: int) -> int:
    return width * height * 3 // 2


# synthetic contents (include/p64gpu.h p64_synth_content)
SYNTH_VNOISE, SYNTH_SURVEY = 0, 1
CONTENTS = {"synth": SYNTH_VNOISE, "survey": SYNTH_SURVEY}


def synth_frame(seed: int, frame: int, width: int, height: int, content: int = SYNTH_VNOISE) -> np.ndarray:
    """Picture `frame` of synthetic stream `seed` (host, integer only).
    content SYNTH_VNOISE: the value-noise texture (seed classes mod 8);
    SYNTH_SURVEY: SURVEY.md 8(d)'s sinusoid texture + N(0,12), (+3,-2) px
    per picture, N(0,4) temporal noise."""
    out = np.empty(picture_bytes(width, height), np.uint8)
    _check(lib().p64_synth_frame_content(content, seed, frame, width, height, out.ctypes.data))
    return out


def synth_motion(seed: int) -> tuple[int, int]:
    x, y = ctypes.c_int(), ctypes.c_int()
    lib().p64_synth_motion(seed, ctypes.byref(x), ctypes.byref(y))
    return x.value, y.value


# ---------------------------------------------------------------------------
# device-tensor API (torch tensors on a HIP device)

def synth_frames_device(width: int, height: int, seed0: int, nseeds: int, frame0: int,
                        nslots: int, out=None, content: int = SYNTH_VNOISE):
    """Device copy of synth_frame for nslots x nseeds pictures, slot-major:
    out[t, s] = synth_frame(seed0 + s, frame0 + t, content=content)."""
    torch = _torch()
    pic = picture_bytes(width, height)
    if out is None:
        out = torch.empty((nslots, nseeds, pic), dtype=torch.uint8, device="cuda")
    _dev_check(out, torch.uint8, "out")
    if out.numel() < nslots * nseeds * pic:
        raise P64GpuError("out too small")
    # one launch covers at most 65535 pictures (its grid's y extent): slot chunks
    step = max(1, 65535 // nseeds)
    for t0 in range(0, nslots, step):
        n = min(step, nslots - t0)
        _check(lib().p64gpu_synth_content(content, width, height, seed0, nseeds, frame0 + t0, n, pic,
                                          out.data_ptr() + t0 * nseeds * pic, _stream(torch)))
    return out

def _torch():
    import torch
    if not torch.cuda.is_available():
        raise P64GpuError("no HIP device visible: the p64_amd hot path has no CPU fallback")
    return torch


def _stream(torch):
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev_check(t, dtype, name):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise P64GpuError(f"{name} must be a device tensor")
    if t.dtype != dtype or not t.is_contiguous():
        raise P64GpuError(f"{name} must be contiguous {dtype}")


def clock_probe(microseconds: int) -> int:
    """Median shader clock (MHz) the chip holds while every SIMD runs v_sad_u8
    chains for `microseconds` (p64gpu_clock_probe; synchronises the current
    stream)."""
    torch = _torch()
    mhz = ctypes.c_int(0)
    _check(lib().p64gpu_clock_probe(int(microseconds), ctypes.byref(mhz), _stream(torch)))
    return mhz.value


def block_op(op: int, blocks, dcq: int = 8, acq: int = 8, out=None):
    """Run one reference block routine over a batch of int32 [..., 64] device blocks."""
    torch = _torch()
    _dev_check(blocks, torch.int32, "blocks")
    if blocks.shape[-1] != 64:
        raise P64GpuError("blocks must have a trailing dimension of 64")
    if out is None:
        out = torch.empty_like(blocks)
    n = blocks.numel() // 64
    _check(lib().p64gpu_block_op(op, blocks.data_ptr(), out.data_ptr(), n, dcq, acq, _stream(torch)))
    return out


def ChenDct(x):  # chendct.c:97
    return block_op(OP_DCT, x)


def ChenIDct(x):  # chendct.c:217
    return block_op(OP_IDCT, x)


def CCITTQuantize(m, dcq, acq):  # transform.c:271 (returns a new tensor)
    return block_op(OP_QUANT_INTER, m, dcq, acq)


def CCITTFlatQuantize(m, dcq, acq):  # transform.c:317
    return block_op(OP_QUANT_INTRA, m, dcq, acq)


def ICCITTQuantize(m, dcq, acq):  # transform.c:400
    return block_op(OP_IQUANT_INTER, m, dcq, acq)


def ICCITTFlatQuantize(m, dcq, acq):  # transform.c:359
    return block_op(OP_IQUANT_INTRA, m, dcq, acq)


def BoundDctMatrix(m):  # transform.c:460
    return block_op(OP_BOUND_DCT, m)


def BoundIDctMatrix(m):  # transform.c:483
    return block_op(OP_BOUND_IDCT, m)


def FlatBoundQuantizeMatrix(m):  # transform.c:502
    return block_op(OP_BOUND_QFLAT, m)


def BoundQuantizeMatrix(m):  # transform.c:526
    return block_op(OP_BOUND_QUANT, m)


def ZigzagMatrix(m):  # transform.c:561
    return block_op(OP_ZIGZAG, m)


def IZigzagMatrix(m):  # transform.c:546
    return block_op(OP_IZIGZAG, m)


def MotionEstimation(ref, cur, width: int, height: int, mode: int = ME_TSS,
                     search_limit: int = 15, frame_stride: int | None = None, out=None):
    """me.c:340 over a batch: ref/cur are uint8 device tensors holding nframes
    pictures (or luma planes) `frame_stride` bytes apart.  Returns an int32
    tensor [nframes, nmb, 7] = (MeX, MeY, MeVal, MeOVal, MeVAR, MeVAROR, MeMWOR)
    (written into `out` when given)."""
    torch = _torch()
    _dev_check(ref, torch.uint8, "ref")
    _dev_check(cur, torch.uint8, "cur")
    stride = frame_stride or picture_bytes(width, height)
    nframes = cur.numel() // stride
    if nframes < 1 or ref.numel() < (nframes - 1) * stride + width * height:
        raise P64GpuError("ref/cur hold fewer pictures than the geometry needs")
    nmb = (width // 16) * (height // 16)
    if out is None:
        out = torch.empty((nframes, nmb, 7), dtype=torch.int32, device=cur.device)
    else:
        _dev_check(out, torch.int32, "out")
        if out.numel() < nframes * nmb * 7:
            raise P64GpuError("out smaller than nframes x nmb records")
    _check(lib().p64gpu_motion_estimation(width, height, nframes, stride, ref.data_ptr(),
                                          cur.data_ptr(), mode, search_limit, out.data_ptr(),
                                          _stream(torch)))
    return out


@dataclass
class FrameBatchOut:
    coef: object        # int16 [nframes, nmb, 6, 64]; inter pictures write only the
                        # blocks with a nonzero level (include/p64gpu.h)
    mb: object          # int8  [nframes, nmb, 4]  (mtype, cbp, mvx, mvy)
    me: object          # int32 [nframes, nmb, 7] or None
    nz: object = None   # uint8 [nframes, nmb] or None: bit 5-b set iff block b
                        # has a nonzero level (its levels were stored)
    vlc_bits: object = None  # int16 [nframes, nmb, 8] or None: entry 1 + b = block b's
                        # coded bits for the entropy coder (stream.vlc_pictures blk_bits)


def encode_frames(cur, ref, recon, last_intra, *, width: int, height: int, intra: bool,
                  quant: int = 8, me_mode: int = ME_TSS, search_limit: int = 15,
                  quant_mb=None, mtype_override=None, out: FrameBatchOut | None = None,
                  want_me: bool = True, me_given: bool = False, search_only: bool = False) -> FrameBatchOut:
    """One picture of each of `nframes` independent sequences (p64.c:622-1013).
    me_given: out.me already holds the batch's ME records (MotionEstimation
    over the same pictures, search mode and limit): the search is not run
    again (P64GPU_FLAG_ME_GIVEN).  search_only: the search alone into out.me
    (P64GPU_FLAG_SEARCH_ONLY; then the same call with me_given finishes the
    encode)."""
    torch = _torch()
    stride = picture_bytes(width, height)
    nframes = cur.numel() // stride
    nmb = (width // 16) * (height // 16)
    dev = cur.device
    _dev_check(cur, torch.uint8, "cur")
    _dev_check(recon, torch.uint8, "recon")
    _dev_check(last_intra, torch.uint8, "last_intra")
    if not intra:
        _dev_check(ref, torch.uint8, "ref")
    if quant_mb is not None:
        _dev_check(quant_mb, torch.uint8, "quant_mb")
    if mtype_override is not None:
        _dev_check(mtype_override, torch.int8, "mtype_override")
    need = nframes * stride
    nmb_all = nframes * nmb
    if nframes < 1 or recon.numel() < need or last_intra.numel() < nmb_all or \
            (not intra and ref.numel() < need) or \
            (quant_mb is not None and quant_mb.numel() < nmb_all) or \
            (mtype_override is not None and mtype_override.numel() < nmb_all):
        raise P64GpuError("buffer sizes do not match nframes x picture geometry")
    if out is None:
        out = FrameBatchOut(
            # zeroed: an inter picture's levels are written for the blocks with a
            # nonzero level only (P64GPU coef contract, include/p64gpu.h)
            coef=torch.zeros((nframes, nmb, 6, 64), dtype=torch.int16, device=dev),
            mb=torch.empty((nframes, nmb, 4), dtype=torch.int8, device=dev),
            me=torch.empty((nframes, nmb, 7), dtype=torch.int32, device=dev) if want_me else None)
    else:  # caller-supplied outputs: the kernels write nmb_all records into them
        _dev_check(out.coef, torch.int16, "out.coef")
        _dev_check(out.mb, torch.int8, "out.mb")
        if out.coef.numel() < nmb_all * 384 or out.mb.numel() < nmb_all * 4:
            raise P64GpuError("out.coef / out.mb smaller than nframes x nmb records")
        if out.vlc_bits is not None:
            _dev_check(out.vlc_bits, torch.int16, "out.vlc_bits")
            if out.vlc_bits.numel() < nmb_all * 8:
                raise P64GpuError("out.vlc_bits smaller than nframes x nmb x 8")
        if out.nz is not None:
            _dev_check(out.nz, torch.uint8, "out.nz")
            if out.nz.numel() < nmb_all:
                raise P64GpuError("out.nz smaller than nframes x nmb")
        if out.me is not None:
            _dev_check(out.me, torch.int32, "out.me")
            if out.me.numel() < nmb_all * 7:
                raise P64GpuError("out.me smaller than nframes x nmb records")
    # inter pictures always hand the library an ME-record buffer: a torch
    # allocation is stream- and graph-safe (the caching allocator), so the
    # library's own per-stream scratch is never needed from Python
    me = out.me
    if me_given and (intra or me is None):
        raise P64GpuError("me_given needs an inter batch and out.me holding its records")
    if search_only and (intra or me is None or me_given):
        raise P64GpuError("search_only needs an inter batch with out.me (and not me_given)")
    if me is None and not intra:
        me = torch.empty((nframes, nmb, 7), dtype=torch.int32, device=dev)
    a = EncodeArgs(width=width, height=height, nframes=nframes, intra=int(bool(intra)),
                   quant=quant, me_mode=me_mode, search_limit=search_limit,
                   flags=(P64GPU_FLAG_ME_GIVEN if me_given else 0) | (P64GPU_FLAG_SEARCH_ONLY if search_only else 0),
                   frame_stride=stride, cur=cur.data_ptr(),
                   ref=(ref.data_ptr() if ref is not None else None), recon=recon.data_ptr(),
                   last_intra=last_intra.data_ptr(),
                   quant_mb=(quant_mb.data_ptr() if quant_mb is not None else None),
                   mtype_override=(mtype_override.data_ptr() if mtype_override is not None else None),
                   coef=out.coef.data_ptr(), mb=out.mb.data_ptr(),
                   me=(me.data_ptr() if me is not None else None),
                   nzmask=(out.nz.data_ptr() if out.nz is not None else None),
                   vlc_bits=(out.vlc_bits.data_ptr() if out.vlc_bits is not None else None))
    _check(lib().p64gpu_encode_frames(ctypes.byref(a), _stream(torch)))
    return out


def prepare_encode(cur, ref, recon, last_intra, *, width: int, height: int, intra: bool, quant: int = 8,
                   me_mode: int = ME_TSS, search_limit: int = 15, out: FrameBatchOut, stream=None,
                   me_given: bool = False, search_only: bool = False):
    """encode_frames' launch with its arguments checked and packed once: the
    returned function issues it again with the same buffers (no per-call
    Python checks -- for host loops that relaunch the same step shapes, e.g.
    bench.py's fed path).  The tensors must outlive the returned function."""
    torch = _torch()
    stride = picture_bytes(width, height)
    nframes = cur.numel() // stride
    for t, dt, name in ((cur, torch.uint8, "cur"), (recon, torch.uint8, "recon"),
                        (last_intra, torch.uint8, "last_intra"), (out.coef, torch.int16, "out.coef"),
                        (out.mb, torch.int8, "out.mb")):
        _dev_check(t, dt, name)
    nmb_all = nframes * (width // 16) * (height // 16)
    if nframes < 1 or recon.numel() < nframes * stride or last_intra.numel() < nmb_all or \
            (not intra and (ref is None or ref.numel() < nframes * stride)) or \
            out.coef.numel() < nmb_all * 384 or out.mb.numel() < nmb_all * 4:
        raise P64GpuError("prepare_encode: buffer sizes do not match nframes x picture geometry")
    if out.me is None and not intra:
        raise P64GpuError("prepare_encode: inter batches need out.me")
    if (me_given or search_only) and (intra or (me_given and search_only)):
        raise P64GpuError("prepare_encode: me_given / search_only: one of them, inter batches only")
    flags = (P64GPU_FLAG_ME_GIVEN if me_given else 0) | (P64GPU_FLAG_SEARCH_ONLY if search_only else 0)
    a = EncodeArgs(width=width, height=height, nframes=nframes, intra=int(bool(intra)), quant=quant,
                   me_mode=me_mode, search_limit=search_limit, flags=flags, frame_stride=stride,
                   cur=cur.data_ptr(), ref=(ref.data_ptr() if ref is not None else None), recon=recon.data_ptr(),
                   last_intra=last_intra.data_ptr(), quant_mb=None, mtype_override=None,
                   coef=out.coef.data_ptr(), mb=out.mb.data_ptr(),
                   me=(out.me.data_ptr() if out.me is not None else None),
                   nzmask=(out.nz.data_ptr() if out.nz is not None else None),
                   vlc_bits=(out.vlc_bits.data_ptr() if out.vlc_bits is not None else None))
    st = ctypes.c_void_p((stream or torch.cuda.current_stream()).cuda_stream)
    L, ref_a = lib(), ctypes.byref(a)

    def launch():
        _check(L.p64gpu_encode_frames(ref_a, st))
    launch.args = a  # (kept alive with the function)
    return launch


def decode_recon(ref, recon, coef, mb, quant_mb, coded_mask, *, width: int, height: int):
    """Decoder reconstruction (p64.c:1179-1237 + 971-1013) of coded MBs into recon."""
    torch = _torch()
    for t, dt, name in ((ref, torch.uint8, "ref"), (recon, torch.uint8, "recon"),
                        (coef, torch.int16, "coef"), (mb, torch.int8, "mb"),
                        (quant_mb, torch.uint8, "quant_mb"), (coded_mask, torch.uint8, "coded_mask")):
        _dev_check(t, dt, name)
    stride = picture_bytes(width, height)
    nframes = recon.numel() // stride
    nmb_all = nframes * (width // 16) * (height // 16)
    if nframes < 1 or ref.numel() < nframes * stride or coef.numel() < nmb_all * 384 or \
            mb.numel() < nmb_all * 4 or quant_mb.numel() < nmb_all or coded_mask.numel() < nmb_all:
        raise P64GpuError("buffer sizes do not match nframes x picture geometry")
    _check(lib().p64gpu_decode_recon(width, height, nframes, stride, ref.data_ptr(),
                                     recon.data_ptr(), coef.data_ptr(), mb.data_ptr(),
                                     quant_mb.data_ptr(), coded_mask.data_ptr(), _stream(torch)))
    return recon


def decode_recon_packed(ref, recon, levels, nlevels: int, index, mb, quant_mb, coded_mask, *, width: int,
                        height: int):
    """decode_recon from the packed level layout (ABI v3,
    p64gpu_decode_recon_packed): levels int16 [>= nlevels, 64] holds only the
    transmitted blocks' levels in raster order, index uint32 [groups, 4] the
    per-64-block group entries (stream.pack_levels / pack_levels_device)."""
    torch = _torch()
    for t, dt, name in ((ref, torch.uint8, "ref"), (recon, torch.uint8, "recon"),
                        (levels, torch.int16, "levels"), (index, torch.int32, "index"), (mb, torch.int8, "mb"),
                        (quant_mb, torch.uint8, "quant_mb"), (coded_mask, torch.uint8, "coded_mask")):
        _dev_check(t, dt, name)
    stride = picture_bytes(width, height)
    nframes = recon.numel() // stride
    nmb = (width // 16) * (height // 16)
    nmb_all = nframes * nmb
    ngr = (nframes * 6 * nmb + 63) // 64  # groups of 64 blocks over the batch
    if nframes < 1 or ref.numel() < nframes * stride or levels.numel() < nlevels * 64 or \
            index.numel() < ngr * 4 or mb.numel() < nmb_all * 4 or quant_mb.numel() < nmb_all or \
            coded_mask.numel() < nmb_all:
        raise P64GpuError("buffer sizes do not match nframes x picture geometry")
    _check(lib().p64gpu_decode_recon_packed(width, height, nframes, stride, ref.data_ptr(), recon.data_ptr(),
                                            levels.data_ptr(), int(nlevels), index.data_ptr(), mb.data_ptr(),
                                            quant_mb.data_ptr(), coded_mask.data_ptr(), _stream(torch)))
    return recon


def pack_levels_device(coef, mb, coded_mask, width: int, height: int):
    """The packed layout of decode_recon_packed from device arrays in the
    dense layout (an encoder's levels and records, or the reader's): the
    same entries p64s_pack_levels makes on the host, by torch ops (a bench /
    test helper: the reader's host output goes through stream.pack_levels).
    Returns (levels [n, 64] int16, n, index [groups, 4] int32)."""
    torch = _torch()
    nmb = (width // 16) * (height // 16)
    mbr = mb.reshape(-1, nmb, 4)
    nf = mbr.shape[0]
    mt = mbr[..., 0].long()
    tc = torch.tensor(TCOEFF_MTYPE, device=mb.device)[mt]
    hc = torch.tensor(CBP_MTYPE, device=mb.device)[mt]
    cbp = torch.where(hc == 1, mbr[..., 1].long() & 63, torch.full_like(mt, 63))
    bits = (cbp[..., None] >> (5 - torch.arange(6, device=mb.device))) & 1  # [nf, nmb, 6]
    tx = (bits * tc[..., None] * (coded_mask.reshape(nf, nmb)[..., None] != 0)).reshape(-1)
    ngr = (nf * 6 * nmb + 63) // 64  # groups of 64 consecutive blocks of the batch
    pad = torch.zeros(ngr * 64, dtype=torch.long, device=mb.device)
    pad[:tx.numel()] = tx
    g = pad.reshape(ngr, 64)
    cnt = g.sum(dim=1)
    start = torch.cumsum(cnt, 0) - cnt
    w = (g.reshape(-1, 64) << torch.arange(64, device=mb.device)).sum(dim=1)  # (int64 wraps: bit 63 fine)
    index = torch.stack([start, torch.zeros_like(start), w & 0xFFFFFFFF, (w >> 32) & 0xFFFFFFFF], dim=1)
    index = index.to(torch.int64).to(torch.int32)
    sel = tx.nonzero().squeeze(1)
    levels = coef.reshape(-1, 64).index_select(0, sel).contiguous()
    return levels, int(sel.numel()), index.contiguous()


class Encoder:
    """Host-buffer closed-loop encoder (p64EncodeSequence/p64EncodeFrame,
    p64.c:524-683) through the C ABI's p64gpu_encoder_* context: numpy in,
    numpy out, reconstruction kept on the device between pictures."""

    def __init__(self, width: int, height: int, me_mode: int = ME_TSS, search_limit: int = 15,
                 device: int = 0):
        self.width, self.height = width, height
        self.nmb = (width // 16) * (height // 16)
        self._h = ctypes.c_void_p()
        _check(lib().p64gpu_encoder_open(device, width, height, me_mode, search_limit,
                                         ctypes.byref(self._h)))

    def frame(self, picture: np.ndarray, *, intra: bool, quant: int = 8, mtype_override=None,
              want_recon: bool = False):
        pic = np.ascontiguousarray(picture, dtype=np.uint8)
        if pic.size != picture_bytes(self.width, self.height):
            raise P64GpuError("picture has the wrong size")
        coef = np.empty((self.nmb, 6, 64), np.int16)
        mb = np.empty(self.nmb, MB_DTYPE)
        me = np.zeros(self.nmb, ME_DTYPE)
        recon = np.empty_like(pic) if want_recon else None
        ov = None
        if mtype_override is not None:
            ov = np.ascontiguousarray(mtype_override, dtype=np.int8)
        _check(lib().p64gpu_encoder_frame(self._h, pic.ctypes.data, int(bool(intra)), quant,
                                          ov.ctypes.data if ov is not None else None,
                                          coef.ctypes.data, mb.ctypes.data, me.ctypes.data,
                                          recon.ctypes.data if recon is not None else None))
        return coef, mb, me, recon

    def close(self):
        if self._h:
            lib().p64gpu_encoder_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
