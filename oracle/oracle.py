"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the PVRG-P64 hot path (p64_oracle.c).  Importable only
from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the
product (p64_amd/) never touches it.  Pinned against the reference by
tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

ME_TSS, ME_FULL = 0, 1
ME_DTYPE = np.dtype([(n, "<i4") for n in ("mx", "my", "sad", "sad0", "var", "varor", "mwor")])
MB_DTYPE = np.dtype([(n, "i1") for n in ("mtype", "cbp", "mvx", "mvy")])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i = ctypes.c_void_p, ctypes.c_int
        for n in ("orc_chen_dct", "orc_chen_idct", "orc_zigzag", "orc_izigzag"):
            getattr(L, n).argtypes = [vp, vp]
        for n in ("orc_quant_inter", "orc_quant_intra", "orc_iquant_intra", "orc_iquant_inter"):
            getattr(L, n).argtypes = [vp, i, i]
        for n in ("orc_bound_dct", "orc_bound_idct", "orc_bound_quant_flat", "orc_bound_quant"):
            getattr(L, n).argtypes = [vp]
        L.orc_sad16.argtypes = [vp, i, vp, i]
        L.orc_sad16.restype = i
        L.orc_me_mb.argtypes = [vp, vp, i, i, i, i, i, i, vp]
        L.orc_motion_estimation.argtypes = [vp, vp, i, i, i, i, vp]
        L.orc_load_filter.argtypes = [vp, i, vp]
        L.orc_encode_frame.argtypes = [i, i, vp, vp, vp, i, i, vp, vp, vp, i, i, vp, vp, vp, vp]
        L.orc_decode_mb.argtypes = [i, i, vp, vp, i, i, i, i, i, i, i, vp]
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _ptr(a):
    return a.ctypes.data if a is not None else None


def block_apply(name: str, blocks: np.ndarray, *qargs) -> np.ndarray:
    """Apply one oracle block routine to every [64] block of `blocks`."""
    src = _i32(blocks).reshape(-1, 64)
    out = np.empty_like(src)
    f = getattr(lib(), name)
    for k in range(src.shape[0]):
        if name in ("orc_chen_dct", "orc_chen_idct", "orc_zigzag", "orc_izigzag"):
            f(src[k].ctypes.data, out[k].ctypes.data)
        else:
            out[k] = src[k]
            f(out[k].ctypes.data, *qargs)
    return out.reshape(np.shape(blocks))


def motion_estimation(ref_y: np.ndarray, cur_y: np.ndarray, width: int, height: int,
                      mode: int = ME_TSS, search_limit: int = 15) -> np.ndarray:
    nmb = (width // 16) * (height // 16)
    recs = np.zeros(nmb, ME_DTYPE)
    r = np.ascontiguousarray(ref_y, np.uint8)
    c = np.ascontiguousarray(cur_y, np.uint8)
    lib().orc_motion_estimation(r.ctypes.data, c.ctypes.data, width, height, mode, search_limit,
                                recs.ctypes.data)
    return recs


def encode_frame(width, height, cur, ref, last_intra, *, intra, quant=8, me_mode=ME_TSS,
                 search_limit=15, quant_mb=None, mtype_override=None, me_in=None):
    """One picture (p64.c:622-1013).  Returns (coef[nmb,6,64] int16, mb recs,
    me recs or None, recon picture); last_intra is updated in place."""
    nmb = (width // 16) * (height // 16)
    cur = np.ascontiguousarray(cur, np.uint8)
    ref = np.ascontiguousarray(ref, np.uint8) if ref is not None else np.zeros_like(cur)
    recon = np.zeros_like(cur)
    coef = np.zeros((nmb, 6, 64), np.int16)
    mb = np.zeros(nmb, MB_DTYPE)
    me = None if intra else np.zeros(nmb, ME_DTYPE)
    assert last_intra.dtype == np.uint8 and last_intra.flags.c_contiguous
    qmb = np.ascontiguousarray(quant_mb, np.uint8) if quant_mb is not None else None
    ov = np.ascontiguousarray(mtype_override, np.int8) if mtype_override is not None else None
    mi = np.ascontiguousarray(me_in, ME_DTYPE) if me_in is not None else None
    lib().orc_encode_frame(width, height, cur.ctypes.data, ref.ctypes.data, recon.ctypes.data,
                           int(bool(intra)), quant, _ptr(qmb), _ptr(ov), last_intra.ctypes.data,
                           me_mode, search_limit, _ptr(mi), _ptr(me), coef.ctypes.data,
                           mb.ctypes.data)
    return coef, mb, me, recon


def encode_sequence(frames, width, height, *, quant=8, me_mode=ME_TSS, search_limit=15,
                    mtype_override=None):
    """Closed-loop sequence (p64EncodeSequence p64.c:524): first picture intra,
    each later picture predicted from the previous reconstruction."""
    nmb = (width // 16) * (height // 16)
    li = np.zeros(nmb, np.uint8)
    ref = None
    outs = []
    for t, f in enumerate(frames):
        ov = None if (mtype_override is None or t == 0) else mtype_override
        coef, mb, me, recon = encode_frame(width, height, f, ref, li, intra=(t == 0), quant=quant,
                                           me_mode=me_mode, search_limit=search_limit,
                                           mtype_override=ov)
        outs.append((coef, mb, me, recon))
        ref = recon
    return outs


def decode_mb(width, height, ref, recon, mbx, mby, mtype, cbp, mvx, mvy, quant, coef):
    c = np.ascontiguousarray(coef, np.int16)
    lib().orc_decode_mb(width, height, ref.ctypes.data, recon.ctypes.data, mbx, mby, mtype, cbp,
                        mvx, mvy, quant, c.ctypes.data)
