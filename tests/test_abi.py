"""CPU-side checks of the C ABI (no GPU needed): the library loads, exports
every entry point include/p64gpu.h declares, lays out its structs the way the
ctypes mirror does, and rejects bad arguments before touching a device."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

HEADERS = [os.path.join(REPO, "include", h) for h in ("p64gpu.h", "p64stream.h", "p64seq.h")]


def declared_functions():
    names = set()
    for hdr in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
        names |= set(re.findall(r"\b(p64(?:gpu|seq|s)?_\w+)\s*\(", text))
    return sorted(names)


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ("p64gpu_block_op", "p64gpu_motion_estimation", "p64gpu_encode_frames",
              "p64gpu_decode_recon", "p64gpu_encoder_open", "p64gpu_encoder_frame",
              "p64gpu_encoder_close", "p64gpu_synth_frames", "p64_synth_frame",
              "p64gpu_copy_on_device", "p64s_write_picture", "p64s_write_end",
              "p64s_read_picture", "p64s_reader_open", "p64gpu_encode_mb_list",
              "p64s_write_mb", "p64seq_open", "p64seq_encode", "p64seq_finish",
              "p64gpu_decode_recon_packed", "p64s_pack_levels", "p64s_write_bits"):
        assert n in names


def test_library_exports_every_declared_symbol(p64):
    out = subprocess.run(["nm", "-D", "--defined-only", p64.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_abi_version_and_strings(p64):
    L = p64.lib()
    assert L.p64gpu_abi_version() == 3 == p64.ABI_VERSION
    assert L.p64gpu_strerror(0) == b"ok"
    assert L.p64gpu_strerror(-1) == b"invalid argument"


def test_struct_layout_matches_ctypes(p64, tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "p64gpu.h"
#define O(f) printf("%s %zu\n", #f, offsetof(p64gpu_encode_args, f))
int main(void) {
  printf("sizeof_args %zu\nsizeof_me %zu\nsizeof_mb %zu\n", sizeof(p64gpu_encode_args),
         sizeof(p64_me_rec), sizeof(p64_mb_rec));
  O(width); O(height); O(nframes); O(intra); O(quant); O(me_mode); O(search_limit);
  O(flags); O(frame_stride); O(cur); O(ref); O(recon); O(last_intra); O(quant_mb);
  O(mtype_override); O(coef); O(mb); O(me); O(nzmask); O(vlc_bits);
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                 check=True).stdout.splitlines())
    assert int(got["sizeof_args"]) == ctypes.sizeof(p64.EncodeArgs)
    assert int(got["sizeof_me"]) == ctypes.sizeof(p64.MeRec) == p64.ME_DTYPE.itemsize
    assert int(got["sizeof_mb"]) == ctypes.sizeof(p64.MbRec) == p64.MB_DTYPE.itemsize
    for name, _ in p64.EncodeArgs._fields_:
        assert int(got[name]) == getattr(p64.EncodeArgs, name).offset, name


def test_invalid_arguments_rejected_without_device(p64):
    L = p64.lib()
    a = p64.EncodeArgs(width=100, height=64, nframes=1, quant=8, frame_stride=9600)
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"multiples of 16" in L.p64gpu_last_error()
    assert L.p64gpu_encode_frames(None, None) == -1
    a = p64.EncodeArgs(width=176, height=144, nframes=1, quant=0, frame_stride=38016,
                       cur=16, recon=16, last_intra=16, coef=16, mb=16, intra=1)
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"quant" in L.p64gpu_last_error()
    # flags: unknown bits, and P64GPU_FLAG_ME_GIVEN without an inter batch with records
    a = p64.EncodeArgs(width=176, height=144, nframes=1, quant=8, frame_stride=38016, me_mode=1,
                       search_limit=31, cur=16, ref=16, recon=16, last_intra=16, coef=16, mb=16,
                       flags=4)
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"flags" in L.p64gpu_last_error()
    a.flags = p64.P64GPU_FLAG_SEARCH_ONLY  # args.me is NULL
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"SEARCH_ONLY" in L.p64gpu_last_error()
    a.flags = p64.P64GPU_FLAG_SEARCH_ONLY | p64.P64GPU_FLAG_ME_GIVEN
    a.me = 16
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"SEARCH_ONLY" in L.p64gpu_last_error()
    a.me = None
    a.flags = p64.P64GPU_FLAG_ME_GIVEN  # args.me is NULL
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"ME_GIVEN" in L.p64gpu_last_error()
    a.me, a.intra = 16, 1
    assert L.p64gpu_encode_frames(ctypes.byref(a), None) == -1
    assert b"ME_GIVEN" in L.p64gpu_last_error()
    assert L.p64gpu_block_op(99, 16, 16, 1, 8, 8, None) == -1
    assert L.p64gpu_block_op(2, 16, 16, 1, 8, 0, None) == -1  # acq 0
    assert L.p64gpu_block_op(0, None, None, 0, 8, 8, None) == 0  # empty batch is a no-op
    assert L.p64gpu_motion_estimation(176, 144, 1, 176 * 144, 16, 16, 7, 15, 16, None) == -1
    assert L.p64gpu_motion_estimation(176, 144, 1, 176 * 144, 16, 16, 1, 32, 16, None) == -1
    assert L.p64gpu_synth_frames(176, 144, 1, 0, 0, 1, 38016, 16, None) == -1
    assert L.p64gpu_synth_content(7, 176, 144, 1, 1, 0, 1, 38016, 16, None) == -1
    assert b"content" in L.p64gpu_last_error()
    out = np.empty(176 * 144 * 3 // 2, np.uint8)
    assert L.p64_synth_frame_content(2, 1, 0, 176, 144, out.ctypes.data) == -1
    # entropy coder: flags must be 0, scratch 8-byte aligned (ABI version 2)
    from p64_amd import stream as p64s
    stride = (int(L.p64gpu_vlc_max_bytes(176, 144)) + 3) // 4 * 4
    v = p64s.VlcArgs(width=176, height=144, nframes=1, flags=1, mb=16, coef=16, gquant=16, tr=16,
                     out=16, out_stride=stride, bits=16, scratch=16)
    assert L.p64gpu_vlc_pictures(ctypes.byref(v), None) == -1
    assert b"flags" in L.p64gpu_last_error()
    v.flags, v.scratch = 0, 20
    assert L.p64gpu_vlc_pictures(ctypes.byref(v), None) == -1
    assert b"aligned" in L.p64gpu_last_error()


def test_vlc_args_layout_matches_ctypes(p64, tmp_path):
    from p64_amd import stream as p64s
    src = tmp_path / "vlayout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "p64gpu.h"
#define O(f) printf("%s %zu\n", #f, offsetof(p64gpu_vlc_args, f))
int main(void) {
  printf("sizeof_args %zu\n", sizeof(p64gpu_vlc_args));
  O(width); O(height); O(nframes); O(flags); O(mb); O(coef); O(gquant); O(mquant); O(tr);
  O(phase); O(out); O(out_stride); O(bits); O(scratch); O(blk_bits); O(seq_bits); O(max_bits);
  return 0;
}''')
    exe = tmp_path / "vlayout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                 check=True).stdout.splitlines())
    assert int(got["sizeof_args"]) == ctypes.sizeof(p64s.VlcArgs)
    for name, _ in p64s.VlcArgs._fields_:
        assert int(got[name]) == getattr(p64s.VlcArgs, name).offset, name


def test_device_count_without_gpu_is_not_an_error(p64):
    n = ctypes.c_int(-1)
    assert p64.lib().p64gpu_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


def test_synth_is_deterministic_and_moves(p64):
    a = p64.synth_frame(9, 3, 176, 144)
    b = p64.synth_frame(9, 3, 176, 144)
    assert np.array_equal(a, b)
    mvx, mvy = p64.synth_motion(9)
    f0 = p64.synth_frame(6, 0, 176, 144)[: 176 * 144].reshape(144, 176)  # seed 6: no noise
    f1 = p64.synth_frame(6, 1, 176, 144)[: 176 * 144].reshape(144, 176)
    mx, my = p64.synth_motion(6)
    # frame 1 at (x, y) == frame 0 at (x + mx, y + my) for the noise-free class
    assert np.array_equal(f1[20:100, 20:100], f0[20 + my:100 + my, 20 + mx:100 + mx])
    assert (mvx, mvy) == (9 % 7 - 3, (9 // 7) % 5 - 2)


def test_survey_content_follows_survey_8d(p64):
    """--content survey: deterministic; picture t is picture
    t-1 translated by (+3, -2) px up to the N(0,4) temporal noise (the
    residual at the true shift has sigma 4 sqrt 2); the texture's spread is
    that of 50 sin cos + 30 sin + N(0,12) (sigma ~35); chroma is derived from
    the 2x2-averaged luma; seeds differ."""
    w, h = 352, 288
    S = p64.SYNTH_SURVEY
    a = p64.synth_frame(3, 5, w, h, content=S)
    assert np.array_equal(a, p64.synth_frame(3, 5, w, h, content=S))
    assert not np.array_equal(a, p64.synth_frame(4, 5, w, h, content=S))
    f = [p64.synth_frame(3, t, w, h, content=S) for t in range(3)]
    Y = [x[:w * h].reshape(h, w).astype(np.int32) for x in f]
    for t in (1, 2):
        d = Y[t][0:h - 2, 3:w] - Y[t - 1][2:h, 0:w - 3]  # (x, y) <- (x - 3, y + 2)
        assert abs(d.mean()) < 0.2 and 5.3 < d.std() < 6.1, (d.mean(), d.std())
        assert (Y[t] - Y[t - 1]).std() > 15  # the zero vector is far worse
    assert 127 < Y[0].mean() < 129.5 and 32 < Y[0].std() < 38
    U = f[0][w * h:w * h + w * h // 4].reshape(h // 2, w // 2).astype(np.int32)
    a4 = Y[0][0::2, 0::2] + Y[0][1::2, 0::2] + Y[0][0::2, 1::2] + Y[0][1::2, 1::2]
    a = (a4 + 2) >> 2
    np.testing.assert_array_equal(U, np.clip(128 + np.trunc((a - 128) / 2).astype(np.int32), 0, 255))
    # the sinusoid part: the 1/7 rad/px carrier is among the strongest
    # components of the luma's power spectrum
    P = np.abs(np.fft.rfft2(Y[0] - Y[0].mean())) ** 2
    fy, fx = np.unravel_index(np.argsort(P, axis=None)[-8:], P.shape)
    fxs = {round(2 * np.pi * x / w, 2) for x in fx}
    assert any(abs(v - 1 / 7) < 0.03 for v in fxs), fxs


def test_host_driver_built():
    exe = os.path.join(REPO, "p64_amd", "p64gpu")
    assert os.access(exe, os.X_OK)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr


def test_product_does_not_reference_oracle():
    """The product path never routes through the checker."""
    for root in ("p64_amd",):
        for dirpath, _, files in os.walk(os.path.join(REPO, root)):
            for f in files:
                if f.endswith((".py", ".hip", ".c", ".h")):
                    text = open(os.path.join(dirpath, f), errors="ignore").read()
                    assert "import oracle" not in text and "liboracle" not in text, f
                    assert "orc_" not in text, f
