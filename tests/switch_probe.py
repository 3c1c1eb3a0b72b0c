"""Helper for test_gpu_parity.test_env_switches_same_bytes (not a test module):
encodes an intra and a FULL-search inter picture of two CIF sequences and
decodes the inter picture, then prints one SHA-256 over every output.  Run in
a subprocess so that the library reads its environment switches afresh."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p64_amd  # noqa: E402


def main():
    w, h, S = 352, 288, 2
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    fr = [torch.from_numpy(np.stack([p64_amd.synth_frame(41 + s, t, w, h) for s in range(S)])).cuda()
          for t in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    r0 = torch.zeros(S * pic, dtype=torch.uint8, device="cuda")
    r1 = torch.zeros_like(r0)
    o0 = p64_amd.encode_frames(fr[0].reshape(-1), None, r0, li, width=w, height=h, intra=True, quant=7)
    o1 = p64_amd.encode_frames(fr[1].reshape(-1), r0, r1, li, width=w, height=h, intra=False, quant=7,
                               me_mode=p64_amd.ME_FULL, search_limit=31)
    qmb = torch.full((S * nmb,), 7, dtype=torch.uint8, device="cuda")
    d1 = torch.zeros_like(r0)
    p64_amd.decode_recon(r0, d1, o1.coef, o1.mb, qmb, torch.ones_like(qmb), width=w, height=h)
    torch.cuda.synchronize()
    hsh = hashlib.sha256()
    for t in (o0.coef, o0.mb, r0, o1.coef, o1.mb, o1.me, r1, d1, li):
        hsh.update(t.cpu().numpy().tobytes())
    print(hsh.hexdigest())


if __name__ == "__main__":
    main()
