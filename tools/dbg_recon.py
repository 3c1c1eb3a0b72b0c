#!/usr/bin/env python3
"""Debug aid: encode a golden sequence's first pictures on the GPU and list
the macroblocks whose reconstruction differs from the CPU oracle's (type,
CBP, vector, which blocks, first differing row)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "oracle"), os.path.join(R, "tests")]


def main(name="cif_full31", n=2):
    import torch
    import oracle
    import p64_amd as p64
    from test_oracle_golden import load, sequence_frames
    from test_gpu_parity import sequence_params
    z = load(f"seq_{name}.npz")
    w, h = int(z["width"]), int(z["height"])
    prm = sequence_params(z)
    frames = sequence_frames(p64, z)[:n]
    exp = oracle.encode_sequence(frames, w, h, quant=prm["quant"], me_mode=prm["me_mode"],
                                 search_limit=prm["search_limit"])
    nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
    li = torch.zeros(nmb, dtype=torch.uint8, device="cuda")
    bufs = [torch.zeros(pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for t, f in enumerate(frames):
        cur = torch.from_numpy(f).cuda()
        o = p64.encode_frames(cur, bufs[(t + 1) % 2], bufs[t % 2], li, width=w, height=h, intra=(t == 0),
                              quant=prm["quant"], me_mode=prm["me_mode"], search_limit=prm["search_limit"])
        rec = bufs[t % 2].cpu().numpy()
        mb = o.mb.cpu().numpy()[0]
        erec = exp[t][3]
        print(f"picture {t}: coef equal {np.array_equal(o.coef.cpu().numpy()[0], exp[t][0])}, "
              f"recon equal {np.array_equal(rec, erec)}")
        if np.array_equal(rec, erec):
            continue
        Y = rec[:w * h].reshape(h, w).astype(int)
        EY = erec[:w * h].reshape(h, w).astype(int)
        shown = 0
        for k in range(nmb):
            by, bx = divmod(k, w // 16)
            d = Y[16 * by:16 * by + 16, 16 * bx:16 * bx + 16] - EY[16 * by:16 * by + 16, 16 * bx:16 * bx + 16]
            cd = []
            for c in range(2):
                uo = w * h + c * (w // 2) * (h // 2) + (8 * by) * (w // 2) + 8 * bx
                cu = [rec[uo + r * (w // 2):uo + r * (w // 2) + 8] for r in range(8)]
                ce = [erec[uo + r * (w // 2):uo + r * (w // 2) + 8] for r in range(8)]
                cd.append(any(not np.array_equal(a, b) for a, b in zip(cu, ce)))
            cd = tuple(cd) if any(cd) else False
            if d.any() or cd:
                blocks = [b for b in range(4) if d[8 * (b >> 1):8 * (b >> 1) + 8, 8 * (b & 1):8 * (b & 1) + 8].any()]
                print(f"  MB {k} ({bx},{by}) mtype {mb[k][0]} cbp {mb[k][1] & 63:#04x} mv ({mb[k][2]},{mb[k][3]}) "
                      f"exp mtype {exp[t][1][k]['mtype']} luma blocks {blocks} UV diff {cd} "
                      f"maxdiff {np.abs(d).max()}")
                shown += 1
                if shown > 20:
                    break


if __name__ == "__main__":
    main(*sys.argv[1:2])
