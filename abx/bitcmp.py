#!/usr/bin/env python3
"""Bit-identity check of an A/B variant against another: decode fixed C3,
C5 and LSF batches plus the C2 spectra with the library MP3D_LIB points at
and save PCM + state (python abx/bitcmp.py save OUT.npz), then compare two
saves (python abx/bitcmp.py cmp A.npz B.npz)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def save(out):
    import torch
    import _gen
    import mp3_amd
    res = {}
    lsf = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)
    for name, cfg, n, F in (("c3", _gen.C3, 1024, 16), ("c5", _gen.C5, 1024, 16), ("lsf", lsf, 512, 16)):
        buf, offs, sizes = _gen.batch(cfg, 4242, n, F, threads=8)
        for f32 in (False, True):
            dec = mp3_amd.BatchDecoder(n, F)
            pcm, infos = dec.decode(buf, offs, sizes, F, f32=f32)
            res["%s_%d_pcm" % (name, f32)] = pcm
            res["%s_%d_st" % (name, f32)] = dec.get_state(0, n)
    xr, bt, mx = _gen.c2_spectra(1024, 32, 2, seed=77)
    dec = mp3_amd.BatchDecoder(1024, 32)
    res["c2_pcm"] = dec.synth_only(xr, bt, mx, 2, 44100)
    res["c2_st"] = dec.get_state(0, 1024)
    torch.cuda.synchronize()
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k], B[k])
        if not same:
            bad += 1
            d = np.abs(A[k].astype(np.float64) - B[k].astype(np.float64)) if "pcm" in k else None
            print("DIFF", k, "" if d is None else "max %g, %d elements" % (d.max(), int((d > 0).sum())))
    print("bitcmp %s vs %s: %s" % (a, b, "IDENTICAL" if not bad else "%d arrays differ" % bad))
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
