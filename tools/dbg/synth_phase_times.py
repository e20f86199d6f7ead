#!/usr/bin/env python3
"""Where k_synth's wave time goes (diagnostic; MP3D_LIB=build_ab/PT.so from
abx/ptime.py): one C3 decode step (65 536 x 32 by default), then the summed
per-wave cycles of phases Q, I, M, W and the loop head as fractions, and
cycles per granule per wave."""
import ctypes
import json
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    assert "build_ab/PT" in os.environ.get("MP3D_LIB", ""), "set MP3D_LIB=build_ab/PT.so (or PT2.so)"
    import torch
    import _gen
    import mp3_amd
    cfg = _gen.C5 if os.environ.get("CONFIG") == "5" else _gen.C3
    n, F = int(os.environ.get("STREAMS", 65536)), 32
    buf, offs, sizes = _gen.batch(cfg, 3_000_003, n, F, threads=16)
    d_in = torch.from_numpy(buf).cuda()
    pcm = torch.empty((n, F, 2304), dtype=torch.int16, device="cuda")
    dec = mp3_amd.BatchDecoder(n, F)
    L = mp3_amd.lib()
    L.mp3d_dbg_ptime.argtypes = [ctypes.c_void_p]
    out = np.zeros(8, np.uint64)
    dec.decode(d_in, offs, sizes, F, pcm=pcm)  # warm-up
    torch.cuda.synchronize()
    L.mp3d_dbg_ptime(out.ctypes.data)
    dec.decode(d_in, offs, sizes, F, pcm=pcm)
    torch.cuda.synchronize()
    assert L.mp3d_dbg_ptime(out.ctypes.data) == 0
    names = ["Q", "I", "M", "W", "head", "Q:scales", "Q:requant", "Q:esc+stereo"]
    tot = float(out[:5].sum())
    gran = n * F * 2
    frac = {k: round(float(out[i]) / tot, 3) for i, k in enumerate(names)}
    frac["Q:scatter"] = round(frac["Q"] - frac["Q:scales"] - frac["Q:requant"] - frac["Q:esc+stereo"], 3)
    print(json.dumps({"fraction": frac,
                      "cycles_per_granule_per_wave": {k: round(float(out[i]) / gran, 1) for i, k in enumerate(names)},
                      "total_per_granule": round(tot / gran, 1), "streams": n}))


if __name__ == "__main__":
    main()
