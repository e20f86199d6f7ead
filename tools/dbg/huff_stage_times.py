#!/usr/bin/env python3
"""Where k_huffman wave time goes (diagnostic; MP3D_LIB=build_ab/HT.so from
abx/htime.py): one C3 decode step (65 536 x 32 by default), then the summed
per-wave cycles of its stages (ranking, round set-up, staging,
scalefactors, big_values, count1, meta) as fractions, and cycles per unit
per wave."""
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
    assert os.environ.get("MP3D_LIB", "").endswith("HT.so"), "set MP3D_LIB=build_ab/HT.so"
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
    names = ["rank", "round", "stage", "scalefactors", "big_values", "count1", "meta_store", "meta_build"]
    tot = float(out[:8].sum())
    units = n * F * 4
    print(json.dumps({"fraction": {k: round(float(out[i]) / tot, 3) for i, k in enumerate(names)},
                      "cycles_per_unit_per_wave": {k: round(float(out[i]) / units, 1) for i, k in enumerate(names)},
                      "streams": n}))

if __name__ == "__main__":
    main()
