#!/usr/bin/env python3
"""Phase times of k_frame inside the per-frame call (diagnostic).  Run with
MP3D_LIB=build_ab/FRT.so (abx/variants.py FRT): after every mp3d_decode_frame the
variant's g_fdbg holds s_memtime at kernel start, after wave 0's frame
staging and demux, after waves 1-3's table staging, after the barriers, at each
wave's Huffman end, after the synthesis and after the completion fence.  Prints medians (us) as one
JSON line, plus the host-side call time for comparison."""
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    assert os.environ.get("MP3D_LIB", "").endswith("FRT.so"), "set MP3D_LIB=build_ab/FRT.so"
    import _gen
    import mp3_amd
    data, offs = _gen.stream(_gen.C3, 7_000_001, 300)
    L = mp3_amd.lib()
    L.mp3d_dbg_read.argtypes = [ctypes.c_void_p]
    d = mp3_amd.Decoder()
    pcm = np.zeros(2304, np.int16)
    info = mp3_amd.FrameInfo()
    dbg = np.zeros(64, np.uint64)
    rows, lat = [], []
    pos = 0
    for f in range(len(offs)):
        t = time.perf_counter()
        n = L.mp3d_decode_frame(d._h, data[pos:], len(data) - pos, pcm.ctypes.data, ctypes.byref(info))
        lat.append(time.perf_counter() - t)
        assert n == 1152
        pos += info.frame_bytes
        assert L.mp3d_dbg_read(dbg.ctypes.data) == 0
        if f >= 20:
            rows.append(dbg.astype(np.int64).copy())
    a = np.array(rows)
    ghz = float(np.median((a[:, 12] - a[:, 0]) / ((a[:, 21] - a[:, 20]) * 10.0)))
    us = lambda i, j: float(np.median(a[:, j] - a[:, i]) / ghz / 1e3)
    out = {"clock_ghz": ghz,
           "frame_stage_us": us(0, 1), "demux_us": us(1, 2), "tables_waves123_us": us(0, 3),
           "barrier1_us": us(2, 5), "huff_wave_us": [us(5, 6 + w) for w in range(4)], "barrier3_us": us(5, 10),
           "synth_us": us(10, 11), "fence_us": us(11, 12), "kernel_us": us(0, 12),
           "call_median_us": float(np.median(np.array(lat[20:]) * 1e6))}
    h = a[:, 32:].reshape(len(a), 4, 8)  # per unit: staged, scalefactors, big_values, count1 stamps
    hu = lambda x: [round(float(np.median(x[:, w])) / ghz / 1e3, 2) for w in range(4)]
    out["huff_unit_us"] = {"until_staged": hu(h[:, :, 0] - a[:, 5:6]), "scalefactors": hu(h[:, :, 1] - h[:, :, 0]),
                           "big_values": hu(h[:, :, 2] - h[:, :, 1]), "count1": hu(h[:, :, 3] - h[:, :, 2])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
