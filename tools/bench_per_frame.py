#!/usr/bin/env python3
"""Latency of the per-frame C-ABI call (mp3d_decode_frame, the player's decode
call) on one GPU: host buffer in, host PCM out, one frame per call (4 kernel
launches + copies + a stream sync).  Prints one JSON line."""
import ctypes
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import _gen
    import mp3_amd
    data, offs = _gen.stream(_gen.C3, 7_000_001, 400)
    L = mp3_amd.lib()
    d = mp3_amd.Decoder()
    pcm = np.zeros(2304, np.int16)
    info = mp3_amd.FrameInfo()
    lat = []
    pos = 0
    for f in range(len(offs)):
        t = time.perf_counter()
        n = L.mp3d_decode_frame(d._h, data[pos:], len(data) - pos, pcm.ctypes.data, ctypes.byref(info))
        lat.append(time.perf_counter() - t)
        assert n == 1152
        pos += info.frame_bytes
    lat = np.array(lat[20:]) * 1e6  # after warm-up
    print(json.dumps({"workload": "per-frame mp3d_decode_frame, 128 kbps 44.1 kHz stereo, host buffers",
                      "frames": int(lat.size), "median_us": float(np.median(lat)), "p99_us": float(np.percentile(lat, 99)),
                      "realtime_x": 1152 / 44100 / (np.median(lat) * 1e-6)}))


if __name__ == "__main__":
    main()
