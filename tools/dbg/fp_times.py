#!/usr/bin/env python3
"""k_demux_fp phase times from the FPT build (abx/variants.py): decode
tests/golden/long_c3_512 through the per-frame call and print, per read-ahead
run, the s_memrealtime deltas (us) the kernel left in the bitrate of the
run's first four frame infos: staging, state loads, wave 0's parse +
resolve, wave 0's emits."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _golden  # noqa: E402
import mp3_amd  # noqa: E402

data, _ = _golden.case("long_c3_512")
d = mp3_amd.Decoder()
rows = []
for rep in range(3):
    d.reset()
    pos, k, cur = 0, 0, []
    while pos < len(data):
        n, _, info = d.decode_frame(data[pos:])
        if info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        cur.append(info.bitrate_kbps)
        k += 1
    for r0 in range(0, len(cur) - 3, 64):
        rows.append([x / 100.0 for x in cur[r0:r0 + 4]])
a = np.array(rows)
print("runs", len(a))
print("median us: staging %.2f  state %.2f  parse + resolve %.2f  emit %.2f" % tuple(np.median(a, axis=0)))
