#!/usr/bin/env python3
"""Decode tests/golden/long_c3_512 through the per-frame call once (the
read-ahead runs), for rocprof timing of the run kernels (MP3D_LIB picks an
A/B build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _golden  # noqa: E402
import mp3_amd  # noqa: E402

data, _ = _golden.case("long_c3_512")
d = mp3_amd.Decoder()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    d.reset()
    pcm = d.decode_stream(data)
print("frames", pcm.shape)
