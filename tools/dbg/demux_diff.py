"""Debug: first PCM difference between the wave and lane demux paths on the
test corpus (tests/test_gpu_demux_paths.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import test_gpu_demux_paths as T  # noqa: E402

streams = T._corpus()
a = T._run("wave", streams, 16, 0, False)
b = T._run("lane", streams, 16, 0, False)
names = T._golden.names()
for c, ((pa, ia, sa), (pb, ib, sb)) in enumerate(zip(a, b)):
    d = np.nonzero((pa != pb).any(axis=2))
    print("call", c, "differing (stream, frame):", list(zip(d[0].tolist(), d[1].tolist()))[:20])
    for s in sorted(set(d[0].tolist()))[:6]:
        nm = names[s] if s < len(names) else "gen/garbage %d" % (s - len(names))
        fr = d[1][d[0] == s]
        print("  stream", s, nm, "len", len(streams[s]), "frames", fr.tolist()[:10])
        print("   infos", ia[s][:6].tolist())

# UnitMeta / is[] of the differing stream through huffman_only, both paths
s = 16
data = streams[s]
half = len(data) // 2
blob = np.frombuffer(data[:half] + b"\0" * 64, np.uint8)
res = {}
for path in ("wave", "lane"):
    os.environ["MP3D_DEMUX"] = path
    dec = T.mp3_amd.BatchDecoder(1, 16)
    res[path] = dec.huffman_only(blob, np.array([0], np.uint64), np.array([half], np.uint32), 16)
    os.environ.pop("MP3D_DEMUX")
for k in range(len(res["wave"])):
    x, y = np.asarray(res["wave"][k]), np.asarray(res["lane"][k])
    print("output", k, x.shape, x.dtype, "equal", np.array_equal(x, y))
    if not np.array_equal(x, y) and x.ndim >= 1:
        idx = np.argwhere(x != y)
        print("  first diffs", idx[:10].tolist())
        print("  wave", x.reshape(-1)[np.flatnonzero(x != y)[:10]].tolist(), "lane", y.reshape(-1)[np.flatnonzero(x != y)[:10]].tolist())
