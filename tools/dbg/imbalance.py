#!/usr/bin/env python3
"""How much does k_synth lose to uneven work inside a workgroup?  (round 5
diagnosis).  A k_synth workgroup runs 8 streams, one per wave, and frees its
LDS only when its slowest wave ends.  Three C3 batches of 65 536 x 32 frames:
  N  every stream distinct (the bench's input)
  W  8 consecutive streams (one workgroup) share one stream's bytes: no
     imbalance inside a workgroup, the same variety across workgroups
  U  all 65 536 streams the same bytes
Prints the per-kernel HIP-event times of each (median of 5 calls)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gen  # noqa: E402
import mp3_amd  # noqa: E402

N, F = 65536, 32
buf, offs, sizes = _gen.batch(_gen.C3, 3_000_003, N, F, threads=16)
d_in = torch.from_numpy(buf).cuda()
cases = {
    "N": (offs, sizes),
    "W": (offs[(np.arange(N) // 8) * 8], sizes[(np.arange(N) // 8) * 8]),
    "U": (np.full(N, offs[0], np.uint64), np.full(N, sizes[0], np.uint32)),
}
dec = mp3_amd.BatchDecoder(N, F)
pcm = torch.empty((N, F, 2304), dtype=torch.int16, device="cuda")
infos = torch.zeros((N, F, 6), dtype=torch.int32, device="cuda")
res = {}
for name, (o, z) in cases.items():
    for _ in range(2):
        dec.reset()
        dec.decode(d_in, o, z, F, pcm=pcm, infos=infos)
    dec.set_timing(True)
    t = {"demux": [], "huffman": [], "synth": []}
    for _ in range(5):
        dec.reset()
        dec.decode(d_in, o, z, F, pcm=pcm, infos=infos)
        for k, v in dec.kernel_times_us().items():
            t[k].append(v)
    dec.set_timing(False)
    torch.cuda.synchronize()
    assert int((infos[..., 5] > 0).sum()) == N * F
    res[name] = {k: float(np.median(v)) for k, v in t.items()}
    print(name, " ".join("%s %.0f us" % kv for kv in res[name].items()), flush=True)
print("synth W/N %.3f, U/N %.3f; huffman W/N %.3f" % (res["W"]["synth"] / res["N"]["synth"],
                                                     res["U"]["synth"] / res["N"]["synth"],
                                                     res["W"]["huffman"] / res["N"]["huffman"]))
