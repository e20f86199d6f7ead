#!/usr/bin/env python3
"""Does k_huffman's time depend on where the batch buffers land?  (round 5:
the same box ran k_huffman at 3.17 and 3.65 ms in two bench processes whose
only difference was one more 9.66 GB PCM buffer allocated before the
decoder).  Allocates a pad of P GB, then a C3 decoder (65 536 x 32), decodes
and prints the per-kernel HIP-event times (median of 3) and the buffers'
addresses (MP3D_DEBUG_ADDR)."""
import os
import sys

import numpy as np
import torch

os.environ["MP3D_DEBUG_ADDR"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gen  # noqa: E402
import mp3_amd  # noqa: E402

N, F = 65536, 32
buf, offs, sizes = _gen.batch(_gen.C3, 3_000_003, N, F, threads=16)
d_in = torch.from_numpy(buf).cuda()
pcm = torch.empty((N, F, 2304), dtype=torch.int16, device="cuda")
infos = torch.zeros((N, F, 6), dtype=torch.int32, device="cuda")
args = sys.argv[1:]
if args and args[0].startswith("warm"):  # warmN: N seconds of HBM copies first (clock ramp?)
    secs = float(args.pop(0)[4:] or 1)
    a = torch.empty(int(2e9), dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    import time
    t0 = time.time()
    while time.time() - t0 < secs:
        b.copy_(a)
        torch.cuda.synchronize()
    del a, b
for pad_gb in [float(x) for x in (args or ["0", "9.66", "1", "2.5", "4", "0.3"])]:
    pad = torch.empty(int(pad_gb * 1e9) + 1, dtype=torch.uint8, device="cuda")
    dec = mp3_amd.BatchDecoder(N, F)
    if os.environ.get("PLACE_SLEEP"):  # idle after the allocations (a background VRAM clear?)
        import time
        time.sleep(float(os.environ["PLACE_SLEEP"]))
    dec.decode(d_in, offs, sizes, F, pcm=pcm, infos=infos)
    dec.set_timing(True)
    t = {"demux": [], "huffman": [], "synth": []}
    for _ in range(3):
        dec.reset()
        dec.decode(d_in, offs, sizes, F, pcm=pcm, infos=infos)
        for k, v in dec.kernel_times_us().items():
            t[k].append(v)
    torch.cuda.synchronize()
    print("pad %.2f GB:" % pad_gb, " ".join("%s %.0f" % (k, np.median(v)) for k, v in t.items()), flush=True)
    dec.close()
    del dec, pad
    torch.cuda.empty_cache()
