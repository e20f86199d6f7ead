#!/usr/bin/env python3
"""Every stream of the full-size C3 and C5 batches (65 536 streams x 32
frames each; and an LSF batch of the same size) against the oracle (oracle/liboracle.so, the double-precision
checker, on a 16-thread pool): the largest |GPU - oracle| per stream in
int16 LSB, as a histogram (tests/test_gpu_scale.py checks a stride-256
sample of the same batches).  Prints one JSON line.

    python tools/dbg/full_parity.py [c3|c5 ...]
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _gen  # noqa: E402
import _golden  # noqa: E402
import _oracle  # noqa: E402
import mp3_amd  # noqa: E402

CFG = {"c3": (_gen.C3, 3_000_000), "c5": (_gen.C5, 5_000_000),
       "lsf": (dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40), 7_000_000)}  # MPEG-2 / 2.5 LSF, all six rates


def run(name):
    cfg, base = CFG[name]
    n, F = 65536, 32
    t0 = time.time()
    buf, offs, sizes = _gen.batch(cfg, base, n, F, threads=16)
    d_in = torch.from_numpy(buf).cuda()
    pcm = torch.zeros((n, F, 2304), dtype=torch.int16, device="cuda")
    inf = torch.zeros((n, F, 6), dtype=torch.int32, device="cuda")
    mp3_amd.BatchDecoder(n, F).decode(d_in, offs, sizes, F, pcm=pcm, infos=inf)
    torch.cuda.synchronize()
    pcm = pcm.cpu().numpy()
    infs = inf.cpu().numpy().reshape(-1).view(mp3_amd.FRAME_INFO_DT).reshape(n, F)
    _oracle.lib()

    def one(s):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        o = _golden.to_int16(_oracle.decode_stream(data)[0])
        g = mp3_amd.pcm_to_planar(pcm[s], infs[s])
        if g.shape != o.shape:
            return 1 << 20
        return int(np.abs(g.astype(np.int32) - o.astype(np.int32)).max())

    with ThreadPoolExecutor(max_workers=16) as ex:
        d = np.fromiter(ex.map(one, range(n)), np.int64, n)
    hist = {str(k): int((d == k).sum()) for k in (0, 1)}
    hist[">1"] = int((d > 1).sum())
    return {"config": name, "streams": n, "frames": n * F, "max_lsb": int(d.max()), "streams_by_max_lsb": hist,
            "worst_streams": [int(s) for s in np.argsort(-d)[:5] if d[s] > 1], "seconds": round(time.time() - t0, 1)}


def main():
    out = []
    for name in sys.argv[1:] or ["c3", "c5"]:
        out.append(run(name))
        print(json.dumps(out[-1]), flush=True)
    sys.exit(0 if all(r["max_lsb"] <= 1 for r in out) else 1)


if __name__ == "__main__":
    main()
