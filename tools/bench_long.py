#!/usr/bin/env python3
"""Throughput of the frame-parallel long-stream decode (mp3d_batch_decode_long,
SURVEY.md §8(f) row 2) on one GPU: ONE synthetic 128 kbps 44.1 kHz joint
stereo stream of --frames frames (65 536 frames = 28.5 minutes of audio),
bytes and PCM resident in HBM, for several segment lengths L.  Prints one JSON
line per L: frames/s, warm-up overhead ((decoded - output) / output frames)
and the sequential reference point (the same stream as ONE batch stream is
latency-bound: one wave walks it)."""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--L", type=str, default="16,32,64,128")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seq-frames", type=int, default=2048, help="frames for the sequential reference point")
    args = ap.parse_args()
    import torch

    import _gen
    import mp3_amd
    data, _ = _gen.stream(_gen.C3, 4_000_001, args.frames)
    d_in = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    n = args.frames
    for L in [int(x) for x in args.L.split(",")]:
        offs, seg, wmax = mp3_amd.long_plan(data, L)
        K = len(seg)
        dec = mp3_amd.BatchDecoder(K, L + wmax)
        d_pcm = torch.empty((n, 2304), dtype=torch.int16, device="cuda")
        dec.decode_long(d_in, L, max_frames=n, pcm=d_pcm)  # warm-up (allocations, tables)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            dec.decode_long(d_in, L, max_frames=n, pcm=d_pcm)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        t = min(ts)
        decoded = int(sum(min(n, (k + 1) * L) - int(a) for k, a in enumerate(seg)))
        print(json.dumps({"workload": "one %d-frame C3 stream" % n, "L": L, "segments": K, "max_warmup": wmax,
                          "warmup_overhead": round(decoded / n - 1, 4), "s": round(t, 5),
                          "frames_per_s": round(n / t, 1), "audio_x_realtime": round(n * 1152 / 44100 / t, 1)}),
              flush=True)
        dec.close()
    # sequential reference: the stream as ONE batch stream (one wave walks it)
    m = min(args.seq_frames, n)
    end = int(mp3_amd.long_plan(data, 1)[0][m]) if m < n else len(data)
    dec = mp3_amd.BatchDecoder(1, m)
    d_pcm = torch.empty((1, m, 2304), dtype=torch.int16, device="cuda")
    dec.decode(d_in, [0], [end], m, pcm=d_pcm)
    dec.reset()
    torch.cuda.synchronize()
    t = time.perf_counter()
    dec.decode(d_in, [0], [end], m, pcm=d_pcm)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    print(json.dumps({"workload": "sequential: one stream, one batch stream", "frames": m, "s": round(t, 5),
                      "frames_per_s": round(m / t, 1)}), flush=True)


if __name__ == "__main__":
    main()
