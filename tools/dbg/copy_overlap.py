"""Can a step's PCM copy hide behind the next step's decode on one GPU?
(VERDICT r05 "do this" 8: the world-1 gather hid 11 % of itself.)

Times, on one MI355X, for the C3 workload (65 536 streams x 32 frames):
  decode alone            (mp3d_batch_decode on stream A)
  copy alone              (the step's 9.66 GB of int16 PCM into a receive
                           buffer: torch copy_ on stream B = hipMemcpyAsync
                           device to device)
  decode + copy together  (step k+1's decode on A while step k's copy runs
                           on B, double-buffered PCM, as bench.py --gather)
and prints one JSON line: hidden fraction = (decode + copy - together) / copy.
Usage: python tools/dbg/copy_overlap.py [--steps 6] [--streams 65536]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _gen  # noqa: E402
import mp3_amd  # noqa: E402
from mp3_amd import shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--frames", type=int, default=32)
    a = ap.parse_args()
    n, F = a.streams, a.frames
    dev = torch.device("cuda:0")
    buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(0, n, shard.BASE_SEED_C3), n, F, threads=16)
    d_in = torch.from_numpy(buf).to(dev)
    pcm = [torch.empty((n, F, 2304), dtype=torch.int16, device=dev) for _ in range(2)]
    recv = [torch.empty_like(pcm[0]) for _ in range(2)]
    dec = mp3_amd.BatchDecoder(n, F, device=0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def decode(k):
        dec.decode(d_in, offs, sizes, F, pcm=pcm[k % 2], stream=sa.cuda_stream)

    def copy(k):
        with torch.cuda.stream(sb):
            recv[k % 2].copy_(pcm[k % 2], non_blocking=True)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    for k in range(2):
        decode(k)
        copy(k)
    torch.cuda.synchronize()
    t_dec = timed(lambda: [decode(k) for k in range(a.steps)])
    t_cp = timed(lambda: [copy(k) for k in range(a.steps)])
    done = [torch.cuda.Event(), torch.cuda.Event()]
    decoded = [torch.cuda.Event(), torch.cuda.Event()]

    def together():
        for k in range(a.steps + 1):
            if k < a.steps:
                if k >= 2:
                    sa.wait_event(done[k % 2])  # decode k overwrites the buffer copy k-2 reads
                decode(k)
                decoded[k % 2].record(sa)
            if k >= 1:
                j = k - 1
                sb.wait_event(decoded[j % 2])
                copy(j)
                done[j % 2].record(sb)
    t_both = timed(together)
    ok = bool(torch.equal(recv[(a.steps - 1) % 2], pcm[(a.steps - 1) % 2]))
    print(json.dumps({"probe": "copy_overlap", "streams": n, "frames": F, "copy_bytes": pcm[0].numel() * 2,
                      "ms_decode": t_dec, "ms_copy": t_cp, "ms_together": t_both,
                      "copy_GBs": pcm[0].numel() * 2 / t_cp / 1e6,
                      "hidden_fraction": (t_dec + t_cp - t_both) / t_cp, "copy_ok": ok}))


if __name__ == "__main__":
    main()
