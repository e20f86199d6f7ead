#!/usr/bin/env python3
"""Batch-path first-call stress (the batch side): fresh
BatchDecoders, alternately with and without MP3D_DEBUG_POISON, each decode
the same batch twice (the second call continues the streams: carry, overlap
and synthesis history from the first), and every output -- PCM of both calls
and the streams' state after them -- must equal the first decoder's bit for
bit.  Batches: a wide MPEG-1 mixed corpus (k_walk +
k_mdcopy + k_huffman), a wide LSF one, and a narrow one (k_demux,
k_huffman_wave).  One progress line per round, one JSON line at the end.

    python tools/dbg/batch_stress.py [ROUNDS] [--seconds S]
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

import _gen  # noqa: E402
import mp3_amd  # noqa: E402


def _new(n, F, poison):
    keep = os.environ.get("MP3D_DEBUG_POISON")
    if poison:
        os.environ["MP3D_DEBUG_POISON"] = "1"
    else:
        os.environ.pop("MP3D_DEBUG_POISON", None)
    try:
        return mp3_amd.BatchDecoder(n, F)
    finally:
        if keep is None:
            os.environ.pop("MP3D_DEBUG_POISON", None)
        else:
            os.environ["MP3D_DEBUG_POISON"] = keep


def _run(case, poison):
    buf, offs, sizes, n, F = case
    d = _new(n, F, poison)
    # the batch twice: the second call continues every stream (carry, overlap
    # and synthesis history from the first; its first frames' reservoir
    # reaches into the first call's tail)
    out = []
    for _ in range(2):
        pcm, _ = d.decode(buf, offs, sizes, F)
        out.append(np.asarray(pcm).copy())
    out.append(np.asarray(d.get_state(0, n)).copy())
    return out


def _case(cfg, seed, n, F):
    buf, offs, sizes = _gen.batch(cfg, seed, n, F, threads=8)
    return buf, offs, sizes, n, F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rounds", type=int, nargs="?", default=10)
    ap.add_argument("--seconds", type=float, default=150.0)
    a = ap.parse_args()
    lsf = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)
    cases = {"wide_mpeg1": _case(_gen.C5, 4711, 512, 8), "wide_lsf": _case(lsf, 4712, 512, 8),
             "narrow": _case(_gen.C5, 4713, 32, 8)}
    ref = {k: _run(c, False) for k, c in cases.items()}
    t0, runs, bad, r = time.time(), 0, [], 0
    for r in range(a.rounds):
        for i, (k, c) in enumerate(cases.items()):
            got = _run(c, (r + i) % 2 == 0)
            runs += 1
            for j, (x, y) in enumerate(zip(got, ref[k])):
                if not np.array_equal(x, y):
                    bad.append({"case": k, "round": r, "output": j})
        print("round %d: %d fresh decoders, %d mismatches, %.0f s" % (r, runs, len(bad), time.time() - t0),
              flush=True)
        if time.time() - t0 > a.seconds:
            break
    print(json.dumps({"rounds": r + 1, "cases": list(cases), "fresh_decoders": runs, "mismatches": bad,
                      "seconds": round(time.time() - t0, 1)}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
