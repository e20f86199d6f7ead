#!/usr/bin/env python3
"""Read-ahead first-call stress (round 4's one-off
first-call mismatch on lsf_scale_24k_is).  For R rounds, every golden stream
is decoded through the per-frame call by a FRESH decoder with read-ahead
(16 frames per run), alternately with and without MP3D_DEBUG_POISON, and
compared frame by frame with one single-frame-path decode (read-ahead 0) of
the same stream.  A mismatch prints its stream, round and frame.  One process,
one progress line per round.  Prints one JSON line at the end.

    python tools/dbg/ra_stress.py [ROUNDS] [--seconds S]
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

import _golden  # noqa: E402
import mp3_amd  # noqa: E402


def _dec(ra, poison):
    keep = {k: os.environ.get(k) for k in ("MP3D_PF_READAHEAD", "MP3D_DEBUG_POISON")}
    os.environ["MP3D_PF_READAHEAD"] = str(ra)
    if poison:
        os.environ["MP3D_DEBUG_POISON"] = "1"
    else:
        os.environ.pop("MP3D_DEBUG_POISON", None)
    try:
        return mp3_amd.Decoder()
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _decode(d, data):
    pos, out = 0, []
    while pos < len(data) and len(out) < 600:
        n, pcm, info = d.decode_frame(data[pos:], last=True)
        if info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        out.append(pcm.copy())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rounds", type=int, nargs="?", default=10)
    ap.add_argument("--seconds", type=float, default=150.0, help="stop after this long (whole rounds)")
    a = ap.parse_args()
    names = _golden.names()
    ref = {}
    for nm in names:
        data, _ = _golden.case(nm)
        ref[nm] = (data, _decode(_dec(0, False), data))
    t0, fresh, frames, bad = time.time(), 0, 0, []
    r = 0
    for r in range(a.rounds):
        for i, nm in enumerate(names):
            data, want = ref[nm]
            got = _decode(_dec(16, (r + i) % 2 == 1), data)
            fresh += 1
            frames += len(got)
            if len(got) != len(want):
                bad.append({"stream": nm, "round": r, "frames": [len(got), len(want)]})
                continue
            for f, (x, y) in enumerate(zip(got, want)):
                if not np.array_equal(x, y):
                    bad.append({"stream": nm, "round": r, "frame": f})
                    break
        print("round %d: %d fresh decoders, %d frames, %d mismatches, %.0f s" % (r, fresh, frames, len(bad),
                                                                               time.time() - t0), flush=True)
        if time.time() - t0 > a.seconds:
            break
    print(json.dumps({"rounds": r + 1, "streams": len(names), "fresh_decoders": fresh, "frames": frames,
                      "mismatches": bad, "seconds": round(time.time() - t0, 1)}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
