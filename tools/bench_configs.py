#!/usr/bin/env python3
"""Throughput on BASELINE.json's other single-GPU configurations (bench.py's
headline line stays C3).  One JSON line per workload, inputs resident in HBM,
timed with synchronize on both sides of --steps calls after --warmup calls:

  c2   configs[1]: 1 024 streams, IMDCT + polyphase synthesis only from
       synthetic spectra (xr ~ N(0, sigma_k^2) with spectral
       tilt, 85 % long blocks, start/short/stop runs, some mixed), F = 64
  c5   configs[4]: mixed corpus -- VBR 32-320 kbps, mono / stereo / joint
       M/S / IS, 32 / 44.1 / 48 kHz, short + mixed blocks, CRC on some
       streams (per-stream divergence); frames/s and GB/s on actual bytes
  lsf  MPEG-2/2.5 LSF corpus (16-24 kHz and 8-12 kHz, VBR, all modes)
  c3_f32  C3 decoded to the float32 PCM sink (9 216 B/frame out)
  c3_crc  C3 streams with CRC protection, MP3D_OPT_CRC_CHECK on

Usage: python tools/bench_configs.py [--only c2,c5,lsf]"""
import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps


def c2(args):
    import torch
    import mp3_amd
    n, F, nch = 1024, 64, 2
    rng = np.random.default_rng(1_000_003 * 2)
    sig = (0.05 * (1 + np.arange(576) / 16.0) ** -1.5).astype(np.float32)
    xr = (rng.standard_normal((n, F, 2, nch, 576), dtype=np.float32) * sig)
    bt = np.zeros((n, F, 2, nch), np.uint8)
    mx = np.zeros((n, F, 2, nch), np.uint8)
    # ~15 % of granules in start -> short -> short -> stop runs, 5 % of short granules mixed
    for s in range(n):
        for f in range(1, F - 2, 8):
            if rng.random() < 0.6:
                bt[s, f, 1] = 1
                bt[s, f + 1, :] = 2
                bt[s, f + 2, 0] = 3
                if rng.random() < 0.1:
                    mx[s, f + 1, :] = 1
    d_xr, d_bt, d_mx = (torch.from_numpy(a).cuda() for a in (xr, bt, mx))
    pcm = torch.empty((n, F, 2304), dtype=torch.int16, device="cuda")
    dec = mp3_amd.BatchDecoder(n, F)
    strm = torch.cuda.current_stream().cuda_stream
    t = timed(lambda: dec.synth_only(d_xr, d_bt, d_mx, nch, 44100, pcm=pcm, stream=strm), args.steps, args.warmup)
    frames = n * F
    short = float((bt == 2).mean())
    return {"workload": "c2: synth only (IMDCT + polyphase), %d streams x %d frames, synthetic spectra" % (n, F),
            "frames_per_s": frames / t, "ms_per_step": t * 1e3, "short_granule_frac": round(short, 3),
            "algorithmic_GBs": frames * (9216 + 4608) / t / 1e9,
            "note": "1 024 streams fill 256 workgroups = 1 wave per SIMD; the latency-bound per-stream walk "
                    "is the limit (C3's 65 536 streams fill the chip)"}


def decode_corpus(args, name, cfg, n, F, f32=False, opts=0):
    import torch
    import _gen
    import mp3_amd
    buf, offs, sizes = _gen.batch(cfg, 5_000_011, n, F, threads=min(16, os.cpu_count() or 1))
    d_in = torch.from_numpy(buf).cuda()
    pcm = torch.empty((n, F, 2304), dtype=torch.float32 if f32 else torch.int16, device="cuda")
    infos = torch.zeros((n, F, 6), dtype=torch.int32, device="cuda")
    dec = mp3_amd.BatchDecoder(n, F)
    dec.set_options(opts)
    strm = torch.cuda.current_stream().cuda_stream
    t = timed(lambda: dec.decode(d_in, offs, sizes, F, pcm=pcm, infos=infos, stream=strm, f32=f32), args.steps,
              args.warmup)
    inf = infos.cpu().numpy()
    frames = int((inf[..., 5] > 0).sum())
    samples = int((inf[..., 5] * inf[..., 1]).sum())
    nbytes = int(sizes.astype(np.int64).sum())
    return {"workload": "%s: %d streams x %d frames" % (name, n, F), "frames_per_s": frames / t,
            "ms_per_step": t * 1e3, "frames_with_audio": frames, "in_GBs": nbytes / t / 1e9,
            "rw_GBs": (nbytes + (4 if f32 else 2) * samples) / t / 1e9, "mean_frame_bytes": round(nbytes / (n * F), 1),
            "hz_mix": {str(int(h)): int((inf[..., 2] == h).sum()) for h in np.unique(inf[..., 2]) if h}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c2,c5,lsf,c3_f32,c3_crc")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--frames", type=int, default=32)
    args = ap.parse_args()
    import _gen
    import mp3_amd
    for w in args.only.split(","):
        if w == "c2":
            r = c2(args)
        elif w == "c5":
            r = decode_corpus(args, "c5 mixed corpus (VBR 32-320 kbps, mono/stereo/MS/IS, 32/44.1/48 kHz, "
                                    "short+mixed blocks, CRC)", _gen.C5, args.streams, args.frames)
        elif w == "lsf":
            r = decode_corpus(args, "MPEG-2/2.5 LSF corpus (8-24 kHz, VBR, all modes)",
                              dict(_gen.C5, sr_idx=-2, short_pct=15, mixed_pct=25), args.streams, args.frames)
        elif w == "c3_f32":
            r = decode_corpus(args, "C3 with the float32 PCM sink", _gen.C3, args.streams, args.frames, f32=True)
        elif w == "c3_crc":
            r = decode_corpus(args, "C3 with CRC-protected frames and MP3D_OPT_CRC_CHECK on",
                              dict(_gen.C3, crc_pct=100), args.streams, args.frames, opts=mp3_amd.OPT_CRC_CHECK)
        else:
            raise SystemExit("unknown workload " + w)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
