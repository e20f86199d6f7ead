#!/usr/bin/env python3
"""Benchmark: stereo MP3 frames/s (128 kbps, 44.1 kHz) on MI355X.

Workload (BASELINE.json configs[2]): 65,536 synthetic CBR
128 kbps 44.1 kHz joint-stereo streams x 32 frames per step, per GPU.  A step
is one mp3d_batch_decode call over every stream's next 32 frames (the full
hot path: demux + reservoir + Huffman + requantise/stereo + IMDCT +
polyphase synthesis -> int16 PCM), inputs resident in HBM, PCM written to
HBM.  Per-stream decoder state stays resident across steps.

Multi-GPU: one process per GPU (torchrun), streams sharded by global stream
id (seed 3_000_003 + id), no collective on the data path -> weak scaling.
Timing: barrier + synchronize on both sides of exactly K steps, max over
ranks.  The dominant kernel's duration comes from HIP events recorded on
the stream the kernels run on (mp3d_batch_kernel_times).

The CPU baseline is the oracle restatement (oracle/liboracle.so, "port")
on a bounded sample of the same workload, rank 0 only.
"""
import argparse
import ctypes
import json
import os
import pathlib
import sys
import threading
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3       # FP32 vector == FP32 MFMA (MI355X_MICROARCH.md)
BYTES_IN_PER_FRAME = 417.96    # 128 kbps @ 44.1 kHz
PCM_BYTES_PER_FRAME = 4608.0   # 1152 x 2 ch x int16
# algorithmic FLOPs per stereo frame: dense 32x32 matrixing
# + 512-tap window per slot (72 slot-channels) + IMDCT (4 units x 32 sb x 2*18*18)
FLOP_PER_FRAME = 72 * (2 * 32 * 32 + 2 * 512) + 4 * 32 * 2 * 18 * 18
# MFMA work of the DCT tile (phase M): 24 v_mfma_f32_16x16x4_f32 (2 048 flop
# each) per granule, 2 granules per frame -- the butterfly-halved matrixing
MFMA_FLOP_PER_FRAME = 2 * 24 * 2048
# k_synth algorithmic bytes per frame: is[] int16 in (4 x 576 x 2) + PCM out
SYNTH_BYTES_PER_FRAME = 4 * 576 * 2 + PCM_BYTES_PER_FRAME


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(buf, offs, sizes, F, threads=None, budget_s=12.0):
    """Oracle (scalar C restatement, oracle/liboracle.so) decoding the first
    streams of the SAME C3 input the GPU decodes, one stream per task on all
    host threads, stopping after ~budget_s seconds (bounded sample)."""
    import _oracle
    threads = threads or min(16, os.cpu_count() or 1)
    L = _oracle.lib()
    n_streams = len(offs)
    out = [np.zeros((2, F * 1152), np.float32) for _ in range(threads)]
    _oracle.decode_stream(bytes(buf[offs[0]:offs[0] + sizes[0]]), F)  # init tables before threads
    done = [0] * threads
    streams_done = [0] * threads
    t_end = [0.0]

    def work(tid):
        nch, hz = ctypes.c_int(), ctypes.c_int()
        for s in range(tid, n_streams, threads):
            if time.perf_counter() > t_end[0]:
                break
            d = bytes(buf[offs[s]:offs[s] + sizes[s]])
            done[tid] += L.orc_decode_stream(d, len(d), out[tid].ctypes.data, F, ctypes.byref(nch), ctypes.byref(hz))
            streams_done[tid] += 1

    t0 = time.perf_counter()
    t_end[0] = t0 + budget_s
    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    frames = sum(done)
    # single-thread point on a short sample (single- and all-core)
    t1, f1 = time.perf_counter(), 0
    nch, hz = ctypes.c_int(), ctypes.c_int()
    for s in range(n_streams - 1, -1, -1):
        if time.perf_counter() - t1 > budget_s / 4:
            break
        d = bytes(buf[offs[s]:offs[s] + sizes[s]])
        f1 += L.orc_decode_stream(d, len(d), out[0].ctypes.data, F, ctypes.byref(nch), ctypes.byref(hz))
    dt1 = time.perf_counter() - t1
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "single_thread_value": f1 / dt1, "cpu_model": model, "host_cpus": os.cpu_count(),
            "sample": "first %d streams x %d frames (%d frames) of the same C3 input, decoded by "
                      "oracle/liboracle.so (double-precision scalar restatement, gcc -O2) on %d host threads in "
                      "%.1f s; single thread: %d frames in %.1f s" % (sum(streams_done), F, frames, threads, dt, f1, dt1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=65536, help="streams per GPU")
    ap.add_argument("--frames", type=int, default=32, help="frames per stream per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true", help="also time an RCCL PCM gather to rank 0 (reported apart)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank path with several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import _gen
    import mp3_amd
    from mp3_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; ranks beyond the visible GPUs (a gloo rehearsal on a
    # one-GPU box) share them round-robin
    gpu = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", gpu)
    n, F = args.streams, args.frames

    # --- synthetic C3 shard of this rank (seed by global stream id) -------
    t0 = time.time()
    gen_threads = min(16, os.cpu_count() or 1)
    buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(rank, n), n, F, threads=gen_threads)
    log("rank %d: generated %d streams x %d frames (%.1f MB) in %.1fs" % (rank, n, F, buf.size / 1e6, time.time() - t0))
    d_in = torch.from_numpy(buf).to(dev)
    pcm = torch.empty((n, F, 2304), dtype=torch.int16, device=dev)
    infos = torch.zeros((n, F, 6), dtype=torch.int32, device=dev)
    dec = mp3_amd.BatchDecoder(n, F, device=gpu)
    strm = torch.cuda.current_stream(dev).cuda_stream

    def step():
        dec.decode(d_in, offs, sizes, F, pcm=pcm, infos=infos, stream=strm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ok = int((infos[..., 5] == 1152).sum().item())
    if ok != n * F:
        raise SystemExit("decode produced %d/%d frames" % (ok, n * F))

    # --- timed region -------------------------------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = shard.max_over_ranks(time.perf_counter() - t0, dev)
    frames_total = n * F * world * args.steps
    value = frames_total / dt
    ms_per_step = dt / args.steps * 1e3

    # --- per-kernel device time (HIP events on the decode stream) ---------
    dec.set_timing(True)
    kt = {"demux": 0.0, "huffman": 0.0, "synth": 0.0}
    reps = max(1, min(3, args.steps))
    for _ in range(reps):
        step()
        for k, v in dec.kernel_times_us().items():
            kt[k] += v / reps
    dec.set_timing(False)
    torch.cuda.synchronize(dev)
    dom = max(kt, key=kt.get)
    frames_per_launch = n * F
    synth_s = kt["synth"] * 1e-6
    flops = FLOP_PER_FRAME * frames_per_launch
    achieved_tf = flops / synth_s / 1e12 if synth_s > 0 else 0.0

    traffic = mfma_util = None
    prof = ROOT / "profiles" / "pmc_traffic.json"
    if prof.exists():
        try:
            pj = json.loads(prof.read_text())
            if pj.get("streams") == n and pj.get("frames") == F:
                traffic = pj.get("k_synth_hbm_bytes_per_launch")
                mfma_util = pj.get("k_synth_mfma_util")
        except Exception:
            traffic = mfma_util = None

    gather = None
    if args.gather and world > 1:
        # optional xGMI PCM gather to rank 0 (RCCL), timed apart from decode
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        shard.gather_to_root(pcm)
        torch.cuda.synchronize(dev)
        gather = {"ms": (time.perf_counter() - tg) * 1e3, "bytes": pcm.numel() * 2 * world}

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(buf, offs, sizes, F)
        step_s = dt / args.steps
        res = {
            "metric": "stereo MP3 frames/s (128 kbps 44.1 kHz) at 1/2/4/8 GPU; % HBM roofline",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded generator: valid CBR 128 kbps 44.1 kHz joint-stereo MP3 frames)",
            "config": {"workload": "C3: full Layer III decode (Huffman->PCM), %d streams x %d frames per GPU per step"
                                   % (n, F),
                       "streams_per_gpu": n, "frames_per_stream": F, "bitrate_kbps": 128, "hz": 44100,
                       "parallelism": "streams sharded, 1 process per GPU, no data-path collective"},
            "roofline": {
                "kernel": "k_synth", "bound": "mfma", "unit": "TFLOP/s",
                "achieved": achieved_tf, "peak": FP32_PEAK_TFLOPS, "frac": achieved_tf / FP32_PEAK_TFLOPS,
                "flop_per_frame": FLOP_PER_FRAME, "frames_per_launch": frames_per_launch,
                "launch_us": kt["synth"],
                "achieved_GBs_algorithmic": SYNTH_BYTES_PER_FRAME * frames_per_launch / synth_s / 1e9 if synth_s else 0,
                "traffic": traffic,
                "dct_tile": {
                    "mfma_flop_per_frame": MFMA_FLOP_PER_FRAME,
                    "mfma_tflops": MFMA_FLOP_PER_FRAME * frames_per_launch / synth_s / 1e12 if synth_s else 0,
                    "mfma_util_pmc": mfma_util,
                    "note": "matrix-core busy fraction of k_synth from rocprofv3 (SQ_VALU_MFMA_BUSY_CYCLES, "
                            "profiles/pmc_traffic.json); peak 157.3 TFLOP/s FP32 MFMA",
                },
            },
            "hbm": {
                "hbm_rw_frac": value / world * (BYTES_IN_PER_FRAME + PCM_BYTES_PER_FRAME) / (HBM_PEAK_GBS * 1e9),
                "hbm_read_frac": value / world * BYTES_IN_PER_FRAME / (HBM_PEAK_GBS * 1e9),
                "bytes_per_frame_rw": BYTES_IN_PER_FRAME + PCM_BYTES_PER_FRAME,
            },
            "kernel_us": kt,
            "dominant_kernel": "k_" + dom,
            "cpu_baseline": cpu,
        }
        if gather:
            res["gather"] = gather
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
