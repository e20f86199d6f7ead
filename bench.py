#!/usr/bin/env python3
"""Benchmark: stereo MP3 frames/s (128 kbps, 44.1 kHz) on MI355X.

Workloads (BASELINE.json configs); --config picks one:
  3 (default)  65,536 synthetic CBR 128 kbps 44.1 kHz joint-stereo streams x 32
               frames per GPU per step: one mp3d_batch_decode call over every
               stream's next 32 frames (the full hot path: demux + reservoir +
               Huffman + requantise/stereo + IMDCT + polyphase synthesis ->
               int16 PCM), inputs resident in HBM, PCM written to HBM,
               per-stream decoder state resident across steps.  At --gpus 8
               this is configs[3] (C4: 524,288 streams over 8 GPUs).
  2            1,024 streams x 64 frames, IMDCT + polyphase synthesis only from
               synthetic spectra (mp3d_batch_synth_only), per GPU.
  5            mixed corpus (VBR 32-320 kbps, mono / stereo / M/S / IS,
               32 / 44.1 / 48 kHz, short + mixed blocks, CRC), 65,536 x 32 per GPU.
  1            one 128 kbps stream (tests/golden/keypress_128k_js.mp3) through
               the per-frame drop-in call (mp3d_decode_frame), host buffers.

Multi-GPU: one process per GPU.  `bench.py --gpus N` without WORLD_SIZE in
the environment starts the N rank processes itself (fresh children, before
anything touches a GPU; the parent never does) and relays rank 0's JSON line;
under torchrun (WORLD_SIZE set) it is one rank.  Streams are sharded by global
stream id (seed base + id), no collective on the data path -> weak scaling.
Timing: barrier + synchronize on both sides of exactly K steps, max over
ranks.  --gather adds a second timed loop in which an RCCL PCM gather of step
k to rank 0 runs on the process group's stream while step k+1 decodes; it is
reported apart and never enters `value`.  The dominant kernel's duration
comes from HIP events on the stream the kernels run on
(mp3d_batch_kernel_times).

The CPU baseline (rank 0, N = 1 only) is the oracle restatement built in
single precision at -O3 with AVX-512 (oracle/liboracle_f32.so, "port": the
reference has no decoder to build), timed on a bounded sample of the same
input on the host threads this process may use, plus single-thread points
for it and for the double-precision checker build.
"""
import argparse
import ctypes
import json
import os
import pathlib
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

METRIC = "stereo MP3 frames/s (128 kbps 44.1 kHz) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3       # FP32 vector == FP32 MFMA (MI355X_MICROARCH.md)
BYTES_IN_PER_FRAME = 417.96    # 128 kbps @ 44.1 kHz
PCM_BYTES_PER_FRAME = 4608.0   # 1152 x 2 ch x int16
# algorithmic FLOPs per stereo frame: dense 32x32 matrixing
# + 512-tap window per slot (72 slot-channels) + IMDCT (4 units x 32 sb x 2*18*18)
FLOP_PER_FRAME = 72 * (2 * 32 * 32 + 2 * 512) + 4 * 32 * 2 * 18 * 18
# FLOPs k_synth actually issues per stereo frame: fast 36-point
# IMDCT ~250 per (unit, subband) incl. window + overlap (4 x 32 x 250), the
# butterfly-halved matrixing on 48 MFMA columns (2 gr x 24 x 2 048) + its
# butterfly adds (2 x 36 x 32), the window (72 x 1 024), requantise (4 x 576 x 2)
EXEC_FLOP_PER_FRAME = 4 * 32 * 250 + 2 * 24 * 2048 + 2 * 36 * 32 + 72 * 1024 + 4 * 576 * 2
# MFMA work of the DCT tile (phase M): 24 v_mfma_f32_16x16x4_f32 (2 048 flop
# each) per granule, 2 granules per frame -- the butterfly-halved matrixing
MFMA_FLOP_PER_FRAME = 2 * 24 * 2048
# C2 algorithmic bytes per frame: xr f32 in (2 gr x 2 ch x 576 x 4) + PCM out
C2_BYTES_PER_FRAME = 2 * 2 * 576 * 4 + PCM_BYTES_PER_FRAME
C2_FLOP_PER_FRAME = FLOP_PER_FRAME  # IMDCT + matrixing + window (requantise is outside C2)


_json_out = sys.stdout  # the JSON line's stream (main() points it at the real stdout)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads():
    """Host threads this process may use: the box's CPU share (OMP_NUM_THREADS
    is set to it on the GPU box) within the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_model():
    try:
        return next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        return ""


# ----------------------------------------------------------------------------
# CPU baseline (oracle restatement; test infrastructure, timed, never shipped)
# ----------------------------------------------------------------------------
def _oracle_libs():
    import _oracle
    L64 = _oracle.lib()
    p32 = ROOT / "oracle" / "liboracle_f32.so"
    if not p32.exists():
        subprocess.check_call(["make", "-s", "-C", str(ROOT / "oracle")])
    L32 = ctypes.CDLL(str(p32))
    for L in (L32,):
        L.orc_decode_stream.argtypes = L64.orc_decode_stream.argtypes
        L.orc_decode_stream.restype = ctypes.c_long
        L.orc_create.restype = ctypes.c_void_p
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        L.orc_synth_only.argtypes = L64.orc_synth_only.argtypes
    return L32, L64


def _timed_pool(task, n_tasks, threads, budget_s):
    """Run task(i, tid) -> frames for i = 0.. on `threads` threads until the
    budget is spent (ctypes drops the GIL inside the C call)."""
    done = [0] * threads
    tasks = [0] * threads
    t_end = time.perf_counter() + budget_s

    def work(tid):
        for i in range(tid, n_tasks, threads):
            if time.perf_counter() > t_end:
                break
            done[tid] += task(i, tid)
            tasks[tid] += 1

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return sum(done), sum(tasks), time.perf_counter() - t0


def cpu_baseline_decode(buf, offs, sizes, F, budget_s=12.0):
    """Oracle decoding the SAME input the GPU decodes, one stream per task."""
    L32, L64 = _oracle_libs()
    threads = host_threads()
    outs = [np.zeros((2, F * 1152), np.float32) for _ in range(threads)]
    n = len(offs)

    def task_for(L):
        def task(s, tid):
            nch, hz = ctypes.c_int(), ctypes.c_int()
            d = bytes(buf[offs[s]:offs[s] + sizes[s]])
            return L.orc_decode_stream(d, len(d), outs[tid].ctypes.data, F, ctypes.byref(nch), ctypes.byref(hz))
        return task

    task_for(L32)(0, 0)  # tables initialised before the threads start
    task_for(L64)(0, 0)
    frames, streams, dt = _timed_pool(task_for(L32), n, threads, budget_s)
    f1, _, dt1 = _timed_pool(task_for(L32), n, 1, budget_s / 6)
    g1, _, gt1 = _timed_pool(task_for(L64), n, 1, budget_s / 6)
    return {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "single_thread_value": f1 / dt1, "f64_single_thread_value": g1 / gt1,
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": "first %d streams x %d frames (%d frames) of the same input, decoded by oracle/liboracle_f32.so "
                      "(the oracle restatement in float32, gcc -O3 -march=x86-64-v4) on %d host threads (the "
                      "process's CPU share) in %.1f s; single thread %d frames in %.1f s; the double-precision "
                      "checker build (-O2) %d frames in %.1f s on one thread"
                      % (streams, F, frames, threads, dt, f1, dt1, g1, gt1)}


def cpu_baseline_synth(xr, bt, mx, nch, budget_s=10.0):
    """Oracle stages a8..a11 (orc_synth_only) on the same C2 spectra."""
    L32, _ = _oracle_libs()
    threads = host_threads()
    n, F = xr.shape[0], xr.shape[1]
    pcms = [np.zeros((F, 1152, nch), np.int16) for _ in range(threads)]

    def task(s, tid):
        d = L32.orc_create()
        L32.orc_synth_only(d, xr[s].ctypes.data, bt[s].ctypes.data, mx[s].ctypes.data, F, nch, 0,
                           pcms[tid].ctypes.data, None)
        L32.orc_destroy(d)
        return F

    task(0, 0)
    frames, streams, dt = _timed_pool(task, n, threads, budget_s)
    f1, _, dt1 = _timed_pool(task, n, 1, budget_s / 4)
    return {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "single_thread_value": f1 / dt1, "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": "first %d streams x %d frames of the same C2 spectra through orc_synth_only "
                      "(oracle/liboracle_f32.so, float32 -O3 -march=x86-64-v4) on %d threads in %.1f s"
                      % (streams, F, threads, dt)}


# ----------------------------------------------------------------------------
# Rank launcher (--gpus N without torchrun)
# ----------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """Start n rank processes of this script (one per GPU) and relay rank
    0's stdout.  The parent touches no GPU: the children are fresh processes,
    not forks or execs of a process that has initialised HIP.  Exits with the
    first non-zero child status (the other ranks are then terminated)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", str(pathlib.Path(__file__).resolve())] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []
    relay = threading.Thread(target=lambda: out.extend(procs[0].stdout), daemon=True)
    relay.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    relay.join(timeout=10)
    for line in out:  # the JSON line to stdout, anything else (library chatter) to stderr
        (sys.stdout if line.startswith(b"{") else sys.stderr).write(line.decode())
    sys.stdout.flush()
    if rc:
        log("bench.py: a rank exited with status %d" % rc)
    return rc


# ----------------------------------------------------------------------------
# Workloads
# ----------------------------------------------------------------------------
class Ctx:
    pass


def setup_decode(c, cfg_name):
    import torch
    import _gen
    import mp3_amd
    from mp3_amd import shard
    cfg = _gen.C3 if cfg_name == "c3" else _gen.C5
    base = c.seed if c.seed is not None else shard.BASE_SEED_C3 if cfg_name == "c3" else 5_000_011
    t0 = time.time()
    # the ranks share the host: each generates with its share of the threads
    c.gen_threads = max(1, min(16, host_threads() // c.world))
    buf, offs, sizes = _gen.batch(cfg, shard.shard_seed_base(c.rank, c.n, base), c.n, c.F, threads=c.gen_threads)
    c.setup_s = time.time() - t0
    log("rank %d: generated %d streams x %d frames (%.1f MB) on %d threads in %.1fs"
        % (c.rank, c.n, c.F, buf.size / 1e6, c.gen_threads, c.setup_s))
    c.buf, c.offs, c.sizes = buf, offs, sizes
    c.d_in = torch.from_numpy(buf).to(c.dev)
    c.pcm = [torch.empty((c.n, c.F, 2304), dtype=torch.int16, device=c.dev) for _ in range(2 if c.gather else 1)]
    c.infos = torch.zeros((c.n, c.F, 6), dtype=torch.int32, device=c.dev)
    c.dec = mp3_amd.BatchDecoder(c.n, c.F, device=c.gpu)

    def step(k=0):
        c.dec.decode(c.d_in, offs, sizes, c.F, pcm=c.pcm[k % len(c.pcm)], infos=c.infos, stream=c.strm)
    c.step = step
    c.in_bytes = int(sizes.astype(np.int64).sum())
    c.cfg_gen, c.seed_base = cfg, base


def setup_streaming(c, segments):
    """The streaming loop of a server or player: streams
    of segments x F frames, and step k decodes frames [F (k mod segments),
    F (k mod segments) + F) of every stream, so the stream geometry (offsets
    and sizes) handed to mp3d_batch_decode changes on EVERY call; the
    decoder state carries on in HBM (after the last segment the streams run
    on from their first frame, like concatenated files).  Each segment's
    offsets come from the previous call's frame infos in an untimed setup
    pass, exactly as a streaming caller advances them."""
    import torch
    import _gen
    import mp3_amd
    from mp3_amd import shard
    t0 = time.time()
    FF = segments * c.F
    buf, offs, sizes = _gen.batch(c.cfg_gen, shard.shard_seed_base(c.rank, c.n, c.seed_base), c.n, FF,
                                  threads=c.gen_threads)
    d_in = torch.from_numpy(buf).to(c.dev)
    dec = mp3_amd.BatchDecoder(c.n, c.F, device=c.gpu)
    infos = torch.zeros((c.n, c.F, 6), dtype=torch.int32, device=c.dev)
    geo, pos = [], offs.astype(np.uint64).copy()
    end = offs.astype(np.uint64) + sizes.astype(np.uint64)
    for j in range(segments):
        sz = (end - pos).astype(np.uint32)  # the rest of each stream, as a streaming caller hands it over
        dec.decode(d_in, pos, sz, c.F, pcm=c.pcm[0], infos=infos, stream=c.strm)
        used = infos[..., 0].sum(1).cpu().numpy().astype(np.uint64)
        geo.append((pos.copy(), sz))
        pos = pos + used
    dec.reset()
    log("rank %d: streaming set-up (%d streams x %d frames, %d segments) in %.1fs"
        % (c.rank, c.n, FF, segments, time.time() - t0))
    c.stream_buf = (buf, d_in, dec, infos, geo)

    def step(k=0):
        o, z = geo[k % segments]
        dec.decode(d_in, o, z, c.F, pcm=c.pcm[k % len(c.pcm)], infos=infos, stream=c.strm)
    return step


def setup_synth(c):
    import torch
    import _gen
    import mp3_amd
    from mp3_amd import shard
    xr, bt, mx = _gen.c2_spectra(c.n, c.F, 2, seed=shard.shard_seed_base(c.rank, c.n,
                                                                           c.seed if c.seed is not None else 1_000_003 * 2))
    c.xr, c.bt, c.mx = xr, bt, mx
    c.d_xr, c.d_bt, c.d_mx = (torch.from_numpy(a).to(c.dev) for a in (xr, bt, mx))
    c.pcm = [torch.empty((c.n, c.F, 2304), dtype=torch.int16, device=c.dev) for _ in range(2 if c.gather else 1)]
    c.dec = mp3_amd.BatchDecoder(c.n, c.F, device=c.gpu)

    def step(k=0):
        c.dec.synth_only(c.d_xr, c.d_bt, c.d_mx, 2, 44100, pcm=c.pcm[k % len(c.pcm)], stream=c.strm)
    c.step = step


def run_per_frame(args):
    """configs[0]: one stream through the per-frame drop-in call."""
    import _golden
    import mp3_amd
    data, _ = _golden.case("keypress_128k_js")
    # the call through a pointer into the file (no per-call copy of the rest
    # of the buffer, which Python's slicing would add to every call's time)
    L = ctypes.CDLL(str(mp3_amd.LIB_PATH))
    L.mp3d_decode_frame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                    ctypes.POINTER(mp3_amd.FrameInfo)]
    mp3_amd.lib()
    d = mp3_amd.Decoder(device=0)
    data_np = np.frombuffer(data, np.uint8)
    base = data_np.ctypes.data
    pcm = np.zeros(2304, np.int16)
    pcm_p = pcm.ctypes.data
    info = mp3_amd.FrameInfo()
    info_p = ctypes.byref(info)

    def one_pass():
        d.reset()
        pos, nf, lat = 0, 0, []
        while pos < len(data):
            t = time.perf_counter()
            n = L.mp3d_decode_frame(d._h, base + pos, len(data) - pos, pcm_p, info_p)
            lat.append(time.perf_counter() - t)
            if n < 0 or info.frame_bytes <= 0:
                break
            pos += info.frame_bytes
            nf += n > 0
        return nf, lat

    for _ in range(args.warmup):
        one_pass()
    t0 = time.perf_counter()
    frames, lats = 0, []
    for _ in range(args.steps):
        nf, lat = one_pass()
        frames += nf
        lats += lat
    dt = time.perf_counter() - t0
    lat_us = np.array(lats) * 1e6
    # steady state of a long stream (the player's case: the read-ahead's
    # next run decodes behind the served calls): a 512-frame 128 kbps golden
    # stream, one call per frame, every call's latency; the first call of a
    # pass (cold: nothing read ahead yet) reported apart
    long_data, _ = _golden.case("long_c3_512")
    long_np = np.frombuffer(long_data, np.uint8)
    lbase = long_np.ctypes.data
    sl, first = [], []
    for _ in range(max(1, args.steps // 4)):
        d.reset()
        pos, k = 0, 0
        while pos < len(long_data):
            t = time.perf_counter()
            n = L.mp3d_decode_frame(d._h, lbase + pos, len(long_data) - pos, pcm_p, info_p)
            el = time.perf_counter() - t
            if n < 0 or info.frame_bytes <= 0:
                break
            (first if k == 0 else sl).append(el)
            pos += info.frame_bytes
            k += 1
    sl_us, first_us = np.array(sl) * 1e6, np.array(first) * 1e6
    # the same with the calls paced (a busy wait between calls, as a player
    # slower than the GPU's single-stream decode makes them): the next run
    # then completes behind the served calls and no call waits for a refill
    pace_us = 40.0
    pl = []
    d.reset()
    pos, k = 0, 0
    while pos < len(long_data):
        t = time.perf_counter()
        n = L.mp3d_decode_frame(d._h, lbase + pos, len(long_data) - pos, pcm_p, info_p)
        el = time.perf_counter() - t
        if n < 0 or info.frame_bytes <= 0:
            break
        if k:
            pl.append(el)
        pos += info.frame_bytes
        k += 1
        while time.perf_counter() - t < pace_us * 1e-6:
            pass
    pl_us = np.array(pl) * 1e6
    steady = {"stream": "tests/golden/long_c3_512.mp3 (512 frames, 128 kbps 44.1 kHz joint stereo)",
              "calls": int(sl_us.size), "median": float(np.median(sl_us)), "p90": float(np.percentile(sl_us, 90)),
              "p99": float(np.percentile(sl_us, 99)), "max": float(sl_us.max()), "mean": float(sl_us.mean()),
              "first_call_median": float(np.median(first_us)),
              "frames_per_s": float(sl_us.size / (sl_us.sum() * 1e-6)),
              "paced": {"pace_us": pace_us, "calls": int(pl_us.size), "median": float(np.median(pl_us)),
                        "p99": float(np.percentile(pl_us, 99)), "max": float(pl_us.max())}}
    L32, _ = _oracle_libs()
    out = np.zeros((2, 64 * 1152), np.float32)
    nch, hz = ctypes.c_int(), ctypes.c_int()
    t1, f1 = time.perf_counter(), 0
    while time.perf_counter() - t1 < 2.0:
        f1 += L32.orc_decode_stream(data, len(data), out.ctypes.data, 64, ctypes.byref(nch), ctypes.byref(hz))
    cpu = {"value": f1 / (time.perf_counter() - t1), "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": "the same file decoded repeatedly for 2 s by oracle/liboracle_f32.so on one thread",
           "cpu_model": cpu_model()}
    return {"metric": METRIC, "value": frames / dt, "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "tests/golden/keypress_128k_js.mp3",
            "config": {"workload": "C1: one 128 kbps 44.1 kHz joint-stereo stream (21 audio frames + Info frame) "
                                   "through mp3d_decode_frame, host buffers, one call per frame",
                       "streams_per_gpu": 1, "parallelism": "none (per-frame player call)"},
            "latency_us": {"median": float(np.median(lat_us)), "p90": float(np.percentile(lat_us, 90)),
                           "p99": float(np.percentile(lat_us, 99)), "mean": float(lat_us.mean())},
            "steady_latency_us": steady,
            "readahead_frames": int(os.environ.get("MP3D_PF_READAHEAD", 64)),
            "note": "one call per frame as a player's loop makes them, the rest of the file passed each time: the "
                    "decoder reads up to readahead_frames frames ahead in one batch call and serves the next calls "
                    "from it, while the run after it decodes behind them (MP3D_PF_READAHEAD=0: every call decodes "
                    "its own frame).  latency_us: every call of the 22-frame file, each pass from reset, so one "
                    "call in 22 is a cold start; steady_latency_us: a 512-frame stream, its first call apart",
            "roofline": None, "cpu_baseline": cpu}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3, choices=(1, 2, 3, 4, 5),
                    help="BASELINE.json configs[k-1]; 4 = 3 at --gpus 8 (65,536 streams per GPU)")
    ap.add_argument("--streams", type=int, default=None, help="streams per GPU (default: the config's)")
    ap.add_argument("--frames", type=int, default=None, help="frames per stream per step (default: the config's)")
    ap.add_argument("--seed", type=int, default=None,
                    help="generator seed of global stream 0 (stream g uses seed + g; default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="also time an RCCL PCM gather to rank 0 overlapped with the next step (reported apart)")
    ap.add_argument("--gather-priority", default="normal", choices=("high", "normal"),
                    help="stream priority of the process group's collectives (the gather); measured at world 1: "
                         "neither overlaps the decode, whose kernels fill every CU's VGPRs (DESIGN §6)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank path, e.g. several ranks on one GPU)")
    ap.add_argument("--streaming", type=int, default=None, metavar="SEGMENTS",
                    help="also time the streaming loop: streams of SEGMENTS x frames, each step decoding the next "
                         "frames (new offsets every call); reported as `streaming` (default 4 at N = 1, 0 = off)")
    ap.add_argument("--plumbing", action="store_true",
                    help="no GPU: exercise the launcher, rendezvous, sharding, barriers, max-over-ranks timing and "
                         "the gather on CPU tensors (gloo); value is null (tests/test_bench_launch.py)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # stdout carries exactly the one JSON line: anything a library prints
    # there (RCCL's version banner at communicator set-up, ...) goes to stderr
    global _json_out
    _json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.config == 1:
        if args.gpus != 1:
            raise SystemExit("config 1 is a single-stream, single-GPU workload")
        print(json.dumps(run_per_frame(args)), file=_json_out, flush=True)
        return

    import torch
    import torch.distributed as dist
    from mp3_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    c = Ctx()
    c.rank, c.world, c.gather, c.seed = rank, world, args.gather, args.seed
    backend = "gloo" if args.plumbing else args.dist_backend
    if args.plumbing:
        c.dev = torch.device("cpu")
        c.gpu = None
    else:
        # one process per GPU; ranks beyond the visible GPUs (a gloo rehearsal
        # on a one-GPU box) share them round-robin
        c.gpu = local % max(1, torch.cuda.device_count())
        c.dev = torch.device("cuda", c.gpu)
    # --gather at N = 1 still initialises a (one-rank) RCCL group, so the
    # branch an 8-GPU run takes -- init with device_id, the async gather into
    # preallocated receive lists, work.wait() ordering -- executes on one GPU
    use_group = world > 1 or (args.gather and not args.plumbing and backend == "nccl")
    if use_group:
        if backend == "nccl":
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                os.environ["MASTER_PORT"] = str(_free_port())
            os.environ.setdefault("RANK", str(rank))
            os.environ.setdefault("WORLD_SIZE", str(world))
            torch.cuda.set_device(c.gpu)
            # the group's collectives on a high-priority stream (--gather-priority):
            # the gather's RCCL kernels then take a CU as soon as one frees up,
            # instead of queueing behind the decode's workgroups
            opts = None
            if args.gather_priority == "high":
                from torch.distributed import ProcessGroupNCCL
                opts = ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=c.dev, pg_options=opts)
        else:
            if c.gpu is not None:
                torch.cuda.set_device(c.gpu)
            dist.init_process_group(backend)
        # what the initialised group reports, not the environment
        world, backend = dist.get_world_size(), dist.get_backend()
        c.world = world
    cfg = {2: "c2", 3: "c3", 4: "c3", 5: "c5"}[args.config]
    c.n = args.streams or (1024 if cfg == "c2" else 65536)
    c.F = args.frames or (64 if cfg == "c2" else 32)
    c.gen_threads = max(1, min(16, host_threads() // world))
    c.setup_s = 0.0
    if args.gather and use_group:
        # rank 0's receive lists (one per gather in flight) must fit beside
        # the batch buffers; checked at the FULL per-rank size even when
        # --plumbing shrinks the data, against the device's real memory
        dev_bytes = shard.DEVICE_BYTES_DEFAULT
        if c.gpu is not None:
            dev_bytes = torch.cuda.get_device_properties(c.gpu).total_memory
        plan = shard.gather_plan(c.n, c.F, world, device_bytes=dev_bytes, decoder_bytes=decoder_bytes(c.n, c.F))
        if not plan["fits"]:
            raise SystemExit("bench.py: the --gather receive lists need %.1f GB on rank 0, more than %.1f GB"
                             % (plan["need_bytes"] / 1e9, plan["device_bytes"] / 1e9))
        c.gather_plan = plan
    if args.plumbing:
        import _gen
        c.n, c.F = min(c.n, 8), min(c.F, 4)
        t0 = time.time()
        buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(rank, c.n), c.n, c.F, threads=c.gen_threads)
        c.setup_s = time.time() - t0
        c.pcm = [torch.full((c.n, c.F, 2304), rank, dtype=torch.int16) for _ in range(2 if c.gather else 1)]
        c.step = lambda k=0: None
        sync = lambda: None  # noqa: E731
    else:
        c.strm = torch.cuda.current_stream(c.dev).cuda_stream
        if cfg == "c2":
            setup_synth(c)
        else:
            setup_decode(c, cfg)
        sync = lambda: torch.cuda.synchronize(c.dev)  # noqa: E731

    for k in range(args.warmup):
        c.step(k)
    sync()
    frames_per_step = c.n * c.F
    if cfg != "c2" and not args.plumbing:
        inf = c.infos.cpu().numpy()
        frames_per_step = int((inf[..., 5] > 0).sum())
        if cfg == "c3" and frames_per_step != c.n * c.F:
            raise SystemExit("decode produced %d/%d frames" % (frames_per_step, c.n * c.F))

    # --- timed region -------------------------------------------------------
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        c.step(k)
    sync()
    if world > 1:
        dist.barrier()
    dt_rank = time.perf_counter() - t0
    dt = shard.max_over_ranks(dt_rank, c.dev)
    per_rank_dt = shard.all_ranks(dt_rank, c.dev)
    per_rank_frames = shard.all_ranks(float(frames_per_step), c.dev)
    frames_total = sum(per_rank_frames) * args.steps
    value = frames_total / dt
    ms_per_step = dt / args.steps * 1e3

    # --- per-kernel device time (HIP events on the decode stream) ---------
    kt = {"demux": 0.0, "huffman": 0.0, "synth": 0.0}
    if not args.plumbing:
        c.dec.set_timing(True)
        # the median of the timed calls: C2's calls are ~0.3 ms, and single
        # ones ran up to 35 % long (clock ramp after the host-side gaps)
        reps = max(1, min(9 if cfg == "c2" else 3, args.steps))
        samples = {key: [] for key in kt}
        for k in range(reps):
            c.step(k)
            for key, v in c.dec.kernel_times_us().items():
                samples[key].append(v)
        kt = {key: float(np.median(v)) if v else 0.0 for key, v in samples.items()}
        c.kt_reps = reps
        c.dec.set_timing(False)
        sync()

    # --- streaming loop: new stream geometry on every call ----------------
    streaming = None
    segs = args.streaming if args.streaming is not None else (4 if world == 1 else 0)
    if segs > 0 and cfg != "c2" and not args.plumbing:
        sstep = setup_streaming(c, segs)
        for k in range(args.warmup):
            sstep(k)
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for k in range(args.steps):
            sstep(k)
        sync()
        if world > 1:
            dist.barrier()
        sdt = shard.max_over_ranks(time.perf_counter() - t0, c.dev)
        # the streaming loop's own output: every segment of the last `segs`
        # steps must have decoded all its frames (a geometry-staging bug that
        # drops frames would otherwise still report full throughput)
        sinf = c.stream_buf[3]
        sframes = int((sinf[..., 5] > 0).sum())
        if cfg == "c3" and sframes != c.n * c.F:
            raise SystemExit("streaming decode produced %d/%d frames" % (sframes, c.n * c.F))
        sval = sum(per_rank_frames) * args.steps / sdt
        streaming = {"value": sval, "ms_per_step": sdt / args.steps * 1e3, "segments": segs,
                     "vs_fixed_offsets": sval / value,
                     "note": "streams of %d x %d frames; step k decodes frames [%d (k mod %d), +%d) of every stream, "
                             "so offsets and sizes change on every mp3d_batch_decode call (async geometry staging)"
                             % (segs, c.F, c.F, segs, c.F)}
        c.stream_buf = None

    # --- optional RCCL PCM gather, overlapped with the next step ----------
    gather = None
    if args.gather and use_group:
        c.ms_decode = ms_per_step
        gather = time_gather(c, args, dist, shard, torch, sync)

    setup_all = shard.all_ranks(c.setup_s, c.dev)  # collective: every rank takes part
    if rank != 0:
        if use_group:
            dist.destroy_process_group()
        return
    res = {"metric": METRIC, "value": None if args.plumbing else value, "unit": "frames/s", "n_gpus": world,
           "ranks": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "per_rank_frames_per_s": [f * args.steps / t for f, t in zip(per_rank_frames, per_rank_dt)],
           "dist_backend": backend if use_group else None,
           "setup_s_per_rank": setup_all, "gen_threads_per_rank": c.gen_threads}
    if args.plumbing:
        res.update(plumbing_only=True, data="synthetic C3 shard per rank (generated, not decoded)",
                   config={"workload": "plumbing rehearsal: %d ranks x %d streams x %d frames" % (world, c.n, c.F),
                           "streams_per_gpu": c.n, "frames_per_stream": c.F,
                           "first_stream_seed_per_rank": [shard.shard_seed_base(r, c.n) for r in range(world)]})
    elif cfg == "c2":
        res.update(report_c2(c, args, value, kt))
    else:
        res.update(report_decode(c, args, cfg, value, kt, frames_per_step))
    if gather:
        res["gather"] = gather
    if streaming:
        res["streaming"] = streaming
    print(json.dumps(res), file=_json_out, flush=True)
    if use_group:
        dist.destroy_process_group()


def time_gather(c, args, dist, shard, torch, sync):
    """Second timed loop: step k's PCM gathered to rank 0 while step k+1
    decodes (RCCL runs the gather on the process group's stream; the decode
    of step k+2 waits for the gather that read its PCM buffer).  gloo gathers
    host tensors synchronously, so that rehearsal shows no overlap."""
    nbytes = c.pcm[0].numel() * c.pcm[0].element_size()
    # one receive list per gather in flight: the two overlapped gathers never
    # write the same buffers (a real pipelined consumer reads slot b while
    # the other fills)
    recv = [None, None]
    if c.rank == 0 and dist.get_backend() != "gloo":
        recv = [[torch.empty_like(c.pcm[0]) for _ in range(c.world)] for _ in range(2)]
    # gather alone (no decode beside it)
    dist.barrier()
    sync()
    tg = time.perf_counter()
    shard.gather_to_root(c.pcm[0], out=recv[0])
    sync()
    alone = shard.max_over_ranks(time.perf_counter() - tg, c.dev)
    pending = [None, None]
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        b = k % 2
        if pending[b] is not None:
            pending[b].wait()  # decode k overwrites the buffer gather k-2 reads
            pending[b] = None
        c.step(k)
        if dist.get_backend() == "gloo":
            sync()
            shard.gather_to_root(c.pcm[b])
        else:
            _, pending[b] = shard.gather_to_root(c.pcm[b], async_op=True, out=recv[b])
    for w in pending:
        if w is not None:
            w.wait()
    sync()
    dist.barrier()
    dt = shard.max_over_ranks(time.perf_counter() - t0, c.dev)
    # rank 0's xGMI ingress bounds the gather at world > 1: it receives the
    # world - 1 other shards over its 7 links.  XGMI_INGRESS is the nominal
    # 7 x 153.6 GB/s; if that figure counts both directions, the
    # one-way ingress and this bound are half of it
    xgmi_bytes = nbytes * (c.world - 1)
    bound = c.n * c.F * c.world / (xgmi_bytes / XGMI_INGRESS) if xgmi_bytes else None
    return {"ms_alone": alone * 1e3, "bytes_per_step": nbytes * c.world, "xgmi_bytes_per_step": xgmi_bytes,
            "xgmi_ingress_bound_frames_per_s": bound, "xgmi_ingress_assumed_bytes_per_s": XGMI_INGRESS,
            "priority": args.gather_priority,
            "ms_per_step_decode_plus_gather": dt / args.steps * 1e3,
            # the share of the gather hidden behind the decode: (decode + gather
            # alone - both overlapped) / gather alone
            "hidden_fraction": (c.ms_decode + alone * 1e3 - dt / args.steps * 1e3) / (alone * 1e3) if alone > 0 else None,
            "frames_per_s_with_gather": c.n * c.F * c.world * args.steps / dt,
            "overlapped": dist.get_backend() != "gloo",
            "world": c.world, "backend": dist.get_backend(),
            "self_gather_only": c.world == 1,
            "rank0_memory_plan": getattr(c, "gather_plan", None),
            "note": "PCM of step k gathered to rank 0 over RCCL (xGMI) on the process group's stream while step "
                    "k+1 decodes; reported apart from `value`" + (
                        "; world 1: a one-rank RCCL group gathers rank 0's PCM to itself (device copy, no xGMI), "
                        "which runs the same init / async gather / wait code an 8-GPU run takes" if c.world == 1
                        else "")}


XGMI_INGRESS = 7 * 153.6e9  # bytes/s into one MI355X over its 7 xGMI links (nominal)


def decoder_bytes(n, F):
    """Device bytes of one BatchDecoder(n, F) plus its resident input (C3
    sizes): state, frame records, side words, is[] rows, unit meta, infos,
    md region and the input frames."""
    units = n * F * 4
    return int(n * 8832 + n * F * (32 + 24 + 418 + 400) + units * (8 + 1152 + 224))


def load_pmc(key, n, F):
    prof = ROOT / "profiles" / "pmc_traffic.json"
    if not prof.exists():
        return {}
    try:
        pj = json.loads(prof.read_text())
    except ValueError:
        return {}
    ent = pj.get(key, pj if key == "c3" else {})
    if ent.get("streams") == n and ent.get("frames") == F:
        return ent
    return {}


def report_decode(c, args, cfg, value, kt, frames_per_step):
    n, F, world = c.n, c.F, c.world
    synth_s = kt["synth"] * 1e-6
    frames_per_launch = n * F
    achieved_tf = FLOP_PER_FRAME * frames_per_launch / synth_s / 1e12 if synth_s > 0 else 0.0
    pmc = load_pmc(cfg, n, F)
    in_per_frame = c.in_bytes / max(1, frames_per_step)
    if cfg == "c3":
        if world == 8 and n == 65536:
            wl = "C4: 524,288 concurrent streams sharded across 8 GPUs (65,536 x 32 frames per GPU per step)"
        else:
            wl = "C3: full Layer III decode (Huffman->PCM), %d streams x %d frames per GPU per step" % (n, F)
        data = "synthetic (seeded generator: valid CBR 128 kbps 44.1 kHz joint-stereo MP3 frames)"
    else:
        wl = "C5: mixed corpus (VBR 32-320 kbps, mono/stereo/MS/IS, 32/44.1/48 kHz, short+mixed blocks, CRC), " \
             "%d streams x %d frames per GPU per step" % (n, F)
        data = "synthetic (seeded generator: mixed-corpus MP3 streams)"
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline_decode(c.buf, c.offs, c.sizes, F)
    dom = max(kt, key=kt.get)
    return {
        "data": data,
        "config": {"workload": wl, "streams_per_gpu": n, "frames_per_stream": F, "bitrate_kbps": 128 if cfg == "c3"
                   else "32-320 VBR", "hz": 44100 if cfg == "c3" else "32000/44100/48000",
                   "seed": c.seed if c.seed is not None else "default",
                   "parallelism": "streams sharded, 1 process per GPU, no data-path collective"},
        "roofline": {
            "kernel": "k_synth", "bound": "mfma", "roofline_class": "FP32 compute", "unit": "TFLOP/s",
            "bound_detail": "compute roofline at the dense FP32 peak (MFMA rate = vector rate); the kernel's limiter is "
                            "VALU issue and dependent-chain latency (see limiter)",
            "achieved": achieved_tf, "peak": FP32_PEAK_TFLOPS, "frac": achieved_tf / FP32_PEAK_TFLOPS,
            "traffic": pmc.get("k_synth_hbm_bytes_per_launch"),
            "limiter": "FP32 compute roofline (vector rate = matrix rate, 157.3 TF); the PMC counters "
                       "(profiles/) show k_synth limited by VALU issue and dependent-chain latency, not by the "
                       "matrix cores (see mfma_util_pmc)",
            "flop_per_frame": FLOP_PER_FRAME, "frames_per_launch": frames_per_launch, "launch_us": kt["synth"],
            "clock_mhz_pmc": pmc.get("k_synth_clock_mhz"),
            "frac_at_clock": (achieved_tf / (FP32_PEAK_TFLOPS * pmc["k_synth_clock_mhz"] / 2400.0)
                              if pmc.get("k_synth_clock_mhz") else None),
            "clock_note": "k_synth's mean engine clock in the committed PMC profile (GRBM_GUI_ACTIVE / 8 XCDs / "
                          "duration, profiles/pmc_traffic.json): power-limited below the 2400 MHz the peak assumes; "
                          "frac_at_clock = achieved / the FP32 peak at that clock",
            "executed_flop_per_frame": EXEC_FLOP_PER_FRAME,
            "executed_frac": EXEC_FLOP_PER_FRAME * frames_per_launch / synth_s / 1e12 / FP32_PEAK_TFLOPS
            if synth_s else 0,
            "dct_tile": {
                "mfma_flop_per_frame": MFMA_FLOP_PER_FRAME,
                "mfma_tflops": MFMA_FLOP_PER_FRAME * frames_per_launch / synth_s / 1e12 if synth_s else 0,
                "mfma_util_pmc": pmc.get("k_synth_mfma_util"),
                "note": "matrix-core busy fraction of k_synth from rocprofv3 (SQ_VALU_MFMA_BUSY_CYCLES, "
                        "profiles/pmc_traffic.json); peak 157.3 TFLOP/s FP32 MFMA"},
        },
        "hbm": {
            "hbm_rw_frac": value / world * (in_per_frame + PCM_BYTES_PER_FRAME) / (HBM_PEAK_GBS * 1e9),
            "hbm_read_frac": value / world * in_per_frame / (HBM_PEAK_GBS * 1e9),
            "bytes_per_frame_rw": in_per_frame + PCM_BYTES_PER_FRAME,
            "step_traffic_pmc": pmc.get("step_hbm_bytes"),
        },
        "kernel_us": kt,
        "kernel_us_stat": "median over %d HIP-event-timed calls after the timed loop" % getattr(c, "kt_reps", 0),
        "dominant_kernel": "k_" + dom,
        "cpu_baseline": cpu,
    }


def report_c2(c, args, value, kt):
    n, F, world = c.n, c.F, c.world
    synth_s = kt["synth"] * 1e-6
    fpl = n * F
    achieved_tf = C2_FLOP_PER_FRAME * fpl / synth_s / 1e12 if synth_s > 0 else 0.0
    gbs = C2_BYTES_PER_FRAME * fpl / synth_s / 1e9 if synth_s > 0 else 0.0
    pmc = load_pmc("c2", n, F)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline_synth(c.xr, c.bt, c.mx, 2)
    return {
        "data": "synthetic spectra (SURVEY.md §8(d) C2: N(0, sigma_k^2) with spectral tilt, start/short/stop runs, "
                "mixed blocks)",
        "config": {"workload": "C2: IMDCT + polyphase synthesis only (mp3d_batch_synth_only), %d streams x %d "
                               "frames per GPU per step" % (n, F),
                   "streams_per_gpu": n, "frames_per_stream": F, "hz": 44100,
                   "seed": c.seed if c.seed is not None else "default",
                   "parallelism": "streams sharded, 1 process per GPU, no data-path collective"},
        "roofline": {
            "kernel": "k_synth<xr>", "bound": "mfma", "roofline_class": "FP32 compute",
            "bound_detail": "compute roofline at the dense FP32 peak (MFMA rate = vector rate); VALU-issue limited",
            "unit": "TFLOP/s", "achieved": achieved_tf,
            "peak": FP32_PEAK_TFLOPS, "frac": achieved_tf / FP32_PEAK_TFLOPS,
            "traffic": pmc.get("k_synth_hbm_bytes_per_launch"),
            "flop_per_frame": C2_FLOP_PER_FRAME, "frames_per_launch": fpl, "launch_us": kt["synth"],
            "clock_mhz_pmc": pmc.get("k_synth_clock_mhz"),
            "frac_at_clock": (achieved_tf / (FP32_PEAK_TFLOPS * pmc["k_synth_clock_mhz"] / 2400.0)
                              if pmc.get("k_synth_clock_mhz") else None),
            "hbm_GBs_algorithmic": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
            "bytes_per_frame": C2_BYTES_PER_FRAME,
            "limiter": "22 FLOP/B against a machine balance of 19.7: both rooflines are reported"},
        "kernel_us": kt,
        "kernel_us_stat": "median over %d HIP-event-timed calls after the timed loop" % getattr(c, "kt_reps", 0),
        "dominant_kernel": "k_synth",
        "cpu_baseline": cpu,
    }


if __name__ == "__main__":
    main()
