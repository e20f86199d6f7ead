"""bench.py's multi-rank path without a GPU: `--gpus 2` (no WORLD_SIZE in the
environment) must start the two rank processes itself, rendezvous over gloo
on 127.0.0.1, shard the synthetic streams by global id, time with barriers
and max-over-ranks, run the PCM gather, and relay rank 0's single JSON line
(VERDICT r01 "Next round" item 1).  --plumbing replaces the decode step by a
no-op, so value is null: this checks the launcher and the reporting only."""
import json
import os
import pathlib
import subprocess
import sys

from mp3_amd import shard

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--plumbing", "--steps", "2", "--warmup", "1"]
                       + list(extra), env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    r = _run("--gpus", "2", "--gather", "--dist-backend", "gloo")
    assert r["n_gpus"] == 2 and r["ranks"] == 2
    assert r["plumbing_only"] is True and r["value"] is None
    assert len(r["per_rank_frames_per_s"]) == 2
    n = r["config"]["streams_per_gpu"]
    assert r["config"]["first_stream_seed_per_rank"] == [shard.shard_seed_base(k, n) for k in range(2)]
    g = r["gather"]
    assert g["bytes_per_step"] == 2 * n * r["config"]["frames_per_stream"] * 2304 * 2


def test_bench_single_rank_no_spawn():
    r = _run("--gpus", "1")
    assert r["n_gpus"] == 1 and r["ranks"] == 1 and r["dist_backend"] is None


def test_bench_rank_failure_propagates():
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    env["WORLD_SIZE"] = "3"  # torchrun-style single rank whose world disagrees with --gpus
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--plumbing", "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_bench_eight_ranks_gather_plan():
    """C4's launch shape (8 ranks) through the launcher with the gather:
    the line carries the rank count and backend the initialised process
    group reports, per-rank setup times and generator threads (the host's
    threads split over the ranks), and rank 0's receive-list plan, checked
    at the FULL C4 shard size: one receive list per gather in flight, 2 x 8 x
    9.66 GB, beside rank 0's own PCM and decoder buffers within 288 GB."""
    r = _run("--gpus", "8", "--gather", "--dist-backend", "gloo")
    assert r["n_gpus"] == 8 and r["ranks"] == 8 and r["dist_backend"] == "gloo"
    assert len(r["per_rank_frames_per_s"]) == 8 and len(r["setup_s_per_rank"]) == 8
    assert r["gen_threads_per_rank"] >= 1
    plan = r["gather"]["rank0_memory_plan"]
    shard_bytes = 65536 * 32 * 2304 * 2
    assert plan["shard_bytes"] == shard_bytes and plan["recv_bytes"] == 2 * 8 * shard_bytes
    assert plan["fits"] and plan["need_bytes"] <= 288 << 30
    assert plan["decoder_bytes"] > 5e9  # the batch buffers are counted


def test_gather_plan_rejects_oversize():
    p = shard.gather_plan(65536 * 4, 32, 8)
    assert not p["fits"]
