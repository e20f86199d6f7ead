"""Stream sharding across ranks.

Streams are independent, so rank r of W owns the contiguous global stream ids
[r*n, (r+1)*n) and decodes them with no data-path collective (weak scaling:
per-GPU work is fixed as W grows).  Synthetic inputs are seeded by global
stream id, so a stream's bytes do not depend on W.  The optional PCM gather
to rank 0 is a plain torch.distributed gather -- RCCL over xGMI with the
"nccl" backend on MI355X, gloo on CPU -- and is timed apart from decode.
"""
import torch
import torch.distributed as dist

BASE_SEED_C3 = 3_000_003  # global stream g of the C3 workload uses seed BASE_SEED_C3 + g


def shard_range(rank: int, n_per_rank: int):
    """(first global stream id, count) owned by `rank`."""
    return rank * n_per_rank, n_per_rank


def shard_seed_base(rank: int, n_per_rank: int, base: int = BASE_SEED_C3) -> int:
    """Seed of the rank's first stream (the generator adds the local index)."""
    first, _ = shard_range(rank, n_per_rank)
    return base + first


def max_over_ranks(seconds: float, device=None) -> float:
    """Job time = the slowest rank's time (identity when not distributed)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    if dist.get_backend() == "gloo":
        device = "cpu"  # gloo reduces host tensors
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks(value: float, device=None) -> list:
    """Every rank's `value` (rank order), on every rank ([value] when not
    distributed) -- bench.py's per-rank frames/s."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [value]
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def gather_to_root(t: torch.Tensor, root: int = 0, async_op: bool = False, out=None):
    """Gather every rank's equally-shaped tensor to `root` (list there, None
    elsewhere).  gloo has no 8/16-bit gather, so such tensors travel as int32
    words there (PCM rows are 2304 int16 = 1152 words).  async_op=True
    (RCCL): returns (list or None, work handle); the gather runs on the
    process group's own stream after the work queued so far on the current
    stream, and work.wait() makes the current stream wait for it.  out:
    preallocated receive list on root (reused across steps), else allocated."""
    world, rank = dist.get_world_size(), dist.get_rank()
    src = t.contiguous()
    gloo = dist.get_backend() == "gloo"
    if gloo:
        src = src.cpu()  # gloo gathers host tensors
    # wire type: RCCL / NCCL has no int16 ("Unconvertible NCCL type Short"),
    # so PCM travels as bytes there (bit-exact, the receive buffers viewed
    # the same way); gloo has no 8/16-bit gather: int32 words
    wire = None
    if src.dtype in (torch.int16, torch.uint8, torch.int8):
        wire = torch.int32 if gloo else (torch.uint8 if src.dtype == torch.int16 else None)
    if wire is not None:
        src = src.view(wire)
    if rank != root:
        out = None
    elif out is None or gloo:
        out = [torch.empty_like(src) for _ in range(world)]
    else:  # preallocated receive list (device): gather straight into it
        out = [o.view(src.dtype) for o in out]
    work = dist.gather(src, out, dst=root, async_op=async_op)
    if out is not None:
        out = [o.view(t.dtype) for o in out]
    return (out, work) if async_op else out


PCM_ROW_BYTES = 2304 * 2  # one int16 stereo frame
DEVICE_BYTES_DEFAULT = 288 << 30  # MI355X HBM3E; bench.py passes the device's real total


def gather_plan(n_per_rank: int, frames: int, world: int, in_flight: int = 2, device_bytes: int = DEVICE_BYTES_DEFAULT,
                decoder_bytes: int = 0):
    """Device memory rank 0 needs for the overlapped PCM gather (bench.py
    --gather): `in_flight` receive lists of `world` PCM shards each (one list
    per gather in flight, so two overlapped gathers never write the same
    buffers), next to its own double-buffered PCM and the decoder's buffers.
    Returns a dict with the byte counts and whether it fits; at C4 (65 536 x
    32 per rank, 8 ranks) the receive lists are 2 x 8 x 9.66 GB."""
    shard_bytes = n_per_rank * frames * PCM_ROW_BYTES
    recv = in_flight * world * shard_bytes
    own = 2 * shard_bytes
    need = recv + own + decoder_bytes
    return {"shard_bytes": shard_bytes, "recv_bytes": recv, "own_pcm_bytes": own, "decoder_bytes": decoder_bytes,
            "need_bytes": need, "device_bytes": device_bytes, "fits": need <= device_bytes}
