"""GPU: the RCCL branch an 8-GPU C4 run takes, executed on one MI355X
(VERDICT r03 item 1).

A FRESH child process (never a fork or exec of this GPU-initialised test
process) runs as a one-rank group, exactly the way bench.py's ranks do:

- torch.cuda.set_device + dist.init_process_group("nccl", device_id=...);
- decodes the rank-7 shard of C4 at full size (global stream ids
  7*65536 .. 8*65536-1, 32 frames each, shard.shard_seed_base(7, 65536));
- gathers its PCM to rank 0 with shard.gather_to_root(async_op=True,
  out=<preallocated receive list>) while the next step decodes, with the
  double-buffered pending[b].wait() ordering of bench.time_gather;
- checks every gathered shard bit-identical to the local PCM, and records
  the backend and world size the initialised group reports.

The parent then holds the child's stride-256 stream sample against the
oracle (within 1 LSB) and checks the size-independent properties of
test_gpu_scale.test_c3_full_size_properties: every frame decoded, and the
repeat decode after reset identical to the first.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd
from mp3_amd import shard

pytestmark = pytest.mark.gpu

N, F, RANK7 = 65536, 32, 7
STRIDE = N // 256

CHILD = r"""
import json, os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.environ["REPO"] + "/tests")
import _gen, mp3_amd
from mp3_amd import shard
n, F, stride = int(os.environ["N"]), int(os.environ["F"]), int(os.environ["STRIDE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
rec = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "rank": dist.get_rank()}
buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(int(os.environ["SHARD"]), n), n, F, threads=16)
d_in = torch.from_numpy(buf).to(dev)
strm = torch.cuda.current_stream(dev).cuda_stream
dec = mp3_amd.BatchDecoder(n, F, device=0)
pcm = [torch.empty((n, F, 2304), dtype=torch.int16, device=dev) for _ in range(2)]
infos = torch.zeros((n, F, 6), dtype=torch.int32, device=dev)
recv = [[torch.empty_like(pcm[0]) for _ in range(dist.get_world_size())] for _ in range(2)]
pending, first = [None, None], None
for k in range(3):
    b = k % 2
    if pending[b] is not None:
        pending[b].wait()          # decode k overwrites the buffer gather k-2 reads
        pending[b] = None
    if k == 2:
        dec.reset()                # step 2 repeats step 0 from fresh state
    dec.decode(d_in, offs, sizes, F, pcm=pcm[b], infos=infos, stream=strm)
    if k == 0:
        rec["frames_decoded"] = int((infos[..., 5] == 1152).sum())
        first = pcm[0][::stride].cpu()
        inf0 = infos[::stride].cpu()
    out, pending[b] = shard.gather_to_root(pcm[b], async_op=True, out=recv[b])
    rec.setdefault("out_is_prealloc", []).append(all(o.data_ptr() == r.data_ptr() for o, r in zip(out, recv[b])))
for w in pending:
    if w is not None:
        w.wait()
torch.cuda.synchronize()
rec["gather_equal"] = [bool(torch.equal(recv[b][0], pcm[b])) for b in range(2)]
rec["repeat_equal"] = bool(torch.equal(pcm[0][::stride].cpu(), first))
np.save(os.environ["OUT"] + ".pcm.npy", first.numpy())
np.save(os.environ["OUT"] + ".inf.npy", inf0.numpy())
json.dump(rec, open(os.environ["OUT"] + ".json", "w"))
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_one_rank_gather_and_rank7_shard(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    out = str(tmp_path / "r")
    repo = _golden.GOLDEN.parents[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), REPO=str(repo), N=str(N), F=str(F),
               STRIDE=str(STRIDE), SHARD=str(RANK7), OUT=out)
    p = subprocess.run([sys.executable, "-u", str(script)], env=env, timeout=240)
    assert p.returncode == 0
    rec = json.load(open(out + ".json"))
    # what the initialised group reports (the record goes to gpurun_out/ too)
    rec_dir = repo / "gpurun_out"
    rec_dir.mkdir(exist_ok=True)
    (rec_dir / "rccl_branch.json").write_text(json.dumps(rec))
    assert rec["backend"] == "nccl" and rec["world_size"] == 1 and rec["rank"] == 0, rec
    assert rec["out_is_prealloc"] == [True, True, True], rec
    assert rec["gather_equal"] == [True, True], rec
    assert rec["repeat_equal"], rec
    assert rec["frames_decoded"] == N * F, rec
    # the stride-256 sample of the rank-7 shard against the oracle (1 LSB)
    pcm = np.load(out + ".pcm.npy")
    inf = np.load(out + ".inf.npy").reshape(-1).view(mp3_amd.FRAME_INFO_DT).reshape(len(pcm), F)
    base = shard.shard_seed_base(RANK7, N)
    worst = 0
    for i, s in enumerate(range(0, N, STRIDE)):
        data, _ = _gen.stream(_gen.C3, base + s, F)
        o = _golden.to_int16(_oracle.decode_stream(data)[0])
        g = mp3_amd.pcm_to_planar(pcm[i], inf[i])
        assert g.shape == o.shape, (s, g.shape, o.shape)
        worst = max(worst, int(np.abs(g.astype(np.int32) - o.astype(np.int32)).max()))
    assert worst <= 1, worst
