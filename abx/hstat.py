#!/usr/bin/env python3
"""k_huffman's read account: decode the C3 batch once
with the HSTAT build (MP3D_LIB=build_ab/HSTAT.so, abx/variants.py) and print
the staged main-data bytes, the distinct 128-B lines they span and the
per-unit record reads, as one JSON line, next to which profiles/*_pmc.json's
FETCH_SIZE is read."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import _gen  # noqa: E402
import mp3_amd  # noqa: E402
from mp3_amd import shard  # noqa: E402


def main():
    n, F = 65536, 32
    buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(0, n, shard.BASE_SEED_C3), n, F, threads=16)
    d_in = torch.from_numpy(buf).cuda()
    pcm = torch.empty((n, F, 2304), dtype=torch.int16, device="cuda")
    dec = mp3_amd.BatchDecoder(n, F)
    L = mp3_amd.lib()
    out = (ctypes.c_ulonglong * 8)()
    res = []
    for rep in range(2):
        dec.reset()
        dec.decode(d_in, offs, sizes, F, pcm=pcm)
        torch.cuda.synchronize()
        assert L.mp3d_dbg_hstat(out) == 0
        res.append([int(x) for x in out])
    staged, lines, units, stored, batches, rounds, spill, _ = res[-1]
    frames = n * F
    print(json.dumps({
        "probe": "k_huffman read account (HSTAT build)", "streams": n, "frames": frames,
        "decoded_units": units, "staged_bytes": staged, "staged_bytes_per_unit": staged / max(1, units),
        "staged_lines_128B": lines, "staged_line_bytes": 128 * lines,
        "store_bytes": stored, "store_bytes_note": "HSTAT2 builds only: bytes k_huffman's store instructions carry "
        "(big_values groups incl. the dead zero groups of lanes past their big_values, count1, UnitMeta); 0 with HSTAT",
        "staging_batches": batches, "rounds": rounds, "batches_per_round": batches / max(1, rounds),
        "lanes_past_first_batch": spill, "note_batches": "HSTAT3 builds only (0 otherwise)",
        "records_bytes": frames * (32 + 32) + n * 8 + 4 * frames * 4,
        "note": "records = FrameRec 32 B + side words 32 B per frame, md offset 8 B per stream, rank 4 B per unit",
        "input_payload_bytes": int(sizes.astype("int64").sum())}))


if __name__ == "__main__":
    main()
