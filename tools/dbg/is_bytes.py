#!/usr/bin/env python3
"""k_huffman's algorithmic bytes per unit at C3 (GPU box): the Huffman tap
decodes a sample of the bench's C3 streams; per unit, the is[] prefix the
kernel stores (8-line groups through the last nonzero line, a lower bound
of nz_end's), the md bytes it reads (part2_3_length / 8) and the 224-B
UnitMeta.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gen  # noqa: E402
import mp3_amd  # noqa: E402
from mp3_amd import shard  # noqa: E402

n, F = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 32
buf, offs, sizes = _gen.batch(_gen.C3, shard.shard_seed_base(0, 65536, shard.BASE_SEED_C3), n, F, threads=16)
dec = mp3_amd.BatchDecoder(n, F)
is_out, _ = dec.huffman_only(buf, offs, sizes, F)
rows = is_out.reshape(-1, 576)
nz = rows != 0
last = np.where(nz.any(axis=1), 575 - np.argmax(nz[:, ::-1], axis=1), -1)
groups = (last + 8) // 8  # 8-line (16-B) groups through the last nonzero line
is_bytes = 16.0 * groups.mean()
frame_bytes = float(np.mean(sizes)) / F
print(json.dumps({"streams": n, "frames": F, "units": int(rows.shape[0]), "is_prefix_bytes_per_unit": is_bytes,
                  "mean_last_nonzero_line": float(last.mean()), "input_bytes_per_frame": frame_bytes,
                  "meta_bytes_per_unit": 56}))
