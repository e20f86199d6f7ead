"""StreamState blob helpers for the GPU tests."""
import numpy as np

import mp3_amd


def state_view(blobs):
    """The meaningful part of StreamState blobs (mp3d_internal.h): the
    reservoir carry up to res_len (bytes past it are stale), res_len, frames,
    tag, kind, format stamp, IMDCT overlap and synthesis history (partial
    window sums in float-sink units, ABI v5)."""
    sb = mp3_amd.state_bytes()
    dt = np.dtype([("res", np.uint8, 512), ("res_len", np.int32), ("frames", np.int32), ("tag_info", np.uint32),
                   ("tag_frames", np.uint32), ("kind", np.int32), ("pad", np.int32, 2), ("fmt", np.uint32),
                   ("overlap", np.float32, (2, 32, 18)), ("fifo", np.float32, (2, 15, 32))])
    assert dt.itemsize == sb, (dt.itemsize, sb)
    v = np.ascontiguousarray(blobs).reshape(-1).view(dt).copy()
    for r in v:
        r["res"][r["res_len"]:] = 0
    v["pad"] = 0
    return v
