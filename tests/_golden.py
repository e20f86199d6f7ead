"""Access to the committed golden fixtures (tests/golden/)."""
import json
import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def manifest():
    return json.loads((GOLDEN / "manifest.json").read_text())


def case(name):
    data = (GOLDEN / (name + ".mp3")).read_bytes()
    pcm = np.load(GOLDEN / (name + ".pcm16.npy"))
    return data, pcm


def names():
    return sorted(manifest().keys())


def to_int16(x):
    """clamp(floor(x 32768 + 0.5)): the decoder's int16 rounding (k_synth's
    v_cvt_rpi_i32_f32; FFmpeg's fixed-point round_sample adds half and shifts)."""
    return np.clip(np.floor(np.asarray(x, np.float64) * 32768.0 + 0.5), -32768, 32767).astype(np.int16)


def compare(name, ours, ref):
    """Max |ours - ref| in LSB over the frames both decoders emitted, after
    checking our frame count (edge cases: tests/golden/manifest.json notes)."""
    import numpy as np
    meta = manifest()[name]
    spf = meta.get("spf", 1152)  # samples per frame: 576 for MPEG-2 / 2.5 LSF
    want = meta.get("our_frames") or ref.shape[1] // spf
    assert ours.shape[1] == want * spf, (name, ours.shape, want)
    k = min(ours.shape[1], ref.shape[1])
    d = np.abs(ours[:, :k].astype(np.int32) - ref[:, :k].astype(np.int32))
    return int(d.max()), float((d == 0).mean())
