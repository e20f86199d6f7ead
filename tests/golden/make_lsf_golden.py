"""MPEG-2 / MPEG-2.5 LSF golden fixtures (run in the build container only,
like make_golden.py): generated Layer III streams at the six low sampling
frequencies, decoded by FFmpeg (Chromium 88 WebAudio, ffmpeg_oracle.py) and
committed as int16 PCM next to the stream bytes.  Adds its cases to
manifest.json without touching the others.

  lsf_22k_js        22.05 kHz joint stereo (M/S and intensity per frame),
                    short + mixed blocks, VBR 8..160 kbps
  lsf_24k_is        24 kHz intensity stereo only (LSF is_pos tables)
  lsf_16k_mono_crc  16 kHz mono with CRC
  lsf_11k_ms_is     11.025 kHz (MPEG-2.5) M/S + intensity
  lsf_12k_stereo    12 kHz (MPEG-2.5) plain stereo, 64 kbps CBR
  lsf_8k_js         8 kHz (MPEG-2.5) joint stereo, short + mixed blocks
                    (FFmpeg's 8 kHz band tables and region sizes)
  lsf_rand          random LSF rate / mode

At scale (the 16-frame cases pin the LSF reservoir,
intensity and FIFO carry only briefly), 256 frames per class:

  lsf_scale_22k_js    22.05 kHz joint stereo (M/S and intensity per frame),
                      short + mixed blocks, VBR
  lsf_scale_24k_is    24 kHz intensity stereo only
  lsf_scale_16k_mono  16 kHz mono, CRC on half the frames
  lsf_scale_11k_msis  11.025 kHz (MPEG-2.5) M/S + intensity
  lsf_scale_8k_js     8 kHz (MPEG-2.5) joint stereo, short + mixed blocks

Usage:  python tests/golden/make_lsf_golden.py [--scale]   (--scale: only
the 256-frame classes; the 16-frame ones are left as committed)
"""
import json
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))
import ffmpeg_oracle  # noqa: E402
import _gen  # noqa: E402
from make_golden import record_hashes, to_int16  # noqa: E402

HZ = [44100, 48000, 32000, 22050, 24000, 16000, 11025, 12000, 8000]
N_FRAMES = 16
CASES = {
    "lsf_22k_js": dict(sr_idx=3, mode=1, mode_ext=-1, short_pct=30, mixed_pct=40),
    "lsf_24k_is": dict(sr_idx=4, mode=1, mode_ext=1, short_pct=20, mixed_pct=30),
    "lsf_16k_mono_crc": dict(sr_idx=5, mode=3, short_pct=25, mixed_pct=30, crc_pct=100),
    "lsf_11k_ms_is": dict(sr_idx=6, mode=1, mode_ext=3, short_pct=25, mixed_pct=30),
    "lsf_12k_stereo": dict(sr_idx=7, mode=0, short_pct=20, mixed_pct=0, bitrate_idx=8),
    "lsf_8k_js": dict(sr_idx=8, mode=1, mode_ext=-1, short_pct=30, mixed_pct=40),
    "lsf_rand": dict(sr_idx=-2),
}
SCALE_FRAMES = 256
SCALE_CASES = {
    "lsf_scale_22k_js": dict(sr_idx=3, mode=1, mode_ext=-1, short_pct=25, mixed_pct=30),
    "lsf_scale_24k_is": dict(sr_idx=4, mode=1, mode_ext=1, short_pct=20, mixed_pct=25),
    "lsf_scale_16k_mono": dict(sr_idx=5, mode=3, short_pct=20, mixed_pct=25, crc_pct=50),
    "lsf_scale_11k_msis": dict(sr_idx=6, mode=1, mode_ext=3, short_pct=20, mixed_pct=25),
    "lsf_scale_8k_js": dict(sr_idx=8, mode=1, mode_ext=-1, short_pct=25, mixed_pct=30),
}


def main():
    manifest = json.loads((HERE / "manifest.json").read_text())
    todo = [(name, upd, 7_000_003 + i, N_FRAMES) for i, (name, upd) in enumerate(CASES.items())]
    scale = [(name, upd, 7_100_003 + i, SCALE_FRAMES) for i, (name, upd) in enumerate(SCALE_CASES.items())]
    todo = scale if "--scale" in sys.argv[1:] else todo + scale
    for name, upd, seed, nf in todo:
        cfg = dict(_gen.C5)
        cfg.update(upd)
        data, _ = _gen.stream(cfg, seed, nf)
        ver, si = (data[1] >> 3) & 3, (data[2] >> 2) & 3
        hz = HZ[si + (0 if ver == 3 else 3 if ver == 2 else 6)]
        nch = 1 if (data[3] >> 6) == 3 else 2
        ref = ffmpeg_oracle.decode(data, hz, nch)
        assert ref.shape == (nch, nf * 576), ref.shape
        (HERE / (name + ".mp3")).write_bytes(data)
        np.save(HERE / (name + ".pcm16.npy"), to_int16(ref))
        manifest[name] = dict(cfg=cfg, seed=seed, frames=nf, hz=hz, nch=nch, spf=576)
        print(name, hz, nch, len(data))
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True))
    record_hashes()


if __name__ == "__main__":
    main()
