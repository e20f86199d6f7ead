"""FFmpeg goldens at BASELINE-config scale (VERDICT r02 "do this" 1; run in the
build container only -- FFmpeg is the Chromium-88 decoder inside kaleido,
SURVEY.md §8(c) / Appendix B).

The other golden scripts pin at most 21 frames per stream.  This one pins:
  * bench_c3_g<g>  : the bench's own C3 streams, g = 0..7 (seed
                     shard.BASE_SEED_C3 + g, 32 frames: exactly the bytes
                     `bench.py` decodes for global stream g);
  * bench_c5_g<g>  : the bench's own C5 streams, g = 0..3 (seed 5_000_011 + g,
                     32 frames);
  * scale_<class>  : 256 frames per C5 corpus class (mono, intensity, M/S + IS
                     with mixed blocks, dual channel, plain stereo; 32 / 44.1 /
                     48 kHz; CBR and VBR; CRC-protected frames);
  * long_c3_512    : one 512-frame C3 stream, so main_data_begin = 511 and the
                     reservoir / IMDCT / synthesis-FIFO carry are pinned across
                     call splits far past frame 16;
  * probe_flush_*  : intensity-stereo streams whose right-channel bands hold
                     only lines so quiet that FFmpeg's fixed-point requantiser
                     rounds them to 0 (so it treats the band as empty and
                     applies intensity there): they pin that threshold from
                     both sides (oracle/mp3_oracle.c ORC_FFMPEG_FLUSH).  Each is
                     the first `frames` frames of a `gen_frames`-frame
                     generator stream, cut at a frame boundary.
Every case is a generator stream (tests/_gen.py, cfg + seed + gen_frames in
manifest.json), so tests/test_golden_repro.py rebuilds each byte for byte.

Usage:  python tests/golden/make_scale_golden.py
"""
import json
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1]))
import ffmpeg_oracle  # noqa: E402
import _gen  # noqa: E402
from make_golden import record_hashes, to_int16  # noqa: E402
from mp3_amd import shard  # noqa: E402

BENCH_C5_SEED = 5_000_011  # bench.py's C5 seed base (global stream g uses + g)


def cases():
    out = []
    for g in range(8):
        out.append(("bench_c3_g%d" % g, dict(_gen.C3), shard.BASE_SEED_C3 + g, 32))
    for g in range(4):
        out.append(("bench_c5_g%d" % g, dict(_gen.C5), BENCH_C5_SEED + g, 32))
    c5 = dict(_gen.C5)
    classes = {
        # name: overrides of the C5 generator config
        "mono_48k_vbr": dict(sr_idx=1, mode=3, bitrate_idx=0, crc_pct=30, short_pct=20, mixed_pct=30),
        "is_44k_cbr": dict(sr_idx=0, mode=1, mode_ext=1, bitrate_idx=11, crc_pct=0, short_pct=20, mixed_pct=0),
        "msis_mixed_32k": dict(sr_idx=2, mode=1, mode_ext=3, bitrate_idx=0, crc_pct=0, short_pct=30,
                               mixed_pct=50),
        "dual_48k_vbr": dict(sr_idx=1, mode=2, bitrate_idx=0, crc_pct=50, short_pct=20, mixed_pct=25),
        "stereo_32k_vbr": dict(sr_idx=2, mode=0, bitrate_idx=0, crc_pct=0, short_pct=25, mixed_pct=25),
        "js_ms_44k_320": dict(sr_idx=0, mode=1, mode_ext=2, bitrate_idx=14, crc_pct=0, short_pct=15,
                              mixed_pct=20),
        "rand": {},
    }
    for i, (name, upd) in enumerate(classes.items()):
        cfg = dict(c5)
        cfg.update(upd)
        out.append(("scale_" + name, cfg, 5_200_003 + i, 256))
    out.append(("long_c3_512", dict(_gen.C3), 3_100_003, 512))
    return out


def probes():
    """(name, cfg, seed, gen_frames, cut_frames): found by scanning 48 seeded
    IS streams (7_700_000 + i) for frames where FFmpeg's output changes with
    the flush threshold: 30 and 9 / 38 need a flush above 1.395 * 2^-29, 37
    one at most 2.0 * 2^-29."""
    out = []
    for i, cut in ((30, 70), (37, 112), (9, 114), (38, 115)):
        cfg = dict(_gen.C5, mode=1, mode_ext=[1, 3][i % 2], sr_idx=i % 3, crc_pct=0, short_pct=30, mixed_pct=30)
        out.append(("probe_flush_%d" % i, cfg, 7_700_000 + i, 256, cut))
    return out


def main():
    manifest = json.loads((HERE / "manifest.json").read_text())
    for name, cfg, seed, nf in cases():
        data, offs = _gen.stream(cfg, seed, nf)
        hz = [44100, 48000, 32000][(data[2] >> 2) & 3]
        nch = 1 if (data[3] >> 6) == 3 else 2
        ref = ffmpeg_oracle.decode(data, hz, nch)
        assert ref.shape == (nch, nf * 1152), (name, ref.shape)
        (HERE / (name + ".mp3")).write_bytes(data)
        np.save(HERE / (name + ".pcm16.npy"), to_int16(ref))
        manifest[name] = dict(cfg=cfg, seed=seed, frames=nf, hz=hz, nch=nch)
        print(name, hz, nch, nf, len(data))
    for name, cfg, seed, gen_nf, nf in probes():
        full, offs = _gen.stream(cfg, seed, gen_nf)
        data = full[:int(offs[nf])]
        hz = [44100, 48000, 32000][(data[2] >> 2) & 3]
        ref = ffmpeg_oracle.decode(data, hz, 2)
        assert ref.shape == (2, nf * 1152), (name, ref.shape)
        (HERE / (name + ".mp3")).write_bytes(data)
        np.save(HERE / (name + ".pcm16.npy"), to_int16(ref))
        manifest[name] = dict(cfg=cfg, seed=seed, gen_frames=gen_nf, frames=nf, hz=hz, nch=2)
        print(name, hz, nf, len(data))
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True))
    record_hashes()


if __name__ == "__main__":
    main()
