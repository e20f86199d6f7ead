"""Regenerate the committed golden fixtures (run in the build container only).

For each case: the MP3 bytes (tests/golden/<case>.mp3) and FFmpeg's decoded
PCM (tests/golden/<case>.pcm16.npy, int16 [nch, samples], raw/untrimmed).

The FFmpeg decoder in the container is the FIXED-POINT one: Chromium hands
its int16 output to WebAudio as float via n/32767 (n >= 0) and n/32768
(n < 0), so the exact int16 samples are recovered below (all integral to
within float32 rounding, asserted).

Every script here merges its cases into manifest.json and then rewrites
hashes.json (sha256 of every committed fixture file); tests/test_golden_repro.py
checks both, and that the generator still reproduces each generated stream's
committed bytes (so this script regenerates exactly what is committed).

Usage:  python tests/golden/make_golden.py
"""
import hashlib
import json
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))
import ffmpeg_oracle  # noqa: E402
import _gen  # noqa: E402

FIX_SRC = "/opt/conda/lib/python3.9/site-packages/notebook/static/components/MathJax/extensions/a11y/invalid_keypress.mp3"
N_FRAMES = 16


def to_int16(ref):
    n = np.where(ref >= 0, ref.astype(np.float64) * 32767.0, ref.astype(np.float64) * 32768.0)
    r = np.round(n)
    assert np.abs(n - r).max() < 0.01, np.abs(n - r).max()
    return r.astype(np.int16)


def cases():
    c3 = dict(_gen.C3)
    c5 = dict(_gen.C5)
    out = [("c3_s0", c3, 3_000_003), ("c3_s1", c3, 3_000_004)]
    variants = {
        "c5_ms_is_mixed": dict(sr_idx=0, mode=1, mode_ext=3, short_pct=25, mixed_pct=50, crc_pct=0, bitrate_idx=9),
        "c5_is_only_48k": dict(sr_idx=1, mode=1, mode_ext=1, short_pct=20, mixed_pct=0, crc_pct=0, bitrate_idx=11),
        "c5_mono_48k_crc": dict(sr_idx=1, mode=3, short_pct=20, mixed_pct=30, crc_pct=100, bitrate_idx=0),
        "c5_dual_32k_vbr": dict(sr_idx=2, mode=2, short_pct=20, mixed_pct=30, crc_pct=0, bitrate_idx=0),
        "c5_stereo_vbr": dict(sr_idx=-1, mode=0, short_pct=20, mixed_pct=30, crc_pct=50, bitrate_idx=0),
        "c5_rand_a": {},
        "c5_rand_b": {},
    }
    for i, (name, upd) in enumerate(variants.items()):
        cfg = dict(c5)
        cfg.update(upd)
        out.append((name, cfg, 5_000_003 + i))
    return out


def record_hashes():
    """hashes.json: sha256 of every fixture file (.mp3 inputs, .npy PCM)."""
    files = sorted(p for p in HERE.iterdir() if p.suffix in (".mp3", ".npy"))
    h = {p.name: hashlib.sha256(p.read_bytes()).hexdigest() for p in files}
    (HERE / "hashes.json").write_text(json.dumps(h, indent=1, sort_keys=True))


def main():
    manifest = json.loads((HERE / "manifest.json").read_text()) if (HERE / "manifest.json").exists() else {}
    # real-world fixture: MathJax a11y "invalid_keypress.mp3" (Apache-2.0)
    fix = open(FIX_SRC, "rb").read()
    (HERE / "keypress_128k_js.mp3").write_bytes(fix)
    raw = ffmpeg_oracle.decode(fix[253:], 44100, 2)   # tagless: ID3v2 (45 B) + Info frame (208 B) removed
    tagged = ffmpeg_oracle.decode(fix, 44100, 2)      # demuxer trims enc_delay 576 + 529
    np.save(HERE / "keypress_128k_js.pcm16.npy", to_int16(raw))
    np.save(HERE / "keypress_128k_js.tagged.pcm16.npy", to_int16(tagged))
    manifest["keypress_128k_js"] = dict(source="MathJax a11y invalid_keypress.mp3 (Apache-2.0)", tagless_offset=253,
                                        hz=44100, frames=raw.shape[1] // 1152)
    for name, cfg, seed in cases():
        data, offs = _gen.stream(cfg, seed, N_FRAMES)
        hz = [44100, 48000, 32000][(data[2] >> 2) & 3]
        nch = 1 if (data[3] >> 6) == 3 else 2
        ref = ffmpeg_oracle.decode(data, hz, nch)
        assert ref.shape == (nch, N_FRAMES * 1152), ref.shape
        (HERE / (name + ".mp3")).write_bytes(data)
        np.save(HERE / (name + ".pcm16.npy"), to_int16(ref))
        manifest[name] = dict(cfg=cfg, seed=seed, frames=N_FRAMES, hz=hz, nch=nch)
        print(name, hz, nch, len(data))
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True))
    record_hashes()


if __name__ == "__main__":
    main()
