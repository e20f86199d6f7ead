"""Edge-case golden fixtures (run in the build container only, like
make_golden.py): byte streams the reference player meets in practice, each
decoded by FFmpeg (Chromium 88 WebAudio, ffmpeg_oracle.py) and committed as
int16 PCM next to the stream bytes.

  edge_bv_drop    C3 stream, frame 5's first granule has big_values = 300
                  (> 288: FFmpeg drops the frame, reservoir restarts from
                  the frame's post-header bytes)
  edge_midstream  C3 stream entered at frame 4 (reservoir underflow:
                  the first granules decode as silence)
  edge_garbage    C3 stream with junk bytes (no 0xFF) before frame 0 and
                  between frames 3/4 and 9/10 (resync)
  edge_trunc      C3 stream whose last frame is cut short (dropped)
  edge_320k_32k   stereo 320 kbps @ 32 kHz (1441-B frames, long units:
                  exercises the multi-batch LDS staging of k_huffman)
  edge_p23_short  C3 stream, frames 3 and 6: part2_3_length of the first
                  unit cut to 60 % (its big_values run past the unit end --
                  FFmpeg stops decoding pairs there -- and the next unit
                  starts inside its data)
  edge_bt0_drop   C3-like stream (40 % short units), frame 4's first unit
                  has window switching with the reserved block_type 0
                  (FFmpeg: "invalid block type", frame dropped)

Usage:  python tests/golden/make_edge_golden.py [case ...]
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


def set_big_values(frame: bytearray, gr: int, ch: int, value: int):
    """Overwrite big_values of unit (gr, ch) in an MPEG-1 stereo frame's side info."""
    crc = 0 if frame[1] & 1 else 2
    nch = 1 if (frame[3] >> 6) == 3 else 2
    bit = (4 + crc) * 8 + 9 + (5 if nch == 1 else 3) + 4 * nch + 59 * (gr * nch + ch) + 12
    for i in range(9):
        b = bit + i
        v = (value >> (8 - i)) & 1
        frame[b >> 3] = (frame[b >> 3] & ~(0x80 >> (b & 7))) | (v << (7 - (b & 7)))


def set_bit(frame: bytearray, b: int, v: int):
    frame[b >> 3] = (frame[b >> 3] & ~(0x80 >> (b & 7))) | (v << (7 - (b & 7)))


def set_part2_3(frame: bytearray, gr: int, ch: int, value: int):
    """Overwrite part2_3_length of unit (gr, ch) in an MPEG-1 frame's side info."""
    crc = 0 if frame[1] & 1 else 2
    nch = 1 if (frame[3] >> 6) == 3 else 2
    bit = (4 + crc) * 8 + 9 + (5 if nch == 1 else 3) + 4 * nch + 59 * (gr * nch + ch)
    for i in range(12):
        set_bit(frame, bit + i, (value >> (11 - i)) & 1)


def get_part2_3(frame: bytes, gr: int, ch: int):
    crc = 0 if frame[1] & 1 else 2
    nch = 1 if (frame[3] >> 6) == 3 else 2
    bit = (4 + crc) * 8 + 9 + (5 if nch == 1 else 3) + 4 * nch + 59 * (gr * nch + ch)
    return sum(((frame[(bit + i) >> 3] >> (7 - ((bit + i) & 7))) & 1) << (11 - i) for i in range(12))


def cases():
    rng = np.random.default_rng(77)
    out = {}
    data, offs = _gen.stream(_gen.C3, 6_000_001, 16)
    ba = bytearray(data)
    f5 = bytearray(ba[offs[5]:offs[6]])
    set_big_values(f5, 0, 0, 300)
    ba[offs[5]:offs[6]] = f5
    out["edge_bv_drop"] = (bytes(ba), 44100, 2)

    data, offs = _gen.stream(_gen.C3, 6_000_002, 20)
    out["edge_midstream"] = (data[offs[4]:], 44100, 2)

    data, offs = _gen.stream(_gen.C3, 6_000_003, 16)
    junk = lambda n: bytes(rng.integers(0, 0xFF, n, dtype=np.uint8))  # noqa: E731  (never 0xFF)
    bounds = list(offs) + [len(data)]
    parts = [junk(5)]
    for f in range(16):
        parts.append(data[bounds[f]:bounds[f + 1]])
        if f in (3, 9):
            parts.append(junk(37))
    out["edge_garbage"] = (b"".join(parts), 44100, 2)

    data, offs = _gen.stream(_gen.C3, 6_000_004, 17)
    out["edge_trunc"] = (data[:offs[16] + 200], 44100, 2)

    cfg = dict(_gen.C5)
    cfg.update(sr_idx=2, bitrate_idx=14, mode=0, mode_ext=-1, short_pct=20, mixed_pct=20, crc_pct=0)
    data, offs = _gen.stream(cfg, 6_000_005, 16)
    out["edge_320k_32k"] = (data, 32000, 2)

    data, offs = _gen.stream(dict(_gen.C3, short_pct=40), 4242, 12)
    ba = bytearray(data)
    side = (int(offs[4]) + 4) * 8  # frame 4: MPEG-1 stereo, no CRC
    assert ba[(side + 53) >> 3] >> (7 - ((side + 53) & 7)) & 1  # window_switching of (gr 0, ch 0)
    set_bit(ba, side + 54, 0)  # block_type = 0 (reserved with window switching)
    set_bit(ba, side + 55, 0)
    out["edge_bt0_drop"] = (bytes(ba), 44100, 2)

    data, offs = _gen.stream(_gen.C3, 6_000_006, 12)
    ba = bytearray(data)
    for f in (3, 6):
        fr = bytearray(ba[offs[f]:offs[f + 1]])
        set_part2_3(fr, 0, 0, get_part2_3(fr, 0, 0) * 6 // 10)
        ba[offs[f]:offs[f + 1]] = fr
    out["edge_p23_short"] = (bytes(ba), 44100, 2)
    return out


def main():
    man_path = HERE / "manifest.json"
    manifest = json.loads(man_path.read_text())
    only = set(sys.argv[1:])
    for name, (data, hz, nch) in cases().items():
        if only and name not in only:
            continue
        ref = ffmpeg_oracle.decode(data, hz, nch)
        (HERE / (name + ".mp3")).write_bytes(data)
        np.save(HERE / (name + ".pcm16.npy"), to_int16(ref))
        prev = manifest.get(name, {})
        manifest[name] = dict(edge=True, hz=hz, nch=nch, frames=ref.shape[1] // 1152, bytes=len(data),
                              our_frames=prev.get("our_frames"), note=prev.get("note"))
        print(name, hz, nch, len(data), ref.shape)
    man_path.write_text(json.dumps(manifest, indent=1, sort_keys=True))
    record_hashes()


if __name__ == "__main__":
    main()
