"""Segmented (frame-parallel) decode of one long stream: the product's
host-side plan (mp3d_long_plan) checked on the CPU.

The plan splits a stream into segments of L output frames; segment k is
decoded from frame seg_start[k] by a FRESH decoder and its frames from k*L
on must equal a sequential decode of the whole stream.  That claim rests on
the bit-reservoir rule (FFmpeg mp_decode_layer3 semantics, restated in
oracle/mp3_oracle.c orc_decode_frame_f64), so it is checked here with the
oracle itself: every segment decoded per frame by a fresh oracle decoder
must reproduce the sequential oracle decode bit for bit (float equality) --
on the FFmpeg golden streams (tagged, mid-stream entry, dropped frame,
resync over junk, cut-short final frame) and on long generated VBR/mono/
32-320 kbps streams.  No GPU involved."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd


def slot_decode(data, offs, start, end):
    """Oracle PCM of frame slots [start, end) decoded by a fresh decoder
    starting at slot `start` (None for slots without audio)."""
    dec = _oracle.Decoder()
    info_first = start == 0 and _oracle.lib().orc_is_info_frame(data[offs[0]:], len(data) - int(offs[0])) if len(offs) else False
    out = []
    for j in range(start, end):
        o = int(offs[j])
        fb = (144000 * (32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320)[(data[o + 2] >> 4) - 1]
              // (44100, 48000, 32000)[(data[o + 2] >> 2) & 3] + ((data[o + 2] >> 1) & 1))
        if j == 0 and info_first:
            out.append(None)
            continue
        frame = data[o:o + fb]
        if len(frame) < fb:
            frame = frame + b"\0" * (fb - len(frame))  # cut-short final frame: zeros (FFmpeg)
        r, pcm, info = dec.decode_frame(frame)
        out.append(pcm.copy() if r > 0 else None)
    return out


def check_segmented(data, L):
    offs, seg, wmax = mp3_amd.long_plan(data, L)
    n = len(offs)
    assert len(seg) == (n + L - 1) // L
    assert wmax == max([k * L - int(a) for k, a in enumerate(seg)] + [0])
    ref = slot_decode(data, offs, 0, n)
    for k, a in enumerate(seg):
        a = int(a)
        assert 0 <= a <= max(k * L - 2, 0)
        e = min(n, (k + 1) * L)
        got = slot_decode(data, offs, a, e)[k * L - a:]
        for j, g in zip(range(k * L, e), got):
            r = ref[j]
            assert (g is None) == (r is None), (L, k, j)
            if r is not None:
                assert np.array_equal(g, r), (L, k, j, float(np.abs(g - r).max()))
    return n


@pytest.mark.parametrize("name", ["keypress_128k_js", "edge_midstream", "edge_bv_drop", "edge_garbage",
                                  "edge_trunc", "c5_dual_32k_vbr", "c5_rand_b", "edge_320k_32k"])
@pytest.mark.parametrize("L", [1, 3, 5])
def test_segments_match_sequential_golden(name, L):
    data, _ = _golden.case(name)
    check_segmented(data, L)


@pytest.mark.parametrize("cfg,seed,L", [(_gen.C5, 801, 4), (_gen.C5, 802, 16), (_gen.C3, 803, 8)])
def test_segments_match_sequential_long(cfg, seed, L):
    data, _ = _gen.stream(cfg, seed, 120)
    assert check_segmented(data, L) == 120


def test_plan_frame_slots_match_oracle_walk():
    """frame_off agrees with the oracle's own sync/resync walk."""
    for name in ("keypress_128k_js", "edge_garbage", "edge_trunc"):
        data, _ = _golden.case(name)
        offs, seg, _ = mp3_amd.long_plan(data, 8)
        pos, walk = int(_oracle.lib().orc_skip_id3v2(data, len(data))), []
        while pos + 4 <= len(data):
            b = data[pos:pos + 3]
            ok = b[0] == 0xFF and (b[1] & 0xFE) == 0xFA and 0 < (b[2] >> 4) < 15 and ((b[2] >> 2) & 3) != 3
            if not ok:
                pos += 1
                continue
            fb = (144000 * (32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320)[(b[2] >> 4) - 1]
                  // (44100, 48000, 32000)[(b[2] >> 2) & 3] + ((b[2] >> 1) & 1))
            nch = 1 if (data[pos + 3] >> 6) == 3 else 2
            need = 4 + (0 if b[1] & 1 else 2) + (17 if nch == 1 else 32)
            if pos + fb > len(data) and pos + need > len(data):
                break
            walk.append(pos)
            pos += fb
        assert list(map(int, offs)) == walk, name


def test_plan_edges():
    assert len(mp3_amd.long_plan(b"", 4)[0]) == 0
    assert len(mp3_amd.long_plan(b"\0" * 1000, 4)[0]) == 0
    data, _ = _golden.case("keypress_128k_js")
    with pytest.raises(mp3_amd.MP3DError):
        mp3_amd.long_plan(data, 4, max_frames=5)  # capacity
    with pytest.raises(mp3_amd.MP3DError):
        mp3_amd.long_plan(data, 0)
