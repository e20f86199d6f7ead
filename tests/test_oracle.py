"""The CPU oracle (oracle/mp3_oracle.c) pinned against the FFmpeg golden
vectors (tests/golden/, produced by tests/golden/make_golden.py) and the
generator's by-construction integer truth."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle


@pytest.mark.parametrize("name", _golden.names())
def test_oracle_matches_ffmpeg_golden(name):
    data, ref = _golden.case(name)
    pcm, hz = _oracle.decode_stream(data)
    ours = _golden.to_int16(pcm)
    worst, exact = _golden.compare(name, ours, ref)
    assert worst <= 1, (name, worst)  # ±1 LSB (north_star tolerance)
    assert exact > 0.6  # FFmpeg is fixed-point: ~75% exact


def test_keypress_bitstream_facts():
    """21 audio frames, 128 kbps joint stereo M/S,
    part2_3_length == 0 in frames 12-21, main_data_begin in 0..511."""
    data, _ = _golden.case("keypress_128k_js")
    pos = 253
    dec = _oracle.Decoder()
    mdbs, nonempty = [], 0
    for f in range(21):
        fb = 144000 * 128 // 44100 + ((data[pos + 2] >> 1) & 1)
        r, pcm, info = dec.decode_frame(data[pos:pos + fb])
        assert r == 1152 and info.bitrate_kbps == 128 and info.channels == 2
        assert (data[pos + 3] >> 6) == 1 and ((data[pos + 3] >> 4) & 3) == 2
        is_, sf, xr, side = dec.taps()
        mdbs.append(int(side[0, 0, 15]))
        p23 = side[:, :, 0]
        if f >= 11:
            assert (p23 == 0).all()
        nonempty += int((p23 > 0).sum())
        # bit accounting: every unit consumes exactly part2_3_length bits
        assert np.array_equal(side[:, :, 16], p23), (f, side[:, :, 16], p23)
        pos += fb
    assert pos == len(data)
    assert max(mdbs) == 511 and min(mdbs) == 0
    assert nonempty == 37  # measured (SURVEY App. C quotes 44 = all units of frames 1-11)


LSF = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)


@pytest.mark.parametrize("cfg,seed", [(_gen.C3, 11), (_gen.C3, 12), (_gen.C5, 13), (_gen.C5, 14), (_gen.C5, 15),
                                      (LSF, 16), (LSF, 17), (LSF, 18), (dict(LSF, sr_idx=8), 19),
                                      (dict(LSF, mode=1, mode_ext=1), 20)])
def test_integer_stage_roundtrip(cfg, seed):
    """Generator-encoded is[] / scalefactors decode back exactly (bit-exact);
    MPEG-1 and MPEG-2/2.5 LSF (one granule, LSF scalefactor groups)."""
    nf = 12
    data, offs, truth = _gen.stream(cfg, seed, nf, truth=True)
    dec = _oracle.Decoder()
    for f in range(nf):
        end = offs[f + 1] if f + 1 < nf else len(data)
        r, pcm, info = dec.decode_frame(data[offs[f]:end])
        ngr = 2 if info.hz >= 32000 else 1
        assert r == 576 * ngr
        is_, sf, xr, side = dec.taps()
        for gr in range(ngr):
            for ch in range(info.channels):
                assert np.array_equal(is_[gr, ch], truth[f, gr, ch]["is"]), (f, gr, ch)
                assert np.array_equal(sf[gr, ch], truth[f, gr, ch]["sf"]), (f, gr, ch)
                assert side[gr, ch, 0] == truth[f, gr, ch]["part2_3_length"]
                assert side[gr, ch, 16] == side[gr, ch, 0]


def test_oracle_gapless_matches_ffmpeg_tagged_output():
    """The LAME tag of the real file (Lavc56.30: delay 576, padding 0, 21
    frames) read as FFmpeg's demuxer does: trimming delay + 529 samples from
    the oracle's full decode reproduces the FFmpeg output of the tagged file
    (23 087 samples) within 1 LSB."""
    import mp3_amd
    data, _ = _golden.case("keypress_128k_js")
    ref = np.load(_golden.GOLDEN / "keypress_128k_js.tagged.pcm16.npy")
    found, tag = _oracle.info_tag(data)
    assert found and tag["has_lame"] and tag["enc_delay"] == 576 and tag["enc_padding"] == 0
    assert tag["total_frames"] == 21 and tag["skip_samples"] == 1105
    pcm, _ = _oracle.decode_stream(data)
    ours = mp3_amd.gapless_trim(_golden.to_int16(pcm), tag)
    assert ours.shape == ref.shape, (ours.shape, ref.shape)
    assert int(np.abs(ours.astype(np.int32) - ref.astype(np.int32)).max()) <= 1


def test_oracle_no_tag_no_trim():
    data, _ = _golden.case("c3_s0")
    found, tag = _oracle.info_tag(data)
    assert not found and not tag["has_lame"] and tag["skip_samples"] == 0


def _crc16_cms(data: bytes, crc=0xFFFF):
    """CRC-16 with polynomial 0x8005, MSB first, initial 0xFFFF, no final
    xor (the catalogued CRC-16/CMS; FFmpeg AV_CRC_16_ANSI seeded 0xFFFF)."""
    for byte in data:
        crc ^= byte << 8
        for _ in range(8):
            crc = ((crc << 1) ^ 0x8005) & 0xFFFF if crc & 0x8000 else (crc << 1) & 0xFFFF
    return crc


def _corrupt_crc(data, offs, frames):
    b = bytearray(data)
    for f in frames:
        b[int(offs[f]) + 5] ^= 0x5A
    return bytes(b)


CRC_CFG = dict(_gen.C5, crc_pct=100)


def test_crc16_known_answer_and_generator_crcs():
    """The CRC recipe matches the catalogue check value, and every frame the
    generator protects carries the CRC of its header bytes 2..3 + side info
    (ISO 11172-3 2.4.3.1) -- so the option below is pinned independently of
    the oracle's own implementation."""
    assert _crc16_cms(b"123456789") == 0xAEE7
    for cfg, seed in [(CRC_CFG, 31), (dict(CRC_CFG, sr_idx=-2), 32)]:
        data, offs = _gen.stream(cfg, seed, 10)
        for o in offs:
            o = int(o)
            assert data[o + 1] & 1 == 0  # protection bit 0 = CRC present
            lsf = (data[o + 1] >> 3) & 3 != 3
            mono = data[o + 3] >> 6 == 3
            side = (9 if mono else 17) if lsf else (17 if mono else 32)
            crc = _crc16_cms(data[o + 2:o + 4] + data[o + 6:o + 6 + side])
            assert crc == (data[o + 4] << 8 | data[o + 5])


def test_oracle_crc_option_drops_bad_frames():
    """ORC_OPT_CRC_CHECK: frames with a corrupted CRC are dropped (FFmpeg
    err_detect=crccheck+explode); without the option the CRC is ignored
    (FFmpeg's default, the golden decoder's behaviour)."""
    data, offs = _gen.stream(CRC_CFG, 33, 12)
    bad = _corrupt_crc(data, offs, [3, 7])
    ref, _ = _oracle.decode_stream(data)
    ign, _ = _oracle.decode_stream(bad)
    assert np.array_equal(ign, ref)
    chk, _ = _oracle.decode_stream(bad, opts=_oracle.OPT_CRC_CHECK)
    assert chk.shape[1] == ref.shape[1] - 2 * 1152
    assert np.array_equal(chk[:, :3 * 1152], ref[:, :3 * 1152])
    clean, _ = _oracle.decode_stream(data, opts=_oracle.OPT_CRC_CHECK)
    assert np.array_equal(clean, ref)


def test_flush_threshold_pinned():
    """FFmpeg's fixed-point requantiser rounds |xr| < 0.5 * 1.759 * 2^-28 to 0,
    and its intensity-stereo boundary then sees the right channel's band as
    empty (oracle/mp3_oracle.c ORC_FFMPEG_FLUSH).  The probe fixtures pin that
    threshold from both sides: no flush (the float decoder's rule) or a
    threshold of 1.30 * 2^-29 misses the FFmpeg output on a probe, 2.05 *
    2^-29 over-flushes on another, and the derived 1.759 * 2^-29 matches all."""
    import ctypes
    L = _oracle.lib()
    L.orc_set_flush.argtypes = [ctypes.c_double]
    probes = [n for n in _golden.names() if n.startswith("probe_flush_")] + ["scale_msis_mixed_32k"]

    def worst_over_probes():
        out = {}
        for n in probes:
            data, ref = _golden.case(n)
            out[n] = _golden.compare(n, _golden.to_int16(_oracle.decode_stream(data)[0]), ref)[0]
        return out

    try:
        for t in (0.0, 1.30 * 2.0 ** -29, 2.05 * 2.0 ** -29):
            L.orc_set_flush(t)
            assert max(worst_over_probes().values()) > 1, t
        L.orc_set_flush(-1.0)  # back to the FFmpeg threshold
        assert max(worst_over_probes().values()) <= 1
    finally:
        L.orc_set_flush(-1.0)
