"""Gapless playback: the demux kernel reads the
stream's leading Xing/Info frame and its LAME encoder extension; trimming
enc_delay + 529 leading samples (FFmpeg's demuxer, libavformat/mp3dec.c)
reproduces the FFmpeg output of the tagged real file.  Checked against the
committed FFmpeg golden of the tagged file (tests/golden/
keypress_128k_js.tagged.pcm16.npy) and the oracle's reading of the tag."""
import numpy as np
import pytest

import _golden
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu


def _tagged():
    data, _ = _golden.case("keypress_128k_js")
    return data, np.load(_golden.GOLDEN / "keypress_128k_js.tagged.pcm16.npy")


def test_stream_info_matches_oracle_tag_reading():
    data, _ = _tagged()
    dec = mp3_amd.BatchDecoder(2, 24)
    buf = np.frombuffer(data + data[253:], np.uint8)  # stream 1: same audio, tag stripped
    dec.decode(buf, [0, len(data)], [len(data), len(data) - 253], 24)
    info = dec.stream_info(2)
    found, tag = _oracle.info_tag(data)
    assert found and info[0].has_tag == 1
    for k in ("has_lame", "enc_delay", "enc_padding", "total_frames", "skip_samples", "end_sample"):
        assert getattr(info[0], k) == tag[k], (k, getattr(info[0], k), tag[k])
    assert info[1].has_tag == 0 and info[1].has_lame == 0 and info[1].skip_samples == 0


def test_batch_gapless_matches_ffmpeg_tagged():
    data, ref = _tagged()
    dec = mp3_amd.BatchDecoder(1, 24)
    pcm, infos = dec.decode(np.frombuffer(data, np.uint8), [0], [len(data)], 24)
    got = mp3_amd.gapless_trim(mp3_amd.pcm_to_planar(pcm[0], infos[0]), dec.stream_info(1)[0])
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert int(np.abs(got.astype(np.int32) - ref.astype(np.int32)).max()) <= 1


def test_per_frame_gapless_matches_ffmpeg_tagged():
    data, ref = _tagged()
    got = mp3_amd.Decoder().decode_stream(data, gapless=True)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert int(np.abs(got.astype(np.int32) - ref.astype(np.int32)).max()) <= 1


def test_tag_split_across_calls():
    """The Info frame and one audio frame in the first call, the rest of the
    audio in calls of 5 frames: state and tag carry across calls."""
    data, ref = _tagged()
    offs, pos = [], 253
    while pos + 4 <= len(data):
        offs.append(pos)
        pos += 144000 * 128 // 44100 + ((data[pos + 2] >> 1) & 1)
    offs.append(len(data))
    dec = mp3_amd.BatchDecoder(1, 8)
    cuts = [0, offs[1]] + offs[1::5][1:] + ([len(data)] if offs[1::5][-1] != len(data) else [])
    outs = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        pcm, infos = dec.decode(np.frombuffer(data[a:b], np.uint8), [0], [b - a], 8)
        outs.append(mp3_amd.pcm_to_planar(pcm[0], infos[0]))
    got = mp3_amd.gapless_trim(np.concatenate([o for o in outs if o.size], axis=1), dec.stream_info(1)[0])
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert int(np.abs(got.astype(np.int32) - ref.astype(np.int32)).max()) <= 1
