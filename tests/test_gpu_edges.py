"""GPU parity on ragged and awkward batches (through the C ABI): odd stream
and frame counts (tails of the 64-unit / 256-unit Huffman work groups),
streams of different lengths and kinds in one batch (the edge-case golden
streams side by side), empty streams, a stream holding only an ID3v2 tag,
and high-bitrate streams whose units overflow one LDS staging batch.
Reference: the CPU oracle (itself pinned to FFmpeg, tests/test_oracle.py);
PCM within +-1 LSB, integer stage bit-exact."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu


def oracle_pcm16(data, max_frames=100000):
    pcm, hz = _oracle.decode_stream(data, max_frames)
    return _golden.to_int16(pcm)


def check_batch(streams, F):
    n = len(streams)
    sizes = np.array([len(d) for d in streams], np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(streams) + b"\0" * 16, np.uint8)
    dec = mp3_amd.BatchDecoder(n, F)
    pcm, infos = dec.decode(blob, offs, sizes, F)
    for s, data in enumerate(streams):
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        o = oracle_pcm16(data, F) if len(data) else np.zeros((1, 0), np.int16)
        if o.shape[1] == 0:
            assert got.shape[1] == 0, s
            continue
        assert got.shape == o.shape, (s, got.shape, o.shape)
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s


@pytest.mark.parametrize("cfg,seed,n,F", [(_gen.C5, 501, 37, 5), (_gen.C3, 502, 3, 7), (_gen.C5, 503, 65, 3)])
def test_odd_shapes_pcm(cfg, seed, n, F):
    buf, offs, sizes = _gen.batch(cfg, seed, n, F)
    check_batch([bytes(buf[offs[s]:offs[s] + sizes[s]]) for s in range(n)], F)


def test_odd_shapes_huffman_bitexact():
    cfg, seed, n, F = _gen.C5, 504, 37, 5
    buf, offs, sizes = _gen.batch(cfg, seed, n, F)
    dec = mp3_amd.BatchDecoder(n, F)
    is_out, sf_out = dec.huffman_only(buf, offs, sizes, F)
    for s in range(n):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        _, _, truth = _gen.stream(cfg, seed + s, F, truth=True)
        nch = 1 if (data[3] >> 6) == 3 else 2
        for f in range(F):
            for gr in range(2):
                for ch in range(nch):
                    assert np.array_equal(is_out[s, f, gr, ch], truth[f, gr, ch]["is"]), (s, f, gr, ch)
                    assert np.array_equal(sf_out[s, f, gr, ch], truth[f, gr, ch]["sf"]), (s, f, gr, ch)


def test_ragged_mixed_batch():
    """The edge-case golden streams (drop, mid-stream entry, junk, cut-short
    final frame, 320 kbps) plus an empty stream and a tag-only stream, all
    in one batch."""
    names = ["edge_bv_drop", "edge_midstream", "edge_garbage", "edge_trunc", "edge_320k_32k", "c5_mono_48k_crc",
             "keypress_128k_js"]
    streams = [_golden.case(nm)[0] for nm in names]
    id3_only = b"ID3\x04\x00\x00\x00\x00\x00\x05" + b"TSSE\x00"
    streams += [b"", id3_only]
    check_batch(streams, 24)


def test_high_bitrate_staging_batches():
    """320 kbps @ 32 kHz: a 64-unit round needs ~23 KB of main data, more
    than one 9.6 KB LDS staging batch."""
    cfg = dict(_gen.C5)
    cfg.update(sr_idx=2, bitrate_idx=14, mode=0, mode_ext=-1, short_pct=20, mixed_pct=20, crc_pct=0)
    n, F = 40, 4
    buf, offs, sizes = _gen.batch(cfg, 505, n, F)
    check_batch([bytes(buf[offs[s]:offs[s] + sizes[s]]) for s in range(n)], F)
    dec = mp3_amd.BatchDecoder(n, F)
    is_out, sf_out = dec.huffman_only(buf, offs, sizes, F)
    for s in range(0, n, 7):
        _, _, truth = _gen.stream(cfg, 505 + s, F, truth=True)
        for f in range(F):
            for gr in range(2):
                for ch in range(2):
                    assert np.array_equal(is_out[s, f, gr, ch], truth[f, gr, ch]["is"]), (s, f, gr, ch)
