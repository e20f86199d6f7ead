"""GPU: the kernel variants chosen by batch width produce identical PCM,
frame infos and stream infos, call after call (carry, tags, family lock), on
every golden fixture, generated streams of both families, CRC-protected
streams under both CRC options, unaligned stream placements and garbage with
embedded sync words:
- demux: one wave per stream (k_demux; small batches, the per-frame decoder)
  vs one lane per stream (k_walk + k_mdcopy; from MP3D_WIDE_STREAMS
  streams), forced by MP3D_DEMUX;
- Huffman: one wave per unit (k_huffman_wave; up to MP3D_WAVE_HUFF_UNITS
  units) vs one lane per unit (k_huffman), forced by MP3D_HUFF."""
import os

import numpy as np
import pytest

import _gen
import _golden
import mp3_amd
from test_oracle import CRC_CFG, _corrupt_crc

pytestmark = pytest.mark.gpu

LSF = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)


def _corpus():
    streams = [_golden.case(n)[0] for n in _golden.names()]
    for k, cfg in enumerate([_gen.C3, _gen.C5, LSF]):
        for j in range(6):
            streams.append(_gen.stream(cfg, 7000 + 10 * k + j, 12)[0])
    for k, cfg in enumerate([CRC_CFG, dict(CRC_CFG, sr_idx=-2)]):
        data, offs = _gen.stream(cfg, 7100 + k, 10)
        streams.append(_corrupt_crc(data, offs, [3, 7]))
    rng = np.random.default_rng(71)
    for s in range(12):
        b = bytearray(rng.integers(0, 256, int(rng.integers(0, 2500)), dtype=np.uint8).tobytes())
        for _ in range(8):
            if len(b) < 8:
                break
            p = int(rng.integers(0, len(b) - 4))
            b[p], b[p + 1], b[p + 2] = 0xFF, int(rng.choice([0xFB, 0xFA, 0xF3, 0xE3])), int(rng.integers(0, 256)) & 0xFD
        if s % 4 == 0 and len(b) > 20:
            b[:3] = b"ID3"
        streams.append(bytes(b))
    return streams


def _run(path, streams, F, opts, pad, var="MP3D_DEMUX"):
    """two calls per stream: bytes [0, n/2), then [n/2, n) with the state
    carried (cut-short frames, mid-frame resync, reservoir carry)"""
    os.environ[var] = path
    try:
        chunks, offs, o = [], [], 0
        for s, d in enumerate(streams):
            gap = (s * 7) % 16 if pad else 0  # misaligned stream starts
            chunks.append(b"\xA5" * gap + d)
            offs.append(o + gap)
            o += gap + len(d)
        blob = np.frombuffer(b"".join(chunks) + b"\0" * 64, np.uint8)
        offs = np.array(offs, np.uint64)
        n = np.array([len(d) for d in streams], np.uint32)
        half = n // 2
        dec = mp3_amd.BatchDecoder(len(streams), F)
        dec.set_options(opts)
        out = []
        for of, sz in ((offs, half), (offs + half, n - half)):
            pcm, inf = dec.decode(blob, of, sz, F)
            info = [bytes(x) for x in dec.stream_info(len(streams))]
            out.append((pcm.copy(), inf.copy(), info))
        return out
    finally:
        os.environ.pop(var, None)


@pytest.mark.parametrize("opts", [0, mp3_amd.OPT_CRC_CHECK])
@pytest.mark.parametrize("pad", [False, True])
def test_paths_identical(opts, pad):
    streams = _corpus()
    a = _run("wave", streams, 16, opts, pad)
    b = _run("lane", streams, 16, opts, pad)
    for (pa, ia, sa), (pb, ib, sb) in zip(a, b):
        assert np.array_equal(ia, ib)
        assert np.array_equal(pa, pb)
        assert sa == sb


@pytest.mark.parametrize("opts", [0, mp3_amd.OPT_CRC_CHECK])
def test_huffman_kernels_identical(opts):
    streams = _corpus()
    a = _run("lane", streams, 16, opts, True, var="MP3D_HUFF")
    b = _run("wave", streams, 16, opts, True, var="MP3D_HUFF")
    for (pa, ia, sa), (pb, ib, sb) in zip(a, b):
        assert np.array_equal(ia, ib)
        assert np.array_equal(pa, pb)
        assert sa == sb


def test_huffman_kernels_identical_integer_stage():
    """is[] rows (up to nz_end) and scalefactors of both Huffman kernels"""
    streams = _corpus()
    sz = np.array([len(d) for d in streams], np.uint32)
    of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(streams) + b"\0" * 64, np.uint8)
    res = {}
    dec = mp3_amd.BatchDecoder(len(streams), 16)  # one handle: units no kernel writes hold the same bytes
    for path in ("lane", "wave"):
        os.environ["MP3D_HUFF"] = path
        try:
            dec.reset()
            res[path] = dec.huffman_only(blob, of, sz, 16)
        finally:
            os.environ.pop("MP3D_HUFF", None)
    assert np.array_equal(res["lane"][0], res["wave"][0])
    assert np.array_equal(res["lane"][1], res["wave"][1])
