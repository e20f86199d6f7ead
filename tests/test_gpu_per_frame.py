"""The per-frame decoder's one-launch path (k_frame: demux, Huffman and
synthesis in one workgroup, completion by a mapped word instead of a stream
sync) against its three-kernel path (MP3D_PF_FUSED=0) and the FFmpeg golden
PCM, over every golden stream: bit-identical PCM and frame infos between the
two paths, within 1 LSB of the golden (the per-frame API over every golden,
ADVICE r01)."""
import os

import numpy as np
import pytest

import _golden
import mp3_amd

pytestmark = pytest.mark.gpu


def _decoder(fused, opts=0, readahead=0):
    """readahead=0: every call through the single-frame path under test
    (the read-ahead has its own tests, tests/test_gpu_readahead.py)"""
    env = {"MP3D_PF_FUSED": "1" if fused else "0", "MP3D_PF_READAHEAD": str(readahead)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = mp3_amd.Decoder()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    if opts:
        d.set_options(opts)
    return d


def _frames(dec, data, f32=False):
    """every frame's (samples, pcm, info fields) through mp3d_decode_frame_ex"""
    pos, out = 0, []
    while pos < len(data):
        try:
            n, pcm, info = dec.decode_frame(data[pos:], f32=f32, last=True)
        except mp3_amd.MP3DError:
            break
        if info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        out.append((n, pcm.copy(), (info.frame_bytes, info.channels, info.hz, info.bitrate_kbps, info.samples)))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert x[0] == y[0] and x[2] == y[2], i
        assert np.array_equal(x[1], y[1]), i


@pytest.mark.parametrize("name", _golden.names())
def test_fused_equals_three_kernel_path_and_golden(name):
    data, ref = _golden.case(name)
    fused = _frames(_decoder(True), data)
    _same(fused, _frames(_decoder(False), data))
    got = [p.reshape(n, -1) for n, p, _ in fused if n]
    got = np.concatenate(got).T if got else np.zeros((0, 0), np.int16)
    worst, _ = _golden.compare(name, got, ref)
    assert worst <= 1, (name, worst)


@pytest.mark.parametrize("name", ["keypress_128k_js", "lsf_24k_is"])
def test_fused_f32(name):
    data, _ = _golden.case(name)
    _same(_frames(_decoder(True), data, f32=True), _frames(_decoder(False), data, f32=True))


def test_fused_crc_option():
    names = [n for n in _golden.names() if "crc" in n]
    assert names
    for name in names:
        data, _ = _golden.case(name)
        bad = bytearray(data)
        bad[len(bad) // 2] ^= 0x5A  # one corrupted byte: a CRC-protected frame may drop
        for d in (bytes(data), bytes(bad)):
            _same(_frames(_decoder(True, mp3_amd.OPT_CRC_CHECK), d),
                  _frames(_decoder(False, mp3_amd.OPT_CRC_CHECK), d))


def test_fused_mixed_family_stream():
    """MPEG-1 frames then LSF frames in one stream: the family of the first
    frame holds, the others are skipped as junk -- the same on both paths."""
    a, _ = _golden.case("keypress_128k_js")
    b, _ = _golden.case("lsf_24k_is")
    data = a[: len(a) // 4] + b
    _same(_frames(_decoder(True), data), _frames(_decoder(False), data))


def test_fused_state_round_trip():
    """get_state after k frames, set_state on a fresh decoder: the rest of
    the stream decodes as in one pass (the one-launch path leaves the batch
    state consistent without a stream sync)."""
    data, _ = _golden.case("keypress_128k_js")
    one = _frames(_decoder(True), data)
    d = _decoder(True)
    pos, k = 0, 0
    while k < 10:
        n, _, info = d.decode_frame(data[pos:], last=True)
        pos += info.frame_bytes
        k += 1
    st = d.get_state()
    d2 = _decoder(True)
    d2.set_state(st)
    _same(one[10:], _frames(d2, data[pos:]))
