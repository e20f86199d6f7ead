"""GPU: MP3D_OPT_CRC_CHECK (CRC-16 of error-protected frames, ISO 11172-3
2.4.3.1).  Off (default): the CRC is ignored, as FFmpeg's default decoder
does.  On: a frame whose CRC mismatches is dropped like a bad frame, as
FFmpeg with err_detect=crccheck+explode does.  The oracle's option is
pinned by tests/test_oracle.py (catalogue check value + generator CRCs);
PCM within 1 LSB of it."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd
from test_oracle import CRC_CFG, _corrupt_crc

pytestmark = pytest.mark.gpu


def _streams():
    out = []
    for k, cfg in enumerate([CRC_CFG, dict(CRC_CFG, sr_idx=-2), dict(CRC_CFG, mode=3)]):
        data, offs = _gen.stream(cfg, 900 + k, 10)
        out.append(_corrupt_crc(data, offs, [2 + k, 6]))
    data, offs = _gen.stream(CRC_CFG, 910, 10)  # intact CRCs
    out.append(data)
    return out


@pytest.mark.parametrize("opts", [0, mp3_amd.OPT_CRC_CHECK])
def test_batch_crc_option_vs_oracle(opts):
    streams = _streams()
    sz = np.array([len(d) for d in streams], np.uint32)
    of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(streams) + b"\0" * 16, np.uint8)
    dec = mp3_amd.BatchDecoder(len(streams), 10)
    dec.set_options(opts)
    pcm, infos = dec.decode(blob, of, sz, 10)
    for s, data in enumerate(streams):
        ref = _oracle.decode_stream(data, opts=opts)[0]
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        o = _golden.to_int16(ref)
        assert got.shape == o.shape, (s, opts, got.shape, o.shape)
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, (s, opts)
        dropped = int((infos[s]["samples"] == 0).sum())
        assert dropped == (2 if opts and s < 3 else 0), (s, opts, dropped)


def test_per_frame_crc_option():
    data, offs = _gen.stream(CRC_CFG, 920, 8)
    bad = _corrupt_crc(data, offs, [4])
    d = mp3_amd.Decoder()
    assert d.decode_stream(bad).shape[1] == 8 * 1152
    d2 = mp3_amd.Decoder()
    d2.set_options(mp3_amd.OPT_CRC_CHECK)
    assert d2.decode_stream(bad).shape[1] == 7 * 1152
