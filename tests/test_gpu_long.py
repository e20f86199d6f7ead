"""GPU: frame-parallel decode of one long stream (mp3d_batch_decode_long,
SURVEY.md §8(f) row 2) is bit-identical to the sequential GPU decode of the
same stream (one virtual stream, all frames in order), for int16 and float32
PCM, host and device buffers, segment lengths from 1 frame up, and handles
smaller than the segment count (several launches).  The sequential path is
itself checked against the oracle / FFmpeg golden PCM in test_gpu_parity.py;
the warm-up rule is checked against the oracle on CPU in test_long_plan.py."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu


def sequential(data, f32=False):
    n = len(mp3_amd.long_plan(data, 1)[0])
    dec = mp3_amd.BatchDecoder(1, n + 1)
    blob = np.frombuffer(data + b"\0" * 16, np.uint8)
    pcm, inf = dec.decode(blob, [0], [len(data)], n + 1, f32=f32)
    si = dec.stream_info(1)[0]
    return pcm[0, :n], inf[0, :n], si


def check(data, L, streams=64, f32=False):
    ref, rinf, rsi = sequential(data, f32)
    dec = mp3_amd.BatchDecoder(streams, L + 11)
    pcm, inf, si = dec.decode_long(data, L, f32=f32)
    assert pcm.shape == ref.shape
    assert np.array_equal(inf, rinf)
    audio = rinf["samples"] > 0
    for j in np.flatnonzero(audio):
        m = 1152 * int(rinf["channels"][j])
        assert np.array_equal(pcm[j, :m], ref[j, :m]), (L, j)
        assert not pcm[j, m:].any(), (L, j)
    assert not pcm[~audio].any()
    assert si.as_dict() == rsi.as_dict()
    return pcm, inf


@pytest.mark.parametrize("name", ["keypress_128k_js", "edge_midstream", "edge_bv_drop", "edge_garbage",
                                  "edge_trunc", "c5_dual_32k_vbr", "edge_320k_32k"])
@pytest.mark.parametrize("L", [1, 4])
def test_long_golden_matches_sequential(name, L):
    data, _ = _golden.case(name)
    check(data, L)


@pytest.mark.parametrize("cfg,seed,nf,L,streams", [(_gen.C3, 901, 600, 32, 64), (_gen.C5, 902, 500, 7, 16),
                                                   (_gen.C5, 903, 300, 2, 5)])
def test_long_generated_matches_sequential(cfg, seed, nf, L, streams):
    data, _ = _gen.stream(cfg, seed, nf)
    pcm, inf = check(data, L, streams)
    assert len(pcm) == nf


def test_long_f32_and_oracle():
    data, _ = _gen.stream(_gen.C3, 904, 256)
    pcm, inf = check(data, 16, f32=True)
    o, _ = _oracle.decode_stream(data)
    got = mp3_amd.pcm_to_planar(pcm, inf)
    assert got.shape == o.shape
    assert float(np.abs(got - o).max()) <= 2.0 ** -15


def test_long_device_buffers():
    import torch
    data, _ = _gen.stream(_gen.C5, 905, 200)
    ref, rinf, _ = sequential(data)
    n = len(ref)
    d_in = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    d_pcm = torch.full((n + 4, 2304), 7, dtype=torch.int16, device="cuda")
    d_inf = torch.zeros((n + 4, 6), dtype=torch.int32, device="cuda")
    dec = mp3_amd.BatchDecoder(8, 8 + 11)
    pcm, inf, _ = dec.decode_long(d_in, 8, max_frames=n + 4, pcm=d_pcm, infos=d_inf)
    torch.cuda.synchronize()
    assert pcm.shape[0] == n
    inf = inf.cpu().numpy().view(mp3_amd.FRAME_INFO_DT).reshape(n)
    assert np.array_equal(inf, rinf)
    audio = rinf["samples"] > 0
    got = pcm.cpu().numpy()
    for j in np.flatnonzero(audio):
        m = 1152 * int(rinf["channels"][j])
        assert np.array_equal(got[j, :m], ref[j, :m]), j
    assert (d_pcm[n:] == 7).all()  # rows past the stream untouched


def test_long_capacity_errors():
    data, _ = _golden.case("keypress_128k_js")
    dec = mp3_amd.BatchDecoder(4, 6)
    with pytest.raises(mp3_amd.MP3DError):
        dec.decode_long(data, 4)  # handle max_frames < L + warm-up
    dec2 = mp3_amd.BatchDecoder(4, 20)
    with pytest.raises(mp3_amd.MP3DError):
        dec2.decode_long(data, 4, max_frames=10)  # 22 slots > 10
