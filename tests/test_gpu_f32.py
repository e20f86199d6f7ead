"""Float32 PCM sink (mp3d_batch_decode_f32 / mp3d_decode_frame_f32, SURVEY.md
§8(f) row 3): the same synthesis sums as the int16 sink, unscaled and
unclipped (FFmpeg's float decoder convention).  Checked (1) exactly against
the int16 sink (int16 == clamp(floor(f32 * 32768 + 0.5)) bit for bit), (2) against
the double-precision oracle within 2^-15 (the ±1 LSB north_star tolerance,
stated on the float scale) and (3) per-frame vs batch API."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu

TOL = 2.0 ** -15  # one int16 LSB on the float scale


@pytest.mark.parametrize("name", ["keypress_128k_js", "c5_mono_48k_crc", "c5_ms_is_mixed", "edge_320k_32k"])
def test_f32_sink_vs_int16_and_oracle(name):
    data, _ = _golden.case(name)
    nf = 80
    dec16, dec32 = mp3_amd.BatchDecoder(1, nf), mp3_amd.BatchDecoder(1, nf)
    buf = np.frombuffer(data, np.uint8)
    p16, i16 = dec16.decode(buf, [0], [len(data)], nf)
    p32, i32 = dec32.decode(buf, [0], [len(data)], nf, f32=True)
    assert p32.dtype == np.float32 and np.array_equal(i16, i32)
    g16 = mp3_amd.pcm_to_planar(p16[0], i16[0])
    g32 = mp3_amd.pcm_to_planar(p32[0], i32[0])
    assert np.array_equal(_golden.to_int16(g32), g16)
    o, _ = _oracle.decode_stream(data)
    assert o.shape == g32.shape
    d = np.abs(g32.astype(np.float64) - o)
    assert d.max() <= TOL and d.mean() < 1e-6, (name, d.max(), d.mean())


def test_f32_batch_many_streams_device_tensors():
    import torch
    n, F = 33, 5
    buf, offs, sizes = _gen.batch(_gen.C5, 77, n, F, threads=4)
    dec = mp3_amd.BatchDecoder(n, F)
    d_pcm = torch.zeros((n, F, 2304), dtype=torch.float32, device="cuda")
    d_inf = torch.zeros((n, F, 6), dtype=torch.int32, device="cuda")
    dec.decode(torch.from_numpy(buf).cuda(), offs, sizes, F, pcm=d_pcm, infos=d_inf, f32=True)
    torch.cuda.synchronize()
    pcm = d_pcm.cpu().numpy()
    inf = d_inf.cpu().numpy().view(mp3_amd.FRAME_INFO_DT).reshape(n, F)
    for s in range(n):
        o, _ = _oracle.decode_stream(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        g = mp3_amd.pcm_to_planar(pcm[s], inf[s])
        assert g.shape == o.shape and np.abs(g - o).max() <= TOL, s


def test_f32_per_frame_equals_batch():
    data, _ = _golden.case("c5_stereo_vbr")
    a = mp3_amd.Decoder().decode_stream(data, f32=True)
    dec = mp3_amd.BatchDecoder(1, 64)
    p, i = dec.decode(np.frombuffer(data, np.uint8), [0], [len(data)], 64, f32=True)
    assert np.array_equal(a, mp3_amd.pcm_to_planar(p[0], i[0]))
