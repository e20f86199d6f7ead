"""k_synth phase Q's two requantiser paths: the fused
path (lane = subband, MPEG-1 granules with long blocks in every channel and
neither intensity nor M/S) and the scatter path (M/S, intensity, short or
mixed blocks).  Batches whose granules take one path, the other, or switch
between them granule by granule, each within 1 LSB of the oracle and bit-
identical between one call and two calls of half the frames."""
import numpy as np
import pytest

import _gen
import mp3_amd
from test_gpu_parity import oracle_pcm16

pytestmark = pytest.mark.gpu

BASE = dict(_gen.C3, short_pct=0, mixed_pct=0)
CASES = [
    ("fused_stereo_lr", dict(BASE, mode=0, mode_ext=0), 8_100_001),     # L/R stereo: fused
    ("fused_mono", dict(BASE, mode=3, mode_ext=0), 8_100_002),          # mono: fused
    ("scatter_ms", dict(BASE, mode=1, mode_ext=2), 8_100_003),          # M/S: scatter
    ("scatter_is", dict(BASE, mode=1, mode_ext=1), 8_100_004),          # intensity: scatter
    ("switching", dict(_gen.C3, mode=0, mode_ext=0, short_pct=30, mixed_pct=20), 8_100_005),
]


@pytest.mark.parametrize("name,cfg,seed", CASES, ids=[c[0] for c in CASES])
def test_requantiser_paths_vs_oracle(name, cfg, seed):
    n, F = 64, 12
    buf, offs, sizes = _gen.batch(cfg, seed, n, F)
    dec = mp3_amd.BatchDecoder(n, F)
    pcm, infos = dec.decode(buf, offs, sizes, F)
    for s in range(0, n, 9):
        o = oracle_pcm16(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        assert got.shape == o.shape, (name, s)
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, (name, s)
    # two calls of F / 2 frames (state carried) == one call of F
    half = []
    for s in range(n):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        fo = [int(x) for x in mp3_amd.long_plan(data, segment_frames=F)[0]] + [len(data)]
        half.append((data[:fo[F // 2]], data[fo[F // 2]:]))
    two = mp3_amd.BatchDecoder(n, F // 2)
    parts = []
    for k in range(2):
        chunks = [h[k] for h in half]
        sz = np.array([len(x) for x in chunks], np.uint32)
        of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
        p, _ = two.decode(np.frombuffer(b"".join(chunks), np.uint8), of, sz, F // 2)
        parts.append(p.copy())
    assert np.array_equal(np.concatenate(parts, axis=1), pcm), name
