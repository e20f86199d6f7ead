"""Phase Q's chunk skipping (QZ): the requantiser runs
2, 3 or 5 of its 128-line chunks by the granule's largest nz_end.  Streams
from nearly silent to full bit budgets put granules in every class
(last nonzero line below 256, 256..383, from 384, none at all), checked
with the Huffman tap; their PCM is within 1 LSB of the oracle."""
import numpy as np
import pytest

import _gen
import mp3_amd
from test_gpu_parity import oracle_pcm16

pytestmark = pytest.mark.gpu


def test_requantiser_chunk_classes_vs_oracle():
    F = 8
    parts = []
    for k, (fill, br) in enumerate([(3, 9), (20, 9), (60, 11), (100, 14), (100, 9), (40, 5)]):
        parts.append(_gen.batch(dict(_gen.C3, fill_pct=fill, bitrate_idx=br), 8_200_001 + 977 * k, 16, F))
    buf = np.concatenate([p[0] for p in parts])
    offs, sizes, base = [], [], 0
    for b, o, s in parts:
        offs.append(o + base)
        sizes.append(s)
        base += len(b)
    offs, sizes = np.concatenate(offs).astype(np.uint64), np.concatenate(sizes).astype(np.uint32)
    n = len(offs)
    is_rows, _ = mp3_amd.BatchDecoder(n, F).huffman_only(buf, offs, sizes, F)
    rows = is_rows.reshape(n, F, 2, 2, 576)
    nz = rows != 0
    last = np.where(nz.any(-1), 575 - np.argmax(nz[..., ::-1], axis=-1), -1)  # [n, F, gr, ch]
    gmax = last.max(axis=-1)  # per granule, over both channels
    assert (gmax < 0).any(), "no silent granule"
    assert ((gmax >= 0) & (gmax < 256)).any()
    assert ((gmax >= 256) & (gmax < 384)).any()
    assert (gmax >= 384).any()
    dec = mp3_amd.BatchDecoder(n, F)
    pcm, infos = dec.decode(buf, offs, sizes, F)
    for s in range(0, n, 5):
        o = oracle_pcm16(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        assert got.shape == o.shape, s
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s
