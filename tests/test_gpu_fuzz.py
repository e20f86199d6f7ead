"""GPU robustness: arbitrary bytes never fault the kernels, and corrupted
main data still decodes exactly as the oracle does.

- Random garbage (with and without embedded sync words / valid headers of
  both MPEG families) in a ragged batch: every call returns OK and frame
  infos stay within the format's limits.
- Valid MPEG-1 and LSF streams with random bytes of their main data
  overwritten (headers and side info intact): the Huffman decoder meets
  invalid codes, escape values and count1 overreads in arbitrary places;
  PCM must still match the oracle within 1 LSB (FFmpeg semantics on both
  sides; "parity unpinned" by FFmpeg output for these inputs)."""
import numpy as np
import pytest

import _gen
import _golden
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu

LSF = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)


def _batch(streams, F):
    sz = np.array([len(d) for d in streams], np.uint32)
    of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(streams) + b"\0" * 64, np.uint8)
    dec = mp3_amd.BatchDecoder(len(streams), F)
    return dec.decode(blob, of, sz, F)


def test_random_garbage_never_faults():
    rng = np.random.default_rng(77)
    streams = []
    for s in range(96):
        n = int(rng.integers(0, 3000))
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        # sprinkle sync words and plausible header bytes of both families
        for _ in range(int(rng.integers(0, 12))):
            if n < 8:
                break
            p = int(rng.integers(0, n - 4))
            b[p] = 0xFF
            b[p + 1] = int(rng.choice([0xFB, 0xFA, 0xF3, 0xF2, 0xE3, 0xE2]))
            b[p + 2] = int(rng.integers(0, 256)) & 0xFD
        if s % 8 == 0 and n > 20:
            b[:3] = b"ID3"  # ID3v2 header with a random (possibly huge) size
        streams.append(bytes(b))
    pcm, infos = _batch(streams, 24)
    assert ((infos["samples"] == 0) | (infos["samples"] == 576) | (infos["samples"] == 1152)).all()
    assert (infos["frame_bytes"] >= 0).all() and (infos["frame_bytes"] <= 2881).all()
    assert np.isin(infos["channels"], [0, 1, 2]).all()


@pytest.mark.parametrize("cfg,seed", [(_gen.C5, 1201), (LSF, 1202)])
def test_corrupted_main_data_vs_oracle(cfg, seed):
    rng = np.random.default_rng(seed)
    streams = []
    for s in range(24):
        data, offs = _gen.stream(cfg, seed * 100 + s, 8)
        b = bytearray(data)
        ends = list(offs[1:]) + [len(data)]
        for o, e in zip(offs, ends):
            o, e = int(o), int(e)
            lsf = (b[o + 1] >> 3) & 3 != 3
            mono = b[o + 3] >> 6 == 3
            head = 4 + (0 if b[o + 1] & 1 else 2) + ((9 if mono else 17) if lsf else (17 if mono else 32))
            for _ in range(int(rng.integers(1, 6))):
                if o + head < e:
                    b[int(rng.integers(o + head, e))] = int(rng.integers(0, 256))
        streams.append(bytes(b))
    pcm, infos = _batch(streams, 8)
    for s, data in enumerate(streams):
        o = _golden.to_int16(_oracle.decode_stream(data)[0])
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        assert got.shape == o.shape, (s, got.shape, o.shape)
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s
