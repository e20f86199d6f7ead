"""GPU parity for MPEG-2 / 2.5 low sampling frequency (LSF) streams
(ISO 13818-3: 16 / 22.05 / 24 kHz, 8 / 11.025 / 12 kHz; one granule of 576
samples per frame, LSF scalefactor groups, LSF intensity stereo).

The oracle's LSF decode is pinned to FFmpeg by the lsf_* golden fixtures
(tests/test_oracle.py); here the HIP path is held to the oracle and to the
generator's integer truth.  Tolerances as tests/test_gpu_parity.py: integer
stage bit-exact, PCM within 1 LSB."""
import numpy as np
import pytest

import _gen
import _oracle
import mp3_amd
from test_gpu_parity import oracle_pcm16

pytestmark = pytest.mark.gpu

LSF = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)
LSF_CASES = [(LSF, 501), (dict(LSF, sr_idx=8), 502), (dict(LSF, mode=1, mode_ext=1), 503),
             (dict(LSF, mode=1, mode_ext=3), 504), (dict(LSF, mode=3), 505)]


@pytest.mark.parametrize("cfg,seed", LSF_CASES)
def test_lsf_huffman_bitexact_vs_truth(cfg, seed):
    n, F = 32, 6
    buf, offs, sizes = _gen.batch(cfg, seed, n, F)
    dec = mp3_amd.BatchDecoder(n, F)
    is_out, sf_out = dec.huffman_only(buf, offs, sizes, F)
    for s in range(n):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        _, _, truth = _gen.stream(cfg, seed + s, F, truth=True)
        nch = 1 if (data[3] >> 6) == 3 else 2
        for f in range(F):
            for ch in range(nch):  # one granule per LSF frame
                assert np.array_equal(is_out[s, f, 0, ch], truth[f, 0, ch]["is"]), (s, f, ch)
                assert np.array_equal(sf_out[s, f, 0, ch], truth[f, 0, ch]["sf"]), (s, f, ch)


@pytest.mark.parametrize("cfg,seed", LSF_CASES)
def test_lsf_batch_pcm_vs_oracle(cfg, seed):
    n, F = 64, 8
    buf, offs, sizes = _gen.batch(cfg, seed, n, F)
    dec = mp3_amd.BatchDecoder(n, F)
    pcm, infos = dec.decode(buf, offs, sizes, F)
    assert (infos["samples"] == 576).all()
    worst = 0
    for s in range(n):
        o = oracle_pcm16(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        assert got.shape == o.shape, (s, got.shape, o.shape)
        worst = max(worst, int(np.abs(got.astype(np.int32) - o.astype(np.int32)).max()))
    assert worst <= 1


def test_mixed_family_batch():
    """MPEG-1 and LSF streams interleaved in one batch: each k_synth family
    variant decodes its own streams and leaves the others alone."""
    F = 6
    b1, o1, s1 = _gen.batch(_gen.C5, 601, 24, F)
    b2, o2, s2 = _gen.batch(LSF, 602, 24, F)
    buf = np.concatenate([b1, b2])
    offs = np.empty(48, np.uint64)
    sizes = np.empty(48, np.uint32)
    offs[0::2], sizes[0::2] = o1, s1          # even slots MPEG-1
    offs[1::2], sizes[1::2] = o2 + len(b1), s2  # odd slots LSF
    dec = mp3_amd.BatchDecoder(48, F)
    pcm, infos = dec.decode(buf, offs, sizes, F)
    for s in range(48):
        assert (infos[s]["samples"] == (1152 if s % 2 == 0 else 576)).all(), s
        o = oracle_pcm16(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        got = mp3_amd.pcm_to_planar(pcm[s], infos[s])
        assert got.shape == o.shape, (s, got.shape, o.shape)
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s


def test_mixed_family_wide_batch_persistent_lsf_grid():
    """A wide batch (k_walk demux) with 2 048 LSF streams among 4 096: k_walk
    tags the family word, and the LSF k_synth variant runs its persistent
    grid (one resident round, fewer workgroups than blocks, so each walks
    several).  Bit-identical to the wave-per-stream demux path, which leaves
    the family word out and launches one workgroup per block; a stride
    sample within 1 LSB of the oracle; then an all-MPEG-1 call on the same
    decoder (family word of an older call: the LSF grid leaves at once)."""
    import os
    n, F = 4096, 2
    b1, o1, s1 = _gen.batch(_gen.C3, 611, n // 2, F, threads=8)
    b2, o2, s2 = _gen.batch(LSF, 612, n // 2, F, threads=8)
    buf = np.concatenate([b1, b2])
    offs = np.empty(n, np.uint64)
    sizes = np.empty(n, np.uint32)
    offs[0::2], sizes[0::2] = o1, s1
    offs[1::2], sizes[1::2] = o2 + len(b1), s2
    dec = mp3_amd.BatchDecoder(n, F)
    pcm_w, inf_w = dec.decode(buf, offs, sizes, F)
    pcm_w, inf_w = pcm_w.copy(), inf_w.copy()
    os.environ["MP3D_DEMUX"] = "wave"
    try:
        ref = mp3_amd.BatchDecoder(n, F)
        pcm_v, inf_v = ref.decode(buf, offs, sizes, F)
    finally:
        os.environ.pop("MP3D_DEMUX", None)
    assert np.array_equal(inf_w, inf_v)
    assert np.array_equal(pcm_w, pcm_v)
    for s in range(1, n, 258):  # odd slots: LSF
        assert (inf_w[s]["samples"] == 576).all(), s
        o = oracle_pcm16(bytes(buf[offs[s]:offs[s] + sizes[s]]))
        got = mp3_amd.pcm_to_planar(pcm_w[s], inf_w[s])
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s
    # the next call: MPEG-1 streams only, fresh states
    b3, o3, s3 = _gen.batch(_gen.C3, 613, n, F, threads=8)
    dec2 = mp3_amd.BatchDecoder(n, F)
    dec2.decode(buf, offs, sizes, F)           # tags the family word
    dec2.reset()
    pcm3, inf3 = dec2.decode(b3, o3, s3, F)    # no LSF stream: the LSF grid leaves
    assert (inf3["samples"] == 1152).all()
    for s in range(0, n, 511):
        o = oracle_pcm16(bytes(b3[o3[s]:o3[s] + s3[s]]))
        got = mp3_amd.pcm_to_planar(pcm3[s], inf3[s])
        assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1, s


def test_lsf_state_carries_across_calls():
    """Two calls of 4 frames == one call of 8 (reservoir, overlap, FIFO and
    the MPEG-family lock resident in HBM between calls)."""
    n, F = 16, 8
    buf, offs, sizes = _gen.batch(dict(LSF, mode=1, mode_ext=3), 701, n, F)
    one = mp3_amd.BatchDecoder(n, F)
    pcm1, _ = one.decode(buf, offs, sizes, F)
    halves = [[], []]
    for s in range(n):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        fo = [int(x) for x in mp3_amd.long_plan(data, segment_frames=F)[0]] + [len(data)]
        halves[0].append(data[:fo[4]])
        halves[1].append(data[fo[4]:])
    two = mp3_amd.BatchDecoder(n, 4)
    parts = []
    for h in halves:
        sz = np.array([len(x) for x in h], np.uint32)
        of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
        p, _ = two.decode(np.frombuffer(b"".join(h), np.uint8), of, sz, 4)
        parts.append(p)
    assert np.array_equal(np.concatenate(parts, axis=1), pcm1)


def test_lsf_per_frame_api():
    data, _, _ = _gen.stream(dict(LSF, sr_idx=4, mode=1, mode_ext=3), 801, 10, truth=True)
    got = mp3_amd.Decoder().decode_stream(data)
    o = oracle_pcm16(data)
    assert got.shape == o.shape == (2, 5760), (got.shape, o.shape)
    assert np.abs(got.astype(np.int32) - o.astype(np.int32)).max() <= 1


def test_lsf_long_stream_segments():
    """Frame-parallel decode of one long LSF stream equals the sequential
    decode bit for bit (the warm-up rule holds for 8-bit main_data_begin)."""
    data, _ = _gen.stream(dict(LSF, sr_idx=3, mode=1, mode_ext=2), 901, 200)
    seq = mp3_amd.Decoder().decode_stream(data)
    dec = mp3_amd.BatchDecoder(16, 64)
    pcm, infos, _ = dec.decode_long(data, segment_frames=16)
    got = mp3_amd.pcm_to_planar(pcm, infos)
    assert np.array_equal(got, seq)
