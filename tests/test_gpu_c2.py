"""GPU: BASELINE configs[1] (C2) at its full size -- 1,024 streams x 64 frames
of synthetic spectra through mp3d_batch_synth_only -- against the oracle
(orc_synth_only, double precision) on a stream subset, PCM within 1 LSB.

At 1,024 streams the library splits every stream into frame-parallel
segments (k_synth, one warm-up frame each); the test also pins that the
segmented decode is bit-identical to the one-wave-per-stream decode
(MP3D_SEG_FRAMES = F), including the per-stream state carried into a second
call."""
import os

import numpy as np
import pytest
import torch

import _gen
import _oracle
import mp3_amd

pytestmark = pytest.mark.gpu

N, F, NCH = 1024, 64, 2
SUBSET = [0, 1, 2, 511, 777, 1023]


def _oracle_pcm(xr, bt, mx, s, frames):
    L = _oracle.lib()
    d = L.orc_create()
    ref = np.zeros((frames, 1152, NCH), np.int16)
    L.orc_synth_only(d, np.ascontiguousarray(xr[s, :frames]).ctypes.data, np.ascontiguousarray(bt[s, :frames]).ctypes.data,
                     np.ascontiguousarray(mx[s, :frames]).ctypes.data, frames, NCH, 0, ref.ctypes.data, None)
    L.orc_destroy(d)
    return ref


def _run(xr, bt, mx, seg=None, calls=1, state=False):
    """decode F frames per call, `calls` calls, device buffers; PCM [N, calls*F, 2304]
    (and the final per-stream state blobs with state=True); seg: segment
    length for every call, or a list with one per call"""
    segs = seg if isinstance(seg, list) else [seg] * calls
    try:
        dec = mp3_amd.BatchDecoder(N, F)
        out = []
        for c in range(calls):
            if segs[c] is None:
                os.environ.pop("MP3D_SEG_FRAMES", None)
            else:
                os.environ["MP3D_SEG_FRAMES"] = str(segs[c])
            sl = slice(c * F, (c + 1) * F)
            d_xr, d_bt, d_mx = (torch.from_numpy(np.ascontiguousarray(a[:, sl])).cuda() for a in (xr, bt, mx))
            pcm = torch.zeros((N, F, 2304), dtype=torch.int16, device="cuda")
            dec.synth_only(d_xr, d_bt, d_mx, NCH, 44100, pcm=pcm)
            torch.cuda.synchronize()
            out.append(pcm.cpu().numpy())
        pcm = np.concatenate(out, axis=1)
        return (pcm, dec.get_state(0, N)) if state else pcm
    finally:
        os.environ.pop("MP3D_SEG_FRAMES", None)


def test_c2_full_size_vs_oracle():
    xr, bt, mx = _gen.c2_spectra(N, F, NCH)
    assert (bt == 2).mean() > 0.05 and mx.any()
    pcm = _run(xr, bt, mx)
    for s in SUBSET:
        ref = _oracle_pcm(xr, bt, mx, s, F)
        got = pcm[s, :, :1152 * NCH].reshape(F, 1152, NCH)
        assert np.abs(got.astype(np.int32) - ref.astype(np.int32)).max() <= 1, s


def test_c2_segments_bit_identical_across_calls():
    xr, bt, mx = _gen.c2_spectra(N, 2 * F, NCH, seed=4242)
    seq = _run(xr, bt, mx, seg=F, calls=2)   # one wave per stream
    for seg in (None, 4, 7):                  # library choice, short and ragged segments
        got = _run(xr, bt, mx, seg=seg, calls=2)
        assert np.array_equal(got, seq), seg
    for s in SUBSET[:3]:
        ref = _oracle_pcm(xr, bt, mx, s, 2 * F)
        g = seq[s, :, :1152 * NCH].reshape(2 * F, 1152, NCH)
        assert np.abs(g.astype(np.int32) - ref.astype(np.int32)).max() <= 1, s


def test_c2_state_tails_across_calls():
    """Segmented synth-only calls leave each stream's overlap + FIFO in a
    packed tail that the next segmented call reads (two tails in turn, no
    state copy per call); a one-segment call or a state read first copies
    the live tail back into the stream state.  Every mix of the two must be
    bit-identical to the one-wave-per-stream decode, PCM and final state."""
    xr, bt, mx = _gen.c2_spectra(N, 3 * F, NCH, seed=777)
    ref_pcm, ref_st = _run(xr, bt, mx, seg=F, calls=3, state=True)
    for sched in ([None, None, None], [None, None, F], [F, None, None], [None, F, 7]):
        pcm, st = _run(xr, bt, mx, seg=sched, calls=3, state=True)
        assert np.array_equal(pcm, ref_pcm), sched
        assert np.array_equal(st, ref_st), sched


def test_clipping_saturates_like_the_oracle():
    """Spectra scaled far past full scale: int16 PCM saturates to -32768 / 32767
    exactly where the oracle's clamp(floor(x 32768 + 0.5)) does (the decode paths
    convert with saturating int32 / packed-int16 conversions)."""
    n, F = 8, 6
    xr, bt, mx = _gen.c2_spectra(n, F, NCH, seed=99)
    xr = (xr * np.float32(40.0)).astype(np.float32)
    pcm = mp3_amd.BatchDecoder(n, F).synth_only(xr, bt, mx, NCH, 44100)
    clipped = 0
    for s in range(n):
        ref = _oracle_pcm(xr, bt, mx, s, F)
        got = pcm[s, :, :1152 * NCH].reshape(F, 1152, NCH)
        assert np.abs(got.astype(np.int32) - ref.astype(np.int32)).max() <= 1, s
        clipped += int((np.abs(ref.astype(np.int32)) >= 32767).sum())
    assert clipped > 1000
