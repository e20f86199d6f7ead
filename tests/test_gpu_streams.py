"""Batch calls on the caller's HIP streams (VERDICT r02
item 2): the handle orders a call on a new stream after its previous call
(an event, never the old stream handle), sync / get_state / reset wait on
that event even after the caller destroyed the stream of the last call, and
a streaming loop whose offsets move on every call, each call on a new
caller stream, is bit-identical to one call over all frames."""
import numpy as np
import pytest
import torch

import _gen
import mp3_amd
from _state import state_view as _state_view

pytestmark = pytest.mark.gpu


def _hip():
    import ctypes
    L = ctypes.CDLL("libamdhip64.so")
    L.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    L.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return L


def test_calls_on_changing_streams_and_destroyed_stream():
    import ctypes
    hip = _hip()
    n, W, K = 96, 8, 4
    buf, offs, sizes = _gen.batch(_gen.C5, 9100, n, W * K, threads=4)
    d_in = torch.from_numpy(buf).cuda()
    ref = mp3_amd.BatchDecoder(n, W * K)
    p_ref = torch.zeros((n, W * K, 2304), dtype=torch.int16, device="cuda")
    i_ref = torch.zeros((n, W * K, 6), dtype=torch.int32, device="cuda")
    ref.decode(d_in, offs, sizes, W * K, pcm=p_ref, infos=i_ref)
    torch.cuda.synchronize()
    st_ref = ref.get_state(0, n)
    fb = i_ref[..., 0].cpu().numpy().astype(np.int64)

    dec = mp3_amd.BatchDecoder(n, W)
    parts = [torch.zeros((n, W, 2304), dtype=torch.int16, device="cuda") for _ in range(K)]
    torch.cuda.synchronize()  # the zero fills, before calls on streams torch does not know
    raw = []
    for k in range(K):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        raw.append(h)
        a = fb[:, : k * W].sum(1).astype(np.uint64)
        b = fb[:, : (k + 1) * W].sum(1).astype(np.uint64)
        # a new stream per call: each call is ordered after the previous one
        dec.decode(d_in, offs + a, (b - a).astype(np.uint32), W, pcm=parts[k], stream=h.value)
    # the callers' streams go away (work still queued) before the host asks
    for h in raw:
        assert hip.hipStreamDestroy(h) == 0
    st = dec.get_state(0, n)  # waits on the handle's end-of-call event
    dec.sync()
    assert torch.equal(torch.cat(parts, 1), p_ref)
    assert np.array_equal(_state_view(st), _state_view(st_ref))
    dec.reset()
    z = dec.get_state(0, n)
    assert (z[:, 540:544].copy().view(np.uint32) == 0x05050505).all()  # StreamState.fmt, the format stamp
    z[:, 540:544] = 0
    assert not z.any()


def test_state_buffer_size_checks():
    dec = mp3_amd.BatchDecoder(4, 2)
    sb = mp3_amd.state_bytes()
    with pytest.raises(ValueError):
        dec.get_state(0, 2, out=np.zeros(sb, np.uint8))  # one blob for two streams
    with pytest.raises(ValueError):
        dec.get_state(3, 2)  # past max_streams
    with pytest.raises(ValueError):
        dec.set_state(np.zeros(sb + 1, np.uint8))  # not whole blobs
    st = dec.get_state(0, 4)
    dec.set_state(torch.from_numpy(st.view(np.int32)).cuda(), first=0)  # 4 blobs as int32 words
    assert np.array_equal(dec.get_state(0, 4), st)


def test_geometry_cache_large_batch():
    """The geometry cache (mp3d_host.cpp prepare_geometry) at more than 1 024
    streams: a call with the same offsets and sizes skips the staging copy, a
    call that changes them (same count) stages again.  Three calls on one
    handle -- batch A, batch B with A's geometry but other bytes, batch C with
    other sizes -- each equal a fresh handle's decode of the same batch."""
    n, F = 1500, 3
    bufA, offs, sizes = _gen.batch(_gen.C5, 9300, n, F, threads=4)
    bufB = bufA.copy()
    # batch B: every stream's bytes replaced by another stream's (same sizes where they match)
    bufC, offsC, sizesC = _gen.batch(_gen.C5, 9400, n, F, threads=4)
    assert not np.array_equal(sizes, sizesC)
    perm = np.roll(np.arange(n), 1)
    same = sizes[perm] == sizes
    for i in np.nonzero(same)[0]:
        j = perm[i]
        bufB[int(offs[i]):int(offs[i]) + int(sizes[i])] = bufA[int(offs[j]):int(offs[j]) + int(sizes[j])]
    cases = [(bufA, offs, sizes), (bufB, offs, sizes), (bufC, offsC, sizesC)]
    dec = mp3_amd.BatchDecoder(n, F)
    for buf, o, z in cases:
        d_in = torch.from_numpy(buf).cuda()
        dec.reset()
        got, gi = dec.decode(d_in, o, z, F)
        ref_dec = mp3_amd.BatchDecoder(n, F)
        ref, ri = ref_dec.decode(d_in, o, z, F)
        ref_dec.close()
        assert np.array_equal(gi, ri)
        assert np.array_equal(got, ref)
    dec.close()
