"""GPU: C-ABI argument and capacity errors are negative codes (never a
crash), options validate their flags, and a handle keeps working after an
error (SURVEY §8(b) error contract)."""
import ctypes

import numpy as np
import pytest

import _gen
import mp3_amd

pytestmark = pytest.mark.gpu


def test_error_codes_and_recovery():
    L = mp3_amd.lib()
    buf, offs, sizes = _gen.batch(_gen.C3, 1301, 4, 3)
    dec = mp3_amd.BatchDecoder(4, 3)
    pcm = np.zeros((8, 3, 2304), np.int16)
    h = dec._h
    # more streams / frames than the handle was created for
    assert L.mp3d_batch_decode(h, buf.ctypes.data, np.zeros(8, np.uint64).ctypes.data,
                               np.zeros(8, np.uint32).ctypes.data, 8, 3, pcm.ctypes.data, None, None) == -5
    assert L.mp3d_batch_decode(h, buf.ctypes.data, offs.ctypes.data, sizes.ctypes.data, 4, 4, pcm.ctypes.data,
                               None, None) == -5
    # NULL / non-positive arguments
    assert L.mp3d_batch_decode(h, None, offs.ctypes.data, sizes.ctypes.data, 4, 3, pcm.ctypes.data, None, None) == -1
    assert L.mp3d_batch_decode(h, buf.ctypes.data, offs.ctypes.data, sizes.ctypes.data, 0, 3, pcm.ctypes.data,
                               None, None) == -1
    assert L.mp3d_batch_decode(None, buf.ctypes.data, offs.ctypes.data, sizes.ctypes.data, 4, 3, pcm.ctypes.data,
                               None, None) == -1
    assert L.mp3d_batch_set_options(h, 0x100) == -1
    assert L.mp3d_batch_synth_only(h, pcm.ctypes.data, pcm.ctypes.data, pcm.ctypes.data, 1, 1, 2, 22050,
                                   pcm.ctypes.data, None) == -1  # synth_only: MPEG-1 rates only
    assert L.mp3d_strerror(-5) == b"batch exceeds handle capacity"
    # the handle still decodes correctly after the rejected calls
    out, infos = dec.decode(buf, offs, sizes, 3)
    assert (infos["samples"] == 1152).all()
    ref = mp3_amd.BatchDecoder(4, 3).decode(buf, offs, sizes, 3)[0]
    assert np.array_equal(out, ref)


def test_per_frame_need_more_and_garbage():
    d = mp3_amd.Decoder()
    L = mp3_amd.lib()
    info = mp3_amd.FrameInfo()
    pcm = np.zeros(2304, np.int16)
    assert L.mp3d_decode_frame(d._h, b"\x00\x01\x02", 3, pcm.ctypes.data, ctypes.byref(info)) == -6
    data, offs = _gen.stream(_gen.C3, 1302, 3)
    # a frame cut in half: no complete frame in the buffer
    assert L.mp3d_decode_frame(d._h, data[:200], 200, pcm.ctypes.data, ctypes.byref(info)) == -6
    n = L.mp3d_decode_frame(d._h, data, len(data), pcm.ctypes.data, ctypes.byref(info))
    assert n == 1152 and info.frame_bytes == offs[1]
