"""GPU: per-stream state save / restore (ABI v4, SURVEY §5 "checkpoint /
resume analogue"), handle isolation of the frame-parallel long decode, the
host PCM sink's untouched bytes, the per-frame call over every golden, and
stream placement at unaligned buffer ends (VERDICT r01 items 4, 7, 10;
ADVICE r01)."""
import ctypes

import numpy as np
import pytest
import torch

import _gen
import _golden
import mp3_amd
from test_gpu_parity import split_frames

pytestmark = pytest.mark.gpu


def _chunks(buf, offs, sizes, n, k0, k1):
    """frames [k0, k1) of each generated stream, packed as a new batch"""
    parts = []
    for s in range(n):
        data = bytes(buf[offs[s]:offs[s] + sizes[s]])
        fo = split_frames(data) + [len(data)]
        parts.append(data[fo[k0]:fo[k1]])
    sz = np.array([len(p) for p in parts], np.uint32)
    of = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    return np.frombuffer(b"".join(parts), np.uint8), of, sz


def test_batch_state_moves_between_handles():
    """Decode 4 frames, save the state, restore it into a second handle (in
    other stream slots, through a device buffer) and decode the next 4 there:
    identical to one handle decoding all 8."""
    n, F = 24, 8
    buf, offs, sizes = _gen.batch(_gen.C5, 1401, n, F)
    ref, rinf = mp3_amd.BatchDecoder(n, F).decode(buf, offs, sizes, F)
    a = mp3_amd.BatchDecoder(n, 4)
    b = mp3_amd.BatchDecoder(2 * n, 4)
    p1, _ = a.decode(*_chunks(buf, offs, sizes, n, 0, 4), 4)
    st = a.get_state(0, n)
    assert st.shape == (n, mp3_amd.state_bytes())
    dst = torch.from_numpy(st.copy()).cuda()
    b.set_state(dst, first=n)
    blob, of, sz = _chunks(buf, offs, sizes, n, 4, 8)
    # streams land in slots n .. 2n - 1 of handle b (slots 0 .. n - 1 get empty input)
    of2 = np.concatenate([np.zeros(n, np.uint64), of])
    sz2 = np.concatenate([np.zeros(n, np.uint32), sz])
    p2, _ = b.decode(blob, of2, sz2, 4)
    assert np.array_equal(np.concatenate([p1, p2[n:]], axis=1), ref)
    # the host blob round-trips bit for bit
    back = b.get_state(n, n)
    assert back.shape == st.shape


def test_per_frame_seek_by_state():
    """Per-frame decoder: save the state after frame k, decode on, restore
    the saved state in a fresh decoder, decode from frame k again: the
    output equals the uninterrupted decode."""
    data, ref = _golden.case("c5_ms_is_mixed")
    d = mp3_amd.Decoder()
    pos, out, saved = 0, [], None
    for k in range(40):
        if pos >= len(data):
            break
        if k == 7:
            saved, saved_pos, saved_len = d.get_state(), pos, len(out)
        n, pcm, info = d.decode_frame(data[pos:], last=True)
        if info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        if n:
            out.append(pcm.copy())
    assert saved is not None
    e = mp3_amd.Decoder()
    e.set_state(saved)
    pos, tail = saved_pos, []
    while pos < len(data):
        n, pcm, info = e.decode_frame(data[pos:], last=True)
        if info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        if n:
            tail.append(pcm.copy())
    assert len(tail) == len(out) - saved_len
    for x, y in zip(tail, out[saved_len:]):
        assert np.array_equal(x, y)


def test_decode_long_leaves_handle_state():
    """mp3d_batch_decode_long between two streaming calls of the same handle
    does not disturb those streams (it used to zero them)."""
    n, F = 6, 4
    buf, offs, sizes = _gen.batch(_gen.C3, 1402, n, 2 * F)
    ref, _ = mp3_amd.BatchDecoder(n, 2 * F).decode(buf, offs, sizes, 2 * F)
    h = mp3_amd.BatchDecoder(n, F + 11)
    p1, _ = h.decode(*_chunks(buf, offs, sizes, n, 0, F), F)
    long_data, _ = _gen.stream(_gen.C3, 1403, 40)
    pl, il, _ = h.decode_long(long_data, segment_frames=4)
    assert len(pl) == 40 and (il["samples"] == 1152).all()
    p2, _ = h.decode(*_chunks(buf, offs, sizes, n, F, 2 * F), F)
    assert np.array_equal(np.concatenate([p1[:, :F], p2[:, :F]], axis=1), ref)


def test_host_sink_keeps_unwritten_bytes():
    """Host PCM: rows without audio and the second half of mono rows keep the
    caller's bytes; rows with audio equal a device-sink decode."""
    streams = [_gen.stream(dict(_gen.C5, mode=3), 1404, 5)[0], _gen.stream(_gen.C3, 1405, 3)[0]]
    sz = np.array([len(d) for d in streams], np.uint32)
    of = np.array([0, sz[0]], np.uint64)
    blob = np.frombuffer(b"".join(streams), np.uint8)
    F = 6
    host = np.full((2, F, 2304), 0x5A5A, np.int16)
    _, inf = mp3_amd.BatchDecoder(2, F).decode(blob, of, sz, F, pcm=host)
    dev = torch.full((2, F, 2304), 0x5A5A, dtype=torch.int16, device="cuda")
    mp3_amd.BatchDecoder(2, F).decode(torch.from_numpy(blob.copy()).cuda(), of, sz, F, pcm=dev)
    dev = dev.cpu().numpy()
    for s in range(2):
        for f in range(F):
            w = int(inf[s, f]["samples"]) * int(inf[s, f]["channels"])
            assert np.array_equal(host[s, f, :w], dev[s, f, :w]), (s, f)
            assert (host[s, f, w:] == 0x5A5A).all(), (s, f, w)
    assert int(inf[0, 0]["channels"]) == 1 and int(inf[1, 3]["samples"]) == 0


@pytest.mark.parametrize("name", _golden.names())
def test_per_frame_api_every_golden(name):
    """The player-facing per-frame call over every golden fixture (tags,
    junk, dropped frames, cut-short final frame, LSF), within 1 LSB."""
    data, ref = _golden.case(name)
    got = mp3_amd.Decoder().decode_stream(data)
    worst, _ = _golden.compare(name, got, ref)
    assert worst <= 1, (name, worst)


def test_per_frame_cut_short_needs_last_flag():
    data, ref = _golden.case("edge_trunc")
    d = mp3_amd.Decoder()
    L = mp3_amd.lib()
    info = mp3_amd.FrameInfo()
    pcm = np.zeros(2304, np.int16)
    pos, frames = 0, 0
    while True:
        r = L.mp3d_decode_frame(d._h, data[pos:], len(data) - pos, pcm.ctypes.data, ctypes.byref(info))
        if r < 0 or info.frame_bytes <= 0:
            break
        pos += info.frame_bytes
        frames += r > 0
    assert r == -6 and pos < len(data)  # without the flag: "need more"
    r = L.mp3d_decode_frame_ex(d._h, data[pos:], len(data) - pos, pcm.ctypes.data, mp3_amd.FRAME_LAST,
                               ctypes.byref(info))
    assert r == 1152 and pos + info.frame_bytes == len(data)


def test_unaligned_stream_ends_read_exactly():
    """Streams placed at every byte alignment, each followed directly by junk
    that looks like headers: the decode ignores every byte past a stream's
    end (k_demux reads aligned dwords and masks them at the end)."""
    base = [_gen.stream(_gen.C5, 1406 + s, 4)[0] for s in range(8)]
    F = 5
    junk = bytes([0xFF, 0xFB, 0x90, 0x64] * 8)
    parts, offs, sizes, pos = [], [], [], 0
    for s, d in enumerate(base):
        cut = d[: len(d) - (s % 4) * 37]  # some streams end inside a frame
        pad = b"\x00" * (s % 4)  # shift the next stream's start
        parts.append(pad + cut + junk)
        offs.append(pos + len(pad))
        sizes.append(len(cut))
        pos += len(pad) + len(cut) + len(junk)
    blob = b"".join(parts)
    off, sz = np.array(offs, np.uint64), np.array(sizes, np.uint32)
    t = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
    got, gi = mp3_amd.BatchDecoder(8, F).decode(t, off, sz, F)
    # the same streams, each alone with zero padding after it
    for s in range(8):
        d = blob[offs[s]:offs[s] + sizes[s]]
        one, oi = mp3_amd.BatchDecoder(1, F).decode(np.frombuffer(d + b"\0" * 64, np.uint8), [0], [len(d)], F)
        assert np.array_equal(gi[s], oi[0]), s
        for f in range(F):
            w = int(oi[0, f]["samples"]) * int(oi[0, f]["channels"])
            assert np.array_equal(got[s, f, :w], one[0, f, :w]), (s, f)


def test_batch_sync_is_stream_scoped():
    n, F = 8, 2
    buf, offs, sizes = _gen.batch(_gen.C3, 1407, n, F)
    dec = mp3_amd.BatchDecoder(n, F)
    s = torch.cuda.Stream()
    d_in = torch.from_numpy(buf).cuda()
    pcm = torch.zeros((n, F, 2304), dtype=torch.int16, device="cuda")
    dec.decode(d_in, offs, sizes, F, pcm=pcm, stream=s.cuda_stream)
    dec.sync()  # waits for the caller's stream the call ran on
    assert s.query()
    assert int((pcm != 0).sum()) > 0
