"""The per-frame call's read-ahead (mp3d_host.cpp
ra_fill / ra_settle): one call decodes up to 16 of the frames in the
caller's buffer in one batch call, the next calls are served from it after
a byte check.  Every output must be bit-identical to the single-frame path
(MP3D_PF_READAHEAD=0): over every golden stream, int16 and float sinks,
and through every way of leaving the read-ahead early -- a state save, a
seek (set_state), a jump ahead in the buffer, a sink change, new options
and a reset."""
import os

import numpy as np
import pytest

import _gen
import _golden
import mp3_amd
from _state import state_view

pytestmark = pytest.mark.gpu


def _dec(ra):
    old = os.environ.get("MP3D_PF_READAHEAD")
    os.environ["MP3D_PF_READAHEAD"] = str(ra)
    try:
        return mp3_amd.Decoder()
    finally:
        if old is None:
            del os.environ["MP3D_PF_READAHEAD"]
        else:
            os.environ["MP3D_PF_READAHEAD"] = old


def _call(d, data, pos, f32=False):
    n, pcm, info = d.decode_frame(data[pos:], f32=f32, last=True)
    return n, pcm.copy(), (info.frame_bytes, info.channels, info.hz, info.bitrate_kbps, info.samples)


def _run(d, data, script):
    """script: a list of ('call', f32) / ('skip', frames) / ('state',) /
    ('seek', saved index) / ('opts', flags) / ('reset',) steps; returns every
    output and the position after each call"""
    pos, out, saved = 0, [], []
    for step in script:
        if step[0] == "call":
            if pos >= len(data):
                break
            r = _call(d, data, pos, step[1])
            if r[2][0] <= 0:
                break
            pos += r[2][0]
            out.append(r)
        elif step[0] == "skip":
            for _ in range(step[1]):  # frames jumped over: found with a throw-away decoder
                pos += _call(_dec(0), data, pos)[2][0]
        elif step[0] == "state":
            saved.append((d.get_state(), pos))
            out.append(("state", saved[-1][0].copy()))
        elif step[0] == "seek":
            st, pos = saved[step[1]]
            d.set_state(st)
        elif step[0] == "opts":
            d.set_options(step[1])
        elif step[0] == "reset":
            d.reset()
            pos = 0
    return out


def _same(a, b):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        if x[0] == "state":
            assert y[0] == "state" and np.array_equal(state_view(x[1]), state_view(y[1])), i
            continue
        assert x[0] == y[0] and x[2] == y[2], (i, x[2], y[2])
        assert np.array_equal(x[1], y[1]), i


@pytest.mark.parametrize("name", _golden.names())
def test_readahead_bit_identical_every_golden(name):
    data, _ = _golden.case(name)
    script = [("call", False)] * 600
    _same(_run(_dec(16), data, script), _run(_dec(0), data, script))


def test_readahead_float_sink_and_sink_change():
    data, _ = _golden.case("bench_c5_g1")
    script = [("call", True)] * 5 + [("call", False)] * 7 + [("call", True)] * 30
    _same(_run(_dec(16), data, script), _run(_dec(0), data, script))


def test_readahead_early_exits():
    data, _ = _gen.stream(_gen.C5, 77_001, 90)
    call = [("call", False)]
    script = (call * 3 + [("state",)] + call * 20 + [("skip", 3)] + call * 4 + [("seek", 0)] + call * 6 +
              [("opts", mp3_amd.OPT_CRC_CHECK)] + call * 9 + [("opts", 0)] + call * 2 + [("state",)] + call * 17 +
              [("reset",)] + call * 40)
    _same(_run(_dec(16), data, script), _run(_dec(0), data, script))
    for k in (2, 5, 64):  # other read-ahead lengths
        _same(_run(_dec(k), data, script), _run(_dec(0), data, script))


def test_readahead_backoff_state_every_frame():
    """A player saving its state every frame: each save settles
    a read-ahead after one frame, so the decoder backs off (1, 2, 4 .. 64
    calls without read-ahead); the output stays bit-identical, through a
    whole read-ahead served afterwards (back-off cleared) and a reset."""
    data, _ = _gen.stream(_gen.C5, 77_003, 200)
    call = [("call", False)]
    script = (call + [("state",)]) * 90 + call * 70 + [("state",)] + [("reset",)] + (call + [("state",)]) * 20
    _same(_run(_dec(32), data, script), _run(_dec(0), data, script))


def _dec_env(ra, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return _dec(ra)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("ra", [16, 32, 64])
def test_readahead_next_run_boundaries(ra):
    """Two runs (the next one decoding behind the served calls, k_demux_fp
    demuxing both): leaving at every kind of point of a 512-frame stream --
    a state save right after a fill (next run pending), a jump at the run
    boundary (the next run dropped), a sink change at a boundary, a state
    save mid-run -- stays bit-identical to frame-by-frame decoding."""
    data, _ = _golden.case("long_c3_512")
    call = [("call", False)]
    script = (call + [("state",)] + call * (ra - 1) + [("skip", 1)] + call * (2 * ra) + [("call", True)] +
              call * 3 + [("state",)] + call * (ra + 5) + [("seek", 1)] + call * 150)
    _same(_run(_dec(ra), data, script), _run(_dec(0), data, script))


def test_readahead_next_run_off_same_output():
    """MP3D_PF_RA_NEXT=0 (one run at a time), MP3D_PF_RA_THREAD=0 (the next
    run launched on the calling thread) and the default (launched by the
    helper thread) give the same bits over a long stream and an LSF stream."""
    for name in ("long_c3_512", "lsf_scale_24k_is"):
        data, _ = _golden.case(name)
        script = [("call", False)] * 300
        ref = _run(_dec(32), data, script)
        _same(_run(_dec_env(32, MP3D_PF_RA_NEXT=0), data, script), ref)
        _same(_run(_dec_env(32, MP3D_PF_RA_THREAD=0), data, script), ref)
