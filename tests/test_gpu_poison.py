"""GPU: the first-call suites with every buffer poisoned (VERDICT r05 "do this" 1).

MP3D_DEBUG_POISON=1 (read when a handle is created, mp3d_host.cpp poison_env)
fills every device and pinned allocation of the handle with 0xFF when it is
made -- at create and at every grow() -- before the zeroing the code does on
purpose, and fills the whole LDS of every CU with 0xFF before each of the
handle's kernel launches (k_lds_poison).  A read of bytes that nothing wrote
then sees NaNs, all-ones words and huge lengths on EVERY run instead of
whatever an earlier allocation or workgroup left, so a read-before-write
fails deterministically here rather than once in a while.

The tests are the existing read-ahead, state-format, per-frame, long-stream
and scale-golden tests, called unchanged under the poison (their modules are
imported, not re-collected).  Every comparison they make is bit-exact between
paths or within 1 LSB of the FFmpeg golden PCM.

The helper thread that launches the next read-ahead run is checked the same
way: MP3D_DEBUG_RA_DELAY_US makes it sleep before each launch, so a served call
that depended on the launch having happened (a host flag instead of the run's
event) would read a run that is not there yet.  MP3D_DEBUG_RA_FAIL makes one
next-run launch report an error after its kernels ran: the
decoder must then refuse every call until a reset, never continue from the
advanced state.
"""
import numpy as np
import pytest

import _golden
import mp3_amd
import test_gpu_golden_scale as GS
import test_gpu_per_frame as PF
import test_gpu_readahead as RA
import test_gpu_state as ST
import test_gpu_state_format as SF

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def poison(monkeypatch):
    monkeypatch.setenv("MP3D_DEBUG_POISON", "1")


@pytest.mark.parametrize("name", _golden.names())
def test_poison_readahead_every_golden(name):
    RA.test_readahead_bit_identical_every_golden(name)


@pytest.mark.parametrize("name", _golden.names())
def test_poison_per_frame_every_golden(name):
    ST.test_per_frame_api_every_golden(name)


@pytest.mark.parametrize("name", ["keypress_128k_js", "lsf_24k_is", "lsf_scale_24k_is", "bench_c5_g1", "edge_garbage"])
def test_poison_fused_vs_three_kernels(name):
    PF.test_fused_equals_three_kernel_path_and_golden(name)


def test_poison_readahead_early_exits():
    RA.test_readahead_early_exits()


def test_poison_readahead_sink_change():
    RA.test_readahead_float_sink_and_sink_change()


@pytest.mark.parametrize("ra", [0, 32])
@pytest.mark.parametrize("name", ["bench_c5_g1", "lsf_scale_24k_is"])
def test_poison_per_frame_sink_switch(ra, name):
    SF.test_per_frame_sink_switch(ra, name)


@pytest.mark.parametrize("first_f32", [False, True])
def test_poison_batch_sink_switch(first_f32):
    SF.test_batch_sink_switch_keeps_history(first_f32)


def test_poison_state_stamp():
    SF.test_state_blob_format_stamp()


def test_poison_scale_goldens():
    GS.test_scale_goldens_one_batch_and_split_calls()


def test_poison_long_and_host_sink():
    ST.test_decode_long_leaves_handle_state()
    ST.test_host_sink_keeps_unwritten_bytes()


@pytest.mark.parametrize("name", ["lsf_scale_24k_is", "bench_c5_g1", "keypress_128k_js", "c5_ms_is_mixed"])
def test_helper_delay_readahead(monkeypatch, name):
    """The helper thread sleeps 3 ms before each next-run launch: the calls
    served meanwhile come from the current run, the switch to the next run
    waits for its launch (ra_join) and its event; output bit-identical to
    frame-by-frame decoding, with and without the poison."""
    monkeypatch.setenv("MP3D_DEBUG_RA_DELAY_US", "3000")
    data, _ = _golden.case(name)
    script = [("call", False)] * 600
    for ra in (16, 64):
        RA._same(RA._run(RA._dec(ra), data, script), RA._run(RA._dec(0), data, script))


def test_helper_delay_early_exits(monkeypatch):
    monkeypatch.setenv("MP3D_DEBUG_RA_DELAY_US", "3000")
    RA.test_readahead_early_exits()


def _stream():
    import _gen
    data, _ = _gen.stream(_gen.C5, 77_011, 200)
    return data


def test_failed_next_run_is_sticky(monkeypatch):
    """The first next-run launch fails after its kernels ran (so the device
    state is past the frames served): the decoder reports the error at the
    call that needs that run and at every call after it, until a reset; after
    the reset it decodes the stream from the start bit for bit."""
    data = _stream()
    script = [("call", False)] * 200
    ref = RA._run(RA._dec(0), data, script)
    monkeypatch.setenv("MP3D_DEBUG_RA_FAIL", "1")
    d = RA._dec(16)
    pos, k, err = 0, 0, None
    while pos < len(data) and k < len(ref):
        try:
            r = RA._call(d, data, pos)
        except mp3_amd.MP3DError as e:
            err = e
            break
        assert r[2] == ref[k][2] and np.array_equal(r[1], ref[k][1]), k
        pos += r[2][0]
        k += 1
    assert err is not None, "the injected failure was never reported"
    for _ in range(3):  # sticky: no call continues from the advanced state
        with pytest.raises(mp3_amd.MP3DError):
            RA._call(d, data, pos)
    d.reset()
    monkeypatch.delenv("MP3D_DEBUG_RA_FAIL")
    RA._same(RA._run(d, data, script), ref)


def test_failed_next_run_then_set_state(monkeypatch):
    """After the sticky error, a state saved before the failure puts the
    decoder back (set_state clears the error): the stream then decodes from
    that point bit for bit like a decoder that never read ahead."""
    data = _stream()
    script = [("call", False)] * 120
    ref = RA._run(RA._dec(0), data, script)
    monkeypatch.setenv("MP3D_DEBUG_RA_FAIL", "1")
    d = RA._dec(16)
    saved = d.get_state()  # at the stream start (nothing read ahead yet)
    pos, failed = 0, False
    for _ in script:
        try:
            r = RA._call(d, data, pos)
        except mp3_amd.MP3DError:
            failed = True
            break
        pos += r[2][0]
    assert failed, "the injected failure was never reported"
    with pytest.raises(mp3_amd.MP3DError):
        d.get_state()  # (sticky: no state past the served frames leaks out)
    d.set_state(saved)
    monkeypatch.delenv("MP3D_DEBUG_RA_FAIL")
    RA._same(RA._run(d, data, script), ref)


# ---- the batch paths under the poison (round 6): every golden through the
# batch API, odd and ragged shapes, LSF, CRC, corrupted main data, both demux
# paths, the segmented synth-only entry, the long-stream decode and gapless
import test_gpu_c2 as C2  # noqa: E402
import test_gpu_crc as CRC  # noqa: E402
import test_gpu_demux_paths as DP  # noqa: E402
import test_gpu_edges as ED  # noqa: E402
import test_gpu_fuzz as FZ  # noqa: E402
import test_gpu_gapless as GL  # noqa: E402
import test_gpu_long as LG  # noqa: E402
import test_gpu_lsf as LSF  # noqa: E402
import test_gpu_parity as PA  # noqa: E402


@pytest.mark.parametrize("name", _golden.names())
def test_poison_batch_every_golden(name):
    PA.test_golden_cases_batch_api(name)


def test_poison_edges():
    for args in ((ED._gen.C5, 501, 37, 5), (ED._gen.C3, 502, 3, 7)):
        ED.test_odd_shapes_pcm(*args)
    ED.test_ragged_mixed_batch()
    ED.test_high_bitrate_staging_batches()


def test_poison_lsf():
    LSF.test_mixed_family_batch()
    LSF.test_mixed_family_wide_batch_persistent_lsf_grid()
    LSF.test_lsf_state_carries_across_calls()
    LSF.test_lsf_per_frame_api()


@pytest.mark.parametrize("opts", [0, mp3_amd.OPT_CRC_CHECK])
def test_poison_crc(opts):
    CRC.test_batch_crc_option_vs_oracle(opts)


def test_poison_corrupted_main_data():
    FZ.test_corrupted_main_data_vs_oracle(FZ._gen.C5, 1201)
    FZ.test_random_garbage_never_faults()


@pytest.mark.parametrize("pad", [False, True])
def test_poison_demux_paths(pad):
    DP.test_paths_identical(0, pad)


def test_poison_c2_segments():
    C2.test_c2_segments_bit_identical_across_calls()
    C2.test_c2_state_tails_across_calls()


@pytest.mark.parametrize("name", ["keypress_128k_js", "edge_bv_drop", "edge_garbage"])
def test_poison_long_goldens(name):
    LG.test_long_golden_matches_sequential(name, 4)


def test_poison_gapless():
    GL.test_batch_gapless_matches_ffmpeg_tagged()
    GL.test_per_frame_gapless_matches_ffmpeg_tagged()
    GL.test_tag_split_across_calls()
