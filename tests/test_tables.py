"""ISO 11172-3 constant tables: structural checks + byte-presence in the
FFmpeg copy of the same tables in the container's kaleido binary (SURVEY.md
Appendix B.3; skipped where that binary is absent, e.g. on the GPU box)."""
import os

import numpy as np
import pytest

import _tables as T

KBIN = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/bin/kaleido"
t = T.load()


@pytest.mark.parametrize("num", T.HTAB_ISO)
def test_huffman_complete_prefix_code(num):
    codes, lens = T.htab(t, num)
    assert sum(2.0 ** -int(l) for l in lens) == pytest.approx(1.0, abs=1e-12)
    words = [format(int(c), "0%db" % int(l)) for c, l in zip(codes, lens)]
    assert len(set(words)) == len(words)
    for i, a in enumerate(words):
        for j, b in enumerate(words):
            assert i == j or not b.startswith(a)
    assert int(lens.max()) <= 19


def test_quad_tables():
    for q in range(2):
        assert sum(2.0 ** -int(l) for l in t["MP3D_QUAD_LEN"][q]) == pytest.approx(1.0)
    assert list(t["MP3D_QUAD_CODE"][1]) == list(range(15, -1, -1))


def test_band_tables():
    assert t["MP3D_SFB_LONG_WIDTH"].shape == (9, 22) and t["MP3D_SFB_SHORT_WIDTH"].shape == (9, 13)
    for s in range(9):
        assert int(t["MP3D_SFB_LONG_WIDTH"][s].sum()) == 576
        assert int(t["MP3D_SFB_SHORT_WIDTH"][s].sum()) == 192
        # the mixed-block boundary: 8 (MPEG-1) / 6 (LSF) long bands cover the
        # lines of 3 short bands x 3 windows (36; 72 at MPEG-2.5 8 kHz)
        nl = 8 if s < 3 else 6
        edge = int(t["MP3D_SFB_LONG_WIDTH"][s][:nl].sum())
        assert edge == int(t["MP3D_SFB_SHORT_WIDTH"][s][:3].sum()) * 3 == (72 if s == 8 else 36)
        # every band width is even: a bitstream line pair (2k, 2k + 1) never
        # straddles two bands (k_synth reads one scale per pair, DevTables.lpair)
        assert not (t["MP3D_SFB_LONG_WIDTH"][s] % 2).any() and not (t["MP3D_SFB_SHORT_WIDTH"][s] % 2).any()


def test_lsf_tables():
    assert list(t["MP3D_SAMPLE_RATE"]) == [44100, 48000, 32000, 22050, 24000, 16000, 11025, 12000, 8000]
    nsf = t["MP3D_LSF_NSF"].astype(int)
    # every slen table covers 21 long bands, 12 short bands x 3 windows, or
    # 6 long + 9 short bands x 3 (mixed)
    for row in nsf:
        assert [int(row[b].sum()) for b in range(3)] == [21, 36, 33]


def test_synthesis_window_shape():
    w = t["MP3D_SYNTH_WINDOW_Q16"].astype(np.int64)
    assert w.shape == (257,) and w[0] == 0 and w[256] == 75038
    D = np.zeros(512)
    D[:257] = w / 65536.0
    for i in range(1, 256):
        D[512 - i] = D[i] if i % 64 == 0 else -D[i]
    # the window's DC gain is the filterbank's passband normalisation
    assert abs(D[256]) == D.__abs__().max()


def test_select_maps():
    sel = t["MP3D_HTAB_OF_SELECT"]
    assert sel[0] == -1 and sel[4] == -1 and sel[14] == -1
    assert all(sel[16:24] == 13) and all(sel[24:32] == 14)
    assert list(t["MP3D_LINBITS"][16:]) == [1, 2, 3, 4, 6, 8, 10, 13, 4, 5, 6, 7, 8, 9, 11, 13]


@pytest.mark.skipif(not os.path.exists(KBIN), reason="kaleido binary only in the build container")
def test_tables_present_in_ffmpeg_copy():
    kb = open(KBIN, "rb").read()
    region = (26_340_000, 26_360_000)  # FFmpeg mpegaudiodec tables

    def in_region(b):
        i = kb.find(b, region[0], region[1])
        return i >= 0

    for num in T.HTAB_ISO:
        codes, lens = T.htab(t, num)
        if num == 1:
            continue  # 4-entry table: too short to be a unique pattern
        assert in_region(codes.astype("<u2").tobytes()), num
        assert in_region(lens.tobytes()), num
    assert in_region(t["MP3D_QUAD_CODE"][0].tobytes()) and in_region(t["MP3D_QUAD_LEN"][0].tobytes())
    assert in_region(t["MP3D_SYNTH_WINDOW_Q16"].astype("<i4").tobytes())
    assert in_region(t["MP3D_PRETAB"].tobytes())
    # whole 9-rate blocks (MPEG-1 + LSF), as FFmpeg's band_size_long / _short
    assert in_region(t["MP3D_SFB_LONG_WIDTH"].tobytes())
    assert in_region(t["MP3D_SFB_SHORT_WIDTH"].tobytes())
    assert in_region(t["MP3D_LSF_NSF"].tobytes())  # FFmpeg lsf_nsf_table
    assert in_region(t["MP3D_BITRATE_L3"].astype("<u2").tobytes())
    assert in_region(t["MP3D_BITRATE_L3_LSF"].astype("<u2").tobytes())
    assert kb.find(t["MP3D_SLEN"].tobytes()) >= 0
    assert kb.find(t["MP3D_ALIAS_C"].astype("<f4").tobytes()) >= 0


def test_pow43_escape_recipe():
    """k_synth computes |is|^(4/3) for 256 <= |is| <= 8206 (escape values) without
    a table: y = exp2(log2(x) / 3), one Newton step on y^3 = x, times x
    (pow43_big in mp3d_synth.hip).  Emulated in float32 with the log/exp
    results perturbed by up to 3 ulp (the hardware v_log_f32 / v_exp_f32 are
    approximate), it stays within 2 ulp of the correctly rounded value."""
    a = np.arange(256, 8207)
    ref = (a.astype(np.float64) ** (4.0 / 3.0)).astype(np.float32)
    x = a.astype(np.float32)
    for pert in (-3, -1, 0, 1, 3):
        lg = (np.log2(x).astype(np.float32).view(np.int32) + pert).view(np.float32)
        y = np.exp2((lg * np.float32(1.0 / 3.0)).astype(np.float32)).astype(np.float32)
        y = (y.view(np.int32) - pert).view(np.float32)
        y2 = (y * y).astype(np.float32)
        r = (y2.astype(np.float64) * y - x).astype(np.float32)  # fmaf
        rc = (np.float32(1.0) / (np.float32(3.0) * y2)).astype(np.float32)
        y = (y - (r * rc).astype(np.float32)).astype(np.float32)
        p = (x * y).astype(np.float32)
        ulp = np.abs(p.view(np.int32).astype(np.int64) - ref.view(np.int32))
        assert ulp.max() <= 2, (pert, int(ulp.max()))


def test_kernel_literal_tables_match_recipe():
    """mp3_amd/csrc/mp3d_consts.h (the k_synth IMDCT-12 / short-window /
    alias coefficients compiled in as literals) is exactly what
    tools/gen_consts.py renders from the ISO formulas (the library also
    checks it against its own host recipe at init)."""
    import importlib.util
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("gen_consts", root / "tools" / "gen_consts.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert (root / "mp3_amd" / "csrc" / "mp3d_consts.h").read_text() == mod.render()
