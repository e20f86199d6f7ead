"""examples/mp3d_play.c: a plain-C host program over the C ABI (the player's
decode loop) builds, links against libmp3d.so, fails loudly
without a GPU, and on the GPU reproduces FFmpeg's PCM for the real 128 kbps
file (untrimmed, and with the LAME gapless trim)."""
import subprocess
import wave

import numpy as np
import pytest

import _golden
from mp3_amd import _build


def _run(args):
    exe = _build.build_examples()
    return subprocess.run([str(exe)] + [str(a) for a in args], capture_output=True, text=True, timeout=120)


def _wav(path):
    with wave.open(str(path)) as w:
        pcm = np.frombuffer(w.readframes(w.getnframes()), "<i2").reshape(-1, w.getnchannels()).T
        return pcm, w.getframerate()


def test_example_builds_and_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    r = _run([_golden.GOLDEN / "keypress_128k_js.mp3", tmp_path / "o.wav"])
    assert r.returncode == 2 and "no usable HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("gapless", [False, True])
def test_example_decodes_keypress(tmp_path, gapless):
    data, ref = _golden.case("keypress_128k_js")
    if gapless:
        ref = np.load(_golden.GOLDEN / "keypress_128k_js.tagged.pcm16.npy")
    out = tmp_path / "o.wav"
    r = _run([_golden.GOLDEN / "keypress_128k_js.mp3", out] + (["--gapless"] if gapless else []))
    assert r.returncode == 0, r.stderr
    pcm, hz = _wav(out)
    assert hz == 44100 and pcm.shape == ref.shape, (pcm.shape, ref.shape)
    assert np.abs(pcm.astype(np.int32) - ref.astype(np.int32)).max() <= 1
