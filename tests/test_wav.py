"""WAV sink (mp3_amd/wav.py): int16 PCM readable by the standard library's
wave module; float32 written as IEEE float with a fact chunk."""
import io
import wave

import numpy as np

from mp3_amd import wav


def test_int16_roundtrip_stdlib(tmp_path):
    rng = np.random.default_rng(5)
    pcm = rng.integers(-32768, 32767, (2, 1000), dtype=np.int16)
    p = tmp_path / "a.wav"
    wav.write(p, pcm, 44100)
    with wave.open(str(p)) as w:
        assert w.getnchannels() == 2 and w.getframerate() == 44100 and w.getsampwidth() == 2
        got = np.frombuffer(w.readframes(1000), "<i2").reshape(-1, 2).T
    assert np.array_equal(got, pcm)
    back, hz = wav.read(p)
    assert hz == 44100 and np.array_equal(back, pcm)


def test_float32_mono(tmp_path):
    pcm = np.linspace(-1.2, 1.2, 777, dtype=np.float32)[None]
    p = tmp_path / "f.wav"
    n = wav.write(p, pcm, 48000)
    blob = p.read_bytes()
    assert n == len(blob) and blob[:4] == b"RIFF" and b"fact" in blob
    back, hz = wav.read(p)
    assert hz == 48000 and back.dtype == np.float32 and np.array_equal(back, pcm)


def test_rejects_bad_shapes():
    import pytest
    with pytest.raises(ValueError):
        wav.wav_bytes(np.zeros((3, 10), np.int16), 44100)
    with pytest.raises(TypeError):
        wav.wav_bytes(np.zeros((2, 10), np.int32), 44100)
    buf = io.BytesIO()
    wav.write(buf, np.zeros((1, 4), np.int16), 32000)
    assert buf.getvalue()[8:12] == b"WAVE"
