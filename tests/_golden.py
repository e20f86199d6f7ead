"""Access to the committed golden fixtures (tests/golden/)."""
import json
import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def manifest():
    return json.loads((GOLDEN / "manifest.json").read_text())


def case(name):
    data = (GOLDEN / (name + ".mp3")).read_bytes()
    pcm = np.load(GOLDEN / (name + ".pcm16.npy"))
    return data, pcm


def names():
    return sorted(manifest().keys())


def to_int16(x):
    return np.clip(np.rint(np.asarray(x, np.float64) * 32768.0), -32768, 32767).astype(np.int16)
