"""Golden-vector generator: FFmpeg's MPEG-audio decoder (inside Chromium 88,
statically linked in the container's kaleido binary) driven through WebAudio
`OfflineAudioContext.decodeAudioData`.

Runs ONLY in the build container (needs kaleido); its outputs are committed as
small .npy fixtures under tests/golden/ so nothing here travels to the GPU box.
The decoder is a third-party CPU decoder used as an independent checker.
"""
import base64
import json
import pathlib

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
_scope = None


def _get_scope():
    global _scope
    if _scope is None:
        from kaleido.scopes.plotly import PlotlyScope
        _scope = PlotlyScope(
            plotlyjs=str(_HERE / "ffmpeg_stub.js"),
            chromium_args=("--disable-gpu", "--allow-file-access-from-files", "--disable-breakpad",
                           "--disable-dev-shm-usage", "--no-sandbox", "--single-process"))
    return _scope


def decode(mp3_bytes: bytes, sample_rate: int, nch: int = 2) -> np.ndarray:
    """Return float32 PCM [nch, n] as FFmpeg's float decoder produced it."""
    meta = {"mp3": base64.b64encode(mp3_bytes).decode(), "sr": int(sample_rate), "nch": int(nch)}
    r = _get_scope().transform({"data": [], "layout": {"meta": meta}}, format="json")
    j = json.loads(r)
    if "error" in j:
        raise RuntimeError("oracle decode failed: %s" % j["error"])
    if int(j["sr"]) != int(sample_rate):
        raise RuntimeError("oracle resampled (%s != %s)" % (j["sr"], sample_rate))
    return np.stack([np.frombuffer(base64.b64decode(c), dtype="<f4") for c in j["ch"]])
