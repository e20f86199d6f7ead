"""The committed golden fixtures are reproducible:
hashes.json pins every fixture file by sha256, and the seeded generator
(mp3_amd/csrc/mp3gen.c) still rebuilds every generated stream -- the plain
ones of make_golden.py / make_lsf_golden.py and the edited ones of
make_edge_golden.py -- byte for byte, so re-running those scripts (which
also re-decode with FFmpeg, in the build container only) regenerates exactly
what is committed.  No FFmpeg here: only the inputs are rebuilt."""
import hashlib
import json
import pathlib
import sys

import pytest

import _gen
import _golden

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))


def test_every_fixture_hashed():
    hashes = json.loads((GOLDEN / "hashes.json").read_text())
    files = sorted(p.name for p in GOLDEN.iterdir() if p.suffix in (".mp3", ".npy"))
    assert sorted(hashes) == files
    for name in files:
        assert hashlib.sha256((GOLDEN / name).read_bytes()).hexdigest() == hashes[name], name


@pytest.mark.parametrize("name", [n for n, e in sorted(_golden.manifest().items()) if "cfg" in e])
def test_generated_stream_reproduces(name):
    e = _golden.manifest()[name]
    data, offs = _gen.stream(e["cfg"], e["seed"], e.get("gen_frames", e["frames"]))
    if "gen_frames" in e:  # the first `frames` frames of a longer stream
        data = data[:int(offs[e["frames"]])]
    assert data == (GOLDEN / (name + ".mp3")).read_bytes()


def test_edge_streams_reproduce():
    import make_edge_golden  # builds the edited streams; FFmpeg is not touched here
    for name, (data, hz, nch) in make_edge_golden.cases().items():
        assert data == (GOLDEN / (name + ".mp3")).read_bytes(), name
        e = _golden.manifest()[name]
        assert e["hz"] == hz and e["nch"] == nch and e["bytes"] == len(data)
