"""ASan + UBSan over the C/C++ CPU code (SURVEY.md §5 "race detection /
sanitizers"): the library's host-side byte parsing
(mp3_amd/csrc/mp3d_hostparse.h -- walk_frames, long_plan, the per-frame
frame search) and the CPU oracle (oracle/mp3_oracle.c), each built with
-fsanitize=address,undefined into tests/native/_build and run over a fuzz
corpus: random bytes with sync words / ID3 headers of both MPEG families,
generator streams (MPEG-1, mixed corpus, LSF, CRC) cut at random points, and
every golden fixture.  Every stream is an exact-size heap copy, so a read
past its end is an ASan error.  The GPU kernels are not covered here (GPU
sanitizers are unavailable on the pool); k_demux's reads are bounded by
construction (mp3d_demux.hip load_win) and tested on the GPU
(tests/test_gpu_state.py::test_unaligned_stream_ends_read_exactly)."""
import os
import pathlib
import shutil
import struct
import subprocess

import numpy as np
import pytest

import _gen
import _golden

ROOT = pathlib.Path(__file__).resolve().parents[1]
NATIVE = ROOT / "tests" / "native"
OUT = NATIVE / "_build"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
ENV.pop("LD_PRELOAD", None)


def _build(name, compiler, src, extra):
    if shutil.which(compiler) is None:
        pytest.skip("%s not available" % compiler)
    OUT.mkdir(exist_ok=True)
    exe = OUT / name
    subprocess.check_call([compiler] + SAN + extra + ["-o", str(exe), str(src)] + (["-lm"] if compiler == "gcc" else []))
    return exe


def _corpus(path, n_garbage=120, oracle=False):
    rng = np.random.default_rng(2024)
    recs = []
    for s in range(n_garbage):
        n = int(rng.integers(0, 2500))
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        for _ in range(int(rng.integers(0, 16))):
            if n < 8:
                break
            p = int(rng.integers(0, n - 4))
            b[p:p + 3] = bytes([0xFF, int(rng.choice([0xFB, 0xFA, 0xF3, 0xF2, 0xE3, 0xE2])),
                                int(rng.integers(0, 256)) & 0xFD])
        if s % 7 == 0 and n > 12:
            b[:3] = b"ID3"
        recs.append(bytes(b))
    lsf = dict(_gen.C5, sr_idx=-2, short_pct=30, mixed_pct=40)
    for k, cfg in enumerate([_gen.C3, _gen.C5, lsf, dict(_gen.C3, crc_pct=100)]):
        for s in range(6 if oracle else 12):
            data, _ = _gen.stream(cfg, 9_000_000 + 100 * k + s, 6)
            cut = int(rng.integers(0, len(data) + 1))
            recs += [data, data[:cut], data[cut // 2:]]
    for name in _golden.names():
        data, _ = _golden.case(name)
        recs.append(data)
        recs.append(data[: len(data) - 3])
    with open(path, "wb") as f:
        for r in recs:
            f.write(struct.pack("<I", len(r)))
            f.write(r)
    return len(recs)


def _run(exe, corpus):
    p = subprocess.run([str(exe), str(corpus)], env=ENV, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


def test_host_parsing_under_asan_ubsan(tmp_path):
    exe = _build("host_fuzz", "g++", NATIVE / "host_fuzz.cpp", ["-std=c++17", "-I", str(ROOT / "mp3_amd" / "csrc")])
    corpus = tmp_path / "corpus.bin"
    n = _corpus(corpus)
    out = _run(exe, corpus)
    assert ("%d records" % n) in out


def test_oracle_under_asan_ubsan(tmp_path):
    exe = _build("oracle_fuzz", "gcc", NATIVE / "oracle_fuzz.c", ["-std=gnu11"])
    corpus = tmp_path / "corpus.bin"
    n = _corpus(corpus, n_garbage=60, oracle=True)
    out = _run(exe, corpus)
    assert ("%d records" % n) in out
