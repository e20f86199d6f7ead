"""Build the native libraries in-tree (hipcc for gfx950; gcc for CPU tools).

  mp3_amd/libmp3d.so    HIP kernels + C ABI (the product)
  mp3_amd/libmp3gen.so  synthetic stream generator (bench/test input)
  oracle/liboracle.so   CPU restatement (test infrastructure only)
"""
import os
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "mp3_amd" / "csrc"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MP3D_ARCH", "gfx950")


def _stale(target, deps):
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_hip(force=False):
    out = ROOT / "mp3_amd" / "libmp3d.so"
    srcs = [CSRC / "mp3d_demux.hip", CSRC / "mp3d_huffman.hip", CSRC / "mp3d_synth.hip", CSRC / "mp3d_host.cpp"]
    deps = srcs + [CSRC / "mp3d_internal.h", CSRC / "mp3d_tables.h", CSRC / "mp3d_consts.h", CSRC / "mp3d_device.h",
                   CSRC / "mp3d_hostparse.h",
                   ROOT / "include" / "mp3d.h"]
    if force or _stale(out, deps):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-fPIC", "-shared", "-std=c++17", "-fvisibility=hidden",
               "-Wall", "-o", str(out)] + [str(s) for s in srcs]
        subprocess.check_call(cmd)
    return out


def build_gen(force=False):
    out = ROOT / "mp3_amd" / "libmp3gen.so"
    deps = [CSRC / "mp3gen.c", CSRC / "mp3d_tables.h"]
    if force or _stale(out, deps):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-fvisibility=hidden", "-o", str(out),
                               str(CSRC / "mp3gen.c"), "-lm"])
    return out


def build_oracle(force=False):
    out = ROOT / "oracle" / "liboracle.so"
    deps = [ROOT / "oracle" / "mp3_oracle.c", CSRC / "mp3d_tables.h"]
    if force or _stale(out, deps):
        subprocess.check_call(["make", "-s", "-B" if force else "-s", "-C", str(ROOT / "oracle")])
    return out


def build_examples(force=False):
    """examples/mp3d_play: the player's decode loop in C over the C ABI."""
    out = ROOT / "examples" / "mp3d_play"
    deps = [ROOT / "examples" / "mp3d_play.c", ROOT / "include" / "mp3d.h", ROOT / "mp3_amd" / "libmp3d.so"]
    if force or _stale(out, deps):
        subprocess.check_call(["make", "-s", "-B", "-C", str(ROOT / "examples")])
    return out


def build_all(force=False):
    build_hip(force)
    build_gen(force)
    build_oracle(force)
    build_examples(force)


if __name__ == "__main__":
    build_all(force=True)
