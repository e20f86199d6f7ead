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


# per-file code generation flags.  k_synth without the SLP vectorizer: its
# packed pairs are written explicitly (f32x2 window FMAs); the vectorizer's
# extra pairings cost moves, SGPR spills and +2.7 % k_synth time, while
# k_demux is 6.7 % faster WITH it (A/B NOSLP, profiles/r02_ab.txt).
FILE_FLAGS = {"mp3d_synth.hip": ["-fno-slp-vectorize"]}
HIP_SRCS = ["mp3d_demux.hip", "mp3d_huffman.hip", "mp3d_synth.hip", "mp3d_host.cpp"]
HIP_HDRS = ["mp3d_internal.h", "mp3d_tables.h", "mp3d_consts.h", "mp3d_device.h", "mp3d_hostparse.h",
            "mp3d_demux_dev.h", "mp3d_huffman_dev.h"]


def compile_hip(src_dir, out, obj_dir, extra=()):
    """Each source to an object (its FILE_FLAGS), in parallel, then one link."""
    src_dir, obj_dir = pathlib.Path(src_dir), pathlib.Path(obj_dir)
    obj_dir.mkdir(parents=True, exist_ok=True)
    base = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall"]
    procs, objs = [], []
    for name in HIP_SRCS:
        obj = obj_dir / (name + ".o")
        objs.append(str(obj))
        cmd = base + FILE_FLAGS.get(name, []) + list(extra) + ["-c", "-o", str(obj), str(src_dir / name)]
        procs.append((cmd, subprocess.Popen(cmd)))
    for cmd, p in procs:
        if p.wait():
            raise subprocess.CalledProcessError(p.returncode, cmd)
    pathlib.Path(out).parent.mkdir(parents=True, exist_ok=True)
    subprocess.check_call([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", str(out)] + objs)
    return out


def build_hip(force=False):
    out = ROOT / "mp3_amd" / "libmp3d.so"
    deps = [CSRC / n for n in HIP_SRCS + HIP_HDRS] + [ROOT / "include" / "mp3d.h", pathlib.Path(__file__)]
    if force or _stale(out, deps):
        compile_hip(CSRC, out, ROOT / "mp3_amd" / "_obj")
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
