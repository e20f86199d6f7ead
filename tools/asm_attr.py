#!/usr/bin/env python3
"""Static instruction attribution of a kernel by source region (-g line tables).

  python tools/asm_attr.py [--kernel k_synth\\<false,false,false\\>] [--src mp3d_synth.hip] [--asm FILE]

Compiles mp3_amd/csrc/<src> for gfx950 to assembly with line tables (the
product's flags), takes the named kernel's body and counts its instructions
per class (VALU, packed FMA, MFMA, SALU, LDS, VMEM, wait) per source region.
Regions are the phase markers of k_synth (Q / I / M / W), the rare paths
inside them (escapes, intensity stereo, short-block IMDCT, non-long band
scales) and everything else (prologue, state in / out, tables).  The counts
are static: the granule loop is unrolled twice (two granules per frame), so
the per-granule figure of a region on the common path is its count / 2.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mp3_amd", "csrc")


def regions_synth(path):
    """source line ranges of k_synth's phases and rare paths, found by markers"""
    lines = open(path).read().split("\n")

    def find(s, start=0):
        for i in range(start, len(lines)):
            if s in lines[i]:
                return i + 1
        raise SystemExit("marker not found: " + s)

    q = find("phase Q: requantise + stereo")
    i_ = find("phase I: alias + IMDCT + overlap")
    m = find("phase M: matrixing on the matrix cores")
    w = find("phase W: 512-tap window -> PCM")
    wend = find("state out: the stream's last segment", w)
    esc = find("rare path (escapes |is| >= 256)", q)
    isb = find("if (is_on) {", q)
    ism = find("the next granule's loads fly during phases I, M, W", isb)
    bsl = find("const bool lng = lane < 22;", q)
    bsl_end = find("Wd.scale[1][lane] = band_scale", bsl)
    shi = find("/* z[6w+6+i] += y_w[i] * win12[i], w = 0..2, i = 0..11 */", i_)
    shi_end = find("if (PF == 1) { /* granule 0's overlap for the other wave */", shi)
    dct = find("__device__ __forceinline__ void dct3_9p(")
    imd_end = find("/* 36-point IMDCT of one subband's 18 lines")
    return [
        ("Q.rare:escape", esc, isb - 1),
        ("Q.rare:intensity", isb, ism - 1),
        ("Q.rare:band_scale_short", bsl, bsl_end),
        ("I.rare:short_imdct", shi, shi_end - 1),
        ("Q", q, i_ - 1),
        ("I", i_, m - 1),
        ("I.dct", dct, imd_end - 1),
        ("M", m, w - 1),
        ("W", w, wend - 1),
    ]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_fma") or op.startswith("v_pk_mul") or op.startswith("v_pk_add"):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op == "s_waitcnt" or op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop") or op.startswith("s_setprio") or op.startswith("s_barrier"):
        return "misc"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("buffer_") or op.startswith("global_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "vmem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="mp3d_synth.hip")
    ap.add_argument("--kernel", default="_ZN4mp3d7k_synthILb0ELb0ELb0EE")
    ap.add_argument("--asm", default=None, help="existing .s (skips the compile)")
    ap.add_argument("--flags", default="-fno-slp-vectorize")
    args = ap.parse_args()
    src = os.path.join(CSRC, args.src)
    asm = args.asm
    if asm is None:
        asm = "/tmp/asm_attr.s"
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-g",
                               "--cuda-device-only", "-S", "-o", asm, src] + args.flags.split(),
                              stderr=subprocess.DEVNULL)
    text = open(asm).read().split("\n")
    files = {}
    start = None
    for n, l in enumerate(text):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2))
        if start is None and l.startswith(args.kernel) and re.match(r"^\S+:", l):
            start = n
    if start is None:
        raise SystemExit("kernel not found: " + args.kernel)
    regs = regions_synth(src) if args.src == "mp3d_synth.hip" else []
    base = os.path.basename(src)
    counts = collections.defaultdict(collections.Counter)
    cur = ("?", 0)
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if not s or s.startswith(".") or s.startswith(";") or s.endswith(":"):
            continue
        op = s.split()[0]
        reg = "other"
        if os.path.basename(cur[0]) == base:
            for name, a, b in regs:
                if a <= cur[1] <= b:
                    reg = name
                    break
        elif cur[0] != "?":
            reg = "other:" + os.path.basename(cur[0])
        counts[reg][classify(op)] += 1
    cls = ["valu", "valu_pk", "mfma", "salu", "lds", "vmem", "wait", "misc", "other"]
    print("%-26s" % "region" + "".join("%9s" % c for c in cls))
    tot = collections.Counter()
    for r in sorted(counts):
        tot.update(counts[r])
        print("%-26s" % r + "".join("%9d" % counts[r][c] for c in cls))
    print("%-26s" % "TOTAL" + "".join("%9d" % tot[c] for c in cls))


if __name__ == "__main__":
    sys.exit(main())
