#!/usr/bin/env python3
"""Basic blocks of one kernel with their instruction mix, source lines and
branches (static; -g line tables) -- the companion of tools/asm_attr.py for
following a kernel's common path by hand.

  python tools/asm_blocks.py [--src mp3d_synth.hip] [--kernel SYMBOL_PREFIX] [--min-valu N]
"""
import argparse
import collections
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="mp3d_synth.hip")
    ap.add_argument("--kernel", default="_ZN4mp3d7k_synthILb0ELb0ELb0EE")
    ap.add_argument("--flags", default="-fno-slp-vectorize")
    ap.add_argument("--min-valu", type=int, default=0)
    args = ap.parse_args()
    src = os.path.join(ROOT, "mp3_amd", "csrc", args.src)
    asm = "/tmp/asm_blocks.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-g",
                           "--cuda-device-only", "-S", "-o", asm, src] + args.flags.split(), stderr=subprocess.DEVNULL)
    text = open(asm).read().split("\n")
    files, start = {}, None
    for n, l in enumerate(text):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
        if start is None and l.startswith(args.kernel) and re.match(r"^\S+:", l):
            start = n
    blocks, cur, loc = [], ["entry", [], collections.Counter(), []], ("?", 0)
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), [], collections.Counter(), []]
            continue
        s = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if s and not s.startswith((".", ";")):
            op = s.split()[0]
            cur[1].append(op)
            if op.startswith(("s_cbranch", "s_branch")):
                cur[3].append(s)
            if loc[0] == args.src:
                cur[2][loc[1]] += 1
    blocks.append(cur)
    for name, ops, lc, br in blocks:
        v = sum(o.startswith("v_") and not o.startswith("v_mfma") for o in ops)
        if v < args.min_valu and not br:
            continue
        cnt = lambda p: sum(o.startswith(p) for o in ops)  # noqa: E731
        lines = sorted(k for k in lc if k > 0)
        print("%-10s v=%4d pk=%3d mov=%3d mf=%2d s=%3d ds=%3d vm=%3d L%s-%s %s" % (
            name, v, cnt("v_pk"), cnt("v_mov"), cnt("v_mfma"), cnt("s_"), cnt("ds_"), cnt(("buffer", "global")),
            lines[0] if lines else "-", lines[-1] if lines else "-", " | ".join(br)))


if __name__ == "__main__":
    main()
