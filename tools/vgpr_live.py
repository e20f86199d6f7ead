#!/usr/bin/env python3
"""Live VGPRs per instruction of one kernel, from its final assembly (a
register-pressure map for the occupancy work; diagnostic only).

Builds the basic blocks of the kernel, runs a backward liveness dataflow over
the architected VGPRs (a def under a partial EXEC is taken as a full kill, so
the counts are a lower bound there) and prints, per source line (-g line
tables), the largest live count seen at it, plus the hottest lines overall.

  python tools/vgpr_live.py [--src mp3d_synth.hip] [--kernel PREFIX] [--flags ...] [--top N]
"""
import argparse
import collections
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
BR = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+(\.\w+)")
# opcodes whose first operand is NOT a vector register def
NO_DEF = ("ds_write", "ds_store", "buffer_store", "global_store", "scratch_store", "flat_store", "v_cmp", "v_cmpx",
          "v_readlane", "v_readfirstlane", "s_", "ds_add_u32", "ds_add_u64", "buffer_atomic", "global_atomic")
BOTH = ("v_permlane32_swap", "v_permlane16_swap", "v_swap")


def regs(text):
    out = []
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(asm, kernel):
    lines = open(asm).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel) and re.match(r"^\S+:", l))
    insts, labels, loc, chain = [], {}, ("?", 0), ()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (files.get(m.group(1), "?"), int(m.group(2)))
            # the inlined-at chain in the comment: every (file, line) from the innermost out
            chain = tuple((f.split("/")[-1], int(n)) for f, n in re.findall(r"([\w./-]+):(\d+):\d+", l.split(";", 1)[-1]))
            continue
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = l.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        insts.append((s, loc, chain))
    return insts, labels


def analyse(insts, labels):
    n = len(insts)
    defs, uses, succ = [], [], []
    for i, (s, _, _) in enumerate(insts):
        op, _, rest = s.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        d, u = set(), set()
        if op.startswith(BOTH):
            for o in ops:
                d.update(regs(o))
                u.update(regs(o))
        elif ops and not op.startswith(NO_DEF) and (op.startswith("v_") or op.startswith(("ds_", "buffer_load",
                                                                                       "global_load", "scratch_load",
                                                                                       "flat_load"))):
            d.update(regs(ops[0]))
            for o in ops[1:]:
                u.update(regs(o))
        else:
            for o in ops:
                u.update(regs(o))
        defs.append(d)
        uses.append(u)
        m = BR.match(s)
        nx = []
        if m:
            tgt = labels.get(m.group(2))
            if tgt is not None:
                nx.append(tgt)
            if m.group(1) != "s_branch" and i + 1 < n:
                nx.append(i + 1)
        elif op not in ("s_endpgm", "s_setpc_b64") and i + 1 < n:
            nx.append(i + 1)
        succ.append(nx)
    live_in = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for i in range(n - 1, -1, -1):
            out = set()
            for j in succ[i]:
                out |= live_in[j]
            new = (out - defs[i]) | uses[i]
            if new != live_in[i]:
                live_in[i] = new
                changed = True
    return live_in, defs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="mp3d_synth.hip")
    ap.add_argument("--kernel", default="_ZN4mp3d7k_synthILb0ELb0ELb0EE")
    ap.add_argument("--flags", default="-fno-slp-vectorize")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--asm", default=None, help="use this .s instead of compiling")
    ap.add_argument("--phases", default="",
                    help="NAME:FIRST-LAST,... source line ranges of --src: the largest live count of the "
                         "instructions whose inlined-at chain passes through each range")
    ap.add_argument("--why", type=int, default=0,
                    help="at the hottest instruction of this source line: the live VGPRs by the source line of "
                         "their nearest preceding def")
    args = ap.parse_args()
    asm = args.asm
    if asm is None:
        asm = "/tmp/vgpr_live.s"
        src = args.src if os.path.isabs(args.src) else os.path.join(ROOT, "mp3_amd", "csrc", args.src)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-g",
                               "--cuda-device-only", "-S", "-o", asm, src] + args.flags.split(),
                              stderr=subprocess.DEVNULL)
    insts, labels = parse(asm, args.kernel)
    live, defs = analyse(insts, labels)
    per_line = collections.defaultdict(int)
    for (s, loc, _), lv in zip(insts, live):
        per_line[loc] = max(per_line[loc], len(lv))
    print("instructions %d, max live VGPRs %d" % (len(insts), max(len(x) for x in live)))
    if args.phases:
        src = os.path.basename(args.src)
        for ph in args.phases.split(","):
            name, rng = ph.split(":")
            a, b = (int(x) for x in rng.split("-"))
            sel = [len(lv) for (_, loc, ch), lv in zip(insts, live)
                   if any(f == src and a <= n <= b for f, n in (loc,) + ch)]
            print("phase %-4s lines %4d-%4d: %5d instructions, max live %3d" % (name, a, b, len(sel), max(sel or [0])))
    if args.why:
        cand = [i for i, (_, loc, _) in enumerate(insts) if loc[1] == args.why]
        i0 = max(cand, key=lambda i: len(live[i]))
        by = collections.Counter()
        for r in live[i0]:
            j = i0 - 1
            while j >= 0 and r not in defs[j]:
                j -= 1
            by[insts[j][1] if j >= 0 else ("entry", 0)] += 1
        print("at %s (live %d):" % (insts[i0][0], len(live[i0])))
        for loc, c in by.most_common():
            print("   %3d defined at %s:%d" % (c, loc[0], loc[1]))
    for loc, c in sorted(per_line.items(), key=lambda x: -x[1])[:args.top]:
        print("%4d  %s:%d" % (c, loc[0], loc[1]))


if __name__ == "__main__":
    main()
