#!/usr/bin/env python3
"""How often does a big_values pair need k_huffman's second LUT level?  For
generator C3 streams: each pair's Huffman code length (ISO tables, from
mp3d_tables.h via a small host helper compiled here) in the unit's region
table, then, over 64-unit rounds in k_rank's order (each 4 096-unit segment
by descending big_values), the share of pair steps in which at least one
lane's code is longer than a first level of b1 bits.  CPU only.
Usage: python tools/dbg/codelen_stats.py [N_STREAMS]"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gen  # noqa: E402
import _sideinfo  # noqa: E402

DUMP = r'''
#include <cstdio>
#include <cstdint>
#include "mp3d_tables.h"
int main() {
    printf("{\"rowlen\": [");
    for (int t = 0; t < MP3D_NUM_HTABS; t++) printf("%s%d", t ? "," : "", MP3D_HTAB_ROWLEN[t]);
    printf("], \"of_select\": [");
    for (int i = 0; i < 32; i++) printf("%s%d", i ? "," : "", MP3D_HTAB_OF_SELECT[i]);
    printf("], \"lens\": [");
    for (int t = 0; t < MP3D_NUM_HTABS; t++) {
        const int n = MP3D_HTAB_ROWLEN[t];
        printf("%s[", t ? "," : "");
        for (int i = 0; i < n * n; i++) printf("%s%d", i ? "," : "", MP3D_HTAB_LENS[t][i]);
        printf("]");
    }
    printf("]}\n");
}
'''


def tables():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "dump.cpp"), os.path.join(d, "dump")
        open(src, "w").write(DUMP)
        subprocess.check_call(["g++", "-std=c++17", "-I", os.path.join(ROOT, "mp3_amd", "csrc"), "-o", exe, src])
        return json.loads(subprocess.check_output([exe]))


def main(ns):
    t = tables()
    lens, rl, osel = [np.array(v) for v in t["lens"]], t["rowlen"], t["of_select"]
    units = []
    for s in range(ns):
        data, _, tr = _gen.stream(_gen.C3, 3_000_003 + s, 32, truth=True)
        data = bytes(data)
        for f, (off, h) in enumerate(_sideinfo.frames(data)):
            si = _sideinfo.side_info(data, off, h)
            for gr in range(2):
                for ch in range(2):
                    u, isv = si["units"][gr][ch], np.abs(tr[f, gr, ch]["is"].astype(np.int32))
                    end = 2 * u["big_values"]
                    if u["window_switching"]:
                        r1, r2 = 36, 576
                    else:
                        sfb = _sideinfo.SFB_LONG[h["hz"]]
                        r1 = sfb[min(u["region0_count"] + 1, 22)]
                        r2 = sfb[min(u["region0_count"] + u["region1_count"] + 2, 22)]
                    r1, r2 = min(r1, end), min(r2, end)
                    cl = []
                    for k in range(0, end, 2):
                        ti = osel[u["table_select"][0 if k < r1 else (1 if k < r2 else 2)]]
                        n = rl[ti] if ti >= 0 else 0
                        cl.append(0 if ti < 0 else lens[ti][min(isv[k], 15) * n + min(isv[k + 1], 15)])
                    units.append(np.array(cl, dtype=np.int32))
    every = np.concatenate([u for u in units if len(u)])
    order = []
    for s0 in range(0, len(units), 4096):
        order += sorted(range(s0, min(s0 + 4096, len(units))), key=lambda i: -len(units[i]))
    print("units %d, big_values pairs %d" % (len(units), len(every)))
    for b1 in (8, 9, 10, 11, 12):
        steps = need = 0
        for g0 in range(0, len(order), 64):
            grp = [units[i] for i in order[g0:g0 + 64]]
            for k in range(max(len(u) for u in grp)):
                steps += 1
                need += any(len(u) > k and u[k] > b1 for u in grp)
        print("first level %2d bits: pairs with a longer code %.3f, pair steps needing level 2 %.3f"
              % (b1, (every > b1).mean(), need / max(steps, 1)))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
