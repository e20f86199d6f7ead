#!/usr/bin/env python3
"""Build build_ab/HT.so: k_huffman with per-stage cycle accounting (diagnostic;
the output is unchanged).  Each wave sums s_memtime deltas of: ranking,
round set-up, staging, scalefactors, big_values, count1, meta stores; lane
0 adds them to g_htime with one global atomic per stage at the end;
mp3d_dbg_ptime() reads and clears them (tools/dbg/huff_stage_times.py).
Usage: python abx/htime.py"""
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mp3_amd import _build  # noqa: E402

T = "__builtin_amdgcn_s_memtime()"


def main():
    src = open("mp3_amd/csrc/mp3d_huffman.hip").read()
    reps = [
        ("namespace mp3d {\n", "namespace mp3d {\n__device__ unsigned long long g_htime[8];\n", 1),
        ("    const int n_super = (n_units + HUFF_SUPER - 1) / HUFF_SUPER;\n",
         "    const int n_super = (n_units + HUFF_SUPER - 1) / HUFF_SUPER;\n"
         "    unsigned long long ht_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tm_ = 0, tx_ = 0;\n", 1),
        ("        const int ubase = sc * HUFF_SUPER;\n", "        tm_ = %s;\n        const int ubase = sc * HUFF_SUPER;\n" % T, 1),
        ("        for (int rd = 0; rd < HUFF_ROUNDS; rd++) {\n",
         "        tx_ = %s; ht_[0] += tx_ - tm_;\n        for (int rd = 0; rd < HUFF_ROUNDS; rd++) {\n"
         "            tm_ = %s;\n" % (T, T), 1),
        ("            bool pending = dec;\n", "            tx_ = %s; ht_[1] += tx_ - tm_;\n            bool pending = dec;\n" % T, 1),
        ("            while (__ballot(pending)) {\n", "            while (__ballot(pending)) {\n                tm_ = %s;\n" % T, 1),
        ("                if (inb) {\n                    const uint32_t seg",
         "                tx_ = %s; ht_[2] += tx_ - tm_; tm_ = tx_;\n                if (inb) {\n                    const uint32_t seg" % T, 1),
        ("                    /* big_values: region boundaries",
         "                    tx_ = %s; ht_[3] += tx_ - tm_; tm_ = tx_;\n                    /* big_values: region boundaries" % T, 1),
        ("                    k = bv2;\n", "                    tx_ = %s; ht_[4] += tx_ - tm_; tm_ = tx_;\n                    k = bv2;\n" % T, 1),
        ("                    const int nz_end = k;\n",
         "                    tx_ = %s; ht_[5] += tx_ - tm_; tm_ = tx_;\n                    const int nz_end = k;\n" % T, 1),
        ("                    /* everything after sf[40]: one 16-B store */\n",
         "                    tx_ = %s; ht_[7] += tx_ - tm_; tm_ = tx_;\n                    /* everything after sf[40]: one 16-B store */\n" % T, 1),
        ("                pending = pending && !inb;\n",
         "                tx_ = %s; ht_[6] += tx_ - tm_;\n                pending = pending && !inb;\n" % T, 1),
        ("    }\n}\n\n/* k_huffman_wave",
         "    }\n    if (lane == 0)\n        for (int k = 0; k < 8; k++) atomicAdd(&g_htime[k], ht_[k]);\n}\n\n/* k_huffman_wave", 1),
    ]
    for a, b, n in reps:
        assert src.count(a) == n, a
        src = src.replace(a, b)
    src += ("\nnamespace mp3d {\nhipError_t dbg_htime(unsigned long long *out) {\n"
            "    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_htime), 8 * 8);\n"
            "    unsigned long long z[8] = {};\n    if (!e) e = hipMemcpyToSymbol(HIP_SYMBOL(g_htime), z, 8 * 8);\n"
            "    return e;\n}\n}\n")
    host = open("mp3_amd/csrc/mp3d_host.cpp").read()
    host += ("\nnamespace mp3d { hipError_t dbg_htime(unsigned long long *); }\n"
             "extern \"C\" __attribute__((visibility(\"default\"))) int mp3d_dbg_ptime(unsigned long long *o) "
             "{ return mp3d::dbg_htime(o) ? -1 : 0; }\n")
    d = "/tmp/vars/HT"
    os.makedirs(d, exist_ok=True)
    for h in _build.HIP_HDRS:
        shutil.copy("mp3_amd/csrc/" + h, d)
    for k in ("mp3d_demux.hip", "mp3d_synth.hip"):
        shutil.copy("mp3_amd/csrc/" + k, d)
    open(d + "/mp3d_huffman.hip", "w").write(src)
    open(d + "/mp3d_host.cpp", "w").write(host)
    os.makedirs(d + "/../../include", exist_ok=True)
    shutil.copy("include/mp3d.h", d + "/../../include/")
    _build.compile_hip(d, "build_ab/HT.so", d + "/obj")
    print("build_ab/HT.so")


if __name__ == "__main__":
    main()
