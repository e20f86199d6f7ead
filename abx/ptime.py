#!/usr/bin/env python3
"""Build build_ab/PT.so: k_synth with per-phase cycle accounting (diagnostic; the
output is unchanged).  Each wave sums s_memtime deltas over its granules for
phases Q, I, M, W and the loop head, then adds them to g_ptime with one
global atomic per phase; mp3d_dbg_ptime() reads and clears them
(tools/dbg/synth_phase_times.py).  Usage: python abx/ptime.py"""
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mp3_amd import _build  # noqa: E402

Q = "            /* ---------------- phase Q: requantise + stereo -> LDS ---------- */"
I = "            /* ---------------- phase I: alias + IMDCT + overlap ------------ */"
M = "            /* ---------------- phase M: matrixing on the matrix cores ------- */"
W = "            /* ---------------- phase W: 512-tap window -> PCM --------------- */"
E = "            wave_sync(); /* X reads done before the next granule's xr */"
S = "    /* state out: the stream's last segment.  With several segments the"


def main():
    src = open("mp3_amd/csrc/mp3d_synth.hip").read()
    mark = os.environ.get("PT_MARK", "")
    reps = [
        ("namespace mp3d {\n", "namespace mp3d {\n__device__ unsigned long long g_ptime[8];\n"),
        ("    for (int f = fw; f < f1; f++) {\n",
         "    unsigned long long pt_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl_ = __builtin_amdgcn_s_memtime();\n"
         "    for (int f = fw; f < f1; f++) {\n"),
        (Q, "            unsigned long long tq_ = __builtin_amdgcn_s_memtime(); pt_[4] += tq_ - tl_;\n" + Q),
        (I, "            unsigned long long ti_ = __builtin_amdgcn_s_memtime(); pt_[0] += ti_ - tq_;\n" + I),
        (M, "            unsigned long long tm_ = __builtin_amdgcn_s_memtime(); pt_[1] += tm_ - ti_;\n" + M),
        (W, "            unsigned long long tw_ = __builtin_amdgcn_s_memtime(); pt_[2] += tw_ - tm_;\n" + W),
        (E, E + "\n            tl_ = __builtin_amdgcn_s_memtime(); pt_[3] += tl_ - tw_;"),
        (S, "    if ((threadIdx.x & 63) == 0 && !SRC_XR && PF == 0)\n"
            "        for (int k = 0; k < 8; k++) atomicAdd(&g_ptime[k], pt_[k]);\n" + S),
    ]
    if mark == "w":
        # slots 5, 6 split phase W instead: its vmcnt(0) drain, then the X /
        # tap loads (up to their lgkmcnt(0)); the rest of W = window + stores
        reps += [
            ("            if (!SRC_XR) WAIT_VMCNT0();\n",
             "            if (!SRC_XR) WAIT_VMCNT0();\n"
             "            unsigned long long tw1_ = __builtin_amdgcn_s_memtime(); pt_[5] += tw1_ - tw_;\n"),
            ("                xb17 = sBuf[pb + 17 * XROW];\n",
             "                xb17 = sBuf[pb + 17 * XROW];\n"
             "                __builtin_amdgcn_s_waitcnt(0xC07F);\n"
             "                unsigned long long tw2_ = __builtin_amdgcn_s_memtime(); pt_[6] += tw2_ - tw1_;\n"),
        ]
    else:
        # phase Q sub-marks (decode path): after the band scales, after the
        # requantise loop, after escapes + stereo (the rest of Q = scatter)
        reps += [
            ("                (void)m12a;\n",
             "                (void)m12a;\n                unsigned long long tq1_ = __builtin_amdgcn_s_memtime(); pt_[5] += tq1_ - tq_;\n"),
            ("                if (__ballot((bigacc & 0xF800F800u) != 0u)) {\n",
             "                unsigned long long tq2_ = __builtin_amdgcn_s_memtime(); pt_[6] += tq2_ - tq1_;\n"
             "                if (__ballot((bigacc & 0xF800F800u) != 0u)) {\n"),
        ]
        if mark == "prefetch":  # the last Q sub-mark after the next granule's prefetch is issued
            reps.append(("                /* scatter in (short-block reordered) position; M/S-only frames\n",
                         "                pt_[7] += __builtin_amdgcn_s_memtime() - tq2_;\n"
                         "                /* scatter in (short-block reordered) position; M/S-only frames\n"))
        else:
            reps.append(("                /* the next granule's loads fly during phases I, M, W (issued\n",
                         "                pt_[7] += __builtin_amdgcn_s_memtime() - tq2_;\n"
                         "                /* the next granule's loads fly during phases I, M, W (issued\n"))
    for a, b in reps:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    src += ("\nnamespace mp3d {\nhipError_t dbg_ptime(unsigned long long *out) {\n"
            "    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptime), 8 * 8);\n"
            "    unsigned long long z[8] = {};\n    if (!e) e = hipMemcpyToSymbol(HIP_SYMBOL(g_ptime), z, 8 * 8);\n"
            "    return e;\n}\n}\n")
    host = open("mp3_amd/csrc/mp3d_host.cpp").read()
    host += ("\nnamespace mp3d { hipError_t dbg_ptime(unsigned long long *); }\n"
             "extern \"C\" __attribute__((visibility(\"default\"))) int mp3d_dbg_ptime(unsigned long long *o) "
             "{ return mp3d::dbg_ptime(o) ? -1 : 0; }\n")
    d = "/tmp/vars/PT"
    os.makedirs(d, exist_ok=True)
    for h in _build.HIP_HDRS:
        shutil.copy("mp3_amd/csrc/" + h, d)
    for k in ("mp3d_demux.hip", "mp3d_huffman.hip"):
        shutil.copy("mp3_amd/csrc/" + k, d)
    open(d + "/mp3d_synth.hip", "w").write(src)
    open(d + "/mp3d_host.cpp", "w").write(host)
    os.makedirs(d + "/../../include", exist_ok=True)
    shutil.copy("include/mp3d.h", d + "/../../include/")
    out = {"prefetch": "build_ab/PT2.so", "w": "build_ab/PTW.so"}.get(mark, "build_ab/PT.so")
    _build.compile_hip(d, out, d + "/obj")
    print(out)


if __name__ == "__main__":
    main()
