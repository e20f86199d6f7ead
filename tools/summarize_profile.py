#!/usr/bin/env python3
"""Condense a tools/profile.sh run (gpurun_out/prof_TAG/) into committed
summaries under profiles/:

  profiles/TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/TAG_pmc.json           per-kernel PMC counters (mean per dispatch)
  profiles/pmc_traffic.json       HBM bytes per k_synth launch for bench.py

HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores.
Usage: python tools/summarize_profile.py TAG [--streams N --frames F]
"""
import argparse
import collections
import csv
import json
import pathlib
import shutil

ROOT = pathlib.Path(__file__).resolve().parents[1]


def counters(d):
    rows = list(csv.DictReader(open(d / "run_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = r["Kernel_Name"]
        if "mp3d::" not in name:
            continue
        k = name.split("(")[0].replace("void ", "").replace("mp3d::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
            # the launch's mean engine clock: GRBM_GUI_ACTIVE is summed over the
            # 8 XCDs (MI355X_MICROARCH.md DVFS note), timestamps in ns
            dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if dt > 0:
                agg[k]["clock_mhz"].append(float(r["Counter_Value"]) / 8.0 / dt * 1e3)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--config", default="c3", help="key of the entry in profiles/pmc_traffic.json")
    a = ap.parse_args()
    src = ROOT / "gpurun_out" / ("prof_" + a.tag)
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    shutil.copy(src / "stats" / "run_kernel_stats.csv", dst / (a.tag + "_kernel_stats.csv"))
    out = {}
    for p in ("pmc_sq1", "pmc_sq2", "pmc_fetch", "pmc_write", "pmc_mfma"):
        if not (src / p / "run_counter_collection.csv").exists():
            continue
        for k, cs in counters(src / p).items():
            out.setdefault(k, {}).update(cs)
    for k, cs in out.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            cs["hbm_bytes_per_launch"] = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024.0
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and cs.get("GRBM_GUI_ACTIVE"):
            # rocprofv3's MfmaUtil: MFMA busy cycles summed over the 1 024 SIMDs
            # / (per-XCD GRBM_GUI_ACTIVE x SIMDs); GRBM_GUI_ACTIVE as collected
            # here is the sum over the 8 XCDs (MI355X_MICROARCH.md, DVFS note)
            cs["mfma_util"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cs["GRBM_GUI_ACTIVE"] / 8.0 * 1024)
            cs["mfma_f32_flop_per_launch"] = cs.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) * 512
    (dst / (a.tag + "_pmc.json")).write_text(json.dumps(out, indent=1, sort_keys=True))
    # the MPEG-1 int16 decode variant (k_synth<SRC_XR=false, F32=false, LSF=false>), or the
    # synth-only one for C2; entries per workload config, read by bench.py
    want = ("k_synth<true,false,false>",) if a.config == "c2" else ("k_synth<false,false,false>", "k_synth<false>")
    key = next((k for k in out if k.replace(" ", "") in want), None)
    synth = out.get(key, {})
    if "hbm_bytes_per_launch" in synth:
        tp = dst / "pmc_traffic.json"
        allp = json.loads(tp.read_text()) if tp.exists() else {}
        if "tag" in allp:  # older flat layout (C3 only)
            allp = {"c3": allp}
        allp[a.config] = {
            "tag": a.tag, "streams": a.streams, "frames": a.frames,
            "k_synth_hbm_bytes_per_launch": synth["hbm_bytes_per_launch"],
            "k_synth_fetch_kib": synth["FETCH_SIZE"], "k_synth_write_kib": synth["WRITE_SIZE"],
            "k_synth_mfma_util": synth.get("mfma_util"),
            "k_synth_clock_mhz": synth.get("clock_mhz"),
            "k_synth_mfma_f32_flop_per_launch": synth.get("mfma_f32_flop_per_launch"),
            "step_hbm_bytes": sum(cs.get("hbm_bytes_per_launch", 0.0) for cs in out.values()),
            "per_kernel_hbm_bytes": {k: cs.get("hbm_bytes_per_launch") for k, cs in out.items()},
            "method": "2 x FETCH_SIZE + WRITE_SIZE, separate rocprofv3 --pmc passes (tools/profile.sh)"}
        tp.write_text(json.dumps(allp, indent=1, sort_keys=True))
    for k, cs in sorted(out.items()):
        print(k, {c: "%.4g" % v for c, v in cs.items()})


if __name__ == "__main__":
    main()
