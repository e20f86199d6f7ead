#!/usr/bin/env python3
"""Per-launch GPU clock of a kernel from a rocprofv3 GRBM_GUI_ACTIVE pass
(is k_synth<xr>'s slow-down over back-to-back C2 steps a
clock (power) drop?).

    rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d DIR -o run \\
        -- python3 bench.py --config 2 --steps 20 --warmup 2 --no-cpu-baseline
    python tools/dbg/launch_clock.py DIR [--kernel k_synth]

GRBM_GUI_ACTIVE as collected here is the sum over the 8 XCDs of the busy
cycles at the GPU clock (MI355X_MICROARCH.md DVFS note), so the launch's mean
clock = GRBM_GUI_ACTIVE / 8 / duration.  Prints one JSON line: per launch in
dispatch order the duration (us) and the clock (MHz)."""
import argparse
import csv
import json
import pathlib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_synth")
    a = ap.parse_args()
    d = pathlib.Path(a.dir)
    rows = list(csv.DictReader(open(next(d.rglob("run_counter_collection.csv")))))
    out = []
    for r in rows:
        name = r["Kernel_Name"]
        if a.kernel not in name or r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        t0 = int(r.get("Start_Timestamp") or r.get("Begin_Timestamp") or 0)
        t1 = int(r.get("End_Timestamp") or 0)
        dur_ns = t1 - t0
        cyc = float(r["Counter_Value"])
        out.append({"dispatch": int(r.get("Dispatch_Id") or 0), "us": dur_ns / 1e3,
                    "mhz": cyc / 8.0 / dur_ns * 1e3 if dur_ns > 0 else None})
    out.sort(key=lambda x: x["dispatch"])
    print(json.dumps({"kernel": a.kernel, "launches": out}))


if __name__ == "__main__":
    main()
