#!/usr/bin/env python3
"""Per-kernel instruction counters of an abx/pmc.sh pass, per granule
(C3: 65 536 streams x 32 frames x 2 granules per launch)."""
import collections
import csv
import glob
import sys

d, tag = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mp3d::", "").replace(" ", "")
    if "k_" in k:
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
gran = 65536 * 32 * 2
for k, cs in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    if m.get("SQ_WAVES", 0) < 1000:
        continue
    print("%s %-28s VALU/gr %.1f SALU/gr %.1f LDS/gr %.1f VMEM_RD/gr %.2f wait %.3f conflict/LDS %.2f" % (
        tag, k, m["SQ_INSTS_VALU"] / gran, m["SQ_INSTS_SALU"] / gran, m["SQ_INSTS_LDS"] / gran,
        m["SQ_INSTS_VMEM_RD"] / gran, m["SQ_WAIT_INST_ANY"] / max(1.0, m["SQ_WAVE_CYCLES"]),
        m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_INSTS_LDS"])))
