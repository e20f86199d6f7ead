#!/usr/bin/env python3
"""Every counter of an abx/pmcx.sh pass, averaged per launch of each kernel
(kernels with >= 1000 waves or any counter named like a size)."""
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
for k, cs in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print("%s %-34s %s" % (tag, k, " ".join("%s %.4g" % (c, v) for c, v in sorted(m.items()))))
