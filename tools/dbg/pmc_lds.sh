# LDS / VALU busy counters of one build_ab variant (C3, 2 steps); one rocprofv3 --pmc pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
v=${1:?variant}
MP3D_LIB=build_ab/$v.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmcl_$v -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --streaming 0 > /dev/null 2> gpurun_out/pmcl_$v.err || exit 1
python3 - gpurun_out/pmcl_$v <<'PY'
import collections, csv, glob, sys
d = sys.argv[1]
f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0]
kt = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mp3d::", "").replace(" ", "")
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(kt)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mp3d::", "").replace(" ", "")
    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k, cs in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    if m.get("SQ_WAVES", 0) < 1000:
        continue
    t = sum(dur[k]) / max(1, len(dur[k]))
    cu_cycles = t * 2.4e9 * 256
    print(k, "dur %.3f ms" % (t * 1e3), " ".join("%s=%.4g" % (c, v) for c, v in sorted(m.items())),
          "| LDS_IDX_ACTIVE/CU-cycle %.3f  ACTIVE_INST_LDS/CU-cycle %.3f  VALU/CU-cycle %.3f  waves/SIMD %.2f" % (
              m["SQ_LDS_IDX_ACTIVE"] / cu_cycles, m["SQ_ACTIVE_INST_LDS"] / cu_cycles,
              m["SQ_ACTIVE_INST_VALU"] / cu_cycles, m["SQ_WAVE_CYCLES"] / (t * 2.4e9 * 1024)))
PY
