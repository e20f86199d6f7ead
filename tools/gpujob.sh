#!/bin/bash
# One parametrised runner for GPU-box jobs (replaces the one-off
# tools/gpu_round2*.sh scripts).  Every step has its own time limit and
# stops the job on failure, so steps chain with &&:
#
#   /usr/local/graft/bin/gpurun --timeout 900 -- \
#     'bash tools/gpujob.sh suite && bash tools/gpujob.sh bench c3 && bash tools/gpujob.sh profile r03a'
#
#   suite [pytest args]      GPU test suite (default: all of tests/ -m gpu)
#   smoke                    __graft_entry__.smoke()
#   bench TAG [bench args]   python bench.py ... > gpurun_out/bench_TAG.json (one summary line printed)
#   profile TAG [bench args] tools/profile.sh TAG (rocprof stats + PMC passes)
#   ab [variants]            abx/ab.sh (A/B of prebuilt abx/*.so variants)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cmd=${1:?usage: gpujob.sh suite|smoke|bench|profile|ab ...}; shift
case $cmd in
suite)
    args=("$@"); [ ${#args[@]} = 0 ] && args=(tests)
    timeout -k 10 900 python -u -m pytest "${args[@]}" -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/pytest.log 2>&1
    rc=$?; tail -5 gpurun_out/pytest.log; exit $rc ;;
smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
bench)
    tag=${1:?tag}; shift
    timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
        || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
    python - "$tag" <<'EOF'
import json, sys
r = json.load(open("gpurun_out/bench_%s.json" % sys.argv[1]))
keys = ("value", "ms_per_step", "kernel_us", "latency_us", "streaming")
print(sys.argv[1], {k: r[k] for k in keys if k in r}, "frac", (r.get("roofline") or {}).get("frac"))
EOF
    ;;
profile)
    tag=${1:?tag}; shift
    bash tools/profile.sh "$tag" "$@" ;;
ab)
    bash abx/ab.sh "$@" ;;
*)
    echo "unknown job $cmd" >&2; exit 2 ;;
esac
