# per-frame call: where the time goes (kernel + copy trace, no counters)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/pf_prof -o pf -- python tools/bench_per_frame.py > gpurun_out/pf2.json 2> gpurun_out/pf2.err || { tail -20 gpurun_out/pf2.err; exit 1; }
cat gpurun_out/pf2.json
find gpurun_out/pf_prof -name "*stats*" | head
for f in $(find gpurun_out/pf_prof -name "*stats.csv"); do echo == $f; head -12 $f; done
