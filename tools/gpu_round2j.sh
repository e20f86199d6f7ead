# round-2 checkpoint 3 (re-entry): GPU suite, smoke, pipelined-parts A/B on C3 and C5, bench configs, profiles
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_j.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_j.log 2>&1 || { tail gpurun_out/smoke_j.log; exit 1; }
tail -1 gpurun_out/smoke_j.log
for c in 3 5; do for p in 1 2 4 8 1 2 4 8; do
  MP3D_PIPE=$p timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pipe_c${c}_$p.json 2> gpurun_out/pipe_c${c}_$p.err || { tail gpurun_out/pipe_c${c}_$p.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/pipe_c${c}_$p.json'));print('config $c pipe $p', r['value'], r['ms_per_step'], r.get('kernel_us'))"
done; done
for c in 2 1; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { tail gpurun_out/bench_c$c.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/bench_c$c.json'));print('config $c', r['value'], r.get('kernel_us'), (r.get('roofline') or {}).get('frac'), (r.get('cpu_baseline') or {}).get('value'))"
done
bash tools/profile.sh r02d || exit 1
