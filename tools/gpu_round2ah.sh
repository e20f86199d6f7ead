# round 2 end rehearsal at HEAD: the driver's commands (GPU suite, smoke, default bench), the 2-rank gloo rehearsal
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ah.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ah.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ah.log 2>&1 || { tail gpurun_out/smoke_ah.log; exit 1; }
tail -1 gpurun_out/smoke_ah.log
timeout -k 10 300 python bench.py > gpurun_out/bench_ah.json 2> gpurun_out/bench_ah.err || { tail gpurun_out/bench_ah.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/bench_ah.json'));print('default', r['value'], r['ms_per_step'], r['roofline']['frac'], r['cpu_baseline']['value'], r['cpu_baseline']['cores'])"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/bench_ah_g2.json 2> gpurun_out/bench_ah_g2.err || { tail gpurun_out/bench_ah_g2.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/bench_ah_g2.json'));print('2 ranks', r['n_gpus'], r['value'], r['per_rank_frames_per_s'])"
