# round 2: the driver's default bench line at HEAD, and the per-frame call (C1) over 100 passes for a tighter median
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/bench_default.json'));print('default', r['value'], r['ms_per_step'], r['steps'], r['warmup'], r['roofline']['frac'])"
timeout -k 10 300 python bench.py --config 1 --steps 100 --warmup 5 > gpurun_out/bench_c1_100.json 2> gpurun_out/bench_c1_100.err || { tail gpurun_out/bench_c1_100.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/bench_c1_100.json'));print('C1 x100', r['value'], r['latency_us'])"
