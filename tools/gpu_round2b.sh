# round 2: GPU suite, per-frame latency, A/B of k_demux waves_per_eu and synth-only at 4 waves/SIMD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest3.log 2>&1
rc=$?; tail -15 gpurun_out/pytest3.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --config 1 --steps 30 --warmup 3 > gpurun_out/c1b.json 2>/dev/null || exit 1
python -c "import json;r=json.load(open('gpurun_out/c1b.json'));print('c1',r['value'],r['latency_us'])"
timeout -k 10 200 python tools/bench_per_frame.py > gpurun_out/pf.json 2>/dev/null && cat gpurun_out/pf.json
bash abx/ab.sh BASE DMW0 || exit 1
CONFIG=2 bash abx/ab.sh BASE XW4 || exit 1
