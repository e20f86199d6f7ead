# round 2 checkpoint 6 at HEAD (phase-Q priority): smoke, every bench config, 2-rank rehearsal, profiles (C3 + C2)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_z.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_z.log; [ $rc = 0 ] || exit 1
python -c "import sys; sys.path.insert(0, 'tests'); import _gen; d, o = _gen.stream(_gen.C3, 7000001, 400); open('gpurun_out/c3_400.mp3', 'wb').write(d)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g.log 2>&1 || { tail gpurun_out/smoke_g.log; exit 1; }
tail -1 gpurun_out/smoke_g.log
for c in 3 2 5 1; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { tail gpurun_out/bench_c$c.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/bench_c$c.json'));print('config $c', r['value'], r.get('kernel_us'), (r.get('roofline') or {}).get('frac'), (r.get('cpu_baseline') or {}).get('value'), r.get('latency_us'))"
done
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --gather > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || { tail gpurun_out/bench_g2.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/bench_g2.json'));print('2 ranks', r['value'], r['per_rank_frames_per_s'])"
bash tools/profile.sh r02g || exit 1
bash tools/profile.sh r02g_c2 --config 2 || exit 1
timeout -k 10 60 examples/mp3d_play gpurun_out/c3_400.mp3 gpurun_out/c3_400.wav --time 2> gpurun_out/play_time.txt || exit 1
cat gpurun_out/play_time.txt
