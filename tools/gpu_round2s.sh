# round 2: GPU suite on CY1 (k_frame reservoir carry in / out by wave 3; in-tree), per-frame A/B PF2 vs CY1,
# k_huffman ranking-key probes RK1 / RK2 vs PF2 on C3
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_s.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for v in PF2 CY1; do
  MP3D_LIB=abx/$v.so timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c1_$v.json 2>/dev/null || exit 1
  python -c "import json;r=json.load(open('gpurun_out/c1_$v.json'));print('$v C1', r['value'], r['latency_us'])"
done; done
python -c "import sys; sys.path.insert(0, 'tests'); import _gen; d, o = _gen.stream(_gen.C3, 7000001, 400); open('gpurun_out/c3_400.mp3', 'wb').write(d)"
timeout -k 10 60 examples/mp3d_play gpurun_out/c3_400.mp3 gpurun_out/c3_400.wav --time 2> gpurun_out/play_time.txt || exit 1
cat gpurun_out/play_time.txt
bash abx/ab.sh PF2 RK1 RK2 || exit 1
