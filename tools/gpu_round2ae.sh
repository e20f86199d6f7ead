# round 2: k_frame with per-granule unit waits (PW1, abx/PW1.so): per-frame tests first under a short limit, then the
# GPU suite, per-frame A/B vs HEAD (BASE) and the C player
mkdir -p gpurun_out
MP3D_LIB=abx/PW1.so timeout -k 10 150 python -u -m pytest tests/test_gpu_per_frame.py -q -x --timeout 60 --timeout-method thread > gpurun_out/pytest_ae0.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ae0.log; [ $rc = 0 ] || exit 1
MP3D_LIB=abx/PW1.so timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_ae.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ae.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for v in BASE PW1; do
  MP3D_LIB=abx/$v.so timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c1_$v.json 2>/dev/null || exit 1
  python -c "import json;r=json.load(open('gpurun_out/c1_$v.json'));print('$v C1', r['value'], r['latency_us'])"
done; done
