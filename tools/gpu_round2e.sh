# branch-free is[] prefetch: parity + A/B against the previous build
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_lsf.py tests/test_gpu_c2.py tests/test_gpu_fuzz.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest4.log 2>&1; rc=$?; tail -3 gpurun_out/pytest4.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE PF2 || exit 1
