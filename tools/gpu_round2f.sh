# k_demux window prefetch kept asynchronous: parity subset + A/B (C3)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_state.py tests/test_gpu_fuzz.py tests/test_gpu_lsf.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest6.log 2>&1; rc=$?; tail -3 gpurun_out/pytest6.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE DM2 || exit 1
