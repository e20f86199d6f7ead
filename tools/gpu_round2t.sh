# round 2: GPU suite on IN1 (frame infos written in place into a device array, no D2D copy; in-tree), A/B vs HEAD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_t.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE IN1 || exit 1
CONFIG=5 bash abx/ab.sh BASE IN1 || exit 1
