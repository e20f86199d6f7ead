# round 2: GPU suite on HF3 (pre-shifted table select, unclamped window index; in-tree), A/B vs HF2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_n.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh HF2 HF3 || exit 1
CONFIG=5 bash abx/ab.sh HF2 HF3 || exit 1
