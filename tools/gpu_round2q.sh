# round 2: GPU suite on MC4 (k_mdcopy word quadruples per lane; in-tree), A/B vs BASE (HEAD) on C3 and C5
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE MC4 || exit 1
CONFIG=5 bash abx/ab.sh BASE MC4 || exit 1
