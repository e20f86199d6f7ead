# round 2: GPU suite on SPQ (k_synth decode path at priority 1 through phase Q; in-tree), A/B vs HEAD on C3, C5, C2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_x.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE SPQ || exit 1
CONFIG=5 bash abx/ab.sh BASE SPQ || exit 1
CONFIG=2 bash abx/ab.sh BASE SPQ || exit 1
