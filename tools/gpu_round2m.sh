# round 2: GPU suite on the branch-free count1 decode (in-tree library, HF2), A/B vs HF1 (window/sign rework) and HEAD (BASE)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_m.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE HF1 HF2 || exit 1
CONFIG=5 bash abx/ab.sh HF1 HF2 || exit 1
