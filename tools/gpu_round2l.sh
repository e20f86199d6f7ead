# round 2: GPU suite on the k_huffman window/sign rework (in-tree library), A/B vs HEAD (BASE) on C3 and C5
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_l.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE HF1 || exit 1
CONFIG=5 bash abx/ab.sh BASE HF1 || exit 1
