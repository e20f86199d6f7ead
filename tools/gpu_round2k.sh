# round 2: GPU suite on the packed-IMDCT k_synth (in-tree library), then A/B: HEAD (BASE) vs packed IMDCT (PK1),
# and timing-only probes of k_huffman with conflict-free window (HW0) / LUT (LUT0) reads
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE PK1 HW0 LUT0 || exit 1
CONFIG=2 bash abx/ab.sh BASE PK1 || exit 1
