# round 2: compiler scheduling knobs (SC1 max-ilp, SC2 max-memory-clause, SC3 metric bias 0, SC4 LLVM wave-priority
# pass; all kernels) vs HEAD (BASE), C3 and C5
mkdir -p gpurun_out
bash abx/ab.sh BASE SC1 SC2 SC3 SC4 || exit 1
CONFIG=5 bash abx/ab.sh BASE SC1 SC2 SC3 SC4 || exit 1
