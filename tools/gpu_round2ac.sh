# round 2: GPU suite against PF1 (k_synth next-granule prefetch issued at the start of phase Q; abx/PF1.so), A/B vs HEAD
mkdir -p gpurun_out
MP3D_LIB=abx/PF1.so timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_ac.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ac.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE PF1 || exit 1
CONFIG=5 bash abx/ab.sh BASE PF1 || exit 1
bash abx/ab.sh BASE PF1 || exit 1
