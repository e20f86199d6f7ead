# round 2: GPU suite on HF5 (k_huffman pair loop carrying pos + 31; abx/HF5.so); A/B vs HEAD (BASE) of HF5 and the
# k_synth LDS-read priority variants SW1 / SI1 / SM1, C3 and C5
mkdir -p gpurun_out
MP3D_LIB=abx/HF5.so timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc = 0 ] || exit 1
bash abx/ab.sh BASE HF5 SW1 SI1 SM1 || exit 1
CONFIG=5 bash abx/ab.sh BASE HF5 SW1 SI1 SM1 || exit 1
