# round 2: k_synth priority while issuing LDS reads (phase W: SW1, phase I: SI1, phase M: SM1) vs HEAD, C3 and C5
mkdir -p gpurun_out
bash abx/ab.sh BASE SW1 SI1 SM1 || exit 1
CONFIG=5 bash abx/ab.sh BASE SW1 SI1 SM1 || exit 1
