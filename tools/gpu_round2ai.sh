# round 2: k_synth with 6 streams per workgroup (SW6) vs HEAD (BASE), C3, C5, C2
mkdir -p gpurun_out
bash abx/ab.sh BASE SW6 || exit 1
CONFIG=5 bash abx/ab.sh BASE SW6 || exit 1
CONFIG=2 bash abx/ab.sh BASE SW6 || exit 1
