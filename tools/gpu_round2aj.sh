# round 2: phase-Q priority on the synth-only entry (SPX) vs HEAD, C2, four alternations
mkdir -p gpurun_out
CONFIG=2 bash abx/ab.sh BASE SPX || exit 1
CONFIG=2 bash abx/ab.sh BASE SPX || exit 1
