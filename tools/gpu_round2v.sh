# round 2: k_synth wave-priority probes (s_setprio through phase M: SP1; through phase Q: SP2) vs HEAD (BASE), C3 and C2
mkdir -p gpurun_out
bash abx/ab.sh BASE SP1 SP2 || exit 1
CONFIG=2 bash abx/ab.sh BASE SP1 SP2 || exit 1
