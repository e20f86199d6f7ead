# round 2: wave-priority sweep for k_synth (SP2-SP6), k_huffman staging priority (HP1), phase Q table-word reuse (LP1)
mkdir -p gpurun_out
bash abx/ab.sh BASE SP2 SP3 SP4 SP5 SP6 HP1 LP1 || exit 1
CONFIG=2 bash abx/ab.sh BASE SP2 SP4 SP5 || exit 1
