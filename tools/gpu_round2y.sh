# round 2: k_huffman priority probes (count1 loop HP2, big_values loop HP3) vs HEAD (BASE), C3 and C5
mkdir -p gpurun_out
bash abx/ab.sh BASE HP2 HP3 || exit 1
CONFIG=5 bash abx/ab.sh BASE HP2 HP3 || exit 1
