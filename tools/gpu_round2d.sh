# Huffman LDS-conflict probes (timing only) + PMC profile of HEAD (C3)
mkdir -p gpurun_out
bash abx/ab.sh BASE HW0 LUT0 || exit 1
bash tools/profile.sh r02a || exit 1
