#!/bin/bash
# abx/ab.sh VARIANT... : alternate bench runs of build_ab/VARIANT.so (built by abx/variants.py / abx/build.sh), print kernel times
for rep in 1 2; do
for v in "$@"; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 200 python bench.py --config ${CONFIG:-3} --no-cpu-baseline --streaming 0 --steps ${STEPS:-5} --warmup 2 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); k=d['kernel_us']; print('$v', 'synth %.0f huff %.0f demux %.0f  %.1fM f/s' % (k['synth'], k['huffman'], k['demux'], d['value']/1e6))" || exit 1
done; done
