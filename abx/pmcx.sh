#!/bin/bash
# abx/pmcx.sh "COUNTERS" VARIANT... : one rocprofv3 --pmc pass per variant with the
# given counters (C3, 2 steps), then abx/pmc_any.py prints them per kernel launch
mkdir -p gpurun_out
export TMPDIR=/tmp
ctrs=$1; shift
for v in "$@"; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
    -d gpurun_out/pmcx_$v -o run -- python3 bench.py --config ${CONFIG:-3} --steps 2 --warmup 1 --no-cpu-baseline \
    --streaming 0 > /dev/null 2> gpurun_out/pmcx_$v.err || exit 1
  python3 abx/pmc_any.py gpurun_out/pmcx_$v $v || exit 1
  rm -rf gpurun_out/pmcx_$v
done
