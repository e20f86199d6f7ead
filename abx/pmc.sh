#!/bin/bash
# abx/pmc.sh VARIANT... : per-kernel instruction counters (one rocprofv3 --pmc
# pass per variant, C3 at 65 536 x 32, 2 steps) of build_ab/VARIANT.so, then
# abx/pmc_sum.py prints VALU / SALU / LDS instructions per granule
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pmc_$v -o run \
    -- python3 bench.py --config ${CONFIG:-3} --steps 2 --warmup 1 --no-cpu-baseline --streaming 0 > /dev/null 2> gpurun_out/pmc_$v.err || exit 1
  python3 abx/pmc_sum.py gpurun_out/pmc_$v $v || exit 1
done
