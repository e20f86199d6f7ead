#!/bin/bash
# Kernel-time and PMC-counter profile of the bench workload (run on the GPU
# box via gpurun).  Usage: tools/profile.sh TAG [extra bench args]
# Writes gpurun_out/prof_TAG/{stats,pmc_*}/ ; summaries are copied into
# profiles/ by hand.  Each counter group is its own rocprofv3 pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950); the last pass
# gives the matrix-core utilisation of the DCT tile (MfmaUtil recipe).
set -e
TAG=${1:?tag}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $BENCH > $OUT/stats.json 2> $OUT/stats.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $OUT/pmc_sq1 -o run -- python3 $BENCH > /dev/null 2> $OUT/pmc_sq1.err
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_sq2 -o run -- python3 $BENCH > /dev/null 2> $OUT/pmc_sq2.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $BENCH > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $BENCH > /dev/null 2> $OUT/pmc_write.err
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_mfma -o run -- python3 $BENCH > /dev/null 2> $OUT/pmc_mfma.err
echo profile $TAG done
