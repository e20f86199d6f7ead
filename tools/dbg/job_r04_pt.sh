# round-4 diagnostic job (gpurun): k_synth phase times (abx/ptime.py builds)
# and A/B kernel times of the build_ab/ variants named on the command line
set -o pipefail
mkdir -p gpurun_out
for v in PT_DMA8c; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 200 python tools/dbg/synth_phase_times.py > gpurun_out/pt_$v.txt 2>gpurun_out/pt_$v.err || { tail -5 gpurun_out/pt_$v.err; exit 1; }
  echo $v; cat gpurun_out/pt_$v.txt
done
bash abx/ab.sh "$@"
