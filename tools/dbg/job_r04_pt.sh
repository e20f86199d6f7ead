# round-4 diagnostic job (gpurun): k_synth phase times (abx/ptime.py builds
# named on the command line; PTW = phase W split: slots Q:scales / Q:requant
# read as W:vmcnt-drain / W:X-loads there)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 200 python tools/dbg/synth_phase_times.py > gpurun_out/pt_$v.txt 2>gpurun_out/pt_$v.err || { tail -5 gpurun_out/pt_$v.err; exit 1; }
  echo $v; cat gpurun_out/pt_$v.txt
done
