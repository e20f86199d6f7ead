# round-4 diagnostic job (gpurun): the batch parity test against each build_ab/ variant named
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  MP3D_LIB=build_ab/$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 > gpurun_out/bisect_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/bisect_$v.log)"
done
