# C2 segment-length sweep (MP3D_SEG_FRAMES), k_synth<xr> HIP-event time and frames/s
set -o pipefail
for L in ${SEG_LS:-0 22 16 11 8 6}; do
  if [ $L = 0 ]; then unset MP3D_SEG_FRAMES; else export MP3D_SEG_FRAMES=$L; fi
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('L=$L', 'synth %.0f us' % d['kernel_us']['synth'], '%.1fM f/s' % (d['value']/1e6), 'frac %.3f' % d['roofline']['frac'])" || exit 1
  done
done
