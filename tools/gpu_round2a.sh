mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c2.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest2.log 2>&1 || { tail -30 gpurun_out/pytest2.log; exit 1; }
tail -3 gpurun_out/pytest2.log
for sg in 0 4 8 11 16; do
  if [ $sg = 0 ]; then unset MP3D_SEG_FRAMES; else export MP3D_SEG_FRAMES=$sg; fi
  timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c2_$sg.json 2> gpurun_out/c2_$sg.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/c2_$sg.json'));print('seg',$sg,r['value'],r['kernel_us'],r['roofline']['frac'])"
done
unset MP3D_SEG_FRAMES
timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/c3.json'));print('c3',r['value'],r['kernel_us'],r['cpu_baseline']['value'],r['cpu_baseline']['cores'],r['cpu_baseline']['single_thread_value'])"
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/c5.json'));print('c5',r['value'],r['kernel_us'])"
timeout -k 10 300 python bench.py --config 1 --steps 20 --warmup 2 > gpurun_out/c1.json 2> gpurun_out/c1.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/c1.json'));print('c1',r['value'],r['latency_us'])"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --streams 16384 --steps 5 --warmup 1 --gather > gpurun_out/g2.json 2> gpurun_out/g2.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/g2.json'));print('g2',r['n_gpus'],r['value'],r['per_rank_frames_per_s'],r.get('gather'))"
