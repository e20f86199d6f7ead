# round 2: k_frame phase times at HEAD (abx FRT probe: s_memtime stamps; tools/dbg/frame_timing.py)
mkdir -p gpurun_out
MP3D_LIB=abx/FRT.so timeout -k 10 200 python tools/dbg/frame_timing.py > gpurun_out/frame_timing.json || exit 1
cat gpurun_out/frame_timing.json
