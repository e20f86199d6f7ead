#!/bin/bash
# abx/build.sh NAME [extra hipcc flags...]: build mp3_amd/csrc as build_ab/NAME.so (A/B experiments)
set -e
mkdir -p build_ab
N=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -fvisibility=hidden -o build_ab/$N.so "$@" \
  mp3_amd/csrc/mp3d_demux.hip mp3_amd/csrc/mp3d_huffman.hip mp3_amd/csrc/mp3d_synth.hip \
  mp3_amd/csrc/mp3d_host.cpp
