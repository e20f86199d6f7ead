/*
 * mp3d_device.h -- device-side definitions shared by the kernels of the
 * batched MP3 decode hot path (mp3d_demux.hip, mp3d_huffman.hip,
 * mp3d_synth.hip; ISO/IEC 11172-3 / 13818-3).
 *
 * Pipeline for one batch call (all on one HIP stream, state resident in HBM):
 *   k_demux    wave   / stream  : header + side-info walk, bit-reservoir map,
 *                                 main-data bytes -> contiguous md region
 *   k_huffman  thread / unit    : scalefactors + Huffman (LDS LUT) -> is[576]
 *   k_synth    wave   / stream  : requantise, stereo, alias, IMDCT, overlap,
 *                                 32-band matrixing + 512-tap window -> PCM
 * A unit is one (frame, granule, channel).  Streams are independent, so the
 * batch is embarrassingly parallel over streams; frames of one stream are
 * walked in order inside k_demux / k_synth, which keep the per-stream state
 * (reservoir, overlap, synthesis FIFO) in registers / LDS between frames.
 * The reference (lxm0851/mp3) has no decoder source: its player's decode
 * loop (REF/README.md:2-3) is the path these kernels replace.
 */
#pragma once
#include <hip/hip_runtime.h>

#include "mp3d_internal.h"
#include "mp3d_tables.h"

namespace mp3d {

struct DevInfo { /* mirrors mp3d_frame_info (include/mp3d.h) */
    int32_t frame_bytes, channels, hz, layer, bitrate_kbps, samples;
};

#define REC_TAG 0x80  /* FrameRec.first_gr high bit: Xing/Info tag frame           */
#define REC_DROP 0x40 /* dropped frame (invalid side info, CRC mismatch)            */

/* One wave per data region: LDS operations of a wave complete in issue
 * order, so an LDS hand-off between lanes of ONE wave only needs the
 * compiler not to reorder across it -- no s_barrier and, unlike
 * __syncthreads(), no vmcnt(0) drain of loads/stores still in flight.    */
__device__ __forceinline__ void wave_sync() { __asm__ volatile("" ::: "memory"); }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

} // namespace mp3d
