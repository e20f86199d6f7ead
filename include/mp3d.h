/*
 * mp3d.h -- C ABI of the MI355X-native batched MP3 (MPEG-1 and MPEG-2 / 2.5
 * Layer III) decoder.
 *
 * Drop-in boundary for the decode hot path of lxm0851/mp3.  The reference
 * snapshot contains no decoder source and therefore no FFI surface to copy
 * (SURVEY.md §8(b)): the player it describes (REF/README.md:2-3, "audio
 * player ... crackle and noise during playback") decodes MP3 frame by frame
 * in its playback loop, and REF/README.md:44 says it runs from source.  The
 * per-frame entry point below replaces that (absent) per-frame decode call
 * with the conventional shape of public C MP3 decoders (decoder handle,
 * frame bytes in, interleaved int16 PCM + frame info out); the batch entry
 * points expose the same path for tens of thousands of concurrent streams.
 * INTEGRATION.md shows the ctypes / cffi / C++ bindings a host adds.
 *
 * Conventions
 *  - Plain C types only.  All calls return >= 0 on success, a negative
 *    MP3D_E* code on failure; nothing throws or aborts across the ABI.
 *  - Caller owns every buffer passed in.  A handle owns its device memory
 *    and decoder state; *_destroy frees it.
 *  - PCM is int16 (or float32 with the _f32 entry points), interleaved L/R,
 *    1152 samples per channel per MPEG-1 frame, 576 per MPEG-2 / 2.5 (LSF)
 *    frame, at the start of the frame's 2304-sample row.
 *  - The compute path is HIP on an AMD Instinct MI355X (gfx950).  There is
 *    no CPU fallback: without a usable GPU, create calls fail with
 *    MP3D_E_NO_DEVICE.
 */
#ifndef MP3D_H
#define MP3D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: the state blob's synthesis history is partial window sums in float
 *    units, with a format stamp (blobs of v4 are refused by set_state) */
#define MP3D_ABI_VERSION 5

#if defined(__GNUC__) || defined(__clang__)
#define MP3D_API __attribute__((visibility("default")))
#else
#define MP3D_API
#endif

/* error codes */
#define MP3D_OK 0
#define MP3D_E_ARG (-1)        /* bad argument                                 */
#define MP3D_E_NO_DEVICE (-2)  /* no HIP device / device ordinal out of range  */
#define MP3D_E_HIP (-3)        /* HIP runtime error (see mp3d_last_hip_error)  */
#define MP3D_E_NOMEM (-4)      /* device or host allocation failed             */
#define MP3D_E_CAPACITY (-5)   /* batch larger than the handle was created for */
#define MP3D_E_NEED_MORE (-6)  /* buffer holds no complete frame               */

typedef struct mp3d_frame_info {
    int frame_bytes;  /* bytes consumed (0: no frame found)                */
    int channels;     /* 1 or 2                                            */
    int hz;           /* 32000 / 44100 / 48000 (MPEG-1), 8000 .. 24000 LSF */
    int layer;        /* 3                                                 */
    int bitrate_kbps; /* 32..320 (MPEG-1), 8..160 (LSF)                    */
    int samples;      /* PCM samples per channel: 1152, 576 (LSF) or 0    */
} mp3d_frame_info;

typedef struct mp3d_dec mp3d_dec;
typedef struct mp3d_batch mp3d_batch;

/* ---- per-frame decoder (the player's decode call) ---------------------- *
 * One decoder per audio stream and host thread.  mp3d_decode_frame finds
 * the next frame in buf (skipping an ID3v2 tag / garbage before the sync
 * word), decodes it on the GPU and returns samples per channel: 1152 (576
 * for an MPEG-2 / 2.5 LSF frame), or 0
 * when bytes were consumed without audio (Xing/Info tag frame, invalid
 * frame).  info->frame_bytes (+ any skipped prefix) tells how far to
 * advance; pcm may be NULL (decode for state only).  Reservoir underflow
 * (a stream entered mid-way) follows FFmpeg: the affected granules decode
 * as silence.  A HIP error while the decoder was reading ahead (or putting
 * a read-ahead back) leaves its state undefined: that error is returned by
 * every later decode / get_state / set_options call until mp3d_dec_reset or
 * a successful mp3d_dec_set_state.                                          */
MP3D_API int mp3d_dec_create(mp3d_dec **out);
MP3D_API int mp3d_dec_create_on(int device, mp3d_dec **out);
MP3D_API void mp3d_dec_destroy(mp3d_dec *dec);
MP3D_API void mp3d_dec_reset(mp3d_dec *dec);
MP3D_API int mp3d_decode_frame(mp3d_dec *dec, const uint8_t *buf, size_t bytes, int16_t *pcm /* <= 2304 */,
                      mp3d_frame_info *info);
/* the same with float32 PCM (FFmpeg's float convention: full scale 1.0,
 * not clipped; the int16 output is clamp(floor(x * 32768 + 0.5)) of these
 * values, saturated to [-32768, 32767]: FFmpeg's fixed-point round_sample
 * convention, so an exact .5 tie rounds up, unlike rint's ties-to-even) */
MP3D_API int mp3d_decode_frame_f32(mp3d_dec *dec, const uint8_t *buf, size_t bytes, float *pcm /* <= 2304 */,
                          mp3d_frame_info *info);
/* (ABI v4) either of the above by flags: MP3D_FRAME_F32 selects float32 PCM;
 * MP3D_FRAME_LAST says buf holds the rest of the stream, so a final frame cut
 * short (header and side info present) is decoded with its missing bytes as
 * zeros -- as the batch path and FFmpeg do -- instead of MP3D_E_NEED_MORE;
 * info->frame_bytes then counts the bytes that were present.              */
#define MP3D_FRAME_F32 1
#define MP3D_FRAME_LAST 2
MP3D_API int mp3d_decode_frame_ex(mp3d_dec *dec, const uint8_t *buf, size_t bytes, void *pcm, int flags,
                                  mp3d_frame_info *info);

/* ---- batched decoder (many concurrent streams on one GPU) -------------- *
 * A batch handle keeps per-stream decoder state resident in HBM across
 * calls: call k decodes frames [k*F, (k+1)*F) of every stream.
 *
 * frames           all streams' bytes; host memory or a device pointer on
 *                  the handle's GPU (detected per call)
 * offsets, sizes   host arrays [n_streams]: stream s occupies
 *                  frames[offsets[s] .. offsets[s] + sizes[s])
 * pcm              [n_streams][frames_per_stream][2304] int16, host or
 *                  device; frames with info.samples == 0 are left untouched
 * infos            [n_streams][frames_per_stream] or NULL, host or device
 * hip_stream       hipStream_t to run on (NULL: the handle's own stream)
 * The call is asynchronous when every pointer is device memory; otherwise
 * it synchronises before returning.                                         */
MP3D_API int mp3d_batch_create(int device, int max_streams, int max_frames, mp3d_batch **out);
MP3D_API void mp3d_batch_destroy(mp3d_batch *b);
MP3D_API int mp3d_batch_reset(mp3d_batch *b); /* forget all per-stream state         */
MP3D_API int mp3d_batch_decode(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes,
                      int n_streams, int frames_per_stream, int16_t *pcm, mp3d_frame_info *infos,
                      void *hip_stream);
/* float32 PCM sink: pcm [n_streams][frames_per_stream][2304] float */
MP3D_API int mp3d_batch_decode_f32(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets,
                          const uint32_t *sizes, int n_streams, int frames_per_stream, float *pcm,
                          mp3d_frame_info *infos, void *hip_stream);
MP3D_API int mp3d_batch_sync(mp3d_batch *b);

/* ---- decode options (ABI v3) --------------------------------------------- *
 * MP3D_OPT_CRC_CHECK: verify the CRC-16 of error-protected frames (ISO
 *   11172-3 2.4.3.1: polynomial 0x8005 over header bytes 2..3 and the side
 *   info) and drop a frame whose CRC mismatches, like a bad frame
 *   (info.samples = 0; the bit reservoir restarts from the frame's own
 *   bytes).  FFmpeg behaves so with err_detect = crccheck + explode; its
 *   default, and this library's, ignores the CRC.
 * Options apply to later decode calls of the handle.                        */
#define MP3D_OPT_CRC_CHECK 1
MP3D_API int mp3d_batch_set_options(mp3d_batch *b, int flags);
MP3D_API int mp3d_dec_set_options(mp3d_dec *dec, int flags);

/* ---- staged entry points (parity taps / BASELINE config 2) ------------- *
 * huffman_only: run demux + reservoir + scalefactors + Huffman and return
 *   is_out [n_streams][F][2][2][576] int16 and sf_out [..][2][2][40] uint8
 *   (either may be NULL).  Advances per-stream state like a decode.
 * synth_only: stages a8..a11 from spectra: xr [n_streams][F][2 gr][nch][576]
 *   f32 (requantised, after stereo, bitstream order), block_type / mixed
 *   [n_streams][F][2][nch]; pcm as in mp3d_batch_decode.                    */
MP3D_API int mp3d_batch_huffman_only(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes,
                            int n_streams, int frames_per_stream, int16_t *is_out, uint8_t *sf_out,
                            void *hip_stream);
/* synth_only takes MPEG-1 rates (32 / 44.1 / 48 kHz) */
MP3D_API int mp3d_batch_synth_only(mp3d_batch *b, const float *xr, const uint8_t *block_type, const uint8_t *mixed,
                          int n_streams, int frames_per_stream, int nch, int sample_rate_hz, int16_t *pcm,
                          void *hip_stream);

/* ---- stream-level info: Xing/Info tag and gapless playback ------------- *
 * Filled from the stream's leading Xing/Info frame (read by the demux kernel
 * on the stream's first call).  Gapless trim follows FFmpeg's demuxer
 * (libavformat/mp3dec.c): with a LAME / Lavf / Lavc encoder extension the
 * first enc_delay + 529 decoded samples per channel are encoder/decoder
 * delay, and when the tag also carries a frame count, samples from
 * total_frames * 1152 (576 for MPEG-2/2.5 LSF) + 529 - enc_padding on are padding.  The decoder
 * always emits every decoded frame; apply the trim when concatenating.      */
typedef struct mp3d_stream_info {
    int has_tag;          /* a Xing/Info frame opened the stream               */
    int has_lame;         /* ... with a LAME / Lavf / Lavc encoder extension   */
    int enc_delay;        /* encoder delay, samples per channel (0 if none)    */
    int enc_padding;      /* encoder padding, samples per channel (0 if none)  */
    int total_frames;     /* Xing frame count (-1 if absent)                   */
    int skip_samples;     /* gapless: leading samples to drop (0 if none)      */
    long long end_sample; /* gapless: index of the first padding sample, -1    */
} mp3d_stream_info;

/* out[n_streams]; valid once the call that decoded a stream's first frame
 * has completed (synchronises the handle's stream).                       */
MP3D_API int mp3d_batch_stream_info(mp3d_batch *b, int n_streams, mp3d_stream_info *out);
MP3D_API int mp3d_dec_stream_info(mp3d_dec *dec, mp3d_stream_info *out);

/* ---- one long stream at full-GPU speed (frame-parallel) ---------------- *
 * Decodes a whole stream (data[0 .. bytes), host or device) by splitting it
 * into segments of L output frames that run as concurrent virtual streams
 * of one batch call.  Each segment starts a few frames early (payloads of
 * >= 511 bytes, the largest main_data_begin, before its first frame but one),
 * so its output is bit-identical to a sequential decode; the warm-up frames'
 * output is discarded.  The handle (mp3d_batch_create) needs max_streams
 * >= 1 and max_frames >= L + 11: the warm-up is 4 frames at 128 kbps
 * stereo and at most 11 (32 kbps); more max_streams runs more segments per
 * kernel launch.
 * pcm     [max_frames][2304] int16, or float with f32 != 0; host or device.
 *         Row j is frame slot j of the stream, zero for slots without
 *         audio (Xing/Info frame, dropped frame); a mono row holds 1152
 *         samples and zeros.
 * infos   [max_frames] or NULL, host or device.
 * n_frames   out: frame slots found (MP3D_E_CAPACITY if > max_frames).
 * sinfo   stream info (Xing/Info tag, gapless trim) or NULL.
 * Synchronous.  The segments decode on scratch state: the handle's own
 * per-stream state (for mp3d_batch_decode) is left untouched.              */
MP3D_API int mp3d_batch_decode_long(mp3d_batch *b, const uint8_t *data, size_t bytes, int L, void *pcm, int f32,
                                    long long max_frames, mp3d_frame_info *infos, long long *n_frames,
                                    mp3d_stream_info *sinfo);

/* Host-side plan of mp3d_batch_decode_long (no GPU needed): the stream's
 * frame slots (frame_off[n_frames], byte offset of each frame header) and
 * the first frame of each segment's warm-up (seg_start[ceil(n_frames / L)]);
 * either array may be NULL.  max_warmup = max over segments of
 * k * L - seg_start[k].  data must be host memory.  A caller can shard the
 * segments of one stream over several GPUs with it.                        */
MP3D_API int mp3d_long_plan(const uint8_t *data, size_t bytes, int L, long long max_frames, uint64_t *frame_off,
                            long long *seg_start, long long *n_frames, int *max_warmup);

/* ---- per-stream state save / restore (ABI v4) --------------------------- *
 * A stream's decoder state -- bit-reservoir carry, IMDCT overlap, synthesis
 * history, MPEG family, Xing/LAME tag, frame count -- is an opaque blob of
 * mp3d_state_bytes() bytes, valid for handles of the same ABI version and
 * for either PCM sink (a stream may switch between int16 and float calls).
 * batch_get_state copies the state of streams [first, first + n) out of the
 * handle into buf; batch_set_state writes it into those slots (of this or
 * another handle) and fails with MP3D_E_ARG, writing nothing, when a blob
 * lacks this version's format stamp (e.g. one saved by an ABI v4 build).  A player seeks by saving the state at a frame boundary
 * and restoring it before decoding from that frame's bytes again; a server
 * moves a stream between batches or GPUs the same way.  buf: host or device
 * memory.  Both order after the handle's last call and return when done.  */
MP3D_API size_t mp3d_state_bytes(void);
MP3D_API int mp3d_batch_get_state(mp3d_batch *b, int first, int n, void *buf);
MP3D_API int mp3d_batch_set_state(mp3d_batch *b, int first, int n, const void *buf);
MP3D_API int mp3d_dec_get_state(mp3d_dec *dec, void *buf);
MP3D_API int mp3d_dec_set_state(mp3d_dec *dec, const void *buf);

/* ---- diagnostics -------------------------------------------------------- */
MP3D_API const char *mp3d_strerror(int err);
MP3D_API int mp3d_last_hip_error(void);
MP3D_API int mp3d_abi_version(void);
/* device-side microseconds of each pipeline kernel in the last batch call
 * (demux, huffman, synth); needs mp3d_batch_set_timing(b, 1).               */
MP3D_API int mp3d_batch_set_timing(mp3d_batch *b, int enable);
MP3D_API int mp3d_batch_kernel_times(mp3d_batch *b, float *us3);

#ifdef __cplusplus
}
#endif
#endif /* MP3D_H */
