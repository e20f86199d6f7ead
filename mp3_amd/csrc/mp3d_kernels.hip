/*
 * mp3d_kernels.hip -- MI355X (gfx950) kernels of the batched MPEG-1 Layer III
 * decode hot path (ISO/IEC 11172-3 clause per
 * kernel).  The reference (lxm0851/mp3) has no decoder source: its player's
 * decode loop (REF/README.md:2-3) is the path these kernels replace.
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
 */
#include <hip/hip_runtime.h>

#include "mp3d_internal.h"
#include "mp3d_tables.h"
#include "mp3d_consts.h" /* IMDCT-12 / short window / alias coefficients as literals */

namespace mp3d {

/* ------------------------------------------------------------------------ */
/* Constant-memory tables (uniform access -> scalar loads)                   */
/* ------------------------------------------------------------------------ */
__constant__ float c_win36[4][36];    /* long windows x IMDCT output scale (imdct36_w) */
__constant__ float c_is_ratio[7][2];  /* MPEG-1 intensity: k/(1+k), 1/(1+k) */
__constant__ float c_pow2q[4];        /* 2^(i/4) */
__constant__ float c_is_lsf[2][16][2];
/* Layer III frame bytes without padding per (sample-rate index 0..8,
 * bitrate index): 144000 kbps / Hz (MPEG-1), 72000 kbps / Hz (LSF); 0 for
 * free format / bad index.  A table read instead of a scalar division in
 * the per-frame header check. */
__constant__ uint16_t c_frame_bytes[9][16];/* LSF intensity [intensity_scale][is_pos]: L, R */

struct DevInfo { /* mirrors mp3d_frame_info (include/mp3d.h) */
    int32_t frame_bytes, channels, hz, layer, bitrate_kbps, samples;
};

#define REC_TAG 0x80 /* FrameRec.first_gr high bit: Xing/Info tag frame   */
#define REC_DROP 0x40 /* invalid side info (big_values > 288): dropped      */

/* ------------------------------------------------------------------------ */
/* Header / side-info helpers (ISO 2.4.1.3, 2.4.1.7)                          */
/* ------------------------------------------------------------------------ */
/* Layer III header bytes 1, 2 (after 0xFF) -> frame bytes, or -1.  MPEG-1
 * (ISO 11172-3 2.4.2.3) and MPEG-2 / 2.5 LSF (ISO 13818-3: 72000 instead of
 * 144000, LSF bitrates); kind = the stream's family (StreamState.kind: 0
 * any, 1 MPEG-1, 2 LSF) -- headers of the other family are not frames. */
__device__ __forceinline__ int hdr_kind(uint32_t b1) { return ((b1 >> 3) & 3) == 3 ? 1 : 2; }
__device__ __forceinline__ int hdr_sr_idx(uint32_t b1, uint32_t b2) {
    const uint32_t ver = (b1 >> 3) & 3, si = (b2 >> 2) & 3;
    return (int)si + (ver == 3 ? 0 : ver == 2 ? 3 : 6);
}
__device__ __forceinline__ int hdr_frame_bytes(uint32_t b1, uint32_t b2, int kind) {
    if ((b1 & 0xE0) != 0xE0 || ((b1 >> 1) & 3) != 1 || ((b1 >> 3) & 3) == 1) return -1;
    const int bi = (int)(b2 >> 4);
    if (bi == 0 || bi == 15 || ((b2 >> 2) & 3) == 3) return -1;
    if (kind && hdr_kind(b1) != kind) return -1;
    return (int)c_frame_bytes[hdr_sr_idx(b1, b2)][bi] + (int)((b2 >> 1) & 1);
}

/* bit offset of unit (gr, ch) inside the side info: MPEG-1 9-bit
 * main_data_begin, private bits, scfsi, 59-bit units; LSF 8-bit
 * main_data_begin, 1 / 2 private bits, one granule of 63-bit units */
__device__ __forceinline__ uint32_t side_unit_bit(int nch, int gr, int ch, bool lsf) {
    return lsf ? 8 + nch + 63 * ch : 9 + (nch == 1 ? 5 : 3) + 4 * nch + 59 * (gr * nch + ch);
}

/* ------------------------------------------------------------------------ */
/* k_demux: one wave per stream.  Walks the stream's frames (ISO 2.4.1.3),   */
/* maps each frame's main data into the stream's md region (bit reservoir,  */
/* ISO 2.4.3.4 main_data_begin, FFmpeg's underflow / drop rules), writes    */
/* FrameRec + per-unit side words, and copies the payload bytes into md --  */
/* the demux and the main-data gather in one pass.  The next frame's 64-B   */
/* header window is loaded while the current payload is copied, so the     */
/* serial header walk costs about one load latency per frame.              */
/* ------------------------------------------------------------------------ */
struct HdrWin {        /* 64 bytes at a stream position, spread over lanes 0..15 */
    uint32_t le;       /* lane i: little-endian dword at (pos & ~3) + 4 i        */
    uint32_t pos;
};

__device__ __forceinline__ HdrWin load_win(const uint8_t *p0, uint32_t len, uint32_t pos, int lane) {
    HdrWin w;
    w.pos = pos;
    const uint32_t a = (pos & ~3u) + 4u * (uint32_t)lane;
    /* a dword is read only if it starts inside the stream: it then cannot
     * leave the caller's allocation */
    w.le = (lane < 16 && a < len) ? *(const uint32_t *)(p0 + a) : 0u;
    return w;
}

/* byte k of the window (uniform k; k + (pos & 3) < 64) */
__device__ __forceinline__ uint32_t win_byte(const HdrWin &w, uint32_t k) {
    const uint32_t i = k + (w.pos & 3u);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)w.le, (int)(i >> 2));
    return (d >> (8 * (i & 3u))) & 0xFFu;
}

/* 64 bits of the window's big-endian bit string starting at bit b of byte
 * position (w.pos & ~3) -- per lane b (lane-varying) */
__device__ __forceinline__ uint64_t win_bits64(const HdrWin &w, uint32_t b) {
    const uint32_t be = __builtin_bswap32(w.le);
    const int wi = (int)(b >> 5);
    const uint32_t x0 = (uint32_t)__shfl((int)be, wi), x1 = (uint32_t)__shfl((int)be, wi + 1),
                   x2 = (uint32_t)__shfl((int)be, wi + 2);
    const uint32_t sh = b & 31u;
    const uint64_t hi = ((uint64_t)x0 << 32) | x1;
    return sh ? (hi << sh) | ((uint64_t)x2 >> (32 - sh)) : hi;
}

/* CRC-16 of a protected frame in the header window (ISO 11172-3 2.4.3.1;
 * FFmpeg handle_crc, AV_CRC_16_ANSI: polynomial 0x8005, MSB first, initial
 * 0xFFFF) over header bytes 2..3 and the side info, against bytes 4..5.
 * Wave-uniform bytes, so the loop runs on the scalar unit; opt-in only. */
__device__ bool crc16_ok(const HdrWin &w, uint32_t side_bytes) {
    uint32_t crc = 0xFFFFu;
    for (uint32_t i = 2; i < 6u + side_bytes; i++) {
        if (i == 4) i = 6; /* the stored CRC is not covered */
        crc ^= win_byte(w, i) << 8;
#pragma unroll
        for (int k = 0; k < 8; k++) crc = (crc & 0x8000u) ? ((crc << 1) ^ 0x8005u) & 0xFFFFu : (crc << 1) & 0xFFFFu;
    }
    return crc == ((win_byte(w, 4) << 8) | win_byte(w, 5));
}

/* Xing/Info tag + LAME encoder extension of a stream's first frame, as
 * FFmpeg's demuxer reads it (libavformat/mp3dec.c mp3_parse_info_tag):
 * "Xing"/"Info", BE32 flags, optional frame count (1), byte count (2), TOC
 * (4, 100 B), quality (8); then a 9-byte encoder string and, 21 bytes after
 * its start, BE24 = encoder delay << 12 | padding, honoured only for
 * "LAME" / "Lavf" / "Lavc" encoders.  t points at "Xing"/"Info", n bytes of
 * the frame follow it.  Returns StreamState.tag_info. */
__device__ uint32_t parse_info_tag(const uint8_t *t, uint32_t n, uint32_t &frames) {
    auto be32 = [&](uint32_t o) {
        return (uint32_t)t[o] << 24 | (uint32_t)t[o + 1] << 16 | (uint32_t)t[o + 2] << 8 | t[o + 3];
    };
    uint32_t info = MP3D_TAG_SEEN;
    if (n < 8) return info;
    const uint32_t flags = be32(4);
    uint32_t o = 8;
    if (flags & 1u) {
        if (o + 4 > n) return info;
        frames = be32(o);
        info |= MP3D_TAG_FRAMES;
        o += 4;
    }
    if (flags & 2u) o += 4;
    if (flags & 4u) o += 100;
    if (flags & 8u) o += 4;
    if (o + 24 > n) return info;
    const uint32_t ver = be32(o);
    if (ver == 0x4C414D45u /* LAME */ || ver == 0x4C617666u /* Lavf */ || ver == 0x4C617663u /* Lavc */) {
        const uint32_t v = (uint32_t)t[o + 21] << 16 | (uint32_t)t[o + 22] << 8 | t[o + 23];
        info |= MP3D_TAG_LAME | (v & 0xFFFFFFu);
    }
    return info;
}

__global__ void __launch_bounds__(64) k_demux(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                              const uint32_t *__restrict__ in_len, uint8_t *__restrict__ md,
                                              const uint64_t *__restrict__ md_off, StreamState *__restrict__ st,
                                              FrameRec *__restrict__ rec, uint64_t *__restrict__ sideu,
                                              DevInfo *__restrict__ infos, int F, int opts) {
    const int s = blockIdx.x;
    const int lane = threadIdx.x;
    const uint8_t *p0 = in + in_off[s];
    const uint32_t len = in_len[s];
    uint8_t *dst = md + md_off[s];
    StreamState &S = st[s];
    const int carry_in = S.res_len;
    const bool stream_start = S.frames == 0;
    int kind = S.kind; /* MPEG family lock (0 until the first frame) */
    for (int i = lane; i < (carry_in + 3) / 4; i += 64) ((uint32_t *)dst)[i] = ((const uint32_t *)S.res)[i];
    __threadfence_block(); /* carry words may spill past carry_in into payload 0's head */

    uint32_t P = (uint32_t)carry_in; /* md position of the next payload         */
    int avail = carry_in;            /* bytes after the previous main-data end */
    uint32_t cur = 0;
    HdrWin w = load_win(p0, len, 0, lane);
    if (stream_start && len >= 10 && win_byte(w, 0) == 'I' && win_byte(w, 1) == 'D' && win_byte(w, 2) == '3') {
        const uint32_t sz = (win_byte(w, 6) & 0x7Fu) << 21 | (win_byte(w, 7) & 0x7Fu) << 14 |
                            (win_byte(w, 8) & 0x7Fu) << 7 | (win_byte(w, 9) & 0x7Fu);
        cur = 10 + sz + ((win_byte(w, 5) & 0x10u) ? 10u : 0u);
        w = load_win(p0, len, cur, lane);
    }
    int decoded = 0;
    for (int f = 0; f < F; f++) {
        const size_t fi = (size_t)s * F + f;
        /* ---- sync: the next valid header at or after cur (resync over junk) */
        int fb = -1;
        while (cur + 4 <= len) {
            if (w.pos != cur) w = load_win(p0, len, cur, lane);
            const uint32_t lim = min(57u, len - cur - 4);
            uint32_t k = 0;
            for (; k <= lim; k++) {
                if (win_byte(w, k) == 0xFFu) {
                    fb = hdr_frame_bytes(win_byte(w, k + 1), win_byte(w, k + 2), kind);
                    if (fb > 0) break;
                }
            }
            cur += k;
            if (fb > 0) break;
        }
        FrameRec r;
        r.frame_off = 0; r.md_bit = 0; r.payload_md = P; r.frame_bytes = 0; r.payload_len = 0;
        r.hdr1 = r.hdr2 = r.hdr3 = 0; r.nch = 0; r.side_off = 4; r.first_gr = 0; r.sr_idx = 0; r.lsf = 0;
        r.payload_avail = 0;
        DevInfo inf = {0, 0, 0, 0, 0, 0};
        uint64_t sw = 0; /* lane q < 4: side word of unit q = gr * 2 + ch */
        bool copy = false;
        uint32_t src_off = 0;
        if (fb > 0) {
            if (w.pos != cur) w = load_win(p0, len, cur, lane);
            const uint32_t h1 = win_byte(w, 1), h2 = win_byte(w, 2), h3 = win_byte(w, 3);
            const int nch = (h3 >> 6) == 3 ? 1 : 2;
            const int crc = (h1 & 1) ? 0 : 2;
            const bool lsf = hdr_kind(h1) == 2;
            const int ngr = lsf ? 1 : 2;
            const int side_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
            kind = hdr_kind(h1);
            const uint32_t need = 4u + (uint32_t)crc + (uint32_t)side_bytes;
            /* a final frame cut short still decodes (FFmpeg: the missing bytes
             * read as zeros) once its header and side info are present */
            if (cur + (uint32_t)fb <= len || cur + need <= len) {
                const uint32_t have = min(len - cur, (uint32_t)fb);
                const int plen = fb - 4 - crc - side_bytes;
                r.frame_off = in_off[s] + cur;
                r.frame_bytes = (uint16_t)fb;
                r.payload_len = (uint16_t)(plen > 0 ? plen : 0);
                r.hdr1 = (uint8_t)h1; r.hdr2 = (uint8_t)h2; r.hdr3 = (uint8_t)h3;
                r.nch = (uint8_t)nch;
                r.side_off = (uint8_t)(4 + crc);
                r.sr_idx = (uint8_t)hdr_sr_idx(h1, h2);
                r.lsf = (uint8_t)lsf;
                inf.frame_bytes = fb; inf.channels = nch; inf.hz = (int)MP3D_SAMPLE_RATE[r.sr_idx];
                inf.layer = 3; inf.bitrate_kbps = lsf ? MP3D_BITRATE_L3_LSF[h2 >> 4] : MP3D_BITRATE_L3[h2 >> 4];
                /* side info: bit offsets relative to the window's dword base */
                const uint32_t sbit = 8u * ((cur & 3u) + 4u + (uint32_t)crc);
                const int mdb = (int)(win_bits64(w, sbit) >> (lsf ? 56 : 55));
                const int q = lane & 3, qgr = q >> 1, qch = q & 1;
                const uint32_t ub = sbit + side_unit_bit(nch, qgr, qch, lsf);
                const bool unit_ok = lane < 4 && qch < nch && qgr < ngr;
                uint64_t v59;
                uint32_t low5; /* side word bits 4..0: scfsi << 1 (MPEG-1) | scalefac_compress >> 4 (LSF) */
                if (lsf) {
                    /* 63-bit LSF unit (13818-3 2.4.1.7): part2_3 12, big_values 9,
                     * global_gain 8, scalefac_compress 9, window switching 1 +
                     * 22, scalefac_scale 1, count1table 1 -> the MPEG-1 layout
                     * with scalefac_compress bits 0..3 in its 4-bit slot, the
                     * intensity-right-channel flag in the preflag slot, bits
                     * 4..8 in the side word's low 5 bits */
                    const uint64_t v63 = win_bits64(w, ub) >> 1;
                    const uint32_t sfc9 = (uint32_t)(v63 >> 25) & 511u;
                    const uint64_t low25 = v63 & 0x1FFFFFFull;
                    const bool is_right = (h3 >> 6) == 1 && ((h3 >> 4) & 1) && qch == 1;
                    v59 = ((v63 >> 34) << 30) | ((uint64_t)(sfc9 & 15u) << 26) | ((low25 >> 2) << 3) |
                          ((uint64_t)is_right << 2) | (low25 & 3u);
                    low5 = sfc9 >> 4;
                } else {
                    v59 = win_bits64(w, ub) >> 5;
                    low5 = (uint32_t)(win_bits64(w, sbit + 9 + (nch == 1 ? 5 : 3) + 4 * qch) >> 60) << 1;
                }
                const uint32_t myp23 = unit_ok ? (uint32_t)(v59 >> 47) : 0u;
                /* FFmpeg drops the frame: big_values > 288, or
                 * window switching with the reserved block_type 0 */
                const bool mybad = unit_ok && (((v59 >> 38) & 0x1FFu) > 288u || (v59 & (7ull << 23)) == (4ull << 23));
                sw = unit_ok ? (v59 << 5) | low5 : 0ull;
                int p23[2][2];
                p23[0][0] = __builtin_amdgcn_readlane((int)myp23, 0);
                p23[0][1] = __builtin_amdgcn_readlane((int)myp23, 1);
                p23[1][0] = __builtin_amdgcn_readlane((int)myp23, 2);
                p23[1][1] = __builtin_amdgcn_readlane((int)myp23, 3);
                /* MP3D_OPT_CRC_CHECK: a protected frame whose CRC-16 mismatches
                 * is dropped like a bad one (FFmpeg handle_crc + explode) */
                const bool crc_bad = (opts & MP3D_OPT_CRC_CHECK) && crc && !crc16_ok(w, (uint32_t)side_bytes);
                const bool bad = plen < 0 || __ballot(mybad) != 0ull || crc_bad;
                const uint32_t tgo = 4u + (uint32_t)crc + (uint32_t)side_bytes;
                const bool tag = stream_start && f == 0 && plen >= 4 && have == (uint32_t)fb &&
                                 ((win_byte(w, tgo) == 'X' && win_byte(w, tgo + 1) == 'i' && win_byte(w, tgo + 2) == 'n' &&
                                   win_byte(w, tgo + 3) == 'g') ||
                                  (win_byte(w, tgo) == 'I' && win_byte(w, tgo + 1) == 'n' && win_byte(w, tgo + 2) == 'f' &&
                                   win_byte(w, tgo + 3) == 'o'));
                if (tag) {
                    r.first_gr = REC_TAG;
                    if (lane == 0) S.tag_info = parse_info_tag(p0 + cur + tgo, (uint32_t)fb - tgo, S.tag_frames);
                } else if (bad) {
                    /* FFmpeg drops the frame; its reservoir restarts as the frame's
                     * last min(512, bytes - 4) post-header bytes (mp_decode_frame) */
                    r.first_gr = REC_DROP;
                    r.payload_len = (uint16_t)(fb - 4);
                    avail = fb - 4 < MP3D_RES_BYTES ? fb - 4 : MP3D_RES_BYTES;
                    P += (uint32_t)r.payload_len;
                } else {
                    int gr0 = 0;
                    uint32_t mdbit;
                    if (mdb <= avail) {
                        mdbit = (P - (uint32_t)mdb) * 8u;
                    } else {
                        uint32_t bits = (uint32_t)avail * 8u;
                        while (gr0 < ngr && (int)(bits >> 3) < mdb) {
                            for (int ch = 0; ch < nch; ch++) bits += (uint32_t)p23[gr0][ch];
                            gr0++;
                        }
                        mdbit = (P - (uint32_t)avail) * 8u + bits - 8u * (uint32_t)mdb;
                    }
                    uint32_t end = mdbit;
                    for (int gr = gr0; gr < 2; gr++)
                        for (int ch = 0; ch < nch; ch++) end += (uint32_t)p23[gr][ch];
                    r.md_bit = mdbit;
                    r.first_gr = (uint8_t)gr0;
                    P += (uint32_t)plen;
                    const int64_t after = (int64_t)P - (int64_t)((end + 7u) >> 3);
                    avail = after < 0 ? 0 : (int)after;
                    inf.samples = lsf ? 576 : 1152;
                    decoded++;
                }
                const uint32_t body = (r.first_gr & REC_DROP) ? 4u : need;
                const uint32_t av = have > body ? have - body : 0u;
                r.payload_avail = (uint16_t)(av < r.payload_len ? av : r.payload_len);
                copy = !(r.first_gr & REC_TAG);
                src_off = cur + body;
                cur = have == (uint32_t)fb ? cur + (uint32_t)fb : len;
            } else {
                cur = len;
            }
        }
        /* next frame's header window in flight while this payload copies */
        if (cur + 4 <= len && f + 1 < F) w = load_win(p0, len, cur, lane);
        if (lane == 0) {
            rec[fi] = r;
            if (infos) infos[fi] = inf;
        }
        if (lane < 4) sideu[fi * 4 + lane] = sw;
        if (copy) {
            const uint8_t *src = p0 + src_off;
            const uint32_t Pm = r.payload_md, L = r.payload_avail;
            for (uint32_t i = L + lane; i < r.payload_len; i += 64) dst[Pm + i] = 0; /* cut-short final frame */
            const uint32_t h = min((4u - (Pm & 3u)) & 3u, L);     /* head bytes up to an aligned word */
            const uint32_t wb = (Pm + h) >> 2, we = (Pm + L) >> 2; /* whole words [wb, we)           */
            if ((uint32_t)lane < h) dst[Pm + lane] = src[lane];
            /* tail bytes [t0, L) after the last whole word -- or after the head
             * when there is none (an LSF payload can be < 8 bytes) */
            const uint32_t t0 = 4u * we > Pm + h ? 4u * we - Pm : h; /* h <= t0 <= L */
            if ((uint32_t)lane < L - t0) dst[Pm + t0 + lane] = src[t0 + lane];
            if (wb < we) {
                const uint64_t sa0 = (uint64_t)(src + (4u * wb - Pm));
                const uint32_t sh = (uint32_t)(sa0 & 3u) * 8u;
                const uint32_t *swd = (const uint32_t *)(sa0 & ~(uint64_t)3);
                for (uint32_t k = lane; k < we - wb; k += 64) {
                    const uint32_t lo = swd[k];
                    ((uint32_t *)dst)[wb + k] = sh ? __builtin_amdgcn_alignbit(swd[k + 1], lo, sh) : lo;
                }
            }
        }
    }
    /* carry: the last min(avail, 512) md bytes become the next call's carry-in */
    __syncthreads();
    int c = avail < MP3D_RES_BYTES ? avail : MP3D_RES_BYTES;
    if ((uint32_t)c > P) c = (int)P;
    for (int i = lane; i < c; i += 64) S.res[i] = dst[P - c + i];
    if (lane == 0) {
        S.res_len = c;
        S.frames += decoded;
        S.kind = kind;
    }
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* ------------------------------------------------------------------------ */
/* k_huffman: one lane per unit (ISO 2.4.2.7 + Annex B), 64 consecutive     */
/* units (16 frames) per wave.  Each wave first stages its units' main-data */
/* words into LDS (byte-swapped, one contiguous segment per lane, placed by */
/* a wave prefix sum; segments that do not fit are decoded in a further    */
/* batch), then decodes from LDS: a 96-bit window per codeword, two-level  */
/* u16 LUT (15 code tables + count1 table A, LDS), and linbits + sign bits */
/* taken from the same window, so the big_values loop is branch-free and   */
/* runs max(big_values) iterations per wave whatever the region tables.     */
/* Side info arrives pre-extracted by k_demux (one u64 per unit).           */
/* ------------------------------------------------------------------------ */
#define HUFF_WAVES 4
#define HUFF_ROUNDS 4                    /* 64-unit rounds per super-chunk          */
#define HUFF_SUPER (64 * HUFF_ROUNDS)    /* units ranked together by big_values     */
#define HUFF_BLOCK (64 * HUFF_WAVES)
#define HUFF_CAPW 2400 /* LDS words per wave (9.6 KB): staging + round order    */
#define HUFF_STAGEW (HUFF_CAPW - HUFF_SUPER / 2) /* staging words; the u16 order follows */

/* One wave per data region: LDS operations of a wave complete in issue
 * order, so an LDS hand-off between lanes of ONE wave only needs the
 * compiler not to reorder across it -- no s_barrier and, unlike
 * __syncthreads(), no vmcnt(0) drain of loads/stores still in flight.    */
__device__ __forceinline__ void wave_sync() { __asm__ volatile("" ::: "memory"); }

/* 64 bits of a staged (big-endian word) bitstream starting at bit pos;
 * 64-bit funnel shifts keep it branch-free (sh = 0 included) */
__device__ __forceinline__ void win64(const uint32_t *bits, uint32_t pos, uint32_t &hi, uint32_t &lo) {
    uint32_t w = pos >> 5;
    w = w < HUFF_CAPW ? w : HUFF_CAPW;
    const uint32_t sh = 32u - (pos & 31u);
    const uint32_t w0 = bits[w], w1 = bits[w + 1], w2 = bits[w + 2];
    hi = (uint32_t)((((uint64_t)w0 << 32) | w1) >> sh);
    lo = (uint32_t)((((uint64_t)w1 << 32) | w2) >> sh);
}
__device__ __forceinline__ uint32_t win32(const uint32_t *bits, uint32_t pos) {
    uint32_t w = pos >> 5;
    w = w < HUFF_CAPW ? w : HUFF_CAPW;
    const uint32_t w0 = bits[w], w1 = bits[w + 1];
    return (uint32_t)((((uint64_t)w0 << 32) | w1) >> (32u - (pos & 31u)));
}
/* top 32 bits of (hi:lo) << n, 0 <= n <= 32 */
__device__ __forceinline__ uint32_t shl64hi(uint32_t hi, uint32_t lo, uint32_t n) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (32u - n));
}

/* Scalefactors are built in 10 packed registers (byte j of UnitMeta.sf in
 * byte j & 3 of w[j >> 2]) with compile-time positions and stored with
 * three wide stores: per-byte global stores from 64 lanes to 64 different
 * records are the slow, uncoalesced store pattern of this kernel.       */
template <int BASE, int CNT>
__device__ __forceinline__ uint32_t sf_group(const uint32_t *bits, uint32_t pos, int sl, uint32_t *w) {
    uint32_t v = win32(bits, pos);
#pragma unroll
    for (int i = 0; i < CNT; i++) {
        const uint32_t x = sl ? v >> (32 - sl) : 0u;
        v = sl ? v << sl : 0u;
        const int j = BASE + i;
        w[j >> 2] = (w[j >> 2] & ~(0xFFu << (8 * (j & 3)))) | (x << (8 * (j & 3)));
    }
    return pos + (uint32_t)(CNT * sl);
}

/* Scalefactors (part 2), ISO 2.4.2.7, read in place: groups whose scfsi bit
 * is set keep the granule-0 values already in w (layout as UnitMeta.sf). */
__device__ __forceinline__ uint32_t read_sf(const uint32_t *bits, uint32_t pos, uint64_t side, int scfsi, uint32_t *w,
                                            const uint8_t *slen) {
    const int sfc = (int)(side >> 31) & 15, ws = (int)(side >> 30) & 1;
    const int bt = ws ? (int)(side >> 28) & 3 : 0, mixed = ws ? (int)(side >> 27) & 1 : 0;
    const int slen1 = slen[sfc], slen2 = slen[16 + sfc];
    if (bt == 2) {
        /* (mixed) 17 / 18 values of slen1 then 18 of slen2: written as the
         * 18 + 18 layout, then shifted down one byte from 17 when mixed */
#pragma unroll
        for (int i = 0; i < 10; i++) w[i] = 0u;
        pos = sf_group<0, 6>(bits, pos, slen1, w);
        pos = sf_group<6, 6>(bits, pos, slen1, w);
        if (mixed) pos = sf_group<12, 5>(bits, pos, slen1, w);
        else pos = sf_group<12, 6>(bits, pos, slen1, w);
        pos = sf_group<18, 6>(bits, pos, slen2, w);
        pos = sf_group<24, 6>(bits, pos, slen2, w);
        pos = sf_group<30, 6>(bits, pos, slen2, w);
        if (mixed) {
            uint32_t sh[5];
#pragma unroll
            for (int k = 0; k < 5; k++) sh[k] = __builtin_amdgcn_alignbit(w[5 + k], w[4 + k], 8);
            w[4] = (w[4] & 0xFFu) | (sh[0] & 0xFFFFFF00u);
#pragma unroll
            for (int k = 1; k < 5; k++) w[4 + k] = sh[k];
            w[9] >>= 8;
        }
    } else {
        if (!(scfsi & 8)) pos = sf_group<0, 6>(bits, pos, slen1, w);
        if (!(scfsi & 4)) pos = sf_group<6, 5>(bits, pos, slen1, w);
        if (!(scfsi & 2)) pos = sf_group<11, 5>(bits, pos, slen2, w);
        if (!(scfsi & 1)) pos = sf_group<16, 5>(bits, pos, slen2, w);
        w[5] &= 0xFFu; /* bytes 21 .. 39 are zero */
#pragma unroll
        for (int i = 6; i < 10; i++) w[i] = 0u;
    }
    return pos;
}

/* LSF scalefactors (ISO 13818-3 2.4.3.2; FFmpeg mp_decode_layer3): slen[4]
 * from the 9-bit scalefac_compress (intensity right channel: its half and
 * other ranges), group sizes from MP3D_LSF_NSF, read in coding order and
 * stored byte by byte into the canonical UnitMeta.sf layout (mixed blocks:
 * short bands from sf[8]).  LSF units only -- off the MPEG-1 path, so the
 * plain per-byte global stores are fine.  *preflag = scalefac_compress >= 500. */
typedef const __attribute__((address_space(3))) uint32_t *lds_cu32;
__device__ __attribute__((noinline)) uint32_t read_sf_lsf(lds_cu32 bits, uint32_t pos, uint64_t side, uint8_t *sf,
                                                          int *preflag) {
    const int ws = (int)(side >> 30) & 1, bt = ws ? (int)(side >> 28) & 3 : 0;
    const int tindex = bt == 2 ? (((side >> 27) & 1) ? 2 : 1) : 0;
    const bool is_right = (side >> 7) & 1;
    int sfc = (int)((side >> 31) & 15) | (int)((side & 31) << 4);
    int n1, n2, n3, t2;
    *preflag = 0;
    if (is_right) {
        sfc >>= 1;
        if (sfc < 180) { n1 = 6; n2 = 6; n3 = 0; t2 = 3; }
        else if (sfc < 244) { sfc -= 180; n1 = 4; n2 = 4; n3 = 0; t2 = 4; }
        else { sfc -= 244; n1 = 3; n2 = 0; n3 = 0; t2 = 5; }
    } else {
        if (sfc < 400) { n1 = 5; n2 = 4; n3 = 4; t2 = 0; }
        else if (sfc < 500) { sfc -= 400; n1 = 5; n2 = 4; n3 = 0; t2 = 1; }
        else { sfc -= 500; n1 = 3; n2 = 0; n3 = 0; t2 = 2; *preflag = 1; }
    }
    int slen[4];
    if (n3) { slen[3] = sfc % n3; sfc /= n3; } else slen[3] = 0;
    if (n2) { slen[2] = sfc % n2; sfc /= n2; } else slen[2] = 0;
    slen[1] = sfc % n1;
    slen[0] = sfc / n1;
    *(uint4 *)sf = make_uint4(0u, 0u, 0u, 0u);
    *(uint4 *)(sf + 16) = make_uint4(0u, 0u, 0u, 0u);
    *(uint2 *)(sf + 32) = make_uint2(0u, 0u);
    int j = 0;
    for (int k = 0; k < 4; k++) {
        const int sl = slen[k], n = MP3D_LSF_NSF[t2][tindex][k];
        for (int i = 0; i < n; i++, j++) {
            uint32_t v = 0u;
            if (sl) { /* ds_read (the staged words are LDS; no flat access) */
                const uint32_t w = pos >> 5;
                const uint64_t pr = ((uint64_t)bits[w] << 32) | bits[w + 1];
                v = (uint32_t)(pr >> (64u - (pos & 31u) - (uint32_t)sl)) & ((1u << sl) - 1u);
            }
            pos += (uint32_t)sl;
            sf[tindex == 2 && j >= 6 ? j + 2 : j] = (uint8_t)v;
        }
    }
    return pos;
}

/* is[] row writer: words (2 x int16) are shifted through 4 registers and
 * stored 16 B at a time (one dwordx4 per 8 lines instead of 4 dword stores) */
struct RowWriter {
    int16_t *out;
    uint32_t w0, w1, w2, w3;
    int nw; /* words pushed */
    __device__ __forceinline__ void push(uint32_t v) {
        w0 = w1;
        w1 = w2;
        w2 = w3;
        w3 = v;
        nw++;
        if ((nw & 3) == 0) *(uint4 *)(out + 2 * (nw - 4)) = make_uint4(w0, w1, w2, w3);
    }
    /* flush the last partial 16-B chunk.  Lines from 2 nw (UnitMeta.nz_end)
     * to 575 are the rzero region: NOT stored (k_synth masks them), which
     * removes ~2/3 of the row stores -- one row per lane is the slow,
     * uncoalesced store pattern of this kernel. */
    __device__ __forceinline__ void finish() {
        const int r = nw & 3;
        if (r == 3) *(uint4 *)(out + 2 * (nw - 3)) = make_uint4(w1, w2, w3, 0u);
        else if (r == 2) *(uint2 *)(out + 2 * (nw - 2)) = make_uint2(w2, w3);
        else if (r == 1) *(uint32_t *)(out + 2 * (nw - 1)) = w3;
    }
};

__global__ void __launch_bounds__(HUFF_BLOCK) k_huffman(const uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off,
                                                        const FrameRec *__restrict__ rec,
                                                        const uint64_t *__restrict__ sideu,
                                                        const DevTables *__restrict__ tab, int16_t *__restrict__ is_buf,
                                                        UnitMeta *__restrict__ meta, int n_units, int F) {
    __shared__ uint16_t s_lut[MP3D_LUT_MAX];
    __shared__ __attribute__((aligned(16))) uint32_t s_bits[HUFF_WAVES][HUFF_CAPW + 4];
    __shared__ uint32_t s_tsel[32]; /* table_select -> LUT base | bits1 << 16 | linbits << 24 */
    __shared__ uint16_t s_lbnd[9][24]; /* long sfb start line per sample-rate index (23 bounds) */
    __shared__ uint8_t s_slen[32];     /* MPEG-1 slen1 | slen2 per scalefac_compress          */
    const int lut_n = tab->lut_hdr.base[MP3D_LUT_TABLES - 1] + (1 << tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1]);
    const int zbase = (lut_n + 1) & ~1; /* 2-entry all-zero table for table_select 0, 4, 14 */
    for (int i = threadIdx.x; i < (lut_n + 1) / 2; i += blockDim.x)
        ((uint32_t *)s_lut)[i] = ((const uint32_t *)tab->lut)[i];
    if (threadIdx.x == 0) ((uint32_t *)s_lut)[zbase / 2] = 0u;
    if (threadIdx.x < 9) {
        int acc = 0;
        for (int i = 0; i < 22; i++) {
            s_lbnd[threadIdx.x][i] = (uint16_t)acc;
            acc += MP3D_SFB_LONG_WIDTH[threadIdx.x][i];
        }
        s_lbnd[threadIdx.x][22] = (uint16_t)acc;
    }
    if (threadIdx.x < 32) s_slen[threadIdx.x] = MP3D_SLEN[threadIdx.x >> 4][threadIdx.x & 15];
    if (threadIdx.x < 32) {
        const int t = MP3D_HTAB_OF_SELECT[threadIdx.x];
        s_tsel[threadIdx.x] = t < 0 ? (uint32_t)zbase | (1u << 16)
                                    : (uint32_t)tab->lut_hdr.base[t] | ((uint32_t)tab->lut_hdr.bits1[t] << 16) |
                                          ((uint32_t)MP3D_LINBITS[threadIdx.x] << 24);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t *bits = s_bits[wv];
    const uint32_t qbase = tab->lut_hdr.base[MP3D_LUT_TABLES - 1];
    const int qb1 = tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1];
    const int n_super = (n_units + HUFF_SUPER - 1) / HUFF_SUPER;

    for (int sc = blockIdx.x * HUFF_WAVES + wv; sc < n_super; sc += gridDim.x * HUFF_WAVES) {
        /* ---- order the super-chunk's units by big_values (counting sort in
         * LDS: histogram by ds_add_rtn, wave scan), so each 64-unit round
         * holds units of similar length -- the big_values loop runs
         * max-over-lanes iterations.  The order (u16) lives past the
         * staging area, the histogram in it. */
        const int ubase = sc * HUFF_SUPER;
        uint16_t *order16 = (uint16_t *)(bits + HUFF_STAGEW + 4);
        wave_sync();
        for (int i = lane; i < 320; i += 64) bits[i] = 0u;
        wave_sync();
        uint32_t bvk[HUFF_ROUNDS], slot[HUFF_ROUNDS];
#pragma unroll
        for (int j = 0; j < HUFF_ROUNDS; j++) {
            const int u = ubase + 64 * j + lane;
            bvk[j] = u < n_units ? (uint32_t)(sideu[u] >> 43) & 0x1FFu : 0u;
            bvk[j] = bvk[j] < 320u ? bvk[j] : 319u;
            slot[j] = atomicAdd(&bits[bvk[j]], 1u);
        }
        wave_sync();
        {   /* exclusive prefix over the 320 bins: lane owns bins 5 lane .. +4 */
            uint32_t c[5], sum = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                c[k] = bits[5 * lane + k];
                sum += c[k];
            }
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            uint32_t run = incl - sum;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                bits[5 * lane + k] = run;
                run += c[k];
            }
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < HUFF_ROUNDS; j++) order16[bits[bvk[j]] + slot[j]] = (uint16_t)(64 * j + lane);
        wave_sync();

        for (int rd = 0; rd < HUFF_ROUNDS; rd++) {
            const int u = ubase + (int)order16[64 * rd + lane];
            const int fr = u >> 2, gr = (u >> 1) & 1, ch = u & 1;
            bool valid = u < n_units;
            FrameRec r;
            uint64_t sq[4] = {0, 0, 0, 0};
            if (valid) {
                r = rec[fr];
                valid = r.frame_bytes && !(r.first_gr & (REC_TAG | REC_DROP)) && ch < r.nch && (gr == 0 || !r.lsf);
                const ulonglong2 a = *(const ulonglong2 *)&sideu[u & ~3];
                const ulonglong2 b = *(const ulonglong2 *)&sideu[(u & ~3) + 2];
                sq[0] = a.x; sq[1] = a.y; sq[2] = b.x; sq[3] = b.y;
            }
            const int first_gr = valid ? (r.first_gr & 3) : 0;
            const int nch = valid ? r.nch : 1;
            const bool dec = valid && gr >= first_gr;
            const int q = u & 3;
            const uint64_t side = sq[q];
            const uint32_t p23 = dec ? (uint32_t)(side >> 52) : 0u;
            /* unit start = md_bit + part2_3 lengths of the frame's earlier
             * decoded units (gr >= first_gr, ch < nch) */
            uint32_t before = 0;
#pragma unroll
            for (int qq = 0; qq < 3; qq++)
                if (qq < q && (qq >> 1) >= first_gr && (qq & 1) < nch) before += (uint32_t)(sq[qq] >> 52);
            const uint32_t start = dec ? r.md_bit + before : 0u;
            const int scfsi_raw = (int)(side >> 1) & 15;
            const bool long_blk = !(((side >> 30) & 1) && ((side >> 28) & 3) == 2);
            const int scfsi = (gr == 1 && long_blk) ? scfsi_raw : 0;
            const bool need_g0 = dec && scfsi && first_gr == 0;
            const uint32_t g0_start = r.md_bit + (ch ? (uint32_t)(sq[0] >> 52) : 0u);
            const uint32_t lo_bit = need_g0 ? g0_start : start;
            const uint32_t w0 = lo_bit >> 5;
            /* words [w0, w0 + len): through the unit end + 2 words of window
             * margin, rounded to 4 words (16-B LDS stores) */
            const uint32_t len = dec ? ((((start + p23 + 31) >> 5) + 2 - w0 + 3) & ~3u) : 0u;
            uint32_t incl = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            const uint32_t off = incl - len;
            const uint32_t *src = (const uint32_t *)(md + (dec ? md_off[fr / F] : 0)) + w0;

            bool pending = dec;
            while (__ballot(pending)) {
                uint32_t mo = pending ? off : 0xFFFFFFFFu;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) mo = min(mo, (uint32_t)__shfl_xor(mo, o));
                const uint32_t base = mo;
                const bool inb = pending && off + len - base <= HUFF_STAGEW;
                wave_sync();
                /* stage: each lane copies its own segment, 4 x 16 B in flight */
                if (inb) {
                    uint32_t *dst = bits + (off - base);
                    for (uint32_t i = 0; i < len; i += 16) {
                        uint4 v[4];
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if (i + 4 * k < len) v[k] = *(const uint4 *)(src + i + 4 * k);
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if (i + 4 * k < len)
                                *(uint4 *)(dst + i + 4 * k) =
                                    make_uint4(bswap32(v[k].x), bswap32(v[k].y), bswap32(v[k].z), bswap32(v[k].w));
                    }
                }
                wave_sync();
                if (inb) {
                    const uint32_t seg = 32u * (off - base) - 32u * w0; /* md bit -> staged bit */
                    uint32_t pos = start + seg;
                    int lsf_pre = 0;
                    if (r.lsf) {
                        /* off the MPEG-1 path: a call keeps its registers out of
                         * the kernel's allocation; bits passed as an LDS pointer */
                        pos = read_sf_lsf((lds_cu32)bits, pos, side, (uint8_t *)&meta[u], &lsf_pre);
                    } else {
                        uint32_t sfw[10];
#pragma unroll
                        for (int i = 0; i < 10; i++) sfw[i] = 0u;
                        if (need_g0) {
                            /* scfsi reuse: granule 0's scalefactors of this channel
                             * first, then granule 1's read over them in place */
                            read_sf(bits, g0_start + seg, sq[ch], 0, sfw, s_slen);
                        }
                        pos = read_sf(bits, pos, side, scfsi, sfw, s_slen);
                        uint8_t *mrec = (uint8_t *)&meta[u];
                        *(uint4 *)mrec = make_uint4(sfw[0], sfw[1], sfw[2], sfw[3]);
                        *(uint4 *)(mrec + 16) = make_uint4(sfw[4], sfw[5], sfw[6], sfw[7]);
                        *(uint2 *)(mrec + 32) = make_uint2(sfw[8], sfw[9]);
                    }
                    /* big_values: region boundaries (ISO 2.4.2.7; FFmpeg clamp) */
                    const int ws = (int)(side >> 30) & 1;
                    const int bv2 = 2 * ((int)(side >> 43) & 0x1FF);
                    int r1, r2;
                    uint32_t ts0, ts1, ts2;
                    if (ws) {
                        /* region0: 36 lines; FFmpeg LSF: 54 for long-type units
                         * (108 at 8 kHz), 72 for short units at 8 kHz */
                        const bool sh = ((side >> 28) & 3) == 2;
                        r1 = r.sr_idx < 3 ? 36 : sh ? (r.sr_idx == 8 ? 72 : 36) : (r.sr_idx == 8 ? 108 : 54);
                        r2 = 576;
                        ts0 = s_tsel[(side >> 22) & 31];
                        ts1 = s_tsel[(side >> 17) & 31];
                        ts2 = ts1;
                    } else {
                        const int rc0 = (int)(side >> 11) & 15, rc1 = (int)(side >> 8) & 7;
                        const int b1 = rc0 + 1;
                        int b2 = rc0 + rc1 + 2;
                        if (b2 > 22) b2 = 22;
                        r1 = s_lbnd[r.sr_idx][b1];
                        r2 = s_lbnd[r.sr_idx][b2];
                        ts0 = s_tsel[(side >> 25) & 31];
                        ts1 = s_tsel[(side >> 20) & 31];
                        ts2 = s_tsel[(side >> 15) & 31];
                    }
                    r1 = r1 < bv2 ? r1 : bv2;
                    r2 = r2 < bv2 ? r2 : bv2;
                    RowWriter rw;
                    rw.out = is_buf + (size_t)u * 576;
                    rw.nw = 0;
                    rw.w0 = rw.w1 = rw.w2 = rw.w3 = 0u;
                    int k = 0;
                    const uint32_t end_bit = start + seg + p23;
                    for (; k < bv2; k += 2) {
                        const uint32_t ts = k < r1 ? ts0 : (k < r2 ? ts1 : ts2);
                        const uint32_t tb = ts & 0xFFFFu, b1 = (ts >> 16) & 15u, lin = ts >> 24;
                        uint32_t hi, lo;
                        win64(bits, pos, hi, lo);
                        const uint32_t i1 = tb + (hi >> (32 - b1));
                        const uint32_t e1 = s_lut[i1];
                        /* second level, branch-free: i2 = i1 for a leaf */
                        const uint32_t nb = (e1 >> 11) & 15u;
                        const uint32_t sub =
                            ((e1 & 0x7FFu) << 2) + (uint32_t)((((uint64_t)hi << b1) & 0xFFFFFFFFull) >> (32u - nb));
                        const uint32_t i2 = (e1 & 0x8000u) ? sub : i1;
                        const uint32_t e = s_lut[i2];
                        const uint32_t x = (e >> 4) & 15u, y = e & 15u, len_c = (e >> 8) & 31u;
                        /* linbits and signs follow the code: <= 28 bits, all in
                         * the window (code <= 19 bits) */
                        uint32_t rb = shl64hi(hi, lo, len_c);
                        const uint32_t nx = x == 15u ? lin : 0u, ny = y == 15u ? lin : 0u;
                        const uint32_t ex = nx ? rb >> (32 - nx) : 0u;
                        rb <<= nx;
                        const uint32_t sx = x != 0u, sgx = rb >> 31;
                        rb <<= sx;
                        const uint32_t ey = ny ? rb >> (32 - ny) : 0u;
                        rb <<= ny;
                        const uint32_t sy = y != 0u, sgy = rb >> 31;
                        /* FFmpeg: no pair starts at or past the part2_3 end
                         * (a truncated unit's remaining lines read as zeros) */
                        const bool live = pos < end_bit;
                        pos += live ? len_c + nx + sx + ny + sy : 0u;
                        int X = (int)(x + ex), Y = (int)(y + ey);
                        X = !live ? 0 : (sx && sgx) ? -X : X;
                        Y = !live ? 0 : (sy && sgy) ? -Y : Y;
                        rw.push((uint32_t)(uint16_t)X | ((uint32_t)(uint16_t)Y << 16));
                    }
                    /* count1 quadruples until the part2_3 end; a quadruple that
                     * overreads it is discarded (FFmpeg) */
                    const bool c1b = (side >> 5) & 1;
                    while (k <= 572 && pos < end_bit) {
                        const uint32_t hw = win32(bits, pos);
                        uint32_t v, lq;
                        if (c1b) {
                            v = 15u - (hw >> 28);
                            lq = 4u;
                        } else {
                            const uint32_t e = s_lut[qbase + (hw >> (32 - qb1))];
                            v = e & 15u;
                            lq = (e >> 8) & 31u;
                        }
                        const uint32_t ns = __builtin_popcount(v);
                        if (pos + lq + ns > end_bit) break;
                        const uint32_t sbits = (hw << lq) >> (32 - (ns ? ns : 1));
                        int bit = (int)ns;
                        int q0 = (v >> 3) & 1, q1 = (v >> 2) & 1, q2 = (v >> 1) & 1, q3 = v & 1;
                        if (q0) { bit--; if ((sbits >> bit) & 1) q0 = -1; }
                        if (q1) { bit--; if ((sbits >> bit) & 1) q1 = -1; }
                        if (q2) { bit--; if ((sbits >> bit) & 1) q2 = -1; }
                        if (q3) { bit--; if ((sbits >> bit) & 1) q3 = -1; }
                        pos += lq + ns;
                        rw.push((uint32_t)(uint16_t)q0 | ((uint32_t)(uint16_t)q1 << 16));
                        rw.push((uint32_t)(uint16_t)q2 | ((uint32_t)(uint16_t)q3 << 16));
                        k += 4;
                    }
                    const int nz_end = 2 * rw.nw;
                    rw.finish();
                    UnitMeta m;
                    m.global_gain = (uint8_t)(side >> 35);
                    m.block_type = (uint8_t)(ws ? (side >> 28) & 3 : 0);
                    m.mixed = (uint8_t)(ws && ((side >> 28) & 3) == 2 ? (side >> 27) & 1 : 0);
                    m.scalefac_scale = (uint8_t)((side >> 6) & 1);
                    m.preflag = (uint8_t)(r.lsf ? lsf_pre : (int)((side >> 7) & 1));
                    m.sbg[0] = (uint8_t)(ws ? (side >> 14) & 7 : 0);
                    m.sbg[1] = (uint8_t)(ws ? (side >> 11) & 7 : 0);
                    m.sbg[2] = (uint8_t)(ws ? (side >> 8) & 7 : 0);
                    m.nz_end = (uint16_t)nz_end;
                    m.part2_3_length = (uint16_t)p23;
                    m.used_bits = (uint16_t)(pos - start - seg);
                    m.flags = (uint16_t)(r.lsf ? ((side >> 31) & 1) << 1 : 0); /* LSF intensity_scale */
                    /* everything after sf[40]: one 16-B store */
                    *(uint4 *)((uint8_t *)&meta[u] + 40) = *(const uint4 *)((const uint8_t *)&m + 40);
                }
                pending = pending && !inb;
            }
            if (valid && !dec) {
                /* granule lost to a reservoir underflow: silence (FFmpeg) */
                int16_t *out = is_buf + (size_t)u * 576;
                for (int kk = 0; kk < 576; kk += 8) *(uint4 *)(out + kk) = make_uint4(0, 0, 0, 0);
                UnitMeta m;
#pragma unroll
                for (int i = 0; i < 10; i++) ((uint32_t *)m.sf)[i] = 0u;
                const int ws = (int)(side >> 30) & 1;
                m.global_gain = (uint8_t)(side >> 35);
                m.block_type = (uint8_t)(ws ? (side >> 28) & 3 : 0);
                m.mixed = (uint8_t)(ws && ((side >> 28) & 3) == 2 ? (side >> 27) & 1 : 0);
                m.scalefac_scale = (uint8_t)((side >> 6) & 1);
                m.preflag = (uint8_t)(r.lsf ? 0 : (int)((side >> 7) & 1));
                m.sbg[0] = (uint8_t)(ws ? (side >> 14) & 7 : 0);
                m.sbg[1] = (uint8_t)(ws ? (side >> 11) & 7 : 0);
                m.sbg[2] = (uint8_t)(ws ? (side >> 8) & 7 : 0);
                m.nz_end = 0;
                m.part2_3_length = 0;
                m.used_bits = 0;
                m.flags = (uint16_t)(1 | (r.lsf ? ((side >> 31) & 1) << 1 : 0));
                meta[u] = m;
            }
        }
    }
}

/* 9-point DCT-III: v[n] = sum_m a[m] cos(pi m (2n+1) / 18), n = 0..8, via the
 * symmetry v[8-n] = sum_m (-1)^m a[m] cos(...): even / odd m partial sums */
__device__ __forceinline__ void dct3_9(const float *a, float *v) {
    const float C10 = 9.848077530e-01f; /* cos(10 deg) */
    const float C20 = 9.396926208e-01f; /* cos(20 deg) */
    const float C30 = 8.660254038e-01f; /* cos(30 deg) */
    const float C40 = 7.660444431e-01f; /* cos(40 deg) */
    const float C50 = 6.427876097e-01f; /* cos(50 deg) */
    const float C70 = 3.420201433e-01f; /* cos(70 deg) */
    const float C80 = 1.736481777e-01f; /* cos(80 deg) */
    const float ev0 = fmaf(a[8], C80, fmaf(a[6], 0.5f, fmaf(a[4], C40, fmaf(a[2], C20, a[0]))));
    const float od0 = fmaf(a[7], C70, fmaf(a[5], C50, fmaf(a[3], C30, a[1] * C10)));
    v[0] = ev0 + od0;
    v[8] = ev0 - od0;
    const float ev1 = fmaf(a[8], -0.5f, (fmaf(a[4], -0.5f, fmaf(a[2], 0.5f, a[0])) - a[6]));
    const float od1 = fmaf(a[7], -C30, fmaf(a[5], -C30, a[1] * C30));
    v[1] = ev1 + od1;
    v[7] = ev1 - od1;
    const float ev2 = fmaf(a[8], C40, fmaf(a[6], 0.5f, fmaf(a[4], -C20, fmaf(a[2], -C80, a[0]))));
    const float od2 = fmaf(a[7], C10, fmaf(a[5], -C70, fmaf(a[3], -C30, a[1] * C50)));
    v[2] = ev2 + od2;
    v[6] = ev2 - od2;
    const float ev3 = fmaf(a[8], -C20, fmaf(a[6], 0.5f, fmaf(a[4], C80, fmaf(a[2], -C40, a[0]))));
    const float od3 = fmaf(a[7], -C50, fmaf(a[5], C10, fmaf(a[3], -C30, a[1] * C70)));
    v[3] = ev3 + od3;
    v[5] = ev3 - od3;
    v[4] = a[0] - a[2] + a[4] - a[6] + a[8];
}


/* 36-point IMDCT of one subband's 18 lines (ISO 2.4.3.4) without the 18x36
 * matrix: x_i = y_(i+9) / -y_(26-i) / -y_(i-27) with y the 18-point DCT-IV
 * of X; y_n = w_n / (2 cos(pi (2n+1) / 72)) (scale folded into c_win36), w
 * the 18-point DCT-III of Z_k = X_k + X_(k-1), split into the 9-point
 * DCT-III of Z_2m (even) and of Z_(2m+1) + Z_(2m-1) (odd, scaled by
 * 1 / (2 cos(pi (2n+1) / 36))).  ~150 flops instead of 324 FMAs.        */
__device__ __forceinline__ void imdct36_w(const float *X, float *w) {
    float e[9], p[9], E[9], P[9];
    float zprev = 0.f;
#pragma unroll
    for (int m = 0; m < 9; m++) {
        e[m] = m ? X[2 * m] + X[2 * m - 1] : X[0];
        const float zo = X[2 * m + 1] + X[2 * m];
        p[m] = zo + zprev;
        zprev = zo;
    }
    dct3_9(e, E);
    dct3_9(p, P);
    const float K[9] = {5.019099188e-01f, 5.176380902e-01f, 5.516889595e-01f, 6.103872944e-01f, 7.071067812e-01f,
                        8.717233978e-01f, 1.183100792e+00f, 1.931851653e+00f, 5.736856623e+00f};
#pragma unroll
    for (int n = 0; n < 9; n++) {
        const float o = P[n] * K[n];
        w[n] = E[n] + o;
        w[17 - n] = E[n] - o;
    }
}

/* ------------------------------------------------------------------------ */
/* k_synth: one wave (64 lanes) per stream, frames and granules in order,   */
/* SYN_WAVES streams per workgroup sharing the read-only tables in LDS      */
/* (line tables of the variant's sample rates, |is|^(4/3), long windows,  */
/* the intensity ratios, the matrixing A fragments and the synthesis       */
/* window): after the prologue the granule loop issues no vector-memory    */
/* load but the one-granule-ahead                                           */
/* prefetch of is[] / UnitMeta / FrameRec, so no s_waitcnt vmcnt drains the */
/* PCM stores or the prefetch early.  Every phase exchanges data through   */
/* ONE 5 KB per-wave LDS buffer; a wave keeps only the per-stream state     */
/* (IMDCT overlap, synthesis history) in VGPRs.                             */
/*  Q  lane = line pair: requantise both channels (ISO 2.4.3.4, per-band   */
/*     2^(q/4) precomputed by lane = band), joint stereo paired by          */
/*     bitstream line, scatter into LDS in short-block reordered position.  */
/*  I  lane = (ch, sb): alias reduction (neighbours read from LDS), IMDCT   */
/*     36 / 3x12 + window + overlap + frequency inversion -> S[ch,t][sb].   */
/*  M  32-point matrixing X = C.S on the matrix cores (v_mfma_f32_16x16x4): */
/*     rows m, cols (ch, t), K = sb; A = C fragments, B = S rows (LDS).     */
/*  W  lane = (ch, j): 512-tap window over 16 slots; the 29 X values of the */
/*     previous granule this lane needs live in registers -> int16 PCM,     */
/*     L/R pairs joined across the half-waves (v_permlane32_swap) into one  */
/*     4-B store per lane and slot pair.                                    */
/* Templates: SRC_XR config-2 entry (spectra given as f32 xr, after        */
/* stereo); F32 float PCM sink; LSF MPEG-2 / 2.5 streams (one granule per  */
/* frame, LSF rates and intensity ratios) -- each launch decodes only the  */
/* streams of its MPEG family (StreamState.kind).                           */
/* ------------------------------------------------------------------------ */
#define SYN_WAVES 4
#define SROW 36      /* LDS row stride of S (floats): 16-B rows, few conflicts */
#define SYN_BUF 1296 /* floats: max(xr 2x576, S 36x36, X 36x36)              */
#define XROW 36      /* LDS row stride of X: 16-B rows, conflict-free b128 writes */

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

/* Opaque copy of a loop-invariant LDS index: keeps the compiler from
 * hoisting one address VGPR per unrolled access out of the frame loop
 * (it would rather hold ~60 of them live than fold immediate offsets). */
__device__ __forceinline__ int opaque(int v) {
    __asm__ volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ float pow2_quarter(int q) { /* 2^(q/4), exact table */
    const int r = q & 3;
    const float f = r == 0 ? 1.0f : r == 1 ? 1.18920711500272106672f : r == 2 ? 1.41421356237309504880f
                                                                              : 1.68179283050742908606f;
    return ldexpf(f, q >> 2);
}

/* |is|^(4/3) for 256 <= |is| <= 8206 without the 33 KB table: cube root
 * from v_log_f32 / v_exp_f32, one Newton step, times |is|; within 2 ulp of
 * the correctly rounded value for every such |is| (checked exhaustively in
 * tests/test_tables.py against the same float32 recipe). */
__device__ __forceinline__ float pow43_big(int a) {
    const float x = (float)a;
    float y = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(x) * (1.0f / 3.0f));
    const float y2 = y * y;
    y = y - fmaf(y2, y, -x) * __builtin_amdgcn_rcpf(3.0f * y2);
    return x * y;
}

template <bool LSF> struct SynShared { /* read-only, one copy per workgroup        */
    /* tab->lvar (u16 pairs) [rate][variant] of the variant's family: MPEG-1
     * rates 0..2, or the six LSF rates 3..8                                */
    uint32_t lvar[LSF ? 6 : 3][3][288];
    float ce[16][16], co[16][16];    /* matrixing A: C[2m][i], C[2m+1][i], i < 16  */
    float dw[32][16];                /* window taps per output j                   */
    float p43[256];                  /* |is|^(4/3) for |is| < 256                  */
    float w36[4][36];                /* long-block windows (x IMDCT output scale)  */
    float isr[LSF ? 32 : 7][2];      /* intensity ratios: MPEG-1 [is_pos], LSF      */
                                     /* [intensity_scale * 16 + is_pos]            */
};
struct SynWave {                     /* one per wave (stream)                      */
    float buf[SYN_BUF];              /* xr -> S -> X hand-offs                     */
    float scale[2][64];              /* 2^(q/4) per (ch, band idx): long b | 22 + 3 b + w */
    UnitMeta m[2];
    uint8_t is[64];                  /* intensity position per right band idx, 0xFF none */
};

#define WAIT_VMCNT0() __builtin_amdgcn_s_waitcnt(0x0F70) /* vmcnt(0), other counters free */

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <bool SRC_XR, bool F32, bool LSF>
__global__ void __launch_bounds__(64 * SYN_WAVES) __attribute__((amdgpu_waves_per_eu(3, 8)))
k_synth(const FrameRec *__restrict__ rec, const int16_t *__restrict__ is_buf, const UnitMeta *__restrict__ meta,
        const float *__restrict__ xr_in, const uint8_t *__restrict__ xr_bt, const uint8_t *__restrict__ xr_mixed,
        const DevTables *__restrict__ tab, StreamState *__restrict__ st, void *__restrict__ pcm, int n_streams,
        int F, int xr_nch, int xr_sr) {
    __shared__ __attribute__((aligned(16))) SynShared<LSF> T;
    __shared__ __attribute__((aligned(16))) SynWave Wv[SYN_WAVES];
    constexpr int NRATE = LSF ? 6 : 3;
    if (!SRC_XR) {
        /* one variant per MPEG family (StreamState.kind, fixed by k_demux):
         * MPEG-1 takes kinds 0 / 1, LSF kind 2.  A workgroup holding no
         * stream of its variant leaves before staging any table (the same
         * decision in every lane: no barrier is skipped by part of it). */
        bool any = false;
#pragma unroll
        for (int k = 0; k < SYN_WAVES; k++) {
            const int sk = blockIdx.x * SYN_WAVES + k;
            if (sk < n_streams) any |= (st[sk].kind == 2) == LSF;
        }
        if (!any) return;
    }
    {
        const int tid = threadIdx.x;
        for (int i = tid; i < NRATE * 3 * 288; i += 64 * SYN_WAVES)
            (&T.lvar[0][0][0])[i] = ((const uint32_t *)&tab->lvar[LSF ? 3 : 0][0][0])[i];
        for (int i = tid; i < 256; i += 64 * SYN_WAVES) {
            const int r = i >> 4, c = i & 15;
            T.ce[r][c] = tab->dct_c[2 * r][c];
            T.co[r][c] = tab->dct_c[2 * r + 1][c];
            T.p43[i] = tab->pow43[i];
        }
        for (int i = tid; i < 32 * 16; i += 64 * SYN_WAVES) (&T.dw[0][0])[i] = (&tab->dwin[0][0])[i];
        for (int i = tid; i < 4 * 36; i += 64 * SYN_WAVES) (&T.w36[0][0])[i] = (&c_win36[0][0])[i];
        if (LSF) {
            if (tid < 64) (&T.isr[0][0])[tid] = (&c_is_lsf[0][0][0])[tid];
        } else if (tid < 14) (&T.isr[0][0])[tid] = (&c_is_ratio[0][0])[tid];
        __syncthreads();
    }
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); /* wave-uniform (SGPR) */
    const int s = blockIdx.x * SYN_WAVES + wid;
    if (s >= n_streams) return; /* after the only workgroup barrier */
    if (!SRC_XR && (st[s].kind == 2) != LSF) return; /* the other variant's stream */
    SynWave &Wd = Wv[wid];
    float *const sBuf = Wd.buf;
    const int lane = threadIdx.x & 63;
    const int ch = lane >> 5;
    const int sb = lane & 31; /* phase I: subband; phase W: output j */
    constexpr int MW = (int)(sizeof(UnitMeta) / 4); /* 14 words per unit */

    StreamState &S = st[s];
    const int wa = tab->win_a[sb], wb = tab->win_b[sb];
    float ov[18];
#pragma unroll
    for (int i = 0; i < 18; i++) ov[i] = S.overlap[ch][sb][i];
    /* synthesis history: ha[k] = X_{k-14}[wa], hb[k] = X_{k-15}[wb] (slot
     * index relative to the granule's first slot; fifo[t] = slot t - 15)  */
    float ha[14], hb[15];
#pragma unroll
    for (int k = 0; k < 14; k++) ha[k] = S.fifo[ch][k + 1][wa];
#pragma unroll
    for (int k = 0; k < 15; k++) hb[k] = S.fifo[ch][k][wb];

    /* Per-stream buffer resources: every granule access below is a buffer
     * instruction with a uniform byte offset in an SGPR and the lane offset
     * in one VGPR, instead of a 64-bit address pair per lane and load. */
    const int gb = 2 * 576 * 2;                   /* is[] bytes per granule (2 ch) */
    const __amdgpu_buffer_rsrc_t r_is = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(is_buf + (size_t)s * F * 4 * 576), 0, F * 2 * gb, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_meta = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(meta + (size_t)s * F * 4), 0, F * 4 * (int)sizeof(UnitMeta), 0x00020000);
    const __amdgpu_buffer_rsrc_t r_rec = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(rec + (size_t)s * F), 0, F * (int)sizeof(FrameRec), 0x00020000);
    constexpr int PB = F32 ? 4 : 2; /* bytes per output sample: f32 or int16 */
    const __amdgpu_buffer_rsrc_t r_pcm = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((uint8_t *)pcm + (size_t)s * F * 2304 * PB), 0, F * 2304 * PB, 0x00020000);

    /* granule prefetch, one granule ahead of use: is[] words (lane owns
     * lines 2 lane + 128 i, +1), UnitMeta words of both channels (lanes
     * 0 .. 27) and the granule's FrameRec words (lanes 32 .. 39) */
    uint32_t nis[2][5], nmeta = 0;
    auto prefetch = [&](int g) { /* g = granule index inside the stream */
        const int lo = opaque(lane * 4);
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int i = 0; i < 4; i++)
                nis[c][i] = __builtin_amdgcn_raw_buffer_load_b32(r_is, lo + c * 1152 + 256 * i, g * gb, 0);
        nis[0][4] = nis[1][4] = 0u;
        if (lane < 32) {
            nis[0][4] = __builtin_amdgcn_raw_buffer_load_b32(r_is, lo + 1024, g * gb, 0);
            nis[1][4] = __builtin_amdgcn_raw_buffer_load_b32(r_is, lo + 1152 + 1024, g * gb, 0);
        }
        nmeta = 0u;
        if (lane < 2 * MW) nmeta = __builtin_amdgcn_raw_buffer_load_b32(r_meta, lo, g * 2 * (int)sizeof(UnitMeta), 0);
        else if (lane >= 32 && lane < 40)
            nmeta = __builtin_amdgcn_raw_buffer_load_b32(r_rec, lo - 128, (g >> 1) * (int)sizeof(FrameRec), 0);
    };
    if (!SRC_XR) {
        prefetch(0);
        /* explicit drain on the entry path, so the compiler's wait before
         * each prefetch use is set by the loop path (stores after it) */
        WAIT_VMCNT0();
    }

    for (int f = 0; f < F; f++) {
        int nch, sr, mode = 0, mext = 0;
        const size_t fr = (size_t)s * F + f;
        if (SRC_XR) {
            nch = xr_nch;
            sr = xr_sr;
        } else {
            /* FrameRec words 4 .. 6 from the prefetch (lanes 36 .. 38) */
            const uint32_t r4 = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 36);
            const uint32_t r5 = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 37);
            const uint32_t r6 = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 38);
            const uint32_t first_gr = (r6 >> 8) & 0xFFu;
            if (!(r4 & 0xFFFFu) || (first_gr & (REC_TAG | REC_DROP))) {
                /* no audio in this frame: fetch the next frame's granule 0
                 * now and wait for it here, off the common path */
                if (f + 1 < F) prefetch(2 * (f + 1));
                WAIT_VMCNT0();
                continue;
            }
            nch = (int)(r5 >> 24);
            sr = (int)((r6 >> 16) & 15u) - (LSF ? 3 : 0); /* FrameRec.sr_idx in the family */
            mode = (int)(r5 >> 22) & 3;
            mext = (int)(r5 >> 20) & 3;
        }
        const bool active = ch < nch;
        const uint32_t(*lvar)[288] = T.lvar[sr];
        for (int gr = 0; gr < (LSF ? 1 : 2); gr++) { /* LSF: one granule per frame */
            /* lane-derived indices are re-derived from an opaque copy each
             * granule so they are not hoisted and held live across the loop */
            const int lane = opaque((int)(threadIdx.x & 63));
            const int ch = lane >> 5, sb = lane & 31;
            /* block structure of both channels (uniform) */
            int bt0, mx0, bt1 = 0, mx1 = 0;
            /* ---------------- phase Q: requantise + stereo -> LDS ---------- */
            if (SRC_XR) {
                const size_t ux = (fr * 2 + gr) * (size_t)nch;
                bt0 = xr_bt[ux];
                mx0 = bt0 == 2 ? xr_mixed[ux] : 0;
                if (nch == 2) {
                    bt1 = xr_bt[ux + 1];
                    mx1 = bt1 == 2 ? xr_mixed[ux + 1] : 0;
                }
                const uint16_t *lv0 = (const uint16_t *)lvar[bt0 == 2 ? (mx0 ? 2 : 1) : 0];
                const uint16_t *lv1 = (const uint16_t *)lvar[bt1 == 2 ? (mx1 ? 2 : 1) : 0];
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    const int l = lane + 64 * i;
                    sBuf[lv0[l] >> 6] = xr_in[ux * 576 + l];
                    if (nch == 2) sBuf[576 + (lv1[l] >> 6)] = xr_in[(ux + 1) * 576 + l];
                }
            } else {
                uint32_t cis[2][5];
#pragma unroll
                for (int c = 0; c < 2; c++)
#pragma unroll
                    for (int i = 0; i < 5; i++) cis[c][i] = nis[c][i];
                /* UnitMeta into LDS for the (rare) intensity path; the common
                 * path reads the prefetched words straight from registers */
                if (lane < 2 * MW && lane / MW < nch) ((uint32_t *)&Wd.m[0])[lane] = nmeta;
                /* words 10..12: gain, block type, mixed, scalefac_scale |
                 * preflag, sbg[3] | nz_end (UnitMeta layout) */
                const uint32_t m10a = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 10);
                const uint32_t m11a = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 11);
                const uint32_t m12a = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, 12);
                const uint32_t m10b = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, MW + 10);
                const uint32_t m11b = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, MW + 11);
                const uint32_t m12b = (uint32_t)__builtin_amdgcn_readlane((int)nmeta, MW + 12);
                bt0 = (int)(m10a >> 8) & 0xFF;
                mx0 = (int)(m10a >> 16) & 0xFF;
                if (nch == 2) {
                    bt1 = (int)(m10b >> 8) & 0xFF;
                    mx1 = (int)(m10b >> 16) & 0xFF;
                }
                const int var[2] = {bt0 == 2 ? (mx0 ? 2 : 1) : 0, bt1 == 2 ? (mx1 ? 2 : 1) : 0};
                const bool is_on = mode == 1 && nch == 2 && (mext & 1);
                const bool ms_fold = mode == 1 && nch == 2 && mext == 2; /* M/S only: 1/sqrt2 in the scale */
                const float isq = 0.70710678118654752f;
                /* per-band scale 2^(q/4), lane = band idx (long b | 22 + 3 b + w);
                 * the lane's scalefactor byte comes from the prefetched meta
                 * words by one cross-lane read per channel */
                {
                    const bool lng = lane < 22;
                    const int b = (lane - 22) / 3, w = lane - 22 - 3 * b;
                    auto band_scale = [&](uint32_t g10, uint32_t g11, int cbase) {
                        const int gain = (int)(g10 & 0xFFu) - 210, shift = (int)(g10 >> 24) + 1;
                        const bool mixed = ((g10 >> 16) & 0xFFu) != 0u, preflag = (g11 & 0xFFu) != 0u;
                        int j = mixed ? 8 + 3 * (b - 3) + w : 3 * b + w;
                        j = lng ? lane : (j < 0 ? 0 : (j > 39 ? 39 : j));
                        const uint32_t wd = (uint32_t)__shfl((int)nmeta, cbase + (j >> 2));
                        const int sf = (int)(wd >> (8 * (j & 3))) & 0xFF;
                        const int pre = preflag ? (int)(MP3D_PRETAB_BITS >> (2 * (lane & 31))) & 3 : 0;
                        const int sbg = (int)(g11 >> (8 * (1 + (w < 3 ? w : 0)))) & 0xFF;
                        const int q = lng ? gain - ((sf + pre) << shift) : gain - 8 * sbg - (sf << shift);
                        return ms_fold ? pow2_quarter(q) * isq : pow2_quarter(q);
                    };
                    Wd.scale[0][lane] = band_scale(m10a, m11a, 0);
                    if (nch == 2) Wd.scale[1][lane] = band_scale(m10b, m11b, MW);
                }
                wave_sync();
                const int nz[2] = {(int)(m12a & 0xFFFFu), nch == 2 ? (int)(m12b & 0xFFFFu) : 0};
                float xv[2][10];
                bool big = false; /* some |is| >= 256 (escape) in this lane */
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    const int l0 = 2 * lane + 128 * i;
                    const bool ok = i < 4 || lane < 32;
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        const uint32_t tv2 = ok ? lvar[var[c]][l0 >> 1] : 0u;
#pragma unroll
                        for (int e = 0; e < 2; e++) {
                            const int l = l0 + e;
                            int v = (int)(int16_t)(e ? (cis[c][i] >> 16) : (cis[c][i] & 0xFFFFu));
                            v = l < nz[c] ? v : 0; /* rzero lines are not stored by k_huffman */
                            const int a = v < 0 ? -v : v;
                            big |= a >= 256;
                            const float mag = T.p43[a & 255] * Wd.scale[c][(e ? tv2 >> 16 : tv2) & 63u];
                            xv[c][2 * i + e] = v < 0 ? -mag : mag;
                        }
                    }
                }
                if (__ballot(big)) {
                    /* rare path (escapes |is| >= 256): patch those lines with
                     * the in-register |is|^(4/3); one block, so the loop above
                     * stays branch-free and its LDS reads batch */
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const int l0 = 2 * lane + 128 * i;
#pragma unroll
                        for (int c = 0; c < 2; c++) {
#pragma unroll
                            for (int e = 0; e < 2; e++) {
                                int v = (int)(int16_t)(e ? (cis[c][i] >> 16) : (cis[c][i] & 0xFFFFu));
                                v = l0 + e < nz[c] ? v : 0;
                                const int a = v < 0 ? -v : v;
                                if (a >= 256) {
                                    const uint32_t tv2 = lvar[var[c]][l0 >> 1];
                                    const float mag = pow43_big(a) * Wd.scale[c][(e ? tv2 >> 16 : tv2) & 63u];
                                    xv[c][2 * i + e] = v < 0 ? -mag : mag;
                                }
                            }
                        }
                    }
                }
                if (is_on) {
                    /* joint stereo with MPEG-1 intensity (ISO 2.4.3.4), paired by
                     * bitstream line; the right channel's block structure and
                     * its highest nonzero band (per window) decide the IS bands
                     * (FFmpeg compute_stereo; oracle/mp3_oracle.c orc_stereo).
                     * nzR bit = right-channel band idx holding a nonzero line. */
                    /* no intensity for is_pos >= 7 (MPEG-1), >= 16 (LSF, FFmpeg) */
                    constexpr int IS_ILLEGAL = LSF ? 16 : 7;
                    uint64_t nzR = 0;
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const int l0 = 2 * lane + 128 * i;
                        const uint32_t tv2 = (i < 4 || lane < 32) ? lvar[var[1]][l0 >> 1] : 0u;
                        if (xv[1][2 * i] != 0.f) nzR |= 1ull << (tv2 & 63u);
                        if (xv[1][2 * i + 1] != 0.f) nzR |= 1ull << ((tv2 >> 16) & 63u);
                    }
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) nzR |= __shfl_xor(nzR, o);
                    const UnitMeta &R = Wd.m[1];
                    int ip = 0xFF;
                    if (lane < 22) {
                        /* long bands of a mixed block: 8 (MPEG-1), 6 (LSF) */
                        if (bt1 != 2 || (mx1 && lane < (LSF ? 6 : 8))) {
                            const int p = R.sf[lane == 21 ? 20 : lane];
                            const bool short_nz = (nzR >> 22) != 0ull;
                            if (!short_nz && ((uint32_t)(nzR & 0x3FFFFFull) >> lane) == 0u && p < IS_ILLEGAL) ip = p;
                        }
                    } else if (lane < 61 && bt1 == 2) {
                        const int b = (lane - 22) / 3, w = lane - 22 - 3 * b;
                        if (!mx1 || b >= 3) {
                            const int kb = b == 12 ? 11 : b;
                            const int p = R.sf[mx1 ? 8 + 3 * (kb - 3) + w : 3 * kb + w];
                            /* no nonzero line in window w at bands >= b */
                            uint64_t above = 0;
                            for (int bb = b; bb < 13; bb++) above |= 1ull << (22 + 3 * bb + w);
                            if ((nzR & above) == 0ull && p < IS_ILLEGAL) ip = p;
                        }
                    }
                    /* LSF: ratio row by intensity_scale (UnitMeta.flags bit 1) */
                    if (LSF && ip != 0xFF) ip += (int)(R.flags & 2u) << 3;
                    Wd.is[lane] = (uint8_t)ip;
                    wave_sync();
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const int l0 = 2 * lane + 128 * i;
                        const uint32_t tv2 = (i < 4 || lane < 32) ? lvar[var[1]][l0 >> 1] : 0u;
#pragma unroll
                        for (int e = 0; e < 2; e++) {
                            const int k = 2 * i + e;
                            const float lv = xv[0][k], rv = xv[1][k];
                            const int ipl = Wd.is[(e ? tv2 >> 16 : tv2) & 63u];
                            if (ipl != 0xFF) {
                                xv[0][k] = lv * T.isr[ipl][0];
                                xv[1][k] = lv * T.isr[ipl][1];
                            } else if (mext & 2) {
                                xv[0][k] = (lv + rv) * isq;
                                xv[1][k] = (lv - rv) * isq;
                            }
                        }
                    }
                } else if (ms_fold) {
#pragma unroll
                    for (int k = 0; k < 10; k++) {
                        const float lv = xv[0][k], rv = xv[1][k];
                        xv[0][k] = lv + rv;
                        xv[1][k] = lv - rv;
                    }
                }
                /* the next granule's loads fly during phases I, M, W (issued
                 * after cis is consumed: fewer live registers in phase Q) */
                if (LSF ? f + 1 < F : (gr == 0 || f + 1 < F)) prefetch(LSF ? 2 * f + 2 : 2 * f + gr + 1);
                /* scatter in (short-block reordered) position */
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    if (i < 4 || lane < 32) {
                        const int l0 = 2 * lane + 128 * i;
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            if (c < nch) {
                                if (var[c] == 0) { /* long block: in place, one 8-B store */
                                    *(float2 *)&sBuf[576 * c + l0] = make_float2(xv[c][2 * i], xv[c][2 * i + 1]);
                                } else {
                                    const uint32_t tv2 = lvar[var[c]][l0 >> 1];
                                    sBuf[576 * c + (tv2 >> 6 & 1023u)] = xv[c][2 * i];
                                    sBuf[576 * c + (tv2 >> 22)] = xv[c][2 * i + 1];
                                }
                            }
                        }
                    }
                }
            }
            wave_sync();
            /* ---------------- phase I: alias + IMDCT + overlap ------------ */
            const int bt = ch ? bt1 : bt0, mixed = ch ? mx1 : mx0;
            float o18[18];
            {
                const int base = ch * 576 + 18 * sb;
                float x[18], up[8], dn[8];
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    const float2 v = *(const float2 *)&sBuf[base + 2 * i];
                    x[2 * i] = v.x;
                    x[2 * i + 1] = v.y;
                }
                const int pb = sb ? base - 8 : base, nb = sb < 31 ? base + 18 : base;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float2 p = *(const float2 *)&sBuf[pb + 2 * i];
                    const float2 n = *(const float2 *)&sBuf[nb + 2 * i];
                    up[7 - 2 * i] = p.x; /* up[k] = x_{sb-1}[17 - k] */
                    up[6 - 2 * i] = p.y;
                    dn[2 * i] = n.x;     /* dn[k] = x_{sb+1}[k]      */
                    dn[2 * i + 1] = n.y;
                }
                /* alias reduction (ISO 2.4.3.4): all 31 boundaries (long),
                 * the first one (mixed), none (short) */
                const bool upper = (bt != 2 && sb >= 1) || (bt == 2 && mixed && sb == 1);
                const bool lower = (bt != 2 && sb <= 30) || (bt == 2 && mixed && sb == 0);
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const float lo = x[17 - k], hi = x[k];
                    if (upper) x[k] = hi * MP3D_K_ALIAS_CS[k] + up[k] * MP3D_K_ALIAS_CA[k];
                    if (lower) x[17 - k] = lo * MP3D_K_ALIAS_CS[k] - dn[k] * MP3D_K_ALIAS_CA[k];
                }
                const bool long_imdct = bt != 2 || (mixed && sb < 2);
                if (long_imdct) {
                    const float *wv = T.w36[bt == 2 ? 0 : bt];
                    float w[18];
                    imdct36_w(x, w);
#pragma unroll
                    for (int i = 0; i < 9; i++) {
                        o18[i] = fmaf(w[9 + i], wv[i], ov[i]);
                        o18[17 - i] = fmaf(w[9 + i], wv[17 - i], ov[17 - i]);
                        const float n0 = w[8 - i] * wv[18 + i];
                        const float n1 = w[8 - i] * wv[35 - i];
                        ov[i] = active ? n0 : ov[i];
                        ov[17 - i] = active ? n1 : ov[17 - i];
                    }
                } else {
                    /* z[6w+6+i] += y_w[i] * win12[i], w = 0..2, i = 0..11 */
                    float z[24]; /* z[6..29] */
#pragma unroll
                    for (int i = 0; i < 24; i++) z[i] = 0.f;
#pragma unroll
                    for (int w = 0; w < 3; w++) {
                        float h[6];
#pragma unroll
                        for (int o = 0; o < 6; o++) {
                            float acc = 0.f;
#pragma unroll
                            for (int k = 0; k < 6; k++) acc = fmaf(x[3 * k + w], MP3D_K_IMDCT12[k][o], acc);
                            h[o] = acc;
                        }
#pragma unroll
                        for (int i = 0; i < 3; i++) {
                            z[6 * w + i] = fmaf(h[i], MP3D_K_WIN12[i], z[6 * w + i]);
                            z[6 * w + 5 - i] = fmaf(-h[i], MP3D_K_WIN12[5 - i], z[6 * w + 5 - i]);
                            z[6 * w + 6 + i] = fmaf(h[3 + i], MP3D_K_WIN12[6 + i], z[6 * w + 6 + i]);
                            z[6 * w + 11 - i] = fmaf(h[3 + i], MP3D_K_WIN12[11 - i], z[6 * w + 11 - i]);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 18; i++) o18[i] = (i < 6 ? 0.f : z[i - 6]) + ov[i];
#pragma unroll
                    for (int i = 0; i < 18; i++) {
                        const float n = i < 12 ? z[12 + i] : 0.f;
                        ov[i] = active ? n : ov[i];
                    }
                }
            }
            wave_sync(); /* every lane has read its xr before S overwrites it */
            {
                const int sw = opaque(18 * ch * SROW + sb);
#pragma unroll
                for (int t = 0; t < 18; t++) sBuf[sw + t * SROW] = ((sb & 1) && (t & 1)) ? -o18[t] : o18[t];
            }
            wave_sync();
            /* ---------------- phase M: matrixing on the matrix cores ------- */
            /* one butterfly level of the 32-point DCT-II (ISO Annex A matrixing):
             *   X[2m]   = sum_i C[2m][i]   (S_i + S_31-i)
             *   X[2m+1] = sum_i C[2m+1][i] (S_i - S_31-i),  i, m < 16
             * = two 16x16 products: half the MFMAs of the dense 32x32.
             * v_mfma_f32_16x16x4_f32, rows m, cols n = (ch, t), K order
             * i = 4 q + ks (q = lane >> 4): a lane's 4 B values and their
             * mirrors are two 16-B runs of an S row. */
            {
                const int q = lane >> 4, r16 = lane & 15;
                const float4 ae = *(const float4 *)&T.ce[r16][4 * q];
                const float4 ao = *(const float4 *)&T.co[r16][4 * q];
                const float Ae[4] = {ae.x, ae.y, ae.z, ae.w}, Ao[4] = {ao.x, ao.y, ao.z, ao.w};
                float Be[3][4], Bo[3][4];
#pragma unroll
                for (int nt = 0; nt < 3; nt++) {
                    int n = 16 * nt + r16;
                    n = n < 36 ? n : 35;
                    const float4 a4 = *(const float4 *)&sBuf[n * SROW + 4 * q];
                    const float4 b4 = *(const float4 *)&sBuf[n * SROW + 28 - 4 * q]; /* S[31-i] = b4[3-ks] */
                    const float av[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {b4.w, b4.z, b4.y, b4.x};
#pragma unroll
                    for (int ks = 0; ks < 4; ks++) {
                        Be[nt][ks] = av[ks] + bv[ks];
                        Bo[nt][ks] = av[ks] - bv[ks];
                    }
                }
                f32x4 ce[3], co[3];
#pragma unroll
                for (int nt = 0; nt < 3; nt++) ce[nt] = co[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 4; ks++)
#pragma unroll
                    for (int nt = 0; nt < 3; nt++) {
                        ce[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ae[ks], Be[nt][ks], ce[nt], 0, 0, 0);
                        co[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ao[ks], Bo[nt][ks], co[nt], 0, 0, 0);
                    }
                wave_sync(); /* all S reads retired before X overwrites them */
                /* D[row m = 4 q + r][col n] -> X[n][2m] (even), X[n][2m+1] (odd) */
#pragma unroll
                for (int nt = 0; nt < 3; nt++) {
                    const int n = 16 * nt + r16;
                    if (n < 36) {
                        *(f32x4 *)&sBuf[n * XROW + 8 * q] = (f32x4){ce[nt][0], co[nt][0], ce[nt][1], co[nt][1]};
                        *(f32x4 *)&sBuf[n * XROW + 8 * q + 4] = (f32x4){ce[nt][2], co[nt][2], ce[nt][3], co[nt][3]};
                    }
                }
            }
            wave_sync();
            /* ---------------- phase W: 512-tap window -> PCM --------------- */
            {
                float Dw[16];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float4 d = *(const float4 *)&T.dw[sb][4 * i];
                    Dw[4 * i] = d.x; Dw[4 * i + 1] = d.y; Dw[4 * i + 2] = d.z; Dw[4 * i + 3] = d.w;
                }
                float xa[18], xb[18];
                const int pa = opaque(18 * ch * XROW + wa), pb = opaque(18 * ch * XROW + wb);
#pragma unroll
                for (int t = 0; t < 18; t++) {
                    xa[t] = sBuf[pa + t * XROW];
                    xb[t] = sBuf[pb + t * XROW];
                }
                /* output slots in pairs (t0, t1): lanes 0-31 hold L, lanes
                 * 32-63 R; one half-wave swap leaves lane j with (L, R) of
                 * slot t0 and lane 32 + j with (L, R) of slot t1 */
                /* two output slots (2 tp, 2 tp + 1) at once: packed FMAs
                 * (v_pk_fma_f32, tap broadcast), half the VALU issues of the
                 * scalar form; the same fma order per slot, so bit-identical */
                auto out2 = [&](int tp) {
                    f32x2 o = {0.f, 0.f};
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int ka = 2 * tp - 2 * i, kb = ka - 1;
                        f32x2 va, vb;
                        va.x = ka >= 0 ? xa[ka] : ha[ka + 14];
                        va.y = ka + 1 >= 0 ? xa[ka + 1] : ha[ka + 15];
                        vb.x = kb >= 0 ? xb[kb] : hb[kb + 15];
                        vb.y = kb + 1 >= 0 ? xb[kb + 1] : hb[kb + 16];
                        o = __builtin_elementwise_fma((f32x2){Dw[2 * i], Dw[2 * i]}, va, o);
                        o = __builtin_elementwise_fma((f32x2){Dw[2 * i + 1], Dw[2 * i + 1]}, vb, o);
                    }
                    return o;
                };
                auto to_pcm = [&](float v) {
                    const float p = rintf(v * 32768.f);
                    return (int)fminf(fmaxf(p, -32768.f), 32767.f);
                };
                const int so = f * 2304 * PB + gr * 576 * nch * PB;
                if (F32) {
                    /* float sink: the same sums, unscaled and unclipped (FFmpeg's
                     * float decoder convention); (L, R) = 8 B per lane and slot */
                    if (nch == 2) {
                        const int vo = opaque((sb + 32 * ch) * 8);
#pragma unroll
                        for (int tp = 0; tp < 9; tp++) {
                            const f32x2 o = out2(tp);
                            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(o.x), __float_as_uint(o.y),
                                                                            false, false);
                            __builtin_amdgcn_raw_buffer_store_b64((u32x2){r[0], r[1]}, r_pcm, vo + 512 * tp, so, 0);
                        }
                    } else {
                        const int vo = opaque(sb * 4);
#pragma unroll
                        for (int tp = 0; tp < 9; tp++) {
                            const f32x2 o = out2(tp);
                            if (active) {
                                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o.x), r_pcm, vo + 256 * tp, so, 0);
                                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o.y), r_pcm, vo + 256 * tp + 128, so, 0);
                            }
                        }
                    }
                } else if (nch == 2) {
                    const int vo = opaque((sb + 32 * ch) * 4);
#pragma unroll
                    for (int tp = 0; tp < 9; tp++) {
                        const f32x2 o = out2(tp);
                        const int p0 = to_pcm(o.x), p1 = to_pcm(o.y);
                        const auto r = __builtin_amdgcn_permlane32_swap(p0, p1, false, false);
                        __builtin_amdgcn_raw_buffer_store_b32(((uint32_t)r[0] & 0xFFFFu) | ((uint32_t)r[1] << 16),
                                                              r_pcm, vo + 256 * tp, so, 0);
                    }
                } else {
                    const int vo = opaque(sb * 2);
#pragma unroll
                    for (int tp = 0; tp < 9; tp++) {
                        const f32x2 o = out2(tp);
                        if (active) {
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)to_pcm(o.x), r_pcm, vo + 128 * tp, so, 0);
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)to_pcm(o.y), r_pcm, vo + 128 * tp + 64, so, 0);
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < 14; k++) ha[k] = active ? xa[k + 4] : ha[k];
#pragma unroll
                for (int k = 0; k < 15; k++) hb[k] = active ? xb[k + 3] : hb[k];
            }
            wave_sync(); /* X reads done before the next granule's xr */
        }
    }
    /* state out */
#pragma unroll
    for (int i = 0; i < 18; i++) S.overlap[ch][sb][i] = ov[i];
#pragma unroll
    for (int k = 0; k < 14; k++) S.fifo[ch][k + 1][wa] = ha[k];
#pragma unroll
    for (int k = 0; k < 15; k++) S.fifo[ch][k][wb] = hb[k];
}
/* ------------------------------------------------------------------------ */
/* k_gather_frames: segmented long-stream decode (mp3d_batch_decode_long).  */
/* Output frame j of the long stream is frame (j - a[k]) of virtual stream  */
/* k - k0 (k = j / L) in the batch output; copies its PCM row (16-B words)   */
/* and frame info (zero-filled: rows without audio, the unused part of a   */
/* mono / LSF row).  One workgroup per output frame.                        */
/* ------------------------------------------------------------------------ */
__global__ void __launch_bounds__(256) k_gather_frames(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                       const DevInfo *__restrict__ isrc, DevInfo *__restrict__ idst,
                                                       const int *__restrict__ a, int L, int F, int k0, int row16) {
    const int jl = blockIdx.x;           /* output frame relative to segment k0's first */
    const int k = jl / L;                /* segment relative to k0                      */
    const int j = (k0 + k) * L + jl % L; /* global output frame                         */
    const size_t sf = (size_t)k * F + (j - a[k]);
    const DevInfo inf = isrc[sf];
    /* words holding audio: samples x channels of the 2304-sample row (mono
     * 1152, LSF 576 per channel); the rest is zero-filled */
    const int lim = inf.samples * inf.channels * row16 / 2304;
    for (int i = threadIdx.x; i < row16; i += blockDim.x)
        dst[(size_t)jl * row16 + i] = i < lim ? src[sf * row16 + i] : make_uint4(0u, 0u, 0u, 0u);
    if (idst && threadIdx.x == 0) idst[jl] = isrc[sf];
}

/* ------------------------------------------------------------------------ */
/* Host-side launchers                                                       */
/* ------------------------------------------------------------------------ */
hipError_t upload_constants(const float *win36, const float *is_ratio, const float *pow2q, const float *is_lsf,
                            const uint16_t *frame_bytes) {
    hipError_t e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_frame_bytes), frame_bytes, sizeof(uint16_t) * 9 * 16))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_win36), win36, sizeof(float) * 4 * 36))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_is_ratio), is_ratio, sizeof(float) * 14))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_pow2q), pow2q, sizeof(float) * 4))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_is_lsf), is_lsf, sizeof(float) * 64))) return e;
    return hipSuccess;
}

void launch_demux(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint8_t *md,
                  const uint64_t *md_off, StreamState *st, FrameRec *rec, uint64_t *sideu, void *infos, int n_streams,
                  int F, int opts, hipStream_t strm) {
    hipLaunchKernelGGL(k_demux, dim3(n_streams), dim3(64), 0, strm, in, in_off, in_len, md, md_off, st, rec, sideu,
                       (DevInfo *)infos, F, opts);
}

void launch_huffman(const uint8_t *md, const uint64_t *md_off, const FrameRec *rec, const uint64_t *sideu,
                    const DevTables *tab, int16_t *is_buf, UnitMeta *meta, int n_streams, int F, int n_cu,
                    hipStream_t strm) {
    int n_units = n_streams * F * 4;
    int supers = (n_units + HUFF_SUPER - 1) / HUFF_SUPER;
    /* one super-chunk per wave, no grid-stride: the hardware hands out
     * blocks as CUs free up, so uneven super-chunks balance themselves */
    int blocks = (supers + HUFF_WAVES - 1) / HUFF_WAVES;
    (void)n_cu;
    hipLaunchKernelGGL(k_huffman, dim3(blocks), dim3(HUFF_BLOCK), 0, strm, md, md_off, rec, sideu, tab, is_buf, meta,
                       n_units, F);
}

void launch_synth(const FrameRec *rec, const int16_t *is_buf, const UnitMeta *meta, const DevTables *tab,
                  StreamState *st, void *pcm, bool f32, int n_streams, int F, hipStream_t strm) {
    const dim3 grid((n_streams + SYN_WAVES - 1) / SYN_WAVES), block(64 * SYN_WAVES);
    /* both family variants; a workgroup without a stream of its variant
     * exits after SYN_WAVES scalar loads (the LSF launch on an all-MPEG-1
     * batch costs only its workgroup dispatch) */
#define MP3D_SYNTH_LAUNCH(F32_, LSF_)                                                                            \
    hipLaunchKernelGGL((k_synth<false, F32_, LSF_>), grid, block, 0, strm, rec, is_buf, meta, (const float *)nullptr, \
                       (const uint8_t *)nullptr, (const uint8_t *)nullptr, tab, st, pcm, n_streams, F, 2, 0)
    if (f32) {
        MP3D_SYNTH_LAUNCH(true, false);
        MP3D_SYNTH_LAUNCH(true, true);
    } else {
        MP3D_SYNTH_LAUNCH(false, false);
        MP3D_SYNTH_LAUNCH(false, true);
    }
#undef MP3D_SYNTH_LAUNCH
}

void launch_synth_xr(const float *xr, const uint8_t *bt, const uint8_t *mixed, const DevTables *tab, StreamState *st,
                     int16_t *pcm, int n_streams, int F, int nch, int sr, hipStream_t strm) {
    hipLaunchKernelGGL((k_synth<true, false, false>), dim3((n_streams + SYN_WAVES - 1) / SYN_WAVES), dim3(64 * SYN_WAVES), 0,
                       strm, (const FrameRec *)nullptr, (const int16_t *)nullptr, (const UnitMeta *)nullptr, xr, bt,
                       mixed, tab, st, (void *)pcm, n_streams, F, nch, sr);
}

void launch_gather_frames(const void *src, void *dst, const void *isrc, void *idst, const int *a, int L, int F, int k0,
                          int n_out, int bytes_per_row, hipStream_t strm) {
    hipLaunchKernelGGL(k_gather_frames, dim3(n_out), dim3(256), 0, strm, (const uint4 *)src, (uint4 *)dst,
                       (const DevInfo *)isrc, (DevInfo *)idst, a, L, F, k0, bytes_per_row / 16);
}

} // namespace mp3d
