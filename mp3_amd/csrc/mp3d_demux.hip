/*
 * mp3d_demux.hip -- k_demux (§8(f) rows 1
 * and 4): per stream, frame sync over ID3v2 / junk, MPEG-1 and MPEG-2 / 2.5
 * LSF headers and side info, Xing/Info + LAME tag, optional CRC-16 check,
 * bit-reservoir map and main-data copy into the stream's md region.
 * Pipeline overview: mp3d_device.h.
 */
#include "mp3d_device.h"

namespace mp3d {

/* Layer III frame bytes without padding per (sample-rate index 0..8,
 * bitrate index): 144000 kbps / Hz (MPEG-1), 72000 kbps / Hz (LSF); 0 for
 * free format / bad index.  A table read instead of a scalar division in
 * the per-frame header check. */
__constant__ uint16_t c_frame_bytes[9][16];
/* CRC-16 check tables (crc16_ok): x^(8 j) mod P and 0xFFFF x^(8 n) mod P */
__constant__ uint32_t c_crc_pow[40];
__constant__ uint32_t c_crc_init[40];

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
    uint32_t raw;      /* lane i: little-endian dword at stream offset pos - mis + 4 i */
    uint32_t keep;     /* byte mask of raw inside the stream (applied at use: the   */
                       /* load stays in flight until the window is read)           */
    uint32_t pos;
    uint32_t mis;      /* (address of stream byte pos) & 3: the dwords are aligned  */
    __device__ __forceinline__ uint32_t le() const { return raw & keep; }
};

/* Every load is an ALIGNED dword that holds at least one byte of the stream
 * [0, len), so it never leaves the pages of the caller's buffer, however the
 * stream is placed; bytes outside the stream read as zero. */
__device__ __forceinline__ HdrWin load_win(const uint8_t *p0, uint32_t len, uint32_t pos, int lane) {
    HdrWin w;
    w.pos = pos;
    w.mis = (uint32_t)((uintptr_t)(p0 + pos) & 3u);
    const int64_t a = (int64_t)pos - (int64_t)w.mis + 4 * lane; /* stream offset of the lane's dword */
    const int64_t over = a + 4 - (int64_t)len;                   /* bytes past the stream end */
    w.keep = (lane >= 16 || over >= 4) ? 0u : over > 0 ? 0xFFFFFFFFu >> (8 * over) : 0xFFFFFFFFu;
    w.raw = w.keep ? *(const uint32_t *)(p0 + a) : 0u;
    return w;
}

/* byte k of the window (uniform k; k + mis < 64) */
__device__ __forceinline__ uint32_t win_byte(const HdrWin &w, uint32_t k) {
    const uint32_t i = k + w.mis;
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)w.le(), (int)(i >> 2));
    return (d >> (8 * (i & 3u))) & 0xFFu;
}

/* 64 bits of the window's big-endian bit string starting at bit b of the
 * window's first dword (stream byte pos - mis) -- per lane b (lane-varying) */
__device__ __forceinline__ uint64_t win_bits64(const HdrWin &w, uint32_t b) {
    const uint32_t be = __builtin_bswap32(w.le());
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
 * Lane-parallel, by linearity over GF(2): for the n message bytes m_i,
 *   crc = 0xFFFF x^(8n) mod P  xor  sum_i m_i x^16 x^(8 (n-1-i)) mod P,
 * lane i computing its byte's term (8 shift steps, then a 16-step Horner
 * product with x^(8 (n-1-i)) mod P from c_crc_pow) and a wave xor-reduce
 * adding them: ~100 VALU per frame instead of a 272-step serial loop. */
__device__ __forceinline__ uint32_t crc_mulx(uint32_t c) { /* c x mod P */
    return (c & 0x8000u) ? ((c << 1) ^ 0x8005u) & 0xFFFFu : (c << 1) & 0xFFFFu;
}
__device__ bool crc16_ok(const HdrWin &w, uint32_t side_bytes, int lane) {
    const uint32_t n = 2u + side_bytes; /* message bytes: header 2..3, side info */
    uint32_t term = 0u;
    /* message byte i sits at frame byte 2 + i (header) or 4 + i (side info);
     * the cross-lane read runs in every lane (all source lanes active) */
    const uint32_t k = (uint32_t)(lane < 34 ? lane : 33) + (lane < 2 ? 2u : 4u) + w.mis;
    const uint32_t d = (uint32_t)__shfl((int)w.le(), (int)(k >> 2));
    if ((uint32_t)lane < n) {
        uint32_t c = ((d >> (8u * (k & 3u))) & 0xFFu) << 8;
#pragma unroll
        for (int b = 0; b < 8; b++) c = crc_mulx(c); /* m_i x^16 mod P */
        const uint32_t m = c_crc_pow[n - 1u - (uint32_t)lane];
#pragma unroll
        for (int b = 15; b >= 0; b--) term = crc_mulx(term) ^ (((m >> b) & 1u) ? c : 0u);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) term ^= (uint32_t)__shfl_xor((int)term, o);
    return (term ^ c_crc_init[n]) == ((win_byte(w, 4) << 8) | win_byte(w, 5));
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

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) k_demux(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
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
        uint32_t src_off = 0, frame_at = 0; /* payload and header positions in the stream */
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
                const uint32_t sbit = 8u * (w.mis + 4u + (uint32_t)crc);
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
                const bool crc_bad = (opts & MP3D_OPT_CRC_CHECK) && crc && !crc16_ok(w, (uint32_t)side_bytes, lane);
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
                frame_at = cur;
                cur = have == (uint32_t)fb ? cur + (uint32_t)fb : len;
            } else {
                cur = len;
            }
        }
        if (lane == 0) {
            rec[fi] = r;
            if (infos) infos[fi] = inf;
        }
        if (lane < 4) sideu[fi * 4 + lane] = sw;
        /* next frame's header window in flight while this payload copies
         * (issued after the record stores: a store issued behind a pending
         * load made the compiler drain vmcnt(0) before it, i.e. wait for the
         * window right here) */
        if (cur + 4 <= len && f + 1 < F) w = load_win(p0, len, cur, lane);
        if (copy) {
            const uint8_t *src = p0 + src_off;
            const uint32_t Pm = r.payload_md, L = r.payload_avail;
            for (uint32_t i = L + lane; i < r.payload_len; i += 64) dst[Pm + i] = 0; /* cut-short final frame */
            const uint32_t h = min((4u - (Pm & 3u)) & 3u, L);     /* head bytes up to an aligned word */
            const uint32_t wb = (Pm + h) >> 2, we = (Pm + L) >> 2; /* whole words [wb, we)           */
            /* tail bytes [t0, L) after the last whole word -- or after the head
             * when there is none (an LSF payload can be < 8 bytes) */
            const uint32_t t0 = 4u * we > Pm + h ? 4u * we - Pm : h; /* h <= t0 <= L */
            /* edge-byte loads first, stored after the words' loads: every
             * load of the payload is in flight before the first store waits */
            /* (unconditional: lanes without an edge byte re-read the frame's
             * first header byte, which is always in the stream) */
            const uint8_t *hb0 = p0 + frame_at;
            const uint8_t hbv = *((uint32_t)lane < h ? src + lane : hb0);
            const uint8_t tbv = *((uint32_t)lane < L - t0 ? src + t0 + lane : hb0);
            if (wb < we) {
                /* pointer arithmetic, not an integer round trip: the loads
                 * stay global_load (a flat load waits on lgkmcnt too) */
                const uint8_t *sb = src + (4u * wb - Pm);
                const uint32_t mis = (uint32_t)((uintptr_t)sb & 3u);
                const uint32_t sh = mis * 8u;
                const uint32_t *swd = (const uint32_t *)(sb - mis);
                /* all words in flight before the first store (straight-line,
                 * so no loop-header wait drains them early): one load latency
                 * per frame instead of one per 64-word round; the next header
                 * window (issued above) lands with them.  A payload is at most
                 * 1437 B (1441-B frame) = 360 words < 6 x 64. */
                /* Loads are unconditional (lanes past the payload re-read word
                 * 0) and the shift is branch-free (alignbit by 0 = lo): with a
                 * load under a branch the compiler's waitcnt pass loses track
                 * at the join and drains vmcnt before every store.  The high
                 * word is read only for a misaligned source (index select, not
                 * a branch): it then still holds payload bytes.  Both words
                 * are aligned dwords holding at least one payload byte, so no
                 * load leaves the pages of the caller's buffer. */
                const uint32_t nwd = we - wb;
                uint32_t v[6];
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    const uint32_t k = 64u * j + (uint32_t)lane;
                    const uint32_t kk = k < nwd ? k : 0u;
                    v[j] = __builtin_amdgcn_alignbit(swd[sh ? kk + 1 : kk], swd[kk], sh);
                }
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    const uint32_t k = 64u * j + (uint32_t)lane;
                    if (k < nwd) ((uint32_t *)dst)[wb + k] = v[j];
                }
                for (uint32_t k = 384u + (uint32_t)lane; k < nwd; k += 64) { /* not reached (see above) */
                    const uint32_t l = swd[k];
                    ((uint32_t *)dst)[wb + k] = sh ? __builtin_amdgcn_alignbit(swd[k + 1], l, sh) : l;
                }
            }
            if ((uint32_t)lane < h) dst[Pm + lane] = hbv;
            if ((uint32_t)lane < L - t0) dst[Pm + t0 + lane] = tbv;
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


/* ------------------------------------------------------------------------ */
/* Wide batches: k_walk + k_mdcopy, the same results as k_demux.            */
/* k_demux walks a stream with one wave, its per-frame decisions uniform,   */
/* so they run on the scalar unit: ~330 scalar instructions per frame, and  */
/* the CU's one scalar unit (shared by its 4 SIMDs) is the kernel's limit   */
/* at C3 (SQ_INSTS_SALU, profiles/).  k_walk gives each stream ONE LANE:    */
/* the header chain of 64 streams runs side by side as vector arithmetic,   */
/* each lane staging a 64-B window of its stream at the frame position in   */
/* LDS.  k_mdcopy then copies every frame's payload into the md region      */
/* (one wave per stream; no frame waits on another's header).  k_walk       */
/* leaves the md end and the next carry length in StreamState.pad_ for     */
/* k_mdcopy, which moves the carry (StreamState.res) in and out.           */
/* ------------------------------------------------------------------------ */
#define WALK_WORDS 17 /* LDS dwords per lane: a 64-B window (+1: odd stride) */
#define WALK_LANES 64 /* streams per wave (lanes past it idle)              */

struct LaneWin {        /* one lane's 64-B window of its stream, staged in LDS */
    uint32_t *w;        /* the lane's LDS words                                */
    uint32_t pos, mis;  /* stream offset of window byte mis; mis = address & 15 */
    __device__ __forceinline__ uint32_t byte(uint32_t k) const { /* stream byte pos + k, k < 64 - mis */
        return ((const uint8_t *)w)[mis + k];
    }
    /* 64 bits of the big-endian bit string starting at bit b after pos */
    __device__ __forceinline__ uint64_t bits64(uint32_t b) const {
        const uint32_t a = 8u * mis + b, wi = a >> 5, sh = a & 31u;
        const uint64_t hi = ((uint64_t)__builtin_bswap32(w[wi]) << 32) | __builtin_bswap32(w[wi + 1]);
        const uint32_t x2 = __builtin_bswap32(w[wi + 2]);
        return sh ? (hi << sh) | ((uint64_t)x2 >> (32 - sh)) : hi;
    }
};

/* the four 16-B aligned blocks around stream offset pos: every block holds
 * a stream byte (so none leaves the pages of the caller's buffer, which are
 * 16-B aligned units) or is not loaded; bytes at or past len read as zero */
__device__ __forceinline__ void walk_load(LaneWin &W, const uint8_t *p0, uint32_t len, uint32_t pos) {
    W.pos = pos;
    W.mis = (uint32_t)((uintptr_t)(p0 + pos) & 15u);
    const uint4 *base = (const uint4 *)(p0 + pos - W.mis);
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t first = (int64_t)pos - (int64_t)W.mis + 16 * j; /* stream offset of the block */
        v[j] = make_uint4(0u, 0u, 0u, 0u);
        if (first < (int64_t)len) v[j] = base[j];
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t over = (int64_t)pos - (int64_t)W.mis + 16 * j + 16 - (int64_t)len; /* bytes past the end */
        uint32_t q[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t o = over - 4 * (3 - i); /* bytes of word i past the end */
            q[i] = o >= 4 ? 0u : o > 0 ? q[i] & (0xFFFFFFFFu >> (8 * o)) : q[i];
            W.w[4 * j + i] = q[i];
        }
    }
}

/* CRC-16 (poly 0x8005, init 0xFFFF, MSB first) over header bytes 2..3 and
 * the side info (window bytes 6 ..), against bytes 4..5 -- one lane, bitwise;
 * only for protected frames under MP3D_OPT_CRC_CHECK */
__device__ __forceinline__ bool walk_crc_ok(const LaneWin &W, uint32_t side_bytes) {
    uint32_t c = 0xFFFFu;
    for (uint32_t i = 0; i < 2u + side_bytes; i++) {
        const uint32_t m = W.byte(i < 2u ? 2u + i : 4u + i);
        c ^= m << 8;
#pragma unroll
        for (int b = 0; b < 8; b++) c = crc_mulx(c);
    }
    return c == ((W.byte(4) << 8) | W.byte(5));
}

__global__ void __launch_bounds__(64) k_walk(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                             const uint32_t *__restrict__ in_len, StreamState *__restrict__ st,
                                             FrameRec *__restrict__ rec, uint64_t *__restrict__ sideu,
                                             DevInfo *__restrict__ infos, int n_streams, int F, int opts) {
    __shared__ uint32_t s_win[64 * WALK_WORDS];
    const int lane = threadIdx.x;
    const int s = blockIdx.x * WALK_LANES + lane;
    if (lane >= WALK_LANES || s >= n_streams) return; /* no barrier below */
    LaneWin W;
    W.w = s_win + lane * WALK_WORDS;
    const uint8_t *p0 = in + in_off[s];
    const uint32_t len = in_len[s];
    StreamState &S = st[s];
    const int carry_in = S.res_len;
    const bool stream_start = S.frames == 0;
    int kind = S.kind;
    uint32_t P = (uint32_t)carry_in;
    int avail = carry_in;
    uint32_t cur = 0;
    walk_load(W, p0, len, 0);
    if (stream_start && len >= 10 && W.byte(0) == 'I' && W.byte(1) == 'D' && W.byte(2) == '3') {
        const uint32_t sz = (W.byte(6) & 0x7Fu) << 21 | (W.byte(7) & 0x7Fu) << 14 | (W.byte(8) & 0x7Fu) << 7 |
                            (W.byte(9) & 0x7Fu);
        cur = 10 + sz + ((W.byte(5) & 0x10u) ? 10u : 0u);
    }
    int decoded = 0;
    for (int f = 0; f < F; f++) {
        const size_t fi = (size_t)s * F + f;
        /* ---- sync: the next valid header at or after cur (resync over junk) */
        int fb = -1;
        while (cur + 4 <= len) {
            if (W.pos != cur) walk_load(W, p0, len, cur);
            const uint32_t lim = min(46u, len - cur - 4);
            uint32_t k = 0;
            for (; k <= lim; k++) {
                if (W.byte(k) == 0xFFu) {
                    fb = hdr_frame_bytes(W.byte(k + 1), W.byte(k + 2), kind);
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
        uint64_t sw[4] = {0ull, 0ull, 0ull, 0ull};
        if (fb > 0) {
            if (W.pos != cur) walk_load(W, p0, len, cur);
            const uint32_t h1 = W.byte(1), h2 = W.byte(2), h3 = W.byte(3);
            const int nch = (h3 >> 6) == 3 ? 1 : 2;
            const int crc = (h1 & 1) ? 0 : 2;
            const bool lsf = hdr_kind(h1) == 2;
            const int ngr = lsf ? 1 : 2;
            const int side_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
            kind = hdr_kind(h1);
            const uint32_t need = 4u + (uint32_t)crc + (uint32_t)side_bytes;
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
                const uint32_t sbit = 8u * (4u + (uint32_t)crc);
                const int mdb = (int)(W.bits64(sbit) >> (lsf ? 56 : 55));
                uint32_t p23[2][2] = {{0u, 0u}, {0u, 0u}};
                bool anybad = false;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int qgr = q >> 1, qch = q & 1;
                    if (qch < nch && qgr < ngr) {
                        const uint32_t ub = sbit + side_unit_bit(nch, qgr, qch, lsf);
                        uint64_t v59;
                        uint32_t low5;
                        if (lsf) { /* the 63-bit LSF unit in the MPEG-1 layout (k_demux) */
                            const uint64_t v63 = W.bits64(ub) >> 1;
                            const uint32_t sfc9 = (uint32_t)(v63 >> 25) & 511u;
                            const uint64_t low25 = v63 & 0x1FFFFFFull;
                            const bool is_right = (h3 >> 6) == 1 && ((h3 >> 4) & 1) && qch == 1;
                            v59 = ((v63 >> 34) << 30) | ((uint64_t)(sfc9 & 15u) << 26) | ((low25 >> 2) << 3) |
                                  ((uint64_t)is_right << 2) | (low25 & 3u);
                            low5 = sfc9 >> 4;
                        } else {
                            v59 = W.bits64(ub) >> 5;
                            low5 = (uint32_t)(W.bits64(sbit + 9 + (nch == 1 ? 5 : 3) + 4 * qch) >> 60) << 1;
                        }
                        p23[qgr][qch] = (uint32_t)(v59 >> 47);
                        anybad |= ((v59 >> 38) & 0x1FFu) > 288u || (v59 & (7ull << 23)) == (4ull << 23);
                        sw[q] = (v59 << 5) | low5;
                    }
                }
                const bool crc_bad = (opts & MP3D_OPT_CRC_CHECK) && crc && !walk_crc_ok(W, (uint32_t)side_bytes);
                const bool bad = plen < 0 || anybad || crc_bad;
                const uint32_t tgo = 4u + (uint32_t)crc + (uint32_t)side_bytes;
                const bool tag = stream_start && f == 0 && plen >= 4 && have == (uint32_t)fb &&
                                 ((W.byte(tgo) == 'X' && W.byte(tgo + 1) == 'i' && W.byte(tgo + 2) == 'n' &&
                                   W.byte(tgo + 3) == 'g') ||
                                  (W.byte(tgo) == 'I' && W.byte(tgo + 1) == 'n' && W.byte(tgo + 2) == 'f' &&
                                   W.byte(tgo + 3) == 'o'));
                if (tag) {
                    r.first_gr = REC_TAG;
                    S.tag_info = parse_info_tag(p0 + cur + tgo, (uint32_t)fb - tgo, S.tag_frames);
                } else if (bad) {
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
                            bits += p23[gr0][0] + p23[gr0][1];
                            gr0++;
                        }
                        mdbit = (P - (uint32_t)avail) * 8u + bits - 8u * (uint32_t)mdb;
                    }
                    /* units past nch / ngr hold 0 */
                    const uint32_t end = mdbit + (gr0 == 0 ? p23[0][0] + p23[0][1] : 0u) +
                                         (gr0 <= 1 ? p23[1][0] + p23[1][1] : 0u);
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
                cur = have == (uint32_t)fb ? cur + (uint32_t)fb : len;
            } else {
                cur = len;
            }
        }
        rec[fi] = r;
        if (infos) infos[fi] = inf;
        ulonglong2 *sd = (ulonglong2 *)&sideu[fi * 4];
        sd[0] = make_ulonglong2(sw[0], sw[1]);
        sd[1] = make_ulonglong2(sw[2], sw[3]);
        /* the next frame's window in flight while this frame's records store */
        if (cur + 4 <= len && f + 1 < F) walk_load(W, p0, len, cur);
    }
    int c = avail < MP3D_RES_BYTES ? avail : MP3D_RES_BYTES;
    if ((uint32_t)c > P) c = (int)P;
    S.frames += decoded;
    S.kind = kind;
    S.pad_[0] = (int32_t)P; /* md end, for k_mdcopy */
    S.pad_[1] = c;          /* next carry length   */
}

/* k_mdcopy: one wave per stream, 4 streams per workgroup.  Carry-in, then
 * the payloads four frames at a time (16 lanes each, so four frames' loads
 * are in flight together), then the next carry.  Each lane first loads the
 * copy descriptor of one frame (lane f: frame f of a 64-frame chunk), so the
 * frame loop reads no record from memory.  Payload words: the destination
 * is written in aligned words, each from one 8-B source load funnel-shifted
 * by the source misalignment (the k_demux copy; edge bytes and a cut-short
 * tail as there).  All loads of an iteration are straight-line and
 * unconditional (lanes without work re-read a valid word): a load under a
 * branch makes the compiler's waitcnt pass drain vmcnt(0) at the join.  An
 * aligned source loads words (k - 1, k) instead of (k, k + 1), so no load
 * passes the payload's last word (word -1 is side info or header). */
#define MDC_WAVES 4
#define MDC_ROUNDS 8 /* 16-lane rounds per frame in the unrolled part: 512 B */
__global__ void __launch_bounds__(64 * MDC_WAVES) k_mdcopy(const uint8_t *__restrict__ in, uint8_t *__restrict__ md,
                                                         const uint64_t *__restrict__ md_off,
                                                         StreamState *__restrict__ st,
                                                         const FrameRec *__restrict__ rec, int n_streams, int F) {
    const int lane = threadIdx.x & 63;
    /* wave-uniform (SGPR): the buffer resource below must not be per lane */
    const int s = blockIdx.x * MDC_WAVES + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (s >= n_streams) return; /* wave-level sync only below */
    uint8_t *dst = md + md_off[s];
    const __amdgpu_buffer_rsrc_t r_md = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7FFFFFFF, 0x00020000);
    StreamState &S = st[s];
    const int carry_in = S.res_len;
    for (int i = lane; i < (carry_in + 3) / 4; i += 64) ((uint32_t *)dst)[i] = ((const uint32_t *)S.res)[i];
    __threadfence_block(); /* carry words may spill past carry_in into payload 0's head */
    const int qf = lane >> 4, ql = lane & 15;
    for (int c0 = 0; c0 < F; c0 += 64) {
        /* lane f: copy descriptor of frame c0 + f */
        uint32_t d_fo0 = 0u, d_fo1 = 0u, d_pmd = 0u, d_len = 0u, d_body = 0u;
        if (c0 + lane < F) {
            const FrameRec r = rec[(size_t)s * F + c0 + lane];
            const bool copy = r.frame_bytes && !(r.first_gr & REC_TAG);
            const uint32_t side_bytes = r.lsf ? (r.nch == 1 ? 9u : 17u) : (r.nch == 1 ? 17u : 32u);
            d_fo0 = (uint32_t)r.frame_off;
            d_fo1 = (uint32_t)(r.frame_off >> 32);
            d_pmd = r.payload_md;
            d_len = (uint32_t)r.payload_len | (uint32_t)r.payload_avail << 16;
            d_body = copy ? ((r.first_gr & REC_DROP) ? 4u : (uint32_t)r.side_off + side_bytes) : 0u;
        }
        /* drained here, once: otherwise the compiler waits for vmcnt(0) at
         * the descriptors' first use in every iteration, i.e. for the
         * previous frames' stores */
        __builtin_amdgcn_s_waitcnt(0x0F70);
        const int nf = min(64, F - c0);
        for (int f0 = 0; f0 < nf; f0 += 4) {
            /* the descriptor of this quarter's frame, read in every lane (a
             * cross-lane read from a lane outside the branch below would
             * not see its value) */
            const int fl = min(f0 + qf, 63);
            const uint32_t body = (uint32_t)__shfl((int)d_body, fl);
            const uint64_t fo = (uint64_t)(uint32_t)__shfl((int)d_fo0, fl) |
                                (uint64_t)(uint32_t)__shfl((int)d_fo1, fl) << 32;
            const uint32_t Pm = (uint32_t)__shfl((int)d_pmd, fl), lens = (uint32_t)__shfl((int)d_len, fl);
            if (f0 + qf < nf && body) {
                const uint32_t plen = lens & 0xFFFFu, L = lens >> 16;
                const uint8_t *hb0 = in + fo;
                const uint8_t *src = hb0 + body;
                const uint32_t h = min((4u - (Pm & 3u)) & 3u, L);
                const uint32_t wb = (Pm + h) >> 2, we = (Pm + L) >> 2;
                const uint32_t t0 = 4u * we > Pm + h ? 4u * we - Pm : h;
                const uint8_t *sb = src + (4u * wb - Pm);
                const uint32_t mis = (uint32_t)((uintptr_t)sb & 3u), sh = mis * 8u;
                const uint32_t nwd = we - wb;
                /* (pointer arithmetic only: an integer round trip would make
                 * these flat loads, which wait on both counters) */
                const uint32_t *lp = nwd ? (const uint32_t *)(sb - mis) - (sh ? 0 : 1)
                                         : (const uint32_t *)(hb0 - ((uintptr_t)hb0 & 3u));
                const uint8_t hbv = *((uint32_t)ql < h ? src + ql : hb0);
                const uint8_t tbv = *((uint32_t)ql < L - t0 ? src + t0 + ql : hb0);
                uint32_t v[MDC_ROUNDS];
#pragma unroll
                for (int j = 0; j < MDC_ROUNDS; j++) {
                    const uint32_t k = 16u * j + (uint32_t)ql;
                    const uint2 x = *(const uint2 *)(lp + (k < nwd ? k : 0u));
                    v[j] = __builtin_amdgcn_alignbit(x.y, sh ? x.x : x.y, sh);
                }
                /* stores masked by an out-of-range offset, not a branch (the
                 * compiler would sink each load into its store's branch) */
#pragma unroll
                for (int j = 0; j < MDC_ROUNDS; j++) {
                    const uint32_t k = 16u * j + (uint32_t)ql;
                    __builtin_amdgcn_raw_buffer_store_b32(v[j], r_md, k < nwd ? 4u * (wb + k) : 0x80000000u, 0, 0);
                }
                for (uint32_t k = 16u * MDC_ROUNDS + (uint32_t)ql; k < nwd; k += 16) {
                    const uint2 x = *(const uint2 *)(lp + k);
                    ((uint32_t *)dst)[wb + k] = __builtin_amdgcn_alignbit(x.y, sh ? x.x : x.y, sh);
                }
                for (uint32_t i = L + ql; i < plen; i += 16) dst[Pm + i] = 0; /* cut-short final frame */
                if ((uint32_t)ql < h) dst[Pm + ql] = hbv;
                if ((uint32_t)ql < L - t0) dst[Pm + t0 + ql] = tbv;
            }
        }
    }
    __threadfence_block();
    const uint32_t P = (uint32_t)S.pad_[0];
    const int c = S.pad_[1];
    for (int i = lane; i < c; i += 64) S.res[i] = dst[P - c + i];
    if (lane == 0) S.res_len = c;
}

/* ------------------------------------------------------------------------ */
/* Host-side launchers                                                       */
/* ------------------------------------------------------------------------ */
hipError_t upload_demux_constants(const uint16_t *frame_bytes) {
    hipError_t e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_frame_bytes), frame_bytes, sizeof(uint16_t) * 9 * 16))) return e;
    /* x^(8 j) mod P and 0xFFFF x^(8 n) mod P, P = x^16 + x^15 + x^2 + 1 */
    uint32_t pw[40], in[40];
    auto mulx = [](uint32_t c) { return (c & 0x8000u) ? ((c << 1) ^ 0x8005u) & 0xFFFFu : (c << 1) & 0xFFFFu; };
    uint32_t p = 1u, q = 0xFFFFu;
    for (int j = 0; j < 40; j++) {
        pw[j] = p;
        in[j] = q;
        for (int b = 0; b < 8; b++) { p = mulx(p); q = mulx(q); }
    }
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_crc_pow), pw, sizeof(pw)))) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_crc_init), in, sizeof(in));
}

/* wide: k_walk + k_mdcopy (batches of many streams); else one k_demux wave
 * per stream (fewer launches: the per-frame decoder, small batches) */
void launch_demux(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint8_t *md,
                  const uint64_t *md_off, StreamState *st, FrameRec *rec, uint64_t *sideu, void *infos, int n_streams,
                  int F, int opts, bool wide, hipStream_t strm) {
    if (wide) {
        hipLaunchKernelGGL(k_walk, dim3((n_streams + WALK_LANES - 1) / WALK_LANES), dim3(64), 0, strm, in, in_off, in_len, st, rec, sideu,
                           (DevInfo *)infos, n_streams, F, opts);
        hipLaunchKernelGGL(k_mdcopy, dim3((n_streams + MDC_WAVES - 1) / MDC_WAVES), dim3(64 * MDC_WAVES), 0, strm, in,
                           md, md_off, st, (const FrameRec *)rec, n_streams, F);
        return;
    }
    hipLaunchKernelGGL(k_demux, dim3(n_streams), dim3(64), 0, strm, in, in_off, in_len, md, md_off, st, rec, sideu,
                       (DevInfo *)infos, F, opts);
}

} // namespace mp3d
