/*
 * mp3d_demux_dev.h -- device side of the per-stream demux (SURVEY.md §8(a)
 * rows a1-a3, a12; §8(f) rows 1 and 4): frame sync over ID3v2 / junk, MPEG-1
 * and MPEG-2 / 2.5 LSF headers and side info, Xing/Info + LAME tag, optional
 * CRC-16 check, bit-reservoir map and main-data copy into the stream's md
 * region.  Included by mp3d_demux.hip (k_demux, k_walk, k_mdcopy) and by
 * mp3d_synth.hip (the fused per-frame kernel k_frame); each translation unit
 * holds its own constant tables (upload_demux_tables).
 */
#ifndef MP3D_DEMUX_DEV_H
#define MP3D_DEMUX_DEV_H
#include "mp3d_device.h"

/* the constants have external linkage (a static __constant__ is reached
 * through the GOT: one more scalar load); an inline namespace per
 * translation unit keeps the two copies' host symbols apart */
#ifndef MP3D_DEMUX_TU
#define MP3D_DEMUX_TU demux_tu
#endif

namespace mp3d {
inline namespace MP3D_DEMUX_TU {

/* Layer III frame bytes without padding per (sample-rate index 0..8,
 * bitrate index): 144000 kbps / Hz (MPEG-1), 72000 kbps / Hz (LSF); 0 for
 * free format / bad index -- in the low 16 bits, the bitrate in kbps in the
 * high 16.  A table read instead of a scalar division in the per-frame
 * header check; dwords, so that a wave-uniform index is a scalar load (a
 * sub-dword load is a vector load, and its wait drains the stream's
 * outstanding payload stores with it). */
__constant__ uint32_t c_frame_word[9][16];
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
/* the header tables: the __constant__ copies, or a kernel's LDS copy
 * (k_demux_fp: a scalar load from L2 or HBM per frame was a round trip on
 * every wave's chain of frames) */
struct HdrTabConst {
    __device__ __forceinline__ uint32_t fw(int sr, int bi) const { return c_frame_word[sr][bi]; }
    __device__ __forceinline__ uint32_t hz(int sr) const { return MP3D_SAMPLE_RATE[sr]; }
};
struct HdrTabLds {
    const __attribute__((address_space(3))) uint32_t *t; /* [9][16] frame words, then [9] sample rates */
    __device__ __forceinline__ uint32_t fw(int sr, int bi) const { return t[16 * sr + bi]; }
    __device__ __forceinline__ uint32_t hz(int sr) const { return t[144 + sr]; }
};
#define HDR_TAB_WORDS (9 * 16 + 9)
/* an HdrTabLds table's words (tid < HDR_TAB_WORDS; the caller's barrier follows) */
__device__ __forceinline__ void hdr_tab_stage(uint32_t *t, int tid) {
    if (tid < 9 * 16) t[tid] = (&c_frame_word[0][0])[tid];
    else if (tid < HDR_TAB_WORDS) t[tid] = MP3D_SAMPLE_RATE[tid - 9 * 16];
}
template <class T = HdrTabConst>
__device__ __forceinline__ int hdr_frame_bytes(uint32_t b1, uint32_t b2, int kind, const T &tab = T()) {
    if ((b1 & 0xE0) != 0xE0 || ((b1 >> 1) & 3) != 1 || ((b1 >> 3) & 3) == 1) return -1;
    const int bi = (int)(b2 >> 4);
    if (bi == 0 || bi == 15 || ((b2 >> 2) & 3) == 3) return -1;
    if (kind && hdr_kind(b1) != kind) return -1;
    return (int)(tab.fw(hdr_sr_idx(b1, b2), bi) & 0xFFFFu) + (int)((b2 >> 1) & 1);
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

/* Where demux_stream reads the stream's bytes: global memory (the caller's
 * buffer in HBM or a mapped host buffer) or LDS (a stream staged whole by
 * k_demux, the frame staged by k_frame) -- typed pointers, so that the loads
 * are global_load / ds_read and never flat (a flat load waits on both the
 * vector-memory and the LDS counter). */
struct SrcGlobal {
    typedef const uint8_t u8;
    typedef const uint32_t u32;
};
struct SrcLds {
    typedef const __attribute__((address_space(3))) uint8_t u8;
    typedef const __attribute__((address_space(3))) uint32_t u32;
};

/* Every load is an ALIGNED dword that holds at least one byte of the stream
 * [0, len), so it never leaves the pages of the caller's buffer, however the
 * stream is placed; bytes outside the stream read as zero. */
template <class M>
__device__ __forceinline__ HdrWin load_win(typename M::u8 *p0, uint32_t len, uint32_t pos, int lane) {
    HdrWin w;
    w.pos = pos;
    w.mis = (uint32_t)((uintptr_t)(p0 + pos) & 3u);
    const int64_t a = (int64_t)pos - (int64_t)w.mis + 4 * lane; /* stream offset of the lane's dword */
    const int64_t over = a + 4 - (int64_t)len;                   /* bytes past the stream end */
    w.keep = (lane >= 16 || over >= 4) ? 0u : over > 0 ? 0xFFFFFFFFu >> (8 * over) : 0xFFFFFFFFu;
    w.raw = w.keep ? *(typename M::u32 *)(p0 + a) : 0u;
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
template <class P> __device__ uint32_t parse_info_tag(P t, uint32_t n, uint32_t &frames) {
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

/* One frame's header and side info, parsed from the header window at its
 * sync position (ISO 2.4.1.3 / 2.4.1.7; 13818-3 for LSF): everything about
 * the frame that does not depend on the frames before it.  The bit-reservoir
 * map (resolve_frame) is the only serial step of a stream's demux: k_demux
 * runs parse / resolve / emit frame by frame in one wave, k_demux_fp parses
 * and emits the frames of a pre-located run in parallel around one serial
 * resolve.  Uniform fields; sw is per lane (lane q < 4: unit q's side word). */
struct FrameParse {
    int fb;               /* frame bytes; 0: no frame (cut too short)         */
    int nch, crc, side_bytes, ngr, plen, mdb;
    uint32_t h1, h2, h3, have, need;
    int p00, p01, p10, p11; /* part2_3_length of unit (gr, ch), by select     */
    bool lsf, bad, tag;
    uint64_t sw;
    __device__ __forceinline__ int p23(int gr, int ch) const { return gr ? (ch ? p11 : p10) : (ch ? p01 : p00); }
};

/* parse the frame of fb bytes whose header is at stream offset cur (window
 * w at cur); f0 = the stream's first frame of the stream's first call (the
 * Xing/Info tag check); r / inf get the frame's fields.  The tag's LAME
 * fields go to S (lane 0). */
template <class M, class T = HdrTabConst>
__device__ __forceinline__ void parse_frame(const HdrWin &w, typename M::u8 *p0, uint64_t base, uint32_t cur,
                                            uint32_t len, int fb, bool f0, int opts, StreamState &S, FrameParse &fp,
                                            FrameRec &r, DevInfo &inf, int lane, const T &tab = T()) {
    fp.fb = 0;
    fp.sw = 0;
    fp.bad = fp.tag = false;
    const uint32_t h1 = win_byte(w, 1), h2 = win_byte(w, 2), h3 = win_byte(w, 3);
    const int nch = (h3 >> 6) == 3 ? 1 : 2;
    const int crc = (h1 & 1) ? 0 : 2;
    const bool lsf = hdr_kind(h1) == 2;
    const int ngr = lsf ? 1 : 2;
    const int side_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
    const uint32_t need = 4u + (uint32_t)crc + (uint32_t)side_bytes;
    fp.h1 = h1; fp.h2 = h2; fp.h3 = h3;
    fp.nch = nch; fp.crc = crc; fp.lsf = lsf; fp.ngr = ngr; fp.side_bytes = side_bytes; fp.need = need;
    /* a final frame cut short still decodes (FFmpeg: the missing bytes read
     * as zeros) once its header and side info are present */
    if (!(cur + (uint32_t)fb <= len || cur + need <= len)) return;
    const uint32_t have = min(len - cur, (uint32_t)fb);
    const int plen = fb - 4 - crc - side_bytes;
    fp.fb = fb; fp.have = have; fp.plen = plen;
    r.frame_off = base + cur;
    r.frame_bytes = (uint16_t)fb;
    r.payload_len = (uint16_t)(plen > 0 ? plen : 0);
    r.hdr1 = (uint8_t)h1; r.hdr2 = (uint8_t)h2; r.hdr3 = (uint8_t)h3;
    r.nch = (uint8_t)nch;
    r.side_off = (uint8_t)(4 + crc);
    r.sr_idx = (uint8_t)hdr_sr_idx(h1, h2);
    r.lsf = (uint8_t)lsf;
    inf.frame_bytes = fb; inf.channels = nch; inf.hz = (int)tab.hz(r.sr_idx);
    inf.layer = 3; inf.bitrate_kbps = (int)(tab.fw(r.sr_idx, (int)(h2 >> 4)) >> 16);
    /* side info: bit offsets relative to the window's dword base */
    const uint32_t sbit = 8u * (w.mis + 4u + (uint32_t)crc);
    fp.mdb = (int)(win_bits64(w, sbit) >> (lsf ? 56 : 55));
    const int q = lane & 3, qgr = q >> 1, qch = q & 1;
    const uint32_t ub = sbit + side_unit_bit(nch, qgr, qch, lsf);
    const bool unit_ok = lane < 4 && qch < nch && qgr < ngr;
    uint64_t v59;
    uint32_t low5; /* side word bits 4..0: scfsi << 1 (MPEG-1) | scalefac_compress >> 4 (LSF) */
    if (lsf) {
        /* 63-bit LSF unit (13818-3 2.4.1.7): part2_3 12, big_values 9,
         * global_gain 8, scalefac_compress 9, window switching 1 + 22,
         * scalefac_scale 1, count1table 1 -> the MPEG-1 layout with
         * scalefac_compress bits 0..3 in its 4-bit slot, the
         * intensity-right-channel flag in the preflag slot, bits 4..8 in the
         * side word's low 5 bits */
        const uint64_t v63 = win_bits64(w, ub) >> 1;
        const uint32_t sfc9 = (uint32_t)(v63 >> 25) & 511u;
        const uint64_t low25 = v63 & 0x1FFFFFFull;
        const bool is_right = (h3 >> 6) == 1 && ((h3 >> 4) & 1) && qch == 1;
        v59 = ((v63 >> 34) << 30) | ((uint64_t)(sfc9 & 15u) << 26) | ((low25 >> 2) << 3) | ((uint64_t)is_right << 2) |
              (low25 & 3u);
        low5 = sfc9 >> 4;
    } else {
        v59 = win_bits64(w, ub) >> 5;
        low5 = (uint32_t)(win_bits64(w, sbit + 9 + (nch == 1 ? 5 : 3) + 4 * qch) >> 60) << 1;
    }
    const uint32_t myp23 = unit_ok ? (uint32_t)(v59 >> 47) : 0u;
    /* FFmpeg drops the frame: big_values > 288, or window
     * switching with the reserved block_type 0 */
    const bool mybad = unit_ok && (((v59 >> 38) & 0x1FFu) > 288u || (v59 & (7ull << 23)) == (4ull << 23));
    fp.sw = unit_ok ? (v59 << 5) | low5 : 0ull;
    fp.p00 = __builtin_amdgcn_readlane((int)myp23, 0);
    fp.p01 = __builtin_amdgcn_readlane((int)myp23, 1);
    fp.p10 = __builtin_amdgcn_readlane((int)myp23, 2);
    fp.p11 = __builtin_amdgcn_readlane((int)myp23, 3);
    /* MP3D_OPT_CRC_CHECK: a protected frame whose CRC-16 mismatches is
     * dropped like a bad one (FFmpeg handle_crc + explode) */
    const bool crc_bad = (opts & MP3D_OPT_CRC_CHECK) && crc && !crc16_ok(w, (uint32_t)side_bytes, lane);
    fp.bad = plen < 0 || __ballot(mybad) != 0ull || crc_bad;
    const uint32_t tgo = 4u + (uint32_t)crc + (uint32_t)side_bytes;
    fp.tag = f0 && plen >= 4 && have == (uint32_t)fb &&
             ((win_byte(w, tgo) == 'X' && win_byte(w, tgo + 1) == 'i' && win_byte(w, tgo + 2) == 'n' &&
               win_byte(w, tgo + 3) == 'g') ||
              (win_byte(w, tgo) == 'I' && win_byte(w, tgo + 1) == 'n' && win_byte(w, tgo + 2) == 'f' &&
               win_byte(w, tgo + 3) == 'o'));
    if (fp.tag && lane == 0) S.tag_info = parse_info_tag(p0 + cur + tgo, (uint32_t)fb - tgo, S.tag_frames);
}

/* The serial step: the bit-reservoir map of a parsed frame (ISO 2.4.3.4
 * main_data_begin; FFmpeg's underflow and drop rules).  P = md position of
 * the next payload, avail = md bytes after the previous main-data end (both
 * updated); sets r.first_gr, md_bit, payload_md, the dropped frame's
 * payload_len, and inf.samples; returns 1 for a frame with audio. */
__device__ __forceinline__ int resolve_frame(const FrameParse &fp, uint32_t &P, int &avail, FrameRec &r,
                                             DevInfo &inf) {
    r.payload_md = P;
    if (fp.tag) {
        r.first_gr = REC_TAG;
        return 0;
    }
    if (fp.bad) {
        /* FFmpeg drops the frame; its reservoir restarts as the frame's last
         * min(512, bytes - 4) post-header bytes (mp_decode_frame) */
        r.first_gr = REC_DROP;
        r.payload_len = (uint16_t)(fp.fb - 4);
        avail = fp.fb - 4 < MP3D_RES_BYTES ? fp.fb - 4 : MP3D_RES_BYTES;
        P += (uint32_t)r.payload_len;
        return 0;
    }
    int gr0 = 0;
    uint32_t mdbit;
    if (fp.mdb <= avail) {
        mdbit = (P - (uint32_t)fp.mdb) * 8u;
    } else {
        uint32_t bits = (uint32_t)avail * 8u;
        while (gr0 < fp.ngr && (int)(bits >> 3) < fp.mdb) {
            for (int ch = 0; ch < fp.nch; ch++) bits += (uint32_t)fp.p23(gr0, ch);
            gr0++;
        }
        mdbit = (P - (uint32_t)avail) * 8u + bits - 8u * (uint32_t)fp.mdb;
    }
    uint32_t end = mdbit;
    for (int gr = gr0; gr < 2; gr++)
        for (int ch = 0; ch < fp.nch; ch++) end += (uint32_t)fp.p23(gr, ch);
    r.md_bit = mdbit;
    r.first_gr = (uint8_t)gr0;
    P += (uint32_t)fp.plen;
    const int64_t after = (int64_t)P - (int64_t)((end + 7u) >> 3);
    avail = after < 0 ? 0 : (int)after;
    inf.samples = fp.lsf ? 576 : 1152;
    return 1;
}

/* A resolved frame's payload bytes [L, payload_len) zero (cut short), then
 * [0, L) from the stream at src_off into md at r.payload_md, in aligned
 * words built by v_alignbit and the <= 3 edge bytes as bytes.  frame_at =
 * the frame's header position (always in the stream). */
template <class M>
__device__ __forceinline__ void copy_payload(typename M::u8 *p0, uint8_t *__restrict__ dst, const FrameRec &r,
                                             uint32_t src_off, uint32_t frame_at, int lane) {
    typename M::u8 *src = p0 + src_off;
    const uint32_t Pm = r.payload_md, L = r.payload_avail;
    for (uint32_t i = L + lane; i < r.payload_len; i += 64) dst[Pm + i] = 0; /* cut-short final frame */
    const uint32_t h = min((4u - (Pm & 3u)) & 3u, L);     /* head bytes up to an aligned word */
    const uint32_t wb = (Pm + h) >> 2, we = (Pm + L) >> 2; /* whole words [wb, we)           */
    /* tail bytes [t0, L) after the last whole word -- or after the head when
     * there is none (an LSF payload can be < 8 bytes) */
    const uint32_t t0 = 4u * we > Pm + h ? 4u * we - Pm : h; /* h <= t0 <= L */
    /* edge-byte loads first, stored after the words' loads: every load of
     * the payload is in flight before the first store waits (unconditional:
     * lanes without an edge byte re-read the frame's first header byte, which
     * is always in the stream) */
    typename M::u8 *hb0 = p0 + frame_at;
    const uint8_t hbv = *((uint32_t)lane < h ? src + lane : hb0);
    const uint8_t tbv = *((uint32_t)lane < L - t0 ? src + t0 + lane : hb0);
    if (wb < we) {
        /* pointer arithmetic, not an integer round trip: the loads stay
         * global_load (a flat load waits on lgkmcnt too) */
        typename M::u8 *sb = src + (4u * wb - Pm);
        const uint32_t mis = (uint32_t)((uintptr_t)sb & 3u);
        const uint32_t sh = mis * 8u;
        typename M::u32 *swd = (typename M::u32 *)(sb - mis);
        /* all words in flight before the first store (straight-line, so no
         * loop-header wait drains them early): one load latency per frame
         * instead of one per 64-word round.  A payload is at most 1437 B
         * (1441-B frame) = 360 words < 6 x 64.  Loads are unconditional
         * (lanes past the payload re-read word 0) and the shift is
         * branch-free (alignbit by 0 = lo): with a load under a branch the
         * compiler's waitcnt pass loses track at the join and drains vmcnt
         * before every store.  The high word is read only for a misaligned
         * source (index select, not a branch): it then still holds payload
         * bytes.  Both words are aligned dwords holding at least one payload
         * byte, so no load leaves the pages of the caller's buffer. */
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

/* a resolved frame's payload_avail and copy source (the body after the
 * header and side info; a dropped frame's after the header) */
__device__ __forceinline__ uint32_t frame_body(const FrameParse &fp, FrameRec &r) {
    const uint32_t body = (r.first_gr & REC_DROP) ? 4u : fp.need;
    const uint32_t av = fp.have > body ? fp.have - body : 0u;
    r.payload_avail = (uint16_t)(av < r.payload_len ? av : r.payload_len);
    return body;
}

__device__ __forceinline__ void rec_init(FrameRec &r, uint32_t P, DevInfo &inf) {
    r.frame_off = 0; r.md_bit = 0; r.payload_md = P; r.frame_bytes = 0; r.payload_len = 0;
    r.hdr1 = r.hdr2 = r.hdr3 = 0; r.nch = 0; r.side_off = 4; r.first_gr = 0; r.sr_idx = 0; r.lsf = 0;
    r.payload_avail = 0;
    inf = {0, 0, 0, 0, 0, 0};
}

/* one stream's demux (k_demux's wave; also the per-frame k_frame's first
 * phase): stream s, lane 0..63 of the calling wave, its bytes [0, len) at p0
 * (global memory or LDS, M), base = their offset in the call's input (the
 * FrameRec frame_off origin).  No workgroup barrier inside, so one wave of a
 * larger workgroup may run it. */
template <class M>
__device__ __forceinline__ void demux_stream(typename M::u8 *p0, uint64_t base, uint32_t len, uint8_t *__restrict__ md,
                                             const uint64_t *__restrict__ md_off, StreamState *__restrict__ st,
                                             FrameRec *__restrict__ rec, uint64_t *__restrict__ sideu,
                                             DevInfo *__restrict__ infos, int F, int opts, int s, int lane) {
    uint8_t *dst = md + md_off[s];
    StreamState &S = st[s];
    /* the state's scalars in SGPRs before the frame loop: a loop-invariant
     * value still pending in a VGPR makes the compiler wait for vmcnt(0) at
     * the loop header -- every frame, behind the previous frame's stores */
    const int carry_in = __builtin_amdgcn_readfirstlane(S.res_len);
    const bool stream_start = __builtin_amdgcn_readfirstlane((int)S.frames) == 0;
    int kind = __builtin_amdgcn_readfirstlane(S.kind); /* MPEG family lock (0 until the first frame) */
    for (int i = lane; i < (carry_in + 3) / 4; i += 64) ((uint32_t *)dst)[i] = ((const uint32_t *)S.res)[i];
    __threadfence_block(); /* carry words may spill past carry_in into payload 0's head */

    uint32_t P = (uint32_t)carry_in; /* md position of the next payload         */
    int avail = carry_in;            /* bytes after the previous main-data end */
    uint32_t cur = 0;
    HdrWin w = load_win<M>(p0, len, 0, lane);
    if (stream_start && len >= 10 && win_byte(w, 0) == 'I' && win_byte(w, 1) == 'D' && win_byte(w, 2) == '3') {
        const uint32_t sz = (win_byte(w, 6) & 0x7Fu) << 21 | (win_byte(w, 7) & 0x7Fu) << 14 |
                            (win_byte(w, 8) & 0x7Fu) << 7 | (win_byte(w, 9) & 0x7Fu);
        cur = 10 + sz + ((win_byte(w, 5) & 0x10u) ? 10u : 0u);
        w = load_win<M>(p0, len, cur, lane);
    }
    int decoded = 0;
    for (int f = 0; f < F; f++) {
        const size_t fi = (size_t)s * F + f;
        /* ---- sync: the next valid header at or after cur (resync over junk) */
        int fb = -1;
        while (cur + 4 <= len) {
            if (w.pos != cur) w = load_win<M>(p0, len, cur, lane);
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
        DevInfo inf;
        rec_init(r, P, inf);
        uint64_t sw = 0; /* lane q < 4: side word of unit q = gr * 2 + ch */
        bool copy = false;
        uint32_t src_off = 0, frame_at = 0; /* payload and header positions in the stream */
        if (fb > 0) {
            if (w.pos != cur) w = load_win<M>(p0, len, cur, lane);
            FrameParse fp;
            parse_frame<M>(w, p0, base, cur, len, fb, stream_start && f == 0, opts, S, fp, r, inf, lane);
            kind = hdr_kind(fp.h1);
            if (fp.fb) {
                sw = fp.sw;
                decoded += resolve_frame(fp, P, avail, r, inf);
                const uint32_t body = frame_body(fp, r);
                copy = !(r.first_gr & REC_TAG);
                src_off = cur + body;
                frame_at = cur;
                cur = fp.have == (uint32_t)fb ? cur + (uint32_t)fb : len;
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
        if (cur + 4 <= len && f + 1 < F) w = load_win<M>(p0, len, cur, lane);
        if (copy) copy_payload<M>(p0, dst, r, src_off, frame_at, lane);
    }
    /* carry: the last min(avail, 512) md bytes become the next call's carry-in
     * (the wave's md stores complete before it reads them back) */
    __threadfence_block();
    int c = avail < MP3D_RES_BYTES ? avail : MP3D_RES_BYTES;
    if ((uint32_t)c > P) c = (int)P;
    for (int i = lane; i < c; i += 64) S.res[i] = dst[P - c + i];
    if (lane == 0) {
        S.res_len = c;
        S.frames += decoded;
        S.kind = kind;
    }
}

/* this translation unit's copies of the demux constants */
static inline hipError_t upload_demux_tables(const uint16_t *frame_bytes) {
    hipError_t e;
    uint32_t fw[9][16];
    for (int sr = 0; sr < 9; sr++)
        for (int bi = 0; bi < 16; bi++)
            fw[sr][bi] = frame_bytes[16 * sr + bi] |
                         (uint32_t)(bi < 15 ? (sr < 3 ? MP3D_BITRATE_L3[bi] : MP3D_BITRATE_L3_LSF[bi]) : 0) << 16;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_frame_word), fw, sizeof(fw)))) return e;
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

} // namespace MP3D_DEMUX_TU
} // namespace mp3d
#endif
