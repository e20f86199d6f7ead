/*
 * mp3d_demux.hip -- k_demux (§8(f) rows 1
 * and 4): per stream, frame sync over ID3v2 / junk, MPEG-1 and MPEG-2 / 2.5
 * LSF headers and side info, Xing/Info + LAME tag, optional CRC-16 check,
 * bit-reservoir map and main-data copy into the stream's md region.
 * Pipeline overview: mp3d_device.h.
 */
#include "mp3d_demux_dev.h"

namespace mp3d {

/* k_demux: one wave per stream (demux_stream, mp3d_demux_dev.h).  The
 * frame walk is serial: each header's position follows from the previous
 * frame's size, so from global memory every frame costs a dependent HBM
 * round trip (~2.5 us a frame on MI355X).  A stream of at most DMX_STAGE
 * bytes is first staged whole into LDS -- its aligned 16-B blocks, all
 * loads of a round in flight together -- and walked from there: the serial
 * chain then runs on LDS latency.  Longer streams walk global memory. */
#define DMX_STAGE (48 * 1024)
#define DMX_ROUND 16 /* 16-B blocks per lane in flight per staging round */
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 8)))
k_demux(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ in_len,
        uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off, StreamState *__restrict__ st,
        FrameRec *__restrict__ rec, uint64_t *__restrict__ sideu, DevInfo *__restrict__ infos, int F, int opts) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4))); /* (an array of HIP's uint4 stays in scratch) */
    __shared__ __attribute__((aligned(16))) u32x4 s_stage[DMX_STAGE / 16];
    const int s = blockIdx.x, lane = threadIdx.x;
    const uint64_t base = in_off[s];
    const uint32_t len = in_len[s];
    const uint8_t *g = in + base;
    /* the blocks holding stream bytes: each is an aligned 16-B block with at
     * least one byte of [g, g + len), so no load leaves the caller's pages */
    const uintptr_t g0 = (uintptr_t)g & ~(uintptr_t)15;
    const uint32_t nblk = len ? (uint32_t)(((uintptr_t)g + len - g0 + 15) / 16) : 0u;
    if (nblk + 1u <= DMX_STAGE / 16) {
        const u32x4 *src = (const u32x4 *)g0;
        for (uint32_t b0 = 0; b0 < nblk; b0 += 64u * DMX_ROUND) {
            u32x4 v[DMX_ROUND];
#pragma unroll
            for (int k = 0; k < DMX_ROUND; k++) {
                const uint32_t i = b0 + 64u * k + (uint32_t)lane;
                v[k] = src[i < nblk ? i : 0u]; /* unconditional: the loads stay in flight together */
            }
#pragma unroll
            for (int k = 0; k < DMX_ROUND; k++) {
                const uint32_t i = b0 + 64u * k + (uint32_t)lane;
                if (i < nblk) s_stage[i] = v[k];
            }
        }
        if (lane == 0) s_stage[nblk] = (u32x4){0u, 0u, 0u, 0u};
        wave_sync(); /* one wave: its LDS stores land before its loads */
        SrcLds::u8 *p0 = (SrcLds::u8 *)(uintptr_t)s_stage + ((uintptr_t)g - g0);
        demux_stream<SrcLds>(p0, base, len, md, md_off, st, rec, sideu, infos, F, opts, s, lane);
    } else {
        demux_stream<SrcGlobal>(g, base, len, md, md_off, st, rec, sideu, infos, F, opts, s, lane);
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

/* a window's four 16-B aligned blocks around stream offset pos, as loaded
 * (walk_fetch) and then masked into the lane's LDS words (walk_commit): the
 * loads of the next frame's window go out before the current frame's record
 * stores, so its wait does not also wait for them (one vmcnt counter) */
struct WinRaw {
    uint4 v[4];
    uint32_t pos, mis;
};
/* every loaded block holds a stream byte (so none leaves the pages of the
 * caller's buffer, which are 16-B aligned units) or is not loaded */
__device__ __forceinline__ void walk_fetch(WinRaw &R, const uint8_t *p0, uint32_t len, uint32_t pos) {
    R.pos = pos;
    R.mis = (uint32_t)((uintptr_t)(p0 + pos) & 15u);
    const uint4 *base = (const uint4 *)(p0 + pos - R.mis);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t first = (int64_t)pos - (int64_t)R.mis + 16 * j; /* stream offset of the block */
        R.v[j] = make_uint4(0u, 0u, 0u, 0u);
        if (first < (int64_t)len) R.v[j] = base[j];
    }
}
/* pos < len: block 0 holds a stream byte, and a block past the end re-reads
 * it (walk_commit zeroes its bytes) -- no branch around the loads */
__device__ __forceinline__ void walk_fetch_in(WinRaw &R, const uint8_t *p0, uint32_t len, uint32_t pos) {
    R.pos = pos;
    R.mis = (uint32_t)((uintptr_t)(p0 + pos) & 15u);
    const uint4 *base = (const uint4 *)(p0 + pos - R.mis);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t first = (int64_t)pos - (int64_t)R.mis + 16 * j;
        R.v[j] = *(first < (int64_t)len ? base + j : base);
    }
}
/* bytes at or past len read as zero */
__device__ __forceinline__ void walk_commit(LaneWin &W, const WinRaw &R, uint32_t len) {
    W.pos = R.pos;
    W.mis = R.mis;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t over = (int64_t)R.pos - (int64_t)R.mis + 16 * j + 16 - (int64_t)len; /* bytes past the end */
        uint32_t q[4] = {R.v[j].x, R.v[j].y, R.v[j].z, R.v[j].w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t o = over - 4 * (3 - i); /* bytes of word i past the end */
            q[i] = o >= 4 ? 0u : o > 0 ? q[i] & (0xFFFFFFFFu >> (8 * o)) : q[i];
            W.w[4 * j + i] = q[i];
        }
    }
}
__device__ __forceinline__ void walk_load(LaneWin &W, const uint8_t *p0, uint32_t len, uint32_t pos) {
    WinRaw R;
    walk_fetch(R, p0, len, pos);
    walk_commit(W, R, len);
}

/* the header's frame word from the workgroup's LDS copy of c_frame_word
 * (frame bytes | bitrate << 16, padding added), or 0: not a Layer III
 * header of the stream's family (hdr_frame_bytes' checks) */
__device__ __forceinline__ uint32_t walk_frame_word(const uint32_t *s_fw, uint32_t b1, uint32_t b2, int kind) {
    if ((b1 & 0xE0) != 0xE0 || ((b1 >> 1) & 3) != 1 || ((b1 >> 3) & 3) == 1) return 0u;
    const uint32_t bi = b2 >> 4;
    if (bi == 0 || bi == 15 || ((b2 >> 2) & 3) == 3) return 0u;
    if (kind && hdr_kind(b1) != kind) return 0u;
    return s_fw[16 * hdr_sr_idx(b1, b2) + bi] + ((b2 >> 1) & 1u);
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
                                             DevInfo *__restrict__ infos, int n_streams, int F, int opts,
                                             uint32_t *__restrict__ fam, uint32_t seq) {
    __shared__ uint32_t s_win[64 * WALK_WORDS];
    /* frame words and sample rates in LDS: a constant-table read per frame
     * from L2 was a round trip on the frame chain */
    __shared__ uint32_t s_fw[9 * 16], s_hz[9];
    const int lane = threadIdx.x;
    for (int i = lane; i < 9 * 16; i += 64) s_fw[i] = (&c_frame_word[0][0])[i];
    if (lane < 9) s_hz[lane] = MP3D_SAMPLE_RATE[lane];
    __syncthreads();
    const int s = blockIdx.x * WALK_LANES + lane;
    if (lane >= WALK_LANES || s >= n_streams) return; /* no barrier below */
    LaneWin W;
    W.w = s_win + lane * WALK_WORDS;
    const uint64_t off_s = in_off[s];
    const uint8_t *p0 = in + off_s;
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
        uint32_t fw = 0u;
        while (cur + 4 <= len) {
            if (W.pos != cur) walk_load(W, p0, len, cur);
            const uint32_t lim = min(46u, len - cur - 4);
            uint32_t k = 0;
            for (; k <= lim; k++) {
                if (W.byte(k) == 0xFFu) {
                    fw = walk_frame_word(s_fw, W.byte(k + 1), W.byte(k + 2), kind);
                    fb = fw ? (int)(fw & 0xFFFFu) : -1;
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
                r.frame_off = off_s + cur;
                r.frame_bytes = (uint16_t)fb;
                r.payload_len = (uint16_t)(plen > 0 ? plen : 0);
                r.hdr1 = (uint8_t)h1; r.hdr2 = (uint8_t)h2; r.hdr3 = (uint8_t)h3;
                r.nch = (uint8_t)nch;
                r.side_off = (uint8_t)(4 + crc);
                r.sr_idx = (uint8_t)hdr_sr_idx(h1, h2);
                r.lsf = (uint8_t)lsf;
                inf.frame_bytes = fb; inf.channels = nch; inf.hz = (int)s_hz[r.sr_idx];
                inf.layer = 3; inf.bitrate_kbps = (int)(fw >> 16);
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
        /* the next frame's window loads first, then this frame's record
         * stores, then the window into LDS (its wait leaves the stores in
         * flight); a lane without a next frame re-reads its side words */
        ulonglong2 *sd = (ulonglong2 *)&sideu[fi * 4];
        const bool more = cur + 4 <= len && f + 1 < F;
        WinRaw nx;
        walk_fetch_in(nx, more ? p0 : (const uint8_t *)sd, more ? len : 16u, more ? cur : 0u);
        rec[fi] = r;
        if (infos) infos[fi] = inf;
        sd[0] = make_ulonglong2(sw[0], sw[1]);
        sd[1] = make_ulonglong2(sw[2], sw[3]);
        if (more) walk_commit(W, nx, len);
    }
    int c = avail < MP3D_RES_BYTES ? avail : MP3D_RES_BYTES;
    if ((uint32_t)c > P) c = (int)P;
    S.frames += decoded;
    S.kind = kind;
    /* the batch holds an LSF stream: tag the family word with this call's
     * seq (lanes store the same value; k_synth's LSF variant reads it) */
    if (fam && kind == 2) *fam = seq;
    S.pad_[0] = (int32_t)P; /* md end, for k_mdcopy */
    S.pad_[1] = c;          /* next carry length   */
}

/* k_mdcopy: one wave per stream, 4 streams per workgroup.  Carry-in, then
 * the payloads four frames at a time (16 lanes each, so four frames' loads
 * are in flight together), then the next carry.  Each lane first loads the
 * copy descriptor of one frame (lane f: frame f of a 64-frame chunk), so the
 * frame loop reads no record from memory.  Payload words: the destination
 * is written in aligned words, each funnel-shifted from two source words by
 * the source misalignment (the k_demux copy; edge bytes and a cut-short
 * tail as there), four per lane and store.  All loads of an iteration are straight-line and
 * unconditional (lanes without work re-read a valid word): a load under a
 * branch makes the compiler's waitcnt pass drain vmcnt(0) at the join.  An
 * aligned source loads words (k - 1, k) instead of (k, k + 1), so no load
 * passes the payload's last word (word -1 is side info or header). */
#define MDC_WAVES 16
#define MDC_QROUNDS 2 /* 16-lane rounds of word quadruples per frame, unrolled: 512 B */
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
                /* whole quadruples of words: lane ql builds words 4 q .. 4 q + 3
                 * (q = 16 j + ql) from source words 4 q .. 4 q + 4 (one 16-B and
                 * one 4-B load, dword-aligned) and stores them with one 16-B
                 * store: a quarter of the stores and half the loads of one word
                 * per lane.  A quadruple reads up to word 4 q + 4 <= nwd, so only
                 * whole ones (q < nq) are copied here; the others load from the
                 * stream's own md region (>= 20 readable bytes, unlike a cut-short
                 * final frame's source) and their stores are masked by an
                 * out-of-range offset (not a branch: the compiler would sink each
                 * load into its store's branch). */
                const uint32_t nq = nwd >> 2;
                uint4 v[MDC_QROUNDS];
#pragma unroll
                for (int j = 0; j < MDC_QROUNDS; j++) {
                    const uint32_t q = 16u * j + (uint32_t)ql;
                    const uint32_t *L = q < nq ? lp + 4u * q : (const uint32_t *)dst;
                    uint4 a;
                    __builtin_memcpy(&a, L, 16);
                    const uint32_t e = L[4];
                    v[j] = make_uint4(__builtin_amdgcn_alignbit(a.y, sh ? a.x : a.y, sh),
                                      __builtin_amdgcn_alignbit(a.z, sh ? a.y : a.z, sh),
                                      __builtin_amdgcn_alignbit(a.w, sh ? a.z : a.w, sh),
                                      __builtin_amdgcn_alignbit(e, sh ? a.w : e, sh));
                }
#pragma unroll
                for (int j = 0; j < MDC_QROUNDS; j++) {
                    const uint32_t q = 16u * j + (uint32_t)ql;
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v[j]), r_md,
                        q < nq ? 4u * (wb + 4u * q) : 0x80000000u, 0, 0);
                }
                /* the rest one word per lane: the last partial quadruple and
                 * payloads past the unrolled 16 MDC_QROUNDS quadruples */
                for (uint32_t k = 4u * min(nq, 16u * MDC_QROUNDS) + (uint32_t)ql; k < nwd; k += 16) {
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
hipError_t upload_demux_constants(const uint16_t *frame_bytes) { return upload_demux_tables(frame_bytes); }

/* wide: k_walk + k_mdcopy (batches of many streams); else one k_demux wave
 * per stream (fewer launches: the per-frame decoder, small batches) */
/* ------------------------------------------------------------------------ */
/* k_demux_fp: one stream's run of pre-located, complete frames (the per-  */
/* frame decoder's read-ahead runs, mp3d_host.cpp ra_fill: the host has     */
/* found every frame, fo[f] = its header offset in the run's bytes, passed  */
/* as kernel arguments) demuxed frame-parallel in ONE workgroup, with the   */
/* same results as k_demux: the run's bytes are staged in LDS, wave 0       */
/* parses every frame's header and side info on its own lane and runs the  */
/* bit-reservoir map over them (a prefix scan: resolve_frame's rules), then */
/* the waves write the records and copy the payloads in parallel.  It also  */
/* does the run's state book-keeping that would otherwise be separate       */
/* copies: the previous run's synthesis tail into StreamState (tail_in, may */
/* be null) and then the snapshot of the state before the run (snap) that a */
/* settle restores.                                                        */
/* ------------------------------------------------------------------------ */
#define FP_WAVES 16
#define FP_MAX 64   /* frames per run (MP3D_PF_READAHEAD <= 64): one lane of wave 0 each */
struct FpRes {      /* what the serial resolve needs of a parsed frame */
    int fb, plen, mdb;
    uint32_t need, at; /* at: the header's offset in the run */
    int p00, p01, p10, p11;
    uint32_t flags; /* bit 0 lsf, 1 bad, 2 tag, 3 two channels */
};
struct FpOut {      /* what it decides */
    uint32_t payload_md, md_bit, lens; /* lens: payload_len | payload_avail << 16 */
    uint32_t gr_samples;              /* first_gr | samples << 8 */
};
/* the run's frame offsets, by value (kernel arguments: scalar loads, no
 * round trip to the host buffer) */
struct FpOffs {
    uint32_t o[FP_MAX];
};
#define FP_STAGE (FP_MAX * MP3D_MAX_FRAME_BYTES + 64) /* the run's bytes staged in LDS */
__global__ void __launch_bounds__(64 * FP_WAVES)
k_demux_fp(const uint8_t *__restrict__ in, uint32_t len, FpOffs fo, uint8_t *__restrict__ md,
           StreamState *__restrict__ st, const float *__restrict__ tail_in, StreamState *__restrict__ snap,
           FrameRec *__restrict__ rec, uint64_t *__restrict__ sideu, DevInfo *__restrict__ infos, int F, int opts) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) u32x4 s_run[(FP_STAGE + 15) / 16];
    __shared__ FpRes s_res[FP_MAX];
    __shared__ FpOut s_out[FP_MAX];
    __shared__ uint32_t s_h1[FP_MAX];
    __shared__ FrameRec s_rec[FP_MAX];
    __shared__ DevInfo s_inf[FP_MAX];
    __shared__ int s_fin[3];
    __shared__ uint32_t s_tab[HDR_TAB_WORDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    constexpr int NT = 64 * FP_WAVES;
    StreamState &S = st[0];
    /* the frame offsets (kernel arguments): all 64 loaded here, together,
     * into lane f of every wave -- as fo.o[f] inside the frame loop each was
     * a scalar load with its own round trip (8 of the kernel's 22 us) */
    uint32_t fo_lane = 0u;
#pragma unroll
    for (int k = 0; k < FP_MAX; k++) fo_lane = lane == k ? fo.o[k] : fo_lane;
    /* the run's bytes (the mapped host buffer, 16-B aligned) into LDS: every
     * block's load in flight at once -- one bus round trip for the run; the
     * parse and the payload copy then read LDS */
    const uint32_t nblk = (len + 15u) / 16u;
    constexpr int PER = ((FP_STAGE + 15) / 16 + NT - 1) / NT;
    u32x4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t i = (uint32_t)tid + (uint32_t)(NT * k);
        v[k] = ((const u32x4 *)in)[i < nblk ? i : 0u]; /* unconditional: the loads stay in flight together */
    }
    /* meanwhile: the previous run's final overlap + history (a segmented
     * synthesis leaves them in the handle's tail) into the state, and the
     * state before this run (tail applied) into the snapshot, in one pass */
    constexpr int TAIL0 = (int)(offsetof(StreamState, overlap) / 4);
    constexpr int TAILW = (int)(sizeof(S.overlap) + sizeof(S.fifo)) / 4;
    for (int i = tid; i < (int)(sizeof(StreamState) / 4); i += NT) {
        const bool t = tail_in && i >= TAIL0 && i < TAIL0 + TAILW;
        const uint32_t x = t ? ((const uint32_t *)tail_in)[i - TAIL0] : ((const uint32_t *)&S)[i];
        if (t) ((uint32_t *)&S)[i] = x;
        ((uint32_t *)snap)[i] = x;
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t i = (uint32_t)tid + (uint32_t)(NT * k);
        if (i < nblk) s_run[i] = v[k];
    }
    if (tid == 0) s_run[nblk] = (u32x4){0u, 0u, 0u, 0u}; /* (the tail: the host zeroed 64 B past the frames too) */
    hdr_tab_stage(s_tab, tid);
    const HdrTabLds ht = {(const __attribute__((address_space(3))) uint32_t *)s_tab};
    __syncthreads(); /* the staged bytes; every read of the state before the run (the tag write below) */
    SrcLds::u8 *p0 = (SrcLds::u8 *)(uintptr_t)s_run;
    uint8_t *dst = md;
    const int carry_in = __builtin_amdgcn_readfirstlane(S.res_len);
    const bool stream_start = __builtin_amdgcn_readfirstlane((int)S.frames) == 0;
    if (wv == FP_WAVES - 1)
        for (int i = lane; i < (carry_in + 3) / 4; i += 64) ((uint32_t *)dst)[i] = ((const uint32_t *)S.res)[i];
    /* Wave 0 alone: the frames' headers and side info, lane f = frame f
     * (k_walk's lane-per-stream parse, over the staged run), then the
     * bit-reservoir map over them.  (A wave per frame, four frames in turn
     * per wave, spent 8.7 of the kernel's 22 us on its chains of cross-lane
     * reads: s_memrealtime stamps, build FPT.)
     * The map (resolve_frame's rules) for all frames at once: each
     * payload's md position is a prefix sum of the payload lengths; the
     * bytes available after a frame depend on the frames before it only
     * through the underflow test mdb > avail, so every frame's "avail after"
     * is first taken as if no frame underflowed, the avail before each frame
     * found by a last-setter scan, and the frames that do underflow
     * recomputed until nothing changes (one pass unless a stream starts
     * mid-way or a frame is dropped).  Done serially by one wave this step
     * took 17 of the kernel's 30 us (32 frames). */
    if (wv == 0) {
        const bool live = lane < F;
        FpRes q = {0, 0, 0, 0u, 0u, 0, 0, 0, 0, 0u};
        FrameRec r;
        DevInfo inf;
        rec_init(r, 0u, inf);
        uint32_t h1 = 0u; /* stays 0: no header found (a valid one has h1 >= 0xE0) */
        uint64_t sw[4] = {0ull, 0ull, 0ull, 0ull};
        if (live) {
            const uint32_t cur = fo_lane;
            LaneWin W; /* the frame's bytes where they are staged (64 zero bytes follow the run) */
            W.w = (uint32_t *)s_run + (cur >> 2);
            W.pos = cur;
            W.mis = cur & 3u;
            const uint32_t b1 = W.byte(1), b2 = W.byte(2), b3 = W.byte(3);
            /* (the family was checked on the host: every frame's header is of
             * the stream's family) */
            const int fb = hdr_frame_bytes(b1, b2, 0, ht);
            const int nch = (b3 >> 6) == 3 ? 1 : 2;
            const int crc = (b1 & 1) ? 0 : 2;
            const bool lsf = hdr_kind(b1) == 2;
            const int ngr = lsf ? 1 : 2;
            const int side_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
            const uint32_t need = 4u + (uint32_t)crc + (uint32_t)side_bytes;
            /* a final frame cut short still decodes (FFmpeg: the missing
             * bytes read as zeros) once its header and side info are present */
            if (fb > 0 && (cur + (uint32_t)fb <= len || cur + need <= len)) {
                const uint32_t have = min(len - cur, (uint32_t)fb);
                const int plen = fb - 4 - crc - side_bytes;
                r.frame_off = cur;
                r.frame_bytes = (uint16_t)fb;
                r.payload_len = (uint16_t)(plen > 0 ? plen : 0);
                r.hdr1 = (uint8_t)b1; r.hdr2 = (uint8_t)b2; r.hdr3 = (uint8_t)b3;
                r.nch = (uint8_t)nch;
                r.side_off = (uint8_t)(4 + crc);
                r.sr_idx = (uint8_t)hdr_sr_idx(b1, b2);
                r.lsf = (uint8_t)lsf;
                inf.frame_bytes = fb; inf.channels = nch; inf.hz = (int)ht.hz(r.sr_idx);
                inf.layer = 3; inf.bitrate_kbps = (int)(ht.fw(r.sr_idx, (int)(b2 >> 4)) >> 16);
                const uint32_t sbit = 8u * (4u + (uint32_t)crc);
                const int mdb = (int)(W.bits64(sbit) >> (lsf ? 56 : 55));
                uint32_t p23[4] = {0u, 0u, 0u, 0u};
                bool anybad = false;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int qgr = u >> 1, qch = u & 1;
                    if (qch < nch && qgr < ngr) {
                        const uint32_t ub = sbit + side_unit_bit(nch, qgr, qch, lsf);
                        uint64_t v59;
                        uint32_t low5;
                        if (lsf) { /* the 63-bit LSF unit in the MPEG-1 layout (parse_frame) */
                            const uint64_t v63 = W.bits64(ub) >> 1;
                            const uint32_t sfc9 = (uint32_t)(v63 >> 25) & 511u;
                            const uint64_t low25 = v63 & 0x1FFFFFFull;
                            const bool is_right = (b3 >> 6) == 1 && ((b3 >> 4) & 1) && qch == 1;
                            v59 = ((v63 >> 34) << 30) | ((uint64_t)(sfc9 & 15u) << 26) | ((low25 >> 2) << 3) |
                                  ((uint64_t)is_right << 2) | (low25 & 3u);
                            low5 = sfc9 >> 4;
                        } else {
                            v59 = W.bits64(ub) >> 5;
                            low5 = (uint32_t)(W.bits64(sbit + 9 + (nch == 1 ? 5 : 3) + 4 * qch) >> 60) << 1;
                        }
                        p23[u] = (uint32_t)(v59 >> 47);
                        /* FFmpeg drops the frame: big_values > 288, or window
                         * switching with the reserved block_type 0 */
                        anybad |= ((v59 >> 38) & 0x1FFu) > 288u || (v59 & (7ull << 23)) == (4ull << 23);
                        sw[u] = (v59 << 5) | low5;
                    }
                }
                const bool crc_bad = (opts & MP3D_OPT_CRC_CHECK) && crc && !walk_crc_ok(W, (uint32_t)side_bytes);
                const uint32_t tgo = 4u + (uint32_t)crc + (uint32_t)side_bytes;
                const bool tag = stream_start && lane == 0 && plen >= 4 && have == (uint32_t)fb &&
                                 ((W.byte(tgo) == 'X' && W.byte(tgo + 1) == 'i' && W.byte(tgo + 2) == 'n' &&
                                   W.byte(tgo + 3) == 'g') ||
                                  (W.byte(tgo) == 'I' && W.byte(tgo + 1) == 'n' && W.byte(tgo + 2) == 'f' &&
                                   W.byte(tgo + 3) == 'o'));
                if (tag) S.tag_info = parse_info_tag(p0 + cur + tgo, (uint32_t)fb - tgo, S.tag_frames);
                q.fb = fb; q.plen = plen; q.mdb = mdb; q.need = need; q.at = cur;
                q.p00 = (int)p23[0]; q.p01 = (int)p23[1]; q.p10 = (int)p23[2]; q.p11 = (int)p23[3];
                q.flags = (lsf ? 1u : 0u) | ((plen < 0 || anybad || crc_bad) ? 2u : 0u) | (tag ? 4u : 0u) |
                          (nch == 2 ? 8u : 0u);
                h1 = b1;
            }
            ulonglong2 *sd = (ulonglong2 *)&sideu[(size_t)lane * 4];
            sd[0] = make_ulonglong2(sw[0], sw[1]);
            sd[1] = make_ulonglong2(sw[2], sw[3]);
            s_res[lane] = q;
            s_h1[lane] = h1;
            s_rec[lane] = r;
            s_inf[lane] = inf;
        }
        const bool found = live && q.fb != 0;
        const bool tag = found && (q.flags & 4u);
        const bool bad = found && !tag && (q.flags & 2u);
        const bool aud = found && !tag && !bad;
        const int delta = bad ? q.fb - 4 : aud ? q.plen : 0;
        int incl = delta;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        const uint32_t Pb = (uint32_t)carry_in + (uint32_t)(incl - delta), Pa = Pb + (uint32_t)delta;
        const uint32_t g0 = (uint32_t)(q.p00 + q.p01), g1 = (uint32_t)(q.p10 + q.p11); /* per granule (0 if absent) */
        const int ngr = (q.flags & 1u) ? 1 : 2;
        const bool sets = bad || aud; /* tags and empty slots pass avail through */
        /* avail after this frame from avail before it (resolve_frame) */
        auto after = [&](int av_prev, int &gr0, uint32_t &mdbit) {
            if (bad) return q.fb - 4 < MP3D_RES_BYTES ? q.fb - 4 : MP3D_RES_BYTES;
            gr0 = 0;
            if (q.mdb <= av_prev) {
                mdbit = (Pb - (uint32_t)q.mdb) * 8u;
            } else {
                uint32_t bits = (uint32_t)av_prev * 8u;
                while (gr0 < ngr && (int)(bits >> 3) < q.mdb) {
                    bits += gr0 ? g1 : g0;
                    gr0++;
                }
                mdbit = (Pb - (uint32_t)av_prev) * 8u + bits - 8u * (uint32_t)q.mdb;
            }
            const uint32_t end = mdbit + (gr0 == 0 ? g0 : 0u) + (gr0 <= 1 ? g1 : 0u);
            const int64_t a = (int64_t)Pa - (int64_t)((end + 7u) >> 3);
            return a < 0 ? 0 : (int)a;
        };
        int gr0 = 0;
        uint32_t mdbit = 0u;
        int av = sets ? after(1 << 30, gr0, mdbit) : 0; /* as if nothing underflowed */
        int av_prev = carry_in, last = carry_in;
        for (int it = 0; it <= 64; it++) {
            /* last setter at or before each lane (inclusive), then shifted */
            int val = av, set = sets ? 1 : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int tv = __shfl_up(val, o), ts = __shfl_up(set, o);
                if (lane >= o && !set) {
                    val = tv;
                    set = ts;
                }
            }
            const int pv = __shfl_up(val, 1), ps = __shfl_up(set, 1);
            av_prev = (lane == 0 || !ps) ? carry_in : pv;
            last = __shfl(set ? val : carry_in, F > 0 ? F - 1 : 0);
            const int av2 = sets ? after(av_prev, gr0, mdbit) : 0;
            const bool changed = __ballot(av2 != av) != 0ull;
            av = av2;
            if (!changed) break;
        }
        if (live) {
            FpOut o;
            o.payload_md = Pb;
            o.md_bit = aud ? mdbit : 0u;
            const uint32_t plen = bad ? (uint32_t)(q.fb - 4) : (uint32_t)(q.plen > 0 ? q.plen : 0);
            const uint32_t body = bad ? 4u : q.need;
            const uint32_t avb = (uint32_t)q.fb > body ? (uint32_t)q.fb - body : 0u; /* complete frames */
            o.lens = plen | (found ? (avb < plen ? avb : plen) : 0u) << 16;
            o.gr_samples = tag ? (uint32_t)REC_TAG
                               : bad ? (uint32_t)REC_DROP
                                     : aud ? (uint32_t)gr0 | (uint32_t)((q.flags & 1u) ? 576 : 1152) << 8 : 0u;
            s_out[lane] = o;
        }
        const uint32_t P_end = F > 0 ? (uint32_t)__shfl((int)Pa, F - 1) : (uint32_t)carry_in;
        const int decoded = __popcll(__ballot(aud));
        if (lane == 0) {
            s_fin[0] = (int)P_end;
            s_fin[1] = F > 0 ? last : carry_in;
            s_fin[2] = decoded;
        }
    }
    __syncthreads();
    /* records and payloads, the wave's own frames */
#pragma unroll 1
    for (int f = wv; f < F; f += FP_WAVES) {
        const FpOut o = s_out[f];
        const FpRes q = s_res[f];
        FrameRec r = s_rec[f];
        DevInfo inf = s_inf[f];
        r.payload_md = o.payload_md;
        if (q.fb) {
            r.md_bit = o.md_bit;
            r.payload_len = (uint16_t)(o.lens & 0xFFFFu);
            r.payload_avail = (uint16_t)(o.lens >> 16);
            r.first_gr = (uint8_t)(o.gr_samples & 0xFFu);
            inf.samples = (int)(o.gr_samples >> 8);
        }
        if (lane == 0) {
            rec[f] = r;
            if (infos) infos[f] = inf;
        }
        if (q.fb && !(r.first_gr & REC_TAG)) {
            const uint32_t body = (r.first_gr & REC_DROP) ? 4u : q.need;
            copy_payload<SrcLds>(p0, dst, r, q.at + body, q.at, lane);
        }
    }
    if (wv == 0) {
        /* the next carry: md bytes [P - c, P), taken from the staged run (or,
         * before the run's first payload, from the carry-in), not read back
         * from md -- so no barrier waits for the other waves' md stores */
        const uint32_t P = (uint32_t)s_fin[0];
        const int avail = s_fin[1];
        int c = avail < MP3D_RES_BYTES ? avail : MP3D_RES_BYTES;
        if ((uint32_t)c > P) c = (int)P;
        for (int i = lane; i < c; i += 64) {
            const uint32_t x = P - (uint32_t)c + (uint32_t)i;
            /* the frame whose copied payload holds md byte x (payloads are
             * back to back in md; a tag frame copies none) */
            int f = F - 1;
            for (; f >= 0; f--) {
                const FpOut o = s_out[f];
                const uint32_t plen = (o.gr_samples & REC_TAG) ? 0u : (o.lens & 0xFFFFu);
                if (x >= o.payload_md && x < o.payload_md + plen) break;
            }
            uint32_t v;
            if (f < 0) {
                v = S.res[x]; /* the carry-in (md [0, carry_in)); x >= i: read before overwritten */
            } else {
                const FpOut o = s_out[f];
                const FpRes q = s_res[f];
                const uint32_t off = x - o.payload_md;
                const uint32_t body = (o.gr_samples & REC_DROP) ? 4u : q.need;
                v = off < (o.lens >> 16) ? (uint32_t)p0[q.at + body + off] : 0u; /* past the bytes present: zeros */
            }
            S.res[i] = (uint8_t)v;
        }
        /* the family of the last frame found (k_demux: of every frame) */
        int kind = __builtin_amdgcn_readfirstlane(S.kind);
        for (int f = 0; f < F; f++)
            if (s_h1[f]) kind = hdr_kind(s_h1[f]);
        if (lane == 0) {
            S.res_len = c;
            S.frames += s_fin[2];
            S.kind = kind;
        }
    }
}

/* one pre-located run (k_demux_fp): in = its bytes (len), fo = its F frame
 * offsets (host array, passed by value), md = the handle's md region (stream
 * 0 at offset 0) */
void launch_demux_fp(const uint8_t *in, uint32_t len, const uint32_t *fo, uint8_t *md, StreamState *st,
                     const float *tail_in, StreamState *snap, FrameRec *rec, uint64_t *sideu, void *infos, int F,
                     int opts, hipStream_t strm) {
    FpOffs o = {};
    for (int f = 0; f < F && f < FP_MAX; f++) o.o[f] = fo[f];
    hipLaunchKernelGGL(k_demux_fp, dim3(1), dim3(64 * FP_WAVES), 0, strm, in, len, o, md, st, tail_in, snap, rec,
                       sideu, (DevInfo *)infos, F, opts);
}

void launch_demux(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint8_t *md,
                  const uint64_t *md_off, StreamState *st, FrameRec *rec, uint64_t *sideu, void *infos, int n_streams,
                  int F, int opts, bool wide, uint32_t *fam, uint32_t seq, hipStream_t strm) {
    if (wide) {
        hipLaunchKernelGGL(k_walk, dim3((n_streams + WALK_LANES - 1) / WALK_LANES), dim3(64), 0, strm, in, in_off,
                           in_len, st, rec, sideu, (DevInfo *)infos, n_streams, F, opts, fam, seq);
        hipLaunchKernelGGL(k_mdcopy, dim3((n_streams + MDC_WAVES - 1) / MDC_WAVES), dim3(64 * MDC_WAVES), 0, strm, in,
                           md, md_off, st, (const FrameRec *)rec, n_streams, F);
        return;
    }
    hipLaunchKernelGGL(k_demux, dim3(n_streams), dim3(64), 0, strm, in, in_off, in_len, md, md_off, st, rec, sideu,
                       (DevInfo *)infos, F, opts);
}

} // namespace mp3d
