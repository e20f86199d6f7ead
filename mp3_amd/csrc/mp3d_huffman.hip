/*
 * mp3d_huffman.hip -- k_huffman (ISO 11172-3
 * 2.4.2.7 + Annex B, 13818-3 2.4.3.2): scalefactors (MPEG-1 scfsi reuse, LSF
 * groups) and the big_values / count1 Huffman decode of every unit into
 * is[576] + UnitMeta.  Pipeline overview: mp3d_device.h.
 */
#include <algorithm>

#include "mp3d_huffman_dev.h"

namespace mp3d {

/* ---- ranking (k_rank): the units of each RANK_SEG-unit segment in
 * descending big_values order, by a counting sort in LDS, so each 64-unit
 * round of k_huffman holds units of (nearly) one length: the branch-free
 * big_values loop runs max-over-lanes iterations.  On C3 (generator side
 * info) rounds ranked over 256 units run 1.50x the lane-steps of an exact
 * order, over 4 096 units 1.03x.  A whole-launch order (1.00x) scattered
 * each round's rows over the whole is[] buffer and ran slower.  The order
 * inside a bin is the order of the LDS atomics (not deterministic): it
 * changes which lane decodes a unit, not what is decoded. */
#define RANK_BINS 320   /* big_values 0 .. 319 (the field's legal range is 0 .. 288) */
#define RANK_BLOCK 1024
#define RANK_PER 4      /* units per thread */
#define RANK_SEG (RANK_BLOCK * RANK_PER)
__global__ void __launch_bounds__(RANK_BLOCK) k_rank(const uint64_t *__restrict__ sideu, int n_units,
                                                     uint32_t *__restrict__ perm) {
    __shared__ uint32_t h[RANK_BINS];
    const int tid = threadIdx.x, seg0 = blockIdx.x * RANK_SEG;
    for (int i = tid; i < RANK_BINS; i += RANK_BLOCK) h[i] = 0u;
    __syncthreads();
    uint32_t bin[RANK_PER], r[RANK_PER];
#pragma unroll
    for (int j = 0; j < RANK_PER; j++) {
        const int u = seg0 + j * RANK_BLOCK + tid;
        const uint32_t bv = u < n_units ? (uint32_t)(sideu[u] >> 43) & 0x1FFu : 0u;
        bin[j] = RANK_BINS - 1u - (bv < RANK_BINS ? bv : RANK_BINS - 1u); /* descending big_values */
        r[j] = u < n_units ? atomicAdd(&h[bin[j]], 1u) : 0u;
    }
    __syncthreads();
    if (tid < 64) {
        /* exclusive scan of the counts: lane owns bins 5 lane .. +4 */
        uint32_t c[5], sum = 0u;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            c[k] = h[5 * tid + k];
            sum += c[k];
        }
        const uint32_t incl = wave_incl_scan(sum);
        uint32_t run = incl - sum;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            h[5 * tid + k] = run;
            run += c[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RANK_PER; j++) {
        const int u = seg0 + j * RANK_BLOCK + tid;
        if (u < n_units) perm[seg0 + h[bin[j]] + r[j]] = (uint32_t)u;
    }
}

/* k_huffman: one lane per unit (its layout constants and helpers: mp3d_huffman_dev.h) */
/* work: the handle's work-item counter (zeroed before the launch); perm: each
 * segment's units in descending big_values order (k_rank).  Work item t =
 * units perm[64 t .. 64 t + 63]. */
__global__ void __launch_bounds__(HUFF_BLOCK) k_huffman(const uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off,
                                                        const FrameRec *__restrict__ rec,
                                                        const uint64_t *__restrict__ sideu,
                                                        const DevTables *__restrict__ tab, int16_t *__restrict__ is_buf,
                                                        UnitMeta *__restrict__ meta, int n_units, int F,
                                                        uint32_t *__restrict__ work, const uint32_t *__restrict__ perm) {
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[MP3D_LUT_MAX];
    /* per-wave staging areas after a 4-word guard: win64g / win32g read the
     * word below a window that starts on a word boundary */
    __shared__ __attribute__((aligned(16))) uint32_t s_bits[4 + HUFF_WAVES * (HUFF_CAPW + 4)];
    __shared__ uint32_t s_tsel[32]; /* table_select -> LUT base | (32 - bits1) << 16 | linbits << 24 */
    __shared__ uint16_t s_lbnd[9][24]; /* long sfb start line per sample-rate index (23 bounds) */
    __shared__ uint8_t s_slen[32];     /* MPEG-1 slen1 | slen2 per scalefac_compress          */
    /* count1 values with their signs, by (value bits v, the 4 bits after the
     * code): signed bytes [q2, q0, q3, q1], so each 2 x int16 output word is
     * one v_perm_b32 (sign-extension selectors read odd bytes only) */
    __shared__ uint32_t s_c1s[256];
    huff_tables_lane(tab, s_lut, s_tsel, s_lbnd, s_slen);
    static_assert(HUFF_BLOCK >= 256, "s_c1s: one entry per thread");
    if (threadIdx.x < 256) {
        const uint32_t v = threadIdx.x >> 4, s4 = threadIdx.x & 15u;
        int q[4], j = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int bit = (int)(v >> (3 - i)) & 1;
            q[i] = bit && ((s4 >> (3 - j)) & 1u) ? -1 : bit;
            j += bit;
        }
        s_c1s[threadIdx.x] = (uint32_t)(uint8_t)q[2] | (uint32_t)(uint8_t)q[0] << 8 | (uint32_t)(uint8_t)q[3] << 16 |
                             (uint32_t)(uint8_t)q[1] << 24;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t *bits = s_bits + 4 + wv * (HUFF_CAPW + 4);
    const uint32_t qbase = tab->lut_hdr.base[MP3D_LUT_TABLES - 1];
    const int qb1 = tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1];
    /* count1 table B: after the zero table (huff_tables_lane) */
    const uint32_t c1b_base = ((qbase + (1u << qb1) + 1u) & ~1u) + MP3D_C1B_OFF;
    for (;;) {
        uint32_t t = 0u;
        if (lane == 0) t = atomicAdd(work, 1u);
        const int ubase = 64 * (int)__builtin_amdgcn_readfirstlane(t);
        if (ubase >= n_units) break;
        {
            const int u = ubase + lane < n_units ? (int)perm[ubase + lane] : n_units;
            const int fr = u >> 2, gr = (u >> 1) & 1, ch = u & 1;
            bool valid = u < n_units;
            /* the stream's md base, loaded together with the frame record (not
             * after it: one memory latency less per round) */
            const uint64_t mdo = md_off[(valid ? fr : 0) / F];
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
            /* the lane's staged words: for scfsi reuse (need_g0) first a piece
             * of HUFF_G0W words at granule 0's scalefactors (their <= 126 bits
             * from any bit offset, plus the window margin), then the unit's own
             * words [w0, w0 + lenB): through the unit end + 2 words of window
             * margin, rounded to 4 words (16-B LDS stores).  (Staged as one
             * span from granule 0's start, such a unit took granule 0 of both
             * channels too: C3's mean staged unit was 43 words, over the
             * 2 304-word area's 36 per lane of a 64-unit round.) */
            const uint32_t lenA = need_g0 ? HUFF_G0W : 0u;
            const uint32_t w0 = start >> 5;
            /* granule 0's piece, in words before the unit's own (from src) */
            const uint32_t dA = need_g0 ? w0 - (g0_start >> 5) : 0u;
            const uint32_t lenB = dec ? ((((start + p23 + 31) >> 5) + 2 - w0 + 3) & ~3u) : 0u;
            const uint32_t len = lenA + lenB;
            const uint32_t incl = wave_incl_scan(len);
            const uint32_t off = incl - len;
            const uint32_t *src = (const uint32_t *)(md + (dec ? mdo : 0)) + w0;

            bool pending = dec;
            while (__ballot(pending)) {
                const uint32_t base = wave_min(pending ? off : 0xFFFFFFFFu);
                const bool inb = pending && off + len - base <= HUFF_STAGEW;
                wave_sync();
                /* stage: each lane copies its own segment, 4 x 16 B in flight */
                if (inb) {
                    uint32_t *dst = bits + (off - base);
                    for (uint32_t i = 0; i < len; i += 16) {
                        uint4 v[4];
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            const uint32_t q = i + 4 * k; /* (lenA is a multiple of 4: a block is in one piece) */
                            if (q < len) v[k] = *(const uint4 *)(src + (int)(q < lenA ? q - dA : q - lenA));
                        }
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if (i + 4 * k < len)
                                *(uint4 *)(dst + i + 4 * k) =
                                    make_uint4(bswap32(v[k].x), bswap32(v[k].y), bswap32(v[k].z), bswap32(v[k].w));
                    }
                }
                wave_sync();
                if (inb) {
                    const uint32_t seg = 32u * (off - base + lenA) - 32u * w0; /* md bit -> staged bit */
                    uint32_t pos = start + seg;
                    int lsf_pre = 0;
                    if (r.lsf) {
                        /* off the MPEG-1 path: a call keeps its registers out of
                         * the kernel's allocation; bits passed as an LDS pointer */
                        const uint32_t pp = read_sf_lsf((lds_cu32)bits, pos, side, (uint8_t *)&meta[u]);
                        pos = pp & 0x7FFFFFFFu;
                        lsf_pre = (int)(pp >> 31);
                    } else {
                        uint32_t sfw[10];
#pragma unroll
                        for (int i = 0; i < 10; i++) sfw[i] = 0u;
                        if (need_g0) {
                            /* scfsi reuse: granule 0's scalefactors of this channel
                             * first, then granule 1's read over them in place */
                            read_sf(bits, g0_start + seg - 32u * (lenA - dA), sq[ch], 0, sfw, s_slen); /* (its piece) */
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
                    /* big_values pairs in groups of 4 (one 16-B row store per
                     * group, 8 lines; rows are 72 such groups): k is uniform,
                     * the wave runs while any lane has pairs left, and a pair
                     * at or past the lane's big_values, or starting at or past
                     * the part2_3 end (FFmpeg: a truncated unit's remaining
                     * lines read as zeros), stores a zero word and consumes no
                     * bits -- the count1 lines then overwrite the group's tail */
                    int16_t *row = is_buf + (size_t)u * MP3D_IS_ROW;
                    int k = 0;
                    const uint32_t end_bit = start + seg + p23;
                    /* stored two groups at a time: a lane writes 32 B (a whole
                     * sector of its row's line) per store pair, not 16 B per
                     * group -- a line evicted before the lane completes it then
                     * holds only whole sectors (A/B ST32: -2.7 % k_huffman) */
                    uint4 pend = make_uint4(0u, 0u, 0u, 0u);
                    bool held = false;
                    for (; __ballot(k < bv2); k += 8) {
                        uint32_t wv[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const int kk = k + 2 * j;
                            const uint32_t ts = kk < r1 ? ts0 : (kk < r2 ? ts1 : ts2);
                            const uint32_t tb = ts & 0xFFFFu, s1 = (ts >> 16) & 63u, lin = ts >> 24;
                            uint32_t hi, lo;
                            win64g(bits, pos, hi, lo);
                            const uint32_t i1 = tb + (hi >> s1);
                            const uint32_t e1 = s_lut[i1];
                            /* second level, branch-free: i2 = i1 for a leaf */
                            const uint32_t nb = __builtin_amdgcn_ubfe(e1, 11, 4);
                            /* the nb bits after the first level's b1 = 32 - s1: (hi << b1) >> (32 - nb); a
                             * zero-width field (leaf, nb = 0) extracts 0.  The base by v_bfe + v_lshl_add
                             * (as (e1 & 0x7FF) << 2 the compiler spent three ops) */
                            uint32_t b11 = __builtin_amdgcn_ubfe(e1, 0, 11);
                            __asm__("" : "+v"(b11)); /* one v_lshl_add below, not a shift + mask + add */
                            const uint32_t sub = (b11 << 2) + __builtin_amdgcn_ubfe(hi, s1 - nb, nb);
                            const uint32_t i2 = (e1 & 0x8000u) ? sub : i1;
                            const uint32_t e = s_lut[i2];
                            const uint32_t x = (e >> 4) & 15u, y = e & 15u, len_c = (e >> 8) & 31u;
                            const uint32_t sx = (e >> 13) & 1u, sy = (e >> 14) & 1u;
                            /* after the code: [x linbits][x sign][y linbits][y sign],
                             * <= 28 bits, all in the window (code <= 19 bits); a
                             * zero-width field extracts 0 (v_bfe_u32) */
                            /* len_c = 0 only for table 0, whose x = y = 0 need no bits */
                            const uint32_t rb = shl64hi_a(hi, lo, len_c);
                            const uint32_t nx = x == 15u ? lin : 0u, ny = y == 15u ? lin : 0u;
                            /* field offsets counted down from the top of rb */
                            const uint32_t t0 = 32u - nx, t1 = t0 - sx, t2 = t1 - ny, t3 = t2 - sy;
                            const uint32_t ex = __builtin_amdgcn_ubfe(rb, t0, nx);
                            const uint32_t ey = __builtin_amdgcn_ubfe(rb, t2, ny);
                            /* sign bits as 0 / -1 masks (signed 1-bit fields): v = (v ^ m) - m */
                            const int mx = __builtin_amdgcn_sbfe((int)rb, t1, 1u), my = __builtin_amdgcn_sbfe((int)rb, t3, 1u);
                            const bool live = kk < bv2 && pos < end_bit;
                            pos += live ? len_c + (32u - t3) : 0u;
                            /* x = 0 gives X = 0 whatever the (absent) sign bit */
                            const int X = ((int)(x + ex) ^ mx) - mx, Y = ((int)(y + ey) ^ my) - my;
                            /* low halves of X and Y -> one word (v_perm_b32) */
                            wv[j] = live ? __builtin_amdgcn_perm((uint32_t)Y, (uint32_t)X, 0x05040100u) : 0u;
                        }
                        const uint4 cur = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        if (held) { /* (k is uniform: no divergence) */
                            *(uint4 *)(row + k - 8) = pend;
                            *(uint4 *)(row + k) = cur;
                        } else {
                            pend = cur;
                        }
                        held = !held;
                    }
                    if (held) *(uint4 *)(row + k - 8) = pend; /* (before the count1 stores overwrite its tail) */
                    k = bv2;
                    /* count1 quadruples until the part2_3 end; a quadruple that
                     * overreads it is discarded (FFmpeg); lines
                     * k .. k + 3 each, stored in pairs (an unpaired last one by
                     * an 8-B store) */
                    /* table A or B (count1table_select) as one LUT read, no branch */
                    const bool c1b = (side >> 5) & 1;
                    const uint32_t c1base = c1b ? c1b_base : qbase, c1sh = c1b ? 28u : 32u - (uint32_t)qb1;
                    /* (q0, q1) from bytes 1, 3 of se, (q2, q3) from bytes 5, 7 of
                     * se << 8, each sign-extended to 16 bits (selectors 8..11) */
                    auto c1_store = [&](int kq, uint32_t se) {
                        *(uint2 *)(row + kq) = make_uint2(__builtin_amdgcn_perm(se, se, 0x09030801u),
                                                          __builtin_amdgcn_perm(se << 8, se, 0x0B070A05u));
                    };
                    /* one quadruple from the window hw (its code at the top):
                     * its signed values (s_c1s) and bit count.  The signs follow
                     * the code, one per nonzero value in order: the 4 bits after
                     * the code and v index the table. */
                    auto c1_dec = [&](uint32_t hw, uint32_t &se, uint32_t &nb) {
                        const uint32_t e = s_lut[c1base + (hw >> c1sh)];
                        const uint32_t v = e & 15u, lq = (e >> 8) & 31u;
                        nb = lq + __builtin_popcount(v);
                        se = s_c1s[(v << 4) | ((hw << lq) >> 28)];
                    };
                    /* two quadruples per iteration from one 32-bit window (a
                     * quadruple takes <= 10 bits, so the second's code and signs
                     * are in hw << n0) and one 16-B store (4-B aligned: k is
                     * even) -- half the store instructions of the 8-B form, each
                     * touching a line per lane, and half the window reads; a
                     * quadruple that overreads the part2_3 end ends the loop */
                    while (k <= 572 && pos < end_bit) {
                        const uint32_t hw = win32g(bits, pos);
                        uint32_t se0, n0, se1, n1;
                        c1_dec(hw, se0, n0);
                        if (pos + n0 > end_bit) break;
                        pos += n0;
                        bool two = k <= 568 && pos < end_bit;
                        if (two) {
                            c1_dec(hw << n0, se1, n1);
                            two = pos + n1 <= end_bit;
                        }
                        if (!two) {
                            c1_store(k, se0);
                            k += 4;
                            break;
                        }
                        pos += n1;
                        const uint4 q = make_uint4(
                            __builtin_amdgcn_perm(se0, se0, 0x09030801u), __builtin_amdgcn_perm(se0 << 8, se0, 0x0B070A05u),
                            __builtin_amdgcn_perm(se1, se1, 0x09030801u), __builtin_amdgcn_perm(se1 << 8, se1, 0x0B070A05u));
                        __builtin_memcpy(row + k, &q, 16);
                        k += 8;
                    }
                    const int nz_end = k;
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
                int16_t *out = is_buf + (size_t)u * MP3D_IS_ROW;
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

/* k_huffman_wave: one wave per unit (huffman_wave_unit, mp3d_huffman_dev.h) */
__global__ void __launch_bounds__(64 * HW_UNITS) k_huffman_wave(const uint8_t *__restrict__ md,
                                                              const uint64_t *__restrict__ md_off,
                                                              const FrameRec *__restrict__ rec,
                                                              const uint64_t *__restrict__ sideu,
                                                              const DevTables *__restrict__ tab,
                                                              int16_t *__restrict__ is_buf,
                                                              UnitMeta *__restrict__ meta, int n_units, int F) {
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[MP3D_LUT_MAX];
    __shared__ __attribute__((aligned(16))) uint32_t s_bits[HW_UNITS][HW_WORDS + 4];
    __shared__ uint32_t s_tsel[32];
    __shared__ uint16_t s_lbnd[9][24];
    __shared__ uint8_t s_slen[32];
    huff_tables<64 * HW_UNITS>(tab, s_lut, s_tsel, s_lbnd, s_slen, threadIdx.x);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int u = blockIdx.x * HW_UNITS + wv;
    if (u >= n_units) return; /* after the only barrier */
    huffman_wave_unit(md, md_off, rec, sideu, tab, is_buf, meta, F, u, lane, s_bits[wv], s_lut, s_tsel, s_lbnd, s_slen);
}

/* ------------------------------------------------------------------------ */
/* Host-side launchers                                                       */
/* ------------------------------------------------------------------------ */
/* wave: one wave per unit (k_huffman_wave; small batches), else one lane
 * per unit (k_huffman) */
/* work: k_huffman's work-item counter (4 B of device memory per handle);
 * rank: one word per unit (k_rank) */
void launch_huffman(const uint8_t *md, const uint64_t *md_off, const FrameRec *rec, const uint64_t *sideu,
                    const DevTables *tab, int16_t *is_buf, UnitMeta *meta, int n_streams, int F, int n_cu, bool wave,
                    uint32_t *work, uint32_t *rank, hipStream_t strm) {
    int n_units = n_streams * F * 4;
    if (wave) {
        hipLaunchKernelGGL(k_huffman_wave, dim3((n_units + HW_UNITS - 1) / HW_UNITS), dim3(64 * HW_UNITS), 0, strm, md,
                           md_off, rec, sideu, tab, is_buf, meta, n_units, F);
        return;
    }
    /* one workgroup per CU (its LDS is the whole CU's), fewer when there
     * are fewer rounds than waves; the waves take rounds from the counter */
    const int rounds = (n_units + 63) / 64;
    int blocks = (rounds + HUFF_WAVES - 1) / HUFF_WAVES;
    const int cus = n_cu > 0 ? n_cu : 256; /* (device_init's attribute query failed) */
    blocks = blocks < cus ? (blocks > 0 ? blocks : 1) : cus;
    /* the counter restarts at 0 with every launch (a memset node of a few
     * us): a launch that failed can never leave the next one's tickets off */
    (void)hipMemsetAsync(work, 0, sizeof(uint32_t), strm);
    hipLaunchKernelGGL(k_rank, dim3((n_units + RANK_SEG - 1) / RANK_SEG), dim3(RANK_BLOCK), 0, strm, sideu, n_units, rank);
    hipLaunchKernelGGL(k_huffman, dim3(blocks), dim3(HUFF_BLOCK), 0, strm, md, md_off, rec, sideu, tab, is_buf, meta,
                       n_units, F, work, (const uint32_t *)rank);
}

} // namespace mp3d
