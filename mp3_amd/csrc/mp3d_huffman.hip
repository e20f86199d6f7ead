/*
 * mp3d_huffman.hip -- k_huffman (ISO 11172-3
 * 2.4.2.7 + Annex B, 13818-3 2.4.3.2): scalefactors (MPEG-1 scfsi reuse, LSF
 * groups) and the big_values / count1 Huffman decode of every unit into
 * is[576] + UnitMeta.  Pipeline overview: mp3d_device.h.
 */
#include "mp3d_device.h"

namespace mp3d {

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

/* the block's LDS tables: the LUT (+ a 2-entry all-zero table for
 * table_select 0, 4, 14), table_select -> LUT base | bits1 << 16 | linbits
 * << 24, long sfb start lines per sample-rate index, MPEG-1 slen pairs */
__device__ __forceinline__ void huff_tables(const DevTables *tab, uint16_t *s_lut, uint32_t *s_tsel,
                                            uint16_t (*s_lbnd)[24], uint8_t *s_slen) {
    const int lut_n = tab->lut_hdr.base[MP3D_LUT_TABLES - 1] + (1 << tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1]);
    const int zbase = (lut_n + 1) & ~1;
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
}

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
    huff_tables(tab, s_lut, s_tsel, s_lbnd, s_slen);
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
            const uint32_t *src = (const uint32_t *)(md + (dec ? mdo : 0)) + w0;

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
                    /* big_values pairs in groups of 4 (one 16-B row store per
                     * group, 8 lines; rows are 72 such groups): k is uniform,
                     * the wave runs while any lane has pairs left, and a pair
                     * at or past the lane's big_values, or starting at or past
                     * the part2_3 end (FFmpeg: a truncated unit's remaining
                     * lines read as zeros), stores a zero word and consumes no
                     * bits -- the count1 lines then overwrite the group's tail */
                    int16_t *row = is_buf + (size_t)u * 576;
                    int k = 0;
                    const uint32_t end_bit = start + seg + p23;
                    for (; __ballot(k < bv2); k += 8) {
                        uint32_t wv[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const int kk = k + 2 * j;
                            const uint32_t ts = kk < r1 ? ts0 : (kk < r2 ? ts1 : ts2);
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
                            const uint32_t sx = (e >> 13) & 1u, sy = (e >> 14) & 1u;
                            /* after the code: [x linbits][x sign][y linbits][y sign],
                             * <= 28 bits, all in the window (code <= 19 bits); a
                             * zero-width field extracts 0 (v_bfe_u32) */
                            const uint32_t rb = shl64hi(hi, lo, len_c);
                            const uint32_t nx = x == 15u ? lin : 0u, ny = y == 15u ? lin : 0u;
                            const uint32_t ex = __builtin_amdgcn_ubfe(rb, 32u - nx, nx);
                            const uint32_t q1 = nx + sx;
                            const uint32_t sgx = __builtin_amdgcn_ubfe(rb, 32u - q1, 1u);
                            const uint32_t ey = __builtin_amdgcn_ubfe(rb, 32u - q1 - ny, ny);
                            const uint32_t q2 = q1 + ny + sy;
                            const uint32_t sgy = __builtin_amdgcn_ubfe(rb, 32u - q2, 1u);
                            const bool live = kk < bv2 && pos < end_bit;
                            pos += live ? len_c + q2 : 0u;
                            /* x = 0 gives X = 0 whatever the (absent) sign bit */
                            int X = (int)(x + ex), Y = (int)(y + ey);
                            X = sgx ? -X : X;
                            Y = sgy ? -Y : Y;
                            wv[j] = live ? (uint32_t)(uint16_t)X | ((uint32_t)(uint16_t)Y << 16) : 0u;
                        }
                        *(uint4 *)(row + k) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                    }
                    k = bv2;
                    /* count1 quadruples until the part2_3 end; a quadruple that
                     * overreads it is discarded (FFmpeg); one
                     * 8-B store each (lines k .. k + 3) */
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
                        *(uint2 *)(row + k) = make_uint2((uint32_t)(uint16_t)q0 | ((uint32_t)(uint16_t)q1 << 16),
                                                         (uint32_t)(uint16_t)q2 | ((uint32_t)(uint16_t)q3 << 16));
                        k += 4;
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

/* ------------------------------------------------------------------------ */
/* k_huffman_wave: one WAVE per unit, for small batches (the per-frame      */
/* decoder), where one unit's codeword chain is the whole critical path.     */
/* Each round, lane L decodes the pair (or count1 quadruple) that would      */
/* start at bit pos + L with the region's table; the real chain then hops    */
/* through those speculative decodes by cross-lane reads (next start = this */
/* start + this length): a few scalar steps per codeword instead of three   */
/* dependent LDS reads.  A round ends at a region boundary, at the part2_3  */
/* end, or where the next codeword starts past offset 63.  The decoded words */
/* collect one per lane of an accumulator and store 256 B at a time.  Same  */
/* results as k_huffman (FFmpeg: pairs at or past the part2_3 end are zeros; */
/* a quadruple that overreads it is discarded).                             */
/* ------------------------------------------------------------------------ */
#define HW_UNITS 4
#define HW_WORDS 520 /* staged md words per unit: four 4095-bit units + margin */

__device__ __forceinline__ void hw_win64(const uint32_t *bits, uint32_t pos, uint32_t &hi, uint32_t &lo) {
    uint32_t w = pos >> 5;
    w = w < HW_WORDS ? w : HW_WORDS;
    const uint32_t sh = 32u - (pos & 31u);
    const uint32_t w0 = bits[w], w1 = bits[w + 1], w2 = bits[w + 2];
    hi = (uint32_t)((((uint64_t)w0 << 32) | w1) >> sh);
    lo = (uint32_t)((((uint64_t)w1 << 32) | w2) >> sh);
}

/* one big_values pair at bit p with table word ts (the k_huffman pair decode):
 * total bits and the packed (x, y) word */
__device__ __forceinline__ void hw_pair(const uint16_t *s_lut, const uint32_t *bits, uint32_t p, uint32_t ts,
                                        uint32_t &tl, uint32_t &word) {
    const uint32_t tb = ts & 0xFFFFu, b1 = (ts >> 16) & 15u, lin = ts >> 24;
    uint32_t hi, lo;
    hw_win64(bits, p, hi, lo);
    const uint32_t i1 = tb + (hi >> (32 - b1));
    const uint32_t e1 = s_lut[i1];
    const uint32_t nb = (e1 >> 11) & 15u;
    const uint32_t sub = ((e1 & 0x7FFu) << 2) + (uint32_t)((((uint64_t)hi << b1) & 0xFFFFFFFFull) >> (32u - nb));
    const uint32_t e = s_lut[(e1 & 0x8000u) ? sub : i1];
    const uint32_t x = (e >> 4) & 15u, y = e & 15u, len_c = (e >> 8) & 31u;
    const uint32_t sx = (e >> 13) & 1u, sy = (e >> 14) & 1u;
    const uint32_t rb = shl64hi(hi, lo, len_c);
    const uint32_t nx = x == 15u ? lin : 0u, ny = y == 15u ? lin : 0u;
    const uint32_t ex = __builtin_amdgcn_ubfe(rb, 32u - nx, nx);
    const uint32_t q1 = nx + sx;
    const uint32_t sgx = __builtin_amdgcn_ubfe(rb, 32u - q1, 1u);
    const uint32_t ey = __builtin_amdgcn_ubfe(rb, 32u - q1 - ny, ny);
    const uint32_t q2 = q1 + ny + sy;
    const uint32_t sgy = __builtin_amdgcn_ubfe(rb, 32u - q2, 1u);
    int X = (int)(x + ex), Y = (int)(y + ey);
    X = sgx ? -X : X;
    Y = sgy ? -Y : Y;
    tl = len_c + q2;
    word = (uint32_t)(uint16_t)X | ((uint32_t)(uint16_t)Y << 16);
}

struct HwOut { /* the unit's is[] row, one word per lane of acc, 64 words per store */
    uint32_t *row;
    uint32_t acc;
    int nw;
    int lane;
    __device__ __forceinline__ void emit(uint32_t w) { /* w uniform */
        acc = lane == (nw & 63) ? w : acc;
        nw++;
        if ((nw & 63) == 0) row[nw - 64 + lane] = acc;
    }
    __device__ __forceinline__ void flush() {
        if ((nw & 63) && lane < (nw & 63)) row[(nw & ~63) + lane] = acc;
    }
};

__global__ void __launch_bounds__(64 * HW_UNITS) k_huffman_wave(const uint8_t *__restrict__ md,
                                                              const uint64_t *__restrict__ md_off,
                                                              const FrameRec *__restrict__ rec,
                                                              const uint64_t *__restrict__ sideu,
                                                              const DevTables *__restrict__ tab,
                                                              int16_t *__restrict__ is_buf,
                                                              UnitMeta *__restrict__ meta, int n_units, int F) {
    __shared__ uint16_t s_lut[MP3D_LUT_MAX];
    __shared__ __attribute__((aligned(16))) uint32_t s_bits[HW_UNITS][HW_WORDS + 4];
    __shared__ uint32_t s_tsel[32];
    __shared__ uint16_t s_lbnd[9][24];
    __shared__ uint8_t s_slen[32];
    huff_tables(tab, s_lut, s_tsel, s_lbnd, s_slen);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int u = blockIdx.x * HW_UNITS + wv;
    if (u >= n_units) return; /* after the only barrier */
    uint32_t *bits = s_bits[wv];
    const uint32_t qbase = tab->lut_hdr.base[MP3D_LUT_TABLES - 1];
    const int qb1 = tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1];
    const int fr = u >> 2, gr = (u >> 1) & 1, ch = u & 1;
    const FrameRec r = rec[fr];
    const bool valid = r.frame_bytes && !(r.first_gr & (REC_TAG | REC_DROP)) && ch < r.nch && (gr == 0 || !r.lsf);
    if (!valid) return;
    uint64_t sq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) sq[q] = sideu[(u & ~3) + q];
    const int first_gr = r.first_gr & 3;
    const int nch = r.nch;
    const bool dec = gr >= first_gr;
    const int q = u & 3;
    const uint64_t side = sq[q];
    if (!dec) {
        /* granule lost to a reservoir underflow: silence (FFmpeg) */
        uint4 *out = (uint4 *)(is_buf + (size_t)u * 576);
        for (int i = lane; i < 72; i += 64) out[i] = make_uint4(0u, 0u, 0u, 0u);
        if (lane == 0) {
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
        return;
    }
    const uint32_t p23 = (uint32_t)(side >> 52);
    uint32_t before = 0;
#pragma unroll
    for (int qq = 0; qq < 3; qq++)
        if (qq < q && (qq >> 1) >= first_gr && (qq & 1) < nch) before += (uint32_t)(sq[qq] >> 52);
    const uint32_t start = r.md_bit + before;
    const int scfsi_raw = (int)(side >> 1) & 15;
    const bool long_blk = !(((side >> 30) & 1) && ((side >> 28) & 3) == 2);
    const int scfsi = (gr == 1 && long_blk) ? scfsi_raw : 0;
    const bool need_g0 = scfsi && first_gr == 0;
    const uint32_t g0_start = r.md_bit + (ch ? (uint32_t)(sq[0] >> 52) : 0u);
    const uint32_t lo_bit = need_g0 ? g0_start : start;
    const uint32_t w0 = lo_bit >> 5;
    uint32_t len = ((start + p23 + 31) >> 5) + 4 - w0;
    len = len < HW_WORDS ? len : HW_WORDS;
    const uint32_t *src = (const uint32_t *)(md + md_off[fr / F]) + w0;
    for (uint32_t i = lane; i < len; i += 64) bits[i] = bswap32(src[i]);
    wave_sync();
    const uint32_t seg = 0u - 32u * w0; /* md bit -> staged bit */
    uint32_t pos = start + seg;
    int lsf_pre = 0;
    if (r.lsf) {
        uint32_t p0 = 0;
        if (lane == 0) p0 = read_sf_lsf((lds_cu32)bits, pos, side, (uint8_t *)&meta[u], &lsf_pre);
        pos = (uint32_t)__builtin_amdgcn_readlane((int)p0, 0);
        lsf_pre = __builtin_amdgcn_readlane(lsf_pre, 0);
    } else {
        uint32_t sfw[10];
#pragma unroll
        for (int i = 0; i < 10; i++) sfw[i] = 0u;
        if (need_g0) read_sf(bits, g0_start + seg, sq[ch], 0, sfw, s_slen);
        pos = read_sf(bits, pos, side, scfsi, sfw, s_slen);
        if (lane == 0) {
            uint8_t *mrec = (uint8_t *)&meta[u];
            *(uint4 *)mrec = make_uint4(sfw[0], sfw[1], sfw[2], sfw[3]);
            *(uint4 *)(mrec + 16) = make_uint4(sfw[4], sfw[5], sfw[6], sfw[7]);
            *(uint2 *)(mrec + 32) = make_uint2(sfw[8], sfw[9]);
        }
    }
    const int ws = (int)(side >> 30) & 1;
    const int bv2 = 2 * ((int)(side >> 43) & 0x1FF);
    int r1, r2;
    uint32_t ts0, ts1, ts2;
    if (ws) {
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
    /* all of these are wave-uniform; said so, so that the chain loop runs on
     * scalar registers (LDS-derived values otherwise stay per lane) */
    r1 = __builtin_amdgcn_readfirstlane(r1);
    r2 = __builtin_amdgcn_readfirstlane(r2);
    ts0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ts0);
    ts1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ts1);
    ts2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ts2);
    pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)pos);
    HwOut out;
    out.row = (uint32_t *)(is_buf + (size_t)u * 576);
    out.acc = 0u;
    out.nw = 0;
    out.lane = lane;
    const uint32_t end_bit = start + seg + p23;
    int k = 0;
    while (k < bv2) {
        if (pos >= end_bit) { /* the rest of big_values reads as zeros */
            for (; k < bv2; k += 2) out.emit(0u);
            break;
        }
        const uint32_t ts = k < r1 ? ts0 : (k < r2 ? ts1 : ts2);
        const int kend = k < r1 ? r1 : (k < r2 ? r2 : bv2);
        /* two speculative decodes per lane (offsets lane, 64 + lane; their
         * latencies overlap): a round follows the chain over 128 bits */
        uint32_t tl0, wd0, tl1, wd1;
        hw_pair(s_lut, bits, pos + (uint32_t)lane, ts, tl0, wd0);
        hw_pair(s_lut, bits, pos + 64u + (uint32_t)lane, ts, tl1, wd1);
        uint32_t o = 0;
        do {
            const bool lo = o < 64u;
            const int ol = (int)(o & 63u);
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? wd0 : wd1), ol);
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)(lo ? tl0 : tl1), ol);
            out.emit(w);
            o += t;
            k += 2;
        } while (k < kend && o < 128u && pos + o < end_bit);
        pos += o;
    }
    const bool c1b = (side >> 5) & 1;
    while (k <= 572 && pos < end_bit) {
        const uint32_t p = pos + (uint32_t)lane;
        uint32_t w = p >> 5;
        w = w < HW_WORDS ? w : HW_WORDS;
        const uint32_t hw = (uint32_t)((((uint64_t)bits[w] << 32) | bits[w + 1]) >> (32u - (p & 31u)));
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
        const uint32_t sbits = (hw << lq) >> (32 - (ns ? ns : 1));
        int bit = (int)ns;
        int q0 = (v >> 3) & 1, q1 = (v >> 2) & 1, q2 = (v >> 1) & 1, q3 = v & 1;
        if (q0) { bit--; if ((sbits >> bit) & 1) q0 = -1; }
        if (q1) { bit--; if ((sbits >> bit) & 1) q1 = -1; }
        if (q2) { bit--; if ((sbits >> bit) & 1) q2 = -1; }
        if (q3) { bit--; if ((sbits >> bit) & 1) q3 = -1; }
        const uint32_t tq = lq + ns;
        const uint32_t wa = (uint32_t)(uint16_t)q0 | ((uint32_t)(uint16_t)q1 << 16);
        const uint32_t wb = (uint32_t)(uint16_t)q2 | ((uint32_t)(uint16_t)q3 << 16);
        uint32_t o = 0;
        bool over = false;
        do {
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tq, (int)o);
            if (pos + o + t > end_bit) {
                over = true;
                break;
            }
            out.emit((uint32_t)__builtin_amdgcn_readlane((int)wa, (int)o));
            out.emit((uint32_t)__builtin_amdgcn_readlane((int)wb, (int)o));
            o += t;
            k += 4;
        } while (k <= 572 && o < 64u && pos + o < end_bit);
        pos += o;
        if (over) break;
    }
    out.flush();
    if (lane == 0) {
        UnitMeta m;
        m.global_gain = (uint8_t)(side >> 35);
        m.block_type = (uint8_t)(ws ? (side >> 28) & 3 : 0);
        m.mixed = (uint8_t)(ws && ((side >> 28) & 3) == 2 ? (side >> 27) & 1 : 0);
        m.scalefac_scale = (uint8_t)((side >> 6) & 1);
        m.preflag = (uint8_t)(r.lsf ? lsf_pre : (int)((side >> 7) & 1));
        m.sbg[0] = (uint8_t)(ws ? (side >> 14) & 7 : 0);
        m.sbg[1] = (uint8_t)(ws ? (side >> 11) & 7 : 0);
        m.sbg[2] = (uint8_t)(ws ? (side >> 8) & 7 : 0);
        m.nz_end = (uint16_t)(2 * out.nw);
        m.part2_3_length = (uint16_t)p23;
        m.used_bits = (uint16_t)(pos - start - seg);
        m.flags = (uint16_t)(r.lsf ? ((side >> 31) & 1) << 1 : 0);
        *(uint4 *)((uint8_t *)&meta[u] + 40) = *(const uint4 *)((const uint8_t *)&m + 40);
    }
}

/* ------------------------------------------------------------------------ */
/* Host-side launchers                                                       */
/* ------------------------------------------------------------------------ */
/* wave: one wave per unit (k_huffman_wave; small batches), else one lane
 * per unit (k_huffman) */
void launch_huffman(const uint8_t *md, const uint64_t *md_off, const FrameRec *rec, const uint64_t *sideu,
                    const DevTables *tab, int16_t *is_buf, UnitMeta *meta, int n_streams, int F, int n_cu, bool wave,
                    hipStream_t strm) {
    int n_units = n_streams * F * 4;
    int supers = (n_units + HUFF_SUPER - 1) / HUFF_SUPER;
    /* one super-chunk per wave, no grid-stride: the hardware hands out
     * blocks as CUs free up, so uneven super-chunks balance themselves */
    int blocks = (supers + HUFF_WAVES - 1) / HUFF_WAVES;
    (void)n_cu;
    if (wave) {
        hipLaunchKernelGGL(k_huffman_wave, dim3((n_units + HW_UNITS - 1) / HW_UNITS), dim3(64 * HW_UNITS), 0, strm, md,
                           md_off, rec, sideu, tab, is_buf, meta, n_units, F);
        return;
    }
    hipLaunchKernelGGL(k_huffman, dim3(blocks), dim3(HUFF_BLOCK), 0, strm, md, md_off, rec, sideu, tab, is_buf, meta,
                       n_units, F);
}

} // namespace mp3d
