/*
 * mp3d_huffman_dev.h -- device side of the Huffman stage (SURVEY.md §8(a)
 * rows a4, a5; ISO 11172-3 2.4.2.7 + Annex B, 13818-3 2.4.3.2): LDS bit
 * windows, scalefactors (MPEG-1 scfsi reuse, LSF groups), the block's LDS
 * tables and the one-wave-per-unit decode.  Included by mp3d_huffman.hip
 * (k_huffman, k_huffman_wave) and by mp3d_synth.hip (the fused per-frame
 * kernel k_frame).
 */
#ifndef MP3D_HUFFMAN_DEV_H
#define MP3D_HUFFMAN_DEV_H
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
/* One 16-wave workgroup per CU (4 waves per SIMD at <= 128 VGPRs), sharing
 * one copy of the LUT; the waves take 64-unit rounds of the launch's
 * big_values order from a work counter (persistent).  4-wave workgroups held
 * 3 LUT copies per CU and fit only 3 waves per SIMD beside the staging
 * areas. */
#define HUFF_WAVES 16
#define MP3D_C1B_OFF 2 /* count1 table B after the zero table (huff_tables_lane) */
#define HUFF_BLOCK (64 * HUFF_WAVES)
#define HUFF_CAPW 2304 /* LDS words per wave (9.2 KB) of main-data staging; 16 waves + the tables in 160 KB */
#define HUFF_STAGEW HUFF_CAPW /* staging words */
#define HUFF_G0W 8u /* words staged at granule 0's scalefactors for scfsi reuse (<= 31 + 126 bits + the window margin) */

/* wave-wide scan / min by ds_bpermute with the lane id re-derived at each
 * use (HIP's __shfl_up / __shfl_xor add width bounds whose lane-derived
 * constants the compiler held across the super-chunk loop and spilled at
 * 128 VGPRs; a spill reload's vmcnt(0) then waited for the row stores) */
__device__ __forceinline__ int lane_now() {
    int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    __asm__ volatile("" : "+v"(l));
    return l;
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_now();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__builtin_amdgcn_ds_bpermute((l - o) << 2, (int)v);
        if (l >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    const int l = lane_now();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = min(v, (uint32_t)__builtin_amdgcn_ds_bpermute((l ^ o) << 2, (int)v));
    return v;
}

/* 32 bits of a staged (big-endian word) bitstream starting at bit pos (the
 * scalefactor readers; a 64-bit funnel shift, so sh = 0 needs no case) */
__device__ __forceinline__ uint32_t win32(const uint32_t *bits, uint32_t pos) {
    uint32_t w = pos >> 5;
    w = w < HUFF_CAPW ? w : HUFF_CAPW;
    const uint32_t w0 = bits[w], w1 = bits[w + 1];
    return (uint32_t)((((uint64_t)w0 << 32) | w1) >> (32u - (pos & 31u)));
}
/* win64 / win32 by 32-bit funnel shifts (v_alignbit_b32, shift = -pos mod
 * 32): the word pair is picked from pos + 31, so a shift of 0 (pos a
 * multiple of 32) selects the pair's second word.  Reads one word BELOW
 * pos / 32 in that case (its value is not used): bits[-1] must be
 * readable LDS (k_huffman's staging areas have a guard word). */
/* No index clamp: k_huffman reads only while pos is inside the lane's staged
 * segment (pos <= the unit end + 47 bits < its 2-word margin). */
__device__ __forceinline__ void win64g(const uint32_t *bits, uint32_t pos, uint32_t &hi, uint32_t &lo) {
    /* (the barrier keeps the word index whole, so its byte address is one
     * v_lshl_add; combined, the compiler spent a shift, a mask and an add) */
    uint32_t w = (pos + 31u) >> 5;
    __asm__("" : "+v"(w));
    const uint32_t w0 = bits[(int)w - 1], w1 = bits[w], w2 = bits[w + 1];
    hi = __builtin_amdgcn_alignbit(w0, w1, 0u - pos);
    lo = __builtin_amdgcn_alignbit(w1, w2, 0u - pos);
}
__device__ __forceinline__ uint32_t win32g(const uint32_t *bits, uint32_t pos) {
    const uint32_t w = (pos + 31u) >> 5;
    return __builtin_amdgcn_alignbit(bits[(int)w - 1], bits[w], 0u - pos);
}
/* top 32 bits of (hi:lo) << n for 1 <= n <= 32 (n = 0 gives lo, not hi) */
__device__ __forceinline__ uint32_t shl64hi_a(uint32_t hi, uint32_t lo, uint32_t n) {
    return __builtin_amdgcn_alignbit(hi, lo, 32u - n);
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
__device__ __forceinline__ uint32_t read_sf_lsf_i(lds_cu32 bits, uint32_t pos, uint64_t side, uint8_t *sf,
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
/* k_huffman's call: out of line, so its registers stay out of the kernel's
 * allocation (the one-wave-per-unit decode inlines read_sf_lsf_i: no call,
 * no stack).  Returns pos | preflag << 31 (pos < 2^31): a preflag returned
 * through a pointer lived in scratch, and reloading it at the UnitMeta store
 * waited for vmcnt(0) -- for every is[] row store of the round. */
__device__ __attribute__((noinline)) uint32_t read_sf_lsf(lds_cu32 bits, uint32_t pos, uint64_t side, uint8_t *sf) {
    int pre;
    const uint32_t p = read_sf_lsf_i(bits, pos, side, sf, &pre);
    return p | (uint32_t)pre << 31;
}

/* the block's LDS tables: the LUT (the whole array: past the last table it
 * holds the zero table of table_select 0, 4, 14), table_select -> LUT base |
 * bits1 << 16 | linbits << 24, long sfb start lines per sample-rate index,
 * MPEG-1 slen pairs.  Every load is independent (one memory latency): the
 * per-frame path's kernels wait on it. */
template <int NT>
__device__ __forceinline__ void huff_tables(const DevTables *tab, uint16_t *s_lut, uint32_t *s_tsel,
                                            uint16_t (*s_lbnd)[24], uint8_t *s_slen, int t) {
    /* NT threads (t = 0 .. NT - 1); the LUT in uint4 chunks, the index clamped
     * instead of guarded so every load is issued before the first store
     * (the last chunk is written by several lanes, with the same value) */
    constexpr int LUT4 = MP3D_LUT_MAX / 8;
    static_assert(NT >= 9 * 24 / 2, "huff_tables: one word of lbnd per thread");
    const uint4 *src = (const uint4 *)tab->lut;
    uint4 *dst = (uint4 *)s_lut;
#pragma unroll
    for (int j = 0; j < (LUT4 + NT - 1) / NT; j++) {
        const int i = min(t + NT * j, LUT4 - 1);
        dst[i] = src[i];
    }
    if (t < 32) s_tsel[t] = tab->tsel[t];
    if (t < 9 * 24 / 2) ((uint32_t *)s_lbnd)[t] = ((const uint32_t *)tab->lbnd)[t];
    if (t < 32) s_slen[t] = MP3D_SLEN[t >> 4][t & 15];
}

/* k_huffman's staging of the same tables, computed in the block from the
 * LUT header (two loads deep; latency does not matter there, and the
 * one-deep version above measured +0.8 % k_huffman on C3: A/B HTOLD,
 * profiles/r02_ab.txt).  Its zero-table selects lack the bit-20 flag,
 * which only k_huffman_wave reads. */
__device__ __forceinline__ void huff_tables_lane(const DevTables *tab, uint16_t *s_lut, uint32_t *s_tsel,
                                            uint16_t (*s_lbnd)[24], uint8_t *s_slen) {
    const int lut_n = tab->lut_hdr.base[MP3D_LUT_TABLES - 1] + (1 << tab->lut_hdr.bits1[MP3D_LUT_TABLES - 1]);
    const int zbase = (lut_n + 1) & ~1;
    for (int i = threadIdx.x; i < (lut_n + 1) / 2; i += blockDim.x)
        ((uint32_t *)s_lut)[i] = ((const uint32_t *)tab->lut)[i];
    if (threadIdx.x == 0) ((uint32_t *)s_lut)[zbase / 2] = 0u;
    /* count1 table B (4-bit codes, value = 15 - code) as a 16-entry table at
     * zbase + 2 (MP3D_C1B_OFF), so both count1 tables are one LUT read */
    if (threadIdx.x < 16) s_lut[zbase + MP3D_C1B_OFF + threadIdx.x] = (uint16_t)((4u << 8) | (15u - threadIdx.x));
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
        /* k_huffman's encoding: 32 - bits1 (the first level's shift) in bits 16..21 */
        s_tsel[threadIdx.x] = t < 0 ? (uint32_t)zbase | (31u << 16)
                                    : (uint32_t)tab->lut_hdr.base[t] | ((32u - tab->lut_hdr.bits1[t]) << 16) |
                                          ((uint32_t)MP3D_LINBITS[threadIdx.x] << 24);
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

/* m with bit i set (i < 64, wave-uniform): one scalar instruction */
__device__ __forceinline__ uint64_t set_bit64(uint64_t m, uint32_t i) {
    __asm__("s_bitset1_b64 %0, %1" : "+s"(m) : "s"(i));
    return m;
}

/* position of the set bit of rank k (k < popcount(m)) of a wave-uniform mask */
__device__ __forceinline__ uint32_t kth_bit(uint64_t m, int k, int lane) {
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const bool sel = ((m >> lane) & 1u) && r == (uint32_t)k;
    return (uint32_t)__builtin_ctzll(__ballot(sel));
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
    /* (hi << b1) >> (32 - nb) as one field extract (nb = 0 for a leaf: 0) */
    const uint32_t sub = ((e1 & 0x7FFu) << 2) + __builtin_amdgcn_ubfe(hi, 32u - b1 - nb, nb);
    const uint32_t e = s_lut[(e1 & 0x8000u) ? sub : i1];
    const uint32_t x = (e >> 4) & 15u, y = e & 15u, len_c = (e >> 8) & 31u;
    const uint32_t sx = (e >> 13) & 1u, sy = (e >> 14) & 1u;
    const uint32_t rb = shl64hi_a(hi, lo, len_c); /* len_c = 0: table 0, no bits read */
    const uint32_t nx = x == 15u ? lin : 0u, ny = y == 15u ? lin : 0u;
    /* fields counted down from the top of rb; signs as 0 / -1 masks */
    const uint32_t t0 = 32u - nx, t1 = t0 - sx, t2 = t1 - ny, t3 = t2 - sy;
    const uint32_t ex = __builtin_amdgcn_ubfe(rb, t0, nx), ey = __builtin_amdgcn_ubfe(rb, t2, ny);
    const int mx = __builtin_amdgcn_sbfe((int)rb, t1, 1u), my = __builtin_amdgcn_sbfe((int)rb, t3, 1u);
    const int X = ((int)(x + ex) ^ mx) - mx, Y = ((int)(y + ey) ^ my) - my;
    tl = len_c + (32u - t3);
    word = __builtin_amdgcn_perm((uint32_t)Y, (uint32_t)X, 0x05040100u);
}


/* one unit's decode by one wave (k_huffman_wave; also the per-frame
 * k_frame's second phase): unit u, lane 0..63 of the calling wave, bits =
 * the wave's md staging words, the block's LDS tables from huff_tables.
 * No workgroup barrier inside. */
__device__ __forceinline__ void huffman_wave_unit(const uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off,
                                                  const FrameRec *__restrict__ rec, const uint64_t *__restrict__ sideu,
                                                  const DevTables *__restrict__ tab, int16_t *__restrict__ is_buf,
                                                  UnitMeta *__restrict__ meta, int F, int u, int lane, uint32_t *bits,
                                                  const uint16_t *s_lut, const uint32_t *s_tsel,
                                                  const uint16_t (*s_lbnd)[24], const uint8_t *s_slen) {
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
        uint4 *out = (uint4 *)(is_buf + (size_t)u * MP3D_IS_ROW);
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
        if (lane == 0) p0 = read_sf_lsf_i((lds_cu32)bits, pos, side, (uint8_t *)&meta[u], &lsf_pre);
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
    /* the unit's is[] row as words (line pairs), nw written so far */
    uint32_t *row = (uint32_t *)(is_buf + (size_t)u * MP3D_IS_ROW);
    int nw = 0;
    const uint32_t end_bit = (uint32_t)__builtin_amdgcn_readfirstlane((int)(start + seg + p23));
    const int bvu = __builtin_amdgcn_readfirstlane(bv2);
    int k = 0;
    while (k < bvu) {
        const uint32_t ts = k < r1 ? ts0 : (k < r2 ? ts1 : ts2);
        const int kend = k < r1 ? r1 : (k < r2 ? r2 : bvu);
        if (pos >= end_bit || ((ts >> 20) & 1u)) {
            /* past the part2_3 end the rest of big_values reads as zeros;
             * the zero table (table_select 0, 4, 14) codes zeros in no
             * bits: either way the lines are stored as zeros */
            const int kz = pos >= end_bit ? bvu : kend;
            for (int i = lane; i < (kz - k) / 2; i += 64) row[nw + i] = 0u;
            nw += (kz - k) / 2;
            k = kz;
            continue;
        }
        /* two speculative decodes per lane (offsets lane, 64 + lane; their
         * latencies overlap): the chain over these 128 starts runs on scalar
         * registers -- one cross-lane read per codeword, which marks the
         * codeword's start in a 128-bit mask; the marked lanes then store
         * their words in chain order (start order) */
        uint32_t tl0, wd0, tl1, wd1;
        hw_pair(s_lut, bits, pos + (uint32_t)lane, ts, tl0, wd0);
        hw_pair(s_lut, bits, pos + 64u + (uint32_t)lane, ts, tl1, wd1);
        /* a pair starts before the part2_3 end; at most 128 bits a round */
        const uint32_t lim = end_bit - pos < 128u ? end_bit - pos : 128u;
        /* the hop loops test only the bit position (5 scalar-side
         * instructions a codeword); a region ending inside the round is cut
         * afterwards: its first `left` codewords stay, and the next one
         * starts at the start mark of rank `left` */
        const uint32_t lim0 = lim < 64u ? lim : 64u;
        uint64_t m0 = 0, m1 = 0;
        uint32_t o = 0;
        do {
            m0 = set_bit64(m0, o);
            o += (uint32_t)__builtin_amdgcn_readlane((int)tl0, (int)o);
        } while (o < lim0);
        if (o < lim) {
            do {
                m1 = set_bit64(m1, o & 63u);
                o += (uint32_t)__builtin_amdgcn_readlane((int)tl1, (int)(o & 63u));
            } while (o < lim);
        }
        const int left = (kend - k) / 2;
        if (__builtin_popcountll(m0) + __builtin_popcountll(m1) > left) {
            const int c0 = __builtin_popcountll(m0);
            if (left < c0) {
                o = kth_bit(m0, left, lane);
                m0 &= (1ull << o) - 1ull;
                m1 = 0;
            } else {
                const uint32_t b = kth_bit(m1, left - c0, lane);
                m1 &= (1ull << b) - 1ull;
                o = 64u + b;
            }
        }
        const uint32_t r0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
        const uint32_t rk1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
        const int n0 = __builtin_popcountll(m0), n1 = __builtin_popcountll(m1);
        if ((m0 >> lane) & 1u) row[nw + (int)r0] = wd0;
        if ((m1 >> lane) & 1u) row[nw + n0 + (int)rk1] = wd1;
        nw += n0 + n1;
        k += 2 * (n0 + n1);
        pos += o;
    }
    /* count1 quadruples until the part2_3 end (one per 2 words); a quadruple
     * that overreads it is discarded (FFmpeg) */
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
        /* sign bits by prefix counts of v (k_huffman's count1 decode) */
        const uint32_t rb = hw << lq;
        const uint32_t p1 = v >> 3, p2 = __builtin_popcount(v >> 2), p3 = __builtin_popcount(v >> 1);
        const int m0 = __builtin_amdgcn_sbfe((int)rb, 31u, 1u), m1 = __builtin_amdgcn_sbfe((int)rb, 31u - p1, 1u);
        const int m2 = __builtin_amdgcn_sbfe((int)rb, 31u - p2, 1u), m3 = __builtin_amdgcn_sbfe((int)rb, 31u - p3, 1u);
        const int q0 = ((int)p1 ^ m0) - m0, q1 = ((int)((v >> 2) & 1u) ^ m1) - m1;
        const int q2 = ((int)((v >> 1) & 1u) ^ m2) - m2, q3 = ((int)(v & 1u) ^ m3) - m3;
        const uint32_t tq = lq + ns;
        const uint32_t wa = __builtin_amdgcn_perm((uint32_t)q1, (uint32_t)q0, 0x05040100u);
        const uint32_t wb = __builtin_amdgcn_perm((uint32_t)q3, (uint32_t)q2, 0x05040100u);
        /* a quadruple ends at or before the part2_3 end */
        const uint32_t lim = end_bit - pos;
        const uint32_t lim0 = lim < 64u ? lim : 64u;
        uint64_t m = 0;
        uint32_t o = 0;
        bool over = false;
        do {
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tq, (int)o);
            if (o + t > lim) {
                over = true;
                break;
            }
            m = set_bit64(m, o);
            o += t;
        } while (o < lim0);
        /* quadruples only up to line 575 (k <= 572): cut as above */
        const int left = (572 - k) / 4 + 1;
        if (__builtin_popcountll(m) > left) {
            o = kth_bit(m, left, lane);
            m &= (1ull << o) - 1ull;
            over = false;
        }
        const uint32_t rq = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const int nq = __builtin_popcountll(m);
        if ((m >> lane) & 1u) *(uint2 *)(row + nw + 2 * (int)rq) = make_uint2(wa, wb);
        nw += 2 * nq;
        k += 4 * nq;
        pos += o;
        if (over) break;
    }
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
        m.nz_end = (uint16_t)(2 * nw);
        m.part2_3_length = (uint16_t)p23;
        m.used_bits = (uint16_t)(pos - start - seg);
        m.flags = (uint16_t)(r.lsf ? ((side >> 31) & 1) << 1 : 0);
        *(uint4 *)((uint8_t *)&meta[u] + 40) = *(const uint4 *)((const uint8_t *)&m + 40);
    }
}

} // namespace mp3d
#endif
