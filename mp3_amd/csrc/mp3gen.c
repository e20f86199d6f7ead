/*
 * mp3gen.c -- seeded synthetic MPEG-1 / MPEG-2 / MPEG-2.5 Layer III stream
 * generator.
 *
 * Produces VALID bitstreams (header, side info, bit reservoir, scalefactors,
 * Huffman big_values / count1 regions) from seeded random quantised spectra,
 * so the integer stage has ground truth by construction (the is[] values and
 * scalefactors it encoded) and the float stages can be checked against the
 * CPU oracle and the FFmpeg golden vectors.  It is the input generator for
 * BASELINE.json configs 3-5 and for the parity tests.
 *
 * It is an encoder of the ISO 11172-3 bitstream syntax (2.4.1), and of the
 * ISO 13818-3 low-sampling-frequency (LSF) syntax for sample-rate indices
 * 3..8 (MPEG-2 22.05/24/16 kHz, MPEG-2.5 11.025/12/8 kHz: one granule per
 * frame, 8-bit main_data_begin, 9-bit scalefac_compress with the LSF slen /
 * nr_of_sfb tables, LSF intensity positions) -- the reverse of the hot path,
 * sharing only the standards' constant tables.
 *
 * Scalefactor layout of gunit.sf and of the truth records ("canonical", the
 * layout of the decoder's UnitMeta.sf): long band b at b; short band b
 * window w at 3 b + w; mixed blocks: long bands at b (8 of them MPEG-1, 6
 * LSF), short band b >= 3 window w at 8 + 3 (b - 3) + w.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mp3d_tables.h"

#define GEN_API __attribute__((visibility("default")))

/* ---------------- rng: xoshiro256** seeded by splitmix64 ----------------- */
typedef struct { uint64_t s[4]; } rng_t;
static uint64_t splitmix64(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t *r, uint64_t seed) {
    for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&seed);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t rng_next(rng_t *r) {
    uint64_t *s = r->s, res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static int rng_int(rng_t *r, int lo, int hi) { /* inclusive */
    return lo + (int)(rng_next(r) % (uint64_t)(hi - lo + 1));
}
static double rng_unif(rng_t *r) { return (rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }

/* ---------------- bit writer --------------------------------------------- */
typedef struct { uint8_t *buf; long cap_bits, pos; } bw_t;
static void bw_put(bw_t *w, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) {
        if (w->pos < w->cap_bits) {
            long p = w->pos;
            uint8_t m = (uint8_t)(0x80 >> (p & 7));
            if ((v >> i) & 1) w->buf[p >> 3] |= m; else w->buf[p >> 3] &= (uint8_t)~m;
        }
        w->pos++;
    }
}

/* ---------------- configuration ------------------------------------------ */
typedef struct {
    int sr_idx;        /* 0..8 (3..8 LSF), -1: random 0..2, -2: random 3..8  */
    int bitrate_idx;   /* 1..14 CBR, or 0: VBR (random index per frame)     */
    int mode;          /* 0..3, or -1: random per stream                    */
    int mode_ext;      /* joint stereo mode_ext 0..3, or -1: random/frame   */
    int short_pct;     /* % of granules that start a start/short/stop run    */
    int mixed_pct;     /* % of short granules that are mixed blocks          */
    int crc_pct;       /* % of streams with CRC protection                   */
    int fill_pct;      /* target fill of the frame's bit budget (percent)    */
    int max_reservoir; /* cap on main_data_begin (<= 511)                    */
} gen_cfg;

/* Truth record per (frame, gr, ch) for the integer-stage round trip. */
typedef struct {
    int16_t is[576];
    uint8_t sf[40];
    int32_t part2_3_length, big_values, global_gain, block_type, mixed, count1;
} gen_truth;

typedef struct {
    int window_switching, block_type, mixed, table_select[3], subblock_gain[3];
    int region0_count, region1_count, preflag, scalefac_scale, count1table_select;
    int scalefac_compress, global_gain, big_values, part2_3_length, scfsi;
    int lsf, is_right;      /* LSF unit / right channel of an intensity frame */
    int slen[4], nsf[4];    /* LSF scalefactor groups (slen bits, count)      */
    int16_t is[576];
    uint8_t sf[40];
    int count1; /* number of count1 quadruples */
} gunit;

/* ---------------- Huffman encoding --------------------------------------- */
static int pair_bits(int sel, int x, int y, bw_t *w) {
    int tab = MP3D_HTAB_OF_SELECT[sel];
    if (tab < 0) return 0;
    int lin = MP3D_LINBITS[sel], n = MP3D_HTAB_ROWLEN[tab];
    int ax = abs(x), ay = abs(y);
    int cx = lin && ax > 15 ? 15 : ax, cy = lin && ay > 15 ? 15 : ay;
    int idx = cx * n + cy;
    int bits = MP3D_HTAB_LENS[tab][idx];
    if (w) bw_put(w, MP3D_HTAB_CODES[tab][idx], MP3D_HTAB_LENS[tab][idx]);
    if (lin && cx == 15) { bits += lin; if (w) bw_put(w, (uint32_t)(ax - 15), lin); }
    if (x) { bits++; if (w) bw_put(w, x < 0, 1); }
    if (lin && cy == 15) { bits += lin; if (w) bw_put(w, (uint32_t)(ay - 15), lin); }
    if (y) { bits++; if (w) bw_put(w, y < 0, 1); }
    return bits;
}

static int quad_bits(int sel, const int16_t *q, bw_t *w) {
    int v = (q[0] != 0) * 8 + (q[1] != 0) * 4 + (q[2] != 0) * 2 + (q[3] != 0);
    int bits = MP3D_QUAD_LEN[sel][v];
    if (w) bw_put(w, MP3D_QUAD_CODE[sel][v], MP3D_QUAD_LEN[sel][v]);
    for (int i = 0; i < 4; i++)
        if (q[i]) { bits++; if (w) bw_put(w, q[i] < 0, 1); }
    return bits;
}

static void region_ends(const gunit *u, int sr_idx, int *r1, int *r2) {
    int bv2 = u->big_values * 2;
    if (u->window_switching) {
        /* FFmpeg: region0 of window-switched units is 36 lines, except 54
         * for LSF long-type at 22.05..12 kHz and 72 for short at 8 kHz */
        if (u->block_type == 2) *r1 = sr_idx == 8 ? 72 : 36;
        else *r1 = sr_idx <= 2 ? 36 : sr_idx == 8 ? 108 : 54;
        *r2 = 576;
    } else {
        int b1 = u->region0_count + 1, b2 = u->region0_count + u->region1_count + 2;
        if (b2 > 22) b2 = 22;
        *r1 = 0; for (int i = 0; i < b1 && i < 22; i++) *r1 += MP3D_SFB_LONG_WIDTH[sr_idx][i];
        *r2 = 0; for (int i = 0; i < b2; i++) *r2 += MP3D_SFB_LONG_WIDTH[sr_idx][i];
    }
    if (*r1 > bv2) *r1 = bv2;
    if (*r2 > bv2) *r2 = bv2;
}

/* Scalefactor bits (part 2) in the FFmpeg/our sf[] layout. */
/* canonical sf index of the i-th coded LSF scalefactor */
static int lsf_sf_index(const gunit *u, int i) {
    return (u->window_switching && u->block_type == 2 && u->mixed && i >= 6) ? i + 2 : i;
}

static int part2_bits(const gunit *u, const uint8_t *sf_gr0, bw_t *w) {
    int slen1 = MP3D_SLEN[0][u->scalefac_compress & 15], slen2 = MP3D_SLEN[1][u->scalefac_compress & 15];
    int bits = 0, j = 0;
    (void)sf_gr0;
    if (u->lsf) {
        for (int k = 0; k < 4; k++)
            for (int i = 0; i < u->nsf[k]; i++, j++) {
                bits += u->slen[k];
                if (w && u->slen[k]) bw_put(w, u->sf[lsf_sf_index(u, j)], u->slen[k]);
            }
        return bits;
    }
    if (u->window_switching && u->block_type == 2) {
        int n = u->mixed ? 17 : 18;
        for (int i = 0; i < n; i++) { bits += slen1; if (w) bw_put(w, u->sf[j], slen1); j++; }
        for (int i = 0; i < 18; i++) { bits += slen2; if (w) bw_put(w, u->sf[j], slen2); j++; }
    } else {
        for (int k = 0; k < 4; k++) {
            int n = k == 0 ? 6 : 5, slen = k < 2 ? slen1 : slen2;
            if (u->scfsi & (8 >> k)) { j += n; continue; }
            for (int i = 0; i < n; i++) { bits += slen; if (w) bw_put(w, u->sf[j], slen); j++; }
        }
    }
    return bits;
}

/* Total part2_3 bits; writes if w != NULL. */
static int unit_bits(const gunit *u, int sr_idx, const uint8_t *sf_gr0, bw_t *w) {
    int bits = part2_bits(u, sf_gr0, w);
    int r1, r2, bv2 = u->big_values * 2;
    region_ends(u, sr_idx, &r1, &r2);
    int k = 0;
    for (int reg = 0; reg < 3; reg++) {
        int end = reg == 0 ? r1 : reg == 1 ? r2 : bv2;
        for (; k < end; k += 2) bits += pair_bits(u->table_select[reg], u->is[k], u->is[k + 1], w);
    }
    for (int q = 0; q < u->count1; q++, k += 4) bits += quad_bits(u->count1table_select, &u->is[k], w);
    return bits;
}

/* max |value| representable by a table_select */
static int sel_max(int sel) {
    int tab = MP3D_HTAB_OF_SELECT[sel];
    if (tab < 0) return 0;
    int n = MP3D_HTAB_ROWLEN[tab];
    return MP3D_LINBITS[sel] ? 15 + (1 << MP3D_LINBITS[sel]) - 1 : n - 1;
}

/* Draw one quantised value for a region whose table_select is sel, biased
 * to small magnitudes as real spectra are; escape tables reach big values. */
static int draw_value(rng_t *r, int sel, int esc_scale) {
    int m = sel_max(sel);
    if (m == 0) return 0;
    double u = rng_unif(r);
    int v;
    if (MP3D_LINBITS[sel] && u < 0.25) {
        int cap = m < esc_scale ? m : esc_scale;
        v = 15 + (int)((cap - 15) * pow(rng_unif(r), 3.0));
    } else {
        int cap = m > 15 ? 15 : m;
        v = (int)floor(pow(rng_unif(r), 1.6) * (cap + 1));
        if (v > cap) v = cap;
    }
    if (v && (rng_next(r) & 1)) v = -v;
    return v;
}

static const int SEL_CHOICES[] = {0, 1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15,
                                  16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31};

/* Fill unit spectrum; `scale` in (0,1] shrinks the nonzero extent. */
static void fill_spectrum(rng_t *r, gunit *u, int sr_idx, double scale, int is_bound) {
    memset(u->is, 0, sizeof(u->is));
    int limit = is_bound >= 0 ? is_bound : 576;
    int bv = (int)(rng_int(r, 20, 210) * scale);
    if (bv * 2 > limit) bv = limit / 2;
    if (bv > 288) bv = 288;
    u->big_values = bv;
    for (int reg = 0; reg < 3; reg++) {
        int s = SEL_CHOICES[rng_int(r, 0, (int)(sizeof(SEL_CHOICES) / sizeof(int)) - 1)];
        if (rng_unif(r) < 0.05) s = 0;
        u->table_select[reg] = s;
    }
    if (u->window_switching) u->table_select[2] = 0;
    int r1, r2;
    region_ends(u, sr_idx, &r1, &r2);
    int esc_scale = 15 + (rng_unif(r) < 0.3 ? (int)(8191 * pow(rng_unif(r), 2.0)) : 40);
    int k = 0;
    for (int reg = 0; reg < 3; reg++) {
        int end = reg == 0 ? r1 : reg == 1 ? r2 : bv * 2;
        for (; k < end; k++) u->is[k] = (int16_t)draw_value(r, u->table_select[reg], esc_scale);
    }
    int room = (limit - bv * 2) / 4;
    int c1 = (int)(rng_int(r, 10, 60) * scale);
    if (c1 > room) c1 = room;
    if (c1 < 0) c1 = 0;
    u->count1 = c1;
    for (int q = 0; q < c1 * 4; q++) {
        int v = rng_unif(r) < 0.45 ? (rng_next(r) & 1 ? 1 : -1) : 0;
        u->is[bv * 2 + q] = (int16_t)v;
    }
    /* FFmpeg/ISO: a trailing all-zero count1 quadruple decodes the same as
     * rzero, so keep it -- it is legal syntax and exercises the decoder. */
}

/* FFmpeg lsf_sf_expand: slen[] from a scalefac_compress sub-range */
static void lsf_expand(int *slen, int sf, int n1, int n2, int n3) {
    if (n3) { slen[3] = sf % n3; sf /= n3; } else slen[3] = 0;
    if (n2) { slen[2] = sf % n2; sf /= n2; } else slen[2] = 0;
    slen[1] = sf % n1;
    slen[0] = sf / n1;
}

/* LSF scalefac_compress -> slen[4], nr_of_sfb[4], preflag (ISO 13818-3
 * 2.4.3.2; FFmpeg mp_decode_layer3) */
static void lsf_groups(gunit *u) {
    int sf = u->scalefac_compress, t2;
    int tindex = u->window_switching && u->block_type == 2 ? (u->mixed ? 2 : 1) : 0;
    u->preflag = 0;
    if (u->is_right) {
        sf >>= 1;
        if (sf < 180) { lsf_expand(u->slen, sf, 6, 6, 0); t2 = 3; }
        else if (sf < 244) { lsf_expand(u->slen, sf - 180, 4, 4, 0); t2 = 4; }
        else { lsf_expand(u->slen, sf - 244, 3, 0, 0); t2 = 5; }
    } else {
        if (sf < 400) { lsf_expand(u->slen, sf, 5, 4, 4); t2 = 0; }
        else if (sf < 500) { lsf_expand(u->slen, sf - 400, 5, 4, 0); t2 = 1; }
        else { lsf_expand(u->slen, sf - 500, 3, 0, 0); t2 = 2; u->preflag = 1; }
    }
    for (int k = 0; k < 4; k++) u->nsf[k] = MP3D_LSF_NSF[t2][tindex][k];
}

/* slen of canonical sf index j of an LSF unit (0 if not coded) */
static int lsf_slen_at(const gunit *u, int j) {
    int i = 0;
    for (int k = 0; k < 4; k++)
        for (int n = 0; n < u->nsf[k]; n++, i++)
            if (lsf_sf_index(u, i) == j) return u->slen[k];
    return 0;
}

static void fill_scalefactors(rng_t *r, gunit *u, const gunit *gr0, int is_bound_sfb_long, int is_ch1,
                              int sr_idx) {
    (void)sr_idx;
    if (u->lsf) {
        /* 9-bit scalefac_compress; the IS right channel's carries
         * intensity_scale in bit 0 and its range selects the IS slen table */
        u->scalefac_compress = rng_int(r, 0, 511);
        lsf_groups(u);
        memset(u->sf, 0, sizeof(u->sf));
        int i = 0;
        for (int k = 0; k < 4; k++)
            for (int n = 0; n < u->nsf[k]; n++, i++)
                u->sf[lsf_sf_index(u, i)] = (uint8_t)(u->slen[k] ? rng_int(r, 0, (1 << u->slen[k]) - 1) : 0);
        return;
    }
    u->scalefac_compress = rng_int(r, 0, 15);
    int slen1 = MP3D_SLEN[0][u->scalefac_compress], slen2 = MP3D_SLEN[1][u->scalefac_compress];
    memset(u->sf, 0, sizeof(u->sf));
    if (u->window_switching && u->block_type == 2) {
        int n = u->mixed ? 17 : 18;
        for (int i = 0; i < n; i++) u->sf[i] = (uint8_t)(slen1 ? rng_int(r, 0, (1 << slen1) - 1) : 0);
        for (int i = 0; i < 18; i++) u->sf[n + i] = (uint8_t)(slen2 ? rng_int(r, 0, (1 << slen2) - 1) : 0);
    } else {
        int j = 0;
        for (int k = 0; k < 4; k++) {
            int n = k == 0 ? 6 : 5, slen = k < 2 ? slen1 : slen2;
            for (int i = 0; i < n; i++, j++) {
                if (u->scfsi & (8 >> k)) u->sf[j] = gr0->sf[j];
                else u->sf[j] = (uint8_t)(slen ? rng_int(r, 0, (1 << slen) - 1) : 0);
            }
        }
    }
    (void)is_bound_sfb_long;
    (void)is_ch1;
}

/* CRC-16 (poly 0x8005, init 0xFFFF) over header bytes 2..3 + side info. */
static uint16_t crc16_bits(uint16_t crc, const uint8_t *p, int nbytes) {
    for (int i = 0; i < nbytes; i++)
        for (int b = 7; b >= 0; b--) {
            int bit = (p[i] >> b) & 1;
            int top = (crc >> 15) & 1;
            crc = (uint16_t)(crc << 1);
            if (top ^ bit) crc ^= 0x8005;
        }
    return crc;
}

/* frame bytes: 144000 * kbps / Hz (MPEG-1), 72000 * kbps / Hz (LSF) */
static int frame_num(int br_idx, int sr_idx) {
    return sr_idx < 3 ? 144000 * MP3D_BITRATE_L3[br_idx] : 72000 * MP3D_BITRATE_L3_LSF[br_idx];
}
static int frame_len(int br_idx, int sr_idx, int pad) {
    return frame_num(br_idx, sr_idx) / (int)MP3D_SAMPLE_RATE[sr_idx] + pad;
}

/* Pick IS boundary (first line of the intensity region of channel 1) on a
 * scalefactor-band edge, and the is_pos values of the bands above it. */
static int pick_is_bound(rng_t *r, const gunit *u, int sr_idx) {
    if (u->window_switching && u->block_type == 2) {
        /* short: bound on a short-band edge (all 3 windows), in lines of the
         * window-grouped bitstream order */
        int b0 = u->mixed ? 3 : 0;
        int band = rng_int(r, b0 + 1, 12);
        int line = u->mixed ? (sr_idx == 8 ? 72 : 36) : 0;
        for (int i = b0; i < band; i++) line += 3 * MP3D_SFB_SHORT_WIDTH[sr_idx][i];
        return line;
    }
    int band = rng_int(r, 4, 21);
    int line = 0;
    for (int i = 0; i < band; i++) line += MP3D_SFB_LONG_WIDTH[sr_idx][i];
    return line;
}

/* Set the scalefactors of the IS bands of channel 1 to random is_pos. */
static void set_is_positions(rng_t *r, gunit *u, int sr_idx, int bound) {
    if (u->lsf) {
        /* LSF: any coded value; FFmpeg treats is_pos >= 16 as "not IS" */
        if (u->window_switching && u->block_type == 2) {
            int b0 = u->mixed ? 3 : 0, line = u->mixed ? (sr_idx == 8 ? 72 : 36) : 0;
            for (int i = b0; i < 12; i++) {
                for (int w = 0; w < 3; w++) {
                    int j = u->mixed ? 8 + 3 * (i - 3) + w : 3 * i + w, sl = lsf_slen_at(u, j);
                    if (line >= bound && sl) u->sf[j] = (uint8_t)rng_int(r, 0, (1 << sl) - 1);
                }
                line += 3 * MP3D_SFB_SHORT_WIDTH[sr_idx][i];
            }
        } else {
            int line = 0;
            for (int i = 0; i < 21; i++) {
                int sl = lsf_slen_at(u, i);
                if (line >= bound && sl) u->sf[i] = (uint8_t)rng_int(r, 0, (1 << sl) - 1);
                line += MP3D_SFB_LONG_WIDTH[sr_idx][i];
            }
        }
        return;
    }
    int slen1 = MP3D_SLEN[0][u->scalefac_compress], slen2 = MP3D_SLEN[1][u->scalefac_compress];
    if (u->window_switching && u->block_type == 2) {
        int b0 = u->mixed ? 3 : 0, line = u->mixed ? 36 : 0, j = u->mixed ? 8 : 0;
        for (int i = b0; i < 12; i++) {
            int slen = (i < 6) ? slen1 : slen2;
            for (int w = 0; w < 3; w++, j++)
                if (line >= bound && slen) u->sf[j] = (uint8_t)rng_int(r, 0, ((1 << slen) - 1) < 7 ? (1 << slen) - 1 : 7);
            line += 3 * MP3D_SFB_SHORT_WIDTH[sr_idx][i];
        }
    } else {
        int line = 0;
        for (int i = 0; i < 21; i++) {
            int slen = i < 11 ? slen1 : slen2;
            if (line >= bound && slen && !(u->scfsi & (8 >> (i < 6 ? 0 : i < 11 ? 1 : i < 16 ? 2 : 3))))
                u->sf[i] = (uint8_t)rng_int(r, 0, ((1 << slen) - 1) < 7 ? (1 << slen) - 1 : 7);
            line += MP3D_SFB_LONG_WIDTH[sr_idx][i];
        }
    }
}

static double unit_peak(const gunit *u) {
    int m = 0;
    for (int i = 0; i < 576; i++) if (abs(u->is[i]) > m) m = abs(u->is[i]);
    return pow((double)m, 4.0 / 3.0);
}

/*
 * Generate one stream of n_frames frames into out (capacity cap bytes).
 * Returns bytes written, or -1 on capacity overflow.  frame_off (optional)
 * receives the byte offset of each frame; truth (optional) receives
 * n_frames*2*2 unit records.
 */
GEN_API long mp3gen_stream(const gen_cfg *cfg, uint64_t seed, int n_frames, uint8_t *out, long cap,
                           uint32_t *frame_off, gen_truth *truth) {
    rng_t R;
    rng_seed(&R, seed);
    int sr_idx = cfg->sr_idx >= 0 ? cfg->sr_idx : cfg->sr_idx == -2 ? rng_int(&R, 3, 8) : rng_int(&R, 0, 2);
    int mode = cfg->mode >= 0 ? cfg->mode : rng_int(&R, 0, 3);
    int nch = mode == 3 ? 1 : 2;
    int crc = rng_int(&R, 0, 99) < cfg->crc_pct;
    const int lsf = sr_idx >= 3, ngr = lsf ? 1 : 2;
    int side_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
    const int res_cap = lsf ? 255 : 511; /* main_data_begin: 8 / 9 bits */
    int max_res = cfg->max_reservoir > res_cap ? res_cap : cfg->max_reservoir;
    /* main-data byte stream: payloads concatenated, pre-filled with noise
     * (ancillary bytes must never be read by a correct decoder) */
    long md_cap = (long)n_frames * 1441 + 4096;
    uint8_t *md = (uint8_t *)malloc((size_t)md_cap);
    if (!md) return -1;
    for (long i = 0; i < md_cap; i++) md[i] = (uint8_t)rng_next(&R);
    int *flen = (int *)malloc(sizeof(int) * (size_t)n_frames);
    int *fbr = (int *)malloc(sizeof(int) * (size_t)n_frames);
    int *fpad = (int *)malloc(sizeof(int) * (size_t)n_frames);
    int *fmext = (int *)malloc(sizeof(int) * (size_t)n_frames);
    long *fmd = (long *)malloc(sizeof(long) * (size_t)n_frames); /* payload start in md */
    uint8_t (*side)[32] = (uint8_t (*)[32])malloc(32 * (size_t)n_frames);
    long md_pos = 0;
    int R_avail = 0;      /* bytes after previous main-data end */
    int pad_acc = 0;
    int bt_state = 0;     /* block type state machine, shared by channels */
    int short_left = 0;
    int run_mixed = 0;    /* a short run is either all mixed or all pure: the
                           * canonical sequences (FFmpeg's short IMDCT relies
                           * on them: it skips overlap slots 12..17) */
    for (int f = 0; f < n_frames; f++) {
        int br = cfg->bitrate_idx > 0 ? cfg->bitrate_idx : rng_int(&R, 1, 14);
        /* ISO padding: keep the average frame length exact */
        int hz = (int)MP3D_SAMPLE_RATE[sr_idx];
        int rem = frame_num(br, sr_idx) % hz;
        pad_acc += rem;
        int pad = 0;
        if (pad_acc >= hz) { pad = 1; pad_acc -= hz; }
        int fb = frame_len(br, sr_idx, pad);
        int plen = fb - 4 - (crc ? 2 : 0) - side_bytes;
        int mext = 0;
        if (mode == 1) mext = cfg->mode_ext >= 0 ? cfg->mode_ext : rng_int(&R, 0, 3);
        flen[f] = fb; fbr[f] = br; fpad[f] = pad; fmext[f] = mext; fmd[f] = md_pos;

        /* block types for the two granules (shared by channels) */
        int bts[2] = {0, 0}, mixeds[2] = {0, 0};
        for (int gr = 0; gr < ngr; gr++) {
            int mx = 0;
            if (bt_state == 0) {
                if (rng_int(&R, 0, 99) < cfg->short_pct) bt_state = 1;
            } else if (bt_state == 1) {
                bt_state = 2; short_left = rng_int(&R, 1, 3);
                run_mixed = rng_int(&R, 0, 99) < cfg->mixed_pct;
            } else if (bt_state == 2) {
                if (--short_left <= 0) bt_state = 3;
            } else {
                bt_state = 0;
            }
            if (bt_state == 2) mx = run_mixed;
            bts[gr] = bt_state; mixeds[gr] = mx;
        }

        int budget_bits = (plen + (R_avail < max_res ? R_avail : max_res)) * 8;
        int target = (int)(budget_bits * (cfg->fill_pct / 100.0) * (0.55 + 0.5 * rng_unif(&R)));
        gunit U[2][2];
        int total_bits = 0;
        double scale = 1.0;
        uint8_t unit_bytes_ok = 0;
        for (int attempt = 0; attempt < 40 && !unit_bytes_ok; attempt++) {
            total_bits = 0;
            for (int gr = 0; gr < ngr; gr++)
                for (int ch = 0; ch < nch; ch++) {
                    gunit *u = &U[gr][ch];
                    memset(u, 0, sizeof(*u));
                    u->lsf = lsf;
                    u->is_right = lsf && mode == 1 && (mext & 1) && ch == 1;
                    u->block_type = bts[gr];
                    u->window_switching = bts[gr] != 0;
                    u->mixed = bts[gr] == 2 ? mixeds[gr] : 0;
                    u->scalefac_scale = rng_int(&R, 0, 1);
                    u->preflag = u->window_switching && u->block_type == 2 ? 0 : rng_int(&R, 0, 1);
                    u->count1table_select = rng_int(&R, 0, 1);
                    for (int w = 0; w < 3; w++) u->subblock_gain[w] = u->block_type == 2 ? rng_int(&R, 0, 3) : 0;
                    u->region0_count = rng_int(&R, 0, 15);
                    u->region1_count = rng_int(&R, 0, 7);
                    if (u->window_switching) {
                        u->region0_count = u->block_type == 2 ? 8 : 7; /* implied, not coded */
                        u->region1_count = 36;
                    }
                    u->scfsi = 0;
                    if (gr == 1 && !u->window_switching && !U[0][ch].window_switching)
                        u->scfsi = rng_int(&R, 0, 15);
                    int is_bound = -1;
                    if (mode == 1 && (mext & 1) && ch == 1) is_bound = pick_is_bound(&R, u, sr_idx);
                    fill_spectrum(&R, u, sr_idx, scale, is_bound);
                    fill_scalefactors(&R, u, &U[0][ch], 0, ch, sr_idx);
                    if (is_bound >= 0) set_is_positions(&R, u, sr_idx, is_bound);
                    double pk = unit_peak(u);
                    double amp = 0.01 + 0.12 * rng_unif(&R);
                    int gg = pk > 0 ? 210 + (int)floor(4.0 * log2(amp / pk)) : rng_int(&R, 100, 200);
                    if (gg < 0) gg = 0;
                    if (gg > 255) gg = 255;
                    u->global_gain = gg;
                    u->part2_3_length = unit_bits(u, sr_idx, U[0][ch].sf, NULL);
                    total_bits += u->part2_3_length;
                }
            int used = (total_bits + 7) / 8;
            int lo = used - plen; if (lo < 0) lo = 0;
            int hi = R_avail < max_res ? R_avail : max_res;
            if (hi > used - 1) hi = used - 1;
            int bad = 0;
            for (int gr = 0; gr < ngr; gr++)
                for (int ch = 0; ch < nch; ch++) if (U[gr][ch].part2_3_length > 4095) bad = 1;
            if (!bad && used >= 1 && lo <= hi && total_bits <= target + 400) unit_bytes_ok = 1;
            else {
                /* shrink toward the target in proportion to the overshoot */
                double ratio = total_bits > 0 ? 0.95 * (double)target / (double)total_bits : 0.5;
                scale *= ratio < 0.8 ? (ratio > 0.1 ? ratio : 0.1) : 0.8;
            }
        }
        if (!unit_bytes_ok) { /* fall back to silence units */
            total_bits = 0;
            for (int gr = 0; gr < ngr; gr++)
                for (int ch = 0; ch < nch; ch++) {
                    memset(&U[gr][ch], 0, sizeof(gunit));
                    U[gr][ch].global_gain = 150;
                    U[gr][ch].lsf = lsf;
                    U[gr][ch].is_right = lsf && mode == 1 && (mext & 1) && ch == 1;
                    if (lsf) lsf_groups(&U[gr][ch]);
                }
        }
        int used = (total_bits + 7) / 8;
        int lo = used - plen; if (lo < 0) lo = 0;
        int hi = R_avail < max_res ? R_avail : max_res;
        if (hi > used - 1) hi = used - 1;
        if (hi < lo) hi = lo;
        int mdb = total_bits == 0 ? 0 : (rng_int(&R, 0, 3) == 0 ? rng_int(&R, lo, hi) : hi);
        if (mdb > R_avail) mdb = R_avail < lo ? lo : R_avail; /* never reached for valid input */
        /* write main data */
        bw_t w = {md, md_cap * 8, (md_pos - mdb) * 8};
        for (int gr = 0; gr < ngr; gr++)
            for (int ch = 0; ch < nch; ch++) {
                long p0 = w.pos;
                unit_bits(&U[gr][ch], sr_idx, U[0][ch].sf, &w);
                (void)p0;
            }
        /* zero-pad the last partial byte so bits are deterministic */
        while (w.pos & 7) bw_put(&w, 0, 1);
        R_avail = plen + mdb - used;
        if (total_bits == 0) R_avail = plen + mdb;
        /* side info */
        uint8_t *sp = side[f];
        memset(sp, 0, 32);
        bw_t sw = {sp, side_bytes * 8, 0};
        if (lsf) {
            bw_put(&sw, (uint32_t)mdb, 8);
            bw_put(&sw, 0, nch == 1 ? 1 : 2);
        } else {
            bw_put(&sw, (uint32_t)mdb, 9);
            bw_put(&sw, 0, nch == 1 ? 5 : 3);
            for (int ch = 0; ch < nch; ch++) bw_put(&sw, (uint32_t)U[1][ch].scfsi, 4);
        }
        for (int gr = 0; gr < ngr; gr++)
            for (int ch = 0; ch < nch; ch++) {
                gunit *u = &U[gr][ch];
                bw_put(&sw, (uint32_t)u->part2_3_length, 12);
                bw_put(&sw, (uint32_t)u->big_values, 9);
                bw_put(&sw, (uint32_t)u->global_gain, 8);
                bw_put(&sw, (uint32_t)u->scalefac_compress, lsf ? 9 : 4);
                bw_put(&sw, (uint32_t)u->window_switching, 1);
                if (u->window_switching) {
                    bw_put(&sw, (uint32_t)u->block_type, 2);
                    bw_put(&sw, (uint32_t)u->mixed, 1);
                    bw_put(&sw, (uint32_t)u->table_select[0], 5);
                    bw_put(&sw, (uint32_t)u->table_select[1], 5);
                    for (int k = 0; k < 3; k++) bw_put(&sw, (uint32_t)u->subblock_gain[k], 3);
                } else {
                    for (int k = 0; k < 3; k++) bw_put(&sw, (uint32_t)u->table_select[k], 5);
                    bw_put(&sw, (uint32_t)u->region0_count, 4);
                    bw_put(&sw, (uint32_t)u->region1_count, 3);
                }
                if (!lsf) bw_put(&sw, (uint32_t)u->preflag, 1); /* LSF: implied by scalefac_compress */
                bw_put(&sw, (uint32_t)u->scalefac_scale, 1);
                bw_put(&sw, (uint32_t)u->count1table_select, 1);
                if (truth) {
                    gen_truth *t = &truth[((long)f * 2 + gr) * 2 + ch];
                    memcpy(t->is, u->is, sizeof(t->is));
                    memcpy(t->sf, u->sf, sizeof(t->sf));
                    t->part2_3_length = u->part2_3_length;
                    t->big_values = u->big_values;
                    t->global_gain = u->global_gain;
                    t->block_type = u->window_switching ? u->block_type : 0;
                    t->mixed = u->mixed;
                    t->count1 = u->count1;
                }
            }
        if (truth && nch == 1)
            for (int gr = 0; gr < ngr; gr++) memset(&truth[((long)f * 2 + gr) * 2 + 1], 0, sizeof(gen_truth));
        if (truth && lsf) memset(&truth[((long)f * 2 + 1) * 2], 0, 2 * sizeof(gen_truth)); /* no granule 1 */
        md_pos += plen;
    }
    /* assemble frames */
    long o = 0;
    for (int f = 0; f < n_frames; f++) {
        int fb = flen[f];
        if (o + fb > cap) { o = -1; break; }
        uint8_t *p = out + o;
        if (frame_off) frame_off[f] = (uint32_t)o;
        /* version bits: 3 MPEG-1, 2 MPEG-2, 0 MPEG-2.5; layer bits 01 = III */
        const int ver = sr_idx < 3 ? 3 : sr_idx < 6 ? 2 : 0;
        p[0] = 0xFF;
        p[1] = (uint8_t)(0xE0 | (ver << 3) | 0x2 | (crc ? 0 : 1));
        p[2] = (uint8_t)((fbr[f] << 4) | ((sr_idx % 3) << 2) | (fpad[f] << 1));
        p[3] = (uint8_t)((mode << 6) | (fmext[f] << 4) | 0x4 /* original */);
        int hdr = 4;
        if (crc) {
            uint16_t c = crc16_bits(0xFFFF, p + 2, 2);
            c = crc16_bits(c, side[f], side_bytes);
            p[4] = (uint8_t)(c >> 8);
            p[5] = (uint8_t)c;
            hdr = 6;
        }
        memcpy(p + hdr, side[f], (size_t)side_bytes);
        int plen = fb - hdr - side_bytes;
        memcpy(p + hdr + side_bytes, md + fmd[f], (size_t)plen);
        o += fb;
    }
    free(md); free(flen); free(fbr); free(fpad); free(fmext); free(fmd); free(side);
    return o;
}

GEN_API int mp3gen_truth_size(void) { return (int)sizeof(gen_truth); }
GEN_API int mp3gen_cfg_size(void) { return (int)sizeof(gen_cfg); }

/* Upper bound on bytes for n_frames of a configuration. */
GEN_API long mp3gen_max_bytes(const gen_cfg *cfg, int n_frames) {
    int maxfb = 0;
    for (int sr = 0; sr < 9; sr++) {
        if (cfg->sr_idx >= 0 && sr != cfg->sr_idx) continue;
        if (cfg->sr_idx == -1 && sr >= 3) continue;
        if (cfg->sr_idx == -2 && sr < 3) continue;
        for (int br = 1; br <= 14; br++) {
            if (cfg->bitrate_idx > 0 && br != cfg->bitrate_idx) continue;
            int fb = frame_len(br, sr, 1);
            if (fb > maxfb) maxfb = fb;
        }
    }
    return (long)maxfb * n_frames;
}

/*
 * Batch: n_streams streams of n_frames each, stream s seeded with
 * seed_base + s, packed back to back.  offsets/sizes receive each stream's
 * byte range.  Returns total bytes, or -1.  Multi-threaded over streams.
 */
GEN_API long mp3gen_batch(const gen_cfg *cfg, uint64_t seed_base, int n_streams, int n_frames, uint8_t *out,
                          long cap, uint64_t *offsets, uint32_t *sizes, int n_threads) {
    long stride = mp3gen_max_bytes(cfg, n_frames);
    if (stride * (long)n_streams > cap) return -1;
    int fail = 0;
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads > 0 ? n_threads : 1)
    for (int s = 0; s < n_streams; s++) {
        long n = mp3gen_stream(cfg, seed_base + (uint64_t)s, n_frames, out + (long)s * stride, stride, NULL, NULL);
        if (n < 0) fail = 1;
        sizes[s] = (uint32_t)(n < 0 ? 0 : n);
    }
    if (fail) return -1;
    long o = 0;
    for (int s = 0; s < n_streams; s++) {
        if (o != (long)s * stride) memmove(out + o, out + (long)s * stride, sizes[s]);
        offsets[s] = (uint64_t)o;
        o += sizes[s];
    }
    return o;
}
