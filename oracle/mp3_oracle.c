/*
 * mp3_oracle.c -- CPU restatement of the MPEG-1 Layer III decode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) -- never as the product path.
 *
 * The reference (lxm0851/mp3) ships no decoder source: REF/README.md:2-3
 * describes an audio player whose decode loop is this path, and REF/ holds
 * only README.md and LICENSE.  Every stage below therefore
 * restates ISO/IEC 11172-3 (clauses cited per function) and mirrors the
 * FFmpeg conventions that the in-container golden oracle (Chromium 88's
 * FFmpeg mpegaudiodec) follows where ISO leaves freedom
 * (SURVEY.md Appendix A.9).  Parity is pinned by committed golden PCM from
 * that oracle (tests/golden/), not by reference tests (none exist).
 *
 * Arithmetic is double precision throughout (orc_real = double), so this
 * file is an independent high-precision restatement, not a bit-copy of the
 * GPU path.  Built with -DORC_REAL=float (liboracle_f32.so, -O3) the same
 * source is the single-precision CPU decoder that bench.py times as the CPU
 * baseline; the tests check only the double build.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../mp3_amd/csrc/mp3d_tables.h"

#define ORC_API __attribute__((visibility("default")))

#ifndef ORC_REAL
#define ORC_REAL double
#endif
typedef ORC_REAL orc_real;

/* ------------------------------------------------------------------------ */
/* Header, ISO 2.4.1.3 / 2.4.2.3                                             */
/* ------------------------------------------------------------------------ */
typedef struct {
    int protection_absent, bitrate_idx, sr_idx, padding, mode, mode_ext;
    int nch, kbps, hz, frame_bytes, side_bytes, crc_bytes;
    int lsf, ngr; /* MPEG-2 / 2.5 low sampling frequency: 1 granule / frame */
} orc_hdr;

/* Returns frame length in bytes, or -1 if `p` is not a Layer III header
 * (MPEG-1, MPEG-2 or MPEG-2.5; ISO 11172-3 2.4.2.3, 13818-3 2.4.2.3) with
 * a non-free-format bitrate.  sr_idx = sampling_frequency + 3 (MPEG-2) or
 * + 6 (MPEG-2.5), FFmpeg's sample_rate_index. */
ORC_API int orc_parse_header(const uint8_t *p, orc_hdr *h) {
    if (p[0] != 0xFF || (p[1] & 0xE0) != 0xE0) return -1; /* 11-bit sync */
    const int ver = (p[1] >> 3) & 3, layer = (p[1] >> 1) & 3;
    if (ver == 1 || layer != 1) return -1; /* reserved version; Layer III only */
    int bi = p[2] >> 4, si = (p[2] >> 2) & 3;
    if (bi == 0 || bi == 15 || si == 3) return -1;
    h->lsf = ver != 3;
    h->ngr = h->lsf ? 1 : 2;
    h->protection_absent = p[1] & 1;
    h->bitrate_idx = bi;
    h->sr_idx = si + (ver == 3 ? 0 : ver == 2 ? 3 : 6);
    h->padding = (p[2] >> 1) & 1;
    h->mode = p[3] >> 6;
    h->mode_ext = (p[3] >> 4) & 3;
    h->nch = h->mode == 3 ? 1 : 2;
    h->kbps = h->lsf ? MP3D_BITRATE_L3_LSF[bi] : MP3D_BITRATE_L3[bi];
    h->hz = (int)MP3D_SAMPLE_RATE[h->sr_idx];
    h->frame_bytes = (h->lsf ? 72000 : 144000) * h->kbps / h->hz + h->padding;
    h->crc_bytes = h->protection_absent ? 0 : 2;
    h->side_bytes = h->lsf ? (h->nch == 1 ? 9 : 17) : (h->nch == 1 ? 17 : 32);
    return h->frame_bytes;
}

/* ------------------------------------------------------------------------ */
/* Bit reader (MSB first), reads zeros past the end.                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t *buf;
    long nbits, pos;
} orc_bits;

static unsigned orc_get1(orc_bits *b) {
    unsigned v = 0;
    if (b->pos >= 0 && b->pos < b->nbits) v = (b->buf[b->pos >> 3] >> (7 - (b->pos & 7))) & 1;
    b->pos++;
    return v;
}
static unsigned orc_get(orc_bits *b, int n) {
    unsigned v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | orc_get1(b);
    return v;
}

/* ------------------------------------------------------------------------ */
/* Side information, ISO 2.4.1.7 / 2.4.2.7                                   */
/* ------------------------------------------------------------------------ */
typedef struct {
    int part2_3_length, big_values, global_gain, scalefac_compress;
    int window_switching, block_type, mixed, table_select[3], subblock_gain[3];
    int region0_count, region1_count, preflag, scalefac_scale, count1table_select;
    int scfsi;
    int lsf, is_right; /* LSF unit; right channel of an intensity-stereo LSF frame */
} orc_gr;

typedef struct {
    int main_data_begin;
    orc_gr gr[2][2]; /* [granule][channel] */
} orc_side;

/* Side info; LSF (13818-3 2.4.1.7): 8-bit main_data_begin, 1 / 2 private
 * bits, no scfsi, one granule, 9-bit scalefac_compress, no preflag bit
 * (implied by scalefac_compress, set in orc_read_scalefactors). */
static void orc_parse_side(const uint8_t *p, const orc_hdr *h, orc_side *s) {
    const int nch = h->nch, lsf = h->lsf;
    orc_bits b = {p, h->side_bytes * 8, 0};
    memset(s->gr, 0, sizeof(s->gr));
    s->main_data_begin = (int)orc_get(&b, lsf ? 8 : 9);
    orc_get(&b, lsf ? nch : (nch == 1 ? 5 : 3)); /* private bits */
    int scfsi[2] = {0, 0};
    if (!lsf)
        for (int ch = 0; ch < nch; ch++) scfsi[ch] = (int)orc_get(&b, 4);
    for (int gr = 0; gr < h->ngr; gr++)
        for (int ch = 0; ch < nch; ch++) {
            orc_gr *g = &s->gr[gr][ch];
            memset(g, 0, sizeof(*g));
            g->lsf = lsf;
            g->is_right = lsf && h->mode == 1 && (h->mode_ext & 1) && ch == 1;
            g->scfsi = gr == 1 ? scfsi[ch] : 0;
            g->part2_3_length = (int)orc_get(&b, 12);
            g->big_values = (int)orc_get(&b, 9);
            g->global_gain = (int)orc_get(&b, 8);
            g->scalefac_compress = (int)orc_get(&b, lsf ? 9 : 4);
            g->window_switching = (int)orc_get(&b, 1);
            if (g->window_switching) {
                g->block_type = (int)orc_get(&b, 2);
                g->mixed = (int)orc_get(&b, 1);
                g->table_select[0] = (int)orc_get(&b, 5);
                g->table_select[1] = (int)orc_get(&b, 5);
                for (int w = 0; w < 3; w++) g->subblock_gain[w] = (int)orc_get(&b, 3);
            } else {
                for (int r = 0; r < 3; r++) g->table_select[r] = (int)orc_get(&b, 5);
                g->region0_count = (int)orc_get(&b, 4);
                g->region1_count = (int)orc_get(&b, 3);
            }
            g->preflag = lsf ? 0 : (int)orc_get(&b, 1);
            g->scalefac_scale = (int)orc_get(&b, 1);
            g->count1table_select = (int)orc_get(&b, 1);
        }
}

/* ------------------------------------------------------------------------ */
/* Huffman decode trees (built from Annex B Table B.7 code/length lists).    */
/* ------------------------------------------------------------------------ */
typedef struct {
    int16_t child[2][600]; /* >0 node index, <=0 leaf: -(value) */
    int n;
} orc_tree;
static orc_tree g_trees[MP3D_NUM_HTABS + 1]; /* last = count1 table A */
static int g_trees_ready = 0;
static orc_real g_pow43[8207 + 16];
static orc_real g_imdct36[18][36], g_imdct12[6][12], g_win[4][36], g_synthN[64][32], g_D[512];

static void orc_tree_add(orc_tree *t, unsigned code, int len, int value) {
    int node = 0;
    for (int i = len - 1; i >= 0; i--) {
        int bit = (code >> i) & 1;
        if (i == 0) {
            t->child[bit][node] = (int16_t)(-value);
        } else {
            if (t->child[bit][node] <= 0) t->child[bit][node] = (int16_t)(t->n++);
            node = t->child[bit][node];
        }
    }
}

static void orc_init_tables(void) {
    if (g_trees_ready) return;
    for (int t = 0; t < MP3D_NUM_HTABS; t++) {
        orc_tree *tr = &g_trees[t];
        memset(tr, 0, sizeof(*tr));
        tr->n = 1;
        int n = MP3D_HTAB_ROWLEN[t];
        for (int x = 0; x < n; x++)
            for (int y = 0; y < n; y++)
                orc_tree_add(tr, MP3D_HTAB_CODES[t][x * n + y], MP3D_HTAB_LENS[t][x * n + y], x * 16 + y);
    }
    orc_tree *q = &g_trees[MP3D_NUM_HTABS];
    memset(q, 0, sizeof(*q));
    q->n = 1;
    for (int v = 0; v < 16; v++) orc_tree_add(q, MP3D_QUAD_CODE[0][v], MP3D_QUAD_LEN[0][v], v);
    for (int i = 0; i < 8207 + 16; i++) g_pow43[i] = pow((double)i, 4.0 / 3.0);
    /* ISO 2.4.3.4 IMDCT kernels and windows */
    for (int i = 0; i < 36; i++)
        for (int k = 0; k < 18; k++) g_imdct36[k][i] = cos(M_PI / 72.0 * (2 * i + 19) * (2 * k + 1));
    for (int i = 0; i < 12; i++)
        for (int k = 0; k < 6; k++) g_imdct12[k][i] = cos(M_PI / 24.0 * (2 * i + 7) * (2 * k + 1));
    for (int i = 0; i < 36; i++) {
        g_win[0][i] = sin(M_PI / 36.0 * (i + 0.5));
        g_win[1][i] = i < 18 ? sin(M_PI / 36.0 * (i + 0.5))
                    : i < 24 ? 1.0
                    : i < 30 ? sin(M_PI / 12.0 * (i - 18 + 0.5)) : 0.0;
        g_win[3][i] = i < 6 ? 0.0
                    : i < 12 ? sin(M_PI / 12.0 * (i - 6 + 0.5))
                    : i < 18 ? 1.0 : sin(M_PI / 36.0 * (i + 0.5));
        g_win[2][i] = i < 12 ? sin(M_PI / 12.0 * (i + 0.5)) : 0.0;
    }
    /* ISO Annex A synthesis: N[i][k] = cos((16+i)(2k+1)pi/64); window D. */
    for (int i = 0; i < 64; i++)
        for (int k = 0; k < 32; k++) g_synthN[i][k] = cos((16 + i) * (2 * k + 1) * M_PI / 64.0);
    for (int i = 0; i <= 256; i++) {
        double v = MP3D_SYNTH_WINDOW_Q16[i] / 65536.0;
        g_D[i] = v;
        if (i > 0) g_D[512 - i] = (i % 64) ? -v : v;
    }
    g_trees_ready = 1;
}

static int orc_tree_decode(const orc_tree *t, orc_bits *b) {
    int node = 0;
    for (int depth = 0; depth < 24; depth++) {
        int c = t->child[orc_get1(b)][node];
        if (c <= 0) return -c;
        node = c;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Decoder state.                                   */
/* ------------------------------------------------------------------------ */
#define ORC_HIST 4096
typedef struct {
    uint8_t hist[ORC_HIST]; /* main-data byte history (previous payloads) */
    int hist_len;           /* bytes in hist                              */
    int avail;              /* bytes after the previous main-data end     */
    orc_real overlap[2][32][18];
    orc_real V[2][1024];
    /* taps of the last decoded frame (parity taps) */
    int16_t is[2][2][576];
    uint8_t sf[2][2][40];
    int32_t used_bits[2][2]; /* bits actually consumed by part2+part3 */
    orc_real xr[2][2][576]; /* after stereo, before reorder (config-2 input) */
    orc_side side;
    orc_hdr hdr;
    int frames;
    int opts; /* ORC_OPT_* (orc_set_options) */
} orc_dec;

/* Option: verify the CRC-16 of protected frames; a mismatch drops the
 * frame (FFmpeg with err_detect = crccheck + explode; its default -- and so
 * the golden decoder's -- ignores the CRC). */
#define ORC_OPT_CRC_CHECK 1

typedef struct {
    int frame_bytes, channels, hz, layer, bitrate_kbps;
} orc_info;

ORC_API orc_dec *orc_create(void) {
    orc_init_tables();
    return (orc_dec *)calloc(1, sizeof(orc_dec));
}
ORC_API void orc_destroy(orc_dec *d) { free(d); }
ORC_API void orc_reset(orc_dec *d) {
    const int opts = d->opts;
    memset(d, 0, sizeof(*d));
    d->opts = opts;
}
ORC_API void orc_set_options(orc_dec *d, int opts) { d->opts = opts; }

/* CRC-16 of a protected frame (ISO 11172-3 2.4.3.1; FFmpeg handle_crc with
 * AV_CRC_16_ANSI: polynomial 0x8005, MSB first, initial 0xFFFF) over header
 * bytes 2..3 and the side info, checked against the stored bytes 4..5. */
static int orc_crc_ok(const uint8_t *buf, int side_bytes) {
    unsigned crc = 0xFFFF;
    for (int i = 2; i < 6 + side_bytes; i++) {
        if (i == 4) i = 6; /* the stored CRC itself is not covered */
        for (int k = 7; k >= 0; k--) {
            const unsigned bit = ((buf[i] >> k) & 1u) ^ ((crc >> 15) & 1u);
            crc = (crc << 1) & 0xFFFFu;
            if (bit) crc ^= 0x8005u;
        }
    }
    return crc == (((unsigned)buf[4] << 8) | buf[5]);
}
ORC_API int orc_state_bytes(void) { return (int)sizeof(orc_dec); }

/* ------------------------------------------------------------------------ */
/* Scalefactors (part 2), ISO 2.4.2.7; FFmpeg array layout:                  */
/*   long:  sf[0..20] bands 0..20, sf[21] = 0                                 */
/*   short: sf[3*b + w], b = 0..11 (+3 zeros for band 12)                     */
/*   mixed: sf[0..7] long bands 0..7, then sf[8 + 3*(b-3) + w], b = 3..11     */
/* ------------------------------------------------------------------------ */
/* FFmpeg lsf_sf_expand */
static void orc_lsf_expand(int *slen, int sf, int n1, int n2, int n3) {
    if (n3) { slen[3] = sf % n3; sf /= n3; } else slen[3] = 0;
    if (n2) { slen[2] = sf % n2; sf /= n2; } else slen[2] = 0;
    slen[1] = sf % n1;
    slen[0] = sf / n1;
}

/* LSF scalefactors (13818-3 2.4.3.2, FFmpeg mp_decode_layer3): slen[4] and
 * nr_of_sfb from the 9-bit scalefac_compress (intensity right channel: its
 * half, other tables); preflag = scalefac_compress >= 500.  Read in coding
 * order, stored in the canonical layout (mixed: short bands from sf[8]). */
static void orc_read_scalefactors_lsf(orc_bits *b, orc_gr *g, uint8_t *sf) {
    int slen[4], t2, sfc = g->scalefac_compress;
    const int tindex = g->window_switching && g->block_type == 2 ? (g->mixed ? 2 : 1) : 0;
    if (g->is_right) {
        sfc >>= 1;
        if (sfc < 180) { orc_lsf_expand(slen, sfc, 6, 6, 0); t2 = 3; }
        else if (sfc < 244) { orc_lsf_expand(slen, sfc - 180, 4, 4, 0); t2 = 4; }
        else { orc_lsf_expand(slen, sfc - 244, 3, 0, 0); t2 = 5; }
    } else {
        if (sfc < 400) { orc_lsf_expand(slen, sfc, 5, 4, 4); t2 = 0; }
        else if (sfc < 500) { orc_lsf_expand(slen, sfc - 400, 5, 4, 0); t2 = 1; }
        else { orc_lsf_expand(slen, sfc - 500, 3, 0, 0); t2 = 2; g->preflag = 1; }
    }
    memset(sf, 0, 40);
    int j = 0;
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < MP3D_LSF_NSF[t2][tindex][k]; i++, j++)
            sf[tindex == 2 && j >= 6 ? j + 2 : j] = (uint8_t)orc_get(b, slen[k]);
}

static void orc_read_scalefactors(orc_bits *b, orc_gr *g, const uint8_t *sf_gr0, uint8_t *sf) {
    if (g->lsf) {
        orc_read_scalefactors_lsf(b, g, sf);
        return;
    }
    int slen1 = MP3D_SLEN[0][g->scalefac_compress], slen2 = MP3D_SLEN[1][g->scalefac_compress];
    memset(sf, 0, 40);
    int j = 0;
    if (g->window_switching && g->block_type == 2) {
        int n = g->mixed ? 17 : 18;
        for (int i = 0; i < n; i++) sf[j++] = (uint8_t)orc_get(b, slen1);
        for (int i = 0; i < 18; i++) sf[j++] = (uint8_t)orc_get(b, slen2);
    } else {
        for (int k = 0; k < 4; k++) {
            int n = k == 0 ? 6 : 5;
            if (g->scfsi & (8 >> k)) {
                for (int i = 0; i < n; i++, j++) sf[j] = sf_gr0[j];
            } else {
                int slen = k < 2 ? slen1 : slen2;
                for (int i = 0; i < n; i++) sf[j++] = (uint8_t)orc_get(b, slen);
            }
        }
    }
}

/* Huffman decode of part 3, ISO 2.4.2.7 + Annex B; FFmpeg conventions:
 * a count1 quadruple crossing part2_3 end is discarded. */
static long orc_huffman(orc_bits *b, const orc_gr *g, int sr_idx, long end_bit, int16_t *is) {
    memset(is, 0, 576 * sizeof(int16_t));
    int bv2 = g->big_values * 2;
    int r1, r2; /* region ends (lines) */
    if (g->window_switching) {
        /* FFmpeg: 36 lines; LSF long-type units 54 (not at 8 kHz); short
         * units at MPEG-2.5 8 kHz 72 */
        if (g->block_type == 2) r1 = sr_idx == 8 ? 72 : 36;
        else r1 = sr_idx <= 2 ? 36 : sr_idx == 8 ? 108 : 54;
        r2 = 576;
    } else {
        int b1 = g->region0_count + 1, b2 = g->region0_count + g->region1_count + 2;
        if (b2 > 22) b2 = 22;
        r1 = 0;
        for (int i = 0; i < b1 && i < 22; i++) r1 += MP3D_SFB_LONG_WIDTH[sr_idx][i];
        r2 = 0;
        for (int i = 0; i < b2; i++) r2 += MP3D_SFB_LONG_WIDTH[sr_idx][i];
    }
    if (r1 > bv2) r1 = bv2;
    if (r2 > bv2) r2 = bv2;
    int k = 0;
    for (int region = 0; region < 3; region++) {
        int end = region == 0 ? r1 : region == 1 ? r2 : bv2;
        int sel = g->table_select[region];
        int tab = MP3D_HTAB_OF_SELECT[sel];
        int linbits = MP3D_LINBITS[sel];
        for (; k < end; k += 2) {
            /* FFmpeg huffman_decode: no pair starts at or past the unit's
             * part2_3 end (the rest of the unit reads as zeros) */
            if (b->pos >= end_bit) break;
            int x = 0, y = 0;
            if (tab >= 0) {
                int v = orc_tree_decode(&g_trees[tab], b);
                x = v >> 4;
                y = v & 15;
            }
            if (linbits && x == 15) x += (int)orc_get(b, linbits);
            if (x && orc_get1(b)) x = -x;
            if (linbits && y == 15) y += (int)orc_get(b, linbits);
            if (y && orc_get1(b)) y = -y;
            is[k] = (int16_t)x;
            is[k + 1] = (int16_t)y;
        }
    }
    /* count1 region */
    while (k <= 572) {
        long pos = b->pos;
        if (pos >= end_bit) break;
        int v;
        if (g->count1table_select) v = 15 - (int)orc_get(b, 4);
        else v = orc_tree_decode(&g_trees[MP3D_NUM_HTABS], b);
        int q[4] = {(v >> 3) & 1, (v >> 2) & 1, (v >> 1) & 1, v & 1};
        for (int i = 0; i < 4; i++)
            if (q[i] && orc_get1(b)) q[i] = -q[i];
        if (b->pos > end_bit) { /* overread: discard this quadruple */
            b->pos = pos;
            break;
        }
        for (int i = 0; i < 4; i++) is[k + i] = (int16_t)q[i];
        k += 4;
    }
    long consumed_end = b->pos;
    b->pos = end_bit;
    return consumed_end;
}

/* Requantise, ISO 2.4.3.4: xr = sgn(is)|is|^(4/3) 2^(q/4) with quarter
 * exponent q per line (FFmpeg exponents_from_scale_factors layout). */
/* FFmpeg's golden decoder is the fixed-point one: a requantised line whose
 * fixed-point value rounds to 0 IS zero there, and compute_stereo's "band of
 * the right channel holds a nonzero line" test (the intensity boundary) sees
 * it as zero.  Its line value is llrint(|is|^(4/3) 2^(q/4) 2^28 / 1.759)
 * (expval / table_4_3 scale: 2^(FRAC_BITS + 5) over IMDCT_SCALAR), so a line
 * is zero below |xr| = 0.5 * 1.759 * 2^-28.  Pinned by the FFmpeg fixtures
 * scale_msis_mixed_32k and probe_flush_* to (1.395, 2.0] * 2^-29
 * (tests/test_oracle.py::test_flush_threshold_pinned); below 2^-28 of full
 * scale the flush itself changes no PCM sample. */
#define ORC_FFMPEG_FLUSH (0.5 * 1.759 / 268435456.0)
static double g_orc_flush = ORC_FFMPEG_FLUSH;
/* test hook: move the threshold (0 = float decoder, no flush) */
ORC_API void orc_set_flush(double t) { g_orc_flush = t < 0 ? ORC_FFMPEG_FLUSH : t; }
static void orc_requant(const orc_gr *g, int sr_idx, const uint8_t *sf, const int16_t *is, orc_real *xr,
                        int gain_adj) {
    int gain = g->global_gain - 210 + gain_adj;
    int shift = g->scalefac_scale + 1;
    int long_end, short_start;
    if (g->window_switching && g->block_type == 2) {
        long_end = g->mixed ? (g->lsf ? 6 : 8) : 0; /* FFmpeg: 6 long bands in LSF mixed blocks */
        short_start = g->mixed ? 3 : 0;
    } else {
        long_end = 22;
        short_start = 13;
    }
    int line = 0, j = 0;
    for (int i = 0; i < long_end; i++) {
        int pre = g->preflag ? MP3D_PRETAB[i] : 0;
        int q = gain - ((sf[j++] + pre) << shift);
        orc_real s = pow(2.0, 0.25 * q);
        for (int n = 0; n < MP3D_SFB_LONG_WIDTH[sr_idx][i]; n++, line++) {
            int v = is[line];
            xr[line] = v == 0 ? 0.0 : (v < 0 ? -g_pow43[-v] : g_pow43[v]) * s;
            if (fabs(xr[line]) < g_orc_flush) xr[line] = 0.0;
        }
    }
    if (g->mixed && long_end < 22) j = 8; /* canonical layout: short bands from sf[8] */
    for (int i = short_start; i < 13 && long_end < 22; i++) {
        for (int w = 0; w < 3; w++) {
            int q = gain - (g->subblock_gain[w] << 3) - (sf[j++] << shift);
            orc_real s = pow(2.0, 0.25 * q);
            for (int n = 0; n < MP3D_SFB_SHORT_WIDTH[sr_idx][i]; n++, line++) {
                int v = is[line];
                xr[line] = v == 0 ? 0.0 : (v < 0 ? -g_pow43[-v] : g_pow43[v]) * s;
                if (fabs(xr[line]) < g_orc_flush) xr[line] = 0.0;
            }
        }
    }
}

/* Joint stereo, ISO 2.4.3.4 (M/S and MPEG-1 intensity), in bitstream
 * (pre-reorder) order, walking bands from the top as FFmpeg compute_stereo. */
/* Intensity ratios of one is_pos: MPEG-1 tan(is_pos pi / 12) (legal below 7);
 * LSF (13818-3 2.4.3.2, FFmpeg is_table_lsf) i0 = 2^(-1/4) (scalefac_compress
 * bit 0 = 0) or 2^(-1/2): odd is_pos -> (i0^((is_pos + 1) / 2), 1), even ->
 * (1, i0^(is_pos / 2)); FFmpeg treats is_pos >= 16 as "no intensity". */
static int orc_is_ratio(const orc_gr *g1, int p, orc_real *v1, orc_real *v2) {
    if (!g1->lsf) {
        if (p >= 7) return 0;
        double t = tan(p * M_PI / 12.0);
        *v1 = t / (1.0 + t);
        *v2 = 1.0 / (1.0 + t);
        return 1;
    }
    if (p >= 16) return 0;
    const int j = g1->scalefac_compress & 1;
    const double f = pow(2.0, -(j + 1) * ((p + 1) >> 1) / 4.0);
    *v1 = (p & 1) ? f : 1.0;
    *v2 = (p & 1) ? 1.0 : f;
    return 1;
}

static void orc_stereo(const orc_gr *g1, int sr_idx, int mode_ext, const uint8_t *sf1, orc_real *l, orc_real *r) {
    const orc_real isq = 1.0 / sqrt(2.0);
    if (!(mode_ext & 1)) {
        if (mode_ext & 2)
            for (int i = 0; i < 576; i++) {
                orc_real m = l[i], s = r[i];
                l[i] = (m + s) * isq;
                r[i] = (m - s) * isq;
            }
        return;
    }
    int long_end, short_start;
    if (g1->window_switching && g1->block_type == 2) {
        long_end = g1->mixed ? (g1->lsf ? 6 : 8) : 0;
        short_start = g1->mixed ? 3 : 0;
    } else {
        long_end = 22;
        short_start = 13;
    }
    int pos = 576;
    int nz_short[3] = {0, 0, 0};
    /* FFmpeg's index walk; sf1 is in the canonical layout, where a mixed
     * block's short bands start at 8 whatever its long_end */
    int k = (13 - short_start) * 3 + (g1->mixed && long_end < 22 ? 8 : long_end) - 3;
    for (int i = 12; i >= short_start; i--) {
        if (i != 11) k -= 3;
        int len = MP3D_SFB_SHORT_WIDTH[sr_idx][i];
        for (int w = 2; w >= 0; w--) {
            pos -= len;
            int do_is = 0;
            orc_real v1 = 0, v2 = 0;
            if (!nz_short[w]) {
                for (int j = 0; j < len; j++)
                    if (r[pos + j] != 0.0) { nz_short[w] = 1; break; }
                if (!nz_short[w]) do_is = orc_is_ratio(g1, sf1[k + w], &v1, &v2);
            }
            if (do_is) {
                for (int j = 0; j < len; j++) {
                    orc_real x = l[pos + j];
                    l[pos + j] = x * v1;
                    r[pos + j] = x * v2;
                }
            } else if (mode_ext & 2) {
                for (int j = 0; j < len; j++) {
                    orc_real m = l[pos + j], s = r[pos + j];
                    l[pos + j] = (m + s) * isq;
                    r[pos + j] = (m - s) * isq;
                }
            }
        }
    }
    int nz = nz_short[0] | nz_short[1] | nz_short[2];
    for (int i = long_end - 1; i >= 0; i--) {
        int len = MP3D_SFB_LONG_WIDTH[sr_idx][i];
        pos -= len;
        int do_is = 0;
        orc_real v1 = 0, v2 = 0;
        if (!nz) {
            for (int j = 0; j < len; j++)
                if (r[pos + j] != 0.0) { nz = 1; break; }
            int kk = i == 21 ? 20 : i;
            if (!nz) do_is = orc_is_ratio(g1, sf1[kk], &v1, &v2);
        }
        if (do_is) {
            for (int j = 0; j < len; j++) {
                orc_real x = l[pos + j];
                l[pos + j] = x * v1;
                r[pos + j] = x * v2;
            }
        } else if (mode_ext & 2) {
            for (int j = 0; j < len; j++) {
                orc_real m = l[pos + j], s = r[pos + j];
                l[pos + j] = (m + s) * isq;
                r[pos + j] = (m - s) * isq;
            }
        }
    }
}

/* Short-block reorder (ISO 2.4.3.4): window-grouped bands -> (freq, window)
 * interleave, so line 3f+w holds window w's frequency f of the band. */
static void orc_reorder(int block_type, int mixed, int sr_idx, orc_real *xr) {
    if (block_type != 2) return;
    orc_real tmp[576];
    int start = mixed ? (sr_idx == 8 ? 72 : 36) : 0, b0 = mixed ? 3 : 0; /* FFmpeg reorder_block */
    int p = start;
    for (int i = b0; i < 13; i++) {
        int len = MP3D_SFB_SHORT_WIDTH[sr_idx][i];
        for (int f = 0; f < len; f++)
            for (int w = 0; w < 3; w++) tmp[3 * f + w] = xr[p + w * len + f];
        memcpy(xr + p, tmp, sizeof(orc_real) * 3 * len);
        p += 3 * len;
    }
}

/* Alias reduction, ISO 2.4.3.4 with Annex B Table B.9 coefficients. */
static void orc_alias(int block_type, int mixed, orc_real *xr) {
    int nsb = block_type == 2 ? (mixed ? 1 : 0) : 31;
    for (int sb = 1; sb <= nsb; sb++)
        for (int i = 0; i < 8; i++) {
            orc_real c = MP3D_ALIAS_C[i], den = sqrt(1.0 + c * c);
            orc_real cs = 1.0 / den, ca = c / den;
            orc_real bu = xr[18 * sb - 1 - i], bd = xr[18 * sb + i];
            xr[18 * sb - 1 - i] = bu * cs - bd * ca;
            xr[18 * sb + i] = bd * cs + bu * ca;
        }
}

/* IMDCT + windowing + overlap-add + frequency inversion (ISO 2.4.3.4).
 * out[slot][sb], slot 0..17. */
static void orc_imdct(int block_type, int mixed, const orc_real *xr, orc_real ov[32][18], orc_real out[18][32]) {
    for (int sb = 0; sb < 32; sb++) {
        orc_real z[36];
        const orc_real *X = xr + 18 * sb;
        int bt = (mixed && block_type == 2 && sb < 2) ? 0 : block_type;
        if (bt != 2) {
            for (int i = 0; i < 36; i++) {
                orc_real acc = 0;
                for (int k = 0; k < 18; k++) acc += X[k] * g_imdct36[k][i];
                z[i] = acc * g_win[bt][i];
            }
        } else {
            memset(z, 0, sizeof(z));
            for (int w = 0; w < 3; w++)
                for (int i = 0; i < 12; i++) {
                    orc_real acc = 0;
                    for (int k = 0; k < 6; k++) acc += X[3 * k + w] * g_imdct12[k][i];
                    z[6 * w + 6 + i] += acc * g_win[2][i];
                }
        }
        for (int i = 0; i < 18; i++) {
            orc_real v = z[i] + ov[sb][i];
            ov[sb][i] = z[i + 18];
            if ((sb & 1) && (i & 1)) v = -v;
            out[i][sb] = v;
        }
    }
}

/* Polyphase synthesis filterbank, ISO Annex A flowchart (direct form). */
static void orc_synth(orc_real V[1024], const orc_real S[32], orc_real *pcm32) {
    memmove(V + 64, V, sizeof(orc_real) * (1024 - 64));
    for (int i = 0; i < 64; i++) {
        orc_real acc = 0;
        for (int k = 0; k < 32; k++) acc += g_synthN[i][k] * S[k];
        V[i] = acc;
    }
    orc_real U[512];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 32; j++) {
            U[i * 64 + j] = V[i * 128 + j];
            U[i * 64 + 32 + j] = V[i * 128 + 96 + j];
        }
    for (int j = 0; j < 32; j++) {
        orc_real acc = 0;
        for (int i = 0; i < 16; i++) acc += U[j + 32 * i] * g_D[j + 32 * i];
        pcm32[j] = acc;
    }
}

/* Stages a8..a10 for one granule of one channel (xr in bitstream order). */
static void orc_granule_to_pcm(orc_dec *d, int ch, int block_type, int mixed, int sr_idx, orc_real *xr, orc_real *pcm576) {
    orc_real out[18][32];
    orc_reorder(block_type, mixed, sr_idx, xr);
    orc_alias(block_type, mixed, xr);
    orc_imdct(block_type, mixed, xr, d->overlap[ch], out);
    for (int s = 0; s < 18; s++) orc_synth(d->V[ch], out[s], pcm576 + 32 * s);
}

/* ------------------------------------------------------------------------ */
/* One frame.  buf points at the sync word; bytes >= frame length.           */
/* pcm: planar double [2][1152] (may be NULL).  Returns samples/channel     */
/* (1152, or 576 for LSF), 0 for a frame that produced no audio, <0 on     */
/* error.                                                                   */
/* ------------------------------------------------------------------------ */
ORC_API int orc_decode_frame_f64(orc_dec *d, const uint8_t *buf, int bytes, double *pcm, orc_info *info) {
    orc_hdr h;
    int fb = orc_parse_header(buf, &h);
    if (fb < 0) return -1;
    if (fb > bytes) return -2;
    if (info) {
        info->frame_bytes = fb;
        info->channels = h.nch;
        info->hz = h.hz;
        info->layer = 3;
        info->bitrate_kbps = h.kbps;
    }
    d->hdr = h;
    const uint8_t *side = buf + 4 + h.crc_bytes;
    orc_side *s = &d->side;
    orc_parse_side(side, &h, s);
    const int crc_bad = (d->opts & ORC_OPT_CRC_CHECK) && h.crc_bytes && !orc_crc_ok(buf, h.side_bytes);
    for (int gr = 0; gr < h.ngr; gr++)
        for (int ch = 0; ch < h.nch; ch++)
            if (crc_bad || s->gr[gr][ch].big_values > 288 ||
                (s->gr[gr][ch].window_switching && s->gr[gr][ch].block_type == 0)) {
                /* dropped (FFmpeg mp_decode_layer3 rejects
                 * big_values > 288 and the reserved block_type 0 under window
                 * switching, tests/golden edge_bt0_drop); mp_decode_frame then keeps
                 * the frame's last min(BACKSTEP_SIZE = 512, bytes - 4) post-
                 * header bytes as the whole reservoir */
                int keep = fb - 4 < 512 ? fb - 4 : 512;
                memcpy(d->hist, buf + fb - keep, (size_t)keep);
                d->hist_len = keep;
                d->avail = keep;
                return -3;
            }
    const uint8_t *payload = side + h.side_bytes;
    int plen = fb - 4 - h.crc_bytes - h.side_bytes;
    if (plen < 0) return -4;

    /* main-data buffer = history + payload (bit reservoir, ISO 2.4.3.4) */
    static __thread uint8_t mdbuf[ORC_HIST + 2048];
    int H = d->hist_len;
    memcpy(mdbuf, d->hist, (size_t)H);
    memcpy(mdbuf + H, payload, (size_t)plen);
    orc_bits b = {mdbuf, (long)(H + plen) * 8, 0};
    int mdb = s->main_data_begin;
    int gr0 = 0;
    long start_bit;
    int avail = d->avail < H ? d->avail : H;
    if (mdb <= avail) {
        start_bit = (long)(H - mdb) * 8;
    } else {
        /* reservoir underflow: FFmpeg skips whole granules until the missing
         * bytes are covered (mp_decode_layer3), zero spectra meanwhile. */
        long bits = (long)avail * 8;
        while (gr0 < h.ngr && (bits >> 3) < mdb) {
            for (int ch = 0; ch < h.nch; ch++) bits += s->gr[gr0][ch].part2_3_length;
            gr0++;
        }
        start_bit = (long)(H - avail) * 8 + bits - 8L * mdb;
    }
    b.pos = start_bit;

    orc_real pcm_local[2][1152];
    memset(d->is, 0, sizeof(d->is));
    memset(d->sf, 0, sizeof(d->sf));
    memset(d->xr, 0, sizeof(d->xr));
    memset(d->used_bits, 0, sizeof(d->used_bits));
    int ms_only = h.mode == 1 && (h.mode_ext & 2) && !(h.mode_ext & 1);
    (void)ms_only;
    for (int gr = 0; gr < h.ngr; gr++) {
        for (int ch = 0; ch < h.nch; ch++) {
            orc_gr *g = &s->gr[gr][ch];
            if (gr < gr0) {
                memset(d->xr[gr][ch], 0, sizeof(d->xr[gr][ch]));
                continue;
            }
            long p2 = b.pos;
            orc_read_scalefactors(&b, g, d->sf[0][ch], d->sf[gr][ch]);
            d->used_bits[gr][ch] = (int32_t)(orc_huffman(&b, g, h.sr_idx, p2 + g->part2_3_length, d->is[gr][ch]) - p2);
            orc_requant(g, h.sr_idx, d->sf[gr][ch], d->is[gr][ch], d->xr[gr][ch], 0);
        }
        if (h.mode == 1 && h.nch == 2 && gr >= gr0)
            orc_stereo(&s->gr[gr][1], h.sr_idx, h.mode_ext, d->sf[gr][1], d->xr[gr][0], d->xr[gr][1]);
        for (int ch = 0; ch < h.nch; ch++) {
            orc_gr *g = &s->gr[gr][ch];
            int bt = g->window_switching ? g->block_type : 0;
            int mx = g->window_switching && g->block_type == 2 ? g->mixed : 0;
            orc_real xr[576];
            memcpy(xr, d->xr[gr][ch], sizeof(xr));
            if (gr < gr0) bt = 0, mx = 0;
            orc_granule_to_pcm(d, ch, bt, mx, h.sr_idx, xr, &pcm_local[ch][576 * gr]);
        }
    }
    /* bytes after this frame's main-data end become the next reservoir */
    long end_bit = b.pos;
    long end_byte = (end_bit + 7) >> 3;
    int total = H + plen;
    int after = total - (int)end_byte;
    if (after < 0) after = 0;
    d->avail = after;
    /* keep the last ORC_HIST bytes of history */
    if (total > ORC_HIST) {
        memcpy(d->hist, mdbuf + total - ORC_HIST, ORC_HIST);
        d->hist_len = ORC_HIST;
    } else {
        memcpy(d->hist, mdbuf, (size_t)total);
        d->hist_len = total;
    }
    if (pcm) {
        for (int ch = 0; ch < h.nch; ch++)
            for (int i = 0; i < 576 * h.ngr; i++) pcm[1152 * ch + i] = pcm_local[ch][i];
    }
    d->frames++;
    return 576 * h.ngr;
}

/* float32 planar output convenience wrapper */
ORC_API int orc_decode_frame(orc_dec *d, const uint8_t *buf, int bytes, float *pcm, orc_info *info) {
    double tmp[2][1152];
    int r = orc_decode_frame_f64(d, buf, bytes, (double *)tmp, info);
    if (r > 0 && pcm) {
        int nch = d->hdr.nch;
        for (int ch = 0; ch < nch; ch++)
            for (int i = 0; i < r; i++) pcm[1152 * ch + i] = (float)tmp[ch][i];
    }
    return r;
}

ORC_API void orc_get_taps(const orc_dec *d, int16_t *is /*[2][2][576]*/, uint8_t *sf /*[2][2][40]*/,
                          float *xr /*[2][2][576]*/, int32_t *side /*[2][2][20]*/) {
    if (is) memcpy(is, d->is, sizeof(d->is));
    if (sf) memcpy(sf, d->sf, sizeof(d->sf));
    if (xr)
        for (int i = 0; i < 2 * 2 * 576; i++) xr[i] = (float)((const orc_real *)d->xr)[i];
    if (side) {
        memset(side, 0, sizeof(int32_t) * 2 * 2 * 20);
        for (int gr = 0; gr < d->hdr.ngr; gr++)
            for (int ch = 0; ch < 2; ch++) {
                const orc_gr *g = &d->side.gr[gr][ch];
                int32_t *o = side + (gr * 2 + ch) * 20;
                o[0] = g->part2_3_length; o[1] = g->big_values; o[2] = g->global_gain;
                o[3] = g->scalefac_compress; o[4] = g->window_switching; o[5] = g->block_type;
                o[6] = g->mixed; o[7] = g->table_select[0]; o[8] = g->table_select[1];
                o[9] = g->table_select[2]; o[10] = g->region0_count; o[11] = g->region1_count;
                o[12] = g->preflag; o[13] = g->scalefac_scale; o[14] = g->count1table_select;
                o[15] = d->side.main_data_begin;
                o[16] = d->used_bits[gr][ch];
                o[17] = g->subblock_gain[0]; o[18] = g->subblock_gain[1]; o[19] = g->subblock_gain[2];
            }
    }
}

/* ------------------------------------------------------------------------ */
/* Stream helpers: ID3v2 skip, Xing/Info detection.     */
/* ------------------------------------------------------------------------ */
ORC_API long orc_skip_id3v2(const uint8_t *buf, long len) {
    if (len >= 10 && buf[0] == 'I' && buf[1] == 'D' && buf[2] == '3') {
        long sz = ((long)(buf[6] & 0x7F) << 21) | ((long)(buf[7] & 0x7F) << 14) | ((buf[8] & 0x7F) << 7) | (buf[9] & 0x7F);
        return 10 + sz + ((buf[5] & 0x10) ? 10 : 0);
    }
    return 0;
}

/* 1 if the frame at buf is a Xing/Info tag frame (no audio). */
ORC_API int orc_is_info_frame(const uint8_t *buf, long len) {
    orc_hdr h;
    int fb = orc_parse_header(buf, &h);
    if (fb < 0 || fb > len) return 0;
    const uint8_t *t = buf + 4 + h.crc_bytes + h.side_bytes;
    return (!memcmp(t, "Xing", 4) || !memcmp(t, "Info", 4));
}

/* Gapless info of a stream's leading Xing/Info frame, restating FFmpeg's
 * demuxer (libavformat/mp3dec.c mp3_parse_info_tag, the FFmpeg inside the
 * golden decoder): "Xing"/"Info" at 4 + side-info bytes,
 * BE32 flags, [frames] [bytes] [100-B TOC] [quality], 9-byte encoder
 * string, then 12 bytes on a BE24 delay << 12 | padding, honoured for LAME
 * / Lavf / Lavc.  out[0..5] = has_lame, enc_delay, enc_padding, frames
 * (-1 absent), skip_samples (delay + 529), samples per frame (1152 / 576
 * LSF).  Returns 1 if a tag was found. */
ORC_API int orc_parse_info_tag(const uint8_t *buf, long len, int *out) {
    long pos = orc_skip_id3v2(buf, len);
    out[0] = out[1] = out[2] = out[4] = 0;
    out[5] = 1152;
    out[3] = -1;
    while (pos + 4 <= len) {
        orc_hdr h;
        if (orc_parse_header(buf + pos, &h) > 0) break;
        pos++;
    }
    if (pos + 4 > len || !orc_is_info_frame(buf + pos, len - pos)) return 0;
    orc_hdr h;
    const int fb = orc_parse_header(buf + pos, &h);
    out[5] = 576 * h.ngr;
    const uint8_t *t = buf + pos + 4 + h.crc_bytes + h.side_bytes;
    const long n = fb - (4 + h.crc_bytes + h.side_bytes);
#define BE32(o) ((uint32_t)t[o] << 24 | (uint32_t)t[(o) + 1] << 16 | (uint32_t)t[(o) + 2] << 8 | t[(o) + 3])
    const uint32_t flags = BE32(4);
    long o = 8;
    if (flags & 1) { out[3] = (int)BE32(o); o += 4; }
    if (flags & 2) o += 4;
    if (flags & 4) o += 100;
    if (flags & 8) o += 4;
    if (o + 24 <= n && (!memcmp(t + o, "LAME", 4) || !memcmp(t + o, "Lavf", 4) || !memcmp(t + o, "Lavc", 4))) {
        const uint32_t v = (uint32_t)t[o + 21] << 16 | (uint32_t)t[o + 22] << 8 | t[o + 23];
        out[0] = 1;
        out[1] = (int)(v >> 12);
        out[2] = (int)(v & 4095);
        out[4] = out[1] + 529;
    }
#undef BE32
    return 1;
}

/* Decode a whole stream into planar float PCM [nch][max_frames*1152]
 * (frames packed back to back: 1152 samples per MPEG-1 frame, 576 per LSF
 * frame).  Skips an ID3v2 tag and a leading Xing/Info frame (as FFmpeg's
 * demuxer).  Returns audio frames decoded; *samples_out = samples per
 * channel written. */
ORC_API long orc_decode_stream_opts(const uint8_t *buf, long len, float *pcm, long max_frames, int *nch_out,
                                    int *hz_out, long *samples_out, int opts) {
    orc_dec *d = orc_create();
    d->opts = opts;
    long pos = orc_skip_id3v2(buf, len);
    long nf = 0, ns = 0;
    int first = 1;
    int nch = 0, hz = 0;
    float tmp[2][1152];
    while (pos + 4 <= len && nf < max_frames) {
        orc_hdr h;
        int fb = orc_parse_header(buf + pos, &h);
        if (fb < 0) { pos++; continue; }
        int r;
        orc_info info;
        if (pos + fb > len) {
            /* a final frame cut short: FFmpeg still decodes it, the missing
             * bytes reading as zeros */
            if (len - pos < 4 + h.crc_bytes + h.side_bytes) break;
            uint8_t *pad = (uint8_t *)calloc((size_t)fb, 1);
            memcpy(pad, buf + pos, (size_t)(len - pos));
            r = orc_decode_frame(d, pad, fb, &tmp[0][0], &info);
            free(pad);
            pos = len;
        } else {
            if (first && orc_is_info_frame(buf + pos, len - pos)) { pos += fb; first = 0; continue; }
            r = orc_decode_frame(d, buf + pos, fb, &tmp[0][0], &info);
            pos += fb;
        }
        first = 0;
        if (r <= 0) continue;
        nch = info.channels;
        hz = info.hz;
        for (int ch = 0; ch < nch; ch++) memcpy(pcm + (size_t)ch * max_frames * 1152 + ns, tmp[ch], sizeof(float) * r);
        ns += r;
        nf++;
    }
    if (nch_out) *nch_out = nch;
    if (hz_out) *hz_out = hz;
    if (samples_out) *samples_out = ns;
    orc_destroy(d);
    return nf;
}

ORC_API long orc_decode_stream_n(const uint8_t *buf, long len, float *pcm, long max_frames, int *nch_out, int *hz_out,
                                 long *samples_out) {
    return orc_decode_stream_opts(buf, len, pcm, max_frames, nch_out, hz_out, samples_out, 0);
}

ORC_API long orc_decode_stream(const uint8_t *buf, long len, float *pcm, long max_frames, int *nch_out, int *hz_out) {
    return orc_decode_stream_n(buf, len, pcm, max_frames, nch_out, hz_out, NULL);
}

/* ------------------------------------------------------------------------ */
/* Config-2 restatement: stages a8..a11 from synthetic spectra.              */
/* xr: [n_frames][2 gr][nch][576] f32 (after stereo, bitstream order);       */
/* block_type/mixed: [n_frames][2][nch]; pcm: int16 [n_frames][1152][nch]    */
/* ------------------------------------------------------------------------ */
ORC_API void orc_synth_only(orc_dec *d, const float *xr, const uint8_t *block_type, const uint8_t *mixed,
                            int n_frames, int nch, int sr_idx, int16_t *pcm, float *pcm_f32) {
    for (int f = 0; f < n_frames; f++)
        for (int gr = 0; gr < 2; gr++) {
            orc_real out[2][576];
            for (int ch = 0; ch < nch; ch++) {
                orc_real x[576];
                const float *src = xr + (((size_t)f * 2 + gr) * nch + ch) * 576;
                for (int i = 0; i < 576; i++) x[i] = src[i];
                int bt = block_type[(f * 2 + gr) * nch + ch], mx = mixed[(f * 2 + gr) * nch + ch];
                orc_granule_to_pcm(d, ch, bt, bt == 2 ? mx : 0, sr_idx, x, out[ch]);
            }
            for (int i = 0; i < 576; i++)
                for (int ch = 0; ch < nch; ch++) {
                    orc_real v = out[ch][i];
                    size_t o = ((size_t)f * 1152 + gr * 576 + i) * nch + ch;
                    if (pcm_f32) pcm_f32[o] = (float)v;
                    if (pcm) {
                        double r = nearbyint(v * 32768.0);
                        pcm[o] = (int16_t)(r > 32767 ? 32767 : r < -32768 ? -32768 : r);
                    }
                }
        }
}
