/*
 * mp3d_internal.h -- device data layout shared by the HIP kernels
 * (mp3d_demux.hip, mp3d_huffman.hip, mp3d_synth.hip) and the host library (mp3d_host.cpp).
 *
 * HBM layout of one batch (SoA, one process per GPU):
 *   input   : caller's frame bytes, stream s at in_off[s] (u64), in_len[s]
 *   rec     : FrameRec[n_streams * F]         (k_demux, 32 B per frame)
 *   md      : per-stream main-data byte region (carry-in + payloads),
 *             stream s at md_off[s] (16-B aligned), read as big-endian words
 *   is_buf  : int16 [n_streams * F * 4][MP3D_IS_ROW]  (k_huffman -> k_synth; 576 lines used)
 *   meta    : UnitMeta[n_streams * F * 4]    (scalefactors + gains)
 *   state   : StreamState[max_streams]        (reservoir, overlap, V FIFO)
 *   pcm     : int16 [n_streams * F][1152 * 2] (interleaved L/R; mono: 1152)
 * Unit index u = ((s * F + f) * 2 + gr) * 2 + ch.
 */
#ifndef MP3D_INTERNAL_H
#define MP3D_INTERNAL_H

#include <stdint.h>

#define MP3D_RES_BYTES 512       /* carried main-data history per stream   */
#define MP3D_FIFO_SLOTS 15       /* synthesis history slots carried        */
#define MP3D_MAX_FRAME_BYTES 1441
#ifndef MP3D_OPT_CRC_CHECK
#define MP3D_OPT_CRC_CHECK 1     /* = include/mp3d.h (the kernels do not include it) */
#endif
#define MP3D_TAG_SEEN (1u << 31)
#define MP3D_TAG_LAME (1u << 30)
#define MP3D_TAG_FRAMES (1u << 29)

/* MPEG-1 pretab (ISO Table B.6, MP3D_PRETAB in mp3d_tables.h) as 2 bits
 * per long band, for lane-indexed use without a memory load; checked
 * against the table when the device is initialised (mp3d_host.cpp). */
#define MP3D_PRETAB_BITS 0x2fe95400000ull

/* Per-frame record written by k_demux. */
struct FrameRec {
    uint64_t frame_off;  /* byte offset of the frame header in input        */
    uint32_t md_bit;     /* bit offset of main-data start inside md region   */
    uint32_t payload_md; /* byte offset of this frame's payload in md region */
    uint16_t frame_bytes;/* 0: no frame (stream ended / invalid)             */
    uint16_t payload_len;
    uint8_t hdr1, hdr2, hdr3; /* header bytes 1..3                           */
    uint8_t nch;
    uint8_t side_off;    /* 4 or 6 (CRC)                                     */
    uint8_t first_gr;    /* first decoded granule (reservoir underflow)      */
    uint8_t sr_idx;      /* 0..2 MPEG-1, 3..5 MPEG-2, 6..8 MPEG-2.5 (LSF)    */
    uint8_t lsf;         /* 1: MPEG-2 / 2.5 low sampling frequency frame,    */
                         /*    one granule (ISO 13818-3)                     */
    uint16_t payload_avail; /* payload bytes present (< payload_len: the final
                             * frame was cut short; the rest reads as zeros) */
};

/* Per-unit side information + scalefactors, written by k_huffman. */
struct __attribute__((aligned(8))) UnitMeta {
    uint8_t sf[40];
    uint8_t global_gain;
    uint8_t block_type;  /* 0 unless window switching                      */
    uint8_t mixed;
    uint8_t scalefac_scale;
    uint8_t preflag;
    uint8_t sbg[3];
    uint16_t nz_end;     /* lines produced by big_values + count1          */
    uint16_t part2_3_length;
    uint16_t used_bits;  /* bits consumed (== part2_3_length when valid)   */
    uint16_t flags;      /* bit 0: granule lost to a reservoir underflow;  */
                         /* bit 1: LSF intensity_scale (scalefac_compress  */
                         /* bit 0 of an intensity frame's right channel)   */
};

/* Persistent per-stream decoder state. */
struct StreamState {
    uint8_t res[MP3D_RES_BYTES];           /* main-data carry (oldest first) */
    int32_t res_len;                       /* bytes valid in res             */
    int32_t frames;                        /* frames decoded so far          */
    /* leading Xing/Info frame (k_demux; 0 = none seen): bit 31 tag, bit 30
     * LAME/Lavf/Lavc extension, bit 29 frame count present, bits 12..23
     * encoder delay, bits 0..11 encoder padding; tag_frames = Xing count */
    uint32_t tag_info;
    uint32_t tag_frames;
    /* MPEG version family, fixed by the stream's first frame (k_demux):
     * 0 none yet, 1 MPEG-1, 2 MPEG-2 / 2.5 LSF.  Headers of the other
     * family are skipped as junk; k_synth runs one variant per family. */
    int32_t kind;
    int32_t pad_[2];                       /* k_walk -> k_mdcopy: md end, next carry */
    /* state format stamp, MP3D_STATE_FMT in every handle's slots (written by
     * the host at create / reset, never by a kernel): set_state refuses a
     * blob without it, e.g. one saved by a build whose fifo meant raw X */
    uint32_t fmt;
    float overlap[2][32][18];              /* IMDCT overlap (true values)    */
    /* synthesis history as partial window sums (round 4): fifo[ch][t][j] =
     * the terms of the NEXT granule's output slot t (< 15) that read this
     * granule's matrixing outputs, in float-sink units (full scale 1.0):
     * the int16 variant scales by 2^-15 on the way out and 2^15 on the way
     * in (exact), so a stream may switch sinks between calls */
    float fifo[2][MP3D_FIFO_SLOTS][32];
};
/* 0x05 in every byte: one hipMemset2D per slot array; 5 = the format of
 * ABI v5 (fifo = partial sums in float units) */
/* int16 elements per unit row of is_buf (576 lines; a longer row only
 * pads: the A/B of row placement in the L2) */
#ifndef MP3D_IS_ROW
#define MP3D_IS_ROW 576
#endif
#define MP3D_STATE_FMT 0x05050505u
#define MP3D_STATE_FMT_BYTE 0x05

/* Huffman LUT layout (u16 entries, two levels, first level <= 8 bits):
 * leaf:    bit15 = 0, bits 8..12 code length, bits 4..7 x, bits 0..3 y,
 *          big_values tables: bit 13 x != 0, bit 14 y != 0 (sign bits)
 * pointer: bit15 = 1, bits 11..14 sub-index bits, bits 0..10 absolute
 *          sub-table index / 4 (sub-tables are 4-entry aligned)          */
#define MP3D_LUT_TABLES 16 /* 15 big_values code tables + count1 table A   */
#define MP3D_LUT_MAX 7168
struct HuffLutHeader {
    uint16_t base[MP3D_LUT_TABLES];
    uint8_t bits1[MP3D_LUT_TABLES];
};

/* Constant tables uploaded once per batch (built on the host). */
struct DevTables {
    float pow43[8208];         /* |is|^(4/3), |is| <= 8206               */
    float dct_c[32][32];       /* C[m][sb] = cos(m (2 sb + 1) pi / 64)  */
    float dwin[32][16];        /* per output j: signed window taps       */
    /* per (sample-rate index 0..8, block variant long / short / mixed, bitstream
     * line pair 2k, 2k + 1): bits 0..7 = 4 x scale index of the pair (long
     * band b, or 22 + 3 b + w for short band b window w; every band width is
     * even, so a pair never straddles two bands), bits 8..17 / 18..27 the
     * two lines' positions after the short reorder                       */
    uint32_t lpair[9][3][288];
    uint8_t win_a[32];         /* V[j] = sgn * X[a[j]]                   */
    uint8_t win_b[32];         /* V[32 + j] = sgn * X[b[j]]              */
    uint16_t lut[MP3D_LUT_MAX];  /* entries past the last table are 0: the    */
                                 /* zero table of table_select 0, 4, 14 at    */
                                 /* tsel's base for those selects             */
    struct HuffLutHeader lut_hdr;
    /* table_select -> LUT base | first-level bits << 16 | zero table << 20 |
     * linbits << 24, and
     * the long sfb start lines per sample-rate index (23 bounds): built on
     * the host so k_huffman's table staging is one load deep              */
    uint32_t tsel[32];
    uint16_t lbnd[9][24];
};

#endif
