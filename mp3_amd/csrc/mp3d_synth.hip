/*
 * mp3d_synth.hip -- k_synth (ISO 11172-3
 * 2.4.3.4 + Annex A, 13818-3 2.4.3.2): requantise, stereo, alias reduction,
 * IMDCT + overlap, polyphase synthesis (matrixing on the matrix cores) ->
 * int16 / float PCM; k_gather_frames for the frame-parallel long-stream
 * decode (§8(f) row 2); k_frame, the per-frame decoder's one-launch call.
 * Pipeline overview: mp3d_device.h.
 */
#include "mp3d_device.h"
#include "mp3d_consts.h" /* IMDCT-12 / short window / alias coefficients as literals */
/* the per-frame k_frame below runs the demux and Huffman stages too: this
 * translation unit's own copies of their device code and constants */
#define MP3D_DEMUX_TU frame_tu
#include "mp3d_demux_dev.h"
#include "mp3d_huffman_dev.h"

namespace mp3d {

/* ------------------------------------------------------------------------ */
/* Constant-memory tables (uniform access -> scalar loads)                   */
/* ------------------------------------------------------------------------ */
__constant__ float c_win36[4][36];     /* long windows x IMDCT output scale (imdct36_w)  */
__constant__ float c_is_ratio[7][2];   /* MPEG-1 intensity: k/(1+k), 1/(1+k)             */
__constant__ float c_pow2q[4];         /* 2^(i/4)                                        */
__constant__ float c_is_lsf[2][16][2]; /* LSF intensity [intensity_scale][is_pos]: L, R */

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


typedef float f32x2 __attribute__((ext_vector_type(2)));
template <bool V> struct BoolC { static constexpr bool value = V; }; /* a compile-time flag argument */
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 bc(float c) { return (f32x2){c, c}; }

/* dct3_9 on packed pairs: both 9-point DCT-IIIs of the fast IMDCT (the even
 * input in .x, the odd one in .y) in one pass of packed FP32 ops
 * (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: half the VALU issues); per
 * element the same operations in the same order as dct3_9, so bit-identical */
/* the packed constants (c, c) come from LDS (kc, a broadcast read per use):
 * as literals they take SGPR pairs, which the kernel does not have to spare
 * (spills) */
#define IMDCT36_K {5.019099188e-01f, 5.176380902e-01f, 5.516889595e-01f, 6.103872944e-01f, 7.071067812e-01f, \
                   8.717233978e-01f, 1.183100792e+00f, 1.931851653e+00f, 5.736856623e+00f}
#define DCT9_KC {9.848077530e-01f, 9.396926208e-01f, 8.660254038e-01f, 7.660444431e-01f, \
                 6.427876097e-01f, 3.420201433e-01f, 1.736481777e-01f}
__device__ __forceinline__ void dct3_9p(const f32x2 *a, f32x2 *v, const f32x2 *kc) {
    auto ld = [&](int i) { return ((const __attribute__((address_space(3))) f32x2 *)(uintptr_t)kc)[i]; };
    const f32x2 C10 = ld(0), C20 = ld(1), C30 = ld(2), C40 = ld(3), C50 = ld(4), C70 = ld(5), C80 = ld(6);
    const f32x2 ev0 = pfma(a[8], C80, pfma(a[6], bc(0.5f), pfma(a[4], C40, pfma(a[2], C20, a[0]))));
    const f32x2 od0 = pfma(a[7], C70, pfma(a[5], C50, pfma(a[3], C30, a[1] * C10)));
    v[0] = ev0 + od0;
    v[8] = ev0 - od0;
    const f32x2 ev1 = pfma(a[8], bc(-0.5f), (pfma(a[4], bc(-0.5f), pfma(a[2], bc(0.5f), a[0])) - a[6]));
    const f32x2 od1 = pfma(a[7], -C30, pfma(a[5], -C30, a[1] * C30));
    v[1] = ev1 + od1;
    v[7] = ev1 - od1;
    const f32x2 ev2 = pfma(a[8], C40, pfma(a[6], bc(0.5f), pfma(a[4], -C20, pfma(a[2], -C80, a[0]))));
    const f32x2 od2 = pfma(a[7], C10, pfma(a[5], -C70, pfma(a[3], -C30, a[1] * C50)));
    v[2] = ev2 + od2;
    v[6] = ev2 - od2;
    const f32x2 ev3 = pfma(a[8], -C20, pfma(a[6], bc(0.5f), pfma(a[4], C80, pfma(a[2], -C40, a[0]))));
    const f32x2 od3 = pfma(a[7], -C50, pfma(a[5], C10, pfma(a[3], -C30, a[1] * C70)));
    v[3] = ev3 + od3;
    v[5] = ev3 - od3;
    v[4] = a[0] - a[2] + a[4] - a[6] + a[8];
}

/* imdct36_w with the two 9-point DCT-IIIs packed (dct3_9p) and the output
 * in pairs W[n] = (w[n], w[17 - n]), n < 9: the window stage takes w[9 + i]
 * and w[8 - i] from one pair.  Bit-identical to imdct36_w. */
__device__ __forceinline__ void imdct36_wp(const float *X, f32x2 *W, const f32x2 *kc) {
    f32x2 a[9], V[9];
    float zprev = 0.f;
#pragma unroll
    for (int m = 0; m < 9; m++) {
        const float e = m ? X[2 * m] + X[2 * m - 1] : X[0];
        const float zo = X[2 * m + 1] + X[2 * m];
        a[m] = (f32x2){e, zo + zprev};
        zprev = zo;
    }
    dct3_9p(a, V, kc);
    /* w[n] = E[n] + P[n] K[n], w[17 - n] = E[n] - P[n] K[n]: one packed fma
     * with the pair (K[n], -K[n]) (kc[7 + n]); fused like the scalar form */
    const __attribute__((address_space(3))) f32x2 *kk = (const __attribute__((address_space(3))) f32x2 *)(uintptr_t)kc;
#pragma unroll
    for (int n = 0; n < 9; n++) W[n] = pfma((f32x2){V[n].y, V[n].y}, kk[7 + n], (f32x2){V[n].x, V[n].x});
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
#define SROW 36      /* LDS row stride of S (floats): 16-B rows, few conflicts */
#define SYN_BUF 1296 /* floats: max(xr 2x576, S 36x36, X 36x36)              */
#define XROW 36      /* LDS row stride of X: 16-B rows, conflict-free b128 writes;
                      * row n = X[n][0, 2, .., 30] then X[n][1, 3, .., 31] (the
                      * even / odd matrixing halves as the MFMA leaves them) */

typedef float f32x4 __attribute__((ext_vector_type(4)));

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
    /* tab->lpair [rate][variant][line pair] of the variant's family: MPEG-1
     * rates 0..2, or the six LSF rates 3..8                                */
    uint32_t lpair[LSF ? 6 : 3][3][288];
    float ce[16][16], co[16][16];    /* matrixing A: C[2m][i], C[2m+1][i], i < 16  */
    /* window taps as (D[j][2i], D[j][2i + 1]) pairs, tap-pair major: step i
     * of the window reads dwp[i][j], 8 B per lane at consecutive addresses,
     * conflict-free (as dw[j][16], a ds_read_b64 of 32 lanes 64 B apart
     * was an 8-way bank conflict) */
    f32x2 dwp[8][32];
    float p43s[512];                 /* sign(k - 256) |k - 256|^(4/3), k < 512     */
    /* long-block windows (x IMDCT output scale) in output pairs (i, 17 - i)
     * of both halves, wp[par][bt][i] = (w[i], w[17 - i], w[18 + i],
     * w[35 - i]), with the frequency inversion folded in for odd subbands
     * (par = sb & 1: the odd output slots negated, which the overlap then
     * carries negated too; StreamState holds the true values) */
    f32x4 wp[2][4][9];
    /* packed-op constants: the 9-point DCT-III cosines (c, c) (DCT9_KC),
     * then the DCT-IV output scales (K, -K) (IMDCT36_K) */
    f32x2 kc[7 + 9];
    float p2q[4]; /* 2^(i/4): pow2_quarter's mantissas, a branch-free lookup */
    uint16_t xcol[2][64]; /* phase W: lane (ch, j)'s X offsets in buf, columns win_a[j], win_b[j] */
    float isr[LSF ? 32 : 7][2];      /* intensity ratios: MPEG-1 [is_pos], LSF      */
                                     /* [intensity_scale * 16 + is_pos]            */
};
#define SYN_QOFF 1152 /* floats: phase Q's own data sits after the xr scatter area */
struct __attribute__((aligned(256))) SynWave { /* one per wave (stream)       */
    /* buf: xr -> S -> X hand-offs.  Phase Q's band scales, UnitMeta words and
     * intensity positions live only while buf holds xr (2 x 576 floats), so
     * they share buf's tail: 5.4 KB per wave, 39.4 KB per 4-wave workgroup
     * (<= 40 KB: 4 workgroups per CU) */
    union {
        float buf[SYN_BUF];
        struct {
            float xr_[SYN_QOFF];
            /* 2^(q/4) per (ch, band idx): long b | 22 + 3 b + w.  256-B
             * aligned rows, so a line pair's scale address is base |
             * (lpair & 0xFC): one VALU op */
            float scale[2][64];
            UnitMeta m[2];
            uint8_t is[64]; /* intensity position per right band idx, 0xFF none */
        };
    };
};
static_assert(SYN_QOFF * 4 % 256 == 0, "SynWave::scale rows 256-B aligned");
typedef __attribute__((address_space(3))) const float lds_cf32;

/* per-lane select on a wave mask, opaque to the optimizer: written as
 * `c ? t : f` the compiler sinks t's computation into a divergent branch
 * (exec save / restore and register copies around each state update) */
__device__ __forceinline__ float lane_sel(uint64_t m, float f, float t) {
    float r;
    __asm__("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}

#define WAIT_VMCNT0() __builtin_amdgcn_s_waitcnt(0x0F70) /* vmcnt(0), other counters free */

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

/* the workgroup's read-only tables, staged by NT threads (tid = 0 .. NT - 1;
 * the caller's barrier follows) */
template <bool F32, bool LSF, int NT>
__device__ __forceinline__ void synth_tables(SynShared<LSF> &T, const DevTables *__restrict__ tab, int tid) {
    constexpr int NRATE = LSF ? 6 : 3;
    static_assert(NT >= 64, "synth_tables: the LSF intensity ratios take 64 threads");
    for (int i = tid; i < NRATE * 3 * 288; i += NT)
        (&T.lpair[0][0][0])[i] = (&tab->lpair[LSF ? 3 : 0][0][0])[i];
    for (int i = tid; i < 256; i += NT) {
        const int r = i >> 4, c = i & 15;
        T.ce[r][c] = tab->dct_c[2 * r][c];
        T.co[r][c] = tab->dct_c[2 * r + 1][c];
    }
    for (int i = tid; i < 512; i += NT)
        T.p43s[i] = i >= 256 ? tab->pow43[i - 256] : -tab->pow43[256 - i];
    /* int16 sinks: taps x 32768 (exact, a power of two), so the sums
     * arrive in PCM units without a multiply per sample */
    for (int i = tid; i < 32 * 16; i += NT)
        ((float *)&T.dwp[0][0])[((i & 15) >> 1) * 64 + (i >> 4) * 2 + (i & 1)] = (&tab->dwin[0][0])[i] * (F32 ? 1.0f : 32768.0f);
    if (tid < 7 + 9) {
        const float c9[7] = DCT9_KC, k9[9] = IMDCT36_K;
        T.kc[tid] = tid < 7 ? (f32x2){c9[tid], c9[tid]} : (f32x2){k9[tid - 7], -k9[tid - 7]};
    }
    if (tid < 4) T.p2q[tid] = pow2_quarter(tid);
    if (tid < 128) {
        const int l = tid & 63, c = l >> 5, j = l & 31;
        const int w = (tid >> 6) ? tab->win_b[j] : tab->win_a[j];
        T.xcol[tid >> 6][l] = (uint16_t)(18 * c * XROW + (w & 1) * 16 + (w >> 1));
    }
    for (int k = tid; k < 2 * 4 * 9; k += NT) {
        const int par = k / 36, bt = (k / 9) % 4, i = k % 9;
        const float *w = c_win36[bt];
        const float sa = (par && (i & 1)) ? -1.f : 1.f, sb = (par && !(i & 1)) ? -1.f : 1.f; /* slots i, 17 - i */
        T.wp[par][bt][i] = (f32x4){sa * w[i], sb * w[17 - i], sa * w[18 + i], sb * w[35 - i]};
    }
    if (LSF) {
        if (tid < 64) (&T.isr[0][0])[tid] = (&c_is_lsf[0][0][0])[tid];
    } else if (tid < 14) (&T.isr[0][0])[tid] = (&c_is_ratio[0][0])[tid];
}

/* One stream (or frame segment) of k_synth's work by one wave; also the
 * last phase of the per-frame k_frame.  Frame-parallel segments (SRC_XR;
 * DESIGN.md §4): segment seg of nseg decodes frames [f0, f1) of stream s
 * after a one-frame warm-up from zero state.  The warm-up frame's granule 0
 * fixes the IMDCT overlap (the last 18 outputs of a granule's IMDCT do not
 * depend on the state), its granule 1 then yields exact S, X and the 15
 * carried X slots, so [f0, f1) is bit-identical to the sequential decode.
 * One segment (seg_len >= F): the stream's state in and out.  T = the
 * workgroup's tables (synth_tables), Wd = the wave's LDS buffer.  No
 * workgroup barrier inside. */
/* PF (k_frame's two-wave synthesis of one MPEG-1 frame): 0 =
 * the normal path; 1 = granule 0 only, publishing its IMDCT overlap (after
 * phase I) and its synthesis history (after phase W) in xch, no state out;
 * 2 = granule 1 only, taking them from xch, state out.  The two waves meet
 * at two workgroup barriers (every other wave of the workgroup runs two
 * as well). */
template <bool SRC_XR, bool F32, bool LSF, int PF = 0>
__device__ __forceinline__ void synth_stream(const FrameRec *__restrict__ rec, const int16_t *__restrict__ is_buf,
                                             const UnitMeta *__restrict__ meta, const float *__restrict__ xr_in,
                                             const uint8_t *__restrict__ xr_bt, const uint8_t *__restrict__ xr_mixed,
                                             const DevTables *__restrict__ tab, StreamState *__restrict__ st,
                                             void *__restrict__ pcm, int F, int xr_nch, int xr_sr, int seg_len,
                                             float *__restrict__ st_tail, const float *__restrict__ st_tail_in,
                                             SynShared<LSF> &T, SynWave &Wd, int s, int seg, int nseg,
                                             float *xch = nullptr, uint32_t *isq = nullptr) {
    static_assert(PF == 0 || (!SRC_XR && !LSF), "PF: k_frame's MPEG-1 decode path only");
    const int f0 = seg * seg_len, f1 = min(F, f0 + seg_len);
    /* first frame decoded (warm-up frames below f0 leave state, no PCM) and
     * where the state starts: the call's state (StreamState or the previous
     * call's tail) for segment 0; zeros before a warm-up that fixes it */
    int fw = seg ? f0 - 1 : 0;
    /* the last audio frame before f0 (decode path): its last granule is the
     * last warm-up granule, the one whose X fixes the synthesis history */
    int wlast = -1;
    bool from_state = seg == 0, ch1_state = false;
    if (!SRC_XR && seg > 0) {
        /* decode path (frame-parallel segments of a stream):
         * the state at f0 is fixed by the last audio frame before it (its
         * granule 0 the IMDCT overlap, granule 1 the 15 FIFO slots; an LSF
         * frame has one granule, so the last two).  Frames without audio
         * (tag, dropped) leave the state alone and are skipped.  A mono
         * warm-up fixes channel 0 only: channel 1 keeps the call's state,
         * unless a stereo frame came in between -- then, as when fewer audio
         * frames precede f0, the segment decodes from the call's state at
         * frame 0 (exact, just longer). */
        const uint32_t *rw = (const uint32_t *)(rec + (size_t)s * F);
        auto audio = [&](int f) {
            const uint32_t r4 = __builtin_amdgcn_readfirstlane(rw[8 * f + 4]);
            const uint32_t r6 = __builtin_amdgcn_readfirstlane(rw[8 * f + 6]);
            return (r4 & 0xFFFFu) != 0u && !(((r6 >> 8) & 0xFFu) & (REC_TAG | REC_DROP));
        };
        auto stereo = [&](int f) { return (__builtin_amdgcn_readfirstlane(rw[8 * f + 5]) >> 24) == 2u; };
        const int need = LSF ? 2 : 1;
        int found = 0, fa = f0;
        bool mono = false;
        for (int f = f0 - 1; f >= 0 && found < need; f--)
            if (audio(f)) {
                if (!found) wlast = f;
                found++;
                fa = f;
                mono = mono || !stereo(f);
            }
        bool stereo_before = false;
        if (found == need && mono)
            for (int f = 0; f < fa && !stereo_before; f++) stereo_before = audio(f) && stereo(f);
        if (found < need || stereo_before) {
            fw = 0;
            from_state = true;
        } else {
            fw = fa;
            ch1_state = mono;
        }
    }
    float *const sBuf = Wd.buf;
    const int lane = threadIdx.x & 63;
    const int ch = lane >> 5;
    const int sb = lane & 31; /* phase I: subband; phase W: output j */
    constexpr int MW = (int)(sizeof(UnitMeta) / 4); /* 14 words per unit */

    StreamState &S = st[s];
    /* IMDCT overlap in output pairs ovp[i] = (ov[i], ov[17 - i]), with the
     * odd slots of odd subbands negated (the frequency inversion folded into
     * the window tables, SynShared::wp); state in and out as true values */
    f32x2 ovp[9];
    const float sgo = (sb & 1) ? -1.f : 1.f; /* slot sign of odd slots */
    const f32x2 sgp[2] = {(f32x2){1.f, sgo}, (f32x2){sgo, 1.f}}; /* pair i even / odd */
    /* synthesis history as partial sums: the
     * window terms of the NEXT granule's output slots t = 0 .. 14 that read
     * this granule's matrixing outputs (slot t's taps i with t - 2 i < 0, or
     * t - 2 i - 1 < 0), summed when this granule's X is at hand.  hp[tp] =
     * (H_2tp, H_2tp+1) for lane (ch, j); H_15 = 0.  16 registers instead of
     * the 29 raw X values (ha / hb) the window read them from before.
     * StreamState.fifo[ch][t][j] holds H_t. */
    f32x2 hp[8];
    constexpr int TAIL = (int)(sizeof(S.overlap) + sizeof(S.fifo)) / 4; /* floats per stream tail */
    if (from_state || (ch1_state && ch == 1)) {
        /* state in: StreamState, or the previous call's tail (the same
         * overlap + fifo layout, packed per stream) */
        const float *ovi = st_tail_in ? st_tail_in + (size_t)s * TAIL : &S.overlap[0][0][0];
        const float *ffi = ovi + sizeof(S.overlap) / 4;
#pragma unroll
        for (int i = 0; i < 9; i++)
            ovp[i] = (f32x2){ovi[(ch * 32 + sb) * 18 + i], ovi[(ch * 32 + sb) * 18 + 17 - i]} * sgp[i & 1];
        /* the state holds H_t in float-sink units: int16 sinks run the
         * window in PCM units (taps x 2^15), so x 2^15 in (exact) */
        const f32x2 hsc = bc(F32 ? 1.0f : 32768.0f);
#pragma unroll
        for (int tp = 0; tp < 8; tp++)
            hp[tp] = (f32x2){ffi[(ch * MP3D_FIFO_SLOTS + 2 * tp) * 32 + sb],
                             2 * tp + 1 < MP3D_FIFO_SLOTS ? ffi[(ch * MP3D_FIFO_SLOTS + 2 * tp + 1) * 32 + sb] : 0.f} *
                     hsc;
    } else {
#pragma unroll
        for (int i = 0; i < 9; i++) ovp[i] = (f32x2){0.f, 0.f};
#pragma unroll
        for (int tp = 0; tp < 8; tp++) hp[tp] = (f32x2){0.f, 0.f};
    }

    /* Per-stream buffer resources: every granule access below is a buffer
     * instruction with a uniform byte offset in an SGPR and the lane offset
     * in one VGPR, instead of a 64-bit address pair per lane and load. */
    const int rb = 2 * MP3D_IS_ROW, gb = 2 * rb; /* is[] bytes per row, per granule (2 ch) */
    const __amdgpu_buffer_rsrc_t r_is = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(is_buf + (size_t)s * F * 4 * MP3D_IS_ROW), 0, F * 2 * gb, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_meta = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(meta + (size_t)s * F * 4), 0, F * 4 * (int)sizeof(UnitMeta), 0x00020000);
    const __amdgpu_buffer_rsrc_t r_rec = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(rec + (size_t)s * F), 0, F * (int)sizeof(FrameRec), 0x00020000);
    constexpr int PB = F32 ? 4 : 2; /* bytes per output sample: f32 or int16 */
    const __amdgpu_buffer_rsrc_t r_pcm = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((uint8_t *)pcm + (size_t)s * F * 2304 * PB), 0, F * 2304 * PB, 0x00020000);

    /* granule prefetch: is[] words one granule ahead of use (lane owns
     * lines 2 lane + 128 i, +1), the UnitMeta words of both channels (lanes
     * 0 .. 27) and the FrameRec words (lanes 32 .. 39) TWO granules ahead,
     * so each is[] load is masked by its unit's nz_end: the rzero tail that
     * k_huffman never wrote is not fetched (HBM read traffic ~ nonzero
     * prefix, not 2 x 576 lines).  wm / wr = the UnitMeta / FrameRec words
     * of two consecutive granules.  MPEG-1 decode (PAR): slot = granule
     * parity, with the granule loop unrolled, so each load writes its
     * loop-carried register directly; otherwise slot 0 = the current
     * granule, slot 1 the next, shifted after each prefetch. */
    constexpr bool PAR = !SRC_XR && !LSF && PF == 0;
    constexpr bool XDMA = SRC_XR && !LSF && PF == 0;
    /* PAR (the batch's MPEG-1 decode, 8-wave workgroups): the is[] words go
     * by LDS-DMA (buffer_load ... lds) into the wave's isq area [ch][320]
     * (256-B pieces; the fifth piece's upper half is padding) instead of
     * ten registers held through phases I, M and W: the register budget
     * of 4 waves per SIMD.  Otherwise into nis. */
    uint32_t nis[2][5], wm[2] = {0u, 0u}, wr[2] = {0u, 0u};
    constexpr int GSTEP = LSF ? 2 : 1; /* is[] granule slots per decoded granule */
    /* two unconditional loads; a lane outside a word range gets an offset
     * past the buffer (reads 0), and so do granules past F.  (As one value
     * loaded in two divergent branches, the merged result was copied into
     * the loop-carried register right after the loads -- a vmcnt(0) wait
     * that made the whole prefetch synchronous.) */
    auto load_words = [&](int g, uint32_t &vm, uint32_t &vr) {
        const int lo = opaque(lane * 4);
        const int om = lane < 2 * MW ? lo : 0x40000000, orr = (lane >= 32 && lane < 40) ? lo - 128 : 0x40000000;
        vm = __builtin_amdgcn_raw_buffer_load_b32(r_meta, om, g * 2 * (int)sizeof(UnitMeta), 0);
        vr = __builtin_amdgcn_raw_buffer_load_b32(r_rec, orr, (g >> 1) * (int)sizeof(FrameRec), 0);
    };
    /* (The loads are nt: each is[] row is read once.)
     * The LDS-DMA as inline asm, one block per channel: M0 = the channel's
     * LDS area (saved and restored), the five 256-B pieces at instruction
     * offsets 0 .. 1024 (the offset moves the memory AND the LDS address:
     * LDS = M0 + offset + 4 lane, probed on the box, tools/dbg/
     * lds_dma_probe.hip), and a descriptor per channel whose byte range is the
     * row's nonzero prefix (2 nz_end bytes): every word at or past nz_end,
     * and past the row, reads as 0, with no per-lane offset arithmetic.  As
     * __builtin_amdgcn_raw_ptr_buffer_load_lds the compiler's wait-count
     * pass, which cannot tell these LDS writes from the kernel's other LDS
     * accesses, waited for the DMA (vmcnt) before every later LDS read --
     * the prefetch turned synchronous.  Completion is the kernel's own
     * vmcnt(0) before phase W (and after prefetch_full); the hardware counts
     * these loads like any other, so the compiler's counted waits for its
     * own loads can only over-wait. */
    const uint64_t isb = (uint64_t)(uintptr_t)(is_buf + (size_t)s * F * 4 * MP3D_IS_ROW);
    auto dma_is = [&](int g, int nz0, int nz1) {
        const int lo = opaque(lane * 4);
        const uint32_t lds0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_cf32 *)(const float *)isq);
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const uint64_t ra = isb + (uint64_t)(uint32_t)(g * gb + c * rb);
            const u32x4 rs = {(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ra),
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ra >> 32)) & 0xFFFFu,
                              (uint32_t)__builtin_amdgcn_readfirstlane(2 * (c ? nz1 : nz0)), 0x00020000u};
            uint32_t keep;
            /* lgkmcnt(0) first: this granule's LDS reads of the area (the
             * fused requantiser's iw[] words may be waited on only where they
             * are used, which the compiler can place after this block) */
            __asm__ volatile("s_waitcnt lgkmcnt(0)\n\t"
                             "s_mov_b32 %0, m0\n\t"
                             "s_mov_b32 m0, %2\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dword %1, %3, 0 offen nt lds\n\t"
                             "buffer_load_dword %1, %3, 0 offen offset:256 nt lds\n\t"
                             "buffer_load_dword %1, %3, 0 offen offset:512 nt lds\n\t"
                             "buffer_load_dword %1, %3, 0 offen offset:768 nt lds\n\t"
                             "buffer_load_dword %1, %3, 0 offen offset:1024 nt lds\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep)
                             : "v"(lo), "s"(lds0 + 1280u * c), "s"(rs)
                             : "memory");
        }
    };
    auto load_is = [&](int g, int nz0, int nz1) {
        if (PAR) {
            dma_is(g, nz0, nz1);
            return;
        }
        const int lo = opaque(lane * 4);
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int nz = c ? nz1 : nz0;
#pragma unroll
            for (int i = 0; i < 5; i++) {
                nis[c][i] = 0u;
                if ((i < 4 || lane < 32) && 2 * lane + 128 * i < nz)
                    nis[c][i] = __builtin_amdgcn_raw_buffer_load_b32(r_is, lo + c * rb + 256 * i, g * gb, 0);
            }
        }
    };
    /* is[g] masked by granule g's nz_end from its meta words m (channel 1
     * only in a stereo frame: FrameRec.nch, lane 37): every line >= nz_end
     * then reads as 0 in registers, so phase Q needs no rzero mask */
    auto load_is_masked = [&](int g, uint32_t mm, uint32_t mr) {
        const bool st = ((uint32_t)__builtin_amdgcn_readlane((int)mr, 37) >> 24) == 2u;
        const int nz0 = __builtin_amdgcn_readlane((int)mm, 12) & 0xFFFF;
        const int nz1 = st ? __builtin_amdgcn_readlane((int)mm, MW + 12) & 0xFFFF : 0;
        load_is(g, nz0, nz1);
    };
    /* steady state, from granule slot cs: is[g] masked by the next
     * granule's words, then granule g + 1's words (PAR: into the slot the
     * current granule frees; else a shift).  As one rotated variable, the
     * merged load result was copied into the loop-carried register right
     * after the loads -- a vmcnt(0) wait that made the prefetch synchronous
     * (k_synth spent ~28 % of its wave time there, abx/ptime.py). */
    auto prefetch = [&](int g, int cs) {
        load_is_masked(g, wm[cs ^ 1], wr[cs ^ 1]);
        if (PAR) {
            load_words(g + GSTEP, wm[cs], wr[cs]);
        } else {
            wm[0] = wm[1];
            wr[0] = wr[1];
            load_words(g + GSTEP, wm[1], wr[1]);
        }
    };
    /* entry and after a frame without audio (g even for PAR): the words
     * first, drained, then the masked is[] (off the common path) */
    auto prefetch_full = [&](int g) {
        load_words(g, wm[0], wr[0]);
        load_words(g + GSTEP, wm[1], wr[1]);
        WAIT_VMCNT0();
        load_is_masked(g, wm[0], wr[0]);
    };
    /* SRC_XR (config 2): the next granule's spectra (lane: line pairs
     * lane + 64 i of both channels, as is[] on the decode path) and block
     * types (lanes 0..3: bt0, bt1, mixed0, mixed1) are loaded one granule
     * ahead; granules past F read as zero (buffer range). */
    f32x2 nxr[2][5];
    uint32_t nbt = 0u;
    const __amdgpu_buffer_rsrc_t r_xr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(xr_in + (SRC_XR ? (size_t)s * F * 2 * xr_nch * 576 : 0)), 0, SRC_XR ? F * 2 * xr_nch * 2304 : 0,
        0x00020000);
    /* XDMA (the synth-only entry at 4 waves / SIMD, 8-wave workgroups):
     * channel 0's 576 floats go by LDS-DMA into the wave's isq area (nine
     * 256-B pieces, the dma_is recipe; a granule past F reads 0), channel 1
     * into nxr[1] -- 10 registers instead of 20 held through I, M and W */
    auto dma_xr = [&](int g) {
        const int lo = opaque(lane * 4);
        const uint32_t lds0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_cf32 *)(const float *)isq);
        const uint64_t ra = (uint64_t)(uintptr_t)(xr_in + (size_t)s * F * 2 * xr_nch * 576);
        const u32x4 rs = {(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ra),
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ra >> 32)) & 0xFFFFu,
                          (uint32_t)(F * 2 * xr_nch * 2304), 0x00020000u};
        const int so = __builtin_amdgcn_readfirstlane(g * xr_nch * 2304);
        uint32_t keep;
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n\t" /* this granule's reads of the area are done */
                         "s_mov_b32 %0, m0\n\t"
                         "s_mov_b32 m0, %2\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dword %1, %3, %4 offen nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:256 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:512 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:768 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:1024 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:1280 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:1536 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:1792 nt lds\n\t"
                         "buffer_load_dword %1, %3, %4 offen offset:2048 nt lds\n\t"
                         "s_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(lo), "s"(lds0), "s"(rs), "s"(so)
                         : "memory");
        /* and channel 1's last chunk (lines 512 .. 575, lanes < 32 only:
         * half the lanes of a register pair) into the area's last 256 B */
        if (xr_nch == 2) {
            uint32_t keep1;
            __asm__ volatile("s_mov_b32 %0, m0\n\t"
                             "s_mov_b32 m0, %2\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dword %1, %3, %4 offen nt lds\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep1)
                             : "v"(lo), "s"(lds0 + 2304u), "s"(rs), "s"(so + 2304 + 2048)
                             : "memory");
        }
    };
    auto load_xr = [&](int g) {
        const int lo = opaque(lane * 8);
        if (XDMA) dma_xr(g);
#pragma unroll
        for (int c = XDMA ? 1 : 0; c < 2; c++)
#pragma unroll
            for (int i = 0; i < (XDMA ? 4 : 5); i++) { /* XDMA: channel 1's chunk 4 by DMA */
                nxr[c][i] = (f32x2){0.f, 0.f};
                if (c < xr_nch && (i < 4 || lane < 32))
                    nxr[c][i] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                                              r_xr, lo + 512 * i + 2304 * c, g * xr_nch * 2304, 0));
            }
        /* block type (lanes 0, 1) and mixed flag (lanes 2, 3) of channel
         * lane & 1: two unconditional byte loads from the uniform array
         * bases with 32-bit lane offsets (a per-lane 64-bit address was
         * held across the loop and spilled) */
        const int lq = opaque((int)(threadIdx.x & 63)), q = lq & 1;
        const bool okq = lq < 4 && q < xr_nch && g < 2 * F;
        const uint32_t ob = okq ? (uint32_t)(((s * F * 2) + g) * xr_nch + q) : 0u;
        const uint32_t vb = xr_bt[ob], vm = xr_mixed[ob];
        nbt = okq ? (lq < 2 ? vb : vm) : 0u;
    };
    if (SRC_XR) {
        load_xr(2 * fw);
        if (XDMA) WAIT_VMCNT0(); /* channel 0 lands in LDS before the first phase Q */
    }
    if (!SRC_XR) {
        prefetch_full(2 * fw + (PF == 2 ? 1 : 0));
        /* explicit drain on the entry path, so the compiler's wait before
         * each prefetch use is set by the loop path (stores after it) */
        WAIT_VMCNT0();
    }

    /* phase M's S / X row offsets of this lane (lane constants, held across
     * the loop: recomputed from the lane id they cost 14 VALU a granule; A/B
     * MH -0.9 % k_synth): row block 0 / 1 at m_off_a (+ 16 rows), block 2
     * (rows 32..35, clamped) at m_off_c */
    const int mlane_ = (int)(threadIdx.x & 63);
    /* xin's one read address: 8 words below the lane's 18 lines (the previous
     * subband's last 8), every read an immediate offset from it; subbands 0
     * and 31 read neighbour words they do not use (the LDS objects have a pad
     * below wave 0's buffer) instead of selecting their own (A/B XIN) */
    const uint32_t xin_off = (uint32_t)(((mlane_ >> 5) * 576 + 18 * (mlane_ & 31) - 8) * 4);
    const uint32_t m_off_a = (uint32_t)(((mlane_ & 15) * SROW + 4 * (mlane_ >> 4)) * 4);
    const uint32_t m_off_c = (uint32_t)((((mlane_ & 15) < 4 ? 32 + (mlane_ & 15) : 35) * SROW + 4 * (mlane_ >> 4)) * 4);
    for (int f = fw; f < f1; f++) {
        int nch, sr, mode = 0, mext = 0;
        const size_t fr = (size_t)s * F + f;
        if (SRC_XR) {
            nch = xr_nch;
            sr = xr_sr;
        } else {
            /* FrameRec words 4 .. 6 from the prefetch (lanes 36 .. 38) */
            const uint32_t r4 = (uint32_t)__builtin_amdgcn_readlane((int)wr[0], 36);
            const uint32_t r5 = (uint32_t)__builtin_amdgcn_readlane((int)wr[0], 37);
            const uint32_t r6 = (uint32_t)__builtin_amdgcn_readlane((int)wr[0], 38);
            const uint32_t first_gr = (r6 >> 8) & 0xFFu;
            if (!(r4 & 0xFFFFu) || (first_gr & (REC_TAG | REC_DROP))) {
                /* no audio in this frame: fetch the next frame's granule 0
                 * now and wait for it here, off the common path */
                if (f + 1 < f1) prefetch_full(2 * (f + 1));
                WAIT_VMCNT0();
                continue;
            }
            nch = (int)(r5 >> 24);
            sr = (int)((r6 >> 16) & 15u) - (LSF ? 3 : 0); /* FrameRec.sr_idx in the family */
            mode = (int)(r5 >> 22) & 3;
            mext = (int)(r5 >> 20) & 3;
        }
        /* lanes of coded channels: channel 0's half, or all -- from nch
         * alone, no lane id (held across the loop for a ballot, the lane id
         * was the synth-only variant's last spill) */
        const uint64_t amask = nch == 2 ? ~0ull : 0xFFFFFFFFull;
        const uint32_t(*lpair)[288] = T.lpair[sr];
#pragma unroll /* the words' slot (cs) is then a constant per copy */
        for (int gr = PF == 2 ? 1 : 0; gr < (LSF || PF == 1 ? 1 : 2); gr++) { /* LSF: one granule per frame */
            const int cs = PAR ? gr : 0; /* slot of this granule's words */
            /* lane-derived indices are re-derived from an opaque copy each
             * granule so they are not hoisted and held live across the loop */
            const int lane = opaque((int)(threadIdx.x & 63));
            const int ch = lane >> 5, sb = lane & 31;
            /* block structure of both channels (uniform) */
            int bt0, mx0, bt1 = 0, mx1 = 0;
            /* decode path: the wave issues at raised priority through phase Q
             * (its next-granule prefetch and LDS table reads go out ahead of
             * the other waves' VALU phases; A/B SP2: -2 % k_synth on C3; the
             * synth-only entry measured within noise, so it stays at 0) */
            if (!SRC_XR) __builtin_amdgcn_s_setprio(1);
            bool fusedq = false; /* phase Q's fused requantiser ran */
            /* phase I's input: lane (ch, sb)'s 18 lines and the alias
             * neighbours up[k] = x_{sb-1}[17 - k], dn[k] = x_{sb+1}[k] */
            float xf[18], up[8], dn[8];
            /* ... read back from the xr scatter (after the wave's LDS stores
             * land), at the end of each scatter path of phase Q (as one
             * read after the paths merge, the fused path's xf was held
             * across the scatter paths' registers and spilled) */
            auto xin = [&]() {
                wave_sync();
                typedef __attribute__((address_space(3))) const f32x2 lds_cf2;
                lds_cf2 *const P = (lds_cf2 *)(uintptr_t)((uint32_t)(uintptr_t)(lds_cf32 *)(const float *)sBuf + xin_off);
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    const f32x2 v = P[4 + i];
                    xf[2 * i] = v.x;
                    xf[2 * i + 1] = v.y;
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const f32x2 p = P[i];
                    const f32x2 n = P[13 + i];
                    up[7 - 2 * i] = p.x;
                    up[6 - 2 * i] = p.y;
                    dn[2 * i] = n.x;
                    dn[2 * i + 1] = n.y;
                }
            };
            /* ---------------- phase Q: requantise + stereo -> LDS ---------- */
            if (SRC_XR) {
                (void)fr;
                f32x2 cx[2][5];
#pragma unroll
                for (int c = 0; c < 2; c++)
#pragma unroll
                    for (int i = 0; i < 5; i++)
                        cx[c][i] = XDMA && (c == 0 || i == 4)
                                       ? (c == 0 || (nch == 2 && lane < 32)
                                              ? *(const f32x2 *)((const float *)isq + 576 * c + 2 * lane + 128 * i - 512 * c)
                                              : (f32x2){0.f, 0.f})
                                       : nxr[c][i];
                bt0 = __builtin_amdgcn_readlane((int)nbt, 0);
                mx0 = bt0 == 2 ? __builtin_amdgcn_readlane((int)nbt, 2) : 0;
                if (nch == 2) {
                    bt1 = __builtin_amdgcn_readlane((int)nbt, 1);
                    mx1 = bt1 == 2 ? __builtin_amdgcn_readlane((int)nbt, 3) : 0;
                }
                if (f + 1 < f1 || gr == 0) load_xr(2 * f + gr + 1); /* next granule, in flight through I, M, W */
                const int xv[2] = {bt0 == 2 ? (mx0 ? 2 : 1) : 0, bt1 == 2 ? (mx1 ? 2 : 1) : 0};
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    if (i < 4 || lane < 32) {
                        const int k = lane + 64 * i;
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            if (c < nch) {
                                if (xv[c] == 0) {
                                    *(f32x2 *)&sBuf[576 * c + 2 * k] = cx[c][i];
                                } else {
                                    const uint32_t tv2 = lpair[xv[c]][k];
                                    sBuf[576 * c + ((tv2 >> 8) & 1023u)] = cx[c][i][0];
                                    sBuf[576 * c + ((tv2 >> 18) & 1023u)] = cx[c][i][1];
                                }
                            }
                        }
                    }
                }
                xin();
            } else {
                /* nz_end per channel (UnitMeta word 12, uniform): the 128-line
                 * chunks i at or past max(nz_end) are all zero, so their
                 * words are not read and their lines not requantised.  Three
                 * straight-line copies (2, 3 or 5 live chunks; C3 granules
                 * mostly end below line 256 or 384), each keeping its LDS
                 * reads batched -- a branch per chunk made every chunk wait
                 * out its own reads. */
                const int nzq0 = __builtin_amdgcn_readlane((int)wm[cs], 12) & 0xFFFF;
                const int nzq1 = nch == 2 ? __builtin_amdgcn_readlane((int)wm[cs], MW + 12) & 0xFFFF : 0;
                const int nzmax = nzq0 > nzq1 ? nzq0 : nzq1;
                const int nlive = nzmax <= 256 ? 2 : (nzmax <= 384 ? 3 : 5); /* uniform */
                uint32_t cis[2][5];
                auto read_cis = [&](auto nic) {
                    constexpr int NI = decltype(nic)::value;
#pragma unroll
                    for (int c = 0; c < 2; c++)
#pragma unroll
                        for (int i = 0; i < 5; i++)
                            cis[c][i] = i < NI ? (PAR ? isq[320 * c + 64 * i + lane] : nis[c][i]) : 0u;
                };
                /* UnitMeta into LDS for the (rare) intensity path; the common
                 * path reads the prefetched words straight from registers */
                if (lane < nch * MW) ((uint32_t *)&Wd.m[0])[lane] = wm[cs]; /* lane / MW < nch, no division */
                /* words 10..12: gain, block type, mixed, scalefac_scale |
                 * preflag, sbg[3] | nz_end (UnitMeta layout) */
                const uint32_t m10a = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], 10);
                const uint32_t m11a = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], 11);
                const uint32_t m12a = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], 12);
                const uint32_t m10b = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], MW + 10);
                const uint32_t m11b = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], MW + 11);
                const uint32_t m12b = (uint32_t)__builtin_amdgcn_readlane((int)wm[cs], MW + 12);
                bt0 = (int)(m10a >> 8) & 0xFF;
                mx0 = (int)(m10a >> 16) & 0xFF;
                if (nch == 2) {
                    bt1 = (int)(m10b >> 8) & 0xFF;
                    mx1 = (int)(m10b >> 16) & 0xFF;
                }
                const int var[2] = {bt0 == 2 ? (mx0 ? 2 : 1) : 0, bt1 == 2 ? (mx1 ? 2 : 1) : 0};
                const bool is_on = mode == 1 && nch == 2 && (mext & 1);
                const bool ms_fold = mode == 1 && nch == 2 && mext == 2; /* M/S only: 1/sqrt2 in the scale */
                /* fused requantiser: MPEG-1 decode, long blocks in every
                 * channel, neither intensity nor M/S (uniform).  With M/S a
                 * lane pairs its lines with lane +- 32's (v_permlane32_swap
                 * of a line with itself, then one FMA: bit-exact), but the 36
                 * VALU per granule cost more than the LDS round trip saved
                 * (A/B FQ: C3 +2 % k_synth) */
                fusedq = PAR && var[0] == 0 && var[1] == 0 && !is_on && !ms_fold;
                const float rsq2 = 0.70710678118654752f;
                /* per-band scale 2^(q/4), lane = band idx (long b | 22 + 3 b + w);
                 * the lane's scalefactor byte comes from the prefetched meta
                 * words by one cross-lane read per channel */
                /* 2^(q/4) = ldexp(2^((q & 3) / 4), q >> 2): the mantissa from a
                 * 4-entry LDS table (as a select chain the compiler built
                 * divergent branches) */
                /* uniform: one multiply, no select; the select on integer
                 * bits so it stays scalar (as a float select its constant was
                 * held in a VGPR across the loop) */
                const float msf = __int_as_float(__builtin_amdgcn_readfirstlane(ms_fold ? 0x3f3504f3 : 0x3f800000));
                auto p2q = [&](int q) { return ldexpf(T.p2q[q & 3], q >> 2) * msf; };
                if (var[0] == 0 && (nch == 1 || var[1] == 0)) {
                    /* long blocks in every coded channel (the common case): both
                     * channels' 22 band scales in one pass, lane = (ch, band) */
                    const int c = lane >> 5, bl = lane & 31, j = bl < 22 ? bl : 21;
                    const uint32_t g10 = c ? m10b : m10a, g11 = c ? m11b : m11a;
                    const int gain = (int)(g10 & 0xFFu) - 210, shift = (int)(g10 >> 24) + 1;
                    const uint32_t wd = (uint32_t)__shfl((int)wm[cs], c * MW + (j >> 2));
                    const int sf = (int)(wd >> (8 * (j & 3))) & 0xFF;
                    const int pre = (g11 & 0xFFu) ? (int)(MP3D_PRETAB_BITS >> (2 * j)) & 3 : 0;
                    const float v = p2q(gain - ((sf + pre) << shift));
                    if (bl < 22) Wd.scale[c][bl] = v;
                } else {
                    const bool lng = lane < 22;
                    const int b = (lane - 22) / 3, w = lane - 22 - 3 * b;
                    auto band_scale = [&](uint32_t g10, uint32_t g11, int cbase) {
                        const int gain = (int)(g10 & 0xFFu) - 210, shift = (int)(g10 >> 24) + 1;
                        const bool mixed = ((g10 >> 16) & 0xFFu) != 0u, preflag = (g11 & 0xFFu) != 0u;
                        int j = mixed ? 8 + 3 * (b - 3) + w : 3 * b + w;
                        j = lng ? lane : (j < 0 ? 0 : (j > 39 ? 39 : j));
                        const uint32_t wd = (uint32_t)__shfl((int)wm[cs], cbase + (j >> 2));
                        const int sf = (int)(wd >> (8 * (j & 3))) & 0xFF;
                        const int pre = preflag ? (int)(MP3D_PRETAB_BITS >> (2 * (lane & 31))) & 3 : 0;
                        const int sbg = (int)(g11 >> (8 * (1 + (w < 3 ? w : 0)))) & 0xFF;
                        return p2q(lng ? gain - ((sf + pre) << shift) : gain - 8 * sbg - (sf << shift));
                    };
                    Wd.scale[0][lane] = band_scale(m10a, m11a, 0);
                    if (nch == 2) Wd.scale[1][lane] = band_scale(m10b, m11b, MW);
                }
                wave_sync();
                (void)m12a;
                (void)m12b;
                /* line pairs (2 i + e) kept as register pairs: the long-block
                 * scatter stores them with one ds_write_b64, no moves */
                f32x2 xp[2][5];
#define XV(c, k) xp[c][(k) >> 1][(k) & 1]
                /* per is[] word (two int16 lines): t = 4 (both halves + 256),
                 * one packed u16 op, is the byte offset into the signed table
                 * p43s; a half outside 0 .. 2047 (is >= 256 or < -256) is an
                 * escape, collected over the words in bigacc and patched
                 * below.  Both lines of a pair share one band (every long and
                 * short band width is even, tests/test_tables.py): one scale
                 * read per pair. */
                uint32_t bigacc = 0u;
                uint32_t k1024 = 1024u; /* in an SGPR (a literal is not a VOP3P operand here) */
                __asm__ volatile("" : "+s"(k1024));
                const uint32_t sc_base[2] = {(uint32_t)(uintptr_t)(lds_cf32 *)&Wd.scale[0][0],
                                             (uint32_t)(uintptr_t)(lds_cf32 *)&Wd.scale[1][0]};
                const uint8_t *p43b = (const uint8_t *)T.p43s;
                if (fusedq) {
                    /* lane (ch, sb) requantises its own subband's 18 lines
                     * (is[] words 9 sb .. 9 sb + 8 of its channel's prefetch
                     * area, stride 9: conflict-free) straight into phase I's
                     * registers: no xr scatter through LDS and no reads back;
                     * phase I takes the alias neighbours by DPP lane shifts */
                    const int lq = opaque((int)(threadIdx.x & 63));
                    const int fc = lq >> 5, fsb = lq & 31;
                    const uint32_t *iw = isq + 320 * fc + 9 * fsb;
                    const uint32_t *lpw = &lpair[0][9 * fsb];
                    const uint32_t scb = fc ? sc_base[1] : sc_base[0];
                    uint32_t bigf = 0u;
#pragma unroll
                    for (int m = 0; m < 9; m++) {
                        const uint32_t tv2 = lpw[m];
                        uint32_t t;
                        __asm__("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,0]" : "=v"(t) : "v"(iw[m]), "s"(k1024));
                        bigf |= t;
                        const float sc = *(lds_cf32 *)(uintptr_t)(scb | (tv2 & 0xFCu));
                        xf[2 * m] = *(const float *)(p43b + (t & 0x7FCu)) * sc;
                        xf[2 * m + 1] = *(const float *)(p43b + ((t >> 16) & 0x7FCu)) * sc;
                    }
                    if (__ballot((bigf & 0xF800F800u) != 0u)) {
                        /* rare: escapes (|is| >= 256), the words read again */
#pragma unroll
                        for (int m = 0; m < 9; m++) {
                            const uint32_t w = iw[m];
#pragma unroll
                            for (int e = 0; e < 2; e++) {
                                const int v = (int)(int16_t)(e ? (w >> 16) : (w & 0xFFFFu));
                                const int a = v < 0 ? -v : v;
                                if ((uint32_t)(v + 256) >= 512u) {
                                    const float mag = pow43_big(a) * *(lds_cf32 *)(uintptr_t)(scb | (lpw[m] & 0xFCu));
                                    xf[2 * m + e] = v < 0 ? -mag : mag;
                                }
                            }
                        }
                    }
                    /* the alias neighbours by DPP whole-wave shifts: lane
                     * i - 1 (wave_shr) and i + 1 (wave_shl); across the
                     * channel boundary (sb 31 | 0) they are not used */
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        up[k] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(xf[17 - k]), 0x138, 0xF, 0xF, false));
                        dn[k] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(xf[k]), 0x130, 0xF, 0xF, false));
                    }
                } else {
                /* (read here, not before the band scales: read early, the
                 * words were held through the fused path and spilled) */
                if (nlive == 2) read_cis(std::integral_constant<int, 2>{});
                else if (nlive == 3) read_cis(std::integral_constant<int, 3>{});
                else read_cis(std::integral_constant<int, 5>{});
                auto requant = [&](auto nic) {
                constexpr int NI = decltype(nic)::value;
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    const bool ok = i < 4 || lane < 32;
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        if (i >= NI) {
                            XV(c, 2 * i) = 0.f;
                            XV(c, 2 * i + 1) = 0.f;
                            continue;
                        }
                        const uint32_t tv2 = ok ? lpair[var[c]][lane + 64 * i] : 0u;
                        /* lines >= nz_end arrive as 0 (load_is_masked) */
                        /* one v_pk_mad_u16: 4 v + 1024 in both halves (as C the
                         * compiler emitted a packed shift and a packed add) */
                        uint32_t t;
                        __asm__("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,0]" : "=v"(t) : "v"(cis[c][i]), "s"(k1024));
                        bigacc |= t;
                        const float sc = *(lds_cf32 *)(uintptr_t)(sc_base[c] | (tv2 & 0xFCu));
                        XV(c, 2 * i) = *(const float *)(p43b + (t & 0x7FCu)) * sc;
                        XV(c, 2 * i + 1) = *(const float *)(p43b + ((t >> 16) & 0x7FCu)) * sc;
                    }
                }
                };
                if (nlive == 2) requant(std::integral_constant<int, 2>{});
                else if (nlive == 3) requant(std::integral_constant<int, 3>{});
                else requant(std::integral_constant<int, 5>{});
                if (__ballot((bigacc & 0xF800F800u) != 0u)) {
                    /* rare path (escapes |is| >= 256): patch those lines with
                     * the in-register |is|^(4/3); one block, so the loop above
                     * stays branch-free and its LDS reads batch */
#pragma unroll
                    for (int i = 0; i < 5; i++) {
#pragma unroll
                        for (int c = 0; c < 2; c++) {
#pragma unroll
                            for (int e = 0; e < 2; e++) {
                                const int v = (int)(int16_t)(e ? (cis[c][i] >> 16) : (cis[c][i] & 0xFFFFu));
                                const int a = v < 0 ? -v : v;
                                if ((uint32_t)(v + 256) >= 512u) {
                                    const uint32_t tv2 = lpair[var[c]][lane + 64 * i];
                                    const float mag = pow43_big(a) * Wd.scale[c][(tv2 >> 2) & 63u];
                                    XV(c, 2 * i + e) = v < 0 ? -mag : mag;
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
                    /* a line counts as nonzero from FFmpeg's fixed-point
                     * resolution up: its requantiser rounds |xr| below
                     * 0.5 * 1.759 * 2^-28 to 0 (oracle ORC_FFMPEG_FLUSH,
                     * pinned by the probe_flush_* fixtures) */
                    constexpr float FLUSH = 0.5f * 1.759f / 268435456.0f;
                    uint64_t nzR = 0;
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const uint32_t tv2 = (i < 4 || lane < 32) ? lpair[var[1]][lane + 64 * i] : 0u;
                        if (fmaxf(fabsf(XV(1, 2 * i)), fabsf(XV(1, 2 * i + 1))) >= FLUSH)
                            nzR |= 1ull << ((tv2 >> 2) & 63u);
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
                            if (!short_nz && ((uint32_t)(nzR & 0x3FFFFFull) >> lane) == 0u && p < opaque(IS_ILLEGAL)) ip = p;
                        }
                    } else if (lane < 61 && bt1 == 2) {
                        const int b = (lane - 22) / 3, w = lane - 22 - 3 * b;
                        if (!mx1 || b >= 3) {
                            const int kb = b == 12 ? 11 : b;
                            const int p = R.sf[mx1 ? 8 + 3 * (kb - 3) + w : 3 * kb + w];
                            /* no nonzero line in window w at bands >= b */
                            uint64_t above = 0;
                            for (int bb = b; bb < 13; bb++) above |= 1ull << (22 + 3 * bb + w);
                            if ((nzR & above) == 0ull && p < opaque(IS_ILLEGAL)) ip = p;
                        }
                    }
                    /* LSF: ratio row by intensity_scale (UnitMeta.flags bit 1) */
                    if (LSF && ip != 0xFF) ip += (int)(R.flags & 2u) << 3;
                    Wd.is[lane] = (uint8_t)ip;
                    wave_sync();
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const uint32_t tv2 = (i < 4 || lane < 32) ? lpair[var[1]][lane + 64 * i] : 0u;
                        const int ipl = Wd.is[(tv2 >> 2) & 63u];
#pragma unroll
                        for (int e = 0; e < 2; e++) {
                            const int k = 2 * i + e;
                            const float lv = XV(0, k), rv = XV(1, k);
                            if (ipl != 0xFF) {
                                const f32x2 rr = *(const __attribute__((address_space(3))) f32x2 *)(uintptr_t)(uint32_t)(
                                    opaque((int)(uintptr_t)(lds_cf32 *)&T.isr[0][0]) + 8 * ipl);
                                XV(0, k) = lv * rr.x;
                                XV(1, k) = lv * rr.y;
                            } else if (mext & 2) {
                                XV(0, k) = (lv + rv) * rsq2;
                                XV(1, k) = (lv - rv) * rsq2;
                            }
                        }
                    }
                }
                /* scatter in (short-block reordered) position; M/S-only frames
                 * store (L + R, L - R) from their own copy of the loop (as an
                 * in-place update before one scatter, the branch merge cost a
                 * register copy per line pair) */
                auto scatter = [&](int i, int c, f32x2 v) {
                    if (var[c] == 0) { /* long block: in place, one 8-B store */
                        *(f32x2 *)&sBuf[576 * c + 2 * lane + 128 * i] = v;
                    } else {
                        const uint32_t tv2 = lpair[var[c]][lane + 64 * i];
                        sBuf[576 * c + ((tv2 >> 8) & 1023u)] = v.x;
                        sBuf[576 * c + ((tv2 >> 18) & 1023u)] = v.y;
                    }
                };
                if (ms_fold) {
#pragma unroll
                    for (int i = 0; i < 5; i++)
                        if (i < 4 || lane < 32) {
                            scatter(i, 0, xp[0][i] + xp[1][i]);
                            scatter(i, 1, xp[0][i] - xp[1][i]);
                        }
                } else {
#pragma unroll
                    for (int i = 0; i < 5; i++)
                        if (i < 4 || lane < 32) {
#pragma unroll
                            for (int c = 0; c < 2; c++)
                                if (c < nch) scatter(i, c, xp[c][i]);
                        }
                }
                xin();
                } /* !fusedq */
                /* the next granule's loads fly during phases I, M, W (issued
                 * after phase Q read this granule's words), from ONE call
                 * site: issued in both requantiser paths, the loaded words
                 * merged at the join with a register copy, i.e. a vmcnt(0)
                 * wait that made the prefetch synchronous */
                if (PF == 0 && (LSF ? f + 1 < f1 : (gr == 0 || f + 1 < f1))) prefetch(LSF ? 2 * f + 2 : 2 * f + gr + 1, cs);
            }
            wave_sync();
#undef XV
            if (!SRC_XR) __builtin_amdgcn_s_setprio(0);
            /* ---------------- phase I: alias + IMDCT + overlap ------------ */
            if (PF == 2) { /* granule 0's overlap from the other wave */
                __syncthreads();
#pragma unroll
                for (int i = 0; i < 9; i++) ovp[i] = (f32x2){xch[2 * i * 64 + lane], xch[(2 * i + 1) * 64 + lane]};
            }
            const int bt = ch ? bt1 : bt0, mixed = ch ? mx1 : mx0;
            float o18[18];
            f32x2 nvp[9]; /* the next overlap (folded sign convention) */
            {
                const int base = ch * 576 + 18 * sb;
                /* the subband's lines and its neighbours' alias inputs,
                 * defined at the end of every phase-Q path (xin / the fused
                 * requantiser): one set of registers, no merge copies */
                float(&x)[18] = xf;
                (void)base;
                /* alias reduction (ISO 2.4.3.4): all 31 boundaries (long),
                 * the first one (mixed), none (short) */
                const bool upper = (bt != 2 && sb >= 1) || (bt == 2 && mixed && sb == 1);
                const bool lower = (bt != 2 && sb <= 30) || (bt == 2 && mixed && sb == 0);
                /* both butterflies computed, then selected: written as
                 * conditional stores the compiler built a divergent branch
                 * plus ~50 register copies around it */
                /* scalar: as packed pairs the operands need a register move
                 * each (they arrive as consecutive pairs from LDS; r03 AL1:
                 * with op_sel swizzles and LDS coefficient pairs -8 VALU but
                 * +3 VGPRs, 168 of 168) */
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const float lo = x[17 - k], hi = x[k];
                    const float nh = fmaf(up[k], MP3D_K_ALIAS_CA[k], hi * MP3D_K_ALIAS_CS[k]);
                    const float nl = fmaf(-dn[k], MP3D_K_ALIAS_CA[k], lo * MP3D_K_ALIAS_CS[k]);
                    x[k] = upper ? nh : hi;
                    x[17 - k] = lower ? nl : lo;
                }
                const bool long_imdct = bt != 2 || (mixed && sb < 2);
                if (long_imdct) {
                    /* packed window + overlap: pair i = output slots (i, 17 - i)
                     * from W[8 - i] = (w[8 - i], w[9 + i]) */
                    const f32x4 *wq = T.wp[sb & 1][bt == 2 ? 0 : bt];
                    f32x2 W[9];
                    /* the constants' LDS address from an opaque copy: the
                     * reads then take immediate offsets from ONE register
                     * (as absolute addresses the compiler held 8 of them live
                     * across the loop) */
                    imdct36_wp(x, W, (const f32x2 *)(uintptr_t)(uint32_t)opaque((int)(uintptr_t)(lds_cf32 *)(const float *)&T.kc[0]));
#pragma unroll
                    for (int i = 0; i < 9; i++) {
                        const f32x4 q = wq[i];
                        const f32x2 o = pfma(bc(W[8 - i].y), (f32x2){q.x, q.y}, ovp[i]);
                        o18[i] = o.x;
                        o18[17 - i] = o.y;
                        nvp[i] = bc(W[8 - i].x) * (f32x2){q.z, q.w};
                    }
                } else {
                    /* the odd-slot sign of odd subbands, from the granule's
                     * lane copy (held across the loop it spilled) */
                    const float sgo = (sb & 1) ? -1.f : 1.f;
                    const f32x2 sgp[2] = {(f32x2){1.f, sgo}, (f32x2){sgo, 1.f}};
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
                    /* true overlap in, slots in the folded sign convention out */
                    float ovt[18];
#pragma unroll
                    for (int i = 0; i < 9; i++) {
                        const f32x2 t = ovp[i] * sgp[i & 1];
                        ovt[i] = t.x;
                        ovt[17 - i] = t.y;
                    }
#pragma unroll
                    for (int i = 0; i < 18; i++) o18[i] = ((i < 6 ? 0.f : z[i - 6]) + ovt[i]) * ((i & 1) ? sgo : 1.f);
#pragma unroll
                    for (int i = 0; i < 9; i++)
                        nvp[i] = (f32x2){i < 12 ? z[12 + i] : 0.f, 17 - i < 12 ? z[29 - i] : 0.f} * sgp[i & 1];
                }
                /* overlap update: a mono frame's channel-1 lanes keep theirs
                 * (a per-lane select, on mono frames only: on the stereo
                 * path the select kept register copies alive) */
                if (nch == 2) {
#pragma unroll
                    for (int i = 0; i < 9; i++) ovp[i] = nvp[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 9; i++) {
                        ovp[i].x = lane_sel(amask, ovp[i].x, nvp[i].x);
                        ovp[i].y = lane_sel(amask, ovp[i].y, nvp[i].y);
                    }
                }
            }
            if (PF == 1) { /* granule 0's overlap for the other wave */
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    xch[2 * i * 64 + lane] = ovp[i].x;
                    xch[(2 * i + 1) * 64 + lane] = ovp[i].y;
                }
                __syncthreads();
            }
            /* a warm-up granule before the last one (frame-parallel
             * segments): only its IMDCT overlap is used (the next granule's S
             * reads it), so it skips S, phases M and W -- the synthesis
             * history is rebuilt from one granule's X alone, the last warm-up
             * granule's, and no warm-up output is stored */
            if (!SRC_XR && PF == 0 && f < wlast + (LSF || gr == 1 ? 0 : 1)) {
                WAIT_VMCNT0(); /* (phase W's drain: the next granule's prefetch has landed) */
                wave_sync();
                continue;
            }
            wave_sync(); /* every lane has read its xr before S overwrites it */
            {
                /* S row layout: subbands 0..15, then 31 down to 16, so the
                 * matrixing's mirror run S[31 - i] is in register order */
                const int sw = opaque(18 * ch * SROW + (sb < 16 ? sb : 47 - sb));
#pragma unroll
                for (int t = 0; t < 18; t++) sBuf[sw + t * SROW] = o18[t]; /* frequency inversion already in */
            }
            wave_sync();
            /* ---------------- phase M: matrixing on the matrix cores ------- */
            /* one butterfly level of the 32-point DCT-II (ISO Annex A matrixing):
             *   X[2m]   = sum_i C[2m][i]   (S_i + S_31-i)
             *   X[2m+1] = sum_i C[2m+1][i] (S_i - S_31-i),  i, m < 16
             * = two 16x16 products: half the MFMAs of the dense 32x32.
             * v_mfma_f32_16x16x4_f32, rows m, cols n = (ch, t), K order
             * i = 4 q + ks (q = lane >> 4): a lane's 4 B values and their
             * mirrors are two 16-B runs of an S row (the mirror run stored
             * reversed by phase I), so the butterfly is 2 + 2 packed ops. */
            {
                const int q = lane >> 4, r16 = lane & 15;
                const float4 ae = *(const float4 *)&T.ce[r16][4 * q];
                const float4 ao = *(const float4 *)&T.co[r16][4 * q];
                const float Ae[4] = {ae.x, ae.y, ae.z, ae.w}, Ao[4] = {ao.x, ao.y, ao.z, ao.w};
                float Be[3][4], Bo[3][4];
                typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
                const uint32_t sbase_ = (uint32_t)(uintptr_t)(lds_cf32 *)(const float *)sBuf;
                lds_f32x4 *const pA = (lds_f32x4 *)(uintptr_t)(sbase_ + m_off_a);
                lds_f32x4 *const pC = (lds_f32x4 *)(uintptr_t)(sbase_ + m_off_c);
#pragma unroll
                for (int nt = 0; nt < 3; nt++) {
                    lds_f32x4 *const pr = nt == 2 ? pC : pA + nt * (16 * SROW / 4);
                    const f32x4 a4 = pr[0];
                    const f32x4 b4 = pr[4]; /* S[31 - 4 q - ks] */
                    const f32x2 e01 = pfma(bc(1.f), a4.xy, b4.xy), e23 = pfma(bc(1.f), a4.zw, b4.zw);
                    const f32x2 o01 = pfma(bc(-1.f), b4.xy, a4.xy), o23 = pfma(bc(-1.f), b4.zw, a4.zw);
                    Be[nt][0] = e01.x; Be[nt][1] = e01.y; Be[nt][2] = e23.x; Be[nt][3] = e23.y;
                    Bo[nt][0] = o01.x; Bo[nt][1] = o01.y; Bo[nt][2] = o23.x; Bo[nt][3] = o23.y;
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
                /* D[row m = 4 q + r][col n]: X[n][2m] (even) at row n, 4 q + r;
                 * X[n][2m+1] (odd) at 16 + 4 q + r -- one 16-B store each */
                static_assert(XROW == SROW, "X rows reuse the S row offsets");
#pragma unroll
                for (int nt = 0; nt < 3; nt++) {
                    const int n = 16 * nt + r16;
                    if (n < 36) {
                        lds_f32x4 *const pr = nt == 2 ? pC : pA + nt * (16 * XROW / 4);
                        pr[0] = ce[nt];
                        pr[4] = co[nt];
                    }
                }
            }
            wave_sync();
            /* ---------------- phase W: 512-tap window -> PCM --------------- */
            /* Drain vmcnt HERE, before this granule's PCM stores: the next
             * granule's prefetch (issued in phase Q, then I and M ran) and the
             * previous granule's stores are long done, and with no load left
             * pending the compiler needs no wait after the stores.  (Its
             * waitcnt pass treats loads and stores pending together as out of
             * order and would otherwise emit vmcnt(0) right after them.) */
            if (!SRC_XR || XDMA) WAIT_VMCNT0();
            if (PF == 2) { /* granule 0's synthesis history from the other wave */
                __syncthreads();
#pragma unroll
                for (int tp = 0; tp < 8; tp++)
                    hp[tp] = (f32x2){xch[(18 + 2 * tp) * 64 + lane], xch[(19 + 2 * tp) * 64 + lane]};
            }
            {
                /* the lane's X columns in buf (wa / wb of output j, ISO Annex
                 * A matrixing folded to 32 outputs; X index k sits at (k & 1)
                 * 16 + k / 2 of its row), one table read each: held across the
                 * loop they spilled, recomputed they cost ~14 VALU a granule */
                const int pa = T.xcol[0][lane], pb = T.xcol[1][lane];
                /* loaded straight into the register pairs the packed FMAs
                 * take: xap[m] = (xa[2m], xa[2m + 1]), xbp[m] = (xb[2m + 1],
                 * xb[2m + 2]) (loaded as (xb[0], xb[1]), ... pairs, the odd
                 * pairing cost a register copy per value and, at 128 VGPRs,
                 * spills) */
                f32x2 xap[9], xbp[8];
                float xb0, xb17;
#pragma unroll
                for (int m = 0; m < 9; m++) xap[m] = (f32x2){sBuf[pa + 2 * m * XROW], sBuf[pa + (2 * m + 1) * XROW]};
                {
                    /* the shifted pairs (rows 2m + 1, 2m + 2) by ds_read2_b32
                     * straight into aligned register pairs, from three bases
                     * (offsets <= 255 words): as C the compiler paired rows
                     * (2m, 2m + 1) and rebuilt the pairs with 14 v_mov per
                     * granule (A/B WXB: -1 % k_synth, bit-identical) */
                    static_assert(XROW == 36, "xbp offsets below assume 36-word X rows");
                    const uint32_t ba = (uint32_t)(uintptr_t)(lds_cf32 *)&sBuf[pb];
                    const uint32_t bb = ba + 7u * 4u * XROW, bz = ba + 15u * 4u * XROW;
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:36 offset1:72" : "=v"(xbp[0]) : "v"(ba));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:108 offset1:144" : "=v"(xbp[1]) : "v"(ba));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:180 offset1:216" : "=v"(xbp[2]) : "v"(ba));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:0 offset1:36" : "=v"(xbp[3]) : "v"(bb));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:72 offset1:108" : "=v"(xbp[4]) : "v"(bb));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:144 offset1:180" : "=v"(xbp[5]) : "v"(bb));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:216 offset1:252" : "=v"(xbp[6]) : "v"(bb));
                    __asm__ volatile("ds_read2_b32 %0, %1 offset0:0 offset1:36" : "=v"(xbp[7]) : "v"(bz));
                }
                xb0 = sBuf[pb];
                xb17 = sBuf[pb + 17 * XROW];
                /* the compiler does not count the asm loads: this wait, with
                 * the pairs as its operands, orders every use after them */
                __asm__ volatile("s_waitcnt lgkmcnt(0)"
                                 : "+v"(xbp[0]), "+v"(xbp[1]), "+v"(xbp[2]), "+v"(xbp[3]), "+v"(xbp[4]), "+v"(xbp[5]),
                                   "+v"(xbp[6]), "+v"(xbp[7]));
                /* mono frame: channel 1 keeps its synthesis history.  Its
                 * lanes park their partial sums in the channel-1 half of the
                 * X buffer (rows 18..35, which only channel-1 lanes read, and
                 * after their own reads) and take them back below */
                const int park = opaque(18 * XROW + 16 * sb);
                if (nch == 1) {
                    if (ch == 1) {
#pragma unroll
                        for (int tp = 0; tp < 8; tp++) *(f32x2 *)&sBuf[park + 2 * tp] = hp[tp];
                    }
                }
                /* int16 sinks (taps pre-scaled by 32768): clamp(floor(x + 0.5)),
                 * FFmpeg's fixed-point rounding (round_sample: add half, shift),
                 * by one v_cvt_rpi_i32_f32 per sample: floor of the exact x + 0.5,
                 * saturating to int32 (tools/dbg/cvt_probe.hip) */
                auto to_i32 = [&](float v) {
                    int r;
                    __asm__("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
                    return r;
                };
                const int so = f * 2304 * PB + gr * 576 * nch * PB;
                /* output slots (2 tp, 2 tp + 1): lanes 0-31 hold L, lanes 32-63
                 * R; one half-wave swap leaves lane j with (L, R) of slot 2 tp
                 * and lane 32 + j with (L, R) of slot 2 tp + 1 */
                /* The stereo stores are non-temporal (cache policy nt): each
                 * instruction writes whole 128-B lines (256 / 512 B per wave)
                 * that no kernel reads again, and streaming them past the L2
                 * made the next step's demux -3 % and k_synth -0.5..1 % (C3,
                 * C5, C2; profiles/r06_ab_bounds.txt box 24, with the nt is[]
                 * loads above).  (k_huffman's is[] row stores must not be nt:
                 * their lines fill over several stores) */
                /* STEREO: a stereo frame past the warm-up (the common case):
                 * branch-free stores, so the window loop below is one basic
                 * block; otherwise the general sink (mono lanes, warm-up) */
                /* the lane's PCM byte offsets, once per granule (in the
                 * stores they were recomputed at each slot pair) */
                const int vo_st = opaque((sb + 32 * ch) * (F32 ? 8 : 4)), vo_mo = opaque(sb * (F32 ? 4 : 2));
                auto emit = [&](auto stereo, int tp, f32x2 o) {
                    if (decltype(stereo)::value) {
                        if (F32) {
                            /* float sink: the same sums, unscaled and unclipped
                             * (FFmpeg's float decoder convention); (L, R) = 8 B
                             * per lane and slot */
                            const int vo = vo_st;
                            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(o.x), __float_as_uint(o.y),
                                                                            false, false);
                            __builtin_amdgcn_raw_buffer_store_b64((u32x2){r[0], r[1]}, r_pcm, vo + 512 * tp, so, 2 /* nt */);
                        } else {
                            /* floor(x + 0.5) -> int32, then v_cvt_pk_i16_i32
                             * saturates to int16 and packs (L, R): 4 VALU per
                             * slot pair */
                            const int vo = vo_st;
                            const int p0 = to_i32(o.x), p1 = to_i32(o.y);
                            const auto r = __builtin_amdgcn_permlane32_swap(p0, p1, false, false);
                            __builtin_amdgcn_raw_buffer_store_b32(
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16((int)r[0], (int)r[1])), r_pcm,
                                vo + 256 * tp, so, 2 /* nt */);
                        }
                    } else if (f < f0) {
                        /* warm-up frame: state only, no PCM */
                    } else if (nch == 2) { /* (stereo frames take the other copy) */
                    } else if (ch == 0) { /* mono: channel 0's lanes */
                        if (F32) {
                            const int vo = vo_mo;
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o.x), r_pcm, vo + 256 * tp, so, 0);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o.y), r_pcm, vo + 256 * tp + 128, so, 0);
                        } else {
                            /* saturated by v_cvt_pk_i16_i32 (a v_med3 clamp held its
                             * 0x7fff bound in a VGPR across the loop) */
                            const int vo = vo_mo;
                            const uint32_t pk =
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(to_i32(o.x), to_i32(o.y)));
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)pk, r_pcm, vo + 128 * tp, so, 0);
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(pk >> 16), r_pcm, vo + 128 * tp + 64, so, 0);
                        }
                    }
                };
                /* The 512-tap window (ISO Annex A: 16 taps per output sample,
                 * alternately on columns wa and wb of the X FIFO), two output
                 * slots at a time with packed FMAs (v_pk_fma_f32, the tap
                 * broadcast).  Slot t = sum_i D[2i] A(t - 2i) + D[2i+1] B(t - 2i
                 * - 1) with A / B this granule's X (index >= 0) or the previous
                 * granule's (< 0).  Per slot ONE fma chain: the previous
                 * granule's terms (hp, taps i ascending) first, then this
                 * granule's (taps i ascending).  Step i (taps 2i, 2i + 1, read
                 * from LDS at the step) advances the slot pairs tp >= i and
                 * completes pair i (stored at once), and sums this granule's
                 * terms of the NEXT granule's pairs tp < i into hp (pair i
                 * starts there): at every step 9 pairs (18 registers) are live,
                 * and the 9 chains are independent. */
                auto window = [&](auto stereo) {
                    f32x2 acc[9];
#pragma unroll
                    for (int tp = 0; tp < 8; tp++) acc[tp] = hp[tp];
                    acc[8] = (f32x2){0.f, 0.f};
                    const int dwo = opaque(sb);
                    /* the taps of step i + 1 are read at the start of step i
                     * (one step ahead, 2 registers): read at their own step,
                     * each step waited for its LDS read */
                    f32x2 dn = (&T.dwp[0][0])[dwo];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const f32x2 d = dn;
                        if (i < 7) dn = (&T.dwp[0][0])[dwo + 32 * (i + 1)];
#pragma unroll
                        for (int tp = i; tp < 9; tp++) {
                            /* A = (xa[k], xa[k + 1]), B = (xb[k - 1], xb[k]), k = 2 (tp - i) */
                            acc[tp] = pfma(bc(d.x), xap[tp - i], acc[tp]);
                            if (tp > i)
                                acc[tp] = pfma(bc(d.y), xbp[tp - i - 1], acc[tp]);
                            else /* slot 2 tp + 1's B(0); slot 2 tp's B(-1) is in hp */
                                acc[tp].y = fmaf(d.y, xb0, acc[tp].y);
                        }
                        emit(stereo, i, acc[i]);
                        hp[i] = (f32x2){d.y * xb17, 0.f}; /* H_2i: B(-1) = this X_17 */
#pragma unroll
                        for (int tp = 0; tp < i; tp++) {
                            /* k = 2 (tp - i) + 18: A = xap[k / 2], B = xbp[k / 2 - 1] */
                            hp[tp] = pfma(bc(d.x), xap[tp - i + 9], hp[tp]);
                            hp[tp] = pfma(bc(d.y), xbp[tp - i + 8], hp[tp]);
                        }
                    }
                    emit(stereo, 8, acc[8]);
                };
                if (nch == 2 && f >= f0)
                    window(BoolC<true>{});
                else
                    window(BoolC<false>{});
                if (nch == 1) {
                    wave_sync();
#pragma unroll
                    for (int tp = 0; tp < 8; tp++) {
                        const f32x2 v = *(const f32x2 *)&sBuf[park + 2 * tp];
                        hp[tp].x = lane_sel(amask, v.x, hp[tp].x);
                        hp[tp].y = lane_sel(amask, v.y, hp[tp].y);
                    }
                }
                if (PF == 1) {
#pragma unroll
                    for (int tp = 0; tp < 8; tp++) {
                        xch[(18 + 2 * tp) * 64 + lane] = hp[tp].x;
                        xch[(19 + 2 * tp) * 64 + lane] = hp[tp].y;
                    }
                    __syncthreads();
                }
            }
            wave_sync(); /* X reads done before the next granule's xr */
        }
    }
    /* state out: the stream's last segment.  With several segments the
     * first one may still be reading the state, so it goes to st_tail (the
     * overlap + fifo tail of StreamState, packed per stream): the next
     * synth-only call reads it from there (st_tail_in), any other use of the
     * handle first copies it into StreamState (mp3d_host.cpp flush_tail). */
    if (f1 == F && PF != 1) {
        const int lane = opaque((int)(threadIdx.x & 63)); /* lane values re-derived: not held across the loop */
        const int ch = lane >> 5, sb = lane & 31;
        const float sgo = (sb & 1) ? -1.f : 1.f;
        const f32x2 sgp[2] = {(f32x2){1.f, sgo}, (f32x2){sgo, 1.f}};
        float *ovo = st_tail ? st_tail + (size_t)s * TAIL : &S.overlap[0][0][0];
        float *ffo = ovo + sizeof(S.overlap) / 4;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const f32x2 t = ovp[i] * sgp[i & 1];
            ovo[(ch * 32 + sb) * 18 + i] = t.x;
            ovo[(ch * 32 + sb) * 18 + 17 - i] = t.y;
        }
        const float hsc = F32 ? 1.0f : 1.0f / 32768.0f; /* to float-sink units (exact) */
#pragma unroll
        for (int tp = 0; tp < 8; tp++) {
            ffo[(ch * MP3D_FIFO_SLOTS + 2 * tp) * 32 + sb] = hp[tp].x * hsc;
            if (2 * tp + 1 < MP3D_FIFO_SLOTS) ffo[(ch * MP3D_FIFO_SLOTS + 2 * tp + 1) * 32 + sb] = hp[tp].y * hsc;
        }
    }
}

/* streams (waves) per k_synth workgroup: the MPEG-1 decode runs 8 (two
 * workgroups = 4 waves per SIMD, the tables shared by 8 waves leave LDS for
 * the is[] prefetch areas); the synth-only and LSF variants run 4 at 3 waves
 * per SIMD */
template <bool SRC_XR, bool LSF> struct SynCfg {
    static constexpr bool DMA = !LSF; /* is[] (decode) or channel-0 spectra (synth only) by LDS-DMA */
    static constexpr int WAVES = DMA ? 8 : 4;
};

template <bool SRC_XR, bool F32, bool LSF>
/* MPEG-1 decode and synth only: 4 waves / SIMD (<= 128 VGPRs), the next
 * granule's is[] words or channel-0 spectra prefetched by LDS-DMA into the
 * wave's isq area; LSF: 3 waves / SIMD (168 VGPRs).  (Round 2: without any
 * prefetch the synth-only entry fitted 4 waves but was slower than 3 waves
 * with it, A/B XPF3 / XPF4.) */
__global__ void __launch_bounds__((64 * SynCfg<SRC_XR, LSF>::WAVES))
    __attribute__((amdgpu_waves_per_eu(SynCfg<SRC_XR, LSF>::DMA ? 4 : 3, 8)))
k_synth(const FrameRec *__restrict__ rec, const int16_t *__restrict__ is_buf, const UnitMeta *__restrict__ meta,
        const float *__restrict__ xr_in, const uint8_t *__restrict__ xr_bt, const uint8_t *__restrict__ xr_mixed,
        const DevTables *__restrict__ tab, StreamState *__restrict__ st, void *__restrict__ pcm, int n_streams,
        int F, int xr_nch, int xr_sr, int seg_len, float *__restrict__ st_tail,
        const float *__restrict__ st_tail_in, const uint32_t *__restrict__ fam, uint32_t seq) {
    constexpr int SYN_WAVES = SynCfg<SRC_XR, LSF>::WAVES;
    /* one LDS object in a fixed order: the per-wave buffers at 0 (their
     * row offsets then fit ds_read2's 8-bit offsets from the wave's base),
     * the shared tables next and below 64 KB (every table address fits a
     * DS instruction's 16-bit offset; as separate variables the compiler
     * placed them last, above 64 KB: a v_add per table read), the is[]
     * prefetch areas last */
    struct Lds {
        float pad_[64]; /* xin's look-back of wave 0, subband 0 (words it does not use) */
        SynWave Wv[SYN_WAVES];
        SynShared<LSF> T;
        uint32_t isq[SynCfg<SRC_XR, LSF>::DMA ? SYN_WAVES : 1][2 * 320];
    };
    static_assert(offsetof(Lds, T) + sizeof(SynShared<LSF>) <= 65536, "k_synth: tables within DS offset reach");
    /* two MPEG-1 workgroups per CU (4 waves per SIMD): <= half of the CU's 160 KB */
    static_assert(LSF || SRC_XR || sizeof(Lds) <= 160 * 1024 / 2, "k_synth: LDS for two workgroups per CU");
    __shared__ __attribute__((aligned(16))) Lds L;
    SynShared<LSF> &T = L.T;
    SynWave *Wv = L.Wv;
    auto &s_isq = L.isq;
    /* LSF variant of a batch decode (fam given): k_walk tagged the family
     * word with this call's seq if any stream is LSF; otherwise the whole
     * (small, persistent) grid leaves at once.  With LSF streams each
     * workgroup walks blocks blockIdx.x, + gridDim.x, ... */
    if (LSF && !SRC_XR && fam && *fam != seq) return;
    if (!SRC_XR && !(LSF && fam)) {
        /* one variant per MPEG family (StreamState.kind, fixed by k_demux):
         * MPEG-1 takes kinds 0 / 1, LSF kind 2.  A workgroup holding no
         * stream of its variant leaves before staging any table (the same
         * decision in every lane: no barrier is skipped by part of it). */
        bool any = false;
        const int nsg = (F + seg_len - 1) / seg_len;
#pragma unroll
        for (int k = 0; k < SYN_WAVES; k++) {
            const int sk = (blockIdx.x * SYN_WAVES + k) / nsg;
            if (sk < n_streams) any |= (st[sk].kind == 2) == LSF;
        }
        if (!any) return;
    }
    synth_tables<F32, LSF, 64 * SYN_WAVES>(T, tab, threadIdx.x);
    __syncthreads();
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); /* wave-uniform (SGPR) */
    const int nseg = (F + seg_len - 1) / seg_len;
    const int nblk = (n_streams * nseg + SYN_WAVES - 1) / SYN_WAVES;
    /* one block, or (LSF variant, persistent grid) blocks blockIdx.x +
     * k gridDim.x; the loop only there: around the 4-wave variants' bodies
     * it held loop-invariant addresses across the stream and spilled */
    auto run = [&](int blk) {
        const int vs = blk * SYN_WAVES + wid;
        if (vs >= n_streams * nseg) return false; /* after the only workgroup barrier */
        const int s = vs / nseg, seg = vs - s * nseg;
        if (!SRC_XR && (st[s].kind == 2) != LSF) return true; /* the other variant's stream */
        synth_stream<SRC_XR, F32, LSF>(rec, is_buf, meta, xr_in, xr_bt, xr_mixed, tab, st, pcm, F, xr_nch, xr_sr,
                                       seg_len, st_tail, st_tail_in, T, Wv[wid], s, seg, nseg, nullptr,
                                       SynCfg<SRC_XR, LSF>::DMA ? s_isq[SynCfg<SRC_XR, LSF>::DMA ? wid : 0] : nullptr);
        return true;
    };
    if constexpr (LSF && !SRC_XR) {
        for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x)
            if (!run(blk)) break;
    } else {
        run(blockIdx.x);
    }
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
/* k_frame: the per-frame decoder's call (mp3d_decode_frame) in ONE launch  */
/* of one 256-thread workgroup.  Wave 0 stages the frame from the caller's */
/* mapped pinned buffer into LDS (one bus round trip) and demuxes it        */
/* (demux_stream, input from LDS) while waves 1-3 stage the Huffman and     */
/* synthesis tables; then the four waves decode the frame's granule         */
/* channels (huffman_wave_unit), waves 0 and 1 synthesise the PCM of one   */
/* granule each (MPEG-1; one wave for LSF) straight into the mapped output */
/* (synth_stream PF = 1, 2) and wave 0, after a system-scope fence, writes  */
/* the call's sequence number into a mapped completion word the host polls  */
/* (no stream synchronisation).  The hand-offs between the phases use the   */
/* batch's device buffers exactly as the three-kernel path does, so the     */
/* results are the same bit for bit (tests/test_gpu_per_frame.py).          */
/* ------------------------------------------------------------------------ */
#define PF_BYTES 4096 /* = MP3D_PF_BYTES (mp3d_host.cpp): the staged stream length */

template <bool F32, bool LSF>
__global__ void __launch_bounds__(256) k_frame(const uint8_t *__restrict__ in_host, uint32_t in_have,
                                               const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ in_len,
                                               uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off,
                                               StreamState *__restrict__ st, FrameRec *__restrict__ rec,
                                               uint64_t *__restrict__ sideu, DevInfo *__restrict__ infos, int opts,
                                               const DevTables *__restrict__ tab, int16_t *__restrict__ is_buf,
                                               UnitMeta *__restrict__ meta, void *__restrict__ pcm,
                                               uint32_t *__restrict__ done, uint32_t seq) {
    __shared__ __attribute__((aligned(16))) SynShared<LSF> T;
    /* a pad below wave 0's buffer: xin's look-back of subband 0 */
    __shared__ struct {
        float pad_[64];
        SynWave w[2];
    } WvP;
    SynWave *const Wv = WvP.w;
    __shared__ float s_xch[47 * 64]; /* granule 0 -> 1 hand-off: overlap (18), history (14 + 15) per lane */
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[MP3D_LUT_MAX];
    __shared__ __attribute__((aligned(16))) uint32_t s_bits[HW_UNITS][HW_WORDS + 4];
    __shared__ uint32_t s_tsel[32];
    __shared__ uint16_t s_lbnd[9][24];
    __shared__ uint8_t s_slen[32];
    __shared__ __attribute__((aligned(16))) uint32_t s_in[PF_BYTES / 4];
    static_assert(PF_BYTES == 256 * 16 && MP3D_MAX_FRAME_BYTES <= 128 * 16, "k_frame: frame staging by wave 0");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wv == 0) {
        /* wave 0: the stream state's first lines into the cache (the demux
         * reads them after the frame has arrived), then the frame's bytes
         * [0, in_have) from the mapped buffer, 16 B per lane and chunk (one
         * bus round trip), zeros after them (the host does not clear the
         * pinned buffer's tail); then the demux, reading the frame from LDS
         * (the wave's own stores: no barrier) */
        const uint4 sp = ((const uint4 *)st)[lane];
        __asm__ volatile("" ::"v"(sp.x), "v"(sp.y), "v"(sp.z), "v"(sp.w));
        const uint32_t n16 = (in_have + 15u) / 16u; /* <= 91 (1441-B frame) */
        uint4 v[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t c = (uint32_t)lane + 64u * k;
            v[k] = c < n16 ? ((const uint4 *)in_host)[c] : make_uint4(0u, 0u, 0u, 0u);
            if (c + 1u == n16 && (in_have & 15u)) {
                /* bytes past in_have inside the last chunk read as zeros */
                const uint32_t keep = in_have & 15u;
                uint32_t *w = (uint32_t *)&v[k];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int nb = (int)keep - 4 * q; /* bytes of word q kept */
                    w[q] = nb >= 4 ? w[q] : nb <= 0 ? 0u : w[q] & (0xFFFFFFFFu >> (32 - 8 * nb));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) ((uint4 *)s_in)[lane + 64 * k] = k < 2 ? v[k] : make_uint4(0u, 0u, 0u, 0u);
        wave_sync();
        demux_stream<SrcLds>((SrcLds::u8 *)(uintptr_t)s_in + in_off[0], in_off[0], in_len[0], md, md_off, st, rec, sideu,
                             infos, 1, opts, 0, lane);
    } else {
        /* waves 1..3 meanwhile: the Huffman and synthesis tables */
        huff_tables<192>(tab, s_lut, s_tsel, s_lbnd, s_slen, tid - 64);
        synth_tables<F32, LSF, 192>(T, tab, tid - 64);
    }
    __syncthreads(); /* rec, side words, md region and state visible to the workgroup */
    huffman_wave_unit(md, md_off, rec, sideu, tab, is_buf, meta, 1, wv, lane, s_bits[wv], s_lut, s_tsel, s_lbnd,
                      s_slen);
    __syncthreads(); /* is[] rows and UnitMeta visible to the synthesis waves */
    /* a frame of the other MPEG family than the stream's was skipped as
     * junk by the demux: no audio (as k_synth's variant check) */
    const bool fam = (st[0].kind == 2) == LSF;
    const FrameRec r0 = rec[0];
    /* MPEG-1 frame with audio: wave 0 synthesises granule 0 and wave 1
     * granule 1 side by side (synth_stream PF = 1, 2): wave 1 requantises
     * its granule while wave 0 runs granule 0's phases Q and I, takes
     * granule 0's IMDCT overlap at the first barrier and its synthesis
     * history at the second.  Same operations in the same order per value
     * as one wave doing both granules, so bit-identical.  The condition is
     * the one under which synth_stream decodes the frame (so every wave
     * meets the same two barriers). */
    const bool split = !LSF && fam && r0.frame_bytes && !(r0.first_gr & (REC_TAG | REC_DROP));
    if constexpr (!LSF) if (split) {
        if (wv == 0)
            synth_stream<false, F32, LSF, 1>(rec, is_buf, meta, nullptr, nullptr, nullptr, tab, st, pcm, 1, 2, 0, 1,
                                             nullptr, nullptr, T, Wv[0], 0, 0, 1, s_xch);
        else if (wv == 1)
            synth_stream<false, F32, LSF, 2>(rec, is_buf, meta, nullptr, nullptr, nullptr, tab, st, pcm, 1, 2, 0, 1,
                                             nullptr, nullptr, T, Wv[1], 0, 0, 1, s_xch);
        else {
            __syncthreads();
            __syncthreads();
        }
        if (wv == 1) __threadfence_system(); /* granule 1's PCM and the state, before the barrier */
        __syncthreads();
    }
    if (!split && wv == 0 && fam) {
        synth_stream<false, F32, LSF>(rec, is_buf, meta, nullptr, nullptr, nullptr, tab, st, pcm, 1, 2, 0, 1, nullptr,
                                      nullptr, T, Wv[0], 0, 0, 1);
    }
    if (wv == 0) {
        __threadfence_system(); /* PCM, frame info and state before the completion word */
        if (lane == 0) __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* ------------------------------------------------------------------------ */
/* Host-side launchers                                                       */
/* ------------------------------------------------------------------------ */
hipError_t upload_synth_constants(const float *win36, const float *is_ratio, const float *pow2q, const float *is_lsf) {
    hipError_t e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_win36), win36, sizeof(float) * 4 * 36))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_is_ratio), is_ratio, sizeof(float) * 14))) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_pow2q), pow2q, sizeof(float) * 4))) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_is_lsf), is_lsf, sizeof(float) * 64);
}

/* k_frame's copies of the demux constants (this translation unit's) */
hipError_t upload_frame_constants(const uint16_t *frame_bytes) { return upload_demux_tables(frame_bytes); }

void launch_frame(const uint8_t *in_host, uint32_t in_have, const uint64_t *in_off, const uint32_t *in_len,
                  uint8_t *md, const uint64_t *md_off, StreamState *st, FrameRec *rec, uint64_t *sideu, void *infos,
                  int opts, const DevTables *tab, int16_t *is_buf, UnitMeta *meta, void *pcm, bool f32, bool lsf,
                  uint32_t *done, uint32_t seq, hipStream_t strm) {
#define MP3D_FRAME_LAUNCH(F32_, LSF_)                                                                              \
    hipLaunchKernelGGL((k_frame<F32_, LSF_>), dim3(1), dim3(256), 0, strm, in_host, in_have, in_off, in_len, md,    \
                       md_off, st, rec, sideu, (DevInfo *)infos, opts, tab, is_buf, meta, pcm, done, seq)
    if (f32) {
        if (lsf) MP3D_FRAME_LAUNCH(true, true);
        else MP3D_FRAME_LAUNCH(true, false);
    } else {
        if (lsf) MP3D_FRAME_LAUNCH(false, true);
        else MP3D_FRAME_LAUNCH(false, false);
    }
#undef MP3D_FRAME_LAUNCH
}

/* seg_len < F: frame-parallel segments (one wave each, warm-up frames
 * before each; synth_stream); the final overlap + fifo then go to st_tail
 * (st_tail_in, when given, holds the streams' state in place of st) */
void launch_synth(const FrameRec *rec, const int16_t *is_buf, const UnitMeta *meta, const DevTables *tab,
                  StreamState *st, void *pcm, bool f32, int n_streams, int F, int kinds, int seg_len, float *st_tail,
                  const float *st_tail_in, const uint32_t *fam, uint32_t seq, int n_cu, hipStream_t strm) {
    const int waves = n_streams * ((F + seg_len - 1) / seg_len);
    /* the family variants in `kinds` (bit 0 MPEG-1, bit 1 LSF; a batch
     * launches both); a workgroup without a stream of its variant exits
     * after its streams' scalar loads.  With the family word (fam, seq; wide
     * demux) the LSF variant runs a persistent grid of one resident round
     * (3 workgroups of 4 waves per CU at 3 waves / SIMD) that all leave at
     * once on an all-MPEG-1 batch (its 16 384 workgroups' dispatch and loads
     * cost 39 us per C3 step) */
    const int lsf_grid = 3 * (n_cu > 0 ? n_cu : 256);
#define MP3D_SYNTH_LAUNCH(F32_, LSF_)                                                                              \
    do {                                                                                                           \
        constexpr int NW = SynCfg<false, LSF_>::WAVES;                                                             \
        int nb = (waves + NW - 1) / NW;                                                                            \
        if (LSF_ && fam && nb > lsf_grid) nb = lsf_grid;                                                           \
        hipLaunchKernelGGL((k_synth<false, F32_, LSF_>), dim3(nb), dim3(64 * NW), 0, strm, rec, is_buf, meta,       \
                           (const float *)nullptr, (const uint8_t *)nullptr, (const uint8_t *)nullptr, tab, st, pcm,  \
                           n_streams, F, 2, 0, seg_len, st_tail, st_tail_in, LSF_ ? fam : nullptr, seq);           \
    } while (0)
    if (f32) {
        if (kinds & 1) MP3D_SYNTH_LAUNCH(true, false);
        if (kinds & 2) MP3D_SYNTH_LAUNCH(true, true);
    } else {
        if (kinds & 1) MP3D_SYNTH_LAUNCH(false, false);
        if (kinds & 2) MP3D_SYNTH_LAUNCH(false, true);
    }
#undef MP3D_SYNTH_LAUNCH
}

/* seg_len < F: frame-parallel segments (k_synth); st_tail then receives the
 * streams' final overlap + fifo, which the caller copies into st */
void launch_synth_xr(const float *xr, const uint8_t *bt, const uint8_t *mixed, const DevTables *tab, StreamState *st,
                     int16_t *pcm, int n_streams, int F, int nch, int sr, int seg_len, float *st_tail,
                     const float *st_tail_in, hipStream_t strm) {
    const int waves = n_streams * ((F + seg_len - 1) / seg_len);
    constexpr int NW = SynCfg<true, false>::WAVES;
    hipLaunchKernelGGL((k_synth<true, false, false>), dim3((waves + NW - 1) / NW), dim3(64 * NW), 0,
                       strm, (const FrameRec *)nullptr, (const int16_t *)nullptr, (const UnitMeta *)nullptr, xr, bt,
                       mixed, tab, st, (void *)pcm, n_streams, F, nch, sr, seg_len, st_tail, st_tail_in,
                       (const uint32_t *)nullptr, 0u);
}

/* MP3D_DEBUG_POISON only (mp3d_host.cpp poison_env): fill the whole LDS of
 * every CU with 0xFF before each of the handle's launches, so the first
 * workgroup the next kernel places on a CU finds all-ones words (NaN as
 * float) in any LDS it reads before writing, on every run -- not whatever
 * the previous kernel on that CU left.  160 KB per workgroup, so one per CU
 * at a time; 4 per CU. */
#define LDS_POISON_WORDS (160 * 1024 / 4)
__global__ void __launch_bounds__(1024) k_lds_poison() {
    __shared__ uint32_t s[LDS_POISON_WORDS];
    /* volatile: LDS is dead at kernel end, so plain stores are removed */
    volatile uint32_t *v = s;
    for (int i = threadIdx.x; i < LDS_POISON_WORDS; i += 1024) v[i] = 0xFFFFFFFFu;
}

void launch_lds_poison(int n_cu, hipStream_t strm) {
    hipLaunchKernelGGL(k_lds_poison, dim3(4 * (n_cu > 0 ? n_cu : 256)), dim3(1024), 0, strm);
}

void launch_gather_frames(const void *src, void *dst, const void *isrc, void *idst, const int *a, int L, int F, int k0,
                          int n_out, int bytes_per_row, hipStream_t strm) {
    hipLaunchKernelGGL(k_gather_frames, dim3(n_out), dim3(256), 0, strm, (const uint4 *)src, (uint4 *)dst,
                       (const DevInfo *)isrc, (DevInfo *)idst, a, L, F, k0, bytes_per_row / 16);
}

} // namespace mp3d
