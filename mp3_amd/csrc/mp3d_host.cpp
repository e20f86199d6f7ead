/*
 * mp3d_host.cpp -- host side of the MI355X MP3 decoder: the C ABI declared
 * in include/mp3d.h, constant-table construction (ISO 11172-3 Annex B and
 * 2.4.3.4 formulas), batch buffer management and kernel launches.
 *
 * No CPU decode path exists here: every frame is decoded by the HIP kernels
 * in mp3d_demux.hip, mp3d_huffman.hip and mp3d_synth.hip; without a device
 * the create calls fail.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mp3d.h"
#include "mp3d_internal.h"
#include "mp3d_tables.h"
#include "mp3d_consts.h"
#include "mp3d_hostparse.h"

namespace mp3d {
hipError_t upload_synth_constants(const float *, const float *, const float *, const float *);
hipError_t upload_demux_constants(const uint16_t *);
void launch_demux(const uint8_t *, const uint64_t *, const uint32_t *, uint8_t *, const uint64_t *, StreamState *,
                  FrameRec *, uint64_t *, void *, int, int, int, bool, uint32_t *, uint32_t, hipStream_t);
void launch_demux_fp(const uint8_t *, uint32_t, const uint32_t *, uint8_t *, StreamState *, const float *,
                     StreamState *, FrameRec *, uint64_t *, void *, int, int, hipStream_t);
void launch_huffman(const uint8_t *, const uint64_t *, const FrameRec *, const uint64_t *, const DevTables *, int16_t *,
                    UnitMeta *, int, int, int, bool, uint32_t *, uint32_t *, hipStream_t);
void launch_synth(const FrameRec *, const int16_t *, const UnitMeta *, const DevTables *, StreamState *, void *, bool, int,
                  int, int, int, float *, const float *, const uint32_t *, uint32_t, int, hipStream_t);
void launch_synth_xr(const float *, const uint8_t *, const uint8_t *, const DevTables *, StreamState *, int16_t *, int,
                     int, int, int, int, float *, const float *, hipStream_t);
void launch_gather_frames(const void *, void *, const void *, void *, const int *, int, int, int, int, int,
                          hipStream_t);
hipError_t upload_frame_constants(const uint16_t *);
void launch_lds_poison(int, hipStream_t);
void launch_frame(const uint8_t *, uint32_t, const uint64_t *, const uint32_t *, uint8_t *, const uint64_t *,
                  StreamState *, FrameRec *, uint64_t *, void *, int, const DevTables *, int16_t *, UnitMeta *, void *,
                  bool, bool, uint32_t *, uint32_t, hipStream_t);
} // namespace mp3d

using namespace mp3d;

static thread_local int g_last_hip = 0;
#define HIPCHK(x)                                                                                                      \
    do {                                                                                                               \
        hipError_t _e = (x);                                                                                           \
        if (_e != hipSuccess) {                                                                                        \
            g_last_hip = (int)_e;                                                                                      \
            return _e == hipErrorOutOfMemory ? MP3D_E_NOMEM : MP3D_E_HIP;                                              \
        }                                                                                                              \
    } while (0)

/* ------------------------------------------------------------------------ */
/* Constant tables                                                          */
/* ------------------------------------------------------------------------ */
static void build_huffman_lut(DevTables &t) {
    /* two-level LUT: first level min(8, maxlen) bits; codes longer than that
     * go through one sub-table per first-level prefix (mp3d_internal.h) */
    std::vector<uint16_t> lut;
    const uint16_t UNUSED = 0xFFFF;
    for (int ti = 0; ti < MP3D_LUT_TABLES; ti++) {
        std::vector<uint32_t> code, len, val;
        if (ti < MP3D_NUM_HTABS) {
            int n = MP3D_HTAB_ROWLEN[ti];
            for (int x = 0; x < n; x++)
                for (int y = 0; y < n; y++) {
                    code.push_back(MP3D_HTAB_CODES[ti][x * n + y]);
                    len.push_back(MP3D_HTAB_LENS[ti][x * n + y]);
                    val.push_back((uint32_t)(x << 4 | y));
                }
        } else {
            for (int v = 0; v < 16; v++) {
                code.push_back(MP3D_QUAD_CODE[0][v]);
                len.push_back(MP3D_QUAD_LEN[0][v]);
                val.push_back((uint32_t)v);
            }
        }
        uint32_t maxlen = *std::max_element(len.begin(), len.end());
        int b1 = (int)std::min<uint32_t>(8, maxlen);
        if (lut.size() & 1) lut.push_back(UNUSED);
        size_t base = lut.size();
        t.lut_hdr.base[ti] = (uint16_t)base;
        t.lut_hdr.bits1[ti] = (uint8_t)b1;
        lut.resize(base + (1u << b1), UNUSED);
        std::vector<int> subbits(1u << b1, 0);
        for (size_t i = 0; i < code.size(); i++)
            if ((int)len[i] > b1) {
                uint32_t p = code[i] >> (len[i] - b1);
                subbits[p] = std::max(subbits[p], (int)len[i] - b1);
            }
        std::vector<size_t> subbase(1u << b1, 0);
        for (uint32_t p = 0; p < (1u << b1); p++)
            if (subbits[p]) {
                while (lut.size() & 3) lut.push_back(UNUSED); /* sub-tables 4-entry aligned */
                const size_t abs4 = lut.size() / 4;
                if (abs4 > 0x7FF || subbits[p] > 15) {
                    fprintf(stderr, "mp3d: LUT pointer overflow\n");
                    abort();
                }
                subbase[p] = lut.size();
                lut.resize(lut.size() + (1u << subbits[p]), UNUSED);
                lut[base + p] = (uint16_t)(0x8000u | ((uint32_t)subbits[p] << 11) | (uint32_t)abs4);
            }
        for (size_t i = 0; i < code.size(); i++) {
            /* big_values leaves: bits 13 / 14 flag x != 0 / y != 0 (a sign bit follows) */
            const uint32_t sgn = ti < MP3D_NUM_HTABS ? ((val[i] >> 4) != 0) << 13 | ((val[i] & 15) != 0) << 14 : 0u;
            uint16_t leaf = (uint16_t)((len[i] << 8) | val[i] | sgn);
            if ((int)len[i] <= b1) {
                uint32_t first = code[i] << (b1 - len[i]), cnt = 1u << (b1 - len[i]);
                for (uint32_t k = 0; k < cnt; k++) lut[base + first + k] = leaf;
            } else {
                uint32_t p = code[i] >> (len[i] - b1);
                int nb = subbits[p];
                uint32_t rest = code[i] & ((1u << (len[i] - b1)) - 1);
                uint32_t first = rest << (nb - (len[i] - b1)), cnt = 1u << (nb - (len[i] - b1));
                for (uint32_t k = 0; k < cnt; k++) lut[subbase[p] + first + k] = leaf;
            }
        }
    }
    if (lut.size() > MP3D_LUT_MAX) {
        fprintf(stderr, "mp3d: LUT overflow %zu\n", lut.size());
        abort();
    }
    for (size_t i = 0; i < lut.size(); i++) t.lut[i] = lut[i] == UNUSED ? (uint16_t)(1u << 8) : lut[i];
    /* table_select 0, 4, 14: a 2-entry all-zero table (zero-length leaves)
     * right after the last table (t.lut is zeroed past lut.size()) */
    const size_t zbase = (lut.size() + 1) & ~(size_t)1;
    if (zbase + 2 + 16 > MP3D_LUT_MAX) { /* + count1 table B in k_huffman's LDS copy */
        fprintf(stderr, "mp3d: LUT overflow %zu\n", zbase + 2);
        abort();
    }
    for (int i = 0; i < 32; i++) {
        const int ti = MP3D_HTAB_OF_SELECT[i];
        t.tsel[i] = ti < 0 ? (uint32_t)zbase | (1u << 16) | (1u << 20)
                           : (uint32_t)t.lut_hdr.base[ti] | ((uint32_t)t.lut_hdr.bits1[ti] << 16) |
                                 ((uint32_t)MP3D_LINBITS[i] << 24);
    }
    for (int sr = 0; sr < 9; sr++) {
        int acc = 0;
        for (int b = 0; b < 22; b++) {
            t.lbnd[sr][b] = (uint16_t)acc;
            acc += MP3D_SFB_LONG_WIDTH[sr][b];
        }
        t.lbnd[sr][22] = (uint16_t)acc;
    }
}

static_assert(offsetof(DevTables, lut) % 16 == 0, "k_huffman stages the LUT in 16-B loads");
static void build_tables(DevTables &t) {
    memset(&t, 0, sizeof(t));
    for (int i = 0; i < 8208; i++) t.pow43[i] = (float)pow((double)i, 4.0 / 3.0);
    for (int m = 0; m < 32; m++)
        for (int k = 0; k < 32; k++) t.dct_c[m][k] = (float)cos(m * (2 * k + 1) * M_PI / 64.0);
    double D[512];
    for (int i = 0; i <= 256; i++) {
        double v = MP3D_SYNTH_WINDOW_Q16[i] / 65536.0;
        D[i] = v;
        if (i > 0) D[512 - i] = (i % 64) ? -v : v;
    }
    for (int j = 0; j < 32; j++) {
        int a, sa, b, sbn = -1;
        if (j < 16) { a = 16 + j; sa = 1; b = 16 - j; }
        else if (j == 16) { a = 0; sa = 0; b = 0; }
        else { a = 48 - j; sa = -1; b = j - 16; }
        t.win_a[j] = (uint8_t)a;
        t.win_b[j] = (uint8_t)b;
        for (int i = 0; i < 8; i++) {
            t.dwin[j][2 * i] = (float)(sa * D[64 * i + j]);
            t.dwin[j][2 * i + 1] = (float)(sbn * D[64 * i + 32 + j]);
        }
    }
    for (int sr = 0; sr < 9; sr++) {
        /* mixed blocks: long bands below line 36 (72 at MPEG-2.5 8 kHz, whose
         * bands are twice as wide): 8 MPEG-1 bands, 6 LSF bands (FFmpeg) */
        const int mix_end = sr == 8 ? 72 : 36;
        int lb[576], sidx[576], sdst[576];
        int l = 0;
        for (int b = 0; b < 22; b++)
            for (int n = 0; n < MP3D_SFB_LONG_WIDTH[sr][b]; n++) lb[l++] = b;
        int p = 0;
        for (int b = 0; b < 13; b++) {
            int w = MP3D_SFB_SHORT_WIDTH[sr][b];
            for (int off = 0; off < 3 * w; off++) {
                int win = off / w, f = off % w;
                sidx[p + off] = 22 + 3 * b + win;
                sdst[p + off] = p + 3 * f + win;
            }
            p += 3 * w;
        }
        for (int k = 0; k < 288; k++) {
            for (int v = 0; v < 3; v++) {
                int band[2], pos[2];
                for (int e = 0; e < 2; e++) {
                    const int i = 2 * k + e;
                    const bool lng = v == 0 || (v == 2 && i < mix_end);
                    band[e] = lng ? lb[i] : sidx[i];
                    pos[e] = lng ? i : sdst[i];
                }
                if (band[0] != band[1]) abort(); /* odd band width: impossible (ISO tables) */
                t.lpair[sr][v][k] = (uint32_t)(4 * band[0]) | (uint32_t)pos[0] << 8 | (uint32_t)pos[1] << 18;
            }
        }
    }
    build_huffman_lut(t);
}

static int upload_symbols() {
    float imdct12[6][6], win36[4][36], win12[12], cs[8], ca[8], isr[7][2], p2q[4], isl[2][16][2];
    for (int k = 0; k < 6; k++)
        for (int o = 0; o < 6; o++) {
            int i = o < 3 ? o : 6 + (o - 3);
            imdct12[k][o] = (float)cos(M_PI / 24.0 * (2 * i + 7) * (2 * k + 1));
        }
    /* long windows (block types 0, 1, 3) with the fast IMDCT's output
     * scale s_n = 1 / (2 cos(pi (2n+1) / 72)) and signs folded in
     * (mp3d_synth.hip imdct36_w): out i<9 uses y_(9+i), i in 9..17 -y_(26-i),
     * 18..26 -y_(26-i), 27..35 -y_(i-27)                                   */
    for (int bt = 0; bt < 4; bt++)
        for (int i = 0; i < 36; i++) {
            double w;
            if (bt == 0 || bt == 2) w = sin(M_PI / 36.0 * (i + 0.5));
            else if (bt == 1) w = i < 18 ? sin(M_PI / 36.0 * (i + 0.5)) : i < 24 ? 1.0 : i < 30 ? sin(M_PI / 12.0 * (i - 18 + 0.5)) : 0.0;
            else w = i < 6 ? 0.0 : i < 12 ? sin(M_PI / 12.0 * (i - 6 + 0.5)) : i < 18 ? 1.0 : sin(M_PI / 36.0 * (i + 0.5));
            int n = i < 9 ? 9 + i : i < 27 ? 26 - i : i - 27;
            double sc = 1.0 / (2.0 * cos(M_PI * (2 * n + 1) / 72.0));
            win36[bt][i] = (float)((i < 9 ? 1.0 : -1.0) * w * sc);
        }
    for (int i = 0; i < 12; i++) win12[i] = (float)sin(M_PI / 12.0 * (i + 0.5));
    for (int i = 0; i < 8; i++) {
        double c = MP3D_ALIAS_C[i], d = sqrt(1.0 + c * c);
        cs[i] = (float)(1.0 / d);
        ca[i] = (float)(c / d);
    }
    for (int p = 0; p < 7; p++) {
        if (p == 6) { isr[p][0] = 1.f; isr[p][1] = 0.f; continue; }
        double tn = tan(p * M_PI / 12.0);
        isr[p][0] = (float)(tn / (1.0 + tn));
        isr[p][1] = (float)(1.0 / (1.0 + tn));
    }
    /* LSF intensity (13818-3 2.4.3.2; FFmpeg is_table_lsf): is_pos p with
     * intensity_scale j -> (2^(-(j+1) ((p+1)/2) / 4), 1) for odd p, swapped
     * for even p (L = x * [0], R = x * [1]) */
    for (int j = 0; j < 2; j++)
        for (int p = 0; p < 16; p++) {
            const float f = (float)pow(2.0, -(j + 1) * ((p + 1) >> 1) / 4.0);
            isl[j][p][0] = (p & 1) ? f : 1.f;
            isl[j][p][1] = (p & 1) ? 1.f : f;
        }
    for (int i = 0; i < 4; i++) p2q[i] = (float)pow(2.0, i / 4.0);
    for (int i = 0; i < 22; i++)
        if (((MP3D_PRETAB_BITS >> (2 * i)) & 3u) != MP3D_PRETAB[i]) return MP3D_E_ARG; /* table drift */
    /* the kernel's literal tables (mp3d_consts.h, tools/gen_consts.py) must
     * equal this recipe bit for bit */
    for (int k = 0; k < 6; k++)
        for (int o = 0; o < 6; o++)
            if (imdct12[k][o] != MP3D_K_IMDCT12[k][o]) return MP3D_E_ARG;
    for (int i = 0; i < 12; i++)
        if (win12[i] != MP3D_K_WIN12[i]) return MP3D_E_ARG;
    for (int i = 0; i < 8; i++)
        if (cs[i] != MP3D_K_ALIAS_CS[i] || ca[i] != MP3D_K_ALIAS_CA[i]) return MP3D_E_ARG;
    uint16_t fbt[9][16] = {};
    for (int sr = 0; sr < 9; sr++)
        for (int bi = 1; bi < 15; bi++)
            fbt[sr][bi] = (uint16_t)((sr < 3 ? 144000 * (int)MP3D_BITRATE_L3[bi] : 72000 * (int)MP3D_BITRATE_L3_LSF[bi]) /
                                     (int)MP3D_SAMPLE_RATE[sr]);
    HIPCHK(upload_synth_constants(&win36[0][0], &isr[0][0], p2q, &isl[0][0][0]));
    HIPCHK(upload_demux_constants(&fbt[0][0]));
    HIPCHK(upload_frame_constants(&fbt[0][0]));
    return MP3D_OK;
}

/* per-device one-time init: constant symbols + table buffer */
struct DeviceCtx {
    bool ready = false;
    DevTables *tables = nullptr;
    int n_cu = 256;
};
static std::mutex g_mu;
static DeviceCtx g_dev[64];

static int device_init(int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MP3D_E_NO_DEVICE;
    if (device < 0 || device >= n || device >= 64) return MP3D_E_NO_DEVICE;
    DeviceCtx &c = g_dev[device];
    HIPCHK(hipSetDevice(device));
    if (c.ready) return MP3D_OK;
    int r = upload_symbols();
    if (r) return r;
    static DevTables host_tables;
    static bool built = false;
    if (!built) {
        build_tables(host_tables);
        built = true;
    }
    HIPCHK(hipMalloc(&c.tables, sizeof(DevTables)));
    HIPCHK(hipMemcpy(c.tables, &host_tables, sizeof(DevTables), hipMemcpyHostToDevice));
    /* the uploads above run on the null stream, and every handle's kernels
     * on non-blocking streams, which do not order after it: complete them
     * here, once per device */
    HIPCHK(hipDeviceSynchronize());
    (void)hipDeviceGetAttribute(&c.n_cu, hipDeviceAttributeMultiprocessorCount, device);
    c.ready = true;
    return MP3D_OK;
}

/* ------------------------------------------------------------------------ */
/* Batch                                                                    */
/* ------------------------------------------------------------------------ */
struct mp3d_batch {
    int device = 0, max_streams = 0, max_frames = 0;
    hipStream_t own = nullptr;
    StreamState *st = nullptr;
    FrameRec *rec = nullptr;
    uint64_t *sideu = nullptr; /* per-unit side info (k_demux -> k_huffman) */
    int16_t *is_buf = nullptr;
    uint32_t *rank = nullptr; /* k_rank: the units in big_values order per segment */
    UnitMeta *meta = nullptr;
    /* Stream geometry of a call (input offsets, sizes, md-region offsets) in
     * two device slots, each filled from its own pinned host buffer by an
     * async copy on the handle's copy stream: a call with new geometry (a
     * streaming loop's offsets advance every call) stages it and returns
     * without waiting; the copy overlaps the previous call's kernels.
     * Layout per slot for a call of n streams: in_off[n] u64, md_off[n] u64,
     * in_len[n] u32. */
    struct Geo {
        uint64_t *d = nullptr;
        uint64_t *h = nullptr;       /* pinned */
        hipEvent_t staged = nullptr; /* the copy h -> d is complete        */
        hipEvent_t freed = nullptr;  /* the last kernel reading d is done */
        bool fresh = false;          /* freed recorded by the slot's last reader */
        int n = -1;
        uint64_t *in_off() const { return d; }
        uint64_t *md_off() const { return d + n; }
        uint32_t *in_len() const { return (uint32_t *)(d + 2 * (size_t)n); }
    } geo[2];
    int geo_i = 0;
    /* d_work[0]: k_huffman's super-chunk counter (device; reset by each
     * launch's memset on the call's stream, and a handle's calls are
     * ordered).  d_work[1]: the family word, = call_seq when k_walk saw an
     * LSF stream in this call (fam_ok: this call's demux was k_walk) */
    uint32_t *d_work = nullptr;
    uint32_t call_seq = 0;
    bool fam_ok = false;
    hipStream_t copy = nullptr;
    mp3d_frame_info *d_infos = nullptr;
    uint8_t *md = nullptr;
    size_t md_cap = 0;
    uint8_t *d_in = nullptr; /* staging for host input */
    size_t in_cap = 0;
    int16_t *d_pcm = nullptr; /* staging for host output */
    size_t pcm_cap = 0;
    float *d_xr = nullptr;
    uint8_t *d_bt = nullptr, *d_mx = nullptr;
    size_t xr_cap = 0;
    /* segmented synth-only calls: the final overlap + fifo per stream go to
     * a packed tail (the first segment may still be reading the state), and
     * the next synth-only call reads them from there: two tails used in
     * turn, so steady config-2 calls never copy state.  tail_live = the tail
     * holding streams [0, tail_n)'s current overlap + fifo (-1: StreamState
     * does); any other use of the handle first copies it back (flush_tail). */
    float *st_tail[2] = {};
    size_t tail_cap[2] = {};
    int tail_live = -1, tail_n = 0;
    bool timing = false;
    int opts = 0; /* MP3D_OPT_* */
    /* End of the handle's last call when it ran on a caller's stream,
     * recorded on that stream: sync, reset and state copies wait on this
     * event, never on the caller's stream handle (which the caller may have
     * destroyed since), and a call on another stream is ordered after it.
     * Calls on the handle's own stream (the per-frame decoder) record
     * nothing: own-stream order covers them. */
    hipEvent_t ev_done = nullptr;
    hipStream_t last_s = nullptr; /* compared with the next call's, never used */
    hipEvent_t ev[4] = {};
    bool poison = false; /* MP3D_DEBUG_POISON at create */
};

/* an event after all of the handle's work issued so far */
static hipEvent_t end_event(mp3d_batch *b) {
    if (!b->last_s || b->last_s == b->own) (void)hipEventRecord(b->ev_done, b->own);
    return b->ev_done;
}

/* StreamState slots [0, n) zeroed with their format stamp, on stream s (the
 * caller orders / waits) */
static hipError_t state_clear(StreamState *st, int n, hipStream_t s) {
    hipError_t e = hipMemsetAsync(st, 0, sizeof(StreamState) * (size_t)n, s);
    if (e == hipSuccess)
        e = hipMemset2DAsync(&st[0].fmt, sizeof(StreamState), MP3D_STATE_FMT_BYTE, sizeof(uint32_t), (size_t)n, s);
    return e;
}

/* MP3D_DEBUG_POISON=1 at create: every device and
 * pinned allocation of the handle is filled with 0xFF when it is made, at
 * create and at every grow(), before the zeroing the code does on purpose.
 * A read of bytes nobody wrote then sees NaNs / huge lengths / all-ones
 * words on EVERY run, instead of whatever an earlier allocation left --
 * tests/test_gpu_poison.py runs the read-ahead, state and golden suites so. */
static bool poison_env() {
    const char *e = getenv("MP3D_DEBUG_POISON");
    return e && e[0] && strcmp(e, "0") != 0;
}
static int poison_dev(bool on, void *p, size_t bytes, hipStream_t s) {
    if (!on || !p || !bytes) return MP3D_OK;
    HIPCHK(hipMemsetAsync(p, 0xFF, bytes, s));
    HIPCHK(hipStreamSynchronize(s));
    return MP3D_OK;
}
static void poison_host(bool on, void *p, size_t bytes) {
    if (on && p) memset(p, 0xFF, bytes);
}

static int grow(mp3d_batch *b, void **p, size_t *cap, size_t need) {
    if (need <= *cap) return MP3D_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(p, need));
    *cap = need;
    return poison_dev(b->poison, *p, need, b->own);
}

/* Frames per k_synth segment for n streams x F frames: few streams leave
 * the chip idle (one wave walks one stream), so each stream is split into
 * frame-parallel segments (one wave each, warm-up frames before; k_synth)
 * until one round of resident waves (4 per SIMD) is in the grid, keeping
 * segments >= min_len frames (C2, 1 024 x 64: 4 segments of 16 frames;
 * at 3 waves per SIMD, 2 rounds of 11 frames measured 4 % slower than one
 * of 22, tools/dbg/job_c2_seg.sh).
 * MP3D_SEG_FRAMES overrides (0 = never split). */
static int seg_frames(int n, int F, int n_cu, int min_len) {
    int seg_len = F;
    const long long want = 4LL * 4 * n_cu; /* one round at 4 waves per SIMD */
    if ((long long)n < want && F >= 2 * min_len) {
        const int nseg = (int)std::min<long long>((want + n - 1) / n, F / min_len);
        seg_len = (F + nseg - 1) / nseg;
    }
    const char *e = getenv("MP3D_SEG_FRAMES");
    if (e && atoi(e) > 0) seg_len = std::min(F, atoi(e));
    if (e && atoi(e) == 0 && e[0] == '0') seg_len = F;
    return seg_len;
}

/* where k_synth takes each stream's overlap + fifo from and puts them:
 * in = the live tail when it holds these n streams (else StreamState, after
 * copying back a tail of another shape); out = the other tail when the
 * call is segmented (the first segment may still be reading the state),
 * else StreamState.  tail_commit() after the launch. */
struct TailPlan {
    const float *in = nullptr;
    float *out = nullptr;
    int t_out = 0;
};
static int tail_plan(mp3d_batch *b, int n, int F, int seg_len, hipStream_t s, TailPlan *tp);
static void tail_commit(mp3d_batch *b, int n, int F, int seg_len, const TailPlan &tp) {
    if (seg_len < F) {
        b->tail_live = tp.t_out;
        b->tail_n = n;
    }
}

static constexpr size_t STATE_TAIL = sizeof(((StreamState *)0)->overlap) + sizeof(((StreamState *)0)->fifo);

/* the live tail back into StreamState (on stream s) */
static int flush_tail(mp3d_batch *b, hipStream_t s) {
    if (b->tail_live < 0) return MP3D_OK;
    HIPCHK(hipMemcpy2DAsync(&b->st[0].overlap[0][0][0], sizeof(StreamState), b->st_tail[b->tail_live], STATE_TAIL,
                            STATE_TAIL, b->tail_n, hipMemcpyDeviceToDevice, s));
    b->tail_live = -1;
    return MP3D_OK;
}

static int tail_plan(mp3d_batch *b, int n, int F, int seg_len, hipStream_t s, TailPlan *tp) {
    if (b->tail_live >= 0 && (seg_len >= F || b->tail_n != n)) {
        int r = flush_tail(b, s);
        if (r) return r;
    }
    tp->in = b->tail_live >= 0 ? b->st_tail[b->tail_live] : nullptr;
    tp->t_out = b->tail_live >= 0 ? b->tail_live ^ 1 : 0;
    tp->out = nullptr;
    if (seg_len < F) {
        const size_t need = STATE_TAIL * (size_t)n;
        const bool fresh = need > b->tail_cap[tp->t_out];
        int r = grow(b, (void **)&b->st_tail[tp->t_out], &b->tail_cap[tp->t_out], need);
        if (r) return r;
        /* k_synth writes the fifo slots the synthesis reads back (slot 0 only
         * at the columns some lane's window needs): zero the rest once, as
         * StreamState is, so a flushed tail leaves the same state bytes */
        if (fresh) HIPCHK(hipMemsetAsync(b->st_tail[tp->t_out], 0, b->tail_cap[tp->t_out], s));
        tp->out = b->st_tail[tp->t_out];
    }
    return MP3D_OK;
}

/* a call on stream s: order it after the handle's previous call (the
 * handle's buffers are shared).  Only two calls in a row on the handle's own
 * stream skip the wait; after a call on a caller's stream the wait is made
 * even when s compares equal, since a destroyed stream's handle value can be
 * reused by the caller's next stream (a no-op once the event completed). */
static int call_begin(mp3d_batch *b, hipStream_t s) {
    HIPCHK(hipSetDevice(b->device));
    if (b->last_s && (b->last_s != s || s != b->own)) HIPCHK(hipStreamWaitEvent(s, end_event(b), 0));
    return MP3D_OK;
}

/* the own stream (sync, reset, state copies) after the handle's last call */
static int own_after_last(mp3d_batch *b) {
    if (b->last_s && b->last_s != b->own) HIPCHK(hipStreamWaitEvent(b->own, b->ev_done, 0));
    return MP3D_OK;
}

/* when a public call returns: ev_done on a caller's stream */
struct CallEnd {
    mp3d_batch *b;
    hipStream_t s;
    ~CallEnd() {
        if (s == b->own || hipEventRecord(b->ev_done, s) == hipSuccess) b->last_s = s;
    }
};

/* Where a caller's buffer lives, seen from the handle's device: its own
 * device memory (or managed memory) is read and written in place by the
 * kernels; host memory and another GPU's memory are staged through the
 * handle's buffers with hipMemcpyDefault copies (no peer access assumed). */
enum PtrKind { PTR_HOST, PTR_DEV, PTR_OTHER_DEV };
static PtrKind ptr_kind(const void *p, int device) {
    if (!p) return PTR_HOST;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return PTR_HOST;
    }
    if (a.type == hipMemoryTypeManaged) return PTR_DEV;
    if (a.type != hipMemoryTypeDevice) return PTR_HOST;
    return a.device == device ? PTR_DEV : PTR_OTHER_DEV;
}
/* memory the handle's kernels may read / write in place */
static bool is_device_ptr(const void *p, int device) { return ptr_kind(p, device) == PTR_DEV; }


extern "C" int mp3d_batch_create(int device, int max_streams, int max_frames, mp3d_batch **out) {
    if (!out || max_streams <= 0 || max_frames <= 0) return MP3D_E_ARG;
    *out = nullptr;
    int r = device_init(device);
    if (r) return r;
    mp3d_batch *b = new (std::nothrow) mp3d_batch;
    if (!b) return MP3D_E_NOMEM;
    b->device = device;
    b->max_streams = max_streams;
    b->max_frames = max_frames;
    size_t units = (size_t)max_streams * max_frames * 4;
#define BALLOC(ptr, bytes)                                                                                             \
    do {                                                                                                               \
        hipError_t _e = hipMalloc((void **)&(ptr), (bytes));                                                           \
        if (_e != hipSuccess) {                                                                                        \
            g_last_hip = (int)_e;                                                                                      \
            mp3d_batch_destroy(b);                                                                                     \
            return MP3D_E_NOMEM;                                                                                       \
        }                                                                                                              \
    } while (0)
    BALLOC(b->st, sizeof(StreamState) * max_streams);
    BALLOC(b->rec, sizeof(FrameRec) * (size_t)max_streams * max_frames);
    BALLOC(b->sideu, sizeof(uint64_t) * units);
    BALLOC(b->is_buf, sizeof(int16_t) * MP3D_IS_ROW * units);
    BALLOC(b->meta, sizeof(UnitMeta) * units);
    BALLOC(b->rank, sizeof(uint32_t) * units); /* k_huffman's big_values order (k_rank) */
    for (auto &g : b->geo) BALLOC(g.d, 20 * (size_t)max_streams);
    BALLOC(b->d_infos, sizeof(mp3d_frame_info) * (size_t)max_streams * max_frames);
    BALLOC(b->d_work, 256);
#undef BALLOC
    bool ok = hipStreamCreateWithFlags(&b->own, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&b->copy, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming) == hipSuccess;
    for (auto &g : b->geo)
        ok = ok && hipHostMalloc((void **)&g.h, 20 * (size_t)max_streams) == hipSuccess &&
             hipEventCreateWithFlags(&g.staged, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&g.freed, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        mp3d_batch_destroy(b);
        return MP3D_E_HIP;
    }
    for (int i = 0; i < 4; i++) (void)hipEventCreate(&b->ev[i]);
    b->poison = poison_env();
    if (b->poison) {
        const size_t fr = (size_t)max_streams * max_frames;
        const struct { void *p; size_t n; } bufs[] = {
            {b->st, sizeof(StreamState) * max_streams}, {b->rec, sizeof(FrameRec) * fr},
            {b->sideu, sizeof(uint64_t) * units},       {b->is_buf, sizeof(int16_t) * MP3D_IS_ROW * units},
            {b->meta, sizeof(UnitMeta) * units},        {b->rank, sizeof(uint32_t) * units},
            {b->geo[0].d, 20 * (size_t)max_streams},    {b->geo[1].d, 20 * (size_t)max_streams},
            {b->d_infos, sizeof(mp3d_frame_info) * fr}, {b->d_work, 256}};
        for (const auto &x : bufs)
            if (poison_dev(true, x.p, x.n, b->own)) {
                mp3d_batch_destroy(b);
                return MP3D_E_HIP;
            }
        for (auto &g : b->geo) poison_host(true, g.h, 20 * (size_t)max_streams);
    }
    if (getenv("MP3D_DEBUG_ADDR")) /* placement diagnostics (tools/dbg/place.py) */
        fprintf(stderr, "mp3d: st %p rec %p sideu %p is_buf %p meta %p infos %p\n", (void *)b->st, (void *)b->rec,
                (void *)b->sideu, (void *)b->is_buf, (void *)b->meta, (void *)b->d_infos);
    /* zeroed on the handle's own stream and waited for: a null-stream
     * hipMemset is asynchronous for device memory and does not order before
     * kernels on non-blocking streams (a first call could read the previous
     * owner's bytes as its streams' state) */
    if (state_clear(b->st, max_streams, b->own) != hipSuccess ||
        hipMemsetAsync(b->d_work, 0, 256, b->own) != hipSuccess || hipStreamSynchronize(b->own) != hipSuccess) {
        mp3d_batch_destroy(b);
        return MP3D_E_HIP;
    }
    *out = b;
    return MP3D_OK;
}

extern "C" void mp3d_batch_destroy(mp3d_batch *b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->ev_done) (void)hipEventSynchronize(b->ev_done);
    if (b->own) (void)hipStreamSynchronize(b->own);
    if (b->copy) (void)hipStreamSynchronize(b->copy);
    void *ptrs[] = {b->st, b->rec, b->sideu, b->is_buf, b->meta, b->rank, b->geo[0].d, b->geo[1].d, b->d_work,
                    b->d_infos, b->md, b->d_in, b->d_pcm, b->d_xr, b->d_bt, b->d_mx, b->st_tail[0], b->st_tail[1]};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    for (auto &g : b->geo) {
        if (g.h) (void)hipHostFree(g.h);
        if (g.staged) (void)hipEventDestroy(g.staged);
        if (g.freed) (void)hipEventDestroy(g.freed);
    }
    for (hipEvent_t e : b->ev)
        if (e) (void)hipEventDestroy(e);
    if (b->ev_done) (void)hipEventDestroy(b->ev_done);
    if (b->own) (void)hipStreamDestroy(b->own);
    if (b->copy) (void)hipStreamDestroy(b->copy);
    delete b;
}

extern "C" int mp3d_batch_reset(mp3d_batch *b) {
    if (!b) return MP3D_E_ARG;
    HIPCHK(hipSetDevice(b->device));
    int r = own_after_last(b);
    if (r) return r;
    b->tail_live = -1; /* the state is zeroed whole */
    HIPCHK(state_clear(b->st, b->max_streams, b->own));
    HIPCHK(hipStreamSynchronize(b->own));
    return MP3D_OK;
}

extern "C" int mp3d_batch_set_options(mp3d_batch *b, int flags) {
    if (!b || (flags & ~MP3D_OPT_CRC_CHECK)) return MP3D_E_ARG;
    b->opts = flags;
    return MP3D_OK;
}

/* waits for this handle's work only: its last call (through ev_done, on
 * whatever stream it ran) and its own stream, never the whole device */
extern "C" int mp3d_batch_sync(mp3d_batch *b) {
    if (!b) return MP3D_E_ARG;
    HIPCHK(hipSetDevice(b->device));
    if (b->last_s && b->last_s != b->own) HIPCHK(hipEventSynchronize(b->ev_done));
    HIPCHK(hipStreamSynchronize(b->own));
    return MP3D_OK;
}

extern "C" int mp3d_batch_set_timing(mp3d_batch *b, int enable) {
    if (!b) return MP3D_E_ARG;
    b->timing = enable != 0;
    return MP3D_OK;
}

extern "C" int mp3d_batch_kernel_times(mp3d_batch *b, float *us3) {
    if (!b || !us3) return MP3D_E_ARG;
    if (!b->timing) return MP3D_E_ARG;
    HIPCHK(hipEventSynchronize(b->ev[3]));
    for (int i = 0; i < 3; i++) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, b->ev[i], b->ev[i + 1]));
        us3[i] = ms * 1000.f;
    }
    return MP3D_OK;
}

/* batches from this many streams take k_walk + k_mdcopy */
#define MP3D_WIDE_STREAMS 256
/* MP3D_DEMUX=lane | wave forces the demux path (tests run both) */
static bool demux_wide(int n) {
    const char *e = getenv("MP3D_DEMUX");
    if (e && !strcmp(e, "lane")) return true;
    if (e && !strcmp(e, "wave")) return false;
    return n >= MP3D_WIDE_STREAMS;
}

/* batches of at most this many units (frame granule channels) decode one
 * unit per wave (k_huffman_wave); MP3D_HUFF=wave | lane forces the kernel */
#define MP3D_WAVE_HUFF_UNITS 1024
static bool huffman_wave(int n_units) {
    const char *e = getenv("MP3D_HUFF");
    if (e && !strcmp(e, "wave")) return true;
    if (e && !strcmp(e, "lane")) return false;
    return n_units <= MP3D_WAVE_HUFF_UNITS;
}

/* a call compares the new geometry with the current slot's and skips the
 * copy when it is unchanged (host time: a memcmp of up to 0.8 MB while the
 * GPU runs the previous call; the staging copy it saves ran on the GPU's
 * timeline between calls, 29 us of copy + 17 us before the next kernel at
 * 65 536 streams, memory-copy trace, round 5) */
#define MP3D_GEO_CACHE_STREAMS (1 << 30)

/* Stage the call's stream geometry (input offsets and sizes, md-region
 * offsets) into the next device slot, asynchronously (struct Geo), size the
 * md region, and make stream s wait for the copy.  Never blocks the host
 * except on the copy of two calls ago. */
static int prepare_geometry(mp3d_batch *b, const uint64_t *offsets, const uint32_t *sizes, int n, hipStream_t s) {
    {
        mp3d_batch::Geo &g = b->geo[b->geo_i];
        if (n <= MP3D_GEO_CACHE_STREAMS && g.n == n && !memcmp(g.h, offsets, sizeof(uint64_t) * n) &&
            !memcmp(g.h + 2 * (size_t)n, sizes, sizeof(uint32_t) * n)) {
            HIPCHK(hipStreamWaitEvent(s, g.staged, 0)); /* a no-op once the copy is done */
            return MP3D_OK;
        }
    }
    b->geo_i ^= 1;
    mp3d_batch::Geo &g = b->geo[b->geo_i];
    /* the slot holds no valid geometry until its copy is queued: a failed
     * stage below can never be served from the cache by a retried call */
    g.n = -1;
    HIPCHK(hipEventSynchronize(g.staged)); /* this slot's last copy has read g.h */
    uint64_t *h_md = g.h + n;
    size_t o = 0;
    for (int i = 0; i < n; i++) {
        h_md[i] = o;
        /* carry-in + payloads; a cut-short final frame is completed with
         * zeros, so allow one maximal frame beyond the stream's bytes */
        o += ((size_t)sizes[i] + MP3D_RES_BYTES + MP3D_MAX_FRAME_BYTES + 16 + 15) & ~(size_t)15;
    }
    memcpy(g.h, offsets, sizeof(uint64_t) * n);
    memcpy(g.h + 2 * (size_t)n, sizes, sizeof(uint32_t) * n);
    /* growing md frees the old region: hipFree waits for the device */
    const size_t md_was = b->md_cap;
    int r = grow(b, (void **)&b->md, &b->md_cap, o + 8192);
    if (r) return r;
    /* a new region starts zeroed: the Huffman staging reads whole words up
     * to 2 past a unit's end, and a corrupt unit may decode past its
     * payload -- those bits then read as zeros (FFmpeg's buffer padding),
     * never as a previous allocation's bytes */
    if (b->md_cap != md_was) HIPCHK(hipMemsetAsync(b->md, 0, b->md_cap, s));
    /* after the call that last read this slot */
    HIPCHK(hipStreamWaitEvent(b->copy, g.fresh ? g.freed : end_event(b), 0));
    HIPCHK(hipMemcpyAsync(g.d, g.h, 20 * (size_t)n, hipMemcpyHostToDevice, b->copy));
    HIPCHK(hipEventRecord(g.staged, b->copy));
    HIPCHK(hipStreamWaitEvent(s, g.staged, 0));
    g.n = n;
    return MP3D_OK;
}

/* Front half shared by decode and huffman_only: input staging, k_demux,
 * k_huffman. */
/* mapped: frames (and dev_infos) are host memory the device reads / writes
 * directly (the per-frame decoder's pinned buffers): no staging copies */
static int run_front(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes, int n,
                     int F, hipStream_t s, bool *sync_needed, bool mapped = false,
                     mp3d_frame_info *dev_infos = nullptr) {
    if (!b || !frames || !offsets || !sizes || n <= 0 || F <= 0) return MP3D_E_ARG;
    if (n > b->max_streams || F > b->max_frames) return MP3D_E_CAPACITY;
    int r = call_begin(b, s); /* (the demux and Huffman stages never touch a live tail's overlap / fifo) */
    if (r) return r;
    uint64_t total = 0;
    for (int i = 0; i < n; i++) total = std::max<uint64_t>(total, offsets[i] + sizes[i]);
    const uint8_t *din = frames;
    if (!mapped && !is_device_ptr(frames, b->device)) {
        r = grow(b, (void **)&b->d_in, &b->in_cap, total + 64);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(b->d_in, frames, total, hipMemcpyDefault, s));
        din = b->d_in;
        *sync_needed = true;
    }
    r = prepare_geometry(b, offsets, sizes, n, s);
    if (r) return r;
    const mp3d_batch::Geo &g = b->geo[b->geo_i];
    DeviceCtx &dc = g_dev[b->device];
    if (b->timing) HIPCHK(hipEventRecord(b->ev[0], s));
    /* demux + main-data gather: lane-per-stream walk + payload copy for wide
     * batches, one wave per stream below MP3D_WIDE_STREAMS (fewer launches) */
    const bool wide = demux_wide(n);
    if (++b->call_seq == 0) b->call_seq = 1; /* (d_work[1] starts at 0) */
    b->fam_ok = wide;
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_demux(din, g.in_off(), g.in_len(), b->md, g.md_off(), b->st, b->rec, b->sideu,
                 dev_infos ? (void *)dev_infos : b->d_infos, n, F, b->opts, wide, b->d_work + 1, b->call_seq, s);
    if (b->timing) HIPCHK(hipEventRecord(b->ev[1], s));
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_huffman(b->md, g.md_off(), b->rec, b->sideu, dc.tables, b->is_buf, b->meta, n, F, dc.n_cu,
                   huffman_wave(n * F * 4), b->d_work, b->rank, s);
    HIPCHK(hipEventRecord(g.freed, s)); /* the slot's last reader */
    b->geo[b->geo_i].fresh = true;
    if (b->timing) HIPCHK(hipEventRecord(b->ev[2], s));
    HIPCHK(hipGetLastError());
    return MP3D_OK;
}

/* One run of pre-located, complete frames of one stream (the per-frame
 * decoder's read-ahead, mp3d_host.cpp ra_fill): the bytes and the frame
 * offsets in mapped host memory, read by k_demux_fp directly (no copy); the
 * previous run's synthesis tail flushed and the state snapshot taken inside
 * that kernel; no stream geometry to stage (one stream at md offset 0).  A
 * run costs three kernel launches and no copy. */
struct FpRun {
    const uint8_t *in;   /* device address of the run's bytes (mapped)    */
    uint32_t len;
    const uint32_t *fo;  /* the frame offsets (host; passed as kernel arguments) */
    const float *tail_in; /* the handle's live synthesis tail, or null     */
    StreamState *snap;   /* receives the state before the run             */
};
static int run_front_fp(mp3d_batch *b, const FpRun &fp, int F, hipStream_t s, mp3d_frame_info *dev_infos) {
    if (b->max_streams != 1 || F <= 0 || F > 64 || F > b->max_frames) return MP3D_E_ARG;
    int r = call_begin(b, s);
    if (r) return r;
    if (b->md_cap < (size_t)fp.len + MP3D_RES_BYTES + 8192) return MP3D_E_CAPACITY; /* sized at create */
    DeviceCtx &dc = g_dev[b->device];
    if (b->timing) HIPCHK(hipEventRecord(b->ev[0], s));
    if (++b->call_seq == 0) b->call_seq = 1;
    b->fam_ok = false;
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_demux_fp(fp.in, fp.len, fp.fo, b->md, b->st, fp.tail_in, fp.snap, b->rec, b->sideu,
                    dev_infos ? (void *)dev_infos : b->d_infos, F, b->opts, s);
    if (b->timing) HIPCHK(hipEventRecord(b->ev[1], s));
    /* md offset of the one stream: a zero word of d_work (d_work[4..5]) */
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_huffman(b->md, (const uint64_t *)(b->d_work + 4), b->rec, b->sideu, dc.tables, b->is_buf, b->meta, 1, F,
                   dc.n_cu, true, b->d_work, nullptr, s);
    if (b->timing) HIPCHK(hipEventRecord(b->ev[2], s));
    HIPCHK(hipGetLastError());
    return MP3D_OK;
}

/* decode into int16 (f32 = false) or float32 PCM, both [n][F][2304] */
/* kinds: k_synth family variants to launch (bit 0 MPEG-1, bit 1 LSF); 3 for
 * a batch, one bit for the per-frame decoder, which knows its frame's family */
/* mapped: frames, pcm and infos are device-accessible pinned host memory
 * (the per-frame decoder): the kernels read and write them in place and the
 * call ends with one stream sync */
/* async (mapped only): return without waiting; the caller records an event */
static int batch_decode(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes, int n,
                        int F, void *pcm, bool f32, mp3d_frame_info *infos, void *hip_stream, bool overwrite,
                        int kinds = 3, bool mapped = false, int seg_len_req = 0, const FpRun *fp = nullptr,
                        bool async = false) {
    if (!b || !pcm) return MP3D_E_ARG;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : b->own;
    CallEnd done{b, s};
    bool sync_needed = mapped;
    /* frame infos: written in place when the caller's array is device memory
     * (or the per-frame decoder's mapped buffer), else into d_infos and
     * copied to the host after the call */
    const bool inf_host = infos && !mapped && !is_device_ptr(infos, b->device); /* or another GPU's */
    mp3d_frame_info *dinf = infos && !inf_host ? infos : b->d_infos;
    int r = fp ? run_front_fp(b, *fp, F, s, dinf) : run_front(b, frames, offsets, sizes, n, F, s, &sync_needed, mapped, dinf);
    if (r) return r;
    if (async && !mapped) return MP3D_E_ARG;
    const size_t PB = f32 ? sizeof(float) : sizeof(int16_t), row = 2304 * PB;
    const size_t pcm_bytes = (size_t)n * F * row;
    void *dpcm = pcm;
    const PtrKind pk = mapped ? PTR_DEV : ptr_kind(pcm, b->device);
    bool pcm_host = pk == PTR_HOST;
    if (pk != PTR_DEV) {
        r = grow(b, (void **)&b->d_pcm, &b->pcm_cap, pcm_bytes);
        if (r) return r;
        dpcm = b->d_pcm;
        /* another GPU's buffer: its rows the kernel does not write keep their
         * bytes, as in place (copied over, decoded into, copied back) */
        if (pk == PTR_OTHER_DEV) HIPCHK(hipMemcpyAsync(dpcm, pcm, pcm_bytes, hipMemcpyDefault, s));
    }
    DeviceCtx &dc = g_dev[b->device];
    /* few streams: frame-parallel segments per stream (>= 4 frames each,
     * or the caller's seg_len) */
    const int seg_len = seg_len_req > 0 ? std::min(F, seg_len_req) : seg_frames(n, F, dc.n_cu, 4);
    TailPlan tp;
    r = tail_plan(b, n, F, seg_len, s, &tp);
    if (r) return r;
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_synth(b->rec, b->is_buf, b->meta, dc.tables, b->st, dpcm, f32, n, F, kinds, seg_len, tp.out, tp.in,
                 b->fam_ok ? b->d_work + 1 : nullptr, b->call_seq, dc.n_cu, s);
    if (b->timing) HIPCHK(hipEventRecord(b->ev[3], s));
    HIPCHK(hipGetLastError());
    tail_commit(b, n, F, seg_len, tp);
    const size_t ib = sizeof(mp3d_frame_info) * (size_t)n * F;
    if (pcm_host && !overwrite) {
        /* A host sink is read back whole, but each row keeps the caller's
         * bytes the kernel did not write (rows without audio, the second
         * half of a mono / LSF row): those few spans are saved from the
         * caller's buffer and put back after the copy -- no host-to-device
         * copy of the whole PCM buffer first. */
        std::vector<mp3d_frame_info> tmp;
        mp3d_frame_info *hi = inf_host ? infos : nullptr;
        if (!hi) {
            tmp.resize((size_t)n * F);
            hi = tmp.data();
        }
        HIPCHK(hipMemcpyAsync(hi, dinf, ib, hipMemcpyDefault, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<size_t> at;
        std::vector<uint8_t> kept;
        for (size_t i = 0; i < (size_t)n * F; i++) {
            const size_t w = (size_t)hi[i].samples * (size_t)hi[i].channels * PB;
            if (w >= row) continue;
            at.push_back(i);
            kept.insert(kept.end(), (const uint8_t *)pcm + i * row + w, (const uint8_t *)pcm + (i + 1) * row);
        }
        HIPCHK(hipMemcpyAsync(pcm, dpcm, pcm_bytes, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        size_t k = 0;
        for (size_t i : at) {
            const size_t w = (size_t)hi[i].samples * (size_t)hi[i].channels * PB;
            memcpy((uint8_t *)pcm + i * row + w, kept.data() + k, row - w);
            k += row - w;
        }
        return MP3D_OK;
    }
    if (pk != PTR_DEV) { /* another GPU's buffer, or internal callers that read only the rows with audio */
        HIPCHK(hipMemcpyAsync(pcm, dpcm, pcm_bytes, hipMemcpyDefault, s));
        sync_needed = pcm_host;
    }
    if (inf_host) {
        HIPCHK(hipMemcpyAsync(infos, b->d_infos, ib, hipMemcpyDefault, s));
        sync_needed = sync_needed || ptr_kind(infos, b->device) == PTR_HOST;
    }
    if (sync_needed && !async) HIPCHK(hipStreamSynchronize(s));
    return MP3D_OK;
}

extern "C" int mp3d_batch_decode(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes,
                                 int n, int F, int16_t *pcm, mp3d_frame_info *infos, void *hip_stream) {
    return batch_decode(b, frames, offsets, sizes, n, F, pcm, false, infos, hip_stream, false);
}

extern "C" int mp3d_batch_decode_f32(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets,
                                     const uint32_t *sizes, int n, int F, float *pcm, mp3d_frame_info *infos,
                                     void *hip_stream) {
    return batch_decode(b, frames, offsets, sizes, n, F, pcm, true, infos, hip_stream, false);
}

extern "C" int mp3d_batch_huffman_only(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets,
                                       const uint32_t *sizes, int n, int F, int16_t *is_out, uint8_t *sf_out,
                                       void *hip_stream) {
    if (!b) return MP3D_E_ARG;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : b->own;
    CallEnd done{b, s};
    bool sync_needed = false;
    size_t units = (size_t)n * F * 4;
    if (n > 0 && F > 0 && n <= b->max_streams && F <= b->max_frames) {
        /* k_huffman stores only each row's nonzero prefix (nz_end); the tap
         * returns whole rows, so clear them first */
        int r = call_begin(b, s);
        if (r) return r;
        HIPCHK(hipMemsetAsync(b->is_buf, 0, units * MP3D_IS_ROW * sizeof(int16_t), s));
    }
    int r = run_front(b, frames, offsets, sizes, n, F, s, &sync_needed);
    if (r) return r;
    if (is_out) {
        HIPCHK(hipMemcpy2DAsync(is_out, 576 * sizeof(int16_t), b->is_buf, MP3D_IS_ROW * sizeof(int16_t),
                                576 * sizeof(int16_t), units, hipMemcpyDefault, s));
        sync_needed |= ptr_kind(is_out, b->device) == PTR_HOST;
    }
    if (sf_out) {
        HIPCHK(hipMemcpy2DAsync(sf_out, 40, b->meta, sizeof(UnitMeta), 40, units, hipMemcpyDefault, s));
        sync_needed |= ptr_kind(sf_out, b->device) == PTR_HOST;
    }
    if (sync_needed) HIPCHK(hipStreamSynchronize(s));
    return MP3D_OK;
}

extern "C" int mp3d_batch_synth_only(mp3d_batch *b, const float *xr, const uint8_t *block_type, const uint8_t *mixed,
                                     int n, int F, int nch, int hz, int16_t *pcm, void *hip_stream) {
    if (!b || !xr || !block_type || !mixed || !pcm || n <= 0 || F <= 0 || (nch != 1 && nch != 2)) return MP3D_E_ARG;
    if (n > b->max_streams || F > b->max_frames) return MP3D_E_CAPACITY;
    int sr = hz == 44100 ? 0 : hz == 48000 ? 1 : hz == 32000 ? 2 : -1;
    if (sr < 0) return MP3D_E_ARG;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : b->own;
    {
        int r = call_begin(b, s);
        if (r) return r;
    }
    CallEnd done{b, s};
    bool sync_needed = false;
    size_t nx = (size_t)n * F * 2 * nch;
    const float *dxr = xr;
    const uint8_t *dbt = block_type, *dmx = mixed;
    if (!is_device_ptr(xr, b->device) || !is_device_ptr(block_type, b->device) || !is_device_ptr(mixed, b->device)) {
        size_t need = nx * 576 * sizeof(float) + 2 * nx + 64;
        int r = grow(b, (void **)&b->d_xr, &b->xr_cap, need);
        if (r) return r;
        uint8_t *base = (uint8_t *)b->d_xr;
        HIPCHK(hipMemcpyAsync(base, xr, nx * 576 * sizeof(float), hipMemcpyDefault, s));
        HIPCHK(hipMemcpyAsync(base + nx * 576 * sizeof(float), block_type, nx, hipMemcpyDefault, s));
        HIPCHK(hipMemcpyAsync(base + nx * 576 * sizeof(float) + nx, mixed, nx, hipMemcpyDefault, s));
        dxr = (const float *)base;
        dbt = base + nx * 576 * sizeof(float);
        dmx = dbt + nx;
        sync_needed = true;
    }
    size_t pcm_bytes = (size_t)n * F * 2304 * sizeof(int16_t);
    int16_t *dpcm = pcm;
    const PtrKind pk = ptr_kind(pcm, b->device);
    const bool pcm_host = pk != PTR_DEV; /* host, or another GPU's (staged like host) */
    if (pcm_host) {
        int r = grow(b, (void **)&b->d_pcm, &b->pcm_cap, pcm_bytes);
        if (r) return r;
        dpcm = b->d_pcm;
        /* mono rows are half written: the rest keeps the caller's bytes */
        if (pk == PTR_OTHER_DEV || nch == 1) HIPCHK(hipMemcpyAsync(dpcm, pcm, pcm_bytes, hipMemcpyDefault, s));
    }
    DeviceCtx &dc = g_dev[b->device];
    if (b->timing) {
        for (int i = 0; i < 3; i++) HIPCHK(hipEventRecord(b->ev[i], s));
    }
    /* few streams: frame-parallel segments (seg_frames; one warm-up frame
     * each, so >= 4 frames per segment: warm-up overhead <= 25 %) */
    const int seg_len = seg_frames(n, F, dc.n_cu, 4);
    TailPlan tp;
    {
        int r = tail_plan(b, n, F, seg_len, s, &tp);
        if (r) return r;
    }
    if (b->poison) launch_lds_poison(dc.n_cu, s);
    launch_synth_xr(dxr, dbt, dmx, dc.tables, b->st, dpcm, n, F, nch, sr, seg_len, tp.out, tp.in, s);
    if (b->timing) HIPCHK(hipEventRecord(b->ev[3], s));
    HIPCHK(hipGetLastError());
    tail_commit(b, n, F, seg_len, tp);
    if (pcm_host) {
        HIPCHK(hipMemcpyAsync(pcm, dpcm, pcm_bytes, hipMemcpyDefault, s));
        sync_needed = sync_needed || pk == PTR_HOST;
    }
    if (sync_needed) HIPCHK(hipStreamSynchronize(s));
    return MP3D_OK;
}

static void tag_to_info(uint32_t tag, uint32_t frames, int kind, mp3d_stream_info *o) {
    memset(o, 0, sizeof(*o));
    o->has_tag = (tag & MP3D_TAG_SEEN) != 0;
    o->has_lame = (tag & MP3D_TAG_LAME) != 0;
    o->total_frames = (tag & MP3D_TAG_FRAMES) ? (int)frames : -1;
    o->end_sample = -1;
    if (o->has_lame) {
        o->enc_delay = (int)((tag >> 12) & 0xFFFu);
        o->enc_padding = (int)(tag & 0xFFFu);
        o->skip_samples = o->enc_delay + 529; /* FFmpeg: start_pad + 528 + 1 */
        if (o->total_frames > 0) o->end_sample = (long long)o->total_frames * (kind == 2 ? 576 : 1152) + 529 - o->enc_padding;
    }
}

extern "C" int mp3d_batch_stream_info(mp3d_batch *b, int n, mp3d_stream_info *out) {
    if (!b || !out || n <= 0) return MP3D_E_ARG;
    if (n > b->max_streams) return MP3D_E_CAPACITY;
    HIPCHK(hipSetDevice(b->device));
    /* StreamState tag_info, tag_frames, kind: three consecutive words */
    std::vector<uint32_t> tag((size_t)n * 3);
    int r = own_after_last(b); /* after the handle's last call, on any stream */
    if (r) return r;
    HIPCHK(hipMemcpy2DAsync(tag.data(), 3 * sizeof(uint32_t), &b->st[0].tag_info, sizeof(StreamState),
                            3 * sizeof(uint32_t), n, hipMemcpyDeviceToHost, b->own));
    HIPCHK(hipStreamSynchronize(b->own));
    for (int i = 0; i < n; i++) tag_to_info(tag[3 * i], tag[3 * i + 1], (int)tag[3 * i + 2], &out[i]);
    return MP3D_OK;
}

/* ------------------------------------------------------------------------ */
/* Segmented decode of one long stream               */
/* ------------------------------------------------------------------------ */
extern "C" int mp3d_long_plan(const uint8_t *data, size_t bytes, int L, long long max_frames, uint64_t *frame_off,
                              long long *seg_start, long long *n_frames, int *max_warmup) {
    if (!data || L <= 0 || max_frames < 0 || !n_frames) return MP3D_E_ARG;
    std::vector<uint64_t> off;
    std::vector<long long> a;
    int wmax = 0;
    *n_frames = 0;
    const int r = long_plan(data, bytes, L, max_frames, off, a, &wmax);
    if (r) return r;
    *n_frames = (long long)off.size();
    if (frame_off) std::copy(off.begin(), off.end(), frame_off);
    if (seg_start) std::copy(a.begin(), a.end(), seg_start);
    if (max_warmup) *max_warmup = wmax;
    return MP3D_OK;
}

static int batch_decode(mp3d_batch *b, const uint8_t *frames, const uint64_t *offsets, const uint32_t *sizes, int n,
                        int F, void *pcm, bool f32, mp3d_frame_info *infos, void *hip_stream, bool overwrite,
                        int kinds, bool mapped, int seg_len_req, const FpRun *fp, bool async);

extern "C" int mp3d_batch_decode_long(mp3d_batch *b, const uint8_t *data, size_t bytes, int L, void *pcm, int f32,
                                      long long max_frames, mp3d_frame_info *infos, long long *n_frames,
                                      mp3d_stream_info *sinfo) {
    if (!b || !data || !pcm || L <= 0 || max_frames <= 0 || !n_frames) return MP3D_E_ARG;
    *n_frames = 0;
    HIPCHK(hipSetDevice(b->device));
    const bool dev_in = ptr_kind(data, b->device) != PTR_HOST; /* any GPU's: the walk needs a host copy */
    std::vector<uint8_t> host_copy;
    const uint8_t *hp = data;
    if (dev_in) { /* the frame walk runs on the host */
        host_copy.resize(bytes);
        HIPCHK(hipMemcpy(host_copy.data(), data, bytes, hipMemcpyDefault));
        hp = host_copy.data();
    }
    std::vector<uint64_t> off;
    std::vector<long long> a;
    int wmax = 0;
    long long N = 0;
    {
        const int r = long_plan(hp, bytes, L, max_frames, off, a, &wmax);
        if (r) return r;
        N = (long long)off.size();
    }
    *n_frames = N;
    if (N == 0) return MP3D_OK;
    const long long K = (long long)a.size();
    const int F = L + wmax;
    if (F > b->max_frames) return MP3D_E_CAPACITY;
    hipStream_t s = b->own;
    {
        int r = own_after_last(b);
        if (!r) r = flush_tail(b, s); /* before b->st points at the scratch states */
        if (r) return r;
    }
    const uint8_t *din = data;
    if (!is_device_ptr(data, b->device)) { /* host or another GPU's: staged */
        int r = grow(b, (void **)&b->d_in, &b->in_cap, bytes + 64);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(b->d_in, data, bytes, hipMemcpyDefault, s));
        din = b->d_in;
    }
    const size_t row = 2304 * (f32 ? sizeof(float) : sizeof(int16_t));
    const bool pcm_dev = is_device_ptr(pcm, b->device), inf_dev = infos && is_device_ptr(infos, b->device);
    const int chunk = b->max_streams;
    void *seg_pcm = nullptr, *out_pcm = nullptr;
    int *d_a = nullptr;
    /* the virtual streams decode on a state array of their own: the handle's
     * per-stream state (reservoir, overlap, FIFO, tag) is left as it was */
    StreamState *const own_st = b->st, *seg_st = nullptr;
    std::vector<int> a32;
    mp3d_frame_info *out_inf = nullptr;
    int rc = MP3D_OK;
#define LCHK(x)                                                                                                        \
    do {                                                                                                               \
        hipError_t _e = (x);                                                                                           \
        if (_e != hipSuccess) {                                                                                        \
            g_last_hip = (int)_e;                                                                                      \
            rc = MP3D_E_HIP;                                                                                           \
            goto done;                                                                                                 \
        }                                                                                                              \
    } while (0)
    LCHK(hipMalloc(&seg_pcm, (size_t)std::min<long long>(chunk, K) * F * row));
    LCHK(hipMalloc(&seg_st, sizeof(StreamState) * (size_t)std::min<long long>(chunk, K)));
    if (b->poison && (poison_dev(true, seg_pcm, (size_t)std::min<long long>(chunk, K) * F * row, s) ||
                      poison_dev(true, seg_st, sizeof(StreamState) * (size_t)std::min<long long>(chunk, K), s))) {
        rc = MP3D_E_HIP;
        goto done;
    }
    b->st = seg_st;
    LCHK(hipMalloc(&d_a, sizeof(int) * K));
    a32.assign(a.begin(), a.end());
    LCHK(hipMemcpyAsync(d_a, a32.data(), sizeof(int) * K, hipMemcpyHostToDevice, s));
    out_pcm = pcm_dev ? pcm : nullptr;
    if (!pcm_dev) LCHK(hipMalloc(&out_pcm, (size_t)N * row));
    if (infos) {
        out_inf = inf_dev ? infos : nullptr;
        if (!inf_dev) LCHK(hipMalloc(&out_inf, sizeof(mp3d_frame_info) * (size_t)N));
    }
    if (b->poison && ((!pcm_dev && poison_dev(true, out_pcm, (size_t)N * row, s)) ||
                      (infos && !inf_dev && poison_dev(true, out_inf, sizeof(mp3d_frame_info) * (size_t)N, s)))) {
        rc = MP3D_E_HIP;
        goto done;
    }
    for (long long k0 = 0; k0 < K; k0 += chunk) {
        const int ns = (int)std::min<long long>(chunk, K - k0);
        std::vector<uint64_t> so(ns);
        std::vector<uint32_t> ss(ns);
        for (int i = 0; i < ns; i++) {
            const long long k = k0 + i, e = std::min(N, (k + 1) * L);
            so[i] = k == 0 ? 0 : off[a[k]];
            ss[i] = (uint32_t)((e < N ? off[e] : bytes) - so[i]);
        }
        /* fresh decoder state for every virtual stream */
        LCHK(state_clear(b->st, ns, s));
        b->tail_live = -1; /* fresh states: no tail of the previous chunk */
        rc = batch_decode(b, din, so.data(), ss.data(), ns, F, seg_pcm, f32 != 0, nullptr, s, false);
        if (rc) goto done;
        if (k0 == 0 && sinfo) rc = mp3d_batch_stream_info(b, 1, sinfo);
        if (rc) goto done;
        const long long j0 = k0 * L, j1 = std::min(N, (k0 + ns) * L);
        launch_gather_frames(seg_pcm, (uint8_t *)out_pcm + (size_t)j0 * row, b->d_infos, out_inf ? out_inf + j0 : nullptr,
                             d_a + k0, L, F, (int)k0, (int)(j1 - j0), (int)row, s);
        LCHK(hipGetLastError());
    }
    if (!pcm_dev) LCHK(hipMemcpyAsync(pcm, out_pcm, (size_t)N * row, hipMemcpyDefault, s));
    if (infos && !inf_dev) LCHK(hipMemcpyAsync(infos, out_inf, sizeof(mp3d_frame_info) * (size_t)N, hipMemcpyDefault, s));
    LCHK(hipStreamSynchronize(s));
done:
#undef LCHK
    (void)hipStreamSynchronize(s);
    b->st = own_st;
    b->tail_live = -1; /* a tail left by the segments belongs to the scratch states */
    if (seg_st) (void)hipFree(seg_st);
    if (seg_pcm) (void)hipFree(seg_pcm);
    if (d_a) (void)hipFree(d_a);
    if (!pcm_dev && out_pcm) (void)hipFree(out_pcm);
    if (infos && !inf_dev && out_inf) (void)hipFree(out_inf);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Per-frame decoder                                                         */
/* ------------------------------------------------------------------------ */
/* Per-frame decoder: a one-stream batch plus pinned staging, so a call is
 * one small DMA each way and one stream sync.  The frame is staged
 * zero-padded to a fixed MP3D_PF_BYTES, which keeps the batch geometry
 * constant (uploaded once) across calls. */
#define MP3D_PF_BYTES 4096
#define MP3D_PF_READAHEAD 64 /* frames per read-ahead by default (k_demux_fp: <= 64) */
#define MP3D_PF_RA_SEG 1     /* synthesis segment (frames) of a read-ahead */
struct mp3d_dec {
    mp3d_batch *b = nullptr;
    long frames = 0;
    int kind = 0; /* MPEG family of the stream's first frame (StreamState.kind) */
    uint8_t *h_in = nullptr;            /* pinned: the frame, zero-padded      */
    float *h_out = nullptr;             /* pinned: one frame of PCM            */
    mp3d_frame_info *h_info = nullptr;  /* pinned: its frame info              */
    /* device addresses of the three (mapped): the kernels read the frame and
     * write PCM + info in place, no copies (null: staged copies instead) */
    uint8_t *m_in = nullptr;
    float *m_out = nullptr;
    mp3d_frame_info *m_info = nullptr;
    /* one-launch path (k_frame): the kernel writes the call's sequence
     * number into this mapped word after its PCM; the host polls it */
    uint32_t *h_done = nullptr, *m_done = nullptr;
    uint32_t seq = 0;
    bool fused = false;
    /* Read-ahead: the player hands over the
     * rest of its buffer, so one call decodes up to ra_max of the frames
     * found there in ONE batch call (n = 1, F = ra_max; the host-located
     * frames demuxed frame-parallel by k_demux_fp, frame-parallel synthesis
     * segments) into mapped buffers, and the next calls are served from them
     * after checking that the caller's bytes at the located frame are the
     * same.  Two runs: while the calls are served from one, the next run
     * (the frames after it in the same buffer) decodes behind them, launched
     * without waiting, so a player's steady state never waits for a refill.
     * Any other input (a seek, a new buffer, other options or sink) settles
     * first: the state saved before the run being served is restored and
     * the frames already served are decoded again (exact), the next run is
     * dropped, then the call runs normally.  MP3D_PF_READAHEAD = frames per
     * run (0 / 1: off); MP3D_PF_RA_NEXT=0: no next run (one run at a time). */
    int ra_max = 0;
    int ra_seg = MP3D_PF_RA_SEG; /* MP3D_PF_RA_SEG env: synthesis segment of a read-ahead */
    bool ra_next_on = true;
    struct RaEnt {
        uint32_t off, len; /* the frame's bytes in the run's in buffer */
        size_t pos;        /* bytes skipped before it in its call's buffer */
    };
    struct Run {
        uint8_t *in = nullptr;        /* pinned, mapped: frames back to back, then the u32 frame offsets */
        uint8_t *in_m = nullptr;      /* its device address: k_demux_fp reads it in place (all frames at
                                       * once, so one PCIe round trip per phase, not one per frame) */
        void *pcm = nullptr, *pcm_m = nullptr; /* [ra_max][2304] f32-sized slots (mapped) */
        mp3d_frame_info *inf = nullptr, *inf_m = nullptr;
        StreamState *snap = nullptr;  /* device: the state before the run */
        hipEvent_t done = nullptr;    /* the run's batch call has completed */
        std::vector<RaEnt> ents;
        uint32_t fo_at = 0;           /* byte offset of the frame offsets in in / dev */
        bool f32 = false;
        bool pending = false;         /* launched without waiting (the next run) */
    } run[2];
    int cur = 0;       /* run[cur] is served; run[cur ^ 1] is the next run, if any */
    size_t ra_next = 0; /* next entry of run[cur] to serve */
    /* back-off: a settle that drops frames decoded ahead wasted
     * them, so the next ra_cool calls decode their own frame only; each such
     * settle doubles the pause (up to 64 calls), a read-ahead served whole
     * clears it.  A player that saves its state every frame then pays one
     * read-ahead per ~65 frames instead of two batch decodes per frame. */
    int ra_cool = 0, ra_backoff = 0;
    /* A read-ahead launch or settle that failed part-way may have advanced
     * the device state (k_demux_fp writes it and the snapshot first) with no
     * record of where to: every later call returns this error until
     * mp3d_dec_reset or a successful mp3d_dec_set_state. */
    std::atomic<int> broken{0}; /* (written by the helper thread, read by the caller's) */
    /* MP3D_DEBUG_RA_DELAY_US: the helper thread sleeps this long before each
     * launch (tests: the served calls must not depend on its timing) */
    int wk_delay_us = 0;
    /* MP3D_DEBUG_RA_FAIL=n: the n-th next-run launch reports MP3D_E_HIP after
     * its kernels were queued (the state then sits past the served frames) */
    int dbg_fail = 0, dbg_launches = 0;
    /* The next run's launch (its HIP calls: three kernel launches and an
     * event, tens of microseconds of host time) runs on a helper thread, so
     * the call that hands it over returns at once; the frames are staged
     * into the run's buffer by the calling thread first (the caller's buffer
     * is valid only during its call).  Every call that touches the batch
     * handle joins the helper first (ra_join); a call served from the
     * current run does not.  MP3D_PF_RA_THREAD=0: launch on the calling
     * thread. */
    bool wk_on = true;
    std::thread wk;
    std::mutex wk_mu;
    std::condition_variable wk_cv;
    bool wk_job = false, wk_quit = false;
    int wk_rc = 0;
    struct WkJob {
        Run *u;
        uint32_t o;
        int kinds;
        bool f32;
    } wk_arg{};
    mp3d_dec::Run &R() { return run[cur]; }
    mp3d_dec::Run &N() { return run[cur ^ 1]; }
};

static void dec_free(mp3d_dec *d) {
    if (d->wk.joinable()) {
        {
            std::lock_guard<std::mutex> lk(d->wk_mu);
            d->wk_quit = true;
        }
        d->wk_cv.notify_all();
        d->wk.join(); /* (after its last job) */
    }
    if (d->b) mp3d_batch_destroy(d->b); /* (waits for the handle's work, a next run included) */
    if (d->h_in) (void)hipHostFree(d->h_in);
    if (d->h_out) (void)hipHostFree(d->h_out);
    if (d->h_info) (void)hipHostFree(d->h_info);
    if (d->h_done) (void)hipHostFree(d->h_done);
    for (auto &u : d->run) {
        if (u.in) (void)hipHostFree(u.in);
        if (u.pcm) (void)hipHostFree(u.pcm);
        if (u.inf) (void)hipHostFree(u.inf);
        if (u.snap) (void)hipFree(u.snap);
        if (u.done) (void)hipEventDestroy(u.done);
    }
    delete d;
}

static void ra_worker(mp3d_dec *d);
extern "C" int mp3d_dec_create_on(int device, mp3d_dec **out) {
    if (!out) return MP3D_E_ARG;
    *out = nullptr;
    mp3d_dec *d = new (std::nothrow) mp3d_dec;
    if (!d) return MP3D_E_NOMEM;
    {
        const char *e = getenv("MP3D_PF_READAHEAD");
        d->ra_max = e ? std::max(0, std::min(64, atoi(e))) : MP3D_PF_READAHEAD;
        const char *g = getenv("MP3D_PF_RA_SEG");
        if (g) d->ra_seg = std::max(1, atoi(g));
        if (d->ra_max < 2) d->ra_max = 0;
        const char *nx = getenv("MP3D_PF_RA_NEXT");
        d->ra_next_on = !(nx && !strcmp(nx, "0"));
        const char *th = getenv("MP3D_PF_RA_THREAD");
        d->wk_on = !(th && !strcmp(th, "0"));
        /* test hooks: the helper's launch delayed, the n-th next-run launch
         * failed after it ran (tests/test_gpu_poison.py) */
        const char *dl = getenv("MP3D_DEBUG_RA_DELAY_US");
        d->wk_delay_us = dl ? std::max(0, atoi(dl)) : 0;
        const char *fl = getenv("MP3D_DEBUG_RA_FAIL");
        d->dbg_fail = fl ? std::max(0, atoi(fl)) : 0;
    }
    int r = mp3d_batch_create(device, 1, std::max(1, d->ra_max), &d->b);
    if (r) {
        dec_free(d);
        return r;
    }
    /* the buffers the device writes are coherent (not cached in the GPU's
     * L2), so the completion word's fence orders them for the host */
    const unsigned co = hipHostMallocMapped | hipHostMallocCoherent;
    if (hipHostMalloc((void **)&d->h_in, MP3D_PF_BYTES) != hipSuccess ||
        hipHostMalloc((void **)&d->h_out, sizeof(float) * 2304, co) != hipSuccess ||
        hipHostMalloc((void **)&d->h_info, sizeof(mp3d_frame_info), co) != hipSuccess ||
        hipHostMalloc((void **)&d->h_done, 64, co) != hipSuccess) {
        dec_free(d);
        return MP3D_E_NOMEM;
    }
    if (d->b->poison) { /* MP3D_DEBUG_POISON: the per-call pinned buffers too */
        poison_host(true, d->h_in, MP3D_PF_BYTES);
        poison_host(true, d->h_out, sizeof(float) * 2304);
        poison_host(true, d->h_info, sizeof(mp3d_frame_info));
    }
    *d->h_done = 0u;
    if (!getenv("MP3D_PF_STAGED") && hipHostGetDevicePointer((void **)&d->m_in, d->h_in, 0) == hipSuccess &&
        hipHostGetDevicePointer((void **)&d->m_out, d->h_out, 0) == hipSuccess &&
        hipHostGetDevicePointer((void **)&d->m_info, d->h_info, 0) == hipSuccess &&
        hipHostGetDevicePointer((void **)&d->m_done, d->h_done, 0) == hipSuccess) {
        /* MP3D_PF_FUSED=0: the three-kernel path with a stream sync (tests
         * compare the two) */
        const char *e = getenv("MP3D_PF_FUSED");
        d->fused = !(e && !strcmp(e, "0"));
    } else {
        (void)hipGetLastError();
        d->m_in = nullptr;
        d->m_out = nullptr;
        d->m_info = nullptr;
        d->m_done = nullptr;
    }
    if (d->ra_max && d->m_in) {
        const size_t K = (size_t)d->ra_max;
        /* the md region of a run (k_demux_fp stages no geometry): carry +
         * payloads of K maximal frames + the staging margin, zeroed */
        const size_t md_need = MP3D_RES_BYTES + K * MP3D_MAX_FRAME_BYTES + MP3D_MAX_FRAME_BYTES + 16 + 8192;
        /* zeroed on the handle's own stream and waited for (a null-stream
         * hipMemset does not order before kernels on non-blocking streams;
         * ADVICE r05) */
        if (grow(d->b, (void **)&d->b->md, &d->b->md_cap, md_need) != MP3D_OK ||
            hipMemsetAsync(d->b->md, 0, d->b->md_cap, d->b->own) != hipSuccess ||
            hipStreamSynchronize(d->b->own) != hipSuccess) {
            dec_free(d);
            return MP3D_E_NOMEM;
        }
        /* frames, 64 zero bytes, then the frame offsets (4-B aligned) */
        const size_t in_bytes = K * MP3D_MAX_FRAME_BYTES + 64 + 4 + 4 * K;
        for (auto &u : d->run)
            if (hipHostMalloc((void **)&u.in, in_bytes, hipHostMallocMapped) != hipSuccess ||
                hipHostGetDevicePointer((void **)&u.in_m, u.in, 0) != hipSuccess ||
                hipHostMalloc(&u.pcm, K * 2304 * sizeof(float), co) != hipSuccess ||
                hipHostMalloc((void **)&u.inf, K * sizeof(mp3d_frame_info), co) != hipSuccess ||
                hipMalloc((void **)&u.snap, sizeof(StreamState)) != hipSuccess ||
                hipHostGetDevicePointer(&u.pcm_m, u.pcm, 0) != hipSuccess ||
                hipHostGetDevicePointer((void **)&u.inf_m, u.inf, 0) != hipSuccess ||
                hipEventCreateWithFlags(&u.done, hipEventDisableTiming) != hipSuccess) {
                dec_free(d);
                return MP3D_E_NOMEM;
            }
        if (d->b->poison) /* (the runs' buffers; MP3D_DEBUG_POISON) */
            for (auto &u : d->run) {
                poison_host(true, u.in, in_bytes);
                poison_host(true, u.pcm, K * 2304 * sizeof(float));
                poison_host(true, u.inf, K * sizeof(mp3d_frame_info));
                if (poison_dev(true, u.snap, sizeof(StreamState), d->b->own)) {
                    dec_free(d);
                    return MP3D_E_HIP;
                }
            }
    } else {
        d->ra_max = 0;
    }
    /* the helper thread that launches the next run, started here: started
     * on the first call that reads ahead past one run, its creation (tens of
     * us) landed on that call's latency */
    if (d->ra_max && d->ra_next_on && d->wk_on) {
        try {
            d->wk = std::thread(ra_worker, d);
        } catch (...) {
            d->wk_on = false; /* (the calling thread launches the next run) */
        }
    }
    *out = d;
    return MP3D_OK;
}

extern "C" int mp3d_dec_create(mp3d_dec **out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return mp3d_dec_create_on(dev, out);
}

extern "C" void mp3d_dec_destroy(mp3d_dec *d) {
    if (!d) return;
    dec_free(d);
}

static int ra_settle(mp3d_dec *d);
static int ra_join(mp3d_dec *d);

/* forget both read-ahead runs; a run still decoding is waited for first
 * (its host buffers are reused by the next fill) */
static void ra_drop(mp3d_dec *d) {
    for (auto &u : d->run) {
        if (u.pending) (void)hipEventSynchronize(u.done);
        u.pending = false;
        u.ents.clear();
    }
    d->ra_next = 0;
}

extern "C" void mp3d_dec_reset(mp3d_dec *d) {
    if (!d) return;
    (void)ra_join(d);
    ra_drop(d); /* the state is zeroed whole */
    d->ra_cool = d->ra_backoff = 0;
    d->broken = 0;
    (void)mp3d_batch_reset(d->b);
    d->frames = 0;
    d->kind = 0;
}

extern "C" int mp3d_dec_set_options(mp3d_dec *d, int flags) {
    if (!d) return MP3D_E_ARG;
    const int r = ra_settle(d); /* frames read ahead under the old options */
    if (r) return r;
    return mp3d_batch_set_options(d->b, flags);
}

extern "C" int mp3d_dec_stream_info(mp3d_dec *d, mp3d_stream_info *out) {
    if (!d || !out) return MP3D_E_ARG;
    {
        const int rj = ra_join(d);
        if (rj) return rj;
    }
    return mp3d_batch_stream_info(d->b, 1, out);
}

/* One frame through k_frame (one launch), then a poll of the mapped
 * completion word instead of a stream sync (~5 us less per
 * call).  The frame is in d->h_in[0, have).  Every few thousand polls a
 * stream query catches a kernel that faulted or aborted; a kernel that
 * never completes keeps the stream busy, so after ~1 ms of polling the host
 * stops spinning and blocks in hipStreamSynchronize (a hung kernel then
 * costs a blocked thread, not a spinning core). */
static int pf_fused(mp3d_dec *d, uint32_t have, bool f32, bool lsf) {
    mp3d_batch *b = d->b;
    hipStream_t s = b->own;
    int r = call_begin(b, s);
    if (r) return r;
    CallEnd done{b, s};
    const uint64_t off = 0;
    const uint32_t sz = MP3D_PF_BYTES;
    r = prepare_geometry(b, &off, &sz, 1, s); /* uploaded once, then cached */
    if (!r) r = flush_tail(b, s); /* k_frame reads the state from StreamState */
    if (r) return r;
    const mp3d_batch::Geo &g = b->geo[b->geo_i];
    const uint32_t seq = ++d->seq ? d->seq : ++d->seq; /* never 0, the word's initial value */
    if (b->poison) launch_lds_poison(g_dev[b->device].n_cu, s);
    launch_frame(d->m_in, have, g.in_off(), g.in_len(), b->md, g.md_off(), b->st, b->rec, b->sideu, d->m_info,
                 b->opts, g_dev[b->device].tables, b->is_buf, b->meta, d->m_out, f32, lsf, d->m_done, seq, s);
    HIPCHK(hipGetLastError());
    b->geo[b->geo_i].fresh = false; /* no event per call here: end_event covers it */
    for (uint32_t n = 1;; n++) {
        if (__atomic_load_n(d->h_done, __ATOMIC_ACQUIRE) == seq) return MP3D_OK;
        if ((n & 4095u) == 0) {
            const hipError_t e = n >= (64u << 12) ? hipStreamSynchronize(s) : hipStreamQuery(s);
            if (e == hipErrorNotReady) continue;
            HIPCHK(e);
            /* the stream is idle: the word must be there now */
            if (__atomic_load_n(d->h_done, __ATOMIC_ACQUIRE) == seq) return MP3D_OK;
            return MP3D_E_HIP;
        }
    }
}

/* Settle the read-ahead: the frames decoded ahead but not served are
 * dropped, and the device state is put back to "after the frames served":
 * the state saved before the run being served, then its frames served so
 * far decoded again (the same bytes, so the same state) -- or, when that
 * run was served whole and only the next one is ahead, the state saved
 * before the next run.  A no-op without a read-ahead. */
static int ra_join(mp3d_dec *d);
static int ra_settle_(mp3d_dec *d);
static int ra_settle(mp3d_dec *d) {
    if (d->broken) return d->broken;
    const int r = ra_settle_(d);
    if (r) d->broken = r; /* the restore may have run part-way */
    return r;
}
static int ra_settle_(mp3d_dec *d) {
    {
        const int rj = ra_join(d); /* a launch still on the helper thread */
        if (rj) return rj;
    }
    mp3d_dec::Run &c = d->R(), &n = d->N();
    if (c.ents.empty() && n.ents.empty()) return MP3D_OK;
    const size_t served = d->ra_next;
    const bool cur_all = served == c.ents.size();
    if (cur_all && n.ents.empty()) { /* every frame was served: the state is where the caller is */
        ra_drop(d);
        d->ra_backoff = 0;
        return MP3D_OK;
    }
    d->ra_backoff = std::min(64, std::max(1, 2 * d->ra_backoff));
    d->ra_cool = d->ra_backoff;
    mp3d_batch *b = d->b;
    HIPCHK(hipSetDevice(b->device));
    int r = own_after_last(b); /* (the next run, if any, is on the own stream before this) */
    if (r) return r;
    b->tail_live = -1; /* the tail holds the state after the last run */
    if (cur_all) {
        HIPCHK(hipMemcpyAsync(b->st, n.snap, sizeof(StreamState), hipMemcpyDeviceToDevice, b->own));
        HIPCHK(hipStreamSynchronize(b->own));
    } else {
        HIPCHK(hipMemcpyAsync(b->st, c.snap, sizeof(StreamState), hipMemcpyDeviceToDevice, b->own));
        if (served) {
            const uint64_t off = 0;
            const uint32_t len = c.ents[served - 1].off + c.ents[served - 1].len;
            (void)off;
            const FpRun fp = {c.in_m, len, (const uint32_t *)(c.in + c.fo_at), nullptr, c.snap};
            r = batch_decode(b, c.in_m, &off, &len, 1, (int)served, c.pcm_m, c.f32, c.inf_m, nullptr, true, 3, true,
                             d->ra_seg, &fp, false);
            if (r) return r;
        } else {
            HIPCHK(hipStreamSynchronize(b->own));
        }
    }
    ra_drop(d);
    return MP3D_OK;
}

/* Stage run u from the call's buffer [buf, buf + bytes): the complete
 * frames found there (up to ra_max, located exactly as consecutive calls
 * would locate them: the first one with the stream-start rules when first is
 * set, the MPEG family locked to *kind once known) copied back to back into
 * u.in, then their offsets.  Host work only.  Returns the frames (0 for
 * fewer than 2: nothing staged); *o_out = their bytes, *kinds_out = their
 * families. */
static int ra_stage(mp3d_dec *d, mp3d_dec::Run &u, const uint8_t *buf, size_t bytes, bool first, int *kind,
                    uint32_t *o_out, int *kinds_out) {
    size_t cur = 0;
    uint32_t o = 0;
    int kinds = 0;
    u.ents.clear();
    for (int j = 0; j < d->ra_max; j++) {
        size_t pos = 0, have = 0;
        int fb = -1;
        if (pf_locate(buf + cur, bytes - cur, *kind, first && j == 0, false, &pos, &fb, &have) <= 0 ||
            have < (size_t)fb)
            break;
        memcpy(u.in + o, buf + cur + pos, (size_t)fb);
        u.ents.push_back({o, (uint32_t)fb, pos});
        const int k = host_frame_kind(buf + cur + pos);
        if (!*kind) *kind = k; /* checked again when each is served */
        kinds |= k;
        o += (uint32_t)fb;
        cur += pos + (size_t)fb;
    }
    if (u.ents.size() < 2) {
        u.ents.clear();
        return 0;
    }
    /* 64 zero bytes after the frames, then the frame offsets (k_demux_fp) */
    memset(u.in + o, 0, 64);
    u.fo_at = (o + 64 + 3) & ~3u;
    for (size_t j = 0; j < u.ents.size(); j++) ((uint32_t *)(u.in + u.fo_at))[j] = u.ents[j].off;
    *o_out = o;
    *kinds_out = kinds;
    return (int)u.ents.size();
}

/* Decode a staged run in one batch call -- synchronously, or launched
 * without waiting (async: the next run; its done event is recorded). */
static int ra_launch(mp3d_dec *d, mp3d_dec::Run &u, uint32_t o, int kinds, bool f32, bool async) {
    mp3d_batch *b = d->b;
    HIPCHK(hipSetDevice(b->device));
    int r = own_after_last(b);
    if (r) return r;
    /* the previous run's synthesis tail is flushed into the state, and the
     * state before this run saved to u.snap (for ra_settle), by k_demux_fp */
    const float *tail = b->tail_live >= 0 ? b->st_tail[b->tail_live] : nullptr;
    b->tail_live = -1;
    const uint64_t off = 0;
    const FpRun fp = {u.in_m, o, (const uint32_t *)(u.in + u.fo_at), tail, u.snap};
    r = batch_decode(b, u.in_m, &off, &o, 1, (int)u.ents.size(), u.pcm_m, f32, u.inf_m, nullptr, true, kinds, true,
                     d->ra_seg, &fp, async);
    if (r) return r;
    if (async && d->dbg_fail && ++d->dbg_launches == d->dbg_fail) {
        (void)hipStreamSynchronize(b->own);
        return MP3D_E_HIP;
    }
    u.f32 = f32;
    u.pending = async;
    if (async) HIPCHK(hipEventRecord(u.done, b->own));
    return MP3D_OK;
}

/* wait for the helper thread's launch, if one was handed over; its status */
static int ra_join(mp3d_dec *d) {
    if (!d->wk.joinable()) return MP3D_OK;
    std::unique_lock<std::mutex> lk(d->wk_mu);
    d->wk_cv.wait(lk, [d] { return !d->wk_job; });
    const int rc = d->wk_rc;
    d->wk_rc = 0;
    return rc;
}

static void ra_worker(mp3d_dec *d) {
    for (;;) {
        std::unique_lock<std::mutex> lk(d->wk_mu);
        d->wk_cv.wait(lk, [d] { return d->wk_job || d->wk_quit; });
        if (!d->wk_job) return; /* quit */
        const mp3d_dec::WkJob j = d->wk_arg;
        lk.unlock();
        if (d->wk_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(d->wk_delay_us));
        const int rc = ra_launch(d, *j.u, j.o, j.kinds, j.f32, true);
        lk.lock();
        if (rc) {
            j.u->ents.clear(); /* (the caller sees no next run, and rc at its next join) */
            d->broken = rc;    /* the state may be past the served frames */
        }
        d->wk_rc = rc;
        d->wk_job = false;
        lk.unlock();
        d->wk_cv.notify_all();
    }
}

/* Fill run u synchronously: stage + launch + wait.  Returns 1 for a run of
 * >= 2 frames, else 0 and nothing launched. */
static int ra_fill(mp3d_dec *d, mp3d_dec::Run &u, const uint8_t *buf, size_t bytes, bool f32, bool first, int *kind) {
    uint32_t o = 0;
    int kinds = 0;
    if (!ra_stage(d, u, buf, bytes, first, kind, &o, &kinds)) return 0;
    const int r = ra_launch(d, u, o, kinds, f32, false);
    if (r) {
        u.ents.clear();
        d->broken = r;
        return r;
    }
    return 1;
}

/* the next run: the frames after run[cur] in the call's buffer (which starts
 * at run[cur]'s first frame), staged here and launched by the helper thread,
 * decoding behind the calls served from run[cur] */
static int ra_launch_next(mp3d_dec *d, const uint8_t *buf, size_t bytes, bool f32) {
    if (!d->ra_next_on) return MP3D_OK;
    size_t at = 0;
    for (const auto &e : d->R().ents) at += e.pos + e.len;
    if (at >= bytes) return MP3D_OK;
    /* the family lock: the stream's, or its first frame's (run[cur]'s first) */
    int kind = d->kind ? d->kind : host_frame_kind(buf + d->R().ents[0].pos);
    mp3d_dec::Run &u = d->N();
    uint32_t o = 0;
    int kinds = 0;
    if (!ra_stage(d, u, buf + at, bytes - at, false, &kind, &o, &kinds)) return MP3D_OK;
    if (!d->wk_on) {
        const int r = ra_launch(d, u, o, kinds, f32, true);
        if (r) {
            u.ents.clear();
            d->broken = r;
        }
        return r;
    }
    if (!d->wk.joinable()) d->wk = std::thread(ra_worker, d);
    {
        std::lock_guard<std::mutex> lk(d->wk_mu);
        d->wk_arg = {&u, o, kinds, f32};
        d->wk_job = true;
    }
    d->wk_cv.notify_all();
    return MP3D_OK;
}

static int decode_frame(mp3d_dec *d, const uint8_t *buf, size_t bytes, void *pcm, bool f32, bool last,
                        mp3d_frame_info *info) {
    if (!d || !buf) return MP3D_E_ARG;
    if (d->broken) return d->broken;
    mp3d_frame_info tmp;
    if (!info) info = &tmp;
    memset(info, 0, sizeof(*info));
    size_t pos = 0, have = 0;
    int fb = -1;
    /* next frame (ID3v2 / junk skipped); a final frame cut short only with
     * MP3D_FRAME_LAST: decoded with the missing bytes as zeros (k_demux) */
    const int loc = pf_locate(buf, bytes, d->kind, d->frames == 0, last, &pos, &fb, &have);
    /* a frame read ahead: the same bytes at the same place, the same sink */
    auto same = [&](const mp3d_dec::Run &u, const mp3d_dec::RaEnt &e) {
        return loc > 0 && f32 == u.f32 && pos == e.pos && have == (size_t)fb && (size_t)fb == e.len &&
               !memcmp(buf + pos, u.in + e.off, e.len);
    };
    if (d->ra_next < d->R().ents.size()) {
        if (!same(d->R(), d->R().ents[d->ra_next])) {
            const int r = ra_settle(d);
            if (r) return r;
        }
    } else if (!d->R().ents.empty()) {
        /* the run being served is used up: on to the next run when this call
         * asks for its first frame (it was decoding behind the served calls),
         * and launch the one after it */
        const int rj = ra_join(d); /* the helper's launch of it (its status) */
        if (rj) return rj;
        mp3d_dec::Run &n = d->N();
        if (!n.ents.empty() && same(n, n.ents[0])) {
            if (n.pending) HIPCHK(hipEventSynchronize(n.done));
            n.pending = false;
            d->R().ents.clear();
            d->cur ^= 1;
            d->ra_next = 0;
            d->ra_backoff = 0;
            const int r = ra_launch_next(d, buf, bytes, f32);
            if (r) return r;
        } else {
            const int r = ra_settle(d); /* (served whole: a no-op unless a next run is dropped) */
            if (r) return r;
        }
    }
    if (loc <= 0) {
        info->frame_bytes = (int)pos;
        return loc;
    }
    bool cached = d->ra_next < d->R().ents.size();
    if (!cached) { /* the batch handle is used below */
        const int rj = ra_join(d);
        if (rj) return rj;
    }
    if (!cached && have == (size_t)fb && d->ra_max) {
        if (d->ra_cool > 0) { /* backing off after a wasted read-ahead */
            d->ra_cool--;
        } else {
            int kind = d->kind;
            const int r = ra_fill(d, d->R(), buf, bytes, f32, d->frames == 0, &kind);
            if (r < 0) return r;
            cached = r == 1;
            if (cached) {
                d->ra_next = 0;
                const int r2 = ra_launch_next(d, buf, bytes, f32);
                if (r2) return r2;
            }
        }
    }
    mp3d_frame_info fi;
    const void *out;
    if (cached) {
        const mp3d_dec::Run &c = d->R();
        fi = c.inf[d->ra_next];
        out = (const uint8_t *)c.pcm + d->ra_next * 2304 * (f32 ? sizeof(float) : sizeof(int16_t));
        d->ra_next++;
    } else {
        uint64_t off = 0;
        uint32_t sz = MP3D_PF_BYTES;
        memcpy(d->h_in, buf + pos, have); /* have <= fb <= MP3D_MAX_FRAME_BYTES */
        int r;
        if (d->fused) {
            r = pf_fused(d, (uint32_t)have, f32, host_frame_kind(buf + pos) == 2);
        } else {
            memset(d->h_in + have, 0, MP3D_PF_BYTES - have);
            /* mapped pinned buffers: the kernels read the frame and write PCM +
             * info in place (three launches + one sync); else staged copies */
            const bool mapped = d->m_in != nullptr;
            r = mapped ? batch_decode(d->b, d->m_in, &off, &sz, 1, 1, d->m_out, f32, d->m_info, nullptr, true,
                                      host_frame_kind(buf + pos), true, 0, nullptr, false)
                       : batch_decode(d->b, d->h_in, &off, &sz, 1, 1, d->h_out, f32, d->h_info, nullptr, true,
                                      host_frame_kind(buf + pos), false, 0, nullptr, false); /* 1 MPEG-1, 2 LSF */
        }
        if (r) return r;
        fi = *d->h_info;
        out = d->h_out;
    }
    d->frames++;
    if (fi.frame_bytes) d->kind = host_frame_kind(buf + pos);
    *info = fi;
    info->frame_bytes = (int)pos + (int)std::min<size_t>((size_t)fi.frame_bytes, have);
    if (fi.samples && pcm) memcpy(pcm, out, (f32 ? sizeof(float) : sizeof(int16_t)) * (size_t)fi.samples * fi.channels);
    return fi.samples;
}

extern "C" int mp3d_decode_frame(mp3d_dec *d, const uint8_t *buf, size_t bytes, int16_t *pcm, mp3d_frame_info *info) {
    return decode_frame(d, buf, bytes, pcm, false, false, info);
}

extern "C" int mp3d_decode_frame_f32(mp3d_dec *d, const uint8_t *buf, size_t bytes, float *pcm,
                                     mp3d_frame_info *info) {
    return decode_frame(d, buf, bytes, pcm, true, false, info);
}

extern "C" int mp3d_decode_frame_ex(mp3d_dec *d, const uint8_t *buf, size_t bytes, void *pcm, int flags,
                                    mp3d_frame_info *info) {
    if (flags & ~(MP3D_FRAME_F32 | MP3D_FRAME_LAST)) return MP3D_E_ARG;
    return decode_frame(d, buf, bytes, pcm, (flags & MP3D_FRAME_F32) != 0, (flags & MP3D_FRAME_LAST) != 0, info);
}

/* ------------------------------------------------------------------------ */
/* Per-stream state save / restore                                          */
/* ------------------------------------------------------------------------ */
extern "C" size_t mp3d_state_bytes(void) { return sizeof(StreamState); }

/* every blob must carry this build's format stamp (StreamState.fmt): a blob
 * of another state format would decode with wrong history.  Reads only the
 * blob (a device blob through the handle's own stream, after its last call);
 * the handle's state is untouched. */
static int blob_check(mp3d_batch *b, int n, const void *src) {
    std::vector<uint32_t> fmt((size_t)n);
    const uint8_t *f0 = (const uint8_t *)src + offsetof(StreamState, fmt);
    if (ptr_kind(src, b->device) == PTR_HOST) {
        for (int i = 0; i < n; i++) memcpy(&fmt[i], f0 + sizeof(StreamState) * (size_t)i, sizeof(uint32_t));
    } else {
        HIPCHK(hipSetDevice(b->device));
        int r = own_after_last(b);
        if (r) return r;
        HIPCHK(hipMemcpy2DAsync(fmt.data(), sizeof(uint32_t), f0, sizeof(StreamState), sizeof(uint32_t), (size_t)n,
                                hipMemcpyDefault, b->own));
        HIPCHK(hipStreamSynchronize(b->own));
    }
    for (int i = 0; i < n; i++)
        if (fmt[i] != MP3D_STATE_FMT) return MP3D_E_ARG;
    return MP3D_OK;
}

static int state_copy(mp3d_batch *b, int first, int n, void *dst, const void *src, bool out) {
    if (!b || !(out ? dst : src) || first < 0 || n <= 0) return MP3D_E_ARG;
    if ((long long)first + n > b->max_streams) return MP3D_E_CAPACITY;
    if (!out) {
        const int rb = blob_check(b, n, src); /* before anything is written */
        if (rb) return rb;
    }
    HIPCHK(hipSetDevice(b->device));
    hipStream_t s = b->own;
    int r = own_after_last(b); /* after the handle's last call, on any stream */
    if (r) return r;
    r = flush_tail(b, s);
    if (r) return r;
    StreamState *at = b->st + first;
    HIPCHK(hipMemcpyAsync(out ? dst : (void *)at, out ? (const void *)at : src, sizeof(StreamState) * (size_t)n,
                          hipMemcpyDefault, s));
    HIPCHK(hipStreamSynchronize(s));
    return MP3D_OK;
}

extern "C" int mp3d_batch_get_state(mp3d_batch *b, int first, int n, void *buf) {
    return state_copy(b, first, n, buf, nullptr, true);
}

extern "C" int mp3d_batch_set_state(mp3d_batch *b, int first, int n, const void *buf) {
    return state_copy(b, first, n, nullptr, buf, false);
}

extern "C" int mp3d_dec_get_state(mp3d_dec *d, void *buf) {
    if (!d) return MP3D_E_ARG;
    const int r = ra_settle(d); /* the state after the frames served, not after those read ahead */
    if (r) return r;
    return mp3d_batch_get_state(d->b, 0, 1, buf);
}

extern "C" int mp3d_dec_set_state(mp3d_dec *d, const void *buf) {
    if (!d || !buf) return MP3D_E_ARG;
    {
        /* a refused blob writes nothing (mp3d.h): checked BEFORE the read-ahead
         * is forgotten, so the decoder stays at the frame it served */
        (void)ra_join(d); /* (a failed launch left d->broken, which a new state clears) */
        const int rb = blob_check(d->b, 1, buf);
        if (rb) return rb;
    }
    ra_drop(d); /* replaced whole: nothing read ahead applies */
    const int r = mp3d_batch_set_state(d->b, 0, 1, buf);
    if (r) return r;
    d->broken = 0; /* a whole new state: a failed read-ahead no longer matters */
    /* host mirror of the family lock and "past the stream start" (ID3v2 skip) */
    StreamState h;
    HIPCHK(hipMemcpy(&h, d->b->st, sizeof(h), hipMemcpyDeviceToHost));
    d->kind = h.kind;
    d->frames = (long)h.frames + (h.tag_info ? 1 : 0);
    return MP3D_OK;
}

/* ------------------------------------------------------------------------ */
extern "C" const char *mp3d_strerror(int e) {
    switch (e) {
    case MP3D_OK: return "ok";
    case MP3D_E_ARG: return "bad argument";
    case MP3D_E_NO_DEVICE: return "no usable HIP device (MI355X required; no CPU fallback)";
    case MP3D_E_HIP: return "HIP runtime error";
    case MP3D_E_NOMEM: return "out of memory";
    case MP3D_E_CAPACITY: return "batch exceeds handle capacity";
    case MP3D_E_NEED_MORE: return "no complete frame in buffer";
    default: return "unknown error";
    }
}
extern "C" int mp3d_last_hip_error(void) { return g_last_hip; }
extern "C" int mp3d_abi_version(void) { return MP3D_ABI_VERSION; }
