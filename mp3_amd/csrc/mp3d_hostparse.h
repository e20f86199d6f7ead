/*
 * mp3d_hostparse.h -- the host-side byte parsing of the library, free of
 * HIP so that the sanitizer harness (tests/native/host_fuzz.cpp, built with
 * -fsanitize=address,undefined by tests/test_sanitize.py) runs it on CPU:
 *
 *   host_frame_*    Layer III header -> family, frame bytes, header + side
 *                   info bytes (ISO 11172-3 2.4.2.3, 13818-3; = k_demux's
 *                   hdr_frame_bytes)
 *   id3v2_end       end of a leading ID3v2 tag
 *   walk_frames     frame slots of a stream exactly as k_demux enumerates
 *                   them (mp3d_batch_decode_long, mp3d_long_plan)
 *   long_plan       segment plan of the frame-parallel long-stream decode
 *   pf_locate       the per-frame call's search for the next frame
 *                   (mp3d_decode_frame / _ex)
 */
#ifndef MP3D_HOSTPARSE_H
#define MP3D_HOSTPARSE_H

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/mp3d.h"
#include "mp3d_internal.h"
#include "mp3d_tables.h"

namespace mp3d {

/* MPEG family of a header: 1 MPEG-1, 2 MPEG-2 / 2.5 LSF */
static inline int host_frame_kind(const uint8_t *p) { return ((p[1] >> 3) & 3) == 3 ? 1 : 2; }

/* Layer III frame bytes of the 4-byte header at p, or -1: MPEG-1 and
 * MPEG-2 / 2.5 LSF; kind 0 any family, 1 MPEG-1 only, 2 LSF only */
static inline int host_frame_bytes(const uint8_t *p, int kind) {
    const int ver = (p[1] >> 3) & 3;
    if (p[0] != 0xFF || (p[1] & 0xE0) != 0xE0 || ((p[1] >> 1) & 3) != 1 || ver == 1) return -1;
    const int bi = p[2] >> 4, si = (p[2] >> 2) & 3;
    if (bi == 0 || bi == 15 || si == 3) return -1;
    const int k = host_frame_kind(p);
    if (kind && k != kind) return -1;
    const int hz = (int)MP3D_SAMPLE_RATE[si + (ver == 3 ? 0 : ver == 2 ? 3 : 6)];
    return (k == 1 ? 144000 * (int)MP3D_BITRATE_L3[bi] : 72000 * (int)MP3D_BITRATE_L3_LSF[bi]) / hz +
           ((p[2] >> 1) & 1);
}

/* header + CRC + side-info bytes */
static inline int host_frame_head(const uint8_t *p) {
    const bool mono = (p[3] >> 6) == 3, lsf = host_frame_kind(p) == 2;
    return 4 + ((p[1] & 1) ? 0 : 2) + (lsf ? (mono ? 9 : 17) : (mono ? 17 : 32));
}

/* end of a leading ID3v2 tag (10-byte header, syncsafe size, optional
 * footer), or 0; may lie beyond len */
static inline size_t id3v2_end(const uint8_t *p, size_t len) {
    if (len < 10 || p[0] != 'I' || p[1] != 'D' || p[2] != '3') return 0;
    return 10 + (((size_t)(p[6] & 0x7F) << 21) | ((size_t)(p[7] & 0x7F) << 14) | ((size_t)(p[8] & 0x7F) << 7) |
                 (p[9] & 0x7F)) +
           ((p[5] & 0x10) ? 10 : 0);
}

/* Frame slots of a stream exactly as k_demux enumerates them: ID3v2 skip,
 * resync on the next valid header of the stream's family, a cut-short final
 * frame kept while its header and side info are present.  payload = bytes
 * after the side info. */
static inline void walk_frames(const uint8_t *p, size_t len, std::vector<uint64_t> &off,
                               std::vector<uint32_t> &payload) {
    size_t cur = id3v2_end(p, len);
    int kind = 0; /* MPEG family lock, as k_demux */
    while (cur + 4 <= len) {
        int fb = -1;
        for (; cur + 4 <= len; cur++)
            if ((fb = host_frame_bytes(p + cur, kind)) > 0) break;
        if (fb <= 0) break;
        kind = host_frame_kind(p + cur);
        const size_t need = (size_t)host_frame_head(p + cur);
        if (cur + fb > len && cur + need > len) break;
        off.push_back(cur);
        payload.push_back(fb > (int)need ? (uint32_t)(fb - need) : 0u);
        cur = cur + fb <= len ? cur + fb : len;
    }
}

/* Split the stream into segments of L output frames decoded as independent
 * virtual streams of one batch call.  Segment k (k >= 1) starts at frame
 * a_k < kL, chosen so that the payloads of frames [a_k, kL - 2) hold >= 511
 * bytes (the largest main_data_begin).  Why that suffices (k_demux's
 * reservoir rule): the bytes available after a frame, P + plen - end, do not
 * depend on the history once the frame's main-data start P - mdb is inside
 * the virtual stream's md region, i.e. from frame kL - 2 on; frame kL - 1
 * then decodes from real bytes with the sequential decoder's reservoir
 * decision, and its second granule alone feeds frame kL's IMDCT overlap and
 * synthesis FIFO (15 slots < 18 per granule).  Output frames [kL, (k+1)L)
 * are therefore bit-exact with a sequential decode of the whole stream;
 * warm-up output is dropped. */
static inline int long_plan(const uint8_t *p, size_t bytes, int L, long long max_frames, std::vector<uint64_t> &off,
                            std::vector<long long> &a, int *wmax) {
    std::vector<uint32_t> pay;
    walk_frames(p, bytes, off, pay);
    const long long N = (long long)off.size();
    if (N > max_frames) return MP3D_E_CAPACITY;
    const long long K = (N + L - 1) / L;
    a.assign((size_t)K, 0);
    *wmax = 0;
    for (long long k = 0; k < K; k++) {
        long long j = std::max(0LL, k * L - 2), acc = 0;
        while (j > 0 && acc < MP3D_RES_BYTES - 1) acc += pay[(size_t)--j];
        a[(size_t)k] = j;
        *wmax = std::max(*wmax, (int)(k * L - j));
    }
    return MP3D_OK;
}

/* The per-frame call's frame search in buf[0 .. bytes): skips a leading
 * ID3v2 tag (first call of a stream) and junk up to the next header of the
 * stream's family.  Returns 1 with *pos, *fb (frame bytes) and *have (bytes
 * of it present: < fb only for a final frame cut short, accepted with
 * `last` once its header and side info are present); 0 when the bytes up to
 * *pos hold no frame (consume them); MP3D_E_NEED_MORE when nothing can be
 * consumed yet. */
static inline int pf_locate(const uint8_t *buf, size_t bytes, int kind, bool stream_start, bool last, size_t *pos,
                            int *fb, size_t *have) {
    size_t p = stream_start ? id3v2_end(buf, bytes) : 0;
    int f = -1;
    while (p + 4 <= bytes) {
        f = host_frame_bytes(buf + p, kind);
        if (f > 0) break;
        p++;
    }
    const bool cut = f > 0 && p + (size_t)f > bytes;
    if (f <= 0 || (cut && !(last && p + (size_t)host_frame_head(buf + p) <= bytes))) {
        *pos = std::min(p, bytes);
        return *pos ? 0 : MP3D_E_NEED_MORE;
    }
    *pos = p;
    *fb = f;
    *have = cut ? bytes - p : (size_t)f;
    return 1;
}

} // namespace mp3d
#endif
