/*
 * host_fuzz.cpp -- sanitizer harness for the library's host-side byte parsing
 * (mp3_amd/csrc/mp3d_hostparse.h: walk_frames, long_plan, pf_locate), built
 * with -fsanitize=address,undefined by tests/test_sanitize.py and run over a
 * fuzz corpus (random bytes with sync words, generator streams cut at random
 * points, the golden fixtures).  Corpus file: records of [u32 len][len bytes].
 * Also checks the invariants the GPU path relies on.  Exit status 0 = clean.
 */
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mp3d_hostparse.h"

using namespace mp3d;

#define CHECK(c)                                                                                                       \
    do {                                                                                                               \
        if (!(c)) {                                                                                                    \
            fprintf(stderr, "check failed: %s (record %zu)\n", #c, rec);                                             \
            return 1;                                                                                                  \
        }                                                                                                              \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    size_t rec = 0, frames = 0, pf_frames = 0;
    for (;;) {
        uint32_t n;
        if (fread(&n, 4, 1, f) != 1) break;
        /* exact-size heap copy: ASan flags any read past the stream's end */
        uint8_t *p = (uint8_t *)malloc(n ? n : 1);
        if (n && fread(p, 1, n, f) != n) return 2;
        std::vector<uint64_t> off;
        std::vector<uint32_t> pay;
        walk_frames(p, n, off, pay);
        for (size_t i = 0; i < off.size(); i++) {
            CHECK(off[i] + 4 <= n);
            CHECK(i == 0 || off[i] > off[i - 1]);
            CHECK(pay[i] <= MP3D_MAX_FRAME_BYTES);
        }
        frames += off.size();
        for (int L : {1, 2, 3, 7, 32}) {
            std::vector<uint64_t> o2;
            std::vector<long long> a;
            int wmax = -1;
            CHECK(long_plan(p, n, L, (long long)n + 8, o2, a, &wmax) == MP3D_OK);
            CHECK(o2 == off);
            CHECK((long long)a.size() == ((long long)off.size() + L - 1) / L);
            for (size_t k = 0; k < a.size(); k++) CHECK(a[k] >= 0 && a[k] <= (long long)k * L);
            CHECK(wmax >= 0);
            if (!off.empty()) CHECK(long_plan(p, n, L, (long long)off.size() - 1, o2, a, &wmax) == MP3D_E_CAPACITY);
        }
        /* the per-frame call's walk over the whole buffer, as decode_stream */
        for (int last = 0; last < 2; last++) {
            size_t cur = 0, start = 1;
            int kind = 0;
            while (cur < n) {
                size_t pos = 0, have = 0;
                int fb = -1;
                const int r = pf_locate(p + cur, n - cur, kind, start != 0, last != 0, &pos, &fb, &have);
                if (r < 0) break;
                if (r == 0) {
                    CHECK(pos > 0 && cur + pos <= n);
                    cur += pos;
                    continue;
                }
                CHECK(cur + pos + 4 <= n && have > 0 && have <= (size_t)fb && cur + pos + have <= n);
                CHECK(fb <= MP3D_MAX_FRAME_BYTES + 1);
                kind = host_frame_kind(p + cur + pos);
                start = 0;
                cur += pos + have;
                pf_frames++;
            }
        }
        free(p);
        rec++;
    }
    fclose(f);
    printf("host_fuzz: %zu records, %zu frame slots, %zu per-frame frames\n", rec, frames, pf_frames);
    return 0;
}
