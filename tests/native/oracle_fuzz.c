/*
 * oracle_fuzz.c -- sanitizer harness for the CPU oracle (oracle/mp3_oracle.c,
 * compiled into this file with -fsanitize=address,undefined by
 * tests/test_sanitize.py): decodes every record of a fuzz corpus ([u32
 * len][len bytes]) from an exact-size heap copy, with and without the CRC
 * option, and reads its Xing/LAME tag.  Exit status 0 = clean.
 */
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/mp3_oracle.c"

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    enum { MAXF = 64 };
    float *pcm = (float *)malloc(sizeof(float) * 2 * MAXF * 1152);
    long recs = 0, frames = 0;
    for (;;) {
        uint32_t n;
        if (fread(&n, 4, 1, f) != 1) break;
        uint8_t *p = (uint8_t *)malloc(n ? n : 1);
        if (n && fread(p, 1, n, f) != n) return 2;
        for (int opts = 0; opts < 2; opts++) {
            int nch = 0, hz = 0;
            long ns = 0;
            frames += orc_decode_stream_opts(p, (long)n, pcm, MAXF, &nch, &hz, &ns, opts);
        }
        int tag[6];
        (void)orc_parse_info_tag(p, (long)n, tag);
        free(p);
        recs++;
    }
    fclose(f);
    free(pcm);
    printf("oracle_fuzz: %ld records, %ld frames\n", recs, frames);
    return 0;
}
