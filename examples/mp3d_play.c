/* mp3d_play: the player's decode loop in plain C over the C ABI
 * (include/mp3d.h) -- what a host application links against instead of its
 * CPU decoder.  Reads an MP3 file, decodes it frame by frame
 * on the GPU with mp3d_decode_frame, optionally applies the LAME gapless trim
 * (mp3d_dec_stream_info), and writes a 16-bit PCM WAV file.
 *
 *   mp3d_play in.mp3 out.wav [--gapless] [--crc] [--time]
 *
 * --time prints the median and p99 wall time of the mp3d_decode_frame calls
 * (after 20 warm-up frames) to stderr: the per-frame latency as a C caller
 * sees it.
 *
 * Build: make -C examples (gcc, links mp3_amd/libmp3d.so).  Exit status 0 on
 * success, 1 on a usage / file error, 2 when the library reports an error
 * (no GPU: MP3D_E_NO_DEVICE -- there is no CPU fallback). */
#include <stdint.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include "mp3d.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}
static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static void put_u32(FILE *f, uint32_t v) {
    const uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
    fwrite(b, 1, 4, f);
}
static void put_u16(FILE *f, uint16_t v) {
    const uint8_t b[2] = {(uint8_t)v, (uint8_t)(v >> 8)};
    fwrite(b, 1, 2, f);
}

static int write_wav(const char *path, const int16_t *pcm, long long frames, int nch, int hz) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    const uint32_t data = (uint32_t)(frames * nch * 2);
    fwrite("RIFF", 1, 4, f);
    put_u32(f, 36 + data);
    fwrite("WAVEfmt ", 1, 8, f);
    put_u32(f, 16);
    put_u16(f, 1); /* WAVE_FORMAT_PCM */
    put_u16(f, (uint16_t)nch);
    put_u32(f, (uint32_t)hz);
    put_u32(f, (uint32_t)(hz * nch * 2));
    put_u16(f, (uint16_t)(nch * 2));
    put_u16(f, 16);
    fwrite("data", 1, 4, f);
    put_u32(f, data);
    for (long long i = 0; i < frames * nch; i++) put_u16(f, (uint16_t)pcm[i]); /* little-endian */
    return fclose(f) == 0 ? 0 : -1;
}

int main(int argc, char **argv) {
    int gapless = 0, crc = 0, timing = 0;
    if (argc < 3) {
        fprintf(stderr, "usage: %s in.mp3 out.wav [--gapless] [--crc] [--time]\n", argv[0]);
        return 1;
    }
    for (int i = 3; i < argc; i++) {
        if (!strcmp(argv[i], "--gapless")) gapless = 1;
        else if (!strcmp(argv[i], "--crc")) crc = 1;
        else if (!strcmp(argv[i], "--time")) timing = 1;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *buf = (uint8_t *)malloc((size_t)len + 1);
    if (!buf || fread(buf, 1, (size_t)len, f) != (size_t)len) { fclose(f); fprintf(stderr, "read error\n"); return 1; }
    fclose(f);

    mp3d_dec *dec;
    int rc = mp3d_dec_create(&dec);
    if (rc < 0) { fprintf(stderr, "mp3d_dec_create: %s\n", mp3d_strerror(rc)); return 2; }
    if (crc) mp3d_dec_set_options(dec, MP3D_OPT_CRC_CHECK);

    /* interleaved PCM grows as frames arrive (1152 or 576 samples each) */
    long long cap = 1 << 20, n = 0; /* samples per channel */
    int nch = 0, hz = 0;
    int16_t *pcm = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)cap);
    int16_t frame[2304];
    mp3d_frame_info info;
    size_t pos = 0;
    long n_lat = 0;
    double *lat = (double *)malloc(sizeof(double) * ((size_t)len / 24 + 2)); /* >= frames in the file */
    while (pos < (size_t)len) {
        const double t0 = timing ? now_us() : 0.0;
        const int got = mp3d_decode_frame(dec, buf + pos, (size_t)len - pos, frame, &info);
        if (timing) lat[n_lat++] = now_us() - t0;
        if (got == MP3D_E_NEED_MORE) break; /* no complete frame left */
        if (got < 0) { fprintf(stderr, "mp3d_decode_frame: %s\n", mp3d_strerror(got)); return 2; }
        if (info.frame_bytes <= 0) break;
        pos += (size_t)info.frame_bytes;
        if (got == 0) continue; /* tag frame, dropped frame */
        if (nch && (info.channels != nch || info.hz != hz)) continue; /* keep one output format */
        nch = info.channels;
        hz = info.hz;
        if (n + got > cap) {
            cap *= 2;
            pcm = (int16_t *)realloc(pcm, sizeof(int16_t) * 2 * (size_t)cap);
        }
        memcpy(pcm + n * nch, frame, sizeof(int16_t) * (size_t)got * nch);
        n += got;
    }
    long long start = 0, stop = n;
    if (gapless) {
        mp3d_stream_info si;
        if (mp3d_dec_stream_info(dec, &si) == MP3D_OK && si.has_lame) {
            start = si.skip_samples < n ? si.skip_samples : n;
            if (si.end_sample >= 0 && si.end_sample < stop) stop = si.end_sample;
            if (stop < start) stop = start;
        }
    }
    mp3d_dec_destroy(dec);
    if (timing && n_lat > 40) {
        qsort(lat + 20, (size_t)(n_lat - 20), sizeof(double), cmp_d);
        const long m = n_lat - 20;
        fprintf(stderr, "mp3d_decode_frame: %ld calls, median %.2f us, p99 %.2f us\n", m, lat[20 + m / 2],
                lat[20 + (m * 99) / 100]);
    }
    free(lat);
    if (!nch) nch = 2, hz = 44100; /* no audio: an empty WAV */
    rc = write_wav(argv[2], pcm + start * nch, stop - start, nch, hz);
    free(pcm);
    free(buf);
    if (rc) { perror(argv[2]); return 1; }
    printf("%lld samples x %d ch @ %d Hz\n", stop - start, nch, hz);
    return 0;
}
