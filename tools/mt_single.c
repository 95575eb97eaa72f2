/* mt_single.c -- aggregate rate of concurrent single-call qlz_decompress callers (tools only).
 *
 * The calls store/item.go:167 makes once per GET, from many goroutines (cgo runs each blocking
 * call on its own OS thread).  N pthreads decode DISTINCT values through `lib` (dlopen:
 * libqlzx.so or the reference oracle/_ref build) for S seconds: thread t walks the value set
 * from value t * count / N on, so no thread decodes one value twice in a row and the set (>= 1024
 * values) is far larger than a branch predictor's memory.  Every 16th result is compared with
 * the expected bytes.  Prints one JSON line.
 *
 * VALUES file: repeated [u32 clen][u32 dlen][clen compressed bytes][dlen plain bytes].
 * build: gcc -O2 -pthread -o mt_single tools/mt_single.c -ldl
 * usage: mt_single LIB VALUES THREADS SECONDS
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef size_t (*dec_fn)(const char *, void *, char *);
static dec_fn dec;
static const char **comp;
static const unsigned char **want;
static uint32_t *dlen;
static long count, nthreads;
static size_t maxd;
static atomic_int stop;
static atomic_long total, bad, bytes;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *worker(void *arg) {
    const long t = (long)(intptr_t)arg;
    unsigned char *out = malloc(maxd + 64);
    char *scratch = malloc(528400);
    long n = 0, b = 0, k = t * count / nthreads, by = 0;
    while (!atomic_load_explicit(&stop, memory_order_relaxed)) {
        const size_t d = dec(comp[k], out, scratch);
        if (d != dlen[k] || ((n & 15) == 0 && memcmp(out, want[k], d))) b++;
        by += dlen[k];
        n++;
        if (++k == count) k = 0;
    }
    atomic_fetch_add(&total, n);
    atomic_fetch_add(&bad, b);
    atomic_fetch_add(&bytes, by);
    free(out);
    free(scratch);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 5) return fprintf(stderr, "usage: %s LIB VALUES THREADS SECONDS\n", argv[0]), 2;
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) return fprintf(stderr, "dlopen: %s\n", dlerror()), 1;
    dec = (dec_fn)dlsym(h, "qlz_decompress");
    if (!dec) return fprintf(stderr, "qlz_decompress missing\n"), 1;
    FILE *f = fopen(argv[2], "rb");
    if (!f) return perror("open"), 1;
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = malloc(len);
    if (fread(buf, 1, len, f) != (size_t)len) return fprintf(stderr, "short read\n"), 1;
    fclose(f);
    for (long p = 0; p + 8 <= len; count++) {
        uint32_t c, d;
        memcpy(&c, buf + p, 4);
        memcpy(&d, buf + p + 4, 4);
        p += 8 + (long)c + (long)d;
    }
    comp = malloc(sizeof(char *) * count);
    want = malloc(sizeof(char *) * count);
    dlen = malloc(sizeof(uint32_t) * count);
    long p = 0;
    for (long i = 0; i < count; i++) {
        uint32_t c;
        memcpy(&c, buf + p, 4);
        memcpy(&dlen[i], buf + p + 4, 4);
        comp[i] = buf + p + 8;
        want[i] = (const unsigned char *)buf + p + 8 + c;
        p += 8 + (long)c + dlen[i];
        if (dlen[i] > maxd) maxd = dlen[i];
    }
    nthreads = atoi(argv[3]);
    const double secs = atof(argv[4]);
    pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
    const double t0 = now();
    for (long i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, (void *)(intptr_t)i);
    struct timespec ts = {(time_t)secs, (long)((secs - (time_t)secs) * 1e9)};
    nanosleep(&ts, NULL);
    atomic_store(&stop, 1);
    for (long i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    const double dt = now() - t0;
    const long n = atomic_load(&total);
    printf("{\"lib\": \"%s\", \"threads\": %ld, \"values\": %ld, \"dsize\": %zu, \"calls\": %ld, \"bad\": %ld, "
           "\"seconds\": %.3f, \"calls_per_s\": %.0f, \"GiBps\": %.3f, \"us_per_call_per_thread\": %.2f}\n",
           argv[1], nthreads, count, maxd, n, atomic_load(&bad), dt, n / dt, atomic_load(&bytes) / dt / (1 << 30),
           dt * 1e6 * nthreads / (n ? n : 1));
    return atomic_load(&bad) ? 1 : 0;
}
