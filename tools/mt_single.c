/* mt_single.c -- aggregate rate of concurrent single-call qlz_decompress callers (tools only).
 *
 * The calls store/item.go:167 makes once per GET, from many goroutines (cgo runs each blocking
 * call on its own OS thread).  N pthreads each decode the same compressed value in a loop for
 * S seconds through `lib` (dlopen: libqlzx.so or the reference oracle/_ref build); every result
 * is checked against the first call's output.  Prints one JSON line.
 *
 * build: gcc -O2 -pthread -o mt_single tools/mt_single.c -ldl
 * usage: mt_single LIB COMPRESSED_FILE THREADS SECONDS
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
static const char *comp;
static size_t dsize;
static unsigned char *want;
static atomic_int stop;
static atomic_long total, bad;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *worker(void *arg) {
    (void)arg;
    unsigned char *out = malloc(dsize + 64);
    char *scratch = malloc(528400);
    long n = 0, b = 0;
    while (!atomic_load_explicit(&stop, memory_order_relaxed)) {
        if (dec(comp, out, scratch) != dsize || memcmp(out, want, dsize)) b++;
        n++;
    }
    atomic_fetch_add(&total, n);
    atomic_fetch_add(&bad, b);
    free(out);
    free(scratch);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 5) return fprintf(stderr, "usage: %s LIB FILE THREADS SECONDS\n", argv[0]), 2;
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) return fprintf(stderr, "dlopen: %s\n", dlerror()), 1;
    dec = (dec_fn)dlsym(h, "qlz_decompress");
    size_t (*sz)(const char *) = (size_t(*)(const char *))dlsym(h, "qlz_size_decompressed");
    if (!dec || !sz) return fprintf(stderr, "symbols missing\n"), 1;
    FILE *f = fopen(argv[2], "rb");
    if (!f) return perror("open"), 1;
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *c = malloc(len);
    if (fread(c, 1, len, f) != (size_t)len) return fprintf(stderr, "short read\n"), 1;
    fclose(f);
    comp = c;
    dsize = sz(comp);
    want = malloc(dsize + 64);
    char *scratch = malloc(528400);
    if (dec(comp, want, scratch) != dsize) return fprintf(stderr, "first decode failed\n"), 1;
    const int nt = atoi(argv[3]);
    const double secs = atof(argv[4]);
    pthread_t *th = malloc(sizeof(pthread_t) * nt);
    const double t0 = now();
    for (int i = 0; i < nt; i++) pthread_create(&th[i], NULL, worker, NULL);
    struct timespec ts = {(time_t)secs, (long)((secs - (time_t)secs) * 1e9)};
    nanosleep(&ts, NULL);
    atomic_store(&stop, 1);
    for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
    const double dt = now() - t0;
    const long n = atomic_load(&total);
    printf("{\"lib\": \"%s\", \"threads\": %d, \"dsize\": %zu, \"calls\": %ld, \"bad\": %ld, \"seconds\": %.3f, "
           "\"calls_per_s\": %.0f, \"GiBps\": %.3f, \"us_per_call_per_thread\": %.2f}\n",
           argv[1], nt, dsize, n, atomic_load(&bad), dt, n / dt, n * (double)dsize / dt / (1 << 30),
           dt * 1e6 * nt / (n ? n : 1));
    return atomic_load(&bad) ? 1 : 0;
}
