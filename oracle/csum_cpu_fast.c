/*
 * csum_cpu_fast.c — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * The "honest best CPU" line SURVEY.md §8d asks for beside the Go-faithful
 * baseline: the same raw sums as transport/tcp/tcp.go:72-95 (no prefix), but
 * computed the way a tuned CPU library would — 8-byte little-endian loads summed
 * as 32-bit halves into u64 accumulators (auto-vectorised at -O3), folded, and
 * byte-swapped when the segment starts at an even stream position (the same
 * byte-order identity the GPU kernels use) — over contiguous index
 * shards on `threads` pthreads. Used only by bench.py's cpu_baseline leg (as
 * extra reference numbers) and checked against oracle_go_checksum in
 * tests/test_oracle.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#define FAST_EXPORT __attribute__((visibility("default")))

static inline uint32_t fold(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint32_t)s;
}

/* Raw sum of prefix ‖ seg[0, len) as a stream starting at an even position, the
 * prefix given as its BE-word partial (the d_prefix_partial convention). */
static uint16_t fast_one(const uint8_t* p, size_t len, uint32_t partial) {
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        uint64_t w[4];
        memcpy(w, p + i, 32);
        a0 += (w[0] & 0xFFFFFFFFu) + (w[0] >> 32);
        a1 += (w[1] & 0xFFFFFFFFu) + (w[1] >> 32);
        a2 += (w[2] & 0xFFFFFFFFu) + (w[2] >> 32);
        a3 += (w[3] & 0xFFFFFFFFu) + (w[3] >> 32);
    }
    uint64_t s = a0 + a1 + a2 + a3;
    for (; i + 2 <= len; i += 2) s += (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8);  /* LE halves */
    if (i < len) s += p[i];  /* odd tail: low byte of an LE half = high byte of its BE word */
    uint32_t le = fold(s);
    return (uint16_t)fold((uint64_t)(((le & 0xFFu) << 8) | (le >> 8)) + partial); /* LE sum → BE sum */
}

typedef struct {
    const uint8_t* base; uint64_t stride; uint32_t seg_len; uint64_t lo, hi; const uint32_t* partial; uint16_t* out;
} fast_arg;

static void* fast_run(void* a_) {
    fast_arg* a = (fast_arg*)a_;
    for (uint64_t i = a->lo; i < a->hi; i++) a->out[i] = fast_one(a->base + i * a->stride, a->seg_len, a->partial ? a->partial[i] : 0u);
    return NULL;
}

/* partial (nullable): per-segment pseudo-header partials, as nsx_csum_fixed_dev takes them. */
FAST_EXPORT void cpu_fast_batch_fixed(const uint8_t* base, uint64_t stride, uint32_t seg_len, uint64_t n,
                                      const uint32_t* partial, uint16_t* out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    fast_arg args[256];
    for (int t = 0; t < threads; t++) {
        args[t] = (fast_arg){base, stride, seg_len, n * t / threads, n * (t + 1) / threads, partial, out};
        pthread_create(&th[t], NULL, fast_run, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
