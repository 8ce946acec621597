/*
 * TEST INFRASTRUCTURE (oracle/) — never linked into the product.
 *
 * Deterministic synthetic-weight generator used by the CPU oracle.  The product
 * (deepseek-ocr.rs_amd/csrc/common/synth.hpp) carries its own copy of the same
 * published recipe; tests/test_synth.py checks the two agree byte for byte.
 *
 * Recipe (the reference ships no checkpoint in this container):
 *   key  = fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15)
 *   z    = splitmix64(key + (i + 1) * 0x9E3779B97F4A7C15)
 *   c    = byte0(z) + byte1(z) + byte2(z) + byte3(z) - 510      (Irwin-Hall, std 147.80)
 *   v    = (float)c * (float)(std / 147.80) + mean              (one rounding each)
 *   bf16 = round-to-nearest-even(v)
 * The values are bf16 because the real DeepSeek-OCR checkpoint is bf16
 * (reference tests/config.rs:36 pins torch_dtype "bfloat16").
 */
#include <stdint.h>
#include <string.h>

static uint64_t fnv1a64(const char *s) {
    uint64_t h = 1469598103934665603ULL;
    while (*s) { h ^= (uint8_t)(*s++); h *= 1099511628211ULL; }
    return h;
}

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u; memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* Fill out[0..n) with bf16 bit patterns. */
void dsocr_oracle_synth_bf16(const char *name, uint64_t seed, double mean, double std,
                             uint64_t n, uint16_t *out) {
    const uint64_t key = fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15ULL);
    const float scale = (float)(std / 147.80);
    const float fmean = (float)mean;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint64_t z = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        int c = (int)(z & 0xff) + (int)((z >> 8) & 0xff) + (int)((z >> 16) & 0xff) +
                (int)((z >> 24) & 0xff) - 510;
        float v = (float)c * scale;
        v = v + fmean;
        out[i] = f32_to_bf16_rne(v);
    }
}
