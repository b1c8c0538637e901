/*
 * vds_oracle.c -- TEST INFRASTRUCTURE ONLY (see vds_oracle.h).
 *
 * Plain-C restatement of lboss75/vds kernel/vds_data/{gf.h,chunk.h}.  It keeps
 * the reference's structure on purpose (log/antilog tables, `% 0xFFFF`, one
 * pass per replica, byte-wise big-endian cell packing) so that it is both a
 * faithful parity checker and a fair single-thread CPU baseline.
 */
#include "vds_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ gf<m> */

/* gf.h:42-67: for each of the m bits of b (LSB first): if set, xor a into the
 * product; then shift a left one bit and, if the bit that fell off was the
 * top bit (gf.h:18-19,57), xor in the low polynomial bytes (gf.h:100-126). */
uint32_t vds_oracle_gf_mul_bitserial(unsigned m, uint32_t poly_low, uint32_t a, uint32_t b)
{
    const unsigned bytes = (m + 7) / 8; /* gf<m>::ArraySize, gf.h:21 */
    const uint32_t width_mask = bytes >= 4 ? 0xFFFFFFFFu : ((1u << (8 * bytes)) - 1u);
    const uint32_t hi_bit = 1u << (m - 1);
    uint32_t prod = 0;
    for (unsigned i = 0; i < m; ++i) {
        if (b & 1u) prod ^= a;
        int hi = (a & hi_bit) != 0;
        a = (a << 1) & width_mask; /* shift_left over ArraySize bytes (gf.h:268-281) */
        if (hi) a ^= poly_low;
        b >>= 1;                   /* shift_right (gf.h:282-295) */
    }
    return prod;
}

/* ------------------------------------------------------------ gf_math<> */

static uint8_t g8_v2l[256], g8_l2v[256];
static uint16_t g16_v2l[65536], g16_l2v[65536];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

void vds_oracle_gf8_tables(uint8_t *value2log, uint8_t *log2value)
{
    /* gf.h:135-154 */
    memset(value2log, 0, 256);
    memset(log2value, 0, 256);
    log2value[0] = 1;
    value2log[1] = 0;
    uint32_t k = 2;
    for (unsigned log = 1; log < 255; ++log) {
        log2value[log] = (uint8_t)k;
        value2log[k] = (uint8_t)log;
        k = vds_oracle_gf_mul_bitserial(8, 0x1D, k, 2);
    }
}

void vds_oracle_gf16_tables(uint16_t *value2log, uint16_t *log2value)
{
    /* gf.h:197-216; log2value[0xFFFF] keeps its static zero (never read). */
    memset(value2log, 0, 65536 * sizeof(uint16_t));
    memset(log2value, 0, 65536 * sizeof(uint16_t));
    log2value[0] = 1;
    value2log[1] = 0;
    uint32_t k = 2;
    for (unsigned log = 1; log < 0xFFFF; ++log) {
        log2value[log] = (uint16_t)k;
        value2log[k] = (uint16_t)log;
        k = vds_oracle_gf_mul_bitserial(16, 0x100B, k, 2);
    }
}

static void init_tables(void)
{
    vds_oracle_gf8_tables(g8_v2l, g8_l2v);
    vds_oracle_gf16_tables(g16_v2l, g16_l2v);
}

static inline void ensure_tables(void) { pthread_once(&g_once, init_tables); }

/* gf.h:156-165 */
static inline uint8_t mul8(uint8_t a, uint8_t b)
{
    if (a == 0 || b == 0) return 0;
    return g8_l2v[((unsigned)g8_v2l[a] + (unsigned)g8_v2l[b]) % 255];
}
/* gf.h:167-179 */
static inline uint8_t div8(uint8_t a, uint8_t b)
{
    if (a == 0 || b == 0) return 0;
    int dif = (int)g8_v2l[a] - (int)g8_v2l[b];
    while (dif < 0) dif += 255;
    return g8_l2v[dif % 255];
}
/* gf.h:218-227 */
static inline uint16_t mul16(uint16_t a, uint16_t b)
{
    if (a == 0 || b == 0) return 0;
    return g16_l2v[((unsigned)g16_v2l[a] + (unsigned)g16_v2l[b]) % 0xFFFF];
}
/* gf.h:229-241 */
static inline uint16_t div16(uint16_t a, uint16_t b)
{
    if (a == 0 || b == 0) return 0;
    int dif = (int)g16_v2l[a] - (int)g16_v2l[b];
    while (dif < 0) dif += 0xFFFF;
    return g16_l2v[dif % 0xFFFF];
}

uint8_t vds_oracle_gf8_mul(uint8_t a, uint8_t b) { ensure_tables(); return mul8(a, b); }
uint8_t vds_oracle_gf8_div(uint8_t a, uint8_t b) { ensure_tables(); return div8(a, b); }
uint16_t vds_oracle_gf16_mul(uint16_t a, uint16_t b) { ensure_tables(); return mul16(a, b); }
uint16_t vds_oracle_gf16_div(uint16_t a, uint16_t b) { ensure_tables(); return div16(a, b); }

/* --------------------------------------------------------- multipliers */

/* chunk.h:183-194 */
void vds_oracle_multipliers16(uint16_t k, uint16_t n, uint16_t *out)
{
    ensure_tables();
    uint16_t value = 1;
    for (uint16_t i = 0; i < k; ++i) {
        out[i] = value;
        value = mul16(value, n);
    }
}

void vds_oracle_multipliers8(uint8_t k, uint8_t n, uint8_t *out)
{
    ensure_tables();
    uint8_t value = 1;
    for (uint8_t i = 0; i < k; ++i) {
        out[i] = value;
        value = mul8(value, n);
    }
}

/* ---------------------------------------------------------------- encode */

size_t vds_oracle_replica_size(unsigned cell_bytes, unsigned k, size_t size, int write_padding)
{
    /* chunk.h:248 expected_size + chunk.h:274 uint16 trailer */
    size_t stripe = (size_t)cell_bytes * k;
    size_t cells = (size + stripe - 1) / stripe;
    return cells * cell_bytes + (write_padding ? 2 : 0);
}

/* chunk.h:245-281 (cell_type = uint16_t) */
size_t vds_oracle_encode16(uint16_t k, uint16_t replica, const uint8_t *data, size_t size,
                           int write_padding, uint8_t *out)
{
    ensure_tables();
    uint16_t *mult = (uint16_t *)malloc(sizeof(uint16_t) * (k ? k : 1));
    vds_oracle_multipliers16(k, replica, mult);
    const size_t stripe = 2u * (size_t)k;
    size_t pos = 0;
    for (size_t i = 0; i < size; i += stripe) {
        uint16_t value = 0;
        for (uint16_t j = 0; j < k; ++j) {
            uint16_t item = 0;
            for (size_t off = 0; off < 2; ++off) {
                item = (uint16_t)(item << 8);
                if (i + 2u * j + off < size) item |= data[i + 2u * j + off];
            }
            value ^= mul16(mult[j], item);
        }
        out[pos++] = (uint8_t)(value >> 8); /* binary_serialize.cpp:18-22 */
        out[pos++] = (uint8_t)(value & 0xFF);
    }
    if (write_padding) {
        uint16_t pad = (uint16_t)(size % stripe); /* chunk.h:274 */
        out[pos++] = (uint8_t)(pad >> 8);
        out[pos++] = (uint8_t)(pad & 0xFF);
    }
    free(mult);
    return pos;
}

/* chunk.h:245-281 (cell_type = uint8_t): one byte per cell, uint16 trailer */
size_t vds_oracle_encode8(uint8_t k, uint8_t replica, const uint8_t *data, size_t size,
                          int write_padding, uint8_t *out)
{
    ensure_tables();
    uint8_t mult[256];
    vds_oracle_multipliers8(k, replica, mult);
    const size_t stripe = k;
    size_t pos = 0;
    for (size_t i = 0; i < size; i += stripe) {
        uint8_t value = 0;
        for (uint8_t j = 0; j < k; ++j) {
            uint8_t item = (i + j < size) ? data[i + j] : 0;
            value ^= mul8(mult[j], item);
        }
        out[pos++] = value;
    }
    if (write_padding) {
        uint16_t pad = (uint16_t)(size % stripe);
        out[pos++] = (uint8_t)(pad >> 8);
        out[pos++] = (uint8_t)(pad & 0xFF);
    }
    return pos;
}

/* --------------------------------------------------------------- inverse */

/* chunk.h:290-375, written once for both cell widths through macros so the
 * two instantiations stay textually identical to the reference's template. */
#define DEFINE_INVERSE(NAME, CELL, MUL, DIV, MULTS)                                       \
    int NAME(CELL k, const CELL *nodes, CELL *M)                                          \
    {                                                                                     \
        ensure_tables();                                                                  \
        size_t kk = (size_t)k;                                                            \
        CELL *left = (CELL *)malloc(sizeof(CELL) * (kk * kk ? kk * kk : 1));              \
        for (size_t i = 0; i < kk; ++i) { /* prepare, chunk.h:296-306 */                 \
            MULTS(k, nodes[i], left + kk * i);                                            \
            for (size_t j = 0; j < kk; ++j) M[kk * i + j] = (CELL)(i == j ? 1 : 0);       \
        }                                                                                 \
        for (size_t i = 0; i < kk; ++i) { /* first, chunk.h:308-329 */                   \
            CELL m1 = left[kk * i + i];                                                   \
            for (size_t j = i + 1; j < kk; ++j) {                                         \
                CELL m2 = left[kk * j + i];                                               \
                for (size_t c = 0; c < kk; ++c) {                                         \
                    left[kk * j + c] = (CELL)(MUL(m1, left[kk * j + c]) ^ MUL(m2, left[kk * i + c])); \
                    M[kk * j + c] = (CELL)(MUL(m1, M[kk * j + c]) ^ MUL(m2, M[kk * i + c]));          \
                }                                                                         \
            }                                                                             \
        }                                                                                 \
        for (size_t i = 0; i < kk; ++i) { /* normalise, chunk.h:331-345 */               \
            CELL m1 = left[kk * i + i];                                                   \
            for (size_t c = 0; c < kk; ++c) {                                             \
                if (c >= i) left[kk * i + c] = DIV(left[kk * i + c], m1);                 \
                M[kk * i + c] = DIV(M[kk * i + c], m1);                                   \
            }                                                                             \
        }                                                                                 \
        for (size_t i = kk; i > 0; --i) { /* reverse, chunk.h:347-360 */                 \
            for (size_t j = i - 1; j > 0; --j) {                                          \
                CELL m1 = left[kk * (j - 1) + (i - 1)];                                   \
                for (size_t c = 0; c < kk; ++c) {                                         \
                    left[kk * (j - 1) + c] ^= MUL(left[kk * (i - 1) + c], m1);            \
                    M[kk * (j - 1) + c] ^= MUL(M[kk * (i - 1) + c], m1);                  \
                }                                                                         \
            }                                                                             \
        }                                                                                 \
        int ok = 0; /* validate, chunk.h:362-373 */                                       \
        for (size_t i = 0; i < kk; ++i)                                                   \
            for (size_t c = 0; c < kk; ++c)                                               \
                if (left[kk * i + c] != (CELL)(i == c ? 1 : 0)) ok = -1;                  \
        free(left);                                                                       \
        return ok;                                                                        \
    }

DEFINE_INVERSE(vds_oracle_inverse16, uint16_t, mul16, div16, vds_oracle_multipliers16)
DEFINE_INVERSE(vds_oracle_inverse8, uint8_t, mul8, div8, vds_oracle_multipliers8)

/* --------------------------------------------------------------- restore */

/* chunk.h:402-444 (cell_type = uint16_t) */
size_t vds_oracle_restore16(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                            size_t size, uint8_t *out)
{
    ensure_tables();
    if (k == 0 || size < 2) return (size_t)-1; /* reference: UB (reads data()[size-2]) */
    size_t kk = k;
    uint16_t *M = (uint16_t *)malloc(sizeof(uint16_t) * kk * kk);
    vds_oracle_inverse16(k, nodes, M);
    uint16_t padding = (uint16_t)((chunks[0][size - 2] << 8) | chunks[0][size - 1]);
    size_t expected = (size - 2) * kk;
    if (padding != 0) {
        expected -= kk * 2;
        expected += padding;
    }
    size_t produced = 0;
    size_t result = (size_t)-1;
    for (size_t index = 0; index < size && result == (size_t)-1; index += 2) {
        const uint16_t *m = M;
        for (size_t i = 0; i < kk; ++i) {
            uint16_t value = 0;
            for (size_t j = 0; j < kk; ++j) {
                uint16_t cell = (uint16_t)((chunks[j][index] << 8) | chunks[j][index + 1]);
                value ^= mul16(*m++, cell);
            }
            /* s << value, then "if (s.size() >= expected_size) return" */
            if (produced < expected) out[produced] = (uint8_t)(value >> 8);
            if (produced + 1 < expected) out[produced + 1] = (uint8_t)(value & 0xFF);
            produced += 2;
            if (produced >= expected) { result = expected; break; }
        }
    }
    free(M);
    return result;
}

/* chunk.h:402-444 (cell_type = uint8_t) */
size_t vds_oracle_restore8(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                           size_t size, uint8_t *out)
{
    ensure_tables();
    if (k == 0 || size < 2) return (size_t)-1;
    size_t kk = k;
    uint8_t *M = (uint8_t *)malloc(kk * kk);
    vds_oracle_inverse8(k, nodes, M);
    uint16_t padding = (uint16_t)((chunks[0][size - 2] << 8) | chunks[0][size - 1]);
    size_t expected = (size - 2) * kk;
    if (padding != 0) {
        expected -= kk;
        expected += padding;
    }
    size_t produced = 0;
    size_t result = (size_t)-1;
    for (size_t index = 0; index < size && result == (size_t)-1; index += 1) {
        const uint8_t *m = M;
        for (size_t i = 0; i < kk; ++i) {
            uint8_t value = 0;
            for (size_t j = 0; j < kk; ++j) value ^= mul8(*m++, chunks[j][index]);
            if (produced < expected) out[produced] = value;
            produced += 1;
            if (produced >= expected) { result = expected; break; }
        }
    }
    free(M);
    return result;
}

/* ------------------------------------------------------------ cell arrays */

/* chunk.h:206-224 */
size_t vds_oracle_chunk_cells16(uint16_t k, uint16_t n, const uint16_t *data, size_t len,
                                uint16_t *out)
{
    ensure_tables();
    uint16_t *mult = (uint16_t *)malloc(sizeof(uint16_t) * (k ? k : 1));
    vds_oracle_multipliers16(k, n, mult);
    size_t cells = 0;
    for (size_t i = 0; i < len; i += k) {
        uint16_t value = 0;
        for (uint16_t j = 0; j < k; ++j)
            if (i + j < len) value ^= mul16(mult[j], data[i + j]);
        out[cells++] = value;
    }
    free(mult);
    return cells;
}

size_t vds_oracle_chunk_cells8(uint8_t k, uint8_t n, const uint8_t *data, size_t len, uint8_t *out)
{
    ensure_tables();
    uint8_t mult[256];
    vds_oracle_multipliers8(k, n, mult);
    size_t cells = 0;
    for (size_t i = 0; i < len; i += k) {
        uint8_t value = 0;
        for (uint8_t j = 0; j < k; ++j)
            if (i + j < len) value ^= mul8(mult[j], data[i + j]);
        out[cells++] = value;
    }
    return cells;
}

/* chunk.h:383-400 */
void vds_oracle_restore_cells16(uint16_t k, const uint16_t *nodes, const uint16_t *const *chunks,
                                size_t cells, uint16_t *out)
{
    size_t kk = k;
    uint16_t *M = (uint16_t *)malloc(sizeof(uint16_t) * (kk * kk ? kk * kk : 1));
    vds_oracle_inverse16(k, nodes, M);
    size_t pos = 0;
    for (size_t index = 0; index < cells; ++index) {
        const uint16_t *m = M;
        for (size_t i = 0; i < kk; ++i) {
            uint16_t value = 0;
            for (size_t j = 0; j < kk; ++j) value ^= mul16(*m++, chunks[j][index]);
            out[pos++] = value;
        }
    }
    free(M);
}

void vds_oracle_restore_cells8(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                               size_t cells, uint8_t *out)
{
    size_t kk = k;
    uint8_t *M = (uint8_t *)malloc(kk * kk ? kk * kk : 1);
    vds_oracle_inverse8(k, nodes, M);
    size_t pos = 0;
    for (size_t index = 0; index < cells; ++index) {
        const uint8_t *m = M;
        for (size_t i = 0; i < kk; ++i) {
            uint8_t value = 0;
            for (size_t j = 0; j < kk; ++j) value ^= mul8(*m++, chunks[j][index]);
            out[pos++] = value;
        }
    }
    free(M);
}

/* --------------------------------------------------------------- inputs */

void vds_oracle_gf16_mul_n(const uint16_t *a, const uint16_t *b, uint16_t *out, size_t n)
{
    ensure_tables();
    for (size_t i = 0; i < n; ++i) out[i] = mul16(a[i], b[i]);
}

void vds_oracle_gf16_div_n(const uint16_t *a, const uint16_t *b, uint16_t *out, size_t n)
{
    ensure_tables();
    for (size_t i = 0; i < n; ++i) out[i] = div16(a[i], b[i]);
}

void vds_oracle_gf8_mul_n(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n)
{
    ensure_tables();
    for (size_t i = 0; i < n; ++i) out[i] = mul8(a[i], b[i]);
}

void vds_oracle_gf8_div_n(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n)
{
    ensure_tables();
    for (size_t i = 0; i < n; ++i) out[i] = div8(a[i], b[i]);
}

void vds_oracle_splitmix_fill(uint64_t seed, uint8_t *out, size_t size)
{
    uint64_t state = seed;
    size_t i = 0;
    while (i < size) {
        uint64_t z = (state += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int b = 0; b < 8 && i < size; ++b, ++i) out[i] = (uint8_t)(z >> (8 * b));
    }
}
