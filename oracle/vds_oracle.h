/*
 * vds_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of lboss75/vds kernel/vds_data (gf.h + chunk.h), used as
 * the parity checker for the HIP product path and as the "port" CPU
 * baseline in bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product (vds_amd/, libvds_ec)
 * never links or calls it.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - GF tables/products: compared entry-for-entry against the reference's own
 *     kernel/vds_data/gf.h compiled unmodified (oracle/_ref/gf_ref, built by
 *     oracle/Makefile from /root/reference where it lies).
 *   - Encode bytes / inverse rows: the known-answer vectors recorded from the
 *     reference build in SURVEY.md section 8(c) (tests/golden/survey_kats.json).
 *   - gf_tests.test_mul GF(2^3) table (tests/test_vds_data/gf_tests.cpp:9-38).
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef VDS_ORACLE_H_
#define VDS_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gf.h:42-67 -- bit-serial GF(2^m) multiply, polynomial given as the low
 * m bits of the reduction polynomial (gf.h:100-126: m=3 -> 0x0B incl. x^3,
 * m=8 -> 0x1D, m=16 -> 0x100B). */
uint32_t vds_oracle_gf_mul_bitserial(unsigned m, uint32_t poly_low, uint32_t a, uint32_t b);

/* gf.h:135-154 / gf.h:197-216 -- build the log/antilog tables.
 * value2log/log2value must hold 256 (gf8) or 65536 (gf16) entries. */
void vds_oracle_gf8_tables(uint8_t *value2log, uint8_t *log2value);
void vds_oracle_gf16_tables(uint16_t *value2log, uint16_t *log2value);

/* gf.h:156-179 and gf.h:218-241 (mul/div through the tables; div(x,0)=0). */
uint8_t vds_oracle_gf8_mul(uint8_t a, uint8_t b);
uint8_t vds_oracle_gf8_div(uint8_t a, uint8_t b);
uint16_t vds_oracle_gf16_mul(uint16_t a, uint16_t b);
uint16_t vds_oracle_gf16_div(uint16_t a, uint16_t b);

/* Bulk forms of the above (element-wise), for the table-pinning tests. */
void vds_oracle_gf16_mul_n(const uint16_t *a, const uint16_t *b, uint16_t *out, size_t n);
void vds_oracle_gf16_div_n(const uint16_t *a, const uint16_t *b, uint16_t *out, size_t n);
void vds_oracle_gf8_mul_n(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n);
void vds_oracle_gf8_div_n(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n);

/* chunk.h:183-194 -- multipliers[j] = n^j, j < k, with n^0 = 1. */
void vds_oracle_multipliers16(uint16_t k, uint16_t n, uint16_t *out);
void vds_oracle_multipliers8(uint8_t k, uint8_t n, uint8_t *out);

/* Replica size produced by chunk_generator<cell>::write (chunk.h:248,274). */
size_t vds_oracle_replica_size(unsigned cell_bytes, unsigned k, size_t size, int write_padding);

/* chunk.h:245-281 -- encode ONE replica (byte API, BE cells, optional trailer).
 * out must hold vds_oracle_replica_size(...) bytes.  Returns bytes written. */
size_t vds_oracle_encode16(uint16_t k, uint16_t replica, const uint8_t *data, size_t size,
                           int write_padding, uint8_t *out);
size_t vds_oracle_encode8(uint8_t k, uint8_t replica, const uint8_t *data, size_t size,
                          int write_padding, uint8_t *out);

/* chunk.h:290-375 -- the reference's cross-multiplied Gauss-Jordan (no
 * pivoting) inverse of V[i][c] = n_i^c.  out: k*k row-major. Returns 0 when
 * the validation block (chunk.h:362-373) would pass, -1 otherwise (the
 * reference only asserts there; the matrix is still written). */
int vds_oracle_inverse16(uint16_t k, const uint16_t *nodes, uint16_t *out);
int vds_oracle_inverse8(uint8_t k, const uint8_t *nodes, uint8_t *out);

/* chunk.h:402-444 -- decode bytes from k replicas (byte API).
 * chunks[j] pairs with nodes[j]; every chunk has chunk_size bytes.
 * out must hold chunk_size*k bytes (all the reference's loop can produce
 * before giving up).  Returns the restored size, or
 * (size_t)-1 for the reference's "Fatal error at chunk_restore::restore". */
size_t vds_oracle_restore16(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                            size_t chunk_size, uint8_t *out);
size_t vds_oracle_restore8(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                           size_t chunk_size, uint8_t *out);

/* chunk.h:206-224 -- cell-array encode (test path; native cells, no trailer).
 * out holds ceil(len/k) cells.  Returns the cell count. */
size_t vds_oracle_chunk_cells16(uint16_t k, uint16_t n, const uint16_t *data, size_t len,
                                uint16_t *out);
size_t vds_oracle_chunk_cells8(uint8_t k, uint8_t n, const uint8_t *data, size_t len, uint8_t *out);

/* chunk.h:383-400 -- cell-array restore; out holds cells*k cells. */
void vds_oracle_restore_cells16(uint16_t k, const uint16_t *nodes, const uint16_t *const *chunks,
                                size_t cells, uint16_t *out);
void vds_oracle_restore_cells8(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                               size_t cells, uint8_t *out);

/* Deterministic input generator shared with the GPU path and the golden
 * fixtures: splitmix64 seeded with `seed`, successive
 * outputs written little-endian. */
void vds_oracle_splitmix_fill(uint64_t seed, uint8_t *out, size_t size);

#ifdef __cplusplus
}
#endif

#endif /* VDS_ORACLE_H_ */
