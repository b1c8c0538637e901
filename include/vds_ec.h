/*
 * vds_ec.h -- C ABI of the MI355X-native object-chunk erasure codec.
 *
 * This is the boundary that replaces the CPU arithmetic of lboss75/vds
 * kernel/vds_data (chunk.h, gf.h, chunk_storage.cpp).  The reference's codec
 * is header-only C++ templates; the drop-in headers in vds_amd/include/vds_data/
 * keep that exact template API and forward the uint8_t / uint16_t
 * instantiations to the entry points below (see INTEGRATION.md for the
 * binding).  Plain pointers, sizes and int status codes only.
 *
 * Terminology (reference): an object of S bytes is cut into stripes of
 * k cells; a "replica" (horcrux) with id r holds, per stripe, the evaluation
 * at r of the polynomial whose coefficients are the stripe's cells
 * (chunk.h:245-281), followed by a 2-byte big-endian trailer S mod (k*cell).
 * Any k distinct replicas restore the object (chunk.h:290-444).
 *
 * Memory: *_device entry points take device pointers and enqueue work on the
 * given hipStream_t (NULL = the current device's null stream) without
 * synchronising; parameters too large for the kernel arguments (k > 32
 * inverses, k > 64 chunk tables) are staged stream-ordered through a pinned
 * ring (growing it, on first use of a larger size, allocates).  *_host entry points take host pointers, stage through
 * pinned buffers on the current device and return when the result is in host
 * memory.  Every entry point fails with VDS_EC_ENODEV if no GPU is usable --
 * there is no CPU fallback.
 */
#ifndef VDS_EC_H_
#define VDS_EC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ----------------------------------------------------------- status codes */
#define VDS_EC_OK 0
#define VDS_EC_EINVAL (-1)    /* bad argument (k == 0, null pointer, size)     */
#define VDS_EC_ENODEV (-2)    /* no usable GPU / HIP runtime error at init    */
#define VDS_EC_ENOMEM (-3)    /* device or pinned allocation failed           */
#define VDS_EC_ESINGULAR (-4) /* replica ids not distinct: V not invertible   */
#define VDS_EC_ERESTORE (-5)  /* "Fatal error at chunk_restore::restore"      */
#define VDS_EC_EHIP (-6)      /* HIP runtime error during a launch / copy     */
/* base64::to_bytes failures (encoding.cpp:181-247), by the reference's text: */
#define VDS_EC_EB64_LENGTH (-7)  /* "Non-Valid base64!" (length % 4 != 0)      */
#define VDS_EC_EB64_PADDING (-8) /* "Invalid Padding in Base 64!"              */
#define VDS_EC_EB64_CHAR (-9)    /* "Non-Valid Character in Base 64!"          */

/* ----------------------------------------------------------------- flags */
/* write_padding = false in chunk_generator::write (chunk.h:79,273-278):
 * no trailer; the caller guarantees size % (k*cell) == 0.                  */
#define VDS_EC_F_NO_TRAILER 0x1u
/* Cell-array form (test path, chunk.h:206-224 and chunk.h:383-400): data is
 * an array of native-endian cells, no trailer, restore is not trimmed.     */
#define VDS_EC_F_CELLS 0x2u

#define VDS_EC_MAX_K 65535u

const char *vds_ec_strerror(int status);
int vds_ec_version(void);
/* Host staging contexts (pinned + device buffers and a stream per calling
 * thread and device) created so far, and how many of them sit idle in the
 * pool that exited threads return theirs to (diagnostics; host only).      */
int vds_ec_host_ctx_stats(uint64_t *created, uint64_t *pooled);
/* Number of HIP devices usable by the library (0 on a machine with none). */
int vds_ec_device_count(int *count);

/* Bytes chunk_generator<cell>::write appends for one replica
 * (chunk.h:248 expected_size + chunk.h:274 trailer).  cell_bytes = 1 | 2. */
uint64_t vds_ec_replica_size(unsigned cell_bytes, unsigned k, uint64_t size, unsigned flags);
/* Bytes chunk_restore<cell>::restore returns for replicas of replica_size
 * bytes with trailer `padding` (chunk.h:415-419).                           */
uint64_t vds_ec_restored_size(unsigned cell_bytes, unsigned k, uint64_t replica_size, uint16_t padding);

/* ---------------------------------------------------- field / matrix helpers
 * Replace gf_math<uint16_t>() / gf_math<uint8_t>() (gf.h:131-253),
 * chunk<cell>::generate_multipliers (chunk.h:183-194) and the
 * chunk_restore<cell> constructor (chunk.h:290-375).  Host-only, no GPU.   */
int vds_ec_gf16_tables(uint16_t *value2log, uint16_t *log2value); /* 65536 each */
int vds_ec_gf8_tables(uint8_t *value2log, uint8_t *log2value);    /* 256 each   */
int vds_ec_multipliers16(uint16_t k, uint16_t node, uint16_t *out);
int vds_ec_multipliers8(uint8_t k, uint8_t node, uint8_t *out);
/* out = V^{-1} (k*k, row-major) for V[i][c] = nodes[i]^c.  Returns
 * VDS_EC_ESINGULAR when two nodes coincide (the reference computes garbage
 * there: its validation is vds_assert, compiled out).        */
int vds_ec_inverse16(uint16_t k, const uint16_t *nodes, uint16_t *out);
int vds_ec_inverse8(uint8_t k, const uint8_t *nodes, uint8_t *out);

/* -------------------------------------------------------- device entry points
 * Encode `count` objects of `size` bytes each: object o at in + o*in_stride.
 * For each of the n replica ids, replica r_i of object o is written at
 * outs[i] + o*out_stride (outs is a HOST array of n device pointers) and
 * occupies vds_ec_replica_size(...) bytes.  Replaces n calls of
 * chunk_generator<uint16_t>(k, r_i).write(s, data, size) per object
 * (chunk.h:245-281; caller loops dht_network_client.cpp:75-77, :589-591).  */
int vds_ec_encode16_device(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in,
                           uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                           uint64_t out_stride, unsigned flags, void *stream);
int vds_ec_encode8_device(uint8_t k, const uint8_t *replicas, uint32_t n, const uint8_t *in,
                          uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                          uint64_t out_stride, unsigned flags, void *stream);

/* Restore `count` objects from k replicas each: replica j (id nodes[j]) of
 * object o at chunks[j] + o*chunk_stride (chunks: HOST array of k device
 * pointers), chunk_size bytes each (trailer included).  The restored object
 * o is written at out + o*out_stride; its size (identical for all objects,
 * taken from the trailer of object 0's first chunk ON THE HOST -- so the
 * caller passes it in `padding`) is vds_ec_restored_size(...).  Replaces
 * chunk_restore<uint16_t>(k, nodes).restore(chunks) (chunk.h:290-444;
 * caller dht_network_client.cpp:887-888).                                   */
int vds_ec_restore16_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                            uint64_t chunk_size, uint64_t chunk_stride, uint16_t padding,
                            uint32_t count, uint8_t *out, uint64_t out_stride, unsigned flags,
                            void *stream);
int vds_ec_restore8_device(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                           uint64_t chunk_size, uint64_t chunk_stride, uint16_t padding,
                           uint32_t count, uint8_t *out, uint64_t out_stride, unsigned flags,
                           void *stream);

/* Regenerate lost replicas from k survivors without materialising the object
 * (SURVEY.md 8(f) row 3).  The reference's repair restores the object and
 * re-encodes it (sync_process.cpp:313-335 -> restore_async + save_data,
 * dht_network_client.cpp:582-658); replica t is P(t) stripe by stripe, so one
 * pass over the survivors yields it directly.  Survivor j (id nodes[j]) of
 * object o at chunks[j] + o*chunk_stride (HOST array of k device pointers,
 * chunk_size bytes = cells + BE16 trailer); replica targets[i] of object o is
 * written to outs[i] + o*out_stride (chunk_size bytes, trailer included).
 * Bytes equal chunk_generator(k, t).write(restore(...)) -- the reference's
 * route, restored object trimmed to E bytes, last stripe zero-padded, trailer
 * E mod 2k -- for ANY survivors, codeword or not, whose first chunk's trailer
 * p is at most 2k.  For p > 2k that route has no chunk_size-byte answer (it
 * fails, or re-encodes to chunk_size + 2 bytes): the *_host forms return
 * VDS_EC_ERESTORE, the device forms leave those objects' replicas unspecified. */
int vds_ec_regenerate16_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                               uint64_t chunk_stride, uint32_t count, const uint16_t *targets, uint32_t ntargets,
                               uint8_t *const *outs, uint64_t out_stride, void *stream);

/* Batched restore / regenerate with a survivor set, size and output PER
 * OBJECT -- the shape of the download and repair loops (restore_async takes
 * the first k replicas found for each object, dht_network_client.cpp:851-901;
 * sync_process repairs object by object, sync_process.cpp:313-335).  Object
 * o's survivor j (replica id nodes[o*k + j]) is at chunks[o*k + j] (HOST
 * array of count*k device pointers), chunk_sizes[o] bytes (trailer included);
 * paddings[o] is its trailer value (the caller has it: the chunks came from
 * files or sockets).  Restore writes vds_ec_restored_size(2, k,
 * chunk_sizes[o], paddings[o]) bytes to outs[o].  Regenerate writes replica
 * targets[o*nt + i] (chunk_sizes[o] bytes, trailer included) to
 * outs[o*nt + i].  Objects whose survivors lie within the syndrome kernel's
 * points (k in {16, 32}, ids < k + k/4) share ONE launch, those with other
 * ids below 256 (same k) one runtime-coefficient launch; the rest take one
 * launch each.  Every object is validated before anything is enqueued
 * (pointers, lengths, distinct ids: VDS_EC_ESINGULAR otherwise); nothing
 * synchronises.  count < 2^30 (VDS_EC_EINVAL otherwise).  Regenerate bytes as
 * vds_ec_regenerate16_device.                                                 */
int vds_ec_restore16_batch_device(uint16_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                                  const uint64_t *chunk_sizes, const uint16_t *paddings, uint8_t *const *outs,
                                  unsigned flags, void *stream);
int vds_ec_regenerate16_batch_device(uint16_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                                     const uint64_t *chunk_sizes, uint32_t ntargets, const uint16_t *targets,
                                     uint8_t *const *outs, void *stream);

/* ---------------------------------------------------------- host entry points
 * Same operations on host memory (pinned staging, H2D -> kernel -> D2H on
 * the calling thread's current device).  outs: n host buffers of
 * vds_ec_replica_size(...) bytes.  This is what chunk_generator::write and
 * chunk_storage::generate_replica (chunk_storage.cpp:41-60) call.            */
int vds_ec_encode16_host(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data,
                         uint64_t size, uint8_t *const *outs, unsigned flags);
int vds_ec_encode8_host(uint8_t k, const uint8_t *replicas, uint32_t n, const uint8_t *data,
                        uint64_t size, uint8_t *const *outs, unsigned flags);
/* chunks: k host buffers of chunk_size bytes; out must hold chunk_size*k
 * bytes (the most the reference's loop can produce: (chunk_size-2)*k for a
 * well-formed trailer, more when the trailer is corrupt); *out_size
 * receives the restored length (chunk.h:402-444, chunk_storage.cpp:62-86). */
int vds_ec_restore16_host(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                          uint64_t chunk_size, uint8_t *out, uint64_t *out_size, unsigned flags);
int vds_ec_restore8_host(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                         uint64_t chunk_size, uint8_t *out, uint64_t *out_size, unsigned flags);

/* Host-memory form of vds_ec_regenerate16_device: chunks are k host buffers
 * of chunk_size bytes, outs ntargets host buffers of chunk_size bytes.      */
int vds_ec_regenerate16_host(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                             const uint16_t *targets, uint32_t ntargets, uint8_t *const *outs);

/* Batched host-memory encode across every visible GPU (one host thread,
 * pinned ring and stream pair per device; object o -> device o % devices).
 * objs[o] has sizes[o] bytes; replica i of object o goes to outs[o*n + i].
 * This is the save_temp / save_data formulation.    */
int vds_ec_encode16_host_batch(uint16_t k, const uint16_t *replicas, uint32_t n,
                               const uint8_t *const *objs, const uint64_t *sizes, uint32_t count,
                               uint8_t *const *outs, unsigned flags, int max_devices);

/* Batched host-memory restore across every visible GPU (the restore side of
 * the batch above; chunk_storage::restore_data, chunk_storage.cpp:62-85, per
 * object).  Object o is restored from the k host chunks chunks[o*k + j] of
 * chunk_sizes[o] bytes holding replicas nodes[o*k + j]; on entry out_sizes[o]
 * is the capacity of outs[o], on success the restored length (trailer-trimmed
 * as vds_ec_restore16_host).  Every object is validated before any transfer. */
int vds_ec_restore16_host_batch(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                                const uint64_t *chunk_sizes, uint32_t count, uint8_t *const *outs, uint64_t *out_sizes,
                                unsigned flags, int max_devices);

/* Caller-owned pinned memory for the host batches (the
 * path starts and ends in host memory).  vds_ec_host_alloc returns
 * page-locked, device-mapped memory usable from every device;
 * vds_ec_host_register pins (and maps) a caller's existing range for as long
 * as it stays registered.  When a host batch group's objects -- or replicas,
 * survivors, restored objects -- lie back to back in one such range (the
 * slab layouts: objects [count][size], replicas [count][n][L], survivors
 * [count][k][chunk_size], restored objects [count][E]), the H2D DMA reads the
 * caller's bytes and the results are written into the caller's pages by the
 * device: no staging copies in host memory.  Anything else is staged as
 * before.  Free / unregister only when no call using the range is running. */
int vds_ec_host_alloc(uint64_t bytes, void **ptr);
int vds_ec_host_free(void *ptr);
int vds_ec_host_register(void *ptr, uint64_t bytes);
int vds_ec_host_unregister(void *ptr);

/* ---------------------------------------------------- stripe-range split
 * One object split by stripe range [t0, t1), e.g. over GPUs.
 * Cell t of every replica depends on stripe t alone, so the ranges are
 * independent.  encode: in = the whole object (device, size bytes); writes
 * replica bytes [2 t0, 2 t1) of outs[i] (whole replica buffers), and the
 * trailer with the range that ends at T = ceil(size / 2k).  t0 < t1 <= T
 * (T == 0: the range [0, 0), trailer only).  restore: chunks = the whole
 * survivor buffers, padding = their trailer value; writes object bytes
 * [2k t0, min(2k t1, E)) of out for t1 <= ceil(E / 2k) (E =
 * vds_ec_restored_size).  Byte API only (no VDS_EC_F_CELLS).                */
int vds_ec_encode16_range_device(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in, uint64_t size,
                                 uint64_t t0, uint64_t t1, uint8_t *const *outs, unsigned flags, void *stream);
int vds_ec_restore16_range_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                                  uint16_t padding, uint64_t t0, uint64_t t1, uint8_t *out, unsigned flags,
                                  void *stream);
/* One host object over several GPUs: its stripes in `parts` ranges of whole
 * 2048-stripe tiles (0 = one per device), range r on device r % devices, each
 * with its own PCIe link.  Same arguments and results as
 * vds_ec_encode16_host / vds_ec_restore16_host (out_size: capacity in,
 * restored length out).                                                     */
int vds_ec_encode16_host_split(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                               uint8_t *const *outs, unsigned flags, int max_devices, uint32_t parts);
int vds_ec_restore16_host_split(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                                uint8_t *out, uint64_t *out_size, unsigned flags, int max_devices, uint32_t parts);

/* ---------------------------------------------------------- replica names
 * The reference names each replica by SHA-256 of its bytes (save_temp /
 * save_data: dht_network_client.cpp:79, :593 -> hash::signature(sha256),
 * kernel/vds_crypto/hash.cpp:91-101, OpenSSL EVP_sha256).  Digests of count
 * device messages of len bytes at base + j*stride (any alignment) go to
 * digests + 32*j (device memory).                                             */
int vds_ec_sha256_device(const uint8_t *base, uint64_t len, uint64_t stride, uint32_t count, uint8_t *digests,
                         void *stream);
/* SHA-256 of ONE host message on the calling thread (no GPU): upload_data's
 * body hash (server_api.cpp:16) is a single chain of dependent compressions,
 * ~3 us a block in one GPU lane, so vds_ec_save_temp16_host computes it here
 * while the device encodes and names the replicas.  x86 SHA extensions when
 * the CPU has them, else portable code (FIPS 180-4 6.2).                     */
int vds_ec_sha256_host(const uint8_t *data, uint64_t len, uint8_t *digest);
/* vds_ec_encode16_host plus the SHA-256 of every replica, computed on the
 * device before the copy-back: digests receives n*32 bytes (host).          */
int vds_ec_encode16_hash_host(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                              uint8_t *const *outs, uint8_t *digests, unsigned flags);

/* Content-addressed storage path of a replica from its SHA-256 name (host,
 * no GPU): base64 (standard alphabet, '=' padding, encoding.cpp:136-174) with
 * '+' -> '#' and '/' -> '_', split as chars [0,10) "/" [10,20) "/" [20,44)
 * (dht_network_client.cpp:483-505, :632-653).  out receives count
 * NUL-terminated paths of VDS_EC_PATH_BYTES bytes each.                     */
#define VDS_EC_PATH_BYTES 48
int vds_ec_replica_paths(const uint8_t *digests, uint32_t count, char *out);

/* ------------------------------------------- upload path
 * The live upload: websocket "upload" with a base64 body
 * (websocket_api.cpp:141-155) -> server_api::upload_data (server_api.cpp:12-30:
 * data hash = SHA-256 of the body) -> _client::save_temp
 * (dht_network_client.cpp:62-107: replicas 0..n-1 written, each named by its
 * SHA-256 and kept as <root>/tmp/<tmp name>) -> the JSON answer
 * (websocket_api.cpp:467-485).  Host code except vds_ec_save_temp16_host,
 * which runs the encode and every hash on the current device.              */
/* base64::to_bytes with its quirks (see vds_ec_wire.cpp); *out_len receives
 * vds_ec_base64_decoded_size(in, len) bytes written to out.                 */
size_t vds_ec_base64_decoded_size(const char *in, size_t len);
int vds_ec_base64_decode(const char *in, size_t len, uint8_t *out, size_t *out_len);
/* base64::from_bytes; out == NULL queries the length (excluding the NUL). */
int vds_ec_base64_encode(const uint8_t *in, size_t len, char *out, size_t cap, size_t *out_len);
/* save_temp's tmp-file names: base64 of each digest with '+' -> '#' and
 * '/' -> '_' (dht_network_client.cpp:91-95), NUL-terminated, 45 bytes each. */
#define VDS_EC_NAME_BYTES 45
int vds_ec_tmp_names(const uint8_t *digests, uint32_t count, char *out);
/* The "upload" answer {"id":..,"result":{"replicas":[..],"hash":..,
 * "replica_size":..}} exactly as json_writer serialises it; out == NULL
 * queries the length (excluding the NUL).                                   */
int vds_ec_upload_response_json(int id, const uint8_t *replica_digests, uint32_t n, const uint8_t *data_digest,
                                 uint32_t replica_size, char *out, size_t cap, size_t *out_len);
/* save_temp + upload_data's hashing: replicas 0..n-1 of the body (host,
 * size bytes) into outs (n host buffers of vds_ec_replica_size bytes), their
 * SHA-256 names into replica_digests (n*32 host bytes) -- encode and names on
 * the device --, the body's SHA-256 into data_digest (32 host bytes),
 * computed on the calling thread meanwhile (vds_ec_sha256_host).            */
int vds_ec_save_temp16_host(uint16_t k, uint32_t n, const uint8_t *data, uint64_t size, uint8_t *const *outs,
                            uint8_t *replica_digests, uint8_t *data_digest, uint32_t *replica_size);

/* ----------------------------------------------------------------- utilities */
/* Fill `size` device bytes at dst with the splitmix64 stream of `seed`
 * (little-endian 8-byte words) -- the synthetic-object generator used by
 * bench.py and the parity tests (SURVEY.md 8(c) "Input PRNG").               */
int vds_ec_fill_splitmix_device(uint8_t *dst, uint64_t size, uint64_t seed, void *stream);

/* Which kernel path a device call with these parameters takes: 4 = the
 * survivor set's own run-time compiled kernel (vds_ec_jit_*) for the full
 * tiles, 3 = syndrome
 * restore (erasure-pattern-independent XOR programs, survivors within
 * 0..k+k/4-1) for the full tiles, 2 = bit-sliced fast path for the full tiles
 * (+ generic tail; objects under one tile whose stripes are whole 512-stripe
 * groups ride it in batches), 1 = generic path only.  The restore query takes
 * the trailer's padding and the batch's object count, as
 * vds_ec_restore16_device does (restore planning is shared with it).
 * (A -DVDS_RESTORE_PATH_BS=1 build of the library disables path 3: A/B.)  */
int vds_ec_encode16_path(uint16_t k, const uint16_t *replicas, uint32_t n, uint64_t size);
int vds_ec_restore16_path(uint16_t k, const uint16_t *nodes, uint64_t chunk_size, uint16_t padding, uint32_t count);
/* 4 = the regenerate runs the survivor set's run-time compiled kernel
 * (vds_ec_jit_*), 3 = the regenerate rides the syndrome kernel (every target
 * an erased point of a compiled (k, n)) for the full tiles, 2 = the runtime-coefficient
 * bit-sliced kernel (k in {16, 32}, at most k targets, >= 512 full stripes),
 * 1 = generic path only.                                                    */
int vds_ec_regenerate16_path(uint16_t k, const uint16_t *nodes, const uint16_t *targets, uint32_t ntargets,
                             uint64_t chunk_size);

/* ------------------------------------------- run-time compiled restore kernels
 * A restore whose survivors are k distinct points of 0..k+k/4-1 (k in {16,
 * 32}) runs k_restore_syn: fixed syndrome programs plus a runtime recovery of
 * the erased points.  For each such survivor set a device restore meets, the
 * library also generates the set's own XOR programs (the erased points below
 * k as fixed combinations of the survivors) and, from the set's second use,
 * compiles that kernel in the background (hiprtc, gfx950); later restores of
 * the set use it.  Same bytes.  Mode (vds_ec_jit_set_mode, initially from
 * VDS_EC_JIT): 0 = off (VDS_EC_JIT=0), 1 = background (default), 2 = compile
 * on the calling thread at the first use (VDS_EC_JIT=sync).
 * No counterpart in the reference (its restore is a CPU loop, chunk.h:402-444).
 *
 * vds_ec_jit_wait:    block until no compile is queued or running.
 * vds_ec_jit_build16: compile the kernel of survivor set `nodes` and return
 *                     its code object size (no device needed; EINVAL for a set
 *                     the syndrome kernel does not serve, EHIP if hiprtc fails).
 * vds_ec_jit_ready16: 1 when that set's kernel is compiled, else 0.
 * vds_ec_jit_dump16:  compile the kernel of survivor set `nodes` (regen != 0:
 *                     its fused-regenerate kernel) and write its source and
 *                     code object as dir/jit_<k>_<n>_<mask>[_regen].{hip,co}
 *                     (inspection: register use, spills; no device needed).  */
int vds_ec_jit_set_mode(int mode);
int vds_ec_jit_wait(void);
int vds_ec_jit_build16(uint16_t k, const uint16_t *nodes, uint64_t *code_bytes);
int vds_ec_jit_ready16(uint16_t k, const uint16_t *nodes);
int vds_ec_jit_dump16(uint16_t k, const uint16_t *nodes, int regen, const char *dir);

#ifdef __cplusplus
}
#endif

#endif /* VDS_EC_H_ */
