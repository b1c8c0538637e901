// ec_internal.hpp -- launch interface between the C ABI (vds_ec_api.cpp) and
// the kernels (ec_generic.hip, ec_encode.hip, ec_restore_bs.hip, ec_restore_syn.hip).  Internal to libvds_ec.so.
#pragma once

#ifndef __HIPCC_RTC__  // (hiprtc sees the launch structs only: vds_ec_jit.cpp)
#include <hip/hip_runtime_api.h>
#endif

#include <cstdint>

namespace vds_ec {

constexpr int kMaxLaunchReplicas = 64;  // replicas per generic encode launch
constexpr int kMaxFastK = 32;
constexpr uint32_t kTileStripes = 2048;  // 64 lanes x 32 bit-sliced slots

struct GenericEncodeArgs {
  const uint8_t *in;
  uint64_t size;       // object bytes (cell arrays: bytes too)
  uint64_t in_stride;  // bytes between objects
  uint32_t count;      // objects
  uint32_t k;
  uint32_t cell_bytes; // 1 or 2
  uint32_t flags;
  uint32_t nrep;
  uint64_t t_begin;    // first stripe handled
  uint64_t t_count;    // stripes handled (the trailer is one extra index)
  uint64_t stripes;    // total stripes T of an object
  uint32_t write_trailer;
  uint64_t out_stride;
  uint16_t nodes[kMaxLaunchReplicas];
  uint8_t *outs[kMaxLaunchReplicas];
};

constexpr int kInlineChunks = 64;   // chunk pointers carried in the kernel arguments
constexpr int kInlineMatrixK = 32;  // k*k inverse carried in the kernel arguments

// Where chunk j lives (first match): chunk_pitch != 0 -> chunk_base + j*pitch
// (contiguous staging of the host path); chunk_table != nullptr -> device
// table; otherwise chunk_ptr[j] (k <= kInlineChunks).  The inverse is inline
// (two coefficients per dword) unless matrix_dev is set.  No stream-ordered
// allocations are involved, so a launch never depends on a freed table.
struct GenericRestoreArgs {
  const uint8_t *chunk_ptr[kInlineChunks];
  const uint8_t *chunk_base;
  uint64_t chunk_pitch;
  const uint8_t *const *chunk_table;
  const uint16_t *matrix_dev;
  uint32_t matrix_inline[kInlineMatrixK * kInlineMatrixK / 2];
  uint64_t chunk_stride;
  uint32_t count;
  uint32_t k;
  uint32_t cell_bytes;
  uint32_t flags;
  uint64_t t_begin;
  uint64_t t_count;
  uint8_t *out;
  uint64_t out_stride;
  uint64_t out_len;  // bytes of the restored object (trim bound)
};

// Bit-sliced encode: the full stripes of `count` objects, F = 128
// groups_per_obj per object, as one stream of 2048-stripe tiles (k >= 8:
// tiles may straddle objects; k = 4: groups_per_obj % 16 == 0).
struct FastEncodeArgs {
  const uint8_t *in;
  uint64_t in_stride;
  uint64_t out_stride;
  uint32_t groups_per_obj;
  uint32_t total_tiles;
  // 1: also write every replica's trailer -- zero, as the launch covers every
  // stripe of objects whose size is a multiple of 2k -- at cell T (k >= 8)
  uint32_t trailer0;
  uint8_t *outs[kMaxLaunchReplicas];  // outs[r] for replica id r = 0..N-1
};

// Bit-sliced runtime-coefficient restore over 512-stripe groups: the first
// groups_per_obj groups of every object as one stream of 4-group tiles.
struct FastRestoreArgs {
  const uint8_t *chunks[kMaxFastK];
  uint64_t chunk_stride;
  uint8_t *out;
  uint64_t out_stride;
  uint32_t groups_per_obj;
  uint32_t total_tiles;
  // k x k inverse, row-major, two coefficients per dword (low half = even
  // column) so the wave-uniform reads are scalar s_load_dword.
  uint32_t matrix2[kMaxFastK * kMaxFastK / 2];
  // regenerate mode (k_restore_bs<..., true>): output m < nt is replica
  // bytes (cells in stripe order) at regen[m] + o * out_stride, the matrix
  // rows are V_targets V_S^{-1} (rows nt.. zero)
  uint8_t *regen[kMaxFastK];
  uint32_t nt;
};

// Erasure-pattern-independent restore (k_restore_syn<K,N>): survivors are K
// distinct points of 0..N-1 (N - K == K / 4).  Syndromes and the fixed
// interpolation are compile-time XOR programs; only the M x M solve
// c_E = R * S (R = W_E^{-1}) is runtime.
struct SynRestoreArgs {
  const uint8_t *chunks[kMaxFastK];  // chunk j holds point point[j]
  uint8_t point[kMaxFastK];
  uint8_t erased[kMaxFastK / 4];     // the M erased points
  uint64_t chunk_stride;
  uint8_t *out;
  uint64_t out_stride;
  uint32_t tiles_per_obj;
  uint32_t total_tiles;
  // R = W_E^{-1} as bit selections: byte (b & 3) of solve_sel[i][b >> 2] has
  // bit j set iff bit b of R[i][j] is set (row i = erased[i], M <= 8)
  uint32_t solve_sel[kMaxFastK / 4][4];
  // regenerate mode (k_restore_syn<..., true>): the recovered point erased[w]
  // is written as replica bytes to regen[w] + o * regen_stride (nullptr: not
  // requested); the interpolation is skipped
  uint8_t *regen[kMaxFastK / 4];
  uint64_t regen_stride;
  // batch mode (launch_restore_syn_batch): everything per object from tables
  const struct SynBatchObj *objs;
  const struct SynBatchPlan *plans;
  const struct SynBatchTile *tiles;
};

constexpr int kInlineCoef = 512;  // regenerate coefficients carried in the kernel arguments

// Generic regenerate (any k, any targets): replica targets[i] of object o is
// sum_j coef[i][j] * chunk_j cell by cell (coef = V_targets V_S^{-1}, nt x k
// row-major), for cells [t_begin, t_begin + t_count), then the trailer (cell
// index T) copied from chunk 0 -- the bytes restore + re-encode would give
// (sync_process.cpp:313-335 -> chunk.h:402-444 then chunk.h:245-281).
struct RegenArgs {
  const uint8_t *chunk_ptr[kInlineChunks];
  const uint8_t *const *chunk_table;  // used when k > kInlineChunks
  uint64_t chunk_stride;
  const uint16_t *coef_dev;           // used when nt * k > kInlineCoef
  uint32_t coef_inline[kInlineCoef / 2];
  uint32_t count;
  uint32_t k;
  uint32_t cell_bytes;
  uint32_t nt;
  uint64_t t_begin;
  uint64_t t_count;
  uint64_t T;
  uint8_t *outs[kMaxLaunchReplicas];
  uint64_t out_stride;
};

// Batched k_restore_syn (per-object survivor sets, sizes and outputs; one
// launch over every tile of every object).  Device tables, built on the host:
// objs[o] per object (its survivors in its plan's point order), plans[p] per
// distinct erased set, tiles[t] per tile.  A tile is two halves of
// kHalfStripes stripes; each half is a stripe range of any object of the
// tile's plan, so small objects (the live 64 KiB ones: 1024 stripes at
// k = 32) pair up instead of filling half a tile each.
constexpr uint32_t kHalfStripes = kTileStripes / 2;
// Runtime-coefficient batch mode (k_restore_syn<..., RT>): survivor sets
// outside the syndrome kernel's points -- the live n = 64 shape losing more
// than k/4 of replicas 0..k+k/4-1, where restore_async's first k found reach
// ids past k+k/4-1 (dht_network_client.cpp:851-901).  Slot j < K of an object
// holds point j when that replica survives, else one of its survivors beyond
// point K-1 ("borrowed" slot: point j itself is erased).  Output row m is a
// combination of the K slots with the coefficients coef[m][0..K): restore:
// the value at the erased point epoint[m] < K (then the fixed interpolation
// from points 0..K-1 gives the object); regenerate: replica epoint[m].  The
// rows are Lagrange over the slots' points, computed on the device
// (launch_rt_coefs) from spoint / epoint.
struct SynBatchRt {
  // ne x K, row-major, slot order (device); coefficient c as the spread word
  // (c & 0xFF) | (c >> 8) << 16, the form the RT walk builds its masks from
  const uint32_t *coef;
  uint64_t borrowed;          // bit j: slot j holds a survivor beyond K-1
  uint32_t ne;                // rows
  uint32_t mode;              // restore, k = 32: 1 = RT2 rows (kRt2MaxRows, below), else 0
  uint8_t epoint[kMaxFastK];  // point of output row m
  uint8_t spoint[kMaxFastK];  // point held by slot j
};
// RT2 (restore, k = 32, every survivor below 2k, at most kRt2MaxRows erased
// points below k): with A the survivors below k, E the erased points and b_j
// the survivor borrowed into slot e_j, P = P0 + Z Q where P0 interpolates the
// values on U = {0..k-1} with zeros at E (so P0(b) is the PERM program's
// permuted sum), Z = prod_{a in A} (X + a) and deg Q < |E|.  Then
//   P(e_m) = sum_j c[m][j] r_j,  r_j = y_(b_j) + P0(b_j),
//   c[m][j] = Z(e_m) prod_{i != j} (e_m + b_i) / (Z(b_j) prod_{i != j} (b_j + b_i)):
// |E| fixed PERM evaluations and |E|^2 runtime products instead of RT's
// |E| k.  coef holds c (row m, column j < ne) in RT's spread form.
// (two groups of r_j through the free LDS slots K..K+7 of the k = 32 kernel;
// above ~12 rows the |E|^2 products cost more than RT's |E| k)
constexpr uint32_t kRt2MaxRows = 12;
struct SynBatchObj {
  const uint8_t *chunks[kMaxFastK];  // survivor j = the chunk of plan point j (K used); RT: of slot j
  uint8_t *out;                      // restore: the object's bytes
  uint8_t *regen[kMaxFastK / 4];     // regenerate: replica erased[w] (nullptr: not requested); RT: of row w
  uint64_t out_len;                  // restore: E bytes to write
  uint64_t chunk_len;                // L = 2 T + 2 bytes of every survivor (and regenerated replica)
  uint32_t plan;                     // its plan (the regenerate tail reads it)
  uint32_t first;                    // plan position (RT: slot) of the caller's chunk 0 (whose trailer restore reads)
  SynBatchRt rt;                     // RT mode only
};
// SMALL batch mode (small-M syndromes, restore_syn.hpp): the survivors lie in
// A = {0..K+MS-1} (MS <= kSmallMaxM), so the MS checks over A and an MS x MS
// solve give the erased points; the rows recovered are erased[0..nrec).
constexpr int kSmallMaxM = 2;
struct SynBatchPlan {
  uint8_t erased[kMaxFastK / 4];  // SMALL: A's MS erased points ascending, then the syndrome slots
  uint8_t point[kMaxFastK];       // the survivors' points, ascending
  union {
    uint32_t solve_sel[kMaxFastK / 4][4];  // as SynRestoreArgs::solve_sel
    // SMALL: bit b of small_mask[m][j][i] = bit i of R[m][j] x^b (R = W_E^{-1}):
    // output plane i of recovered row m is the XOR over j, b of syndrome j's
    // plane b where the bit is set
    uint16_t small_mask[kSmallMaxM][kSmallMaxM][16];
  };
  uint32_t nrec;  // SMALL: rows recovered (restore: erased points below K; regenerate: MS; 0 = none)
  uint32_t cls;   // MULTI: the plan's phase 2 (kClsSyn, kClsSmall1, kClsSmall2, kClsPerm; restore_syn.hpp)
};
struct SynBatchTile {
  uint32_t obj[2];      // object of each half (an unused half: the batch's empty object)
  uint32_t stripe0[2];  // its first stripe
  uint32_t plan;        // (RT: unused)
  uint32_t trailer;     // regenerate: bit h = half h also copies its object's trailer cell
  uint32_t nm;          // RT: rows of the tile = max ne over its halves
  uint32_t mode;        // RT: SynBatchRt::mode of both halves (the host never pairs two modes); else kTileDual or 0
};
// mode of a syndrome-route tile whose halves are objects of different
// plans (plan = half 0's; half 1's from its object: restore_syn.hpp kDual)
constexpr uint32_t kTileDual = 2;

// Reference-route tail of a regenerate.  The reference repairs a replica by
// restoring the object -- trimmed to E bytes (chunk.h:415-419, 437-438) --
// and re-encoding it: the last stripe zero-padded past E, trailer E mod 2k
// (chunk.h:251-275; sync_process.cpp:313-335 -> dht_network_client.cpp:582-658).
// The main regenerate kernels write P(t) of the untrimmed decode.  The two
// agree on every cell but the last, and there only when the survivors are
// not one codeword (a codeword's decode is already zero past E).  These
// kernels rewrite, after the main ones on the same stream, the last cell and
// the trailer of every target replica as the reference route writes them:
// with p = the trailer of the caller's first survivor (the one restore reads,
// chunk.h:408) and 0 < p < 2k, the decoded last stripe keeps bytes [0, p)
// only.  p == 0 or p == 2k trim nothing (trailer 0 for both: E mod 2k).
// p > 2k leaves the replica as the main kernels wrote it: the reference's
// route either fails ("Fatal error", p > 4k) or writes a replica 2 bytes
// longer than its survivors, so there is no chunk_size-byte answer; the host
// entry points reject such survivors (VDS_EC_ERESTORE).
struct RegenTailArgs {  // one survivor set, `count` objects at strides, any k
  const uint8_t *chunk_ptr[kInlineChunks];
  const uint8_t *const *chunk_table;  // used when k > kInlineChunks
  uint64_t chunk_stride;
  const uint16_t *matrix_dev;  // V_S^{-1} (k x k row-major) when k > kInlineMatrixK
  uint32_t matrix_inline[kInlineMatrixK * kInlineMatrixK / 2];
  uint64_t chunk_size;  // L = 2 T + 2
  uint32_t k, count, nt;
  uint16_t targets[kMaxLaunchReplicas];
  uint8_t *outs[kMaxLaunchReplicas];
  uint64_t out_stride;
};
#ifndef __HIPCC_RTC__
hipError_t launch_regen_tail(const RegenTailArgs &a, hipStream_t s);
// The batched k_restore_syn regenerate's objects objs[0..count) (device
// tables of the batch launch; survivor points from their plans, targets the
// plans' erased points with regen[w] set): the last stripe interpolated on
// the device, one wave per object (k <= 64).
hipError_t launch_regen_tail_batch(uint32_t k, uint32_t m, const SynBatchObj *objs, const SynBatchPlan *plans,
                                   uint32_t count, hipStream_t s);
// The same for RT objects (survivor points rt.spoint, targets rt.epoint[0..ne)).
hipError_t launch_regen_tail_rt(uint32_t k, const SynBatchObj *objs, uint32_t count, hipStream_t s);
// RT coefficient rows of objs[0..count) (one wave per object, k <= 64): row m,
// column j = l_j(epoint[m]), the Lagrange basis polynomial of slot j over the
// slots' points spoint evaluated at epoint[m] -- the unique polynomial through
// the k survivors, evaluated where it is needed.
hipError_t launch_rt_coefs(uint32_t k, const SynBatchObj *objs, uint32_t count, hipStream_t s);
// Batched RT restore / regenerate: a.objs / a.tiles / a.total_tiles set (every
// object's rt filled, its coef rows computed); regenerate rows ne <= n - k.
hipError_t launch_restore_rt_batch(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen);

hipError_t launch_encode_generic(const GenericEncodeArgs &a, hipStream_t s);
bool has_restore_syn(uint32_t k, uint32_t n);
// W[j][a] = v_a a^j of the syndrome map for (k, n); nullptr if not compiled.
const uint16_t *restore_syn_weights(uint32_t k, uint32_t n);
hipError_t launch_restore_syn(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen = false);
// The run-time compiled restore kernel of a's survivor set (vds_ec_jit.cpp) on
// the current device, or nullptr (disabled, not compiled yet -- then queued --
// or failed): a.point[0..k) set by the plan.
hipFunction_t jit_restore_function(uint32_t k, uint32_t n, const SynRestoreArgs &a, bool regen = false);
// the set's kernel is loaded and the module is enabled (path queries)
bool jit_ready(uint32_t k, uint32_t n, const SynRestoreArgs &a, bool regen);
bool jit_enabled();  // mode != 0 (vds_ec_jit_set_mode)
hipError_t launch_restore_syn_jit(hipFunction_t fn, uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s);
// a.objs / a.plans / a.tiles / a.total_tiles set; the other fields unused
hipError_t launch_restore_syn_batch(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen);
// SMALL batch mode over the points 0..k+ms-1 (ms = 1, 2; k = 16, 32): tables as
// launch_restore_syn_batch, plans with small_mask / nrec.
bool has_restore_small(uint32_t k, uint32_t ms);
// W[j][a] = v_a a^j of the ms checks over A = {0..k+ms-1}; nullptr if not compiled.
const uint16_t *restore_small_weights(uint32_t k, uint32_t ms);
hipError_t launch_restore_small_batch(uint32_t k, uint32_t ms, const SynRestoreArgs &a, hipStream_t s, bool regen);
// PERM batch regenerate (k = 16, 32): survivors exactly 0..k-1, one target
// t = erased[0] of each plan in k..2k-1.
hipError_t launch_regen_perm_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s);
// MULTI: one launch over tiles of every class, each plan's cls choosing its
// phase 2 (k = 16, 32).
hipError_t launch_restore_multi_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s, bool regen);
hipError_t launch_regen_generic(const RegenArgs &a, hipStream_t s);
hipError_t launch_restore_generic(const GenericRestoreArgs &a, hipStream_t s);
// Returns hipErrorNotSupported when no bit-sliced instantiation exists for (k, n).
hipError_t launch_encode_fast(uint32_t k, uint32_t n, const FastEncodeArgs &a, hipStream_t s);
bool has_encode_fast(uint32_t k, uint32_t n);
// SHA-256 of one message on the calling CPU thread (sha256_host.cpp)
void sha256_host(const uint8_t *data, uint64_t len, uint8_t out[32]);
hipError_t launch_restore_fast(uint32_t k, const FastRestoreArgs &a, hipStream_t s, bool regen = false);
bool has_restore_fast(uint32_t k);
// SHA-256 of count messages of len bytes at base + j * stride -> digests + 32 j (sha256.hip).
hipError_t launch_sha256(const uint8_t *base, uint64_t len, uint64_t stride, uint32_t count, uint8_t *digests,
                         hipStream_t s);
hipError_t launch_fill_splitmix(uint8_t *dst, uint64_t size, uint64_t seed, hipStream_t s);
// Device -> mapped pinned host copy by a kernel (dst: the device view of the
// host buffer; both 16-byte aligned).
hipError_t launch_push(uint8_t *dst_host_dev, const uint8_t *src, uint64_t bytes, hipStream_t s);

#endif  // __HIPCC_RTC__

}  // namespace vds_ec
