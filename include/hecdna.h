/*
 * hecdna.h — C-ABI of the MI355X-native CKKS homomorphic linear-algebra engine.
 *
 * This is the drop-in boundary for the reference's hot path
 * (isteiakakis/Homomorphic-Encryption-Algorithms-Diploma-Thesis):
 * every arithmetic step of he::linalg / he::operators goes through a seal::Evaluator member call;
 * each entry point below replaces one of those calls (reference file:line cited per function) and
 * keeps its argument meaning, data layout and error behaviour:
 *
 *   - data layout = SEAL layout: a ciphertext is u64[size][level][N] in NTT form, a plaintext
 *     u64[level][N] in NTT form, a key-switching key (one RelinKeys / GaloisKeys entry, i.e. SEAL's
 *     vector<PublicKey>) u64[L][2][K][N], where K = #coeff_modulus, L = K-1 data primes and
 *     "level" = number of data primes a ciphertext currently has (SEAL chain index + 1);
 *   - all residues canonical in [0, q); every result is bit-identical to this repository's CPU
 *     restatement of SEAL 4.1's Evaluator (oracle/).  Against SEAL itself parity is unpinned:
 *     SEAL is absent here and the reference ships no test vectors;
 *   - errors: SEAL throws std::invalid_argument / std::logic_error; here every call returns a
 *     status (HEC_OK, HEC_EINVAL for invalid_argument, HEC_ELOGIC for logic_error, HEC_EDEVICE for a
 *     HIP failure) and hec_last_error() returns SEAL's message text ("scale mismatch",
 *     "Galois key not present", "end of modulus switching chain reached", ...).
 *
 * Objects are device-resident on the context's GPU; every call is ordered on the context's HIP
 * stream (hec_context_set_stream), downloads synchronise.  One context per device, one host
 * thread per context.  A matvec runs its whole batch on the context's stream by default (one lane); the
 * option "lanes" > 1 (HEC_LANES) splits a batch of >= 32 vectors into concurrent lanes on engine-owned threads
 * and streams, joined before it returns (opt-in).  No torch types cross this boundary.
 */
#ifndef HECDNA_H
#define HECDNA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HEC_OK 0
#define HEC_EINVAL 1
#define HEC_ELOGIC 2
#define HEC_EDEVICE 3

typedef struct hec_context hec_context;
typedef struct hec_ciphertext hec_ciphertext;
typedef struct hec_plaintext hec_plaintext;
typedef struct hec_kswitch_key hec_kswitch_key; /* one KSwitchKeys entry: RelinKeys[0] */
typedef struct hec_galois_keys hec_galois_keys; /* GaloisKeys: galois_elt -> key */

const char *hec_last_error(void);
int hec_version(void);

/* ---------------------------------------------------------------- parameters / context ---- */
/* seal::CoeffModulus::Create(N, bit_sizes) — used at reference matrix_operations.cpp:1050 */
int hec_create_coeff_modulus(uint64_t poly_modulus_degree, const int *bit_sizes, uint64_t count, uint64_t *out);
/* seal::SEALContext(EncryptionParameters{ckks, N, coeff_modulus}) — matrix_operations.cpp:1047-1051.
 * coeff_modulus[K-1] is the special (key) prime.  device = HIP device ordinal. */
int hec_context_create(uint64_t poly_modulus_degree, const uint64_t *coeff_modulus, uint64_t K, int device,
                       hec_context **out);
/* Objects (ciphertexts, plaintexts, keys) may be destroyed before or after their context, in any order, as SEAL's
 * objects holding their context by shared_ptr allow: an object destroyed after its context frees its own device
 * memory and touches nothing else. */
int hec_context_destroy(hec_context *ctx);
int hec_context_set_stream(hec_context *ctx, void *hip_stream); /* NULL = context-owned stream */
int hec_context_synchronize(hec_context *ctx);
/* Engine knobs at run time (no SEAL counterpart; the HEC_* environment switches of DESIGN.md §4.1 set the
 * same knobs at context creation): "lanes", "lane_min_batch", "hoist", "hoist_min", "hmac", "hmac_odd3",
 * "hoist_scan", "fan", "fuse_galois", "fused_modup_mac", "tensor_defer", "tensor_bufs", "tensor_xcd",
 * "split_bfly", "bmac_split", "nttb_shfl" (the forward pass B at 128 points with its exchanges as DPP lane moves
 * instead of LDS: 1, 16 outputs per lane; 2, swapped back for coalesced stores), "nttb_shfl_dr" (the same for the
 * divide-and-round pass B), "moddown1" (the single-pass mod-down at N = 2^15), "hmac_int" (0: the 60-bit hoisted MAC
 * targets on the round-5 loop), "nt_e" (0: the hoisted digits stored with the default cache policy instead of
 * non-temporally), "kernel_memops" (0: workspace fills and device copies through the runtime's
 * hipMemsetAsync / hipMemcpyAsync instead of engine kernels; A/B only), and three debug switches:
 * "poison" (every workspace carve and fresh output buffer is filled with 0xFF bytes before use, so a read of
 * memory the call never wrote becomes a deterministic wrong result), "lane_serial" (batch lanes run one after
 * another) and "debug_lanes" (per-call zero-list and key-table reports on stderr).  Every schedule is
 * bit-identical.  Applies to the context and its batch lanes; HEC_EINVAL for an unknown name, and for a value
 * outside an enumerated knob's range ("split_bfly" 0..4, "hmac" 0..2, "hmac_odd3" 0..1, "hoist_scan" 0..1,
 * "nttb_shfl" 0..2, "nttb_shfl_dr" 0..1, "moddown1" 0..1, "hmac_int" 0..1, "nt_e" 0..1). */
int hec_context_set_option(hec_context *ctx, const char *name, int64_t value);
uint64_t hec_context_poly_degree(const hec_context *ctx);
uint64_t hec_context_key_moduli(const hec_context *ctx); /* K */
/* seal::GaloisTool::get_elt_from_step (rotation step -> Galois element); 0 on error */
uint32_t hec_galois_elt_from_step(const hec_context *ctx, int step);
/* seal::GaloisTool::get_elts_all — the set KeyGenerator::create_galois_keys() makes
 * (matrix_operations.cpp:1063-1064).  Returns the count; writes it when out != NULL. */
uint64_t hec_default_galois_elts(const hec_context *ctx, uint32_t *out);

/* ---------------------------------------------------------------- ciphertext / plaintext -- */
int hec_ciphertext_create(hec_context *ctx, hec_ciphertext **out);
int hec_ciphertext_destroy(hec_ciphertext *ct);
/* host SEAL-layout buffer u64[size][level][N] -> device */
int hec_ciphertext_upload(hec_ciphertext *ct, const uint64_t *host, uint64_t size, uint64_t level, double scale);
/* device -> host (synchronises); host must hold size*level*N words */
int hec_ciphertext_download(const hec_ciphertext *ct, uint64_t *host);
int hec_ciphertext_info(const hec_ciphertext *ct, uint64_t *size, uint64_t *level, double *scale);
int hec_ciphertext_copy(hec_ciphertext *dst, const hec_ciphertext *src); /* value semantics, deep copy */
/* device-to-device import/export of the raw u64 words (for RCCL exchanges done by the caller) */
int hec_ciphertext_export_device(const hec_ciphertext *ct, void *dev_dst);
int hec_ciphertext_import_device(hec_ciphertext *ct, const void *dev_src, uint64_t size, uint64_t level,
                                 double scale);
/* canonicalise every word mod its prime (after an integer sum of partial accumulators) */
int hec_ciphertext_reduce(hec_context *ctx, hec_ciphertext *ct);
/* synthetic input: uniformly random residues (RLWE ciphertexts are pseudo-uniform) */
int hec_ciphertext_fill_uniform(hec_ciphertext *ct, uint64_t size, uint64_t level, double scale, uint64_t seed);

int hec_plaintext_create(hec_context *ctx, hec_plaintext **out);
int hec_plaintext_destroy(hec_plaintext *pt);
int hec_plaintext_upload(hec_plaintext *pt, const uint64_t *host, uint64_t level, double scale);
/* synthetic NTT-form plaintext: uniform residues mod q_i from a seeded device generator (benchmarks) */
int hec_plaintext_fill_uniform(hec_plaintext *pt, uint64_t level, double scale, uint64_t seed);
int hec_plaintext_download(const hec_plaintext *pt, uint64_t *host); /* u64[level][N], synchronises */
int hec_plaintext_info(const hec_plaintext *pt, uint64_t *level, double *scale);
/* seal::CKKSEncoder::encode(values, [parms_id,] scale, destination) on the GPU, for `count` slot vectors at
 * once — the reference encodes every matrix column / diagonal this way before encryption
 * (src/demos/matrix_operations.cpp:1106-1108, client.cpp:228-230, he_math.cpp:32-53 through
 * he_util.h:33-36).  re / im: host doubles, count rows of n_values (n_values <= N/2; missing slots are
 * zero); im = NULL encodes real values (SEAL's vector<double> overload).  out[v] receives an NTT-form
 * plaintext at `level` with `scale`.  Errors as SEAL: "values has invalid size", "scale out of bounds",
 * "encoded values are too large". */
int hec_encode(hec_context *ctx, const double *re, const double *im, uint64_t n_values, uint64_t count, double scale,
               uint64_t level, hec_plaintext *const *out);
/* seal::CKKSEncoder::encode(double value, parms_id, scale, destination) (SEAL 4.1 encode_internal(double, ...)), the
 * scalar form he::util::drop_chain_levels and he::math use (include/he_util.h:33, src/core/he_math.cpp:32,40,53):
 * round(value * scale) as an exact integer, its residue mod every prime of `level` (negated for a negative value),
 * written to every word of that limb (the NTT form of a constant polynomial); no transform runs.  Errors as SEAL:
 * "parms_id is not valid for encryption parameters", "scale out of bounds", "encoded value is too large" (also for a
 * non-finite value). */
int hec_encode_scalar(hec_context *ctx, double value, double scale, uint64_t level, hec_plaintext *out);

/* ---------------------------------------------------------------- keys -------------------- */
/* RelinKeys (KeyGenerator::create_relin_keys, matrix_operations.cpp:1061-1062): data u64[L][2][K][N] */
int hec_kswitch_key_upload(hec_context *ctx, const uint64_t *host, hec_kswitch_key **out);
/* device -> host in the layout of hec_kswitch_key_upload (synchronises) */
int hec_kswitch_key_download(const hec_kswitch_key *key, uint64_t *host);
int hec_kswitch_key_fill_uniform(hec_context *ctx, uint64_t seed, hec_kswitch_key **out);
int hec_kswitch_key_destroy(hec_kswitch_key *key);
/* GaloisKeys (KeyGenerator::create_galois_keys, matrix_operations.cpp:1063-1064) */
int hec_galois_keys_create(hec_context *ctx, hec_galois_keys **out);
int hec_galois_keys_add(hec_galois_keys *gk, uint32_t galois_elt, const uint64_t *host);
/* one Galois key, device -> host in the layout of hec_galois_keys_add (synchronises); HEC_EINVAL "Galois key not
 * present" when the set has no key for galois_elt */
int hec_galois_keys_download(const hec_galois_keys *gk, uint32_t galois_elt, uint64_t *host);
int hec_galois_keys_add_uniform(hec_galois_keys *gk, uint32_t galois_elt, uint64_t seed);
int hec_galois_keys_has(const hec_galois_keys *gk, uint32_t galois_elt);
int hec_galois_keys_destroy(hec_galois_keys *gk);

/* ---------------------------------------------------------------- evaluator --------------- */
/* Each replaces the seal::Evaluator call behind one he::operators operator
 * (reference include/he_operators.h:44-159, src/core/he_operators.cpp:14-237). */
int hec_negate_inplace(hec_context *ctx, hec_ciphertext *a);                                  /* op -= eval     */
int hec_add_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b);           /* a += eval % b  */
int hec_sub_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b);           /* a -= eval % b  */
int hec_add_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p);      /* a += eval % pt */
int hec_sub_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p);      /* a -= eval % pt */
int hec_multiply_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b);      /* a *= eval % b  */
int hec_multiply_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p); /* a *= eval % pt */
int hec_square_inplace(hec_context *ctx, hec_ciphertext *a);                                  /* he_linalg.cpp:647 */
int hec_relinearize_inplace(hec_context *ctx, hec_ciphertext *a, const hec_kswitch_key *rk); /* a &= eval % rk */
int hec_rescale_to_next_inplace(hec_context *ctx, hec_ciphertext *a);                         /* a ^= eval      */
int hec_mod_switch_to_next_inplace(hec_context *ctx, hec_ciphertext *a);                      /* a |= eval      */
/* a <<= eval % gk % steps (left); right rotation = negative steps (he_operators.cpp:204-235) */
int hec_rotate_vector_inplace(hec_context *ctx, hec_ciphertext *a, int steps, const hec_galois_keys *gk);
int hec_apply_galois_inplace(hec_context *ctx, hec_ciphertext *a, uint32_t galois_elt, const hec_galois_keys *gk);

/* ---------------------------------------------------------------- he::linalg hot path ----- */
/* BatchedMatrix::matmul(eval, rk, gk, other), diag(this) x col(other) (he_linalg.cpp:943-1006):
 *   out[i] = rescale(relin( sum_{j<n} rot(cols[i], j) (*) diags[j] )),  i < p
 * n diagonal ciphertexts, p column ciphertexts (the p independent input vectors of a matvec batch).
 * out[i] may be fresh ciphertexts; they receive level = input level - 1. */
int hec_matmul_diag_col(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                        const hec_ciphertext *const *cols, uint64_t p, const hec_kswitch_key *rk,
                        const hec_galois_keys *gk, hec_ciphertext *const *out);
/* Sharded form: size-3 partial sums over diagonals [j_begin, j_end) (no relin / rescale). */
int hec_matmul_diag_col_partial(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                                uint64_t j_begin, uint64_t j_end, const hec_ciphertext *const *cols, uint64_t p,
                                const hec_galois_keys *gk, hec_ciphertext *const *acc_out);
/* Sharded form over an arbitrary set of diagonal indices j_idx[0..nj) (any order, no duplicates): the
 * multi-GPU planner hands each rank whole subtrees of the rotation prefix trie so that no key switch
 * is repeated across ranks.  Summing the partials of a partition of [0, n) mod q gives exactly the
 * accumulator of hec_matmul_diag_col. */
int hec_matmul_diag_col_partial_set(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                                    const uint64_t *j_idx, uint64_t nj, const hec_ciphertext *const *cols, uint64_t p,
                                    const hec_galois_keys *gk, hec_ciphertext *const *acc_out);
/* ct x pt matvec (the plaintext-diagonal form of BatchedMatrix::matmul diag x col,
 * he_linalg.cpp:943-1006, with `*= eval % plain` = multiply_plain_inplace, he_operators.cpp:128-142):
 *   out[i] = rescale_to_next( sum_j diags[j] (x) rot(cols[i], j) )
 * diags: n NTT-form plaintexts at the columns' level (SEAL CKKSEncoder output layout u64[level][N]).
 * The products stay size 2, so there is no relinearization; rotations as in hec_matmul_diag_col. */
int hec_matmul_diagpt_col(hec_context *ctx, const hec_plaintext *const *diags, uint64_t n,
                          const hec_ciphertext *const *cols, uint64_t p, const hec_galois_keys *gk,
                          hec_ciphertext *const *out);
/* relinearize + rescale a batch of size-3 accumulators (he_linalg.cpp:999-1002) */
int hec_matmul_finish(hec_context *ctx, hec_ciphertext *const *acc, uint64_t p, const hec_kswitch_key *rk,
                      hec_ciphertext *const *out);
/* BatchedMatrix::matmul, col(this) x col(other)^T -> diag output:
 *   out[i] = rescale(relin( sum_{j<n} rot(B[j], i) (*) A[j] )), i < p */
int hec_matmul_col_colT(hec_context *ctx, const hec_ciphertext *const *A, uint64_t n,
                        const hec_ciphertext *const *B, uint64_t p, const hec_kswitch_key *rk,
                        const hec_galois_keys *gk, hec_ciphertext *const *out);
/* Matrix::matmul (he_linalg.cpp:202-236): column-major element-wise ciphertext matrices
 * (index i + rows*j, swapped when *_transposed); out has r1*c2 entries, column-major. */
int hec_matrix_matmul(hec_context *ctx, const hec_ciphertext *const *A, uint64_t a_rows, uint64_t a_cols,
                      int a_transposed, const hec_ciphertext *const *B, uint64_t b_rows, uint64_t b_cols,
                      int b_transposed, const hec_kswitch_key *rk, hec_ciphertext *const *out);

/* ---------------------------------------------------------------- multi-GPU (SURVEY 8(b),(e)) */
/* One process per GPU.  The reference is single-threaded (no collective anywhere); the sharded matvec splits
 * the diagonal loop of BatchedMatrix::matmul (he_linalg.cpp:977-997) over the ranks and exchanges the size-3
 * partial sums once over RCCL (xGMI), so a C++ caller of the he_linalg.h drop-in shards through this ABI alone.
 *
 * Planner (host only, no GPU): rank_of_diag[j] = the rank that owns diagonal j < n: whole subtrees of the
 * rotation prefix trie (SEAL's key-switch sequences over the key set key_elts), balanced by key switches. */
int hec_plan_diagonal_shards(uint64_t poly_modulus_degree, uint64_t n, int world, const uint32_t *key_elts,
                             uint64_t nkeys, int32_t *rank_of_diag);
/* ncclGetUniqueId: 128 bytes that rank 0 creates and every rank passes to hec_comm_init (RCCL is loaded on
 * first use from librccl.so.1; HEC_ELOGIC when it is absent). */
int hec_comm_unique_id(void *unique_id);
/* ncclCommInitRank on the context's device; world == 1 needs no id; 1 <= world <= 8 (the partial-sum exchange
 * adds world canonical 60-bit residues in u64).  The communicator lives until hec_context_destroy. */
int hec_comm_init(hec_context *ctx, int rank, int world, const void *unique_id);
/* A host communicator: the caller's own collectives (MPI, a gloo process group, ...) for the sharded
 * matvec, in place of RCCL.  Both callbacks are all-reduces over the world, in place, on host memory, and return
 * 0 on success.  allreduce_f64: op HEC_REDUCE_MIN or HEC_REDUCE_MAX.  allreduce_u64_sum: exact (world <= 8
 * residues < 2^60).  The engine calls them from the thread that called hec_matmul_diag_col_sharded. */
#define HEC_REDUCE_MIN 0
#define HEC_REDUCE_MAX 1
typedef struct hec_comm_ops {
    void *user;
    int (*allreduce_f64)(void *user, double *buf, uint64_t count, int op);
    int (*allreduce_u64_sum)(void *user, uint64_t *buf, uint64_t count);
} hec_comm_ops;
/* hec_comm_init with the caller's collectives (*ops is copied); same world bound. */
int hec_comm_init_ops(hec_context *ctx, int rank, int world, const hec_comm_ops *ops);
/* The agreement step hec_matmul_diag_col_sharded runs before any data moves (host only, no device needed): each
 * rank passes its own check result (status HEC_OK / HEC_EINVAL / HEC_ELOGIC and SEAL's message) and its p output
 * product scales; after two allreduce_f64 calls a failing rank returns its own status and message, every other rank
 * the status of the failing rank with the larger (status << 8 | rank + 1) and "... failed SEAL's checks on rank r";
 * when no rank failed, every rank returns HEC_EINVAL "scale mismatch" if the ranks' scales of one output are not
 * SEAL-close (add_inplace over the whole sum), else HEC_OK.  No rank is left waiting in the exchange.  msg (cap bytes,
 * may be NULL) receives the message.  HEC_EDEVICE / HEC_ELOGIC when a callback fails. */
int hec_shard_agree(const hec_comm_ops *ops, int rank, int status, const char *reason, const double *scales,
                    uint64_t p, char *msg, uint64_t msg_cap);
/* 1 when the context has a communicator (then *rank, *world are set), 0 when not, HEC_EINVAL on NULL */
int hec_context_comm(const hec_context *ctx, int *rank, int *world);
/* BatchedMatrix::matmul diag x col over the world (every rank calls it with the same arguments): rank r
 * computes the partial sums over its planned diagonals (hec_plan_diagonal_shards with the keys of gk): only those
 * diags[j] are read and checked, every other entry is never dereferenced and may be NULL or any handle.  The
 * ranks then agree on the argument checks (hec_shard_agree's protocol: two all-reduces of p + 1 doubles, min and
 * max, over the RCCL or the host communicator, so an error on one rank is returned on all ranks instead of leaving
 * the others in the exchange), run one all-reduce of the partials (RCCL,
 * or the host communicator of hec_comm_init_ops; u64 sum, exact
 * for world <= 8 and 60-bit primes) + reduction mod q, and every rank relinearizes and rescales all p outputs:
 * out[i] is bit-identical to hec_matmul_diag_col on one GPU. */
int hec_matmul_diag_col_sharded(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                                const hec_ciphertext *const *cols, uint64_t p, const hec_kswitch_key *rk,
                                const hec_galois_keys *gk, hec_ciphertext *const *out);

/* ---------------------------------------------------------------- SEAL wire format */
/* seal::Serialization::Save / Load byte layouts of the objects the reference's socket layer exchanges
 * (src/demos/client.cpp:113-115,238-240 saves, src/demos/server.cpp:110-122,140-152 loads): SEALHeader (16 B:
 * magic 0xA15E, header size, version 4.1, compr_mode, size) + members, compr_mode HEC_COMPR_NONE / ZLIB / ZSTD
 * (zlib, zstd loaded on first use).  Host-only functions return HEC_EINVAL with SEAL's wording for malformed
 * input ("loaded SEALHeader is invalid", ...); hec_seal_last_error() holds the message.  Seeded ciphertexts
 * (encrypt_symmetric().save(), client.cpp:113-114) are expanded by hec_seal_ciphertext_load_ex and by the device
 * loader hec_ciphertext_load_seal (Ciphertext::expand_seed); hec_seal_ciphertext_load, which has no moduli,
 * rejects them (HEC_EINVAL).  Decompressed objects are bounded, since the bytes come from a client socket
 * (server.cpp:110-122): 2 GiB per ciphertext; a key object (with every compressed member nested in it) by the
 * caller's max_bytes in the *_ex forms, by 16 GiB in the others, and by a fixed count of key lists in the device
 * loaders (hec_galois_keys_load_seal_ex; it does not depend on the device's free memory).  A payload over its limit is HEC_EINVAL ("decompressed SEAL object exceeds the
 * size limit"); a payload must also hold the words it announces. */
#define HEC_COMPR_NONE 0
#define HEC_COMPR_ZLIB 1
#define HEC_COMPR_ZSTD 2
const char *hec_seal_last_error(void);
/* BLAKE2b (util::HashFunction behind parms_id), outlen <= 64 bytes */
int hec_seal_blake2b(const void *in, uint64_t nbytes, uint64_t outlen, void *out);
/* EncryptionParameters::parms_id() of CKKS {N, coeff_modulus[0..count)} (a ciphertext at level l: its l primes) */
int hec_seal_parms_id(uint64_t poly_modulus_degree, const uint64_t *coeff_modulus, uint64_t count, uint64_t out[4]);
/* Ciphertext::load / save on host buffers: data u64[size][level][N]; *consumed / *written = object bytes
 * (out == NULL: size query) */
int hec_seal_ciphertext_load(const void *bytes, uint64_t nbytes, uint64_t *size, uint64_t *level,
                             uint64_t *poly_modulus_degree, double *scale, uint64_t parms_id[4], uint64_t *data,
                             uint64_t data_words, uint64_t *consumed);
/* Ciphertext::load(context, ...) including a seeded object (c0 + UniformRandomGeneratorInfo, as
 * Encryptor::encrypt_symmetric(...).save writes it: src/demos/client.cpp:113-114): c1 is expanded with SEAL 4.1's
 * Ciphertext::expand_seed (Blake2xbPRNG + sample_poly_uniform) over coeff_modulus[0..level); the parms_id must
 * match; prng_type blake2xb (SEAL's default) or shake256.  coeff_modulus = NULL behaves as hec_seal_ciphertext_load (a seeded object is an error). */
int hec_seal_ciphertext_load_ex(const void *bytes, uint64_t nbytes, const uint64_t *coeff_modulus, uint64_t count,
                                uint64_t *size, uint64_t *level, uint64_t *poly_modulus_degree, double *scale,
                                uint64_t parms_id[4], uint64_t *data, uint64_t data_words, uint64_t *consumed);
/* BLAKE2Xb XOF (SEAL util/blake2xb.c, behind Blake2xbPRNG): outlen bytes of BLAKE2Xb(in) keyed with key */
int hec_seal_blake2xb(const void *in, uint64_t nbytes, const void *key, uint64_t keylen, uint64_t outlen, void *out);
/* SHAKE256 XOF (behind SEAL's Shake256PRNG) */
int hec_seal_shake256(const void *in, uint64_t nbytes, uint64_t outlen, void *out);
int hec_seal_ciphertext_save(const uint64_t *data, uint64_t size, uint64_t level, uint64_t poly_modulus_degree,
                             double scale, const uint64_t *coeff_modulus, int compr_mode, void *out, uint64_t cap,
                             uint64_t *written);
/* EncryptionParameters::load / save (CKKS) */
int hec_seal_parms_load(const void *bytes, uint64_t nbytes, uint64_t *poly_modulus_degree, uint64_t *coeff_modulus,
                        uint64_t cap, uint64_t *count, uint64_t *consumed);
int hec_seal_parms_save(uint64_t poly_modulus_degree, const uint64_t *coeff_modulus, uint64_t count, int compr_mode,
                        void *out, uint64_t cap, uint64_t *written);
/* the decompressed-size limit of the context-free key loaders below: 16 GiB (SEAL's default GaloisKeys at
 * N = 2^16 with 17 primes take 8.84 GB), bounded by half the host's available memory (the object is inflated in host
 * memory), at least 1 GiB */
uint64_t hec_seal_kswitch_keys_default_limit(void);
/* KSwitchKeys (RelinKeys, GaloisKeys) load of key list `index` (RelinKeys 0, GaloisKeys (galois_elt - 1) / 2)
 * in the engine's key layout u64[L][2][K][N]; *lists = the object's list count, *words = that list's words */
int hec_seal_kswitch_keys_load(const void *bytes, uint64_t nbytes, uint64_t index, uint64_t *lists, uint64_t *out,
                               uint64_t cap_words, uint64_t *words, uint64_t *consumed);
/* ... with at most max_bytes decompressed (0: hec_seal_kswitch_keys_default_limit) */
int hec_seal_kswitch_keys_load_ex(const void *bytes, uint64_t nbytes, uint64_t index, uint64_t max_bytes,
                                  uint64_t *lists, uint64_t *out, uint64_t cap_words, uint64_t *words,
                                  uint64_t *consumed);
/* The same object in ONE pass: visit(user, index, words, nwords) is called for every non-empty key list in order
 * (GaloisKeys hold N lists, almost all empty, so a per-index hec_seal_kswitch_keys_load would reparse the object N
 * times).  A non-zero return from visit stops the walk, and the function returns that status unchanged (with
 * hec_seal_last_error() = "key list rejected by the caller").  *lists = the object's list count. */
int hec_seal_kswitch_keys_foreach(const void *bytes, uint64_t nbytes,
                                  int (*visit)(void *user, uint64_t index, const uint64_t *words, uint64_t nwords),
                                  void *user, uint64_t *lists, uint64_t *consumed);
/* ... with at most max_bytes decompressed (0: hec_seal_kswitch_keys_default_limit) */
int hec_seal_kswitch_keys_foreach_ex(const void *bytes, uint64_t nbytes, uint64_t max_bytes,
                                     int (*visit)(void *user, uint64_t index, const uint64_t *words, uint64_t nwords),
                                     void *user, uint64_t *lists, uint64_t *consumed);
int hec_seal_kswitch_keys_save(uint64_t poly_modulus_degree, const uint64_t *coeff_modulus, uint64_t K,
                               const uint64_t *const *keys, const uint64_t *digits, uint64_t nlists, int compr_mode,
                               void *out, uint64_t cap, uint64_t *written);
/* device objects: Ciphertext::load(context, ...) (checks N and the parms_id of its level against the context)
 * and Ciphertext::save(stream, compr_mode); RelinKeys::load; GaloisKeys::load (every non-empty key list) */
int hec_ciphertext_load_seal(hec_ciphertext *ct, const void *bytes, uint64_t nbytes, uint64_t *consumed);
int hec_ciphertext_save_seal(const hec_ciphertext *ct, int compr_mode, void *out, uint64_t cap, uint64_t *written);
int hec_kswitch_key_load_seal(hec_context *ctx, const void *bytes, uint64_t nbytes, hec_kswitch_key **out,
                              uint64_t *consumed);
int hec_galois_keys_load_seal(hec_galois_keys *gk, const void *bytes, uint64_t nbytes, uint64_t *consumed);
/* ... with at most max_lists non-empty key lists (0: the default, hec_galois_keys_load_seal_default_lists: four times
 * SEAL's default set of 2 log2(N) - 1, at least 64, at most N, bounded by half the host's available memory; it does
 * not depend on the device).  More lists, or a compressed object that inflates beyond them, is invalid_argument
 * "decompressed SEAL object exceeds the size limit" (the object is inflated in host memory before it is parsed). */
int hec_galois_keys_load_seal_ex(hec_galois_keys *gk, const void *bytes, uint64_t nbytes, uint64_t max_lists,
                                 uint64_t *consumed);
uint64_t hec_galois_keys_load_seal_default_lists(const hec_context *ctx);

/* ---------------------------------------------------------------- primitives (cfg2) ------- */
/* In-place batched negacyclic NTT over device data u64[npolys][nlimbs][N]; limb j uses prime
 * limb0 + j (SEAL ntt_negacyclic_harvey / inverse_ntt_negacyclic_harvey, canonical in/out). */
int hec_ntt_forward(hec_context *ctx, uint64_t *dev_data, uint64_t limb0, uint64_t nlimbs, uint64_t npolys);
int hec_ntt_inverse(hec_context *ctx, uint64_t *dev_data, uint64_t limb0, uint64_t nlimbs, uint64_t npolys);
/* out = a (*) b (dyadic_product_coeffmod), same layout */
int hec_dyadic_multiply(hec_context *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint64_t limb0,
                        uint64_t nlimbs, uint64_t npolys);
/* device memory helpers for the primitive API and tests */
int hec_device_alloc(hec_context *ctx, uint64_t bytes, void **out);
int hec_device_free(hec_context *ctx, void *p);
int hec_memcpy_h2d(hec_context *ctx, void *dst, const void *src, uint64_t bytes);
int hec_memcpy_d2h(hec_context *ctx, void *dst, const void *src, uint64_t bytes);

/* ---------------------------------------------------------------- measurement ------------- */
/* Time `reps` launches of the batched forward NTT on the context stream with HIP events
 * (average ms per launch written to *ms). */
int hec_time_ntt_forward(hec_context *ctx, uint64_t *dev_data, uint64_t nlimbs, uint64_t npolys, int reps,
                         double *ms);
/* Per-kernel-class GPU timing of the engine's phases (ks_intt, ks_modup_a, ks_bmac, ks_moddown, galois,
 * tensor, relin, rescale, ...).  mode 0 off, 1 event pair + synchronize per phase, 2 asynchronous event
 * pairs (no host synchronisation inside calls; resolved by hec_profile_read).  Read cumulative ms and
 * phase counts per class. */
int hec_profile_enable(hec_context *ctx, int mode);
int hec_profile_read(hec_context *ctx, const char *kernel_class, double *total_ms, uint64_t *launches);
/* The same plus the class's algorithmic bytes (compulsory reads + writes of its kernels, summed over its
 * scopes) and kernel launches.  Classes named "k:<kernel>/<role>" wrap single kernels (k_fan, k_ntt, k_bmac,
 * k_hmacm, k_tensor_multi, k_zscan) inside the phases, so bytes / ms is that kernel's achieved GB/s. */
int hec_profile_read_ex(hec_context *ctx, const char *kernel_class, double *total_ms, uint64_t *scopes,
                        double *alg_bytes, uint64_t *kernel_launches);
/* Newline-separated names of every class recorded since hec_profile_enable; returns the bytes needed
 * (including the terminating NUL), writes at most cap bytes into buf when buf != NULL. */
uint64_t hec_profile_classes(hec_context *ctx, char *buf, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* HECDNA_H */
