// ORACLE C API — test infrastructure only (see oracle.hpp).  Flat extern "C" entry points so
// tests/ (ctypes) and bench.py's cpu_baseline leg can drive the CPU restatement.
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <string>

#include "oracle.hpp"

using namespace oracle;

namespace {
thread_local std::string g_err;

struct OrcCt {  // mirrors the ctypes structure in tests/oracle_py.py
    u64 *data;
    u64 size, level;
    double scale;
};

Ciphertext in_ct(const Context &ctx, const OrcCt *c)
{
    Ciphertext r;
    r.size = c->size; r.level = c->level; r.scale = c->scale;
    r.data.assign(c->data, c->data + c->size * c->level * ctx.N());
    return r;
}
void out_ct(const Ciphertext &r, OrcCt *c)
{
    std::memcpy(c->data, r.data.data(), r.data.size() * sizeof(u64));
    c->size = r.size; c->level = r.level; c->scale = r.scale;
}
KSwitchKey view(const u64 *p) { KSwitchKey k; k.data = p; return k; }
GaloisKeys gkeys(const u32 *elts, const u64 *const *ptrs, u64 n)
{
    GaloisKeys g;
    for (u64 i = 0; i < n; ++i) g[elts[i]] = view(ptrs[i]);
    return g;
}

template <class F>
int guard(F &&f)
{
    try { f(); return 0; }
    catch (const std::invalid_argument &e) { g_err = e.what(); return 1; }
    catch (const std::logic_error &e) { g_err = e.what(); return 2; }
    catch (const std::exception &e) { g_err = e.what(); return 3; }
}
}  // namespace

extern "C" {

const char *orc_last_error() { return g_err.c_str(); }

void *orc_ctx_new(u64 N, u64 K, const u64 *moduli)
{
    Context *c = nullptr;
    if (guard([&] { c = new Context(N, std::vector<u64>(moduli, moduli + K)); })) return nullptr;
    return c;
}
void orc_ctx_free(void *c) { delete static_cast<Context *>(c); }

int orc_create_coeff_modulus(u64 N, u64 n, const int *bits, u64 *out)
{
    return guard([&] {
        auto v = create_coeff_modulus(N, std::vector<int>(bits, bits + n));
        std::memcpy(out, v.data(), v.size() * sizeof(u64));
    });
}
int orc_is_prime(u64 n) { return is_prime(n) ? 1 : 0; }
u64 orc_barrett128(u64 lo, u64 hi, u64 q) { return barrett_reduce_128(lo, hi, Modulus(q)); }
u64 orc_ntt_root(void *c, u64 i) { return static_cast<Context *>(c)->ntt(i).root; }
void orc_ntt_fwd(void *c, u64 i, u64 *a) { ntt_forward(a, static_cast<Context *>(c)->ntt(i)); }
void orc_ntt_inv(void *c, u64 i, u64 *a) { ntt_inverse(a, static_cast<Context *>(c)->ntt(i)); }
u32 orc_elt_from_step(void *c, int step)
{
    u32 e = 0;
    if (guard([&] { e = static_cast<Context *>(c)->elt_from_step(step); })) return 0;
    return e;
}
u64 orc_default_galois_elts(void *c, u32 *out)
{
    auto v = static_cast<Context *>(c)->default_galois_elts();
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(u32));
    return v.size();
}
u64 orc_naf(int value, int *out)
{
    auto v = naf(value);
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(int));
    return v.size();
}
void orc_apply_galois_ntt(void *c, const u64 *in, u64 nlimbs, u32 elt, u64 *out)
{
    apply_galois_ntt(*static_cast<Context *>(c), in, nlimbs, elt, out);
}

// ------------------------------------------------------------------ keys / encode / encrypt ---
int orc_secret_key(void *c, u64 seed, u64 *out)
{
    return guard([&] {
        auto sk = keygen_secret(*static_cast<Context *>(c), seed);
        std::memcpy(out, sk.data.data(), sk.data.size() * sizeof(u64));
    });
}
static SecretKey sk_view(const Context &ctx, const u64 *sk)
{
    SecretKey s;
    s.data.assign(sk, sk + ctx.K() * ctx.N());
    return s;
}
int orc_relin_key(void *c, const u64 *sk, u64 seed, u64 *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto k = gen_relin_key(ctx, sk_view(ctx, sk), seed);
        std::memcpy(out, k.owned.data(), k.owned.size() * sizeof(u64));
    });
}
int orc_galois_key(void *c, const u64 *sk, u32 elt, u64 seed, u64 *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto k = gen_galois_key(ctx, sk_view(ctx, sk), elt, seed);
        std::memcpy(out, k.owned.data(), k.owned.size() * sizeof(u64));
    });
}
int orc_encode(void *c, const double *re, const double *im, u64 n, double scale, u64 level, u64 *out)
{
    return guard([&] {
        std::vector<std::complex<double>> v(n);
        for (u64 i = 0; i < n; ++i) v[i] = {re[i], im ? im[i] : 0.0};
        auto pt = encode(*static_cast<Context *>(c), v, scale, level);
        std::memcpy(out, pt.data.data(), pt.data.size() * sizeof(u64));
    });
}
int orc_encode_scalar(void *c, double value, double scale, u64 level, u64 *out)
{
    return guard([&] {
        auto pt = encode_scalar(*static_cast<Context *>(c), value, scale, level);
        std::memcpy(out, pt.data.data(), pt.data.size() * sizeof(u64));
    });
}
int orc_decode(void *c, const u64 *pt, u64 level, double scale, double *re, double *im)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Plaintext p;
        p.level = level; p.scale = scale;
        p.data.assign(pt, pt + level * ctx.N());
        auto v = decode(ctx, p);
        for (std::size_t i = 0; i < v.size(); ++i) { re[i] = v[i].real(); if (im) im[i] = v[i].imag(); }
    });
}
int orc_encrypt(void *c, const u64 *sk, const u64 *pt, u64 level, double scale, u64 seed, u64 *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Plaintext p;
        p.level = level; p.scale = scale;
        p.data.assign(pt, pt + level * ctx.N());
        auto ct = encrypt_symmetric(ctx, sk_view(ctx, sk), p, seed);
        std::memcpy(out, ct.data.data(), ct.data.size() * sizeof(u64));
    });
}
// encode + encrypt `count` real slot vectors (row v of re: n values) on nthreads threads; ciphertext v uses
// seed0 + v.  Test-input factory for full-size matrices (4096 encrypted diagonals at cfg3).
int orc_encrypt_many(void *c, const u64 *sk, const double *re, u64 n, u64 count, double scale, u64 level, u64 seed0,
                     int nthreads, u64 *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        const SecretKey key = sk_view(ctx, sk);
        const u64 words = 2 * level * ctx.N();
        std::atomic<u64> next{0};
        std::vector<std::string> errs(std::max(1, nthreads));
        auto worker = [&](int tid) {
            try {
                for (u64 v; (v = next.fetch_add(1)) < count;) {
                    std::vector<std::complex<double>> vals(n);
                    for (u64 i = 0; i < n; ++i) vals[i] = {re[v * n + i], 0.0};
                    auto ct = encrypt_symmetric(ctx, key, encode(ctx, vals, scale, level), seed0 + v);
                    std::memcpy(out + v * words, ct.data.data(), words * sizeof(u64));
                }
            } catch (const std::exception &e) { errs[tid] = e.what(); }
        };
        std::vector<std::thread> th;
        for (int t = 0; t < std::max(1, nthreads); ++t) th.emplace_back(worker, t);
        for (auto &t : th) t.join();
        for (auto &e : errs)
            if (!e.empty()) throw std::invalid_argument(e);
    });
}
int orc_decrypt(void *c, const u64 *sk, const OrcCt *ct, u64 *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto pt = decrypt(ctx, sk_view(ctx, sk), in_ct(ctx, ct));
        std::memcpy(out, pt.data.data(), pt.data.size() * sizeof(u64));
    });
}

// ------------------------------------------------------------------ evaluator -----------------
#define ORC_UNARY(name, call)                                              \
    int name(void *c, OrcCt *a)                                            \
    {                                                                      \
        return guard([&] {                                                 \
            auto &ctx = *static_cast<Context *>(c);                        \
            Ciphertext x = in_ct(ctx, a);                                  \
            call;                                                          \
            out_ct(x, a);                                                  \
        });                                                                \
    }
ORC_UNARY(orc_negate, negate_inplace(ctx, x))
ORC_UNARY(orc_square, square_inplace(ctx, x))
ORC_UNARY(orc_rescale, rescale_to_next_inplace(ctx, x))
ORC_UNARY(orc_mod_switch, mod_switch_to_next_inplace(ctx, x))

#define ORC_BINARY(name, call)                                             \
    int name(void *c, OrcCt *a, const OrcCt *b)                            \
    {                                                                      \
        return guard([&] {                                                 \
            auto &ctx = *static_cast<Context *>(c);                        \
            Ciphertext x = in_ct(ctx, a), y = in_ct(ctx, b);               \
            call;                                                          \
            out_ct(x, a);                                                  \
        });                                                                \
    }
ORC_BINARY(orc_add, add_inplace(ctx, x, y))
ORC_BINARY(orc_sub, sub_inplace(ctx, x, y))
ORC_BINARY(orc_multiply, multiply_inplace(ctx, x, y))

static Plaintext pt_in(const Context &ctx, const u64 *pt, u64 level, double scale)
{
    Plaintext p;
    p.level = level; p.scale = scale;
    p.data.assign(pt, pt + level * ctx.N());
    return p;
}
#define ORC_PLAIN(name, call)                                                         \
    int name(void *c, OrcCt *a, const u64 *pt, u64 level, double scale)               \
    {                                                                                 \
        return guard([&] {                                                            \
            auto &ctx = *static_cast<Context *>(c);                                   \
            Ciphertext x = in_ct(ctx, a);                                             \
            Plaintext p = pt_in(ctx, pt, level, scale);                               \
            call;                                                                     \
            out_ct(x, a);                                                             \
        });                                                                           \
    }
ORC_PLAIN(orc_add_plain, add_plain_inplace(ctx, x, p))
ORC_PLAIN(orc_sub_plain, sub_plain_inplace(ctx, x, p))
ORC_PLAIN(orc_multiply_plain, multiply_plain_inplace(ctx, x, p))

int orc_relinearize(void *c, OrcCt *a, const u64 *rk)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Ciphertext x = in_ct(ctx, a);
        relinearize_inplace(ctx, x, view(rk));
        out_ct(x, a);
    });
}
int orc_switch_key(void *c, OrcCt *a, const u64 *target, const u64 *key)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Ciphertext x = in_ct(ctx, a);
        switch_key_inplace(ctx, x, target, view(key));
        out_ct(x, a);
    });
}
int orc_apply_galois(void *c, OrcCt *a, u32 elt, const u32 *elts, const u64 *const *keys, u64 nkeys)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Ciphertext x = in_ct(ctx, a);
        apply_galois_inplace(ctx, x, elt, gkeys(elts, keys, nkeys));
        out_ct(x, a);
    });
}
int orc_rotate(void *c, OrcCt *a, int steps, const u32 *elts, const u64 *const *keys, u64 nkeys)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Ciphertext x = in_ct(ctx, a);
        rotate_vector_inplace(ctx, x, steps, gkeys(elts, keys, nkeys));
        out_ct(x, a);
    });
}

int orc_sum_elems(void *c, OrcCt *a, u64 dim, const u32 *elts, const u64 *const *keys, u64 nkeys)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        Ciphertext x = in_ct(ctx, a);
        sum_elems_inplace(ctx, x, dim, gkeys(elts, keys, nkeys));
        out_ct(x, a);
    });
}

static std::vector<Ciphertext> in_many(const Context &ctx, const OrcCt *v, u64 n)
{
    std::vector<Ciphertext> r;
    r.reserve(n);
    for (u64 i = 0; i < n; ++i) r.push_back(in_ct(ctx, v + i));
    return r;
}
static std::vector<const Ciphertext *> ptrs(const std::vector<Ciphertext> &v)
{
    std::vector<const Ciphertext *> p;
    for (auto &c : v) p.push_back(&c);
    return p;
}

int orc_matmul_diag_col(void *c, const OrcCt *A, u64 n, const OrcCt *X, u64 p, const u64 *rk, const u32 *elts,
                        const u64 *const *keys, u64 nkeys, OrcCt *out, int nthreads, u64 j_begin, u64 j_end,
                        int finish)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto a = in_many(ctx, A, n), x = in_many(ctx, X, p);
        auto r = matmul_diag_col(ctx, ptrs(a), ptrs(x), view(rk), gkeys(elts, keys, nkeys), nthreads, j_begin,
                                 j_end, finish != 0);
        for (u64 i = 0; i < p; ++i) out_ct(r[i], out + i);
    });
}
int orc_matmul_diag_col_set(void *c, const OrcCt *A, const u64 *js, u64 nj, const OrcCt *X, u64 p, const u64 *rk,
                            const u32 *elts, const u64 *const *keys, u64 nkeys, OrcCt *out, int nthreads, int finish)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto a = in_many(ctx, A, nj), x = in_many(ctx, X, p);
        auto r = matmul_diag_col_set(ctx, ptrs(a), std::vector<std::size_t>(js, js + nj), ptrs(x), view(rk),
                                     gkeys(elts, keys, nkeys), nthreads, finish != 0);
        for (u64 i = 0; i < p; ++i) out_ct(r[i], out + i);
    });
}
// pts: nj plaintexts u64[level][N] back to back, all at `level` with `pscale`
int orc_matmul_diagpt_col_set(void *c, const u64 *pts, u64 level, double pscale, const u64 *js, u64 nj, const OrcCt *X,
                              u64 p, const u32 *elts, const u64 *const *keys, u64 nkeys, OrcCt *out, int nthreads,
                              int finish)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        std::vector<Plaintext> P;
        P.reserve(nj);
        for (u64 k = 0; k < nj; ++k) P.push_back(pt_in(ctx, pts + k * level * ctx.N(), level, pscale));
        std::vector<const Plaintext *> pp;
        for (auto &x : P) pp.push_back(&x);
        auto x = in_many(ctx, X, p);
        auto r = matmul_diagpt_col_set(ctx, pp, std::vector<std::size_t>(js, js + nj), ptrs(x),
                                       gkeys(elts, keys, nkeys), nthreads, finish != 0);
        for (u64 i = 0; i < p; ++i) out_ct(r[i], out + i);
    });
}
// CPU baseline (bench.py cpu_baseline leg): one full diag x col matvec (he_linalg.cpp:943-1006, relinearize +
// rescale) of n diagonals over X, timed with steady_clock around the call as the reference's Timer does
// (tic_toc.h:20-28).  The n diagonals cycle over the nA distinct ones given (every step is data-oblivious, so
// the time equals that of n distinct ciphertexts without n copies in memory).  j range [j_begin, j_end).
// out (may be NULL): the p results, so a benchmark run also checks the bits it timed (bench.py's CPU leg)
int orc_bench_matvec(void *c, const OrcCt *A, u64 nA, u64 n, const OrcCt *X, u64 p, const u64 *rk, const u32 *elts,
                     const u64 *const *keys, u64 nkeys, int nthreads, u64 j_begin, u64 j_end, int finish,
                     double *seconds, OrcCt *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto a = in_many(ctx, A, nA), x = in_many(ctx, X, p);
        std::vector<const Ciphertext *> diag(n);
        for (u64 j = 0; j < n; ++j) diag[j] = &a[j % nA];
        const auto gk = gkeys(elts, keys, nkeys);
        const auto t0 = std::chrono::steady_clock::now();
        auto r = matmul_diag_col(ctx, diag, ptrs(x), view(rk), gk, nthreads, j_begin, j_end, finish != 0);
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (out)
            for (u64 i = 0; i < p; ++i) out_ct(r[i], out + i);
    });
}
int orc_matmul_col_colT(void *c, const OrcCt *A, u64 n, const OrcCt *B, u64 p, const u64 *rk, const u32 *elts,
                        const u64 *const *keys, u64 nkeys, OrcCt *out, int nthreads)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto a = in_many(ctx, A, n), b = in_many(ctx, B, n);
        auto r = matmul_col_colT(ctx, ptrs(a), ptrs(b), p, view(rk), gkeys(elts, keys, nkeys), nthreads);
        for (u64 i = 0; i < p; ++i) out_ct(r[i], out + i);
    });
}
int orc_matrix_matmul(void *c, const OrcCt *A, u64 ar, u64 ac, int atr, const OrcCt *B, u64 br, u64 bc, int btr,
                      const u64 *rk, OrcCt *out)
{
    return guard([&] {
        auto &ctx = *static_cast<Context *>(c);
        auto a = in_many(ctx, A, ar * ac), b = in_many(ctx, B, br * bc);
        auto r = matrix_matmul(ctx, ptrs(a), ar, ac, atr != 0, ptrs(b), br, bc, btr != 0, view(rk));
        for (std::size_t i = 0; i < r.size(); ++i) out_ct(r[i], out + i);
    });
}

}  // extern "C"
