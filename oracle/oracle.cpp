// ORACLE — test infrastructure only (see oracle.hpp header).  CPU restatement of SEAL 4.1
// semantics for the reference's he_linalg / he_operators hot path.  Parity vs SEAL: unpinned
// (SURVEY.md §8(c)); pinned by the known-answer tests in tests/test_oracle_*.py.
#include "oracle.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <thread>

namespace oracle {

static constexpr double kPi = 3.14159265358979323846;

// =============================================================== modular arithmetic =========
Modulus::Modulus(u64 q) : value(q)
{
    if (q < 2) throw std::invalid_argument("modulus must be at least 2");
    // floor(2^128 / q): (2^128 - 1) / q is the same unless q | 2^128 (q is odd here, q >= 3)
    u128 all = ~(u128)0;
    u128 r = all / q;
    if (all % q == q - 1) r += 1;
    ratio0 = (u64)r;
    ratio1 = (u64)(r >> 64);
    bit_count = 64 - __builtin_clzll(q);
}

// SEAL util::barrett_reduce_128 (native/src/seal/util/uintarithsmallmod.h)
u64 barrett_reduce_128(u64 in0, u64 in1, const Modulus &m)
{
    u128 p;
    u64 carry = (u64)(((u128)in0 * m.ratio0) >> 64);            // round 1
    p = (u128)in0 * m.ratio1;
    u64 tmp1 = (u64)p + carry;
    u64 tmp3 = (u64)(p >> 64) + (tmp1 < carry);
    p = (u128)in1 * m.ratio0;                                     // round 2
    u64 lo = (u64)p;
    u64 sum = tmp1 + lo;
    carry = (u64)(p >> 64) + (sum < tmp1);
    tmp1 = in1 * m.ratio1 + tmp3 + carry;                         // quotient estimate
    u64 r = in0 - tmp1 * m.value;
    return r >= m.value ? r - m.value : r;
}

u64 pow_mod(u64 base, u64 e, u64 q)
{
    u64 r = 1 % q;
    base %= q;
    while (e) {
        if (e & 1) r = (u64)(((u128)r * base) % q);
        base = (u64)(((u128)base * base) % q);
        e >>= 1;
    }
    return r;
}

u64 inv_mod(u64 a, u64 q)
{
    // extended Euclid on signed 128-bit
    __int128 t = 0, nt = 1, r = q, nr = a % q;
    while (nr != 0) {
        __int128 qt = r / nr;
        __int128 tmp = t - qt * nt; t = nt; nt = tmp;
        tmp = r - qt * nr; r = nr; nr = tmp;
    }
    if (r != 1) throw std::invalid_argument("value is not invertible");
    if (t < 0) t += q;
    return (u64)t;
}

bool is_prime(u64 n)
{
    if (n < 2) return false;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : small) {
        if (n == p) return true;
        if (n % p == 0) return false;
    }
    u64 d = n - 1;
    int s = 0;
    while ((d & 1) == 0) { d >>= 1; ++s; }
    for (u64 a : small) {
        u64 x = pow_mod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int i = 1; i < s; ++i) {
            x = (u64)(((u128)x * x) % n);
            if (x == n - 1) { comp = false; break; }
        }
        if (comp) return false;
    }
    return true;
}

std::vector<u64> create_coeff_modulus(std::size_t N, const std::vector<int> &bit_sizes)
{
    if (N < 2 || (N & (N - 1))) throw std::invalid_argument("poly_modulus_degree is invalid");
    std::map<int, std::size_t> count;
    for (int b : bit_sizes) {
        if (b < 2 || b > 60) throw std::invalid_argument("bit_sizes is invalid");
        ++count[b];
    }
    const u64 factor = 2 * (u64)N;
    std::map<int, std::vector<u64>> table;
    for (auto &[b, c] : count) {
        std::vector<u64> found;
        u64 value = ((((u64)1) << b) - 1) / factor * factor + 1;  // SEAL util::get_primes
        const u64 lower = ((u64)1) << (b - 1);
        std::size_t need = c;
        while (need > 0 && value > lower) {
            if (is_prime(value)) { found.push_back(value); --need; }
            value -= factor;
        }
        if (need > 0) throw std::logic_error("failed to find enough qualifying primes");
        table[b] = std::move(found);
    }
    std::vector<u64> out;
    for (int b : bit_sizes) {  // CoeffModulus::Create: result.emplace_back(back()); pop_back()
        out.push_back(table[b].back());
        table[b].pop_back();
    }
    return out;
}

u64 minimal_primitive_root(u64 two_n, u64 q)
{
    if ((q - 1) % two_n) throw std::invalid_argument("modulus is not NTT-friendly");
    u64 g = 0;
    for (u64 x = 2; x < q; ++x) {
        u64 c = pow_mod(x, (q - 1) / two_n, q);
        if (pow_mod(c, two_n / 2, q) == q - 1) { g = c; break; }
    }
    if (!g) throw std::logic_error("no primitive root found");
    // every primitive 2N-th root is g^k, k odd; take the minimum (SEAL try_minimal_primitive_root)
    u64 g2 = (u64)(((u128)g * g) % q), cur = g, best = g;
    for (u64 k = 0; k < two_n / 2; ++k) {
        best = std::min(best, cur);
        cur = (u64)(((u128)cur * g2) % q);
    }
    return best;
}

// =============================================================== NTT =========================
static inline u64 mul_shoup_lazy(u64 x, u64 w, u64 wq, u64 q)
{
    u64 hi = (u64)(((u128)x * wq) >> 64);
    return x * w - hi * q;  // in [0, 2q)
}

NttTables::NttTables(int log_n_, const Modulus &m) : log_n(log_n_), n(std::size_t(1) << log_n_), mod(m)
{
    const u64 q = m.value;
    root = minimal_primitive_root(2 * (u64)n, q);
    const u64 iroot = inv_mod(root, q);
    psi.assign(n, 0); psi_shoup.assign(n, 0); ipsi.assign(n, 0); ipsi_shoup.assign(n, 0);
    u64 p = 1, ip = 1;
    for (std::size_t i = 0; i < n; ++i) {
        const u32 k = reverse_bits((u32)i, log_n);
        psi[k] = p; ipsi[k] = ip;
        p = (u64)(((u128)p * root) % q);
        ip = (u64)(((u128)ip * iroot) % q);
    }
    for (std::size_t k = 0; k < n; ++k) {
        psi_shoup[k] = shoup_quotient(psi[k], q);
        ipsi_shoup[k] = shoup_quotient(ipsi[k], q);
    }
    ninv = inv_mod((u64)n % q, q);
    ninv_shoup = shoup_quotient(ninv, q);
}

void ntt_forward(u64 *a, const NttTables &t)
{
    const u64 q = t.mod.value, two_q = 2 * q;
    const std::size_t n = t.n;
    std::size_t half = n;
    for (std::size_t m = 1; m < n; m <<= 1) {  // Cooley-Tukey, Harvey lazy butterflies in [0, 4q)
        half >>= 1;
        for (std::size_t i = 0; i < m; ++i) {
            const u64 w = t.psi[m + i], wq = t.psi_shoup[m + i];
            u64 *x = a + 2 * i * half, *y = x + half;
            for (std::size_t j = 0; j < half; ++j) {
                u64 u = x[j];
                if (u >= two_q) u -= two_q;
                const u64 v = mul_shoup_lazy(y[j], w, wq, q);
                x[j] = u + v;
                y[j] = u - v + two_q;
            }
        }
    }
    for (std::size_t j = 0; j < n; ++j) {
        u64 v = a[j];
        if (v >= two_q) v -= two_q;
        if (v >= q) v -= q;
        a[j] = v;
    }
}

void ntt_inverse(u64 *a, const NttTables &t)
{
    const u64 q = t.mod.value, two_q = 2 * q;
    const std::size_t n = t.n;
    for (std::size_t m = n >> 1; m >= 1; m >>= 1) {  // Gentleman-Sande, values in [0, 2q)
        const std::size_t half = n / (2 * m);
        for (std::size_t i = 0; i < m; ++i) {
            const u64 w = t.ipsi[m + i], wq = t.ipsi_shoup[m + i];
            u64 *x = a + 2 * i * half, *y = x + half;
            for (std::size_t j = 0; j < half; ++j) {
                const u64 X = x[j], Y = y[j];
                u64 s = X + Y;
                if (s >= two_q) s -= two_q;
                x[j] = s;
                y[j] = mul_shoup_lazy(X - Y + two_q, w, wq, q);
            }
        }
        if (m == 1) break;
    }
    for (std::size_t j = 0; j < n; ++j) {
        u64 v = mul_shoup_lazy(a[j], t.ninv, t.ninv_shoup, q);
        a[j] = v >= q ? v - q : v;
    }
}

// =============================================================== context =====================
Context::Context(std::size_t N, const std::vector<u64> &coeff_modulus) : N_(N)
{
    if (N < 8 || (N & (N - 1))) throw std::invalid_argument("poly_modulus_degree is invalid");
    if (coeff_modulus.size() < 2) throw std::invalid_argument("need at least one data prime and P");
    log_n_ = __builtin_ctzll(N);
    for (u64 q : coeff_modulus) {
        if (!is_prime(q) || (q - 1) % (2 * N) || (q >> 61)) throw std::invalid_argument("coeff_modulus is invalid");
        mod_.emplace_back(q);
        ntt_.emplace_back(log_n_, mod_.back());
    }
    const std::size_t L = mod_.size() - 1;
    const u64 P = mod_[L].value;
    for (std::size_t i = 0; i < L; ++i) {
        p_mod_.push_back(P % mod_[i].value);
        p_inv_.push_back(inv_mod(P % mod_[i].value, mod_[i].value));
    }
    qlast_inv_.assign(L + 1, {});
    for (std::size_t l = 2; l <= L; ++l)
        for (std::size_t i = 0; i + 1 < l; ++i)
            qlast_inv_[l].push_back(inv_mod(mod_[l - 1].value % mod_[i].value, mod_[i].value));
}

int Context::total_bits(std::size_t level) const
{
    int b = 0;
    for (std::size_t i = 0; i < level; ++i) b += mod_[i].bit_count;
    return b;
}

u32 Context::elt_from_step(int step) const
{
    const u32 n = (u32)N_, m = 2 * n;
    if (step == 0) return m - 1;
    const bool sign = step < 0;
    u32 pos = (u32)std::abs(step);
    if (pos >= (n >> 1)) throw std::invalid_argument("step count too large");
    pos &= m - 1;
    int s = sign ? (int)(n >> 1) - (int)pos : (int)pos;
    u64 elt = 1;
    while (s--) { elt *= 3; elt &= m - 1; }
    return (u32)elt;
}

std::vector<u32> Context::default_galois_elts() const
{
    const u32 m = (u32)(2 * N_);
    std::vector<u32> out{m - 1};
    u64 pos = 3, neg = inv_mod(3, m);
    for (int i = 0; i < log_n_ - 1; ++i) {
        out.push_back((u32)pos);
        pos = (pos * pos) & (m - 1);
        out.push_back((u32)neg);
        neg = (neg * neg) & (m - 1);
    }
    return out;
}

void Ciphertext::resize(std::size_t new_size, std::size_t N)
{
    data.resize(new_size * level * N, 0);
    size = new_size;
}

// =============================================================== sampling ====================
static u64 splitmix64(u64 &x)
{
    u64 z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
Rng::Rng(u64 seed) { for (auto &s : s_) s = splitmix64(seed); }
u64 Rng::next()
{
    auto rotl = [](u64 x, int k) { return (x << k) | (x >> (64 - k)); };
    const u64 r = rotl(s_[1] * 5, 7) * 9, t = s_[1] << 17;
    s_[2] ^= s_[0]; s_[3] ^= s_[1]; s_[1] ^= s_[2]; s_[0] ^= s_[3]; s_[2] ^= t; s_[3] = rotl(s_[3], 45);
    return r;
}
u64 Rng::uniform(u64 q)
{
    const u64 limit = ~(u64)0 - (~(u64)0 % q);
    for (;;) { u64 x = next(); if (x < limit) return x % q; }
}
int Rng::ternary() { return (int)uniform(3) - 1; }
long Rng::gaussian()
{
    for (;;) {
        const double u1 = ((next() >> 11) + 1) * 0x1.0p-53, u2 = (next() >> 11) * 0x1.0p-53;
        const double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(2 * kPi * u2) * 3.2;
        if (std::fabs(z) <= 19.2) return std::lround(z);
    }
}

static inline u64 signed_mod(long v, u64 q) { return v >= 0 ? (u64)v % q : (q - ((u64)(-v) % q)) % q; }

SecretKey keygen_secret(const Context &ctx, u64 seed)
{
    Rng rng(seed);
    const std::size_t N = ctx.N(), K = ctx.K();
    std::vector<int> s(N);
    for (auto &c : s) c = rng.ternary();
    SecretKey sk;
    sk.data.assign(K * N, 0);
    for (std::size_t i = 0; i < K; ++i) {
        u64 *limb = sk.data.data() + i * N;
        for (std::size_t t = 0; t < N; ++t) limb[t] = signed_mod(s[t], ctx.mod(i).value);
        ntt_forward(limb, ctx.ntt(i));
    }
    return sk;
}

// (c0, c1) = (-a*s + e, a) over the first `nlimbs` primes of `primes` (indices into ctx moduli)
static void encrypt_zero_sym(const Context &ctx, const SecretKey &sk, const std::vector<std::size_t> &primes,
                             Rng &rng, u64 *c0, u64 *c1)
{
    const std::size_t N = ctx.N();
    std::vector<long> e(N);
    for (auto &x : e) x = rng.gaussian();
    for (std::size_t li = 0; li < primes.size(); ++li) {
        const std::size_t pi = primes[li];
        const Modulus &m = ctx.mod(pi);
        u64 *a = c1 + li * N, *b = c0 + li * N;
        const u64 *s = sk.data.data() + pi * N;
        for (std::size_t t = 0; t < N; ++t) a[t] = rng.uniform(m.value);
        std::vector<u64> el(N);
        for (std::size_t t = 0; t < N; ++t) el[t] = signed_mod(e[t], m.value);
        ntt_forward(el.data(), ctx.ntt(pi));
        for (std::size_t t = 0; t < N; ++t) b[t] = sub_mod(el[t], mul_mod(a[t], s[t], m), m.value);
    }
}

KSwitchKey gen_kswitch_key(const Context &ctx, const SecretKey &sk, const u64 *new_key, u64 seed)
{
    const std::size_t N = ctx.N(), K = ctx.K(), L = ctx.L();
    Rng rng(seed);
    KSwitchKey key;
    key.owned.assign(L * 2 * K * N, 0);
    std::vector<std::size_t> all(K);
    for (std::size_t i = 0; i < K; ++i) all[i] = i;
    for (std::size_t J = 0; J < L; ++J) {
        u64 *c0 = key.owned.data() + (J * 2 + 0) * K * N;
        u64 *c1 = key.owned.data() + (J * 2 + 1) * K * N;
        encrypt_zero_sym(ctx, sk, all, rng, c0, c1);
        const Modulus &m = ctx.mod(J);
        const u64 factor = ctx.p_mod(J);
        for (std::size_t t = 0; t < N; ++t)
            c0[J * N + t] = add_mod(c0[J * N + t], mul_mod(new_key[J * N + t], factor, m), m.value);
    }
    key.data = key.owned.data();
    return key;
}

KSwitchKey gen_relin_key(const Context &ctx, const SecretKey &sk, u64 seed)
{
    const std::size_t N = ctx.N(), K = ctx.K();
    std::vector<u64> s2(K * N);
    for (std::size_t i = 0; i < K; ++i)
        for (std::size_t t = 0; t < N; ++t)
            s2[i * N + t] = mul_mod(sk.data[i * N + t], sk.data[i * N + t], ctx.mod(i));
    return gen_kswitch_key(ctx, sk, s2.data(), seed);
}

KSwitchKey gen_galois_key(const Context &ctx, const SecretKey &sk, u32 elt, u64 seed)
{
    std::vector<u64> rot(ctx.K() * ctx.N());
    apply_galois_ntt(ctx, sk.data.data(), ctx.K(), elt, rot.data());
    return gen_kswitch_key(ctx, sk, rot.data(), seed);
}

// =============================================================== CKKS encoder ================
using cd = std::complex<double>;

static void fft(std::vector<cd> &a, int sign)  // a_t <- sum_k a_k exp(sign * 2 pi i t k / n)
{
    const std::size_t n = a.size();
    const int logn = __builtin_ctzll(n);
    for (std::size_t i = 0; i < n; ++i) {
        const std::size_t j = reverse_bits((u32)i, logn);
        if (i < j) std::swap(a[i], a[j]);
    }
    for (std::size_t len = 2; len <= n; len <<= 1) {
        const double ang = sign * 2 * kPi / (double)len;
        for (std::size_t i = 0; i < n; i += len)
            for (std::size_t j = 0; j < len / 2; ++j) {
                const cd w = std::polar(1.0, ang * (double)j);
                const cd u = a[i + j], v = a[i + j + len / 2] * w;
                a[i + j] = u + v;
                a[i + j + len / 2] = u - v;
            }
    }
}

// ---- SEAL 4.1 CKKSEncoder::encode_internal, restated operation for operation.  Each step below was checked
// against the reference's own build/demo (SEAL statically linked), read as data, never run:
//   * CKKSEncoder::CKKSEncoder (0x6b570): matrix_reps_index_map_[i] = bitrev((3^i mod 2N - 1) / 2, logN),
//     [N/2 + i] = bitrev((2N - 3^i mod 2N - 1) / 2, logN); inv_root_powers_[i] = conj(get_root(bitrev(i - 1, logN)
//     + 1)), i = 1 .. N - 1 (the pxor on the imaginary part at 0x6bf63);
//   * ComplexRoots::ComplexRoots(2N) (0xad280): roots_[i] = (cos t, sin t), t = (i * 6.283185307179586) / 2N, for
//     i <= 2N / 8, with glibc cos and sin called separately (0xad438, 0xad448);
//   * ComplexRoots::get_root (0xad500): the 8-fold symmetry below;
//   * encode_internal<double> (0x513b0) is instantiated in the reference's own translation units, built without -O
//     and without FMA (no vfmadd anywhere in build/demo): scatter, DWTHandler::transform_from_rev (0x13a6a) with
//     fix = scale / N, then round / signbit / barrett_reduce_64 or _128 / negate_uint_mod per prime, then the NTT;
//   * complex * complex there is a call to libgcc's __muldc3 (0x1134f): (ac - bd, ad + bc), each product rounded;
//     complex * double multiplies both parts (0xf2c1).
static cd seal_complex_root(std::size_t m, const std::vector<cd> &roots, std::size_t index)
{
    index &= m - 1;
    if (index <= m / 8) return roots[index];
    if (index <= m / 4) {  // mirror: swap the parts
        const cd a = roots[m / 4 - index];
        return cd(a.imag(), a.real());
    }
    if (index <= m / 2) {  // -conj(x) = (-re, im)
        const cd a = seal_complex_root(m, roots, m / 2 - index);
        return cd(-a.real(), a.imag());
    }
    if (index <= 3 * m / 4) {
        const cd a = seal_complex_root(m, roots, index - m / 2);
        return cd(-a.real(), -a.imag());
    }
    const cd a = seal_complex_root(m, roots, m - index);
    return cd(a.real(), -a.imag());
}

void ckks_encoder_tables(std::size_t N, std::vector<u32> &map, std::vector<cd> &inv_roots)
{
    const int logn = __builtin_ctzll(N);
    const u64 m = 2 * N, slots = N / 2;
    map.assign(N, 0);
    u64 pos = 1;
    for (u64 i = 0; i < slots; ++i) {
        map[i] = reverse_bits((u32)((pos - 1) >> 1), logn);
        map[slots | i] = reverse_bits((u32)((m - pos - 1) >> 1), logn);
        pos = (pos * 3) & (m - 1);
    }
    // cos and sin as two separate glibc calls (never fused into sincos), as the reference binary calls them
    double (*volatile vcos)(double) = std::cos;
    double (*volatile vsin)(double) = std::sin;
    std::vector<cd> roots(m / 8 + 1);
    for (u64 i = 0; i <= m / 8; ++i) {
        const double t = ((double)i * 6.283185307179586) / (double)m;
        roots[i] = cd(vcos(t), vsin(t));
    }
    inv_roots.assign(N, cd(0, 0));
    for (u64 i = 1; i < N; ++i) {
        const cd r = seal_complex_root(m, roots, (std::size_t)reverse_bits((u32)(i - 1), logn) + 1);
        inv_roots[i] = cd(r.real(), -r.imag());
    }
}

// libgcc __muldc3 for finite operands: (a + bi)(c + di) = (ac - bd) + (ad + bc) i, every product rounded
static inline cd cmul(const cd &x, const cd &w)
{
    const double ac = x.real() * w.real(), bd = x.imag() * w.imag();
    const double ad = x.real() * w.imag(), bc = x.imag() * w.real();
    return cd(ac - bd, ad + bc);
}

// DWTHandler<complex<double>, complex<double>, double>::transform_from_rev(values, log_n, roots, scalar)
static void seal_transform_from_rev(cd *values, int log_n, const cd *roots, const double *scalar)
{
    const std::size_t n = std::size_t(1) << log_n;
    std::size_t gap = 1, m = n >> 1;
    const cd *r = roots;
    for (; m > 1; m >>= 1) {
        std::size_t offset = 0;
        for (std::size_t i = 0; i < m; i++) {
            const cd w = *++r;
            cd *x = values + offset, *y = x + gap;
            for (std::size_t j = 0; j < gap; j++) {
                const cd u = *x, v = *y;
                *x++ = cd(u.real() + v.real(), u.imag() + v.imag());
                *y++ = cmul(cd(u.real() - v.real(), u.imag() - v.imag()), w);
            }
            offset += gap << 1;
        }
        gap <<= 1;
    }
    const cd w = *++r;
    cd *x = values, *y = x + gap;
    if (scalar) {
        const double s = *scalar;
        const cd sw(w.real() * s, w.imag() * s);  // mul_root_scalar
        for (std::size_t j = 0; j < gap; j++) {
            const cd u = *x, v = *y;
            *x++ = cd((u.real() + v.real()) * s, (u.imag() + v.imag()) * s);  // mul_scalar(add(u, v), s)
            *y++ = cmul(cd(u.real() - v.real(), u.imag() - v.imag()), sw);
        }
    } else {
        for (std::size_t j = 0; j < gap; j++) {
            const cd u = *x, v = *y;
            *x++ = cd(u.real() + v.real(), u.imag() + v.imag());
            *y++ = cmul(cd(u.real() - v.real(), u.imag() - v.imag()), w);
        }
    }
}

// |round(v)| mod q for any finite integer-valued double a >= 0, exactly: SEAL's three decompositions (64-bit,
// 128-bit fmod / divide split, the multi-word loop) all give the exact integer, so its residue is all that matters
u64 encode_residue(double a, u64 q)
{
    if (a < 0x1.0p64) return (u64)a % q;
    int e = 0;
    const double f = std::frexp(a, &e);           // a = f 2^e, 0.5 <= f < 1
    const u64 mant = (u64)std::ldexp(f, 53);      // a = mant 2^(e - 53), e - 53 > 0 here
    u64 r = mant % q, pw = 2 % q;
    for (int k = e - 53; k > 0; k >>= 1) {        // r *= 2^(e - 53) mod q
        if (k & 1) r = (u64)((u128)r * pw % q);
        pw = (u64)((u128)pw * pw % q);
    }
    return r;
}

Plaintext encode(const Context &ctx, const std::vector<cd> &values, double scale, std::size_t level)
{
    const std::size_t N = ctx.N(), slots = N / 2;
    if (values.size() > slots) throw std::invalid_argument("values has invalid size");
    if (level < 1 || level > ctx.L()) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    if (scale <= 0 || (int)std::log2(scale) >= ctx.total_bits(level)) throw std::invalid_argument("scale out of bounds");
    std::vector<u32> map;
    std::vector<cd> inv_roots;
    ckks_encoder_tables(N, map, inv_roots);
    std::vector<cd> v(N, cd(0, 0));
    for (std::size_t i = 0; i < values.size(); ++i) {
        v[map[i]] = values[i];
        v[map[i + slots]] = cd(values[i].real(), -values[i].imag());  // std::conj
    }
    const double fix = scale / (double)N;
    seal_transform_from_rev(v.data(), __builtin_ctzll(N), inv_roots.data(), &fix);
    double max_coeff = 0;  // over the unrounded real parts, as SEAL
    for (std::size_t k = 0; k < N; ++k) {
        // a NaN or infinite coefficient (from a non-finite input) is rejected as too large, as the GPU encoder
        // rejects it; SEAL's std::max would skip a NaN and then cast it to an integer (undefined behaviour)
        if (!std::isfinite(v[k].real())) throw std::invalid_argument("encoded values are too large");
        max_coeff = std::max(max_coeff, std::fabs(v[k].real()));
    }
    const int max_bits = (int)std::ceil(std::log2(std::max(max_coeff, 1.0))) + 1;
    if (max_bits >= ctx.total_bits(level)) throw std::invalid_argument("encoded values are too large");
    Plaintext pt;
    pt.level = level;
    pt.scale = scale;
    pt.data.assign(level * N, 0);
    for (std::size_t k = 0; k < N; ++k) {
        const double c = std::round(v[k].real());
        const bool neg = std::signbit(c);
        const double a = std::fabs(c);
        for (std::size_t i = 0; i < level; ++i) {
            const u64 q = ctx.mod(i).value, r = encode_residue(a, q);
            pt.data[i * N + k] = neg && r ? q - r : r;  // negate_uint_mod
        }
    }
    for (std::size_t i = 0; i < level; ++i) ntt_forward(pt.data.data() + i * N, ctx.ntt(i));
    return pt;
}

// CKKSEncoder::encode(double value, parms_id, scale, destination): SEAL 4.1 encode_internal(double, ...) restated
// in its own three cases (a different route to the exact residue than encode_residue's mantissa / exponent split,
// so the GPU's scalar encoder is checked against an independent reduction):
//   coeff_bit_count = int(log2 |value scale|) + 2 <= 64:  (u64) |round| mod q       (barrett_reduce_64)
//                                                 <= 128: {fmod(c, 2^64), c / 2^64} mod q  (barrett_reduce_128)
//   otherwise: base-2^64 digits by repeated fmod / division, then reduced mod q    (RNSBase::decompose)
// negated for a negative value (negate_uint_mod), and written to every coefficient of the NTT-form limb (fill_n):
// the NTT of a constant polynomial.  A non-finite value is rejected as too large (SEAL would cast it to int).
Plaintext encode_scalar(const Context &ctx, double value, double scale, std::size_t level)
{
    if (level < 1 || level > ctx.L()) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    const int total = ctx.total_bits(level);
    if (scale <= 0 || (int)std::log2(scale) >= total) throw std::invalid_argument("scale out of bounds");
    value *= scale;
    if (!std::isfinite(value)) throw std::invalid_argument("encoded value is too large");
    const int bits = value == 0.0 ? INT32_MIN + 2 : (int)std::log2(std::fabs(value)) + 2;
    if (bits >= total) throw std::invalid_argument("encoded value is too large");
    const double two64 = std::pow(2.0, 64);
    double cd = std::round(value);
    const bool neg = std::signbit(cd);
    cd = std::fabs(cd);
    Plaintext pt;
    pt.level = level;
    pt.scale = scale;
    pt.data.assign(level * ctx.N(), 0);
    for (std::size_t j = 0; j < level; ++j) {
        const u64 q = ctx.mod(j).value;
        u64 r;
        if (bits <= 64) {
            r = (u64)cd % q;
        } else if (bits <= 128) {
            const u128 w = ((u128)(u64)(cd / two64) << 64) | (u64)std::fmod(cd, two64);
            r = (u64)(w % q);
        } else {
            std::vector<u64> digits;
            for (double t = cd; t >= 1; t /= two64) digits.push_back((u64)std::fmod(t, two64));
            r = 0;
            for (std::size_t k = digits.size(); k-- > 0;) r = (u64)((((u128)r << 64) | digits[k]) % q);
        }
        if (neg && r) r = q - r;
        std::fill(pt.data.begin() + j * ctx.N(), pt.data.begin() + (j + 1) * ctx.N(), r);
    }
    return pt;
}

// little-endian multi-word unsigned helpers for CRT composition
using Big = std::vector<u64>;
static void big_mul_add(Big &acc, const Big &x, u64 s)  // acc += x * s
{
    u64 carry = 0;
    for (std::size_t i = 0; i < acc.size(); ++i) {
        const u128 t = (u128)(i < x.size() ? x[i] : 0) * s + acc[i] + carry;
        acc[i] = (u64)t;
        carry = (u64)(t >> 64);
    }
}
static int big_cmp(const Big &a, const Big &b)
{
    for (std::size_t i = a.size(); i-- > 0;) {
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    }
    return 0;
}
static void big_sub(Big &a, const Big &b)  // a -= b (a >= b)
{
    u64 borrow = 0;
    for (std::size_t i = 0; i < a.size(); ++i) {
        const u128 t = (u128)a[i] - b[i] - borrow;
        a[i] = (u64)t;
        borrow = (t >> 64) ? 1 : 0;
    }
}
static double big_to_double(const Big &a)
{
    double d = 0;
    for (std::size_t i = a.size(); i-- > 0;) d = d * 0x1.0p64 + (double)a[i];
    return d;
}

std::vector<cd> decode(const Context &ctx, const Plaintext &pt)
{
    const std::size_t N = ctx.N(), l = pt.level, W = l + 2;
    const u64 m = 2 * N;
    std::vector<u64> limbs(pt.data);
    for (std::size_t i = 0; i < l; ++i) ntt_inverse(limbs.data() + i * N, ctx.ntt(i));
    Big Q(W, 0);
    Q[0] = 1;
    for (std::size_t i = 0; i < l; ++i) { Big t(W, 0); big_mul_add(t, Q, ctx.mod(i).value); Q = t; }
    std::vector<Big> Qi(l);
    std::vector<u64> inv(l);
    for (std::size_t i = 0; i < l; ++i) {
        Big t(W, 0); t[0] = 1;
        u64 qi_mod = 1;
        for (std::size_t j = 0; j < l; ++j) {
            if (j == i) continue;
            Big u(W, 0); big_mul_add(u, t, ctx.mod(j).value); t = u;
            qi_mod = mul_mod(qi_mod, ctx.mod(j).value % ctx.mod(i).value, ctx.mod(i));
        }
        Qi[i] = t;
        inv[i] = inv_mod(qi_mod, ctx.mod(i).value);
    }
    Big halfQ(W, 0);
    { u64 carry = 0; for (std::size_t i = W; i-- > 0;) { halfQ[i] = (Q[i] >> 1) | carry; carry = Q[i] << 63; } }
    std::vector<cd> u(N);
    for (std::size_t k = 0; k < N; ++k) {
        Big acc(W, 0);
        for (std::size_t i = 0; i < l; ++i)
            big_mul_add(acc, Qi[i], mul_mod(limbs[i * N + k], inv[i], ctx.mod(i)));
        while (big_cmp(acc, Q) >= 0) big_sub(acc, Q);
        double c;
        if (big_cmp(acc, halfQ) > 0) { Big t = Q; big_sub(t, acc); c = -big_to_double(t); }
        else c = big_to_double(acc);
        u[k] = std::polar(1.0, kPi * (double)k / (double)N) * (c / pt.scale);
    }
    fft(u, +1);
    std::vector<cd> out(N / 2);
    u64 pos = 1;
    for (std::size_t i = 0; i < N / 2; ++i) {
        out[i] = u[(pos - 1) >> 1];
        pos = (pos * 3) & (m - 1);
    }
    return out;
}

Ciphertext encrypt_symmetric(const Context &ctx, const SecretKey &sk, const Plaintext &pt, u64 seed)
{
    const std::size_t N = ctx.N(), l = pt.level;
    Rng rng(seed);
    Ciphertext ct;
    ct.size = 2; ct.level = l; ct.scale = pt.scale;
    ct.data.assign(2 * l * N, 0);
    std::vector<std::size_t> primes(l);
    for (std::size_t i = 0; i < l; ++i) primes[i] = i;
    encrypt_zero_sym(ctx, sk, primes, rng, ct.poly(0, N), ct.poly(1, N));
    for (std::size_t i = 0; i < l; ++i)
        for (std::size_t t = 0; t < N; ++t)
            ct.data[i * N + t] = add_mod(ct.data[i * N + t], pt.data[i * N + t], ctx.mod(i).value);
    return ct;
}

Plaintext decrypt(const Context &ctx, const SecretKey &sk, const Ciphertext &ct)
{
    const std::size_t N = ctx.N(), l = ct.level;
    Plaintext pt;
    pt.level = l; pt.scale = ct.scale;
    pt.data.assign(l * N, 0);
    for (std::size_t i = 0; i < l; ++i) {
        const Modulus &m = ctx.mod(i);
        const u64 *s = sk.data.data() + i * N;
        for (std::size_t t = 0; t < N; ++t) {
            u64 acc = 0, sp = 1;  // Horner-free: sum_k c_k s^k
            for (std::size_t k = 0; k < ct.size; ++k) {
                acc = add_mod(acc, mul_mod(ct.poly(k, N)[i * N + t], sp, m), m.value);
                sp = mul_mod(sp, s[t], m);
            }
            pt.data[i * N + t] = acc;
        }
    }
    return pt;
}

// =============================================================== evaluator ===================
static bool are_close(double a, double b)  // SEAL util::are_close
{
    const double sf = std::max({std::fabs(a), std::fabs(b), 1.0});
    return std::fabs(a - b) < std::numeric_limits<double>::epsilon() * sf;
}
static bool scale_ok(const Context &ctx, double scale, std::size_t level)  // is_scale_within_bounds
{
    return !(scale <= 0 || (int)std::log2(scale) >= ctx.total_bits(level));
}
static void check_ct(const Context &ctx, const Ciphertext &a)
{
    if (a.level < 1 || a.level > ctx.L() || a.size < 2 || a.data.size() != a.size * a.level * ctx.N())
        throw std::invalid_argument("encrypted is not valid for encryption parameters");
}

void negate_inplace(const Context &ctx, Ciphertext &a)
{
    check_ct(ctx, a);
    const std::size_t N = ctx.N();
    for (std::size_t k = 0; k < a.size; ++k)
        for (std::size_t i = 0; i < a.level; ++i) {
            const u64 q = ctx.mod(i).value;
            u64 *p = a.poly(k, N) + i * N;
            for (std::size_t t = 0; t < N; ++t) p[t] = p[t] ? q - p[t] : 0;
        }
}

static void add_sub(const Context &ctx, Ciphertext &a, const Ciphertext &b, bool sub)
{
    check_ct(ctx, a); check_ct(ctx, b);
    if (a.level != b.level) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
    if (!are_close(a.scale, b.scale)) throw std::invalid_argument("scale mismatch");
    const std::size_t N = ctx.N(), mn = std::min(a.size, b.size), mx = std::max(a.size, b.size);
    const std::size_t old = a.size;
    a.resize(mx, N);
    for (std::size_t k = 0; k < mx; ++k)
        for (std::size_t i = 0; i < a.level; ++i) {
            const u64 q = ctx.mod(i).value;
            u64 *x = a.poly(k, N) + i * N;
            if (k < mn) {
                const u64 *y = b.poly(k, N) + i * N;
                for (std::size_t t = 0; t < N; ++t) x[t] = sub ? sub_mod(x[t], y[t], q) : add_mod(x[t], y[t], q);
            } else if (k >= old) {  // copy (or negate) the extra polys of b
                const u64 *y = b.poly(k, N) + i * N;
                for (std::size_t t = 0; t < N; ++t) x[t] = sub ? (y[t] ? q - y[t] : 0) : y[t];
            }
        }
}
void add_inplace(const Context &ctx, Ciphertext &a, const Ciphertext &b) { add_sub(ctx, a, b, false); }
void sub_inplace(const Context &ctx, Ciphertext &a, const Ciphertext &b) { add_sub(ctx, a, b, true); }

static void plain_addsub(const Context &ctx, Ciphertext &a, const Plaintext &p, bool sub)
{
    check_ct(ctx, a);
    if (a.level != p.level) throw std::invalid_argument("encrypted and plain parameter mismatch");
    if (!are_close(a.scale, p.scale)) throw std::invalid_argument("scale mismatch");
    const std::size_t N = ctx.N();
    for (std::size_t i = 0; i < a.level; ++i) {
        const u64 q = ctx.mod(i).value;
        u64 *x = a.poly(0, N) + i * N;
        const u64 *y = p.data.data() + i * N;
        for (std::size_t t = 0; t < N; ++t) x[t] = sub ? sub_mod(x[t], y[t], q) : add_mod(x[t], y[t], q);
    }
}
void add_plain_inplace(const Context &ctx, Ciphertext &a, const Plaintext &p) { plain_addsub(ctx, a, p, false); }
void sub_plain_inplace(const Context &ctx, Ciphertext &a, const Plaintext &p) { plain_addsub(ctx, a, p, true); }

void multiply_inplace(const Context &ctx, Ciphertext &a, const Ciphertext &b)
{
    check_ct(ctx, a); check_ct(ctx, b);
    if (a.level != b.level) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
    const double new_scale = a.scale * b.scale;
    if (!scale_ok(ctx, new_scale, a.level)) throw std::invalid_argument("scale out of bounds");
    const std::size_t N = ctx.N(), l = a.level, ds = a.size + b.size - 1;
    Ciphertext r;
    r.size = ds; r.level = l; r.scale = new_scale;
    r.data.assign(ds * l * N, 0);
    for (std::size_t i = 0; i < l; ++i) {  // ckks_multiply: c_k = sum_{x+y=k} a_x * b_y (dyadic)
        const Modulus &m = ctx.mod(i);
        for (std::size_t x = 0; x < a.size; ++x)
            for (std::size_t y = 0; y < b.size; ++y) {
                const u64 *pa = a.poly(x, N) + i * N, *pb = b.poly(y, N) + i * N;
                u64 *pr = r.poly(x + y, N) + i * N;
                for (std::size_t t = 0; t < N; ++t) pr[t] = add_mod(pr[t], mul_mod(pa[t], pb[t], m), m.value);
            }
    }
    a = std::move(r);
}

void square_inplace(const Context &ctx, Ciphertext &a)
{
    Ciphertext b = a;
    multiply_inplace(ctx, a, b);
}

void multiply_plain_inplace(const Context &ctx, Ciphertext &a, const Plaintext &p)
{
    check_ct(ctx, a);
    if (a.level != p.level) throw std::invalid_argument("encrypted_ntt and plain_ntt parameter mismatch");
    const double new_scale = a.scale * p.scale;
    if (!scale_ok(ctx, new_scale, a.level)) throw std::invalid_argument("scale out of bounds");
    const std::size_t N = ctx.N();
    for (std::size_t k = 0; k < a.size; ++k)
        for (std::size_t i = 0; i < a.level; ++i) {
            const Modulus &m = ctx.mod(i);
            u64 *x = a.poly(k, N) + i * N;
            const u64 *y = p.data.data() + i * N;
            for (std::size_t t = 0; t < N; ++t) x[t] = mul_mod(x[t], y[t], m);
        }
    a.scale = new_scale;
}

// y (coefficient form mod `last`, canonical) -> per target prime i: NTT_i( (y + h) mod last - h  mod q_i )
// where h = last >> 1.  Returns the NTT-form rounding correction for divide-and-round by `last`.
static void round_correction(const Context &ctx, const u64 *y_coeff, std::size_t last_idx, std::size_t i, u64 *out)
{
    const std::size_t N = ctx.N();
    const u64 last = ctx.mod(last_idx).value, h = last >> 1;
    const Modulus &mi = ctx.mod(i);
    const u64 fix = mi.value - barrett_reduce_64(h, mi);
    for (std::size_t t = 0; t < N; ++t) {
        u64 v = y_coeff[t] + h;                     // (y + h) mod last
        if (v >= last) v -= last;
        v = barrett_reduce_64(v, mi) + fix;        // ((y+h) mod last) mod q_i  - h mod q_i
        out[t] = v >= mi.value ? v - mi.value : v;
    }
    ntt_forward(out, ctx.ntt(i));
}

void switch_key_inplace(const Context &ctx, Ciphertext &a, const u64 *target, const KSwitchKey &key)
{
    const std::size_t N = ctx.N(), l = a.level, K = ctx.K();
    // (1) copy target, INTT its l limbs
    std::vector<u64> coeff(target, target + l * N);
    for (std::size_t J = 0; J < l; ++J) ntt_inverse(coeff.data() + J * N, ctx.ntt(J));
    // (2)+(3) per target modulus I in {0..l-1, P}: sum_J NTT_I(digit_J mod q_I) * key[J][k][I]
    std::vector<u64> prod(2 * (l + 1) * N);  // [k][I][N], I == l is the special prime
    std::vector<u64> tmp(N);
    std::vector<u128> acc0(N), acc1(N);
    for (std::size_t I = 0; I <= l; ++I) {
        const std::size_t ki = (I == l) ? K - 1 : I;
        const Modulus &mI = ctx.mod(ki);
        std::fill(acc0.begin(), acc0.end(), 0);
        std::fill(acc1.begin(), acc1.end(), 0);
        for (std::size_t J = 0; J < l; ++J) {
            const u64 *op;
            if (I == J) op = target + J * N;  // NTT-form input reused (bit-neutral)
            else {
                const u64 *src = coeff.data() + J * N;
                for (std::size_t t = 0; t < N; ++t) tmp[t] = barrett_reduce_64(src[t], mI);
                ntt_forward(tmp.data(), ctx.ntt(ki));
                op = tmp.data();
            }
            const u64 *k0 = key.at(J, 0, ki, ctx), *k1 = key.at(J, 1, ki, ctx);
            for (std::size_t t = 0; t < N; ++t) {  // 128-bit lazy accumulation (exact for l < 256)
                acc0[t] += (u128)op[t] * k0[t];
                acc1[t] += (u128)op[t] * k1[t];
            }
        }
        u64 *p0 = prod.data() + (0 * (l + 1) + I) * N, *p1 = prod.data() + (1 * (l + 1) + I) * N;
        for (std::size_t t = 0; t < N; ++t) {
            p0[t] = barrett_reduce_128((u64)acc0[t], (u64)(acc0[t] >> 64), mI);
            p1[t] = barrett_reduce_128((u64)acc1[t], (u64)(acc1[t] >> 64), mI);
        }
    }
    // (4) mod-down by P with rounding, add into ct[k]
    for (std::size_t k = 0; k < 2; ++k) {
        u64 *y = prod.data() + (k * (l + 1) + l) * N;
        ntt_inverse(y, ctx.ntt(K - 1));
        for (std::size_t i = 0; i < l; ++i) {
            const Modulus &mi = ctx.mod(i);
            round_correction(ctx, y, K - 1, i, tmp.data());
            const u64 *x = prod.data() + (k * (l + 1) + i) * N;
            u64 *c = a.poly(k, N) + i * N;
            const u64 pinv = ctx.p_inv(i);
            for (std::size_t t = 0; t < N; ++t)
                c[t] = add_mod(c[t], mul_mod(sub_mod(x[t], tmp[t], mi.value), pinv, mi), mi.value);
        }
    }
}

void relinearize_inplace(const Context &ctx, Ciphertext &a, const KSwitchKey &rk)
{
    check_ct(ctx, a);
    if (a.size == 2) return;
    if (a.size > 3) throw std::invalid_argument("not enough relinearization keys");
    const std::size_t N = ctx.N();
    std::vector<u64> target(a.poly(2, N), a.poly(2, N) + a.level * N);
    switch_key_inplace(ctx, a, target.data(), rk);
    a.resize(2, N);
}

static void drop_last_limb(const Context &ctx, Ciphertext &a)
{
    const std::size_t N = ctx.N(), l = a.level;
    std::vector<u64> d(a.size * (l - 1) * N);
    for (std::size_t k = 0; k < a.size; ++k)
        std::memcpy(d.data() + k * (l - 1) * N, a.data.data() + k * l * N, (l - 1) * N * sizeof(u64));
    a.data = std::move(d);
    a.level = l - 1;
}

void rescale_to_next_inplace(const Context &ctx, Ciphertext &a)
{
    check_ct(ctx, a);
    if (a.level == 1) throw std::invalid_argument("end of modulus switching chain reached");
    const std::size_t N = ctx.N(), l = a.level;
    std::vector<u64> y(N), corr(N);
    for (std::size_t k = 0; k < a.size; ++k) {  // RNSTool::divide_and_round_q_last_ntt_inplace
        u64 *poly = a.poly(k, N);
        std::memcpy(y.data(), poly + (l - 1) * N, N * sizeof(u64));
        ntt_inverse(y.data(), ctx.ntt(l - 1));
        for (std::size_t i = 0; i + 1 < l; ++i) {
            const Modulus &mi = ctx.mod(i);
            round_correction(ctx, y.data(), l - 1, i, corr.data());
            u64 *c = poly + i * N;
            const u64 inv = ctx.qlast_inv(l, i);
            for (std::size_t t = 0; t < N; ++t) c[t] = mul_mod(sub_mod(c[t], corr[t], mi.value), inv, mi);
        }
    }
    const double q_last = (double)ctx.mod(l - 1).value;
    drop_last_limb(ctx, a);
    a.scale = a.scale / q_last;
}

void mod_switch_to_next_inplace(const Context &ctx, Ciphertext &a)
{
    check_ct(ctx, a);
    if (a.level == 1) throw std::invalid_argument("end of modulus switching chain reached");
    if (!scale_ok(ctx, a.scale, a.level - 1)) throw std::invalid_argument("scale out of bounds");
    drop_last_limb(ctx, a);
}

void apply_galois_ntt(const Context &ctx, const u64 *in, std::size_t nlimbs, u32 elt, u64 *out)
{
    const std::size_t N = ctx.N();
    const int logn = ctx.log_n();
    std::vector<u32> tbl(N);
    for (std::size_t t = 0; t < N; ++t) {  // GaloisTool::generate_table_ntt
        const u64 rev = 2 * (u64)reverse_bits((u32)t, logn) + 1;
        const u64 idx = ((u64)elt * rev >> 1) & (N - 1);
        tbl[t] = reverse_bits((u32)idx, logn);
    }
    for (std::size_t i = 0; i < nlimbs; ++i)
        for (std::size_t t = 0; t < N; ++t) out[i * N + t] = in[i * N + tbl[t]];
}

void apply_galois_inplace(const Context &ctx, Ciphertext &a, u32 elt, const GaloisKeys &gk)
{
    check_ct(ctx, a);
    const std::size_t N = ctx.N(), l = a.level;
    auto it = gk.find(elt);
    if (it == gk.end()) throw std::invalid_argument("Galois key not present");
    if (!(elt & 1) || elt >= 2 * N) throw std::invalid_argument("Galois element is not valid");
    if (a.size > 2) throw std::invalid_argument("encrypted size must be 2");
    std::vector<u64> tmp(l * N);
    apply_galois_ntt(ctx, a.poly(0, N), l, elt, tmp.data());
    std::memcpy(a.poly(0, N), tmp.data(), l * N * sizeof(u64));
    apply_galois_ntt(ctx, a.poly(1, N), l, elt, tmp.data());
    std::fill(a.poly(1, N), a.poly(1, N) + l * N, 0);
    switch_key_inplace(ctx, a, tmp.data(), it->second);
}

std::vector<int> naf(int value)
{
    std::vector<int> res;
    const bool sign = value < 0;
    value = std::abs(value);
    for (int i = 0; value; ++i) {
        const int zi = (value & 1) ? 2 - (value & 3) : 0;
        value = (value - zi) >> 1;
        if (zi) res.push_back((sign ? -zi : zi) * (1 << i));
    }
    return res;
}

void rotate_vector_inplace(const Context &ctx, Ciphertext &a, int steps, const GaloisKeys &gk)
{
    check_ct(ctx, a);
    if (steps == 0) return;  // Evaluator::rotate_internal
    const u32 elt = ctx.elt_from_step(steps);
    if (gk.count(elt)) { apply_galois_inplace(ctx, a, elt, gk); return; }
    const std::vector<int> terms = naf(steps);
    if (terms.size() == 1) throw std::invalid_argument("Galois key not present");
    for (int s : terms)
        if ((std::size_t)std::abs(s) != (ctx.N() >> 1)) rotate_vector_inplace(ctx, a, s, gk);
}

// =============================================================== he::linalg ==================
// BatchedVector::sum_elems_inplace (he_linalg.cpp:667-713): every slot r receives the sum of the dim slots
// r, r+1, ..., r+dim-1, built over the binary expansion of dim with rotate-and-add steps (power-of-two
// windows), in the reference's order of rotations and additions.
void sum_elems_inplace(const Context &ctx, Ciphertext &v, std::size_t dim, const GaloisKeys &gk)
{
    Ciphertext rest = v;   // the slots not yet folded in, rotated past what has been summed so far
    Ciphertext part, t;
    int win = 1;
    bool started = false;  // v already holds a partial sum (odd dim: the first slot on its own)
    if (dim & 1) {
        started = true;
        rotate_vector_inplace(ctx, rest, win, gk);
    }
    for (std::size_t bits = dim >> 1; bits; bits >>= 1) {
        win <<= 1;
        if (!(bits & 1)) continue;
        int step = win >> 1;
        t = rest;
        rotate_vector_inplace(ctx, t, step, gk);
        Ciphertext &w = started ? part : v;   // a window of win slots: rest + rot(rest, win/2) + ...
        w = rest;
        add_inplace(ctx, w, t);
        for (step >>= 1; step; step >>= 1) {
            t = w;
            rotate_vector_inplace(ctx, t, step, gk);
            add_inplace(ctx, w, t);
        }
        if (started) add_inplace(ctx, v, part);
        started = true;
        if (bits != 1) rotate_vector_inplace(ctx, rest, win, gk);
    }
}

std::vector<Ciphertext> matmul_diag_col_set(const Context &ctx, const std::vector<const Ciphertext *> &A,
                                            const std::vector<std::size_t> &js,
                                            const std::vector<const Ciphertext *> &X, const KSwitchKey &rk,
                                            const GaloisKeys &gk, int nthreads, bool finish)
{
    // A[k] is diagonal js[k]; out[i] = sum_k A[k] (*) rot(X[i], js[k])  (he_linalg.cpp:977-997 restricted
    // to the diagonals js; a partition of [0, n) summed mod q gives the full loop's accumulator)
    const std::size_t nj = js.size(), p = X.size();
    if (nj == 0 || A.size() != nj) throw std::invalid_argument("empty diagonal range");
    nthreads = std::max(1, nthreads);
    const std::size_t chunks = std::min<std::size_t>((std::size_t)nthreads, nj);
    std::vector<std::vector<Ciphertext>> part(p, std::vector<Ciphertext>(chunks));
    std::atomic<std::size_t> next{0};
    std::vector<std::string> errs(nthreads);
    auto worker = [&](int tid) {
        try {
            for (;;) {
                const std::size_t w = next.fetch_add(1);
                if (w >= p * chunks) break;
                const std::size_t i = w / chunks, c = w % chunks;
                const std::size_t kb = nj * c / chunks, ke = nj * (c + 1) / chunks;
                Ciphertext acc;
                for (std::size_t k = kb; k < ke; ++k) {  // he_linalg.cpp:977-997
                    Ciphertext t = *X[i];
                    rotate_vector_inplace(ctx, t, (int)js[k], gk);  // always from the original column (:988)
                    multiply_inplace(ctx, t, *A[k]);
                    if (k == kb) acc = std::move(t);
                    else add_inplace(ctx, acc, t);
                }
                part[i][c] = std::move(acc);
            }
        } catch (const std::exception &e) { errs[tid] = e.what(); }
    };
    if (nthreads == 1) worker(0);
    else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
        for (auto &t : th) t.join();
    }
    for (auto &e : errs)
        if (!e.empty()) throw std::invalid_argument(e);
    std::vector<Ciphertext> out(p);
    for (std::size_t i = 0; i < p; ++i) {
        out[i] = std::move(part[i][0]);
        for (std::size_t c = 1; c < chunks; ++c) add_inplace(ctx, out[i], part[i][c]);
        if (finish) {  // SMART_RELIN == 1: he_linalg.cpp:999-1002
            relinearize_inplace(ctx, out[i], rk);
            rescale_to_next_inplace(ctx, out[i]);
        }
    }
    return out;
}

// The ct x pt form of the same loop: BatchedMatrix::matmul's diag x col with plaintext
// diagonals, `*=` = multiply_plain_inplace (he_operators.cpp:128-142), products stay size 2 (no relinearization),
// then rescale_to_next per output when finish.  P[k] is diagonal js[k]; threads over (output, diagonal chunk) with
// the chunk partials summed mod q (modular addition is exact and order free).
std::vector<Ciphertext> matmul_diagpt_col_set(const Context &ctx, const std::vector<const Plaintext *> &P,
                                              const std::vector<std::size_t> &js,
                                              const std::vector<const Ciphertext *> &X, const GaloisKeys &gk,
                                              int nthreads, bool finish)
{
    const std::size_t nj = js.size(), p = X.size();
    if (nj == 0 || P.size() != nj) throw std::invalid_argument("empty diagonal range");
    nthreads = std::max(1, nthreads);
    const std::size_t chunks = std::min<std::size_t>((std::size_t)nthreads, nj);
    std::vector<std::vector<Ciphertext>> part(p, std::vector<Ciphertext>(chunks));
    std::atomic<std::size_t> next{0};
    std::vector<std::string> errs(nthreads);
    auto worker = [&](int tid) {
        try {
            for (;;) {
                const std::size_t w = next.fetch_add(1);
                if (w >= p * chunks) break;
                const std::size_t i = w / chunks, c = w % chunks;
                const std::size_t kb = nj * c / chunks, ke = nj * (c + 1) / chunks;
                Ciphertext acc;
                for (std::size_t k = kb; k < ke; ++k) {
                    Ciphertext t = *X[i];
                    rotate_vector_inplace(ctx, t, (int)js[k], gk);
                    multiply_plain_inplace(ctx, t, *P[k]);
                    if (k == kb) acc = std::move(t);
                    else add_inplace(ctx, acc, t);
                }
                part[i][c] = std::move(acc);
            }
        } catch (const std::exception &e) { errs[tid] = e.what(); }
    };
    if (nthreads == 1) worker(0);
    else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
        for (auto &t : th) t.join();
    }
    for (auto &e : errs)
        if (!e.empty()) throw std::invalid_argument(e);
    std::vector<Ciphertext> out(p);
    for (std::size_t i = 0; i < p; ++i) {
        out[i] = std::move(part[i][0]);
        for (std::size_t c = 1; c < chunks; ++c) add_inplace(ctx, out[i], part[i][c]);
        if (finish) rescale_to_next_inplace(ctx, out[i]);
    }
    return out;
}

std::vector<Ciphertext> matmul_diag_col(const Context &ctx, const std::vector<const Ciphertext *> &A,
                                        const std::vector<const Ciphertext *> &X, const KSwitchKey &rk,
                                        const GaloisKeys &gk, int nthreads, std::size_t j_begin,
                                        std::size_t j_end, bool finish)
{
    j_end = std::min(j_end, A.size());
    if (j_begin >= j_end) throw std::invalid_argument("empty diagonal range");
    std::vector<std::size_t> js;
    std::vector<const Ciphertext *> a;
    for (std::size_t j = j_begin; j < j_end; ++j) { js.push_back(j); a.push_back(A[j]); }
    return matmul_diag_col_set(ctx, a, js, X, rk, gk, nthreads, finish);
}

std::vector<Ciphertext> matmul_col_colT(const Context &ctx, const std::vector<const Ciphertext *> &A,
                                        const std::vector<const Ciphertext *> &B, std::size_t p,
                                        const KSwitchKey &rk, const GaloisKeys &gk, int nthreads)
{
    // he_linalg.cpp:977-1002 with btype_is_col: out[i] = sum_j rot(B[j], i) (*) A[j]; outputs on threads
    const std::size_t n = A.size();
    if (B.size() != n) throw std::invalid_argument("dimension mismatch");
    std::vector<Ciphertext> out(p);
    std::atomic<std::size_t> next{0};
    nthreads = std::max(1, nthreads);
    std::vector<std::string> errs(nthreads);
    auto worker = [&](int tid) {
        try {
            for (std::size_t i; (i = next.fetch_add(1)) < p;) {
                for (std::size_t j = 0; j < n; ++j) {
                    Ciphertext t = *B[j];
                    rotate_vector_inplace(ctx, t, (int)i, gk);
                    multiply_inplace(ctx, t, *A[j]);
                    if (j == 0) out[i] = std::move(t);
                    else add_inplace(ctx, out[i], t);
                }
                relinearize_inplace(ctx, out[i], rk);
                rescale_to_next_inplace(ctx, out[i]);
            }
        } catch (const std::exception &e) { errs[tid] = e.what(); }
    };
    if (nthreads == 1) worker(0);
    else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
        for (auto &t : th) t.join();
    }
    for (auto &e : errs)
        if (!e.empty()) throw std::invalid_argument(e);
    return out;
}

std::vector<Ciphertext> matrix_matmul(const Context &ctx, const std::vector<const Ciphertext *> &A,
                                      std::size_t a_rows, std::size_t a_cols, bool a_tr,
                                      const std::vector<const Ciphertext *> &B, std::size_t b_rows,
                                      std::size_t b_cols, bool b_tr, const KSwitchKey &rk)
{
    // Matrix::ij_to_idx (he_linalg.cpp:376-379); get_dims swaps when transposed (:25-28)
    auto at = [](const std::vector<const Ciphertext *> &M, std::size_t rows, bool tr, std::size_t i, std::size_t j) {
        return M[(tr ? j : i) + rows * (tr ? i : j)];
    };
    const std::size_t r1 = a_tr ? a_cols : a_rows, c1 = a_tr ? a_rows : a_cols;
    const std::size_t r2 = b_tr ? b_cols : b_rows, c2 = b_tr ? b_rows : b_cols;
    if (c1 != r2) throw std::invalid_argument("dimension mismatch");
    std::vector<Ciphertext> out(r1 * c2);
    for (std::size_t j = 0; j < c2; ++j)
        for (std::size_t i = 0; i < r1; ++i) {
            Ciphertext &res = out[i + r1 * j];
            for (std::size_t k = 0; k < c1; ++k) {
                Ciphertext t = *at(A, a_rows, a_tr, i, k);
                multiply_inplace(ctx, t, *at(B, b_rows, b_tr, k, j));
                if (k == 0) res = std::move(t);
                else add_inplace(ctx, res, t);
            }
            relinearize_inplace(ctx, res, rk);
            rescale_to_next_inplace(ctx, res);
        }
    (void)r2;
    return out;
}

}  // namespace oracle
