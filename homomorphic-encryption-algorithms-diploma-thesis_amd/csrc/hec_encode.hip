// CKKS encoder on the GPU: SEAL 4.1 CKKSEncoder::encode of complex (or real) slot vectors
// into NTT-form plaintexts, for `count` vectors per launch.  The reference encodes every matrix column / diagonal
// this way before encryption (src/demos/matrix_operations.cpp:1106-1108, client.cpp:228-230) and the ct x pt
// matvec's plaintext diagonals come from it.
//
// The sequence is SEAL's encode_internal, operation for operation (DESIGN.md §4.7 lists the places in the
// reference's build/demo, read as data, that pin each step):
//   1. conj_values[matrix_reps_index_map_[i]] = v_i, conj_values[matrix_reps_index_map_[N/2 + i]] = conj(v_i)
//      (the map folds in the bit reversal: bitrev((3^i mod 2N - 1) / 2));
//   2. DWTHandler::transform_from_rev over N complex points with inv_root_powers_ (host table, ComplexRoots +
//      get_root, glibc cos / sin): log2 N - 1 Gentleman-Sande layers x' = u + v, y' = (u - v) w, gap 1 .. N/4, then
//      the last layer with the scalar fix = scale / N folded in: x' = (u + v) fix, y' = (u - v)(w fix);
//   3. coefficient k = std::round(Re), max |Re| (unrounded) for SEAL's "encoded values are too large" check, and
//      the residue of the exact integer mod every data prime, negated when the sign bit is set (negate_uint_mod);
//   4. per data prime the forward NTT (the engine's k_ntt).
// Every butterfly is the IEEE result of the stated expression with no contraction (this file is built with
// -ffp-contract=off and the pragma below; complex products as libgcc's __muldc3: (ac - bd, ad + bc)), so the layers
// may run in any order that respects their data dependences and still give SEAL's bits.
// Layout: layers with gap < C = 2^LOGC (LOGC = min(11, log2 N - 1)) run inside contiguous C-point chunks staged in
// LDS (k_enc_dwt_lds); the remaining log2 N - LOGC layers, the scalar layer last, run on the 2^TS points r + t C of
// column r held in registers (k_enc_finish), which then rounds and writes the residues.
// Not on the matvec's timed path: diagonals are encoded once per matrix.
#include "hec_internal.h"

#pragma clang fp contract(off)

namespace hec {

namespace {

__device__ __forceinline__ double2 cmul(double2 x, double2 w)  // __muldc3 for finite operands
{
    return make_double2(x.x * w.x - x.y * w.y, x.x * w.y + x.y * w.x);
}
__device__ __forceinline__ void gs(double2 &X, double2 &Y, double2 w)
{
    const double2 u = X, v = Y;
    X = make_double2(u.x + v.x, u.y + v.y);
    Y = cmul(make_double2(u.x - v.x, u.y - v.y), w);
}

// step 1: one thread per slot i of vector blockIdx.y (the work area is zeroed first: SEAL allocates it with 0)
__global__ void __launch_bounds__(256) k_enc_scatter(const double *__restrict__ re, const double *__restrict__ im,
                                                     u64 nv, const u32 *__restrict__ map, double2 *__restrict__ a,
                                                     int logN)
{
    const u64 slots = 1ull << (logN - 1);
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= nv) return;
    const u64 v = blockIdx.y;
    const double2 z = make_double2(re[v * nv + i], im ? im[v * nv + i] : 0.0);
    double2 *av = a + (v << logN);
    av[map[i]] = z;
    av[map[slots + i]] = make_double2(z.x, -z.y);  // std::conj
}

// step 2, layers gap = 1 .. C/2 inside contiguous chunks of C = 2^LOGC points staged in LDS.  Layer s (gap 2^s) of
// an N-point transform has N >> (s + 1) groups; group i uses inv_root_powers_[N - (N >> s) + i + 1] (SEAL's
// `*++roots` walk).
template <int LOGC>
__global__ void __launch_bounds__(256) k_enc_dwt_lds(double2 *__restrict__ a, const double2 *__restrict__ roots,
                                                     int logN)
{
    constexpr int C = 1 << LOGC;
    __shared__ double2 s[C];
    const u64 N = 1ull << logN, base = (u64)blockIdx.x * C;
    double2 *av = a + ((u64)blockIdx.y << logN) + base;
    for (int k = threadIdx.x; k < C; k += 256) s[k] = av[k];
    __syncthreads();
#pragma unroll 1
    for (int lg = 0; lg < LOGC; ++lg) {
        const int gap = 1 << lg;
        const double2 *w = roots + (N - (N >> lg)) + 1;
        for (int b = threadIdx.x; b < C / 2; b += 256) {
            const int j = b & (gap - 1);
            const int x = ((b >> lg) << (lg + 1)) + j;       // upper element of the pair, local index
            const u64 grp = (base + (u64)x) >> (lg + 1);     // global group index
            gs(s[x], s[x + gap], w[grp]);
        }
        __syncthreads();
    }
    for (int k = threadIdx.x; k < C; k += 256) av[k] = s[k];
}

// |round(v)| mod q for a finite integer-valued double a >= 0, exactly (the integer SEAL decomposes into words)
__device__ __forceinline__ u64 enc_residue(double a, const DevPrime &p)
{
    if (a < 0x1.0p64) return barrett64((u64)a, p.q, p.r1);
    int e = 0;
    const double f = frexp(a, &e);                 // a = f 2^e, 0.5 <= f < 1, e > 64
    u64 r = barrett64((u64)ldexp(f, 53), p.q, p.r1), pw = 2 % p.q;
    for (int k = e - 53; k > 0; k >>= 1) {         // times 2^(e - 53) mod q
        if (k & 1) r = mulmod(r, pw, p);
        pw = mulmod(pw, pw, p);
    }
    return r;
}

// step 2's remaining layers gap = C .. N/2 on the 2^TS points r + t C of column r held in registers (the last one
// with the scalar fix), then step 3: out[v][i][k] for i < level, and the largest unrounded |Re| per vector
template <int TS>
__global__ void __launch_bounds__(256) k_enc_finish(const double2 *__restrict__ a, const double2 *__restrict__ roots,
                                                    int logN, int logC, double fix, int level,
                                                    const DevPrime *__restrict__ primes, u64 *__restrict__ out,
                                                    unsigned long long *__restrict__ maxabs)
{
    constexpr int R = 1 << TS;
    const u64 N = 1ull << logN, C = 1ull << logC;
    const u64 r = (u64)blockIdx.x * 256 + threadIdx.x;
    if (r >= C) return;
    const u64 v = blockIdx.y;
    const double2 *av = a + (v << logN);
    double2 x[R];
#pragma unroll
    for (int t = 0; t < R; ++t) x[t] = av[r + t * C];
#pragma unroll
    for (int st = 0; st + 1 < TS; ++st) {  // layer s = logC + st, gap C 2^st; pair (t, t + 2^st)
        const int s = logC + st;
        const double2 *w = roots + (N - (N >> s)) + 1;
#pragma unroll
        for (int t = 0; t < R; ++t) {
            if (t & (1 << st)) continue;
            gs(x[t], x[t + (1 << st)], w[t >> (st + 1)]);
        }
    }
    {  // the last layer (gap N/2, root N - 1) with the scalar: mul_scalar(add(u, v), fix), mul_root(sub, w fix)
        const double2 w = roots[N - 1];
        const double2 sw = make_double2(w.x * fix, w.y * fix);
#pragma unroll
        for (int t = 0; t < R / 2; ++t) {
            const double2 u = x[t], y = x[t + R / 2];
            x[t] = make_double2((u.x + y.x) * fix, (u.y + y.y) * fix);
            x[t + R / 2] = cmul(make_double2(u.x - y.x, u.y - y.y), sw);
        }
    }
    double mx = 0.0;
    u64 *ov = out + v * (u64)level * N;
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const u64 k = r + t * C;
        const double ax = fabs(x[t].x);
        mx = ax != ax ? __builtin_inf() : fmax(mx, ax);  // NaN input: rejected as "too large" like an infinity
        const double c = round(x[t].x);  // std::round: halves away from zero
        const bool neg = signbit(c);
        const double ac = fabs(c);
        if (!(ac < 0x1.0p1023)) continue;  // not finite: the caller rejects the vector ("too large")
        for (int i = 0; i < level; ++i) {
            const DevPrime p = primes[i];
            const u64 m = enc_residue(ac, p);
            ov[(u64)i * N + k] = (neg && m) ? p.q - m : m;  // negate_uint_mod
        }
    }
    // non-negative doubles order like their bit patterns
    atomicMax(maxabs + v, (unsigned long long)__double_as_longlong(mx));
}

}  // namespace

void encode_batch(Ctx &c, const double *re, const double *im, u64 nv, int count, double scale, int level, double *work,
                  u64 *out, u64 *maxabs)
{
    const int logN = c.logN;
    const u64 N = c.N;
    const int logc = logN - 1 < 11 ? logN - 1 : 11, ts = logN - logc;
    const double2 *roots = reinterpret_cast<const double2 *>(c.enc_tw);
    double2 *a = reinterpret_cast<double2 *>(work);
    dev_zero(c, maxabs, count * sizeof(u64));
    dev_zero(c, work, (u64)count * N * sizeof(double2));
    if (nv) {
        k_enc_scatter<<<dim3((unsigned)((nv + 255) / 256), count), 256, 0, c.stream>>>(re, im, nv, c.enc_map, a, logN);
        HEC_HIP(hipGetLastError());
    }
    const dim3 gl((unsigned)(N >> logc), count);
    switch (logc) {
    case 11: k_enc_dwt_lds<11><<<gl, 256, 0, c.stream>>>(a, roots, logN); break;
    case 10: k_enc_dwt_lds<10><<<gl, 256, 0, c.stream>>>(a, roots, logN); break;
    case 9: k_enc_dwt_lds<9><<<gl, 256, 0, c.stream>>>(a, roots, logN); break;
    default: throw std::invalid_argument("encode: N must be 2^10 .. 2^16");
    }
    HEC_HIP(hipGetLastError());
    const double fix = scale / (double)N;
    const dim3 gf((unsigned)(((N >> ts) + 255) / 256), count);
    auto *mx = reinterpret_cast<unsigned long long *>(maxabs);
    switch (ts) {
    case 1: k_enc_finish<1><<<gf, 256, 0, c.stream>>>(a, roots, logN, logc, fix, level, c.primes, out, mx); break;
    case 2: k_enc_finish<2><<<gf, 256, 0, c.stream>>>(a, roots, logN, logc, fix, level, c.primes, out, mx); break;
    case 3: k_enc_finish<3><<<gf, 256, 0, c.stream>>>(a, roots, logN, logc, fix, level, c.primes, out, mx); break;
    case 4: k_enc_finish<4><<<gf, 256, 0, c.stream>>>(a, roots, logN, logc, fix, level, c.primes, out, mx); break;
    case 5: k_enc_finish<5><<<gf, 256, 0, c.stream>>>(a, roots, logN, logc, fix, level, c.primes, out, mx); break;
    default: throw std::invalid_argument("encode: N must be 2^10 .. 2^16");
    }
    HEC_HIP(hipGetLastError());
    int pmap[HEC_MAXL + 1];
    for (int i = 0; i <= HEC_MAXL; ++i) pmap[i] = i;
    ntt_strided(c, false, out, (u64)level * N, out, (u64)level * N, level, pmap, count * level);
}

}  // namespace hec
