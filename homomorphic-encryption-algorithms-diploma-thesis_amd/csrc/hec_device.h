// Device-side modular arithmetic for the CKKS engine (gfx950).
//
// All residues are u64 < q < 2^61.  CDNA4 has no 64x64->128 multiply: __umul64hi lowers to
// v_mul_hi_u32 / v_mad_u64_u32 sequences, so the hot paths use Shoup multiplication (one mulhi +
// two low multiplies per product) with precomputed quotients, and Barrett only where both operands
// vary (ciphertext tensor products, key-switch accumulators).  Every routine here returns the
// canonical residue when its name does not say "lazy", so results are bit-identical to SEAL's
// canonical outputs regardless of the lazy-reduction schedule inside a kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint64_t u64;
typedef uint32_t u32;

#define HEC_MAXL 32  // max RNS limbs handled by per-limb constant tables passed by value

struct DevPrime {
    u64 q;
    u64 r0, r1;         // floor(2^128 / q) = r1:r0 (SEAL Modulus::const_ratio)
    u64 ninv, ninv_q;   // N^-1 mod q and its Shoup quotient
    double qd, qinv, ninv_d;  // FP64 path (q < 2^42 only): q, 1/q, N^-1 as doubles
    int fp;                   // 1 -> NTT kernels use the exact FP64 arithmetic below
};

// primes[i] read through the constant address space: with a block-uniform i the loads are scalar (lgkmcnt), so a
// kernel that stores and then looks up its next prime does not wait for its stores (a vector load's vmcnt wait
// includes every store issued before it)
__device__ __forceinline__ DevPrime cprime(const DevPrime *primes, int i)
{
    typedef __attribute__((address_space(4))) const u64 cword;
    static_assert(sizeof(DevPrime) % 8 == 0, "DevPrime is copied as words");
    u64 w[sizeof(DevPrime) / 8];
#pragma unroll
    for (unsigned k = 0; k < sizeof(DevPrime) / 8; ++k) w[k] = ((cword *)(primes + i))[k];
    DevPrime r;
    __builtin_memcpy(&r, w, sizeof(DevPrime));
    return r;
}

__device__ __forceinline__ u64 mulhi64(u64 a, u64 b) { return __umul64hi(a, b); }

// x * w mod q in [0, 2q) for any x < 2^64, w < q, wq = floor(w * 2^64 / q)
__device__ __forceinline__ u64 shoup_lazy(u64 x, u64 w, u64 wq, u64 q) { return x * w - mulhi64(x, wq) * q; }
__device__ __forceinline__ u64 csub(u64 x, u64 q) { return x >= q ? x - q : x; }
__device__ __forceinline__ u64 shoup(u64 x, u64 w, u64 wq, u64 q) { return csub(shoup_lazy(x, w, wq, q), q); }

// SEAL util::barrett_reduce_64: any 64-bit x -> x mod q
__device__ __forceinline__ u64 barrett64(u64 x, u64 q, u64 r1) { return csub(x - mulhi64(x, r1) * q, q); }

// full 64x64 -> 128 product from the four 32x32 -> 64 partial products (v_mad_u64_u32 each); the compiler's
// separate a * b and __umul64hi(a, b) take six multiplies
__device__ __forceinline__ void mul128(u64 a, u64 b, u64 &lo, u64 &hi)
{
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = (u64)a0 * b0;
    const u64 p01 = (u64)a0 * b1 + (p00 >> 32);  // < 2^64
    const u64 p10 = (u64)a1 * b0 + (u32)p01;     // < 2^64
    hi = (u64)a1 * b1 + ((p01 >> 32) + (p10 >> 32));
    lo = (p10 << 32) | (u32)p00;
}

// SEAL util::barrett_reduce_128: 128-bit (hi:lo) -> mod q
__device__ __forceinline__ u64 barrett128(u64 lo, u64 hi, u64 q, u64 r0, u64 r1)
{
    u64 carry = mulhi64(lo, r0);
    u64 t_lo = lo * r1, t_hi = mulhi64(lo, r1);
    u64 tmp1 = t_lo + carry;
    u64 tmp3 = t_hi + (tmp1 < carry);
    u64 u_lo = hi * r0, u_hi = mulhi64(hi, r0);
    u64 sum = tmp1 + u_lo;
    carry = u_hi + (sum < tmp1);
    u64 est = hi * r1 + tmp3 + carry;
    return csub(lo - est * q, q);
}
__device__ __forceinline__ u64 mulmod(u64 a, u64 b, const DevPrime &p)
{
    return barrett128(a * b, mulhi64(a, b), p.q, p.r0, p.r1);
}
__device__ __forceinline__ u64 addmod(u64 a, u64 b, u64 q) { return csub(a + b, q); }
__device__ __forceinline__ u64 submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

// 128-bit accumulator
struct U128 {
    u64 lo, hi;
};
__device__ __forceinline__ void mac128(U128 &acc, u64 a, u64 b)
{
    u64 plo, phi;
    mul128(a, b, plo, phi);
    acc.lo += plo;
    acc.hi += phi + (acc.lo < plo);
}

// Cooley-Tukey (Harvey) forward butterfly, inputs/outputs in [0, 4q)
__device__ __forceinline__ void ct_bfly(u64 &X, u64 &Y, u64 w, u64 wq, u64 q, u64 two_q)
{
    u64 x = X >= two_q ? X - two_q : X;
    const u64 t = shoup_lazy(Y, w, wq, q);
    X = x + t;
    Y = x - t + two_q;
}
// Gentleman-Sande inverse butterfly, inputs/outputs in [0, 2q); w = inverse twiddle
__device__ __forceinline__ void gs_bfly(u64 &X, u64 &Y, u64 w, u64 wq, u64 q, u64 two_q)
{
    const u64 s = X + Y;
    const u64 d = X - Y + two_q;
    X = s >= two_q ? s - two_q : s;
    Y = shoup_lazy(d, w, wq, q);
}

// Split-input Shoup product (round 5; q < 2^60, Y < 4q): t = Y w mod q in [0, 2q) with eight 32-bit multiplies
// instead of shoup_lazy's ten.  Y = y1 2^31 + y0 (y0, y1 < 2^31) and Y w == y1 a + y0 w (mod q), a = w 2^31 mod q (a
// per-twiddle table).  The quotient of that sum T < 2^32 q comes from the 32-bit factors a' = floor(a 2^32 / q) and
// w' = floor(w 2^32 / q), which are bits of the Shoup factor wq = floor(w 2^64 / q) the twiddle already carries:
// w' = wq >> 32 and a' = (wq >> 1) mod 2^32 (a 2^32 / q = w 2^63 / q - floor(w 2^31 / q) 2^32).  qh = (y1 a' + y0 w')
// >> 32 (the sum < 2^64) is T's quotient or one less, so T - qh q, taken mod 2^64, lies in [0, 2q): the same range
// and residue as shoup_lazy, so butterflies built on it keep Harvey's bounds and every output's bits.
// Measured 97-98 vs 117 cycles per butterfly per wave on gfx950 (tools/micro_bfly.hip, profiles/r05o_micro_bfly.txt).
__device__ __forceinline__ u64 shoup_split_lazy(u64 Y, u64 w, u64 wq, u64 a, u64 q)
{
    const u32 y0 = (u32)Y & 0x7fffffffu, y1 = (u32)(Y >> 31);
    const u32 qh = (u32)(((u64)y1 * (u32)(wq >> 1) + (u64)y0 * (u32)(wq >> 32)) >> 32);
    const u64 lo = (u64)y0 * (u32)w + (u64)y1 * (u32)a;
    const u32 hi = y0 * (u32)(w >> 32) + y1 * (u32)(a >> 32);
    return lo + ((u64)hi << 32) - ((u64)qh * (u32)q + ((u64)(qh * (u32)(q >> 32)) << 32));
}
__device__ __forceinline__ void ct_bfly_s(u64 &X, u64 &Y, u64 w, u64 wq, u64 a, u64 q, u64 two_q)
{
    u64 x = X >= two_q ? X - two_q : X;
    const u64 t = shoup_split_lazy(Y, w, wq, a, q);
    X = x + t;
    Y = x - t + two_q;
}
__device__ __forceinline__ void gs_bfly_s(u64 &X, u64 &Y, u64 w, u64 wq, u64 a, u64 q, u64 two_q)
{
    const u64 s = X + Y;
    const u64 d = X - Y + two_q;
    X = s >= two_q ? s - two_q : s;
    Y = shoup_split_lazy(d, w, wq, a, q);
}

__device__ __forceinline__ u32 bitrev(u32 x, int bits) { return __brev(x) >> (32 - bits); }

// SEAL GaloisTool::apply_galois_ntt source index: out[t] = in[galois_src(t)],
//   galois_src(t) = bitrev(((elt (2 bitrev(t) + 1)) >> 1) & (N - 1)); elt = 1 is the identity.
// Adjacent pairs map to adjacent pairs: galois_src(2w + 1) = galois_src(2w) ^ 1.
__device__ __forceinline__ u32 galois_src(u32 t, u32 elt, int logN)
{
    const u32 r = 2u * bitrev(t, logN) + 1u;
    return bitrev(((elt * r) & ((2u << logN) - 1u)) >> 1, logN);
}

// ------------------------------------------------------------------ exact FP64 modular arithmetic
// For q < 2^42 (fp = 1) residues are carried as integer-valued doubles.  gfx950 issues an FP64
// FMA in 4 cycles per wave vs 8 for a 32-bit integer multiply, and a 64x64->128 product needs
// 9 such multiplies, so this path is several times cheaper than Shoup on u64.
// fp_mulmod(y, w): TwoProduct  h + l = y*w exactly (h = fl(y*w), l = fma(y, w, -h));
// k = rint(h * (1/q)) is within 0.5 + 3|y| 2^-53 of y*w/q (w < q), so for |y| <= 10 q < 2^45.4
// r = (h - k q) + l is computed exactly (every intermediate is an integer below 2^53) and
// r = y*w - k q lies in [-0.53q, 0.53q].
// The result is congruent to y*w mod q; canonical residues are taken only at kernel outputs, so the
// final bits equal any other exact implementation's.
#pragma clang fp contract(off)
__device__ __forceinline__ double fp_mulmod(double y, double w, double q, double qinv)
{
    const double h = y * w;
    const double l = __fma_rn(y, w, -h);
    const double k = rint(h * qinv);
    const double r = __fma_rn(-k, q, h);
    return r + l;
}
__device__ __forceinline__ double fp_reduce(double x, double q, double qinv)  // -> [-0.53q, 0.53q]
{
    return __fma_rn(-rint(x * qinv), q, x);
}
// forward CT: |X| grows by <= 0.53q per stage (< 10q after 16 stages from inputs < 2q)
__device__ __forceinline__ void ct_bfly_fp(double &X, double &Y, double w, double q, double qinv)
{
    const double t = fp_mulmod(Y, w, q, qinv);
    Y = X - t;
    X = X + t;
}
// inverse GS: sums are re-centred every stage so magnitudes stay below q
__device__ __forceinline__ void gs_bfly_fp(double &X, double &Y, double w, double q, double qinv)
{
    const double s = X + Y, dlt = X - Y;
    X = fp_reduce(s, q, qinv);
    Y = fp_mulmod(dlt, w, q, qinv);
}
#pragma clang fp contract(on)
// exact u64 <-> double for 0 <= x < 2^52 through the 2^52 magic number
__device__ __forceinline__ double u2d(u64 x) { return __longlong_as_double((long long)(x | 0x4330000000000000ull)) - 4503599627370496.0; }
__device__ __forceinline__ u64 d2u(double x) { return (u64)__double_as_longlong(x + 4503599627370496.0) - 0x4330000000000000ull; }
// integer-valued double with |x| < 2^52 -> canonical residue, as a double and as u64
__device__ __forceinline__ double fp_canon_d(double x, double q, double qinv)
{
    const double r = fp_reduce(x, q, qinv);
    return r < 0 ? r + q : r;
}
__device__ __forceinline__ u64 fp_canon(double x, double q, double qinv) { return d2u(fp_canon_d(x, q, qinv)); }
