// Single-pass mod-down (round 6; HEC_MODDOWN1 / option "moddown1", N = 2^15 only).
//
// SEAL's divide_and_round_q_last (switch_key_inplace step 4) for every data limb i of every (batch entry b, poly k) in
// one kernel: a 1024-thread workgroup owns one target limb, takes the coefficient-form special-prime limb y of (b, k),
// forms the rounding limb (y + floor(P/2)) mod P mod q_i - floor(P/2) mod q_i, runs the whole forward NTT of it in
// registers and LDS, and finishes the divide-and-round on its own outputs: OUT_i = (ACC_i - NTT(r)) P^-1 (+ IN_i).
// The rounding limbs Z never go to HBM: the two-pass path writes them in the fan-out (k_fan2, pass-A domain) and reads
// them back in the divide-and-round pass B (2 B l limbs each way per key switch).
//
// The transform is the engine's own single-pass layout (round 1, HEC_NTT1, then measured 0.199 vs 0.245 us per FP64
// limb): element e = h 1024 + m 32 + l (5 bits each), thread t = a 32 + b; round 1 (stages 0..4) holds h = 0..31,
// round 2 (5..9) m = 0..31, round 3 (10..14) l = 0..31, i.e. 32 consecutive outputs.  A limb (256 KiB) does not fit
// the 160 KiB LDS, so each exchange runs in two phases over a 132 KiB window with 33-word rows (no bank conflicts).
// Both arithmetic classes: exact FP64 butterflies for q_i < 2^42, Harvey's lazy 60-bit butterflies otherwise, with
// the same rounding transform and post-op as the two-pass path (FanDivRound::xf16, DivRoundIOB::store/store_fp), so
// every output word is the same integer.
#include <mutex>

#include "hec_internal.h"

namespace hec {

namespace {

constexpr int kLogN = 15;
constexpr int MD1_LDS_WORDS = 2 * 16 * 16 * 33;  // 16,896 words = 135,168 B

template <bool FP>
__device__ __forceinline__ void md1_bfly(u64 &x, u64 &y, const void *tw, u64 idx, const DevPrime &pr)
{
    if constexpr (FP) {
        double X = __longlong_as_double((long long)x), Y = __longlong_as_double((long long)y);
        ct_bfly_fp(X, Y, static_cast<const double *>(tw)[idx], pr.qd, pr.qinv);
        x = (u64)__double_as_longlong(X);
        y = (u64)__double_as_longlong(Y);
    } else {
        const ulonglong2 w = static_cast<const ulonglong2 *>(tw)[idx];
        ct_bfly(x, y, w.x, w.y, pr.q, 2 * pr.q);
    }
}

// stages S0 .. S0 + 4 on the thread's 32 registers (register index = the round's 5-bit digit); the pair at digit r
// of stage S0 + j takes twiddle 2^(S0 + j) + (base << j) + (r >> (5 - j)) (SEAL's bit-reversed root powers)
template <bool FP, int S0>
__device__ __forceinline__ void md1_round(u64 *v, const void *tw, u64 base, const DevPrime &pr)
{
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int half = 16 >> j;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & half) continue;
            md1_bfly<FP>(v[r], v[r + half], tw, (1ull << (S0 + j)) + (base << j) + (u64)(r >> (5 - j)), pr);
        }
    }
}

// exchange 1 (h <-> m across all threads): phase P moves the elements with h4 ^ m4 == P; a thread writes and re-reads
// half X = a4 ^ P of its registers (a4 = a >> 4 is wave-uniform, so every register index stays compile-time)
template <int X>
__device__ __forceinline__ void md1_exch1_half(u64 *v, u64 *lds, int a, int b)
{
    const int a4 = a >> 4, ap = a & 15;
#pragma unroll
    for (int hp = 0; hp < 16; ++hp) lds[((a4 * 16 + hp) * 16 + ap) * 33 + b] = v[X * 16 + hp];
    __syncthreads();
#pragma unroll
    for (int mp = 0; mp < 16; ++mp) v[X * 16 + mp] = lds[((X * 16 + ap) * 16 + mp) * 33 + b];
    __syncthreads();
}

__device__ __forceinline__ void md1_exchange1(u64 *v, u64 *lds, int a, int b)
{
    if ((a >> 4) == 0) {
        md1_exch1_half<0>(v, lds, a, b);
        md1_exch1_half<1>(v, lds, a, b);
    } else {
        md1_exch1_half<1>(v, lds, a, b);
        md1_exch1_half<0>(v, lds, a, b);
    }
}

// exchange 2 (m <-> l inside each group of 32 threads with the same h): the waves with a4 == phase, per phase
__device__ __forceinline__ void md1_exchange2(u64 *v, u64 *lds, int a, int b)
{
    const int a4 = a >> 4, ap = a & 15;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
        if (a4 == ph) {
#pragma unroll
            for (int m = 0; m < 32; ++m) lds[(ap * 32 + m) * 33 + b] = v[m];
        }
        __syncthreads();
        if (a4 == ph) {
#pragma unroll
            for (int l = 0; l < 32; ++l) v[l] = lds[(ap * 32 + b) * 33 + l];
        }
        __syncthreads();
    }
}

struct MD1Args {
    const u64 *Y;  // coefficient-form special-prime limb of (b, k): Y + b ysb + k ysk
    u64 ysb, ysk;
    PolyArr X;     // ACC data limbs: X.p + b X.sb + k X.sk + (i << logN)
    PolyArr IN;    // added for polys k < in_nk, read through the Galois permutation of elt (IN.p == nullptr: none)
    int in_nk;
    u32 elt;
    PolyArr OUT;
    int B, nk, nl;
    int nt, ti[HEC_MAXL];  // this launch's target limbs (one arithmetic class per launch)
    u64 last, half;
    unsigned sub1;
    u64 fix[HEC_MAXL];
    double c30[HEC_MAXL];
    u64 inv[HEC_MAXL], inv_q[HEC_MAXL];
};

template <bool FP>
__device__ __forceinline__ void md1_body(const MD1Args &A, u64 *lds, const DevPrime &pr, const void *tw, int g, int i)
{
    const int t = threadIdx.x, a = t >> 5, b = t & 31;
    const int bb = g / A.nk, k = g % A.nk;
    const u64 *y = A.Y + (u64)bb * A.ysb + (u64)k * A.ysk;
    u64 v[32];
#pragma unroll
    for (int h = 0; h < 32; ++h) v[h] = y[h * 1024 + t];
    // the rounding limb: (y + floor(P/2)) mod P, reduced mod q_i, plus fix_i = q_i - floor(P/2) mod q_i
    // (FanDivRound::src_fix / xf16: an integer-valued double in (-0.51 q_i, 1.51 q_i + 2^30) at FP64 targets with
    // q_i > 2^32, else a value in [0, 2 q_i))
    const u64 fixi = A.fix[i];
    const double c30 = A.c30[i];
    const bool sub1 = ((A.sub1 >> i) & 1u) != 0;
#pragma unroll
    for (int h = 0; h < 32; ++h) {
        u64 s = v[h] + A.half;
        s = s >= A.last ? s - A.last : s;
        if (FP && c30 != 0.0) {
            const double hs = u2d(s >> 30) * 1073741824.0;
            v[h] = (u64)__double_as_longlong(fp_reduce(hs, pr.qd, pr.qinv) + ((double)(u32)(s & 0x3fffffffull) +
                                                                             (double)fixi));
        } else {
            const u64 r = (sub1 ? csub(s, pr.q) : barrett64(s, pr.q, pr.r1)) + fixi;
            v[h] = FP ? (u64)__double_as_longlong(u2d(r)) : r;
        }
    }
    md1_round<FP, 0>(v, tw, 0, pr);
    md1_exchange1(v, lds, a, b);
    md1_round<FP, 5>(v, tw, (u64)a, pr);
    md1_exchange2(v, lds, a, b);
    md1_round<FP, 10>(v, tw, (u64)t, pr);
    // divide-and-round on the thread's 32 consecutive outputs o = 32 t + l (DivRoundIOB::store_fp / store)
    const u64 li = (u64)i << kLogN, o0 = (u64)t * 32;
    const u64 *xa = A.X.p + (u64)bb * A.X.sb + (u64)k * A.X.sk + li;
    u64 *out = A.OUT.p + (u64)bb * A.OUT.sb + (u64)k * A.OUT.sk + li;
    const u64 *in = (A.IN.p != nullptr && k < A.in_nk) ? A.IN.p + (u64)bb * A.IN.sb + (u64)k * A.IN.sk + li : nullptr;
    const u64 w = A.inv[i], wq = A.inv_q[i];
#pragma unroll
    for (int l = 0; l < 32; l += 2) {
        const u64 o = o0 + l;
        const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(xa + o);
        ulonglong2 iv{0, 0};
        if (in) {
            if (A.elt == 1) {
                iv = *reinterpret_cast<const ulonglong2 *>(in + o);
            } else {  // adjacent outputs map to adjacent sources (galois_src(2w + 1) = galois_src(2w) ^ 1)
                const u32 s0 = galois_src((u32)o, A.elt, kLogN);
                const ulonglong2 p = *reinterpret_cast<const ulonglong2 *>(in + (s0 & ~1u));
                iv = (s0 & 1) ? ulonglong2{p.y, p.x} : p;
            }
        }
        u64 r[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const u64 xv = e ? x.y : x.x, inv_ = e ? iv.y : iv.x;
            if constexpr (FP) {
                double d = fp_mulmod(u2d(xv) - __longlong_as_double((long long)v[l + e]), u2d(w), pr.qd, pr.qinv);
                if (in) d += u2d(inv_);
                r[e] = fp_canon(d, pr.qd, pr.qinv);
            } else {
                const u64 vv = csub(csub(v[l + e], 2 * pr.q), pr.q);
                u64 s = shoup(xv + pr.q - vv, w, wq, pr.q);
                if (in) s = addmod(s, inv_, pr.q);
                r[e] = s;
            }
        }
        *reinterpret_cast<ulonglong2 *>(out + o) = ulonglong2{r[0], r[1]};
    }
}

// One arithmetic class per launch (each keeps its own 128-VGPR budget: 16 waves per CU).  XCD-aware order: the nt
// targets of one (b, k) run back to back on one XCD (blocks x, x + 8, ...), so the source limb y comes from HBM for
// the first and from that XCD's L2 for the others
template <bool FP>
__global__ void __launch_bounds__(1024) k_moddown1(const MD1Args A, const u64 *__restrict__ twi,
                                                   const double *__restrict__ twf, const DevPrime *__restrict__ primes)
{
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    const int x = blockIdx.x, xcd = x & 7, tq = x >> 3;
    const int g = (tq / A.nt) * 8 + xcd, i = A.ti[tq % A.nt];
    if (g >= A.B * A.nk) return;  // uniform per block
    const DevPrime pr = primes[i];
    if constexpr (FP) md1_body<true>(A, lds, pr, twf + ((u64)i << kLogN), g, i);
    else md1_body<false>(A, lds, pr, twi + ((u64)i << (kLogN + 1)), g, i);
}

}  // namespace

bool moddown1(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, PolyArr X, PolyArr IN, int in_nk, PolyArr OUT, int B, int nk,
              int nl, int last_idx, u32 elt)
{
    if (c.logN != kLogN || B <= 0 || nl <= 0 || nl > HEC_MAXL) return false;
    MD1Args A{};
    A.Y = Y; A.ysb = ysb; A.ysk = ysk; A.X = X; A.IN = IN; A.in_nk = in_nk; A.elt = elt; A.OUT = OUT;
    A.B = B; A.nk = nk; A.nl = nl;
    A.last = c.q[last_idx]; A.half = A.last >> 1;
    for (int i = 0; i < nl; ++i) {
        A.fix[i] = c.q[i] - (A.half % c.q[i]);
        A.c30[i] = c.q[i] < (1ull << 42) && c.q[i] > (1ull << 32) ? (double)((1ull << 30) % c.q[i]) : 0.0;
        if (A.last < 2 * c.q[i] && i < 32) A.sub1 |= 1u << i;
        A.inv[i] = c.p_inv[i];
        A.inv_q[i] = c.p_inv_q[i];
    }
    constexpr int bytes = MD1_LDS_WORDS * 8;
    static std::once_flag attr;  // lanes may launch from several host threads
    std::call_once(attr, [] {
        HEC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_moddown1<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
        HEC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_moddown1<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    });
    const unsigned groups = (unsigned)((B * nk + 7) / 8 * 8);
    for (int fp = 0; fp < 2; ++fp) {  // the integer targets first (fewer, slower blocks start early)
        A.nt = 0;
        for (int i = 0; i < nl; ++i)
            if ((c.hprimes[i].fp != 0) == (fp != 0)) A.ti[A.nt++] = i;
        if (A.nt == 0) continue;
        if (fp)
            k_moddown1<true><<<dim3(groups * (unsigned)A.nt), 1024, bytes, c.stream>>>(
                A, reinterpret_cast<const u64 *>(c.tw), c.twf, c.primes);
        else
            k_moddown1<false><<<dim3(groups * (unsigned)A.nt), 1024, bytes, c.stream>>>(
                A, reinterpret_cast<const u64 *>(c.tw), c.twf, c.primes);
        HEC_HIP(hipGetLastError());
    }
    return true;
}

}  // namespace hec
