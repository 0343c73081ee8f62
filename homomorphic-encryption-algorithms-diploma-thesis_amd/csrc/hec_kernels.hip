// CDNA4 (gfx950) kernels of the CKKS engine.
//
// NTT: an N-point negacyclic NTT (SEAL convention: Cooley-Tukey with bit-reversed twiddles
// psi^bitrev(k), bit-reversed output) is split into two LDS-staged passes over
// N = R x C (R = 2^ceil(logN/2) rows, C = 2^floor(logN/2) columns):
//   pass A: global stages 0..logR-1 run independently on each column (stride-C elements);
//   pass B: global stages logR..logN-1 run independently on each contiguous chunk of C elements.
// At local stage s of a P-point sub-transform the butterfly whose upper element has local index x
// uses global twiddle index  base*2^s + (x >> (logP - s)),  base = 1 in pass A and R + chunk in
// pass B, so both passes read the same SEAL-ordered twiddle table.  Inside a pass every thread
// owns 16 elements and does 4 radix-2 stages in registers per round (2 rounds), exchanging through
// LDS between rounds; the global<->LDS copies are linear so that every wave reads/writes one
// contiguous 512-B run.  Pre-/post-operations (mod-up reduction, mod-down rounding, P^-1 scaling,
// accumulation into the ciphertext) are fused into the first-pass load and last-pass store through
// small IO functors, so the key switch never materialises them separately.
#include "hec_internal.h"

#include <type_traits>

namespace hec {

// =============================================================================== NTT IO ====
// 16-B accesses of the word pair (g, g + 1), g even, p 16-B aligned (engine buffers)
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ ulonglong2 ld2(const u64 *p, u64 g)
{
    const u64x2 w = *reinterpret_cast<const u64x2 *>(p + g);
    return make_ulonglong2(w.x, w.y);
}
// Non-temporal stores for the step's large streaming intermediates (round 6): each is written once and read by a
// later kernel, and none fits the caches (GB per launch), so keeping their lines only delays write-back into the next
// kernel's time.  Bits of HEC_NT_MASK: 1 the fan-outs' target tiles (Z, mod-up pass-A tiles), 2 the divide-and-round
// output, 4 the hoisted MAC's accumulators; the hoisted digits E are Ctx::nt_e (ModUpIO_BT).
#ifndef HEC_NT_MASK
#define HEC_NT_MASK 0
#endif
constexpr int kNtMask = HEC_NT_MASK;
template <int BIT>
__device__ __forceinline__ void st1m(u64 *p, u64 v)
{
    if constexpr ((kNtMask & BIT) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <int BIT>
__device__ __forceinline__ void st2m(u64 *p, ulonglong2 v)
{
    u64x2 w;
    w.x = v.x;
    w.y = v.y;
    if constexpr ((kNtMask & BIT) != 0) __builtin_nontemporal_store(w, reinterpret_cast<u64x2 *>(p));
    else *reinterpret_cast<u64x2 *>(p) = w;
}
// a non-temporal 16-B store (the nt cache policy: the line is not kept for reuse)
__device__ __forceinline__ void st2_nt(u64 *p, u64 g, u64 a, u64 b)
{
    u64x2 w;
    w.x = a;
    w.y = b;
    __builtin_nontemporal_store(w, reinterpret_cast<u64x2 *>(p + g));
}
__device__ __forceinline__ void st2(u64 *p, u64 g, u64 a, u64 b)
{
    u64x2 w;
    w.x = a;
    w.y = b;
    *reinterpret_cast<u64x2 *>(p + g) = w;
}

// job -> (poly = job / nl, limb = job % nl); src/dst may alias (in place).  elt != 1 loads through the
// Galois permutation (apply_galois_ntt fused into the load: src[galois_src(g)]).
struct StridedIO {
    const u64 *src;
    u64 *dst;
    u64 ps_src, ps_dst;
    int nl, logN;
    u32 elt;
    int pmap[HEC_MAXL + 1];
    struct Bound {
        const u64 *s;
        u64 *d;
        int prime;
        u32 elt;
        int logN;
        bool valid = true;
        struct Pre {};
        __device__ Pre pre(u64) const { return {}; }
        __device__ u64 load(u64 g) const { return s[elt == 1 ? g : galois_src((u32)g, elt, logN)]; }
        __device__ void store(u64 g, u64 v, Pre) const { d[g] = v; }
    };
    __device__ Bound bind(int job) const
    {
        const int poly = job / nl, limb = job % nl;
        return Bound{src + (u64)poly * ps_src + ((u64)limb << logN), dst + (u64)poly * ps_dst + ((u64)limb << logN),
                     pmap[limb], elt, logN};
    }
};

// Key-switch mod-up: job t -> (b, I, J), I in [0, l] (I == l is the special prime P), J in [0, l),
// I != J.  E layout [b][I][J][N].
// With Il set (a class-filtered launch) job -> (b, I = Il[.], J in [0, l)), the J == I jobs being empty.
struct ModUpMap {
    int l, logN, kP;
    const int *Il = nullptr;
    int nI = 0;
    __device__ void map(int job, int &b, int &I, int &J) const
    {
        if (Il) {
            const int per = nI * l;
            b = job / per;
            const int t = job % per;
            I = Il[t / l];
            J = t % l;
            return;
        }
        const int per = l * l;
        b = job / per;
        const int t = job % per;
        if (t < l * (l - 1)) {
            I = t / (l - 1);
            const int r = t % (l - 1);
            J = r < I ? r : r + 1;
        } else {
            I = l;
            J = t - l * (l - 1);
        }
    }
    __device__ u64 eoff(int b, int I, int J) const { return ((u64)((b * (l + 1) + I) * l + J)) << logN; }
};
struct ModUpIO_A {  // load digit J (coefficient form, canonical mod q_J) reduced mod q_I
    ModUpMap m;
    const u64 *D;
    u64 *E;
    const DevPrime *primes;
    struct Bound {
        const u64 *s;
        u64 *d;
        u64 q, r1;
        int prime;
        bool valid = true;
        struct Pre {};
        __device__ Pre pre(u64) const { return {}; }
        __device__ u64 load(u64 g) const { return barrett64(s[g], q, r1); }
        __device__ void store(u64 g, u64 v, Pre) const { d[g] = v; }
    };
    __device__ Bound bind(int job) const
    {
        int b, I, J;
        m.map(job, b, I, J);
        const int p = I == m.l ? m.kP : I;
        return Bound{D + ((u64)(b * m.l + J) << m.logN), E + m.eoff(b, I, J), primes[p].q, primes[p].r1, p, I != J};
    }
};
// NT: the digits stored non-temporally (HEC_NT_E, A/B)
template <bool NT>
struct ModUpIO_BT {
    ModUpMap m;
    u64 *E;
    int mform = 0;  // 1: the final store writes the MAC form k_hmacm reads (mform(), round 6)
    struct Bound {
        u64 *p;
        int prime;
        bool valid = true;
        bool mform = false;
        static constexpr bool kPair = true;
        static constexpr bool kMForm = true;
        struct Pre {};
        __device__ Pre pre(u64) const { return {}; }
        __device__ u64 load(u64 g) const { return p[g]; }
        __device__ void store(u64 g, u64 v, Pre) const
        {
            if constexpr (NT) __builtin_nontemporal_store(v, p + g);
            else p[g] = v;
        }
        __device__ ulonglong2 load2(u64 g) const { return ld2(p, g); }
        __device__ void pre2(u64, Pre &, Pre &) const {}
        __device__ void store2(u64 g, u64 a, u64 b, Pre, Pre) const
        {
            if constexpr (NT) st2_nt(p, g, a, b);
            else st2(p, g, a, b);
        }
    };
    __device__ Bound bind(int job) const
    {
        int b, I, J;
        m.map(job, b, I, J);
        return Bound{E + m.eoff(b, I, J), I == m.l ? m.kP : I, I != J, mform != 0};
    }
};

using ModUpIO_B = ModUpIO_BT<false>;

// Divide-and-round by a prime `last` (key-switch mod-down by P, or rescale by q_{l-1}):
// pass A loads y (coefficient form of the last limb, canonical mod last) and emits
//   ((y + h) mod last) mod q_i + (q_i - h mod q_i),  h = last >> 1     (in [0, 2 q_i))
// pass B stores  OUT = IN + (X - NTT(that)) * last^-1 mod q_i.
struct DivRoundIO_A {
    const u64 *Y;
    u64 ysb, ysk;
    u64 *Z;
    int nk, nl, logN;
    u64 last, half;
    const DevPrime *primes;
    u64 fix[HEC_MAXL];
    struct Bound {
        const u64 *y;
        u64 *z;
        u64 last, half, q, r1, fix;
        int prime;
        bool valid = true;
        struct Pre {};
        __device__ Pre pre(u64) const { return {}; }
        __device__ u64 load(u64 g) const
        {
            u64 v = y[g] + half;
            v = v >= last ? v - last : v;
            return barrett64(v, q, r1) + fix;
        }
        __device__ void store(u64 g, u64 v, Pre) const { z[g] = v; }
    };
    __device__ Bound bind(int job) const
    {
        const int i = job % nl, t = job / nl, k = t % nk, b = t / nk;
        return Bound{Y + b * ysb + k * ysk, Z + ((u64)job << logN), last, half, primes[i].q, primes[i].r1, fix[i], i};
    }
};
// Bound types whose pass B moves word pairs (load2 / pre2 / store2; HasPair).  Only the mod-up pass B (1,046-1,059
// vs 1,088-1,095 ms per step, round 4): the divide-and-round pass B measured slower with pairs (2,011-2,026 vs
// 1,852 ms) and so did the plain strided forward pass B (cfg2: 0.0762 vs 0.0681 ms per launch)
template <class T, class = void>
struct HasPair : std::false_type {};
template <class T>
struct HasPair<T, std::void_t<decltype(T::kPair)>> : std::bool_constant<T::kPair> {};
// Bound types whose post-op operands are loaded at the store instead of before the rounds (HasLatePre)
template <class T, class = void>
struct HasLatePre : std::false_type {};
template <class T>
struct HasLatePre<T, std::void_t<decltype(T::kLatePre)>> : std::bool_constant<T::kLatePre> {};
// Bound types whose final store may write the MAC form (a run-time flag `mform`, HasMForm)
template <class T, class = void>
struct HasMForm : std::false_type {};
template <class T>
struct HasMForm<T, std::void_t<decltype(T::kMForm)>> : std::bool_constant<T::kMForm> {};
// Bound types with a store_fp(g, double, Pre, prime) post-op for FP64 primes (HasFpStore)
template <class T, class = void>
struct HasFpStore : std::false_type {};
template <class T>
struct HasFpStore<T, std::void_t<decltype(T::kFpStore)>> : std::bool_constant<T::kFpStore> {};

// HAS_IN = false: no IN term (the hoisted children's mod-downs, whose IN the sibling-fused MAC already folded into
// ACC as IN P mod q_i).  The post-op then has one operand, loaded at the store (kLatePre): 104 instead of 209 VGPRs,
// 4 waves/SIMD (preloaded before the rounds: 142 VGPRs, 3 waves, 20-30 ms per step slower at B = 192)
template <bool HAS_IN>
struct DivRoundIOB {
    u64 *Z;
    PolyArr X, IN, OUT;
    int nk, nl, logN, in_nk;  // IN is added for polys k < in_nk only
    u32 elt;                  // IN is read through the Galois permutation (elt != 1)
    int fpstore;              // FP64 primes: the post-op in FP64 (store_fp)
    const DevPrime *primes;
    u64 inv[HEC_MAXL], inv_q[HEC_MAXL];
    struct Bound {
        static constexpr bool kFpStore = true;
        static constexpr bool kLatePre = !HAS_IN;  // the one operand is loaded at the store (4 waves/SIMD)
        const u64 *z, *x, *in;
        u64 *out;
        u64 q, w, wq;
        int prime;
        u32 elt;
        int logN;
        bool fpstore;
        bool valid = true;
        struct Pre {  // operands of the post-op, loaded before the butterfly rounds
            u64 x, in;
        };
        __device__ Pre pre(u64 g) const
        {
            if constexpr (!HAS_IN) return Pre{x[g], 0};
            else return Pre{x[g], in ? in[elt == 1 ? g : galois_src((u32)g, elt, logN)] : 0};
        }
        __device__ u64 load(u64 g) const { return z[g]; }
        __device__ void store(u64 g, u64 v, Pre p) const
        {
            u64 r = shoup(p.x + q - v, w, wq, q);
            if (HAS_IN && in) r = addmod(r, p.in, q);
            st1m<2>(out + g, r);
        }
        // v: the FP64 NTT output before canonicalisation (|v| < 10 q): (x - v) P^-1 (+ in) with one exact
        // fp_mulmod (|x - v| < 11 q) and one canonicalisation, instead of Shoup on u64 plus fp_canon
        __device__ void store_fp(u64 g, double v, Pre p, const DevPrime &pr) const
        {
            double r = fp_mulmod(u2d(p.x) - v, u2d(w), pr.qd, pr.qinv);
            if (HAS_IN && in) r += u2d(p.in);
            st1m<2>(out + g, fp_canon(r, pr.qd, pr.qinv));
        }
    };
    __device__ Bound bind(int job) const
    {
        const int i = job % nl, t = job / nl, k = t % nk, b = t / nk;
        const u64 li = (u64)i << logN;
        return Bound{Z + ((u64)job << logN), X.p + b * X.sb + k * X.sk + li,
                     (IN.p && k < in_nk) ? IN.p + b * IN.sb + k * IN.sk + li : nullptr, OUT.p + b * OUT.sb + k * OUT.sk + li,
                     primes[i].q, inv[i], inv_q[i], i, elt, logN, fpstore != 0};
    }
};
using DivRoundIO_B = DivRoundIOB<true>;

// =============================================================================== NTT core ==
// Twiddle tables per prime: integer {w, w_shoup} pairs (60-bit primes) and integer-valued doubles
// (primes < 2^42, FP64 arithmetic), each in SEAL order for pass A and re-laid for pass B.
struct TwTables {
    const ulonglong2 *a, *b;  // integer: pass A (SEAL order), pass B ([s][i][chunk])
    const double *fa, *fb;    // FP64 twins
    const u64 *sa = nullptr;  // w 2^31 mod q for a (the split-input Shoup butterflies, hec_device.h)
    const u64 *sb = nullptr;  // the same for b
};

// One round: stages [S0, S1) of a P = 2^LOGP point sub-transform.  Thread `ts` of its segment owns
// EPT elements = EPT / 2^D groups of 2^D elements (D = S1 - S0).  FP selects the arithmetic: the LDS
// words then hold the bits of integer-valued doubles.  TO_REG keeps the results in `regs` (group
// order: regs[gi 2^D + a]) instead of writing them back to LDS; in a final round (S1 == LOGP) the
// thread's EPT elements are then the consecutive slots ts*EPT .. ts*EPT + EPT - 1.
// Twiddle getters: (global stage s, index i within the stage) -> w.  GlobalTw reads the SEAL-ordered /
// pass-B re-laid tables in HBM (L2-resident); LdsTw a per-segment copy staged in LDS.
template <class IdxF>
struct GlobalTw {
    IdxF idx;
    const ulonglong2 *tw;
    const double *twf;
    __device__ double f(int s, int i) const { return twf[idx(s, i)]; }
    __device__ ulonglong2 w(int s, int i) const { return tw[idx(s, i)]; }
};
// The SEAL-ordered table read through the constant address space: with a block-uniform index the loads are scalar
// (s_load, counted by lgkmcnt), so they never wait behind the wave's outstanding vector stores and loads (on CDNA
// a vector load's vmcnt wait also waits for every store issued before it)
struct ConstTw {
    typedef __attribute__((address_space(4))) const double cdouble;
    typedef __attribute__((address_space(4))) const u64 cword;
    const ulonglong2 *tw;
    const double *twf;
    __device__ double f(int s, int i) const { return ((cdouble *)twf)[(1u << s) + (unsigned)i]; }
    __device__ ulonglong2 w(int s, int i) const
    {
        const unsigned k = 2 * ((1u << s) + (unsigned)i);
        const u64 a = ((cword *)tw)[k], b = ((cword *)tw)[k + 1];
        return ulonglong2{a, b};
    }
};
// The same SEAL-ordered tables with the split-input Shoup word a = w 2^31 mod q of each integer twiddle (kSplit):
// the integer butterflies then run shoup_split_lazy (8 instead of 10 32-bit multiplies, hec_device.h)
template <class IdxF>
struct GlobalTwS : GlobalTw<IdxF> {
    static constexpr bool kSplit = true;
    const u64 *ta;
    __device__ u64 a(int s, int i) const { return ta[this->idx(s, i)]; }
};
struct ConstTwS : ConstTw {
    static constexpr bool kSplit = true;
    const u64 *ta;
    __device__ u64 a(int s, int i) const
    {
        typedef __attribute__((address_space(4))) const u64 cword;
        return ((cword *)ta)[(1u << s) + (unsigned)i];
    }
};
struct LdsTwS;
template <class T, class = void>
struct HasSplitTw : std::false_type {};
template <class T>
struct HasSplitTw<T, std::void_t<decltype(T::kSplit)>> : std::bool_constant<T::kSplit> {};

struct LdsTw {  // entry k = 2^s - 1 + i of this segment; FP: one word (double bits), integer: {w, w_shoup}
    const u64 *row;
    __device__ double f(int s, int i) const { return __longlong_as_double((long long)row[(1 << s) - 1 + i]); }
    __device__ ulonglong2 w(int s, int i) const
    {
        const u64 *p = row + 2 * ((1 << s) - 1 + i);
        return ulonglong2{p[0], p[1]};
    }
};
struct LdsTwS : LdsTw {  // with the split-input Shoup words (entry k of arow)
    static constexpr bool kSplit = true;
    const u64 *arow;
    __device__ u64 a(int s, int i) const { return arow[(1 << s) - 1 + i]; }
};

// The D = S1 - S0 stages of one element group (NQ = 2^D registers): group g of a round, hi = its index above
// the round's stages.  Round-stage st uses twiddle twidx(S0+st, hi 2^st + m), m = a >> (D - st) the top st bits
// of the element slot a.  The group's 2^D - 1 twiddles do not depend on data: GroupTw loads them first, so their
// latency overlaps the data loads.
template <int S0, int D, bool FP, bool SPL = false>
struct GroupTw {
    static constexpr int NQ = 1 << D;
    double wf[FP ? NQ - 1 : 1];
    ulonglong2 wi[FP ? 1 : NQ - 1];
    u64 wa[(FP || !SPL) ? 1 : NQ - 1];  // SPL: the split-input words (a TwG with kSplit)
    template <class TwG>
    __device__ __forceinline__ void load(int hi, const TwG &twg)
    {
#pragma unroll
        for (int st = 0; st < D; ++st)
#pragma unroll
            for (int m = 0; m < (1 << st); ++m) {
                if constexpr (FP) wf[(1 << st) - 1 + m] = twg.f(S0 + st, (hi << st) | m);
                else wi[(1 << st) - 1 + m] = twg.w(S0 + st, (hi << st) | m);
                if constexpr (!FP && SPL) wa[(1 << st) - 1 + m] = twg.a(S0 + st, (hi << st) | m);
            }
    }
    template <bool INV>
    __device__ __forceinline__ void run(u64 *v, const DevPrime &pr) const
    {
        const u64 q = pr.q, two_q = 2 * q;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const int st = INV ? D - 1 - k : k;
            const int bit = 1 << (D - 1 - st);
#pragma unroll
            for (int a = 0; a < NQ; ++a) {
                if (a & bit) continue;
                const int wk = (1 << st) - 1 + (a >> (D - st));
                if constexpr (FP) {
                    double X = __longlong_as_double((long long)v[a]), Y = __longlong_as_double((long long)v[a | bit]);
                    if constexpr (!INV) ct_bfly_fp(X, Y, wf[wk], pr.qd, pr.qinv);
                    else gs_bfly_fp(X, Y, wf[wk], pr.qd, pr.qinv);
                    v[a] = (u64)__double_as_longlong(X);
                    v[a | bit] = (u64)__double_as_longlong(Y);
                } else if constexpr (SPL) {
                    if constexpr (!INV) ct_bfly_s(v[a], v[a | bit], wi[wk].x, wi[wk].y, wa[wk], q, two_q);
                    else gs_bfly_s(v[a], v[a | bit], wi[wk].x, wi[wk].y, wa[wk], q, two_q);
                } else {
                    if constexpr (!INV) ct_bfly(v[a], v[a | bit], wi[wk].x, wi[wk].y, q, two_q);
                    else gs_bfly(v[a], v[a | bit], wi[wk].x, wi[wk].y, q, two_q);
                }
            }
        }
    }
};

// One round (stages [S0, S1)) of a P = 2^LOGP point transform through LDS: thread ts owns G = EPT / 2^D groups;
// group g holds the elements xb | (a << (LOGP - S1)), xb = (hi << (LOGP - S0)) | lo, g = hi 2^(LOGP - S1) + lo.
template <int LOGP, int S0, int S1, int EPT, bool INV, bool FP, bool TO_REG, class AddrF, class TwG>
__device__ __forceinline__ void ntt_round_g(u64 *lds, const AddrF &addr, int ts, const TwG &twg, const DevPrime &pr,
                                            u64 *regs)
{
    constexpr int LE = EPT == 16 ? 4 : EPT == 8 ? 3 : EPT == 4 ? 2 : 1;
    constexpr int D = S1 - S0, G = 1 << (LE - D), NQ = 1 << D;
    static_assert(D >= 1 && D <= LE, "round covers 1..log2(EPT) stages");
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int g = ts * G + gi;
        const int lo = g & ((1 << (LOGP - S1)) - 1);
        const int hi = g >> (LOGP - S1);
        const int xb = (hi << (LOGP - S0)) | lo;
        GroupTw<S0, D, FP, !FP && HasSplitTw<TwG>::value> gt;
        gt.load(hi, twg);
        u64 v[NQ];
#pragma unroll
        for (int a = 0; a < NQ; ++a) v[a] = lds[addr(xb | (a << (LOGP - S1)))];
        gt.template run<INV>(v, pr);
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
            if constexpr (TO_REG) regs[gi * NQ + a] = v[a];
            else lds[addr(xb | (a << (LOGP - S1)))] = v[a];
        }
    }
}

// a round of the 16-element LDS pass (stages [S0, S1)) with its groups' twiddles already loaded: gts[gi] is group
// gi's GroupTw (ntt_round_g's groups: g = ts G + gi)
template <int LOGP, int S0, int S1, bool INV, bool FP, class AddrF>
__device__ __forceinline__ void ntt_round_pre(u64 *lds, const AddrF &addr, int ts, const GroupTw<S0, S1 - S0, FP> *gts,
                                              const DevPrime &pr)
{
    constexpr int D = S1 - S0, G = 1 << (4 - D), NQ = 1 << D;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int g = ts * G + gi;
        const int lo = g & ((1 << (LOGP - S1)) - 1), hi = g >> (LOGP - S1);
        const int xb = (hi << (LOGP - S0)) | lo;
        u64 v[NQ];
#pragma unroll
        for (int a = 0; a < NQ; ++a) v[a] = lds[addr(xb | (a << (LOGP - S1)))];
        gts[gi].template run<INV>(v, pr);
#pragma unroll
        for (int a = 0; a < NQ; ++a) lds[addr(xb | (a << (LOGP - S1)))] = v[a];
    }
}

// the two-pass NTT's rounds: 16 elements per thread, stages [4 RND, min(4 RND + 4, LOGP))
template <int LOGP, int RND, bool INV, bool FP, class AddrF, class TwF>
__device__ __forceinline__ void ntt_round(u64 *lds, const AddrF &addr, int ts, const TwF &twidx, const ulonglong2 *tw,
                                          const double *twf, const DevPrime &pr)
{
    constexpr int S0 = RND * 4;
    constexpr int S1 = (S0 + 4 < LOGP) ? S0 + 4 : LOGP;
    const GlobalTw<TwF> twg{twidx, tw, twf};
    ntt_round_g<LOGP, S0, S1, 16, INV, FP, false>(lds, addr, ts, twg, pr, nullptr);
}

template <int LOGP, int NSEG, bool INV, bool PASS_A, bool FINAL, bool FP, class Bound>
__device__ __forceinline__ void ntt_pass_body(u64 *lds, const Bound &bio, const DevPrime &pr, const TwTables &tt,
                                              int logN)
{
    constexpr int P = 1 << LOGP, TPS = P / 16, THREADS = NSEG * TPS;
    // PAIR: pass B moves word pairs (x, x + 1) of a chunk per lane: 16-B loads and stores (8 per thread instead
    // of 16 8-B ones; the IO's load2 / pre2 / store2)
    constexpr bool PAIR = !PASS_A && HasPair<Bound>::value;
    // SWZ (the pair path, round 6): unpadded chunk rows with word x of segment sg at x ^ sg.  The padded rows (P + 1
    // words) put an odd row's pairs at 8-B-aligned addresses, so each pair moved as two strided 8-B LDS accesses:
    // 2.67 bank-conflict cycles per LDS instruction in the mod-up pass B (profiles/r06t_sq_final_by_instance_B128.json).
    // Swizzled, a pair is one aligned 16-B slot (its two words swapped in odd rows), and the rounds' accesses (16
    // segments at one x) still fall on 16 distinct bank pairs.
    constexpr bool SWZ = PAIR && NSEG <= P;
    constexpr int LD = PASS_A ? (NSEG + 1) : (SWZ ? P : P + 1);
    constexpr bool FIRST = !FINAL;  // forward: A then B; inverse: B then A
    (void)TPS;
    const u64 q = pr.q, two_q = 2 * q;
    const int seg0 = blockIdx.x * NSEG;
    const int lc = logN - LOGP;  // pass A: log2(#columns)
    const ulonglong2 *tw = (PASS_A ? tt.a : tt.b) + ((u64)bio.prime << logN);
    const double *twf = (PASS_A ? tt.fa : tt.fb) + ((u64)bio.prime << logN);

    constexpr int PB2 = P / 2;
    if constexpr (!PAIR) {
        // every tile load issued before the first LDS store (round 6, VERDICT r05 item 5: with a load and its LDS
        // store per iteration the compiler waited for each load in turn whenever the IO's load has a branch, as
        // StridedIO's Galois permutation does: the plain forward pass B at cfg2 ran 0.0757-0.0794 instead of
        // 0.064 ms per launch, the round-4 code's rate, on one box)
        constexpr int NIT = P * NSEG / THREADS;
        u64 tv[NIT];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int li = threadIdx.x + it * THREADS;
            u64 g;
            if constexpr (PASS_A) g = ((u64)(li / NSEG) << lc) + seg0 + li % NSEG;
            else g = ((u64)(seg0 + li / P) << LOGP) + li % P;
            tv[it] = bio.load(g);
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int li = threadIdx.x + it * THREADS;
            int x, sg;
            if constexpr (PASS_A) { x = li / NSEG; sg = li % NSEG; }
            else { sg = li / P; x = li % P; }
            u64 v = tv[it];
            if constexpr (FP && FIRST) v = (u64)__double_as_longlong(u2d(v));  // integer input -> double bits
            lds[PASS_A ? x * LD + sg : sg * LD + x] = v;
        }
    } else {
#pragma unroll
        for (int it = 0; it < P * NSEG / THREADS / 2; ++it) {
            const int li = threadIdx.x + it * THREADS;
            const int sg = li / PB2, x = 2 * (li % PB2);
            const ulonglong2 w = bio.load2(((u64)(seg0 + sg) << LOGP) + x);
            u64 a = w.x, b = w.y;
            if constexpr (FP && FIRST) {
                a = (u64)__double_as_longlong(u2d(a));
                b = (u64)__double_as_longlong(u2d(b));
            }
            if constexpr (SWZ)
                *reinterpret_cast<ulonglong2 *>(lds + sg * LD + (x ^ (sg & ~1))) = (sg & 1) ? ulonglong2{b, a}
                                                                                        : ulonglong2{a, b};
            else {
                lds[sg * LD + x] = a;
                lds[sg * LD + x + 1] = b;
            }
        }
    }
    __syncthreads();

    const int ts = threadIdx.x / NSEG, sg = threadIdx.x % NSEG;
    // pass A: SEAL table index 2^s + i (shared by all columns: broadcast reads).
    // pass B: the per-chunk index (R + r) 2^s + i is served from the re-laid table
    //         twb[s][i][r] = tw[(R + r) 2^s + i] at R (2^s - 1) + i R + r, so lanes (consecutive
    //         chunks r) read consecutive entries.
    const u64 R = 1ull << (logN - LOGP), chunk = (u64)(seg0 + sg);
    auto twidx = [=](int s, int i) -> u64 {
        if constexpr (PASS_A) return (1ull << s) + (u64)i;
        else return R * ((1ull << s) - 1) + (u64)i * R + chunk;
    };
    // a forward final pass loads round 0's twiddles before the post-op operands: vector loads complete in issue
    // order (one vmcnt), so round 0 then waits for its twiddles only and the operands arrive under its work
    // (divide-and-round pass B 1,852 vs 1,886 ms per step; round 1's as well at FP64 primes measured slower, 1,890)
    constexpr bool TW0 = FINAL && !INV;
    GroupTw<0, 4, FP> gt0[1];
    if constexpr (TW0) gt0[0].load(ts >> (LOGP - 4), GlobalTw<decltype(twidx)>{twidx, tw, twf});
    // post-op operands of this thread's output words: issue their loads now so they overlap the rounds
    constexpr int ITS = P * NSEG / THREADS;
    // (for the two-operand divide-and-round, loading them at the store instead frees 64+ VGPRs but measured slower:
    // 1313 vs 1271 ms/step; its one-operand form without IN does load at the store, HasLatePre)
    constexpr bool LATE = HasLatePre<Bound>::value;
    typename Bound::Pre pre[FINAL ? ITS : 1];
    if constexpr (FINAL && !LATE) {
        if constexpr (!PAIR) {
#pragma unroll
            for (int it = 0; it < ITS; ++it) {
                const int li = threadIdx.x + it * THREADS;
                u64 g;
                if constexpr (PASS_A) g = ((u64)(li / NSEG) << lc) + seg0 + li % NSEG;
                else g = ((u64)(seg0 + li / P) << LOGP) + li % P;
                pre[it] = bio.pre(g);
            }
        } else {
#pragma unroll
            for (int it = 0; it < ITS / 2; ++it) {
                const int li = threadIdx.x + it * THREADS;
                bio.pre2(((u64)(seg0 + li / PB2) << LOGP) + 2 * (li % PB2), pre[2 * it], pre[2 * it + 1]);
            }
        }
    }
    auto addr = [sg](int x) { return PASS_A ? x * LD + sg : sg * LD + (SWZ ? (x ^ sg) : x); };
    if constexpr (!INV) {
        if constexpr (TW0) ntt_round_pre<LOGP, 0, 4, false, FP>(lds, addr, ts, gt0, pr);
        else ntt_round<LOGP, 0, false, FP>(lds, addr, ts, twidx, tw, twf, pr);
        __syncthreads();
        ntt_round<LOGP, 1, false, FP>(lds, addr, ts, twidx, tw, twf, pr);
    } else {
        ntt_round<LOGP, 1, true, FP>(lds, addr, ts, twidx, tw, twf, pr);
        __syncthreads();
        ntt_round<LOGP, 0, true, FP>(lds, addr, ts, twidx, tw, twf, pr);
    }
    __syncthreads();

    if constexpr (PAIR) {
#pragma unroll
        for (int it = 0; it < ITS / 2; ++it) {
            const int li = threadIdx.x + it * THREADS;
            const int s2 = li / PB2, x = 2 * (li % PB2);
            u64 a, b;
            if constexpr (SWZ) {
                const ulonglong2 w = *reinterpret_cast<const ulonglong2 *>(lds + s2 * LD + (x ^ (s2 & ~1)));
                a = (s2 & 1) ? w.y : w.x;
                b = (s2 & 1) ? w.x : w.y;
            } else {
                a = lds[s2 * LD + x];
                b = lds[s2 * LD + x + 1];
            }
            const u64 g = ((u64)(seg0 + s2) << LOGP) + x;
            if constexpr (FINAL) {
                if constexpr (FP) {
                    double da = __longlong_as_double((long long)a), db = __longlong_as_double((long long)b);
                    if constexpr (INV) {
                        da = fp_mulmod(da, pr.ninv_d, pr.qd, pr.qinv);
                        db = fp_mulmod(db, pr.ninv_d, pr.qd, pr.qinv);
                    }
                    if constexpr (HasMForm<Bound>::value) {
                        if (bio.mform) {  // MAC form: the canonical integer-valued double itself
                            a = (u64)__double_as_longlong(fp_canon_d(da, pr.qd, pr.qinv));
                            b = (u64)__double_as_longlong(fp_canon_d(db, pr.qd, pr.qinv));
                            bio.store2(g, a, b, pre[2 * it], pre[2 * it + 1]);
                            continue;
                        }
                    }
                    a = fp_canon(da, pr.qd, pr.qinv);
                    b = fp_canon(db, pr.qd, pr.qinv);
                } else if constexpr (!INV) {
                    a = csub(csub(a, two_q), q);
                    b = csub(csub(b, two_q), q);
                } else {
                    a = shoup(a, pr.ninv, pr.ninv_q, q);
                    b = shoup(b, pr.ninv, pr.ninv_q, q);
                }
                bio.store2(g, a, b, pre[2 * it], pre[2 * it + 1]);
            } else {
                bio.store2(g, a, b, typename Bound::Pre{}, typename Bound::Pre{});
            }
        }
        return;
    }
    if constexpr (FINAL && LATE && !PAIR) {  // the operands now, all issued before the first store
#pragma unroll
        for (int it = 0; it < ITS; ++it) {
            const int li = threadIdx.x + it * THREADS;
            if constexpr (PASS_A) pre[it] = bio.pre(((u64)(li / NSEG) << lc) + seg0 + li % NSEG);
            else pre[it] = bio.pre(((u64)(seg0 + li / P) << LOGP) + li % P);
        }
    }
#pragma unroll
    for (int it = 0; it < P * NSEG / THREADS; ++it) {
        const int li = threadIdx.x + it * THREADS;
        u64 v, g;
        if constexpr (PASS_A) {
            const int x = li / NSEG, s2 = li % NSEG;
            v = lds[x * LD + s2];
            g = ((u64)x << lc) + seg0 + s2;
        } else {
            const int s2 = li / P, x = li % P;
            v = lds[s2 * LD + x];
            g = ((u64)(seg0 + s2) << LOGP) + x;
        }
        if constexpr (FINAL) {
            if constexpr (FP) {
                double d = __longlong_as_double((long long)v);
                if constexpr (INV) d = fp_mulmod(d, pr.ninv_d, pr.qd, pr.qinv);
                if constexpr (HasFpStore<Bound>::value) {  // the post-op in FP64 on the uncanonicalised value
                    if (bio.fpstore) {
                        bio.store_fp(g, d, pre[it], pr);
                        continue;
                    }
                }
                v = fp_canon(d, pr.qd, pr.qinv);
            } else {
                if constexpr (!INV) v = csub(csub(v, two_q), q);
                else v = shoup(v, pr.ninv, pr.ninv_q, q);
            }
            bio.store(g, v, pre[it]);
        } else {
            bio.store(g, v, typename Bound::Pre{});
        }
    }
}

// ------------------------------------------------------------------ register-direct NTT pass (RD)
// One round on 16 register-resident elements (the twiddles of each group issued first): thread ts holds, for
// stages [S0, S1), v[gi 2^D + a] <-> x = xb(ts G + gi) | (a << (LOGP - S1)) as in ntt_round_g.
template <int LOGP, int S0, int S1, bool INV, bool FP, class TwG>
__device__ __forceinline__ void ntt_round_rg(u64 *v, int ts, const TwG &twg, const DevPrime &pr)
{
    constexpr int D = S1 - S0, G = 1 << (4 - D), NQ = 1 << D;
    static_assert(D >= 1 && D <= 4, "round covers 1..4 stages");
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        GroupTw<S0, D, FP> gt;
        gt.load((ts * G + gi) >> (LOGP - S1), twg);
        gt.template run<INV>(v + gi * NQ, pr);
    }
}

// LDS word stride of a pass-B chunk in ntt_pass_body_rd: at least P + P/8 (two pad words per 16 elements) and
// 16 mod 32, so the 16-B pair reads of two chunks fill the 64 banks and the 16-element block reads of 8 threads
// land 36 dwords apart
constexpr int nttb_ld(int logp) { return ((1 << logp) + (1 << logp) / 8 + 15) / 32 * 32 + 16; }

// A pass of the two-pass NTT with its rounds on registers (k_fan2's scheme for k_ntt).  Rounds [0, SM) and
// [SM, LOGP), SM = LOGP - 4, on two element sets of a P-point column / chunk per thread ts:
//   set 0 (stages [0, SM)): x0(k) = ts G0 + k / 2^SM + 16 (k % 2^SM), G0 = 2^(4 - SM)
//                           (pass A at P = 256: the stride set ts + 16 k; pass B at P = 128: pairs x, x + 1)
//   set 1 (stages [SM, LOGP)): x1(k) = 16 ts + k (the block set).
// Pass A (columns, lanes = consecutive columns): both sets load and store coalesced, so a pass exchanges
// through LDS once instead of three times.  Pass B (contiguous chunks, lanes = consecutive pairs of a chunk):
// set 0 is coalesced (16-B pairs), set 1 is not, so the forward pass stores through one more exchange and the
// inverse pass loads through one (two exchanges instead of three).
template <int LOGP, int NSEG, bool INV, bool PASS_A, bool FINAL, bool FP, class Bound>
__device__ __forceinline__ void ntt_pass_body_rd(u64 *lds, const Bound &bio, const DevPrime &pr, const TwTables &tt,
                                                 int logN)
{
    constexpr int P = 1 << LOGP, TPS = P / 16, SM = LOGP - 4, NQ0 = 1 << SM, G0 = 16 / NQ0;
    constexpr int LDA = NSEG + 1, LDB = nttb_ld(LOGP), TILE = PASS_A ? P * LDA : NSEG * LDB;
    constexpr bool FIRST = !FINAL;
    static_assert(LOGP >= 5 && LOGP <= 8, "two rounds: [0, LOGP - 4) and 4 stages");
    const u64 q = pr.q, two_q = 2 * q;
    const int seg0 = blockIdx.x * NSEG, lc = logN - LOGP;
    const ulonglong2 *tw = (PASS_A ? tt.a : tt.b) + ((u64)bio.prime << logN);
    const double *twf = (PASS_A ? tt.fa : tt.fb) + ((u64)bio.prime << logN);
    const int ts = PASS_A ? (int)threadIdx.x / NSEG : (int)threadIdx.x % TPS;
    const int sg = PASS_A ? (int)threadIdx.x % NSEG : (int)threadIdx.x / TPS;
    auto gidx = [&](int x) -> u64 { return PASS_A ? ((u64)x << lc) + seg0 + sg : ((u64)(seg0 + sg) << LOGP) + x; };
    auto addr = [sg](int x) { return PASS_A ? x * LDA + sg : sg * LDB + x + 2 * (x >> 4); };
    auto x0 = [ts](int k) { return ts * G0 + k / NQ0 + 16 * (k % NQ0); };
    auto x1 = [ts](int k) { return 16 * ts + k; };
    const u64 R = 1ull << lc, chunk = (u64)(seg0 + sg);
    auto twidx = [=](int s, int i) -> u64 {
        if constexpr (PASS_A) return (1ull << s) + (u64)i;
        else return R * ((1ull << s) - 1) + (u64)i * R + chunk;
    };
    const GlobalTw<decltype(twidx)> twg{twidx, tw, twf};
    constexpr bool IN_X1 = INV;              // the first round's set: forward set 0, inverse set 1
    constexpr bool OUT_X1 = !INV;            // the last round's set
    constexpr bool IN_T = !PASS_A && IN_X1;  // pass B loads set 1 through an LDS transposition
    constexpr bool OUT_T = !PASS_A && OUT_X1;
    auto xin = [&](int k) { return (IN_X1 && !IN_T) ? x1(k) : x0(k); };    // loaded positions
    auto xout = [&](int k) { return (OUT_X1 && !OUT_T) ? x1(k) : x0(k); }; // stored positions
    // one LDS tile (a second one would halve the pass-B blocks per CU); a barrier before each reuse
    u64 *t0 = lds, *t1 = lds;
    auto ad0 = [&](int x) { return addr(x); };
    (void)TILE;

    u64 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        u64 t = bio.load(gidx(xin(k)));
        if constexpr (FP && FIRST) t = (u64)__double_as_longlong(u2d(t));  // integer input -> double bits
        v[k] = t;
    }
    typename Bound::Pre pre[FINAL ? 16 : 1];  // post-op operands of the outputs, issued before the rounds
    if constexpr (FINAL) {
#pragma unroll
        for (int k = 0; k < 16; ++k) pre[k] = bio.pre(gidx(xout(k)));
    }
    if constexpr (IN_T) {  // pass B inverse: loaded as set 0, the first round needs set 1
#pragma unroll
        for (int k = 0; k < 16; ++k) t1[ad0(x0(k))] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = t1[ad0(x1(k))];
        __syncthreads();  // the tile is rewritten by the round exchange
    }
    if constexpr (!INV) {
        ntt_round_rg<LOGP, 0, SM, false, FP>(v, ts, twg, pr);
#pragma unroll
        for (int k = 0; k < 16; ++k) t0[ad0(x0(k))] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = t0[ad0(x1(k))];
        ntt_round_rg<LOGP, SM, LOGP, false, FP>(v, ts, twg, pr);
    } else {
        ntt_round_rg<LOGP, SM, LOGP, true, FP>(v, ts, twg, pr);
#pragma unroll
        for (int k = 0; k < 16; ++k) t0[ad0(x1(k))] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = t0[ad0(x0(k))];
        ntt_round_rg<LOGP, 0, SM, true, FP>(v, ts, twg, pr);
    }
    if constexpr (OUT_T) {  // pass B forward: the last round left set 1, store set 0
        __syncthreads();  // every thread has read the round exchange
#pragma unroll
        for (int k = 0; k < 16; ++k) t1[ad0(x1(k))] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = t1[ad0(x0(k))];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const u64 g = gidx(xout(k));
        u64 val = v[k];
        if constexpr (FINAL) {
            if constexpr (FP) {
                double d = __longlong_as_double((long long)val);
                if constexpr (INV) d = fp_mulmod(d, pr.ninv_d, pr.qd, pr.qinv);
                val = fp_canon(d, pr.qd, pr.qinv);
            } else {
                if constexpr (!INV) val = csub(csub(val, two_q), q);
                else val = shoup(val, pr.ninv, pr.ninv_q, q);
            }
            bio.store(g, val, pre[k]);
        } else {
            bio.store(g, val, typename Bound::Pre{});
        }
    }
}

// ------------------------------------------------------------------ wave-shuffle forward pass B (round 6)
// The forward NTT's pass B at P = 128 (N = 2^15: stages 8..14, contiguous chunks of 128 words) with every exchange
// inside the wavefront (the north-star's "wavefront shuffles"): a chunk's 8 lanes hold 16 elements each, and the three
// stages whose butterfly distance is a lane bit are brought into registers by three exchange steps between partner
// lanes (DPP moves of the 32-bit halves), not through an LDS tile: no LDS, no workgroup barrier, every wave runs on
// its own.  Element x of the chunk (bits 0..6):
//   loaded:   lane L (0..7) holds x = 16 j + 2 L + h in v[2 j + h]   (16-B word pairs: coalesced 128-B runs)
//   stages 0..2 (distance bits 6, 5, 4 = register bits 3, 2, 1): in registers, two groups of 8 (h = 0, 1)
//   3 swaps (register bit 3 <-> lane bit 2, bit 2 <-> lane bit 1, bit 1 <-> lane bit 0): lane L' then holds
//             x = 16 L' + r in v[r]
//   stages 3..6 (distance bits 3..0 = register bits 3..0): in registers, one group of 16 (GroupTw<3, 4>)
//   stored:   16 consecutive words per lane (8 x 16-B pairs)
// A swap step trades 8 of a lane's 16 words with its partner lane: 16 dword DPP moves (xor 1 and 2: quad_perm;
// xor 4: row_shl:4 and row_shr:4 and a select by the lane bit) and selects on fixed register indices, no LDS access.
template <int M>
__device__ __forceinline__ u32 xor_lane32(u32 v)
{
    static_assert(M == 1 || M == 2 || M == 4, "partner lanes within 8");
    if constexpr (M == 1) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    else {
        const u32 hi = (u32)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xF, 0xF, false);  // row_shl:4: lane i <- i + 4
        const u32 lo = (u32)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, false);  // row_shr:4: lane i <- i - 4
        return (threadIdx.x & 4) ? lo : hi;
    }
}
template <int M>
__device__ __forceinline__ u64 xor_lane64(u64 v)
{
    return (u64)xor_lane32<M>((u32)v) | ((u64)xor_lane32<M>((u32)(v >> 32)) << 32);
}
// swap register bit RB with lane bit LB (lane = threadIdx.x & 7 within the chunk's 8 lanes); every register is
// assigned on both sides of the select, so v[] keeps fixed indices and stays in VGPRs
template <int RB, int LB>
__device__ __forceinline__ void swap_bits(u64 *v, int lane)
{
    const bool up = (lane >> LB) & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (r & (1 << RB)) continue;
        const int ra = r, rb = r | (1 << RB);           // register bit RB = 0 / 1
        const u64 a = v[ra], b = v[rb];
        const u64 recv = xor_lane64<1 << LB>(up ? a : b);  // the lower lane keeps its ra, the upper lane its rb
        v[ra] = up ? recv : a;
        v[rb] = up ? b : recv;
    }
}

// CO: the three swaps again after the last stages, back to the load layout (lane L holds x = 16 j + 2 L + h), so the
// stores are coalesced 128-B runs like the loads instead of 16 consecutive words per lane
template <bool FP, bool CO, class Bound>
__device__ __forceinline__ void nttb_shfl_body(const Bound &bio, const DevPrime &pr, const TwTables &tt, int logN)
{
    constexpr int LOGP = 7;
    const u64 q = pr.q, two_q = 2 * q;
    const int lane = threadIdx.x & 7;
    const u64 chunk = (u64)blockIdx.x * 32 + (threadIdx.x >> 3);
    const u64 base = chunk << LOGP;
    const u64 R = 1ull << (logN - LOGP);
    const ulonglong2 *tw = tt.b + ((u64)bio.prime << logN);
    const double *twf = tt.fb + ((u64)bio.prime << logN);
    auto twidx = [=](int s, int i) -> u64 { return R * ((1ull << s) - 1) + (u64)i * R + chunk; };
    const GlobalTw<decltype(twidx)> twg{twidx, tw, twf};
    u64 v[16];
    GroupTw<0, 3, FP> g0;
    g0.load(0, twg);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const u64 g = base + 16 * j + 2 * lane;
        if constexpr (HasPair<Bound>::value) {
            const ulonglong2 w = bio.load2(g);
            v[2 * j] = w.x;
            v[2 * j + 1] = w.y;
        } else {
            v[2 * j] = bio.load(g);
            v[2 * j + 1] = bio.load(g + 1);
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u64 grp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) grp[j] = v[2 * j + h];
        g0.template run<false>(grp, pr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[2 * j + h] = grp[j];
    }
    swap_bits<3, 2>(v, lane);
    swap_bits<2, 1>(v, lane);
    swap_bits<1, 0>(v, lane);
    // output position of v[r]: 16 consecutive words per lane, or (CO) the load layout
    auto opos = [&](int r) -> u64 {
        return CO ? base + 16 * (u64)(r >> 1) + 2 * (u64)lane + (r & 1) : base + 16 * (u64)lane + r;
    };
    constexpr bool LATE = HasLatePre<Bound>::value;
    typename Bound::Pre pre[16];
    if constexpr (!LATE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) pre[r] = bio.pre(opos(r));
    }
    GroupTw<3, 4, FP> g1;
    g1.load(lane, twg);
    g1.template run<false>(v, pr);
    if constexpr (CO) {
        swap_bits<1, 0>(v, lane);
        swap_bits<2, 1>(v, lane);
        swap_bits<3, 2>(v, lane);
    }
    if constexpr (LATE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) pre[r] = bio.pre(opos(r));
    }
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        u64 a = v[r], b = v[r + 1];
        const u64 g = opos(r);
        if constexpr (FP) {
            const double da = __longlong_as_double((long long)a), db = __longlong_as_double((long long)b);
            if constexpr (HasFpStore<Bound>::value) {
                if (bio.fpstore) {
                    bio.store_fp(g, da, pre[r], pr);
                    bio.store_fp(g + 1, db, pre[r + 1], pr);
                    continue;
                }
            }
            if constexpr (HasMForm<Bound>::value) {
                if (bio.mform) {
                    a = (u64)__double_as_longlong(fp_canon_d(da, pr.qd, pr.qinv));
                    b = (u64)__double_as_longlong(fp_canon_d(db, pr.qd, pr.qinv));
                } else {
                    a = fp_canon(da, pr.qd, pr.qinv);
                    b = fp_canon(db, pr.qd, pr.qinv);
                }
            } else {
                a = fp_canon(da, pr.qd, pr.qinv);
                b = fp_canon(db, pr.qd, pr.qinv);
            }
        } else {
            a = csub(csub(a, two_q), q);
            b = csub(csub(b, two_q), q);
        }
        if constexpr (HasPair<Bound>::value) {
            bio.store2(g, a, b, pre[r], pre[r + 1]);
        } else {
            bio.store(g, a, pre[r]);
            bio.store(g + 1, b, pre[r + 1]);
        }
    }
}

template <class IO, bool CO>
__global__ void __launch_bounds__(256) k_nttb_shfl(const IO io, TwTables tt, const DevPrime *__restrict__ primes,
                                                   int logN)
{
    const auto bio = io.bind(blockIdx.y);
    if (!bio.valid) return;  // uniform per block
    const DevPrime pr = primes[bio.prime];
    if (pr.fp) nttb_shfl_body<true, CO>(bio, pr, tt, logN);
    else nttb_shfl_body<false, CO>(bio, pr, tt, logN);
}

// A per-block branch on the prime's arithmetic class.  RD: the register-direct pass (ntt_pass_body_rd); otherwise
// every round through LDS (ntt_pass_body: the forward pass B, where register-direct measured slower)
template <int LOGP, int NSEG, bool INV, bool PASS_A, bool FINAL, class IO, bool RD = false>
__global__ void __launch_bounds__(NSEG *(1 << LOGP) / 16)
    k_ntt(const IO io, TwTables tt, const DevPrime *__restrict__ primes, int logN)
{
    static_assert(LOGP >= 5 && LOGP <= 8, "two rounds of 4 stages");
    constexpr int WORDS = !RD ? (PASS_A ? (1 << LOGP) * (NSEG + 1) : NSEG * ((1 << LOGP) + 1))
                              : (PASS_A ? (1 << LOGP) * (NSEG + 1) : NSEG * nttb_ld(LOGP));
    __shared__ __attribute__((aligned(16))) u64 lds[WORDS];  // 16-B pair accesses (SWZ)
    const auto bio = io.bind(blockIdx.y);
    if (!bio.valid) return;  // uniform per block
    const DevPrime pr = primes[bio.prime];
    if constexpr (RD) {
        if (pr.fp) ntt_pass_body_rd<LOGP, NSEG, INV, PASS_A, FINAL, true>(lds, bio, pr, tt, logN);
        else ntt_pass_body_rd<LOGP, NSEG, INV, PASS_A, FINAL, false>(lds, bio, pr, tt, logN);
    } else if (pr.fp) ntt_pass_body<LOGP, NSEG, INV, PASS_A, FINAL, true>(lds, bio, pr, tt, logN);
    else ntt_pass_body<LOGP, NSEG, INV, PASS_A, FINAL, false>(lds, bio, pr, tt, logN);
}

template <int LOGR, int LOGC, int NA, int NB, bool INV, class IO1, class IO2>
static void run_ntt2(Ctx &c, int njobs, const IO1 &first, const IO2 &second, int stages)
{
    constexpr int R = 1 << LOGR, C = 1 << LOGC;
    const dim3 gA(C / NA, njobs), gB(R / NB, njobs);
    constexpr int TA = NA * R / 16, TB = NB * C / 16;
    const TwTables fwd{c.tw, c.twb, c.twf, c.twbf}, inv{c.itw, c.itwb, c.itwf, c.itwbf};
    if constexpr (!INV) {  // the forward pass B stays on ntt_pass_body (register-direct measured slower:
                           // divide-and-round pass B 1,948 vs 1,894 ms, mod-up pass B 1,152 vs 1,077 ms per step;
                           // SQ counters: a third fewer LDS and VMEM instructions, no bank conflicts either way,
                           // but 2.2x the cycles waiting on load dependencies and 15 % more wave cycles)
        if (stages & 1) k_ntt<LOGR, NA, false, true, false, IO1, true><<<gA, TA, 0, c.stream>>>(first, fwd, c.primes, c.logN);
        if (stages & 2) {
            // the wave-shuffle pass B (k_nttb_shfl: 32 chunks per 256-thread block) for the plain transform and the
            // mod-up digits; the divide-and-round post-op keeps the LDS pass (its 16 outputs and post-op operands
            // in registers at once would cost it a wave per SIMD)
            constexpr bool kDR = std::is_same_v<IO2, DivRoundIOB<false>> || std::is_same_v<IO2, DivRoundIOB<true>>;
            if constexpr (LOGC == 7 && (std::is_same_v<IO2, StridedIO> || std::is_same_v<IO2, ModUpIO_B> ||
                                        std::is_same_v<IO2, ModUpIO_BT<true>> || kDR)) {
                if (c.nttb_shfl && (!kDR || c.nttb_shfl_dr)) {
                    if (c.nttb_shfl == 2)
                        k_nttb_shfl<IO2, true><<<dim3(R / 32, njobs), 256, 0, c.stream>>>(second, fwd, c.primes, c.logN);
                    else
                        k_nttb_shfl<IO2, false><<<dim3(R / 32, njobs), 256, 0, c.stream>>>(second, fwd, c.primes, c.logN);
                    HEC_HIP(hipGetLastError());
                    return;
                }
            }
            k_ntt<LOGC, NB, false, false, true><<<gB, TB, 0, c.stream>>>(second, fwd, c.primes, c.logN);
        }
    } else {
        if (stages & 1) k_ntt<LOGC, NB, true, false, false, IO1, true><<<gB, TB, 0, c.stream>>>(first, inv, c.primes, c.logN);
        if (stages & 2) k_ntt<LOGR, NA, true, true, true, IO2, true><<<gA, TA, 0, c.stream>>>(second, inv, c.primes, c.logN);
    }
    HEC_HIP(hipGetLastError());
}

// forward: first = pass A IO (pre-op load), second = pass B IO (post-op store);
// inverse: first = pass B IO, second = pass A IO.
template <bool INV, class IO1, class IO2>
static void ntt_dispatch(Ctx &c, int njobs, const IO1 &first, const IO2 &second, int stages = 3)
{
    if (njobs <= 0) return;
    switch (c.logN) {
    case 10: run_ntt2<5, 5, 32, 32, INV>(c, njobs, first, second, stages); break;
    case 11: run_ntt2<6, 5, 32, 64, INV>(c, njobs, first, second, stages); break;
    case 12: run_ntt2<6, 6, 64, 64, INV>(c, njobs, first, second, stages); break;
    case 13: run_ntt2<7, 6, 32, 64, INV>(c, njobs, first, second, stages); break;
    case 14: run_ntt2<7, 7, 32, 32, INV>(c, njobs, first, second, stages); break;
    case 15: run_ntt2<8, 7, 16, 16, INV>(c, njobs, first, second, stages); break;
    case 16: run_ntt2<8, 8, 16, 16, INV>(c, njobs, first, second, stages); break;
    default: throw std::invalid_argument("poly_modulus_degree must be 2^10 .. 2^16");
    }
}

static StridedIO strided(const u64 *src, u64 *dst, u64 ps_src, u64 ps_dst, int nl, int logN, const int *pmap,
                         u32 elt = 1)
{
    StridedIO io{};
    io.src = src; io.dst = dst; io.ps_src = ps_src; io.ps_dst = ps_dst; io.nl = nl; io.logN = logN; io.elt = elt;
    for (int i = 0; i < nl && i <= HEC_MAXL; ++i) io.pmap[i] = pmap[i];
    return io;
}

void ntt_strided(Ctx &c, bool inverse, const u64 *src, u64 ps_src, u64 *dst, u64 ps_dst, int nl, const int *pmap,
                 int njobs, u32 elt, int stages)
{
    if (nl > HEC_MAXL + 1) throw std::invalid_argument("too many limbs");
    const StridedIO first = strided(src, dst, ps_src, ps_dst, nl, c.logN, pmap, elt);
    const StridedIO second = strided(dst, dst, ps_dst, ps_dst, nl, c.logN, pmap);
    if (inverse) ntt_dispatch<true>(c, njobs, first, second, stages);
    else ntt_dispatch<false>(c, njobs, first, second, stages);
}

void ks_modup(Ctx &c, const u64 *D, u64 *E, int B, int l, int stages, bool mform)
{
    ModUpMap m{l, c.logN, (int)c.K - 1};
    ModUpIO_A a{m, D, E, c.primes};
    if (c.nt_e) {
        ModUpIO_BT<true> b{m, E, mform ? 1 : 0};
        ntt_dispatch<false>(c, B * l * l, a, b, stages);
    } else {
        ModUpIO_B b{m, E, mform ? 1 : 0};
        ntt_dispatch<false>(c, B * l * l, a, b, stages);
    }
}

void divide_round(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, PolyArr X, PolyArr IN, int in_nk, PolyArr OUT, int B,
                  int nk, int nl, int last_idx, const u64 *inv, const u64 *inv_q, u64 *Z, u32 in_elt, int stages)
{
    if (nl > HEC_MAXL) throw std::invalid_argument("too many limbs");
    DivRoundIO_A a{};
    a.Y = Y; a.ysb = ysb; a.ysk = ysk; a.Z = Z; a.nk = nk; a.nl = nl; a.logN = c.logN;
    a.last = c.q[last_idx]; a.half = a.last >> 1; a.primes = c.primes;
    for (int i = 0; i < nl; ++i) a.fix[i] = c.q[i] - (a.half % c.q[i]);
    auto run = [&](auto b) {
        b.Z = Z; b.X = X; b.IN = IN; b.OUT = OUT; b.nk = nk; b.nl = nl; b.logN = c.logN; b.in_nk = in_nk;
        b.elt = in_elt; b.primes = c.primes;
        b.fpstore = 1;
        for (int i = 0; i < nl; ++i) { b.inv[i] = inv[i]; b.inv_q[i] = inv_q[i]; }
        ntt_dispatch<false>(c, B * nk * nl, a, b, stages);
    };
    if (IN.p != nullptr && in_nk > 0) run(DivRoundIOB<true>{});
    else run(DivRoundIOB<false>{});
}

// =============================================================== fan-out: INTT pass A -> fwd passes A ==
// A block owns NSEG columns (R rows) of one source limb whose inverse pass B already ran.  It finishes
// the INTT (inverse pass A, N^-1 scaling, canonical residues), keeps the coefficient-form column values
// in registers and, for every target prime t of the source, transforms them (FAN::xf: the mod-up
// reduction mod q_t, or the mod-down rounding) and runs the forward pass A for q_t, storing the
// pass-A-domain tile for the following pass-B kernel (k_bmac / the divide-and-round pass B).  The
// coefficient-form limb is never stored, and it is read once instead of once per target.
// kDirect: D already holds the canonical coefficient form (hoisted mod-up), so there is no inverse pass.
// one zero coefficient g of digit limb `limb` in the zero lists (layout: see k_zscan)
__device__ __forceinline__ void zero_record(int *zl, int *zflag, int limb, int g)
{
    atomicAdd(zl, 1);
    int *z = zl + 1 + limb * (HEC_ZCAP + 1);
    const int k = atomicAdd(z, 1);
    if (k < HEC_ZCAP) z[1 + k] = g;
    else atomicOr(zflag, 1);
}

template <bool DIRECT>
struct FanModUpT {  // source (b, J) = D[b][J] (inverse pass-B domain) -> E[b][I][J], I != J, mod q_I
    static constexpr bool kDirect = DIRECT;
    static constexpr bool kScan = !DIRECT;
    static constexpr bool kSplit = false;
    static constexpr bool kSrcDouble = !DIRECT;  // an FP64-class source stays a double (xf16's sdbl)
    static constexpr int kJobs = 2;              // source jobs per block (k_fan2j: the next one's words prefetched)
    const u64 *D;
    u64 *E;
    int l, logN, kP;
    const DevPrime *primes;
    int *zl = nullptr, *zflag = nullptr;  // non-direct hoisted mod-up: list the zero coefficients of the source
                                          // (k_zscan's format) while the INTT's values are in registers
    struct Src { const u64 *in; int prime; };
    // red: how digit J (canonical, < q_J) reduces mod q_I: 0 nothing (q_J <= q_I: the 40-bit digits at the
    // 60-bit targets), 1 one conditional subtraction (q_J <= 2 q_I: 40-bit digit, 40-bit target), 2 Barrett
    struct Tgt { bool valid; int prime; u64 *out; u64 q, r1; int red; };
    __device__ int ntargets() const { return l + 1; }
    __device__ Src src(int job) const { return Src{D + ((u64)job << logN), job % l}; }
    __device__ Tgt tgt(int job, int I) const
    {
        const int b = job / l, J = job % l, p = I == l ? kP : I;
        const DevPrime pp = cprime(primes, p);
        const u64 qI = pp.q, qJ = cprime(primes, J).q;
        return Tgt{I != J, p, E + (((u64)((b * (l + 1) + I) * l + J)) << logN), qI, pp.r1,
                   qJ <= qI ? 0 : (qJ <= 2 * qI ? 1 : 2)};
    }
    __device__ u64 src_fix(u64 d) const { return d; }
    __device__ u64 xf(const Tgt &t, u64 d) const
    {
        return t.red == 0 ? d : t.red == 1 ? csub(d, t.q) : barrett64(d, t.q, t.r1);
    }
    // the 16 values of a thread as the target's NTT input (k_fan2; the class branch is block-uniform).  FP64
    // targets take any congruent integer-valued double with |x| < 2 q_I (their forward butterflies stay below
    // 10 q_I over all stages and every output is canonicalised): a digit with q_J <= 2 q_I needs no
    // reduction at all, only the conversion
    // sdbl: the source (an FP64-class digit, q_J < 2^42) is held as the bits of its canonical integer-valued double,
    // converted once per block instead of once per FP64 target; the two integer targets convert it back
    __device__ void xf16(const Tgt &t, bool fp, const u64 *d, const u32 *, u64 *v, bool sdbl = false) const
    {
        if (sdbl) {
            if (fp) {
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = d[k];  // q_J < 2 q_I: no reduction (see above)
                return;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const u64 y = d2u(__longlong_as_double((long long)d[k]));
                v[k] = t.red == 1 ? csub(y, t.q) : y;  // red == 2 needs q_J > 2 q_I: only the 60-bit digit J = 0
            }
            return;
        }
        if (t.red == 2 && fp && t.q > (1ull << 32)) {  // the 60-bit digit at an FP64 target: hi 2^30 + lo as above
            const DevPrime p = cprime(primes, t.prime);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                u64 y = d[k];
                asm volatile("" : "+v"(y));  // per target (see FanDivRound::xf16)
                const double hi = u2d(y >> 30) * 1073741824.0, lo = u2d(y & 0x3fffffffull);
                v[k] = (u64)__double_as_longlong(fp_reduce(hi, p.qd, p.qinv) + lo);  // (-0.51 q, 0.51 q + 2^30)
            }
            return;
        }
        if (t.red == 2) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = barrett64(d[k], t.q, t.r1);
        } else if (t.red == 1 && !fp) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = csub(d[k], t.q);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = d[k];
        }
        if (fp) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = (u64)__double_as_longlong(u2d(v[k]));
        }
    }
};
using FanModUp = FanModUpT<false>;
struct FanDivRound {  // source (b, k) = last limb (inverse pass-B domain) -> Z[b][k][i] for i < nl
    static constexpr bool kDirect = false;
    static constexpr bool kScan = false;
    // the source value y < P < 2^60 is split once per block into hs = (y >> 30) 2^30 (an exact double, kept in d's
    // bits) and lo = y & (2^30 - 1) (u32), so an FP64 target only reduces hs (one FMA) and adds lo: 6 FP64 operations
    // per value and target instead of 13 mixed ones
    static constexpr bool kSplit = true;
    static constexpr bool kSrcDouble = false;
    static constexpr int kJobs = 1;  // (2 per block: 256 VGPRs + 50 AGPRs, one wave per SIMD)
    int *zl = nullptr, *zflag = nullptr;
    const u64 *Y;
    u64 ysb, ysk;
    u64 *Z;
    int nk, nl, logN, last_idx;
    u64 last, half;
    const DevPrime *primes;
    u64 fix[HEC_MAXL];
    double c30[HEC_MAXL];  // 2^30 mod q_i (split reduction at FP64 targets with q_i > 2^32, else 0)
    unsigned sub1;         // bit i: P < 2 q_i, so y < P reduces mod q_i by one conditional subtraction
    struct Src { const u64 *in; int prime; };
    struct Tgt { bool valid; int prime; u64 *out; u64 q, r1, fix; double qd, qinv, c30; bool sub1; };
    __device__ int ntargets() const { return nl; }
    __device__ Src src(int job) const { return Src{Y + (u64)(job / nk) * ysb + (u64)(job % nk) * ysk, last_idx}; }
    __device__ Tgt tgt(int job, int i) const
    {
        const DevPrime p = cprime(primes, i);
        return Tgt{true, i, Z + ((u64)(job * nl + i) << logN), p.q, p.r1, fix[i], p.qd, p.qinv, c30[i],
                   ((sub1 >> i) & 1u) != 0};
    }
    // y -> (y + floor(P/2)) mod P, once per source value (the rounding offset is the same for every target)
    __device__ u64 src_fix(u64 d) const
    {
        const u64 v = d + half;
        return v >= last ? v - last : v;
    }
    __device__ u64 xf(const Tgt &t, u64 d) const { return (t.sub1 ? csub(d, t.q) : barrett64(d, t.q, t.r1)) + t.fix; }
    // FP64 targets with q_i > 2^32: y = hi 2^30 + lo, y == fp_reduce(hi 2^30) + lo (+ fix) mod q_i: hi 2^30 < 2^60 is
    // an exact double and its reduction r = hi 2^30 - rint(hi 2^30 / q_i) q_i is exact in one FMA (|r| <= 0.5 q_i),
    // so the value is an integer-valued double in (-0.51 q_i, 1.51 q_i + 2^30), within the FP64 forward NTT's
    // |x| < 2 q_i input range
    // (no 64-bit Barrett: ~6 FP64 operations per value instead of 7 integer multiplies).  Smaller FP64 primes
    // and the integer targets keep Barrett on y rebuilt from its halves.
    __device__ static void split(u64 *d, u32 *lo)  // once per block: d[k] = y -> bits of (y >> 30) 2^30, lo[k]
    {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            lo[k] = (u32)(d[k] & 0x3fffffffull);
            d[k] = (u64)__double_as_longlong(u2d(d[k] >> 30) * 1073741824.0);
        }
    }
    __device__ static u64 join(u64 hs, u32 lo)
    {
        return (d2u(__longlong_as_double((long long)hs) * (1.0 / 1073741824.0)) << 30) | lo;
    }
    __device__ void xf16(const Tgt &t, bool fp, const u64 *d, const u32 *lo, u64 *v, bool = false) const
    {
        if (fp && t.c30 != 0.0) {
            const double fx = (double)t.fix;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                u64 h = d[k];
                u32 l = lo[k];
                asm volatile("" : "+v"(h), "+v"(l));  // per target: the conversions are not hoisted out of the target
                                                      // loop (32 more live doubles: 256 VGPRs, one wave per SIMD)
                const double hs = __longlong_as_double((long long)h);
                v[k] = (u64)__double_as_longlong(fp_reduce(hs, t.qd, t.qinv) + ((double)l + fx));
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = xf(t, join(d[k], lo[k]));
        if (fp) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = (u64)__double_as_longlong(u2d(v[k]));
        }
    }
};

// ------------------------------------------------------------------ register-direct fan-out (k_fan2)
// The stages of one round on 16 register-resident elements: thread ts of a P = 2^LOGP point column holds the
// elements ntt_round_g gives it for stages [S0, S1): v[gi 2^D + a] <-> x = xb(ts G + gi) | (a << (LOGP - S1)).
// Round 0 (stages 0..3) owns x = ts + k TPS ("stride set"), round 1 (stages 4..LOGP-1) x = 16 ts + k ("block
// set"), k = 0..15, TPS = P / 16.
// UNI: every group of the round has hi = 0 (round 0 of a column transform: ts < 2^(LOGP - 4)), so the twiddle
// indices are compile-time offsets from a block-uniform table base (with ConstTw: scalar loads)
template <int LOGP, int S0, int S1, bool INV, bool FP, class TwG, bool UNI = false>
__device__ __forceinline__ void ntt_round_r(u64 *v, int ts, const TwG &twg, const DevPrime &pr)
{
    constexpr int D = S1 - S0, G = 1 << (4 - D), NQ = 1 << D;
    static_assert(D >= 1 && D <= 4, "round covers 1..4 stages");
    const u64 q = pr.q, two_q = 2 * q;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int g = ts * G + gi;
        const int hi = UNI ? 0 : g >> (LOGP - S1);
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const int st = INV ? D - 1 - k : k;
            const int bit = 1 << (D - 1 - st);
#pragma unroll
            for (int a = 0; a < NQ; ++a) {
                if (a & bit) continue;
                const int m = a >> (D - st);
                u64 &X = v[gi * NQ + a], &Y = v[gi * NQ + (a | bit)];
                if constexpr (FP) {
                    double x = __longlong_as_double((long long)X), y = __longlong_as_double((long long)Y);
                    const double w = twg.f(S0 + st, (hi << st) | m);
                    if constexpr (!INV) ct_bfly_fp(x, y, w, pr.qd, pr.qinv);
                    else gs_bfly_fp(x, y, w, pr.qd, pr.qinv);
                    X = (u64)__double_as_longlong(x);
                    Y = (u64)__double_as_longlong(y);
                } else if constexpr (HasSplitTw<TwG>::value) {
                    const ulonglong2 w = twg.w(S0 + st, (hi << st) | m);
                    const u64 wa = twg.a(S0 + st, (hi << st) | m);
                    if constexpr (!INV) ct_bfly_s(X, Y, w.x, w.y, wa, q, two_q);
                    else gs_bfly_s(X, Y, w.x, w.y, wa, q, two_q);
                } else {
                    const ulonglong2 w = twg.w(S0 + st, (hi << st) | m);
                    if constexpr (!INV) ct_bfly(X, Y, w.x, w.y, q, two_q);
                    else gs_bfly(X, Y, w.x, w.y, q, two_q);
                }
            }
        }
    }
}

// The fan-out with the NTT rounds on registers: the source is loaded straight into the thread's element set and
// the target tiles are stored straight from it, so each transform (the INTT and every target's forward
// pass) exchanges through LDS once (round 1's LDS-round k_fan exchanged three times; deleted in round 3), with one
// barrier per exchange (two LDS tiles alternate between consecutive exchanges).
// DB: two alternating LDS tiles and one barrier per exchange (2 blocks per CU at N = 2^15); DB = false: one
// tile and a second barrier per target.  (One tile with 3 waves per SIMD forced, 168 VGPRs and 20-30 spilled,
// measured slower: k_fan 3,565 vs 2,601 ms per step.)
// SPL: the integer primes' butterflies as split-input Shoup (inv.sa / fwd.sa, hec_device.h shoup_split_lazy), bit 0 in
// the round on scalar (block-uniform) twiddles, bit 1 in the round on per-thread twiddles
template <int LOGP, int NSEG, class FAN, int SPL, bool DB = true>
__global__ void __launch_bounds__(NSEG *(1 << LOGP) / 16)
    k_fan2(const FAN fan, TwTables inv, TwTables fwd, const DevPrime *__restrict__ primes, int logN)
{
    constexpr int P = 1 << LOGP, TPS = P / 16, LD = NSEG + 1, TILE = P * LD;
    __shared__ u64 lds[(DB ? 2 : 1) * TILE];
    const int seg0 = blockIdx.x * NSEG, lc = logN - LOGP;
    const int ts = threadIdx.x / NSEG, sg = threadIdx.x % NSEG;
    auto gstride = [&](int k) { return ((u64)(ts + k * TPS) << lc) + seg0 + sg; };
    auto gblock = [&](int k) { return ((u64)(16 * ts + k) << lc) + seg0 + sg; };
    auto lstride = [&](int k) { return (ts + k * TPS) * LD + sg; };
    auto lblock = [&](int k) { return (16 * ts + k) * LD + sg; };
    auto twidx = [](int s, int i) -> u64 { return (1ull << s) + (u64)i; };
    const auto src = fan.src(blockIdx.y);
    const DevPrime ps = cprime(primes, src.prime);
    int buf = 0;
    u64 d[16];  // canonical coefficient-form values of the source, stride set
    u32 lo[FAN::kSplit ? 16 : 1];  // kSplit: the low 30 bits (d then holds the high part as a double)
    if constexpr (FAN::kDirect) {
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = src.in[gstride(k)];
    } else {
        u64 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = src.in[gblock(k)];
        const GlobalTw<decltype(twidx)> tg{twidx, inv.a + ((u64)src.prime << logN), inv.fa + ((u64)src.prime << logN)};
        const ConstTw ctg{inv.a + ((u64)src.prime << logN), inv.fa + ((u64)src.prime << logN)};
        const GlobalTwS<decltype(twidx)> tgs{tg, SPL ? inv.sa + ((u64)src.prime << logN) : nullptr};
        const ConstTwS ctgs{ctg, SPL ? inv.sa + ((u64)src.prime << logN) : nullptr};
        if (ps.fp) ntt_round_r<LOGP, 4, LOGP, true, true>(v, ts, tg, ps);
        else if constexpr ((SPL & 2) != 0) ntt_round_r<LOGP, 4, LOGP, true, false>(v, ts, tgs, ps);
        else ntt_round_r<LOGP, 4, LOGP, true, false>(v, ts, tg, ps);
#pragma unroll
        for (int k = 0; k < 16; ++k) lds[lblock(k)] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = lds[lstride(k)];
        buf = 1;
        if (ps.fp) {
            ntt_round_r<LOGP, 0, 4, true, true, ConstTw, true>(v, ts, ctg, ps);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double c = fp_mulmod(__longlong_as_double((long long)v[k]), ps.ninv_d, ps.qd, ps.qinv);
                d[k] = fp_canon(c, ps.qd, ps.qinv);
                // the canonical residue as an exact double (its bits; +0.0 for zero, so the zero scan is unchanged)
                if constexpr (FAN::kSrcDouble) d[k] = (u64)__double_as_longlong(u2d(d[k]));
            }
        } else {
            if constexpr ((SPL & 1) != 0) ntt_round_r<LOGP, 0, 4, true, false, ConstTwS, true>(v, ts, ctgs, ps);
            else ntt_round_r<LOGP, 0, 4, true, false, ConstTw, true>(v, ts, ctg, ps);
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = shoup(v[k], ps.ninv, ps.ninv_q, ps.q);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = fan.src_fix(d[k]);
        if constexpr (FAN::kSplit) FAN::split(d, lo);
        if constexpr (FAN::kScan) {
            if (fan.zl != nullptr && blockIdx.z == 0) {  // the canonical coefficient form's zeros (k_zscan)
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if (d[k] == 0) zero_record(fan.zl, fan.zflag, (int)blockIdx.y, (int)gstride(k) & ((1 << logN) - 1));
            }
        }
    }
    const int nt = fan.ntargets(), t0 = blockIdx.z * nt / gridDim.z, t1 = (blockIdx.z + 1) * nt / gridDim.z;
    for (int t = t0; t < t1; ++t) {
        const auto tgt = fan.tgt(blockIdx.y, t);
        if (!tgt.valid) continue;
        const DevPrime pt = cprime(primes, tgt.prime);
        const GlobalTw<decltype(twidx)> tw{twidx, fwd.a + ((u64)tgt.prime << logN), fwd.fa + ((u64)tgt.prime << logN)};
        const ConstTw ctw{fwd.a + ((u64)tgt.prime << logN), fwd.fa + ((u64)tgt.prime << logN)};
        const GlobalTwS<decltype(twidx)> tws{tw, SPL ? fwd.sa + ((u64)tgt.prime << logN) : nullptr};
        const ConstTwS ctws{ctw, SPL ? fwd.sa + ((u64)tgt.prime << logN) : nullptr};
        u64 *tile = lds + (DB ? buf * TILE : 0);
        buf ^= 1;
        if (!DB) __syncthreads();  // the previous exchange's reads are done
        u64 v[16];
        if (pt.fp) {
            fan.xf16(tgt, true, d, lo, v, FAN::kSrcDouble && ps.fp);
            ntt_round_r<LOGP, 0, 4, false, true, ConstTw, true>(v, ts, ctw, pt);
        } else {
            fan.xf16(tgt, false, d, lo, v, FAN::kSrcDouble && ps.fp);
            if constexpr ((SPL & 1) != 0) ntt_round_r<LOGP, 0, 4, false, false, ConstTwS, true>(v, ts, ctws, pt);
            else ntt_round_r<LOGP, 0, 4, false, false, ConstTw, true>(v, ts, ctw, pt);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) tile[lstride(k)] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = tile[lblock(k)];
        if (pt.fp) ntt_round_r<LOGP, 4, LOGP, false, true>(v, ts, tw, pt);
        else if constexpr ((SPL & 2) != 0) ntt_round_r<LOGP, 4, LOGP, false, false>(v, ts, tws, pt);
        else ntt_round_r<LOGP, 4, LOGP, false, false>(v, ts, tw, pt);
        // (16-B stores and loads through lane-pair trades measured slower: 2,613 vs 2,580 ms per step, round 4)
#pragma unroll
        for (int k = 0; k < 16; ++k) st1m<1>(tgt.out + gblock(k), v[k]);
    }
}

// k_fan2 over JPB source jobs per block (FanModUpT): the next job's source words are loaded during the current
// job's last target.  A separate kernel: folded into k_fan2, the restructured body costs the divide-and-round
// fan-out (one job per block) 12 VGPRs and a wave.
template <int LOGP, int NSEG, class FAN, int JPB, int SPL, bool DB = true>
__global__ void __launch_bounds__(NSEG *(1 << LOGP) / 16, 2)  // 2 waves per SIMD (<= 256 VGPRs) with the split words too
    k_fan2j(const FAN fan, TwTables inv, TwTables fwd, const DevPrime *__restrict__ primes, int logN, int njobs)
{
    constexpr int P = 1 << LOGP, TPS = P / 16, LD = NSEG + 1, TILE = P * LD;
    constexpr int D1 = LOGP - 4, G1 = 1 << (4 - D1);
    __shared__ u64 lds[(DB ? 2 : 1) * TILE];
    const int seg0 = blockIdx.x * NSEG, lc = logN - LOGP;
    const int ts = threadIdx.x / NSEG, sg = threadIdx.x % NSEG;
    auto gstride = [&](int k) { return ((u64)(ts + k * TPS) << lc) + seg0 + sg; };
    auto gblock = [&](int k) { return ((u64)(16 * ts + k) << lc) + seg0 + sg; };
    auto lstride = [&](int k) { return (ts + k * TPS) * LD + sg; };
    auto lblock = [&](int k) { return (16 * ts + k) * LD + sg; };
    auto twidx = [](int s, int i) -> u64 { return (1ull << s) + (u64)i; };
    // the raw source words of a job: the canonical coefficient form (direct) or the inverse pass-B domain (block set)
    auto load_src = [&](int job, u64 *w) {
        const auto sr = fan.src(job);
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = sr.in[FAN::kDirect ? gstride(k) : gblock(k)];
    };
    const int nt = fan.ntargets(), t0 = blockIdx.z * nt / gridDim.z, t1 = (blockIdx.z + 1) * nt / gridDim.z;
    const int job0 = blockIdx.y * JPB;
    int buf = 0;
    u64 d[16];  // canonical coefficient-form values of the source, stride set
    u32 lo[FAN::kSplit ? 16 : 1];  // kSplit: the low 30 bits (d then holds the high part as a double)
    load_src(job0, d);
    // JPB jobs per block: the next job's source words are loaded during the current job's last target (into d, dead
    // after that target's xf16), after that target's round-1 twiddles, so no round waits for them in issue order
    for (int jj = 0; jj < JPB; ++jj) {
        const int job = job0 + jj;
        if (job >= njobs) break;  // block-uniform
        const auto src = fan.src(job);
        const DevPrime ps = cprime(primes, src.prime);
        if constexpr (!FAN::kDirect) {
            u64 v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = d[k];
            const GlobalTw<decltype(twidx)> tg{twidx, inv.a + ((u64)src.prime << logN), inv.fa + ((u64)src.prime << logN)};
            const ConstTw ctg{inv.a + ((u64)src.prime << logN), inv.fa + ((u64)src.prime << logN)};
            const GlobalTwS<decltype(twidx)> tgs{tg, SPL ? inv.sa + ((u64)src.prime << logN) : nullptr};
            const ConstTwS ctgs{ctg, SPL ? inv.sa + ((u64)src.prime << logN) : nullptr};
            if (ps.fp) ntt_round_r<LOGP, 4, LOGP, true, true>(v, ts, tg, ps);
            else if constexpr ((SPL & 2) != 0) ntt_round_r<LOGP, 4, LOGP, true, false>(v, ts, tgs, ps);
            else ntt_round_r<LOGP, 4, LOGP, true, false>(v, ts, tg, ps);
            u64 *tile = lds + (DB ? buf * TILE : 0);
            if (!DB || jj > 0) __syncthreads();  // the previous job's last exchange reads are done
#pragma unroll
            for (int k = 0; k < 16; ++k) tile[lblock(k)] = v[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = tile[lstride(k)];
            buf ^= 1;
            if (ps.fp) {
                ntt_round_r<LOGP, 0, 4, true, true, ConstTw, true>(v, ts, ctg, ps);
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const double c = fp_mulmod(__longlong_as_double((long long)v[k]), ps.ninv_d, ps.qd, ps.qinv);
                    d[k] = fp_canon(c, ps.qd, ps.qinv);
                    // the canonical residue as an exact double (its bits; +0.0 for zero, so the zero scan is unchanged)
                    if constexpr (FAN::kSrcDouble) d[k] = (u64)__double_as_longlong(u2d(d[k]));
                }
            } else {
                if constexpr ((SPL & 1) != 0) ntt_round_r<LOGP, 0, 4, true, false, ConstTwS, true>(v, ts, ctgs, ps);
                else ntt_round_r<LOGP, 0, 4, true, false, ConstTw, true>(v, ts, ctg, ps);
#pragma unroll
                for (int k = 0; k < 16; ++k) d[k] = shoup(v[k], ps.ninv, ps.ninv_q, ps.q);
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = fan.src_fix(d[k]);
            if constexpr (FAN::kSplit) FAN::split(d, lo);
            if constexpr (FAN::kScan) {
                if (fan.zl != nullptr && blockIdx.z == 0) {  // the canonical coefficient form's zeros (k_zscan)
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        if (d[k] == 0) zero_record(fan.zl, fan.zflag, job, (int)gstride(k) & ((1 << logN) - 1));
                }
            }
        }
        int tl = -1;  // the last valid target: it loads the next job's source
        if (jj + 1 < JPB && job + 1 < njobs)
            for (int t = t1 - 1; t >= t0; --t)
                if (fan.tgt(job, t).valid) {
                    tl = t;
                    break;
                }
        for (int t = t0; t < t1; ++t) {
            const auto tgt = fan.tgt(job, t);
            if (!tgt.valid) continue;
            const DevPrime pt = cprime(primes, tgt.prime);
            const GlobalTw<decltype(twidx)> tw{twidx, fwd.a + ((u64)tgt.prime << logN), fwd.fa + ((u64)tgt.prime << logN)};
            const ConstTw ctw{fwd.a + ((u64)tgt.prime << logN), fwd.fa + ((u64)tgt.prime << logN)};
            const GlobalTwS<decltype(twidx)> tws{tw, SPL ? fwd.sa + ((u64)tgt.prime << logN) : nullptr};
            const ConstTwS ctws{ctw, SPL ? fwd.sa + ((u64)tgt.prime << logN) : nullptr};
            u64 *tile = lds + (DB ? buf * TILE : 0);
            buf ^= 1;
            if (!DB) __syncthreads();  // the previous exchange's reads are done
            u64 v[16];
            if (pt.fp) {
                fan.xf16(tgt, true, d, lo, v, FAN::kSrcDouble && ps.fp);
                ntt_round_r<LOGP, 0, 4, false, true, ConstTw, true>(v, ts, ctw, pt);
            } else {
                fan.xf16(tgt, false, d, lo, v, FAN::kSrcDouble && ps.fp);
                if constexpr ((SPL & 1) != 0) ntt_round_r<LOGP, 0, 4, false, false, ConstTwS, true>(v, ts, ctws, pt);
                else ntt_round_r<LOGP, 0, 4, false, false, ConstTw, true>(v, ts, ctw, pt);
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) tile[lstride(k)] = v[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = tile[lblock(k)];
            if (t == tl) {  // round 1's twiddles, then the next job's source, then round 1
                if (pt.fp) {
                    GroupTw<4, D1, true> g1[G1];
#pragma unroll
                    for (int gi = 0; gi < G1; ++gi) g1[gi].load(ts * G1 + gi, tw);
                    asm volatile("" ::: "memory");
                    load_src(job + 1, d);
#pragma unroll
                    for (int gi = 0; gi < G1; ++gi) g1[gi].template run<false>(v + gi * (1 << D1), pt);
                } else {
                    GroupTw<4, D1, false, (SPL & 2) != 0> g1[G1];
#pragma unroll
                    for (int gi = 0; gi < G1; ++gi) {
                        if constexpr ((SPL & 2) != 0) g1[gi].load(ts * G1 + gi, tws);
                        else g1[gi].load(ts * G1 + gi, tw);
                    }
                    asm volatile("" ::: "memory");
                    load_src(job + 1, d);
#pragma unroll
                    for (int gi = 0; gi < G1; ++gi) g1[gi].template run<false>(v + gi * (1 << D1), pt);
                }
            } else if (pt.fp) {
                ntt_round_r<LOGP, 4, LOGP, false, true>(v, ts, tw, pt);
            } else if constexpr ((SPL & 2) != 0) {
                ntt_round_r<LOGP, 4, LOGP, false, false>(v, ts, tws, pt);
            } else {
                ntt_round_r<LOGP, 4, LOGP, false, false>(v, ts, tw, pt);
            }
            // (16-B stores and loads through lane-pair trades measured slower: 2,613 vs 2,580 ms per step, round 4)
#pragma unroll
            for (int k = 0; k < 16; ++k) st1m<1>(tgt.out + gblock(k), v[k]);
        }
        // a target slice [t0, t1) without a valid target for this job (gridDim.z > 1) loaded nothing above: the next
        // job's source still has to replace d (block-uniform, never taken with one target group)
        if (tl < 0 && jj + 1 < JPB && job + 1 < njobs) load_src(job + 1, d);
    }
}

template <int LOGR, int LOGC, int NA, class FAN>
static void run_fan(Ctx &c, int njobs, const FAN &fan, int groups)
{
    constexpr int R = 1 << LOGR, C = 1 << LOGC;
    const TwTables fwd{c.tw, c.twb, c.twf, c.twbf, c.tws}, inv{c.itw, c.itwb, c.itwf, c.itwbf, c.itws};
    constexpr int JPB = FAN::kJobs;
    const dim3 grid(C / NA, (njobs + JPB - 1) / JPB, groups);
    // c.split_bfly (HEC_SPLIT_BFLY): 0 plain Shoup everywhere; 1 split-input Shoup in k_fan2 (the mod-down fan-out);
    // 2 also in k_fan2j's per-thread-twiddle rounds; 3 in all of k_fan2j's rounds; 4 k_fan2j's scalar-twiddle round only
    const int sp = c.split_bfly;
    if constexpr (JPB > 1) {
        if (sp == 4)
            k_fan2j<LOGR, NA, FAN, JPB, 1><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN, njobs);
        else if (sp == 3)
            k_fan2j<LOGR, NA, FAN, JPB, 3><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN, njobs);
        else if (sp == 2)
            k_fan2j<LOGR, NA, FAN, JPB, 2><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN, njobs);
        else
            k_fan2j<LOGR, NA, FAN, JPB, 0><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN, njobs);
    } else if (sp >= 1) {
        k_fan2<LOGR, NA, FAN, 3><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN);
    } else {
        k_fan2<LOGR, NA, FAN, 0><<<grid, NA * R / 16, 0, c.stream>>>(fan, inv, fwd, c.primes, c.logN);
    }
    HEC_HIP(hipGetLastError());
}
template <class FAN>
static void fan_dispatch(Ctx &c, int njobs, const FAN &fan, int groups = 1)
{
    groups = std::max(1, groups);
    switch (c.logN) {
    case 10: run_fan<5, 5, 32>(c, njobs, fan, groups); break;
    case 11: run_fan<6, 5, 32>(c, njobs, fan, groups); break;
    case 12: run_fan<6, 6, 64>(c, njobs, fan, groups); break;
    case 13: run_fan<7, 6, 32>(c, njobs, fan, groups); break;
    case 14: run_fan<7, 7, 32>(c, njobs, fan, groups); break;
    case 15: run_fan<8, 7, 16>(c, njobs, fan, groups); break;
    case 16: run_fan<8, 8, 16>(c, njobs, fan, groups); break;
    default: throw std::invalid_argument("poly_modulus_degree must be 2^10 .. 2^16");
    }
}

void fan_modup(Ctx &c, const u64 *D, u64 *E, int B, int l, bool direct, int *zl)
{
    const int g = 1;  // target groups per source (gridDim.z): more than one measured slower
    if (direct) {
        fan_dispatch(c, B * l, FanModUpT<true>{D, E, l, c.logN, (int)c.K - 1, c.primes}, g);
        return;
    }
    FanModUp f{D, E, l, c.logN, (int)c.K - 1, c.primes};
    if (zl) {
        dev_zero(c, zl, (1 + (std::size_t)B * l * (HEC_ZCAP + 1)) * sizeof(int));
        f.zl = zl;
        f.zflag = c.zflag;
    }
    fan_dispatch(c, B * l, f, g);
}

// Device fills and copies as engine kernels on the context stream (c.kernel_memops, the default), in place of the
// runtime's hipMemsetAsync / device-to-device hipMemcpyAsync (see hec_internal.h)
__global__ void __launch_bounds__(256) k_fill32(u32 *__restrict__ p, u32 v, u64 n)
{
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) p[i] = v;
}
__global__ void __launch_bounds__(256) k_copy64(u64 *__restrict__ dst, const u64 *__restrict__ src, u64 n)
{
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) dst[i] = src[i];
}
void dev_fill32(Ctx &c, void *p, u32 v, std::size_t bytes)
{
    const u64 n = bytes / 4;
    if (!n) return;
    k_fill32<<<(unsigned)std::min<u64>((n + 255) / 256, 8192), 256, 0, c.stream>>>((u32 *)p, v, n);
    HEC_HIP(hipGetLastError());
}
void dev_copy64(Ctx &c, u64 *dst, const u64 *src, std::size_t words)
{
    if (!words) return;
    k_copy64<<<(unsigned)std::min<u64>((words + 255) / 256, 8192), 256, 0, c.stream>>>(dst, src, words);
    HEC_HIP(hipGetLastError());
}
void dev_fill(Ctx &c, void *p, u32 v, std::size_t bytes)  // bytes: a multiple of 4
{
    if (c.kernel_memops) dev_fill32(c, p, v, bytes);
    else if (v == 0 || v == 0xFFFFFFFFu) HEC_HIP(hipMemsetAsync(p, (int)(v & 0xFF), bytes, c.stream));
    else HEC_HIP(hipMemsetD32Async((hipDeviceptr_t)p, (int)v, bytes / 4, c.stream));
}
void dev_zero(Ctx &c, void *p, std::size_t bytes) { dev_fill(c, p, 0, bytes); }

// debug (HEC_DEBUG_LANES): count the hoisted nodes whose zero list is not empty (uniform residues almost never have a
// zero coefficient, so a count is a sign the list was read before it was written)
__global__ void __launch_bounds__(64) k_dbg_zl(const int *__restrict__ zl, int *cnt)
{
    if (threadIdx.x == 0 && zl[0] != 0) atomicAdd(cnt, 1);
}
void debug_count_zl(Ctx &c, const int *zl, int *cnt)
{
    k_dbg_zl<<<1, 64, 0, c.stream>>>(zl, cnt);
    HEC_HIP(hipGetLastError());
}

// ================================================================================ hoisted mod-up ==
// A trie node's rotations all key-switch digits of the same polynomial, permuted.  With D = INTT(c1)
// of the node (canonical, coefficient form) the child for Galois element elt has digit J
//   d'_J[t] = D_J[u]            if u = t elt^-1 mod 2N < N
//           = q_J - D_J[u - N]  if u >= N and D_J[u - N] != 0,   0 if D_J[u - N] == 0,
// so for I != J, mod q_I and in the NTT domain (SEAL's apply_galois_ntt permutation, gal()):
//   NTT_I(d'_J mod q_I)[k] = E_J[I][gal(k)] + (q_J mod q_I) W_elt,I[k]
//                            - (q_J mod q_I) sum over zeros D_J[u] = 0 that land negated at t of psi_I^((2 bitrev(k) + 1) t)
// with E_J[I] = NTT_I(D_J mod q_I) computed once per node and W_elt,I = NTT_I(sign mask of elt) once
// per key.  Every term is exact mod q_I, so each child's key-switch input equals SEAL's bit for bit,
// while the node's mod-up NTTs are shared by all its children.  Zero positions are listed per (b, J)
// by k_zscan (at most HEC_ZCAP; more raises zflag and the caller recomputes without hoisting).
// zl layout: zl[0] = zeros in the node (any limb), then per limb: count, HEC_ZCAP positions
__global__ void __launch_bounds__(256) k_zscan(const u64 *__restrict__ D, int *__restrict__ zl, int *zflag, int logN)
{
    const u64 N = 1ull << logN;
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    if (g >= N) return;
    const int limb = blockIdx.y;
    if (D[((u64)limb << logN) + g] == 0) zero_record(zl, zflag, limb, (int)g);
}

void zero_scan(Ctx &c, const u64 *D, int nlimbs, int *zl)
{
    dev_zero(c, zl, (1 + (std::size_t)nlimbs * (HEC_ZCAP + 1)) * sizeof(int));
    k_zscan<<<dim3((unsigned)(c.N / 256), nlimbs), 256, 0, c.stream>>>(D, zl, c.zflag, c.logN);
    HEC_HIP(hipGetLastError());
}

// The hoisted key MAC of one child: ACC[b][k][I] = sum_J e_J[I] key[J][k][I] over the node's canonical
// NTT-form digits E[b][I][J] (J != I) through the child's permutation plus the sign-mask term above,
// and the child's own NTT-form target T = gal(c1) for J == I.  A thread owns two adjacent coefficients
// (their sources are adjacent too) for BT batch entries, so each key and W word is read once per BT.
// Grid: 1-D, XCD-aware like k_bmac (the batch groups of one (coefficient block, I) share an XCD).
// zero corrections for the (b, J) digit of coefficients k0, k0 + 1 (rare: only zeros of D_J that this
// child negates)
__device__ __forceinline__ void hmac_zero_fix(u64 &e0, u64 &e1, const int *z, u64 c, u64 k0, u32 elt, int logN,
                                              const u64 *__restrict__ pp, const DevPrime &pr)
{
    const u64 N = 1ull << logN;
    const int nz = min(z[0], HEC_ZCAP);
    for (int zi = 0; zi < nz; ++zi) {
        u64 tt = ((u64)z[1 + zi] * elt) & (2 * N - 1);
        if (tt < N) continue;
        tt -= N;
        const u64 ex0 = ((2 * (u64)bitrev((u32)k0, logN) + 1) * tt) & (2 * N - 1);
        const u64 ex1 = ((2 * (u64)bitrev((u32)k0 + 1, logN) + 1) * tt) & (2 * N - 1);
        e0 = submod(e0, mulmod(c, pp[ex0], pr), pr.q);
        e1 = submod(e1, mulmod(c, pp[ex1], pr), pr.q);
    }
}

template <int BT, bool FP>
__device__ __forceinline__ void hmac_body(PolyArr X1, const u64 *__restrict__ E, const u64 *__restrict__ W,
                                          const int *__restrict__ zl, const u64 *__restrict__ key,
                                          u64 *__restrict__ ACC, int B, int l, int K, int logN, const DevPrime &pr,
                                          int I, int kI, u64 k0, int b0, const u64 *__restrict__ cji,
                                          const u64 *__restrict__ psipow, u32 elt)
{
    const u32 gs = galois_src((u32)k0, elt, logN);  // gal(k0 + 1) = gs ^ 1
    const u64 sp = gs & ~1u;
    const bool swp = gs & 1;
    const ulonglong2 wv = *(const ulonglong2 *)(W + ((u64)kI << logN) + k0);
    const bool zeros = zl[0] != 0;  // any zero coefficient in the node's digits (rare)
    const u64 *pp = psipow + ((u64)kI << (logN + 1));
    double f0[FP ? BT : 1][2], f1[FP ? BT : 1][2];
    U128 a0[FP ? 1 : BT][2], a1[FP ? 1 : BT][2];
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        if constexpr (FP) f0[t][0] = f0[t][1] = f1[t][0] = f1[t][1] = 0.0;
        else a0[t][0] = a0[t][1] = a1[t][0] = a1[t][1] = U128{0, 0};
    }
    for (int J = 0; J < l; ++J) {
        const ulonglong2 key0 = *(const ulonglong2 *)(key + (((u64)(J * 2 + 0) * K + kI) << logN) + k0);
        const ulonglong2 key1 = *(const ulonglong2 *)(key + (((u64)(J * 2 + 1) * K + kI) << logN) + k0);
        const u64 c = cji[J * K + kI];
        u64 cw0 = 0, cw1 = 0;
        double cf0 = 0, cf1 = 0, k00 = 0, k01 = 0, k10 = 0, k11 = 0;
        if constexpr (FP) {
            if (J != I) {
                cf0 = fp_mulmod(u2d(c), u2d(wv.x), pr.qd, pr.qinv);
                cf1 = fp_mulmod(u2d(c), u2d(wv.y), pr.qd, pr.qinv);
            }
            k00 = u2d(key0.x); k01 = u2d(key0.y); k10 = u2d(key1.x); k11 = u2d(key1.y);
        } else if (J != I) {
            cw0 = mulmod(c, wv.x, pr);
            cw1 = mulmod(c, wv.y, pr);
        }
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b >= B) break;
            const u64 *src = J == I ? X1.p + b * X1.sb + ((u64)J << logN)
                                    : E + (((u64)((b * (l + 1) + I) * l + J)) << logN);
            const ulonglong2 v = *(const ulonglong2 *)(src + sp);
            u64 e0 = swp ? v.y : v.x, e1 = swp ? v.x : v.y;
            if (J != I && zeros) hmac_zero_fix(e0, e1, zl + 1 + (b * l + J) * (HEC_ZCAP + 1), c, k0, elt, logN, pp, pr);
            if constexpr (FP) {
                const double d0 = u2d(e0) + cf0, d1 = u2d(e1) + cf1;  // |d| < 1.6 q
                f0[t][0] += fp_mulmod(d0, k00, pr.qd, pr.qinv);
                f0[t][1] += fp_mulmod(d1, k01, pr.qd, pr.qinv);
                f1[t][0] += fp_mulmod(d0, k10, pr.qd, pr.qinv);
                f1[t][1] += fp_mulmod(d1, k11, pr.qd, pr.qinv);
            } else {
                if (J != I) {
                    e0 = addmod(e0, cw0, pr.q);
                    e1 = addmod(e1, cw1, pr.q);
                }
                mac128(a0[t][0], e0, key0.x);
                mac128(a0[t][1], e1, key0.y);
                mac128(a1[t][0], e0, key1.x);
                mac128(a1[t][1], e1, key1.y);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        const int b = b0 + t;
        if (b >= B) break;
        u64 *o0 = ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + k0;
        u64 *o1 = ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + k0;
        if constexpr (FP) {
            *(ulonglong2 *)o0 = ulonglong2{fp_canon(f0[t][0], pr.qd, pr.qinv), fp_canon(f0[t][1], pr.qd, pr.qinv)};
            *(ulonglong2 *)o1 = ulonglong2{fp_canon(f1[t][0], pr.qd, pr.qinv), fp_canon(f1[t][1], pr.qd, pr.qinv)};
        } else {
            *(ulonglong2 *)o0 = ulonglong2{barrett128(a0[t][0].lo, a0[t][0].hi, pr.q, pr.r0, pr.r1),
                                           barrett128(a0[t][1].lo, a0[t][1].hi, pr.q, pr.r0, pr.r1)};
            *(ulonglong2 *)o1 = ulonglong2{barrett128(a1[t][0].lo, a1[t][0].hi, pr.q, pr.r0, pr.r1),
                                           barrett128(a1[t][1].lo, a1[t][1].hi, pr.q, pr.r0, pr.r1)};
        }
    }
}

// The hoisted key MAC of one child: ACC[b][k][I] = sum_J e_J[I] key[J][k][I] over the node's canonical
// NTT-form digits E[b][I][J] (J != I) through the child's permutation plus the sign-mask term above,
// and the child's own NTT-form target T = gal(c1) for J == I.  A thread owns two adjacent coefficients
// (their sources are adjacent too) for BT batch entries, so each key and W word is read once per BT.
// FP64 primes accumulate exact fp_mulmod products, 60-bit primes 128-bit sums (SEAL's lazy MAC).
// Grid: 1-D, XCD-aware like k_bmac (the batch groups of one (coefficient block, I) share an XCD).
template <int BT>
__global__ void __launch_bounds__(256)
    k_hmac(PolyArr X1, const u64 *__restrict__ E, const u64 *__restrict__ W, const int *__restrict__ zl,
           const u64 *__restrict__ key, u64 *__restrict__ ACC, int B, int l, int K, int logN,
           const DevPrime *__restrict__ primes, const int *__restrict__ Imap, int nI, const u64 *__restrict__ cji,
           const u64 *__restrict__ psipow, u32 elt, int gpad)
{
    const u64 N = 1ull << logN;
    const int nbg = (B + BT - 1) / BT;
    const int w = blockIdx.x;
    const int g8 = w & 7, rest = w >> 3, bg = rest % nbg, G = (rest / nbg) * 8 + g8;
    const int X = (int)(N / 512);
    if (G >= X * nI) return;
    const int yi = G / X, xb = G % X;
    const int I = Imap[yi];
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    const u64 k0 = (u64)xb * 512 + 2 * threadIdx.x;  // this thread's coefficients k0, k0 + 1
    if (pr.fp)
        hmac_body<BT, true>(X1, E, W, zl, key, ACC, B, l, K, logN, pr, I, kI, k0, bg * BT, cji, psipow, elt);
    else
        hmac_body<BT, false>(X1, E, W, zl, key, ACC, B, l, K, logN, pr, I, kI, k0, bg * BT, cji, psipow, elt);
}

void hoisted_mac(Ctx &c, PolyArr X1, const u64 *E, const u64 *W, const int *zl, const u64 *key, u64 *ACC, int B,
                 int l, u32 elt)
{
    constexpr int BT = 4;
    const int nbg = (B + BT - 1) / BT, X = (int)(c.N / 512), gpad = (X * (l + 1) + 7) / 8 * 8;
    k_hmac<BT><<<dim3((unsigned)(gpad * nbg)), 256, 0, c.stream>>>(X1, E, W, zl, key, ACC, B, l, (int)c.K, c.logN,
                                                                    c.primes, c.imap_at(l), l + 1, c.cji, c.psipow,
                                                                    elt, gpad);
    HEC_HIP(hipGetLastError());
}

// Sibling-fused hoisted MAC: the thread owns two adjacent SOURCE positions s, s + 1 of the node's digits
// (read once, contiguous) and scatters their products to up to CG children: child c's output position is
// k_c = gal_c^-1(s) (the inverse permutation is the Galois map of elt^-1), its key, sign-mask and zero
// terms are gathered there.  The digits, the largest stream, are read once per CG children.
struct HChild {
    u32 elt, einv;
    const u64 *key, *W;
    u64 *ACC;
    const u64 *KW;
    const u64 *MK;  // the key in MAC form and source order (mac_key_table)
};
template <int CG>
struct HChildren {
    HChild c[CG];
    int n;
};

// The sign-mask term is linear in the digits, so it leaves the digit loop:
//   ACC = sum_J key_J (E_J o gal - c_J Z_J) + W_elt KW,  KW = sum_{J != I} c_J key_J  (k_keyw, per key and level)
// with c_J = q_J mod q_I and Z_J the (rare) zero corrections: one modular product per child and output word
// instead of one per digit.  Every term is exact mod q_I, so the canonical result is unchanged.
// X0.p != nullptr: the node's c0, folded into every child's c0 accumulator at the data primes as X0 (P mod q_I), so
// the mod-down's (ACC - r) P^-1 already carries the IN term and its pass B reads one operand less (DivRoundIOB<false>).
// The output position k of child c has source position gal_c(k) = s (hmacm's thread positions), so the term is the
// same word X0[s] for every child.
// MAC form (round 6): the FP64-class operands of the hoisted MAC as the k_hmacm loop consumes them, so it converts
// nothing: the canonical residue as the bits of its integer-valued double.  The digits E of a hoisted node are stored
// this way at the FP64 targets by their pass B (ModUpIO_B mform), the children's keys by mac_key_table (per Galois
// key, also permuted into the node's source order, below).  (A split form for the 60-bit targets, lo30 | hi30 << 32
// with four v_mad_u64_u32 per product and no carry chain, fit the register budget only at one batch entry per thread
// and lost: k_hmacm 2,699-2,720 vs 2,501-2,540 ms per step at B = 128; the 60-bit targets keep the u64 loop.)
__device__ __forceinline__ u64 mform(u64 v, bool fp) { return fp ? (u64)__double_as_longlong(u2d(v)) : v; }

// The digit loop of k_hmacm at the FP64 targets on MAC-form operands (round 6).  The thread's two source positions
// s0, s0 + 1 read the digit words E[b][I][J][s0..] and each child's key words MK_c[J][k][I][s0..] (mac_key_table:
// key_c at gal_c(s) = galois_src(s, einv_c), so both streams are contiguous and in the same order, and no pair swap
// happens inside the loop); the accumulators stay in source order and take the child's output order (kc, sw) at the
// store.  The loop is unrolled by two with explicit double buffers (digit J + 1's words load while digit J
// multiplies), so no register is copied per digit; exact fp_mulmod products summed as doubles.  The J == I digit is
// the child's own NTT-form c1 (canonical u64, converted once).  The zero corrections are k_hmacm_zfix's.
template <int BT, int CG>
__device__ __forceinline__ void hmacm_body(PolyArr X1, PolyArr X0, const u64 *__restrict__ E, const HChildren<CG> &ch,
                                           int B, int l, int K, int logN, const DevPrime &pr, u64 Pq, int I, int kI,
                                           u64 s0, int b0)
{
    const u64 N = 1ull << logN;
    u64 kc[CG];         // even slot of child c's output pair
    bool sw[CG];        // output pair swapped
    double f[CG][BT][4];
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        double wk[4] = {0, 0, 0, 0};  // W KW in source order: (k = 0: s0, s0 + 1), (k = 1: s0, s0 + 1)
        if (q < ch.n) {
            const u32 t = galois_src((u32)s0, ch.c[q].einv, logN);
            kc[q] = t & ~1u;
            sw[q] = t & 1;
            const ulonglong2 w = *(const ulonglong2 *)(ch.c[q].W + ((u64)kI << logN) + kc[q]);
            const ulonglong2 m0 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)I << logN) + kc[q]);
            const ulonglong2 m1 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)(l + 1 + I) << logN) + kc[q]);
            // the exact FP64 products (residues in [-0.53 q, 0.53 q]) start the sums
            const double wx = u2d(w.x), wy = u2d(w.y);
            wk[0] = fp_mulmod(wx, u2d(m0.x), pr.qd, pr.qinv);
            wk[1] = fp_mulmod(wy, u2d(m0.y), pr.qd, pr.qinv);
            wk[2] = fp_mulmod(wx, u2d(m1.x), pr.qd, pr.qinv);
            wk[3] = fp_mulmod(wy, u2d(m1.y), pr.qd, pr.qinv);
            if (sw[q]) {
                double x = wk[0]; wk[0] = wk[1]; wk[1] = x;
                x = wk[2]; wk[2] = wk[3]; wk[3] = x;
            }
        }
#pragma unroll
        for (int t = 0; t < BT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) f[q][t][r] = wk[r];
    }
    if (X0.p != nullptr && I < l) {  // + X0 (P mod q_I) on the c0 accumulators (exact residues, as every other term)
        const double pmd = u2d(barrett64(Pq, pr.q, pr.r1));
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const ulonglong2 x0 = *(const ulonglong2 *)(X0.p + min(b0 + t, B - 1) * X0.sb + ((u64)I << logN) + s0);
            const double t0 = fp_mulmod(u2d(x0.x), pmd, pr.qd, pr.qinv);
            const double t1 = fp_mulmod(u2d(x0.y), pmd, pr.qd, pr.qinv);
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                f[q][t][0] += t0;
                f[q][t][1] += t1;
            }
        }
    }
    // The digit and key streams as buffer loads: a block-uniform descriptor per stream (E of batch entry t at (b, I),
    // digit 0; MK of child q at limb kI, digit 0), the digit's uniform byte offset in an SGPR (soffset) and the
    // thread's source offset so = 8 s0 as the one VGPR offset of every load: no per-load address arithmetic, and
    // no address registers beside the double buffers.  A missing batch entry (b >= B, last batch group only) reads
    // entry B - 1's words and stores nothing.
    const u32 so = (u32)s0 * 8u, NB = (u32)(N * 8), KNB = (u32)(((u64)K << logN) * 8);
    __amdgpu_buffer_rsrc_t rE[BT], rK[CG];
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        const int b = min(b0 + t, B - 1);
        rE[t] = __builtin_amdgcn_make_buffer_rsrc((void *)(E + (((u64)((b * (l + 1) + I) * l)) << logN)), (short)0,
                                                  (int)((u32)l * NB), 0x00020000);
    }
#pragma unroll
    for (int q = 0; q < CG; ++q)
        rK[q] = __builtin_amdgcn_make_buffer_rsrc((void *)(ch.c[q < ch.n ? q : 0].MK + ((u64)kI << logN)), (short)0,
                                                  (int)((u32)(2 * l) * KNB), 0x00020000);
    auto ld = [](__amdgpu_buffer_rsrc_t r, u32 vo, u32 soff) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, soff, 0);
        return ulonglong2{(u64)v[1] << 32 | v[0], (u64)v[3] << 32 | v[2]};
    };
    // every load is issued unconditionally (a missing child reads child 0's words, unused): a load under a branch
    // would make every later wait count the loads of the path without it, and the waits would drain the prefetch
    auto load = [&](int J, ulonglong2 *e, ulonglong2 (*k)[2]) {
#pragma unroll
        for (int t = 0; t < BT; ++t) e[t] = ld(rE[t], so, (u32)J * NB);
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            k[q][0] = ld(rK[q], so, (u32)(2 * J) * KNB);
            k[q][1] = ld(rK[q], so, (u32)(2 * J + 1) * KNB);
        }
    };
    // one product's dependency chain at a time (A/B round 6: the products interleaved two by two, with one key buffer
    // reloaded per child as its products issue, measured slower: k_hmacm 2,405-2,440 vs 2,378-2,398 ms per step)
    auto mac = [&](const ulonglong2 *e, ulonglong2 (*k)[2]) {
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            if (q >= ch.n) break;
#pragma unroll
            for (int t = 0; t < BT; ++t) {
                if (b0 + t >= B) break;
                const double d0 = __longlong_as_double((long long)e[t].x);
                const double d1 = __longlong_as_double((long long)e[t].y);
                f[q][t][0] += fp_mulmod(d0, __longlong_as_double((long long)k[q][0].x), pr.qd, pr.qinv);
                f[q][t][1] += fp_mulmod(d1, __longlong_as_double((long long)k[q][0].y), pr.qd, pr.qinv);
                f[q][t][2] += fp_mulmod(d0, __longlong_as_double((long long)k[q][1].x), pr.qd, pr.qinv);
                f[q][t][3] += fp_mulmod(d1, __longlong_as_double((long long)k[q][1].y), pr.qd, pr.qinv);
            }
        }
    };
    ulonglong2 eA[BT], eB[BT], kA[CG][2], kB[CG][2];
    // the digits J != I of the loop (I == l, the special prime, has no J == I digit)
    const int nd = I < l ? l - 1 : l;
    auto dig = [I](int k) { return k + (k >= I ? 1 : 0); };
    if (I < l) {  // the J == I digit: the child's own NTT-form c1 (canonical u64), converted here
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const ulonglong2 v = *(const ulonglong2 *)(X1.p + min(b0 + t, B - 1) * X1.sb + ((u64)I << logN) + s0);
            eB[t] = ulonglong2{mform(v.x, true), mform(v.y, true)};
        }
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            kB[q][0] = ld(rK[q], so, (u32)(2 * I) * KNB);
            kB[q][1] = ld(rK[q], so, (u32)(2 * I + 1) * KNB);
        }
        if (nd > 0) load(dig(0), eA, kA);
        mac(eB, kB);
    } else if (nd > 0) {
        load(dig(0), eA, kA);
    }
    // the loop body's loads are unconditional (the tail is peeled): a load under a branch would make the waits after
    // it count the loads of the path without it, and they would drain the prefetch
    int k = 0;
    for (; k + 2 < nd; k += 2) {
        load(dig(k + 1), eB, kB);
        mac(eA, kA);
        load(dig(k + 2), eA, kA);
        mac(eB, kB);
    }
    if (k + 1 < nd) {  // two digits left
        load(dig(k + 1), eB, kB);
        mac(eA, kA);
        mac(eB, kB);
    } else if (k < nd) {
        mac(eA, kA);
    }
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        if (q >= ch.n) break;
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b >= B) break;
            u64 r[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = fp_canon(f[q][t][i], pr.qd, pr.qinv);
            u64 *o0 = ch.c[q].ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + kc[q];
            u64 *o1 = ch.c[q].ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + kc[q];
            st2m<4>(o0, sw[q] ? ulonglong2{r[1], r[0]} : ulonglong2{r[0], r[1]});
            st2m<4>(o1, sw[q] ? ulonglong2{r[3], r[2]} : ulonglong2{r[2], r[3]});
        }
    }
}

// The round-5 digit loop for the 60-bit targets (HEC_HMAC_INT=0; the default is hmacm_body_int below): canonical u64
// operands, the original key gathered at the child's output slots, 128-bit lazy sums, BT batch entries per thread.
template <int BT, int CG>
__device__ __forceinline__ void hmacm_body_u64(PolyArr X1, PolyArr X0, const u64 *__restrict__ E,
                                           const HChildren<CG> &ch, int B, int l, int K, int logN, const DevPrime &pr,
                                           u64 Pq, int I, int kI, u64 s0, int b0)
{
    u64 kc[CG];       // even slot of child c's output pair
    bool sw[CG];      // output pair swapped
    u64 wk[CG][4];    // W KW in source order: (k = 0: s0, s0 + 1), (k = 1: s0, s0 + 1)
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        if (q >= ch.n) break;
        const u32 t = galois_src((u32)s0, ch.c[q].einv, logN);
        kc[q] = t & ~1u;
        sw[q] = t & 1;
        const ulonglong2 w = *(const ulonglong2 *)(ch.c[q].W + ((u64)kI << logN) + kc[q]);
        const ulonglong2 m0 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)I << logN) + kc[q]);
        const ulonglong2 m1 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)(l + 1 + I) << logN) + kc[q]);
        wk[q][0] = mulmod(w.x, m0.x, pr);
        wk[q][1] = mulmod(w.y, m0.y, pr);
        wk[q][2] = mulmod(w.x, m1.x, pr);
        wk[q][3] = mulmod(w.y, m1.y, pr);
        if (sw[q]) {
            u64 x = wk[q][0]; wk[q][0] = wk[q][1]; wk[q][1] = x;
            x = wk[q][2]; wk[q][2] = wk[q][3]; wk[q][3] = x;
        }
    }
    // the folded c0 words, loaded first: their wait (for the products below) is then the oldest in issue order and
    // does not include the digit and key prefetches issued after them
    const bool fold = X0.p != nullptr && I < l;
    ulonglong2 x0v[BT];
    if (fold) {
#pragma unroll
        for (int t = 0; t < BT; ++t)
            x0v[t] = b0 + t < B ? *(const ulonglong2 *)(X0.p + (b0 + t) * X0.sb + ((u64)I << logN) + s0)
                                : ulonglong2{0, 0};
    }
    U128 a[CG][BT][4];
#pragma unroll
    for (int q = 0; q < CG; ++q)
#pragma unroll
        for (int t = 0; t < BT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) a[q][t][r] = U128{q < ch.n ? wk[q][r] : 0, 0};
    if (fold) {  // + X0 (P mod q_I) on the c0 accumulators (exact residues, as every other term)
        const u64 pm = barrett64(Pq, pr.q, pr.r1);
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const u64 t0 = mulmod(x0v[t].x, pm, pr), t1 = mulmod(x0v[t].y, pm, pr);
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                a[q][t][0].lo += t0;
                a[q][t][0].hi += a[q][t][0].lo < t0;
                a[q][t][1].lo += t1;
                a[q][t][1].hi += a[q][t][1].lo < t1;
            }
        }
    }
    auto digit = [&](int J, int t) -> ulonglong2 {
        const int b = b0 + t;
        const u64 *src = J == I ? X1.p + b * X1.sb + ((u64)J << logN) : E + (((u64)((b * (l + 1) + I) * l + J)) << logN);
        return b < B ? *(const ulonglong2 *)(src + s0) : ulonglong2{0, 0};
    };
    // software pipeline: digit J + 1 is loaded before digit J's products, so a wave keeps its next HBM reads in
    // flight through its own MAC work (round 3: 1,961 vs 2,266 ms per step at cfg3)
    ulonglong2 pf[BT];
#pragma unroll
    for (int t = 0; t < BT; ++t) pf[t] = digit(0, t);
    auto keyw = [&](int J, int q, int k) -> ulonglong2 {
        return *(const ulonglong2 *)(ch.c[q].key + (((u64)(J * 2 + k) * K + kI) << logN) + kc[q]);
    };
    ulonglong2 kpf[CG][2];  // and the children's key words of digit J + 1 (143 VGPRs, 3 waves/SIMD: 1,898-1,904 vs
                            // 1,929-1,934 ms with the digits alone ahead)
#pragma unroll
    for (int q = 0; q < CG; ++q)
        if (q < ch.n) kpf[q][0] = keyw(0, q, 0), kpf[q][1] = keyw(0, q, 1);
    for (int J = 0; J < l; ++J) {
        u64 ev[BT][2];
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            ev[t][0] = pf[t].x;
            ev[t][1] = pf[t].y;
        }
        if (J + 1 < l) {
#pragma unroll
            for (int t = 0; t < BT; ++t) pf[t] = digit(J + 1, t);
        }
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            if (q >= ch.n) break;
            ulonglong2 k0 = kpf[q][0], k1 = kpf[q][1];
            if (J + 1 < l) kpf[q][0] = keyw(J + 1, q, 0), kpf[q][1] = keyw(J + 1, q, 1);
            if (sw[q]) {
                k0 = ulonglong2{k0.y, k0.x};
                k1 = ulonglong2{k1.y, k1.x};
            }
#pragma unroll
            for (int t = 0; t < BT; ++t) {
                if (b0 + t >= B) break;
                const u64 e0 = ev[t][0], e1 = ev[t][1];
                mac128(a[q][t][0], e0, k0.x);
                mac128(a[q][t][1], e1, k0.y);
                mac128(a[q][t][2], e0, k1.x);
                mac128(a[q][t][3], e1, k1.y);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        if (q >= ch.n) break;
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b >= B) break;
            u64 r[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = barrett128(a[q][t][i].lo, a[q][t][i].hi, pr.q, pr.r0, pr.r1);
            u64 *o0 = ch.c[q].ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + kc[q];
            u64 *o1 = ch.c[q].ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + kc[q];
            st2m<4>(o0, sw[q] ? ulonglong2{r[1], r[0]} : ulonglong2{r[0], r[1]});
            st2m<4>(o1, sw[q] ? ulonglong2{r[3], r[2]} : ulonglong2{r[2], r[3]});
        }
    }
}

// The 60-bit targets on the MAC-form streams (round 6): the FP64 body's loads (source-ordered key table MK, canonical
// u64 at these limbs; buffer loads; the J == I digit before the loop; unconditional double-buffered loads) with SEAL's
// 128-bit lazy sums, one Barrett reduction per output word.  HEC_HMAC_INT=0: the round-5 loop above.
template <int BT, int CG>
__device__ __forceinline__ void hmacm_body_int(PolyArr X1, PolyArr X0, const u64 *__restrict__ E, const HChildren<CG> &ch,
                                               int B, int l, int K, int logN, const DevPrime &pr, u64 Pq, int I,
                                               int kI, u64 s0, int b0)
{
    const u64 N = 1ull << logN;
    u64 kc[CG];
    bool sw[CG];
    U128 a[CG][BT][4];
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        u64 wk[4] = {0, 0, 0, 0};
        if (q < ch.n) {
            const u32 t = galois_src((u32)s0, ch.c[q].einv, logN);
            kc[q] = t & ~1u;
            sw[q] = t & 1;
            const ulonglong2 w = *(const ulonglong2 *)(ch.c[q].W + ((u64)kI << logN) + kc[q]);
            const ulonglong2 m0 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)I << logN) + kc[q]);
            const ulonglong2 m1 = *(const ulonglong2 *)(ch.c[q].KW + ((u64)(l + 1 + I) << logN) + kc[q]);
            wk[0] = mulmod(w.x, m0.x, pr);
            wk[1] = mulmod(w.y, m0.y, pr);
            wk[2] = mulmod(w.x, m1.x, pr);
            wk[3] = mulmod(w.y, m1.y, pr);
            if (sw[q]) {
                u64 x = wk[0]; wk[0] = wk[1]; wk[1] = x;
                x = wk[2]; wk[2] = wk[3]; wk[3] = x;
            }
        }
#pragma unroll
        for (int t = 0; t < BT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) a[q][t][r] = U128{wk[r], 0};
    }
    if (X0.p != nullptr && I < l) {  // + X0 (P mod q_I) on the c0 accumulators
        const u64 pm = barrett64(Pq, pr.q, pr.r1);
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const ulonglong2 x0 = *(const ulonglong2 *)(X0.p + min(b0 + t, B - 1) * X0.sb + ((u64)I << logN) + s0);
            const u64 t0 = mulmod(x0.x, pm, pr), t1 = mulmod(x0.y, pm, pr);
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                a[q][t][0].lo += t0;
                a[q][t][0].hi += a[q][t][0].lo < t0;
                a[q][t][1].lo += t1;
                a[q][t][1].hi += a[q][t][1].lo < t1;
            }
        }
    }
    const u32 so = (u32)s0 * 8u, NB = (u32)(N * 8), KNB = (u32)(((u64)K << logN) * 8);
    __amdgpu_buffer_rsrc_t rE[BT], rK[CG];
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        const int b = min(b0 + t, B - 1);
        rE[t] = __builtin_amdgcn_make_buffer_rsrc((void *)(E + (((u64)((b * (l + 1) + I) * l)) << logN)), (short)0,
                                                  (int)((u32)l * NB), 0x00020000);
    }
#pragma unroll
    for (int q = 0; q < CG; ++q)
        rK[q] = __builtin_amdgcn_make_buffer_rsrc((void *)(ch.c[q < ch.n ? q : 0].MK + ((u64)kI << logN)), (short)0,
                                                  (int)((u32)(2 * l) * KNB), 0x00020000);
    auto ld = [](__amdgpu_buffer_rsrc_t r, u32 vo, u32 soff) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, soff, 0);
        return ulonglong2{(u64)v[1] << 32 | v[0], (u64)v[3] << 32 | v[2]};
    };
    auto load = [&](int J, ulonglong2 *e, ulonglong2 (*k)[2]) {
#pragma unroll
        for (int t = 0; t < BT; ++t) e[t] = ld(rE[t], so, (u32)J * NB);
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            k[q][0] = ld(rK[q], so, (u32)(2 * J) * KNB);
            k[q][1] = ld(rK[q], so, (u32)(2 * J + 1) * KNB);
        }
    };
    auto mac = [&](const ulonglong2 *e, ulonglong2 (*k)[2]) {
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            if (q >= ch.n) break;
#pragma unroll
            for (int t = 0; t < BT; ++t) {
                if (b0 + t >= B) break;
                mac128(a[q][t][0], e[t].x, k[q][0].x);
                mac128(a[q][t][1], e[t].y, k[q][0].y);
                mac128(a[q][t][2], e[t].x, k[q][1].x);
                mac128(a[q][t][3], e[t].y, k[q][1].y);
            }
        }
    };
    ulonglong2 eA[BT], eB[BT], kA[CG][2], kB[CG][2];
    const int nd = I < l ? l - 1 : l;
    auto dig = [I](int k) { return k + (k >= I ? 1 : 0); };
    if (I < l) {  // the J == I digit: the child's own NTT-form c1
#pragma unroll
        for (int t = 0; t < BT; ++t)
            eB[t] = *(const ulonglong2 *)(X1.p + min(b0 + t, B - 1) * X1.sb + ((u64)I << logN) + s0);
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            kB[q][0] = ld(rK[q], so, (u32)(2 * I) * KNB);
            kB[q][1] = ld(rK[q], so, (u32)(2 * I + 1) * KNB);
        }
        if (nd > 0) load(dig(0), eA, kA);
        mac(eB, kB);
    } else if (nd > 0) {
        load(dig(0), eA, kA);
    }
    int k = 0;
    for (; k + 2 < nd; k += 2) {
        load(dig(k + 1), eB, kB);
        mac(eA, kA);
        load(dig(k + 2), eA, kA);
        mac(eB, kB);
    }
    if (k + 1 < nd) {
        load(dig(k + 1), eB, kB);
        mac(eA, kA);
        mac(eB, kB);
    } else if (k < nd) {
        mac(eA, kA);
    }
#pragma unroll
    for (int q = 0; q < CG; ++q) {
        if (q >= ch.n) break;
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b >= B) break;
            u64 r[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = barrett128(a[q][t][i].lo, a[q][t][i].hi, pr.q, pr.r0, pr.r1);
            u64 *o0 = ch.c[q].ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + kc[q];
            u64 *o1 = ch.c[q].ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + kc[q];
            st2m<4>(o0, sw[q] ? ulonglong2{r[1], r[0]} : ulonglong2{r[0], r[1]});
            st2m<4>(o1, sw[q] ? ulonglong2{r[3], r[2]} : ulonglong2{r[2], r[3]});
        }
    }
}

// The MAC-form key table of one Galois key for the hoisted MAC: MK[J][k][I][s] = mform(key[J][k][I][galois_src(s,
// einv)]) over the key's L digits, 2 polys and K limbs (einv = elt^-1 mod 2N: the child's output position of source s)
__global__ void __launch_bounds__(256) k_mac_key(const u64 *__restrict__ key, u64 *__restrict__ MK, u32 einv, int K,
                                                 int logN, const DevPrime *__restrict__ primes)
{
    const u64 N = 1ull << logN;
    const u64 s = (u64)blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y, I = row % K;  // row = (J 2 + k) K + I
    if (s >= N) return;
    const bool fp = cprime(primes, I).fp != 0;
    const u64 v = key[((u64)row << logN) + galois_src((u32)s, einv, logN)];
    MK[((u64)row << logN) + s] = mform(v, fp);
}

void mac_key_table(Ctx &c, const u64 *key, u64 *MK, u32 einv)
{
    k_mac_key<<<dim3((unsigned)((c.N + 255) / 256), (unsigned)(c.L * 2 * c.K)), 256, 0, c.stream>>>(
        key, MK, einv, (int)c.K, c.logN, c.primes);
    HEC_HIP(hipGetLastError());
}

// KW[k][I][t] = sum_{J<l, J != I} (q_J mod q_I) key[J][k][I][t] mod q_I (128-bit lazy sum, one Barrett)
__global__ void __launch_bounds__(256) k_keyw(const u64 *__restrict__ key, u64 *__restrict__ KW, int l, int K,
                                              int logN, const DevPrime *__restrict__ primes,
                                              const u64 *__restrict__ cji)
{
    const u64 N = 1ull << logN;
    const u64 t = (u64)blockIdx.x * 256 + threadIdx.x;
    const int I = blockIdx.y, k = blockIdx.z;
    if (t >= N) return;
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    U128 acc{0, 0};
    for (int J = 0; J < l; ++J)
        if (J != I) mac128(acc, cji[J * K + kI], key[(((u64)(J * 2 + k) * K + kI) << logN) + t]);
    KW[((u64)(k * (l + 1) + I) << logN) + t] = barrett128(acc.lo, acc.hi, pr.q, pr.r0, pr.r1);
}

void key_wsum(Ctx &c, const u64 *key, u64 *KW, int l)
{
    k_keyw<<<dim3((unsigned)(c.N / 256), l + 1, 2), 256, 0, c.stream>>>(key, KW, l, (int)c.K, c.logN, c.primes,
                                                                        c.cji);
    HEC_HIP(hipGetLastError());
}

// Children slots of one k_hmacm launch: NS groups of CG siblings (round 5: a whole sibling group of up to 6 in one
// launch, 3 slots of 2, instead of one launch per pair)
template <int CG, int NS>
struct HSlots {
    HChildren<CG> s[NS];
    int ns;
};

// Two grid segments: the integer-arithmetic targets (Imap[0, nint), 128-bit accumulators) with BTI batch
// entries per thread, then the FP64 targets with BTF, so neither class carries the other's register
// budget.  Each segment is XCD-aware: the batch groups of one (coefficient block, I) share an XCD, and the ns slots
// of one (coefficient block, I, batch group) — the same digit tile E, the node's c1 / c0 words, different children —
// are consecutive blocks of that XCD (ids w, w + 8, w + 16): the tile comes from HBM for the first and from the XCD's
// L2 for the others, so the digits, the kernel's largest stream, cross HBM once per sibling group, not per pair.
template <int BTF, int BTI, int CG, int MINW, int NS>
__global__ void __launch_bounds__(256, MINW)  // MINW waves per SIMD: 3 -> <= 168 VGPRs, 2 -> <= 256
    k_hmacm(PolyArr X1, PolyArr X0, const u64 *__restrict__ E, const int *__restrict__ zl, const HSlots<CG, NS> S,
            int B, int l, int K, int logN, const DevPrime *__restrict__ primes, const int *__restrict__ Imap, int nI,
            int nint, const u64 *__restrict__ cji, const u64 *__restrict__ psipow, int wsplit, int int_mform)
{
    const u64 N = 1ull << logN;
    const int X = (int)(N / 512);
    const int ns = NS == 1 ? 1 : S.ns;
    const int t8 = (int)blockIdx.x >> 3, slot = NS == 1 ? 0 : t8 % ns;
    const int wb = (NS == 1 ? t8 : t8 / ns) * 8 + ((int)blockIdx.x & 7);  // the block index without the slot
    const HChildren<CG> ch = S.s[slot];
    const bool integer = wb < wsplit;
    const int bt = integer ? BTI : BTF;
    const int nbg = (B + bt - 1) / bt;
    const int w = integer ? wb : wb - wsplit;
    const int g8 = w & 7, rest = w >> 3, bg = rest % nbg, G = (rest / nbg) * 8 + g8;
    if (G >= X * (integer ? nint : nI - nint)) return;
    const int yi = G / X + (integer ? 0 : nint), xb = G % X;
    const int I = Imap[yi];
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    const u64 s0 = (u64)xb * 512 + 2 * threadIdx.x;
    const u64 Pq = cprime(primes, K - 1).q;
    if (!integer)
        hmacm_body<BTF, CG>(X1, X0, E, ch, B, l, K, logN, pr, Pq, I, kI, s0, bg * BTF);
    else if (int_mform)
        hmacm_body_int<BTI, CG>(X1, X0, E, ch, B, l, K, logN, pr, Pq, I, kI, s0, bg * BTI);
    else
        hmacm_body_u64<BTI, CG>(X1, X0, E, ch, B, l, K, logN, pr, Pq, I, kI, s0, bg * BTI);
}

// The zero corrections of the sibling-fused hoisted MAC (§4.6 of DESIGN.md), as their own pass over the children's
// accumulators (round 6; they were a branch after k_hmacm's digit loop, whose registers every thread carried):
//   ACC_c[b][k][I][o] -= sum_{J != I} C_J(o) key_c[J][k][I][o]  (mod q_I),
//   C_J(o) = sum over the zeros z of D_J[b] that child c negates (tt = z elt mod 2N >= N) of
//            (q_J mod q_I) psi_I^((2 bitrev(o) + 1)(tt - N)).
// The MAC is linear and every term is exact mod q_I, so subtracting them from the canonical MAC gives the same bits as
// adding them inside it.  Uniform residues almost never have a zero coefficient: a small fixed grid that exits at once
// when the node has none (zl[0] == 0), else strides over (child, b, I, o).
template <int CG, int NS>
__global__ void __launch_bounds__(256)
    k_hmacm_zfix(const HSlots<CG, NS> S, const int *__restrict__ zl, int B, int l, int K, int logN,
                 const DevPrime *__restrict__ primes, const int *__restrict__ Imap, int nI, const u64 *__restrict__ cji,
                 const u64 *__restrict__ psipow)
{
    if (zl[0] == 0) return;
    const u64 N = 1ull << logN, N2 = 2 * N;
    const int ns = NS == 1 ? 1 : S.ns;
    const u64 total = (u64)ns * CG * B * nI * N;
    for (u64 w = (u64)blockIdx.x * 256 + threadIdx.x; w < total; w += (u64)gridDim.x * 256) {
        const u64 o = w % N;
        u64 r = w / N;
        const int yi = (int)(r % nI);
        r /= nI;
        const int b = (int)(r % B), ci = (int)(r / B);
        const HChildren<CG> &ch = S.s[ci / CG];
        if (ci % CG >= ch.n) continue;
        const HChild &c = ch.c[ci % CG];
        const int I = Imap[yi], kI = I == l ? K - 1 : I;
        const DevPrime pr = primes[kI];
        const u64 *pp = psipow + ((u64)kI << (logN + 1));
        const u64 bo = 2 * (u64)bitrev((u32)o, logN) + 1;
        u64 corr0 = 0, corr1 = 0;
        for (int J = 0; J < l; ++J) {
            if (J == I) continue;
            const int *z = zl + 1 + (b * l + J) * (HEC_ZCAP + 1);
            const int nz = min(z[0], HEC_ZCAP);
            if (nz == 0) continue;
            const u64 cj = cji[J * K + kI];
            u64 cc = 0;
            for (int zi = 0; zi < nz; ++zi) {
                u64 tt = ((u64)z[1 + zi] * c.elt) & (N2 - 1);
                if (tt < N) continue;
                cc = addmod(cc, mulmod(cj, pp[(bo * (tt - N)) & (N2 - 1)], pr), pr.q);
            }
            if (cc == 0) continue;
            corr0 = addmod(corr0, mulmod(cc, c.key[(((u64)(J * 2 + 0) * K + kI) << logN) + o], pr), pr.q);
            corr1 = addmod(corr1, mulmod(cc, c.key[(((u64)(J * 2 + 1) * K + kI) << logN) + o], pr), pr.q);
        }
        if ((corr0 | corr1) == 0) continue;
        u64 *a0 = c.ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + o;
        u64 *a1 = c.ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + o;
        *a0 = submod(*a0, corr0, pr.q);
        *a1 = submod(*a1, corr1, pr.q);
    }
}

// nkids children in slots of CG (the last slot may hold fewer), at most NS slots
template <int BTF, int BTI, int CG, int NS = 1, int MINW = (BTF * CG <= 8 && BTI * CG <= 8) ? 3 : 2>
static void launch_hmacm(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids,
                         int nkids, int B, int l)
{
    HSlots<CG, NS> S{};
    S.ns = (nkids + CG - 1) / CG;
    if (nkids < 1 || S.ns > NS) throw std::invalid_argument("hoisted MAC: children per launch");
    for (int q = 0; q < nkids; ++q) {
        HChildren<CG> &ch = S.s[q / CG];
        ch.c[q % CG] = HChild{kids[q].elt, kids[q].einv, kids[q].key, kids[q].W, kids[q].ACC, kids[q].KW, kids[q].MK};
        ch.n = q % CG + 1;
    }
    const int nint = c.imap_nint[l], X = (int)(c.N / 512);
    const int gI = (X * nint + 7) / 8 * 8, gF = (X * (l + 1 - nint) + 7) / 8 * 8;
    const int wsplit = gI * ((B + BTI - 1) / BTI), total = wsplit + gF * ((B + BTF - 1) / BTF);
    k_hmacm<BTF, BTI, CG, MINW, NS><<<dim3((unsigned)(total * S.ns)), 256, 0, c.stream>>>(
        X1, X0, E, zl, S, B, l, (int)c.K, c.logN, c.primes, c.imap_at(l), l + 1, nint, c.cji, c.psipow, wsplit,
        c.hmac_int);
    HEC_HIP(hipGetLastError());
    k_hmacm_zfix<CG, NS><<<256, 256, 0, c.stream>>>(S, zl, B, l, (int)c.K, c.logN, c.primes, c.imap_at(l), l + 1, c.cji,
                                                    c.psipow);
    HEC_HIP(hipGetLastError());
}

int hoisted_group(const Ctx &c) { return c.hmac_cfg == 2 ? HMAC_MAX_CHILDREN : c.hmac_cfg ? 2 : 1; }

void hoisted_mac_group(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int nkids,
                       int B, int l)
{
    static_assert(HMAC_MAX_CHILDREN <= 2 * 3, "3 slots of 2 children");
    launch_hmacm<4, 2, 2, 3>(c, X1, X0, E, zl, kids, nkids, B, l);
}

void hoisted_mac_multi(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int nkids,
                       int B, int l)
{
    if (nkids < 1 || nkids > 2) throw std::invalid_argument("hoisted_mac_multi: group size");
    // <FP64 batch entries, integer batch entries, children> per thread (the 1x4, 2x2, 3x2, 4x4 ...
    // shapes measured slower)
    if (c.hmac_cfg) launch_hmacm<4, 2, 2>(c, X1, X0, E, zl, kids, nkids, B, l);
    else if (X0.p != nullptr) throw std::logic_error("hoisted_mac_multi: the one-child MAC does not fold IN");
    else hoisted_mac(c, X1, E, kids[0].W, zl, kids[0].key, kids[0].ACC, B, l, kids[0].elt);
}

void hoisted_mac_3(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int B, int l)
{
    launch_hmacm<4, 2, 3>(c, X1, X0, E, zl, kids, 3, B, l);
}

void fan_divide_round(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, u64 *Z, int B, int nk, int nl, int last_idx)
{
    if (nl > HEC_MAXL) throw std::invalid_argument("too many limbs");
    FanDivRound f{};
    f.Y = Y; f.ysb = ysb; f.ysk = ysk; f.Z = Z; f.nk = nk; f.nl = nl; f.logN = c.logN; f.last_idx = last_idx;
    f.last = c.q[last_idx]; f.half = f.last >> 1; f.primes = c.primes;
    for (int i = 0; i < nl; ++i) {
        f.fix[i] = c.q[i] - (f.half % c.q[i]);
        f.c30[i] = c.q[i] < (1ull << 42) && c.q[i] > (1ull << 32) ? (double)((1ull << 30) % c.q[i]) : 0.0;
        if (f.last < 2 * c.q[i] && i < 32) f.sub1 |= 1u << i;
    }
    fan_dispatch(c, B * nk, f);
}

// ====================================================================== fused mod-up B + MAC ==
// Key-switch steps (2b)+(3) in one kernel, so the NTT-form digits never go back to HBM.  A block owns
// NSEG contiguous chunks (NSEG * P coefficients) of one target prime I for one batch entry b and
// loops over the digits J:
//   * the pass-A output E[b][I][J] of digit J (J == I: the NTT-form target T[b][I]) is staged into
//     LDS from registers that were loaded one iteration earlier (software prefetch), and the key
//     words key[J][k][I] of the thread's output coefficients are issued before the rounds;
//   * the pass-B stages run in 8-element rounds (3 + 3 + 1 stages for P = 128); the last round
//     leaves each thread with 8 consecutive NTT outputs in registers;
//   * those are multiplied by the key words and accumulated: FP primes (< 2^42) as exact FP64
//     products (|acc| <= 0.53 q l, canonicalised once), 60-bit primes in 128-bit accumulators
//     (SEAL's lazy MAC), one Barrett reduction at the end.  (Barrett-reduced 64-bit accumulators
//     would bring the kernel to 3 waves/SIMD but measured 15 % slower: the integer blocks set the tail.)
// Grid (R / NSEG, l + 1, B): blocks of one (chunk block, I) for different b are R/NSEG * (l+1) apart,
// a multiple of 8 for logN >= 14, so they run on one XCD and share its L2 copy of the key chunk.
// The integer target primes come first in Imap: their blocks are the slowest, so they start first.
// k_bmac chunk rows at P = 2^7 / 2^8 (the cfg3 / cfg5 sizes): an XOR swizzle instead of padding.  Element x of
// a chunk lives at word x ^ f(x), f linear over GF(2) in the four bits from SH up and touching bits 1..4 only, so
// an element pair (2w, 2w + 1) stays one 16-B aligned pair and swz(xb | y) = swz(xb) ^ swz(y) for disjoint bits.
// The masks M[j] (for bit SH + j) come from the bank model (tools/lds_banks.py, bmac_swizzle): at P = 128 every
// round's ds_read_b64 / ds_write_b64, the 16-B staging stores and the 16-B final-round reads are conflict-free
// (the padded layout: 4-way reads in the second round, 2-way elsewhere); at P = 256 one round's reads are 2-way.
template <int LOGP>
struct BSwz {
    static constexpr bool on = false;
    static constexpr int SH = 0;
    static constexpr int M[4] = {0, 0, 0, 0};
};
template <>
struct BSwz<7> {
    static constexpr bool on = true;
    static constexpr int SH = 3;
    static constexpr int M[4] = {6, 2, 10, 20};
};
template <>
struct BSwz<8> {
    static constexpr bool on = true;
    static constexpr int SH = 4;
    static constexpr int M[4] = {8, 4, 26, 0};
};
template <int LOGP>
__host__ __device__ constexpr int bswz_c(int x)  // compile-time form
{
    int f = 0;
    for (int j = 0; j < 4; ++j)
        if ((x >> (BSwz<LOGP>::SH + j)) & 1) f ^= BSwz<LOGP>::M[j];
    return x ^ f;
}
template <int LOGP>
__host__ __device__ constexpr u64 bswz_lut()  // f(x) >> 1 for the 16 values of bits SH .. SH + 3, 4 bits each
{
    u64 t = 0;
    for (int i = 0; i < 16; ++i) t |= (u64)(bswz_c<LOGP>(i << BSwz<LOGP>::SH) ^ (i << BSwz<LOGP>::SH)) >> 1 << (4 * i);
    return t;
}
template <int LOGP>
__device__ __forceinline__ int bswz(int x)
{
    constexpr u64 L = bswz_lut<LOGP>();
    return x ^ (int)(((L >> (4 * ((x >> BSwz<LOGP>::SH) & 15))) & 15) << 1);
}
// k_bmac LDS segment stride (words): swizzled rows are P words; otherwise P data words + P/8 (one pad word per 16
// elements, and spare)
constexpr int bmac_ld(int logp)
{
    return (logp == 7 || logp == 8) ? (1 << logp) : (1 << logp) + (1 << logp) / 8;
}

// ntt_round_g on one swizzled chunk row: the group's base word swz(xb) once, its elements by XOR with constants;
// a final round that keeps its results in registers reads element pairs as 16-B words
template <int LOGP, int S0, int S1, int EPT, bool INV, bool FP, bool TO_REG, class TwG>
__device__ __forceinline__ void ntt_round_x(u64 *row, int ts, const TwG &twg, const DevPrime &pr, u64 *regs)
{
    constexpr int LE = EPT == 16 ? 4 : EPT == 8 ? 3 : EPT == 4 ? 2 : 1;
    constexpr int D = S1 - S0, G = 1 << (LE - D), NQ = 1 << D;
    static_assert(D >= 1 && D <= LE, "round covers 1..log2(EPT) stages");
    constexpr bool PAIRS = TO_REG && S1 == LOGP;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int g = ts * G + gi;
        const int lo = g & ((1 << (LOGP - S1)) - 1);
        const int hi = g >> (LOGP - S1);
        const int xb = bswz<LOGP>((hi << (LOGP - S0)) | lo);
        GroupTw<S0, D, FP, !FP && HasSplitTw<TwG>::value> gt;
        gt.load(hi, twg);
        u64 v[NQ];
        if constexpr (PAIRS) {
#pragma unroll
            for (int a = 0; a < NQ; a += 2) {
                const ulonglong2 w = *(const ulonglong2 *)(row + (xb ^ bswz_c<LOGP>(a)));
                v[a] = w.x;
                v[a + 1] = w.y;
            }
        } else {
#pragma unroll
            for (int a = 0; a < NQ; ++a) v[a] = row[xb ^ bswz_c<LOGP>(a << (LOGP - S1))];
        }
        gt.template run<INV>(v, pr);
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
            if constexpr (TO_REG) regs[gi * NQ + a] = v[a];
            else row[xb ^ bswz_c<LOGP>(a << (LOGP - S1))] = v[a];
        }
    }
}

// SPL (integer targets): the pass-B butterflies as split-input Shoup, their extra twiddle words staged in ltwa
template <int LOGP, int NSEG, int EPT, bool FP, bool SPL = false>
__device__ __forceinline__ void bmac_body(u64 *lds, u64 *ltw, u64 *ltwa, PolyArr T, const u64 *__restrict__ E,
                                          const u64 *__restrict__ key,
                                          u64 *__restrict__ ACC, const TwTables &tt, const DevPrime &pr, int I, int kI,
                                          int b, int xb, int logN, int l, int K, u32 elt)
{
    // segment-major lane layout: the P / EPT threads of one chunk are consecutive lanes.  At P = 128 and 256 (the
    // cfg3 / cfg5 sizes) a chunk row is exactly P words with the XOR swizzle of BSwz (element x at word x ^ f(x),
    // element pairs stay 16-B aligned); at P <= 64 a row is P + P/8 words with one pad word per 16 elements.  The
    // swizzled rows take 0.275 bank-conflict cycles per LDS instruction (tools/lds_banks.py, bmac_swizzle)
    constexpr int P = 1 << LOGP, THREADS = NSEG * P / EPT, LD = bmac_ld(LOGP), TWS = 2 * P + 2;
    static_assert(BSwz<LOGP>::on || LOGP <= 6, "P = 128 / 256 chunk rows are swizzled: the padded rounds stop at P = 64");
    static_assert(BSwz<LOGP>::on == (LD == P), "bmac_ld must match the row layout");
    const u64 N = 1ull << logN;
    const int seg0 = xb * NSEG;
    const u64 base = (u64)seg0 << LOGP;
    const ulonglong2 *tw = tt.b + ((u64)kI << logN);
    const double *twf = tt.fb + ((u64)kI << logN);
    const u64 *twa = SPL ? tt.sb + ((u64)kI << logN) : nullptr;
    const int ts = (int)threadIdx.x % (P / EPT), sg = (int)threadIdx.x / (P / EPT);
    auto addr = [sg](int x) { return sg * LD + x + (x >> 4); };
    const u64 R = 1ull << (logN - LOGP);
    // the pass-B twiddles of a chunk do not depend on the digit J: stage the block's (NSEG chunks x
    // (P - 1) entries) once into LDS, rows padded to TWS words (bank spread), lanes = consecutive chunks
    // so the re-laid table reads coalesce
    for (int t = threadIdx.x; t < NSEG * (P - 1); t += THREADS) {
        const int sl = t % NSEG, k = t / NSEG;
        const int st = 31 - __clz(k + 1), i = k + 1 - (1 << st);
        const u64 gi = R * ((1ull << st) - 1) + (u64)i * R + (u64)(seg0 + sl);
        if constexpr (FP) ltw[sl * TWS + k] = (u64)__double_as_longlong(twf[gi]);
        else {
            const ulonglong2 w = tw[gi];
            ltw[sl * TWS + 2 * k] = w.x;
            ltw[sl * TWS + 2 * k + 1] = w.y;
            if constexpr (SPL) ltwa[sl * P + k] = twa[gi];
        }
    }
    const LdsTw twg0{ltw + sg * TWS};
    const LdsTwS twgs{{ltw + sg * TWS}, ltwa + sg * P};
    const u64 g0 = ((u64)(seg0 + sg) << LOGP) + (u64)ts * EPT;  // first of this thread's outputs
    auto src = [&](int J) -> const u64 * {
        return J == I ? T.p + b * T.sb + (u64)J * N : E + (((u64)((b * (l + 1) + I) * l + J)) << logN);
    };

    double f0[FP ? EPT : 1], f1[FP ? EPT : 1];
    U128 i0[FP ? 1 : EPT], i1[FP ? 1 : EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        if constexpr (FP) f0[e] = f1[e] = 0.0;
        else i0[e] = i1[e] = U128{0, 0};
    }
    auto load_keys = [&](int J, u64 *k0, u64 *k1) {
        const u64 *kp0 = key + (((u64)(J * 2 + 0) * K + kI) << logN) + g0;
        const u64 *kp1 = key + (((u64)(J * 2 + 1) * K + kI) << logN) + g0;
#pragma unroll
        for (int e = 0; e < EPT; e += 2) {
            const ulonglong2 a = *(const ulonglong2 *)(kp0 + e), c = *(const ulonglong2 *)(kp1 + e);
            k0[e] = a.x; k0[e + 1] = a.y; k1[e] = c.x; k1[e + 1] = c.y;
        }
    };
    // digit tiles move as 16-B pairs: pair w = threadIdx.x + e THREADS holds block elements 2w, 2w + 1
    u64 nx[EPT];
    auto load_tile = [&](int J) {
        if (J == I && elt != 1) {  // the NTT-form target through the Galois permutation (pairs stay pairs)
            const u64 *sp = src(J);
#pragma unroll
            for (int e = 0; e < EPT / 2; ++e) {
                const u32 t = galois_src((u32)(base + 2 * (threadIdx.x + e * THREADS)), elt, logN);
                const ulonglong2 w = *(const ulonglong2 *)(sp + (t & ~1u));
                nx[2 * e] = (t & 1) ? w.y : w.x;
                nx[2 * e + 1] = (t & 1) ? w.x : w.y;
            }
            return;
        }
        const ulonglong2 *sp = (const ulonglong2 *)(src(J) + base);
#pragma unroll
        for (int e = 0; e < EPT / 2; ++e) {
            const ulonglong2 w = sp[threadIdx.x + e * THREADS];
            nx[2 * e] = w.x;
            nx[2 * e + 1] = w.y;
        }
    };
    constexpr bool SWZ = BSwz<LOGP>::on;
    u64 *const row = lds + sg * LD;
    load_tile(0);
    for (int J = 0; J < l; ++J) {
        const bool ntt = J != I;
#pragma unroll
        for (int e = 0; e < EPT; e += 2) {
            const int li = 2 * (threadIdx.x + (e / 2) * THREADS);
            u64 v0 = nx[e], v1 = nx[e + 1];
            if constexpr (FP) {
                if (!ntt) {  // canonical integer target
                    v0 = (u64)__double_as_longlong(u2d(v0));
                    v1 = (u64)__double_as_longlong(u2d(v1));
                }
            }
            if constexpr (SWZ) {
                *(ulonglong2 *)(lds + (li / P) * LD + bswz<LOGP>(li % P)) = ulonglong2{v0, v1};
            } else {
                lds[(li / P) * LD + (li % P) + ((li % P) >> 4)] = v0;
                lds[(li / P) * LD + (li % P) + 1 + (((li % P) + 1) >> 4)] = v1;
            }
        }
        // the key words of digit J before the prefetch of tile J + 1: vector loads complete in issue order (one
        // vmcnt), so the MAC's wait for its keys does not also wait for the next tile
        u64 k0[EPT], k1[EPT];
        load_keys(J, k0, k1);  // before the rounds: their latency hides behind the LDS work
        if (J + 1 < l) load_tile(J + 1);
        __syncthreads();
        u64 v[EPT];
        auto rounds = [&](const auto &twg) {
            static_assert(LOGP >= 5 && LOGP <= 8, "pass-B sizes 2^5 .. 2^8");
            static_assert(EPT == 4, "rounds of 2 stages");
            if constexpr (SWZ) {
                ntt_round_x<LOGP, 0, 2, EPT, false, FP, false>(row, ts, twg, pr, nullptr);
                __syncthreads();
                ntt_round_x<LOGP, 2, 4, EPT, false, FP, false>(row, ts, twg, pr, nullptr);
                __syncthreads();
                ntt_round_x<LOGP, 4, 6, EPT, false, FP, false>(row, ts, twg, pr, nullptr);
                __syncthreads();
                ntt_round_x<LOGP, 6, LOGP, EPT, false, FP, true>(row, ts, twg, pr, v);
            } else if constexpr (LOGP <= 6) {
                ntt_round_g<LOGP, 0, 2, EPT, false, FP, false>(lds, addr, ts, twg, pr, nullptr);
                __syncthreads();
                ntt_round_g<LOGP, 2, 4, EPT, false, FP, false>(lds, addr, ts, twg, pr, nullptr);
                __syncthreads();
                ntt_round_g<LOGP, 4, LOGP, EPT, false, FP, true>(lds, addr, ts, twg, pr, v);
            }
        };
        if (ntt) {
            if constexpr (!FP && SPL) rounds(twgs);
            else rounds(twg0);
        } else if constexpr (SWZ) {
            const int xb = bswz<LOGP>(ts * EPT);
#pragma unroll
            for (int e = 0; e < EPT; e += 2) {
                const ulonglong2 w = *(const ulonglong2 *)(row + (xb ^ bswz_c<LOGP>(e)));
                v[e] = w.x;
                v[e + 1] = w.y;
            }
        } else {
#pragma unroll
            for (int e = 0; e < EPT; ++e) v[e] = lds[addr(ts * EPT + e)];
        }
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            if constexpr (FP) {
                const double dv = __longlong_as_double((long long)v[e]);
                f0[e] += fp_mulmod(dv, u2d(k0[e]), pr.qd, pr.qinv);
                f1[e] += fp_mulmod(dv, u2d(k1[e]), pr.qd, pr.qinv);
            } else {
                mac128(i0[e], v[e], k0[e]);  // v < 4q: sum of l products < 2^126
                mac128(i1[e], v[e], k1[e]);
            }
        }
        __syncthreads();
    }
    u64 *o0 = ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + g0;
    u64 *o1 = ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + g0;
#pragma unroll
    for (int e = 0; e < EPT; e += 2) {
        if constexpr (FP) {
            *(ulonglong2 *)(o0 + e) = ulonglong2{fp_canon(f0[e], pr.qd, pr.qinv), fp_canon(f0[e + 1], pr.qd, pr.qinv)};
            *(ulonglong2 *)(o1 + e) = ulonglong2{fp_canon(f1[e], pr.qd, pr.qinv), fp_canon(f1[e + 1], pr.qd, pr.qinv)};
        } else {
            *(ulonglong2 *)(o0 + e) = ulonglong2{barrett128(i0[e].lo, i0[e].hi, pr.q, pr.r0, pr.r1),
                                                 barrett128(i0[e + 1].lo, i0[e + 1].hi, pr.q, pr.r0, pr.r1)};
            *(ulonglong2 *)(o1 + e) = ulonglong2{barrett128(i1[e].lo, i1[e].hi, pr.q, pr.r0, pr.r1),
                                                 barrett128(i1[e + 1].lo, i1[e + 1].hi, pr.q, pr.r0, pr.r1)};
        }
    }
}

// one launch: Imap lists every target prime, the first nint integer ones (per-block branch; blocks of both
// kinds overlap)
template <int LOGP, int NSEG, int EPT, bool SPL>
__global__ void __launch_bounds__(NSEG *(1 << LOGP) / EPT, 4)  // 4 waves per SIMD (<= 128 VGPRs), as without SPL
    k_bmac(PolyArr T, const u64 *__restrict__ E, const u64 *__restrict__ key, u64 *__restrict__ ACC, TwTables tt,
           const DevPrime *__restrict__ primes, const int *__restrict__ Imap, int nI, int logN, int l, int K,
           int nint, int gpad, u32 elt)
{
    __shared__ __attribute__((aligned(16))) u64 lds[NSEG * bmac_ld(LOGP)];  // 16-B pair accesses
    __shared__ __attribute__((aligned(16))) u64 ltw[NSEG * (2 * (1 << LOGP) + 2)];  // rows of 2P + 2 words: 16-B pairs
    __shared__ u64 ltwa[SPL ? NSEG * (1 << LOGP) : 1];  // SPL: the integer twiddles' split-input words
    // 1-D grid, XCD-aware: workgroup w runs on XCD w % 8.  The B blocks of one (chunk block, I) group
    // read the same key chunk, so they get ids G8*8*B + b*8 + (G % 8): one XCD, dispatched together,
    // and the key chunk is fetched into that XCD's L2 once instead of once per b.
    const int w = blockIdx.x, B = gridDim.x / gpad;
    const int g8 = w & 7, rest = w >> 3, b = rest % B, G = (rest / B) * 8 + g8;
    const int X = (1 << (logN - LOGP)) / NSEG;
    if (G >= X * nI) return;
    const int yi = G / X, xb = G % X;
    const int I = Imap[yi];
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    if (yi < nint)
        bmac_body<LOGP, NSEG, EPT, false, SPL>(lds, ltw, ltwa, T, E, key, ACC, tt, pr, I, kI, b, xb, logN, l, K, elt);
    else
        bmac_body<LOGP, NSEG, EPT, true>(lds, ltw, ltwa, T, E, key, ACC, tt, pr, I, kI, b, xb, logN, l, K, elt);
}

// k_bmac: EPT = 4 elements per thread (rounds of 2 stages, 118 VGPRs, 4 waves/SIMD); 8 per thread (3-stage rounds,
// 200 VGPRs, 2 waves/SIMD) measured 1,062 vs 951 ms per step at cfg3 (round 3, gpurun_out/r03s)
template <int LOGR, int LOGC, int NA, int NB2, int EPT = 4>
static void run_modup_fused(Ctx &c, const u64 *D, u64 *E, PolyArr T, const u64 *key, u64 *ACC, int B, int l,
                            int part, u32 elt)
{
    constexpr int R = 1 << LOGR, C = 1 << LOGC;
    const TwTables fwd{c.tw, c.twb, c.twf, c.twbf, c.tws, c.twbs};
    // (2a) pass A of every mod-up NTT (B * l * l jobs), output E[b][I][J] (lazy, pass-A domain)
    const int nint = c.imap_nint[l];
    const int *dm = c.imap_at(l);
    if (part & 1) {
        ModUpMap m{l, c.logN, (int)c.K - 1};
        k_ntt<LOGR, NA, false, true, false><<<dim3(C / NA, B * l * l), NA * R / 16, 0, c.stream>>>(
            ModUpIO_A{m, D, E, c.primes}, fwd, c.primes, c.logN);
    }
    if (!(part & 2)) {
        HEC_HIP(hipGetLastError());
        return;
    }
    // (2b)+(3) fused; integer target primes first (slowest blocks start first)
    constexpr int TB = NB2 * C / EPT;
    constexpr int X = R / NB2;
    const int gpad = (X * (l + 1) + 7) / 8 * 8;
    if (c.bmac_split)
        k_bmac<LOGC, NB2, EPT, true><<<dim3(gpad * B), TB, 0, c.stream>>>(T, E, key, ACC, fwd, c.primes, dm, l + 1,
                                                                          c.logN, l, (int)c.K, nint, gpad, elt);
    else
        k_bmac<LOGC, NB2, EPT, false><<<dim3(gpad * B), TB, 0, c.stream>>>(T, E, key, ACC, fwd, c.primes, dm, l + 1,
                                                                           c.logN, l, (int)c.K, nint, gpad, elt);
    HEC_HIP(hipGetLastError());
}

void ks_modup_mac(Ctx &c, const u64 *D, u64 *E, PolyArr T, const u64 *key, u64 *ACC, int B, int l, int part,
                  u32 elt)
{
    // <LOGR, LOGC, pass-A columns per block, fused pass-B chunks per block>: k_bmac blocks of 64-128
    // threads (4 chunks at N = 2^15: 110 us per B = 8 call vs 128 / 166 us at 16 / 32 chunks) keep the
    // serial digit loop of the slow integer-prime blocks short
    switch (c.logN) {
    case 10: run_modup_fused<5, 5, 32, 16>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 11: run_modup_fused<6, 5, 32, 16>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 12: run_modup_fused<6, 6, 64, 8>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 13: run_modup_fused<7, 6, 32, 8>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 14: run_modup_fused<7, 7, 32, 4>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 15: run_modup_fused<8, 7, 16, 4>(c, D, E, T, key, ACC, B, l, part, elt); break;
    case 16: run_modup_fused<8, 8, 16, 4>(c, D, E, T, key, ACC, B, l, part, elt); break;
    default: throw std::invalid_argument("poly_modulus_degree must be 2^10 .. 2^16");
    }
}

// =============================================================================== key MAC ===
// ACC[b][k][I] = sum_J E[b][I][J] * key[J][k][I]  (E[b][I][I] = T[b][I], the NTT-form target),
// 128-bit lazy accumulation then one Barrett reduction (SEAL switch_key_inplace step 3).
// A thread owns one coefficient for BT batch entries, so each key word is read once per BT targets.
template <int BT>
__device__ __forceinline__ void ks_mac_int(PolyArr T, const u64 *__restrict__ E, const u64 *__restrict__ key,
                                           u64 *__restrict__ ACC, int B, int l, int K, int logN,
                                           const DevPrime *__restrict__ primes, int I, u32 elt)
{
    const u64 N = 1ull << logN;
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    const u64 tg = elt == 1 ? g : galois_src((u32)g, elt, logN);
    const int b0 = blockIdx.z * BT;
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    U128 a0[BT], a1[BT];
#pragma unroll
    for (int t = 0; t < BT; ++t) a0[t] = a1[t] = U128{0, 0};
    for (int J = 0; J < l; ++J) {
        const u64 k0 = key[((u64)(J * 2 + 0) * K + kI) * N + g];
        const u64 k1 = key[((u64)(J * 2 + 1) * K + kI) * N + g];
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b < B) {
                const u64 e = (I == J) ? T.p[b * T.sb + (u64)J * N + tg]
                                       : E[((u64)((b * (l + 1) + I) * l + J) << logN) + g];
                mac128(a0[t], e, k0);
                mac128(a1[t], e, k1);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        const int b = b0 + t;
        if (b < B) {
            ACC[((u64)((b * 2 + 0) * (l + 1) + I) << logN) + g] = barrett128(a0[t].lo, a0[t].hi, pr.q, pr.r0, pr.r1);
            ACC[((u64)((b * 2 + 1) * (l + 1) + I) << logN) + g] = barrett128(a1[t].lo, a1[t].hi, pr.q, pr.r0, pr.r1);
        }
    }
}

// FP64 variant for target primes < 2^42: each thread owns two adjacent coefficients (16-B loads),
// products by fp_mulmod (exact, |r| <= 0.53 q), sums kept as integer-valued doubles (|acc| <= 0.53 q l).
template <int BT>
__device__ __forceinline__ void ks_mac_fp(PolyArr T, const u64 *__restrict__ E, const u64 *__restrict__ key,
                                          u64 *__restrict__ ACC, int B, int l, int K, int logN,
                                          const DevPrime *__restrict__ primes, int I, u32 elt)
{
    const u64 N = 1ull << logN;
    if ((u64)blockIdx.x * 512 >= N) return;  // FP blocks own two coefficients per thread
    const u64 g = 2 * ((u64)blockIdx.x * 256 + threadIdx.x);
    const int b0 = blockIdx.z * BT;
    const int kI = I == l ? K - 1 : I;
    const DevPrime pr = primes[kI];
    double a0[BT][2], a1[BT][2];
#pragma unroll
    for (int t = 0; t < BT; ++t) a0[t][0] = a0[t][1] = a1[t][0] = a1[t][1] = 0.0;
    for (int J = 0; J < l; ++J) {
        const ulonglong2 k0 = *(const ulonglong2 *)(key + ((u64)(J * 2 + 0) * K + kI) * N + g);
        const ulonglong2 k1 = *(const ulonglong2 *)(key + ((u64)(J * 2 + 1) * K + kI) * N + g);
        const double k00 = u2d(k0.x), k01 = u2d(k0.y), k10 = u2d(k1.x), k11 = u2d(k1.y);
#pragma unroll
        for (int t = 0; t < BT; ++t) {
            const int b = b0 + t;
            if (b < B) {
                ulonglong2 e;
                if (I == J) {
                    const u64 *tp = T.p + b * T.sb + (u64)J * N;
                    e = elt == 1 ? *(const ulonglong2 *)(tp + g)
                                 : ulonglong2{tp[galois_src((u32)g, elt, logN)], tp[galois_src((u32)g + 1, elt, logN)]};
                } else {
                    e = *(const ulonglong2 *)(E + (((u64)((b * (l + 1) + I) * l + J)) << logN) + g);
                }
                const double e0 = u2d(e.x), e1 = u2d(e.y);
                a0[t][0] += fp_mulmod(e0, k00, pr.qd, pr.qinv);
                a0[t][1] += fp_mulmod(e1, k01, pr.qd, pr.qinv);
                a1[t][0] += fp_mulmod(e0, k10, pr.qd, pr.qinv);
                a1[t][1] += fp_mulmod(e1, k11, pr.qd, pr.qinv);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < BT; ++t) {
        const int b = b0 + t;
        if (b < B) {
            *(ulonglong2 *)(ACC + (((u64)((b * 2 + 0) * (l + 1) + I)) << logN) + g) =
                ulonglong2{fp_canon(a0[t][0], pr.qd, pr.qinv), fp_canon(a0[t][1], pr.qd, pr.qinv)};
            *(ulonglong2 *)(ACC + (((u64)((b * 2 + 1) * (l + 1) + I)) << logN) + g) =
                ulonglong2{fp_canon(a1[t][0], pr.qd, pr.qinv), fp_canon(a1[t][1], pr.qd, pr.qinv)};
        }
    }
}

// one launch: blockIdx.y < nint -> integer target primes, the rest FP64 primes (run concurrently)
template <int BT>
__global__ void __launch_bounds__(256)
    k_ks_mac(PolyArr T, const u64 *__restrict__ E, const u64 *__restrict__ key, u64 *__restrict__ ACC, int B, int l,
             int K, int logN, const DevPrime *__restrict__ primes, const int *__restrict__ Imap, int nint, u32 elt)
{
    const int I = Imap[blockIdx.y];
    if ((int)blockIdx.y < nint) ks_mac_int<BT>(T, E, key, ACC, B, l, K, logN, primes, I, elt);
    else ks_mac_fp<BT>(T, E, key, ACC, B, l, K, logN, primes, I, elt);
}

void ks_mac(Ctx &c, PolyArr T, const u64 *E, const u64 *key, u64 *ACC, int B, int l, u32 elt)
{
    constexpr int BT = 8;
    const int nint = c.imap_nint[l];
    const unsigned bz = (B + BT - 1) / BT;
    k_ks_mac<BT><<<dim3((unsigned)(c.N / 256), l + 1, bz), 256, 0, c.stream>>>(T, E, key, ACC, B, l, (int)c.K,
                                                                              c.logN, c.primes, c.imap_at(l), nint, elt);
    HEC_HIP(hipGetLastError());
}

// =============================================================================== Galois ====
// SEAL GaloisTool::apply_galois_ntt: out[t] = in[tbl[t]],
//   tbl[t] = bitrev(((elt * (2 bitrev(t) + 1)) >> 1) & (N - 1))
__global__ void __launch_bounds__(256)
    k_galois(PolyArr in, PolyArr out, int nk, int nl, u32 elt, int logN, u64 total)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const u64 mask = (1ull << logN) - 1;
    const u32 t = (u32)(idx & mask);
    u64 rest = idx >> logN;
    const int i = (int)(rest % nl);
    rest /= nl;
    const int k = (int)(rest % nk);
    const u64 b = rest / nk;
    const u64 rev = 2ull * bitrev(t, logN) + 1;
    const u32 src = bitrev((u32)(((u64)elt * rev >> 1) & mask), logN);
    const u64 li = (u64)i << logN;
    out.p[b * out.sb + k * out.sk + li + t] = in.p[b * in.sb + k * in.sk + li + src];
}

void galois_permute(Ctx &c, PolyArr in, PolyArr out, int B, int nk, int nl, u32 elt)
{
    const u64 total = (u64)B * nk * nl * c.N;
    k_galois<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(in, out, nk, nl, elt, c.logN, total);
    HEC_HIP(hipGetLastError());
}

// =============================================================================== tensor ====
// ACC[b] (size 3) (=|+=) R[b] (x) A  (SEAL ckks_multiply 2x2 -> 3, then add_inplace).  A is read once
// per coefficient for the whole batch.
__global__ void __launch_bounds__(256)
    k_tensor_acc(PolyArr R, const u64 *__restrict__ A, u64 a_sk, PolyArr ACC, int B, int logN, u64 total,
                 int assign, const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int i = (int)(idx >> logN);
    const DevPrime pr = primes[i];
    const u64 a0 = A[idx], a1 = A[a_sk + idx];
    for (int b = 0; b < B; ++b) {
        const u64 *r = R.p + b * R.sb;
        const u64 r0 = r[idx], r1 = r[R.sk + idx];
        const u64 d0 = mulmod(r0, a0, pr), d2 = mulmod(r1, a1, pr);
        U128 t{r0 * a1, mulhi64(r0, a1)};
        mac128(t, r1, a0);
        const u64 d1 = barrett128(t.lo, t.hi, pr.q, pr.r0, pr.r1);
        u64 *o = ACC.p + b * ACC.sb;
        if (assign) {
            o[idx] = d0; o[ACC.sk + idx] = d1; o[2 * ACC.sk + idx] = d2;
        } else {
            o[idx] = addmod(o[idx], d0, pr.q);
            o[ACC.sk + idx] = addmod(o[ACC.sk + idx], d1, pr.q);
            o[2 * ACC.sk + idx] = addmod(o[2 * ACC.sk + idx], d2, pr.q);
        }
    }
}

void tensor_acc(Ctx &c, PolyArr R, const u64 *A, u64 a_sk, PolyArr ACC, int B, int l, bool assign)
{
    const u64 total = (u64)l * c.N;
    k_tensor_acc<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(R, A, a_sk, ACC, B, c.logN, total,
                                                                         assign ? 1 : 0, c.primes);
    HEC_HIP(hipGetLastError());
}

// Deferred tensor products: ACC[b] (=|+=) sum_t R_t[b] (x) A_t for T rotated inputs at once, so the
// size-3 accumulator is read and written once per T diagonals instead of once per diagonal.  Every
// product is reduced (SEAL ckks_multiply) and the sums are taken mod q, so the bits equal T
// successive k_tensor_acc calls.  FP64 primes: exact fp_mulmod products (|.| <= 0.53 q) summed as
// integer-valued doubles (|sum| <= 1.6 q T < 2^53), canonicalised once.
// PT: the A_t are plaintexts (ct x pt: d0 = r0 p, d1 = r1 p, multiply_plain), ACC has 2 polys.
// The deferred tensor products with the batch split over the grid (k_tensor_multi2; round 2's one-thread-per-coefficient
// k_tensor_multi was deleted in round 3): a thread owns one coefficient of BG batch entries
// (blockIdx.y picks the group), loads each diagonal word once for its BG entries and keeps BG sets of
// accumulators, so a wave has BG rotated-input loads in flight per diagonal and the diagonals are re-read
// B / BG times (from L2) instead of B times.  Products are reduced as SEAL reduces them; sums are exact
// (FP64: |sum| < 12 x 0.53 q; 60-bit primes: 128-bit sums of < 2^120 products) and canonicalised once.
// (Blocks of 4 waves on 4 batch groups sharing the diagonal words through L1 measured slower: 556 vs 522 ms per
// step, round 4.)
// xs > 0: a 1-D grid in clusters of xs batch groups per coefficient block, each cluster's blocks consecutive on one
// XCD (ids w, w + 8, ...), so a coefficient block's diagonal words come from HBM once per cluster and from that XCD's
// L2 for the rest, while every batch group still streams its rotated inputs over consecutive coefficient blocks
template <bool PT, int BG>
__global__ void __launch_bounds__(256)
    k_tensor_multi2(TensorBatch tb, u64 r_sb, u64 r_sk, u64 a_sk, PolyArr ACC, int B, int logN, u64 total, int assign,
                    const DevPrime *__restrict__ primes, int xs, int ncb)
{
    int cb = blockIdx.x, bgi = blockIdx.y;
    if (xs > 0) {
        const int t = (int)blockIdx.x >> 3, s = t % xs, c = (t / xs) * 8 + ((int)blockIdx.x & 7);
        cb = c % ncb;
        bgi = (c / ncb) * xs + s;
        if (bgi * BG >= B) return;
    }
    const u64 idx = (u64)cb * 256 + threadIdx.x;
    if (idx >= total) return;
    const int b0 = bgi * BG;
    const int nb = min(BG, B - b0);
    const DevPrime pr = primes[idx >> logN];
    u64 d0[BG], d1[BG], d2[BG];
    if (pr.fp) {
        double s0[BG], s1[BG], s2[BG];
#pragma unroll
        for (int g = 0; g < BG; ++g) s0[g] = s1[g] = s2[g] = 0;
        for (int t = 0; t < tb.T; ++t) {
            const double a0 = u2d(tb.a[t][idx]);
            const double a1 = PT ? 0.0 : u2d(tb.a[t][a_sk + idx]);
            const u64 *r = tb.r[t] + (u64)b0 * r_sb;
#pragma unroll
            for (int g = 0; g < BG; ++g) {
                if (g >= nb) break;
                const double r0 = u2d(r[g * r_sb + idx]), r1 = u2d(r[g * r_sb + r_sk + idx]);
                s0[g] += fp_mulmod(r0, a0, pr.qd, pr.qinv);
                if constexpr (PT) {
                    s1[g] += fp_mulmod(r1, a0, pr.qd, pr.qinv);
                } else {
                    s1[g] += fp_mulmod(r0, a1, pr.qd, pr.qinv) + fp_mulmod(r1, a0, pr.qd, pr.qinv);
                    s2[g] += fp_mulmod(r1, a1, pr.qd, pr.qinv);
                }
            }
        }
#pragma unroll
        for (int g = 0; g < BG; ++g) {
            d0[g] = fp_canon(s0[g], pr.qd, pr.qinv);
            d1[g] = fp_canon(s1[g], pr.qd, pr.qinv);
            d2[g] = PT ? 0 : fp_canon(s2[g], pr.qd, pr.qinv);
        }
    } else {
#pragma unroll
        for (int g = 0; g < BG; ++g) d0[g] = d1[g] = d2[g] = 0;
        for (int t = 0; t < tb.T; ++t) {
            const u64 a0 = tb.a[t][idx];
            const u64 a1 = PT ? 0 : tb.a[t][a_sk + idx];
            const u64 *r = tb.r[t] + (u64)b0 * r_sb;
#pragma unroll
            for (int g = 0; g < BG; ++g) {
                if (g >= nb) break;
                const u64 r0 = r[g * r_sb + idx], r1 = r[g * r_sb + r_sk + idx];
                d0[g] = addmod(d0[g], mulmod(r0, a0, pr), pr.q);
                if constexpr (PT) {
                    d1[g] = addmod(d1[g], mulmod(r1, a0, pr), pr.q);
                } else {
                    U128 m{r0 * a1, mulhi64(r0, a1)};
                    mac128(m, r1, a0);
                    d1[g] = addmod(d1[g], barrett128(m.lo, m.hi, pr.q, pr.r0, pr.r1), pr.q);
                    d2[g] = addmod(d2[g], mulmod(r1, a1, pr), pr.q);
                }
            }
        }
    }
#pragma unroll
    for (int g = 0; g < BG; ++g) {
        if (g >= nb) break;
        u64 *o = ACC.p + (u64)(b0 + g) * ACC.sb;
        if (assign) {
            o[idx] = d0[g]; o[ACC.sk + idx] = d1[g];
            if constexpr (!PT) o[2 * ACC.sk + idx] = d2[g];
        } else {
            o[idx] = addmod(o[idx], d0[g], pr.q);
            o[ACC.sk + idx] = addmod(o[ACC.sk + idx], d1[g], pr.q);
            if constexpr (!PT) o[2 * ACC.sk + idx] = addmod(o[2 * ACC.sk + idx], d2[g], pr.q);
        }
    }
}

void tensor_multi(Ctx &c, const TensorBatch &tb, u64 r_sb, u64 r_sk, u64 a_sk, PolyArr ACC, int B, int l, bool assign,
                  bool plain)
{
    const u64 total = (u64)l * c.N;
    constexpr int BG = 2;  // batch entries per thread (round 3, r03t: 533 vs 578 ms per step for 4, 577 for 8)
    const int ncb = (int)((total + 255) / 256), nbg = (B + BG - 1) / BG;
    const int xs = std::min(std::max(0, c.tensor_xcd), nbg);
    dim3 g2((unsigned)ncb, (unsigned)nbg);
    if (xs > 0) {  // clusters of xs batch groups: ncb * ceil(nbg / xs) clusters, padded to whole XCD rounds
        const long clusters = (long)ncb * ((nbg + xs - 1) / xs);
        g2 = dim3((unsigned)((clusters + 7) / 8 * 8 * xs), 1);
    }
    if (plain)
        k_tensor_multi2<true, BG><<<g2, 256, 0, c.stream>>>(tb, r_sb, r_sk, a_sk, ACC, B, c.logN, total, assign ? 1 : 0,
                                                           c.primes, xs, ncb);
    else
        k_tensor_multi2<false, BG><<<g2, 256, 0, c.stream>>>(tb, r_sb, r_sk, a_sk, ACC, B, c.logN, total,
                                                            assign ? 1 : 0, c.primes, xs, ncb);
    HEC_HIP(hipGetLastError());
}

// ACC (size 3) = sum_b R[b] (x) A[b]  (col x col^T form: one output, the batch is the j-sum)
__global__ void __launch_bounds__(256)
    k_tensor_sum(PolyArr R, PolyArr A, u64 *__restrict__ ACC, u64 acc_sk, int B, int logN, u64 total,
                 const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int i = (int)(idx >> logN);
    const DevPrime pr = primes[i];
    U128 s0{0, 0}, s1{0, 0}, s2{0, 0};
    for (int b = 0; b < B; ++b) {  // reduce each product (SEAL reduces per multiply), add canonically
        const u64 *r = R.p + b * R.sb, *a = A.p + b * A.sb;
        const u64 r0 = r[idx], r1 = r[R.sk + idx], a0 = a[idx], a1 = a[A.sk + idx];
        U128 t{r0 * a1, mulhi64(r0, a1)};
        mac128(t, r1, a0);
        s0.lo = addmod(s0.lo, mulmod(r0, a0, pr), pr.q);
        s1.lo = addmod(s1.lo, barrett128(t.lo, t.hi, pr.q, pr.r0, pr.r1), pr.q);
        s2.lo = addmod(s2.lo, mulmod(r1, a1, pr), pr.q);
    }
    ACC[idx] = s0.lo;
    ACC[acc_sk + idx] = s1.lo;
    ACC[2 * acc_sk + idx] = s2.lo;
}

void tensor_sum(Ctx &c, PolyArr R, PolyArr A, u64 *ACC, u64 acc_sk, int B, int l)
{
    const u64 total = (u64)l * c.N;
    k_tensor_sum<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(R, A, ACC, acc_sk, B, c.logN, total, c.primes);
    HEC_HIP(hipGetLastError());
}

// =============================================================================== misc ======
__global__ void __launch_bounds__(256) k_ew_add(PolyArr a, PolyArr b, PolyArr out, int nk, int nl, int logN,
                                                 u64 total, int mode, const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const u64 N = 1ull << logN, t = idx & (N - 1);
    u64 rest = idx >> logN;
    const int i = (int)(rest % nl);
    rest /= nl;
    const int k = (int)(rest % nk);
    const u64 bb = rest / nk;
    const u64 q = primes[i].q, off = ((u64)i << logN) + t;
    const u64 x = a.p[bb * a.sb + k * a.sk + off];
    const u64 y = b.p ? b.p[bb * b.sb + k * b.sk + off] : 0;
    u64 r;
    if (mode == 0) r = addmod(x, y, q);
    else if (mode == 1) r = submod(x, y, q);
    else r = y ? q - y : 0;  // mode 2: out = -b (sub with a missing left operand)
    out.p[bb * out.sb + k * out.sk + off] = r;
}

void ew_add(Ctx &c, PolyArr a, PolyArr b, PolyArr out, int B, int nk, int nl, int mode)
{
    const u64 total = (u64)B * nk * nl * c.N;
    if (!total) return;
    k_ew_add<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(a, b, out, nk, nl, c.logN, total, mode,
                                                                     c.primes);
    HEC_HIP(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_negate(u64 *p, int nl, int logN, u64 total, const DevPrime *primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int i = (int)((idx >> logN) % nl);
    const u64 v = p[idx];
    p[idx] = v ? primes[i].q - v : 0;
}

void ew_negate(Ctx &c, PolyArr a, int B, int nk, int nl)
{
    // contiguous [k][i][N] per entry (sb == nk * sk)
    for (int b = 0; b < B; ++b) {
        const u64 total = (u64)nk * nl * c.N;
        k_negate<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(a.p + b * a.sb, nl, c.logN, total,
                                                                        c.primes);
    }
    HEC_HIP(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_mul_plain(u64 *a, const u64 *__restrict__ pt, int nl, int logN,
                                                    u64 total, const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const u64 per = (u64)nl << logN;
    const u64 off = idx % per;
    const int i = (int)(off >> logN);
    a[idx] = mulmod(a[idx], pt[off], primes[i]);
}

void ew_mul_plain(Ctx &c, PolyArr a, const u64 *pt, int nk, int nl)
{
    const u64 total = (u64)nk * nl * c.N;
    k_mul_plain<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(a.p, pt, nl, c.logN, total, c.primes);
    HEC_HIP(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_dyadic(const u64 *__restrict__ a, const u64 *__restrict__ b, u64 *out,
                                                 int limb0, int nl, int logN, u64 total,
                                                 const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int i = (int)((idx >> logN) % nl);
    out[idx] = mulmod(a[idx], b[idx], primes[limb0 + i]);
}

void ew_dyadic(Ctx &c, const u64 *a, const u64 *b, u64 *out, int limb0, int nl, int npolys)
{
    const u64 total = (u64)npolys * nl * c.N;
    k_dyadic<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(a, b, out, limb0, nl, c.logN, total, c.primes);
    HEC_HIP(hipGetLastError());
}

// general ciphertext product (sizes sa x sb -> sa + sb - 1), out must not alias the inputs
__global__ void __launch_bounds__(256) k_ct_mul(const u64 *__restrict__ a, int sa, const u64 *__restrict__ b,
                                                 int sb, u64 *__restrict__ out, int nl, int logN, u64 total,
                                                 const DevPrime *__restrict__ primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;  // (i, t) within one poly
    if (idx >= total) return;
    const int i = (int)(idx >> logN);
    const DevPrime pr = primes[i];
    const u64 ps = total;  // words per poly
    for (int k = 0; k < sa + sb - 1; ++k) {
        U128 acc{0, 0};
        const int x0 = k - (sb - 1) > 0 ? k - (sb - 1) : 0, x1 = k < sa - 1 ? k : sa - 1;
        for (int x = x0; x <= x1; ++x) mac128(acc, a[x * ps + idx], b[(k - x) * ps + idx]);
        out[k * ps + idx] = barrett128(acc.lo, acc.hi, pr.q, pr.r0, pr.r1);
    }
}

void ct_multiply(Ctx &c, const u64 *a, int sa, const u64 *b, int sb, u64 *out, int nl)
{
    const u64 total = (u64)nl * c.N;
    k_ct_mul<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(a, sa, b, sb, out, nl, c.logN, total, c.primes);
    HEC_HIP(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_reduce(u64 *p, int nl, int logN, u64 total, const DevPrime *primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const DevPrime pr = primes[(idx >> logN) % nl];
    p[idx] = barrett64(p[idx], pr.q, pr.r1);
}

void ew_reduce(Ctx &c, u64 *p, int npoly, int nl)
{
    const u64 total = (u64)npoly * nl * c.N;
    k_reduce<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(p, nl, c.logN, total, c.primes);
    HEC_HIP(hipGetLastError());
}

__device__ __forceinline__ u64 mix64(u64 z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_fill(u64 *p, int nl, int logN, u64 total, u64 seed, int prime0,
                                               const DevPrime *primes)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const DevPrime pr = primes[prime0 + (int)((idx >> logN) % nl)];
    p[idx] = barrett64(mix64(seed + 0x9E3779B97F4A7C15ull * (idx + 1)), pr.q, pr.r1);
}

void fill_uniform(Ctx &c, u64 *p, int npoly, int nl, int limb_prime0, int, u64 seed)
{
    const u64 total = (u64)npoly * nl * c.N;
    k_fill<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(p, nl, c.logN, total, seed, limb_prime0,
                                                                   c.primes);
    HEC_HIP(hipGetLastError());
}

// every word of limb i = v.w[i] (the NTT form of a constant polynomial: CKKSEncoder::encode of a scalar)
struct LimbWords {
    u64 w[HEC_MAXL + 1];
};
__global__ void __launch_bounds__(256) k_fill_limbs(u64 *p, int logN, u64 total, LimbWords v)
{
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    p[idx] = v.w[idx >> logN];
}

void fill_limbs(Ctx &c, u64 *p, int nl, const u64 *words)
{
    if (nl > HEC_MAXL + 1) throw std::invalid_argument("too many limbs");
    LimbWords v{};
    for (int i = 0; i < nl; ++i) v.w[i] = words[i];
    const u64 total = (u64)nl * c.N;
    k_fill_limbs<<<(unsigned)((total + 255) / 256), 256, 0, c.stream>>>(p, c.logN, total, v);
    HEC_HIP(hipGetLastError());
}

}  // namespace hec
