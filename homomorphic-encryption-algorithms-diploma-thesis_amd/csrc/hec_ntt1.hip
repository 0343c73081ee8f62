// Single-pass negacyclic NTT for N = 2^15: one 1024-thread workgroup owns a whole limb (32 residues
// per thread in registers), so a limb makes one HBM round trip instead of the two-pass kernel's two
// (k_ntt pass A + pass B, hec_kernels.hip).  SEAL's convention as everywhere in the engine: forward
// Cooley-Tukey with bit-reversed twiddles psi^bitrev(k), stage s pairs (e, e + 2^(14 - s)) with
// twiddle index 2^s + (e >> (15 - s)), bit-reversed output.
//
// Element e = (h, m, l) = h 1024 + m 32 + l (5 bits each); thread t = a 32 + b (a = t >> 5, b = t & 31).
//   round 1, stages 0..4 (bits of h):  thread (m, l) = (a, b) holds h = 0..31; twiddles uniform;
//   round 2, stages 5..9 (bits of m):  thread (h, l) = (a, b) holds m = 0..31;
//   round 3, stages 10..14 (bits of l): thread (h, m) = (a, b) holds l = 0..31 (32 consecutive outputs).
// The exchanges between rounds go through LDS.  A limb (256 KiB) does not fit the 160 KiB LDS, so each
// exchange runs in two phases over a 132 KiB window:
//   exchange 1 (h <-> m across all threads): phase P moves the elements with h4 ^ m4 == P; a thread
//     writes and re-reads the same half X = a4 ^ P of its registers (a4 = a >> 4 is wave-uniform, so
//     every register index stays compile-time);
//   exchange 2 (m <-> l inside each group of 32 threads with the same h): waves with a4 == P in phase P.
// Padded strides (33 words) keep both access patterns of each exchange free of bank conflicts.
#include <mutex>

#include "hec_internal.h"

namespace hec {

namespace {

constexpr int NTT1_LDS_WORDS = 2 * 16 * 16 * 33;  // 16,896 words = 135,168 B

template <bool FP>
__device__ __forceinline__ void bfly1(u64 &x, u64 &y, const u64 *tw2, u64 idx, const DevPrime &pr)
{
    if constexpr (FP) {
        double X = __longlong_as_double((long long)x), Y = __longlong_as_double((long long)y);
        ct_bfly_fp(X, Y, __longlong_as_double((long long)tw2[idx]), pr.qd, pr.qinv);
        x = (u64)__double_as_longlong(X);
        y = (u64)__double_as_longlong(Y);
    } else {
        const ulonglong2 w = reinterpret_cast<const ulonglong2 *>(tw2)[idx];
        ct_bfly(x, y, w.x, w.y, pr.q, 2 * pr.q);
    }
}

// five stages S0 .. S0+4 on the thread's 32 registers (register index = the round's 5-bit digit);
// twiddle index of the pair at digit position r with the digit's top bits r >> (5 - j) at stage S0 + j:
//   2^(S0+j) + (base << j) + (r >> (5 - j))
template <bool FP, int S0>
__device__ __forceinline__ void round5(u64 *v, const u64 *tw, u64 base, const DevPrime &pr)
{
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int half = 16 >> j;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & half) continue;
            bfly1<FP>(v[r], v[r + half], tw, (1ull << (S0 + j)) + (base << j) + (u64)(r >> (5 - j)), pr);
        }
    }
}

template <int X>
__device__ __forceinline__ void exch1_half(u64 *v, u64 *lds, int a, int b)
{
    const int a4 = a >> 4, ap = a & 15;
#pragma unroll
    for (int hp = 0; hp < 16; ++hp) lds[((a4 * 16 + hp) * 16 + ap) * 33 + b] = v[X * 16 + hp];
    __syncthreads();
#pragma unroll
    for (int mp = 0; mp < 16; ++mp) v[X * 16 + mp] = lds[((X * 16 + ap) * 16 + mp) * 33 + b];
    __syncthreads();
}

__device__ __forceinline__ void exchange1(u64 *v, u64 *lds, int a, int b)
{
    if ((a >> 4) == 0) {  // phase 0 moves half X = a4, phase 1 half X = a4 ^ 1
        exch1_half<0>(v, lds, a, b);
        exch1_half<1>(v, lds, a, b);
    } else {
        exch1_half<1>(v, lds, a, b);
        exch1_half<0>(v, lds, a, b);
    }
}

__device__ __forceinline__ void exchange2(u64 *v, u64 *lds, int a, int b)
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

// forward NTT of one limb: v[h] holds element h 1024 + t on entry (canonical), v[l] element t 32 + l
// on exit (canonical)
template <bool FP>
__device__ __forceinline__ void ntt1_forward(u64 *v, u64 *lds, const u64 *tw, const DevPrime &pr)
{
    const int t = threadIdx.x, a = t >> 5, b = t & 31;
    if constexpr (FP) {
#pragma unroll
        for (int r = 0; r < 32; ++r) v[r] = (u64)__double_as_longlong(u2d(v[r]));
    }
    round5<FP, 0>(v, tw, 0, pr);
    exchange1(v, lds, a, b);
    round5<FP, 5>(v, tw, (u64)a, pr);
    exchange2(v, lds, a, b);
    round5<FP, 10>(v, tw, (u64)t, pr);
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        if constexpr (FP) v[r] = fp_canon(__longlong_as_double((long long)v[r]), pr.qd, pr.qinv);
        else v[r] = csub(csub(v[r], 2 * pr.q), pr.q);
    }
}

// plain batched forward NTT: job -> (poly = job / nl, limb = job % nl), prime pmap[limb]
struct Ntt1Strided {
    const u64 *src;
    u64 *dst;
    u64 ps_src, ps_dst;
    int nl;
    u32 elt;
    int pmap[HEC_MAXL + 1];
};

template <int CLS>  // 0: per-block branch on the prime's class, 1: FP64 only, 2: integer only
__global__ void __launch_bounds__(1024) k_ntt1_fwd(const Ntt1Strided io, const u64 *__restrict__ twi,
                                                   const u64 *__restrict__ twf, const DevPrime *__restrict__ primes)
{
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    constexpr int logN = 15;
    const int job = blockIdx.x, poly = job / io.nl, limb = job % io.nl;
    const int p = io.pmap[limb];
    const DevPrime pr = primes[p];
    const u64 *s = io.src + (u64)poly * io.ps_src + ((u64)limb << logN);
    u64 *d = io.dst + (u64)poly * io.ps_dst + ((u64)limb << logN);
    const int t = threadIdx.x;
    u64 v[32];
#pragma unroll
    for (int h = 0; h < 32; ++h) {
        const u32 g = (u32)(h * 1024 + t);
        v[h] = s[io.elt == 1 ? g : galois_src(g, io.elt, logN)];
    }
    if (CLS == 1 || (CLS == 0 && pr.fp)) ntt1_forward<true>(v, lds, twf + ((u64)p << logN), pr);
    else ntt1_forward<false>(v, lds, twi + ((u64)p << (logN + 1)), pr);
    u64 *o = d + (u64)t * 32;
#pragma unroll
    for (int l = 0; l < 32; l += 2) *reinterpret_cast<ulonglong2 *>(o + l) = ulonglong2{v[l], v[l + 1]};
}

}  // namespace

bool ntt1_forward_strided(Ctx &c, const u64 *src, u64 ps_src, u64 *dst, u64 ps_dst, int nl, const int *pmap,
                          int njobs, u32 elt)
{
    if (c.logN != 15 || njobs <= 0 || nl > HEC_MAXL + 1) return false;
    if (src == dst && elt != 1) return false;  // the permuted loads gather across the limb
    Ntt1Strided io{};
    io.src = src; io.dst = dst; io.ps_src = ps_src; io.ps_dst = ps_dst; io.nl = nl; io.elt = elt;
    for (int i = 0; i < nl; ++i) io.pmap[i] = pmap[i];
    bool anyfp = false, anyint = false;
    for (int i = 0; i < nl; ++i) (c.hprimes[pmap[i]].fp ? anyfp : anyint) = true;
    const int cls = anyfp && anyint ? 0 : anyfp ? 1 : 2;
    constexpr int bytes = NTT1_LDS_WORDS * 8;
    static std::once_flag attr[3];  // lanes may launch from several host threads
    const void *fn = cls == 0 ? reinterpret_cast<const void *>(&k_ntt1_fwd<0>)
                     : cls == 1 ? reinterpret_cast<const void *>(&k_ntt1_fwd<1>)
                                : reinterpret_cast<const void *>(&k_ntt1_fwd<2>);
    std::call_once(attr[cls],
                   [&] { HEC_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes)); });
    const u64 *twi = reinterpret_cast<const u64 *>(c.tw), *twf = reinterpret_cast<const u64 *>(c.twf);
    const dim3 g((unsigned)njobs);
    if (cls == 0) k_ntt1_fwd<0><<<g, 1024, bytes, c.stream>>>(io, twi, twf, c.primes);
    else if (cls == 1) k_ntt1_fwd<1><<<g, 1024, bytes, c.stream>>>(io, twi, twf, c.primes);
    else k_ntt1_fwd<2><<<g, 1024, bytes, c.stream>>>(io, twi, twf, c.primes);
    HEC_HIP(hipGetLastError());
    return true;
}

}  // namespace hec
