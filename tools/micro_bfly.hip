// Microbenchmark (development tool, not product): cost of one forward (Harvey) NTT butterfly for a
// 60-bit prime under several exact formulations, in VALU cycles per wave, on gfx950.  Every variant's
// outputs are canonicalised at the end and compared with variant 0 (the engine's ct_bfly), so a
// formulation that is fast but wrong shows as FAIL.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_bfly.hip -o tools/micro_bfly.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../homomorphic-encryption-algorithms-diploma-thesis_amd/csrc/hec_device.h"

#define ITERS 1024
#define CHAINS 8
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); exit(1); } } while (0)

struct Tw {
    u64 w, wq;          // Shoup pair
    double fh, fl;      // w / q as a double-double, scaled by 2^31
};

// V1: Shoup with the x0*wq0 high word dropped (quotient low by at most 1) and the q*qhat low product
// using q_hi = 2^28 - 1 (q = 2^60 - c, c < 2^32).  t in [0, 3q) -> one extra conditional subtract.
__device__ __forceinline__ u64 shoup_s(u64 x, u64 w, u64 wq, u64 q)
{
    const u32 x0 = (u32)x, x1 = (u32)(x >> 32);
    const u32 w0 = (u32)w, w1 = (u32)(w >> 32);
    const u32 a0 = (u32)wq, a1 = (u32)(wq >> 32);
    const u64 xw = (u64)x0 * w0 + ((u64)(x1 * w0 + x0 * w1) << 32);
    const u64 t = (u64)x1 * a0;                       // + hi(x0 * a0) dropped
    const u64 u = (u64)x0 * a1 + (u32)t;
    const u64 qh = (u64)x1 * a1 + (t >> 32) + (u >> 32);
    const u32 h0 = (u32)qh, h1 = (u32)(qh >> 32);
    const u32 q0 = (u32)q;
    const u64 hq = (u64)h0 * q0 + ((u64)(h1 * q0 + (h0 << 28) - h0) << 32);
    return xw - hq;
}

// V2: quotient from FP64 (x split 31/31 bits, w/q as a double-double), remainder from two low products.
__device__ __forceinline__ u64 fpq_lazy(u64 x, u64 w, double fh, double fl, u64 q)
{
    const double dh = (double)(u32)(x >> 31), dl = (double)(u32)(x & 0x7fffffffu);
    const double p = dh * fh;                           // fh = (w/q) * 2^31 (hi part)
    const double e = __fma_rn(dh, fh, -p);
    const double rest = __fma_rn(dh, fl, e) + dl * (fh * 4.656612873077393e-10);  // dl * w/q
    const double qa = floor(p * 2.3283064365386963e-10);                           // p / 2^32
    const double rem = __fma_rn(-qa, 4294967296.0, p) + rest - 0.5;
    const long long qb = (long long)floor(rem);
    const u64 qhat = ((u64)(u32)qa << 32) + (u64)qb;
    return x * w - qhat * q;                            // Q - qhat in (0.49, 1.51)
}

// V3: the engine's Shoup product with q = 2^60 - c (c < 2^32, SEAL's 60-bit primes): hi q mod 2^64 =
// (hi << 60) - hi c, two multiplies instead of three.  V4: V3 plus the conditional subtractions by the sign of
// x - 2q (no VCC compare / select).
__device__ __forceinline__ u64 shoup_c(u64 x, u64 w, u64 wq, u32 c)
{
    const u64 hi = mulhi64(x, wq);
    const u64 hc = (u64)(u32)hi * c + ((u64)((u32)(hi >> 32) * c) << 32);
    return x * w + hc - (hi << 60);
}
__device__ __forceinline__ u64 csub_sign(u64 x, u64 m)  // x < 2m... : x - m if x >= m, as x + (-m) then add back
{
    const u64 d = x - m;
    const u64 s = (u64)((long long)d >> 63);
    return d + (m & s);
}

// V6 / V7 (round 5): split-input Shoup.  Y = y1 2^31 + y0 (Y < 4q < 2^62, y0, y1 < 2^31), so
//   Y w = y1 a + y0 b (mod q),  a = w 2^31 mod q, b = w,
// and the quotient comes from two 32-bit Shoup factors a' = floor(a 2^32 / q), b' = floor(b 2^32 / q):
//   qh = (y1 a' + y0 b') >> 32  (the sum < 2^63 + 2^63, exact in one v_mad_u64_u32 chain),
// T / q - qh < (y1 + y0) / 2^32 + 1 < 2, so qh is Q or Q - 1 and t = T - qh q is in [0, 2q) (no extra subtraction).
// Multiplies: 2 (quotient) + 4 (T mod 2^64) + 1 (qh q with q = 2^60 - c, V6) or 2 (any q, V7), against Shoup's 10.
struct TwS { u64 a, b; u32 ap, bp; };
__device__ __forceinline__ u64 shoup_split(u64 Y, const TwS &w, u64 q, u32 c, bool special)
{
    const u32 y0 = (u32)Y & 0x7fffffffu, y1 = (u32)(Y >> 31);
    const u64 qs = (u64)y1 * w.ap + (u64)y0 * w.bp;
    const u32 qh = (u32)(qs >> 32);
    const u64 T = (u64)y1 * (u32)w.a + (u64)y0 * (u32)w.b +
                  ((u64)(y1 * (u32)(w.a >> 32) + y0 * (u32)(w.b >> 32)) << 32);
    if (special) return T + (u64)qh * c - ((u64)qh << 60);
    return T - ((u64)qh * (u32)q + ((u64)(qh * (u32)(q >> 32)) << 32));
}

// V8: V7 with the quotient product folded into the same multiply-add chain through nq = 2^64 - q: t = (y0 b + y1 a +
// qh nq) mod 2^64, the low words in one v_mad_u64_u32 chain, the high words as three 32-bit products
__device__ __forceinline__ u64 shoup_split_nq(u64 Y, const TwS &w, u64 nq)
{
    const u32 y0 = (u32)Y & 0x7fffffffu, y1 = (u32)(Y >> 31);
    const u32 qh = (u32)(((u64)y1 * w.ap + (u64)y0 * w.bp) >> 32);
    const u64 lo = (u64)y0 * (u32)w.b + (u64)y1 * (u32)w.a + (u64)qh * (u32)nq;
    const u32 hi = y0 * (u32)(w.b >> 32) + y1 * (u32)(w.a >> 32) + qh * (u32)(nq >> 32);
    return lo + ((u64)hi << 32);
}

template <int V>
__global__ void __launch_bounds__(256) k_bfly(u64 *io, const u64 *tw_in, const double *twd, u64 q, int iters)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    u64 X[CHAINS], Y[CHAINS], W[CHAINS], WQ[CHAINS];
    double FH[CHAINS], FL[CHAINS];
    TwS WS[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        WS[c].a = tw_in[2 * CHAINS + 3 * c];
        WS[c].b = tw_in[2 * CHAINS + 3 * c + 1];
        WS[c].ap = (u32)tw_in[2 * CHAINS + 3 * c + 2];
        WS[c].bp = (u32)(tw_in[2 * CHAINS + 3 * c + 2] >> 32);
        X[c] = io[(size_t)g * 2 * CHAINS + 2 * c];
        Y[c] = io[(size_t)g * 2 * CHAINS + 2 * c + 1];
        W[c] = tw_in[2 * c];
        WQ[c] = tw_in[2 * c + 1];
        FH[c] = twd[2 * c];
        FL[c] = twd[2 * c + 1];
    }
    const u64 two_q = 2 * q;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (V == 0) {
                ct_bfly(X[c], Y[c], W[c], WQ[c], q, two_q);
            } else if constexpr (V == 1) {
                const u64 x = X[c] >= two_q ? X[c] - two_q : X[c];
                u64 t = shoup_s(Y[c], W[c], WQ[c], q);
                t = t >= two_q ? t - two_q : t;
                X[c] = x + t;
                Y[c] = x - t + two_q;
            } else if constexpr (V == 3) {
                const u64 x = X[c] >= two_q ? X[c] - two_q : X[c];
                const u64 tt = shoup_c(Y[c], W[c], WQ[c], (u32)((1ull << 60) - q));
                X[c] = x + tt;
                Y[c] = x - tt + two_q;
            } else if constexpr (V == 4) {
                const u64 x = csub_sign(X[c], two_q);
                const u64 tt = shoup_c(Y[c], W[c], WQ[c], (u32)((1ull << 60) - q));
                X[c] = x + tt;
                Y[c] = x - tt + two_q;
            } else if constexpr (V == 5) {
                const u64 x = csub_sign(X[c], two_q);
                const u64 tt = shoup_lazy(Y[c], W[c], WQ[c], q);
                X[c] = x + tt;
                Y[c] = x - tt + two_q;
            } else if constexpr (V == 6 || V == 7) {
                const u64 x = X[c] >= two_q ? X[c] - two_q : X[c];
                const u64 tt = shoup_split(Y[c], WS[c], q, (u32)((1ull << 60) - q), V == 6);
                X[c] = x + tt;
                Y[c] = x - tt + two_q;
            } else if constexpr (V == 8) {
                const u64 x = X[c] >= two_q ? X[c] - two_q : X[c];
                const u64 tt = shoup_split_nq(Y[c], WS[c], 0 - q);
                X[c] = x + tt;
                Y[c] = x - tt + two_q;
            } else if constexpr (V == 2) {
                const u64 x = X[c] >= two_q ? X[c] - two_q : X[c];
                const u64 t = fpq_lazy(Y[c], W[c], FH[c], FL[c], q);  // in (0.49q, 1.51q)
                X[c] = x + t;
                Y[c] = x - t + two_q;
            }
        }
    }
    for (int c = 0; c < CHAINS; ++c) {
        io[(size_t)g * 2 * CHAINS + 2 * c] = X[c] % q;
        io[(size_t)g * 2 * CHAINS + 2 * c + 1] = Y[c] % q;
    }
}

static u64 mulmod_h(u64 a, u64 b, u64 q) { return (u64)((unsigned __int128)a * b % q); }

template <int V>
void run(const char *name, u64 q, const std::vector<u64> &init, u64 *d_io, u64 *d_tw, double *d_twd,
         std::vector<u64> &ref)
{
    const int blocks = 256 * 8;
    const size_t n = init.size();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipMemcpy(d_io, init.data(), n * 8, hipMemcpyHostToDevice));
    k_bfly<V><<<blocks, 256>>>(d_io, d_tw, d_twd, q, ITERS);  // warm
    CK(hipMemcpy(d_io, init.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipEventRecord(a));
    k_bfly<V><<<blocks, 256>>>(d_io, d_tw, d_twd, q, ITERS);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<u64> out(n);
    CK(hipMemcpy(out.data(), d_io, n * 8, hipMemcpyDeviceToHost));
    bool ok = true;
    if (V == 0) ref = out;
    else for (size_t i = 0; i < n; ++i) ok &= out[i] == ref[i];
    const double waves_per_simd = blocks * 4.0 / (256 * 4);
    const double bfly_per_wave = (double)ITERS * CHAINS;
    const double cycles = ms * 1e-3 * 2.4e9;
    printf("V%d %-28s %.3f ms  %.1f cycles/butterfly/wave  %s\n", V, name, ms, cycles / (waves_per_simd * bfly_per_wave),
           ok ? "ok" : "FAIL");
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main()
{
    const u64 q = 1152921504606584833ull;  // 2^60 - 262143, SEAL's first 60-bit prime for N = 2^15
    const int blocks = 256 * 8;
    const size_t n = (size_t)blocks * 256 * 2 * CHAINS;
    std::vector<u64> init(n);
    u64 s = 88172645463325252ull;
    for (auto &v : init) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = s % (4 * q); }
    std::vector<u64> tw(5 * CHAINS);
    std::vector<double> twd(2 * CHAINS);
    for (int c = 0; c < CHAINS; ++c) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const u64 w = s % q;
        tw[2 * c] = w;
        tw[2 * c + 1] = (u64)(((unsigned __int128)w << 64) / q);
        const u64 a = (u64)(((unsigned __int128)w << 31) % q);
        tw[2 * CHAINS + 3 * c] = a;
        tw[2 * CHAINS + 3 * c + 1] = w;
        tw[2 * CHAINS + 3 * c + 2] = (u64)(((unsigned __int128)a << 32) / q) | ((u64)(((unsigned __int128)w << 32) / q) << 32);
        const long double f = (long double)w / (long double)q * 2147483648.0L;
        twd[2 * c] = (double)f;
        twd[2 * c + 1] = (double)(f - (long double)twd[2 * c]);
    }
    (void)mulmod_h;
    u64 *d_io, *d_tw;
    double *d_twd;
    CK(hipMalloc(&d_io, n * 8));
    CK(hipMalloc(&d_tw, tw.size() * 8));
    CK(hipMalloc(&d_twd, twd.size() * 8));
    CK(hipMemcpy(d_tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_twd, twd.data(), twd.size() * 8, hipMemcpyHostToDevice));
    std::vector<u64> ref;
    run<0>("shoup (engine ct_bfly)", q, init, d_io, d_tw, d_twd, ref);
    run<1>("shoup approx-hi + q_hi", q, init, d_io, d_tw, d_twd, ref);
    run<2>("fp64 quotient", q, init, d_io, d_tw, d_twd, ref);
    run<3>("shoup, q = 2^60 - c", q, init, d_io, d_tw, d_twd, ref);
    run<4>("shoup, q = 2^60 - c, sign csub", q, init, d_io, d_tw, d_twd, ref);
    run<5>("shoup, sign csub", q, init, d_io, d_tw, d_twd, ref);
    run<6>("split-input shoup, 2^60 - c", q, init, d_io, d_tw, d_twd, ref);
    run<7>("split-input shoup, any q", q, init, d_io, d_tw, d_twd, ref);
    run<8>("split-input shoup, nq chain", q, init, d_io, d_tw, d_twd, ref);
    return 0;
}
