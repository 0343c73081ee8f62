// CKKS encoder on the GPU: SEAL CKKSEncoder::encode of complex (or real) slot
// vectors into NTT-form plaintexts, for `count` vectors per launch.  The reference encodes every
// matrix column / diagonal this way before encryption (src/demos/matrix_operations.cpp:1106-1108,
// client.cpp:228-230) and the ct x pt matvec's plaintext diagonals come from it.
//
// Steps (SEAL CKKSEncoder::encode_internal, with a radix-2 FFT for SEAL's inverse DWT):
//   1. slot i -> position bitrev((3^i mod 2N - 1) / 2), its conjugate -> bitrev((2N - 3^i mod 2N - 1) / 2)
//      (SEAL's matrix_reps_index_map_ with the FFT's bit-reversal folded into the scatter);
//   2. radix-2 decimation-in-time FFT over N complex points, stage len = 2 .. N, twiddle
//      w_j = polar(1, (-2 pi / len) j) from a host-built table (glibc cos/sin);
//   3. coefficient k = round(Re(v_k polar(1, -pi k / N)) / N * scale), the largest |coefficient| kept
//      per vector for SEAL's "encoded values are too large" check;
//   4. per data prime: signed residue, then the forward NTT (the engine's k_ntt).
// The arithmetic is plain IEEE double with no contraction (this file is built with -ffp-contract=off
// and the pragma below), so every intermediate is the IEEE result of the stated expression, the same
// on any host that evaluates it in that order without contraction (tests/test_gpu_encode.py).
// Not on the matvec's timed path: diagonals are encoded once per matrix.
#include "hec_internal.h"

#pragma clang fp contract(off)

namespace hec {

namespace {

__device__ __forceinline__ double2 cmul(double2 x, double2 w)  // std::complex<double> x * w
{
    return make_double2(x.x * w.x - x.y * w.y, x.x * w.y + x.y * w.x);
}

// step 1: one thread per slot i of vector blockIdx.y
__global__ void __launch_bounds__(256) k_enc_scatter(const double *__restrict__ re, const double *__restrict__ im,
                                                     u64 nv, const u32 *__restrict__ map, double2 *__restrict__ a,
                                                     int logN)
{
    const u64 slots = 1ull << (logN - 1);
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= slots) return;
    const u64 v = blockIdx.y;
    double2 z = make_double2(0.0, 0.0);
    if (i < nv) z = make_double2(re[v * nv + i], im ? im[v * nv + i] : 0.0);
    double2 *av = a + (v << logN);
    av[map[i]] = z;
    av[map[slots + i]] = make_double2(z.x, -z.y);
}

// step 2, stages len = 2 .. 2^LOGC inside contiguous chunks of 2^LOGC points staged in LDS
template <int LOGC>
__global__ void __launch_bounds__(256) k_enc_fft_lds(double2 *__restrict__ a, const double2 *__restrict__ tw, int logN)
{
    constexpr int C = 1 << LOGC;
    __shared__ double2 s[C];
    double2 *base = a + ((u64)blockIdx.y << logN) + (u64)blockIdx.x * C;
    for (int k = threadIdx.x; k < C; k += 256) s[k] = base[k];
    __syncthreads();
#pragma unroll 1
    for (int lg = 1; lg <= LOGC; ++lg) {
        const int half = 1 << (lg - 1);
        const double2 *w = tw + (half - 1);
        for (int b = threadIdx.x; b < C / 2; b += 256) {
            const int j = b & (half - 1);
            const int i0 = ((b >> (lg - 1)) << lg) + j;
            const double2 u = s[i0], v = cmul(s[i0 + half], w[j]);
            s[i0] = make_double2(u.x + v.x, u.y + v.y);
            s[i0 + half] = make_double2(u.x - v.x, u.y - v.y);
        }
        __syncthreads();
    }
    for (int k = threadIdx.x; k < C; k += 256) base[k] = s[k];
}

// step 2's remaining stages (len = 2C .. N, C = N >> TS) on the 2^TS points r + t C of column r held
// in registers, then steps 3 and 4's residues: out[v][i][k] for i < level
template <int TS>
__global__ void __launch_bounds__(256) k_enc_finish(const double2 *__restrict__ a, const double2 *__restrict__ tw,
                                                    const double2 *__restrict__ twist, int logN, double scale,
                                                    int level, const DevPrime *__restrict__ primes,
                                                    u64 *__restrict__ out, unsigned long long *__restrict__ maxabs)
{
    constexpr int R = 1 << TS;
    const u64 N = 1ull << logN, C = N >> TS;
    const u64 r = (u64)blockIdx.x * 256 + threadIdx.x;
    if (r >= C) return;
    const u64 v = blockIdx.y;
    const double2 *av = a + (v << logN);
    double2 x[R];
#pragma unroll
    for (int t = 0; t < R; ++t) x[t] = av[r + t * C];
#pragma unroll
    for (int s = 0; s < TS; ++s) {
        const u64 half = C << s;
        const double2 *w = tw + (half - 1);
#pragma unroll
        for (int t = 0; t < R; ++t) {
            if (t & (1 << s)) continue;
            const u64 j = r + (u64)(t & ((1 << s) - 1)) * C;
            const double2 u = x[t], y = cmul(x[t + (1 << s)], w[j]);
            x[t] = make_double2(u.x + y.x, u.y + y.y);
            x[t + (1 << s)] = make_double2(u.x - y.x, u.y - y.y);
        }
    }
    double mx = 0.0;
    u64 *ov = out + v * (u64)level * N;
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const u64 k = r + t * C;
        const double c = round(cmul(x[t], twist[k]).x / (double)N * scale);
        const double ac = fabs(c);
        mx = fmax(mx, ac);
        // |c| >= 2^62 is rejected by the caller ("encoded values are too large"); keep the cast defined
        const u64 mag = ac < 0x1.0p62 ? (u64)ac : 0;
        for (int i = 0; i < level; ++i) {
            const u64 q = primes[i].q, m = mag % q;
            ov[(u64)i * N + k] = (c < 0 && m) ? q - m : m;
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
    const int logc = logN < 11 ? logN : 11, ts = logN - logc;
    const double2 *tw = reinterpret_cast<const double2 *>(c.enc_tw), *twist = reinterpret_cast<const double2 *>(c.enc_twist);
    double2 *a = reinterpret_cast<double2 *>(work);
    HEC_HIP(hipMemsetAsync(maxabs, 0, count * sizeof(u64), c.stream));
    k_enc_scatter<<<dim3((unsigned)((N / 2 + 255) / 256), count), 256, 0, c.stream>>>(re, im, nv, c.enc_map, a, logN);
    HEC_HIP(hipGetLastError());
    const dim3 gl((unsigned)(N >> logc), count);
    switch (logc) {
    case 11: k_enc_fft_lds<11><<<gl, 256, 0, c.stream>>>(a, tw, logN); break;
    case 10: k_enc_fft_lds<10><<<gl, 256, 0, c.stream>>>(a, tw, logN); break;
    default: throw std::invalid_argument("encode: N must be 2^10 .. 2^16");
    }
    HEC_HIP(hipGetLastError());
    const dim3 gf((unsigned)(((N >> ts) + 255) / 256), count);
    auto *mx = reinterpret_cast<unsigned long long *>(maxabs);
    switch (ts) {
    case 0: k_enc_finish<0><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    case 1: k_enc_finish<1><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    case 2: k_enc_finish<2><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    case 3: k_enc_finish<3><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    case 4: k_enc_finish<4><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    case 5: k_enc_finish<5><<<gf, 256, 0, c.stream>>>(a, tw, twist, logN, scale, level, c.primes, out, mx); break;
    default: throw std::invalid_argument("encode: N must be 2^10 .. 2^16");
    }
    HEC_HIP(hipGetLastError());
    int pmap[HEC_MAXL + 1];
    for (int i = 0; i <= HEC_MAXL; ++i) pmap[i] = i;
    ntt_strided(c, false, out, (u64)level * N, out, (u64)level * N, level, pmap, count * level);
}

}  // namespace hec
