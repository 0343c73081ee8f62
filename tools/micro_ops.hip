// Microbenchmark (development tool, not product): per-wave issue cost of the integer / FP64
// instructions a 64-bit modular butterfly is built from on gfx950.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_ops.hip -o /tmp/micro_ops
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint64_t u64;
typedef uint32_t u32;

#define ITERS 4096
#define CHAINS 8

template <int OP>
__global__ void __launch_bounds__(256) k_op(u64 *out, u64 seed)
{
    u64 v[CHAINS];
    double d[CHAINS];
    u32 w[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        v[c] = seed * (threadIdx.x + 1 + c) | 1;
        d[c] = (double)(v[c] >> 20);
        w[c] = (u32)v[c];
    }
    const u64 k = seed | 3;
    const double dk = 1.0000001;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (OP == 0) v[c] = __umul64hi(v[c], k);                     // 64x64 high
            if constexpr (OP == 1) v[c] = v[c] * k;                                // 64x64 low
            if constexpr (OP == 2) v[c] = (u64)w[c] * (u32)k + v[c];              // mad_u64_u32
            if constexpr (OP == 3) w[c] = w[c] * (u32)k + 1;                      // mul_lo_u32
            if constexpr (OP == 4) w[c] = __umulhi(w[c], (u32)k) ^ 1;            // mul_hi_u32
            if constexpr (OP == 5) d[c] = fma(d[c], dk, 1.0);                     // fma_f64
            if constexpr (OP == 6) v[c] = v[c] + k;                               // add_u64
            if constexpr (OP == 7) w[c] = __mul24(w[c], (u32)k) + 1;             // mul_u32_u24
            if constexpr (OP == 8) d[c] = rint(d[c] * dk);                        // mul + rint f64
        }
    }
    u64 acc = 0;
    for (int c = 0; c < CHAINS; ++c) acc += v[c] + w[c] + (u64)d[c];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int OP>
float run(u64 *out)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 8;
    k_op<OP><<<blocks, 256>>>(out, 12345);
    hipEventRecord(a);
    k_op<OP><<<blocks, 256>>>(out, 12345);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // ops per SIMD: waves = blocks*4 ; per SIMD = waves / (256 CU * 4 SIMD)
    const double waves_per_simd = blocks * 4.0 / (256 * 4);
    const double ops_per_wave = (double)ITERS * CHAINS;
    const double cycles = ms * 1e-3 * 2.4e9;  // at 2.4 GHz nominal
    printf("op %d: %.3f ms  -> %.2f cycles per wave-op (at 2.4 GHz, per SIMD)\n", OP, ms,
           cycles / (waves_per_simd * ops_per_wave));
    return ms;
}

int main()
{
    u64 *out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(u64));
    const char *names[] = {"umul64hi", "mul64lo", "mad_u64_u32", "mul_lo_u32", "mul_hi_u32", "fma_f64", "add_u64",
                           "mul_u32_u24", "mul_f64+rint"};
    run<0>(out); run<1>(out); run<2>(out); run<3>(out); run<4>(out); run<5>(out); run<6>(out); run<7>(out);
    run<8>(out);
    for (auto n : names) printf("%s ", n);
    printf("\n");
    return 0;
}
