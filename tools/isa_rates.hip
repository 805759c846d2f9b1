// Issue cost of the sampler's instruction classes on gfx950 (round 6 measurement tool):
// one wave alone on a SIMD runs 8 independent chains of one instruction, N iterations; the
// shader-clock delta per instruction is that instruction's issue cost for one wave.  Then the
// same loop at 8 waves per SIMD over the whole chip (events), cycles per instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/isa_rates.hip -o tools/isa_rates && ./tools/isa_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int OP>
__global__ void k(int n, unsigned long long* cyc, double* sink) {
    double d0 = threadIdx.x * 1e-3 + 1.0, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    unsigned u0 = threadIdx.x + 1, u1 = u0 * 3, u2 = u0 * 5, u3 = u0 * 7, u4 = u0 * 11, u5 = u0 * 13, u6 = u0 * 17, u7 = u0 * 19;
    float f0 = d0, f1 = d1, f2 = d2, f3 = d3, f4 = d4, f5 = d5, f6 = d6, f7 = d7;
    unsigned long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#define R8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
        if constexpr (OP == 0) {  // v_fma_f64
#define M(j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d##j) : "v"(d0), "v"(d1));
            R8(M)
#undef M
        } else if constexpr (OP == 1) {  // v_mad_u64_u32
#define M(j) { unsigned long long r; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(u##j), "v"(u1) : "vcc"); u##j = (unsigned)r ^ (unsigned)(r >> 32); }
            R8(M)
#undef M
        } else if constexpr (OP == 2) {  // v_mul_lo_u32
#define M(j) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u##j) : "v"(u1));
            R8(M)
#undef M
        } else if constexpr (OP == 3) {  // v_fma_f32
#define M(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f##j) : "v"(f0), "v"(f1));
            R8(M)
#undef M
        } else if constexpr (OP == 4) {  // v_rcp_f64
#define M(j) asm volatile("v_rcp_f64 %0, %0" : "+v"(d##j));
            R8(M)
#undef M
        } else if constexpr (OP == 5) {  // v_xor_b32
#define M(j) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u##j) : "v"(u1));
            R8(M)
#undef M
        } else if constexpr (OP == 6) {  // v_mul_hi_u32
#define M(j) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u##j) : "v"(u1));
            R8(M)
#undef M
        } else if constexpr (OP == 7) {  // v_mul_u32_u24
#define M(j) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u##j) : "v"(u1));
            R8(M)
#undef M
        } else if constexpr (OP == 8) {  // v_pk_fma_f32
#define M(j) { double x = d##j; asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(d0), "v"(d1)); d##j = x; }
            R8(M)
#undef M
        } else if constexpr (OP == 9) {  // v_rsq_f64
#define M(j) asm volatile("v_rsq_f64 %0, %0" : "+v"(d##j));
            R8(M)
#undef M
        } else if constexpr (OP == 10) {  // v_add_f64
#define M(j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d##j) : "v"(d0));
            R8(M)
#undef M
        } else if constexpr (OP == 11) {  // v_cvt_f64_u32
#define M(j) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d##j) : "v"(u##j));
            R8(M)
#undef M
        }
    }
    unsigned long long t1 = clock64();
    if (threadIdx.x == 0 && cyc) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 + u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7 +
                                                  f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
}

template <int OP>
int run(const char* name) {
    const int n = 4096;
    unsigned long long* cyc; double* sink;
    CHK(hipMalloc(&cyc, 8 * 4096)); CHK(hipMalloc(&sink, 8 * 64 * 8192));
    hipLaunchKernelGGL(k<OP>, dim3(1), dim3(64), 0, 0, n, cyc, sink);
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k<OP>, dim3(1), dim3(64), 0, 0, n, cyc, sink);
    unsigned long long c = 0;
    CHK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    // throughput: 256 CUs x 4 SIMDs x 8 waves
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const int blocks = 256 * 8;  // 4-wave blocks: 8 per CU = 8 waves per SIMD
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, n, nullptr, sink);
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, n, nullptr, sink);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    int mhz = 0; CHK(hipDeviceGetAttribute(&mhz, hipDeviceAttributeClockRate, 0));
    const double instr_per_simd = 8.0 * n * 8;  // 8 waves x n x 8 instructions
    printf("%-16s one wave: %6.2f shader clocks / instr   chip: %6.2f cycles / instr / SIMD (at %d MHz)\n", name,
           (double)c / (8.0 * n), ms * 1e-3 * mhz * 1e3 / instr_per_simd, mhz / 1000);
    CHK(hipFree(cyc)); CHK(hipFree(sink));
    return 0;
}

int main() {
    return run<0>("v_fma_f64") | run<10>("v_add_f64") | run<3>("v_fma_f32") | run<8>("v_pk_fma_f32") |
           run<1>("v_mad_u64_u32") | run<2>("v_mul_lo_u32") | run<6>("v_mul_hi_u32") | run<7>("v_mul_u32_u24") |
           run<5>("v_xor_b32") | run<4>("v_rcp_f64") | run<9>("v_rsq_f64") | run<11>("v_cvt_f64_u32");
}
