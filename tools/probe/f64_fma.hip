// f64 vector FMA throughput probe (development tool): every CU full of waves, each thread
// runs 8 independent v_fma_f64 chains; prints TFLOP/s (2 flop per FMA).  The C5 roofline
// quotes this measured rate: MI355X_MICROARCH.md lists the f32 peaks but no f64 figure.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) fma_f64(double* out, int iters, double a, double b) {
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
    for (int k = 0; k < iters; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], a, b);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    if (s == 12345.678) out[0] = s;        // keeps the chains alive
}

int main() {
    double* d;
    hipMalloc(&d, 8);
    const int blocks = 256 * 8, iters = 20000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    fma_f64<<<blocks, 256>>>(d, 100, 0.999, 1e-3);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        fma_f64<<<blocks, 256>>>(d, iters, 0.999, 1e-3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double flop = 2.0 * 8 * (double)iters * blocks * 256;
    printf("{\"f64_fma_tflops\": %.2f, \"ms\": %.3f}\n", flop / (best * 1e-3) / 1e12, best);
    return 0;
}
