// mfma_f64_occ.hip -- fp64 MFMA throughput vs waves per SIMD and independent
// accumulators per wave (v_mfma_f64_16x16x4f64, 2048 flop each).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ void __launch_bounds__(1024) loop(int iters, double *out) {
    d4 acc[ACC];
    for (int a = 0; a < ACC; ++a) acc[a] = d4{0.0, 0.0, 0.0, 0.0};
    double x = 1.0 + threadIdx.x * 1e-3, y = 1.0 - threadIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int a = 0; a < ACC; ++a) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[a], 0, 0, 0);
    }
    double s = 0.0;
    for (int a = 0; a < ACC; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
    if (s == 12345.678) out[0] = s;
}

template <int ACC>
void run(int wps, double *d) {
    // one block per CU of wps*4 waves
    const int threads = 256 * wps, blocks = 256, iters = 32768 / ACC;
    hipLaunchKernelGGL(loop<ACC>, dim3(blocks), dim3(threads), 0, 0, 64, d);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL(loop<ACC>, dim3(blocks), dim3(threads), 0, 0, iters, d);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const double flop = (double)blocks * (threads / 64) * iters * ACC * 2048.0;
    const double mfma_per_simd = (double)(threads / 64) / 4 * iters * ACC;
    printf("{\"waves_per_simd\": %d, \"acc\": %d, \"tflops\": %.2f, \"ns_per_mfma_per_simd\": %.2f}\n", wps, ACC,
           flop / (best * 1e-3) / 1e12, best * 1e6 / mfma_per_simd);
}

int main() {
    double *d;
    (void)hipMalloc(&d, 8);
    for (int w : {1, 2, 4}) {
        run<4>(w, d);
        run<8>(w, d);
        run<16>(w, d);
    }
    return 0;
}
