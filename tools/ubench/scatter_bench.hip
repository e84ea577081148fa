// scatter_bench.hip -- HBM write efficiency of the partition scatters' write
// pattern: every workgroup streams its input once and appends runs of R 8-byte
// records to S output streams per tile (stream s of workgroup g at (s*G+g)*len,
// the bucket-major layout of the level-1/level-2 scatters), with the stream
// starts 128-byte aligned or shifted by a random number of records.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scatter_bench.hip -o scatter_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int T = 1024;

// shift[s*G+g] = record offset of the stream start (0 when aligned)
__global__ void __launch_bounds__(T) scatter(const uint64_t *in, uint64_t *out, int S, int R, int64_t tiles,
                                             int64_t slen, const uint32_t *shift, int xcd) {
    const int G = gridDim.x;
    const int bx = blockIdx.x;
    const int g = xcd ? (bx % 8) * (G / 8) + bx / 8 : bx;
    const int tile = S * R;
    const int64_t base_in = (int64_t)g * tiles * tile;
    for (int64_t k = 0; k < tiles; ++k) {
        const uint64_t *src = in + base_in + k * tile;
        for (int j = threadIdx.x; j < tile; j += T) {
            const int s = j / R, i = j - s * R;
            const int64_t st = (int64_t)s * G + g;
            out[st * slen + shift[st] + k * R + i] = src[j];
        }
    }
}

__global__ void copy(const uint64_t *in, uint64_t *out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int main(int argc, char **argv) {
    const int G = 256;
    const int64_t n_target = argc > 1 ? atoll(argv[1]) : 500000000LL;
    uint64_t *in, *out;
    uint32_t *shift;
    const int64_t cap = n_target + (int64_t)G * 4096 * 16 + (1 << 20);
    CK(hipMalloc(&in, cap * 8));
    CK(hipMalloc(&out, cap * 8 + (int64_t)G * 4096 * 16 * 8));
    CK(hipMalloc(&shift, (int64_t)G * 4096 * 4));
    CK(hipMemset(in, 1, cap * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(copy, dim3(4096), dim3(256), 0, 0, in, out, n_target);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("copy            n=%lld  %.3f ms  %.0f GB/s\n", (long long)n_target, ms, 16.0 * n_target / ms / 1e6);
    const int cfg[][2] = {{1024, 16}, {1024, 8}, {1024, 32}, {512, 32}, {256, 64}, {64, 256}, {2048, 8}};
    uint32_t *h_shift = (uint32_t *)malloc((size_t)G * 4096 * 4);
    for (auto &c : cfg) {
        const int S = c[0], R = c[1];
        const int64_t tiles = n_target / ((int64_t)G * S * R);
        const int64_t slen = tiles * R + 16;         // records per stream region (+ room for the shift)
        const int64_t n = tiles * G * S * R;
        if ((int64_t)S * G * slen > cap + (int64_t)G * 4096 * 16) continue;
        for (int al = 0; al < 2; ++al)
            for (int xcd = 0; xcd < 2; ++xcd) {
                for (int64_t i = 0; i < (int64_t)G * S; ++i) h_shift[i] = al ? 0u : (uint32_t)((i * 2654435761ull >> 7) % 16);
                CK(hipMemcpy(shift, h_shift, (size_t)G * S * 4, hipMemcpyHostToDevice));
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipEventRecord(a));
                    hipLaunchKernelGGL(scatter, dim3(G), dim3(T), 0, 0, in, out, S, R, tiles, slen, shift, xcd);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                }
                printf("S=%4d R=%3d %-9s %-6s  %.3f ms  %.0f GB/s (%.2f ms per 1e9 records)\n", S, R,
                       al ? "aligned" : "shifted", xcd ? "xcd" : "linear", ms, 16.0 * n / ms / 1e6, ms * 1e9 / n);
            }
    }
    return 0;
}
