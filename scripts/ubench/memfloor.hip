// Memory floor of the encode access pattern (k=128 inputs, r=32 outputs, 64 KiB symbols, 8192 stripes):
// each block reads CH contiguous bytes of every input symbol of one stripe and writes CH bytes of every
// output symbol; W = bytes per lane per load. Prints GB/s of algorithmic bytes (k + r) * S per stripe.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int W> struct V;
template <> struct V<4> { typedef uint32_t T; };
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <> struct V<8> { typedef u32x2 T; };
template <> struct V<16> { typedef u32x4 T; };
__device__ inline uint32_t fold(uint32_t a) { return a; }
__device__ inline uint32_t fold(u32x2 a) { return a.x ^ a.y; }
__device__ inline uint32_t fold(u32x4 a) { return a.x ^ a.y ^ a.z ^ a.w; }
template <int W> __device__ inline typename V<W>::T mk(uint32_t v) { typename V<W>::T t; memset(&t, 0, sizeof t); *(uint32_t*)&t = v; return t; }

// ORDER 0: grid (chunk, stripe); 1: grid (stripe-group-major: chunk fastest within groups of G stripes)
template <int CH, int W, int UNR, int NT>
__global__ void k_mem(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t sstride, int64_t sym, int K, int R) {
    typedef typename V<W>::T T;
    const int64_t stripe = blockIdx.y;
    const int64_t off = int64_t(blockIdx.x) * CH + int64_t(threadIdx.x) * W;
    const uint8_t* b = src + stripe * sstride + off;
    uint32_t acc = 0;
    for (int i = 0; i < K; i += UNR) {
        T v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load((const T*)(b + int64_t(i + u) * sym)) : *(const T*)(b + int64_t(i + u) * sym);
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc ^= fold(v[u]) + u;
    }
    uint8_t* d = dst + stripe * sstride + int64_t(K) * sym + off;
    for (int p = 0; p < R; ++p) *(T*)(d + int64_t(p) * sym) = mk<W>(acc ^ p);
}

template <int CH, int W, int UNR, int NT = 0>
void run(uint8_t* buf, int64_t n, int64_t S, int K, int R) {
    const int64_t sstride = int64_t(K + R) * S;
    dim3 grid(unsigned(S / CH), unsigned(n)), blk(CH / W);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k_mem<CH, W, UNR, NT>), grid, blk, 0, 0, buf, buf, sstride, S, K, R);
    hipEventRecord(a);
    const int it = 5;
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL((k_mem<CH, W, UNR, NT>), grid, blk, 0, 0, buf, buf, sstride, S, K, R);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    ms /= it;
    const double bytes = double(n) * (K + R) * S;
    printf("{\"CH\": %d, \"W\": %d, \"UNR\": %d, \"NT\": %d, \"threads\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n", CH, W, UNR, NT, CH / W, ms, bytes / ms / 1e6);
}

int main() {
    const int64_t n = 8192, S = 65536; const int K = 128, R = 32;
    uint8_t* buf; 
    if (hipMalloc(&buf, size_t(n) * (K + R) * S) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 1, size_t(n) * (K + R) * S);
    run<256, 4, 8>(buf, n, S, K, R);
    run<256, 4, 8, 1>(buf, n, S, K, R);
    run<256, 4, 16>(buf, n, S, K, R);
    run<512, 8, 8>(buf, n, S, K, R);
    run<1024, 16, 8>(buf, n, S, K, R);
    run<1024, 4, 8>(buf, n, S, K, R);
    run<2048, 8, 8>(buf, n, S, K, R);
    run<4096, 16, 8>(buf, n, S, K, R);
    run<2048, 16, 8>(buf, n, S, K, R);
    hipFree(buf);
    return 0;
}
