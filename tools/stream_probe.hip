// What this box's HBM sustains for the access mixes of the edge kernels (tools/stream_probe.hip):
//   rd2wr1  c = a + b      (the backward row GEMM: do, sigma' operand -> do')
//   rd2     sum(a * b)     (the dS TN GEMM: x, do)
//   rd1wr1  c = a          (the forward row GEMM: x^{l-1} -> x^l)
//   rd1     sum(a)         (the tail segmented reduction)
//   wr1     c = 1          (the layer-1 combine)
// float4 per lane, U independent 16-B accesses in flight per lane, grid-stride over 1 GiB tables
// (4M x 256 fp32, the config-3 edge-table size).  Plain loads / stores, or nontemporal (NT = 1).
// build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int MODE, int U, bool NT>
__global__ __launch_bounds__(256) void probe(long long n4, const f4* __restrict__ a, const f4* __restrict__ b,
                                             f4* __restrict__ c, float* __restrict__ part) {
    const long long stride = (long long)gridDim.x * 256 * U;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long i0 = ((long long)blockIdx.x * 256) * U + threadIdx.x; i0 < n4; i0 += stride) {
        f4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + u * 256;
            if (i < n4) {
                if constexpr (MODE != 4) va[u] = ld<U, NT>(a + i);
                if constexpr (MODE == 0 || MODE == 1) vb[u] = ld<U, NT>(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + u * 256;
            if (i >= n4) continue;
            if constexpr (MODE == 0) st<NT>(c + i, va[u] + vb[u]);
            else if constexpr (MODE == 1) acc += va[u] * vb[u];
            else if constexpr (MODE == 2) st<NT>(c + i, va[u]);
            else if constexpr (MODE == 3) acc += va[u];
            else st<NT>(c + i, f4{1.f, 1.f, 1.f, 1.f});
        }
    }
    if constexpr (MODE == 1 || MODE == 3) part[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

template <int MODE, int U, bool NT>
void run(const char* name, long long n4, f4* a, f4* b, f4* c, float* part, int blocks, double bytes_per_f4) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((probe<MODE, U, NT>), dim3(blocks), dim3(256), 0, 0, n4, a, b, c, part);
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<MODE, U, NT>), dim3(blocks), dim3(256), 0, 0, n4, a, b, c, part);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-7s U=%d nt=%d blocks=%5d  %8.3f ms  %7.0f GB/s\n", name, U, (int)NT, blocks, ms,
           n4 * bytes_per_f4 / (ms * 1e-3) / 1e9);
}

template <int U, bool NT>
void all(long long n4, f4* a, f4* b, f4* c, float* part, int blocks) {
    run<0, U, NT>("rd2wr1", n4, a, b, c, part, blocks, 48);
    run<1, U, NT>("rd2", n4, a, b, c, part, blocks, 32);
    run<2, U, NT>("rd1wr1", n4, a, b, c, part, blocks, 32);
    run<3, U, NT>("rd1", n4, a, b, c, part, blocks, 16);
    run<4, U, NT>("wr1", n4, a, b, c, part, blocks, 16);
}

int main() {
    const long long n4 = 4000000LL * 256 / 4;
    f4 *a, *b, *c;
    float* part;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMalloc(&c, n4 * 16));
    CK(hipMalloc(&part, 65536LL * 256 * 4));
    CK(hipMemset(a, 0, n4 * 16));
    CK(hipMemset(b, 0, n4 * 16));
    for (int blocks : {2048, 8192}) {
        all<4, false>(n4, a, b, c, part, blocks);
        all<8, false>(n4, a, b, c, part, blocks);
        all<4, true>(n4, a, b, c, part, blocks);
    }
    return 0;
}
