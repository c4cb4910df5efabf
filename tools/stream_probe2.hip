// Round-3 re-measurement of the box's HBM ceiling for the edge kernels' access mixes (VERDICT r02 item 5:
// round 2's probe, tools/stream_probe.hip, topped out at 5.3 TB/s for read+write mixes against the guide's
// 6.29 TB/s float4 copy).  Variables swept here, one at a time against a base:
//   order   grid-stride (G: consecutive workgroups on consecutive 16-KB chunks, round 2's form) or
//           block-contiguous (B: each workgroup owns one contiguous range), or XCD-contiguous (X: the
//           workgroups of one XCD (blockIdx % 8) own one contiguous eighth of the table)
//   U       independent 16-B loads in flight per lane (4, 8, 16)
//   policy  plain, nontemporal loads only, nontemporal loads and stores
//   threads 256 or 512 per workgroup, workgroups 1024 .. 8192
//   size    1 GiB tables (config-3 edge table) and 4 GiB
// plus hipMemcpyDeviceToDevice of the same bytes.  Bandwidth = bytes read + bytes written per second.
// build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe2.hip -o tools/stream_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

template <int P>
__device__ __forceinline__ f4 ld(const f4* p) {
    if constexpr (P >= 1) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int P>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if constexpr (P >= 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// MODE 0: c = a + b (rd2wr1), 1: c = a (rd1wr1), 2: sum a (rd1), 3: sum a*b (rd2)
template <int MODE, int U, int P, int ORDER, int NT>
__global__ __launch_bounds__(NT) void probe(long long n4, const f4* __restrict__ a, const f4* __restrict__ b,
                                            f4* __restrict__ c, float* __restrict__ part) {
    const long long step = (long long)NT * U;  // f4 per workgroup iteration
    long long begin, end, stride;
    if constexpr (ORDER == 0) {             // grid-stride
        begin = (long long)blockIdx.x * step;
        end = n4;
        stride = (long long)gridDim.x * step;
    } else if constexpr (ORDER == 1) {      // block-contiguous
        const long long per = (n4 + gridDim.x - 1) / gridDim.x;
        const long long per_al = (per + step - 1) / step * step;
        begin = (long long)blockIdx.x * per_al;
        end = begin + per_al < n4 ? begin + per_al : n4;
        stride = step;
    } else {                                // XCD-contiguous: workgroup b runs on XCD b % 8
        const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
        const long long per = (n4 + 7) / 8;
        const long long lo = (long long)xcd * per, hi = lo + per < n4 ? lo + per : n4;
        begin = lo + (long long)slot * step;
        end = hi;
        stride = (long long)nslot * step;
    }
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long i0 = begin + threadIdx.x; i0 < end; i0 += stride) {
        f4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + (long long)u * NT;
            if (i < end) {
                va[u] = ld<P>(a + i);
                if constexpr (MODE == 0 || MODE == 3) vb[u] = ld<P>(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + (long long)u * NT;
            if (i >= end) continue;
            if constexpr (MODE == 0) st<P>(c + i, va[u] + vb[u]);
            else if constexpr (MODE == 1) st<P>(c + i, va[u]);
            else if constexpr (MODE == 2) acc += va[u];
            else acc += va[u] * vb[u];
        }
    }
    if constexpr (MODE >= 2) part[blockIdx.x * NT + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

static const char* MODE_NAME[] = {"rd2wr1", "rd1wr1", "rd1", "rd2"};
static const int MODE_F4B[] = {48, 32, 16, 32};
static const char ORDER_NAME[] = {'G', 'B', 'X'};

template <int MODE, int U, int P, int ORDER, int NT>
void run(long long n4, f4* a, f4* b, f4* c, float* part, int blocks) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = probe<MODE, U, P, ORDER, NT>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), 0, 0, n4, a, b, c, part);
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), 0, 0, n4, a, b, c, part);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-7s order=%c U=%2d pol=%d thr=%d blocks=%5d size=%5.2f GiB  %8.3f ms  %6.0f GB/s\n", MODE_NAME[MODE],
           ORDER_NAME[ORDER], U, P, NT, blocks, n4 * 16.0 / (1 << 30), ms, n4 * (double)MODE_F4B[MODE] / (ms * 1e-3) / 1e9);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int MODE>
void sweep(long long n4, f4* a, f4* b, f4* c, float* part) {
    // base: round 2's best form, then one variable at a time
    run<MODE, 8, 0, 0, 256>(n4, a, b, c, part, 2048);
    run<MODE, 8, 0, 1, 256>(n4, a, b, c, part, 2048);
    run<MODE, 8, 0, 2, 256>(n4, a, b, c, part, 2048);
    run<MODE, 16, 0, 1, 256>(n4, a, b, c, part, 2048);
    run<MODE, 4, 0, 1, 256>(n4, a, b, c, part, 4096);
    run<MODE, 8, 1, 1, 256>(n4, a, b, c, part, 2048);
    run<MODE, 8, 2, 1, 256>(n4, a, b, c, part, 2048);
    run<MODE, 8, 0, 1, 512>(n4, a, b, c, part, 1024);
    run<MODE, 8, 0, 1, 512>(n4, a, b, c, part, 2048);
    run<MODE, 8, 0, 1, 256>(n4, a, b, c, part, 1024);
    run<MODE, 8, 0, 1, 256>(n4, a, b, c, part, 8192);
    run<MODE, 4, 0, 2, 512>(n4, a, b, c, part, 2048);
    run<MODE, 8, 1, 2, 256>(n4, a, b, c, part, 2048);
}

int main() {
    const long long big = 4LL << 30;  // bytes per table at the largest size
    f4 *a, *b, *c;
    float* part;
    CK(hipMalloc(&a, big));
    CK(hipMalloc(&b, big));
    CK(hipMalloc(&c, big));
    CK(hipMalloc(&part, 8192LL * 512 * 4));
    CK(hipMemset(a, 0, big));
    CK(hipMemset(b, 0, big));
    CK(hipMemset(c, 0, big));
    for (long long bytes : {4000000LL * 256 * 4, big}) {
        const long long n4 = bytes / 16;
        sweep<1>(n4, a, b, c, part);
        sweep<0>(n4, a, b, c, part);
        sweep<2>(n4, a, b, c, part);
        sweep<3>(n4, a, b, c, part);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipMemcpy(c, a, bytes, hipMemcpyDeviceToDevice));
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) CK(hipMemcpyAsync(c, a, bytes, hipMemcpyDeviceToDevice, 0));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("hipMemcpyDtoD size=%5.2f GiB  %8.3f ms  %6.0f GB/s (read + write)\n", bytes / double(1 << 30), ms,
               2.0 * bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    }
    return 0;
}
