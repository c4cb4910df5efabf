// Instruction-level probe of the packed-fp32 op_sel hazard suspected in DESIGN.md §Determinism (round 3-4): the LOW
// lane of a v_pk_fma_f32 whose src1 op_sel selects the HIGH register of its pair (op_sel:[0,1,0], the form hipcc's SLP
// vectoriser emitted for acc[1] += w[1] * d in the tail reduction) returned the low register's value now and then,
// only while another kernel's waves shared the CUs.
//
// pk_probe: every lane runs `iters` steps of  acc.lo += x.lo * w.hi ; acc.hi += x.hi * w.hi  with ONE
// v_pk_fma_f32 ... op_sel:[0,1,0] (inline asm, so the library's no-packed-fp32 flag does not matter here), where the
// w pair is freshly loaded each step and moved through a v_mov_b64 (the producer pattern of the original code), and
// beside it the same sums with two scalar v_fma_f32 (also inline asm).  Every lane whose packed result differs bitwise
// from its scalar twin is counted (on the host).  The control runs it alone; the test runs it on one stream while a
// noise kernel (MFMA + LDS + HBM traffic, persistent) occupies the CUs from another stream.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/pkfma_probe tools/pkfma_probe.hip
// usage: tools/pkfma_probe [reps] [iters] [noise kind: all | mfma | lds | mem | valu]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(256) void pk_probe(const f2* __restrict__ W, const f2* __restrict__ X, long long n,
                                                int iters, f2* __restrict__ sink) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n) return;
    f2 acc = {0.f, 0.f};
    float r0 = 0.f, r1 = 0.f;
    for (int it = 0; it < iters; ++it) {
        const long long k = (gid + (long long)it * 977) & (n - 1);    // n: a power of two
        f2 wl = W[k];                 // the weight pair (w0, w1) of this step
        const f2 x = X[(k * 7) & (n - 1)];
        f2 w;
        asm volatile("v_mov_b64 %0, %1" : "=v"(w) : "v"(wl));
        // a few unrelated VALU ops between the producer and the packed FMA, as in the compiled loop
        float f = x[0];
        asm volatile("v_add_f32 %0, %0, 1.0\n\tv_mul_f32 %0, %0, 0.5" : "+v"(f));
        acc += f2{f, f} * 0.f;        // keeps f live without changing acc
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(x), "v"(w));
        float xl = x[0], xh = x[1], wh = w[1];
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r0) : "v"(xl), "v"(wh));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r1) : "v"(xh), "v"(wh));
    }
    // packed result and its scalar twin stored side by side; compared bitwise on the host (a device-side compare of
    // the asm outputs was folded wrongly by the compiler: it compared acc.lo with r1)
    sink[2 * gid] = acc;
    sink[2 * gid + 1] = f2{r0, r1};
}

// pk_probe2: as pk_probe, with the next step's w and x loads issued before the current step's packed FMA (software
// pipelined, so loads are in flight at the FMA, as in the compiled tail reduction where the next edge group was in
// flight) and the w pair moved by v_mov_b64 ~20 VALU instructions before its use
__global__ __launch_bounds__(256) void pk_probe2(const f2* __restrict__ W, const f2* __restrict__ X, long long n,
                                                 int iters, f2* __restrict__ sink) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n) return;
    f2 acc = {0.f, 0.f};
    float r0 = 0.f, r1 = 0.f;
    long long k = gid & (n - 1);
    f2 wn = W[k], xn = X[(k * 7) & (n - 1)];
    for (int it = 0; it < iters; ++it) {
        f2 w;
        asm volatile("v_mov_b64 %0, %1" : "=v"(w) : "v"(wn));
        const f2 x = xn;
        k = (gid + (long long)(it + 1) * 977) & (n - 1);
        wn = W[k];                    // next step's operands in flight during this step's packed FMA
        xn = X[(k * 7) & (n - 1)];
        float f = x[0];
        asm volatile("v_add_f32 %0, %0, 1.0\n\tv_mul_f32 %0, %0, 0.5\n\tv_add_f32 %0, %0, 1.0\n\tv_mul_f32 %0, %0, 0.5\n\t"
                     "v_add_f32 %0, %0, 1.0\n\tv_mul_f32 %0, %0, 0.5\n\tv_add_f32 %0, %0, 1.0\n\tv_mul_f32 %0, %0, 0.5"
                     : "+v"(f));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(x), "v"(w));
        float xl = x[0], xh = x[1], wh = w[1];
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r0) : "v"(xl), "v"(wh));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r1) : "v"(xh), "v"(wh));
        asm volatile("" :: "v"(f));
    }
    sink[2 * gid] = acc;
    sink[2 * gid + 1] = f2{r0, r1};
}

// noise: persistent MFMA + LDS + streaming-read work on another stream (bf16 MFMAs on LDS-staged random data)
__global__ __launch_bounds__(256) void noise(const f4* __restrict__ src, long long n4, int loops, f4* __restrict__ out) {
    __shared__ f4 tile[256 * 4];
    const int t = threadIdx.x;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < loops; ++l) {
        const long long base = ((long long)blockIdx.x * loops + l) * 1024 % (n4 - 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[t + 256 * j] = src[base + t + 256 * j];
        __syncthreads();
        const f4 a = tile[(t * 4 + l) & 1023];
        const bf8 av = __builtin_bit_cast(bf8, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, c, 0, 0, 0);
        s += a;
        __syncthreads();
    }
    out[(long long)blockIdx.x * 256 + t] = c + s;
}

// single-resource noise kernels (which co-running activity triggers the hazard): MFMA on registers only, LDS traffic only,
// HBM streaming only, plain VALU only
__global__ __launch_bounds__(256) void noise_mfma(int loops, f4* __restrict__ out) {
    f4 c = {0.f, 0.f, 0.f, 0.f};
    const float v = (float)threadIdx.x * 1e-3f;
    const bf8 a = __builtin_bit_cast(bf8, f4{v, v + 1.f, v + 2.f, v + 3.f});
    for (int l = 0; l < loops; ++l)
#pragma unroll
        for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c, 0, 0, 0);
    out[(long long)blockIdx.x * 256 + threadIdx.x] = c;
}
__global__ __launch_bounds__(256) void noise_lds(int loops, f4* __restrict__ out) {
    __shared__ f4 tile[1024];
    const int t = threadIdx.x;
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < loops; ++l) {
        tile[(t * 4 + l) & 1023] = s + 1.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) s += tile[(t + 256 * j + l) & 1023];
        __syncthreads();
    }
    out[(long long)blockIdx.x * 256 + t] = s;
}
__global__ __launch_bounds__(256) void noise_mem(const f4* __restrict__ src, long long n4, int loops, f4* __restrict__ out) {
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < loops; ++l) {
        const long long base = ((long long)blockIdx.x * loops + l) * 1024 % (n4 - 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) s += src[base + threadIdx.x + 256 * j];
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void noise_valu(int loops, f4* __restrict__ out) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int l = 0; l < loops * 64; ++l) a = fmaf(a, b, 1e-7f);
    out[(long long)blockIdx.x * 256 + threadIdx.x] = f4{a, a, a, a};
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const int iters = argc > 2 ? atoi(argv[2]) : 4096;
    const char* kind = argc > 3 ? argv[3] : "all";     // noise kernel: all | mfma | lds | mem | valu
    const long long n = 1 << 22;                  // 4M lanes per probe launch
    std::vector<f2> h(n);
    unsigned s = 12345u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xffff) / 65536.0f - 0.5f; };
    for (auto& v : h) v = f2{rnd(), rnd()};
    f2 *W, *X, *sink;
    CK(hipMalloc(&W, n * sizeof(f2)));
    CK(hipMalloc(&X, n * sizeof(f2)));
    CK(hipMalloc(&sink, 2 * n * sizeof(f2)));
    std::vector<f2> hs(2 * n);

    CK(hipMemcpy(W, h.data(), n * sizeof(f2), hipMemcpyHostToDevice));
    for (auto& v : h) v = f2{rnd(), rnd()};
    CK(hipMemcpy(X, h.data(), n * sizeof(f2), hipMemcpyHostToDevice));
    const long long n4 = 1ll << 26;               // 1 GiB of noise source
    f4 *src, *nout;
    CK(hipMalloc(&src, n4 * sizeof(f4)));
    CK(hipMemset(src, 0x3c, n4 * sizeof(f4)));
    CK(hipMalloc(&nout, 2048ll * 256 * sizeof(f4)));
    hipStream_t sa, sb;
    CK(hipStreamCreate(&sa));
    CK(hipStreamCreate(&sb));
    const unsigned grid = (unsigned)((n + 255) / 256);
    for (int phase = 0; phase < 4; ++phase) {     // probe (1, 2) x (alone, beside the noise kernel)
        const bool with_noise = phase & 1, v2 = phase >= 2;
        unsigned total = 0;
        for (int r = 0; r < reps; ++r) {
            if (with_noise) {
                if (!strcmp(kind, "mfma")) hipLaunchKernelGGL(noise_mfma, dim3(2048), dim3(256), 0, sb, 2048, nout);
                else if (!strcmp(kind, "lds")) hipLaunchKernelGGL(noise_lds, dim3(2048), dim3(256), 0, sb, 1024, nout);
                else if (!strcmp(kind, "mem")) hipLaunchKernelGGL(noise_mem, dim3(2048), dim3(256), 0, sb, src, n4, 512, nout);
                else if (!strcmp(kind, "valu")) hipLaunchKernelGGL(noise_valu, dim3(2048), dim3(256), 0, sb, 1024, nout);
                else hipLaunchKernelGGL(noise, dim3(2048), dim3(256), 0, sb, src, n4, 256, nout);
            }
            if (v2) hipLaunchKernelGGL(pk_probe2, dim3(grid), dim3(256), 0, sa, W, X, n, iters, sink);
            else hipLaunchKernelGGL(pk_probe, dim3(grid), dim3(256), 0, sa, W, X, n, iters, sink);
            CK(hipGetLastError());
            CK(hipMemcpyAsync(hs.data(), sink, 2 * n * sizeof(f2), hipMemcpyDeviceToHost, sa));
            CK(hipStreamSynchronize(sa));
            CK(hipStreamSynchronize(sb));
            unsigned m = 0;
            long long first = -1;
            for (long long i = 0; i < n; ++i) {
                const f2 a = hs[2 * i], b = hs[2 * i + 1];
                if (memcmp(&a, &b, sizeof(f2)) != 0) {
                    ++m;
                    if (first < 0) first = i;
                }
            }
            if (first >= 0)
                printf("  first differing lane %lld: packed %.9g %.9g, scalar %.9g %.9g\n", first, hs[2 * first][0],
                       hs[2 * first][1], hs[2 * first + 1][0], hs[2 * first + 1][1]);
            printf("probe%d %s rep %d: %u of %lld lanes differ\n", v2 ? 2 : 1, with_noise ? "with noise" : "alone", r, m, n);
            fflush(stdout);
            total += m;
        }
        printf("probe%d %s%s: %u mismatching lanes over %d reps x %lld lanes x %d packed FMAs each\n", v2 ? 2 : 1,
               with_noise ? "with noise " : "alone", with_noise ? kind : "", total, reps, n, iters);
    }
    return 0;
}
