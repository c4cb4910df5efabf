// libiddgcn_hip — negative sampling on the device, bit-exact to the reference's host recipe
// (prediction/utils1.py:646-655, generate_negative_samples_np):
//
//     np.random.seed(seed)
//     condition_mask  = np.random.randint(0, 2, size=heads.shape)
//     random_entities = np.random.randint(0, num_entities, size=heads.shape)
//     neg_heads = where(condition_mask == 0, heads, random_entities)
//     neg_tails = where(condition_mask == 1, tails, random_entities)
//
// numpy's legacy RandomState is MT19937 seeded by init_genrand, and its int64 randint over a range
// that fits 32 bits draws 32-bit words, masks them with the smallest all-ones mask >= (high-1-low)
// and rejects values above it (buffered_bounded_masked_uint32).  So the negatives are a pure function
// of the MT19937 word stream: the first M words give the condition bits (range 1: mask 1, never
// rejected), the following words the entities (masked rejection; num_entities == 1 draws no words).
//
// MT19937 is a recurrence: each block of 624 words is a "twist" of the previous block, and inside a
// twist word i >= 227 depends on the new word i - 227.  One workgroup holds the state in LDS and
// runs each twist as three dependent phases (227, 227, 170 lanes), tempering and storing the 624
// words between twists; the rejection compaction and the triple assembly are ordinary parallel
// passes (per-chunk counts, one scan, ordered scatter by wave ballots).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/iddgcn_sampling.h"

namespace {

constexpr int MT_N = 624, MT_M = 397, MT_NM = MT_N - MT_M;     // 227
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
constexpr int CHUNK = 1024;                                     // words per compaction chunk (one wave)

__device__ __forceinline__ uint32_t twist(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & UPPER) | (b & LOWER);
    return c ^ (y >> 1) ^ ((0u - (y & 1u)) & MATRIX_A);
}
__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// init_genrand (numpy mt19937_seed): key[0] = seed, key[i] = 1812433253 (key[i-1] ^ key[i-1] >> 30) + i
__global__ void mt_seed_kernel(uint32_t seed, uint32_t* __restrict__ state) {
    if (threadIdx.x != 0) return;
    uint32_t s = seed;
    for (int i = 0; i < MT_N; ++i) {
        state[i] = s;
        s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    state[MT_N] = MT_N;            // position: the first draw twists
}

// n tempered words of the stream continuing at state (key[624] + position), state advanced.
__global__ __launch_bounds__(1024) void mt_generate_kernel(uint32_t* __restrict__ state, long long n,
                                                           uint32_t* __restrict__ out) {
    __shared__ uint32_t S[2][MT_N];
    const int tid = threadIdx.x;
    if (tid < MT_N) S[0][tid] = state[tid];
    int pos = (int)state[MT_N];
    __syncthreads();
    int cur = 0;
    long long done = 0;
    {   // words left in the current block
        const long long left = MT_N - pos;
        const int take = (int)(n < left ? n : left);
        for (int i = tid; i < take; i += blockDim.x) out[i] = temper(S[cur][pos + i]);
        done = take;
        pos += take;
    }
    while (done < n) {
        const int nx = cur ^ 1;
        if (tid < MT_NM) S[nx][tid] = twist(S[cur][tid], S[cur][tid + 1], S[cur][tid + MT_M]);
        __syncthreads();
        if (tid < MT_NM) {
            const int i = MT_NM + tid;                                 // 227 .. 453
            S[nx][i] = twist(S[cur][i], S[cur][i + 1], S[nx][i - MT_NM]);
        }
        __syncthreads();
        if (tid < MT_N - 2 * MT_NM) {                                  // 454 .. 623
            const int i = 2 * MT_NM + tid;
            S[nx][i] = i < MT_N - 1 ? twist(S[cur][i], S[cur][i + 1], S[nx][i - MT_NM])
                                    : twist(S[cur][MT_N - 1], S[nx][0], S[nx][MT_M - 1]);
        }
        __syncthreads();
        cur = nx;
        const long long left = n - done;
        const int take = (int)(left < MT_N ? left : MT_N);
        for (int i = tid; i < take; i += blockDim.x) out[done + i] = temper(S[cur][i]);
        done += take;
        pos = take;
    }
    __syncthreads();
    if (tid < MT_N) state[tid] = S[cur][tid];
    if (tid == 0) state[MT_N] = (uint32_t)pos;
}

// accepted words (w & mask) <= rng per CHUNK-word chunk
__global__ __launch_bounds__(256) void accept_count_kernel(const uint32_t* __restrict__ w, long long n, uint32_t mask,
                                                           uint32_t rng, int* __restrict__ counts, long long n_chunks) {
    const long long c = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x & 63;
    if (c >= n_chunks) return;
    int cnt = 0;
    for (int k = 0; k < CHUNK; k += 64) {
        const long long i = c * CHUNK + k + lane;
        const bool ok = i < n && (w[i] & mask) <= rng;
        cnt += __popcll(__ballot(ok));
    }
    if (lane == 0) counts[c] = cnt;
}

// exclusive scan of the chunk counts (one workgroup), total in offs[n_chunks]
__global__ __launch_bounds__(1024) void chunk_scan_kernel(const int* __restrict__ counts, long long n_chunks,
                                                          long long* __restrict__ offs) {
    __shared__ long long part[1024];
    const int tid = threadIdx.x;
    const long long per = (n_chunks + 1023) / 1024;
    const long long b = tid * per, e = (b + per < n_chunks) ? b + per : n_chunks;
    long long s = 0;
    for (long long i = b; i < e; ++i) s += counts[i];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {                    // inclusive Hillis-Steele over 1024 partials
        const long long v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    long long run = tid > 0 ? part[tid - 1] : 0;
    for (long long i = b; i < e; ++i) {
        offs[i] = run;
        run += counts[i];
    }
    if (tid == 1023) offs[n_chunks] = part[1023];
}

// the k-th accepted word (k < M), in stream order, as the entity of negative k
__global__ __launch_bounds__(256) void accept_scatter_kernel(const uint32_t* __restrict__ w, long long n, uint32_t mask,
                                                             uint32_t rng, const long long* __restrict__ offs,
                                                             long long n_chunks, long long M,
                                                             int* __restrict__ ent) {
    const long long c = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x & 63;
    if (c >= n_chunks) return;
    long long base = offs[c];
    if (base >= M) return;
    for (int k = 0; k < CHUNK; k += 64) {
        const long long i = c * CHUNK + k + lane;
        const uint32_t v = i < n ? (w[i] & mask) : 0u;
        const bool ok = i < n && v <= rng;
        const unsigned long long bal = __ballot(ok);
        const long long pos = base + __popcll(bal & ((1ull << lane) - 1ull));
        if (ok && pos < M) ent[pos] = (int)v;
        base += __popcll(bal);
    }
}

// neg_h = cond == 0 ? h : ent, neg_t = cond == 1 ? t : ent; relation copied
__global__ __launch_bounds__(256) void negatives_kernel(long long M, const long long* __restrict__ tri,
                                                        const uint32_t* __restrict__ cond_words,
                                                        const int* __restrict__ ent, long long* __restrict__ out) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const uint32_t c = cond_words[k] & 1u;
    const long long e = ent ? (long long)ent[k] : 0;
    out[3 * k + 0] = c == 0 ? tri[3 * k + 0] : e;
    out[3 * k + 1] = tri[3 * k + 1];
    out[3 * k + 2] = c == 1 ? tri[3 * k + 2] : e;
}

inline int st(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }
inline int last() { return st(hipGetLastError()); }

}  // namespace

extern "C" {

uint32_t iddgcn_randint_mask(uint32_t rng) {
    uint32_t m = rng;
    m |= m >> 1;
    m |= m >> 2;
    m |= m >> 4;
    m |= m >> 8;
    m |= m >> 16;
    return m;
}

int iddgcn_mt19937_seed(void* stream, uint32_t seed, uint32_t* state) {
    if (!state) return IDDGCN_SMP_E_ARG;
    hipLaunchKernelGGL(mt_seed_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed, state);
    return last();
}

int iddgcn_mt19937_generate(void* stream, uint32_t* state, long long n, uint32_t* out) {
    if (!state || n < 0 || (n > 0 && !out)) return IDDGCN_SMP_E_ARG;
    if (n == 0) return 0;
    hipLaunchKernelGGL(mt_generate_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, state, n, out);
    return last();
}

long long iddgcn_accept_chunks(long long n_words) { return (n_words + CHUNK - 1) / CHUNK; }

int iddgcn_masked_accept(void* stream, const uint32_t* words, long long n_words, uint32_t rng, long long M,
                         int* counts, long long* offs, int* ent) {
    if (n_words < 0 || M < 0 || (n_words > 0 && (!words || !counts || !offs || !ent))) return IDDGCN_SMP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    const long long nc = iddgcn_accept_chunks(n_words);
    if (nc == 0) {
        if (offs) (void)hipMemsetAsync(offs, 0, sizeof(long long), s);
        return last();
    }
    const uint32_t mask = iddgcn_randint_mask(rng);
    const unsigned grid = (unsigned)((nc * 64 + 255) / 256);
    hipLaunchKernelGGL(accept_count_kernel, dim3(grid), dim3(256), 0, s, words, n_words, mask, rng, counts, nc);
    hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(1024), 0, s, counts, nc, offs);
    hipLaunchKernelGGL(accept_scatter_kernel, dim3(grid), dim3(256), 0, s, words, n_words, mask, rng, offs, nc, M, ent);
    return last();
}

int iddgcn_assemble_negatives(void* stream, long long M, const long long* triples, const uint32_t* cond_words,
                              const int* ent, long long* out) {
    if (M < 0 || (M > 0 && (!triples || !cond_words || !out))) return IDDGCN_SMP_E_ARG;
    if (M == 0) return 0;
    hipLaunchKernelGGL(negatives_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, (hipStream_t)stream, M,
                       triples, cond_words, ent, out);
    return last();
}

}  // extern "C"
