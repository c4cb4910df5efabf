// graph_build.hip — device graph build for gfx950 (include/iddgcn_graph.h).
//
// Everything is integer work and HBM-bound.  The core is a stable LSD radix sort, 8-bit digits,
// in the reduce-then-scan form (three launches per pass):
//   hist    : per 4096-key tile, the 256-bin digit histogram -> hist[digit][tile]
//   scan    : one workgroup per digit scans its row of tiles (exclusive) and emits the digit total
//   scatter : per tile, the stable in-tile rank of every key (wave64 peer match: 8 ballots give
//             the lanes holding the same digit, v_mbcnt their order), an LDS reorder into digit
//             runs, then runs written out contiguously at digit_base + hist[digit][tile].
// A tile is 512 threads = 8 waves; wave w owns the 512 consecutive keys [w*512, w*512+512) of
// the tile and walks them in 8 rounds of 64, so "earlier round, or same round and lower lane"
// is exactly "earlier in the input": the rank, hence the sort, is stable.
//
// The graph builders compose the sort with small gather / compact / pointer kernels.  CSR row
// pointers come from a lower_bound per pointer entry (uniform work however skewed the degrees).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "iddgcn.h"
#include "iddgcn_graph.h"

namespace gb {

constexpr int RB = 8;                        // digit bits
constexpr int RADIX = 1 << RB;
constexpr int NT = 512;                      // threads per tile
constexpr int NW = NT / 64;                  // waves per tile
constexpr int IPT = 8;                       // keys per thread
constexpr int TILE = NT * IPT;               // 4096 keys per tile
constexpr int WAVE_KEYS = 64 * IPT;          // consecutive keys one wave owns

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63; }

// number of lanes in `m` below this lane
__device__ __forceinline__ unsigned mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// lanes of this wave that are valid and hold the same digit as this lane (0 for invalid lanes);
// digits have `nb` (<= RB) bits
__device__ __forceinline__ uint64_t peers_of(unsigned d, bool valid, int nb) {
    uint64_t m = __ballot(valid);
    for (int b = 0; b < nb; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return valid ? m : 0ull;
}

__device__ __forceinline__ unsigned wave_incl_scan(unsigned x) {
    const unsigned lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o, 64);
        if (lane >= (unsigned)o) x += y;
    }
    return x;
}

// XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8), so give XCD x
// one contiguous range of tiles.  Consecutive tiles of one XCD then write adjacent hist entries and
// adjacent digit runs, and the partial lines at run boundaries merge in that XCD's L2 instead of
// being written from two XCDs.
__device__ __forceinline__ int tile_index(int ntiles) {
    const int b = blockIdx.x, x = b & 7;
    int start = 0;
    for (int y = 0; y < x; ++y) start += (ntiles - y + 7) >> 3;
    return start + (b >> 3);
}

template <typename K>
__device__ __forceinline__ unsigned digit_of(K k, int shift, unsigned mask) {
    return (unsigned)(k >> shift) & mask;
}

// ---- pass kernel 1: per-tile digit histogram -> hist[d * ntiles + tile] ------------------------
template <typename K>
__global__ __launch_bounds__(NT) void radix_hist_kernel(const K* __restrict__ keys, long long n, int shift,
                                                        unsigned mask, unsigned* __restrict__ hist, int ntiles) {
    __shared__ unsigned wcnt[NW][RADIX];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < NW * RADIX; i += NT) (&wcnt[0][0])[i] = 0;
    const int tile = tile_index(ntiles);
    const long long base = (long long)tile * TILE + wave * WAVE_KEYS + lane;
    K k[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + j * 64;
        k[j] = i < n ? keys[i] : (K)0;
    }
    __syncthreads();
    // wave-private bins, LDS integer atomics (no return value): the counts do not depend on the order
#pragma unroll
    for (int j = 0; j < IPT; ++j)
        if (base + j * 64 < n) atomicAdd(&wcnt[wave][digit_of(k[j], shift, mask)], 1u);
    __syncthreads();
    if (tid < RADIX) {
        unsigned s = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) s += wcnt[w][tid];
        hist[(size_t)tid * ntiles + tile] = s;
    }
}

// ---- pass kernel 2 (and the compaction scan): exclusive scan of each row of `data` in place ----
// One 1024-thread workgroup per row; row_total[row] = the row's sum (row_total may be NULL).
__global__ __launch_bounds__(1024) void scan_rows_kernel(unsigned* __restrict__ data, int ncols,
                                                         unsigned* __restrict__ row_total) {
    __shared__ unsigned wsum[16];
    __shared__ unsigned carry;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    unsigned* row = data + (size_t)blockIdx.x * ncols;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < ncols; c0 += 1024) {
        const int c = c0 + tid;
        const unsigned x = c < ncols ? row[c] : 0u;
        const unsigned incl = wave_incl_scan(x);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        unsigned pre = carry;
        for (int w = 0; w < wave; ++w) pre += wsum[w];
        if (c < ncols) row[c] = pre + incl - x;
        __syncthreads();
        if (tid == 1023) carry = pre + incl;
        __syncthreads();
    }
    if (tid == 0 && row_total) row_total[blockIdx.x] = carry;
}

// ---- pass kernel 3: stable in-tile rank, LDS reorder, run-contiguous scatter --------------------
// VMODE: 0 keys only, 1 values loaded from vin, 2 values = input position (argsort)
template <typename K, int VMODE>
__global__ __launch_bounds__(NT) void radix_scatter_kernel(const K* __restrict__ kin, const unsigned* __restrict__ vin,
                                                           K* __restrict__ kout, unsigned* __restrict__ vout,
                                                           long long n, int shift, unsigned mask, int nbits,
                                                           const unsigned* __restrict__ hist,
                                                           const unsigned* __restrict__ dtotal, int ntiles) {
    __shared__ K skey[TILE];
    __shared__ unsigned sval[VMODE ? TILE : 1];
    __shared__ unsigned wcnt[NW][RADIX];
    __shared__ unsigned dstart[RADIX];
    __shared__ unsigned gbase[RADIX];
    __shared__ unsigned part[2][RADIX / 64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tile = tile_index(ntiles);
    const long long tile0 = (long long)tile * TILE;
    const long long base = tile0 + wave * WAVE_KEYS + lane;
    for (int i = tid; i < NW * RADIX; i += NT) (&wcnt[0][0])[i] = 0;
    K k[IPT];
    unsigned v[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + j * 64;
        k[j] = i < n ? kin[i] : (K)0;
        if (VMODE == 1) v[j] = i < n ? vin[i] : 0u;
        if (VMODE == 2) v[j] = (unsigned)i;
    }
    __syncthreads();
    unsigned rk[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const bool ok = base + j * 64 < n;
        const unsigned d = digit_of(k[j], shift, mask);
        const uint64_t p = peers_of(d, ok, nbits);
        const unsigned below = mbcnt(p);
        unsigned before = 0;
        if (ok) before = wcnt[wave][d];
        // all lanes of the group read before the group's highest lane writes: ds ops of one wave
        // execute in issue order
        if (ok && below + 1 == (unsigned)__popcll(p)) wcnt[wave][d] = before + below + 1;
        rk[j] = before + below;
    }
    __syncthreads();
    unsigned tc = 0, dt = 0, a = 0, b = 0;
    if (tid < RADIX) {
        unsigned s = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const unsigned c = wcnt[w][tid];
            wcnt[w][tid] = s;
            s += c;
        }
        tc = s;
        dt = dtotal[tid];
        a = wave_incl_scan(tc);
        b = wave_incl_scan(dt);
        if (lane == 63) {
            part[0][wave] = a;
            part[1][wave] = b;
        }
    }
    __syncthreads();
    if (tid < RADIX) {
        unsigned pa = 0, pb = 0;
        for (int w = 0; w < wave; ++w) {
            pa += part[0][w];
            pb += part[1][w];
        }
        const unsigned ds = pa + a - tc;                 // this tile's first slot of digit tid
        const unsigned db = pb + b - dt;                 // global first slot of digit tid
        dstart[tid] = ds;
        gbase[tid] = db + hist[(size_t)tid * ntiles + tile] - ds;   // mod 2^32; n < 2^31
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (base + j * 64 < n) {
            const unsigned d = digit_of(k[j], shift, mask);
            const unsigned pos = dstart[d] + wcnt[wave][d] + rk[j];
            skey[pos] = k[j];
            if (VMODE) sval[pos] = v[j];
        }
    }
    __syncthreads();
    const int tile_n = (int)((n - tile0) < TILE ? (n - tile0) : TILE);
    for (int p = tid; p < tile_n; p += NT) {
        const K kk = skey[p];
        const unsigned g = gbase[digit_of(kk, shift, mask)] + (unsigned)p;
        kout[g] = kk;
        if (VMODE) vout[g] = sval[p];
    }
}

__global__ void iota_u32_kernel(unsigned* __restrict__ out, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (unsigned)i;
}

// ---- graph kernels ----------------------------------------------------------------------------
// Adjacency key of triple (h, r, t): ((r*N + h)*N + t)*2 + 1; the placeholder of relation r is
// (r*N*N)*2 (sorts just before a real (r,0,0)); ignored rows get the sentinel (R*N*N)*2.
__global__ void adj_keys_kernel(const long long* __restrict__ tr, long long M, int N, int R,
                                uint64_t* __restrict__ keys, int* __restrict__ err) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t NN = (uint64_t)N * (uint64_t)N;
    if (i < M) {
        const long long h = tr[3 * i], r = tr[3 * i + 1], t = tr[3 * i + 2];
        const bool ent = h >= 0 && h < N && t >= 0 && t < N;
        if (!ent) atomicOr(err, 1);
        keys[i] = (ent && r >= 0 && r < R)
                      ? ((((uint64_t)r * (uint64_t)N + (uint64_t)h) * (uint64_t)N + (uint64_t)t) << 1) | 1ull
                      : ((uint64_t)R * NN) << 1;
    } else if (i < M + R) {
        keys[i] = ((uint64_t)(i - M) * NN) << 1;
    }
}

// keep a sorted key: the first copy of a real edge; a placeholder only if its relation has no
// real edge (the next key is already in another relation); never the sentinel
__device__ __forceinline__ bool adj_keep(const uint64_t* __restrict__ K, long long i, long long n, uint64_t k,
                                         uint64_t sentinel, uint64_t NN) {
    if (k >= sentinel) return false;
    if (k & 1ull) return i == 0 || K[i - 1] != k;
    return i + 1 == n || (K[i + 1] >> 1) >= (k >> 1) + NN;
}

__global__ __launch_bounds__(NT) void adj_count_kernel(const uint64_t* __restrict__ K, long long n, uint64_t sentinel,
                                                       uint64_t NN, unsigned* __restrict__ tile_cnt) {
    __shared__ unsigned wc[NW];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long long base = (long long)blockIdx.x * TILE + wave * WAVE_KEYS + lane;
    unsigned c = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + j * 64;
        const bool keep = i < n && adj_keep(K, i, n, K[i], sentinel, NN);
        c += (unsigned)__popcll(__ballot(keep));
    }
    if (lane == 0) wc[wave] = c;
    __syncthreads();
    if (tid == 0) {
        unsigned s = 0;
        for (int w = 0; w < NW; ++w) s += wc[w];
        tile_cnt[blockIdx.x] = s;
    }
}

// compaction in sorted order: forward CSR entries + the backward sort keys (the column)
__global__ __launch_bounds__(NT) void adj_compact_kernel(const uint64_t* __restrict__ K, long long n, uint64_t sentinel,
                                                         uint64_t NN, int N, const unsigned* __restrict__ tile_off,
                                                         int* __restrict__ fwd_seg, int* __restrict__ fwd_col,
                                                         float* __restrict__ fwd_val, unsigned* __restrict__ bkey,
                                                         int* __restrict__ counts) {
    __shared__ unsigned wc[NW];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long long base = (long long)blockIdx.x * TILE + wave * WAVE_KEYS + lane;
    uint64_t k[IPT];
    bool keep[IPT];
    unsigned c = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + j * 64;
        k[j] = i < n ? K[i] : 0ull;
        keep[j] = i < n && adj_keep(K, i, n, k[j], sentinel, NN);
        c += (unsigned)__popcll(__ballot(keep[j]));
    }
    if (lane == 0) wc[wave] = c;
    __syncthreads();
    unsigned off = tile_off[blockIdx.x];
    for (int w = 0; w < wave; ++w) off += wc[w];
    unsigned ph = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t b = __ballot(keep[j]);
        if (keep[j]) {
            const unsigned o = off + mbcnt(b);
            const uint64_t x = k[j] >> 1;              // r*N*N + h*N + t
            const uint64_t seg = x / (uint64_t)N;      // r*N + h
            const int col = (int)(x - seg * (uint64_t)N);
            fwd_seg[o] = (int)seg;
            fwd_col[o] = col;
            const bool real = k[j] & 1ull;
            fwd_val[o] = real ? 1.0f : 0.0f;
            bkey[o] = (unsigned)col;
            ph += real ? 0u : 1u;
        }
        off += (unsigned)__popcll(b);
    }
    if (ph) atomicAdd(&counts[1], (int)ph);            // an integer count: order-independent
}

// ptr[r*(n_rows+1) + i] = lower_bound(seg[0:n), r*n_rows + i)   for r < n_rel, i <= n_rows
template <typename S>
__global__ void csr_ptr_kernel(const S* __restrict__ seg, const int* __restrict__ n_dev, long long n_host, int n_rel,
                               int n_rows, int* __restrict__ ptr) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (long long)n_rel * (n_rows + 1)) return;
    const long long n = n_dev ? (long long)*n_dev : n_host;
    const long long r = j / (n_rows + 1);
    const long long target = j - r;
    long long lo = 0, hi = n;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if ((long long)seg[mid] < target) lo = mid + 1;
        else hi = mid;
    }
    ptr[j] = (int)lo;
}

__global__ void adj_bwd_gather_kernel(const unsigned* __restrict__ bsrc, const int* __restrict__ fwd_seg,
                                      const float* __restrict__ fwd_val, const int* __restrict__ nnz,
                                      int* __restrict__ bwd_col, float* __restrict__ bwd_val) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= *nnz) return;
    const unsigned s = bsrc[k];
    bwd_col[k] = fwd_seg[s];
    bwd_val[k] = fwd_val[s];
}

__global__ void edges_keys_kernel(const long long* __restrict__ tr, long long T, int N, int R,
                                  unsigned* __restrict__ tkey, int* __restrict__ err) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T) return;
    const long long h = tr[3 * i], r = tr[3 * i + 1], t = tr[3 * i + 2];
    if (h < 0 || h >= N || t < 0 || t >= N) atomicOr(err, 1);
    if (r < 0 || r >= R) atomicOr(err, 2);
    tkey[i] = (unsigned)t;
}

__global__ void edges_gather_kernel(const long long* __restrict__ tr, const float* __restrict__ labels,
                                    const unsigned* __restrict__ order, long long T, int* __restrict__ h,
                                    int* __restrict__ r, float* __restrict__ y, long long* __restrict__ inv,
                                    unsigned* __restrict__ hkey) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= T) return;
    const unsigned o = order[k];
    const int hh = (int)tr[3 * (long long)o];
    h[k] = hh;
    hkey[k] = (unsigned)hh;
    r[k] = (int)tr[3 * (long long)o + 1];
    if (labels) y[k] = labels[o];
    inv[o] = k;
}

// ---- host side --------------------------------------------------------------------------------
#define GB_CHECK(x)                              \
    do {                                         \
        const hipError_t e_ = (x);               \
        if (e_ != hipSuccess) return (int)e_;    \
    } while (0)

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
inline long long ntiles_of(long long n) { return (n + TILE - 1) / TILE; }
inline unsigned grid1(long long n, int b) { return (unsigned)((n + b - 1) / b); }

inline int bit_length(uint64_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

long long sort_ws(long long n, int kb) {
    const long long nt = ntiles_of(n);
    return (long long)(al((size_t)n * kb) + al((size_t)n * 4) + al((size_t)nt * RADIX * 4) + al(RADIX * 4));
}

template <typename K>
int radix_sort(hipStream_t st, long long n, int end_bit, const K* kin, const unsigned* vin, K* kout,
               unsigned* vout, char* ws) {
    if (n == 0) return 0;
    const long long nt = ntiles_of(n);
    K* kalt = (K*)ws;
    unsigned* valt = (unsigned*)(ws + al((size_t)n * sizeof(K)));
    unsigned* hist = (unsigned*)((char*)valt + al((size_t)n * 4));
    unsigned* dtot = (unsigned*)((char*)hist + al((size_t)nt * RADIX * 4));
    // as few passes as 8-bit digits need, with the digits as narrow as that allows: fewer buckets
    // mean longer digit runs per tile (fuller written lines) and fewer ballots per key
    const int passes = (end_bit + RB - 1) / RB;
    const int dbits = passes ? (end_bit + passes - 1) / passes : 0;
    if (passes == 0) {
        GB_CHECK(hipMemcpyAsync(kout, kin, (size_t)n * sizeof(K), hipMemcpyDeviceToDevice, st));
        if (vout) {
            if (vin) GB_CHECK(hipMemcpyAsync(vout, vin, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
            else hipLaunchKernelGGL(iota_u32_kernel, dim3(grid1(n, 256)), dim3(256), 0, st, vout, n);
        }
        return (int)hipGetLastError();
    }
    const K* ksrc = kin;
    const unsigned* vsrc = vin;
    for (int p = 0; p < passes; ++p) {
        const int shift = p * dbits;
        const int nb = end_bit - shift < dbits ? end_bit - shift : dbits;
        const unsigned mask = (1u << nb) - 1u;
        const bool last_dst = ((passes - 1 - p) & 1) == 0;
        K* kdst = last_dst ? kout : kalt;
        unsigned* vdst = last_dst ? vout : valt;
        hipLaunchKernelGGL(radix_hist_kernel<K>, dim3((unsigned)nt), dim3(NT), 0, st, ksrc, n, shift, mask, hist,
                           (int)nt);
        hipLaunchKernelGGL(scan_rows_kernel, dim3(RADIX), dim3(1024), 0, st, hist, (int)nt, dtot);
        if (!vout)
            hipLaunchKernelGGL((radix_scatter_kernel<K, 0>), dim3((unsigned)nt), dim3(NT), 0, st, ksrc, vsrc, kdst,
                               vdst, n, shift, mask, nb, hist, dtot, (int)nt);
        else if (p == 0 && !vin)
            hipLaunchKernelGGL((radix_scatter_kernel<K, 2>), dim3((unsigned)nt), dim3(NT), 0, st, ksrc, vsrc, kdst,
                               vdst, n, shift, mask, nb, hist, dtot, (int)nt);
        else
            hipLaunchKernelGGL((radix_scatter_kernel<K, 1>), dim3((unsigned)nt), dim3(NT), 0, st, ksrc, vsrc, kdst,
                               vdst, n, shift, mask, nb, hist, dtot, (int)nt);
        ksrc = kdst;
        vsrc = vdst;
    }
    return (int)hipGetLastError();
}

struct AdjWs {
    size_t keys, skeys, seg, bkey, bkey_s, tcnt, sort, total;
};

inline AdjWs adj_ws(long long M, int R) {
    const long long C = M + R;
    AdjWs w;
    size_t o = 0;
    w.keys = o;   o += al((size_t)C * 8);
    w.skeys = o;  o += al((size_t)C * 8);
    w.seg = o;    o += al((size_t)C * 4);
    w.bkey = o;   o += al((size_t)C * 4);
    w.bkey_s = o; o += al((size_t)C * 4);
    w.tcnt = o;   o += al((size_t)ntiles_of(C) * 4);
    w.sort = o;   o += (size_t)sort_ws(C, 8);          // >= the 4-byte sort's need
    w.total = o;
    return w;
}

inline bool adj_sizes_ok(long long M, int N, int R) {
    if (M < 0 || N < 1 || R < 1) return false;
    if ((long long)R * N >= (1ll << 31) || M + R >= (1ll << 31)) return false;
    return bit_length(((uint64_t)R * (uint64_t)N * (uint64_t)N) << 1) <= 63 &&
           (uint64_t)R * (uint64_t)N <= (1ull << 62) / ((uint64_t)N);
}

struct EdgeWs {
    size_t tkey, hkey, hks, order, sort, total;
};

inline EdgeWs edge_ws(long long T) {
    EdgeWs w;
    size_t o = 0;
    w.tkey = o;  o += al((size_t)T * 4);
    w.hkey = o;  o += al((size_t)T * 4);
    w.hks = o;   o += al((size_t)T * 4);
    w.order = o; o += al((size_t)T * 4);
    w.sort = o;  o += (size_t)sort_ws(T, 4);
    w.total = o;
    return w;
}

}  // namespace gb

extern "C" {

long long iddgcn_radix_sort_workspace(long long n, int key_bytes) {
    if (n < 0 || n >= (1ll << 31) || (key_bytes != 4 && key_bytes != 8)) return IDDGCN_E_BAD_ARG;
    return gb::sort_ws(n, key_bytes);
}

int iddgcn_radix_sort_pairs(void* stream, long long n, int key_bytes, int end_bit, const void* keys_in,
                            const unsigned* vals_in, void* keys_out, unsigned* vals_out, void* workspace,
                            long long workspace_bytes) {
    const long long need = iddgcn_radix_sort_workspace(n, key_bytes);
    if (need < 0 || end_bit < 0 || end_bit > 8 * key_bytes) return IDDGCN_E_BAD_ARG;
    if (n > 0 && (!keys_in || !keys_out || !workspace || workspace_bytes < need)) return IDDGCN_E_BAD_ARG;
    if (vals_in && !vals_out) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (key_bytes == 8)
        return gb::radix_sort<uint64_t>(st, n, end_bit, (const uint64_t*)keys_in, vals_in, (uint64_t*)keys_out,
                                        vals_out, (char*)workspace);
    return gb::radix_sort<unsigned>(st, n, end_bit, (const unsigned*)keys_in, vals_in, (unsigned*)keys_out, vals_out,
                                    (char*)workspace);
}

long long iddgcn_adjacency_workspace(long long M, int N, int R) {
    if (!gb::adj_sizes_ok(M, N, R)) return IDDGCN_E_BAD_ARG;
    return (long long)gb::adj_ws(M, R).total;
}

int iddgcn_build_adjacency(void* stream, long long M, int N, int R, const long long* triples, int* fwd_ptr,
                           int* fwd_col, float* fwd_val, int* bwd_ptr, int* bwd_col, int* bwd_src, float* bwd_val,
                           int* counts, void* workspace, long long workspace_bytes) {
    using namespace gb;
    const long long need = iddgcn_adjacency_workspace(M, N, R);
    if (need < 0) return IDDGCN_E_BAD_ARG;
    if ((M > 0 && !triples) || !fwd_ptr || !fwd_col || !fwd_val || !bwd_ptr || !bwd_col || !bwd_src || !bwd_val ||
        !counts || !workspace || workspace_bytes < need)
        return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const AdjWs w = adj_ws(M, R);
    char* ws = (char*)workspace;
    uint64_t* keys = (uint64_t*)(ws + w.keys);
    uint64_t* skeys = (uint64_t*)(ws + w.skeys);
    int* seg = (int*)(ws + w.seg);
    unsigned* bkey = (unsigned*)(ws + w.bkey);
    unsigned* bkey_s = (unsigned*)(ws + w.bkey_s);
    unsigned* tcnt = (unsigned*)(ws + w.tcnt);
    const long long C = M + R;
    const uint64_t NN = (uint64_t)N * (uint64_t)N;
    const uint64_t sentinel = ((uint64_t)R * NN) << 1;
    GB_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(int), st));
    GB_CHECK(hipMemsetD32Async((hipDeviceptr_t)bkey, (int)N, (size_t)C, st));   // slots past nnz sort last
    hipLaunchKernelGGL(adj_keys_kernel, dim3(grid1(C, 256)), dim3(256), 0, st, triples, M, N, R, keys, counts + 2);
    int rc = radix_sort<uint64_t>(st, C, bit_length(sentinel), keys, nullptr, skeys, nullptr, ws + w.sort);
    if (rc) return rc;
    const long long nt = ntiles_of(C);
    hipLaunchKernelGGL(adj_count_kernel, dim3((unsigned)nt), dim3(NT), 0, st, skeys, C, sentinel, NN, tcnt);
    hipLaunchKernelGGL(scan_rows_kernel, dim3(1), dim3(1024), 0, st, tcnt, (int)nt, (unsigned*)counts);
    hipLaunchKernelGGL(adj_compact_kernel, dim3((unsigned)nt), dim3(NT), 0, st, skeys, C, sentinel, NN, N, tcnt, seg,
                       fwd_col, fwd_val, bkey, counts);
    hipLaunchKernelGGL(csr_ptr_kernel<int>, dim3(grid1((long long)R * (N + 1), 256)), dim3(256), 0, st, seg,
                       counts, 0ll, R, N, fwd_ptr);
    // backward: the compacted entries are (r, m, c)-sorted, so a stable sort on c alone yields
    // (c, r, m) order = the merged CSR of the A_r^T
    rc = radix_sort<unsigned>(st, C, bit_length((uint64_t)N), bkey, nullptr, bkey_s, (unsigned*)bwd_src,
                              ws + w.sort);
    if (rc) return rc;
    hipLaunchKernelGGL(adj_bwd_gather_kernel, dim3(grid1(C, 256)), dim3(256), 0, st, (const unsigned*)bwd_src, seg,
                       fwd_val, counts, bwd_col, bwd_val);
    hipLaunchKernelGGL(csr_ptr_kernel<unsigned>, dim3(grid1((long long)N + 1, 256)), dim3(256), 0, st, bkey_s, counts,
                       0ll, 1, N, bwd_ptr);
    return (int)hipGetLastError();
}

long long iddgcn_scored_edges_workspace(long long T, int N) {
    if (T < 0 || T >= (1ll << 31) || N < 1) return IDDGCN_E_BAD_ARG;
    return (long long)gb::edge_ws(T).total;
}

int iddgcn_build_scored_edges(void* stream, long long T, int N, int R, const long long* triples, const float* labels,
                              int* h, int* r, int* t, float* y, int* tptr, int* hperm, int* hptr, long long* inv,
                              int* err, void* workspace, long long workspace_bytes) {
    using namespace gb;
    const long long need = iddgcn_scored_edges_workspace(T, N);
    if (need < 0 || R < 1) return IDDGCN_E_BAD_ARG;
    if ((T > 0 && (!triples || !h || !r || !t || !hperm || !inv)) || (labels && !y) || !tptr || !hptr || !err ||
        !workspace || workspace_bytes < need)
        return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const EdgeWs w = edge_ws(T);
    char* ws = (char*)workspace;
    unsigned* tkey = (unsigned*)(ws + w.tkey);
    unsigned* hkey = (unsigned*)(ws + w.hkey);
    unsigned* hks = (unsigned*)(ws + w.hks);
    unsigned* order = (unsigned*)(ws + w.order);
    const int eb = bit_length((uint64_t)(N - 1));
    GB_CHECK(hipMemsetAsync(err, 0, sizeof(int), st));
    if (T > 0) {
        hipLaunchKernelGGL(edges_keys_kernel, dim3(grid1(T, 256)), dim3(256), 0, st, triples, T, N, R, tkey, err);
        int rc = radix_sort<unsigned>(st, T, eb, tkey, nullptr, (unsigned*)t, order, ws + w.sort);
        if (rc) return rc;
        hipLaunchKernelGGL(edges_gather_kernel, dim3(grid1(T, 256)), dim3(256), 0, st, triples, labels, order, T, h, r,
                           y, inv, hkey);
        rc = radix_sort<unsigned>(st, T, eb, hkey, nullptr, hks, (unsigned*)hperm, ws + w.sort);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(csr_ptr_kernel<int>, dim3(grid1((long long)N + 1, 256)), dim3(256), 0, st, (const int*)t,
                       (const int*)nullptr, T, 1, N, tptr);
    hipLaunchKernelGGL(csr_ptr_kernel<unsigned>, dim3(grid1((long long)N + 1, 256)), dim3(256), 0, st,
                       (const unsigned*)hks, (const int*)nullptr, T, 1, N, hptr);
    return (int)hipGetLastError();
}

}  // extern "C"
