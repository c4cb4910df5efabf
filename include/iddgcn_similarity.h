/*
 * iddgcn_similarity.h — feature-similarity graph construction of libiddgcn_hip.so
 * (SURVEY §8(f) row 4).
 *
 * Replaces prediction/feat_similarity.py:9-44: caculat_distance (sklearn cosine_similarity,
 * float64) -> creat_similar_mat (`mat > threshold`) -> simat2triple (i < j, row-major,
 * (i + start, relation, j + start)).  The dense N x N matrix is never materialised: the product
 * runs tile by tile on f32 MFMA, the threshold decision is exact against float64 (pairs whose f32
 * similarity lies within the f32 error band of the threshold are re-decided in float64), and the
 * accepted pairs come out as keys i*N + j to be radix-sorted (iddgcn_radix_sort_pairs) into the
 * reference's row-major order.
 *
 * Conventions as in iddgcn.h (device pointers, caller-owned buffers, no synchronisation).
 */
#ifndef IDDGCN_SIMILARITY_H_
#define IDDGCN_SIMILARITY_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Workspace bytes for iddgcn_similarity_pairs (normalised rows, f64 and padded f32); < 0 if
 * the sizes are invalid (N, F >= 1, N*N < 2^62). */
long long iddgcn_similarity_workspace(int N, int F);

/* X: (N, F) float64 row-major node features (feat_similarity.py:6-8, NaN rows already dropped).
 * Appends key i*N + j for every i < j with cosine(X_i, X_j) > threshold to keys[0:capacity), and
 * the f32-undecidable candidates to band[0:band_capacity) (scratch).  counts[2] (device, u64):
 * [accepted, band candidates]; when a count exceeds its capacity the keys past it were dropped
 * and the call must be repeated with larger buffers.  Keys are unordered (the set is exact). */
int iddgcn_similarity_pairs(void* stream, int N, int F, const double* X, double threshold,
                            unsigned long long* keys, long long capacity,
                            unsigned long long* band, long long band_capacity,
                            unsigned long long* counts, void* workspace, long long workspace_bytes);

/* triples[q] = (i + start, relation, j + start) for sorted_keys[q] = i*N + j, q < n_pairs,
 * as an (n_pairs, 3) int64 array (simat2triple, feat_similarity.py:37-47). */
int iddgcn_similarity_triples(void* stream, long long n_pairs, int N, int relation, long long start,
                              const unsigned long long* sorted_keys, long long* triples);

#ifdef __cplusplus
}
#endif

#endif /* IDDGCN_SIMILARITY_H_ */
