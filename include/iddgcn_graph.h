/*
 * iddgcn_graph.h — device graph build of libiddgcn_hip.so.
 *
 * The reference builds the per-relation adjacency on the host with np.unique + tf.sparse.reorder
 * (utils1.py:415-451) and Keras feeds the scored triples as given (IDDGCN.py:399-407).  This
 * module builds, on the GPU and bit-identical to the host build in iddgcn_amd/graph.py:
 *   - every A_r as CSR in (row, col) sorted-unique order (the reference's edge order), with the
 *     (0,0)=0.0 placeholder of an empty relation (utils1.py:427-429), plus the merged CSR of
 *     all A_r^T the backward walks;
 *   - the scored triples laid out tail-sorted (stable) with the head-sorted permutation and the
 *     inverse permutation back to the caller's order.
 * Both are built from LSD radix sorts (8-bit digits, stable) whose passes are one
 * histogram, one per-digit scan and one LDS-staged scatter each; no float arithmetic, no
 * atomics whose order could show in the result, so the output is a pure function of the input.
 *
 * Conventions as in iddgcn.h: device pointers, caller-owned outputs and workspace (size from
 * the *_workspace query, a pure host function), `stream` = hipStream_t as void*, return 0 / a
 * positive hipError_t / a negative IDDGCN_E_* (nothing launched).  Nothing here synchronises:
 * counts and error flags are written to device memory for the caller to read.
 */
#ifndef IDDGCN_GRAPH_H_
#define IDDGCN_GRAPH_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Workspace bytes for iddgcn_radix_sort_pairs on n keys of key_bytes (4 or 8); < 0 if invalid. */
long long iddgcn_radix_sort_workspace(long long n, int key_bytes);

/* Stable LSD radix sort of n keys (uint32 if key_bytes == 4, uint64 if 8) on bits [0, end_bit).
 * vals_in == NULL with vals_out != NULL sorts the identity permutation (argsort, stable);
 * vals_out == NULL sorts keys only.  keys_in/vals_in are not modified and must not alias the
 * outputs.  n < 2^31.  The primitive under np.unique / np.lexsort / np.argsort(kind="stable")
 * of utils1.py:416,436 and graph.py. */
int iddgcn_radix_sort_pairs(void* stream, long long n, int key_bytes, int end_bit,
                            const void* keys_in, const unsigned* vals_in,
                            void* keys_out, unsigned* vals_out,
                            void* workspace, long long workspace_bytes);

/* Workspace bytes for iddgcn_build_adjacency; < 0 if the sizes are out of range. */
long long iddgcn_adjacency_workspace(long long M, int N, int R);

/* utils1.get_adj_mats (utils1.py:420-451) + the CSR layouts of graph.DeviceAdjacency.
 * triples: (M, 3) int64 (obj, rel, sbj) rows, device memory; rows whose rel is outside [0, R)
 * are ignored (the reference selects data[:,1] == i for i < R).  Capacity C = M + R.
 *   fwd_ptr  [R*(N+1)]  per-relation row pointers, absolute offsets into fwd_col/fwd_val
 *   fwd_col  [C], fwd_val [C]     columns / values (1.0, or 0.0 for an empty relation's (0,0))
 *   bwd_ptr  [N+1], bwd_col [C]   merged CSR of [A_0^T | A_1^T | ...]: row c lists r*N + m for
 *                                 every (m, c) of A_r, relation-major then by m
 *   bwd_src  [C], bwd_val [C]     forward-CSR position of each backward entry / its value
 *   counts   [3] int              [nnz, placeholders, error]; error = 1 if an entity index of
 *                                 any row is outside [0, N) (get_adj_mats raises then)
 * Entries past nnz are unspecified.  Requires R*N < 2^31, 2*R*N*N < 2^63, M + R < 2^31. */
int iddgcn_build_adjacency(void* stream, long long M, int N, int R, const long long* triples,
                           int* fwd_ptr, int* fwd_col, float* fwd_val,
                           int* bwd_ptr, int* bwd_col, int* bwd_src, float* bwd_val,
                           int* counts, void* workspace, long long workspace_bytes);

/* Workspace bytes for iddgcn_build_scored_edges; < 0 if the sizes are out of range. */
long long iddgcn_scored_edges_workspace(long long T, int N);

/* graph.ScoredEdges: the T scored (h, r, t) triples (int64 (T, 3), device) sorted by tail
 * (stable), as int32 h/r/t [T]; labels (T floats, or NULL) gathered into y [T] (may be NULL then);
 * tptr [N+1] tail-segment pointers; hperm [T] the stable argsort of the sorted h; hptr [N+1] its
 * segment pointers; inv [T] int64 with inv[order[k]] = k.  err [1] int: 1 if an entity is outside
 * [0, N), 2 if a relation is outside [0, R) (ScoredEdges raises then).  T < 2^31. */
int iddgcn_build_scored_edges(void* stream, long long T, int N, int R, const long long* triples,
                              const float* labels, int* h, int* r, int* t, float* y,
                              int* tptr, int* hperm, int* hptr, long long* inv, int* err,
                              void* workspace, long long workspace_bytes);

#ifdef __cplusplus
}
#endif

#endif /* IDDGCN_GRAPH_H_ */
