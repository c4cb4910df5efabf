/*
 * iddgcn_sampling.h — C-ABI of the device negative sampler in libiddgcn_hip.so.
 *
 * Replaces the host recipe prediction/utils1.py:646-655 (generate_negative_samples_np):
 *   np.random.seed(seed); cond = randint(0, 2, M); ent = randint(0, N, M);
 *   neg_h = cond == 0 ? h : ent;  neg_t = cond == 1 ? t : ent
 * bit-exactly: numpy's legacy RandomState stream (MT19937, init_genrand seeding, tempered 32-bit
 * words) and its int64 randint over a 32-bit range (smallest all-ones mask >= high-1-low, reject
 * above: buffered_bounded_masked_uint32).  The host wrapper (iddgcn_amd/ops.py negative_samples):
 *   1. iddgcn_mt19937_seed; iddgcn_mt19937_generate M words -> the condition bits;
 *   2. (N > 1) generate words, iddgcn_masked_accept (rng = N - 1) -> the first M accepted values;
 *      if offs[chunks] < M, generate more words after them (the state continues) and run again;
 *   3. iddgcn_assemble_negatives (ent = NULL when N == 1: randint(0, 1) draws no words, all 0).
 * Conventions as include/iddgcn.h: device pointers, caller-allocated, stream-ordered, int status.
 */
#ifndef IDDGCN_SAMPLING_H_
#define IDDGCN_SAMPLING_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IDDGCN_SMP_E_ARG (-3)

/* the mask numpy's masked rejection uses for an inclusive range [0, rng] */
uint32_t iddgcn_randint_mask(uint32_t rng);

/* state: 625 uint32 (624 key words + position), init_genrand(seed) (np.random.seed(seed)) */
int iddgcn_mt19937_seed(void* stream, uint32_t seed, uint32_t* state);

/* out[0..n): the next n tempered 32-bit words of the stream; the state advances by n */
int iddgcn_mt19937_generate(void* stream, uint32_t* state, long long n, uint32_t* out);

/* number of 1024-word chunks of a word array (sizes of counts / offs below) */
long long iddgcn_accept_chunks(long long n_words);

/* ent[k] = the k-th (k < M) accepted value (w & mask, kept when <= rng) of words[0..n_words), in stream
 * order.  counts: accept_chunks ints; offs: accept_chunks + 1 long longs, offs[accept_chunks] = the
 * number of accepted words (the caller reads it: < M means more words are needed). */
int iddgcn_masked_accept(void* stream, const uint32_t* words, long long n_words, uint32_t rng, long long M,
                         int* counts, long long* offs, int* ent);

/* out (M x 3 int64) from triples (M x 3 int64, obj/rel/sbj), the M condition words and ent (or NULL) */
int iddgcn_assemble_negatives(void* stream, long long M, const long long* triples, const uint32_t* cond_words,
                              const int* ent, long long* out);

#ifdef __cplusplus
}
#endif
#endif /* IDDGCN_SAMPLING_H_ */
