// C ABI of the host-side data pipeline: raw sequence files → the per-sequence index
// tensors of the training / evaluation batches and the transition-graph edges, bit-exact with the
// reference's Python (including its consumption of CPython's `random` MT19937 stream), as a CPU
// library (c2dsr_amd/libc2dsr_prep.so, built with g++ -O3 from c2dsr_amd/csrc_host/prep.cpp).
//
// Plain pointers and sizes; return 0 on success, a negative code on error (c2dsr_prep_error() gives
// the message).  The MT19937 state is CPython's `random.getstate()[1]`: 624 state words followed by
// the position index; the functions advance it exactly as the reference's draws would, so the caller
// writes it back with random.setstate() and later Python draws continue the same stream.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Parse a raw `{mode}_new.txt` (user \t id \t item|ts|... per line; items stable-sorted by ts).
// Replaces dataloader.py:39-58 (read_raw) and utils/graph.py:36-47.  Returns a handle or NULL.
void* c2dsr_prep_open(const char* path);
void c2dsr_prep_close(void* h);
// number of sequences and of items over all sequences
int c2dsr_prep_sizes(void* h, int64_t* n_seq, int64_t* n_items);
// items of every sequence: offsets [n_seq + 1], items [n_items]
int c2dsr_prep_sequences(void* h, int64_t* offsets, int64_t* items);

// dataloader.py:60-161 (preprocess_train): out [n_seq, 14, len_max] int64 (rows of dropped sequences
// are not emitted; *n_out = rows written).  Field order as the reference's 14 lists.
int c2dsr_prep_train(void* h, int n_a, int n_b, int len_max, uint32_t* mt_state, int64_t* out, int64_t* n_out);

// dataloader.py:163-228 (preprocess_evaluate): seqs [n_seq, 6, len_max], last [n_seq, 4]
// (idx_last_a, idx_last_b, xory_last, gt_last), neg [n_seq, n_neg] (random.sample order).
int c2dsr_prep_eval(void* h, int n_a, int n_b, int len_max, int n_neg, uint32_t* mt_state, int64_t* seqs,
                    int64_t* last, int64_t* neg);

// utils/graph.py:54-81: transition edges in the reference's emission order; share [n_items, 2] and
// specific [n_items, 2] buffers (upper bounds), *n_share / *n_spec = edges written.
int c2dsr_prep_edges(void* h, int n_a, int64_t* share, int64_t* n_share, int64_t* spec, int64_t* n_spec);

const char* c2dsr_prep_error(void);

#ifdef __cplusplus
}
#endif
