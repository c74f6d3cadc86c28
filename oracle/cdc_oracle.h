/* oracle/cdc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference ReMPI Clock Delta Compression (CDC) codec, written
 * from a written behaviour spec of the reference's CDC path and pinned against the
 * reference's own encoder/decoder (oracle/_ref/ref_cdc, built from the unmodified
 * sources by oracle/Makefile) and the committed golden fixtures in tests/golden/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline: the product path (rempi_amd, libcdcx)
 * never calls into it.
 */
#ifndef CDC_ORACLE_H
#define CDC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes (shared with include/cdcx.h). */
#define ORACLE_OK 0
#define ORACLE_ERR_ARG 1
#define ORACLE_ERR_TRUNCATED_EPOCH 2  /* a table's last event has with_next != 0 */
#define ORACLE_ERR_CLOCK_ORDER 3      /* a source's clock does not strictly increase */
#define ORACLE_ERR_CORRUPT 4          /* malformed record file */

/* Encode one rank's canonical record stream (n x 8 int32, rempi_event.h:40-48 layout,
 * already run-length merged as rempi_event_list::push leaves it) exactly as
 * rempi_io_thread::write_record + rempi_encoder_cdc would write rank_<r>.rempi:
 * chunks, the size_t 0 separator and the footer.  *out is malloc'ed. */
int oracle_encode(const int32_t* rec, size_t n, int64_t max_len, uint8_t** out, size_t* out_len,
                  size_t* footer_off);
/* Same, with rep != 0 selecting the REMPI_ENCODE=7 encoder (rempi_encoder_rep.cpp:50-146):
 * every table keeps set id, count and epoch line; all later sections are empty. */
int oracle_encode_ex(const int32_t* rec, size_t n, int64_t max_len, int rep, uint8_t** out, size_t* out_len,
                     size_t* footer_off);

/* Decode a whole rank_<r>.rempi byte image into the int64 table dump described in
 * oracle/tables_format.md (the same dump oracle/_ref/ref_cdc writes). *out is malloc'ed. */
int oracle_decode(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len);

/* Permutation core only: given c[0..M) (observed row -> clock order), return the
 * un-predicted (id, delta) pairs rempi_clock_delta_compression::compress emits before
 * linear prediction.  ids/deltas must hold M entries; *P receives the pair count. */
int oracle_cdc_pairs(const int32_t* c, int64_t M, int32_t* ids, int32_t* deltas, int64_t* P);

/* cdc_prepare_decode_indices: pairs (already inverse-predicted) -> perm[M].
 * One deliberate difference from the reference, shared with the device path: a delay that
 * would walk more than once round the list (|delay| > M, never written by the encoder) is
 * ORACLE_ERR_CORRUPT.  The reference's std::advance keeps stepping through the std::list
 * sentinel; oracle_set_reference_walk(1) restores exactly that (for the test that pins it
 * against the reference decoder), oracle_set_reference_walk(0) the default. */
void oracle_set_reference_walk(int on);
int oracle_decode_perm(const int64_t* ids, const int64_t* delays, int64_t P, int64_t M, int32_t* perm);

/* Iteration order of a libstdc++ std::unordered_map<size_t,size_t> after inserting the
 * given keys in order (duplicates ignored): writes the keys in iteration order, returns
 * the number of distinct keys.  Used to pin the device-side hash-order emulation. */
int64_t oracle_umap_order(const int64_t* keys, int64_t n, int64_t* out);
/* Same for std::unordered_set<int> (the footer's all_epoch_rank_uset). */
int64_t oracle_uset_int_order(const int32_t* keys, int64_t n, int32_t* out);

/* Events-level decode for records parity (the fields a replay can rebuild):
 * for every unit (chunk, table) of the file, rebuild the table's observed stream of
 * 32-B canonical records, given the unit's clock-sorted (source, clock) keys.
 * keys: concatenation over units (file order) of M_u pairs {source, clock} int32.
 * out: n_out x 8 int32 (malloc'ed). */
int oracle_reconstruct(const uint8_t* in, size_t len, const int32_t* sorted_keys, size_t n_keys,
                       int32_t** out, size_t* n_out);

/* Split a rank's records into per-unit clock-sorted key lists in file order
 * (helper for oracle_reconstruct tests). keys: malloc'ed {src, clock} pairs. */
int oracle_sorted_keys(const int32_t* rec, size_t n, int64_t max_len, int32_t** keys, size_t* n_keys);

void oracle_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
