/* cdcx.h -- C ABI of libcdcx.so, the MI355X (gfx950) Clock Delta Compression codec that
 * drops in behind ReMPI's CDC record writer / replay reader.
 *
 * Plain C: pointers, sizes and int status codes only.  Each entry point names the
 * reference interface it replaces (paths relative to PRUNERS/ReMPI src/rempi/).
 *
 * Byte format: identical to rempi_encoder_cdc with REMPI_GZIP=0:
 *   rank file = ( [size_t payload_len][payload] )* [size_t 0][footer]
 *   payload   = per matching-set table, ascending set id: int32 set_id, int32 count,
 *               size_t epoch bytes, size_t ranks[], size_t clocks[], size_t wp_len,
 *               size_t wp_bytes, size_t LP(with_previous)[], size_t mi_len, size_t mi_bytes,
 *               size_t matched_index[], size_t uid_bytes, size_t LP(unmatched_id)[],
 *               size_t ucnt_bytes, size_t unmatched_count[], size_t pair_bytes,
 *               int32 LP(ids)[], int32 LP(deltas)[]
 *   footer    = size_t n, int32 ranks[n] (all_epoch_rank_uset order), int32 L,
 *               size_t msg_ids[L], int32 set_ids[L] (the matching-set-id map in
 *               unordered_map<size_t,int> order; L = 0 unless a map was registered)
 *
 * Input records: the reference's 8 x int32 test event (rempi_event.h:40-48):
 *   [0] event_count [1] type [2] flag [3] rank [4] with_next [5] index [6] clock
 *   [7] matching_set_id
 * as rempi_event_list::push leaves them (consecutive duplicates already merged).
 * Decoded records (what the files let a replay rebuild, per table in observed order): a matched
 * event comes back as {1, 2, 1, rank, with_next != 0, index, clock, set id}, a run of unmatched
 * polls as {event_count summed over the run, 2, 0, 0, 0, 0, 0, set id}.
 * Implementation limit: 0 <= matching_set_id < 256 (REMPI_MAX_RECV_TEST_ID is 128).
 */
#ifndef CDCX_H
#define CDCX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  The reference reports the same conditions with REMPI_ERR
 * (print + abort, rempi_err.cpp:100-112); the drop-in shim maps non-zero codes to it. */
#define CDCX_OK 0
#define CDCX_ERR_ARG 1             /* bad argument */
#define CDCX_ERR_TRUNCATED_EPOCH 2 /* "The events in this epoch are truncated" (rempi_encoder_cdc.cpp:231) */
#define CDCX_ERR_CLOCK_ORDER 3     /* "Later message has smaller clock ..." (rempi_encoder_cdc.cpp:251) */
#define CDCX_ERR_CORRUPT 4         /* "Record data is broken" / inconsistent sizes (:952, :1288) */
#define CDCX_ERR_HIP 5             /* HIP runtime failure */
#define CDCX_ERR_LIMIT 6           /* implementation limit (set id range, sources per table) */
#define CDCX_ERR_NOMEM 7           /* device or host allocation failure */

typedef struct cdcx_opts {
  int64_t max_event_length; /* REMPI_MAX (rempi_config.cpp:103-108); default 131072 */
  int32_t gzip;             /* REMPI_GZIP (0 or 1): the host-buffer entry points (encode/decode/
                               reconstruct stream, encode chunk, transcode) apply the zlib stage
                               on the host; the device-resident batch entry points carry plain
                               CDC and return CDCX_ERR_ARG on a gzip context */
  int32_t device;           /* HIP device ordinal */
  int32_t encode;           /* REMPI_ENCODE (rempi_config.h:46-48): 0 or 4 = CDC; 7 = rep
                               (rempi_encoder_rep.cpp:50-146: every table keeps its set id,
                               count and epoch line, all other sections empty) */
  int32_t pad;
  int64_t reserved[3];
} cdcx_opts;

typedef struct cdcx_ctx cdcx_ctx;

/* Replaces `new rempi_encoder_cdc(mode, path)` (rempi_recorder_cdc.cpp:135) for the codec
 * part: one context per device, reusable across calls, not shared between threads. */
cdcx_ctx* cdcx_create(const cdcx_opts* opts);
void cdcx_destroy(cdcx_ctx* ctx);
/* Human-readable description of the last failure on this context. */
const char* cdcx_last_error(const cdcx_ctx* ctx);
/* Releases buffers returned by the host-memory entry points below. */
void cdcx_free(void* p);
/* Number of device kernels; name of each (for profiling tables). */
int cdcx_kernel_count(void);
const char* cdcx_kernel_name(int k);

/* ---------------------------------------------------------------------------------------
 * Record side (rempi_io_thread::write_record, rempi_io_thread.cpp:56-97 driving
 * extract_encoder_input_format_chunk (rempi_encoder_cdc.cpp:740-778), encode (:781-802),
 * write_record_file (:804-845) and close_record_file/write_footer (:2085-2135)).
 */

/* Host buffers: encode one rank's whole stream; *out (cdcx_free) receives the complete
 * rank_<r>.rempi image (chunks, separator, footer). */
int cdcx_encode_stream(cdcx_ctx* ctx, const int32_t* rec8, size_t n_rec, uint8_t** out,
                       size_t* out_len);

/* REMPI_GZIP=1 stage of a whole rank file, on the host: every chunk
 * payload replaced by its zlib stream (rempi_encoder_cdc::write_record_file,
 * rempi_encoder_cdc.cpp:804-844, deflate at Z_DEFAULT_COMPRESSION as in
 * rempi_compression_util.cpp:233-325) or back (read_record_file, :960-978); the separator
 * and footer are kept.  No context or GPU needed.  *out is freed with cdcx_free.
 * CDCX_ERR_CORRUPT for bad framing or a bad zlib stream. */
int cdcx_gzip_file(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len);
int cdcx_gunzip_file(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len);

/* Basic -> CDC transcoder.  A REMPI_ENCODE=0 record file holds one
 * rank's canonical event stream as [size_t len][len bytes of 8 x int32 events] chunks
 * (rempi_encoder_basic::write_record_file, rempi_encoder_basic.cpp:205-224; read back by
 * :238-321), so its CDC image is cdcx_encode_stream of the concatenated chunks.  The n_files
 * rank files are encoded as one device batch; outs[i] (cdcx_free) receives file i's
 * complete rank_<r>.rempi image (out_lens[i] bytes).  CDCX_ERR_ARG for a truncated file, a
 * chunk that is not a whole number of records, or a record whose type is not
 * REMPI_MPI_EVENT_TYPE_TEST (2): basic files may hold MPI_Recv events, which the CDC
 * recorder never records.  REMPI_GZIP=1 basic files are zlib streams: inflate them on the
 * host first. */
int cdcx_transcode_basic(cdcx_ctx* ctx, size_t n_files, const uint8_t* const* files, const size_t* lens,
                         uint8_t** outs, size_t* out_lens);

/* Host buffers: encode exactly one chunk (the records of one
 * extract_encoder_input_format_chunk call).  *payload (cdcx_free) is what
 * write_record_file emits after the size_t length; *epoch_ranks (cdcx_free, may be NULL
 * when n is 0) are the ranks format() inserts into all_epoch_rank_uset, in order. */
int cdcx_encode_chunk(cdcx_ctx* ctx, const int32_t* rec8, size_t n_rec, uint8_t** payload,
                      size_t* payload_len, int32_t** epoch_ranks, size_t* n_epoch_ranks);

/* Device-resident batch: n_ranks independent rank streams.
 *   d_rec    device pointer, records of all ranks concatenated (int32 x 8 each)
 *   rec_off  host array [n_ranks+1], record offsets of each rank in d_rec
 * On success *d_out points to a context-owned device buffer holding the n_ranks rank
 * files; file r is the out_len[r] bytes at out_off[r] (host arrays [n_ranks]; files start
 * 16-byte aligned).  The buffer stays valid until the next encode call on ctx.
 * `stream` is a hipStream_t (NULL = default stream). */
int cdcx_encode_batch_device(cdcx_ctx* ctx, int32_t n_ranks, const int32_t* d_rec,
                             const int64_t* rec_off, const uint8_t** d_out, int64_t* out_off,
                             int64_t* out_len, void* stream);

/* After cdcx_encode_batch_device: the clock-sorted (source, clock) keys of every unit
 * (table within chunk) of the batch, in file order (int32 pairs, context-owned device
 * buffer).  These are the keys a replaying process receives from the wire; the records
 * reconstruction below takes them as side input. */
int cdcx_batch_sorted_keys(cdcx_ctx* ctx, const int32_t** d_keys, int64_t* n_keys);

/* ---------------------------------------------------------------------------------------
 * Replay side (read_record_file (:933-978), decode (:1016-1299),
 * cdc_prepare_decode_indices (:1301-1386), read_footer (:2015-2083)).
 */

/* Host buffers: decode a whole rank file into the int64 table dump of
 * oracle/tables_format.md (per chunk: table count; per table: set id, count, epoch ranks,
 * epoch clocks, with_previous, matched_index, unmatched (id,count) sorted by id, ids,
 * delays, permutated indices).  *dump is released with cdcx_free. */
int cdcx_decode_stream(cdcx_ctx* ctx, const uint8_t* in, size_t len, uint8_t** dump,
                       size_t* dump_len);

/* Host buffers: decode a rank file and rebuild each table's observed stream of canonical
 * records (the fields a replay can rebuild: see cdcx_reconstruct_chunk).  sorted_keys: per
 * unit, file order, the clock-sorted {source, clock} pairs.  *rec8 (cdcx_free) gets n_out x 8 int32. */
int cdcx_reconstruct_stream(cdcx_ctx* ctx, const uint8_t* in, size_t len,
                            const int32_t* sorted_keys, size_t n_keys, int32_t** rec8,
                            size_t* n_out);

/* One decoded matching-set table of a chunk: the fields decode() (:1016-1299) leaves in
 * rempi_encoder_input_format_test_table, as flat arrays.  Every pointer points into the one
 * block that cdcx_tables.tables heads. */
typedef struct cdcx_table {
  int32_t set_id;                 /* test_tables_map key (matching_set_id) */
  int32_t count;                  /* test_table->count: matched events */
  size_t n_epoch;                 /* epoch_rank_vec / epoch_clock_vec, file order */
  const uint64_t* epoch_rank;
  const uint64_t* epoch_clock;
  size_t n_with_previous;         /* with_previous_vec (inverse LP applied) */
  const uint64_t* with_previous;
  size_t n_matched_index;         /* matched_index_vec */
  const uint64_t* matched_index;
  size_t n_unmatched;             /* (id, count) in file order: unmatched_events_umap[id] = count */
  const uint64_t* unmatched_id;
  const uint64_t* unmatched_count;
  size_t n_pairs;                 /* matched_events_id_vec / matched_events_delay_vec */
  const uint64_t* ids;
  const uint64_t* delays;
  const int32_t* perm;            /* matched_events_permutated_indices_vec [count] */
} cdcx_table;

typedef struct cdcx_tables {
  size_t n_tables;    /* tables of the chunk, ascending set id (std::map order); a later table
                         with the same id replaces an earlier one, as test_tables_map[id] = does */
  cdcx_table* tables; /* release with cdcx_free(tables): one block holds everything */
} cdcx_tables;

/* Host buffers: decode ONE chunk -- the payload read_record_file (:933-978) hands to decode()
 * (:1016-1299; on a gzip context the zlib stream as stored in the file) -- into flat tables,
 * including cdc_prepare_decode_indices (:1301-1386).  This is what a replacement of
 * rempi_encoder_cdc::decode calls from progress_decoding's DECODE state (:877-882).
 * CDCX_ERR_CORRUPT where the reference reports "Inconsistent size" (:1288) or would read out
 * of bounds. */
int cdcx_decode_chunk(cdcx_ctx* ctx, const uint8_t* payload, size_t len, cdcx_tables* out);

/* Host buffers: records reconstruction of ONE chunk payload (decoded records as defined
 * above, the consumer side being cdc_decode_ordering :1655-1879): sorted_keys are the clock-sorted
 * {source, clock} pairs of the chunk's tables in ascending set id.  *rec8 (cdcx_free) gets
 * n_out x 8 int32. */
int cdcx_reconstruct_chunk(cdcx_ctx* ctx, const uint8_t* payload, size_t len, const int32_t* sorted_keys,
                           size_t n_keys, int32_t** rec8, size_t* n_out);

/* The bytes write_footer (:2085-2126) appends at close_record_file: size_t 0 separator,
 * size_t n, the n distinct ranks in the iteration order of the unordered_set<int>
 * all_epoch_rank_uset after inserting epoch_ranks[0..n_in) in that order, then int32 0 (no
 * matching-set-id map).  No context or GPU needed.  out may be NULL to query the size;
 * otherwise *len holds its capacity on entry.  On return *len = footer bytes.
 * CDCX_ERR_ARG when the capacity is too small. */
int cdcx_footer(const int32_t* epoch_ranks, size_t n_in, uint8_t* out, size_t* len);

/* Device-resident batch decode of n_ranks rank files (file r = in_len[r] bytes at
 * d_in + in_off[r], 8-byte aligned; host arrays) plus records reconstruction from d_keys
 * (int32 {source, clock} pairs, units in file order; NULL = tables only).  Outputs stay in
 * context-owned device buffers:
 *   *d_rec_out  reconstructed records (int32 x 8), units in file order
 *   *n_rec_out  number of records
 *   *d_perm     per-unit matched_events_permutated_indices, concatenated (int32)
 * They stay valid until the next encode or decode call on ctx (decode scratch reuses the
 * encoder's scratch; the encoder's *d_out and sorted keys are not touched by decode). */
int cdcx_decode_batch_device(cdcx_ctx* ctx, int32_t n_ranks, const uint8_t* d_in,
                             const int64_t* in_off, const int64_t* in_len,
                             const int32_t* d_keys, int64_t n_keys,
                             const int32_t** d_rec_out, int64_t* n_rec_out,
                             const int32_t** d_perm, void* stream);

/* The one entry point that allocates nothing.  It has no counterpart in the reference; it is
 * for callers that cannot allocate device memory: tight replay loops, harnesses that forbid
 * hipMalloc.  (Not for a stream under HIP graph capture: the call waits for the stream and
 * copies its status words to the host, neither of which a capturing stream allows.)  A variant
 * of cdcx_decode_batch_device (tables
 * only) for ONE chunk already in device memory: d_payload is the chunk payload (what follows
 * the size_t length in the file, plain CDC), and d_perm receives the
 * matched_events_permutated_indices (cdc_prepare_decode_indices, :1301-1386) of the chunk's
 * tables in file order, concatenated: the same int32 values *d_perm of
 * cdcx_decode_batch_device holds for that chunk.  *n_perm = entries written (sum of the
 * tables' counts); perm_capacity = entries d_perm can hold.
 * All scratch (unit table, pair rows, list links; 7 MiB) is a file-scope device array that
 * each GPU the library runs on holds until the process ends.  Limits: at most 256 tables and
 * sum(count + 1) <= 262144 per chunk (REMPI_MAX = 131072 chunks fit), else CDCX_ERR_LIMIT.
 * d_payload must be 8-byte aligned and d_perm 4-byte aligned (CDCX_ERR_ARG otherwise, as for a
 * REMPI_GZIP context: the payload must be plain CDC).
 * Calls no hipMalloc / hipFree; it does wait for the stream once, to read the status.
 * Every call on a GPU uses that GPU's one array: calls that overlap on one GPU (other
 * streams, other contexts or threads) race -- serialise them. */
int cdcx_decode_chunk_perm_static(cdcx_ctx* ctx, const uint8_t* d_payload, size_t len, int32_t* d_perm,
                                  size_t perm_capacity, int64_t* n_perm, void* stream);

/* After cdcx_decode_batch_device of n_ranks files: where each rank's part of *d_rec_out and
 * *d_perm begins (host arrays [n_ranks + 1]; records, and int32 perm entries = matched
 * events; entry n_ranks = the totals). */
int cdcx_decode_rank_offsets(cdcx_ctx* ctx, int32_t n_ranks, int64_t* rec_off, int64_t* perm_off);

/* Round-trip check on the device (the size-independent parity property of the batch path;
 * no counterpart in the reference, whose tests compare validation hashes after replay,
 * rempi_recorder.cpp:47-79).  Call right after cdcx_encode_batch_device(d_rec, ...) followed by
 * cdcx_decode_batch_device of its files with its sorted keys on the same context: every
 * decoded record is compared with the input record it must reproduce (per chunk, per table,
 * observed order; decoded records as defined above: a run of polls that the encoder merged
 * is one record with the summed count).  *mismatches = decoded records that differ. */
int cdcx_verify_roundtrip_device(cdcx_ctx* ctx, const int32_t* d_rec, int64_t* mismatches, void* stream);

/* ---------------------------------------------------------------------------------------
 * Replay-side streaming decode of a whole record directory.  Replaces one
 * read_record_file (:933-978) + decode (:1016-1299) + cdc_prepare_decode_indices
 * (:1301-1386) loop per rank process, which progress_decoding (:851-930) runs over
 * REMPI_DIR/rank_<r>.rempi, by one pass over many rank files.
 *
 * The n_files files at paths[] are decoded in batches of consecutive files of about
 * batch_bytes (<= 0: 256 MiB) each.  One host thread per context runs its own batches on its
 * own non-blocking HIP stream: file reads into a pinned host buffer (inflated first on a
 * gzip context), H2D, the decode kernels, D2H of the tables, so one context's reads and
 * copies overlap another's kernels.  Contexts may share a device.  For every file, in
 * completion order, sink(user, i, dump, n_words) receives file i's table dump (the int64
 * format of cdcx_decode_stream, valid only during the call).  Sink calls are serialised.  A
 * non-zero sink return stops the pipeline with CDCX_ERR_ARG.  stats (may be NULL) gets
 * totals.  On error the failing context's cdcx_last_error says why. */
typedef int (*cdcx_replay_sink)(void* user, int32_t file_index, const int64_t* dump, size_t n_words);
typedef struct cdcx_replay_stats {
  int64_t files;      /* rank files decoded */
  int64_t file_bytes; /* bytes read from the files (before inflating) */
  int64_t chunks;     /* chunks (read_record_file calls that returned data) */
  int64_t units;      /* matching-set tables */
  int64_t records;    /* canonical records the tables describe: matched + unmatched runs */
  int64_t batches;    /* device batches */
  int64_t dump_bytes; /* bytes of table dumps handed to the sink */
  double seconds;     /* wall time of the whole call */
  double read_s;      /* thread-seconds per phase, summed over contexts: file reads (+ inflate) */
  double device_s;    /* H2D + decode kernels + D2H of the tables */
  double dump_s;      /* host formatting of the per-rank table dumps */
  double sink_s;      /* inside the sink */
} cdcx_replay_stats;
int cdcx_replay_decode_files(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                             int64_t batch_bytes, cdcx_replay_sink sink, void* user, cdcx_replay_stats* stats);

/* The same pipeline delivering what the reference's replay engine consumes: for every file,
 * sink(user, i, n_chunks, chunks) receives one cdcx_tables per chunk (in file order) -- the
 * flat test tables decode() (:1016-1299) would have filled for that chunk, i.e. the inputs of
 * insert_encoder_input_format_chunk_recv_test_id / cdc_decode_ordering (:1390-1973).  Nothing
 * is formatted or copied on the host: the arrays point into the context's pinned buffers (the
 * file image and the packed device output) and are valid only during the call.  The contexts
 * may live on different devices (one worker thread each sets its context's device).
 * stats->dump_bytes counts the table descriptors handed over. */
typedef int (*cdcx_replay_table_sink)(void* user, int32_t file_index, size_t n_chunks, const cdcx_tables* chunks);
int cdcx_replay_decode_tables(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                              int64_t batch_bytes, cdcx_replay_table_sink sink, void* user, cdcx_replay_stats* stats);

/* ---------------------------------------------------------------------------------------
 * Footer contents (write_footer :2085-2126, read_footer :2015-2083).
 */

/* rempi_reqmg_set_matching_set_id_map (rempi_request_mg.cpp:1136-1143): register message id ->
 * matching set id entries on the context, in this order; an id registered before keeps its
 * place and takes the new set id (unordered_map operator[]).  n == 0 forgets all entries.
 * The rank files written by the host-buffer entry points of this context (cdcx_encode_stream,
 * cdcx_transcode_basic) then end with the map as write_footer emits it -- int32 L,
 * size_t msg_ids[L], int32 set_ids[L], in the iteration order of the reference's
 * unordered_map<size_t, int> comm_tag_to_matching_set_id (rempi_request_mg.cpp:1083-1094).
 * The device-resident batch path always writes L = 0 (the map is host state of a recording
 * process, not trace data). */
int cdcx_set_matching_set_id_map(cdcx_ctx* ctx, const uint64_t* msg_ids, const int32_t* set_ids, size_t n);

/* write_footer with a map: as cdcx_footer, plus the n_ids map entries given in registration
 * order.  Same length protocol as cdcx_footer. */
int cdcx_footer_ex(const int32_t* epoch_ranks, size_t n_ranks, const uint64_t* msg_ids, const int32_t* set_ids,
                   size_t n_ids, uint8_t* out, size_t* len);

/* read_footer: the footer of a rank file image (plain or REMPI_GZIP=1: the footer is stored
 * plain either way): the global predecessor ranks in file order (the reference reads and drops
 * them, :2044-2054) and the matching-set-id map in file order, as read_footer hands it to
 * rempi_reqmg_set_matching_set_id_map (:2057-2073).  *out is one block: cdcx_free(*out).
 * CDCX_ERR_CORRUPT for a file without separator or with a footer shorter than it says. */
typedef struct cdcx_footer_info {
  size_t n_ranks;
  const int32_t* ranks;
  size_t n_ids;
  const uint64_t* msg_ids;
  const int32_t* set_ids;
} cdcx_footer_info;
int cdcx_read_footer(const uint8_t* file, size_t len, cdcx_footer_info** out);

/* cdcx_replay_decode_tables that also delivers every file's footer: footer_sink(user, i, info)
 * is called (serialised with the table sink, right before file i's tables) with the parsed
 * footer of file i, valid during the call.  footer_sink may be NULL. */
typedef int (*cdcx_replay_footer_sink)(void* user, int32_t file_index, const cdcx_footer_info* footer);
int cdcx_replay_decode_tables_ex(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                                 int64_t batch_bytes, cdcx_replay_table_sink sink, cdcx_replay_footer_sink footer_sink,
                                 void* user, cdcx_replay_stats* stats);

/* ---------------------------------------------------------------------------------------
 * Synthetic workload (definition in rempi_amd/csrc/gen.h), generated
 * directly in device memory: n_ranks consecutive ranks starting at first_rank of a job of
 * world_size ranks, ~events_per_rank records each.  *d_rec (context-owned) and rec_off
 * (host, [n_ranks+1]) describe the result.  Also available on the host for tests. */
typedef struct cdcx_gen_params {
  int32_t world_size;   /* ranks in the job (sources are other ranks) */
  int32_t senders;      /* senders per rank (capped at world_size-1) */
  int32_t sets;         /* matching sets per rank */
  int32_t jitter;       /* arrival jitter J in clock units */
  int64_t events_per_rank;
  uint64_t seed_salt;   /* 0 for the reference workload */
} cdcx_gen_params;

int cdcx_generate_device(cdcx_ctx* ctx, const cdcx_gen_params* p, int32_t first_rank,
                         int32_t n_ranks, const int32_t** d_rec, int64_t* rec_off, void* stream);
int cdcx_generate_host(const cdcx_gen_params* p, int32_t rank, int32_t** rec8, size_t* n_rec);

/* Per-kernel device time (ms) accumulated since the last reset, measured with HIP events
 * on the launch stream when profiling is enabled. */
int cdcx_set_profiling(cdcx_ctx* ctx, int enabled);
int cdcx_kernel_times(cdcx_ctx* ctx, double* ms, int64_t* launches, int n);
int cdcx_reset_kernel_times(cdcx_ctx* ctx);

/* Diagnostics of the chain kernel (enabled by the environment variable CDCX_CHAIN_STATS at
 * context creation): events, slow-path events, winner-search iterations, climb steps, k*
 * searches, leaf-list spills, open-column steps, max leaves; copied into out[0..n) and
 * reset.  Returns CDCX_ERR_ARG when diagnostics are off. */
int cdcx_chain_stats(cdcx_ctx* ctx, int64_t* out, int n);

/* Segments that entered each chain tier in the last device encode: out[0] all segments
 * (16-lane groups), out[1] segments whose leaf list outgrew 16 slots (64-lane groups),
 * out[2] segments that outgrew 64 slots (lane kernel, global-memory leaf list). */
int cdcx_chain_tiers(cdcx_ctx* ctx, int64_t* out);

/* Totals of the last device encode (what add() / format() / compress() counted over the batch,
 * rempi_encoder_cdc.cpp:178-272, rempi_clock_delta_compression.cpp:465-672): out[0] records,
 * out[1] matched events, out[2] unmatched runs, out[3] with_previous entries, out[4] epoch
 * sources, out[5] (id, delay) pairs, out[6] tables, out[7] chunks. */
int cdcx_encode_totals(cdcx_ctx* ctx, int64_t* out);

/* Tables that entered each tier of the permutation rebuild (cdc_prepare_decode_indices,
 * rempi_encoder_cdc.cpp:1301-1386) in the last decode: out[0] all tables (pair segments),
 * out[1] tables with a segment that did not finish or did not check out (whole table in a
 * 16-lane group), out[2] tables that left that one (256-slot window), out[3] tables replayed
 * on the sequential list; out[4] the pair segments of the first tier, out[5] segment reruns
 * (a segment whose replayed start differed from its predecessor's final state runs again from
 * that state), out[6] segments that did not finish or still differed and sent their table on. */
int cdcx_decode_tiers(cdcx_ctx* ctx, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* CDCX_H */
