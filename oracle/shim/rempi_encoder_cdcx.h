// rempi_encoder_cdcx.h -- the drop-in binding a ReMPI maintainer adds next to
// rempi_encoder_cdc (MPI_VERSION == 3 && !REMPI_LITE): the CDC encoder with its codec work
// (format / encode / decode) done by libcdcx.so through the C ABI of include/cdcx.h.
//
// In this repository it is TEST INFRASTRUCTURE: oracle/Makefile compiles it against the
// unmodified reference headers under /root/reference/src/rempi and links it with the
// reference objects into oracle/_ref/shim_cdc, so that the reference's own record loop
// (rempi_io_thread.cpp:56-97) and replay read loop (rempi_encoder_cdc.cpp:851-930:
// read_record_file -> decode) run over the GPU codec and are compared with the reference's
// bytes and tables.  Nothing of the reference is copied here; the class only overrides the
// virtuals of rempi_encoder.h:196-288 / :291-301 / :335-432.
#pragma once
#include <cstring>
#include <list>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "rempi_encoder.h"
#include "rempi_err.h"
#include "rempi_mem.h"

#include "cdcx.h"

// Record side: keeps the chunk's canonical 8 x int32 records in stream order.  The base
// add() still runs, so length() and last_added_event (the chunk-closing rule of
// extract_encoder_input_format_chunk, rempi_encoder_cdc.cpp:740-778) stay the reference's.
class rempi_encoder_cdcx_input_format : public rempi_encoder_cdc_input_format {
 public:
  std::vector<int32_t> rec8;
  virtual void add(rempi_event* e) {
    for (int k = 0; k < REMPI_MPI_EVENT_INPUT_NUM; k++) rec8.push_back(e->mpi_inputs[k]);
    rempi_encoder_cdc_input_format::add(e);
  }
  // sort, epoch line, clock order: done on the GPU inside cdcx_encode_chunk
  virtual void format() {}
};

class rempi_encoder_cdcx : public rempi_encoder_cdc {
  cdcx_ctx* ctx_;
  uint8_t* payload_;

  void fail(const char* what, int st) {
    REMPI_ERR("%s failed (%d): %s", what, st, cdcx_last_error(ctx_));
  }

 public:
  rempi_encoder_cdcx(int mode, string path, int device = 0) : rempi_encoder_cdc(mode, path), ctx_(NULL), payload_(NULL) {
    cdcx_opts o = {};
    o.max_event_length = rempi_max_event_length;  // REMPI_MAX
    o.gzip = 0;  // write_record_file / read_record_file keep the reference's zlib stage
    o.device = device;
    o.encode = 4;
    ctx_ = cdcx_create(&o);
    if (!ctx_) REMPI_ERR("cdcx_create failed");
  }
  ~rempi_encoder_cdcx() {
    cdcx_free(payload_);
    cdcx_destroy(ctx_);
  }

  virtual rempi_encoder_input_format* create_encoder_input_format() { return new rempi_encoder_cdcx_input_format(); }

  // rempi_encoder_cdc::encode (rempi_encoder_cdc.cpp:781-802): one (pointer, size) entry in
  // the write queue instead of one per section; write_record_file (:804-845) is unchanged.
  virtual void encode() {
    rempi_encoder_cdcx_input_format* f = static_cast<rempi_encoder_cdcx_input_format*>(input_format);
    size_t len = 0, n_ranks = 0;
    int32_t* ranks = NULL;
    cdcx_free(payload_);
    payload_ = NULL;
    int st = cdcx_encode_chunk(ctx_, f->rec8.data(), f->rec8.size() / 8, &payload_, &len, &ranks, &n_ranks);
    if (st != CDCX_OK) fail("cdcx_encode_chunk", st);
    std::vector<int32_t>().swap(f->rec8);  // the caller deletes the format through its base class
    // what format() (:261-267) would have added, in its order: write_footer (:2085-2126)
    // then emits the reference's footer
    for (size_t i = 0; i < n_ranks; i++) rempi_encoder_input_format_test_table::all_epoch_rank_uset.insert(ranks[i]);
    cdcx_free(ranks);
    f->write_queue_vec.assign(1, (char*)payload_);
    f->write_size_queue_vec.assign(1, len);
  }

  // rempi_encoder_cdc::decode (rempi_encoder_cdc.cpp:1016-1299): the payload pieces that
  // read_record_file (:933-978) queued are joined, decoded by cdcx_decode_chunk, and every
  // field decode() leaves in the chunk's test tables is filled from the flat arrays.
  virtual void decode() {
    rempi_encoder_input_format* f = input_format;
    char* joined = (char*)rempi_malloc(f->decompressed_size);
    size_t at = 0;
    for (size_t i = 0; i < f->write_queue_vec.size(); i++) {
      memcpy(joined + at, f->write_queue_vec[i], f->write_size_queue_vec[i]);
      free(f->write_queue_vec[i]);
      at += f->write_size_queue_vec[i];
    }
    f->decompressed_record_char = joined;  // freed by rempi_encoder_input_format::clear

    cdcx_tables tabs;
    int st = cdcx_decode_chunk(ctx_, (const uint8_t*)joined, at, &tabs);
    if (st != CDCX_OK) fail("cdcx_decode_chunk", st);

    std::unordered_set<int> recv_ranks;
    for (size_t k = 0; k < tabs.n_tables; k++) {
      const cdcx_table& t = tabs.tables[k];
      rempi_encoder_input_format_test_table* tt = new rempi_encoder_input_format_test_table(t.set_id);
      f->test_tables_map[t.set_id] = tt;
      tt->count = t.count;
      tt->epoch_size = t.n_epoch * sizeof(size_t);
      for (size_t i = 0; i < t.n_epoch; i++) {
        const size_t rank = t.epoch_rank[i], clock = t.epoch_clock[i];
        tt->epoch_umap[rank] = clock;
        tt->epoch_line_umap[rank] = clock;
        tt->epoch_rank_vec.push_back(rank);
        tt->epoch_clock_vec.push_back(clock);
        tt->pending_event_count_umap[(int)rank] = 0;
        tt->current_epoch_line_umap[(int)rank] = 0;
        recv_ranks.insert((int)rank);
      }
      tt->compressed_with_previous_size = t.n_with_previous * sizeof(size_t);
      tt->with_previous_vec.assign(t.with_previous, t.with_previous + t.n_with_previous);
      if (t.n_with_previous > 0) {
        tt->with_previous_bool_vec.resize(t.count, false);
        for (size_t i = 0; i < t.n_with_previous; i++) tt->with_previous_bool_vec[t.with_previous[i]] = true;
      }
      tt->compressed_matched_index_size = t.n_matched_index * sizeof(size_t);
      tt->matched_index_vec.assign(t.matched_index, t.matched_index + t.n_matched_index);
      for (size_t i = 0; i < t.n_unmatched; i++) tt->unmatched_events_umap[t.unmatched_id[i]] = t.unmatched_count[i];
      tt->compressed_matched_events_size = 2 * t.n_pairs * sizeof(int);
      tt->matched_events_id_vec.assign(t.ids, t.ids + t.n_pairs);
      tt->matched_events_delay_vec.assign(t.delays, t.delays + t.n_pairs);
      tt->matched_events_permutated_indices_vec.assign(t.perm, t.perm + t.count);
    }
    cdcx_free(tabs.tables);

    // look-ahead clock bookkeeping of the replay engine (:1225-1282): the ranks this rank
    // receives from in this epoch, and one next-clock map per matching set
    f->mc_length = (int)recv_ranks.size();
    f->mc_recv_ranks = (int*)rempi_malloc(sizeof(int) * recv_ranks.size());
    int n = 0;
    for (std::unordered_set<int>::const_iterator it = recv_ranks.begin(); it != recv_ranks.end(); ++it)
      f->mc_recv_ranks[n++] = *it;
    if (!solid_mc_next_clocks_umap_umap.empty() && solid_mc_next_clocks_umap_umap.size() < f->test_tables_map.size())
      REMPI_ERR("test_table_map size increased: use a larger REMPI_MAX");
    for (std::map<int, rempi_encoder_input_format_test_table*>::iterator it = f->test_tables_map.begin();
         it != f->test_tables_map.end(); ++it) {
      if (solid_mc_next_clocks_umap_umap.find(it->first) != solid_mc_next_clocks_umap_umap.end()) {
        if (solid_mc_next_clocks_umap_umap.size() != recv_ranks.size())
          REMPI_ERR("solid_mc_next_clocks_umap_umap.size() changes from %lu to %lu", solid_mc_next_clocks_umap_umap.size(),
                    recv_ranks.size());
        continue;
      }
      std::unordered_map<int, size_t>* next = new std::unordered_map<int, size_t>();
      for (std::unordered_set<int>::const_iterator r = recv_ranks.begin(); r != recv_ranks.end(); ++r) (*next)[*r] = 0;
      solid_mc_next_clocks_umap_umap[it->first] = next;
    }
    this->mc_recv_ranks = f->mc_recv_ranks;
    this->mc_length = f->mc_length;
    if (this->mc_length > 1024) REMPI_ERR("mc_length > 1024");
  }

  // test harness only: decode() keeps look-ahead state across chunks and the reference aborts
  // on the next chunk whenever #tables != #epoch ranks (:1262-1267); that state is not decoded data
  void reset_replay_state() { solid_mc_next_clocks_umap_umap.clear(); }
};
