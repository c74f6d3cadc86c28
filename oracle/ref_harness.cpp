// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured
// as the product).  Drives the *reference* ReMPI CDC encoder/decoder, compiled from
// the unmodified sources under /root/reference/src/rempi by oracle/Makefile, so that
// the C++ restatement (oracle/cdc_oracle.cpp) and the HIP path can be pinned to
// bytes produced by the reference itself.
//
//   ref_cdc encode <in.rec> <out.rempi> <REMPI_MAX> [gzip|rep]
//        (`rep`: the REMPI_ENCODE=7 encoder, rempi_encoder_rep: epoch lines only)
//        in.rec = n x 8 x int32 canonical records (rempi_event.h:40-48 layout).
//        Each record is pushed through rempi_event_list::push (rempi_event_list.cpp:66-99,
//        run-length merge), then the record loop of rempi_io_thread::write_record
//        (rempi_io_thread.cpp:56-97) is replayed: extract_encoder_input_format_chunk ->
//        encode -> write_record_file, then close_record_file (footer,
//        rempi_encoder_cdc.cpp:2085-2135).  Prints "encode_s <seconds>".
//   ref_cdc encode_basic <in.rec> <out.basic> <REMPI_MAX> [gzip]
//        the same push, then the REMPI_ENCODE=0 record loop with rempi_encoder_basic
//        (rempi_encoder_basic.cpp:81-224): a sequence of [size_t len][len bytes of 8 x int32
//        events] chunks (with `gzip`, REMPI_GZIP=1: each payload a zlib stream).  These files
//        are what the basic -> CDC transcoder reads.
//   ref_cdc decode <in.rempi> <out.tables> [gzip]
//        (`gzip`: REMPI_GZIP=1, chunk payloads are zlib streams)
//        read_record_file + decode per chunk (rempi_encoder_cdc.cpp:933-1299), dumping the
//        decoded tables (int64 little-endian, layout in oracle/tables_format.md).
//        Prints "decode_s <seconds>".
//   REF_CDC_IDMAP=<file> ref_cdc encode ...
//        before the footer is written, registers the matching-set-id map of <file> (L x
//        {uint64 msg id, int64 set id}) with the reference's own
//        rempi_reqmg_set_matching_set_id_map (rempi_request_mg.cpp:1136-1143), entry by entry in
//        file order, so that write_footer (:2105-2121) emits it.
//   ref_cdc footer <in.rempi> <out.map>
//        constructs the encoder in replay mode -- its constructor runs read_footer (:2015-2083),
//        which feeds the footer's map back through rempi_reqmg_set_matching_set_id_map -- and
//        dumps what rempi_reqmg_get_matching_set_id_map (:1068-1096) then returns: int64 L,
//        L msg ids, L set ids.
#include <mpi.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#include "rempi_encoder.h"
#include "rempi_event_list.h"
#include "rempi_config.h"
#include "rempi_event.h"
#include "rempi_request_mg.h"

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Dump {
  FILE* f;
  void v(int64_t x) { fwrite(&x, sizeof x, 1, f); }
  template <class Vec> void vec(const Vec& a) {
    v((int64_t)a.size());
    for (auto x : a) v((int64_t)x);
  }
};

int do_encode(const char* in, const char* out, int max_len, int gzip, int rep) {
  FILE* f = fopen(in, "rb");
  if (!f) { perror(in); return 2; }
  std::vector<int32_t> buf;
  int32_t r[8];
  while (fread(r, sizeof r, 1, f) == 1) buf.insert(buf.end(), r, r + 8);
  fclose(f);
  size_t n = buf.size() / 8;

  rempi_mode = 0;
  rempi_gzip = gzip;
  rempi_max_event_length = max_len;
  rempi_event_list<rempi_event*> events((size_t)1 << 40, 100);
  for (size_t i = 0; i < n; i++) {
    const int32_t* q = &buf[8 * i];
    // create_test_event(event_count, flag, rank, with_next, index, msg_id, matching_id)
    events.push(rempi_event::create_test_event(q[0], q[2], q[3], q[4], q[5], q[6], q[7]));
  }
  events.push_all();

  rempi_encoder_cdc cdc(0, out);
  rempi_encoder_rep repe(0, out);
  rempi_encoder_cdc& enc = rep ? repe : cdc;
  enc.open_record_file();
  double t0 = now_s();
  while (true) {
    rempi_encoder_input_format* fmt = enc.create_encoder_input_format();
    if (!enc.extract_encoder_input_format_chunk(events, fmt)) { delete fmt; break; }
    enc.encode();
    enc.write_record_file();
    // The reference's write_queue_vec points into fmt; it is consumed by write_record_file.
  }
  if (const char* mapf = getenv("REF_CDC_IDMAP")) {
    FILE* mf = fopen(mapf, "rb");
    if (!mf) { perror(mapf); return 2; }
    int64_t e[2];
    while (fread(e, sizeof e, 1, mf) == 1) {
      size_t id = (size_t)e[0];
      int sid = (int)e[1];
      rempi_reqmg_set_matching_set_id_map(&id, &sid, 1);
    }
    fclose(mf);
  }
  enc.close_record_file();
  double t1 = now_s();
  printf("encode_s %.6f records %zu\n", t1 - t0, n);
  return 0;
}

int do_encode_basic(const char* in, const char* out, int max_len, int gzip) {
  FILE* f = fopen(in, "rb");
  if (!f) { perror(in); return 2; }
  std::vector<int32_t> buf;
  int32_t r[8];
  while (fread(r, sizeof r, 1, f) == 1) buf.insert(buf.end(), r, r + 8);
  fclose(f);
  size_t n = buf.size() / 8;

  rempi_mode = 0;
  rempi_gzip = gzip;
  rempi_max_event_length = max_len;
  rempi_event_list<rempi_event*> events((size_t)1 << 40, 100);
  for (size_t i = 0; i < n; i++) {
    const int32_t* q = &buf[8 * i];
    events.push(rempi_event::create_test_event(q[0], q[2], q[3], q[4], q[5], q[6], q[7]));
  }
  events.push_all();

  rempi_encoder_basic enc(0, out);
  enc.open_record_file(out);
  while (true) {
    rempi_encoder_input_format* fmt = enc.create_encoder_input_format();
    if (!enc.extract_encoder_input_format_chunk(events, fmt)) { delete fmt; break; }
    enc.encode();
    enc.write_record_file();
  }
  enc.close_record_file();
  printf("encode_basic records %zu\n", n);
  return 0;
}

// rempi_encoder_cdc::decode keeps replay-engine state across chunks and aborts on the
// second chunk whenever #tables != #epoch ranks (rempi_encoder_cdc.cpp:1262-1267); that
// state is not part of the decoded data, so the harness clears it before each chunk.
struct Dec : rempi_encoder_cdc {
  explicit Dec(const char* p) : rempi_encoder_cdc(1, p) {}
  void reset_replay_state() { solid_mc_next_clocks_umap_umap.clear(); }
};

int do_decode(const char* in, const char* out, int gzip) {
  rempi_mode = 1;
  rempi_gzip = gzip;
  Dec dec(in);
  dec.open_record_file();
  FILE* f = fopen(out, "wb");
  if (!f) { perror(out); return 2; }
  Dump d{f};
  double total = 0;
  int64_t chunks = 0;
  std::vector<rempi_encoder_input_format*> keep;
  while (true) {
    rempi_encoder_input_format* fmt = dec.create_encoder_input_format();
    double t0 = now_s();
    if (dec.read_record_file(fmt)) { delete fmt; break; }
    dec.reset_replay_state();
    dec.decode();
    total += now_s() - t0;
    chunks++;
    d.v((int64_t)fmt->test_tables_map.size());
    for (auto& kv : fmt->test_tables_map) {
      rempi_encoder_input_format_test_table* t = kv.second;
      d.v(kv.first);
      d.v(t->count);
      d.vec(t->epoch_rank_vec);
      d.vec(t->epoch_clock_vec);
      d.vec(t->with_previous_vec);
      d.vec(t->matched_index_vec);
      std::vector<std::pair<size_t, size_t>> um(t->unmatched_events_umap.begin(), t->unmatched_events_umap.end());
      std::sort(um.begin(), um.end());
      d.v((int64_t)um.size());
      for (auto& p : um) { d.v((int64_t)p.first); d.v((int64_t)p.second); }
      d.vec(t->matched_events_id_vec);
      d.vec(t->matched_events_delay_vec);
      d.vec(t->matched_events_permutated_indices_vec);
    }
    keep.push_back(fmt);  // decode() hands pointers into fmt to the encoder; keep alive
  }
  fclose(f);
  printf("decode_s %.6f chunks %lld\n", total, (long long)chunks);
  return 0;
}
int do_footer(const char* in, const char* out) {
  rempi_mode = 1;
  rempi_gzip = 0;
  Dec dec(in);  // (read_footer runs in the constructor)
  size_t* ids = nullptr;
  int* sets = nullptr;
  int L = 0;
  rempi_reqmg_get_matching_set_id_map(&ids, &sets, &L);
  FILE* f = fopen(out, "wb");
  if (!f) { perror(out); return 2; }
  Dump d{f};
  d.v(L);
  for (int i = 0; i < L; i++) d.v((int64_t)ids[i]);
  for (int i = 0; i < L; i++) d.v(sets[i]);
  fclose(f);
  printf("footer_map %d\n", L);
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc >= 4 && std::string(argv[1]) == "footer") return do_footer(argv[2], argv[3]);
  if (argc >= 5 && std::string(argv[1]) == "encode")
    return do_encode(argv[2], argv[3], atoi(argv[4]), argc >= 6 && std::string(argv[5]) == "gzip",
                     argc >= 6 && std::string(argv[5]) == "rep");
  if (argc >= 5 && std::string(argv[1]) == "encode_basic")
    return do_encode_basic(argv[2], argv[3], atoi(argv[4]), argc >= 6 && std::string(argv[5]) == "gzip");
  if (argc >= 4 && std::string(argv[1]) == "decode")
    return do_decode(argv[2], argv[3], argc >= 5 && std::string(argv[4]) == "gzip");
  fprintf(stderr,
          "usage: ref_cdc encode <in.rec> <out.rempi> <REMPI_MAX> [gzip|rep] | encode_basic <in.rec> <out.basic> <REMPI_MAX> [gzip] |"
          " decode <in.rempi> <out.tables> [gzip]\n");
  return 1;
}
