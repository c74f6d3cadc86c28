// oracle/shim/shim_harness.cpp -- TEST INFRASTRUCTURE ONLY.  Drives the reference's own
// record loop and replay read loop with rempi_encoder_cdcx (the GPU codec behind the C ABI)
// in place of rempi_encoder_cdc.  Same command line and outputs as oracle/ref_harness.cpp,
// so the two binaries' files can be compared byte for byte:
//
//   shim_cdc encode <in.rec> <out.rempi> <REMPI_MAX> [gzip]
//        events -> rempi_event_list::push -> extract_encoder_input_format_chunk -> encode
//        (cdcx_encode_chunk) -> write_record_file -> close_record_file (reference footer)
//   shim_cdc decode <in.rempi> <out.tables> [gzip]
//        read_record_file -> decode (cdcx_decode_chunk) per chunk; dumps the test tables the
//        replay engine would consume (int64 layout of oracle/tables_format.md)
//   shim_cdc batch <list>
//        one encode/decode command per line of <list>, in one process
#include <mpi.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rempi_encoder_cdcx.h"
#include "rempi_config.h"
#include "rempi_event.h"
#include "rempi_event_list.h"

namespace {

struct Dump {
  FILE* f;
  void v(int64_t x) { fwrite(&x, sizeof x, 1, f); }
  template <class Vec>
  void vec(const Vec& a) {
    v((int64_t)a.size());
    for (size_t i = 0; i < a.size(); i++) v((int64_t)a[i]);
  }
};

int run_encode(const char* in, const char* out, int max_len, int gzip) {
  FILE* f = fopen(in, "rb");
  if (!f) { perror(in); return 2; }
  std::vector<int32_t> buf;
  int32_t r[8];
  while (fread(r, sizeof r, 1, f) == 1) buf.insert(buf.end(), r, r + 8);
  fclose(f);
  rempi_mode = 0;
  rempi_gzip = gzip;
  rempi_max_event_length = max_len;
  rempi_event_list<rempi_event*> events((size_t)1 << 40, 100);
  for (size_t i = 0; i + 8 <= buf.size(); i += 8)
    events.push(rempi_event::create_test_event(buf[i], buf[i + 2], buf[i + 3], buf[i + 4], buf[i + 5], buf[i + 6], buf[i + 7]));
  events.push_all();
  rempi_encoder_cdcx enc(0, out);
  enc.open_record_file();
  size_t chunks = 0;
  for (;;) {
    rempi_encoder_input_format* fmt = enc.create_encoder_input_format();
    const bool ready = enc.extract_encoder_input_format_chunk(events, fmt);
    if (!ready) { delete fmt; break; }
    enc.encode();
    enc.write_record_file();
    delete fmt;
    chunks++;
  }
  enc.close_record_file();
  printf("shim_encode chunks %zu records %zu\n", chunks, buf.size() / 8);
  return 0;
}

int run_decode(const char* in, const char* out, int gzip) {
  rempi_mode = 1;
  rempi_gzip = gzip;
  rempi_encoder_cdcx dec(1, in);
  dec.open_record_file();
  FILE* f = fopen(out, "wb");
  if (!f) { perror(out); return 2; }
  Dump d{f};
  size_t chunks = 0;
  for (;;) {
    rempi_encoder_input_format* fmt = dec.create_encoder_input_format();
    if (dec.read_record_file(fmt)) { delete fmt; break; }
    dec.reset_replay_state();
    dec.decode();
    chunks++;
    d.v((int64_t)fmt->test_tables_map.size());
    for (std::map<int, rempi_encoder_input_format_test_table*>::iterator kv = fmt->test_tables_map.begin();
         kv != fmt->test_tables_map.end(); ++kv) {
      rempi_encoder_input_format_test_table* t = kv->second;
      d.v(kv->first);
      d.v(t->count);
      d.vec(t->epoch_rank_vec);
      d.vec(t->epoch_clock_vec);
      d.vec(t->with_previous_vec);
      d.vec(t->matched_index_vec);
      std::vector<std::pair<size_t, size_t> > um(t->unmatched_events_umap.begin(), t->unmatched_events_umap.end());
      std::sort(um.begin(), um.end());
      d.v((int64_t)um.size());
      for (size_t i = 0; i < um.size(); i++) { d.v((int64_t)um[i].first); d.v((int64_t)um[i].second); }
      d.vec(t->matched_events_id_vec);
      d.vec(t->matched_events_delay_vec);
      d.vec(t->matched_events_permutated_indices_vec);
      // the consumer (cdc_decode_ordering) reads with_previous_bool_vec: cross-check it here
      for (size_t i = 0; i < t->with_previous_vec.size(); i++)
        if (!t->with_previous_bool_vec[t->with_previous_vec[i]]) { fprintf(stderr, "with_previous_bool_vec mismatch\n"); return 3; }
    }
    delete fmt;
  }
  fclose(f);
  printf("shim_decode chunks %zu\n", chunks);
  return 0;
}

// batch <list>: one "encode ..." / "decode ..." command per line, run in this process (one
// device context start-up for many small files); stops at the first failure.
int run_batch(const char* list) {
  FILE* f = fopen(list, "r");
  if (!f) { perror(list); return 2; }
  char line[4096];
  int n = 0;
  while (fgets(line, sizeof line, f)) {
    std::vector<std::string> a;
    for (char* t = strtok(line, " \t\n"); t; t = strtok(NULL, " \t\n")) a.push_back(t);
    if (a.empty()) continue;
    // static, one rank per command; a fresh set, since clear() keeps the bucket count and the
    // footer order follows the buckets
    std::unordered_set<int>().swap(rempi_encoder_input_format_test_table::all_epoch_rank_uset);
    int rc = 1;
    if (a[0] == "encode" && a.size() >= 4)
      rc = run_encode(a[1].c_str(), a[2].c_str(), atoi(a[3].c_str()), a.size() >= 5 && a[4] == "gzip");
    else if (a[0] == "decode" && a.size() >= 3)
      rc = run_decode(a[1].c_str(), a[2].c_str(), a.size() >= 4 && a[3] == "gzip");
    if (rc) { fprintf(stderr, "batch line %d failed (%d)\n", n + 1, rc); fclose(f); return rc; }
    n++;
  }
  fclose(f);
  printf("shim_batch commands %d\n", n);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string cmd = argc > 1 ? argv[1] : "";
  if (cmd == "batch" && argc >= 3) return run_batch(argv[2]);
  if (cmd == "encode" && argc >= 5) return run_encode(argv[2], argv[3], atoi(argv[4]), argc >= 6 && std::string(argv[5]) == "gzip");
  if (cmd == "decode" && argc >= 4) return run_decode(argv[2], argv[3], argc >= 5 && std::string(argv[4]) == "gzip");
  fprintf(stderr, "usage: shim_cdc encode <in.rec> <out.rempi> <REMPI_MAX> [gzip] | decode <in.rempi> <out.tables> [gzip]\n");
  return 1;
}
