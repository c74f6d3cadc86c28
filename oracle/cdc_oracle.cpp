// oracle/cdc_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see cdc_oracle.h).
//
// A deliberately plain, sequential CPU restatement of the reference CDC codec, written from
// a written behaviour spec rather than translated from the reference classes.
// Every function cites the reference code whose observable behaviour it reproduces
// (paths relative to /root/reference/src/rempi).  Pinned by tests/test_oracle_golden.py
// against bytes and tables produced by the reference itself (oracle/_ref/ref_cdc).
#include "cdc_oracle.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using u64 = uint64_t;

// ---------------------------------------------------------------------------------------
// Byte sink: the reference writes raw host-endian int / size_t values (x86-64: LE).
struct Sink {
  std::vector<uint8_t> b;
  void put_i32(int32_t v) { put(&v, 4); }
  void put_u64(u64 v) { put(&v, 8); }
  void put(const void* p, size_t n) {
    const uint8_t* q = static_cast<const uint8_t*>(p);
    b.insert(b.end(), q, q + n);
  }
};

// Record field indices, rempi_event.h:40-48.
enum { F_COUNT = 0, F_TYPE = 1, F_FLAG = 2, F_RANK = 3, F_WITH_NEXT = 4, F_INDEX = 5, F_CLOCK = 6, F_SET = 7 };

inline u64 as_size_t(int32_t v) { return static_cast<u64>(static_cast<int64_t>(v)); }

// Second-order linear predictor, rempi_compression_util.cpp:117-154 (forward) and
// :157-168 (inverse).  Unsigned arithmetic gives the two's-complement wrap of the
// reference's int / size_t instantiations.
template <class U>
void lp_forward(std::vector<U>& x) {
  U p1 = 0, p2 = 0;
  for (auto& v : x) {
    U cur = v;
    v = static_cast<U>(cur - static_cast<U>(2 * p1) + p2);
    p2 = p1;
    p1 = cur;
  }
}
template <class U>
void lp_inverse(std::vector<U>& y) {
  U p1 = 0, p2 = 0;
  for (auto& v : y) {
    U cur = static_cast<U>(v + static_cast<U>(2 * p1) - p2);
    v = cur;
    p2 = p1;
    p1 = cur;
  }
}

// ---------------------------------------------------------------------------------------
// Permutation core: the chain search of rempi_clock_delta_compression.cpp:93-257 and the
// diff/delta emission of :160-181, :318-334, :336-400.
//
// Nodes are the matched events in observed order, node i at (row i, column c[i]); the
// column search of :259-316 always lands on column == clock order.  A node's level is
// 1 + the highest level among earlier nodes with a smaller column.  Its parent is found by
// scanning the childless nodes ("leaves") in creation order: for each leaf, climb to the
// first ancestor whose column is smaller than the new node's; the first leaf whose climb
// reaches the maximal level provides the parent (strict improvement, :213).  A leaf that
// is itself chosen stops being a leaf (:243-246).  Leaves left of the first unmatched
// column are dropped when a node lands on that column (:252-254, output-neutral).
struct ChainBuilder {
  std::vector<int32_t> col, lvl, par;  // per node
  std::vector<int32_t> leaves;         // node ids, creation order

  int32_t add(int32_t row, int32_t column, int32_t first_open_col) {
    (void)row;  // every existing node has a smaller row
    int32_t best_lvl = 0, best = -1, best_leaf_pos = -1;
    for (size_t li = 0; li < leaves.size(); li++) {
      int32_t s = leaves[li];
      while (s >= 0 && col[s] >= column) s = par[s];
      if (s >= 0 && lvl[s] > best_lvl) {
        best_lvl = lvl[s];
        best = s;
        best_leaf_pos = (s == leaves[li]) ? (int32_t)li : -1;
      }
    }
    int32_t id = (int32_t)col.size();
    col.push_back(column);
    lvl.push_back(best_lvl + 1);
    par.push_back(best);
    if (best_leaf_pos >= 0) leaves.erase(leaves.begin() + best_leaf_pos);
    leaves.push_back(id);
    if (column == first_open_col) {
      size_t w = 0;
      for (size_t li = 0; li < leaves.size(); li++)
        if (col[leaves[li]] >= first_open_col) leaves[w++] = leaves[li];
      leaves.resize(w);
    }
    return id;
  }
};

// Emits the pairs for permutation c (row -> clock order); returns P.
int64_t cdc_pairs(const int32_t* c, int64_t M, std::vector<int32_t>& ids, std::vector<int32_t>& deltas) {
  ChainBuilder cb;
  cb.col.reserve(M + 1);
  cb.lvl.reserve(M + 1);
  cb.par.reserve(M + 1);
  std::vector<uint8_t> taken(M + 1, 0);
  int32_t open = 0;
  for (int64_t i = 0; i < M; i++) {
    cb.add((int32_t)i, c[i], open);
    taken[c[i]] = 1;
    while (open < M && taken[open]) open++;
  }
  int32_t fin = cb.add((int32_t)M, (int32_t)M, open);

  // Chain rows/cols from the root down to the final node.
  std::vector<int32_t> chain;
  for (int32_t s = cb.par[fin]; s >= 0; s = cb.par[s]) chain.push_back(s);
  std::reverse(chain.begin(), chain.end());

  // Forward edit sequence (:160-181 builds it reversed): per gap, ADD the skipped rows
  // (as clock-order ids, :318-334) ascending, REMOVE the skipped columns ascending, then
  // IGNORE the chain node itself (not after the final node).
  enum : int8_t { IGN = 0, ADD = 1, REM = -1 };
  std::vector<int32_t> sid;
  std::vector<int8_t> sty;
  sid.reserve(2 * M + 1);
  sty.reserve(2 * M + 1);
  int32_t pr = -1, pc = -1;
  for (size_t k = 0; k <= chain.size(); k++) {
    int32_t r = (k < chain.size()) ? chain[k] : (int32_t)M;
    int32_t cc = (k < chain.size()) ? cb.col[chain[k]] : (int32_t)M;
    for (int32_t q = pr + 1; q < r; q++) { sid.push_back(c[q]); sty.push_back(ADD); }
    for (int32_t q = pc + 1; q < cc; q++) { sid.push_back(q); sty.push_back(REM); }
    if (k < chain.size()) { sid.push_back(cc); sty.push_back(IGN); }
    pr = r;
    pc = cc;
  }

  // :358-396: at an id's second occurrence, count the entries strictly between its two
  // occurrences that sit in the decoder's list at that moment.
  std::vector<int64_t> first(M, -1);  // position of first occurrence while pending
  ids.clear();
  deltas.clear();
  for (int64_t p = 0; p < (int64_t)sid.size(); p++) {
    if (sty[p] == IGN) continue;
    int32_t x = sid[p];
    if (first[x] < 0) { first[x] = p; continue; }
    int32_t d = 0;
    for (int64_t q = first[x] + 1; q < p; q++) {
      if (sty[q] == IGN) d++;
      else if (sty[q] == REM) d += (first[sid[q]] >= 0);
      else d += (first[sid[q]] < 0);
    }
    ids.push_back(x);
    deltas.push_back(sty[p] == REM ? -d : d);
    first[x] = -1;
  }
  return (int64_t)ids.size();
}

// ---------------------------------------------------------------------------------------
// One matching-set table inside one chunk (rempi_encoder.h test_table, CDC fields).
struct Table {
  int32_t set_id = 0;
  int32_t count = 0;
  std::vector<int32_t> src, clk;  // matched events, observed order
  std::vector<u64> with_prev;     // events_vec index of with_next events (:191-195)
  std::vector<u64> mindex;        // index field per matched event (:196)
  std::vector<u64> um_id, um_cnt; // unmatched runs (:199-212)
};

struct Encoder {
  int64_t max_len;
  int rep = 0;  // REMPI_ENCODE=7 (rempi_encoder_rep.cpp:50-146): epoch lines only
  std::unordered_set<int> footer_ranks;  // rempi_encoder_cdc.cpp:60, :266
  Sink out;

  // rempi_encoder_cdc_input_format::add, rempi_encoder_cdc.cpp:178-218.  Returns the
  // increment of input_format->length().
  static int add(std::map<int32_t, Table>& tabs, const int32_t* r) {
    auto it = tabs.find(r[F_SET]);
    if (it == tabs.end()) {
      it = tabs.emplace(r[F_SET], Table()).first;
      it->second.set_id = r[F_SET];
    }
    Table& t = it->second;
    if (r[F_FLAG] == 1) {
      t.src.push_back(r[F_RANK]);
      t.clk.push_back(r[F_CLOCK]);
      if (r[F_WITH_NEXT] != 0) t.with_prev.push_back(t.src.size() - 1);
      t.mindex.push_back(as_size_t(r[F_INDEX]));
      t.count++;
      return 1;
    }
    if (!t.um_id.empty() && t.um_id.back() == t.src.size()) {
      t.um_cnt.back() += as_size_t(r[F_COUNT]);
      return 0;
    }
    t.um_id.push_back(t.src.size());
    t.um_cnt.push_back(as_size_t(r[F_COUNT]));
    return 1;
  }

  // format() (:220-272) + encode() (:781-802) + write_record_file() (:804-845), gzip off.
  int emit_chunk(std::map<int32_t, Table>& tabs, const int32_t* last) {
    (void)last;
    Sink body;
    for (auto& kv : tabs) {
      Table& t = kv.second;
      const int64_t M = (int64_t)t.src.size();
      // A table must not end inside a with_next group (:229-233).
      if (M > 0) {
        // The last *matched* event of the table is what the reference checks.
        // with_prev holds indices of with_next events; the last one being M-1 means so.
        if (!t.with_prev.empty() && (int64_t)t.with_prev.back() == M - 1) return ORACLE_ERR_TRUNCATED_EPOCH;
      }
      // Clock order: sort by (clock, source) (:152-162, :235-239).  Equal keys are only
      // legal with clock 0 and their order is unspecified in the reference (std::sort);
      // ties are broken by observed position here ("parity unpinned" for that case).
      std::vector<int32_t> order(M);
      for (int64_t i = 0; i < M; i++) order[i] = (int32_t)i;
      std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        if (t.clk[a] != t.clk[b]) return t.clk[a] < t.clk[b];
        return t.src[a] < t.src[b];
      });
      std::vector<int32_t> c(M);
      for (int64_t r = 0; r < M; r++) c[order[r]] = (int32_t)r;
      // Epoch line (:246-267): last clock per source in sorted order, listed in the
      // iteration order of the reference's unordered_map<size_t,size_t>.
      std::unordered_map<size_t, size_t> epoch;
      for (int64_t r = 0; r < M; r++) {
        int32_t e = order[r];
        size_t key = as_size_t(t.src[e]);
        size_t val = as_size_t(t.clk[e]);
        auto f = epoch.find(key);
        if (f != epoch.end() && f->second >= val && t.clk[e] != 0) return ORACLE_ERR_CLOCK_ORDER;
        epoch[key] = val;
      }
      std::vector<u64> ep_rank, ep_clock;
      for (auto& e : epoch) {
        ep_rank.push_back(e.first);
        ep_clock.push_back(e.second);
        footer_ranks.insert((int)e.first);
      }
      // compress_non_matched_events (:627-703).
      body.put_i32(t.set_id);
      body.put_i32(t.count);
      body.put_u64(8 * ep_rank.size());
      body.put(ep_rank.data(), 8 * ep_rank.size());
      body.put(ep_clock.data(), 8 * ep_clock.size());
      if (rep) {
        // rempi_encoder_rep::compress_non_matched_events (:88-133): wp length/size, mi
        // length/size, uid size, ucnt size all 0; compress_matched_events (:137-145): pair size 0.
        for (int k = 0; k < 7; k++) body.put_u64(0);
        continue;
      }
      std::vector<u64> wp = t.with_prev;
      lp_forward(wp);
      body.put_u64(wp.size());
      body.put_u64(8 * wp.size());
      body.put(wp.data(), 8 * wp.size());
      body.put_u64(t.mindex.size());
      body.put_u64(8 * t.mindex.size());
      body.put(t.mindex.data(), 8 * t.mindex.size());
      std::vector<u64> uid = t.um_id;
      lp_forward(uid);
      body.put_u64(8 * uid.size());
      body.put(uid.data(), 8 * uid.size());
      body.put_u64(8 * t.um_cnt.size());
      body.put(t.um_cnt.data(), 8 * t.um_cnt.size());
      // compress_matched_events (:706-721) -> compress (rempi_clock_delta_compression.cpp:465-672).
      std::vector<int32_t> ids, dl;
      int64_t P = cdc_pairs(c.data(), M, ids, dl);
      std::vector<uint32_t> uids(ids.begin(), ids.end()), udl(dl.begin(), dl.end());
      lp_forward(uids);
      lp_forward(udl);
      body.put_u64(8 * (u64)P);
      body.put(uids.data(), 4 * P);
      body.put(udl.data(), 4 * P);
    }
    out.put_u64(body.b.size());
    out.put(body.b.data(), body.b.size());
    return ORACLE_OK;
  }

  // rempi_encoder_cdc::write_footer (:2085-2126); no request-manager map in this path.
  void emit_footer() {
    out.put_u64(0);
    out.put_u64(footer_ranks.size());
    for (int r : footer_ranks) out.put_i32(r);
    out.put_i32(0);
  }

  // The chunk loop of rempi_io_thread::write_record (rempi_io_thread.cpp:56-97) with
  // extract_encoder_input_format_chunk (rempi_encoder_cdc.cpp:740-778).
  int run(const int32_t* rec, size_t n) {
    size_t pos = 0;
    while (pos < n) {
      std::map<int32_t, Table> tabs;
      int64_t length = 0;
      const int32_t* last = nullptr;
      while (pos < n) {
        if (length > max_len && last[F_WITH_NEXT] == 0) break;
        last = rec + 8 * pos;
        length += add(tabs, last);
        pos++;
      }
      int rc = emit_chunk(tabs, last);
      if (rc) return rc;
    }
    emit_footer();
    return ORACLE_OK;
  }
};

// ---------------------------------------------------------------------------------------
// Decoder side.
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <class T> T get() {
    T v{};
    if ((size_t)(end - p) < sizeof(T)) { ok = false; return v; }
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  const uint8_t* take(u64 n) {
    if ((u64)(end - p) < n) { ok = false; return nullptr; }
    const uint8_t* q = p;
    p += n;
    return q;
  }
};

struct DecodedTable {
  int32_t set_id = 0, count = 0;
  std::vector<u64> ep_rank, ep_clock, with_prev, mindex, ids, delays;
  std::vector<std::pair<u64, u64>> unmatched;  // (id, count) sorted by id
  std::vector<int32_t> perm;
};

// cdc_prepare_decode_indices (rempi_encoder_cdc.cpp:1301-1386): start from the list
// 0..M-1; for each pair, take `id` out, step `delay` nodes from its old successor and put
// it back in front of that node.  perm[v] = final position of v.  The list is circular
// with a sentinel (index M) as libstdc++'s std::list is.
// 0 (default): a delay that walks more than once round the list is refused, as the device path
// refuses it; 1: walk on through the sentinel however far, as std::advance on libstdc++'s
// circular std::list does in the reference (oracle_set_reference_walk).
static int g_reference_walk = 0;

int decode_perm(const u64* ids, const u64* delays, int64_t P, int64_t M, int32_t* perm) {
  std::vector<int64_t> nx(M + 1), pv(M + 1);
  for (int64_t i = 0; i <= M; i++) {
    nx[i] = (i + 1) % (M + 1);
    pv[i] = (i + M) % (M + 1);
  }
  for (int64_t k = 0; k < P; k++) {
    int64_t id = (int64_t)(int)ids[k];
    int64_t dl = (int64_t)(int)delays[k];
    if (id < 0 || id >= M) return ORACLE_ERR_CORRUPT;
    // The encoder never writes a delay that walks more than once round the list; the
    // reference would keep stepping through the std::list sentinel.  Treated as corrupt so
    // that damaged files cost O(M) per pair at most.
    if (!g_reference_walk && (dl > M || dl < -M)) return ORACLE_ERR_CORRUPT;
    int64_t at = nx[id];
    nx[pv[id]] = nx[id];
    pv[nx[id]] = pv[id];
    for (; dl > 0; dl--) at = nx[at];
    for (; dl < 0; dl++) at = pv[at];
    int64_t before = pv[at];
    nx[before] = id;
    pv[id] = before;
    nx[id] = at;
    pv[at] = id;
  }
  int64_t q = nx[M];
  for (int64_t i = 0; i < M; i++, q = nx[q]) perm[q] = (int32_t)i;
  return ORACLE_OK;
}

// read_record_file (:933-978) + decode (:1016-1299) for one chunk payload.
int decode_chunk(const uint8_t* b, u64 len, std::vector<DecodedTable>& out) {
  Reader rd{b, b + len};
  std::map<int32_t, DecodedTable> tabs;  // test_tables_map (ascending id)
  while (rd.ok && rd.p < rd.end) {
    DecodedTable t;
    t.set_id = rd.get<int32_t>();
    t.count = rd.get<int32_t>();
    u64 esz = rd.get<u64>();
    const uint8_t* er = rd.take(esz);
    const uint8_t* ec = rd.take(esz);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    t.ep_rank.resize(esz / 8);
    t.ep_clock.resize(esz / 8);
    memcpy(t.ep_rank.data(), er, 8 * (esz / 8));
    memcpy(t.ep_clock.data(), ec, 8 * (esz / 8));
    (void)rd.get<u64>();  // with_previous length (the size field is what decode uses)
    u64 wsz = rd.get<u64>();
    const uint8_t* w = rd.take(wsz);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    t.with_prev.resize(wsz / 8);
    memcpy(t.with_prev.data(), w, 8 * (wsz / 8));
    lp_inverse(t.with_prev);
    (void)rd.get<u64>();
    u64 msz = rd.get<u64>();
    const uint8_t* mi = rd.take(msz);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    t.mindex.resize(msz / 8);
    memcpy(t.mindex.data(), mi, 8 * (msz / 8));
    u64 usz = rd.get<u64>();
    const uint8_t* ui = rd.take(usz);
    u64 csz = rd.get<u64>();
    const uint8_t* uc = rd.take(csz);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    std::vector<u64> uid(usz / 8), ucnt(csz / 8);
    memcpy(uid.data(), ui, 8 * uid.size());
    memcpy(ucnt.data(), uc, 8 * ucnt.size());
    lp_inverse(uid);
    if (csz > 0) {
      std::map<u64, u64> um;
      for (size_t i = 0; i < uid.size() && i < ucnt.size(); i++) um[uid[i]] = ucnt[i];
      t.unmatched.assign(um.begin(), um.end());
    }
    u64 psz = rd.get<u64>();
    const uint8_t* pb = rd.take(psz);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    u64 P = psz / 4 / 2;
    t.ids.resize(P);
    t.delays.resize(P);
    for (u64 k = 0; k < P; k++) {
      int32_t a, d;
      memcpy(&a, pb + 4 * k, 4);
      memcpy(&d, pb + 4 * (P + k), 4);
      t.ids[k] = as_size_t(a);
      t.delays[k] = as_size_t(d);
    }
    lp_inverse(t.ids);
    lp_inverse(t.delays);
    if (t.count < 0) return ORACLE_ERR_CORRUPT;
    t.perm.assign(t.count, 0);
    int rc = decode_perm(t.ids.data(), t.delays.data(), (int64_t)P, t.count, t.perm.data());
    if (rc) return rc;
    tabs[t.set_id] = std::move(t);
  }
  if (!rd.ok) return ORACLE_ERR_CORRUPT;
  for (auto& kv : tabs) out.push_back(std::move(kv.second));
  return ORACLE_OK;
}

// Walks [size_t len][payload]... [size_t 0][footer] (A12/A13).
template <class F>
int for_each_chunk(const uint8_t* in, size_t len, F&& f) {
  Reader rd{in, in + len};
  while (true) {
    u64 n = rd.get<u64>();
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    if (n == 0) break;
    const uint8_t* b = rd.take(n);
    if (!rd.ok) return ORACLE_ERR_CORRUPT;
    int rc = f(b, n);
    if (rc) return rc;
  }
  u64 nr = rd.get<u64>();
  rd.take(4 * nr);
  (void)rd.get<int32_t>();
  return rd.ok ? ORACLE_OK : ORACLE_ERR_CORRUPT;
}

template <class T>
int give(const std::vector<T>& v, T** out, size_t* n) {
  *n = v.size();
  *out = static_cast<T*>(malloc(sizeof(T) * (v.size() ? v.size() : 1)));
  if (!*out) return ORACLE_ERR_ARG;
  if (!v.empty()) memcpy(*out, v.data(), sizeof(T) * v.size());
  return ORACLE_OK;
}

}  // namespace

extern "C" {

int oracle_encode(const int32_t* rec, size_t n, int64_t max_len, uint8_t** out, size_t* out_len,
                  size_t* footer_off) {
  return oracle_encode_ex(rec, n, max_len, 0, out, out_len, footer_off);
}

int oracle_encode_ex(const int32_t* rec, size_t n, int64_t max_len, int rep, uint8_t** out, size_t* out_len,
                     size_t* footer_off) {
  if (!out || !out_len || (n && !rec)) return ORACLE_ERR_ARG;
  Encoder e;
  e.max_len = max_len;
  e.rep = rep;
  size_t pos = 0;
  // run() inline so the footer offset can be reported.
  while (pos < n) {
    std::map<int32_t, Table> tabs;
    int64_t length = 0;
    const int32_t* last = nullptr;
    while (pos < n) {
      if (length > max_len && last[F_WITH_NEXT] == 0) break;
      last = rec + 8 * pos;
      length += Encoder::add(tabs, last);
      pos++;
    }
    int rc = e.emit_chunk(tabs, last);
    if (rc) return rc;
  }
  if (footer_off) *footer_off = e.out.b.size();
  e.emit_footer();
  return give(e.out.b, out, out_len);
}

int oracle_decode(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len) {
  Sink d;
  auto v = [&](int64_t x) { d.put(&x, 8); };
  auto vec = [&](const auto& a) {
    v((int64_t)a.size());
    for (auto x : a) v((int64_t)x);
  };
  int rc = for_each_chunk(in, len, [&](const uint8_t* b, u64 n) {
    std::vector<DecodedTable> tabs;
    int r = decode_chunk(b, n, tabs);
    if (r) return r;
    v((int64_t)tabs.size());
    for (auto& t : tabs) {
      v(t.set_id);
      v(t.count);
      vec(t.ep_rank);
      vec(t.ep_clock);
      vec(t.with_prev);
      vec(t.mindex);
      v((int64_t)t.unmatched.size());
      for (auto& p : t.unmatched) { v((int64_t)p.first); v((int64_t)p.second); }
      vec(t.ids);
      vec(t.delays);
      vec(t.perm);
    }
    return ORACLE_OK;
  });
  if (rc) return rc;
  return give(d.b, out, out_len);
}

int oracle_cdc_pairs(const int32_t* c, int64_t M, int32_t* ids, int32_t* deltas, int64_t* P) {
  if (M < 0 || (M && (!c || !ids || !deltas)) || !P) return ORACLE_ERR_ARG;
  std::vector<int32_t> a, d;
  *P = cdc_pairs(c, M, a, d);
  std::copy(a.begin(), a.end(), ids);
  std::copy(d.begin(), d.end(), deltas);
  return ORACLE_OK;
}

void oracle_set_reference_walk(int on) { g_reference_walk = on != 0; }

int oracle_decode_perm(const int64_t* ids, const int64_t* delays, int64_t P, int64_t M, int32_t* perm) {
  std::vector<u64> a(ids, ids + P), d(delays, delays + P);
  return decode_perm(a.data(), d.data(), P, M, perm);
}

int64_t oracle_umap_order(const int64_t* keys, int64_t n, int64_t* out) {
  std::unordered_map<size_t, size_t> m;
  for (int64_t i = 0; i < n; i++) m[(size_t)keys[i]] = 0;
  int64_t k = 0;
  for (auto& e : m) out[k++] = (int64_t)e.first;
  return k;
}

int64_t oracle_uset_int_order(const int32_t* keys, int64_t n, int32_t* out) {
  std::unordered_set<int> s;
  for (int64_t i = 0; i < n; i++) s.insert(keys[i]);
  int64_t k = 0;
  for (int v : s) out[k++] = v;
  return k;
}

int oracle_sorted_keys(const int32_t* rec, size_t n, int64_t max_len, int32_t** keys, size_t* n_keys) {
  std::vector<int32_t> kv;
  size_t pos = 0;
  while (pos < n) {
    std::map<int32_t, Table> tabs;
    int64_t length = 0;
    const int32_t* last = nullptr;
    while (pos < n) {
      if (length > max_len && last[F_WITH_NEXT] == 0) break;
      last = rec + 8 * pos;
      length += Encoder::add(tabs, last);
      pos++;
    }
    for (auto& t : tabs) {
      const Table& tb = t.second;
      std::vector<int32_t> order(tb.src.size());
      for (size_t i = 0; i < order.size(); i++) order[i] = (int32_t)i;
      std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        if (tb.clk[a] != tb.clk[b]) return tb.clk[a] < tb.clk[b];
        return tb.src[a] < tb.src[b];
      });
      for (int32_t e : order) { kv.push_back(tb.src[e]); kv.push_back(tb.clk[e]); }
    }
  }
  size_t cnt;
  int rc = give(kv, keys, &cnt);
  *n_keys = cnt / 2;
  return rc;
}

int oracle_reconstruct(const uint8_t* in, size_t len, const int32_t* sorted_keys, size_t n_keys,
                       int32_t** out, size_t* n_out) {
  std::vector<int32_t> recs;
  size_t kpos = 0;
  int rc = for_each_chunk(in, len, [&](const uint8_t* b, u64 n) {
    std::vector<DecodedTable> tabs;
    int r = decode_chunk(b, n, tabs);
    if (r) return r;
    for (auto& t : tabs) {
      const int64_t M = t.count;
      if (kpos + (size_t)M > n_keys) return ORACLE_ERR_ARG;
      std::vector<int32_t> c(M);
      for (int64_t v = 0; v < M; v++) c[t.perm[v]] = (int32_t)v;  // row -> clock order
      std::vector<uint8_t> wn(M, 0);
      for (u64 w : t.with_prev) if ((int64_t)w < M) wn[w] = 1;
      size_t ui = 0;
      for (int64_t i = 0; i <= M; i++) {
        while (ui < t.unmatched.size() && (int64_t)t.unmatched[ui].first == i) {
          int32_t r8[8] = {(int32_t)t.unmatched[ui].second, 2, 0, 0, 0, 0, 0, t.set_id};
          recs.insert(recs.end(), r8, r8 + 8);
          ui++;
        }
        if (i == M) break;
        const int32_t* k = sorted_keys + 2 * (kpos + c[i]);
        int32_t r8[8] = {1, 2, 1, k[0], wn[i], (int32_t)t.mindex[i], k[1], t.set_id};
        recs.insert(recs.end(), r8, r8 + 8);
      }
      kpos += M;
    }
    return ORACLE_OK;
  });
  if (rc) return rc;
  size_t cnt;
  rc = give(recs, out, &cnt);
  *n_out = cnt / 8;
  return rc;
}

void oracle_free(void* p) { free(p); }

}  // extern "C"
