// api.hip -- host orchestration of the CDC kernels and the C ABI of include/cdcx.h.
//
// The host side only sequences launches, sizes buffers and lays out offsets; every byte
// of codec output is produced by the device kernels.  There is no CPU fallback: if the
// device or a launch fails the call returns CDCX_ERR_HIP.
#include <hip/hip_runtime.h>

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cdcx.h"
#include "cdcx_kernels.h"
#include "gzip_stage.h"
#include "hash_order.h"

using namespace cdcx;

namespace {

enum KernelId {
  K_SET_DENSE, K_TILE_HIST, K_HIST_SCAN, K_SCATTER, K_RANK_SCAN,
  K_CHUNKS, K_UNITS_LB, K_LISTS, K_UNIT_PREP, K_WINDOW_RANK, K_SORT_TILES, K_RANK_TILES, K_EPOCH, K_CUTS, K_SEG_LIST, K_SEG_SORT, K_CHAIN_G8, K_CHAIN_G16, K_CHAIN_G64, K_CHAIN_SEG, K_CHAIN_EXITS, K_CHAIN_ENTRIES, K_CHAIN_MARK, K_POSITIONS, K_DELTAS,
  K_WRITE_UNITS, K_CHUNK_HEADERS, K_FOOTER_ORDER, K_FOOTER_WRITE, K_WRITE_KEYS,
  K_DEC_COUNT_CHUNKS, K_DEC_LIST_CHUNKS, K_DEC_UNITS, K_DEC_SECTIONS, K_DEC_PAIRS, K_DEC_SEG, K_DEC_REDO, K_DEC_CHECK, K_DEC_WIN1, K_DEC_WIN4, K_DEC_PERM, K_DEC_RECORDS, K_DEC_PACK, K_VERIFY,
  K_GEN_TILE_SUMS, K_GEN_RANK_SCAN, K_GEN_FRAMES, K_GEN_AKEYS, K_GEN_ARRIVAL, K_GEN_RECORDS,
  K_COUNT
};
const char* kKernelNames[K_COUNT] = {
  "k_set_dense", "k_tile_hist", "k_hist_scan", "k_scatter", "k_rank_scan",
  "k_chunks", "k_units_lb", "k_lists", "k_unit_prep", "k_window_rank", "k_sort_tiles", "k_rank_tiles", "k_epoch", "k_cuts", "k_seg_list", "k_seg_sort", "k_chain_grp8", "k_chain_grp16", "k_chain_grp64", "k_chain_seg", "k_chain_exits", "k_chain_entries", "k_chain_mark",
  "k_positions", "k_deltas", "k_write_units", "k_chunk_headers", "k_footer_order", "k_footer_write", "k_write_keys",
  "k_dec_count_chunks", "k_dec_list_chunks", "k_dec_units", "k_dec_sections", "k_dec_pair_scan", "k_dec_perm_seg", "k_dec_perm_redo", "k_dec_perm_check", "k_dec_perm_grp", "k_dec_perm_window4", "k_dec_perm_lane", "k_dec_records", "k_dec_pack_tables", "k_verify_roundtrip",
  "k_gen_tile_sums", "k_gen_rank_scan", "k_gen_frames", "k_gen_akeys", "k_gen_arrival", "k_gen_records"};

struct HipError {
  hipError_t e;
  const char* what;
};
struct CdcxError {
  int code;
  std::string msg;
};

#define HIPCHK(x)                                 \
  do {                                            \
    hipError_t e_ = (x);                          \
    if (e_ != hipSuccess) throw HipError{e_, #x}; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Decode scratch lives in encode scratch that is dead by then (one context = one stream,
// encode and decode never overlap): grow-only named buffers shared by both phases.
constexpr const char* kAliasRecs = "dec_recs"; // decoded records: a buffer of their own (the T-order records keep the
                                              // stream positions that cdcx_verify_roundtrip_device maps them by)
constexpr const char* kAliasIdd = "mkey";     // pair ids              <- observed-order keys
constexpr const char* kAliasDld = "chainbuf"; // pair delays           <- chain / edit-sequence scratch (the clock-order keys, "skey", are the decoder's input)
constexpr const char* kAliasWpd = "run_cnt";  // with_previous         <- unmatched run counts
constexpr const char* kAliasUidd = "cuts2";   // unmatched ids         <- segment ends / first untaken columns / edit-sequence ids
constexpr const char* kAliasPerm = "cord";    // perm                  <- clock order of rows
constexpr const char* kAliasCinv = "inv";     // perm^-1               <- row of each clock
constexpr const char* kAliasWnf = "chain";    // with_next flags       <- chain flags

}  // namespace

// ---------------------------------------------------------------------------------------
// Scratch of the entry point that allocates nothing (cdcx_decode_chunk_perm_static): one
// file-scope device array per GPU, carved into the unit table, the pair rows and the list
// links of one chunk.  `scratch` is only a host-side handle: its device address is looked up
// once per device in cdcx_create (static_scratch_of) and kept; kernels, copies and fills
// always get that address.
namespace {
constexpr int32_t kStaticMaxUnits = 256;          // tables per chunk (matching_set_id < 256)
constexpr int64_t kStaticMaxRows = 262144;        // sum over the chunk's tables of count + 1
constexpr size_t kStaticHdrOff = 0;               // int32[64] header
constexpr size_t kStaticOrderOff = 256;           // int32[kStaticMaxUnits]
constexpr size_t kStaticUnitsOff = kStaticOrderOff + 4 * kStaticMaxUnits;
constexpr size_t kStaticIddOff = (kStaticUnitsOff + sizeof(DUnit) * kStaticMaxUnits + 255) / 256 * 256;
constexpr size_t kStaticDldOff = kStaticIddOff + 8 * kStaticMaxRows;
constexpr size_t kStaticCinvOff = kStaticDldOff + 8 * kStaticMaxRows;
constexpr size_t kStaticNxOff = kStaticCinvOff + 4 * kStaticMaxRows;
constexpr size_t kStaticPvOff = kStaticNxOff + 4 * kStaticMaxRows;
constexpr size_t kStaticScratchBytes = kStaticPvOff + 4 * kStaticMaxRows;  // ~7.0 MiB
}  // namespace
static __device__ __align__(256) unsigned char scratch[kStaticScratchBytes];
namespace {
constexpr int kMaxDevices = 64;
std::mutex g_static_mu;
unsigned char* g_static_scratch[kMaxDevices] = {};  // device address of `scratch` on each GPU

// Device address of this GPU's copy of `scratch` (the device must be current).
hipError_t static_scratch_of(int device, unsigned char** out) {
  std::lock_guard<std::mutex> g(g_static_mu);
  if (device < 0 || device >= kMaxDevices) return hipErrorInvalidDevice;
  if (!g_static_scratch[device]) {
    void* p = nullptr;
    const hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
    if (e != hipSuccess) return e;
    g_static_scratch[device] = static_cast<unsigned char*>(p);
  }
  *out = g_static_scratch[device];
  return hipSuccess;
}
}  // namespace

// Gate of the kernels that keep every SIMD busy by themselves (the chain simulation, the
// permutation rebuild): the contexts of a process on one device take turns with them.  Two of
// these kernels side by side each run at half speed and leave at the same time, so lanes that
// met in one of them once stay in step ever after -- all in their issue-bound kernels together,
// then all in their bandwidth-bound ones, each resource idle while the other is the limit.
// With one such kernel at a time the lanes spread out, and the other lanes' bandwidth-bound
// kernels run beside it.  A context entering a gate makes its stream wait for the event the
// previous holder recorded behind its kernel; the order is the order of the host calls, so
// the waits cannot form a cycle.
struct Gate {
  std::mutex m;
  // the events behind the latest kernels that went through, newest last, and their contexts;
  // a gate of depth d lets d kernels run side by side: a new one waits for the d-th newest
  hipEvent_t last[4] = {nullptr, nullptr, nullptr, nullptr};
  const void* owner[4] = {nullptr, nullptr, nullptr, nullptr};
};
// 0: chain, 1: permutation rebuild, 2: the scatter (CDCX_GATE bit 3) -- bandwidth-bound; two of
// them side by side share the HBM and both take twice as long, one at a time gives each lane
// its T-order records sooner
constexpr int kGateKinds = 3;
constexpr int kGateDevices = 16;
static Gate g_gates[kGateDevices][kGateKinds];

// Library calls in flight per device (guarded()).  The chain kernel is a work queue whose grid
// decides how much of every CU it holds for its ten-odd milliseconds: five blocks per CU (1280)
// make it fastest alone; beside other contexts' kernels 3.5 per CU (896) leave them the LDS and
// wave slots they are short of, and the step of four lanes is 3 % shorter.
static std::atomic<int> g_calls_in_flight[kGateDevices];
struct InFlight {
  int d;
  explicit InFlight(int dev) : d(dev) {
    if (d >= 0 && d < kGateDevices) g_calls_in_flight[d].fetch_add(1, std::memory_order_relaxed);
  }
  ~InFlight() {
    if (d >= 0 && d < kGateDevices) g_calls_in_flight[d].fetch_sub(1, std::memory_order_relaxed);
  }
  InFlight(const InFlight&) = delete;
  InFlight& operator=(const InFlight&) = delete;
};
inline int64_t chain_blocks(int64_t forced, int device) {
  if (forced > 0) return forced;
  const bool shared = device >= 0 && device < kGateDevices && g_calls_in_flight[device].load(std::memory_order_relaxed) > 1;
  return shared ? 896 : 1280;
}

struct cdcx_ctx {
  int device = 0;
  unsigned char* static_scratch = nullptr;  // this device's `scratch` (static_scratch_of)
  int gzip = 0;  // REMPI_GZIP: host-buffer encode/decode apply the zlib stage (gzip_stage.hip)
  bool rep = false;  // REMPI_ENCODE=7: epoch lines only (rempi_encoder_rep.cpp:50-146)
  int64_t max_len = 131072;
  std::string err;
  std::map<std::string, DevBuf> bufs;
  bool profiling = false;
  std::vector<double> ktime = std::vector<double>(K_COUNT, 0.0);
  std::vector<int64_t> klaunch = std::vector<int64_t>(K_COUNT, 0);
  struct Pending {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
  hipStream_t stream = nullptr;
  struct Pinned {  // grow-only page-locked host buffer
    uint8_t* p = nullptr;
    size_t cap = 0;
  };
  Pinned pin_in, pin_tab;  // replay pipeline: rank files in; packed decoded tables out
  Pinned pin_mail;         // small read-backs between kernels (Mail)

  // results of the last encode
  uint8_t* d_out = nullptr;
  int2* d_keys = nullptr;
  int64_t n_keys = 0;
  std::vector<Unit> enc_units;       // units of the last encode (file order); see host_enc_units
  Unit* d_enc_units = nullptr;       // ... on the device
  int32_t n_enc_units = 0;
  bool enc_units_stale = false;      // enc_units not downloaded yet
  std::vector<int64_t> enc_rec_off;  // record offsets of its ranks
  // results of the last decode
  std::vector<DUnit> dunits;
  std::vector<DChunk> dchunks;
  std::vector<int32_t> dfirst_unit, dnunits;
  std::vector<int32_t> dcbase;  // first chunk of each rank file of the last decode (R + 1)
  // ... the same tables on the device; the host copies above are fetched on demand (host_dec_units)
  DUnit* d_dunits = nullptr;
  DChunk* d_dchunks = nullptr;
  int32_t* d_dnunits = nullptr;
  int32_t* d_dfirst_unit = nullptr;
  int32_t n_dunits = 0, n_dchunks = 0;
  bool dec_host_stale = false;
  hipStream_t dec_stream = nullptr;  // stream of the last decode
  int32_t* d_rec_out = nullptr;
  int64_t n_rec_out = 0;
  int32_t* d_perm = nullptr;
  const int32_t* d_gen = nullptr;
  int32_t last_fallback_units = 0;
  bool chain_stats = getenv("CDCX_CHAIN_STATS") != nullptr;
  // First chain tier (diagnostics / tests): 0 = 16-lane groups, 1 = 64-lane groups, 2 = lane kernel.
  int chain_tier = getenv("CDCX_CHAIN_TIER") ? atoi(getenv("CDCX_CHAIN_TIER")) : 0;
  // First permutation-rebuild tier (diagnostics / tests): 0 = pair segments in 16-lane groups,
  // 1 = whole units in 16-lane groups, 2 = 256-slot window, 3 = sequential list.
  int dec_tier = getenv("CDCX_DEC_TIER") ? atoi(getenv("CDCX_DEC_TIER")) : 0;
  // 1: every unit takes the tile sort (skips the windowed rank), for tests
  int rank_tier = getenv("CDCX_RANK_TIER") ? atoi(getenv("CDCX_RANK_TIER")) : 0;
  // blocks of the first chain tier (a work queue); 0 = by what else runs on the device (chain_blocks())
  int64_t chain_grid = getenv("CDCX_CHAIN_GRID") ? std::max(1, atoi(getenv("CDCX_CHAIN_GRID"))) : 0;
  bool chain_g16 = getenv("CDCX_CHAIN_G16") != nullptr;  // first tier on 16-lane groups (A/B timing)
  // segments of at least this many events run at raised wave priority in the 8-lane chain tier
  int chain_long = getenv("CDCX_CHAIN_LONG") ? atoi(getenv("CDCX_CHAIN_LONG")) : 1536;
  // which bandwidth-bound kernels take turns on gate 2 (bits: tile_hist, scatter, unit_prep, dec_records,
  // positions, write_units, deltas, window_rank)
  int gate_bw = getenv("CDCX_GATE_BW") ? atoi(getenv("CDCX_GATE_BW")) : 2;
  // gates in use: bit 0 chain, bit 1 permutation rebuild, bit 2 both kinds through one gate, bit 3 scatter
  // (on the bench batch: + 1 % over 3 steps from a common start, + 2.7 % over 12 steps)
  int gate_mode = getenv("CDCX_GATE") ? atoi(getenv("CDCX_GATE")) : 11;
  // kernels of a kind allowed side by side (1 .. 4): {chain, permutation rebuild}
  int gate_depth[kGateKinds] = {getenv("CDCX_GATE_CHAIN") ? atoi(getenv("CDCX_GATE_CHAIN")) : 1,
                                getenv("CDCX_GATE_PERM") ? atoi(getenv("CDCX_GATE_PERM")) : 1,
                                getenv("CDCX_GATE_SCATTER") ? atoi(getenv("CDCX_GATE_SCATTER")) : 1};
  hipEvent_t gate_ev[kGateKinds][4] = {};
  int gate_next[kGateKinds] = {};
  // matching-set-id map (cdcx_set_matching_set_id_map), registration order, ids distinct
  std::vector<uint64_t> map_ids;
  std::vector<int32_t> map_sets;
  int64_t chain_tier_counts[3] = {0, 0, 0};  // segments entering each tier in the last encode
  int32_t chain_cnt0[4] = {0, 0, 0, 0};      // (host image of the tiers' counters at launch)
  int64_t enc_totals[8] = {};                // records, matched, runs, with_next, sources, pairs, tables, chunks of the last encode
  int64_t dec_tier_counts[7] = {0, 0, 0, 0, 0, 0, 0};  // tables entering each rebuild tier in the last decode; segments

  template <class T>
  T* buf(const std::string& name, size_t count) {
    DevBuf& b = bufs[name];
    size_t bytes = std::max<size_t>(count * sizeof(T), 64);
    if (bytes > b.cap) {
      if (b.p) HIPCHK(hipFree(b.p));
      b.p = nullptr;
      b.cap = 0;
      size_t want = bytes + bytes / 32;  // (a little room: the ranks of a job differ by a few records)
      if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        if (hipMalloc(&b.p, bytes) != hipSuccess) {
          (void)hipGetLastError();
          throw CdcxError{CDCX_ERR_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes for " + name + " failed"};
        }
        want = bytes;
      }
      b.cap = want;
    }
    return static_cast<T*>(b.p);
  }
  void release(const std::string& name) {
    auto it = bufs.find(name);
    if (it != bufs.end()) {
      if (it->second.p) (void)hipFree(it->second.p);
      bufs.erase(it);
    }
  }
  template <class T>
  T* upload(const std::string& name, const std::vector<T>& v, hipStream_t s) {
    T* d = buf<T>(name, v.size());
    if (!v.empty()) HIPCHK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return d;
  }
  template <class T>
  std::vector<T> download(const T* d, size_t n, hipStream_t s) {
    std::vector<T> v(n);
    if (n) HIPCHK(hipMemcpyAsync(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return v;
  }
  hipEvent_t event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
  }
  template <class K, class... Args>
  void launch(int kid, K kernel, dim3 g, dim3 b, hipStream_t s, Args... args) {
    if (g.x == 0 || g.y == 0 || g.z == 0) return;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (profiling) {
      e0 = event();
      HIPCHK(hipEventRecord(e0, s));
    }
    hipLaunchKernelGGL(kernel, g, b, 0, s, args...);
    HIPCHK(hipGetLastError());
    if (profiling) {
      e1 = event();
      HIPCHK(hipEventRecord(e1, s));
      pending.push_back({kid, e0, e1});
    }
  }
  // launch() of a kernel that passes through gate `kind` (see Gate)
  // `big`: only launches that fill the GPU take turns; a small one (a replay batch of a few
  // hundred tables is bound by latency, not by issue) would only wait.
  template <class K, class... Args>
  void launch_gated(int kind, bool big, int kid, K kernel, dim3 g, dim3 b, hipStream_t s, Args... args) {
    if (!big || !((gate_mode >> (kind == 2 ? 3 : kind)) & 1) || device >= kGateDevices) {
      launch(kid, kernel, g, b, s, args...);
      return;
    }
    Gate& gt = g_gates[device][(gate_mode & 4) ? 0 : kind];
    const int depth = std::min(4, std::max(1, gate_depth[kind]));
    std::lock_guard<std::mutex> lk(gt.m);
    if (gt.last[4 - depth] && gt.owner[4 - depth] != this) HIPCHK(hipStreamWaitEvent(s, gt.last[4 - depth], 0));
    launch(kid, kernel, g, b, s, args...);
    hipEvent_t& e = gate_ev[kind][gate_next[kind]];
    gate_next[kind] = (gate_next[kind] + 1) & 3;
    if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e, s));
    for (int q = 0; q < 3; q++) {
      gt.last[q] = gt.last[q + 1];
      gt.owner[q] = gt.owner[q + 1];
    }
    gt.last[3] = e;
    gt.owner[3] = this;
  }
  void collect(hipStream_t s) {
    HIPCHK(hipStreamSynchronize(s));
    for (auto& p : pending) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
      ktime[p.kid] += ms;
      klaunch[p.kid]++;
      event_pool.push_back(p.a);
      event_pool.push_back(p.b);
    }
    pending.clear();
  }
  void check_err(uint32_t* d_err, hipStream_t s) {
    uint32_t e = 0;
    HIPCHK(hipMemcpyAsync(&e, d_err, 4, hipMemcpyDeviceToHost, s));
    collect(s);
    raise_device_error(e);
  }
  // The batch error word (bit = CDCX_ERR_* code) as an exception; 0 = no error.
  static void raise_device_error(uint32_t e) {
    if (!e) return;
    for (int code : {CDCX_ERR_TRUNCATED_EPOCH, CDCX_ERR_CLOCK_ORDER, CDCX_ERR_LIMIT, CDCX_ERR_CORRUPT}) {
      if (e & (1u << code)) {
        const char* what = code == CDCX_ERR_TRUNCATED_EPOCH ? "The events in this epoch are truncated"
                           : code == CDCX_ERR_CLOCK_ORDER   ? "Later message has smaller clock than earlier message"
                           : code == CDCX_ERR_LIMIT         ? "implementation limit exceeded (set id range or sources per table)"
                                                            : "Record data is broken";
        throw CdcxError{code, what};
      }
    }
    throw CdcxError{CDCX_ERR_CORRUPT, "device error word " + std::to_string(e)};
  }
};

namespace {

template <class F>
int guarded(cdcx_ctx* c, F&& f) {
  if (!c) return CDCX_ERR_ARG;
  try {
    HIPCHK(hipSetDevice(c->device));
    InFlight in_flight(c->device);
    f();
    c->err.clear();
    return CDCX_OK;
  } catch (const HipError& e) {
    c->err = std::string(e.what) + ": " + hipGetErrorString(e.e);
    c->pending.clear();
    return CDCX_ERR_HIP;
  } catch (const CdcxError& e) {
    c->err = e.msg;
    c->pending.clear();
    return e.code;
  } catch (const std::bad_alloc&) {
    c->err = "host allocation failed";
    return CDCX_ERR_NOMEM;
  } catch (const GzipError& e) {
    c->err = std::string("zlib stage: ") + e.msg;
    return CDCX_ERR_CORRUPT;
  }
}

inline unsigned blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

void append_id_map(const cdcx_ctx* c, std::vector<uint8_t>& file);  // (with the footer code below)

// Grow-only page-locked host buffer.
uint8_t* pinned(cdcx_ctx::Pinned& b, size_t bytes) {
  if (bytes > b.cap) {
    if (b.p) HIPCHK(hipHostFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&b.p), want, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      b.p = nullptr;
      throw CdcxError{CDCX_ERR_NOMEM, "pinned host allocation of " + std::to_string(want) + " bytes failed"};
    }
    b.cap = want;
  }
  return b.p;
}

// Several small device arrays read back with one wait, through page-locked memory.
struct Mail {
  cdcx_ctx* c;
  hipStream_t s;
  uint8_t* p;
  size_t used = 0, cap;
  Mail(cdcx_ctx* c_, hipStream_t s_, size_t bytes) : c(c_), s(s_), cap(bytes + 64) { p = pinned(c->pin_mail, cap); }
  size_t add(const void* d, size_t bytes) {
    const size_t off = (used + 7) & ~size_t(7);
    if (off + bytes > cap) throw CdcxError{CDCX_ERR_ARG, "read-back buffer too small"};
    if (bytes) HIPCHK(hipMemcpyAsync(p + off, d, bytes, hipMemcpyDeviceToHost, s));
    used = off + bytes;
    return off;
  }
  const uint8_t* wait() {
    c->collect(s);
    return p;
  }
};
inline void raise_device_error(uint32_t e) { cdcx_ctx::raise_device_error(e); }

// Units of the last encode on the host (downloaded on first use).
const std::vector<Unit>& host_enc_units(cdcx_ctx* c, hipStream_t s) {
  if (c->enc_units_stale) {
    c->enc_units = c->download(c->d_enc_units, (size_t)c->n_enc_units, s);
    c->enc_units_stale = false;
  }
  return c->enc_units;
}

// ---------------------------------------------------------------------------------------
// Encode a batch of rank streams already in device memory.
// Outputs: c->d_out with the rank files at file_off[r] (16-aligned), file_len[r].
//
// The work lists between the kernels (chunks, units, sort tiles, segment offsets, output
// layout) are built on the device (lists.hip).  The host waits three times, each time for a
// few hundred bytes: the chunk and table counts of the ranks, the unit / segment totals, and
// the file offsets with the error word (and the chain tiers' hand-over counts) at the end.
void encode_batch(cdcx_ctx* c, int32_t R, const int32_t* d_rec, const int64_t* rec_off_h, std::vector<int64_t>& file_off,
                  std::vector<int64_t>& file_len, hipStream_t s) {
  const int64_t N = rec_off_h[R];
  const int64_t maxl = c->max_len;
  std::vector<int64_t> rec_off(rec_off_h, rec_off_h + R + 1), nrec(R);
  std::vector<int32_t> tile0(R), ntiles(R);
  int64_t NT = 0;
  for (int r = 0; r < R; r++) {
    nrec[r] = rec_off[r + 1] - rec_off[r];
    // (a record's stream position travels in 30 bits of its T-order record)
    if (nrec[r] > (int64_t)kInfoPos) throw CdcxError{CDCX_ERR_LIMIT, "more than 2^30 records in one rank stream"};
    tile0[r] = (int32_t)NT;
    ntiles[r] = (int32_t)((nrec[r] + kTile - 1) / kTile);
    NT += ntiles[r];
    if (NT > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many records in one batch"};
  }
  int64_t* d_rec_off = c->upload("rec_off", rec_off, s);
  int64_t* d_nrec = c->upload("nrec", nrec, s);
  int32_t* d_tile0 = c->upload("tile0", tile0, s);
  int32_t* d_ntiles = c->upload("ntiles", ntiles, s);
  Tile* d_tiles = c->buf<Tile>("tiles", NT);
  c->launch(K_LISTS, k_build_tiles, dim3(R), dim3(256), s, (const int64_t*)d_rec_off, (const int32_t*)d_tile0, d_tiles);
  uint32_t* d_err = c->buf<uint32_t>("err", 1);
  HIPCHK(hipMemsetAsync(d_err, 0, 4, s));

  uint32_t* d_presence = c->buf<uint32_t>("presence", (size_t)R * (kMaxSets / 32));
  HIPCHK(hipMemsetAsync(d_presence, 0, (size_t)R * (kMaxSets / 32) * 4, s));
  int16_t* d_dense = c->buf<int16_t>("dense", (size_t)R * kMaxSets);
  int32_t* d_setlist = c->buf<int32_t>("setlist", (size_t)R * kMaxSets);
  int32_t* d_nsets = c->buf<int32_t>("nsets", R);
  uint32_t* d_hist = c->buf<uint32_t>("hist", NT * kMaxSets);
  int32_t* d_base = c->buf<int32_t>("base", NT * kMaxSets);
  int32_t* d_tstart = c->buf<int32_t>("tstart", (size_t)R * (kMaxSets + 1));
  uint8_t* d_prevm = c->buf<uint8_t>("prevm", NT * kMaxSets);
  TRec* d_trec = c->buf<TRec>("trec", N);
  uint8_t* d_inc0 = c->buf<uint8_t>("inc0s", NT * kTile);  // per tile: a rank's flags start kTile-aligned
  int32_t* d_tsum = c->buf<int32_t>("tsum", NT);
  int32_t* d_toff = c->buf<int32_t>("toff", NT);
  int32_t* d_rtot = c->buf<int32_t>("rtot", R);
  std::vector<int64_t> ccap_off(R + 1, 0);
  for (int r = 0; r < R; r++) ccap_off[r + 1] = ccap_off[r] + nrec[r] / (maxl + 1 > 0 ? maxl + 1 : 1) + 2;
  int64_t* d_ccap = c->upload("ccap_off", ccap_off, s);
  int2* d_chunk_cap = c->buf<int2>("chunk_cap", ccap_off[R]);
  int32_t* d_nchunks = c->buf<int32_t>("nchunks", R);

  c->launch_gated(2, NT >= 65536 && (c->gate_bw & 1), K_TILE_HIST, k_tile_hist, dim3(NT), dim3(256), s, d_rec, (const Tile*)d_tiles, d_hist, d_presence, d_err);
  c->launch(K_SET_DENSE, k_set_dense, dim3(R), dim3(kMaxSets), s, (const uint32_t*)d_presence, d_dense, d_setlist, d_nsets);
  c->launch(K_HIST_SCAN, k_hist_scan, dim3(R), dim3(256), s, (const uint32_t*)d_hist, (const int32_t*)d_tile0,
            (const int32_t*)d_ntiles, (const int32_t*)d_nsets, (const int32_t*)d_setlist, d_base, d_tstart, d_prevm);
  // (the scatter also forms the records' length increments and their tile sums)
  c->launch_gated(2, NT >= 65536 && (c->gate_bw & 2), K_SCATTER, k_scatter, dim3(NT), dim3(256), s, d_rec, (const Tile*)d_tiles, (const int16_t*)d_dense,
            (const int32_t*)d_base, (const uint8_t*)d_prevm, (const int32_t*)d_nsets, (const int64_t*)d_rec_off, d_trec,
            d_inc0, d_tsum);
  c->launch(K_RANK_SCAN, k_rank_scan, dim3(R), dim3(256), s, (const int32_t*)d_tsum, (const int32_t*)d_tile0,
            (const int32_t*)d_ntiles, d_toff, d_rtot);
  c->launch(K_CHUNKS, k_chunks, dim3(R), dim3(64), s, d_rec, (const int64_t*)d_rec_off, (const int64_t*)d_nrec,
            (const int32_t*)d_toff, (const int32_t*)d_rtot, (const int32_t*)d_tile0, (const uint8_t*)d_inc0,
            (const TRec*)d_trec, (const int32_t*)d_tstart, (const int32_t*)d_nsets, (const int64_t*)d_ccap, maxl,
            d_chunk_cap, d_nchunks);

  // Wait 1: tables and chunks per rank -> number of chunks and of (chunk, table) slots.
  std::vector<int32_t> cbase(R + 1, 0);
  std::vector<int64_t> lbase(R + 1, 0);
  {
    Mail m(c, s, 64 + 8 * (size_t)R);
    const size_t o_err = m.add(d_err, 4), o_ns = m.add(d_nsets, 4 * (size_t)R), o_nc = m.add(d_nchunks, 4 * (size_t)R);
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    const int32_t* nsets = reinterpret_cast<const int32_t*>(h + o_ns);
    const int32_t* nchunks = reinterpret_cast<const int32_t*>(h + o_nc);
    for (int r = 0; r < R; r++) {
      if ((int64_t)cbase[r] + nchunks[r] > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many chunks in one batch"};
      cbase[r + 1] = cbase[r] + nchunks[r];
      lbase[r + 1] = lbase[r] + (int64_t)nchunks[r] * nsets[r];
    }
  }
  const int32_t C = cbase[R];
  const int64_t lbn = lbase[R];  // upper bound of the unit count: empty tables of a chunk are skipped
  if (lbn > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many tables in one batch"};
  int32_t* d_cbase = c->upload("cbase", cbase, s);
  int64_t* d_lbase = c->upload("lbase", lbase, s);
  Chunk* d_chunks = c->buf<Chunk>("chunks", C);
  int64_t* d_lb_off = c->buf<int64_t>("lb_off", C);
  int2* d_lohi = c->buf<int2>("lohi", lbn);
  int32_t* d_ucnt = c->buf<int32_t>("ucnt", C);
  int64_t* d_uw = c->buf<int64_t>("uw", C);
  int64_t* d_cw1 = c->buf<int64_t>("cw1", C);
  int32_t* d_ufirst = c->buf<int32_t>("ufirst", R);
  int32_t* d_nunits = c->buf<int32_t>("nunits", R);
  EncTotals* d_tot = c->buf<EncTotals>("enc_totals", 1);
  HIPCHK(hipMemsetAsync(d_tot, 0, sizeof(EncTotals), s));
  // Units past the batch's count stay all-zero: the per-unit kernels before the count is
  // known run over `lbn` units and find nothing to do in those.
  Unit* d_units = c->buf<Unit>("units", lbn);
  HIPCHK(hipMemsetAsync(d_units, 0, (size_t)lbn * sizeof(Unit), s));
  int64_t* d_w1 = c->buf<int64_t>("w1", lbn);
  c->launch(K_LISTS, k_build_chunks, dim3(R), dim3(256), s, (const int2*)d_chunk_cap, (const int64_t*)d_ccap,
            (const int32_t*)d_nchunks, (const int32_t*)d_nsets, (const int32_t*)d_cbase, (const int64_t*)d_lbase, d_chunks,
            d_lb_off);
  c->launch(K_UNITS_LB, k_units_lb, dim3(C), dim3(kMaxSets), s, (const Chunk*)d_chunks, C, (const int64_t*)d_lb_off,
            (const int32_t*)d_nsets, (const int32_t*)d_tstart, (const int64_t*)d_rec_off, (const TRec*)d_trec, d_lohi,
            d_ucnt, d_uw);
  c->launch(K_LISTS, k_scan_chunks, dim3(1), dim3(kScanBlock), s, d_chunks, C, (const int32_t*)d_ucnt, (const int64_t*)d_uw,
            (const int32_t*)d_cbase, R, d_ufirst, d_nunits, d_cw1, d_tot);
  c->launch(K_LISTS, k_fill_units, dim3(C), dim3(kMaxSets), s, (const Chunk*)d_chunks, (const int64_t*)d_lb_off,
            (const int2*)d_lohi, (const int32_t*)d_nsets, (const int32_t*)d_setlist, (const int64_t*)d_rec_off,
            (const int64_t*)d_cw1, d_units, d_w1);
  // (one more word per table: the lane tier's leaf lists and the chain exits live here once the ranks are known)
  uint64_t* d_mkey = c->buf<uint64_t>("mkey", (size_t)(N + lbn));
  int32_t* d_midx = c->buf<int32_t>("midx", N);
  int32_t* d_wp = c->buf<int32_t>("wp", N);
  int32_t* d_run_id = c->buf<int32_t>("run_id", N);
  uint64_t* d_run_cnt = c->buf<uint64_t>("run_cnt", N);
  c->launch_gated(2, NT >= 65536 && (c->gate_bw & 4), K_UNIT_PREP, k_unit_prep, dim3((unsigned)lbn), dim3(256), s, d_units, (const TRec*)d_trec, d_mkey, d_midx, d_wp,
            d_run_id, d_run_cnt, d_err);

  // Clock-order rank: the windowed pass for every unit (tiles of kSortTile events); the units
  // it flags (wfail) are ranked again by the tile sort after the next wait, then get their
  // epoch line and cuts (both skip flagged units until then).
  c->launch(K_LISTS, k_units_scan_prep, dim3(1), dim3(kScanBlock), s, d_units, (int32_t)c->rank_tier, d_tot);
  const int64_t NSmax = N / kSortTile + lbn;  // >= sum of ceil(M / kSortTile)
  SortTile* d_st = c->buf<SortTile>("sort_tiles", NSmax);
  HIPCHK(hipMemsetAsync(d_st, 0xFF, (size_t)NSmax * sizeof(SortTile), s));  // unit -1: no tile
  c->launch(K_LISTS, k_fill_sort_tiles, dim3((unsigned)lbn), dim3(256), s, (const Unit*)d_units, d_st);
  int32_t* d_cord = c->buf<int32_t>("cord", N);
  int32_t* d_inv = c->buf<int32_t>("inv", N);
  uint64_t* d_skey = c->buf<uint64_t>("skey", N);
  if (c->rank_tier == 0)
  {
    c->launch_gated(2, NT >= 65536 && (c->gate_bw & 128), K_WINDOW_RANK, k_window_rank, dim3((unsigned)NSmax), dim3(256), s, d_units, (const SortTile*)d_st,
              (const uint64_t*)d_mkey, d_cord, d_inv, d_skey);
    c->launch(K_WINDOW_RANK, k_window_rank_wide, dim3((unsigned)lbn), dim3(256), s, d_units, (const uint64_t*)d_mkey, d_cord,
              d_inv, d_skey);
  }
  // Epoch lines: kMaxUnitSources entries per table when that is less than one per record
  // (few large tables, the usual case), else at the table's T-order start.
  const int64_t ep_stride = (lbn * (int64_t)kMaxUnitSources < N) ? kMaxUnitSources : 0;
  const size_t ep_n = ep_stride ? (size_t)(lbn * ep_stride) : (size_t)N;
  uint64_t* d_ep_rank = c->buf<uint64_t>("ep_rank", ep_n);
  uint64_t* d_ep_clk = c->buf<uint64_t>("ep_clk", ep_n);
  // Scratch of the chain and the edit sequence, reused as the phases follow each other:
  //   cuts2    [segend | opn]            (k_cuts -> k_seg_list / the chain tiers), then sx (k_pos_cols -> k_deltas)
  //   chainbuf [par | exta | topg | qn]  (chain tiers -> exits, entries, mark), then [posA | crow | seq] (positions -> deltas)
  //   mkey     observed-order keys       (k_unit_prep -> rank), then the lane tier's leaf lists, then qexit (exits -> entries)
  const size_t Np = (size_t)(N + lbn + 63) / 64 * 64;
  int32_t* d_cuts2 = c->buf<int32_t>("cuts2", 2 * Np);
  int32_t* d_segend = d_cuts2;
  int32_t* d_opn = d_cuts2 + Np;  // column + open flag of every row (k_cuts)
  int64_t* d_bound = c->buf<int64_t>("fbound", R);
  EncTotals tot{};
  std::vector<int64_t> bound(R, 0);
  // Wait 2 (again after the rare re-rank / big-epoch detours): totals and epoch sources per rank.
  auto totals = [&]() {
    HIPCHK(hipMemsetAsync(d_bound, 0, 8 * (size_t)R, s));
    c->launch(K_LISTS, k_units_scan_cuts, dim3(1), dim3(kScanBlock), s, d_units, d_bound, d_tot);
    Mail m(c, s, 64 + sizeof(EncTotals) + 8 * (size_t)R);
    const size_t o_err = m.add(d_err, 4), o_tot = m.add(d_tot, sizeof(EncTotals)), o_b = m.add(d_bound, 8 * (size_t)R);
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    memcpy(&tot, h + o_tot, sizeof(tot));
    memcpy(bound.data(), h + o_b, 8 * (size_t)R);
  };
  auto epoch_cuts = [&](unsigned grid) {
    c->launch(K_EPOCH, k_epoch<512>, dim3(grid), dim3(256), s, d_units, (const uint64_t*)d_skey, d_ep_rank, d_ep_clk, ep_stride, d_err);
    // Chain: closed-prefix segments simulated independently, then stitched (chain.hip).
    c->launch(K_CUTS, k_cuts, dim3(grid), dim3(256), s, d_units, (const int32_t*)d_inv, d_segend, d_opn);
    totals();
  };
  epoch_cuts((unsigned)lbn);
  const int32_t NU = tot.n_units;
  const int64_t NS = tot.n_sort_tiles;
  if (tot.n_fail > 0) {
    std::vector<Unit> units = c->download(d_units, NU, s);
    std::vector<SortTile> fst;
    for (int32_t u = 0; u < NU; u++)
      if (units[u].wfail)
        for (int32_t q = 0; q * kSortTile < units[u].M; q++) fst.push_back(SortTile{u, q});
    SortTile* d_fst = c->upload("sort_tiles_fb", fst, s);
    uint64_t* d_tkey = c->buf<uint64_t>("tkey", N);
    int32_t* d_lrank = c->buf<int32_t>("lrank", N);
    uint64_t* d_tmm = c->buf<uint64_t>("tminmax", 2 * NS);
    c->launch(K_SORT_TILES, k_sort_tiles, dim3((unsigned)fst.size()), dim3(256), s, (const Unit*)d_units,
              (const SortTile*)d_fst, (const uint64_t*)d_mkey, d_tkey, d_lrank, d_tmm);
    c->launch(K_RANK_TILES, k_rank_tiles, dim3((unsigned)fst.size()), dim3(256), s, (const Unit*)d_units,
              (const SortTile*)d_fst, (const uint64_t*)d_mkey, (const uint64_t*)d_tkey, (const int32_t*)d_lrank,
              (const uint64_t*)d_tmm, d_cord, d_inv, d_skey);
    for (Unit& u : units) u.wfail = u.wfail ? 0 : 2;  // epoch and cuts for the re-ranked units only
    d_units = c->upload("units", units, s);
    c->launch(K_EPOCH, k_epoch<512>, dim3(NU), dim3(256), s, d_units, (const uint64_t*)d_skey, d_ep_rank, d_ep_clk, ep_stride, d_err);
    c->launch(K_CUTS, k_cuts, dim3(NU), dim3(256), s, d_units, (const int32_t*)d_inv, d_segend, d_opn);
    c->launch(K_LISTS, k_units_clear_wfail, dim3(blocks(NU, 256)), dim3(256), s, d_units, NU);
    totals();
  }
  if (tot.n_big > 0) {  // > 256 sources in some table
    c->launch(K_EPOCH, k_epoch<2 * kMaxUnitSources>, dim3(NU), dim3(256), s, d_units, (const uint64_t*)d_skey, d_ep_rank,
              d_ep_clk, ep_stride, d_err);
    totals();
  }
  const int64_t nsegs = tot.n_segs;
  if (nsegs > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many segments in one batch"};
  const int64_t key_run = tot.matched;

  // Footer scratch and order: needs the epoch lines only, so it runs ahead of the chain.
  std::vector<int64_t> fk_off(R + 1, 0), fb_off(R + 1, 0);
  int64_t foot_max = 0;
  for (int r = 0; r < R; r++) {
    fk_off[r + 1] = fk_off[r] + bound[r] + 1;
    fb_off[r + 1] = fb_off[r] + (int64_t)hash_bucket_capacity((uint64_t)bound[r]) + 1;
    foot_max += 20 + 4 * bound[r] + 16;
  }
  int64_t* d_fk_off = c->upload("fk_off", fk_off, s);
  int64_t* d_fb_off = c->upload("fb_off", fb_off, s);
  uint64_t* d_fkey = c->buf<uint64_t>("fkey", fk_off[R]);
  int32_t* d_fnext = c->buf<int32_t>("fnext", fk_off[R]);
  int32_t* d_fbucket = c->buf<int32_t>("fbucket", fb_off[R]);
  int32_t* d_fcount = c->buf<int32_t>("fcount", R);
  c->launch(K_FOOTER_ORDER, k_footer_order, dim3(R), dim3(256), s, (const Unit*)d_units,
            (const int32_t*)d_ufirst, (const int32_t*)d_nunits, (const uint64_t*)d_ep_rank, ep_stride, R, (const int64_t*)d_fk_off,
            (const int64_t*)d_fb_off, d_fkey, d_fnext, d_fbucket, d_fcount);

  // Output layout on the device: as soon as the pair counts are known (after the chain), so
  // that k_deltas writes the pair sections straight into the files.  The output buffer is
  // sized for P = M in every unit (a few bytes per record more than the files take).
  const int64_t total_max = 8ll * C + 72ll * NU + 16ll * tot.sources + foot_max +
                            (c->rep ? 0 : 8ll * tot.with_next + 16ll * tot.matched + 16ll * tot.runs);
  uint8_t* d_out = c->buf<uint8_t>("out", total_max);
  // the units' clock-ordered keys, dense in file order since the rank pass: the replay side's key stream
  int2* d_keys = reinterpret_cast<int2*>(d_skey);
  int64_t* d_upre = c->buf<int64_t>("upre", (size_t)NU + 1);
  int64_t* d_cpre = c->buf<int64_t>("cpre", (size_t)C + 1);
  int64_t* d_files = c->buf<int64_t>("file_layout", 3 * (size_t)R + 2);  // file_off[R], file_len[R], foot_off[R], total, table bytes
  auto out_layout = [&] {
    c->launch(K_LISTS, k_out_layout, dim3(1), dim3(kScanBlock), s, d_units, d_chunks, C, (const int32_t*)d_cbase, R,
              (const int32_t*)d_fcount, (int32_t)c->rep, (const EncTotals*)d_tot, d_upre, d_cpre, d_files, d_files + R,
              d_files + 2 * R, d_files + 3 * R);
  };

  if (!c->rep) {  // the rep encoder writes no matched-event sections: no chain, no edit sequence
  Seg* d_segs = c->buf<Seg>("segs", nsegs);
  c->launch(K_SEG_LIST, k_seg_list, dim3(NU), dim3(256), s, (const Unit*)d_units, (const int32_t*)d_segend, d_segs);
  int32_t* d_seghist = c->buf<int32_t>("seghist", 4096);
  int32_t* d_segord = c->buf<int32_t>("segord", nsegs);
  HIPCHK(hipMemsetAsync(d_seghist, 0, 4096 * 4, s));
  c->launch(K_SEG_SORT, k_seg_hist, dim3(blocks(nsegs, 1024)), dim3(256), s, (const Seg*)d_segs, (int32_t)nsegs, d_seghist);
  c->launch(K_SEG_SORT, k_seg_bins, dim3(1), dim3(256), s, d_seghist);
  c->launch(K_SEG_SORT, k_seg_order, dim3(blocks(nsegs, 1024)), dim3(256), s, (const Seg*)d_segs, (int32_t)nsegs, d_seghist,
            d_segord);
  int32_t* d_chainbuf = c->buf<int32_t>("chainbuf", 4 * Np);
  int32_t* d_par = d_chainbuf;
  int32_t* d_exta = d_chainbuf + Np;
  int32_t* d_topg = d_chainbuf + 2 * Np;
  int32_t* d_qn = d_chainbuf + 3 * Np;
  uint8_t* d_chain = c->buf<uint8_t>("chain", N);  // every row written by k_chain_mark
  // Tiers: 8-lane groups with 16 leaf slots; segments whose leaf list outgrows them go to
  // 64-lane groups, then to the lane kernel's exact global-memory path.  Each tier rewrites
  // every output of the segments it takes.
  int32_t* d_cnt = c->buf<int32_t>("chain_cnt", 4);
  int32_t* d_ovf1 = c->buf<int32_t>("chain_ovf1", nsegs);
  int32_t* d_ovf2 = c->buf<int32_t>("chain_ovf2", nsegs);
  {
    c->chain_cnt0[0] = (int32_t)nsegs;
    HIPCHK(hipMemcpyAsync(d_cnt, c->chain_cnt0, sizeof(c->chain_cnt0), hipMemcpyHostToDevice, s));
    const int32_t* list = d_segord;
    const int32_t* nlist = d_cnt;
    int64_t n = nsegs;
    if (c->chain_tier <= 0) {
      // (the 8-lane kernel addresses rows by 32-bit byte offsets)
      if (c->chain_g16 || N >= (int64_t(1) << 30))
        c->launch(K_CHAIN_G16, k_chain_grp<16>,
                  dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(chain_blocks(c->chain_grid, c->device), blocks(n, 64)))), dim3(256), s,
                  (const Unit*)d_units, d_segs, list, nlist, (const int32_t*)d_cord, (const int32_t*)d_opn, d_par, d_exta,
                  d_topg, d_qn, d_ovf1, d_cnt + 1, d_err);
      else
        c->launch_gated(0, n >= 65536, K_CHAIN_G8, k_chain_grp8,
                  dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(chain_blocks(c->chain_grid, c->device), blocks(n, 128)))), dim3(256), s,
                  (const Unit*)d_units, d_segs, list, nlist, (const int32_t*)d_cord, (const int32_t*)d_opn, d_par, d_exta,
                  d_topg, d_qn, d_ovf1, d_cnt + 1, (int32_t)c->chain_long, d_err);
      list = d_ovf1;
      nlist = d_cnt + 1;
    }
    // Every tier reads the number of segments handed to it from the device (d_cnt), so the host
    // does not wait between them; the counts travel back with the file layout at the end.
    if (c->chain_tier <= 1) {
      const int64_t g64 = c->chain_tier <= 0 ? std::min<int64_t>(1024, blocks(nsegs, 4)) : blocks(n, 4);
      c->launch(K_CHAIN_G64, k_chain_grp<64>, dim3((unsigned)std::max<int64_t>(1, g64)), dim3(256), s,
                (const Unit*)d_units, d_segs, list, nlist, (const int32_t*)d_cord, (const int32_t*)d_opn, d_par, d_exta,
                d_topg, d_qn, d_ovf2, d_cnt + 2, d_err);
      list = d_ovf2;
      nlist = d_cnt + 2;
    }
    // The lane tier's exact leaf lists live where the observed-order keys were (the ranks are known).
    int2* d_leaves = reinterpret_cast<int2*>(d_mkey);
    c->launch(K_CHAIN_SEG, k_chain_seg<16>,
              dim3((unsigned)(c->chain_tier >= 2 ? std::max<int64_t>(1, std::min<int64_t>(1024, blocks(nsegs, 256))) : 16)),
              dim3(256), s, (const Unit*)d_units, d_segs, nlist, list, (const int32_t*)d_cord, (const int32_t*)d_opn, d_par,
              d_exta, d_topg, d_qn, d_leaves, (const int64_t*)d_w1, d_err,
              c->chain_stats ? c->buf<unsigned long long>("chain_stats", 8) : (unsigned long long*)nullptr);
  }
  int32_t* d_qexit = reinterpret_cast<int32_t*>(d_mkey);  // (the leaf lists are done with)
  c->launch(K_CHAIN_EXITS, k_chain_exits, dim3((unsigned)std::min<int64_t>(8192, blocks(nsegs, 256))), dim3(256), s,
            (const Unit*)d_units, (const Seg*)d_segs, (int32_t)nsegs, (const int32_t*)d_par, (const int32_t*)d_exta,
            (const int32_t*)d_qn, d_qexit, d_err);
  c->launch(K_CHAIN_ENTRIES, k_chain_entries, dim3(blocks(NU, 64)), dim3(64), s, d_units, NU, d_segs,
            (const int32_t*)d_qexit);
  c->launch(K_CHAIN_MARK, k_chain_mark, dim3((unsigned)std::min<int64_t>(8192, blocks(nsegs, 4))), dim3(256), s, (const Unit*)d_units,
            (const Seg*)d_segs, (int32_t)nsegs, (const int32_t*)d_par, (const int32_t*)d_qn, d_chain);
  out_layout();  // (the pair counts are final: k_chain_entries)
  // (par, exta, topg, qn, segend and opn are done with: k_chain_mark was their last reader)
  int32_t* d_posA = d_chainbuf;
  int32_t* d_crow = d_chainbuf + Np;
  uint32_t* d_seq = reinterpret_cast<uint32_t*>(d_chainbuf + 2 * Np);
  int32_t* d_sx = d_cuts2;
  c->launch_gated(2, NU >= 4096 && (c->gate_bw & 16), K_POSITIONS, k_pos_rows, dim3(NU), dim3(256), s, (const Unit*)d_units, (const int32_t*)d_cord,
            (const uint8_t*)d_chain, d_posA, d_crow);
  c->launch_gated(2, NU >= 4096 && (c->gate_bw & 16), K_POSITIONS, k_pos_cols, dim3(NU), dim3(256), s, (const Unit*)d_units, (const int32_t*)d_inv,
            (const uint8_t*)d_chain, (const int32_t*)d_posA, (const int32_t*)d_crow, d_seq, d_sx);
  c->launch_gated(2, NU >= 4096 && (c->gate_bw & 64), K_DELTAS, k_deltas, dim3(NU), dim3(256), s, (const Unit*)d_units, (const uint32_t*)d_seq, (const int32_t*)d_sx,
            d_out);
  }

  if (c->rep) out_layout();
  c->launch_gated(2, NU >= 4096 && (c->gate_bw & 32), K_WRITE_UNITS, k_write_units, dim3(NU), dim3(256), s, (const Unit*)d_units, (const int32_t*)d_midx,
            (const int32_t*)d_wp, (const int32_t*)d_run_id, (const uint64_t*)d_run_cnt, (const uint64_t*)d_ep_rank,
            (const uint64_t*)d_ep_clk, ep_stride, (int32_t)c->rep, d_out);
  c->launch(K_CHUNK_HEADERS, k_chunk_headers, dim3(blocks(C, 256)), dim3(256), s, (const Chunk*)d_chunks, C, d_out);
  c->launch(K_FOOTER_WRITE, k_footer_write, dim3(blocks(R, 64)), dim3(64), s, (const int64_t*)d_fk_off,
            (const int64_t*)d_fb_off, (const uint64_t*)d_fkey, (const int32_t*)d_fnext, (const int32_t*)d_fbucket,
            (const int32_t*)d_fcount, (const int64_t*)(d_files + 2 * R), R, d_out);
  {  // wait 3: error word, file offsets and lengths, the chain tiers' counts
    Mail m(c, s, 128 + 8 * (3 * (size_t)R + 2));
    const size_t o_err = m.add(d_err, 4), o_f = m.add(d_files, 8 * (3 * (size_t)R + 2));
    const size_t o_cnt = m.add(c->rep ? (const void*)d_err : (const void*)c->buf<int32_t>("chain_cnt", 4), c->rep ? 4 : 12);
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    if (!c->rep) {
      const int32_t* cnt = reinterpret_cast<const int32_t*>(h + o_cnt);
      c->chain_tier_counts[0] = cnt[0];
      c->chain_tier_counts[1] = c->chain_tier <= 0 ? cnt[1] : cnt[0];
      c->chain_tier_counts[2] = c->chain_tier <= 1 ? cnt[2] : cnt[0];
    }
    const int64_t* f = reinterpret_cast<const int64_t*>(h + o_f);
    file_off.assign(f, f + R);
    file_len.assign(f + R, f + 2 * R);
    if (f[3 * R] > total_max) throw CdcxError{CDCX_ERR_CORRUPT, "output layout exceeds its bound"};
    const int64_t fixed = 72ll * NU + 16ll * tot.sources + (c->rep ? 0 : 8ll * tot.with_next + 8ll * tot.matched + 16ll * tot.runs);
    const int64_t totals[8] = {N, tot.matched, tot.runs, tot.with_next, tot.sources, c->rep ? 0 : (f[3 * R + 1] - fixed) / 8, NU, C};
    std::copy(totals, totals + 8, c->enc_totals);
  }
  c->d_out = d_out;
  c->d_keys = d_keys;
  c->n_keys = key_run;
  c->d_enc_units = d_units;
  c->n_enc_units = NU;
  c->enc_units.clear();
  c->enc_units_stale = true;
  c->enc_rec_off = rec_off;
}

// ---------------------------------------------------------------------------------------
// Decode a batch of rank files in device memory (d_in; file r at off[r], len[r], 8-aligned).
//
// The chunk, unit, launch-order and record-tile lists are built on the device (lists.hip); the
// host waits for the chunk counts, the unit count, the scratch totals, the first tier's failure
// count and the error word -- a few words each -- and fetches the unit table itself only when
// a caller asks for the decoded tables (host_dec_units).
void decode_batch(cdcx_ctx* c, int32_t R, const uint8_t* d_in, const std::vector<int64_t>& off,
                  const std::vector<int64_t>& len, const int2* d_keys, int64_t n_keys, bool records, bool pairs,
                  hipStream_t s) {
  for (int r = 0; r < R; r++)
    if (off[r] & 7) throw CdcxError{CDCX_ERR_ARG, "rank files must start 8-byte aligned"};
  int64_t* d_off = c->upload("d_off", off, s);
  int64_t* d_len = c->upload("d_len", len, s);
  uint32_t* d_err = c->buf<uint32_t>("err", 1);
  HIPCHK(hipMemsetAsync(d_err, 0, 4, s));
  int32_t* d_nch = c->buf<int32_t>("d_nchunks", R);
  c->launch(K_DEC_COUNT_CHUNKS, k_dec_count_chunks, dim3(blocks(R, 64)), dim3(64), s, d_in, (const int64_t*)d_off,
            (const int64_t*)d_len, R, d_nch, d_err);
  std::vector<int32_t> cbase(R + 1, 0);
  {
    Mail m(c, s, 64 + 4 * (size_t)R);
    const size_t o_err = m.add(d_err, 4), o_n = m.add(d_nch, 4 * (size_t)R);
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    const int32_t* nch = reinterpret_cast<const int32_t*>(h + o_n);
    for (int r = 0; r < R; r++) {
      if ((int64_t)cbase[r] + nch[r] > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many chunks in one batch"};
      cbase[r + 1] = cbase[r] + nch[r];
    }
  }
  const int32_t C = cbase[R];
  int32_t* d_cbase = c->upload("d_cbase", cbase, s);
  c->dcbase = cbase;
  DChunk* d_ch = c->buf<DChunk>("d_chunks", C);
  c->launch(K_DEC_LIST_CHUNKS, k_dec_list_chunks, dim3(blocks(R, 64)), dim3(64), s, d_in, (const int64_t*)d_off,
            (const int32_t*)d_cbase, (const int32_t*)d_nch, R, d_ch);
  int32_t* d_nu = c->buf<int32_t>("d_nunits", C);
  int32_t* d_fu = c->buf<int32_t>("d_first_unit", C);
  DecTotals* d_tot = c->buf<DecTotals>("dec_totals", 1);
  HIPCHK(hipMemsetAsync(d_tot, 0, sizeof(DecTotals), s));
  c->launch(K_DEC_UNITS, k_dec_units, dim3(blocks(C, 64)), dim3(64), s, d_in, (const DChunk*)d_ch, C,
            (const int32_t*)nullptr, d_nu, (DUnit*)nullptr, d_err);
  c->launch(K_LISTS, k_dec_scan_chunks, dim3(1), dim3(kScanBlock), s, (const int32_t*)d_nu, C, d_fu, d_tot);
  DecTotals tot{};
  auto totals = [&]() {
    Mail m(c, s, 64 + sizeof(DecTotals));
    const size_t o_err = m.add(d_err, 4), o_t = m.add(d_tot, sizeof(DecTotals));
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    memcpy(&tot, h + o_t, sizeof(tot));
  };
  totals();
  if (tot.n_units > INT32_MAX) throw CdcxError{CDCX_ERR_LIMIT, "too many tables in one batch"};
  const int32_t NU = (int32_t)tot.n_units;
  DUnit* d_units = c->buf<DUnit>("d_units", NU);
  int32_t* d_rt0 = c->buf<int32_t>("d_rec_tile0", (size_t)NU + 1);
  c->launch(K_DEC_UNITS, k_dec_units, dim3(blocks(C, 64)), dim3(64), s, d_in, (const DChunk*)d_ch, C, (const int32_t*)d_fu,
            (int32_t*)nullptr, d_units, d_err);
  c->launch(K_LISTS, k_dec_scan_units, dim3(1), dim3(kScanBlock), s, d_units, NU, (int32_t)std::min(std::max(c->dec_tier, 0), 3),
            d_rt0, d_tot);
  totals();
  const int64_t wb = tot.rows, ro = tot.records, ko = tot.keys;
  if (records && n_keys < ko) throw CdcxError{CDCX_ERR_ARG, "fewer sorted keys than matched events in the files"};
  c->d_dunits = d_units;
  c->d_dchunks = d_ch;
  c->d_dnunits = d_nu;
  c->d_dfirst_unit = d_fu;
  c->n_dunits = NU;
  c->n_dchunks = C;
  c->dec_host_stale = true;
  c->dec_stream = s;
  c->dunits.clear();
  uint64_t* d_wpd = c->buf<uint64_t>(kAliasWpd, wb);
  uint64_t* d_uidd = c->buf<uint64_t>(kAliasUidd, wb);
  uint64_t* d_idd = c->buf<uint64_t>(kAliasIdd, wb);  // written by k_dec_pair_scan when somebody reads them
  uint64_t* d_dld = c->buf<uint64_t>(kAliasDld, wb);
  int32_t* d_perm = c->buf<int32_t>(kAliasPerm, ko);
  uint8_t* d_wnf = c->buf<uint8_t>(kAliasWnf, wb);
  HIPCHK(hipMemsetAsync(d_wnf, 0, wb, s));
  c->launch(K_DEC_SECTIONS, k_dec_sections, dim3(NU), dim3(256), s, (const DUnit*)d_units, d_in, d_wpd, d_uidd, d_wnf,
            d_err);
  // Permutation rebuild (decode.hip).  First tier: the pair list of every unit in segments of
  // kSegPairs pairs, one per 16-lane group -- k_dec_pair_scan inverts the pair sections' LP and
  // lays the segments out, k_dec_perm_seg replays them, k_dec_perm_check compares the state every
  // segment started from with the state its predecessor ended in.  Units that do not pass go,
  // whole, to a 16-lane group each, then to the 256-slot settle-when-full window, then to the
  // sequential list.
  const int64_t nsegs = tot.segs;
  int32_t* d_cinv = c->buf<int32_t>(kAliasCinv, ko);
  int32_t* d_nfail = c->buf<int32_t>("d_nfail", 8);  // units leaving tiers 0..2, -, segments not finished / not checking out
  HIPCHK(hipMemsetAsync(d_nfail, 0, 32, s));
  DSeg* d_segs = c->buf<DSeg>("d_segs", nsegs);
  int64_t* d_pcar = c->buf<int64_t>("d_pcar", 4 * nsegs);
  int32_t* d_dump_t = c->buf<int32_t>("d_dump_t", (size_t)nsegs * kSegWin);
  int32_t* d_dump_w = c->buf<int32_t>("d_dump_w", (size_t)nsegs * kSegWin);
  c->launch(K_DEC_PAIRS, k_dec_pair_scan, dim3(NU), dim3(64), s, (const DUnit*)d_units, d_in, 1 | (pairs ? 4 : 0), d_segs,
            d_pcar, d_idd, d_dld);
  c->launch_gated(1, NU >= 4096, K_DEC_SEG, k_dec_perm_seg<1>, dim3(blocks(nsegs, 4)), dim3(64), s, d_units,
                  (const int32_t*)nullptr, (const DSeg*)d_segs, nsegs, 0, d_in, (const int64_t*)d_pcar, d_perm, d_cinv,
                  d_dump_t, d_dump_w, d_nfail);
  // Segments that did not start from their predecessor's final state (a few in 10^5 on the bench
  // traces) run again from that state, twice if the first rerun changed what a neighbour started
  // from; what still differs then sends its unit to the next tier.
  constexpr int32_t kRedoCap = 1024, kRedoRounds = 2;
  int32_t* d_redo = c->buf<int32_t>("d_redo", (size_t)kRedoRounds * (kRedoCap + 1));
  int32_t* d_redone = c->buf<int32_t>("d_redone", NU);
  HIPCHK(hipMemsetAsync(d_redo, 0, sizeof(int32_t) * kRedoRounds * (kRedoCap + 1), s));
  HIPCHK(hipMemsetAsync(d_redone, 0, sizeof(int32_t) * (size_t)NU, s));
  if (nsegs > NU)
    for (int32_t round = 0; round <= kRedoRounds; round++) {
      int32_t* list = round < kRedoRounds ? d_redo + round * (kRedoCap + 1) : nullptr;
      c->launch(K_DEC_CHECK, k_dec_perm_check, dim3(blocks(nsegs, 8)), dim3(256), s, d_units, (const DSeg*)d_segs, nsegs,
                (const int32_t*)d_dump_t, (const int32_t*)d_dump_w, list, kRedoCap, d_redone, d_nfail);
      if (list)
        c->launch(K_DEC_REDO, k_dec_perm_seg<2>, dim3(kRedoCap / 4), dim3(64), s, d_units, (const int32_t*)list,
                  (const DSeg*)d_segs, (int64_t)kRedoCap, 0, d_in, (const int64_t*)d_pcar, d_perm, d_cinv, d_dump_t,
                  d_dump_w, d_nfail);
    }
  c->launch(K_DEC_CHECK, k_dec_perm_inv, dim3(NU), dim3(256), s, (const DUnit*)d_units, (const int32_t*)d_redone,
            (const int32_t*)d_cinv, d_perm);
  // The record tiles are listed while the rebuild runs; the reconstruction itself is launched
  // before the wait for the failure count when no unit can have failed into a later tier.
  int4* d_rt = nullptr;
  int32_t* d_recs = nullptr;
  if (records) {
    d_rt = c->buf<int4>("d_rec_tiles", tot.rec_tiles);
    d_recs = c->buf<int32_t>(kAliasRecs, 8 * ro);
    c->launch(K_LISTS, k_dec_fill_tiles, dim3(NU), dim3(256), s, (const DUnit*)d_units, (const int32_t*)d_rt0,
              (const uint64_t*)d_uidd, d_rt);
  }
  // An input the kernels flagged must not reach the record reconstruction (it trusts the
  // sections' checks and the permutation): the error word travels with the failure count.
  int32_t nf = NU;
  {
    Mail m(c, s, 64);
    const size_t o_err = m.add(d_err, 4), o = m.add(d_nfail, 32);
    const uint8_t* h = m.wait();
    raise_device_error(*reinterpret_cast<const uint32_t*>(h + o_err));
    const int32_t* cnt = reinterpret_cast<const int32_t*>(h + o);
    if (c->dec_tier <= 0) nf = cnt[0];
    c->dec_tier_counts[5] = cnt[5];
    c->dec_tier_counts[6] = cnt[4] + cnt[6];
  }
  c->dec_tier_counts[0] = NU;
  c->dec_tier_counts[1] = nf;
  c->dec_tier_counts[2] = c->dec_tier_counts[3] = 0;
  c->dec_tier_counts[4] = nsegs;
  if (nf > 0) {
    if (!pairs)  // the later tiers read the decoded pair arrays
      c->launch(K_DEC_PAIRS, k_dec_pair_scan, dim3(NU), dim3(64), s, (const DUnit*)d_units, d_in, 2, (DSeg*)nullptr,
                (int64_t*)nullptr, d_idd, d_dld);
    int32_t* d_order = c->buf<int32_t>("d_perm_order", NU);
    c->launch(K_LISTS, k_dec_order, dim3(blocks(NU, 256)), dim3(256), s, (const DUnit*)d_units, NU, d_order);
    c->launch(K_DEC_WIN1, k_dec_perm_seg<0>, dim3(blocks(NU, 4)), dim3(64), s, d_units, (const int32_t*)d_order,
              (const DSeg*)nullptr, (int64_t)NU, 1, d_in, (const int64_t*)nullptr, d_perm, d_cinv, (int32_t*)nullptr,
              (int32_t*)nullptr, d_nfail + 1);
    const int32_t nf1 = c->dec_tier > 1 ? NU : c->download(d_nfail + 1, 1, s)[0];
    c->dec_tier_counts[2] = nf1;
    if (nf1 > 0) {
      c->launch(K_DEC_WIN4, k_dec_perm_window<4>, dim3(NU), dim3(64), s, d_units, NU, 2, (const uint64_t*)d_idd,
                (const uint64_t*)d_dld, d_perm, d_nfail + 2);
      const int32_t nf2 = c->dec_tier > 2 ? NU : c->download(d_nfail + 2, 1, s)[0];
      c->dec_tier_counts[3] = nf2;
      if (nf2 > 0) {
        int32_t* d_nx = c->buf<int32_t>("d_nx", wb);  // the sequential list only exists when needed
        int32_t* d_pv = c->buf<int32_t>("d_pv", wb);
        c->launch(K_DEC_PERM, k_dec_perm_lane, dim3(blocks(NU, 64)), dim3(64), s, (const DUnit*)d_units, NU,
                  (const uint64_t*)d_idd, (const uint64_t*)d_dld, d_nx, d_pv, d_perm, d_err);
      }
    }
    c->launch(K_DEC_PERM, k_dec_cinv, dim3(NU), dim3(256), s, (const DUnit*)d_units, (const int32_t*)d_perm, d_cinv);
    c->check_err(d_err, s);
  }
  c->last_fallback_units = nf;
  c->d_perm = d_perm;
  c->n_rec_out = ro;
  if (records) {
    c->launch_gated(2, NU >= 4096 && (c->gate_bw & 8), K_DEC_RECORDS, k_dec_records, dim3((unsigned)tot.rec_tiles), dim3(256), s, (const DUnit*)d_units,
              (const int4*)d_rt, d_in, (const int32_t*)d_cinv, (const uint8_t*)d_wnf, (const uint64_t*)d_uidd, d_keys,
              (int4*)d_recs);
    c->d_rec_out = d_recs;
  }
  c->check_err(d_err, s);
}

// Unit and chunk tables of the last decode on the host (downloaded on first use).
void host_dec_units(cdcx_ctx* c, hipStream_t s) {
  if (!c->dec_host_stale) return;
  c->dunits = c->download((const DUnit*)c->d_dunits, (size_t)c->n_dunits, s);
  c->dchunks = c->download((const DChunk*)c->d_dchunks, (size_t)c->n_dchunks, s);
  c->dnunits = c->download((const int32_t*)c->d_dnunits, (size_t)c->n_dchunks, s);
  c->dfirst_unit = c->download((const int32_t*)c->d_dfirst_unit, (size_t)c->n_dchunks, s);
  c->dec_host_stale = false;
}

// Host-side table dump of the last decode (tests / drop-in shim): mirrors the fields the
// reference keeps in rempi_encoder_input_format_test_table after decode().
// The decoded per-unit arrays of the last decode, packed on the device (k_dec_pack_tables:
// per unit with_previous[W], unmatched ids[U], ids[P], delays[P]) and copied into pinned
// host memory with perm[] in one D2H each.
struct DecodedTables {
  const uint64_t* pk = nullptr;  // packed words
  std::vector<int64_t> pk_off;   // per unit, into pk
  const int32_t* perm = nullptr;
};

DecodedTables download_tables(cdcx_ctx* c, hipStream_t s) {
  host_dec_units(c, s);
  const int32_t NU = (int32_t)c->dunits.size();
  DecodedTables t;
  t.pk_off.resize(NU + 1);
  int64_t pw = 0, ko = 0;
  for (int32_t q = 0; q < NU; q++) {
    const DUnit& u = c->dunits[q];
    t.pk_off[q] = pw;
    pw += (int64_t)u.W + (u.Uc > 0 ? u.U : 0) + 2ll * u.P;
    ko = std::max(ko, u.key_off + u.M);
  }
  t.pk_off[NU] = pw;
  uint8_t* h = pinned(c->pin_tab, (size_t)(8 * pw + 4 * ko + 8));
  if (NU) {
    int64_t* d_pko = c->upload("d_pack_off", t.pk_off, s);
    uint64_t* d_pk = c->buf<uint64_t>("d_pack", (size_t)pw);
    c->launch(K_DEC_PACK, k_dec_pack_tables, dim3(NU), dim3(256), s, (const DUnit*)c->buf<DUnit>("d_units", 0),
              (const int64_t*)d_pko, (const uint64_t*)c->buf<uint64_t>(kAliasWpd, 0),
              (const uint64_t*)c->buf<uint64_t>(kAliasUidd, 0), (const uint64_t*)c->buf<uint64_t>(kAliasIdd, 0),
              (const uint64_t*)c->buf<uint64_t>(kAliasDld, 0), d_pk);
    if (pw) HIPCHK(hipMemcpyAsync(h, d_pk, 8 * pw, hipMemcpyDeviceToHost, s));
    if (ko) HIPCHK(hipMemcpyAsync(h + 8 * pw, c->d_perm, 4 * ko, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  t.pk = reinterpret_cast<const uint64_t*>(h);
  t.perm = reinterpret_cast<const int32_t*>(h + 8 * pw);
  return t;
}

// Dump of chunks [k0, k1) of the last decode (one rank file's chunks when the batch held
// several).  `in` is the host image of the decoded batch buffer (same offsets as d_in).
void dump_chunks(const cdcx_ctx* c, const DecodedTables& t, const uint8_t* in, int32_t k0, int32_t k1,
                 std::vector<int64_t>& d) {
  std::vector<std::pair<uint64_t, int32_t>> um;  // (unmatched id, position): sorted, last write wins
  for (int32_t k = k0; k < k1; k++) {
    std::map<int32_t, int32_t> bysid;  // test_tables_map: last table with an id wins
    for (int32_t q = 0; q < c->dnunits[k]; q++) bysid[c->dunits[c->dfirst_unit[k] + q].set_id] = c->dfirst_unit[k] + q;
    d.push_back((int64_t)bysid.size());
    for (auto& kv : bysid) {
      const DUnit& u = c->dunits[kv.second];
      const uint64_t* wpd = t.pk + t.pk_off[kv.second];
      const uint64_t* uidd = wpd + u.W;
      const uint64_t* idd = uidd + (u.Uc > 0 ? u.U : 0);
      const uint64_t* dld = idd + u.P;
      um.clear();
      if (u.Uc > 0) {
        for (int32_t i = 0; i < u.U; i++) um.emplace_back(uidd[i], i);
        std::stable_sort(um.begin(), um.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        size_t w = 0;  // keep the last of equal ids (unordered_map operator[] assignment)
        for (size_t i = 0; i < um.size(); i++) {
          if (w && um[w - 1].first == um[i].first) w--;
          um[w++] = um[i];
        }
        um.resize(w);
      }
      const size_t n0 = d.size();
      d.resize(n0 + 10 + 2 * (size_t)u.S + u.W + u.Mi + 2 * um.size() + 2 * (size_t)u.P + u.M);
      int64_t* o = d.data() + n0;
      *o++ = u.set_id;
      *o++ = u.M;
      *o++ = u.S;
      memcpy(o, in + u.ep_off, 8ull * u.S);
      o += u.S;
      *o++ = u.S;
      memcpy(o, in + u.ep_off + 8ll * u.S, 8ull * u.S);
      o += u.S;
      *o++ = u.W;
      memcpy(o, wpd, 8ull * u.W);
      o += u.W;
      *o++ = u.Mi;
      memcpy(o, in + u.mi_off, 8ull * u.Mi);
      o += u.Mi;
      *o++ = (int64_t)um.size();
      for (auto& p : um) {
        uint64_t cnt;
        memcpy(&cnt, in + u.ucnt_off + 8ll * p.second, 8);
        *o++ = (int64_t)p.first;
        *o++ = (int64_t)cnt;
      }
      *o++ = u.P;
      memcpy(o, idd, 8ull * u.P);
      o += u.P;
      *o++ = u.P;
      memcpy(o, dld, 8ull * u.P);
      o += u.P;
      *o++ = u.M;
      const int32_t* pm = t.perm + u.key_off;
      for (int32_t i = 0; i < u.M; i++) o[i] = pm[i];
    }
  }
}

std::vector<int64_t> tables_dump(cdcx_ctx* c, const uint8_t* in, hipStream_t s) {
  std::vector<int64_t> d;
  const DecodedTables tb = download_tables(c, s);  // (fetches the chunk table first)
  dump_chunks(c, tb, in, 0, (int32_t)c->dchunks.size(), d);
  return d;
}

template <class T>
T* host_copy(const std::vector<T>& v) {
  T* p = static_cast<T*>(malloc(std::max<size_t>(v.size() * sizeof(T), 1)));
  if (!p) throw std::bad_alloc();
  if (!v.empty()) memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

}  // namespace

// =========================================================================================
extern "C" {

cdcx_ctx* cdcx_create(const cdcx_opts* opts) {
  cdcx_ctx* c = new (std::nothrow) cdcx_ctx();
  if (!c) return nullptr;
  if (opts) {
    c->device = opts->device;
    if (opts->max_event_length > 0) c->max_len = opts->max_event_length;
    if (opts->gzip != 0 && opts->gzip != 1) {
      delete c;
      return nullptr;
    }
    c->gzip = opts->gzip;
    if (opts->encode != 0 && opts->encode != 4 && opts->encode != 7) {
      delete c;
      return nullptr;
    }
    c->rep = opts->encode == 7;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || c->device < 0 || c->device >= n || hipSetDevice(c->device) != hipSuccess) {
    (void)hipGetLastError();
    delete c;
    return nullptr;
  }
  if (static_scratch_of(c->device, &c->static_scratch) != hipSuccess) {
    (void)hipGetLastError();
    delete c;
    return nullptr;
  }
  return c;
}

void cdcx_destroy(cdcx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (auto& kv : c->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  if (c->pin_in.p) (void)hipHostFree(c->pin_in.p);
  if (c->pin_tab.p) (void)hipHostFree(c->pin_tab.p);
  if (c->pin_mail.p) (void)hipHostFree(c->pin_mail.p);
  if (c->device < kGateDevices)
    for (int k = 0; k < kGateKinds; k++) {
      std::lock_guard<std::mutex> lk(g_gates[c->device][k].m);
      for (int q = 0; q < 4; q++)
        if (g_gates[c->device][k].owner[q] == c) {
          g_gates[c->device][k].last[q] = nullptr;
          g_gates[c->device][k].owner[q] = nullptr;
        }
    }
  for (auto& ks : c->gate_ev)
    for (auto e : ks)
      if (e) (void)hipEventDestroy(e);
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  for (auto& p : c->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  delete c;
}

const char* cdcx_last_error(const cdcx_ctx* c) { return c ? c->err.c_str() : "null context"; }
void cdcx_free(void* p) { free(p); }
int cdcx_kernel_count(void) { return K_COUNT; }
const char* cdcx_kernel_name(int k) { return (k >= 0 && k < K_COUNT) ? kKernelNames[k] : ""; }

int cdcx_encode_batch_device(cdcx_ctx* c, int32_t n_ranks, const int32_t* d_rec, const int64_t* rec_off,
                             const uint8_t** d_out, int64_t* out_off, int64_t* out_len, void* stream) {
  if (!c || n_ranks <= 0 || !rec_off || !d_out || !out_off || !out_len || c->gzip) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    std::vector<int64_t> fo, fl;
    encode_batch(c, n_ranks, d_rec, rec_off, fo, fl, (hipStream_t)stream);
    *d_out = c->d_out;
    std::copy(fo.begin(), fo.end(), out_off);
    std::copy(fl.begin(), fl.end(), out_len);
  });
}

int cdcx_batch_sorted_keys(cdcx_ctx* c, const int32_t** d_keys, int64_t* n_keys) {
  if (!c || !d_keys || !n_keys) return CDCX_ERR_ARG;
  *d_keys = reinterpret_cast<const int32_t*>(c->d_keys);
  *n_keys = c->n_keys;
  return CDCX_OK;
}

int cdcx_encode_stream(cdcx_ctx* c, const int32_t* rec8, size_t n, uint8_t** out, size_t* out_len) {
  if (!c || (n && !rec8) || !out || !out_len) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    hipStream_t s = c->stream;
    int32_t* d = c->buf<int32_t>("h_in", 8 * n);
    if (n) HIPCHK(hipMemcpyAsync(d, rec8, 32 * n, hipMemcpyHostToDevice, s));
    int64_t ro[2] = {0, (int64_t)n};
    std::vector<int64_t> fo, fl;
    encode_batch(c, 1, d, ro, fo, fl, s);
    std::vector<uint8_t> h(fl[0]);
    HIPCHK(hipMemcpyAsync(h.data(), c->d_out + fo[0], fl[0], hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    append_id_map(c, h);
    if (c->gzip) h = gzip_file(h.data(), h.size());
    *out = host_copy(h);
    *out_len = h.size();
  });
}

int cdcx_transcode_basic(cdcx_ctx* c, size_t nf, const uint8_t* const* files, const size_t* lens, uint8_t** outs,
                         size_t* out_lens) {
  if (!c || (nf && (!files || !lens || !outs || !out_lens)) || nf > (size_t)INT32_MAX) return CDCX_ERR_ARG;
  for (size_t f = 0; f < nf; f++) {
    outs[f] = nullptr;
    out_lens[f] = 0;
  }
  return guarded(c, [&] {
    // framing (rempi_encoder_basic.cpp:238-321): chunks of whole 32 B TEST records
    struct Span {
      const uint8_t* p;
      size_t n;
    };
    std::vector<Span> spans;
    std::vector<int64_t> ro(nf + 1, 0);
    for (size_t f = 0; f < nf; f++) {
      const uint8_t* b = files[f];
      size_t p = 0, recs = 0;
      if (lens[f] && !b) throw CdcxError{CDCX_ERR_ARG, "null basic file"};
      while (p < lens[f]) {
        if (lens[f] - p < 8) throw CdcxError{CDCX_ERR_ARG, "truncated basic record file"};
        uint64_t n;
        memcpy(&n, b + p, 8);
        p += 8;
        if (n % 32 || n > lens[f] - p) throw CdcxError{CDCX_ERR_ARG, "basic chunk is not a whole number of records"};
        for (uint64_t k = 0; k < n; k += 32) {
          int32_t type;
          memcpy(&type, b + p + k + 4, 4);
          if (type != 2) throw CdcxError{CDCX_ERR_ARG, "basic record is not a test event (type 2)"};
        }
        if (n) spans.push_back(Span{b + p, (size_t)n});
        recs += n / 32;
        p += n;
      }
      ro[f + 1] = ro[f] + (int64_t)recs;
    }
    hipStream_t s = c->stream;
    int32_t* d = c->buf<int32_t>("h_in", 8 * ro[nf]);
    size_t off = 0;
    for (const Span& sp : spans) {
      HIPCHK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(d) + off, sp.p, sp.n, hipMemcpyHostToDevice, s));
      off += sp.n;
    }
    std::vector<int64_t> fo, fl;
    encode_batch(c, (int32_t)nf, d, ro.data(), fo, fl, s);
    std::vector<std::vector<uint8_t>> h(nf);
    for (size_t f = 0; f < nf; f++) {
      h[f].resize(fl[f]);
      HIPCHK(hipMemcpyAsync(h[f].data(), c->d_out + fo[f], fl[f], hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    for (size_t f = 0; f < nf; f++) {
      append_id_map(c, h[f]);
      if (c->gzip) h[f] = gzip_file(h[f].data(), h[f].size());
      outs[f] = host_copy(h[f]);
      out_lens[f] = h[f].size();
    }
  });
}

int cdcx_encode_chunk(cdcx_ctx* c, const int32_t* rec8, size_t n, uint8_t** payload, size_t* payload_len,
                      int32_t** epoch_ranks, size_t* n_epoch_ranks) {
  if (!c || (n && !rec8) || !payload || !payload_len || !epoch_ranks || !n_epoch_ranks) return CDCX_ERR_ARG;
  const int64_t saved = c->max_len;
  c->max_len = INT64_MAX / 4;
  int rc = guarded(c, [&] {
    hipStream_t s = c->stream;
    std::vector<uint8_t> h;
    if (n) {
      int32_t* d = c->buf<int32_t>("h_in", 8 * n);
      HIPCHK(hipMemcpyAsync(d, rec8, 32 * n, hipMemcpyHostToDevice, s));
      int64_t ro[2] = {0, (int64_t)n};
      std::vector<int64_t> fo, fl;
      encode_batch(c, 1, d, ro, fo, fl, s);
      h.resize(fl[0]);
      HIPCHK(hipMemcpyAsync(h.data(), c->d_out + fo[0], fl[0], hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    std::vector<uint8_t> pl;
    std::vector<int32_t> er;
    if (!h.empty()) {
      uint64_t plen;
      memcpy(&plen, h.data(), 8);
      pl.assign(h.begin() + 8, h.begin() + 8 + plen);
      // epoch ranks in table order, as format() inserts them (rempi_encoder_cdc.cpp:261-267)
      size_t q = 0;
      while (q < pl.size()) {
        uint64_t esz;
        memcpy(&esz, &pl[q + 8], 8);
        for (uint64_t i = 0; i < esz / 8; i++) {
          uint64_t v;
          memcpy(&v, &pl[q + 16 + 8 * i], 8);
          er.push_back((int32_t)v);
        }
        size_t p = q + 16 + 2 * esz;
        uint64_t w;
        memcpy(&w, &pl[p + 8], 8);
        p += 16 + w;
        memcpy(&w, &pl[p + 8], 8);
        p += 16 + w;
        memcpy(&w, &pl[p], 8);
        p += 8 + w;
        memcpy(&w, &pl[p], 8);
        p += 8 + w;
        memcpy(&w, &pl[p], 8);
        p += 8 + w;
        q = p;
      }
    }
    if (c->gzip && !pl.empty()) pl = deflate_payload(pl.data(), pl.size());
    *payload = host_copy(pl);
    *payload_len = pl.size();
    *epoch_ranks = host_copy(er);
    *n_epoch_ranks = er.size();
  });
  c->max_len = saved;
  return rc;
}

int cdcx_decode_stream(cdcx_ctx* c, const uint8_t* in, size_t len, uint8_t** dump, size_t* dump_len) {
  if (!c || (len && !in) || !dump || !dump_len) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    std::vector<uint8_t> plain;
    if (c->gzip) {
      plain = gunzip_file(in, len);
      in = plain.data();
      len = plain.size();
    }
    hipStream_t s = c->stream;
    uint8_t* d = c->buf<uint8_t>("h_file", len);
    if (len) HIPCHK(hipMemcpyAsync(d, in, len, hipMemcpyHostToDevice, s));
    decode_batch(c, 1, d, {0}, {(int64_t)len}, nullptr, 0, false, true, s);
    std::vector<int64_t> t = tables_dump(c, in, s);
    *dump = reinterpret_cast<uint8_t*>(host_copy(t));
    *dump_len = t.size() * 8;
  });
}

}  // extern "C"

namespace {

// One chunk payload as a one-chunk rank file image in device memory (length word, payload,
// separator, empty footer), so that the batch decoder's framing walk applies unchanged.
// The payload starts at byte 8 of the image.
uint8_t* upload_chunk_image(cdcx_ctx* c, const uint8_t* payload, size_t len, int64_t* image_len, hipStream_t s) {
  if (len & 7) throw CdcxError{CDCX_ERR_CORRUPT, "chunk payload is not a multiple of 8 bytes"};
  if (len == 0) throw CdcxError{CDCX_ERR_CORRUPT, "empty chunk payload (0 is the footer separator)"};
  const uint64_t head = len;
  const uint64_t tail[3] = {0, 0, 0};  // separator, footer rank count 0, int32 map length 0 (+ pad)
  uint8_t* d = c->buf<uint8_t>("h_file", len + 32);
  HIPCHK(hipMemcpyAsync(d, &head, 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + 8, payload, len, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + 8 + len, tail, 20, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));  // head/tail live on this frame
  *image_len = (int64_t)len + 28;
  return d;
}

}  // namespace

extern "C" {

int cdcx_decode_chunk(cdcx_ctx* c, const uint8_t* payload, size_t len, cdcx_tables* out) {
  if (!c || !payload || !out) return CDCX_ERR_ARG;
  out->n_tables = 0;
  out->tables = nullptr;
  return guarded(c, [&] {
    std::vector<uint8_t> plain;
    if (c->gzip) {
      plain = inflate_payload(payload, len);
      payload = plain.data();
      len = plain.size();
    }
    hipStream_t s = c->stream;
    int64_t L = 0;
    uint8_t* d = upload_chunk_image(c, payload, len, &L, s);
    decode_batch(c, 1, d, {0}, {L}, nullptr, 0, false, true, s);
    const DecodedTables t = download_tables(c, s);
    // test_tables_map: ascending set id, the last table of an id wins
    std::map<int32_t, int32_t> bysid;
    for (int32_t q = 0; q < (int32_t)c->dunits.size(); q++) bysid[c->dunits[q].set_id] = q;
    size_t words = 0, perms = 0;
    for (auto& kv : bysid) {
      const DUnit& u = c->dunits[kv.second];
      words += 2 * (size_t)u.S + u.W + u.Mi + 2 * (size_t)(u.Uc > 0 ? u.U : 0) + 2 * (size_t)u.P;
      perms += (size_t)u.M;
    }
    const size_t head_bytes = align_up((int64_t)(bysid.size() * sizeof(cdcx_table)), 16);
    uint8_t* block = static_cast<uint8_t*>(malloc(std::max<size_t>(head_bytes + 8 * words + 4 * perms, 16)));
    if (!block) throw std::bad_alloc();
    cdcx_table* tabs = reinterpret_cast<cdcx_table*>(block);
    uint64_t* w = reinterpret_cast<uint64_t*>(block + head_bytes);
    int32_t* pm = reinterpret_cast<int32_t*>(block + head_bytes + 8 * words);
    auto put = [&](const void* src, size_t n) {
      uint64_t* at = w;
      if (n) memcpy(w, src, 8 * n);
      w += n;
      return at;
    };
    size_t k = 0;
    for (auto& kv : bysid) {
      const DUnit& u = c->dunits[kv.second];
      const uint8_t* in = payload - 8;  // section offsets are relative to the image
      const uint64_t* wpd = t.pk + t.pk_off[kv.second];
      const size_t U = u.Uc > 0 ? (size_t)u.U : 0;
      const uint64_t* uidd = wpd + u.W;
      const uint64_t* idd = uidd + U;
      const uint64_t* dld = idd + u.P;
      cdcx_table& o = tabs[k++];
      o.set_id = u.set_id;
      o.count = u.M;
      o.n_epoch = (size_t)u.S;
      o.epoch_rank = put(in + u.ep_off, u.S);
      o.epoch_clock = put(in + u.ep_off + 8ll * u.S, u.S);
      o.n_with_previous = (size_t)u.W;
      o.with_previous = put(wpd, u.W);
      o.n_matched_index = (size_t)u.Mi;
      o.matched_index = put(in + u.mi_off, u.Mi);
      o.n_unmatched = U;
      o.unmatched_id = put(uidd, U);
      o.unmatched_count = put(in + u.ucnt_off, U);
      o.n_pairs = (size_t)u.P;
      o.ids = put(idd, u.P);
      o.delays = put(dld, u.P);
      o.perm = pm;
      if (u.M) memcpy(pm, t.perm + u.key_off, 4 * (size_t)u.M);
      pm += u.M;
    }
    out->n_tables = bysid.size();
    out->tables = tabs;
  });
}

int cdcx_reconstruct_chunk(cdcx_ctx* c, const uint8_t* payload, size_t len, const int32_t* keys, size_t n_keys,
                           int32_t** rec8, size_t* n_out) {
  if (!c || !payload || (n_keys && !keys) || !rec8 || !n_out) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    std::vector<uint8_t> plain;
    if (c->gzip) {
      plain = inflate_payload(payload, len);
      payload = plain.data();
      len = plain.size();
    }
    hipStream_t s = c->stream;
    int64_t L = 0;
    uint8_t* d = upload_chunk_image(c, payload, len, &L, s);
    int2* dk = c->buf<int2>("h_keys", n_keys);
    if (n_keys) HIPCHK(hipMemcpyAsync(dk, keys, 8 * n_keys, hipMemcpyHostToDevice, s));
    decode_batch(c, 1, d, {0}, {L}, dk, (int64_t)n_keys, true, false, s);
    std::vector<int32_t> r = c->download(c->d_rec_out, 8 * c->n_rec_out, s);
    *rec8 = host_copy(r);
    *n_out = (size_t)c->n_rec_out;
  });
}

}  // extern "C"

namespace {

// Keys in the iteration order of a libstdc++ unordered container with identity hash after
// inserting them in the given order (hash_order.h); positions of the first insertions.
std::vector<size_t> hash_iteration_order(const std::vector<uint64_t>& keys_in_order) {
  const size_t n = keys_in_order.size();
  std::vector<uint64_t> key(n + 1);
  std::vector<int32_t> next(n + 1), bucket(hash_bucket_capacity(n) + 1);
  std::vector<size_t> first;  // node -> index of its first insertion
  HashOrder h;
  h.init(key.data(), next.data(), bucket.data());
  for (size_t i = 0; i < n; i++)
    if (!h.contains(keys_in_order[i])) {
      h.insert_new(keys_in_order[i]);
      first.push_back(i);
    }
  std::vector<size_t> out;
  for (int32_t p = h.head; p != -1; p = h.next[p]) out.push_back(first[p]);
  return out;
}

// write_footer (rempi_encoder_cdc.cpp:2085-2126): separator, distinct ranks in
// unordered_set<int> order, the matching-set-id map in unordered_map<size_t,int> order.
std::vector<uint8_t> footer_bytes(const int32_t* epoch_ranks, size_t n_in, const uint64_t* msg_ids, const int32_t* set_ids,
                                  size_t n_ids) {
  std::vector<uint64_t> rk(n_in);
  for (size_t i = 0; i < n_in; i++) rk[i] = (uint64_t)(int64_t)epoch_ranks[i];  // std::hash<int>: the sign-extended value
  const std::vector<size_t> ro = hash_iteration_order(rk);
  // the map: a later entry of an id overwrites the set id and keeps the id's node
  std::vector<uint64_t> ids(msg_ids, msg_ids + n_ids);
  const std::vector<size_t> mo = hash_iteration_order(ids);
  std::map<uint64_t, int32_t> last;
  for (size_t i = 0; i < n_ids; i++) last[msg_ids[i]] = set_ids[i];
  std::vector<uint8_t> out(16 + 4 * ro.size() + 4 + 12 * mo.size());
  uint64_t v = 0;
  memcpy(out.data(), &v, 8);
  v = ro.size();
  memcpy(out.data() + 8, &v, 8);
  size_t q = 16;
  for (size_t i : ro) {
    memcpy(out.data() + q, &epoch_ranks[i], 4);
    q += 4;
  }
  const int32_t L = (int32_t)mo.size();
  memcpy(out.data() + q, &L, 4);
  q += 4;
  for (size_t i : mo) {
    memcpy(out.data() + q, &msg_ids[i], 8);
    q += 8;
  }
  for (size_t i : mo) {
    const int32_t sid = last[msg_ids[i]];
    memcpy(out.data() + q, &sid, 4);
    q += 4;
  }
  return out;
}

// A rank file as the device wrote it (footer ending in int32 0) with the context's map appended.
void append_id_map(const cdcx_ctx* c, std::vector<uint8_t>& file) {
  if (c->map_ids.empty() || file.size() < 4) return;
  const std::vector<uint8_t> f = footer_bytes(nullptr, 0, c->map_ids.data(), c->map_sets.data(), c->map_ids.size());
  file.resize(file.size() - 4);                        // the device's int32 0
  file.insert(file.end(), f.begin() + 16, f.end());    // int32 L, ids, set ids
}

struct FooterView {
  size_t n_ranks = 0, n_ids = 0;
  const uint8_t* ranks = nullptr;    // int32[n_ranks], maybe unaligned
  const uint8_t* msg_ids = nullptr;  // size_t[n_ids]
  const uint8_t* set_ids = nullptr;  // int32[n_ids]
};
// read_footer (rempi_encoder_cdc.cpp:2015-2083): skip the chunks, then parse.
bool parse_footer(const uint8_t* b, size_t len, FooterView* fv) {
  size_t p = 0;
  while (true) {
    if (len - p < 8) return false;
    uint64_t n;
    memcpy(&n, b + p, 8);
    p += 8;
    if (n == 0) break;
    if (n > len - p) return false;
    p += n;
  }
  if (len - p < 8) return false;
  uint64_t nr;
  memcpy(&nr, b + p, 8);
  p += 8;
  if (nr > (len - p) / 4) return false;
  fv->n_ranks = nr;
  fv->ranks = b + p;
  p += 4 * nr;
  if (len - p < 4) return false;
  int32_t L;
  memcpy(&L, b + p, 4);
  p += 4;
  if (L > 0) {
    if ((uint64_t)L > (len - p) / 12) return false;
    fv->n_ids = (size_t)L;
    fv->msg_ids = b + p;
    fv->set_ids = b + p + 8 * (size_t)L;
  }
  return true;
}
// One malloc block: the struct, then 8-aligned copies of the arrays.
cdcx_footer_info* footer_info_block(const FooterView& fv) {
  const size_t head = (sizeof(cdcx_footer_info) + 15) / 16 * 16;
  const size_t bytes = head + 8 * fv.n_ids + 4 * fv.n_ids + 4 * fv.n_ranks + 16;
  uint8_t* blk = static_cast<uint8_t*>(malloc(bytes));
  if (!blk) throw std::bad_alloc();
  cdcx_footer_info* fi = reinterpret_cast<cdcx_footer_info*>(blk);
  uint8_t* ids = blk + head;
  uint8_t* sets = ids + 8 * fv.n_ids;
  uint8_t* ranks = sets + 4 * fv.n_ids;
  if (fv.n_ids) memcpy(ids, fv.msg_ids, 8 * fv.n_ids);
  if (fv.n_ids) memcpy(sets, fv.set_ids, 4 * fv.n_ids);
  if (fv.n_ranks) memcpy(ranks, fv.ranks, 4 * fv.n_ranks);
  fi->n_ranks = fv.n_ranks;
  fi->ranks = reinterpret_cast<const int32_t*>(ranks);
  fi->n_ids = fv.n_ids;
  fi->msg_ids = reinterpret_cast<const uint64_t*>(ids);
  fi->set_ids = reinterpret_cast<const int32_t*>(sets);
  return fi;
}

}  // namespace

extern "C" {

int cdcx_footer_ex(const int32_t* epoch_ranks, size_t n_in, const uint64_t* msg_ids, const int32_t* set_ids, size_t n_ids,
                   uint8_t* out, size_t* len) {
  if ((n_in && !epoch_ranks) || (n_ids && (!msg_ids || !set_ids)) || !len || n_in > (size_t)INT32_MAX - 1 ||
      n_ids > (size_t)INT32_MAX - 1)
    return CDCX_ERR_ARG;
  try {
    const std::vector<uint8_t> f = footer_bytes(epoch_ranks, n_in, msg_ids, set_ids, n_ids);
    if (out) {
      if (*len < f.size()) {
        *len = f.size();
        return CDCX_ERR_ARG;
      }
      memcpy(out, f.data(), f.size());
    }
    *len = f.size();
    return CDCX_OK;
  } catch (const std::bad_alloc&) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_footer(const int32_t* epoch_ranks, size_t n_in, uint8_t* out, size_t* len) {
  return cdcx_footer_ex(epoch_ranks, n_in, nullptr, nullptr, 0, out, len);
}

int cdcx_set_matching_set_id_map(cdcx_ctx* c, const uint64_t* msg_ids, const int32_t* set_ids, size_t n) {
  if (!c || (n && (!msg_ids || !set_ids))) return CDCX_ERR_ARG;
  try {
    if (n == 0) {
      c->map_ids.clear();
      c->map_sets.clear();
    }
    for (size_t i = 0; i < n; i++) {
      const auto it = std::find(c->map_ids.begin(), c->map_ids.end(), msg_ids[i]);
      if (it != c->map_ids.end()) {
        c->map_sets[it - c->map_ids.begin()] = set_ids[i];
      } else {
        c->map_ids.push_back(msg_ids[i]);
        c->map_sets.push_back(set_ids[i]);
      }
    }
    return CDCX_OK;
  } catch (const std::bad_alloc&) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_read_footer(const uint8_t* file, size_t len, cdcx_footer_info** out) {
  if (!file || !out) return CDCX_ERR_ARG;
  *out = nullptr;
  try {
    FooterView fv;
    if (!parse_footer(file, len, &fv)) return CDCX_ERR_CORRUPT;
    *out = footer_info_block(fv);
    return CDCX_OK;
  } catch (const std::bad_alloc&) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_reconstruct_stream(cdcx_ctx* c, const uint8_t* in, size_t len, const int32_t* keys, size_t n_keys,
                            int32_t** rec8, size_t* n_out) {
  if (!c || (len && !in) || (n_keys && !keys) || !rec8 || !n_out) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    std::vector<uint8_t> plain;
    if (c->gzip) {
      plain = gunzip_file(in, len);
      in = plain.data();
      len = plain.size();
    }
    hipStream_t s = c->stream;
    uint8_t* d = c->buf<uint8_t>("h_file", len);
    if (len) HIPCHK(hipMemcpyAsync(d, in, len, hipMemcpyHostToDevice, s));
    int2* dk = c->buf<int2>("h_keys", n_keys);
    if (n_keys) HIPCHK(hipMemcpyAsync(dk, keys, 8 * n_keys, hipMemcpyHostToDevice, s));
    decode_batch(c, 1, d, {0}, {(int64_t)len}, dk, (int64_t)n_keys, true, false, s);
    std::vector<int32_t> r = c->download(c->d_rec_out, 8 * c->n_rec_out, s);
    *rec8 = host_copy(r);
    *n_out = (size_t)c->n_rec_out;
  });
}

int cdcx_gzip_file(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len) {
  if ((len && !in) || !out || !out_len) return CDCX_ERR_ARG;
  try {
    std::vector<uint8_t> v = gzip_file(in, len);
    *out = host_copy(v);
    *out_len = v.size();
    return CDCX_OK;
  } catch (const GzipError&) {
    return CDCX_ERR_CORRUPT;
  } catch (const std::bad_alloc&) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_gunzip_file(const uint8_t* in, size_t len, uint8_t** out, size_t* out_len) {
  if ((len && !in) || !out || !out_len) return CDCX_ERR_ARG;
  try {
    std::vector<uint8_t> v = gunzip_file(in, len);
    *out = host_copy(v);
    *out_len = v.size();
    return CDCX_OK;
  } catch (const GzipError&) {
    return CDCX_ERR_CORRUPT;
  } catch (const std::bad_alloc&) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_decode_batch_device(cdcx_ctx* c, int32_t n_ranks, const uint8_t* d_in, const int64_t* in_off,
                             const int64_t* in_len, const int32_t* d_keys, int64_t n_keys, const int32_t** d_rec_out,
                             int64_t* n_rec_out, const int32_t** d_perm, void* stream) {
  if (!c || n_ranks <= 0 || !d_in || !in_off || !in_len || !d_rec_out || !n_rec_out || !d_perm || c->gzip)
    return CDCX_ERR_ARG;
  return guarded(c, [&] {
    std::vector<int64_t> off(in_off, in_off + n_ranks), len(in_len, in_len + n_ranks);
    decode_batch(c, n_ranks, d_in, off, len, reinterpret_cast<const int2*>(d_keys), n_keys, d_keys != nullptr, false,
                 (hipStream_t)stream);
    *d_rec_out = c->d_rec_out;
    *n_rec_out = c->n_rec_out;
    *d_perm = c->d_perm;
  });
}

int cdcx_decode_chunk_perm_static(cdcx_ctx* c, const uint8_t* d_payload, size_t len, int32_t* d_perm,
                                  size_t perm_capacity, int64_t* n_perm, void* stream) {
  if (!c || !d_payload || !d_perm || !n_perm) return CDCX_ERR_ARG;
  *n_perm = 0;
  // (the kernels read the payload as 8-byte and 4-byte words; a gzip context's payloads are zlib streams)
  if (c->gzip || (reinterpret_cast<uintptr_t>(d_payload) & 7) || (reinterpret_cast<uintptr_t>(d_perm) & 3)) {
    c->err = "cdcx_decode_chunk_perm_static: plain-CDC context, 8-byte aligned payload and 4-byte aligned perm required";
    return CDCX_ERR_ARG;
  }
  if (len == 0 || (len & 7) || len > ((size_t)1 << 40)) {
    c->err = "chunk payload length must be a positive multiple of 8";
    return CDCX_ERR_CORRUPT;
  }
  // No allocation anywhere below: fixed-size launches over this device's static scratch, one
  // small D2H of the header at the end.
  hipStream_t s = (hipStream_t)stream;
  if (hipSetDevice(c->device) != hipSuccess || !c->static_scratch) {
    (void)hipGetLastError();
    c->err = "no static scratch on this device";
    return CDCX_ERR_HIP;
  }
  unsigned char* sc = c->static_scratch;
  int32_t* hdr = reinterpret_cast<int32_t*>(sc + kStaticHdrOff);
  int32_t* order = reinterpret_cast<int32_t*>(sc + kStaticOrderOff);
  DUnit* units = reinterpret_cast<DUnit*>(sc + kStaticUnitsOff);
  uint64_t* idd = reinterpret_cast<uint64_t*>(sc + kStaticIddOff);
  uint64_t* dld = reinterpret_cast<uint64_t*>(sc + kStaticDldOff);
  int32_t* cinv = reinterpret_cast<int32_t*>(sc + kStaticCinvOff);
  int32_t* nx = reinterpret_cast<int32_t*>(sc + kStaticNxOff);
  int32_t* pv = reinterpret_cast<int32_t*>(sc + kStaticPvOff);
  const int64_t cap = (int64_t)std::min<size_t>(perm_capacity, (size_t)kStaticMaxRows);
  hipLaunchKernelGGL(k_dec_chunk_units, dim3(1), dim3(64), 0, s, d_payload, (int64_t)len, kStaticMaxUnits, kStaticMaxRows, cap,
                     hdr, order, units);
  hipLaunchKernelGGL(k_dec_pair_scan, dim3(kStaticMaxUnits), dim3(64), 0, s, (const DUnit*)units, d_payload, 4, (DSeg*)nullptr,
                     (int64_t*)nullptr, idd, dld);
  hipLaunchKernelGGL(k_dec_perm_seg<0>, dim3(kStaticMaxUnits / 4), dim3(64), 0, s, units, (const int32_t*)order,
                     (const DSeg*)nullptr, (int64_t)kStaticMaxUnits, 1, d_payload, (const int64_t*)nullptr, d_perm, cinv,
                     (int32_t*)nullptr, (int32_t*)nullptr, hdr + 2);
  hipLaunchKernelGGL(k_dec_perm_window<4>, dim3(kStaticMaxUnits), dim3(64), 0, s, units, kStaticMaxUnits, 2,
                     (const uint64_t*)idd, (const uint64_t*)dld, d_perm, hdr + 3);
  hipLaunchKernelGGL(k_dec_perm_lane, dim3(kStaticMaxUnits / 64), dim3(64), 0, s, (const DUnit*)units, kStaticMaxUnits,
                     (const uint64_t*)idd, (const uint64_t*)dld, nx, pv, d_perm, reinterpret_cast<uint32_t*>(hdr));
  int32_t h[6] = {0, 0, 0, 0, 0, 0};
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h, hdr, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    c->err = std::string("cdcx_decode_chunk_perm_static: ") + hipGetErrorString(e);
    return CDCX_ERR_HIP;
  }
  const uint32_t bits = (uint32_t)h[0];
  if (bits & (1u << CDCX_ERR_LIMIT)) {
    c->err = "chunk exceeds the static scratch (sum of count + 1 over its tables > 262144, more than 256 tables, or "
             "more matched events than perm_capacity)";
    return CDCX_ERR_LIMIT;
  }
  if (bits) {
    c->err = "Record data is broken";
    return CDCX_ERR_CORRUPT;
  }
  *n_perm = (int64_t)(((uint64_t)(uint32_t)h[5] << 32) | (uint32_t)h[4]);
  c->err.clear();
  return CDCX_OK;
}

int cdcx_decode_rank_offsets(cdcx_ctx* c, int32_t n_ranks, int64_t* rec_off, int64_t* perm_off) {
  if (!c || n_ranks < 0 || !rec_off || !perm_off || (size_t)n_ranks + 1 != c->dcbase.size()) return CDCX_ERR_ARG;
  const int rc = guarded(c, [&] { host_dec_units(c, c->dec_stream); });
  if (rc != CDCX_OK) return rc;
  const size_t NU = c->dunits.size(), C = c->dfirst_unit.size();
  int64_t rec_end = 0, perm_end = 0;
  if (NU) {
    const DUnit& u = c->dunits[NU - 1];
    rec_end = u.rec_off + u.M + (u.Uc > 0 ? u.U : 0);
    perm_end = u.key_off + u.M;
  }
  for (int32_t r = 0; r <= n_ranks; r++) {
    // first unit of the first chunk of rank r or of any later rank (chunks may hold no table)
    size_t k = (size_t)c->dcbase[r];
    while (k < C && c->dnunits[k] == 0) k++;
    const bool have = k < C;
    rec_off[r] = have ? c->dunits[c->dfirst_unit[k]].rec_off : rec_end;
    perm_off[r] = have ? c->dunits[c->dfirst_unit[k]].key_off : perm_end;
  }
  return CDCX_OK;
}

int cdcx_verify_roundtrip_device(cdcx_ctx* c, const int32_t* d_rec, int64_t* mismatches, void* stream) {
  if (!c || !d_rec || !mismatches) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    hipStream_t s = (hipStream_t)stream;
    host_enc_units(c, s);
    host_dec_units(c, s);
    const int32_t NU = (int32_t)c->enc_units.size();
    if (c->dunits.size() != c->enc_units.size())
      throw CdcxError{CDCX_ERR_ARG, "the last decode does not hold the units of the last encode"};
    std::vector<int64_t> dec_off(NU + 1, 0);
    for (int32_t q = 0; q < NU; q++) {
      const Unit& u = c->enc_units[q];
      const DUnit& d = c->dunits[q];
      if (d.M != u.M || d.set_id != u.set_id || d.rec_off != dec_off[q])
        throw CdcxError{CDCX_ERR_CORRUPT, "decoded unit " + std::to_string(q) + " does not match the encoder's unit"};
      dec_off[q + 1] = dec_off[q] + u.M + u.U;  // (one record per matched event and per run of polls)
    }
    if (dec_off[NU] != c->n_rec_out || !c->d_rec_out)
      throw CdcxError{CDCX_ERR_ARG, "the last decode did not reconstruct records"};
    int64_t* d_dec_off = c->upload("v_dec_off", dec_off, s);
    int64_t* d_rec_off = c->upload("rec_off", c->enc_rec_off, s);
    unsigned long long* d_bad = c->buf<unsigned long long>("v_bad", 1);
    HIPCHK(hipMemsetAsync(d_bad, 0, 8, s));
    c->launch(K_VERIFY, k_verify_roundtrip, dim3(NU), dim3(256), s, (const Unit*)c->buf<Unit>("units", 0),
              (const int64_t*)d_dec_off, (const int64_t*)d_rec_off, (const TRec*)c->buf<TRec>("trec", 0),
              reinterpret_cast<const int4*>(d_rec), reinterpret_cast<const int4*>(c->d_rec_out), d_bad);
    *mismatches = (int64_t)c->download(d_bad, 1, s)[0];
  });
}

// Replay-side streaming decode: one host thread per context, each
// taking whole batches of consecutive rank files off a shared counter.
}  // extern "C"

namespace {

struct ReplayJob {
  const char* const* paths;
  std::vector<int64_t> size;                  // file sizes (stat)
  std::vector<int32_t> first;                 // batch b = files [first[b], first[b + 1])
  std::atomic<int32_t> next{0};
  std::atomic<bool> stop{false};
  std::mutex sink_mu;
  cdcx_replay_sink sink = nullptr;              // int64 dumps, or
  cdcx_replay_table_sink table_sink = nullptr;  // flat tables pointing into the pinned buffers
  cdcx_replay_footer_sink footer_sink = nullptr;  // ... preceded by the file's parsed footer
  void* user;
  std::atomic<int64_t> chunks{0}, units{0}, records{0}, bytes{0}, dump_bytes{0};
  std::atomic<int64_t> ns_read{0}, ns_device{0}, ns_dump{0}, ns_sink{0};  // thread time per phase
};

inline int64_t ns_since(std::chrono::steady_clock::time_point& t) {
  const auto now = std::chrono::steady_clock::now();
  const int64_t d = std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
  t = now;
  return d;
}

std::vector<uint8_t> read_file(const char* path, int64_t size) {
  std::vector<uint8_t> v((size_t)size);
  FILE* f = fopen(path, "rb");
  if (!f) throw CdcxError{CDCX_ERR_ARG, std::string("cannot open ") + path};
  const size_t got = size ? fread(v.data(), 1, (size_t)size, f) : 0;
  fclose(f);
  if (got != (size_t)size) throw CdcxError{CDCX_ERR_ARG, std::string("short read of ") + path};
  return v;
}

void replay_batch(cdcx_ctx* c, ReplayJob& job, int32_t b, hipStream_t s) {
  const int32_t f0 = job.first[b], f1 = job.first[b + 1], R = f1 - f0;
  auto t = std::chrono::steady_clock::now();
  std::vector<int64_t> off(R), len(R);
  std::vector<std::vector<uint8_t>> plain;  // gzip contexts: inflated images
  int64_t pos = 0;
  if (c->gzip) {
    plain.resize(R);
    for (int32_t r = 0; r < R; r++) {
      std::vector<uint8_t> z = read_file(job.paths[f0 + r], job.size[f0 + r]);
      plain[r] = gunzip_file(z.data(), z.size());
      off[r] = pos;
      len[r] = (int64_t)plain[r].size();
      pos = align_up(pos + len[r], 8);
    }
  } else {
    for (int32_t r = 0; r < R; r++) {
      off[r] = pos;
      len[r] = job.size[f0 + r];
      pos = align_up(pos + len[r], 8);
    }
  }
  uint8_t* h = pinned(c->pin_in, (size_t)std::max<int64_t>(pos, 8));
  for (int32_t r = 0; r < R; r++) {
    if (c->gzip) {
      if (len[r]) memcpy(h + off[r], plain[r].data(), (size_t)len[r]);
      continue;
    }
    FILE* f = fopen(job.paths[f0 + r], "rb");
    if (!f) throw CdcxError{CDCX_ERR_ARG, std::string("cannot open ") + job.paths[f0 + r]};
    const size_t got = len[r] ? fread(h + off[r], 1, (size_t)len[r], f) : 0;
    fclose(f);
    if (got != (size_t)len[r]) throw CdcxError{CDCX_ERR_ARG, std::string("short read of ") + job.paths[f0 + r]};
  }
  job.ns_read += ns_since(t);
  uint8_t* d = c->buf<uint8_t>("h_file", (size_t)std::max<int64_t>(pos, 8));
  if (pos) HIPCHK(hipMemcpyAsync(d, h, (size_t)pos, hipMemcpyHostToDevice, s));
  decode_batch(c, R, d, off, len, nullptr, 0, false, true, s);
  const DecodedTables tb = download_tables(c, s);
  job.ns_device += ns_since(t);
  job.chunks += (int64_t)c->dchunks.size();
  job.units += (int64_t)c->dunits.size();
  job.records += c->n_rec_out;
  if (job.table_sink) {
    // Flat tables of every chunk of every file, nothing copied on the host: epoch lines,
    // matched_index and unmatched counts are read in place from the file image in the pinned
    // input buffer, the inverted sections and permutations from the packed D2H buffer.
    std::vector<cdcx_table> tabs;
    std::vector<cdcx_tables> chunks;
    std::map<int32_t, int32_t> bysid;
    for (int32_t r = 0; r < R; r++) {
      tabs.clear();
      chunks.clear();
      std::vector<size_t> first;
      for (int32_t k = c->dcbase[r]; k < c->dcbase[r + 1]; k++) {
        bysid.clear();  // test_tables_map: ascending set id, the last table of an id wins
        for (int32_t q = 0; q < c->dnunits[k]; q++) bysid[c->dunits[c->dfirst_unit[k] + q].set_id] = c->dfirst_unit[k] + q;
        first.push_back(tabs.size());
        for (auto& kv : bysid) {
          const DUnit& u = c->dunits[kv.second];
          const uint64_t* wpd = tb.pk + tb.pk_off[kv.second];
          const size_t U = u.Uc > 0 ? (size_t)u.U : 0;
          cdcx_table o;
          o.set_id = u.set_id;
          o.count = u.M;
          o.n_epoch = (size_t)u.S;
          o.epoch_rank = reinterpret_cast<const uint64_t*>(h + u.ep_off);
          o.epoch_clock = o.epoch_rank + u.S;
          o.n_with_previous = (size_t)u.W;
          o.with_previous = wpd;
          o.n_matched_index = (size_t)u.Mi;
          o.matched_index = reinterpret_cast<const uint64_t*>(h + u.mi_off);
          o.n_unmatched = U;
          o.unmatched_id = wpd + u.W;
          o.unmatched_count = reinterpret_cast<const uint64_t*>(h + u.ucnt_off);
          o.n_pairs = (size_t)u.P;
          o.ids = o.unmatched_id + U;
          o.delays = o.ids + u.P;
          o.perm = tb.perm + u.key_off;
          tabs.push_back(o);
        }
      }
      first.push_back(tabs.size());
      for (size_t k = 0; k + 1 < first.size(); k++) chunks.push_back(cdcx_tables{first[k + 1] - first[k], tabs.data() + first[k]});
      job.dump_bytes += (int64_t)(tabs.size() * sizeof(cdcx_table));
      job.ns_dump += ns_since(t);
      std::lock_guard<std::mutex> g(job.sink_mu);
      if (job.stop) return;
      if (job.footer_sink) {
        FooterView fv;
        if (!parse_footer(h + off[r], (size_t)len[r], &fv))
          throw CdcxError{CDCX_ERR_CORRUPT, "no footer in rank file " + std::to_string(f0 + r)};
        cdcx_footer_info* fi = footer_info_block(fv);
        const int rc = job.footer_sink(job.user, f0 + r, fi);
        free(fi);
        if (rc != 0) throw CdcxError{CDCX_ERR_ARG, "replay sink stopped the pipeline at file " + std::to_string(f0 + r)};
      }
      if (job.table_sink(job.user, f0 + r, chunks.size(), chunks.data()) != 0)
        throw CdcxError{CDCX_ERR_ARG, "replay sink stopped the pipeline at file " + std::to_string(f0 + r)};
      job.ns_sink += ns_since(t);
    }
    for (int32_t r = 0; r < R; r++) job.bytes += job.size[f0 + r];
    return;
  }
  std::vector<int64_t> dump;
  for (int32_t r = 0; r < R; r++) {
    dump.clear();
    dump_chunks(c, tb, h, c->dcbase[r], c->dcbase[r + 1], dump);
    job.dump_bytes += 8 * (int64_t)dump.size();
    job.ns_dump += ns_since(t);
    std::lock_guard<std::mutex> g(job.sink_mu);
    if (job.stop) return;
    if (job.sink(job.user, f0 + r, dump.data(), dump.size()) != 0)
      throw CdcxError{CDCX_ERR_ARG, "replay sink stopped the pipeline at file " + std::to_string(f0 + r)};
    job.ns_sink += ns_since(t);
  }
  for (int32_t r = 0; r < R; r++) job.bytes += job.size[f0 + r];
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {
int replay_run(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths, int64_t batch_bytes,
               cdcx_replay_sink sink, cdcx_replay_table_sink table_sink, cdcx_replay_footer_sink footer_sink, void* user,
               cdcx_replay_stats* stats);
}

extern "C" {

int cdcx_replay_decode_files(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                             int64_t batch_bytes, cdcx_replay_sink sink, void* user, cdcx_replay_stats* stats) {
  if (!sink) return CDCX_ERR_ARG;
  return replay_run(ctxs, n_ctx, n_files, paths, batch_bytes, sink, nullptr, nullptr, user, stats);
}

int cdcx_replay_decode_tables(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                              int64_t batch_bytes, cdcx_replay_table_sink sink, void* user, cdcx_replay_stats* stats) {
  if (!sink) return CDCX_ERR_ARG;
  return replay_run(ctxs, n_ctx, n_files, paths, batch_bytes, nullptr, sink, nullptr, user, stats);
}

int cdcx_replay_decode_tables_ex(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths,
                                 int64_t batch_bytes, cdcx_replay_table_sink sink, cdcx_replay_footer_sink footer_sink,
                                 void* user, cdcx_replay_stats* stats) {
  if (!sink) return CDCX_ERR_ARG;
  return replay_run(ctxs, n_ctx, n_files, paths, batch_bytes, nullptr, sink, footer_sink, user, stats);
}

}  // extern "C"

namespace {

int replay_run(cdcx_ctx* const* ctxs, int32_t n_ctx, int32_t n_files, const char* const* paths, int64_t batch_bytes,
               cdcx_replay_sink sink, cdcx_replay_table_sink table_sink, cdcx_replay_footer_sink footer_sink, void* user,
               cdcx_replay_stats* stats) {
  if (!ctxs || n_ctx <= 0 || n_files < 0 || (n_files && !paths)) return CDCX_ERR_ARG;
  for (int32_t i = 0; i < n_ctx; i++) {
    if (!ctxs[i]) return CDCX_ERR_ARG;
    for (int32_t k = 0; k < i; k++)
      if (ctxs[k] == ctxs[i]) {  // one worker thread per entry: a context must not be shared
        ctxs[i]->err = "the same context was passed twice";
        return CDCX_ERR_ARG;
      }
  }
  const auto t0 = std::chrono::steady_clock::now();
  ReplayJob job;
  job.paths = paths;
  job.sink = sink;
  job.table_sink = table_sink;
  job.footer_sink = footer_sink;
  job.user = user;
  job.size.resize(n_files);
  for (int32_t i = 0; i < n_files; i++) {
    struct stat st;
    if (!paths[i] || stat(paths[i], &st) != 0) {
      ctxs[0]->err = std::string("cannot stat rank file ") + (paths[i] ? paths[i] : "(null)");
      return CDCX_ERR_ARG;
    }
    job.size[i] = (int64_t)st.st_size;
  }
  const int64_t cap = batch_bytes > 0 ? batch_bytes : (int64_t)256 << 20;
  job.first.push_back(0);
  for (int32_t i = 0; i < n_files;) {
    int64_t sum = 0;
    int32_t j = i;
    while (j < n_files && (j == i || sum + job.size[j] <= cap)) sum += job.size[j++];
    job.first.push_back(j);
    i = j;
  }
  const int32_t nb = (int32_t)job.first.size() - 1;
  std::vector<int> rc(n_ctx, CDCX_OK);
  auto worker = [&](int32_t w) {
    cdcx_ctx* c = ctxs[w];
    hipStream_t s = nullptr;
    rc[w] = guarded(c, [&] {
      HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      for (int32_t b; !job.stop && (b = job.next++) < nb;) replay_batch(c, job, b, s);
      HIPCHK(hipStreamSynchronize(s));
    });
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
    if (rc[w] != CDCX_OK) job.stop = true;
  };
  std::vector<std::thread> th;
  for (int32_t w = 1; w < n_ctx; w++) th.emplace_back(worker, w);
  worker(0);
  for (auto& t : th) t.join();
  if (stats) {
    stats->files = n_files;
    stats->file_bytes = job.bytes;
    stats->chunks = job.chunks;
    stats->units = job.units;
    stats->records = job.records;
    stats->batches = nb;
    stats->dump_bytes = job.dump_bytes;
    stats->read_s = job.ns_read * 1e-9;
    stats->device_s = job.ns_device * 1e-9;
    stats->dump_s = job.ns_dump * 1e-9;
    stats->sink_s = job.ns_sink * 1e-9;
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  for (int32_t w = 0; w < n_ctx; w++)
    if (rc[w] != CDCX_OK) return rc[w];
  return CDCX_OK;
}

}  // namespace

extern "C" {

int cdcx_generate_host(const cdcx_gen_params* p, int32_t rank, int32_t** rec8, size_t* n_rec) {
  if (!p || !rec8 || !n_rec || p->world_size < 2 || p->events_per_rank < 0) return CDCX_ERR_ARG;
  try {
    GenArgs g{gen::shape(p->world_size, p->senders, p->sets, p->jitter), 0, p->events_per_rank, p->seed_salt};
    if (g.sh.T > 16) return CDCX_ERR_LIMIT;
    std::vector<int32_t> v = generate_host(g, rank);
    *rec8 = host_copy(v);
    *n_rec = v.size() / 8;
    return CDCX_OK;
  } catch (...) {
    return CDCX_ERR_NOMEM;
  }
}

int cdcx_generate_device(cdcx_ctx* c, const cdcx_gen_params* p, int32_t first_rank, int32_t n_ranks,
                         const int32_t** d_rec, int64_t* rec_off, void* stream) {
  if (!c || !p || n_ranks <= 0 || !d_rec || !rec_off || p->world_size < 2 || p->events_per_rank <= 0) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    hipStream_t s = (hipStream_t)stream;
    GenArgs g{gen::shape(p->world_size, p->senders, p->sets, p->jitter), first_rank, p->events_per_rank, p->seed_salt};
    if (g.sh.T > 16) throw CdcxError{CDCX_ERR_LIMIT, "generator supports at most 16 sets"};
    const int64_t F = p->events_per_rank;  // frames per rank (upper bound: >= 1 record each)
    const int32_t tpr = (int32_t)((F + 1023) / 1024);
    const int64_t NTt = (int64_t)tpr * n_ranks;
    int32_t* tsr = c->buf<int32_t>("g_tsr", NTt);
    int32_t* tss = c->buf<int32_t>("g_tss", NTt * 16);
    int32_t* roff = c->buf<int32_t>("g_roff", F * n_ranks);
    int32_t* koff = c->buf<int32_t>("g_koff", F * n_ranks);
    int32_t* nfr = c->buf<int32_t>("g_nfr", n_ranks);
    int32_t* nmt = c->buf<int32_t>("g_nmt", 16 * n_ranks);
    int32_t* nrc = c->buf<int32_t>("g_nrc", n_ranks);
    HIPCHK(hipMemsetAsync(nfr, 0, 4 * n_ranks, s));
    HIPCHK(hipMemsetAsync(nmt, 0, 64 * n_ranks, s));
    HIPCHK(hipMemsetAsync(nrc, 0, 4 * n_ranks, s));
    c->launch(K_GEN_TILE_SUMS, k_gen_tile_sums, dim3(NTt), dim3(256), s, g, F, tpr, tsr, tss);
    c->launch(K_GEN_RANK_SCAN, k_gen_rank_scan, dim3(n_ranks), dim3(256), s, g, tpr, tsr, tss);
    c->launch(K_GEN_FRAMES, k_gen_frames, dim3(NTt), dim3(256), s, g, F, tpr, (const int32_t*)tsr, (const int32_t*)tss,
              roff, koff, nfr, nmt, nrc);
    std::vector<int32_t> nr = c->download(nrc, n_ranks, s);
    int64_t* akey = c->buf<int64_t>("g_akey", F * n_ranks);
    int32_t* inv = c->buf<int32_t>("g_inv", F * n_ranks);
    c->launch(K_GEN_AKEYS, k_gen_akeys, dim3(blocks(F, 256), n_ranks), dim3(256), s, g, F, (const int32_t*)nmt, akey);
    c->launch(K_GEN_ARRIVAL, k_gen_arrival, dim3(blocks(F, 256), n_ranks), dim3(256), s, g, F, (const int32_t*)nmt,
              (const int64_t*)akey, inv);
    rec_off[0] = 0;
    for (int r = 0; r < n_ranks; r++) rec_off[r + 1] = rec_off[r] + nr[r];
    std::vector<int64_t> ro(rec_off, rec_off + n_ranks + 1);
    int64_t* d_ro = c->upload("g_rec_off", ro, s);
    int32_t* out = c->buf<int32_t>("g_rec", 8 * rec_off[n_ranks]);
    c->launch(K_GEN_RECORDS, k_gen_records, dim3(blocks(F, 256), n_ranks), dim3(256), s, g, F, F, (const int32_t*)roff,
              (const int32_t*)koff, (const int32_t*)nfr, (const int32_t*)nmt, (const int32_t*)inv, (const int64_t*)d_ro,
              (int4*)out);
    c->collect(s);
    c->release("g_akey");
    c->release("g_inv");
    c->release("g_roff");
    c->release("g_koff");
    *d_rec = out;
  });
}

int cdcx_set_profiling(cdcx_ctx* c, int enabled) {
  if (!c) return CDCX_ERR_ARG;
  c->profiling = enabled != 0;
  return CDCX_OK;
}

int cdcx_kernel_times(cdcx_ctx* c, double* ms, int64_t* launches, int n) {
  if (!c) return CDCX_ERR_ARG;
  for (int k = 0; k < n && k < K_COUNT; k++) {
    if (ms) ms[k] = c->ktime[k];
    if (launches) launches[k] = c->klaunch[k];
  }
  return CDCX_OK;
}

int cdcx_chain_tiers(cdcx_ctx* c, int64_t* out) {
  if (!c || !out) return CDCX_ERR_ARG;
  for (int k = 0; k < 3; k++) out[k] = c->chain_tier_counts[k];
  return CDCX_OK;
}

int cdcx_encode_totals(cdcx_ctx* c, int64_t* out) {
  if (!c || !out) return CDCX_ERR_ARG;
  std::copy(c->enc_totals, c->enc_totals + 8, out);
  return CDCX_OK;
}

int cdcx_decode_tiers(cdcx_ctx* c, int64_t* out) {
  if (!c || !out) return CDCX_ERR_ARG;
  for (int k = 0; k < 7; k++) out[k] = c->dec_tier_counts[k];
  return CDCX_OK;
}

int cdcx_chain_stats(cdcx_ctx* c, int64_t* out, int n) {
  if (!c || !out || !c->chain_stats) return CDCX_ERR_ARG;
  return guarded(c, [&] {
    unsigned long long* d = c->buf<unsigned long long>("chain_stats", 8);
    std::vector<unsigned long long> h = c->download(d, 8, c->stream);
    for (int k = 0; k < n && k < 8; k++) out[k] = (int64_t)h[k];
    HIPCHK(hipMemsetAsync(d, 0, 64, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  });
}

int cdcx_reset_kernel_times(cdcx_ctx* c) {
  if (!c) return CDCX_ERR_ARG;
  std::fill(c->ktime.begin(), c->ktime.end(), 0.0);
  std::fill(c->klaunch.begin(), c->klaunch.end(), 0);
  return CDCX_OK;
}

}  // extern "C"
