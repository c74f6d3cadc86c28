// cdcx_layout.h -- descriptors shared by the host orchestrator and the kernels.
//
// Vocabulary:
//   rank   one process's record stream (one rank_<r>.rempi file)
//   chunk  one extract_encoder_input_format_chunk epoch (<= REMPI_MAX length units)
//   table  one matching set inside a chunk
//   unit   (rank, chunk, table): the independent unit of CDC work
//   T-order  the records of a rank stably partitioned by table (then stream order); every
//            unit is a contiguous range of it, so per-unit scratch arrays are indexed by the
//            unit's T-order start `a` without any further allocation.
#pragma once
#include <stdint.h>

namespace cdcx {

constexpr int kMaxSets = 256;       // matching_set_id in [0, 256)
constexpr int kTile = 1024;         // records per tile in record-parallel kernels
constexpr int kSortTile = 1024;     // matched events per LDS sort tile
constexpr int kRecTile = 1024;      // decoded rows per tile of the record reconstruction
constexpr int kRankWin = 64;        // k_window_rank: D (pairs more than D apart must be in order)
constexpr int kMaxUnitSources = 2048;  // distinct sources per unit held in LDS (epoch)

// Error bits (bit index == CDCX_ERR_* code).
constexpr uint32_t kErrTruncated = 2, kErrClockOrder = 3, kErrCorrupt = 4, kErrLimit = 6;

struct Tile {
  int32_t rank;
  int32_t len;
  int64_t start;  // global record index
  int32_t index_in_rank;
  int32_t pad;
};

// T-order compact record: {src, clock, index-or-count, info}; info bit 31 = matched, bit 30 =
// with_next (matched only), bits 0-29 = the record's stream position in its rank (a rank trace
// holds fewer than 2^30 records).  For unmatched records `x` holds event_count.
struct TRec {
  int32_t src;
  int32_t clk;
  int32_t x;
  uint32_t info;
};
constexpr uint32_t kInfoMatched = 0x80000000u, kInfoWithNext = 0x40000000u, kInfoPos = 0x3fffffffu;

struct Chunk {
  int32_t rank;
  int32_t s, e;        // stream positions (inclusive) within the rank
  int32_t first_unit;  // global unit index
  int32_t n_units;
  int32_t pad;
  int64_t out_off;     // byte offset of the chunk's size_t header in the batch output
  int64_t payload;     // payload bytes
};

struct Unit {
  int64_t a;        // T-order start (global)
  int32_t n;        // T-order length
  int32_t rank;
  int32_t chunk;    // global chunk index
  int32_t set_id;
  int32_t M, U, W, S, P;  // matched, unmatched runs, with_next, epoch sources, pairs
  int32_t K;              // chain length (M - P)
  int32_t sort_tile0;     // first global sort tile of the unit
  int32_t nseg;           // closed-prefix segments of the clock-order permutation
  int32_t seg0;           // first global segment index
  int32_t wfail;          // k_window_rank could not rank it (1); epoch/cuts skip units != 0
  int64_t out_off;        // byte offset of the unit in the batch output
  int64_t key_off;        // offset of its sorted keys in the batch key list
};

// Decoder-side unit: section offsets inside the input buffer.
struct DUnit {
  int64_t base;     // byte offset of the unit's first field
  int32_t rank;
  int32_t set_id;
  int32_t M;        // count
  int32_t S, W, Mi, U, Uc, P;
  int64_t ep_off, wp_off, mi_off, uid_off, ucnt_off, pair_off;
  int64_t wbase;    // element offset into decoder scratch (sum of M + 1 over earlier units)
  int64_t rec_off;  // record offset of the unit's reconstructed stream
  int64_t key_off;  // offset of its sorted keys
  int32_t fb;       // permutation rebuild tier the unit is at: 0 pair segments, 1 whole unit in a 16-lane
                    // group, 2 one wave with a 256-slot window, 3 sequential list
  int32_t nseg;     // pair segments of the unit (dec_nseg(P))
  int64_t seg0;     // first of its segments in the batch's segment list
};

// Pair segments of the permutation rebuild (decode.hip): the pair list of a unit is cut every
// kSegPairs pairs; a segment replays the kSegWarm pairs before its own from the untouched list
// first, and its state then is checked against the state its predecessor ends in.
constexpr int32_t kSegPairs = 2048;   // pairs per segment (multiple of 8 * kSegWarm)
constexpr int32_t kSegWarm = 128;     // pairs replayed before a segment's own (multiple of 32)
constexpr int32_t kSegDelta = 32;     // a segment's positions start this far below its smallest pair id
constexpr int32_t kSegWin = 128;      // list positions compared between neighbouring segments (= the window)
constexpr int32_t kSegMaxP = 262144;  // units with more pairs are rebuilt as one segment
constexpr int32_t kSegNoCap = 0x7ffffff0;
__host__ __device__ inline int32_t dec_nseg(int32_t P) {
  return (P <= kSegPairs || P > kSegMaxP) ? 1 : (P + kSegPairs - 1) / kSegPairs;
}
struct DSeg {
  int32_t unit;
  int32_t s;      // ordinal within the unit
  int32_t ka, ke; // its own pairs [ka, ke); the pairs [ka - kSegWarm, ka) are replayed first when s > 0
  int32_t own;    // first list position the segment owns (multiple of 16; 0 for s == 0)
  int32_t cap;    // first position of the next segment (kSegNoCap for the last one)
  int32_t base0;  // window base at the start of the replay
  int32_t pad;
};


// A closed-prefix segment of one unit's permutation: rows [start, start+len) hold exactly
// the columns [start, start+len) (max(c[0..start+len-1]) == start+len-1).
struct Seg {
  int32_t unit;
  int32_t ord;    // ordinal within the unit
  int32_t start;  // first row (= first column)
  int32_t len;
  int32_t lmax;   // highest relative level reached (chain levels inside the segment)
  int32_t qcount; // nodes at lmax
  int32_t entry;  // index into the segment's max-level list where the chain enters
  int32_t pad;
};

struct SortTile {
  int32_t unit;
  int32_t tile;
};

// Totals of a batch that the host reads back to size buffers and grids (lists.hip).
struct EncTotals {
  int32_t n_units;       // non-empty (chunk, table) pairs
  int32_t n_sort_tiles;  // sum of ceil(M / kSortTile)
  int32_t n_fail;        // units the windowed rank could not rank
  int32_t n_big;         // units with more epoch sources than the small k_epoch instance holds
  int64_t n_segs;        // closed-prefix segments
  int64_t matched, with_next, runs, sources;  // sums of M, W, U, S
  int64_t w1n;           // sum of n + 1 (lane-tier leaf scratch rows)
};
struct DecTotals {
  int64_t n_units;
  int64_t rows;       // sum of M + 1 (decoder scratch rows)
  int64_t records;    // reconstructed records
  int64_t keys;       // sum of M
  int64_t rec_tiles;  // k_dec_records tiles
  int64_t segs;       // pair segments (sum of dec_nseg(P))
};

struct DChunk {
  int64_t off;  // absolute payload offset in the input buffer
  int64_t len;
  int32_t rank;
  int32_t pad;
};

}  // namespace cdcx
