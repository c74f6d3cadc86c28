// cdcx_kernels.h -- declarations of the device kernels (definitions in encode.hip,
// decode.hip, gen.hip) for the host orchestrator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "cdcx_layout.h"
#include "gen.h"

namespace cdcx {

constexpr int kScanBlock = 256;  // threads of the single-workgroup list scans (lists.hip)

struct GenArgs {
  gen::Shape sh;
  int32_t first_rank;
  int64_t events;
  uint64_t salt;
};

// encode.hip
__global__ void k_set_dense(const uint32_t*, int16_t*, int32_t*, int32_t*);
__global__ void k_tile_hist(const int32_t*, const Tile*, uint32_t*, uint32_t*, uint32_t*);
__global__ void k_hist_scan(const uint32_t*, const int32_t*, const int32_t*, const int32_t*, const int32_t*, int32_t*,
                            int32_t*, uint8_t*);
__global__ void k_scatter(const int32_t*, const Tile*, const int16_t*, const int32_t*, const uint8_t*, const int32_t*,
                          const int64_t*, TRec*, uint8_t*, int32_t*);
__global__ void k_rank_scan(const int32_t*, const int32_t*, const int32_t*, int32_t*, int32_t*);
__global__ void k_chunks(const int32_t*, const int64_t*, const int64_t*, const int32_t*, const int32_t*, const int32_t*,
                         const uint8_t*, const TRec*, const int32_t*, const int32_t*, const int64_t*, int64_t, int2*,
                         int32_t*);
__global__ void k_units_lb(const Chunk*, int32_t, const int64_t*, const int32_t*, const int32_t*, const int64_t*,
                           const TRec*, int2*, int32_t*, int64_t*);
__global__ void k_unit_prep(Unit*, const TRec*, uint64_t*, int32_t*, int32_t*, int32_t*, uint64_t*, uint32_t*);
__global__ void k_window_rank(Unit*, const SortTile*, const uint64_t*, int32_t*, int32_t*, uint64_t*);
__global__ void k_window_rank_wide(Unit*, const uint64_t*, int32_t*, int32_t*, uint64_t*);
__global__ void k_sort_tiles(const Unit*, const SortTile*, const uint64_t*, uint64_t*, int32_t*, uint64_t*);
__global__ void k_rank_tiles(const Unit*, const SortTile*, const uint64_t*, const uint64_t*, const int32_t*,
                             const uint64_t*, int32_t*, int32_t*, uint64_t*);
template <int HCAP>
__global__ void k_epoch(Unit*, const uint64_t*, uint64_t*, uint64_t*, int64_t, uint32_t*);
// chain.hip
__global__ void k_cuts(Unit*, const int32_t*, int32_t*, int32_t*);
__global__ void k_seg_list(const Unit*, const int32_t*, Seg*);
__global__ void k_seg_hist(const Seg*, int32_t, int32_t*);
__global__ void k_seg_bins(int32_t*);
__global__ void k_seg_order(const Seg*, int32_t, int32_t*, int32_t*);
template <int NL>
__global__ void k_chain_seg(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*, int32_t*,
                            int32_t*, int32_t*, int32_t*, int2*, const int64_t*, uint32_t*, unsigned long long*);
template <int G>
__global__ void k_chain_grp(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*, int32_t*,
                            int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, uint32_t*);
// chain_group8.hip
__global__ void k_chain_grp8(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*, int32_t*,
                             int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t, uint32_t*);
__global__ void k_chain_exits(const Unit*, const Seg*, int32_t, const int32_t*, const int32_t*, const int32_t*, int32_t*,
                              uint32_t*);
__global__ void k_chain_entries(Unit*, int32_t, Seg*, const int32_t*);
__global__ void k_chain_mark(const Unit*, const Seg*, int32_t, const int32_t*, const int32_t*, uint8_t*);
__global__ void k_pos_rows(const Unit*, const int32_t*, const uint8_t*, int32_t*, int32_t*);
__global__ void k_pos_cols(const Unit*, const int32_t*, const uint8_t*, const int32_t*, const int32_t*, uint32_t*,
                           int32_t*);
__global__ void k_deltas(const Unit*, const uint32_t*, const int32_t*, uint8_t*);
__global__ void k_write_units(const Unit*, const int32_t*, const int32_t*, const int32_t*, const uint64_t*,
                              const uint64_t*, const uint64_t*, int64_t, int32_t, uint8_t*);
__global__ void k_chunk_headers(const Chunk*, int32_t, uint8_t*);
__global__ void k_footer_order(const Unit*, const int32_t*, const int32_t*, const uint64_t*, int64_t, int32_t, const int64_t*,
                               const int64_t*, uint64_t*, int32_t*, int32_t*, int32_t*);
__global__ void k_footer_write(const int64_t*, const int64_t*, const uint64_t*, const int32_t*, const int32_t*,
                               const int32_t*, const int64_t*, int32_t, uint8_t*);

// lists.hip
__global__ void k_build_tiles(const int64_t*, const int32_t*, Tile*);
__global__ void k_build_chunks(const int2*, const int64_t*, const int32_t*, const int32_t*, const int32_t*, const int64_t*,
                               Chunk*, int64_t*);
__global__ void k_scan_chunks(Chunk*, int32_t, const int32_t*, const int64_t*, const int32_t*, int32_t, int32_t*, int32_t*,
                              int64_t*, EncTotals*);
__global__ void k_fill_units(const Chunk*, const int64_t*, const int2*, const int32_t*, const int32_t*, const int64_t*,
                             const int64_t*, Unit*, int64_t*);
__global__ void k_units_scan_prep(Unit*, int32_t, EncTotals*);
__global__ void k_fill_sort_tiles(const Unit*, SortTile*);
__global__ void k_units_scan_cuts(Unit*, int64_t*, EncTotals*);
__global__ void k_units_clear_wfail(Unit*, int32_t);
__global__ void k_out_layout(Unit*, Chunk*, int32_t, const int32_t*, int32_t, const int32_t*, int32_t, const EncTotals*,
                             int64_t*, int64_t*, int64_t*, int64_t*, int64_t*, int64_t*);
__global__ void k_dec_scan_chunks(const int32_t*, int32_t, int32_t*, DecTotals*);
__global__ void k_dec_scan_units(DUnit*, int32_t, int32_t, int32_t*, DecTotals*);
__global__ void k_dec_order(const DUnit*, int32_t, int32_t*);
__global__ void k_dec_fill_tiles(const DUnit*, const int32_t*, const uint64_t*, int4*);

// decode.hip
__global__ void k_dec_count_chunks(const uint8_t*, const int64_t*, const int64_t*, int32_t, int32_t*, uint32_t*);
__global__ void k_dec_list_chunks(const uint8_t*, const int64_t*, const int32_t*, const int32_t*, int32_t, DChunk*);
__global__ void k_dec_units(const uint8_t*, const DChunk*, int32_t, const int32_t*, int32_t*, DUnit*, uint32_t*);
__global__ void k_dec_chunk_units(const uint8_t*, int64_t, int32_t, int64_t, int64_t, int32_t*, int32_t*, DUnit*);
__global__ void k_dec_sections(const DUnit*, const uint8_t*, uint64_t*, uint64_t*, uint8_t*, uint32_t*);
__global__ void k_dec_perm_lane(const DUnit*, int32_t, const uint64_t*, const uint64_t*, int32_t*, int32_t*, int32_t*,
                                uint32_t*);
__global__ void k_dec_pair_scan(const DUnit*, const uint8_t*, int32_t, DSeg*, int64_t*, uint64_t*, uint64_t*);
template <int MODE>
__global__ void k_dec_perm_seg(DUnit*, const int32_t*, const DSeg*, int64_t, int32_t, const uint8_t*, const int64_t*,
                               int32_t*, int32_t*, int32_t*, int32_t*, int32_t*);
__global__ void k_dec_perm_check(DUnit*, const DSeg*, int64_t, const int32_t*, const int32_t*, int32_t*, int32_t, int32_t*,
                                 int32_t*);
__global__ void k_dec_perm_inv(const DUnit*, const int32_t*, const int32_t*, int32_t*);

__global__ void k_dec_cinv(const DUnit*, const int32_t*, int32_t*);
template <int K>
__global__ void k_dec_perm_window(DUnit*, int32_t, int32_t, const uint64_t*, const uint64_t*, int32_t*, int32_t*);
__global__ void k_dec_records(const DUnit*, const int4*, const uint8_t*, const int32_t*, const uint8_t*, const uint64_t*,
                              const int2*, int4*);
__global__ void k_verify_roundtrip(const Unit*, const int64_t*, const int64_t*, const TRec*, const int4*, const int4*,
                                   unsigned long long*);
__global__ void k_dec_pack_tables(const DUnit*, const int64_t*, const uint64_t*, const uint64_t*, const uint64_t*,
                                  const uint64_t*, uint64_t*);

// gen.hip
__global__ void k_gen_tile_sums(GenArgs, int64_t, int32_t, int32_t*, int32_t*);
__global__ void k_gen_rank_scan(GenArgs, int32_t, int32_t*, int32_t*);
__global__ void k_gen_frames(GenArgs, int64_t, int32_t, const int32_t*, const int32_t*, int32_t*, int32_t*, int32_t*,
                             int32_t*, int32_t*);
__global__ void k_gen_akeys(GenArgs, int64_t, const int32_t*, int64_t*);
__global__ void k_gen_arrival(GenArgs, int64_t, const int32_t*, const int64_t*, int32_t*);
__global__ void k_gen_records(GenArgs, int64_t, int64_t, const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                              const int32_t*, const int64_t*, int4*);
std::vector<int32_t> generate_host(const GenArgs& g, int32_t r);

}  // namespace cdcx
