// hash_order.h -- iteration order of libstdc++'s std::unordered_{map,set} with an identity
// hash (std::hash<size_t>, std::hash<int>), reproduced on host and device.
//
// Two on-disk sections of a CDC record depend on it:
//  * the epoch line of each table, emitted by iterating unordered_map<size_t,size_t>
//    (rempi_encoder_cdc.cpp:246-267), and
//  * the footer rank list, emitted by iterating the static unordered_set<int>
//    all_epoch_rank_uset (rempi_encoder_cdc.cpp:60, :266, :2094-2103).
//
// Model (libstdc++ _Hashtable, unique keys): singly linked node list headed by a
// "before begin" sentinel; bucket b stores the node *preceding* its first node.  A new key
// goes to the front of its bucket, or to the front of the whole list when its bucket is
// empty.  Before an insertion that would make size > bucket_count the table is rehashed to
// the next count of kHashBuckets, re-threading nodes in list order.  The bucket schedule
// was read off the image's libstdc++ (GCC 11) and is re-checked against the live
// std::unordered_map / unordered_set by tests/test_hash_order.py.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CDCX_HD __host__ __device__
#else
#define CDCX_HD
#endif

namespace cdcx {

// bucket_count after growth, starting from the empty table's single bucket.
static constexpr int kNumHashBuckets = 20;
CDCX_HD inline uint64_t hash_bucket_count(int step) {
  const uint64_t t[kNumHashBuckets] = {1,       13,       29,       59,       127,      257,     541,
                                       1109,    2357,     5087,     10273,    20753,    42043,   85229,
                                       172933,  351061,   712697,   1447153,  2938679,  5967347};
  return t[step < kNumHashBuckets ? step : kNumHashBuckets - 1];
}

// Emulator over caller-provided storage: key/next arrays of capacity `cap` nodes and a
// bucket array of capacity >= the largest bucket count reached (next count above cap).
// Node indices are int32; -1 = null.  Bucket slots: -1 empty, -2 = before-begin sentinel,
// else the index of the node preceding the bucket's first node.
struct HashOrder {
  uint64_t* key;
  int32_t* next;
  int32_t* bucket;
  int32_t head;
  int32_t size;
  int step;

  CDCX_HD void init(uint64_t* k, int32_t* n, int32_t* b) {
    key = k;
    next = n;
    bucket = b;
    head = -1;
    size = 0;
    step = 0;
    bucket[0] = -1;
  }
  CDCX_HD uint64_t nb() const { return hash_bucket_count(step); }
  CDCX_HD int32_t after(int32_t slot) const { return slot == -2 ? head : next[slot]; }
  CDCX_HD void set_after(int32_t slot, int32_t v) {
    if (slot == -2) head = v; else next[slot] = v;
  }
  CDCX_HD void rehash() {
    step++;
    const uint64_t n = nb();
    for (uint64_t i = 0; i < n; i++) bucket[i] = -1;
    int32_t p = head;
    head = -1;
    uint64_t bbegin = 0;
    while (p != -1) {
      int32_t nx = next[p];
      uint64_t b = key[p] % n;
      if (bucket[b] == -1) {
        next[p] = head;
        head = p;
        bucket[b] = -2;
        if (next[p] != -1) bucket[bbegin] = p;
        bbegin = b;
      } else {
        int32_t prev = bucket[b];
        next[p] = after(prev);
        set_after(prev, p);
      }
      p = nx;
    }
  }
  // Insert a key known NOT to be present yet.
  CDCX_HD void insert_new(uint64_t k) {
    if ((uint64_t)size + 1 > nb()) rehash();
    const uint64_t n = nb();
    const uint64_t b = k % n;
    int32_t id = size++;
    key[id] = k;
    if (bucket[b] != -1) {
      int32_t prev = bucket[b];
      next[id] = after(prev);
      set_after(prev, id);
    } else {
      next[id] = head;
      head = id;
      if (next[id] != -1) bucket[key[next[id]] % n] = id;
      bucket[b] = -2;
    }
  }
  // Membership test by walking the key's bucket.
  CDCX_HD bool contains(uint64_t k) const {
    const uint64_t n = nb();
    const uint64_t b = k % n;
    if (size == 0 || bucket[b] == -1) return false;
    for (int32_t p = after(bucket[b]); p != -1 && key[p] % n == b; p = next[p])
      if (key[p] == k) return true;
    return false;
  }
};

// Largest bucket count the emulator reaches for `n` distinct keys (bucket storage size).
CDCX_HD inline uint64_t hash_bucket_capacity(uint64_t n) {
  int s = 0;
  while (s + 1 < kNumHashBuckets && hash_bucket_count(s) < n) s++;
  return hash_bucket_count(s);
}

}  // namespace cdcx
