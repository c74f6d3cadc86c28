// gzip_stage.h -- host-side REMPI_GZIP=1 stage of CDC rank files (gzip_stage.hip).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace cdcx {

struct GzipError {
  const char* msg;
};

// One chunk payload as the reference compresses it (zlib stream, Z_DEFAULT_COMPRESSION).
std::vector<uint8_t> deflate_payload(const uint8_t* p, size_t n);
std::vector<uint8_t> inflate_payload(const uint8_t* p, size_t n);
// Whole rank files: every chunk payload (de)compressed, separator and footer kept.
std::vector<uint8_t> gzip_file(const uint8_t* in, size_t len);
std::vector<uint8_t> gunzip_file(const uint8_t* in, size_t len);

}  // namespace cdcx
