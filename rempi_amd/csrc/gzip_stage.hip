// gzip_stage.hip -- the REMPI_GZIP=1 stage of a CDC rank file, on the host.
//
// With REMPI_GZIP=1 the reference writes each chunk as [size_t compressed size][one zlib stream
// of the chunk payload] (rempi_encoder_cdc::write_record_file, rempi_encoder_cdc.cpp:804-844;
// the stream is deflateInit(Z_DEFAULT_COMPRESSION) over the chunk's write queue with
// Z_NO_FLUSH between pieces and Z_FINISH at the end, rempi_compression_util.cpp:233-325), and
// reads it back by inflating (:960-978).  The separator (size_t 0) and the footer (:2085-2135)
// are written as they are.  Deflate's output does not depend on how its input is split into
// pieces, so one deflate call per chunk payload gives the reference's bytes (with the same
// zlib; both use the system libz of the image).  The deflate output cannot be made on the GPU
// and still match zlib byte for byte, so this stage stays on the host; chunks are
// independent and are compressed on several threads.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "gzip_stage.h"

namespace cdcx {

namespace {

struct Piece {
  size_t off, len;  // payload in the input
};

// Chunk payloads of a framed rank file: [size_t n][n bytes]... until the separator (0);
// *rest = offset of the separator (len when the file has none).
std::vector<Piece> chunks_of(const uint8_t* in, size_t len, size_t* rest) {
  std::vector<Piece> v;
  size_t p = 0;
  while (p < len) {
    if (len - p < 8) throw GzipError{"truncated chunk length"};
    uint64_t n;
    memcpy(&n, in + p, 8);
    if (n == 0) break;  // all_epoch_rank_separator: the footer follows
    if (n > len - p - 8) throw GzipError{"chunk runs past the end of the file"};
    v.push_back(Piece{p + 8, (size_t)n});
    p += 8 + n;
  }
  *rest = p;
  return v;
}

template <class F>
void parallel_for(size_t n, F&& f) {
  const size_t nt = std::min<size_t>(n, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (nt <= 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> err(nt);
  for (size_t t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      try {
        for (size_t i; (i = next++) < n;) f(i);
      } catch (...) {
        err[t] = std::current_exception();
      }
    });
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

std::vector<uint8_t> frame(const std::vector<std::vector<uint8_t>>& z, const uint8_t* in, size_t rest, size_t len) {
  size_t total = len - rest;
  for (auto& b : z) total += 8 + b.size();
  std::vector<uint8_t> out;
  out.reserve(total);
  for (auto& b : z) {
    const uint64_t n = b.size();
    out.insert(out.end(), reinterpret_cast<const uint8_t*>(&n), reinterpret_cast<const uint8_t*>(&n) + 8);
    out.insert(out.end(), b.begin(), b.end());
  }
  out.insert(out.end(), in + rest, in + len);
  return out;
}

}  // namespace

// zlib counts input and output in uInt: larger buffers are fed in pieces (the stream does not
// depend on how its input or output space is split).
constexpr size_t kZPiece = (size_t)1 << 30;

std::vector<uint8_t> deflate_payload(const uint8_t* p, size_t n) {
  z_stream s{};
  if (deflateInit(&s, Z_DEFAULT_COMPRESSION) != Z_OK) throw GzipError{"deflateInit failed"};
  // deflateBound takes a uLong (64-bit here); add the per-piece slack of stored blocks
  std::vector<uint8_t> out((size_t)deflateBound(&s, (uLong)n) + 64);
  size_t in_pos = 0, out_pos = 0;
  int rc = Z_OK;
  do {
    const size_t take = std::min(kZPiece, n - in_pos);
    s.next_in = const_cast<Bytef*>(p + in_pos);
    s.avail_in = (uInt)take;
    in_pos += take;
    const int flush = (in_pos == n) ? Z_FINISH : Z_NO_FLUSH;
    do {
      const size_t room = std::min(kZPiece, out.size() - out_pos);
      if (room == 0) {
        deflateEnd(&s);
        throw GzipError{"deflate output exceeds deflateBound"};
      }
      s.next_out = out.data() + out_pos;
      s.avail_out = (uInt)room;
      rc = deflate(&s, flush);
      out_pos += room - s.avail_out;
      if (rc == Z_STREAM_ERROR) break;
    } while (s.avail_out == 0 && rc != Z_STREAM_END);
    if (rc == Z_STREAM_ERROR) break;
  } while (in_pos < n);
  deflateEnd(&s);
  if (rc != Z_STREAM_END) throw GzipError{"deflate did not finish"};
  out.resize(out_pos);
  return out;
}

// One chunk = exactly one zlib stream (rempi_encoder_cdc.cpp:960-978 inflates the whole
// chunk): input that ends inside the stream, or bytes left after its end, are corrupt.
std::vector<uint8_t> inflate_payload(const uint8_t* p, size_t n) {
  z_stream s{};
  if (inflateInit(&s) != Z_OK) throw GzipError{"inflateInit failed"};
  std::vector<uint8_t> out(std::max<size_t>(4 * n, 4096));
  size_t in_pos = 0, out_pos = 0;
  int rc = Z_OK;
  while (true) {
    if (s.avail_in == 0 && in_pos < n) {
      const size_t take = std::min(kZPiece, n - in_pos);
      s.next_in = const_cast<Bytef*>(p + in_pos);
      s.avail_in = (uInt)take;
      in_pos += take;
    }
    if (out_pos == out.size()) out.resize(out.size() * 2);
    const size_t room = std::min(kZPiece, out.size() - out_pos);
    s.next_out = out.data() + out_pos;
    s.avail_out = (uInt)room;
    rc = inflate(&s, Z_NO_FLUSH);
    out_pos += room - s.avail_out;
    if (rc == Z_STREAM_END) break;
    if (rc != Z_OK && rc != Z_BUF_ERROR) break;
    if (s.avail_out != 0 && s.avail_in == 0 && in_pos == n) {
      rc = Z_DATA_ERROR;  // input ended inside the stream
      break;
    }
  }
  const bool trailing = (rc == Z_STREAM_END) && (s.avail_in != 0 || in_pos != n);
  inflateEnd(&s);
  if (rc != Z_STREAM_END) throw GzipError{"corrupt zlib chunk"};
  if (trailing) throw GzipError{"bytes after the end of a chunk's zlib stream"};
  out.resize(out_pos);
  return out;
}

std::vector<uint8_t> gzip_file(const uint8_t* in, size_t len) {
  size_t rest;
  const std::vector<Piece> pc = chunks_of(in, len, &rest);
  std::vector<std::vector<uint8_t>> z(pc.size());
  parallel_for(pc.size(), [&](size_t i) { z[i] = deflate_payload(in + pc[i].off, pc[i].len); });
  return frame(z, in, rest, len);
}

std::vector<uint8_t> gunzip_file(const uint8_t* in, size_t len) {
  size_t rest;
  const std::vector<Piece> pc = chunks_of(in, len, &rest);
  std::vector<std::vector<uint8_t>> z(pc.size());
  parallel_for(pc.size(), [&](size_t i) { z[i] = inflate_payload(in + pc[i].off, pc[i].len); });
  return frame(z, in, rest, len);
}

}  // namespace cdcx
