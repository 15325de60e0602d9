// HPACK (RFC 7541) for the native HTTP/2 gRPC server and its load-generator client.
//
// Decoder: full static + dynamic table, Huffman strings, table-size updates - kubelet
// (grpc-go) and grpcio both index and Huffman-code their request headers.
// Encoder: stateless (static-table references and literals "without indexing"), so a
// response never depends on per-connection encoder state.
#pragma once

#include <cstddef>
#include <cstdint>
#include <deque>
#include <string>
#include <string_view>
#include <vector>

namespace amdgpu_dp {
namespace hpack {

struct Header {
  std::string name;
  std::string value;
};

bool huffman_decode(const uint8_t* p, size_t n, std::string* out);
void huffman_encode(std::string_view s, std::string* out);
size_t huffman_encoded_len(std::string_view s);

// Integer with an N-bit prefix; `first` carries the representation's flag bits.
void encode_int(std::string* out, uint8_t first, int prefix_bits, uint64_t v);
bool decode_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v);

// Encoder helpers (stateless).
void encode_indexed(std::string* out, int static_index);
void encode_literal(std::string* out, std::string_view name, std::string_view value, bool huffman = false);
void encode_literal_name_index(std::string* out, int static_name_index, std::string_view value, bool huffman = false);
int static_index(std::string_view name, std::string_view value, bool* value_match);

// Bit-by-bit canonical decoder: the reference the table-driven huffman_decode is
// tested against.
bool huffman_decode_bitwise(const uint8_t* p, size_t n, std::string* out);

// Visitor for Decoder::decode: name/value views are valid only during the call (they
// point into the static table, the dynamic table, the input block or scratch space).
using HeaderFn = void (*)(void* ctx, std::string_view name, std::string_view value);

class Decoder {
 public:
  explicit Decoder(size_t max_table_size = 4096) : limit_(max_table_size), max_(max_table_size) {}
  // Decodes one complete header block.  false = COMPRESSION_ERROR (connection fatal).
  bool decode(const uint8_t* p, size_t n, std::vector<Header>* out);
  // Same, without materialising headers: static-table and dynamic-table entries and
  // raw literals are passed as views (no allocation); Huffman literals decode into
  // reused scratch buffers.  The request hot path of the gRPC server.
  bool decode(const uint8_t* p, size_t n, HeaderFn fn, void* ctx);
  size_t table_size() const { return size_; }
  size_t table_entries() const { return dyn_.size(); }

 private:
  bool get(uint64_t index, Header* h) const;
  void insert(Header h);
  void evict();
  bool name_of(uint64_t index, std::string_view* name) const;
  bool entry(uint64_t index, std::string_view* name, std::string_view* value) const;
  std::deque<Header> dyn_;  // front = most recent (index 62)
  std::string name_buf_, value_buf_;  // Huffman scratch for the visitor decode
  size_t size_ = 0;
  size_t limit_;  // SETTINGS_HEADER_TABLE_SIZE we advertised
  size_t max_;    // current max set by the encoder's size updates
};

}  // namespace hpack
}  // namespace amdgpu_dp
