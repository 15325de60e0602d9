// libFuzzer target: HPACK (RFC 7541) decoder and Huffman codec (hpack.cpp).
//
// Properties checked beyond memory safety:
//  * a block that decodes re-encodes (literal, never-indexed, Huffman or not) into a
//    block that a fresh decoder decodes to the same header list;
//  * Huffman encode -> decode is the identity on arbitrary bytes;
//  * the dynamic table never exceeds the advertised 4096-octet limit;
//  * the server's visitor decode (views, no header strings) accepts/rejects the same
//    blocks, yields the same headers and leaves the same dynamic-table state as the
//    vector decode;
//  * the table-driven Huffman decoder agrees with the bit-by-bit reference.
// The first input byte splits the rest into two header blocks decoded on one decoder,
// so dynamic-table state carried across blocks (and size updates) is exercised.
#include <cstdint>
#include <cstdlib>

#include "fuzz_common.h"

using namespace amdgpu_dp;

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  if (const char* dir = fuzzutil::seed_dir()) {
    std::string b = fuzzutil::grpc_headers("/v1beta1.DevicePlugin/Allocate", false);
    fuzzutil::write_seed(dir, "grpc_plain", std::string(1, static_cast<char>(b.size())) + b + b);
    b = fuzzutil::grpc_headers("/v1beta1.DevicePlugin/ListAndWatch", true);
    fuzzutil::write_seed(dir, "grpc_huffman", std::string(1, static_cast<char>(b.size())) + b);
    // incremental indexing (0x40) then a reference to the new entry (index 62) in block 2
    std::string inc = "\x40\x0a" "custom-key" "\x0d" "custom-header";
    fuzzutil::write_seed(dir, "indexed_dynamic", std::string(1, static_cast<char>(inc.size())) + inc + "\xbe");
    // dynamic table size update to 0 and back
    fuzzutil::write_seed(dir, "size_update", std::string("\x03\x20\x3f\xe1\x1f", 5));
    std::exit(0);
  }
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  const size_t split = std::min<size_t>(data[0], size - 1);
  const uint8_t* p = data + 1;
  hpack::Decoder d;
  std::vector<hpack::Header> h1, h2;
  const bool ok1 = d.decode(p, split, &h1);
  if (d.table_size() > 4096) std::abort();
  if (ok1) {
    (void)d.decode(p + split, size - 1 - split, &h2);
    if (d.table_size() > 4096) std::abort();
    for (int huff = 0; huff < 2; ++huff) {
      std::string blk;
      for (const auto& h : h1) hpack::encode_literal(&blk, h.name, h.value, huff != 0);
      hpack::Decoder fresh;
      std::vector<hpack::Header> back;
      if (!fresh.decode(reinterpret_cast<const uint8_t*>(blk.data()), blk.size(), &back)) std::abort();
      if (back.size() != h1.size()) std::abort();
      for (size_t i = 0; i < back.size(); ++i)
        if (back[i].name != h1[i].name || back[i].value != h1[i].value) std::abort();
    }
  }
  {  // differential: visitor decode vs vector decode, over the same two blocks
    hpack::Decoder a, b;
    std::vector<hpack::Header> va;
    std::vector<std::pair<std::string, std::string>> vb;
    auto sink = [](void* ctx, std::string_view n, std::string_view v) {
      static_cast<std::vector<std::pair<std::string, std::string>>*>(ctx)->emplace_back(n, v);
    };
    const uint8_t* blocks[2] = {p, p + split};
    const size_t lens[2] = {split, size - 1 - split};
    for (int k = 0; k < 2; ++k) {
      va.clear();
      vb.clear();
      const bool ra = a.decode(blocks[k], lens[k], &va);
      const bool rb = b.decode(blocks[k], lens[k], sink, &vb);
      if (ra != rb) std::abort();
      if (!ra) break;
      if (va.size() != vb.size() || a.table_size() != b.table_size() || a.table_entries() != b.table_entries())
        std::abort();
      for (size_t i = 0; i < va.size(); ++i)
        if (va[i].name != vb[i].first || va[i].value != vb[i].second) std::abort();
    }
  }
  {
    std::string x, y;
    const bool rx = hpack::huffman_decode(p, size - 1, &x);
    const bool ry = hpack::huffman_decode_bitwise(p, size - 1, &y);
    if (rx != ry || (rx && x != y)) std::abort();
  }
  const std::string_view raw(reinterpret_cast<const char*>(p), size - 1);
  std::string enc, dec;
  hpack::huffman_encode(raw, &enc);
  if (enc.size() != hpack::huffman_encoded_len(raw)) std::abort();
  if (!hpack::huffman_decode(reinterpret_cast<const uint8_t*>(enc.data()), enc.size(), &dec) || dec != raw)
    std::abort();
  dec.clear();
  (void)hpack::huffman_decode(p, size - 1, &dec);
  return 0;
}
