#include "hpack.h"

#include <algorithm>
#include <array>

namespace amdgpu_dp {
namespace hpack {

namespace {

struct Sym {
  uint32_t code;
  uint32_t len;
};

const Sym kHuff[257] = {
#include "hpack_huffman.inc"
};

// RFC 7541 Appendix A
const char* const kStatic[61][2] = {
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""},
    {"cache-control", ""}, {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""},
    {"content-length", ""}, {"content-location", ""}, {"content-range", ""}, {"content-type", ""},
    {"cookie", ""}, {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""},
    {"proxy-authenticate", ""}, {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""},
    {"retry-after", ""}, {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""},
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""},
};

// Canonical-code decode tables: per bit length, the first code, the count and the
// offset into the (length, symbol)-sorted symbol list.
struct Canon {
  uint32_t first[32] = {};
  uint32_t count[32] = {};
  uint32_t offset[32] = {};
  uint16_t syms[257] = {};
  Canon() {
    std::array<uint16_t, 257> order;
    for (int i = 0; i < 257; ++i) order[i] = static_cast<uint16_t>(i);
    std::stable_sort(order.begin(), order.end(),
                     [](uint16_t a, uint16_t b) { return kHuff[a].len < kHuff[b].len; });
    for (int i = 0; i < 257; ++i) syms[i] = order[i];
    uint32_t idx = 0;
    for (uint32_t L = 1; L < 32; ++L) {
      offset[L] = idx;
      bool seen = false;
      while (idx < 257 && kHuff[order[idx]].len == L) {
        if (!seen) {
          first[L] = kHuff[order[idx]].code;
          seen = true;
        }
        ++count[L];
        ++idx;
      }
    }
  }
};

const Canon& canon() {
  static const Canon c;
  return c;
}

}  // namespace

bool huffman_decode_bitwise(const uint8_t* p, size_t n, std::string* out) {
  const Canon& c = canon();
  uint32_t code = 0;
  uint32_t len = 0;
  for (size_t i = 0; i < n; ++i) {
    for (int b = 7; b >= 0; --b) {
      code = (code << 1) | ((p[i] >> b) & 1u);
      ++len;
      if (len > 30) return false;
      if (c.count[len] && code >= c.first[len] && code - c.first[len] < c.count[len]) {
        const uint16_t sym = c.syms[c.offset[len] + (code - c.first[len])];
        if (sym == 256) return false;  // EOS inside a string is an error
        out->push_back(static_cast<char>(sym));
        code = 0;
        len = 0;
      }
    }
  }
  // padding: < 8 bits, all ones (the most significant bits of EOS)
  if (len >= 8) return false;
  return code == ((1u << len) - 1u);
}

namespace {

// Primary lookup on the next kPeek bits: every code of length <= kPeek (all of
// printable ASCII except a few symbols) resolves in one step; longer codes fall back
// to the canonical first/count search from length kPeek+1.
constexpr int kPeek = 10;

struct FastTable {
  uint16_t sym[1 << kPeek];
  uint8_t len[1 << kPeek];  // 0 = no code of length <= kPeek has this prefix
  FastTable() {
    for (int i = 0; i < (1 << kPeek); ++i) len[i] = 0;
    for (int s = 0; s < 257; ++s) {
      const int L = static_cast<int>(kHuff[s].len);
      if (L > kPeek) continue;
      const uint32_t base = kHuff[s].code << (kPeek - L);
      for (uint32_t k = 0; k < (1u << (kPeek - L)); ++k) {
        sym[base + k] = static_cast<uint16_t>(s);
        len[base + k] = static_cast<uint8_t>(L);
      }
    }
  }
};

const FastTable& fast_table() {
  static const FastTable t;
  return t;
}

}  // namespace

bool huffman_decode(const uint8_t* p, size_t n, std::string* out) {
  const FastTable& ft = fast_table();
  const Canon& c = canon();
  uint64_t acc = 0;  // bit buffer, the next `bits` bits right-aligned
  int bits = 0;
  size_t i = 0;
  out->reserve(out->size() + n * 8 / 5 + 1);
  for (;;) {
    while (bits <= 56 && i < n) {
      acc = (acc << 8) | p[i++];
      bits += 8;
    }
    if (bits == 0) return true;
    // peek kPeek bits; past the end pad with ones (EOS prefix), as a valid string's padding is
    const uint32_t peek = bits >= kPeek
                              ? static_cast<uint32_t>(acc >> (bits - kPeek)) & ((1u << kPeek) - 1)
                              : static_cast<uint32_t>(((acc << (kPeek - bits)) | ((1u << (kPeek - bits)) - 1)) &
                                                      ((1u << kPeek) - 1));
    int L = ft.len[peek];
    uint16_t sym = ft.sym[peek];
    if (L == 0) {  // code longer than kPeek bits
      L = -1;
      for (int len = kPeek + 1; len <= 30 && len <= bits; ++len) {
        const uint32_t code = static_cast<uint32_t>(acc >> (bits - len)) & ((1u << len) - 1);
        if (c.count[len] && code >= c.first[len] && code - c.first[len] < c.count[len]) {
          sym = c.syms[c.offset[len] + (code - c.first[len])];
          L = len;
          break;
        }
      }
      if (L < 0) {  // not enough bits left for any code: must be padding
        if (i < n) return false;  // (cannot happen with 56+ bits buffered)
        if (bits >= 8) return false;
        return (acc & ((1u << bits) - 1)) == ((1u << bits) - 1);
      }
    }
    if (L > bits) {  // the match used padding ones: the rest is padding
      if (bits >= 8) return false;
      return (acc & ((1u << bits) - 1)) == ((1u << bits) - 1);
    }
    if (sym == 256) return false;  // EOS inside a string is an error
    out->push_back(static_cast<char>(sym));
    bits -= L;
    acc &= bits ? ((uint64_t{1} << bits) - 1) : 0;
  }
}

size_t huffman_encoded_len(std::string_view s) {
  uint64_t bits = 0;
  for (unsigned char ch : s) bits += kHuff[ch].len;
  return static_cast<size_t>((bits + 7) / 8);
}

void huffman_encode(std::string_view s, std::string* out) {
  uint64_t acc = 0;
  int nbits = 0;
  for (unsigned char ch : s) {
    acc = (acc << kHuff[ch].len) | kHuff[ch].code;
    nbits += static_cast<int>(kHuff[ch].len);
    while (nbits >= 8) {
      nbits -= 8;
      out->push_back(static_cast<char>((acc >> nbits) & 0xFF));
    }
  }
  if (nbits > 0) out->push_back(static_cast<char>(((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)) & 0xFF));
}

void encode_int(std::string* out, uint8_t first, int prefix_bits, uint64_t v) {
  const uint64_t maxp = (1u << prefix_bits) - 1;
  if (v < maxp) {
    out->push_back(static_cast<char>(first | v));
    return;
  }
  out->push_back(static_cast<char>(first | maxp));
  v -= maxp;
  while (v >= 128) {
    out->push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

bool decode_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v) {
  if (p >= end) return false;
  const uint64_t maxp = (1u << prefix_bits) - 1;
  uint64_t x = *p++ & maxp;
  if (x < maxp) {
    *v = x;
    return true;
  }
  for (int shift = 0; shift < 56; shift += 7) {
    if (p >= end) return false;
    const uint8_t b = *p++;
    x += static_cast<uint64_t>(b & 0x7F) << shift;
    if (!(b & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}

static void encode_string(std::string* out, std::string_view s, bool huffman) {
  if (huffman) {
    encode_int(out, 0x80, 7, huffman_encoded_len(s));
    huffman_encode(s, out);
  } else {
    encode_int(out, 0x00, 7, s.size());
    out->append(s.data(), s.size());
  }
}

static bool decode_string(const uint8_t*& p, const uint8_t* end, std::string* out) {
  if (p >= end) return false;
  const bool huff = (*p & 0x80) != 0;
  uint64_t len;
  if (!decode_int(p, end, 7, &len)) return false;
  if (len > static_cast<uint64_t>(end - p)) return false;
  out->clear();
  if (huff) {
    if (!huffman_decode(p, static_cast<size_t>(len), out)) return false;
  } else {
    out->assign(reinterpret_cast<const char*>(p), static_cast<size_t>(len));
  }
  p += len;
  return true;
}

void encode_indexed(std::string* out, int idx) { encode_int(out, 0x80, 7, static_cast<uint64_t>(idx)); }

void encode_literal(std::string* out, std::string_view name, std::string_view value, bool huffman) {
  out->push_back(0x00);  // literal without indexing, new name
  encode_string(out, name, huffman);
  encode_string(out, value, huffman);
}

void encode_literal_name_index(std::string* out, int idx, std::string_view value, bool huffman) {
  encode_int(out, 0x00, 4, static_cast<uint64_t>(idx));
  encode_string(out, value, huffman);
}

int static_index(std::string_view name, std::string_view value, bool* value_match) {
  int name_only = 0;
  for (int i = 0; i < 61; ++i) {
    if (name == kStatic[i][0]) {
      if (value == kStatic[i][1]) {
        *value_match = true;
        return i + 1;
      }
      if (!name_only) name_only = i + 1;
    }
  }
  *value_match = false;
  return name_only;
}

bool Decoder::get(uint64_t index, Header* h) const {
  if (index == 0) return false;
  if (index <= 61) {
    h->name = kStatic[index - 1][0];
    h->value = kStatic[index - 1][1];
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) return false;
  *h = dyn_[static_cast<size_t>(d)];
  return true;
}

void Decoder::evict() {
  while (size_ > max_ && !dyn_.empty()) {
    size_ -= dyn_.back().name.size() + dyn_.back().value.size() + 32;
    dyn_.pop_back();
  }
}

void Decoder::insert(Header h) {
  const size_t sz = h.name.size() + h.value.size() + 32;
  if (sz > max_) {  // larger than the table: empties it (RFC 7541 §4.4)
    dyn_.clear();
    size_ = 0;
    return;
  }
  size_ += sz;
  dyn_.push_front(std::move(h));
  evict();
}

bool Decoder::name_of(uint64_t index, std::string_view* name) const {
  if (index == 0) return false;
  if (index <= 61) {
    *name = kStatic[index - 1][0];
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) return false;
  *name = dyn_[static_cast<size_t>(d)].name;
  return true;
}

bool Decoder::entry(uint64_t index, std::string_view* name, std::string_view* value) const {
  if (index == 0) return false;
  if (index <= 61) {
    *name = kStatic[index - 1][0];
    *value = kStatic[index - 1][1];
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) return false;
  const Header& h = dyn_[static_cast<size_t>(d)];
  *name = h.name;
  *value = h.value;
  return true;
}

namespace {

// A string literal as a view: raw bytes in place, Huffman decoded into `scratch`.
bool string_view_of(const uint8_t*& p, const uint8_t* end, std::string* scratch, std::string_view* out) {
  if (p >= end) return false;
  const bool huff = (*p & 0x80) != 0;
  uint64_t len;
  if (!decode_int(p, end, 7, &len)) return false;
  if (len > static_cast<uint64_t>(end - p)) return false;
  if (huff) {
    scratch->clear();
    if (!huffman_decode(p, static_cast<size_t>(len), scratch)) return false;
    *out = *scratch;
  } else {
    *out = std::string_view(reinterpret_cast<const char*>(p), static_cast<size_t>(len));
  }
  p += len;
  return true;
}

}  // namespace

bool Decoder::decode(const uint8_t* p, size_t n, HeaderFn fn, void* ctx) {
  const uint8_t* end = p + n;
  bool header_seen = false;
  while (p < end) {
    const uint8_t b = *p;
    std::string_view name, value;
    if (b & 0x80) {  // indexed
      uint64_t idx;
      if (!decode_int(p, end, 7, &idx) || !entry(idx, &name, &value)) return false;
      fn(ctx, name, value);
      header_seen = true;
    } else if ((b & 0xE0) == 0x20) {  // dynamic table size update
      if (header_seen) return false;
      uint64_t sz;
      if (!decode_int(p, end, 5, &sz) || sz > limit_) return false;
      max_ = static_cast<size_t>(sz);
      evict();
    } else {
      const bool indexing = (b & 0xC0) == 0x40;  // else without indexing / never indexed
      uint64_t idx;
      if (!decode_int(p, end, indexing ? 6 : 4, &idx)) return false;
      if (idx) {
        if (!name_of(idx, &name)) return false;
      } else if (!string_view_of(p, end, &name_buf_, &name)) {
        return false;
      }
      if (!string_view_of(p, end, &value_buf_, &value)) return false;
      if (indexing) {  // table state must follow the encoder: copy first (views may
                       // point into entries the insertion evicts), insert, view the entry
        Header h{std::string(name), std::string(value)};
        if (h.name.size() + h.value.size() + 32 <= max_) {
          insert(std::move(h));
          fn(ctx, dyn_.front().name, dyn_.front().value);
        } else {  // larger than the table: delivered, and the table is emptied (§4.4)
          fn(ctx, h.name, h.value);
          dyn_.clear();
          size_ = 0;
        }
      } else {
        fn(ctx, name, value);
      }
      header_seen = true;
    }
  }
  return true;
}

bool Decoder::decode(const uint8_t* p, size_t n, std::vector<Header>* out) {
  const uint8_t* end = p + n;
  bool header_seen = false;
  while (p < end) {
    const uint8_t b = *p;
    Header h;
    if (b & 0x80) {  // indexed
      uint64_t idx;
      if (!decode_int(p, end, 7, &idx) || !get(idx, &h)) return false;
      out->push_back(std::move(h));
      header_seen = true;
    } else if ((b & 0xC0) == 0x40) {  // literal with incremental indexing
      uint64_t idx;
      if (!decode_int(p, end, 6, &idx)) return false;
      if (idx) {
        Header nh;
        if (!get(idx, &nh)) return false;
        h.name = std::move(nh.name);
      } else if (!decode_string(p, end, &h.name)) {
        return false;
      }
      if (!decode_string(p, end, &h.value)) return false;
      insert(h);
      out->push_back(std::move(h));
      header_seen = true;
    } else if ((b & 0xE0) == 0x20) {  // dynamic table size update
      if (header_seen) return false;  // must come first in a block
      uint64_t sz;
      if (!decode_int(p, end, 5, &sz) || sz > limit_) return false;
      max_ = static_cast<size_t>(sz);
      evict();
    } else {  // literal without indexing (0000) / never indexed (0001)
      uint64_t idx;
      if (!decode_int(p, end, 4, &idx)) return false;
      if (idx) {
        Header nh;
        if (!get(idx, &nh)) return false;
        h.name = std::move(nh.name);
      } else if (!decode_string(p, end, &h.name)) {
        return false;
      }
      if (!decode_string(p, end, &h.value)) return false;
      out->push_back(std::move(h));
      header_seen = true;
    }
  }
  return true;
}

}  // namespace hpack
}  // namespace amdgpu_dp
