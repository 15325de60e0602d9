// Minimal protobuf wire codec for the kubelet v1beta1 hot messages.
//
// The reference builds fresh Go protobuf structs on every RPC (plugin/plugin.go:
// 173-225).  Here Allocate / ListAndWatch / GetPreferredAllocation responses are
// assembled from pre-encoded per-device fragments, so the per-call work is a
// decode + a few memcpy.  Field numbers: SURVEY.md Appendix A (golden-tested in
// tests/test_v1beta1_wire.py against the runtime-descriptor messages).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace amdgpu_dp {
namespace pb {

struct DecodeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void put_varint(std::string* out, uint64_t v) {
  char buf[10];
  int n = 0;
  while (v >= 0x80) {
    buf[n++] = static_cast<char>((v & 0x7F) | 0x80);
    v >>= 7;
  }
  buf[n++] = static_cast<char>(v);
  out->append(buf, n);
}

inline void put_tag(std::string* out, uint32_t field, uint32_t wire) { put_varint(out, (field << 3) | wire); }

inline void put_bytes(std::string* out, uint32_t field, std::string_view s) {
  put_tag(out, field, 2);
  put_varint(out, s.size());
  out->append(s.data(), s.size());
}

// proto3: empty strings / zero scalars are not emitted
inline void put_string_nz(std::string* out, uint32_t field, std::string_view s) {
  if (!s.empty()) put_bytes(out, field, s);
}

inline void put_int_nz(std::string* out, uint32_t field, int64_t v) {
  if (v == 0) return;
  put_tag(out, field, 0);
  put_varint(out, static_cast<uint64_t>(v));
}

inline void put_bool_nz(std::string* out, uint32_t field, bool v) {
  if (!v) return;
  put_tag(out, field, 0);
  put_varint(out, 1);
}

class Reader {
 public:
  Reader(const char* p, size_t n) : p_(p), end_(p + n) {}
  explicit Reader(std::string_view s) : Reader(s.data(), s.size()) {}
  bool done() const { return p_ >= end_; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p_ >= end_) throw DecodeError("truncated varint");
      const uint8_t b = static_cast<uint8_t>(*p_++);
      v |= static_cast<uint64_t>(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
    }
    throw DecodeError("varint too long");
  }
  // Reads next tag; returns false at end.
  bool next(uint32_t* field, uint32_t* wire) {
    if (p_ >= end_) return false;
    const uint64_t t = varint();
    *field = static_cast<uint32_t>(t >> 3);
    *wire = static_cast<uint32_t>(t & 7);
    if (*field == 0) throw DecodeError("field number 0");
    return true;
  }
  std::string_view bytes() {
    const uint64_t n = varint();
    if (n > static_cast<uint64_t>(end_ - p_)) throw DecodeError("truncated length-delimited field");
    std::string_view s(p_, n);
    p_ += n;
    return s;
  }
  void skip(uint32_t wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: advance(8); break;
      case 2: bytes(); break;
      case 5: advance(4); break;
      default: throw DecodeError("unsupported wire type");
    }
  }

 private:
  void advance(size_t n) {
    if (n > static_cast<size_t>(end_ - p_)) throw DecodeError("truncated fixed field");
    p_ += n;
  }
  const char* p_;
  const char* end_;
};

// AllocateRequest{ repeated ContainerAllocateRequest{ repeated string devices_ids = 1 } = 1 }
// also PreStartContainerRequest{ repeated string devices_ids = 1 } via decode_string_list
inline std::vector<std::vector<std::string_view>> decode_allocate_request(std::string_view buf) {
  std::vector<std::vector<std::string_view>> out;
  Reader r(buf);
  uint32_t f, w;
  while (r.next(&f, &w)) {
    if (f == 1 && w == 2) {
      Reader c(r.bytes());
      out.emplace_back();
      uint32_t cf, cw;
      while (c.next(&cf, &cw)) {
        if (cf == 1 && cw == 2) out.back().push_back(c.bytes());
        else c.skip(cw);
      }
    } else {
      r.skip(w);
    }
  }
  return out;
}

struct PreferredRequest {
  std::vector<std::string_view> available;
  std::vector<std::string_view> must_include;
  int32_t size = 0;
};

// PreferredAllocationRequest{ repeated ContainerPreferredAllocationRequest = 1 }
inline std::vector<PreferredRequest> decode_preferred_request(std::string_view buf) {
  std::vector<PreferredRequest> out;
  Reader r(buf);
  uint32_t f, w;
  while (r.next(&f, &w)) {
    if (f == 1 && w == 2) {
      Reader c(r.bytes());
      out.emplace_back();
      uint32_t cf, cw;
      while (c.next(&cf, &cw)) {
        if (cf == 1 && cw == 2) out.back().available.push_back(c.bytes());
        else if (cf == 2 && cw == 2) out.back().must_include.push_back(c.bytes());
        else if (cf == 3 && cw == 0) out.back().size = static_cast<int32_t>(c.varint());
        else c.skip(cw);
      }
    } else {
      r.skip(w);
    }
  }
  return out;
}

}  // namespace pb
}  // namespace amdgpu_dp
