// Shared helpers for the libFuzzer targets in this directory.
//
// The targets feed untrusted bytes into every parser that faces a peer: the kubelet
// protobuf decoders (pbwire.h), the HPACK decoder, the HTTP/2 gRPC server on its unix
// socket, and the HTTP/1.1 ops server.  The reference (Go, grpc-go/echo) never fuzzed
// anything; here the parsers are hand-written C++, so they are fuzzed
// under ASan+UBSan.
//
// Seeds: with FUZZ_WRITE_SEEDS=<dir> set, LLVMFuzzerInitialize writes well-formed
// inputs built with the same encoders the production code uses into <dir> and exits.
#pragma once

#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "device_table.h"
#include "hpack.h"
#include "pbwire.h"

namespace fuzzutil {

using namespace amdgpu_dp;

// A CPX-style node: `ngpu` GPUs x `nparts` partitions, full xGMI mesh with one link
// down, two NUMA nodes, plus every device advertised with `replicas` "::k" replicas
// when replicas > 0 (exercises the distributed policy).
inline std::shared_ptr<DeviceTable> make_table(int ngpu, int nparts, int replicas = 0, bool pre_start = false) {
  std::vector<TableDevice> devs;
  for (int g = 0; g < ngpu; ++g)
    for (int p = 0; p < nparts; ++p) {
      const std::string base = "gpu" + std::to_string(g) + (nparts > 1 ? "-xcp" + std::to_string(p) : "");
      const int nrep = replicas > 0 ? replicas : 1;
      for (int r = 0; r < nrep; ++r) {
        TableDevice d;
        d.id = replicas > 0 ? base + "::" + std::to_string(r) : base;
        d.gpu = g;
        d.partition = nparts > 1 ? p : -1;
        d.numa = g / 4;
        d.replica = replicas > 0 ? r : -1;
        d.host_paths = {"/dev/dri/renderD" + std::to_string(128 + g * nparts + p)};
        devs.push_back(d);
      }
    }
  Topology topo;
  topo.resize(ngpu);
  for (int a = 0; a < ngpu; ++a)
    for (int b = 0; b < ngpu; ++b)
      if (a != b) {
        Link& l = topo.at(a, b);
        l.type = kLinkXgmi;
        l.hops = 1;
        l.weight = 15;
        l.p2p = true;
        l.up = !((a == 0 && b == 5) || (a == 5 && b == 0));
      }
  TableConfig cfg;
  cfg.reject_unhealthy = true;
  cfg.pre_start_required = pre_start;
  return std::make_shared<DeviceTable>(cfg, devs, topo);
}

inline std::string alloc_req(const std::vector<std::vector<std::string>>& containers) {
  std::string r;
  for (auto& ids : containers) {
    std::string c;
    for (auto& id : ids) pb::put_bytes(&c, 1, id);
    pb::put_bytes(&r, 1, c);
  }
  return r;
}

inline std::string preferred_req(const std::vector<std::string>& avail, const std::vector<std::string>& must,
                                 int size) {
  std::string c, r;
  for (auto& id : avail) pb::put_bytes(&c, 1, id);
  for (auto& id : must) pb::put_bytes(&c, 2, id);
  pb::put_int_nz(&c, 3, size);
  pb::put_bytes(&r, 1, c);
  return r;
}

// ---- HTTP/2 framing for seeds ----
inline void h2_frame(std::string* o, uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload) {
  const uint32_t len = static_cast<uint32_t>(payload.size());
  o->push_back(static_cast<char>(len >> 16));
  o->push_back(static_cast<char>(len >> 8));
  o->push_back(static_cast<char>(len));
  o->push_back(static_cast<char>(type));
  o->push_back(static_cast<char>(flags));
  o->push_back(static_cast<char>((sid >> 24) & 0x7f));
  o->push_back(static_cast<char>(sid >> 16));
  o->push_back(static_cast<char>(sid >> 8));
  o->push_back(static_cast<char>(sid));
  o->append(payload);
}

inline std::string grpc_headers(const std::string& path, bool huffman) {
  std::string b;
  hpack::encode_indexed(&b, 3);  // :method POST
  hpack::encode_indexed(&b, 6);  // :scheme http
  hpack::encode_literal_name_index(&b, 4, path, huffman);        // :path
  hpack::encode_literal_name_index(&b, 1, "localhost", huffman); // :authority
  hpack::encode_literal_name_index(&b, 31, "application/grpc", huffman);
  hpack::encode_literal(&b, "te", "trailers", huffman);
  return b;
}

inline std::string grpc_body(const std::string& msg) {
  std::string o(1, '\0');
  const uint32_t n = static_cast<uint32_t>(msg.size());
  o.push_back(static_cast<char>(n >> 24));
  o.push_back(static_cast<char>(n >> 16));
  o.push_back(static_cast<char>(n >> 8));
  o.push_back(static_cast<char>(n));
  o.append(msg);
  return o;
}

// HEADERS (END_HEADERS) + DATA (END_STREAM) for one unary call on stream `sid`.
inline std::string h2_call(uint32_t sid, const std::string& path, const std::string& msg, bool huffman = false) {
  std::string o;
  h2_frame(&o, 0x1, 0x4, sid, grpc_headers(path, huffman));
  h2_frame(&o, 0x0, 0x1, sid, grpc_body(msg));
  return o;
}

// ---- sockets ----
// libFuzzer's -timeout watchdog is a 1 s SIGALRM, so every blocking call here can see
// EINTR; an interrupted connect() keeps connecting in the background.
inline bool connect_retry(int fd, const sockaddr* addr, socklen_t len) {
  if (connect(fd, addr, len) == 0) return true;
  if (errno != EINTR && errno != EINPROGRESS) return false;
  for (;;) {
    struct pollfd p {fd, POLLOUT, 0};
    const int r = poll(&p, 1, 5000);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    int err = 0;
    socklen_t el = sizeof(err);
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el);
    return err == 0;
  }
}

// Reads until the peer closes.  false = nothing arrived for 5 s (the server is stuck).
inline bool drain_until_close(int fd, std::string* into) {
  char buf[65536];
  for (;;) {
    struct pollfd p {fd, POLLIN, 0};
    const int r = poll(&p, 1, 5000);
    if (r < 0 && errno == EINTR) continue;
    if (r == 0) return false;
    const ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return true;
    if (into) into->append(buf, static_cast<size_t>(n));
  }
}

// ---- seed corpus ----
inline const char* seed_dir() { return std::getenv("FUZZ_WRITE_SEEDS"); }

inline void write_seed(const char* dir, const std::string& name, const std::string& bytes) {
  mkdir(dir, 0755);
  const std::string path = std::string(dir) + "/" + name;
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return;
  std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
}

}  // namespace fuzzutil
