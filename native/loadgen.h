// Load generators for the BASELINE.md measurement protocol.
//
//   http_load : N keep-alive HTTP/1.1 connections issuing GET <path>; closed-loop (max
//               rate) or open-loop at a fixed target rate, where latency is measured from
//               each request's *scheduled* send time (no coordinated omission).
//   grpc_load : N native HTTP/2 clients issuing unary calls, closed-loop.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace amdgpu_dp {

struct LoadResult {
  uint64_t ok = 0;
  uint64_t errors = 0;
  uint64_t bytes = 0;
  double elapsed_s = 0;
  std::vector<double> latencies_s;  // one per completed request
};

LoadResult http_load(const std::string& host, int port, const std::string& path, int conns, double duration_s,
                     double target_rps, bool accept_gzip = false);

LoadResult grpc_load(const std::string& socket_path, const std::string& method, const std::string& req, int conns,
                     double duration_s);

}  // namespace amdgpu_dp
