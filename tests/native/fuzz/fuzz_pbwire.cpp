// libFuzzer target: kubelet request decoding + Allocate / GetPreferredAllocation on the
// DeviceTable (pbwire.h, device_table.cpp, allocator.cpp).
//
// Input byte 0 picks the table (8 whole GPUs, 8x8 CPX partitions, replicated GPUs for
// the distributed policy) and the RPC; the rest is the request message.  Beyond "no
// crash / no UB", every successful GetPreferredAllocation answer must satisfy the
// allocator contract (reference go-gpuallocator contract):
// distinct ids, every must_include id present, every id from available or must_include,
// and exactly allocation_size ids.
#include <cstdint>
#include <cstdlib>
#include <set>

#include "fuzz_common.h"

using namespace amdgpu_dp;

namespace {

std::shared_ptr<DeviceTable> g_tables[3];

void check_contract(const DeviceTable& t, std::string_view input) {
  std::vector<pb::PreferredRequest> reqs;
  try {
    reqs = pb::decode_preferred_request(input);
  } catch (const pb::DecodeError&) {
    return;
  }
  std::vector<std::string> avail, must, ids;
  for (const auto& r : reqs) {
    avail.assign(r.available.begin(), r.available.end());
    must.assign(r.must_include.begin(), r.must_include.end());
    AllocResult ar = t.preferred_ids(avail, must, r.size, &ids);
    if (!ar.ok) continue;
    if (r.size <= 0) {
      if (!ids.empty()) std::abort();  // non-positive size must yield no devices
      continue;
    }
    std::set<std::string> seen(ids.begin(), ids.end());
    if (seen.size() != ids.size()) std::abort();  // duplicate id in the answer
    const std::set<std::string> a(avail.begin(), avail.end()), m(must.begin(), must.end());
    for (const auto& id : m)
      if (!seen.count(id)) std::abort();  // must_include dropped
    for (const auto& id : ids)
      if (!a.count(id) && !m.count(id)) std::abort();  // invented an id
    if (static_cast<int64_t>(ids.size()) != r.size) std::abort();
  }
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  g_tables[0] = fuzzutil::make_table(8, 1);
  g_tables[1] = fuzzutil::make_table(8, 8);
  // the CPX table carries the round-3 link terms: a half-rate link and links that other
  // multi-GPU pods already span
  g_tables[1]->set_link_bandwidth(0, 1, 304.0);
  g_tables[1]->set_link_bandwidth(2, 5, 456.0);
  std::vector<int> pods(64, 0);
  pods[0 * 8 + 2] = pods[2 * 8 + 0] = 1;
  pods[4 * 8 + 6] = pods[6 * 8 + 4] = 3;
  g_tables[1]->set_link_pods(pods);
  g_tables[2] = fuzzutil::make_table(4, 1, 4);
  if (const char* dir = fuzzutil::seed_dir()) {
    using fuzzutil::alloc_req;
    using fuzzutil::preferred_req;
    fuzzutil::write_seed(dir, "alloc_gpu", std::string(1, '\x00') + alloc_req({{"gpu3"}}));
    fuzzutil::write_seed(dir, "alloc_two_containers", std::string(1, '\x02') + alloc_req({{"gpu0-xcp1", "gpu0-xcp2"}, {"gpu7-xcp7"}}));
    fuzzutil::write_seed(dir, "alloc_unknown", std::string(1, '\x00') + alloc_req({{"nope"}}));
    fuzzutil::write_seed(dir, "pref_pair", std::string(1, '\x01') +
                                               preferred_req({"gpu0", "gpu1", "gpu4", "gpu5", "gpu6"}, {"gpu0"}, 2));
    fuzzutil::write_seed(dir, "pref_quad_cpx",
                         std::string(1, '\x03') + preferred_req({"gpu1-xcp0", "gpu1-xcp1", "gpu2-xcp0", "gpu2-xcp3",
                                                                 "gpu3-xcp5", "gpu6-xcp6"},
                                                                {}, 4));
    fuzzutil::write_seed(dir, "pref_replicas",
                         std::string(1, '\x05') + preferred_req({"gpu0::0", "gpu0::1", "gpu1::0", "gpu2::3"}, {}, 2));
    std::exit(0);
  }
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  const DeviceTable& t = *g_tables[(data[0] % 6) / 2 % 3];
  const std::string_view msg(reinterpret_cast<const char*>(data + 1), size - 1);
  std::string out;
  if (data[0] & 1) {
    (void)t.preferred(msg, &out);
    check_contract(t, msg);
  } else {
    (void)t.allocate(msg, &out);
  }
  return 0;
}
