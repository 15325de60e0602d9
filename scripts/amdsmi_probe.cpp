// Read-only amdsmi probe for the MI355X box.
//
//  1. Partition model as the driver reports it: every accelerator partition profile the
//     GPU supports (amdsmi_get_gpu_accelerator_partition_profile_config), the current
//     one, and the memory-partition (NPS) caps and mode.
//  2. Per-partition telemetry through amdsmi_get_gpu_partition_metrics_info on every
//     processor handle, next to the socket blob's xcp_stats.
//  3. Does amdsmi serialise calls?  A background thread loops a slow device call
//     (amdsmi_get_link_metrics, ~1 ms) while the main thread times cheap calls: a call
//     that waits behind the slow one shows its median rise by a large fraction of the
//     slow call's duration.  Calls that touch no device (library version, processor
//     type, the BDF cached in the handle) waiting too would mean a library-wide lock.
//
// Build: g++ -O2 -std=c++17 -I/opt/rocm/include scripts/amdsmi_probe.cpp
//          -L/opt/rocm/lib -lamd_smi -Wl,-rpath,/opt/rocm/lib -pthread -o scripts/bin/amdsmi_probe
// Prints one JSON document.  Nothing is written to the device.
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* ptype(int t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_PARTITION_SPX: return "SPX";
    case AMDSMI_ACCELERATOR_PARTITION_DPX: return "DPX";
    case AMDSMI_ACCELERATOR_PARTITION_TPX: return "TPX";
    case AMDSMI_ACCELERATOR_PARTITION_QPX: return "QPX";
    case AMDSMI_ACCELERATOR_PARTITION_CPX: return "CPX";
    default: return "INVALID";
  }
}

const char* rtype(int t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_XCC: return "XCC";
    case AMDSMI_ACCELERATOR_ENCODER: return "ENCODER";
    case AMDSMI_ACCELERATOR_DECODER: return "DECODER";
    case AMDSMI_ACCELERATOR_DMA: return "DMA";
    case AMDSMI_ACCELERATOR_JPEG: return "JPEG";
    default: return "?";
  }
}

std::string nps_list(uint32_t mask) {
  std::string s = "[";
  const char* names[] = {"NPS1", "NPS2", "NPS4", "NPS8"};
  bool first = true;
  for (int b = 0; b < 4; ++b)
    if (mask & (1u << b)) {
      s += first ? "\"" : ",\"";
      s += names[b];
      s += "\"";
      first = false;
    }
  return s + "]";
}

struct Stats {
  double p50 = 0, p90 = 0, mean = 0;
  int n = 0;
};

Stats time_calls(const std::function<void()>& fn, int n) {
  std::vector<double> v;
  v.reserve(n);
  for (int i = 0; i < n; ++i) {
    const double t = now_us();
    fn();
    v.push_back(now_us() - t);
  }
  std::sort(v.begin(), v.end());
  Stats s;
  s.n = n;
  s.p50 = v[n / 2];
  s.p90 = v[(n * 9) / 10];
  double sum = 0;
  for (double x : v) sum += x;
  s.mean = sum / n;
  return s;
}

void print_stats(const char* name, const Stats& solo, const Stats& busy, bool last) {
  std::printf("      \"%s\": {\"solo_p50_us\": %.2f, \"solo_p90_us\": %.2f, \"busy_p50_us\": %.2f, "
              "\"busy_p90_us\": %.2f, \"n\": %d}%s\n",
              name, solo.p50, solo.p90, busy.p50, busy.p90, solo.n, last ? "" : ",");
}

}  // namespace

int main() {
  if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
    std::printf("{\"error\": \"amdsmi_init failed\"}\n");
    return 1;
  }
  uint32_t nsock = 0;
  amdsmi_get_socket_handles(&nsock, nullptr);
  std::vector<amdsmi_socket_handle> socks(nsock);
  amdsmi_get_socket_handles(&nsock, socks.data());
  std::vector<amdsmi_processor_handle> procs;
  for (auto s : socks) {
    uint32_t np = 0;
    if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    amdsmi_get_processor_handles(s, &np, ph.data());
    for (auto h : ph) {
      processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
      if (amdsmi_get_processor_type(h, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        procs.push_back(h);
    }
  }
  std::printf("{\n  \"sockets\": %u, \"processors\": %zu,\n", nsock, procs.size());
  if (procs.empty()) {
    std::printf("  \"error\": \"no GPU processors\"\n}\n");
    return 1;
  }
  amdsmi_processor_handle h0 = procs[0];

  // ---- 1. partition model ----
  amdsmi_accelerator_partition_profile_config_t cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  double t = now_us();
  amdsmi_status_t st = amdsmi_get_gpu_accelerator_partition_profile_config(h0, &cfg);
  std::printf("  \"profile_config\": {\"status\": %d, \"call_us\": %.1f", static_cast<int>(st), now_us() - t);
  if (st == AMDSMI_STATUS_SUCCESS) {
    std::printf(", \"num_profiles\": %u, \"default_profile_index\": %u, \"profiles\": [", cfg.num_profiles,
                cfg.default_profile_index);
    for (uint32_t i = 0; i < cfg.num_profiles && i < AMDSMI_MAX_ACCELERATOR_PROFILE; ++i) {
      const auto& p = cfg.profiles[i];
      std::printf("%s\n    {\"type\": \"%s\", \"num_partitions\": %u, \"memory_caps\": %s, \"profile_index\": %u, "
                  "\"num_resources\": %u}",
                  i ? "," : "", ptype(p.profile_type), p.num_partitions, nps_list(p.memory_caps.nps_cap_mask).c_str(),
                  p.profile_index, p.num_resources);
    }
    std::printf("], \"resource_profiles\": [");
    for (uint32_t i = 0; i < cfg.num_resource_profiles && i < AMDSMI_MAX_CP_PROFILE_RESOURCES; ++i) {
      const auto& r = cfg.resource_profiles[i];
      std::printf("%s\n    {\"profile_index\": %u, \"resource\": \"%s\", \"per_partition\": %u, \"shared_by\": %u}",
                  i ? "," : "", r.profile_index, rtype(r.resource_type), r.partition_resource,
                  r.num_partitions_share_resource);
    }
    std::printf("]");
  }
  std::printf("},\n");

  amdsmi_accelerator_partition_profile_t cur;
  std::memset(&cur, 0, sizeof(cur));
  uint32_t part_ids[AMDSMI_MAX_ACCELERATOR_PARTITIONS] = {};
  st = amdsmi_get_gpu_accelerator_partition_profile(h0, &cur, part_ids);
  std::printf("  \"current_profile\": {\"status\": %d, \"type\": \"%s\", \"num_partitions\": %u, \"memory_caps\": %s, "
              "\"profile_index\": %u},\n",
              static_cast<int>(st), ptype(cur.profile_type), cur.num_partitions,
              nps_list(cur.memory_caps.nps_cap_mask).c_str(), cur.profile_index);

  amdsmi_memory_partition_config_t mcfg;
  std::memset(&mcfg, 0, sizeof(mcfg));
  st = amdsmi_get_gpu_memory_partition_config(h0, &mcfg);
  std::printf("  \"memory_partition_config\": {\"status\": %d, \"caps\": %s, \"mode\": %d, \"num_numa_ranges\": %u},\n",
              static_cast<int>(st), nps_list(mcfg.partition_caps.nps_cap_mask).c_str(), static_cast<int>(mcfg.mp_mode),
              mcfg.num_numa_ranges);
  char buf[64] = {0};
  amdsmi_get_gpu_compute_partition(h0, buf, sizeof(buf));
  std::printf("  \"compute_partition\": \"%s\",", buf);
  std::memset(buf, 0, sizeof(buf));
  amdsmi_get_gpu_memory_partition(h0, buf, sizeof(buf));
  std::printf(" \"memory_partition\": \"%s\",\n", buf);

  // ---- 2. per-partition metrics ----
  amdsmi_gpu_metrics_t blob;
  std::memset(&blob, 0, sizeof(blob));
  st = amdsmi_get_gpu_metrics_info(h0, &blob);
  auto busy = [](const amdsmi_gpu_xcp_metrics_t& x, std::string* out) {
    int n = 0;
    double sum = 0;
    *out = "[";
    for (int i = 0; i < AMDSMI_MAX_NUM_XCC; ++i) {
      if (x.gfx_busy_inst[i] == 0xFFFF) continue;
      *out += (n ? "," : "") + std::to_string(x.gfx_busy_inst[i]);
      sum += x.gfx_busy_inst[i];
      ++n;
    }
    *out += "]";
    return n ? sum / n : -1.0;
  };
  std::printf("  \"socket_blob\": {\"status\": %d, \"format\": %u, \"content\": %u, \"num_partition\": %u, "
              "\"gfx_activity\": %u, \"xcp_busy\": [",
              static_cast<int>(st), blob.common_header.format_revision, blob.common_header.content_revision,
              blob.num_partition, blob.average_gfx_activity);
  for (int p = 0; p < AMDSMI_MAX_NUM_XCP; ++p) {
    std::string inst;
    const double m = busy(blob.xcp_stats[p], &inst);
    std::printf("%s{\"xcp\": %d, \"mean\": %.1f, \"inst\": %s}", p ? ", " : "", p, m, inst.c_str());
  }
  std::printf("]},\n  \"partition_metrics\": [");
  for (size_t i = 0; i < procs.size(); ++i) {
    amdsmi_gpu_metrics_t pm;
    std::memset(&pm, 0, sizeof(pm));
    t = now_us();
    st = amdsmi_get_gpu_partition_metrics_info(procs[i], &pm);
    const double us = now_us() - t;
    std::string inst;
    const double m = busy(pm.xcp_stats[0], &inst);
    std::printf("%s\n    {\"processor\": %zu, \"status\": %d, \"call_us\": %.1f, \"format\": %u, \"content\": %u, "
                "\"num_partition\": %u, \"xcp0_mean\": %.1f, \"xcp0_inst\": %s, \"gfx_activity\": %u, "
                "\"power\": %u, \"temp_hotspot\": %u}",
                i ? "," : "", i, static_cast<int>(st), us, pm.common_header.format_revision,
                pm.common_header.content_revision, pm.num_partition, m, inst.c_str(), pm.average_gfx_activity,
                pm.current_socket_power, pm.temperature_hotspot);
    amdsmi_vram_usage_t vu{};
    if (amdsmi_get_gpu_vram_usage(procs[i], &vu) == AMDSMI_STATUS_SUCCESS)
      std::printf(",\n    {\"processor\": %zu, \"vram_total_mb\": %u, \"vram_used_mb\": %u}", i, vu.vram_total,
                  vu.vram_used);
  }
  std::printf("],\n");

  // ---- 3. serialisation ----
  const int n = 2000;
  std::vector<std::pair<const char*, std::function<void()>>> calls = {
      {"lib_version", [] { amdsmi_version_t v; amdsmi_get_lib_version(&v); }},
      {"processor_type", [h0] { processor_type_t pt; amdsmi_get_processor_type(h0, &pt); }},
      {"device_bdf", [h0] { amdsmi_bdf_t b; amdsmi_get_gpu_device_bdf(h0, &b); }},
      {"vram_usage", [h0] { amdsmi_vram_usage_t v; amdsmi_get_gpu_vram_usage(h0, &v); }},
      {"total_ecc", [h0] { amdsmi_error_count_t e; amdsmi_get_gpu_total_ecc_count(h0, &e); }},
      {"gpu_metrics", [h0] { static amdsmi_gpu_metrics_t m; amdsmi_get_gpu_metrics_info(h0, &m); }},
  };
  std::vector<Stats> solo;
  for (auto& c : calls) solo.push_back(time_calls(c.second, c.first[0] == 'g' ? 300 : n));
  amdsmi_link_metrics_t lm;
  const Stats slow = time_calls([&] { amdsmi_get_link_metrics(h0, &lm); }, 200);
  std::atomic<bool> stop{false};
  std::atomic<long> slow_calls{0};
  std::thread bg([&] {
    amdsmi_link_metrics_t l2;
    while (!stop.load()) {
      amdsmi_get_link_metrics(h0, &l2);
      slow_calls.fetch_add(1);
    }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  std::vector<Stats> busy_s;
  for (auto& c : calls) busy_s.push_back(time_calls(c.second, c.first[0] == 'g' ? 300 : n));
  stop.store(true);
  bg.join();
  std::printf("  \"serialisation\": {\"background_call\": \"link_metrics\", \"background_p50_us\": %.1f, "
              "\"background_calls\": %ld, \"calls\": {\n",
              slow.p50, slow_calls.load());
  for (size_t i = 0; i < calls.size(); ++i) print_stats(calls[i].first, solo[i], busy_s[i], i + 1 == calls.size());
  std::printf("  }}\n}\n");
  amdsmi_shut_down();
  return 0;
}
