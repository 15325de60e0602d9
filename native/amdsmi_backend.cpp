// Real MI355X backend over libamd_smi (ROCm 7.2).
//
// Replaces: NVML device queries (reference device/device.go:37-181), NVML MIG
// enumeration (device/device_map.go:78-98, resource/resources.go:22-51), the
// sysfs NUMA lookup (device/device.go:69-93) and go-gpuallocator's NVLink graph
// (plugin/plugin.go:259-264).  Every call that talks to one GPU runs on that GPU's lane
// (lanes.h, backend.cpp: one owner thread per physical GPU, waited for with a bound), so
// a call wedged in the driver stalls that GPU only; the library session is guarded by a
// gate that a re-initialisation closes (SURVEY.md §7.5 hard part 6).
#include <amd_smi/amdsmi.h>
#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <atomic>
#include <cmath>
#include <ctime>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "backend.h"
#include "drm_reset.h"

namespace amdgpu_dp {

namespace {

std::mutex g_init_mu;
int g_init_refs = 0;
// amdsmi_available(keep=true) keeps its session open as one reference, which the next
// backend adopts: amdsmi_init costs ~25 ms on MI355X, and start-up probes and then opens.
// Probe-only callers pass keep=false, or drop an unadopted session with
// amdsmi_release_probe(), so no process holds a session that nothing owns.
bool g_probe_ref = false;

// A sysfs attribute of the GPU's PCI device kept open: pread at offset 0 runs the
// attribute's show() again without the path walk and open/close of a fresh read (4.1 us
// -> 0.5 us for mem_info_vram_used on MI355X, scripts/sysfs_cost_probe.py).
struct SysfsAttr {
  int fd = -1;
  explicit SysfsAttr(const std::string& path) : fd(::open(path.c_str(), O_RDONLY | O_CLOEXEC)) {}
  ~SysfsAttr() {
    if (fd >= 0) ::close(fd);
  }
  SysfsAttr(const SysfsAttr&) = delete;
  SysfsAttr& operator=(const SysfsAttr&) = delete;
  // bytes read into buf (NUL-terminated), -1 on error (a removed device: ENODEV)
  ssize_t read(char* buf, size_t cap) const {
    if (fd < 0 || cap == 0) return -1;
    ssize_t r;
    do {
      r = ::pread(fd, buf, cap - 1, 0);
    } while (r < 0 && errno == EINTR);
    if (r >= 0) buf[r] = 0;
    return r;
  }
};

std::string pci_sysfs_dir(const std::string& bdf) {
  std::string b = bdf;
  for (auto& c : b) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return "/sys/bus/pci/devices/" + b;
}

std::string status_str(amdsmi_status_t st) {
  const char* s = nullptr;
  if (amdsmi_status_code_to_string(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
  return "amdsmi status " + std::to_string(static_cast<int>(st));
}

void check(amdsmi_status_t st, const char* what) {
  if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error(std::string(what) + ": " + status_str(st));
}

std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(b.domain_number),
                static_cast<unsigned>(b.bus_number), static_cast<unsigned>(b.device_number),
                static_cast<unsigned>(b.function_number));
  return buf;
}

uint64_t bdf_key(const amdsmi_bdf_t& b) {  // physical device key (function masked)
  return (static_cast<uint64_t>(b.domain_number) << 16) | (static_cast<uint64_t>(b.bus_number) << 8) |
         (static_cast<uint64_t>(b.device_number) << 3);
}

// target_graphics_version: KFD encoding major*10000 + minor*100 + stepping (90500 ->
// gfx950); older amdsmi returned the hex gfx id (0x950).
std::string gfx_name(uint64_t v) {
  if (v == 0 || v == ~0ull) return "";
  char buf[32];
  if (v >= 10000) {
    const unsigned major = static_cast<unsigned>(v / 10000), minor = static_cast<unsigned>((v / 100) % 100),
                   step = static_cast<unsigned>(v % 100);
    std::snprintf(buf, sizeof(buf), "gfx%u%x%x", major, minor, step);
  } else {
    std::snprintf(buf, sizeof(buf), "gfx%llx", static_cast<unsigned long long>(v));
  }
  return buf;
}

int sysfs_numa(const std::string& bdf) {
  std::ifstream f("/sys/bus/pci/devices/" + bdf + "/numa_node");
  int n = -1;
  if (f >> n) return n;
  return -1;
}

bool valid16(uint16_t v) { return v != 0xFFFF; }
bool valid64(uint64_t v) { return v != ~0ull; }

struct Proc {
  amdsmi_processor_handle h;
  amdsmi_bdf_t bdf;
  uint32_t partition_id;
};

const char* profile_type_name(amdsmi_accelerator_partition_type_t t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_PARTITION_SPX: return "SPX";
    case AMDSMI_ACCELERATOR_PARTITION_DPX: return "DPX";
    case AMDSMI_ACCELERATOR_PARTITION_TPX: return "TPX";
    case AMDSMI_ACCELERATOR_PARTITION_QPX: return "QPX";
    case AMDSMI_ACCELERATOR_PARTITION_CPX: return "CPX";
    default: return "";
  }
}

// Fallback only: processors a compute-partition mode implies on CDNA3/4 (8 XCDs on
// MI355X), used when the driver reports no accelerator partition profile; 0 = unknown.
int partitions_of_mode(const std::string& mode) {
  if (mode == "SPX") return 1;
  if (mode == "DPX") return 2;
  if (mode == "TPX") return 3;
  if (mode == "QPX") return 4;
  if (mode == "CPX") return 8;
  return 0;
}

}  // namespace

bool amdsmi_available(bool keep) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_init_refs > 0) return true;
  if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return false;
  uint32_t n = 0;
  const bool ok = amdsmi_get_socket_handles(&n, nullptr) == AMDSMI_STATUS_SUCCESS && n > 0;
  if (!ok || !keep) {
    amdsmi_shut_down();
    return ok;
  }
  g_init_refs = 1;  // held for the backend that follows
  g_probe_ref = true;
  return true;
}

void amdsmi_release_probe() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (!g_probe_ref) return;
  g_probe_ref = false;
  if (--g_init_refs == 0) amdsmi_shut_down();
}

bool amdsmi_probe_held() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  return g_probe_ref;
}

// Enters the library session for a call made off the lanes (enumeration, event wait,
// disarm); leaves it on scope exit.
class GateGuard {
 public:
  explicit GateGuard(SessionGate& g) : g_(g) { g_.enter(0); }
  ~GateGuard() { g_.leave(); }

 private:
  SessionGate& g_;
};

class AmdSmiBackend : public Backend {
 public:
  AmdSmiBackend() {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (g_probe_ref) {
      g_probe_ref = false;  // adopt the probe's session and its reference
      return;
    }
    if (g_init_refs == 0) check(amdsmi_init(AMDSMI_INIT_AMD_GPUS), "amdsmi_init");
    ++g_init_refs;
  }
  ~AmdSmiBackend() override { shutdown(); }

  std::string name() const override { return "amdsmi"; }

  void shutdown() override {
    {
      std::lock_guard<std::mutex> lk(life_mu_);
      if (closed_.exchange(true)) return;
    }
    evt_live_.store(false);
    // amdsmi_shut_down only with no call inside the library: a call stuck in a wedged
    // driver keeps the session (and its reference) for the rest of the process.
    if (!gate().close(1000)) return;
    {
      std::lock_guard<std::mutex> ek(evt_mu_);
      disarm_locked();
    }
    {
      std::lock_guard<std::mutex> ilk(g_init_mu);
      if (--g_init_refs == 0) amdsmi_shut_down();
    }
    gate().reopen();  // later calls see another session and leave at once
  }

  bool reinit() override {
    if (closed_.load() || !gate().close(call_timeout_ms())) return false;
    bool ok = false;
    try {
      ok = reopen_session();
    } catch (...) {
      gate().reopen();
      throw;
    }
    gate().reopen();
    return ok;
  }

  int reinit_count() const override { return reinits_.load(); }

  std::vector<CallCost> sample_costs() const override {
    std::vector<CallCost> out;
    for (int c = 0; c < kCallCount; ++c) out.push_back({kCallNames[c], cost_ns_[c].load() * 1e-9, cost_n_[c].load()});
    // how many link samples took the full amdsmi path vs the gpu_metrics blob (counts only)
    out.push_back({"xgmi_links_full_path", 0.0, link_full_.load()});
    out.push_back({"xgmi_links_blob_path", 0.0, link_fast_.load()});
    // partitions whose busy figure came from the partition API vs the socket blob
    out.push_back({"partition_busy_from_partition_api", 0.0, part_from_api_.load()});
    out.push_back({"partition_busy_from_socket_blob", 0.0, part_from_blob_.load()});
    // ECC totals asked of amdsmi vs reused (no RAS counter file changed / the RAS event
    // state did not move); VRAM from sysfs vs amdsmi
    out.push_back({"ecc_count_reads_library", 0.0, ecc_library_.load()});
    out.push_back({"ecc_count_reads_unchanged", 0.0, ecc_unchanged_.load()});
    out.push_back({"ecc_count_reads_event_gated", 0.0, ecc_gated_.load()});
    out.push_back({"vram_reads_sysfs", 0.0, vram_sysfs_.load()});
    out.push_back({"vram_reads_library", 0.0, vram_library_.load()});
    out.push_back({"vram_reads_sysfs_disagreed", 0.0, vram_mismatch_.load()});
    return out;
  }

  void arm_events() override {
    arm_wanted_.store(true);
    arm_on_lanes(inventory());
  }

  int armed_event_sources() const override { return armed_count_.load(); }

  // The blocking wait enters the session first, then takes evt_mu_: disarming (which
  // takes the same lock) waits for an in-flight wait to return instead of stopping
  // notification underneath it, and a re-initialisation (gate closed) never waits on it.
  bool delivers_events() const override { return evt_live_.load() && !closed_.load(); }
  // armed (a privileged or CDI-patched pod): one wake-up a second while nothing happens;
  // stop() waits for at most that long
  int event_wait_ms() const override { return 1000; }

  int wait_events(int timeout_ms, std::vector<HwEvent>* out) override {
    amdsmi_evt_notification_data_t data[16];
    uint32_t num = 16;
    amdsmi_status_t st = AMDSMI_STATUS_NOT_INIT;
    bool waited = false;
    if (evt_live_.load() && !closed_.load()) {
      GateGuard g(gate());
      std::lock_guard<std::mutex> ek(evt_mu_);
      if (evt_live_.load()) {
        st = amdsmi_get_gpu_event_notification(timeout_ms, &num, data);
        waited = true;
      }
    }
    if (!waited) {
      // nothing armed (e.g. unprivileged container): the health monitor polls instead
      struct timespec ts{timeout_ms / 1000, (timeout_ms % 1000) * 1000000L};
      nanosleep(&ts, nullptr);
      return 0;
    }
    if (st != AMDSMI_STATUS_SUCCESS) return 0;
    auto inv = inventory();
    int added = 0;
    for (uint32_t i = 0; i < num; ++i) {
      HwEvent e;
      e.ts_ns = now_ns();
      e.message = data[i].message;
      switch (data[i].event) {
        case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: e.kind = kEvtPreReset; break;
        case AMDSMI_EVT_NOTIF_GPU_POST_RESET: e.kind = kEvtPostReset; break;
        case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: e.kind = kEvtThermal; break;
        case AMDSMI_EVT_NOTIF_VMFAULT: e.kind = kEvtVmFault; break;
        default: continue;
      }
      locate(*inv, data[i].processor_handle, &e.gpu, &e.partition);
      e.key = inv->key_of(e.gpu);
      out->push_back(e);
      ++added;
    }
    return added;
  }

 protected:
  // Sockets -> processors -> physical GPUs (BDF order).  Nothing here waits on a device:
  // the processor list, BDFs and KFD partition ids come from amdsmi's enumeration at
  // init and from KFD topology; the UUID is read once per BDF and remembered.
  void enumerate(std::vector<DeviceRef>* refs) override {
    if (closed_.load()) throw std::runtime_error("amdsmi backend is shut down");
    GateGuard g(gate());
    uint32_t nsock = 0;
    check(amdsmi_get_socket_handles(&nsock, nullptr), "amdsmi_get_socket_handles(count)");
    std::vector<amdsmi_socket_handle> socks(nsock);
    check(amdsmi_get_socket_handles(&nsock, socks.data()), "amdsmi_get_socket_handles");
    std::map<uint64_t, std::vector<Proc>> groups;  // ordered by BDF -> deterministic indices
    for (uint32_t s = 0; s < nsock; ++s) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      check(amdsmi_get_processor_handles(socks[s], &np, ph.data()), "amdsmi_get_processor_handles");
      for (uint32_t i = 0; i < np; ++i) {
        processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
        if (amdsmi_get_processor_type(ph[i], &t) != AMDSMI_STATUS_SUCCESS || t != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
        Proc p{ph[i], {}, 0};
        check(amdsmi_get_gpu_device_bdf(ph[i], &p.bdf), "amdsmi_get_gpu_device_bdf");
        amdsmi_kfd_info_t kfd{};
        p.partition_id = (amdsmi_get_gpu_kfd_info(ph[i], &kfd) == AMDSMI_STATUS_SUCCESS &&
                          kfd.current_partition_id != 0xFFFFFFFFu)
                             ? kfd.current_partition_id
                             : static_cast<uint32_t>(p.bdf.function_number);
        groups[bdf_key(p.bdf)].push_back(p);
      }
    }
    std::lock_guard<std::mutex> lk(uuid_mu_);
    for (auto& kv : groups) {
      auto& plist = kv.second;
      std::stable_sort(plist.begin(), plist.end(),
                       [](const Proc& a, const Proc& b) { return a.partition_id < b.partition_id; });
      DeviceRef r;
      amdsmi_bdf_t b0 = plist.front().bdf;
      b0.function_number = 0;
      r.bdf = bdf_str(b0);
      r.order = kv.first;
      for (const auto& p : plist) r.handles.push_back(p.h);
      auto it = uuid_of_bdf_.find(kv.first);
      if (it == uuid_of_bdf_.end()) it = uuid_of_bdf_.emplace(kv.first, uuid_of(plist.front().h)).first;
      r.key = it->second.empty() ? r.bdf : it->second;
      refs->push_back(std::move(r));
    }
  }

  // Everything discovery reads from one GPU, on its lane: identity, partition model,
  // per-partition render/KFD nodes, and this GPU's view of its links.
  void describe(const DeviceRef& ref, const std::vector<DeviceRef>& all, GpuInfo* out,
                std::vector<Link>* row) override {
    GpuInfo& g = *out;
    amdsmi_processor_handle h0 = ref.handles.front();
    g.bdf = ref.bdf;
    g.uuid = ref.key == ref.bdf ? uuid_of(h0) : ref.key;
    amdsmi_asic_info_t asic{};
    if (amdsmi_get_gpu_asic_info(h0, &asic) == AMDSMI_STATUS_SUCCESS) {
      g.market_name = asic.market_name;
      g.serial = asic.asic_serial;
      g.gfx_target = gfx_name(asic.target_graphics_version);
      if (asic.num_of_compute_units != 0xFFFFFFFFu) g.num_compute_units = static_cast<int>(asic.num_of_compute_units);
      g.device_id = static_cast<uint32_t>(asic.device_id & 0xFFFF);
      if (asic.oam_id != 0xFFFFFFFFu && asic.oam_id != 0xFFFFu) g.oam_id = static_cast<int>(asic.oam_id);
    }
    amdsmi_driver_info_t drv{};
    if (amdsmi_get_gpu_driver_info(h0, &drv) == AMDSMI_STATUS_SUCCESS) g.driver_version = normalize_driver_version(drv.driver_version);
    amdsmi_vbios_info_t vb{};
    if (amdsmi_get_gpu_vbios_info(h0, &vb) == AMDSMI_STATUS_SUCCESS) g.vbios_version = vb.version;
    if (g.market_name.empty()) g.market_name = "AMD Instinct";
    amdsmi_vram_info_t vram{};
    if (amdsmi_get_gpu_vram_info(h0, &vram) == AMDSMI_STATUS_SUCCESS)
      g.vram_total_bytes = static_cast<uint64_t>(vram.vram_size) << 20;
    char buf[64] = {0};
    if (amdsmi_get_gpu_compute_partition(h0, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) g.compute_partition = buf;
    std::memset(buf, 0, sizeof(buf));
    if (amdsmi_get_gpu_memory_partition(h0, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) g.memory_partition = buf;
    amdsmi_memory_partition_config_t mcfg{};
    if (amdsmi_get_gpu_memory_partition_config(h0, &mcfg) == AMDSMI_STATUS_SUCCESS)
      g.nps_caps = mcfg.partition_caps.nps_cap_mask & 0xF;
    // The driver's own profile of the current mode: partition count and NPS caps come
    // from it rather than from a table keyed by the mode string.
    amdsmi_accelerator_partition_profile_t prof;
    std::memset(&prof, 0, sizeof(prof));
    uint32_t part_ids[AMDSMI_MAX_ACCELERATOR_PARTITIONS] = {};
    if (amdsmi_get_gpu_accelerator_partition_profile(h0, &prof, part_ids) == AMDSMI_STATUS_SUCCESS &&
        prof.num_partitions > 0 && prof.num_partitions <= AMDSMI_MAX_ACCELERATOR_PARTITIONS &&
        profile_type_name(prof.profile_type)[0] != '\0') {
      g.partition_profile = profile_type_name(prof.profile_type);
      g.profile_partitions = static_cast<int>(prof.num_partitions);
      g.profile_index = static_cast<int>(prof.profile_index);
      if (g.compute_partition.empty()) g.compute_partition = g.partition_profile;
      if (g.nps_caps == 0) g.nps_caps = prof.memory_caps.nps_cap_mask & 0xF;
    }
    // Every profile the GPU supports (the reference's mixed strategy asks NVML for every
    // MIG profile, resource/resources.go:43-51 VisitMigProfiles).
    // The list needs root (AMDSMI_STATUS_NO_PERM as an ordinary user on the MI355X box,
    // profiles/r4/amdsmi_probe.json); then only the current profile is known supported.
    auto cfg = std::make_unique<amdsmi_accelerator_partition_profile_config_t>();
    std::memset(cfg.get(), 0, sizeof(*cfg));
    const amdsmi_status_t cst = amdsmi_get_gpu_accelerator_partition_profile_config(h0, cfg.get());
    g.profiles_status = cst == AMDSMI_STATUS_SUCCESS ? "ok" : status_str(cst);
    if (cst == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t i = 0; i < cfg->num_profiles && i < AMDSMI_MAX_ACCELERATOR_PROFILE; ++i) {
        const auto& p = cfg->profiles[i];
        if (profile_type_name(p.profile_type)[0] == '\0' || p.num_partitions == 0) continue;
        PartitionProfile pp;
        pp.type = profile_type_name(p.profile_type);
        pp.partitions = static_cast<int>(p.num_partitions);
        pp.nps_caps = p.memory_caps.nps_cap_mask & 0xF;
        pp.index = static_cast<int>(p.profile_index);
        g.supported_profiles.push_back(pp);
      }
    }
    if (g.supported_profiles.empty() && !g.partition_profile.empty()) {
      PartitionProfile pp;
      pp.type = g.partition_profile;
      pp.partitions = g.profile_partitions;
      pp.nps_caps = g.nps_caps;
      pp.index = g.profile_index;
      pp.source = "current";
      g.supported_profiles.push_back(pp);
    }
    if (g.compute_partition.empty()) g.compute_partition = ref.handles.size() == 1 ? "SPX" : "UNKNOWN";
    if (g.memory_partition.empty()) g.memory_partition = "NPS1";
    uint32_t thr = 0;  // needs root; -1 when not readable
    if (amdsmi_get_gpu_bad_page_threshold(h0, &thr) == AMDSMI_STATUS_SUCCESS) g.bad_page_threshold = static_cast<int>(thr);
    int32_t numa = -1;
    if (amdsmi_get_gpu_topo_numa_affinity(h0, &numa) != AMDSMI_STATUS_SUCCESS || numa < 0) numa = sysfs_numa(g.bdf);
    g.numa_node = numa;
    for (size_t k = 0; k < ref.handles.size(); ++k) {
      amdsmi_processor_handle h = ref.handles[k];
      PartitionInfo part;
      part.index = static_cast<int>(k);
      part.uuid = uuid_of(h);
      part.id = ref.handles.size() == 1 ? g.uuid : g.uuid + "-xcp" + std::to_string(k);
      amdsmi_enumeration_info_t en{};
      if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
        part.render_minor = static_cast<int>(en.drm_render);
        part.card_minor = static_cast<int>(en.drm_card);
        part.hip_id = static_cast<int>(en.hip_id);
        part.hsa_id = static_cast<int>(en.hsa_id);
      }
      amdsmi_kfd_info_t kfd{};
      if (amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS && kfd.node_id != 0xFFFFFFFFu)
        part.kfd_node = kfd.node_id;
      part.numa_node = g.numa_node;
      amdsmi_vram_usage_t vu{};
      if (amdsmi_get_gpu_vram_usage(h, &vu) == AMDSMI_STATUS_SUCCESS)
        part.vram_bytes = static_cast<uint64_t>(vu.vram_total) << 20;
      if (part.vram_bytes == 0) part.vram_bytes = g.vram_total_bytes / ref.handles.size();
      g.partitions.push_back(part);
    }
    // This GPU's view of its links: class, hops and weight per peer, then xGMI health and
    // trained bandwidth from the link metrics (which name each link's peer by BDF).
    row->assign(all.size(), Link{});
    for (size_t p = 0; p < all.size(); ++p) {
      if (all[p].order == ref.order || all[p].handles.empty()) continue;
      Link& l = (*row)[p];
      amdsmi_processor_handle hp = all[p].handles.front();
      uint64_t hops = 0;
      amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
      if (amdsmi_topo_get_link_type(h0, hp, &hops, &t) == AMDSMI_STATUS_SUCCESS) {
        l.type = static_cast<int>(t);
        l.hops = static_cast<int>(hops);
      }
      uint64_t w = 0;
      if (amdsmi_topo_get_link_weight(h0, hp, &w) == AMDSMI_STATUS_SUCCESS) l.weight = w;
      amdsmi_link_type_t pt;
      amdsmi_p2p_capability_t cap{};
      if (amdsmi_topo_get_p2p_status(h0, hp, &pt, &cap) == AMDSMI_STATUS_SUCCESS) l.p2p = true;
    }
    auto ds = dev(ref.key);
    ds->links = LinkCache{};  // indexes may have moved: take the full path and re-verify
    GpuSample s;
    amdsmi_gpu_metrics_t gm;
    std::memset(&gm, 0, sizeof(gm));
    if (amdsmi_get_gpu_metrics_info(h0, &gm) == AMDSMI_STATUS_SUCCESS && valid16(gm.xgmi_link_width) &&
        gm.xgmi_link_width != 0)
      s.xgmi_link_width = gm.xgmi_link_width;
    link_state(*ds, h0, all, &s, nullptr);
    g.num_xgmi_links = s.num_links;
    for (int k = 0; k < s.num_links; ++k) {
      const int p = s.link_peer[k];  // position in `all` here
      if (p < 0) continue;
      if (s.link_up[k] == 0) (*row)[p].up = false;
      if (s.link_trained_gbps[k] > 0) (*row)[p].bw_gbps = s.link_trained_gbps[k];
    }
  }

  bool sample_device(const Inventory& inv, int gpu, GpuSample* s) override {
    if (closed_.load()) return false;
    const DeviceRef& ref = inv.refs[gpu];
    amdsmi_processor_handle h0 = ref.handles.front();
    auto ds = dev(ref.key);
    s->ts_ns = now_ns();
    amdsmi_gpu_metrics_t m;
    std::memset(&m, 0, sizeof(m));
    int64_t t = mono_ns();
    const amdsmi_status_t mst = amdsmi_get_gpu_metrics_info(h0, &m);
    t = charge(kCallGpuMetrics, t);  // the blob's parsing below is not charged to any call
    const int nparts = static_cast<int>(ref.handles.size());
    if (mst == AMDSMI_STATUS_SUCCESS) {
      s->ok = true;
      if (valid16(m.current_socket_power) && m.current_socket_power != 0) s->power_w = m.current_socket_power;
      else if (valid16(m.average_socket_power)) s->power_w = m.average_socket_power;
      if (valid64(m.energy_accumulator)) s->energy_j = m.energy_accumulator * 15.259e-6;  // 15.259 uJ / count
      if (valid16(m.temperature_edge) && m.temperature_edge != 0) s->temp_edge_c = m.temperature_edge;
      if (valid16(m.temperature_hotspot)) s->temp_hotspot_c = m.temperature_hotspot;
      if (valid16(m.temperature_mem)) s->temp_mem_c = m.temperature_mem;
      s->num_hbm = 0;
      for (int i = 0; i < AMDSMI_NUM_HBM_INSTANCES && i < kMaxHbm; ++i)
        if (valid16(m.temperature_hbm[i]) && m.temperature_hbm[i] != 0) s->temp_hbm_c[s->num_hbm++] = m.temperature_hbm[i];
      if (valid16(m.average_gfx_activity)) s->gfx_activity_pct = m.average_gfx_activity;
      if (valid16(m.average_umc_activity)) s->umc_activity_pct = m.average_umc_activity;
      if (valid16(m.current_gfxclks[0]) && m.current_gfxclks[0] != 0) s->gfxclk_mhz = m.current_gfxclks[0];
      else if (valid16(m.average_gfxclk_frequency)) s->gfxclk_mhz = m.average_gfxclk_frequency;
      if (valid16(m.current_uclk)) s->uclk_mhz = m.current_uclk;
      if (m.throttle_status != 0xFFFFFFFFu) s->throttle_status = m.throttle_status;
      if (valid16(m.xgmi_link_width)) s->xgmi_link_width = m.xgmi_link_width;
      if (valid16(m.xgmi_link_speed)) s->xgmi_link_speed = m.xgmi_link_speed;
      if (valid16(m.pcie_link_width) && m.pcie_link_width != 0) s->pcie_link_width = m.pcie_link_width;
      if (valid16(m.pcie_link_speed) && m.pcie_link_speed != 0) s->pcie_link_speed_gtps = m.pcie_link_speed * 0.1;
      if (valid64(m.pcie_replay_count_acc)) s->pcie_replays = static_cast<double>(m.pcie_replay_count_acc);
      if (valid64(m.pcie_l0_to_recov_count_acc)) s->pcie_recoveries = static_cast<double>(m.pcie_l0_to_recov_count_acc);
      if (valid64(m.firmware_timestamp) && m.firmware_timestamp != 0) s->fw_clock_s = m.firmware_timestamp * 1e-8;
    }
    if (reset_query()) {  // the kernel's reset count, through the GPU's first render node
      const auto& parts = inv.gpus[gpu].partitions;
      const int minor = parts.empty() ? -1 : parts.front().render_minor;
      if (minor > 0) {
        const std::string path = "/dev/dri/renderD" + std::to_string(minor);
        if (!ds->reset_watch || ds->reset_watch->path() != path) ds->reset_watch = std::make_unique<DrmResetWatch>(path);
        s->reset_count = ds->reset_watch->poll();
      }
    } else if (ds->reset_watch) {
      ds->reset_watch.reset();
    }
    s->num_partitions = std::min(nparts, kMaxPartitions);
    partition_busy(*ds, ref, mst == AMDSMI_STATUS_SUCCESS ? &m : nullptr, s);
    t = charge(kCallPartitionMetrics, t);
    double used = 0, total = 0;
    bool have_vram = false;
    const bool shared_pool = inv.gpus[gpu].memory_partition == "NPS1";
    if (shared_pool && vram_direct(*ds, inv.gpus[gpu].bdf, h0, &used, &total)) {
      have_vram = true;
      s->partition_vram_used_bytes[0] = used;
    }
    for (size_t p = 0; p < ref.handles.size() && !have_vram; ++p) {
      amdsmi_vram_usage_t vu{};
      if (amdsmi_get_gpu_vram_usage(ref.handles[p], &vu) == AMDSMI_STATUS_SUCCESS) {
        have_vram = true;
        used += static_cast<double>(vu.vram_used) * 1048576.0;
        total += static_cast<double>(vu.vram_total) * 1048576.0;
        if (static_cast<int>(p) < kMaxPartitions) s->partition_vram_used_bytes[p] = static_cast<double>(vu.vram_used) * 1048576.0;
        vram_library_.fetch_add(1, std::memory_order_relaxed);
        if (shared_pool) break;  // partitions share one VRAM pool in NPS1; do not double count
      }
    }
    if (have_vram) {
      s->vram_used_bytes = used;
      s->vram_total_bytes = total;
      s->ok = true;
    }
    t = charge(kCallVram, t);
    ecc_totals(*ds, inv.gpus[gpu].bdf, h0, s);
    amdsmi_xgmi_status_t xs = AMDSMI_XGMI_STATUS_NO_ERRORS;
    if (amdsmi_gpu_xgmi_error_status(h0, &xs) == AMDSMI_STATUS_SUCCESS) s->xgmi_error_status = static_cast<int>(xs);
    t = charge(kCallEcc, t);
    link_state(*ds, h0, inv.refs, s, mst == AMDSMI_STATUS_SUCCESS ? &m : nullptr);
    t = charge(kCallLinks, t);
    bad_pages(*ds, h0, s);
    charge(kCallBadPages, t);
    return s->ok;
  }

  bool handles_stale(const std::vector<GpuInfo>& described) override {
    // amdsmi enumerates processors once, at amdsmi_init.  After an operator switches a
    // GPU's compute partition mode (amd-smi set --compute-partition), the cached handle
    // list no longer matches the mode the GPU reports: re-initialise and enumerate again.
    for (const auto& g : described) {
      const int want = g.profile_partitions > 0 ? g.profile_partitions : partitions_of_mode(g.compute_partition);
      if (want > 0 && want != static_cast<int>(g.partitions.size())) return true;
    }
    return false;
  }

  // amdsmi is process-global: only the sole owner may shut it down and start it again.
  // Runs with the session gate closed (no call inside the library).
  bool reopen_session() override {
    std::lock_guard<std::mutex> ilk(g_init_mu);
    if (g_init_refs != 1 || closed_.load()) return false;
    {
      std::lock_guard<std::mutex> ek(evt_mu_);
      disarm_locked();
    }
    amdsmi_shut_down();
    check(amdsmi_init(AMDSMI_INIT_AMD_GPUS), "amdsmi_init (re-init)");
    reinits_.fetch_add(1);
    {
      std::lock_guard<std::mutex> lk(devs_mu_);
      devs_.clear();  // caches of the old handles
    }
    return true;
  }

  // Keeps event delivery armed across re-discovery; re-arms only when the processor set
  // changed (handles from a re-init are new objects).
  void installed(const std::shared_ptr<const Inventory>& inv) override {
    if (!arm_wanted_.load()) return;
    std::vector<void*> flat;
    for (const auto& r : inv->refs) flat.insert(flat.end(), r.handles.begin(), r.handles.end());
    {
      std::lock_guard<std::mutex> ek(arm_mu_);
      if (flat == armed_for_) return;
    }
    {
      GateGuard g(gate());
      std::lock_guard<std::mutex> ek(evt_mu_);
      disarm_locked();
    }
    arm_on_lanes(inv);
  }

 private:
  static std::string key_of(const GpuInfo& g) { return g.uuid.empty() ? g.bdf : g.uuid; }

  std::string uuid_of(amdsmi_processor_handle h) {
    char ubuf[AMDSMI_MAX_STRING_LENGTH] = {0};
    unsigned int ulen = sizeof(ubuf);
    if (amdsmi_get_gpu_device_uuid(h, &ulen, ubuf) == AMDSMI_STATUS_SUCCESS && ubuf[0]) return ubuf;
    amdsmi_bdf_t b{};
    amdsmi_get_gpu_device_bdf(h, &b);
    return "amdgpu-" + bdf_str(b);
  }

  static void locate(const Inventory& inv, amdsmi_processor_handle h, int* gpu, int* part) {
    for (size_t g = 0; g < inv.refs.size(); ++g)
      for (size_t p = 0; p < inv.refs[g].handles.size(); ++p)
        if (inv.refs[g].handles[p] == h) {
          *gpu = static_cast<int>(g);
          *part = inv.refs[g].handles.size() == 1 ? -1 : static_cast<int>(p);
          return;
        }
  }

  // Arms event notification on every processor, each on its GPU's lane.  Every handle a
  // job arms is recorded in armed_handles_ by the job itself, under arm_mu_:
  // one that finishes after the wait below still gets disarmed.  armed_for_ lists only
  // the processors whose job ran (armed, or refused by the driver - an unprivileged pod):
  // a GPU whose lane was wedged, or whose job missed the deadline, is armed again at the
  // next discovery instead of never.
  void arm_on_lanes(const std::shared_ptr<const Inventory>& inv) {
    if (closed_.load()) return;
    const uint64_t mask = AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_PRE_RESET) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_POST_RESET) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_THERMAL_THROTTLE) |
                          AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_VMFAULT);
    std::vector<std::shared_ptr<LaneJob>> jobs;
    std::vector<std::vector<void*>> handles;
    const uint64_t batch = next_batch();  // posted to every lane at once
    const uint64_t epoch = arm_epoch_.fetch_add(1) + 1;
    for (const auto& r : inv->refs) {
      const std::vector<void*> hs = r.handles;
      handles.push_back(hs);
      jobs.push_back(post_job(r.key, "arm", inv->session, [this, hs, mask, epoch] {
        for (auto h : hs) {
          if (amdsmi_init_gpu_event_notification(h) != AMDSMI_STATUS_SUCCESS) continue;
          if (amdsmi_set_gpu_event_notification_mask(h, mask) != AMDSMI_STATUS_SUCCESS) {
            amdsmi_stop_gpu_event_notification(h);
            continue;
          }
          std::lock_guard<std::mutex> ak(arm_mu_);
          armed_handles_.push_back(h);
          armed_count_.store(static_cast<int>(armed_handles_.size()));
          evt_live_.store(true);
          if (arm_epoch_.load() != epoch) break;  // disarmed / re-armed meanwhile: stop here
        }
      }, batch));
    }
    const int64_t deadline = mono_ns() + static_cast<int64_t>(call_timeout_ms()) * 1000000;
    std::vector<void*> ran;
    for (size_t g = 0; g < jobs.size(); ++g) {
      if (!jobs[g] || !jobs[g]->wait(std::max<int64_t>(0, (deadline - mono_ns()) / 1000000)) || jobs[g]->dropped())
        continue;
      ran.insert(ran.end(), handles[g].begin(), handles[g].end());
    }
    std::lock_guard<std::mutex> ek(arm_mu_);
    armed_for_ = ran;
  }

  // evt_mu_ held, inside the session (or with the gate closed)
  void disarm_locked() {
    std::lock_guard<std::mutex> ak(arm_mu_);
    arm_epoch_.fetch_add(1);  // an arm job still running stops after its current handle
    evt_live_.store(false);
    for (auto h : armed_handles_) amdsmi_stop_gpu_event_notification(h);
    armed_handles_.clear();
    armed_for_.clear();
    armed_count_.store(0);
  }

  // ---- per-GPU state, touched only on the GPU's lane ----
  // Peer lookup for every xGMI link of every sample: peers are cached by BDF order key at
  // discovery (7 links x 8 GPUs per tick would otherwise re-query amdsmi 8 times per link).
  // amdsmi_get_link_metrics resolves every link's peer BDF and costs ~0.9-1.3 ms per GPU
  // on MI355X (test_amdsmi_sample_cost_breakdown), while the per-link byte counters and
  // up/down status it reports are also in the gpu_metrics blob sample() has just read.  So
  // the full call (plus amdsmi_get_gpu_xgmi_link_status) runs at discovery and every
  // kLinkRefreshNs, and cross-checks the blob index for index: counters within a small
  // skew of the blob's and, separately, blob status equal to the link-status call.
  // Between refreshes a verified GPU takes counters (and, if verified, status) from the
  // blob and peers / rates from the cache; an unverified one takes the full path.
  // (60 s: with the sampler's 5 s idle period a shorter one made every other idle sample
  // take the ~1 ms full path)
  static constexpr int64_t kLinkRefreshNs = 60'000'000'000;
  struct LinkCache {
    int64_t read_ns = 0;
    bool counters_ok = false;  // blob counters line up with link_metrics
    bool status_ok = false;    // blob status lines up with the link-status call
    int n = 0;
    int k[kMaxXgmiLinks] = {};            // metrics index of reported link i
    uint64_t peer[kMaxXgmiLinks] = {};    // peer's BDF order key (0 = unknown)
    double bitrate[kMaxXgmiLinks] = {}, maxbw[kMaxXgmiLinks] = {};
  };
  // RAS retired-page records change only when the driver retires a page: re-read them
  // every kBadPageRefreshNs and report the cached counts in between.
  static constexpr int64_t kBadPageRefreshNs = 60'000'000'000LL;
  struct BadPages {
    int64_t read_ns = 0;
    int64_t reserved = -1, pending = -1, unreservable = -1;
  };
  // ECC totals (the health monitor's UE latch reads them).  amdsmi's total re-reads every
  // RAS block's counter file, and the feature mask once per block: ~0.6 ms per GPU on
  // MI355X, of which the kernel's own work is ~0.27 ms (the ras/aca_* reads query the
  // firmware's error banks: 19-87 us each, scripts/sysfs_cost_probe.py).  The reported
  // counts are always amdsmi's; what decides when to ask it again:
  //  * eccEventGate (default) and ras/event_state present: that file (0.7 us) carries the
  //    driver's RAS event sequence - fatal errors, poison creation and consumption, which
  //    is how an uncorrectable error surfaces on MI300/MI350 - so amdsmi is asked when it
  //    moved, and every kEccRefreshNs regardless (correctable counts, which raise no
  //    event, are at most that old);
  //  * otherwise the block files are kept open and read each sample, and amdsmi is asked
  //    when any of them changed (and every kEccRefreshNs).
  static constexpr int64_t kEccRefreshNs = 30'000'000'000LL;
  struct EccWatch {
    bool opened = false;
    std::vector<std::unique_ptr<SysfsAttr>> files;  // ras/aca_* (MI355X) or ras/*_err_count
    std::unique_ptr<SysfsAttr> events;              // ras/event_state
    std::string seen, scratch;  // the files' contents at amdsmi's last read / this sample's
    std::string events_seen;    // event_state at amdsmi's last read
    int64_t read_ns = 0;
    bool have = false;
    int64_t ce = 0, ue = 0;
  };
  // VRAM usage of a GPU with one memory pool (NPS1): the kernel's mem_info_vram_used /
  // mem_info_vram_total, the counters amdsmi's usage call reports in MiB (~85 us per call
  // there, 0.5 us per pread here).  Checked against amdsmi on first use and every
  // kVramVerifyNs; a disagreement switches the GPU back to amdsmi for good.
  static constexpr int64_t kVramVerifyNs = 60'000'000'000LL;
  struct VramDirect {
    int state = 0;  // 0 untried, 1 agrees with amdsmi, -1 amdsmi only
    std::unique_ptr<SysfsAttr> used, total;
    int64_t verified_ns = 0;
  };
  struct DevState {
    LinkCache links;
    BadPages pages;
    EccWatch ecc;
    VramDirect vram;
    std::unique_ptr<DrmResetWatch> reset_watch;  // the render node's amdgpu context (health.resetQuery)
    int partition_api = 0;  // amdsmi_get_gpu_partition_metrics_info: 0 untried, 1 answers, -1 not supported
  };
  std::shared_ptr<DevState> dev(const std::string& key) {
    std::lock_guard<std::mutex> lk(devs_mu_);
    auto& d = devs_[key];
    if (!d) d = std::make_shared<DevState>();
    return d;
  }

  static int position_of(const std::vector<DeviceRef>& refs, uint64_t order) {
    for (size_t i = 0; i < refs.size(); ++i)
      if (refs[i].order == order) return static_cast<int>(i);
    return -1;
  }

  void ecc_totals(DevState& ds, const std::string& bdf, amdsmi_processor_handle h, GpuSample* s) {
    EccWatch& ew = ds.ecc;
    if (!ew.opened) {
      ew.opened = true;
      const std::string ras = pci_sysfs_dir(bdf) + "/ras";
      std::vector<std::string> names;
      if (DIR* d = opendir(ras.c_str())) {
        while (const dirent* e = readdir(d)) {
          const std::string n = e->d_name;
          if (n.rfind("aca_", 0) == 0 || (n.size() > 10 && n.compare(n.size() - 10, 10, "_err_count") == 0))
            names.push_back(n);
        }
        closedir(d);
      }
      std::sort(names.begin(), names.end());
      for (const auto& n : names) {
        auto a = std::make_unique<SysfsAttr>(ras + "/" + n);
        if (a->fd >= 0) ew.files.push_back(std::move(a));
      }
      auto ev = std::make_unique<SysfsAttr>(ras + "/event_state");
      if (ev->fd >= 0) ew.events = std::move(ev);
    }
    const int64_t now = mono_ns();
    char buf[512];
    bool look = !ew.have || now - ew.read_ns >= kEccRefreshNs;
    std::string events_now;
    bool gated = false;
    if (ecc_event_gate() && ew.events) {
      const ssize_t r = ew.events->read(buf, sizeof(buf));
      if (r >= 0) {
        gated = true;
        events_now.assign(buf, static_cast<size_t>(r));
        look = look || events_now != ew.events_seen;
      }
    }
    bool direct = false;
    std::string& cur = ew.scratch;
    cur.clear();
    if (!gated) {  // the block files themselves (also read when looking: the next baseline)
      direct = !ew.files.empty();
      for (const auto& f : ew.files) {
        const ssize_t r = f->read(buf, sizeof(buf));
        if (r < 0) {
          direct = false;
          break;
        }
        cur.append(buf, static_cast<size_t>(r));
        cur.push_back('\x1f');
      }
      look = look || !direct || cur != ew.seen;
    }
    if (look) {
      amdsmi_error_count_t ec{};
      ew.have = amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS;
      if (ew.have) {
        ew.ce = static_cast<int64_t>(ec.correctable_count);
        ew.ue = static_cast<int64_t>(ec.uncorrectable_count);
      }
      ew.seen = direct ? cur : std::string();
      ew.events_seen = gated ? events_now : std::string();
      ew.read_ns = now;
      ecc_library_.fetch_add(1, std::memory_order_relaxed);
    } else {
      (gated ? ecc_gated_ : ecc_unchanged_).fetch_add(1, std::memory_order_relaxed);
    }
    if (ew.have) {
      s->ecc_correctable = ew.ce;
      s->ecc_uncorrectable = ew.ue;
    }
  }

  // bytes used / total of a one-pool GPU from sysfs; false: use amdsmi
  bool vram_direct(DevState& ds, const std::string& bdf, amdsmi_processor_handle h, double* used, double* total) {
    VramDirect& v = ds.vram;
    if (v.state < 0) return false;
    if (!v.used) {
      const std::string dir = pci_sysfs_dir(bdf);
      v.used = std::make_unique<SysfsAttr>(dir + "/mem_info_vram_used");
      v.total = std::make_unique<SysfsAttr>(dir + "/mem_info_vram_total");
    }
    char b1[64], b2[64];
    if (v.used->read(b1, sizeof(b1)) <= 0 || v.total->read(b2, sizeof(b2)) <= 0) {
      v.state = -1;
      return false;
    }
    char* e1 = nullptr;
    char* e2 = nullptr;
    const double u = std::strtod(b1, &e1), t = std::strtod(b2, &e2);
    if (e1 == b1 || e2 == b2 || t <= 0) {
      v.state = -1;
      return false;
    }
    const int64_t now = mono_ns();
    if (v.state == 0 || now - v.verified_ns >= kVramVerifyNs) {
      amdsmi_vram_usage_t vu{};
      if (amdsmi_get_gpu_vram_usage(h, &vu) != AMDSMI_STATUS_SUCCESS) {
        v.state = -1;
        return false;
      }
      const double mib = 1048576.0, lt = static_cast<double>(vu.vram_total) * mib,
                   lu = static_cast<double>(vu.vram_used) * mib;
      // totals agree to the MiB amdsmi rounds to; usage within what moves between two reads
      if (std::fabs(lt - t) > 2 * mib || std::fabs(lu - u) > std::max(256 * mib, 0.05 * lt)) {
        v.state = -1;
        vram_mismatch_.fetch_add(1, std::memory_order_relaxed);
        return false;
      }
      v.state = 1;
      v.verified_ns = now;
    }
    *used = u;
    *total = t;
    vram_sysfs_.fetch_add(1, std::memory_order_relaxed);
    return true;
  }

  void bad_pages(DevState& ds, amdsmi_processor_handle h, GpuSample* s) {
    BadPages& bp = ds.pages;
    const int64_t now = mono_ns();
    if (bp.read_ns == 0 || now - bp.read_ns >= kBadPageRefreshNs) {
      bp.read_ns = now;
      bp.reserved = bp.pending = bp.unreservable = -1;
      uint32_t n = 0;
      if (amdsmi_get_gpu_bad_page_info(h, &n, nullptr) == AMDSMI_STATUS_SUCCESS) {
        bp.reserved = bp.pending = bp.unreservable = 0;
        if (n > 0) {
          std::vector<amdsmi_retired_page_record_t> rec(n);
          if (amdsmi_get_gpu_bad_page_info(h, &n, rec.data()) == AMDSMI_STATUS_SUCCESS) {
            for (uint32_t i = 0; i < n && i < rec.size(); ++i) {
              if (rec[i].status == AMDSMI_MEM_PAGE_STATUS_PENDING) ++bp.pending;
              else if (rec[i].status == AMDSMI_MEM_PAGE_STATUS_UNRESERVABLE) ++bp.unreservable;
              else ++bp.reserved;
            }
          } else {
            bp.reserved = n;  // count known, statuses not
          }
        }
      }
    }
    s->retired_pages = bp.reserved;
    s->pending_pages = bp.pending;
    s->unreservable_pages = bp.unreservable;
  }

  // Per-partition compute busy.  Preferred source: the partition's own metrics
  // (amdsmi_get_gpu_partition_metrics_info on the partition's processor);
  // fallback: the socket blob's xcp_stats[p] (assumes partition order == XCP order).
  void partition_busy(DevState& ds, const DeviceRef& ref, const amdsmi_gpu_metrics_t* blob, GpuSample* s) {
    auto mean = [](const amdsmi_gpu_xcp_metrics_t& x) {
      double sum = 0;
      int cnt = 0;
      for (int i = 0; i < AMDSMI_MAX_NUM_XCC; ++i)  // uint32 fields: all-ones = not reported
        if (x.gfx_busy_inst[i] != 0xFFFFFFFFu && x.gfx_busy_inst[i] <= 100) {
          sum += x.gfx_busy_inst[i];
          ++cnt;
        }
      return cnt ? sum / cnt : -1.0;
    };
    for (int p = 0; p < s->num_partitions; ++p) {
      double v = -1;
      if (ds.partition_api >= 0) {
        auto pm = std::make_unique<amdsmi_gpu_metrics_t>();
        std::memset(pm.get(), 0, sizeof(*pm));
        const amdsmi_status_t st = amdsmi_get_gpu_partition_metrics_info(ref.handles[p], pm.get());
        if (st == AMDSMI_STATUS_SUCCESS) {
          // a partition's table carries its own XCP's stats; take the slot with data
          // (slot p when it carries the whole socket's)
          int with_data = 0, first = -1;
          for (int x = 0; x < AMDSMI_MAX_NUM_XCP; ++x)
            if (mean(pm->xcp_stats[x]) >= 0) {
              ++with_data;
              if (first < 0) first = x;
            }
          if (first >= 0) v = mean(pm->xcp_stats[with_data > 1 && p < AMDSMI_MAX_NUM_XCP ? p : first]);
          if (v >= 0) ds.partition_api = 1;
        } else if (st == AMDSMI_STATUS_NOT_SUPPORTED || st == AMDSMI_STATUS_NOT_YET_IMPLEMENTED) {
          ds.partition_api = -1;
        }
      }
      if (v >= 0) {
        s->partition_busy_source[p] = 1;
        part_from_api_.fetch_add(1, std::memory_order_relaxed);
      } else if (blob && p < AMDSMI_MAX_NUM_XCP) {
        v = mean(blob->xcp_stats[p]);
        if (v < 0 && s->num_partitions == 1) v = s->gfx_activity_pct;
        if (v >= 0) {
          s->partition_busy_source[p] = 2;
          part_from_blob_.fetch_add(1, std::memory_order_relaxed);
        }
      }
      s->partition_gfx_busy_pct[p] = v;
    }
  }

  static int blob_up(uint16_t v) { return v == 1 ? 1 : (v == 0 ? 0 : -1); }

  // Fills per-link peer/up/read/write/rate; peers are positions in `refs`.
  void link_state(DevState& ds, amdsmi_processor_handle h0, const std::vector<DeviceRef>& refs, GpuSample* s,
                  const amdsmi_gpu_metrics_t* m) {
    LinkCache& lc = ds.links;
    const int64_t now = mono_ns();
    s->num_links = 0;
    if (m && lc.counters_ok && lc.read_ns != 0 && now - lc.read_ns < kLinkRefreshNs) {
      link_fast_.fetch_add(1, std::memory_order_relaxed);
      amdsmi_xgmi_link_status_t ls;
      bool have_status = false;
      if (!lc.status_ok) {
        std::memset(&ls, 0, sizeof(ls));
        have_status = amdsmi_get_gpu_xgmi_link_status(h0, &ls) == AMDSMI_STATUS_SUCCESS;
      }
      s->num_links = lc.n;
      for (int i = 0; i < lc.n; ++i) {
        const int k = lc.k[i];
        s->link_peer[i] = lc.peer[i] ? position_of(refs, lc.peer[i]) : -1;
        s->link_read_kb[i] = static_cast<double>(m->xgmi_read_data_acc[k]);
        s->link_write_kb[i] = static_cast<double>(m->xgmi_write_data_acc[k]);
        s->link_bitrate_gbps[i] = lc.bitrate[i];
        s->link_max_gbps[i] = lc.maxbw[i];
        if (lc.status_ok)
          s->link_up[i] = blob_up(m->xgmi_link_status[k]);
        else if (have_status && static_cast<uint32_t>(k) < ls.total_links)
          s->link_up[i] = ls.status[k] == AMDSMI_XGMI_LINK_UP ? 1 : (ls.status[k] == AMDSMI_XGMI_LINK_DOWN ? 0 : -1);
        else
          s->link_up[i] = -1;
      }
      fill_trained(s);
      return;
    }
    link_full_.fetch_add(1, std::memory_order_relaxed);
    lc.read_ns = now;
    lc.counters_ok = lc.status_ok = false;
    lc.n = 0;
    amdsmi_link_metrics_t lm;
    std::memset(&lm, 0, sizeof(lm));
    if (amdsmi_get_link_metrics(h0, &lm) != AMDSMI_STATUS_SUCCESS) return;
    amdsmi_xgmi_link_status_t ls;
    std::memset(&ls, 0, sizeof(ls));
    const bool have_status = amdsmi_get_gpu_xgmi_link_status(h0, &ls) == AMDSMI_STATUS_SUCCESS;
    const uint32_t nl = std::min<uint32_t>(lm.num_links, std::min<uint32_t>(kMaxXgmiLinks, AMDSMI_MAX_NUM_XGMI_LINKS));
    bool counters_ok = m != nullptr, status_ok = m != nullptr && have_status;
    for (uint32_t k = 0; k < nl; ++k) {
      if (lm.links[k].link_type != AMDSMI_LINK_TYPE_XGMI) continue;
      const int i = s->num_links++;
      const uint64_t peer = bdf_key(lm.links[k].bdf);
      s->link_peer[i] = position_of(refs, peer);
      s->link_read_kb[i] = static_cast<double>(lm.links[k].read);
      s->link_write_kb[i] = static_cast<double>(lm.links[k].write);
      s->link_bitrate_gbps[i] = lm.links[k].bit_rate != 0xFFFFFFFFu ? lm.links[k].bit_rate : 0;
      s->link_max_gbps[i] = lm.links[k].max_bandwidth != 0xFFFFFFFFu ? lm.links[k].max_bandwidth : 0;
      if (have_status && k < ls.total_links)
        s->link_up[i] = ls.status[k] == AMDSMI_XGMI_LINK_UP ? 1 : (ls.status[k] == AMDSMI_XGMI_LINK_DOWN ? 0 : -1);
      else
        s->link_up[i] = -1;
      lc.k[i] = static_cast<int>(k);
      lc.peer[i] = s->link_peer[i] >= 0 ? peer : 0;
      lc.bitrate[i] = s->link_bitrate_gbps[i];
      lc.maxbw[i] = s->link_max_gbps[i];
      if (m) {
        // link_metrics is read after the blob: its counters may only be ahead, by at
        // most what a link moves in a few ms (allow 5% or 1 GiB)
        auto close = [](uint64_t later, uint64_t blob) {
          if (!valid64(blob) || later < blob) return false;
          const uint64_t d = later - blob;
          return d <= (1ull << 20) || d <= later / 20;
        };
        counters_ok = counters_ok && close(lm.links[k].read, m->xgmi_read_data_acc[k]) &&
                      close(lm.links[k].write, m->xgmi_write_data_acc[k]);
        status_ok = status_ok && blob_up(m->xgmi_link_status[k]) == s->link_up[i];
      }
    }
    lc.n = s->num_links;
    lc.counters_ok = counters_ok && lc.n > 0;
    lc.status_ok = lc.counters_ok && status_ok;
    fill_trained(s);
  }

  // Trained bandwidth of each link: its current per-lane rate (link metrics bit_rate)
  // times the GPU's current link width (gpu_metrics; set by the caller when known).
  // max_bandwidth is the capability and stays 608 Gb/s on a link that trained narrower.
  static void fill_trained(GpuSample* s) {
    for (int i = 0; i < s->num_links; ++i)
      s->link_trained_gbps[i] = (s->link_bitrate_gbps[i] > 0 && s->xgmi_link_width > 0)
                                    ? s->link_bitrate_gbps[i] * s->xgmi_link_width
                                    : s->link_max_gbps[i];
  }

  // per-call cost accounting for sample_device()
  enum SampleCall { kCallGpuMetrics, kCallPartitionMetrics, kCallVram, kCallEcc, kCallLinks, kCallBadPages, kCallCount };
  static constexpr const char* kCallNames[kCallCount] = {"gpu_metrics", "partition_metrics", "vram_usage",
                                                         "ecc_count", "xgmi_links", "bad_pages"};
  int64_t charge(int call, int64_t since) {
    const int64_t now = mono_ns();
    cost_ns_[call].fetch_add(now - since, std::memory_order_relaxed);
    cost_n_[call].fetch_add(1, std::memory_order_relaxed);
    return now;
  }
  std::atomic<int64_t> cost_ns_[kCallCount] = {};
  std::atomic<uint64_t> cost_n_[kCallCount] = {};
  std::atomic<uint64_t> link_fast_{0}, link_full_{0}, part_from_api_{0}, part_from_blob_{0};
  std::atomic<uint64_t> ecc_library_{0}, ecc_unchanged_{0}, ecc_gated_{0}, vram_sysfs_{0}, vram_library_{0}, vram_mismatch_{0};

  std::mutex life_mu_;
  std::atomic<bool> closed_{false};
  std::mutex devs_mu_;  // the map only; a DevState's contents belong to its GPU's lane
  std::map<std::string, std::shared_ptr<DevState>> devs_;
  std::mutex uuid_mu_;
  std::map<uint64_t, std::string> uuid_of_bdf_;  // BDF order key -> UUID (read once)
  std::mutex evt_mu_;                   // held across the blocking event wait
  std::mutex arm_mu_;                   // armed_handles_ / armed_for_
  std::atomic<bool> evt_live_{false};   // armed with at least one source
  std::atomic<bool> arm_wanted_{false};
  std::atomic<int> armed_count_{0};
  std::vector<amdsmi_processor_handle> armed_handles_;
  std::vector<void*> armed_for_;        // processors whose arm job ran (see arm_on_lanes)
  std::atomic<uint64_t> arm_epoch_{0};  // bumped by every arming and disarming
  std::atomic<int> reinits_{0};
};

std::shared_ptr<Backend> make_amdsmi_backend() { return std::make_shared<AmdSmiBackend>(); }

}  // namespace amdgpu_dp
