// Hardware backend interface of the MI355X device plugin.
//
// Replaces the reference's NVML + go-nvlib stack (reference: plugin/manager.go:44
// nvml.New(), device/device.go:37-181 per-device NVML queries, device/device_map.go:
// 48-98 VisitDevices/VisitMigDevices).  One physical MI355X (an amdsmi *socket*) owns
// 1..8 compute partitions (SPX..CPX, amdsmi *processors*); each partition is a KFD node
// with its own DRM render node, which is what a container needs mounted.
//
// Two implementations:
//   * AmdSmiBackend  (amdsmi_backend.cpp)  - real gfx950 hardware via libamd_smi
//   * FixtureBackend (fixture_backend.cpp) - scripted topologies / telemetry / faults
//                                             for CPU tests and the 8x8 CPX configs
#pragma once

#include <sys/socket.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <cctype>
#include <string>
#include <vector>

#include "lanes.h"

namespace amdgpu_dp {

// Link classes between two physical GPUs (mirrors amdsmi_link_type_t values).
enum LinkType : int {
  kLinkInternal = 0,  // same physical GPU (on-package Infinity Fabric)
  kLinkPcie = 1,
  kLinkXgmi = 2,
  kLinkNotApplicable = 3,
  kLinkUnknown = 4,
};

struct PartitionInfo {
  int gpu = -1;           // physical GPU index (socket order, sorted by BDF)
  int index = 0;          // partition index inside the GPU (0..num_partitions-1)
  std::string id;         // stable device id advertised to kubelet
  std::string uuid;       // amdsmi uuid of this processor
  int render_minor = -1;  // /dev/dri/renderD<render_minor>
  int card_minor = -1;    // /dev/dri/card<card_minor>
  int hip_id = -1;
  int hsa_id = -1;
  int64_t kfd_node = -1;
  int numa_node = -1;
  uint64_t vram_bytes = 0;
};

// amdsmi_get_gpu_driver_info's version: "6.14.14" for a packaged amdgpu module, but the
// whole /proc/version banner (blanks removed, "Linuxversion6.18.54-...(gcc...)#1...") when
// amdgpu is built into the kernel.  Keeps the first dotted version and its suffix.
inline std::string normalize_driver_version(const std::string& s) {
  auto digit = [](char c) { return c >= '0' && c <= '9'; };
  for (size_t i = 0; i < s.size(); ++i) {
    if (!digit(s[i]) || (i > 0 && (digit(s[i - 1]) || s[i - 1] == '.'))) continue;
    size_t j = i;
    while (j < s.size() && digit(s[j])) ++j;
    if (j + 1 >= s.size() || s[j] != '.' || !digit(s[j + 1])) continue;  // not "N.N"
    while (j < s.size() && (digit(s[j]) || s[j] == '.')) ++j;
    if (j < s.size() && (s[j] == '-' || s[j] == '+' || s[j] == '~'))
      while (j < s.size() && (std::isalnum(static_cast<unsigned char>(s[j])) || s[j] == '.' || s[j] == '-' ||
                              s[j] == '+' || s[j] == '_' || s[j] == '~'))
        ++j;
    return s.substr(i, j - i);
  }
  return s;
}

// One accelerator partition profile the GPU supports
// (amdsmi_get_gpu_accelerator_partition_profile_config).
struct PartitionProfile {
  std::string type;   // SPX/DPX/TPX/QPX/CPX
  int partitions = 0;
  uint32_t nps_caps = 0;  // memory modes allowed with it (bit0 NPS1 .. bit3 NPS8)
  int index = -1;
  // "driver": the driver's profile list (amdsmi_get_gpu_accelerator_partition_profile_config,
  // needs root); "current": only the current profile is known (the list was not readable)
  std::string source = "driver";
};

struct GpuInfo {
  int index = -1;
  std::string key;            // Backend::gpu_key: the identity lanes and health are keyed by
  std::string uuid;
  std::string bdf;            // dddd:bb:dd.f
  std::string market_name;    // e.g. "AMD Instinct MI355X"
  std::string gfx_target;     // e.g. "gfx950"
  std::string serial;
  int numa_node = -1;
  uint64_t vram_total_bytes = 0;
  std::string compute_partition;  // SPX/DPX/TPX/QPX/CPX
  std::string memory_partition;   // NPS1/NPS2/NPS4/NPS8
  uint32_t nps_caps = 0;          // bit0 NPS1, bit1 NPS2, bit2 NPS4, bit3 NPS8
  // The accelerator partition profile the driver reports for the current mode
  // (amdsmi_get_gpu_accelerator_partition_profile): its type and partition count.
  // Empty / 0 when the driver does not report one; the mode string decides then.
  std::string partition_profile;
  int profile_partitions = 0;
  int profile_index = -1;
  // Every profile the driver reports for the GPU (empty: not reported).
  std::vector<PartitionProfile> supported_profiles;
  std::string profiles_status;    // "ok", or why the driver's profile list was not read
  int num_compute_units = 0;
  uint32_t device_id = 0;         // PCI device id (0 = unknown)
  int oam_id = -1;                // OAM slot on the baseboard (-1 = not reported)
  std::string driver_version;     // amdgpu kernel driver
  std::string vbios_version;      // VBIOS / IFWI version string
  int num_xgmi_links = 0;
  int bad_page_threshold = -1;    // RAS retired-page threshold (-1 = not readable)
  std::vector<PartitionInfo> partitions;
};

struct Link {
  int type = kLinkUnknown;
  int hops = 0;
  uint64_t weight = 0;  // amdsmi link weight (lower = closer)
  bool up = true;       // all physical xGMI links between the pair are up
  bool p2p = false;
  double bw_gbps = 0;   // trained bandwidth of the link (all lanes), Gb/s; 0 = unknown
  int pods = 0;         // multi-GPU pods already placed across this GPU pair (share the link)
};

struct Topology {
  int n = 0;
  std::vector<Link> links;  // n*n, row-major; diagonal = internal
  const Link& at(int a, int b) const { return links[static_cast<size_t>(a) * n + b]; }
  Link& at(int a, int b) { return links[static_cast<size_t>(a) * n + b]; }
  void resize(int count) {
    n = count;
    links.assign(static_cast<size_t>(count) * count, Link{});
    for (int i = 0; i < count; ++i) {
      at(i, i).type = kLinkInternal;
      at(i, i).p2p = true;
    }
  }
};

constexpr int kMaxXgmiLinks = 8;
constexpr int kMaxHbm = 8;
constexpr int kMaxPartitions = 8;

// One telemetry sample of a physical GPU.  NaN / negative = unavailable.
struct GpuSample {
  std::string key;  // Backend::gpu_key of the GPU this sample read (set even when it failed)
  // link_peer[k] as identities, resolved against the inventory the sample was read with
  // (an index means another GPU once a re-discovery has moved the indices)
  std::string link_peer_key[kMaxXgmiLinks];
  int64_t ts_ns = 0;
  double power_w = -1;
  double energy_j = -1;            // accumulated
  double temp_edge_c = -1;
  double temp_hotspot_c = -1;
  double temp_mem_c = -1;
  int num_hbm = 0;
  double temp_hbm_c[kMaxHbm] = {};
  double gfx_activity_pct = -1;
  double umc_activity_pct = -1;
  double gfxclk_mhz = -1;
  double uclk_mhz = -1;
  double vram_used_bytes = -1;
  double vram_total_bytes = -1;
  int64_t ecc_correctable = -1;
  int64_t ecc_uncorrectable = -1;
  int64_t throttle_status = -1;
  // RAS retired (bad) HBM pages by status; -1 = unavailable.  Refreshed at a slower
  // cadence than the rest of the sample (the page table rarely changes).
  int64_t retired_pages = -1;
  int64_t pending_pages = -1;
  int64_t unreservable_pages = -1;
  int num_links = 0;
  int link_peer[kMaxXgmiLinks] = {};  // physical GPU index of the peer, -1 unknown
  int link_up[kMaxXgmiLinks] = {};    // 1 up, 0 down, -1 unknown/disabled
  double link_read_kb[kMaxXgmiLinks] = {};
  double link_write_kb[kMaxXgmiLinks] = {};
  double link_bitrate_gbps[kMaxXgmiLinks] = {};   // per-lane signalling rate, Gb/s (0 = unknown)
  double link_max_gbps[kMaxXgmiLinks] = {};       // link capability (all lanes, max rate), Gb/s (0 = unknown)
  // What the link trained at: its current per-lane rate x the GPU's current link width
  // (gpu_metrics); falls back to the capability when either is unknown.  0 = unknown.
  double link_trained_gbps[kMaxXgmiLinks] = {};
  // gpu_metrics: the GPU's current xGMI link width (lanes) and per-lane rate; -1 = unknown
  double xgmi_link_width = -1;
  double xgmi_link_speed = -1;
  // amdsmi_gpu_xgmi_error_status: 0 no errors, 1 an error, 2 multiple (latched until an
  // operator clears them); -1 = unknown
  int xgmi_error_status = -1;
  // gpu_metrics: the host PCIe link (a link that re-trained narrower or slower, and
  // replay / recovery counts, are the classic signs of a failing riser or retimer)
  double pcie_link_width = -1;      // lanes
  double pcie_link_speed_gtps = -1; // GT/s
  double pcie_replays = -1;         // accumulated
  double pcie_recoveries = -1;      // accumulated L0 -> recovery transitions
  int num_partitions = 0;
  double partition_gfx_busy_pct[kMaxPartitions] = {};
  // where partition_gfx_busy_pct[p] came from: 0 unavailable, 1 the partition's own
  // metrics (amdsmi_get_gpu_partition_metrics_info), 2 the socket blob's xcp_stats[p]
  int partition_busy_source[kMaxPartitions] = {};
  double partition_vram_used_bytes[kMaxPartitions] = {};
  // The power-management firmware's own clock, seconds since the firmware started
  // (gpu_metrics firmware_timestamp, 10 ns ticks).  A GPU reset reloads the firmware, so
  // the clock restarting is a reset an unprivileged reader can see without amdsmi event
  // notification (which needs /dev/kfd).  -1 = not reported.
  double fw_clock_s = -1;
  // GPU resets the kernel reports for this device since the backend started watching it
  // (amdgpu context query on the GPU's render node: the driver's own reset counter moved).
  // Attested by the kernel, so it covers resets that leave the firmware running (mode-2,
  // engine resets).  -1 = not available (the render node cannot be opened here).
  int64_t reset_count = -1;
  bool ok = false;
};

// Health-relevant hardware event.
enum EventKind : int {
  kEvtNone = 0,
  kEvtPreReset = 1,     // GPU_PRE_RESET  -> Unhealthy
  kEvtPostReset = 2,    // GPU_POST_RESET -> re-probe -> Healthy
  kEvtEccUncorrectable = 3,
  kEvtLinkDown = 4,
  kEvtLinkUp = 5,
  kEvtThermal = 6,      // informational
  kEvtVmFault = 7,      // informational
  kEvtDeviceLost = 8,   // device disappeared / unrecoverable -> Unhealthy
  kEvtDeviceRecovered = 9,
  kEvtRetiredPagesExceeded = 10,  // retired + pending pages >= threshold -> Unhealthy
  kEvtRetiredPagesCleared = 11,   // back below the threshold (threshold raised, GPU swapped)
  kEvtLinkQuality = 12,   // an up xGMI link re-trained at another bandwidth (value = Gb/s)
  kEvtPcieDegraded = 13,  // host PCIe link below the configured floor -> Unhealthy
  kEvtPcieRestored = 14,  // back at or above it
  // A reset seen by polling (no event delivery): the firmware clock restarted, or the GPU
  // came back from a telemetry outage on a GPU that reports no firmware clock.  Acts
  // like POST_RESET: clears the reset and uncorrectable-ECC latches.
  kEvtResetObserved = 15,
  // The GPU came back from a telemetry outage of failed samples (what a reset looks like
  // to a poller) but nothing confirms a reset: no kernel reset count, no firmware clock
  // restart, no reset uncorrectable-ECC counter.  Informational: the latches hold; the
  // manager re-verifies the GPU with the recovery canary when it is configured.
  kEvtResetCandidate = 16,
  // Latches (uncorrectable ECC, reset in progress) dropped by a re-verification or an
  // operator (HealthMonitor::clear_latches): acts like a reset for the health state.
  kEvtLatchCleared = 17,
};

const char* event_kind_name(int kind);

struct HwEvent {
  int64_t ts_ns = 0;
  int kind = kEvtNone;
  int gpu = -1;        // physical GPU (-1 = all)
  int partition = -1;  // -1 = whole GPU
  int peer = -1;       // for link events
  std::string message;
  // Identity (gpu_key) of `gpu` / `peer` when the event was raised, if the source knew it:
  // an index may be re-used by another GPU after re-enumeration, an identity never is.
  std::string key, peer_key;
  double value = 0;  // kEvtLinkQuality: the link's bandwidth now, Gb/s
};

// A GPU as enumeration finds it, before any call that talks to the device: its identity
// (which names its lane and its health state) and what the backend needs to reach it.
struct DeviceRef {
  std::string key;                 // stable identity (UUID, else BDF)
  std::string bdf;
  uint64_t order = 0;              // enumeration order (BDF)
  std::vector<void*> handles;      // backend handles, partition order (amdsmi processors)
  int slot = -1;                   // fixture slot
};

// The node as one discover() installed it.  Immutable once published: readers take a
// reference and never lock anything a hardware call holds.
struct Inventory {
  uint64_t gen = 0;                // bumped by every discover()
  uint64_t session = 0;            // hardware-library session the handles belong to
  std::vector<DeviceRef> refs;     // index order
  std::vector<GpuInfo> gpus;
  int index_of(const std::string& key) const {
    for (size_t i = 0; i < refs.size(); ++i)
      if (refs[i].key == key) return static_cast<int>(i);
    return -1;
  }
  std::string key_of(int gpu) const {
    return gpu >= 0 && gpu < static_cast<int>(refs.size()) ? refs[gpu].key : std::string();
  }
};

// What the last discover() could not read fresh.  A GPU whose lane is wedged (or whose
// description did not arrive within the call bound) keeps the description of the last
// discovery that reached it; one that no discovery ever reached is left out.
struct DiscoveryReport {
  struct Stale {
    int index = -1;      // in the installed inventory (-1: left out)
    std::string key;
    std::string reason;
  };
  std::vector<Stale> stale;
  double seconds = 0;
  uint64_t gen = 0;
  bool reinit_deferred = false;  // handles looked stale but a call was still inside the library
};

// One GPU's lane as seen from the inventory's index space.
struct LaneReport {
  int index = -1;
  LaneState lane;
};

class Backend : public std::enable_shared_from_this<Backend> {
 public:
  Backend();
  virtual ~Backend() = default;
  virtual std::string name() const = 0;

  // ---- what the plugin calls ----
  // (Re)discover GPUs/partitions/topology.  Throws std::runtime_error when enumeration
  // fails.  Every per-GPU query runs on that GPU's lane and is waited for at most the call
  // bound (set_call_timeout_ms): a wedged GPU costs one bound once, then nothing (its lane
  // refuses work), and is described from the previous discovery (last_discovery()).
  void discover(std::vector<GpuInfo>* gpus, Topology* topo);
  // Telemetry for GPU `gpu` (index of the latest discover()), waited for at most the call
  // bound; false when unavailable or still in flight.
  bool sample(int gpu, GpuSample* out);
  // The same call without waiting: null when there is no such GPU or its lane refused the
  // job (wedged).  The job fills *out; read it only once job->done() && !job->dropped().
  // `key` (optional): the GPU's identity; it is looked up in the current inventory, so a
  // caller holding indices of an older discovery never samples the GPU that moved into
  // that index (null when the GPU is gone).
  std::shared_ptr<LaneJob> sample_async(int gpu, std::shared_ptr<GpuSample> out, const std::string& key = "");
  // Stable identity (UUID, else BDF) of the GPU at index `gpu` of the latest discover(),
  // in the index space sample() and events use; "" when unknown.  Health state is keyed
  // by it: when a GPU drops off the bus and the node re-enumerates, every later GPU moves
  // down one index, and its health must not move with the index.  Never blocks.
  virtual std::string gpu_key(int gpu) const;
  std::shared_ptr<const Inventory> inventory() const;
  DiscoveryReport last_discovery() const;
  // Lanes of the inventory's GPUs (index order) and, after them, lanes of GPUs that left it
  // with a call still in flight (index -1).
  std::vector<LaneReport> lanes() const;
  // mono ns at which the latest hardware call on any lane ended (0: none yet)
  int64_t last_completion_ns() const;
  void set_call_timeout_ms(int ms) { call_timeout_ms_.store(ms > 0 ? ms : 10000); }
  int call_timeout_ms() const { return call_timeout_ms_.load(); }
  // A lane whose call has been in flight longer than this takes no more work (0: never).
  void set_stall_ms(int ms) { stall_ms_.store(ms > 0 ? ms : 0); }
  int stall_ms() const { return stall_ms_.load(); }
  // health.resetQuery: samples read the kernel's reset count through an amdgpu context on
  // each GPU's render node (GpuSample::reset_count) where the node can be opened.
  void set_reset_query(bool on) { reset_query_.store(on); }
  bool reset_query() const { return reset_query_.load(); }
  // health.eccEventGate: the ECC totals are re-read when the driver's RAS event state
  // (fatal errors, poison creation / consumption) moved, and every 30 s otherwise,
  // instead of every sample (amdsmi backend; where the kernel has that file).
  void set_ecc_event_gate(bool on) { ecc_event_gate_.store(on); }
  bool ecc_event_gate() const { return ecc_event_gate_.load(); }

  // Block up to timeout_ms for hardware events; append to *out.  Returns count.
  virtual int wait_events(int timeout_ms, std::vector<HwEvent>* out) = 0;
  // Arm event delivery for the discovered GPUs (idempotent).
  virtual void arm_events() {}
  // Number of processors with hardware event delivery armed (0 = polling only).  Never blocks.
  virtual int armed_event_sources() const { return 0; }
  // Whether wait_events has anything to wait on (armed sources, a fixture's scripts).  When
  // not, the health monitor's event thread sleeps a second at a time instead of calling it.
  virtual bool delivers_events() const { return true; }
  // How long one wait_events call may block: the event thread's stop latency and its idle
  // wake-up rate (a backend whose wait cannot be interrupted keeps this short).
  virtual int event_wait_ms() const { return 200; }
  // Drop cached device handles so the next discover() enumerates afresh (a compute
  // partition change creates new processors).  Returns false when not possible.
  virtual bool reinit() { return true; }
  // Times the backend re-initialised its hardware library (stale-handle recovery).
  virtual int reinit_count() const { return 0; }
  // Cumulative cost of the hardware calls inside sample(): (call, seconds, calls).
  struct CallCost {
    std::string call;
    double seconds = 0;
    uint64_t calls = 0;
  };
  virtual std::vector<CallCost> sample_costs() const { return {}; }
  virtual void shutdown() {}

 protected:
  // ---- what a backend implements ----
  // The GPUs present, in a stable order, without talking to any one device (amdsmi keeps
  // its processor list from amdsmi_init).  Throws on failure.
  virtual void enumerate(std::vector<DeviceRef>* refs) = 0;
  // Everything discovery reads from one GPU, on that GPU's lane: its description (index
  // fields are set by the caller) and its view of the link to each GPU of `all` (row[i]:
  // the link to all[i]).  Throws (or leaves out->partitions empty) on failure.
  virtual void describe(const DeviceRef& ref, const std::vector<DeviceRef>& all, GpuInfo* out,
                        std::vector<Link>* row) = 0;
  // One telemetry sample of inv.refs[index], on that GPU's lane.
  virtual bool sample_device(const Inventory& inv, int index, GpuSample* out) = 0;
  // Handles are out of date (e.g. amdsmi enumerates processors once, at init, and a
  // compute-partition change created new ones): called with discovery's fresh
  // descriptions; return true to have the library re-initialised (reopen_session) and
  // the node enumerated again.
  virtual bool handles_stale(const std::vector<GpuInfo>& described) { return false; }
  // Re-initialises the hardware library with no call inside it (the gate is closed).
  virtual bool reopen_session() { return false; }
  // After an inventory was installed (the handles to arm event delivery on, say).
  virtual void installed(const std::shared_ptr<const Inventory>& inv) {}

  // Runs fn on the lane of `key` inside the library session (see SessionGate); waits at
  // most ms.  false: refused (wedged lane, stale session) or not done in time.
  bool run_on_lane(const std::string& key, const char* what, uint64_t session, std::function<void()> fn,
                   int64_t ms);
  // Same, without waiting: null when the lane refused it.
  std::shared_ptr<LaneJob> post_job(const std::string& key, const char* what, uint64_t session,
                                    std::function<void()> fn, uint64_t batch = 0);
  // a fresh batch number for jobs posted to several lanes at once (see LaneJob)
  uint64_t next_batch() { return batch_seq_.fetch_add(1) + 1; }
  SessionGate& gate() { return gate_; }
  LaneSet& lanes_set() { return lanes_; }

 private:
  struct Described {
    GpuInfo info;
    std::map<std::string, Link> links;  // peer key -> this GPU's view of the link
  };
  LaneSet lanes_;
  std::atomic<uint64_t> batch_seq_{0};
  SessionGate gate_;
  std::atomic<int> call_timeout_ms_{10000};
  std::atomic<bool> reset_query_{true};
  std::atomic<bool> ecc_event_gate_{true};
  std::atomic<int> stall_ms_{0};
  std::atomic<int64_t> last_completion_ns_{0};
  // one discovery at a time (a flag + condition: libstdc++'s timed mutex waits are not
  // visible to GCC 11's ThreadSanitizer)
  std::mutex discover_mu_;
  std::condition_variable discover_cv_;
  bool discovering_ = false;               // guarded by discover_mu_
  std::map<std::string, Described> last_described_;  // by key; owned by the running discovery
  mutable std::mutex inv_mu_;              // inv_ and report_ only, never held across a call
  std::shared_ptr<const Inventory> inv_;
  DiscoveryReport report_;
  uint64_t gen_ = 0;                       // owned by the running discovery
};

std::shared_ptr<Backend> make_amdsmi_backend();
// Is an AMD GPU visible to amdsmi?  keep=true leaves the session open for the next
// make_amdsmi_backend() to adopt; amdsmi_release_probe() drops it if none does.
bool amdsmi_available(bool keep = false);
void amdsmi_release_probe();
bool amdsmi_probe_held();

int64_t now_ns();
int64_t mono_ns();

// Background threads (sampler, watchdog, lanes, event wait, access log) name themselves
// and, with set_background_batch(true), switch to SCHED_BATCH: still a fair share of the
// CPU, but a batch thread that wakes never preempts the thread running on its CPU.  Off by
// default (config backgroundSched): on an idle box it did not change the Allocate tail.
// Threads started before the switch keep their policy.
void set_background_batch(bool on);
bool background_batch();
int64_t background_batched_threads();  // threads switched so far
void background_thread(const char* name);
void foreground_thread();  // back to SCHED_OTHER if the creator was a batch thread

// accept4 (non-blocking, close-on-exec) for a level-triggered listener that sheds load
// instead of spinning when the process runs out of file descriptors: the pending
// connection would stay in the backlog and keep the listener readable, and every
// epoll_wait would return at once.  *spare is the caller's reserve descriptor (-1: opened
// lazily); on EMFILE/ENFILE it is given up for one accept whose connection is closed at
// once.  Returns the connection fd, or -1 with errno (EAGAIN: backlog empty;
// ECONNABORTED: one connection was shed, *shed set; call again).
int accept_or_shed(int lfd, struct sockaddr* addr, socklen_t* len, int* spare, bool* shed);

// Timed condition-variable wait.  libstdc++ implements steady-clock waits with
// pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not intercept (it then
// reports bogus double-locks/races); TSan builds wait on the system clock instead.
template <class Pred>
bool cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, int64_t ms, Pred pred) {
#if defined(__SANITIZE_THREAD__)
  return cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), pred);
#else
  return cv.wait_for(lk, std::chrono::milliseconds(ms), pred);
#endif
}

}  // namespace amdgpu_dp
