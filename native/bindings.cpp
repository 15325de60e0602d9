// pybind11 module `k8s_gpu_device_plugin_amd._native`.
// Long-blocking calls (health pop, inotify read, server stop, scrapes) release the GIL.
#include <sched.h>

#include <chrono>
#include <thread>

#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "allocator.h"
#include "backend.h"
#include "core_escape.h"
#include "device_table.h"
#include "fixture_backend.h"
#include "grpc_h2.h"
#include "hpack.h"
#include "health.h"
#include "httpd.h"
#include "metrics.h"
#include "profiler.h"
#include "telemetry.h"
#include "watch.h"

namespace py = pybind11;
using namespace amdgpu_dp;

namespace {

py::tuple ok_bytes(bool ok, const std::string& s) {
  if (ok) return py::make_tuple(true, py::bytes(s));
  return py::make_tuple(false, py::str(s));
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X device plugin native core (amdsmi backend, allocator, exporter, httpd)";

  py::class_<PartitionInfo>(m, "PartitionInfo")
      .def(py::init<>())
      .def_readwrite("gpu", &PartitionInfo::gpu)
      .def_readwrite("index", &PartitionInfo::index)
      .def_readwrite("id", &PartitionInfo::id)
      .def_readwrite("uuid", &PartitionInfo::uuid)
      .def_readwrite("render_minor", &PartitionInfo::render_minor)
      .def_readwrite("card_minor", &PartitionInfo::card_minor)
      .def_readwrite("hip_id", &PartitionInfo::hip_id)
      .def_readwrite("hsa_id", &PartitionInfo::hsa_id)
      .def_readwrite("kfd_node", &PartitionInfo::kfd_node)
      .def_readwrite("numa_node", &PartitionInfo::numa_node)
      .def_readwrite("vram_bytes", &PartitionInfo::vram_bytes);

  py::class_<PartitionProfile>(m, "PartitionProfile")
      .def(py::init([](const std::string& type, int partitions, uint32_t nps_caps, int index,
                       const std::string& source) {
             PartitionProfile p;
             p.type = type;
             p.partitions = partitions;
             p.nps_caps = nps_caps;
             p.index = index;
             p.source = source;
             return p;
           }),
           py::arg("type") = "", py::arg("partitions") = 0, py::arg("nps_caps") = 0, py::arg("index") = -1,
           py::arg("source") = "driver")
      .def_readwrite("source", &PartitionProfile::source)
      .def_readwrite("type", &PartitionProfile::type)
      .def_readwrite("partitions", &PartitionProfile::partitions)
      .def_readwrite("nps_caps", &PartitionProfile::nps_caps)
      .def_readwrite("index", &PartitionProfile::index)
      .def("__repr__", [](const PartitionProfile& p) {
        return "<PartitionProfile " + p.type + " x" + std::to_string(p.partitions) + " nps_caps=" +
               std::to_string(p.nps_caps) + ">";
      });

  py::class_<GpuInfo>(m, "GpuInfo")
      .def(py::init<>())
      .def_readwrite("index", &GpuInfo::index)
      .def_readwrite("key", &GpuInfo::key)
      .def_readwrite("uuid", &GpuInfo::uuid)
      .def_readwrite("bdf", &GpuInfo::bdf)
      .def_readwrite("market_name", &GpuInfo::market_name)
      .def_readwrite("gfx_target", &GpuInfo::gfx_target)
      .def_readwrite("serial", &GpuInfo::serial)
      .def_readwrite("numa_node", &GpuInfo::numa_node)
      .def_readwrite("vram_total_bytes", &GpuInfo::vram_total_bytes)
      .def_readwrite("compute_partition", &GpuInfo::compute_partition)
      .def_readwrite("memory_partition", &GpuInfo::memory_partition)
      .def_readwrite("nps_caps", &GpuInfo::nps_caps)
      .def_readwrite("partition_profile", &GpuInfo::partition_profile)
      .def_readwrite("profile_partitions", &GpuInfo::profile_partitions)
      .def_readwrite("profile_index", &GpuInfo::profile_index)
      .def_readwrite("num_compute_units", &GpuInfo::num_compute_units)
      .def_readwrite("device_id", &GpuInfo::device_id)
      .def_readwrite("oam_id", &GpuInfo::oam_id)
      .def_readwrite("driver_version", &GpuInfo::driver_version)
      .def_readwrite("vbios_version", &GpuInfo::vbios_version)
      .def_readwrite("num_xgmi_links", &GpuInfo::num_xgmi_links)
      .def_readwrite("bad_page_threshold", &GpuInfo::bad_page_threshold)
      .def_readwrite("supported_profiles", &GpuInfo::supported_profiles)
      .def_readwrite("profiles_status", &GpuInfo::profiles_status)
      .def_readwrite("partitions", &GpuInfo::partitions);

  py::class_<Link>(m, "Link")
      .def(py::init<>())
      .def(py::init([](int type, int hops, uint64_t weight, bool up, bool p2p, double bw_gbps, int pods) {
             Link l;
             l.type = type;
             l.hops = hops;
             l.weight = weight;
             l.up = up;
             l.p2p = p2p;
             l.bw_gbps = bw_gbps;
             l.pods = pods;
             return l;
           }),
           py::arg("type") = static_cast<int>(kLinkXgmi), py::arg("hops") = 1, py::arg("weight") = 15,
           py::arg("up") = true, py::arg("p2p") = true, py::arg("bw_gbps") = 0.0, py::arg("pods") = 0)
      .def_readwrite("bw_gbps", &Link::bw_gbps)
      .def_readwrite("pods", &Link::pods)
      .def_readwrite("type", &Link::type)
      .def_readwrite("hops", &Link::hops)
      .def_readwrite("weight", &Link::weight)
      .def_readwrite("up", &Link::up)
      .def_readwrite("p2p", &Link::p2p);

  py::class_<Topology>(m, "Topology")
      .def(py::init<>())
      .def(py::init([](int n) {
        Topology t;
        t.resize(n);
        return t;
      }))
      .def_readonly("n", &Topology::n)
      .def("link", [](const Topology& t, int a, int b) {
        if (a < 0 || b < 0 || a >= t.n || b >= t.n) throw py::index_error("gpu index");
        return t.at(a, b);
      })
      .def("set_link", [](Topology& t, int a, int b, const Link& l) {
        if (a < 0 || b < 0 || a >= t.n || b >= t.n) throw py::index_error("gpu index");
        t.at(a, b) = l;
        t.at(b, a) = l;
      });

  py::class_<GpuSample>(m, "GpuSample")
      .def(py::init<>())
      .def_readonly("key", &GpuSample::key)
      .def_property_readonly("link_peer_keys", [](const GpuSample& s) {
        return std::vector<std::string>(s.link_peer_key, s.link_peer_key + std::max(0, std::min(s.num_links, kMaxXgmiLinks)));
      })
      .def_readonly("ts_ns", &GpuSample::ts_ns)
      .def_readonly("ok", &GpuSample::ok)
      .def_readonly("power_w", &GpuSample::power_w)
      .def_readonly("energy_j", &GpuSample::energy_j)
      .def_readonly("temp_edge_c", &GpuSample::temp_edge_c)
      .def_readonly("temp_hotspot_c", &GpuSample::temp_hotspot_c)
      .def_readonly("temp_mem_c", &GpuSample::temp_mem_c)
      .def_property_readonly("temp_hbm_c", [](const GpuSample& s) {
        return std::vector<double>(s.temp_hbm_c, s.temp_hbm_c + s.num_hbm);
      })
      .def_readonly("gfx_activity_pct", &GpuSample::gfx_activity_pct)
      .def_readonly("umc_activity_pct", &GpuSample::umc_activity_pct)
      .def_readonly("gfxclk_mhz", &GpuSample::gfxclk_mhz)
      .def_readonly("uclk_mhz", &GpuSample::uclk_mhz)
      .def_readonly("vram_used_bytes", &GpuSample::vram_used_bytes)
      .def_readonly("vram_total_bytes", &GpuSample::vram_total_bytes)
      .def_readonly("ecc_correctable", &GpuSample::ecc_correctable)
      .def_readonly("ecc_uncorrectable", &GpuSample::ecc_uncorrectable)
      .def_readonly("retired_pages", &GpuSample::retired_pages)
      .def_readonly("pending_pages", &GpuSample::pending_pages)
      .def_readonly("unreservable_pages", &GpuSample::unreservable_pages)
      .def_readonly("throttle_status", &GpuSample::throttle_status)
      .def_readonly("xgmi_link_width", &GpuSample::xgmi_link_width)
      .def_readonly("xgmi_link_speed", &GpuSample::xgmi_link_speed)
      .def_readonly("xgmi_error_status", &GpuSample::xgmi_error_status)
      .def_readonly("pcie_link_width", &GpuSample::pcie_link_width)
      .def_readonly("pcie_link_speed_gtps", &GpuSample::pcie_link_speed_gtps)
      .def_readonly("pcie_replays", &GpuSample::pcie_replays)
      .def_readonly("pcie_recoveries", &GpuSample::pcie_recoveries)
      .def_readonly("fw_clock_s", &GpuSample::fw_clock_s)
      .def_readonly("reset_count", &GpuSample::reset_count)
      .def_property_readonly("links", [](const GpuSample& s) {
        py::list l;
        for (int k = 0; k < s.num_links; ++k)
          l.append(py::make_tuple(s.link_peer[k], s.link_up[k], s.link_read_kb[k], s.link_write_kb[k],
                                  s.link_bitrate_gbps[k], s.link_max_gbps[k], s.link_trained_gbps[k]));
        return l;
      })
      .def_property_readonly("partition_gfx_busy_pct", [](const GpuSample& s) {
        return std::vector<double>(s.partition_gfx_busy_pct, s.partition_gfx_busy_pct + s.num_partitions);
      })
      .def_property_readonly("partition_busy_source", [](const GpuSample& s) {
        return std::vector<int>(s.partition_busy_source, s.partition_busy_source + s.num_partitions);
      })
      .def_property_readonly("partition_vram_used_bytes", [](const GpuSample& s) {
        return std::vector<double>(s.partition_vram_used_bytes, s.partition_vram_used_bytes + s.num_partitions);
      });

  m.attr("EVT_PRE_RESET") = static_cast<int>(kEvtPreReset);
  m.attr("EVT_POST_RESET") = static_cast<int>(kEvtPostReset);
  m.attr("EVT_ECC_UNCORRECTABLE") = static_cast<int>(kEvtEccUncorrectable);
  m.attr("EVT_LINK_DOWN") = static_cast<int>(kEvtLinkDown);
  m.attr("EVT_LINK_UP") = static_cast<int>(kEvtLinkUp);
  m.attr("EVT_THERMAL") = static_cast<int>(kEvtThermal);
  m.attr("EVT_VM_FAULT") = static_cast<int>(kEvtVmFault);
  m.attr("EVT_DEVICE_LOST") = static_cast<int>(kEvtDeviceLost);
  m.attr("EVT_DEVICE_RECOVERED") = static_cast<int>(kEvtDeviceRecovered);
  m.attr("EVT_RETIRED_PAGES_EXCEEDED") = static_cast<int>(kEvtRetiredPagesExceeded);
  m.attr("EVT_RETIRED_PAGES_CLEARED") = static_cast<int>(kEvtRetiredPagesCleared);
  m.attr("EVT_PCIE_DEGRADED") = static_cast<int>(kEvtPcieDegraded);
  m.attr("EVT_PCIE_RESTORED") = static_cast<int>(kEvtPcieRestored);
  m.attr("EVT_LINK_QUALITY") = static_cast<int>(kEvtLinkQuality);
  m.attr("EVT_RESET_OBSERVED") = static_cast<int>(kEvtResetObserved);
  m.attr("EVT_RESET_CANDIDATE") = static_cast<int>(kEvtResetCandidate);
  m.attr("EVT_LATCH_CLEARED") = static_cast<int>(kEvtLatchCleared);
  m.attr("EVT_FIXTURE_FIRMWARE_RESET") = FixtureBackend::kScriptFirmwareReset;
  m.attr("LINK_INTERNAL") = static_cast<int>(kLinkInternal);
  m.attr("LINK_PCIE") = static_cast<int>(kLinkPcie);
  m.attr("LINK_XGMI") = static_cast<int>(kLinkXgmi);
  m.attr("LINK_UNKNOWN") = static_cast<int>(kLinkUnknown);
  m.def("event_kind_name", &event_kind_name);

  py::class_<HwEvent>(m, "HwEvent")
      .def(py::init([](int kind, int gpu, int partition, int peer, const std::string& msg) {
             HwEvent e;
             e.kind = kind;
             e.gpu = gpu;
             e.partition = partition;
             e.peer = peer;
             e.message = msg;
             return e;
           }),
           py::arg("kind"), py::arg("gpu") = -1, py::arg("partition") = -1, py::arg("peer") = -1,
           py::arg("message") = "")
      .def_readwrite("kind", &HwEvent::kind)
      .def_readwrite("gpu", &HwEvent::gpu)
      .def_readwrite("partition", &HwEvent::partition)
      .def_readwrite("peer", &HwEvent::peer)
      .def_readwrite("message", &HwEvent::message)
      .def_readwrite("key", &HwEvent::key)
      .def_readwrite("value", &HwEvent::value)
      .def_readwrite("peer_key", &HwEvent::peer_key)
      .def_readwrite("ts_ns", &HwEvent::ts_ns);

  py::class_<Backend, std::shared_ptr<Backend>>(m, "Backend")
      .def_property_readonly("name", &Backend::name)
      .def("sample_costs",
           [](const Backend& b) {
             py::dict d;
             for (const auto& c : b.sample_costs()) d[py::str(c.call)] = py::make_tuple(c.seconds, c.calls);
             return d;
           })
      .def("discover",
           [](Backend& b) {
             std::vector<GpuInfo> g;
             Topology t;
             {
               py::gil_scoped_release rel;
               b.discover(&g, &t);
             }
             return py::make_tuple(g, t);
           })
      .def("sample",
           [](Backend& b, int gpu) -> py::object {
             GpuSample s;
             bool ok;
             {
               py::gil_scoped_release rel;
               ok = b.sample(gpu, &s);
             }
             if (!ok) return py::none();
             return py::cast(s);
           })
      .def("gpu_key", &Backend::gpu_key, py::call_guard<py::gil_scoped_release>())
      .def("set_call_timeout_ms", &Backend::set_call_timeout_ms)
      .def_property_readonly("call_timeout_ms", &Backend::call_timeout_ms)
      .def("set_stall_ms", &Backend::set_stall_ms)
      .def("set_reset_query", &Backend::set_reset_query, py::arg("on"))
      .def("set_ecc_event_gate", &Backend::set_ecc_event_gate, py::arg("on"))
      .def_property_readonly("stall_ms", &Backend::stall_ms)
      .def("last_discovery",
           [](const Backend& b) {
             DiscoveryReport r = b.last_discovery();
             py::dict d;
             py::list stale;
             for (const auto& s : r.stale) stale.append(py::make_tuple(s.index, s.key, s.reason));
             d["stale"] = stale;
             d["seconds"] = r.seconds;
             d["generation"] = r.gen;
             d["reinit_deferred"] = r.reinit_deferred;
             return d;
           })
      .def("lanes",  // [(index, key, in-flight call or "", in flight s, completed, queued)]
           [](const Backend& b) {
             py::list out;
             const int64_t now = mono_ns();
             for (const auto& r : b.lanes())
               out.append(py::make_tuple(r.index, r.lane.key, r.lane.inflight_what,
                                         r.lane.inflight_since_ns ? (now - r.lane.inflight_since_ns) * 1e-9 : 0.0,
                                         r.lane.completed, r.lane.queued));
             return out;
           })
      .def("arm_events", &Backend::arm_events, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("armed_event_sources", &Backend::armed_event_sources)
      .def("reinit", &Backend::reinit, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("reinit_count", &Backend::reinit_count)
      .def("shutdown", &Backend::shutdown, py::call_guard<py::gil_scoped_release>());

  py::class_<FixtureBackend, Backend, std::shared_ptr<FixtureBackend>>(m, "FixtureBackend")
      .def(py::init<uint64_t>(), py::arg("seed") = 1)
      .def("add_gpu", &FixtureBackend::add_gpu)
      .def("replace_gpu", &FixtureBackend::replace_gpu)
      .def("slot_info", &FixtureBackend::slot_info)
      .def("clear", &FixtureBackend::clear)
      .def("set_link", &FixtureBackend::set_link)
      .def("set_link_up", &FixtureBackend::set_link_up)
      .def("set_link_bandwidth", &FixtureBackend::set_link_bandwidth)
      .def("schedule_event", &FixtureBackend::schedule_event)
      .def("inject_event", &FixtureBackend::inject_event)
      .def("set_fail_discovery", &FixtureBackend::set_fail_discovery)
      .def("set_ecc_uncorrectable", &FixtureBackend::set_ecc_uncorrectable)
      .def("set_pcie_link", &FixtureBackend::set_pcie_link, py::arg("gpu"), py::arg("width"), py::arg("gts"))
      .def("set_retired_pages", &FixtureBackend::set_retired_pages, py::arg("gpu"), py::arg("reserved"),
           py::arg("pending") = 0)
      .def("set_sample_stall", &FixtureBackend::set_sample_stall, py::call_guard<py::gil_scoped_release>())
      .def("set_serialised", &FixtureBackend::set_serialised, py::arg("on"))
      .def_property_readonly("serialised", &FixtureBackend::serialised)
      .def("set_gpu_present", &FixtureBackend::set_gpu_present)
      .def("reset_firmware", &FixtureBackend::reset_firmware)
      .def("set_fw_clock_reported", &FixtureBackend::set_fw_clock_reported, py::arg("gpu"), py::arg("reported"))
      .def("set_fw_clock_frozen", &FixtureBackend::set_fw_clock_frozen, py::arg("gpu"), py::arg("frozen"),
           py::arg("at_s") = -1.0)
      .def("glitch_fw_clock", &FixtureBackend::glitch_fw_clock, py::arg("gpu"), py::arg("value_s"))
      .def("set_gpu_reset_query", &FixtureBackend::set_gpu_reset_query, py::arg("gpu"), py::arg("available"))
      .def("reset_gpu", &FixtureBackend::reset_gpu, py::arg("gpu"), py::arg("reload_firmware"))
      .def("set_sample_fail", &FixtureBackend::set_sample_fail, py::arg("gpu"), py::arg("fail"))
      .def("set_events_enabled", &FixtureBackend::set_events_enabled, py::arg("on"))
      .def_property_readonly("discover_calls", &FixtureBackend::discover_calls);

  m.def("make_amdsmi_backend", &make_amdsmi_backend, py::call_guard<py::gil_scoped_release>());
  m.def("normalize_driver_version", &normalize_driver_version, py::arg("reported"));
  m.def("amdsmi_available", &amdsmi_available, py::arg("keep") = false, py::call_guard<py::gil_scoped_release>());
  m.def("amdsmi_release_probe", &amdsmi_release_probe, py::call_guard<py::gil_scoped_release>());
  m.def("amdsmi_probe_held", &amdsmi_probe_held);

  // ---- allocator (raw, for tests / Python policies) ----
  py::class_<AllocDevice>(m, "AllocDevice")
      .def(py::init([](int gpu, int partition, int numa, const std::string& base_id, bool annotated) {
             AllocDevice d;
             d.gpu = gpu;
             d.partition = partition;
             d.numa = numa;
             d.base_id = base_id;
             d.annotated = annotated;
             return d;
           }),
           py::arg("gpu"), py::arg("partition") = -1, py::arg("numa") = -1, py::arg("base_id") = "",
           py::arg("annotated") = false)
      .def_readwrite("gpu", &AllocDevice::gpu)
      .def_readwrite("partition", &AllocDevice::partition)
      .def_readwrite("numa", &AllocDevice::numa)
      .def_readwrite("base_id", &AllocDevice::base_id);
  m.def("pair_score", [](const Topology& t, const AllocDevice& a, const AllocDevice& b) { return pair_score(t, a, b); });
  m.def("aligned_alloc", [](const Topology& t, const std::vector<AllocDevice>& d, const std::vector<int>& avail,
                            const std::vector<int>& req, int size) {
    AllocResult r = aligned_alloc(t, d, avail, req, size);
    if (!r.ok) throw std::runtime_error(r.error);
    return r.chosen;
  });
  m.def("bench_aligned_alloc",  // per-call seconds of n aligned_alloc calls (allocator cost alone)
        [](const Topology& t, const std::vector<AllocDevice>& d, const std::vector<int>& avail,
           const std::vector<int>& req, int size, int n) {
          std::vector<double> out;
          out.reserve(static_cast<size_t>(std::max(0, n)));
          py::gil_scoped_release rel;
          for (int i = 0; i < n; ++i) {
            const int64_t t0 = mono_ns();
            AllocResult r = aligned_alloc(t, d, avail, req, size);
            out.push_back((mono_ns() - t0) * 1e-9);
            if (!r.ok) throw std::runtime_error(r.error);
          }
          return out;
        });
  py::class_<RecentAllocations, std::shared_ptr<RecentAllocations>>(m, "RecentAllocations")
      .def(py::init<>())
      .def("record_gpus",
           [](RecentAllocations& r, const std::vector<int>& gpus) {
             uint64_t mask = 0;
             for (int g : gpus)
               if (g >= 0 && g < 64) mask |= 1ull << g;
             r.record(mask, mono_ns());
           })
      .def("set_covered_until", &RecentAllocations::set_covered_until, py::arg("mono_ns"))
      .def("set_ttl_ms", &RecentAllocations::set_ttl_ms)
      .def("live", [](const RecentAllocations& r) { return r.live(mono_ns()); })
      .def("link_pods", [](const RecentAllocations& r, int n) {
        std::vector<int> pods(static_cast<size_t>(std::max(0, n)) * std::max(0, n), 0);
        r.add_link_pods(n, mono_ns(), &pods);
        return pods;
      });
  m.def("mono_ns", &mono_ns);
  m.def("set_background_batch", &set_background_batch, py::arg("on"));
  m.def("background_batch", &background_batch);
  m.def("background_batched_threads", &background_batched_threads);
  m.def("distributed_alloc", [](const std::vector<AllocDevice>& d, const std::vector<int>& avail,
                                const std::vector<int>& req, int size) {
    AllocResult r = distributed_alloc(d, avail, req, size);
    if (!r.ok) throw std::runtime_error(r.error);
    return r.chosen;
  });

  // ---- device table ----
  py::class_<TableDevice>(m, "TableDevice")
      .def(py::init([](const std::string& id, int gpu, int partition, int numa, int replica,
                       const std::vector<std::string>& paths, bool healthy) {
             TableDevice d;
             d.id = id;
             d.gpu = gpu;
             d.partition = partition;
             d.numa = numa;
             d.replica = replica;
             d.host_paths = paths;
             d.healthy = healthy;
             return d;
           }),
           py::arg("id"), py::arg("gpu"), py::arg("partition") = -1, py::arg("numa") = -1, py::arg("replica") = -1,
           py::arg("host_paths") = std::vector<std::string>{}, py::arg("healthy") = true)
      .def_readonly("id", &TableDevice::id)
      .def_readonly("gpu", &TableDevice::gpu)
      .def_readonly("partition", &TableDevice::partition)
      .def_readonly("numa", &TableDevice::numa)
      .def_readonly("replica", &TableDevice::replica)
      .def_readonly("host_paths", &TableDevice::host_paths)
      .def_readonly("healthy", &TableDevice::healthy);

  py::class_<TableConfig>(m, "TableConfig")
      .def(py::init<>())
      .def_readwrite("resource_name", &TableConfig::resource_name)
      .def_readwrite("visible_env", &TableConfig::visible_env)
      .def_readwrite("extra_envs", &TableConfig::extra_envs)
      .def_readwrite("mount_kfd", &TableConfig::mount_kfd)
      .def_readwrite("kfd_path", &TableConfig::kfd_path)
      .def_readwrite("permissions", &TableConfig::permissions)
      .def_readwrite("cdi", &TableConfig::cdi)
      .def_readwrite("cdi_prefix", &TableConfig::cdi_prefix)
      .def_readwrite("reject_unhealthy", &TableConfig::reject_unhealthy)
      .def_readwrite("pre_start_required", &TableConfig::pre_start_required);

  m.attr("RPC_OPTIONS") = static_cast<int>(kRpcOptions);
  m.attr("RPC_LIST_AND_WATCH") = static_cast<int>(kRpcListAndWatch);
  m.attr("RPC_PREFERRED") = static_cast<int>(kRpcPreferred);
  m.attr("RPC_ALLOCATE") = static_cast<int>(kRpcAllocate);
  m.attr("RPC_PRE_START") = static_cast<int>(kRpcPreStart);

  py::class_<ContentionDetector>(m, "ContentionDetector")  // grpc.coreEscape's decision (tests)
      .def(py::init<>())
      .def("note", &ContentionDetector::note, py::arg("svc_ns"), py::arg("now_ns"))
      .def_property_readonly("best_ns", &ContentionDetector::best_ns)
      .def_property_readonly("last_median_ns", &ContentionDetector::last_median_ns);
  m.def("parse_cpu_list", [](const std::string& s) { return parse_cpu_list(s.c_str()); });
  m.def("peer_on_sibling", &peer_on_sibling, py::arg("fd"), py::arg("cpu"), py::arg("now_ns") = 0);
  py::class_<DeviceTable, std::shared_ptr<DeviceTable>>(m, "DeviceTable")
      .def("inherit_stats", &DeviceTable::inherit_stats, py::arg("prev"))
      .def("wait_change", &DeviceTable::wait_change, py::call_guard<py::gil_scoped_release>(), py::arg("seen"),
           py::arg("timeout_ms") = 500)
      .def("wake", &DeviceTable::wake)
      .def(py::init<TableConfig, std::vector<TableDevice>, Topology>())
      .def_property_readonly("resource_name", [](const DeviceTable& t) { return t.config().resource_name; })
      .def("__len__", &DeviceTable::size)
      .def("device", [](const DeviceTable& t, size_t i) {
        if (i >= t.size()) throw py::index_error();
        return t.device(i);
      })
      .def("ids", &DeviceTable::ids)
      .def("index_of", [](const DeviceTable& t, const std::string& id) { return t.index_of(id); })
      .def("contains", &DeviceTable::contains)
      .def_property_readonly("aligned_supported", &DeviceTable::aligned_supported)
      .def("set_health", [](DeviceTable& t, const std::string& id, bool h) { return t.set_health(id, h); })
      .def("set_gpu_health", &DeviceTable::set_gpu_health)
      .def("set_gpu_health_except", &DeviceTable::set_gpu_health_except, py::arg("gpu"), py::arg("held"))
      .def("healthy", [](const DeviceTable& t, const std::string& id) { return t.healthy(id); })
      .def("healthy_count", &DeviceTable::healthy_count)
      .def("set_link_up", &DeviceTable::set_link_up)
      .def("set_link_bandwidth", &DeviceTable::set_link_bandwidth)
      .def("set_link_pods", &DeviceTable::set_link_pods)
      .def("set_recent_allocations", &DeviceTable::set_recent_allocations)
      .def("topology", &DeviceTable::topology)
      .def_property_readonly("version", &DeviceTable::version)
      .def("list_and_watch", [](const DeviceTable& t) { return py::bytes(t.list_and_watch()); })
      .def("options", [](const DeviceTable& t) { return py::bytes(t.options_bytes()); })
      // PreStartContainer job queue (verifier side + the grpcio server's submit)
      .def("submit_prestart",
           [](DeviceTable& t, const py::bytes& req, std::function<void(bool, std::string)> done) {
             std::string err;
             const bool ok = t.submit_prestart(std::string(req),
                                               [done](bool pass, const std::string& e) { done(pass, e); }, &err);
             return py::make_tuple(ok, err);
           })
      .def("pop_prestart",
           [](DeviceTable& t, int timeout_ms) {
             std::vector<PreStartJob> jobs;
             {
               py::gil_scoped_release rel;
               jobs = t.pop_prestart(timeout_ms);
             }
             py::list out;
             for (auto& j : jobs) out.append(py::make_tuple(j.id, j.ids));
             return out;
           },
           py::arg("timeout_ms") = 200)
      .def("complete_prestart", &DeviceTable::complete_prestart)
      .def("cancel_prestart", &DeviceTable::cancel_prestart, py::call_guard<py::gil_scoped_release>())
      .def("resume_prestart", &DeviceTable::resume_prestart)
      .def_property_readonly("prestart_pending", &DeviceTable::prestart_pending)
      .def("allocate",
           [](const DeviceTable& t, const py::bytes& req) {
             std::string out;
             const bool ok = t.allocate(std::string_view(PyBytes_AS_STRING(req.ptr()), PyBytes_GET_SIZE(req.ptr())), &out);
             return ok_bytes(ok, out);
           })
      .def("preferred",
           [](const DeviceTable& t, const py::bytes& req) {
             std::string out;
             const bool ok = t.preferred(std::string_view(PyBytes_AS_STRING(req.ptr()), PyBytes_GET_SIZE(req.ptr())), &out);
             return ok_bytes(ok, out);
           })
      .def("preferred_ids",
           [](const DeviceTable& t, const std::vector<std::string>& avail, const std::vector<std::string>& must,
              int size) {
             std::vector<std::string> ids;
             AllocResult r = t.preferred_ids(avail, must, size, &ids);
             if (!r.ok) throw std::runtime_error(r.error);
             return ids;
           })
      .def("observe", &DeviceTable::observe)
      .def("render_metrics", [](const DeviceTable& t) {
        std::string s;
        t.render_metrics(&s, true);
        return s;
      });

  // ---- health ----
  py::class_<HealthUpdate>(m, "HealthUpdate")
      .def_readonly("ts_ns", &HealthUpdate::ts_ns)
      .def_readonly("kind", &HealthUpdate::kind)
      .def_readonly("gpu", &HealthUpdate::gpu)
      .def_readonly("partition", &HealthUpdate::partition)
      .def_readonly("healthy", &HealthUpdate::healthy)
      .def_readonly("peer", &HealthUpdate::peer)
      .def_readonly("link_up", &HealthUpdate::link_up)
      .def_readonly("reason", &HealthUpdate::reason)
      .def_readonly("key", &HealthUpdate::key)
      .def_readonly("link_gbps", &HealthUpdate::link_gbps)
      .def_readonly("peer_key", &HealthUpdate::peer_key)
      .def("__repr__", [](const HealthUpdate& u) {
        return "<HealthUpdate " + std::string(event_kind_name(u.kind)) + " gpu=" + std::to_string(u.gpu) +
               " healthy=" + std::to_string(u.healthy) + " " + u.reason + ">";
      });

  py::class_<HealthLatch>(m, "HealthLatch")
      .def(py::init<>())
      .def(py::init([](std::string key, int64_t last_ue, double fw_boot_s, std::string reason, int64_t since_ns) {
             HealthLatch l;
             l.key = std::move(key);
             l.ecc_bad = true;
             l.last_ue = last_ue;
             l.fw_boot_s = fw_boot_s;
             l.reason = std::move(reason);
             l.since_ns = since_ns;
             return l;
           }),
           py::arg("key"), py::arg("last_ue") = -1,
           py::arg("fw_boot_s") = std::numeric_limits<double>::quiet_NaN(), py::arg("reason") = "",
           py::arg("since_ns") = 0)
      .def_readwrite("key", &HealthLatch::key)
      .def_readwrite("ecc_bad", &HealthLatch::ecc_bad)
      .def_readwrite("last_ue", &HealthLatch::last_ue)
      .def_readwrite("fw_boot_s", &HealthLatch::fw_boot_s)
      .def_readwrite("reason", &HealthLatch::reason)
      .def_readwrite("since_ns", &HealthLatch::since_ns);
  m.def("boottime_s", &boottime_s);

  py::class_<HealthMonitor, std::shared_ptr<HealthMonitor>>(m, "HealthMonitor")
      .def(py::init<std::shared_ptr<Backend>, int>(), py::arg("backend"), py::arg("lost_after_failures") = 3)
      .def("set_gpu_count", &HealthMonitor::set_gpu_count, py::call_guard<py::gil_scoped_release>())
      .def("set_gpus", &HealthMonitor::set_gpus, py::call_guard<py::gil_scoped_release>())
      .def("unhealthy_keys", &HealthMonitor::unhealthy_keys)
      .def("start", &HealthMonitor::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &HealthMonitor::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &HealthMonitor::running)
      .def("process", &HealthMonitor::process, py::call_guard<py::gil_scoped_release>())
      .def("pop", &HealthMonitor::pop, py::call_guard<py::gil_scoped_release>(), py::arg("timeout_ms") = 200)
      .def("gpu_healthy", &HealthMonitor::gpu_healthy)
      .def("set_fast_tables", &HealthMonitor::set_fast_tables)
      .def("set_fast_recover", &HealthMonitor::set_fast_recover)
      .def("set_disabled_checks", &HealthMonitor::set_disabled_checks, py::call_guard<py::gil_scoped_release>())
      .def("attach_tables", &HealthMonitor::attach_tables, py::arg("tables"), py::arg("fast_recover"),
           py::arg("held_unhealthy"), py::call_guard<py::gil_scoped_release>())
      .def("set_bad_page_thresholds", &HealthMonitor::set_bad_page_thresholds)
      .def("set_pcie_floor", &HealthMonitor::set_pcie_floor, py::arg("min_width"), py::arg("min_gts"),
           py::arg("debounce") = 1, py::call_guard<py::gil_scoped_release>())
      .def("on_sample", &HealthMonitor::on_sample, py::arg("gpu"), py::arg("ok"), py::arg("sample"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("events_seen", &HealthMonitor::events_seen)
      .def("latches", &HealthMonitor::latches)
      .def("restore_latches", &HealthMonitor::restore_latches, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("resets_observed", &HealthMonitor::resets_observed)
      .def_property_readonly("reset_candidates", &HealthMonitor::reset_candidates)
      .def_property_readonly("fw_clock_glitches", &HealthMonitor::fw_clock_glitches)
      .def("clear_latches", &HealthMonitor::clear_latches, py::arg("key"), py::arg("reason"),
           py::call_guard<py::gil_scoped_release>())
      .def("holds", &HealthMonitor::holds, py::arg("key"))
      .def("set_held_partitions", &HealthMonitor::set_held_partitions, py::arg("held"),
           py::call_guard<py::gil_scoped_release>());

  // ---- exporter ----
  py::class_<PartitionLabel>(m, "PartitionLabel")
      .def(py::init([](int gpu, int partition, const std::string& device_id, const std::string& resource,
                       const std::string& hip_ids) {
             PartitionLabel l;
             l.gpu = gpu;
             l.partition = partition;
             l.device_id = device_id;
             l.resource = resource;
             l.hip_ids = hip_ids;
             return l;
           }),
           py::arg("gpu"), py::arg("partition"), py::arg("device_id"), py::arg("resource"), py::arg("hip_ids") = "");

  py::class_<Exporter, std::shared_ptr<Exporter>>(m, "Exporter")
      .def("set_stall_ms", &Exporter::set_stall_ms)
      .def("set_idle_interval", &Exporter::set_idle_interval, py::arg("idle_ms"), py::arg("window_ms"))
      .def_property_readonly("current_interval_ms", &Exporter::current_interval_ms)
      .def_property_readonly("idle_passes", &Exporter::idle_passes)
      .def_property_readonly("stalled_gpu", &Exporter::stalled_gpu)
      .def_property_readonly("stalled_gpus", &Exporter::stalled_gpus)
      .def_property_readonly("blocked_gpus", &Exporter::blocked_gpus)
      .def("sample_age_s", &Exporter::sample_age_s)
      .def(py::init<>())
      .def("set_inventory", &Exporter::set_inventory)
      .def("set_partition_labels", &Exporter::set_partition_labels)
      .def("set_build_info", &Exporter::set_build_info)
      .def("set_tables", &Exporter::set_tables)
      .def("set_extra", &Exporter::set_extra)
      .def("start", &Exporter::start, py::arg("backend"), py::arg("interval_ms"), py::arg("monitor") = nullptr,
           py::call_guard<py::gil_scoped_release>())
      .def("stop", &Exporter::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &Exporter::running)
      .def("sample_once", [](Exporter& e) { e.sample_once(0); }, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("samples_total", &Exporter::samples_total)
      .def("last_sample", &Exporter::last_sample)
      .def("render", [](const Exporter& e) {
        std::string s;
        {
          py::gil_scoped_release rel;
          e.render(&s);
        }
        return s;
      });

  // ---- http ----
  py::class_<HttpConfig>(m, "HttpConfig")
      .def(py::init<>())
      .def_readwrite("host", &HttpConfig::host)
      .def_readwrite("port", &HttpConfig::port)
      .def_readwrite("threads", &HttpConfig::threads)
      .def_readwrite("access_log", &HttpConfig::access_log)
      .def_readwrite("idle_timeout_s", &HttpConfig::idle_timeout_s)
      .def_readwrite("read_timeout_s", &HttpConfig::read_timeout_s)
      .def_readwrite("busy_poll_us", &HttpConfig::busy_poll_us)
      .def_readwrite("restart_local_only", &HttpConfig::restart_local_only)
      .def_readwrite("clear_local_only", &HttpConfig::clear_local_only)
      .def_readwrite("version", &HttpConfig::version);

  py::class_<HttpServer, std::shared_ptr<HttpServer>>(m, "HttpServer")
      .def(py::init<HttpConfig, std::shared_ptr<Exporter>>())
      .def("start", &HttpServer::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &HttpServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &HttpServer::running)
      .def_property_readonly("port", &HttpServer::port)
      .def_property_readonly("requests_total", &HttpServer::requests_total)
      .def_property_readonly("shed_connections", &HttpServer::shed_connections)
      .def_property_readonly("worker_connections", &HttpServer::worker_connections)
      .def("render_http_metrics", [](const HttpServer& s) {
        std::string o;
        s.render_http_metrics(&o);
        return o;
      })
      .def("set_ready", &HttpServer::set_ready, py::arg("ready"), py::arg("reason") = "")
      .def("set_restart_hook", [](HttpServer& s, py::object fn) {
        if (fn.is_none()) {
          s.set_restart_hook(nullptr);
          return;
        }
        // keep the callable alive; destroy it only while holding the GIL
        auto holder = std::shared_ptr<py::object>(new py::object(fn), [](py::object* o) {
          py::gil_scoped_acquire g;
          delete o;
        });
        s.set_restart_hook([holder]() {
          py::gil_scoped_acquire g;
          try {
            (*holder)();
          } catch (py::error_already_set& e) {
            e.discard_as_unraisable("restart hook");
          }
        });
      })
      .def("set_clear_hook", [](HttpServer& s, py::object fn) {
        // fn(query: str) -> (status: int, body: str); GET /health/clear
        if (fn.is_none()) {
          s.set_clear_hook(nullptr);
          return;
        }
        auto holder = std::shared_ptr<py::object>(new py::object(fn), [](py::object* o) {
          py::gil_scoped_acquire g;
          delete o;
        });
        s.set_clear_hook([holder](const std::string& query) -> std::pair<int, std::string> {
          py::gil_scoped_acquire g;
          try {
            auto r = (*holder)(query).cast<std::pair<int, std::string>>();
            return r;
          } catch (py::error_already_set& e) {
            e.discard_as_unraisable("health clear hook");
          } catch (const std::exception&) {
          }
          return {500, "{\"message\":\"Internal Server Error\"}\n"};
        });
      });

  // ---- fs watch ----
  py::class_<DirWatcher, std::shared_ptr<DirWatcher>>(m, "DirWatcher")
      .def(py::init<const std::string&>())
      .def("read",
           [](DirWatcher& w, int timeout_ms) {
             std::vector<FsEvent> evs;
             {
               py::gil_scoped_release rel;
               evs = w.read(timeout_ms);
             }
             py::list out;
             for (auto& e : evs) out.append(py::make_tuple(e.name, e.mask, e.create(), e.remove()));
             return out;
           },
           py::arg("timeout_ms") = 200)
      .def("close", &DirWatcher::close)
      .def("wake", &DirWatcher::wake)
      .def_property_readonly("dir", &DirWatcher::dir);

  // ---- native gRPC (HTTP/2) server + client ----
  py::class_<GrpcServer, std::shared_ptr<GrpcServer>>(m, "GrpcServer")
      .def(py::init<std::string, int, int, int>(), py::arg("socket_path"), py::arg("threads") = 2,
           py::arg("busy_poll_us") = 0, py::arg("admission_poll_us") = 0)
      .def("set_table", &GrpcServer::set_table, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("table_swaps", &GrpcServer::table_swaps)
      .def("set_call_trace", &GrpcServer::set_call_trace, py::arg("path"), py::arg("capacity") = 65536)
      .def("set_idle_wake_ms", &GrpcServer::set_idle_wake_ms, py::arg("ms"))
      .def("set_active_window_ms", &GrpcServer::set_active_window_ms, py::arg("ms"))
      .def("set_peek_reads", &GrpcServer::set_peek_reads, py::arg("on"))
      .def("set_poll_gap_ns", &GrpcServer::set_poll_gap_ns, py::arg("ns"))
      .def("set_core_escape", &GrpcServer::set_core_escape, py::arg("on"))
      .def_property_readonly("core_escapes", &GrpcServer::core_escapes)
      .def_property_readonly("idle_wakeups", &GrpcServer::idle_wakeups)
      .def("add_table", &GrpcServer::set_table)
      .def("start", &GrpcServer::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &GrpcServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("notify", &GrpcServer::notify)
      .def_property_readonly("running", &GrpcServer::running)
      .def_property_readonly("requests", &GrpcServer::requests)
      .def_property_readonly("shed_connections", &GrpcServer::shed_connections)
      .def_property_readonly("admission_windows", &GrpcServer::admission_windows)
      .def_property_readonly("poll_windows_yielded", &GrpcServer::poll_windows_yielded)
      .def_property_readonly("connections", &GrpcServer::connections)
      .def("list_and_watch_streams", &GrpcServer::list_and_watch_streams, py::call_guard<py::gil_scoped_release>())
      .def("list_and_watch_closed_at", &GrpcServer::list_and_watch_closed_at)
      .def("set_failure_hook", &GrpcServer::set_failure_hook, py::arg("hook"))
      .def_property_readonly("worker_connections", &GrpcServer::worker_connections)
      .def_property_readonly("socket_path", &GrpcServer::socket_path)
      .def("failure", &GrpcServer::failure, py::call_guard<py::gil_scoped_release>())
      .def("inject_fault", &GrpcServer::inject_fault)
      .def("set_keep_warm_ms", &GrpcServer::set_keep_warm_ms)
      .def("set_keep_warm_full", &GrpcServer::set_keep_warm_full)
      .def_property_readonly("warm_ticks", &GrpcServer::warm_ticks);

  py::class_<H2Client>(m, "H2Client")
      .def(py::init<std::string, double>(), py::arg("socket_path"), py::arg("timeout_s") = 5.0,
           py::call_guard<py::gil_scoped_release>())
      .def("unary",
           [](H2Client& c, const std::string& path, const py::bytes& req) {
             std::string r(req), resp, msg;
             int st;
             {
               py::gil_scoped_release rel;
               st = c.unary(path, r, &resp, &msg);
             }
             return py::make_tuple(st, py::bytes(resp), msg);
           })
      .def("first_stream_message",
           [](H2Client& c, const std::string& path, const py::bytes& req) {
             std::string r(req), resp;
             {
               py::gil_scoped_release rel;
               c.first_stream_message(path, r, &resp);
             }
             return py::bytes(resp);
           })
      .def("open_stream",
           [](H2Client& c, const std::string& path, const py::bytes& req) {
             std::string r(req);
             py::gil_scoped_release rel;
             c.open_stream(path, r);
           })
      .def(
          "next_stream_message",
          [](H2Client& c, double timeout_s) -> py::object {
            std::string resp;
            int st;
            {
              py::gil_scoped_release rel;
              st = c.next_stream_message(&resp, static_cast<int>(timeout_s * 1000));
            }
            if (st != 0) return py::none();
            return py::bytes(resp);
          },
          py::arg("timeout_s") = 5.0)
      .def("close", &H2Client::close);

  m.def("format_float", [](double v) {  // Prometheus number formatting (exposed for tests)
    std::string s;
    append_float(&s, v);
    return s;
  });
  // hpack (exposed for tests)
  m.def("hpack_huffman_encode", [](const std::string& s) {
    std::string o;
    hpack::huffman_encode(s, &o);
    return py::bytes(o);
  });
  m.def("hpack_huffman_decode", [](const py::bytes& b) -> py::object {
    std::string in(b), out;
    if (!hpack::huffman_decode(reinterpret_cast<const uint8_t*>(in.data()), in.size(), &out)) return py::none();
    return py::bytes(out);
  });
  m.def("hpack_huffman_decode_bitwise", [](const py::bytes& b) -> py::object {
    std::string in(b), out;
    if (!hpack::huffman_decode_bitwise(reinterpret_cast<const uint8_t*>(in.data()), in.size(), &out))
      return py::none();
    return py::bytes(out);
  });
  py::class_<hpack::Decoder>(m, "HpackDecoder")
      .def(py::init<size_t>(), py::arg("max_table_size") = 4096)
      .def("decode",
           [](hpack::Decoder& d, const py::bytes& b) -> py::object {
             std::string in(b);
             std::vector<hpack::Header> hs;
             if (!d.decode(reinterpret_cast<const uint8_t*>(in.data()), in.size(), &hs)) return py::none();
             py::list l;
             for (auto& h : hs) l.append(py::make_tuple(h.name, h.value));
             return l;
           })
      .def("decode_visit",  // the server's non-allocating path; same result contract as decode
           [](hpack::Decoder& d, const py::bytes& b) -> py::object {
             std::string in(b);
             std::vector<std::pair<std::string, std::string>> hs;
             auto fn = [](void* ctx, std::string_view name, std::string_view value) {
               static_cast<std::vector<std::pair<std::string, std::string>>*>(ctx)->emplace_back(name, value);
             };
             if (!d.decode(reinterpret_cast<const uint8_t*>(in.data()), in.size(), fn, &hs)) return py::none();
             py::list out;
             for (auto& h : hs) out.append(py::make_tuple(h.first, h.second));
             return out;
           })
      .def_property_readonly("table_size", &hpack::Decoder::table_size)
      .def_property_readonly("table_entries", &hpack::Decoder::table_entries);

  // ---- whole-process CPU sampling profiler (benchmark: true) ----
  m.def("prof_start", &prof::start, py::arg("hz") = 997);
  m.def("prof_stop", &prof::stop);
  m.def("prof_running", &prof::running);
  m.def("prof_dropped", &prof::dropped);
  m.def("prof_histogram", []() {
    py::list out;  // (module, offset, exported symbol or "", samples)
    for (const auto& kv : prof::histogram()) {
      std::string path, sym;
      uintptr_t base = 0;
      if (prof::module_of(kv.first, &path, &base, &sym))
        out.append(py::make_tuple(path, static_cast<uint64_t>(kv.first - base), sym, kv.second));
      else
        out.append(py::make_tuple(std::string("?"), static_cast<uint64_t>(kv.first), std::string(), kv.second));
    }
    return out;
  });
}
