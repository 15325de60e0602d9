"""The /metrics contract: every metric family the plugin exposes.

The reference's ``metrics`` package is empty (``metrics/metrics.go:1``); its /metrics
carries only the Go runtime/process collectors, ``go_build_info`` (``main.go:26-28``)
and the echo HTTP families (``middleware/echo_metric.go:80-93``).  This registry is the
single place that documents the MI355X plugin's families;
``tests/test_topology_model.py::test_metrics_contract_both_ways``
checks the native exporter against it in both directions.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Family:
    name: str
    type: str
    labels: tuple
    source: str
    help: str


GPU = ("gpu",)
PART = ("gpu", "partition", "device_id", "resource")

FAMILIES = (
    # --- reference-compatible ---
    Family("echo_http_requests_total", "counter", ("handler", "method", "status"), "httpd",
           "Number of HTTP operations (reference middleware/echo_metric.go)"),
    Family("echo_http_request_duration_seconds", "histogram", ("handler", "method"), "httpd",
           "Spend time by processing a route; buckets .0005..30 s as the reference"),
    Family("k8s_gpu_device_plugin_build_info", "gauge", ("app", "version", "python", "native"), "manager",
           "Build information (the go_build_info analogue)"),
    Family("process_cpu_seconds_total", "counter", (), "exporter", "Process CPU time"),
    Family("process_resident_memory_bytes", "gauge", (), "exporter", "Resident memory"),
    Family("process_virtual_memory_bytes", "gauge", (), "exporter", "Virtual memory"),
    Family("process_open_fds", "gauge", (), "exporter", "Open file descriptors"),
    Family("process_max_fds", "gauge", (), "exporter", "File descriptor limit"),
    Family("process_start_time_seconds", "gauge", (), "exporter", "Process start time"),
    # --- per-GPU amdsmi telemetry ---
    Family("amdgpu_info", "gauge", GPU + ("uuid", "bdf", "name", "gfx_target", "compute_partition",
                                          "memory_partition", "numa_node", "driver_version", "vbios_version",
                                          "oam_id"), "exporter",
           "Static inventory (value 1); `oam_id` is the baseboard slot (-1 unknown)"),
    Family("amdgpu_telemetry_up", "gauge", GPU, "exporter", "Last sample succeeded"),
    Family("amdgpu_power_watts", "gauge", GPU, "exporter", "Socket power"),
    Family("amdgpu_energy_joules_total", "counter", GPU, "exporter", "Accumulated energy"),
    Family("amdgpu_gfx_activity_percent", "gauge", GPU, "exporter", "Compute engine activity"),
    Family("amdgpu_umc_activity_percent", "gauge", GPU, "exporter", "HBM controller activity"),
    Family("amdgpu_vram_used_bytes", "gauge", GPU, "exporter", "VRAM used"),
    Family("amdgpu_vram_total_bytes", "gauge", GPU, "exporter", "VRAM capacity"),
    Family("amdgpu_throttle_status", "gauge", GPU, "exporter", "Throttle status bitmask"),
    Family("amdgpu_xgmi_link_width", "gauge", GPU, "exporter", "Current xGMI link width, lanes (16 when fully trained)"),
    Family("amdgpu_xgmi_link_speed_gbps", "gauge", GPU, "exporter", "Current xGMI per-lane rate (38 Gb/s on MI355X)"),
    Family("amdgpu_xgmi_error_status", "gauge", GPU, "exporter", "xGMI error state: 0 none, 1 an error, 2 multiple"),
    Family("amdgpu_pcie_link_width", "gauge", GPU, "exporter", "Current PCIe link width to the host, lanes"),
    Family("amdgpu_pcie_link_speed_gtps", "gauge", GPU, "exporter", "Current PCIe link rate to the host, GT/s"),
    Family("amdgpu_pcie_replays_total", "counter", GPU, "exporter", "PCIe replays on the host link"),
    Family("amdgpu_pcie_recoveries_total", "counter", GPU, "exporter", "PCIe L0 -> recovery transitions"),
    Family("amdgpu_temperature_celsius", "gauge", GPU + ("sensor",), "exporter",
           "Temperature by sensor: edge, hotspot, mem, hbm0..N"),
    Family("amdgpu_clock_mhz", "gauge", GPU + ("clock",), "exporter", "gfx / mem clocks"),
    Family("amdgpu_ecc_errors_total", "counter", GPU + ("type",), "exporter", "ECC (un)correctable counts"),
    Family("amdgpu_retired_pages", "gauge", GPU + ("status",), "exporter",
           "RAS retired HBM pages: reserved / pending / unreservable"),
    Family("amdgpu_retired_pages_threshold", "gauge", GPU, "exporter",
           "Retired + pending pages that make the GPU Unhealthy (health.badPageThreshold or the GPU's RAS threshold)"),
    Family("amdgpu_xgmi_link_up", "gauge", GPU + ("link", "peer"), "exporter", "xGMI link to peer is up"),
    Family("amdgpu_xgmi_read_bytes_total", "counter", GPU + ("link", "peer"), "exporter", "xGMI bytes received"),
    Family("amdgpu_xgmi_write_bytes_total", "counter", GPU + ("link", "peer"), "exporter", "xGMI bytes sent"),
    Family("amdgpu_xgmi_link_bitrate_gbps", "gauge", GPU + ("link", "peer"), "exporter",
           "Per-lane signalling rate (38 on MI355X); a link trained slower than its peers is degraded"),
    Family("amdgpu_xgmi_link_bandwidth_gbps", "gauge", GPU + ("link", "peer"), "exporter",
           "Trained link bandwidth: current per-lane rate x current link width (608 Gb/s on a healthy MI355X link)"),
    # --- per-partition ---
    Family("amdgpu_partition_info", "gauge", PART + ("hip_ids",), "exporter",
           "Partition -> device id / resource / the host HIP ordinals it spans (value 1)"),
    Family("amdgpu_partition_gfx_busy_percent", "gauge", PART + ("source",), "exporter",
           "Per-partition compute busy; source=partition_metrics (the partition's own metrics table) or "
           "xcp_stats (the socket blob, fallback)"),
    Family("amdgpu_partition_profile_supported", "gauge",
           ("gpu", "profile", "partitions", "memory_partition", "source"), "exporter",
           "Compute partition profile x memory mode the GPU supports (1); source=driver (the driver's "
           "profile list, needs root) or current (only the current profile was readable)"),
    Family("amdgpu_partition_vram_used_bytes", "gauge", PART, "exporter", "Per-partition VRAM used"),
    # --- sampler / plugin ---
    Family("amdgpu_telemetry_samples_total", "counter", (), "exporter", "Sampling passes"),
    Family("amdgpu_telemetry_sample_errors_total", "counter", (), "exporter", "Per-GPU sample failures"),
    Family("amdgpu_telemetry_sample_duration_seconds", "histogram", (), "exporter", "One sampling pass"),
    Family("amdgpu_telemetry_interval_seconds", "gauge", (), "exporter",
           "The sampler's current period: telemetry.intervalMs, or telemetry.idleIntervalMs while nothing "
           "reads the GPU metrics and health is settled"),
    Family("amdgpu_telemetry_last_pass_age_seconds", "gauge", (), "exporter",
           "Seconds since the sampler last completed a pass (passes go on while one GPU's call hangs: "
           "it holds that GPU's lane only)"),
    Family("amdgpu_telemetry_sample_age_seconds", "gauge", ("gpu",), "exporter",
           "Seconds since the GPU's last successful sample (grows for a GPU whose call hangs; the others "
           "stay fresh)"),
    Family("amdgpu_telemetry_sample_stalled", "gauge", ("gpu",), "exporter",
           "1 while a hardware call of the GPU (sample, describe, arm) has been in flight longer than "
           "health.sampleStallS (the GPU is then marked lost)"),
    Family("amdgpu_telemetry_sample_blocked", "gauge", ("gpu",), "exporter",
           "1 while the GPU's call is stuck behind another GPU's stalled call (no call has completed "
           "since: the library serialises devices); the GPU is not marked lost for it"),
    Family("amdgpu_device_plugin_device_health", "gauge", ("resource", "device_id"), "exporter",
           "1 Healthy / 0 Unhealthy per advertised device"),
    Family("amdgpu_device_plugin_rpc_duration_seconds", "histogram", ("resource", "rpc"), "device_table",
           "kubelet RPC latency (5 us .. 1 s buckets)"),
    Family("amdgpu_device_plugin_events_total", "counter", ("event",), "manager",
           "Lifecycle events: restarts (api/kubelet/retry), registrations, load failures, health events; "
           "reloads and `table_swaps` (hitless reloads), `resets_observed` (GPU resets seen by polling: the "
           "kernel's reset count, a confirmed firmware clock restart, a UE counter started over), "
           "`reset_candidates` (back from a telemetry outage with no reset confirmed), `latches_cleared_verified` "
           "(a candidate the recovery canary passed), `health_clears` (`GET /health/clear`), `fw_clock_glitches` "
           "(firmware clock readings that went back without being a restart), `latches_restored`, `state_writes` "
           "/ `state_write_errors` (`health.stateFile`), start-up canary runs and skips, "
           "`reregistrations_stream_lost` (kubelet ended a ListAndWatch stream), `reregistrations_restart` (a "
           "`/restart` registered a kept plugin again), `stream_watch_socket_taken` (another instance bound the "
           "socket path), `devices_index_conflicts` / `devices_index_reresolved`"),
    Family("amdgpu_device_plugin_devices", "gauge", ("resource", "health"), "manager",
           "Advertised devices per resource and health"),
    Family("amdgpu_device_plugin_registered", "gauge", ("resource",), "manager",
           "Resource registered with kubelet"),
    Family("amdgpu_device_plugin_ready", "gauge", (), "manager",
           "1 if every resource with devices is registered with kubelet (GET /ready)"),
    Family("amdgpu_device_plugin_health_event_sources", "gauge", (), "manager",
           "GPUs whose hardware event notification (reset, thermal, VM fault) is armed; 0 with GPUs "
           "advertised means resets are only seen as failed telemetry (no /dev/kfd access)"),
    # --- gfx950 canary (health.canary / canaryOnStart / canaryOnPreStart) ---
    Family("amdgpu_canary_last_run_timestamp_seconds", "gauge", ("gpu", "partition"), "manager",
           "Unix time of the partition's last canary run"),
    Family("amdgpu_canary_last_ok", "gauge", ("gpu", "partition"), "manager",
           "1 if the last canary run passed (exact results and the configured performance floors)"),
    Family("amdgpu_canary_errors", "gauge", ("gpu", "partition", "check"), "manager",
           "Mismatches found by the last run: hbm, mfma, gemm, lowp (fp8/bf8/fp4 MFMA), lds"),
    Family("amdgpu_canary_hbm_gbps", "gauge", ("gpu", "partition", "direction"), "manager",
           "HBM bandwidth of the last run: write, read (read + verify)"),
    Family("amdgpu_canary_matrix_tflops", "gauge", ("gpu", "partition", "path"), "manager",
           "Dense matrix-core rate of the last run: mfma_bf16, gemm_bf16 (LDS-staged GEMM), mxfp8, mxfp4"),
    # --- kubelet PodResources (podResources.enabled) ---
    Family("amdgpu_device_plugin_allocation_info", "gauge", ("resource", "device_id", "namespace", "pod", "container"),
           "manager", "Advertised device held by a container (value 1)"),
    Family("amdgpu_device_plugin_pod_resources_up", "gauge", (), "manager",
           "Last kubelet PodResources List succeeded"),
    Family("amdgpu_xgmi_link_pods", "gauge", ("gpu", "peer"), "manager",
           "Multi-GPU pods whose devices span the GPU pair, sharing its xGMI link (the allocator steers new pods off it)"),
)

BY_NAME = {f.name: f for f in FAMILIES}


def family_of(sample_name: str) -> Family | None:
    """Maps a sample name (``x_bucket``/``x_sum``/``x_count``/``x``) to its family."""
    if sample_name in BY_NAME:
        return BY_NAME[sample_name]
    for suffix in ("_bucket", "_sum", "_count"):
        if sample_name.endswith(suffix) and sample_name[: -len(suffix)] in BY_NAME:
            return BY_NAME[sample_name[: -len(suffix)]]
    return None


PROMQL_EXAMPLES = (
    ("Socket power seen per advertised partition (join on the physical GPU)",
     "amdgpu_power_watts * on(gpu) group_right amdgpu_partition_info"),
    ("Hottest HBM stack per GPU", 'max by (gpu) (amdgpu_temperature_celsius{sensor=~"hbm.*"})'),
    ("Unhealthy advertised devices per resource", "count by (resource) (amdgpu_device_plugin_device_health == 0)"),
    ("Allocate p99 over 5 minutes",
     'histogram_quantile(0.99, sum by (le) (rate(amdgpu_device_plugin_rpc_duration_seconds_bucket{rpc="Allocate"}[5m])))'),
    ("Down xGMI links", "amdgpu_xgmi_link_up == 0"),
    ("xGMI links trained slower than the node's fastest link",
     "amdgpu_xgmi_link_bitrate_gbps < on() group_left max(amdgpu_xgmi_link_bitrate_gbps)"),
    ("Partition busy per workload (podResources.enabled)",
     "amdgpu_partition_gfx_busy_percent * on(device_id) group_left(namespace, pod, container) "
     "amdgpu_device_plugin_allocation_info"),
    ("Partitions whose last canary ran below 90% of the node's best bf16 MFMA rate",
     'amdgpu_canary_matrix_tflops{path="mfma_bf16"} < on() group_left 0.9 * max(amdgpu_canary_matrix_tflops{path="mfma_bf16"})'),
    ("GPUs whose host PCIe link trained below the node's widest, or is replaying",
     "amdgpu_pcie_link_width < on() group_left max(amdgpu_pcie_link_width) or rate(amdgpu_pcie_replays_total[5m]) > 0"),
    ("xGMI traffic per link (bytes/s)", "rate(amdgpu_xgmi_read_bytes_total[1m]) + rate(amdgpu_xgmi_write_bytes_total[1m])"),
)


def markdown() -> str:
    """docs/METRICS.md, generated from FAMILIES (tests keep the file in sync)."""
    out = ["# /metrics reference", "",
           "Generated by `python -m k8s_gpu_device_plugin_amd.metrics.families`. Do not edit by hand.",
           "`tests/test_topology_model.py` checks this list against a live exporter in both",
           "directions.", "",
           "| Family | Type | Labels | Source | Meaning |", "|---|---|---|---|---|"]
    for f in FAMILIES:
        out.append("| `%s` | %s | %s | %s | %s |" % (f.name, f.type, ", ".join("`%s`" % x for x in f.labels) or "—",
                                                  f.source, f.help))
    out += ["", "## PromQL examples", ""]
    for title, q in PROMQL_EXAMPLES:
        out += ["%s:" % title, "", "```promql", q, "```", ""]
    return "\n".join(out)


if __name__ == "__main__":
    print(markdown(), end="")
