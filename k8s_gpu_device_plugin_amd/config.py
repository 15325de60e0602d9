"""Configuration: YAML file + defaults + environment overrides, validated early.

Reference: ``config/config.go:9-22`` (struct + viper defaults), ``config.yml:1-13``,
``main.go:31-52`` (``--configFile`` flag, ``./<name>.yml`` lookup, non-fatal read
error).  Kept: the same keys (``webListenAddress``, ``migStrategy``, ``benchmark``,
``log.level``, ``log.fileDir``) and file lookup.  Fixed: D11 (code default listen
address ``"9002"`` has no colon -> ``0.0.0.0:9100``), strategy validated at load
time instead of deep inside device-map building (§5.6).  Added keys for the MI355X
build (plugin dir, backend, partition/resource options, telemetry, health, servers).

Environment overrides: ``AMDGPU_DP_<UPPER_SNAKE_KEY>`` for top-level scalars, e.g.
``AMDGPU_DP_WEB_LISTEN_ADDRESS=127.0.0.1:0``, ``AMDGPU_DP_BACKEND=fixture``.
"""
from __future__ import annotations

import copy
import dataclasses
import os
import re
from dataclasses import dataclass, field
from typing import Any

from .api import v1beta1

STRATEGIES = ("none", "single", "mixed")
# health.disabledChecks names -> the native HealthCheck bits (native/health.h)
HEALTH_CHECKS = {"reset": 1, "ecc": 2, "lost": 4, "retiredpages": 8, "pcie": 16}


def disabled_checks_mask(value: str) -> int:
    mask = 0
    for name in str(value or "").replace(";", ",").split(","):
        name = name.strip().lower()
        if not name:
            continue
        if name == "all":
            mask |= sum(HEALTH_CHECKS.values())
        elif name in HEALTH_CHECKS:
            mask |= HEALTH_CHECKS[name]
        else:
            raise ConfigError("health.disabledChecks: unknown check %r (want %s or all)"
                              % (name, ", ".join(["reset", "ecc", "lost", "retiredPages", "pcie"])))
    return mask


@dataclass
class LogConfig:
    level: str = "debug"
    fileDir: str = "./logs"
    console: bool = True
    maxAgeDays: float = 30.0   # rotated files older than this are deleted (lumberjack MaxAge; 0 = keep)


@dataclass
class ResourceSpec:
    pattern: str = "*"
    name: str = "gpu"


@dataclass
class SharingConfig:
    replicas: int = 1            # >1: advertise "<id>::<n>" time-sliced replicas
    renameByDefault: bool = False  # rename amd.com/gpu -> amd.com/gpu.shared when shared


@dataclass
class TelemetryConfig:
    enabled: bool = True
    intervalMs: int = 1000
    # while nothing has read the GPU metrics (/metrics) for activeWindowS and every GPU's
    # health is settled, sample every idleIntervalMs instead (0 = never slow down); the
    # first read after that wakes the sampler, and while scraped it samples about twice
    # per scrape interval, between intervalMs and idleIntervalMs
    idleIntervalMs: int = 5000
    activeWindowS: float = 120.0


@dataclass
class HealthConfig:
    enabled: bool = True
    lostAfterFailures: int = 3
    canary: bool = False          # gfx950 canary before re-advertising a GPU after a reset
    canaryOnStart: bool = False   # ... and on every partition before the first advertisement
    canaryOnPreStart: bool = False  # pre_start_required: canary the allocated partitions before each container
    canaryBytes: int = 256 << 20
    canaryTimeoutS: float = 120.0
    # performance floors of a canary run (0 = off): a partition whose HBM write or
    # read+verify bandwidth, or whose bf16 MFMA rate, comes out below them fails the
    # canary like a wrong result does (thermal or power throttling, a degraded HBM stack)
    canaryMinHbmGbps: float = 0.0
    canaryMinTflops: float = 0.0
    rejectUnhealthyAllocate: bool = True
    # retired + pending HBM pages at which a GPU goes Unhealthy: 0 = the GPU's own RAS
    # threshold when readable (root), -1 = never, N > 0 = N
    badPageThreshold: int = 0
    # host PCIe link floor: a GPU whose link trained narrower / slower is Unhealthy until it
    # trains back (0 = no floor; e.g. 16 and 32 for an x16 Gen5 MI355X slot)
    pcieMinWidth: int = 0
    pcieMinSpeedGTs: float = 0.0
    # consecutive telemetry samples below (at or above) the PCIe floor that degrade
    # (restore) a GPU: one reading of a link in a power-saving state flaps nothing
    pcieDebounceSamples: int = 3
    # health checks that no longer make a GPU Unhealthy (still logged): comma list or
    # YAML list of reset, ecc, lost, retiredPages, or all (env AMDGPU_DP_DISABLE_HEALTHCHECKS)
    disabledChecks: str = ""
    # a telemetry (amdsmi) call of one GPU in flight for longer than this marks the GPU
    # lost: a wedged driver never returns an error to count (0 = off)
    sampleStallS: float = 10.0
    # every hardware call of one GPU runs on that GPU's lane and is waited for at most this
    # long; a discovery gives a GPU that does not answer in time its last known description
    # (or leaves it out) and reports it on GET /ready
    discoveryTimeoutS: float = 10.0
    # Health latches that must survive a plugin restart (uncorrectable ECC, failed canaries),
    # keyed by GPU identity and the host's boot id: "auto" = <pluginDir>/.amdgpu-device-plugin/
    # health-state.json (kubelet removes only sockets from that directory), a path, or "" /
    # "none" = in memory only
    stateFile: str = "auto"
    # read each GPU's kernel reset count through an amdgpu context on its render node (no
    # privileges; needs the node in the container's device cgroup, e.g. deploy/kfd-cdi-patch
    # .yaml): a reset the driver performs - also one that keeps the GPU firmware running -
    # clears the uncorrectable-ECC latch without amdsmi event notification
    resetQuery: bool = True
    # amdsmi backend: re-read the ECC totals when the driver's RAS event state (fatal error,
    # poison creation / consumption) moved and every 30 s otherwise, instead of every sample
    # (the per-block reads query the firmware's error banks: ~0.27 ms of CPU per GPU per
    # sample on MI355X).  false = every sample, gated by the block files changing
    eccEventGate: bool = True


def state_file_path(cfg) -> str:
    """Where the health latches are persisted ("" = nowhere)."""
    v = str(cfg.health.stateFile or "").strip()
    if v.lower() in ("", "none", "off"):
        return ""
    if v.lower() == "auto":
        return os.path.join(cfg.pluginDir, ".amdgpu-device-plugin", "health-state.json")
    return v


@dataclass
class HttpConfig:
    threads: int = 2
    accessLog: bool = True
    server: str = "native"       # native | python
    busyPollUs: int = 50         # native server: keep polling this long after a request (0 = off)
    restartLocalOnly: bool = False  # GET /restart only from loopback peers (others: 403)
    # GET /health/clear?gpu=<uuid|bdf|index|device id> (an operator drops a GPU's health
    # latches) only from loopback peers (kubectl exec / port-forward); false = any peer
    healthClearLocalOnly: bool = True


@dataclass
class GrpcConfig:
    server: str = "native"       # native (C++ HTTP/2) | python (grpcio)
    threads: int = 4
    busyPollUs: int = 50         # native server: keep polling this long after a request (0 = off)
    admissionPollUs: int = 1000  # ... and this long after a GetPreferredAllocation (its Allocate follows)
    # native server: idle workers with a connection replay canned requests every keepWarmMs
    # (0 = off), so kubelet's sparse calls find that code and data cached
    keepWarmMs: int = 10
    # native server: a worker holding a connection wakes at least this often, doing nothing
    # (0 = off): keeps its core out of deep idle states, which is most of what a call after
    # a long idle pays, at half the CPU of a 1 ms keepWarmMs and without its collisions
    # with calls 1 ms apart (profiles/r5/idle_ab_wake.json, ab_wake_bench.jsonl)
    idleWakeMs: int = 1
    # native server: idleWakeMs and keepWarmMs run only this long after a worker's last
    # kubelet RPC (0 = always).  Outside this admission window the workers sleep: an idle
    # node pays ~1 wake-up per worker every 5 s for the plugin's gRPC server
    activeWindowMs: int = 10000
    # native server: read requests with MSG_PEEK and consume them after the answer is sent
    # (consuming the client's data wakes a client blocked in recv() for nothing).  Off: on
    # the MI355X box the deferred wake-up only moved into send() and the client then woke
    # from a deeper idle state - recv 0.21 vs 0.70 us, but send 0.85 vs 0.34 us and Allocate
    # p50 2.8-3.5 vs 2.55 us (profiles/r6/ab_peek_*.json)
    peekReads: bool = False
    # busy-poll spacing: PAUSE for this long between two empty polls (0 = one PAUSE)
    pollGapNs: int = 0
    # a worker whose calls in a busy-poll window run 35 % over its own best (another busy
    # hardware thread on its core, e.g. the client's) moves to another core of its L3
    coreEscape: bool = False
    keepWarmFull: bool = True    # ... through the whole request path of an in-memory connection (else HPACK + table)
    # native server: per-call trace of unary RPCs in a file-backed ring ("" = off), read by
    # bench.py to attribute slow calls; one record per call, callTraceEntries records
    callTraceFile: str = ""
    callTraceEntries: int = 65536


@dataclass
class PodResourcesConfig:
    enabled: bool = False        # poll kubelet's PodResources API -> allocation_info metric
    socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"
    intervalS: float = 10.0


@dataclass
class AllocatorConfig:
    # A multi-GPU container this plugin allocated counts as load on the xGMI links it
    # spans until the kubelet PodResources map shows it (podResources.enabled), or for
    # this long (0 = only the PodResources map).
    recentAllocationTtlS: float = 30.0


@dataclass
class Config:
    webListenAddress: str = "0.0.0.0:9100"
    migStrategy: str = "none"            # alias partitionStrategy (none|single|mixed)
    benchmark: bool = False
    benchmarkDir: str = ""
    log: LogConfig = field(default_factory=LogConfig)
    pluginDir: str = v1beta1.DEVICE_PLUGIN_PATH
    backend: str = "auto"                 # auto | amdsmi | fixture
    fixture: str = "2gpu_spx"             # builtin name or path, used by backend=fixture
    devices: str = ""                     # physical GPU filter: "0-3", UUIDs, BDFs, "hip:0-3" ("" = all)
    resourcePrefix: str = "amd.com"
    resources: list = field(default_factory=list)  # [ResourceSpec]
    visibleDevicesEnv: str = "AMD_VISIBLE_DEVICES"
    mountCardNodes: bool = False
    cdi: bool = False
    cdiSpecDir: str = "/var/run/cdi"
    nodeFeatureFile: str = ""             # NFD local feature file ("" = off), see labels/nfd.py
    rediscoverIntervalS: float = 60.0     # detect partition-mode / device-set changes (0 = off)
    sharing: SharingConfig = field(default_factory=SharingConfig)
    telemetry: TelemetryConfig = field(default_factory=TelemetryConfig)
    health: HealthConfig = field(default_factory=HealthConfig)
    http: HttpConfig = field(default_factory=HttpConfig)
    grpc: GrpcConfig = field(default_factory=GrpcConfig)
    podResources: PodResourcesConfig = field(default_factory=PodResourcesConfig)
    allocator: AllocatorConfig = field(default_factory=AllocatorConfig)
    retrySeconds: float = 30.0            # plugin start retry (plugin/manager.go:135-138)
    # scheduling policy of the background threads (sampler, watchdog, driver lanes, event
    # wait, manager helpers): "batch" = SCHED_BATCH, which never preempts a gRPC worker on
    # wake-up; "normal" = SCHED_OTHER.  On an idle MI355X box the Allocate tail was the same
    # either way (profiles/r5/ab_sched.jsonl), so the default stays normal
    backgroundSched: str = "normal"

    @property
    def strategy(self) -> str:
        return self.migStrategy

    @property
    def kubelet_socket(self) -> str:
        return os.path.join(self.pluginDir, v1beta1.KUBELET_SOCKET_NAME)

    def listen_host_port(self) -> tuple[str, int]:
        return split_host_port(self.webListenAddress)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


class ConfigError(ValueError):
    pass


def split_host_port(addr: str) -> tuple[str, int]:
    addr = str(addr).strip()
    m = re.fullmatch(r"\[?([^\]]*)\]?:(\d+)", addr)
    if not m:
        raise ConfigError("webListenAddress %r must be host:port (e.g. 0.0.0.0:9100)" % addr)
    host = m.group(1) or "0.0.0.0"
    return host, int(m.group(2))


_NESTED = {"log": LogConfig, "sharing": SharingConfig, "telemetry": TelemetryConfig,
           "health": HealthConfig, "http": HttpConfig, "grpc": GrpcConfig, "podResources": PodResourcesConfig}


def _ci_lookup(d: dict, name: str):
    """viper/mapstructure match keys case-insensitively (§5.6)."""
    for k, v in d.items():
        if str(k).lower() == name.lower():
            return True, v
    return False, None


def _coerce(value: Any, default: Any):
    if isinstance(default, bool):
        if isinstance(value, str):
            return value.strip().lower() in ("1", "true", "yes", "on")
        return bool(value)
    if isinstance(default, int) and not isinstance(default, bool):
        return int(value)
    if isinstance(default, float):
        return float(value)
    if isinstance(default, str):
        if isinstance(value, (list, tuple)):  # e.g. health.disabledChecks: [ecc, reset]
            return ",".join(str(x) for x in value)
        return str(value)
    return value


def from_dict(raw: dict | None) -> Config:
    cfg = Config()
    raw = raw or {}
    if not isinstance(raw, dict):
        raise ConfigError("config root must be a mapping")
    found, ps = _ci_lookup(raw, "partitionStrategy")
    if found and ps is not None:
        raw = dict(raw)
        raw["migStrategy"] = ps
    for f in dataclasses.fields(Config):
        found, v = _ci_lookup(raw, f.name)
        if not found or v is None:
            continue
        if f.name in _NESTED:
            sub = getattr(cfg, f.name)
            if not isinstance(v, dict):
                raise ConfigError("%s must be a mapping" % f.name)
            for sf in dataclasses.fields(sub):
                sfound, sv = _ci_lookup(v, sf.name)
                if sfound and sv is not None:
                    setattr(sub, sf.name, _coerce(sv, getattr(sub, sf.name)))
        elif f.name == "resources":
            specs = []
            for item in v or []:
                if not isinstance(item, dict) or "name" not in item:
                    raise ConfigError("resources entries need {pattern, name}")
                specs.append(ResourceSpec(pattern=str(item.get("pattern", "*")), name=str(item["name"])))
            cfg.resources = specs
        else:
            setattr(cfg, f.name, _coerce(v, getattr(cfg, f.name)))
    return cfg


def unknown_keys(raw: dict | None) -> list[str]:
    """Keys the loader ignores (viper ignores them silently; a typo such as
    ``migStratgy`` would otherwise fall back to a default without a trace)."""
    out: list[str] = []
    if not isinstance(raw, dict):
        return out
    top = {f.name.lower() for f in dataclasses.fields(Config)} | {"partitionstrategy"}
    for k, v in raw.items():
        if str(k).lower() not in top:
            out.append(str(k))
            continue
        for name, cls in _NESTED.items():
            if str(k).lower() == name.lower() and isinstance(v, dict):
                sub = {f.name.lower() for f in dataclasses.fields(cls)}
                out += ["%s.%s" % (k, sk) for sk in v if str(sk).lower() not in sub]
    return out


def apply_env(cfg: Config, environ=None) -> Config:
    environ = os.environ if environ is None else environ
    for f in dataclasses.fields(Config):
        if f.name in _NESTED or f.name == "resources":
            continue
        env = "AMDGPU_DP_" + re.sub(r"(?<!^)(?=[A-Z])", "_", f.name).upper()
        if env in environ:
            setattr(cfg, f.name, _coerce(environ[env], getattr(cfg, f.name)))
    for name in ("LOG_LEVEL", "LOG_FILE_DIR"):
        if "AMDGPU_DP_" + name in environ:
            val = environ["AMDGPU_DP_" + name]
            if name == "LOG_LEVEL":
                cfg.log.level = val
            else:
                cfg.log.fileDir = val
    if "AMDGPU_DP_GRPC_SERVER" in environ:
        cfg.grpc.server = environ["AMDGPU_DP_GRPC_SERVER"]
    if "AMDGPU_DP_DISABLE_HEALTHCHECKS" in environ:
        cfg.health.disabledChecks = environ["AMDGPU_DP_DISABLE_HEALTHCHECKS"]
    if "AMDGPU_DP_HTTP_SERVER" in environ:
        cfg.http.server = environ["AMDGPU_DP_HTTP_SERVER"]
    return cfg


def validate(cfg: Config) -> Config:
    cfg.migStrategy = str(cfg.migStrategy).strip().lower()
    if cfg.migStrategy not in STRATEGIES:
        raise ConfigError("invalid partition (MIG) strategy %r: want one of %s" % (cfg.migStrategy, STRATEGIES))
    split_host_port(cfg.webListenAddress)
    from .utils.log import parse_level
    try:
        parse_level(cfg.log.level)
    except ValueError as e:
        raise ConfigError(str(e)) from None
    if not cfg.allocator.recentAllocationTtlS >= 0:
        raise ConfigError("allocator.recentAllocationTtlS must be >= 0, got %r" % cfg.allocator.recentAllocationTtlS)
    if not cfg.log.maxAgeDays >= 0:
        raise ConfigError("log.maxAgeDays must be >= 0 (0 keeps rotated files), got %r" % cfg.log.maxAgeDays)
    if cfg.backend not in ("auto", "amdsmi", "fixture"):
        raise ConfigError("backend must be auto|amdsmi|fixture, got %r" % cfg.backend)
    disabled_checks_mask(cfg.health.disabledChecks)
    if cfg.health.pcieMinWidth < 0 or cfg.health.pcieMinSpeedGTs < 0:
        raise ConfigError("health.pcieMinWidth / health.pcieMinSpeedGTs must be >= 0 (0 = no floor)")
    if cfg.health.sampleStallS < 0:
        raise ConfigError("health.sampleStallS must be >= 0 (0 = off)")
    if cfg.health.pcieDebounceSamples < 1:
        raise ConfigError("health.pcieDebounceSamples must be >= 1")
    if cfg.health.discoveryTimeoutS <= 0:
        raise ConfigError("health.discoveryTimeoutS must be > 0")
    if cfg.sharing.replicas < 1:
        raise ConfigError("sharing.replicas must be >= 1")
    if cfg.health.canaryOnPreStart and cfg.sharing.replicas > 1:
        # a time-sliced partition already runs another container: its canary would
        # contend with it (or fail to allocate HBM) and mark a shared, healthy GPU Unhealthy
        raise ConfigError("health.canaryOnPreStart cannot be combined with sharing.replicas > 1: the canary would "
                          "run on a partition another container is using")
    from .utils.util import parse_device_selector
    try:
        parse_device_selector(cfg.devices)
    except ValueError as e:
        raise ConfigError("devices: %s" % e) from None
    if cfg.grpc.server not in ("native", "python"):
        raise ConfigError("grpc.server must be native|python")
    for sect in ("grpc", "http"):
        if not 0 <= getattr(cfg, sect).busyPollUs <= 100000:
            raise ConfigError("%s.busyPollUs must be within 0..100000" % sect)
    if not 0 <= cfg.grpc.admissionPollUs <= 100000:
        raise ConfigError("grpc.admissionPollUs must be within 0..100000")
    for key in ("keepWarmMs", "idleWakeMs"):
        if not 0 <= getattr(cfg.grpc, key) <= 100000:
            raise ConfigError("grpc.%s must be within 0..100000 (0 = off)" % key)
    if not 0 <= cfg.grpc.activeWindowMs <= 86400000:
        raise ConfigError("grpc.activeWindowMs must be within 0..86400000 (0 = always)")
    if not 0 <= cfg.grpc.pollGapNs <= 100000:
        raise ConfigError("grpc.pollGapNs must be within 0..100000")
    if cfg.grpc.callTraceFile and not 1 <= cfg.grpc.callTraceEntries <= (1 << 26):
        raise ConfigError("grpc.callTraceEntries must be within 1..%d" % (1 << 26))
    for sect in ("grpc", "http"):
        if not 1 <= getattr(cfg, sect).threads <= 256:
            raise ConfigError("%s.threads must be within 1..256" % sect)
    if cfg.http.server not in ("native", "python"):
        raise ConfigError("http.server must be native|python")
    if cfg.podResources.intervalS <= 0:
        raise ConfigError("podResources.intervalS must be > 0")
    if cfg.backgroundSched not in ("batch", "normal"):
        raise ConfigError("backgroundSched must be batch|normal, got %r" % cfg.backgroundSched)
    if cfg.telemetry.intervalMs < 10:
        raise ConfigError("telemetry.intervalMs must be >= 10")
    if cfg.telemetry.idleIntervalMs < 0 or cfg.telemetry.idleIntervalMs > 3600000:
        raise ConfigError("telemetry.idleIntervalMs must be within 0..3600000")
    if cfg.telemetry.activeWindowS < 0:
        raise ConfigError("telemetry.activeWindowS must be >= 0")
    if not cfg.resourcePrefix or "/" in cfg.resourcePrefix:
        raise ConfigError("resourcePrefix must be a DNS-like prefix without '/'")
    # extended resource prefixes are DNS subdomains (RFC 1123, at most 253 characters);
    # the name part is checked (1..63 characters) when resources are built
    import re
    label = r"[a-z0-9]([-a-z0-9]{0,61}[a-z0-9])?"
    if len(cfg.resourcePrefix) > 253 or not re.fullmatch(r"%s(\.%s)*" % (label, label), cfg.resourcePrefix):
        raise ConfigError("resourcePrefix %r is not a DNS subdomain (lower-case labels of at most 63 "
                          "characters, 253 in total)" % cfg.resourcePrefix[:80])
    return cfg


def load(config_file: str | None = "config", search_dirs=(".",), environ=None, required: bool = False) -> Config:
    """Loads ``<dir>/<config_file>.yml`` (reference lookup, ``main.go:39-41``), or an
    explicit path when ``config_file`` has a ``.yml``/``.yaml`` suffix or a '/'.  A
    missing file is not fatal (``main.go:42-45``) unless ``required``."""
    raw: dict = {}
    path = None
    if config_file:
        if config_file.endswith((".yml", ".yaml")) or os.sep in config_file:
            candidates = [config_file]
        else:
            candidates = [os.path.join(d, config_file + ext) for d in search_dirs for ext in (".yml", ".yaml")]
        for c in candidates:
            if os.path.isfile(c):
                path = c
                break
        if path is None and required:
            raise ConfigError("config file not found: %s" % candidates)
    if path:
        with open(path, "r", encoding="utf-8") as f:
            import yaml  # only when a config file is read
            raw = yaml.safe_load(f) or {}
    unknown = unknown_keys(raw)
    if unknown:
        from .utils.log import get_logger
        get_logger("config").warning("ignoring unknown config key(s) in %s: %s", path, ", ".join(unknown))
    cfg = from_dict(copy.deepcopy(raw))
    apply_env(cfg, environ)
    return validate(cfg)
