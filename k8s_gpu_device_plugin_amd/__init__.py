"""MI355X-native Kubernetes device plugin (capabilities of uppercaveman/k8s-gpu-device-plugin).

Layers, MI355X-first:
  L0 native/            C++ core: amdsmi backend, fixture backend, xGMI allocator,
                        protobuf hot paths, exporter, epoll httpd, HTTP/2 gRPC server
     ops/               HIP/CDNA4 health canary (gfx950)
  L1 device/ resource/  partition model, strategies, resource naming
  L2 plugin/plugin.py   kubelet v1beta1 DevicePlugin endpoints (one per resource)
  L3 plugin/manager.py  lifecycle: kubelet restart, /restart, retries, health
  L4 server/            HTTP ops surface (/, /health, /restart, /metrics)
  L5 cli.py config.py utils/ benchmark/
"""
from .utils.version import VERSION as __version__  # noqa: F401
