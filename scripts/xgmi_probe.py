"""Dumps what amdsmi reports about a GPU's xGMI links: per-link metrics (peer, up,
bit_rate, max_bandwidth) and the gpu_metrics blob's link width / speed."""
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_gpu_device_plugin_amd import native  # noqa: E402

n = native.load()
be = n.make_amdsmi_backend()
gpus, topo = be.discover()
out = []
for g in gpus:
    s = be.sample(g.index)
    out.append({"gpu": g.index, "bdf": g.bdf, "num_xgmi_links": g.num_xgmi_links,
                "blob_xgmi_link_width": s.xgmi_link_width if s else None,
                "blob_xgmi_link_speed": s.xgmi_link_speed if s else None,
                "links": [dict(zip(("peer", "up", "read_kb", "write_kb", "bit_rate", "max_bandwidth", "trained"), l))
                          for l in (s.links if s else [])],
                "topology_row": [(b, topo.link(g.index, b).type, topo.link(g.index, b).hops, topo.link(g.index, b).weight,
                                  topo.link(g.index, b).bw_gbps) for b in range(topo.n)]})
print(json.dumps(out, indent=1))
be.shutdown()
