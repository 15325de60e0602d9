"""Device model, annotated IDs, resource naming and strategy -> device map
(reference device/devices.go, device/device_map.go, resource/*.go semantics)."""
import pytest

from k8s_gpu_device_plugin_amd.api import v1beta1
from k8s_gpu_device_plugin_amd.device import (AnnotatedID, Device, Devices, annotated_ids_get_ids,
                                              any_has_annotations, build_device_map, matches, new_annotated_id,
                                              wildcard_to_regexp)
from k8s_gpu_device_plugin_amd.models import fixtures
from k8s_gpu_device_plugin_amd.resource import ResourceName, new_resource, new_resources


def test_annotated_id_semantics():
    a = new_annotated_id("GPU-1", 3)
    assert a == "GPU-1::3" and a.has_annotations() and a.split() == ("GPU-1", 3) and a.get_id() == "GPU-1"
    plain = AnnotatedID("GPU-2")
    assert not plain.has_annotations() and plain.split() == ("GPU-2", 0) and plain.get_id() == "GPU-2"
    assert AnnotatedID("x::y").split() == ("x", 0)  # ParseInt error ignored, like the reference
    assert AnnotatedID("a::1::2").split() == ("a", 0)  # SplitN(.., 2): "1::2" is not an int
    assert any_has_annotations(["a", "b::0"]) and not any_has_annotations(["a", "b"])
    assert annotated_ids_get_ids(["a::1", "b"]) == ["a", "b"]


def _devs():
    return Devices([Device(id="u%d" % i, index=str(i), gpu=i, paths=["/dev/dri/renderD%d" % (128 + i)],
                           numa_node=i // 2) for i in range(4)])


def test_devices_set_algebra_is_ordered():
    ds = _devs()
    assert ds.get_ids() == ["u0", "u1", "u2", "u3"]
    assert ds.contains("u1", "u3") and not ds.contains("u1", "zz")
    assert ds.get_by_id("u2").index == "2" and ds.get_by_id("zz") is None
    assert ds.get_by_index("3").id == "u3" and ds.get_by_index("9") is None
    sub = ds.subset(["u3", "u0", "missing"])
    assert sub.get_ids() == ["u3", "u0"]
    assert ds.difference(sub).get_ids() == ["u1", "u2"]
    assert ds.get_indices() == ["0", "1", "2", "3"]
    assert ds.get_paths()[0] == "/dev/dri/renderD128"
    assert ds.aligned_allocation_supported()
    pd = ds.get_plugin_devices()
    assert [d.ID for d in pd] == ds.get_ids() and pd[2].topology.nodes[0].ID == 1
    assert all(d.health == v1beta1.HEALTHY for d in pd)


def test_uuids_deduplicate_replicas():
    ds = Devices([Device(id=str(new_annotated_id("g", k)), index="0", gpu=0) for k in range(3)])
    assert ds.get_uuids() == ["g"]
    assert not ds.aligned_allocation_supported()
    d = Device(id="g", index="0:1", gpu=0, partition=1)
    assert d.is_partition() and not Device(id="g", index="0", gpu=0).is_partition()


def test_wildcard_patterns_are_anchored():
    assert wildcard_to_regexp("*MI355*") == "^.*MI355.*$"
    assert matches("*", "AMD Instinct MI355X")
    assert matches("*MI355*", "AMD Instinct MI355X")
    assert not matches("GPU", "AMD Instinct MI355X")          # reference default pattern (D3)
    assert matches("cpx_nps2", "cpx_nps2") and not matches("cpx_nps2", "cpx_nps2x")  # D15
    assert matches("a.b", "a.b") and not matches("a.b", "axb")  # '.' is literal


def test_resource_name_helpers():
    r = ResourceName("amd.com/gpu")
    assert r.split() == ("amd.com", "gpu") and r.get_resource_name() == "gpu"
    assert r.get_resource_name_prefix() == "amd.com"
    assert r.default_shared_rename() == "amd.com/gpu.shared"
    assert ResourceName("gpu").split() == ("", "gpu")
    assert new_resource("*", "gpu").name == "amd.com/gpu"
    assert new_resource("*", "amd.com/gpu").name == "amd.com/gpu"
    with pytest.raises(ValueError):
        new_resource("*", "x" * 64)
    with pytest.raises(ValueError):
        new_resource("*", "bad name")


def _gpus(spec):
    return fixtures.build_backend(spec).discover()[0]


def test_strategy_none_whole_gpus_with_all_render_nodes():
    g = _gpus("8gpu_cpx_nps2")
    dm = build_device_map(g, new_resources(g, "none"), "none")
    assert list(dm) == ["amd.com/gpu"]
    ds = dm["amd.com/gpu"]
    assert len(ds) == 8
    d0 = ds.get_by_index("0")
    assert d0.id == g[0].uuid and len(d0.paths) == 8 and d0.partition == -1
    assert d0.compute_capability == "gfx950" and d0.total_memory == g[0].vram_total_bytes


def test_strategy_single_every_partition():
    g = _gpus("8gpu_cpx_nps2")
    dm = build_device_map(g, new_resources(g, "single"), "single")
    ds = dm["amd.com/gpu"]
    assert len(ds) == 64
    d = ds.get_by_index("3:5")
    assert d.gpu == 3 and d.partition == 5 and d.paths == ["/dev/dri/renderD%d" % (128 + 3 * 8 + 5)]
    assert d.numa_node == 0 and d.profile == "cpx_nps2"
    g1 = _gpus("2gpu_spx")
    ds1 = build_device_map(g1, new_resources(g1, "single"), "single")["amd.com/gpu"]
    assert ds1.get_indices() == ["0", "1"] and ds1.get_by_index("1").partition == -1


def test_strategy_mixed_keeps_unpartitioned_gpus():
    model = fixtures.mi355x_node(2)
    model["gpus"].append({"compute_partition": "CPX", "memory_partition": "NPS2", "numa_node": 1})
    model["gpus"].append({"compute_partition": "QPX", "memory_partition": "NPS2", "numa_node": 1})
    g = fixtures.build_backend(model).discover()[0]
    res = new_resources(g, "mixed")
    assert [str(r.name) for r in res] == ["amd.com/gpu", "amd.com/cpx_nps2", "amd.com/qpx_nps2"]
    dm = build_device_map(g, res, "mixed")
    assert {k: len(v) for k, v in dm.items()} == {"amd.com/gpu": 2, "amd.com/cpx_nps2": 8, "amd.com/qpx_nps2": 4}


def test_unmatched_devices_are_skipped_not_fatal():
    from k8s_gpu_device_plugin_amd.config import ResourceSpec
    g = _gpus("2gpu_spx")
    res = new_resources(g, "none", specs=[ResourceSpec(pattern="*MI300*", name="mi300")])
    dm = build_device_map(g, res, "none")
    assert len(dm["amd.com/mi300"]) == 0


def test_replicas_and_shared_rename():
    g = _gpus("2gpu_spx")
    dm = build_device_map(g, new_resources(g, "single"), "single", replicas=3, rename_shared=True)
    assert list(dm) == ["amd.com/gpu.shared"]
    ds = dm["amd.com/gpu.shared"]
    assert len(ds) == 6 and ds.get_ids()[:3] == ["%s::%d" % (g[0].uuid, k) for k in range(3)]
    assert ds.get_uuids() == [g[0].uuid, g[1].uuid]
    assert all(d.replicas == 3 for d in ds)


def test_invalid_strategy():
    g = _gpus("2gpu_spx")
    with pytest.raises(ValueError):
        build_device_map(g, new_resources(g, "none"), "bogus")
    with pytest.raises(ValueError):
        new_resources(g, "bogus")


def test_fixture_models():
    for name in fixtures.BUILTIN:
        gpus, topo = fixtures.build_backend(name).discover()
        assert topo.n == len(gpus) >= 1
        for g in gpus:
            assert len(g.partitions) == fixtures.PARTITIONS[g.compute_partition]
    gpus, topo = fixtures.build_backend("8gpu_spx_degraded").discover()
    assert not topo.link(0, 5).up and not topo.link(5, 0).up and topo.link(0, 1).up
    assert fixtures.load_model("3gpu_qpx_nps2")["gpus"][0]["compute_partition"] == "QPX"
    with pytest.raises(ValueError):
        fixtures.load_model("nonsense")


def test_device_health_is_read_from_the_native_table(n):
    """One source of truth: once a plugin's table exists, a Device's health is the
    table's (the health monitor writes the table directly, from its own thread), and
    writing the view writes the table."""
    from k8s_gpu_device_plugin_amd.device.devices import Device, Devices
    from k8s_gpu_device_plugin_amd.plugin.plugin import make_table
    devs = Devices([Device("a", "0", 0), Device("b", "1", 1)])
    devs["b"].health = v1beta1.UNHEALTHY  # before the table: initial state
    t = make_table("amd.com/gpu", devs, n.Topology(2), None)
    assert not t.healthy("b") and devs["b"].health == v1beta1.UNHEALTHY
    t.set_gpu_health(0, -1, False)  # e.g. the monitor's fail-fast path
    assert devs["a"].health == v1beta1.UNHEALTHY
    devs["a"].health = v1beta1.HEALTHY
    assert t.healthy("a") and t.version >= 3


def test_fixture_cannot_declare_a_mode_outside_its_caps():
    """the fixture's partition model is pinned to what the MI355X box
    reports (memory caps NPS1|NPS2, profiles/r4/amdsmi_probe.json).  A node model - or an
    operator's simulated re-partitioning - that puts a GPU in a mode outside its profile
    table is rejected; CPX+NPS4 exists only as the declared hypothetical 8gpu_cpx_nps4."""
    from k8s_gpu_device_plugin_amd.models import fixtures
    with pytest.raises(ValueError, match="CPX\\+NPS4, outside its supported profiles"):
        fixtures.build_backend("2gpu_cpx_nps4")
    with pytest.raises(ValueError, match="outside its supported profiles"):
        fixtures.build_backend(fixtures.mi355x_node(2, "QPX", "NPS8"))
    be = fixtures.build_backend("2gpu_cpx_nps2")
    gpus, _ = be.discover()
    assert [(p.type, p.partitions, p.nps_caps) for p in gpus[0].supported_profiles] == [
        ("SPX", 1, 3), ("DPX", 2, 3), ("QPX", 4, 3), ("CPX", 8, 3)]
    with pytest.raises(ValueError, match="outside its supported profiles"):
        fixtures.set_gpu_mode(be, 0, "CPX", "NPS4")
    fixtures.set_gpu_mode(be, 0, "DPX", "NPS1")  # a supported mode is accepted
    assert fixtures.load_model("8gpu_cpx_nps4").get("hypothetical") is True
    hyp, _ = fixtures.build_backend("8gpu_cpx_nps4").discover()
    assert hyp[0].memory_partition == "NPS4" and all(p.nps_caps & 4 for p in hyp[0].supported_profiles)
    assert sum(len(g.partitions) for g in hyp) == 64


def test_supported_profiles_are_exported(n):
    from prometheus_client.parser import text_string_to_metric_families

    from k8s_gpu_device_plugin_amd.models import fixtures
    be = fixtures.build_backend("2gpu_qpx_nps2")
    gpus, _ = be.discover()
    ex = n.Exporter()
    ex.set_inventory(gpus)
    ex.set_partition_labels([n.PartitionLabel(g.index, p.index, p.id, "amd.com/gpu", str(p.hip_id))
                             for g in gpus for p in g.partitions])
    ex.start(be, 50, None)
    try:
        fams = {f.name: f for f in text_string_to_metric_families(ex.render())}
    finally:
        ex.stop()
    rows = {(s.labels["gpu"], s.labels["profile"], s.labels["partitions"], s.labels["memory_partition"])
            for s in fams["amdgpu_partition_profile_supported"].samples}
    assert len(rows) == 2 * 4 * 2 and ("1", "CPX", "8", "NPS2") in rows and ("0", "QPX", "4", "NPS1") in rows
    busy = fams["amdgpu_partition_gfx_busy_percent"].samples
    assert len(busy) == 8 and {s.labels["source"] for s in busy} == {"partition_metrics"}
    info = fams["amdgpu_partition_info"].samples
    assert sorted(int(s.labels["hip_ids"]) for s in info) == list(range(8))
