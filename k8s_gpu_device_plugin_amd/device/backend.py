"""Backend selection (the reference hard-wires ``nvml.New()`` at ``plugin/manager.go:44``
with no injection seam)."""
from __future__ import annotations

from .. import native
from ..utils.log import get_logger

log = get_logger("backend")


def make_backend(cfg):
    """``amdsmi`` (real MI355X), ``fixture`` (scripted node model) or ``auto``.

    ``auto`` never invents devices: without amdsmi-visible GPUs it returns an empty
    fixture node, so the plugin serves its HTTP surface and waits (reference: "No
    devices found. Waiting indefinitely.", ``plugin/manager.go:132-134``)."""
    n = native.load()
    kind = getattr(cfg, "backend", "auto")
    if kind == "fixture":
        from ..models import fixtures
        return fixtures.build_backend(cfg.fixture)
    if kind == "amdsmi":
        return n.make_amdsmi_backend()
    if n.amdsmi_available(keep=True):  # the backend adopts the probe's session
        return n.make_amdsmi_backend()
    log.warning("amdsmi found no AMD GPUs on this node; advertising nothing")
    return n.FixtureBackend(1)
