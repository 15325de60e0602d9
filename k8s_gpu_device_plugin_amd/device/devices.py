"""Device model, ordered device sets and the annotated-ID (replica) scheme.

Reference: ``device/devices.go``.  ``Device`` (``:21-29``) wraps the kubelet
``Device`` with Paths/Index/TotalMemory/ComputeCapability/Replicas; ``Devices``
(``:32-209``) is a Go map with set algebra; ``AnnotatedID`` (``:35-38,221-265``)
parses ``"<id>::<replica>"``.  Differences: ``Devices`` preserves insertion order
(Go map iteration is random: defect D14), the CUDA compute capability becomes the gfx
target (``gfx950``), MIG index ``"i:j"`` becomes ``"<gpu>:<partition>"``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable, Iterator

from ..api import v1beta1

ANNOTATION_SEP = "::"


class AnnotatedID(str):
    """``"<id>::<replica>"`` identifiers of time-sliced replicas."""

    @classmethod
    def new(cls, id_: str, replica: int) -> "AnnotatedID":
        return cls("%s%s%d" % (id_, ANNOTATION_SEP, replica))

    def has_annotations(self) -> bool:
        return ANNOTATION_SEP in self

    def split(self) -> tuple[str, int]:  # type: ignore[override]
        if ANNOTATION_SEP not in self:
            return str(self), 0
        base, rep = str.split(self, ANNOTATION_SEP, 1)
        try:
            return base, int(rep)
        except ValueError:  # Go's ParseInt error is ignored -> 0 (devices.go:238)
            return base, 0

    def get_id(self) -> str:
        return self.split()[0]


def new_annotated_id(id_: str, replica: int) -> AnnotatedID:
    return AnnotatedID.new(id_, replica)


def any_has_annotations(ids: Iterable[str]) -> bool:
    return any(AnnotatedID(i).has_annotations() for i in ids)


def annotated_ids_get_ids(ids: Iterable[str]) -> list[str]:
    return [AnnotatedID(i).get_id() for i in ids]


@dataclass
class Device:
    id: str
    index: str                      # "<gpu>" or "<gpu>:<partition>"
    gpu: int
    partition: int = -1             # -1 = whole physical GPU
    numa_node: int | None = None
    paths: list[str] = field(default_factory=list)  # host device nodes (render/card)
    total_memory: int = 0
    compute_capability: str = ""    # gfx target, e.g. gfx950
    replicas: int = 0
    replica: int = -1
    product: str = ""
    profile: str = ""               # e.g. "cpx_nps2" for partitions
    # Health has one source of truth: the native DeviceTable of the plugin advertising the
    # device (the health monitor writes it directly, ListAndWatch and Allocate read it).
    # Once bound (bind_table) this view reads and writes through to the table; before,
    # it holds the initial state the table is built from.
    _health: str = field(default=v1beta1.HEALTHY, repr=False, compare=False)
    _table: object = field(default=None, repr=False, compare=False)

    @property
    def health(self) -> str:
        if self._table is not None:
            return v1beta1.HEALTHY if self._table.healthy(self.id) else v1beta1.UNHEALTHY
        return self._health

    @health.setter
    def health(self, value: str) -> None:
        if self._table is not None:
            self._table.set_health(self.id, value == v1beta1.HEALTHY)
        else:
            self._health = value

    def bind_table(self, table) -> None:
        self._table = table

    def is_partition(self) -> bool:
        """Reference ``IsMigDevice`` (index contains ':')."""
        return ":" in self.index

    def aligned_allocation_supported(self) -> bool:
        # Reference (devices.go:197-209): false for MIG devices and WSL.  AMD partitions
        # are KFD nodes the xGMI allocator can pack, so only replicas opt out.
        return not AnnotatedID(self.id).has_annotations()

    def get_uuid(self) -> str:
        return AnnotatedID(self.id).get_id()

    def to_plugin_device(self):
        d = v1beta1.Device(ID=self.id, health=self.health)
        if self.numa_node is not None and self.numa_node >= 0:
            d.topology.nodes.add(ID=self.numa_node)
        return d


class Devices:
    """Insertion-ordered ``id -> Device`` set with the reference's set algebra."""

    def __init__(self, devices: Iterable[Device] = ()) -> None:
        self._d: dict[str, Device] = {}
        for d in devices:
            self._d[d.id] = d

    def __len__(self) -> int:
        return len(self._d)

    def __iter__(self) -> Iterator[Device]:
        return iter(self._d.values())

    def __contains__(self, id_: str) -> bool:
        return id_ in self._d

    def __getitem__(self, id_: str) -> Device:
        return self._d[id_]

    def add(self, d: Device) -> None:
        self._d[d.id] = d

    def contains(self, *ids: str) -> bool:
        return all(i in self._d for i in ids)

    def get_by_id(self, id_: str) -> Device | None:
        return self._d.get(id_)

    def get_by_index(self, index: str) -> Device | None:
        for d in self._d.values():
            if d.index == index:
                return d
        return None

    def subset(self, ids: Iterable[str]) -> "Devices":
        return Devices(self._d[i] for i in ids if i in self._d)

    def difference(self, other: "Devices") -> "Devices":
        return Devices(d for d in self._d.values() if d.id not in other)

    def get_ids(self) -> list[str]:
        return list(self._d)

    def get_uuids(self) -> list[str]:
        seen, out = set(), []
        for d in self._d.values():
            u = d.get_uuid()
            if u not in seen:
                seen.add(u)
                out.append(u)
        return out

    def get_plugin_devices(self) -> list:
        return [d.to_plugin_device() for d in self._d.values()]

    def get_indices(self) -> list[str]:
        return [d.index for d in self._d.values()]

    def get_paths(self) -> list[str]:
        out = []
        for d in self._d.values():
            out.extend(d.paths)
        return out

    def aligned_allocation_supported(self) -> bool:
        return all(d.aligned_allocation_supported() for d in self._d.values())
