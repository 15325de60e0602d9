"""Resource names and partition-strategy constants.

Reference: ``resource/resource.go:8-66`` (prefix ``nvidia.com``, MIG strategies
none/single/mixed, ``ResourceName`` split helpers, auto-prefixing ``NewResource``,
``DefaultSharedRename``).  MI355X mapping: prefix ``amd.com``; the MIG strategies
become compute-partition strategies (SPX/DPX/QPX/CPX x NPS1/NPS2/...).
"""
from __future__ import annotations

from dataclasses import dataclass

RESOURCE_NAME_PREFIX = "amd.com"
DEFAULT_SHARED_RESOURCE_NAME_SUFFIX = ".shared"
MAX_RESOURCE_NAME_LENGTH = 63

STRATEGY_NONE = "none"
STRATEGY_SINGLE = "single"
STRATEGY_MIXED = "mixed"
# reference names (resource/resource.go:15-19)
MigStrategyNone, MigStrategySingle, MigStrategyMixed = STRATEGY_NONE, STRATEGY_SINGLE, STRATEGY_MIXED


class ResourceName(str):
    """A fully-qualified extended resource name, e.g. ``amd.com/gpu``."""

    def split(self) -> tuple[str, str]:  # type: ignore[override]
        if "/" not in self:
            return "", str(self)
        prefix, name = str.split(self, "/", 1)
        return prefix, name

    def get_resource_name(self) -> str:
        """Name without prefix (``resource.go:43-46``); used for the socket file name."""
        return self.split()[1]

    def get_resource_name_prefix(self) -> str:
        return self.split()[0]

    def default_shared_rename(self) -> "ResourceName":
        return ResourceName(str(self) + DEFAULT_SHARED_RESOURCE_NAME_SUFFIX)

    def validate(self) -> None:
        name = self.get_resource_name()
        if not name or len(name) > MAX_RESOURCE_NAME_LENGTH:
            raise ValueError("resource name %r must be 1..%d characters" % (name, MAX_RESOURCE_NAME_LENGTH))
        for ch in name:
            if not (ch.isalnum() or ch in "-_."):
                raise ValueError("invalid character %r in resource name %r" % (ch, name))


@dataclass(frozen=True)
class Resource:
    pattern: str
    name: ResourceName


def new_resource(pattern: str, name: str, prefix: str = RESOURCE_NAME_PREFIX) -> Resource:
    """Auto-prefixes ``name`` (``resource.go:32-40``)."""
    if not name.startswith(prefix + "/"):
        name = prefix + "/" + name
    rn = ResourceName(name)
    rn.validate()
    return Resource(pattern=pattern, name=rn)
