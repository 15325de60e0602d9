"""Small shared helpers.

Reference: ``modules/util/util.go:10-23`` (CloseOnce latch, NewID) and
``modules/util/http.go:3-15`` (JSON envelope ``{code,data,msg}``).
"""
from __future__ import annotations

import json
import threading
import uuid


class CloseOnce:
    """A latch that can be closed exactly once and waited on.

    The reference builds ``CloseOnce{C, Once, Close}`` by hand in ``main.go:63-71``
    and then forgets to store it in the manager (defect D1: ``p.ready`` is nil and
    ``ready.Close()`` panics).  Here it is a plain object passed by reference.
    """

    def __init__(self) -> None:
        self._ev = threading.Event()

    def close(self) -> None:
        self._ev.set()

    @property
    def closed(self) -> bool:
        return self._ev.is_set()

    def wait(self, timeout: float | None = None) -> bool:
        return self._ev.wait(timeout)


_libc = None


def name_os_thread(name: str | None = None) -> None:
    """Gives the calling thread its Python name at the OS level too (``py-<name>``, 15
    bytes at most), so ``top -H`` and /proc/<pid>/task/*/comm tell the daemon's Python
    threads apart like its native ones (``dpgrpc-N``, ``dpsampler``, ...)."""
    global _libc
    try:
        import ctypes
        if _libc is None:
            _libc = ctypes.CDLL(None, use_errno=True)
        comm = ("py-" + (name or threading.current_thread().name)).encode()[:15]
        _libc.prctl(15, ctypes.c_char_p(comm), 0, 0, 0)  # PR_SET_NAME
    except Exception:
        pass


def new_id() -> str:
    """Random identifier (reference ``util.NewID``, uuid4 without dashes)."""
    return uuid.uuid4().hex


def success(data) -> dict:
    """``{"code":0,"data":data,"msg":"success"}`` (``modules/util/http.go:9-11``)."""
    return {"code": 0, "data": data, "msg": "success"}


def failed(msg: str) -> dict:
    """``{"code":-1,"data":null,"msg":msg}`` (``modules/util/http.go:13-15``)."""
    return {"code": -1, "data": None, "msg": msg}


def envelope_bytes(obj: dict) -> bytes:
    """Serialises like Go's ``json.Encoder``: compact separators, trailing newline,
    field order code, data, msg."""
    return (json.dumps(obj, separators=(",", ":"), ensure_ascii=False) + "\n").encode()


def parse_device_selector(spec: str | None):
    """``devices``: ``"0-3,6"`` style indices, GPU identities (UUID or PCI BDF) and/or
    host HIP ordinals (``"hip:0-3"``: the GPUs whose partitions the HIP runtime numbers
    0-3, i.e. what ``cuda:0``..``cuda:3`` open), comma-separated.  Returns ``None`` for
    "all", else ``(indices, names)``; HIP ordinals are in ``names`` as ``"hip:<n>"``."""
    if spec is None:
        return None
    spec = str(spec).strip()
    if not spec or spec in ("all", "*"):
        return None
    indices: set[int] = set()
    names: set[str] = set()
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if part.lower().startswith("hip:"):
            hip = parse_index_list(part[4:])
            if not hip:
                raise ValueError("devices: %r names no HIP ordinal" % part)
            names.update("hip:%d" % i for i in hip)
            continue
        a, sep, b = part.partition("-")
        if part.isdigit():
            indices.add(int(part))
        elif sep and a.strip().isdigit() and b.strip().isdigit():
            indices.update(range(int(a), int(b) + 1))
        else:  # a UUID (has dashes) or a BDF such as 0000:75:00.0
            names.add(part.lower())
    return sorted(indices), names


def parse_index_list(spec: str | None) -> list[int] | None:
    """Parses ``"0-3,6"`` into ``[0, 1, 2, 3, 6]``; empty/None means "all"."""
    if spec is None:
        return None
    spec = str(spec).strip()
    if not spec or spec in ("all", "*"):
        return None
    out: list[int] = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))
