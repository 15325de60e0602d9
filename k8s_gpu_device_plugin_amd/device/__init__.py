from .devices import (AnnotatedID, Device, Devices, annotated_ids_get_ids, any_has_annotations,  # noqa: F401
                      new_annotated_id)
from .device_map import build_device_map, matches, wildcard_to_regexp  # noqa: F401
