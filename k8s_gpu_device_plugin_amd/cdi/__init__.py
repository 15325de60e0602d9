from .spec import build_spec, write_spec  # noqa: F401
