from .nfd import node_labels, write_feature_file  # noqa: F401
