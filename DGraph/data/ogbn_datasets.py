"""API-compatibility module: reference path ``DGraph/data/ogbn_datasets.py`` re-exported from ``dgraph_amd.data.ogbn``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.data.ogbn import SUPPORTED_DATASETS, DistributedOGBWrapper, num_classes  # noqa: F401
