"""API-compatibility module: reference path ``DGraph/data/__init__.py`` re-exported from ``dgraph_amd.data``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
