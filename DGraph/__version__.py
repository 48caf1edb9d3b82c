"""API-compatibility module: reference path ``DGraph/__version__.py`` re-exported from ``dgraph_amd.__version__``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.__version__ import __version__  # noqa: F401
