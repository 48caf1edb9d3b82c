"""API-compatibility module: reference path ``DGraph/utils/TimingReport.py`` re-exported from ``dgraph_amd.utils.timing``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.utils.timing import TimingReport  # noqa: F401
