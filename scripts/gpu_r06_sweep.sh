#!/bin/bash
# Link-rate sensitivity: the headline step's W-way rank behind the link
# model at 40 / 75 / 110 / 153 GB/s per peer (box default GPU_MAX_HW_QUEUES). GRAPH=windowed
# (the headline graph) or structureless (--global-frac 1.0); RUNS="W:GBPS ...".
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
if [ "${GRAPH:-windowed}" = structureless ]; then export EXTRA="--global-frac 1.0 ${EXTRA:-}"; fi
TESTS=0 RUNS="${RUNS:-8:40 8:75 8:110 8:153 2:75 2:153}" bash scripts/rehearse_linkdelay.sh
