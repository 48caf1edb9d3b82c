#!/bin/bash
# Compact pulled-halo adjacency (PT): fp32 / link-delay / multi-process GPU tests with the
# windowed W=8 rehearsal, then the structureless W=2 and W=8 rehearsals (153 GB/s).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
TESTS=1 RUNS="8:153" bash scripts/rehearse_linkdelay.sh || exit $?
EXTRA="--global-frac 1.0" TESTS=0 RUNS="2:153 8:153" bash scripts/rehearse_linkdelay.sh
