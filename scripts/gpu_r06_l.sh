#!/bin/bash
# GraphCast aligned ranks 0/1/3 (heavier grid weight), then the W=8/W=2 rehearsals with the
# source-ordered send-row packs (structureless W=8 / W=2 and windowed W=8, 153 GB/s).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
RANKS="0 1 3" TAG=3 bash scripts/gpu_r06_k.sh || exit $?
EXTRA="--global-frac 1.0" TESTS=0 RUNS="8:153 2:153" bash scripts/rehearse_linkdelay.sh
rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
TESTS=0 RUNS="8:153" bash scripts/rehearse_linkdelay.sh
