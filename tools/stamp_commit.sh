#!/bin/bash
# Writes the current commit (plus "-dirty" when kernel sources differ from it) to .build_commit:
# the tree gpurun sends to the GPU box has no .git, and bench.py / tools/traffic.py stamp their
# outputs with it (bench.build_provenance).  Run before a GPU call.
cd "$(dirname "$0")/.."
c=$(git rev-parse --short HEAD)
git diff --quiet HEAD -- nightcore-to-flac-analyzer_amd/csrc include || c="$c-dirty"
echo "$c" > .build_commit
echo "$c"
