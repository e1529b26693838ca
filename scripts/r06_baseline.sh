#!/bin/bash
# round-6 baseline traces at HEAD: C2, C3, C5 (shuffled and natural numbering)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
bash scripts/prof_c2.sh r6_c2 > gpurun_out/r6_c2.grep
bash scripts/prof_c3.sh r6_c3 > gpurun_out/r6_c3.grep
bash scripts/prof_c5.sh r6_c5 > gpurun_out/r6_c5.grep
C5_ARGS="--permute -1" bash scripts/prof_c5.sh r6_c5nat > gpurun_out/r6_c5nat.grep
