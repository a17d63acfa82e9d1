#!/bin/bash
# headline PMC traffic (gpu_r03u.sh), then the CPU-full baseline (gpu_r03t.sh)
set -u
bash "$GRAFT_REPO_ROOT/tools/gpu_r03u.sh" || exit $?
bash "$GRAFT_REPO_ROOT/tools/gpu_r03t.sh"
