#!/bin/bash
# headline (bf16, B = 1) PMC HBM traffic of the decode kernels on the final r03 build
set -u
bash "$GRAFT_REPO_ROOT/tools/pmc_traffic.sh"
