#!/bin/bash
# Round-end evidence: the headline profile (tools/profile.sh) plus per-workload
# trace + traffic passes. Usage (repo root, on the box): bash tools/profile_all.sh <tag>
set -euo pipefail
TAG=${1:-r01e}
bash tools/profile.sh $TAG
for wl in ${WORKLOADS:-apply orswot_csr bincode clock_csr mvreg map map_orswot gcounter}; do
  echo "profiling $wl"
  bash tools/profile_workload.sh $TAG $wl
done
