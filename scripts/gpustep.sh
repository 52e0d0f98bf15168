#!/bin/bash
# Sourced by the GPU-session scripts: `step NAME SECONDS CMD...` runs one GPU step under its own
# time limit, logs to $O/NAME.log and a progress line per step; chain steps with && so the first
# failure / timeout / fault ends the session (pool rules).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=${O:-gpurun_out/session}
mkdir -p "$O"
step() {
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a "$O/progress.log"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$O/progress.log"
  return $rc
}
