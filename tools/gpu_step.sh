#!/bin/bash
# One bounded GPU step: gpu_step.sh <tag> <timeout-s> <cmd...>
# Runs <cmd> under `timeout -k 10`, output to gpurun_out/<tag>.log, prints rc + the log's tail.
# Exits with the command's status, so steps chain with && and a fault / abort / timeout ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 MASTER_ADDR=127.0.0.1
tag=$1 lim=$2; shift 2
timeout -k 10 "$lim" "$@" > "gpurun_out/$tag.log" 2>&1
rc=$?
echo "$tag rc=$rc"
tail -"${TAIL:-2}" "gpurun_out/$tag.log" | cut -c1-600
exit $rc
