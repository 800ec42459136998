#!/usr/bin/env bash
# Runs one GPU step under its own time limit; stops the chain on a crash/abort/timeout.
# usage: scripts/gpu_step.sh SECONDS LOGFILE cmd...   (exit 0/1 of cmd are passed through)
set -u
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] $* -> rc=$rc" | tee -a "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 99; fi
exit 0
