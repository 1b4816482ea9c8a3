#!/usr/bin/env bash
# Run one gpurun call, re-trying ONLY when no box could be acquired (exit 3: nothing ran, nothing
# charged).  Any other exit (including a failing or faulting command) is returned as-is.
#   usage: tools/gpurun_acquire.sh <timeout_s> '<command>'
T="$1"; shift
for attempt in 1 2 3 4 5 6; do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
    rc=$?
    [ "$rc" -ne 3 ] && exit "$rc"
    echo "[acquire] no box (attempt $attempt), waiting"
    sleep 45
done
exit 3
