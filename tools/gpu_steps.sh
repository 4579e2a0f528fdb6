#!/bin/bash
# Run GPU steps in order on the gpurun box: each "name|seconds|command" line of $1 runs under its own
# timeout with output in gpurun_out/<name>.log. An ordinary failure (exit 1: failed tests) moves on;
# a fault, abort, segfault or time limit (any other non-zero status) ends the session there.
mkdir -p gpurun_out
export TMPDIR=/tmp
while IFS='|' read -r name secs cmd; do
    [ -z "$name" ] && continue
    case "$name" in \#*) continue ;; esac
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < "$1"
