#!/bin/bash
# Runs GPU steps in order, each under its own time limit; a step that fails normally (exit 1:
# a failing test or a Python exception) does not stop the sequence, anything else (abort,
# segfault, time limit, signal) ends it there.  Usage: bash scripts/gpu_seq.sh 'name|seconds|command' ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/seq.log
for step in "$@"; do
    name="${step%%|*}"; rest="${step#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc" >> gpurun_out/seq.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
