#!/bin/bash
# Run GPU steps one after the other, each under its own time limit; a step that times out,
# aborts or crashes (exit 124 / 134 / 137 / 139) ends the script -- a test failure (exit 1)
# does not.  Usage: tools/gpu/steps.sh OUTDIR "name:seconds:command" ...
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($secs s): $cmd" | tee -a "$out/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.txt" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a "$out/steps.log"
  tail -3 "$out/$name.txt"
  case $rc in
    124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc ;;
  esac
done
exit 0
