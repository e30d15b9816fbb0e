#!/usr/bin/env bash
# Ad-hoc GPU session: each line of $STEPS_FILE is "<name> <timeout> <command...>"; every step has
# its own time limit and the session stops at the first crash / timeout (rc other than 0 / 1).
# Usage (repo root, on the box):  bash scripts/adhoc.sh <tag> <steps file>
set -u
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
while read -r name lim cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  echo "== $name: $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < "$2"
echo done
