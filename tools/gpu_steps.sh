#!/bin/bash
# Run GPU steps in order; continue after ordinary test failures (rc 1), stop after anything that
# looks like a fault / abort / timeout (rc >= 2).
for step in "$@"; do
  echo "=== $step" >&2
  bash -c "$step"
  rc=$?
  echo "=== rc=$rc : $step" >&2
  if [ $rc -ge 2 ]; then echo "stopping after rc=$rc" >&2; exit $rc; fi
done
