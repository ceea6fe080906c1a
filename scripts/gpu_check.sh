#!/bin/bash
# One GPU session: kernel tests, then a short bench.  Each GPU step has its
# own time limit; a crash/abort/timeout (exit >= 124) ends the session, plain
# test failures (exit 1) do not.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DWAMD_NO_REBUILD=${DWAMD_NO_REBUILD:-0}

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}

step build 300 python -c "import __graft_entry__ as g; g.build()"
[ "${1:-}" = "build" ] && exit 0
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 600 python bench.py --steps ${STEPS:-6} --warmup ${WARMUP:-2}
grep '^{' gpurun_out/bench1.log || true
