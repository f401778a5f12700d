# Run GPU steps in order, each under its own time limit; stop at the first fault, abort, segfault or timeout
# (exit 124/134/137/139 or a signal), continue past ordinary failures (e.g. pytest rc 1).
# usage: bash tools/gpu_steps.sh <outdir> "<name>|<seconds>|<command>" ...
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  tail -3 "$out/$name.log"
  echo "rc=$rc"
  case $rc in
    0|1|2|5) ;;
    *) echo "stopping after $name (rc $rc)"; exit $rc ;;
  esac
done
