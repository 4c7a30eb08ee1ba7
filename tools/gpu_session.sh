# tools/gpu_session.sh -- run several GPU steps in one gpurun call, each under its own time limit.
# usage: bash tools/gpu_session.sh "name:seconds:command" ...
# A step that fails normally (exit 1, a failed test) does not stop the session; a step that times out,
# aborts or crashes (124, 137, 134, 139) ends it: nothing more touches the GPU after that.
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -15 "gpurun_out/$name.log"
  case $rc in 124|137|134|139) echo "=== stopping after $name (rc $rc)"; exit $rc;; esac
done
