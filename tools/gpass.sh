#!/bin/bash
# One GPU pass of named steps (the round-4 one-off tools/r04*.sh folded into one parameterised script):
#   tools/gpass.sh TAG 'NAME|SECONDS|COMMAND' ...
# Each step runs under its own `timeout -k 10 SECONDS`, writes gpurun_out/TAG/NAME.log, and the pass stops
# at the first failing step (no GPU step runs after a fault, abort, or time limit).  Preset steps:
#   tests[:ARGS]      pytest -m gpu (ARGS: extra pytest arguments, e.g. a -k filter)
#   bench[:ARGS]      python bench.py ARGS (the bench line is kept as NAME_line.json)
#   stages[:LIB]      tools/grad_err_stages.py on batch2_div_s10 with the shipped library or variants/LIB
set -o pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
echo "tree $(python -c 'import bench; print(bench.tree_hash())')"
for spec in "$@"; do
  case "$spec" in
    tests*) a=${spec#tests}; a=${a#:}
      spec="tests|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $a" ;;
    bench*) a=${spec#bench}; a=${a#:}
      spec="bench|400|python bench.py $a" ;;
    stages*) a=${spec#stages}; a=${a#:}
      if [ -n "$a" ]; then
        spec="stages_$a|300|PDG_LIB=$R/variants/$a/libpdivgnn_hip.so python tools/grad_err_stages.py batch2_div_s10 --json $O/stages_$a.json"
      else
        spec="stages|300|python tools/grad_err_stages.py batch2_div_s10 --json $O/stages.json"
      fi ;;
  esac
  IFS='|' read -r name secs cmd <<< "$spec"
  echo "== $name"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"
  tail -4 "$O/$name.log"
  grep '^{' "$O/$name.log" | tail -1 > "$O/${name}_line.json" 2>/dev/null || rm -f "$O/${name}_line.json"
  [ -s "$O/${name}_line.json" ] || rm -f "$O/${name}_line.json"
  [ $rc -ne 0 ] && exit $rc
done
echo "all done"
