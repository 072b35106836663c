#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/r04h.sh r04h || exit $?
bash tools/r04i.sh
