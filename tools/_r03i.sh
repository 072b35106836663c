set -o pipefail
bash tools/call_ab.sh r03i "node or model" base || exit 1
bash tools/ab_env.sh r03i "PDG_SEG_SUMS_TRAIN=0" "PDG_SEG_SUMS_TRAIN=1" || exit 1
bash tools/prof_now.sh r03i
