# pq_scatter_bwd node chunking (variants/pqd{2,4,8}: that many equal chunks per XCD; default: 512-node chunks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06y}
for c in 2 3; do for rep in 1 2; do bash tools/ab.sh $TAG $c default pqd2 pqd4 pqd8 || exit 1; done; done
