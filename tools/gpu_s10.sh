set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s10}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
bash tools/gpu_s9.sh "$TAG/a" || exit $?
bash tools/gpu_s8.sh "$TAG/b" || exit $?
