# Round profiles for both workloads (run via gpurun from the repo root)
set -o pipefail
TAG=${1:-r01c}
timeout -k 10 900 bash tools/profile_round.sh $TAG fixed || exit 1
timeout -k 10 900 bash tools/profile_round.sh $TAG csr || exit 1
echo profiles-done
